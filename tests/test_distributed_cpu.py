"""Multi-rank host logic on the CPU: world_size 2 over gloo (127.0.0.1).

What runs here is the product's host side of the N>1 path:
* the halo planner (``kr_halo_plan`` in libkrylov_amd, the same function
  ``kr_system_finalize`` uses) and the local column numbering rule
  (local = global - row0 + pad, pad = halo_lo rounded up to 8);
* the MPI-family plumbing of ``parallel_krylov_amd.v3.gpu.mpi.common``
  (row-block discovery by all-gather, x gathered to rank 0).

The numerics of one rank are emulated with numpy (test code): the local SpMV
on the halo-extended vector after a gloo send/recv exchange that follows the
plan, and dot products as per-rank partials all-gathered and summed in rank
order -- exactly the reduction order the engine uses. Results must equal the
unpartitioned oracle: SpMV bit for bit, CG within the rounding envelope.
"""
import ctypes
import os
import socket

import numpy as np
import pytest

from conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _plan(part, lo, hi, me):
    import parallel_krylov_amd._lib as L
    lib = L.library()
    P = len(part) - 1
    cap = 2 * P + 2
    arr = lambda v: (ctypes.c_int64 * len(v))(*[int(t) for t in v])
    rout = (ctypes.c_int64 * (3 * cap))()
    sout = (ctypes.c_int64 * (3 * cap))()
    nr, ns = ctypes.c_int(), ctypes.c_int()
    rc = lib.kr_halo_plan(P, arr(part), arr(lo), arr(hi), me, rout, ctypes.byref(nr), sout,
                          ctypes.byref(ns), cap)
    assert rc == 0
    return ([tuple(rout[3 * q:3 * q + 3]) for q in range(nr.value)],
            [tuple(sout[3 * q:3 * q + 3]) for q in range(ns.value)])


class RankEmulation:
    """One rank's shard: local CSR in local numbering + halo exchange."""

    def __init__(self, dist, A, part, rank):
        self.dist, self.rank = dist, rank
        r0, r1 = part[rank], part[rank + 1]
        blk = A[r0:r1]
        self.r0, self.n = r0, r1 - r0
        lo = min(int(blk.indices.min()), r0)
        hi = max(int(blk.indices.max()), r1 - 1)
        allr = [None] * dist.get_world_size()
        dist.all_gather_object(allr, (lo, hi))
        los, his = [t[0] for t in allr], [t[1] for t in allr]
        self.recv, self.send = _plan(part, los, his, rank)
        halo_lo = r0 - lo
        self.pad = (halo_lo + 7) // 8 * 8
        self.ld = self.pad + self.n + (hi - (r1 - 1))
        self.blk = blk.copy()
        self.blk.indices = (blk.indices.astype(np.int64) - r0 + self.pad).astype(np.int32)
        self.blk._shape = (self.n, self.ld)

    def local(self, g):
        return g - self.r0 + self.pad

    def exchange(self, v):
        import torch
        reqs = []
        for peer, g0, cnt in self.send:
            t = torch.from_numpy(np.ascontiguousarray(v[self.local(g0):self.local(g0) + cnt]))
            reqs.append(self.dist.isend(t, int(peer)))
        bufs = []
        for peer, g0, cnt in self.recv:
            t = torch.empty(int(cnt), dtype=torch.float64)
            reqs.append(self.dist.irecv(t, int(peer)))
            bufs.append((g0, cnt, t))
        for r in reqs:
            r.wait()
        for g0, cnt, t in bufs:
            v[self.local(g0):self.local(g0) + cnt] = t.numpy()

    def spmv(self, own):
        v = np.zeros(self.ld)
        v[self.pad:self.pad + self.n] = own
        self.exchange(v)
        return self.blk.dot(v)

    def allsum(self, partial):
        out = [None] * self.dist.get_world_size()
        self.dist.all_gather_object(out, np.asarray(partial, dtype=np.float64))
        tot = np.zeros_like(np.asarray(partial, dtype=np.float64))
        for o in out:  # rank order, as the engine
            tot = tot + o
        return tot


def _worker(rank, world, port, result_file):
    import torch.distributed as dist
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle import matrices, v3cpu
    from parallel_krylov_amd.system import balanced_partition
    from parallel_krylov_amd.v3.gpu.mpi.common import _Dist
    import torch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    try:
        A = matrices.poisson(8, 3)
        N = A.shape[0]
        part = balanced_partition(N, world)
        em = RankEmulation(dist, A, part, rank)
        # 1. distributed SpMV, bitwise
        x = np.random.default_rng(5).standard_normal(N)
        y = em.spmv(x[em.r0:em.r0 + em.n])
        out["spmv_bitwise"] = bool(np.array_equal(y, A.dot(x)[em.r0:em.r0 + em.n]))
        # 2. CG with per-rank partial dots summed in rank order
        b = np.random.default_rng(1).standard_normal(N)
        bl = b[em.r0:em.r0 + em.n]
        bnorm = np.sqrt(em.allsum([np.dot(bl, bl)])[0])
        xl = np.zeros(em.n)
        r = bl - em.spmv(xl)
        p = r.copy()
        gamma = em.allsum([np.dot(r, r)])[0]
        res = []
        for it in range(200):
            res.append(np.sqrt(gamma) / bnorm)
            if res[-1] < 1e-10:
                break
            v = em.spmv(p)
            sigma = em.allsum([np.dot(p, v)])[0]
            alpha = gamma / sigma
            xl += alpha * p
            r -= alpha * v
            gnew = em.allsum([np.dot(r, r)])[0]
            beta = gnew / gamma
            gamma = gnew
            p = r + beta * p
        _, info = v3cpu.cg(A, b, tol=1e-10)
        ref = info["residual"]
        out["cg_len_equal"] = len(res) == len(ref)
        m = min(len(res), len(ref))
        out["cg_maxrel"] = float(np.max(np.abs(np.array(res[:m]) - ref[:m]) / ref[:m]))
        # 3. MPI-family plumbing: row blocks and x gather over gloo
        d = _Dist(None)
        counts = d.allgather_int(em.n)
        out["counts_ok"] = counts == [part[i + 1] - part[i] for i in range(world)]
        full = d.gather_x(torch.from_numpy(xl.copy()), counts)
        if rank == 0:
            xs, _ = v3cpu.cg(A, b, tol=1e-10)
            out["x_rel"] = float(np.linalg.norm(full.numpy() - xs) / np.linalg.norm(xs))
        out["plan"] = (em.recv, em.send)
    finally:
        dist.barrier()
        dist.destroy_process_group()
    np.save(result_file.format(rank=rank), out, allow_pickle=True)


@pytest.mark.parametrize("world", [2, 3])
def test_row_partitioned_path_over_gloo(tmp_path, world):
    import torch.multiprocessing as mp
    port = _free_port()
    result = str(tmp_path / "rank{rank}.npy")
    mp.start_processes(_worker, args=(world, port, result), nprocs=world, join=True,
                       start_method="spawn")
    outs = [np.load(result.format(rank=r), allow_pickle=True).item() for r in range(world)]
    for o in outs:
        assert o["spmv_bitwise"]
        assert o["cg_len_equal"]
        assert o["cg_maxrel"] < 1e-12
        assert o["counts_ok"]
    assert outs[0]["x_rel"] < 1e-12
    # every send of one rank is a receive of its peer
    for me, o in enumerate(outs):
        for peer, g0, cnt in o["plan"][1]:
            assert (me, g0, cnt) in outs[peer]["plan"][0]


@pytest.mark.parametrize("env,expect", [(None, None), ("3", [3]), ("2,5", [2, 3, 4, 5]),
                                        ("0,1,2,3", [0, 1, 2, 3]), ("4,4", [4])])
def test_gpu_ids_range(monkeypatch, env, expect):
    """GPU_IDS as the reference reads it: ids[0]..ids[-1] inclusive
    (v3/gpu/mpi/common.py:77-83)."""
    from parallel_krylov_amd.system import gpu_ids_range
    if env is None:
        monkeypatch.delenv("GPU_IDS", raising=False)
    else:
        monkeypatch.setenv("GPU_IDS", env)
    assert gpu_ids_range() == expect


def test_gpu_ids_range_rejects_descending(monkeypatch):
    from parallel_krylov_amd.system import gpu_ids_range
    monkeypatch.setenv("GPU_IDS", "3,1")
    with pytest.raises(ValueError):
        gpu_ids_range()


def test_local_device_gpu_ids_wins_over_local_rank(monkeypatch):
    """GPU_IDS (set per process by the launcher, as the reference's MPI family
    reads it) picks the rank's device even under torchrun's LOCAL_RANK."""
    from parallel_krylov_amd import system
    monkeypatch.setattr(system._lib, "device_count", lambda: 8)
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setenv("GPU_IDS", "3")
    assert system.local_device(1) == 3
    monkeypatch.setenv("GPU_IDS", "4,5")
    assert system.local_device(0) == 4
    monkeypatch.delenv("GPU_IDS")
    assert system.local_device(0) == 1
    monkeypatch.delenv("LOCAL_RANK")
    assert system.local_device(10) == 2


def test_job_wide_gpu_ids_warns_under_torchrun(monkeypatch):
    """A GPU_IDS next to LOCAL_RANK with WORLD_SIZE > 1 (a job-wide export
    under torchrun would stack every rank on the same GPUs) warns once."""
    from parallel_krylov_amd import system
    monkeypatch.setattr(system, "_warned_gpu_ids", False)
    monkeypatch.setenv("LOCAL_RANK", "1")
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("GPU_IDS", "0,1")
    with pytest.warns(RuntimeWarning, match="overrides LOCAL_RANK"):
        assert system.gpu_ids_range() == [0, 1]
    monkeypatch.setattr(system, "_warned_gpu_ids", False)
    monkeypatch.setenv("WORLD_SIZE", "1")
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert system.gpu_ids_range() == [0, 1]  # one rank: nothing to warn about
