"""Bitwise parity with the oracle run in the engine's summation order.

Adaptive k-skip MrR rolls back only on rounding events (MrR's residual is
non-increasing in exact arithmetic), so every reference trajectory that rolls
back is chaotic under a change of summation order (tests/golden/
make_golden.py). The reference fixtures therefore pin the rollback cases only
loosely (test_gpu_solvers.py). Here the oracle (oracle/v3cpu.py, bitwise the
reference given the same dot products) runs with the engine's own dot-product
order (oracle/gpu_order.py). The GPU must then match it BIT FOR BIT through
every rollback: nosl, khistory, every residual entry and x. That pins the
restore point, the i/index/k bookkeeping after a rollback and the resumed
k-skip chain (v3/cpu/adaptivekskipmrr.py:45-69), on one shard, on 2-3
in-process shards (split SpMV, shard partials summed in order) and through
the MPI family on one rank.

CPU tests here check the emulation itself; ``-m gpu`` tests compare with the
GPU (MI355X).
"""
import contextlib
import importlib
import io

import numpy as np
import pytest

from conftest import golden_matrix
from oracle import gpu_order, v3cpu

# (method, matrix, k, shards, k changes the GPU-order oracle makes (entries))
CASES = [
    ("adaptivekskipmrr", ["poisson", 16, 2], 12, 1, [7, 10, 13]),
    ("adaptivekskipmrr", ["poisson", 24, 3], 12, 1, [10, 13]),
    ("adaptivekskipmrr", ["banded", 3000, 31, 256, 0], 12, 1, [6, 9]),
    ("adaptivekskipmrr", ["poisson", 16, 2], 12, 2, [6, 9]),
    ("adaptivekskipmrr", ["poisson", 24, 3], 12, 3, [5, 8]),
    ("adaptivekskipmrr", ["banded", 3000, 31, 256, 0], 12, 2, [4, 7, 11]),
    ("adaptivekskipmrr", ["banded", 3000, 31, 256, 0], 4, 1, []),
    ("kskipmrr", ["poisson", 16, 3], 8, 1, []),
    ("kskipmrr", ["banded", 3000, 31, 256, 0], 6, 2, []),
    ("kskipcg", ["poisson", 16, 2], 4, 1, []),
    # C5's generator (h = 31, W = 256) at N = 200k in C5's own 8-way
    # partition: two rollbacks (k 12 -> 11 -> 10) on the symmetric DIA walk
    ("adaptivekskipmrr", ["banded", 200_000, 31, 256, 0], 12, 8, [9, 13]),
]
IDS = [f"{m}-{'x'.join(map(str, a[1:3]))}-k{k}-s{s}" for m, a, k, s, _ in CASES]


def _rhs(n):
    return np.random.default_rng(1).standard_normal(n)


def _bal(n, p):
    q, r = divmod(n, p)
    out = [0]
    for i in range(p):
        out.append(out[-1] + q + (1 if i < r else 0))
    return out


# ------------------------------------------------------------------ CPU
# (the N = 200k case's oracle takes ~40 s: checked by its GPU test only)
SMALL = [(c, i) for c, i in zip(CASES, IDS) if c[4] and c[1][1] <= 3000]


@pytest.mark.parametrize("case", [c for c, _ in SMALL], ids=[i for _, i in SMALL])
def test_gpu_order_oracle_rolls_back(case):
    """The emulated-order oracle really exercises the rollback branch (the
    k changes the GPU test then has to reproduce exactly)."""
    method, spec, k, shards, changes = case
    A = golden_matrix(spec)
    sc = gpu_order.shard_scheds(A, _bal(A.shape[0], shards))
    _, info = gpu_order.run(method, A, _rhs(A.shape[0]), sc, tol=1e-10, k=k)
    kh = info["khistory"]
    assert (np.nonzero(np.diff(kh))[0] + 1).tolist() == changes
    assert info["residual"][-1] < 1e-10


@pytest.mark.parametrize("n", [8, 16, 24, 32, 64, 96, 128, 256])
def test_products_only_grid_matches_below_512_planes(n):
    """The products-only dual's capped grid (KR_PO_ZMAX, 16) equals the
    general grid on every cube below 512^3 (so the emulation, which sums over
    the general grid, stays exact there) and differs at 512^3 (P x 16 vs
    P x 32 workgroups)."""
    rows = n ** 3
    P = max(1, n * n // 512)
    assert gpu_order.stencil_grid(rows, P, 16) == gpu_order.stencil_grid(rows, P)
    assert gpu_order.stencil_grid(512 ** 3, 512, 16) == 512 * 16
    assert gpu_order.stencil_grid(512 ** 3, 512) == 512 * 32


def test_gpu_order_dot_is_a_dot():
    """Same products, another order: within rounding of numpy's dot, and
    exactly the lane/wave/block order on a case small enough to spell out."""
    rng = np.random.default_rng(0)
    for n, shards in [(1, 1), (255, 1), (256, 1), (3001, 1), (4096, 1), (5000, 3), (70000, 1)]:
        u, v = rng.standard_normal(n), rng.standard_normal(n)
        A = golden_matrix(["banded", n, 1, 1, 0]) if n > 1 else None
        if A is None:
            sc = [gpu_order.ShardSched(n=1, grid=1, spmv_grid=1)]
        else:
            sc = gpu_order.shard_scheds(A, _bal(n, shards))
        o = gpu_order.GpuOrder(sc)
        ref = float(np.dot(u, v))
        scale = float(np.dot(np.abs(u), np.abs(v)))
        assert abs(o.spmv_dot(u, v) - ref) <= 1e-13 * scale
        assert abs(o.ew_dot(u, v) - ref) <= 1e-13 * scale
    # 256 rows, one workgroup: wave trees then ((w0 + w1) + w2) + w3
    p = rng.standard_normal(256)
    o = gpu_order.GpuOrder([gpu_order.ShardSched(n=256, grid=1, spmv_grid=1)])

    def tree(w):
        w = list(w)
        while len(w) > 1:
            h = len(w) // 2
            w = [w[i] + w[i + h] for i in range(h)]
        return w[0]
    waves = [tree(p[64 * i:64 * i + 64]) for i in range(4)]
    expect = ((waves[0] + waves[1]) + waves[2]) + waves[3]
    assert o.spmv_dot(p, np.ones(256)) == 0.0 + expect


def test_shard_scheds_interior_rows():
    """Interior rows = rows with no halo column, shrunk to whole row blocks."""
    A = golden_matrix(["poisson", 24, 3])  # reach 576 rows
    sc = gpu_order.shard_scheds(A, _bal(A.shape[0], 3))
    assert [(s.int_lo, s.int_hi) for s in sc] == [(0, 3840), (768, 3840), (768, 4608)]
    assert all(s.grid == s.spmv_grid == 18 for s in sc)


# ------------------------------------------------------------------ GPU
def _solver(method, family="gpu"):
    mod = importlib.import_module(f"parallel_krylov_amd.v3.{family}.{method}")
    return getattr(mod, method)


def _engine_scheds(A, shards):
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition
    n = A.shape[0]
    sysm = KrylovSystem(n, balanced_partition(n, shards), [0] * shards)
    sysm.set_matrix(A)
    sysm.finalize()
    out = [gpu_order.ShardSched(**sysm.shard_sched(s)) for s in range(shards)]
    sysm.close()
    return out


def _assert_bitwise(x, info, x_ref, info_ref):
    np.testing.assert_array_equal(info["nosl"], info_ref["nosl"])
    if "khistory" in info_ref:
        np.testing.assert_array_equal(info["khistory"], info_ref["khistory"])
    np.testing.assert_array_equal(info["residual"], info_ref["residual"])
    np.testing.assert_array_equal(x.cpu().numpy(), x_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_gpu_bitwise_equals_gpu_order_oracle(monkeypatch, case):
    method, spec, k, shards, changes = case
    A = golden_matrix(spec)
    n = A.shape[0]
    b = _rhs(n)
    sc = _engine_scheds(A, shards)
    assert sc == gpu_order.shard_scheds(A, _bal(n, shards))  # the emulated geometry
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", ",".join(["0"] * shards))
    kw = dict(tol=1e-10, k=k)
    with contextlib.redirect_stdout(io.StringIO()):
        x, info = _solver(method)(A, b, **kw)
    x_ref, info_ref = gpu_order.run(method, A, b, sc, **kw)
    _assert_bitwise(x, info, x_ref, info_ref)
    if "khistory" in info:
        assert (np.nonzero(np.diff(info["khistory"]))[0] + 1).tolist() == changes


STREAM_CASES = [c for c in CASES if c[3] > 1]


@pytest.mark.gpu
@pytest.mark.parametrize("shared", ["0", "2"])
@pytest.mark.parametrize("case", STREAM_CASES, ids=[IDS[CASES.index(c)] for c in STREAM_CASES])
def test_stream_groups_bitwise_gpu_order(monkeypatch, case, shared):
    """Stream groups (kr_system_create, System::groups): by default the
    in-process shards of one device share its stream (the group's halo pieces
    in one gather launch, stream order as the only edge); KR_SHARED_STREAM=0
    gives each shard its own stream (pieces on the comm streams, event edges),
    2 groups the shards in pairs -- on one device, the mixed geometry several
    devices with several shards each would have (gather within a pair, comm
    streams and events between pairs). Every layout is bitwise the same
    GPU-order oracle: streams change the issue, not the arithmetic."""
    method, spec, k, shards, changes = case
    A = golden_matrix(spec)
    b = _rhs(A.shape[0])
    sc = _engine_scheds(A, shards)
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", ",".join(["0"] * shards))
    monkeypatch.setenv("KR_SHARED_STREAM", shared)
    kw = dict(tol=1e-10, k=k)
    with contextlib.redirect_stdout(io.StringIO()):
        x, info = _solver(method)(A, b, **kw)
    x_ref, info_ref = gpu_order.run(method, A, b, sc, **kw)
    _assert_bitwise(x, info, x_ref, info_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("maxiter", [40, 66, 67, 80, 92])
def test_gpu_rollback_bookkeeping_under_maxiter(maxiter):
    """maxiter cutting the solve before, at and after a rollback (2-D Poisson
    16^2, k = 12 in GPU order: rollbacks at i = 66 -> 67 and 91 -> 92;
    maxiter 66 stops just before the first check that rolls back, 67 and 92
    let the rollback and the outer iteration after it run): the exit
    branch's residual recomputation and the overshoot of i."""
    A = golden_matrix(["poisson", 16, 2])
    b = _rhs(A.shape[0])
    sc = _engine_scheds(A, 1)
    kw = dict(tol=1e-10, k=12, maxiter=maxiter)
    with contextlib.redirect_stdout(io.StringIO()):
        x, info = _solver("adaptivekskipmrr")(A, b, **kw)
    x_ref, info_ref = gpu_order.run("adaptivekskipmrr", A, b, sc, **kw)
    _assert_bitwise(x, info, x_ref, info_ref)


@pytest.fixture(scope="module")
def dist_single():
    import os
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29534")
        dist.init_process_group("gloo", rank=0, world_size=1)
    yield dist


@pytest.mark.gpu
@pytest.mark.parametrize("spec", [["poisson", 16, 2], ["banded", 3000, 31, 256, 0]])
def test_gpu_mpi_family_bitwise_equals_gpu_order_oracle(dist_single, spec):
    """v3.gpu.mpi on one rank (RCCL communicator; rank totals summed in rank
    order) through the same rollbacks."""
    A = golden_matrix(spec)
    b = _rhs(A.shape[0])
    sc = _engine_scheds(A, 1)
    with contextlib.redirect_stdout(io.StringIO()):
        x, info = _solver("adaptivekskipmrr", "gpu.mpi")(None, A, b, tol=1e-10, k=12)
    x_ref, info_ref = gpu_order.run("adaptivekskipmrr", A, b, sc, tol=1e-10, k=12)
    _assert_bitwise(x, info, x_ref, info_ref)
    assert np.any(np.diff(info["khistory"]) != 0)


@pytest.mark.gpu
@pytest.mark.parametrize("grid", ["2", "5"])
@pytest.mark.parametrize("method,k", [("kskipmrr", 4), ("adaptivekskipmrr", 12), ("kskipcg", 4)])
def test_dia_walk_long_runs_bitwise_gpu_order(monkeypatch, grid, method, k):
    """The symmetric DIA walk (spmv_diawalk_kernel) with long runs of row
    blocks per workgroup (KR_DIAW_GRID; the default grid gives each workgroup
    one block of this 3000-row C5-family matrix): every epilogue the k-skip
    methods use (head, dual + Gram, fused steps, fused first two steps) is
    bitwise the GPU-order oracle summed over the engine's walk geometry."""
    monkeypatch.setenv("KR_DIAW_GRID", grid)
    A = golden_matrix(["banded", 3000, 31, 256, 0])
    b = _rhs(A.shape[0])
    sc = _engine_scheds(A, 1)
    assert sc[0].dia_walk == 1 and sc[0].spmv_grid == int(grid)
    kw = dict(tol=1e-10, k=k)
    with contextlib.redirect_stdout(io.StringIO()):
        x, info = _solver(method)(A, b, **kw)
    x_ref, info_ref = gpu_order.run(method, A, b, sc, **kw)
    _assert_bitwise(x, info, x_ref, info_ref)


def test_dia_walk_visits_partition_blocks():
    """Walk geometry: every (virtual) row block visited once, in ascending
    runs, split evenly; the boundary launch's gap skipped."""
    for rows, grid, gap_at, gap in [(3000, 12, 0, 0), (3000, 5, 0, 0), (100000, 7, 0, 0),
                                    (3000, 3, 2, 7), (5000, 20, 1, 17)]:
        vis = gpu_order._visits_dia_walk(rows, grid, gap_at, gap)
        nrb = -(-rows // 256)
        flat = [v for run in vis for v in run]
        want = [v for v in range(nrb) if v < gap_at or v >= gap_at + gap]
        assert flat == want
        lens = [len(r) for r in vis]
        assert max(lens) - min(lens) <= 1


def test_dia_walk_detection():
    """shard_scheds marks the symmetric banded shards (band <= 256, <= 31
    upper slots) as walk shards with the resident-workgroup grid, and leaves
    stencils, short rows and perturbed values alone."""
    A = golden_matrix(["banded", 3000, 31, 256, 0])
    assert [s.dia_walk for s in gpu_order.shard_scheds(A, [0, 3000])] == [1]
    big = gpu_order.dia_walk_grid(10_000_000, 27)  # C3: h = 13 -> 3 per CU
    assert big == 768 and gpu_order.dia_walk_grid(50_000_000, 63) == 512  # C5: 2 per CU
    B = A.copy()
    B.data = B.data.copy()
    B.data[B.indptr[11] - 1] += 1e-3  # one upper value off its mirror
    assert [s.dia_walk for s in gpu_order.shard_scheds(B, [0, 1500, 3000])] == [0, 1]
    P = golden_matrix(["poisson", 16, 3])
    assert gpu_order.shard_scheds(P, [0, P.shape[0]])[0].dia_walk == 0


def test_oracle_default_order_untouched():
    """patched() restores the oracle's numpy dot afterwards."""
    A = golden_matrix(["poisson", 8, 2])
    sc = gpu_order.shard_scheds(A, [0, A.shape[0]])
    gpu_order.run("kskipmrr", A, _rhs(A.shape[0]), sc, tol=1e-8, k=2)
    assert v3cpu._dot is np.dot and v3cpu._norm is np.linalg.norm
