"""Runtime of the one-process-per-GPU family (reference v3/gpu/mpi/common.py).

The reference (v3/gpu/mpi/common.py:138-165) all-gathers every SpMV output
so that each rank holds full-length vectors and repeats every dot product over
all N entries. Here each rank keeps only its row block of A and of every
vector; per SpMV it exchanges halo rows with the ranks its columns reach
(RCCL send/recv over xGMI), and per sync point it all-gathers the handful of
partial dot products (RCCL), which every rank sums in rank order -- so every
rank takes identical decisions and the histories are identical everywhere.

``comm`` may be a torch.distributed process group (or None for the default
group) or an mpi4py-style communicator (``Get_rank``/``Get_size``/``bcast``/
``allgather``/``gather``); it only bootstraps RCCL and gathers x at the end.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

from ....system import (Communicator, KrylovSystem, balanced_partition, gpu_ids_range,
                        local_device)
from ...common import _finish, _start
from ..common import _host_vector, _is_tensor, check_maxiter

_COMMS = {}


def start(method_name="", k=None):
    """Banner + timer (v3/gpu/mpi/common.py:15-17; MPI.Wtime -> perf_counter)."""
    _start(method_name, k)
    return time.perf_counter()


def finish(start_time, isConverged, num_of_iter, final_residual, final_k=None):
    elapsed_time = time.perf_counter() - start_time
    _finish(elapsed_time, isConverged, num_of_iter, final_residual, final_k)
    return elapsed_time


class _Dist:
    """Uniform view of a torch.distributed group or an mpi4py-like comm."""

    def __init__(self, comm):
        self.comm = comm
        self.is_mpi = comm is not None and hasattr(comm, "Get_rank")
        if self.is_mpi:
            self.rank, self.size = comm.Get_rank(), comm.Get_size()
        else:
            import torch.distributed as dist
            if not dist.is_initialized():
                raise RuntimeError("torch.distributed is not initialised: call "
                                   "init_process_group first or pass an mpi4py comm")
            self.rank, self.size = dist.get_rank(comm), dist.get_world_size(comm)

    def allgather_int(self, v: int) -> list:
        if self.is_mpi:
            return [int(t) for t in self.comm.allgather(int(v))]
        import torch.distributed as dist
        out = [None] * self.size
        dist.all_gather_object(out, int(v), group=self.comm)
        return [int(t) for t in out]

    def communicator(self, device: int) -> Communicator:
        key = (id(self.comm), device)
        if key not in _COMMS:
            _COMMS[key] = (Communicator.from_mpi(self.comm, device) if self.is_mpi
                           else Communicator.from_torch(self.comm, device))
        return _COMMS[key]

    def gather_x(self, x_local, counts):
        """Full x on rank 0 (device tensor), None elsewhere."""
        import torch
        if self.is_mpi:
            parts = self.comm.gather(x_local.cpu().numpy(), root=0)
            if self.rank != 0:
                return None
            return torch.from_numpy(np.concatenate(parts)).to(x_local.device)
        import torch.distributed as dist
        backend = dist.get_backend(self.comm)
        width = max(counts)
        dev = x_local.device if backend == "nccl" else torch.device("cpu")
        padded = torch.zeros(width, dtype=torch.float64, device=dev)
        padded[: x_local.numel()] = x_local.to(dev)
        out = [torch.empty_like(padded) for _ in range(self.size)]
        dist.all_gather(out, padded, group=self.comm)
        if self.rank != 0:
            return None
        return torch.cat([o[:c] for o, c in zip(out, counts)]).to(x_local.device)


def rank_devices(rank):
    """Devices of this rank's local shards: the GPU_IDS range (the reference's
    per-rank GPU list, v3/gpu/mpi/common.py:77-83), else one GPU
    (local_device). ``KRYLOV_AMD_RANK_SHARDS="0,0"`` overrides it (several
    shards may share a device: the multi-GPU-per-rank path on one GPU)."""
    env = os.environ.get("KRYLOV_AMD_RANK_SHARDS")
    if env:
        return [int(t) for t in env.split(",") if t.strip() != ""]
    gpu_range = gpu_ids_range()
    if gpu_range is not None and len(gpu_range) > 1:
        return gpu_range
    return [local_device(rank)]


def run(method, banner, comm, local_A, b, x=None, tol=1e-05, maxiter=None, k=None,
        exit_nonroot=False):
    """Shared body of the five v3/gpu/mpi solver functions.

    ``local_A`` is this rank's contiguous row block (local_N x N, global
    columns) and ``b`` the full right-hand side, as in the reference
    (v3/gpu/mpi/kskipmrr.py:10, :20). Row blocks may differ in size (the
    reference requires local_N * size == N). Rank 0 returns (x, info); other
    ranks return (None, info), or exit(0) like the reference when
    ``exit_nonroot`` is set (v3/gpu/mpi/kskipmrr.py:121)."""
    import scipy.sparse as sp
    import torch
    d = _Dist(comm)
    bh = _host_vector(b)
    N = bh.size
    local_n = int(local_A.shape[0])
    counts = d.allgather_int(local_n)
    if sum(counts) != N:
        raise ValueError(f"row blocks cover {sum(counts)} rows but b has {N}")
    row0 = sum(counts[: d.rank])
    devices = rank_devices(d.rank)
    # one RCCL rank per process: a rank with several GPUs (GPU_IDS range,
    # MultiGpu.alloc, v3/gpu/mpi/common.py:100-118) keeps them as local
    # shards -- device copies between them, RCCL to the other ranks (a lone
    # rank with several GPUs is the in-process system)
    comm_h = None if (d.size == 1 and len(devices) > 1) else d.communicator(devices[0])
    torch.cuda.set_device(devices[0])
    rows = [row0 + r for r in balanced_partition(local_n, len(devices))]
    sysm = KrylovSystem(N, rows, devices, comm=comm_h)
    try:
        for s_, (r0, r1) in enumerate(zip(rows[:-1], rows[1:])):
            blk = local_A[r0 - row0:r1 - row0]
            if sp.issparse(local_A):
                sysm.adopt_csr(s_, blk)
            else:  # dense row block: GEMV path (v3/gpu/mpi/common.py:124-125)
                sysm.adopt_dense(s_, blk)
        sysm.finalize()
        dev_of = [torch.device("cuda", dv) for dv in devices]
        b_parts = [torch.from_numpy(np.ascontiguousarray(bh[r0:r1])).to(dv)
                   for r0, r1, dv in zip(rows[:-1], rows[1:], dev_of)]
        x0_parts = None
        if isinstance(x, np.ndarray) or _is_tensor(x):
            xh = _host_vector(x)
            x0_parts = [torch.from_numpy(np.ascontiguousarray(xh[r0:r1])).to(dv)
                        for r0, r1, dv in zip(rows[:-1], rows[1:], dev_of)]
        if d.rank == 0:
            _start(banner, k)
        check_maxiter(method, maxiter)
        out = sysm.solve(method, b_parts, x0_parts, tol=tol, maxiter=maxiter, k=k or 0)
        x_local = torch.cat([xs.to(dev_of[0]) for xs in out.x])
        x_full = d.gather_x(x_local, counts)
    finally:
        sysm.close()
    if d.rank == 0:
        final_k = out.final_k if method == "adaptivekskipmrr" else None
        _finish(out.info["time"], out.converged, out.iterations, out.final_residual, final_k)
        return x_full, out.info
    if exit_nonroot:
        sys.exit(0)
    return None, out.info
