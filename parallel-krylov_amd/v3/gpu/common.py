"""Runtime of the single-process GPU family (reference v3/gpu/common.py).

The reference's names are kept -- ``start``, ``finish``, ``init`` and the
``MultiGpu`` class -- but the iteration loops no longer live in Python: each
solver module hands the whole solve to ``KrylovSystem.solve`` (native engine,
HIP kernels) and only formats the result here.
"""
from __future__ import annotations

import time

import numpy as np

from ...system import KrylovSystem, balanced_partition, system_from_matrix, visible_devices
from ..common import _finish, _start


def start(method_name: str = "", k: int = None) -> float:
    """Banner + timer start (v3/gpu/common.py:12-14)."""
    _start(method_name, k)
    return time.perf_counter()


def finish(start_time: float, isConverged: bool, num_of_iter: int, final_residual: float,
           final_k: int = None) -> float:
    """Timer stop + banner (v3/gpu/common.py:18-21)."""
    elapsed_time = time.perf_counter() - start_time
    _finish(elapsed_time, isConverged, num_of_iter, final_residual, final_k)
    return elapsed_time


def init(b, x=None, maxiter=None) -> tuple:
    """Device copies and bookkeeping arrays (v3/gpu/common.py:25-40).

    Returns (b, x, maxiter, b_norm, N, residual, num_of_solution_updates) with
    b and x as float64 device tensors on the first GPU. Histories are host
    arrays (the native engine keeps them on the host and never preallocates
    maxiter+1 device entries)."""
    import torch
    dev = torch.device("cuda", visible_devices()[0])
    bt = _as_tensor(b, dev)
    N = bt.numel()
    xt = _as_tensor(x, dev) if isinstance(x, np.ndarray) or _is_tensor(x) else \
        torch.zeros(N, dtype=torch.float64, device=dev)
    if maxiter is None:
        maxiter = N
    b_norm = torch.linalg.norm(bt)
    return (bt, xt, maxiter, b_norm, N, np.zeros(maxiter + 1, np.float64),
            np.zeros(maxiter + 1, np.int64))


def _is_tensor(v) -> bool:
    try:
        import torch
        return isinstance(v, torch.Tensor)
    except ImportError:  # pragma: no cover
        return False


def _as_tensor(v, dev):
    import torch
    if _is_tensor(v):
        return v.to(device=dev, dtype=torch.float64).contiguous()
    return torch.from_numpy(np.ascontiguousarray(np.asarray(v), dtype=np.float64)).to(dev)


def _host_vector(v) -> np.ndarray:
    if _is_tensor(v):
        return v.detach().to("cpu", dtype=__import__("torch").float64).numpy()
    return np.ascontiguousarray(np.asarray(v), dtype=np.float64)


class MultiGpu:
    """Distributed SpMV over the visible GPUs (v3/gpu/common.py:43-126).

    ``init()`` picks the devices, ``alloc(A, b, T)`` distributes A by rows,
    ``dot(A, x)`` returns A @ x as a device tensor. Unlike the reference, x
    is not broadcast whole to every GPU: each shard receives only its halo."""

    devices: list = []
    system: KrylovSystem = None
    N: int = 0

    @classmethod
    def init(cls):
        cls.devices = visible_devices()

    @classmethod
    def alloc(cls, A, b, T=np.float64):
        if not cls.devices:
            cls.init()
        cls.N = int(np.asarray(b).size) if not _is_tensor(b) else int(b.numel())
        cls.system = system_from_matrix(A, cls.devices)

    @classmethod
    def dot(cls, A, x):
        if cls.system is None:
            cls.alloc(A, np.zeros(A.shape[0]))
        parts = cls.system.split(x)
        return cls.system.gather(cls.system.spmv(parts))


MRR_FAMILY = ("mrr", "kskipmrr", "adaptivekskipmrr")


def check_maxiter(method: str, maxiter) -> None:
    """maxiter = 0 (not None): CG and k-skip CG return the initial residual;
    the MrR family takes its first step unconditionally and writes
    ``num_of_solution_updates[1]`` of a length-1 array, an IndexError in the
    reference (v3/gpu/mrr.py, v3/cpu/mrr.py:31, kskipmrr.py:32). Raised here,
    after the banner, as the reference raises it."""
    if maxiter is not None and int(maxiter) == 0 and method in MRR_FAMILY:
        raise IndexError("index 1 is out of bounds for axis 0 with size 1 "
                         f"({method} with maxiter=0, as in the reference)")


def run(method: str, banner: str, A, b, x=None, tol=1e-05, maxiter=None, k=None):
    """Shared body of the five v3/gpu solver functions.

    Semantics kept from the reference: x is used only if it is an ndarray
    (or a tensor) -- anything else means zeros (v3/gpu/common.py:30-33); the
    caller's x is not modified; maxiter None means N; the printed INFO block
    and the returned info dict match v3/gpu/<method>.py."""
    import torch
    bh = _host_vector(b)
    N = bh.size
    devices = visible_devices()
    sysm = KrylovSystem(N, balanced_partition(N, len(devices)), devices)
    try:
        sysm.set_matrix(A)
        sysm.finalize()
        b_parts = sysm.split(bh)
        x0_parts = sysm.split(_host_vector(x)) if (isinstance(x, np.ndarray) or _is_tensor(x)) \
            else None
        _start(banner, k)
        check_maxiter(method, maxiter)
        out = sysm.solve(method, b_parts, x0_parts, tol=tol, maxiter=maxiter, k=k or 0)
        final_k = out.final_k if method == "adaptivekskipmrr" else None
        _finish(out.info["time"], out.converged, out.iterations, out.final_residual, final_k)
        xs = sysm.gather(out.x)
        if xs.device != torch.device("cuda", devices[0]):
            xs = xs.to(torch.device("cuda", devices[0]))
        return xs, out.info
    finally:
        sysm.close()
