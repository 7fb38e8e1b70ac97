"""Runtime of the preconditioned / pipelined CG variants (reference
v1/threads/pipeline/*.py, with the loop bookkeeping of v1/threads/common.py).

The reference signature is kept -- ``method(A, b, ilu, epsilon, T=np.float64,
pt='cpu')`` returning ``(elapsed_time, num_of_solution_updates, residual)`` --
and the whole loop runs in libkrylov_amd (PipeCgSession, kr_engine.cpp; HIP
kernels EW_PCG / EW_CGG / EW_GROPP* / EW_PIPE). ``pt`` is accepted for
compatibility; both values run on the GPUs (the package has no CPU path).

``ilu`` is the preconditioner: the reference passes an object whose
``solve(v)`` applies M^-1 (pcg.py:26), a scipy SuperLU from ``spilu``. On the
device:
  * ``None``: the identity (d = 1);
  * ``Jacobi(A)`` (or any object with a 1-D ``d`` attribute) or a 1-D array /
    tensor of N values: the diagonal d (M^-1 v = v / d, fused into the
    vector kernels);
  * a SuperLU (``scipy.sparse.linalg.spilu`` / ``splu``: attributes L, U,
    perm_r, perm_c) or a (L, U, perm_r, perm_c) tuple: M = Pr^T L U Pc^T, and
    ``ilu.solve(v)`` = Pc U^-1 L^-1 Pr v runs as two level-scheduled
    triangular sweeps on the device (kr_solve_set_precond_ilu; the system is
    then kept on ONE GPU, the sweeps being sequential over the vector).
Anything else raises TypeError instead of silently falling back.
"""
from __future__ import annotations

import numpy as np

from ....system import KrylovSystem, balanced_partition, visible_devices
from ....v3.gpu.common import _host_vector
from ...common import _end, _start


class Jacobi:
    """Jacobi preconditioner: d = diag(A) (or the given diagonal); ``solve``
    is M^-1 v = v / d, the interface of the reference's ``ilu`` argument."""

    def __init__(self, A=None, d=None):
        if d is None:
            if A is None:
                raise ValueError("Jacobi needs A or d")
            d = A.diagonal() if hasattr(A, "diagonal") else np.diag(np.asarray(A))
        self.d = np.ascontiguousarray(np.asarray(d, dtype=np.float64))
        if not np.all(np.isfinite(self.d) & (self.d != 0.0)):
            raise ValueError("Jacobi: zero or non-finite entry on the diagonal")

    def solve(self, v):
        return v / self.d


def _ilu_factors(ilu, N):
    """(L, U, perm_r, perm_c) of a SuperLU object or such a tuple, else None."""
    def _square(m):
        return getattr(m, "shape", None) is not None and len(m.shape) == 2
    if isinstance(ilu, tuple) and len(ilu) == 4 and _square(ilu[0]) and _square(ilu[1]):
        L, U, pr, pc = ilu  # (a 4-tuple of numbers is a diagonal: _diagonal)
    elif all(hasattr(ilu, a) for a in ("L", "U", "perm_r", "perm_c")):
        L, U, pr, pc = ilu.L, ilu.U, ilu.perm_r, ilu.perm_c
    else:
        return None
    if L.shape != (N, N) or U.shape != (N, N):
        raise ValueError(f"ilu: factors of shape {L.shape} / {U.shape}, the system is N = {N}")
    return L, U, np.asarray(pr), np.asarray(pc)


def _diagonal(ilu, N):
    if ilu is None:
        return None
    d = getattr(ilu, "d", ilu)
    try:
        import torch
        if isinstance(d, torch.Tensor):
            d = d.detach().to("cpu", dtype=torch.float64).numpy()
    except ImportError:  # pragma: no cover
        pass
    if isinstance(d, (np.ndarray, list, tuple)):
        d = np.ascontiguousarray(np.asarray(d, dtype=np.float64))
        if d.ndim != 1 or d.size != N:
            raise ValueError(f"ilu: a diagonal of {N} values is required, got shape {d.shape}")
        # the same check as Jacobi(): u = r / d must stay finite on the device
        bad = ~np.isfinite(d) | (d == 0.0)
        if bad.any():
            raise ValueError(f"ilu: the diagonal has {int(bad.sum())} zero or non-finite "
                             f"entries (first at row {int(np.argmax(bad))})")
        return d
    raise TypeError(
        f"ilu={type(ilu).__name__}: the device path takes None, a diagonal (Jacobi(A) or a "
        "1-D array) or ILU factors (a scipy spilu / splu SuperLU, or (L, U, perm_r, perm_c)) "
        "(DESIGN.md §5b)")


def run(method: str, banner: str, A, b, ilu, epsilon, T=np.float64, pt="cpu", maxiter=None,
        x0=None, return_x=False):
    """Shared body of the four solver functions: 2N iterations at most
    (v1/threads/common.py:47) unless ``maxiter`` is given; the banner of
    v1/common.py. Returns ``(elapsed, nosl, residual)``, plus ``(x, converged)``
    with ``return_x=True`` (the reference returns no x)."""
    if np.dtype(T) != np.float64:
        raise ValueError("only T=np.float64 is supported")
    if pt not in ("cpu", "gpu"):
        raise ValueError(f"pt must be 'cpu' or 'gpu', got {pt!r}")
    bh = _host_vector(b)
    N = bh.size
    factors = _ilu_factors(ilu, N)
    d = None if factors is not None else _diagonal(ilu, N)
    devices = visible_devices()
    if factors is not None:  # the triangular sweeps are sequential: one shard
        devices = devices[:1]
    sysm = KrylovSystem(N, balanced_partition(N, len(devices)), devices)
    try:
        sysm.set_matrix(A)
        sysm.finalize()
        b_parts = sysm.split(bh)
        x0_parts = sysm.split(_host_vector(x0)) if x0 is not None else None
        if factors is not None:
            sysm.set_precond_ilu(factors)
        else:
            sysm.set_precond(sysm.split(d) if d is not None else None)
        _start(banner, None)
        out = sysm.solve(method, b_parts, x0_parts, tol=epsilon,
                         maxiter=2 * N if maxiter is None else maxiter)
        _end(out.info["time"], out.converged, out.iterations, out.final_residual)
        res = (out.info["time"], out.info["nosl"], out.info["residual"])
        if return_x:
            res = res + (sysm.gather(out.x), out.converged)
        return res
    finally:
        sysm.close()
