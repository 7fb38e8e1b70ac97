"""Preconditioned CG on the GPU (drop-in for reference
v1/threads/pipeline/pcg.py:4-48).

Restated as the textbook algorithm the file names (oracle/pipecg.py lists the
reference defects fixed); Jacobi preconditioner on the device. Per iteration:
two reduction points per iteration (<p,s> from the s = A p SpMV epilogue; <r,r> <r,u> fused into the x/r/u update).
"""
import numpy as np

from .common import run


def pcg(A, b, ilu, epsilon, T=np.float64, pt="cpu", maxiter=None, x0=None, return_x=False):
    """Solve A x = b (A symmetric positive definite) to relative residual
    ``epsilon``. Returns (elapsed_time, num_of_solution_updates, residual) as
    the reference does; see common.py for ``ilu``, ``pt`` and the extras."""
    return run("pcg", "Preconditioned CG", A, b, ilu, epsilon, T, pt, maxiter, x0, return_x)
