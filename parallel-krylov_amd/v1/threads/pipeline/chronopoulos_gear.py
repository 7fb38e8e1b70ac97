"""Chronopoulos gear on the GPU (drop-in for reference
v1/threads/pipeline/chronopoulos_gear.py:7-56).

Restated as the textbook algorithm the file names (oracle/pipecg.py lists the
reference defects fixed); Jacobi preconditioner on the device. Per iteration:
ONE reduction point per iteration: <r,r> <r,u> from the fused p/s/x/r/u update and <u,w> from the w = A u SpMV epilogue, read back together.
"""
import numpy as np

from .common import run


def chronopoulos_gear(A, b, ilu, epsilon, T=np.float64, pt="cpu", maxiter=None, x0=None, return_x=False):
    """Solve A x = b (A symmetric positive definite) to relative residual
    ``epsilon``. Returns (elapsed_time, num_of_solution_updates, residual) as
    the reference does; see common.py for ``ilu``, ``pt`` and the extras."""
    return run("chronopoulos_gear", "chronopoulos gear", A, b, ilu, epsilon, T, pt, maxiter, x0, return_x)
