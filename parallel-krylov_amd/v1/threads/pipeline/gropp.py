"""Gropp on the GPU (drop-in for reference
v1/threads/pipeline/gropp.py:7-50).

Restated as the textbook algorithm the file names (oracle/pipecg.py lists the
reference defects fixed); Jacobi preconditioner on the device. Per iteration:
two reduction points; w = A u is enqueued before the host waits for <r,r> <r,u>, so the SpMV overlaps the reduction.
"""
import numpy as np

from .common import run


def gropp(A, b, ilu, epsilon, T=np.float64, pt="cpu", maxiter=None, x0=None, return_x=False):
    """Solve A x = b (A symmetric positive definite) to relative residual
    ``epsilon``. Returns (elapsed_time, num_of_solution_updates, residual) as
    the reference does; see common.py for ``ilu``, ``pt`` and the extras."""
    return run("gropp", "gropp", A, b, ilu, epsilon, T, pt, maxiter, x0, return_x)
