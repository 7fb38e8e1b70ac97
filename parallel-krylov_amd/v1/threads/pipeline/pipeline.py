"""Pipeline on the GPU (drop-in for reference
v1/threads/pipeline/pipeline.py:7-62).

Restated as the textbook algorithm the file names (oracle/pipecg.py lists the
reference defects fixed); Jacobi preconditioner on the device. Per iteration:
ONE reduction point per iteration (<r,r> <r,u> <w,u> fused into the 8-vector update); m = M^-1 w and n = A m are enqueued first.
"""
import numpy as np

from .common import run


def pipeline(A, b, ilu, epsilon, T=np.float64, pt="cpu", maxiter=None, x0=None, return_x=False):
    """Solve A x = b (A symmetric positive definite) to relative residual
    ``epsilon``. Returns (elapsed_time, num_of_solution_updates, residual) as
    the reference does; see common.py for ``ilu``, ``pt`` and the extras."""
    return run("pipeline", "pipeline", A, b, ilu, epsilon, T, pt, maxiter, x0, return_x)
