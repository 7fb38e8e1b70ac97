"""Adaptive k-skip MrR on the GPU (drop-in for reference v3/gpu/adaptivekskipmrr.py:10).

Follows the v3/cpu semantics (v3/cpu/adaptivekskipmrr.py:42-74; see DESIGN.md
for why not v3/gpu/mpi's): when the residual rises above the last accepted
one, x rolls back to the snapshot, r is recomputed from it, a plain MrR step
restarts the recurrence and k drops by one. The snapshot costs no copy: the
engine alternates two x buffers.
"""
from .common import run


def adaptivekskipmrr(A, b, x=None, tol=1e-05, maxiter=None, k=0, M=None, callback=None,
                     atol=None) -> tuple:
    """Solve A x = b with adaptive k-skip MrR. info also holds 'khistory'."""
    return run("adaptivekskipmrr", "Adaptive k-skip MrR + GPU", A, b, x, tol, maxiter, k)
