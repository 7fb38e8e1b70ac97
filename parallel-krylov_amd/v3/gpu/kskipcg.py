"""k-skip CG on the GPU (drop-in for reference v3/gpu/kskipcg.py:9).

Per outer iteration: the basis Ar[1..k], Ap[1..k+1] as k two-vector SpMVs that
read A once for both chains, with the 6k+7 Gram coefficients fused into their
epilogues (the reference issues 2k+1 SpMVs and 6k+7 separate ddot calls);
one device->host copy of the Gram; the scalar recurrence on the host; k+1
fused x/r/p updates each followed by one SpMV.
"""
from .common import run


def kskipcg(A, b, x=None, tol=1e-05, maxiter=None, k=0, M=None, callback=None,
            atol=None) -> tuple:
    """Solve A x = b with k-skip CG. Returns (x, info) like the reference."""
    return run("kskipcg", "k-skip CG + GPU", A, b, x, tol, maxiter, k)
