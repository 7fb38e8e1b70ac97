"""k-skip MrR on the GPU (drop-in for reference v3/gpu/kskipmrr.py:9).

The north-star path. Per outer iteration (v3/gpu/kskipmrr.py:39-99):
k two-vector SpMVs (Ar[m+2], Ay[m+1]) = A (Ar[m+1], Ay[m]) with the 6k+5 Gram
coefficients fused into their epilogues; one device->host copy; the scalar
recurrence on the host (libm pow, no FMA: bitwise the numpy statements); then
k+1 fused (Ay0, z, r, x) updates each followed by Ar1 = A r. The reference's
duplicated Ar[1] SpMV at the top of the basis is not recomputed (same value).
"""
from .common import run


def kskipmrr(A, b, x=None, tol=1e-05, maxiter=None, k=0, M=None, callback=None,
             atol=None) -> tuple:
    """Solve A x = b with k-skip MrR. Returns (x, info) like the reference."""
    return run("kskipmrr", "k-skip MrR + GPU", A, b, x, tol, maxiter, k)
