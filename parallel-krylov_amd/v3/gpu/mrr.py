"""Minimal residual (MrR) on the GPU (drop-in for reference v3/gpu/mrr.py:8).

Per iteration (v3/gpu/mrr.py:40-52): SpMV with fused <r,r>, <y,y>, <y,Ar>;
the s = Ar - gamma*y pass with fused <r,s>, <s,s>; one fused y/z/r/x update.
"""
from .common import run


def mrr(A, b, x=None, tol=1e-05, maxiter=None, M=None, callback=None, atol=None) -> tuple:
    """Solve A x = b with MrR. Returns (x, info) like the reference."""
    return run("mrr", "MrR + GPU", A, b, x, tol, maxiter)
