"""Conjugate gradient on the GPU (drop-in for reference v3/gpu/cg.py:8).

The loop of v3/gpu/cg.py:24-39 runs natively: one SpMV with a fused <p,v>,
one fused x/r update with <r,r>, one p update per iteration; two scalar
syncs per iteration (the reference syncs on every cupy 0-d array).
"""
from .common import run


def cg(A, b, x=None, tol=1e-05, maxiter=None, M=None, callback=None, atol=None) -> tuple:
    """Solve A x = b (A symmetric positive definite). Returns (x, info) with
    info = {'time', 'nosl', 'residual'}; M, callback and atol are accepted and
    ignored, as in the reference."""
    return run("cg", "CG + GPU", A, b, x, tol, maxiter)
