"""Conjugate gradient, one rank per GPU (drop-in for reference v3/gpu/mpi/cg.py:10).

Each rank holds its row block; halos move by RCCL send/recv and the partial
dot products by one RCCL all-gather per sync point (see common.py).
"""
from .common import run


def cg(comm, local_A, b, x=None, tol=1e-05, maxiter=None, M=None, callback=None, atol=None,
       exit_nonroot=False) -> tuple:
    return run("cg", "CG + GPU + MPI", comm, local_A, b, x, tol, maxiter, None, exit_nonroot)
