"""Adaptive k-skip MrR, one rank per GPU (v3/cpu semantics) (drop-in for reference v3/gpu/mpi/adaptivekskipmrr.py:10).

Each rank holds its row block; halos move by RCCL send/recv and the partial
dot products by one RCCL all-gather per sync point (see common.py).
"""
from .common import run


def adaptivekskipmrr(comm, local_A, b, x=None, tol=1e-05, maxiter=None, k=0, M=None,
                     callback=None, atol=None, exit_nonroot=False) -> tuple:
    return run("adaptivekskipmrr", "Adaptive k-skip MrR + GPU + MPI", comm, local_A, b, x, tol,
               maxiter, k, exit_nonroot)
