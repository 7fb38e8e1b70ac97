"""parallel-krylov_amd: MI355X-native inner loop of 5enxia/parallel-krylov.

Drop-in for the reference's ``v3/gpu`` and ``v3/gpu/mpi`` solver families
(CG, MrR, k-skip CG, k-skip MrR, adaptive k-skip MrR):

    from parallel_krylov_amd.v3.gpu.kskipmrr import kskipmrr
    x, info = kskipmrr(A, b, tol=1e-10, k=4)

Every solver iteration runs in ``libkrylov_amd.so`` (hand-written HIP kernels
for gfx950 + a native host engine, C ABI in ``include/krylov_amd.h``). There is
no CPU fallback: without the built library, or without a GPU, the solvers
raise.
"""
__version__ = "0.1.0"

from ._lib import KrylovError, library, library_path  # noqa: E402,F401
from .system import KrylovSystem, METHODS  # noqa: E402,F401
