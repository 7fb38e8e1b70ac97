"""Preconditioned and pipelined CG (reference v1/threads/pipeline), on
libkrylov_amd: pcg, chronopoulos_gear, gropp, pipeline, and the Jacobi
preconditioner they take as ``ilu``."""
from .chronopoulos_gear import chronopoulos_gear  # noqa: F401
from .common import Jacobi  # noqa: F401
from .gropp import gropp  # noqa: F401
from .pcg import pcg  # noqa: F401
from .pipeline import pipeline  # noqa: F401
