"""Import shim for the ``parallel-krylov_amd/`` package directory.

The package directory name contains a hyphen, which Python cannot import
directly; this module gives it the importable name ``parallel_krylov_amd``
(``import parallel_krylov_amd.v3.gpu.kskipmrr`` etc.) by pointing its
``__path__`` at that directory and running the package ``__init__``.
"""
import os as _os

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "parallel-krylov_amd")
__path__ = [_PKG_DIR]
__package__ = __name__
_init = _os.path.join(_PKG_DIR, "__init__.py")
with open(_init) as _f:
    exec(compile(_f.read(), _init, "exec"))
del _f, _init
