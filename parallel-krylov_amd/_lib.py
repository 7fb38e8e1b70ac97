"""ctypes binding of libkrylov_amd.so (C ABI: include/krylov_amd.h).

The library is built in-tree (``__graft_entry__.build()`` or ``make -C
parallel-krylov_amd/csrc``). Loading it never falls back to anything: if it is
missing, ``library()`` raises with the build command.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_NAME = "libkrylov_amd.so"
_lock = threading.Lock()
_lib = None

KR_METHOD = {"cg": 0, "mrr": 1, "kskipcg": 2, "kskipmrr": 3, "adaptivekskipmrr": 4,
             # v1/threads/pipeline/*.py (include/krylov_amd.h KR_METHOD_PCG ..)
             "pcg": 5, "chronopoulos_gear": 6, "gropp": 7, "pipeline": 8}
# include/krylov_amd.h KR_ABI_VERSION: the struct layouts below (SolveParams,
# SolveResult) are this version's; a library of another version is refused.
KR_ABI_VERSION = 205
KR_FORMAT = {0: "csr", 1: "stencil", 2: "dia", 3: "dense", 4: "dia_walk"}  # kr_system_shard_sched


class KrylovError(RuntimeError):
    """A libkrylov_amd call returned a negative status."""

    def __init__(self, code: int, where: str, message: str):
        super().__init__(f"{where} failed ({code}): {message}")
        self.code = code


class SolveParams(ctypes.Structure):
    _fields_ = [("method", ctypes.c_int), ("k", ctypes.c_int), ("tol", ctypes.c_double),
                ("maxiter", ctypes.c_int64), ("profile", ctypes.c_int),
                ("nan_guard", ctypes.c_int)]


class SolveResult(ctypes.Structure):
    _fields_ = [("time_s", ctypes.c_double), ("iterations", ctypes.c_int64),
                ("entries", ctypes.c_int64), ("converged", ctypes.c_int),
                ("final_k", ctypes.c_int), ("final_residual", ctypes.c_double),
                ("diverged", ctypes.c_int)]


class KernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_int64),
                ("total_ms", ctypes.c_double), ("bytes_per_launch", ctypes.c_double),
                ("shards", ctypes.c_int64)]


def library_path() -> str:
    return os.environ.get("KRYLOV_AMD_LIB", os.path.join(_HERE, _LIB_NAME))


_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_D = ctypes.c_double
_PP = ctypes.POINTER(ctypes.c_void_p)
_PI64 = ctypes.POINTER(ctypes.c_int64)
_PI = ctypes.POINTER(ctypes.c_int)
_PD = ctypes.POINTER(ctypes.c_double)

# name -> argtypes (all return int status unless listed in _RESTYPE)
_SIGNATURES = {
    "kr_version": [],
    "kr_last_error": [],
    "kr_device_count": [_PI],
    "kr_spmv_csr_f64": [_P, _I, _P, _P, _I64, _P, _P, _P],
    "kr_spmv2_csr_f64": [_P, _I, _P, _P, _I64, _P, _P, _P, _P, _P],
    "kr_dot_f64": [_P, _P, _I64, _P, _P],
    "kr_multidot_f64": [_PP, _PP, _I, _I64, _P, _P],
    "kr_norm2_f64": [_P, _I64, _P, _P],
    "kr_gram_kskipmrr_f64": [_P, _P, _I, _I64, _I64, _P, _P],
    "kr_gram_kskipcg_f64": [_P, _P, _I, _I64, _I64, _P, _P],
    "kr_update_mrr_f64": [_D, _D, _I, _P, _P, _P, _P, _P, _I64, _P],
    "kr_update_cg_f64": [_D, _P, _P, _P, _P, _I64, _P],
    "kr_kskipmrr_recurrence": [_I, _PD, _PD, _PD, _PD, _PD],
    "kr_kskipcg_recurrence": [_I, _PD, _PD, _PD, _PD, _PD],
    "kr_halo_plan": [_I, _PI64, _PI64, _PI64, _I, _PI64, _PI, _PI64, _PI, _I],
    "kr_comm_unique_id": [_P],
    "kr_comm_init": [_PP, _P, _I, _I, _I],
    "kr_comm_destroy": [_P],
    "kr_allreduce_sum_f64": [_P, _P, _I64, _P],
    "kr_halo_exchange_f64": [_P, _P, _PI64, _I, _PI64, _I, _P],
    "kr_system_create": [_PP, _I64, _I, _PI, _PI64, _P],
    "kr_system_destroy": [_P],
    "kr_system_adopt_csr": [_P, _I, _P, _I, _P, _P],
    "kr_system_adopt_dense": [_P, _I, _P, _I64],
    "kr_system_gen_poisson": [_P, _I, _I64],
    "kr_system_gen_banded": [_P, _I, _I64, _U64, _I],
    "kr_system_finalize": [_P],
    "kr_system_shard_info": [_P, _I, _PI64, _PI64, _PI64, _PI64],
    "kr_system_shard_layout": [_P, _I, _PI, _PI, _PI64, _PI64],
    "kr_system_shard_values": [_P, _I, _PI],
    "kr_system_shard_codes": [_P, _I, _PI],
    "kr_system_shard_code_patterns": [_P, _I, _PI],
    "kr_system_shard_box": [_P, _I, _PI],
    "kr_system_shard_dia_full_blocks": [_P, _I, _PI64, _PI64],
    "kr_system_shard_dia_sym": [_P, _I, _PI],
    "kr_system_shard_sched": [_P, _I, _PI, _PI, _PI, _PI],
    "kr_fill_rhs": [_P, _I, _U64, _P],
    "kr_system_csr": [_P, _I, _PP, _PI, _PP, _PP, _PI64],
    "kr_system_spmv": [_PP, _PP, _PP],
    "kr_solve_begin": [_P, ctypes.POINTER(SolveParams), _PP, _PP],
    "kr_solve_set_precond": [_P, _PP],
    "kr_solve_set_precond_ilu": [_P, _I64, _P, _P, _P, _P, _P, _P, _P, _P],
    "kr_solve_step": [_P, _I64, _PI],
    "kr_solve_end": [_P, _PP, ctypes.POINTER(SolveResult)],
    "kr_solve_history": [_P, _PD, _PI64, _PI64, _I64],
    "kr_solve_kernel_stats": [_P, ctypes.POINTER(KernelStat), _I, _PI],
    "kr_solve_kernel_stats_reset": [_P],
}
_SIGNATURES["kr_system_spmv"] = [_P, _PP, _PP]
_RESTYPE = {"kr_last_error": ctypes.c_char_p}


def exported_symbols():
    return sorted(_SIGNATURES)


def library() -> ctypes.CDLL:
    """Load (once) and return the native library. Raises if it is not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = library_path()
        if not os.path.exists(path):
            raise RuntimeError(
                f"{path} is not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C parallel-krylov_amd/csrc` (hipcc --offload-arch=gfx950)")
        lib = ctypes.CDLL(path)
        for name, argtypes in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPE.get(name, ctypes.c_int)
        got = lib.kr_version()
        if got != KR_ABI_VERSION:
            raise RuntimeError(f"{path}: ABI version {got}, this binding needs {KR_ABI_VERSION} "
                               "(rebuild the library: make -C parallel-krylov_amd/csrc)")
        _lib = lib
        return lib


def check(rc: int, where: str) -> None:
    if rc != 0:
        msg = library().kr_last_error()
        raise KrylovError(rc, where, msg.decode() if msg else "")


def call(name: str, *args) -> None:
    check(getattr(library(), name)(*args), name)


def ptr_array(values):
    """C array of void* from ints (device addresses) / None."""
    arr = (ctypes.c_void_p * len(values))()
    for i, v in enumerate(values):
        arr[i] = v if v else None
    return arr


def device_count() -> int:
    c = ctypes.c_int(0)
    call("kr_device_count", ctypes.byref(c))
    return c.value
