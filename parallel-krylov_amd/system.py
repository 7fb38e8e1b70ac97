"""Host-side mirror of the reference's multi-GPU runtime (``MultiGpu``).

``KrylovSystem`` owns a row-partitioned SPD system on one or more devices and
runs the solver loops natively (``kr_solve_*`` in libkrylov_amd.so). It is the
MI355X replacement for ``MultiGpu.init/alloc/dot`` of the reference
(v3/gpu/common.py:43-126, v3/gpu/mpi/common.py:46-171):

* the reference splits A by rows but REPLICATES every vector and moves full
  vectors per SpMV (peer broadcast + gather, then ``comm.Allgather``);
* here A and every vector stay row-partitioned; a SpMV moves only the halo
  rows its columns reach, and the dot products are reduced once per sync.

Two ways to hold shards, matching the two reference families:
* single process, ``devices`` = list of HIP devices (v3/gpu: all visible GPUs);
  several shards may share one device (used by the tests);
* one process per GPU with a ``Communicator`` (v3/gpu/mpi), RCCL over xGMI.

Device memory is held in torch tensors (PyTorch-ROCm is the allocator and the
bootstrap; no torch op runs on the solver path).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import call, library, ptr_array

METHODS = tuple(_lib.KR_METHOD)


def _torch():
    import torch
    return torch


def balanced_partition(n: int, parts: int) -> list:
    """Contiguous row blocks whose sizes differ by at most one row.

    (The reference uses ``N // G`` rows per GPU and silently drops the
    remainder, v3/gpu/common.py:86; here every row is owned.)"""
    q, r = divmod(n, parts)
    out = [0]
    for p in range(parts):
        out.append(out[-1] + q + (1 if p < r else 0))
    return out


def _is_tensor(v) -> bool:
    try:
        import torch
        return isinstance(v, torch.Tensor)
    except ImportError:  # pragma: no cover
        return False


def visible_devices() -> list:
    """Shard -> device map for the single-process family.

    ``KRYLOV_AMD_SHARDS="0,0,1"`` overrides (several shards may share a
    device); otherwise one shard per visible device, like MultiGpu.init
    (v3/gpu/common.py:62-66)."""
    env = os.environ.get("KRYLOV_AMD_SHARDS")
    if env:
        return [int(t) for t in env.split(",") if t.strip() != ""]
    n = _lib.device_count()
    if n <= 0:
        raise RuntimeError("no HIP device visible: the parallel_krylov_amd solvers need an "
                           "MI355X (gfx950) GPU; there is no CPU fallback")
    return list(range(n))


class Communicator:
    """RCCL communicator, one rank per GPU (replaces mpi4py on the hot path).

    Bootstrapped by broadcasting the RCCL unique id over ``bcast`` (a
    torch.distributed group or an mpi4py-like ``comm.bcast``)."""

    def __init__(self, rank: int, size: int, device: int, bcast):
        self.rank, self.size, self.device = rank, size, device
        uid = (ctypes.c_uint8 * 128)()
        if rank == 0:
            call("kr_comm_unique_id", uid)
        payload = bcast(bytes(uid))
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(payload)
        self.handle = ctypes.c_void_p()
        call("kr_comm_init", ctypes.byref(self.handle), uid, size, rank, device)

    @classmethod
    def from_torch(cls, group=None, device=None):
        import torch.distributed as dist
        rank, size = dist.get_rank(group), dist.get_world_size(group)
        if device is None:
            device = local_device(rank)

        def bcast(data):
            obj = [data]
            dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0)
                                       if group is not None else 0, group=group)
            return obj[0]
        return cls(rank, size, device, bcast)

    @classmethod
    def from_mpi(cls, comm, device=None):
        rank, size = comm.Get_rank(), comm.Get_size()
        if device is None:
            device = local_device(rank)
        return cls(rank, size, device, lambda data: comm.bcast(data, root=0))

    def close(self):
        if getattr(self, "handle", None):
            library().kr_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gpu_ids_range():
    """The rank's GPU range from GPU_IDS, ids[0]..ids[-1] inclusive, as the
    reference reads it (v3/gpu/mpi/common.py:77-83), or None when unset."""
    env = os.environ.get("GPU_IDS")
    if not env:
        return None
    ids = [int(t) for t in env.split(",") if t.strip() != ""]
    if not ids or ids[-1] < ids[0]:
        raise ValueError(f"GPU_IDS={env!r}: expected 'first,...,last' with last >= first")
    _warn_gpu_ids_over_local_rank(env)
    return list(range(ids[0], ids[-1] + 1))


_warned_gpu_ids = False


def _warn_gpu_ids_over_local_rank(env):
    """GPU_IDS takes precedence over LOCAL_RANK (the reference's launcher
    sets GPU_IDS per process). Under torchrun with several ranks a GPU_IDS
    exported for the whole job would put every rank on the same GPU(s):
    say so once, loudly, instead of silently stacking the ranks."""
    global _warned_gpu_ids
    if _warned_gpu_ids or int(os.environ.get("WORLD_SIZE", "1")) <= 1 \
            or "LOCAL_RANK" not in os.environ:
        return
    _warned_gpu_ids = True
    import warnings
    warnings.warn(f"GPU_IDS={env!r} overrides LOCAL_RANK={os.environ['LOCAL_RANK']} with "
                  f"WORLD_SIZE={os.environ['WORLD_SIZE']}: every rank whose environment holds "
                  "this GPU_IDS runs on these GPUs (set it per rank, or unset it to place "
                  "ranks by LOCAL_RANK)", RuntimeWarning, stacklevel=3)


def local_device(rank: int) -> int:
    """Device of this rank: the first id of GPU_IDS when it is set (the
    reference's per-rank GPU range, v3/gpu/mpi/common.py:77-83: the launcher
    sets it per process), else LOCAL_RANK (torchrun; more ranks than GPUs
    share them round-robin), else rank modulo the device count."""
    rng = gpu_ids_range()
    if rng is not None:
        return rng[0]
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"]) % max(_lib.device_count(), 1)
    n = _lib.device_count()
    return rank % max(n, 1)


@dataclass
class SolveOutput:
    x: list                      # per local shard: torch float64 tensor of own rows
    info: dict                   # reference info dict (time, nosl, residual[, khistory])
    converged: bool
    iterations: int
    final_k: int
    final_residual: float
    kernel_stats: list = field(default_factory=list)
    diverged: bool = False


def nan_guard_default() -> bool:
    """KRYLOV_AMD_NAN_GUARD=1: stop a solve at its first NaN/Inf residual
    (Status: diverged). Off by default: the reference runs a NaN trajectory on
    to maxiter (no test ever fires on NaN, v3/cpu/kskipmrr.py:39-42)."""
    return os.environ.get("KRYLOV_AMD_NAN_GUARD", "0") not in ("", "0")


class KrylovSystem:
    """A row-partitioned SPD system resident on HIP devices."""

    def __init__(self, n_global: int, row_begin, devices, comm: Communicator | None = None):
        torch = _torch()
        self.n_global = int(n_global)
        self.row_begin = [int(r) for r in row_begin]
        self.devices = [int(d) for d in devices]
        self.comm = comm
        if len(self.row_begin) != len(self.devices) + 1:
            raise ValueError("row_begin needs one more entry than devices")
        self._keep = []
        self._finalized = False
        self.handle = ctypes.c_void_p()
        for d in set(self.devices):
            torch.cuda.set_device(d)  # initialise the context before the library uses it
        devs = (ctypes.c_int * len(self.devices))(*self.devices)
        rb = (ctypes.c_int64 * len(self.row_begin))(*self.row_begin)
        call("kr_system_create", ctypes.byref(self.handle), self.n_global, len(self.devices),
             devs, rb, comm.handle if comm is not None else None)

    # ------------------------------------------------------------- building
    @property
    def nshards(self) -> int:
        return len(self.devices)

    def shard_rows(self, s: int):
        return self.row_begin[s], self.row_begin[s + 1]

    def device(self, s: int):
        return _torch().device("cuda", self.devices[s])

    def adopt_csr(self, s: int, block) -> None:
        """Upload the CSR block of shard s (its rows, GLOBAL column indices).

        ``block`` is a scipy sparse matrix/array (any format) or a
        (indptr, indices, data) triple. Column indices are uploaded as int32
        and rewritten on the device to the shard's halo-local numbering."""
        torch = _torch()
        if isinstance(block, tuple):
            indptr, indices, data = block
        else:
            import scipy.sparse as sp
            csr = sp.csr_matrix(block) if not sp.isspmatrix_csr(block) else block
            indptr, indices, data = csr.indptr, csr.indices, csr.data
        indptr = np.asarray(indptr)
        nnz = int(indptr[-1] - indptr[0])
        rp64 = nnz >= 2 ** 31 - 1 or indptr.dtype == np.int64 and int(indptr[-1]) >= 2 ** 31 - 1
        dev = self.device(s)
        def host(a, dt):  # contiguous + writable (memory-mapped files are read-only)
            return torch.from_numpy(np.require(a, dt, ["C", "W"]))

        t_rp = host(indptr, np.int64 if rp64 else np.int32).to(dev)
        t_col = host(indices, np.int32).to(dev)
        t_val = host(data, np.float64).to(dev)
        torch.cuda.synchronize(dev)
        self._keep += [t_rp, t_col, t_val]
        call("kr_system_adopt_csr", self.handle, s, t_rp.data_ptr(), int(rp64),
             t_col.data_ptr(), t_val.data_ptr())

    def adopt_dense(self, s: int, block) -> None:
        """Upload the dense row block of shard s (its rows x all N columns,
        a numpy array or tensor): the GEMV path (v3/gpu/common.py:100-101)."""
        torch = _torch()
        blk = block if _is_tensor(block) else np.asarray(block)
        if blk.ndim != 2 or blk.shape[1] != self.n_global:
            raise ValueError(f"dense block must be (rows, {self.n_global})")
        if _is_tensor(blk):
            t = blk.to(device=self.device(s), dtype=torch.float64).contiguous()
        else:
            t = torch.from_numpy(np.require(blk, np.float64, ["C", "W"])).to(self.device(s))
        torch.cuda.synchronize(self.device(s))
        self._keep.append(t)
        call("kr_system_adopt_dense", self.handle, s, t.data_ptr(), int(t.shape[1]))

    def set_matrix(self, A) -> None:
        """Distribute a whole matrix over the local shards (in-process
        family): scipy sparse (any format) as CSR, a dense ndarray/tensor as
        dense row blocks (GEMV), like the reference's two branches."""
        import scipy.sparse as sp
        if not sp.issparse(A) and (isinstance(A, np.ndarray) or _is_tensor(A)):
            for s in range(self.nshards):
                r0, r1 = self.shard_rows(s)
                self.adopt_dense(s, A[r0:r1])
            return
        A = sp.csr_matrix(A) if not sp.isspmatrix_csr(A) else A
        for s in range(self.nshards):
            r0, r1 = self.shard_rows(s)
            self.adopt_csr(s, A[r0:r1])

    def gen_poisson(self, n_side: int, dim: int) -> None:
        call("kr_system_gen_poisson", self.handle, dim, n_side)

    def gen_banded(self, h: int, width: int, seed: int, rowptr64: bool = False) -> None:
        call("kr_system_gen_banded", self.handle, h, width, seed, int(rowptr64))

    def finalize(self) -> None:
        call("kr_system_finalize", self.handle)
        self._finalized = True

    def shard_info(self, s: int) -> dict:
        v = [ctypes.c_int64() for _ in range(4)]
        call("kr_system_shard_info", self.handle, s, *[ctypes.byref(t) for t in v])
        return dict(zip(("n_local", "halo_lo", "halo_hi", "nnz"), [t.value for t in v]))

    def shard_layout(self, s: int) -> dict:
        """SpMV storage of shard s: mask_bits (0 = CSR columns), n_offsets,
        interior row range [interior_lo, interior_hi), dict_values (0 = 8-byte
        values, else the size of the value dictionary), code_bits (stencil
        SpMV: bits per slot code = bytes of A per row; 0 otherwise),
        code_patterns (stencil SpMV: distinct 512-row code blocks read from a
        table instead of the per-row stream; 0 = per-row stream), dia_sym
        (1: symmetric diagonal-offset values, lower entries read as the
        mirrored upper ones), dia_full_blocks / dia_full_first (DIA walk: the
        run of 256-row blocks whose all-ones offset masks are not loaded),
        box (1: constant-coefficient 7-point box stencil with n = 512, the
        k-skip basis pairs can run matrix-free)."""
        mb, no = ctypes.c_int(), ctypes.c_int()
        lo, hi = ctypes.c_int64(), ctypes.c_int64()
        call("kr_system_shard_layout", self.handle, s, ctypes.byref(mb), ctypes.byref(no),
             ctypes.byref(lo), ctypes.byref(hi))
        dv, cb, ds, cp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        bx = ctypes.c_int()
        call("kr_system_shard_box", self.handle, s, ctypes.byref(bx))
        call("kr_system_shard_values", self.handle, s, ctypes.byref(dv))
        call("kr_system_shard_codes", self.handle, s, ctypes.byref(cb))
        call("kr_system_shard_code_patterns", self.handle, s, ctypes.byref(cp))
        call("kr_system_shard_dia_sym", self.handle, s, ctypes.byref(ds))
        fb0, fbn = ctypes.c_int64(), ctypes.c_int64()
        call("kr_system_shard_dia_full_blocks", self.handle, s, ctypes.byref(fb0), ctypes.byref(fbn))
        return dict(mask_bits=mb.value, n_offsets=no.value, interior_lo=lo.value,
                    interior_hi=hi.value, dict_values=dv.value, code_bits=cb.value,
                    code_patterns=cp.value, dia_sym=ds.value, dia_full_blocks=fbn.value,
                    dia_full_first=fb0.value, box=bx.value)

    def shard_sched(self, s: int) -> dict:
        """Launch geometry of shard s: elementwise and SpMV grids plus the
        interior rows of the split SpMV -- what fixes the engine's dot-product
        summation order (oracle/gpu_order.py restates it for the tests)."""
        g, sg, sw, fm = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        call("kr_system_shard_sched", self.handle, s, ctypes.byref(g), ctypes.byref(sg),
             ctypes.byref(sw), ctypes.byref(fm))
        lay = self.shard_layout(s)
        return dict(n=self.row_begin[s + 1] - self.row_begin[s], grid=g.value,
                    spmv_grid=sg.value, int_lo=lay["interior_lo"], int_hi=lay["interior_hi"],
                    stencil_walk=sw.value,
                    dia_walk=1 if _lib.KR_FORMAT[fm.value] == "dia_walk" else 0)

    def shard_format(self, s: int) -> str:
        """The SpMV kernel family serving shard s: "csr" (row walk), "stencil",
        "dia" (diagonal-offset values), "dia_walk" (symmetric diagonal-offset
        values, row-block walk with the mirrors in LDS) or "dense" (GEMV)."""
        fm = ctypes.c_int()
        call("kr_system_shard_sched", self.handle, s, None, None, None, ctypes.byref(fm))
        return _lib.KR_FORMAT[fm.value]

    def csr_pointers(self, s: int) -> dict:
        """Raw device CSR of shard s (local columns after finalize)."""
        rp, col, val = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        rp64, pad = ctypes.c_int(), ctypes.c_int64()
        call("kr_system_csr", self.handle, s, ctypes.byref(rp), ctypes.byref(rp64),
             ctypes.byref(col), ctypes.byref(val), ctypes.byref(pad))
        return dict(rowptr=rp.value, rowptr64=rp64.value, col=col.value, val=val.value,
                    pad=pad.value)

    # ------------------------------------------------------------- vectors
    def split(self, v) -> list:
        """Own-row device tensors of a full-length host/device vector."""
        torch = _torch()
        out = []
        for s in range(self.nshards):
            r0, r1 = self.shard_rows(s)
            seg = v[r0:r1]
            if isinstance(seg, np.ndarray):
                seg = torch.from_numpy(np.ascontiguousarray(seg, dtype=np.float64))
            out.append(seg.to(device=self.device(s), dtype=torch.float64).contiguous())
        return out

    def rhs(self, seed: int) -> list:
        """Synthetic b (2u-1, counter hash) generated on the device per shard."""
        torch = _torch()
        out = []
        for s in range(self.nshards):
            r0, r1 = self.shard_rows(s)
            t = torch.empty(r1 - r0, dtype=torch.float64, device=self.device(s))
            call("kr_fill_rhs", self.handle, s, seed, t.data_ptr())
            out.append(t)
        return out

    def gather(self, parts) -> "object":
        torch = _torch()
        if len(parts) == 1:
            return parts[0]
        d0 = self.device(0)
        return torch.cat([p.to(d0) for p in parts])

    # ------------------------------------------------------------- compute
    def spmv(self, x_parts) -> list:
        """Distributed y = A x through the halo exchange (own rows in/out)."""
        torch = _torch()
        ys = [torch.empty_like(x) for x in x_parts]
        for s in range(self.nshards):
            torch.cuda.synchronize(self.device(s))
        call("kr_system_spmv", self.handle, ptr_array([x.data_ptr() for x in x_parts]),
             ptr_array([y.data_ptr() for y in ys]))
        return ys

    def set_precond(self, d_parts=None) -> None:
        """Jacobi diagonal (own rows per shard, float64 device tensors) of the
        preconditioned / pipelined CG sessions begun afterwards
        (kr_solve_set_precond); None restores the identity."""
        if d_parts is None:
            self._precond = None
            call("kr_solve_set_precond", self.handle, None)
            return
        self._precond = list(d_parts)  # kept alive until the next call
        for s, t in enumerate(self._precond):
            n_own = self.row_begin[s + 1] - self.row_begin[s]
            if t.numel() != n_own or t.dtype != _torch().float64 or not t.is_cuda:
                raise ValueError(f"preconditioner part {s}: need {n_own} float64 device values")
        call("kr_solve_set_precond", self.handle, ptr_array([t.data_ptr() for t in self._precond]))

    def set_precond_ilu(self, factors) -> None:
        """ILU preconditioner of the preconditioned / pipelined CG sessions
        begun afterwards (kr_solve_set_precond_ilu; one-shard systems):
        ``factors`` = (L, U, perm_r, perm_c) with L, U scipy CSR factors incl.
        the diagonal and SuperLU's permutations (A ~ Pr^T L U Pc^T); None
        clears it. The library validates and copies the host arrays."""
        if factors is None:
            call("kr_solve_set_precond_ilu", self.handle, 0, None, None, None, None, None, None,
                 None, None)
            return
        L, U, perm_r, perm_c = factors
        n = self.n_global

        def csr(T, name):
            import scipy.sparse as sp
            T = sp.csr_matrix(T)
            if T.shape != (n, n):
                raise ValueError(f"ILU {name}: shape {T.shape}, the system is {n} x {n}")
            T.sum_duplicates()
            T.sort_indices()
            return (np.ascontiguousarray(T.indptr, np.int64),
                    np.ascontiguousarray(T.indices, np.int32),
                    np.ascontiguousarray(T.data, np.float64))

        lr, lc, lv = csr(L, "L")
        ur, uc, uv = csr(U, "U")
        pr = np.ascontiguousarray(perm_r, np.int64)
        pc = np.ascontiguousarray(perm_c, np.int64)
        if pr.shape != (n,) or pc.shape != (n,):
            raise ValueError(f"ILU permutations must have {n} entries")
        ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        call("kr_solve_set_precond_ilu", self.handle, n, ptr(lr), ptr(lc), ptr(lv), ptr(ur),
             ptr(uc), ptr(uv), ptr(pr), ptr(pc))

    def solve(self, method: str, b_parts, x0_parts=None, tol=1e-5, maxiter=None, k=0,
              profile=False, max_outer=None, nan_guard=None) -> SolveOutput:
        """Run one solver to completion (or for ``max_outer`` outer steps).
        nan_guard: stop at the first non-finite residual (default:
        KRYLOV_AMD_NAN_GUARD, off = the reference's run-on semantics)."""
        torch = _torch()
        if not self._finalized:
            self.finalize()
        if method not in _lib.KR_METHOD:
            raise ValueError(f"unknown method {method!r}")
        self._guard = nan_guard_default() if nan_guard is None else bool(nan_guard)
        prm = _lib.SolveParams(method=_lib.KR_METHOD[method], k=int(k or 0), tol=float(tol),
                               maxiter=-1 if maxiter is None else int(maxiter),
                               profile=int(profile) if profile else 0,
                               nan_guard=int(self._guard))
        for s in range(self.nshards):
            torch.cuda.synchronize(self.device(s))
        b_arr = ptr_array([t.data_ptr() for t in b_parts])
        x0_arr = ptr_array([t.data_ptr() for t in x0_parts]) if x0_parts is not None else None
        call("kr_solve_begin", self.handle, ctypes.byref(prm), b_arr, x0_arr)
        done = ctypes.c_int(0)
        call("kr_solve_step", self.handle, (1 << 62) if max_outer is None else int(max_outer),
             ctypes.byref(done))
        return self.finish(method)

    def begin(self, method, b_parts, x0_parts=None, tol=1e-5, maxiter=None, k=0,
              profile=False, nan_guard=None) -> None:
        torch = _torch()
        if not self._finalized:
            self.finalize()
        self._guard = nan_guard_default() if nan_guard is None else bool(nan_guard)
        prm = _lib.SolveParams(method=_lib.KR_METHOD[method], k=int(k or 0), tol=float(tol),
                               maxiter=-1 if maxiter is None else int(maxiter),
                               profile=int(profile) if profile else 0,
                               nan_guard=int(self._guard))
        for s in range(self.nshards):
            torch.cuda.synchronize(self.device(s))
        b_arr = ptr_array([t.data_ptr() for t in b_parts])
        x0_arr = ptr_array([t.data_ptr() for t in x0_parts]) if x0_parts is not None else None
        call("kr_solve_begin", self.handle, ctypes.byref(prm), b_arr, x0_arr)

    def step(self, n_outer: int) -> bool:
        done = ctypes.c_int(0)
        call("kr_solve_step", self.handle, int(n_outer), ctypes.byref(done))
        return bool(done.value)

    def finish(self, method: str) -> SolveOutput:
        torch = _torch()
        xs = [torch.empty(self.row_begin[s + 1] - self.row_begin[s], dtype=torch.float64,
                          device=self.device(s)) for s in range(self.nshards)]
        # the engine writes x on its own streams: torch's pending work on the
        # recycled memory must be done first
        for dv in sorted(set(self.devices)):
            torch.cuda.synchronize(dv)
        res = _lib.SolveResult()
        call("kr_solve_end", self.handle, ptr_array([x.data_ptr() for x in xs]),
             ctypes.byref(res))
        n = int(res.entries)
        residual = np.zeros(n, np.float64)
        nosl = np.zeros(n, np.int64)
        khist = np.zeros(n, np.int64)
        call("kr_solve_history", self.handle,
             residual.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
             nosl.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
             khist.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), n)
        info = {"time": float(res.time_s), "nosl": nosl, "residual": residual}
        if method == "adaptivekskipmrr":
            info["khistory"] = khist
        if getattr(self, "_guard", False):  # only with the (non-reference) guard on
            info["diverged"] = bool(res.diverged)
        return SolveOutput(x=xs, info=info, converged=bool(res.converged),
                           iterations=int(res.iterations), final_k=int(res.final_k),
                           final_residual=float(res.final_residual),
                           kernel_stats=self.kernel_stats(), diverged=bool(res.diverged))

    def reset_kernel_stats(self) -> None:
        call("kr_solve_kernel_stats_reset", self.handle)

    def kernel_stats(self) -> list:
        cap = 64
        arr = (_lib.KernelStat * cap)()
        cnt = ctypes.c_int(0)
        call("kr_solve_kernel_stats", self.handle, arr, cap, ctypes.byref(cnt))
        return [dict(name=arr[i].name.decode(), launches=int(arr[i].launches),
                     total_ms=float(arr[i].total_ms),
                     bytes_per_launch=float(arr[i].bytes_per_launch),
                     shards=int(arr[i].shards))
                for i in range(min(cnt.value, cap))]

    def close(self) -> None:
        if getattr(self, "handle", None):
            library().kr_system_destroy(self.handle)
            self.handle = None
            self._keep = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def system_from_matrix(A, devices=None) -> KrylovSystem:
    """Single-process system over ``devices`` (default: all visible GPUs)."""
    import scipy.sparse as sp
    devices = visible_devices() if devices is None else list(devices)
    if sp.issparse(A):
        A = sp.csr_matrix(A) if not sp.isspmatrix_csr(A) else A
    n = A.shape[0]
    sysm = KrylovSystem(n, balanced_partition(n, len(devices)), devices)
    sysm.set_matrix(A)
    sysm.finalize()
    return sysm
