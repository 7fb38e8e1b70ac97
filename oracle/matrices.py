"""Synthetic SPD systems on the host (TEST INFRASTRUCTURE ONLY).

This module belongs to the oracle: only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it. The product path
(``parallel-krylov_amd``) generates the same matrices on the device
(``kr_system_gen_poisson`` / ``kr_system_gen_banded``); the definitions below
are the specification both follow, integer for integer, so the host and device
CSR arrays are bit-identical (checked in tests/test_gpu_kernels.py).

The reference ships no matrices (``.gitignore:14-17`` drops ``*.npz``/``*.mtx``);
SURVEY.md §8d defines the synthetic families:

* Poisson: ``kronsum`` of ``tridiag(-1, 2, -1)`` (2D 5-point / 3D 7-point),
  row-major lexicographic order, sorted columns.
* Symmetric random banded: one set of ``h`` distinct offsets in ``[1, W]``
  shared by all rows, ``a(i, i±o) = -u``, diagonal ``= sum|off| + 1``.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

_MASK = (1 << 64) - 1
_K1, _K2, _K3 = 0x9E3779B97F4A7C15, 0xC2B2AE3D27D4EB4F, 0x165667B19E3779F9


def _mix64_np(x: np.ndarray) -> np.ndarray:
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def mix64(x: int) -> int:
    """Scalar splitmix64 finaliser (kr_hash.h ``mix64``)."""
    x = (x + 0x9E3779B97F4A7C15) & _MASK
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _MASK
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _MASK
    return x ^ (x >> 31)


def unit_uniform(seed: int, a, b) -> np.ndarray:
    """u in [0, 1) with 53 random bits (kr_hash.h ``unit_uniform``)."""
    with np.errstate(over="ignore"):
        a = np.asarray(a, dtype=np.uint64)
        b = np.asarray(b, dtype=np.uint64)
        key = (np.uint64((seed * _K1) & _MASK) ^ (a * np.uint64(_K2)) ^ (b * np.uint64(_K3)))
        return (_mix64_np(key) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def rhs(n: int, seed: int, row0: int = 0) -> np.ndarray:
    """Synthetic right-hand side b_i = 2u - 1 (kr_hash.h ``rhs_value``)."""
    i = np.arange(row0, row0 + n, dtype=np.uint64)
    return 2.0 * unit_uniform(seed, i, 0xB5) - 1.0


def _pool_map(fn, items):
    """fn over items on min(16, affinity cores) threads (fn writes disjoint slices)."""
    import os
    from concurrent.futures import ThreadPoolExecutor
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    if threads == 1 or len(items) < 2:
        for it in items:
            fn(it)
        return
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(fn, items))


def poisson(n_side: int, dim: int, dtype_index=np.int32) -> sp.csr_matrix:
    """5-point (dim=2) / 7-point (dim=3) Poisson matrix, sorted CSR."""
    if dim not in (2, 3):
        raise ValueError("dim must be 2 or 3")
    N = n_side ** dim
    strides = [n_side ** d for d in range(dim)]
    offsets = [-strides[d] for d in reversed(range(dim))] + [0] + strides
    values = np.array([-1.0] * dim + [2.0 * dim] + [-1.0] * dim)

    def stencil(g):
        """(cols, mask) of rows g, slots in sorted column order."""
        coords = [(g // s) % n_side for s in strides]
        masks = [coords[d] > 0 for d in reversed(range(dim))] + [np.ones(g.size, bool)] + \
                [coords[d] < n_side - 1 for d in range(dim)]
        return np.stack([g + o for o in offsets], axis=1), np.stack(masks, axis=1)

    # Rows in chunks (bounded temporaries at 512^3), chunks on a thread pool:
    # numpy releases the GIL in these array operations, and every chunk writes
    # its own slice, so the arrays are the sequential build's bit for bit
    # (512^3: 64 s -> 15 s on 8 cores; the bench's cpu_baseline and the C4
    # parity test build this matrix).
    chunk = 1 << 20
    starts = range(0, N, chunk)
    indptr = np.zeros(N + 1, dtype=np.int64)

    def count(c0):
        g = np.arange(c0, min(N, c0 + chunk), dtype=np.int64)
        _, M = stencil(g)
        indptr[c0 + 1:c0 + 1 + g.size] = M.sum(axis=1)

    _pool_map(count, starts)
    np.cumsum(indptr, out=indptr)
    nnz = int(indptr[-1])
    indices = np.empty(nnz, dtype=dtype_index)
    data = np.empty(nnz, dtype=np.float64)

    def fill(c0):
        g = np.arange(c0, min(N, c0 + chunk), dtype=np.int64)
        C, M = stencil(g)
        s0, s1 = indptr[c0], indptr[c0 + g.size]
        indices[s0:s1] = C[M]
        data[s0:s1] = np.broadcast_to(values, C.shape)[M]

    _pool_map(fill, starts)
    A = sp.csr_matrix((data, indices, indptr.astype(dtype_index)), shape=(N, N))
    A.has_sorted_indices = True
    return A


def banded_offsets(h: int, width: int, seed: int) -> np.ndarray:
    """h distinct offsets in [1, width] (kr_capi.cpp ``banded_offsets``)."""
    pool = list(range(1, width + 1))
    for t in range(h):
        r = mix64((seed * 0x2545F4914F6CDD1D + t) & _MASK)
        j = t + r % (width - t)
        pool[t], pool[j] = pool[j], pool[t]
    return np.array(sorted(pool[:h]), dtype=np.int64)


def banded_arrays(N: int, h: int, width: int, seed: int):
    """The symmetric random banded SPD matrix as raw CSR arrays (indptr int64,
    indices int32, data float64) -- the arrays ``banded`` wraps. Rows are built
    in chunks on a thread pool (numpy releases the GIL; each chunk writes its
    own slice), so the arrays are the sequential build's bit for bit; C5's
    N = 50M (3.15 G entries) needs the int64 indptr."""
    off = banded_offsets(h, width, seed)
    # row i's entries: lower (offsets descending = columns ascending), the
    # diagonal, upper (offsets ascending); a slot exists when its column does

    def present(g):
        ml = [(g - o) >= 0 for o in off[::-1]]
        mu = [(g + o) < N for o in off]
        return ml, mu

    chunk = 1 << 20
    starts = range(0, N, chunk)
    indptr = np.zeros(N + 1, dtype=np.int64)

    def count(c0):
        g = np.arange(c0, min(N, c0 + chunk), dtype=np.int64)
        ml, mu = present(g)
        indptr[c0 + 1:c0 + 1 + g.size] = 1 + np.sum(ml, axis=0) + np.sum(mu, axis=0)

    _pool_map(count, starts)
    np.cumsum(indptr, out=indptr)
    nnz = int(indptr[-1])
    indices = np.empty(nnz, dtype=np.int32)
    data = np.empty(nnz, dtype=np.float64)

    def fill(c0):
        g = np.arange(c0, min(N, c0 + chunk), dtype=np.int64)
        cols, vals, masks = [], [], []
        for o in off[::-1]:  # lower part, ascending column
            lo = g - o
            m = lo >= 0
            cols.append(lo)
            vals.append(-unit_uniform(seed, np.where(m, lo, 0), o))
            masks.append(m)
        upper = []
        for o in off:
            hi = g + o
            m = hi < N
            upper.append((hi, -unit_uniform(seed, g, o), m))
        # diagonal: sum of |off| in column order (lower then upper), then + 1
        s = np.zeros(g.size)
        for v, m in zip(vals, masks):
            s = s + np.where(m, np.abs(v), 0.0)
        for _, v, m in upper:
            s = s + np.where(m, np.abs(v), 0.0)
        cols.append(g); vals.append(s + 1.0); masks.append(np.ones(g.size, bool))
        for c, v, m in upper:
            cols.append(c); vals.append(v); masks.append(m)
        C = np.stack(cols, axis=1)
        V = np.stack(vals, axis=1)
        M = np.stack(masks, axis=1)
        s0, s1 = indptr[c0], indptr[c0 + g.size]
        indices[s0:s1] = C[M]
        data[s0:s1] = V[M]

    _pool_map(fill, starts)
    return indptr, indices, data


def banded(N: int, h: int, width: int, seed: int, dtype_index=np.int32) -> sp.csr_matrix:
    """Symmetric random banded SPD matrix (device twin: banded_fill_kernel)."""
    indptr, indices, data = banded_arrays(N, h, width, seed)
    A = sp.csr_matrix((data, indices.astype(dtype_index, copy=False),
                       indptr.astype(dtype_index, copy=False)), shape=(N, N))
    A.has_sorted_indices = True
    return A


class ParCSR:
    """A CSR operator for the oracle whose ``dot`` is oracle/csrmv.c: every row
    summed in stored order from 0.0 like scipy's csr_matvec (bitwise; pinned
    in tests/test_oracle.py), rows spread over OpenMP threads. For the
    full-size parity tests, where scipy's one-thread matvec over billions of
    entries would take minutes (C5: 3.15 G entries at N = 50M). Needs
    oracle/liboracle_csrmv.so (oracle/build.sh, run by build())."""

    _lib = None

    @staticmethod
    def lib_path():
        import os
        return os.path.join(os.path.dirname(os.path.abspath(__file__)), "liboracle_csrmv.so")

    @staticmethod
    def available():
        """True when oracle/build.sh has built the helper (build() runs it;
        its failure does not fail the product build)."""
        import os
        return os.path.exists(ParCSR.lib_path())

    def __init__(self, indptr, indices, data, shape):
        import ctypes
        if ParCSR._lib is None:
            if not ParCSR.available():
                raise FileNotFoundError(f"{ParCSR.lib_path()} is missing: run oracle/build.sh")
            lib = ctypes.CDLL(ParCSR.lib_path())
            P = ctypes.c_void_p
            lib.oracle_csrmv.argtypes = [ctypes.c_int64, P, P, P, P, P]
            lib.oracle_csrmv.restype = None
            ParCSR._lib = lib
        self.indptr = np.ascontiguousarray(indptr, dtype=np.int64)
        self.indices = np.ascontiguousarray(indices, dtype=np.int32)
        self.data = np.ascontiguousarray(data, dtype=np.float64)
        self.shape = shape

    @classmethod
    def from_scipy(cls, A):
        A = A.tocsr()
        return cls(A.indptr, A.indices, A.data, A.shape)

    def dot(self, v):
        v = np.ascontiguousarray(v, dtype=np.float64)
        y = np.empty(self.shape[0], dtype=np.float64)
        ParCSR._lib.oracle_csrmv(self.shape[0], self.indptr.ctypes.data, self.indices.ctypes.data,
                                 self.data.ctypes.data, v.ctypes.data, y.ctypes.data)
        return y

    __matmul__ = dot


def csr_digest(A: sp.csr_matrix) -> str:
    """sha256 over (indptr as int64, indices as int64, data as float64)."""
    import hashlib
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(A.indptr, dtype=np.int64).tobytes())
    h.update(np.ascontiguousarray(A.indices, dtype=np.int64).tobytes())
    h.update(np.ascontiguousarray(A.data, dtype=np.float64).tobytes())
    return h.hexdigest()
