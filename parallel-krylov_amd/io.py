"""Matrix ingest: on-disk formats -> sharded device CSR.

The reference's MPI drivers hand each rank a row block read from ``.npz``
(scipy sparse) or ``.npy`` (dense) files (``v3/gpu/mpi/common.py:123-129``;
the files themselves are gitignored, ``.gitignore:14-17``). Here:

* ``read_rows(path, r0, r1)`` returns rows [r0, r1) of a stored matrix as
  the reference would hold them: a ``.npz`` (scipy CSR) block as
  (indptr, indices, data, n_cols) with GLOBAL columns, a ``.npy`` block as a
  DENSE float64 ndarray -- the reference keeps dense row blocks dense
  (``v3/gpu/mpi/common.py:123-125``, cupy dgemv), so they run the GEMV kernel
  here too (8 B per entry streamed, no index stream). For an uncompressed
  ``.npz`` (``scipy.sparse.save_npz(..., compressed=False)``) or a ``.npy``,
  the arrays are memory-mapped, so a rank touches only its own block's bytes;
  a compressed ``.npz`` is inflated once. ``read_csr_rows`` is the CSR view
  of either (a ``.npy`` block converted).
* ``load_system(path, devices=None)`` builds a single-process
  ``KrylovSystem`` (one shard per device) from a file: CSR shards for a
  ``.npz``, dense shards for a ``.npy``.
* ``load_local_block(path, comm)`` is the MPI-family helper: this rank's
  balanced row block (scipy CSR, or a dense ndarray for a ``.npy``), ready
  for ``v3.gpu.mpi.<method>(comm, local_A, b)``.

Files are read with ``allow_pickle=False`` only.
"""
from __future__ import annotations

import os
import zipfile

import numpy as np

from .system import KrylovSystem, balanced_partition, visible_devices


def _npz_member_mmap(path, name):
    """Memory-map one array stored uncompressed inside an .npz, or None."""
    with zipfile.ZipFile(path) as zf:
        info = zf.getinfo(name + ".npy")
        if info.compress_type != zipfile.ZIP_STORED:
            return None
        with open(path, "rb") as f:
            f.seek(info.header_offset)
            local = f.read(30)
            name_len = int.from_bytes(local[26:28], "little")
            extra_len = int.from_bytes(local[28:30], "little")
            start = info.header_offset + 30 + name_len + extra_len
            f.seek(start)
            version = np.lib.format.read_magic(f)
            if version == (1, 0):
                shape, fortran, dtype = np.lib.format.read_array_header_1_0(f)
            else:
                shape, fortran, dtype = np.lib.format.read_array_header_2_0(f)
            offset = f.tell()
    if fortran or dtype.hasobject:
        return None
    return np.memmap(path, dtype=dtype, mode="r", offset=offset, shape=shape)


def _npz_array(path, name):
    arr = _npz_member_mmap(path, name)
    if arr is not None:
        return arr
    with np.load(path, allow_pickle=False) as z:
        return z[name]


def matrix_shape(path) -> tuple:
    if path.endswith(".npy"):
        return tuple(np.load(path, mmap_mode="r", allow_pickle=False).shape)
    with np.load(path, allow_pickle=False) as z:
        fmt = z["format"].item()
        fmt = fmt.decode() if isinstance(fmt, bytes) else str(fmt)
        if fmt != "csr":
            raise ValueError(f"{path}: only CSR .npz files are supported (found {fmt!r})")
        return tuple(int(v) for v in z["shape"])


def read_rows(path: str, r0: int, r1: int):
    """Rows [r0, r1) of a stored matrix: a dense float64 ndarray for a .npy,
    else (indptr from 0, indices, data, n_cols) of the CSR block."""
    if path.endswith(".npy"):
        dense = np.load(path, mmap_mode="r", allow_pickle=False)
        return np.ascontiguousarray(dense[r0:r1], dtype=np.float64)
    return read_csr_rows(path, r0, r1)


def read_csr_rows(path: str, r0: int, r1: int):
    """Rows [r0, r1) of a stored matrix as CSR: (indptr from 0, indices, data,
    n_cols); a .npy block is converted (its nonzero entries)."""
    if path.endswith(".npy"):
        dense = np.load(path, mmap_mode="r", allow_pickle=False)
        blk = np.asarray(dense[r0:r1], dtype=np.float64)
        rows, cols = np.nonzero(blk)
        indptr = np.zeros(r1 - r0 + 1, dtype=np.int64)
        np.add.at(indptr, rows + 1, 1)
        np.cumsum(indptr, out=indptr)
        return indptr, cols.astype(np.int32), blk[rows, cols], dense.shape[1]
    shape = matrix_shape(path)
    indptr_all = _npz_array(path, "indptr")
    lo, hi = int(indptr_all[r0]), int(indptr_all[r1])
    indptr = np.asarray(indptr_all[r0:r1 + 1], dtype=np.int64) - lo
    indices = np.asarray(_npz_array(path, "indices")[lo:hi], dtype=np.int32)
    data = np.asarray(_npz_array(path, "data")[lo:hi], dtype=np.float64)
    return indptr, indices, data, shape[1]


def load_system(path: str, devices=None) -> KrylovSystem:
    """Single-process sharded system straight from a file (one row block per
    device; each block is read and uploaded on its own)."""
    n, m = matrix_shape(path)
    if n != m:
        raise ValueError(f"{path}: matrix is {n}x{m}, the solvers need a square system")
    devices = visible_devices() if devices is None else list(devices)
    sysm = KrylovSystem(n, balanced_partition(n, len(devices)), devices)
    for s in range(sysm.nshards):
        r0, r1 = sysm.shard_rows(s)
        blk = read_rows(path, r0, r1)
        if isinstance(blk, np.ndarray):  # .npy: dense row block, GEMV
            sysm.adopt_dense(s, blk)
        else:
            indptr, indices, data, _ = blk
            sysm.adopt_csr(s, (indptr, indices, data))
    sysm.finalize()
    return sysm


def load_local_block(path: str, comm=None):
    """This rank's balanced row block for the MPI family, as the reference
    holds it: a scipy CSR matrix (global columns) for a .npz, a dense ndarray
    for a .npy (v3/gpu/mpi/common.py:123-125):
    ``x, info = kskipmrr(comm, load_local_block(p, comm), b)``."""
    import scipy.sparse as sp
    if comm is not None and hasattr(comm, "Get_rank"):
        rank, size = comm.Get_rank(), comm.Get_size()
    else:
        import torch.distributed as dist
        rank, size = dist.get_rank(comm), dist.get_world_size(comm)
    n, m = matrix_shape(path)
    part = balanced_partition(n, size)
    blk = read_rows(path, part[rank], part[rank + 1])
    if isinstance(blk, np.ndarray):
        return blk
    indptr, indices, data, ncols = blk
    return sp.csr_matrix((data, indices, indptr), shape=(part[rank + 1] - part[rank], ncols))


def save_npz_uncompressed(path: str, A) -> None:
    """scipy.sparse.save_npz(..., compressed=False): the layout read_csr_rows
    memory-maps."""
    import scipy.sparse as sp
    sp.save_npz(path, sp.csr_matrix(A), compressed=False)
    if not os.path.exists(path) and os.path.exists(path + ".npz"):
        os.replace(path + ".npz", path)
