"""The engine's dot-product summation order, restated in numpy (TEST INFRASTRUCTURE ONLY).

The oracle (oracle/v3cpu.py) is bitwise the reference given the reference's
dot products (numpy/OpenBLAS order). The GPU path computes every SpMV row,
vector update and scalar recurrence bitwise like the reference; ONLY the
summation order of its dot products differs. For k-skip
methods with large k the trajectory amplifies that rounding difference into
a different history (adaptive k-skip MrR's rollbacks are rounding events), so
a history check against the reference fixtures is only loose there.

This module restates the engine's fixed summation order so that the oracle
can run with EXACTLY the GPU's dot products: ``with gpu_order.patched(sched):
v3cpu.adaptivekskipmrr(...)`` must then equal the GPU run bit for bit --
nosl, khistory, every residual entry and x -- through every rollback.

What is restated (single process; shards in shard order, RCCL ranks in rank
order, as System::reduce and scalar_kernel sum them):

* SpMV epilogue products (kr_spmv.h ``epi_products``), row-walk kernels:
  lane ``tid`` of workgroup ``b`` owns rows ``rb*256 + tid`` of the row
  blocks RowSched gives it (XCD-aware when the grid is a multiple of 8,
  kr_spmv.h RowSched::init) and accumulates ``acc = acc + p[row]`` from 0.0
  in visit order. Stencil kernel (kr_stencil.h, shards with stencil codes):
  512-row blocks, lane ``tid`` owns rows ``2 tid`` and ``2 tid + 1`` and
  adds them in that order; workgroup (XCD q, plane segment s, position p)
  visits the blocks z*P + p of its planes;
  ``block_reduce_store`` folds each wave with the ``__shfl_down`` tree
  (offsets 32..1) and the 4 waves as ``((w0 + w1) + w2) + w3``. A sharded
  system splits each SpMV into an interior launch and one boundary launch that
  ADDS its partials (kr_engine.cpp System::spmv).
* Elementwise-kernel products (kr_kernels.hip ``ew_kernel``, 16-byte pairs):
  thread ``t0`` adds ``p[2q]`` then ``p[2q+1]`` for q = t0, t0 + stride, ...;
  an odd tail element goes to thread 0 of block 0 last.
* Finalize (kr_kernels.hip ``block_slot_sum``): thread i sums partials
  i, i+256, ... from 0.0, then the same wave tree and wave order; the host
  adds the shards' totals to 0.0 in order.

Which kernel computes which dot is a property of the method: in k-skip MrR,
adaptive k-skip MrR and k-skip CG every dot after ||b|| comes from an SpMV
epilogue (EPI_BMINUS, EPI_XY, EPI_HEAD_*, EPI_DUAL_*); ||b|| comes from
EW_DOT. ``patched`` installs exactly that mapping.
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass

import numpy as np

BLOCK = 256  # kBlock (kr_internal.h)


@dataclass
class ShardSched:
    """One shard's launch geometry (KrylovSystem.shard_sched)."""
    n: int           # own rows
    grid: int        # elementwise-kernel workgroups (default_grid)
    spmv_grid: int   # SpMV workgroups (spmv_grid_for)
    int_lo: int = 0  # interior rows [int_lo, int_hi) of the split SpMV
    int_hi: int = 0
    stencil_walk: int = 0  # P > 0: the stencil SpMV (512-row blocks), 0: row walk
    dia_walk: int = 0      # 1: the symmetric DIA walk (kr_spmv.h spmv_diawalk_kernel)


def _stencil_walk(blk, r0, nnz_row_mean):
    """kr_engine.cpp build_masks / build_vdict / build_stencil: P of the
    stencil SpMV for this row block, or 0 (row walk)."""
    n = blk.shape[0]
    if n < 2 or n % 2 or nnz_row_mean >= 12.0 or blk.nnz < 8:
        return 0
    rows = np.repeat(np.arange(n), np.diff(blk.indptr))
    offs = np.unique(blk.indices.astype(np.int64) - (r0 + rows))
    if offs.size == 0 or offs.size > 8:
        return 0
    if np.unique(blk.data.view(np.uint64)).size > 255:
        return 0
    W = max([int(o) for o in offs if o > 0 and o % 512 == 0 and -o in offs], default=0)
    if W == 0:
        return 0
    far = [int(o) for o in offs if o not in (0, W, -W) and abs(o) > 2]
    if len(far) > 4 or any(o % 2 for o in far):
        return 0
    return W // 512


def stencil_pm(P):
    """kr_engine.cpp stencil_pm: the position-major walk (P % 8 == 0)."""
    return P % 8 == 0


def stencil_grid(rows, P, zmax=0):
    """kr_engine.cpp stencil_grid: position-major P x Zt segments, or
    plane-major 8 XCDs x P positions x Z segments. zmax > 0 caps Z: the
    products-only dual's grid on position-major shards (Shard::spmv_grid_po,
    zmax 16), which differs from the general grid only on shards of >= 512
    planes; the emulation below
    sums every SpMV's products over the general grid, so it is exact for
    shards under that size (test_products_only_grid_matches_below_512_planes)."""
    nrb = -(-rows // 512)
    planes = -(-nrb // P)
    pm = stencil_pm(P)
    cols = P if pm else 8 * P
    Z = 1
    if pm:
        while cols * Z < 16384 and planes // (Z * 2) >= 16:
            Z *= 2
        while cols * Z < 1024 and planes // (Z * 2) >= 8:
            Z *= 2
    else:
        while cols * Z < 2048 and planes // (8 * Z * 2) >= 8:
            Z *= 2
    if zmax > 0 and Z > zmax:
        Z = zmax
    return cols * Z


DIA_WALK_H = (7, 13, 15, 31)  # kr_internal.h dia_walk_h_supported


def dia_walk_grid(rows, nm, cus=256):
    """kr_engine.cpp dia_walk_grid: the resident workgroups of the walk kernel
    (LDS: h x 2 KiB of mirror buffers + two 6 KiB x windows + 1 KiB, 160 KiB per CU)."""
    nrb = max(1, -(-rows // BLOCK))
    lds = 8 * ((nm // 2 + 1) * BLOCK + 2 * 768) + 1024
    h = nm // 2
    by_regs = 2 if h >= 16 else 3 if h >= 8 else 4  # waves per SIMD by VGPRs
    per_cu = max(1, min(by_regs, 160 * 1024 // lds))
    return min(nrb, cus * per_cu)


def _dia_walk(blk, r0, n):
    """kr_engine.cpp build_masks: 0, or nm of a shard served by the symmetric
    DIA walk -- diagonal-offset values (mean >= 12 nnz/row, <= 64 distinct
    offsets), offsets symmetric around 0 with the mirrored values equal
    (dia_symcheck over the shard's own rows), band <= 256, an upper-slot
    count the kernel is compiled for (DIA_WALK_H)."""
    if n == 0 or blk.nnz < 12.0 * n:
        return 0
    rows = np.repeat(np.arange(n), np.diff(blk.indptr))
    offs = np.unique(blk.indices.astype(np.int64) - (r0 + rows))
    nm = offs.size
    if nm > 64 or nm % 2 == 0 or offs[nm // 2] != 0 or not np.array_equal(offs, -offs[::-1]):
        return 0
    if offs[-1] > 256 or nm // 2 not in DIA_WALK_H:
        return 0
    import scipy.sparse as sp
    sq = sp.coo_matrix(blk[:, r0:r0 + n])  # entries whose column is one of the shard's rows
    lo = sq.col < sq.row
    up = sq.col > sq.row
    # every stored lower entry (i, j) needs a stored mirror (j, i) with the same bits
    lkey = sq.row[lo].astype(np.int64) * n + sq.col[lo]
    ukey = sq.col[up].astype(np.int64) * n + sq.row[up]  # (j, i) keyed as (i, j)
    order = np.argsort(ukey)
    ukey, uval = ukey[order], sq.data[up][order]
    pos = np.minimum(np.searchsorted(ukey, lkey), max(ukey.size - 1, 0))
    if lkey.size and (ukey.size == 0 or not np.array_equal(ukey[pos], lkey) or
                      not np.array_equal(uval[pos].view(np.uint64),
                                         sq.data[lo].view(np.uint64))):
        return 0
    return nm


def shard_scheds(A, part, cus: int = 256):
    """The launch geometry kr_system_finalize gives the row blocks part[s]..
    part[s+1] of A (kr_engine.cpp default_grid / spmv_grid_for /
    stencil_grid / interior rows; MI355X: 256 CUs x 8 workgroups). The GPU
    tests read the engine's own values (KrylovSystem.shard_sched) and check
    them against this."""
    import scipy.sparse as sp
    A = sp.csr_matrix(A)
    cap = cus * 8
    out = []
    for s in range(len(part) - 1):
        r0, r1 = part[s], part[s + 1]
        n = r1 - r0
        blk = A[r0:r1]
        rows = np.repeat(np.arange(n), np.diff(blk.indptr))
        cols = blk.indices.astype(np.int64)
        reach = int(np.max(np.abs(cols - (r0 + rows)))) if cols.size else 0
        below = rows[cols < r0]
        above = rows[cols > r1 - 1]
        h0 = int(below.max()) + 1 if below.size else 0
        h1 = int(above.min()) if above.size else n
        int_lo = min(-(-h0 // BLOCK) * BLOCK, n)
        int_hi = max(h1 // BLOCK * BLOCK, int_lo)
        nrb = max(1, -(-n // BLOCK))
        base = min(nrb, cap)
        P = _stencil_walk(blk, r0, blk.nnz / max(n, 1))
        walk_nm = 0 if P else _dia_walk(blk, r0, n)
        if walk_nm:
            g = dia_walk_grid(n, walk_nm, cus)
        elif P:
            int_lo = min(-(-int_lo // 512) * 512, n)
            int_hi = max(int_hi // 512 * 512, int_lo)
            g = stencil_grid(n, P)
        else:
            rb = -(-reach // BLOCK)
            if rb * 8 <= base or rb * 8 > cap * 8 or rb * 8 > nrb:
                g = base
            else:
                g = rb * 8
                while g // 2 >= base and g > nrb // 16 and (g // 2) % 8 == 0:
                    g //= 2
        out.append(ShardSched(n=n, grid=base, spmv_grid=g, int_lo=int_lo, int_hi=int_hi,
                              stencil_walk=P, dia_walk=1 if walk_nm else 0))
    return out


def _visits(rows: int, grid: int, gap_at: int = 0, gap: int = 0):
    """Row blocks (launch-local) each workgroup visits, in order (RowSched)."""
    nrb = -(-rows // BLOCK) - gap
    out = []
    for b in range(grid):
        if grid % 8 == 0:
            q, j0, jstep = b & 7, b >> 3, grid >> 3
            chunk = (nrb + 7) // 8
            base = q * chunk
            jcount = max(0, min(nrb, base + chunk) - base)
        else:
            j0, jstep, jcount, base = b, grid, nrb, 0
        vis = []
        for v in range(j0, jcount, jstep):
            r = base + v
            vis.append(r if r < gap_at else r + gap)
        out.append(vis)
    return out


def _visits_dia_walk(rows: int, grid: int, gap_at: int = 0, gap: int = 0):
    """Row blocks each workgroup of the symmetric DIA walk visits, in order
    (kr_spmv.h spmv_diawalk_kernel: workgroup g owns the virtual blocks
    [g nvb / G, (g+1) nvb / G) -- block g when nvb <= G -- physical = v, or
    v + gap past the gap)."""
    nvb = -(-rows // BLOCK) - gap

    def run(g):
        if nvb <= grid:  # workgroup g takes block g
            return range(min(g, nvb), min(g + 1, nvb))
        return range(g * nvb // grid, (g + 1) * nvb // grid)
    return [[v if v < gap_at else v + gap for v in run(g)] for g in range(grid)]


def _wave_tree(v):
    """Lane 0 after ``v += __shfl_down(v, off)`` for off = 32, 16, ..., 1."""
    v = np.asarray(v, dtype=np.float64)
    off = 32
    while off >= 1:
        v = v[:off] + v[off:2 * off]
        off >>= 1
    return v[0]


def _block_total(acc):
    """block_reduce_store / block_slot_sum: 4 wave trees, ((w0+w1)+w2)+w3."""
    w = [_wave_tree(acc[64 * i:64 * (i + 1)]) for i in range(4)]
    t = w[0]
    t = t + w[1]
    t = t + w[2]
    t = t + w[3]
    return np.float64(t)


def _visits_stencil(rows: int, grid: int, P: int, gap_at: int = 0, gap: int = 0):
    """512-row blocks each workgroup of the stencil SpMV visits, in order
    (kr_stencil.h: XCD q = b & 7, position p and plane segment s of b >> 3,
    position-major for P % 8 == 0, else plane-major;
    a launch with a row-block gap -- the boundary launch, RELOAD -- visits
    blocks b, b + grid, b + 2 grid, ...)."""
    nrb = -(-rows // 512) - gap
    if gap > 0:
        return [[v if v < gap_at else v + gap for v in range(b, nrb, grid)]
                for b in range(grid)]
    planes = -(-nrb // P)
    pm = stencil_pm(P)
    out = []
    for b in range(grid):
        q, w = b & 7, b >> 3
        if pm:  # XCD q: positions [q P/8, (q+1) P/8), segment w // (P/8) of grid/P
            PP, Zt = P // 8, grid // P
            p, zs = q * PP + w % PP, w // PP
            z0, z1 = planes * zs // Zt, planes * (zs + 1) // Zt
        else:
            Z = grid // (8 * P)
            p, zs = w % P, w // P
            pl0 = planes * q // 8
            npl = planes * (q + 1) // 8 - pl0
            z0, z1 = pl0 + npl * zs // Z, pl0 + npl * (zs + 1) // Z
        vis = []
        for z in range(z0, z1):
            v = z * P + p
            if v >= nrb:
                break
            vis.append(v if v < gap_at else v + gap)
        out.append(vis)
    return out


def _launch_partials(p, rows, grid, gap_at=0, gap=0, P=0, walk=0):
    """Per-workgroup partials of one SpMV launch over products p[0:rows]."""
    out = np.zeros(grid, np.float64)
    lanes = np.arange(BLOCK)
    if P:
        for b, vis in enumerate(_visits_stencil(rows, grid, P, gap_at, gap)):
            acc = np.zeros(BLOCK, np.float64)
            for rb in vis:
                lo = rb * 512 + 2 * lanes
                act = lo < rows  # rows is even: both rows of a pair or neither
                acc[act] = acc[act] + p[lo[act]]
                acc[act] = acc[act] + p[lo[act] + 1]
            out[b] = _block_total(acc)
        return out
    visits = _visits_dia_walk if walk else _visits
    for b, vis in enumerate(visits(rows, grid, gap_at, gap)):
        acc = np.zeros(BLOCK, np.float64)
        for rb in vis:
            r = rb * BLOCK + lanes
            act = r < rows
            acc[act] = acc[act] + p[r[act]]
        out[b] = _block_total(acc)
    return out


def finalize(partials):
    """block_slot_sum over the slot's partials (fixed order)."""
    acc = np.zeros(BLOCK, np.float64)
    for i0 in range(0, len(partials), BLOCK):
        chunk = np.asarray(partials[i0:i0 + BLOCK], dtype=np.float64)
        acc[:chunk.size] = acc[:chunk.size] + chunk
    return _block_total(acc)


def spmv_shard_total(p, s: ShardSched, split: bool):
    """One shard's total of the epilogue products p (length s.n)."""
    P = s.stencil_walk
    W = s.dia_walk
    if not split:
        return finalize(_launch_partials(p, s.n, s.spmv_grid, P=P, walk=W))
    part = _launch_partials(p[s.int_lo:s.int_hi], s.int_hi - s.int_lo, s.spmv_grid, P=P, walk=W)
    rbs = 512 if P else BLOCK
    nb_lo = s.int_lo // rbs
    nb_gap = (s.int_hi - s.int_lo) // rbs
    nb_all = -(-s.n // rbs)
    if nb_all - nb_gap > 0:
        g = min(s.spmv_grid, nb_all - nb_gap)
        bnd = _launch_partials(p, s.n, g, nb_lo, nb_gap, P=P, walk=W)
        part[:g] = part[:g] + bnd
    return finalize(part)


def ew_shard_total(p, s: ShardSched):
    """One shard's total of elementwise-kernel products (ew_kernel, pairs)."""
    n = s.n
    stride = s.grid * BLOCK
    npairs = n // 2
    acc = np.zeros((s.grid, BLOCK), np.float64).reshape(-1)
    for q0 in range(0, npairs, stride):
        q = np.arange(q0, min(q0 + stride, npairs))
        t = q - q0
        acc[t] = acc[t] + p[2 * q]
        acc[t] = acc[t] + p[2 * q + 1]
    if n & 1:
        acc[0] = acc[0] + p[n - 1]
    acc = acc.reshape(s.grid, BLOCK)
    return finalize([_block_total(acc[b]) for b in range(s.grid)])


class GpuOrder:
    """Dot products summed like the engine over the given shards."""

    def __init__(self, shards):
        self.shards = list(shards)
        self.split = len(self.shards) > 1 and all(s.int_lo < s.int_hi for s in self.shards)
        self.bounds = np.cumsum([0] + [s.n for s in self.shards])

    def _total(self, p, kind):
        tot = np.float64(0.0)
        for i, s in enumerate(self.shards):
            seg = p[self.bounds[i]:self.bounds[i + 1]]
            t = spmv_shard_total(seg, s, self.split) if kind == "spmv" else ew_shard_total(seg, s)
            tot = tot + t
        return np.float64(tot)

    def spmv_dot(self, u, v):
        return self._total(np.asarray(u, np.float64) * np.asarray(v, np.float64), "spmv")

    def ew_dot(self, u, v):
        return self._total(np.asarray(u, np.float64) * np.asarray(v, np.float64), "ew")


SPMV_ONLY_METHODS = ("kskipmrr", "adaptivekskipmrr", "kskipcg")


@contextlib.contextmanager
def patched(order: GpuOrder):
    """Run oracle.v3cpu's k-skip methods with the engine's dot order.

    The first norm a solver takes is ||b|| (oracle _History), which the engine
    computes with EW_DOT; every later dot and norm of the k-skip methods is an
    SpMV epilogue product."""
    from . import v3cpu
    saved = (v3cpu._dot, v3cpu._norm)
    state = {"first": True}

    def norm(v):
        if state["first"]:
            state["first"] = False
            return np.float64(np.sqrt(order.ew_dot(v, v)))
        return np.float64(np.sqrt(order.spmv_dot(v, v)))

    v3cpu._dot = order.spmv_dot
    v3cpu._norm = norm
    try:
        yield
    finally:
        v3cpu._dot, v3cpu._norm = saved


def run(method, A, b, shards, **kw):
    """oracle.v3cpu.<method> with the engine's summation order."""
    from . import v3cpu
    if method not in SPMV_ONLY_METHODS:
        raise ValueError(f"{method}: GPU-order emulation covers {SPMV_ONLY_METHODS}")
    with patched(GpuOrder(shards)), np.errstate(all="ignore"):
        return v3cpu.METHODS[method](A, b, **kw)
