"""The stencil SpMV (kr_stencil.h): 512-row blocks, two rows per lane, the
walk carrying x[row - W] and x[row] in registers, +-1 neighbours from an LDS
line, one row's dictionary codes in 8 slots of 2, 4 or 8 bits (2 / 4 / 8
bytes per row; the narrow widths for <= 3 / <= 15 values, 7-point pattern).

It serves masked short-row shards with a value dictionary whose offsets hold
a +-W pair (W a multiple of 512: 3-D stencils with n^2 % 512 == 0, 2-D ones
with n % 512 == 0), up to 8 offsets, others within +-2 or even (<= 4).
CPU tests pin which matrices qualify (oracle/gpu_order.py restates the
engine's decision); ``-m gpu`` tests check it bit for bit:

* y = A x equals scipy's csr_matvec BITWISE (every row summed in stored
  order) -- cubes, boxes with partial last planes / blocks, 2-D, banded
  stencils with FAR offsets, 1-3 shards (split SpMV with a row-block gap);
* the solver histories equal the oracle run in the engine's summation order
  bit for bit (kr_stencil.h's lane/visit order, oracle/gpu_order.py),
  including adaptive rollbacks, on 1-3 shards;
* fused k-skip steps (EPI_STEP_*, steps 0+1 in one SpMV) equal the unfused
  ones bit for bit on the stencil kernel;
* KR_STENCIL=0 (the row walk) gives the same y bitwise.
"""
import contextlib
import importlib
import io

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_matrix
from oracle import gpu_order


def box(nx, ny, nz=None):
    """7-point (5-point without nz) Poisson on an nx x ny (x nz) grid, x fastest."""
    def T(m):
        return sp.diags([-1.0, 2.0, -1.0], [-1, 0, 1], shape=(m, m))
    K = sp.kronsum(T(nx), T(ny))
    if nz is not None:
        K = sp.kronsum(K, T(nz))
    K = sp.csr_matrix(K)
    K.sort_indices()
    return K


def stencil_band(n, offs, seed=0):
    """Symmetric banded SPD matrix with the given positive offsets (few
    distinct values: a dictionary applies)."""
    rng = np.random.default_rng(seed)
    vals = {o: -float(rng.integers(1, 4)) / 4 for o in offs}
    diags = [np.full(n - o, vals[o]) for o in offs]
    A = sp.diags(diags + diags + [np.full(n, 2.0 * sum(-v for v in vals.values()) + 1.0)],
                 list(offs) + [-o for o in offs] + [0], shape=(n, n))
    A = sp.csr_matrix(A)
    A.sort_indices()
    return A


def aniso(nx, ny, nz, cx, cy, cz):
    """Anisotropic 7-point operator: 4 distinct values (4-bit stencil codes)."""
    def T(m, c):
        return sp.diags([-c, 2.0 * c, -c], [-1, 0, 1], shape=(m, m))
    K = sp.csr_matrix(sp.kronsum(sp.kronsum(T(nx, cx), T(ny, cy)), T(nz, cz)))
    K.sort_indices()
    return K


def revalued(A, nvals, seed=3):
    """A's pattern with values drawn from nvals distinct numbers (SpMV only)."""
    A = A.copy()
    pool = np.random.default_rng(seed).standard_normal(nvals)
    A.data = pool[np.random.default_rng(seed + 1).integers(0, nvals, A.nnz)]
    A.data[:nvals] = pool  # every value present
    return A


def _bal(n, p):
    q, r = divmod(n, p)
    out = [0]
    for i in range(p):
        out.append(out[-1] + q + (1 if i < r else 0))
    return out


MATRICES = {
    "p3d32": lambda: golden_matrix(["poisson", 32, 3]),
    "p3d64": lambda: golden_matrix(["poisson", 64, 3]),
    "box32x32x7": lambda: box(32, 32, 7),        # 7168 rows: 14 blocks, 7 planes of 2
    "box64x16x9": lambda: box(64, 16, 9),        # W = 1024: P = 2
    "box48x32x5": lambda: box(48, 32, 5),        # W = 1536: P = 3, n % 512 == 0
    "box32x32x3": lambda: box(32, 32, 3),        # 3 planes only
    "p2d512x6": lambda: box(512, 6),             # 2-D: W = 512 = the line
    "band_far": lambda: stencil_band(6144, [1, 6, 512]),
    "band_far2": lambda: stencil_band(5120, [2, 14, 1024]),
    "box64x64x20": lambda: box(64, 64, 20),      # W = 4096: P = 8, position-major walk
    "box128x32x9": lambda: box(128, 32, 9),      # W = 4096, 9 planes: short walks
    "aniso32x32x7": lambda: aniso(32, 32, 7, 1.0, 0.5, 0.25),  # 4 values: 4-bit codes
    "vals3_32x32x7": lambda: revalued(box(32, 32, 7), 3),      # 3 values: 2-bit, code 2 used
    "vals15_64x64x9": lambda: revalued(box(64, 64, 9), 15),    # 15 values: 4-bit, P = 8
    "vals40_32x32x7": lambda: revalued(box(32, 32, 7), 40),    # 40 values: 8-bit codes
    # n = 512 (the +-n offsets are whole 512-row blocks): the fused basis pair
    "box512x8x16": lambda: box(512, 8, 16),                    # W = 4096: P = 8
    "box512x16x12": lambda: box(512, 16, 12),                  # P = 16, 12 planes
    "aniso512x8x12": lambda: aniso(512, 8, 12, 1.0, 0.5, 0.25),  # 4-bit codes
    # P % 16 == 0: position pairs (KR_STENCIL_PAIR)
    "box128x64x20": lambda: box(128, 64, 20),                  # W = 8192: P = 16
    "aniso64x128x18": lambda: aniso(64, 128, 18, 1.0, 0.5, 0.25),  # P = 16, 4-bit codes
    "vals40_128x64x10": lambda: revalued(box(128, 64, 10), 40),    # P = 16, 8-bit codes
    "box128x128x16": lambda: box(128, 128, 16),                # P = 32
    # n = 512 and P % 16 == 0: the tiled fused pair (KR_ST2=2)
    "box512x32x10": lambda: box(512, 32, 10),                  # P = 32
    "aniso512x16x12": lambda: aniso(512, 16, 12, 1.0, 0.5, 0.25),  # P = 16, 4-bit codes
    "box512x16x64": lambda: box(512, 16, 64),                  # P = 16, 64 planes: 8 segments
}
# stencil code width (bits per slot) the engine picks for the 7-point pattern
EXPECT_CB = {"aniso32x32x7": 4, "vals3_32x32x7": 2, "vals15_64x64x9": 4, "vals40_32x32x7": 8,
             "p3d32": 2, "p3d64": 2, "box64x64x20": 2, "box512x8x16": 2, "aniso512x8x12": 4,
             "aniso64x128x18": 4, "vals40_128x64x10": 8, "box128x64x20": 2}
# expected stencil walk P (0: the row walk serves the matrix)
EXPECT_P = {"p3d32": 2, "p3d64": 8, "box32x32x7": 2, "box64x16x9": 2, "box48x32x5": 3,
            "box32x32x3": 2, "p2d512x6": 1, "band_far": 1, "band_far2": 2,
            "box64x64x20": 8, "box128x32x9": 8, "aniso32x32x7": 2, "vals3_32x32x7": 2,
            "vals15_64x64x9": 8, "vals40_32x32x7": 2, "box512x8x16": 8, "box512x16x12": 16,
            "aniso512x8x12": 8, "box128x64x20": 16, "aniso64x128x18": 16,
            "vals40_128x64x10": 16, "box128x128x16": 32, "box512x32x10": 32,
            "aniso512x16x12": 16, "box512x16x64": 16}
NOT_STENCIL = {
    "p3d24": lambda: golden_matrix(["poisson", 24, 3]),      # 576 % 512 != 0
    "p3d16": lambda: golden_matrix(["poisson", 16, 3]),
    "odd_rows": lambda: box(32, 32, 7)[:7167, :7167],        # odd n
    "odd_far": lambda: stencil_band(4096, [3, 512]),         # FAR offset 3 is odd
    "nine_offsets": lambda: stencil_band(6000, [1, 6, 40, 512]),
    "band27": lambda: golden_matrix(["banded", 3000, 13, 64, 0]),  # long rows (DIA)
}


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("name", sorted(MATRICES))
def test_stencil_kernel_is_chosen(name):
    A = MATRICES[name]()
    sc = gpu_order.shard_scheds(A, [0, A.shape[0]])[0]
    assert sc.stencil_walk == EXPECT_P[name]
    P = sc.stencil_walk
    # position-major walks (P % 8 == 0) take P x segments, plane-major 8 P x segments
    assert sc.spmv_grid % (P if P % 8 == 0 else 8 * P) == 0 and sc.spmv_grid % 8 == 0


@pytest.mark.parametrize("name", sorted(NOT_STENCIL))
def test_row_walk_keeps_the_rest(name):
    A = NOT_STENCIL[name]()
    assert gpu_order.shard_scheds(A, [0, A.shape[0]])[0].stencil_walk == 0


def test_stencil_sharded_interior_on_512_blocks():
    A = MATRICES["p3d64"]()
    for s in gpu_order.shard_scheds(A, _bal(A.shape[0], 4)):
        assert s.stencil_walk == 8
        assert s.int_lo % 512 == 0 and s.int_hi % 512 == 0 and s.int_lo < s.int_hi
    # 262144 rows over 3 shards: 87382 (even: stencil) + 2 x 87381 (odd: row walk)
    assert [s.stencil_walk for s in gpu_order.shard_scheds(A, _bal(A.shape[0], 3))] == [8, 0, 0]


# ------------------------------------------------------------------ GPU
def _system(A, shards, env=None, monkeypatch=None):
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    n = A.shape[0]
    sysm = KrylovSystem(n, balanced_partition(n, shards), [0] * shards)
    sysm.set_matrix(A)
    sysm.finalize()
    return sysm


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [1, 2, 3])
@pytest.mark.parametrize("name", sorted(MATRICES))
def test_stencil_spmv_bitwise_scipy(monkeypatch, name, shards):
    A = MATRICES[name]()
    n = A.shape[0]
    sysm = _system(A, shards)
    sc = [sysm.shard_sched(s) for s in range(shards)]
    assert [s["stencil_walk"] for s in sc] == \
        [s.stencil_walk for s in gpu_order.shard_scheds(A, _bal(n, shards))]
    assert sc[0]["stencil_walk"] > 0 or shards > 1
    assert [sysm.shard_format(s) for s in range(shards)] == \
        ["stencil" if s_["stencil_walk"] else "csr" for s_ in sc]
    x = np.random.default_rng(5).standard_normal(n)
    y = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
    sysm.close()
    np.testing.assert_array_equal(y, A @ x)
    # the row walk agrees bit for bit
    sysm = _system(A, shards, {"KR_STENCIL": "0"}, monkeypatch)
    assert all(sysm.shard_sched(s)["stencil_walk"] == 0 for s in range(shards))
    y0 = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
    sysm.close()
    np.testing.assert_array_equal(y0, y)


@pytest.mark.gpu
@pytest.mark.parametrize("want", [None, "4", "8"])
@pytest.mark.parametrize("name", sorted(EXPECT_CB))
def test_stencil_code_width_bitwise_scipy(monkeypatch, name, want):
    """Narrow codes (2 / 4 bits per slot; KR_STENCIL_CB asks for at least a
    width) give y = A x bitwise scipy's, on 1 and 2 shards."""
    A = MATRICES[name]()
    n = A.shape[0]
    x = np.random.default_rng(7).standard_normal(n)
    for shards in (1, 2):
        sysm = _system(A, shards, {"KR_STENCIL_CB": want} if want else None, monkeypatch)
        cb = EXPECT_CB[name] if want is None else max(EXPECT_CB[name], int(want))
        assert [sysm.shard_layout(s)["code_bits"] for s in range(shards)] == [cb] * shards
        y = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
        sysm.close()
        np.testing.assert_array_equal(y, A @ x)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["p3d32", "p3d64", "box64x64x20", "box48x32x5", "p2d512x6",
                                  "vals15_64x64x9", "random_codes"])
def test_stencil_code_patterns_bitwise_scipy(monkeypatch, name):
    """Code patterns (System::build_code_patterns): a constant-coefficient
    box stencil has a handful of distinct 512-row code blocks, which the walk
    reads from a table instead of the per-row code stream; random values give
    one pattern per block (a 3-value dictionary over 320 blocks: more than
    the 256-pattern cap, so the row stream stays). y = A x is bitwise scipy's
    either way, on 1 and 3 shards, and equals the row-stream result
    (KR_STENCIL_PATTERNS=0)."""
    A = revalued(box(64, 64, 40), 3) if name == "random_codes" else MATRICES[name]()
    n = A.shape[0]
    x = np.random.default_rng(11).standard_normal(n)
    for shards in (1, 3):
        sysm = _system(A, shards)
        lay = [sysm.shard_layout(s) for s in range(shards)]
        walks = [sysm.shard_sched(s)["stencil_walk"] for s in range(shards)]
        y = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
        sysm.close()
        np.testing.assert_array_equal(y, A @ x)
        for lo, w in zip(lay, walks):
            if not w:
                assert lo["code_patterns"] == 0
            elif name == "random_codes":  # one pattern per block: 320 > 256 on one shard
                if shards == 1:
                    assert lo["code_patterns"] == 0
                else:  # ~107 blocks per shard, all distinct
                    assert lo["code_patterns"] > 100
            elif name.startswith("vals"):
                assert lo["code_patterns"] > 16  # random values: ~one per block
            else:
                assert 1 <= lo["code_patterns"] <= 16
    sysm = _system(A, 1, {"KR_STENCIL_PATTERNS": "0"}, monkeypatch)
    assert sysm.shard_layout(0)["code_patterns"] == 0
    y0 = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
    sysm.close()
    np.testing.assert_array_equal(y0, A @ x)


def _solver(method):
    mod = importlib.import_module(f"parallel_krylov_amd.v3.gpu.{method}")
    return getattr(mod, method)


CASES = [
    ("adaptivekskipmrr", "p3d32", 12, 1), ("adaptivekskipmrr", "p3d32", 12, 3),
    ("adaptivekskipmrr", "box32x32x7", 8, 2), ("kskipmrr", "p3d32", 4, 1),
    ("kskipmrr", "box64x16x9", 3, 2), ("kskipcg", "p3d32", 3, 1), ("kskipcg", "band_far", 2, 3),
    ("kskipmrr", "band_far2", 5, 1), ("adaptivekskipmrr", "p2d512x6", 6, 1),
    ("kskipmrr", "box64x64x20", 4, 1), ("adaptivekskipmrr", "box64x64x20", 6, 2),
    ("kskipcg", "box128x32x9", 3, 3), ("kskipmrr", "aniso32x32x7", 4, 1),
    ("adaptivekskipmrr", "aniso32x32x7", 8, 2), ("kskipmrr", "box128x64x20", 4, 1),
    ("adaptivekskipmrr", "box128x128x16", 6, 2),
    # the fused basis pair (one shard, n = 512): level 1 stays on chip, both
    # duals' products summed in the dual launches' order
    ("kskipmrr", "box512x8x16", 4, 1), ("kskipmrr", "box512x16x12", 5, 1),
    ("adaptivekskipmrr", "box512x16x12", 8, 1), ("kskipmrr", "aniso512x8x12", 2, 1),
    ("kskipmrr", "box512x8x16", 4, 2),
]
# cases also run with the fused basis pair (opt-in KR_ST2=1)
PAIR_ORACLE = {("kskipmrr", "box512x8x16", 4, 1), ("kskipmrr", "box512x16x12", 5, 1),
               ("adaptivekskipmrr", "box512x16x12", 8, 1), ("kskipmrr", "aniso512x8x12", 2, 1)}


@pytest.mark.gpu
@pytest.mark.parametrize("st2", ["0", "1"])
@pytest.mark.parametrize("method,name,k,shards", CASES)
def test_stencil_solvers_bitwise_gpu_order_oracle(monkeypatch, method, name, k, shards, st2):
    if st2 == "1" and (method, name, k, shards) not in PAIR_ORACLE:
        pytest.skip("the fused basis pair serves one-shard n = 512 stencils only")
    monkeypatch.setenv("KR_ST2", st2)
    A = MATRICES[name]()
    n = A.shape[0]
    b = np.random.default_rng(1).standard_normal(n)
    sysm = _system(A, shards)
    sc = [gpu_order.ShardSched(**sysm.shard_sched(s)) for s in range(shards)]
    sysm.close()
    assert sc == gpu_order.shard_scheds(A, _bal(n, shards))
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", ",".join(["0"] * shards))
    kw = dict(tol=1e-10, k=k, maxiter=600)
    with contextlib.redirect_stdout(io.StringIO()):
        x, info = _solver(method)(A, b, **kw)
    x_ref, ref = gpu_order.run(method, A, b, sc, **kw)
    np.testing.assert_array_equal(info["nosl"], ref["nosl"])
    if "khistory" in ref:
        np.testing.assert_array_equal(info["khistory"], ref["khistory"])
    np.testing.assert_array_equal(info["residual"], ref["residual"])
    np.testing.assert_array_equal(x.cpu().numpy(), x_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("shards", ["0", "0,0,0"])
@pytest.mark.parametrize("method,name,k", [("kskipmrr", "p3d32", 1), ("kskipmrr", "p3d32", 4),
                                           ("kskipmrr", "box32x32x7", 3),
                                           ("kskipcg", "p3d64", 3),
                                           ("adaptivekskipmrr", "p3d32", 6),
                                           ("kskipmrr", "band_far", 2)])
def test_stencil_fused_steps_bitwise_equal_unfused(monkeypatch, shards, method, name, k):
    A = MATRICES[name]()
    b = np.random.default_rng(3).standard_normal(A.shape[0])
    kw = dict(tol=1e-10, maxiter=300, k=k)
    out = []
    for env in ({"KR_FUSE": "0"}, {"KR_FUSE": "1", "KR_FUSE_FIRST": "1"},
                {"KR_FUSE": "1", "KR_FUSE_FIRST": "0"}):
        monkeypatch.setenv("KRYLOV_AMD_SHARDS", shards)
        for kk, vv in env.items():
            monkeypatch.setenv(kk, vv)
        with contextlib.redirect_stdout(io.StringIO()):
            x, info = _solver(method)(A, b, **kw)
        out.append((x.cpu().numpy(), info))
    for x1, i1 in out[1:]:
        np.testing.assert_array_equal(i1["nosl"], out[0][1]["nosl"])
        np.testing.assert_array_equal(i1["residual"], out[0][1]["residual"])
        np.testing.assert_array_equal(x1, out[0][0])


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["cg", "mrr"])
def test_stencil_cg_mrr_match_reference_contract(method):
    """CG / MrR (head-less epilogues EPI_XY, EPI_MRR_LOOP, EPI_BMINUS on the
    stencil kernel) against the oracle: SURVEY.md 8(c) contract."""
    from oracle import v3cpu
    A = MATRICES["p3d32"]()
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    with contextlib.redirect_stdout(io.StringIO()):
        x, info = _solver(method)(A, b, tol=1e-10)
    x_ref, ref = v3cpu.METHODS[method](A, b, tol=1e-10)
    np.testing.assert_array_equal(info["nosl"], ref["nosl"])
    rel = np.abs(info["residual"] - ref["residual"]) / ref["residual"]
    assert rel.max() <= 1e-12
    assert np.linalg.norm(x.cpu().numpy() - x_ref) <= 1e-11 * np.linalg.norm(x_ref)


PAIR_CASES = [("kskipmrr", "box512x8x16", 2), ("kskipmrr", "box512x8x16", 3),
              ("kskipmrr", "box512x16x12", 4), ("kskipmrr", "aniso512x8x12", 5),
              ("adaptivekskipmrr", "box512x16x12", 6), ("adaptivekskipmrr", "aniso512x8x12", 8)]


@pytest.mark.gpu
@pytest.mark.parametrize("method,name,k", PAIR_CASES)
def test_stencil_pair_bitwise_equal_duals(monkeypatch, method, name, k):
    """The fused basis pair (spmv_stencil2_kernel: two chained duals in one
    walk, level 1 kept on chip) against the dual SpMVs (KR_ST2=0): the same
    rows summed the same way and the same products in the same order, so the
    histories and x are equal bit for bit -- odd k ends with a single dual,
    adaptive k shrinks through rollbacks."""
    A = MATRICES[name]()
    b = np.random.default_rng(5).standard_normal(A.shape[0])
    kw = dict(tol=1e-10, maxiter=400, k=k)
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", "0")
    out = []
    for st2 in ("0", "1"):
        monkeypatch.setenv("KR_ST2", st2)
        with contextlib.redirect_stdout(io.StringIO()):
            x, info = _solver(method)(A, b, **kw)
        out.append((x.cpu().numpy(), info))
    (x0, i0), (x1, i1) = out
    np.testing.assert_array_equal(i1["nosl"], i0["nosl"])
    if "khistory" in i0:
        np.testing.assert_array_equal(i1["khistory"], i0["khistory"])
    np.testing.assert_array_equal(i1["residual"], i0["residual"])
    np.testing.assert_array_equal(x1, x0)


# the tiled pair (KR_ST2=2, two positions per workgroup, P % 16 == 0); env:
# KR_PO_ZMAX=1 gives the products-only dual a 1-segment grid against the
# general grid's 8 (the pair then flushes level 1 every 8 planes inside one
# 64-plane walk), KR_ST2T_Z=1 makes every pair walk 64 planes (both levels flush)
TILED_CASES = [("kskipmrr", "box512x16x12", 4, {}), ("kskipmrr", "box512x16x12", 5, {}),
               ("adaptivekskipmrr", "box512x16x12", 8, {}), ("kskipmrr", "aniso512x16x12", 4, {}),
               ("kskipmrr", "box512x32x10", 3, {}), ("kskipcg", "box512x16x12", 4, {}),
               ("kskipcg", "box512x32x10", 5, {}),
               ("kskipmrr", "box512x16x64", 4, {"KR_PO_ZMAX": "1"}),
               ("kskipmrr", "box512x16x64", 4, {"KR_PO_ZMAX": "1", "KR_ST2T_Z": "1"}),
               ("kskipcg", "box512x16x64", 4, {"KR_PO_ZMAX": "2", "KR_ST2T_Z": "1"})]


@pytest.mark.gpu
@pytest.mark.parametrize("method,name,k,env", TILED_CASES,
                         ids=[f"{m}-{n}-k{k}-{len(e)}" for m, n, k, e in TILED_CASES])
def test_stencil_tiled_pair_bitwise_equal_duals(monkeypatch, method, name, k, env):
    """The tiled fused basis pair (spmv_stencil2t_kernel: two positions per
    workgroup, level 1 on chip) against the dual SpMVs (KR_ST2=0): histories
    and x bit for bit -- every row summed in stored order and every product
    accumulated in the dual launches' order into their partials, through
    segment boundaries of either dual grid inside one walk, for k-skip MrR,
    adaptive k-skip MrR and k-skip CG, odd and even k, 2- and 4-bit codes."""
    A = MATRICES[name]()
    b = np.random.default_rng(5).standard_normal(A.shape[0])
    kw = dict(tol=1e-10, maxiter=400, k=k)
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", "0")
    for key, val in env.items():
        monkeypatch.setenv(key, val)
    out = []
    for st2 in ("0", "2"):
        monkeypatch.setenv("KR_ST2", st2)
        with contextlib.redirect_stdout(io.StringIO()):
            x, info = _solver(method)(A, b, **kw)
        out.append((x.cpu().numpy(), info))
    (x0, i0), (x1, i1) = out
    np.testing.assert_array_equal(i1["nosl"], i0["nosl"])
    if "khistory" in i0:
        np.testing.assert_array_equal(i1["khistory"], i0["khistory"])
    np.testing.assert_array_equal(i1["residual"], i0["residual"])
    np.testing.assert_array_equal(x1, x0)


@pytest.mark.gpu
@pytest.mark.parametrize("method,k", [("kskipmrr", 4), ("kskipmrr", 3), ("kskipcg", 4)])
def test_stencil_tiled_pair_is_used(monkeypatch, method, k):
    """KR_ST2=2 runs k // 2 tiled pair launches per outer iteration (the last
    products-only for even k) and k % 2 single duals on a qualifying shard."""
    monkeypatch.setenv("KR_ST2", "2")
    A = MATRICES["box512x16x12"]()
    sysm = _system(A, 1)
    tag = "mrr" if method == "kskipmrr" else "kcg"
    try:
        b = sysm.split(np.random.default_rng(1).standard_normal(A.shape[0]))
        sysm.begin(method, b, None, tol=0.0, maxiter=8 * (k + 1) + 2, k=k, profile=1)
        sysm.step(4)
        st = {r["name"]: r["launches"] for r in sysm.kernel_stats()}
        sysm.finish(method)
    finally:
        sysm.close()
    npair = st.get(f"spmv2x2_gram_{tag}", 0) + st.get(f"spmv2x2_gram_{tag}_last", 0)
    ndual = st.get(f"spmv2_gram_{tag}", 0) + st.get(f"spmv2_gram_{tag}_last", 0)
    assert npair == 4 * (k // 2) and ndual == 4 * (k % 2), st
    assert st.get(f"spmv2x2_gram_{tag}_last", 0) == (4 if k % 2 == 0 else 0), st


@pytest.mark.gpu
@pytest.mark.parametrize("name,k,pairs,st2", [("box512x8x16", 4, True, "1"),
                                              ("box512x8x16", 3, True, "1"),
                                              ("box512x8x16", 4, False, "0"),
                                              ("p3d64", 4, False, "1")])
def test_stencil_pair_is_used(monkeypatch, name, k, pairs, st2):
    """With KR_ST2=1 the k-skip MrR basis runs as fused pairs exactly where the
    shard qualifies (n = 512, one shard): k // 2 pair launches per outer
    iteration, the last one products-only for even k, and k % 2 single duals;
    by default (no KR_ST2) the dual launches."""
    monkeypatch.setenv("KR_ST2", st2)
    A = MATRICES[name]()
    sysm = _system(A, 1)
    try:
        b = sysm.split(np.random.default_rng(1).standard_normal(A.shape[0]))
        sysm.begin("kskipmrr", b, None, tol=0.0, maxiter=8 * (k + 1) + 2, k=k, profile=1)
        sysm.step(4)
        st = {r["name"]: r["launches"] for r in sysm.kernel_stats()}
        sysm.finish("kskipmrr")
    finally:
        sysm.close()
    npair = st.get("spmv2x2_gram_mrr", 0) + st.get("spmv2x2_gram_mrr_last", 0)
    ndual = st.get("spmv2_gram_mrr", 0) + st.get("spmv2_gram_mrr_last", 0)
    if pairs:
        assert npair == 4 * (k // 2) and ndual == 4 * (k % 2), st
        assert st.get("spmv2x2_gram_mrr_last", 0) == (4 if k % 2 == 0 else 0), st
    else:
        assert npair == 0 and ndual == 4 * k, st


@pytest.mark.gpu
@pytest.mark.parametrize("method,name,k,shards", [("kskipmrr", "p3d32", 4, "0"),
                                                  ("kskipmrr", "box64x64x20", 4, "0,0"),
                                                  ("adaptivekskipmrr", "box512x8x16", 6, "0"),
                                                  ("kskipcg", "box128x32x9", 3, "0"),
                                                  ("kskipmrr", "aniso32x32x7", 4, "0,0,0")])
def test_stencil_dpp_neighbours_bitwise(monkeypatch, method, name, k, shards):
    """The +-1 neighbours moved by DPP wave shifts (+ the waves' edge rows
    through the scalar cache; KR_STENCIL_DPP=2: every 7-point launch, 1: the
    products-only dual, 0: the LDS line) give the same histories and x bit
    for bit -- cubes, boxes, sharded (boundary launches), VIRT epilogues."""
    A = MATRICES[name]()
    b = np.random.default_rng(7).standard_normal(A.shape[0])
    kw = dict(tol=1e-10, maxiter=300, k=k)
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", shards)
    out = []
    for dpp in ("0", "1", "2"):
        monkeypatch.setenv("KR_STENCIL_DPP", dpp)
        with contextlib.redirect_stdout(io.StringIO()):
            x, info = _solver(method)(A, b, **kw)
        out.append((x.cpu().numpy(), info))
    for x1, i1 in out[1:]:
        np.testing.assert_array_equal(i1["nosl"], out[0][1]["nosl"])
        np.testing.assert_array_equal(i1["residual"], out[0][1]["residual"])
        np.testing.assert_array_equal(x1, out[0][0])


@pytest.mark.gpu
@pytest.mark.parametrize("method,name,k,shards", [
    ("kskipmrr", "box128x64x20", 4, "0"),
    ("kskipmrr", "box512x16x12", 4, "0"),
    ("kskipmrr", "box128x64x20", 4, "0,0"),
    ("adaptivekskipmrr", "aniso64x128x18", 6, "0"),
    ("kskipcg", "vals40_128x64x10", 3, "0"),
    ("kskipmrr", "box128x128x16", 5, "0,0,0,0"),
    ("cg", "box128x128x16", 0, "0"),
    ("mrr", "box128x64x20", 0, "0,0"),
    ("kskipmrr", "box64x64x20", 4, "0"),     # P = 8: never paired
    # n = 512 (FAR offsets -+512 = the positions p -+ 1): bit 32 takes the
    # inner +-n line of each half from the other half's LDS line
    ("kskipmrr", "box512x32x10", 4, "0"),
    ("adaptivekskipmrr", "aniso512x16x12", 6, "0"),
    ("kskipcg", "box512x16x64", 3, "0,0"),
    ("cg", "box512x32x10", 0, "0"),
])
def test_stencil_position_pairs_bitwise(monkeypatch, method, name, k, shards):
    """Two adjacent positions per workgroup (KR_STENCIL_PAIR bit mask: 1
    products-only duals, 2 storing duals, 4/8 the fused steps, 16 the rest;
    32: the inner +-n line from the other half's LDS line where n = 512) run
    the same virtual workgroups as the unpaired walk, and so does the reversed
    dispatch order of every other launch (KR_ZIGZAG): the same histories and
    x bit for bit, sharded (boundary launches stay unpaired) or not."""
    A = MATRICES[name]()
    b = np.random.default_rng(11).standard_normal(A.shape[0])
    kw = dict(tol=1e-10, maxiter=200)
    if k:
        kw["k"] = k
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", shards)
    out = []
    for mask, zz in (("0", "0"), ("0", "1"), ("3", "1"), ("31", "0"), ("63", "0")):
        monkeypatch.setenv("KR_STENCIL_PAIR", mask)
        monkeypatch.setenv("KR_ZIGZAG", zz)
        with contextlib.redirect_stdout(io.StringIO()):
            x, info = _solver(method)(A, b, **kw)
        out.append((x.cpu().numpy(), info))
    for x1, i1 in out[1:]:
        np.testing.assert_array_equal(i1["nosl"], out[0][1]["nosl"])
        np.testing.assert_array_equal(i1["residual"], out[0][1]["residual"])
        np.testing.assert_array_equal(x1, out[0][0])


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["csr", "rowwalk", "dia_walk", "stencil"])
@pytest.mark.parametrize("method,k", [("kskipmrr", 4), ("kskipmrr", 3), ("kskipcg", 3),
                                      ("adaptivekskipmrr", 4)])
@pytest.mark.parametrize("shards", [1, 2])
def test_products_only_every_format_bitwise(monkeypatch, fmt, method, k, shards):
    """Round 5: the last basis dual of every outer iteration (its outputs
    feed only the Gram products) skips its y1/y2 stores in EVERY SpMV format
    -- plain CSR row walk, the masked/dictionary row walk, the symmetric DIA
    walk and the stencil walk -- and runs under its own stat name. Same
    products, so the history, k structure and x equal the storing run
    (KR_PRODUCTS_ONLY=0) bit for bit."""
    env = {"csr": {"KR_MASK": "0", "KR_VDICT": "0", "KR_STENCIL": "0"},
           "rowwalk": {"KR_STENCIL": "0"}, "dia_walk": {}, "stencil": {}}[fmt]
    A = (golden_matrix(["banded", 3000, 31, 256, 0]) if fmt == "dia_walk"
         else MATRICES["p3d32"]())
    b = np.random.default_rng(4).standard_normal(A.shape[0])
    tag = "kcg" if method == "kskipcg" else "mrr"
    runs = []
    for po in ("1", "0"):
        monkeypatch.setenv("KR_PRODUCTS_ONLY", po)
        sysm = _system(A, shards, env, monkeypatch)
        try:
            want = {"csr": "csr", "rowwalk": "csr", "dia_walk": "dia_walk", "stencil": "stencil"}
            assert [sysm.shard_format(s) for s in range(shards)] == [want[fmt]] * shards
            if fmt == "csr":  # plain CSR: no masks, no dictionary
                assert all(sysm.shard_layout(s)["mask_bits"] == 0 and
                           sysm.shard_layout(s)["dict_values"] == 0 for s in range(shards))
            sysm.begin(method, sysm.split(b), None, tol=1e-10, maxiter=60, k=k, profile=1)
            while not sysm.step(4):
                pass
            st = {r["name"]: r["launches"] for r in sysm.kernel_stats()}
            out = sysm.finish(method)
            x = np.concatenate([t.cpu().numpy() for t in out.x])
        finally:
            sysm.close()
        runs.append((st, out.info, x))
    (st1, i1, x1), (st0, i0, x0) = runs
    assert st1.get(f"spmv2_gram_{tag}_last", 0) > 0, st1
    assert st0.get(f"spmv2_gram_{tag}_last", 0) == 0, st0
    np.testing.assert_array_equal(i1["nosl"], i0["nosl"])
    if "khistory" in i0:
        np.testing.assert_array_equal(i1["khistory"], i0["khistory"])
    np.testing.assert_array_equal(i1["residual"], i0["residual"])
    np.testing.assert_array_equal(x1, x0)
