"""The box fused basis pair (kr_pair.hip, spmv_stencil2b_kernel; KR_ST2=3).

A constant-coefficient 7-point stencil on an n = 512 box (every entry of an
offset the same value, absent entries exactly the box faces) is recognised
at finalize (System::build_box, ``shard_layout()["box"]``); its k-skip basis
pairs then run without reading the matrix: the absent operands are read as
0.0 (zero LDS pads, out-of-range loads, zeroed level-1 planes), which leaves
every row sum bit for bit scipy's, and both duals' products are accumulated
in the dual launches' order into their partials. So the histories and x
must equal the two-dual path (KR_ST2=0) BITWISE -- which the GPU-order
oracle already pins to the reference's statements (test_gpu_stencil.py).
"""
import contextlib
import importlib
import io

import numpy as np
import pytest
import scipy.sparse as sp

from test_gpu_stencil import MATRICES, _system, aniso, box


def _solver(method):
    mod = importlib.import_module(f"parallel_krylov_amd.v3.gpu.{method}")
    return getattr(mod, method)


def perturbed_value(A, row=5 * 512 * 16 + 3 * 512 + 100):
    """One interior off-diagonal entry changed: no longer constant-coefficient."""
    A = A.tolil(copy=True)
    A[row, row + 1] = A[row, row + 1] * 1.5
    A = sp.csr_matrix(A)
    A.sort_indices()
    return A


def dropped_entry(A, row=5 * 512 * 16 + 3 * 512 + 100):
    """One interior +1 entry removed (stored structure off the box faces)."""
    A = A.tolil(copy=True)
    A[row, row + 1] = 0.0
    A = sp.csr_matrix(A)
    A.eliminate_zeros()
    A.sort_indices()
    return A


BOX = {
    "box512x16x12": 1, "box512x32x10": 1, "aniso512x16x12": 1, "box512x16x64": 1,
    "box512x8x16": 1, "p3d64": 0, "box128x64x20": 0, "vals40_128x64x10": 0,
}


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(BOX))
def test_box_flag(name):
    sysm = _system(MATRICES[name](), 1)
    try:
        assert sysm.shard_layout(0)["box"] == BOX[name]
    finally:
        sysm.close()


@pytest.mark.gpu
@pytest.mark.parametrize("make", [perturbed_value, dropped_entry])
def test_box_flag_rejects_irregular(make):
    sysm = _system(make(box(512, 16, 12)), 1)
    try:
        assert sysm.shard_layout(0)["box"] == 0
    finally:
        sysm.close()


@pytest.mark.gpu
def test_box_flag_anisotropic_and_negative_values():
    """Per-offset constants (not one global value), a negative diagonal."""
    A = -aniso(512, 16, 10, 2.0, 0.75, 0.3)
    sysm = _system(sp.csr_matrix(A), 1)
    try:
        assert sysm.shard_layout(0)["box"] == 1
    finally:
        sysm.close()


# KR_PO_ZMAX=1 gives the products-only dual a 1-segment grid against the
# general grid's (the pair then flushes level 1 inside one walk), KR_ST2B_Z=1
# makes every pair walk the whole box (both levels flush); KR_ST2B_Z=2 two
# walk segments
BOX_CASES = [("kskipmrr", "box512x16x12", 4, {}), ("kskipmrr", "box512x16x12", 5, {}),
             ("adaptivekskipmrr", "box512x16x12", 8, {}), ("kskipmrr", "aniso512x16x12", 4, {}),
             ("kskipmrr", "box512x32x10", 3, {}), ("kskipmrr", "box512x32x10", 2, {}),
             ("kskipcg", "box512x16x12", 4, {}), ("kskipcg", "box512x32x10", 5, {}),
             ("kskipmrr", "box512x16x64", 4, {"KR_PO_ZMAX": "1"}),
             ("kskipmrr", "box512x16x64", 4, {"KR_PO_ZMAX": "1", "KR_ST2B_Z": "1"}),
             ("kskipmrr", "box512x16x64", 6, {"KR_ST2B_Z": "2"}),
             ("kskipcg", "box512x16x64", 4, {"KR_PO_ZMAX": "2", "KR_ST2B_Z": "1"}),
             ("adaptivekskipmrr", "box512x16x64", 6, {}),
             # x segments per line (KR_ST2B_XS, default 1): quarters, halves
             ("kskipmrr", "box512x16x12", 4, {"KR_ST2B_XS": "4", "KR_ST2B_XS_PO": "4"}),
             ("kskipmrr", "box512x32x10", 5, {"KR_ST2B_XS": "2"}),
             ("kskipcg", "box512x16x12", 4, {"KR_ST2B_XS": "2", "KR_ST2B_XS_PO": "2"}),
             ("adaptivekskipmrr", "aniso512x16x12", 6, {"KR_ST2B_XS": "4"}),
             ("kskipmrr", "box512x16x64", 4, {"KR_PO_ZMAX": "1", "KR_ST2B_Z": "1",
                                              "KR_ST2B_XS": "2"})]


@pytest.mark.gpu
@pytest.mark.parametrize("method,name,k,env", BOX_CASES,
                         ids=[f"{m}-{n}-k{k}-{len(e)}" for m, n, k, e in BOX_CASES])
def test_box_pair_bitwise_equal_duals(monkeypatch, method, name, k, env):
    """Histories and x bit for bit against the dual launches (KR_ST2=0):
    k-skip MrR, adaptive k-skip MrR, k-skip CG; odd k ends with a single dual;
    flushes at either grid's segment boundaries inside one walk."""
    A = MATRICES[name]()
    b = np.random.default_rng(5).standard_normal(A.shape[0])
    kw = dict(tol=1e-10, maxiter=400, k=k)
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", "0")
    for key, val in env.items():
        monkeypatch.setenv(key, val)
    out = []
    for st2 in ("0", "3"):
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


def _launches(A, method, k, st2, monkeypatch):
    monkeypatch.setenv("KR_ST2", st2)
    sysm = _system(A, 1)
    try:
        b = sysm.split(np.random.default_rng(1).standard_normal(A.shape[0]))
        sysm.begin(method, b, None, tol=0.0, maxiter=8 * (k + 1) + 2, k=k, profile=1)
        sysm.step(4)
        st = {r["name"]: r["launches"] for r in sysm.kernel_stats()}
        sysm.finish(method)
    finally:
        sysm.close()
    return st


@pytest.mark.gpu
@pytest.mark.parametrize("method,k", [("kskipmrr", 4), ("kskipmrr", 3), ("kskipcg", 4)])
def test_box_pair_is_used(monkeypatch, method, k):
    """KR_ST2=3 runs k // 2 box-pair launches per outer iteration (the last
    products-only for even k) and k % 2 single duals on a box shard."""
    st = _launches(MATRICES["box512x16x12"](), method, k, "3", monkeypatch)
    tag = "mrr" if method == "kskipmrr" else "kcg"
    npair = st.get(f"spmv2x2_gram_{tag}", 0) + st.get(f"spmv2x2_gram_{tag}_last", 0)
    ndual = st.get(f"spmv2_gram_{tag}", 0) + st.get(f"spmv2_gram_{tag}_last", 0)
    assert npair == 4 * (k // 2) and ndual == 4 * (k % 2), st
    assert st.get(f"spmv2x2_gram_{tag}_last", 0) == (4 if k % 2 == 0 else 0), st


@pytest.mark.gpu
def test_box_pair_not_used_off_the_box(monkeypatch):
    """An irregular matrix (one interior entry dropped) keeps the dual launches
    under KR_ST2=3, and its history still equals the KR_ST2=0 run."""
    A = dropped_entry(box(512, 16, 12))
    st = _launches(A, "kskipmrr", 4, "3", monkeypatch)
    assert st.get("spmv2x2_gram_mrr", 0) == 0 and st.get("spmv2_gram_mrr", 0) > 0, st


# the box step walks (KR_STEP2, default on for box shards): steps 0-2 in one
# walk (the step triple, KR_STEP3) and pairs of the later steps in one walk
# each (x2 / nox / x kinds), against the step launches
STEP2_CASES = [("kskipmrr", "box512x16x12", 4, {}), ("kskipmrr", "box512x16x12", 5, {}),
               ("kskipmrr", "box512x32x10", 3, {}), ("kskipmrr", "box512x32x10", 6, {}),
               ("kskipmrr", "box512x16x12", 2, {}), ("kskipmrr", "box512x16x12", 7, {}),
               ("kskipmrr", "aniso512x16x12", 4, {}), ("adaptivekskipmrr", "box512x16x12", 8, {}),
               ("adaptivekskipmrr", "box512x16x64", 6, {}),
               ("adaptivekskipmrr", "aniso512x16x12", 3, {}),
               ("kskipmrr", "box512x16x64", 4, {"KR_STEP2_Z": "1"}),
               ("kskipmrr", "box512x16x64", 4, {"KR_STEP2_Z": "3"}),
               ("kskipmrr", "box512x16x12", 4, {"KR_STEP3": "0"}),
               ("kskipmrr", "box512x16x12", 5, {"KR_STEP3": "0"}),
               ("kskipmrr", "box512x16x12", 4, {"KR_FUSE_FIRST": "0"}),
               ("kskipmrr", "box512x16x12", 5, {"KR_FUSE_FIRST": "0"}),
               ("adaptivekskipmrr", "box512x16x12", 6, {"KR_FUSE_FIRST": "0"}),
               ("kskipmrr", "box512x16x12", 4, {"KR_ST2": "0"}),
               ("kskipmrr", "box512x16x12", 4, {"KR_STEP2H": "0"}),
               ("kskipmrr", "box512x16x64", 6, {"KR_STENCIL_Z": "16"}),
               ("adaptivekskipmrr", "box512x16x64", 4, {"KR_STENCIL_Z": "8"})]


@pytest.mark.gpu
@pytest.mark.parametrize("method,name,k,env", STEP2_CASES,
                         ids=[f"{m}-{n}-k{k}-{'-'.join(e)}" for m, n, k, e in STEP2_CASES])
def test_box_step_pair_bitwise_equal_steps(monkeypatch, method, name, k, env):
    """Histories and x bit for bit against the step launches (KR_STEP2=0):
    even and odd k (every pair of step kinds, the deferred x), adaptive
    rollbacks, walks of 1 / 3 segments, pairs without the triple, without
    the fused first steps, with the dual launches instead of the box pair."""
    A = MATRICES[name]()
    b = np.random.default_rng(7).standard_normal(A.shape[0])
    kw = dict(tol=1e-10, maxiter=400, k=k)
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", "0")
    for key, val in env.items():
        monkeypatch.setenv(key, val)
    out = []
    for on in ("0", "1"):
        monkeypatch.setenv("KR_STEP2", on)
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
@pytest.mark.parametrize("k,triples,pairs,fused", [(4, 1, 0, 1), (5, 1, 1, 0), (2, 1, 0, 0),
                                                   (3, 1, 0, 0), (6, 1, 1, 1), (1, 0, 0, 0)])
def test_box_step_pair_is_used(monkeypatch, k, triples, pairs, fused):
    """k-skip MrR on a box shard: per outer iteration one step-triple launch
    (steps 0-2), one step-pair launch per later pair of steps, and the last
    pair of steps (steps k-1, k) with the next head SpMV in one walk
    (spmv_step2h) -- then no separate head launch."""
    monkeypatch.delenv("KR_STEP2", raising=False)
    st = _launches(MATRICES["box512x16x12"](), "kskipmrr", k, "3", monkeypatch)
    assert st.get("spmv_step3_mrr_stencil", 0) == 4 * triples, st
    assert st.get("spmv_step2_mrr_stencil", 0) == 4 * pairs, st
    assert st.get("spmv_step2h_mrr_stencil", 0) == 4 * fused, st
    # (plus the solve's first head, before the first outer iteration)
    assert st.get("spmv_head_mrr", 0) == 1 + 4 * (1 - fused), st


# the step pair + head against the step pair and the head launch, bitwise,
# over head grids whose segments flush inside one walk (KR_STENCIL_Z), walk
# segment counts (KR_STEP2_Z), the x kinds (xdefer, adaptive)
STEP2H_CASES = [("kskipmrr", "box512x16x12", 4, {}), ("kskipmrr", "box512x32x10", 6, {}),
                ("kskipmrr", "box512x16x64", 4, {"KR_STENCIL_Z": "16"}),
                ("kskipmrr", "box512x16x64", 4, {"KR_STENCIL_Z": "8", "KR_STEP2_Z": "2"}),
                ("kskipmrr", "box512x16x64", 4, {"KR_STEP2_Z": "1"}),
                ("kskipmrr", "aniso512x16x12", 4, {}),
                ("adaptivekskipmrr", "box512x16x12", 4, {}),
                ("adaptivekskipmrr", "box512x16x64", 6, {"KR_STENCIL_Z": "4"})]


@pytest.mark.gpu
@pytest.mark.parametrize("method,name,k,env", STEP2H_CASES,
                         ids=[f"{m}-{n}-k{k}-{'-'.join(e)}" for m, n, k, e in STEP2H_CASES])
def test_box_step_pair_head_bitwise_equal(monkeypatch, method, name, k, env):
    """Histories and x bit for bit against KR_STEP2H=0 (the step pair, then
    the head launch)."""
    A = MATRICES[name]()
    b = np.random.default_rng(11).standard_normal(A.shape[0])
    kw = dict(tol=1e-10, maxiter=400, k=k)
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", "0")
    for key, val in env.items():
        monkeypatch.setenv(key, val)
    out = []
    for on in ("0", "1"):
        monkeypatch.setenv("KR_STEP2H", on)
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
@pytest.mark.parametrize("method,name,k", [("kskipmrr", "box512x16x12", 4),
                                           ("adaptivekskipmrr", "box512x32x10", 4),
                                           ("kskipmrr", "aniso512x16x12", 6)])
def test_box_walks_low_residual_vs_oracle(method, name, k):
    """The box walks (pairs, step triple, step pair + head) against the oracle
    itself (oracle.v3cpu, bitwise the reference's v3/cpu) down to tol =
    1e-12, the low-residual regime of SURVEY.md 8(c) at the headline's
    n = 512 line geometry: nosl (and khistory) identical, entries >= 1e-8
    within 1e-12 relative, entries below within max(1e-12, 10x the oracle's
    reordering envelope: its dots summed in 256-element blocks), x within
    max(1e-11, 10x its envelope)."""
    from oracle import v3cpu
    from test_gpu_fullsize import _oracle_blocked_dots
    A = MATRICES[name]()
    b = np.random.default_rng(13).standard_normal(A.shape[0])
    kw = dict(tol=1e-12, k=k)
    with contextlib.redirect_stdout(io.StringIO()):
        x, info = _solver(method)(A, b, **kw)
    x = x.cpu().numpy()
    fn = getattr(v3cpu, method)
    x_ref, ref = fn(A, b, **kw)
    x_p, ref_p = _oracle_blocked_dots(fn, A, b, **kw)
    assert len(ref_p["residual"]) == len(ref["residual"])
    env = np.abs(ref_p["residual"] - ref["residual"]) / np.abs(ref["residual"])
    x_env = np.linalg.norm(x_p - x_ref) / np.linalg.norm(x_ref)
    res = np.asarray(info["residual"])
    assert ref["residual"][-1] < 1e-12 and np.sum(ref["residual"] < 1e-8) >= 2
    np.testing.assert_array_equal(info["nosl"], ref["nosl"])
    if "khistory" in ref:
        np.testing.assert_array_equal(info["khistory"], ref["khistory"])
    rel = np.abs(res - ref["residual"]) / np.abs(ref["residual"])
    contract = np.abs(ref["residual"]) >= 1e-8
    assert np.all(rel[contract] <= 1e-12), rel[contract].max()
    assert np.all(rel[~contract] <= np.maximum(1e-12, 10.0 * env[~contract])), (rel, env)
    xrel = np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref)
    assert xrel <= max(1e-11, 10.0 * x_env), (xrel, x_env)


# thin and short boxes: 1-3 planes (walk and grid segment counts clamp to
# the plane count), P = 16 / 32, every box-walk kind against the dual path
THIN = [("kskipmrr", 512, 16, 1, 4), ("kskipmrr", 512, 16, 2, 4), ("kskipmrr", 512, 16, 3, 5),
        ("kskipmrr", 512, 32, 2, 6), ("adaptivekskipmrr", 512, 16, 3, 4),
        ("kskipcg", 512, 16, 2, 4), ("kskipmrr", 512, 16, 5, 2)]


@pytest.mark.gpu
@pytest.mark.parametrize("method,nx,ny,nz,k", THIN,
                         ids=[f"{m}-{nx}x{ny}x{nz}-k{k}" for m, nx, ny, nz, k in THIN])
def test_box_walks_thin_boxes_bitwise_dual_path(monkeypatch, method, nx, ny, nz, k):
    """Histories and x bit for bit against KR_BOX=0 (no box walks)."""
    A = box(nx, ny, nz)
    b = np.random.default_rng(17).standard_normal(A.shape[0])
    kw = dict(tol=1e-10, maxiter=300, k=k)
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", "0")
    out = []
    for on in ("0", "1"):
        monkeypatch.setenv("KR_BOX", on)
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
def test_box_walks_need_position_major_grids(monkeypatch):
    """KR_STENCIL_PM=0 (plane-major stencil grids): the box walks that write
    Gram partials (the pairs, the step pair + head) write them in the
    position-major grids' workgroup order, so they step aside; the step
    walks (no partials) stay. The history equals KR_BOX=0's bit for bit."""
    A = MATRICES["box512x16x12"]()
    monkeypatch.setenv("KR_STENCIL_PM", "0")
    st = _launches(A, "kskipmrr", 4, "3", monkeypatch)
    assert not any(k.startswith(("spmv2x2", "spmv_step2h")) for k in st), st
    assert st.get("spmv_step3_mrr_stencil", 0) > 0 and st.get("spmv_step2_mrr_stencil", 0) > 0, st
    b = np.random.default_rng(19).standard_normal(A.shape[0])
    out = []
    for on in ("0", "1"):
        monkeypatch.setenv("KR_BOX", on)
        with contextlib.redirect_stdout(io.StringIO()):
            x, info = _solver("kskipmrr")(A, b, tol=1e-10, maxiter=200, k=4)
        out.append((x.cpu().numpy(), info))
    np.testing.assert_array_equal(out[1][1]["residual"], out[0][1]["residual"])
    np.testing.assert_array_equal(out[1][0], out[0][0])
