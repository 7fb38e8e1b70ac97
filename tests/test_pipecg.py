"""Preconditioned / pipelined CG (reference
v1/threads/pipeline/*.py, restated in oracle/pipecg.py).

CPU: the oracle's PCG with M = I is the reference's v3/cpu CG statement for
statement, so it reproduces the reference-generated CG fixtures bit for bit
(the pin); the four variants agree with each other (same Krylov iteration);
the Python API's argument handling and the v1 banner.
GPU: every variant x {identity, Jacobi} x {1, 3 shards} against the oracle
on the same system: identical iteration counts, residual entries >= 1e-8
within the tolerance stated per variant, x within 1e-9 relative.
"""
import contextlib
import io

import numpy as np
import pytest

from conftest import golden_case, golden_manifest, golden_matrix

METHODS = ["pcg", "chronopoulos_gear", "gropp", "pipeline"]
# Residual-history tolerance (entries >= 1e-8) and x tolerance against the
# oracle. The GPU's dot products sum in another order than OpenBLAS, so the
# bar is 10x each variant's own reduction-order envelope (SURVEY.md §8c's
# rule), measured by test_oracle_reduction_order_envelope below (oracle vs the
# oracle with GPU-like 4096-lane strided dots, 2-D/3-D Poisson and band2000,
# identity and Jacobi): pcg and chronopoulos_gear recompute u = M^-1 r and
# stay at CG's envelope (<= 1.1e-14; the CG contract 1e-12); gropp's u and the
# pipelined u, w, z, q are recurrences, which amplify rounding like a k-skip
# method (gropp + Jacobi 2.6e-10, pipeline 3.6e-8).
RTOL = {"pcg": 1e-12, "chronopoulos_gear": 1e-12, "gropp": 3e-9, "pipeline": 5e-7}
XTOL = {"pcg": 1e-10, "chronopoulos_gear": 1e-10, "gropp": 1e-9, "pipeline": 1e-7}

CG_FIXTURES = [c for c in golden_manifest() if c["method"] == "cg"]


# ----------------------------------------------------------------- CPU
@pytest.mark.parametrize("c", CG_FIXTURES, ids=lambda c: c["name"])
def test_oracle_pcg_identity_is_reference_cg_bitwise(c):
    """The pin: PCG with M = I is v3/cpu/cg.py statement for statement."""
    from oracle import pipecg
    g = golden_case(c["name"])
    A = golden_matrix(c["matrix"])
    x0 = None if c["x0"] is None else np.random.default_rng(c["x0"]).standard_normal(A.shape[0])
    maxiter = None if c["maxiter"] is None else c["maxiter"] + 1  # v1: range(1, max_iter)
    _, nosl, res, x, _ = pipecg.pcg(A, g["b"], None, c["tol"], maxiter=maxiter, x0=x0,
                                    return_x=True)
    assert np.array_equal(res, g["residual"])
    assert np.array_equal(nosl, g["nosl"])
    assert np.array_equal(x, g["x"])


@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("spec", [("poisson", 16, 2), ("banded", 2000, 13, 64, 0)])
def test_oracle_variants_agree(method, spec):
    """Same Krylov iteration in exact arithmetic: every variant, preconditioned
    or not, tracks PCG's history and reaches the same x."""
    from oracle import pipecg
    A = golden_matrix(spec)
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    for pre in (None, pipecg.Jacobi(A)):
        _, n0, r0, x0, c0 = pipecg.pcg(A, b, pre, 1e-10, return_x=True)
        _, n1, r1, x1, c1 = pipecg.METHODS[method](A, b, pre, 1e-10, return_x=True)
        assert c0 and c1 and len(r1) == len(r0)
        keep = r0 >= 1e-8
        assert np.max(np.abs(r1[keep] - r0[keep]) / r0[keep]) < 1e-6
        assert np.linalg.norm(x1 - x0) / np.linalg.norm(x0) < 1e-8
        assert np.array_equal(n1, np.arange(len(r1)))


def _gpu_like_dot(a, b):
    """Dot product in a GPU-like order: 4096 lane-strided partials, then a sum."""
    p = a * b
    pad = np.zeros(-(-p.size // 4096) * 4096)
    pad[:p.size] = p
    return float(np.sum(pad.reshape(-1, 4096).sum(axis=0)))


@pytest.mark.parametrize("method", METHODS)
def test_oracle_reduction_order_envelope(monkeypatch, method):
    """The basis of RTOL / XTOL: the oracle against itself with another
    reduction order stays 10x inside them (same iteration counts)."""
    from oracle import pipecg
    worst = wx = 0.0
    for spec in (("poisson", 16, 2), ("poisson", 16, 3), ("banded", 2000, 13, 64, 0)):
        A = golden_matrix(spec)
        b = np.random.default_rng(1).standard_normal(A.shape[0])
        for pre in (None, pipecg.Jacobi(A)):
            monkeypatch.setattr(pipecg, "_dot", np.dot)
            _, n0, r0, x0, _ = pipecg.METHODS[method](A, b, pre, 1e-10, return_x=True)
            monkeypatch.setattr(pipecg, "_dot", _gpu_like_dot)
            _, n1, r1, x1, _ = pipecg.METHODS[method](A, b, pre, 1e-10, return_x=True)
            assert np.array_equal(n0, n1)
            keep = r0 >= 1e-8
            worst = max(worst, float(np.max(np.abs(r1[keep] - r0[keep]) / r0[keep])))
            wx = max(wx, float(np.linalg.norm(x1 - x0) / np.linalg.norm(x0)))
    assert worst * 10 <= RTOL[method], worst
    assert wx * 10 <= XTOL[method], wx


def test_jacobi_reduces_iterations_on_varying_diagonal():
    """Jacobi pays on a badly scaled SPD system (row scaling 1..1e4)."""
    import scipy.sparse as sp
    from oracle import pipecg
    A0 = golden_matrix(("banded", 2000, 13, 64, 0))
    s = sp.diags(np.sqrt(np.logspace(0, 4, A0.shape[0])))
    A = (s @ A0 @ s).tocsr()
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    _, _, r_id = pipecg.pcg(A, b, None, 1e-10)
    _, _, r_j = pipecg.pcg(A, b, pipecg.Jacobi(A), 1e-10)
    assert len(r_j) < len(r_id) // 2


def test_ilu_argument_forms():
    import scipy.sparse.linalg as spla
    from parallel_krylov_amd.v1.threads.pipeline.common import Jacobi, _diagonal, _ilu_factors
    A = golden_matrix(("banded", 200, 3, 8, 0)).tocsc()
    d = A.diagonal()
    assert _diagonal(None, 200) is None
    assert np.array_equal(_diagonal(Jacobi(A), 200), d)
    assert np.array_equal(_diagonal(d, 200), d)
    assert np.array_equal(_diagonal(list(d), 200), d)
    with pytest.raises(ValueError):
        _diagonal(d[:10], 200)
    # a SuperLU is taken as ILU factors (run() checks _ilu_factors first);
    # any other object is refused
    ilu = spla.spilu(A)
    L, U, pr, pc = _ilu_factors(ilu, 200)
    assert L.shape == U.shape == (200, 200) and np.array_equal(pr, ilu.perm_r)
    assert _ilu_factors((L, U, pr, pc), 200)[0] is L
    assert _ilu_factors(Jacobi(A), 200) is None and _ilu_factors(None, 200) is None
    # N = 4: a 4-tuple of numbers is a diagonal, not (L, U, perm_r, perm_c)
    assert _ilu_factors((2.0, 3.0, 4.0, 5.0), 4) is None
    assert np.array_equal(_diagonal((2.0, 3.0, 4.0, 5.0), 4), [2.0, 3.0, 4.0, 5.0])
    with pytest.raises(ValueError):
        _ilu_factors(ilu, 100)
    with pytest.raises(TypeError, match="ILU factors"):
        _diagonal(object(), 200)
    with pytest.raises(ValueError):
        Jacobi(d=np.zeros(3))
    with pytest.raises(ValueError):
        Jacobi(d=np.array([1.0, np.nan]))
    # a raw diagonal gets Jacobi's check: zero / non-finite entries are refused
    for bad in (0.0, np.inf, np.nan):
        dd = d.copy()
        dd[7] = bad
        with pytest.raises(ValueError, match="row 7"):
            _diagonal(dd, 200)


ILU_SYSTEMS = [("p2d32", ("poisson", 32, 2)), ("p3d10", ("poisson", 10, 3)),
               ("band2000", ("banded", 2000, 13, 64, 0))]


def _spilu(A, drop_tol):
    import scipy.sparse.linalg as spla
    return spla.spilu(A.tocsc(), drop_tol=drop_tol)


@pytest.mark.parametrize("drop_tol", [1e-4, 1e-2])
@pytest.mark.parametrize("sysname,spec", ILU_SYSTEMS, ids=[s[0] for s in ILU_SYSTEMS])
def test_ilu_sweeps_match_superlu(sysname, spec, drop_tol):
    """The oracle's restatement of the device sweeps (row-oriented, ascending
    columns) against scipy SuperLU's own solve -- the reference's `ilu` object
    (v1/threads/pipeline/pcg.py:26): equal to rounding (SuperLU's supernodal
    column solve orders the same subtractions differently)."""
    from oracle import pipecg
    A = golden_matrix(spec)
    ilu = _spilu(A, drop_tol)
    assert not np.array_equal(ilu.perm_c, np.arange(A.shape[0]))  # COLAMD: permutations used
    sw = pipecg.IluSweeps(ilu)
    for seed in range(3):
        v = np.random.default_rng(seed).standard_normal(A.shape[0])
        ref = ilu.solve(v)
        got = sw.solve(v)
        assert np.max(np.abs(got - ref)) / np.max(np.abs(ref)) < 1e-13


@pytest.mark.parametrize("method", METHODS)
def test_oracle_ilu_converges_faster(method):
    """ILU-preconditioned variants (spilu as the reference passes it) converge
    in far fewer iterations than M = I, and the four variants agree."""
    from oracle import pipecg
    A = golden_matrix(("poisson", 32, 2))
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    sw = pipecg.IluSweeps(_spilu(A, 1e-2))
    _, n_i, r_i = pipecg.METHODS[method](A, b, None, 1e-10)
    _, n_l, r_l = pipecg.METHODS[method](A, b, sw, 1e-10)
    assert r_l[-1] < 1e-10 and len(r_l) < len(r_i) // 2
    _, _, r_p = pipecg.pcg(A, b, sw, 1e-10)
    assert abs(len(r_l) - len(r_p)) <= 1


def test_v1_banner_text():
    from parallel_krylov_amd.v1.common import _end, _start
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        _start("pipeline", None)
        _end(1.5, False, 7, 0.25)
    assert buf.getvalue() == (
        "\033[32m# ================ INFO ================ #\033[0m\n"
        "Method:\t\tpipeline\ninitial_k:\tNone\ntime:\t\t1.5 s\nstatus:\t\tdiverged\n"
        "iteration:\t7 times\nfinal residual:\t0.25\n"
        "\033[32m# ====================================== #\033[0m\n")


def test_methods_registered():
    from parallel_krylov_amd import _lib
    for i, m in enumerate(METHODS):
        assert _lib.KR_METHOD[m] == 5 + i


# ----------------------------------------------------------------- GPU
def _systems():
    return [("p2d16", ("poisson", 16, 2)), ("p3d16", ("poisson", 16, 3)),
            ("band2000", ("banded", 2000, 13, 64, 0))]


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [1, 3])
@pytest.mark.parametrize("jacobi", [False, True])
@pytest.mark.parametrize("sysname,spec", _systems(), ids=[s[0] for s in _systems()])
@pytest.mark.parametrize("method", METHODS)
def test_gpu_matches_oracle(monkeypatch, method, sysname, spec, jacobi, shards):
    import importlib
    from oracle import pipecg
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", ",".join(["0"] * shards))
    mod = importlib.import_module(f"parallel_krylov_amd.v1.threads.pipeline.{method}")
    A = golden_matrix(spec)
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    pre_o = pipecg.Jacobi(A) if jacobi else None
    _, n_o, r_o, x_o, c_o = pipecg.METHODS[method](A, b, pre_o, 1e-10, return_x=True)
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        el, nosl, res, x, conv = getattr(mod, method)(A, b, A.diagonal() if jacobi else None,
                                                      1e-10, return_x=True)
    assert conv == c_o and "status:\t\tconverged" in out.getvalue()
    assert np.array_equal(nosl, n_o), (len(nosl), len(n_o))
    keep = r_o >= 1e-8
    rel = np.abs(res - r_o) / r_o
    assert rel[keep].max() < RTOL[method], rel[keep].max()
    assert rel.max() < 1e-5, rel.max()
    xh = x.cpu().numpy()
    assert np.linalg.norm(xh - x_o) / np.linalg.norm(x_o) < XTOL[method]


@pytest.mark.gpu
def test_gpu_pcg_identity_matches_reference_cg_fixture():
    """The GPU PCG with M = I against the reference-generated CG fixture
    (the CG parity contract: entries within 1e-12, same nosl)."""
    from parallel_krylov_amd.v1.threads.pipeline import pcg
    c = next(c for c in CG_FIXTURES if c["name"] == "band2000_cg")
    g = golden_case(c["name"])
    A = golden_matrix(c["matrix"])
    with contextlib.redirect_stdout(io.StringIO()):
        _, nosl, res = pcg(A, g["b"], None, c["tol"])
    assert np.array_equal(nosl, g["nosl"])
    assert np.max(np.abs(res - g["residual"]) / g["residual"]) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("method", METHODS)
def test_gpu_maxiter_truncation(method):
    """maxiter=m: iterations 1..m-1 (v1's range(1, max_iter)); not converged."""
    from oracle import pipecg
    import importlib
    mod = importlib.import_module(f"parallel_krylov_amd.v1.threads.pipeline.{method}")
    A = golden_matrix(("poisson", 16, 2))
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    _, n_o, r_o = pipecg.METHODS[method](A, b, None, 1e-10, maxiter=8)
    with contextlib.redirect_stdout(io.StringIO()):
        _, nosl, res, _, conv = getattr(mod, method)(A, b, None, 1e-10, maxiter=8,
                                                     return_x=True)
    assert not conv and len(res) == 8 and np.array_equal(nosl, n_o)
    assert np.max(np.abs(res - r_o) / r_o) < RTOL[method]


# (system, spilu drop_tol, shards requested) of the GPU ILU parity tests; 3-D
# Poisson at spilu's default 1e-4 is left out: its factors are not SPD there
# and every variant runs its 2N iterations without converging (oracle too).
ILU_CASES = [("p2d32", ("poisson", 32, 2), 1e-4, 1), ("p2d32", ("poisson", 32, 2), 1e-2, 1),
             ("p2d32", ("poisson", 32, 2), 1e-2, 3), ("p3d10", ("poisson", 10, 3), 1e-2, 1),
             ("band2000", ("banded", 2000, 13, 64, 0), 1e-4, 1),
             ("band2000", ("banded", 2000, 13, 64, 0), 1e-2, 3)]


@pytest.mark.gpu
@pytest.mark.parametrize("sysname,spec,drop_tol,shards", ILU_CASES,
                         ids=[f"{c[0]}-{c[2]:g}-{c[3]}" for c in ILU_CASES])
@pytest.mark.parametrize("method", METHODS)
def test_gpu_ilu_matches_oracle(monkeypatch, method, sysname, spec, drop_tol, shards):
    """ILU preconditioning on the device (kr_solve_set_precond_ilu: the two
    level-scheduled sweeps) with the reference's `ilu` object, a scipy spilu
    SuperLU, against the oracle run with the same factors through
    oracle.pipecg.IluSweeps (the device's sweep arithmetic): same nosl,
    residuals within each variant's dot-order envelope (RTOL), x within XTOL.
    A 3-shard request still runs the ILU system on one shard (the sweeps are
    sequential over the vector)."""
    import importlib
    from oracle import pipecg
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", ",".join(["0"] * shards))
    mod = importlib.import_module(f"parallel_krylov_amd.v1.threads.pipeline.{method}")
    A = golden_matrix(spec)
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    ilu = _spilu(A, drop_tol)
    _, n_o, r_o, x_o, c_o = pipecg.METHODS[method](A, b, pipecg.IluSweeps(ilu), 1e-10,
                                                  return_x=True)
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        _, nosl, res, x, conv = getattr(mod, method)(A, b, ilu, 1e-10, return_x=True)
    assert conv and c_o and "status:\t\tconverged" in out.getvalue()
    assert np.array_equal(nosl, n_o), (len(nosl), len(n_o))
    keep = r_o >= 1e-8
    rel = np.abs(res - r_o) / r_o
    assert rel[keep].max() < RTOL[method], rel[keep].max()
    xh = x.cpu().numpy()
    assert np.linalg.norm(xh - x_o) / np.linalg.norm(x_o) < XTOL[method]


@pytest.mark.gpu
@pytest.mark.parametrize("spec,drop_tol", [(("poisson", 32, 2), 1e-2), (("poisson", 10, 3), 1e-2),
                                           (("banded", 2000, 13, 64, 0), 1e-4)])
@pytest.mark.parametrize("method", ["pcg", "pipeline"])
def test_gpu_ilu_wide_levels_bitwise(monkeypatch, method, spec, drop_tol):
    """Wide levels get a launch of their own over the grid (IluSeg,
    KR_ILU_WIDE rows): with the threshold at 4 rows nearly every level of
    these small factors takes that path, and the solve is bitwise the one
    with every level in the single workgroup (KR_ILU_WIDE=0) -- every row is
    one thread's same arithmetic either way."""
    import importlib
    mod = importlib.import_module(f"parallel_krylov_amd.v1.threads.pipeline.{method}")
    A = golden_matrix(spec)
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    ilu = _spilu(A, drop_tol)
    out = {}
    for wide in ("0", "4"):
        monkeypatch.setenv("KR_ILU_WIDE", wide)
        with contextlib.redirect_stdout(io.StringIO()):
            _, nosl, res, x, conv = getattr(mod, method)(A, b, ilu, 1e-10, return_x=True)
        out[wide] = (nosl, res, x.cpu().numpy(), conv)
    assert out["0"][3] and out["4"][3]
    for q in range(3):
        np.testing.assert_array_equal(out["4"][q], out["0"][q])


@pytest.mark.gpu
@pytest.mark.parametrize("method", METHODS)
def test_gpu_ilu_against_superlu_solve(method):
    """The same solve against the oracle driven by SuperLU's own `solve` (the
    reference's call, pcg.py:41): the preconditioner applications differ in
    rounding only, so the iteration counts agree to one and both converge."""
    import importlib
    from oracle import pipecg
    mod = importlib.import_module(f"parallel_krylov_amd.v1.threads.pipeline.{method}")
    A = golden_matrix(("poisson", 32, 2))
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    ilu = _spilu(A, 1e-2)
    _, n_o, r_o = pipecg.METHODS[method](A, b, ilu, 1e-10)
    with contextlib.redirect_stdout(io.StringIO()):
        _, nosl, res = getattr(mod, method)(A, b, ilu, 1e-10)
    assert abs(len(res) - len(r_o)) <= 1 and res[-1] < 1e-10
    m = min(len(res), len(r_o)) - 2
    assert np.max(np.abs(res[:m] - r_o[:m]) / r_o[:m]) < 1e-6


@pytest.mark.gpu
def test_gpu_ilu_refused_on_several_shards():
    """kr_solve_set_precond_ilu on a multi-shard system is an error, not a
    silent per-shard (block) ILU."""
    import scipy.sparse.linalg as spla
    from parallel_krylov_amd._lib import KrylovError
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition
    A = golden_matrix(("poisson", 16, 2))
    n = A.shape[0]
    sysm = KrylovSystem(n, balanced_partition(n, 2), [0, 0])
    try:
        sysm.set_matrix(A)
        sysm.finalize()
        ilu = spla.spilu(A.tocsc())
        with pytest.raises(KrylovError, match="one-shard"):
            sysm.set_precond_ilu((ilu.L, ilu.U, ilu.perm_r, ilu.perm_c))
    finally:
        sysm.close()


def test_ilu0_c2_tool_factors():
    """tools/ilu_c2.py's ILU(0) of the 3-D Poisson matrix (the factors its
    C2-size measurement feeds kr_solve_set_precond_ilu): L unit lower, U upper
    with A's pattern, and L U equal to A on A's pattern (fill dropped)."""
    import importlib.util
    import os
    import scipy.sparse as sp
    from conftest import REPO
    spec = importlib.util.spec_from_file_location("ilu_c2", os.path.join(REPO, "tools", "ilu_c2.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    n = 6
    L, U, pr, pc = mod.ilu0_poisson3d(n)
    A = golden_matrix(("poisson", n, 3))
    assert np.array_equal(L.diagonal(), np.ones(n ** 3))
    assert sp.triu(L, 1).nnz == 0 and sp.tril(U, -1).nnz == 0
    assert (sp.tril(L, -1) != 0).sum() + (sp.triu(U) != 0).sum() == A.nnz
    D = (L @ U - A).tocsr()
    on = A.copy()
    on.data[:] = 1.0
    assert np.max(np.abs(D.multiply(on).data)) < 1e-14
    assert np.array_equal(pr, np.arange(n ** 3)) and np.array_equal(pc, pr)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [10, 17])
def test_gpu_ilu0_level_ordered_rows_bitwise(monkeypatch, n):
    """ILU(0) factors of a 3-D Poisson matrix (tools/ilu_c2.py; <= 3 entries
    per factor row) take the level-ordered rows (IluSweepArgs::ew, one round
    of loads indexed by the level position before the x loads); the solve is
    bitwise the CSR-chain sweep (KR_ILU_ELL=0), with and without the wide-level
    launches."""
    import importlib.util
    import os
    from conftest import REPO
    spec = importlib.util.spec_from_file_location("ilu_c2", os.path.join(REPO, "tools", "ilu_c2.py"))
    tool = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tool)
    from parallel_krylov_amd.v1.threads.pipeline.pcg import pcg
    A = golden_matrix(("poisson", n, 3))
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    factors = tool.ilu0_poisson3d(n)
    out = {}
    for ell in ("0", "1"):
        for wide in ("0", "8"):
            monkeypatch.setenv("KR_ILU_ELL", ell)
            monkeypatch.setenv("KR_ILU_WIDE", wide)
            with contextlib.redirect_stdout(io.StringIO()):
                _, nosl, res, x, conv = pcg(A, b, factors, 1e-10, return_x=True)
            out[ell, wide] = (nosl, res, x.cpu().numpy(), conv)
    ref = out["0", "0"]
    assert ref[3]
    for key, got in out.items():
        for q in range(3):
            np.testing.assert_array_equal(got[q], ref[q], err_msg=str(key))
