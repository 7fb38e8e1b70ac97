"""Edge semantics of the drop-in API (MI355X): maxiter = 0 and the optional
divergence guard, against the oracle (the reference's v3/cpu arithmetic).

* maxiter = 0 (not None): CG and k-skip CG return the initial residual; the
  MrR family takes its first step unconditionally and writes nosl[1] of a
  length-1 array -- an IndexError in the reference (v3/cpu/mrr.py:31,
  kskipmrr.py:32), raised here too (both families).
* A residual that becomes NaN/Inf: the reference never tests for it (NaN
  passes neither `res < tol` nor `res > pre_res`), so the loop runs on to
  maxiter and prints `Status: diverged` (v3/common.py:17). That stays the
  default; KRYLOV_AMD_NAN_GUARD=1 stops at the first non-finite entry and
  returns the history so far (info['diverged'] = True).
  System: A = diag(+1, -1, ...), b = ones (indefinite: CG's <p, Ap> = 0 at
  the first step, MrR's Gram determinant 0 at the second).
"""
import contextlib
import importlib
import io

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_matrix
from oracle import v3cpu

pytestmark = pytest.mark.gpu


def _solver(method, family="gpu"):
    mod = importlib.import_module(f"parallel_krylov_amd.v3.{family}.{method}")
    return getattr(mod, method)


@pytest.fixture(scope="module")
def dist_single():
    import os
    import torch.distributed as dist
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29535")
        dist.init_process_group("gloo", rank=0, world_size=1)
    yield dist


@pytest.mark.parametrize("method,k", [("cg", None), ("kskipcg", 3)])
def test_maxiter_zero_returns_initial_residual(method, k):
    A = golden_matrix(["poisson", 16, 2])
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    kw = dict(tol=1e-10, maxiter=0)
    if k:
        kw["k"] = k
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        x, info = _solver(method)(A, b, **kw)
    x_ref, ref = v3cpu.METHODS[method](A, b, **kw)
    np.testing.assert_array_equal(info["nosl"], ref["nosl"])
    assert info["residual"].size == ref["residual"].size == 1
    assert abs(info["residual"][0] - ref["residual"][0]) <= 1e-14 * ref["residual"][0]
    np.testing.assert_array_equal(x.cpu().numpy(), x_ref)  # x0 = 0 untouched
    assert "Iteration:\t0 times" in out.getvalue()


@pytest.mark.parametrize("family", ["gpu", "gpu.mpi"])
@pytest.mark.parametrize("method", ["mrr", "kskipmrr", "adaptivekskipmrr"])
def test_maxiter_zero_mrr_family_raises_like_reference(dist_single, family, method):
    A = golden_matrix(["poisson", 8, 2])
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    kw = dict(tol=1e-10, maxiter=0)
    if "kskip" in method:
        kw["k"] = 2
    with pytest.raises(IndexError):
        v3cpu.METHODS[method](A, b, **kw)
    args = (A, b) if family == "gpu" else (None, A, b)
    with contextlib.redirect_stdout(io.StringIO()), pytest.raises(IndexError):
        _solver(method, family)(*args, **kw)


def _indefinite(n=512):
    return sp.diags(np.where(np.arange(n) % 2 == 0, 1.0, -1.0)).tocsr(), np.ones(n)


CASES = [("cg", None, 1), ("mrr", None, 2), ("kskipmrr", 2, 2), ("adaptivekskipmrr", 2, 2),
         ("kskipcg", 2, 1)]


@pytest.mark.parametrize("method,k,first_bad", CASES)
def test_nonfinite_default_runs_on_like_reference(monkeypatch, method, k, first_bad):
    monkeypatch.delenv("KRYLOV_AMD_NAN_GUARD", raising=False)
    A, b = _indefinite()
    kw = dict(tol=1e-10, maxiter=12)
    if k:
        kw["k"] = k
    out = io.StringIO()
    with contextlib.redirect_stdout(out), np.errstate(all="ignore"):
        x, info = _solver(method)(A, b, **kw)
        _, ref = v3cpu.METHODS[method](A, b, **kw)
    np.testing.assert_array_equal(info["nosl"], ref["nosl"])
    np.testing.assert_array_equal(info["residual"], ref["residual"])  # NaN where NaN
    assert not np.isfinite(info["residual"][first_bad])
    assert "diverged" not in info
    assert "Status:\t\tdiverged" in out.getvalue()


@pytest.mark.parametrize("family", ["gpu", "gpu.mpi"])
@pytest.mark.parametrize("method,k,first_bad", CASES)
def test_nan_guard_stops_at_first_nonfinite(dist_single, monkeypatch, family, method, k,
                                            first_bad):
    monkeypatch.setenv("KRYLOV_AMD_NAN_GUARD", "1")
    A, b = _indefinite()
    kw = dict(tol=1e-10, maxiter=12)
    if k:
        kw["k"] = k
    args = (A, b) if family == "gpu" else (None, A, b)
    out = io.StringIO()
    with contextlib.redirect_stdout(out), np.errstate(all="ignore"):
        x, info = _solver(method, family)(*args, **kw)
        _, ref = v3cpu.METHODS[method](A, b, **kw)
    assert info["diverged"] is True
    assert info["residual"].size == first_bad + 1
    np.testing.assert_array_equal(info["nosl"], ref["nosl"][:first_bad + 1])
    np.testing.assert_array_equal(info["residual"], ref["residual"][:first_bad + 1])
    assert "Status:\t\tdiverged" in out.getvalue()
    assert f"Iteration:\t{int(ref['nosl'][first_bad])} times" in out.getvalue()


def test_nan_guard_keeps_converging_runs_identical(monkeypatch):
    """The guard changes nothing on a finite trajectory (bitwise)."""
    A = golden_matrix(["poisson", 16, 2])
    b = np.random.default_rng(1).standard_normal(A.shape[0])
    res = []
    for g in ("0", "1"):
        monkeypatch.setenv("KRYLOV_AMD_NAN_GUARD", g)
        with contextlib.redirect_stdout(io.StringIO()):
            x, info = _solver("kskipmrr")(A, b, tol=1e-10, k=4)
        res.append((x.cpu().numpy(), info))
    np.testing.assert_array_equal(res[0][1]["residual"], res[1][1]["residual"])
    np.testing.assert_array_equal(res[0][0], res[1][0])
    assert res[1][1]["diverged"] is False
