"""Multi-shard runs with every engine allocation poisoned (KR_POISON_ALLOC=1).

Round 3 saw one wrong history on the in-process multi-shard path: k-skip CG
on p3d64, k=3, three shards of one device, KR_FUSE=0, gave 76 entries where
every other run gives 70 ("Ordering audit"). A deterministic
solver can only do that through a missing happens-before edge or a read of
memory nothing wrote. KR_POISON_ALLOC=1 fills every device buffer the engine
allocates -- vectors with their pad and halo rows, reduction partials, slot
totals, gather and staging buffers, scalar state, stencil codes and masks --
with all-ones bytes (a NaN in every double) instead of zeros, so an
uninitialised read turns the history into NaN on the first run; the bitwise
comparisons against the GPU-order oracle (oracle/gpu_order.py) and the
reference fixtures then fail loudly.

In-process shards of one device share that device's stream by default
(KR_SHARED_STREAM=1, stream groups: stream order is the only edge); the
per-shard streams (KR_SHARED_STREAM=0) and pairs of shards per stream
(KR_SHARED_STREAM=2, the mixed geometry of several devices with several shards
each) take the cross-stream event edges (ev_in / ev_out, comm-stream copies,
ext_readers waits) that multi-device runs use, and the host-ordering knobs
(one host thread, wait-all, per-piece copies) only act there. So every case
below runs in all three stream layouts.

The cases are the multi-shard k-skip cases of test_gpu_stencil.py, the
round-3 failure itself (unfused and fused, per-shard host threads on and
off, and the round-2 "wait for every shard's copies" edge set), the sharded
golden fixtures, and CG / MrR with device-resident scalars on three shards.
"""
import contextlib
import dataclasses
import io

import numpy as np
import pytest

from conftest import golden_case, golden_manifest, golden_matrix
from oracle import gpu_order
from test_gpu_solvers import _solver, check_parity
from test_gpu_stencil import MATRICES, _bal, _system

pytestmark = pytest.mark.gpu

# (method, matrix, k, shards): multi-shard stencil / row-walk / banded cases
KSKIP = [
    ("kskipcg", "p3d64", 3, 3),  # the round-3 failure
    ("adaptivekskipmrr", "p3d32", 12, 3),
    ("adaptivekskipmrr", "box32x32x7", 8, 2),
    ("kskipmrr", "box64x16x9", 3, 2),
    ("kskipcg", "band_far", 2, 3),
    ("kskipcg", "box128x32x9", 3, 3),
    ("kskipmrr", "p3d32", 4, 3),
]


def _run(monkeypatch, env, method, A, b, shards, **kw):
    monkeypatch.setenv("KR_POISON_ALLOC", "1")
    monkeypatch.setenv("KRYLOV_AMD_SHARDS", ",".join(["0"] * shards))
    for key, val in env.items():
        monkeypatch.setenv(key, val)
    with contextlib.redirect_stdout(io.StringIO()):
        x, info = _solver(method)(A, b, **kw)
    return x.cpu().numpy(), info


# stream layouts of in-process shards (KR_SHARED_STREAM): one stream per
# device (default), one per shard, pairs of shards per stream
STREAMS = pytest.mark.parametrize("streams", ["1", "0", "2"],
                                  ids=["shared-stream", "stream-per-shard", "stream-pairs"])


@STREAMS
@pytest.mark.parametrize("env", [{"KR_FUSE": "0"}, {"KR_FUSE": "1"}],
                         ids=["unfused", "fused"])
@pytest.mark.parametrize("method,name,k,shards", KSKIP)
def test_poisoned_kskip_bitwise_gpu_order_oracle(monkeypatch, method, name, k, shards, env,
                                                 streams):
    """Every multi-shard k-skip history and x under poisoned allocations equal
    the GPU-order oracle bit for bit (no NaN, no stale operand), in every
    stream layout."""
    env = dict(env, KR_SHARED_STREAM=streams)
    A = MATRICES[name]()
    n = A.shape[0]
    b = np.random.default_rng(3).standard_normal(n)
    sysm = _system(A, shards)
    sc = [gpu_order.ShardSched(**sysm.shard_sched(s)) for s in range(shards)]
    sysm.close()
    assert sc == gpu_order.shard_scheds(A, _bal(n, shards))
    kw = dict(tol=1e-10, k=k, maxiter=300)
    x, info = _run(monkeypatch, env, method, A, b, shards, **kw)
    assert np.all(np.isfinite(info["residual"])) and np.all(np.isfinite(x))
    x_ref, ref = gpu_order.run(method, A, b, sc, **kw)
    np.testing.assert_array_equal(info["nosl"], ref["nosl"])
    if "khistory" in ref:
        np.testing.assert_array_equal(info["khistory"], ref["khistory"])
    np.testing.assert_array_equal(info["residual"], ref["residual"])
    np.testing.assert_array_equal(x, x_ref)


@STREAMS
@pytest.mark.parametrize("env", [
    {"KR_FUSE": "0", "KR_HOST_THREADS": "0"},
    {"KR_FUSE": "0", "KR_BOUNDARY_WAIT_ALL": "1"},
    {"KR_FUSE": "0", "KR_HALO_KERNEL": "0"},
    {"KR_FUSE": "0", "KR_OVERLAP": "0"},
], ids=["one-thread", "wait-all", "halo-copies", "no-split"])
def test_poisoned_round3_case_every_ordering(monkeypatch, env, streams):
    """The round-3 case under each host ordering the engine offers: one host
    thread, the round-2 edge set (every boundary launch waits for every
    shard's halo copies), per-piece copies instead of the gather launch, and
    the un-split SpMV (summed as one launch per shard, which the oracle
    restates when no shard has interior rows) -- all bitwise the GPU-order
    oracle. The three orderings act on the cross-stream edges, so they are
    real only with a stream per shard or per pair (the shared stream has no
    such edge); every layout is run."""
    env = dict(env, KR_SHARED_STREAM=streams)
    A = MATRICES["p3d64"]()
    n = A.shape[0]
    b = np.random.default_rng(3).standard_normal(n)
    sc = gpu_order.shard_scheds(A, _bal(n, 3))
    if env.get("KR_OVERLAP") == "0":  # one launch per shard: the oracle's un-split order
        sc = [dataclasses.replace(s, int_lo=0, int_hi=0) for s in sc]
    kw = dict(tol=1e-10, k=3, maxiter=300)
    x, info = _run(monkeypatch, env, "kskipcg", A, b, 3, **kw)
    x_ref, ref = gpu_order.run("kskipcg", A, b, sc, **kw)
    np.testing.assert_array_equal(info["nosl"], ref["nosl"])
    np.testing.assert_array_equal(info["residual"], ref["residual"])
    np.testing.assert_array_equal(x, x_ref)


SHARDED = ["p3d16_cg", "p3d16_mrr", "p3d16_kskipcg_k4", "p3d16_kskipmrr_k4",
           "p3d16_adaptivekskipmrr_k4", "band2000_kskipmrr_k4", "band2000_mrr",
           "band3000w256_adaptivekskipmrr_k12"]


@STREAMS
@pytest.mark.parametrize("name", [n for n in SHARDED
                                  if any(c["name"] == n for c in golden_manifest())])
def test_poisoned_shards_match_reference(monkeypatch, name, streams):
    """The reference fixtures on three poisoned shards keep the §8(c) contract."""
    c = next(c for c in golden_manifest() if c["name"] == name)
    g = golden_case(name)
    A = golden_matrix(c["matrix"])
    kw = dict(tol=c["tol"], maxiter=c["maxiter"])
    if c["k"] is not None:
        kw["k"] = c["k"]
    x, info = _run(monkeypatch, {"KR_SHARED_STREAM": streams}, c["method"], A, g["b"], 3, **kw)
    check_parity(c, g, x, info)


@STREAMS
@pytest.mark.parametrize("method", ["cg", "mrr"])
def test_poisoned_device_scalars_bitwise_clean(monkeypatch, method, streams):
    """CG / MrR with device scalars on three shards: the poisoned run equals
    the run on zeroed allocations bit for bit."""
    A = MATRICES["p3d64"]()
    b = np.random.default_rng(11).standard_normal(A.shape[0])
    kw = dict(tol=1e-10, maxiter=200)
    x1, i1 = _run(monkeypatch, {"KR_SHARED_STREAM": streams}, method, A, b, 3, **kw)
    monkeypatch.setenv("KR_POISON_ALLOC", "0")
    with contextlib.redirect_stdout(io.StringIO()):
        x0, i0 = _solver(method)(A, b, **kw)
    np.testing.assert_array_equal(i1["nosl"], i0["nosl"])
    np.testing.assert_array_equal(i1["residual"], i0["residual"])
    np.testing.assert_array_equal(x1, x0.cpu().numpy())


@pytest.mark.parametrize("name", ["p3d64", "box64x16x9", "band_far", "p2d512x6"])
def test_poisoned_spmv_bitwise_scipy(monkeypatch, name):
    """y = A x on three poisoned shards (split SpMV, halo gather) is scipy's."""
    monkeypatch.setenv("KR_POISON_ALLOC", "1")
    A = MATRICES[name]()
    x = np.random.default_rng(7).standard_normal(A.shape[0])
    sysm = _system(A, 3)
    y = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
    sysm.close()
    np.testing.assert_array_equal(y, A @ x)
