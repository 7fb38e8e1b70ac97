"""Generate the golden vectors under tests/golden/ by running the REFERENCE.

Run in the build container only (the reference tree is not present on the GPU
box):  python tests/golden/make_golden.py

The reference (5enxia/parallel-krylov v3/cpu) has no tests and no fixtures
(.gitignore:14-17), so the known answers are produced here by
importing /root/reference/v3/cpu and running it on small synthetic systems.
Two harness shims are needed, and only here:
  * ``numpy.int = int`` -- the reference uses the alias numpy >= 1.24 removed
    (v3/cpu/common.py:34, v3/cpu/adaptivekskipmrr.py:18);
  * ``v3.cpu.kskipcg.dot`` / ``v3.cpu.adaptivekskipmrr.dot`` rebound to a
    function that sends sparse operands to ``A @ x`` (the reference calls
    ``numpy.dot(A, x)``, which raises on scipy sparse matrices).

Each case file stores the inputs (matrix spec + sha256 of its CSR arrays, b,
x0, parameters) and the reference's outputs (x, residual, nosl, khistory), plus
an ``envelope``: the per-entry relative change of the residual history when
the oracle's dot products are summed in other orders (max over blocked partial
sums as a GPU does, the exactly rounded sum, and six shuffled pairwise sums).
It is the measured rounding sensitivity of each entry and
scales the tolerance of the GPU parity tests.
"""
from __future__ import annotations

import contextlib
import io
import json
import math
import os
import sys

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REFERENCE = os.environ.get("KRYLOV_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from oracle import matrices  # noqa: E402
from oracle import v3cpu  # noqa: E402

CASES = []


def case(name, matrix, method, k=None, tol=1e-10, maxiter=None, x0=None):
    CASES.append(dict(name=name, matrix=matrix, method=method, k=k, tol=tol,
                      maxiter=maxiter, x0=x0))


P2D16 = ["poisson", 16, 2]
P3D16 = ["poisson", 16, 3]
P3D24 = ["poisson", 24, 3]
BAND = ["banded", 2000, 13, 64, 0]
for m in ("cg", "mrr"):
    case(f"p2d16_{m}", P2D16, m)
    case(f"p3d16_{m}", P3D16, m)
    case(f"band2000_{m}", BAND, m)
    case(f"p2d16_{m}_maxiter7", P2D16, m, maxiter=7)
    case(f"p2d16_{m}_x0", P2D16, m, x0=2)
for m in ("kskipcg", "kskipmrr", "adaptivekskipmrr"):
    for k in (0, 1, 4):
        case(f"p2d16_{m}_k{k}", P2D16, m, k=k)
    case(f"p3d16_{m}_k4", P3D16, m, k=4)
    case(f"band2000_{m}_k4", BAND, m, k=4)
    case(f"p2d16_{m}_k2_maxiter7", P2D16, m, k=2, maxiter=7)
    case(f"p2d16_{m}_k4_x0", P2D16, m, k=4, x0=2)
case("p3d24_adaptivekskipmrr_k12", P3D24, "adaptivekskipmrr", k=12, tol=1e-10)
case("p3d16_kskipmrr_k8_tol1e-12", P3D16, "kskipmrr", k=8, tol=1e-12)
# Round 2. The C5 generator (h = 31 offsets in [1, 256]: 63 nnz/row) at
# N = 3000: adaptive k = 4 is strictly checkable (no k change, envelope
# 8e-5); k = 12 and 2-D Poisson k = 12 roll back (reference: k changes at
# entries 4, 8, 12 and 7, 10), but a rollback is a rounding event of the
# k-skip recurrence, so those trajectories are chaotic under any change of
# summation order (entry 2 already moves by 1e-2..1e0). Their exact pin is
# tests/test_gpu_order.py (the oracle with the engine's summation order).
BAND5 = ["banded", 3000, 31, 256, 0]
case("band3000w256_adaptivekskipmrr_k4", BAND5, "adaptivekskipmrr", k=4)
case("band3000w256_kskipmrr_k4", BAND5, "kskipmrr", k=4)
case("band3000w256_mrr", BAND5, "mrr")
case("band3000w256_adaptivekskipmrr_k12", BAND5, "adaptivekskipmrr", k=12)
case("p2d16_adaptivekskipmrr_k12", P2D16, "adaptivekskipmrr", k=12)
# Round 3. C1 itself (BASELINE.json configs[0]: CG on 2-D 5-point Poisson
# 256^2 to tol 1e-10, ~880 iterations), so the GPU's C1 run is pinned against
# the reference's own history and x (tests/test_gpu_solvers.py picks every
# manifest case up).
case("p2d256_cg", ["poisson", 256, 2], "cg")
# Round 5. The C4 family (3-D 7-point Poisson, k-skip MrR k = 4) into the
# low-residual regime where the k-skip contract is defined:
# 64^3 to tol 1e-12, 64 history entries, 18 of them below 1e-8 (envelope up
# to ~2e-5 there: the k-skip recurrence amplifies rounding near convergence,
# but every perturbed order keeps the same nosl). b is not stored for
# N > 65536 (regenerated: default_rng(1).standard_normal(N), conftest).
case("p3d64_kskipmrr_k4_tol1e-12", ["poisson", 64, 3], "kskipmrr", k=4, tol=1e-12)


def build_matrix(spec):
    if spec[0] == "poisson":
        return matrices.poisson(spec[1], spec[2])
    if spec[0] == "banded":
        return matrices.banded(*spec[1:])
    raise ValueError(spec)


def import_reference():
    sys.path.insert(0, REFERENCE)
    np.int = int  # shim 1 (harness only)
    import v3.cpu.adaptivekskipmrr as ad
    import v3.cpu.cg as cg
    import v3.cpu.kskipcg as kc
    import v3.cpu.kskipmrr as km
    import v3.cpu.mrr as mr

    def sparse_dot(a, b):  # shim 2 (harness only)
        return a @ b if sp.issparse(a) else np.dot(a, b)

    kc.dot = sparse_dot
    ad.dot = sparse_dot
    return {"cg": cg.cg, "mrr": mr.mrr, "kskipcg": kc.kskipcg, "kskipmrr": km.kskipmrr,
            "adaptivekskipmrr": ad.adaptivekskipmrr}


def blocked_dot(u, v, block=256):
    p = np.asarray(u, dtype=np.float64) * np.asarray(v, dtype=np.float64)
    pad = (-p.size) % block
    if pad:
        p = np.concatenate([p, np.zeros(pad)])
    parts = p.reshape(-1, block).sum(axis=1)
    total = 0.0
    for q in parts:
        total += q
    return np.float64(total)


def exact_dot(u, v):
    return np.float64(math.fsum(np.asarray(u, dtype=np.float64) * np.asarray(v, dtype=np.float64)))


def permuted_dot(seed):
    def dot(u, v):
        p = np.asarray(u, dtype=np.float64) * np.asarray(v, dtype=np.float64)
        perm = np.random.default_rng(seed + p.size).permutation(p.size)
        return np.float64(np.sum(p[perm]))
    return dot


# Summation orders a GPU reduction could plausibly use: blocked partial sums,
# exactly rounded, and pairwise sums of shuffled products.
PERTURBATIONS = [blocked_dot, exact_dot] + [permuted_dot(s) for s in range(6)]


def run_perturbed(method, A, b, kwargs, dot):
    saved = (v3cpu._dot, v3cpu._norm)
    v3cpu._dot = dot
    v3cpu._norm = lambda v: np.float64(math.sqrt(dot(v, v)))
    try:
        with np.errstate(all="ignore"):
            return v3cpu.METHODS[method](A, b, **kwargs)
    finally:
        v3cpu._dot, v3cpu._norm = saved


def main(only=None):
    """Regenerate every case, or only the named ones (merged into the
    existing manifest, other fixture files untouched)."""
    ref = import_reference()
    manifest = []
    if only:
        with open(os.path.join(HERE, "manifest.json")) as f:
            manifest = [m for m in json.load(f) if m["name"] not in only]
    for c in CASES:
        if only and c["name"] not in only:
            continue
        A = build_matrix(c["matrix"])
        N = A.shape[0]
        b = np.random.default_rng(1).standard_normal(N)
        x0 = None if c["x0"] is None else np.random.default_rng(c["x0"]).standard_normal(N)
        kwargs = dict(tol=c["tol"], maxiter=c["maxiter"])
        if c["k"] is not None:
            kwargs["k"] = c["k"]
        with contextlib.redirect_stdout(io.StringIO()):
            x, info = ref[c["method"]](A, b, x=None if x0 is None else x0.copy(), **kwargs)
        res = np.asarray(info["residual"], dtype=np.float64)
        env = np.zeros(res.size)
        x_env = 0.0
        same_length = True
        for dot in PERTURBATIONS:
            xp, infop = run_perturbed(c["method"], A, b, dict(kwargs, x=x0), dot)
            resp = np.asarray(infop["residual"], dtype=np.float64)
            m = min(res.size, resp.size)
            d = np.full(res.size, np.inf)
            d[:m] = np.abs(resp[:m] - res[:m]) / np.maximum(np.abs(res[:m]), 1e-300)
            env = np.maximum(env, d)
            same_length &= resp.size == res.size and np.array_equal(infop["nosl"], info["nosl"])
            x_env = max(x_env, float(np.linalg.norm(xp - x) / np.linalg.norm(x)))
        out = dict(
            b=b, x=np.asarray(x, dtype=np.float64), residual=res,
            nosl=np.asarray(info["nosl"], dtype=np.int64), envelope=env,
            x_envelope=np.float64(x_env),
            same_length=np.bool_(same_length),
        )
        if x0 is not None:
            out["x0"] = x0
        if N > 65536:  # b = default_rng(1).standard_normal(N), regenerated by the loader
            del out["b"]
        if "khistory" in info:
            out["khistory"] = np.asarray(info["khistory"], dtype=np.int64)
        np.savez_compressed(os.path.join(HERE, c["name"] + ".npz"), **out)
        entry = dict(c, n=N, nnz=int(A.nnz), csr_sha256=matrices.csr_digest(A),
                     entries=int(res.size), iterations=int(out["nosl"][-1]))
        manifest.append(entry)
        print(f"{c['name']:34s} N={N:6d} entries={res.size:4d} "
              f"iters={entry['iterations']:4d} final={res[-1]:.3e} "
              f"env_max={np.max(env[np.isfinite(env)]) if np.isfinite(env).any() else 0:.1e}")
    order = [c["name"] for c in CASES]
    manifest.sort(key=lambda m: order.index(m["name"]))
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:] or None)
