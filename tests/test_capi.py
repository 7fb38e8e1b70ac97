"""The C-ABI library on the CPU: it loads, exports every declared symbol, and
its host-only entry points (scalar recurrences, halo planner) agree with the
oracle. No device compute is called here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO, golden_case, golden_manifest, golden_matrix
from oracle import v3cpu

HEADER = os.path.join(REPO, "include", "krylov_amd.h")


def _lib():
    import parallel_krylov_amd._lib as L
    return L.library()


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(kr_\w+)\s*\(", text, re.M)))


def test_library_exports_every_declared_symbol():
    lib = _lib()
    names = declared_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    import parallel_krylov_amd._lib as L
    assert sorted(L.exported_symbols()) == names  # ctypes table covers the header


def test_version_and_device_count_without_gpu():
    lib = _lib()
    import parallel_krylov_amd._lib as L
    assert lib.kr_version() == L.KR_ABI_VERSION == 205
    c = ctypes.c_int(-1)
    assert lib.kr_device_count(ctypes.byref(c)) == 0
    assert c.value >= 0


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _native_kskipmrr(k, alpha, beta, delta):
    lib = _lib()
    a, b, d = alpha.copy(), beta.copy(), delta.copy()
    z = np.zeros(k + 1)
    e = np.zeros(k + 1)
    assert lib.kr_kskipmrr_recurrence(k, _dp(a), _dp(b), _dp(d), _dp(z), _dp(e)) == 0
    return z, e


def _native_kskipcg(k, a, f, c):
    lib = _lib()
    a, f, c = a.copy(), f.copy(), c.copy()
    al = np.zeros(k + 1)
    be = np.zeros(k + 1)
    assert lib.kr_kskipcg_recurrence(k, _dp(a), _dp(f), _dp(c), _dp(al), _dp(be)) == 0
    return al, be


def _basis_gram_mrr(A, r, y, k):
    """Gram arrays of a real k-skip MrR outer iteration (oracle order)."""
    Ar = [r]
    for _ in range(k + 1):
        Ar.append(A.dot(Ar[-1]))
    Ay = [y]
    for _ in range(k):
        Ay.append(A.dot(Ay[-1]))
    alpha = np.array([np.dot(Ar[j // 2], Ar[j // 2 + j % 2]) for j in range(2 * k + 3)])
    beta = np.zeros(2 * k + 2)
    for j in range(1, 2 * k + 2):
        beta[j] = np.dot(Ay[j // 2], Ar[j // 2 + j % 2])
    delta = np.array([np.dot(Ay[j // 2], Ay[j // 2 + j % 2]) for j in range(2 * k + 1)])
    return alpha, beta, delta


@pytest.mark.parametrize("k", [0, 1, 2, 4, 8, 12])
def test_kskipmrr_recurrence_bitwise_vs_oracle(k):
    A = golden_matrix(["poisson", 12, 2])
    rng = np.random.default_rng(k)
    for trial in range(20):
        r = rng.standard_normal(A.shape[0])
        y = rng.standard_normal(A.shape[0])
        alpha, beta, delta = _basis_gram_mrr(A, r, y, k)
        ref = v3cpu.kskipmrr_scalars(k, alpha.copy(), beta.copy(), delta.copy())
        z, e = _native_kskipmrr(k, alpha, beta, delta)
        np.testing.assert_array_equal(z, np.array([p[0] for p in ref]))
        np.testing.assert_array_equal(e, np.array([p[1] for p in ref]))


@pytest.mark.parametrize("k", [0, 1, 2, 4, 8])
def test_kskipcg_recurrence_bitwise_vs_oracle(k):
    A = golden_matrix(["poisson", 12, 2])
    rng = np.random.default_rng(100 + k)
    for trial in range(20):
        r = rng.standard_normal(A.shape[0])
        p = rng.standard_normal(A.shape[0])
        Ar = [r]
        for _ in range(k + 1):
            Ar.append(A.dot(Ar[-1]))
        Ap = [p]
        for _ in range(k + 2):
            Ap.append(A.dot(Ap[-1]))
        Ap.append(np.zeros_like(p))
        a = np.zeros(2 * k + 2)
        f = np.zeros(2 * k + 4)
        c = np.zeros(2 * k + 2)
        for j in range(2 * k + 1):
            a[j] = np.dot(Ar[j // 2], Ar[j // 2 + j % 2])
        for j in range(2 * k + 4):
            f[j] = np.dot(Ap[j // 2], Ap[j // 2 + j % 2]) if j < 2 * k + 3 else 0.0
        for j in range(2 * k + 2):
            c[j] = np.dot(Ar[j // 2], Ap[j // 2 + j % 2])
        ref = v3cpu.kskipcg_scalars(k, a.copy(), f.copy(), c.copy())
        al, be = _native_kskipcg(k, a, f, c)
        np.testing.assert_array_equal(al, np.array([q[0] for q in ref]))
        np.testing.assert_array_equal(be, np.array([q[1] for q in ref]))


def test_recurrence_uses_libm_pow_not_square():
    # Inputs where pow(x, 2) != x*x: the native recurrence must follow pow.
    import math
    rng = np.random.default_rng(0)
    xs = rng.standard_normal(200000)
    diff = [v for v in xs if math.pow(v, 2.0) != v * v]
    assert diff, "expected some inputs where libm pow differs from x*x"
    # k = 0 k-skip CG: beta = alpha**2 * f2 / a0 - 1 with alpha = a0 / f1
    for v in diff[:50]:
        a = np.array([v, 0.0])
        f = np.array([0.0, 1.0, 1.0, 0.0])
        c = np.zeros(2)
        al, be = _native_kskipcg(0, a, f, c)
        alpha = np.float64(v) / np.float64(1.0)
        assert be[0] == alpha ** 2 * np.float64(1.0) / np.float64(v) - 1


def _plan(part, lo, hi, me):
    lib = _lib()
    P = len(part) - 1
    cap = 2 * P
    arr = lambda v: (ctypes.c_int64 * len(v))(*v)
    rout = (ctypes.c_int64 * (3 * cap))()
    sout = (ctypes.c_int64 * (3 * cap))()
    nr, ns = ctypes.c_int(), ctypes.c_int()
    assert lib.kr_halo_plan(P, arr(part), arr(lo), arr(hi), me, rout, ctypes.byref(nr), sout,
                            ctypes.byref(ns), cap) == 0
    r = [tuple(rout[3 * q:3 * q + 3]) for q in range(nr.value)]
    s = [tuple(sout[3 * q:3 * q + 3]) for q in range(ns.value)]
    return r, s


@pytest.mark.parametrize("P", [1, 2, 3, 8])
def test_halo_plan_is_consistent(P):
    from parallel_krylov_amd.system import balanced_partition
    A = golden_matrix(["poisson", 10, 3])
    n = A.shape[0]
    part = balanced_partition(n, P)
    lo, hi = [], []
    for t in range(P):
        blk = A[part[t]:part[t + 1]]
        lo.append(min(int(blk.indices.min()), part[t]))
        hi.append(max(int(blk.indices.max()), part[t + 1] - 1))
    plans = [_plan(part, lo, hi, me) for me in range(P)]
    for me, (recv, send) in enumerate(plans):
        # received rows = exactly the needed rows outside my block
        got = set()
        for peer, g0, cnt in recv:
            assert part[peer] <= g0 and g0 + cnt <= part[peer + 1]
            got.update(range(g0, g0 + cnt))
        need = set(range(lo[me], hi[me] + 1)) - set(range(part[me], part[me + 1]))
        assert got == need
        # every send of mine is a recv of the peer, same range
        for peer, g0, cnt in send:
            assert (me, g0, cnt) in plans[peer][0]
    # one shard: no exchange at all
    if P == 1:
        assert plans[0] == ([], [])


def _row_sched(nrb, slab, grid, sub=0):
    """Host restatement of the SpMV row-block schedule (RowSched in
    kr_kernels.hip): the row blocks every workgroup visits."""
    out = []
    for blk in range(grid):
        if grid % 8 == 0:
            q, j, step = blk & 7, blk >> 3, grid >> 3
            if slab >= 8:
                off, w = slab * q // 8, slab * (q + 1) // 8 - slab * q // 8
                planes = (nrb + slab - 1) // slab
                full, rem = planes - 1, nrb - (planes - 1) * slab
                sw = min(sub, w) if sub > 0 else w
                nc = (w + sw - 1) // sw
                chunks = []
                for c in range(nc):
                    wc = min(sw, w - c * sw)
                    chunks.append((c, wc, full * wc + min(wc, max(0, rem - off - c * sw))))
                count = sum(ch[2] for ch in chunks)

                def rb(v, off=off, sw=sw, chunks=chunks):
                    for c, wc, cnt in chunks:
                        if v < cnt:
                            return (v // wc) * slab + off + c * sw + v % wc
                        v -= cnt
                    raise AssertionError("v out of range")
            else:
                chunk = (nrb + 7) // 8
                base = q * chunk
                count = max(0, min(nrb, base + chunk) - base)
                rb = lambda v, base=base: base + v  # noqa: E731
        else:
            j, step, count = blk, grid, nrb
            rb = lambda v: v  # noqa: E731
        while j < count:
            out.append(rb(j))
            j += step
    return out


@pytest.mark.parametrize("nrb", [1, 7, 8, 250, 1023, 5003])
@pytest.mark.parametrize("slab", [0, 8, 13, 250, 1024, 100000])
@pytest.mark.parametrize("grid", [1, 24, 2048])
@pytest.mark.parametrize("sub", [0, 1, 5, 32])
def test_row_schedule_visits_every_block_once(nrb, slab, grid, sub):
    assert sorted(_row_sched(nrb, slab, grid, sub)) == list(range(nrb))
