"""HIP kernels through the C ABI vs the oracle (MI355X only).

Bitwise where the arithmetic is fixed-order: SpMV rows (scipy csr_matvec
order), the fused vector updates (numpy statement rounding) and the synthetic
generators. Dot products are deterministic but use a tree order, so they are
compared with a rounding bound instead.
"""
import ctypes
import math

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_matrix
from oracle import matrices

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch.device("cuda", 0)


def _lib():
    import parallel_krylov_amd._lib as L
    return L.library()


def _t(a, dev, dtype=None):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a if dtype is None else a.astype(dtype))).to(dev)


def _sync():
    import torch
    torch.cuda.synchronize()


def _irregular(n, seed):
    """Random sparse matrix with empty rows, a very long row and ragged rows."""
    rng = np.random.default_rng(seed)
    rows, cols = [], []
    for i in range(n):
        if i % 97 == 5:
            continue  # empty row
        cnt = 6000 if i == n // 2 else int(rng.integers(1, 40))
        c = np.unique(rng.integers(0, n, size=cnt))
        rows.append(np.full(c.size, i))
        cols.append(c)
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    v = rng.standard_normal(r.size)
    A = sp.csr_matrix((v, (r, c)), shape=(n, n))
    A.sort_indices()
    return A


MATRICES = {
    "poisson2d_33": lambda: golden_matrix(["poisson", 33, 2]),
    "poisson3d_17": lambda: golden_matrix(["poisson", 17, 3]),
    "banded_3001": lambda: golden_matrix(["banded", 3001, 13, 64, 0]),
    "banded63_2000": lambda: golden_matrix(["banded", 2000, 31, 256, 0]),
    "irregular_5000": lambda: _irregular(5000, 1),
    "single_row": lambda: sp.csr_matrix(np.array([[4.0]])),
}


@pytest.mark.parametrize("variant", ["0", "8", "10", "14"])
@pytest.mark.parametrize("name", list(MATRICES))
@pytest.mark.parametrize("rp64", [0, 1])
def test_spmv_bitwise_vs_scipy(torch_dev, monkeypatch, name, rp64, variant):
    """The SpMV kernels (row walk v1 0 and v2 10, product-then-sum v1 8 and v2 14) are
    bitwise scipy."""
    monkeypatch.setenv("KR_SPMV_VARIANT", variant)
    A = MATRICES[name]()
    n = A.shape[0]
    rng = np.random.default_rng(7)
    x = rng.standard_normal(n)
    x2 = rng.standard_normal(n)
    rp = _t(A.indptr, torch_dev, np.int64 if rp64 else np.int32)
    col = _t(A.indices, torch_dev, np.int32)
    val = _t(A.data, torch_dev, np.float64)
    xt, x2t = _t(x, torch_dev), _t(x2, torch_dev)
    import torch
    y = torch.full((n,), np.nan, dtype=torch.float64, device=torch_dev)
    y2 = torch.full((n,), np.nan, dtype=torch.float64, device=torch_dev)
    y3 = torch.full((n,), np.nan, dtype=torch.float64, device=torch_dev)
    _sync()
    lib = _lib()
    assert lib.kr_spmv_csr_f64(rp.data_ptr(), rp64, col.data_ptr(), val.data_ptr(), n,
                               xt.data_ptr(), y.data_ptr(), None) == 0
    assert lib.kr_spmv2_csr_f64(rp.data_ptr(), rp64, col.data_ptr(), val.data_ptr(), n,
                                xt.data_ptr(), x2t.data_ptr(), y2.data_ptr(), y3.data_ptr(),
                                None) == 0
    _sync()
    ref = A.dot(x)
    np.testing.assert_array_equal(y.cpu().numpy(), ref)
    np.testing.assert_array_equal(y2.cpu().numpy(), ref)
    np.testing.assert_array_equal(y3.cpu().numpy(), A.dot(x2))


def test_spmv_empty_and_errors(torch_dev):
    lib = _lib()
    assert lib.kr_spmv_csr_f64(None, 0, None, None, 0, None, None, None) == 0  # n = 0
    assert lib.kr_spmv_csr_f64(None, 0, None, None, 5, None, None, None) < 0
    assert b"NULL" in lib.kr_last_error()


@pytest.mark.parametrize("n", [1, 2, 255, 256, 257, 100003, 3 * 2 ** 20 + 1])
def test_dot_deterministic_and_accurate(torch_dev, n):
    import torch
    rng = np.random.default_rng(n)
    u = rng.standard_normal(n)
    v = rng.standard_normal(n)
    ut, vt = _t(u, torch_dev), _t(v, torch_dev)
    out = torch.zeros(2, dtype=torch.float64, device=torch_dev)
    _sync()
    lib = _lib()
    for i in range(2):
        assert lib.kr_dot_f64(ut.data_ptr(), vt.data_ptr(), n, out[i:].data_ptr(), None) == 0
    _sync()
    o = out.cpu().numpy()
    assert o[0] == o[1]  # deterministic
    exact = math.fsum(u * v)
    bound = 2 * n * np.finfo(float).eps * float(np.abs(u * v).sum()) + 1e-300
    assert abs(o[0] - exact) <= bound


def test_multidot_matches_dot(torch_dev):
    import torch
    n = 50001
    rng = np.random.default_rng(0)
    V = [_t(rng.standard_normal(n), torch_dev) for _ in range(5)]
    pairs = [(i, j) for i in range(5) for j in range(i, 5)][:13]
    us = (ctypes.c_void_p * len(pairs))(*[V[i].data_ptr() for i, _ in pairs])
    vs = (ctypes.c_void_p * len(pairs))(*[V[j].data_ptr() for _, j in pairs])
    out = torch.zeros(len(pairs), dtype=torch.float64, device=torch_dev)
    _sync()
    assert _lib().kr_multidot_f64(us, vs, len(pairs), n, out.data_ptr(), None) == 0
    _sync()
    Vh = [t.cpu().numpy() for t in V]
    for q, (i, j) in enumerate(pairs):
        exact = math.fsum(Vh[i] * Vh[j])
        assert abs(out[q].item() - exact) <= 1e-12 * np.abs(Vh[i] * Vh[j]).sum()


def test_norm2(torch_dev):
    import torch
    n = 123457
    u = np.random.default_rng(5).standard_normal(n)
    out = torch.zeros(1, dtype=torch.float64, device=torch_dev)
    ut = _t(u, torch_dev)
    _sync()
    assert _lib().kr_norm2_f64(ut.data_ptr(), n, out.data_ptr(), None) == 0
    _sync()
    assert abs(out.item() - math.sqrt(math.fsum(u * u))) <= 1e-13 * out.item()


def _gram_ref(rows_u, rows_v, m):
    """out[j] = <U[j//2], V[j//2 + j%2]> for j < m (the reference's Gram loops)."""
    return [math.fsum(rows_u[j // 2] * rows_v[j // 2 + j % 2]) for j in range(m)]


@pytest.mark.parametrize("k", [0, 1, 4, 12])
def test_gram_kskipmrr_matches_reference_loops(torch_dev, k):
    """kr_gram_kskipmrr_f64 = the alpha/beta/delta loops of
    v3/gpu/kskipmrr.py:53-61 (k=12: 77 dots, more than one multidot range),
    on strided basis rows (ld > n)."""
    import torch
    n, ld = 20011, 20011 + 5
    rng = np.random.default_rng(k)
    Ar = rng.standard_normal((k + 2, ld))
    Ay = rng.standard_normal((k + 1, ld))
    out = torch.full((6 * k + 6,), np.nan, dtype=torch.float64, device=torch_dev)
    art, ayt = _t(Ar, torch_dev), _t(Ay, torch_dev)
    _sync()
    assert _lib().kr_gram_kskipmrr_f64(art.data_ptr(), ayt.data_ptr(), k, n, ld,
                                       out.data_ptr(), None) == 0
    _sync()
    o = out.cpu().numpy()
    Arn, Ayn = Ar[:, :n], Ay[:, :n]
    alpha = _gram_ref(Arn, Arn, 2 * k + 3)
    beta = [0.0] + _gram_ref(Ayn, Arn, 2 * k + 2)[1:]
    delta = _gram_ref(Ayn, Ayn, 2 * k + 1)
    ref = np.array(alpha + beta + delta)
    assert o[2 * k + 3] == 0.0
    np.testing.assert_allclose(o, ref, rtol=0, atol=1e-12 * n)


@pytest.mark.parametrize("k", [0, 3, 10])
def test_gram_kskipcg_matches_reference_loops(torch_dev, k):
    """kr_gram_kskipcg_f64 = the a/f/c loops of v3/gpu/kskipcg.py:44-52, with
    f[2k+3] = 0 (the reference dots Ap[k+1] with the never-computed Ap[k+2])."""
    import torch
    n, ld = 9001, 9001
    rng = np.random.default_rng(100 + k)
    Ar = rng.standard_normal((k + 1, ld))
    Ap = rng.standard_normal((k + 2, ld))
    out = torch.full((6 * k + 7,), np.nan, dtype=torch.float64, device=torch_dev)
    art, apt = _t(Ar, torch_dev), _t(Ap, torch_dev)
    _sync()
    assert _lib().kr_gram_kskipcg_f64(art.data_ptr(), apt.data_ptr(), k, n, ld,
                                      out.data_ptr(), None) == 0
    _sync()
    o = out.cpu().numpy()
    Ap0 = np.vstack([Ap, np.zeros((1, ld))])
    a = _gram_ref(Ar, Ar, 2 * k + 1)
    f = _gram_ref(Ap0, Ap0, 2 * k + 4)
    c = _gram_ref(Ar, Ap0, 2 * k + 2)
    np.testing.assert_allclose(o, np.array(a + f + c), rtol=0, atol=1e-12 * n)
    assert o[2 * k + 1 + 2 * k + 3] == 0.0


def test_comm_single_rank_allreduce_and_halo(torch_dev):
    """The RCCL primitives on a one-rank communicator: the all-reduce leaves
    the buffer as is; a halo exchange with pieces to and from rank 0 itself
    copies the sent rows to the received positions (ncclSend/ncclRecv to self)."""
    import torch
    from parallel_krylov_amd.system import Communicator
    comm = Communicator(0, 1, torch_dev.index or 0, lambda data: data)
    lib = _lib()
    buf = _t(np.arange(7, dtype=np.float64), torch_dev)
    _sync()
    assert lib.kr_allreduce_sum_f64(comm.handle, buf.data_ptr(), 7, None) == 0
    _sync()
    np.testing.assert_array_equal(buf.cpu().numpy(), np.arange(7.0))
    x = np.random.default_rng(9).standard_normal(5000)
    xt = _t(x, torch_dev)
    send = (ctypes.c_int64 * 6)(0, 100, 300, 0, 2000, 17)
    recv = (ctypes.c_int64 * 6)(0, 4000, 300, 0, 4500, 17)
    _sync()
    assert lib.kr_halo_exchange_f64(comm.handle, xt.data_ptr(), recv, 2, send, 2, None) == 0
    _sync()
    ref = x.copy()
    ref[4000:4300] = x[100:400]
    ref[4500:4517] = x[2000:2017]
    np.testing.assert_array_equal(xt.cpu().numpy(), ref)
    bad = (ctypes.c_int64 * 3)(1, 0, 1)  # peer 1 of a one-rank communicator
    assert lib.kr_halo_exchange_f64(comm.handle, xt.data_ptr(), bad, 1, None, 0, None) < 0
    comm.close()


@pytest.mark.parametrize("n,offset", [(1, 0), (4097, 0), (4097, 1), (300000, 0)])
@pytest.mark.parametrize("first", [0, 1])
def test_update_mrr_bitwise(torch_dev, n, offset, first):
    import torch
    rng = np.random.default_rng(n + first)
    y, ar1, z, r, x = [rng.standard_normal(n + offset) for _ in range(5)]
    eta, zeta = -0.3141592653589793, 1.2345678901234567
    T = [_t(a, torch_dev) for a in (y, ar1, z, r, x)]
    P = [t[offset:].data_ptr() for t in T]  # offset 1: unaligned, scalar path
    _sync()
    assert _lib().kr_update_mrr_f64(eta, zeta, first, P[0], P[1], P[2], P[3], P[4], n,
                                    None) == 0
    _sync()
    y, ar1, z, r, x = [a[offset:] for a in (y, ar1, z, r, x)]
    if first:
        y_ref = zeta * ar1
        z_ref = -zeta * r
    else:
        y_ref = eta * y + zeta * ar1
        z_ref = eta * z - zeta * r
    r_ref = r - y_ref
    x_ref = x - z_ref
    for t, ref in zip((T[0], T[2], T[3], T[4]), (y_ref, z_ref, r_ref, x_ref)):
        np.testing.assert_array_equal(t[offset:].cpu().numpy(), ref)


def test_update_cg_bitwise(torch_dev):
    n = 12345
    rng = np.random.default_rng(5)
    x, p, r, v = [rng.standard_normal(n) for _ in range(4)]
    alpha = 0.7071067811865476
    T = [_t(a, torch_dev) for a in (x, p, r, v)]
    _sync()
    assert _lib().kr_update_cg_f64(alpha, *[t.data_ptr() for t in T], n, None) == 0
    _sync()
    np.testing.assert_array_equal(T[0].cpu().numpy(), x + alpha * p)
    np.testing.assert_array_equal(T[2].cpu().numpy(), r - alpha * v)


@pytest.mark.parametrize("spec,shards", [
    (("poisson", 19, 2), 1), (("poisson", 13, 3), 1), (("poisson", 13, 3), 3),
    (("banded", 4099, 13, 64, 0), 1), (("banded", 4099, 13, 64, 0), 4),
    (("banded", 3000, 31, 256, 5), 2),
])
def test_device_generators_and_sharded_spmv_bitwise(torch_dev, spec, shards):
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition
    A = golden_matrix(list(spec))
    n = A.shape[0]
    sysm = KrylovSystem(n, balanced_partition(n, shards), [0] * shards)
    if spec[0] == "poisson":
        sysm.gen_poisson(spec[1], spec[2])
    else:
        sysm.gen_banded(spec[2], spec[3], spec[4])
    sysm.finalize()
    for s in range(shards):
        r0, r1 = sysm.shard_rows(s)
        assert sysm.shard_info(s)["nnz"] == A[r0:r1].nnz
    x = np.random.default_rng(3).standard_normal(n)
    y = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
    np.testing.assert_array_equal(y, A.dot(x))
    b = sysm.gather(sysm.rhs(11)).cpu().numpy()
    np.testing.assert_array_equal(b, matrices.rhs(n, 11))
    sysm.close()


@pytest.mark.parametrize("side,nz,shards", [(13, 5, 1), (16, 7, 2), (9, 20, 3)])
def test_device_poisson_box_matches_scipy(torch_dev, side, nz, shards):
    """The Poisson generator on a side x side x nz box (n_global = side^2 nz):
    the 7-point operator of scipy's kronsum with a z-size of nz, bitwise."""
    import scipy.sparse as sp
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition

    def t(m):
        return sp.diags([-np.ones(m - 1), 2 * np.ones(m), -np.ones(m - 1)], [-1, 0, 1])
    A = sp.kronsum(sp.kronsum(t(side), t(side)), t(nz)).tocsr()
    A.sort_indices()
    n = A.shape[0]
    sysm = KrylovSystem(n, balanced_partition(n, shards), [0] * shards)
    sysm.gen_poisson(side, 3)
    sysm.finalize()
    for q in range(shards):
        r0, r1 = sysm.shard_rows(q)
        assert sysm.shard_info(q)["nnz"] == A[r0:r1].nnz
    x = np.random.default_rng(4).standard_normal(n)
    y = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
    np.testing.assert_array_equal(y, A.dot(x))
    sysm.close()


def test_adopted_csr_sharded_spmv_bitwise(torch_dev):
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition
    A = _irregular(3000, 2)
    n = A.shape[0]
    for shards in (1, 2, 5):
        sysm = KrylovSystem(n, balanced_partition(n, shards), [0] * shards)
        sysm.set_matrix(A)
        sysm.finalize()
        x = np.random.default_rng(shards).standard_normal(n)
        y = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
        np.testing.assert_array_equal(y, A.dot(x))
        sysm.close()


@pytest.mark.parametrize("slab", ["0", "8", "13", "37", "250", "4000", "37/2", "250/16"])
@pytest.mark.parametrize("spec", [("poisson", 40, 3), ("banded", 64000, 13, 64, 0)])
def test_slab_schedule_spmv_bitwise(torch_dev, monkeypatch, spec, slab):
    """KR_SLAB=S forces the slab row-block schedule (S row blocks per plane):
    every row block visited once, for the short-row and the product kernels,
    with a partial last plane and S not a multiple of 8."""
    from parallel_krylov_amd.system import KrylovSystem
    slab, _, sub = slab.partition("/")
    monkeypatch.setenv("KR_SLAB", slab)
    monkeypatch.setenv("KR_SLAB_SUB", sub or "0")
    A = golden_matrix(list(spec))
    n = A.shape[0]
    sysm = KrylovSystem(n, [0, n], [0])
    if spec[0] == "poisson":
        sysm.gen_poisson(spec[1], spec[2])
    else:
        sysm.gen_banded(spec[2], spec[3], spec[4])
    sysm.finalize()
    x = np.random.default_rng(5).standard_normal(n)
    y = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
    np.testing.assert_array_equal(y, A.dot(x))
    # the fused dual SpMV's Gram partials cover every row too (dot order
    # differs between schedules: compare with the contiguous one to rounding)
    out = sysm.solve("kskipmrr", sysm.rhs(1), tol=0.0, maxiter=10, k=4)
    sysm.close()
    monkeypatch.setenv("KR_SLAB", "0")
    ref_sys = KrylovSystem(n, [0, n], [0])
    ref_sys.set_matrix(A)
    ref_sys.finalize()
    ref = ref_sys.solve("kskipmrr", ref_sys.rhs(1), tol=0.0, maxiter=10, k=4)
    ref_sys.close()
    np.testing.assert_array_equal(out.info["nosl"], ref.info["nosl"])
    np.testing.assert_allclose(out.info["residual"], ref.info["residual"], rtol=1e-10)


def _offset_matrix(n, offsets, per_row, seed, sort=True):
    """Rows with `per_row` entries at column offsets drawn from `offsets`
    (clipped at the edges): a short-row matrix with len(offsets) distinct
    offsets, for the offset-mask layout."""
    rng = np.random.default_rng(seed)
    offsets = np.asarray(offsets)
    rows, cols = [], []
    for i in range(n):
        c = i + rng.choice(offsets, size=per_row, replace=False)
        c = c[(c >= 0) & (c < n)]
        rows.append(np.full(c.size, i))
        cols.append(c)
    A = sp.csr_matrix((rng.standard_normal(sum(c.size for c in cols)),
                       (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))
    A.sort_indices()
    if not sort:  # reverse each row's stored order (same matrix, unsorted)
        for i in range(n):
            a, b = A.indptr[i], A.indptr[i + 1]
            A.indices[a:b] = A.indices[a:b][::-1].copy()
            A.data[a:b] = A.data[a:b][::-1].copy()
        A.has_sorted_indices = False
    return A


def _nearly_symmetric(A):
    A = A.tocsr(copy=True)
    A[1000, 1001] = A[1000, 1001] * (1 + 2 ** -40)
    return A


MASKED = {
    # name: (builder, expected mask bits)
    "poisson2d_40": (lambda: golden_matrix(["poisson", 40, 2]), 8),
    "poisson3d_21": (lambda: golden_matrix(["poisson", 21, 3]), 8),
    "banded7_4099": (lambda: golden_matrix(["banded", 4099, 3, 64, 0]), 8),
    "offsets13": (lambda: _offset_matrix(6000, np.arange(-6, 7) * 37, 5, 1), 16),
    "offsets31": (lambda: _offset_matrix(6000, np.arange(-15, 16) * 5, 6, 2), 32),
    "offsets64": (lambda: _offset_matrix(6000, np.arange(-32, 32) * 3 + 1, 8, 3), 64),
    "offsets65": (lambda: _offset_matrix(6000, np.arange(-32, 33) * 3, 8, 4), 0),
    "unsorted": (lambda: _offset_matrix(3000, np.arange(-3, 4), 4, 5, sort=False), 0),
    # structurally symmetric, one value off its mirror
    "nearly_symmetric": (lambda: _nearly_symmetric(golden_matrix(["poisson", 14, 3])), 8),
    # long rows: masks (and the diagonal-offset values) only with KR_DIA on
    "long_rows": (lambda: golden_matrix(["banded", 3001, 13, 64, 0]), 32),
    "long_rows_63": (lambda: golden_matrix(["banded", 2000, 31, 256, 0]), 64),
}


@pytest.mark.parametrize("dia", ["2", "2/offset-major", "1", "0"])
@pytest.mark.parametrize("shards", [1, 3])
@pytest.mark.parametrize("name", list(MASKED))
def test_offset_mask_layout_spmv_bitwise(torch_dev, monkeypatch, name, shards, dia):
    """Matrices with <= 64 distinct column offsets (stencils, banded) use the
    offset-mask layout: the diagonal-offset SpMV (long rows by default,
    KR_DIA=1; every masked shard with KR_DIA=2; values row-block-major, or
    offset-major with KR_DIA_LAYOUT=0) or the short-row row walk without a
    column stream (short rows; KR_DIA=0 for every shard).
    The SpMV stays bitwise scipy's, with KR_MASK=0 (plain columns) as the
    control."""
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition
    builder, bits = MASKED[name]
    if dia.endswith("offset-major"):
        monkeypatch.setenv("KR_DIA_LAYOUT", "0")
        dia = dia.split("/")[0]
    if dia == "0" and name.startswith("long_rows"):
        bits = 0
    monkeypatch.setenv("KR_DIA", dia)
    A = builder()
    n = A.shape[0]
    x = np.random.default_rng(9).standard_normal(n)
    ref = sp.csr_matrix(A).dot(x) if name != "unsorted" else A.toarray().dot(x)
    for mask_env in ("1", "0"):
        monkeypatch.setenv("KR_MASK", mask_env)
        sysm = KrylovSystem(n, balanced_partition(n, shards), [0] * shards)
        sysm.set_matrix(A)
        sysm.finalize()
        lay = sysm.shard_layout(0)
        assert lay["mask_bits"] == (bits if mask_env == "1" else 0)
        y = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
        if name == "unsorted":  # stored order differs from scipy's sorted sum
            np.testing.assert_allclose(y, ref, rtol=1e-13, atol=1e-13)
        else:
            np.testing.assert_array_equal(y, A.dot(x))
        sysm.close()


def _few_values_matrix(n, nvals, seed, per_row=9, zeros=False):
    """Random-pattern CSR (plain columns: too many offsets for masks) whose
    values are drawn from `nvals` distinct doubles; with zeros=True the set
    holds +0.0 and -0.0 as two explicit stored values."""
    rng = np.random.default_rng(seed)
    table = rng.standard_normal(nvals)
    if zeros:
        table[0], table[1] = 0.0, -0.0
    rows, cols = [], []
    for i in range(n):
        c = np.unique(rng.integers(0, n, size=per_row))
        rows.append(np.full(c.size, i))
        cols.append(c)
    r, c = np.concatenate(rows), np.concatenate(cols)
    v = table[rng.integers(0, nvals, size=r.size)]
    v[:nvals] = table  # every value occurs
    A = sp.csr_matrix((v, (r, c)), shape=(n, n))  # (i, j) unique: no summing
    A.sort_indices()
    return A


VALUE_SETS = {
    # name: (builder, expected dictionary size)
    "poisson3d_21": (lambda: golden_matrix(["poisson", 21, 3]), 2),
    "poisson2d_40": (lambda: golden_matrix(["poisson", 40, 2]), 2),
    "cols_3": (lambda: _few_values_matrix(5000, 3, 1), 3),
    "cols_signed_zeros": (lambda: _few_values_matrix(5000, 5, 2, zeros=True), 5),
    "cols_256": (lambda: _few_values_matrix(6000, 256, 3), 256),
    "cols_257": (lambda: _few_values_matrix(6000, 257, 4), 0),
    "banded7_random": (lambda: golden_matrix(["banded", 4099, 3, 64, 0]), 0),
    "irregular": (lambda: _irregular(3000, 2), 0),
    "long_rows": (lambda: golden_matrix(["banded", 3001, 13, 64, 0]), 0),
}


@pytest.mark.parametrize("shards", [1, 3])
@pytest.mark.parametrize("name", list(VALUE_SETS))
def test_value_dictionary_spmv_bitwise(torch_dev, monkeypatch, name, shards):
    """Short-row blocks whose stored values take <= 256 distinct bit patterns
    stream 1-byte codes into a value table (row walk v2, with offset masks or
    plain columns); the SpMV stays bitwise scipy's, signed zeros included,
    with KR_VDICT=0 (8-byte values) as the control. 257 values, random
    values and long rows keep the 8-byte stream."""
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition
    builder, nd = VALUE_SETS[name]
    A = builder()
    n = A.shape[0]
    x = np.random.default_rng(11).standard_normal(n)
    x[::7] *= -1e-300  # tiny products: a -0.0 table entry must stay -0.0
    ref = A.dot(x)
    for vd in ("1", "0"):
        monkeypatch.setenv("KR_VDICT", vd)
        sysm = KrylovSystem(n, balanced_partition(n, shards), [0] * shards)
        sysm.set_matrix(A)
        sysm.finalize()
        got = [sysm.shard_layout(s)["dict_values"] for s in range(shards)]
        if vd == "0" or nd == 0:
            assert got == [0] * shards
        elif shards == 1:
            assert got == [nd]
        else:
            assert all(0 < g <= nd for g in got)
        y = sysm.gather(sysm.spmv(sysm.split(x))).cpu().numpy()
        np.testing.assert_array_equal(y, ref)
        assert np.array_equal(np.signbit(y), np.signbit(ref))
        sysm.close()


@pytest.mark.parametrize("grid", ["auto", "1", "2", "5"])
@pytest.mark.parametrize("shards", [1, 3])
@pytest.mark.parametrize("spec", [["banded", 3001, 13, 64, 0], ["banded", 2000, 31, 256, 0],
                                  ["banded", 4100, 7, 256, 3]])
def test_dia_symmetric_values_read_mirrored(torch_dev, monkeypatch, spec, shards, grid):
    """Symmetric banded values: the DIA SpMV reads every lower entry as the
    mirrored upper entry of an earlier row (kr_system_shard_dia_sym = 1) and
    stays bitwise scipy's; one perturbed value (pattern still symmetric)
    turns it off for the shard holding it, and KR_DIA_SYM=0 everywhere.
    With symmetric values and a band <= 256 the shard runs the row-block walk
    (format "dia_walk": mirrors from the LDS copy of this and the previous
    row block). KR_DIAW_GRID = 1, 2, 5 force long runs of blocks per
    workgroup at these sizes (the default grid gives every workgroup one
    block here), so the previous block's tails, segment starts and uneven
    runs are all exercised."""
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition
    if grid != "auto":
        monkeypatch.setenv("KR_DIAW_GRID", grid)
    A = golden_matrix(spec).tocsr()
    n = A.shape[0]
    B = A.copy()
    B.data = B.data.copy()
    r = 10
    B.data[B.indptr[r + 1] - 1] += 1e-3  # an upper entry of row 10, its mirror unchanged
    x = np.random.default_rng(3).standard_normal(n)
    # (the check is per shard: only the shard holding row 10 loses it)
    for M, env, want in ((A, "1", [1] * shards), (B, "1", [0] + [1] * (shards - 1)),
                         (A, "0", [0] * shards)):
        monkeypatch.setenv("KR_DIA_SYM", env)
        sysm = KrylovSystem(n, balanced_partition(n, shards), [0] * shards)
        try:
            sysm.set_matrix(M)
            sysm.finalize()
            assert [sysm.shard_format(s) for s in range(shards)] == \
                ["dia_walk" if w else "dia" for w in want]
            assert [sysm.shard_layout(s)["dia_sym"] for s in range(shards)] == want
            if grid != "auto":  # (capped at the shard's row blocks)
                assert all(sysm.shard_sched(s)["spmv_grid"] ==
                           min(int(grid), -(-sysm.shard_sched(s)["n"] // 256))
                           for s in range(shards) if want[s])
            y = sysm.gather(sysm.spmv(sysm.split(x)))
            np.testing.assert_array_equal(y.cpu().numpy(), M.dot(x))
        finally:
            sysm.close()


@pytest.mark.parametrize("grid", ["auto", "1", "3"])
@pytest.mark.parametrize("shards", [1, 3])
def test_dia_walk_mirror_positions_at_block_edges(torch_dev, monkeypatch, shards, grid):
    """The walk's one-store mirrors (KR_DIAW_MODE 3): lane p of a row block
    stores its upper value of offset o at position (p + o) & 255, the
    previous block's value when p + o >= 256 and this block's otherwise. The
    offsets here sit on every boundary of that rule -- 1 and 2, the wave edges
    63 / 64 / 65, 127 / 128 / 129, 191 / 192 / 193, and 254 / 255 / 256 (the
    largest band the walk takes) -- with random symmetric values, so a store
    at a wrong position or from the wrong block changes some row's sum. y is
    bitwise scipy's over 1 and 3 shards and forced walk grids (long runs)."""
    import scipy.sparse as sp
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition
    if grid != "auto":
        monkeypatch.setenv("KR_DIAW_GRID", grid)
    offs = [1, 2, 63, 64, 65, 127, 128, 129, 191, 192, 193, 200, 254, 255, 256]
    n = 5000
    rng = np.random.default_rng(11)
    rows, cols, vals = [np.arange(n)], [np.arange(n)], [np.full(n, 2.0 * len(offs) + 1.0)]
    for o in offs:
        i = np.arange(n - o)
        v = -rng.random(n - o)
        rows += [i, i + o]
        cols += [i + o, i]
        vals += [v, v]
    A = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                      shape=(n, n))
    A.sort_indices()
    x = rng.standard_normal(n)
    sysm = KrylovSystem(n, balanced_partition(n, shards), [0] * shards)
    try:
        sysm.set_matrix(A)
        sysm.finalize()
        assert [sysm.shard_format(s) for s in range(shards)] == ["dia_walk"] * shards
        y = sysm.gather(sysm.spmv(sysm.split(x)))
        np.testing.assert_array_equal(y.cpu().numpy(), A.dot(x))
    finally:
        sysm.close()


def _longest_full_run(M, lo, hi):
    """The DIA walk's run of full row blocks of shard rows [lo, hi), as
    finalize picks it (kr_engine.cpp build_masks): a 256-row block is full
    when it is whole and every row holds every offset of the shard; the
    first of the longest runs wins. Returns (first block, count)."""
    S = M[lo:hi]
    rows = np.repeat(np.arange(lo, hi), np.diff(S.indptr))
    nm = np.unique(S.indices - rows).size
    per_row = np.diff(S.indptr)
    nb = -(-(hi - lo) // 256)
    best, run, first = 0, 0, 0
    for b in range(nb):
        r = per_row[256 * b:256 * b + 256]
        full = r.size == 256 and bool(np.all(r == nm))
        run = run + 1 if full else 0
        if run > best:
            best, first = run, b + 1 - run
    return (first, best) if best else (0, 0)


@pytest.mark.parametrize("grid", ["auto", "2", "5"])
@pytest.mark.parametrize("shards", [1, 3])
def test_dia_walk_full_block_run_split_mid_band(torch_dev, monkeypatch, shards, grid):
    """The DIA walk's full-block run (masks not loaded, KR_DIAW_FULLRUN):
    a band matrix with one symmetric off-diagonal pair dropped in the middle
    of a shard splits its run of full blocks in two, so finalize must pick
    the longer part (dia_full_blocks / dia_full_first against a restatement),
    and the interior and boundary launches see the run shifted by their
    first row block. y is bitwise scipy's with the run and with every mask
    loaded (KR_DIAW_FULLRUN=0), over several forced walk grids."""
    import scipy.sparse as sp
    from parallel_krylov_amd.system import KrylovSystem, balanced_partition
    if grid != "auto":
        monkeypatch.setenv("KR_DIAW_GRID", grid)
    A = golden_matrix(["banded", 6000, 13, 64, 0]).tocsr().tolil()
    n = A.shape[0]
    part = balanced_partition(n, shards)
    # drop the pair (i, j), (j, i) 40 % into the last shard (symmetric values
    # stay symmetric, so the shard keeps the walk)
    i = part[-2] + (part[-1] - part[-2]) * 2 // 5
    j = max(c for c in A.rows[i] if c > i)
    A[i, j] = 0.0
    A[j, i] = 0.0
    A = sp.csr_matrix(A)
    A.eliminate_zeros()
    x = np.random.default_rng(5).standard_normal(n)
    want = [_longest_full_run(A, part[s], part[s + 1]) for s in range(shards)]
    # the dropped pair split the last shard's run: its longest part is shorter
    # than the run of the untouched matrix would be
    assert want[-1][1] < -(-(part[-1] - part[-2]) // 256) - 2
    for fullrun in ("1", "0"):
        monkeypatch.setenv("KR_DIAW_FULLRUN", fullrun)
        sysm = KrylovSystem(n, part, [0] * shards)
        try:
            sysm.set_matrix(A)
            sysm.finalize()
            assert [sysm.shard_format(s) for s in range(shards)] == ["dia_walk"] * shards
            got = [(sysm.shard_layout(s)["dia_full_first"], sysm.shard_layout(s)["dia_full_blocks"])
                   for s in range(shards)]
            assert got == (want if fullrun == "1" else [(0, 0)] * shards)
            y = sysm.gather(sysm.spmv(sysm.split(x)))
            np.testing.assert_array_equal(y.cpu().numpy(), A.dot(x))
        finally:
            sysm.close()
