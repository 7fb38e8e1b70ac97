"""The oracle against the reference's own outputs (CPU only).

tests/golden/*.npz were produced by running the reference v3/cpu code
(tests/golden/make_golden.py). The restatement in oracle/v3cpu.py must
reproduce them bit for bit on the same machine: same numpy/scipy calls in the
same order. Matrix builders are pinned by sha256 and against scipy.kronsum.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_case, golden_manifest, golden_matrix
from oracle import matrices, v3cpu

CASES = golden_manifest()


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_oracle_matches_reference_bitwise(c):
    g = golden_case(c["name"])
    A = golden_matrix(c["matrix"])
    assert matrices.csr_digest(A) == c["csr_sha256"]
    kw = dict(tol=c["tol"], maxiter=c["maxiter"])
    if c["k"] is not None:
        kw["k"] = c["k"]
    x, info = v3cpu.METHODS[c["method"]](A, g["b"], x=g.get("x0"), **kw)
    np.testing.assert_array_equal(info["nosl"], g["nosl"])
    np.testing.assert_array_equal(info["residual"], g["residual"])
    np.testing.assert_array_equal(x, g["x"])
    if "khistory" in g:
        np.testing.assert_array_equal(info["khistory"], g["khistory"])


@pytest.mark.parametrize("n,dim", [(7, 2), (16, 2), (5, 3), (16, 3)])
def test_poisson_equals_scipy_kronsum(n, dim):
    T = sp.diags([-1.0, 2.0, -1.0], [-1, 0, 1], shape=(n, n))
    K = T
    for _ in range(dim - 1):
        K = sp.kronsum(K, T)
    K = sp.csr_matrix(K)
    K.sort_indices()
    A = matrices.poisson(n, dim)
    assert A.nnz == K.nnz
    np.testing.assert_array_equal(A.indptr, K.indptr)
    np.testing.assert_array_equal(A.indices, K.indices)
    np.testing.assert_array_equal(A.data, K.data)


def test_banded_is_spd_and_symmetric():
    A = matrices.banded(500, 13, 64, 0)
    assert (A != A.T).nnz == 0
    assert A.nnz / A.shape[0] > 24  # 27 per interior row, fewer near the ends
    d = A.diagonal()
    off = np.asarray(abs(A).sum(axis=1)).ravel() - d
    assert np.all(d > off)  # strictly diagonally dominant => SPD
    off_sorted = matrices.banded_offsets(13, 64, 0)
    assert len(set(off_sorted)) == 13 and off_sorted.min() >= 1 and off_sorted.max() <= 64


def test_rhs_is_exact_and_in_range():
    b = matrices.rhs(10000, 7)
    assert b.min() >= -1.0 and b.max() < 1.0
    # 2u - 1 with u on a 2^-53 grid is exact: recovering u gives integers
    m = (b + 1.0) / 2.0 * 2.0 ** 53
    assert np.all(m == np.floor(m))
    np.testing.assert_array_equal(matrices.rhs(100, 7, row0=50), b[50:150])


def test_scalar_recurrences_follow_reference_order():
    # k-skip MrR: the oracle's recurrence helpers equal an inline restatement
    rng = np.random.default_rng(3)
    for k in (0, 1, 3, 4, 8):
        a = rng.standard_normal(2 * k + 3)
        b = rng.standard_normal(2 * k + 2)
        d = rng.standard_normal(2 * k + 1)
        out = v3cpu.kskipmrr_scalars(k, a.copy(), b.copy(), d.copy())
        assert len(out) == k + 1
        assert all(np.isfinite(z) or True for z, _ in out)


def test_parcsr_matvec_is_scipy_bitwise():
    """oracle.matrices.ParCSR (oracle/csrmv.c: rows over OpenMP threads, each
    summed in stored order from 0.0) equals scipy's csr_matvec bit for bit --
    on the golden families, an irregular matrix with empty and long rows, and
    x with wide exponents -- so the full-size parity tests may use it as the
    oracle's A.dot."""
    import scipy.sparse as sp
    from oracle import matrices
    if not matrices.ParCSR.available():
        pytest.skip("oracle/liboracle_csrmv.so not built (oracle/build.sh failed or not run)")
    rng = np.random.default_rng(7)
    n = 4001
    rows = np.repeat(np.arange(n), rng.integers(0, 40, n))
    rows = np.concatenate([rows, np.full(3000, n // 2)])
    cols = rng.integers(0, n, rows.size)
    irr = sp.csr_matrix((rng.standard_normal(rows.size) * 10.0 ** rng.integers(-8, 8, rows.size),
                         (rows, cols)), shape=(n, n))
    irr.sum_duplicates()
    mats = [matrices.poisson(17, 3), matrices.poisson(40, 2), matrices.banded(3000, 31, 256, 0),
            matrices.banded(2000, 13, 64, 0), irr]
    for A in mats:
        x = rng.standard_normal(A.shape[0]) * 10.0 ** rng.integers(-5, 5, A.shape[0])
        P = matrices.ParCSR.from_scipy(A)
        np.testing.assert_array_equal(P.dot(x), A.dot(x))


def test_banded_arrays_int64_rowptr():
    """banded_arrays builds the same rows as the scipy matrix with an int64
    row pointer (C5 at N = 50M has 3.15 G entries) and int32 columns."""
    from oracle import matrices
    ip, ix, dt = matrices.banded_arrays(5000, 31, 256, 3)
    A = matrices.banded(5000, 31, 256, 3)
    assert ip.dtype == np.int64 and ix.dtype == np.int32
    np.testing.assert_array_equal(ip, A.indptr)
    np.testing.assert_array_equal(ix, A.indices)
    np.testing.assert_array_equal(dt, A.data)
