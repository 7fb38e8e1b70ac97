"""Matrix ingest (parallel_krylov_amd.io): row blocks read from .npz / .npy
files equal the in-memory matrix's rows (CPU), and a file-loaded system solves
like the golden case (GPU)."""
import contextlib
import io as _io

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_case, golden_matrix


@pytest.mark.parametrize("compressed", [False, True])
def test_npz_row_blocks(tmp_path, compressed):
    from parallel_krylov_amd import io
    A = golden_matrix(["banded", 3000, 13, 64, 0])
    path = str(tmp_path / "A.npz")
    sp.save_npz(path, A, compressed=compressed)
    assert io.matrix_shape(path) == A.shape
    mm = io._npz_member_mmap(path, "indices")
    assert (mm is not None) == (not compressed)
    for r0, r1 in [(0, 1), (0, 3000), (17, 1234), (2999, 3000), (1500, 1500)]:
        indptr, indices, data, ncols = io.read_csr_rows(path, r0, r1)
        ref = A[r0:r1]
        assert ncols == 3000
        np.testing.assert_array_equal(indptr, ref.indptr)
        np.testing.assert_array_equal(indices, ref.indices)
        np.testing.assert_array_equal(data, ref.data)


def test_npy_dense_rows(tmp_path):
    from parallel_krylov_amd import io
    A = golden_matrix(["poisson", 9, 2]).toarray()
    path = str(tmp_path / "A.npy")
    np.save(path, A)
    indptr, indices, data, ncols = io.read_csr_rows(path, 10, 40)
    ref = sp.csr_matrix(A[10:40])
    np.testing.assert_array_equal(indptr, ref.indptr)
    np.testing.assert_array_equal(indices, ref.indices)
    np.testing.assert_array_equal(data, ref.data)


def test_npy_rows_stay_dense(tmp_path):
    """A .npy row block is handed over dense (the reference keeps dense
    blocks dense, v3/gpu/mpi/common.py:123-125)."""
    from parallel_krylov_amd import io
    A = np.random.default_rng(0).standard_normal((50, 50))
    path = str(tmp_path / "A.npy")
    np.save(path, A)
    blk = io.read_rows(path, 10, 40)
    assert isinstance(blk, np.ndarray) and blk.dtype == np.float64
    np.testing.assert_array_equal(blk, A[10:40])
    npz = str(tmp_path / "S.npz")
    io.save_npz_uncompressed(npz, sp.csr_matrix(A))
    assert isinstance(io.read_rows(npz, 0, 5), tuple)


def test_rejects_non_csr(tmp_path):
    from parallel_krylov_amd import io
    path = str(tmp_path / "A.npz")
    sp.save_npz(path, sp.coo_matrix(np.eye(4)))
    with pytest.raises(ValueError):
        io.matrix_shape(path)


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [1, 3])
def test_file_loaded_system_solves_golden(tmp_path, shards):
    from parallel_krylov_amd import io
    g = golden_case("p3d16_kskipmrr_k4")
    A = golden_matrix(["poisson", 16, 3])
    path = str(tmp_path / "A.npz")
    io.save_npz_uncompressed(path, A)
    sysm = io.load_system(path, devices=[0] * shards)
    out = sysm.solve("kskipmrr", sysm.split(g["b"]), tol=1e-10, k=4)
    np.testing.assert_array_equal(out.info["nosl"], g["nosl"])
    rel = np.abs(out.info["residual"] - g["residual"]) / g["residual"]
    assert np.all(rel <= np.maximum(1e-12, 10 * g["envelope"]))
    sysm.close()


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [1, 2])
def test_npy_system_runs_gemv_and_matches_oracle(tmp_path, shards):
    """A .npy system loads as dense shards (GEMV kernel) and solves like the
    oracle on the same dense matrix."""
    from oracle import v3cpu
    from parallel_krylov_amd import io
    rng = np.random.default_rng(3)
    B = rng.uniform(0.5, 1.5, size=(400, 400)) / 400
    A = B @ B.T + np.diag(rng.uniform(1.0, 2.0, size=400))
    path = str(tmp_path / "A.npy")
    np.save(path, A)
    sysm = io.load_system(path, devices=[0] * shards)
    assert [sysm.shard_format(s) for s in range(shards)] == ["dense"] * shards
    b = rng.standard_normal(400)
    out = sysm.solve("kskipmrr", sysm.split(b), tol=1e-10, k=3)
    sysm.close()
    _, ref = v3cpu.kskipmrr(A, b, tol=1e-10, k=3)
    np.testing.assert_array_equal(out.info["nosl"], ref["nosl"])
    big = ref["residual"] > 1e-8
    assert np.all(np.abs(out.info["residual"][big] - ref["residual"][big])
                  <= 1e-6 * ref["residual"][big])
