/* Row-parallel CSR matvec for the oracle (TEST INFRASTRUCTURE ONLY).
 *
 * y[i] = sum over the row's stored entries, in stored order, of a[j] * x[c[j]],
 * starting from 0.0 -- statement for statement scipy's csr_matvec
 * (scipy/sparse/sparsetools/csr.h: `T sum = 0; for jj in row: sum +=
 * Ax[jj] * Xx[Aj[jj]]; Yx[i] = sum;` for A.dot(x)), which is what the
 * reference's v3/cpu solvers run (A.dot / A @ x). Each row is one thread's
 * sequential sum, so splitting the rows over OpenMP threads changes no bit;
 * built with -ffp-contract=off (no FMA), as scipy's baseline-x86-64 build
 * runs it. Used by the full-size parity tests, where scipy's single-threaded
 * matvec over 3.15 G entries (C5, N = 50M) would take minutes per solve.
 * Pinned against scipy bitwise in tests/test_oracle.py.
 */
#include <stdint.h>

void oracle_csrmv(int64_t n, const int64_t* indptr, const int32_t* indices,
                  const double* data, const double* x, double* y) {
#pragma omp parallel for schedule(static, 4096)
  for (int64_t i = 0; i < n; ++i) {
    double sum = 0.0;
    for (int64_t j = indptr[i]; j < indptr[i + 1]; ++j) sum += data[j] * x[indices[j]];
    y[i] = sum;
  }
}
