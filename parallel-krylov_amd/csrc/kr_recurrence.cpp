// Host scalar recurrences of the k-skip methods.
//
// These run on the host in fp64, statement for statement with the
// reference, so that given the same Gram coefficients they return the same
// bits as the numpy code:
//   * Python evaluates left to right: `2 * eta * zeta * beta` = ((2*eta)*zeta)*beta
//   * numpy float64 `x ** 2` is libm pow(x, 2.0), which is NOT always x*x
//     (it differs near half-ulp ties); LLVM folds a visible pow(x, 2.0) into
//     x*x, so pow is called through a volatile function pointer.
//   * no FMA contraction (built with -ffp-contract=off).
// Nothing here touches the GPU: the recurrence needs only the 6k+5 (6k+7)
// Gram scalars that one device->host copy per outer iteration delivers.
#include <cmath>

#include "kr_internal.h"

namespace kr {

namespace {
double (*volatile g_pow)(double, double) = &std::pow;
inline double sq(double v) { return g_pow(v, 2.0); }
}  // namespace

// v3/cpu/kskipmrr.py:62-64 (step 0) and :73-88 (k further steps); the GPU
// family repeats it at v3/gpu/kskipmrr.py:64-66, 74-90.
void kskipmrr_recurrence(int k, double* alpha, double* beta, double* delta, double* zeta_out,
                         double* eta_out) {
  auto coefficients = [&](double& zeta, double& eta) {
    const double d = alpha[2] * delta[0] - sq(beta[1]);
    zeta = alpha[1] * delta[0] / d;
    eta = (-alpha[1]) * beta[1] / d;
  };
  double zeta, eta;
  coefficients(zeta, eta);
  zeta_out[0] = zeta;
  eta_out[0] = eta;
  for (int j = 0; j < k; ++j) {
    const double zz = sq(zeta), ee = sq(eta);
    delta[0] = zz * alpha[2] + eta * zeta * beta[1];
    alpha[0] = alpha[0] - zeta * alpha[1];
    delta[1] = ee * delta[1] + 2.0 * eta * zeta * beta[2] + zz * alpha[3];
    beta[1] = eta * beta[1] + zeta * alpha[2] - delta[1];
    alpha[1] = -beta[1];
    const int lmax = 2 * (k - j);
    for (int l = 2; l <= lmax; ++l) {
      delta[l] = ee * delta[l] + 2.0 * eta * zeta * beta[l + 1] + zz * alpha[l + 2];
      const double tau = eta * beta[l] + zeta * alpha[l + 1];
      beta[l] = tau - delta[l];
      alpha[l] = alpha[l] - (tau + beta[l]);
    }
    coefficients(zeta, eta);
    zeta_out[j + 1] = zeta;
    eta_out[j + 1] = eta;
  }
}

// v3/cpu/kskipcg.py:51-52 (step 0) and :59-68 (k further steps); GPU family
// v3/gpu/kskipcg.py:55-56, 64-72.
void kskipcg_recurrence(int k, double* a, double* f, double* c, double* alpha_out,
                        double* beta_out) {
  auto coefficients = [&](double& alpha, double& beta) {
    alpha = a[0] / f[1];
    beta = sq(alpha) * f[2] / a[0] - 1.0;
  };
  double alpha, beta;
  coefficients(alpha, beta);
  alpha_out[0] = alpha;
  beta_out[0] = beta;
  for (int j = 0; j < k; ++j) {
    const int lmax = 2 * (k - j);
    for (int l = 0; l <= lmax; ++l) {
      a[l] = a[l] + alpha * (alpha * f[l + 2] - 2.0 * c[l + 1]);
      const double d = c[l] - alpha * f[l + 1];
      c[l] = a[l] + d * beta;
      f[l] = c[l] + beta * (d + beta * f[l]);
    }
    coefficients(alpha, beta);
    alpha_out[j + 1] = alpha;
    beta_out[j + 1] = beta;
  }
}

}  // namespace kr
