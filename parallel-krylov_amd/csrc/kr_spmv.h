// SpMV device code (gfx950): epilogue tables, LDS staging, row walks, the
// product-then-sum kernel and the per-epilogue dispatch. Included by
// kr_kernels.hip (reductions, launchers) and by kr_spmv_inst.hip, which
// instantiates one epilogue per object file.
//
// Numerics contract: see kr_kernels.hip (compiled with -ffp-contract=off;
// rows summed in stored order, bitwise scipy csr_matvec).
#pragma once

#include <cstdlib>
#include <initializer_list>
#include <type_traits>

#include "kr_internal.h"

// Timing-only ablation macros (KR_ST_AB, KR_DIAW_AB, KR_AB_NO_PROLOGUE,
// KR_ST2T_TIMING; kr_pair.hip has KR_ST2B_AB) compile parts of kernels out
// and give WRONG results: a build that sets one must also define
// KR_ALLOW_WRONG_RESULTS, and only A/B libraries with their own file names
// do (tools/micro/pair_ab_build.sh, tools/lib_ab.sh with EXTRA=...).
#if ((defined(KR_ST_AB) && KR_ST_AB) || (defined(KR_DIAW_AB) && KR_DIAW_AB) || \
     defined(KR_AB_NO_PROLOGUE) || defined(KR_ST2T_TIMING)) &&                   \
    !defined(KR_ALLOW_WRONG_RESULTS)
#error "ablation build (wrong results): define KR_ALLOW_WRONG_RESULTS, A/B libraries only"
#endif

namespace kr {

template <int E>
void spmv_launch_epi(const SpmvArgs& a, int nblocks, hipStream_t s);

namespace {

typedef double dbl2v __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------
// Block-level deterministic reduction of NP per-thread accumulators into
// partials[p * grid + blockIdx.x].
// ---------------------------------------------------------------------------
template <int NP>
__device__ __forceinline__ void block_reduce_store(double (&acc)[NP > 0 ? NP : 1],
                                                   double* partials, int grid,
                                                   double* s_red /* NP*4 */,
                                                   int accumulate = 0,
                                                   int tid = threadIdx.x,
                                                   int64_t bid = blockIdx.x) {
  if constexpr (NP > 0) {
    const int lane = tid & 63;
    const int wave = tid >> 6;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      double v = acc[p];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
      if (lane == 0) s_red[p * 4 + wave] = v;
    }
    __syncthreads();
    if (tid < NP) {
      const double* r = s_red + tid * 4;
      double t = r[0];
      t = t + r[1];
      t = t + r[2];
      t = t + r[3];
      double* dst = partials + (int64_t)tid * grid + bid;
      *dst = accumulate ? *dst + t : t;  // accumulate: a later launch of the same SpMV
    }
  }
}

// ---------------------------------------------------------------------------
// SpMV epilogue product tables.
// ---------------------------------------------------------------------------
template <int EPI>
struct EpiTraits;
template <>
struct EpiTraits<EPI_NONE> {
  static constexpr int NP = 0, NV = 1;
  static constexpr bool kX = false, kX2 = false, kE = false;
};
template <>
struct EpiTraits<EPI_BMINUS> {
  static constexpr int NP = 1, NV = 1;
  static constexpr bool kX = false, kX2 = false, kE = false;
};
template <>
struct EpiTraits<EPI_XY> {
  static constexpr int NP = 3, NV = 1;
  static constexpr bool kX = true, kX2 = false, kE = false;
};
template <>
struct EpiTraits<EPI_HEAD_MRR> {
  static constexpr int NP = 5, NV = 1;
  static constexpr bool kX = true, kX2 = false, kE = true;
};
template <>
struct EpiTraits<EPI_HEAD_KCG> {
  static constexpr int NP = 6, NV = 1;
  static constexpr bool kX = true, kX2 = false, kE = true;
};
template <>
struct EpiTraits<EPI_MRR_LOOP> {
  static constexpr int NP = 3, NV = 1;
  static constexpr bool kX = true, kX2 = false, kE = true;
};
template <>
struct EpiTraits<EPI_DUAL_NONE> {
  static constexpr int NP = 0, NV = 2;
  static constexpr bool kX = false, kX2 = false, kE = false;
};
template <>
struct EpiTraits<EPI_DUAL_MRR> {
  static constexpr int NP = 7, NV = 2;
  static constexpr bool kX = true, kX2 = true, kE = false;
};
template <>
struct EpiTraits<EPI_DUAL_KCG> {
  static constexpr int NP = 7, NV = 2;
  static constexpr bool kX = true, kX2 = true, kE = false;
};
// Fused k-skip steps: no products, one input vector.
struct EpiStepTraits {
  static constexpr int NP = 0, NV = 1;
  static constexpr bool kX = false, kX2 = false, kE = false;
};
template <>
struct EpiTraits<EPI_STEP_MRR_NOX> : EpiStepTraits {};
template <>
struct EpiTraits<EPI_STEP_MRR_X2> : EpiStepTraits {};
template <>
struct EpiTraits<EPI_STEP_MRR_X> : EpiStepTraits {};
template <>
struct EpiTraits<EPI_STEP_KCG> : EpiStepTraits {};
template <>
struct EpiTraits<EPI_STEP_MRR_FIRST2> : EpiStepTraits {};
template <>
struct EpiTraits<EPI_XY_VP> {  // x = p_old, x2 = r at the row (p formed from them)
  static constexpr int NP = 3, NV = 1;
  static constexpr bool kX = true, kX2 = true, kE = false;
};
template <>
struct EpiTraits<EPI_MRR_V> {  // products of EPI_MRR_LOOP over the new vectors
  static constexpr int NP = 3, NV = 1;
  static constexpr bool kX = false, kX2 = false, kE = false;
};
template <int EPI>
constexpr bool is_step() {
  return EPI == EPI_STEP_MRR_NOX || EPI == EPI_STEP_MRR_X2 || EPI == EPI_STEP_MRR_X ||
         EPI == EPI_STEP_KCG || EPI == EPI_STEP_MRR_FIRST2 || EPI == EPI_MRR_V;
}
// The SpMV input is virtual: r1 = r0 - (c0*y0 + c1*Ar1) at every column.
template <int EPI>
constexpr bool is_virtual() {
  return EPI == EPI_STEP_MRR_FIRST2 || EPI == EPI_XY_VP || EPI == EPI_MRR_V;
}
// Epilogues whose own-row operands include r, y, Ar of the virtual input
// (x1, x2, x3 at the row) and the x source (us).
template <int EPI>
constexpr bool is_vstep() {
  return EPI == EPI_STEP_MRR_FIRST2 || EPI == EPI_MRR_V;
}
// r1 at one column, rounded exactly like ew_kernel<EW_MRR_NOX>'s step 0:
// y1 = fl(fl(c0*y0) + fl(c1*ar1)), r1 = fl(r0 - y1).
__device__ __forceinline__ double virtual_r1(double c0, double c1, double r0, double y0,
                                             double ar1) {
  const double t1 = c0 * y0;
  const double t2 = c1 * ar1;
  const double y = t1 + t2;
  return r0 - y;
}
// Sum of the `cnt` partials of one slot in the fixed order of the finalize
// kernels: lane t adds partials t, t + 256, ... in that order, then the
// shuffle tree, then waves 0..3. The lane's partials are loaded 8 at a time
// before they are added (in order), so a prologue pays about one load
// latency instead of cnt / 256. Called by the whole workgroup; every thread
// gets the result. s_red: 4 doubles.
__device__ __forceinline__ double slot_sum(const double* __restrict__ part, int cnt,
                                           double* s_red) {
  constexpr int U = 8;
  double t = 0.0;
  for (int i0 = threadIdx.x; i0 < cnt; i0 += U * kBlock) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * kBlock;
      v[u] = part[i < cnt ? i : i0];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * kBlock < cnt) t += v[u];
  }
  for (int off = 32; off > 0; off >>= 1) t += __shfl_down(t, off, 64);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = t;
  __syncthreads();
  double r = s_red[0];
  r = r + s_red[1];
  r = r + s_red[2];
  r = r + s_red[3];
  __syncthreads();  // s_red may be reused by the caller
  return r;
}

// CG's p = r + beta * p_old at one column, rounded as ew_kernel<EW_CG_P>.
__device__ __forceinline__ double virtual_p(double beta, double p_old, double r) {
  const double bp = beta * p_old;
  return r + bp;
}
// The virtual SpMV input of epilogue EPI at one column from the physical
// inputs x1, x2, x3 there (x3 unused by EPI_XY_VP).
template <int EPI>
__device__ __forceinline__ double virt_in(const SpmvArgs& a, double v1, double v2, double v3) {
  if constexpr (EPI == EPI_XY_VP)
    return virtual_p(a.c0, v1, v2);
  else
    return virtual_r1(a.c0, a.c1, v1, v2, v3);
}

// EPI_XY_VP's scalar step, run by every workgroup at kernel entry (after the
// stop test): beta = gnew / gamma from the EW_CG partials (slot 0, summed in
// the finalize order like ew_prologue / scalar_kernel), the convergence test
// on gnew; workgroup 0 writes the state. Sets a.c0 = beta; false when the
// test fired (the launch then does nothing, as EW_CG_P skips itself).
__device__ __forceinline__ bool spmv_prologue_beta(SpmvArgs& a) {
  __shared__ double s_r[4];
  const double gnew = 0.0 + slot_sum(a.pro_part, a.pro_cnt[0], s_r);
  double* st = a.st;
  a.c0 = gnew / st[gamma_slot(a.pro_par)];
  const bool conv = a.pro_check && gnew >= 0.0 && gnew < a.pro_thr;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st[ST_HIST + a.pro_h] = gnew;
    st[gamma_slot(a.pro_par ^ 1)] = gnew;
    if (conv) {  // the test at the top of the next iteration
      st[ST_STOP_AT] = (double)(a.pro_it + 1);
      st[ST_STOP] = 1.0;
    }
  }
  return !conv;
}
// Kernel entry of every SpMV kernel that serves virtual inputs.
template <int EPI>
__device__ __forceinline__ bool spmv_entry(SpmvArgs& a) {
  if (a.stop && *a.stop != 0.0) return false;  // converged (device-resident scalars)
  if constexpr (EPI == EPI_XY_VP) {
#ifdef KR_AB_NO_PROLOGUE  // timing-only ablation builds (wrong beta)
    a.c0 = 0.5;
#else
    if (a.pro && !spmv_prologue_beta(a)) return false;
#endif
  }
  if constexpr (EPI == EPI_MRR_V) {
    // SC_MRR_ZETA (v3/gpu/mrr.py:47-49) from the EW_MRR_S partials, summed in
    // the finalize order like ew_prologue: zeta = <r,s>/<s,s>, eta = -zeta*gamma
    if (a.pro) {
      __shared__ double s_r[4];
      const double rs = 0.0 + slot_sum(a.pro_part + (int64_t)3 * a.pro_stride, a.pro_cnt[3], s_r);
      const double ss = 0.0 + slot_sum(a.pro_part + (int64_t)4 * a.pro_stride, a.pro_cnt[4], s_r);
      const double zeta = rs / ss;
      a.c0 = (-zeta) * a.st[ST_GAMMA];
      a.c1 = zeta;
    }
  }
  return true;
}

// Products of one row. x/x2: inputs at the row, y/y2: results, e: extra.
template <int EPI>
__device__ __forceinline__ void epi_products(double x, double x2, double y, double y2,
                                             double e,
                                             double (&acc)[EpiTraits<EPI>::NP > 0
                                                               ? EpiTraits<EPI>::NP
                                                               : 1]) {
  if constexpr (EPI == EPI_BMINUS) {
    acc[0] += y * y;
  } else if constexpr (EPI == EPI_XY) {
    acc[0] += x * x;
    acc[1] += x * y;
    acc[2] += y * y;
  } else if constexpr (EPI == EPI_HEAD_MRR) {  // x=Ar0 y=Ar1 e=Ay0
    acc[0] += x * x;                           // alpha[0]
    acc[1] += x * y;                           // alpha[1]
    acc[2] += y * y;                           // alpha[2]
    acc[3] += e * y;                           // beta[1]
    acc[4] += e * e;                           // delta[0]
  } else if constexpr (EPI == EPI_HEAD_KCG) {  // x=Ap0 y=Ap1 e=Ar0
    acc[0] += e * e;                           // a[0]
    acc[1] += x * x;                           // f[0]
    acc[2] += x * y;                           // f[1]
    acc[3] += y * y;                           // f[2]
    acc[4] += e * x;                           // c[0]
    acc[5] += e * y;                           // c[1]
  } else if constexpr (EPI == EPI_MRR_LOOP) {  // x=r y=Ar e=y
    acc[0] += x * x;                           // <r,r>
    acc[1] += e * e;                           // mu
    acc[2] += e * y;                           // nu
  } else if constexpr (EPI == EPI_DUAL_MRR) {  // x=Ar[m+1] x2=Ay[m] y=Ar[m+2] y2=Ay[m+1]
    acc[0] += x * y;                           // alpha[2m+3]
    acc[1] += y * y;                           // alpha[2m+4]
    acc[2] += y2 * y2;                         // delta[2m+2]
    acc[3] += x2 * y2;                         // delta[2m+1]
    acc[4] += y2 * y;                          // beta[2m+3]
    acc[5] += x2 * x;                          // beta[2m+1]
    acc[6] += y2 * x;                          // beta[2m+2]
  } else if constexpr (EPI == EPI_DUAL_KCG) {  // x=Ar[j-1] x2=Ap[j] y=Ar[j] y2=Ap[j+1]
    acc[0] += x * y;                           // a[2j-1]
    acc[1] += y * y;                           // a[2j]
    acc[2] += x2 * y2;                         // f[2j+1]
    acc[3] += y2 * y2;                         // f[2j+2]
    acc[4] += x * x2;                          // c[2j-1]
    acc[5] += y * x2;                          // c[2j]
    acc[6] += y * y2;                          // c[2j+1]
  }
}

// Row epilogue shared by the SpMV kernels: y = A x of one row (sum1, sum2)
// is stored with its products, or -- EPI_STEP_* -- consumed by the next
// k-skip vector step, statement for statement as the reference writes it
// (v3/gpu/kskipmrr.py:88-95, v3/gpu/kskipcg.py:71-76; numpy rounding, every
// product rounded, no FMA): the same operations as ew_kernel<EW_MRR*> /
// <EW_KCG> followed by the SpMV, without storing A x or re-reading x.
// The row's own-row operands (EpiIn) are loaded when the row block starts,
// so their latency hides under the row walk (epi_load / epi_row_in).
struct EpiIn {
  double u1 = 0, u2 = 0, us = 0, e = 0, x = 0, x2 = 0;
};
// NOX: operands the caller fills itself (the DIA walk, from its window):
// bit 0 EpiIn::x, bit 1 EpiIn::x2, bit 2 the virtual step's e (x3 at the row)
template <int EPI, int NOX = 0>
__device__ __forceinline__ EpiIn epi_load(const SpmvArgs& a, int64_t row) {
  using T = EpiTraits<EPI>;
  EpiIn in;
  if constexpr (!(NOX & 1) && (is_step<EPI>() || T::kX)) in.x = a.x1[a.xoff + row];
  if constexpr (!(NOX & 2) && T::kX2) in.x2 = a.x2[a.xoff + row];
  if constexpr (is_step<EPI>()) {
    in.u1 = a.u1[row];
    in.u2 = a.u2[row];
    if constexpr (EPI == EPI_STEP_MRR_X2 || EPI == EPI_STEP_MRR_X || is_vstep<EPI>())
      in.us = a.us[row];
    if constexpr (is_vstep<EPI>()) {
      if constexpr (!(NOX & 2)) in.x2 = a.x2[a.xoff + row];  // y0
      if constexpr (!(NOX & 4)) in.e = a.x3[a.xoff + row];   // Ar1
    }
  } else if constexpr (EPI == EPI_BMINUS) {
    in.e = a.b[row];
  } else if constexpr (T::kE) {
    in.e = a.e[row];
  }
  return in;
}

// The values one row's epilogue stores (statement for statement as above),
// separated from the stores so the 2-rows-per-lane stencil kernel can store
// row pairs as 16-byte accesses.
struct EpiVals {
  double y1 = 0, y2 = 0, u1 = 0, u2 = 0, ud = 0;
};
template <int EPI>
constexpr bool epi_writes_ud() {
  return EPI == EPI_STEP_MRR_X2 || EPI == EPI_STEP_MRR_X || is_vstep<EPI>();
}

template <int EPI>
__device__ __forceinline__ EpiVals epi_values(const SpmvArgs& a, double sum1, double sum2,
                                              const EpiIn& in,
                                              double (&acc)[EpiTraits<EPI>::NP > 0
                                                                ? EpiTraits<EPI>::NP
                                                                : 1]) {
  using T = EpiTraits<EPI>;
  EpiVals o;
  if constexpr (EPI == EPI_STEP_MRR_FIRST2) {
    // step 0 at the own row (c0 = eta0, c1 = zeta0; x = r0, x2 = y0, e = Ar1,
    // u2 = z0), then step 1 (c2 = eta1, c3 = zeta1) with sum1 = (A r1)[row]
    const double t1 = a.c0 * in.x2;
    const double t2 = a.c1 * in.e;
    const double y1 = t1 + t2;
    const double t3 = a.c0 * in.u2;
    const double t4 = a.c1 * in.x;
    const double z1 = t3 - t4;
    const double r1 = in.x - y1;
    const double s1 = a.c2 * y1;
    const double s2 = a.c3 * sum1;
    const double y2 = s1 + s2;
    const double s3 = a.c2 * z1;
    const double s4 = a.c3 * r1;
    const double z2 = s3 - s4;
    const double xs = a.xpend ? in.us - in.u2 : in.us;  // the previous outer's last x -= z
    const double xm = xs - z1;  // x -= z of step 0, deferred
    o.ud = xm - z2;
    o.u1 = y2;
    o.u2 = z2;
    o.y1 = r1 - y2;  // Ar0 of step 2
  } else if constexpr (EPI == EPI_MRR_V) {
    // the previous iteration's EW_MRR step at the own row (c0 = eta,
    // c1 = zeta; x = r, x2 = y, e = Ar, u2 = z, us = x), statement for
    // statement as ew_kernel<EW_MRR>; sum1 = (A r_new)[row]
    const double t1 = a.c0 * in.x2;
    const double t2 = a.c1 * in.e;
    const double y = t1 + t2;
    const double t3 = a.c0 * in.u2;
    const double t4 = a.c1 * in.x;
    const double z = t3 - t4;
    const double r = in.x - y;
    o.ud = in.us - z;
    o.u1 = y;
    o.u2 = z;
    o.y2 = r;
    o.y1 = sum1;
    epi_products<EPI_MRR_LOOP>(r, 0.0, sum1, 0.0, y, acc);  // <r,r> mu nu
  } else if constexpr (EPI == EPI_XY_VP) {
    const double pv = virtual_p(a.c0, in.x, in.x2);  // p at the own row
    o.u1 = pv;
    o.y1 = sum1;
    epi_products<EPI_XY>(pv, 0.0, sum1, 0.0, 0.0, acc);
  } else if constexpr (is_step<EPI>()) {
    const double xv = in.x;
    if constexpr (EPI == EPI_STEP_KCG) {  // x = Ap0, sum1 = Ap1; u1 = x, u2 = Ar0
      const double a0 = a.c0 * xv;
      const double a1 = a.c0 * sum1;
      o.u1 = in.u1 + a0;
      const double r = in.u2 - a1;
      o.u2 = r;
      const double bp = a.c1 * xv;
      o.y1 = r + bp;  // Ap0 of the next step
    } else {  // x = Ar0, sum1 = Ar1; u1 = Ay0, u2 = z; c0 = eta, c1 = zeta
      const double t1 = a.c0 * in.u1;
      const double t2 = a.c1 * sum1;
      const double y = t1 + t2;
      const double t3 = a.c0 * in.u2;
      const double t4 = a.c1 * xv;
      const double z = t3 - t4;
      if constexpr (EPI == EPI_STEP_MRR_X2) {
        const double xm = in.us - in.u2;  // the deferred x -= z of the previous step
        o.ud = xm - z;
      } else if constexpr (EPI == EPI_STEP_MRR_X) {
        o.ud = in.us - z;
      }
      o.u1 = y;
      o.u2 = z;
      o.y1 = xv - y;  // Ar0 of the next step
    }
  } else {
    double y1 = sum1;
    if constexpr (EPI == EPI_BMINUS) y1 = in.e - sum1;
    o.y1 = y1;
    if constexpr (T::NV == 2) o.y2 = sum2;
    if constexpr (T::NP > 0) epi_products<EPI>(in.x, in.x2, y1, sum2, in.e, acc);
  }
  return o;
}

// POM: how a two-vector SpMV honours SpmvArgs::products_only (outputs nobody
// reads: no y stores). -1 tests it at run time; 0 / 1 are kernels the host
// launches only for storing / products-only SpMVs (no store under a run-time
// branch: such a branch shifts the compiler's vmcnt waits, 2.6 % on the
// plain-CSR dual).
template <int EPI, int POM>
__device__ __forceinline__ bool epi_po_skip(const SpmvArgs& a) {
  if constexpr (EpiTraits<EPI>::NV != 2 || is_step<EPI>() || POM == 0)
    return false;
  else if constexpr (POM == 1)
    return true;
  else
    return a.products_only != 0;
}

template <int EPI, int POM = -1>
__device__ __forceinline__ void epi_store_row(const SpmvArgs& a, int64_t row, const EpiVals& o) {
  if constexpr (is_step<EPI>()) {
    if constexpr (epi_writes_ud<EPI>()) a.ud[row] = o.ud;
    a.u1[row] = o.u1;
    a.u2[row] = o.u2;
    a.y1[row] = o.y1;
    if constexpr (EPI == EPI_MRR_V) a.y2[row] = o.y2;
  } else {
    if (epi_po_skip<EPI, POM>(a)) return;
    a.y1[row] = o.y1;
    if constexpr (EpiTraits<EPI>::NV == 2) a.y2[row] = o.y2;
    if constexpr (EPI == EPI_XY_VP) a.u1[row] = o.u1;
  }
}

// One row's epilogue stores with store kind SK: 0 plain, 1 non-temporal
// (the row walks' default with a non-temporal matrix stream: a plain-CSR dual
// SpMV at 512^3 spends 0.72 of its 3.3 ms on the 2.15 GB of y1 / y2 stores,
// and non-temporal ones cut 0.15 ms of that; tools/micro/csr_micro), 2
// agent-scope relaxed atomic stores (sc1: the line leaves the XCD's L2;
// measured no faster than plain).
template <int SK>
__device__ __forceinline__ void st1(double* p, double v) {
  if constexpr (SK == 1)
    __builtin_nontemporal_store(v, p);
  else if constexpr (SK == 2)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}
template <int EPI, int SK, int POM = -1>
__device__ __forceinline__ void epi_store_row_k(const SpmvArgs& a, int64_t row, const EpiVals& o) {
  if constexpr (is_step<EPI>()) {
    if constexpr (epi_writes_ud<EPI>()) st1<SK>(a.ud + row, o.ud);
    st1<SK>(a.u1 + row, o.u1);
    st1<SK>(a.u2 + row, o.u2);
    st1<SK>(a.y1 + row, o.y1);
    if constexpr (EPI == EPI_MRR_V) st1<SK>(a.y2 + row, o.y2);
  } else {
    if (epi_po_skip<EPI, POM>(a)) return;
    st1<SK>(a.y1 + row, o.y1);
    if constexpr (EpiTraits<EPI>::NV == 2) st1<SK>(a.y2 + row, o.y2);
    if constexpr (EPI == EPI_XY_VP) st1<SK>(a.u1 + row, o.u1);
  }
}

// Rows row, row + 1 (row even: own-row vectors are 16-byte aligned there);
// ok = false sends the pair to SpmvArgs::scratch instead (lanes past the
// last row store unconditionally, see kr_stencil.h).
template <int EPI, bool NT = false>
__device__ __forceinline__ void epi_store_pair(const SpmvArgs& a, int64_t row, const EpiVals& lo,
                                               const EpiVals& hi, bool ok = true) {
  auto st2 = [&](double* p, double u, double v) {
    dbl2v* d = reinterpret_cast<dbl2v*>(ok ? p + row : a.scratch);
    if constexpr (NT)
      __builtin_nontemporal_store(dbl2v{u, v}, d);
    else
      *d = dbl2v{u, v};
  };
  if constexpr (is_step<EPI>()) {
    if constexpr (epi_writes_ud<EPI>()) st2(a.ud, lo.ud, hi.ud);
    st2(a.u1, lo.u1, hi.u1);
    st2(a.u2, lo.u2, hi.u2);
    st2(a.y1, lo.y1, hi.y1);
    if constexpr (EPI == EPI_MRR_V) st2(a.y2, lo.y2, hi.y2);
  } else {
    st2(a.y1, lo.y1, hi.y1);
    if constexpr (EpiTraits<EPI>::NV == 2) st2(a.y2, lo.y2, hi.y2);
    if constexpr (EPI == EPI_XY_VP) st2(a.u1, lo.u1, hi.u1);
  }
}

template <int EPI, int POM = -1>
__device__ __forceinline__ void epi_row_in(const SpmvArgs& a, int64_t row, double sum1,
                                           double sum2, const double* __restrict__ x1,
                                           const double* __restrict__ x2, const EpiIn& in,
                                           double (&acc)[EpiTraits<EPI>::NP > 0
                                                             ? EpiTraits<EPI>::NP
                                                             : 1]) {
  epi_store_row<EPI, POM>(a, row, epi_values<EPI>(a, sum1, sum2, in, acc));
}

template <int EPI>
__device__ __forceinline__ void epi_row(const SpmvArgs& a, int64_t row, double sum1,
                                        double sum2, const double* __restrict__ x1,
                                        const double* __restrict__ x2,
                                        double (&acc)[EpiTraits<EPI>::NP > 0
                                                          ? EpiTraits<EPI>::NP
                                                          : 1]) {
  epi_row_in<EPI>(a, row, sum1, sum2, x1, x2, epi_load<EPI>(a, row), acc);
}

// ---------------------------------------------------------------------------
// CSR SpMV, one lane per row, matrix entries staged through LDS.
//   Row block = kBlock consecutive rows. Its nnz range is staged into LDS in
//   windows of kWindow entries: every lane first issues all of its 16-byte
//   loads (4 entries per slot, kSlots slots: vals as 2 x 16 B, cols as 16 B),
//   then writes them to LDS, so a wave has 3*kSlots loads in flight instead of
//   a load/wait/store chain. Each lane then walks its own row inside the
//   window in stored order, issuing up to kGather x-gathers before it adds
//   them -- in order -- to its running sum (bitwise scipy csr_matvec).
//   Grid-stride over row blocks; reductions accumulate per lane across row
//   blocks and are reduced once per workgroup at the end.
// ---------------------------------------------------------------------------
typedef int int4v __attribute__((ext_vector_type(4)));
constexpr int kSlots = kWindow / (4 * kBlock);
// x gathers in flight per lane: 7 = one batch for 7-point rows (8 issued a
// redundant 8th load per row; measured +1-2 %).
constexpr int kGather = 7;
static_assert(kSlots * 4 * kBlock == kWindow, "window must be a multiple of 4*kBlock");

// Registers holding one staged window. Values move as one 16-byte double2 per
// lane per slot and columns as one 16-byte int4, so consecutive lanes touch
// consecutive 16-byte LDS slots (bank-conflict-free ds_write_b128) and every
// wave-instruction reads 1 KiB of contiguous HBM.
constexpr int kVSlots = kWindow / (2 * kBlock);
constexpr int kCSlots = kWindow / (4 * kBlock);
struct Stage {
  dbl2v v[kVSlots];
  int4v c[kCSlots];
};

template <bool VEC, bool NT = false, bool COLS = true>
__device__ __forceinline__ void stage_load(Stage& st, const double* __restrict__ val,
                                           const int32_t* __restrict__ col, int64_t ws,
                                           int64_t bs, int64_t be, int tid) {
#pragma unroll
  for (int q = 0; q < kVSlots; ++q) {
    const int64_t g0 = ws + (int64_t)(tid + q * kBlock) * 2;
    if (VEC && g0 >= bs && g0 + 2 <= be) {
      if constexpr (NT)
        st.v[q] = __builtin_nontemporal_load(reinterpret_cast<const dbl2v*>(val + g0));
      else
        st.v[q] = *reinterpret_cast<const dbl2v*>(val + g0);
    } else {
      const bool ok0 = g0 >= bs && g0 < be, ok1 = g0 + 1 >= bs && g0 + 1 < be;
      st.v[q] = dbl2v{ok0 ? val[g0] : 0.0, ok1 ? val[g0 + 1] : 0.0};
    }
  }
  if constexpr (!COLS) return;
#pragma unroll
  for (int q = 0; q < kCSlots; ++q) {
    const int64_t g0 = ws + (int64_t)(tid + q * kBlock) * 4;
    if (VEC && g0 >= bs && g0 + 4 <= be) {
      if constexpr (NT)
        st.c[q] = __builtin_nontemporal_load(reinterpret_cast<const int4v*>(col + g0));
      else
        st.c[q] = *reinterpret_cast<const int4v*>(col + g0);
    } else {
      int tc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t g = g0 + u;
        tc[u] = (g >= bs && g < be) ? col[g] : 0;
      }
      st.c[q] = int4v{tc[0], tc[1], tc[2], tc[3]};
    }
  }
}

template <bool COLS = true>
__device__ __forceinline__ void stage_commit(const Stage& st, double* s_val, int32_t* s_col,
                                             int tid) {
#pragma unroll
  for (int q = 0; q < kVSlots; ++q) reinterpret_cast<dbl2v*>(s_val)[tid + q * kBlock] = st.v[q];
  if constexpr (COLS) {
#pragma unroll
    for (int q = 0; q < kCSlots; ++q)
      reinterpret_cast<int4v*>(s_col)[tid + q * kBlock] = st.c[q];
  }
}

// Offset-mask rows (SpmvArgs::mask): the row's columns are xrow + M[b] for
// the set bits b of its mask, in increasing order (M ascending, columns
// strictly increasing in the row), so the k-th stored entry uses the k-th set
// bit. The lane's remaining mask carries across windows.
template <int MW>
struct MaskType {
  using type = uint64_t;
};
template <>
struct MaskType<8> {
  using type = uint8_t;
};
template <>
struct MaskType<16> {
  using type = uint16_t;
};
template <>
struct MaskType<32> {
  using type = uint32_t;
};

// LDS view of a window's values for the dictionary path (spmv_kernel2 VI):
// the window holds 1-byte codes, decoded through the LDS table on read.
struct CodeView {
  const uint8_t* c;
  const double* t;
  __device__ __forceinline__ double operator[](int j) const { return t[c[j]]; }
};

template <int NV, int GATHER, typename W, typename VS>
__device__ __forceinline__ void row_window_mask(VS s_val, const int32_t* s_M,
                                                const double* __restrict__ x1,
                                                const double* __restrict__ x2, int64_t xrow,
                                                int js, int je, W& mrem, double& sum1,
                                                double& sum2) {
  for (int j = js; j < je; j += GATHER) {
    double v[GATHER], p1[GATHER], p2[GATHER];
#pragma unroll
    for (int u = 0; u < GATHER; ++u) {
      const bool ok = j + u < je;
      v[u] = s_val[ok ? j + u : js];
      int64_t c = xrow;
      if (ok) {
        c += s_M[sizeof(W) == 8 ? __builtin_ctzll((unsigned long long)mrem)
                                : __builtin_ctz((unsigned)mrem)];
        mrem &= mrem - 1;
      }
      p1[u] = x1[c];
      if constexpr (NV == 2) p2[u] = x2[c];
    }
#pragma unroll
    for (int u = 0; u < GATHER; ++u) {
      if (j + u < je) {
        sum1 = sum1 + v[u] * p1[u];
        if constexpr (NV == 2) sum2 = sum2 + v[u] * p2[u];
      }
    }
  }
}

// One lane's entries [js, je) of the staged window, in stored order.
template <int NV, int GATHER = kGather, typename VS = const double*>
__device__ __forceinline__ void row_window(VS s_val, const int32_t* s_col,
                                           const double* __restrict__ x1,
                                           const double* __restrict__ x2, int js, int je,
                                           double& sum1, double& sum2) {
  for (int j = js; j < je; j += GATHER) {
    double v[GATHER], p1[GATHER], p2[GATHER];
#pragma unroll
    for (int u = 0; u < GATHER; ++u) {
      const int jj = (j + u < je) ? j + u : js;
      v[u] = s_val[jj];
      const int c = s_col[jj];
      p1[u] = x1[c];
      if constexpr (NV == 2) p2[u] = x2[c];
    }
#pragma unroll
    for (int u = 0; u < GATHER; ++u) {
      if (j + u < je) {
        sum1 = sum1 + v[u] * p1[u];
        if constexpr (NV == 2) sum2 = sum2 + v[u] * p2[u];
      }
    }
  }
}

// Further gather batches of a row whose input is virtual (is_virtual):
// x(c) = r1 at column c from r0 = x1, y0 = x2, Ar1 = x3 (SpmvArgs), summed in
// stored order. Columns from the LDS column window or the offset masks.
template <int EPI, int GATHER, typename W, typename VS>
__device__ __forceinline__ void row_window_virtual(VS s_val, const int32_t* s_col,
                                                   const int32_t* s_M, int64_t xrow,
                                                   const SpmvArgs& a, int js, int je, W& mrem,
                                                   double& sum1) {
  for (int j = js; j < je; j += GATHER) {
    double v[GATHER], p1[GATHER], p2[GATHER], p3[GATHER];
#pragma unroll
    for (int u = 0; u < GATHER; ++u) {
      const bool ok = j + u < je;
      const int jj = ok ? j + u : js;
      v[u] = s_val[jj];
      int64_t c;
      if (s_col) {
        c = s_col[jj];
      } else {
        c = xrow;
        if (ok) {
          c += s_M[sizeof(W) == 8 ? __builtin_ctzll((unsigned long long)mrem)
                                  : __builtin_ctz((unsigned)mrem)];
          mrem &= mrem - 1;
        }
      }
      p1[u] = a.x1[c];
      p2[u] = a.x2[c];
      p3[u] = a.x3[c];
    }
#pragma unroll
    for (int u = 0; u < GATHER; ++u)
      if (j + u < je) sum1 = sum1 + v[u] * virt_in<EPI>(a, p1[u], p2[u], p3[u]);
  }
}

// Software pipeline over a stream of LDS windows. A workgroup walks its row
// blocks (256 rows each); a row block's entries are one or more 2048-entry
// windows. While one window is multiplied out of LDS, the NEXT window is
// already in flight in registers: the next window of the same row block, or
// the first window of the next row block (whose nnz range was requested as
// scalar loads one row block earlier). So a window waits on one memory round
// trip, for short-row (Poisson: one window per row block) and long-row
// (banded 27-63 nnz/row: 4-8 windows per row block) matrices alike.
// Row-block schedule: a workgroup visits rb(j) for j = j0, j0 + jstep, ...
// < jcount. XCD-aware: workgroups b and b+8 share an XCD (and its L2) under
// the observed round-robin dispatch, so the workgroups with equal b % 8 work
// on rows close together and the x entries that neighbouring row blocks
// gather stay in one L2. Contiguous mode: each XCD sweeps one eighth of the
// rows (neighbours +-1, +-n reused). Slab mode (S = the matrix's column reach
// in row blocks): the rows are cut into "planes" of S row blocks and XCD q
// owns the q-th eighth of every plane, visited plane after plane, so the x
// rows one plane away (+-n^2 of a 3-D stencil) are still in its L2 when the
// next plane reads them. With a sub-slab width (slab_sub), XCD q's eighth is
// cut further into sub-slabs that are swept plane after plane one at a time,
// which shortens the reuse distance to what its 4 MB L2 holds. Placement only
// changes speed: every row block is visited exactly once.
struct RowSched {
  int64_t j0, jstep, jcount, base = 0, off = 0, w = 0, S = 0, sub = 0, full = 0, rem = 0;
  int64_t gap_at = 0, gap = 0;  // SpmvArgs::rb_gap_at / rb_gap (virtual -> physical)
  int nc = 0;
  // row blocks of sub-slab c (width wc, all planes; the last plane is partial)
  __device__ int64_t chunk_count(int c, int64_t wc) const {
    return full * wc + min(wc, max((int64_t)0, rem - off - c * sub));
  }
  __device__ void init(int64_t nrb, int64_t slab, int64_t slab_sub, bool xcd) {
    if (xcd && (gridDim.x & 7) == 0) {
      const int64_t q = blockIdx.x & 7;
      j0 = blockIdx.x >> 3;
      jstep = gridDim.x >> 3;
      if (slab >= 8) {
        S = slab;
        off = S * q / 8;
        w = S * (q + 1) / 8 - off;
        const int64_t planes = (nrb + S - 1) / S;
        full = planes - 1;
        rem = nrb - full * S;
        sub = slab_sub > 0 ? min(slab_sub, w) : w;
        nc = (int)((w + sub - 1) / sub);
        jcount = 0;
        for (int c = 0; c < nc; ++c) jcount += chunk_count(c, min(sub, w - c * sub));
      } else {
        const int64_t chunk = (nrb + 7) / 8;
        base = q * chunk;
        jcount = max((int64_t)0, min(nrb, base + chunk) - base);
      }
    } else {
      j0 = blockIdx.x;
      jstep = gridDim.x;
      jcount = nrb;
    }
  }
  __device__ int64_t rb_virtual(int64_t v) const {
    if (!w) return base + v;
    // sub-slab after sub-slab; inside one, plane after plane
    for (int c = 0; c < nc; ++c) {
      const int64_t wc = min(sub, w - c * sub);
      const int64_t cnt = chunk_count(c, wc);
      if (v < cnt) return (v / wc) * S + off + c * sub + v % wc;
      v -= cnt;
    }
    return -1;  // unreachable: v < jcount
  }
  __device__ int64_t rb(int64_t v) const {
    const int64_t r = rb_virtual(v);
    return r < gap_at ? r : r + gap;
  }
};

template <typename RP, int EPI, bool VEC, int GATHER = kGather, bool XCD = true, bool NT = false,
          int MW = 0>
__global__ __launch_bounds__(kBlock) void spmv_kernel(SpmvArgs a) {
  if (a.stop && *a.stop != 0.0) return;  // converged (device-resident scalars)
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  constexpr bool COLS = MW == 0;  // else: offset masks, no column stream
  using MT = typename MaskType<MW>::type;
  using W = typename std::conditional<(MW > 32), uint64_t, uint32_t>::type;
  __shared__ __attribute__((aligned(16))) double s_val[kWindow];
  __shared__ __attribute__((aligned(16))) int32_t s_col[COLS ? kWindow : 4];
  __shared__ int32_t s_M[COLS ? 1 : 64];
  const MT* __restrict__ mask = static_cast<const MT*>(a.mask);
  if constexpr (!COLS) {
    if ((int)threadIdx.x < a.nm) s_M[threadIdx.x] = a.moff[threadIdx.x];  // seen after 1st barrier
  }
  __shared__ int32_t s_rp[kBlock + 1];  // row pointers relative to the block start
  __shared__ double s_red[(NP > 0 ? NP : 1) * 4];

  const RP* __restrict__ rowptr = static_cast<const RP*>(a.rowptr);
  const double* __restrict__ val = a.val;
  const int32_t* __restrict__ col = a.col;
  const double* __restrict__ x1 = a.x1;
  const double* __restrict__ x2 = a.x2;
  const int tid = threadIdx.x;

  double acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) acc[p] = 0.0;

  const int64_t nrb = (a.n + kBlock - 1) / kBlock - a.rb_gap;
  RowSched sched;
  sched.init(nrb, a.slab, a.slab_sub, XCD);
  sched.gap_at = a.rb_gap_at;
  sched.gap = a.rb_gap;
  int64_t j = sched.j0;
  const int64_t jstep = sched.jstep, jcount = sched.jcount;
  auto rb_of = [&](int64_t v) { return sched.rb(v); };
  if (j >= jcount) {
    block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
    return;
  }
  auto block_rows = [&](int64_t b) { return (int)min((int64_t)kBlock, a.n - b * kBlock); };
  auto wstart = [](int64_t e) { return VEC ? (e & ~(int64_t)3) : e; };

  // current row block
  int64_t r0 = rb_of(j) * kBlock;
  int nr = block_rows(rb_of(j));
  int64_t bs = (int64_t)rowptr[r0];
  int64_t be = (int64_t)rowptr[r0 + nr];
  int64_t my_end = tid < nr ? (int64_t)rowptr[r0 + tid + 1] : 0;
  W my_mask = 0, my_mask_n = 0, mrem = 0;
  if constexpr (!COLS) my_mask = tid < nr ? (W)mask[r0 + tid] : 0;
  // next row block: nnz range as scalars (issued now, used one block later)
  int64_t bsn = 0, ben = 0;
  if (j + jstep < jcount) {
    const int64_t rbn = rb_of(j + jstep);
    const int64_t r0n = rbn * kBlock;
    bsn = (int64_t)rowptr[r0n];
    ben = (int64_t)rowptr[r0n + block_rows(rbn)];
  }
  Stage st;  // the window in flight
  int64_t ws = wstart(bs);
  stage_load<VEC, NT, COLS>(st, val, col, ws, bs, be, tid);
  bool first_window = true;
  int rs = 0, re = 0;
  double sum1 = 0.0, sum2 = 0.0;
  // the next row block's state, loaded when its first window is issued
  int64_t r0n = 0, my_end_n = 0, bsnn = 0, bennn = 0;
  int nrn = 0;
  (void)bennn;

  EpiIn pin;  // this lane's own-row epilogue operands, loaded at row-block start
  for (;;) {
    if (first_window) {
      if (tid < nr) s_rp[tid + 1] = (int32_t)(my_end - bs);
      if (tid == 0) s_rp[0] = 0;
      if (tid < nr && !a.epi_late) pin = epi_load<EPI>(a, r0 + tid);
    }
    stage_commit<COLS>(st, s_val, s_col, tid);
    __syncthreads();
    const bool active = tid < nr;
    if (first_window) {
      rs = active ? s_rp[tid] : 0;
      re = active ? s_rp[tid + 1] : 0;
      mrem = my_mask;
    }
    // issue the next window before working on this one
    const bool last_window = ws + kWindow >= be;
    const int64_t j_next = j + jstep;
    const bool has_next = j_next < jcount;
    const int64_t rb_next = has_next ? rb_of(j_next) : 0;
    if (!last_window) {
      stage_load<VEC, NT, COLS>(st, val, col, ws + kWindow, bs, be, tid);
    } else if (has_next) {
      r0n = rb_next * kBlock;
      nrn = block_rows(rb_next);
      my_end_n = tid < nrn ? (int64_t)rowptr[r0n + tid + 1] : 0;
      if constexpr (!COLS) my_mask_n = tid < nrn ? (W)mask[r0n + tid] : 0;
      stage_load<VEC, NT, COLS>(st, val, col, wstart(bsn), bsn, ben, tid);
      if (j_next + jstep < jcount) {
        const int64_t rb_nn = rb_of(j_next + jstep);
        const int64_t r0nn = rb_nn * kBlock;
        bsnn = (int64_t)rowptr[r0nn];
        bennn = (int64_t)rowptr[r0nn + block_rows(rb_nn)];
      }
    }
    // this lane's entries inside the window (window offsets)
    if (active) {
      const int64_t off = bs - ws;
      const int js = (int)max((int64_t)rs + off, (int64_t)0);
      const int je = (int)min((int64_t)re + off, (int64_t)kWindow);
      if constexpr (COLS)
        row_window<NV, GATHER>(s_val, s_col, x1, x2, js, je, sum1, sum2);
      else
        row_window_mask<NV, GATHER>(s_val, s_M, x1, x2, a.xoff + r0 + tid, js, je, mrem, sum1,
                                    sum2);
    }
    if (!last_window) {
      __syncthreads();  // LDS is rewritten by the next window
      ws += kWindow;
      first_window = false;
      continue;
    }
    if (active) {
      epi_row_in<EPI>(a, r0 + tid, sum1, sum2, x1, x2,
                      a.epi_late ? epi_load<EPI>(a, r0 + tid) : pin, acc);
    }
    if (!has_next) break;
    __syncthreads();  // LDS and s_rp are rewritten by the next row block
    j = j_next;
    r0 = r0n;
    nr = nrn;
    bs = bsn;
    be = ben;
    bsn = bsnn;
    ben = bennn;
    my_end = my_end_n;
    my_mask = my_mask_n;
    ws = wstart(bs);
    first_window = true;
    sum1 = 0.0;
    sum2 = 0.0;
  }
  __syncthreads();
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
}

// Product-then-sum SpMV for long rows (variant 8; chosen by the host when
// nnz/row is large). Each window's entries are multiplied entry-parallel:
// lane t owns entries 2(t + 256q) + {0,1} (a 16-byte value load and an 8-byte
// column load per slot), gathers x for all of them at once, and writes the
// products fl(v * x) to LDS. Then each lane adds its own row's products in
// stored order, carrying the running sum across windows -- the same
// operations in the same order as scipy, so the result is still bitwise.
// Every lane gathers in every window, however few rows the window holds.
constexpr int kPSlots = kWindow / (2 * kBlock);
typedef int int2v __attribute__((ext_vector_type(2)));

struct PStage {
  dbl2v v[kPSlots];
  int2v c[kPSlots];
};

template <bool VEC>
__device__ __forceinline__ void pstage_load(PStage& st, const double* __restrict__ val,
                                            const int32_t* __restrict__ col, int64_t ws,
                                            int64_t bs, int64_t be, int tid) {
#pragma unroll
  for (int q = 0; q < kPSlots; ++q) {
    const int64_t g0 = ws + (int64_t)(tid + q * kBlock) * 2;
    if (VEC && g0 >= bs && g0 + 2 <= be) {
      st.v[q] = *reinterpret_cast<const dbl2v*>(val + g0);
      st.c[q] = *reinterpret_cast<const int2v*>(col + g0);
    } else {
      const bool ok0 = g0 >= bs && g0 < be, ok1 = g0 + 1 >= bs && g0 + 1 < be;
      st.v[q] = dbl2v{ok0 ? val[g0] : 0.0, ok1 ? val[g0 + 1] : 0.0};
      st.c[q] = int2v{ok0 ? col[g0] : -1, ok1 ? col[g0 + 1] : -1};
    }
  }
}

template <int NV>
__device__ __forceinline__ void pstage_products(const PStage& st, const double* __restrict__ x1,
                                                const double* __restrict__ x2, double* s_p1,
                                                double* s_p2, int tid) {
  double g1[2 * kPSlots], g2[2 * kPSlots];
#pragma unroll
  for (int q = 0; q < kPSlots; ++q) {
    const int c0 = st.c[q].x, c1 = st.c[q].y;
    g1[2 * q] = c0 >= 0 ? x1[c0] : 0.0;
    g1[2 * q + 1] = c1 >= 0 ? x1[c1] : 0.0;
    if constexpr (NV == 2) {
      g2[2 * q] = c0 >= 0 ? x2[c0] : 0.0;
      g2[2 * q + 1] = c1 >= 0 ? x2[c1] : 0.0;
    }
  }
#pragma unroll
  for (int q = 0; q < kPSlots; ++q) {
    reinterpret_cast<dbl2v*>(s_p1)[tid + q * kBlock] =
        dbl2v{st.v[q].x * g1[2 * q], st.v[q].y * g1[2 * q + 1]};
    if constexpr (NV == 2)
      reinterpret_cast<dbl2v*>(s_p2)[tid + q * kBlock] =
          dbl2v{st.v[q].x * g2[2 * q], st.v[q].y * g2[2 * q + 1]};
  }
}

template <typename RP, int EPI, bool VEC>
__global__ __launch_bounds__(kBlock) void spmv_kernel_prod(SpmvArgs a) {
  if (a.stop && *a.stop != 0.0) return;  // converged (device-resident scalars)
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  __shared__ __attribute__((aligned(16))) double s_p1[kWindow];
  __shared__ __attribute__((aligned(16))) double s_p2[NV == 2 ? kWindow : 2];
  __shared__ int32_t s_rp[kBlock + 1];
  __shared__ double s_red[(NP > 0 ? NP : 1) * 4];

  const RP* __restrict__ rowptr = static_cast<const RP*>(a.rowptr);
  const double* __restrict__ val = a.val;
  const int32_t* __restrict__ col = a.col;
  const double* __restrict__ x1 = a.x1;
  const double* __restrict__ x2 = a.x2;
  const int tid = threadIdx.x;

  double acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) acc[p] = 0.0;

  const int64_t nrb = (a.n + kBlock - 1) / kBlock - a.rb_gap;
  RowSched sched;  // as spmv_kernel
  sched.init(nrb, a.slab, a.slab_sub, true);
  sched.gap_at = a.rb_gap_at;
  sched.gap = a.rb_gap;
  int64_t j = sched.j0;
  const int64_t jstep = sched.jstep, jcount = sched.jcount;
  auto rb_of = [&](int64_t v) { return sched.rb(v); };
  if (j >= jcount) {
    block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
    return;
  }
  auto block_rows = [&](int64_t b) { return (int)min((int64_t)kBlock, a.n - b * kBlock); };
  auto wstart = [](int64_t e) { return VEC ? (e & ~(int64_t)1) : e; };

  int64_t r0 = rb_of(j) * kBlock;
  int nr = block_rows(rb_of(j));
  int64_t bs = (int64_t)rowptr[r0];
  int64_t be = (int64_t)rowptr[r0 + nr];
  int64_t my_end = tid < nr ? (int64_t)rowptr[r0 + tid + 1] : 0;
  int64_t bsn = 0, ben = 0;
  if (j + jstep < jcount) {
    const int64_t rbn = rb_of(j + jstep);
    const int64_t r0n = rbn * kBlock;
    bsn = (int64_t)rowptr[r0n];
    ben = (int64_t)rowptr[r0n + block_rows(rbn)];
  }
  PStage st;
  int64_t ws = wstart(bs);
  pstage_load<VEC>(st, val, col, ws, bs, be, tid);
  bool first_window = true;
  int rs = 0, re = 0;
  double sum1 = 0.0, sum2 = 0.0;
  int64_t r0n = 0, my_end_n = 0, bsnn = 0, bennn = 0;
  int nrn = 0;

  EpiIn pin;  // this lane's own-row epilogue operands, loaded at row-block start
  for (;;) {
    if (first_window) {
      if (tid < nr) s_rp[tid + 1] = (int32_t)(my_end - bs);
      if (tid == 0) s_rp[0] = 0;
      if (tid < nr && !a.epi_late) pin = epi_load<EPI>(a, r0 + tid);
    }
    pstage_products<NV>(st, x1, x2, s_p1, s_p2, tid);
    __syncthreads();
    const bool active = tid < nr;
    if (first_window) {
      rs = active ? s_rp[tid] : 0;
      re = active ? s_rp[tid + 1] : 0;
    }
    const bool last_window = ws + kWindow >= be;
    const int64_t j_next = j + jstep;
    const bool has_next = j_next < jcount;
    const int64_t rb_next = has_next ? rb_of(j_next) : 0;
    if (!last_window) {
      pstage_load<VEC>(st, val, col, ws + kWindow, bs, be, tid);
    } else if (has_next) {
      r0n = rb_next * kBlock;
      nrn = block_rows(rb_next);
      my_end_n = tid < nrn ? (int64_t)rowptr[r0n + tid + 1] : 0;
      pstage_load<VEC>(st, val, col, wstart(bsn), bsn, ben, tid);
      if (j_next + jstep < jcount) {
        const int64_t rb_nn = rb_of(j_next + jstep);
        const int64_t r0nn = rb_nn * kBlock;
        bsnn = (int64_t)rowptr[r0nn];
        bennn = (int64_t)rowptr[r0nn + block_rows(rb_nn)];
      }
    }
    if (active) {
      const int64_t off = bs - ws;
      const int js = (int)max((int64_t)rs + off, (int64_t)0);
      const int je = (int)min((int64_t)re + off, (int64_t)kWindow);
      for (int j = js; j < je; ++j) {
        sum1 = sum1 + s_p1[j];
        if constexpr (NV == 2) sum2 = sum2 + s_p2[j];
      }
    }
    if (!last_window) {
      __syncthreads();
      ws += kWindow;
      first_window = false;
      continue;
    }
    if (active) {
      epi_row_in<EPI>(a, r0 + tid, sum1, sum2, x1, x2,
                      a.epi_late ? epi_load<EPI>(a, r0 + tid) : pin, acc);
    }
    if (!has_next) break;
    __syncthreads();
    j = j_next;
    r0 = r0n;
    nr = nrn;
    bs = bsn;
    be = ben;
    bsn = bsnn;
    ben = bennn;
    my_end = my_end_n;
    ws = wstart(bs);
    first_window = true;
    sum1 = 0.0;
    sum2 = 0.0;
  }
  __syncthreads();
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
}

// Uniform loads through the scalar cache: the row-block boundaries
// rowptr[r0], rowptr[r0 + nr] are the same for every lane, and the matrix is
// constant while the kernel runs, so they are read as constant-address-space
// (s_load) values. A vector load here would make the next window's address
// computation wait (vmcnt, in order) for every vector load issued before it.
template <typename T>
__device__ __forceinline__ T load_uniform(const T* p, int64_t i) {
  return ((const __attribute__((address_space(4))) T*)p)[i];
}

// Window staging for spmv_kernel2. EVERY lane issues exactly the same loads
// whatever the window: a slot past the window's last entry re-reads the
// 16-byte chunk holding that entry (same line, no new traffic) instead of
// being skipped, and there is no edge branch. Entries outside [bs, be) land
// in LDS but no row reads them. Equal load counts on every path let the
// compiler wait for exactly the loads it needs (vmcnt counts in issue order;
// with a skippable load it has to assume the fewer-loads path and waits for
// everything). Needs >= 4 entries in the matrix (host check).
template <bool COLS, bool NT = false, bool VALS = true>
__device__ __forceinline__ void stage_load2(Stage& st, const double* __restrict__ val,
                                            const int32_t* __restrict__ col, int64_t ws,
                                            int64_t be, int tid) {
  const int64_t vlast = max((be - 1) & ~(int64_t)1, (int64_t)0);
#pragma unroll
  for (int q = 0; q < (VALS ? kVSlots : 0); ++q) {
    const int64_t g0 = min(ws + (int64_t)(tid + q * kBlock) * 2, vlast);
    if constexpr (NT)
      st.v[q] = __builtin_nontemporal_load(reinterpret_cast<const dbl2v*>(val + g0));
    else
      st.v[q] = *reinterpret_cast<const dbl2v*>(val + g0);
  }
  if constexpr (COLS) {
    const int64_t clast = max((be - 1) & ~(int64_t)3, (int64_t)0);
#pragma unroll
    for (int q = 0; q < kCSlots; ++q) {
      const int64_t g0 = min(ws + (int64_t)(tid + q * kBlock) * 4, clast);
      if constexpr (NT)
        st.c[q] = __builtin_nontemporal_load(reinterpret_cast<const int4v*>(col + g0));
      else
        st.c[q] = *reinterpret_cast<const int4v*>(col + g0);
    }
  }
}

// Row walk, version 2 (default for short rows). Same arithmetic and order as
// spmv_kernel (bitwise scipy csr_matvec), reorganised around the in-order
// completion of vector loads (vmcnt): per window, a lane FIRST issues its
// first batch of x gathers, THEN the loads of the next window (values, its
// row range and mask), so waiting for the gathers does not wait for the
// next window's HBM round trip, which stays in flight across the row sums,
// the epilogue and the next LDS commit. The block boundaries come through
// the scalar cache (load_uniform), the LDS windows are double-buffered (one
// barrier per window), and each lane loads its own row range (no LDS
// exchange of row pointers).
// VI: values through the dictionary (SpmvArgs::vcode): each lane loads the 8
// one-byte codes of its 8 window entries (one 8-byte load: windows start on a
// multiple of 8) and commits them to an LDS code window (2 KiB instead of the
// 16 KiB value window); entries are decoded through the LDS table on read.
template <typename RP, int EPI, bool VEC, int MW, bool DB = true, bool NT = false,
          bool VI = false, bool PO = false>
__device__ __forceinline__ void spmv2_body(SpmvArgs& a) {
  if (!spmv_entry<EPI>(a)) return;  // converged / the fused scalar step's test fired
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  constexpr bool VIRT = is_virtual<EPI>();
  constexpr int G = kGather;
  constexpr bool COLS = MW == 0;  // else: offset masks, no column stream
  using MT = typename MaskType<(MW > 0 ? MW : 64)>::type;
  using W = typename std::conditional<(MW > 32), uint64_t, uint32_t>::type;
  // DB: double-buffered windows, one barrier per window; else one buffer
  // (half the LDS: more workgroups per CU) and a second barrier.
  constexpr int NB = DB ? 2 : 1;
  // VI: the window holds 1-byte codes (s_code), decoded through s_tab on read
  __shared__ __attribute__((aligned(16))) double s_val[NB][VI ? 2 : kWindow];
  __shared__ __attribute__((aligned(16))) uint8_t s_code[VI ? NB : 1][VI ? kWindow : 16];
  __shared__ __attribute__((aligned(16))) int32_t s_col[COLS ? NB : 1][COLS ? kWindow : 4];
  __shared__ int32_t s_M[COLS ? 1 : 64];
  __shared__ double s_red[(NP > 0 ? NP : 1) * 4];

  const RP* __restrict__ rowptr = static_cast<const RP*>(a.rowptr);
  const MT* __restrict__ mask = static_cast<const MT*>(a.mask);
  const double* __restrict__ val = a.val;
  const int32_t* __restrict__ col = a.col;
  const double* __restrict__ x1 = a.x1;
  const double* __restrict__ x2 = a.x2;
  const int tid = threadIdx.x;
  if constexpr (!COLS) {
    if (tid < a.nm) s_M[tid] = a.moff[tid];  // seen after the first barrier
  }
  static_assert(!VI || (VEC && kWindow == 8 * kBlock), "dictionary staging: 8 codes per lane");
  __shared__ double s_tab[VI ? kVdMax : 1];
  if constexpr (VI) {
    if (tid < a.ntab) s_tab[tid] = a.vtab[tid];
    __syncthreads();  // the first commit decodes through s_tab
  }

  double acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) acc[p] = 0.0;

  const int64_t nrb = (a.n + kBlock - 1) / kBlock - a.rb_gap;
  RowSched sched;
  sched.init(nrb, a.slab, a.slab_sub, true);
  sched.gap_at = a.rb_gap_at;
  sched.gap = a.rb_gap;
  int64_t j = sched.j0;
  const int64_t jstep = sched.jstep, jcount = sched.jcount;
  if (j >= jcount) {
    block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
    return;
  }
  auto block_rows = [&](int64_t b) { return (int)min((int64_t)kBlock, a.n - b * kBlock); };
  auto wstart = [](int64_t e) { return VI ? (e & ~(int64_t)7) : VEC ? (e & ~(int64_t)3) : e; };

  // current row block: boundaries (uniform), this lane's row range and mask
  int64_t r0 = sched.rb(j) * kBlock;
  int nr = block_rows(sched.rb(j));
  int64_t bs = (int64_t)load_uniform(rowptr, r0);
  int64_t be = (int64_t)load_uniform(rowptr, r0 + nr);
  RP rlo = 0, rhi = 0;  // converted at use: a conversion here would wait on the load
  W my_mask = 0;
  {
    const int64_t ri = min(r0 + tid, a.n - 1);
    rlo = rowptr[ri];
    rhi = rowptr[ri + 1];
    if constexpr (!COLS) my_mask = (W)mask[ri];
  }
  int64_t bsn = 0, ben = 0;  // next row block's boundaries
  if (j + jstep < jcount) {
    const int64_t rbn = sched.rb(j + jstep);
    bsn = (int64_t)load_uniform(rowptr, rbn * kBlock);
    ben = (int64_t)load_uniform(rowptr, rbn * kBlock + block_rows(rbn));
  }
  Stage st;
  uint64_t cw = 0;  // VI: this lane's 8 codes of the staged window
  int64_t ws = wstart(bs);
  auto stage = [&](int64_t w, int64_t lo, int64_t hi) {
    if constexpr (VI) {
      // same load count on every path (see stage_load2): clamp to the last
      // 8-code chunk holding an entry of the block (codes are padded by 8)
      const int64_t c0 = min(w + (int64_t)tid * 8, max((hi - 1) & ~(int64_t)7, (int64_t)0));
      const uint64_t* cp = reinterpret_cast<const uint64_t*>(a.vcode + c0);
      if constexpr (NT)
        cw = __builtin_nontemporal_load(cp);
      else
        cw = *cp;
      if constexpr (COLS) stage_load2<COLS, NT, false>(st, val, col, w, hi, tid);
    } else if constexpr (VEC) {
      stage_load2<COLS, NT>(st, val, col, w, hi, tid);
    } else {
      stage_load<false, false, COLS>(st, val, col, w, lo, hi, tid);
    }
  };
  stage(ws, bs, be);
  int buf = 0;
  bool first_window = true;
  W mrem = 0;
  EpiIn pin;
  double sum1 = 0.0, sum2 = 0.0;
  // next row block's lane state (loaded while the current window is summed)
  int64_t r0n = 0;
  RP rlo_n = 0, rhi_n = 0;
  int nrn = 0;
  W mask_n = 0;

  for (;;) {
    using VS = typename std::conditional<VI, CodeView, const double*>::type;
    VS sv;
    if constexpr (VI)
      sv = CodeView{s_code[DB ? buf : 0], s_tab};
    else
      sv = s_val[DB ? buf : 0];
    int32_t* sc = s_col[COLS && DB ? buf : 0];
    if constexpr (VI) {
      reinterpret_cast<uint64_t*>(s_code[DB ? buf : 0])[tid] = cw;
      if constexpr (COLS) {
#pragma unroll
        for (int q = 0; q < kCSlots; ++q)
          reinterpret_cast<int4v*>(sc)[tid + q * kBlock] = st.c[q];
      }
    } else {
      stage_commit<COLS>(st, s_val[DB ? buf : 0], sc, tid);
    }
    __syncthreads();
    const bool active = tid < nr;
    if (first_window) {
      mrem = my_mask;
      // own-row epilogue operands, issued before the gathers so that
      // waiting for the gathers covers them
      pin = epi_load<EPI>(a, active ? r0 + tid : r0);
    }
    const int64_t off = bs - ws;
    const int js = active ? (int)max((int64_t)rlo - bs + off, (int64_t)0) : 0;
    const int je = active ? (int)min((int64_t)rhi - bs + off, (int64_t)kWindow) : 0;
    // lanes past the block's last row gather at row r0 (their products are
    // dropped): x + xoff + r0 + tid may lie past the vector's end when the
    // shard has no halo above it
    const int64_t xrow = a.xoff + r0 + (active ? tid : 0);

    // (1) first gather batch of this window
    double v[G], p1[G], p2[G], p3[VIRT ? G : 1];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const bool ok = js + u < je;
      v[u] = sv[ok ? js + u : 0];
      int64_t c;
      if constexpr (COLS) {
        c = sc[ok ? js + u : 0];
      } else {
        c = xrow;
        if (ok) {
          c += s_M[sizeof(W) == 8 ? __builtin_ctzll((unsigned long long)mrem)
                                  : __builtin_ctz((unsigned)mrem)];
          mrem &= mrem - 1;
        }
      }
      p1[u] = x1[c];
      if constexpr (NV == 2 || VIRT) p2[u] = x2[c];
      if constexpr (VIRT) p3[u] = a.x3[c];
    }

    // (2) the next window's loads: they stay in flight while this one is summed
    const bool last_window = ws + kWindow >= be;
    const int64_t j_next = j + jstep;
    const bool has_next = j_next < jcount;
    // Issued unconditionally, from ONE call site, with the same count on
    // every path (see stage_load2): the last window of the last row block
    // re-reads itself. Two call sites would get two register sets and a copy
    // that waits for the loads.
    {
      const bool nb = last_window && has_next;  // next row block
      const int64_t nws = !last_window ? ws + kWindow : nb ? wstart(bsn) : ws;
      stage(nws, nb ? bsn : bs, nb ? ben : be);
      if (nb) {
        const int64_t rb_next = sched.rb(j_next);
        r0n = rb_next * kBlock;
        nrn = block_rows(rb_next);
      }
      const int64_t ri = min((nb ? r0n : r0) + tid, a.n - 1);  // clamped: no branch
      rlo_n = rowptr[ri];
      rhi_n = rowptr[ri + 1];
      if constexpr (!COLS) mask_n = (W)mask[ri];
    }

    // (3) sums, in stored order: the first batch, then any further batches
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (js + u < je) {
        if constexpr (VIRT) {
          sum1 = sum1 + v[u] * virt_in<EPI>(a, p1[u], p2[u], p3[u]);
        } else {
          sum1 = sum1 + v[u] * p1[u];
          if constexpr (NV == 2) sum2 = sum2 + v[u] * p2[u];
        }
      }
    }
    if (je - js > G) {
      if constexpr (VIRT) {
        if constexpr (COLS)
          row_window_virtual<EPI, G>(sv, sc, nullptr, 0, a, js + G, je, mrem, sum1);
        else
          row_window_virtual<EPI, G>(sv, nullptr, s_M, xrow, a, js + G, je, mrem, sum1);
      } else if constexpr (COLS) {
        row_window<NV, G>(sv, sc, x1, x2, js + G, je, sum1, sum2);
      } else {
        row_window_mask<NV, G>(sv, s_M, x1, x2, xrow, js + G, je, mrem, sum1, sum2);
      }
    }
    buf ^= 1;
    if constexpr (!DB) __syncthreads();  // the single buffer is rewritten next
    if (!last_window) {
      ws += kWindow;
      first_window = false;
      continue;
    }
    // NT: the matrix stream AND the result stores non-temporal (variant 13,
    // chosen at launch for shards >= 4M rows: SpmvArgs::nt_stores). A
    // run-time choice between the two stores measured 2.6 % slower on the
    // plain-CSR dual (a store under a branch shifts the compiler's waits).
    if (active)
      epi_store_row_k<EPI, NT ? 1 : 0, PO ? 1 : 0>(a, r0 + tid,
                                                   epi_values<EPI>(a, sum1, sum2, pin, acc));
    if (!has_next) break;
    // advance to the next row block; its boundaries after it come through
    // the scalar cache now (used one row block later)
    j = j_next;
    r0 = r0n;
    nr = nrn;
    bs = bsn;
    be = ben;
    rlo = rlo_n;
    rhi = rhi_n;
    my_mask = mask_n;
    if (j + jstep < jcount) {
      const int64_t rbnn = sched.rb(j + jstep);
      bsn = (int64_t)load_uniform(rowptr, rbnn * kBlock);
      ben = (int64_t)load_uniform(rowptr, rbnn * kBlock + block_rows(rbnn));
    }
    ws = wstart(bs);
    first_window = true;
    sum1 = 0.0;
    sum2 = 0.0;
  }
  __syncthreads();
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
}

template <typename RP, int EPI, bool VEC, int MW, bool DB = true, bool NT = false,
          bool VI = false>
__global__ __launch_bounds__(kBlock) void spmv_kernel2(SpmvArgs a) {
  spmv2_body<RP, EPI, VEC, MW, DB, NT, VI, false>(a);
}
// Products-only duals (the last basis dual of a k-skip outer iteration: no y
// stores) as their own kernel, under their own symbol (rocprofv3 tells them
// from the storing duals: tools/pmc_summary.py "_last").
template <typename RP, int EPI, bool VEC, int MW, bool DB = true, bool NT = false,
          bool VI = false>
__global__ __launch_bounds__(kBlock) void spmv_kernel2_po(SpmvArgs a) {
  spmv2_body<RP, EPI, VEC, MW, DB, NT, VI, true>(a);
}

// Every spmv_kernel2 launch: the products-only kernel for a products-only
// dual (spmv_kernel2 itself always stores).
template <typename RP, int E, bool VEC, int MW, bool DB, bool NT, bool VI = false>
void spmv2_go(const SpmvArgs& a, dim3 grid, dim3 block, hipStream_t s) {
  if constexpr (EpiTraits<E>::NV == 2 && !is_step<E>()) {
    if (a.products_only) {
      spmv_kernel2_po<RP, E, VEC, MW, DB, NT, VI><<<grid, block, 0, s>>>(a);
      return;
    }
  }
  spmv_kernel2<RP, E, VEC, MW, DB, NT, VI><<<grid, block, 0, s>>>(a);
}

template <typename RP, int E, bool VEC, bool DB, bool NT>
void spmv2_launch_vi(const SpmvArgs& a, dim3 grid, dim3 block, hipStream_t s) {
  switch (a.mask ? a.mw : 0) {
    case 8: return spmv2_go<RP, E, VEC, 8, DB, NT, true>(a, grid, block, s);
    case 16: return spmv2_go<RP, E, VEC, 16, DB, NT, true>(a, grid, block, s);
    case 32: return spmv2_go<RP, E, VEC, 32, DB, NT, true>(a, grid, block, s);
    case 64: return spmv2_go<RP, E, VEC, 64, DB, NT, true>(a, grid, block, s);
    default: return spmv2_go<RP, E, VEC, 0, DB, NT, true>(a, grid, block, s);
  }
}

template <typename RP, int E, bool VEC, bool DB = true, bool NT = false>
void spmv2_launch(const SpmvArgs& a, dim3 grid, dim3 block, hipStream_t s) {
  if constexpr (VEC) {
    if (a.vcode) {
      spmv2_launch_vi<RP, E, VEC, DB, NT>(a, grid, block, s);
      return;
    }
  }
  switch (a.mask ? a.mw : 0) {
    case 8: return spmv2_go<RP, E, VEC, 8, DB, NT>(a, grid, block, s);
    case 16: return spmv2_go<RP, E, VEC, 16, DB, NT>(a, grid, block, s);
    case 32: return spmv2_go<RP, E, VEC, 32, DB, NT>(a, grid, block, s);
    case 64: return spmv2_go<RP, E, VEC, 64, DB, NT>(a, grid, block, s);
    default: return spmv2_go<RP, E, VEC, 0, DB, NT>(a, grid, block, s);
  }
}

// ---------------------------------------------------------------------------
// Product-then-sum, version 2 (default for long rows). The operations and
// their order are spmv_kernel_prod's (bitwise scipy), organised like
// spmv_kernel2 around the in-order completion of vector loads, as a two-stage
// software pipeline over windows: while the products of window t are formed
// and its rows summed, the gathers of window t+1 and the loads of window t+2
// are in flight. Per iteration: wait for the gathers of t (issued one
// iteration earlier), write its products to LDS; wait for the loads of t+1,
// issue its gathers; issue the loads of t+2; barrier; sum window t. Gathers
// and window loads are issued unconditionally (a drained stage re-issues
// valid addresses) so every path has the same load count after the gathers
// and the waits stay exact; every gathered column is a real entry's column.
// ---------------------------------------------------------------------------
struct PWin {  // one staging window, uniform across the workgroup
  int64_t ws = 0, bs = 0, be = 0, r0 = 0;
  int nr = 0, first = 0, last = 0, valid = 0;
};

// PS slots of 2 entries per lane: a window of PS * 2 * kBlock entries.
template <int PS>
struct PStageN {
  dbl2v v[PS];
  int2v c[PS];
};

template <bool NT, int PS>
__device__ __forceinline__ void pstage_load2(PStageN<PS>& st, const double* __restrict__ val,
                                             const int32_t* __restrict__ col, int64_t ws,
                                             int64_t be, int tid) {
  const int64_t last = max((be - 1) & ~(int64_t)1, (int64_t)0);
#pragma unroll
  for (int q = 0; q < PS; ++q) {
    const int64_t g0 = min(ws + (int64_t)(tid + q * kBlock) * 2, last);
    if constexpr (NT)
      st.v[q] = __builtin_nontemporal_load(reinterpret_cast<const dbl2v*>(val + g0));
    else
      st.v[q] = *reinterpret_cast<const dbl2v*>(val + g0);
    st.c[q] = *reinterpret_cast<const int2v*>(col + g0);
  }
}

// PS slots per lane (window PS * 512 entries): 4 for one vector; 2 for two
// vectors, whose doubled gather and product registers would otherwise cost a
// wave per SIMD (144 VGPRs at 4 slots).
template <typename RP, int EPI, bool DB, bool NT, int PS>
__global__ __launch_bounds__(kBlock) void spmv_kernel_prod2(SpmvArgs a) {
  if (a.stop && *a.stop != 0.0) return;  // converged (device-resident scalars)
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  constexpr int NB = DB ? 2 : 1;  // product buffers
  constexpr int NE = 2 * PS;      // entries per lane per window
  constexpr int KW = PS * 2 * kBlock;  // window entries
  __shared__ __attribute__((aligned(16))) double s_p1[NB][KW];
  __shared__ __attribute__((aligned(16))) double s_p2[NV == 2 ? NB : 1][NV == 2 ? KW : 2];
  __shared__ double s_red[(NP > 0 ? NP : 1) * 4];

  const RP* __restrict__ rowptr = static_cast<const RP*>(a.rowptr);
  const double* __restrict__ val = a.val;
  const int32_t* __restrict__ col = a.col;
  const double* __restrict__ x1 = a.x1;
  const double* __restrict__ x2 = a.x2;
  const int tid = threadIdx.x;

  double acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) acc[p] = 0.0;

  const int64_t nrb = (a.n + kBlock - 1) / kBlock - a.rb_gap;
  RowSched sched;
  sched.init(nrb, a.slab, a.slab_sub, true);
  sched.gap_at = a.rb_gap_at;
  sched.gap = a.rb_gap;
  const int64_t jstep = sched.jstep, jcount = sched.jcount;
  if (sched.j0 >= jcount) {
    block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
    return;
  }
  auto block_rows = [&](int64_t b) { return (int)min((int64_t)kBlock, a.n - b * kBlock); };
  auto wstart = [](int64_t e) { return e & ~(int64_t)1; };

  // Window generator: gj is the schedule index of the block of the newest
  // window, (bsn, ben) the bounds of the block after it (scalar cache).
  int64_t gj = sched.j0, bsn = 0, ben = 0;
  auto fetch_next_bounds = [&]() {
    if (gj + jstep < jcount) {
      const int64_t rb = sched.rb(gj + jstep);
      bsn = (int64_t)load_uniform(rowptr, rb * kBlock);
      ben = (int64_t)load_uniform(rowptr, rb * kBlock + block_rows(rb));
    }
  };
  PWin w0;
  {
    const int64_t rb = sched.rb(gj);
    w0.r0 = rb * kBlock;
    w0.nr = block_rows(rb);
    w0.bs = (int64_t)load_uniform(rowptr, w0.r0);
    w0.be = (int64_t)load_uniform(rowptr, w0.r0 + w0.nr);
    w0.ws = wstart(w0.bs);
    w0.first = 1;
    w0.last = w0.ws + KW >= w0.be;
    w0.valid = 1;
  }
  fetch_next_bounds();
  auto advance = [&](const PWin& w) {
    PWin o = w;
    if (!w.valid) return o;
    if (!w.last) {
      o.ws = w.ws + KW;
      o.first = 0;
      o.last = o.ws + KW >= o.be;
      return o;
    }
    if (gj + jstep >= jcount) {
      o.valid = 0;
      return o;
    }
    gj += jstep;
    const int64_t rb = sched.rb(gj);
    o.r0 = rb * kBlock;
    o.nr = block_rows(rb);
    o.bs = bsn;
    o.be = ben;
    o.ws = wstart(bsn);
    o.first = 1;
    o.last = o.ws + KW >= o.be;
    fetch_next_bounds();
    return o;
  };

  // stage registers: st = loads of the load-stage window; pv/g1/g2 = values
  // and gathered x of the gather-stage window; row ranges of the sum-,
  // gather- and load-stage windows' blocks (rlo_s/_g/_l)
  PStageN<PS> st;
  dbl2v pv[PS];
  double g1[NE], g2[NV == 2 ? NE : 1];
  RP rlo_l = 0, rhi_l = 0, rlo_g = 0, rhi_g = 0, rlo_s = 0, rhi_s = 0;
  EpiIn pin_g, pin_s;
  double sum1 = 0.0, sum2 = 0.0;
  {
    const int64_t ri = min(w0.r0 + tid, a.n - 1);
    rlo_g = rowptr[ri];
    rhi_g = rowptr[ri + 1];
  }
  pstage_load2<NT, PS>(st, val, col, w0.ws, w0.be, tid);
  PWin wsum, wg = w0;  // wsum invalid: the pipeline fills first
  int it = 0;
  for (;;) {
    if (!wsum.valid && !wg.valid) break;
    // (a) products of the sum-stage window (its gathers were issued last round)
    if constexpr (!DB) __syncthreads();  // the single buffer's last readers are done
    if (wsum.valid) {
      double* p1 = s_p1[DB ? (it & 1) : 0];
#pragma unroll
      for (int q = 0; q < PS; ++q) {
        reinterpret_cast<dbl2v*>(p1)[tid + q * kBlock] =
            dbl2v{pv[q].x * g1[2 * q], pv[q].y * g1[2 * q + 1]};
        if constexpr (NV == 2) {
          double* p2 = s_p2[DB ? (it & 1) : 0];
          reinterpret_cast<dbl2v*>(p2)[tid + q * kBlock] =
              dbl2v{pv[q].x * g2[2 * q], pv[q].y * g2[2 * q + 1]};
        }
      }
    }
    // (b) gather stage: the gather-stage window's loads have landed. A slot
    // holds entries (e, e+1) of a real chunk (pstage_load2's clamp), but the
    // second entry of the last chunk can lie past the matrix end: columns of
    // entries at or past the block end are replaced by 0 (a valid x index;
    // the product lands in a slot no row reads).
    const int64_t wlast = max((wg.be - 1) & ~(int64_t)1, (int64_t)0);
#pragma unroll
    for (int q = 0; q < PS; ++q) {
      pv[q] = st.v[q];
      const int64_t e0 = min(wg.ws + (int64_t)(tid + q * kBlock) * 2, wlast);
      const int c0 = e0 < wg.be ? st.c[q].x : 0;
      const int c1 = e0 + 1 < wg.be ? st.c[q].y : 0;
      g1[2 * q] = x1[c0];
      g1[2 * q + 1] = x1[c1];
      if constexpr (NV == 2) {
        g2[2 * q] = x2[c0];
        g2[2 * q + 1] = x2[c1];
      }
    }
    if (wg.valid && wg.last) pin_g = epi_load<EPI>(a, min(wg.r0 + tid, a.n - 1));
    // (c) load stage: the window after the gather-stage one (row range first)
    const PWin wl = advance(wg);
    if (wl.valid && wl.first) {  // a new block: its row ranges
      const int64_t ri = min(wl.r0 + tid, a.n - 1);
      rlo_l = rowptr[ri];
      rhi_l = rowptr[ri + 1];
    } else {  // same block as the gather-stage window
      rlo_l = rlo_g;
      rhi_l = rhi_g;
    }
    const PWin& wld = wl.valid ? wl : wg;  // drained: re-issue valid addresses
    pstage_load2<NT, PS>(st, val, col, wld.ws, wld.be, tid);
    // (d) sum the sum-stage window's rows, in stored order
    __syncthreads();
    if (wsum.valid) {
      const double* p1 = s_p1[DB ? (it & 1) : 0];
      const double* p2 = s_p2[NV == 2 && DB ? (it & 1) : 0];
      if (wsum.first) {
        sum1 = 0.0;
        sum2 = 0.0;
      }
      if (tid < wsum.nr) {
        const int js = (int)max((int64_t)rlo_s - wsum.ws, (int64_t)0);
        const int je = (int)min((int64_t)rhi_s - wsum.ws, (int64_t)KW);
        for (int j = js; j < je; ++j) {
          sum1 = sum1 + p1[j];
          if constexpr (NV == 2) sum2 = sum2 + p2[j];
        }
        if (wsum.last) epi_row_in<EPI>(a, wsum.r0 + tid, sum1, sum2, x1, x2, pin_s, acc);
      }
    }
    // rotate the stages
    wsum = wg;
    wg = wl;
    rlo_s = rlo_g;
    rhi_s = rhi_g;
    rlo_g = rlo_l;
    rhi_g = rhi_l;
    pin_s = pin_g;
    ++it;
  }
  __syncthreads();
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
}

// ---------------------------------------------------------------------------
// Diagonal-offset SpMV (long rows with offset masks: banded, 27-point).
// The values are stored per row block of 256 rows, offset by offset
// (SpmvArgs::dia): for one offset, the entries of the block's consecutive
// rows are contiguous, and so are the x entries they multiply (x[row + M[b]]);
// a workgroup streams one contiguous nm x 2 KiB chunk. One lane per row, rows summed in stored order
// (increasing offset = increasing column, as in CSR) from 0.0: bitwise scipy.
// No LDS staging, no row pointers, no barrier: every load is a coalesced
// 512-byte wave access, and latency is hidden by occupancy (8 waves/SIMD).
// Loads are unconditional (absent entries read a valid slot and x[row]) and
// absent entries are skipped by a select, so the sum is exactly the CSR one.
// ---------------------------------------------------------------------------
// x[xi], x[xi + 1] (xi even): one 16-byte load inside [0, xlen), clamped
// scalar loads at the vector's ends (those window entries are never used).
__device__ __forceinline__ double2 window_pair(const double* __restrict__ x, int64_t xi,
                                               int64_t xlen) {
  if (xi >= 0 && xi + 1 < xlen) return *reinterpret_cast<const double2*>(x + xi);
  const int64_t i0 = min(max(xi, (int64_t)0), xlen - 1);
  const int64_t i1 = min(max(xi + 1, (int64_t)0), xlen - 1);
  return make_double2(x[i0], x[i1]);
}

// SYMUP > 0 (SpmvArgs::dia_sym, at most SYMUP diagonal + upper slots): the
// row's own diagonal and upper values are loaded first, all at once, then the
// lower entries as the mirrored upper entries of earlier rows -- which the
// neighbouring row block's workgroup, at the same point of its own row
// block, is loading at that moment (its upper values come first too), so
// one of the two reads hits L2. The sums keep the stored (ascending) order.
template <int EPI, int MW, int CH, bool XL, int SYMUP = 0>
__global__ __launch_bounds__(kBlock) void spmv_dia_kernel(SpmvArgs a) {
  if (!spmv_entry<EPI>(a)) return;  // converged / the fused scalar step's test fired
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  constexpr bool VIRT = is_virtual<EPI>();
  using MT = typename MaskType<MW>::type;
  using W = typename std::conditional<(MW > 32), uint64_t, uint32_t>::type;
  __shared__ double s_red[(NP > 0 ? NP : 1) * 4];
  const MT* __restrict__ mask = static_cast<const MT*>(a.mask);
  const double* __restrict__ dia = a.dia;
  const double* __restrict__ x1 = a.x1;
  const double* __restrict__ x2 = a.x2;
  const int tid = threadIdx.x;
  const int nm = a.nm;
  double acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) acc[p] = 0.0;

  const int64_t nrb = (a.n + kBlock - 1) / kBlock - a.rb_gap;
  RowSched sched;
  sched.init(nrb, a.slab, a.slab_sub, true);
  sched.gap_at = a.rb_gap_at;
  sched.gap = a.rb_gap;
  // XL: the x rows the row block reaches are staged in LDS and the gathers
  // read LDS, so the vector-memory pipe carries the value stream plus a few
  // 16-byte window loads instead of one gather per entry. The window is up
  // to 4 segments of consecutive rows (one per cluster of offsets: a narrow
  // band is one segment, a 3-D stencil three: -n^2 / -n..n / +n^2); offset k
  // of the row at lr in the block sits at s_xw[lr + woff[k]].
  extern __shared__ __attribute__((aligned(16))) double s_xw[];
  const int wlen = a.dia_wlen;
  for (int64_t j = sched.j0; j < sched.jcount; j += sched.jstep) {
    const int64_t rb0 = sched.rb(j) * kBlock;
    const int64_t row = rb0 + tid;
    const bool active = row < a.n;
    const int64_t rr = active ? row : a.n - 1;  // loads stay in bounds
    const W m = active ? (W)mask[rr] : (W)0;
    const EpiIn pin = epi_load<EPI>(a, rr);
    const int64_t xrow = a.xoff + rr;
    if constexpr (XL) {
      __syncthreads();  // the previous row block is done with the window
      // unrolled: constant indices into a.seg_* (a runtime index into the
      // kernel argument, once a prologue has written a.c0, puts the whole
      // SpmvArgs copy in scratch)
#pragma unroll
      for (int g = 0; g < SpmvArgs::kMaxSeg; ++g) {
        if (g >= a.nseg) break;
        // segment starts are even (host), xoff and rb0 too: 16-byte loads
        const int64_t src = a.xoff + rb0 + a.seg_lo[g];
        const int half = a.seg_len[g] >> 1;
        double2* d1 = reinterpret_cast<double2*>(s_xw + a.seg_base[g]);
        double2* d2 = reinterpret_cast<double2*>(s_xw + wlen + a.seg_base[g]);
        for (int t = tid; t < half; t += kBlock) {
          const int64_t xi = src + 2 * t;
          const double2 w1 = window_pair(x1, xi, a.xlen);
          if constexpr (VIRT) {  // r1 formed once per column, rounded as at every gather
            const double2 w2 = window_pair(x2, xi, a.xlen);
            const double2 w3 = window_pair(a.x3, xi, a.xlen);
            d1[t] = make_double2(virt_in<EPI>(a, w1.x, w2.x, w3.x),
                                 virt_in<EPI>(a, w1.y, w2.y, w3.y));
          } else {
            d1[t] = w1;
          }
          if constexpr (NV == 2) d2[t] = window_pair(x2, xi, a.xlen);
        }
      }
      __syncthreads();
    }
    const int lx = (int)(rr - rb0);  // own row in the block
    const double* dia_row = dia + (rr / kDiaRows) * a.dia_bs + (rr % kDiaRows);
    double sum1 = 0.0, sum2 = 0.0;
    // x of offset slot k at this row (window or gather) and the sum of one
    // entry, rounded as everywhere (product, then the add; absent: skipped)
    auto fetch_x = [&](int k, bool ok, double& p1, double& p2, double& p3) {
      if constexpr (XL) {
        const int lc = lx + load_uniform(a.woff, k);  // inside the window even if absent
        p1 = s_xw[lc];
        if constexpr (NV == 2) p2 = s_xw[wlen + lc];
      } else {
        const int64_t c = ok ? xrow + load_uniform(a.moff, k) : xrow;
        p1 = x1[c];
        if constexpr (NV == 2 || VIRT) p2 = x2[c];
        if constexpr (VIRT) p3 = a.x3[c];
      }
    };
    auto add_entry = [&](bool ok, double v, double p1, double p2, double p3) {
      if constexpr (VIRT && !XL) {
        const double t = sum1 + v * virt_in<EPI>(a, p1, p2, p3);
        sum1 = ok ? t : sum1;
      } else {
        const double t1 = sum1 + v * p1;
        sum1 = ok ? t1 : sum1;
        if constexpr (NV == 2) {
          const double t2 = sum2 + v * p2;
          sum2 = ok ? t2 : sum2;
        }
      }
    };
    if constexpr (SYMUP > 0) {
      const int h = nm / 2;  // lower slots 0..h-1, the diagonal h, upper h+1..nm-1
      double up[SYMUP];
#pragma unroll
      for (int u = 0; u < SYMUP; ++u) up[u] = dia_row[(int64_t)min(h + u, nm - 1) * a.dia_ks];
      for (int k0 = 0; k0 < h; k0 += CH) {
        double v[CH], p1[CH], p2[CH], p3[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int k = min(k0 + u, h - 1);
          const bool ok = k0 + u < h && ((m >> k) & 1);
          // lower entry k of row rr = upper entry nm-1-k of row rr + M[k]
          // (bitwise equal, checked at finalize); own copy before the launch's rows
          const int64_t jm = rr + load_uniform(a.moff, k);
          v[u] = ok && jm >= 0 ? dia[(jm / kDiaRows) * a.dia_bs +
                                     (int64_t)(nm - 1 - k) * a.dia_ks + jm % kDiaRows]
                               : dia_row[(int64_t)k * a.dia_ks];
          fetch_x(k, ok, p1[u], p2[u], p3[u]);
        }
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const bool ok = k0 + u < h && ((m >> min(k0 + u, h - 1)) & 1);
          add_entry(ok, v[u], p1[u], p2[u], p3[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < SYMUP; ++u) {
        const int k = min(h + u, nm - 1);
        const bool ok = h + u < nm && ((m >> k) & 1);
        double p1 = 0.0, p2 = 0.0, p3 = 0.0;
        fetch_x(k, ok, p1, p2, p3);
        add_entry(ok, up[u], p1, p2, p3);
      }
    } else {
      for (int k0 = 0; k0 < nm; k0 += CH) {
        double v[CH], p1[CH], p2[CH], p3[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int k = min(k0 + u, nm - 1);
          const bool ok = k0 + u < nm && ((m >> k) & 1);
          if (a.dia_sym) {  // mirrored lower entries in stored order (KR_DIA_SYMUP=0)
            const int64_t jm = rr + load_uniform(a.moff, k);
            v[u] = ok && 2 * k < nm - 1 && jm >= 0
                       ? dia[(jm / kDiaRows) * a.dia_bs + (int64_t)(nm - 1 - k) * a.dia_ks +
                             jm % kDiaRows]
                       : dia_row[(int64_t)k * a.dia_ks];
          } else {
            v[u] = __builtin_nontemporal_load(dia_row + (int64_t)k * a.dia_ks);
          }
          fetch_x(k, ok, p1[u], p2[u], p3[u]);
        }
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const bool ok = k0 + u < nm && ((m >> min(k0 + u, nm - 1)) & 1);
          add_entry(ok, v[u], p1[u], p2[u], p3[u]);
        }
      }
    }
    if (active) epi_row_in<EPI>(a, row, sum1, sum2, x1, x2, pin, acc);
  }
  __syncthreads();
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
}

template <int E, bool XL, int SYMUP>
void spmv_dia_launch_sym(const SpmvArgs& a, int nblocks, hipStream_t s) {
  const size_t lds = XL ? sizeof(double) * a.dia_wlen * EpiTraits<E>::NV : 0;  // virtual: NV 1
  switch (a.mw) {
    case 8: spmv_dia_kernel<E, 8, 8, XL, SYMUP><<<nblocks, kBlock, lds, s>>>(a); return;
    case 16: spmv_dia_kernel<E, 16, 8, XL, SYMUP><<<nblocks, kBlock, lds, s>>>(a); return;
    case 32: spmv_dia_kernel<E, 32, 8, XL, SYMUP><<<nblocks, kBlock, lds, s>>>(a); return;
    default: spmv_dia_kernel<E, 64, 8, XL, SYMUP><<<nblocks, kBlock, lds, s>>>(a); return;
  }
}

template <int E, bool XL>
void spmv_dia_launch_xl(const SpmvArgs& a, int nblocks, hipStream_t s) {
  // symmetric values: diagonal + upper slots = nm - nm/2 <= 16 or 32 registers
  // (KR_DIA_SYMUP=0: mirrored lower entries read in stored order instead)
  static const int upfirst = [] {
    const char* e = getenv("KR_DIA_SYMUP");
    return e ? atoi(e) : 1;
  }();
  if (a.dia_sym && upfirst && a.nm - a.nm / 2 <= 16)
    return spmv_dia_launch_sym<E, XL, 16>(a, nblocks, s);
  if (a.dia_sym && upfirst && a.nm - a.nm / 2 <= 32)
    return spmv_dia_launch_sym<E, XL, 32>(a, nblocks, s);
  spmv_dia_launch_sym<E, XL, 0>(a, nblocks, s);
}

template <int E>
void spmv_diawalk_launch(const SpmvArgs& a, int nblocks, hipStream_t s);

template <int E>
void spmv_dia_launch(const SpmvArgs& a, int nblocks, hipStream_t s) {
  if (a.dia_walk) return spmv_diawalk_launch<E>(a, nblocks, s);
  if (a.dia_wlen > 0) return spmv_dia_launch_xl<E, true>(a, nblocks, s);
  spmv_dia_launch_xl<E, false>(a, nblocks, s);
}

// ---------------------------------------------------------------------------
// Symmetric diagonal-offset SpMV as a row-block WALK (SpmvArgs::dia_walk:
// shards whose values are symmetric, dia_sym, and whose band is at most one
// row block wide, M[nm-1] <= 256: the banded systems C3 and C5).
//
// Workgroup g owns the consecutive virtual row blocks [g nvb / G, (g+1) nvb / G)
// (block g when nvb <= G) and walks them in order, one lane per row, rows
// summed in stored order from 0.0 (bitwise scipy, as every SpMV here). Only
// the diagonal and upper values are streamed from HBM (one non-temporal pass,
// 8 (h+1) bytes per row). The lower entry of row l at offset -o is the upper
// entry of row l - o (bitwise equal, dia_symcheck at finalize), which lies in
// this row block or the previous one, and both are in LDS, PRE-SHIFTED so
// that row l reads position l: lower slot k (offset -o, o = M[nm-1-k]) has a
// buffer s_low[k][256] in which the lane of row p stores its upper value of
// offset o at position (p + o) & 255 -- before the sums when p + o < 256
// (the reader is row p + o of this block), after them otherwise (the reader
// is row p + o - 256 of the next block). A segment start (or the boundary
// launch's gap) stores instead the block's OWN lower values (the same
// numbers) at positions l < o. The read is then one ds_read_b64 at the lane's
// own address with a compile-time offset: no index arithmetic per entry.
// x rows: a window of 768 rows per vector, rows rb0 - 256 .. rb0 + 511
// (band <= 256), shifted by one block per step inside each lane's own slots
// (lane t: win[t] <- win[t+256] <- win[t+512] <- the new row, loaded one block
// ahead), so the shift needs no barrier. One block ahead too: every lane's
// diagonal + upper values, its mask and its epilogue operands, so the next
// block's HBM stream is in flight while this block is summed.
// Rows whose mask is full in the whole workgroup (every block of a band
// matrix but its first and last) take a path without the absent-entry
// selects.
// LDS: 8 (256 h + 768 NV) bytes; the grid is the resident workgroup count
// (Shard::spmv_grid, dia_walk_grid). Round 2 read the mirrors from global
// memory (an L2 hit only when the neighbouring workgroup happened to stream
// them at the same moment): C5's dual moved 21.4 GB per launch against the
// 14.4 GB it must stream. First versions of this kernel were issue-bound
// (a scalar load per entry drains every LDS read in flight; wrapped ring
// indices cost 3 VALU per entry).
// ---------------------------------------------------------------------------
constexpr int kWalkWin = 768;  // x window, rows per vector (band <= 256)
#ifndef KR_DIAW_MODE
#define KR_DIAW_MODE 3
#endif
// Ablations for tools/micro/walk_micro (timing only, wrong sums; never in the
// library build): bit 0 no epilogue products / stores (the sums kept live),
// 1 no mirror stores, 2 no lower sums, 3 no window reads in the sums, 4 no
// full-block ballot, 5 no window shift.
#ifndef KR_DIAW_AB
#define KR_DIAW_AB 0
#endif

// NH = h, the number of upper (= lower) offsets, is a template parameter:
// every loop over the offsets is then straight-line code, so the compiler
// keeps up to 15 LDS reads in flight instead of waiting after each one
// behind a run-time bound (the runtime-h version ran at 3 TB/s on C5).
// (2 workgroups per CU for NH > 15: at most 256 VGPRs; the LDS allows no
// more anyway)
template <int EPI, int NH, bool PO = false>
__global__ __launch_bounds__(kBlock, NH > 15 ? 2 : 1) void spmv_diawalk_kernel(SpmvArgs a) {
  if (!spmv_entry<EPI>(a)) return;  // converged / the fused scalar step's test fired
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  constexpr bool VIRT = is_virtual<EPI>();
  constexpr int NM = 2 * NH + 1;
  constexpr int MW = NM <= 8 ? 8 : NM <= 16 ? 16 : NM <= 32 ? 32 : 64;
  using MT = typename MaskType<MW>::type;
  using W = typename std::conditional<(MW > 32), uint64_t, uint32_t>::type;
  constexpr W kFull = NM >= 64 ? ~(W)0 : (((W)1 << NM) - 1);
  __shared__ double s_red[(NP > 0 ? NP : 1) * 4];
  __shared__ int s_full[4];
  extern __shared__ __attribute__((aligned(16))) double s_dyn[];
  double* s_win = s_dyn;                          // NV x kWalkWin
  double* s_low = s_dyn + NV * kWalkWin;          // NH x kBlock, lower slot k at k * kBlock
  double* s_junk = s_low + NH * kBlock;           // kBlock: stores of lanes with nothing to store
  const MT* __restrict__ mask = static_cast<const MT*>(a.mask);
  const int tid = threadIdx.x;
  // The offset table, one entry per lane (lane k: M[k]); offset k is then a
  // readlane (VALU) -- no scalar memory load inside the block loop: an SMEM
  // result needs lgkmcnt(0), which would also drain every LDS read in flight.
  const int mlane = load_uniform(a.moff, min(tid & 63, NM - 1));
  auto moff = [&](int k) { return __builtin_amdgcn_readlane(mlane, k); };
  double acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) acc[p] = 0.0;

  const int64_t nvb = (a.n + kBlock - 1) / kBlock - a.rb_gap;
  const int64_t G = gridDim.x;
  // runs of consecutive blocks; with no more blocks than workgroups,
  // workgroup g takes block g (the strided kernels' assignment there)
  const int64_t gb = blockIdx.x;
  const int64_t v0 = nvb <= G ? min(gb, nvb) : gb * nvb / G;
  const int64_t v1 = nvb <= G ? min(gb + 1, nvb) : (gb + 1) * nvb / G;
  auto phys = [&](int64_t v) { return v < a.rb_gap_at ? v : v + a.rb_gap; };
  auto xload = [&](const double* __restrict__ x, int64_t xi) {
    return x[min(max(xi, (int64_t)0), a.xlen - 1)];
  };
  // The epilogue's own-row x1 / x2 (EpiIn::x, x2) are the window's middle
  // rows, written by this lane: read from LDS instead of loaded again (not
  // for virtual inputs, whose window holds the formed vector). Same values.
  // KR_DIAW_WINX=0 (compile time, A/B builds) loads them as the other kernels.
#ifndef KR_DIAW_WINX
#define KR_DIAW_WINX 1
#endif
  constexpr bool kWinX = KR_DIAW_WINX && !VIRT && (is_step<EPI>() || T::kX);
  static_assert(!(kWinX && T::kX2) || NV == 2, "x2 window for the own-row x2");
  // A virtual step's window holds the formed vector, but its own-row raw
  // x1 / x2 / x3 (r, y, Ar) are the rows this lane loaded for the window one
  // block earlier: kept in registers (own*) instead of loaded again.
  constexpr bool kOwnRaw = KR_DIAW_WINX && is_vstep<EPI>();
  constexpr int kNoX = kWinX ? 3 : kOwnRaw ? 7 : 0;
  auto xform = [&](double r1, double r2, double r3) {  // the window value of vector 0
    if constexpr (VIRT)
      return virt_in<EPI>(a, r1, r2, r3);
    else
      return r1;
  };
  // store v at s_low[slot][pos] when ok. KR_DIAW_MODE (compile time, A/B
  // builds): 0 = the other lanes store to a junk slot, every wave issues the
  // head and the tail store of every offset; 1 = junk slot, but a wave whose
  // rows all store the head (or all the tail) of an offset skips the other
  // store (rows wv0 .. wv0+63, wave-uniform tests); 2 = as 1 with
  // exec-masked stores instead of the junk slot; 3 (default) = ONE store per
  // offset and lane at the top of the block: position (p + o) & 255 takes the
  // previous block's value when p + o >= 256 (its tail, read by this block)
  // and this block's value otherwise (its head) -- the same position, so no
  // select of addresses, no junk slot, no branch (the walk micro put modes
  // 1's stores at 0.52 of the products-only dual's 2.72 ms: per offset a
  // readlane, a scalar test and branch and a generic-pointer select).
  auto low_put = [&](bool ok, int slot, int pos, double v) {
    if constexpr (KR_DIAW_MODE >= 2) {
      if (ok) s_low[slot * kBlock + pos] = v;
    } else {
      double* d = ok ? s_low + slot * kBlock + pos : s_junk + tid;
      *d = v;
    }
  };
  const int wv0 = __builtin_amdgcn_readfirstlane(tid & ~63);
  auto any_tail = [&](int o) { return KR_DIAW_MODE == 0 || wv0 + 63 + o >= kBlock; };
  auto any_head = [&](int o) { return KR_DIAW_MODE == 0 || wv0 + o < kBlock; };

  // one block ahead: values (diagonal + upper), mask, epilogue operands, the
  // window's new rows (raw loads; a virtual input is formed when stored)
  double upn[NH + 1];
  W mn = 0;
  EpiIn pinn;
  double xr1 = 0.0, xr2 = 0.0, xr3 = 0.0;
  auto prefetch = [&](int64_t bb) {
    const int64_t rowb = bb * kBlock + tid;
    const bool act = rowb < a.n;
    const int64_t rrb = act ? rowb : a.n - 1;
    if (bb >= a.full_lo && bb < a.full_hi)  // uniform: a whole, full block
      mn = kFull;
    else
      mn = act ? (W)mask[rrb] : (W)0;
    const double* blk = a.dia + bb * a.dia_bs + tid;
#pragma unroll
    for (int u = 0; u <= NH; ++u)
      upn[u] = __builtin_nontemporal_load(blk + (int64_t)(NH + u) * a.dia_ks);
    pinn = epi_load<EPI, kNoX>(a, rrb);
    const int64_t xi = a.xoff + bb * kBlock + kBlock + tid;
    xr1 = xload(a.x1, xi);
    if constexpr (NV == 2 || VIRT) xr2 = xload(a.x2, xi);
    if constexpr (VIRT && EPI != EPI_XY_VP) xr3 = xload(a.x3, xi);
  };

  double up[NH + 1];
#pragma unroll
  for (int u = 0; u <= NH; ++u) up[u] = 0.0;
  double own1 = 0.0, own2 = 0.0, own3 = 0.0;  // kOwnRaw: this block's row
  double nxt1 = 0.0, nxt2 = 0.0, nxt3 = 0.0;  // kOwnRaw: the next block's row
  if (v0 < v1) prefetch(phys(v0));
  int64_t prev = -2;
  for (int64_t v = v0; v < v1; ++v) {
    const int64_t b = phys(v);
    const bool start = b != prev + 1;  // uniform
    if constexpr (KR_DIAW_MODE == 3) {
      // the previous block's tails and this block's heads, one store each
      // (this block's values: the loads issued one block ago)
      if (!start && !(KR_DIAW_AB & 2)) {
#pragma unroll
        for (int u = 1; u <= NH; ++u) {
          const int pos = tid + moff(NH + u);
          const double val = pos >= kBlock ? up[u] : upn[u];
          s_low[(NH - u) * kBlock + (pos & (kBlock - 1))] = val;
        }
      }
    } else if (!start && !(KR_DIAW_AB & 2)) {
      // --- the previous block's tails (its rows p + o >= 256 feed this block)
#pragma unroll
      for (int u = 1; u <= NH; ++u) {
        const int o = moff(NH + u);
        if (any_tail(o)) low_put(tid + o >= kBlock, NH - u, tid + o - kBlock, up[u]);
      }
    }
    prev = b;
#pragma unroll
    for (int u = 0; u <= NH; ++u) up[u] = upn[u];
    const W m = mn;
    EpiIn pin = pinn;
    const double c1 = xr1, c2 = xr2, c3 = xr3;
    // the next block's loads (the last block re-reads itself: no branch, so
    // nothing below waits for them)
    prefetch(phys(min(v + 1, v1 - 1)));
    const int64_t rb0 = b * kBlock;
    const int64_t row = rb0 + tid;
    const bool active = row < a.n;
    // --- the x window and this block's heads
    if (start) {
      for (int t = tid; t < kWalkWin; t += kBlock) {  // rows rb0 - 256 + t
        const int64_t xi = a.xoff + rb0 - kBlock + t;
        double r1 = xload(a.x1, xi), r2 = 0.0, r3 = 0.0;
        if constexpr (NV == 2 || VIRT) r2 = xload(a.x2, xi);
        if constexpr (VIRT && EPI != EPI_XY_VP) r3 = xload(a.x3, xi);
        s_win[t] = xform(r1, r2, r3);
        if constexpr (NV == 2) s_win[kWalkWin + t] = r2;
        if constexpr (kOwnRaw) {
          if (t == tid + kBlock) {
            own1 = r1, own2 = r2, own3 = r3;
          } else if (t == tid + 2 * kBlock) {
            nxt1 = r1, nxt2 = r2, nxt3 = r3;
          }
        }
      }
      // positions l < o: the block's own lower values (all loads, then the stores)
      const double* blk = a.dia + b * a.dia_bs + tid;
      double lw[NH];
#pragma unroll
      for (int k = 0; k < NH; ++k) lw[k] = blk[(int64_t)k * a.dia_ks];
#pragma unroll
      for (int k = 0; k < NH; ++k) low_put(tid < -moff(k), k, tid, lw[k]);
    } else if (!(KR_DIAW_AB & 32)) {  // shift by one block inside the lane's own slots, append the new row
#pragma unroll
      for (int vv = 0; vv < NV; ++vv) {
        double* w = s_win + vv * kWalkWin + tid;
        const double w1 = w[kBlock], w2 = w[2 * kBlock];
        w[0] = w1;
        w[kBlock] = w2;
      }
      s_win[2 * kBlock + tid] = xform(c1, c2, c3);
      if constexpr (NV == 2) s_win[kWalkWin + 2 * kBlock + tid] = c2;
      if constexpr (kOwnRaw) {
        own1 = nxt1, own2 = nxt2, own3 = nxt3;
        nxt1 = c1, nxt2 = c2, nxt3 = c3;
      }
    }
    if (KR_DIAW_MODE != 3 || start) {
#pragma unroll
      for (int u = 1; u <= NH; ++u) {  // heads: rows p + o < 256 of this block
        const int o = moff(NH + u);
        if (!(KR_DIAW_AB & 2) && any_head(o)) low_put(tid + o < kBlock, NH - u, tid + o, up[u]);
      }
    }
    bool full = true;
    if constexpr (KR_DIAW_AB & 16) {
      __syncthreads();
    } else {
      const bool lane_full = active && m == kFull;
      const uint64_t all = __ballot(lane_full);
      if ((tid & 63) == 0) s_full[tid >> 6] = all == ~0ull ? 1 : 0;
      __syncthreads();
      full = (s_full[0] & s_full[1] & s_full[2] & s_full[3]) != 0;  // uniform
    }
    // --- the row sums: lower entries (mirrors from LDS), diagonal, upper
    double sum1 = 0.0, sum2 = 0.0;
    const double* wl = s_win + kBlock + tid;  // the row's x: wl[offset]
    const double* ll = s_low + tid;           // lower slot k: ll[k * kBlock]
    if (full) {
      if constexpr (!(KR_DIAW_AB & 4)) {
#pragma unroll
        for (int k = 0; k < NH; ++k) {
          const double* w = wl + moff(k);
          const double v = ll[k * kBlock];
          if constexpr (KR_DIAW_AB & 8) {
            sum1 = sum1 + v * 1.5;
            if constexpr (NV == 2) sum2 = sum2 + v * 0.5;
          } else {
            sum1 = sum1 + v * w[0];
            if constexpr (NV == 2) sum2 = sum2 + v * w[kWalkWin];
          }
        }
      }
#pragma unroll
      for (int u = 0; u <= NH; ++u) {
        const double* w = wl + moff(NH + u);
        if constexpr (KR_DIAW_AB & 8) {
          sum1 = sum1 + up[u] * 1.5;
          if constexpr (NV == 2) sum2 = sum2 + up[u] * 0.5;
        } else {
          sum1 = sum1 + up[u] * w[0];
          if constexpr (NV == 2) sum2 = sum2 + up[u] * w[kWalkWin];
        }
      }
    } else {  // absent entries skipped by a select, as every kernel here
      auto add = [&](int k, double v) {
        const bool ok = ((m >> k) & 1) != 0;
        const double* w = wl + moff(k);
        const double t1 = sum1 + v * w[0];
        sum1 = ok ? t1 : sum1;
        if constexpr (NV == 2) {
          const double t2 = sum2 + v * w[kWalkWin];
          sum2 = ok ? t2 : sum2;
        }
      };
#pragma unroll
      for (int k = 0; k < NH; ++k) add(k, ll[k * kBlock]);
#pragma unroll
      for (int u = 0; u <= NH; ++u) add(NH + u, up[u]);
    }
    if constexpr (kWinX) {
      pin.x = wl[0];
      if constexpr (T::kX2) pin.x2 = wl[kWalkWin];
    } else if constexpr (kOwnRaw) {
      pin.x = own1;
      pin.x2 = own2;
      pin.e = own3;
    }
    if constexpr (KR_DIAW_AB & 1)
      acc[0] = acc[0] + sum1 * sum2;
    else if (active)
      epi_row_in<EPI, PO ? 1 : 0>(a, row, sum1, sum2, a.x1, a.x2, pin, acc);
    __syncthreads();
  }
  __syncthreads();
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
}

// LDS of the walk kernel (dia_walk_grid on the host): the mirror buffers, the
// junk slots and the x windows of the epilogue's vectors
template <int E, int NH>
void spmv_diawalk_launch_t(const SpmvArgs& a, int nblocks, hipStream_t s) {
  constexpr int nv = EpiTraits<E>::NV;
  const size_t lds = sizeof(double) * ((size_t)(NH + 1) * kBlock + (size_t)nv * kWalkWin);
  // products-only duals: their own kernel (the storing one never tests
  // SpmvArgs::products_only)
  constexpr bool kPo = EpiTraits<E>::NV == 2 && !is_step<E>();
  if (kPo && a.products_only) {
    static std::atomic<uint64_t> opted{0};  // per device (opt_in_lds)
    if (lds > 64 * 1024)
      opt_in_lds(opted, reinterpret_cast<const void*>(spmv_diawalk_kernel<E, NH, kPo>), lds);
    spmv_diawalk_kernel<E, NH, kPo><<<nblocks, kBlock, lds, s>>>(a);
    return;
  }
  static std::atomic<uint64_t> opted{0};
  if (lds > 64 * 1024)
    opt_in_lds(opted, reinterpret_cast<const void*>(spmv_diawalk_kernel<E, NH>), lds);
  spmv_diawalk_kernel<E, NH><<<nblocks, kBlock, lds, s>>>(a);
}

template <int E>
void spmv_diawalk_launch(const SpmvArgs& a, int nblocks, hipStream_t s) {
  KR_REQUIRE(a.dia_sym && a.nm % 2 == 1 && dia_walk_h_supported(a.nm / 2),
             "walk SpMV: symmetric offsets with a compiled upper-slot count");
  switch (a.nm / 2) {
    case 7: return spmv_diawalk_launch_t<E, 7>(a, nblocks, s);
    case 13: return spmv_diawalk_launch_t<E, 13>(a, nblocks, s);
    case 15: return spmv_diawalk_launch_t<E, 15>(a, nblocks, s);
    default: return spmv_diawalk_launch_t<E, 31>(a, nblocks, s);
  }
}

// Which kernel serves a shard that has diagonal-offset values (long rows by
// default, every masked shard with KR_DIA=2): the DIA kernel for every
// epilogue when the x window fits in LDS; without a window, the row walk v2
// for short-row multi-vector SpMVs (dual, fused first step), where it measured
// faster (512^3 dual 2.77 vs 2.82 ms, first step 3.93 vs 4.20 ms).
// KR_DIA_ALL=1 routes those to the diagonal-offset kernel too (A/B).
template <int E>
bool use_dia(const SpmvArgs& a) {
  if (!a.dia) return false;
  if (a.dia_wlen > 0) return true;  // x window in LDS: every epilogue
  // (EPI_XY_VP routes as EPI_XY: the same kernel, so the same summation order)
  constexpr bool multi = EpiTraits<E>::NV == 2 || E == EPI_STEP_MRR_FIRST2;
  if (!multi || a.long_rows) return true;
  const bool vec = ((reinterpret_cast<uintptr_t>(a.val) | reinterpret_cast<uintptr_t>(a.col)) &
                    15) == 0;
  if (!vec || a.nnz_total < 4) return true;
  return KR_ENV("KR_DIA_ALL", 0) == 1;
}

// ---------------------------------------------------------------------------
// Dense row block (the reference's np.ndarray A branch, v3/gpu/common.py:100-101
// and v3/gpu/mpi/common.py:124-125, where cupy runs a cuBLAS dgemv). One wave
// per row: lane l accumulates columns l, l+64, ... in order (8 independent
// 512-byte loads in flight per lane), then a fixed shuffle tree reduces the
// 64 partial sums -- deterministic, not sequential: dense parity is within
// rounding, as the reference's own dgemv order differs from numpy's. The
// epilogues (products, fused steps) are the SpMV's, applied by lane 0.
// ---------------------------------------------------------------------------
template <int EPI>
__global__ __launch_bounds__(kBlock) void gemv_kernel(SpmvArgs a) {
  if (a.stop && *a.stop != 0.0) return;  // converged (device-resident scalars)
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  constexpr int U = 8;
  __shared__ double s_red[(NP > 0 ? NP : 1) * 4];
  double acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) acc[p] = 0.0;
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (kBlock / 64);
  const double* __restrict__ xf1 = a.x1 + a.xcol0;
  const double* __restrict__ xf2 = NV == 2 ? a.x2 + a.xcol0 : nullptr;
  const int64_t nc = a.ncols;
  for (int64_t row = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); row < a.n;
       row += waves) {
    const double* __restrict__ ar = a.val + row * a.dld;
    double s1 = 0.0, s2 = 0.0;
    int64_t c = lane;
    for (; c + 64 * (U - 1) < nc; c += 64 * U) {
      double av[U], p1[U], p2[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        av[u] = __builtin_nontemporal_load(ar + c + 64 * u);
        p1[u] = xf1[c + 64 * u];
        if constexpr (NV == 2) p2[u] = xf2[c + 64 * u];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        s1 = s1 + av[u] * p1[u];
        if constexpr (NV == 2) s2 = s2 + av[u] * p2[u];
      }
    }
    for (; c < nc; c += 64) {
      const double av = ar[c];
      s1 = s1 + av * xf1[c];
      if constexpr (NV == 2) s2 = s2 + av * xf2[c];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      s1 += __shfl_down(s1, off, 64);
      if constexpr (NV == 2) s2 += __shfl_down(s2, off, 64);
    }
    if (lane == 0) {
      const double* xo1 = a.x1;  // own-row operands use the halo-extended base
      const double* xo2 = a.x2;
      epi_row_in<EPI>(a, row, s1, s2, xo1, xo2, epi_load<EPI>(a, row), acc);
    }
  }
  __syncthreads();
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
}

// The offset-mask row walk (SpmvArgs::mask); false if not applicable.
template <typename RP, int E, bool VEC>
bool spmv_masked(const SpmvArgs& a, dim3 grid, dim3 block, hipStream_t s) {
  if constexpr (VEC) {
    switch (a.mw) {
      case 8: spmv_kernel<RP, E, VEC, kGather, true, false, 8><<<grid, block, 0, s>>>(a); return true;
      case 16: spmv_kernel<RP, E, VEC, kGather, true, false, 16><<<grid, block, 0, s>>>(a); return true;
      case 32: spmv_kernel<RP, E, VEC, kGather, true, false, 32><<<grid, block, 0, s>>>(a); return true;
      case 64: spmv_kernel<RP, E, VEC, kGather, true, false, 64><<<grid, block, 0, s>>>(a); return true;
      default: return false;
    }
  }
  return false;
}

template <typename RP, bool VEC, int E>
void spmv_dispatch_epi(const SpmvArgs& a, int nblocks, hipStream_t s) {
  const dim3 grid(nblocks), block(kBlock);
  // Short rows: row walk v2 with a non-temporal matrix stream (13). Long rows
  // (SpmvArgs::long_rows): product-then-sum v2 (14; C3 +5 %). KR_SPMV_VARIANT
  // overrides for A/B runs: 0 row walk v1, 8 product-then-sum v1, 10 row
  // walk v2 with plain loads, 12 row walk v2 single-buffered, 15
  // product-then-sum v2 with plain loads.
  const int forced = KR_ENV("KR_SPMV_VARIANT", -1);
  // Two-vector long-row SpMVs stay on v1: v2's extra gather registers cost a
  // wave per SIMD there (144 VGPRs) and it measured 7 % slower (C5 dual).
  // short rows: v2 with the non-temporal matrix stream and result stores on
  // large shards (13), plain loads and stores on small ones (10), whose
  // vectors the next kernel finds in L2 / MALL (C1: +2.4 %)
  int variant = forced >= 0 ? forced
                            : (a.long_rows ? (EpiTraits<E>::NV == 1 ? 14 : 8) : a.nt_stores ? 13 : 10);
  // the v2 kernels need 16-byte aligned bases and >= 4 entries
  if (variant >= 10 && (!VEC || a.nnz_total < 4)) variant = a.long_rows ? 8 : 0;
  if constexpr (is_virtual<E>()) {  // implemented by the row walk v2 only
    if (!VEC || a.nnz_total < 4 || a.dense)
      throw Failure(KR_ERR_INVALID, "fused first step needs the row walk v2");
    if (a.nt_stores)
      spmv2_launch<RP, E, VEC, true, true>(a, grid, block, s);
    else
      spmv2_launch<RP, E, VEC, true, false>(a, grid, block, s);
    return;
  } else {
    if constexpr (VEC) {
      switch (variant) {
        case 10: spmv2_launch<RP, E, VEC>(a, grid, block, s); return;
        case 12: spmv2_launch<RP, E, VEC, false>(a, grid, block, s); return;
        case 13: spmv2_launch<RP, E, VEC, true, true>(a, grid, block, s); return;
        case 14:  // one vector: 4 slots, double-buffered; two: 2 slots
          spmv_kernel_prod2<RP, E, true, true, EpiTraits<E>::NV == 1 ? 4 : 2>
              <<<grid, block, 0, s>>>(a);
          return;
        case 15:
          spmv_kernel_prod2<RP, E, true, false, EpiTraits<E>::NV == 1 ? 4 : 2>
              <<<grid, block, 0, s>>>(a);
          return;
        case 16:  // A/B: two vectors with 4 slots, single-buffered (144 VGPRs)
          spmv_kernel_prod2<RP, E, EpiTraits<E>::NV == 1, true, 4><<<grid, block, 0, s>>>(a);
          return;
        default: break;
      }
    }
    if (variant == 8) {
      spmv_kernel_prod<RP, E, VEC><<<grid, block, 0, s>>>(a);
      return;
    }
    if (!(a.mask && spmv_masked<RP, E, VEC>(a, grid, block, s)))
      spmv_kernel<RP, E, VEC><<<grid, block, 0, s>>>(a);
  }
}

#include "kr_stencil.h"

}  // namespace

// One epilogue's launcher: explicitly instantiated, one epilogue per object
// file (kr_spmv_inst.hip, -DKR_EPI=<n>), so the kernel variants build in
// parallel.
template <int E>
void spmv_launch_epi(const SpmvArgs& a, int nblocks, hipStream_t s) {
  if (a.scode) {  // stencil codes (kr_stencil.h): 3-D stencils with a value dictionary
    // the walk needs whole (XCD, position) columns; the boundary launch
    // (row-block gap, block-strided) takes any grid
    KR_REQUIRE(a.rb_gap > 0 || (a.st_pm ? a.st_P % 8 == 0 && nblocks % a.st_P == 0
                                        : nblocks % (8 * a.st_P) == 0),
               "stencil SpMV: grid must be a multiple of P (position-major) or 8 * P");
    spmv_stencil_launch<E>(a, nblocks, s);
    return;
  }
  if (use_dia<E>(a)) {
    spmv_dia_launch<E>(a, nblocks, s);
    return;
  }
  if (a.dense) {
    if constexpr (is_virtual<E>())
      throw Failure(KR_ERR_INVALID, "fused first step has no dense kernel");
    else
      gemv_kernel<E><<<nblocks, kBlock, 0, s>>>(a);
    return;
  }
  // 16-byte staging needs 16-byte aligned val/col bases
  const bool vec = ((reinterpret_cast<uintptr_t>(a.val) | reinterpret_cast<uintptr_t>(a.col)) &
                    15) == 0;
  if (a.rowptr64) {
    if (vec)
      spmv_dispatch_epi<int64_t, true, E>(a, nblocks, s);
    else
      spmv_dispatch_epi<int64_t, false, E>(a, nblocks, s);
  } else {
    if (vec)
      spmv_dispatch_epi<int32_t, true, E>(a, nblocks, s);
    else
      spmv_dispatch_epi<int32_t, false, E>(a, nblocks, s);
  }
}

}  // namespace kr
