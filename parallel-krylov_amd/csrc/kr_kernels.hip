// CDNA4 (gfx950) kernels for the Krylov inner loop.
//
// Numerics contract: this file is compiled with
// -ffp-contract=off, so every `a*b + c` below rounds the product and the sum
// separately, exactly like the numpy statements of the reference
// (v3/cpu/*.py, v3/gpu/*.py). SpMV rows are summed by one lane, sequentially,
// in stored order, starting from 0.0 -- the order of scipy's csr_matvec -- so
// y = A x is bitwise equal to scipy. Dot products use a fixed two-stage tree
// (per-block partials, then kr::launch_finalize), so they are deterministic
// run to run, but they are not OpenBLAS's order.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "kr_hash.h"
#include "kr_internal.h"
#include "kr_spmv.h"

namespace kr {

// SpMV kernels are instantiated per epilogue in kr_spmv_inst.hip.
extern template void spmv_launch_epi<EPI_NONE>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_BMINUS>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_XY>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_HEAD_MRR>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_HEAD_KCG>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_MRR_LOOP>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_DUAL_NONE>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_DUAL_MRR>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_DUAL_KCG>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_STEP_MRR_NOX>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_STEP_MRR_X2>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_STEP_MRR_X>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_STEP_KCG>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_STEP_MRR_FIRST2>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_MRR_V>(const SpmvArgs&, int, hipStream_t);
extern template void spmv_launch_epi<EPI_XY_VP>(const SpmvArgs&, int, hipStream_t);

namespace {

// ---------------------------------------------------------------------------
// Elementwise vector steps. Operand slots p[0..5]; READ/WRITE masks say which
// slots are loaded and stored. Pairs of doubles move as one 16-byte access.
// ---------------------------------------------------------------------------
template <int OP>
struct EwTraits;
template <>
struct EwTraits<EW_DOT> {
  static constexpr int NP = 1, R = 0b000011, W = 0;
};
template <>
struct EwTraits<EW_MRR_FIRST> {  // p: y ar1 z r xs xd
  static constexpr int NP = 0, R = 0b011010, W = 0b101101;
};
template <>
struct EwTraits<EW_MRR> {
  static constexpr int NP = 0, R = 0b011111, W = 0b101101;
};
template <>
struct EwTraits<EW_CG> {  // p: x p r v
  static constexpr int NP = 1, R = 0b001111, W = 0b000101;
};
template <>
struct EwTraits<EW_CG_P> {  // p: p r
  static constexpr int NP = 0, R = 0b000011, W = 0b000001;
};
template <>
struct EwTraits<EW_KCG> {  // p: x ap0 r ap1
  static constexpr int NP = 0, R = 0b001111, W = 0b000111;
};
template <>
struct EwTraits<EW_MRR_S> {  // p: ar y r
  static constexpr int NP = 2, R = 0b000111, W = 0;
};
template <>
struct EwTraits<EW_COPY> {  // p: dst src
  static constexpr int NP = 0, R = 0b000010, W = 0b000001;
};
template <>
struct EwTraits<EW_MRR_NOX> {  // p: y ar1 z r
  static constexpr int NP = 0, R = 0b001111, W = 0b001101;
};
template <>
struct EwTraits<EW_MRR_X2> {  // p: y ar1 z r xs xd
  static constexpr int NP = 0, R = 0b011111, W = 0b101101;
};
template <>
struct EwTraits<EW_CG_NOX> {  // p: x p r v
  static constexpr int NP = 1, R = 0b01100, W = 0b00100;
};
template <>
struct EwTraits<EW_CG_X2> {  // p: x p r v pp
  static constexpr int NP = 1, R = 0b11111, W = 0b00101;
};
template <>
struct EwTraits<EW_AXPY> {  // p: x p
  static constexpr int NP = 0, R = 0b11, W = 0b01;
};
// Preconditioned / pipelined CG family (v1/threads/pipeline/*.py restated,
// DESIGN.md §5b): Jacobi M^-1 v = v / d.
template <>
struct EwTraits<EW_ONE> {  // p: d
  static constexpr int NP = 0, R = 0, W = 0b1;
};
template <>
struct EwTraits<EW_PRE> {  // p: r u d
  static constexpr int NP = 2, R = 0b101, W = 0b010;
};
template <>
struct EwTraits<EW_PCG> {  // p: x p r s u d
  static constexpr int NP = 2, R = 0b101111, W = 0b010101;
};
template <>
struct EwTraits<EW_CGG> {  // p: p u s w x r d
  static constexpr int NP = 2, R = 0b1111111, W = 0b0110111;
};
template <>
struct EwTraits<EW_GROPP1> {  // p: x p r s u d
  static constexpr int NP = 2, R = 0b111111, W = 0b010101;
};
template <>
struct EwTraits<EW_GROPP2> {  // p: p u s w
  static constexpr int NP = 1, R = 0b1111, W = 0b0101;
};
template <>
struct EwTraits<EW_DIV> {  // p: m w d
  static constexpr int NP = 0, R = 0b110, W = 0b001;
};
template <>
struct EwTraits<EW_PIPE> {  // p: z n q m s w p u x r
  static constexpr int NP = 3, R = 0b1111111111, W = 0b1111110101;
};

template <int OP>
__device__ __forceinline__ void ew_elem(double c0, double c1, double (&v)[kEwOps],
                                        double (&acc)[EwTraits<OP>::NP > 0
                                                          ? EwTraits<OP>::NP
                                                          : 1]) {
  if constexpr (OP == EW_DOT) {
    acc[0] += v[0] * v[1];
  } else if constexpr (OP == EW_MRR_FIRST) {  // c1 = zeta
    const double y = c1 * v[1];
    const double z = (-c1) * v[3];
    v[0] = y;
    v[2] = z;
    v[3] = v[3] - y;
    v[5] = v[4] - z;
  } else if constexpr (OP == EW_MRR) {  // c0 = eta, c1 = zeta
    const double t1 = c0 * v[0];
    const double t2 = c1 * v[1];
    const double y = t1 + t2;
    const double t3 = c0 * v[2];
    const double t4 = c1 * v[3];
    const double z = t3 - t4;
    v[0] = y;
    v[2] = z;
    v[3] = v[3] - y;
    v[5] = v[4] - z;
  } else if constexpr (OP == EW_CG) {  // c0 = alpha
    const double ap = c0 * v[1];
    const double av = c0 * v[3];
    v[0] = v[0] + ap;
    v[2] = v[2] - av;
    acc[0] += v[2] * v[2];
  } else if constexpr (OP == EW_CG_NOX) {  // c0 = alpha; x += alpha p deferred
    const double av = c0 * v[3];
    v[2] = v[2] - av;
    acc[0] += v[2] * v[2];
  } else if constexpr (OP == EW_CG_X2) {  // c0 = alpha, c1 = the previous step's alpha
    const double app = c1 * v[4];
    const double xm = v[0] + app;  // the deferred x += alpha_prev p_prev
    const double ap = c0 * v[1];
    v[0] = xm + ap;
    const double av = c0 * v[3];
    v[2] = v[2] - av;
    acc[0] += v[2] * v[2];
  } else if constexpr (OP == EW_AXPY) {  // c0 = alpha
    const double ap = c0 * v[1];
    v[0] = v[0] + ap;
  } else if constexpr (OP == EW_CG_P) {  // c0 = beta
    const double bp = c0 * v[0];
    v[0] = v[1] + bp;
  } else if constexpr (OP == EW_KCG) {  // c0 = alpha, c1 = beta
    const double a0 = c0 * v[1];
    const double a1 = c0 * v[3];
    v[0] = v[0] + a0;
    v[2] = v[2] - a1;
    const double bp = c1 * v[1];
    v[1] = v[2] + bp;
  } else if constexpr (OP == EW_MRR_S) {  // c0 = gamma
    const double gy = c0 * v[1];
    const double s = v[0] - gy;
    acc[0] += v[2] * s;
    acc[1] += s * s;
  } else if constexpr (OP == EW_COPY) {
    v[0] = v[1];
  } else if constexpr (OP == EW_MRR_NOX || OP == EW_MRR_X2) {  // c0 = eta, c1 = zeta
    const double t1 = c0 * v[0];
    const double t2 = c1 * v[1];
    const double y = t1 + t2;
    const double t3 = c0 * v[2];
    const double t4 = c1 * v[3];
    const double z = t3 - t4;
    if constexpr (OP == EW_MRR_X2) {
      const double xm = v[4] - v[2];  // the deferred x -= z of the previous step
      v[5] = xm - z;
    }
    v[0] = y;
    v[2] = z;
    v[3] = v[3] - y;
  } else if constexpr (OP == EW_ONE) {
    v[0] = 1.0;
  } else if constexpr (OP == EW_PRE) {  // u = ilu.solve(r)  (pcg.py:27)
    const double u = v[0] / v[2];
    v[1] = u;
    acc[0] += v[0] * v[0];
    acc[1] += v[0] * u;
  } else if constexpr (OP == EW_PCG) {  // c0 = alpha  (pcg.py:34-43)
    const double ap = c0 * v[1];
    v[0] = v[0] + ap;
    const double as = c0 * v[3];
    const double r = v[2] - as;
    const double u = r / v[5];
    v[2] = r;
    v[4] = u;
    acc[0] += r * r;
    acc[1] += r * u;
  } else if constexpr (OP == EW_CGG) {  // c0 = alpha, c1 = beta  (chronopoulos_gear.py:37-47)
    const double bp = c1 * v[0];
    const double p = v[1] + bp;
    const double bs = c1 * v[2];
    const double sv = v[3] + bs;
    const double ap = c0 * p;
    v[4] = v[4] + ap;
    const double as = c0 * sv;
    const double r = v[5] - as;
    const double u = r / v[6];
    v[0] = p;
    v[2] = sv;
    v[5] = r;
    v[1] = u;
    acc[0] += r * r;
    acc[1] += r * u;
  } else if constexpr (OP == EW_GROPP1) {  // c0 = alpha  (gropp.py:29-39)
    const double q = v[3] / v[5];
    const double ap = c0 * v[1];
    v[0] = v[0] + ap;
    const double as = c0 * v[3];
    const double r = v[2] - as;
    const double aq = c0 * q;
    const double u = v[4] - aq;
    v[2] = r;
    v[4] = u;
    acc[0] += r * r;
    acc[1] += r * u;
  } else if constexpr (OP == EW_GROPP2) {  // c0 = beta  (gropp.py:43-44, 28)
    const double bp = c0 * v[0];
    const double p = v[1] + bp;
    const double bs = c0 * v[2];
    const double sv = v[3] + bs;
    v[0] = p;
    v[2] = sv;
    acc[0] += p * sv;
  } else if constexpr (OP == EW_DIV) {  // m = ilu.solve(w)
    v[0] = v[1] / v[2];
  } else if constexpr (OP == EW_PIPE) {  // c0 = alpha, c1 = beta  (pipeline.py:43-55)
    const double bz = c1 * v[0];
    const double z = v[1] + bz;
    const double bq = c1 * v[2];
    const double q = v[3] + bq;
    const double bs = c1 * v[4];
    const double sv = v[5] + bs;
    const double bp = c1 * v[6];
    const double p = v[7] + bp;
    const double ap = c0 * p;
    v[8] = v[8] + ap;
    const double as = c0 * sv;
    const double r = v[9] - as;
    const double aq = c0 * q;
    const double u = v[7] - aq;
    const double az = c0 * z;
    const double w = v[5] - az;
    v[0] = z;
    v[2] = q;
    v[4] = sv;
    v[5] = w;
    v[6] = p;
    v[7] = u;
    v[9] = r;
    acc[0] += r * r;
    acc[1] += r * u;
    acc[2] += w * u;
  }
}

__device__ double block_slot_sum(const double* __restrict__ part, int cnt, double* s_red);

// The scalar_kernel statement a.pro - 1 run by a whole workgroup of the
// vector kernel that consumes it (EwArgs::pro): the same sums (0.0 + the
// finalize order), the same IEEE statements, so the coefficients are
// bitwise the scalar kernel's. Returns false when the convergence test fired
// (the workgroup then skips its vector work, as the separate vector kernel
// skipped itself on st[ST_STOP]). Only workgroup 0 writes the state; no
// workgroup reads a state entry this launch writes (CG's gamma alternates).
__device__ bool ew_prologue(const EwArgs& a, double* s_red, double& c0, double& c1) {
  double* st = a.st;
  const bool w0 = blockIdx.x == 0 && threadIdx.x == 0;
  auto slot = [&](int q) {
    return 0.0 + block_slot_sum(a.pro_part + (int64_t)q * a.pro_stride, a.pro_cnt[q], s_red);
  };
  auto converged = [&](double g) { return a.pro_check && g >= 0.0 && g < a.pro_thr; };
  c1 = 0.0;
  switch (a.pro - 1) {
    case SC_CG_ALPHA: {  // alpha = gamma / sigma  (v3/gpu/cg.py:33)
      const double sigma = slot(a.pro_s1);
      c0 = st[gamma_slot(a.pro_par)] / sigma;
      if (a.pro_alpha == 1 && w0) st[ST_ALPHA] = c0;  // the deferred x step's alpha
      if (a.pro_alpha == 2) c1 = st[ST_ALPHA];
      return true;
    }
    case SC_CG_BETA: {  // beta = gnew / gamma; gamma = gnew  (v3/gpu/cg.py:36-38)
      const double gnew = slot(0);
      c0 = gnew / st[gamma_slot(a.pro_par)];
      const bool conv = converged(gnew);
      if (w0) {
        st[ST_HIST + a.pro_h] = gnew;
        st[gamma_slot(a.pro_par ^ 1)] = gnew;
        if (conv) {  // the test at the top of the next iteration
          st[ST_STOP_AT] = (double)(a.pro_it + 1);
          st[ST_STOP] = 1.0;
        }
      }
      return !conv;
    }
    case SC_MRR_GAMMA: {  // <r,r>, mu, nu -> test; gamma = nu / mu  (v3/gpu/mrr.py:40-46)
      const double rr = slot(0), mu = slot(1), nu = slot(2);
      const bool conv = converged(rr);
      c0 = nu / mu;
      if (w0) {
        st[ST_HIST + a.pro_h] = rr;
        if (conv) {
          st[ST_STOP_AT] = (double)a.pro_it;
          st[ST_STOP] = 1.0;
        } else {
          st[ST_GAMMA] = c0;
        }
      }
      return !conv;
    }
    case SC_MRR_ZETA: {  // zeta = <r,s>/<s,s>; eta = -zeta * gamma  (v3/gpu/mrr.py:47-49)
      const double rs = slot(3), ss = slot(4);
      const double zeta = rs / ss;
      c0 = (-zeta) * st[ST_GAMMA];
      c1 = zeta;
      return true;
    }
  }
  return true;
}

template <int OP, bool VEC, int U = 1, bool NTS = false>
__global__ __launch_bounds__(kBlock) void ew_kernel(EwArgs a) {
  using T = EwTraits<OP>;
  constexpr int NP = T::NP;
  __shared__ double s_red[(NP > 0 ? NP : 1) * 4];
  // Device-resident scalars (CG/MrR without a host sync): stop once the
  // convergence test fired; coefficients from the scalar kernel's output.
  if (a.stop && *a.stop != 0.0) return;
  double c0 = a.cdev ? a.cdev[0] : a.c0;
  double c1 = a.cdev ? a.cdev[1] : a.c1;
  double acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) acc[p] = 0.0;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t t0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if constexpr (VEC) {
    // U pairs per thread per iteration: all loads of the U pairs are issued
    // before any store (the operands may alias, so the compiler cannot hoist
    // the next iteration's loads above this iteration's stores by itself).
    const int64_t npairs = a.n >> 1;
    double va[U][kEwOps], vb[U][kEwOps];
    auto load = [&](int64_t q0) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t q = q0 + u * stride;
#pragma unroll
        for (int k = 0; k < kEwOps; ++k) {
          if ((T::R & (1 << k)) && q < npairs) {
            const double2 d = reinterpret_cast<const double2*>(a.p[k])[q];
            va[u][k] = d.x;
            vb[u][k] = d.y;
          } else {
            va[u][k] = vb[u][k] = 0.0;
          }
        }
      }
    };
    // The first pairs' operands do not depend on the fused scalar step, so
    // they are in flight while the prologue sums the partials (one memory
    // latency instead of two; the small systems are latency-bound).
    // KR_EW_PREFETCH=0 (a.pro_pre = 0): after it (A/B).
    if (a.pro && a.pro_pre) load(t0);
    if (a.pro && !ew_prologue(a, s_red, c0, c1)) return;
    for (int64_t q0 = t0; q0 < npairs; q0 += U * stride) {
      if (!(a.pro && a.pro_pre) || q0 != t0) load(q0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t q = q0 + u * stride;
        if (q >= npairs) break;
        ew_elem<OP>(c0, c1, va[u], acc);
        ew_elem<OP>(c0, c1, vb[u], acc);
#pragma unroll
        for (int k = 0; k < kEwOps; ++k)
          if (T::W & (1 << k)) {
            double2* dst = reinterpret_cast<double2*>(a.p[k]) + q;
            if constexpr (NTS) {
              typedef double dv2 __attribute__((ext_vector_type(2)));
              __builtin_nontemporal_store(dv2{va[u][k], vb[u][k]}, reinterpret_cast<dv2*>(dst));
            } else {
              *dst = make_double2(va[u][k], vb[u][k]);
            }
          }
      }
    }
    if ((a.n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
      const int64_t i = a.n - 1;
      double v[kEwOps];
#pragma unroll
      for (int k = 0; k < kEwOps; ++k) v[k] = (T::R & (1 << k)) ? a.p[k][i] : 0.0;
      ew_elem<OP>(c0, c1, v, acc);
#pragma unroll
      for (int k = 0; k < kEwOps; ++k)
        if (T::W & (1 << k)) a.p[k][i] = v[k];
    }
  } else {
    if (a.pro && !ew_prologue(a, s_red, c0, c1)) return;
    for (int64_t i = t0; i < a.n; i += stride) {
      double v[kEwOps];
#pragma unroll
      for (int k = 0; k < kEwOps; ++k) v[k] = (T::R & (1 << k)) ? a.p[k][i] : 0.0;
      ew_elem<OP>(c0, c1, v, acc);
#pragma unroll
      for (int k = 0; k < kEwOps; ++k)
        if (T::W & (1 << k)) a.p[k][i] = v[k];
    }
  }
  block_reduce_store<NP>(acc, a.partials, a.stride > 0 ? a.stride : a.grid, s_red);
}

template <int OP>
void ew_dispatch_op(const EwArgs& a, hipStream_t s) {
  bool aligned = true;
  for (int k = 0; k < kEwOps; ++k)
    if (((EwTraits<OP>::R | EwTraits<OP>::W) & (1 << k)) &&
        (reinterpret_cast<uintptr_t>(a.p[k]) & 15))
      aligned = false;
  // KR_EW_VARIANT (A/B only): 0 = 1 pair/thread/iteration, 1 = 2 pairs,
  // 2 = 2 pairs + non-temporal stores.
  const int variant = KR_ENV("KR_EW_VARIANT", 0);
  if (!aligned)
    ew_kernel<OP, false><<<a.grid, kBlock, 0, s>>>(a);
  else if (variant == 1)
    ew_kernel<OP, true, 2><<<a.grid, kBlock, 0, s>>>(a);
  else if (variant == 2)
    ew_kernel<OP, true, 2, true><<<a.grid, kBlock, 0, s>>>(a);
  else
    ew_kernel<OP, true><<<a.grid, kBlock, 0, s>>>(a);
}

// ---------------------------------------------------------------------------
// Fixed-order final reduction: one workgroup per slot.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void finalize_kernel(const double* __restrict__ part,
                                                          int grid, double* __restrict__ out) {
  __shared__ double s_red[4];
  const int slot = blockIdx.x;
  double t = 0.0;
  for (int i = threadIdx.x; i < grid; i += kBlock) t += part[(int64_t)slot * grid + i];
  for (int off = 32; off > 0; off >>= 1) t += __shfl_down(t, off, 64);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = s_red[0];
    r = r + s_red[1];
    r = r + s_red[2];
    r = r + s_red[3];
    out[slot] = r;
  }
}

// Sum of the `cnt` partials of one slot in the fixed order of the finalize
// kernels (lane-strided, shuffle tree, then waves 0..3). Called by the whole
// workgroup; every thread gets the result.
__device__ double block_slot_sum(const double* __restrict__ part, int cnt, double* s_red) {
  return slot_sum(part, cnt, s_red);  // kr_spmv.h
}

// As finalize_kernel, with a per-slot partial count (same fixed order).
__global__ __launch_bounds__(kBlock) void finalize_counts_kernel(const double* __restrict__ part,
                                                                 int stride, SlotCounts c,
                                                                 double* __restrict__ out) {
  __shared__ double s_red[4];
  const int slot = blockIdx.x;
  const double r = block_slot_sum(part + (int64_t)slot * stride, c.n[slot], s_red);
  if (threadIdx.x == 0) out[slot] = r;
}

__global__ __launch_bounds__(kBlock) void finalize_group_kernel(FinalizeGroup g, int stride,
                                                                SlotCounts c, double* out,
                                                                int out_stride) {
  __shared__ double s_red[4];
  const int slot = blockIdx.x, j = blockIdx.y;
  const double r = block_slot_sum(g.part[j] + (int64_t)slot * stride, c.n[slot], s_red);
  if (threadIdx.x == 0) out[(int64_t)j * out_stride + slot] = r;
}

// ---------------------------------------------------------------------------
// Device-resident CG / MrR scalars (one workgroup): the reductions of one
// sync point, summed exactly like finalize_counts + the host's shard sum
// (0.0 + total), then the scalar statements of the reference, then the
// convergence test `sqrt(g)/||b|| < tol` as the equivalent `0 <= g < thr`
// (thr precomputed on the host, see conv_threshold). State in st[ST_*].
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void scalar_kernel(ScalarArgs a) {
  __shared__ double s_red[4];
  double* st = a.st;
  if (st[ST_STOP] != 0.0) return;
  double v[5];
  if (a.gathered) {  // ranks' totals in rank order, as System::reduce sums them
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      double t = 0.0;
      if ((a.need >> q) & 1)
        for (int r = 0; r < a.nranks; ++r) t = t + a.gathered[(int64_t)r * a.gstride + q];
      v[q] = t;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 5; ++q)
      v[q] = (a.need >> q) & 1
                 ? 0.0 + block_slot_sum(a.partials + (int64_t)q * a.stride, a.cnt[q], s_red)
                 : 0.0;
  }
  if (threadIdx.x != 0) return;
  auto converged = [&](double g) {
    return a.check && g >= 0.0 && g < a.thr;
  };
  switch (a.op) {
    case SC_CG_ALPHA:  // alpha = gamma / sigma  (v3/gpu/cg.py:33)
      st[ST_C0] = st[ST_GAMMA] / v[1];
      st[ST_C1] = 0.0;
      break;
    case SC_CG_BETA: {  // beta = gnew / gamma; gamma = gnew  (v3/gpu/cg.py:36-38)
      const double gnew = v[0];
      st[ST_HIST + a.h] = gnew;
      st[ST_C2] = gnew / st[ST_GAMMA];
      st[ST_C3] = 0.0;
      st[ST_GAMMA] = gnew;
      if (converged(gnew)) {  // the test at the top of the next iteration
        st[ST_STOP_AT] = (double)(a.it + 1);
        st[ST_STOP] = 1.0;
      }
      break;
    }
    case SC_MRR_GAMMA: {  // <r,r>, mu, nu -> test; gamma = nu / mu  (v3/gpu/mrr.py:40-46)
      st[ST_HIST + a.h] = v[0];
      if (converged(v[0])) {
        st[ST_STOP_AT] = (double)a.it;
        st[ST_STOP] = 1.0;
        break;
      }
      st[ST_GAMMA] = v[2] / v[1];
      st[ST_C0] = st[ST_GAMMA];
      st[ST_C1] = 0.0;
      break;
    }
    case SC_MRR_ZETA: {  // zeta = <r,s>/<s,s>; eta = -zeta * gamma  (v3/gpu/mrr.py:47-49)
      const double zeta = v[3] / v[4];
      st[ST_C2] = (-zeta) * st[ST_GAMMA];
      st[ST_C3] = zeta;
      break;
    }
  }
}



// ---------------------------------------------------------------------------
// Multi-dot (test/composition primitive), up to 16 products per launch.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void multidot_kernel(MultiDotArgs a, int base) {
  constexpr int NP = 16;
  __shared__ double s_red[NP * 4];
  double acc[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) acc[p] = 0.0;
  const int cnt = min(NP, a.count - base);
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < a.n; i += stride) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
      if (p < cnt) acc[p] += a.u[base + p][i] * a.v[base + p][i];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    double v = acc[p];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if (lane == 0) s_red[p * 4 + wave] = v;
  }
  __syncthreads();
  if (threadIdx.x < cnt) {
    const double* r = s_red + threadIdx.x * 4;
    double t = r[0];
    t = t + r[1];
    t = t + r[2];
    t = t + r[3];
    a.partials[(int64_t)(base + threadIdx.x) * a.grid + blockIdx.x] = t;
  }
}

// ---------------------------------------------------------------------------
// Generators.
// ---------------------------------------------------------------------------
template <typename RP>
// Grid side^(dim-1) x nz (nz = side: the cube of the reference's Poisson).
__global__ void poisson_count_kernel(int dim, int64_t side, int64_t nz, int64_t row0, int64_t n,
                                     RP* rowptr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t g = row0 + i;
  int cnt = 1;
  for (int d = 0; d < dim; ++d) {
    const int64_t sz = d == dim - 1 ? nz : side;
    const int64_t c = g % sz;
    g /= sz;
    cnt += (c > 0) + (c < sz - 1);
  }
  rowptr[i + 1] = (RP)cnt;
}

template <typename RP>
__global__ void poisson_fill_kernel(int dim, int64_t side, int64_t nz, int64_t row0, int64_t n,
                                    const RP* rowptr, int32_t* col, double* val) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t g = row0 + i;
  int64_t coord[3] = {0, 0, 0};
  int64_t stride[3] = {1, side, side * side};
  int64_t size[3] = {side, side, side};
  size[dim - 1] = nz;
  int64_t t = g;
  for (int d = 0; d < dim; ++d) {
    coord[d] = t % size[d];
    t /= size[d];
  }
  int64_t j = (int64_t)rowptr[i];
  // Sorted column order: outermost lower neighbours first.
  for (int d = dim - 1; d >= 0; --d)
    if (coord[d] > 0) {
      col[j] = (int32_t)(g - stride[d]);
      val[j] = -1.0;
      ++j;
    }
  col[j] = (int32_t)g;
  val[j] = 2.0 * dim;
  ++j;
  for (int d = 0; d < dim; ++d)
    if (coord[d] < size[d] - 1) {
      col[j] = (int32_t)(g + stride[d]);
      val[j] = -1.0;
      ++j;
    }
}

template <typename RP>
__global__ void banded_count_kernel(BandSpec b, int64_t row0, int64_t n, RP* rowptr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t g = row0 + i;
  int cnt = 1;
  for (int t = 0; t < b.h; ++t) cnt += (g - b.off[t] >= 0) + (g + b.off[t] < b.n_global);
  rowptr[i + 1] = (RP)cnt;
}

template <typename RP>
__global__ void banded_fill_kernel(BandSpec b, int64_t row0, int64_t n, const RP* rowptr,
                                   int32_t* col, double* val) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t g = row0 + i;
  // Diagonal = (sum of |off| in column order) + 1.
  double s = 0.0;
  for (int t = b.h - 1; t >= 0; --t)
    if (g - b.off[t] >= 0) s = s + fabs(band_value(b.seed, g - b.off[t], b.off[t]));
  for (int t = 0; t < b.h; ++t)
    if (g + b.off[t] < b.n_global) s = s + fabs(band_value(b.seed, g, b.off[t]));
  int64_t j = (int64_t)rowptr[i];
  for (int t = b.h - 1; t >= 0; --t)
    if (g - b.off[t] >= 0) {
      col[j] = (int32_t)(g - b.off[t]);
      val[j] = band_value(b.seed, g - b.off[t], b.off[t]);
      ++j;
    }
  col[j] = (int32_t)g;
  val[j] = s + 1.0;
  ++j;
  for (int t = 0; t < b.h; ++t)
    if (g + b.off[t] < b.n_global) {
      col[j] = (int32_t)(g + b.off[t]);
      val[j] = band_value(b.seed, g, b.off[t]);
      ++j;
    }
}

__global__ void fill_rhs_kernel(uint64_t seed, int64_t row0, int64_t n, double* b) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = rhs_value(seed, (uint64_t)(row0 + i));
}

template <typename RP>
__global__ void col_minmax_kernel(const RP* rowptr, int64_t n, const int32_t* col,
                                  unsigned long long* out) {
  __shared__ int64_t s_min[kBlock], s_max[kBlock];
  const int64_t base = (int64_t)rowptr[0];
  const int64_t nnz = (int64_t)rowptr[n] - base;
  int64_t mn = INT64_MAX, mx = -1;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nnz;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = col[base + j];
    mn = c < mn ? c : mn;
    mx = c > mx ? c : mx;
  }
  s_min[threadIdx.x] = mn;
  s_max[threadIdx.x] = mx;
  __syncthreads();
  for (int off = kBlock / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      s_min[threadIdx.x] = min(s_min[threadIdx.x], s_min[threadIdx.x + off]);
      s_max[threadIdx.x] = max(s_max[threadIdx.x], s_max[threadIdx.x + off]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    atomicMin(&out[0], (unsigned long long)s_min[0]);
    if (s_max[0] >= 0) atomicMax(&out[1], (unsigned long long)s_max[0]);
  }
}

// Interior rows of a shard: out[0] = 1 + the last row with a column below
// [lo, hi], out[1] = the first row with a column above it (global columns).
// out[2] = the column reach max |col - row| (global row = lo + local row).
template <typename RP>
__global__ void interior_kernel(const RP* rowptr, int64_t n, const int32_t* col, int64_t lo,
                                int64_t hi, unsigned long long* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool below = false, above = false;
  int64_t reach = 0;
  for (int64_t j = (int64_t)rowptr[i]; j < (int64_t)rowptr[i + 1]; ++j) {
    below |= col[j] < lo;
    above |= col[j] > hi;
    const int64_t d = (int64_t)col[j] - (lo + i);
    reach = max(reach, d < 0 ? -d : d);
  }
  if (below) atomicMax(&out[0], (unsigned long long)(i + 1));
  if (above) atomicMin(&out[1], (unsigned long long)i);
  if (reach > 0) atomicMax(&out[2], (unsigned long long)reach);
}

// Offset-mask detection. The distinct offsets col - (base + row) of a block
// go into a small open-addressing table (key = offset + 2^32, 0 = empty);
// flags bit 0: a row whose columns are not strictly increasing, bit 1: table
// full.
constexpr int kOffTable = 256;

template <typename RP>
__global__ void offsets_kernel(const RP* rowptr, int64_t n, const int32_t* col, int64_t base,
                               unsigned long long* table, int* flags) {
  int bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    int64_t prev = INT64_MIN;
    for (int64_t j = (int64_t)rowptr[i]; j < (int64_t)rowptr[i + 1]; ++j) {
      const int64_t off = (int64_t)col[j] - (base + i);
      if (off <= prev) bad |= 1;
      prev = off;
      const unsigned long long key = (unsigned long long)(off + (1ll << 32));
      unsigned h = (unsigned)((key * 0x9E3779B97F4A7C15ull) >> 56) & (kOffTable - 1);
      int probe = 0;
      for (; probe < kOffTable; ++probe) {
        const unsigned long long v = __atomic_load_n(&table[h], __ATOMIC_RELAXED);
        if (v == key) break;
        if (v == 0) {
          const unsigned long long old = atomicCAS(&table[h], 0ull, key);
          if (old == 0 || old == key) break;
        }
        h = (h + 1) & (kOffTable - 1);
      }
      if (probe == kOffTable) bad |= 2;
    }
  }
  if (bad) atomicOr(flags, bad);
}

template <typename RP, typename MT>
__global__ void mask_kernel(const RP* rowptr, int64_t n, const int32_t* col, int64_t base,
                            const int32_t* M, int nm, MT* mask) {
  __shared__ int32_t sM[64];
  if ((int)threadIdx.x < nm) sM[threadIdx.x] = M[threadIdx.x];
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    MT m = 0;
    for (int64_t j = (int64_t)rowptr[i]; j < (int64_t)rowptr[i + 1]; ++j) {
      const int64_t off = (int64_t)col[j] - (base + i);
      int b = 0;
      while (b < nm - 1 && sM[b] != off) ++b;
      m |= (MT)((MT)1 << b);
    }
    mask[i] = m;
  }
}

template <typename RP>
__global__ void dia_fill_kernel(const RP* rowptr, int64_t n, const int32_t* col,
                                const double* val, int64_t base, const int32_t* M, int nm,
                                double* dia, int64_t bs, int64_t ks) {
  __shared__ int32_t sM[64];
  if ((int)threadIdx.x < nm) sM[threadIdx.x] = M[threadIdx.x];
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double* di = dia + (i / kDiaRows) * bs + (i % kDiaRows);
    for (int64_t j = (int64_t)rowptr[i]; j < (int64_t)rowptr[i + 1]; ++j) {
      const int64_t off = (int64_t)col[j] - (base + i);
      int b = 0;
      while (b < nm - 1 && sM[b] != off) ++b;
      di[(int64_t)b * ks] = val[j];
    }
  }
}

// Stencil codes (SpmvArgs::scode): byte k of out[i] = the dictionary code of
// row i's entry at offset M[k], 0xFF where the row has none.
template <typename RP>
__global__ void stencil_codes_kernel(const RP* rowptr, int64_t n, const int32_t* col,
                                     const uint8_t* vcode, int64_t base, const int32_t* M,
                                     int nm, uint64_t* out) {
  __shared__ int32_t sM[8];
  if ((int)threadIdx.x < nm) sM[threadIdx.x] = M[threadIdx.x];
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t w = ~0ull;
    for (int64_t j = (int64_t)rowptr[i]; j < (int64_t)rowptr[i + 1]; ++j) {
      const int64_t off = (int64_t)col[j] - (base + i);
      int b = 0;
      while (b < nm - 1 && sM[b] != off) ++b;
      w &= ~(0xFFull << (8 * b));
      w |= (uint64_t)vcode[j] << (8 * b);
    }
    out[i] = w;
  }
}

// Narrow stencil codes (launch_stencil_pack).
template <int CB>
__global__ void stencil_pack_kernel(const uint64_t* __restrict__ in, int64_t n, void* out) {
  constexpr uint32_t m = (1u << CB) - 1u;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t w = in[i];
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t c = (uint32_t)(w >> (8 * k)) & 0xFFu;
      o |= (c == 0xFFu ? m : c) << (CB * k);
    }
    if constexpr (CB == 2)
      static_cast<uint16_t*>(out)[i] = (uint16_t)o;
    else
      static_cast<uint32_t*>(out)[i] = o;
  }
}

template <typename RP>
__global__ void col_shift_kernel(const RP* rowptr, int64_t n, int32_t* col, int64_t delta) {
  const int64_t base = (int64_t)rowptr[0];
  const int64_t nnz = (int64_t)rowptr[n] - base;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nnz;
       j += (int64_t)gridDim.x * blockDim.x)
    col[base + j] = (int32_t)((int64_t)col[base + j] + delta);
}

inline unsigned blocks_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
int spmv_products(SpmvEpi epi) {
  switch (epi) {
    case EPI_NONE: return EpiTraits<EPI_NONE>::NP;
    case EPI_BMINUS: return EpiTraits<EPI_BMINUS>::NP;
    case EPI_XY: return EpiTraits<EPI_XY>::NP;
    case EPI_HEAD_MRR: return EpiTraits<EPI_HEAD_MRR>::NP;
    case EPI_HEAD_KCG: return EpiTraits<EPI_HEAD_KCG>::NP;
    case EPI_MRR_LOOP: return EpiTraits<EPI_MRR_LOOP>::NP;
    case EPI_DUAL_NONE: return EpiTraits<EPI_DUAL_NONE>::NP;
    case EPI_DUAL_MRR: return EpiTraits<EPI_DUAL_MRR>::NP;
    case EPI_DUAL_KCG: return EpiTraits<EPI_DUAL_KCG>::NP;
    case EPI_STEP_MRR_NOX:
    case EPI_STEP_MRR_X2:
    case EPI_STEP_MRR_X:
    case EPI_STEP_KCG:
    case EPI_STEP_MRR_FIRST2: return 0;
    case EPI_XY_VP: return EpiTraits<EPI_XY_VP>::NP;
    case EPI_MRR_V: return EpiTraits<EPI_MRR_V>::NP;
  }
  return 0;
}

void launch_spmv_stencil2t(SpmvEpi epi, const SpmvArgs& a, int nblocks, hipStream_t s) {
  KR_REQUIRE(epi == EPI_DUAL_MRR || epi == EPI_DUAL_KCG, "tiled pair: dual epilogues only");
  if (epi == EPI_DUAL_MRR)
    launch_spmv_stencil2t_mrr(a, nblocks, s);
  else
    launch_spmv_stencil2t_kcg(a, nblocks, s);
}

void launch_spmv(SpmvEpi epi, const SpmvArgs& a, hipStream_t s) {
  launch_spmv_grid(epi, a, a.grid, s);
}

void launch_spmv_grid(SpmvEpi epi, const SpmvArgs& a, int nblocks, hipStream_t s) {
  KR_REQUIRE(a.grid > 0 && nblocks > 0 && nblocks <= a.grid,
             "spmv: need 0 < blocks <= partial stride");
  switch (epi) {
#define KR_CASE(E) \
  case E: spmv_launch_epi<E>(a, nblocks, s); break;
    KR_CASE(EPI_NONE)
    KR_CASE(EPI_BMINUS)
    KR_CASE(EPI_XY)
    KR_CASE(EPI_HEAD_MRR)
    KR_CASE(EPI_HEAD_KCG)
    KR_CASE(EPI_MRR_LOOP)
    KR_CASE(EPI_DUAL_NONE)
    KR_CASE(EPI_DUAL_MRR)
    KR_CASE(EPI_DUAL_KCG)
    KR_CASE(EPI_STEP_MRR_NOX)
    KR_CASE(EPI_STEP_MRR_X2)
    KR_CASE(EPI_STEP_MRR_X)
    KR_CASE(EPI_STEP_KCG)
    KR_CASE(EPI_STEP_MRR_FIRST2)
    KR_CASE(EPI_XY_VP)
    KR_CASE(EPI_MRR_V)
#undef KR_CASE
    default:
      throw Failure(KR_ERR_INVALID, "unknown SpMV epilogue");
  }
  KR_HIP_CHECK(hipGetLastError());
}

int ew_products(EwOp op) {
  switch (op) {
    case EW_DOT: return EwTraits<EW_DOT>::NP;
    case EW_MRR_FIRST: return EwTraits<EW_MRR_FIRST>::NP;
    case EW_MRR: return EwTraits<EW_MRR>::NP;
    case EW_CG: return EwTraits<EW_CG>::NP;
    case EW_CG_P: return EwTraits<EW_CG_P>::NP;
    case EW_KCG: return EwTraits<EW_KCG>::NP;
    case EW_MRR_S: return EwTraits<EW_MRR_S>::NP;
    case EW_COPY: return EwTraits<EW_COPY>::NP;
    case EW_MRR_NOX: return EwTraits<EW_MRR_NOX>::NP;
    case EW_MRR_X2: return EwTraits<EW_MRR_X2>::NP;
    case EW_CG_NOX: return EwTraits<EW_CG_NOX>::NP;
    case EW_CG_X2: return EwTraits<EW_CG_X2>::NP;
    case EW_AXPY: return EwTraits<EW_AXPY>::NP;
    case EW_ONE: return EwTraits<EW_ONE>::NP;
    case EW_PRE: return EwTraits<EW_PRE>::NP;
    case EW_PCG: return EwTraits<EW_PCG>::NP;
    case EW_CGG: return EwTraits<EW_CGG>::NP;
    case EW_GROPP1: return EwTraits<EW_GROPP1>::NP;
    case EW_GROPP2: return EwTraits<EW_GROPP2>::NP;
    case EW_DIV: return EwTraits<EW_DIV>::NP;
    case EW_PIPE: return EwTraits<EW_PIPE>::NP;
  }
  return 0;
}

void launch_ew(EwOp op, const EwArgs& a, hipStream_t s) {
  KR_REQUIRE(a.grid > 0, "elementwise: grid must be positive");
  switch (op) {
    case EW_DOT: ew_dispatch_op<EW_DOT>(a, s); break;
    case EW_MRR_FIRST: ew_dispatch_op<EW_MRR_FIRST>(a, s); break;
    case EW_MRR: ew_dispatch_op<EW_MRR>(a, s); break;
    case EW_CG: ew_dispatch_op<EW_CG>(a, s); break;
    case EW_CG_P: ew_dispatch_op<EW_CG_P>(a, s); break;
    case EW_KCG: ew_dispatch_op<EW_KCG>(a, s); break;
    case EW_MRR_S: ew_dispatch_op<EW_MRR_S>(a, s); break;
    case EW_COPY: ew_dispatch_op<EW_COPY>(a, s); break;
    case EW_MRR_NOX: ew_dispatch_op<EW_MRR_NOX>(a, s); break;
    case EW_MRR_X2: ew_dispatch_op<EW_MRR_X2>(a, s); break;
    case EW_CG_NOX: ew_dispatch_op<EW_CG_NOX>(a, s); break;
    case EW_CG_X2: ew_dispatch_op<EW_CG_X2>(a, s); break;
    case EW_AXPY: ew_dispatch_op<EW_AXPY>(a, s); break;
    case EW_ONE: ew_dispatch_op<EW_ONE>(a, s); break;
    case EW_PRE: ew_dispatch_op<EW_PRE>(a, s); break;
    case EW_PCG: ew_dispatch_op<EW_PCG>(a, s); break;
    case EW_CGG: ew_dispatch_op<EW_CGG>(a, s); break;
    case EW_GROPP1: ew_dispatch_op<EW_GROPP1>(a, s); break;
    case EW_GROPP2: ew_dispatch_op<EW_GROPP2>(a, s); break;
    case EW_DIV: ew_dispatch_op<EW_DIV>(a, s); break;
    case EW_PIPE: ew_dispatch_op<EW_PIPE>(a, s); break;
    default: throw Failure(KR_ERR_INVALID, "unknown elementwise op");
  }
  KR_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Persistent CG (CgPersistArgs). One workgroup per CU at most, each owning a
// contiguous range of rows (one lane per row, strided); every iteration is
// two phases separated by grid barriers:
//   A: v = A p (p formed at every gathered column as r + beta p_old from the
//      previous iteration, rounded as EW_CG_P, own rows stored to the other
//      p buffer), partial <p,v>;            barrier
//      sigma = the partials summed in a fixed order by every workgroup alike;
//   B: x += alpha p; r -= alpha v (rounded as EW_CG), partial <r,r>; barrier
//      gnew summed alike -> beta, the convergence test (every workgroup takes
//      the same branch), state written by workgroup 0.
// Rows are summed in stored order from 0.0 (bitwise scipy's y, as every SpMV
// here). The barrier is a device-scope counter: release fence + atomic add,
// then acquire polling until every workgroup of this phase arrived; a wait
// that exceeds ~1 s sets *err and gives up, so the grid always drains.
namespace {

// Returns false once any workgroup has timed out (*err set): the caller
// returns at once, so after one stuck barrier every workgroup leaves at its
// next barrier instead of spinning out its own timeout on every later one.
// x and r are then undefined (the host raises; kr_solve_* reports the error).
__device__ __forceinline__ bool grid_barrier(unsigned* bar, unsigned target, int* err) {
  __shared__ int s_fail;
  __syncthreads();
  if (threadIdx.x == 0) {
    // release once (write back this XCD's dirty L2 lines), arrive, poll with
    // relaxed device-scope loads (they bypass the non-coherent L2 without
    // invalidating it on every poll), then acquire once
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int fail = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (!fail && __hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 25)) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        fail = 1;
      } else if ((spins & 255u) == 0) {  // another workgroup gave up
        fail = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    s_fail = fail;
  }
  __syncthreads();
  return s_fail == 0;
}

template <typename RP>
__global__ __launch_bounds__(kBlock) void cg_persist_kernel(CgPersistArgs a) {
  __shared__ double s_red[4];
  const int G = gridDim.x;
  const int64_t per = (a.n + G - 1) / G;
  const int64_t lo = min(a.n, (int64_t)blockIdx.x * per);
  const int64_t hi = min(a.n, lo + per);
  const RP* __restrict__ rowptr = static_cast<const RP*>(a.rowptr);
  const int32_t* __restrict__ col = a.col;
  const double* __restrict__ val = a.val;
  double* x = a.x;
  double* r = a.r;
  double* v = a.v;
  double* pc = a.pa;  // p of this iteration (complete at j = 0)
  double* pn = a.pb;  // p of the next one (j > 0: formed in phase A)
  double gamma = a.gamma, beta = 0.0;
  unsigned target = 0;
  for (int j = 0; j < a.m; ++j) {
    // phase A: v = A p ; <p,v>
    double acc[1] = {0.0};
    for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
      const int64_t e = (int64_t)rowptr[i + 1];
      double sum = 0.0;
      for (int64_t k = (int64_t)rowptr[i]; k < e; ++k) {
        const int64_t c = col[k];
        const double pv = j == 0 ? pc[c] : virtual_p(beta, pc[c], r[c]);
        const double t = val[k] * pv;
        sum = sum + t;
      }
      const int64_t o = a.pad + i;
      const double po = j == 0 ? pc[o] : virtual_p(beta, pc[o], r[o]);
      if (j > 0) pn[o] = po;
      v[o] = sum;
      acc[0] += po * sum;
    }
    block_reduce_store<1>(acc, a.part, G, s_red);
    target += G;
    if (!grid_barrier(a.bar, target, a.err)) return;
    const double sigma = 0.0 + slot_sum(a.part, G, s_red);
    const double alpha = gamma / sigma;
    if (j > 0) {
      double* t = pc;
      pc = pn;
      pn = t;
    }
    // phase B: x += alpha p ; r -= alpha v ; <r,r>
    acc[0] = 0.0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
      const int64_t o = a.pad + i;
      const double ap = alpha * pc[o];
      const double av = alpha * v[o];
      x[o] = x[o] + ap;
      const double rn = r[o] - av;
      r[o] = rn;
      acc[0] += rn * rn;
    }
    block_reduce_store<1>(acc, a.part + G, G, s_red);
    target += G;
    if (!grid_barrier(a.bar, target, a.err)) return;
    const double gnew = 0.0 + slot_sum(a.part + G, G, s_red);
    beta = gnew / gamma;
    gamma = gnew;
    const bool conv = gnew >= 0.0 && gnew < a.thr;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      a.st[ST_HIST + j] = gnew;
      if (conv) {  // the test at the top of the next iteration
        a.st[ST_STOP_AT] = (double)(a.it0 + j + 1);
        a.st[ST_STOP] = 1.0;
      }
    }
    if (conv) return;
  }
  // the last iteration's p = r + beta p, own rows, in place
  for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
    const int64_t o = a.pad + i;
    pc[o] = virtual_p(beta, pc[o], r[o]);
  }
}

}  // namespace

int cg_persist_grid(int64_t n) {
  int dev = 0, cus = 0, coop = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev) != hipSuccess)
    return 0;
  if (!coop || cus <= 0) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu, reinterpret_cast<const void*>(cg_persist_kernel<int32_t>), kBlock, 0) !=
          hipSuccess ||
      per_cu < 1)
    return 0;
  const int64_t need = std::max<int64_t>(1, (n + kBlock - 1) / kBlock);
  return (int)std::min<int64_t>(need, cus);
}

void launch_cg_persist(const CgPersistArgs& a, int grid, hipStream_t s) {
  KR_REQUIRE(grid > 0 && a.m > 0 && a.m <= kScalarBatch, "persistent CG: bad launch shape");
  CgPersistArgs arg = a;
  void* params[] = {&arg};
  const void* fn = a.rowptr64 ? reinterpret_cast<const void*>(cg_persist_kernel<int64_t>)
                              : reinterpret_cast<const void*>(cg_persist_kernel<int32_t>);
  KR_HIP_CHECK(hipLaunchCooperativeKernel(fn, dim3(grid), dim3(kBlock), params, 0, s));
}

void launch_finalize(const double* partials, int grid, int nslots, double* out,
                     hipStream_t s) {
  if (nslots <= 0) return;
  finalize_kernel<<<nslots, kBlock, 0, s>>>(partials, grid, out);
  KR_HIP_CHECK(hipGetLastError());
}

__global__ void sqrt_kernel(double* p) {
  if (threadIdx.x == 0) p[0] = sqrt(p[0]);
}

void launch_sqrt(double* p, hipStream_t s) {
  sqrt_kernel<<<1, 64, 0, s>>>(p);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_scalar(const ScalarArgs& a, hipStream_t s) {
  scalar_kernel<<<1, kBlock, 0, s>>>(a);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_finalize_counts(const double* partials, int stride, const SlotCounts& counts,
                            int nslots, double* out, hipStream_t s) {
  if (nslots <= 0) return;
  KR_REQUIRE(nslots <= kFinalizeSlots, "too many reduction slots");
  finalize_counts_kernel<<<nslots, kBlock, 0, s>>>(partials, stride, counts, out);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_finalize_group(const FinalizeGroup& g, int stride, const SlotCounts& counts,
                           int nslots, double* out, int out_stride, hipStream_t s) {
  if (nslots <= 0 || g.n <= 0) return;
  KR_REQUIRE(nslots <= kFinalizeSlots && g.n <= kGroupMax && out_stride >= nslots,
             "grouped finalize: bad sizes");
  finalize_group_kernel<<<dim3((unsigned)nslots, (unsigned)g.n), kBlock, 0, s>>>(
      g, stride, counts, out, out_stride);
  KR_HIP_CHECK(hipGetLastError());
}

namespace {
// blockIdx.y = piece; each workgroup copies kHaloChunk doubles of it (a
// plain copy: the values are moved, never combined, so the halo is bitwise
// the peer's rows as with hipMemcpyAsync).
constexpr int kHaloChunk = 8 * kBlock;
__global__ __launch_bounds__(kBlock) void halo_gather_kernel(HaloGatherArgs a) {
  const int q = blockIdx.y;
  const int64_t cnt = a.count[q];
  const double* __restrict__ src = a.src[q];
  double* __restrict__ dst = a.dst[q];
  const int64_t base = (int64_t)blockIdx.x * kHaloChunk;
  if (base >= cnt) return;
#pragma unroll
  for (int j = 0; j < kHaloChunk / kBlock; ++j) {
    const int64_t i = base + j * kBlock + threadIdx.x;
    if (i < cnt) dst[i] = src[i];
  }
}
}  // namespace

void launch_halo_gather(const HaloGatherArgs& a, hipStream_t s) {
  KR_REQUIRE(a.n >= 0 && a.n <= kHaloPieces, "halo gather: bad piece count");
  if (a.n == 0) return;
  int64_t most = 0;
  for (int q = 0; q < a.n; ++q) most = std::max(most, a.count[q]);
  if (most == 0) return;
  const int64_t gx = (most + kHaloChunk - 1) / kHaloChunk;
  KR_REQUIRE(gx < ((int64_t)1 << 31), "halo gather: piece too long");
  halo_gather_kernel<<<dim3((unsigned)gx, (unsigned)a.n), kBlock, 0, s>>>(a);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_multidot(const MultiDotArgs& a, hipStream_t s) {
  KR_REQUIRE(a.count >= 0 && a.count <= 64, "multidot: count must be in [0, 64]");
  for (int base = 0; base < a.count; base += 16) {
    multidot_kernel<<<a.grid, kBlock, 0, s>>>(a, base);
    KR_HIP_CHECK(hipGetLastError());
  }
}

void launch_poisson_count(int dim, int64_t side, int64_t nz, int64_t row0, int64_t n,
                          void* rowptr, int rowptr64, hipStream_t s) {
  if (n <= 0) return;
  if (rowptr64)
    poisson_count_kernel<int64_t><<<blocks_for(n, 256), 256, 0, s>>>(
        dim, side, nz, row0, n, static_cast<int64_t*>(rowptr));
  else
    poisson_count_kernel<int32_t><<<blocks_for(n, 256), 256, 0, s>>>(
        dim, side, nz, row0, n, static_cast<int32_t*>(rowptr));
  KR_HIP_CHECK(hipGetLastError());
}

void launch_poisson_fill(int dim, int64_t side, int64_t nz, int64_t row0, int64_t n,
                         const void* rowptr, int rowptr64, int32_t* col, double* val,
                         hipStream_t s) {
  if (n <= 0) return;
  if (rowptr64)
    poisson_fill_kernel<int64_t><<<blocks_for(n, 256), 256, 0, s>>>(
        dim, side, nz, row0, n, static_cast<const int64_t*>(rowptr), col, val);
  else
    poisson_fill_kernel<int32_t><<<blocks_for(n, 256), 256, 0, s>>>(
        dim, side, nz, row0, n, static_cast<const int32_t*>(rowptr), col, val);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_banded_count(const BandSpec& b, int64_t row0, int64_t n, void* rowptr,
                         int rowptr64, hipStream_t s) {
  if (n <= 0) return;
  if (rowptr64)
    banded_count_kernel<int64_t><<<blocks_for(n, 256), 256, 0, s>>>(
        b, row0, n, static_cast<int64_t*>(rowptr));
  else
    banded_count_kernel<int32_t><<<blocks_for(n, 256), 256, 0, s>>>(
        b, row0, n, static_cast<int32_t*>(rowptr));
  KR_HIP_CHECK(hipGetLastError());
}

void launch_banded_fill(const BandSpec& b, int64_t row0, int64_t n, const void* rowptr,
                        int rowptr64, int32_t* col, double* val, hipStream_t s) {
  if (n <= 0) return;
  if (rowptr64)
    banded_fill_kernel<int64_t><<<blocks_for(n, 256), 256, 0, s>>>(
        b, row0, n, static_cast<const int64_t*>(rowptr), col, val);
  else
    banded_fill_kernel<int32_t><<<blocks_for(n, 256), 256, 0, s>>>(
        b, row0, n, static_cast<const int32_t*>(rowptr), col, val);
  KR_HIP_CHECK(hipGetLastError());
}

void rowptr_scan(void* rowptr, int rowptr64, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  size_t tmp_bytes = 0;
  if (rowptr64) {
    int64_t* p = static_cast<int64_t*>(rowptr) + 1;
    KR_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, p, p, n, s));
    void* tmp = nullptr;
    KR_HIP_CHECK(hipMalloc(&tmp, tmp_bytes));
    KR_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, p, p, n, s));
    KR_HIP_CHECK(hipStreamSynchronize(s));
    KR_HIP_CHECK(hipFree(tmp));
  } else {
    int32_t* p = static_cast<int32_t*>(rowptr) + 1;
    KR_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, tmp_bytes, p, p, (int)n, s));
    void* tmp = nullptr;
    KR_HIP_CHECK(hipMalloc(&tmp, tmp_bytes));
    KR_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, p, p, (int)n, s));
    KR_HIP_CHECK(hipStreamSynchronize(s));
    KR_HIP_CHECK(hipFree(tmp));
  }
}

void launch_fill_rhs(uint64_t seed, int64_t row0, int64_t n, double* b, hipStream_t s) {
  if (n <= 0) return;
  fill_rhs_kernel<<<blocks_for(n, 256), 256, 0, s>>>(seed, row0, n, b);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_col_minmax(const void* rowptr, int rowptr64, int64_t n, const int32_t* col,
                       int64_t* out2, hipStream_t s) {
  const unsigned long long init[2] = {(unsigned long long)INT64_MAX, 0ull};
  KR_HIP_CHECK(hipMemcpyAsync(out2, init, sizeof(init), hipMemcpyHostToDevice, s));
  if (n <= 0) return;
  auto* o = reinterpret_cast<unsigned long long*>(out2);
  if (rowptr64)
    col_minmax_kernel<int64_t><<<1024, kBlock, 0, s>>>(static_cast<const int64_t*>(rowptr),
                                                        n, col, o);
  else
    col_minmax_kernel<int32_t><<<1024, kBlock, 0, s>>>(static_cast<const int32_t*>(rowptr),
                                                        n, col, o);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_interior(const void* rowptr, int rowptr64, int64_t n, const int32_t* col,
                     int64_t lo, int64_t hi, int64_t* out2, hipStream_t s) {
  const unsigned long long init[3] = {0ull, (unsigned long long)n, 0ull};
  KR_HIP_CHECK(hipMemcpyAsync(out2, init, sizeof(init), hipMemcpyHostToDevice, s));
  if (n <= 0) return;
  auto* o = reinterpret_cast<unsigned long long*>(out2);
  if (rowptr64)
    interior_kernel<int64_t><<<blocks_for(n, 256), 256, 0, s>>>(
        static_cast<const int64_t*>(rowptr), n, col, lo, hi, o);
  else
    interior_kernel<int32_t><<<blocks_for(n, 256), 256, 0, s>>>(
        static_cast<const int32_t*>(rowptr), n, col, lo, hi, o);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_offsets(const void* rowptr, int rowptr64, int64_t n, const int32_t* col,
                    int64_t base, unsigned long long* table, int* flags, hipStream_t s) {
  KR_HIP_CHECK(hipMemsetAsync(table, 0, kOffTable * sizeof(unsigned long long), s));
  KR_HIP_CHECK(hipMemsetAsync(flags, 0, sizeof(int), s));
  if (n <= 0) return;
  const unsigned g = std::min<unsigned>(blocks_for(n, 256), 4096);
  if (rowptr64)
    offsets_kernel<int64_t><<<g, 256, 0, s>>>(static_cast<const int64_t*>(rowptr), n, col, base,
                                              table, flags);
  else
    offsets_kernel<int32_t><<<g, 256, 0, s>>>(static_cast<const int32_t*>(rowptr), n, col, base,
                                              table, flags);
  KR_HIP_CHECK(hipGetLastError());
}

template <typename MT>
static void masks_typed(const void* rowptr, int rowptr64, int64_t n, const int32_t* col,
                        int64_t base, const int32_t* M, int nm, void* mask, hipStream_t s) {
  const unsigned g = std::min<unsigned>(blocks_for(n, 256), 4096);
  if (rowptr64)
    mask_kernel<int64_t, MT><<<g, 256, 0, s>>>(static_cast<const int64_t*>(rowptr), n, col, base,
                                               M, nm, static_cast<MT*>(mask));
  else
    mask_kernel<int32_t, MT><<<g, 256, 0, s>>>(static_cast<const int32_t*>(rowptr), n, col, base,
                                               M, nm, static_cast<MT*>(mask));
}

void launch_masks(const void* rowptr, int rowptr64, int64_t n, const int32_t* col, int64_t base,
                  const int32_t* M, int nm, int mw, void* mask, hipStream_t s) {
  KR_REQUIRE(nm >= 1 && nm <= mw && (mw == 8 || mw == 16 || mw == 32 || mw == 64),
             "offset masks: bad width");
  if (n <= 0) return;
  if (mw == 8) masks_typed<uint8_t>(rowptr, rowptr64, n, col, base, M, nm, mask, s);
  else if (mw == 16) masks_typed<uint16_t>(rowptr, rowptr64, n, col, base, M, nm, mask, s);
  else if (mw == 32) masks_typed<uint32_t>(rowptr, rowptr64, n, col, base, M, nm, mask, s);
  else masks_typed<uint64_t>(rowptr, rowptr64, n, col, base, M, nm, mask, s);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_stencil_codes(const void* rowptr, int rowptr64, int64_t n, const int32_t* col,
                          const uint8_t* vcode, int64_t base, const int32_t* M, int nm,
                          uint64_t* out, hipStream_t s) {
  KR_REQUIRE(nm >= 1 && nm <= 8, "stencil codes: 1..8 offsets");
  if (n <= 0) return;
  const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 65535);
  if (rowptr64)
    stencil_codes_kernel<int64_t><<<g, 256, 0, s>>>(static_cast<const int64_t*>(rowptr), n, col,
                                                    vcode, base, M, nm, out);
  else
    stencil_codes_kernel<int32_t><<<g, 256, 0, s>>>(static_cast<const int32_t*>(rowptr), n, col,
                                                    vcode, base, M, nm, out);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_stencil_pack(const uint64_t* in, int64_t n, int cb, void* out, hipStream_t s) {
  KR_REQUIRE(cb == 2 || cb == 4, "stencil codes: 2 or 4 bits per slot");
  if (n <= 0) return;
  const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 65535);
  if (cb == 2)
    stencil_pack_kernel<2><<<g, 256, 0, s>>>(in, n, out);
  else
    stencil_pack_kernel<4><<<g, 256, 0, s>>>(in, n, out);
  KR_HIP_CHECK(hipGetLastError());
}

namespace {
__global__ void dia_symcheck_kernel(const uint8_t* __restrict__ mask, int mb, int64_t n,
                                    const int32_t* __restrict__ M, int nm,
                                    const double* __restrict__ dia, int64_t bs, int64_t ks,
                                    int* flag) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    for (int k = 0; k < nm / 2; ++k) {
      if (!((mask[i * mb + k / 8] >> (k % 8)) & 1)) continue;
      const int64_t j = i + M[k];
      if (j < 0) continue;
      const int km = nm - 1 - k;
      const bool there = (mask[j * mb + km / 8] >> (km % 8)) & 1;
      const double lo = dia[(i / kDiaRows) * bs + k * ks + i % kDiaRows];
      const double up = dia[(j / kDiaRows) * bs + km * ks + j % kDiaRows];
      if (!there || __double_as_longlong(lo) != __double_as_longlong(up))
        *flag = 1;  // plain vector store: every writer stores 1
    }
  }
}
}  // namespace

void launch_dia_symcheck(const void* mask, int mw, int64_t n, const int32_t* M, int nm,
                         const double* dia, int64_t bs, int64_t ks, int* flag, hipStream_t s) {
  if (n <= 0) return;
  const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 65535);
  dia_symcheck_kernel<<<g, 256, 0, s>>>(static_cast<const uint8_t*>(mask), mw / 8, n, M, nm, dia,
                                        bs, ks, flag);
  KR_HIP_CHECK(hipGetLastError());
}

namespace {
// full[b] = 1 when every row of DIA row block b exists (b * 256 + 255 < n)
// and holds all nm offsets.
__global__ void dia_block_full_kernel(const uint8_t* __restrict__ mask, int mb, int64_t n, int nm,
                                      uint8_t* full, int64_t nb) {
  for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const int64_t i = b * kDiaRows + threadIdx.x;
    bool ok = i < n;
    for (int j = 0; ok && j < mb; ++j) {
      const int lo = 8 * j, hi = min(nm, lo + 8);
      const unsigned want = hi > lo ? (1u << (hi - lo)) - 1u : 0u;
      ok = mask[i * mb + j] == want;
    }
    const int all = __syncthreads_and(ok ? 1 : 0);
    if (threadIdx.x == 0) full[b] = all ? 1 : 0;
  }
}
}  // namespace

void launch_dia_block_full(const void* mask, int mw, int64_t n, int nm, uint8_t* full,
                           hipStream_t s) {
  const int64_t nb = (n + kDiaRows - 1) / kDiaRows;
  if (nb <= 0) return;
  const unsigned g = (unsigned)std::min<int64_t>(nb, 65535);
  dia_block_full_kernel<<<g, kDiaRows, 0, s>>>(static_cast<const uint8_t*>(mask), mw / 8, n, nm,
                                               full, nb);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_dia_fill(const void* rowptr, int rowptr64, int64_t n, const int32_t* col,
                     const double* val, int64_t base, const int32_t* M, int nm, double* dia,
                     int64_t bs, int64_t ks, hipStream_t s) {
  if (n <= 0) return;
  const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 65535);
  if (rowptr64)
    dia_fill_kernel<int64_t><<<g, 256, 0, s>>>(static_cast<const int64_t*>(rowptr), n, col, val,
                                               base, M, nm, dia, bs, ks);
  else
    dia_fill_kernel<int32_t><<<g, 256, 0, s>>>(static_cast<const int32_t*>(rowptr), n, col, val,
                                               base, M, nm, dia, bs, ks);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_col_shift(const void* rowptr, int rowptr64, int64_t n, int32_t* col,
                      int64_t delta, hipStream_t s) {
  if (n <= 0 || delta == 0) return;
  if (rowptr64)
    col_shift_kernel<int64_t><<<2048, kBlock, 0, s>>>(static_cast<const int64_t*>(rowptr),
                                                       n, col, delta);
  else
    col_shift_kernel<int32_t><<<2048, kBlock, 0, s>>>(static_cast<const int32_t*>(rowptr),
                                                       n, col, delta);
  KR_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Value dictionary (SpmvArgs::vcode): a block whose stored values take at most
// kVdMax distinct bit patterns is re-stored as one 8-bit code per entry plus a
// table, so the row walk streams 1 byte per entry instead of 8 (lossless:
// codes map back to the exact bit patterns; CSR-VI, Kourtis et al. 2008).
// ---------------------------------------------------------------------------
namespace {
constexpr int kVdSet = 512;  // per-workgroup LDS set slots (open addressing)
constexpr unsigned long long kVdEmpty = ~0ull;  // a NaN payload: never stored (flag 2)

__device__ __forceinline__ unsigned vd_hash(unsigned long long k, int slots) {
  return (unsigned)((k * 0x9E3779B97F4A7C15ull) >> 40) & (unsigned)(slots - 1);
}

// Distinct bit patterns of val[0, nnz) into gtab[kVdGlobal] (kVdEmpty = free).
// flags[0]: 1 = more than kVdMax patterns, 2 = the sentinel pattern occurs.
// Each workgroup first collects into an LDS set and stops as soon as it holds
// more than kVdMax patterns (matrices with many values exit in one chunk).
__global__ __launch_bounds__(256) void vdict_collect_kernel(const unsigned long long* val,
                                                            int64_t nnz,
                                                            unsigned long long* gtab,
                                                            int* flags) {
  __shared__ unsigned long long set[kVdSet];
  __shared__ int cnt, over;
  for (int i = threadIdx.x; i < kVdSet; i += blockDim.x) set[i] = kVdEmpty;
  if (threadIdx.x == 0) {
    cnt = 0;
    over = 0;
  }
  __syncthreads();
  constexpr int kPer = 64;  // entries per lane per chunk
  const int64_t chunk = (int64_t)blockDim.x * kPer;
  for (int64_t c0 = (int64_t)blockIdx.x * chunk; c0 < nnz; c0 += (int64_t)gridDim.x * chunk) {
    for (int u = 0; u < kPer; ++u) {
      const int64_t j = c0 + (int64_t)u * blockDim.x + threadIdx.x;
      if (j >= nnz) break;
      if (*(volatile int*)&over) break;
      const unsigned long long key = val[j];
      if (key == kVdEmpty) {
        atomicOr(&over, 2);
        break;
      }
      unsigned h = vd_hash(key, kVdSet);
      for (int probe = 0; probe < kVdSet; ++probe) {
        const unsigned long long v = *(volatile unsigned long long*)&set[h];
        if (v == key) break;
        if (v == kVdEmpty) {
          const unsigned long long old = atomicCAS(&set[h], kVdEmpty, key);
          if (old == kVdEmpty) {
            if (atomicAdd(&cnt, 1) >= kVdMax) atomicOr(&over, 1);
            break;
          }
          if (old == key) break;
        }
        h = (h + 1) & (kVdSet - 1);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0 && __atomic_load_n(flags, __ATOMIC_RELAXED)) atomicOr(&over, 1);
    __syncthreads();
    if (over) break;
  }
  if (over) {
    if (threadIdx.x == 0) atomicOr(flags, over);
    return;
  }
  // merge this workgroup's patterns into the global set
  for (int i = threadIdx.x; i < kVdSet; i += blockDim.x) {
    const unsigned long long key = set[i];
    if (key == kVdEmpty) continue;
    unsigned h = vd_hash(key, kVdGlobal);
    int probe = 0;
    for (; probe < kVdGlobal; ++probe) {
      const unsigned long long old = atomicCAS(&gtab[h], kVdEmpty, key);
      if (old == kVdEmpty) {
        if (atomicAdd(&flags[1], 1) >= kVdMax) atomicOr(flags, 1);
        break;
      }
      if (old == key) break;
      h = (h + 1) & (kVdGlobal - 1);
    }
    if (probe == kVdGlobal) atomicOr(flags, 1);
  }
}

// code[j] = index of val[j]'s bit pattern in the ascending table keys[0, nk).
// A pattern missing from the table (the collect pass must have seen every
// one; this checks it) sets *miss, and the host then drops the dictionary.
__global__ __launch_bounds__(256) void vdict_encode_kernel(const unsigned long long* val,
                                                           int64_t nnz,
                                                           const unsigned long long* keys,
                                                           int nk, uint8_t* code, int* miss) {
  __shared__ unsigned long long sk[kVdMax];
  for (int i = threadIdx.x; i < nk; i += blockDim.x) sk[i] = keys[i];
  __syncthreads();
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nnz;
       j += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long key = val[j];
    int lo = 0, hi = nk - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (sk[mid] < key)
        lo = mid + 1;
      else
        hi = mid;
    }
    code[j] = (uint8_t)lo;
    if (sk[lo] != key) *miss = 1;  // plain vector store: every writer stores 1
  }
}
}  // namespace

void launch_vdict_collect(const double* val, int64_t nnz, unsigned long long* gtab, int* flags,
                          hipStream_t s) {
  KR_HIP_CHECK(hipMemsetAsync(gtab, 0xff, kVdGlobal * sizeof(unsigned long long), s));
  KR_HIP_CHECK(hipMemsetAsync(flags, 0, 2 * sizeof(int), s));
  if (nnz <= 0) return;
  const unsigned g = std::min<unsigned>(blocks_for(nnz, 256 * 64), 2048);
  vdict_collect_kernel<<<g, 256, 0, s>>>(reinterpret_cast<const unsigned long long*>(val), nnz,
                                         gtab, flags);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_vdict_encode(const double* val, int64_t nnz, const unsigned long long* keys, int nk,
                         uint8_t* code, int* miss, hipStream_t s) {
  KR_HIP_CHECK(hipMemsetAsync(miss, 0, sizeof(int), s));
  if (nnz <= 0) return;
  const unsigned g = std::min<unsigned>(blocks_for(nnz, 256), 8192);
  vdict_encode_kernel<<<g, 256, 0, s>>>(reinterpret_cast<const unsigned long long*>(val), nnz,
                                        keys, nk, code, miss);
  KR_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// ILU preconditioner sweeps (the reference's `ilu.solve`, a scipy SuperLU:
// v1/threads/pipeline/pcg.py:26,41). M = Pr^T L U Pc^T; M^-1 v = Pc U^-1
// L^-1 Pr v as two level-scheduled triangular sweeps (IluSweepArgs). Rows of
// one level depend only on rows of earlier levels, so each level is a
// parallel step; the levels run in ONE workgroup, separated by barriers: a
// sweep is one launch with no inter-workgroup synchronisation (nothing to
// time out), and the typical level holds tens of rows (a 256^2 Poisson spilu
// has ~1000 levels of ~65 rows), which one workgroup covers. Levels wider
// than KR_ILU_WIDE rows (a 3-D ILU(0) of 256^3: up to ~49,000) get a launch
// of their own over the whole GPU instead (IluSeg). Row i: s = rhs,
// s -= T[i][j] x[j] over the stored strictly-triangular entries in ascending
// column order, x[i] = s / T[i][i].
// ---------------------------------------------------------------------------
namespace {
constexpr int kIluThreads = 1024;

// One row of a sweep (the entry t of the level lists).
template <bool LOWER>
__device__ __forceinline__ void ilu_row(const IluSweepArgs& a, int64_t t) {
  if (a.ew > 0) {  // level-ordered rows: the same statements, fewer dependent loads
    const int32_t i = a.lvl_rows[t];
    const int n = a.ecnt[t];
    double s = a.in[a.ein[t]];
    int32_t c[kIluEll];
    double v[kIluEll];
#pragma unroll
    for (int j = 0; j < kIluEll; ++j) {
      c[j] = j < n ? a.ecol[t * a.ew + j] : 0;
      v[j] = j < n ? a.eval[t * a.ew + j] : 0.0;
    }
    double xs[kIluEll];
#pragma unroll
    for (int j = 0; j < kIluEll; ++j) xs[j] = j < n ? a.x[c[j]] : 0.0;
#pragma unroll
    for (int j = 0; j < kIluEll; ++j)
      if (j < n) s = s - v[j] * xs[j];
    const double xi = s / a.ediag[t];
    a.x[i] = xi;
    if (!LOWER) a.out[a.perm[i]] = xi;
    return;
  }
  const int32_t i = a.lvl_rows[t];
  double s = LOWER ? a.in[a.perm[i]] : a.in[i];  // lower: (Pr v)[i] = v[prinv[i]]
  const int64_t j1 = a.rp[i + 1];
  for (int64_t jj = a.rp[i]; jj < j1; ++jj) s = s - a.val[jj] * a.x[a.col[jj]];
  const double xi = s / a.diag[i];
  a.x[i] = xi;
  if (!LOWER) a.out[a.perm[i]] = xi;  // (Pc z)[j] = z[pc[j]]: out[pcinv[i]] = z[i]
}

// Levels [lev0, lev1) in one workgroup, a barrier between levels.
template <bool LOWER>
__global__ __launch_bounds__(kIluThreads) void ilu_sweep_kernel(IluSweepArgs a) {
  const int tid = threadIdx.x;
  for (int64_t lev = a.lev0; lev < a.lev1; ++lev) {
    const int64_t beg = a.lvl_ptr[lev];  // uniform: scalar loads
    const int64_t end = a.lvl_ptr[lev + 1];
    for (int64_t t = beg + tid; t < end; t += kIluThreads) ilu_row<LOWER>(a, t);
    __syncthreads();  // this level's x visible to the next level's rows
  }
}

// One wide level over the grid: a row per thread.
template <bool LOWER>
__global__ __launch_bounds__(kBlock) void ilu_level_kernel(IluSweepArgs a) {
  const int64_t t = a.lvl_ptr[a.lev0] + (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t < a.lvl_ptr[a.lev0 + 1]) ilu_row<LOWER>(a, t);
}
}  // namespace

void launch_ilu_sweep(bool lower, const IluSweepArgs& a, const IluSeg* segs, int nseg,
                      hipStream_t s) {
  for (int q = 0; q < nseg; ++q) {
    IluSweepArgs b = a;
    b.lev0 = segs[q].lev0;
    b.lev1 = segs[q].lev1;
    KR_REQUIRE(b.lev0 >= 0 && b.lev0 < b.lev1 && b.lev1 <= a.nlev, "ILU: bad level segment");
    if (segs[q].rows > 0) {
      KR_REQUIRE(b.lev1 == b.lev0 + 1, "ILU: a wide segment is one level");
      const int64_t g = (segs[q].rows + kBlock - 1) / kBlock;
      KR_REQUIRE(g < ((int64_t)1 << 31), "ILU: level too wide");
      if (lower)
        ilu_level_kernel<true><<<(unsigned)g, kBlock, 0, s>>>(b);
      else
        ilu_level_kernel<false><<<(unsigned)g, kBlock, 0, s>>>(b);
    } else if (lower) {
      ilu_sweep_kernel<true><<<1, kIluThreads, 0, s>>>(b);
    } else {
      ilu_sweep_kernel<false><<<1, kIluThreads, 0, s>>>(b);
    }
    KR_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace kr
