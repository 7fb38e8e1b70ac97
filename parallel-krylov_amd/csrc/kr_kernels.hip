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

#include <cstdlib>
#include <type_traits>

#include "kr_hash.h"
#include "kr_internal.h"

namespace kr {

namespace {

// ---------------------------------------------------------------------------
// Block-level deterministic reduction of NP per-thread accumulators into
// partials[p * grid + blockIdx.x].
// ---------------------------------------------------------------------------
template <int NP>
__device__ __forceinline__ void block_reduce_store(double (&acc)[NP > 0 ? NP : 1],
                                                   double* partials, int grid,
                                                   double* s_red /* NP*4 */,
                                                   int accumulate = 0) {
  if constexpr (NP > 0) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      double v = acc[p];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
      if (lane == 0) s_red[p * 4 + wave] = v;
    }
    __syncthreads();
    if (threadIdx.x < NP) {
      const double* r = s_red + threadIdx.x * 4;
      double t = r[0];
      t = t + r[1];
      t = t + r[2];
      t = t + r[3];
      double* dst = partials + (int64_t)threadIdx.x * grid + blockIdx.x;
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
typedef double dbl2v __attribute__((ext_vector_type(2)));
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

template <int NV, int GATHER, typename W>
__device__ __forceinline__ void row_window_mask(const double* s_val, const int32_t* s_M,
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
template <int NV, int GATHER = kGather>
__device__ __forceinline__ void row_window(const double* s_val, const int32_t* s_col,
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
  __device__ int64_t rb(int64_t v) const {
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
};

template <typename RP, int EPI, bool VEC, int GATHER = kGather, bool XCD = true, bool NT = false,
          int MW = 0>
__global__ __launch_bounds__(kBlock) void spmv_kernel(SpmvArgs a) {
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

  const int64_t nrb = (a.n + kBlock - 1) / kBlock;
  RowSched sched;
  sched.init(nrb, a.slab, a.slab_sub, XCD);
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

  for (;;) {
    if (first_window) {
      if (tid < nr) s_rp[tid + 1] = (int32_t)(my_end - bs);
      if (tid == 0) s_rp[0] = 0;
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
      const int64_t row = r0 + tid;
      double y1 = sum1;
      if constexpr (EPI == EPI_BMINUS) y1 = a.b[row] - sum1;
      a.y1[row] = y1;
      if constexpr (NV == 2) a.y2[row] = sum2;
      if constexpr (NP > 0) {
        const double xv = T::kX ? x1[a.xoff + row] : 0.0;
        const double x2v = T::kX2 ? x2[a.xoff + row] : 0.0;
        const double ev = T::kE ? a.e[row] : 0.0;
        epi_products<EPI>(xv, x2v, y1, sum2, ev, acc);
      }
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

  const int64_t nrb = (a.n + kBlock - 1) / kBlock;
  RowSched sched;  // as spmv_kernel
  sched.init(nrb, a.slab, a.slab_sub, true);
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

  for (;;) {
    if (first_window) {
      if (tid < nr) s_rp[tid + 1] = (int32_t)(my_end - bs);
      if (tid == 0) s_rp[0] = 0;
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
      const int64_t row = r0 + tid;
      double y1 = sum1;
      if constexpr (EPI == EPI_BMINUS) y1 = a.b[row] - sum1;
      a.y1[row] = y1;
      if constexpr (NV == 2) a.y2[row] = sum2;
      if constexpr (NP > 0) {
        const double xv = T::kX ? x1[a.xoff + row] : 0.0;
        const double x2v = T::kX2 ? x2[a.xoff + row] : 0.0;
        const double ev = T::kE ? a.e[row] : 0.0;
        epi_products<EPI>(xv, x2v, y1, sum2, ev, acc);
      }
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

// Variant 1: no cross-row-block prefetch (lower VGPR count, higher occupancy).
template <typename RP, int EPI, bool VEC>
__global__ __launch_bounds__(kBlock) void spmv_kernel_simple(SpmvArgs a) {
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  __shared__ __attribute__((aligned(16))) double s_val[kWindow];
  __shared__ __attribute__((aligned(16))) int32_t s_col[kWindow];
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

  const int64_t nrb = (a.n + kBlock - 1) / kBlock;
  for (int64_t rb = blockIdx.x; rb < nrb; rb += gridDim.x) {
    const int64_t r0 = rb * kBlock;
    const int nr = (int)min((int64_t)kBlock, a.n - r0);
    const int64_t bs = (int64_t)rowptr[r0];
    const int64_t be = (int64_t)rowptr[r0 + nr];
    if (tid < nr) s_rp[tid + 1] = (int32_t)((int64_t)rowptr[r0 + tid + 1] - bs);
    if (tid == 0) s_rp[0] = 0;
    __syncthreads();
    const bool active = tid < nr;
    const int rs = active ? s_rp[tid] : 0;
    const int re = active ? s_rp[tid + 1] : 0;
    double sum1 = 0.0, sum2 = 0.0;
    // windows start 4-aligned so every slot is one 16-byte access
    const int64_t w0 = VEC ? (bs & ~(int64_t)3) : bs;
    for (int64_t ws = w0; ws < be; ws += kWindow) {
      {
        Stage st;
        stage_load<VEC>(st, val, col, ws, bs, be, tid);
        stage_commit(st, s_val, s_col, tid);
      }
      __syncthreads();
      if (active) {
        // this lane's entries inside the window, as window offsets
        const int64_t off = bs - ws;  // window offset of the block's entry 0
        const int js = (int)max((int64_t)rs + off, (int64_t)0);
        const int je = (int)min((int64_t)re + off, (int64_t)kWindow);
        for (int j = js; j < je; j += kGather) {
          double v[kGather], p1[kGather], p2[kGather];
#pragma unroll
          for (int u = 0; u < kGather; ++u) {
            const int jj = (j + u < je) ? j + u : js;
            v[u] = s_val[jj];
            const int c = s_col[jj];
            p1[u] = x1[c];
            if constexpr (NV == 2) p2[u] = x2[c];
          }
#pragma unroll
          for (int u = 0; u < kGather; ++u) {
            if (j + u < je) {
              sum1 = sum1 + v[u] * p1[u];
              if constexpr (NV == 2) sum2 = sum2 + v[u] * p2[u];
            }
          }
        }
      }
      __syncthreads();
    }
    if (active) {
      const int64_t row = r0 + tid;
      double y1 = sum1;
      if constexpr (EPI == EPI_BMINUS) y1 = a.b[row] - sum1;
      a.y1[row] = y1;
      if constexpr (NV == 2) a.y2[row] = sum2;
      if constexpr (NP > 0) {
        const double xv = T::kX ? x1[a.xoff + row] : 0.0;
        const double x2v = T::kX2 ? x2[a.xoff + row] : 0.0;
        const double ev = T::kE ? a.e[row] : 0.0;
        epi_products<EPI>(xv, x2v, y1, sum2, ev, acc);
      }
    }
    __syncthreads();  // s_rp is rewritten by the next row block
  }
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
}

// Variant 2: wave-independent. Each wave owns 64-row blocks and a private
// LDS window; staging and the row walk need only wave-local ordering (an
// s_waitcnt on the LDS counter), never a workgroup barrier, so the four waves
// of a workgroup stream independently.
constexpr int kWaveRows = 64;
constexpr int kWaveWindow = 512;  // entries per wave window (2 slots of 4 per lane)
constexpr int kWaveSlots = kWaveWindow / (4 * kWaveRows);
static_assert(kWaveSlots * 4 * kWaveRows == kWaveWindow, "wave window layout");

__device__ __forceinline__ void lds_fence() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <typename RP, int EPI, bool VEC>
__global__ __launch_bounds__(kBlock) void spmv_kernel_wave(SpmvArgs a) {
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  constexpr int kWaves = kBlock / 64;
  __shared__ __attribute__((aligned(16))) double s_val_all[kWaves][kWaveWindow];
  __shared__ __attribute__((aligned(16))) int32_t s_col_all[kWaves][kWaveWindow];
  __shared__ double s_red[(NP > 0 ? NP : 1) * 4];

  const RP* __restrict__ rowptr = static_cast<const RP*>(a.rowptr);
  const double* __restrict__ val = a.val;
  const int32_t* __restrict__ col = a.col;
  const double* __restrict__ x1 = a.x1;
  const double* __restrict__ x2 = a.x2;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  double* s_val = s_val_all[w];
  int32_t* s_col = s_col_all[w];

  double acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int p = 0; p < (NP > 0 ? NP : 1); ++p) acc[p] = 0.0;

  const int64_t nwb = (a.n + kWaveRows - 1) / kWaveRows;
  const int64_t gw = (int64_t)blockIdx.x * kWaves + w;
  const int64_t nwaves = (int64_t)gridDim.x * kWaves;
  for (int64_t wb = gw; wb < nwb; wb += nwaves) {
    const int64_t r0 = wb * kWaveRows;
    const int nr = (int)min((int64_t)kWaveRows, a.n - r0);
    const int64_t bs = (int64_t)rowptr[r0];
    const int64_t be = (int64_t)rowptr[r0 + nr];
    const bool active = lane < nr;
    const int64_t my_end = active ? (int64_t)rowptr[r0 + lane + 1] : be;
    // row start = previous lane's end (lane 0: block start)
    const int64_t my_beg = !active ? be : lane == 0 ? bs : (int64_t)rowptr[r0 + lane];
    const int rs = (int)(my_beg - bs), re = (int)(my_end - bs);
    double sum1 = 0.0, sum2 = 0.0;
    const int64_t w0 = VEC ? (bs & ~(int64_t)3) : bs;
    for (int64_t ws = w0; ws < be; ws += kWaveWindow) {
      dbl2v lo[kWaveSlots], hi[kWaveSlots];
      int4v c4[kWaveSlots];
#pragma unroll
      for (int q = 0; q < kWaveSlots; ++q) {
        const int64_t g0 = ws + (int64_t)(lane + q * 64) * 4;
        if (VEC && g0 >= bs && g0 + 4 <= be) {
          lo[q] = *reinterpret_cast<const dbl2v*>(val + g0);
          hi[q] = *reinterpret_cast<const dbl2v*>(val + g0 + 2);
          c4[q] = *reinterpret_cast<const int4v*>(col + g0);
        } else {
          double tv[4];
          int tc[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int64_t g = g0 + u;
            const bool ok = g >= bs && g < be;
            tv[u] = ok ? val[g] : 0.0;
            tc[u] = ok ? col[g] : 0;
          }
          lo[q] = dbl2v{tv[0], tv[1]};
          hi[q] = dbl2v{tv[2], tv[3]};
          c4[q] = int4v{tc[0], tc[1], tc[2], tc[3]};
        }
      }
      lds_fence();  // previous window fully read by every lane of the wave
#pragma unroll
      for (int q = 0; q < kWaveSlots; ++q) {
        const int e0 = (lane + q * 64) * 4;
        *reinterpret_cast<dbl2v*>(&s_val[e0]) = lo[q];
        *reinterpret_cast<dbl2v*>(&s_val[e0 + 2]) = hi[q];
        *reinterpret_cast<int4v*>(&s_col[e0]) = c4[q];
      }
      lds_fence();  // window visible to every lane of the wave
      if (active) {
        const int64_t off = bs - ws;
        row_window<NV>(s_val, s_col, x1, x2, (int)max((int64_t)rs + off, (int64_t)0),
                       (int)min((int64_t)re + off, (int64_t)kWaveWindow), sum1, sum2);
      }
    }
    if (active) {
      const int64_t row = r0 + lane;
      double y1 = sum1;
      if constexpr (EPI == EPI_BMINUS) y1 = a.b[row] - sum1;
      a.y1[row] = y1;
      if constexpr (NV == 2) a.y2[row] = sum2;
      if constexpr (NP > 0) {
        const double xv = T::kX ? x1[a.xoff + row] : 0.0;
        const double x2v = T::kX2 ? x2[a.xoff + row] : 0.0;
        const double ev = T::kE ? a.e[row] : 0.0;
        epi_products<EPI>(xv, x2v, y1, sum2, ev, acc);
      }
    }
  }
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

template <typename RP, bool VEC>
void spmv_dispatch(SpmvEpi epi, const SpmvArgs& a, int nblocks, hipStream_t s) {
  const dim3 grid(nblocks), block(kBlock);
  // Row-walk (0) for short rows, product-then-sum (8) for long rows. The
  // KR_SPMV_VARIANT environment variable overrides the choice for A/B runs
  // (tools/spmv_micro.py): 1 no prefetch, 2 wave-independent, 3 4-deep gathers,
  // 6 no XCD schedule, 7 non-temporal staging.
  const char* env = getenv("KR_SPMV_VARIANT");
  const int variant = env ? atoi(env) : (a.long_rows ? 8 : 0);
  switch (epi) {
#define KR_CASE(E)                                      \
  case E:                                               \
    if (variant == 1)                                   \
      spmv_kernel_simple<RP, E, VEC><<<grid, block, 0, s>>>(a); \
    else if (variant == 2)                              \
      spmv_kernel_wave<RP, E, VEC><<<grid, block, 0, s>>>(a); \
    else if (variant == 3)                              \
      spmv_kernel<RP, E, VEC, 4><<<grid, block, 0, s>>>(a); \
    else if (variant == 9)                              \
      spmv_kernel<RP, E, VEC, 8><<<grid, block, 0, s>>>(a); \
    else if (variant == 8)                              \
      spmv_kernel_prod<RP, E, VEC><<<grid, block, 0, s>>>(a); \
    else if (variant == 6)                              \
      spmv_kernel<RP, E, VEC, kGather, false><<<grid, block, 0, s>>>(a); \
    else if (variant == 7)                              \
      spmv_kernel<RP, E, VEC, kGather, true, true><<<grid, block, 0, s>>>(a); \
    else if (!(a.mask && spmv_masked<RP, E, VEC>(a, grid, block, s))) \
      spmv_kernel<RP, E, VEC><<<grid, block, 0, s>>>(a); \
    break;
    KR_CASE(EPI_NONE)
    KR_CASE(EPI_BMINUS)
    KR_CASE(EPI_XY)
    KR_CASE(EPI_HEAD_MRR)
    KR_CASE(EPI_HEAD_KCG)
    KR_CASE(EPI_MRR_LOOP)
    KR_CASE(EPI_DUAL_NONE)
    KR_CASE(EPI_DUAL_MRR)
    KR_CASE(EPI_DUAL_KCG)
#undef KR_CASE
    default:
      throw Failure(KR_ERR_INVALID, "unknown SpMV epilogue");
  }
}

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

template <int OP>
__device__ __forceinline__ void ew_elem(double c0, double c1, double (&v)[6],
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
  }
}

template <int OP, bool VEC, int U = 1, bool NTS = false>
__global__ __launch_bounds__(kBlock) void ew_kernel(EwArgs a) {
  using T = EwTraits<OP>;
  constexpr int NP = T::NP;
  __shared__ double s_red[(NP > 0 ? NP : 1) * 4];
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
    for (int64_t q0 = t0; q0 < npairs; q0 += U * stride) {
      double va[U][6], vb[U][6];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t q = q0 + u * stride;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          if ((T::R & (1 << k)) && q < npairs) {
            const double2 d = reinterpret_cast<const double2*>(a.p[k])[q];
            va[u][k] = d.x;
            vb[u][k] = d.y;
          } else {
            va[u][k] = vb[u][k] = 0.0;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t q = q0 + u * stride;
        if (q >= npairs) break;
        ew_elem<OP>(a.c0, a.c1, va[u], acc);
        ew_elem<OP>(a.c0, a.c1, vb[u], acc);
#pragma unroll
        for (int k = 0; k < 6; ++k)
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
      double v[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) v[k] = (T::R & (1 << k)) ? a.p[k][i] : 0.0;
      ew_elem<OP>(a.c0, a.c1, v, acc);
#pragma unroll
      for (int k = 0; k < 6; ++k)
        if (T::W & (1 << k)) a.p[k][i] = v[k];
    }
  } else {
    for (int64_t i = t0; i < a.n; i += stride) {
      double v[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) v[k] = (T::R & (1 << k)) ? a.p[k][i] : 0.0;
      ew_elem<OP>(a.c0, a.c1, v, acc);
#pragma unroll
      for (int k = 0; k < 6; ++k)
        if (T::W & (1 << k)) a.p[k][i] = v[k];
    }
  }
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red);
}

template <int OP>
void ew_dispatch_op(const EwArgs& a, hipStream_t s) {
  bool aligned = true;
  for (int k = 0; k < 6; ++k)
    if (((EwTraits<OP>::R | EwTraits<OP>::W) & (1 << k)) &&
        (reinterpret_cast<uintptr_t>(a.p[k]) & 15))
      aligned = false;
  // KR_EW_VARIANT (A/B only): 0 = 1 pair/thread/iteration, 1 = 2 pairs,
  // 2 = 2 pairs + non-temporal stores.
  const char* env = getenv("KR_EW_VARIANT");
  const int variant = env ? atoi(env) : 0;
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
__global__ void poisson_count_kernel(int dim, int64_t side, int64_t row0, int64_t n,
                                     RP* rowptr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t g = row0 + i;
  int cnt = 1;
  for (int d = 0; d < dim; ++d) {
    const int64_t c = g % side;
    g /= side;
    cnt += (c > 0) + (c < side - 1);
  }
  rowptr[i + 1] = (RP)cnt;
}

template <typename RP>
__global__ void poisson_fill_kernel(int dim, int64_t side, int64_t row0, int64_t n,
                                    const RP* rowptr, int32_t* col, double* val) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t g = row0 + i;
  int64_t coord[3] = {0, 0, 0};
  int64_t stride[3] = {1, side, side * side};
  int64_t t = g;
  for (int d = 0; d < dim; ++d) {
    coord[d] = t % side;
    t /= side;
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
    if (coord[d] < side - 1) {
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
  }
  return 0;
}

void launch_spmv(SpmvEpi epi, const SpmvArgs& a, hipStream_t s) {
  launch_spmv_grid(epi, a, a.grid, s);
}

void launch_spmv_grid(SpmvEpi epi, const SpmvArgs& a, int nblocks, hipStream_t s) {
  KR_REQUIRE(a.grid > 0 && nblocks > 0 && nblocks <= a.grid,
             "spmv: need 0 < blocks <= partial stride");
  // 16-byte staging needs 16-byte aligned val/col bases
  const bool vec = ((reinterpret_cast<uintptr_t>(a.val) | reinterpret_cast<uintptr_t>(a.col)) &
                    15) == 0;
  (void)vec;
  if (a.rowptr64) {
    if (vec)
      spmv_dispatch<int64_t, true>(epi, a, nblocks, s);
    else
      spmv_dispatch<int64_t, false>(epi, a, nblocks, s);
  } else {
    if (vec)
      spmv_dispatch<int32_t, true>(epi, a, nblocks, s);
    else
      spmv_dispatch<int32_t, false>(epi, a, nblocks, s);
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
    default: throw Failure(KR_ERR_INVALID, "unknown elementwise op");
  }
  KR_HIP_CHECK(hipGetLastError());
}

void launch_finalize(const double* partials, int grid, int nslots, double* out,
                     hipStream_t s) {
  if (nslots <= 0) return;
  finalize_kernel<<<nslots, kBlock, 0, s>>>(partials, grid, out);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_multidot(const MultiDotArgs& a, hipStream_t s) {
  KR_REQUIRE(a.count >= 0 && a.count <= 64, "multidot: count must be in [0, 64]");
  for (int base = 0; base < a.count; base += 16) {
    multidot_kernel<<<a.grid, kBlock, 0, s>>>(a, base);
    KR_HIP_CHECK(hipGetLastError());
  }
}

void launch_poisson_count(int dim, int64_t side, int64_t row0, int64_t n, void* rowptr,
                          int rowptr64, hipStream_t s) {
  if (n <= 0) return;
  if (rowptr64)
    poisson_count_kernel<int64_t><<<blocks_for(n, 256), 256, 0, s>>>(
        dim, side, row0, n, static_cast<int64_t*>(rowptr));
  else
    poisson_count_kernel<int32_t><<<blocks_for(n, 256), 256, 0, s>>>(
        dim, side, row0, n, static_cast<int32_t*>(rowptr));
  KR_HIP_CHECK(hipGetLastError());
}

void launch_poisson_fill(int dim, int64_t side, int64_t row0, int64_t n,
                         const void* rowptr, int rowptr64, int32_t* col, double* val,
                         hipStream_t s) {
  if (n <= 0) return;
  if (rowptr64)
    poisson_fill_kernel<int64_t><<<blocks_for(n, 256), 256, 0, s>>>(
        dim, side, row0, n, static_cast<const int64_t*>(rowptr), col, val);
  else
    poisson_fill_kernel<int32_t><<<blocks_for(n, 256), 256, 0, s>>>(
        dim, side, row0, n, static_cast<const int32_t*>(rowptr), col, val);
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

}  // namespace kr
