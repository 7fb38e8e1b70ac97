// Round-5 experiments on the plain-CSR SpMV (included by csr_micro.cpp only,
// after kr_spmv.h; not part of the library). Results in profiles/r05a/README.txt:
// the LDS-free walk, fewer requested bytes (diagonal reuse, one row-pointer
// load, exact staging), paired and sc1 stores and a two-deep staging pipeline
// were all within noise or slower; non-temporal stores (-5 %) went into
// spmv_kernel2.
//
// CSR row walk without LDS (spmv_kernel_direct).
//
// The plain-CSR SpMV (column stream + 8-byte values: no offset masks, no
// value dictionary, no stencil codes) of short-row shards. One lane owns one
// row and sums it in stored order from 0.0 -- scipy csr_matvec's order, so
// y is bitwise scipy's -- exactly as spmv_kernel2 does, but every lane loads
// its OWN row's values and columns straight into registers: 16-byte loads
// from the 16-byte chunks holding the row (4 x double2 + 3 x int4 for up to
// 7 entries, whatever the row's alignment), the row's k-th entry then picked
// out of them by its start's alignment. No LDS window, no workgroup barrier:
// the waves of a workgroup run independently, so the CU's waves are spread
// over every phase of the row walk and the stream stays in flight. What
// spmv_kernel2 spent on the LDS round trip (6 ds_write_b128 + 14 ds_read per
// lane and window, one barrier) is gone; the per-wave HBM lines are the same
// (a wave's 64 consecutive rows are one contiguous run of entries, read
// whole across its 4 + 3 loads, which hit L1 after the first touch).
//
// Software pipeline per lane (vmcnt completes in issue order): for row block
// j it issues j's x gathers, then the value/column loads of block j + 1 and
// the row pointers of block j + 2, and only then waits for j's gathers; the
// next block's stream is in flight across the sums and the epilogue. The
// loop is unrolled x2 over two register sets, so no loaded register is ever
// copied (a copy would wait for its load). Rows longer than KC entries
// finish in a plain per-entry loop (correct for any CSR; slow, and not the
// shape this kernel is chosen for). Replaces cupy's cuSPARSE csrmv of
// /root/reference/v3/gpu/common.py:119 (MultiGpu.dot) for such shards.
#pragma once

namespace kr {
namespace {

// KC entries per lane from the row's aligned chunks: NVL double2 loads cover
// 2*NVL >= KC + 1 entries from the even entry at or below the row start, NCL
// int4 loads 4*NCL >= KC + 3 from the multiple of 4 at or below it.
template <int KC>
struct DirectShape {
  static constexpr int NVL = (KC + 2) / 2;
  static constexpr int NCL = (KC + 6) / 4;
  static_assert(2 * NVL >= KC + 1 && 4 * NCL >= KC + 3, "chunk cover");
};

template <int KC>
struct DirectSet {
  dbl2v v[DirectShape<KC>::NVL];
  int4v c[DirectShape<KC>::NCL];
  int64_t rlo = 0, rhi = 0;  // this set's row range (row pointers)
  int64_t row = 0;           // this set's row (clamped to a real row)
  bool active = false;
};

// Issue the value and column loads of a lane's row [rlo, rhi): chunk q is
// clamped to the chunk holding the row's last entry, so no load leaves the
// row's own 16-byte chunks (an empty row re-reads the chunk of entry
// max(rhi - 1, 0), which exists: the dispatch needs >= 4 entries).
template <int KC, bool NT>
__device__ __forceinline__ void direct_load(DirectSet<KC>& s, const double* __restrict__ val,
                                            const int32_t* __restrict__ col) {
  using S = DirectShape<KC>;
  const int64_t last = max(s.rhi - 1, (int64_t)0);
  const int64_t va = s.rlo & ~(int64_t)1, vl = last & ~(int64_t)1;
#pragma unroll
  for (int q = 0; q < S::NVL; ++q) {
    const dbl2v* p = reinterpret_cast<const dbl2v*>(val + min(va + 2 * q, vl));
    if constexpr (NT)
      s.v[q] = __builtin_nontemporal_load(p);
    else
      s.v[q] = *p;
  }
  const int64_t ca = s.rlo & ~(int64_t)3, cl = last & ~(int64_t)3;
#pragma unroll
  for (int q = 0; q < S::NCL; ++q) {
    const int4v* p = reinterpret_cast<const int4v*>(col + min(ca + 4 * q, cl));
    if constexpr (NT)
      s.c[q] = __builtin_nontemporal_load(p);
    else
      s.c[q] = *p;
  }
}

// Per-lane register selects through v_cndmask with the wave's lane mask: a
// plain `c ? r[i + 1] : r[i]` over a register array is folded by the
// compiler into r[i + c], a dynamic index that moves the array to memory.
__device__ __forceinline__ uint32_t pick32(uint64_t m, uint32_t t, uint32_t f) {
  uint32_t r;
  asm volatile("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
  return r;
}
__device__ __forceinline__ double pick64(uint64_t m, double t, double f) {
  const uint64_t tb = (uint64_t)__double_as_longlong(t), fb = (uint64_t)__double_as_longlong(f);
  const uint64_t lo = pick32(m, (uint32_t)tb, (uint32_t)fb);
  const uint64_t hi = pick32(m, (uint32_t)(tb >> 32), (uint32_t)(fb >> 32));
  return __longlong_as_double((long long)(lo | hi << 32));
}

template <typename RP, int EPI, int KC, bool NT, int AB = 0>
__global__ __launch_bounds__(kBlock) void spmv_kernel_direct(SpmvArgs a) {
  if (!spmv_entry<EPI>(a)) return;  // converged / the fused scalar step's test fired
  using T = EpiTraits<EPI>;
  using S = DirectShape<KC>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  constexpr bool VIRT = is_virtual<EPI>();
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
  // the lane's row of visit jj (clamped to the last row; jj past the end
  // re-uses the last visit, so every path issues the same loads)
  const int64_t jlast = sched.j0 + ((jcount - 1 - sched.j0) / jstep) * jstep;
  auto set_row = [&](DirectSet<KC>& s, int64_t jj) __attribute__((always_inline)) {
    const int64_t r = sched.rb(min(jj, jlast)) * kBlock + tid;
    s.active = jj <= jlast && r < a.n;
    s.row = min(r, a.n - 1);
  };
  auto load_rp = [&](DirectSet<KC>& s) __attribute__((always_inline)) {
    s.rlo = (int64_t)rowptr[s.row];
    s.rhi = (int64_t)rowptr[s.row + 1];
  };


  // prologue: visit j0's row range and stream, visit j0 + jstep's row range
  DirectSet<KC> A, B;
  int64_t j = sched.j0;
  set_row(A, j);
  load_rp(A);
  direct_load<KC, NT>(A, val, col);
  set_row(B, j + jstep);
  load_rp(B);

  auto step = [&](DirectSet<KC>& cur, DirectSet<KC>& nxt) __attribute__((always_inline)) {
    const int64_t row = cur.row;
    const bool active = cur.active;
    const int64_t xrow = a.xoff + row;
    const int64_t len = cur.rhi - cur.rlo;
    double v[KC], p1[KC], p2[KC], p3[VIRT ? KC : 1];
    {
      double vv[2 * S::NVL];
      int32_t cc[4 * S::NCL];
#pragma unroll
      for (int q = 0; q < S::NVL; ++q) {
        vv[2 * q] = cur.v[q].x;
        vv[2 * q + 1] = cur.v[q].y;
      }
#pragma unroll
      for (int q = 0; q < S::NCL; ++q) {
        cc[4 * q] = cur.c[q].x;
        cc[4 * q + 1] = cur.c[q].y;
        cc[4 * q + 2] = cur.c[q].z;
        cc[4 * q + 3] = cur.c[q].w;
      }
      const uint64_t m1 = __builtin_amdgcn_ballot_w64((cur.rlo & 1) != 0);
      const uint64_t m2 = __builtin_amdgcn_ballot_w64((cur.rlo & 2) != 0);
#pragma unroll
      for (int u = 0; u < KC; ++u) {
        v[u] = pick64(m1, vv[u + 1], vv[u]);
        const uint32_t c01 = pick32(m1, (uint32_t)cc[u + 1], (uint32_t)cc[u]);
        const uint32_t c23 = pick32(m1, (uint32_t)cc[u + 3], (uint32_t)cc[u + 2]);
        const int32_t cu = (int32_t)pick32(m2, c23, c01);
        const int64_t c = (u < len && AB != 3) ? (int64_t)cu : xrow;
        if constexpr (AB == 1) {
          p1[u] = v[u] + (double)cu;
          p2[u] = v[u];
          continue;
        }
        p1[u] = x1[c];
        if constexpr (NV == 2 || VIRT) p2[u] = x2[c];
        if constexpr (VIRT) p3[u] = a.x3[c];
      }
    }
    const EpiIn pin = epi_load<EPI>(a, row);
    const int64_t rlo = cur.rlo, rhi = cur.rhi;
    // the next visit's stream (its row range arrived one visit ago), then
    // the row range two visits ahead into this set (its columns are used)
    direct_load<KC, NT>(nxt, val, col);
    set_row(cur, j + 2 * jstep);
    load_rp(cur);
    double sum1 = 0.0, sum2 = 0.0;
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      if (u < len) {
        if constexpr (VIRT) {
          sum1 = sum1 + v[u] * virt_in<EPI>(a, p1[u], p2[u], p3[u]);
        } else {
          sum1 = sum1 + v[u] * p1[u];
          if constexpr (NV == 2) sum2 = sum2 + v[u] * p2[u];
        }
      }
    }
    if (len > KC) {  // rows longer than KC: the rest entry by entry, in order
      for (int64_t e = rlo + KC; e < rhi; ++e) {
        const double ve = val[e];
        const int64_t c = col[e];
        if constexpr (VIRT) {
          sum1 = sum1 + ve * virt_in<EPI>(a, x1[c], x2[c], a.x3[c]);
        } else {
          sum1 = sum1 + ve * x1[c];
          if constexpr (NV == 2) sum2 = sum2 + ve * x2[c];
        }
      }
    }
    if constexpr (AB == 2) {
      const EpiVals o = epi_values<EPI>(a, sum1, sum2, pin, acc);
      acc[0] += o.y1 + o.y2;
    } else {
      if (active) epi_row_in<EPI>(a, row, sum1, sum2, x1, x2, pin, acc);
    }
    j += jstep;
  };

  for (;;) {
    step(A, B);
    if (j >= jcount) break;
    step(B, A);
    if (j >= jcount) break;
  }
  __syncthreads();
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
}


// ---------------------------------------------------------------------------
// CSR row walk v3 (spmv_kernel3): spmv_kernel2's LDS-staged row walk for the
// plain column stream, cut down to the vector-memory bytes it REQUESTS. The
// plain-CSR dual SpMV is bound by the texture-address unit, not by HBM: each
// CU's TA takes about 16 bytes of load/store request per clock whether the
// bytes hit a cache or not (PMC over tools/micro/csr_micro: TA_BUSY 94 % of
// the launch, 16.5 B per TA cycle for spmv_kernel2 and the LDS-free walk
// alike), and spmv_kernel2 requests ~248 B per row against the 120 B the row
// needs from HBM. So every requested byte the row does not need is time:
//   FL & 1 (DIAG): the epilogue's own-row inputs x1[row], x2[row] (x3 for
//     the fused first steps) are the gathered values of the row's diagonal
//     entry, picked when the gathers are summed; a row without a stored
//     diagonal entry (or whose diagonal lies past its first gather batch)
//     loads them as before. -16 B per row on a dual.
//   FL & 2 (RP1): one row-pointer load per lane; the row's end is the next
//     lane's start (DPP wave_shl:1), the wave's last lane takes it through
//     the scalar cache. -4 B per row.
//   FL & 4 (BUF): the staging loads are buffer loads on a descriptor that
//     ends at the window's last entry, so the slots past it (kernel2 re-reads
//     the last chunk to keep the load count fixed) return 0 without a memory
//     request. Same instruction count on every path (vmcnt stays exact).
// Same arithmetic in the same order as spmv_kernel2: bitwise scipy.
// ---------------------------------------------------------------------------
template <typename RP>
__device__ __forceinline__ RP rp_next_lane(RP v, RP last) {  // lane t <- lane t+1; lane 63 <- last
  if constexpr (sizeof(RP) == 8) {
    const uint64_t b = (uint64_t)v, o = (uint64_t)last;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)o, (int)(uint32_t)b,
                                                              0x130, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(o >> 32),
                                                              (int)(uint32_t)(b >> 32), 0x130, 0xF,
                                                              0xF, false);
    return (RP)((uint64_t)lo | (uint64_t)hi << 32);
  } else {
    return (RP)__builtin_amdgcn_update_dpp((int)last, (int)v, 0x130, 0xF, 0xF, false);
  }
}

// Lane t's value <- lane t ^ 1's (DPP quad_perm [1,0,3,2]).
__device__ __forceinline__ double dpp_xor1(double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)b, 0xB1, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), 0xB1, 0xF, 0xF, false);
  return __longlong_as_double((long long)((uint64_t)lo | (uint64_t)hi << 32));
}

// The epilogue's own-row stores as 16-byte row pairs (spmv_kernel3 FL & 8):
// lanes 2t, 2t+1 own rows row, row + 1 (row even); for the vectors A, B of a
// pair, the even lane stores (A[row], A[row+1]) and the odd lane (B[row],
// B[row+1]) after one DPP exchange, so the wave stores two vectors with ONE
// 16-byte instruction instead of two 8-byte ones (the same bytes, half the
// store instructions through the texture-address unit). Whole waves only
// (every lane a real row); the same values as epi_store_row.
template <int EPI, bool NT>
__device__ __forceinline__ void epi_store_lane_pairs(const SpmvArgs& a, int64_t row,
                                                     const EpiVals& o) {
  double* dst[5] = {};
  double v[5] = {};
  int k = 0;
  if constexpr (is_step<EPI>()) {
    if constexpr (epi_writes_ud<EPI>()) { dst[k] = a.ud; v[k++] = o.ud; }
    dst[k] = a.u1; v[k++] = o.u1;
    dst[k] = a.u2; v[k++] = o.u2;
    dst[k] = a.y1; v[k++] = o.y1;
    if constexpr (EPI == EPI_MRR_V) { dst[k] = a.y2; v[k++] = o.y2; }
  } else {
    if constexpr (EpiTraits<EPI>::NV == 2)
      if (a.products_only) return;
    dst[k] = a.y1; v[k++] = o.y1;
    if constexpr (EpiTraits<EPI>::NV == 2) { dst[k] = a.y2; v[k++] = o.y2; }
    if constexpr (EPI == EPI_XY_VP) { dst[k] = a.u1; v[k++] = o.u1; }
  }
  const bool odd = (threadIdx.x & 1) != 0;
#pragma unroll
  for (int i = 0; i < 5; i += 2) {
    if (i >= k) break;
    const double va = v[i], pa = dpp_xor1(va);
    if (i + 1 < k) {
      const double vb = v[i + 1], pb = dpp_xor1(vb);
      double* p = odd ? dst[i + 1] + (row - 1) : dst[i] + row;
      const dbl2v w = odd ? dbl2v{pb, vb} : dbl2v{va, pa};
      if constexpr (NT)
        __builtin_nontemporal_store(w, reinterpret_cast<dbl2v*>(p));
      else
        *reinterpret_cast<dbl2v*>(p) = w;
    } else if (!odd) {
      const dbl2v w = dbl2v{va, pa};
      if constexpr (NT)
        __builtin_nontemporal_store(w, reinterpret_cast<dbl2v*>(dst[i] + row));
      else
        *reinterpret_cast<dbl2v*>(dst[i] + row) = w;
    }
  }
}

template <typename RP, int EPI, int FL>
__global__ __launch_bounds__(kBlock) void spmv_kernel3(SpmvArgs a) {
  if (!spmv_entry<EPI>(a)) return;  // converged / the fused scalar step's test fired
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  constexpr bool VIRT = is_virtual<EPI>();
  constexpr int G = kGather;
  constexpr bool DIAG = (FL & 1) != 0, RP1 = (FL & 2) != 0, BUF = (FL & 4) != 0;
  constexpr bool PAIRS = (FL & 8) != 0, NTS = (FL & 16) != 0;
  // single-row stores: FL & 16 non-temporal, FL & 32 sc1 (agent-scope relaxed atomics)
  constexpr int SK = (FL & 32) ? 2 : NTS ? 1 : 0;
  // timing-only ablations (wrong results): FL & 64 no stores, FL & 128 no
  // x gathers (the staged value stands in); FL & 256: one LDS buffer (a
  // second barrier per window, half the LDS)
  constexpr bool AB_NOST = (FL & 64) != 0, AB_NOG = (FL & 128) != 0, SB = (FL & 256) != 0;
  constexpr int NB = SB ? 1 : 2;
  // own-row operands the diagonal gather provides (epi_load NOX bits)
  constexpr bool NEED_X = is_step<EPI>() || T::kX;
  constexpr bool NEED_X2 = T::kX2 || is_vstep<EPI>();
  constexpr bool NEED_X3 = is_vstep<EPI>();
  constexpr int NOX = DIAG ? ((NEED_X ? 1 : 0) | (NEED_X2 ? 2 : 0) | (NEED_X3 ? 4 : 0)) : 0;
  __shared__ __attribute__((aligned(16))) double s_val[NB][kWindow];
  __shared__ __attribute__((aligned(16))) int32_t s_col[NB][kWindow];
  __shared__ double s_red[(NP > 0 ? NP : 1) * 4];

  const RP* __restrict__ rowptr = static_cast<const RP*>(a.rowptr);
  const double* __restrict__ val = a.val;
  const int32_t* __restrict__ col = a.col;
  const double* __restrict__ x1 = a.x1;
  const double* __restrict__ x2 = a.x2;
  const int tid = threadIdx.x;
  const int64_t wlast = 64 * (tid / 64) + 64;  // the row after this wave's last (block-relative)

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
  auto wstart = [](int64_t e) { return e & ~(int64_t)3; };
  // the lane's row range of the block starting at row r: [lo, hi)
  auto lane_rp = [&](int64_t r, RP& lo, RP& hi) {
    if constexpr (RP1) {
      lo = rowptr[min(r + tid, a.n)];
      hi = load_uniform(rowptr, min(r + wlast, a.n));  // lane 63's end (scalar cache)
    } else {
      const int64_t ri = min(r + tid, a.n - 1);
      lo = rowptr[ri];
      hi = rowptr[ri + 1];
    }
  };

  int64_t r0 = sched.rb(j) * kBlock;
  int nr = block_rows(sched.rb(j));
  int64_t bs = (int64_t)load_uniform(rowptr, r0);
  int64_t be = (int64_t)load_uniform(rowptr, r0 + nr);
  RP rlo = 0, rhi = 0;
  lane_rp(r0, rlo, rhi);
  int64_t bsn = 0, ben = 0;
  if (j + jstep < jcount) {
    const int64_t rbn = sched.rb(j + jstep);
    bsn = (int64_t)load_uniform(rowptr, rbn * kBlock);
    ben = (int64_t)load_uniform(rowptr, rbn * kBlock + block_rows(rbn));
  }
  Stage st;
  int64_t ws = wstart(bs);
  // the staging loads of the window [w, w + kWindow) of a block ending at hi
  auto stage = [&](int64_t w, int64_t hi) {
    if constexpr (BUF) {
      const int64_t cnt = min(hi - w, (int64_t)kWindow);  // entries of the window in use
      const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<double*>(val + w), 0, (int)(((cnt + 1) & ~(int64_t)1) * 8), 0x00020000);
      const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<int32_t*>(col + w), 0, (int)(((cnt + 3) & ~(int64_t)3) * 4), 0x00020000);
#pragma unroll
      for (int q = 0; q < kVSlots; ++q)
        st.v[q] = __builtin_bit_cast(
            dbl2v, __builtin_amdgcn_raw_buffer_load_b128(rv, (uint32_t)(tid + q * kBlock) * 16u, 0, 2));
#pragma unroll
      for (int q = 0; q < kCSlots; ++q)
        st.c[q] = __builtin_bit_cast(
            int4v, __builtin_amdgcn_raw_buffer_load_b128(rc, (uint32_t)(tid + q * kBlock) * 16u, 0, 2));
    } else {
      stage_load2<true, true>(st, val, col, w, hi, tid);
    }
  };
  stage(ws, be);
  int buf = 0;
  bool first_window = true;
  EpiIn pin;
  double sum1 = 0.0, sum2 = 0.0;
  bool found = false;  // DIAG: the row's diagonal gather was seen
  double xo1 = 0.0, xo2 = 0.0, xo3 = 0.0;
  int64_t r0n = 0;
  RP rlo_n = 0, rhi_n = 0;
  int nrn = 0;

  for (;;) {
    const double* sv = s_val[SB ? 0 : buf];
    int32_t* sc = s_col[SB ? 0 : buf];
    stage_commit<true>(st, s_val[SB ? 0 : buf], sc, tid);
    __syncthreads();
    const bool active = tid < nr;
    const int64_t row = r0 + (active ? tid : 0);
    if (first_window) {
      pin = epi_load<EPI, NOX>(a, row);
      found = false;
    }
    // RP1: the row's end is the next lane's start (the wave's last lane: hi)
    const int64_t lo = (int64_t)rlo;
    const int64_t hi_ = RP1 ? (int64_t)rp_next_lane<RP>(rlo, rhi) : (int64_t)rhi;
    const int64_t off = bs - ws;
    const int js = active ? (int)max(lo - bs + off, (int64_t)0) : 0;
    const int je = active ? (int)min(hi_ - bs + off, (int64_t)kWindow) : 0;
    const int64_t xrow = a.xoff + row;

    // (1) first gather batch of this window
    double v[G], p1[G], p2[G], p3[VIRT ? G : 1];
    int64_t cg[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const bool ok = js + u < je;
      v[u] = sv[ok ? js + u : 0];
      const int64_t c = sc[ok ? js + u : 0];
      cg[u] = ok ? c : -1;
      if constexpr (AB_NOG) {
        p1[u] = v[u] + (double)c;
        p2[u] = v[u];
        if constexpr (VIRT) p3[u] = v[u];
        continue;
      }
      p1[u] = x1[c];
      if constexpr (NV == 2 || VIRT) p2[u] = x2[c];
      if constexpr (VIRT) p3[u] = a.x3[c];
    }

    // (2) the next window's loads (same count on every path)
    const bool last_window = ws + kWindow >= be;
    const int64_t j_next = j + jstep;
    const bool has_next = j_next < jcount;
    {
      const bool nb = last_window && has_next;
      const int64_t nws = !last_window ? ws + kWindow : nb ? wstart(bsn) : ws;
      stage(nws, nb ? ben : be);
      if (nb) {
        const int64_t rb_next = sched.rb(j_next);
        r0n = rb_next * kBlock;
        nrn = block_rows(rb_next);
      }
      lane_rp(nb ? r0n : r0, rlo_n, rhi_n);
    }

    // (3) sums in stored order; DIAG: the diagonal's gathered inputs
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
      if constexpr (DIAG) {
        const bool d = cg[u] == xrow;
        xo1 = d ? p1[u] : xo1;
        if constexpr (NV == 2 || VIRT) xo2 = d ? p2[u] : xo2;
        if constexpr (VIRT) xo3 = d ? p3[u] : xo3;
        found = found || d;
      }
    }
    if (je - js > G) {
      uint32_t no_mask = 0;  // (column window: the mask argument is unused)
      if constexpr (VIRT)
        row_window_virtual<EPI, G>(sv, sc, nullptr, 0, a, js + G, je, no_mask, sum1);
      else
        row_window<NV, G>(sv, sc, x1, x2, js + G, je, sum1, sum2);
    }
    buf ^= 1;
    if constexpr (SB) __syncthreads();  // the single buffer is rewritten next
    if (!last_window) {
      ws += kWindow;
      first_window = false;
      continue;
    }
    // PAIRS: whole waves store row pairs (every lane of the wave a real row)
    const bool wave_full = PAIRS && nr >= (int)wlast;
    if (active || wave_full) {
      if constexpr (DIAG) {
        if (found) {
          if constexpr (NEED_X) pin.x = xo1;
          if constexpr (NEED_X2) pin.x2 = xo2;
          if constexpr (NEED_X3) pin.e = xo3;
        } else {  // no stored diagonal in the first batch: load as epi_load does
          if constexpr (NEED_X) pin.x = x1[xrow];
          if constexpr (NEED_X2) pin.x2 = x2[xrow];
          if constexpr (NEED_X3) pin.e = a.x3[xrow];
        }
      }
      if constexpr (AB_NOST) {
        const EpiVals o = epi_values<EPI>(a, sum1, sum2, pin, acc);
        acc[0] += o.y1 + o.y2 + o.u1 + o.u2 + o.ud;
      } else if constexpr (PAIRS) {
        const EpiVals o = epi_values<EPI>(a, sum1, sum2, pin, acc);
        if (wave_full)
          epi_store_lane_pairs<EPI, NTS>(a, row, o);
        else
          epi_store_row<EPI>(a, row, o);
      } else {
        epi_store_row_k<EPI, SK>(a, row, epi_values<EPI>(a, sum1, sum2, pin, acc));
      }
    }
    if (!has_next) break;
    j = j_next;
    r0 = r0n;
    nr = nrn;
    bs = bsn;
    be = ben;
    rlo = rlo_n;
    rhi = rhi_n;
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

// ---------------------------------------------------------------------------
// CSR row walk v4 (spmv_kernel4, round 5 experiment): spmv_kernel3 with the
// matrix stream staged TWO windows ahead in two register sets (unrolled x2,
// no register copy), so a window's loads are in flight across two visits
// instead of one; for shards whose row blocks fit one window each (the host
// checks the largest block). vmcnt completes in order: visit t issues the
// gathers of t, then the stage loads of t + 2, and its gather wait then also
// retires the stage loads of t + 1, issued one visit earlier.
// ---------------------------------------------------------------------------
template <typename RP>
struct Blk {  // one row block's visit: uniform bounds + the lane's row range
  int64_t r0 = 0, bs = 0, be = 0;
  int nr = 0;
  RP lo = 0, hi = 0;
  bool valid = false;
};

template <typename RP, int EPI, int FL>
__global__ __launch_bounds__(kBlock) void spmv_kernel4(SpmvArgs a) {
  if (!spmv_entry<EPI>(a)) return;
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  constexpr bool VIRT = is_virtual<EPI>();
  constexpr int G = kGather;
  constexpr bool AB_NOST = (FL & 64) != 0, AB_NOG = (FL & 128) != 0;
  __shared__ __attribute__((aligned(16))) double s_val[2][kWindow];
  __shared__ __attribute__((aligned(16))) int32_t s_col[2][kWindow];
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
  // bounds of visit jj (an invalid visit past the end re-uses the last
  // valid one's block: every path issues the same loads)
  const int64_t jlast = sched.j0 + ((jcount - 1 - sched.j0) / jstep) * jstep;
  auto bounds = [&](Blk<RP>& b, int64_t jj) __attribute__((always_inline)) {
    b.valid = jj < jcount;
    const int64_t rb = sched.rb(min(jj, jlast));
    b.r0 = rb * kBlock;
    b.nr = (int)min((int64_t)kBlock, a.n - b.r0);
    b.bs = (int64_t)load_uniform(rowptr, b.r0);
    b.be = (int64_t)load_uniform(rowptr, b.r0 + b.nr);
  };
  auto lane_rp = [&](Blk<RP>& b) __attribute__((always_inline)) {
    const int64_t ri = min(b.r0 + tid, a.n - 1);
    b.lo = rowptr[ri];
    b.hi = rowptr[ri + 1];
  };
  auto stage = [&](Stage& st, const Blk<RP>& b) __attribute__((always_inline)) {
    stage_load2<true, true>(st, val, col, b.bs & ~(int64_t)3, b.be, tid);
  };

  Stage sA, sB;
  Blk<RP> bA, bB, bN;  // visits t, t + 1 (staged), t + 2 (bounds)
  int64_t j = sched.j0;
  bounds(bA, j);
  lane_rp(bA);
  stage(sA, bA);
  bounds(bB, j + jstep);
  lane_rp(bB);
  stage(sB, bB);
  bounds(bN, j + 2 * jstep);
  int buf = 0;

  auto visit = [&](Stage& st, Blk<RP>& b) __attribute__((always_inline)) {
    stage_commit<true>(st, s_val[buf], s_col[buf], tid);
    __syncthreads();
    const double* sv = s_val[buf];
    const int32_t* sc = s_col[buf];
    const Blk<RP> cur = b;  // this visit (b is refilled below with visit t + 2)
    const bool active = tid < cur.nr && cur.valid;
    const int64_t row = cur.r0 + (active ? tid : 0);
    const EpiIn pin = epi_load<EPI>(a, row);
    const int64_t ws = cur.bs & ~(int64_t)3;
    const int js = active ? (int)((int64_t)cur.lo - ws) : 0;
    const int je = active ? (int)((int64_t)cur.hi - ws) : 0;
    double v[G], p1[G], p2[G], p3[VIRT ? G : 1];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const bool ok = js + u < je;
      v[u] = sv[ok ? js + u : 0];
      const int64_t c = sc[ok ? js + u : 0];
      if constexpr (AB_NOG) {
        p1[u] = v[u] + (double)c;
        p2[u] = v[u];
        if constexpr (VIRT) p3[u] = v[u];
        continue;
      }
      p1[u] = x1[c];
      if constexpr (NV == 2 || VIRT) p2[u] = x2[c];
      if constexpr (VIRT) p3[u] = a.x3[c];
    }
    // visit t + 2 into this set: its bounds were read one visit ago
    b = bN;
    lane_rp(b);
    stage(st, b);
    bounds(bN, j + 3 * jstep);
    double sum1 = 0.0, sum2 = 0.0;
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
      uint32_t no_mask = 0;
      if constexpr (VIRT)
        row_window_virtual<EPI, G>(sv, sc, nullptr, 0, a, js + G, je, no_mask, sum1);
      else
        row_window<NV, G>(sv, sc, x1, x2, js + G, je, sum1, sum2);
    }
    if (active) {
      const EpiVals o = epi_values<EPI>(a, sum1, sum2, pin, acc);
      if constexpr (AB_NOST)
        acc[0] += o.y1 + o.y2 + o.u1 + o.u2 + o.ud;
      else
        epi_store_row_k<EPI, 1>(a, row, o);
    }
    buf ^= 1;
    j += jstep;
  };
  for (;;) {
    visit(sA, bA);
    if (j >= jcount) break;
    visit(sB, bB);
    if (j >= jcount) break;
  }
  __syncthreads();
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
}

}  // namespace
}  // namespace kr

namespace kr {
namespace {

// ---------------------------------------------------------------------------
// CSR row walk v5 (spmv_kernel5, round 5 experiment): the x gathers software-
// pipelined one row block ahead. Visit t commits block t+1's staged window,
// reads its values and columns out of LDS into registers and issues its x
// gathers, issues the staging loads of block t+2, and only then sums block t
// from the values and gathers it read one visit earlier -- so a gather's
// latency and the staging's both overlap a whole visit of work instead of
// the gathers' being waited for in the visit that issued them. Two register
// sets (values + gathers) alternate (loop unrolled x2); one window per block
// (the host checks the largest block); rows longer than G entries finish
// from the LDS window, behind one more barrier in the visits that have them.
// ---------------------------------------------------------------------------
template <int NV, bool VL = false>
struct GSet {
  double v[VL ? 1 : kGather], p1[kGather], p2[NV == 2 ? kGather : 1];
  int js = 0, je = 0;
  int64_t row = 0;
  bool active = false;
  EpiIn pin;
};

// VL: the values are read from the LDS window when the block is finished
// (not kept in registers across the visit: 14 VGPRs per set fewer), which
// needs a second barrier per visit (the window must outlive every wave's
// finish before the next commit overwrites it).
template <typename RP, int EPI, bool VL = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3))) void spmv_kernel5(SpmvArgs a) {
  if (!spmv_entry<EPI>(a)) return;
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;
  constexpr int G = kGather;
  static_assert(!is_virtual<EPI>(), "experiment: plain inputs only");
  __shared__ __attribute__((aligned(16))) double s_val[2][kWindow];
  __shared__ __attribute__((aligned(16))) int32_t s_col[2][kWindow];
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
  const int64_t jlast = sched.j0 + ((jcount - 1 - sched.j0) / jstep) * jstep;
  auto bounds = [&](Blk<RP>& b, int64_t jj) __attribute__((always_inline)) {
    b.valid = jj < jcount;
    const int64_t rb = sched.rb(min(jj, jlast));
    b.r0 = rb * kBlock;
    b.nr = (int)min((int64_t)kBlock, a.n - b.r0);
    b.bs = (int64_t)load_uniform(rowptr, b.r0);
    b.be = (int64_t)load_uniform(rowptr, b.r0 + b.nr);
  };
  auto lane_rp = [&](Blk<RP>& b) __attribute__((always_inline)) {
    const int64_t ri = min(b.r0 + tid, a.n - 1);
    b.lo = rowptr[ri];
    b.hi = rowptr[ri + 1];
  };
  Stage st;
  auto stage = [&](const Blk<RP>& b) __attribute__((always_inline)) {
    stage_load2<true, true>(st, val, col, b.bs & ~(int64_t)3, b.be, tid);
  };

  // gathers of block b from LDS buffer `buf` into set g (b's window committed)
  auto gather = [&](GSet<NV, VL>& g, const Blk<RP>& b, int buf) __attribute__((always_inline)) {
    const double* sv = s_val[buf];
    const int32_t* sc = s_col[buf];
    g.active = tid < b.nr && b.valid;
    g.row = b.r0 + (g.active ? tid : 0);
    const int64_t ws = b.bs & ~(int64_t)3;
    g.js = g.active ? (int)((int64_t)b.lo - ws) : 0;
    g.je = g.active ? (int)((int64_t)b.hi - ws) : 0;
    g.pin = epi_load<EPI>(a, g.row);
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const bool ok = g.js + u < g.je;
      if constexpr (!VL) g.v[u] = sv[ok ? g.js + u : 0];
      const int64_t c = sc[ok ? g.js + u : 0];
      g.p1[u] = x1[c];
      if constexpr (NV == 2) g.p2[u] = x2[c];
    }
    (void)sv;
  };
  // sums + epilogue of the block whose gathers are in g (window still in `buf`)
  auto finish = [&](GSet<NV, VL>& g, int buf) __attribute__((always_inline)) {
    double sum1 = 0.0, sum2 = 0.0;
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const bool ok = g.js + u < g.je;
      const double vu = VL ? s_val[buf][ok ? g.js + u : 0] : g.v[VL ? 0 : u];
      if (ok) {
        sum1 = sum1 + vu * g.p1[u];
        if constexpr (NV == 2) sum2 = sum2 + vu * g.p2[u];
      }
    }
    if (g.je - g.js > G) row_window<NV, G>(s_val[buf], s_col[buf], x1, x2, g.js + G, g.je, sum1, sum2);
    if (g.active)
      epi_store_row_k<EPI, 1>(a, g.row, epi_values<EPI>(a, sum1, sum2, g.pin, acc));
  };

  // prologue: block t0 staged + committed + gathered; block t0+1 staged
  Blk<RP> b0, b1, b2;
  int64_t j = sched.j0;
  bounds(b0, j);
  lane_rp(b0);
  stage(b0);
  bounds(b1, j + jstep);
  lane_rp(b1);
  GSet<NV, VL> gA, gB;
  stage_commit<true>(st, s_val[0], s_col[0], tid);
  int lng = __syncthreads_or(b0.valid && tid < b0.nr && (int64_t)(b0.hi - b0.lo) > G);
  gather(gA, b0, 0);
  stage(b1);
  bounds(b2, j + 2 * jstep);
  int buf = 0;  // LDS buffer of the block being finished

  // visit: finish the block in `cur` (window in buf), gather the next one
  // (its stage arrives now) into `nxt`
  auto visit = [&](GSet<NV, VL>& cur, GSet<NV, VL>& nxt) __attribute__((always_inline)) {
    const int nb = buf ^ 1;
    stage_commit<true>(st, s_val[nb], s_col[nb], tid);
    const int lng_n =
        __syncthreads_or(b1.valid && tid < b1.nr && (int64_t)(b1.hi - b1.lo) > G);
    gather(nxt, b1, nb);
    // the stage of the block after next (its bounds read one visit ago)
    b1 = b2;
    lane_rp(b1);
    stage(b1);
    bounds(b2, j + 3 * jstep);
    finish(cur, buf);
    // a long row read the finished window from LDS: nobody may overwrite it
    // (the next commit targets it) before every wave is done
    if (VL || lng) __syncthreads();
    lng = lng_n;
    buf = nb;
    j += jstep;
  };
  for (;;) {
    visit(gA, gB);
    if (j >= jcount) break;
    visit(gB, gA);
    if (j >= jcount) break;
  }
  __syncthreads();
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate);
}

}  // namespace
}  // namespace kr
