// CSR row walk without LDS (spmv_kernel_direct; included by kr_spmv.h).
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
// Included by kr_spmv.h inside namespace kr's anonymous namespace.
#pragma once

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

