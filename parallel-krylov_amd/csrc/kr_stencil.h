// Stencil SpMV (gfx950): the short-row kernel for offset-structured matrices
// with a value dictionary -- 3-D stencils such as the 512^3 / 256^3 Poisson
// systems of C4 / C2. Included by kr_spmv.h (inside kr::{anon}).
//
// Why a second short-row kernel. The row walk (spmv_kernel2) is bound by
// vector-memory ADDRESS work, not bytes (profiles/r01f/sq_ta_counters.txt:
// TA busy ~83 %, 42 % issue stalls): per row it issues 7 8-byte x gathers
// per input vector, two row-pointer loads, a mask and a code load, plus the
// own-row operands. This kernel issues, per PAIR of rows and input vector,
// about three 16-byte loads:
//
//  * Storage (SpmvArgs::scode): one uint64 per row = the dictionary codes of
//    the row's entries, byte k for offset M[k] (M ascending), 0xFF = no entry.
//    8 B/row instead of rowptr + mask + codes (12-13 B/row); no LDS staging.
//  * 2 rows per lane, 512-row blocks: every own-row access (codes, x, y, the
//    epilogue operands) is one 16-byte load/store per lane.
//  * Walk: workgroup (XCD q, plane segment s, position p) visits the blocks
//    p, p + P, p + 2P, ... of its planes (P = st_P blocks = W / 512 rows,
//    W = the stencil's largest offset, +-n^2 for a 3-D stencil). The rows
//    one walk step apart are the +-W neighbours, so x[row - W] (PREV) and
//    x[row] (CENTER) are the CENTER and NEXT values of the previous visit,
//    carried in registers: per visit only x[row + W] (NEXT) is new.
//  * Offsets |o| <= kSNear (+-1) are read from an LDS line of the block's
//    CENTER values (+ 2 edge values each side); any other offset (FAR: +-n)
//    is one 16-byte load per lane (even offsets only; the host checks).
//  * Software pipeline: the next visit's loads are issued before this
//    visit's sums (vector loads complete in order, see spmv_kernel2), one
//    workgroup barrier per visit (double-buffered line).
//
// Numerics: each row sums its entries in stored order (ascending offset =
// ascending column) from 0.0 with separately rounded products: bitwise
// scipy's csr_matvec, like every SpMV kernel here. The epilogue statements
// are epi_values (shared with the row walks). Dot-product partials: lane t
// adds row 2t's products, then row 2t+1's, visit after visit
// (oracle/gpu_order.py restates this order).
#pragma once

#ifndef KR_ST_W4
#define KR_ST_W4 4
#endif
// Ablations (timing-only library builds for same-box A/B, wrong results;
// never in the library build): bit 0 no result stores, 1 no products, 2 no
// value-table reads (the code itself as the value), 3 the NEAR (+-1)
// operands from the own row (no LDS line / DPP reads).
#ifndef KR_ST_AB
#define KR_ST_AB 0
#endif
constexpr int kSBlock = kStencilBlock;  // rows per stencil row block (2 per lane)
constexpr int kSNear = 2;            // LDS line halo (offsets 0 < |o| <= kSNear)
constexpr int kSLine = kSBlock + 2 * kSNear;
constexpr int kSFarMax = 4;          // FAR offsets (one 16-byte load each)

// Slot kinds (SpmvArgs::st_kind): the source of x[row + M[k]].
enum StencilKind : int {
  SK_CENTER = 0,  // o == 0: carried
  SK_PREV = 1,    // o == -W: carried
  SK_NEXT = 2,    // o == +W: loaded, carried to the next visit as CENTER
  SK_NEAR = 3,    // 0 < |o| <= kSNear: LDS line
  SK_FAR = 4,     // SK_FAR + f: FAR load f
};

// 16-byte load of x[i], x[i+1] (i even), clamped into [0, xlen - 2]: lanes
// past the last row and neighbours past the vector ends read a valid pair
// that is never used (their codes say 0xFF / the row is inactive).
__device__ __forceinline__ dbl2v st_ld2(const double* __restrict__ x, int64_t i, int64_t xlen) {
  i = min(max(i, (int64_t)0), xlen - 2);
  return *reinterpret_cast<const dbl2v*>(x + i);
}

// x at (row + o) for both rows of the lane.
struct SPair {
  double lo, hi;
};

// One visit's prefetched loads.
template <int NX, int NFAR, int CB = 8>
struct SStage {
  using Code = typename std::conditional<CB == 8, uint64_t, uint32_t>::type;
  Code clo, chi;              // codes of rows 2t, 2t+1
  dbl2v nxt[NX];              // x[row + W]
  dbl2v far[NFAR > 0 ? NFAR : 1][NX];
  dbl2v u1, u2, us, e;        // own-row epilogue operands (as the EPI needs)
  dbl2v cen[NX], prv[NX];     // RELOAD: x[row], x[row - W]
  dbl2v el[NX], er[NX];       // the line's edges x[r0-2..r0-1], x[r0+512..r0+513] (uniform)
};

// Absent slots among the first nm of a row's code word (field all ones):
// bit CB k set for an absent slot k.
template <int CB, typename Code>
__device__ __forceinline__ Code st_absent_bits(Code c, int nm) {
  Code m = c;
#pragma unroll
  for (int b = 1; b < CB; ++b) m &= c >> b;
  Code low = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) low |= (k < nm) ? ((Code)1 << (CB * k)) : (Code)0;
  return m & low;
}

// Uniform 16-byte load through the scalar cache (s_load_dwordx4: counted by
// lgkmcnt, so it never lengthens a vector-memory wait). x is read-only while
// the kernel runs. i even, clamped like st_ld2.
__device__ __forceinline__ dbl2v st_ld2_uniform(const double* x, int64_t i, int64_t xlen) {
  i = min(max(i, (int64_t)0), xlen - 2);
  return load_uniform(reinterpret_cast<const dbl2v*>(x), i >> 1);
}

// Buffer resources of one launch (wave-uniform descriptors): the x vectors
// (xlen doubles each) and the codes (n rows). A buffer load takes a 32-bit
// byte offset = a uniform part (SGPR arithmetic) + the lane's constant part,
// and the hardware range check returns 0 for offsets past the buffer (a
// negative uniform part wraps past it too): no per-lane clamp or 64-bit
// address per load. Lanes whose offsets fall outside read 0; their values are
// never used (absent codes, lanes past the last row). The host keeps the
// stencil SpMV to shards with xlen * 8 < 2^31 (System::build_stencil).
struct SRes {
  __amdgpu_buffer_rsrc_t x[3];
  __amdgpu_buffer_rsrc_t code;
};

template <int NX, int CB>
__device__ __forceinline__ SRes st_res(const SpmvArgs& a, const double* const (&xs)[3],
                                       bool pat = false) {
  SRes r;
#pragma unroll
  for (int v = 0; v < NX; ++v)
    r.x[v] = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(xs[v]), 0,
                                               (int)(a.xlen * 8), 0x00020000);
  // codes: the pattern table (SpmvArgs::st_pid) or the per-row stream
  r.code = pat ? __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.st_pat), 0,
                                                   a.st_npat * kStencilBlock * CB, 0x00020000)
               : __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.scode), 0,
                                                   (int)(a.n * CB), 0x00020000);
  return r;
}

// 16 bytes at byte offset `off` of a buffer (aux 2: non-temporal).
template <int AUX = 0>
__device__ __forceinline__ dbl2v st_bld2(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(dbl2v, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
}

// Codes of rows 2t, 2t+1 at byte cbase + 2 CB t of the code buffer (lanes
// past the last row read 0: inactive). AUX 2: non-temporal (the per-row
// stream is read once); a pattern table is re-read by every block (AUX 0).
template <int CB, int AUX, typename Code>
__device__ __forceinline__ void st_codes(Code& clo, Code& chi, __amdgpu_buffer_rsrc_t r,
                                         uint32_t coff) {
  if constexpr (CB == 8) {
    typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
    const u64x2 c = __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(r, coff, 0, AUX));
    clo = c.x;
    chi = c.y;
  } else if constexpr (CB == 4) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 c = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, coff, 0, AUX));
    clo = c.x;
    chi = c.y;
  } else {  // CB == 2: both rows' uint16 codes in one dword
    const uint32_t c = __builtin_amdgcn_raw_buffer_load_b32(r, coff, 0, AUX);
    clo = c & 0xFFFFu;
    chi = c >> 16;
  }
}

// row0: the visit's first row (launch-relative, uniform); the lane's rows are
// row0 + 2 tid, row0 + 2 tid + 1 (may lie past the last own row: x loads use
// them as is -- rows past the own rows are halo rows, which the +-1
// neighbours of the last own rows need); rr: the lane's first row clamped to
// the own rows (own-row operands); cbase: byte offset of the block's codes
// (row0 * CB in the row stream, or its pattern's in the table: pat).
// LF (position pairs with the +-n lines from LDS, NTM bit 8): one FAR load,
// the pair's outer neighbour line at row offset fo, into far[0].
template <int EPI, bool RELOAD, int NTM, int NX, int NFAR, int CB>
__device__ __forceinline__ void st_issue(SStage<NX, NFAR, CB>& st, const SpmvArgs& a,
                                         const SRes& res, int64_t row0, int tid, int64_t rr,
                                         uint32_t cbase, bool pat, int64_t fo = 0) {
  constexpr bool LF = (NTM & 256) && (NTM & 64) && !RELOAD;
  using T = EpiTraits<EPI>;
  constexpr int kCodeAux = (NTM & 1) ? 2 : 0;  // codes: streamed once (non-temporal)
  // x offsets: uniform (xoff + row0 + o) * 8, plus 16 bytes per lane
  const int64_t ub = (a.xoff + row0) * 8;
  const uint32_t lb = (uint32_t)tid * 16u;
  const int64_t W = (int64_t)a.st_P * kSBlock;
#pragma unroll
  for (int v = 0; v < NX; ++v) st.nxt[v] = st_bld2(res.x[v], (uint32_t)(ub + W * 8) + lb);
  if constexpr (LF) {
#pragma unroll
    for (int v = 0; v < NX; ++v) st.far[0][v] = st_bld2(res.x[v], (uint32_t)(ub + fo * 8) + lb);
  } else {
#pragma unroll
    for (int f = 0; f < NFAR; ++f)
#pragma unroll
      for (int v = 0; v < NX; ++v)
        st.far[f][v] = st_bld2(res.x[v], (uint32_t)(ub + (int64_t)a.st_far[f] * 8) + lb);
  }
  if constexpr (is_step<EPI>()) {
    st.u1 = *reinterpret_cast<const dbl2v*>(a.u1 + rr);
    st.u2 = *reinterpret_cast<const dbl2v*>(a.u2 + rr);
    if constexpr (EPI == EPI_STEP_MRR_X2 || EPI == EPI_STEP_MRR_X || is_vstep<EPI>())
      st.us = *reinterpret_cast<const dbl2v*>(a.us + rr);
  } else if constexpr (EPI == EPI_BMINUS) {
    st.e = *reinterpret_cast<const dbl2v*>(a.b + rr);
  } else if constexpr (T::kE) {
    st.e = *reinterpret_cast<const dbl2v*>(a.e + rr);
  }
  if constexpr (RELOAD) {
#pragma unroll
    for (int v = 0; v < NX; ++v) {
      st.cen[v] = st_bld2(res.x[v], (uint32_t)ub + lb);
      st.prv[v] = st_bld2(res.x[v], (uint32_t)(ub - W * 8) + lb);
    }
  }
  // the codes last: with patterns (pat) the block's pattern id comes through
  // the scalar cache, and the wait for it then holds back no vector load
  const uint32_t coff = cbase + (uint32_t)tid * (2 * CB);
  if (pat)  // uniform; one code load on either path
    st_codes<CB, 0>(st.clo, st.chi, res.code, coff);
  else
    st_codes<CB, kCodeAux>(st.clo, st.chi, res.code, coff);
}

// The line's edge pairs (uniform: scalar loads, counted by lgkmcnt). Issued
// after the visit's barrier, whose lgkmcnt(0) would otherwise wait for them.
template <int NX, int NFAR, int CB>
__device__ __forceinline__ void st_issue_edges(SStage<NX, NFAR, CB>& st, const SpmvArgs& a,
                                               const double* const (&xs)[3], int64_t row0) {
#pragma unroll
  for (int v = 0; v < NX; ++v) {
    st.el[v] = st_ld2_uniform(xs[v], a.xoff + row0 - kSNear, a.xlen);
    st.er[v] = st_ld2_uniform(xs[v], a.xoff + row0 + kSBlock, a.xlen);
  }
}

// The +-1 neighbours without LDS (NTM bit 5, the 7-point pattern): inside a
// wave a lane's row 2t-1 is lane t-1's second row and its row 2t+2 lane
// t+1's first, moved by DPP wave shifts; the wave's two edge rows (128 w - 1
// and 128 w + 128 of the block) come through the scalar cache. No LDS line
// and no workgroup barrier per visit.
__device__ __forceinline__ double st_dpp_shr1(double v, double old) {  // lane t <- lane t-1
  const long long b = __builtin_bit_cast(long long, v), o = __builtin_bit_cast(long long, old);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, 0x138, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), 0x138, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (long long)(unsigned)lo | ((long long)hi << 32));
}
__device__ __forceinline__ double st_dpp_shl1(double v, double old) {  // lane t <- lane t+1
  const long long b = __builtin_bit_cast(long long, v), o = __builtin_bit_cast(long long, old);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)b, 0x130, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), 0x130, 0xF, 0xF, false);
  return __builtin_bit_cast(double, (long long)(unsigned)lo | ((long long)hi << 32));
}
template <int NX, int NFAR, int CB>
__device__ __forceinline__ void st_issue_wave_edges(SStage<NX, NFAR, CB>& st, const SpmvArgs& a,
                                                    const double* const (&xs)[3], int64_t row0,
                                                    int wave) {
  const int64_t r = row0 + 128 * (int64_t)wave;
#pragma unroll
  for (int v = 0; v < NX; ++v) {
    st.el[v] = st_ld2_uniform(xs[v], a.xoff + r - 2, a.xlen);    // rows r-2, r-1
    st.er[v] = st_ld2_uniform(xs[v], a.xoff + r + 128, a.xlen);  // rows r+128, r+129
  }
}

// Own-row epilogue of one row from the carried centers (x, x2 / r0, y0, Ar1)
// and the staged operands: the values epi_row_in stores, without the loads.
template <int EPI>
__device__ __forceinline__ EpiIn st_epi_in(double c0, double c1, double c2, double u1, double u2,
                                           double us, double e) {
  EpiIn in;
  in.x = c0;
  in.x2 = c1;
  if constexpr (is_step<EPI>()) {
    in.u1 = u1;
    in.u2 = u2;
    in.us = us;
    if constexpr (is_vstep<EPI>()) in.e = c2;
  } else {
    in.e = e;
  }
  return in;
}

// Slot-kind patterns known at compile time (PAT != 0): 4 bits per slot,
// the slot count in bits 28-31. The 3-D 7-point stencil (offsets -W, -n, -1,
// 0, +1, +n, +W) is the C2 / C4 pattern; any other offset set runs the
// kernel with PAT = 0, which reads st_kind at run time.
constexpr uint32_t st_pat(int nm, std::initializer_list<int> kinds) {
  uint32_t p = (uint32_t)nm << 28;
  int k = 0;
  for (int v : kinds) p |= (uint32_t)v << (4 * k++);
  return p;
}
constexpr uint32_t kPat7 =
    st_pat(7, {SK_PREV, SK_FAR + 0, SK_NEAR, SK_CENTER, SK_NEAR, SK_FAR + 1, SK_NEXT});

// RELOAD: every visit loads its CENTER and PREV (launches whose walk crosses
// a row-block gap: the boundary launch of a split SpMV); otherwise they are
// loaded once per plane segment, before the loop, and carried.
// NTM: bit 0 = non-temporal code loads, bit 1 = non-temporal result stores
// (A/B, KR_STENCIL_NT). CB: bits per slot code (SpmvArgs::st_cb).
template <int EPI, int NFAR, uint32_t PAT, bool RELOAD, int NTM = 3, int CB = 8>
__device__ __forceinline__ void spmv_stencil_body(const SpmvArgs& a) {
  if (a.stop && *a.stop != 0.0) return;  // converged (device-resident scalars)
  using T = EpiTraits<EPI>;
  constexpr int NP = T::NP;
  constexpr int NV = T::NV;                    // sums (input vectors of the SpMV)
  constexpr bool VIRT = is_virtual<EPI>();     // operand r1 formed from x1, x2, x3
  constexpr int NX = VIRT ? (EPI == EPI_XY_VP ? 2 : 3) : NV;  // physical input vectors
  // NTM bit 6: two adjacent positions per workgroup (2 x kBlock threads).
  // Half h of workgroup B runs virtual workgroup 16 (B >> 3) + 8 h + (B & 7):
  // the same XCD, positions p and p + 1 of one plane segment, so the +-n FAR
  // lines one half reads are the rows the other half loads on the same CU in
  // the same visit. Every virtual workgroup visits the same blocks in the
  // same order and writes the same partials as an unpaired launch with twice
  // the grid (the host launches it only where both halves' walks agree).
  constexpr bool PAIRW = (NTM & 64) && !RELOAD;
  // NTM bit 8 (with the pairs, the LDS line path, FAR offsets -+512 = the
  // positions p -+ 1): the inner +-n line of each half is the other half's
  // CENTER line, already in LDS after the visit's barrier -- only the outer
  // one is loaded (half 0: -n, half 1: +n), half the FAR traffic
  constexpr bool LFAR = PAIRW && (NTM & 256) && !(NTM & 32) && PAT == kPat7;
  const int half = PAIRW ? __builtin_amdgcn_readfirstlane(threadIdx.x / kBlock) : 0;
  const int tid = PAIRW ? (int)(threadIdx.x % kBlock) : (int)threadIdx.x;
  const int64_t pb = (!RELOAD && a.st_rev) ? (int64_t)gridDim.x - 1 - blockIdx.x : blockIdx.x;
  const int64_t vb = PAIRW ? 16 * (pb >> 3) + 8 * half + (pb & 7) : pb;
  const int64_t vgrid = PAIRW ? 2 * (int64_t)gridDim.x : (int64_t)gridDim.x;
  __shared__ double s_redx[PAIRW ? 2 : 1][(NP > 0 ? NP : 1) * 4];
  __shared__ double s_tab[kVdMax];
  __shared__ __attribute__((aligned(16))) double s_linex[PAIRW ? 2 : 1][2][NV][kSLine];
  double* const s_red = s_redx[half];
  auto& s_line = s_linex[half];
  if (threadIdx.x < (unsigned)a.ntab) s_tab[threadIdx.x] = a.vtab[threadIdx.x];

  double acc[NP > 0 ? NP : 1];
#pragma unroll
  for (int q = 0; q < (NP > 0 ? NP : 1); ++q) acc[q] = 0.0;

  // ---- the walk: blocks v = z * P + p for the planes z of this segment
  const int64_t P = a.st_P;
  const int64_t W = P * kSBlock;
  const int64_t nrb = (a.n + kSBlock - 1) / kSBlock - a.rb_gap;
  const int64_t planes = (nrb + P - 1) / P;
  const int64_t q = vb & 7;
  const int64_t w = vb >> 3;
  int64_t p, z0, z1;
  if (a.st_pm) {
    // position-major: XCD q walks positions [q P/8, (q+1) P/8) (neighbouring
    // positions, whose x rows are each other's +-512 offsets, share an L2)
    // over plane segment zs of Zt = grid / P; fewer, longer walks than
    // plane-major when the shard has few planes (an 8-GPU slab: 64)
    const int64_t PP = P >> 3, Zt = vgrid / P;
    p = q * PP + w % PP;
    const int64_t zs = w / PP;
    z0 = planes * zs / Zt;
    z1 = planes * (zs + 1) / Zt;
  } else {
    const int64_t Z = vgrid / (8 * P);
    p = w % P;
    const int64_t zs = w / P;
    const int64_t pl0 = planes * q / 8, npl = planes * (q + 1) / 8 - pl0;
    z0 = pl0 + npl * zs / Z;
    z1 = pl0 + npl * (zs + 1) / Z;
  }
  auto phys = [&](int64_t v) { return v < a.rb_gap_at ? v : v + a.rb_gap; };
  // RELOAD (the boundary launch of a split SpMV: a plane or two at each end
  // of the shard) carries nothing along a walk, so it spreads its blocks over
  // the whole grid instead: visit z of workgroup b is block b + z * gridDim.
  // The plane-per-XCD split would leave all but two XCDs idle there.
  const int64_t G = gridDim.x;
  auto blk = [&](int64_t z) { return RELOAD ? (int64_t)blockIdx.x + z * G : z * P + p; };
  // pairs: the odd position's test for both halves (equal wherever the host
  // pairs; never one half at a barrier the other skips)
  const int64_t pt = PAIRW ? (p | 1) : p;
  auto visit_ok = [&](int64_t z) {
    return RELOAD ? blk(z) < nrb : (z < z1 && z * P + pt < nrb);
  };
  constexpr int NM_C = PAT ? (int)(PAT >> 28) : 8;
  const int nm = PAT ? NM_C : a.st_nm;

  const double* const xs[3] = {a.x1, a.x2, a.x3};
  dbl2v cen[NX], prv[NX];  // carried: x at the rows, x at the rows - W
  // NTM bit 3: loads two visits ahead (three stage register sets) instead of one
  constexpr int DEPTH = (!RELOAD && (NTM & 8)) ? 2 : 1;
  // NTM bit 5: +-1 neighbours by DPP within the wave (7-point pattern whose
  // NEAR slots are -1 and +1; the host checks), no LDS line, no barrier
  constexpr bool DPP = (NTM & 32) && PAT == kPat7;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  SStage<NX, NFAR, CB> sA, sB, sC;
  // Code patterns (SpmvArgs::st_pid; carried walks with one visit of
  // prefetch): the pattern id of the block the NEXT issue loads is fetched
  // through the scalar cache one visit ahead, after the visit's barrier with
  // the edge pairs (pid_n), so no issue waits on it.
  const bool pat = !RELOAD && DEPTH == 1 && a.st_pid != nullptr;
  const SRes res = st_res<NX, CB>(a, xs, pat);
  uint32_t pid_n = 0;
  auto pid_of = [&](int64_t z) -> uint32_t { return load_uniform(a.st_pid, phys(blk(z))); };
  int buf = 0;
  auto issue = [&](SStage<NX, NFAR, CB>& st, int64_t z, uint32_t pid) {
    const int64_t row0 = phys(blk(z)) * kSBlock;
    const int64_t rl = row0 + 2 * tid;
    const uint32_t cbase = pat ? pid * (uint32_t)(kSBlock * CB) : (uint32_t)(row0 * CB);
    st_issue<EPI, RELOAD, NTM>(st, a, res, row0, tid, rl < a.n ? rl : a.n - 2, cbase, pat,
                               LFAR ? (int64_t)a.st_far[half] : 0);
  };
  auto issue_edges = [&](SStage<NX, NFAR, CB>& st, int64_t z) {
    if constexpr (DPP)
      st_issue_wave_edges(st, a, xs, phys(blk(z)) * kSBlock, wave);
    else
      st_issue_edges(st, a, xs, phys(blk(z)) * kSBlock);
  };

  // One visit: `cur` holds its loads (issued one visit earlier); the next
  // visit's loads go to `nxs` before anything here waits. The loop below
  // alternates the two stage register sets, so nothing copies a register a
  // load is still writing (a copy would wait for it).
  auto visit = [&](SStage<NX, NFAR, CB>& cur, SStage<NX, NFAR, CB>& nxs, int64_t z) {
    const int64_t rb = phys(blk(z));
    const int64_t row0 = rb * kSBlock;
    const int64_t rl = row0 + 2 * tid;
    // Lanes past the last row (n is even: both rows or neither) run the same
    // instructions; they load x at their true rows (halo rows: the line needs
    // them for the +1 neighbour of the last own row), their products are
    // dropped and they store into SpmvArgs::scratch. No branch around any
    // memory operation: a branch there makes the compiler's wait counts
    // assume the shorter path.
    const bool active = rl < a.n;
    const int lp = tid;
    if constexpr (RELOAD) {
#pragma unroll
      for (int v = 0; v < NX; ++v) {
        cen[v] = cur.cen[v];
        prv[v] = cur.prv[v];
      }
    }
    // (1) the next visit's loads, in flight across this visit's work. Issued
    // unconditionally (the last visit re-reads its own rows): a load under a
    // branch makes the compiler's wait counts assume the shorter path.
    const int64_t zn = visit_ok(z + DEPTH) ? z + DEPTH : z;
    issue(nxs, zn, pid_n);
    // (2) operand values at the rows: centers, the previous plane's centers
    dbl2v opc[NV], opp[NV];
    if constexpr (VIRT) {
      opc[0] = dbl2v{virt_in<EPI>(a, cen[0].x, cen[1].x, cen[NX - 1].x),
                     virt_in<EPI>(a, cen[0].y, cen[1].y, cen[NX - 1].y)};
      opp[0] = dbl2v{virt_in<EPI>(a, prv[0].x, prv[1].x, prv[NX - 1].x),
                     virt_in<EPI>(a, prv[0].y, prv[1].y, prv[NX - 1].y)};
    } else {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        opc[v] = cen[v];
        opp[v] = prv[v];
      }
    }
    // (3) the +-1 neighbours: DPP within the wave (+ the wave's edge rows),
    // or the LDS line of this block's centers and its edge pairs
    double xm1[NV], xp2[NV];  // DPP: x at rows 2t-1 and 2t+2
    if constexpr (DPP) {
      double el[NV], er[NV];
      if constexpr (VIRT) {
        el[0] = virt_in<EPI>(a, cur.el[0].y, cur.el[1].y, cur.el[NX - 1].y);
        er[0] = virt_in<EPI>(a, cur.er[0].x, cur.er[1].x, cur.er[NX - 1].x);
      } else {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          el[v] = cur.el[v].y;
          er[v] = cur.er[v].x;
        }
      }
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        xm1[v] = st_dpp_shr1(opc[v].y, el[v]);
        xp2[v] = st_dpp_shl1(opc[v].x, er[v]);
      }
      issue_edges(nxs, zn);
      if (pat) pid_n = pid_of(visit_ok(zn + 1) ? zn + 1 : zn);
    } else {
#pragma unroll
      for (int v = 0; v < NV; ++v)
        reinterpret_cast<dbl2v*>(&s_line[buf][v][kSNear])[tid] = opc[v];
      if (tid < 2) {
        double* dst = &s_line[buf][0][tid == 0 ? 0 : kSNear + kSBlock];
        const dbl2v* e = tid == 0 ? cur.el : cur.er;
        if constexpr (VIRT) {
          *reinterpret_cast<dbl2v*>(dst) =
              dbl2v{virt_in<EPI>(a, e[0].x, e[1].x, e[NX - 1].x),
                    virt_in<EPI>(a, e[0].y, e[1].y, e[NX - 1].y)};
        } else {
#pragma unroll
          for (int v = 0; v < NV; ++v) *reinterpret_cast<dbl2v*>(dst + v * kSLine) = e[v];
        }
      }
      __syncthreads();
      issue_edges(nxs, zn);
      if (pat) pid_n = pid_of(visit_ok(zn + 1) ? zn + 1 : zn);
    }
    // (4) the two rows' sums, slot by slot in ascending offset order. A
    // visit whose rows (every lane of the wave) have all nm slots present --
    // all but the grid's faces -- runs the straight-line sums (one uniform
    // branch per visit, not per slot: per-slot branches cost phi copies).
    double slo[NV], shi[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) slo[v] = shi[v] = 0.0;
    // Faces: when every lane's absent entries sit in ONE slot (the usual
    // face: the x faces' -1 / +1, the y faces' -n / +n, ...), only that
    // slot takes the per-row selects (7-point pattern; else every slot).
    using AM = typename SStage<NX, NFAR, CB>::Code;
    const AM am = st_absent_bits<CB>(cur.clo, nm) | st_absent_bits<CB>(cur.chi, nm);
    const uint64_t amb = __builtin_amdgcn_ballot_w64(am != 0);
    int sel = -1;  // -1: every slot present; 0..7: only that slot has absents; 8: several
    if (amb != 0) {
      const int l0 = (int)__builtin_ctzll(amb);
      AM m0;
      if constexpr (sizeof(AM) == 8) {
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)am, l0);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(am >> 32), l0);
        m0 = ((AM)hi << 32) | lo;
      } else {
        m0 = (AM)__builtin_amdgcn_readlane((uint32_t)am, l0);
      }
      const bool same = __builtin_amdgcn_ballot_w64(am != 0 && am != m0) == 0;
      const bool one = (m0 & (m0 - 1)) == 0;
      sel = (same && one) ? (int)(__builtin_ctzll((uint64_t)m0) / CB) : 8;
    }
    auto sums = [&](auto sel_c) {
    constexpr int SEL = decltype(sel_c)::value;
#pragma unroll
    for (int k = 0; k < NM_C; ++k) {
      if (k >= nm) break;
      const int kind = PAT ? (int)((PAT >> (4 * k)) & 0xFu) : a.st_kind[k];
      constexpr unsigned kNone = (1u << CB) - 1u;  // no entry
      const unsigned clo = (unsigned)(cur.clo >> (CB * k)) & kNone;
      const unsigned chi = (unsigned)(cur.chi >> (CB * k)) & kNone;
      // an absent code reads an unused table entry (s_tab has kVdMax
      // slots); its product is dropped below
      const double vlo = (KR_ST_AB & 4) ? (double)clo : s_tab[clo];
      const double vhi = (KR_ST_AB & 4) ? (double)chi : s_tab[chi];
      double xlo[NV], xhi[NV];
      if (kind == SK_CENTER) {
#pragma unroll
        for (int v = 0; v < NV; ++v) { xlo[v] = opc[v].x; xhi[v] = opc[v].y; }
      } else if (kind == SK_PREV) {
#pragma unroll
        for (int v = 0; v < NV; ++v) { xlo[v] = opp[v].x; xhi[v] = opp[v].y; }
      } else if (kind == SK_NEAR && (KR_ST_AB & 8)) {
#pragma unroll
        for (int v = 0; v < NV; ++v) { xlo[v] = opc[v].y; xhi[v] = opc[v].x; }
      } else if (kind == SK_NEAR) {
        if constexpr (DPP) {  // kPat7: slot 2 is -1, slot 4 is +1
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            xlo[v] = k == 2 ? xm1[v] : opc[v].y;
            xhi[v] = k == 2 ? opc[v].x : xp2[v];
          }
        } else {
          const int o = a.st_off[k];
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            xlo[v] = s_line[buf][v][kSNear + 2 * lp + o];
            xhi[v] = s_line[buf][v][kSNear + 2 * lp + 1 + o];
          }
        }
      } else if (LFAR && kind != SK_NEXT) {
        // FAR f of half h (position pairs, NTM bit 8): outer (-n of half 0,
        // +n of half 1) the staged load, inner the other half's line in LDS
        // (operand values, as the NEAR slots read their own)
        const bool outer = (kind == SK_FAR) == (half == 0);
        const auto& other = s_linex[PAIRW ? half ^ 1 : 0][buf];
        const dbl2v* o = cur.far[0];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const double ilo = other[v][kSNear + 2 * lp], ihi = other[v][kSNear + 2 * lp + 1];
          double olo, ohi;
          if constexpr (VIRT) {
            olo = virt_in<EPI>(a, o[0].x, o[1].x, o[NX - 1].x);
            ohi = virt_in<EPI>(a, o[0].y, o[1].y, o[NX - 1].y);
          } else {
            olo = o[v].x;
            ohi = o[v].y;
          }
          xlo[v] = outer ? olo : ilo;
          xhi[v] = outer ? ohi : ihi;
        }
      } else {
        // NEXT or FAR f: a staged pair
        dbl2v g[NX];
#pragma unroll
        for (int v = 0; v < NX; ++v) g[v] = cur.nxt[v];
        // selects on values (a branch per f let the compiler index cur.far
        // with the run-time kind: the stage sets went to scratch, PAT = 0)
#pragma unroll
        for (int f = 0; f < NFAR; ++f) {
          const bool s = kind == SK_FAR + f;
#pragma unroll
          for (int v = 0; v < NX; ++v) {
            g[v].x = s ? cur.far[f][v].x : g[v].x;
            g[v].y = s ? cur.far[f][v].y : g[v].y;
          }
        }
        if constexpr (VIRT) {
          xlo[0] = virt_in<EPI>(a, g[0].x, g[1].x, g[NX - 1].x);
          xhi[0] = virt_in<EPI>(a, g[0].y, g[1].y, g[NX - 1].y);
        } else {
#pragma unroll
          for (int v = 0; v < NV; ++v) { xlo[v] = g[v].x; xhi[v] = g[v].y; }
        }
      }
      if (SEL < 0 || (SEL < 8 && k != SEL)) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          slo[v] = slo[v] + vlo * xlo[v];
          shi[v] = shi[v] + vhi * xhi[v];
        }
      } else {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
          const double plo = slo[v] + vlo * xlo[v];
          const double phi = shi[v] + vhi * xhi[v];
          slo[v] = clo != kNone ? plo : slo[v];
          shi[v] = chi != kNone ? phi : shi[v];
        }
      }
    }
    };
    if (sel < 0) {
      sums(std::integral_constant<int, -1>{});
    } else if constexpr (PAT == kPat7) {
      switch (sel) {
        case 0: sums(std::integral_constant<int, 0>{}); break;
        case 1: sums(std::integral_constant<int, 1>{}); break;
        case 2: sums(std::integral_constant<int, 2>{}); break;
        case 3: sums(std::integral_constant<int, 3>{}); break;
        case 4: sums(std::integral_constant<int, 4>{}); break;
        case 5: sums(std::integral_constant<int, 5>{}); break;
        case 6: sums(std::integral_constant<int, 6>{}); break;
        default: sums(std::integral_constant<int, 8>{}); break;
      }
    } else {
      sums(std::integral_constant<int, 8>{});
    }
    // (5) epilogue: row 2t, then row 2t+1 (products in that order)
    {
      const EpiIn ilo = st_epi_in<EPI>(cen[0].x, NX > 1 ? cen[NX > 1 ? 1 : 0].x : 0.0,
                                       NX > 2 ? cen[NX > 2 ? 2 : 0].x : 0.0, cur.u1.x, cur.u2.x,
                                       cur.us.x, cur.e.x);
      const EpiIn ihi = st_epi_in<EPI>(cen[0].y, NX > 1 ? cen[NX > 1 ? 1 : 0].y : 0.0,
                                       NX > 2 ? cen[NX > 2 ? 2 : 0].y : 0.0, cur.u1.y, cur.u2.y,
                                       cur.us.y, cur.e.y);
      double tmp[NP > 0 ? NP : 1];
#pragma unroll
      for (int q = 0; q < (NP > 0 ? NP : 1); ++q) tmp[q] = acc[q];
      const EpiVals olo = epi_values<EPI>(a, slo[0], NV == 2 ? slo[NV - 1] : 0.0, ilo, tmp);
      const EpiVals ohi = epi_values<EPI>(a, shi[0], NV == 2 ? shi[NV - 1] : 0.0, ihi, tmp);
      if constexpr (!(KR_ST_AB & 2)) {
#pragma unroll
        for (int q = 0; q < (NP > 0 ? NP : 1); ++q) acc[q] = active ? tmp[q] : acc[q];
      }
      if constexpr (!(NTM & 4) && !(KR_ST_AB & 1))
        epi_store_pair<EPI, (NTM & 2) != 0>(a, rl, olo, ohi, active);
      else if constexpr (KR_ST_AB & 1)
        acc[0] = acc[0] + olo.y1 * ohi.y2;  // keep the sums live
    }
    // (6) carry along the walk: this visit's centers are the next one's PREV
    if constexpr (!RELOAD) {
#pragma unroll
      for (int v = 0; v < NX; ++v) {
        prv[v] = cen[v];
        cen[v] = cur.nxt[v];
      }
    }
    buf ^= 1;
  };

  int64_t z = RELOAD ? 0 : z0;
  if (visit_ok(z)) {
    issue(sA, z, pat ? pid_of(z) : 0u);
    issue_edges(sA, z);
    if (pat) pid_n = pid_of(visit_ok(z + 1) ? z + 1 : z);
    if constexpr (DEPTH == 2) {
      const int64_t z1n = visit_ok(z + 1) ? z + 1 : z;
      issue(sB, z1n, 0u);
      issue_edges(sB, z1n);
    }
    if constexpr (!RELOAD) {  // CENTER and PREV of the segment's first visit
      const int64_t xi = a.xoff + phys(z * P + p) * kSBlock + 2 * tid;
#pragma unroll
      for (int v = 0; v < NX; ++v) {
        cen[v] = st_ld2(xs[v], xi, a.xlen);
        prv[v] = st_ld2(xs[v], xi - W, a.xlen);
      }
    }
  }
  // Drain the prologue's loads (once per segment): the loop's wait counts
  // then start from an empty queue on every path into it.
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();  // s_tab
  if constexpr (DEPTH == 2) {
    // stage of visit z: A, B, C, A, ...; visit z issues z + 2 into the stage
    // visit z - 1 consumed
    for (;;) {
      if (!visit_ok(z)) break;
      visit(sA, sC, z);
      ++z;
      if (!visit_ok(z)) break;
      visit(sB, sA, z);
      ++z;
      if (!visit_ok(z)) break;
      visit(sC, sB, z);
      ++z;
    }
  } else {
    for (;;) {
      if (!visit_ok(z)) break;
      visit(sA, sB, z);
      ++z;
      if (!visit_ok(z)) break;
      visit(sB, sA, z);
      ++z;
    }
  }
  __syncthreads();
  block_reduce_store<NP>(acc, a.partials, a.grid, s_red, a.accumulate, tid, vb);
}

// Threads per workgroup of a stencil launch: NTM bit 6 pairs two positions.
constexpr int st_threads(int ntm) { return (ntm & 64) ? 2 * kBlock : kBlock; }

template <int EPI, int NFAR, uint32_t PAT, bool RELOAD, int NTM = 3, int CB = 8>
__global__ __launch_bounds__(st_threads(NTM)) void spmv_stencil_kernel(SpmvArgs a) {
  if (!spmv_entry<EPI>(a)) return;  // converged / the fused scalar step's test fired
  spmv_stencil_body<EPI, NFAR, PAT, RELOAD, NTM, CB>(a);
}
// The dual (basis) SpMVs fit 128 VGPRs without spilling: 4 waves per SIMD
// instead of 3 (512^3 dual -1-4 %, products-only -4 %, 64-plane slab -6/-12 %).
// The three-vector first-steps kernel and the RELOAD walk would spill there.
template <int EPI, int NFAR, uint32_t PAT, bool RELOAD, int NTM = 3, int CB = 8>
__global__ __launch_bounds__(st_threads(NTM)) __attribute__((amdgpu_waves_per_eu(KR_ST_W4)))
void spmv_stencil_kernel_w4(SpmvArgs a) {
  if (!spmv_entry<EPI>(a)) return;
  spmv_stencil_body<EPI, NFAR, PAT, RELOAD, NTM, CB>(a);
}
// The products-only dual (a read-only stream, no store epilogue) at its own
// wave target (KR_ST_PO_W, compile time; A/B builds).
#ifndef KR_ST_PO_W
#define KR_ST_PO_W 4
#endif
template <int EPI, int NFAR, uint32_t PAT, bool RELOAD, int NTM = 3, int CB = 8>
__global__ __launch_bounds__(st_threads(NTM)) __attribute__((amdgpu_waves_per_eu(KR_ST_PO_W)))
void spmv_stencil_kernel_po(SpmvArgs a) {
  if (!spmv_entry<EPI>(a)) return;
  spmv_stencil_body<EPI, NFAR, PAT, RELOAD, NTM, CB>(a);
}

// KR_STENCIL_DEPTH=2 (A/B): the dual SpMVs load two visits ahead.
inline int st_depth() {
  return KR_ENV("KR_STENCIL_DEPTH", 1);
}
// The DPP neighbour path (NTM bit 5) for 7-point shards whose NEAR slots are
// -1 and +1. Measured on C4 (one box, A/B): the products-only dual 0.645 ->
// 0.560 ms (a read-only stream: the per-visit barrier was its stall), every
// storing launch 1-2 % slower (dual 0.889 -> 0.908 ms, steps alike). So
// KR_STENCIL_DPP = 1 (default): products-only launches only; 2: every
// 7-point launch; 0: none (A/B).
inline bool st_dpp(const SpmvArgs& a, bool products_only) {
  const int v = KR_ENV("KR_STENCIL_DPP", 1);
  return (v == 2 || (v == 1 && products_only)) && a.st_off[2] == -1 && a.st_off[4] == 1;
}

// Position pairs (NTM bit 6) where both halves of every workgroup walk the
// same planes: position-major, P % 16 == 0 (adjacent positions share an XCD
// eighth), whole planes, a grid of whole (XCD, position) columns; not for the
// EPIs whose kernel entry runs a block-wide prologue sized for kBlock.
// KR_STENCIL_PAIR (bit mask, A/B): 1 products-only duals, 2 storing duals,
// 4 the single-vector fused steps (is_step), 8 the fused first two steps,
// 16 every other 7-point launch, 32 the inner +-n line from LDS (n = 512);
// unset: 2 | 4 | 8 | 32 where bit 32 applies, else no pairs.
template <int E>
inline bool st_pair(const SpmvArgs& a, int nblocks) {
  if constexpr (E == EPI_XY_VP || E == EPI_MRR_V) {
    return false;
  } else {
    // Default (unset): the storing duals, the fused steps and the fused first
    // steps, and only where the inner +-n line can come from LDS (bit 32: n =
    // 512) -- measured on C4 (one box, three rounds, profiles/r04h): dual
    // 0.838 -> 0.813-0.823 ms, first steps 1.71 -> 1.65 ms, 560.7 -> 563-567
    // it/s; plain pairs (the ±n lines loaded by both halves) made the dual 7 %
    // slower instead. Round 5 (profiles/r05e/pair_ab.txt, one box, A/B twice):
    // the steps too (bit 4), spmv_step_mrr_nox 1.049-1.077 -> 1.032 ms, the x2
    // step 1.40-1.69 (bimodal) -> 1.42-1.43 ms, C4 554.3 -> 558.4-559.0 it/s;
    // the head (bit 16) 0.58-0.60 -> 0.60 ms and the products-only dual (bit
    // 1, with or without DPP) 0.59 -> 0.65-0.72 ms stay unpaired.
    const int env = KR_ENV("KR_STENCIL_PAIR", -1);
    const bool lfar = a.st_far[0] == -kSBlock && a.st_far[1] == kSBlock;
    const int m = env >= 0 ? env : (lfar ? 2 | 4 | 8 | 32 : 0);
    constexpr bool dual = E == EPI_DUAL_MRR || E == EPI_DUAL_KCG || E == EPI_DUAL_NONE;
    const int bit = (dual && a.products_only) ? 1
                    : dual                        ? 2
                    : E == EPI_STEP_MRR_FIRST2    ? 8
                    : is_step<E>()                ? 4
                                                  : 16;
    if (!(m & bit) || !a.st_pm || a.rb_gap != 0 || a.st_P <= 0 || a.st_P % 16 != 0) return false;
    const int64_t nrb = (a.n + kSBlock - 1) / kSBlock;
    return nrb % a.st_P == 0 && nblocks % a.st_P == 0 && nblocks % 16 == 0;
  }
}

// The 7-point pattern's launch at the shard's code width.
template <int E, bool RELOAD, int NTM, bool W4>
void st_launch_pat7(const SpmvArgs& a, int nblocks, size_t lds, hipStream_t s) {
  if constexpr (!RELOAD && !(NTM & 64)) {
    if (st_pair<E>(a, nblocks)) {
      // KR_STENCIL_PAIR bit 32: the inner +-n line from the other half's LDS
      // line (needs the LDS path and FAR offsets -+512: n = 512)
      if constexpr (!(NTM & 32)) {
        const int env = KR_ENV("KR_STENCIL_PAIR", -1);
        if ((env < 0 || (env & 32)) && a.st_far[0] == -kSBlock && a.st_far[1] == kSBlock) {
          st_launch_pat7<E, RELOAD, NTM | 64 | 256, W4>(a, nblocks, lds, s);
          return;
        }
      }
      st_launch_pat7<E, RELOAD, NTM | 64, W4>(a, nblocks, lds, s);
      return;
    }
  }
  constexpr int TH = st_threads(NTM);
  const int nb = (NTM & 64) ? nblocks / 2 : nblocks;
  auto go = [&](auto cbc) {
    constexpr int CB = decltype(cbc)::value;
    if constexpr (W4 && (NTM & 4))
      spmv_stencil_kernel_po<E, 2, kPat7, RELOAD, NTM, CB><<<nb, TH, lds, s>>>(a);
    else if constexpr (W4)
      spmv_stencil_kernel_w4<E, 2, kPat7, RELOAD, NTM, CB><<<nb, TH, lds, s>>>(a);
    else
      spmv_stencil_kernel<E, 2, kPat7, RELOAD, NTM, CB><<<nb, TH, lds, s>>>(a);
  };
  switch (a.st_cb) {
    case 2: go(std::integral_constant<int, 2>{}); return;
    case 4: go(std::integral_constant<int, 4>{}); return;
    default: go(std::integral_constant<int, 8>{}); return;
  }
}

template <int E, bool RELOAD>
void spmv_stencil_launch_r(const SpmvArgs& a, int nblocks, hipStream_t s) {
  bool pat7 = a.st_nm == 7 && a.st_nfar == 2;
  for (int k = 0; k < 7 && pat7; ++k) pat7 = a.st_kind[k] == (int)((kPat7 >> (4 * k)) & 0xFu);
  // narrow codes exist only for the 7-point pattern (System::build_stencil)
  KR_REQUIRE(pat7 || a.st_cb == 8, "stencil SpMV: narrow codes need the 7-point pattern");
  // Non-temporal code loads and result stores (NTM = 3): the streamed-once
  // bytes stop displacing the x lines neighbouring workgroups re-read from
  // L2 (C4 +4-7 %). KR_STENCIL_NT=0..2 (A/B; 7-point pattern, 8-bit codes).
  // KR_STENCIL_LDS (A/B): extra LDS per workgroup, i.e. fewer resident
  // workgroups per CU.
  const int ntm = KR_ENV("KR_STENCIL_NT", 3);
  const size_t lds = (size_t)KR_ENV("KR_STENCIL_LDS", 0);
  if constexpr (E == EPI_DUAL_MRR || E == EPI_DUAL_KCG) {
    // products only (SpmvArgs::products_only): NTM bit 2 drops the y1/y2
    // stores (the last basis pair of a k-skip outer iteration feeds only the
    // Gram products)
    if (a.products_only) {
      if (pat7) {
        if (!RELOAD && st_depth() == 2)
          st_launch_pat7<E, RELOAD, 15, false>(a, nblocks, lds, s);
        else if (st_dpp(a, true))
          st_launch_pat7<E, RELOAD, 39, !RELOAD>(a, nblocks, lds, s);
        else
          st_launch_pat7<E, RELOAD, 7, !RELOAD>(a, nblocks, lds, s);
        return;
      }
      switch (a.st_nfar) {
        case 0: spmv_stencil_kernel<E, 0, 0, RELOAD, 7><<<nblocks, kBlock, 0, s>>>(a); return;
        case 1: spmv_stencil_kernel<E, 1, 0, RELOAD, 7><<<nblocks, kBlock, 0, s>>>(a); return;
        case 2: spmv_stencil_kernel<E, 2, 0, RELOAD, 7><<<nblocks, kBlock, 0, s>>>(a); return;
        case 3: spmv_stencil_kernel<E, 3, 0, RELOAD, 7><<<nblocks, kBlock, 0, s>>>(a); return;
        default: spmv_stencil_kernel<E, 4, 0, RELOAD, 7><<<nblocks, kBlock, 0, s>>>(a); return;
      }
    }
  }
  if (pat7) {
    if constexpr (!RELOAD) {
      if (ntm != 3) KR_REQUIRE(a.st_cb == 8, "KR_STENCIL_NT A/B runs with KR_STENCIL_CB=8");
      switch (ntm) {
        case 0: spmv_stencil_kernel<E, 2, kPat7, RELOAD, 0><<<nblocks, kBlock, lds, s>>>(a); return;
        case 1: spmv_stencil_kernel<E, 2, kPat7, RELOAD, 1><<<nblocks, kBlock, lds, s>>>(a); return;
        case 2: spmv_stencil_kernel<E, 2, kPat7, RELOAD, 2><<<nblocks, kBlock, lds, s>>>(a); return;
        default: break;
      }
    }
    constexpr bool w4 = !RELOAD && (E == EPI_DUAL_MRR || E == EPI_DUAL_KCG || E == EPI_DUAL_NONE);
    // KR_STENCIL_DEPTH=2: the duals; 3: every carried 7-point launch (A/B)
    const int depth = st_depth();
    if (!RELOAD && (depth == 3 || (w4 && depth == 2)))
      st_launch_pat7<E, RELOAD, 11, false>(a, nblocks, lds, s);
    else if (st_dpp(a, false))
      st_launch_pat7<E, RELOAD, 35, w4>(a, nblocks, lds, s);
    else
      st_launch_pat7<E, RELOAD, 3, w4>(a, nblocks, lds, s);
    return;
  }
  switch (a.st_nfar) {
    case 0: spmv_stencil_kernel<E, 0, 0, RELOAD, 3><<<nblocks, kBlock, 0, s>>>(a); return;
    case 1: spmv_stencil_kernel<E, 1, 0, RELOAD, 3><<<nblocks, kBlock, 0, s>>>(a); return;
    case 2: spmv_stencil_kernel<E, 2, 0, RELOAD, 3><<<nblocks, kBlock, 0, s>>>(a); return;
    case 3: spmv_stencil_kernel<E, 3, 0, RELOAD, 3><<<nblocks, kBlock, 0, s>>>(a); return;
    default: spmv_stencil_kernel<E, 4, 0, RELOAD, 3><<<nblocks, kBlock, 0, s>>>(a); return;
  }
}

// Launches with a row-block gap (the boundary launch of a split SpMV) reload
// CENTER and PREV at every visit; all others carry them.
template <int E>
void spmv_stencil_launch(const SpmvArgs& a, int nblocks, hipStream_t s) {
  if (a.rb_gap > 0)
    spmv_stencil_launch_r<E, true>(a, nblocks, s);
  else
    spmv_stencil_launch_r<E, false>(a, nblocks, s);
}

// ---------------------------------------------------------------------------
// Two chained basis SpMVs in ONE walk (k-skip MrR, SpmvArgs x1 = Ar[m+1],
// x2 = Ay[m]): level 1 = (Ar[m+2], Ay[m+1]) = A (x1, x2) and level 2 =
// (Ar[m+3], Ay[m+2]) = A level 1, with both duals' Gram products
// (EPI_DUAL_MRR for m -> partials, for m+1 -> partials2) and only level 2
// stored (nothing when PO: the last pair of an outer iteration). Level 1 is
// never written to HBM: the pair moves the bytes of ONE dual SpMV.
//
// 7-point pattern with n = 512 (the +-n offsets are the neighbouring 512-row
// blocks of a plane; W = P blocks). A workgroup walks one column (position p)
// of the plane segment [z0, z1): level 2 of block p at plane z needs level 1
// of blocks p-1 .. p+1 (region R1) at plane z and of block p at z +- 1, and
// level 1 of R1 needs level 0 of blocks p-2 .. p+2 (R0) at its plane and of
// R1 at the planes beside it. Rows are linear indices throughout (block p-1
// of position 0 is the last block of the previous plane), so the regions are
// contiguous row ranges and every neighbour is the same row arithmetic as in
// the single SpMV; rows outside the vectors read 0 (buffer range check) and
// only feed entries the codes mark absent.
//
// Lane t owns rows 2t, 2t+1 of every block, so the +-n neighbours of an R1
// row are the same lane's registers (adjacent blocks); only +-1 crosses
// lanes and goes through LDS (one ds_read2_b64 per block). Every row is
// summed in stored (ascending offset) order from 0.0: -W, -n, -1, 0, +1, +n
// are added when the row's plane arrives (partial sums p1 / p2), +W when the
// next plane does -- bitwise the single SpMV. Step s (planes z0-1 .. z1+1):
// L0[s] arrives (loaded one step ahead) -> L1[s-1] = p1 + (+W term), p1 =
// partial of L1[s]; L1[s-1] -> L2[s-2] = p2 + (+W), p2 = partial of L2[s-1].
// Products: (L0, L1) of plane s-1 and (L1, L2) of plane s-2, each plane in
// order, row 2t then 2t+1 -- the accumulation order of the two dual launches
// on the same grid (oracle/gpu_order.py).
// ---------------------------------------------------------------------------
constexpr int kS2B0 = 5;  // level-0 blocks per plane (R0)
constexpr int kS2B1 = 3;  // level-1 blocks per plane (R1)

// Slots k0 .. k1-1 of rows lo / hi (codes clo / chi) for BOTH chains: the
// slot's code and table value are decoded once and serve the two chains; a
// slot present in every row of the wave (everywhere but the grid faces: the
// ballot) adds without the absent-entry selects.
template <int CB, int K0, int K1>
__device__ __forceinline__ void st2_terms(uint32_t clo, uint32_t chi,
                                          const double* __restrict__ tab,
                                          const double (&xlo)[2][7], const double (&xhi)[2][7],
                                          double (&slo)[2], double (&shi)[2]) {
  constexpr unsigned kNone = (1u << CB) - 1u;
#pragma unroll
  for (int k = K0; k < K1; ++k) {
    const unsigned cl = (clo >> (CB * k)) & kNone, ch = (chi >> (CB * k)) & kNone;
    const double vl = tab[cl], vh = tab[ch];  // tab[kNone]: a valid unused slot
    if (__builtin_amdgcn_ballot_w64(cl == kNone || ch == kNone) == 0) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        slo[c] = slo[c] + vl * xlo[c][k];
        shi[c] = shi[c] + vh * xhi[c][k];
      }
    } else {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const double tl = slo[c] + vl * xlo[c][k], th = shi[c] + vh * xhi[c][k];
        slo[c] = cl != kNone ? tl : slo[c];
        shi[c] = ch != kNone ? th : shi[c];
      }
    }
  }
}

template <int CB, bool PO>
__global__ __launch_bounds__(kBlock, 2) void spmv_stencil2_kernel(SpmvArgs a) {
  if (a.stop && *a.stop != 0.0) return;
  static_assert(CB == 2 || CB == 4, "fused basis pair: narrow codes");
  extern __shared__ __attribute__((aligned(16))) double s2_dyn[];
  double* s_l0 = s2_dyn;                             // [2][kS2B0 * 512]
  double* s_l1 = s2_dyn + 2 * kS2B0 * kSBlock;       // [2][kS2B1 * 512]
  __shared__ double s_tab[kVdMax];
  __shared__ double s_red1[7 * 4], s_red2[7 * 4];
  const int tid = threadIdx.x;
  if (tid < a.ntab) s_tab[tid] = a.vtab[tid];

  double acc1[7], acc2[7];
#pragma unroll
  for (int q = 0; q < 7; ++q) acc1[q] = acc2[q] = 0.0;

  // ---- the column: position-major grid (kr_stencil.h), segment [z0, z1)
  const int64_t P = a.st_P;
  const int64_t W = P * kSBlock;
  const int64_t planes = a.n / W;  // whole planes (the host checks)
  const int64_t q = blockIdx.x & 7, w = blockIdx.x >> 3;
  const int64_t PP = P >> 3, Zt = gridDim.x / P;
  const int64_t p = q * PP + w % PP;
  const int64_t zs = w / PP;
  const int64_t z0 = planes * zs / Zt, z1 = planes * (zs + 1) / Zt;

  const double* const xs[3] = {a.x1, a.x2, a.x2};
  const SRes res = st_res<2, CB>(a, xs);
  const uint32_t lb = (uint32_t)tid * 16u;
  // first row of R0 / R1 at plane z (linear, may be negative)
  auto r0_of = [&](int64_t z) { return z * W + (p - 2) * kSBlock; };
  auto ld = [&](int c, int64_t row) {  // the lane's pair at row + 2 tid of vector c
    return st_bld2(res.x[c], (uint32_t)((a.xoff + row) * 8) + lb);
  };
  auto codes = [&](int64_t row) {  // both rows' codes, packed (CB = 2: 16 bits each)
    if constexpr (CB == 2)
      return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(
          res.code, (uint32_t)(row * 2) + (uint32_t)tid * 4u, 0, 2);
    else
      return (uint32_t)0;
  };
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  auto codes4 = [&](int64_t row) {  // CB = 4: a uint32 per row
    return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(
                                         res.code, (uint32_t)(row * 4) + (uint32_t)tid * 8u, 0, 2));
  };
  auto lo_code = [&](uint32_t c2, u32x2 c4) { return CB == 2 ? (c2 & 0xFFFFu) : c4.x; };
  auto hi_code = [&](uint32_t c2, u32x2 c4) { return CB == 2 ? (c2 >> 16) : c4.y; };

  // ---- registers
  dbl2v nx[2][kS2B0];             // level 0 of the arriving plane (loaded a step ahead)
  uint32_t ncode2[kS2B1];         // its R1 codes
  u32x2 ncode4[kS2B1];
  dbl2v l0p[2][kS2B1];            // level 0 of the previous plane, R1 blocks
  dbl2v p1[2][kS2B1];             // partial level-1 sums of the previous plane
  uint32_t c1p2[kS2B1];           // R1 codes of the previous plane
  u32x2 c1p4[kS2B1];
  dbl2v l1p[2];                   // level 1 two planes back, block p
  dbl2v p2[2];                    // partial level-2 sums, plane s-2 ... (see below)
  uint32_t c2p2 = 0;              // block p's codes two planes back
  u32x2 c2p4 = {0u, 0u};
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    l1p[c] = dbl2v{0.0, 0.0};
    p2[c] = dbl2v{0.0, 0.0};
#pragma unroll
    for (int j = 0; j < kS2B1; ++j) p1[c][j] = dbl2v{0.0, 0.0};
  }
#pragma unroll
  for (int j = 0; j < kS2B1; ++j) {
    c1p2[j] = 0u;
    c1p4[j] = u32x2{0u, 0u};
  }

  auto issue = [&](int64_t z) {  // plane z's level 0 (R0) and R1 codes
    const int64_t r0 = r0_of(z);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int j = 0; j < kS2B0; ++j) nx[c][j] = ld(c, r0 + j * kSBlock);
#pragma unroll
    for (int j = 0; j < kS2B1; ++j) {
      if constexpr (CB == 2)
        ncode2[j] = codes(r0 + (j + 1) * kSBlock);
      else
        ncode4[j] = codes4(r0 + (j + 1) * kSBlock);
    }
  };

  if (z0 < z1) {
    // prologue: level 0 of plane z0-2 (R1 blocks: the -W operand of plane
    // z0-1's level-1 rows), then plane z0-1 in flight
    const int64_t r0 = r0_of(z0 - 2);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int j = 0; j < kS2B1; ++j) l0p[c][j] = ld(c, r0 + (j + 1) * kSBlock);
    issue(z0 - 1);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();                      // s_tab

  for (int64_t s = z0 - 1; s <= z1 + 1 && z0 < z1; ++s) {
    // (1) the arriving plane s: own copies, then the next plane's loads
    dbl2v l0[2][kS2B0];
    uint32_t cc2[kS2B1];
    u32x2 cc4[kS2B1];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int j = 0; j < kS2B0; ++j) l0[c][j] = nx[c][j];
#pragma unroll
    for (int j = 0; j < kS2B1; ++j) {
      cc2[j] = ncode2[j];
      cc4[j] = ncode4[j];
    }
    issue(s + 1 <= z1 + 1 ? s + 1 : s);  // (the last step re-reads its own plane)
    // (2) level 0 of plane s into LDS (the +-1 neighbours)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int j = 0; j < kS2B0; ++j)
        reinterpret_cast<dbl2v*>(s_l0 + c * kS2B0 * kSBlock + j * kSBlock)[tid] = l0[c][j];
    __syncthreads();
    // (3) level 1 of plane s-1 (R1) completed by its +W term; the products of
    // (level 0, level 1) at plane s-1; partial level-1 sums of plane s
    dbl2v l1[2][kS2B1];
#pragma unroll
    for (int j = 0; j < kS2B1; ++j) {
      // +W (slot 6) of plane s-1: x at plane s, same block
      {
        double xl[2][7], xh[2][7], sl[2], sh[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          xl[c][6] = l0[c][j + 1].x;
          xh[c][6] = l0[c][j + 1].y;
          sl[c] = p1[c][j].x;
          sh[c] = p1[c][j].y;
        }
        st2_terms<CB, 6, 7>(lo_code(c1p2[j], c1p4[j]), hi_code(c1p2[j], c1p4[j]), s_tab, xl, xh,
                            sl, sh);
#pragma unroll
        for (int c = 0; c < 2; ++c) l1[c][j] = dbl2v{sl[c], sh[c]};
      }
      // plane s: -W (l0p), -n (block j), -1 (LDS / own), 0, +1 (own / LDS), +n (block j+2)
      double xl[2][7], xh[2][7], sl[2] = {0.0, 0.0}, sh[2] = {0.0, 0.0};
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const double* line = s_l0 + c * kS2B0 * kSBlock + (j + 1) * kSBlock + 2 * tid;
        xl[c][0] = l0p[c][j].x;     xh[c][0] = l0p[c][j].y;
        xl[c][1] = l0[c][j].x;      xh[c][1] = l0[c][j].y;
        xl[c][2] = line[-1];        xh[c][2] = l0[c][j + 1].x;
        xl[c][3] = l0[c][j + 1].x;  xh[c][3] = l0[c][j + 1].y;
        xl[c][4] = l0[c][j + 1].y;  xh[c][4] = line[2];
        xl[c][5] = l0[c][j + 2].x;  xh[c][5] = l0[c][j + 2].y;
      }
      st2_terms<CB, 0, 6>(lo_code(cc2[j], cc4[j]), hi_code(cc2[j], cc4[j]), s_tab, xl, xh, sl, sh);
#pragma unroll
      for (int c = 0; c < 2; ++c) p1[c][j] = dbl2v{sl[c], sh[c]};
    }
    const bool l1ok = s - 1 >= z0 - 1;  // level 1 of plane s-1 is real (s > z0-1)
    if (l1ok && s - 1 >= z0 && s - 1 < z1) {
      // dual m at plane s-1, block p: x = Ar[m+1] (l0p r), x2 = Ay[m] (l0p y)
      epi_products<EPI_DUAL_MRR>(l0p[0][1].x, l0p[1][1].x, l1[0][1].x, l1[1][1].x, 0.0, acc1);
      epi_products<EPI_DUAL_MRR>(l0p[0][1].y, l0p[1][1].y, l1[0][1].y, l1[1][1].y, 0.0, acc1);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int j = 0; j < kS2B1; ++j) l0p[c][j] = l0[c][j + 1];
    // (4) level 1 of plane s-1 into LDS
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int j = 0; j < kS2B1; ++j)
        reinterpret_cast<dbl2v*>(s_l1 + c * kS2B1 * kSBlock + j * kSBlock)[tid] = l1[c][j];
    __syncthreads();
    // (5) level 2 of plane s-2 (block p) completed by its +W term (level 1 of
    // plane s-1); products of (level 1, level 2) at s-2; store; partial sums
    // of plane s-1
    {
      dbl2v l2[2];
      {
        double xl[2][7], xh[2][7], sl[2], sh[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          xl[c][6] = l1[c][1].x;
          xh[c][6] = l1[c][1].y;
          sl[c] = p2[c].x;
          sh[c] = p2[c].y;
        }
        st2_terms<CB, 6, 7>(lo_code(c2p2, c2p4), hi_code(c2p2, c2p4), s_tab, xl, xh, sl, sh);
#pragma unroll
        for (int c = 0; c < 2; ++c) l2[c] = dbl2v{sl[c], sh[c]};
      }
      if (s - 2 >= z0 && s - 2 < z1) {
        epi_products<EPI_DUAL_MRR>(l1p[0].x, l1p[1].x, l2[0].x, l2[1].x, 0.0, acc2);
        epi_products<EPI_DUAL_MRR>(l1p[0].y, l1p[1].y, l2[0].y, l2[1].y, 0.0, acc2);
        if constexpr (!PO) {
          const int64_t row = (s - 2) * W + p * kSBlock + 2 * tid;
          __builtin_nontemporal_store(l2[0], reinterpret_cast<dbl2v*>(a.y1 + row));
          __builtin_nontemporal_store(l2[1], reinterpret_cast<dbl2v*>(a.y2 + row));
        }
      }
      {
        double xl[2][7], xh[2][7], sl[2] = {0.0, 0.0}, sh[2] = {0.0, 0.0};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const double* line = s_l1 + c * kS2B1 * kSBlock + kSBlock + 2 * tid;
          xl[c][0] = l1p[c].x;       xh[c][0] = l1p[c].y;
          xl[c][1] = l1[c][0].x;     xh[c][1] = l1[c][0].y;
          xl[c][2] = line[-1];       xh[c][2] = l1[c][1].x;
          xl[c][3] = l1[c][1].x;     xh[c][3] = l1[c][1].y;
          xl[c][4] = l1[c][1].y;     xh[c][4] = line[2];
          xl[c][5] = l1[c][2].x;     xh[c][5] = l1[c][2].y;
        }
        st2_terms<CB, 0, 6>(lo_code(c1p2[1], c1p4[1]), hi_code(c1p2[1], c1p4[1]), s_tab, xl, xh,
                            sl, sh);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          p2[c] = dbl2v{sl[c], sh[c]};
          l1p[c] = l1[c][1];
        }
      }
      c2p2 = c1p2[1];
      c2p4 = c1p4[1];
    }
#pragma unroll
    for (int j = 0; j < kS2B1; ++j) {
      c1p2[j] = cc2[j];
      c1p4[j] = cc4[j];
    }
  }
  __syncthreads();
  block_reduce_store<7>(acc1, a.partials, a.grid, s_red1, 0);
  block_reduce_store<7>(acc2, a.partials2, a.grid, s_red2, 0);
}

// Dynamic LDS of the fused pair: level 0 (5 blocks) and level 1 (3 blocks) of
// one plane, two chains.
constexpr size_t kS2Lds = sizeof(double) * 2 * (kS2B0 + kS2B1) * kSBlock;

template <int CB, bool PO>
void st2_launch_t(const SpmvArgs& a, int nblocks, hipStream_t s) {
  static std::atomic<uint64_t> opted{0};  // per device (opt_in_lds)
  opt_in_lds(opted, reinterpret_cast<const void*>(spmv_stencil2_kernel<CB, PO>), kS2Lds);
  spmv_stencil2_kernel<CB, PO><<<nblocks, kBlock, kS2Lds, s>>>(a);
  KR_HIP_CHECK(hipGetLastError());
}

inline void spmv_stencil2_launch(const SpmvArgs& a, int nblocks, hipStream_t s) {
  KR_REQUIRE(a.scode && a.st_P % 8 == 0 && a.st_nm == 7 && a.st_nfar == 2 &&
                 a.st_far[0] == -kSBlock && a.st_far[1] == kSBlock &&
                 a.n % ((int64_t)a.st_P * kSBlock) == 0 && a.rb_gap == 0 && a.partials2 &&
                 nblocks % a.st_P == 0 && (a.st_cb == 2 || a.st_cb == 4),
             "fused basis pair: 7-point stencil with n = 512, whole planes, narrow codes");
  const bool po = a.products_only != 0;
  if (a.st_cb == 2)
    po ? st2_launch_t<2, true>(a, nblocks, s) : st2_launch_t<2, false>(a, nblocks, s);
  else
    po ? st2_launch_t<4, true>(a, nblocks, s) : st2_launch_t<4, false>(a, nblocks, s);
}

// ---------------------------------------------------------------------------
// Tiled fused basis pair (spmv_stencil2t_kernel; KR_ST2=2). The pair above
// walks ONE position and must rebuild level 1 on three blocks and load level
// 0 on five for it (3x the level-1 work, 2 waves per SIMD): slower than the
// two dual launches it replaces. Here a 1024-thread workgroup walks TWO
// adjacent positions p0, p0 + 1 (p0 even) of a plane segment; four 256-lane
// groups g = (line H = g >> 1, chain C = g & 1), lane t owning rows 2t and
// 2t + 1 of position p0 + H in chain C (the dual kernel's lane mapping):
//
//   level 0 (loaded)  : positions p0-2 .. p0+3, three per line group
//   level 1 (computed): positions p0-1 .. p0+2, two per line group (one redundant)
//   level 2 (stored)  : positions p0, p0+1, one per line group
//
// so the redundant work is one level-1 line per output line, and a group
// reads three level-0 lines of its chain per plane for two levels (the dual
// reads three per level and chain). Level 0 goes to LDS as it arrives (the
// six lines' +-1 and +-n operands) and the next plane's loads reuse its
// registers at once, so a whole plane step hides them; level 1 of p0 and
// p0 + 1 goes to LDS for level 2. A group holds one chain: ~120 VGPRs, so
// 16 waves (4 per SIMD) share the CU. Two barriers per plane.
//
// Bitwise the two dual launches, products included: every row is summed in
// stored order from 0.0 (-W ... +n when its plane arrives, +W one plane
// later). Dual m's products (level 0 x level 1) of position p0 + H are
// accumulated by group (H, 0), dual m+1's (level 1 x level 2) by group
// (H, 1) -- each lane plane by plane, row 2t then 2t+1, the other chain's
// operands read from LDS -- exactly as the dual launch's workgroup of that
// (position, segment) accumulates them. The walk segment is a union of
// segments of both dual grids (the level-2 grid is the products-only one for
// the last pair); at each grid's segment boundary the group's accumulator is
// reduced into that grid's partial of the virtual workgroup.
// ---------------------------------------------------------------------------
struct St2tLds {
  double x0[2][6 * kSBlock];       // level 0 of positions p0-2 .. p0+3 [chain][line*512 + row]
  double x1[2][2 * kSBlock + 4];   // level 1 of p0, p0+1 [chain][2 + line*512 + row], margins
  double xa[2][kSBlock];           // chain 1's level 0 of plane s-1, own line [line]
  double xb[2][2][kSBlock];        // chain 0's level 1 and level 2 of plane s-2 [line][level]
  double tab[kVdMax];
  double red[4][7 * 4];            // [group]
};
constexpr size_t kSt2tLds = sizeof(St2tLds);

template <int CB>
struct St2tStage {
  dbl2v x[3];               // level 0 of the group's three lines
  uint32_t clo[2], chi[2];  // codes of the two level-1 lines (rows 2t, 2t+1)
};

// One chain of one line: the tiled pair's work of group (H, C).
template <int EPI, int CB, bool PO, int H, int C>
__device__ __forceinline__ void st2t_walk(const SpmvArgs& a, St2tLds& L, int tid, int64_t p0,
                                          int64_t q, int64_t zs, int64_t Zw) {
  constexpr int NP = 7;
  constexpr int IO = H == 0 ? 1 : 0;  // own line among the group's level-1 lines
  constexpr int g = 2 * H + C;
  const int64_t P = a.st_P, W = P * kSBlock, PP = P >> 3;
  const int64_t planes = a.n / W;
  const int64_t z0 = planes * zs / Zw, z1 = planes * (zs + 1) / Zw;
  const int64_t pown = p0 + H;
  const double* const xs[3] = {C == 0 ? a.x1 : a.x2, a.x2, a.x2};
  const SRes res = st_res<1, CB>(a, xs);
  const uint32_t lb = (uint32_t)tid * 16u;
  const double* __restrict__ tab = L.tab;
  // first row of level-0 line l (0..5: positions p0-2 .. p0+3) at plane z
  auto row_of = [&](int64_t z, int l) { return z * W + (p0 - 2 + l) * kSBlock; };
#ifdef KR_ST2T_TIMING  // timing-only A/B build: every level-0 load reads plane 0 (L2 hits)
  auto ld = [&](int64_t row) {
    return st_bld2(res.x[0], (uint32_t)((a.xoff + (row % W + W) % W) * 8) + lb);
  };
#else
  auto ld = [&](int64_t row) { return st_bld2(res.x[0], (uint32_t)((a.xoff + row) * 8) + lb); };
#endif
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  auto issue = [&](St2tStage<CB>& st, int64_t z) {
#pragma unroll
    for (int j = 0; j < 3; ++j) st.x[j] = ld(row_of(z, 3 * H + j));
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t r = row_of(z, 1 + 2 * H + i);
      if constexpr (CB == 2) {
        const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(
            res.code, (uint32_t)(r * 2) + (uint32_t)tid * 4u, 0, 2);
        st.clo[i] = v & 0xFFFFu;
        st.chi[i] = v >> 16;
      } else {
        const u32x2 v = __builtin_bit_cast(
            u32x2, __builtin_amdgcn_raw_buffer_load_b64(res.code, (uint32_t)(r * 4) + (uint32_t)tid * 8u,
                                                        0, 2));
        st.clo[i] = v.x;
        st.chi[i] = v.y;
      }
    }
  };
  // One chain's sums over slots K0 .. K1-1 (st2_terms' rules: a slot present
  // in every row of the wave adds without the absent-entry selects).
  auto terms = [&](auto k0c, auto k1c, uint32_t clo, uint32_t chi, const double (&xl)[7],
                   const double (&xh)[7], double& sl, double& sh) {
    constexpr int K0 = decltype(k0c)::value, K1 = decltype(k1c)::value;
    constexpr unsigned kNone = (1u << CB) - 1u;
#pragma unroll
    for (int k = K0; k < K1; ++k) {
      const unsigned cl = (clo >> (CB * k)) & kNone, ch = (chi >> (CB * k)) & kNone;
      const double vl = tab[cl], vh = tab[ch];
      if (__builtin_amdgcn_ballot_w64(cl == kNone || ch == kNone) == 0) {
        sl = sl + vl * xl[k];
        sh = sh + vh * xh[k];
      } else {
        const double tl = sl + vl * xl[k], th = sh + vh * xh[k];
        sl = cl != kNone ? tl : sl;
        sh = ch != kNone ? th : sh;
      }
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I6 = std::integral_constant<int, 6>;
  using I7 = std::integral_constant<int, 7>;

  // products: group (H, 0) accumulates dual m's (grid 1), group (H, 1) dual
  // m+1's (grid 2) into the partials of the virtual workgroup (position,
  // segment); walk segment zs of Zw starts segment zs Z / Zw of a grid of Z
  double* const part = C == 0 ? a.partials : a.partials2;
  int64_t seg = zs * ((C == 0 ? a.st2_z1 : a.st2_z2) / Zw);  // this group's level's segment
  double acc[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) acc[k] = 0.0;
  // every group joins every flush (it holds a barrier); `mine`: this group's level
  auto flush = [&](bool mine) {
    const int lane = tid & 63, wave = tid >> 6;
    if (mine) {
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        double v = acc[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
        if (lane == 0) L.red[g][k * 4 + wave] = v;
      }
    }
    __syncthreads();
    if (mine) {
      if (tid < NP) {
        const double* r = L.red[g] + tid * 4;
        double t = r[0];
        t = t + r[1];
        t = t + r[2];
        t = t + r[3];
        part[(int64_t)tid * a.grid + 8 * (seg * PP + (pown - q * PP)) + q] = t;
      }
#pragma unroll
      for (int k = 0; k < NP; ++k) acc[k] = 0.0;
      ++seg;
    }
  };
  // a level's products at plane z: flush first when z starts the next
  // segment of that level's grid (the test is uniform: every group joins)
  int64_t sg1 = zs * (a.st2_z1 / Zw), sg2 = zs * (a.st2_z2 / Zw);
  int64_t nb1 = planes * (sg1 + 1) / a.st2_z1;  // level 1's next boundary
  int64_t nb2 = planes * (sg2 + 1) / a.st2_z2;
  auto cross = [&](int64_t z, int level) {
    int64_t& b = level == 1 ? nb1 : nb2;
    int64_t& sgx = level == 1 ? sg1 : sg2;
    const int64_t Zl = level == 1 ? a.st2_z1 : a.st2_z2;
    if (z >= b) {
      flush((level == 1) == (C == 0));
      ++sgx;
      b = planes * (sgx + 1) / Zl;
    }
  };

  // ---- state carried along the walk (step s: level 0 of plane s arrives)
  dbl2v l0p[2];                 // level 0 of plane s-1 at the two level-1 lines
  dbl2v p1[2];                  // partial level-1 sums of plane s-1 (slots -W .. +n)
  uint32_t c1lo[2] = {0u, 0u}, c1hi[2] = {0u, 0u};  // their codes
  dbl2v l1p = dbl2v{0.0, 0.0};  // level 1 of plane s-2, own line
  dbl2v p2 = dbl2v{0.0, 0.0};   // partial level-2 sums of plane s-2
  uint32_t c2lo = 0u, c2hi = 0u;
  dbl2v k1 = dbl2v{0.0, 0.0}, k2 = dbl2v{0.0, 0.0};  // C = 1: own level 1, 2 of plane s-3
  p1[0] = p1[1] = dbl2v{0.0, 0.0};
  const int64_t zlast = z1 + 1;
  St2tStage<CB> st;
  // C = 1: dual m+1's products at plane z = s-3 (level 1, 2 of chain 0 from LDS)
  auto level2_products = [&](int64_t z) {
    if (z >= z0 && z < z1) {
      cross(z, 2);
      if constexpr (C == 1) {
        const dbl2v o1 = reinterpret_cast<const dbl2v*>(L.xb[H][0])[tid];
        const dbl2v o2 = reinterpret_cast<const dbl2v*>(L.xb[H][1])[tid];
        epi_products<EPI>(o1.x, k1.x, o2.x, k2.x, 0.0, acc);
        epi_products<EPI>(o1.y, k1.y, o2.y, k2.y, 0.0, acc);
      }
    }
  };
  auto step = [&](int64_t s) {
    // (1) level 0 of plane s to LDS; chain 1 hands its own line's level 0 of
    // plane s-1 to chain 0 (dual m's x2); the next plane's loads take the
    // stage registers
#pragma unroll
    for (int j = 0; j < 3; ++j) reinterpret_cast<dbl2v*>(L.x0[C] + (3 * H + j) * kSBlock)[tid] = st.x[j];
    if constexpr (C == 1) reinterpret_cast<dbl2v*>(L.xa[H])[tid] = l0p[IO];
    uint32_t clo[2], chi[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      clo[i] = st.clo[i];
      chi[i] = st.chi[i];
    }
    issue(st, s + 1 <= zlast ? s + 1 : s);  // (the last step re-reads its own plane)
    __syncthreads();
    level2_products(s - 3);
    dbl2v x2p = dbl2v{0.0, 0.0};  // C = 0: chain 1's level 0 of plane s-1, own line
    if constexpr (C == 0) x2p = reinterpret_cast<const dbl2v*>(L.xa[H])[tid];
    const dbl2v x1p = l0p[IO];    // own chain's level 0 of plane s-1, own line
    // (2) level 1: plane s-1 completed by +W, plane s started
    dbl2v l1[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const double* line = L.x0[C] + (1 + 2 * H + i) * kSBlock + 2 * tid;
      const dbl2v cx = *reinterpret_cast<const dbl2v*>(line);
      {
        double xl[7], xh[7], sl = p1[i].x, sh = p1[i].y;
        xl[6] = cx.x;
        xh[6] = cx.y;
        terms(I6{}, I7{}, c1lo[i], c1hi[i], xl, xh, sl, sh);
        l1[i] = dbl2v{sl, sh};
      }
      const dbl2v mn = *reinterpret_cast<const dbl2v*>(line - kSBlock);
      const dbl2v pn = *reinterpret_cast<const dbl2v*>(line + kSBlock);
      double xl[7], xh[7], sl = 0.0, sh = 0.0;
      xl[0] = l0p[i].x;  xh[0] = l0p[i].y;
      xl[1] = mn.x;      xh[1] = mn.y;
      xl[2] = line[-1];  xh[2] = cx.x;
      xl[3] = cx.x;      xh[3] = cx.y;
      xl[4] = cx.y;      xh[4] = line[2];
      xl[5] = pn.x;      xh[5] = pn.y;
      terms(I0{}, I6{}, clo[i], chi[i], xl, xh, sl, sh);
      p1[i] = dbl2v{sl, sh};
      l0p[i] = cx;
    }
    // (3) level 1 of plane s-1, own line (+ the outer margin) for level 2
    reinterpret_cast<dbl2v*>(L.x1[C] + 2 + H * kSBlock)[tid] = l1[IO];
    if (H == 0 && tid == kBlock - 1) L.x1[C][1] = l1[0].y;                 // p0-1, row 511
    if (H == 1 && tid == 0) L.x1[C][2 + 2 * kSBlock] = l1[1].x;            // p0+2, row 0
    __syncthreads();
    // (4) dual m's products at plane s-1: level 0 x level 1, both chains
    const int64_t zp1 = s - 1;
    if (zp1 >= z0 && zp1 < z1) {
      cross(zp1, 1);
      if constexpr (C == 0) {
        const dbl2v y2 = reinterpret_cast<const dbl2v*>(L.x1[1] + 2 + H * kSBlock)[tid];
        epi_products<EPI>(x1p.x, x2p.x, l1[IO].x, y2.x, 0.0, acc);
        epi_products<EPI>(x1p.y, x2p.y, l1[IO].y, y2.y, 0.0, acc);
      }
    }
    // (5) level 2: plane s-2 completed by +W (level 1 of plane s-1), plane s-1 started
    {
      double xl[7], xh[7], sl = p2.x, sh = p2.y;
      xl[6] = l1[IO].x;
      xh[6] = l1[IO].y;
      terms(I6{}, I7{}, c2lo, c2hi, xl, xh, sl, sh);
      const int64_t zp2 = s - 2;
      if (zp2 >= z0 && zp2 < z1) {
        if constexpr (!PO) {
          const int64_t row = zp2 * W + pown * kSBlock + 2 * tid;
          __builtin_nontemporal_store(dbl2v{sl, sh},
                                      reinterpret_cast<dbl2v*>((C == 0 ? a.y1 : a.y2) + row));
        }
      }
      if constexpr (C == 0) {  // chain 0's level 1 and 2 of plane s-2 for the level-2 products
        reinterpret_cast<dbl2v*>(L.xb[H][0])[tid] = l1p;
        reinterpret_cast<dbl2v*>(L.xb[H][1])[tid] = dbl2v{sl, sh};
      } else {
        k1 = l1p;
        k2 = dbl2v{sl, sh};
      }
    }
    {
      const double* lx = L.x1[C] + 2 + H * kSBlock + 2 * tid;
      const dbl2v cx = l1[IO];
      const dbl2v mn = H == 0 ? l1[0] : *reinterpret_cast<const dbl2v*>(lx - kSBlock);
      const dbl2v pn = H == 0 ? *reinterpret_cast<const dbl2v*>(lx + kSBlock) : l1[1];
      double xl[7], xh[7], sl = 0.0, sh = 0.0;
      xl[0] = l1p.x;   xh[0] = l1p.y;
      xl[1] = mn.x;    xh[1] = mn.y;
      xl[2] = lx[-1];  xh[2] = cx.x;
      xl[3] = cx.x;    xh[3] = cx.y;
      xl[4] = cx.y;    xh[4] = lx[2];
      xl[5] = pn.x;    xh[5] = pn.y;
      terms(I0{}, I6{}, c1lo[IO], c1hi[IO], xl, xh, sl, sh);
      p2 = dbl2v{sl, sh};
      l1p = cx;
      c2lo = c1lo[IO];
      c2hi = c1hi[IO];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      c1lo[i] = clo[i];
      c1hi[i] = chi[i];
    }
  };

  // prologue: level 0 of plane z0-2 (the -W operand of plane z0-1's level 1),
  // plane z0-1 in flight
#pragma unroll
  for (int i = 0; i < 2; ++i) l0p[i] = ld(row_of(z0 - 2, 1 + 2 * H + i));
  issue(st, z0 - 1);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();                      // tab
  for (int64_t s = z0 - 1; s <= zlast; ++s) step(s);
  __syncthreads();
  level2_products(z1 - 1);  // the last plane's, written by the last step
  flush(C == 0);            // level 1's last segment (group (H, 0))
  flush(C == 1);            // level 2's (group (H, 1))
}

// KR_ST2T_W (compile time, A/B builds): waves-per-SIMD target (0: the
// compiler's choice).
#ifndef KR_ST2T_W
#define KR_ST2T_W 0
#endif
template <int EPI, int CB, bool PO>
__global__ __launch_bounds__(4 * kBlock)
#if KR_ST2T_W > 0
__attribute__((amdgpu_waves_per_eu(KR_ST2T_W)))
#endif
void spmv_stencil2t_kernel(SpmvArgs a) {
  if (a.stop && *a.stop != 0.0) return;
  static_assert(CB == 2 || CB == 4, "tiled fused basis pair: narrow codes");
  extern __shared__ __attribute__((aligned(16))) double s2t_dyn[];
  St2tLds& L = *reinterpret_cast<St2tLds*>(s2t_dyn);
  if (threadIdx.x < (unsigned)a.ntab) L.tab[threadIdx.x] = a.vtab[threadIdx.x];
  // position-major pairs: XCD q = B & 7 walks the position pairs of
  // [q P/8, (q+1) P/8) over the plane segments of the walk grid
  const int64_t P = a.st_P, PP = P >> 3;
  const int64_t B = blockIdx.x, q = B & 7, w2 = B >> 3;
  const int64_t half = PP >> 1, Zw = gridDim.x / (P >> 1);
  const int64_t p0 = q * PP + 2 * (w2 % half);
  const int64_t zs = w2 / half;
  const int g = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kBlock));
  const int tid = (int)(threadIdx.x % kBlock);
  switch (g) {
    case 0: st2t_walk<EPI, CB, PO, 0, 0>(a, L, tid, p0, q, zs, Zw); break;
    case 1: st2t_walk<EPI, CB, PO, 0, 1>(a, L, tid, p0, q, zs, Zw); break;
    case 2: st2t_walk<EPI, CB, PO, 1, 0>(a, L, tid, p0, q, zs, Zw); break;
    default: st2t_walk<EPI, CB, PO, 1, 1>(a, L, tid, p0, q, zs, Zw); break;
  }
}

template <int EPI, int CB, bool PO>
void st2t_launch_t(const SpmvArgs& a, int nblocks, hipStream_t s) {
  static std::atomic<uint64_t> opted{0};  // per device (opt_in_lds)
  opt_in_lds(opted, reinterpret_cast<const void*>(spmv_stencil2t_kernel<EPI, CB, PO>), kSt2tLds);
  spmv_stencil2t_kernel<EPI, CB, PO><<<nblocks, 4 * kBlock, kSt2tLds, s>>>(a);
  KR_HIP_CHECK(hipGetLastError());
}

template <int EPI>
inline void spmv_stencil2t_launch(const SpmvArgs& a, int nblocks, hipStream_t s) {
  const int64_t planes = a.st_P > 0 ? a.n / ((int64_t)a.st_P * kSBlock) : 0;
  KR_REQUIRE(a.scode && a.st_P % 16 == 0 && a.st_nm == 7 && a.st_nfar == 2 &&
                 a.st_far[0] == -kSBlock && a.st_far[1] == kSBlock &&
                 a.n % ((int64_t)a.st_P * kSBlock) == 0 && a.rb_gap == 0 && a.partials2 &&
                 (a.st_cb == 2 || a.st_cb == 4) && a.st2_z1 > 0 && a.st2_z2 > 0 &&
                 nblocks % (a.st_P / 2) == 0 && a.st2_z1 % (2 * nblocks / a.st_P) == 0 &&
                 a.st2_z2 % (2 * nblocks / a.st_P) == 0 && planes >= a.st2_z1 &&
                 planes >= a.st2_z2,
             "tiled fused basis pair: 7-point stencil with n = 512, P % 16 == 0, whole planes, "
             "narrow codes, a walk grid dividing both dual grids");
  const bool po = a.products_only != 0;
  if (a.st_cb == 2)
    po ? st2t_launch_t<EPI, 2, true>(a, nblocks, s) : st2t_launch_t<EPI, 2, false>(a, nblocks, s);
  else
    po ? st2t_launch_t<EPI, 4, true>(a, nblocks, s) : st2t_launch_t<EPI, 4, false>(a, nblocks, s);
}
