// The box walks (gfx950): matrix-free multi-level plane walks for a
// constant-coefficient 7-point stencil on a box with n = 512, each bitwise
// the launches it replaces (DESIGN.md section 5 "Box walks"):
//   spmv_stencil2b_kernel  two k-skip basis duals (+ both Gram products)
//   spmv_step2b_kernel     two k-skip MrR steps (VIRT: steps 0-2)
//   spmv_step2h_kernel     the last two steps + the next outer iteration's head
//
// The box fused basis pair: two chained k-skip basis SpMVs in ONE
// walk for a constant-coefficient 7-point stencil on a box with n = 512
// (System::build_box checks it entry by entry: Shard::st_box).
//
// Same job as spmv_stencil2t_kernel (kr_stencil.h, "Tiled fused basis pair";
// v3/gpu/kskipmrr.py:45-59 -- Ar[m+2], Ay[m+1] = A (Ar[m+1], Ay[m]) and
// Ar[m+3], Ay[m+2] = A (Ar[m+2], Ay[m+1]), with both duals' Gram products):
// level 1 stays on chip, so a pair moves the HBM bytes of ONE dual SpMV.
// Rounds 3-4 measured that kernel issue-bound (~1,300 instructions per plane
// step and wave, ~530 of them scalar -- one scalar unit serves the CU's 16
// waves -- and every row's codes decoded once per level and chain). Here the
// matrix is not read at all:
//
//  * Values: every entry of slot k (offset -W, -n, -1, 0, +1, +n, +W) is the
//    same double V[k] (SpmvArgs::st_v, scalar registers).
//  * Absent entries are exactly the box faces (x = 0 / 511, y = 0 / P-1,
//    z = 0 / planes-1). Their operand is read as 0.0 -- zero halo rows on the
//    x faces, zero lines for positions outside [0, P) (y faces), zero planes
//    outside [0, planes) (z faces; the loads go out of the buffer's range and
//    return 0, level 1 is set to 0 there) -- and V[k] * 0.0 = +-0 added to a
//    running sum leaves it unchanged: a row sum starts at +0.0 and IEEE
//    round-to-nearest addition gives -0 only for (-0) + (-0), so the sum is
//    never -0, and s + (+-0) = s. V[k] is finite (the host checks), so every
//    row equals scipy's csr_matvec bit for bit: its entries in stored order
//    from 0.0, each product rounded, no FMA.
//  * The walk's bookkeeping is 32-bit and incremental; nothing in the loop
//    divides. One plane step is ~30 scalar instructions per wave.
//
// Layout: a workgroup walks x-segment xs (SL = 512 / XS rows) of the adjacent
// positions p0, p0 + 1 (p0 even) over one plane segment; four groups g = (H,
// C) of SL / 2 lanes: line half H, chain C (0: x1 = Ar[m+1], 1: x2 = Ay[m]);
// lane t owns rows 2t, 2t + 1 of the segment (the dual kernel's lane mapping
// within its wave xs * SL / 128 + ...):
//
//   level 0 (loaded)  : positions p0-2 .. p0+3, group (H, C) loads 3H .. 3H+2
//   level 1 (computed): positions p0-1 .. p0+2, group (H, C) computes 2H+1, 2H+2
//   level 2 (stored)  : positions p0, p0+1, group (H, C) owns p0 + H
//
// An LDS line holds the segment's rows and two halo rows on each side (the
// x neighbours of the segment's end rows, loaded with it; 0.0 on an x face).
// The level-1 value of the own line's two halo rows (rows -1 and SL, the +-1
// operands of level 2's end rows) is computed by two lanes of the group.
// XS = 4: 256-thread workgroups, ~29 KB of LDS, four per CU, so one
// workgroup's barriers overlap the others' work; XS = 1: one 1024-thread
// workgroup per CU, halo rows always x faces (no halo loads, stores or
// sums at all). Measured (st2b_xsegments): XS = 1 for both pairs.
//
// Step s (level 0 of plane s arrives, loaded one step ahead): level 1 of
// plane s-1 is completed by its +W term and plane s's sum started (-W .. +n);
// level 2 of plane s-2 is completed the same way and plane s-1's started.
// Level 0 of the plane and level 1 of plane s-1 go through LDS for the +-1
// and +-n operands. Two barriers per step.
//
// Products (bitwise the two dual launches'): dual m's (level 0 x level 1) of
// position p0 + H are accumulated by group (H, 0), dual m+1's (level 1 x
// level 2) by group (H, 1) -- each lane plane by plane, row 2t then 2t+1,
// the other chain's operands read from LDS -- exactly as the dual launch's
// wave of that (position, segment, x quarter) accumulates them; at each
// segment boundary of a level's dual grid each wave's shuffle-reduced value
// goes to its x quarter's slot of SpmvArgs::partq, and st2b_combine_kernel
// sums the four quarters in block_reduce_store's order into the partial of
// the virtual workgroup.
#include "kr_spmv.h"

// Ablations (timing-only library builds, wrong results; same-box A/B, never
// the library build): bit 0 no level-2 sums or stores, 1 no products, 2 the
// +-1 operands from the own rows (no LDS reads for them), 3 no second barrier,
// 4 no level-0 LDS stores, 5 no level-1 LDS stores, 6 no product exchange stores.
#ifndef KR_ST2B_AB
#define KR_ST2B_AB 0
#endif
// The +-1 operands of the level-1 / level-2 sums: by DPP from the own rows
// (wave_shr / wave_shl, the wave's two edge rows from LDS by uniform reads)
// or by per-lane LDS reads of rows 2t-1 and 2t+2 (16-byte lane stride: bank
// conflicts). KR_ST2B_DPP bits: 0 the storing pair's level-1 sums, 1 its
// level-2 sums, 2 / 3 the products-only pair's. Same-box A/B (profiles/r06u): DPP storing pair -0.04 ms of ~1.38,
// products-only pair +0.015 of ~1.06 (the shifts' VALU cost more there than
// the conflicts they remove); the reads' whole price (ablation 4) 0.07 / 0.04.
#ifndef KR_ST2B_DPP
#define KR_ST2B_DPP 3
#endif
// The same choice in the step walks, KR_STEP_DPP bits: 0 / 1 the step pair's
// (sp2b_walk) level 1 / 2, 2 / 3 / 4 the step pair + head's (sp3_walk)
// level 1 / 2 / 3. Same-box A/B (profiles/r06x, r06y): the step pair + head
// with DPP at all three levels -0.126 ms of ~1.78 over four reps (the pairs
// after it +0.03 ms each: the stores' drain moves into them), the step pair
// no measurable change.
#ifndef KR_STEP_DPP
#define KR_STEP_DPP 28
#endif
#if KR_ST2B_AB && !defined(KR_ALLOW_WRONG_RESULTS)
#error "KR_ST2B_AB builds give wrong results: define KR_ALLOW_WRONG_RESULTS (A/B libraries only)"
#endif

namespace kr {
namespace {

template <int XS>
struct St2bLds {
  static constexpr int SL = kSBlock / XS;  // rows per segment
  static constexpr int LL = SL + 4;        // an LDS line: halo rows -2, -1, the segment, SL, SL+1
  double x0[2][6][LL];  // level 0 of plane s: [chain][position p0-2+j][row + 2]
  double x1[2][4][LL];  // level 1 of plane s-1: [chain][position p0-1+j][row + 2]
  double xa[2][2][SL];  // [step parity][H]: chain 1's level 0 of plane s-1, own line
  double xb[2][2][SL];  // [H][level 1, 2]: chain 0's values of plane s-2, own line
};

__device__ __forceinline__ dbl2v lds2(const double* p) { return *reinterpret_cast<const dbl2v*>(p); }
__device__ __forceinline__ void lds2_st(double* p, dbl2v v) { *reinterpret_cast<dbl2v*>(p) = v; }

// Rows 2t-1 and 2t+2 of an LDS line (row0: its row 0; own: rows 2t, 2t+1 of
// lane t, wave wig of the line): DPP from the own rows with the wave's edge
// rows by uniform reads, or per-lane reads.
template <bool DPP>
__device__ __forceinline__ void st2b_nbrs(const double* row0, int t, int wig, dbl2v own,
                                          double& m1, double& q2) {
  if constexpr (DPP) {
    const double* we = row0 + 128 * wig;
    m1 = st_dpp_shr1(own.y, we[-1]);
    q2 = st_dpp_shl1(own.x, we[128]);
  } else {
    m1 = row0[2 * t - 1];
    q2 = row0[2 * t + 2];
  }
}

// One row pair of a 7-point row sum over slots -W .. +n (the +W term is added
// when the next plane arrives): operands xw (-W), mn / pn (-n / +n lines),
// m1 (row 2t-1), own (rows 2t, 2t+1), p2 (row 2t+2).
__device__ __forceinline__ dbl2v st2b_part(const double (&v)[7], dbl2v xw, dbl2v mn, double m1,
                                           dbl2v own, double p2, dbl2v pn) {
  double sl = 0.0, sh = 0.0;
  sl = sl + v[0] * xw.x;   sh = sh + v[0] * xw.y;
  sl = sl + v[1] * mn.x;   sh = sh + v[1] * mn.y;
  sl = sl + v[2] * m1;     sh = sh + v[2] * own.x;
  sl = sl + v[3] * own.x;  sh = sh + v[3] * own.y;
  sl = sl + v[4] * own.y;  sh = sh + v[4] * p2;
  sl = sl + v[5] * pn.x;   sh = sh + v[5] * pn.y;
  return dbl2v{sl, sh};
}
// The same sum for one row.
__device__ __forceinline__ double st2b_part1(const double (&v)[7], double xw, double mn, double m1,
                                             double own, double p1, double pn) {
  double s = 0.0;
  s = s + v[0] * xw;
  s = s + v[1] * mn;
  s = s + v[2] * m1;
  s = s + v[3] * own;
  s = s + v[4] * p1;
  s = s + v[5] * pn;
  return s;
}

template <int EPI, bool PO, int XS, int H, int C>
__device__ __forceinline__ void st2b_walk(const SpmvArgs& a, St2bLds<XS>& L, int t, int p0, int xs,
                                          int q, int zs, int Zw) {
  using Lds = St2bLds<XS>;
  constexpr int SL = Lds::SL;
  // XS = 1: whole lines, every halo row an x face -- no halo loads, stores or
  // halo-row sums (their LDS slots are zeroed once, spmv_stencil2b_kernel)
  constexpr bool XH = XS > 1;
  constexpr int G = SL / 2;      // lanes per group
  constexpr int NWG = G / 64;    // waves per group
  constexpr int NP = 7;
  constexpr bool kDpp1 = (KR_ST2B_DPP >> (PO ? 2 : 0)) & 1;  // level 1's +-1 operands by DPP
  constexpr bool kDpp2 = (KR_ST2B_DPP >> (PO ? 3 : 1)) & 1;  // level 2's
  constexpr int IO = H == 0 ? 1 : 0;  // own line among the group's two level-1 lines
  constexpr int J2 = 2 + H;           // own line's level-0 index (x0), x1 index 1 + H
  const int lane = t & 63, wig = __builtin_amdgcn_readfirstlane(t >> 6);
  const int quarter = xs * NWG + wig;  // the dual workgroup's wave this wave stands for
  const int P = a.st_P, PP = P >> 3;
  const int W = P * kSBlock;
  const int planes = (int)(a.n / W);
  const int z0 = (int)((int64_t)planes * zs / Zw), z1 = (int)((int64_t)planes * (zs + 1) / Zw);
  const int pown = p0 + H;
  double v[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) v[k] = a.st_v[k];

  // level-0 loads: segment xs of line jj (position p0 - 2 + 3H + jj) of
  // chain C at plane z, and its halo chunk (even lanes rows -2, -1; odd lanes
  // rows SL, SL+1); positions outside [0, P), planes outside [0, planes) and
  // halo rows past an x face read 0 (offset past the buffer: the range check
  // returns zeros)
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<double*>(C == 0 ? a.x1 : a.x2), 0, (int)(a.xlen * 8), 0x00020000);
  const uint32_t lb = (uint32_t)t * 16u;
  const uint32_t hb = (lane & 1) ? (uint32_t)SL * 8u : (uint32_t)-16;
  const uint32_t hm = -(uint32_t)((lane & 1) ? xs < XS - 1 : xs > 0);  // all ones: halo not a face
  uint32_t lbase[3], lok[3];
#pragma unroll
  for (int jj = 0; jj < 3; ++jj) {
    const int pos = p0 - 2 + 3 * H + jj;
    lok[jj] = -(uint32_t)(pos >= 0 && pos < P);
    lbase[jj] = (uint32_t)((a.xoff + (int64_t)pos * kSBlock + (int64_t)xs * SL) * 8);
  }
  const uint32_t wbytes = (uint32_t)W * 8u;
  constexpr uint32_t kOut = 0x80000000u;
  // the stage registers: written to LDS as soon as they arrive and reloaded
  // at once with the next plane (the own rows are read back from LDS), so
  // nothing copies a register a load is still writing
  dbl2v st[3], sth[3];
  auto issue = [&](int z) {
    const uint32_t zm = -(uint32_t)((unsigned)z < (unsigned)planes);  // all ones: plane in range
    const uint32_t zo = (uint32_t)z * wbytes;
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      // branch-free selects (a load under a branch costs the compiler's wait counts)
      const uint32_t m = zm & lok[jj], mh = m & hm;
      const uint32_t u = lbase[jj] + zo;
      st[jj] = st_bld2(rx, ((u & m) | (kOut & ~m)) + lb);
      if constexpr (XH) sth[jj] = st_bld2(rx, ((u + hb) & mh) | (kOut & ~mh));
    }
  };
  // level-1 lines outside [0, P) are 0 (the -n / +n of the y faces)
  bool l1ok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int pos = p0 - 1 + 2 * H + i;
    l1ok[i] = pos >= 0 && pos < P;
  }
  double* const ydst =
      (C == 0 ? a.y1 : a.y2) + (int64_t)pown * kSBlock + (int64_t)xs * SL + 2 * t;

  // ---- products: each wave's shuffle-reduced value to its x quarter of the
  // virtual workgroup (position, grid segment); st2b_combine_kernel sums them
  const int Z1 = a.st2_z1, Z2 = a.st2_z2;
  int seg = zs * ((C == 0 ? Z1 : Z2) / Zw);  // this group's level's current grid segment
  double acc[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) acc[k] = 0.0;
  auto flush = [&]() {
    const int64_t vwg = 8 * ((int64_t)seg * PP + (pown - q * PP)) + q;
    double* const dst = a.partq + ((int64_t)(C == 0 ? 0 : NP) * a.grid + vwg) * 4 + quarter;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      double r = acc[k];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) r += __shfl_down(r, off, 64);
      if (lane == 0) dst[(int64_t)k * a.grid * 4] = r;
      acc[k] = 0.0;
    }
    ++seg;
  };
  int sg1 = zs * (Z1 / Zw), sg2 = zs * (Z2 / Zw);
  int nb1 = (int)((int64_t)planes * (sg1 + 1) / Z1);  // level 1's next grid boundary
  int nb2 = (int)((int64_t)planes * (sg2 + 1) / Z2);
  auto cross1 = [&](int z) {
    if (z >= nb1) {
      if constexpr (C == 0) flush();
      ++sg1;
      nb1 = (int)((int64_t)planes * (sg1 + 1) / Z1);
    }
  };
  auto cross2 = [&](int z) {
    if (z >= nb2) {
      if constexpr (C == 1) flush();
      ++sg2;
      nb2 = (int)((int64_t)planes * (sg2 + 1) / Z2);
    }
  };

  // ---- carried state (step s: level 0 of plane s arrives)
  dbl2v l0p[2];                   // level 0 of plane s-1, the two level-1 lines
  dbl2v p1[2];                    // partial level-1 sums of plane s-1
  dbl2v l1p = dbl2v{0.0, 0.0};    // level 1 of plane s-2, own line
  dbl2v p2 = dbl2v{0.0, 0.0};     // partial level-2 sums of plane s-2
  dbl2v k1 = dbl2v{0.0, 0.0}, k2 = dbl2v{0.0, 0.0};  // C = 1: own level 1, 2 of plane s-3
  p1[0] = p1[1] = dbl2v{0.0, 0.0};
  // the own line's level-1 halo rows (lanes 0 / 1 of the group's first wave:
  // row -1 / SL): level 0 of plane s-1 there, partial sum of plane s-1
  double hl0p = 0.0, hp1 = 0.0;
  const bool hlane = wig == 0 && lane < 2;
  const int hr = (lane & 1) ? SL : -1;
  const bool hface = (lane & 1) ? xs == XS - 1 : xs == 0;
  const int tl = 2 + 2 * t;       // the lane's first row in an LDS line

  // C = 1: dual m+1's products at plane z (level 1, 2 of chain 0 from LDS)
  auto level2_products = [&](int z) {
    if (z >= z0 && z < z1) {
      cross2(z);
      if constexpr (C == 1) {
        const dbl2v o1 = lds2(&L.xb[H][0][2 * t]);
        const dbl2v o2 = lds2(&L.xb[H][1][2 * t]);
        if constexpr (!(KR_ST2B_AB & 2)) {
          epi_products<EPI>(o1.x, k1.x, o2.x, k2.x, 0.0, acc);
          epi_products<EPI>(o1.y, k1.y, o2.y, k2.y, 0.0, acc);
        } else {
          acc[0] += o1.x + o2.y;
        }
      }
    }
  };

  auto step = [&](int s) {
    // (1) plane s to LDS (chain 1 also hands its own line's level 0 of plane
    // s-1 to chain 0), then the next plane's loads into the stage registers
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      if constexpr (!(KR_ST2B_AB & 16)) lds2_st(&L.x0[C][3 * H + jj][tl], st[jj]);
      else if (st[jj].x == 1234.5) lds2_st(&L.x0[C][3 * H + jj][tl], st[jj]);
      if constexpr (XH)
        if (wig == 0 && lane < 2) lds2_st(&L.x0[C][3 * H + jj][(lane & 1) ? SL + 2 : 0], sth[jj]);
    }
    if constexpr (C == 1 && !(KR_ST2B_AB & 64)) lds2_st(&L.xa[s & 1][H][2 * t], l0p[IO]);
    issue(s + 1);
    __syncthreads();
    // (2) dual m+1's products of plane s-3
    level2_products(s - 3);
    // (3) level 1: plane s-1 completed (+W = this plane), plane s started
    const dbl2v x1own = l0p[IO];  // level 0 of plane s-1, own line (dual m's x / x2)
    const bool pok = (unsigned)(s - 1) < (unsigned)planes;
    dbl2v l1[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = 1 + 2 * H + i;
      const double* line = &L.x0[C][j][tl];
      const dbl2v own = lds2(line);
      const dbl2v c = dbl2v{p1[i].x + v[6] * own.x, p1[i].y + v[6] * own.y};
      l1[i] = (pok && l1ok[i]) ? c : dbl2v{0.0, 0.0};
      double m1, q2;
      if constexpr (kDpp1) {
        const double* we = &L.x0[C][j][2 + 128 * wig];  // the wave's first row
        m1 = st_dpp_shr1(own.y, we[-1]);
        q2 = st_dpp_shl1(own.x, we[128]);
      } else {
        m1 = (KR_ST2B_AB & 4) ? own.y : line[-1];
        q2 = (KR_ST2B_AB & 4) ? own.x : line[2];
      }
      p1[i] = st2b_part(v, l0p[i], lds2(&L.x0[C][j - 1][tl]), m1, own, q2, lds2(&L.x0[C][j + 1][tl]));
      l0p[i] = own;
    }
    // (4) level 1 of plane s-1 to LDS, with the own line's halo rows
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if constexpr (!(KR_ST2B_AB & 32)) lds2_st(&L.x1[C][2 * H + i][tl], l1[i]);
      else if (l1[i].x == 1234.5) lds2_st(&L.x1[C][2 * H + i][tl], l1[i]);
    if (XH && hlane) {
      const double* ln = &L.x0[C][J2][hr + 2];
      const double own = ln[0];
      const double c = hp1 + v[6] * own;
      L.x1[C][1 + H][hr + 2] = (pok && l1ok[IO] && !hface) ? c : 0.0;
      hp1 = st2b_part1(v, hl0p, L.x0[C][J2 - 1][hr + 2], ln[-1], own, ln[1], L.x0[C][J2 + 1][hr + 2]);
      hl0p = own;
    }
    if constexpr (!(KR_ST2B_AB & 8)) __syncthreads();
    // (5) dual m's products of plane s-1
    if (s - 1 >= z0 && s - 1 < z1) {
      cross1(s - 1);
      if constexpr (C == 0) {
        const dbl2v x2 = lds2(&L.xa[s & 1][H][2 * t]);
        const dbl2v y2 = lds2(&L.x1[1][1 + H][tl]);
        if constexpr (!(KR_ST2B_AB & 2)) {
          epi_products<EPI>(x1own.x, x2.x, l1[IO].x, y2.x, 0.0, acc);
          epi_products<EPI>(x1own.y, x2.y, l1[IO].y, y2.y, 0.0, acc);
        } else {
          acc[0] += x2.x + y2.y;
        }
      }
    }
    // (6) level 2: plane s-2 completed (+W = level 1 of plane s-1), stored;
    // plane s-1 started
    if constexpr (!(KR_ST2B_AB & 1)) {
      const dbl2v own = l1[IO];
      const dbl2v l2 = dbl2v{p2.x + v[6] * own.x, p2.y + v[6] * own.y};
      if constexpr (!PO) {
        if (s - 2 >= z0 && s - 2 < z1)
          __builtin_nontemporal_store(l2, reinterpret_cast<dbl2v*>(ydst + (int64_t)(s - 2) * W));
      }
      if constexpr (C == 0) {
        if constexpr (!(KR_ST2B_AB & 64)) {
          lds2_st(&L.xb[H][0][2 * t], l1p);
          lds2_st(&L.xb[H][1][2 * t], l2);
        } else {
          acc[1] += l2.x;
        }
      } else {
        k1 = l1p;
        k2 = l2;
      }
      const double* lx = &L.x1[C][1 + H][tl];
      double m1, q2;
      if constexpr (kDpp2) {
        const double* we = &L.x1[C][1 + H][2 + 128 * wig];
        m1 = st_dpp_shr1(own.y, we[-1]);
        q2 = st_dpp_shl1(own.x, we[128]);
      } else {
        m1 = (KR_ST2B_AB & 4) ? own.y : lx[-1];
        q2 = (KR_ST2B_AB & 4) ? own.x : lx[2];
      }
      p2 = st2b_part(v, l1p, lds2(&L.x1[C][H][tl]), m1, own, q2, lds2(&L.x1[C][2 + H][tl]));
      l1p = own;
    }
  };

  // prologue: level 0 of plane z0-2 (the -W operand of plane z0-1's level
  // 1), plane z0-1 in flight
  issue(z0 - 2);
#pragma unroll
  for (int i = 0; i < 2; ++i) l0p[i] = st[1 - H + i];
  // the own line's halo rows of plane z0-2 (lane 0: row -1, lane 1: row SL):
  // from the halo chunk (rows -2, -1 / SL, SL+1)
  if constexpr (XH) hl0p = (lane & 1) ? sth[1 - H + IO].x : sth[1 - H + IO].y;
  issue(z0 - 1);
  // one step per trip: two per trip (the carried state alternating registers
  // instead of being copied) measured slower for the products-only pair,
  // 1.015-1.030 -> 1.056-1.064 ms (same box, profiles/r06f), and the storing
  // walks spill at 128 VGPRs
  for (int s = z0 - 1; s <= z1 + 1; ++s) step(s);
  __syncthreads();
  level2_products(z1 - 1);  // the last plane's, written by the last step
  if constexpr (C == 0) flush();  // level 1's last segment (groups (H, 0))
  if constexpr (C == 1) flush();  // level 2's (groups (H, 1))
}

// Waves per SIMD: XS = 4 four 256-thread workgroups per CU (16 waves), XS = 2
// two of 512, XS = 1 one of 1024; <= 128 VGPRs in every case.
template <int EPI, bool PO, int XS>
__global__ __launch_bounds__(4 * kBlock / XS) __attribute__((amdgpu_waves_per_eu(4)))
void spmv_stencil2b_kernel(SpmvArgs a) {
  if (a.stop && *a.stop != 0.0) return;
  extern __shared__ __attribute__((aligned(16))) double s2b_dyn[];
  St2bLds<XS>& L = *reinterpret_cast<St2bLds<XS>*>(s2b_dyn);
  if constexpr (XS == 1) {
    // the x-face pads (rows -2, -1, 512, 513) of every line, read as 0.0;
    // visible after the first step's barrier, never written again
    constexpr int LL = St2bLds<XS>::LL;
    if (threadIdx.x < 80) {
      const int i = threadIdx.x >> 2, e = threadIdx.x & 3;  // line i of 20, pad e
      double* line = i < 12 ? &L.x0[i / 6][i % 6][0] : &L.x1[(i - 12) / 4][(i - 12) % 4][0];
      line[e < 2 ? e : LL - 4 + e] = 0.0;
    }
  }
  // XCD q = B & 7 walks the position pairs of [q P/8, (q+1) P/8): the x
  // segments of a tile, then the tiles, then the plane segments
  const int P = a.st_P, PP = P >> 3;
  const int B = blockIdx.x, q = B & 7, w2 = B >> 3;
  const int half = PP >> 1, Zw = gridDim.x / ((P >> 1) * XS);
  const int xs = w2 % XS, w3 = w2 / XS;
  const int p0 = q * PP + 2 * (w3 % half);
  const int zs = w3 / half;
  constexpr int G = kBlock / XS;  // lanes per group
  const int g = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / G));
  const int t = (int)(threadIdx.x % G);
  switch (g) {
    case 0: st2b_walk<EPI, PO, XS, 0, 0>(a, L, t, p0, xs, q, zs, Zw); break;
    case 1: st2b_walk<EPI, PO, XS, 0, 1>(a, L, t, p0, xs, q, zs, Zw); break;
    case 2: st2b_walk<EPI, PO, XS, 1, 0>(a, L, t, p0, xs, q, zs, Zw); break;
    default: st2b_walk<EPI, PO, XS, 1, 1>(a, L, t, p0, xs, q, zs, Zw); break;
  }
}

// partials[kk * grid + v] = ((q0 + q1) + q2) + q3 of the four x quarters of
// virtual workgroup v (block_reduce_store's order): kk < 7 over the n1
// workgroups of dual m's grid, kk >= 7 over dual m+1's n2.
__global__ __launch_bounds__(kBlock) void st2b_combine_kernel(const double* __restrict__ partq,
                                                               double* __restrict__ partials,
                                                               int grid, int n1, int n2) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int kk = (int)(i / grid), v = (int)(i % grid);
  if (kk >= 14 || v >= (kk < 7 ? n1 : n2)) return;
  const dbl2v lo = *reinterpret_cast<const dbl2v*>(partq + ((int64_t)kk * grid + v) * 4);
  const dbl2v hi = *reinterpret_cast<const dbl2v*>(partq + ((int64_t)kk * grid + v) * 4 + 2);
  double s = lo.x;
  s = s + lo.y;
  s = s + hi.x;
  s = s + hi.y;
  partials[(int64_t)kk * grid + v] = s;
}

template <int EPI, bool PO, int XS>
void st2b_launch_t(const SpmvArgs& a, int nblocks, hipStream_t s) {
  static std::atomic<uint64_t> opted{0};  // per device (opt_in_lds)
  opt_in_lds(opted, reinterpret_cast<const void*>(spmv_stencil2b_kernel<EPI, PO, XS>),
             sizeof(St2bLds<XS>));
  spmv_stencil2b_kernel<EPI, PO, XS><<<nblocks, 4 * kBlock / XS, sizeof(St2bLds<XS>), s>>>(a);
  KR_HIP_CHECK(hipGetLastError());
}

template <int EPI, int XS>
void st2b_launch_x(const SpmvArgs& a, int nblocks, hipStream_t s) {
  if (a.products_only)
    st2b_launch_t<EPI, true, XS>(a, nblocks, s);
  else
    st2b_launch_t<EPI, false, XS>(a, nblocks, s);
}

template <int EPI>
void st2b_launch_e(const SpmvArgs& a, int nblocks, int xs, hipStream_t s) {
  switch (xs) {
    case 1: st2b_launch_x<EPI, 1>(a, nblocks, s); return;
    case 2: st2b_launch_x<EPI, 2>(a, nblocks, s); return;
    default: st2b_launch_x<EPI, 4>(a, nblocks, s); return;
  }
}

// ---------------------------------------------------------------------------
// The box step pair: two consecutive fused k-skip MrR steps in ONE walk
// (v3/gpu/kskipmrr.py:88-95; the unfused kernels are the EPI_STEP_MRR_*
// epilogues, kr_spmv.h epi_values). Step j: Ar1 = A r_a; y_b = eta_j y_a +
// zeta_j Ar1; z_b = eta_j z_a - zeta_j r_a; r_b = r_a - y_b. Step j+1: Ar1' =
// A r_b; y_c = eta' y_b + zeta' Ar1'; z_c = eta' z_b - zeta' r_b; r_c = r_b -
// y_c. x: the two steps' kinds (KskipMrrSession::step_kind) subtract z_a
// (XM bit 0: step j is an x2 step), z_b (bit 1) and z_c (bit 2) in that
// order, each rounded, as the two kernels do. r_b (level 1) and y_b never
// leave the chip: 8 vectors of HBM traffic (r, y, z, x in and out) instead of
// the two kernels' 14 (EPI_STEP_MRR_NOX 6 + EPI_STEP_MRR_X2 8).
//
// VIRT: steps 0, 1 and 2 of an outer iteration (EPI_STEP_MRR_FIRST2's two
// steps, then step 2): level 0 is r_1 = r_0 - (eta_0 y_0 + zeta_0 Ar1_0),
// formed from three gathered vectors as FIRST2 forms it (virtual_r1), level
// 1 step 1 (c2, c3), level 2 step 2 (c4, c5); x = ((x [- z_0 if xpend]) -
// z_1) - z_2 [- z_3: XM bit 2], FIRST2's statements. 9 vectors instead of
// FIRST2's 9 plus the following step's 6.
//
// The box pair's walk with one chain: a 1024-thread workgroup walks the
// positions p0, p0 + 1 of a plane segment; group g (256 lanes, rows 2t, 2t+1)
// owns level-1 line g (position p0-1+g): level 0 of r for lines 0 .. 5
// (group 0 also loads line 0, group 3 line 5), y_a of its line; groups 1 and
// 2 (positions p0, p0+1) also run level 2 and the stores. Every statement is
// the unfused kernels', in their order, so the results are bitwise theirs.
// y and r go to other buffers than they are read from (other workgroups
// still read them on their halo lines); z and x in place (own rows).
// ---------------------------------------------------------------------------
struct Sp2bLds {
  double x0[6][kSBlock + 4];  // level 0 of plane s: [position p0-2+j][row + 2], zero pads
  double x1[4][kSBlock + 4];  // level 1 of plane s-1: [position p0-1+j][row + 2]
};

template <int G, bool VIRT, int XM>
__device__ __forceinline__ void sp2b_walk(const SpmvArgs& a, Sp2bLds& L, int t, int p0, int zs,
                                          int Zw) {
  constexpr bool OUT = G == 1 || G == 2;          // level 2 and the stores
  constexpr int J = G + 1;                        // the group's level-1 line in x0
  constexpr int NL = (G == 0 || G == 3) ? 2 : 1;  // level-0 lines the group loads
  constexpr int L0 = G == 0 ? 0 : G + 1;          // the first of them
  constexpr int NV = VIRT ? 3 : 1;                // gathered vectors per level-0 line
  const int P = a.st_P;
  const int W = P * kSBlock;
  const int planes = (int)(a.n / W);
  const int z0 = (int)((int64_t)planes * zs / Zw), z1 = (int)((int64_t)planes * (zs + 1) / Zw);
  const int wig = __builtin_amdgcn_readfirstlane(t >> 6);  // the lane's wave in its line
  double v[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) v[k] = a.st_v[k];
  // level 1 / level 2 scalars (VIRT: step 0's are c0, c1)
  const double e1 = VIRT ? a.c2 : a.c0, f1 = VIRT ? a.c3 : a.c1;
  const double e2 = VIRT ? a.c4 : a.c2, f2 = VIRT ? a.c5 : a.c3;

  // gathered vectors: r (x1), and VIRT y_0 (x2), Ar1_0 (x3); y_a (x2) of the
  // group's line otherwise
  const __amdgpu_buffer_rsrc_t rv[3] = {
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(a.x1), 0, (int)(a.xlen * 8), 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(a.x2), 0, (int)(a.xlen * 8), 0x00020000),
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(VIRT ? a.x3 : a.x2), 0,
                                        (int)(a.xlen * 8), 0x00020000)};
  const uint32_t lb = (uint32_t)t * 16u;
  const uint32_t wbytes = (uint32_t)W * 8u;
  constexpr uint32_t kOut = 0x80000000u;
  uint32_t lbase[NL], lok[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int pos = p0 - 2 + L0 + i;
    lok[i] = -(uint32_t)(pos >= 0 && pos < P);
    lbase[i] = (uint32_t)((a.xoff + (int64_t)pos * kSBlock) * 8);
  }
  const int posj = p0 - 1 + G;
  const bool jok = posj >= 0 && posj < P;
  const uint32_t jbase = (uint32_t)((a.xoff + (int64_t)posj * kSBlock) * 8);
  const uint32_t jm = -(uint32_t)jok;
  // own rows of the output line (OUT groups): plane 0 row of lane t
  const int64_t orow = (int64_t)posj * kSBlock + 2 * t;

  dbl2v st[NL][NV], sty, stz, stx;
  auto issue = [&](int z) {  // level 0 of plane z, y_a of plane z-1, z_a / x of plane z-2
    const uint32_t zm = -(uint32_t)((unsigned)z < (unsigned)planes);
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const uint32_t m = zm & lok[i];
      const uint32_t u = (((lbase[i] + (uint32_t)z * wbytes) & m) | (kOut & ~m)) + lb;
#pragma unroll
      for (int c = 0; c < NV; ++c) st[i][c] = st_bld2(rv[c], u);
    }
    if constexpr (!VIRT) {
      const uint32_t ym = -(uint32_t)((unsigned)(z - 1) < (unsigned)planes) & jm;
      sty = st_bld2(rv[1], (((jbase + (uint32_t)(z - 1) * wbytes) & ym) | (kOut & ~ym)) + lb);
    }
    if constexpr (OUT) {
      const int zz = (unsigned)(z - 2) < (unsigned)planes ? z - 2 : 0;  // past a face: unused
      stz = *reinterpret_cast<const dbl2v*>(a.u2 + orow + (int64_t)zz * W);
      if constexpr (XM != 0 || VIRT)
        stx = *reinterpret_cast<const dbl2v*>(a.us + orow + (int64_t)zz * W);
    }
  };

  dbl2v l0p = dbl2v{0.0, 0.0};  // level 0 of plane s-1, own column of line J
  dbl2v p1 = dbl2v{0.0, 0.0};   // partial level-1 Ar1 sums of plane s-1
  dbl2v ya1 = dbl2v{0.0, 0.0};  // VIRT: y_1 of plane s-1 (line J)
  dbl2v ra2 = dbl2v{0.0, 0.0};  // OUT: level 0 of plane s-2 (r_a / VIRT r_1)
  dbl2v r0h1 = dbl2v{0.0, 0.0}, r0h2 = dbl2v{0.0, 0.0};  // OUT, VIRT: r_0 of planes s-1, s-2
  dbl2v yb2 = dbl2v{0.0, 0.0};  // OUT: level-1 y of plane s-2
  dbl2v l1p = dbl2v{0.0, 0.0};  // OUT: level 1 of plane s-2
  dbl2v p2 = dbl2v{0.0, 0.0};   // OUT: partial level-2 sums of plane s-2
  const int tl = 2 + 2 * t;

  // level 0 of the arriving plane into LDS (VIRT: r_1 formed from r_0, y_0,
  // Ar1_0 exactly as virtual_r1 / FIRST2's epilogue round it); returns y_1
  // of line J (VIRT)
  auto arrive = [&]() {
    dbl2v yj = dbl2v{0.0, 0.0};
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      dbl2v lv = st[i][0];
      if constexpr (VIRT) {
        const dbl2v r0 = st[i][0], y0 = st[i][1], ar = st[i][2];
        const double t1l = a.c0 * y0.x, t1h = a.c0 * y0.y;
        const double t2l = a.c1 * ar.x, t2h = a.c1 * ar.y;
        const dbl2v y1 = dbl2v{t1l + t2l, t1h + t2h};
        lv = dbl2v{r0.x - y1.x, r0.y - y1.y};
        if (L0 + i == J) yj = y1;
      }
      lds2_st(&L.x0[L0 + i][tl], lv);
    }
    return yj;
  };

  auto step = [&](int s) {
    // (1) level 0 of plane s to LDS; keep y_a (plane s-1), z_a and x (plane s-2)
    const dbl2v yj = arrive();
    dbl2v r0own = dbl2v{0.0, 0.0};
    if constexpr (VIRT && OUT) r0own = st[J - L0][0];
    const dbl2v ya = VIRT ? ya1 : sty;
    dbl2v za = dbl2v{0.0, 0.0}, xa = dbl2v{0.0, 0.0};
    if constexpr (OUT) {
      za = stz;
      if constexpr (XM != 0 || VIRT) xa = stx;
    }
    issue(s + 1);
    __syncthreads();
    // (2) level 1 at plane s-1 (line J): Ar1 completed by its +W term (this
    // plane), then y_b, r_b; plane s's sum started
    const double* line = &L.x0[J][tl];
    const dbl2v own = lds2(line);
    const dbl2v ar = dbl2v{p1.x + v[6] * own.x, p1.y + v[6] * own.y};
    dbl2v yb, rb;
    {
      const double t1l = e1 * ya.x, t1h = e1 * ya.y;
      const double t2l = f1 * ar.x, t2h = f1 * ar.y;
      yb = dbl2v{t1l + t2l, t1h + t2h};
      rb = dbl2v{l0p.x - yb.x, l0p.y - yb.y};
    }
    const bool pok = (unsigned)(s - 1) < (unsigned)planes;
    if (!(pok && jok)) rb = dbl2v{0.0, 0.0};  // level 1 off the box: the absent operand
    const dbl2v ra1 = l0p;  // level 0 of plane s-1
    double m1, q2;
    st2b_nbrs<(KR_STEP_DPP & 1) != 0>(&L.x0[J][2], t, wig, own, m1, q2);
    p1 = st2b_part(v, l0p, lds2(&L.x0[J - 1][tl]), m1, own, q2, lds2(&L.x0[J + 1][tl]));
    l0p = own;
    if constexpr (VIRT) ya1 = yj;
    lds2_st(&L.x1[G][tl], rb);
    __syncthreads();
    if constexpr (OUT) {
      // (3) level 2 at plane s-2 (Ar1' completed by level 1 of plane s-1),
      // the stores; plane s-1's Ar1' sum started
      const dbl2v ar2 = dbl2v{p2.x + v[6] * rb.x, p2.y + v[6] * rb.y};
      if (s - 2 >= z0 && s - 2 < z1) {
        // z and x of the steps before level 2, in the unfused kernels' order
        dbl2v zb, xn = xa;
        if constexpr (VIRT) {
          // FIRST2: z_1 = eta_0 z_0 - zeta_0 r_0; z_2 = eta_1 z_1 - zeta_1 r_1;
          // x = ((xpend ? x - z_0 : x) - z_1) - z_2
          const double t3l = a.c0 * za.x, t3h = a.c0 * za.y;
          const double t4l = a.c1 * r0h2.x, t4h = a.c1 * r0h2.y;
          const dbl2v zz1 = dbl2v{t3l - t4l, t3h - t4h};
          const double s3l = e1 * zz1.x, s3h = e1 * zz1.y;
          const double s4l = f1 * ra2.x, s4h = f1 * ra2.y;
          zb = dbl2v{s3l - s4l, s3h - s4h};
          if (a.xpend) xn = dbl2v{xn.x - za.x, xn.y - za.y};
          xn = dbl2v{xn.x - zz1.x, xn.y - zz1.y};
          xn = dbl2v{xn.x - zb.x, xn.y - zb.y};
        } else {
          // step j: z_b = eta_j z_a - zeta_j r_a; x2: x - z_a, then - z_b
          const double t3l = e1 * za.x, t3h = e1 * za.y;
          const double t4l = f1 * ra2.x, t4h = f1 * ra2.y;
          zb = dbl2v{t3l - t4l, t3h - t4h};
          if constexpr (XM & 1) xn = dbl2v{xn.x - za.x, xn.y - za.y};
          if constexpr (XM & 2) xn = dbl2v{xn.x - zb.x, xn.y - zb.y};
        }
        // the level-2 step (EPI_STEP_MRR_*: y, z, r; x - z_c)
        const double s1l = e2 * yb2.x, s1h = e2 * yb2.y;
        const double s2l = f2 * ar2.x, s2h = f2 * ar2.y;
        const dbl2v yc = dbl2v{s1l + s2l, s1h + s2h};
        const double s3l = e2 * zb.x, s3h = e2 * zb.y;
        const double s4l = f2 * l1p.x, s4h = f2 * l1p.y;
        const dbl2v zc = dbl2v{s3l - s4l, s3h - s4h};
        if constexpr (XM & 4) xn = dbl2v{xn.x - zc.x, xn.y - zc.y};
        const dbl2v rc = dbl2v{l1p.x - yc.x, l1p.y - yc.y};
        const int64_t row = orow + (int64_t)(s - 2) * W;
        __builtin_nontemporal_store(yc, reinterpret_cast<dbl2v*>(a.u1 + row));
        __builtin_nontemporal_store(zc, reinterpret_cast<dbl2v*>(a.u2 + row));
        if constexpr (XM != 0 || VIRT)
          __builtin_nontemporal_store(xn, reinterpret_cast<dbl2v*>(a.ud + row));
        __builtin_nontemporal_store(rc, reinterpret_cast<dbl2v*>(a.y1 + row));
      }
      double n1, n2;
      st2b_nbrs<(KR_STEP_DPP & 2) != 0>(&L.x1[G][2], t, wig, rb, n1, n2);
      p2 = st2b_part(v, l1p, lds2(&L.x1[G - 1][tl]), n1, rb, n2, lds2(&L.x1[G + 1][tl]));
      l1p = rb;
      yb2 = yb;
      ra2 = ra1;
      if constexpr (VIRT) {
        r0h2 = r0h1;
        r0h1 = r0own;
      }
    }
  };

  // prologue: level 0 of plane z0-2 (the -W operand of plane z0-1), plane
  // z0-1 in flight
  issue(z0 - 2);
  {
    const dbl2v yj = arrive();  // LDS lines overwritten by the first step before any read
    l0p = lds2(&L.x0[J][tl]);
    if constexpr (VIRT) ya1 = yj;
    if constexpr (VIRT && OUT) r0h1 = st[J - L0][0];
  }
  issue(z0 - 1);
  for (int s = z0 - 1; s <= z1 + 1; ++s) step(s);
}

template <bool VIRT, int XM>
__global__ __launch_bounds__(4 * kBlock) __attribute__((amdgpu_waves_per_eu(4)))
void spmv_step2b_kernel(SpmvArgs a) {
  if (a.stop && *a.stop != 0.0) return;
  extern __shared__ __attribute__((aligned(16))) double sp2b_dyn[];
  Sp2bLds& L = *reinterpret_cast<Sp2bLds*>(sp2b_dyn);
  // the LDS lines' zero pads (x faces), visible after the first step's barrier
  if (threadIdx.x < 40) {
    const int i = threadIdx.x >> 2, e = threadIdx.x & 3;  // line i of 10, pad e
    double* line = i < 6 ? &L.x0[i][0] : &L.x1[i - 6][0];
    line[e < 2 ? e : kSBlock + e] = 0.0;
  }
  const int P = a.st_P, PP = P >> 3;
  const int B = blockIdx.x, q = B & 7, w2 = B >> 3;
  const int half = PP >> 1, Zw = gridDim.x / (P >> 1);
  const int p0 = q * PP + 2 * (w2 % half);
  const int zs = w2 / half;
  const int g = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kBlock));
  const int t = (int)(threadIdx.x % kBlock);
  switch (g) {
    case 0: sp2b_walk<0, VIRT, XM>(a, L, t, p0, zs, Zw); break;
    case 1: sp2b_walk<1, VIRT, XM>(a, L, t, p0, zs, Zw); break;
    case 2: sp2b_walk<2, VIRT, XM>(a, L, t, p0, zs, Zw); break;
    default: sp2b_walk<3, VIRT, XM>(a, L, t, p0, zs, Zw); break;
  }
}

template <bool VIRT, int XM>
void sp2b_launch_t(const SpmvArgs& a, int nblocks, hipStream_t s) {
  static std::atomic<uint64_t> opted{0};
  opt_in_lds(opted, reinterpret_cast<const void*>(spmv_step2b_kernel<VIRT, XM>), sizeof(Sp2bLds));
  spmv_step2b_kernel<VIRT, XM><<<nblocks, 4 * kBlock, sizeof(Sp2bLds), s>>>(a);
  KR_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// The box step pair + head: the LAST two k-skip MrR steps of an outer
// iteration (k-1, k) and the next outer iteration's head SpMV (EPI_HEAD_MRR,
// v3/gpu/kskipmrr.py:40-44: Ar1 = A r, products <r,r> <r,Ar1> <Ar1,Ar1>
// <y,Ar1> <y,y>) in ONE walk. Levels 1 and 2 are spmv_step2b_kernel's
// statements (r_b, y_b; r_c, y_c, z_c, x); level 3 is the head at the two
// output lines, its Ar1 summed in stored order and its products accumulated
// per (x quarter, head-grid segment) exactly as the head launch's waves
// accumulate them (flushed at its segment boundaries, combined by
// sp3_combine_kernel in block_reduce_store's order). So the results are
// bitwise the step-pair launch followed by the head launch, and the HBM
// traffic is 9 vectors (r, y, z, x in; r, y, z, x, Ar1 out) instead of 8 + 3.
//
// Lines (positions p0 - 3 + j): level 0 (r_a) j = 0..7, level 1 (r_b) j =
// 1..6, level 2 (r_c) j = 2..5, level 3 (Ar1) j = 3, 4. Four groups of 256
// lanes (rows 2t, 2t+1 of whole 512-row lines): group G loads level-0 lines
// 2G, 2G+1; level 1 of lines {1,2}, {3}, {4}, {5,6}; level 2 of line G + 2;
// groups 1 and 2 also level 3 and the stores. Three barriers per plane step.
// ---------------------------------------------------------------------------
struct Sp3Lds {
  double x0[8][kSBlock + 4];  // level 0 of plane s: [line][row + 2], zero pads
  double x1[6][kSBlock + 4];  // level 1 of plane s-1, lines 1..6
  double x2[4][kSBlock + 4];  // level 2 of plane s-2, lines 2..5
};

template <int G, int XM>
__device__ __forceinline__ void sp3_walk(const SpmvArgs& a, Sp3Lds& L, int t, int p0, int q, int zs,
                                         int Zw) {
  constexpr bool OUT = G == 1 || G == 2;              // levels 2's stores, level 3
  constexpr int N1 = (G == 0 || G == 3) ? 2 : 1;     // level-1 lines
  constexpr int J1 = G == 0 ? 1 : G == 3 ? 5 : G + 2;  // the first of them
  constexpr int J2 = G + 2;                           // the level-2 (and level-3) line
  constexpr int I2 = J2 - J1;                         // its index among the level-1 lines
  constexpr int NP = 5;
  const int lane = t & 63, quarter = t >> 6;
  const int wig = __builtin_amdgcn_readfirstlane(t >> 6);  // the lane's wave in its line
  const int P = a.st_P, PP = P >> 3;
  const int W = P * kSBlock;
  const int planes = (int)(a.n / W);
  const int z0 = (int)((int64_t)planes * zs / Zw), z1 = (int)((int64_t)planes * (zs + 1) / Zw);
  double v[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) v[k] = a.st_v[k];
  const double e1 = a.c0, f1 = a.c1, e2 = a.c2, f2 = a.c3;

  const __amdgpu_buffer_rsrc_t rr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(a.x1), 0, (int)(a.xlen * 8), 0x00020000);
  const __amdgpu_buffer_rsrc_t ry =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(a.x2), 0, (int)(a.xlen * 8), 0x00020000);
  const uint32_t lb = (uint32_t)t * 16u;
  const uint32_t wbytes = (uint32_t)W * 8u;
  constexpr uint32_t kOut = 0x80000000u;
  auto line_base = [&](int j) { return (uint32_t)((a.xoff + (int64_t)(p0 - 3 + j) * kSBlock) * 8); };
  auto line_ok = [&](int j) { return p0 - 3 + j >= 0 && p0 - 3 + j < P; };
  uint32_t lbase[2], lok[2], ybase[N1], yok[N1];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    lbase[i] = line_base(2 * G + i);
    lok[i] = -(uint32_t)line_ok(2 * G + i);
  }
  bool l1ok[N1];
#pragma unroll
  for (int i = 0; i < N1; ++i) {
    ybase[i] = line_base(J1 + i);
    yok[i] = -(uint32_t)line_ok(J1 + i);
    l1ok[i] = line_ok(J1 + i);
  }
  const bool l2ok = line_ok(J2);
  const int pown = p0 - 3 + J2;  // OUT: the output line's position
  const int64_t orow = (int64_t)pown * kSBlock + 2 * t;

  dbl2v st[2], sty[N1];
  auto issue = [&](int z) {  // level 0 of plane z, y_a of plane z-1
    const uint32_t zm = -(uint32_t)((unsigned)z < (unsigned)planes);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t m = zm & lok[i];
      st[i] = st_bld2(rr, (((lbase[i] + (uint32_t)z * wbytes) & m) | (kOut & ~m)) + lb);
    }
    const uint32_t ym = -(uint32_t)((unsigned)(z - 1) < (unsigned)planes);
#pragma unroll
    for (int i = 0; i < N1; ++i) {
      const uint32_t m = ym & yok[i];
      sty[i] = st_bld2(ry, (((ybase[i] + (uint32_t)(z - 1) * wbytes) & m) | (kOut & ~m)) + lb);
    }
  };

  // ---- level-3 products (OUT): each wave's shuffle-reduced value to its x
  // quarter of the head launch's workgroup (position, grid segment)
  const int Zh = a.st2_z1;  // the head grid's plane segments
  int seg = zs * (Zh / Zw);
  int nb = (int)((int64_t)planes * (seg + 1) / Zh);
  double acc[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) acc[k] = 0.0;
  auto flush = [&]() {
    const int64_t vwg = 8 * ((int64_t)seg * PP + (pown - q * PP)) + q;
    double* const dst = a.partq + vwg * 4 + quarter;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      double r = acc[k];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) r += __shfl_down(r, off, 64);
      if (lane == 0) dst[(int64_t)k * a.grid * 4] = r;
      acc[k] = 0.0;
    }
  };

  // ---- carried state (step s: level 0 of plane s arrives)
  dbl2v l0p[N1], p1[N1];                          // level 0 of plane s-1, partial level 1 of s-1
  dbl2v yb2 = dbl2v{0.0, 0.0};                    // y_b of plane s-2 (line J2)
  dbl2v l1p = dbl2v{0.0, 0.0};                    // r_b of plane s-2 (line J2)
  dbl2v p2 = dbl2v{0.0, 0.0};                     // partial level 2 of plane s-2
  dbl2v ra2 = dbl2v{0.0, 0.0};                    // OUT: r_a of plane s-2 (line J2)
  dbl2v l2p = dbl2v{0.0, 0.0};                    // OUT: r_c of plane s-3
  dbl2v yc1 = dbl2v{0.0, 0.0};                    // OUT: y_c of plane s-3
  dbl2v p3 = dbl2v{0.0, 0.0};                     // OUT: partial head sums of plane s-3
#pragma unroll
  for (int i = 0; i < N1; ++i) p1[i] = l0p[i] = dbl2v{0.0, 0.0};
  const int tl = 2 + 2 * t;

  auto step = [&](int s) {
    // (1) level 0 of plane s to LDS; keep y_a (s-1), z_a and x (s-2); next loads
#pragma unroll
    for (int i = 0; i < 2; ++i) lds2_st(&L.x0[2 * G + i][tl], st[i]);
    dbl2v ya[N1];
#pragma unroll
    for (int i = 0; i < N1; ++i) ya[i] = sty[i];
    // OUT: z_a and x of plane s-2, loaded in this step (used after two
    // barriers): one step ahead they held 8 more registers across the loop
    dbl2v za = dbl2v{0.0, 0.0}, xa = dbl2v{0.0, 0.0};
    if constexpr (OUT) {
      const int zz = (unsigned)(s - 2) < (unsigned)planes ? s - 2 : 0;  // past a face: unused
      za = *reinterpret_cast<const dbl2v*>(a.u2 + orow + (int64_t)zz * W);
      if constexpr (XM != 0) xa = *reinterpret_cast<const dbl2v*>(a.us + orow + (int64_t)zz * W);
    }
    issue(s + 1);
    __syncthreads();
    // (2) level 1 at plane s-1: Ar1 completed by its +W term, y_b, r_b; plane
    // s's sums started
    const bool pok1 = (unsigned)(s - 1) < (unsigned)planes;
    dbl2v yb[N1], rb[N1];
    const dbl2v ra_now = l0p[I2];  // r_a of plane s-1 at line J2
#pragma unroll
    for (int i = 0; i < N1; ++i) {
      const int j = J1 + i;
      const double* line = &L.x0[j][tl];
      const dbl2v own = lds2(line);
      const dbl2v ar = dbl2v{p1[i].x + v[6] * own.x, p1[i].y + v[6] * own.y};
      const double t1l = e1 * ya[i].x, t1h = e1 * ya[i].y;
      const double t2l = f1 * ar.x, t2h = f1 * ar.y;
      yb[i] = dbl2v{t1l + t2l, t1h + t2h};
      rb[i] = dbl2v{l0p[i].x - yb[i].x, l0p[i].y - yb[i].y};
      if (!(pok1 && l1ok[i])) rb[i] = dbl2v{0.0, 0.0};  // off the box: the absent operand
      double m1, q2;
      st2b_nbrs<(KR_STEP_DPP & 4) != 0>(&L.x0[j][2], t, wig, own, m1, q2);
      p1[i] = st2b_part(v, l0p[i], lds2(&L.x0[j - 1][tl]), m1, own, q2, lds2(&L.x0[j + 1][tl]));
      l0p[i] = own;
      lds2_st(&L.x1[j - 1][tl], rb[i]);
    }
    __syncthreads();
    // (3) level 2 at plane s-2 (Ar1' completed by r_b of plane s-1): y_c, r_c
    // (and OUT: z_c, x, the stores); plane s-1's sums started
    const bool pok2 = (unsigned)(s - 2) < (unsigned)planes;
    const dbl2v rbo = rb[I2];
    const dbl2v ar2 = dbl2v{p2.x + v[6] * rbo.x, p2.y + v[6] * rbo.y};
    const double s1l = e2 * yb2.x, s1h = e2 * yb2.y;
    const double s2l = f2 * ar2.x, s2h = f2 * ar2.y;
    const dbl2v yc = dbl2v{s1l + s2l, s1h + s2h};
    dbl2v rc = dbl2v{l1p.x - yc.x, l1p.y - yc.y};
    if constexpr (OUT) {
      if (s - 2 >= z0 && s - 2 < z1) {
        // step j: z_b = eta_j z_a - zeta_j r_a; x2: x - z_a, then - z_b
        const double t3l = e1 * za.x, t3h = e1 * za.y;
        const double t4l = f1 * ra2.x, t4h = f1 * ra2.y;
        const dbl2v zb = dbl2v{t3l - t4l, t3h - t4h};
        dbl2v xn = xa;
        if constexpr (XM & 1) xn = dbl2v{xn.x - za.x, xn.y - za.y};
        if constexpr (XM & 2) xn = dbl2v{xn.x - zb.x, xn.y - zb.y};
        const double s3l = e2 * zb.x, s3h = e2 * zb.y;
        const double s4l = f2 * l1p.x, s4h = f2 * l1p.y;
        const dbl2v zc = dbl2v{s3l - s4l, s3h - s4h};
        if constexpr (XM & 4) xn = dbl2v{xn.x - zc.x, xn.y - zc.y};
        const int64_t row = orow + (int64_t)(s - 2) * W;
        __builtin_nontemporal_store(yc, reinterpret_cast<dbl2v*>(a.u1 + row));
        __builtin_nontemporal_store(zc, reinterpret_cast<dbl2v*>(a.u2 + row));
        if constexpr (XM != 0) __builtin_nontemporal_store(xn, reinterpret_cast<dbl2v*>(a.ud + row));
        __builtin_nontemporal_store(rc, reinterpret_cast<dbl2v*>(a.y1 + row));
      }
      ra2 = ra_now;
    }
    if (!(pok2 && l2ok)) rc = dbl2v{0.0, 0.0};  // off the box: the head's absent operand
    {
      double n1, n2;
      st2b_nbrs<(KR_STEP_DPP & 8) != 0>(&L.x1[J2 - 1][2], t, wig, rbo, n1, n2);
      p2 = st2b_part(v, l1p, lds2(&L.x1[J2 - 2][tl]), n1, rbo, n2, lds2(&L.x1[J2][tl]));
    }
    l1p = rbo;
    yb2 = yb[I2];
    lds2_st(&L.x2[J2 - 2][tl], rc);
    __syncthreads();
    // (4) level 3 (the head) at plane s-3: Ar1 completed by r_c of plane s-2,
    // products, the store; plane s-2's sums started
    if constexpr (OUT) {
      const dbl2v ar3 = dbl2v{p3.x + v[6] * rc.x, p3.y + v[6] * rc.y};
      const int zh = s - 3;
      if (zh >= z0 && zh < z1) {
        if (zh >= nb) {
          flush();
          ++seg;
          nb = (int)((int64_t)planes * (seg + 1) / Zh);
        }
        epi_products<EPI_HEAD_MRR>(l2p.x, 0.0, ar3.x, 0.0, yc1.x, acc);
        epi_products<EPI_HEAD_MRR>(l2p.y, 0.0, ar3.y, 0.0, yc1.y, acc);
        __builtin_nontemporal_store(ar3, reinterpret_cast<dbl2v*>(a.y2 + orow + (int64_t)zh * W));
      }
      double n1, n2;
      st2b_nbrs<(KR_STEP_DPP & 16) != 0>(&L.x2[J2 - 2][2], t, wig, rc, n1, n2);
      p3 = st2b_part(v, l2p, lds2(&L.x2[J2 - 3][tl]), n1, rc, n2, lds2(&L.x2[J2 - 1][tl]));
      l2p = rc;
      yc1 = yc;
    }
  };

  // prologue: level 0 of plane z0-3 (the -W operand of plane z0-2's level 1),
  // plane z0-2 in flight; the LDS lines are overwritten by the first step
  // before any read
  issue(z0 - 3);
#pragma unroll
  for (int i = 0; i < 2; ++i) lds2_st(&L.x0[2 * G + i][tl], st[i]);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N1; ++i) l0p[i] = lds2(&L.x0[J1 + i][tl]);
  __syncthreads();
  issue(z0 - 2);
  for (int s = z0 - 2; s <= z1 + 2; ++s) step(s);
  if constexpr (OUT) flush();
}

template <int XM>
__global__ __launch_bounds__(4 * kBlock) __attribute__((amdgpu_waves_per_eu(4)))
void spmv_step2h_kernel(SpmvArgs a) {
  if (a.stop && *a.stop != 0.0) return;
  extern __shared__ __attribute__((aligned(16))) double sp3_dyn[];
  Sp3Lds& L = *reinterpret_cast<Sp3Lds*>(sp3_dyn);
  // the x-face pads of every line (rows -2, -1, 512, 513), read as 0.0;
  // visible after the prologue's barrier, never written again
  if (threadIdx.x < 72) {
    const int i = threadIdx.x >> 2, e = threadIdx.x & 3;  // line i of 18, pad e
    double* line = i < 8 ? &L.x0[i][0] : i < 14 ? &L.x1[i - 8][0] : &L.x2[i - 14][0];
    line[e < 2 ? e : kSBlock + e] = 0.0;
  }
  const int P = a.st_P, PP = P >> 3;
  const int B = blockIdx.x, q = B & 7, w2 = B >> 3;
  const int half = PP >> 1, Zw = gridDim.x / (P >> 1);
  const int p0 = q * PP + 2 * (w2 % half);
  const int zs = w2 / half;
  const int g = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kBlock));
  const int t = (int)(threadIdx.x % kBlock);
  switch (g) {
    case 0: sp3_walk<0, XM>(a, L, t, p0, q, zs, Zw); break;
    case 1: sp3_walk<1, XM>(a, L, t, p0, q, zs, Zw); break;
    case 2: sp3_walk<2, XM>(a, L, t, p0, q, zs, Zw); break;
    default: sp3_walk<3, XM>(a, L, t, p0, q, zs, Zw); break;
  }
}

// partials[kk * grid + v] = ((q0 + q1) + q2) + q3 over the four x quarters of
// the head launch's workgroup v (block_reduce_store's order), kk < nk, v < n.
__global__ __launch_bounds__(kBlock) void sp3_combine_kernel(const double* __restrict__ partq,
                                                              double* __restrict__ partials,
                                                              int grid, int nk, int n) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int kk = (int)(i / grid), v = (int)(i % grid);
  if (kk >= nk || v >= n) return;
  const dbl2v lo = *reinterpret_cast<const dbl2v*>(partq + ((int64_t)kk * grid + v) * 4);
  const dbl2v hi = *reinterpret_cast<const dbl2v*>(partq + ((int64_t)kk * grid + v) * 4 + 2);
  double s = lo.x;
  s = s + lo.y;
  s = s + hi.x;
  s = s + hi.y;
  partials[(int64_t)kk * grid + v] = s;
}

template <int XM>
void sp3_launch_t(const SpmvArgs& a, int nblocks, hipStream_t s) {
  static std::atomic<uint64_t> opted{0};
  opt_in_lds(opted, reinterpret_cast<const void*>(spmv_step2h_kernel<XM>), sizeof(Sp3Lds));
  spmv_step2h_kernel<XM><<<nblocks, 4 * kBlock, sizeof(Sp3Lds), s>>>(a);
  KR_HIP_CHECK(hipGetLastError());
}

}  // namespace

// x segments per line (KR_ST2B_XS for the storing pair, KR_ST2B_XS_PO for
// the products-only one: 1, 2 or 4). Measured on C4: first (one box, twice,
// profiles/r06x) storing pair 1.29 / 1.28 / 1.32 ms at 4 / 2 / 1 segments,
// products-only pair 1.26 / 1.24 / 1.13 ms; once whole-line walks stopped
// issuing the x-halo loads they never need (profiles/r06c, r06h, same box,
// twice each) the storing pair runs 1.334-1.361 ms at 1 segment against
// 1.428-1.452 at 4 (C4 826-827 -> 842-845 it/s): whole lines for both.
int st2b_xsegments(bool products_only) {
  const int x = products_only ? KR_ENV("KR_ST2B_XS_PO", 1) : KR_ENV("KR_ST2B_XS", 1);
  return x == 1 || x == 2 ? x : 4;
}

void launch_spmv_stencil2b(SpmvEpi epi, const SpmvArgs& a, int nblocks, int xs, int n1, int n2,
                           hipStream_t s) {
  const int64_t W = (int64_t)a.st_P * kSBlock;
  const int64_t planes = a.st_P > 0 ? a.n / W : 0;
  const int tiles = a.st_P / 2;
  const int zw = tiles > 0 && xs > 0 ? nblocks / (tiles * xs) : 0;
  KR_REQUIRE(a.st_box && a.st_P % 16 == 0 && a.n == planes * W && planes >= 1 && a.rb_gap == 0 &&
                 a.partials && a.partq && a.st2_z1 > 0 && a.st2_z2 > 0 &&
                 (xs == 1 || xs == 2 || xs == 4) && zw > 0 && nblocks == tiles * xs * zw &&
                 a.st2_z1 % zw == 0 && a.st2_z2 % zw == 0 && planes >= a.st2_z1 &&
                 planes >= a.st2_z2 && n1 == a.st_P * a.st2_z1 && n2 == a.st_P * a.st2_z2 &&
                 n1 <= a.grid && n2 <= a.grid && (a.xlen + W) * 8 < (int64_t(1) << 31),
             "box fused basis pair: constant-coefficient 7-point box with n = 512, P % 16 == 0, "
             "whole planes, a walk grid dividing both dual grids");
  if (epi == EPI_DUAL_MRR)
    st2b_launch_e<EPI_DUAL_MRR>(a, nblocks, xs, s);
  else if (epi == EPI_DUAL_KCG)
    st2b_launch_e<EPI_DUAL_KCG>(a, nblocks, xs, s);
  else
    throw Failure(KR_ERR_INVALID, "box fused basis pair: EPI_DUAL_MRR or EPI_DUAL_KCG");
  const int64_t total = (int64_t)14 * a.grid;
  st2b_combine_kernel<<<(int)((total + kBlock - 1) / kBlock), kBlock, 0, s>>>(a.partq, a.partials,
                                                                               a.grid, n1, n2);
  KR_HIP_CHECK(hipGetLastError());
}

void launch_spmv_step2b(const SpmvArgs& a, int nblocks, int virt, int xm, hipStream_t s) {
  const int64_t W = (int64_t)a.st_P * kSBlock;
  const int64_t planes = a.st_P > 0 ? a.n / W : 0;
  const int tiles = a.st_P / 2;
  KR_REQUIRE(a.st_box && a.st_P % 16 == 0 && a.n == planes * W && planes >= 1 && a.rb_gap == 0 &&
                 tiles > 0 && nblocks % tiles == 0 && nblocks / tiles <= planes && a.x1 &&
                 a.x2 && (!virt || a.x3) && a.u1 && a.u2 && a.y1 && (xm == 0 || (a.us && a.ud)) &&
                 (!virt || (a.us && a.ud)) && a.u1 != a.x2 + a.xoff && a.y1 != a.x1 + a.xoff &&
                 (a.xlen + W) * 8 < (int64_t(1) << 31),
             "box step pair: constant-coefficient 7-point box with n = 512, P % 16 == 0, "
             "whole planes; y and r written to other buffers than they are read from");
  if (virt) {
    KR_REQUIRE(xm == 0 || xm == 4, "box step triple: x minus z_3 or nothing more");
    if (xm == 4)
      sp2b_launch_t<true, 4>(a, nblocks, s);
    else
      sp2b_launch_t<true, 0>(a, nblocks, s);
    return;
  }
  switch (xm) {
    case 6: sp2b_launch_t<false, 6>(a, nblocks, s); return;  // (nox, x2)
    case 3: sp2b_launch_t<false, 3>(a, nblocks, s); return;  // (x2, nox)
    case 7: sp2b_launch_t<false, 7>(a, nblocks, s); return;  // (x2, x)
    default: throw Failure(KR_ERR_INVALID, "box step pair: unsupported step kinds");
  }
}

void launch_spmv_step2h(const SpmvArgs& a, int nblocks, int xm, int nhead, hipStream_t s) {
  const int64_t W = (int64_t)a.st_P * kSBlock;
  const int64_t planes = a.st_P > 0 ? a.n / W : 0;
  const int tiles = a.st_P / 2;
  const int zw = tiles > 0 ? nblocks / tiles : 0;
  KR_REQUIRE(a.st_box && a.st_P % 16 == 0 && a.n == planes * W && planes >= 1 && a.rb_gap == 0 &&
                 zw > 0 && nblocks == tiles * zw && zw <= planes && a.st2_z1 > 0 &&
                 a.st2_z1 % zw == 0 && planes >= a.st2_z1 && nhead == a.st_P * a.st2_z1 &&
                 nhead <= a.grid && a.partq && a.partials && a.x1 && a.x2 && a.u1 && a.u2 &&
                 a.y1 && a.y2 && (xm == 0 || (a.us && a.ud)) && a.u1 != a.x2 + a.xoff &&
                 a.y1 != a.x1 + a.xoff && (a.xlen + W) * 8 < (int64_t(1) << 31),
             "box step pair + head: constant-coefficient 7-point box with n = 512, P % 16 == 0, "
             "whole planes, walk segments dividing the head grid's; y and r written to other "
             "buffers than they are read from");
  switch (xm) {
    case 3: sp3_launch_t<3>(a, nblocks, s); break;  // (x2, nox)
    case 7: sp3_launch_t<7>(a, nblocks, s); break;  // (x2, x)
    case 6: sp3_launch_t<6>(a, nblocks, s); break;  // (nox, x2)
    default: throw Failure(KR_ERR_INVALID, "box step pair + head: unsupported step kinds");
  }
  const int64_t total = (int64_t)5 * a.grid;
  sp3_combine_kernel<<<(int)((total + kBlock - 1) / kBlock), kBlock, 0, s>>>(a.partq, a.partials,
                                                                             a.grid, 5, nhead);
  KR_HIP_CHECK(hipGetLastError());
}

}  // namespace kr
