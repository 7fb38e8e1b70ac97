// Internal declarations shared by the HIP kernels and the host engine.
// Nothing in here crosses the C ABI (include/krylov_amd.h is the boundary).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "../../include/krylov_amd.h"

namespace kr {

// Rows per row-block == threads per block: one lane owns one row so every
// row is summed sequentially in stored order (scipy csr_matvec order).
constexpr int kBlock = 256;
// Matrix entries staged in LDS per window (vals 16 KiB + cols 8 KiB).
constexpr int kWindow = 2048;
// Upper bound on fused reduction products in one kernel.
constexpr int kMaxProducts = 8;

struct Failure : std::runtime_error {
  int code;
  Failure(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define KR_HIP_CHECK(expr)                                                        \
  do {                                                                            \
    hipError_t kr_e_ = (expr);                                                    \
    if (kr_e_ != hipSuccess)                                                      \
      throw ::kr::Failure(KR_ERR_HIP, std::string(#expr) + " -> " +               \
                                          hipGetErrorString(kr_e_) + " at " +     \
                                          __FILE__ ":" + std::to_string(__LINE__)); \
  } while (0)

#define KR_REQUIRE(cond, msg)                                        \
  do {                                                               \
    if (!(cond)) throw ::kr::Failure(KR_ERR_INVALID, std::string(msg)); \
  } while (0)

// Dynamic LDS above 64 KiB is opted into per kernel AND per device
// (hipFuncSetAttribute acts on the calling thread's current device). `done`
// holds one bit per device; the per-shard host threads may race here, which
// only repeats an idempotent attribute call.
inline void opt_in_lds(std::atomic<uint64_t>& done, const void* fn, size_t lds) {
  int dev = 0;
  KR_HIP_CHECK(hipGetDevice(&dev));
  const uint64_t bit = uint64_t(1) << (dev & 63);
  if (done.load(std::memory_order_acquire) & bit) return;
  KR_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  done.fetch_or(bit, std::memory_order_acq_rel);
}

// Environment knobs (KR_* A/B switches) on the launch path, read through a
// cache: the hot path reads several per kernel launch, and getenv walks the
// whole environment each time. A cached value is refreshed once g_env_epoch
// moved, which every C-ABI entry point except kr_solve_step does -- so a
// knob changed between two calls (as the tests do) takes effect at the next
// call, and one solve's steps see the values of its kr_solve_begin.
extern std::atomic<uint64_t> g_env_epoch;
// cache word: tag << 33 | set << 32 | uint32 value; 0 = empty. The tag is
// the epoch folded into [1, 2^31 - 1] (31 bits above bit 33; never 0, so an
// empty word never matches), so it keeps matching after 2^31 epochs.
inline int env_cached(std::atomic<uint64_t>& cache, const char* name, int dflt) {
  const uint64_t ep = 1 + g_env_epoch.load(std::memory_order_relaxed) % ((1ull << 31) - 1);
  const uint64_t c = cache.load(std::memory_order_relaxed);
  if ((c >> 33) == ep) return ((c >> 32) & 1) ? (int)(uint32_t)c : dflt;
  const char* e = getenv(name);
  const int v = e ? atoi(e) : 0;
  cache.store((ep << 33) | ((uint64_t)(e != nullptr) << 32) | (uint32_t)v,
              std::memory_order_relaxed);
  return e ? v : dflt;
}
// KR_ENV("KR_X", d): the knob's integer value, d when unset (one cache per use)
#define KR_ENV(name, dflt)                                     \
  ([]() -> int {                                               \
    static std::atomic<uint64_t> kr_env_cache_{0};             \
    return ::kr::env_cached(kr_env_cache_, (name), (dflt));    \
  }())

// KR_POISON_ALLOC=1 (debug): every device buffer the engine allocates starts
// as all-ones bytes (a NaN in every double) instead of zeros or whatever
// hipMalloc left, so a read of memory nothing wrote shows up as NaN on the
// first run. Buffers whose zeros are part of their meaning (DIA slots of
// absent entries, code padding, counters) keep their explicit zero fill.
bool poison_alloc();
// The fill a fresh buffer gets: 0xFF bytes under KR_POISON_ALLOC, else
// `dflt` (0 for buffers the engine zeroes, -1: left as allocated).
void fresh_fill(void* p, size_t bytes, hipStream_t s, int dflt = -1);

// ---------------------------------------------------------------------------
// SpMV with fused epilogue reductions.
// Operand names used by the product tables (per own row r):
//   X1, X2 : the SpMV inputs at row r      Y1, Y2 : the SpMV results at row r
//   E      : an extra vector at row r (own-row indexing)
// ---------------------------------------------------------------------------
enum SpmvEpi : int {
  EPI_NONE = 0,   // y = A x
  EPI_BMINUS,     // y = b - A x ; <y,y>
  EPI_XY,         // <x,x> <x,y> <y,y>
  EPI_HEAD_MRR,   // <x,x> <x,y> <y,y> <e,y> <e,e>       (x=Ar0 y=Ar1 e=Ay0)
  EPI_HEAD_KCG,   // <e,e> <x,x> <x,y> <y,y> <e,x> <e,y> (x=Ap0 y=Ap1 e=Ar0)
  EPI_MRR_LOOP,   // <x,x> <e,e> <e,y>                   (x=r  y=Ar  e=y)
  EPI_DUAL_NONE,  // y1 = A x1, y2 = A x2
  EPI_DUAL_MRR,   // 7 products, see kernels
  EPI_DUAL_KCG,   // 7 products, see kernels
  // Fused k-skip inner steps: y = A x is consumed in the epilogue by the
  // NEXT vector step (its scalars are known from the Gram sync), and only the
  // step's outputs are stored. y1 receives the step's new input vector (a
  // different buffer than x1: other rows still gather x1).
  EPI_STEP_MRR_NOX,  // t=Ax; u1=c0*u1+c1*t; u2=c0*u2-c1*x; y1=x-u1          (u1=Ay0 u2=z)
  EPI_STEP_MRR_X2,   //   ... and ud = (us - u2_old) - u2_new (deferred x -= z, two steps)
  EPI_STEP_MRR_X,    //   ... and ud = us - u2_new
  EPI_STEP_KCG,      // t=Ax; u1+=c0*x; u2-=c0*t; y1=u2+c1*x                 (u1=x u2=Ar0, x=Ap0)
  // Steps 0 AND 1 of a k-skip MrR outer iteration in one SpMV: the input
  // r1 = r0 - (c0*y0 + c1*Ar1) is formed at every gathered column from x1=r0,
  // x2=y0, x3=Ar1 (exactly as the step-0 vector kernel rounds it), then step 1
  // (c2, c3) runs in the epilogue: u1 (y) and y1 (r) are written to buffers
  // other than x2 / x1, which other rows still gather. Row walk v2 only.
  EPI_STEP_MRR_FIRST2,
  // CG with device-resident scalars on one shard: the SpMV runs the
  // SC_CG_BETA scalar step itself (SpmvArgs::pro: beta = gnew / gamma, the
  // convergence test) and multiplies the virtual p = r + beta * p_old,
  // formed at every gathered column from x1 = p_old, x2 = r exactly as
  // ew_kernel<EW_CG_P> rounds it; the own rows' p is stored to u1 (a
  // different buffer than x1: other rows still gather p_old), y1 = A p,
  // products <p,p> <p,y> <y,y> as EPI_XY. Replaces EW_CG_P + EPI_XY.
  EPI_XY_VP,
  // MrR with device-resident scalars on one shard: the previous iteration's
  // vector step runs inside this SpMV. Its SC_MRR_ZETA scalar step is the
  // prologue (c0 = eta, c1 = zeta), the input r_new = r - (eta*y + zeta*Ar)
  // is formed at every gathered column from x1 = r, x2 = y, x3 = Ar (the
  // EW_MRR rounding), the own rows store u1 = y_new, u2 = z_new (in place),
  // ud = x - z_new, y2 = r_new, y1 = A r_new, and the products are
  // EPI_MRR_LOOP's (<r,r> mu nu of the new vectors). Replaces EW_MRR + EPI_MRR_LOOP.
  EPI_MRR_V,
};
int spmv_products(SpmvEpi epi);

struct SpmvArgs {
  const void* rowptr = nullptr;
  int rowptr64 = 0;
  const int32_t* col = nullptr;
  const double* val = nullptr;
  int64_t n = 0;               // rows
  const double* x1 = nullptr;  // indexed by col (halo-extended vector base)
  const double* x2 = nullptr;
  int64_t xoff = 0;            // own row 0 sits at x[xoff]
  double* y1 = nullptr;        // own rows
  double* y2 = nullptr;
  const double* b = nullptr;   // own rows (EPI_BMINUS)
  const double* e = nullptr;   // own rows (extra operand)
  double* partials = nullptr;  // products: partials[p * grid + block]
  int grid = 0;
  int long_rows = 0;           // 1: product-then-sum kernel (mean nnz/row >= kLongRow)
  int accumulate = 0;          // 1: add products to the partials (split SpMV, 2nd+ launch)
  int64_t slab = 0;            // >= 8: slab row-block schedule, S row blocks per plane
  int64_t slab_sub = 0;        // sub-slab width in row blocks (0: one eighth of a plane)
  // Offset masks (optional, short-row kernel): row i's columns are
  // xoff + i + moff[b] for the set bits b of mask[i] (mw bits), in order;
  // col is then not read.
  const void* mask = nullptr;
  const int32_t* moff = nullptr;
  int nm = 0;
  int mw = 0;
  // Diagonal-offset values (optional, with the masks): entry of row i at
  // offset moff[b] is dia[(i / 256) * dia_bs + b * dia_ks + i % 256]
  // (row-block launches offset dia by their first row block). Offset-major:
  // dia_bs = 256, dia_ks = ld; row-block-major (default): dia_bs = 256 * nm,
  // dia_ks = 256. The SpMV then needs neither LDS staging nor rowptr.
  const double* dia = nullptr;
  int64_t dia_bs = 0, dia_ks = 0;
  // Symmetric values (System::build_masks checked A[i][i-o] == A[i-o][i]
  // bitwise for every stored lower entry): a lower entry is read as its
  // mirrored upper entry of row i - o, which the workgroup of that row block
  // streams at the same time (an L2 hit), instead of its own copy (HBM).
  int dia_sym = 0;
  // 1: the row-block walk with the mirrors and an x ring in LDS
  // (spmv_diawalk_kernel; symmetric shards with a band <= 256 rows). The
  // grid (the launch's block count) fixes each workgroup's run of blocks.
  int dia_walk = 0;
  // The walk's run of whole, full row blocks [full_lo, full_hi) (launch-
  // relative): their masks are all-ones and are not loaded. Empty by default.
  int64_t full_lo = 0, full_hi = 0;
  // x window in LDS (spmv_dia_kernel): nseg segments, segment g = rows
  // row0 + seg_lo[g] .. + seg_len[g] - 1 of the row block at s_xw[seg_base[g]]
  // (starts and lengths even), dia_wlen doubles in all (0: gathers from global
  // memory); offset k of row lr of the block is s_xw[lr + woff[k]]. xlen = the
  // doubles of the halo-extended vectors (window loads clamp to it).
  static constexpr int kMaxSeg = 4;
  int dia_wlen = 0, nseg = 0;
  int seg_lo[kMaxSeg] = {}, seg_len[kMaxSeg] = {}, seg_base[kMaxSeg] = {};
  const int32_t* woff = nullptr;
  int64_t xlen = 0;
  // Fused-step operands (EPI_STEP_*), own rows: in/out u1, u2, x source/dest.
  double* u1 = nullptr;
  double* u2 = nullptr;
  const double* us = nullptr;
  double* ud = nullptr;
  double c0 = 0, c1 = 0;
  const double* x3 = nullptr;  // EPI_STEP_MRR_FIRST2: Ar1 (halo-extended)
  const double* stop = nullptr;  // skip the launch when *stop != 0 (EwArgs::stop)
  double c2 = 0, c3 = 0;       // EPI_STEP_MRR_FIRST2: step-1 scalars (eta1, zeta1)
  double c4 = 0, c5 = 0;       // the box step triple (launch_spmv_step2b virt): step 2's
  // EPI_STEP_MRR_FIRST2: the previous outer iteration's last x -= z is still
  // pending (its z is this launch's z input u2): x = ((x - z0) - z1) - z2
  int xpend = 0;
  int epi_late = 0;  // 1: load own-row epilogue operands at the row end (A/B, KR_EPI_LATE)
  // 1: the caller needs only the products (the last basis SpMV of a k-skip
  // outer iteration): a kernel MAY skip storing y1/y2 (the stencil walk does)
  int products_only = 0;
  // the fused basis pair (launch_spmv_stencil2): products of the second dual
  double* partials2 = nullptr;
  int64_t nnz_total = -1;  // entries of val/col (-1: unknown; spmv_kernel2 needs >= 4)
  // 1: the short-row row walk runs its non-temporal variant (matrix stream
  // and result stores; System::spmv sets it for shards >= 4M rows, whose
  // outputs outlive the caches anyway; KR_NT_STORES=0/1 forces it; the
  // stencil walk has its own NTM bit)
  int nt_stores = 0;
  // Dense row block (gemv_kernel): val is n x ncols row-major with leading
  // dimension dld; x1 + xcol0 (x2 + xcol0) is the full input vector.
  int dense = 0;
  int64_t dld = 0, ncols = 0, xcol0 = 0;
  // Row-block gap (boundary launch of a split SpMV): the launch covers the
  // row blocks [0, rb_gap_at) and [rb_gap_at + rb_gap, ceil(n / kBlock)).
  int64_t rb_gap_at = 0, rb_gap = 0;
  // Value dictionary (optional, row walk v2): entry j's value is
  // vtab[vcode[j]] (same index space as val; val stays valid for the other
  // kernels). vtab holds <= kVdMax doubles.
  const uint8_t* vcode = nullptr;
  const double* vtab = nullptr;
  int ntab = 0;
  // Stencil codes (kr_stencil.h; optional, with vtab): scode[i] = the codes
  // of row i's entries, byte k for offset st_off[k] (ascending), 0xFF = no
  // entry. Rows are walked in 512-row blocks, st_P blocks per walk step
  // (W = 512 * st_P rows = the +-W offsets); st_kind[k] = StencilKind of
  // slot k; st_far[f] = the FAR offsets. Launch grids are multiples of
  // 8 * st_P; rowptr, col, val, mask, vcode are not read. st_cb: bits per
  // slot code (8: uint64 per row, 0xFF = no entry; 4: uint32 per row, 0xF;
  // 2: uint16 per row, 0x3 -- narrow codes for dictionaries of <= 15 / <= 3
  // values), so a row streams st_cb bytes of A.
  const void* scode = nullptr;
  int st_cb = 8;
  // Code patterns (optional, with scode): the codes of row block b (512 rows,
  // 512 * st_cb bytes) are pattern st_pid[b] of the table st_pat (st_npat
  // patterns, row blocks past n zero-padded) -- a constant-coefficient
  // stencil on a box has a handful of distinct blocks (interior, faces,
  // edges), so the walk reads its codes from L2 instead of streaming st_cb
  // bytes per row. Same codes, same arithmetic. scode stays valid.
  const uint32_t* st_pid = nullptr;
  const void* st_pat = nullptr;
  int st_npat = 0;
  int st_P = 0, st_nm = 0, st_nfar = 0;
  // 1: position-major walk (st_P % 8 == 0): XCD q takes positions
  // [q P/8, (q+1) P/8) of every plane segment; grid = P x segments.
  // 0: plane-major: XCD q takes an eighth of the planes at every position;
  // grid = 8 P x segments. See kr_stencil.h.
  int st_pm = 0;
  // 1: dispatch order reversed -- workgroup b runs the walk of workgroup
  // grid - 1 - b (same visits, same partials), so the top plane segments go
  // first. The engine alternates it per launch with KR_ZIGZAG=1 (A/B): the
  // next kernel starts on the planes the previous one touched last.
  int st_rev = 0;
  // The tiled fused basis pair (spmv_stencil2t_kernel): plane segments of the
  // two dual grids whose partials it writes (level 1 = dual m, level 2 = dual
  // m+1: general grid, or the products-only grid), the walk runs on their gcd
  int st2_z1 = 0, st2_z2 = 0;
  // The box pair (kr_pair.hip, spmv_stencil2b_kernel): 1 when the shard is a
  // constant-coefficient 7-point box stencil with n = 512 (Shard::st_box);
  // st_v[k] = the value of every entry of slot k (offset st_off[k]).
  int st_box = 0;
  double st_v[8] = {};
  // ... its products: [14 slots][grid][4 x quarters], combined into partials
  // (slot kk at partials + kk * grid) by st2b_combine_kernel
  double* partq = nullptr;
  int32_t st_off[8] = {};
  int32_t st_kind[8] = {};
  int32_t st_far[4] = {};
  double* scratch = nullptr;  // >= 2 doubles, 16-byte aligned: stores of lanes past the last row
  // Fused scalar step (EPI_XY_VP; the fields of EwArgs::pro): every
  // workgroup first runs scalar statement pro - 1 from the reduction
  // partials pro_part[q * pro_stride + 0 .. pro_cnt[q]) and takes c0 from it.
  int pro = 0;
  const double* pro_part = nullptr;
  int pro_stride = 0;
  int pro_cnt[5] = {};
  double* st = nullptr;
  int64_t pro_it = 0;
  int pro_h = 0;
  int pro_par = 0;
  int pro_check = 1;
  double pro_thr = 0;
  int pro_s1 = 1;
};
// Rows per row block of the stencil SpMV (2 per lane; kr_stencil.h).
constexpr int kStencilBlock = 2 * kBlock;
// Stencil codes of a masked CSR block (kr_stencil.h): out[i] = byte k =
// vcode[j] of row i's entry at offset M[k] (local columns: base + i + M[k]),
// 0xFF where row i has none. nm <= 8.
void launch_stencil_codes(const void* rowptr, int rowptr64, int64_t n, const int32_t* col,
                          const uint8_t* vcode, int64_t base, const int32_t* M, int nm,
                          uint64_t* out, hipStream_t s);
// Narrow stencil codes: out (uint16 per row for cb = 2, uint32 for cb = 4)
// slot k = bits [cb k, cb k + cb) = byte k of in[i], all ones where byte k is
// 0xFF (no entry). Every present code must be < 2^cb - 1.
void launch_stencil_pack(const uint64_t* in, int64_t n, int cb, void* out, hipStream_t s);
// Mean row length from which the product-then-sum SpMV is used.
constexpr double kLongRow = 12.0;
void launch_spmv(SpmvEpi epi, const SpmvArgs& a, hipStream_t s);
// Same with gridDim = nblocks (<= a.grid, the partial stride).
void launch_spmv_grid(SpmvEpi epi, const SpmvArgs& a, int nblocks, hipStream_t s);
// Two chained k-skip MrR basis SpMVs in one walk (kr_stencil.h
// spmv_stencil2_kernel): x1, x2 = (Ar[m+1], Ay[m]) -> y1, y2 = (Ar[m+3],
// Ay[m+2]) (not stored when products_only), EPI_DUAL_MRR products of dual m
// at partials, of dual m+1 at partials2. 7-point stencil shards with n = 512.
void launch_spmv_stencil2(const SpmvArgs& a, int nblocks, hipStream_t s);
// The tiled pair (spmv_stencil2t_kernel): two adjacent positions per
// 512-thread workgroup, bitwise the two dual launches (products included);
// EPI_DUAL_MRR or EPI_DUAL_KCG products; nblocks = P/2 x gcd(st2_z1, st2_z2).
void launch_spmv_stencil2t(SpmvEpi epi, const SpmvArgs& a, int nblocks, hipStream_t s);
void launch_spmv_stencil2t_mrr(const SpmvArgs& a, int nblocks, hipStream_t s);
void launch_spmv_stencil2t_kcg(const SpmvArgs& a, int nblocks, hipStream_t s);
// The box pair (kr_pair.hip): the tiled pair's job and products for a
// constant-coefficient 7-point box stencil (SpmvArgs::st_box), the matrix not
// read; nblocks = P/2 tiles x xs x-segments x walk segments; its products
// go through SpmvArgs::partq into the n1 / n2 partials of the two dual grids,
// bitwise the dual launches'.
void launch_spmv_stencil2b(SpmvEpi epi, const SpmvArgs& a, int nblocks, int xs, int n1, int n2,
                           hipStream_t s);
// The box step pair (kr_pair.hip): k-skip MrR steps j and j+1 in one walk on
// a box shard: x1 = r_a (gathered), x2 = y_a (gathered), y1 = r_c, u1 = y_c
// (other buffers), u2 = z (in place), us / ud = x source / destination, c0
// c1 / c2 c3 = the steps' (eta, zeta); xm bits: x minus z_a (step j an x2
// step), z_b, z_c -- 6 (nox, x2), 3 (x2, nox), 7 (x2, x). virt: steps 0, 1,
// 2 (FIRST2 + the next): x3 = Ar1_0, c4 c5 step 2's, xpend, xm 0 or 4 (x minus
// z_3). nblocks = P/2 x walk segments. Bitwise the step launches.
void launch_spmv_step2b(const SpmvArgs& a, int nblocks, int virt, int xm, hipStream_t s);
// The box step pair + head (kr_pair.hip): the last two k-skip MrR steps of
// an outer iteration (launch_spmv_step2b's operands, xm 3, 7 or 6) and the
// head SpMV of the next (y2 = Ar1 = A r_c; EPI_HEAD_MRR products of the head
// grid -- nhead = P x st2_z1 workgroups -- through partq into partials) in
// one walk; nblocks = P/2 x walk segments. Bitwise the step-pair launch
// followed by the head launch.
void launch_spmv_step2h(const SpmvArgs& a, int nblocks, int xm, int nhead, hipStream_t s);
// x segments per line of the box pair (1, 2 or 4; kr_pair.hip)
int st2b_xsegments(bool products_only);

// ---------------------------------------------------------------------------
// Elementwise vector steps with fused reductions (all own-row pointers).
// ---------------------------------------------------------------------------
enum EwOp : int {
  EW_DOT = 0,     // <u,v>                                   (p0 = u, p1 = v)
  EW_MRR_FIRST,   // y = zeta*ar1; z = (-zeta)*r; r -= y; xd = xs - z
  EW_MRR,         // y = eta*y + zeta*ar1; z = eta*z - zeta*r; r -= y; xd = xs - z
  EW_CG,          // x += alpha*p; r -= alpha*v; <r,r>
  EW_CG_P,        // p = r + beta*p
  EW_KCG,         // x += alpha*ap0; r -= alpha*ap1; ap0 = r + beta*ap0
  EW_MRR_S,       // s = ar - gamma*y; <r,s> <s,s>   (s not stored)
  EW_COPY,        // p0 <- p1
  EW_MRR_NOX,     // EW_MRR without the x update (x deferred to the next step)
  EW_MRR_X2,      // EW_MRR with xd = (xs - z_old) - z_new (two steps of x at once)
  // Preconditioned / pipelined CG family (v1/threads/pipeline/*.py, DESIGN.md
  // §5b); d = the Jacobi diagonal, M^-1 v = v / d.
  EW_ONE,         // p0 = 1.0 (identity preconditioner: d = 1, v / 1.0 == v)
  EW_PRE,         // u = r / d; <r,r> <r,u>                  (p: r u d)
  EW_PCG,         // x += a p; r -= a s; u = r / d; <r,r> <r,u>        (x p r s u d)
  EW_CGG,         // p = u + b p; s = w + b s; x += a p; r -= a s; u = r / d;
                  // <r,r> <r,u>                             (p u s w x r d)
  EW_GROPP1,      // x += a p; r -= a s; u -= a (s / d); <r,r> <r,u>  (x p r s u d)
  EW_GROPP2,      // p = u + b p; s = w + b s; <p,s>         (p u s w)
  EW_DIV,         // m = w / d                               (m w d)
  // Fused CG with the x update deferred to every second iteration (x is
  // never read inside the loop): (x p r v pp)
  EW_CG_NOX,      // r -= alpha*v; <r,r>                   (alpha saved to ST_ALPHA)
  EW_CG_X2,       // x = (x + alpha_prev*pp) + alpha*p; r -= alpha*v; <r,r>
  EW_AXPY,        // x += c0*p                              (the flush after a NOX step)
  EW_PIPE,        // z = n + b z; q = m + b q; s = w + b s; p = u + b p; x += a p;
                  // r -= a s; u -= a q; w -= a z; <r,r> <r,u> <w,u>
                  //                                         (z n q m s w p u x r)
};
// Operand slots of an elementwise op (EwArgs::p).
constexpr int kEwOps = 10;
int ew_products(EwOp op);

struct EwArgs {
  double c0 = 0, c1 = 0;           // scalars (eta/alpha/gamma, zeta/beta)
  double* p[kEwOps] = {};          // operand pointers, meaning per op
  int64_t n = 0;
  double* partials = nullptr;
  int grid = 0;                    // workgroups launched
  int stride = 0;                  // partial stride per slot (0: grid)
  const double* cdev = nullptr;    // device-resident c0, c1 (cdev[0], cdev[1]) if set
  const double* stop = nullptr;    // skip the launch when *stop != 0 (converged)
  // Fused scalar step (device scalars on one shard): every workgroup first
  // runs the scalar_kernel statement `pro - 1` (a ScalarOp) itself, from the
  // reduction partials pro_part[q * pro_stride + 0 .. pro_cnt[q]) summed in
  // the finalize order, and takes c0, c1 from it; workgroup 0 writes the
  // state (st). Saves the one-workgroup scalar launch between two kernels.
  int pro = 0;
  const double* pro_part = nullptr;
  int pro_stride = 0;
  int pro_cnt[5] = {};
  double* st = nullptr;
  int64_t pro_it = 0;              // iteration number (ST_STOP_AT)
  int pro_h = 0;                   // ST_HIST index
  int pro_par = 0;                 // CG: gamma of this iteration in st[gamma_slot(par)]
  int pro_check = 1;
  double pro_thr = 0;
  int pro_s1 = 1;                  // SC_CG_ALPHA: sigma's slot (EPI_XY: 1, EPI_XY_VP: 4)
  int pro_alpha = 0;               // SC_CG_ALPHA: 1 save alpha to ST_ALPHA, 2 c1 = ST_ALPHA
  int pro_pre = 1;                 // VEC: the first operands loaded before the prologue
};
void launch_ew(EwOp op, const EwArgs& a, hipStream_t s);

// Device-resident CG / MrR scalars (scalar_kernel). State layout:
enum ScalarState : int {
  ST_GAMMA = 0,    // CG gamma = <r,r> / MrR gamma = nu/mu
  ST_C0 = 1,       // coefficients of the next vector kernels (EwArgs::cdev)
  ST_C1 = 2,
  ST_C2 = 3,
  ST_C3 = 4,
  ST_STOP = 5,     // 1.0 once the convergence test fired
  ST_STOP_AT = 6,  // iteration at whose top it fired
  ST_GAMMA_ALT = 7,  // fused CG steps: gamma of odd iterations (even: ST_GAMMA)
  ST_ALPHA = 8,    // fused CG, deferred x: alpha of the last EW_CG_NOX step
  ST_HIST = 9,     // ring of reduced norms, one per iteration of a batch
};
// Fused CG steps read this iteration's gamma while workgroup 0 writes the
// next one: two slots, alternating with the iteration's parity.
inline __host__ __device__ int gamma_slot(int par) { return par ? ST_GAMMA_ALT : ST_GAMMA; }
constexpr int kScalarBatch = 64;  // iterations per host sync (ring size)
constexpr int kScalarState = ST_HIST + kScalarBatch;
enum ScalarOp : int { SC_CG_ALPHA = 0, SC_CG_BETA, SC_MRR_GAMMA, SC_MRR_ZETA };
struct ScalarArgs {
  int op = 0;
  int need = 0;                    // bit q: reduce slot q
  const double* partials = nullptr;
  int stride = 0;
  int cnt[5] = {};
  double* st = nullptr;
  int64_t it = 0;                  // iteration number (ST_STOP_AT)
  int h = 0;                       // ST_HIST index
  int check = 1;                   // 0: no convergence test
  double thr = 0;                  // converged <=> 0 <= g < thr
  // RCCL ranks: the per-rank slot totals all-gathered as [nranks][gstride];
  // each reduction is then 0.0 + rank 0 + rank 1 + ... (the host's order).
  const double* gathered = nullptr;
  int nranks = 0, gstride = 0;
};
void launch_scalar(const ScalarArgs& a, hipStream_t s);

// Sum partials[slot*grid .. +grid) for slots [0, nslots) into out[slot],
// in a fixed order (deterministic).
void launch_finalize(const double* partials, int grid, int nslots, double* out,
                     hipStream_t s);
// Upper bound on reduction slots of one finalize (engine: kMaxSlots).
constexpr int kFinalizeSlots = 128;
// Same with stride `stride` per slot and count[slot] partials in slot `slot`
// (launches of different grid sizes feed different slots).
struct SlotCounts {
  int n[kFinalizeSlots];
};
void launch_sqrt(double* p, hipStream_t s);  // p[0] = sqrt(p[0]) (cupy.linalg.norm)
void launch_finalize_counts(const double* partials, int stride, const SlotCounts& counts,
                            int nslots, double* out, hipStream_t s);
// The same for the shards of one stream group in one launch (blockIdx.y =
// shard): shard j's slot totals at out + j * out_stride. Every shard has the
// same stride and counts (System::reduce checks).
constexpr int kGroupMax = 16;
struct FinalizeGroup {
  const double* part[kGroupMax];
  int n = 0;
};
void launch_finalize_group(const FinalizeGroup& g, int stride, const SlotCounts& counts,
                           int nslots, double* out, int out_stride, hipStream_t s);

// Halo rows of in-process shards on one device: every (src, dst, count)
// piece of one shard's receive list (all vectors) in ONE launch instead of a
// hipMemcpyAsync per piece (2.4 us of host time each; a launch is 2.5).
// pieces per gather launch: a stream group of 8 shards, 2 neighbours each,
// 3 vectors (the fused first k-skip MrR steps)
constexpr int kHaloPieces = 48;
struct HaloGatherArgs {
  const double* src[kHaloPieces];
  double* dst[kHaloPieces];
  int64_t count[kHaloPieces];
  int n = 0;
};
void launch_halo_gather(const HaloGatherArgs& a, hipStream_t s);

// Many independent dot products in one pass (count <= 64).
struct MultiDotArgs {
  const double* u[64];
  const double* v[64];
  int count;
  int64_t n;
  double* partials;
  int grid;
};
void launch_multidot(const MultiDotArgs& a, hipStream_t s);

// ---------------------------------------------------------------------------
// Synthetic generators (rows [row0, row0+n) of the global matrix).
// ---------------------------------------------------------------------------
// Poisson: counts (rowptr[i+1] = nnz of row i) then fill after the scan.
// Poisson on side^(dim-1) x nz points (nz = side: the cube).
void launch_poisson_count(int dim, int64_t side, int64_t nz, int64_t row0, int64_t n,
                          void* rowptr, int rowptr64, hipStream_t s);
void launch_poisson_fill(int dim, int64_t side, int64_t nz, int64_t row0, int64_t n,
                         const void* rowptr, int rowptr64, int32_t* col, double* val,
                         hipStream_t s);
struct BandSpec {
  int h;
  int64_t off[64];  // sorted ascending, distinct, >= 1
  uint64_t seed;
  int64_t n_global;
};
void launch_banded_count(const BandSpec& b, int64_t row0, int64_t n, void* rowptr,
                         int rowptr64, hipStream_t s);
void launch_banded_fill(const BandSpec& b, int64_t row0, int64_t n, const void* rowptr,
                        int rowptr64, int32_t* col, double* val, hipStream_t s);
// In-place inclusive scan of rowptr[1..n] (rowptr[0] = 0 set by the caller).
void rowptr_scan(void* rowptr, int rowptr64, int64_t n, hipStream_t s);
void launch_fill_rhs(uint64_t seed, int64_t row0, int64_t n, double* b, hipStream_t s);
// Column statistics of a CSR block: min and max column (global numbering).
void launch_col_minmax(const void* rowptr, int rowptr64, int64_t n, const int32_t* col,
                       int64_t* out2 /* device: {min, max} */, hipStream_t s);
// Interior rows [out3[0], out3[1]) of a block: rows whose columns all lie in
// [lo, hi] (global numbering; local row 0 is global row lo). Boundary rows
// need the halo. out3[2] = the column reach max |col - row|.
void launch_interior(const void* rowptr, int rowptr64, int64_t n, const int32_t* col,
                     int64_t lo, int64_t hi, int64_t* out3, hipStream_t s);
// Distinct column offsets col - (base + row) of a block into table[256]
// (key offset + 2^32, 0 empty); flags: 1 = a row not strictly increasing,
// 2 = more than 256 offsets.
constexpr int kMaxMaskBits = 64;
// Diagonal-offset values from a masked CSR block (values of row i at offset
// M[b] land in dia[b * ld + i]; absent entries stay 0).
constexpr int kDiaRows = 256;  // rows per DIA row block (== kBlock)
// flag[0] = 1 unless every stored lower entry dia(i, k) (M[k] < 0, M symmetric)
// equals dia(i + M[k], nm-1-k) bitwise wherever i + M[k] >= 0.
void launch_dia_symcheck(const void* mask, int mw, int64_t n, const int32_t* M, int nm,
                         const double* dia, int64_t bs, int64_t ks, int* flag, hipStream_t s);
// full[b] = 1 when DIA row block b is whole (256 rows < n) and every row
// holds all nm offsets (the walk's full-block run, Shard::dia_full_lo/hi).
void launch_dia_block_full(const void* mask, int mw, int64_t n, int nm, uint8_t* full,
                           hipStream_t s);
void launch_dia_fill(const void* rowptr, int rowptr64, int64_t n, const int32_t* col,
                     const double* val, int64_t base, const int32_t* M, int nm, double* dia,
                     int64_t bs, int64_t ks, hipStream_t s);
constexpr size_t kOffTableBytes = 256 * sizeof(unsigned long long);
void launch_offsets(const void* rowptr, int rowptr64, int64_t n, const int32_t* col,
                    int64_t base, unsigned long long* table, int* flags, hipStream_t s);
// mask[i] (mw-bit integers) = the bits of row i's offsets in M[0..nm).
void launch_masks(const void* rowptr, int rowptr64, int64_t n, const int32_t* col, int64_t base,
                  const int32_t* M, int nm, int mw, void* mask, hipStream_t s);
// Value dictionary (SpmvArgs::vcode). launch_vdict_collect: the distinct bit
// patterns of val[0, nnz) into gtab[kVdGlobal] (~0 = free slot); flags[0] != 0
// if there are more than kVdMax of them (or the ~0 pattern occurs), flags[1] =
// their count. launch_vdict_encode: code[j] = position of val[j]'s pattern in
// the ascending keys[0, nk).
constexpr int kVdMax = 256;
constexpr int kVdGlobal = 1024;
void launch_vdict_collect(const double* val, int64_t nnz, unsigned long long* gtab, int* flags,
                          hipStream_t s);
void launch_vdict_encode(const double* val, int64_t nnz, const unsigned long long* keys, int nk,
                         uint8_t* code, int* miss, hipStream_t s);
// col[j] += delta for all stored entries of the block.
void launch_col_shift(const void* rowptr, int rowptr64, int64_t n, int32_t* col,
                      int64_t delta, hipStream_t s);

// Host-side helpers shared with the oracle definition.
uint64_t splitmix64(uint64_t x);
void banded_offsets(int h, int64_t width, uint64_t seed, int64_t* out_sorted);

// Scratch for the primitive entry points (grown on demand, per device).
double* primitive_scratch(size_t doubles);

// ---------------------------------------------------------------------------
// Persistent CG (small single-shard systems): m iterations of
// v3/gpu/cg.py:31-39 in ONE cooperative launch, grid-wide barriers instead of
// kernel boundaries. Vectors are full bases (Shard::vec), own row i at
// pad + i; the CSR block is in local column numbering. Writes the same scalar
// state as the device-scalar batches (st[ST_HIST + j] = <r,r> after
// iteration j, ST_STOP / ST_STOP_AT); the final p = r + beta p lands in
// p_a if (iterations run - 1) is even, else p_b.
struct CgPersistArgs {
  const void* rowptr = nullptr;
  int rowptr64 = 0;
  const int32_t* col = nullptr;
  const double* val = nullptr;
  int64_t n = 0, pad = 0;
  double *x = nullptr, *r = nullptr, *pa = nullptr, *pb = nullptr, *v = nullptr;
  double* part = nullptr;    // [2][grid] partials
  unsigned* bar = nullptr;   // barrier counter, zero at launch
  int* err = nullptr;        // set to 1 when a barrier wait timed out
  double* st = nullptr;
  double gamma = 0;          // <r,r> at the top of iteration it0
  int64_t it0 = 0;
  int m = 0;
  double thr = 0;            // convergence threshold on <r,r> (0 <= g < thr)
};
// Workgroups of the cooperative launch (all co-resident); 0 if unsupported.
int cg_persist_grid(int64_t n);
void launch_cg_persist(const CgPersistArgs& a, int grid, hipStream_t s);

// One triangular sweep of the ILU preconditioner (kr_kernels.hip
// ilu_sweep_kernel): levels lvl_ptr[0..nlev] of rows lvl_rows (device), the
// strictly-triangular rows in CSR (rp, col, val; ascending columns) and the
// diagonal. Lower: x[i] = (in[perm[i]] - sum L[i][j] x[j]) / diag[i] (perm =
// the inverse row permutation); upper: x[i] = (in[i] - sum U[i][j] x[j]) /
// diag[i], also stored at out[perm[i]] (perm = the inverse column permutation).
struct IluSweepArgs {
  int64_t nlev = 0;
  int64_t lev0 = 0, lev1 = 0;  // the levels one launch sweeps
  const int64_t* lvl_ptr = nullptr;
  const int32_t* lvl_rows = nullptr;
  const int64_t* rp = nullptr;
  const int32_t* col = nullptr;
  const double* val = nullptr;
  const double* diag = nullptr;
  const double* in = nullptr;
  const int32_t* perm = nullptr;
  double* x = nullptr;
  double* out = nullptr;
  // Level-ordered rows (optional, ew > 0: every row has <= kIluEll
  // strictly-triangular entries, e.g. an ILU(0) of a 7-point stencil): entry
  // t of the level lists holds its row's entries at ecol/eval[t * ew + j],
  // j < ecnt[t] (ascending columns), its diagonal at ediag[t] and the index
  // of its right-hand side in `in` at ein[t] (lower: the inverse row
  // permutation; upper: the row), so a row needs one round of loads indexed
  // by t before the x loads instead of a chain through lvl_rows, rp and col.
  int ew = 0;
  const int32_t* ecol = nullptr;
  const double* eval = nullptr;
  const uint8_t* ecnt = nullptr;
  const double* ediag = nullptr;
  const int32_t* ein = nullptr;
};
constexpr int kIluEll = 8;
// A sweep as launches over its level segments: a run of narrow levels in
// one workgroup (ilu_sweep_kernel), a wide level (more than KR_ILU_WIDE rows)
// over the whole GPU in its own launch (ilu_level_kernel); the kernel
// boundary orders the levels. Every row is computed by one thread with the
// same arithmetic either way: the result does not depend on the split.
struct IluSeg {
  int64_t lev0 = 0, lev1 = 0;  // levels [lev0, lev1)
  int64_t rows = 0;            // wide: the level's rows (0: a narrow run)
};
void launch_ilu_sweep(bool lower, const IluSweepArgs& a, const IluSeg* segs, int nseg,
                      hipStream_t s);

int default_grid(int64_t n);
// Workgroups of the SpMV kernels for a block of n rows with column reach `reach` rows.
int spmv_grid_for(int64_t n, int64_t reach);
// Workgroups of the symmetric DIA walk (spmv_diawalk_kernel) for n rows, nm offsets.
int dia_walk_grid(int64_t n, int nm);
// Upper-slot counts h (= nm / 2) the walk kernel is compiled for (its loops
// over the offsets are straight-line code); other symmetric bands keep the
// strided DIA kernel. C3 (27 offsets) h = 13, C5 (63) h = 31.
constexpr bool dia_walk_h_supported(int h) { return h == 7 || h == 13 || h == 15 || h == 31; }

}  // namespace kr
