// Host engine: sharded system, halo exchange, deterministic reductions and
// the solver sessions. One host thread drives every shard the process owns.
#pragma once

#include <cmath>

#include <rccl/rccl.h>

#include <array>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "kr_internal.h"

namespace kr {

void kskipmrr_recurrence(int k, double* alpha, double* beta, double* delta, double* zeta_out,
                         double* eta_out);
void kskipcg_recurrence(int k, double* a, double* f, double* c, double* alpha_out,
                        double* beta_out);

// RCCL communicator, one rank per GPU.
struct Comm {
  ncclComm_t nccl = nullptr;
  int rank = 0, nranks = 1, device = 0;
};
// Local shards per rank with a communicator (kr_system_create).
constexpr int kMaxLocal = 16;

#define KR_NCCL_CHECK(expr)                                                              \
  do {                                                                                   \
    ncclResult_t kr_r_ = (expr);                                                         \
    if (kr_r_ != ncclSuccess)                                                            \
      throw ::kr::Failure(KR_ERR_RCCL, std::string(#expr) + " -> " +                     \
                                           ncclGetErrorString(kr_r_));                   \
  } while (0)

// Slots of fused reduction products per shard (enough for k <= 16).
constexpr int kMaxSlots = 6 + 7 * 16 + 8;
static_assert(kMaxSlots <= kFinalizeSlots, "finalize slot table too small");

// A contiguous range of global rows exchanged with one peer shard/rank.
struct HaloPiece {
  int peer;        // local shard index (in-process) or global shard (communicator)
  int64_t g0;      // first global row
  int64_t count;   // rows
  // Several shards per rank: an RCCL piece of a shard on another device than
  // the communicator's goes through this buffer on the communicator's device
  // (3 vectors x count doubles), so RCCL only touches its own device's memory.
  double* stage = nullptr;
};

// Per kernel name, aggregated over the shards on the first shard's device
// (System::harvest_profile): one launch = one call of the op; total_ms sums
// the device windows (first begin to last end of the call's shards on that
// device); bytes = the algorithmic bytes of all of them; shards = how many
// shards' launches one call covers there.
struct KernelStat {
  int64_t launches = 0;
  double total_ms = 0;
  double bytes = 0;
  int64_t shards = 1;
};

struct Shard {
  int dev = 0;
  hipStream_t stream = nullptr;
  int64_t row0 = 0, n = 0;
  // CSR block (global columns until finalize, local afterwards)
  const void* rowptr = nullptr;
  int rowptr64 = 0;
  int32_t* col = nullptr;
  const double* val = nullptr;
  int64_t nnz = 0;
  // dense row block instead of CSR (kr_system_adopt_dense): n x n_global
  // row-major, leading dimension dld, global column numbering
  const double* dense = nullptr;
  int64_t dld = 0;
  std::vector<void*> owned;
  // halo geometry: vector = [pad | n own rows | halo_hi]; halo_lo rows sit
  // just below the own rows (pad >= halo_lo, pad multiple of 8).
  int64_t col_lo = 0, col_hi = -1;
  int64_t halo_lo = 0, halo_hi = 0, pad = 0, ld = 0;
  std::vector<HaloPiece> recv, send;
  int64_t int_lo = 0, int_hi = 0;  // interior rows: all columns owned (no halo)
  int64_t reach = 0;                // max |col - row| of the block
  int64_t slab = 0;                 // SpMV slab schedule (row blocks per plane), 0: contiguous
  int64_t slab_sub = 0;             // sub-slab width (row blocks)
  void* mask = nullptr;             // offset masks (SpmvArgs::mask), owned
  double* dia = nullptr;            // diagonal-offset values (SpmvArgs::dia), owned
  int64_t dia_bs = 0, dia_ks = 0;  // SpmvArgs::dia_bs / dia_ks
  int dia_sym = 0;                  // SpmvArgs::dia_sym
  int dia_walk = 0;                 // SpmvArgs::dia_walk (spmv_grid = dia_walk_grid)
  int64_t dia_full_lo = 0, dia_full_hi = 0;  // longest run of full row blocks (SpmvArgs::full_lo)
  int dia_wlen = 0, nseg = 0;       // SpmvArgs x window (dia_wlen, nseg, seg_*, woff)
  int seg_lo[4] = {}, seg_len[4] = {}, seg_base[4] = {};
  int32_t* woff = nullptr;
  int32_t* moff = nullptr;
  int nm = 0, mw = 0;
  uint8_t* vcode = nullptr;         // value dictionary codes (SpmvArgs::vcode), val's index space
  double* vtab = nullptr;           // its table (<= kVdMax doubles), owned
  int ntab = 0;
  int64_t nz0 = 0;                  // rowptr[0]: index of the block's first stored entry
  std::vector<int32_t> moff_h;      // host copy of the offset table (moff)
  // stencil codes (SpmvArgs::scode, kr_stencil.h), owned; st_P = 0: not used
  void* scode = nullptr;
  int st_cb = 8;                    // SpmvArgs::st_cb: bits per slot code = bytes per row
  double* scratch = nullptr;        // SpmvArgs::scratch (stencil SpMV), owned
  int st_P = 0, st_nfar = 0;
  int32_t st_kind[8] = {}, st_far[4] = {};
  // code patterns (SpmvArgs::st_pid / st_pat, System::build_code_patterns), owned
  uint32_t* st_pid = nullptr;
  void* st_pat = nullptr;
  int st_npat = 0;
  // constant-coefficient 7-point box stencil with n = 512 (System::build_box):
  // every entry of slot k is st_v[k], absent entries exactly the box faces;
  // the box pair (kr_pair.hip) then runs without reading the matrix
  bool st_box = false;
  double st_v[8] = {};
  double* pairq = nullptr;  // SpmvArgs::partq of the box pair, 14 x pstride x 4, owned
  hipStream_t comm_stream = nullptr;  // halo exchange, overlapped with interior rows
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  int grid = 1;                 // workgroups of the vector kernels
  int spmv_grid = 1;            // workgroups of the SpMV kernels
  int spmv_grid_po = 1;         // ... of a products-only stencil launch (<= spmv_grid)
  std::vector<int> readers;     // in-process: local shards that copy halo rows from this one
  // ... of them, the ones on another stream (their comm streams copy; the
  // others share this shard's stream, System::groups); ext_in: this shard
  // receives halo pieces from a shard on another stream
  std::vector<int> ext_readers;
  bool ext_in = false;
  bool lead = true;             // first shard of its stream group
  int spmv_grid2 = 1;           // ... of the fused basis pair (System::spmv_pair, <= spmv_grid)
  int pstride = 1;              // partial stride per slot: max(grid, spmv_grid)
  std::array<int, kMaxSlots> slot_n{};  // partials written per slot by its last producer
  // reductions
  double* partials = nullptr;   // [kMaxSlots][pstride]
  double* slots = nullptr;      // [kMaxSlots]
  double* gather = nullptr;     // [nranks][kMaxSlots] (RCCL)
  double* host = nullptr;       // pinned [nranks][kMaxSlots]
  double* st = nullptr;         // device-resident CG/MrR scalars [kScalarState]
  double* hst = nullptr;        // pinned copy of st
  // vectors, each ld doubles, zero-initialised; vector i starts i x
  // KR_VEC_STAGGER bytes into its allocation (vec_base)
  std::vector<double*> vec, vec_base;
  int st_flip = 0;  // the next stencil walk launch runs reversed (SpmvArgs::st_rev)
  hipEvent_t ev_a = nullptr, ev_b = nullptr;
  // profiling (event pairs pending until the next sync)
  struct Pending {
    std::string name;
    hipEvent_t t0, t1;
    double bytes;  // algorithmic bytes of the window
    int nsh;       // shards whose launches the window covers (a stream group: its size)
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> event_pool;

  double* own(int id) const { return vec[id] + pad; }
  int64_t local_index(int64_t g) const { return g - row0 + pad; }
};

class Session;

// Operands of a fused k-skip step (SpmvEpi EPI_STEP_*): vector ids of the
// in/out vectors u1, u2, the x source/destination, and the step's scalars.
struct StepOps {
  int u1 = -1, u2 = -1, us = -1, ud = -1;
  double c0 = 0, c1 = 0;
  int x3 = -1;          // EPI_STEP_MRR_FIRST2: Ar1 (gathered with r0 = in1, y0 = in2)
  double c2 = 0, c3 = 0;
  int xpend = 0;        // EPI_STEP_MRR_FIRST2: SpmvArgs::xpend
  int pro = 0;          // EPI_MRR_V: run the SC_MRR_ZETA step in the prologue
};

// Exchange plan of global shard `me`: the rows it receives from / sends to
// every other shard, as contiguous global ranges (pure host arithmetic).
void plan_halo(int P, const int64_t* part, const int64_t* need_lo, const int64_t* need_hi,
               int me, std::vector<HaloPiece>& recv, std::vector<HaloPiece>& send);

// ILU preconditioner of the pipelined CG family (kr_solve_set_precond_ilu):
// the factors of the reference's `ilu` (a scipy SuperLU, M = Pr^T L U Pc^T)
// on shard 0's device, with the level schedules of both triangular sweeps.
struct IluFactors {
  int dev = 0;
  int64_t n = 0, nnz = 0;           // nnz: strictly-triangular entries of L and U
  IluSweepArgs lower, upper;        // in / out / x pointers set per apply
  std::vector<IluSeg> lseg, useg;   // their launches (launch_ilu_sweep)
  double* y = nullptr;              // L^-1 Pr v
  double* z = nullptr;              // U^-1 y
  std::vector<void*> owned;
  ~IluFactors();
};

// Host threads that enqueue per-shard work in parallel (single-process
// multi-shard systems: one host thread issuing every shard's launches, halo
// copies and event waits serially costs ~4 ms per 512^3 k-skip outer
// iteration at 8 shards, 3x one shard's GPU time). run(n, fn) calls fn(li)
// for li = 0 .. n-1 -- li = 0 on the calling thread, the others on workers --
// and returns when all are done, so a run is a barrier between phases; an
// exception in any fn is rethrown by run. Workers spin between runs and
// sleep after ~1 ms idle.
class ShardPool {
 public:
  explicit ShardPool(int nworkers);
  ~ShardPool();
  ShardPool(const ShardPool&) = delete;
  ShardPool& operator=(const ShardPool&) = delete;
  void run(int n, const std::function<void(int)>& fn);
  int workers() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

struct System {
  int64_t n_global = 0;
  std::vector<Shard> shards;
  Comm* comm = nullptr;             // null: single process
  // With a communicator, a rank may own several shards (a GPU range,
  // v3/gpu/mpi/common.py:77-134): global shards are numbered rank after
  // rank, local shards in order; rank_first[r] = rank r's first global shard.
  // Halo pieces between two local shards are device copies, the others RCCL
  // send/recv on the first local shard's stream (one RCCL rank per process).
  std::vector<int> owner;           // comm: rank of every global shard
  std::vector<int> rank_first;      // comm: size nranks + 1
  double* hy_send = nullptr;        // several local shards: slot totals [kMaxLocal][kMaxSlots]
  double* hy_recv = nullptr;        // [nranks][kMaxLocal][kMaxSlots]
  double* hy_host = nullptr;        // pinned copy of hy_recv
  hipEvent_t hy_ev = nullptr;       // the RCCL group of the exchange is done (shards[0] streams)
  // some rank holds several shards (then every rank takes the hybrid paths,
  // so the RCCL call sequence is the same everywhere)
  bool hybrid() const { return comm && nglobal_shards() != comm->nranks; }
  void halo_hybrid(int id1, int id2, int id3, bool async);
  std::vector<int64_t> part;        // global partition, size P+1
  int first_global = 0;             // global index of shards[0]
  bool finalized = false;
  bool profile = false;
  int profile_every = 1;            // events on every profile_every-th outer iteration
  int64_t prof_tick = 0;
  bool prof_active = true;
  // host time blocked in the per-sync-point waits (reduce, scalar_state_read);
  // kr_solve_step books the rest of each outer iteration's wall time as host
  // enqueue ("host_enqueue" / "host_wait" in the kernel stats of shard 0)
  double host_wait_s = 0.0;
  bool overlap = true;              // split SpMV: interior rows || halo exchange
  bool all_interior = false;        // every shard (all ranks) has interior rows
  bool fuse_steps = true;           // k-skip steps fused into the SpMV epilogue
  bool fuse_first = true;           // k-skip MrR steps 0+1 in one SpMV (EPI_STEP_MRR_FIRST2)
  int epi_late = 0;                 // SpmvArgs::epi_late (A/B knob)
  // Set around an SpMV whose outputs nobody reads (SpmvArgs::products_only);
  // KR_PRODUCTS_ONLY=0 ignores it (A/B).
  bool products_only = false;
  bool products_only_on = true;
  std::unique_ptr<Session> session;
  // Stream groups: the local shards sharing one stream (in-process shards of
  // one device, kr_system_create), in shard order; a shard per group when
  // every shard has its own stream. Work of one group is enqueued by one
  // host thread in shard order.
  std::vector<std::vector<int>> groups;
  // per group of several shards: slot totals of all its shards side by side
  // (kMaxSlots apart), device and pinned, for one finalize launch and one
  // copy per group (System::reduce)
  struct GroupSlots {
    double* dev = nullptr;
    double* host = nullptr;
  };
  std::vector<GroupSlots> gslots;
  // host threads, one per further stream group (in-process, KR_HOST_THREADS != 0)
  std::unique_ptr<ShardPool> pool;
  // fn(group) for every stream group: on the pool when there is one, else in
  // order on this thread
  void for_groups(const std::function<void(const std::vector<int>&)>& fn);
  // fn(shard, li) for every local shard, group by group (each fn sets its
  // shard's device)
  void for_shards(const std::function<void(Shard&, size_t)>& fn);

  ~System();
  int nglobal_shards() const { return (int)part.size() - 1; }

  void finalize();
  void alloc_vectors(int count);
  // Halo exchange of up to two vectors (ids), all shards.
  void build_masks(Shard& s);
  void build_vdict(Shard& s);
  void build_stencil(Shard& s);
  void build_code_patterns(Shard& s);
  void plan_window(Shard& s, const std::vector<int32_t>& M);
  void halo(int id1, int id2 = -1, int id3 = -1);
  // The same exchange on the shards' comm streams, ordered after ev_in and
  // signalling ev_out (overlapped path).
  void halo_async(int id1, int id2, int id3 = -1);
  void halo_in_process(Shard& s, int id1, int id2, int id3);
  void halo_group(const std::vector<int>& grp, int id1, int id2, int id3);
  void spmv(SpmvEpi epi, int in1, int in2, int out1, int out2, int e, int b, int slot0,
            const StepOps* st = nullptr);
  // Two chained EPI_DUAL_MRR basis SpMVs in one launch (spmv_stencil2_kernel):
  // (in1, in2) -> level 2 in (out1, out2) (not stored under products_only),
  // products of the first dual at slot0, of the second at slot0 + 7.
  // pair_mode(): which fused basis pair serves the shard (0: none, two dual
  // launches). One shard, no communicator, a 7-point stencil shard with n =
  // 512 and whole planes, narrow codes; KR_ST2=1: one position per workgroup
  // (spmv_stencil2_kernel, measured slower than two duals),
  // KR_ST2=2: two positions per workgroup (spmv_stencil2t_kernel, P % 16 == 0;
  // bitwise the dual launches, products included), both measured slower;
  // KR_ST2=3 or unset: the box pair (kr_pair.hip) on a Shard::st_box shard
  // with P % 16 == 0 -- the tiled pair's grids and products, the matrix not
  // read; faster than the duals, so the default there.
  int pair_mode() const;
  bool pair_ok() const { return pair_mode() != 0; }
  void spmv_pair(int in1, int in2, int out1, int out2, int slot0, SpmvEpi epi = EPI_DUAL_MRR);
  // The box step pair (kr_pair.hip, launch_spmv_step2b): k-skip MrR steps j
  // and j+1 (EPI_STEP_MRR_NOX + EPI_STEP_MRR_X2) in one walk on a box shard
  // (one shard, no communicator, P % 16 == 0). KR_STEP2=0 disables.
  bool step2_ok() const;
  // r: r_in -> r_out, y: y_in -> y_out (other buffers), z in place, x: xs ->
  // xd; xm: which z's x loses (launch_spmv_step2b); ar1 >= 0: the step
  // triple (steps 0-2, Ar1_0 = ar1, c[4..5] step 2's, xpend)
  void spmv_step2(int r_in, int r_out, int y_in, int y_out, int z, int xs, int xd, int xm,
                  const double* c, int ar1 = -1, int xpend = 0);
  // The box step pair + head (kr_pair.hip, launch_spmv_step2h): the last two
  // steps of an outer iteration (spmv_step2's operands; xm 3, 7 or 6) and
  // the next head SpMV (EPI_HEAD_MRR: Ar1 into vector ar1 from the new r,
  // with the new y as e; products at slots 0..4) in one walk. KR_STEP2H=0
  // disables.
  bool step2h_ok() const;
  void spmv_step2h(int r_in, int r_out, int y_in, int y_out, int z, int xs, int xd, int xm,
                   const double* c, int ar1);
  // walk segments of the box step walks (zh > 0: dividing zh; 0: none)
  int step2_segments(int64_t planes, int zh) const;
  // Shard::st_box from the code patterns (host copies h: the codes of every
  // row block, pid / first: the pattern ids and a block holding each)
  void build_box(Shard& s, const std::vector<uint8_t>& h, const std::vector<uint32_t>& pid,
                 const std::vector<int64_t>& first);
  void ew(EwOp op, double c0, double c1, std::array<int, 6> ids, int slot0);
  // The same for ops with more than 6 operands (-1: unused slot).
  void ew_n(EwOp op, double c0, double c1, const std::array<int, kEwOps>& ids, int slot0);
  // Jacobi diagonal of the preconditioned / pipelined CG family, per local
  // shard (own rows; kr_solve_set_precond), copied into the session's d
  // vector at begin; empty / null: the identity (d = 1).
  std::vector<const double*> precond;
  // ILU instead of the diagonal (one shard): M^-1 v by the two sweeps
  // (ilu_apply; the fused vector kernels then run with d = 1)
  // shared: a session captures the factors at kr_solve_begin, so a later
  // kr_solve_set_precond_ilu (or a clear) affects the next solve only, like
  // the Jacobi diagonal, which the session copies at begin
  std::shared_ptr<IluFactors> ilu;
  void ilu_apply(const IluFactors& f, int in, int out);
  // Device-resident scalars (one shard per rank, or every shard in this
  // process): the vector kernel takes c0, c1 from st[coef], st[coef + 1];
  // scalar() runs one scalar_kernel step over the reductions in slots `need`
  // on the first shard (in-process shards: their slot totals gathered there
  // in shard order) and copies the control part of st to the other shards.
  // While dev_stop is set, every SpMV / vector kernel skips itself once the
  // test has fired (each shard reads its own st[ST_STOP]).
  bool device_scalars() const;
  void scalar_state_init(double gamma);
  void ew_dev(EwOp op, int coef, std::array<int, 6> ids, int slot0);
  void scalar(ScalarOp op, int need, int64_t it, int h, double thr, int check = 1);
  void scalar_state_read();  // st -> hst, synchronises the stream
  // One shard, no communicator: the scalar step runs inside the vector
  // kernel that consumes it (EwArgs::pro) instead of its own launch.
  // KR_FUSE_SCALAR=0 keeps the separate scalar kernel (A/B).
  bool fused_scalars() const;
  void ew_pro(EwOp op, ScalarOp sop, std::array<int, 6> ids, int slot0, int64_t it, int h,
              int par, double thr, int s1 = 1, int alpha = 0);
  // CG's p update folded into the next SpMV (EPI_XY_VP): the SpMV runs the
  // SC_CG_BETA step of iteration `it` (ST_HIST slot h, gamma parity par)
  // over the EW_CG partials in slot 0, gathers p = r + beta p_old, stores
  // p_new and v = A p, products <p,p> <p,v> <v,v> in slots 3..5. vp_ok():
  // one shard without a communicator (the fused scalar steps), a stencil or
  // short-row CSR shard, KR_CG_VP != 0.
  struct VpPro {
    int sop = -1;
    int64_t it = 0;
    int h = 0, par = 0;
    double thr = 0;
  } vp_pro;
  bool vp_ok() const;
  void spmv_vp(int p_old, int r, int out, int p_new, int64_t it, int h, int par, double thr);
  bool dev_stop = false;
  // Device->host of the summed slots [0, nslots): the one host sync point.
  std::vector<double> reduce(int nslots);
  void copy_own(int dst, int src);
  void harvest_profile();

  // profiling helpers
  void prof_begin(Shard& s, const char* name, hipEvent_t& t0);
  void prof_end(Shard& s, const char* name, hipEvent_t t0, double bytes, int nsh = 1);
  // kernel statistics of the first shard's device (harvest_profile)
  std::map<std::string, KernelStat> kstats;
};

// Solver session interface (one per kr_solve_begin).
class Session {
 public:
  virtual ~Session() = default;
  virtual void begin(const double* const* b, const double* const* x0) = 0;
  // Returns true when done.
  virtual bool step_once() = 0;
  virtual int result_x() const = 0;  // vector id holding the solution
  // Apply any update of x still deferred (kr_solve_end, before x is read).
  virtual void settle() {}

  System* sys = nullptr;
  kr_solve_params prm{};
  int k = 0;
  double bnorm = 0;
  int64_t i = 0, index = 0;
  bool done = false, converged = false, diverged = false;
  std::vector<double> residual;
  std::vector<int64_t> nosl, khist;
  bool track_k = false;
  double t_start = 0, t_end = 0;
  int64_t hint = 1;  // iterations kr_solve_step still wants (device-scalar batches)

  void set_entry(int64_t idx, double res) {
    if ((int64_t)residual.size() <= idx) residual.resize(idx + 1, 0.0);
    residual[idx] = res;
  }
  void set_nosl(int64_t idx, int64_t v) {
    if ((int64_t)nosl.size() <= idx) nosl.resize(idx + 1, 0);
    nosl[idx] = v;
  }
  void set_k(int64_t idx, int64_t v) {
    if ((int64_t)khist.size() <= idx) khist.resize(idx + 1, 0);
    khist[idx] = v;
  }
  int64_t entries() const { return index + 1; }
  // kr_solve_params::nan_guard: a non-finite residual entry ends the solve
  // (reported not converged); off, NaN runs on to maxiter as in the reference.
  bool guard_stop(int64_t idx) {
    if (prm.nan_guard && !std::isfinite(residual[idx])) {
      diverged = true;
      done = true;
    }
    return diverged;
  }
};

std::unique_ptr<Session> make_session(System* sys, const kr_solve_params& p);
// Validate and upload the ILU factors (host CSR rows of L and U incl. the
// diagonal, ascending columns; SuperLU's perm_r / perm_c) to `dev`.
std::unique_ptr<IluFactors> build_ilu(int dev, hipStream_t stream, int64_t n, const int64_t* lrp,
                                      const int32_t* lcol, const double* lval, const int64_t* urp,
                                      const int32_t* ucol, const double* uval,
                                      const int64_t* perm_r, const int64_t* perm_c);
double now_seconds();
// wait until a stream's work is done (the solver's sync points; KR_SPIN_SYNC)
void host_sync(hipStream_t st);

}  // namespace kr
