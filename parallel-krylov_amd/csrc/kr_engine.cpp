// Host engine: sharded system + solver sessions.
//
// The reference keeps vectors replicated and moves whole vectors per SpMV
// (v3/gpu/common.py:113-126: full-x peer broadcast + gather; the MPI family
// adds comm.Allgather, v3/gpu/mpi/common.py:163). Here A and EVERY vector are
// row-partitioned; a SpMV input is exchanged only over the halo rows its
// columns reach, and the Gram/dot scalars are reduced once per sync point.
#include "kr_engine.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <exception>
#include <mutex>
#include <numeric>
#include <string_view>
#include <thread>
#include <unordered_map>

namespace kr {

std::atomic<uint64_t> g_env_epoch{0};

double now_seconds() {
  using clk = std::chrono::steady_clock;
  return std::chrono::duration<double>(clk::now().time_since_epoch()).count();
}

bool poison_alloc() {
  const char* e = getenv("KR_POISON_ALLOC");  // read per allocation: tests switch it
  return e && atoi(e) != 0;
}

void fresh_fill(void* p, size_t bytes, hipStream_t s, int dflt) {
  if (!p || bytes == 0) return;
  if (poison_alloc())
    KR_HIP_CHECK(hipMemsetAsync(p, 0xFF, bytes, s));
  else if (dflt >= 0)
    KR_HIP_CHECK(hipMemsetAsync(p, dflt, bytes, s));
}

namespace {

int g_grid_cap = 0;

int cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        c > 0)
      cus = c;
    else
      cus = 256;
  }
  return cus;
}

int grid_cap() {
  if (g_grid_cap == 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        cus > 0) {
      // workgroups per CU of the grid-stride kernels (KR_GRID_PER_CU, A/B)
      const char* env = getenv("KR_GRID_PER_CU");
      const int per_cu = env && atoi(env) > 0 ? atoi(env) : 8;
      g_grid_cap = cus * per_cu;
    }
    else
      g_grid_cap = 2048;
  }
  return g_grid_cap;
}

int ew_vectors(EwOp op) {
  switch (op) {
    case EW_DOT: return 2;
    case EW_MRR_FIRST: return 7;
    case EW_MRR: return 9;
    case EW_CG: return 6;
    case EW_CG_P: return 3;
    case EW_KCG: return 7;
    case EW_MRR_S: return 3;
    case EW_COPY: return 2;
    case EW_MRR_NOX: return 7;
    case EW_MRR_X2: return 9;
    case EW_CG_NOX: return 3;
    case EW_CG_X2: return 7;
    case EW_AXPY: return 3;
    case EW_ONE: return 1;
    case EW_PRE: return 3;
    case EW_PCG: return 9;
    case EW_CGG: return 12;
    case EW_GROPP1: return 9;
    case EW_GROPP2: return 6;
    case EW_DIV: return 3;
    case EW_PIPE: return 18;
  }
  return 0;
}

// The products-only variant of a dual SpMV (System::products_only).
const char* epi_name_po(SpmvEpi e) {
  return e == EPI_DUAL_KCG ? "spmv2_gram_kcg_last" : "spmv2_gram_mrr_last";
}

const char* epi_name(SpmvEpi e) {
  switch (e) {
    case EPI_NONE: return "spmv";
    case EPI_BMINUS: return "spmv_bminus";
    case EPI_XY: return "spmv_xy";
    case EPI_HEAD_MRR: return "spmv_head_mrr";
    case EPI_HEAD_KCG: return "spmv_head_kcg";
    case EPI_MRR_LOOP: return "spmv_mrr_loop";
    case EPI_DUAL_NONE: return "spmv2";
    case EPI_DUAL_MRR: return "spmv2_gram_mrr";
    case EPI_DUAL_KCG: return "spmv2_gram_kcg";
    case EPI_STEP_MRR_NOX: return "spmv_step_mrr_nox";
    case EPI_STEP_MRR_X2: return "spmv_step_mrr_x2";
    case EPI_STEP_MRR_X: return "spmv_step_mrr_x";
    case EPI_STEP_KCG: return "spmv_step_kcg";
    case EPI_STEP_MRR_FIRST2: return "spmv_step_mrr_first2";
    case EPI_XY_VP: return "spmv_xy_vp";
    case EPI_MRR_V: return "spmv_mrr_v";
  }
  return "spmv?";
}

const char* ew_name(EwOp op) {
  switch (op) {
    case EW_DOT: return "dot";
    case EW_MRR_FIRST: return "update_mrr_first";
    case EW_MRR: return "update_mrr";
    case EW_CG: return "update_cg";
    case EW_CG_P: return "update_cg_p";
    case EW_KCG: return "update_kcg";
    case EW_MRR_S: return "mrr_s";
    case EW_COPY: return "copy";
    case EW_MRR_NOX: return "update_mrr_nox";
    case EW_MRR_X2: return "update_mrr_x2";
    case EW_CG_NOX: return "update_cg_nox";
    case EW_CG_X2: return "update_cg_x2";
    case EW_AXPY: return "update_x";
    case EW_ONE: return "fill_one";
    case EW_PRE: return "precond";
    case EW_PCG: return "update_pcg";
    case EW_CGG: return "update_cg_gear";
    case EW_GROPP1: return "update_gropp_xru";
    case EW_GROPP2: return "update_gropp_ps";
    case EW_DIV: return "precond_div";
    case EW_PIPE: return "update_pipecg";
  }
  return "ew?";
}

}  // namespace

int default_grid(int64_t n) {
  const int64_t need = std::max<int64_t>(1, (n + kBlock - 1) / kBlock);
  return (int)std::min<int64_t>(need, grid_cap());
}

// SpMV grid. The XCD-aware schedule gives each XCD a contiguous eighth of
// the row blocks, walked with stride jstep = grid / 8; the resident
// workgroups of an XCD cover a strip of consecutive row blocks that moves
// jstep blocks per round. With jstep equal to the matrix's column reach in
// row blocks (one plane of a 3-D stencil), the strip steps exactly one plane
// per round, so the x rows one plane away (+-n^2) are the ones the strip
// read in the previous round and are still in the XCD's L2: 512^3 Poisson,
// reach 1024 row blocks -> grid 8192 measured +5 % over the default 2048,
// while grids whose stride misses the plane (6, 12, 24, 48 per CU) lost
// 10-15 %. Short reaches keep the default. KR_SPMV_GRID overrides.
int spmv_grid_for(int64_t n, int64_t reach) {
  const char* env = getenv("KR_SPMV_GRID");
  const int64_t nrb = std::max<int64_t>(1, (n + kBlock - 1) / kBlock);
  if (env && atoi(env) > 0) return (int)std::min<int64_t>(atoi(env), nrb);
  const int base = default_grid(n);
  const int64_t rb = (reach + kBlock - 1) / kBlock;
  const int64_t cap = (int64_t)grid_cap() * 8;  // 64 workgroups per CU
  if (rb * 8 <= base || rb * 8 > cap || rb * 8 > nrb) return base;
  // At least 16 row blocks per workgroup (halving keeps the stride a
  // power-of-two fraction of the plane): the per-workgroup prologue and
  // partial reduction cost more than the shorter strip saves once a shard is
  // only a few planes per XCD (512^2 x 64 slab of an 8-GPU run: 8192 -> 4096
  // workgroups, +1.6 %; 6144 measured -13 %).
  int64_t g = rb * 8;
  while (g / 2 >= base && g > nrb / 16 && (g / 2) % 8 == 0) g /= 2;
  return (int)g;
}

// Grid of the symmetric DIA walk (spmv_diawalk_kernel): as many workgroups as
// are resident at once, which the LDS sets -- the mirror buffers (h x 2 KiB)
// and the dual SpMV's two x windows (2 x 6 KiB), plus 1 KiB of static LDS
// -- within 160 KiB per CU, and by registers: C5 (h = 31) 2 per CU, C3 (h = 13)
// 3 per CU. Every
// workgroup then walks one run of consecutive row blocks, all concurrently.
// KR_DIAW_GRID overrides (A/B). oracle/gpu_order.py dia_walk_grid restates it.
int dia_walk_grid(int64_t n, int nm) {
  const int64_t nrb = std::max<int64_t>(1, (n + kBlock - 1) / kBlock);
  const char* env = getenv("KR_DIAW_GRID");
  if (env && atoi(env) > 0) return (int)std::min<int64_t>(atoi(env), nrb);
  const int64_t lds = 8 * ((int64_t)(nm / 2 + 1) * kBlock + 2 * 768) + 1024;
  // ... and the registers: the kernel holds 2 x (h + 1) values per lane (this
  // block's and the next one's): 2 waves per SIMD for h = 31, 3 for 13 / 15,
  // 4 for 7
  const int h = nm / 2;
  const int64_t by_regs = h >= 16 ? 2 : h >= 8 ? 3 : 4;
  const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(by_regs, 160 * 1024 / lds));
  return (int)std::min<int64_t>(nrb, (int64_t)cu_count() * per_cu);
}

void plan_halo(int P, const int64_t* part, const int64_t* need_lo, const int64_t* need_hi,
               int me, std::vector<HaloPiece>& recv, std::vector<HaloPiece>& send) {
  recv.clear();
  send.clear();
  const int64_t r0 = part[me], r1 = part[me + 1];
  for (int t = 0; t < P; ++t) {
    if (t == me) continue;
    const int64_t t0 = part[t], t1 = part[t + 1];
    // rows I need that t owns: my needed range minus my own rows, cut by t's rows
    auto add = [](std::vector<HaloPiece>& out, int peer, int64_t a, int64_t b, int64_t c0,
                  int64_t c1) {
      const int64_t x0 = std::max(a, c0), x1 = std::min(b, c1);
      if (x1 > x0) out.push_back({peer, x0, x1 - x0});
    };
    add(recv, t, need_lo[me], r0, t0, t1);
    add(recv, t, r1, need_hi[me] + 1, t0, t1);
    // rows t needs that I own (the matching sends)
    add(send, t, need_lo[t], t0, r0, r1);
    add(send, t, t1, need_hi[t] + 1, r0, r1);
  }
}

System::~System() {
  session.reset();
  pool.reset();
  if (hy_send) (void)hipFree(hy_send);
  if (hy_recv) (void)hipFree(hy_recv);
  if (hy_host) (void)hipHostFree(hy_host);
  if (hy_ev) (void)hipEventDestroy(hy_ev);
  for (auto& s : shards) {
    (void)hipSetDevice(s.dev);
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    for (auto* list : {&s.send, &s.recv})
      for (auto& p : *list)
        if (p.stage) (void)hipFree(p.stage);
    for (double* v : s.vec_base) (void)hipFree(v);
    for (void* p : s.owned) (void)hipFree(p);
    if (s.partials) (void)hipFree(s.partials);
    if (s.slots) (void)hipFree(s.slots);
    if (s.gather) (void)hipFree(s.gather);
    if (s.host) (void)hipHostFree(s.host);
    if (s.st) (void)hipFree(s.st);
    if (s.hst) (void)hipHostFree(s.hst);
    for (auto& p : s.pending) {
      (void)hipEventDestroy(p.t0);
      (void)hipEventDestroy(p.t1);
    }
    for (auto e : s.event_pool) (void)hipEventDestroy(e);
    if (s.ev_in) (void)hipEventDestroy(s.ev_in);
    if (s.ev_out) (void)hipEventDestroy(s.ev_out);
    if (s.comm_stream) (void)hipStreamDestroy(s.comm_stream);
    if (s.ev_a) (void)hipEventDestroy(s.ev_a);
    if (s.ev_b) (void)hipEventDestroy(s.ev_b);
  }
  for (auto& g : gslots) {
    if (g.dev) (void)hipFree(g.dev);
    if (g.host) (void)hipHostFree(g.host);
  }
  // streams last, each once (shards of one device may share one)
  for (size_t li = 0; li < shards.size(); ++li) {
    Shard& s = shards[li];
    bool first = s.stream != nullptr;
    for (size_t t = 0; t < li && first; ++t) first = shards[t].stream != s.stream;
    if (first) {
      (void)hipSetDevice(s.dev);
      (void)hipStreamDestroy(s.stream);
    }
  }
}

// ------------------------------------------------------------- ShardPool
struct ShardPool::Impl {
  std::vector<std::thread> th;
  std::atomic<uint64_t> gen{0};
  std::atomic<int> pending{0};
  std::atomic<bool> stop{false};
  const std::function<void(int)>* fn = nullptr;
  int n = 0;
  std::vector<std::exception_ptr> err;
  std::mutex mu;
  std::condition_variable cv;

  void worker(int w) {
    uint64_t seen = 0;
    for (;;) {
      int spins = 0;
      while (gen.load(std::memory_order_acquire) == seen && !stop.load()) {
        if (++spins < (1 << 14)) {
          __builtin_ia32_pause();
        } else {  // idle: sleep until the next run (no lost wake-up: gen changes under mu)
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [&] { return gen.load() != seen || stop.load(); });
        }
      }
      if (stop.load()) return;
      seen = gen.load(std::memory_order_acquire);
      const int li = w + 1;
      if (li < n) {
        try {
          (*fn)(li);
        } catch (...) {
          err[li] = std::current_exception();
        }
      }
      pending.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
};

ShardPool::ShardPool(int nworkers) : impl_(new Impl) {
  for (int w = 0; w < nworkers; ++w) impl_->th.emplace_back([this, w] { impl_->worker(w); });
}

ShardPool::~ShardPool() {
  {
    std::lock_guard<std::mutex> lk(impl_->mu);
    impl_->stop.store(true);
  }
  impl_->cv.notify_all();
  for (auto& t : impl_->th) t.join();
}

int ShardPool::workers() const { return (int)impl_->th.size(); }

void ShardPool::run(int n, const std::function<void(int)>& fn) {
  Impl& I = *impl_;
  KR_REQUIRE(n <= (int)I.th.size() + 1, "ShardPool: more shards than threads");
  I.fn = &fn;
  I.n = n;
  I.err.assign((size_t)n, nullptr);
  I.pending.store((int)I.th.size(), std::memory_order_release);
  {
    std::lock_guard<std::mutex> lk(I.mu);
    I.gen.fetch_add(1, std::memory_order_acq_rel);
  }
  I.cv.notify_all();
  try {
    fn(0);
  } catch (...) {
    I.err[0] = std::current_exception();
  }
  while (I.pending.load(std::memory_order_acquire) > 0) __builtin_ia32_pause();
  for (auto& e : I.err)
    if (e) std::rethrow_exception(e);
}

// The solver's sync points (reduce, scalar_state_read): the host needs the
// result as soon as the copy lands, to compute the next scalars and enqueue
// the next launches while the GPU idles. KR_SPIN_SYNC (A/B, default on):
// poll the stream instead of hipStreamSynchronize's wait.
void host_sync(hipStream_t st) {
  if (KR_ENV("KR_SPIN_SYNC", 1) == 0) {
    KR_HIP_CHECK(hipStreamSynchronize(st));
    return;
  }
  for (;;) {
    const hipError_t e = hipStreamQuery(st);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) KR_HIP_CHECK(e);
    for (int i = 0; i < 16; ++i) __builtin_ia32_pause();
  }
}

void System::for_groups(const std::function<void(const std::vector<int>&)>& fn) {
  if (pool && groups.size() > 1) {
    pool->run((int)groups.size(), [&](int g) { fn(groups[(size_t)g]); });
    return;
  }
  for (auto& g : groups) fn(g);
}

void System::for_shards(const std::function<void(Shard&, size_t)>& fn) {
  if (groups.empty()) {  // before finalize
    for (size_t li = 0; li < shards.size(); ++li) fn(shards[li], li);
    return;
  }
  for_groups([&](const std::vector<int>& g) {
    for (int li : g) fn(shards[(size_t)li], (size_t)li);
  });
}

IluFactors::~IluFactors() {
  (void)hipSetDevice(dev);
  for (void* p : owned) (void)hipFree(p);
}

namespace {
// Levels of a triangular sweep: level(i) = 1 + the largest level of the rows
// row i reads (0 for none), in sweep order (ascending rows for L, descending
// for U). Returns the rows grouped by level (ascending row index inside a
// level) and the level offsets.
void sweep_levels(int64_t n, const int64_t* rp, const int32_t* col, bool lower,
                  std::vector<int32_t>& rows, std::vector<int64_t>& ptr) {
  std::vector<int32_t> lev((size_t)n, 0);
  int32_t top = -1;
  for (int64_t q = 0; q < n; ++q) {
    const int64_t i = lower ? q : n - 1 - q;
    int32_t l = 0;
    for (int64_t jj = rp[i]; jj < rp[i + 1]; ++jj) l = std::max(l, lev[(size_t)col[jj]] + 1);
    lev[(size_t)i] = l;
    top = std::max(top, l);
  }
  ptr.assign((size_t)top + 2, 0);
  for (int64_t i = 0; i < n; ++i) ++ptr[(size_t)lev[(size_t)i] + 1];
  for (size_t l = 1; l < ptr.size(); ++l) ptr[l] += ptr[l - 1];
  rows.assign((size_t)n, 0);
  std::vector<int64_t> fill(ptr.begin(), ptr.end() - 1);
  for (int64_t i = 0; i < n; ++i) rows[(size_t)fill[(size_t)lev[(size_t)i]]++] = (int32_t)i;
}

// Split one factor (full rows incl. the diagonal, ascending columns) into its
// strictly-triangular CSR and its diagonal, checking the triangle.
void split_factor(int64_t n, const int64_t* rp, const int32_t* col, const double* val, bool lower,
                  std::vector<int64_t>& srp, std::vector<int32_t>& scol, std::vector<double>& sval,
                  std::vector<double>& diag) {
  const char* which = lower ? "L" : "U";
  srp.assign((size_t)n + 1, 0);
  scol.clear();
  sval.clear();
  diag.assign((size_t)n, 0.0);
  KR_REQUIRE(rp[0] == 0, std::string("ILU: ") + which + " row pointer must start at 0");
  for (int64_t i = 0; i < n; ++i) {
    KR_REQUIRE(rp[i + 1] >= rp[i], std::string("ILU: ") + which + " row pointer decreases");
    bool have = false;
    int64_t prev = -1;
    for (int64_t jj = rp[i]; jj < rp[i + 1]; ++jj) {
      const int64_t j = col[jj];
      KR_REQUIRE(j > prev && j < n, std::string("ILU: ") + which +
                                         " columns must ascend within a row and lie in [0, n)");
      prev = j;
      if (j == i) {
        have = true;
        diag[(size_t)i] = val[jj];
      } else {
        KR_REQUIRE(lower ? j < i : j > i,
                   std::string("ILU: ") + which + " has an entry on the wrong side of the diagonal");
        scol.push_back((int32_t)j);
        sval.push_back(val[jj]);
      }
    }
    KR_REQUIRE(have && diag[(size_t)i] != 0.0 && std::isfinite(diag[(size_t)i]),
               std::string("ILU: ") + which + " needs a finite nonzero diagonal in every row (row " +
                   std::to_string(i) + ")");
    srp[(size_t)i + 1] = (int64_t)scol.size();
  }
}

std::vector<int32_t> inverse_perm(int64_t n, const int64_t* p, const char* what) {
  std::vector<int32_t> inv((size_t)n, -1);
  for (int64_t i = 0; i < n; ++i) {
    KR_REQUIRE(p[i] >= 0 && p[i] < n && inv[(size_t)p[i]] < 0,
               std::string("ILU: ") + what + " is not a permutation of 0..n-1");
    inv[(size_t)p[i]] = (int32_t)i;
  }
  return inv;
}
}  // namespace

std::unique_ptr<IluFactors> build_ilu(int dev, hipStream_t stream, int64_t n, const int64_t* lrp,
                                      const int32_t* lcol, const double* lval, const int64_t* urp,
                                      const int32_t* ucol, const double* uval,
                                      const int64_t* perm_r, const int64_t* perm_c) {
  KR_REQUIRE(n > 0 && n < ((int64_t)1 << 31), "ILU: n must lie in [1, 2^31)");
  auto f = std::make_unique<IluFactors>();
  f->dev = dev;
  f->n = n;
  KR_HIP_CHECK(hipSetDevice(dev));
  auto up = [&](const void* h, size_t bytes) {
    void* d = nullptr;
    KR_HIP_CHECK(hipMalloc(&d, std::max<size_t>(bytes, 8)));
    f->owned.push_back(d);
    if (h && bytes) KR_HIP_CHECK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream));
    return d;
  };
  for (int side = 0; side < 2; ++side) {
    const bool lo = side == 0;
    std::vector<int64_t> srp, ptr;
    std::vector<int32_t> scol, rows;
    std::vector<double> sval, diag;
    split_factor(n, lo ? lrp : urp, lo ? lcol : ucol, lo ? lval : uval, lo, srp, scol, sval, diag);
    sweep_levels(n, srp.data(), scol.data(), lo, rows, ptr);
    IluSweepArgs& a = lo ? f->lower : f->upper;
    a.nlev = (int64_t)ptr.size() - 1;
    a.lvl_ptr = static_cast<const int64_t*>(up(ptr.data(), 8 * ptr.size()));
    a.lvl_rows = static_cast<const int32_t*>(up(rows.data(), 4 * rows.size()));
    a.rp = static_cast<const int64_t*>(up(srp.data(), 8 * srp.size()));
    a.col = static_cast<const int32_t*>(up(scol.data(), 4 * scol.size()));
    a.val = static_cast<const double*>(up(sval.data(), 8 * sval.size()));
    a.diag = static_cast<const double*>(up(diag.data(), 8 * diag.size()));
    const std::vector<int32_t> inv =
        inverse_perm(n, lo ? perm_r : perm_c, lo ? "perm_r" : "perm_c");
    a.perm = static_cast<const int32_t*>(up(inv.data(), 4 * inv.size()));
    f->nnz += (int64_t)scol.size();
    // level-ordered rows when every row has <= kIluEll entries (KR_ILU_ELL=0:
    // the CSR chain, A/B)
    int64_t wmax = 0;
    for (int64_t i = 0; i < n; ++i) wmax = std::max(wmax, srp[(size_t)i + 1] - srp[(size_t)i]);
    if (KR_ENV("KR_ILU_ELL", 1) != 0 && wmax <= kIluEll) {
      const int ew = (int)std::max<int64_t>(wmax, 1);
      std::vector<int32_t> ecol((size_t)n * ew, 0), ein((size_t)n);
      std::vector<double> eval((size_t)n * ew, 0.0), ediag((size_t)n);
      std::vector<uint8_t> ecnt((size_t)n);
      for (int64_t t = 0; t < n; ++t) {
        const int64_t i = rows[(size_t)t];
        const int64_t b = srp[(size_t)i], e = srp[(size_t)i + 1];
        ecnt[(size_t)t] = (uint8_t)(e - b);
        for (int64_t jj = b; jj < e; ++jj) {
          ecol[(size_t)t * ew + (jj - b)] = scol[(size_t)jj];
          eval[(size_t)t * ew + (jj - b)] = sval[(size_t)jj];
        }
        ediag[(size_t)t] = diag[(size_t)i];
        ein[(size_t)t] = lo ? inv[(size_t)i] : (int32_t)i;
      }
      a.ew = ew;
      a.ecol = static_cast<const int32_t*>(up(ecol.data(), 4 * ecol.size()));
      a.eval = static_cast<const double*>(up(eval.data(), 8 * eval.size()));
      a.ecnt = static_cast<const uint8_t*>(up(ecnt.data(), ecnt.size()));
      a.ediag = static_cast<const double*>(up(ediag.data(), 8 * ediag.size()));
      a.ein = static_cast<const int32_t*>(up(ein.data(), 4 * ein.size()));
      KR_HIP_CHECK(hipStreamSynchronize(stream));  // the host vectors go out of scope
    }
    // launches: runs of levels of <= KR_ILU_WIDE rows in one workgroup, each
    // wider level over the grid (0: every level in the one workgroup)
    const int64_t wide = KR_ENV("KR_ILU_WIDE", 4096);
    std::vector<IluSeg>& segs = lo ? f->lseg : f->useg;
    for (int64_t l = 0; l < a.nlev; ++l) {
      const int64_t w = ptr[(size_t)l + 1] - ptr[(size_t)l];
      if (wide > 0 && w > wide) {
        segs.push_back({l, l + 1, w});
      } else if (!segs.empty() && segs.back().rows == 0 && segs.back().lev1 == l) {
        segs.back().lev1 = l + 1;
      } else {
        segs.push_back({l, l + 1, 0});
      }
    }
  }
  f->y = static_cast<double*>(up(nullptr, 8 * (size_t)n));
  f->z = static_cast<double*>(up(nullptr, 8 * (size_t)n));
  KR_HIP_CHECK(hipStreamSynchronize(stream));  // the host vectors go out of scope
  return f;
}

bool stencil_pm(int P);

int System::pair_mode() const {
  if (shards.size() != 1 || comm || nglobal_shards() != 1) return 0;
  // KR_ST2: 0 two dual launches; 1, 2 the code-reading pairs (A/B); 3 the box
  // pair; unset: the box pair where the shard is a box (measured on C4, one
  // box, profiles/r06a: the storing pair 1.44-1.46 ms against two duals'
  // 1.68, the products-only pair 1.14-1.16 against 0.84 + 0.59; 545 -> 586
  // it/s), else the duals
  const int env = KR_ENV("KR_ST2", -1);
  const int mode = env < 0 ? 3 : env;
  if (mode != 1 && mode != 2 && mode != 3) return 0;
  const Shard& s = shards[0];
  // (the box pair writes the partials in the position-major dual grids'
  // workgroup order: KR_STENCIL_PM=0 keeps the duals)
  if (mode == 3)
    return s.st_box && s.st_P % 16 == 0 && stencil_pm(s.st_P) && s.spmv_grid % s.st_P == 0 &&
                   s.spmv_grid_po % s.st_P == 0
               ? 3 : 0;
  if (!s.scode || !stencil_pm(s.st_P) || s.nm != 7 || s.st_nfar != 2) return 0;
  if (s.st_far[0] != -kStencilBlock || s.st_far[1] != kStencilBlock) return 0;
  if (s.st_cb != 2 && s.st_cb != 4) return 0;
  const int64_t W = (int64_t)s.st_P * kStencilBlock;
  static const int kPat[7] = {1, 4, 3, 0, 3, 5, 2};  // kPat7: PREV FAR0 NEAR CENTER NEAR FAR1 NEXT
  for (int k = 0; k < 7; ++k)
    if (s.st_kind[k] != kPat[k]) return 0;
  if (s.n % W != 0 || s.n / W < 2) return 0;
  if (mode == 1) return s.spmv_grid2 % s.st_P == 0 ? 1 : 0;
  // the tiled pair writes the partials of both dual grids (general and
  // products-only, position-major: P x segments)
  return s.st_P % 16 == 0 && s.spmv_grid % s.st_P == 0 && s.spmv_grid_po % s.st_P == 0 ? 2 : 0;
}

void System::spmv_pair(int in1, int in2, int out1, int out2, int slot0, SpmvEpi epi) {
  const int mode = pair_mode();
  KR_REQUIRE(mode != 0, "fused basis pair: shard not eligible");
  KR_REQUIRE(mode >= 2 || epi == EPI_DUAL_MRR, "fused basis pair (KR_ST2=1): k-skip MrR only");
  KR_REQUIRE(slot0 + 14 <= kMaxSlots, "reduction slots exhausted");
  Shard& s = shards[0];
  KR_HIP_CHECK(hipSetDevice(s.dev));
  const bool po = products_only && products_only_on;
  const char* nm = epi == EPI_DUAL_KCG ? (po ? "spmv2x2_gram_kcg_last" : "spmv2x2_gram_kcg")
                                       : (po ? "spmv2x2_gram_mrr_last" : "spmv2x2_gram_mrr");
  hipEvent_t t0 = nullptr;
  prof_begin(s, nm, t0);
  SpmvArgs a;
  a.n = s.n;
  a.x1 = s.vec[in1];
  a.x2 = s.vec[in2];
  a.xoff = s.pad;
  a.y1 = s.own(out1);
  a.y2 = s.own(out2);
  a.partials = s.partials + (size_t)slot0 * s.pstride;
  a.partials2 = s.partials + (size_t)(slot0 + 7) * s.pstride;
  a.grid = s.pstride;
  a.vtab = s.vtab;
  a.ntab = s.ntab;
  a.scode = s.scode;
  a.st_cb = s.st_cb;
  a.st_P = s.st_P;
  a.st_pm = 1;
  a.st_nm = s.nm;
  a.st_nfar = s.st_nfar;
  for (int k = 0; k < 8; ++k) {
    a.st_off[k] = k < s.nm ? s.moff_h[k] : 0;
    a.st_kind[k] = s.st_kind[k];
  }
  for (int f = 0; f < 4; ++f) a.st_far[f] = s.st_far[f];
  a.xlen = s.ld;
  a.scratch = s.scratch;
  a.products_only = po ? 1 : 0;
  a.stop = dev_stop ? s.st + ST_STOP : nullptr;
  if (mode == 1) {
    launch_spmv_stencil2(a, s.spmv_grid2, s.stream);
    for (int p = 0; p < 14; ++p) s.slot_n[slot0 + p] = s.spmv_grid2;
  } else {
    // level 1 = dual m on the general grid, level 2 = dual m+1 on the grid
    // its launch would use (the products-only one for the last pair); the
    // walk segments divide both: the largest such count <= KR_ST2T_Z
    const int g1 = s.spmv_grid, g2 = po ? s.spmv_grid_po : s.spmv_grid;
    const int z1 = g1 / s.st_P, z2 = g2 / s.st_P;
    const char* ze = getenv(mode == 3 ? "KR_ST2B_Z" : "KR_ST2T_Z");
    // the box pair: 128-plane walks at 512^3 (KR_ST2B_Z 4 / 8 / 16 / 32: the
    // storing pair 1.385 / 1.395 / 1.444 / 1.542 ms in the first build; same
    // box, twice each, profiles/r06d: 4 / 8 / 16 give the products-only pair
    // 1.013-1.019 / 1.046-1.054 / 1.102-1.107 ms, the storing pair equal)
    const int zcap = ze && atoi(ze) > 0 ? atoi(ze) : (mode == 3 ? 4 : 16);
    const int zg = std::gcd(z1, z2);
    int zw = 1;
    for (int d = 1; d <= zg; ++d)
      if (zg % d == 0 && d <= zcap) zw = d;
    a.st2_z1 = z1;
    a.st2_z2 = z2;
    if (mode == 3) {
      a.st_box = 1;
      for (int k = 0; k < 8; ++k) a.st_v[k] = s.st_v[k];
      if (!s.pairq) {
        const size_t bytes = sizeof(double) * 14 * 4 * (size_t)s.pstride;
        KR_HIP_CHECK(hipMalloc(&s.pairq, bytes));
        s.owned.push_back(s.pairq);
        fresh_fill(s.pairq, bytes, s.stream);
      }
      a.partq = s.pairq;
      const int xs = st2b_xsegments(po);
      launch_spmv_stencil2b(epi, a, (s.st_P / 2) * xs * zw, xs, g1, g2, s.stream);
    } else {
      launch_spmv_stencil2t(epi, a, (s.st_P / 2) * zw, s.stream);
    }
    for (int p = 0; p < 7; ++p) {
      s.slot_n[slot0 + p] = g1;
      s.slot_n[slot0 + 7 + p] = g2;
    }
  }
  // algorithmic bytes in CSR terms, like every SpMV's (bench.py subtracts the
  // stored format's saving): A once, the two input vectors and the two
  // level-2 outputs (none products-only) -- one dual SpMV's; level 1 never
  // leaves the chip
  const double bytes = 12.0 * s.nnz + 4.0 * (s.n + 1) + 16.0 * s.n + (po ? 0.0 : 16.0 * s.n);
  prof_end(s, nm, t0, bytes);
}

bool System::step2_ok() const {
  if (shards.size() != 1 || comm || nglobal_shards() != 1) return false;
  if (KR_ENV("KR_STEP2", 1) == 0) return false;
  const Shard& s = shards[0];
  return s.st_box && s.st_P % 16 == 0;
}

void System::spmv_step2(int r_in, int r_out, int y_in, int y_out, int z, int xs, int xd, int xm,
                        const double* c, int ar1, int xpend) {
  KR_REQUIRE(step2_ok(), "box step pair: shard not eligible");
  KR_REQUIRE(r_out != r_in && y_out != y_in && y_out != r_in && r_out != y_in &&
                 (ar1 < 0 || (ar1 != r_out && ar1 != y_out)),
             "box step pair: r / y outputs alias their gathered inputs");
  const bool virt = ar1 >= 0;
  Shard& s = shards[0];
  KR_HIP_CHECK(hipSetDevice(s.dev));
  const char* nm = virt ? "spmv_step3_mrr_stencil" : "spmv_step2_mrr_stencil";
  hipEvent_t t0 = nullptr;
  prof_begin(s, nm, t0);
  SpmvArgs a;
  a.n = s.n;
  a.x1 = s.vec[r_in];
  a.x2 = s.vec[y_in];
  a.xoff = s.pad;
  a.xlen = s.ld;
  a.y1 = s.own(r_out);
  a.u1 = s.own(y_out);
  a.u2 = s.own(z);
  a.us = s.own(xs);
  a.ud = s.own(xd);
  a.c0 = c[0];
  a.c1 = c[1];
  a.c2 = c[2];
  a.c3 = c[3];
  if (virt) {
    a.x3 = s.vec[ar1];
    a.c4 = c[4];
    a.c5 = c[5];
    a.xpend = xpend;
  }
  a.st_P = s.st_P;
  a.st_box = 1;
  for (int k = 0; k < 8; ++k) a.st_v[k] = s.st_v[k];
  a.stop = dev_stop ? s.st + ST_STOP : nullptr;
  // walk segments: 4 per plane column at 512 planes (128-plane walks), fewer
  // on thinner boxes (>= 8 planes per walk); KR_STEP2_Z overrides. Measured
  // on C4 (same box, twice each, profiles/r06c, r06d): 4 / 8 / 16 / 32
  // segments give the step pair 1.36-1.38 / 1.37-1.41 / 1.39-1.42 / 1.43-1.45
  // ms (the triple varies 1.57-1.79 ms from run to run at any count)
  const int64_t planes = s.n / ((int64_t)s.st_P * kStencilBlock);
  launch_spmv_step2b(a, (s.st_P / 2) * step2_segments(planes, 0), virt ? 1 : 0, xm, s.stream);
  // algorithmic bytes in CSR terms: A once, r, y, (Ar1,) z, x in and r, y,
  // z, x out (x neither way when no step of the pair touches it)
  const double vecs = (virt ? 9.0 : 8.0) - (virt || xm != 0 ? 0.0 : 2.0);
  const double bytes = 12.0 * s.nnz + 4.0 * (s.n + 1) + 8.0 * vecs * s.n;
  prof_end(s, nm, t0, bytes);
}

bool System::step2h_ok() const {
  if (!step2_ok() || KR_ENV("KR_STEP2H", 1) == 0) return false;
  const Shard& s = shards[0];
  // the head's partials in its position-major grid's workgroup order
  if (!stencil_pm(s.st_P) || s.spmv_grid % s.st_P != 0) return false;
  // walk segments (spmv_step2h) dividing the head grid's plane segments
  const int64_t planes = s.n / ((int64_t)s.st_P * kStencilBlock);
  const int zh = s.spmv_grid / s.st_P;
  return zh >= 1 && planes >= zh && step2_segments(planes, zh) > 0;
}

// Walk segments of the box step walks: KR_STEP2_Z, else 4 per plane column at
// 512 planes (128-plane walks), fewer on thinner boxes (>= 8 planes per
// walk). With zh > 0 (the step pair + head) the largest count <= that which
// divides zh (0: none).
int System::step2_segments(int64_t planes, int zh) const {
  int zw = KR_ENV("KR_STEP2_Z", 0);
  if (zw <= 0) {
    zw = 1;
    while (zw < 4 && planes / (2 * zw) >= 8) zw *= 2;
  }
  zw = (int)std::min<int64_t>(zw, planes);
  if (zh > 0) {
    while (zw > 1 && zh % zw != 0) --zw;
    if (zh % zw != 0) return 0;
  }
  return zw;
}

void System::spmv_step2h(int r_in, int r_out, int y_in, int y_out, int z, int xs, int xd, int xm,
                         const double* c, int ar1) {
  KR_REQUIRE(step2h_ok(), "box step pair + head: shard not eligible");
  KR_REQUIRE(r_out != r_in && y_out != y_in && y_out != r_in && r_out != y_in && ar1 != r_in &&
                 ar1 != r_out && ar1 != y_in && ar1 != y_out,
             "box step pair + head: outputs alias their gathered inputs");
  Shard& s = shards[0];
  KR_HIP_CHECK(hipSetDevice(s.dev));
  const char* nm = "spmv_step2h_mrr_stencil";
  hipEvent_t t0 = nullptr;
  prof_begin(s, nm, t0);
  SpmvArgs a;
  a.n = s.n;
  a.x1 = s.vec[r_in];
  a.x2 = s.vec[y_in];
  a.xoff = s.pad;
  a.xlen = s.ld;
  a.y1 = s.own(r_out);
  a.y2 = s.own(ar1);
  a.u1 = s.own(y_out);
  a.u2 = s.own(z);
  a.us = s.own(xs);
  a.ud = s.own(xd);
  a.c0 = c[0];
  a.c1 = c[1];
  a.c2 = c[2];
  a.c3 = c[3];
  a.st_P = s.st_P;
  a.st_box = 1;
  for (int k = 0; k < 8; ++k) a.st_v[k] = s.st_v[k];
  a.stop = dev_stop ? s.st + ST_STOP : nullptr;
  a.partials = s.partials;  // the head's slots 0..4
  a.grid = s.pstride;
  if (!s.pairq) {
    const size_t bytes = sizeof(double) * 14 * 4 * (size_t)s.pstride;
    KR_HIP_CHECK(hipMalloc(&s.pairq, bytes));
    s.owned.push_back(s.pairq);
    fresh_fill(s.pairq, bytes, s.stream);
  }
  a.partq = s.pairq;
  const int64_t planes = s.n / ((int64_t)s.st_P * kStencilBlock);
  const int zh = s.spmv_grid / s.st_P;
  a.st2_z1 = zh;
  const int zw = step2_segments(planes, zh);
  launch_spmv_step2h(a, (s.st_P / 2) * zw, xm, s.spmv_grid, s.stream);
  for (int p = 0; p < 5; ++p) s.slot_n[p] = s.spmv_grid;
  // algorithmic bytes in CSR terms, like the other walks' (A once: bench.py
  // subtracts the stored format's saving once per launch): r, y, z, x in (x
  // only when a step touches it) and r, y, z, x, Ar1 out
  const double vecs = 9.0 - (xm != 0 ? 0.0 : 2.0);
  const double bytes = 12.0 * s.nnz + 4.0 * (s.n + 1) + 8.0 * vecs * s.n;
  prof_end(s, nm, t0, bytes);
}

// M^-1 v (shard 0): w = Pr v folded into the L sweep's loads, y = L^-1 w,
// z = U^-1 y, out = Pc z folded into the U sweep's stores.
void System::ilu_apply(const IluFactors& f, int in, int out) {
  KR_REQUIRE(shards.size() == 1, "ILU apply: more than one shard");
  const IluFactors* ilu = &f;
  Shard& s = shards[0];
  KR_HIP_CHECK(hipSetDevice(s.dev));
  hipEvent_t t0;
  prof_begin(s, "ilu_sweeps", t0);
  IluSweepArgs lo = ilu->lower, hi = ilu->upper;
  lo.in = s.own(in);
  lo.x = ilu->y;
  hi.in = ilu->y;
  hi.x = ilu->z;
  hi.out = s.own(out);
  launch_ilu_sweep(true, lo, ilu->lseg.data(), (int)ilu->lseg.size(), s.stream);
  launch_ilu_sweep(false, hi, ilu->useg.data(), (int)ilu->useg.size(), s.stream);
  // values + columns + row pointers of both factors, the diagonals, and the
  // vectors: v, y (written, read), z (written), out
  prof_end(s, "ilu_sweeps", t0,
           12.0 * (double)ilu->nnz + 8.0 * 2 * (double)(ilu->n + 1) + 8.0 * 8 * (double)ilu->n);
}

// x window of the DIA kernel (SpmvArgs::nseg ...): offsets closer than 256
// rows share a segment; at most 4 segments and 4096 rows (32 KiB per vector),
// else the kernel gathers from global memory. KR_DIA_XL=0 disables (A/B).
void System::plan_window(Shard& s, const std::vector<int32_t>& M) {
  const char* xl = getenv("KR_DIA_XL");
  if (xl && atoi(xl) == 0) return;
  std::vector<std::pair<int64_t, int64_t>> seg;  // [lo, hi] offsets
  for (int32_t o : M) {
    if (!seg.empty() && (int64_t)o - seg.back().second <= kBlock)
      seg.back().second = o;
    else
      seg.push_back({o, o});
  }
  if ((int)seg.size() > SpmvArgs::kMaxSeg) return;
  int base = 0;
  int g = 0;
  std::vector<int32_t> woff(M.size());
  for (auto& [lo, hi] : seg) {
    const int64_t lo_e = lo - (lo & 1);                      // even start
    const int64_t len = (kBlock + hi - lo_e + 1) / 2 * 2;    // even length
    if (base + len > 4096) return;
    s.seg_lo[g] = (int)lo_e;
    s.seg_len[g] = (int)len;
    s.seg_base[g] = base;
    for (size_t b = 0; b < M.size(); ++b)
      if (M[b] >= lo && M[b] <= hi) woff[b] = (int32_t)(base - lo_e + M[b]);
    base += (int)len;
    ++g;
  }
  int32_t* dW = nullptr;
  KR_HIP_CHECK(hipMalloc(&dW, 64 * sizeof(int32_t)));
  s.owned.push_back(dW);
  KR_HIP_CHECK(hipMemcpyAsync(dW, woff.data(), woff.size() * sizeof(int32_t),
                              hipMemcpyHostToDevice, s.stream));
  KR_HIP_CHECK(hipStreamSynchronize(s.stream));
  s.woff = dW;
  s.nseg = g;
  s.dia_wlen = base;
}

void System::build_masks(Shard& s) {
  const char* env = getenv("KR_MASK");
  if (env && atoi(env) == 0) return;
  // Diagonal-offset values for long rows (mean >= kLongRow nnz/row: banded
  // C3 +23 %, C5 +35 % over the product-then-sum kernel). Short rows keep the
  // LDS-staged row walk with masks, which measured equal or up to 5 % faster
  // on 512^3 Poisson (C2 256^3: DIA +3 %). KR_DIA=0 never, KR_DIA=2 always.
  if (s.n == 0) return;
  const char* de = getenv("KR_DIA");
  const int dia_mode = de ? atoi(de) : 1;
  const bool long_rows = (double)s.nnz >= kLongRow * (double)s.n;
  const bool dia_on = dia_mode == 2 || (dia_mode == 1 && long_rows);
  if (!dia_on && long_rows) return;
  if (!dia_on &&
      ((reinterpret_cast<uintptr_t>(s.val) | reinterpret_cast<uintptr_t>(s.col)) & 15))
    return;
  unsigned long long* table = nullptr;
  KR_HIP_CHECK(hipMalloc(&table, kOffTableBytes + 16));
  int* flags = reinterpret_cast<int*>(reinterpret_cast<char*>(table) + kOffTableBytes);
  launch_offsets(s.rowptr, s.rowptr64, s.n, s.col, s.pad, table, flags, s.stream);
  std::vector<unsigned long long> h(kOffTableBytes / 8);
  int hflags = 0;
  KR_HIP_CHECK(hipMemcpyAsync(h.data(), table, kOffTableBytes, hipMemcpyDeviceToHost, s.stream));
  KR_HIP_CHECK(hipMemcpyAsync(&hflags, flags, sizeof(int), hipMemcpyDeviceToHost, s.stream));
  KR_HIP_CHECK(hipStreamSynchronize(s.stream));
  KR_HIP_CHECK(hipFree(table));
  std::vector<int32_t> M;
  for (auto k : h)
    if (k) M.push_back((int32_t)((int64_t)k - (1ll << 32)));
  if (hflags || M.empty() || (int)M.size() > kMaxMaskBits) return;
  std::sort(M.begin(), M.end());
  const int nm = (int)M.size();
  const int mw = nm <= 8 ? 8 : nm <= 16 ? 16 : nm <= 32 ? 32 : 64;
  int32_t* dM = nullptr;
  void* mask = nullptr;
  KR_HIP_CHECK(hipMalloc(&dM, 64 * sizeof(int32_t)));
  KR_HIP_CHECK(hipMalloc(&mask, (size_t)s.n * (mw / 8)));
  s.owned.push_back(dM);
  s.owned.push_back(mask);
  fresh_fill(mask, (size_t)s.n * (mw / 8), s.stream);
  KR_HIP_CHECK(hipMemcpyAsync(dM, M.data(), nm * sizeof(int32_t), hipMemcpyHostToDevice, s.stream));
  launch_masks(s.rowptr, s.rowptr64, s.n, s.col, s.pad, dM, nm, mw, mask, s.stream);
  if (dia_on) {
    // Row-block-major (default): one contiguous nm x 256 chunk per row block,
    // so a workgroup reads one sequential stream. Offset-major (KR_DIA_LAYOUT=0,
    // A/B): nm streams, one per offset, n rows apart.
    const char* dl = getenv("KR_DIA_LAYOUT");
    const bool blocked = !(dl && atoi(dl) == 0);
    const int64_t nb = (s.n + kDiaRows - 1) / kDiaRows;
    const int64_t ld = nb * kDiaRows;
    double* dia = nullptr;
    if (hipMalloc(&dia, sizeof(double) * (size_t)nm * ld) != hipSuccess)
      throw Failure(KR_ERR_NOMEM, "diagonal-offset values: allocation failed");
    s.owned.push_back(dia);
    s.dia_bs = blocked ? (int64_t)nm * kDiaRows : kDiaRows;
    s.dia_ks = blocked ? kDiaRows : ld;
    KR_HIP_CHECK(hipMemsetAsync(dia, 0, sizeof(double) * (size_t)nm * ld, s.stream));
    launch_dia_fill(s.rowptr, s.rowptr64, s.n, s.col, s.val, s.pad, dM, nm, dia, s.dia_bs,
                    s.dia_ks, s.stream);
    s.dia = dia;
    plan_window(s, M);
    // symmetric offsets and values: lower entries read as the mirrored upper
    // ones (SpmvArgs::dia_sym; KR_DIA_SYM=0 disables, A/B)
    const char* se = getenv("KR_DIA_SYM");
    bool symM = blocked && nm % 2 == 1 && M[nm / 2] == 0;
    for (int k = 0; symM && k < nm; ++k) symM = M[k] == -M[nm - 1 - k];
    if (symM && !(se && atoi(se) == 0)) {
      int* flag = nullptr;
      KR_HIP_CHECK(hipMalloc(&flag, sizeof(int)));
      KR_HIP_CHECK(hipMemsetAsync(flag, 0, sizeof(int), s.stream));
      launch_dia_symcheck(mask, mw, s.n, dM, nm, dia, s.dia_bs, s.dia_ks, flag, s.stream);
      int h = 1;
      KR_HIP_CHECK(hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost, s.stream));
      KR_HIP_CHECK(hipStreamSynchronize(s.stream));
      KR_HIP_CHECK(hipFree(flag));
      s.dia_sym = h == 0 ? 1 : 0;
    }
    // the row-block walk with the mirrors in LDS (spmv_diawalk_kernel): every
    // mirror lies in this row block or the previous one (band <= 256 rows);
    // KR_DIA_WALK=0 keeps the strided kernel (A/B)
    const char* we = getenv("KR_DIA_WALK");
    if (s.dia_sym && M[nm - 1] <= kDiaRows && dia_walk_h_supported(nm / 2) &&
        !(we && atoi(we) == 0))
      s.dia_walk = 1;
    // The walk skips the mask loads of the longest run of full row blocks
    // (a band matrix: all but its first and last blocks; C5 -0.4 GB per
    // SpMV). KR_DIAW_FULLRUN=0 loads every mask (A/B).
    const char* fe = getenv("KR_DIAW_FULLRUN");
    if (s.dia_walk && !(fe && atoi(fe) == 0)) {
      uint8_t* dfull = nullptr;
      KR_HIP_CHECK(hipMalloc(&dfull, (size_t)nb));
      launch_dia_block_full(mask, mw, s.n, nm, dfull, s.stream);
      std::vector<uint8_t> full((size_t)nb);
      KR_HIP_CHECK(hipMemcpyAsync(full.data(), dfull, (size_t)nb, hipMemcpyDeviceToHost, s.stream));
      KR_HIP_CHECK(hipStreamSynchronize(s.stream));
      KR_HIP_CHECK(hipFree(dfull));
      int64_t best = 0, run = 0;
      for (int64_t b = 0; b < nb; ++b) {
        run = full[(size_t)b] ? run + 1 : 0;
        if (run > best) {
          best = run;
          s.dia_full_hi = b + 1;
          s.dia_full_lo = b + 1 - run;
        }
      }
    }
  }
  KR_HIP_CHECK(hipStreamSynchronize(s.stream));
  s.mask = mask;
  s.moff = dM;
  s.nm = nm;
  s.mw = mw;
  s.moff_h = M;
}

// Stencil codes (kr_stencil.h) for masked short-row blocks with a value
// dictionary whose offsets hold a +-W pair with W a multiple of 512 rows
// (3-D stencils: W = n^2), at most 8 offsets, other offsets within +-2 rows
// (LDS line) or even (one 16-byte load each, at most 4), and an even number
// of rows. Every row then streams 8 bytes (its codes); x[row - W] and x[row]
// are carried along the walk. KR_STENCIL=0 keeps the row walk (A/B).
void System::build_stencil(Shard& s) {
  const char* env = getenv("KR_STENCIL");
  if (env && atoi(env) == 0) return;
  if (!s.mask || s.dia || !s.vcode || s.ntab > 255 || s.nm > 8 || s.n < 2 || (s.n & 1) ||
      (s.pad & 1))
    return;
  const auto& M = s.moff_h;
  int64_t W = 0;
  for (int32_t o : M)
    if (o > 0 && o % kStencilBlock == 0 && std::find(M.begin(), M.end(), -o) != M.end())
      W = std::max<int64_t>(W, o);
  if (W == 0) return;
  // buffer loads take 32-bit byte offsets: every x offset the walk forms,
  // (ld + W + a block) doubles, stays below 2^31 bytes (kr_stencil.h SRes)
  if ((s.ld + W + 2 * kStencilBlock) * 8 >= (int64_t(1) << 31)) return;
  int nfar = 0;
  int32_t kind[8] = {}, far[4] = {};
  for (int k = 0; k < s.nm; ++k) {
    const int32_t o = M[k];
    if (o == 0) {
      kind[k] = 0;  // SK_CENTER
    } else if (o == -W) {
      kind[k] = 1;  // SK_PREV
    } else if (o == W) {
      kind[k] = 2;  // SK_NEXT
    } else if (o >= -2 && o <= 2) {
      kind[k] = 3;  // SK_NEAR (kSNear = 2)
    } else {
      if ((o & 1) || nfar == 4) return;
      far[nfar] = o;
      kind[k] = 4 + nfar++;  // SK_FAR + f
    }
  }
  uint64_t* code = nullptr;
  double* scratch = nullptr;
  if (hipMalloc(&code, sizeof(uint64_t) * (size_t)s.n) != hipSuccess ||
      hipMalloc(&scratch, 64 * sizeof(double)) != hipSuccess) {
    (void)hipGetLastError();
    if (code) (void)hipFree(code);
    return;  // no room: keep the row walk
  }
  s.owned.push_back(code);
  s.owned.push_back(scratch);
  s.scratch = scratch;
  fresh_fill(code, sizeof(uint64_t) * (size_t)s.n, s.stream);
  fresh_fill(scratch, 64 * sizeof(double), s.stream);
  launch_stencil_codes(s.rowptr, s.rowptr64, s.n, s.col, s.vcode, s.pad, s.moff, s.nm, code,
                       s.stream);
  // Narrow codes for the 7-point pattern (the kernel's compile-time slot
  // pattern kPat7): 2 bits per slot with <= 3 dictionary values (the Poisson
  // systems: 2 B per row instead of 8), 4 bits with <= 15. KR_STENCIL_CB=4/8
  // asks for at least that width (A/B).
  int cb = 8;
  const int32_t pat7[7] = {1, 4, 3, 0, 3, 5, 2};
  if (s.nm == 7 && nfar == 2 && std::equal(pat7, pat7 + 7, kind)) {
    const char* cenv = getenv("KR_STENCIL_CB");
    const int want = cenv ? atoi(cenv) : 2;
    cb = (want <= 2 && s.ntab <= 3) ? 2 : (want <= 4 && s.ntab <= 15) ? 4 : 8;
  }
  void* narrow = nullptr;
  if (cb < 8 && hipMalloc(&narrow, (size_t)cb * (size_t)s.n) != hipSuccess) {
    (void)hipGetLastError();
    narrow = nullptr;
    cb = 8;
  }
  if (narrow) {
    fresh_fill(narrow, (size_t)cb * (size_t)s.n, s.stream);
    launch_stencil_pack(code, s.n, cb, narrow, s.stream);
    KR_HIP_CHECK(hipStreamSynchronize(s.stream));
    s.owned.erase(std::find(s.owned.begin(), s.owned.end(), (void*)code));
    KR_HIP_CHECK(hipFree(code));
    s.owned.push_back(narrow);
    s.scode = narrow;
  } else {
    KR_HIP_CHECK(hipStreamSynchronize(s.stream));
    s.scode = code;
  }
  s.st_cb = cb;
  s.st_P = (int)(W / kStencilBlock);
  s.st_nfar = nfar;
  for (int k = 0; k < 8; ++k) s.st_kind[k] = kind[k];
  for (int f = 0; f < 4; ++f) s.st_far[f] = far[f];
  build_code_patterns(s);
  // the split SpMV's launches start on stencil row blocks
  s.int_lo = std::min<int64_t>((s.int_lo + kStencilBlock - 1) / kStencilBlock * kStencilBlock, s.n);
  s.int_hi = std::max<int64_t>(s.int_hi / kStencilBlock * kStencilBlock, s.int_lo);
}

// Code patterns of a stencil shard (SpmvArgs::st_pid): the distinct 512-row
// blocks of its code stream, each stored once, and one pattern id per block.
// A constant-coefficient stencil on a box has a handful (512^3 7-point: the
// interior line, 4 face lines, 4 edge lines -- 9), so the walk's codes come
// from a table that stays in L2 instead of 2 streamed bytes per row (C4: 0.27
// GB per SpMV). Exact: the blocks are compared byte for byte, rows past n
// are zero codes as the stream's range check reads them. More than
// kMaxPatterns distinct blocks, or KR_STENCIL_PATTERNS=0: the row stream.
void System::build_code_patterns(Shard& s) {
  constexpr int kMaxPatterns = 256;
  if (KR_ENV("KR_STENCIL_PATTERNS", 1) == 0 || !s.scode || s.n == 0) return;
  const int cb = s.st_cb;
  const size_t bb = (size_t)kStencilBlock * cb;  // bytes per row block
  const int64_t nb = (s.n + kStencilBlock - 1) / kStencilBlock;
  std::vector<uint8_t> h((size_t)nb * bb, 0);
  KR_HIP_CHECK(hipSetDevice(s.dev));
  KR_HIP_CHECK(hipMemcpy(h.data(), s.scode, (size_t)cb * (size_t)s.n, hipMemcpyDeviceToHost));
  std::unordered_map<std::string_view, uint32_t> ids;
  std::vector<uint32_t> pid((size_t)nb);
  std::vector<int64_t> first;  // a block holding each pattern
  for (int64_t b = 0; b < nb; ++b) {
    const std::string_view key(reinterpret_cast<const char*>(h.data()) + (size_t)b * bb, bb);
    auto it = ids.find(key);
    if (it == ids.end()) {
      if ((int)first.size() == kMaxPatterns) return;
      it = ids.emplace(key, (uint32_t)first.size()).first;
      first.push_back(b);
    }
    pid[(size_t)b] = it->second;
  }
  std::vector<uint8_t> tab(first.size() * bb);
  for (size_t q = 0; q < first.size(); ++q)
    std::memcpy(tab.data() + q * bb, h.data() + (size_t)first[q] * bb, bb);
  void* dtab = nullptr;
  uint32_t* dpid = nullptr;
  if (hipMalloc(&dtab, tab.size()) != hipSuccess ||
      hipMalloc(&dpid, sizeof(uint32_t) * pid.size()) != hipSuccess) {
    (void)hipGetLastError();
    if (dtab) (void)hipFree(dtab);
    return;  // no room: the row stream
  }
  s.owned.push_back(dtab);
  s.owned.push_back(dpid);
  KR_HIP_CHECK(hipMemcpy(dtab, tab.data(), tab.size(), hipMemcpyHostToDevice));
  KR_HIP_CHECK(hipMemcpy(dpid, pid.data(), sizeof(uint32_t) * pid.size(), hipMemcpyHostToDevice));
  s.st_pat = dtab;
  s.st_pid = dpid;
  s.st_npat = (int)first.size();
  build_box(s, h, pid, first);
}

// Constant-coefficient 7-point box stencil with n = 512 (Shard::st_box): the
// offsets -W, -512, -1, 0, +1, +512, +W (W = P 512-row lines per plane,
// whole planes), every present entry of slot k the same finite value st_v[k],
// and the absent entries exactly the box faces -- -W iff z = 0, -512 iff
// y = 0, -1 iff x = 0, +1 iff x = 511, +512 iff y = P-1, +W iff z = last
// (row = (z P + y) 512 + x). Checked on the code patterns: each pattern
// against the face class of a block holding it, then every block's class
// against its pattern's. The box pair (kr_pair.hip) reads absent operands
// as 0.0, which leaves a row sum unchanged, so it is bitwise the CSR rows.
// KR_BOX=0 disables.
void System::build_box(Shard& s, const std::vector<uint8_t>& h, const std::vector<uint32_t>& pid,
                       const std::vector<int64_t>& first) {
  s.st_box = false;
  if (KR_ENV("KR_BOX", 1) == 0) return;
  static const int32_t kPat[7] = {1, 4, 3, 0, 3, 5, 2};  // kPat7
  if (s.nm != 7 || s.st_nfar != 2 || !std::equal(kPat, kPat + 7, s.st_kind)) return;
  if (s.st_far[0] != -kStencilBlock || s.st_far[1] != kStencilBlock) return;
  const int64_t P = s.st_P, W = P * kStencilBlock;
  if (P < 2 || s.n % W != 0 || s.n / W < 2 || s.ntab <= 0) return;
  const int64_t planes = s.n / W;
  const int32_t want[7] = {(int32_t)-W, -kStencilBlock, -1, 0, 1, kStencilBlock, (int32_t)W};
  if (s.moff_h.size() != 7 || !std::equal(want, want + 7, s.moff_h.begin())) return;
  const int cb = s.st_cb;
  const uint64_t none = cb == 8 ? 0xFFull : (1ull << cb) - 1;
  auto code = [&](int64_t b, int x, int k) {  // slot k's code of row x of block b
    uint64_t w = 0;
    std::memcpy(&w, h.data() + ((size_t)b * kStencilBlock + x) * cb, cb);
    return (w >> (cb * k)) & none;
  };
  // face class of block b = (z, y): bits 0/1 z first/last, 2/3 y first/last
  auto cls = [&](int64_t b) {
    const int64_t z = b / P, y = b % P;
    return (z == 0 ? 1 : 0) | (z == planes - 1 ? 2 : 0) | (y == 0 ? 4 : 0) | (y == P - 1 ? 8 : 0);
  };
  uint64_t c[7];
  for (int k = 0; k < 7; ++k) c[k] = none;
  std::vector<int> pcls(first.size());
  for (size_t q = 0; q < first.size(); ++q) {
    const int f = cls(first[q]);
    pcls[q] = f;
    for (int x = 0; x < kStencilBlock; ++x) {
      const bool absent[7] = {(f & 1) != 0, (f & 4) != 0, x == 0, false, x == kStencilBlock - 1,
                              (f & 8) != 0, (f & 2) != 0};
      for (int k = 0; k < 7; ++k) {
        const uint64_t v = code(first[q], x, k);
        if (absent[k]) {
          if (v != none) return;
        } else {
          if (v == none) return;
          if (c[k] == none) c[k] = v;
          if (v != c[k]) return;
        }
      }
    }
  }
  for (int64_t b = 0; b < (int64_t)pid.size(); ++b)
    if (cls(b) != pcls[pid[(size_t)b]]) return;
  std::vector<double> tab((size_t)s.ntab);
  KR_HIP_CHECK(hipMemcpy(tab.data(), s.vtab, sizeof(double) * tab.size(), hipMemcpyDeviceToHost));
  for (int k = 0; k < 7; ++k) {
    if (c[k] == none || c[k] >= (uint64_t)s.ntab || !std::isfinite(tab[(size_t)c[k]])) return;
    s.st_v[k] = tab[(size_t)c[k]];
  }
  s.st_box = true;
}

// Stencil SpMV grid. Position-major (P % 8 == 0, the 3-D stencils): P
// positions x Zt plane segments (every segment start reloads CENTER and
// PREV: 2 planes per walk, so walks stay long). Plane-major (small P: 2-D and narrow
// bands): 8 XCDs x P positions x Z segments, at least 8 planes per segment.
// KR_STENCIL_Z fixes the segment count, KR_STENCIL_PM=0 forces plane-major.
bool stencil_pm(int P) {
  const char* env = getenv("KR_STENCIL_PM");
  if (env && atoi(env) == 0) return false;
  return P % 8 == 0;
}

int stencil_grid(int64_t rows, int P, int zmax = 0) {
  const int64_t nrb = (rows + kStencilBlock - 1) / kStencilBlock;
  const int64_t planes = (nrb + P - 1) / P;
  const bool pm = stencil_pm(P);
  const int64_t cols = pm ? P : 8 * (int64_t)P;  // workgroups per segment
  int64_t Z = 1;
  const char* env = getenv("KR_STENCIL_Z");
  if (env && atoi(env) > 0) {
    Z = atoi(env);
  } else if (pm) {
    // walks of >= 16 planes up to 16384 workgroups (512^3: 16384 x 16 planes,
    // +1.9 % over 4096 x 64 on C4 -- dual, head and step SpMVs faster, the
    // products-only dual slower; an 8-GPU slab of 64 planes: 2048 x 16, +3 %
    // over plane-major), then >= 8 planes up to 1024 workgroups (mid-size
    // cubes keep their parallelism)
    while (cols * Z < 16384 && planes / (Z * 2) >= 16) Z *= 2;
    while (cols * Z < 1024 && planes / (Z * 2) >= 8) Z *= 2;
  } else {
    while (cols * Z < 2048 && planes / (8 * Z * 2) >= 8) Z *= 2;
  }
  if (zmax > 0 && Z > zmax) Z = zmax;
  return (int)(cols * Z);
}

void System::build_vdict(Shard& s) {
  const char* env = getenv("KR_VDICT");
  if (env && atoi(env) == 0) return;
  // Only the row walk v2 reads codes: short rows, no DIA values, 16-byte
  // aligned val/col, >= 4 entries (the v2 host conditions in spmv_dispatch_epi).
  if (s.n == 0 || s.dense || s.dia || s.nnz < 8) return;
  if ((double)s.nnz >= kLongRow * (double)s.n) return;
  if ((reinterpret_cast<uintptr_t>(s.val) | reinterpret_cast<uintptr_t>(s.col)) & 15) return;
  unsigned long long* gtab = nullptr;
  const size_t tb = kVdGlobal * sizeof(unsigned long long);
  KR_HIP_CHECK(hipMalloc(&gtab, tb + 16));
  int* flags = reinterpret_cast<int*>(reinterpret_cast<char*>(gtab) + tb);
  launch_vdict_collect(s.val + s.nz0, s.nnz, gtab, flags, s.stream);
  std::vector<unsigned long long> h(kVdGlobal);
  int hflags[2] = {0, 0};
  KR_HIP_CHECK(hipMemcpyAsync(h.data(), gtab, tb, hipMemcpyDeviceToHost, s.stream));
  KR_HIP_CHECK(hipMemcpyAsync(hflags, flags, sizeof(hflags), hipMemcpyDeviceToHost, s.stream));
  KR_HIP_CHECK(hipStreamSynchronize(s.stream));
  std::vector<unsigned long long> keys;
  for (auto k : h)
    if (k != ~0ull) keys.push_back(k);
  if (hflags[0] || keys.empty() || (int)keys.size() > kVdMax) {
    KR_HIP_CHECK(hipFree(gtab));
    return;
  }
  std::sort(keys.begin(), keys.end());
  const int nk = (int)keys.size();
  // vcode (indexed like val) must be 8-byte aligned with readable bytes on
  // both sides: windows start at (first entry) & ~7 and load 8 codes per lane.
  // Either allocation failing (or a pattern the encode pass cannot find)
  // leaves the shard on the 8-byte values, with nothing half built.
  const int64_t pre = 8 + (s.nz0 & 7);
  double* tab = nullptr;
  uint8_t* code = nullptr;
  if (hipMalloc(&tab, kVdMax * sizeof(double)) != hipSuccess ||
      hipMalloc(&code, (size_t)(pre + s.nnz + 16)) != hipSuccess) {
    (void)hipGetLastError();
    if (tab) (void)hipFree(tab);
    (void)hipFree(gtab);
    return;  // no room for the dictionary: keep the 8-byte values
  }
  // the sorted keys (bit patterns) double as the value table
  KR_HIP_CHECK(hipMemcpyAsync(gtab, keys.data(), nk * sizeof(unsigned long long),
                              hipMemcpyHostToDevice, s.stream));
  KR_HIP_CHECK(hipMemcpyAsync(tab, keys.data(), nk * sizeof(unsigned long long),
                              hipMemcpyHostToDevice, s.stream));
  KR_HIP_CHECK(hipMemsetAsync(code, 0, (size_t)(pre + s.nnz + 16), s.stream));
  launch_vdict_encode(s.val + s.nz0, s.nnz, gtab, nk, code + pre, flags, s.stream);
  int miss = 0;
  KR_HIP_CHECK(hipMemcpyAsync(&miss, flags, sizeof(int), hipMemcpyDeviceToHost, s.stream));
  KR_HIP_CHECK(hipStreamSynchronize(s.stream));
  KR_HIP_CHECK(hipFree(gtab));
  if (miss) {  // a value outside the table: the codes would be wrong
    (void)hipFree(code);
    (void)hipFree(tab);
    return;
  }
  s.owned.push_back(code);
  s.owned.push_back(tab);
  s.vcode = code + pre - s.nz0;  // indexed like val
  s.vtab = tab;
  s.ntab = nk;
}

void System::finalize() {
  KR_REQUIRE(!finalized, "system already finalized");
  const int P = nglobal_shards();
  const int nranks = comm ? comm->nranks : 1;
  // 1. column range of every local block
  for (auto& s : shards) {
    if (s.dense) {  // every row reaches every column
      s.col_lo = s.n > 0 ? 0 : s.row0;
      s.col_hi = s.n > 0 ? n_global - 1 : s.row0 + s.n - 1;
      s.nnz = s.n * n_global;
      continue;
    }
    KR_REQUIRE(s.rowptr && s.col && s.val, "matrix of a shard is not set");
    KR_HIP_CHECK(hipSetDevice(s.dev));
    int64_t* d = nullptr;
    KR_HIP_CHECK(hipMalloc(&d, 2 * sizeof(int64_t)));
    launch_col_minmax(s.rowptr, s.rowptr64, s.n, s.col, d, s.stream);
    int64_t h[2];
    KR_HIP_CHECK(hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s.stream));
    KR_HIP_CHECK(hipStreamSynchronize(s.stream));
    KR_HIP_CHECK(hipFree(d));
    if (s.n == 0 || h[0] == INT64_MAX) {
      s.col_lo = s.row0;
      s.col_hi = s.row0 + s.n - 1;
    } else {
      s.col_lo = std::min(h[0], s.row0);
      s.col_hi = std::max(h[1], s.row0 + s.n - 1);
    }
    KR_REQUIRE(s.col_lo >= 0 && s.col_hi < n_global, "column index out of range");
    // nnz
    if (s.rowptr64) {
      int64_t e[2];
      KR_HIP_CHECK(hipMemcpy(&e[0], s.rowptr, 8, hipMemcpyDeviceToHost));
      KR_HIP_CHECK(hipMemcpy(&e[1], (const int64_t*)s.rowptr + s.n, 8, hipMemcpyDeviceToHost));
      s.nnz = e[1] - e[0];
      s.nz0 = e[0];
    } else {
      int32_t e[2];
      KR_HIP_CHECK(hipMemcpy(&e[0], s.rowptr, 4, hipMemcpyDeviceToHost));
      KR_HIP_CHECK(hipMemcpy(&e[1], (const int32_t*)s.rowptr + s.n, 4, hipMemcpyDeviceToHost));
      s.nnz = (int64_t)e[1] - e[0];
      s.nz0 = e[0];
    }
  }
  // 2. everybody's needed range [lo, hi]
  std::vector<int64_t> lo(P), hi(P);
  if (comm) {
    // every rank's local shards, kMaxLocal (lo, hi) pairs per rank
    Shard& s = shards[0];
    const int R = comm->nranks;
    constexpr int W = 2 * kMaxLocal;
    KR_HIP_CHECK(hipSetDevice(s.dev));
    int64_t* d = nullptr;
    KR_HIP_CHECK(hipMalloc(&d, (size_t)W * (1 + R) * sizeof(int64_t)));
    std::vector<int64_t> mine(W, 0);
    for (size_t li = 0; li < shards.size(); ++li) {
      mine[2 * li] = shards[li].col_lo;
      mine[2 * li + 1] = shards[li].col_hi;
    }
    KR_HIP_CHECK(hipMemcpy(d, mine.data(), W * sizeof(int64_t), hipMemcpyHostToDevice));
    KR_NCCL_CHECK(ncclAllGather(d, d + W, W, ncclInt64, comm->nccl, s.stream));
    std::vector<int64_t> all((size_t)W * R);
    KR_HIP_CHECK(hipMemcpyAsync(all.data(), d + W, all.size() * 8, hipMemcpyDeviceToHost,
                                s.stream));
    KR_HIP_CHECK(hipStreamSynchronize(s.stream));
    KR_HIP_CHECK(hipFree(d));
    for (int t = 0; t < P; ++t) {
      const int r = owner[t], l = t - rank_first[r];
      lo[t] = all[(size_t)W * r + 2 * l];
      hi[t] = all[(size_t)W * r + 2 * l + 1];
    }
  } else {
    for (int t = 0; t < P; ++t) {
      lo[t] = shards[t].col_lo;
      hi[t] = shards[t].col_hi;
    }
  }
  // 3. halo geometry and exchange plan
  for (size_t li = 0; li < shards.size(); ++li) {
    Shard& s = shards[li];
    const int me = first_global + (int)li;
    s.halo_lo = s.row0 - s.col_lo;
    s.halo_hi = s.col_hi - (s.row0 + s.n - 1);
    s.pad = (s.halo_lo + 7) / 8 * 8;
    s.ld = s.pad + s.n + s.halo_hi;
    s.ld = (s.ld + 7) / 8 * 8;
    KR_REQUIRE(s.ld < (int64_t)INT32_MAX, "shard too large for 32-bit local columns");
    plan_halo(P, part.data(), lo.data(), hi.data(), me, s.recv, s.send);
    if (!comm) {
      for (auto& p : s.recv) p.peer -= first_global;
      s.send.clear();
    }
    // with a communicator the peers stay global shard indices: a peer owned
    // by this rank is a device copy (halo_hybrid), any other RCCL
    // 4. interior rows (every column owned), computed on global columns
    KR_HIP_CHECK(hipSetDevice(s.dev));
    if (s.dense) {  // no interior rows when there are other shards
      const bool alone = P == 1;
      s.int_lo = 0;
      s.int_hi = alone ? s.n : 0;
      s.reach = n_global;
    } else {
      int64_t* d = nullptr;
      KR_HIP_CHECK(hipMalloc(&d, 3 * sizeof(int64_t)));
      launch_interior(s.rowptr, s.rowptr64, s.n, s.col, s.row0, s.row0 + s.n - 1, d, s.stream);
      int64_t h[3];
      KR_HIP_CHECK(hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s.stream));
      KR_HIP_CHECK(hipStreamSynchronize(s.stream));
      KR_HIP_CHECK(hipFree(d));
      // Interior rows, shrunk to whole row blocks so that the two boundary
      // ranges are whole blocks too and run as ONE launch (SpmvArgs::rb_gap).
      s.int_lo = std::min<int64_t>((h[0] + kBlock - 1) / kBlock * kBlock, s.n);
      s.int_hi = std::max<int64_t>(h[1] / kBlock * kBlock, s.int_lo);
      s.reach = h[2];
      // Slab schedule (A/B only, KR_SLAB=S row blocks per plane): keeps x
      // rows one reach apart (3-D stencils) closer in time; measured 5-15 %
      // slower than the contiguous sweep on MI355X.
      const char* env = getenv("KR_SLAB");
      s.slab = env ? atoll(env) : 0;  // measured slower than the contiguous sweep
      if (s.slab < 8) s.slab = 0;
      const char* sub = getenv("KR_SLAB_SUB");
      s.slab_sub = sub ? atoll(sub) : 0;
    }
    if (!s.comm_stream) {
      // The halo exchange is on the critical path of every split SpMV (the
      // boundary rows wait for it) while the interior launch fills the GPU:
      // its queue gets the highest priority, so the command processor
      // dispatches the RCCL / copy work ahead of the interior workgroups
      // still waiting for a slot. KR_COMM_PRIORITY=0: default priority (A/B).
      int lo = 0, hi = 0;
      KR_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      const char* env = getenv("KR_COMM_PRIORITY");
      const bool prio = !(env && atoi(env) == 0);
      KR_HIP_CHECK(hipStreamCreateWithPriority(&s.comm_stream, hipStreamNonBlocking,
                                               prio ? hi : 0));
    }
    if (!s.ev_in) KR_HIP_CHECK(hipEventCreateWithFlags(&s.ev_in, hipEventDisableTiming));
    if (!s.ev_out) KR_HIP_CHECK(hipEventCreateWithFlags(&s.ev_out, hipEventDisableTiming));
    if (!s.dense) {
      // 5. rewrite columns to local numbering: local = global - row0 + pad
      launch_col_shift(s.rowptr, s.rowptr64, s.n, s.col, s.pad - s.row0, s.stream);
      // 6. offset masks for short-row blocks whose rows use at most 64 distinct
      // column offsets (stencils, banded): the SpMV then reads a 1-8 byte mask
      // per row instead of a 4-byte column per entry. KR_MASK=0 disables.
      build_masks(s);
      // 6b. value dictionary for short-row blocks with <= 256 distinct values
      // (stencils): 1-byte codes instead of 8-byte values. KR_VDICT=0 disables.
      build_vdict(s);
      // 6c. stencil codes (one uint64 per row) for 3-D-stencil blocks with a
      // dictionary: the stencil SpMV (kr_stencil.h). KR_STENCIL=0 disables.
      build_stencil(s);
    }
    // 7. reduction buffers
    s.grid = default_grid(s.n);
    // dense: one wave per row, 4 rows per workgroup
    s.spmv_grid = s.dense ? (int)std::max<int64_t>(1, std::min<int64_t>((s.n + 3) / 4,
                                                                         (int64_t)grid_cap() * 4))
                  : s.scode    ? stencil_grid(s.n, s.st_P)
                  : s.dia_walk ? dia_walk_grid(s.n, s.nm)
                               : spmv_grid_for(s.n, s.reach);
    // The products-only dual (a read-only stream: codes and two x vectors)
    // runs faster on fewer, longer walks: 512^3 0.69 -> 0.59 ms at Z <= 16
    // (16 or 8 alike, 32 is the general grid's). Smaller shards already have
    // Z <= 16, so only >= 512-plane shards change; position-major walks
    // (3-D stencils) only, the measured case. KR_PO_ZMAX=0: the general grid.
    {
      const char* ze = getenv("KR_PO_ZMAX");
      const int zmax = ze ? atoi(ze) : 16;
      s.spmv_grid_po = s.scode && zmax > 0 && stencil_pm(s.st_P)
                           ? stencil_grid(s.n, s.st_P, zmax) : s.spmv_grid;
    }
    // The fused basis pair (spmv_stencil2_kernel) walks longer segments on
    // >= 512-plane shards: every segment start re-walks 3 planes (64-plane
    // segments: 5 %; the general grid's 16: 19 %). Smaller shards keep the
    // general grid, so the products' summation order there is the two dual
    // launches' (the GPU-order oracle stays exact). KR_ST2_Z caps the segments.
    {
      const char* ze = getenv("KR_ST2_Z");
      const int z2 = ze ? atoi(ze) : 8;
      const int64_t planes = s.scode && s.st_P > 0 ? s.n / ((int64_t)s.st_P * kStencilBlock) : 0;
      s.spmv_grid2 = s.scode && stencil_pm(s.st_P) && planes >= 512 && z2 > 0
                         ? stencil_grid(s.n, s.st_P, z2) : s.spmv_grid;
    }
    s.pstride = std::max(s.grid, s.spmv_grid);
    s.slot_n.fill(0);
    KR_HIP_CHECK(hipMalloc(&s.partials, sizeof(double) * (size_t)kMaxSlots * s.pstride));
    fresh_fill(s.partials, sizeof(double) * (size_t)kMaxSlots * s.pstride, s.stream, 0);
    KR_HIP_CHECK(hipMalloc(&s.slots, sizeof(double) * kMaxSlots));
    fresh_fill(s.slots, sizeof(double) * kMaxSlots, s.stream);
    // RCCL ranks' (or, on the first shard, in-process shards') slot totals
    const size_t gbytes = sizeof(double) * kMaxSlots * std::max<size_t>(nranks, shards.size());
    KR_HIP_CHECK(hipMalloc(&s.gather, gbytes));
    fresh_fill(s.gather, gbytes, s.stream);
    KR_HIP_CHECK(hipHostMalloc(&s.host, sizeof(double) * kMaxSlots * nranks, 0));
    if (!s.ev_a) KR_HIP_CHECK(hipEventCreateWithFlags(&s.ev_a, hipEventDisableTiming));
    if (!s.ev_b) KR_HIP_CHECK(hipEventCreateWithFlags(&s.ev_b, hipEventDisableTiming));
    KR_HIP_CHECK(hipStreamSynchronize(s.stream));
  }
  if (hybrid()) {  // reduce(): the local slot totals, gathered over the ranks
    Shard& s0 = shards[0];
    // staging on the communicator's device for the RCCL pieces of shards
    // on other devices (halo_hybrid)
    // KR_HYBRID_STAGE=1 stages every RCCL piece (test hook: exercises the
    // path on a one-GPU box)
    const char* fe = getenv("KR_HYBRID_STAGE");
    const bool force = fe && atoi(fe) != 0;
    for (auto& t : shards) {
      if (t.dev == s0.dev && !force) continue;
      KR_HIP_CHECK(hipSetDevice(s0.dev));
      for (auto* list : {&t.send, &t.recv})
        for (auto& p : *list)
          if (owner[p.peer] != comm->rank && p.count > 0) {
            KR_HIP_CHECK(hipMalloc(&p.stage, sizeof(double) * 3 * (size_t)p.count));
            fresh_fill(p.stage, sizeof(double) * 3 * (size_t)p.count, s0.stream);
          }
    }
    KR_HIP_CHECK(hipSetDevice(s0.dev));
    KR_HIP_CHECK(hipMalloc(&hy_send, sizeof(double) * kMaxLocal * kMaxSlots));
    KR_HIP_CHECK(hipMemset(hy_send, 0, sizeof(double) * kMaxLocal * kMaxSlots));
    KR_HIP_CHECK(hipMalloc(&hy_recv, sizeof(double) * kMaxLocal * kMaxSlots * nranks));
    fresh_fill(hy_recv, sizeof(double) * kMaxLocal * kMaxSlots * nranks, s0.stream);
    KR_HIP_CHECK(hipStreamSynchronize(s0.stream));
    KR_HIP_CHECK(hipHostMalloc(&hy_host, sizeof(double) * kMaxLocal * kMaxSlots * nranks, 0));
    if (!hy_ev) KR_HIP_CHECK(hipEventCreateWithFlags(&hy_ev, hipEventDisableTiming));
  }
  // in-process: the shards whose comm streams copy halo rows from each shard
  // (the boundary launch of a shard waits for their copies before its later
  // kernels may overwrite those rows)
  if (!comm) {
    for (auto& s : shards) {
      s.readers.clear();
      s.ext_readers.clear();
      s.ext_in = false;
    }
    for (size_t li = 0; li < shards.size(); ++li)
      for (auto& p : shards[li].recv) {
        Shard& t = shards[(size_t)p.peer];
        auto& r = t.readers;
        if (std::find(r.begin(), r.end(), (int)li) == r.end()) r.push_back((int)li);
        if (t.stream != shards[li].stream) {
          shards[li].ext_in = true;
          auto& x = t.ext_readers;
          if (std::find(x.begin(), x.end(), (int)li) == x.end()) x.push_back((int)li);
        }
      }
  }
  // stream groups (kr_system_create shares a device's stream between its
  // in-process shards): shards in order within a group, groups in order of
  // their first shard
  groups.clear();
  for (size_t li = 0; li < shards.size(); ++li) {
    size_t g = 0;
    while (g < groups.size() && shards[(size_t)groups[g][0]].stream != shards[li].stream) ++g;
    if (g == groups.size()) groups.emplace_back();
    shards[li].lead = groups[g].empty();
    groups[g].push_back((int)li);
  }
  for (auto& g : gslots) {
    if (g.dev) (void)hipFree(g.dev);
    if (g.host) (void)hipHostFree(g.host);
  }
  gslots.assign(groups.size(), GroupSlots{});
  for (size_t g = 0; g < groups.size(); ++g) {
    if (comm || groups[g].size() < 2 || groups[g].size() > (size_t)kGroupMax) continue;
    const size_t bytes = sizeof(double) * kMaxSlots * groups[g].size();
    KR_HIP_CHECK(hipSetDevice(shards[(size_t)groups[g][0]].dev));
    KR_HIP_CHECK(hipMalloc(&gslots[g].dev, bytes));
    fresh_fill(gslots[g].dev, bytes, shards[(size_t)groups[g][0]].stream);
    KR_HIP_CHECK(hipHostMalloc(&gslots[g].host, bytes, 0));
  }
  // The split SpMV needs interior rows on every shard; with RCCL ranks the
  // decision is global, so the summation order (interior + boundary partials)
  // is the one of the same partition in one process (oracle/gpu_order.py).
  all_interior = true;
  for (auto& s : shards) all_interior = all_interior && s.int_lo < s.int_hi;
  if (comm && comm->nranks > 1) {
    Shard& s0 = shards[0];
    KR_HIP_CHECK(hipSetDevice(s0.dev));
    int64_t* d = nullptr;
    KR_HIP_CHECK(hipMalloc(&d, sizeof(int64_t) * (1 + nranks)));
    const int64_t mine = all_interior ? 1 : 0;
    KR_HIP_CHECK(hipMemcpy(d, &mine, sizeof(int64_t), hipMemcpyHostToDevice));
    KR_NCCL_CHECK(ncclAllGather(d, d + 1, 1, ncclInt64, comm->nccl, s0.stream));
    std::vector<int64_t> all(nranks);
    KR_HIP_CHECK(hipMemcpyAsync(all.data(), d + 1, sizeof(int64_t) * nranks,
                                hipMemcpyDeviceToHost, s0.stream));
    KR_HIP_CHECK(hipStreamSynchronize(s0.stream));
    KR_HIP_CHECK(hipFree(d));
    for (int64_t f : all) all_interior = all_interior && f != 0;
  }
  // one host thread per further in-process stream group (KR_HOST_THREADS=0:
  // every shard's work enqueued by the calling thread, A/B)
  {
    const char* ht = getenv("KR_HOST_THREADS");
    if (!comm && groups.size() > 1 && !(ht && atoi(ht) == 0))
      pool = std::make_unique<ShardPool>((int)groups.size() - 1);
  }
  {
    const char* env = getenv("KR_OVERLAP");  // 0 disables the split SpMV (A/B)
    overlap = !(env && atoi(env) == 0);
    const char* pe = getenv("KR_PRODUCTS_ONLY");  // 0: store every basis vector (A/B)
    products_only_on = !(pe && atoi(pe) == 0);
    const char* fz = getenv("KR_FUSE");  // 0: separate vector-step kernels (A/B)
    // Fusion pays for the short-row (row-walk) kernel: C4 +6 %. With the
    // product-then-sum kernel (long rows) the fused SpMV costs more than the
    // separate vector pass (C5: +0.9 ms vs +0.5 ms), so long rows keep it.
    bool long_rows = false;  // long rows on the product-then-sum kernel (no DIA)
    for (auto& s : shards)
      if (s.n > 0 && !s.dia && (double)s.nnz >= kLongRow * (double)s.n) long_rows = true;
    fuse_steps = fz ? atoi(fz) != 0 : !long_rows;
    // Own-row epilogue operands loaded at the row end (default) or at the
    // row-block start (KR_EPI_LATE=0): late measured 1-3 % faster on C4.
    const char* el = getenv("KR_EPI_LATE");
    epi_late = el ? atoi(el) != 0 : 1;
    // Steps 0 and 1 in one SpMV: row walk v2 only (short rows, 16-byte
    // aligned CSR with >= 4 entries, no dense shard, no forced v1 kernel).
    const char* ff = getenv("KR_FUSE_FIRST");
    const char* sv = getenv("KR_SPMV_VARIANT");
    bool v2 = true;  // every shard on the DIA kernel or the row walk v2
    for (auto& s : shards) {
      if (s.dia) continue;
      if (s.dense || s.nnz < 4 || (sv && atoi(sv) != 10 && atoi(sv) != 12 && atoi(sv) != 13) ||
          ((reinterpret_cast<uintptr_t>(s.val) | reinterpret_cast<uintptr_t>(s.col)) & 15))
        v2 = false;
    }
    // Long rows on the DIA kernel: forming r1 at each of ~60 gathered columns
    // per row costs more than one vector pass (C5: 8.97 ms vs 0.54 + 6.32 ms,
    // +3.6 %), so they keep the step-0 vector kernel unless KR_FUSE_FIRST=1;
    // with the x window in LDS, r1 is formed once per column instead.
    bool long_dia = false;
    for (auto& s : shards)
      if (s.n > 0 && s.dia && s.dia_wlen == 0 && (double)s.nnz >= kLongRow * (double)s.n)
        long_dia = true;
    fuse_first = fuse_steps && !long_rows && v2 &&
                 (ff ? atoi(ff) != 0 : !long_dia);
  }
  finalized = true;
}

void System::alloc_vectors(int count) {
  for (auto& s : shards) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    KR_HIP_CHECK(hipStreamSynchronize(s.stream));
    for (double* v : s.vec_base) KR_HIP_CHECK(hipFree(v));
    s.vec.assign(count, nullptr);
    s.vec_base.assign(count, nullptr);
    // KR_VEC_STAGGER (bytes, a multiple of 256): vector i's rows start i x
    // that far into its allocation, so the vectors a walk streams together
    // do not share their low address bits
    const int64_t stagger = KR_ENV("KR_VEC_STAGGER", 0);
    KR_REQUIRE(stagger >= 0 && stagger % 256 == 0, "KR_VEC_STAGGER: a multiple of 256 bytes");
    for (int i = 0; i < count; ++i) {
      const size_t off = (size_t)stagger * (size_t)i;
      if (hipMalloc(&s.vec_base[i], sizeof(double) * (size_t)s.ld + off) != hipSuccess)
        throw Failure(KR_ERR_NOMEM, "vector allocation failed");
      s.vec[i] = s.vec_base[i] + off / sizeof(double);
      // zeros (NaN under KR_POISON_ALLOC): pad and halo rows included, so a
      // halo row read before its exchange, or a pad row read as an operand,
      // is a NaN in the poison run. x0 = 0 is written explicitly (load_bx).
      fresh_fill(s.vec[i], sizeof(double) * (size_t)s.ld, s.stream, 0);
    }
    KR_HIP_CHECK(hipStreamSynchronize(s.stream));
  }
}

void System::prof_begin(Shard& s, const char* name, hipEvent_t& t0) {
  (void)name;
  t0 = nullptr;
  if (!profile || !prof_active) return;
  if (s.event_pool.empty()) {
    hipEvent_t e;
    KR_HIP_CHECK(hipEventCreate(&e));
    s.event_pool.push_back(e);
  }
  t0 = s.event_pool.back();
  s.event_pool.pop_back();
  KR_HIP_CHECK(hipEventRecord(t0, s.stream));
}

void System::prof_end(Shard& s, const char* name, hipEvent_t t0, double bytes, int nsh) {
  if (!profile || !t0) return;
  if (s.event_pool.empty()) {
    hipEvent_t e;
    KR_HIP_CHECK(hipEventCreate(&e));
    s.event_pool.push_back(e);
  }
  hipEvent_t t1 = s.event_pool.back();
  s.event_pool.pop_back();
  KR_HIP_CHECK(hipEventRecord(t1, s.stream));
  s.pending.push_back({name, t0, t1, bytes, nsh});
}

// The k-th window of a kernel name on every shard of the first shard's
// device belongs to the k-th call of that op (a shard records every call of
// an op or none: group leads record the SpMVs of their group, every shard
// its vector kernels, shard 0 the scalar steps). One call's time is its
// device window, from the earliest begin to the latest end of those shards'
// events (events of one device compare across streams), and its bytes are
// theirs summed: so a call reads the same whether its shards share one
// stream (one window per group) or run on a stream each (overlapping
// windows), and the rate bytes / time is the device's.
void System::harvest_profile() {
  if (!profile) return;
  const int dev0 = shards.empty() ? 0 : shards[0].dev;
  std::map<std::string, std::vector<std::vector<const Shard::Pending*>>> by;
  for (size_t li = 0; li < shards.size(); ++li) {
    const Shard& s = shards[li];
    if (s.dev != dev0) continue;
    for (const auto& p : s.pending) {
      auto& lists = by[p.name];
      lists.resize(shards.size());
      lists[li].push_back(&p);
    }
  }
  for (auto& kv : by) {
    size_t calls = 0;
    for (const auto& l : kv.second) calls = std::max(calls, l.size());
    for (size_t k = 0; k < calls; ++k) {
      hipEvent_t ref = nullptr;
      float lo = 0.f, hi = 0.f;
      double bytes = 0.0;
      int64_t nsh = 0;
      for (const auto& l : kv.second) {
        if (k >= l.size()) continue;
        const Shard::Pending* p = l[k];
        KR_HIP_CHECK(hipEventSynchronize(p->t1));
        float b = 0.f, e = 0.f;
        if (!ref) {
          ref = p->t0;
          KR_HIP_CHECK(hipEventElapsedTime(&e, ref, p->t1));
          lo = 0.f;
          hi = e;
        } else {
          KR_HIP_CHECK(hipEventElapsedTime(&b, ref, p->t0));
          KR_HIP_CHECK(hipEventElapsedTime(&e, ref, p->t1));
          lo = std::min(lo, b);
          hi = std::max(hi, e);
        }
        bytes += p->bytes;
        nsh += p->nsh;
      }
      auto& st = kstats[kv.first];
      st.launches += 1;
      st.total_ms += (double)(hi - lo);
      st.bytes = bytes;
      st.shards = nsh;
    }
  }
  for (auto& s : shards) {
    for (auto& p : s.pending) {
      if (s.dev != dev0) KR_HIP_CHECK(hipEventSynchronize(p.t1));
      s.event_pool.push_back(p.t0);
      s.event_pool.push_back(p.t1);
    }
    s.pending.clear();
  }
}

// Several local shards with a communicator: halo pieces from a shard of this
// rank are device copies (as in-process), the others RCCL send/recv, all of
// them on the first local shard's stream (one RCCL rank per process). Both
// sides of a rank pair list their transfers in one order -- vector, then
// receiving global shard, then sending global shard -- so the RCCL
// send/recv pairs match.
void System::halo_hybrid(int id1, int id2, int id3, bool async) {
  Shard& s0 = shards[0];
  auto stream_of = [&](Shard& s) { return async ? s.comm_stream : s.stream; };
  const int me = comm->rank;
  for (auto& s : shards) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    if (!async) KR_HIP_CHECK(hipEventRecord(s.ev_a, s.stream));
  }
  auto ready = [&](Shard& s) { return async ? s.ev_in : s.ev_a; };
  // local pieces: device copies on the receiving shard's stream
  for (auto& s : shards) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    hipStream_t st = stream_of(s);
    if (async) KR_HIP_CHECK(hipStreamWaitEvent(st, s.ev_in, 0));
    for (auto& p : s.recv) {
      if (owner[p.peer] != me) continue;
      Shard& t = shards[p.peer - first_global];
      KR_HIP_CHECK(hipStreamWaitEvent(st, ready(t), 0));
      for (int id : {id1, id2, id3}) {
        if (id < 0) continue;
        double* dst = s.vec[id] + s.local_index(p.g0);
        const double* src = t.vec[id] + t.local_index(p.g0);
        if (s.dev == t.dev)
          KR_HIP_CHECK(hipMemcpyAsync(dst, src, 8 * (size_t)p.count, hipMemcpyDeviceToDevice, st));
        else
          KR_HIP_CHECK(hipMemcpyPeerAsync(dst, s.dev, src, t.dev, 8 * (size_t)p.count, st));
      }
    }
    KR_HIP_CHECK(hipEventRecord(async ? s.ev_out : s.ev_b, st));
  }
  // remote pieces: one RCCL group on the first shard's stream
  struct Xfer {
    int recv_shard, send_shard, peer_rank;
    double* ptr;
    int64_t count;
  };
  std::vector<Xfer> sends, recvs;
  for (size_t li = 0; li < shards.size(); ++li) {
    Shard& s = shards[li];
    const int g = first_global + (int)li;
    for (auto& p : s.send)
      if (owner[p.peer] != me) sends.push_back({p.peer, g, owner[p.peer], nullptr, p.count});
    for (auto& p : s.recv)
      if (owner[p.peer] != me) recvs.push_back({g, p.peer, owner[p.peer], nullptr, p.count});
  }
  auto by_pair = [](const Xfer& a, const Xfer& b) {
    return a.recv_shard != b.recv_shard ? a.recv_shard < b.recv_shard
                                        : a.send_shard < b.send_shard;
  };
  std::sort(sends.begin(), sends.end(), by_pair);
  std::sort(recvs.begin(), recvs.end(), by_pair);
  KR_HIP_CHECK(hipSetDevice(s0.dev));
  hipStream_t st0 = stream_of(s0);
  if (!sends.empty() || !recvs.empty()) {
    for (auto& s : shards) KR_HIP_CHECK(hipStreamWaitEvent(st0, ready(s), 0));
    auto piece = [&](std::vector<HaloPiece>& list, int peer) -> HaloPiece& {
      return *std::find_if(list.begin(), list.end(),
                           [&](const HaloPiece& p) { return p.peer == peer; });
    };
    int slot = 0;  // vector slot of the staging buffers (<= 3 vectors)
    for (int id : {id1, id2, id3}) {  // pieces of shards on other devices: stage out
      if (id < 0) continue;
      for (auto& x : sends) {
        Shard& s = shards[x.send_shard - first_global];
        HaloPiece& p = piece(s.send, x.recv_shard);
        if (p.stage)
          KR_HIP_CHECK(hipMemcpyPeerAsync(p.stage + slot * p.count, s0.dev,
                                          s.vec[id] + s.local_index(p.g0), s.dev,
                                          8 * (size_t)p.count, st0));
      }
      ++slot;
    }
    KR_NCCL_CHECK(ncclGroupStart());
    slot = 0;
    for (int id : {id1, id2, id3}) {
      if (id < 0) continue;
      for (auto& x : sends) {
        Shard& s = shards[x.send_shard - first_global];
        HaloPiece& p = piece(s.send, x.recv_shard);
        const double* src = p.stage ? p.stage + slot * p.count : s.vec[id] + s.local_index(p.g0);
        KR_NCCL_CHECK(ncclSend(src, (size_t)p.count, ncclFloat64, x.peer_rank, comm->nccl, st0));
      }
      for (auto& x : recvs) {
        Shard& s = shards[x.recv_shard - first_global];
        HaloPiece& p = piece(s.recv, x.send_shard);
        double* dst = p.stage ? p.stage + slot * p.count : s.vec[id] + s.local_index(p.g0);
        KR_NCCL_CHECK(ncclRecv(dst, (size_t)p.count, ncclFloat64, x.peer_rank, comm->nccl, st0));
      }
      ++slot;
    }
    KR_NCCL_CHECK(ncclGroupEnd());
    slot = 0;
    for (int id : {id1, id2, id3}) {  // staged pieces in
      if (id < 0) continue;
      for (auto& x : recvs) {
        Shard& s = shards[x.recv_shard - first_global];
        HaloPiece& p = piece(s.recv, x.send_shard);
        if (p.stage)
          KR_HIP_CHECK(hipMemcpyPeerAsync(s.vec[id] + s.local_index(p.g0), s.dev,
                                          p.stage + slot * p.count, s0.dev,
                                          8 * (size_t)p.count, st0));
      }
      ++slot;
    }
  }
  KR_HIP_CHECK(hipEventRecord(hy_ev, st0));
  if (async) return;  // spmv() makes every shard wait for every ev_out and hy_ev
  // Nobody reads or overwrites a vector before every transfer is done.
  for (auto& t : shards) {
    KR_HIP_CHECK(hipSetDevice(t.dev));
    KR_HIP_CHECK(hipStreamWaitEvent(t.stream, hy_ev, 0));
    for (auto& s : shards)
      if (&s != &t) KR_HIP_CHECK(hipStreamWaitEvent(t.stream, s.ev_b, 0));
  }
}

void System::halo(int id1, int id2, int id3) {
  if (hybrid()) {
    halo_hybrid(id1, id2, id3, false);
    return;
  }
  if (comm) {
    Shard& s = shards[0];
    if (s.recv.empty() && s.send.empty()) return;
    hipEvent_t t0 = nullptr;
    prof_begin(s, "halo", t0);
    double bytes = 0;
    KR_HIP_CHECK(hipSetDevice(s.dev));
    KR_NCCL_CHECK(ncclGroupStart());
    for (int id : {id1, id2, id3}) {
      if (id < 0) continue;
      for (auto& p : s.send) {
        KR_NCCL_CHECK(ncclSend(s.vec[id] + s.local_index(p.g0), (size_t)p.count, ncclFloat64,
                               p.peer, comm->nccl, s.stream));
        bytes += 8.0 * p.count;
      }
      for (auto& p : s.recv) {
        KR_NCCL_CHECK(ncclRecv(s.vec[id] + s.local_index(p.g0), (size_t)p.count, ncclFloat64,
                               p.peer, comm->nccl, s.stream));
        bytes += 8.0 * p.count;
      }
    }
    KR_NCCL_CHECK(ncclGroupEnd());
    prof_end(s, "halo", t0, bytes);
    return;
  }
  if (shards.size() < 2) return;
  for (auto& s : shards) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    KR_HIP_CHECK(hipEventRecord(s.ev_a, s.stream));
  }
  for (auto& s : shards) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    for (auto& p : s.recv) {
      Shard& t = shards[p.peer];
      KR_HIP_CHECK(hipStreamWaitEvent(s.stream, t.ev_a, 0));
      for (int id : {id1, id2, id3}) {
        if (id < 0) continue;
        double* dst = s.vec[id] + s.local_index(p.g0);
        const double* src = t.vec[id] + t.local_index(p.g0);
        if (s.dev == t.dev)
          KR_HIP_CHECK(hipMemcpyAsync(dst, src, 8 * (size_t)p.count, hipMemcpyDeviceToDevice,
                                      s.stream));
        else
          KR_HIP_CHECK(hipMemcpyPeerAsync(dst, s.dev, src, t.dev, 8 * (size_t)p.count, s.stream));
      }
    }
    KR_HIP_CHECK(hipEventRecord(s.ev_b, s.stream));
  }
  // Nobody overwrites a vector before every reader has copied its halo.
  for (auto& t : shards) {
    KR_HIP_CHECK(hipSetDevice(t.dev));
    for (auto& s : shards)
      if (&s != &t) KR_HIP_CHECK(hipStreamWaitEvent(t.stream, s.ev_b, 0));
  }
}

void System::halo_async(int id1, int id2, int id3) {
  if (hybrid()) {
    halo_hybrid(id1, id2, id3, true);
    return;
  }
  if (comm) {
    Shard& s = shards[0];
    KR_HIP_CHECK(hipSetDevice(s.dev));
    KR_HIP_CHECK(hipStreamWaitEvent(s.comm_stream, s.ev_in, 0));
    KR_NCCL_CHECK(ncclGroupStart());
    for (int id : {id1, id2, id3}) {
      if (id < 0) continue;
      for (auto& p : s.send)
        KR_NCCL_CHECK(ncclSend(s.vec[id] + s.local_index(p.g0), (size_t)p.count, ncclFloat64,
                               p.peer, comm->nccl, s.comm_stream));
      for (auto& p : s.recv)
        KR_NCCL_CHECK(ncclRecv(s.vec[id] + s.local_index(p.g0), (size_t)p.count, ncclFloat64,
                               p.peer, comm->nccl, s.comm_stream));
    }
    KR_NCCL_CHECK(ncclGroupEnd());
    KR_HIP_CHECK(hipEventRecord(s.ev_out, s.comm_stream));
    return;
  }
  for (auto& g : groups) halo_group(g, id1, id2, id3);
  for (auto& s : shards) halo_in_process(s, id1, id2, id3);
}

// One in-process shard's part of halo_async: its comm stream copies its halo
// rows from the peers after their ev_in, then records ev_out. Touches only
// this shard's streams (the per-shard host threads run it concurrently).
void System::halo_in_process(Shard& s, int id1, int id2, int id3) {
  // pieces from shards on s's own stream: halo_group (the group's gather)
  if (!s.ext_in) return;
  KR_HIP_CHECK(hipSetDevice(s.dev));
  // The copies overwrite s's halo rows: s's own earlier kernels (the
  // previous SpMV's boundary rows read the same halo when consecutive SpMVs
  // share an input vector) must be done first, not only the peer's.
  KR_HIP_CHECK(hipStreamWaitEvent(s.comm_stream, s.ev_in, 0));
  // Peers on this device: one gather launch for every piece (KR_HALO_KERNEL=0:
  // a hipMemcpyAsync per piece); peers on other devices: peer copies.
  const bool gather = KR_ENV("KR_HALO_KERNEL", 1) != 0;
  HaloGatherArgs g;
  for (auto& p : s.recv) {
    Shard& t = shards[p.peer];
    if (t.stream == s.stream) continue;
    KR_HIP_CHECK(hipStreamWaitEvent(s.comm_stream, t.ev_in, 0));
    for (int id : {id1, id2, id3}) {
      if (id < 0) continue;
      double* dst = s.vec[id] + s.local_index(p.g0);
      const double* src = t.vec[id] + t.local_index(p.g0);
      if (s.dev == t.dev && gather && g.n < kHaloPieces) {
        g.src[g.n] = src;
        g.dst[g.n] = dst;
        g.count[g.n] = p.count;
        ++g.n;
      } else if (s.dev == t.dev) {
        KR_HIP_CHECK(hipMemcpyAsync(dst, src, 8 * (size_t)p.count, hipMemcpyDeviceToDevice,
                                    s.comm_stream));
      } else {
        KR_HIP_CHECK(hipMemcpyPeerAsync(dst, s.dev, src, t.dev, 8 * (size_t)p.count,
                                        s.comm_stream));
      }
    }
  }
  launch_halo_gather(g, s.comm_stream);  // after every wait above
  KR_HIP_CHECK(hipEventRecord(s.ev_out, s.comm_stream));
}

// The halo pieces a stream group's shards take from each other, in ONE gather
// launch on the group's stream (up to kHaloPieces pieces per launch): stream
// order alone puts it after the producers of the source rows and the readers
// of the destination rows (every earlier kernel of the group), and before the
// boundary launches that read it -- no events, no comm stream.
void System::halo_group(const std::vector<int>& grp, int id1, int id2, int id3) {
  Shard& s0 = shards[(size_t)grp[0]];
  KR_HIP_CHECK(hipSetDevice(s0.dev));
  // KR_HALO_KERNEL=0 (A/B, as in halo_in_process): one device copy per piece
  // on the group's stream instead of the one gather launch
  const bool gather = KR_ENV("KR_HALO_KERNEL", 1) != 0;
  HaloGatherArgs g;
  for (int li : grp) {
    Shard& s = shards[(size_t)li];
    for (auto& p : s.recv) {
      Shard& t = shards[p.peer];
      if (t.stream != s.stream) continue;
      for (int id : {id1, id2, id3}) {
        if (id < 0) continue;
        if (!gather) {
          KR_HIP_CHECK(hipMemcpyAsync(s.vec[id] + s.local_index(p.g0),
                                      t.vec[id] + t.local_index(p.g0),
                                      sizeof(double) * (size_t)p.count,
                                      hipMemcpyDeviceToDevice, s0.stream));
          continue;
        }
        if (g.n == kHaloPieces) {
          launch_halo_gather(g, s0.stream);
          g = HaloGatherArgs{};
        }
        g.src[g.n] = t.vec[id] + t.local_index(p.g0);
        g.dst[g.n] = s.vec[id] + s.local_index(p.g0);
        g.count[g.n] = p.count;
        ++g.n;
      }
    }
  }
  if (gather) launch_halo_gather(g, s0.stream);
}

void System::spmv(SpmvEpi epi, int in1, int in2, int out1, int out2, int e, int b,
                  int slot0, const StepOps* st) {
  const bool dual = (epi == EPI_DUAL_NONE || epi == EPI_DUAL_MRR || epi == EPI_DUAL_KCG);
  const bool virt = epi == EPI_STEP_MRR_FIRST2 || epi == EPI_MRR_V;
  const bool vp = epi == EPI_XY_VP;  // CG's virtual p (System::spmv_vp)
  KR_REQUIRE(!vp || (in2 >= 0 && st && st->u1 >= 0 && st->u1 != in1 && st->u1 != in2 &&
                     vp_pro.sop == SC_CG_BETA),
             "virtual-p SpMV: r / p output missing or aliased, or no scalar step");
  const bool step = (epi == EPI_STEP_MRR_NOX || epi == EPI_STEP_MRR_X2 ||
                     epi == EPI_STEP_MRR_X || epi == EPI_STEP_KCG || virt);
  KR_REQUIRE(!step || (st && st->u1 >= 0 && st->u2 >= 0 && out1 != in1),
             "fused step: operands missing or output aliases the input");
  const bool step_x = (epi == EPI_STEP_MRR_X2 || epi == EPI_STEP_MRR_X || virt);
  KR_REQUIRE(!step_x || (st->us >= 0 && st->ud >= 0), "fused step: x operands missing");
  KR_REQUIRE(!virt || (in2 >= 0 && st->x3 >= 0 && st->u1 != in2 && st->u1 != st->x3),
             "fused first step: y0/Ar1 missing or y written over a gathered input");
  const int hx2 = (dual || virt || vp) ? in2 : -1;  // vectors whose halo the SpMV reads
  const int hx3 = virt ? st->x3 : -1;
  KR_REQUIRE(slot0 + spmv_products(epi) <= kMaxSlots, "reduction slots exhausted");
  // one decision for every shard of every rank (the same summation order as
  // the partition in one process), even where a shard has no halo piece
  const bool exchange = nglobal_shards() > 1;
  // Split SpMV: the halo exchange runs on a side stream while the interior
  // rows (no halo column) are multiplied; the boundary rows follow it. The
  // boundary launches ADD their reduction partials to the interior launch's
  // (same stream, fixed order: deterministic).
  const bool split = exchange && overlap && all_interior;
  // products only: every SpMV kernel skips the y1/y2 stores of a dual whose
  // outputs nobody reads (the stencil walk by its own flag, every other
  // kernel in epi_store_row*: the row walks, the DIA kernels and their walk,
  // the dense one; own stat name, and 16 N fewer bytes). Round 5: for every
  // format, not only the stencil and the windowed DIA kernel -- stores mixed
  // into the read stream cost ~3x their bytes (plain CSR dual at 512^3: 0.72
  // of 3.3 ms for 2.15 GB; the C5 walk: 0.45-0.6 ms for 0.8 GB).
  bool po = products_only && products_only_on && dual;
  auto po_shard = [&](const Shard& s) { (void)s; return po; };
  bool po_any = false;
  for (auto& s : shards) po_any = po_any || po_shard(s);
  const char* nm = po_any ? epi_name_po(epi) : epi_name(epi);

  auto args_for = [&](Shard& s, int64_t r_begin, int64_t rows, int grid, int acc) {
    SpmvArgs a;
    a.rowptr = s.rowptr64 ? (const void*)((const int64_t*)s.rowptr + r_begin)
                          : (const void*)((const int32_t*)s.rowptr + r_begin);
    a.rowptr64 = s.rowptr64;
    a.col = s.col;
    a.val = s.val;
    a.n = rows;
    a.x1 = s.vec[in1];
    a.x2 = (dual || virt || vp) ? s.vec[in2] : nullptr;
    a.xoff = s.pad + r_begin;
    a.y1 = s.own(out1) + r_begin;
    a.y2 = (dual || epi == EPI_MRR_V) ? s.own(out2) + r_begin : nullptr;
    a.b = b >= 0 ? s.own(b) + r_begin : nullptr;
    a.e = e >= 0 ? s.own(e) + r_begin : nullptr;
    a.partials = s.partials + (size_t)slot0 * s.pstride;
    a.grid = grid;
    a.long_rows = s.n > 0 && (double)s.nnz >= kLongRow * (double)s.n;
    a.accumulate = acc;
    a.slab = s.slab;
    a.slab_sub = s.slab_sub;
    if (s.mask) {
      a.mask = static_cast<const char*>(s.mask) + r_begin * (s.mw / 8);
      a.moff = s.moff;
      a.nm = s.nm;
      a.mw = s.mw;
      if (s.dia) {
        KR_REQUIRE(r_begin % kDiaRows == 0, "DIA launch must start on a row block");
        a.dia = s.dia + (r_begin / kDiaRows) * s.dia_bs;
        a.dia_bs = s.dia_bs;
        a.dia_ks = s.dia_ks;
        a.dia_sym = s.dia_sym;
        a.dia_walk = s.dia_walk;
        if (s.dia_walk && s.dia_full_hi > s.dia_full_lo) {
          // launch-relative, whole blocks of this launch only
          const int64_t rb = r_begin / kDiaRows;
          a.full_lo = std::max<int64_t>(s.dia_full_lo - rb, 0);
          a.full_hi = std::min<int64_t>(s.dia_full_hi - rb, rows / kDiaRows);
          if (a.full_hi < a.full_lo) a.full_hi = a.full_lo;
        }
        a.dia_wlen = s.dia_wlen;
        a.nseg = s.nseg;
        for (int g = 0; g < s.nseg; ++g) {
          a.seg_lo[g] = s.seg_lo[g];
          a.seg_len[g] = s.seg_len[g];
          a.seg_base[g] = s.seg_base[g];
        }
        a.woff = s.woff;
        a.xlen = s.ld;
      }
    }
    if (s.vcode) {
      a.vcode = s.vcode;
      a.vtab = s.vtab;
      a.ntab = s.ntab;
    }
    if (s.scode) {
      KR_REQUIRE(r_begin % kStencilBlock == 0, "stencil launch must start on a row block");
      a.scode = static_cast<const char*>(s.scode) + r_begin * s.st_cb;
      a.st_cb = s.st_cb;
      if (s.st_pid) {
        a.st_pid = s.st_pid + r_begin / kStencilBlock;
        a.st_pat = s.st_pat;
        a.st_npat = s.st_npat;
      }
      a.st_P = s.st_P;
      a.st_pm = stencil_pm(s.st_P) ? 1 : 0;
      a.st_nm = s.nm;
      a.st_nfar = s.st_nfar;
      for (int k = 0; k < 8; ++k) {
        a.st_off[k] = k < s.nm ? s.moff_h[k] : 0;
        a.st_kind[k] = s.st_kind[k];
      }
      for (int f = 0; f < 4; ++f) a.st_far[f] = s.st_far[f];
      a.xlen = s.ld;
      a.scratch = s.scratch;
    }
    a.epi_late = epi_late;
    a.products_only = po_shard(s) ? 1 : 0;
    a.stop = dev_stop ? s.st + ST_STOP : nullptr;
    a.nnz_total = s.nnz;
    // Non-temporal matrix stream and result stores: the row walks of large
    // shards (variant 13: a plain-CSR dual at 512^3 -5 %; C1's 64k rows,
    // whose vectors stay in L2/MALL for the next kernel, lost 8 % with them).
    // Only the row walk reads the flag -- the DIA kernels keep plain stores
    // (C3 / C5 neutral as an A/B build, profiles/r05b/dia_nts) -- so a DIA
    // shard's short-row launches that fall back to the row walk (no x window)
    // get variant 13 like any large shard. KR_NT_STORES=0/1 forces either.
    {
      const int e = KR_ENV("KR_NT_STORES", -1);
      a.nt_stores = e >= 0 ? e : s.n >= ((int64_t)1 << 22) ? 1 : 0;
    }
    if (s.dense) {
      a.dense = 1;
      a.val = s.dense + r_begin * s.dld;
      a.dld = s.dld;
      a.ncols = n_global;
      a.xcol0 = s.pad - s.row0;  // local index of global column 0
    }
    if (vp) {
      a.x3 = s.vec[in2];  // not read by the formula; gathered beside x2 by the row walks
      a.u1 = s.own(st->u1) + r_begin;
      a.pro = (int)SC_CG_BETA + 1;
      a.pro_part = s.partials;
      a.pro_stride = s.pstride;
      for (int q = 0; q < 5; ++q) a.pro_cnt[q] = s.slot_n[q];
      a.st = s.st;
      a.pro_it = vp_pro.it;
      a.pro_h = vp_pro.h;
      a.pro_par = vp_pro.par;
      a.pro_thr = vp_pro.thr;
    }
    if (step) {
      a.u1 = s.own(st->u1) + r_begin;
      a.u2 = s.own(st->u2) + r_begin;
      if (step_x) {
        a.us = s.own(st->us) + r_begin;
        a.ud = s.own(st->ud) + r_begin;
      }
      a.c0 = st->c0;
      a.c1 = st->c1;
      if (virt) {
        a.x3 = s.vec[st->x3];
        a.c2 = st->c2;
        a.c3 = st->c3;
        a.xpend = st->xpend;
      }
      if (epi == EPI_MRR_V && st->pro) {  // SC_MRR_ZETA from the EW_MRR_S partials
        a.pro = (int)SC_MRR_ZETA + 1;
        a.pro_part = s.partials;
        a.pro_stride = s.pstride;
        for (int q = 0; q < 5; ++q) a.pro_cnt[q] = s.slot_n[q];
        a.st = s.st;
      }
    }
    return a;
  };
  auto bytes_of = [&](Shard& s) {
    const double nv = dual ? 2.0 : 1.0;
    // fused step: u1, u2 read and written (+ x read and written)
    // fused first step: inputs r0, y0, Ar1 (3 x 8N, one counted below as
    // x), z and x read, y z r x written
    const double extra = vp ? 16.0 * s.n  // r gathered, p stored
                         : virt ? 64.0 * s.n
                         : step ? (step_x ? 48.0 : 32.0) * s.n
                                : (b >= 0 || e >= 0) ? 8.0 * s.n : 0.0;
    if (s.dense) return 8.0 * s.nnz + nv * 8.0 * (n_global + s.n) + extra;
    const double stores = po_shard(s) ? 0.0 : nv * 8.0 * s.n;  // y1 (, y2)
    return 12.0 * s.nnz + (s.rowptr64 ? 8.0 : 4.0) * (s.n + 1) + nv * 8.0 * s.n + stores + extra;
  };
  // The partial stride is s.pstride for every launch; the full / interior
  // launch writes s.spmv_grid partials per product, the boundary launch (fewer
  // blocks) adds into the first entries.
  const int np = spmv_products(epi);
  auto grid_of = [&](const Shard& s) { return po_shard(s) ? s.spmv_grid_po : s.spmv_grid; };
  // KR_ZIGZAG=1 (A/B): stencil walks alternate their dispatch order launch by
  // launch, so each starts on the plane segments the previous kernel streamed
  // last. Bitwise neutral; measured neutral on C4 (522.3 vs 522.1 it/s, same
  // box, three pairs: the first-steps kernel +2.5 %, the others -0.5-1 %).
  const bool zigzag = KR_ENV("KR_ZIGZAG", 0) != 0;
  auto launch_full = [&](Shard& s, int64_t r_begin, int64_t rows) {
    SpmvArgs a = args_for(s, r_begin, rows, s.pstride, 0);
    if (s.scode && zigzag) {
      a.st_rev = s.st_flip;
      s.st_flip ^= 1;
    }
    launch_spmv_grid(epi, a, grid_of(s), s.stream);
    for (int p = 0; p < np; ++p) s.slot_n[slot0 + p] = grid_of(s);
  };

  if (!split) {
    halo(in1, hx2, hx3);
    for (auto& s : shards) {
      KR_HIP_CHECK(hipSetDevice(s.dev));
      hipEvent_t t0 = nullptr;
      prof_begin(s, nm, t0);
      launch_full(s, 0, s.n);
      prof_end(s, nm, t0, bytes_of(s));
    }
    return;
  }
  std::vector<hipEvent_t> t0s(shards.size(), nullptr);
  const bool wait_all = KR_ENV("KR_BOUNDARY_WAIT_ALL", 0) != 0;
  auto phase_in =[&](Shard& s, size_t li) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    prof_begin(s, nm, t0s[li]);
    KR_HIP_CHECK(hipEventRecord(s.ev_in, s.stream));
  };
  // both boundary ranges in one launch: row blocks [0, int_lo/B) and
  // [int_hi/B, end) (interior bounds are whole blocks, see finalize); the
  // boundary launch adds its partials to the interior launch's
  auto launch_boundary = [&](Shard& s) {
    const int64_t rbs = s.scode ? kStencilBlock : kBlock;  // rows per row block
    const int64_t nb_lo = s.int_lo / rbs, nb_gap = (s.int_hi - s.int_lo) / rbs;
    const int64_t nb_all = (s.n + rbs - 1) / rbs;
    if (nb_all - nb_gap > 0) {
      SpmvArgs ab = args_for(s, 0, s.n, s.pstride, 1);
      ab.rb_gap_at = nb_lo;
      ab.rb_gap = nb_gap;
      // (the stencil kernel's boundary launch spreads its blocks over the grid)
      const int g = (int)std::min<int64_t>(grid_of(s), nb_all - nb_gap);
      launch_spmv_grid(epi, ab, g, s.stream);
    }
  };
  if (!comm) {
    // In-process shards: three phases, stream group by stream group (on the
    // host threads when there are several groups: a phase waits on events the
    // previous one recorded on OTHER groups' streams, so the phases are
    // separated by the pool's barrier). Within a group (shards sharing a
    // stream) stream order is the only edge: one gather launch moves the
    // pieces the group's shards take from each other, then the interior
    // launches, then (phase 3) the boundary launches. Pieces from other
    // streams go through the receiving shard's comm stream between ev_in and
    // ev_out as before. Profiling: one window per group, on its first shard.
    for_shards([&](Shard& s, size_t li) {
      KR_HIP_CHECK(hipSetDevice(s.dev));
      if (s.lead) prof_begin(s, nm, t0s[li]);
      if (s.ext_in || !s.ext_readers.empty()) KR_HIP_CHECK(hipEventRecord(s.ev_in, s.stream));
    });
    for_groups([&](const std::vector<int>& grp) {
      halo_group(grp, in1, hx2, hx3);
      for (int li : grp) halo_in_process(shards[(size_t)li], in1, hx2, hx3);
      for (int li : grp) {
        Shard& s = shards[(size_t)li];
        KR_HIP_CHECK(hipSetDevice(s.dev));
        launch_full(s, s.int_lo, s.int_hi - s.int_lo);  // interior rows
      }
    });
    for_groups([&](const std::vector<int>& grp) {
      double bytes = 0;
      for (int li : grp) {
        Shard& s = shards[(size_t)li];
        KR_HIP_CHECK(hipSetDevice(s.dev));
        // own halo copied by the comm stream, and every shard on another
        // stream that copies from this one done reading its rows (the next
        // kernels may overwrite them)
        if (s.ext_in) KR_HIP_CHECK(hipStreamWaitEvent(s.stream, s.ev_out, 0));
        if (wait_all) {  // KR_BOUNDARY_WAIT_ALL=1 (debug A/B): the round-2 edge set
          for (auto& t : shards)
            if (t.ext_in) KR_HIP_CHECK(hipStreamWaitEvent(s.stream, t.ev_out, 0));
        } else {
          for (int t : s.ext_readers)
            KR_HIP_CHECK(hipStreamWaitEvent(s.stream, shards[(size_t)t].ev_out, 0));
        }
        launch_boundary(s);
        bytes += bytes_of(s);
      }
      Shard& s0 = shards[(size_t)grp[0]];
      KR_HIP_CHECK(hipSetDevice(s0.dev));
      prof_end(s0, nm, t0s[(size_t)grp[0]], bytes, (int)grp.size());
    });
    return;
  }
  // With a communicator (one host thread): ev_in, the exchange on the comm
  // stream(s) (RCCL), interior launches, then each boundary launch after the
  // exchange.
  for (size_t li = 0; li < shards.size(); ++li) phase_in(shards[li], li);
  halo_async(in1, hx2, hx3);
  for (auto& s : shards) {  // interior rows: all blocks write their partials
    KR_HIP_CHECK(hipSetDevice(s.dev));
    launch_full(s, s.int_lo, s.int_hi - s.int_lo);
  }
  for (size_t li = 0; li < shards.size(); ++li) {
    Shard& s = shards[li];
    KR_HIP_CHECK(hipSetDevice(s.dev));
    if (!hybrid()) {
      KR_HIP_CHECK(hipStreamWaitEvent(s.stream, s.ev_out, 0));
    } else {
      // own halo copied, and every reader done with this shard's rows
      for (auto& t : shards) KR_HIP_CHECK(hipStreamWaitEvent(s.stream, t.ev_out, 0));
      KR_HIP_CHECK(hipStreamWaitEvent(s.stream, hy_ev, 0));  // RCCL pieces
    }
    launch_boundary(s);
    prof_end(s, nm, t0s[li], bytes_of(s));
  }
}

void System::ew(EwOp op, double c0, double c1, std::array<int, 6> ids, int slot0) {
  std::array<int, kEwOps> all;
  all.fill(-1);
  for (int q = 0; q < 6; ++q) all[q] = ids[q];
  ew_n(op, c0, c1, all, slot0);
}

void System::ew_n(EwOp op, double c0, double c1, const std::array<int, kEwOps>& ids,
                  int slot0) {
  KR_REQUIRE(slot0 + ew_products(op) <= kMaxSlots, "reduction slots exhausted");
  for_shards([&](Shard& s, size_t) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    EwArgs a;
    a.c0 = c0;
    a.c1 = c1;
    for (int q = 0; q < kEwOps; ++q) a.p[q] = ids[q] >= 0 ? s.own(ids[q]) : nullptr;
    a.n = s.n;
    a.partials = s.partials + (size_t)slot0 * s.pstride;
    a.grid = s.grid;
    a.stride = s.pstride;
    for (int p = 0; p < ew_products(op); ++p) s.slot_n[slot0 + p] = s.grid;
    hipEvent_t t0 = nullptr;
    const char* nm = ew_name(op);
    prof_begin(s, nm, t0);
    launch_ew(op, a, s.stream);
    prof_end(s, nm, t0, 8.0 * ew_vectors(op) * s.n);
  });
}

bool System::device_scalars() const {
  if (KR_ENV("KR_DEVICE_SCALARS", 1) == 0) return false;  // one host sync per reduction (A/B)
  // one shard per RCCL rank, or any number of shards in one process
  return comm ? !hybrid() : true;
}

void System::scalar_state_init(double gamma) {
  Shard& s0 = shards[0];
  for (auto& s : shards) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    if (!s.st) {
      KR_HIP_CHECK(hipMalloc(&s.st, sizeof(double) * kScalarState));
      fresh_fill(s.st, sizeof(double) * kScalarState, s.stream);
    }
  }
  KR_HIP_CHECK(hipSetDevice(s0.dev));
  if (!s0.hst) KR_HIP_CHECK(hipHostMalloc(&s0.hst, sizeof(double) * kScalarState, 0));
  KR_HIP_CHECK(hipStreamSynchronize(s0.stream));  // hst is free
  for (int q = 0; q < kScalarState; ++q) s0.hst[q] = 0.0;
  s0.hst[ST_GAMMA] = gamma;
  for (auto& s : shards) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    KR_HIP_CHECK(hipMemcpyAsync(s.st, s0.hst, sizeof(double) * kScalarState,
                                hipMemcpyHostToDevice, s.stream));
  }
  KR_HIP_CHECK(hipSetDevice(s0.dev));
  KR_HIP_CHECK(hipStreamSynchronize(s0.stream));  // hst is rewritten by the next init
  for (auto& s : shards) KR_HIP_CHECK(hipStreamSynchronize(s.stream));
}

void System::ew_dev(EwOp op, int coef, std::array<int, 6> ids, int slot0) {
  KR_REQUIRE(slot0 + ew_products(op) <= kMaxSlots, "reduction slots exhausted");
  for (auto& s : shards) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    EwArgs a;
    for (int q = 0; q < 6; ++q) a.p[q] = ids[q] >= 0 ? s.own(ids[q]) : nullptr;
    a.n = s.n;
    a.partials = s.partials + (size_t)slot0 * s.pstride;
    a.grid = s.grid;
    a.stride = s.pstride;
    a.cdev = s.st + coef;
    a.stop = dev_stop ? s.st + ST_STOP : nullptr;
    for (int p = 0; p < ew_products(op); ++p) s.slot_n[slot0 + p] = s.grid;
    hipEvent_t t0 = nullptr;
    const char* nm = ew_name(op);
    prof_begin(s, nm, t0);
    launch_ew(op, a, s.stream);
    prof_end(s, nm, t0, 8.0 * ew_vectors(op) * s.n);
  }
}

void System::scalar(ScalarOp op, int need, int64_t it, int h, double thr, int check) {
  Shard& s = shards[0];
  ScalarArgs a;
  a.op = op;
  a.need = need;
  a.partials = s.partials;
  a.stride = s.pstride;
  for (int q = 0; q < 5; ++q) a.cnt[q] = s.slot_n[q];
  a.st = s.st;
  a.it = it;
  a.h = h;
  a.check = check;
  a.thr = thr;
  const int nslots = 32 - __builtin_clz((unsigned)need);
  if (comm) {
    // every rank: its slot totals (finalize order), all-gathered on the
    // compute stream (after this SpMV's halo, before the next one's: one
    // RCCL order on every rank), then the same scalar step everywhere
    KR_HIP_CHECK(hipSetDevice(s.dev));
    SlotCounts cnt{};
    for (int q = 0; q < nslots; ++q) cnt.n[q] = s.slot_n[q];
    launch_finalize_counts(s.partials, s.pstride, cnt, nslots, s.slots, s.stream);
    KR_NCCL_CHECK(ncclAllGather(s.slots, s.gather, (size_t)nslots, ncclFloat64, comm->nccl,
                                s.stream));
    a.gathered = s.gather;
    a.nranks = comm->nranks;
    a.gstride = nslots;
  } else if (shards.size() > 1) {
    // in-process shards: each one's slot totals (finalize order) side by
    // side on the first shard, summed there in shard order like reduce()
    for (auto& t : shards) {
      KR_HIP_CHECK(hipSetDevice(t.dev));
      SlotCounts cnt{};
      for (int q = 0; q < nslots; ++q) cnt.n[q] = t.slot_n[q];
      launch_finalize_counts(t.partials, t.pstride, cnt, nslots, t.slots, t.stream);
      KR_HIP_CHECK(hipEventRecord(t.ev_a, t.stream));
    }
    KR_HIP_CHECK(hipSetDevice(s.dev));
    for (size_t li = 0; li < shards.size(); ++li) {
      Shard& t = shards[li];
      KR_HIP_CHECK(hipStreamWaitEvent(s.stream, t.ev_a, 0));
      KR_HIP_CHECK(hipMemcpyPeerAsync(s.gather + li * nslots, s.dev, t.slots, t.dev,
                                      sizeof(double) * nslots, s.stream));
    }
    a.gathered = s.gather;
    a.nranks = (int)shards.size();
    a.gstride = nslots;
  }
  KR_HIP_CHECK(hipSetDevice(s.dev));
  hipEvent_t t0 = nullptr;
  prof_begin(s, "scalar", t0);
  launch_scalar(a, s.stream);
  prof_end(s, "scalar", t0, 8.0 * s.pstride * __builtin_popcount(need));
  if (!comm && shards.size() > 1) {
    // the coefficients and the stop flag to every other shard (its vector
    // kernels read its own copy); st[ST_HIST...] stays on the first shard
    KR_HIP_CHECK(hipEventRecord(s.ev_b, s.stream));
    for (size_t li = 1; li < shards.size(); ++li) {
      Shard& t = shards[li];
      KR_HIP_CHECK(hipSetDevice(t.dev));
      KR_HIP_CHECK(hipStreamWaitEvent(t.stream, s.ev_b, 0));
      KR_HIP_CHECK(hipMemcpyPeerAsync(t.st, t.dev, s.st, s.dev, sizeof(double) * ST_HIST,
                                      t.stream));
    }
  }
}

bool System::fused_scalars() const {
  if (KR_ENV("KR_FUSE_SCALAR", 1) == 0) return false;
  return !comm && shards.size() == 1;
}

bool System::vp_ok() const {
  if (KR_ENV("KR_CG_VP", 1) == 0) return false;
  if (!fused_scalars()) return false;
  const Shard& s = shards[0];
  if (s.dense || s.n == 0) return false;
  if (s.scode || s.dia) return true;
  // the row walk v2 (16-byte aligned val/col, >= 4 entries, short rows)
  const bool vec = ((reinterpret_cast<uintptr_t>(s.val) | reinterpret_cast<uintptr_t>(s.col)) &
                    15) == 0;
  return vec && s.nnz >= 4 && (double)s.nnz < kLongRow * (double)s.n;
}

void System::spmv_vp(int p_old, int r, int out, int p_new, int64_t it, int h, int par,
                     double thr) {
  vp_pro.sop = SC_CG_BETA;
  vp_pro.it = it;
  vp_pro.h = h;
  vp_pro.par = par;
  vp_pro.thr = thr;
  StepOps st;
  st.u1 = p_new;
  spmv(EPI_XY_VP, p_old, r, out, -1, -1, -1, 3, &st);
  vp_pro.sop = -1;
}

void System::ew_pro(EwOp op, ScalarOp sop, std::array<int, 6> ids, int slot0, int64_t it, int h,
                    int par, double thr, int s1, int alpha) {
  KR_REQUIRE(slot0 + ew_products(op) <= kMaxSlots, "reduction slots exhausted");
  Shard& s = shards[0];
  KR_HIP_CHECK(hipSetDevice(s.dev));
  EwArgs a;
  for (int q = 0; q < 6; ++q) a.p[q] = ids[q] >= 0 ? s.own(ids[q]) : nullptr;
  a.n = s.n;
  a.partials = s.partials + (size_t)slot0 * s.pstride;
  a.grid = s.grid;
  a.stride = s.pstride;
  a.stop = dev_stop ? s.st + ST_STOP : nullptr;
  a.pro = (int)sop + 1;
  a.pro_part = s.partials;
  a.pro_stride = s.pstride;
  for (int q = 0; q < 5; ++q) a.pro_cnt[q] = s.slot_n[q];
  a.st = s.st;
  a.pro_it = it;
  a.pro_h = h;
  a.pro_par = par;
  a.pro_thr = thr;
  a.pro_s1 = s1;
  a.pro_alpha = alpha;
  static const int pre = [] {
    const char* e = getenv("KR_EW_PREFETCH");
    return e ? atoi(e) : 1;
  }();
  a.pro_pre = pre;
  for (int p = 0; p < ew_products(op); ++p) s.slot_n[slot0 + p] = s.grid;
  hipEvent_t t0 = nullptr;
  const char* nm = ew_name(op);
  prof_begin(s, nm, t0);
  launch_ew(op, a, s.stream);
  prof_end(s, nm, t0, 8.0 * ew_vectors(op) * s.n);
}

void System::scalar_state_read() {
  Shard& s = shards[0];
  KR_HIP_CHECK(hipMemcpyAsync(s.hst, s.st, sizeof(double) * kScalarState,
                              hipMemcpyDeviceToHost, s.stream));
  const double w0 = now_seconds();
  host_sync(s.stream);
  host_wait_s += now_seconds() - w0;
  size_t pend = s.pending.size();
  if (pend > 512) harvest_profile();
}

// conv(g) = sqrt(g)/||b|| < tol, the reference's test on a squared norm g,
// is monotone in g >= 0 (sqrt and division by ||b|| > 0 are correctly rounded,
// hence monotone), so it equals 0 <= g < thr for the smallest non-negative
// double thr with !conv(thr): found by bisection over the bit patterns with
// the host's own arithmetic. The device test is then bitwise the host's.
double conv_threshold(double bnorm, double tol) {
  auto conv = [&](double g) { return std::sqrt(g) / bnorm < tol; };
  auto dbl = [](uint64_t b) {
    double d;
    std::memcpy(&d, &b, 8);
    return d;
  };
  if (!conv(0.0)) return 0.0;
  uint64_t lo = 0, hi = 0x7FF0000000000000ull;  // conv(+0) true; conv(+inf) false
  while (hi - lo > 1) {
    const uint64_t mid = lo + (hi - lo) / 2;
    if (conv(dbl(mid)))
      lo = mid;
    else
      hi = mid;
  }
  return dbl(hi);
}

void System::copy_own(int dst, int src) {
  for (auto& s : shards) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    KR_HIP_CHECK(hipMemcpyAsync(s.own(dst), s.own(src), 8 * (size_t)s.n,
                                hipMemcpyDeviceToDevice, s.stream));
  }
}

std::vector<double> System::reduce(int nslots) {
  std::vector<double> tot(nslots, 0.0);
  if (nslots <= 0) return tot;
  KR_REQUIRE(nslots <= kMaxSlots, "too many slots");
  auto finalize_shard = [&](Shard& s, size_t) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    hipEvent_t t0 = nullptr;
    prof_begin(s, "reduce", t0);
    SlotCounts cnt{};
    for (int q = 0; q < nslots; ++q) cnt.n[q] = s.slot_n[q];
    launch_finalize_counts(s.partials, s.pstride, cnt, nslots, s.slots, s.stream);
    if (hybrid()) {
      // gathered below, from the first shard's stream
      KR_HIP_CHECK(hipEventRecord(s.ev_a, s.stream));
    } else if (comm) {
      KR_NCCL_CHECK(ncclAllGather(s.slots, s.gather, (size_t)nslots, ncclFloat64, comm->nccl,
                                  s.stream));
      KR_HIP_CHECK(hipMemcpyAsync(s.host, s.gather, sizeof(double) * nslots * comm->nranks,
                                  hipMemcpyDeviceToHost, s.stream));
    } else {
      KR_HIP_CHECK(hipMemcpyAsync(s.host, s.slots, sizeof(double) * nslots,
                                  hipMemcpyDeviceToHost, s.stream));
    }
    prof_end(s, "reduce", t0, 8.0 * nslots * s.pstride);
  };
  // In-process stream groups whose shards share stride and counts: one
  // finalize launch and one copy for the group (the same sums per shard).
  std::vector<char> grouped(groups.size(), 0);
  if (!comm) {
    for (size_t g = 0; g < groups.size(); ++g) {
      if (!gslots[g].dev) continue;
      const Shard& s0 = shards[(size_t)groups[g][0]];
      bool same = true;
      for (int li : groups[g]) {
        const Shard& s = shards[(size_t)li];
        same = same && s.pstride == s0.pstride;
        for (int q = 0; q < nslots && same; ++q) same = s.slot_n[q] == s0.slot_n[q];
      }
      grouped[g] = same ? 1 : 0;
    }
    for_groups([&](const std::vector<int>& grp) {
      size_t g = 0;
      while (groups[g][0] != grp[0]) ++g;
      if (!grouped[g]) {
        for (int li : grp) finalize_shard(shards[(size_t)li], (size_t)li);
        return;
      }
      Shard& s0 = shards[(size_t)grp[0]];
      KR_HIP_CHECK(hipSetDevice(s0.dev));
      hipEvent_t t0 = nullptr;
      prof_begin(s0, "reduce", t0);
      SlotCounts cnt{};
      for (int q = 0; q < nslots; ++q) cnt.n[q] = s0.slot_n[q];
      FinalizeGroup fg;
      for (int li : grp) fg.part[fg.n++] = shards[(size_t)li].partials;
      launch_finalize_group(fg, s0.pstride, cnt, nslots, gslots[g].dev, kMaxSlots, s0.stream);
      KR_HIP_CHECK(hipMemcpyAsync(gslots[g].host, gslots[g].dev,
                                  sizeof(double) * ((grp.size() - 1) * kMaxSlots + nslots),
                                  hipMemcpyDeviceToHost, s0.stream));
      prof_end(s0, "reduce", t0, 8.0 * nslots * s0.pstride * grp.size(), (int)grp.size());
    });
  } else {
    for (size_t li = 0; li < shards.size(); ++li) finalize_shard(shards[li], li);
  }
  if (hybrid()) {
    // every local shard's slots side by side (kMaxLocal x nslots), one
    // all-gather for the rank; the stride stays fixed so any rank can index
    Shard& s0 = shards[0];
    KR_HIP_CHECK(hipSetDevice(s0.dev));
    for (size_t li = 0; li < shards.size(); ++li) {
      Shard& s = shards[li];
      KR_HIP_CHECK(hipStreamWaitEvent(s0.stream, s.ev_a, 0));
      KR_HIP_CHECK(hipMemcpyPeerAsync(hy_send + li * nslots, s0.dev, s.slots, s.dev,
                                      sizeof(double) * nslots, s0.stream));
    }
    const size_t per = (size_t)kMaxLocal * nslots;
    KR_NCCL_CHECK(ncclAllGather(hy_send, hy_recv, per, ncclFloat64, comm->nccl, s0.stream));
    KR_HIP_CHECK(hipMemcpyAsync(hy_host, hy_recv, sizeof(double) * per * comm->nranks,
                                hipMemcpyDeviceToHost, s0.stream));
  }
  const double w0 = now_seconds();
  for (auto& s : shards) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    host_sync(s.stream);
  }
  host_wait_s += now_seconds() - w0;
  // KR_POISON=1 (debug): the consumed slots' partials become NaN, so a later
  // reduction that reads a partial no launch rewrote shows up as NaN (the GPU
  // suites pass with it: every reduced partial is rewritten before reuse)
  static const bool poison = [] {
    const char* e = getenv("KR_POISON");
    return e && atoi(e) != 0;
  }();
  if (poison)
    for (auto& s : shards) {
      KR_HIP_CHECK(hipSetDevice(s.dev));
      KR_HIP_CHECK(hipMemsetAsync(s.partials, 0xFF, sizeof(double) * (size_t)nslots * s.pstride,
                                  s.stream));
    }
  // Fixed order: global shard 0, 1, ... (identical for in-process and RCCL).
  if (hybrid()) {
    const size_t per = (size_t)kMaxLocal * nslots;
    for (int r = 0; r < comm->nranks; ++r)
      for (int l = 0; l < rank_first[r + 1] - rank_first[r]; ++l)
        for (int q = 0; q < nslots; ++q) tot[q] = tot[q] + hy_host[r * per + l * nslots + q];
  } else if (comm) {
    const double* h = shards[0].host;
    for (int r = 0; r < comm->nranks; ++r)
      for (int q = 0; q < nslots; ++q) tot[q] = tot[q] + h[r * nslots + q];
  } else {
    // shard order (a group need not be a run of it: devices 0, 1, 0, 1)
    std::vector<const double*> h(shards.size());
    for (size_t g = 0; g < groups.size(); ++g)
      for (size_t j = 0; j < groups[g].size(); ++j)
        h[(size_t)groups[g][j]] = grouped[g] ? gslots[g].host + j * kMaxSlots
                                             : shards[(size_t)groups[g][j]].host;
    for (size_t li = 0; li < shards.size(); ++li)
      for (int q = 0; q < nslots; ++q) tot[q] = tot[q] + h[li][q];
  }
  // Profiling events are read back lazily (every few hundred kernels and on
  // kr_solve_kernel_stats), not at every sync point: reading ~30 event pairs
  // here cost ~40 us of host turnaround per k-skip outer iteration, i.e. GPU
  // idle time (≈1 % at 1 GPU, ≈3 % at the 8-GPU shard size).
  size_t pend = 0;
  for (auto& s : shards) pend = std::max(pend, s.pending.size());
  if (pend > 512) harvest_profile();
  return tot;
}

// ===========================================================================
// Solver sessions
// ===========================================================================
namespace {

class Base : public Session {
 protected:
  // Shared start-up: b, x0 into their vectors and ||b||.
  void load_bx(int B, int X, const double* const* b, const double* const* x0) {
    for (size_t li = 0; li < sys->shards.size(); ++li) {
      Shard& s = sys->shards[li];
      KR_HIP_CHECK(hipSetDevice(s.dev));
      KR_REQUIRE(b && b[li], "b is required");
      KR_HIP_CHECK(hipMemcpyAsync(s.own(B), b[li], 8 * (size_t)s.n, hipMemcpyDeviceToDevice,
                                  s.stream));
      if (x0 && x0[li])
        KR_HIP_CHECK(hipMemcpyAsync(s.own(X), x0[li], 8 * (size_t)s.n,
                                    hipMemcpyDeviceToDevice, s.stream));
      else  // x0 = 0 (v3/gpu/cg.py:12): not left to the allocation's fill
        KR_HIP_CHECK(hipMemsetAsync(s.own(X), 0, 8 * (size_t)s.n, s.stream));
    }
    sys->ew(EW_DOT, 0, 0, {B, B, -1, -1, -1, -1}, 0);
    bnorm = std::sqrt(sys->reduce(1)[0]);
  }
  double rel(double sq) const { return std::sqrt(sq) / bnorm; }
  void start_timer() { t_start = now_seconds(); }
};

// Device-resident scalar batches (CG, MrR on one shard): up to
// kScalarBatch iterations are enqueued at once; the scalars live in Shard::st
// and the convergence test runs on the device (scalar_kernel), which then
// stops every later kernel of the batch. The host syncs once per batch and
// replays the bookkeeping from the recorded norms, checking that the device
// stopped exactly where its own test says (conv_threshold makes the two tests
// bitwise the same). KR_DEVICE_SCALARS=0 restores one sync per reduction.
int scalar_batch() {
  const char* env = getenv("KR_SCALAR_BATCH");
  const int b = env ? atoi(env) : 32;
  return std::max(1, std::min(b, kScalarBatch));
}

// --------------------------------------------------------------------- CG
// v3/gpu/cg.py:8-51 (oracle v3/cpu/cg.py:7-48)
class CgSession : public Base {
  enum { X, B, R, P, V, P2, NV };
  int pc = P;  // p's buffer: EPI_XY_VP writes the new p to the other one
  double gamma = 0;
  bool dev = false;
  double thr = 0;
  std::vector<double> q;  // gamma of the iterations of the current batch
  size_t qpos = 0;
  // Persistent batches (small single-shard systems, launch_cg_persist): one
  // cooperative launch per batch instead of 2 launches per iteration; grid
  // size, barrier counter + timeout flag. Opt-in (KR_PERSIST=1): measured
  // slower than the two launches per iteration on C1 (37k vs 58-62k it/s,
  // DESIGN.md §3); KR_PERSIST_MAXN (default 2^19 rows) bounds the size.
  int persist = 0;
  unsigned* pbar = nullptr;

  void persist_batch(int64_t m) {
    Shard& s = sys->shards[0];
    KR_HIP_CHECK(hipSetDevice(s.dev));
    const int other = pc == P ? P2 : P;
    CgPersistArgs a;
    a.rowptr = s.rowptr;
    a.rowptr64 = s.rowptr64;
    a.col = s.col;
    a.val = s.val;
    a.n = s.n;
    a.pad = s.pad;
    a.x = s.vec[X];
    a.r = s.vec[R];
    a.pa = s.vec[pc];
    a.pb = s.vec[other];
    a.v = s.vec[V];
    a.part = s.partials;
    a.bar = pbar;
    a.err = reinterpret_cast<int*>(pbar + 1);
    a.st = s.st;
    a.gamma = gamma;
    a.it0 = i;
    a.m = (int)m;
    a.thr = thr;
    KR_HIP_CHECK(hipMemsetAsync(pbar, 0, 2 * sizeof(unsigned), s.stream));
    hipEvent_t t0 = nullptr;
    sys->prof_begin(s, "cg_persist", t0);
    launch_cg_persist(a, persist, s.stream);
    // per iteration: the CSR SpMV (p and r gathered, p and v stored) + EW_CG
    const double it_bytes = 12.0 * s.nnz + 4.0 * (s.n + 1) + 32.0 * s.n + 48.0 * s.n;
    sys->prof_end(s, "cg_persist", t0, it_bytes * (double)m);
    if ((m - 1) % 2 != 0) pc = other;  // where the final p = r + beta p landed
  }

  // Iterations i .. i+m-1 on the device; q[j] = gamma at the top of i+j+1.
  void run_batch() {
    const int64_t m = std::min<int64_t>({(int64_t)scalar_batch(), std::max<int64_t>(hint, 1),
                                         prm.maxiter - i});
    if (persist) {
      persist_batch(m);
    } else {
    sys->dev_stop = true;
    const bool fused = sys->fused_scalars();
    // fused scalars + virtual p: iteration j > 0 of the batch folds the
    // previous iteration's beta step and p = r + beta p into its SpMV, so an
    // iteration is 2 launches (the batch's last one keeps EW_CG_P, whose
    // beta step the host reads back)
    const bool vpf = fused && sys->vp_ok();
    // x += alpha p deferred in pairs of iterations (x is not read inside the
    // loop): step j (even, j+1 < m) only updates r (EW_CG_NOX, alpha kept in
    // ST_ALPHA), step j+1 does x = (x + alpha_j p_j) + alpha_j+1 p_j+1
    // (EW_CG_X2): the same two roundings per element as two EW_CG steps,
    // one x read and write fewer. p_j is still in the other p buffer then
    // (EPI_XY_VP wrote p_j+1 beside it). KR_CG_XDEFER=0 disables (A/B).
    const char* xenv = getenv("KR_CG_XDEFER");
    const bool defer = vpf && !(xenv && atoi(xenv) == 0);
    std::vector<int> pbuf(m, -1);  // p_j's buffer at the NOX steps
    for (int64_t j = 0; j < m; ++j) {
      if (j > 0) sys->prof_active = (sys->prof_tick++ % sys->profile_every) == 0;
      if (fused) {  // the scalar steps inside the vector kernels: 3 launches
        const int par = (int)((i + j) & 1);
        int s1 = 1;
        if (vpf && j > 0) {
          const int pn = pc == P ? P2 : P;
          sys->spmv_vp(pc, R, V, pn, i + j - 1, (int)j - 1, par ^ 1, thr);  // beta; p; v = A p
          pc = pn;
          s1 = 4;  // sigma: slot 4 (the SpMV's products sit in slots 3..5)
        } else {
          sys->spmv(EPI_XY, pc, -1, V, -1, -1, -1, 0);  // v = A p ; sigma
        }
        if (defer && j % 2 == 0 && j + 1 < m) {
          pbuf[j] = pc;
          sys->ew_pro(EW_CG_NOX, SC_CG_ALPHA, {X, pc, R, V, -1, -1}, 0, i + j, (int)j, par, thr,
                      s1, 1);
        } else if (defer && j % 2 == 1) {
          const int pp = pc == P ? P2 : P;  // p_j-1
          sys->ew_pro(EW_CG_X2, SC_CG_ALPHA, {X, pc, R, V, pp, -1}, 0, i + j, (int)j, par, thr,
                      s1, 2);
        } else {
          sys->ew_pro(EW_CG, SC_CG_ALPHA, {X, pc, R, V, -1, -1}, 0, i + j, (int)j, par, thr, s1);
        }
        if (!vpf || j == m - 1)
          sys->ew_pro(EW_CG_P, SC_CG_BETA, {pc, R, -1, -1, -1, -1}, 0, i + j, (int)j, par, thr);
        continue;
      }
      sys->spmv(EPI_XY, pc, -1, V, -1, -1, -1, 0);              // v = A p ; sigma
      sys->scalar(SC_CG_ALPHA, 1 << 1, i + j, (int)j, thr);     // alpha = gamma / sigma
      sys->ew_dev(EW_CG, ST_C0, {X, pc, R, V, -1, -1}, 0);      // x += a p ; r -= a v
      sys->scalar(SC_CG_BETA, 1 << 0, i + j, (int)j, thr);      // beta, gamma, test
      sys->ew_dev(EW_CG_P, ST_C2, {pc, R, -1, -1, -1, -1}, 0);  // p = r + b p
    }
    sys->dev_stop = false;
    sys->scalar_state_read();
    // stopped right after a NOX step: apply its deferred x += alpha p (the
    // stream runs it before anything reads x)
    const double* hs = sys->shards[0].hst;
    if (hs[ST_STOP] != 0.0) {
      const int64_t jl = (int64_t)hs[ST_STOP_AT] - 1 - i;  // the last step that ran
      if (jl >= 0 && jl < m && pbuf[jl] >= 0)
        sys->ew_dev(EW_AXPY, ST_ALPHA, {X, pbuf[jl], -1, -1, -1, -1}, 0);
    }
    }
    if (persist) {
      sys->scalar_state_read();
      int err = 0;
      KR_HIP_CHECK(hipMemcpy(&err, pbar + 1, sizeof(int), hipMemcpyDeviceToHost));
      if (err) throw Failure(KR_ERR_HIP, "persistent CG: a grid barrier timed out "
                                          "(x and r are undefined after this error)");
    }
    const double* h = sys->shards[0].hst;
    q.assign(h + ST_HIST, h + ST_HIST + m);
    qpos = 0;
    int64_t stop_at = -1;
    for (int64_t j = 0; j < m; ++j)
      if (i + j + 1 < prm.maxiter && rel(q[j]) < prm.tol) {
        stop_at = i + j + 1;
        q.resize(j + 1);
        break;
      }
    const bool dstop = h[ST_STOP] != 0.0;
    if (stop_at >= 0 ? !(dstop && (int64_t)h[ST_STOP_AT] == stop_at)
                     : (dstop && (int64_t)h[ST_STOP_AT] < prm.maxiter))
      throw Failure(KR_ERR_INVALID, "device/host convergence test disagree (CG)");
  }

 public:
  void begin(const double* const* b, const double* const* x0) override {
    sys->alloc_vectors(NV);
    load_bx(B, X, b, x0);
    sys->spmv(EPI_BMINUS, X, -1, R, -1, -1, B, 0);  // r = b - A x
    gamma = sys->reduce(1)[0];                      // gamma = <r,r>
    sys->copy_own(P, R);                            // p = r.copy()
    pc = P;
    dev = sys->device_scalars() && !prm.nan_guard;  // the guard tests every entry on the host
    if (dev) {
      thr = conv_threshold(bnorm, prm.tol);
      sys->scalar_state_init(gamma);
      const char* env = getenv("KR_PERSIST");
      const char* envn = getenv("KR_PERSIST_MAXN");
      const int64_t maxn = envn ? atoll(envn) : (int64_t)1 << 19;
      if (env && atoi(env) == 1 && sys->shards.size() == 1 && !sys->comm) {
        Shard& s = sys->shards[0];
        if (!s.dense && s.col && s.n > 0 && s.n <= maxn) {
          KR_HIP_CHECK(hipSetDevice(s.dev));
          persist = cg_persist_grid(s.n);
          if (persist && !pbar) KR_HIP_CHECK(hipMalloc(&pbar, 2 * sizeof(unsigned)));
        }
      }
    }
    i = 0;
    index = 0;
    set_nosl(0, 0);
    start_timer();
  }
  ~CgSession() override {
    if (pbar) (void)hipFree(pbar);
  }
  bool step_once() override {
    if (i >= prm.maxiter) {  // while-else branch
      set_entry(i, rel(gamma));
      index = i;
      return done = true;
    }
    set_entry(i, rel(gamma));
    index = i;
    if (residual[i] < prm.tol) {
      converged = true;
      return done = true;
    }
    if (guard_stop(i)) return true;
    if (dev) {
      if (qpos >= q.size()) run_batch();
      gamma = q[qpos++];
    } else {
      sys->spmv(EPI_XY, pc, -1, V, -1, -1, -1, 0);  // v = A p ; sigma = <p,v>
      const double sigma = sys->reduce(3)[1];
      const double alpha = gamma / sigma;
      sys->ew(EW_CG, alpha, 0, {X, pc, R, V, -1, -1}, 0);  // x += a p ; r -= a v
      const double gnew = sys->reduce(1)[0];
      const double beta = gnew / gamma;
      gamma = gnew;
      sys->ew(EW_CG_P, beta, 0, {pc, R, -1, -1, -1, -1}, 0);  // p = r + b p
    }
    i += 1;
    set_nosl(i, i);
    index = i;
    set_entry(i, 0.0);
    return false;
  }
  int result_x() const override { return X; }
};

// --------------------------------------------------------------------- MrR
// v3/gpu/mrr.py:8-65 (oracle v3/cpu/mrr.py:7-61)
class MrrSession : public Base {
  enum { X, B, R, Y, Z, AR, R2, Y2, AR2, NV };
  // r, y, Ar alternate with r2, y2, Ar2 when the vector step runs inside the
  // next SpMV (EPI_MRR_V): other rows still gather the old ones
  int r = R, y = Y, ar = AR, r2 = R2, y2 = Y2, ar2 = AR2;
  bool dev = false;
  double thr = 0;
  std::vector<double> q;  // <r,r> at the top of the iterations of the batch
  size_t qpos = 0;

  // Iterations i .. i+m-1 on the device; q[j] = <r,r> at the top of i+j.
  void run_batch() {
    const int64_t m = std::min<int64_t>({(int64_t)scalar_batch(), std::max<int64_t>(hint, 1),
                                         prm.maxiter - i});
    sys->dev_stop = true;
    const bool fused = sys->fused_scalars();
    // One shard, fused scalars, a kernel with virtual inputs (sys->fuse_first):
    // iteration j's vector step runs inside iteration j+1's SpMV (EPI_MRR_V):
    // 2 launches per iteration, r / y / Ar read once for both. MrR 256^3
    // +7 %, 256^2 +15-29 %, C3 (symmetric DIA) +8-9 %. KR_MRR_V=0: off.
    const char* venv = getenv("KR_MRR_V");
    const bool vfuse = fused && sys->fuse_first && !(venv && atoi(venv) == 0);
    // x -= z deferred in pairs of iterations (x is not read inside the loop):
    // step j (even, j+1 < m) EW_MRR_NOX, step j+1 EW_MRR_X2 with
    // x = (x - z_j+1) - z_j+2 -- its z input is z_j+1 -- the same roundings,
    // one x read and write fewer per pair. KR_MRR_XDEFER=0 disables (A/B).
    const char* xenv = getenv("KR_MRR_XDEFER");
    const bool defer = !vfuse && !(xenv && atoi(xenv) == 0);
    auto step_op = [&](int64_t j) {
      if (defer && j % 2 == 0 && j + 1 < m) return EW_MRR_NOX;
      if (defer && j % 2 == 1) return EW_MRR_X2;
      return EW_MRR;
    };
    for (int64_t j = 0; j < m; ++j) {
      if (j > 0) sys->prof_active = (sys->prof_tick++ % sys->profile_every) == 0;
      if (vfuse) {
        if (j == 0) sys->spmv(EPI_MRR_LOOP, r, -1, ar, -1, y, -1, 0);  // Ar = A r ; <r,r> mu nu
        sys->ew_pro(EW_MRR_S, SC_MRR_GAMMA, {ar, y, r, -1, -1, -1}, 3, i + j, (int)j, 0, thr);
        if (j + 1 < m) {  // step j, then Ar = A r of iteration j+1 ; <r,r> mu nu
          StepOps st;
          st.u1 = y2;
          st.u2 = Z;
          st.us = X;
          st.ud = X;
          st.x3 = ar;
          st.pro = 1;
          sys->spmv(EPI_MRR_V, r, y, ar2, r2, -1, -1, 0, &st);
          std::swap(r, r2);
          std::swap(y, y2);
          std::swap(ar, ar2);
        } else {
          sys->ew_pro(EW_MRR, SC_MRR_ZETA, {y, ar, Z, r, X, X}, 0, i + j, (int)j, 0, thr);
        }
        continue;
      }
      sys->spmv(EPI_MRR_LOOP, r, -1, ar, -1, y, -1, 0);            // Ar = A r ; <r,r> mu nu
      if (fused) {  // the scalar steps inside the vector kernels: 3 launches
        sys->ew_pro(EW_MRR_S, SC_MRR_GAMMA, {ar, y, r, -1, -1, -1}, 3, i + j, (int)j, 0, thr);
        sys->ew_pro(step_op(j), SC_MRR_ZETA, {y, ar, Z, r, X, X}, 0, i + j, (int)j, 0, thr);
        continue;
      }
      sys->scalar(SC_MRR_GAMMA, 0x7, i + j, (int)j, thr);          // test ; gamma = nu / mu
      sys->ew_dev(EW_MRR_S, ST_C0, {ar, y, r, -1, -1, -1}, 3);     // s ; <r,s> <s,s>
      sys->scalar(SC_MRR_ZETA, 0x18, i + j, (int)j, thr);          // zeta, eta
      sys->ew_dev(step_op(j), ST_C2, {y, ar, Z, r, X, X}, 0);
    }
    sys->dev_stop = false;
    sys->scalar_state_read();
    const double* h = sys->shards[0].hst;
    if (h[ST_STOP] != 0.0) {  // stopped right after a NOX step: its x -= z
      const int64_t jl = (int64_t)h[ST_STOP_AT] - 1 - i;  // the last update that ran
      if (jl >= 0 && jl < m && defer && step_op(jl) == EW_MRR_NOX)
        sys->ew(EW_AXPY, -1.0, 0, {X, Z, -1, -1, -1, -1}, 0);  // x + (-1) z == x - z
    }
    q.assign(h + ST_HIST, h + ST_HIST + m);
    qpos = 0;
    int64_t stop_at = -1;
    for (int64_t j = 0; j < m; ++j)
      if (rel(q[j]) < prm.tol) {
        stop_at = i + j;
        q.resize(j + 1);
        break;
      }
    const bool dstop = h[ST_STOP] != 0.0;
    if (stop_at >= 0 ? !(dstop && (int64_t)h[ST_STOP_AT] == stop_at) : dstop)
      throw Failure(KR_ERR_INVALID, "device/host convergence test disagree (MrR)");
  }

 public:
  void begin(const double* const* b, const double* const* x0) override {
    sys->alloc_vectors(NV);
    load_bx(B, X, b, x0);
    sys->spmv(EPI_BMINUS, X, -1, R, -1, -1, B, 0);
    set_entry(0, rel(sys->reduce(1)[0]));
    set_nosl(0, 0);
    start_timer();
    sys->spmv(EPI_XY, R, -1, AR, -1, -1, -1, 0);  // Ar = A r
    const auto g = sys->reduce(3);
    const double zeta = g[1] / g[2];  // <r,Ar>/<Ar,Ar>
    sys->ew(EW_MRR_FIRST, 0, zeta, {Y, AR, Z, R, X, X}, 0);
    set_nosl(1, 1);
    i = 1;
    index = 1;
    set_entry(1, 0.0);
    dev = sys->device_scalars() && !prm.nan_guard;  // the guard tests every entry on the host
    if (dev) {
      thr = conv_threshold(bnorm, prm.tol);
      sys->scalar_state_init(0.0);
    }
  }
  bool step_once() override {
    if (i >= prm.maxiter) {
      sys->ew(EW_DOT, 0, 0, {r, r, -1, -1, -1, -1}, 0);
      set_entry(i, rel(sys->reduce(1)[0]));
      index = i;
      return done = true;
    }
    if (dev) {
      if (qpos >= q.size()) run_batch();
      set_entry(i, rel(q[qpos++]));
      index = i;
      if (residual[i] < prm.tol) {
        converged = true;
        return done = true;
      }
    } else {
      sys->spmv(EPI_MRR_LOOP, r, -1, ar, -1, y, -1, 0);  // Ar = A r ; <r,r> mu nu
      const auto g = sys->reduce(3);
      set_entry(i, rel(g[0]));
      index = i;
      if (residual[i] < prm.tol) {
        converged = true;
        return done = true;
      }
      if (guard_stop(i)) return true;
      const double gamma = g[2] / g[1];  // nu / mu
      sys->ew(EW_MRR_S, gamma, 0, {ar, y, r, -1, -1, -1}, 0);
      const auto h = sys->reduce(2);
      const double zeta = h[0] / h[1];
      const double eta = (-zeta) * gamma;
      sys->ew(EW_MRR, eta, zeta, {y, ar, Z, r, X, X}, 0);
    }
    i += 1;
    set_nosl(i, i);
    index = i;
    set_entry(i, 0.0);
    return false;
  }
  int result_x() const override { return X; }
};

// ------------------------------------------------------------ k-skip MrR
// v3/gpu/kskipmrr.py:9-110 (oracle v3/cpu/kskipmrr.py:8-108) and, with
// adaptive = true, v3/cpu/adaptivekskipmrr.py:8-141 semantics.
class KskipMrrSession : public Base {
  // vector ids: fixed ones, then Ar[0..k0+1], Ay[0..k0]. Ar[0] (r) lives in
  // one of two buffers, r0 / r_alt: a fused step SpMV reads r from one and
  // writes the next r into the other (other rows still gather the old r).
  // Ay[0] (y) likewise alternates between y0 / y_alt when steps 0 and 1 run
  // in one SpMV (EPI_STEP_MRR_FIRST2 gathers y0 and writes the new y).
  enum { XA, XB, B, Z, RALT, YALT, FIXED };
  int k0 = 0;
  bool adaptive = false;
  int cur = XA, pre = XB;  // current x buffer / adaptive snapshot buffer
  int xsrc = XA;           // source of the next x update
  int r0 = FIXED, r_alt = RALT;
  int y0 = FIXED, y_alt = YALT;
  double pre_residual = 0;
  int AR(int j) const { return FIXED + j; }
  int AY(int j) const { return FIXED + (k0 + 2) + j; }
  static constexpr int kHead = 5;
  int gram_slots(int kk) const { return kHead + 7 * kk; }

  void head() { sys->spmv(EPI_HEAD_MRR, r0, -1, AR(1), -1, y0, -1, 0); }
  void chain(int kk) {
    // Two basis duals per launch where the shard allows (System::spmv_pair:
    // Ar[m+2], Ay[m+1] stay on chip); an odd count ends with a single dual.
    const bool pairs = sys->pair_ok();
    for (int m = 0; m < kk;) {
      if (pairs && m + 1 < kk) {
        sys->products_only = m + 1 == kk - 1;
        sys->spmv_pair(AR(m + 1), m == 0 ? y0 : AY(m), AR(m + 3), AY(m + 2), kHead + 7 * m);
        sys->products_only = false;
        m += 2;
        continue;
      }
      // the last pair (Ar[kk+1], Ay[kk]) feeds only the Gram products
      sys->products_only = m == kk - 1;
      sys->spmv(EPI_DUAL_MRR, AR(m + 1), m == 0 ? y0 : AY(m), AR(m + 2), AY(m + 1), -1, -1,
                kHead + 7 * m);
      sys->products_only = false;
      ++m;
    }
  }
  // Initial / restart MrR step (v3/cpu/kskipmrr.py:26-31).
  void mrr_first(int x_from) {
    sys->spmv(EPI_XY, r0, -1, AR(1), -1, -1, -1, 0);
    const auto g = sys->reduce(3);
    const double zeta = g[1] / g[2];
    sys->ew(EW_MRR_FIRST, 0, zeta, {y0, AR(1), Z, r0, x_from, cur}, 0);
    xsrc = cur;
  }
  // x -= z is deferred pairwise: step j stores z and leaves x (kind 0), step
  // j+1 applies x = (x - z_j) - z_{j+1} in registers (kind 1) -- the same two
  // roundings as the reference's two statements, one x read+write fewer. The
  // last step of an outer iteration applies its own x -= z (kind 2) -- unless
  // xdefer: then it is left pending too (xpend) and the next outer
  // iteration's fused steps 0+1 apply x = ((x - z_k) - z_1) - z_2, z_k being
  // their z input (even k, non-adaptive: the adaptive rollback snapshots x).
  // Every exit (convergence, maxiter, kr_solve_end) settles it first.
  bool xdefer = false, xpend = false;
  int step_kind(int j) const {
    if (j % 2 == 0 && j < k) return 0;
    if (j % 2 == 1) return 1;
    return xdefer ? 0 : 2;
  }
  void settle() override {
    if (!xpend) return;
    sys->ew(EW_AXPY, -1.0, 0, {xsrc, Z, -1, -1, -1, -1}, 0);  // x + (-1) z == x - z
    xpend = false;
  }

 public:
  explicit KskipMrrSession(bool adapt) : adaptive(adapt) {}

  void begin(const double* const* b, const double* const* x0) override {
    k = prm.k;
    k0 = k;
    KR_REQUIRE(k >= 0 && gram_slots(k) <= kMaxSlots, "k out of range");
    sys->alloc_vectors(FIXED + (k0 + 2) + (k0 + 1));
    r0 = AR(0);
    r_alt = RALT;
    y0 = AY(0);
    y_alt = YALT;
    load_bx(B, XA, b, x0);
    if (adaptive) sys->copy_own(XB, XA);  // pre_x guard = x0
    sys->spmv(EPI_BMINUS, XA, -1, r0, -1, -1, B, 0);
    set_entry(0, rel(sys->reduce(1)[0]));
    pre_residual = residual[0];
    set_nosl(0, 0);
    track_k = adaptive;
    if (adaptive) set_k(0, k);
    start_timer();
    mrr_first(XA);
    set_nosl(1, 1);
    if (adaptive) set_k(1, k);
    i = 1;
    index = 1;
    set_entry(1, 0.0);
    const char* xenv = getenv("KR_KSKIP_XDEFER");
    xdefer = !adaptive && sys->fuse_steps && sys->fuse_first && k >= 2 && k % 2 == 0 &&
             !(xenv && atoi(xenv) == 0);
    xpend = false;
    head();
  }

  bool step_once() override {
    if (i >= prm.maxiter) {
      set_entry(index, rel(sys->reduce(kHead)[0]));
      settle();
      return done = true;
    }
    chain(k);  // speculative: launched before the convergence test
    std::vector<double> g = sys->reduce(gram_slots(k));
    set_entry(index, rel(g[0]));
    if (adaptive) {
      if (residual[index] > pre_residual) {
        // roll back to the snapshot and restart (v3/cpu/adaptivekskipmrr.py:45-66)
        sys->spmv(EPI_BMINUS, pre, -1, r0, -1, -1, B, 0);
        mrr_first(pre);
        i += 1;
        index += 1;
        head();
        const int knew = k > 1 ? k - 1 : k;
        chain(knew);
        g = sys->reduce(gram_slots(knew));
        set_entry(index, rel(g[0]));
        set_nosl(index, i);
        k = knew;
        set_k(index, k);
      } else {
        pre_residual = residual[index];
        std::swap(cur, pre);  // pre_x = x.copy(): the next update writes the other buffer
        xsrc = pre;
      }
    }
    if (residual[index] < prm.tol) {
      converged = true;
      settle();
      return done = true;
    }
    if (guard_stop(index)) {
      settle();
      return true;
    }
    // Gram -> (alpha, beta, delta) as the reference lays them out.
    std::vector<double> alpha(2 * k + 3, 0.0), beta(2 * k + 2, 0.0), delta(2 * k + 1, 0.0);
    alpha[0] = g[0];
    alpha[1] = g[1];
    alpha[2] = g[2];
    beta[1] = g[3];
    delta[0] = g[4];
    for (int m = 0; m < k; ++m) {
      const double* d = &g[kHead + 7 * m];
      alpha[2 * m + 3] = d[0];
      alpha[2 * m + 4] = d[1];
      delta[2 * m + 2] = d[2];
      delta[2 * m + 1] = d[3];
      beta[2 * m + 3] = d[4];
      if (m > 0) beta[2 * m + 1] = d[5];  // same bits as the previous step's d[4]
      beta[2 * m + 2] = d[6];
    }
    std::vector<double> zeta(k + 1), eta(k + 1);
    kskipmrr_recurrence(k, alpha.data(), beta.data(), delta.data(), zeta.data(), eta.data());
    // Step j (v3/gpu/kskipmrr.py:64-71, 88-95): Ay0 = eta Ay0 + zeta Ar1;
    // z = eta z - zeta Ar0; Ar0 -= Ay0; x -= z; Ar1 = A Ar0. All k+1 (zeta,
    // eta) pairs are known here, so step j+1's vector update runs in the
    // epilogue of step j's SpMV (EPI_STEP_MRR_*): Ar1 is never stored.
    auto ew_step = [&](int j) {
      const int kind = step_kind(j);
      if (kind == 0) {
        sys->ew(EW_MRR_NOX, eta[j], zeta[j], {y0, AR(1), Z, r0, -1, -1}, 0);
      } else {
        sys->ew(kind == 1 ? EW_MRR_X2 : EW_MRR, eta[j], zeta[j],
                {y0, AR(1), Z, r0, xsrc, cur}, 0);
        xsrc = cur;
      }
    };
    int j1 = 1;
    const bool step2 = sys->fuse_steps && sys->step2_ok();
    if (step2 && sys->fuse_first && k >= 2 && KR_ENV("KR_STEP3", 1) != 0) {
      // steps 0, 1 (FIRST2's) and 2 in one walk on a box shard: step 2 is an
      // even step, x deferred (kind 0) or applied (kind 2, the last step)
      const int kind2 = step_kind(2);
      const double c[6] = {eta[0], zeta[0], eta[1], zeta[1], eta[2], zeta[2]};
      sys->spmv_step2(r0, r_alt, y0, y_alt, Z, xsrc, cur, kind2 == 2 ? 4 : 0, c, AR(1),
                      xpend ? 1 : 0);
      xpend = kind2 == 0 && k == 2;  // xdefer: step 2's x -= z left to the next outer iteration
      xsrc = cur;
      std::swap(r0, r_alt);
      std::swap(y0, y_alt);
      j1 = 3;
    } else if (sys->fuse_steps && sys->fuse_first && k >= 1) {
      // steps 0 (kind 0) and 1 (kind 1) in one SpMV: r1 is formed at every
      // gathered column from r0, y0, Ar1; new y and r go to the other buffers
      StepOps st;
      st.u1 = y_alt;
      st.u2 = Z;
      st.us = xsrc;
      st.ud = cur;
      st.c0 = eta[0];
      st.c1 = zeta[0];
      st.x3 = AR(1);
      st.c2 = eta[1];
      st.c3 = zeta[1];
      st.xpend = xpend ? 1 : 0;
      sys->spmv(EPI_STEP_MRR_FIRST2, r0, y0, r_alt, -1, -1, -1, 0, &st);
      xpend = false;
      xsrc = cur;
      std::swap(r0, r_alt);
      std::swap(y0, y_alt);
      j1 = 2;
    } else {
      ew_step(0);
    }
    bool headed = false;  // the head ran inside the last step walk
    for (int j = j1; j <= k; ++j) {
      const int ka = step_kind(j), kb = j + 1 <= k ? step_kind(j + 1) : -1;
      if (step2 && kb >= 0 && ka != 2 && j + 1 == k && sys->step2h_ok()) {
        // the last pair of steps and the next head in one walk (the head's
        // Ar1 = A r and products at slots 0..4, as head() writes them)
        const int xm = (ka == 1 ? 3 : 0) | (kb == 1 ? 2 : 0) | (kb >= 1 ? 4 : 0);
        const double c[4] = {eta[j], zeta[j], eta[j + 1], zeta[j + 1]};
        sys->spmv_step2h(r0, r_alt, y0, y_alt, Z, xsrc, cur, xm, c, AR(1));
        if (xm != 0) xsrc = cur;
        if (kb == 0) xpend = true;  // xdefer: left to the next outer iteration
        std::swap(r0, r_alt);
        std::swap(y0, y_alt);
        headed = true;
        ++j;
        continue;
      }
      if (step2 && kb >= 0 && ka != 2) {
        // steps j and j+1 in one walk on a box shard: r and y into their
        // other buffers, z and x as the two step kernels write them
        // (System::spmv_step2; bitwise those). x loses z_j's predecessor
        // and z_j when step j is an x2 step, z_j when step j+1 is, z_{j+1}
        // when step j+1 updates x at all
        const int xm = (ka == 1 ? 3 : 0) | (kb == 1 ? 2 : 0) | (kb >= 1 ? 4 : 0);
        const double c[4] = {eta[j], zeta[j], eta[j + 1], zeta[j + 1]};
        sys->spmv_step2(r0, r_alt, y0, y_alt, Z, xsrc, cur, xm, c);
        if (xm != 0) xsrc = cur;
        if (kb == 0 && j + 1 == k) xpend = true;  // xdefer: left to the next outer iteration
        std::swap(r0, r_alt);
        std::swap(y0, y_alt);
        ++j;
        continue;
      }
      if (sys->fuse_steps) {
        const int kind = step_kind(j);
        StepOps st;
        st.u1 = y0;
        st.u2 = Z;
        if (kind != 0) {
          st.us = xsrc;
          st.ud = cur;
        }
        st.c0 = eta[j];
        st.c1 = zeta[j];
        const SpmvEpi e = kind == 0 ? EPI_STEP_MRR_NOX
                                    : kind == 1 ? EPI_STEP_MRR_X2 : EPI_STEP_MRR_X;
        sys->spmv(e, r0, -1, r_alt, -1, -1, -1, 0, &st);
        if (kind != 0) xsrc = cur;
        if (kind == 0 && j == k) xpend = true;  // xdefer: left to the next outer iteration
        std::swap(r0, r_alt);
      } else {
        sys->spmv(EPI_NONE, r0, -1, AR(1), -1, -1, -1, 0);
        ew_step(j);
      }
    }
    if (!headed) head();
    i += k + 1;
    index += 1;
    set_nosl(index, i);
    if (adaptive) set_k(index, k);
    set_entry(index, 0.0);
    return false;
  }
  int result_x() const override { return xsrc; }
};

// ------------------------------------------------------------- k-skip CG
// v3/gpu/kskipcg.py:9-92 (oracle v3/cpu/kskipcg.py:8-87)
class KskipCgSession : public Base {
  // Ap[0] lives in one of two buffers, p0 / p_alt (see KskipMrrSession).
  enum { X, B, PALT, FIXED };
  int p0 = 0, p_alt = PALT;
  int AR(int j) const { return FIXED + j; }
  int AP(int j) const { return FIXED + (k + 2) + j; }
  static constexpr int kHead = 6;
  int gram_slots() const { return kHead + 7 * k; }
  void head() { sys->spmv(EPI_HEAD_KCG, p0, -1, AP(1), -1, AR(0), -1, 0); }

 public:
  void begin(const double* const* b, const double* const* x0) override {
    k = prm.k;
    KR_REQUIRE(k >= 0 && gram_slots() <= kMaxSlots, "k out of range");
    sys->alloc_vectors(FIXED + (k + 2) + (k + 3));
    p0 = AP(0);
    p_alt = PALT;
    load_bx(B, X, b, x0);
    sys->spmv(EPI_BMINUS, X, -1, AR(0), -1, -1, B, 0);  // Ar[0] = b - A x
    sys->reduce(1);
    sys->copy_own(p0, AR(0));  // Ap[0] = Ar[0]
    i = 0;
    index = 0;
    set_nosl(0, 0);
    set_entry(0, 0.0);
    start_timer();
    head();
  }
  bool step_once() override {
    if (i >= prm.maxiter) {
      set_entry(index, rel(sys->reduce(kHead)[0]));
      return done = true;
    }
    // the tiled fused pair (KR_ST2=2) chains two duals per launch where the
    // shard allows; an odd count ends with a single dual
    const bool pairs = sys->pair_mode() >= 2;
    for (int j = 1; j <= k;) {
      if (pairs && j + 1 <= k) {
        sys->products_only = j + 1 == k;  // Ar[k], Ap[k+1] feed only the Gram products
        sys->spmv_pair(AR(j - 1), AP(j), AR(j + 1), AP(j + 2), kHead + 7 * (j - 1), EPI_DUAL_KCG);
        sys->products_only = false;
        j += 2;
        continue;
      }
      sys->products_only = j == k;  // Ar[k], Ap[k+1] feed only the Gram products
      sys->spmv(EPI_DUAL_KCG, AR(j - 1), AP(j), AR(j), AP(j + 1), -1, -1, kHead + 7 * (j - 1));
      sys->products_only = false;
      ++j;
    }
    const std::vector<double> g = sys->reduce(gram_slots());
    set_entry(index, rel(g[0]));
    if (residual[index] < prm.tol) {
      converged = true;
      return done = true;
    }
    if (guard_stop(index)) return true;
    std::vector<double> a(2 * k + 2, 0.0), f(2 * k + 4, 0.0), c(2 * k + 2, 0.0);
    a[0] = g[0];
    f[0] = g[1];
    f[1] = g[2];
    f[2] = g[3];
    c[0] = g[4];
    c[1] = g[5];
    for (int j = 1; j <= k; ++j) {
      const double* d = &g[kHead + 7 * (j - 1)];
      a[2 * j - 1] = d[0];
      a[2 * j] = d[1];
      f[2 * j + 1] = d[2];
      f[2 * j + 2] = d[3];
      c[2 * j - 1] = d[4];
      c[2 * j] = d[5];
      c[2 * j + 1] = d[6];
    }
    // f[2k+3] = <Ap[k+1], Ap[k+2]> with Ap[k+2] never computed: 0.
    std::vector<double> al(k + 1), be(k + 1);
    kskipcg_recurrence(k, a.data(), f.data(), c.data(), al.data(), be.data());
    // Step j (v3/gpu/kskipcg.py:55-60, 71-76); as in k-skip MrR, step j+1's
    // vector update runs in the epilogue of step j's SpMV (EPI_STEP_KCG).
    sys->ew(EW_KCG, al[0], be[0], {X, p0, AR(0), AP(1), -1, -1}, 0);
    for (int j = 1; j <= k; ++j) {
      if (sys->fuse_steps) {
        StepOps st;
        st.u1 = X;
        st.u2 = AR(0);
        st.c0 = al[j];
        st.c1 = be[j];
        sys->spmv(EPI_STEP_KCG, p0, -1, p_alt, -1, -1, -1, 0, &st);
        std::swap(p0, p_alt);
      } else {
        sys->spmv(EPI_NONE, p0, -1, AP(1), -1, -1, -1, 0);
        sys->ew(EW_KCG, al[j], be[j], {X, p0, AR(0), AP(1), -1, -1}, 0);
      }
    }
    head();
    i += k + 1;
    index += 1;
    set_nosl(index, i);
    set_entry(index, 0.0);
    return false;
  }
  int result_x() const override { return X; }
};

// -------------------------------------------- preconditioned / pipelined CG
// v1/threads/pipeline/{pcg,chronopoulos_gear,gropp,pipeline}.py, restated as
// the textbook algorithms those files name (DESIGN.md §5b lists the defects
// of the reference copies that the restatement fixes; oracle/pipecg.py is the
// statement-for-statement CPU form). M^-1 v = v / d with the Jacobi diagonal
// d (kr_solve_set_precond; none: d = 1, and v / 1.0 == v exactly). Loop
// bookkeeping of v1/threads/common.py:41-52: iterations i = 1 .. maxiter-1,
// residual[i] after the i-th update, nosl[i] = i. Scalars go through the
// host (one sync per reduction point, as the CG host path); the reductions
// that the algorithms make independent are fused into one sync.
class PipeCgSession : public Base {
  enum { X, B, R, U, D, P, S, W, Q, M, NN, Z, NV };
  const int variant;  // KR_METHOD_PCG / _CG_GEAR / _GROPP / _PIPECG
  double gamma = 0, delta = 0, alpha = 0, beta = 0;

  std::array<int, kEwOps> ids(std::initializer_list<int> l) const {
    std::array<int, kEwOps> a;
    a.fill(-1);
    int q = 0;
    for (int v : l) a[q++] = v;
    return a;
  }

 public:
  explicit PipeCgSession(int v) : variant(v) {}
  bool ilu = false;  // M^-1 by the ILU sweeps (System::ilu), d = 1
  std::shared_ptr<IluFactors> ilu_f;  // the factors set when the solve began

  void begin(const double* const* b, const double* const* x0) override {
    sys->alloc_vectors(NV);
    load_bx(B, X, b, x0);
    // d: the caller's diagonal, else ones (ILU: ones, and M^-1 by the sweeps)
    ilu_f = sys->ilu;
    ilu = ilu_f != nullptr;
    const bool have = !ilu && !sys->precond.empty();
    for (size_t li = 0; li < sys->shards.size(); ++li) {
      Shard& s = sys->shards[li];
      if (have && sys->precond[li]) {
        KR_HIP_CHECK(hipSetDevice(s.dev));
        KR_HIP_CHECK(hipMemcpyAsync(s.own(D), sys->precond[li], 8 * (size_t)s.n,
                                    hipMemcpyDeviceToDevice, s.stream));
      }
    }
    if (!have) sys->ew_n(EW_ONE, 0, 0, ids({D}), 0);
    sys->spmv(EPI_BMINUS, X, -1, R, -1, -1, B, 0);      // r = b - A x
    sys->ew_n(EW_PRE, 0, 0, ids({R, U, D}), 1);           // u = M^-1 r ; <r,r> <r,u>
    if (ilu) {                                            // u = ilu.solve(r) ; <r,u>: slot 3
      sys->ilu_apply(*ilu_f, R, U);
      sys->ew(EW_DOT, 0, 0, {R, U, -1, -1, -1, -1}, 3);
    }
    const auto g = sys->reduce(ilu ? 4 : 3);              // slot 0: <r,r> of the SpMV
    set_entry(0, rel(g[0]));
    set_nosl(0, 0);
    gamma = g[ilu ? 3 : 2];                               // <r,u>
    switch (variant) {
      case KR_METHOD_PCG:    // p = u.copy()  (pcg.py:28)
      case KR_METHOD_GROPP:  // p = u.copy(); s = A p  (gropp.py:26-27)
        sys->copy_own(P, U);
        if (variant == KR_METHOD_GROPP) {
          sys->spmv(EPI_XY, P, -1, S, -1, -1, -1, 0);     // s = A p ; <p,s>
          delta = sys->reduce(3)[1];
        }
        break;
      case KR_METHOD_CG_GEAR:  // w = A u; alpha = (r,u)/(w,u); beta = 0
      case KR_METHOD_PIPECG: {  // w = A u; (r,u), (w,u) at the loop top
        sys->spmv(EPI_XY, U, -1, W, -1, -1, -1, 0);       // w = A u ; <u,w>
        delta = sys->reduce(3)[1];
        alpha = gamma / delta;
        beta = 0.0;
        break;
      }
    }
    i = 0;
    index = 0;
    start_timer();
  }

  bool step_once() override {
    if (i + 1 >= prm.maxiter) return done = true;  // for i in range(1, max_iter) exhausted
    const int64_t it = i + 1;
    double rr = 0;
    switch (variant) {
      case KR_METHOD_PCG: {  // pcg.py:31-49
        sys->spmv(EPI_XY, P, -1, S, -1, -1, -1, 0);             // s = A p ; <p,s>
        const double sigma = sys->reduce(3)[1];
        alpha = gamma / sigma;
        sys->ew_n(EW_PCG, alpha, 0, ids({X, P, R, S, U, D}), 0);  // x, r, u ; <r,r> <r,u>
        if (ilu) {  // u = ilu.solve(r) ; <r,u>: slot 2 (unused after the exit test)
          sys->ilu_apply(*ilu_f, R, U);
          sys->ew(EW_DOT, 0, 0, {R, U, -1, -1, -1, -1}, 2);
        }
        const auto g = sys->reduce(ilu ? 3 : 2);
        rr = g[0];
        if (!(rel(rr) < prm.tol)) {
          const double gnew = g[ilu ? 2 : 1];
          beta = gnew / gamma;
          gamma = gnew;
          sys->ew(EW_CG_P, beta, 0, {P, U, -1, -1, -1, -1}, 0);  // p = u + beta p
        }
        break;
      }
      case KR_METHOD_CG_GEAR: {  // chronopoulos_gear.py:36-51: one sync per iteration
        sys->ew_n(EW_CGG, alpha, beta, ids({P, U, S, W, X, R, D}), 0);  // <r,r> <r,u>
        if (ilu) {  // u = ilu.solve(r) ; <r,u>: slot 5
          sys->ilu_apply(*ilu_f, R, U);
          sys->ew(EW_DOT, 0, 0, {R, U, -1, -1, -1, -1}, 5);
        }
        sys->spmv(EPI_XY, U, -1, W, -1, -1, -1, 2);              // w = A u ; <u,w>: slot 3
        const auto g = sys->reduce(ilu ? 6 : 5);
        rr = g[0];
        const double gnew = g[ilu ? 5 : 1];
        delta = g[3];
        beta = gnew / gamma;
        alpha = gnew / (delta - beta * gnew / alpha);
        gamma = gnew;
        break;
      }
      case KR_METHOD_GROPP: {  // gropp.py:30-45
        alpha = gamma / delta;
        if (ilu) {  // q = ilu.solve(s); x += a p; r -= a s ; <r,r>; u -= a q; <r,u>
          sys->ilu_apply(*ilu_f, S, Q);
          sys->ew(EW_CG, alpha, 0, {X, P, R, S, -1, -1}, 0);
          sys->ew(EW_AXPY, -alpha, 0, {U, Q, -1, -1, -1, -1}, 0);  // u + (-a) q == u - a q
          sys->ew(EW_DOT, 0, 0, {R, U, -1, -1, -1, -1}, 1);
        } else {
          sys->ew_n(EW_GROPP1, alpha, 0, ids({X, P, R, S, U, D}), 0);  // <r,r> <r,u>
        }
        sys->spmv(EPI_NONE, U, -1, W, -1, -1, -1, 2);                 // w = A u (overlaps)
        const auto g = sys->reduce(2);
        rr = g[0];
        if (!(rel(rr) < prm.tol)) {
          const double gnew = g[1];
          beta = gnew / gamma;
          gamma = gnew;
          sys->ew_n(EW_GROPP2, beta, 0, ids({P, U, S, W}), 0);  // p, s ; <p,s>
          delta = sys->reduce(1)[0];
        }
        break;
      }
      case KR_METHOD_PIPECG: {  // pipeline.py:31-55: one sync per iteration
        if (ilu)
          sys->ilu_apply(*ilu_f, W, M);                                       // m = ilu.solve(w)
        else
          sys->ew_n(EW_DIV, 0, 0, ids({M, W, D}), 0);                 // m = M^-1 w
        sys->spmv(EPI_NONE, M, -1, NN, -1, -1, -1, 0);                // n = A m
        if (it > 1) {
          beta = gamma / gold;
          alpha = gamma / (delta - beta * gamma / alpha);
        } else {
          beta = 0.0;
          alpha = gamma / delta;
        }
        gold = gamma;
        sys->ew_n(EW_PIPE, alpha, beta, ids({Z, NN, Q, M, S, W, P, U, X, R}), 0);
        const auto g = sys->reduce(3);                                // <r,r> <r,u> <w,u>
        rr = g[0];
        gamma = g[1];
        delta = g[2];
        break;
      }
      default: throw Failure(KR_ERR_INVALID, "unknown pipelined CG variant");
    }
    i = it;
    index = i;
    set_nosl(i, i);
    set_entry(i, rel(rr));
    if (residual[i] < prm.tol) {
      converged = true;
      return done = true;
    }
    if (guard_stop(i)) return true;
    return false;
  }
  int result_x() const override { return X; }

 private:
  double gold = 0;  // pipelined CG: gamma of the previous iteration
};

}  // namespace

std::unique_ptr<Session> make_session(System* sys, const kr_solve_params& p) {
  std::unique_ptr<Session> s;
  switch (p.method) {
    case KR_METHOD_CG: s.reset(new CgSession()); break;
    case KR_METHOD_MRR: s.reset(new MrrSession()); break;
    case KR_METHOD_KSKIPCG: s.reset(new KskipCgSession()); break;
    case KR_METHOD_KSKIPMRR: s.reset(new KskipMrrSession(false)); break;
    case KR_METHOD_ADAPTIVE_KSKIPMRR: s.reset(new KskipMrrSession(true)); break;
    case KR_METHOD_PCG:
    case KR_METHOD_CG_GEAR:
    case KR_METHOD_GROPP:
    case KR_METHOD_PIPECG: s.reset(new PipeCgSession(p.method)); break;
    default: throw Failure(KR_ERR_INVALID, "unknown method");
  }
  s->sys = sys;
  s->prm = p;
  const bool pipe = p.method >= KR_METHOD_PCG && p.method <= KR_METHOD_PIPECG;
  if (s->prm.maxiter < 0)  // None -> N (v3/cpu/common.py:29-30); v1: 2N (v1/threads/common.py:47)
    s->prm.maxiter = pipe ? 2 * sys->n_global : sys->n_global;
  // maxiter = 0: CG and k-skip CG return the initial residual; the MrR family
  // takes its first step unconditionally and writes nosl[1] of a length-1
  // array, an IndexError in the reference (v3/cpu/mrr.py:31, kskipmrr.py:32)
  KR_REQUIRE(s->prm.maxiter > 0 || p.method == KR_METHOD_CG || p.method == KR_METHOD_KSKIPCG || pipe,
             "maxiter=0: the MrR family writes nosl[1] past its maxiter+1 entries (IndexError in the reference)");
  return s;
}

}  // namespace kr
