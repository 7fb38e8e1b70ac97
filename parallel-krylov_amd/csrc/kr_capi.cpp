// extern "C" entry points of libkrylov_amd.so (declared in include/krylov_amd.h).
// Every entry point catches everything: nothing throws across the ABI.
#include <cstring>
#include <map>
#include <mutex>

#include "kr_engine.h"

namespace kr {
namespace {

thread_local std::string g_last_error;

// BUMP: the call re-reads the cached KR_* knobs (kr_internal.h KR_ENV);
// kr_solve_step keeps the values of its solve
template <bool BUMP = true, class F>
int guarded(F&& f) {
  if (BUMP) g_env_epoch.fetch_add(1, std::memory_order_relaxed);
  try {
    f();
    return KR_OK;
  } catch (const Failure& e) {
    g_last_error = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    g_last_error = "host allocation failed";
    return KR_ERR_NOMEM;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return KR_ERR_INVALID;
  } catch (...) {
    g_last_error = "unknown failure";
    return KR_ERR_INVALID;
  }
}

std::mutex g_scratch_mu;
std::map<int, std::pair<double*, size_t>> g_scratch;

}  // namespace

double* primitive_scratch(size_t doubles) {
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  int dev = 0;
  KR_HIP_CHECK(hipGetDevice(&dev));
  auto& slot = g_scratch[dev];
  if (slot.second < doubles) {
    if (slot.first) KR_HIP_CHECK(hipFree(slot.first));
    slot.first = nullptr;
    if (hipMalloc(&slot.first, doubles * sizeof(double)) != hipSuccess)
      throw Failure(KR_ERR_NOMEM, "scratch allocation failed");
    slot.second = doubles;
    fresh_fill(slot.first, doubles * sizeof(double), nullptr);
    if (poison_alloc()) KR_HIP_CHECK(hipDeviceSynchronize());
  }
  return slot.first;
}

void banded_offsets(int h, int64_t width, uint64_t seed, int64_t* out_sorted);

}  // namespace kr

using namespace kr;

extern "C" {

int kr_version(void) { return KR_ABI_VERSION; }

const char* kr_last_error(void) { return g_last_error.c_str(); }

int kr_device_count(int* count) {
  return guarded([&] {
    KR_REQUIRE(count, "count is NULL");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
  });
}

// ----------------------------------------------------------------- primitives
// Entries of a CSR block (rowptr[n] - rowptr[0]), read back for the kernel
// choice (spmv_kernel2 needs >= 4): the primitives are not on the solver path.
static int64_t csr_nnz(const void* rowptr, int rowptr64, int64_t n, hipStream_t s) {
  int64_t e[2] = {0, 0};
  if (rowptr64) {
    KR_HIP_CHECK(hipMemcpyAsync(&e[0], rowptr, 8, hipMemcpyDeviceToHost, s));
    KR_HIP_CHECK(hipMemcpyAsync(&e[1], (const int64_t*)rowptr + n, 8, hipMemcpyDeviceToHost, s));
  } else {
    int32_t f[2] = {0, 0};
    KR_HIP_CHECK(hipMemcpyAsync(&f[0], rowptr, 4, hipMemcpyDeviceToHost, s));
    KR_HIP_CHECK(hipMemcpyAsync(&f[1], (const int32_t*)rowptr + n, 4, hipMemcpyDeviceToHost, s));
    KR_HIP_CHECK(hipStreamSynchronize(s));
    return (int64_t)f[1] - f[0];
  }
  KR_HIP_CHECK(hipStreamSynchronize(s));
  return e[1] - e[0];
}

int kr_spmv_csr_f64(const void* rowptr, int rowptr64, const int32_t* col, const double* val,
                    int64_t n_rows, const double* x, double* y, void* stream) {
  return guarded([&] {
    KR_REQUIRE(n_rows >= 0, "n_rows < 0");
    if (n_rows == 0) return;
    KR_REQUIRE(rowptr && col && val && x && y, "NULL operand");
    SpmvArgs a;
    a.rowptr = rowptr;
    a.rowptr64 = rowptr64;
    a.col = col;
    a.val = val;
    a.n = n_rows;
    a.x1 = x;
    a.y1 = y;
    a.grid = default_grid(n_rows);
    a.partials = primitive_scratch(1);
    a.nnz_total = csr_nnz(rowptr, rowptr64, n_rows, static_cast<hipStream_t>(stream));
    launch_spmv(EPI_NONE, a, static_cast<hipStream_t>(stream));
  });
}

int kr_spmv2_csr_f64(const void* rowptr, int rowptr64, const int32_t* col, const double* val,
                     int64_t n_rows, const double* x1, const double* x2, double* y1,
                     double* y2, void* stream) {
  return guarded([&] {
    KR_REQUIRE(n_rows >= 0, "n_rows < 0");
    if (n_rows == 0) return;
    KR_REQUIRE(rowptr && col && val && x1 && x2 && y1 && y2, "NULL operand");
    SpmvArgs a;
    a.rowptr = rowptr;
    a.rowptr64 = rowptr64;
    a.col = col;
    a.val = val;
    a.n = n_rows;
    a.x1 = x1;
    a.x2 = x2;
    a.y1 = y1;
    a.y2 = y2;
    a.grid = default_grid(n_rows);
    a.partials = primitive_scratch(1);
    a.nnz_total = csr_nnz(rowptr, rowptr64, n_rows, static_cast<hipStream_t>(stream));
    launch_spmv(EPI_DUAL_NONE, a, static_cast<hipStream_t>(stream));
  });
}

int kr_dot_f64(const double* u, const double* v, int64_t n, double* out, void* stream) {
  return guarded([&] {
    KR_REQUIRE(n >= 0 && out, "bad arguments");
    hipStream_t s = static_cast<hipStream_t>(stream);
    EwArgs a;
    a.p[0] = const_cast<double*>(u);
    a.p[1] = const_cast<double*>(v);
    a.n = n;
    a.grid = default_grid(n);
    a.partials = primitive_scratch(a.grid);
    if (n > 0) KR_REQUIRE(u && v, "NULL operand");
    launch_ew(EW_DOT, a, s);
    launch_finalize(a.partials, a.grid, 1, out, s);
  });
}

int kr_multidot_f64(const double* const* u_ptrs, const double* const* v_ptrs, int count,
                    int64_t n, double* out, void* stream) {
  return guarded([&] {
    KR_REQUIRE(count >= 0 && count <= 64 && n >= 0 && out, "bad arguments");
    if (count == 0) return;
    hipStream_t s = static_cast<hipStream_t>(stream);
    MultiDotArgs a{};
    for (int i = 0; i < count; ++i) {
      KR_REQUIRE(n == 0 || (u_ptrs[i] && v_ptrs[i]), "NULL operand");
      a.u[i] = u_ptrs[i];
      a.v[i] = v_ptrs[i];
    }
    a.count = count;
    a.n = n;
    a.grid = default_grid(n);
    a.partials = primitive_scratch((size_t)count * a.grid);
    launch_multidot(a, s);
    launch_finalize(a.partials, a.grid, count, out, s);
  });
}

int kr_norm2_f64(const double* u, int64_t n, double* out, void* stream) {
  return guarded([&] {
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int rc = kr_dot_f64(u, u, n, out, stream);
    if (rc != 0) throw Failure(rc, g_last_error);
    launch_sqrt(out, s);
  });
}

namespace {
// Gram pairs (u row, v row, output index) in ranges of <= 64, one multidot each.
struct GramPair {
  const double* u;
  const double* v;
  int out;
};

void gram_run(const std::vector<GramPair>& pairs, int64_t n, double* out, hipStream_t s) {
  for (size_t base = 0; base < pairs.size(); base += 64) {
    const int count = (int)std::min<size_t>(64, pairs.size() - base);
    MultiDotArgs a{};
    for (int i = 0; i < count; ++i) {
      a.u[i] = pairs[base + i].u;
      a.v[i] = pairs[base + i].v;
    }
    a.count = count;
    a.n = n;
    a.grid = default_grid(n);
    a.partials = primitive_scratch((size_t)count * a.grid);
    // Finalize into a contiguous staging range, then scatter: the outputs of
    // one range are consecutive by construction (pairs are listed in order).
    launch_multidot(a, s);
    launch_finalize(a.partials, a.grid, count, out + pairs[base].out, s);
  }
}
}  // namespace

int kr_gram_kskipmrr_f64(const double* ar, const double* ay, int k, int64_t n, int64_t ld,
                         double* out, void* stream) {
  return guarded([&] {
    KR_REQUIRE(k >= 0 && n >= 0 && ld >= n && out, "bad arguments");
    KR_REQUIRE(n == 0 || (ar && ay), "NULL operand");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int na = 2 * k + 3, nb = 2 * k + 2;
    std::vector<GramPair> pairs;
    for (int j = 0; j < na; ++j)  // alpha[j] = <Ar[j/2], Ar[j/2 + j%2]>
      pairs.push_back({ar + (j / 2) * ld, ar + (j / 2 + j % 2) * ld, j});
    for (int j = 1; j < nb; ++j)  // beta[j] = <Ay[j/2], Ar[j/2 + j%2]>, beta[0] = 0
      pairs.push_back({ay + (j / 2) * ld, ar + (j / 2 + j % 2) * ld, na + j});
    for (int j = 0; j < 2 * k + 1; ++j)  // delta[j] = <Ay[j/2], Ay[j/2 + j%2]>
      pairs.push_back({ay + (j / 2) * ld, ay + (j / 2 + j % 2) * ld, na + nb + j});
    KR_HIP_CHECK(hipMemsetAsync(out + na, 0, sizeof(double), s));
    // alpha (contiguous), then beta[1..] + delta (contiguous from na + 1).
    std::vector<GramPair> first(pairs.begin(), pairs.begin() + na);
    std::vector<GramPair> rest(pairs.begin() + na, pairs.end());
    gram_run(first, n, out, s);
    gram_run(rest, n, out, s);
  });
}

int kr_gram_kskipcg_f64(const double* ar, const double* ap, int k, int64_t n, int64_t ld,
                        double* out, void* stream) {
  return guarded([&] {
    KR_REQUIRE(k >= 0 && n >= 0 && ld >= n && out, "bad arguments");
    KR_REQUIRE(n == 0 || (ar && ap), "NULL operand");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int na = 2 * k + 1, nf = 2 * k + 4, nc = 2 * k + 2;
    std::vector<GramPair> pairs;
    for (int j = 0; j < na; ++j)  // a[j] = <Ar[j/2], Ar[j/2 + j%2]>
      pairs.push_back({ar + (j / 2) * ld, ar + (j / 2 + j % 2) * ld, j});
    for (int j = 0; j < nf - 1; ++j)  // f[j] = <Ap[j/2], Ap[j/2 + j%2]>; f[2k+3] = 0
      pairs.push_back({ap + (j / 2) * ld, ap + (j / 2 + j % 2) * ld, na + j});
    for (int j = 0; j < nc; ++j)  // c[j] = <Ar[j/2], Ap[j/2 + j%2]>
      pairs.push_back({ar + (j / 2) * ld, ap + (j / 2 + j % 2) * ld, na + nf + j});
    KR_HIP_CHECK(hipMemsetAsync(out + na + nf - 1, 0, sizeof(double), s));
    std::vector<GramPair> first(pairs.begin(), pairs.begin() + na + nf - 1);
    std::vector<GramPair> rest(pairs.begin() + na + nf - 1, pairs.end());
    gram_run(first, n, out, s);
    gram_run(rest, n, out, s);
  });
}

int kr_update_mrr_f64(double eta, double zeta, int first, double* y, const double* ar1,
                      double* z, double* r, double* x, int64_t n, void* stream) {
  return guarded([&] {
    KR_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return;
    KR_REQUIRE(y && ar1 && z && r && x, "NULL operand");
    EwArgs a;
    a.c0 = eta;
    a.c1 = zeta;
    a.p[0] = y;
    a.p[1] = const_cast<double*>(ar1);
    a.p[2] = z;
    a.p[3] = r;
    a.p[4] = x;
    a.p[5] = x;
    a.n = n;
    a.grid = default_grid(n);
    a.partials = primitive_scratch(a.grid);
    launch_ew(first ? EW_MRR_FIRST : EW_MRR, a, static_cast<hipStream_t>(stream));
  });
}

int kr_update_cg_f64(double alpha, double* x, const double* p, double* r, const double* v,
                     int64_t n, void* stream) {
  return guarded([&] {
    KR_REQUIRE(n >= 0, "n < 0");
    if (n == 0) return;
    KR_REQUIRE(x && p && r && v, "NULL operand");
    EwArgs a;
    a.c0 = alpha;
    a.p[0] = x;
    a.p[1] = const_cast<double*>(p);
    a.p[2] = r;
    a.p[3] = const_cast<double*>(v);
    a.n = n;
    a.grid = default_grid(n);
    a.partials = primitive_scratch(a.grid);
    launch_ew(EW_CG, a, static_cast<hipStream_t>(stream));
  });
}

int kr_kskipmrr_recurrence(int k, double* alpha, double* beta, double* delta, double* zeta_out,
                           double* eta_out) {
  return guarded([&] {
    KR_REQUIRE(k >= 0 && alpha && beta && delta && zeta_out && eta_out, "bad arguments");
    kskipmrr_recurrence(k, alpha, beta, delta, zeta_out, eta_out);
  });
}

int kr_kskipcg_recurrence(int k, double* a, double* f, double* c, double* alpha_out,
                          double* beta_out) {
  return guarded([&] {
    KR_REQUIRE(k >= 0 && a && f && c && alpha_out && beta_out, "bad arguments");
    kskipcg_recurrence(k, a, f, c, alpha_out, beta_out);
  });
}

int kr_halo_plan(int nshards, const int64_t* part, const int64_t* need_lo,
                 const int64_t* need_hi, int me, int64_t* recv_out, int* nrecv,
                 int64_t* send_out, int* nsend, int cap) {
  return guarded([&] {
    KR_REQUIRE(nshards >= 1 && part && need_lo && need_hi && me >= 0 && me < nshards &&
                   nrecv && nsend,
               "bad arguments");
    std::vector<HaloPiece> recv, send;
    plan_halo(nshards, part, need_lo, need_hi, me, recv, send);
    *nrecv = (int)recv.size();
    *nsend = (int)send.size();
    for (int q = 0; q < (int)recv.size() && q < cap; ++q) {
      recv_out[3 * q] = recv[q].peer;
      recv_out[3 * q + 1] = recv[q].g0;
      recv_out[3 * q + 2] = recv[q].count;
    }
    for (int q = 0; q < (int)send.size() && q < cap; ++q) {
      send_out[3 * q] = send[q].peer;
      send_out[3 * q + 1] = send[q].g0;
      send_out[3 * q + 2] = send[q].count;
    }
  });
}

// ----------------------------------------------------------------- comm
struct kr_comm : Comm {};

int kr_comm_unique_id(uint8_t* id_out) {
  return guarded([&] {
    KR_REQUIRE(id_out, "id_out is NULL");
    static_assert(sizeof(ncclUniqueId) == KR_UNIQUE_ID_BYTES, "unique id size");
    ncclUniqueId id;
    KR_NCCL_CHECK(ncclGetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof(id));
  });
}

int kr_comm_init(kr_comm** comm, const uint8_t* id, int nranks, int rank, int device) {
  return guarded([&] {
    KR_REQUIRE(comm && id && nranks >= 1 && rank >= 0 && rank < nranks, "bad arguments");
    auto c = std::make_unique<kr_comm>();
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    KR_HIP_CHECK(hipSetDevice(device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    KR_NCCL_CHECK(ncclCommInitRank(&c->nccl, nranks, uid, rank));
    *comm = c.release();
  });
}

int kr_comm_destroy(kr_comm* comm) {
  return guarded([&] {
    if (!comm) return;
    if (comm->nccl) ncclCommDestroy(comm->nccl);
    delete comm;
  });
}

int kr_allreduce_sum_f64(kr_comm* comm, double* buf, int64_t count, void* stream) {
  return guarded([&] {
    KR_REQUIRE(comm && count >= 0, "bad arguments");
    if (count == 0) return;
    KR_REQUIRE(buf, "NULL operand");
    if (comm->nranks == 1 || !comm->nccl) return;  // one rank: the sum is the buffer
    KR_NCCL_CHECK(ncclAllReduce(buf, buf, (size_t)count, ncclDouble, ncclSum, comm->nccl,
                                static_cast<hipStream_t>(stream)));
  });
}

int kr_halo_exchange_f64(kr_comm* comm, double* x, const int64_t* recv, int nrecv,
                         const int64_t* send, int nsend, void* stream) {
  return guarded([&] {
    KR_REQUIRE(comm && nrecv >= 0 && nsend >= 0, "bad arguments");
    KR_REQUIRE((nrecv == 0 || recv) && (nsend == 0 || send), "NULL piece list");
    if (nrecv + nsend == 0) return;
    KR_REQUIRE(x, "NULL operand");
    KR_REQUIRE(comm->nccl, "communicator has no RCCL handle");
    for (int q = 0; q < nrecv; ++q)
      KR_REQUIRE(recv[3 * q] >= 0 && recv[3 * q] < comm->nranks && recv[3 * q + 1] >= 0 &&
                     recv[3 * q + 2] >= 0,
                 "bad receive piece");
    for (int q = 0; q < nsend; ++q)
      KR_REQUIRE(send[3 * q] >= 0 && send[3 * q] < comm->nranks && send[3 * q + 1] >= 0 &&
                     send[3 * q + 2] >= 0,
                 "bad send piece");
    hipStream_t s = static_cast<hipStream_t>(stream);
    KR_NCCL_CHECK(ncclGroupStart());
    for (int q = 0; q < nsend; ++q)
      KR_NCCL_CHECK(ncclSend(x + send[3 * q + 1], (size_t)send[3 * q + 2], ncclDouble,
                             (int)send[3 * q], comm->nccl, s));
    for (int q = 0; q < nrecv; ++q)
      KR_NCCL_CHECK(ncclRecv(x + recv[3 * q + 1], (size_t)recv[3 * q + 2], ncclDouble,
                             (int)recv[3 * q], comm->nccl, s));
    KR_NCCL_CHECK(ncclGroupEnd());
  });
}

// ----------------------------------------------------------------- system
struct kr_system : System {};

int kr_system_create(kr_system** out, int64_t n_global, int nshards, const int* devices,
                     const int64_t* row_begin, kr_comm* comm) {
  return guarded([&] {
    KR_REQUIRE(out && devices && row_begin && nshards >= 1 && n_global >= 0, "bad arguments");
    if (comm) KR_REQUIRE(nshards <= kMaxLocal, "too many local shards for one rank");
    for (int s = 0; s < nshards; ++s)
      KR_REQUIRE(row_begin[s] <= row_begin[s + 1], "row_begin must be non-decreasing");
    auto sys = std::make_unique<kr_system>();
    sys->n_global = n_global;
    sys->comm = comm;
    sys->shards.resize(nshards);
    // In-process shards on one device share that device's stream (System::
    // groups). KR_SHARED_STREAM: 1 (default) all of a device's shards, 0 a
    // stream per shard (A/B), g >= 2 runs of g consecutive shards (tests:
    // several stream groups on one device, as several devices would have).
    // With a communicator every local shard keeps its own (the hybrid RCCL paths).
    const int ss = KR_ENV("KR_SHARED_STREAM", 1);
    const bool share = !comm && ss != 0;
    const int run = ss >= 2 ? ss : nshards;
    for (int s = 0; s < nshards; ++s) {
      Shard& sh = sys->shards[s];
      sh.dev = devices[s];
      sh.row0 = row_begin[s];
      sh.n = row_begin[s + 1] - row_begin[s];
      KR_HIP_CHECK(hipSetDevice(sh.dev));
      for (int t = 0; share && t < s && !sh.stream; ++t)
        if (sys->shards[t].dev == sh.dev && t / run == s / run) sh.stream = sys->shards[t].stream;
      if (!sh.stream) KR_HIP_CHECK(hipStreamCreateWithFlags(&sh.stream, hipStreamNonBlocking));
    }
    if (comm) {
      // global partition from every rank's local shards: record = [count,
      // boundaries...], kMaxLocal + 2 int64 per rank, in rank order
      Shard& sh = sys->shards[0];
      const int R = comm->nranks;
      constexpr int W = kMaxLocal + 2;
      int64_t* d = nullptr;
      KR_HIP_CHECK(hipSetDevice(sh.dev));
      KR_HIP_CHECK(hipMalloc(&d, sizeof(int64_t) * W * (1 + R)));
      std::vector<int64_t> mine(W, 0);
      mine[0] = nshards;
      for (int s = 0; s <= nshards; ++s) mine[1 + s] = row_begin[s];
      KR_HIP_CHECK(hipMemcpy(d, mine.data(), sizeof(int64_t) * W, hipMemcpyHostToDevice));
      KR_NCCL_CHECK(ncclAllGather(d, d + W, W, ncclInt64, comm->nccl, sh.stream));
      std::vector<int64_t> all((size_t)W * R);
      KR_HIP_CHECK(hipMemcpyAsync(all.data(), d + W, sizeof(int64_t) * W * R,
                                  hipMemcpyDeviceToHost, sh.stream));
      KR_HIP_CHECK(hipStreamSynchronize(sh.stream));
      KR_HIP_CHECK(hipFree(d));
      sys->part.assign(1, 0);
      sys->rank_first.assign(1, 0);
      sys->owner.clear();
      for (int r = 0; r < R; ++r) {
        const int64_t* rec = &all[(size_t)W * r];
        const int cnt = (int)rec[0];
        KR_REQUIRE(cnt >= 1 && cnt <= kMaxLocal, "bad local shard count of a rank");
        KR_REQUIRE(rec[1] == sys->part.back(),
                   "rank row blocks must be contiguous and in rank order");
        for (int s = 0; s < cnt; ++s) {
          sys->part.push_back(rec[2 + s]);
          sys->owner.push_back(r);
        }
        sys->rank_first.push_back((int)sys->owner.size());
      }
      KR_REQUIRE(sys->part.back() == n_global, "rank row blocks must cover n_global");
      sys->first_global = sys->rank_first[comm->rank];
    } else {
      KR_REQUIRE(row_begin[0] == 0 && row_begin[nshards] == n_global,
                 "in-process shards must cover [0, n_global)");
      sys->part.assign(row_begin, row_begin + nshards + 1);
      sys->first_global = 0;
    }
    {
      // peer access between the distinct devices of the local shards (best
      // effort; halo copies and, with a communicator, the RCCL transfers of
      // shards on other devices than the first go through it)
      for (int a = 0; a < nshards; ++a)
        for (int b = 0; b < nshards; ++b) {
          const int da = devices[a], db = devices[b];
          if (da == db) continue;
          int can = 0;
          if (hipDeviceCanAccessPeer(&can, da, db) == hipSuccess && can) {
            (void)hipSetDevice(da);
            hipError_t e = hipDeviceEnablePeerAccess(db, 0);
            (void)e;
            if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
          }
        }
    }
    *out = sys.release();
  });
}

int kr_system_destroy(kr_system* sys) {
  return guarded([&] { delete sys; });
}

int kr_system_adopt_csr(kr_system* sys, int shard, const void* rowptr, int rowptr64,
                        int32_t* col, const double* val) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    KR_REQUIRE(!sys->finalized, "system already finalized");
    KR_REQUIRE(rowptr && col && val, "NULL CSR operand");
    Shard& s = sys->shards[shard];
    s.rowptr = rowptr;
    s.rowptr64 = rowptr64;
    s.col = col;
    s.val = val;
  });
}

}  // extern "C"

namespace {
void* dmalloc(Shard& s, size_t bytes) {
  void* p = nullptr;
  if (hipMalloc(&p, bytes ? bytes : 8) != hipSuccess)
    throw Failure(KR_ERR_NOMEM, "matrix allocation failed");
  s.owned.push_back(p);
  fresh_fill(p, bytes, s.stream);  // KR_POISON_ALLOC: the generators must write every entry
  return p;
}

template <class Count, class Fill>
void generate(kr_system* sys, int rowptr64_req, int max_row_nnz, Count count, Fill fill) {
  KR_REQUIRE(sys && !sys->finalized, "bad system state");
  for (auto& s : sys->shards) {
    KR_HIP_CHECK(hipSetDevice(s.dev));
    const int rp64 = rowptr64_req || (double)s.n * max_row_nnz >= 2147483647.0;
    const size_t rpb = rp64 ? 8 : 4;
    void* rp = dmalloc(s, rpb * (size_t)(s.n + 1));
    KR_HIP_CHECK(hipMemsetAsync(rp, 0, rpb, s.stream));
    count(s, rp, rp64);
    rowptr_scan(rp, rp64, s.n, s.stream);
    int64_t nnz = 0;
    if (rp64) {
      KR_HIP_CHECK(hipMemcpy(&nnz, (int64_t*)rp + s.n, 8, hipMemcpyDeviceToHost));
    } else {
      int32_t v = 0;
      KR_HIP_CHECK(hipMemcpy(&v, (int32_t*)rp + s.n, 4, hipMemcpyDeviceToHost));
      nnz = v;
    }
    int32_t* col = (int32_t*)dmalloc(s, 4 * (size_t)nnz);
    double* val = (double*)dmalloc(s, 8 * (size_t)nnz);
    fill(s, rp, rp64, col, val);
    KR_HIP_CHECK(hipStreamSynchronize(s.stream));
    s.rowptr = rp;
    s.rowptr64 = rp64;
    s.col = col;
    s.val = val;
    s.nnz = nnz;
  }
}

}  // namespace

extern "C" {

int kr_system_adopt_dense(kr_system* sys, int shard, const double* a, int64_t ld) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    KR_REQUIRE(!sys->finalized, "system already finalized");
    KR_REQUIRE(ld >= sys->n_global, "leading dimension < n_global");
    Shard& s = sys->shards[shard];
    KR_REQUIRE(a || s.n == 0, "NULL dense block");
    s.dense = a;
    s.dld = ld;
  });
}

int kr_system_gen_poisson(kr_system* sys, int dim, int64_t n_side) {
  return guarded([&] {
    KR_REQUIRE(dim == 2 || dim == 3, "dim must be 2 or 3");
    KR_REQUIRE(n_side >= 1, "n_side must be positive");
    // n_global = n_side^(dim-1) * nz: the cube (nz = n_side), or a box of nz
    // planes (outermost dimension), e.g. one rank's slab of a larger cube
    int64_t plane = 1;
    for (int d = 0; d < dim - 1; ++d) plane *= n_side;
    KR_REQUIRE(sys->n_global % plane == 0, "n_global must be n_side^(dim-1) * nz");
    const int64_t nz = sys->n_global / plane;
    generate(
        sys, 0, 2 * dim + 1,
        [&](Shard& s, void* rp, int rp64) {
          launch_poisson_count(dim, n_side, nz, s.row0, s.n, rp, rp64, s.stream);
        },
        [&](Shard& s, void* rp, int rp64, int32_t* col, double* val) {
          launch_poisson_fill(dim, n_side, nz, s.row0, s.n, rp, rp64, col, val, s.stream);
        });
  });
}

int kr_system_gen_banded(kr_system* sys, int h, int64_t width, uint64_t seed, int rowptr64) {
  return guarded([&] {
    KR_REQUIRE(h >= 1 && h <= 64 && width >= h, "need 1 <= h <= 64 and h <= width");
    BandSpec b{};
    b.h = h;
    b.seed = seed;
    b.n_global = sys->n_global;
    banded_offsets(h, width, seed, b.off);
    generate(
        sys, rowptr64, 2 * h + 1,
        [&](Shard& s, void* rp, int rp64) {
          launch_banded_count(b, s.row0, s.n, rp, rp64, s.stream);
        },
        [&](Shard& s, void* rp, int rp64, int32_t* col, double* val) {
          launch_banded_fill(b, s.row0, s.n, rp, rp64, col, val, s.stream);
        });
  });
}

int kr_system_finalize(kr_system* sys) {
  return guarded([&] {
    KR_REQUIRE(sys, "NULL system");
    sys->finalize();
  });
}

int kr_system_shard_info(kr_system* sys, int shard, int64_t* n_local, int64_t* halo_lo,
                         int64_t* halo_hi, int64_t* nnz) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    const Shard& s = sys->shards[shard];
    if (n_local) *n_local = s.n;
    if (halo_lo) *halo_lo = s.halo_lo;
    if (halo_hi) *halo_hi = s.halo_hi;
    if (nnz) *nnz = s.nnz;
  });
}

int kr_system_shard_layout(kr_system* sys, int shard, int* mask_bits, int* n_offsets,
                           int64_t* interior_lo, int64_t* interior_hi) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    KR_REQUIRE(sys->finalized, "system not finalized");
    const Shard& s = sys->shards[shard];
    if (mask_bits) *mask_bits = s.mask ? s.mw : 0;
    if (n_offsets) *n_offsets = s.mask ? s.nm : 0;
    if (interior_lo) *interior_lo = s.int_lo;
    if (interior_hi) *interior_hi = s.int_hi;
  });
}

int kr_system_shard_values(kr_system* sys, int shard, int* dict_values) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    KR_REQUIRE(sys->finalized, "system not finalized");
    if (dict_values) *dict_values = sys->shards[shard].vcode ? sys->shards[shard].ntab : 0;
  });
}

int kr_system_shard_codes(kr_system* sys, int shard, int* code_bits) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    KR_REQUIRE(sys->finalized, "system not finalized");
    const Shard& s = sys->shards[shard];
    if (code_bits) *code_bits = s.scode ? s.st_cb : 0;
  });
}

int kr_system_shard_code_patterns(kr_system* sys, int shard, int* patterns) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    KR_REQUIRE(sys->finalized, "system not finalized");
    const Shard& s = sys->shards[shard];
    if (patterns) *patterns = s.scode && s.st_pid ? s.st_npat : 0;
  });
}

int kr_system_shard_box(kr_system* sys, int shard, int* box) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    KR_REQUIRE(sys->finalized, "system not finalized");
    if (box) *box = sys->shards[shard].st_box ? 1 : 0;
  });
}

int kr_system_shard_dia_full_blocks(kr_system* sys, int shard, int64_t* first, int64_t* count) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    KR_REQUIRE(sys->finalized, "system not finalized");
    const Shard& s = sys->shards[shard];
    const bool on = s.dia && s.dia_walk;
    if (first) *first = on ? s.dia_full_lo : 0;
    if (count) *count = on ? s.dia_full_hi - s.dia_full_lo : 0;
  });
}

int kr_system_shard_dia_sym(kr_system* sys, int shard, int* sym) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    KR_REQUIRE(sys->finalized, "system not finalized");
    const Shard& s = sys->shards[shard];
    if (sym) *sym = s.dia && s.dia_sym ? 1 : 0;
  });
}

int kr_system_shard_sched(kr_system* sys, int shard, int* grid, int* spmv_grid,
                          int* stencil_walk, int* format) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    KR_REQUIRE(sys->finalized, "system not finalized");
    if (grid) *grid = sys->shards[shard].grid;
    if (spmv_grid) *spmv_grid = sys->shards[shard].spmv_grid;
    const Shard& s = sys->shards[shard];
    if (stencil_walk) *stencil_walk = s.scode ? s.st_P : 0;
    if (format)
      *format = s.dense ? KR_FORMAT_DENSE
                : s.scode ? KR_FORMAT_STENCIL
                : s.dia   ? (s.dia_walk ? KR_FORMAT_DIA_WALK : KR_FORMAT_DIA)
                          : KR_FORMAT_CSR;
  });
}

int kr_system_csr(kr_system* sys, int shard, const void** rowptr, int* rowptr64,
                  const int32_t** col, const double** val, int64_t* pad) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    const Shard& s = sys->shards[shard];
    if (rowptr) *rowptr = s.rowptr;
    if (rowptr64) *rowptr64 = s.rowptr64;
    if (col) *col = s.col;
    if (val) *val = s.val;
    if (pad) *pad = s.pad;
  });
}

int kr_fill_rhs(kr_system* sys, int shard, uint64_t seed, double* b) {
  return guarded([&] {
    KR_REQUIRE(sys && shard >= 0 && shard < (int)sys->shards.size(), "bad shard");
    Shard& s = sys->shards[shard];
    KR_HIP_CHECK(hipSetDevice(s.dev));
    launch_fill_rhs(seed, s.row0, s.n, b, s.stream);
    KR_HIP_CHECK(hipStreamSynchronize(s.stream));
  });
}

int kr_system_spmv(kr_system* sys, const double* const* x, double* const* y) {
  return guarded([&] {
    KR_REQUIRE(sys && sys->finalized, "system not finalized");
    KR_REQUIRE(x && y, "NULL operand");
    sys->session.reset();
    sys->alloc_vectors(2);
    for (size_t li = 0; li < sys->shards.size(); ++li) {
      Shard& s = sys->shards[li];
      KR_HIP_CHECK(hipSetDevice(s.dev));
      KR_HIP_CHECK(hipMemcpyAsync(s.own(0), x[li], 8 * (size_t)s.n, hipMemcpyDeviceToDevice,
                                  s.stream));
    }
    sys->spmv(EPI_NONE, 0, -1, 1, -1, -1, -1, 0);
    for (size_t li = 0; li < sys->shards.size(); ++li) {
      Shard& s = sys->shards[li];
      KR_HIP_CHECK(hipSetDevice(s.dev));
      KR_HIP_CHECK(hipMemcpyAsync(y[li], s.own(1), 8 * (size_t)s.n, hipMemcpyDeviceToDevice,
                                  s.stream));
    }
    for (auto& s : sys->shards) {
      KR_HIP_CHECK(hipSetDevice(s.dev));
      KR_HIP_CHECK(hipStreamSynchronize(s.stream));
    }
  });
}

// ----------------------------------------------------------------- solver
int kr_solve_begin(kr_system* sys, const kr_solve_params* params, const double* const* b,
                   const double* const* x0) {
  return guarded([&] {
    KR_REQUIRE(sys && params, "NULL argument");
    if (!sys->finalized) throw Failure(KR_ERR_STATE, "kr_system_finalize was not called");
    sys->session.reset();
    sys->kstats.clear();
    sys->profile = params->profile != 0;
    sys->profile_every = params->profile > 0 ? params->profile : 1;
    sys->prof_tick = 0;
    sys->prof_active = true;
    sys->session = make_session(sys, *params);
    sys->session->begin(b, x0);
  });
}

int kr_solve_set_precond(kr_system* sys, const double* const* d) {
  return guarded([&] {
    KR_REQUIRE(sys && sys->finalized, "system not finalized");
    sys->precond.clear();
    sys->ilu.reset();  // the last preconditioner set wins
    if (d) sys->precond.assign(d, d + sys->shards.size());
  });
}

int kr_solve_set_precond_ilu(kr_system* sys, int64_t n, const int64_t* l_rowptr,
                             const int32_t* l_col, const double* l_val, const int64_t* u_rowptr,
                             const int32_t* u_col, const double* u_val, const int64_t* perm_r,
                             const int64_t* perm_c) {
  return guarded([&] {
    KR_REQUIRE(sys && sys->finalized, "system not finalized");
    if (!l_rowptr) {  // clear
      sys->ilu.reset();
      return;
    }
    KR_REQUIRE(l_col && l_val && u_rowptr && u_col && u_val && perm_r && perm_c, "NULL argument");
    // the sweeps run over the whole vector in one workgroup: one shard, one rank
    KR_REQUIRE(sys->shards.size() == 1 && sys->nglobal_shards() == 1,
               "ILU preconditioning needs a one-shard system (the triangular sweeps are "
               "sequential over the whole vector)");
    KR_REQUIRE(n == sys->n_global, "ILU: factor size differs from the system size");
    Shard& s = sys->shards[0];
    sys->ilu = build_ilu(s.dev, s.stream, n, l_rowptr, l_col, l_val, u_rowptr, u_col, u_val,
                         perm_r, perm_c);
    sys->precond.clear();  // the last preconditioner set wins
  });
}

int kr_solve_step(kr_system* sys, int64_t max_outer, int* done) {
  return guarded<false>([&] {
    KR_REQUIRE(sys, "NULL system");
    if (!sys->session) throw Failure(KR_ERR_STATE, "kr_solve_begin was not called");
    Session& ss = *sys->session;
    for (int64_t c = 0; c < max_outer && !ss.done; ++c) {
      // profile = N: per-kernel events on every N-th outer iteration only
      sys->prof_active = (sys->prof_tick++ % sys->profile_every) == 0;
      ss.hint = max_outer - c;
      const double t0 = now_seconds(), w0 = sys->host_wait_s;
      ss.step_once();
      if (sys->profile) {  // host side of every outer iteration (profiled or not)
        const double wait = sys->host_wait_s - w0;
        auto& st = sys->kstats;
        st["host_enqueue"].launches += 1;
        st["host_enqueue"].total_ms += (now_seconds() - t0 - wait) * 1e3;
        st["host_wait"].launches += 1;
        st["host_wait"].total_ms += wait * 1e3;
      }
    }
    if (done) *done = ss.done ? 1 : 0;
  });
}

int kr_solve_end(kr_system* sys, double* const* x, kr_solve_result* res) {
  return guarded([&] {
    KR_REQUIRE(sys, "NULL system");
    if (!sys->session) throw Failure(KR_ERR_STATE, "kr_solve_begin was not called");
    Session& ss = *sys->session;
    ss.settle();
    for (auto& s : sys->shards) {
      KR_HIP_CHECK(hipSetDevice(s.dev));
      KR_HIP_CHECK(hipStreamSynchronize(s.stream));
    }
    ss.t_end = now_seconds();
    sys->harvest_profile();
    if (res) {
      res->time_s = ss.t_end - ss.t_start;
      res->iterations = ss.i;
      res->entries = ss.entries();
      res->converged = ss.converged ? 1 : 0;
      res->final_k = ss.k;
      res->final_residual = ss.residual.empty() ? 0.0 : ss.residual[ss.index];
      res->diverged = ss.diverged ? 1 : 0;
    }
    if (x) {
      const int id = ss.result_x();
      for (size_t li = 0; li < sys->shards.size(); ++li) {
        Shard& s = sys->shards[li];
        if (!x[li]) continue;
        KR_HIP_CHECK(hipSetDevice(s.dev));
        KR_HIP_CHECK(hipMemcpyAsync(x[li], s.own(id), 8 * (size_t)s.n, hipMemcpyDeviceToDevice,
                                    s.stream));
        KR_HIP_CHECK(hipStreamSynchronize(s.stream));
      }
    }
  });
}

int kr_solve_history(kr_system* sys, double* residual, int64_t* nosl, int64_t* khistory,
                     int64_t capacity) {
  return guarded([&] {
    KR_REQUIRE(sys && sys->session, "no session");
    Session& ss = *sys->session;
    const int64_t n = std::min<int64_t>(capacity, ss.entries());
    for (int64_t q = 0; q < n; ++q) {
      if (residual) residual[q] = q < (int64_t)ss.residual.size() ? ss.residual[q] : 0.0;
      if (nosl) nosl[q] = q < (int64_t)ss.nosl.size() ? ss.nosl[q] : 0;
      if (khistory) khistory[q] = q < (int64_t)ss.khist.size() ? ss.khist[q] : 0;
    }
  });
}

int kr_solve_kernel_stats(kr_system* sys, kr_kernel_stat* stats, int cap, int* count) {
  return guarded([&] {
    KR_REQUIRE(sys && count, "NULL argument");
    sys->harvest_profile();  // events still pending (harvested lazily, see reduce)
    int c = 0;
    if (!sys->shards.empty()) {
      for (auto& kv : sys->kstats) {
        if (c < cap && stats) {
          std::memset(&stats[c], 0, sizeof(kr_kernel_stat));
          std::strncpy(stats[c].name, kv.first.c_str(), sizeof(stats[c].name) - 1);
          stats[c].launches = kv.second.launches;
          stats[c].total_ms = kv.second.total_ms;
          stats[c].bytes_per_launch = kv.second.bytes;
          stats[c].shards = kv.second.shards;
        }
        ++c;
      }
    }
    *count = c;
  });
}

int kr_solve_kernel_stats_reset(kr_system* sys) {
  return guarded([&] {
    KR_REQUIRE(sys, "NULL system");
    sys->harvest_profile();
    sys->kstats.clear();
    // restart the every-N-th sampling with the next outer iteration, so a
    // window of K steps after a reset samples exactly ceil(K / N) of them
    sys->prof_tick = 0;
  });
}

}  // extern "C"

// ------------------------------------------------------------------ helpers
namespace kr {

uint64_t splitmix64(uint64_t x);

void banded_offsets(int h, int64_t width, uint64_t seed, int64_t* out_sorted) {
  // Partial Fisher-Yates over [1, width] driven by the counter hash; the
  // numpy oracle (oracle/matrices.py) restates it integer for integer.
  std::vector<int64_t> pool(width);
  for (int64_t t = 0; t < width; ++t) pool[t] = t + 1;
  for (int t = 0; t < h; ++t) {
    const uint64_t r = splitmix64(seed * 0x2545F4914F6CDD1Dull + (uint64_t)t);
    const int64_t j = t + (int64_t)(r % (uint64_t)(width - t));
    std::swap(pool[t], pool[j]);
  }
  std::vector<int64_t> pick(pool.begin(), pool.begin() + h);
  std::sort(pick.begin(), pick.end());
  for (int t = 0; t < h; ++t) out_sorted[t] = pick[t];
}

uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

}  // namespace kr
