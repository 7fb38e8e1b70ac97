// Plain-CSR dual SpMV microbenchmark (C4's csr sub-record: 512^3 7-point
// Poisson, int32 rowptr/col, fp64 values, two input vectors, EPI_DUAL_MRR's
// seven Gram products). Builds the matrix on the device, runs each kernel
// variant of the library's own headers (kr_spmv.h, instantiated here), checks
// y1 / y2 bitwise against a one-thread-per-row reference (scipy's order), and
// times it with HIP events. Rates are SURVEY.md 8(d)'s CSR bytes per launch
// (12 nnz + 4 (N+1) + 32 N) over the average launch time.
//
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -x hip \
//     -I/opt/rocm/include -o tools/micro/csr_micro tools/micro/csr_micro.cpp
//   tools/micro/csr_micro [n_side=512] [reps=20] [variant ...]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../parallel-krylov_amd/csrc/kr_spmv.h"
#include "csr_variants.h"

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      printf("%s -> %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

using namespace kr;

__global__ void gen_poisson(const int32_t* __restrict__ rp, int32_t* __restrict__ col,
                            double* __restrict__ val, int64_t ns) {
  const int64_t n = ns * ns * ns;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = i % ns, y = (i / ns) % ns, z = i / (ns * ns);
    int64_t p = rp[i];
    auto put = [&](int64_t c, double v) {
      col[p] = (int32_t)c;
      val[p] = v;
      ++p;
    };
    // distinct values per entry (no special structure the kernels could use)
    const double h = 1.0 + (double)((i * 2654435761u) & 1023) * (1.0 / 4096.0);
    if (z > 0) put(i - ns * ns, -h * 0.5);
    if (y > 0) put(i - ns, -h * 0.25);
    if (x > 0) put(i - 1, -h * 0.125);
    put(i, 6.0 * h);
    if (x < ns - 1) put(i + 1, -h * 0.375);
    if (y < ns - 1) put(i + ns, -h * 0.625);
    if (z < ns - 1) put(i + ns * ns, -h * 0.875);
  }
}

__global__ void fill_vec(double* v, int64_t n, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull ^ seed;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    v[i] = (double)(h >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
  }
}

__global__ void ref_spmv2(const int32_t* __restrict__ rp, const int32_t* __restrict__ col,
                          const double* __restrict__ val, const double* __restrict__ x1,
                          const double* __restrict__ x2, double* y1, double* y2, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double s1 = 0.0, s2 = 0.0;
    for (int64_t j = rp[i]; j < rp[i + 1]; ++j) {
      s1 = s1 + val[j] * x1[col[j]];
      s2 = s2 + val[j] * x2[col[j]];
    }
    y1[i] = s1;
    y2[i] = s2;
  }
}

__global__ void count_diff(const double* a, const double* b, int64_t n,
                           unsigned long long* cnt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (__double_as_longlong(a[i]) != __double_as_longlong(b[i])) atomicAdd(cnt, 1ull);
  }
}

// The same bytes as the dual SpMV as plain streams: col, val, rowptr, x1, x2
// read with 16-byte loads, y1 and y2 written (RW = 0: reads only).
template <int RW>
__global__ __launch_bounds__(256) void stream_ref(const int4v* __restrict__ c, int64_t nc,
                                                  const dbl2v* __restrict__ v, int64_t nv,
                                                  const int4v* __restrict__ r, int64_t nr,
                                                  const dbl2v* __restrict__ x1,
                                                  const dbl2v* __restrict__ x2, dbl2v* y1,
                                                  dbl2v* y2, int64_t nx, double* sink) {
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t st = (int64_t)gridDim.x * blockDim.x;
  double acc = 0.0;
  int iacc = 0;
  for (int64_t i = t0; i < nv; i += st) {
    const dbl2v a = __builtin_nontemporal_load(v + i);
    acc += a.x + a.y;
  }
  for (int64_t i = t0; i < nc; i += st) {
    const int4v a = __builtin_nontemporal_load(c + i);
    iacc += a.x ^ a.w;
  }
  for (int64_t i = t0; i < nr; i += st) {
    const int4v a = r[i];
    iacc += a.y;
  }
  for (int64_t i = t0; i < nx; i += st) {
    const dbl2v a = x1[i], b = x2[i];
    if constexpr (RW) {
      y1[i] = a + b;
      y2[i] = a - b;
    } else {
      acc += a.x + b.y;
    }
  }
  if (acc == 12345.0 && iacc == 7) sink[0] = acc;
}

struct Ctx {
  int64_t ns, n, nnz;
  int32_t *rp, *col;
  double *val, *x1, *x2, *y1, *y2, *r1, *r2, *part;
  unsigned long long* cnt;
  double bytes;
  int reps;
};

template <typename F>
float time_it(const Ctx& c, F launch) {
  launch();
  CK(hipDeviceSynchronize());
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  CK(hipEventRecord(s));
  for (int r = 0; r < c.reps; ++r) launch();
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, s, e));
  CK(hipEventDestroy(s));
  CK(hipEventDestroy(e));
  return ms / c.reps;
}

unsigned long long diffs(const Ctx& c) {
  CK(hipMemset(c.cnt, 0, 8));
  count_diff<<<4096, 256>>>(c.y1, c.r1, c.n, c.cnt);
  count_diff<<<4096, 256>>>(c.y2, c.r2, c.n, c.cnt);
  unsigned long long h = 0;
  CK(hipMemcpy(&h, c.cnt, 8, hipMemcpyDeviceToHost));
  return h;
}

SpmvArgs args_for(const Ctx& c, int grid) {
  SpmvArgs a;
  a.rowptr = c.rp;
  a.col = c.col;
  a.val = c.val;
  a.n = c.n;
  a.x1 = c.x1;
  a.x2 = c.x2;
  a.y1 = c.y1;
  a.y2 = c.y2;
  a.partials = c.part;
  a.grid = grid;
  a.nnz_total = c.nnz;
  a.nt_stores = 1;  // the engine's choice for a shard this size
  return a;
}

void report(const Ctx& c, const char* name, int grid, float ms) {
  const unsigned long long d = diffs(c);
  printf("%-34s grid %6d  %8.4f ms  %7.1f GB/s  frac %.4f  diffs %llu\n", name, grid, ms,
         c.bytes / ms * 1e-6, c.bytes / ms * 1e-6 / 8000.0, d);
  fflush(stdout);
}

template <int E, int DB, int NT>
void run_k2(Ctx& c, int grid, const char* name) {
  CK(hipMemset(c.y1, 0, c.n * 8));
  CK(hipMemset(c.y2, 0, c.n * 8));
  SpmvArgs a = args_for(c, grid);
  const float ms = time_it(c, [&] {
    spmv_kernel2<int32_t, E, true, 0, DB, NT, false><<<grid, kBlock>>>(a);
  });
  report(c, name, grid, ms);
}

template <int E, int PS>
void run_prod2(Ctx& c, int grid, const char* name) {
  CK(hipMemset(c.y1, 0, c.n * 8));
  CK(hipMemset(c.y2, 0, c.n * 8));
  SpmvArgs a = args_for(c, grid);
  const float ms = time_it(c, [&] {
    spmv_kernel_prod2<int32_t, E, true, true, PS><<<grid, kBlock>>>(a);
  });
  report(c, name, grid, ms);
}

template <int E, int KC, bool NT, int AB = 0>
void run_direct(Ctx& c, int grid, const char* name) {
  CK(hipMemset(c.y1, 0, c.n * 8));
  CK(hipMemset(c.y2, 0, c.n * 8));
  SpmvArgs a = args_for(c, grid);
  const float ms = time_it(c, [&] {
    spmv_kernel_direct<int32_t, E, KC, NT, AB><<<grid, kBlock>>>(a);
  });
  report(c, name, grid, ms);
}

template <int E, int FL>
void run_k3(Ctx& c, int grid, const char* name) {
  CK(hipMemset(c.y1, 0, c.n * 8));
  CK(hipMemset(c.y2, 0, c.n * 8));
  SpmvArgs a = args_for(c, grid);
  const float ms = time_it(c, [&] {
    spmv_kernel3<int32_t, E, FL><<<grid, kBlock>>>(a);
  });
  report(c, name, grid, ms);
}

template <int E, int FL>
void run_k4(Ctx& c, int grid, const char* name) {
  CK(hipMemset(c.y1, 0, c.n * 8));
  CK(hipMemset(c.y2, 0, c.n * 8));
  SpmvArgs a = args_for(c, grid);
  const float ms = time_it(c, [&] {
    spmv_kernel4<int32_t, E, FL><<<grid, kBlock>>>(a);
  });
  report(c, name, grid, ms);
}

template <int E, bool VL = false>
void run_k5(Ctx& c, int grid, const char* name) {
  CK(hipMemset(c.y1, 0, c.n * 8));
  CK(hipMemset(c.y2, 0, c.n * 8));
  SpmvArgs a = args_for(c, grid);
  const float ms = time_it(c, [&] {
    spmv_kernel5<int32_t, E, VL><<<grid, kBlock>>>(a);
  });
  report(c, name, grid, ms);
}

int main(int argc, char** argv) {
  Ctx c;
  c.ns = argc > 1 ? atoll(argv[1]) : 512;
  c.reps = argc > 2 ? atoi(argv[2]) : 20;
  std::vector<std::string> want;
  for (int i = 3; i < argc; ++i) want.push_back(argv[i]);
  auto on = [&](const char* v) {
    if (want.empty()) return true;
    for (auto& w : want)
      if (w == v) return true;
    return false;
  };
  c.n = c.ns * c.ns * c.ns;
  std::vector<int32_t> hrp(c.n + 1);
  int64_t p = 0;
  for (int64_t i = 0; i < c.n; ++i) {
    hrp[i] = (int32_t)p;
    const int64_t x = i % c.ns, y = (i / c.ns) % c.ns, z = i / (c.ns * c.ns);
    p += 1 + (x > 0) + (x < c.ns - 1) + (y > 0) + (y < c.ns - 1) + (z > 0) + (z < c.ns - 1);
  }
  hrp[c.n] = (int32_t)p;
  c.nnz = p;
  c.bytes = 12.0 * c.nnz + 4.0 * (c.n + 1) + 32.0 * c.n;
  printf("n %lld nnz %lld bytes/launch %.3f GB\n", (long long)c.n, (long long)c.nnz, c.bytes * 1e-9);
  CK(hipMalloc(&c.rp, (c.n + 4) * 4));
  CK(hipMalloc(&c.col, (c.nnz + 8) * 4));
  CK(hipMalloc(&c.val, (c.nnz + 8) * 8));
  for (double** v : {&c.x1, &c.x2, &c.y1, &c.y2, &c.r1, &c.r2}) CK(hipMalloc(v, (c.n + 8) * 8));
  CK(hipMalloc(&c.part, 16 * 65536 * 8));
  CK(hipMalloc(&c.cnt, 8));
  CK(hipMemcpy(c.rp, hrp.data(), (c.n + 1) * 4, hipMemcpyHostToDevice));
  std::vector<int32_t>().swap(hrp);
  gen_poisson<<<8192, 256>>>(c.rp, c.col, c.val, c.ns);
  fill_vec<<<4096, 256>>>(c.x1, c.n, 1);
  fill_vec<<<4096, 256>>>(c.x2, c.n, 2);
  ref_spmv2<<<8192, 256>>>(c.rp, c.col, c.val, c.x1, c.x2, c.r1, c.r2, c.n);
  CK(hipDeviceSynchronize());

  const int g8 = 8192;
  if (on("stream")) {
    const float ms = time_it(c, [&] {
      stream_ref<1><<<2048, 256>>>((const int4v*)c.col, c.nnz / 4, (const dbl2v*)c.val, c.nnz / 2,
                                   (const int4v*)c.rp, c.n / 4, (const dbl2v*)c.x1,
                                   (const dbl2v*)c.x2, (dbl2v*)c.y1, (dbl2v*)c.y2, c.n / 2, c.part);
    });
    printf("%-34s grid %6d  %8.4f ms  %7.1f GB/s  frac %.4f\n", "stream rw (same bytes)", 2048, ms,
           c.bytes / ms * 1e-6, c.bytes / ms * 1e-6 / 8000.0);
    const double rb = c.bytes - 16.0 * c.n;
    const float ms2 = time_it(c, [&] {
      stream_ref<0><<<2048, 256>>>((const int4v*)c.col, c.nnz / 4, (const dbl2v*)c.val, c.nnz / 2,
                                   (const int4v*)c.rp, c.n / 4, (const dbl2v*)c.x1,
                                   (const dbl2v*)c.x2, nullptr, nullptr, c.n / 2, c.part);
    });
    printf("%-34s grid %6d  %8.4f ms  %7.1f GB/s (reads only: %.3f GB)\n", "stream read-only", 2048,
           ms2, rb / ms2 * 1e-6, rb * 1e-9);
  }
  if (on("k2")) run_k2<EPI_DUAL_MRR, 1, 1>(c, g8, "kernel2 dual_mrr DB NT (default)");
  if (on("k2grid")) {
    for (int g : {2048, 4096, 16384}) run_k2<EPI_DUAL_MRR, 1, 1>(c, g, "kernel2 dual_mrr DB NT");
  }
  if (on("k2none")) run_k2<EPI_DUAL_NONE, 1, 1>(c, g8, "kernel2 dual_none DB NT");
  if (on("k2sb")) run_k2<EPI_DUAL_MRR, 0, 1>(c, g8, "kernel2 dual_mrr single-buf NT");
  if (on("k2t")) run_k2<EPI_DUAL_MRR, 1, 0>(c, g8, "kernel2 dual_mrr DB temporal");
  if (on("prod2")) {
    run_prod2<EPI_DUAL_MRR, 2>(c, g8, "prod2 dual_mrr PS2");
    run_prod2<EPI_DUAL_MRR, 4>(c, g8, "prod2 dual_mrr PS4");
    run_prod2<EPI_DUAL_MRR, 2>(c, 2048, "prod2 dual_mrr PS2");
  }
  if (on("direct")) {
    for (int g : {2048, 4096, 8192}) run_direct<EPI_DUAL_MRR, 7, false>(c, g, "direct dual_mrr KC7");
    run_direct<EPI_DUAL_MRR, 7, true>(c, 8192, "direct dual_mrr KC7 NT");
    run_direct<EPI_DUAL_MRR, 7, true>(c, 2048, "direct dual_mrr KC7 NT");
    run_direct<EPI_DUAL_NONE, 7, false>(c, 8192, "direct dual_none KC7");
    run_direct<EPI_DUAL_MRR, 11, false>(c, 8192, "direct dual_mrr KC11");
  }
  if (on("ab")) {
    run_direct<EPI_DUAL_MRR, 7, false, 1>(c, 8192, "direct AB1 no gathers");
    run_direct<EPI_DUAL_MRR, 7, false, 2>(c, 8192, "direct AB2 no stores");
    run_direct<EPI_DUAL_MRR, 7, false, 3>(c, 8192, "direct AB3 own-row gathers");
  }
  if (on("k3")) {
    run_k3<EPI_DUAL_MRR, 0>(c, g8, "kernel3 FL0 (= kernel2)");
    run_k3<EPI_DUAL_MRR, 1>(c, g8, "kernel3 FL1 diag");
    run_k3<EPI_DUAL_MRR, 2>(c, g8, "kernel3 FL2 rp1");
    run_k3<EPI_DUAL_MRR, 4>(c, g8, "kernel3 FL4 buf");
    run_k3<EPI_DUAL_MRR, 7>(c, g8, "kernel3 FL7 all");
    run_k3<EPI_DUAL_MRR, 7>(c, 4096, "kernel3 FL7 all");
    run_k3<EPI_DUAL_MRR, 8>(c, g8, "kernel3 FL8 pairs");
    run_k3<EPI_DUAL_MRR, 24>(c, g8, "kernel3 FL24 pairs NT");
    run_k3<EPI_DUAL_MRR, 15>(c, g8, "kernel3 FL15 all+pairs");
    run_k3<EPI_DUAL_MRR, 31>(c, g8, "kernel3 FL31 all+pairs NT");
  }
  if (on("ntcmp")) {  // the library's NT variant vs kernel3 FL16
    for (int r = 0; r < 2; ++r) {
      run_k2<EPI_DUAL_MRR, 1, 1>(c, g8, "kernel2 NT (compile-time NT stores)");
      run_k3<EPI_DUAL_MRR, 16>(c, g8, "kernel3 FL16 (compile-time NT)");
    }
  }
  if (on("k3ab")) {
    run_k3<EPI_DUAL_MRR, 16>(c, g8, "kernel3 FL16 NT stores");
    run_k3<EPI_DUAL_MRR, 16 + 64>(c, g8, "kernel3 NT, AB no stores");
    run_k3<EPI_DUAL_MRR, 16 + 128>(c, g8, "kernel3 NT, AB no gathers");
    run_k3<EPI_DUAL_MRR, 16 + 64 + 128>(c, g8, "kernel3 NT, AB no st/gathers");
    run_k3<EPI_DUAL_MRR, 16 + 256>(c, g8, "kernel3 NT single-buf");
    run_k3<EPI_DUAL_MRR, 16 + 256 + 64 + 128>(c, g8, "kernel3 NT SB no st/gathers");
    run_k3<EPI_DUAL_MRR, 16 + 7>(c, g8, "kernel3 NT + diag/rp1/buf");
  }
  if (on("k5")) {
    run_k2<EPI_DUAL_MRR, 1, 1>(c, g8, "kernel2 dual_mrr DB NT (default)");
    run_k5<EPI_DUAL_MRR>(c, g8, "kernel5 gathers one block ahead");
    run_k5<EPI_DUAL_MRR>(c, 4096, "kernel5 gathers one block ahead");
    run_k5<EPI_DUAL_MRR, true>(c, g8, "kernel5 VL (values from LDS)");
    run_k5<EPI_DUAL_MRR, true>(c, 4096, "kernel5 VL (values from LDS)");
  }
  if (on("k4")) {
    run_k4<EPI_DUAL_MRR, 0>(c, g8, "kernel4 depth-2 staging");
    run_k4<EPI_DUAL_MRR, 64>(c, g8, "kernel4 AB no stores");
    run_k4<EPI_DUAL_MRR, 64 + 128>(c, g8, "kernel4 AB no st/gathers");
    run_k4<EPI_DUAL_MRR, 0>(c, 4096, "kernel4 depth-2 staging");
    run_k4<EPI_DUAL_MRR, 0>(c, 16384, "kernel4 depth-2 staging");
  }
  if (on("k3s")) {
    run_k3<EPI_DUAL_MRR, 16>(c, g8, "kernel3 FL16 NT stores");
    run_k3<EPI_DUAL_MRR, 32>(c, g8, "kernel3 FL32 sc1 stores");
    run_k3<EPI_DUAL_MRR, 24>(c, g8, "kernel3 FL24 pairs NT");
    run_k3<EPI_DUAL_MRR, 24>(c, 6144, "kernel3 FL24 pairs NT");
    run_k3<EPI_DUAL_MRR, 24>(c, 12288, "kernel3 FL24 pairs NT");
    run_k3<EPI_DUAL_MRR, 24>(c, 16384, "kernel3 FL24 pairs NT");
  }
  if (on("prof")) {  // one launch each for rocprofv3 --pmc
    c.reps = 3;
    run_k2<EPI_DUAL_MRR, 1, 1>(c, g8, "kernel2 dual_mrr DB NT (default)");
    run_direct<EPI_DUAL_MRR, 7, false>(c, 8192, "direct dual_mrr KC7");
    run_k3<EPI_DUAL_MRR, 7>(c, g8, "kernel3 FL7 all");
  }
  return 0;
}
