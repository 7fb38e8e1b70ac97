// C2 ceiling microbenchmark: what a kernel moving exactly
// spmv_xy_vp's bytes at C2 (CG on 256^3 Poisson, N = 16,777,216) can reach on
// MI355X. spmv_xy_vp reads p_old and r (2 x 134 MB, plus the ±n re-reads)
// and writes p and v (2 x 134 MB): 537 MB in ~0.13 ms. Here the same bytes
// as a plain stream: every lane reads 16 B of each input and writes 16 B of
// each output (p = r + b p_old, v = 2 p: the loads, stores and their order,
// no stencil), in the variants
//   0 grid-stride, 256-thread workgroups, G workgroups (G = 1024 .. 65536)
//   1 one 512-row block per workgroup (N / 512 workgroups, the stencil
//     kernel's 2 rows per lane), plain stores
//   2 as 1 with non-temporal stores (the stencil kernel's)
//   3 as 1, 16 consecutive blocks per workgroup walked with one block of
//     loads in flight (the stencil walk's Z = 16 segments)
//   4 reads only (2 x 134 MB)       5 writes only (2 x 134 MB)
// Timing: hipEvents around 48 back-to-back launches after 8 warm-up ones,
// the best of 3 repetitions; prints ms per launch and GB/s on 537 MB. The
// launches rotate over 4 disjoint buffer sets (2.1 GB), so no launch finds
// its operands in the 256 MB MALL left by the one before (a single set
// measured up to ~10% above HBM speed in round 5).
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/c2_stream tools/micro/c2_stream.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr long kN = 256L * 256 * 256;

__global__ __launch_bounds__(256) void stride_k(const dbl2* __restrict__ r,
                                                const dbl2* __restrict__ po, dbl2* __restrict__ p,
                                                dbl2* __restrict__ v, double b, long n2) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n2; i += (long)gridDim.x * 256) {
    const dbl2 a = r[i], c = po[i];
    const dbl2 pn = dbl2{a.x + b * c.x, a.y + b * c.y};
    p[i] = pn;
    v[i] = dbl2{2.0 * pn.x, 2.0 * pn.y};
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void block_k(const dbl2* __restrict__ r,
                                               const dbl2* __restrict__ po, dbl2* __restrict__ p,
                                               dbl2* __restrict__ v, double b, int per) {
  const long base = (long)blockIdx.x * per * 256 + threadIdx.x;
  dbl2 a = r[base], c = po[base];
  for (int k = 0; k < per; ++k) {
    const long i = base + (long)k * 256;
    const long in = k + 1 < per ? i + 256 : i;
    const dbl2 na = MODE == 5 ? dbl2{0.0, 0.0} : r[in], nc = MODE == 5 ? dbl2{0.0, 0.0} : po[in];
    const dbl2 pn = dbl2{a.x + b * c.x, a.y + b * c.y};
    if constexpr (MODE == 4) {
      if (pn.x == 12345.0) p[i] = pn;  // keep the loads live
    } else if constexpr (MODE == 2) {
      __builtin_nontemporal_store(pn, p + i);
      __builtin_nontemporal_store(dbl2{2.0 * pn.x, 2.0 * pn.y}, v + i);
    } else {
      p[i] = pn;
      v[i] = dbl2{2.0 * pn.x, 2.0 * pn.y};
    }
    a = na;
    c = nc;
  }
}

constexpr int kSets = 4;

int main() {
  dbl2 *r[kSets], *po[kSets], *p[kSets], *v[kSets];
  const size_t bytes = sizeof(double) * kN;
  for (int q = 0; q < kSets; ++q) {
    CK(hipMalloc(&r[q], bytes));
    CK(hipMalloc(&po[q], bytes));
    CK(hipMalloc(&p[q], bytes));
    CK(hipMalloc(&v[q], bytes));
    CK(hipMemset(r[q], 0, bytes));
    CK(hipMemset(po[q], 0, bytes));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const long n2 = kN / 2;
  auto run = [&](const char* name, double gb, auto launch) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      for (int i = 0; i < 8; ++i) launch(i % kSets);
      CK(hipEventRecord(e0));
      for (int i = 0; i < 48; ++i) launch(i % kSets);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms / 48 < best) best = ms / 48;
    }
    printf("%-44s %8.4f ms  %7.1f GB/s\n", name, best, gb / best * 1e-6);
    fflush(stdout);
  };
  const double all = 4.0 * bytes, half = 2.0 * bytes;
  for (int g : {1024, 2048, 4096, 8192, 16384, 32768, 65536}) {
    char nm[64];
    snprintf(nm, sizeof nm, "0 grid-stride, %d workgroups", g);
    run(nm, all, [&](int q) { stride_k<<<g, 256>>>(r[q], po[q], p[q], v[q], 0.5, n2); });
  }
  const int blocks = (int)(kN / 512);
  run("1 one 512-row block per workgroup", all,
      [&](int q) { block_k<1><<<blocks, 256>>>(r[q], po[q], p[q], v[q], 0.5, 1); });
  run("2 as 1, non-temporal stores", all,
      [&](int q) { block_k<2><<<blocks, 256>>>(r[q], po[q], p[q], v[q], 0.5, 1); });
  run("3 16 blocks per workgroup, one ahead", all,
      [&](int q) { block_k<1><<<blocks / 16, 256>>>(r[q], po[q], p[q], v[q], 0.5, 16); });
  run("3b 16 blocks per workgroup, nt stores", all,
      [&](int q) { block_k<2><<<blocks / 16, 256>>>(r[q], po[q], p[q], v[q], 0.5, 16); });
  run("4 reads only (268 MB), 16 blocks", half,
      [&](int q) { block_k<4><<<blocks / 16, 256>>>(r[q], po[q], p[q], v[q], 0.5, 16); });
  run("5 writes only (268 MB), 16 blocks", half,
      [&](int q) { block_k<5><<<blocks / 16, 256>>>(r[q], po[q], p[q], v[q], 0.5, 16); });
  return 0;
}
