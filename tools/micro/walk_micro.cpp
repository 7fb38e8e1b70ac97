// Timing micro of the symmetric DIA walk (spmv_diawalk_kernel, kr_spmv.h) at
// C5's shape: n rows (default 50M), h = 31 upper offsets (63 per row, band
// <= 256), row-block-major diagonal values, every block full (masks not
// loaded), the dual SpMV EPI_DUAL_MRR storing and products-only. Values and
// vectors are hashes: this times the kernel; it checks no result (the
// library's DIA bitwise tests do). Ablation builds compile the walk with
// -DKR_DIAW_AB=<bits> (see kr_spmv.h) and print the same lines:
//
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -x hip \
//     -I/opt/rocm/include [-DKR_DIAW_AB=n] -o tools/micro/walk_micro tools/micro/walk_micro.cpp
//   tools/micro/walk_micro [n_rows=50000000] [reps=10]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../parallel-krylov_amd/csrc/kr_spmv.h"

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      printf("%s -> %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

using namespace kr;

__global__ void fill_hash(double* v, int64_t n, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t h = (uint64_t)i * 0x9E3779B97F4A7C15ull ^ seed;
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    v[i] = (double)(h >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  }
}

__global__ void fill_u64(uint64_t* v, int64_t n, uint64_t x) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    v[i] = x;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 50000000;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  constexpr int NH = 31, NM = 2 * NH + 1;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  // offsets: -o_31 .. -o_1, 0, o_1 .. o_31 with o_u = 8u + u % 3 (<= 249)
  std::vector<int32_t> M(NM);
  for (int u = 1; u <= NH; ++u) {
    M[NH + u] = 8 * u + u % 3;
    M[NH - u] = -(8 * u + u % 3);
  }
  M[NH] = 0;
  const int64_t nvb = (n + kBlock - 1) / kBlock;
  const int64_t nvals = nvb * (int64_t)kBlock * NM;
  double *dia, *x1, *x2, *y1, *y2, *part;
  uint64_t* mask;
  int32_t* moff;
  CK(hipMalloc(&dia, nvals * 8));
  CK(hipMalloc(&x1, n * 8));
  CK(hipMalloc(&x2, n * 8));
  CK(hipMalloc(&y1, n * 8));
  CK(hipMalloc(&y2, n * 8));
  CK(hipMalloc(&mask, n * 8));
  CK(hipMalloc(&moff, NM * 4));
  const int grid = 2 * cus;  // dia_walk_grid at h = 31: 2 resident per CU
  CK(hipMalloc(&part, (size_t)grid * 8 * 8));
  CK(hipMemcpy(moff, M.data(), NM * 4, hipMemcpyHostToDevice));
  fill_hash<<<8192, 256>>>(dia, nvals, 1);
  fill_hash<<<4096, 256>>>(x1, n, 2);
  fill_hash<<<4096, 256>>>(x2, n, 3);
  fill_u64<<<4096, 256>>>(mask, n, ~0ull >> 1);
  CK(hipDeviceSynchronize());

  SpmvArgs a;
  a.n = n;
  a.x1 = x1;
  a.x2 = x2;
  a.y1 = y1;
  a.y2 = y2;
  a.xoff = 0;
  a.xlen = n;
  a.partials = part;
  a.grid = grid;
  a.mask = mask;
  a.moff = moff;
  a.nm = NM;
  a.mw = 64;
  a.dia = dia;
  a.dia_bs = (int64_t)kBlock * NM;
  a.dia_ks = kBlock;
  a.dia_sym = 1;
  a.dia_walk = 1;
  a.full_lo = 0;
  a.full_hi = nvb;
  a.nnz_total = n * NM;

  // bytes a dual must stream: the diagonal + upper values, both x, both y
  const double vbytes = 8.0 * (NH + 1) * n;
  const double bytes_st = vbytes + 32.0 * n, bytes_po = vbytes + 16.0 * n;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int po = 0; po < 2; ++po) {
    a.products_only = po;
    for (int r = 0; r < 2; ++r) {
      spmv_diawalk_launch_t<EPI_DUAL_MRR, NH>(a, grid, 0);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) spmv_diawalk_launch_t<EPI_DUAL_MRR, NH>(a, grid, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      const double b = po ? bytes_po : bytes_st;
      printf("AB %3d %-14s %8.4f ms  %6.3f TB/s on %.2f GB  frac %.4f\n", KR_DIAW_AB,
             po ? "products-only" : "storing", ms, b / ms * 1e-9, b * 1e-9, b / ms * 1e-9 / 8.0);
      fflush(stdout);
    }
  }
  return 0;
}
