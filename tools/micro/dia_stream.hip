// Read-stream microbenchmark of the symmetric DIA walk's HBM pattern (C5:
// h = 31, 63 offsets, 50M rows). Each workgroup walks a contiguous run of
// 256-row blocks; per block every lane loads its row's diagonal + upper
// values (32 doubles, one 512-B wave access each), one block ahead, and sums
// them (stand-in compute). Variants:
//   stride 63: the row-block-major layout of the engine (upper half of each
//              63-slot chunk, the lower 31 slots skipped)
//   stride 32: a compact upper-only layout (one contiguous 64-KiB chunk per block)
// grid: workgroups (2, 3, 4 per CU); lds: dynamic LDS per workgroup (limits
// residency like the walk kernel's 76 KiB); depth: blocks loaded ahead (1, 2).
//   hipcc -O3 --offload-arch=gfx950 -o tools/micro/dia_stream tools/micro/dia_stream.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      printf("%s -> %s\n", #x, hipGetErrorString(e));                       \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

constexpr int kB = 256;
constexpr int kU = 32;  // diagonal + 31 upper

template <int STRIDE, int DEPTH>
__global__ __launch_bounds__(256, 2) void walk(const double* __restrict__ dia, int64_t nb,
                                               double* out) {
  extern __shared__ double lds[];
  const int tid = threadIdx.x;
  const int64_t G = gridDim.x, g = blockIdx.x;
  const int64_t v0 = g * nb / G, v1 = (g + 1) * nb / G;
  const int64_t base = STRIDE == 63 ? 31 : 0;
  double buf[DEPTH][kU];
  auto load = [&](int d, int64_t b) {
    const double* p = dia + (b * STRIDE + base) * kB + tid;
#pragma unroll
    for (int u = 0; u < kU; ++u) buf[d][u] = __builtin_nontemporal_load(p + (int64_t)u * kB);
  };
  double acc = 0.0;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) load(d, min(v0 + d, v1 - 1));
  for (int64_t v = v0; v < v1; ++v) {
    double cur[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) cur[u] = buf[0][u];
#pragma unroll
    for (int d = 0; d + 1 < DEPTH; ++d)
#pragma unroll
      for (int u = 0; u < kU; ++u) buf[d][u] = buf[d + 1][u];
    load(DEPTH - 1, min(v + DEPTH, v1 - 1));
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < kU; ++u) s = s + cur[u] * (double)(u + 1);
    acc += s;
  }
  if (tid == 0) lds[0] = acc;
  __syncthreads();
  if (acc == 12345.678) out[g] = lds[0];
}

int main(int argc, char** argv) {
  const int64_t rows = argc > 1 ? atoll(argv[1]) : 50000000;
  const int64_t nb = (rows + kB - 1) / kB;
  const size_t bytes = (size_t)nb * 63 * kB * sizeof(double);
  double* dia = nullptr;
  double* out = nullptr;
  CK(hipMalloc(&dia, bytes));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(dia, 0, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double moved = (double)nb * kU * kB * sizeof(double);
  auto run = [&](auto kern, const char* name, int per_cu, size_t lds) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int G = per_cu * cus;
    for (int w = 0; w < 2; ++w) kern<<<G, 256, lds>>>(dia, nb, out);
    CK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) kern<<<G, 256, lds>>>(dia, nb, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-22s wg/cu %d lds %6zu  %.3f ms  %.2f TB/s\n", name, per_cu, lds, ms,
           moved / (ms * 1e-3) / 1e12);
  };
  for (int per_cu : {2, 3, 4}) {
    const size_t lds = per_cu == 2 ? 77824 : per_cu == 3 ? 52000 : 38000;
    run(walk<63, 1>, "stride63 depth1", per_cu, lds);
    run(walk<32, 1>, "stride32 depth1", per_cu, lds);
    run(walk<63, 2>, "stride63 depth2", per_cu, lds);
    run(walk<32, 2>, "stride32 depth2", per_cu, lds);
  }
  CK(hipFree(dia));
  CK(hipFree(out));
  return 0;
}
