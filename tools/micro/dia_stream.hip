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
// MODE (round 4, which part of the walk costs the stream rate; stride 63,
// depth 1, 2 workgroups per CU):
//   0 the stream alone
//   1 + the walk's two __syncthreads per block
//   2 + its LDS work: 31 pre-shifted mirror stores, barrier, 31 mirror reads
//     and 2 x 63 window reads (a dual's two vectors) summed, barrier
//   3 as 2 without the barriers (wrong sums; the LDS work's cost alone)
//   4 as 2 + the dual's other streams: a uint64 mask per row, one new window
//     row of x1 and x2 per lane (loaded one block ahead), y1 and y2 stored
//   5 as 4 without the mask
//   6 as 4 with non-temporal stores of y1, y2
//   7 as 5 without the stores (x1, x2 rows read only)
//   8 as 5 without the x loads (y1, y2 stored only)
//   9 as 5 with each block's y1, y2 stores deferred until the next block's
//     loads are issued (gfx9 counts loads and stores in one vmcnt)
//  10 as 5 with y1, y2 interleaved in one buffer (4 KiB per block)
//  11 as 5 with the stores of two consecutive blocks issued together (odd
//     blocks store the previous block's rows and their own: 4 KiB per vector)
//  12 as 5 with every workgroup storing into its own 2 x 2 KiB (L2-resident:
//     the store path without the HBM writes)
//  14 the stream + x1, x2 rows + y1, y2 stores, no LDS work and no barriers
//     (~100 VGPRs: run at 2, 3 and 4 workgroups per CU)
//  15 as 14 without the stores
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

template <int STRIDE, int DEPTH, int MODE = 0>
__global__ __launch_bounds__(256, 2) void walk(const double* __restrict__ dia, int64_t nb,
                                               double* out, const uint64_t* __restrict__ mask = nullptr,
                                               const double* __restrict__ x1 = nullptr,
                                               const double* __restrict__ x2 = nullptr,
                                               double* y1 = nullptr, double* y2 = nullptr) {
  constexpr bool STREAMS = MODE >= 4;
  constexpr bool PLAIN = MODE == 14 || MODE == 15;
  constexpr bool MASK = MODE == 4 || MODE == 6;
  constexpr bool DEFER = MODE == 9;
  double q1 = 0.0, q2 = 0.0;
  double ps1 = 0.0, ps2 = 0.0;
  int64_t prow = -1;
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
  uint64_t mn = 0;
  double xn1 = 0.0, xn2 = 0.0;
  auto load_ops = [&](int64_t b) {
    if constexpr (STREAMS) {
      const int64_t r = b * kB + tid;
      if constexpr (MASK) mn = mask[r];
      const int64_t xr = min(r + kB, nb * kB - 1);
      if constexpr (MODE != 8) {
        xn1 = x1[xr];
        xn2 = x2[xr];
      }
    }
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) load(d, min(v0 + d, v1 - 1));
  load_ops(v0);
  for (int64_t v = v0; v < v1; ++v) {
    const uint64_t m = mn;
    const double c1 = xn1, c2 = xn2;
    if constexpr (STREAMS) load_ops(min(v + 1, v1 - 1));
    double cur[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) cur[u] = buf[0][u];
#pragma unroll
    for (int d = 0; d + 1 < DEPTH; ++d)
#pragma unroll
      for (int u = 0; u < kU; ++u) buf[d][u] = buf[d + 1][u];
    load(DEPTH - 1, min(v + DEPTH, v1 - 1));
    if constexpr (DEFER) {
      if (prow >= 0) {
        y1[prow] = ps1;
        y2[prow] = ps2;
      }
    }
    double s = 0.0;
    if constexpr (PLAIN) {
#pragma unroll
      for (int u = 0; u < kU; ++u) s = s + cur[u] * (double)(u + 1);
      const int64_t r = v * kB + tid;
      const double s2 = s * c1 + c2;
      if constexpr (MODE == 14) {
        y1[r] = s;
        y2[r] = s2;
      } else {
        s += s2;
      }
    } else if constexpr (MODE == 0 || MODE == 1) {
#pragma unroll
      for (int u = 0; u < kU; ++u) s = s + cur[u] * (double)(u + 1);
      if constexpr (MODE == 1) __syncthreads();
    } else {
      double* s_low = lds;                  // 31 x 256 mirrors
      double* s_win = lds + (kU - 1) * kB;  // 2 x 768 window
#pragma unroll
      for (int u = 1; u < kU; ++u) s_low[(u - 1) * kB + ((tid + 8 * u + 3) & (kB - 1))] = cur[u];
      if constexpr (STREAMS) {
        s_win[2 * kB + tid] = c1;
        s_win[768 + 2 * kB + tid] = c2;
      } else {
        s_win[2 * kB + tid] = cur[0];
        s_win[768 + 2 * kB + tid] = cur[1];
      }
      if constexpr (MODE != 3) __syncthreads();
      double s2 = 0.0;
      const double* wl = s_win + kB + tid;
#pragma unroll
      for (int k = 0; k < kU - 1; ++k) {
        const double m = s_low[k * kB + tid];
        const int o = -(8 * (kU - 1 - k) + 3);
        s = s + m * wl[o];
        s2 = s2 + m * wl[768 + o];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int o = u == 0 ? 0 : 8 * u + 3;
        s = s + cur[u] * wl[o];
        s2 = s2 + cur[u] * wl[768 + o];
      }
      if constexpr (STREAMS) {
        const int64_t r = v * kB + tid;
        if constexpr (MASK) s = m == ~0ull ? s : 0.0;
        if constexpr (MODE == 12) {
          y1[blockIdx.x * kB + tid] = s;
          y2[blockIdx.x * kB + tid] = s2;
        } else if constexpr (MODE == 10) {
          y1[2 * r] = s;
          y1[2 * r + 1] = s2;
        } else if constexpr (MODE == 11) {
          if (((v - v0) & 1) == 1 || v + 1 == v1) {
            if (((v - v0) & 1) == 1) {
              y1[r - kB] = q1;
              y2[r - kB] = q2;
            }
            y1[r] = s;
            y2[r] = s2;
          } else {
            q1 = s;
            q2 = s2;
          }
        } else if constexpr (DEFER) {
          ps1 = s;
          ps2 = s2;
          prow = r;
        } else if constexpr (MODE == 7) {
          if (s == 12345.678) y1[r] = s2;
        } else if constexpr (MODE == 6) {
          __builtin_nontemporal_store(s, y1 + r);
          __builtin_nontemporal_store(s2, y2 + r);
        } else {
          y1[r] = s;
          y2[r] = s2;
        }
      }
      s += s2;
      if constexpr (MODE != 3) __syncthreads();
    }
    acc += s;
  }
  if constexpr (DEFER) {
    if (prow >= 0) {
      y1[prow] = ps1;
      y2[prow] = ps2;
    }
  }
  __syncthreads();
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
  const size_t vb = (size_t)nb * kB * sizeof(double);
  uint64_t* mask = nullptr;
  double *x1 = nullptr, *x2 = nullptr, *y1 = nullptr, *y2 = nullptr;
  if (argc > 2) {
    CK(hipMalloc(&mask, vb));
    CK(hipMalloc(&x1, vb));
    CK(hipMalloc(&x2, vb));
    CK(hipMalloc(&y1, 2 * vb));
    CK(hipMalloc(&y2, vb));
    CK(hipMemset(mask, 0xff, vb));
    CK(hipMemset(x1, 0, vb));
    CK(hipMemset(x2, 0, vb));
  }
  auto run = [&](auto kern, const char* name, int per_cu, size_t lds, double extra = 0.0) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const int G = per_cu * cus;
    for (int w = 0; w < 2; ++w) kern<<<G, 256, lds>>>(dia, nb, out, mask, x1, x2, y1, y2);
    CK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) kern<<<G, 256, lds>>>(dia, nb, out, mask, x1, x2, y1, y2);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-26s wg/cu %d lds %6zu  %.3f ms  %.2f TB/s\n", name, per_cu, lds, ms,
           (moved + extra) / (ms * 1e-3) / 1e12);
  };
  CK(hipMemset(out, 0, 1 << 20));
  if (argc > 2) {  // the MODE series only
    run(walk<63, 1, 0>, "stride63 stream", 2, 77824);
    run(walk<63, 1, 1>, "stride63 +barriers", 2, 77824);
    run(walk<63, 1, 2>, "stride63 +lds+barriers", 2, 77824);
    run(walk<63, 1, 3>, "stride63 +lds", 2, 77824);
    run(walk<63, 1, 4>, "+lds+barriers+streams", 2, 77824, 5.0 * vb);
    run(walk<63, 1, 5>, "  same, no mask", 2, 77824, 4.0 * vb);
    run(walk<63, 1, 6>, "  same, nt stores", 2, 77824, 5.0 * vb);
    run(walk<63, 1, 7>, "  no mask, no stores", 2, 77824, 2.0 * vb);
    run(walk<63, 1, 8>, "  no mask, no x loads", 2, 77824, 2.0 * vb);
    run(walk<63, 1, 9>, "  no mask, deferred stores", 2, 77824, 4.0 * vb);
    run(walk<63, 1, 10>, "  no mask, y1 y2 interleaved", 2, 77824, 4.0 * vb);
    run(walk<63, 1, 11>, "  no mask, paired-block stores", 2, 77824, 4.0 * vb);
    run(walk<63, 1, 5>, "  no mask (again)", 2, 77824, 4.0 * vb);
    run(walk<63, 1, 12>, "  no mask, L2-resident stores", 2, 77824, 2.0 * vb);
    run(walk<63, 1, 7>, "  no mask, no stores (again)", 2, 77824, 2.0 * vb);
    for (int per_cu : {2, 3, 4}) {
      const size_t lds = per_cu == 2 ? 77824 : per_cu == 3 ? 52000 : 38000;
      run(walk<63, 1, 14>, "plain stream+x+stores", per_cu, lds, 4.0 * vb);
      run(walk<63, 1, 15>, "plain stream+x", per_cu, lds, 2.0 * vb);
    }
    run(walk<63, 1, 0>, "stride63 stream", 2, 77824);
    return 0;
  }
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
