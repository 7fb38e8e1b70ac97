// Host cost of the HIP calls the engine issues per shard and SpMV (event
// record / stream wait / D2D async copy / kernel launch / hipSetDevice),
// from 1 thread and from T threads with their own streams on ONE device --
// the single-process multi-shard enqueue. Build:
//   hipcc -O2 --offload-arch=gfx950 tools/micro/hip_api_cost.hip -o tools/micro/hip_api_cost
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));         \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

__global__ void empty_kernel(double* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p) p[0] += 0.0;
}

struct Ctx {
  hipStream_t s, s2;
  hipEvent_t e;
  double *a, *b;
};

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// us per call of each operation, N calls, on ctx
static void run_ops(Ctx& c, int N, double* out) {
  double t0 = now();
  for (int i = 0; i < N; ++i) CK(hipEventRecord(c.e, c.s));
  out[0] = (now() - t0) / N * 1e6;
  t0 = now();
  for (int i = 0; i < N; ++i) CK(hipStreamWaitEvent(c.s2, c.e, 0));
  out[1] = (now() - t0) / N * 1e6;
  t0 = now();
  for (int i = 0; i < N; ++i) CK(hipMemcpyAsync(c.b, c.a, 1 << 16, hipMemcpyDeviceToDevice, c.s2));
  out[2] = (now() - t0) / N * 1e6;
  t0 = now();
  for (int i = 0; i < N; ++i) empty_kernel<<<256, 256, 0, c.s>>>(nullptr);
  out[3] = (now() - t0) / N * 1e6;
  t0 = now();
  for (int i = 0; i < N; ++i) CK(hipSetDevice(0));
  out[4] = (now() - t0) / N * 1e6;
  CK(hipStreamSynchronize(c.s));
  CK(hipStreamSynchronize(c.s2));
}

int main(int argc, char** argv) {
  const int N = 2000;
  const int T = argc > 1 ? atoi(argv[1]) : 8;
  std::vector<Ctx> ctx(T);
  CK(hipSetDevice(0));
  for (auto& c : ctx) {
    CK(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&c.s2, hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&c.e, hipEventDisableTiming));
    CK(hipMalloc(&c.a, 1 << 16));
    CK(hipMalloc(&c.b, 1 << 16));
  }
  const char* names[5] = {"hipEventRecord", "hipStreamWaitEvent", "hipMemcpyAsync D2D 64KiB",
                          "kernel launch", "hipSetDevice"};
  double one[5];
  run_ops(ctx[0], N, one);  // warm
  run_ops(ctx[0], N, one);
  std::vector<std::array<double, 5>> per(T);
  std::atomic<int> go{0};
  std::vector<std::thread> th;
  double t0 = 0;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      CK(hipSetDevice(0));
      while (!go.load()) {
      }
      run_ops(ctx[t], N, per[t].data());
    });
  t0 = now();
  go = 1;
  for (auto& x : th) x.join();
  const double wall = now() - t0;
  std::printf("us per call        1 thread   %d threads (mean per thread)\n", T);
  for (int k = 0; k < 5; ++k) {
    double m = 0;
    for (int t = 0; t < T; ++t) m += per[t][k];
    std::printf("%-26s %8.2f   %8.2f\n", names[k], one[k], m / T);
  }
  std::printf("%d threads x %d x 5 calls in %.1f ms\n", T, N, wall * 1e3);
  return 0;
}
