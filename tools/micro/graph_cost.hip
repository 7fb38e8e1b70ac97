// Host cost of one k-skip MrR outer iteration of the in-process multi-shard
// path (8 shards on one device, the bench's --local-shards 8 layout), issued
// directly vs replayed as a captured hipGraph. The op pattern per split SpMV
// and shard is the engine's (System::spmv / halo_in_process):
//   record ev_in(s) | comm(s): wait ev_in(s), ev_in(s-1), ev_in(s+1); gather
//   kernel; record ev_out(s) | interior kernel | wait ev_out(s), ev_out(s+-1);
//   boundary kernel
// 9 SpMVs per outer iteration, then per shard a finalize kernel and an 8-slot
// D2H copy into pinned memory. Kernels are empty (a 704-byte argument like
// SpmvArgs), so the GPU side is launch-bound and the host side is the thing
// measured. Graph replay also patches the arguments of 4 step SpMVs x 2
// launches x 8 shards (hipGraphExecKernelNodeSetParams), as the engine would.
//   hipcc -O2 --offload-arch=gfx950 -o tools/micro/graph_cost tools/micro/graph_cost.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

// GRAPH_TRACE=1: every call of the capture section is printed before it runs
// (stdout unbuffered), so a crash names the call it died in.
static bool g_trace = false;
#define CK(x)                                                               \
  do {                                                                      \
    if (g_trace) printf("> %d %s\n", __LINE__, #x);                         \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

struct Args {
  double c[4];
  double* out;
  char pad[704 - 40];
};

__global__ void work(Args a) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && a.c[0] == 12345.0) a.out[0] = a.c[1];
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int S = argc > 1 ? atoi(argv[1]) : 8;       // shards
  const int NSPMV = argc > 2 ? atoi(argv[2]) : 9;   // split SpMVs per outer iteration
  const int iters = argc > 3 ? atoi(argv[3]) : 200;
  const int G = argc > 4 ? atoi(argv[4]) : 64;      // workgroups per launch
  // capture-crash bisection (round 5): 0 the engine's pattern; 1 no waits on
  // the neighbours' events (each comm / compute stream waits its own shard's
  // only); 2 a fresh event for every record (no event recorded twice in one
  // capture); 3 both. Round 6, one edge class at a time: 4 no cross waits on
  // the comm streams only (lines 94-95), 8 on the compute streams only
  // (117-118), 16 no D2H copy per stream (138), 32 no capture-info harvest
  // of the step launches' nodes (107, 127)
  const int MODE = argc > 5 ? atoi(argv[5]) : 0;
  std::vector<hipStream_t> st(S), cs(S);
  std::vector<hipEvent_t> ev_in(S), ev_out(S), ev_join(2 * S);
  std::vector<hipEvent_t> ev_in_m(S * NSPMV), ev_out_m(S * NSPMV);  // MODE & 2
  for (auto& ev : ev_in_m) CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (auto& ev : ev_out_m) CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (int s = 0; s < S; ++s) {
    CK(hipStreamCreateWithFlags(&st[s], hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&cs[s], hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&ev_in[s], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ev_out[s], hipEventDisableTiming));
  }
  for (auto& ej : ev_join) CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
  hipEvent_t ev_fork;
  CK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
  double* dbuf = nullptr;
  CK(hipMalloc(&dbuf, 1 << 20));
  double* host = nullptr;
  CK(hipHostMalloc(&host, sizeof(double) * 64 * S));
  Args a{};
  a.out = dbuf;

  // one outer iteration; `coef` collects the launches whose scalars change
  auto iteration = [&](bool capture, std::vector<hipGraphNode_t>* coef) {
    for (int m = 0; m < NSPMV; ++m) {
      const bool step = m < 4;  // the step SpMVs carry (eta, zeta)
      a.c[0] = m;
      const bool fresh = capture && (MODE & 2);
      const bool cross = !(MODE & 1);
      const bool cross_comm = cross && !(MODE & 4), cross_comp = cross && !(MODE & 8);
      auto EI = [&](int s) { return fresh ? ev_in_m[m * S + s] : ev_in[s]; };
      auto EO = [&](int s) { return fresh ? ev_out_m[m * S + s] : ev_out[s]; };
      for (int s = 0; s < S; ++s) CK(hipEventRecord(EI(s), st[s]));
      for (int s = 0; s < S; ++s) {
        CK(hipStreamWaitEvent(cs[s], EI(s), 0));
        if (cross_comm && s > 0) CK(hipStreamWaitEvent(cs[s], EI(s - 1), 0));
        if (cross_comm && s + 1 < S) CK(hipStreamWaitEvent(cs[s], EI(s + 1), 0));
        if (g_trace) printf("> launch gather s=%d m=%d\n", s, m);
        work<<<G, 256, 0, cs[s]>>>(a);
        CK(hipEventRecord(EO(s), cs[s]));
        if (g_trace) printf("> launch interior s=%d m=%d\n", s, m);
        work<<<G, 256, 0, st[s]>>>(a);
        if (capture && step && coef && !(MODE & 32)) {
          hipStreamCaptureStatus cst;
          unsigned long long cid = 0;
          hipGraph_t cg = nullptr;
          const hipGraphNode_t* deps = nullptr;
          size_t nd = 0;
          CK(hipStreamGetCaptureInfo_v2(st[s], &cst, &cid, &cg, &deps, &nd));
          if (nd < 1 || !deps) {
            printf("capture info: %zu deps\n", nd);
            exit(1);
          }
          coef->push_back(deps[0]);
        }
      }
      for (int s = 0; s < S; ++s) {
        CK(hipStreamWaitEvent(st[s], EO(s), 0));
        if (cross_comp && s > 0) CK(hipStreamWaitEvent(st[s], EO(s - 1), 0));
        if (cross_comp && s + 1 < S) CK(hipStreamWaitEvent(st[s], EO(s + 1), 0));
        if (g_trace) printf("> launch boundary s=%d m=%d\n", s, m);
        work<<<G / 8 + 1, 256, 0, st[s]>>>(a);
        if (capture && step && coef && !(MODE & 32)) {
          hipStreamCaptureStatus cst;
          unsigned long long cid = 0;
          hipGraph_t cg = nullptr;
          const hipGraphNode_t* deps = nullptr;
          size_t nd = 0;
          CK(hipStreamGetCaptureInfo_v2(st[s], &cst, &cid, &cg, &deps, &nd));
          if (nd < 1 || !deps) {
            printf("capture info: %zu deps\n", nd);
            exit(1);
          }
          coef->push_back(deps[0]);
        }
      }
    }
    for (int s = 0; s < S; ++s) {
      work<<<1, 256, 0, st[s]>>>(a);
      if (!(MODE & 16))
        CK(hipMemcpyAsync(host + 64 * s, dbuf + 64 * s, 64, hipMemcpyDeviceToHost, st[s]));
    }
  };

  // ---- direct
  for (int w = 0; w < 5; ++w) {
    iteration(false, nullptr);
    for (int s = 0; s < S; ++s) CK(hipStreamSynchronize(st[s]));
  }
  double enq = 0, tot = 0;
  for (int it = 0; it < iters; ++it) {
    const double t0 = now();
    iteration(false, nullptr);
    const double t1 = now();
    for (int s = 0; s < S; ++s) CK(hipStreamSynchronize(st[s]));
    const double t2 = now();
    enq += t1 - t0;
    tot += t2 - t0;
  }
  printf("direct : enqueue %.3f ms  total %.3f ms per outer iteration (%d shards, %d SpMVs)\n",
         1e3 * enq / iters, 1e3 * tot / iters, S, NSPMV);

  // ---- capture
  printf("capturing\n");
  g_trace = getenv("GRAPH_TRACE") && atoi(getenv("GRAPH_TRACE")) != 0;
  hipGraph_t graph;
  std::vector<hipGraphNode_t> coef;
  double tc0 = now();
  CK(hipStreamBeginCapture(st[0], hipStreamCaptureModeRelaxed));
  CK(hipEventRecord(ev_fork, st[0]));
  for (int s = 0; s < S; ++s) {
    if (s > 0) CK(hipStreamWaitEvent(st[s], ev_fork, 0));
    CK(hipStreamWaitEvent(cs[s], ev_fork, 0));
  }
  iteration(true, &coef);
  for (int s = 0; s < S; ++s) {
    if (s > 0) {
      CK(hipEventRecord(ev_join[s], st[s]));
      CK(hipStreamWaitEvent(st[0], ev_join[s], 0));
    }
    CK(hipEventRecord(ev_join[S + s], cs[s]));
    CK(hipStreamWaitEvent(st[0], ev_join[S + s], 0));
  }
  CK(hipStreamEndCapture(st[0], &graph));
  size_t nn = 0;
  CK(hipGraphGetNodes(graph, nullptr, &nn));
  hipGraphExec_t exec;
  CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  printf("instantiated\n");
  g_trace = false;
  const double tc1 = now();
  printf("capture+instantiate %.3f ms, %zu nodes, %zu patched launches\n", 1e3 * (tc1 - tc0), nn,
         coef.size());
  std::vector<hipKernelNodeParams> kp(coef.size());
  std::vector<Args> kargs(coef.size());
  std::vector<void*> kptr(coef.size());
  for (size_t i = 0; i < coef.size(); ++i) {
    CK(hipGraphKernelNodeGetParams(coef[i], &kp[i]));
    if (!kp[i].kernelParams || !kp[i].kernelParams[0]) {
      printf("node %zu: kernelParams %p extra %p\n", i, (void*)kp[i].kernelParams, (void*)kp[i].extra);
      exit(1);
    }
    memcpy(&kargs[i], kp[i].kernelParams[0], sizeof(Args));
    kptr[i] = &kargs[i];
    kp[i].kernelParams = &kptr[i];
  }
  for (int w = 0; w < 5; ++w) {
    CK(hipGraphLaunch(exec, st[0]));
    CK(hipStreamSynchronize(st[0]));
  }
  double patch = 0, launch = 0, total = 0;
  for (int it = 0; it < iters; ++it) {
    const double t0 = now();
    for (size_t i = 0; i < coef.size(); ++i) {
      kargs[i].c[1] = it;
      CK(hipGraphExecKernelNodeSetParams(exec, coef[i], &kp[i]));
    }
    const double t1 = now();
    CK(hipGraphLaunch(exec, st[0]));
    const double t2 = now();
    CK(hipStreamSynchronize(st[0]));
    const double t3 = now();
    patch += t1 - t0;
    launch += t2 - t1;
    total += t3 - t0;
  }
  printf("graph  : patch %.3f ms  launch %.3f ms  total %.3f ms per outer iteration\n",
         1e3 * patch / iters, 1e3 * launch / iters, 1e3 * total / iters);
  // correctness of the patch: a patched scalar reaches the kernel
  kargs[0].c[0] = 12345.0;
  kargs[0].c[1] = 777.0;
  CK(hipGraphExecKernelNodeSetParams(exec, coef[0], &kp[0]));
  CK(hipGraphLaunch(exec, st[0]));
  CK(hipStreamSynchronize(st[0]));
  double got = 0;
  CK(hipMemcpy(&got, dbuf, sizeof(double), hipMemcpyDeviceToHost));
  printf("patched scalar seen by the kernel: %s (%g)\n", got == 777.0 ? "yes" : "NO", got);
  CK(hipGraphExecDestroy(exec));
  CK(hipGraphDestroy(graph));
  printf("ok\n");
  return 0;
}
