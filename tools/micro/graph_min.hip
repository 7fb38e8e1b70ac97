// Minimal hipGraph capture patterns (round 5): which
// cross-stream dependency among forked capture streams makes
// hipStreamEndCapture crash (tools/micro/graph_cost.hip: 2+ shards whose comm
// stream waits on a NEIGHBOUR's event crash there; each stream waiting only
// on its own shard's events captures and replays correctly).
//   hipcc -O2 --offload-arch=gfx950 -o tools/micro/graph_min tools/micro/graph_min.hip
//   tools/micro/graph_min <pattern>
// pattern 0: origin s0 forks s1, s2; s1 kernel, record e1; s2 waits e1 (a
//            forked stream waits on ANOTHER forked stream); join s1, s2.
// pattern 1: as 0, but s2 waits on an event recorded on the ORIGIN s0.
// pattern 2: as 0 with s1 waiting on s2's event too (a two-way edge).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
  do {                                                                           \
    printf("> %d %s\n", __LINE__, #x);                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("%s -> %s\n", #x, hipGetErrorString(e_));                           \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ void k(int* p, int v) {
  if (threadIdx.x == 0 && p) p[v & 7] = v;
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int pat = argc > 1 ? atoi(argv[1]) : 0;
  hipStream_t s0, s1, s2;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t fork, e0, e1, e2, j1, j2;
  for (hipEvent_t* e : {&fork, &e0, &e1, &e2, &j1, &j2})
    CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  int* d = nullptr;
  CK(hipMalloc(&d, 64));
  hipGraph_t g;
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeRelaxed));
  CK(hipEventRecord(fork, s0));
  CK(hipStreamWaitEvent(s1, fork, 0));
  CK(hipStreamWaitEvent(s2, fork, 0));
  k<<<1, 64, 0, s0>>>(d, 0);
  CK(hipEventRecord(e0, s0));
  k<<<1, 64, 0, s1>>>(d, 1);
  CK(hipEventRecord(e1, s1));
  k<<<1, 64, 0, s2>>>(d, 2);
  CK(hipEventRecord(e2, s2));
  if (pat == 1) {
    CK(hipStreamWaitEvent(s2, e0, 0));
  } else {
    CK(hipStreamWaitEvent(s2, e1, 0));
    if (pat == 2) CK(hipStreamWaitEvent(s1, e2, 0));
  }
  k<<<1, 64, 0, s1>>>(d, 3);
  k<<<1, 64, 0, s2>>>(d, 4);
  CK(hipEventRecord(j1, s1));
  CK(hipEventRecord(j2, s2));
  CK(hipStreamWaitEvent(s0, j1, 0));
  CK(hipStreamWaitEvent(s0, j2, 0));
  CK(hipStreamEndCapture(s0, &g));
  hipGraphExec_t x;
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(x, s0));
  CK(hipStreamSynchronize(s0));
  printf("pattern %d ok\n", pat);
  return 0;
}
