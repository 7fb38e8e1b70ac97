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
// Round 6: the smallest crashing graph_cost variant (2 shards, ONE split SpMV,
// only the comm-stream cross waits: `graph_cost 2 1 200 64 56`), restated:
// streams st0 (origin), st1 (compute), cs0, cs1 (comm), all forked from st0;
// ev_in(s) recorded on st(s); cs(s) waits ev_in(s) and the neighbour's
// ev_in; gather kernel on cs(s), ev_out(s) recorded there; interior kernel
// on st(s); st(s) waits ev_out(s); boundary kernel; join everything to st0.
// pattern 3: both cross waits (cs0 on ev_in(1), cs1 on ev_in(0));
// pattern 4: only cs1 waits on ev_in(0) (the ORIGIN's event);
// pattern 5: only cs0 waits on ev_in(1) (a forked stream's event).
// pattern 6: as 4 with a kernel on st0 before the ev_in records (the origin's
//            event then carries a captured node);
// pattern 7: as 4 with cs1 waiting on ev_in(0) BEFORE its own ev_in(1).
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
  if (pat >= 3) {
    hipStream_t st[2] = {s0, s1}, cs[2] = {s2, nullptr};
    CK(hipStreamCreateWithFlags(&cs[1], hipStreamNonBlocking));
    hipEvent_t ein[2], eout[2], jn[3];
    for (hipEvent_t* e : {&ein[0], &ein[1], &eout[0], &eout[1], &jn[0], &jn[1], &jn[2]})
      CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    CK(hipStreamBeginCapture(s0, hipStreamCaptureModeRelaxed));
    CK(hipEventRecord(fork, s0));
    CK(hipStreamWaitEvent(st[1], fork, 0));
    CK(hipStreamWaitEvent(cs[0], fork, 0));
    CK(hipStreamWaitEvent(cs[1], fork, 0));
    if (pat == 6) k<<<1, 64, 0, st[0]>>>(d, 9);
    for (int q = 0; q < 2; ++q) CK(hipEventRecord(ein[q], st[q]));
    for (int q = 0; q < 2; ++q) {
      const bool cross = pat == 3 || ((pat == 4 || pat == 6 || pat == 7) && q == 1) ||
                         (pat == 5 && q == 0);
      if (cross && pat == 7) CK(hipStreamWaitEvent(cs[q], ein[1 - q], 0));
      CK(hipStreamWaitEvent(cs[q], ein[q], 0));
      if (cross && pat != 7) CK(hipStreamWaitEvent(cs[q], ein[1 - q], 0));
      k<<<1, 64, 0, cs[q]>>>(d, 10 + q);
      CK(hipEventRecord(eout[q], cs[q]));
      k<<<1, 64, 0, st[q]>>>(d, 20 + q);
    }
    for (int q = 0; q < 2; ++q) {
      CK(hipStreamWaitEvent(st[q], eout[q], 0));
      k<<<1, 64, 0, st[q]>>>(d, 30 + q);
    }
    CK(hipEventRecord(jn[0], st[1]));
    CK(hipEventRecord(jn[1], cs[0]));
    CK(hipEventRecord(jn[2], cs[1]));
    for (int q = 0; q < 3; ++q) CK(hipStreamWaitEvent(s0, jn[q], 0));
    CK(hipStreamEndCapture(s0, &g));
    hipGraphExec_t x;
    CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(x, s0));
    CK(hipStreamSynchronize(s0));
    printf("pattern %d ok\n", pat);
    return 0;
  }
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
