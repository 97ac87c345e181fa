// graph_events.hip — can a launch graph time its kernels under the HIP runtime the process binds to?
// Captures two spin kernels on one stream (no events inside the capture), then adds event-record nodes
// through the graph API (hipGraphAddEventRecordNode: one ahead of the first kernel, one after each), and
// replays it; prints the error codes and the spans.  Built by hand:
//   hipcc --offload-arch=gfx950 -shared -fPIC -o tools/micro/libgraph_events.so tools/micro/graph_events.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_spin2(unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) {
  }
}

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      printf("%s -> %s\n", #x, hipGetErrorString(e_));                        \
      return 1;                                                               \
    }                                                                         \
  } while (0)

extern "C" int probe_graph_events() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int rate = 0;
  CK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0));
  const unsigned long long ticks = (unsigned long long)rate / 10u;  // 100 us
  hipGraph_t g;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(k_spin2, dim3(1), dim3(64), 0, s, ticks);
  hipLaunchKernelGGL(k_spin2, dim3(1), dim3(64), 0, s, 2 * ticks);
  CK(hipStreamEndCapture(s, &g));
  size_t n = 0;
  CK(hipGraphGetNodes(g, nullptr, &n));
  hipGraphNode_t nodes[8];
  CK(hipGraphGetNodes(g, nodes, &n));
  // order the two kernel nodes (root first)
  hipGraphNode_t k0 = nullptr, k1 = nullptr;
  for (size_t i = 0; i < n; ++i) {
    size_t nd = 0;
    CK(hipGraphNodeGetDependencies(nodes[i], nullptr, &nd));
    if (nd == 0) k0 = nodes[i]; else k1 = nodes[i];
  }
  hipEvent_t e[3];
  for (auto& x : e) CK(hipEventCreate(&x));
  hipGraphNode_t r0, r1, r2;
  // e0 ahead of k0: k0 now depends on it
  CK(hipGraphAddEventRecordNode(&r0, g, nullptr, 0, e[0]));
  CK(hipGraphAddDependencies(g, &r0, &k0, 1));
  CK(hipGraphAddEventRecordNode(&r1, g, &k0, 1, e[1]));
  CK(hipGraphAddDependencies(g, &r1, &k1, 1));
  CK(hipGraphAddEventRecordNode(&r2, g, &k1, 1, e[2]));
  hipGraphExec_t x;
  CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
  for (int it = 0; it < 3; ++it) {
    CK(hipGraphLaunch(x, s));
    CK(hipStreamSynchronize(s));
    float a = 0, b = 0;
    CK(hipEventElapsedTime(&a, e[0], e[1]));
    CK(hipEventElapsedTime(&b, e[1], e[2]));
    printf("replay %d: k0 %.3f ms (100 us spin), k1 %.3f ms (200 us spin)\n", it, a, b);
  }
  // re-point the event nodes at fresh events (per-replay pool events)
  hipEvent_t f[3];
  for (auto& y : f) CK(hipEventCreate(&y));
  CK(hipGraphExecEventRecordNodeSetEvent(x, r0, f[0]));
  CK(hipGraphExecEventRecordNodeSetEvent(x, r1, f[1]));
  CK(hipGraphExecEventRecordNodeSetEvent(x, r2, f[2]));
  CK(hipGraphLaunch(x, s));
  CK(hipStreamSynchronize(s));
  float a = 0, b = 0;
  CK(hipEventElapsedTime(&a, f[0], f[1]));
  CK(hipEventElapsedTime(&b, f[1], f[2]));
  printf("re-pointed: k0 %.3f ms, k1 %.3f ms\n", a, b);
  printf("ok\n");
  return 0;
}
