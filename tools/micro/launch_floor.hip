// Launch-cost microbenchmark (MI355X): how long does a dependent chain of resident-grid launches
// take per launch, with and without hipGraph, for an empty body, an LDS allocation, and a
// 2048-count prologue like the stage kernels' seg_scan?  Prints us per launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 100000) p[0] = 1;
}
__global__ void k_lds(int* p) {
  extern __shared__ int s[];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (p && s[255 - threadIdx.x] < 0) p[0] = 1;
}
__global__ void k_scan(const unsigned* cnt, int* p) {
  __shared__ unsigned s[2048 + 1];
  unsigned v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = cnt[threadIdx.x * 8 + j];
  unsigned sum = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) sum += v[j];
  s[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x == 0 && s[17] == 12345u && p) p[0] = 1;
}

__global__ void k_scratch(const unsigned* cnt, int* p) {
  unsigned arr[84];
  const unsigned n = cnt[blockIdx.x & 1023];  // 0: the loop below never runs
  for (unsigned i = 0; i < n; ++i) arr[(threadIdx.x + i) % 84] = i;
  if (n && p) p[0] = arr[threadIdx.x % 84];
}
__global__ void k_scratch_touch(const unsigned* cnt, int* p) {
  volatile unsigned arr[84];
  arr[threadIdx.x % 84] = threadIdx.x;
  if (p && arr[(threadIdx.x + 1) % 84] == 77777u) p[0] = 1;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned* cnt;
  CK(hipMalloc(&cnt, 4096 * 4));
  CK(hipMemset(cnt, 0, 4096 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int N = 200;
  for (int grid : {256, 1024, 2048, 4096}) {
    for (int kind = 0; kind < 5; ++kind) {
      auto launch = [&]() {
        if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s, nullptr);
        else if (kind == 1) hipLaunchKernelGGL(k_lds, dim3(grid), dim3(256), 12800, s, nullptr);
        else if (kind == 2) hipLaunchKernelGGL(k_scan, dim3(grid), dim3(256), 0, s, cnt, nullptr);
        else if (kind == 3) hipLaunchKernelGGL(k_scratch, dim3(grid), dim3(256), 0, s, cnt, nullptr);
        else hipLaunchKernelGGL(k_scratch_touch, dim3(grid), dim3(256), 0, s, cnt, nullptr);
      };
      for (int i = 0; i < 20; ++i) launch();
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(a, s));
      for (int i = 0; i < N; ++i) launch();
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      // graph of 20 launches
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int i = 0; i < 20; ++i) launch();
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(a, s));
      for (int i = 0; i < N / 20; ++i) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float msg = 0;
      CK(hipEventElapsedTime(&msg, a, b));
      printf("grid %5d kind %s: stream %.2f us/launch, graph %.2f us/launch\n", grid,
             kind == 0 ? "empty" : kind == 1 ? "lds  " : kind == 2 ? "scan " : kind == 3 ? "scr0 " : "scr1 ", ms * 1e3 / N, msg * 1e3 / N);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
