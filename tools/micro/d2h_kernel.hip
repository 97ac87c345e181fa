// Device-to-host rate of a 1080p RGB8 frame (6.2 MB) into a caller's page-locked buffer: the SDMA copy
// (hipMemcpyAsync) against a copy kernel that stores 16-B words straight into the buffer's mapped device
// address, for a hipHostRegister'd std::vector and a hipHostMalloc allocation.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/d2h_kernel tools/micro/d2h_kernel.hip && /tmp/d2h_kernel [blocks]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

__global__ void k_copy16(const uint4* __restrict__ src, uint4* dst, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? std::atoi(argv[1]) : 512;
  const size_t bytes = 1920ull * 1080 * 3;  // 6 220 800 = 388 800 x 16
  const int iters = 50;
  uint8_t* d = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(d, 7, bytes));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<uint8_t> vec(bytes + 4096);
  uint8_t* vp = vec.data();
  CK(hipHostRegister(vp, bytes, hipHostRegisterMapped));
  uint8_t* hm = nullptr;
  CK(hipHostMalloc(&hm, bytes, hipHostMallocDefault));
  struct Target {
    const char* name;
    uint8_t* h;
  } targets[2] = {{"registered vector", vp}, {"hipHostMalloc", hm}};
  for (const Target& t : targets) {
    void* dp = nullptr;
    CK(hipHostGetDevicePointer(&dp, t.h, 0));
    for (int mode = 0; mode < 2; ++mode) {
      auto run = [&]() {
        if (mode == 0) CK(hipMemcpyAsync(t.h, d, bytes, hipMemcpyDeviceToHost, s));
        else hipLaunchKernelGGL(k_copy16, dim3(blocks), dim3(256), 0, s, (const uint4*)d, (uint4*)dp, bytes / 16);
      };
      for (int i = 0; i < 5; ++i) run();
      CK(hipStreamSynchronize(s));
      std::memset(t.h, 0, bytes);
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < iters; ++i) run();
      CK(hipEventRecord(e1, s));
      CK(hipStreamSynchronize(s));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      size_t bad = 0;
      for (size_t i = 0; i < bytes; ++i) bad += t.h[i] != 7;
      std::printf("%-18s %-6s %7.1f us/frame %6.1f GB/s  wrong bytes %zu\n", t.name, mode ? "kernel" : "sdma",
                  1e3 * ms / iters, bytes * iters / (ms * 1e6), bad);
    }
  }
  CK(hipHostUnregister(vp));
  CK(hipHostFree(hm));
  CK(hipFree(d));
  return 0;
}
