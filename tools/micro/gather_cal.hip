// FETCH_SIZE calibration for the access shapes of the BVH traversal.
//
// MI355X_MICROARCH.md §HBM calibrates rocprofv3's FETCH_SIZE only for 16-B-per-lane coalesced
// streams (it reports half their bytes).  The trace and shadow kernels read 64-B wide-BVH nodes
// (four 16-B loads of one lane at a 64-B-aligned address) and 48-B triangles (three 16-B loads) at
// random addresses.  Each mode below reads a KNOWN set of distinct bytes from a 4 GiB buffer (16x the
// 256 MiB Infinity Cache, every address touched once per launch), so FETCH_SIZE per launch against the
// known bytes gives the counter's factor for that shape, and the launch time gives the useful-byte
// rate beside the plain stream's.
//   stream  16 B per lane, coalesced (the guide's calibrated shape: expect FETCH x2 = bytes)
//   line    128 B per lane (8 x 16 B) at a random 128-B line (a bijection over the lines)
//   half    64 B per lane at the first half of a random 128-B line (no other half ever read)
//   node    64 B per lane (4 x 16 B) at a random 64-B block (both halves of a line may be read,
//           by different lanes at different times: the traversal's node shape)
//   tri     48 B per lane (3 x 16 B) at a random 48-B record (the triangle shape)
//   r16     16 B per lane at a random 16-B slot
// usage: gather_cal <mode> [launches]     prints one JSON line per mode with the event time
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr unsigned long long kBufBytes = 4ull << 30;

// a bijection of [0, 2^bits): odd multiplies and xor-shifts, each invertible mod 2^bits
__device__ __forceinline__ unsigned perm(unsigned i, unsigned bits) {
  const unsigned m = bits == 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
  unsigned x = i & m;
  x = (x * 0x9E3779B1u) & m;
  x ^= x >> (bits / 2);
  x = (x * 0x85EBCA6Bu) & m;
  x ^= x >> (bits / 3 + 1);
  x = (x * 0xC2B2AE35u) & m;
  x ^= x >> (bits / 2 + 1);
  return x;
}

template <int kLoads>
__device__ __forceinline__ float sum_loads(const float4* p) {
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < kLoads; ++j) {
    const float4 v = p[j];
    s += v.x + v.y + v.z + v.w;
  }
  return s;
}

// mode 0 stream, 1 line, 2 half, 3 node, 4 tri, 5 r16; n accesses
__global__ void k_read(const float4* buf, unsigned n, int mode, unsigned bits, float* sink) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.0f;
  switch (mode) {
    case 0: s = sum_loads<1>(buf + i); break;
    case 1: s = sum_loads<8>(buf + 8ull * perm(i, bits)); break;
    case 2: s = sum_loads<4>(buf + 8ull * perm(i, bits)); break;
    case 3: s = sum_loads<4>(buf + 4ull * perm(i, bits)); break;
    case 4: {
      // 48-B records: a bijection over 2^bits record slots of a 3 * 2^bits float4 region
      s = sum_loads<3>(buf + 3ull * perm(i, bits));
      break;
    }
    default: s = sum_loads<1>(buf + perm(i, bits)); break;
  }
  if (s == 1234.5678f) sink[i & 1023] = s;  // never true: keeps the loads, writes nothing
}

int main(int argc, char** argv) {
  const char* names[] = {"stream", "line", "half", "node", "tri", "r16"};
  const int bytes_per[] = {16, 128, 64, 64, 48, 16};
  int launches = argc > 2 ? atoi(argv[2]) : 5;
  float4* buf = nullptr;
  float* sink = nullptr;
  CK(hipMalloc(&buf, kBufBytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(buf, 0, kBufBytes));
  for (int mode = 0; mode < 6; ++mode) {
    if (argc > 1 && strcmp(argv[1], "all") != 0 && strcmp(argv[1], names[mode]) != 0) continue;
    // accesses per launch: 1 GiB of distinct bytes (the stream mode: the first GiB, coalesced);
    // bits: the permutation domain, sized so every access lands on a distinct unit of the 4 GiB buffer
    unsigned n = 0, bits = 0;
    switch (mode) {
      case 0: n = (1u << 30) / 16; bits = 0; break;
      case 1: bits = 25; n = 1u << 23; break;   // 2^25 lines of 128 B = 4 GiB; 2^23 x 128 B = 1 GiB
      case 2: bits = 25; n = 1u << 24; break;   // first halves of 2^24 distinct lines
      case 3: bits = 26; n = 1u << 24; break;   // 2^26 blocks of 64 B = 4 GiB; 2^24 distinct blocks
      case 4: bits = 26; n = 1u << 24; break;   // 2^26 records of 48 B = 3 GiB; 2^24 distinct records
      default: bits = 28; n = 1u << 26; break;  // 2^28 slots of 16 B = 4 GiB
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_read, dim3((n + 255) / 256), dim3(256), 0, 0, buf, n, mode, bits, sink);  // warm-up
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int l = 0; l < launches; ++l)
      hipLaunchKernelGGL(k_read, dim3((n + 255) / 256), dim3(256), 0, 0, buf, n, mode, bits, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.0f;
    CK(hipEventElapsedTime(&ms, a, b));
    const double known = (double)n * bytes_per[mode];
    const double us = ms * 1e3 / launches;
    printf("{\"mode\": \"%s\", \"accesses\": %u, \"bytes_per_access\": %d, \"known_bytes\": %.0f, \"us_per_launch\": %.2f, "
           "\"useful_GBps\": %.1f}\n",
           names[mode], n, bytes_per[mode], known, us, known / us / 1e3);
    fflush(stdout);
  }
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
