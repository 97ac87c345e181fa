// crmath_check.hip — exhaustive / dense check that the fast correctly-rounded helpers of
// simple-path-tracer_amd/csrc/cr_math.h are bit-identical to the compiler's IEEE operators on
// gfx950 over their stated domains.  Built and run by tests/test_gpu_crmath.py.
//   sqrt_nrm : every float in [2^-96, 2^100]
//   rcp_nrm  : every float in [2^-100, 2^100]; inv_len_nrm and inv_len_unit (closed form within
//              1024 ulps of 1.0, general sequence elsewhere) over the same floats
//   inv_len  : every one of the 2^32 float bit patterns (NaN == NaN), against 1.0f / sqrtf(x)
//   div_nrm  : divisors 1..8192 and the bench/test image sizes, 2^22 dividends each of the form
//              float(x) + j (x integer pixel coordinate < b, j a 24-bit jitter), plus random floats;
//              and 2^30 random pairs with divisors in [1/2, 1), dividends in [-1, 1] down to 2^-100
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "cr_math.h"

using namespace sptr;

__device__ unsigned long long g_bad[5];
__device__ unsigned int g_first[5];

__global__ void k_sqrt(uint32_t lo, uint32_t hi) {
  for (uint64_t u = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u <= hi; u += (uint64_t)gridDim.x * blockDim.x) {
    const float x = __uint_as_float((uint32_t)u);
    if (__float_as_uint(sqrt_nrm(x)) != __float_as_uint(sqrtf(x))) {
      atomicAdd(&g_bad[0], 1ull);
      atomicMin(&g_first[0], (uint32_t)u);
    }
  }
}

__global__ void k_rcp(uint32_t lo, uint32_t hi) {
  for (uint64_t u = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u <= hi; u += (uint64_t)gridDim.x * blockDim.x) {
    const float y = __uint_as_float((uint32_t)u);
    const float ref = 1.0f / y;
    const uint32_t il = __float_as_uint(1.0f / sqrtf(y));
    if (__float_as_uint(rcp_nrm(y)) != __float_as_uint(ref) || __float_as_uint(inv_len_nrm(y)) != il ||
        __float_as_uint(inv_len_unit(y)) != il ||
        ((__float_as_uint(y) + 1024u - 0x3F800000u) <= 2048u && __float_as_uint(inv_len_unit_cf(y)) != il)) {
      atomicAdd(&g_bad[1], 1ull);
      atomicMin(&g_first[1], (uint32_t)u);
    }
  }
}

__global__ void k_invlen_all() {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u <= 0xFFFFFFFFull; u += (uint64_t)gridDim.x * blockDim.x) {
    const float x = __uint_as_float((uint32_t)u);
    const float got = inv_len(x), ref = 1.0f / sqrtf(x);
    const bool same = __float_as_uint(got) == __float_as_uint(ref) || (got != got && ref != ref);
    if (!same) {
      atomicAdd(&g_bad[3], 1ull);
      atomicMin(&g_first[3], (uint32_t)u);
    }
  }
}

__device__ __forceinline__ uint32_t hash(uint32_t a) {
  a = (a ^ 61u) ^ (a >> 16u);
  a *= 9u;
  a = a ^ (a >> 4u);
  a *= 0x27d4eb2du;
  return a ^ (a >> 15u);
}

__global__ void k_div(const float* divisors, int nd, uint32_t samples) {
  const float b = divisors[blockIdx.y];
  const DivBy d = div_by(b);
  const uint32_t ib = (uint32_t)b;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < samples; s += gridDim.x * blockDim.x) {
    const uint32_t h = hash(s * 2654435761u ^ blockIdx.y * 97u);
    float a;
    if (s & 1u) {
      const uint32_t x = ib ? hash(h) % (ib + 1u) : 0u;
      a = float(x) + float(h & 0x00FFFFFFu) / float(0x01000000u);  // pixel + jitter, as raygen
    } else {
      a = __uint_as_float(0x0D800000u + hash(h) % (0x72000000u - 0x0D800000u));  // [2^-100, 2^100)
    }
    if (__float_as_uint(div_nrm(a, d)) != __float_as_uint(a / b)) {
      atomicAdd(&g_bad[2], 1ull);
      atomicMin(&g_first[2], __float_as_uint(a));
    }
  }
}

// divisors in [1/2, 1) (the cubemap's major axis, 1/sqrt(3)..1), dividends in [-1, 1] with exponents
// down to 2^-100 (the face coordinates): 2^30 random pairs
__global__ void k_div_unit(uint32_t samples) {
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < samples; s += gridDim.x * blockDim.x) {
    const uint32_t h = hash(s * 2654435761u + 12345u), g = hash(h ^ 0x9E3779B9u);
    const float b = __uint_as_float(0x3F000000u | (h & 0x007FFFFFu));                         // [0.5, 1)
    const uint32_t e = 27u + g % 100u;                                                          // 2^-100 .. 2^-1
    const float a = __uint_as_float(((g >> 8) & 1u) << 31 | e << 23 | (hash(g) & 0x007FFFFFu));
    if (__float_as_uint(div_nrm(a, div_by(b))) != __float_as_uint(a / b)) {
      atomicAdd(&g_bad[4], 1ull);
      atomicMin(&g_first[4], __float_as_uint(a));
    }
  }
}

int main() {
  const unsigned long long zero[5] = {0, 0, 0, 0, 0};
  const unsigned int big[5] = {~0u, ~0u, ~0u, ~0u, ~0u};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bad), zero, sizeof(zero));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_first), big, sizeof(big));
  const uint32_t s_lo = 0x0F800000u, s_hi = 0x71800000u;  // 2^-96 .. 2^100
  const uint32_t r_lo = 0x0D800000u, r_hi = 0x71800000u;  // 2^-100 .. 2^100
  hipLaunchKernelGGL(k_sqrt, dim3(8192), dim3(256), 0, 0, s_lo, s_hi);
  hipLaunchKernelGGL(k_rcp, dim3(8192), dim3(256), 0, 0, r_lo, r_hi);
  hipLaunchKernelGGL(k_invlen_all, dim3(16384), dim3(256), 0, 0);
  std::vector<float> dv;
  for (int b = 1; b <= 8192; ++b) dv.push_back((float)b);
  for (float b : {3840.0f, 2160.0f, 7680.0f, 4320.0f, 15360.0f}) dv.push_back(b);
  float* ddv = nullptr;
  (void)hipMalloc(&ddv, dv.size() * sizeof(float));
  (void)hipMemcpy(ddv, dv.data(), dv.size() * sizeof(float), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_div, dim3(16, (unsigned)dv.size()), dim3(256), 0, 0, ddv, (int)dv.size(), 1u << 18);
  hipLaunchKernelGGL(k_div_unit, dim3(8192), dim3(256), 0, 0, 1u << 30);
  if (hipDeviceSynchronize() != hipSuccess) {
    std::printf("hip error\n");
    return 2;
  }
  unsigned long long bad[5];
  unsigned int first[5];
  (void)hipMemcpyFromSymbol(bad, HIP_SYMBOL(g_bad), sizeof(bad));
  (void)hipMemcpyFromSymbol(first, HIP_SYMBOL(g_first), sizeof(first));
  const char* names[5] = {"sqrt_nrm", "rcp_nrm/inv_len_nrm/inv_len_unit", "div_nrm", "inv_len (all 2^32)",
                          "div_nrm unit divisors"};
  int rc = 0;
  for (int i = 0; i < 5; ++i) {
    std::printf("%s: %llu mismatches%s", names[i], bad[i], bad[i] ? "" : "\n");
    if (bad[i]) {
      std::printf(" (first input bits 0x%08x)\n", first[i]);
      rc = 1;
    }
  }
  (void)hipFree(ddv);
  return rc;
}
