// cr_math.h — correctly rounded f32 sqrt, reciprocal and division by a loop-invariant divisor,
// for the operand ranges the path tracer uses, without the denormal pre-scaling, VCC scaling and
// special-case fix-ups of the compiler's general gfx950 expansions.
//
// Each helper replays the compiler's own correction sequence (v_sqrt + the +-1 ulp residual test;
// v_rcp + the Newton/Markstein fma chain of v_div_scale/v_div_fmas/v_div_fixup), so for in-range
// operands the result is bit-identical to sqrtf(x), 1.0f / x and a / b.  That claim is checked
// exhaustively on the GPU (every float of the ranges below) by tests/hip/crmath_check.hip, run by
// tests/test_gpu_crmath.py.  Callers guard the range and fall back to the IEEE operators.
#pragma once
#include <hip/hip_runtime.h>

namespace sptr {

constexpr float kCrLo = 0x1p-96f;  // sqrt_nrm domain: [kCrLo, kCrHi]
constexpr float kCrHi = 0x1p100f;

// sqrtf(x) for x in [2^-96, FLT_MAX]
__device__ __forceinline__ float sqrt_nrm(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u);
  const float sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float em = __builtin_fmaf(-sm, s, x);
  const float ep = __builtin_fmaf(-sp, s, x);
  float r = (0.0f >= em) ? sm : s;
  r = (0.0f < ep) ? sp : r;
  return r;
}

// 1.0f / y for y in [2^-100, 2^100]
__device__ __forceinline__ float rcp_nrm(float y) {
  const float r0 = __builtin_amdgcn_rcpf(y);
  const float r1 = __builtin_fmaf(__builtin_fmaf(-y, r0, 1.0f), r0, r0);
  const float q1 = __builtin_fmaf(__builtin_fmaf(-y, r1, 1.0f), r1, r1);
  return __builtin_fmaf(__builtin_fmaf(-y, q1, 1.0f), r1, q1);
}

// Loop-invariant divisor b (|b| in [2^-100, 2^100]): the refined reciprocal is computed once.
struct DivBy {
  float b, r;
};
__device__ __forceinline__ DivBy div_by(float b) {
  const float r0 = __builtin_amdgcn_rcpf(b);
  return DivBy{b, __builtin_fmaf(__builtin_fmaf(-b, r0, 1.0f), r0, r0)};
}
// a / d.b for a = 0 or |a| in [2^-100, 2^100] with the quotient in the normal range
__device__ __forceinline__ float div_nrm(float a, const DivBy& d) {
  const float q0 = a * d.r;
  const float q1 = __builtin_fmaf(__builtin_fmaf(-d.b, q0, a), d.r, q0);
  return __builtin_fmaf(__builtin_fmaf(-d.b, q1, a), d.r, q1);
}

// 1 / sqrt(l2) as glm's normalize evaluates it (two correctly rounded operations), for l2 in
// [2^-96, 2^100]: the squared length of a direction-like vector (callers: normalize_dir).
__device__ __forceinline__ float inv_len_nrm(float l2) { return rcp_nrm(sqrt_nrm(l2)); }

// 1 / sqrt(l2) as inv_len_nrm, in closed form when l2 lies within 1024 ulps of 1.0 — the squared
// length of a vector that is already unit length up to rounding (re-normalized ray directions,
// normals, reflections, cosine samples).  With l2 = 1 + d ulps: for d >= 0 (ulp 2^-23),
// sqrt = 1 + floor(d/2) 2^-23 and its reciprocal 1 - floor(d/2) 2^-23, i.e. bits 0x3F800000 -
// (d & ~1); for d < 0 (ulp 2^-24), sqrt = 1 - j 2^-24 with j = ceil(-d/2) and the reciprocal is
// 1 + ceil(j/2) 2^-23.  The neglected second-order terms stay below a quarter ulp for |d| < 2900;
// checked against 1.0f / sqrtf over the whole window on the CPU (tests/test_cr_math_cpu.py) and on
// the GPU (tests/hip/crmath_check.hip).  Other l2 take the general sequence.
// inv_len_unit_cf: the closed form alone, both signs of d evaluated and selected (no divergent
// branch), for l2 of a vector that came out of a normalization (|d| a few ulps), where inv_len_unit's
// range test cannot fail.  On the bits b of l2 (0x3F800000 is even): d >= 0 gives 0x7F000000 -
// (b & ~1); d < 0 gives 0x3F800000 + ceil(-d / 4) = 0x3F800000 + ((0x3F800003 - b) >> 2).
__device__ __forceinline__ float inv_len_unit_cf(float l2) {
  const uint32_t b = __float_as_uint(l2);
  const uint32_t up = 0x7F000000u - (b & ~1u), dn = 0x3F800000u + ((0x3F800003u - b) >> 2);
  return __uint_as_float((int)b >= 0x3F800000 ? up : dn);
}
__device__ __forceinline__ float inv_len_unit(float l2) {
  const int d = (int)__float_as_uint(l2) - 0x3F800000;
  if (__builtin_expect(d < -1024 || d > 1024, 0)) return inv_len_nrm(l2);
  return inv_len_unit_cf(l2);
}

// 1 / sqrt(l2) for every float l2 (bit-identical to 1.0f / sqrtf(l2), checked over all 2^32 inputs by
// tests/hip/crmath_check.hip).  Out-of-domain inputs are scaled by an even power of two, which
// commutes exactly with the correctly rounded sqrt (the scaled root stays normal), so there is no
// separate IEEE slow path for the compiler to if-convert into every normalize.
__device__ __forceinline__ float inv_len(float l2) {
  const bool lo = l2 < kCrLo, hi = l2 > kCrHi;
  const float sc = lo ? 0x1p100f : (hi ? 0x1p-100f : 1.0f);
  const float un = lo ? 0x1p-50f : (hi ? 0x1p50f : 1.0f);  // 1 / sqrt(sc)
  const float s = sqrt_nrm(l2 * sc) * un;
  const float r = rcp_nrm(s);
  return s == 0.0f ? __builtin_copysignf(__builtin_huge_valf(), s) : (s == __builtin_huge_valf() ? 0.0f : r);
}

}  // namespace sptr
