// sptr_math.h — float3 arithmetic with the evaluation order of the reference's glm usage, for the
// HIP kernels and the host layer of libsptr_hip.  Every operation is written out so that, compiled
// with -ffp-contract=off and correctly rounded div/sqrt (HIP default), device results equal the CPU
// reference operation for operation.  Reference semantics followed:
//   glm::normalize  -> v * (1/sqrt(dot))         (used by Camera.cpp:45-47, Material.cpp:85)
//   wf::safe_normalize -> 0 if dot<=0            (include/wavefront/wf_math.h:28-33)
//   glm::reflect    -> I - N*dot(N,I)*2          (wf_pt_cpu.cpp:153)
//   glm::mix        -> x*(1-a) + y*a             (EnvironmentManager.cpp:45, Material.h:48)
//   wf::wang_hash / default_rand01               (include/wavefront/wf_math.h:35-49)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>

#include "cr_math.h"
#define SPTR_HD __host__ __device__ __forceinline__
#else
#include <cmath>
#define SPTR_HD inline
#endif

namespace sptr {

struct vec3 {
  float x, y, z;
};

SPTR_HD vec3 v3(float x, float y, float z) { return vec3{x, y, z}; }
SPTR_HD vec3 operator+(vec3 a, vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
SPTR_HD vec3 operator-(vec3 a, vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
SPTR_HD vec3 operator-(vec3 a) { return v3(-a.x, -a.y, -a.z); }
SPTR_HD vec3 operator*(vec3 a, vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
SPTR_HD vec3 operator*(vec3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
SPTR_HD vec3 operator*(float s, vec3 a) { return v3(s * a.x, s * a.y, s * a.z); }
SPTR_HD vec3 operator/(vec3 a, vec3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
SPTR_HD vec3 operator/(vec3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
SPTR_HD vec3 operator+(vec3 a, float s) { return v3(a.x + s, a.y + s, a.z + s); }
SPTR_HD vec3 operator-(float s, vec3 a) { return v3(s - a.x, s - a.y, s - a.z); }

SPTR_HD float fmax_g(float a, float b) { return (a < b) ? b : a; }  // glm::max / std::max
SPTR_HD float fmin_g(float a, float b) { return (b < a) ? b : a; }  // glm::min / std::min
SPTR_HD float clamp_g(float x, float lo, float hi) { return fmin_g(fmax_g(x, lo), hi); }
SPTR_HD vec3 clamp_g(vec3 v, float lo, float hi) { return v3(clamp_g(v.x, lo, hi), clamp_g(v.y, lo, hi), clamp_g(v.z, lo, hi)); }
SPTR_HD float dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
SPTR_HD vec3 cross(vec3 a, vec3 b) { return v3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
SPTR_HD vec3 reflect(vec3 i, vec3 n) { return i - n * dot(n, i) * 2.0f; }
SPTR_HD vec3 mix(vec3 a, vec3 b, float t) { return a * (1.0f - t) + b * t; }

#if defined(__HIPCC__)
SPTR_HD float sq_root(float x) { return sqrtf(x); }
#else
inline float sq_root(float x) { return std::sqrt(x); }
#endif
// 1/sqrt(l2) with both operations correctly rounded.  Device code uses the short correction
// sequences of cr_math.h (bit-identical in range, verified exhaustively on gfx950).
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ float inv_length(float l2) { return inv_len(l2); }
__device__ __forceinline__ float inv_length_dir(float l2) { return inv_len_nrm(l2); }
__device__ __forceinline__ float inv_length_unit(float l2) { return inv_len_unit(l2); }
__device__ __forceinline__ float inv_length_renorm(float l2) { return inv_len_unit_cf(l2); }
#else
SPTR_HD float inv_length(float l2) { return 1.0f / sq_root(l2); }
SPTR_HD float inv_length_dir(float l2) { return 1.0f / sq_root(l2); }
SPTR_HD float inv_length_unit(float l2) { return 1.0f / sq_root(l2); }
SPTR_HD float inv_length_renorm(float l2) { return 1.0f / sq_root(l2); }
#endif
SPTR_HD vec3 normalize(vec3 v) { return v * inv_length(dot(v, v)); }
SPTR_HD vec3 safe_normalize(vec3 v) {
  const float l2 = dot(v, v);
  if (l2 <= 0.0f) return v3(0.0f, 0.0f, 0.0f);
  return v * inv_length(l2);
}
// The same operations for direction-like vectors whose squared length is known to lie in
// [2^-96, 2^100] (camera and ray directions, reflections, refractions, cosine samples, tangents:
// lengths between ~0.04 and ~2), where the device skips the range handling of inv_len.
SPTR_HD vec3 normalize_dir(vec3 v) { return v * inv_length_dir(dot(v, v)); }
SPTR_HD vec3 safe_normalize_dir(vec3 v) {
  const float l2 = dot(v, v);
  if (l2 <= 0.0f) return v3(0.0f, 0.0f, 0.0f);
  return v * inv_length_dir(l2);
}
// The same results again, for vectors that are unit length up to a few roundings already (ray
// directions looked up in the environment, face-forwarded normals, reflections, refractions and
// cosine samples of unit vectors): the device takes cr_math.h's closed form near |v| = 1.
SPTR_HD vec3 renormalize_dir(vec3 v) { return v * inv_length_unit(dot(v, v)); }
SPTR_HD vec3 safe_renormalize_dir(vec3 v) {
  const float l2 = dot(v, v);
  if (l2 <= 0.0f) return v3(0.0f, 0.0f, 0.0f);
  return v * inv_length_unit(l2);
}
// The same result again for the output of a normalization (normalize_dir, renormalize_dir,
// renormalized_again): its squared length lies within a few ulps of 1, never 0, so neither the zero
// test of safe_renormalize_dir nor inv_len_unit's range test can fire, and the device evaluates the
// closed form with no branch.  (A NaN vector stays NaN: its l2 gives a NaN scale.)
SPTR_HD vec3 renormalized_again(vec3 v) { return v * inv_length_renorm(dot(v, v)); }

// normalize(vec3(0.3, 0.6, -0.8)), the sun direction of EnvironmentManager::getSkyColor
// (src/EnvironmentManager.cpp:48), evaluated once in glm's order; tests/cpp/test_index_math.cpp checks
// the literal against normalize() on the host.  (The device's correctly rounded normalize sequence
// is not constant-folded by the compiler.)
constexpr float kSunDirX = 0x1.263e86p-2f, kSunDirY = 0x1.263e86p-1f, kSunDirZ = -0x1.88535ep-1f;

SPTR_HD uint32_t wang_hash(uint32_t a) {
  a = (a ^ 61u) ^ (a >> 16u);
  a *= 9u;
  a = a ^ (a >> 4u);
  a *= 0x27d4eb2du;
  a = a ^ (a >> 15u);
  return a;
}
SPTR_HD float rand01(uint32_t& s) {
  s = wang_hash(s);
  return float(s & 0x00FFFFFFu) / float(0x01000000u);
}

}  // namespace sptr
