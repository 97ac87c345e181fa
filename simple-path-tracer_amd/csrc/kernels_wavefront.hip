// kernels_wavefront.hip — the wavefront stages of the MI355X (gfx950) path tracer.
//
//   raygen    : path init (seeding, jitter, camera ray) is a device function evaluated inside the
//               bounce-0 trace and shade kernels: bounce 0 covers every path densely, so it needs
//               no queue and no path-state round trip.  (GLRenderer.cpp:384-408, Camera.cpp:95-106)
//   k_trace   : closest-hit BVH2 traversal + Embree-style Moeller-Trumbore triangles + the
//               reference's quadratic spheres, one thread per queued path.   (wf_pt_cpu.cpp:28-56)
//   k_shade   : miss/env, emission, direct-light shadow tasks, metal/glass/diffuse continuation;
//               survivors and shadow rays are compacted by wave64 ballot + per-wave LDS staging,
//               one global atomic per ~450 queue entries.                        (wf_pt_cpu.cpp:94-248)
//   k_shadow  : any-hit traversal of the shadow tasks, adds unoccluded light. (Light.cpp:16-40)
//   k_accum   : per-pixel sum of the wave's samples in accumulation order.  (GLRenderer.cpp:411-413)
//   k_resolve : mean -> ACES -> gamma 1/2.2 -> clamp -> 8-bit truncation.   (GLRenderer.cpp:416-431)
//
// Kernels run a fixed grid (<= 8 blocks per CU); each block takes a contiguous slice of the
// device-side queue, so a wavefront batch needs no host round trip between stages.  Arithmetic order follows the CPU reference line
// for line (see sptr_math.h); the file is compiled with -ffp-contract=off.  Box tests are the one
// place that uses fma: they only prune traversal and are padded to stay conservative.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>

#include "sptr_internal.h"

// Occupancy hints (min waves per SIMD); 1 = let the register allocator decide.
#ifndef SPTR_TRACE_WAVES
#define SPTR_TRACE_WAVES 7  // measured: 7 -> +6% on C2 (SGPR-limited to 6 otherwise)
#endif
#ifndef SPTR_TRACE_PM_WAVES
#define SPTR_TRACE_PM_WAVES SPTR_TRACE_WAVES
#endif
#ifndef SPTR_TRACE_WP_WAVES
#define SPTR_TRACE_WP_WAVES SPTR_TRACE_WAVES  // lane-group bounce 0 (sharded LDS-scene batches)
#endif
#ifndef SPTR_TRACE4_WAVES
#define SPTR_TRACE4_WAVES 7  // wide BVH, bounces >= 1 (refilling kernels, no packed FP32): C5 16.0 -> 15.2-15.6 ms/step (r02 ab24/25)
                             // (bounce 0 stays at 7: coherent rays gain more from occupancy, 8.4 -> 5.4)
#endif
#ifndef SPTR_SHADE_WAVES
#define SPTR_SHADE_WAVES 5  // 111 -> 96 VGPRs, 4 -> 5 waves, no spills: C2 shade 0.971 -> 0.907 ms
#endif                      // (6 waves spills 48-76 B/lane; profiles/r01f_variants.txt)
#ifndef SPTR_BOUNCE_WAVES
#define SPTR_BOUNCE_WAVES 6  // r02 ab23 (no packed FP32): 8-way shard 0.548 -> 0.525 ms, 2-way 1.662 -> 1.638; 7 spills
#endif
#ifndef SPTR_TAIL_WAVES
#define SPTR_TAIL_WAVES 4  // scenes traversed from L2/HBM; r03: 1 -> 4 waves/SIMD, C5 tail (bounces 3-5) 1.46 ->
#endif                     // 1.22 ms, C3 (2-5) 0.77 -> 0.50 (8 waves: C3 0.80)
#ifndef SPTR_PT_WAVES
#define SPTR_PT_WAVES 1  // the path-per-thread integrators (k_pathtracer, k_optix)
#endif
#ifndef SPTR_TAIL_WAVES_LDS
#define SPTR_TAIL_WAVES_LDS 1  // LDS-staged scenes (sharded C2: 4 waves 0.569 vs 1 wave 0.558 ms per rank at G = 8)
#endif
#ifndef SPTR_SHADOW_WAVES
#define SPTR_SHADOW_WAVES 6  // LDS-staged BVH2 scenes: 7 waves measured slower on C2 (0.409 -> 0.426 ms)
#endif
#ifndef SPTR_SKY_ILP
#define SPTR_SKY_ILP 4  // independent samples per step of k_sky's per-pixel loop
#endif
#define SPTR_STR2(x) #x
#define SPTR_STR(x) SPTR_STR2(x)  // a register name for an occupancy cap's clobber list
// A launch timed by the stage timer (g_launch_timing set: the dispatch records its start and/or end into
// the events), else a plain launch.
#define SPTR_TIMED_LAUNCH(kern, grid, block, lds, stream, ...)                                              \
  do {                                                                                                   \
    if (g_launch_timing.start || g_launch_timing.stop) {                                                 \
      const LaunchTiming lt_ = g_launch_timing;                                                          \
      g_launch_timing = LaunchTiming{};                                                                  \
      hipExtLaunchKernelGGL(kern, grid, block, lds, stream, lt_.start, lt_.stop, 0u, __VA_ARGS__);         \
    } else {                                                                                             \
      hipLaunchKernelGGL(kern, grid, block, lds, stream, __VA_ARGS__);                                   \
    }                                                                                                    \
  } while (0)
#ifndef SPTR_SHADOW4_WAVES
#define SPTR_SHADOW4_WAVES 7  // BVH4 from L2/HBM with 64-B nodes: C5 shadow 7.85 -> 7.44 ms/step (r02 ab2;
#endif                        // 5 -> 6 waves was 8.34 -> 7.19 with 128-B nodes)

namespace sptr {
thread_local LaunchTiming g_launch_timing;
thread_local unsigned long long* g_tslot = nullptr;
// w with the timing slot the stage timer set for this launch (taken: the next launch is untimed)
WaveView with_tslot(const WaveView& w) {
  WaveView t = w;
  t.tslot = g_tslot;
  g_tslot = nullptr;
  return t;
}  // (sptr_internal.h)
// Any-hit wide walks visit the farthest hit child first: a ray leaving a surface has no occluder among
// the boxes around its origin, so the near-first order explores them before the far occluder (r03b A/B:
// C5 shadow 4.42 -> 3.88 ms/step, C3 0.81 -> 0.80).  The any-hit BVH2 walk of LDS scenes stays
// near-first (far-first: no change on C2).
constexpr bool kAnyHitFar = true;
}  // namespace sptr

namespace sptr {

// --------------------------------------------------------------------------------- small helpers
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Block-local dense append: one LDS atomic per wave; the lanes' outputs land contiguously in the
// block's segment.  Every lane of the wave must call it together (it ballots).
__device__ __forceinline__ uint32_t block_append(uint32_t* s_cnt, bool pred) {
  const unsigned long long m = __ballot(pred);
  if (m == 0ull) return 0u;
  const uint32_t lane = lane_id();
  const int leader = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0u;
  if ((int)lane == leader) base = atomicAdd(s_cnt, (uint32_t)__popcll(m));
  base = __shfl(base, leader);
  return base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}
// Block-local work counter: every lane with pred takes the next index (one LDS atomic per wave).
__device__ __forceinline__ uint32_t block_take(uint32_t* s_next, bool pred) { return block_append(s_next, pred); }
// XCD-aware logical block index.  Workgroups are dispatched round-robin over the 8 XCDs, so with
// the identity mapping neighbouring slices (neighbouring image regions for bounce 0) land on
// different XCDs and every XCD's private 4 MB L2 has to hold the BVH working set of the whole
// frame.  Remapping gives XCD x the contiguous logical range [x*G/8, (x+1)*G/8).
constexpr uint32_t kXcds = 8;
constexpr uint64_t kL2BytesPerXcd = 4ull << 20;
__device__ __forceinline__ uint32_t logical_block() {
  const uint32_t g = gridDim.x, b = blockIdx.x;
  return (g % kXcds) ? b : (b % kXcds) * (g / kXcds) + b / kXcds;
}
// Work schedule of the stage kernels: block-sized chunks dealt round-robin over the (logical)
// blocks, chunk c -> block c % G.  Per-item cost varies by orders of magnitude across the image
// (sky vs a 10M-triangle mesh), so contiguous per-block slices leave the kernel waiting on the
// blocks that drew the expensive region; dealing chunks balances statistically and keeps all CUs
// on one band of the frame at a time (shared BVH working set).  Every block processes at most
// `per` items, which is the stride of its output segment: seg0 = logical block * per.
struct Sched {
  uint32_t first, step, per, seg0, end;  // items first + j*step + [0, kBlock), below end
};
__device__ __forceinline__ Sched block_sched(uint32_t n) {
  Sched s;
  const uint32_t lb = logical_block();
  const uint32_t span = gridDim.x * kBlock;
  s.per = (n + span - 1) / span * kBlock;
  s.seg0 = lb * s.per;
  s.first = lb * kBlock;
  s.step = span;
  s.end = n;
  return s;
}

// Consumer prologue: exclusive scan of the producer's per-block segment counts into LDS
// (s_off[0..nseg]); returns the total.  Contains block barriers: call from every thread.
__device__ uint32_t seg_scan(const SegTable& t, uint32_t nseg, uint32_t* s_off, uint32_t& per) {
  __shared__ uint32_t s_wave[kBlock / 64];
  // every count load is issued before the first use (unrolled, predicated), so the prologue costs
  // one memory round trip instead of one per segment: it bounds the duration of the short launches
  // of the deep bounces (and of every launch in a small, e.g. 8-way sharded, batch)
  constexpr uint32_t kChunk = kMaxSegs / kBlock;
  const uint32_t chunk = (nseg + kBlock - 1) / kBlock;
  const uint32_t b0 = threadIdx.x * chunk;
  const uint32_t per_v = *t.per;
  uint32_t v[kChunk];
#pragma unroll
  for (uint32_t j = 0; j < kChunk; ++j) v[j] = (j < chunk && b0 + j < nseg) ? t.cnt[b0 + j] : 0u;
  uint32_t sum = 0u;
#pragma unroll
  for (uint32_t j = 0; j < kChunk; ++j) sum += v[j];
  uint32_t incl = sum;
  const uint32_t lane = lane_id();
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t v = __shfl_up(incl, off);
    if (lane >= (uint32_t)off) incl += v;
  }
  if (lane == 63u) s_wave[threadIdx.x >> 6] = incl;
  __syncthreads();
  uint32_t run = incl - sum;
  for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) run += s_wave[w];
#pragma unroll
  for (uint32_t j = 0; j < kChunk; ++j)
    if (j < chunk && b0 + j < nseg) {
      s_off[b0 + j] = run;
      run += v[j];
    }
  if (threadIdx.x == 0) {
    uint32_t tot = 0u;
    for (uint32_t w = 0; w < kBlock / 64; ++w) tot += s_wave[w];
    s_off[nseg] = tot;
  }
  per = per_v;
  __syncthreads();
  return s_off[nseg];
}
// Compacted index i -> physical slot: the largest segment b with s_off[b] <= i (a fixed 11-step
// search over LDS; empty segments are skipped because the largest such b is the non-empty one).
// Candidates past the last segment read s_off[nseg] = the total, which exceeds every valid i, so
// each step is an unconditional LDS read and a select (r05: the bounds test in front of the read
// made every step a branch with its own exec-mask bookkeeping and a full memory wait).
__device__ __forceinline__ uint32_t seg_slot(const uint32_t* s_off, uint32_t nseg, uint32_t per, uint32_t i) {
  uint32_t b = 0u;
#pragma unroll
  for (uint32_t step = kMaxSegs / 2; step; step >>= 1) {
    const uint32_t c = min(b + step, nseg);
    b = s_off[c] <= i ? c : b;
  }
  return b * per + (i - s_off[b]);
}
// Producer epilogue: publish this block's output count (and, from block 0, the segment stride).
__device__ __forceinline__ void seg_publish(const SegTable& t, const uint32_t* s_cnt, uint32_t per) {
  __syncthreads();
  if (threadIdx.x == 0) {
    t.cnt[logical_block()] = *s_cnt;
    if (blockIdx.x == 0) *t.per = per;
  }
}

__device__ __forceinline__ vec3 xyz(float4 a) { return v3(a.x, a.y, a.z); }
__device__ __forceinline__ float4 f4(vec3 a, float w) { return make_float4(a.x, a.y, a.z, w); }
__device__ __forceinline__ float clamp_std(float v, float lo, float hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }

// SPTR_ABLATE timing experiments (sptr_api.cpp frame_view): compiled out of normal builds, so the
// production kernels carry neither the field nor its branches.
__device__ __forceinline__ uint32_t ablate(const FrameView& f) {
#ifdef SPTR_EXPERIMENT_KNOBS
  return f.ablate;
#else
  (void)f;
  return 0u;
#endif
}
__device__ __forceinline__ uint32_t grid_threads() { return gridDim.x * blockDim.x; }

// tile-packed local pixel -> image coordinates (interleaved 32x32 tile sharding)
__device__ __forceinline__ bool local_pixel(const FrameView& f, uint32_t l, int& x, int& y) {
  const uint32_t lt = l >> 10, w = l & 1023u;
  const uint32_t t = lt * (uint32_t)f.G + (uint32_t)f.R;
  const uint32_t tyu = fast_div(f.div_ntx, t);
  const int tx = (int)(t - tyu * (uint32_t)f.ntx), ty = (int)tyu;
  x = tx * kTile + (int)(w & 31u);
  y = ty * kTile + (int)(w >> 5);
  return x < f.W && y < f.H;
}

// Per-call values that a captured launch graph must not bake in (sptr_api.cpp run_graph): the call's
// first accumulation index and whether it restarts the accumulation, written by k_frame_dyn at the
// head of every render call; the FrameView carries the batch's offset in acc0 and a candidate reset
// flag (1 for the call's first batch).  f.dyn == null (query kernels): acc0 / reset are absolute.
__device__ __forceinline__ FrameView frame_dyn(FrameView f) {
  if (f.dyn) {
    f.acc0 = f.dyn[0] + f.acc0;
    f.reset = f.reset & f.dyn[1];
  }
  return f;
}
// clear (may be null): the two words after an in-sequence k_cull's list (its unculled pixel count and a
// spare), zeroed here instead of by a memset node of their own.  t0 (may be null): the start word of the
// call span's timing slot (the call's last k_accum takes its end, ktime_end).
__global__ void k_frame_dyn(uint32_t* dyn, uint32_t frame_begin, uint32_t reset, uint32_t total, uint32_t* clear,
                            unsigned long long* t0) {
  if (threadIdx.x == 0) {
    dyn[0] = frame_begin;
    dyn[1] = reset;
    dyn[2] = total;
    if (t0) t0[0] = (unsigned long long)wall_clock64();
  }
  if (threadIdx.x == 0) {
    if (clear) {
      clear[0] = 0u;
      clear[1] = 0u;
    }
  }
}

// Camera::getRayDirection
__device__ __forceinline__ vec3 camera_dir(const FrameView& f, float u, float v) {
  const float nx = (u - 0.5f) * 2.0f;
  const float ny = -(v - 0.5f) * 2.0f;
  const vec3 d = f.cam_f + nx * f.half_w * f.cam_r + ny * f.half_h * f.cam_u;
  return normalize_dir(d);
}

// --------------------------------------------------------------------------------- intersection
struct Ray {
  vec3 o, d, inv, oinv;
};
__device__ __forceinline__ Ray make_ray(vec3 o, vec3 d) {
  Ray r;
  r.o = o;
  r.d = d;
  // v_rcp_f32 (1 ulp): the inverse direction only feeds the conservative box test
  const float eps = 1e-20f;
  r.inv = v3(__builtin_amdgcn_rcpf(fabsf(d.x) > eps ? d.x : copysignf(eps, d.x)),
             __builtin_amdgcn_rcpf(fabsf(d.y) > eps ? d.y : copysignf(eps, d.y)),
             __builtin_amdgcn_rcpf(fabsf(d.z) > eps ? d.z : copysignf(eps, d.z)));
  r.oinv = v3(0.0f, 0.0f, 0.0f);
  return r;
}

// Slab test of one child box.  (b - o) * inv avoids the cancellation of the fma(b, inv, -o*inv)
// form near the origin; the exit distance is padded by 2^-20 relative (~8 ulp) to absorb the
// subtraction, product and v_rcp rounding, so the test only prunes and never rejects a box that
// the exact test would accept at a primitive's hit distance.
__device__ __forceinline__ bool slab(float xlo, float xhi, float ylo, float yhi, float zlo, float zhi, const Ray& r,
                                     float tnear, float tfar, float& tent) {
  const float tx0 = (xlo - r.o.x) * r.inv.x, tx1 = (xhi - r.o.x) * r.inv.x;
  const float ty0 = (ylo - r.o.y) * r.inv.y, ty1 = (yhi - r.o.y) * r.inv.y;
  const float tz0 = (zlo - r.o.z) * r.inv.z, tz1 = (zhi - r.o.z) * r.inv.z;
  const float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), tnear));
  const float tmax = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tfar));
  tent = tmin;
  return tmin <= tmax * 1.00000095f;
}

__device__ __forceinline__ float e_dot(vec3 a, vec3 b) {
  return __builtin_fmaf(a.x, b.x, __builtin_fmaf(a.y, b.y, a.z * b.z));
}
__device__ __forceinline__ vec3 e_cross(vec3 a, vec3 b) {
  return v3(__builtin_fmaf(a.y, b.z, -(a.z * b.y)), __builtin_fmaf(a.z, b.x, -(a.x * b.z)),
            __builtin_fmaf(a.x, b.y, -(a.y * b.x)));
}
__device__ __forceinline__ float xorsign(float x, float s) {
  return __uint_as_float(__float_as_uint(x) ^ (__float_as_uint(s) & 0x80000000u));
}

// Embree default Moeller-Trumbore (restated; see oracle/wf_oracle.cpp tri_hit): accepts
// tnear*|den| < T <= tfar*|den|.  Triangle record: v0, e1 = v0-v1, e2 = v2-v0, Ng = cross(e2,e1).
__device__ __forceinline__ bool tri_hit4(float4 a, float4 b, float4 c, const Ray& r, float tnear, float tfar, float& t) {
  const vec3 v0 = v3(a.x, a.y, a.z), e1 = v3(a.w, b.x, b.y), e2 = v3(b.z, b.w, c.x), ng = v3(c.y, c.z, c.w);
  const vec3 C = v0 - r.o;
  const vec3 R = e_cross(C, r.d);
  const float den = e_dot(ng, r.d);
  const float aden = fabsf(den);
  const float U = xorsign(e_dot(R, e2), den);
  const float V = xorsign(e_dot(R, e1), den);
  if (!(den != 0.0f && U >= 0.0f && V >= 0.0f && U + V <= aden)) return false;
  const float T = xorsign(e_dot(ng, C), den);
  if (!(aden * tnear < T && T <= aden * tfar)) return false;
  t = T / aden;
  return true;
}
__device__ __forceinline__ bool tri_hit(const float4* tris, uint32_t i, const Ray& r, float tnear, float tfar, float& t) {
  return tri_hit4(tris[3 * i + 0], tris[3 * i + 1], tris[3 * i + 2], r, tnear, tfar, t);
}

// EmbreeBackend.cpp:223-314 sphere callbacks, same evaluation order.
__device__ __forceinline__ bool sphere_roots(float4 s, const Ray& r, float& t1, float& t2) {
  const vec3 D = r.d;
  const float ox = r.o.x - s.x, oy = r.o.y - s.y, oz = r.o.z - s.z;
  const float a = D.x * D.x + D.y * D.y + D.z * D.z;
  const float b = 2.0f * (ox * D.x + oy * D.y + oz * D.z);
  const float c = ox * ox + oy * oy + oz * oz - s.w * s.w;
  const float disc = b * b - 4.0f * a * c;
  if (!(disc >= 0.0f)) return false;
  const float sq = sqrtf(disc);
  t1 = (-b - sq) / (2.0f * a);
  t2 = (-b + sq) / (2.0f * a);
  return true;
}
__device__ __forceinline__ bool sphere_hit(float4 s, const Ray& r, float tnear, float tfar, float& t) {
  float t1, t2;
  if (!sphere_roots(s, r, t1, t2)) return false;
  float tt = -1.0f;
  if (t1 > tnear && t1 < tfar) tt = t1;
  else if (t2 > tnear && t2 < tfar) tt = t2;
  if (!(tt > 0.0f && tt < tfar)) return false;
  t = tt;
  return true;
}
__device__ __forceinline__ bool sphere_occ(float4 s, const Ray& r, float tnear, float tfar) {
  float t1, t2;
  if (!sphere_roots(s, r, t1, t2)) return false;
  return (t1 > tnear && t1 < tfar) || (t2 > tnear && t2 < tfar);
}

struct Visits {
  uint32_t nodes = 0, tris = 0, sph = 0;
  uint32_t stack_overflow = 0;  // a push was dropped (reported through kTotStackOverflow)
};

// Leaf = contiguous range of sorted primitive references (LBVH subtrees cover contiguous ranges):
// every primitive of the range is tested in a uniform loop; or, with kDirect (links read from wide
// nodes), possibly one primitive named by the link itself (kLeafDirect: one dependent load less per
// leaf).  Closest: updates tfar/ref.  Any-hit: returns on the first occluder.
template <bool kAny, bool kCount, bool kDirect = false>
__device__ __forceinline__ bool leaf_test(uint32_t link, const uint32_t* prim_ref, const float4* tris, const float4* sph,
                                          const Ray& r, float tnear, float& tfar, uint32_t& ref, Visits& vc) {
  const bool direct = kDirect && (link & kLeafDirect) != 0u;
  const uint32_t start = (link & ~kLeafBit) >> kLeafCountBits, cnt = direct ? 1u : (link & kLeafRangeMask) + 1u;
  bool hit = false;
  for (uint32_t j = 0; j < cnt; ++j) {
    const uint32_t pr = direct ? (start | ((link & kLeafDirectSphere) ? kSphereBit : 0u)) : prim_ref[start + j];
    const uint32_t idx = pr & kIndexMask;
    float t;
    if (pr & kSphereBit) {
      if (kCount) ++vc.sph;
      const float4 s = sph[idx];
      if (kAny) {
        if (sphere_occ(s, r, tnear, tfar)) return true;
      } else if (sphere_hit(s, r, tnear, tfar, t)) {
        tfar = t;
        ref = pr;
        hit = true;
      }
    } else {
      if (kCount) ++vc.tris;
      if (tri_hit(tris, idx, r, tnear, tfar, t)) {
        if (kAny) return true;
        tfar = t;
        ref = pr;
        hit = true;
      }
    }
  }
  return hit;
}

// Traversal stack: the top kLdsStack entries live in LDS (one column per thread, entry-major so a
// wave's pushes at equal depth hit 64 distinct banks); deeper entries spill to a private array
// (scratch), which only very deep traversals touch.  Scratch-only stacks put a ~500-cycle
// dependent load on every pop.
constexpr int kLdsStack = 12;  // kernels that also stage the scene in LDS
#ifndef SPTR_LDS_STACK_G
#define SPTR_LDS_STACK_G 12
#endif
constexpr int kLdsStackG = SPTR_LDS_STACK_G;  // kernels traversing from L2/HBM (LDS holds only the stack)
template <int N>
struct TravStack {
  uint32_t* lds;  // &s_stack[0][threadIdx.x]
  uint32_t spill[kStack - N];
  __device__ __forceinline__ void put(int i, uint32_t v) {
    if (i < N) lds[i * kBlock] = v;
    else spill[i - N] = v;
  }
  __device__ __forceinline__ uint32_t get(int i) const { return i < N ? lds[i * kBlock] : spill[i - N]; }
};
template <int N>
struct alignas(16) LdsStackN {
  uint32_t e[N][kBlock];
};
using LdsStack = LdsStackN<kLdsStack>;
template <bool kLds>
using KernelStack = LdsStackN<kLds ? kLdsStack : kLdsStackG>;
static_assert(sizeof(LdsStack) % 16 == 0 && sizeof(LdsStackN<kLdsStackG>) % 16 == 0, "keeps the dynamic-LDS base aligned");

// BVH2 stack traversal: nearest child first; leaf children are tested as soon as their box is hit.
// Resumable BVH2 walk (the WideWalk state): up to `steps` node visits; true when the traversal is
// over.  traverse runs it to the end in one go.
template <bool kAny, bool kCount, int N>
__device__ __forceinline__ bool bvh2_walk(uint32_t& cur, int& sp, bool& hit, TravStack<N>& stack, const BvhNode* nodes,
                                          const uint32_t* prim_ref, const float4* tris, const float4* sph, const Ray& r,
                                          float tnear, float& tfar, uint32_t& ref, Visits& vc, int steps) {
  for (int it = 0; it < steps; ++it) {
    const BvhNode* nd = nodes + cur;
    const float4 lxy = nd->lxy, rxy = nd->rxy, z = nd->z;
    const uint4 ln = nd->link;
    if (kCount) ++vc.nodes;
    float tl, tr;
    bool hl = slab(lxy.x, lxy.y, lxy.z, lxy.w, z.x, z.y, r, tnear, tfar, tl);
    bool hr = slab(rxy.x, rxy.y, rxy.z, rxy.w, z.z, z.w, r, tnear, tfar, tr);
    uint32_t L = ln.x, R = ln.y;
    if (hl && (L & kLeafBit)) {
      if (leaf_test<kAny, kCount>(L, prim_ref, tris, sph, r, tnear, tfar, ref, vc)) {
        hit = true;
        if (kAny) return true;
      }
      hl = false;
    }
    if (hr && (R & kLeafBit)) {
      if (leaf_test<kAny, kCount>(R, prim_ref, tris, sph, r, tnear, tfar, ref, vc)) {
        hit = true;
        if (kAny) return true;
      }
      hr = false;
    }
    if (hl && hr) {
      if (tr < tl) {
        const uint32_t s = L;
        L = R;
        R = s;
      }
      if (sp < kStack) stack.put(sp++, R);
      else vc.stack_overflow = 1u;
      cur = L;
    } else if (hl) {
      cur = L;
    } else if (hr) {
      cur = R;
    } else {
      if (sp == 0) return true;
      cur = stack.get(--sp);
    }
  }
  return false;
}
template <bool kAny, bool kCount, int N>
__device__ __forceinline__ bool traverse(const BvhNode* nodes, const uint32_t* prim_ref, const float4* tris,
                                         const float4* sph, uint32_t root, const Ray& r, float tnear, float& tfar,
                                         uint32_t& ref, Visits& vc, LdsStackN<N>& ls) {
  if (root == kNoHit) return false;
  if (root & kLeafBit) return leaf_test<kAny, kCount>(root, prim_ref, tris, sph, r, tnear, tfar, ref, vc);
  TravStack<N> stack;
  stack.lds = &ls.e[0][threadIdx.x];
  int sp = 0;
  uint32_t cur = root;
  bool hit = false;
  (void)bvh2_walk<kAny, kCount>(cur, sp, hit, stack, nodes, prim_ref, tris, sph, r, tnear, tfar, ref, vc, 0x7FFFFFFF);
  return hit;
}

// One axis of a quantised wide node (WideNode) in the ray's frame: the plane org + q * 2^e maps to
// t = q * A + B with A = 2^e * inv (exact) and B = (org - o) * inv.  The fma evaluation errs by at
// most ~2^-22 (|B| + 255 |A|) against (plane - o) * inv; the pad of 2^-20 (|B| + 256 |A|) pushes
// near planes down and far planes up by more than that, so the decoded slab contains the exact
// one.  qn / qf: the plane words that are near / far for this ray direction.
struct QAxis {
  float A, Bn, Bf;
  uint32_t qn[1], qf[1];
};
__device__ __forceinline__ QAxis q_axis(float org, uint32_t ebyte, const uint32_t* qlo, const uint32_t* qhi, float ro,
                                        float inv) {
  QAxis a;
  a.A = __uint_as_float(ebyte << 23) * inv;
  const float B = (org - ro) * inv;
  const float pad = __builtin_fmaf(fabsf(a.A), 256.0f, fabsf(B)) * 0x1p-20f;
  a.Bn = B - pad;
  a.Bf = B + pad;
  const bool pos = inv >= 0.0f;
  a.qn[0] = pos ? qlo[0] : qhi[0];
  a.qf[0] = pos ? qhi[0] : qlo[0];
  return a;
}
__device__ __forceinline__ float q_byte(const uint32_t* w, int k) { return (float)((w[k / 4] >> (8 * (k % 4))) & 0xFFu); }
__device__ __forceinline__ bool q_slab(int k, const QAxis& x, const QAxis& y, const QAxis& z, float tnear, float tfar,
                                       float& tent) {
  const float tnx = __builtin_fmaf(q_byte(x.qn, k), x.A, x.Bn), tfx = __builtin_fmaf(q_byte(x.qf, k), x.A, x.Bf);
  const float tny = __builtin_fmaf(q_byte(y.qn, k), y.A, y.Bn), tfy = __builtin_fmaf(q_byte(y.qf, k), y.A, y.Bf);
  const float tnz = __builtin_fmaf(q_byte(z.qn, k), z.A, z.Bn), tfz = __builtin_fmaf(q_byte(z.qf, k), z.A, z.Bf);
  const float tmin = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, tnear));
  const float tmax = fminf(fminf(tfx, tfy), fminf(tfz, tfar));
  tent = tmin;
  return tmin <= tmax * 1.00000095f;
}

// Wide-BVH traversal: kWide slab tests per quantised node; leaf children are tested as soon as their
// box is hit; the nearest internal child is visited next (lowest slot on ties) and the other hit
// children are pushed, highest slot first.  Written as a resumable walk (WideWalk: the node to
// visit next, the stack depth, whether a hit was found) so that the refilling kernels
// (k_trace_dyn, k_shadow_dyn) can run a ray a few node visits at a time; traverse_wide runs it to
// the end in one go.
struct WideWalk {
  uint32_t cur;
  int sp;
  bool hit;
};
// up to `steps` node visits; true when the traversal is over
// top / ntop: an LDS copy of the wide nodes 0..ntop-1 (the top kTopLevels levels, stage_top), read
// instead of L2/HBM for those indices (ntop = 0: every node from `nodes`).
template <bool kAny, bool kCount, int N>
__device__ __forceinline__ bool wide_walk_inl(WideWalk& wk, TravStack<N>& stack, const WideNode* nodes, const uint4* top,
                                          uint32_t ntop, const uint32_t* prim_ref, const float4* tris, const float4* sph,
                                          const Ray& r, float tnear, float& tfar, uint32_t& ref, Visits& vc, int steps) {
  for (int it = 0; it < steps; ++it) {
    const uint4* nq = reinterpret_cast<const uint4*>(nodes + wk.cur);
    uint4 h, l4, q4;
    uint2 q2;
    if (wk.cur < ntop) {
      const uint4* t = top + 4u * wk.cur;
      h = t[0];
      l4 = t[1];
      q4 = t[2];
      q2 = *reinterpret_cast<const uint2*>(t + 3);
      // pins the LDS loads inside this branch: otherwise the compiler sinks both branches' loads
      // past the join as flat loads of a selected address
      asm volatile("" ::"v"(h.x), "v"(l4.x), "v"(q4.x), "v"(q2.x));
    } else {
      h = nq[0];
      l4 = nq[1];
      q4 = nq[2];
      q2 = *reinterpret_cast<const uint2*>(nq + 3);
    }
    const uint32_t ln[4] = {l4.x, l4.y, l4.z, l4.w};
    const uint32_t qw[6] = {q4.x, q4.y, q4.z, q4.w, q2.x, q2.y};
    if (kCount) ++vc.nodes;
    const QAxis ax = q_axis(__uint_as_float(h.x), h.w & 0xFFu, qw + 0, qw + 1, r.o.x, r.inv.x);
    const QAxis ay = q_axis(__uint_as_float(h.y), (h.w >> 8) & 0xFFu, qw + 2, qw + 3, r.o.y, r.inv.y);
    const QAxis az = q_axis(__uint_as_float(h.z), (h.w >> 16) & 0xFFu, qw + 4, qw + 5, r.o.z, r.inv.z);
    float t[kWide];
    bool hc[kWide];
#pragma unroll
    for (int k = 0; k < kWide; ++k) hc[k] = q_slab(k, ax, ay, az, tnear, tfar, t[k]) && ln[k] != kNoHit;
    // Hit leaf children, in slot order (a direct link's primitive needs no prim_ref load).  r03 A/B:
    // fetching the direct leaves of a node two or four at a time before testing them (one memory
    // latency per batch) spilled at 7 waves/SIMD and read 48 B of the node itself for every non-leaf
    // child slot of the batch: C5 11.7 -> 21.0 / 33.5 ms per step.
#pragma unroll
    for (int k = 0; k < kWide; ++k) {
      if (hc[k] && (ln[k] & kLeafBit)) {
        if (leaf_test<kAny, kCount, true>(ln[k], prim_ref, tris, sph, r, tnear, tfar, ref, vc)) {
          wk.hit = true;
          if (kAny) return true;
        }
        hc[k] = false;
      }
    }
    // next node: the nearest hit internal child; any-hit walks take the farthest (kAnyHitFar)
    int kn = kWide;
    float tn = __builtin_huge_valf();
    uint32_t npush = 0u;
#pragma unroll
    for (int k = 0; k < kWide; ++k) {
      const bool better = (kAny && kAnyHitFar) ? t[k] > tn : t[k] < tn;
      if (hc[k] && (kn == kWide || better)) {
        tn = t[k];
        kn = k;
      }
      npush += hc[k] ? 1u : 0u;
    }
    if (kn < kWide) {
      if (wk.sp + (int)npush - 1 > kStack) vc.stack_overflow = 1u;
#pragma unroll
      for (int k = kWide - 1; k >= 0; --k)
        if (hc[k] && k != kn && wk.sp < kStack) stack.put(wk.sp++, ln[k]);
      wk.cur = ln[kn];
    } else {
      if (wk.sp == 0) return true;
      wk.cur = stack.get(--wk.sp);
    }
  }
  return false;
}
// The same traversal with one fetch per lane per step (the unified walk): a step visits one item,
// an internal node or a leaf.  A node's hit children — leaves included — are ordered like internal
// children (the nearest is visited next, the others pushed), so a leaf's primitive is tested on a
// step of its own.  Every lane issues its step's loads from one selected address (the node's 56 B,
// or a direct leaf's triangle / sphere record; the primitive buffers carry a 64-B tail so that the
// node-sized read stays in bounds) before any lane branches, so a wave waits for one memory latency
// per step, where wide_walk serialises a latency per hit leaf child inside the node's step.  Range
// leaves (leaf size > 1) are tested with leaf_test on their step.  Same hits: the closest hit is the
// minimum over the same set of primitives tested against the same rays (ties at exactly equal t
// may resolve to another primitive, as with any change of traversal order).
// Walk forms: the leaf-inline walk (wide_walk_inl), the unified walk (one item per step) as r04's
// branchy step (walk_fetch + walk_apply) or as the branch-free step (walk_step_bf, r05).  The two
// unified forms visit the same items in the same order (k_strag resumes either's state).
enum : int { kWalkInline = 0, kWalkUnified = 1, kWalkBranchFree = 2 };
// The unified walk of every query except camera rays takes the branch-free step (r05: C5 SALU/VALU of the
// shadow launches 0.65 -> 0.30).  Camera rays (k_trace_dyn<primary>) keep r04's step (r05d
// A/B: C5 bounce-0 trace 1.57-1.59 ms with the branch-free step vs 1.46: coherent waves rarely split, and
// the branch-free step runs both the node and the triangle test).
constexpr int kWalkU = kWalkBranchFree;
constexpr int kWalkPrimary = kWalkUnified;
// the branch-free step reads every node from L2/HBM, so kernels stage the LDS top levels only for the others
__host__ __device__ constexpr bool walk_reads_top(int kind) { return kind != kWalkBranchFree; }
// One step of the unified walk: its fetch (the 56 B of the item wk.cur names: a wide node from the
// LDS top levels or L2/HBM, or a direct leaf's triangle / sphere record) and the step proper.
struct WalkItem {
  uint4 h, l4, q4;
  uint2 q2;
};
__device__ __forceinline__ WalkItem walk_fetch(uint32_t cur, const WideNode* nodes, const uint4* top, uint32_t ntop,
                                               const float4* tris, const float4* sph) {
  const bool leaf = (cur & kLeafBit) != 0u;
  const bool direct = (cur & (kLeafBit | kLeafDirect)) == (kLeafBit | kLeafDirect);
  const bool dsph = direct && (cur & kLeafDirectSphere) != 0u;
  const uint32_t slot = (cur & ~kLeafBit) >> kLeafCountBits;
  const uint4* a = !leaf ? reinterpret_cast<const uint4*>(nodes + cur)
                         : (dsph ? reinterpret_cast<const uint4*>(sph + slot)
                                 : reinterpret_cast<const uint4*>(tris + (direct ? 3u * slot : 0u)));
  WalkItem it;
  if (cur < ntop) {
    const uint4* t = top + 4u * cur;
    it.h = t[0];
    it.l4 = t[1];
    it.q4 = t[2];
    it.q2 = *reinterpret_cast<const uint2*>(t + 3);
    // pins the LDS loads inside this branch: otherwise the compiler sinks both branches' loads past
    // the join as flat loads of a selected address
    asm volatile("" ::"v"(it.h.x), "v"(it.l4.x), "v"(it.q4.x), "v"(it.q2.x));
  } else {
    it.h = a[0];
    it.l4 = a[1];
    it.q4 = a[2];
    it.q2 = *reinterpret_cast<const uint2*>(a + 3);
  }
  return it;
}
// the step on the fetched item; true when the traversal is over
template <bool kAny, bool kCount, int N>
__device__ __forceinline__ bool walk_apply(WideWalk& wk, TravStack<N>& stack, const WalkItem& it, const uint32_t* prim_ref,
                                           const float4* tris, const float4* sph, const Ray& r, float tnear, float& tfar,
                                           uint32_t& ref, Visits& vc) {
  const uint32_t cur = wk.cur;
  const bool leaf = (cur & kLeafBit) != 0u;
  const bool direct = (cur & (kLeafBit | kLeafDirect)) == (kLeafBit | kLeafDirect);
  const bool dsph = direct && (cur & kLeafDirectSphere) != 0u;
  const uint32_t slot = (cur & ~kLeafBit) >> kLeafCountBits;
  if (leaf) {
    bool hit = false;
    if (direct) {
      const float4 p0 = make_float4(__uint_as_float(it.h.x), __uint_as_float(it.h.y), __uint_as_float(it.h.z), __uint_as_float(it.h.w));
      float t;
      if (dsph) {
        if (kCount) ++vc.sph;
        if (kAny) hit = sphere_occ(p0, r, tnear, tfar);
        else if (sphere_hit(p0, r, tnear, tfar, t)) {
          tfar = t;
          ref = slot | kSphereBit;
          hit = true;
        }
      } else {
        if (kCount) ++vc.tris;
        const float4 p1 = make_float4(__uint_as_float(it.l4.x), __uint_as_float(it.l4.y), __uint_as_float(it.l4.z), __uint_as_float(it.l4.w));
        const float4 p2 = make_float4(__uint_as_float(it.q4.x), __uint_as_float(it.q4.y), __uint_as_float(it.q4.z), __uint_as_float(it.q4.w));
        if (tri_hit4(p0, p1, p2, r, tnear, tfar, t)) {
          if (!kAny) {
            tfar = t;
            ref = slot;
          }
          hit = true;
        }
      }
    } else {
      hit = leaf_test<kAny, kCount>(cur, prim_ref, tris, sph, r, tnear, tfar, ref, vc);
    }
    if (hit) {
      wk.hit = true;
      if (kAny) return true;
    }
    if (wk.sp == 0) return true;
    wk.cur = stack.get(--wk.sp);
    return false;
  }
  const uint32_t ln[4] = {it.l4.x, it.l4.y, it.l4.z, it.l4.w};
  const uint32_t qw[6] = {it.q4.x, it.q4.y, it.q4.z, it.q4.w, it.q2.x, it.q2.y};
  if (kCount) ++vc.nodes;
  const QAxis ax = q_axis(__uint_as_float(it.h.x), it.h.w & 0xFFu, qw + 0, qw + 1, r.o.x, r.inv.x);
  const QAxis ay = q_axis(__uint_as_float(it.h.y), (it.h.w >> 8) & 0xFFu, qw + 2, qw + 3, r.o.y, r.inv.y);
  const QAxis az = q_axis(__uint_as_float(it.h.z), (it.h.w >> 16) & 0xFFu, qw + 4, qw + 5, r.o.z, r.inv.z);
  float t[4];
  bool hc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) hc[k] = q_slab(k, ax, ay, az, tnear, tfar, t[k]) && ln[k] != kNoHit;
  int kn = 4;
  float tn = __builtin_huge_valf();
  uint32_t npush = 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool better = (kAny && kAnyHitFar) ? t[k] > tn : t[k] < tn;
    if (hc[k] && (kn == 4 || better)) {
      tn = t[k];
      kn = k;
    }
    npush += hc[k] ? 1u : 0u;
  }
  if (kn < 4) {
    if (wk.sp + (int)npush - 1 > kStack) vc.stack_overflow = 1u;
#pragma unroll
    for (int k = 3; k >= 0; --k)
      if (hc[k] && k != kn && wk.sp < kStack) stack.put(wk.sp++, ln[k]);
    wk.cur = ln[kn];
    return false;
  }
  if (wk.sp == 0) return true;
  wk.cur = stack.get(--wk.sp);
  return false;
}
template <bool kAny, bool kCount, int N>
__device__ __forceinline__ bool wide_walk_u(WideWalk& wk, TravStack<N>& stack, const WideNode* nodes, const uint4* top,
                                            uint32_t ntop, const uint32_t* prim_ref, const float4* tris, const float4* sph,
                                            const Ray& r, float tnear, float& tfar, uint32_t& ref, Visits& vc, int steps) {
  static_assert(kWide == 4, "unified walk: 4-wide nodes");
  for (int it = 0; it < steps; ++it) {
    const WalkItem item = walk_fetch(wk.cur, nodes, top, ntop, tris, sph);
    if (walk_apply<kAny, kCount>(wk, stack, item, prim_ref, tris, sph, r, tnear, tfar, ref, vc)) return true;
  }
  return false;
}

// The unified step without divergent branches (r05).  r04's step (walk_fetch + walk_apply) split the
// wave at every per-lane decision — leaf or node, top-LDS or global fetch, sphere or triangle, each
// push into the LDS part or the scratch part of the stack, pop or descend — and every split costs
// exec-mask bookkeeping (s_and_saveexec / s_xor / s_cbranch_execz / s_or: 430 of k_shadow_dyn's 882
// SALU).  Here every lane runs one instruction stream per step:
//   * one 64-B fetch from a selected address (node, direct triangle or sphere record; the top levels
//     are read from L2 like the rest — the LDS copy measured within noise on C5, r02g);
//   * the four quantised slab tests and the triangle test both evaluated, their results selected by
//     the item's kind (the division of a triangle hit runs only in lanes that hit);
//   * the child order by selects; the pushes as unconditional LDS writes at the running push
//     position (a slot that is not a push is overwritten by the next push or lies above the new
//     stack top), while the stack top stays below the LDS part (sp + 3 < N); a lane that may cross
//     into the scratch part takes the branchy put of the r04 step;
//   * the pop as an LDS read of row min(sp - 1, N - 1), replaced from scratch only below the LDS part.
// Spheres and range leaves (leaf size > 1: LDS-staged scenes in BVH4 test mode) keep a branch: they
// are rare or absent in the scenes this walk serves.  Same node order, same tests, same hits as the r04
// step (k_strag resumes either's state).
template <bool kAny, bool kCount, int N>
__device__ __forceinline__ bool walk_step_bf(WideWalk& wk, TravStack<N>& stack, const WideNode* nodes,
                                             const uint32_t* prim_ref, const float4* tris, const float4* sph,
                                             const Ray& r, float tnear, float& tfar, uint32_t& ref, Visits& vc) {
  const uint32_t cur = wk.cur;
  const int sp = wk.sp;
  const bool leaf = (cur & kLeafBit) != 0u;
  const bool direct = (cur & (kLeafBit | kLeafDirect)) == (kLeafBit | kLeafDirect);
  const bool dsph = direct && (cur & kLeafDirectSphere) != 0u;
  const uint32_t slot = (cur & ~kLeafBit) >> kLeafCountBits;
  // pointer arithmetic on the kernel's global pointers (an address computed through an integer would
  // lose their address space, and the fetch would become flat loads, which also wait on the LDS counter)
  const uint4* an = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(nodes) + (size_t)cur * sizeof(WideNode));
  const uint4* ap = dsph ? reinterpret_cast<const uint4*>(sph + slot) : reinterpret_cast<const uint4*>(tris + 3u * (direct ? slot : 0u));
  const uint4* a = leaf ? ap : an;
  const uint4 h = a[0], l4 = a[1], q4 = a[2];
  const uint2 q2 = *reinterpret_cast<const uint2*>(a + 3);
  // the pop candidate: row min(sp - 1, N - 1) of the LDS part (an LDS read by address space, and pinned:
  // otherwise the compiler selects between the LDS and the scratch address and issues a flat load),
  // replaced from scratch below the LDS part
  const int ps = sp > 0 ? sp - 1 : 0;
  uint32_t popv = *(const __attribute__((address_space(3))) uint32_t*)(stack.lds + (ps < N ? ps : N - 1) * kBlock);
  asm volatile("" : "+v"(popv));
  if (ps >= N) popv = stack.spill[ps - N];
  // node: quantised slab tests of the four children
  const uint32_t ln[4] = {l4.x, l4.y, l4.z, l4.w};
  const uint32_t qw[6] = {q4.x, q4.y, q4.z, q4.w, q2.x, q2.y};
  const QAxis ax = q_axis(__uint_as_float(h.x), h.w & 0xFFu, qw + 0, qw + 1, r.o.x, r.inv.x);
  const QAxis ay = q_axis(__uint_as_float(h.y), (h.w >> 8) & 0xFFu, qw + 2, qw + 3, r.o.y, r.inv.y);
  const QAxis az = q_axis(__uint_as_float(h.z), (h.w >> 16) & 0xFFu, qw + 4, qw + 5, r.o.z, r.inv.z);
  float t[4];
  bool hc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) hc[k] = q_slab(k, ax, ay, az, tnear, tfar, t[k]) & (ln[k] != kNoHit) & !leaf;
  // leaf: a direct triangle (Embree's test, tri_hit4, with the division deferred to the lanes that hit)
  bool lhit = false;
  {
    const float4 p0 = make_float4(__uint_as_float(h.x), __uint_as_float(h.y), __uint_as_float(h.z), __uint_as_float(h.w));
    const float4 p1 = make_float4(__uint_as_float(l4.x), __uint_as_float(l4.y), __uint_as_float(l4.z), __uint_as_float(l4.w));
    const float4 p2 = make_float4(__uint_as_float(q4.x), __uint_as_float(q4.y), __uint_as_float(q4.z), __uint_as_float(q4.w));
    const vec3 v0 = v3(p0.x, p0.y, p0.z), e1 = v3(p0.w, p1.x, p1.y), e2 = v3(p1.z, p1.w, p2.x), ng = v3(p2.y, p2.z, p2.w);
    const vec3 C = v0 - r.o;
    const vec3 R = e_cross(C, r.d);
    const float den = e_dot(ng, r.d);
    const float aden = fabsf(den);
    const float U = xorsign(e_dot(R, e2), den);
    const float V = xorsign(e_dot(R, e1), den);
    const float T = xorsign(e_dot(ng, C), den);
    const bool tri = direct && !dsph;
    const bool inside = (den != 0.0f) & (U >= 0.0f) & (V >= 0.0f) & (U + V <= aden);
    const bool range = (aden * tnear < T) & (T <= aden * tfar);
    lhit = tri & inside & range;
    if (kCount) vc.tris += tri ? 1u : 0u;
    if (!kAny && lhit) {
      tfar = T / aden;
      ref = slot;
    }
  }
  if (dsph) {  // a direct sphere (rare: the reference's analytic spheres)
    if (kCount) ++vc.sph;
    const float4 p0 = make_float4(__uint_as_float(h.x), __uint_as_float(h.y), __uint_as_float(h.z), __uint_as_float(h.w));
    float ts;
    if (kAny) lhit = sphere_occ(p0, r, tnear, tfar);
    else if (sphere_hit(p0, r, tnear, tfar, ts)) {
      tfar = ts;
      ref = slot | kSphereBit;
      lhit = true;
    }
  }
  if (leaf && !direct) lhit = leaf_test<kAny, kCount>(cur, prim_ref, tris, sph, r, tnear, tfar, ref, vc);  // range leaf
  if (kCount) vc.nodes += leaf ? 0u : 1u;
  // child order: the nearest hit child next (far-first for any-hit, kAnyHitFar), lowest slot on ties
  int kn = 4;
  float tn = __builtin_huge_valf();
  uint32_t nxt = 0u, nh = 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool better = (kAny && kAnyHitFar) ? t[k] > tn : t[k] < tn;
    const bool take = hc[k] & ((kn == 4) | better);
    tn = take ? t[k] : tn;
    kn = take ? k : kn;
    nxt = take ? ln[k] : nxt;
    nh += hc[k] ? 1u : 0u;
  }
  const bool descend = kn < 4;
  // pushes: the other hit children, highest slot first
  if (sp + 3 < N) {
    int pos = sp;
#pragma unroll
    for (int k = 3; k >= 0; --k) {
      stack.lds[pos * kBlock] = ln[k];
      pos += (hc[k] & (k != kn)) ? 1 : 0;
    }
  } else {
    if (sp + (int)nh - 1 > kStack) vc.stack_overflow = 1u;
    int pos = sp;
#pragma unroll
    for (int k = 3; k >= 0; --k)
      if (hc[k] && k != kn && pos < kStack) stack.put(pos++, ln[k]);
  }
  const int spd = sp + (int)nh - 1;
  wk.hit = wk.hit | lhit;
  wk.cur = descend ? nxt : popv;
  wk.sp = descend ? (spd < kStack ? spd : kStack) : ps;
  return (kAny && lhit) || (!descend && sp == 0);
}
template <bool kAny, bool kCount, int N>
__device__ __forceinline__ bool wide_walk_bf(WideWalk& wk, TravStack<N>& stack, const WideNode* nodes,
                                             const uint32_t* prim_ref, const float4* tris, const float4* sph,
                                             const Ray& r, float tnear, float& tfar, uint32_t& ref, Visits& vc, int steps) {
  for (int it = 0; it < steps; ++it)
    if (walk_step_bf<kAny, kCount>(wk, stack, nodes, prim_ref, tris, sph, r, tnear, tfar, ref, vc)) return true;
  return false;
}
// kKind: the walk form (kWalk*); callers choose per ray class (see the kernels)
template <bool kAny, bool kCount, int kKind = kWalkU, int N>
__device__ __forceinline__ bool wide_walk(WideWalk& wk, TravStack<N>& stack, const WideNode* nodes, const uint4* top,
                                          uint32_t ntop, const uint32_t* prim_ref, const float4* tris, const float4* sph,
                                          const Ray& r, float tnear, float& tfar, uint32_t& ref, Visits& vc, int steps) {
  if constexpr (kKind == kWalkBranchFree)
    return wide_walk_bf<kAny, kCount>(wk, stack, nodes, prim_ref, tris, sph, r, tnear, tfar, ref, vc, steps);
  else if constexpr (kKind == kWalkUnified)
    return wide_walk_u<kAny, kCount>(wk, stack, nodes, top, ntop, prim_ref, tris, sph, r, tnear, tfar, ref, vc, steps);
  else
    return wide_walk_inl<kAny, kCount>(wk, stack, nodes, top, ntop, prim_ref, tris, sph, r, tnear, tfar, ref, vc, steps);
}
// Starts a walk at root; true when it is already over (empty scene, or a root leaf tested here).
template <bool kAny, bool kCount>
__device__ __forceinline__ bool wide_start(WideWalk& wk, uint32_t root, const uint32_t* prim_ref, const float4* tris,
                                           const float4* sph, const Ray& r, float tnear, float& tfar, uint32_t& ref,
                                           Visits& vc) {
  wk.cur = root;
  wk.sp = 0;
  wk.hit = false;
  if (root == kNoHit) return true;
  if (root & kLeafBit) {
    wk.hit = leaf_test<kAny, kCount>(root, prim_ref, tris, sph, r, tnear, tfar, ref, vc);
    return true;
  }
  return false;
}
template <bool kAny, bool kCount, int N>
__device__ __forceinline__ bool traverse_wide(const WideNode* nodes, const uint32_t* prim_ref, const float4* tris,
                                              const float4* sph, uint32_t root, const Ray& r, float tnear, float& tfar,
                                              uint32_t& ref, Visits& vc, LdsStackN<N>& ls) {
  WideWalk wk;
  if (wide_start<kAny, kCount>(wk, root, prim_ref, tris, sph, r, tnear, tfar, ref, vc)) return wk.hit;
  TravStack<N> stack;
  stack.lds = &ls.e[0][threadIdx.x];
  (void)wide_walk<kAny, kCount>(wk, stack, nodes, nullptr, 0u, prim_ref, tris, sph, r, tnear, tfar, ref, vc, 0x7FFFFFFF);
  return wk.hit;
}

// Stage the whole scene (nodes, triangles, spheres) into LDS when it fits (SceneView::lds_bytes).
struct Staged {
  const BvhNode* nodes;
  const WideNode* nodes4;
  const uint32_t* prim_ref;
  const float4* tris;
  const float4* sph;
};
template <bool kLds>
__device__ __forceinline__ Staged stage_scene(const SceneView& sv, float4* lds) {
  Staged s{sv.nodes, sv.nodes4, sv.prim_ref, sv.tris, sv.sph};
  if (kLds) {
    const bool w4 = sv.width == (uint32_t)kWide;
    const uint32_t nn = (w4 ? sv.num_nodes4 * (uint32_t)sizeof(WideNode) : sv.num_nodes * (uint32_t)sizeof(BvhNode)) / 16u,
                   nt = sv.num_tris * 3u, ns = sv.num_sph;
    const uint32_t np = (sv.num_tris + sv.num_sph + 3u) / 4u;  // prim refs, in float4 units
    const float4* gn = w4 ? reinterpret_cast<const float4*>(sv.nodes4) : reinterpret_cast<const float4*>(sv.nodes);
    const float4* gp = reinterpret_cast<const float4*>(sv.prim_ref);
    for (uint32_t i = threadIdx.x; i < nn; i += blockDim.x) lds[i] = gn[i];
    for (uint32_t i = threadIdx.x; i < nt; i += blockDim.x) lds[nn + i] = sv.tris[i];
    for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) lds[nn + nt + i] = sv.sph[i];
    for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) lds[nn + nt + ns + i] = gp[i];
    __syncthreads();
    s.nodes = reinterpret_cast<const BvhNode*>(lds);
    s.nodes4 = reinterpret_cast<const WideNode*>(lds);
    s.tris = lds + nn;
    s.sph = lds + nn + nt;
    s.prim_ref = reinterpret_cast<const uint32_t*>(lds + nn + nt + ns);
  }
  return s;
}

// Copy the wide BVH's top levels (nodes 0..num_top4-1, SceneView::num_top4) to LDS at dst; the
// caller's next block barrier (seg_scan's, or its own) publishes them.  Kernels traversing the wide
// BVH from L2/HBM read these first node visits of every ray from LDS (wide_walk).
__device__ __forceinline__ const uint4* stage_top(const SceneView& sv, float4* dst) {
  const uint32_t n = sv.num_top4 * (uint32_t)(sizeof(WideNode) / 16);
  const uint4* g = reinterpret_cast<const uint4*>(sv.nodes4);
  uint4* d = reinterpret_cast<uint4*>(dst);
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) d[i] = g[i];
  return d;
}
// float4 offset of the top-level copy in a kernel's dynamic LDS: after the staged scene (kLds) or
// after the segment offsets s_off[0..nseg] of a consumer (!kPrimary)
__device__ __forceinline__ uint32_t top_lds_offset(const SceneView& sv, bool lds, bool primary, uint32_t nseg) {
  return (lds ? sv.lds_bytes / 16u : 0u) + (primary ? 0u : (4u * (nseg + 1u) + 15u) / 16u);
}

template <bool kW4, bool kAny, bool kCount, int N>
__device__ __forceinline__ bool traverse_w(const Staged& sc, const SceneView& sv, const Ray& r, float tnear, float& tfar,
                                           uint32_t& ref, Visits& vc, LdsStackN<N>& ls) {
  if (kW4) return traverse_wide<kAny, kCount>(sc.nodes4, sc.prim_ref, sc.tris, sc.sph, sv.root4, r, tnear, tfar, ref, vc, ls);
  return traverse<kAny, kCount>(sc.nodes, sc.prim_ref, sc.tris, sc.sph, sv.root, r, tnear, tfar, ref, vc, ls);
}

// traverse_w with the wide BVH's top levels read from an LDS copy (stage_top; ntop = 0: none) — the
// path-per-thread kernels of L2/HBM scenes (k_tail, k_strag), whose every ray starts at the root
template <bool kW4, bool kAny, bool kCount, int N>
__device__ __forceinline__ bool traverse_w_top(const Staged& sc, const SceneView& sv, const uint4* top, uint32_t ntop,
                                               const Ray& r, float tnear, float& tfar, uint32_t& ref, Visits& vc,
                                               LdsStackN<N>& ls) {
  if constexpr (kW4) {
    WideWalk wk;
    if (wide_start<kAny, kCount>(wk, sv.root4, sc.prim_ref, sc.tris, sc.sph, r, tnear, tfar, ref, vc)) return wk.hit;
    TravStack<N> stack;
    stack.lds = &ls.e[0][threadIdx.x];
    (void)wide_walk<kAny, kCount>(wk, stack, sc.nodes4, top, ntop, sc.prim_ref, sc.tris, sc.sph, r, tnear, tfar, ref, vc,
                                  0x7FFFFFFF);
    return wk.hit;
  }
  return traverse<kAny, kCount>(sc.nodes, sc.prim_ref, sc.tris, sc.sph, sv.root, r, tnear, tfar, ref, vc, ls);
}

// Per-bounce and per-ray statistics (sptr_stats traced_by_depth / nodes_by_depth / *_visit_hist).
__device__ __forceinline__ uint32_t stat_depth(int depth) { return depth < kStatDepths - 1 ? (uint32_t)depth : kStatDepths - 1u; }
// The instrumented pass bins every ray's node visits into a block-local LDS histogram (s_hist, zeroed
// before the kernel's first barrier), flushed with one global add per bin per block at its end.
__device__ __forceinline__ void hist_ray(uint32_t* s_hist, uint32_t visits) {
  const uint32_t b = visits ? (uint32_t)(32 - __clz(visits)) : 0u;
  atomicAdd(&s_hist[b < (uint32_t)kHistBins ? b : kHistBins - 1u], 1u);
}
__device__ __forceinline__ void hist_init(uint32_t* s_hist) {
  if (threadIdx.x < (uint32_t)kHistBins) s_hist[threadIdx.x] = 0u;
}
// call from every thread of the block (barrier)
__device__ __forceinline__ void hist_flush(const uint32_t* s_hist, unsigned long long* tot, int base) {
  __syncthreads();
  if (threadIdx.x < (uint32_t)kHistBins && s_hist[threadIdx.x]) atomicAdd(&tot[base + threadIdx.x], (unsigned long long)s_hist[threadIdx.x]);
}
__device__ __forceinline__ void flush_depth_nodes(const Visits& vc, unsigned long long* tot, int depth) {
  unsigned long long a = vc.nodes;
  for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off);
  if (lane_id() == 0) atomicAdd(&tot[kTotNodesD + stat_depth(depth)], a);
}

// Sticky stack-overflow report (one store per wave that saw a dropped push).
__device__ __forceinline__ void report_stack(const Visits& vc, unsigned long long* tot) {
  if (__ballot(vc.stack_overflow != 0u) && lane_id() == 0u) tot[kTotStackOverflow] = 1ull;
}

__device__ __forceinline__ void flush_visits(const Visits& vc, unsigned long long* tot, int base) {
  unsigned long long a = vc.nodes, b = vc.tris, c = vc.sph;
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off);
    b += __shfl_xor(b, off);
    c += __shfl_xor(c, off);
  }
  if (lane_id() == 0) {
    atomicAdd(&tot[base + 0], a);
    atomicAdd(&tot[base + 1], b);
    if (base == kTotNodes || base == kTotNodesP || base == kTotStragNodes) atomicAdd(&tot[base + 2], c);
  }
}

// --------------------------------------------------------------------------------- path init
// GLRenderer::renderWavefrontTileTask seeding + WavefrontPathTracerCPU::traceRay's first rng, for
// path p = sample_slot * P + local pixel.  Returns false for tile slots outside the image.
struct Primary {
  vec3 d;
  uint32_t rng;
};
// dW, dH: the image width and height as loop-invariant divisors (cr_math.h; (x + jx) / W stays
// correctly rounded, with the divisor's reciprocal refined once per thread instead of per path).
struct ImageDiv {
  DivBy w, h;
};
__device__ __forceinline__ ImageDiv image_div(const FrameView& f) { return ImageDiv{div_by(float(f.W)), div_by(float(f.H))}; }
// pixel (x, y) with pixel_seed ps = y*W + x, accumulation index acc
__device__ __forceinline__ void primary_at(const FrameView& f, const ImageDiv& dv, int x, int y, uint32_t ps,
                                           uint32_t acc, Primary& out) {
  uint32_t r = wang_hash(ps ^ acc * 9781u);
  const float jx = rand01(r);
  const float jy = rand01(r);
  const vec3 dir = camera_dir(f, div_nrm(float(x) + jx, dv.w), div_nrm(float(y) + jy, dv.h));
  out.d = renormalized_again(dir);  // dir: camera_dir normalized it
  out.rng = wang_hash((ps ^ acc) ^ 1u);
}
__device__ __forceinline__ bool primary_path(const FrameView& f, const ImageDiv& dv, uint32_t p, Primary& out,
                                             uint32_t& l) {
  const uint32_t s = fast_div(f.div_P, p);
  l = p - s * f.P;
  int x, y;
  if (!local_pixel(f, l, x, y)) return false;
  primary_at(f, dv, x, y, (uint32_t)(y * f.W + x), f.acc0 + s, out);
  return true;
}
__device__ __forceinline__ bool primary_path(const FrameView& f, const ImageDiv& dv, uint32_t p, Primary& out) {
  uint32_t l;
  return primary_path(f, dv, p, out, l);
}

// --------------------------------------------------------------------------------- pixel culling
// Bounce-0 pixel-frustum culling.  All camera rays of local pixel (x, y) — any jitter — start at the
// camera and run inside the pyramid spanned by the pixel's corner directions (Camera::getRayDirection
// at u in [x, x+1] / W, v in [y, y+1] / H).  When that pyramid, widened by kCullMarginPx pixels, lies
// outside every box of the BVH's top kCullDepth levels, no such ray can hit any primitive, and bounce 0
// skips their traversal: it would return no hit.  The test is a separating-plane test against the
// pyramid's four side planes (the box's corner farthest along each inward normal), with a relative
// margin of kCullSlack on the plane distance.  Both margins are orders of magnitude above the
// rounding of the per-sample ray directions (~1e-6 relative, vs 1/64 pixel = 7.5e-6 rad at 4K) and of
// this test itself, so a pixel is culled only when its rays certainly miss.
constexpr float kCullMarginPx = 1.0f / 64.0f;
constexpr float kCullSlack = 1e-4f;
// BVH2 levels below the root whose boxes the test visits (FrameView::cull_depth, chosen per call by
// cull_depth_for): r02 A/B, 2 -> 4 levels: C2 primary trace 1.12 -> 1.09 ms; 4 -> 8 (r02i): C5
// primary trace 3.11 -> 2.87 ms, C2/C3 unchanged (profiles/r02i_ab_cull_depth.txt).  The mask is
// recomputed whenever the camera moves, so calls of few samples per pixel (the interactive 1 spp
// per frame) keep the cheaper 4-level test.
constexpr int kCullDepthMax = 8;
struct Box {
  vec3 lo, hi;
};
__device__ __forceinline__ bool box_outside(const Box& b, const vec3 n[4], vec3 o) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const vec3 p = v3(n[k].x >= 0.0f ? b.hi.x : b.lo.x, n[k].y >= 0.0f ? b.hi.y : b.lo.y,
                      n[k].z >= 0.0f ? b.hi.z : b.lo.z);
    const vec3 q = p - o;
    const float d = n[k].x * q.x + n[k].y * q.y + n[k].z * q.z;
    const float mag = fabsf(n[k].x * q.x) + fabsf(n[k].y * q.y) + fabsf(n[k].z * q.z);
    if (d < -kCullSlack * mag) return true;
  }
  return false;
}
// The pyramid of the pixel rectangle [x, x + npx) x [y, y + npx) (k_cull tests 2x2 pixel quads: a quad
// whose pyramid misses every box culls its four pixels, a subset of what per-pixel pyramids would
// cull, at a quarter of the tests).
__device__ __forceinline__ bool pixel_frustum_misses(const SceneView& sv, const FrameView& f, int x, int y, int npx = 1) {
  if (sv.num_nodes == 0u || (sv.root & kLeafBit)) return false;
  const float u0 = (float(x) - kCullMarginPx) / float(f.W), u1 = (float(x + npx) + kCullMarginPx) / float(f.W);
  const float v0 = (float(y) - kCullMarginPx) / float(f.H), v1 = (float(y + npx) + kCullMarginPx) / float(f.H);
  auto dir = [&](float u, float v) {
    return f.cam_f + ((u - 0.5f) * 2.0f * f.half_w) * f.cam_r + (-(v - 0.5f) * 2.0f * f.half_h) * f.cam_u;
  };
  const vec3 c[4] = {dir(u0, v0), dir(u1, v0), dir(u1, v1), dir(u0, v1)};
  vec3 n[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    n[k] = cross(c[k], c[(k + 1) & 3]);
    if (dot(n[k], c[(k + 2) & 3]) < 0.0f) n[k] = -n[k];  // inward
  }
  // the BVH2's top kCullDepth levels, depth first: a box outside the pyramid prunes its subtree;
  // a box that may intersect it at the cut depth (or a leaf's box) means the pixel is not culled
  struct Entry {
    uint32_t link, depth;
    Box b;
  };
  Entry st[2 * kCullDepthMax + 2];
  int sp = 0;
  {
    const BvhNode r = sv.nodes[0];
    st[sp++] = Entry{r.link.y, 1u, Box{v3(r.rxy.x, r.rxy.z, r.z.z), v3(r.rxy.y, r.rxy.w, r.z.w)}};
    st[sp++] = Entry{r.link.x, 1u, Box{v3(r.lxy.x, r.lxy.z, r.z.x), v3(r.lxy.y, r.lxy.w, r.z.y)}};
  }
  while (sp > 0) {
    const Entry e = st[--sp];
    if (box_outside(e.b, n, f.cam_pos)) continue;
    if ((e.link & kLeafBit) || e.depth >= f.cull_depth) return false;
    const BvhNode g = sv.nodes[e.link];
    st[sp++] = Entry{g.link.y, e.depth + 1u, Box{v3(g.rxy.x, g.rxy.z, g.z.z), v3(g.rxy.y, g.rxy.w, g.z.w)}};
    st[sp++] = Entry{g.link.x, e.depth + 1u, Box{v3(g.lxy.x, g.lxy.z, g.z.x), v3(g.lxy.y, g.lxy.w, g.z.y)}};
  }
  return true;
}
// bit l of mask: pixel l is culled (see above).  plist: the valid pixels that are not culled, from
// plist[0] (count at plist[P], zeroed before).  One block per local tile: thread (qx, qy) tests the 2x2
// pixel quad at (2qx, 2qy) of the tile and sets the quad's bits in the tile's 32 LDS row words; then
// each thread lists the pixels of 4 consecutive local indices, the tile's run at a range one atomic per
// tile reserves.  (r02: a pyramid per pixel and one atomic per wave, C2 108 us; per pixel and per tile
// 65-75 us.)
__global__ void __launch_bounds__(kBlock) k_cull(SceneView sv, FrameView f, uint32_t* mask, uint32_t* plist) {
  static_assert(kTile == 32 && kBlock == 256, "16 x 16 quads per 32 x 32 tile");
  __shared__ uint32_t s_row[kTile];
  __shared__ uint32_t s_cnt[kBlock / 64u];
  __shared__ uint32_t s_base;
  const uint32_t t0 = blockIdx.x * kTilePixels;  // the tile's first local pixel
  if (threadIdx.x < (uint32_t)kTile) s_row[threadIdx.x] = 0u;
  __syncthreads();
  {
    const uint32_t qx = threadIdx.x & 15u, qy = threadIdx.x >> 4;
    int x = 0, y = 0;
    (void)local_pixel(f, t0 + 2u * qy * kTile + 2u * qx, x, y);  // the quad's corner (in or out of the image)
    if (x < f.W && y < f.H && pixel_frustum_misses(sv, f, x, y, 2)) {
      atomicOr(&s_row[2u * qy], 3u << (2u * qx));
      atomicOr(&s_row[2u * qy + 1u], 3u << (2u * qx));
    }
  }
  __syncthreads();
  // four consecutive local pixels per thread: l = t0 + 4 * tid + j (row tid / 8, columns 4 * (tid % 8) + j)
  const uint32_t row = threadIdx.x >> 3, col = (threadIdx.x & 7u) * 4u;
  const uint32_t bits = (s_row[row] >> col) & 0xFu;
  uint32_t keep = 0u;
#pragma unroll
  for (uint32_t j = 0; j < 4u; ++j) {
    int x, y;
    if (local_pixel(f, t0 + 4u * threadIdx.x + j, x, y) && !((bits >> j) & 1u)) keep |= 1u << j;
  }
  // mask bits of invalid pixels stay 0 (the trace kernels skip them by their own test)
  const uint32_t valid_bits = [&] {
    uint32_t v = 0u;
#pragma unroll
    for (uint32_t j = 0; j < 4u; ++j) {
      int x, y;
      if (local_pixel(f, t0 + 4u * threadIdx.x + j, x, y)) v |= 1u << j;
    }
    return v;
  }();
  const uint32_t mbits = bits & valid_bits;
  // mask word (32 pixels) = the nibbles of 8 consecutive threads
  uint32_t w = mbits << col;
  for (int off = 1; off < 8; off <<= 1) w |= __shfl_xor(w, off);
  if ((threadIdx.x & 7u) == 0u) mask[(t0 >> 5) + row] = w;
  // list the kept pixels: per-thread counts, wave scans, block offsets, one atomic per tile
  const uint32_t n = (uint32_t)__popc(keep), lane = lane_id();
  uint32_t incl = n;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t v = __shfl_up(incl, off);
    if (lane >= (uint32_t)off) incl += v;
  }
  if (lane == 63u) s_cnt[threadIdx.x >> 6] = incl;
  __syncthreads();
  if (threadIdx.x == 0u) {
    uint32_t run = 0u;
    for (uint32_t i = 0; i < kBlock / 64u; ++i) {
      const uint32_t c = s_cnt[i];
      s_cnt[i] = run;
      run += c;
    }
    s_base = run ? atomicAdd(&plist[f.P], run) : 0u;
  }
  __syncthreads();
  uint32_t o = s_base + s_cnt[threadIdx.x >> 6] + incl - n;
#pragma unroll
  for (uint32_t j = 0; j < 4u; ++j)
    if ((keep >> j) & 1u) plist[o++] = t0 + 4u * threadIdx.x + j;
}
// Path-major bounce 0 over the unculled pixel list (f.plist: nlist pixels x k samples): compacted
// item i -> path p.  Items run in groups of kPrimaryGroup listed pixels — neighbours, since k_cull lists
// each tile's unculled pixels in pixel order — times all k samples, sample-major inside a group.  The
// k samples of a pixel take near-identical paths down the BVH (they differ by the sub-pixel jitter),
// so a group's rays reuse one small set of nodes and primitives while it is in flight, on one XCD
// (consecutive chunks go to consecutive logical blocks).  With the whole list as one group (sample
// layer after sample layer over the frame) a scene larger than the MALL is streamed from HBM once per
// sample.  The order changes no result: every path is traced and shaded independently and k_accum
// sums in sample order.  SPTR_PRIMARY_GROUP=0: one group (the order before r03).
#ifndef SPTR_PRIMARY_GROUP
#define SPTR_PRIMARY_GROUP 64
#endif
__device__ __forceinline__ uint32_t primary_item(const FrameView& f, uint32_t nlist, uint32_t i) {
  const uint32_t grp = SPTR_PRIMARY_GROUP ? (uint32_t)SPTR_PRIMARY_GROUP : nlist;
  const uint32_t gk = grp * f.k;
  const uint32_t g = i / gk, r = i - g * gk;
  const uint32_t first = g * grp;
  const uint32_t gs = min(grp, nlist - first);
  const uint32_t smp = r / gs;
  return smp * f.P + f.plist[first + (r - smp * gs)];
}
// Camera rays a bounce-0 trace kernel traverses: the k samples of every valid pixel that k_cull did
// not cull (the culled ones are answered without a traversal).  Reported as traced_primary.
__device__ __forceinline__ unsigned long long primary_traced(const FrameView& f) {
  return (unsigned long long)(f.unculled ? *f.unculled : f.valid) * f.k;
}
__device__ __forceinline__ bool pixel_culled(const FrameView& f, uint32_t l) {
  return f.cull != nullptr && ((f.cull[l >> 5] >> (l & 31u)) & 1u) != 0u;
}

// --------------------------------------------------------------------------------- shading math
// The two library calls of the wavefront path whose last bit may differ from glibc's (the CPU
// reference links glibc; this is ocml): the cosine sample's sin / cos of phi = 2 pi r1
// (wf_math.h:51-72; r1 takes the 2^24 values k / 2^24) and the resolve's pow(c, 1/2.2)
// (GLRenderer.cpp:416-430).  One definition each, shared by the kernels and by k_eval_math, which
// tabulates them for the parity tests' residue classifier (tests/test_gpu_configs.py).
__device__ __forceinline__ void cosine_sincos(float r1, float& s, float& c) {
  const float phi = 2.0f * 3.14159265358979323846264338327950288f * r1;
  s = sinf(phi);
  c = cosf(phi);
}
__device__ __forceinline__ float gamma_pow(float x) { return powf(x, 1.0f / 2.2f); }

// Integer powers of x in [0,1] (the reference's pow(sun_dot, 64/8) and the Fresnel pow(.., 5)):
// squaring chain in double, rounded once to float.  x^2 is exact in double; every later product
// carries <= 2^-53 relative error, so the float result equals the correctly rounded pow except
// when the exact value lies within ~6*2^-53 of a rounding midpoint (probability ~1e-8).
__device__ __forceinline__ void pow8_64(float x, float& p8, float& p64) {
  const double s = (double)x, s2 = s * s, s4 = s2 * s2, s8 = s4 * s4, s16 = s8 * s8, s32 = s16 * s16;
  p8 = (float)s8;
  p64 = (float)(s32 * s32);
}
__device__ __forceinline__ float pow5(float x) {
  const double s = (double)x, s2 = s * s;
  return (float)((s2 * s2) * s);
}

// EnvironmentManager::getSkyColor
__device__ __forceinline__ vec3 sky_color(vec3 d) {
  float t = 0.5f * (d.y + 1.0f);
  {
    const float u = clamp_g((t - 0.0f) / (1.0f - 0.0f), 0.0f, 1.0f);
    t = u * u * (3.0f - 2.0f * u);
  }
  vec3 c = mix(v3(0.7f, 0.8f, 0.9f), v3(0.2f, 0.4f, 0.8f), t);
  const vec3 sd = v3(kSunDirX, kSunDirY, kSunDirZ);  // normalize(vec3(0.3, 0.6, -0.8)), precomputed
  const float sdot = fmax_g(dot(d, sd), 0.0f);
  float p8, p64;
  pow8_64(sdot, p8, p64);
  const float si = p64;
  const float sg = p8 * 0.3f;
  c = c + v3(1.0f, 0.9f, 0.7f) * (si + sg);
  return c * 0.8f;
}

// Cubemap::sample + EnvironmentManager::getCubemapColor
__device__ __forceinline__ vec3 cube_texel(const float4* env, int S, int face, int x, int y) {
  const float4 t = env[((size_t)face * S + y) * S + x];
  return v3(t.x, t.y, t.z);
}
// kCube: the environment is a cubemap (sh.env != null), else the procedural sky; a template
// parameter so that the kernels of the common sky case carry no cubemap code or registers
template <bool kCube>
__device__ __forceinline__ vec3 env_color(const EnvView& sh, vec3 dir) {
  if (!kCube) return sky_color(dir);
  const vec3 d = renormalized_again(dir);  // every caller passes a normalized direction
  const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
  // Cubemap::directionToUV's face cases as selects: x-major, else y-major, else z-major, in the
  // reference's order of tests.  The conditions are combined with & (no short-circuit, which the
  // compiler turned into divergent branches), and the cases share their operands: the major component
  // dmaj (face sign, ma = |dmaj|), the u component (d.z on x faces, else d.x) and the v component (d.z on
  // y faces, else d.y), each negated by a sign-bit flip as the face's case says.
  const bool xm = (ax >= ay) & (ax >= az);
  const bool ym = !xm & (ay >= ax) & (ay >= az);
  const float dmaj = xm ? d.x : (ym ? d.y : d.z);
  const float ma = fabsf(dmaj);
  const bool pos = dmaj > 0.0f;
  const int face = (xm ? 0 : (ym ? 2 : 4)) + (pos ? 0 : 1);
  const bool uneg = xm ? pos : (!ym & !pos);  // x: pos ? -d.z : d.z; y: d.x; z: pos ? d.x : -d.x
  const bool vneg = !ym | !pos;               // x, z: -d.y; y: pos ? d.z : -d.z
  const float uc = __uint_as_float(__float_as_uint(xm ? d.z : d.x) ^ (uneg ? 0x80000000u : 0u));
  const float vc = __uint_as_float(__float_as_uint(ym ? d.z : d.y) ^ (vneg ? 0x80000000u : 0u));
  // uc / ma and vc / ma share the divisor (ma in [1/sqrt(3), 1]): correctly rounded for |uc| >=
  // 2^-100 (cr_math.h div_nrm, checked by tests/hip/crmath_check.hip); below that the quotient is
  // under 2^-99 either way and q + 1 rounds to 1 exactly
  const DivBy dm = div_by(ma);
  const float u = clamp_g((div_nrm(uc, dm) + 1.0f) * 0.5f, 0.0f, 1.0f);
  const float v = clamp_g((div_nrm(vc, dm) + 1.0f) * 0.5f, 0.0f, 1.0f);
  const int S = sh.env_size;
  const float fx_ = u * float(S - 1), fy_ = v * float(S - 1);
  const int x0 = (int)floorf(fx_), y0 = (int)floorf(fy_);
  const int x1 = min(x0 + 1, S - 1), y1 = min(y0 + 1, S - 1);
  const float fx = fx_ - float(x0), fy = fy_ - float(y0);
  // texel (face, x, y) = env[(face * S + y) * S + x]; 24-bit multiplies (S <= 4096)
  const uint32_t r0 = __umul24((uint32_t)(face * S + y0), (uint32_t)S), r1 = __umul24((uint32_t)(face * S + y1), (uint32_t)S);
  const float4 t00 = sh.env[r0 + (uint32_t)x0], t10 = sh.env[r0 + (uint32_t)x1];
  const float4 t01 = sh.env[r1 + (uint32_t)x0], t11 = sh.env[r1 + (uint32_t)x1];
  const vec3 c0 = mix(xyz(t00), xyz(t10), fx);
  const vec3 c1 = mix(xyz(t01), xyz(t11), fx);
  vec3 c = mix(c0, c1, fy);
  c = v3(fmin_g(c.x, sh.env_clamp), fmin_g(c.y, sh.env_clamp), fmin_g(c.z, sh.env_clamp));
  return c * sh.env_intensity;
}

// Material::evaluateBRDF (Material.cpp:84-117).  The GGX denominator is double as in the reference
// (M_PI is a double literal there).
__device__ __forceinline__ vec3 eval_brdf(const DevMaterial& m, vec3 N, vec3 V, vec3 L) {
  const vec3 albedo = v3(m.albedo[0], m.albedo[1], m.albedo[2]);
  const vec3 H = normalize(V + L);
  const float NdotV = fmax_g(dot(N, V), 0.0f);
  const float NdotL = fmax_g(dot(N, L), 0.0f);
  const float HdotV = fmax_g(dot(H, V), 0.0f);
  const float r = clamp_g(m.roughness, 0.02f, 1.0f);
  const float alpha = r * r;
  const float a2 = alpha * alpha;
  const float NdotH = fmax_g(dot(N, H), 0.0f);
  const float NdotH2 = NdotH * NdotH;
  float dden = (NdotH2 * (a2 - 1.0f) + 1.0f);
  dden = (float)(3.14159265358979323846 * (double)dden * (double)dden);
  const float D = a2 / dden;
  const float rr = clamp_g(sqrtf(fmax_g(alpha, 0.0f)), 0.02f, 1.0f);
  const float kq = (rr + 1.0f);
  const float k = (kq * kq) / 8.0f;
  const float g_v = NdotV / (NdotV * (1.0f - k) + k);
  const float g_l = NdotL / (NdotL * (1.0f - k) + k);
  const float G = g_l * g_v;
  float f0d = (m.ior - 1.0f) / (m.ior + 1.0f);
  f0d *= f0d;
  const vec3 F0 = mix(v3(f0d, f0d, f0d), albedo, m.metallic);
  const float pw = pow5(clamp_g(1.0f - HdotV, 0.0f, 1.0f));
  const vec3 F = F0 + (1.0f - F0) * pw;
  const vec3 numer = (D * G) * F;
  const float denom = 4.0f * NdotV * NdotL + 0.0001f;
  const vec3 spec = numer / denom;
  const vec3 kD = 1.0f - F;
  const vec3 diffuse = (albedo * (1.0f - m.metallic)) / float(3.14159265358979323846);
  return (kD * diffuse + spec) * NdotL;
}

// --------------------------------------------------------------------------------- launch timing
// A slot-timed launch (WaveView::tslot set by the stage timer: one launch chain) leaves the device's
// constant-rate wall clock (wall_clock64, 100 MHz) in its slot: block 0, the first dispatched, stores
// its start in word 0, and every block's thread 0, once the block is done, takes the maximum of its end
// into one of kTimeEndLines words on lines of their own (atomicMax on a zeroed slot).  No packet sits
// between the launch and its neighbours: the 8-way C2 shard 0.541-0.544 ms with dispatch events,
// 0.525-0.532 with slots (r05zzj).  One shared end word made it 0.71 ms (thousands of atomics on one
// address); every wave's end on 64 words 0.541-0.543.  The kernels have no early return: every thread
// reaches ktime_end's barrier.  The two kernels of the pixel lanes' chains (k_trace_wp, k_bounce) carry
// it only in their kTimed instantiation: the slot pointer held across them cost spills, and the
// end-of-block barrier keeps a block's wave slots until its last wave is done, which the other lane
// would fill (two-lane C2 2.61-2.66 ms with it compiled in, 2.55-2.61 without; the lanes' launches are
// timed by dispatch events, Context::time_by_events).
__device__ __forceinline__ void ktime_begin(const WaveView& w) {
  if (w.tslot && blockIdx.x == 0 && threadIdx.x == 0) w.tslot[0] = (unsigned long long)wall_clock64();
}
__device__ __forceinline__ void ktime_end(const WaveView& w) {
  if (!w.tslot) return;  // (uniform: a kernel argument)
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(w.tslot + kTimeLineWords * (1u + (blockIdx.x & (kTimeEndLines - 1u))), (unsigned long long)wall_clock64());
}

// --------------------------------------------------------------------------------- k_trace
// Bounce 0, pixel-major (f.pixel_major == kFoldThread: LDS-staged scenes, where every primary ray
// costs about the same, in batches with >= kPixelMajorItems pixels per resident thread): thread <-
// local pixel l, looping over the batch's k sample slots in sample order (path p = s*P + l, as
// everywhere else).  Misses before the pixel's first hit are summed straight into the accumulator
// — the same adds, in the same order, that k_accum would do — so an all-sky pixel writes no
// radiance at all and k_accum skips it; from the first hit on, misses go to rad[p] and k_accum
// resumes there (accum.w = resume slot).  A kernel of its own (not a branch of k_trace), so that
// its registers are allocated for this loop alone.
//
// Work distribution: 256-pixel chunks dealt round-robin over the blocks (block_sched).  (r04 A/B: a
// global 64-pixel queue in k_cull's unculled-first order left this launch unchanged and slowed k_shade,
// whose hit records then came from all over the frame)
template <bool kCount, bool kW4, bool kCube>
__global__ void __launch_bounds__(kBlock, kW4 ? SPTR_TRACE4_WAVES : SPTR_TRACE_PM_WAVES)
    k_trace_pm(SceneView sv, EnvView sh, FrameView fin, WaveView w) {
  ktime_begin(w);
  const FrameView f = frame_dyn(fin);
  __shared__ LdsStack s_stack;
  extern __shared__ float4 lds[];
  __shared__ uint32_t s_cnt;
  __shared__ uint32_t s_hist[kCount ? kHistBins : 1];
  if (threadIdx.x == 0) s_cnt = 0u;
  if (kCount) hist_init(s_hist);
  const Staged sc = stage_scene<true>(sv, lds);
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    atomicAdd(&w.tot[kTotClosest], (unsigned long long)((unsigned long long)f.valid * f.k));
    atomicAdd(&w.tot[kTotTracedP], (unsigned long long)(primary_traced(f)));
    atomicAdd(&w.tot[kTotTracedD], (unsigned long long)(primary_traced(f)));
  }
  const ImageDiv idiv = image_div(f);
  Visits vc;
  const Sched sd = block_sched(f.P);
  const uint32_t per = sd.per * f.k;  // hit-record segment stride: the block's pixels x k records
  const uint32_t seg0 = logical_block() * per;
  for (uint32_t it = 0;; ++it) {
    const uint32_t base = sd.first + it * sd.step;
    if (base >= sd.end) break;
    const uint32_t l = base + threadIdx.x;
    int x = 0, y = 0;
    const bool valid = l < f.P && local_pixel(f, l, x, y);
    const uint32_t ps = valid ? (uint32_t)(y * f.W + x) : 0u;
    const bool culled = valid && pixel_culled(f, l);
    vec3 a = v3(0.0f, 0.0f, 0.0f);
    if (valid && !f.reset) a = xyz(f.accum[l]);
    bool fold = true;
    uint32_t resume = f.k;
    for (uint32_t smp = 0; smp < f.k; ++smp) {
      bool hit = false;
      uint32_t ref = kNoHit;
      float tfar = __builtin_huge_valf();
      const uint32_t p = smp * f.P + l;
      if (valid) {
        Primary pr;
        primary_at(f, idiv, x, y, ps, f.acc0 + smp, pr);
        // SPTR_ABLATE (timing experiments only, wrong images): 2 = primary rays skip traversal,
        // 1 = constant environment, 4 = primary misses add no radiance
        if (!(ablate(f) & 2u) && !culled) {
          const Ray r = make_ray(f.cam_pos, pr.d);
          const uint32_t v0 = vc.nodes;
          hit = traverse_w<kW4, false, kCount>(sc, sv, r, 0.0f, tfar, ref, vc, s_stack);
          if (kCount) hist_ray(s_hist, vc.nodes - v0);
        }
        if (!hit) {
          vec3 rv = v3(0.0f, 0.0f, 0.0f);
          if (sh.debug_mode != 1) {
            const vec3 e = (ablate(f) & 1u) ? pr.d : env_color<kCube>(sh, renormalized_again(pr.d));
            rv = v3(0.0f, 0.0f, 0.0f) + v3(1.0f, 1.0f, 1.0f) * e;
          }
          if (!fold) w.rad[p] = f4(rv, 0.0f);
          else if (!(ablate(f) & 4u)) a = a + rv;
        } else if (fold) {
          fold = false;
          resume = smp;
        }
      }
      const uint32_t j = block_append(&s_cnt, hit);
      if (hit) {
        if (seg0 + j < w.hrec_cap) w.hrec.put(seg0 + j, p, __float_as_uint(tfar), ref);
        else w.tot[kTotOverflow] = 1ull;  // cannot happen (ensure_wave slack); reported, never written
      }
    }
    if (l < f.P) f.accum[l] = make_float4(a.x, a.y, a.z, __uint_as_float(resume));
  }
  seg_publish(w.segH, &s_cnt, per);
  if (kCount && threadIdx.x == 0) atomicAdd(&w.tot[kTotHitP], (unsigned long long)s_cnt);
  report_stack(vc, w.tot);
  if (kCount) {
    flush_visits(vc, w.tot, kTotNodes);
    flush_visits(vc, w.tot, kTotNodesP);
    flush_depth_nodes(vc, w.tot, 0);
    hist_flush(s_hist, w.tot, kTotHistT);
  }
  ktime_end(w);
}

// Bounce 0, lane groups per pixel (f.pixel_major == kFoldWave: LDS-staged scenes in batches of >=
// kWaveFoldMinK samples where the thread-per-pixel loop above would leave resident threads idle,
// i.e. the per-rank share of a sharded frame).
// A wave owns 8 local pixels; the 8 lanes of pixel g trace its samples 8 at a time (lane q takes
// sample r*8 + q of round r), so a wave's rays come from 8 neighbouring pixels.  A pixel's leading
// misses (the samples before its first hit) are summed into the accumulator in sample order — an
// 8-step shuffle loop per round, the same adds in the same order as k_accum; later misses go to
// rad[p] and accum.w records where k_accum resumes.  Blocks take 32-pixel chunks round-robin (a
// global queue in k_cull's order measured slower, r04f).  (Measured on the 8-way C2 shard: 4 lanes per pixel with DPP quad broadcasts
// 289 us, 8 lanes 234 us, 64 lanes 449 us; path-major 196 us + 54 us more in k_accum.)
constexpr uint32_t kFoldLanes = 8;  // samples per pixel per round = lanes per pixel group
// kHiOcc: 8 waves/SIMD for shards whose pixels fill the resident waves only a few times (r04u: the
// 8-way C2 shard 0.554 -> 0.541 ms, while 2- and 4-way shards lose ~1.5 % at 8 waves)
template <bool kLds, bool kCount, bool kW4, bool kCube, bool kHiOcc = false, bool kTimed = false>
__global__ void __launch_bounds__(kBlock, kW4 ? SPTR_TRACE4_WAVES : (kHiOcc ? 8 : SPTR_TRACE_WP_WAVES))
    k_trace_wp(SceneView sv, EnvView sh, FrameView fin, WaveView w) {
  if constexpr (kTimed) ktime_begin(w);
  const FrameView f = frame_dyn(fin);
  __shared__ KernelStack<kLds> s_stack;
  extern __shared__ float4 lds[];
  __shared__ uint32_t s_cnt;
  __shared__ uint32_t s_hist[kCount ? kHistBins : 1];
  __shared__ float4 s_fold[kBlock];  // the round's values of the wave's pixel groups (the fold below)
  if (threadIdx.x == 0) s_cnt = 0u;
  if (kCount) hist_init(s_hist);
  const Staged sc = stage_scene<kLds>(sv, lds);
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    atomicAdd(&w.tot[kTotClosest], (unsigned long long)((unsigned long long)f.valid * f.k));
    atomicAdd(&w.tot[kTotTracedP], (unsigned long long)(primary_traced(f)));
    atomicAdd(&w.tot[kTotTracedD], (unsigned long long)(primary_traced(f)));
  }
  const ImageDiv idiv = image_div(f);
  Visits vc;
  constexpr uint32_t kPix = kBlock / kFoldLanes;   // pixels per block round of the static share
  const uint32_t lane = lane_id(), q = lane & (kFoldLanes - 1u), g0 = lane & ~(kFoldLanes - 1u);
  const uint32_t lb = logical_block();
  const uint32_t step = gridDim.x * kPix;
  const uint32_t cap = (f.P + step - 1u) / step * kPix;  // pixels per block at most
  const uint32_t per = cap * f.k;                          // hit-record segment stride
  const uint32_t seg0 = lb * per;
  const uint32_t rounds = (f.k + kFoldLanes - 1u) / kFoldLanes;
  for (uint32_t it = 0;; ++it) {
    const uint32_t base = lb * kPix + it * step;
    if (base >= f.P) break;
    const uint32_t l = base + threadIdx.x / kFoldLanes;
    int x = 0, y = 0;
    const bool valid = l < f.P && local_pixel(f, l, x, y);
    const uint32_t ps = valid ? (uint32_t)(y * f.W + x) : 0u;
    const bool culled = valid && pixel_culled(f, l);
    vec3 a = v3(0.0f, 0.0f, 0.0f);
    if (valid && !f.reset) a = xyz(f.accum[l]);
    bool fold = true;
    uint32_t resume = f.k;
    for (uint32_t r = 0; r < rounds; ++r) {
      const uint32_t smp = r * kFoldLanes + q;
      const bool act = valid && smp < f.k;
      bool hit = false;
      uint32_t ref = kNoHit;
      float tfar = __builtin_huge_valf();
      const uint32_t p = smp * f.P + l;
      vec3 rv = v3(0.0f, 0.0f, 0.0f);
      if (act) {
        Primary pr;
        primary_at(f, idiv, x, y, ps, f.acc0 + smp, pr);
        if (!culled) {
          const Ray r = make_ray(f.cam_pos, pr.d);
          const uint32_t v0 = vc.nodes;
          hit = traverse_w<kW4, false, kCount>(sc, sv, r, 0.0f, tfar, ref, vc, s_stack);
          if (kCount) hist_ray(s_hist, vc.nodes - v0);
        }
        if (!hit && sh.debug_mode != 1) rv = v3(0.0f, 0.0f, 0.0f) + v3(1.0f, 1.0f, 1.0f) * env_color<kCube>(sh, renormalized_again(pr.d));
      }
      // this pixel group's hits of the round -> number of leading misses still to fold
      const uint32_t hm = (uint32_t)(__ballot(hit) >> g0) & ((1u << kFoldLanes) - 1u);
      const uint32_t nact = f.k - r * kFoldLanes < kFoldLanes ? f.k - r * kFoldLanes : kFoldLanes;
      const uint32_t nfold = fold ? (hm ? (uint32_t)__builtin_ctz(hm) : nact) : 0u;
      // the group's values through LDS: one write per lane, and the group's first lane (the one that
      // stores the sum) reads and adds them in sample order; the wave's own LDS accesses are in order.
      // (r06: 24 shuffles per round before, with every lane of the group adding: C2 2.373-2.38 -> 2.321-2.331
      // ms/step, the 8-way shard 0.481-0.504 -> 0.476-0.478, gpurun_out/r06s)
      s_fold[threadIdx.x] = make_float4(rv.x, rv.y, rv.z, 0.0f);
      __builtin_amdgcn_wave_barrier();
      if (q == 0u) {
#pragma unroll
        for (uint32_t j = 0; j < kFoldLanes; ++j) {
          if (j < nfold) {
            const float4 v = s_fold[threadIdx.x + j];
            a = v3(a.x + v.x, a.y + v.y, a.z + v.z);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
      if (fold && hm) {
        fold = false;
        resume = r * kFoldLanes + nfold;
      }
      if (act && !hit && q >= nfold) w.rad[p] = f4(rv, 0.0f);
      const uint32_t j = block_append(&s_cnt, hit);
      if (hit) {
        if (seg0 + j < w.hrec_cap) w.hrec.put(seg0 + j, p, __float_as_uint(tfar), ref);
        else w.tot[kTotOverflow] = 1ull;  // cannot happen (ensure_wave slack); reported, never written
      }
    }
    if (q == 0u && l < f.P) f.accum[l] = make_float4(a.x, a.y, a.z, __uint_as_float(valid ? resume : f.k));
  }
  seg_publish(w.segH, &s_cnt, per);
  if (kCount && threadIdx.x == 0) atomicAdd(&w.tot[kTotHitP], (unsigned long long)s_cnt);
  report_stack(vc, w.tot);
  if (kCount) {
    flush_visits(vc, w.tot, kTotNodes);
    flush_visits(vc, w.tot, kTotNodesP);
    flush_depth_nodes(vc, w.tot, 0);
    hist_flush(s_hist, w.tot, kTotHistT);
  }
  if constexpr (kTimed) ktime_end(w);
}
// Closest hit for every ray of this bounce.  A miss ends the path here: the environment term
// (wf_pt_cpu.cpp:98-103) is added to rad[p] in place, so only hits go on to k_shade, as dense hit
// records in this block's segment.  kPrimary: bounce 0, one thread per path slot, camera ray
// computed in place (no input stream at all).  Input of later bounces: the dense ray stream
// rs[depth&1] written by the previous k_shade, addressed through its segment table.
template <bool kLds, bool kCount, bool kPrimary, bool kW4, bool kCube>
__global__ void __launch_bounds__(kBlock, (kW4 && !kPrimary) ? SPTR_TRACE4_WAVES : SPTR_TRACE_WAVES)
    k_trace(SceneView sv, EnvView sh, FrameView fin, WaveView w, int depth, uint32_t nseg_in) {
  ktime_begin(w);
  const FrameView f = frame_dyn(fin);
  __shared__ KernelStack<kLds> s_stack;
  extern __shared__ float4 lds[];
  __shared__ uint32_t s_cnt;
  uint32_t* s_off = reinterpret_cast<uint32_t*>(lds + (kLds ? sv.lds_bytes / 16u : 0u));
  __shared__ uint32_t s_hist[kCount ? kHistBins : 1];
  if (threadIdx.x == 0) s_cnt = 0u;
  if (kCount) hist_init(s_hist);
  const Staged sc = stage_scene<kLds>(sv, lds);
  // Bounce 0 path-major (thread <- path slot): batches of fewer than kWaveFoldMinK samples (e.g.
  // the interactive 1 spp per call).  Later bounces: thread <- queued ray.
  uint32_t n, per_in = 0u, nlist = 0u;
  if (kPrimary) {
    // with a cull list (f.plist, path-major + k_sky) only the unculled pixels' paths are traced:
    // compacted item i -> sample i / Q of listed pixel i % Q, so waves hold no culled lanes
    nlist = f.plist ? f.plist[f.P] : 0u;
    n = f.plist ? nlist * f.k : f.P * f.k;
    __syncthreads();
  } else {
    n = seg_scan(w.segN, nseg_in, s_off, per_in);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    atomicAdd(&w.tot[kTotClosest], (unsigned long long)(kPrimary ? (unsigned long long)f.valid * f.k : n));
    const unsigned long long t = kPrimary ? primary_traced(f) : (unsigned long long)n;
    atomicAdd(&w.tot[kPrimary ? kTotTracedP : kTotTracedB], (unsigned long long)(t));
    atomicAdd(&w.tot[kTotTracedD + stat_depth(depth)], (unsigned long long)(t));
  }
  const ImageDiv idiv = image_div(f);
  const RayStream rs = w.rs[depth & 1];
  Visits vc;
  const Sched sd = block_sched(n);
  for (uint32_t base = sd.first; base < sd.end; base += sd.step) {
    const uint32_t i = base + threadIdx.x;
    bool active = i < n, hit = false, culled = false;
    uint32_t id = 0u, pid = 0u, ref = kNoHit;
    float tfar = __builtin_huge_valf();
    vec3 o, d;
    if (active) {
      if (kPrimary) {
        Primary pr;
        uint32_t l, p = i;
        if (f.plist) p = primary_item(f, nlist, i);
        id = pid = p;
        active = primary_path(f, idiv, p, pr, l);
        culled = !f.plist && pixel_culled(f, l);
        o = f.cam_pos;
        d = pr.d;
      } else {
        id = seg_slot(s_off, nseg_in, per_in, i);
        const float4 o4 = rs.o[id], d4 = rs.d[id];
        o = xyz(o4);
        d = xyz(d4);
        pid = __float_as_uint(d4.w);
      }
    }
    if (active) {
      const Ray r = make_ray(o, d);
      // SPTR_ABLATE (timing experiments only, wrong images): 2 = primary rays skip traversal,
      // 1 = constant environment, 4 = primary misses write no radiance
      if (!(kPrimary && ((ablate(f) & 2u) || culled))) {
        const uint32_t v0 = vc.nodes;
        hit = traverse_w<kW4, false, kCount>(sc, sv, r, 0.0f, tfar, ref, vc, s_stack);
        if (kCount) hist_ray(s_hist, vc.nodes - v0);
      }
      if (kPrimary && !hit && (ablate(f) & 4u)) {
      } else if (!hit) {
        if (sh.debug_mode == 1) {
          w.rad[pid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        } else {
          const vec3 e = (ablate(f) & 1u) ? d : env_color<kCube>(sh, renormalized_again(d));
          vec3 rv;
          if (kPrimary) rv = v3(0.0f, 0.0f, 0.0f) + v3(1.0f, 1.0f, 1.0f) * e;
          else rv = xyz(w.rad[pid]) + xyz(rs.thr[id]) * e;
          w.rad[pid] = f4(rv, 0.0f);
        }
      }
    }
    const uint32_t j = block_append(&s_cnt, hit);
    if (hit) {
      if (sd.seg0 + j < w.hrec_cap) w.hrec.put(sd.seg0 + j, id, __float_as_uint(tfar), ref);
      else w.tot[kTotOverflow] = 1ull;  // cannot happen (ensure_wave slack); reported, never written
    }
  }
  seg_publish(w.segH, &s_cnt, sd.per);
  if (kCount && threadIdx.x == 0) atomicAdd(&w.tot[kPrimary ? kTotHitP : kTotHitB], (unsigned long long)s_cnt);
  report_stack(vc, w.tot);
  if (kCount) {
    flush_visits(vc, w.tot, kTotNodes);
    if (kPrimary) flush_visits(vc, w.tot, kTotNodesP);
    flush_depth_nodes(vc, w.tot, depth);
    hist_flush(s_hist, w.tot, kTotHistT);
  }
  ktime_end(w);
}

// BVH2 (LDS-staged) or wide walk over the staged / global scene pointers
template <bool kAny, bool kCount, bool kW4>
__device__ __forceinline__ bool walk_start(WideWalk& wk, const Staged& sc, uint32_t root, const Ray& r, float tnear,
                                           float& tfar, uint32_t& ref, Visits& vc) {
  return wide_start<kAny, kCount>(wk, root, sc.prim_ref, sc.tris, sc.sph, r, tnear, tfar, ref, vc);
}
template <bool kAny, bool kCount, bool kW4, int kKind = kWalkU, int N>
__device__ __forceinline__ bool walk_steps(WideWalk& wk, TravStack<N>& stack, const Staged& sc, const uint4* top,
                                           uint32_t ntop, const Ray& r, float tnear, float& tfar, uint32_t& ref, Visits& vc,
                                           int steps) {
  if (kW4)
    return wide_walk<kAny, kCount, kKind>(wk, stack, sc.nodes4, top, ntop, sc.prim_ref, sc.tris, sc.sph, r, tnear, tfar, ref, vc,
                                   steps);
  return bvh2_walk<kAny, kCount>(wk.cur, wk.sp, wk.hit, stack, sc.nodes, sc.prim_ref, sc.tris, sc.sph, r, tnear, tfar, ref,
                                 vc, steps);
}

// --------------------------------------------------------------------------------- refilling trace
// k_trace for wide BVHs traversed from L2/HBM (C3, C5): the same per-ray work, but each lane takes
// a new ray from the block's items as soon as its current one is done, instead of waiting for the
// slowest lane of its wave.  Rays there differ in cost by orders of magnitude (a sky ray ends after
// one node, a ray into a 10M-triangle mesh visits dozens), so a statically assigned wave holds its
// registers for its longest ray with most lanes idle; refilling keeps the wave's lanes, and with
// them the memory requests in flight, busy.  Lanes advance kDynSteps node visits between refills.
// The block still owns exactly the items of its static schedule (chunk c: sd.first + c * sd.step
// + [0, kBlock)), so its hit-record segment and the consumer's mapping are unchanged.
#ifndef SPTR_DYN_STEPS
#define SPTR_DYN_STEPS 8
#endif
constexpr int kDynSteps = SPTR_DYN_STEPS;
__device__ __forceinline__ uint32_t block_items(const Sched& sd, uint32_t n) {
  if (sd.first >= sd.end) return 0u;
  const uint32_t rest = sd.end - sd.first, full = rest / sd.step, tail = rest - full * sd.step;
  return full * kBlock + (tail < kBlock ? tail : kBlock);
}
__device__ __forceinline__ uint32_t block_item(const Sched& sd, uint32_t k) {
  return sd.first + (k / kBlock) * sd.step + (k % kBlock);
}

// Per-XCD work queues (k_shadow_dyn and k_trace_dyn of scenes larger than an XCD's L2): one counter
// per XCD (128 B apart) hands out that XCD's 256-item chunks of the static round-robin schedule in
// order, a 64-item quarter at a time to a wave whose quarter is used up.  The schedule's L2 locality
// stays (an XCD works through its own chunks in order), each counter sees an eighth of the grabs, and
// no wave idles while its XCD holds unstarted items.  A producer with an output segment per block
// (k_trace_dyn) reserves room for a quarter in its block's segment (s_taken, cap items) before taking
// it; the segments hold twice the static shares, so while items remain some block of the XCD has room.
constexpr uint32_t kQueueChunk = 64u;
struct XcdQueue {
  uint32_t* counter;
  uint32_t xcd, per_xcd, n;
  uint32_t cbase, cend;  // the wave's current quarter [cbase, cend) (wave-uniform)
  bool drained;          // no unstarted item is left for this wave
};
__device__ __forceinline__ XcdQueue xcd_queue(uint32_t* counters, uint32_t n) {
  XcdQueue q;
  const bool xm = (gridDim.x % kXcds) == 0u;
  q.xcd = xm ? blockIdx.x % kXcds : 0u;
  q.per_xcd = xm ? gridDim.x / kXcds : gridDim.x;  // logical blocks per XCD
  q.counter = counters + q.xcd * 32u;
  q.n = n;
  q.cbase = q.cend = 0u;
  q.drained = false;
  return q;
}
// The next item for each lane with `need` (kNoHit for the others, or when nothing is left); every lane
// of the wave calls it together.
__device__ __forceinline__ uint32_t xcd_take(XcdQueue& q, bool need, uint32_t* s_taken, uint32_t cap) {
  const uint32_t lane = lane_id();
  const unsigned long long below = (1ull << lane) - 1ull;
  const unsigned long long m = __ballot(need);
  uint32_t item = kNoHit;
  if (m == 0ull || q.drained) return item;
  const uint32_t cnt = (uint32_t)__popcll(m), rank = (uint32_t)__popcll(m & below);
  const uint32_t t1 = min(cnt, q.cend - q.cbase);
  if (need && rank < t1) item = q.cbase + rank;
  q.cbase += t1;
  if (cnt > t1) {  // the quarter ran out: the next one from the queue
    uint32_t u = kNoHit;
    if (lane == 0u) {
      const bool room = s_taken == nullptr || atomicAdd(s_taken, kQueueChunk) + kQueueChunk <= cap;
      if (room) u = atomicAdd(q.counter, 1u);
    }
    u = __shfl(u, 0);
    if (u == kNoHit) {  // this block's output segment is full: the XCD's other blocks take the rest
      q.drained = true;
      return item;
    }
    // unit u: quarter u % 4 of this XCD's (u / 4)-th chunk c = j * G + xcd * per_xcd + rr
    const uint32_t kq = u >> 2, j = kq / q.per_xcd, rr = kq - j * q.per_xcd;
    const uint64_t c = (uint64_t)j * gridDim.x + (uint64_t)q.xcd * q.per_xcd + rr;
    const uint64_t b0 = c * kBlock + (u & 3u) * kQueueChunk;
    if (b0 >= q.n) {
      q.drained = true;
    } else {
      q.cbase = (uint32_t)b0;
      q.cend = min((uint32_t)b0 + kQueueChunk, q.n);
      const uint32_t t2 = min(cnt - t1, q.cend - q.cbase);
      if (need && rank >= t1 && rank - t1 < t2) item = q.cbase + (rank - t1);
      q.cbase += t2;
    }
  }
  return item;
}

// kQueue (scenes larger than an XCD's L2, r04): items come from the per-XCD work queues (xcd_take,
// counters zeroed by k_shade and k_accum) instead of the block's static share, so the launch does not
// wait for the blocks that drew the costly rays; hit records stay in the block's segment, sized for
// twice its static share.
template <bool kLds, bool kCount, bool kPrimary, bool kW4, bool kCube, bool kQueue>
__global__ void __launch_bounds__(kBlock, (kW4 && !kPrimary) ? SPTR_TRACE4_WAVES : SPTR_TRACE_WAVES)
    k_trace_dyn(SceneView sv, EnvView sh, FrameView fin, WaveView w, int depth, uint32_t nseg_in) {
  ktime_begin(w);
  const FrameView f = frame_dyn(fin);
  __shared__ KernelStack<kLds> s_stack;
  extern __shared__ float4 lds[];
  __shared__ uint32_t s_cnt, s_next, s_hits, s_taken;
  __shared__ uint32_t s_hist[kCount ? kHistBins : 1];
  uint32_t* s_off = reinterpret_cast<uint32_t*>(lds + (kLds ? sv.lds_bytes / 16u : 0u));
  if (threadIdx.x == 0) s_cnt = s_next = s_hits = s_taken = 0u;
  if (kCount) hist_init(s_hist);
  const Staged sc = stage_scene<kLds>(sv, lds);
  constexpr int kKind = kPrimary ? kWalkPrimary : kWalkU;
  const uint32_t ntop = (kW4 && !kLds && walk_reads_top(kKind)) ? sv.num_top4 : 0u;
  const uint4* top = ntop ? stage_top(sv, lds + top_lds_offset(sv, kLds, kPrimary, nseg_in)) : nullptr;
  uint32_t n, per_in = 0u, nlist = 0u;
  if (kPrimary) {
    nlist = f.plist ? f.plist[f.P] : 0u;
    n = f.plist ? nlist * f.k : f.P * f.k;
    __syncthreads();
  } else {
    n = seg_scan(w.segN, nseg_in, s_off, per_in);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    atomicAdd(&w.tot[kTotClosest], (unsigned long long)(kPrimary ? (unsigned long long)f.valid * f.k : n));
    const unsigned long long t = kPrimary ? primary_traced(f) : (unsigned long long)n;
    atomicAdd(&w.tot[kPrimary ? kTotTracedP : kTotTracedB], (unsigned long long)(t));
    atomicAdd(&w.tot[kTotTracedD + stat_depth(depth)], (unsigned long long)(t));
  }
  const ImageDiv idiv = image_div(f);
  const RayStream rs = w.rs[depth & 1];
  Visits vc;
  const Sched sd = block_sched(n);
  const uint32_t nb = block_items(sd, n);
  const uint32_t cap = kQueue ? 2u * sd.per : sd.per;  // records of the block's hit-record segment
  const uint32_t seg0 = logical_block() * cap;
  XcdQueue xq = xcd_queue(w.work + kWorkTraceQueue, n);
  TravStack<kLds ? kLdsStack : kLdsStackG> stack;
  stack.lds = &s_stack.e[0][threadIdx.x];
  bool have = false, done = false;
  uint32_t id = 0u, pid = 0u, ref = kNoHit;
  uint32_t v0 = 0u;  // kCount: the lane's node visits when its current ray started
  float tfar = 0.0f;
  Ray r;
  WideWalk wk;
  bool drained = false;  // (wave-uniform) a lane of this wave asked for a ray and none was left
  for (;;) {
    uint32_t item = kNoHit;
    bool more;  // unstarted items may remain for this wave
    if constexpr (kQueue) {
      item = xcd_take(xq, !have, &s_taken, cap);
      more = !xq.drained;
      drained = xq.drained;
    } else {
      const uint32_t k = block_take(&s_next, !have);
      if (!have && k < nb) item = block_item(sd, k);
      more = __ballot(!have && k < nb) != 0ull;
      if (__ballot(!have && k >= nb) != 0ull) drained = true;
    }
    if (item != kNoHit) {
      const uint32_t i = item;
      bool valid = true, culled = false;
      vec3 o, d;
      if (kPrimary) {
        Primary pr;
        uint32_t l, p = i;
        if (f.plist) p = primary_item(f, nlist, i);
        id = pid = p;
        valid = primary_path(f, idiv, p, pr, l);
        culled = !f.plist && pixel_culled(f, l);
        o = f.cam_pos;
        d = pr.d;
      } else {
        id = seg_slot(s_off, nseg_in, per_in, i);
        const float4 o4 = rs.o[id], d4 = rs.d[id];
        o = xyz(o4);
        d = xyz(d4);
        pid = __float_as_uint(d4.w);
      }
      if (valid) {
        r = make_ray(o, d);
        tfar = __builtin_huge_valf();
        ref = kNoHit;
        if (kCount) v0 = culled ? ~0u : vc.nodes;  // culled camera rays are not traversals
        done = walk_start<false, kCount, kW4>(wk, sc, culled ? kNoHit : (kW4 ? sv.root4 : sv.root), r, 0.0f, tfar, ref,
                                              vc);
        have = true;
      }
    }
    if (__ballot(have) == 0ull) {
      if (!more) break;  // nothing left for this wave
      continue;          // only invalid (outside-image) items taken
    }
    // the unified walk for camera rays as well (r03zy, with the pole ring's degenerate triangles out of
    // the tree and the launches overlapped: C5 8.45 inline vs 8.22 ms/step unified, means of 3; r03x,
    // before both: 2.15 vs 2.37 ms for the bounce-0 trace)
    if (have && !done)
      done = walk_steps<false, kCount, kW4, kKind>(wk, stack, sc, top, ntop, r, 0.0f, tfar, ref, vc,
                                                                          kDynSteps);
    // Straggler hand-off: the wave has no rays left to start and at most strag_lanes lanes are still
    // tracing (the long rays that would otherwise set the launch's length while the rest of the chip
    // idles).  Their rays and walk states (node, stack, closest hit so far) are written to the bounce's
    // straggler records; k_strag, beside the chain, resumes each walk where it stopped and carries its
    // path to the end.  No hit record is written here.
    if (!kCount && w.strag_lanes != 0u && drained && (uint32_t)depth < kStragBounces) {
      const unsigned long long act = __ballot(have && !done);
      if (act != 0ull && (uint32_t)__popcll(act) <= w.strag_lanes && have && !done) {
        const uint32_t slot = atomicAdd(&w.work[kWorkStrag + (uint32_t)depth * 32u], 1u);
        if (slot < w.strag_cap) {
          float4* rec = w.strag + ((size_t)depth * w.strag_cap + slot) * kStragRec;
          // the walk as it stands (k_strag resumes it: same node order, same hit)
          rec[3] = make_float4(__uint_as_float(wk.cur), __uint_as_float((uint32_t)wk.sp | (wk.hit ? 0x10000u : 0u)),
                               __uint_as_float(ref), tfar);
          uint32_t* st = reinterpret_cast<uint32_t*>(rec + 4);
          for (int q = 0; q < wk.sp; ++q) st[q] = stack.get(q);
          if (kPrimary) {
            Primary pr;
            (void)primary_path(f, idiv, pid, pr);
            rec[0] = f4(f.cam_pos, __uint_as_float(pr.rng));
            rec[1] = f4(r.d, __uint_as_float(pid));
            rec[2] = make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(0u));
          } else {
            rec[0] = rs.o[id];
            rec[1] = rs.d[id];
            rec[2] = f4(xyz(rs.thr[id]), __uint_as_float((uint32_t)depth));
          }
          have = false;
        }
      }
    }
    const bool fin = have && done;
    if (kCount && fin && v0 != ~0u) hist_ray(s_hist, vc.nodes - v0);
    const bool defer = !kPrimary && w.defer_miss != 0u;
    if (fin && !wk.hit) {
      if (defer) {  // the miss record's slot carries thr * env (k_shade adds it to rad[pid])
        if (sh.debug_mode != 1) rs.thr[id] = f4(xyz(rs.thr[id]) * env_color<kCube>(sh, renormalized_again(r.d)), 0.0f);
      } else if (sh.debug_mode == 1) {
        w.rad[pid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      } else {
        const vec3 e = env_color<kCube>(sh, renormalized_again(r.d));
        vec3 rv;
        if (kPrimary) rv = v3(0.0f, 0.0f, 0.0f) + v3(1.0f, 1.0f, 1.0f) * e;
        else rv = xyz(w.rad[pid]) + xyz(rs.thr[id]) * e;
        w.rad[pid] = f4(rv, 0.0f);
      }
    }
    const bool rec = fin && (wk.hit || defer);
    const uint32_t j = block_append(&s_cnt, rec);
    if (kCount) {
      const uint32_t nh = (uint32_t)__popcll(__ballot(fin && wk.hit));
      if (nh && lane_id() == 0u) atomicAdd(&s_hits, nh);
    }
    if (rec) {
      if (seg0 + j < w.hrec_cap) w.hrec.put(seg0 + j, id, wk.hit ? __float_as_uint(tfar) : pid, wk.hit ? ref : kNoHit);
      else w.tot[kTotOverflow] = 1ull;
    }
    if (fin) have = false;
  }
  seg_publish(w.segH, &s_cnt, cap);
  if (kCount && threadIdx.x == 0) atomicAdd(&w.tot[kPrimary ? kTotHitP : kTotHitB], (unsigned long long)s_hits);
  report_stack(vc, w.tot);
  if (kCount) {
    flush_visits(vc, w.tot, kTotNodes);
    if (kPrimary) flush_visits(vc, w.tot, kTotNodesP);
    flush_depth_nodes(vc, w.tot, depth);
    hist_flush(s_hist, w.tot, kTotHistT);
  }
  ktime_end(w);
}

// --------------------------------------------------------------------------------- shading steps
// The per-hit steps of WavefrontPathTracerCPU::traceRay (wf_pt_cpu.cpp:106-247), shared by the
// wavefront k_shade and the path-per-thread k_tail so both evaluate every path identically.
struct Surface {
  vec3 P, n;      // hit point, face-forwarded normal
  DevMaterial m;  // MaterialManager::getMaterialFromHit
};
__device__ __forceinline__ Surface surface_at(const SceneView& sv, const ShadeView& sh, const DevMaterial* smat,
                                              uint32_t nm, vec3 ro, vec3 rd, float t, uint32_t ref) {
  Surface s;
  s.P = ro + t * rd;
  const uint32_t idx = ref & kIndexMask;
  vec3 ng;
  uint32_t mid;
  if (ref & kSphereBit) {
    const float4 c = sv.sph[idx];
    ng = v3((s.P.x - c.x) / c.w, (s.P.y - c.y) / c.w, (s.P.z - c.z) / c.w);
    mid = sh.geom_mat[sv.sph_geom[idx]];
  } else {
    const float4 c = sv.tris[3 * idx + 2];
    ng = v3(c.y, c.z, c.w);
    mid = sh.tri_mat ? sh.tri_mat[idx] : sh.geom_mat[sv.tri_geom[idx]];
  }
  s.n = safe_normalize(ng);
  if (dot(s.n, rd) > 0.0f) s.n = -s.n;
  s.m = (mid < nm) ? smat[mid] : sh.mats[mid];
  return s;
}

// Light::getRadiance + direction/distance (Light.cpp:43-79)
__device__ __forceinline__ void light_at(const DevLight& Lt, vec3 P, vec3& ldir, float& ldist, vec3& Li) {
  if (Lt.type == 0) {
    ldir = v3(Lt.v[0], Lt.v[1], Lt.v[2]);
    ldist = __builtin_huge_valf();
    Li = v3(Lt.radiance[0], Lt.radiance[1], Lt.radiance[2]);
  } else {
    const vec3 lv = v3(Lt.v[0], Lt.v[1], Lt.v[2]) - P;
    ldist = sqrtf(dot(lv, lv));
    ldir = lv / ldist;
    const float att = 1.0f + 0.09f * ldist + 0.032f * ldist * ldist;
    Li = v3(Lt.radiance[0], Lt.radiance[1], Lt.radiance[2]) / att;
  }
}
__device__ __forceinline__ bool light_faces(const DevLight& Lt, const Surface& s) {
  vec3 ldir;
  if (Lt.type == 0) {
    ldir = v3(Lt.v[0], Lt.v[1], Lt.v[2]);
  } else {
    const vec3 lv = v3(Lt.v[0], Lt.v[1], Lt.v[2]) - s.P;
    ldir = lv / sqrtf(dot(lv, lv));
  }
  return fmax_g(dot(s.n, ldir), 0.0f) > 0.0f;
}
// Direct-light term of one light (wf_pt_cpu.cpp:127-147 with Light::isOccluded's shadow ray,
// Light.cpp:21-33): false when the light is behind the surface; else the shadow ray {so, ldir,
// [1e-4, tfar]} and the contribution added when it is unoccluded.
__device__ __forceinline__ bool light_term(const DevLight& Lt, const Surface& s, vec3 view, vec3 thr, vec3& so,
                                           vec3& ldir, float& tfar, vec3& contrib) {
  float ldist;
  vec3 Li;
  light_at(Lt, s.P, ldir, ldist, Li);
  const float cs = fmax_g(dot(s.n, ldir), 0.0f);
  if (cs <= 0.0f) return false;
  const float eps = 1e-4f * fmax_g(1.0f, fmax_g(fmax_g(fabsf(s.P.x), fabsf(s.P.y)), fabsf(s.P.z)));
  so = s.P + s.n * eps;
  tfar = ldist - 1e-4f;
  const vec3 fr = eval_brdf(s.m, s.n, view, ldir);
  contrib = thr * (fr * Li * cs);
  return true;
}

// Continuation: metal mirror, glass Fresnel/refraction, diffuse cosine sample + Russian roulette
// (wf_pt_cpu.cpp:151-247).  Updates thr and rng; false when the path is terminated.
__device__ __forceinline__ bool continue_path(const Surface& s, vec3 rd, uint32_t depth, vec3& thr, uint32_t& rng,
                                              vec3& no, vec3& nd) {
  const DevMaterial& m = s.m;
  const vec3 P = s.P, nrm = s.n;
  const vec3 albedo = v3(m.albedo[0], m.albedo[1], m.albedo[2]);
  if (m.metallic > 0.5f) {
    no = P + nrm * 1e-4f;
    nd = safe_renormalize_dir(reflect(rd, nrm));
    thr = thr * (albedo * m.metallic);
    return true;
  }
  if (m.metallic < 0.1f && m.ior > 1.3f) {
    const float ior = m.ior;
    const float cosine = -dot(rd, nrm);
    const float eta = (cosine >= 0.0f) ? (1.0f / ior) : ior;
    const float tr = clamp_g((ior - 1.0f) / 0.7f, 0.0f, 0.95f);
    float r0 = (1.0f - ior) / (1.0f + ior);
    r0 = r0 * r0;
    const float xc = 1.0f - clamp_std(fabsf(cosine), 0.0f, 1.0f);
    const float F = r0 + (1.0f - r0) * xc * xc * xc * xc * xc;
    const float xi = rand01(rng);
    if (xi < F) {
      no = P + nrm * 1e-4f;
      nd = safe_renormalize_dir(reflect(rd, nrm));
      thr = thr * v3(1.0f - tr, 1.0f - tr, 1.0f - tr);
    } else {
      const float ci = -dot(nrm, rd);
      const float kk = 1.0f - eta * eta * (1.0f - ci * ci);
      vec3 refr = v3(0.0f, 0.0f, 0.0f);
      if (!(kk < 0.0f)) refr = eta * rd + (eta * ci - sqrtf(kk)) * nrm;
      if (dot(refr, refr) > 0.0f) {
        no = P - nrm * 1e-4f;
        nd = safe_renormalize_dir(refr);
        thr = thr * v3(tr, tr, tr);
      } else {
        no = P + nrm * 1e-4f;
        nd = safe_renormalize_dir(reflect(rd, nrm));
      }
    }
    return true;
  }
  const float r1 = rand01(rng);
  const float r2 = rand01(rng);
  float sp, cp;
  cosine_sincos(r1, sp, cp);
  const float rr = sqrtf(r2);
  const float lx = rr * cp, ly = rr * sp;
  const float lz = sqrtf(fmax_g(0.0f, 1.0f - r2));
  const vec3 nn = renormalized_again(nrm);  // s.n: safe_normalize's output (or its negation)
  const vec3 tg = (fabsf(nn.z) < 0.999f) ? normalize_dir(cross(nn, v3(0.0f, 0.0f, 1.0f)))
                                         : normalize_dir(cross(nn, v3(0.0f, 1.0f, 0.0f)));
  const vec3 bt = cross(tg, nn);
  const vec3 sdir = safe_renormalize_dir(tg * lx + bt * ly + nn * lz);
  no = P + nrm * 1e-4f;
  const float surv = fmax_g(fmax_g(albedo.x, albedo.y), albedo.z);
  const float xi = rand01(rng);
  bool cont = true;
  if (depth > 2u) {
    if (xi >= surv) cont = false;
    else thr = thr * (albedo / fmax_g(surv, 1e-6f));
  } else {
    thr = thr * albedo;
  }
  nd = renormalized_again(sdir);  // sdir: safe_renormalize_dir's output
  return cont;
}

__device__ __forceinline__ uint32_t stage_materials(const ShadeView& sh, DevMaterial* smat) {
  const uint32_t nm = sh.num_mats < 32u ? sh.num_mats : 32u;
  for (uint32_t i = threadIdx.x; i < nm * 12u; i += blockDim.x)
    reinterpret_cast<float*>(smat)[i] = reinterpret_cast<const float*>(sh.mats)[i];
  return nm;
}

// --------------------------------------------------------------------------------- k_shade
// One thread per hit record of this bounce.  Radiance is read lazily (only when something is
// added) and written back once; bounce 0 starts from zero radiance and unit throughput in
// registers.  Outputs, each dense in this block's segment: the continuation rays (rs[(d+1)&1]) and
// one shadow record per path with >= 1 lit light: L tasks {origin.xyz, tfar} {contrib.xyz, p}
// [{dir.xyz}] (valid = contrib slot w != 0 is encoded by p+1; the direction slot exists only when a
// point light is present).
//
// kFuse (LDS-staged scenes with one light): the shadow ray is traced in place instead — the scene is
// staged into LDS next to the segment table, the lit light's any-hit query runs in this thread and
// its contribution is added to the radiance held in registers after the emission, exactly the
// update k_shadow would make next (Light::isOccluded), without the shadow-task stream, the
// radiance round trip and one launch per bounce.  Any-hit queries are tallied per block in bstat,
// as k_shadow does.
constexpr int kFuseStack = 6;  // LDS part of the in-shade traversal stack (C2's BVH2 is 9 deep)
template <bool kPrimary, bool kFuse>
__global__ void __launch_bounds__(kBlock, SPTR_SHADE_WAVES)
    k_shade(SceneView sv, ShadeView sh, FrameView fin, WaveView w, int depth, uint32_t nseg_in) {
  const FrameView f = frame_dyn(fin);
  extern __shared__ float4 lds[];
  uint32_t* s_off = reinterpret_cast<uint32_t*>(lds + (kFuse ? sv.lds_bytes / 16u : 0u));
  __shared__ DevMaterial smat[32];
  __shared__ uint32_t s_cnt_n, s_cnt_s, s_rays;
  __shared__ LdsStackN<kFuse ? kFuseStack : 1> s_stack;
  const uint32_t nm = stage_materials(sh, smat);
  if (threadIdx.x == 0) s_cnt_n = s_cnt_s = s_rays = 0u;
  if (blockIdx.x == 0 && threadIdx.x < kXcds) {
    w.work[((uint32_t)depth % 2u) * 256u + threadIdx.x * 32u] = 0u;  // k_shadow_dyn's queues of this bounce
    w.work[kWorkTraceQueue + threadIdx.x * 32u] = 0u;                 // k_trace_dyn's, for the next bounce
  }
  const Staged sc = stage_scene<kFuse>(sv, lds);
  Visits vc;
  uint32_t rays = 0u;
  uint32_t per_in = 0u;
  const uint32_t n = seg_scan(w.segH, nseg_in, s_off, per_in);

  const RayStream rin = w.rs[depth & 1], rout = w.rs[(depth + 1) & 1];
  const bool last = (uint32_t)(depth + 1) >= f.max_depth;
  const ImageDiv idiv = image_div(f);
  const uint32_t ts = w.tstride, L = w.L;
  const Sched sd = block_sched(n);
  for (uint32_t base = sd.first; base < sd.end; base += sd.step) {
    const uint32_t i = base + threadIdx.x;
    bool active = i < n;
    bool cont = false, shadow = false, dirty = kPrimary;
    uint32_t p = 0u, rng = 0u;
    vec3 rd, thr, radv = v3(0.0f, 0.0f, 0.0f), no, nd;
    Surface sf;
    uint3 h = make_uint3(0u, 0u, 0u);
    if (active) w.hrec.get(seg_slot(s_off, nseg_in, per_in, i), h.x, h.y, h.z);
    if (!kPrimary && active && h.z == kNoHit) {
      // a deferred miss of this bounce's trace (WaveView::defer_miss): rad[p] + thr * env, the update
      // the trace makes itself otherwise (record: slot, path id, kNoHit; the slot's throughput holds
      // thr * env)
      p = h.y;
      w.rad[p] = sh.debug_mode == 1 ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : f4(xyz(w.rad[p]) + xyz(rin.thr[h.x]), 0.0f);
      active = false;
    }
    if (active) {
      vec3 ro;
      if (kPrimary) {
        Primary pr;
        p = h.x;
        primary_path(f, idiv, p, pr);
        ro = f.cam_pos;
        rd = pr.d;
        thr = v3(1.0f, 1.0f, 1.0f);
        rng = pr.rng;
      } else {
        const float4 o4 = rin.o[h.x], d4 = rin.d[h.x];
        ro = xyz(o4);
        rd = xyz(d4);
        thr = xyz(rin.thr[h.x]);
        rng = __float_as_uint(o4.w);
        p = __float_as_uint(d4.w);
      }
      if (sh.debug_mode == 1) {
        radv = v3(1.0f, 1.0f, 1.0f);
        dirty = true;
      } else {
        sf = surface_at(sv, sh, smat, nm, ro, rd, __uint_as_float(h.y), h.z);
        const vec3 emission = v3(sf.m.emission[0], sf.m.emission[1], sf.m.emission[2]);
        if (dot(emission, emission) > 0.0f) {
          if (!kPrimary) radv = xyz(w.rad[p]);
          radv = radv + thr * emission;
          dirty = true;
        }
        // any light facing the surface -> this path gets a shadow record
        for (uint32_t li = 0; li < sh.num_lights; ++li)
          if (light_faces(sh.lights[li], sf)) shadow = true;
      }
    }
    // kFuse (one light): the shadow ray's query is prepared now, with the throughput before the
    // continuation, and traced after the continuation ray is written, so that little state lives
    // across the traversal
    vec3 so, ldir, contrib;
    float stfar = 0.0f;
    bool lit = false;
    if (kFuse) {
      if (shadow) lit = light_term(sh.lights[0], sf, -rd, thr, so, ldir, stfar, contrib);
      shadow = false;
    }
    const uint32_t js = kFuse ? 0u : block_append(&s_cnt_s, shadow);
    if (shadow && sd.seg0 + js >= w.seg_cap) {
      shadow = false;
      w.tot[kTotOverflow] = 1ull;
    }
    // shadow carry (WaveView::carry_depth, one light): the task's tag is written once the continuation
    // is known — 0 (k_shadow_dyn skips it; k_tail traces it) for a path that continues to the tail
    const bool carry = !kFuse && (uint32_t)depth == w.carry_depth;
    bool lit0 = false;
    vec3 c0 = v3(0.0f, 0.0f, 0.0f);
    if (shadow) {
      // direct light: shadow tasks carry the precomputed contribution, added if unoccluded
      float4* task = w.stask + (size_t)(sd.seg0 + js) * L * ts;
      const vec3 view = -rd;
      for (uint32_t li = 0; li < L; ++li, task += ts) {
        vec3 so, ldir, contrib;
        float tfar;
        if (!light_term(sh.lights[li], sf, view, thr, so, ldir, tfar, contrib)) {
          task[1] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(0u));
          continue;
        }
        task[0] = f4(so, tfar);
        if (ts > 2u) task[2] = f4(ldir, 0.0f);
        if (carry) {
          lit0 = true;
          c0 = contrib;
        } else {
          task[1] = f4(contrib, __uint_as_float(p + 1u));
        }
      }
    }
    if (active && sh.debug_mode != 1) cont = continue_path(sf, rd, (uint32_t)depth, thr, rng, no, nd) && !last;
    if (!kFuse && active && dirty) w.rad[p] = f4(radv, 0.0f);
    const uint32_t jn = block_append(&s_cnt_n, cont);
    if (cont && sd.seg0 + jn >= w.seg_cap) {
      cont = false;
      w.tot[kTotOverflow] = 1ull;
    }
    if (lit0) w.stask[(size_t)(sd.seg0 + js) * ts + 1u] = f4(c0, __uint_as_float(cont ? 0u : p + 1u));
    if (cont) {
      rout.o[sd.seg0 + jn] = f4(no, __uint_as_float(rng));
      rout.d[sd.seg0 + jn] = f4(nd, __uint_as_float(p));
      rout.thr[sd.seg0 + jn] = f4(thr, __uint_as_float(lit0 ? sd.seg0 + js + 1u : 0u));
    }
    if (kFuse) {
      if (lit) {
        const Ray r = make_ray(so, ldir);
        uint32_t ref = kNoHit;
        ++rays;
        if (!traverse_w<false, true, false>(sc, sv, r, 1e-4f, stfar, ref, vc, s_stack)) {
          if (!dirty) radv = xyz(w.rad[p]);  // kPrimary starts dirty at zero radiance
          dirty = true;
          radv = radv + contrib;
        }
      }
      if (active && dirty) w.rad[p] = f4(radv, 0.0f);
    }
  }
  if (kFuse) {
    for (int off = 32; off > 0; off >>= 1) rays += __shfl_xor(rays, off);
    if (lane_id() == 0u) atomicAdd(&s_rays, rays);
    report_stack(vc, w.tot);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    w.segN.cnt[logical_block()] = s_cnt_n;
    w.segS.cnt[logical_block()] = s_cnt_s;
    if (kFuse) w.bstat[blockIdx.x] += s_rays;
    if (blockIdx.x == 0) {
      *w.segN.per = sd.per;
      *w.segS.per = sd.per;
    }
  }
}

// --------------------------------------------------------------------------------- k_bounce
// One whole bounce d >= 1 of an LDS-staged one-light scene in one launch: k_trace (closest hit; a
// miss adds thr * env to rad[p]) and k_shade with its in-place shadow ray (emission, the light's
// contribution if unoccluded, continuation) per queued ray, with the per-path operations and the
// order of the radiance updates of the two kernels — so no hit-record stream and one launch less
// per bounce.  Input: the rays of w.segN / rs[d & 1]; output: the continuation rays in this
// block's segment of w.segH / rs[(d + 1) & 1] (the host alternates the two tables between bounces).
template <bool kCube, bool kTimed = false>
__global__ void __launch_bounds__(kBlock, SPTR_BOUNCE_WAVES)
    k_bounce(SceneView sv, ShadeView sh, FrameView fin, WaveView w, int depth, uint32_t nseg_in) {
  if constexpr (kTimed) ktime_begin(w);
  const FrameView f = frame_dyn(fin);
  extern __shared__ float4 lds[];
  uint32_t* s_off = reinterpret_cast<uint32_t*>(lds + sv.lds_bytes / 16u);
  __shared__ DevMaterial smat[32];
  __shared__ uint32_t s_cnt_n, s_rays;
  __shared__ LdsStack s_stack;
  const uint32_t nm = stage_materials(sh, smat);
  if (threadIdx.x == 0) s_cnt_n = s_rays = 0u;
  const Staged sc = stage_scene<true>(sv, lds);
  uint32_t per_in = 0u;
  const uint32_t n = seg_scan(w.segN, nseg_in, s_off, per_in);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    atomicAdd(&w.tot[kTotClosest], (unsigned long long)(n));
    atomicAdd(&w.tot[kTotTracedF], (unsigned long long)(n));
    atomicAdd(&w.tot[kTotTracedD + stat_depth(depth)], (unsigned long long)(n));
  }
  const RayStream rin = w.rs[depth & 1], rout = w.rs[(depth + 1) & 1];
  const bool last = (uint32_t)(depth + 1) >= f.max_depth;
  Visits vc;
  uint32_t rays = 0u;
  const Sched sd = block_sched(n);
  for (uint32_t base = sd.first; base < sd.end; base += sd.step) {
    const uint32_t i = base + threadIdx.x;
    bool cont = false, dirty = false, lit = false;
    uint32_t p = 0u, rng = 0u;
    vec3 thr, radv = v3(0.0f, 0.0f, 0.0f), no, nd, so, ldir, contrib;
    float stfar = 0.0f;
    if (i < n) {
      const uint32_t id = seg_slot(s_off, nseg_in, per_in, i);
      const float4 o4 = rin.o[id], d4 = rin.d[id];
      const vec3 ro = xyz(o4), rd = xyz(d4);
      p = __float_as_uint(d4.w);
      rng = __float_as_uint(o4.w);
      thr = xyz(rin.thr[id]);
      float tfar = __builtin_huge_valf();
      uint32_t ref = kNoHit;
      if (!traverse_w<false, false, false>(sc, sv, make_ray(ro, rd), 0.0f, tfar, ref, vc, s_stack)) {
        if (sh.debug_mode == 1) {
          w.rad[p] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        } else {
          const vec3 e = env_color<kCube>(sh.env, renormalized_again(rd));
          w.rad[p] = f4(xyz(w.rad[p]) + thr * e, 0.0f);
        }
      } else if (sh.debug_mode == 1) {
        radv = v3(1.0f, 1.0f, 1.0f);
        dirty = true;
      } else {
        const Surface sf = surface_at(sv, sh, smat, nm, ro, rd, tfar, ref);
        const vec3 emission = v3(sf.m.emission[0], sf.m.emission[1], sf.m.emission[2]);
        if (dot(emission, emission) > 0.0f) {
          radv = xyz(w.rad[p]) + thr * emission;
          dirty = true;
        }
        if (light_faces(sh.lights[0], sf)) lit = light_term(sh.lights[0], sf, -rd, thr, so, ldir, stfar, contrib);
        cont = continue_path(sf, rd, (uint32_t)depth, thr, rng, no, nd) && !last;
      }
    }
    const uint32_t jn = block_append(&s_cnt_n, cont);
    if (cont && sd.seg0 + jn >= w.seg_cap) {
      cont = false;
      w.tot[kTotOverflow] = 1ull;
    }
    if (cont) {
      rout.o[sd.seg0 + jn] = f4(no, __uint_as_float(rng));
      rout.d[sd.seg0 + jn] = f4(nd, __uint_as_float(p));
      rout.thr[sd.seg0 + jn] = f4(thr, 0.0f);
    }
    if (lit) {
      uint32_t ref = kNoHit;
      ++rays;
      if (!traverse_w<false, true, false>(sc, sv, make_ray(so, ldir), 1e-4f, stfar, ref, vc, s_stack)) {
        if (!dirty) radv = xyz(w.rad[p]);
        dirty = true;
        radv = radv + contrib;
      }
    }
    if (dirty) w.rad[p] = f4(radv, 0.0f);
  }
  for (int off = 32; off > 0; off >>= 1) rays += __shfl_xor(rays, off);
  if (lane_id() == 0u) atomicAdd(&s_rays, rays);
  report_stack(vc, w.tot);
  __syncthreads();
  if (threadIdx.x == 0) {
    w.segH.cnt[logical_block()] = s_cnt_n;
    w.bstat[blockIdx.x] += s_rays;
    if (blockIdx.x == 0) *w.segH.per = sd.per;
  }
  if constexpr (kTimed) ktime_end(w);
}

// --------------------------------------------------------------------------------- k_bounce01
// The shading of bounce 0's hits and the whole of bounce 1 in one launch (LDS-staged one-light scenes whose
// bounces fuse, after a lane-group or pixel-major bounce 0): per hit record of bounce 0, k_shade<primary,
// fuse>'s steps (the path's camera ray recomputed from its id, emission, the light's contribution if its
// in-place shadow ray is unoccluded, the continuation), then k_bounce's steps on that continuation, with the
// path's radiance held in a register in between — the same float operations in the same order as the two
// launches, which wrote it to rad[p] and read it back.  Every hit of bounce 0 continues (Russian roulette
// starts after bounce 2), so the lanes stay as full as k_shade's.  Input: the hit records of w.segH (the
// bounce-0 trace's); output: the rays of bounce 2 in w.segN / rs[0].  No continuation ray of bounce 1 is
// written or read back, and the k_shade launch and its tail are gone.  
#ifndef SPTR_BOUNCE01_WAVES
#define SPTR_BOUNCE01_WAVES 5
#endif
template <bool kCube, bool kTimed = false>
__global__ void __launch_bounds__(kBlock, SPTR_BOUNCE01_WAVES)
    k_bounce01(SceneView sv, ShadeView sh, FrameView fin, WaveView w, uint32_t nseg_in) {
  if constexpr (kTimed) ktime_begin(w);
  const FrameView f = frame_dyn(fin);
  extern __shared__ float4 lds[];
  uint32_t* s_off = reinterpret_cast<uint32_t*>(lds + sv.lds_bytes / 16u);
  __shared__ DevMaterial smat[32];
  __shared__ uint32_t s_cnt_n, s_rays, s_traced;
  __shared__ LdsStack s_stack;
  const uint32_t nm = stage_materials(sh, smat);
  if (threadIdx.x == 0) s_cnt_n = s_rays = s_traced = 0u;
  const Staged sc = stage_scene<true>(sv, lds);
  uint32_t per_in = 0u;
  const uint32_t n = seg_scan(w.segH, nseg_in, s_off, per_in);
  const RayStream rout = w.rs[0];
  const bool last1 = 1u >= f.max_depth, last2 = 2u >= f.max_depth;
  const ImageDiv idiv = image_div(f);
  Visits vc;
  uint32_t rays = 0u, traced = 0u;
  const Sched sd = block_sched(n);
  for (uint32_t base = sd.first; base < sd.end; base += sd.step) {
    const uint32_t i = base + threadIdx.x;
    bool cont = false, active = i < n;
    uint32_t p = 0u, rng = 0u;
    vec3 thr = v3(1.0f, 1.0f, 1.0f), radv = v3(0.0f, 0.0f, 0.0f), ro, rd;
    if (active) {  // bounce 0's shading (k_shade<true, true>)
      uint3 h;
      w.hrec.get(seg_slot(s_off, nseg_in, per_in, i), h.x, h.y, h.z);
      p = h.x;
      Primary pr;
      primary_path(f, idiv, p, pr);
      rng = pr.rng;
      if (sh.debug_mode == 1) {
        radv = v3(1.0f, 1.0f, 1.0f);
        active = false;
      } else {
        const Surface sf = surface_at(sv, sh, smat, nm, f.cam_pos, pr.d, __uint_as_float(h.y), h.z);
        const vec3 emission = v3(sf.m.emission[0], sf.m.emission[1], sf.m.emission[2]);
        if (dot(emission, emission) > 0.0f) radv = radv + thr * emission;
        vec3 so, ldir, contrib;
        float stfar = 0.0f;
        const bool lit = light_faces(sh.lights[0], sf) && light_term(sh.lights[0], sf, -pr.d, thr, so, ldir, stfar, contrib);
        active = continue_path(sf, pr.d, 0u, thr, rng, ro, rd) && !last1;
        if (lit) {
          uint32_t sref = kNoHit;
          ++rays;
          if (!traverse_w<false, true, false>(sc, sv, make_ray(so, ldir), 1e-4f, stfar, sref, vc, s_stack)) radv = radv + contrib;
        }
      }
    }
    bool lit = false;
    vec3 no, nd, so, ldir, contrib;
    float stfar = 0.0f;
    if (active) {  // bounce 1 (k_bounce, depth 1): radv holds what rad[p] would
      ++traced;
      float tfar = __builtin_huge_valf();
      uint32_t ref = kNoHit;
      if (!traverse_w<false, false, false>(sc, sv, make_ray(ro, rd), 0.0f, tfar, ref, vc, s_stack)) {
        radv = radv + thr * env_color<kCube>(sh.env, renormalized_again(rd));
      } else {
        const Surface sf = surface_at(sv, sh, smat, nm, ro, rd, tfar, ref);
        const vec3 emission = v3(sf.m.emission[0], sf.m.emission[1], sf.m.emission[2]);
        if (dot(emission, emission) > 0.0f) radv = radv + thr * emission;
        if (light_faces(sh.lights[0], sf)) lit = light_term(sh.lights[0], sf, -rd, thr, so, ldir, stfar, contrib);
        cont = continue_path(sf, rd, 1u, thr, rng, no, nd) && !last2;
      }
    }
    const uint32_t jn = block_append(&s_cnt_n, cont);
    if (cont && sd.seg0 + jn >= w.seg_cap) {
      cont = false;
      w.tot[kTotOverflow] = 1ull;  // cannot happen (ensure_wave slack); reported, never written
    }
    if (cont) {
      rout.o[sd.seg0 + jn] = f4(no, __uint_as_float(rng));
      rout.d[sd.seg0 + jn] = f4(nd, __uint_as_float(p));
      rout.thr[sd.seg0 + jn] = f4(thr, 0.0f);
    }
    if (lit) {
      uint32_t sref = kNoHit;
      ++rays;
      if (!traverse_w<false, true, false>(sc, sv, make_ray(so, ldir), 1e-4f, stfar, sref, vc, s_stack)) radv = radv + contrib;
    }
    if (i < n) w.rad[p] = f4(radv, 0.0f);
  }
  for (int off = 32; off > 0; off >>= 1) {
    rays += __shfl_xor(rays, off);
    traced += __shfl_xor(traced, off);
  }
  if (lane_id() == 0u) {
    atomicAdd(&s_rays, rays);
    atomicAdd(&s_traced, traced);
  }
  report_stack(vc, w.tot);
  __syncthreads();
  if (threadIdx.x == 0) {
    w.segN.cnt[logical_block()] = s_cnt_n;
    w.bstat[blockIdx.x] += s_rays;
    if (blockIdx.x == 0) *w.segN.per = sd.per;
    atomicAdd(&w.tot[kTotClosest], (unsigned long long)s_traced);
    atomicAdd(&w.tot[kTotTracedF], (unsigned long long)s_traced);
    atomicAdd(&w.tot[kTotTracedD + 1], (unsigned long long)s_traced);
  }
  if constexpr (kTimed) ktime_end(w);
}

// --------------------------------------------------------------------------------- k_shadow
// One thread per shadow record: any-hit test of each of its light tasks in light order; the
// unoccluded contributions are added to rad[p] (Light::isOccluded, Light.cpp:21-40).  Any-hit
// queries issued are tallied per block (bstat) and reduced by k_accum: no global atomics.
template <bool kLds, bool kCount, bool kW4>
__global__ void __launch_bounds__(kBlock, kW4 ? SPTR_SHADOW4_WAVES : SPTR_SHADOW_WAVES) k_shadow(SceneView sv, ShadeView sh, WaveView w, int depth, uint32_t nseg_in) {
  ktime_begin(w);
  __shared__ KernelStack<kLds> s_stack;
  extern __shared__ float4 lds[];
  __shared__ uint32_t s_rays;
  __shared__ uint32_t s_hist[kCount ? kHistBins : 1];
  uint32_t* s_off = reinterpret_cast<uint32_t*>(lds + (kLds ? sv.lds_bytes / 16u : 0u));
  if (threadIdx.x == 0) s_rays = 0u;
  if (kCount) hist_init(s_hist);
  const Staged sc = stage_scene<kLds>(sv, lds);
  uint32_t per_in = 0u;
  const uint32_t n = seg_scan(w.segS, nseg_in, s_off, per_in);
  const uint32_t ts = w.tstride, L = w.L;
  Visits vc;
  uint32_t rays = 0u;
  const Sched sd = block_sched(n);
  for (uint32_t i = sd.first + threadIdx.x; i < sd.end; i += sd.step) {
    const float4* task = w.stask + (size_t)seg_slot(s_off, nseg_in, per_in, i) * L * ts;
    bool any = false;
    uint32_t p = 0u;
    vec3 rv = v3(0.0f, 0.0f, 0.0f);
    for (uint32_t li = 0; li < L; ++li, task += ts) {
      const float4 c = task[1];
      const uint32_t tag = __float_as_uint(c.w);
      if (tag == 0u) continue;
      p = tag - 1u;
      const float4 a = task[0];
      const vec3 dir = (ts > 2u && sh.lights[li].type != 0)
                           ? xyz(task[2])
                           : v3(sh.lights[li].v[0], sh.lights[li].v[1], sh.lights[li].v[2]);
      const Ray r = make_ray(xyz(a), dir);
      float tfar = a.w;
      uint32_t ref = kNoHit;
      ++rays;
      const uint32_t v0 = vc.nodes;
      const bool occ = traverse_w<kW4, true, kCount>(sc, sv, r, 1e-4f, tfar, ref, vc, s_stack);
      if (kCount) hist_ray(s_hist, vc.nodes - v0);
      if (!occ) {
        if (!any) rv = xyz(w.rad[p]);
        any = true;
        rv = rv + xyz(c);
      }
    }
    if (any) w.rad[p] = f4(rv, 0.0f);
  }
  for (int off = 32; off > 0; off >>= 1) rays += __shfl_xor(rays, off);
  if (lane_id() == 0u) atomicAdd(&s_rays, rays);
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(&w.bstat[blockIdx.x], (unsigned long long)s_rays);  // (k_tail may run beside: shadow carry)
  report_stack(vc, w.tot);
  if (kCount) {
    flush_visits(vc, w.tot, kTotShNodes);
    hist_flush(s_hist, w.tot, kTotHistS);
  }
  ktime_end(w);
}

// k_shadow for wide BVHs traversed from L2/HBM with one light (C3, C5): the any-hit queries of the
// shadow records, with lanes refilled as in k_trace_dyn.  Per record: the same query, and the same
// radiance update when it is unoccluded.
// kQueue (scenes traversed from HBM): the block's tasks are handed out by per-XCD work queues
// (below) instead of the block's static share.  Measured (r02i, profiles/r02i_ab_shadow_queue.txt):
// C5 shadow 4.97 -> 4.78 ms/step; C3 (L2 scene, 0.14-ms launches) 0.82 -> 0.87, so L2 scenes keep
// the static share.
template <bool kCount, bool kQueue>
__global__ void __launch_bounds__(kBlock, SPTR_SHADOW4_WAVES) k_shadow_dyn(SceneView sv, ShadeView sh, WaveView w, int depth,
                                                                           uint32_t nseg_in) {
  ktime_begin(w);
  __shared__ KernelStack<false> s_stack;
  extern __shared__ float4 lds[];
  __shared__ uint32_t s_rays, s_next;
  __shared__ uint32_t s_hist[kCount ? kHistBins : 1];
  uint32_t* s_off = reinterpret_cast<uint32_t*>(lds);
  if (threadIdx.x == 0) s_rays = s_next = 0u;
  if (kCount) hist_init(s_hist);
  constexpr int kKind = kQueue ? kWalkU : kWalkInline;
  const uint32_t ntop = walk_reads_top(kKind) ? sv.num_top4 : 0u;
  const uint4* top = ntop ? stage_top(sv, lds + top_lds_offset(sv, false, false, nseg_in)) : nullptr;
  uint32_t per_in = 0u;
  const uint32_t n = seg_scan(w.segS, nseg_in, s_off, per_in);
  const uint32_t ts = w.tstride;
  Visits vc;
  uint32_t rays = 0u;
  const Sched sd = block_sched(n);
  const uint32_t nb = block_items(sd, n);
  TravStack<kLdsStackG> stack;
  stack.lds = &s_stack.e[0][threadIdx.x];
  bool have = false, done = false;
  uint32_t p = 0u, ref = kNoHit;
  uint32_t v0 = 0u;  // kCount: the lane's node visits when its current query started
  float tfar = 0.0f;
  vec3 contrib;
  Ray r;
  WideWalk wk;
  // kQueue: the per-XCD work queues (xcd_take; counters zeroed by k_shade).  Any block may trace any
  // of its XCD's tasks: they only add to rad[p], there is no output stream.
  XcdQueue xq = xcd_queue(w.work + ((uint32_t)depth % 2u) * 256u, n);
  for (;;) {
    uint32_t item = kNoHit;
    bool more;  // unstarted tasks may remain for this wave
    if constexpr (kQueue) {
      item = xcd_take(xq, !have, nullptr, 0u);
      more = !xq.drained;
    } else {
      const uint32_t k = block_take(&s_next, !have);
      if (!have && k < nb) item = block_item(sd, k);
      more = __ballot(!have && k < nb) != 0ull;
    }
    if (item != kNoHit) {
      const float4* task = w.stask + (size_t)seg_slot(s_off, nseg_in, per_in, item) * ts;
      const float4 c = task[1];
      const uint32_t tag = __float_as_uint(c.w);
      if (tag != 0u) {
        p = tag - 1u;
        contrib = xyz(c);
        const float4 a = task[0];
        const vec3 dir = (ts > 2u && sh.lights[0].type != 0) ? xyz(task[2])
                                                            : v3(sh.lights[0].v[0], sh.lights[0].v[1], sh.lights[0].v[2]);
        r = make_ray(xyz(a), dir);
        tfar = a.w;
        ref = kNoHit;
        ++rays;
        if (kCount) v0 = vc.nodes;
        done = wide_start<true, kCount>(wk, sv.root4, sv.prim_ref, sv.tris, sv.sph, r, 1e-4f, tfar, ref, vc);
        have = true;
      }
    }
    if (__ballot(have) == 0ull) {
      if (!more) break;  // every lane idle and nothing left to take
      continue;          // only unlit tasks taken
    }
    // the unified walk for scenes beyond an XCD's L2 (kQueue): one memory latency per step instead of one
    // per hit leaf (r03x A/B: C5 shadow 2.65 -> 2.12 ms/step); L2-resident scenes keep the leaf-inline
    // walk, whose serial leaf fetches are L2 hits (C3 0.30 inline vs 0.35 unified)
    if (have && !done)
      done = wide_walk<true, kCount, kKind>(wk, stack, sv.nodes4, top, ntop, sv.prim_ref, sv.tris,
                                                                   sv.sph, r, 1e-4f, tfar, ref, vc, kDynSteps);
    if (have && done) {
      if (kCount) hist_ray(s_hist, vc.nodes - v0);
      if (!wk.hit) w.rad[p] = f4(xyz(w.rad[p]) + contrib, 0.0f);
      have = false;
    }
  }
  for (int off = 32; off > 0; off >>= 1) rays += __shfl_xor(rays, off);
  if (lane_id() == 0u) atomicAdd(&s_rays, rays);
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(&w.bstat[blockIdx.x], (unsigned long long)s_rays);  // (k_tail may run beside: shadow carry)
  report_stack(vc, w.tot);
  if (kCount) {
    flush_visits(vc, w.tot, kTotShNodes);
    hist_flush(s_hist, w.tot, kTotHistS);
  }
  ktime_end(w);
}

// --------------------------------------------------------------------------------- k_tail
// The last bounces (depth0 .. max_depth-1), one thread per surviving path carried to its end in
// registers: closest hit -> miss/env, or emission + the shadow rays of the lit lights traced in
// place + continuation -> next bounce.  Late bounces hold few, incoherent rays; as wavefront
// stages they cost three dependent launches per bounce, a path-state round trip through HBM and a
// shadow-task stream.  Per path the operations and the order of the radiance updates are those of
// k_trace + k_shade + k_shadow (wf_pt_cpu.cpp:94-248), so the image does not depend on where the
// wavefront hands over (test_tail_depth_invariance).  Closest-hit and any-hit queries are tallied
// per block (bstat_closest / bstat) and folded by k_accum.
template <bool kLds, bool kW4, bool kCube>
__global__ void __launch_bounds__(kBlock, kLds ? SPTR_TAIL_WAVES_LDS : SPTR_TAIL_WAVES) k_tail(SceneView sv, ShadeView sh, FrameView f, WaveView w, int depth0,
                                                 uint32_t nseg_in) {
  __shared__ KernelStack<kLds> s_stack;
  extern __shared__ float4 lds[];
  __shared__ DevMaterial smat[32];
  __shared__ uint32_t s_rays[2], s_next;
  uint32_t* s_off = reinterpret_cast<uint32_t*>(lds + (kLds ? sv.lds_bytes / 16u : 0u));
  const uint32_t nm = stage_materials(sh, smat);
  if (threadIdx.x < 2u) s_rays[threadIdx.x] = 0u;
  if (threadIdx.x == 0u) s_next = 0u;
  const Staged sc = stage_scene<kLds>(sv, lds);
  // the wide BVH's top levels in LDS (L2/HBM scenes), published by seg_scan's barriers
  const uint32_t ntop = (walk_reads_top(kWalkU) && kW4 && !kLds) ? sv.num_top4 : 0u;
  const uint4* top = ntop ? stage_top(sv, lds + top_lds_offset(sv, kLds, false, nseg_in)) : nullptr;
  uint32_t per_in = 0u;
  const uint32_t n = seg_scan(w.segN, nseg_in, s_off, per_in);
  const RayStream rin = w.rs[depth0 & 1];
  const uint32_t L = w.L, D = f.max_depth;
  Visits vc;
  uint32_t n_closest = 0u, n_shadow = 0u;
  const Sched sd = block_sched(n);
  const uint32_t nb = block_items(sd, n);
  // Lanes are refilled per bounce: a lane whose path ended takes the block's next path, so a wave
  // waits on its slowest lane for one bounce at a time instead of for whole paths.
  bool have = false, loaded = false;  // loaded: rad[p] is read at the first update
  vec3 ro, rd, thr, radv;
  uint32_t rng = 0u, p = 0u, depth = 0u;
  uint32_t cslot = 0u;  // the path's carried shadow task (slot + 1; WaveView::carry_depth), 0: none
  const bool carried = w.carry_depth != kNoHit && (uint32_t)depth0 == w.carry_depth + 1u;
  for (;;) {
    const uint32_t k = block_take(&s_next, !have);
    if (!have && k < nb) {
      const uint32_t id = seg_slot(s_off, nseg_in, per_in, block_item(sd, k));
      const float4 o4 = rin.o[id], d4 = rin.d[id], t4 = rin.thr[id];
      ro = xyz(o4);
      rd = xyz(d4);
      thr = xyz(t4);
      cslot = carried ? __float_as_uint(t4.w) : 0u;
      rng = __float_as_uint(o4.w);
      p = __float_as_uint(d4.w);
      radv = v3(0.0f, 0.0f, 0.0f);
      loaded = false;
      depth = (uint32_t)depth0;
      have = depth < D;
    }
    if (__ballot(have) == 0ull) break;  // every lane idle after a take: the block's paths are done
    if (!have) continue;
    bool fin = true;
    do {  // one bounce of this lane's path; fin = false when it continues
      if (cslot) {  // the shadow ray of the path's previous bounce, handed over by k_shade: first, as k_shadow would
        const float4* task = w.stask + (size_t)(cslot - 1u) * w.tstride;
        const float4 a = task[0], c = task[1];
        const vec3 sdir = (w.tstride > 2u && sh.lights[0].type != 0) ? xyz(task[2])
                                                                    : v3(sh.lights[0].v[0], sh.lights[0].v[1], sh.lights[0].v[2]);
        ++n_shadow;
        float st = a.w;
        uint32_t sref = kNoHit;
        if (!traverse_w_top<kW4, true, false>(sc, sv, top, ntop, make_ray(xyz(a), sdir), 1e-4f, st, sref, vc, s_stack)) {
          if (!loaded) {
            radv = xyz(w.rad[p]);
            loaded = true;
          }
          radv = radv + xyz(c);
        }
        cslot = 0u;
      }
      ++n_closest;
      float tfar = __builtin_huge_valf();
      uint32_t ref = kNoHit;
      const bool hit = traverse_w_top<kW4, false, false>(sc, sv, top, ntop, make_ray(ro, rd), 0.0f, tfar, ref, vc, s_stack);
      if (sh.debug_mode == 1) {  // hit/miss visualisation (never continues past bounce 0)
        radv = hit ? v3(1.0f, 1.0f, 1.0f) : v3(0.0f, 0.0f, 0.0f);
        loaded = true;
        break;
      }
      if (!loaded) {
        radv = xyz(w.rad[p]);
        loaded = true;
      }
      if (!hit) {
        radv = radv + thr * env_color<kCube>(sh.env, renormalized_again(rd));
        break;
      }
      const Surface sf = surface_at(sv, sh, smat, nm, ro, rd, tfar, ref);
      const vec3 emission = v3(sf.m.emission[0], sf.m.emission[1], sf.m.emission[2]);
      if (dot(emission, emission) > 0.0f) radv = radv + thr * emission;
      const vec3 view = -rd;
      for (uint32_t li = 0; li < L; ++li) {
        vec3 so, ldir, contrib;
        float st;
        if (!light_term(sh.lights[li], sf, view, thr, so, ldir, st, contrib)) continue;
        ++n_shadow;
        uint32_t sref = kNoHit;
        if (!traverse_w_top<kW4, true, false>(sc, sv, top, ntop, make_ray(so, ldir), 1e-4f, st, sref, vc, s_stack))
          radv = radv + contrib;
      }
      vec3 no, nd;
      if (!continue_path(sf, rd, depth, thr, rng, no, nd)) break;
      ro = no;
      rd = nd;
      fin = ++depth >= D;
    } while (false);
    if (fin) {
      if (loaded) w.rad[p] = f4(radv, 0.0f);
      have = false;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    n_closest += __shfl_xor(n_closest, off);
    n_shadow += __shfl_xor(n_shadow, off);
  }
  if (lane_id() == 0u) {
    atomicAdd(&s_rays[0], n_closest);
    atomicAdd(&s_rays[1], n_shadow);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // atomics: with the shadow carry k_shadow_dyn of the previous bounce runs beside (same tallies)
    atomicAdd(&w.bstat_closest[blockIdx.x], (unsigned long long)s_rays[0]);
    atomicAdd(&w.bstat[blockIdx.x], (unsigned long long)s_rays[1]);
  }
  report_stack(vc, w.tot);
}

// --------------------------------------------------------------------------------- k_strag
// The paths whose bounce-`depth0` ray k_trace_dyn handed off (WaveView::strag), one thread per path,
// refilled per bounce as in k_tail: the handed-off walk resumes from the state k_trace_dyn saved (the same
// walk form, node order, stack and closest hit so far — kStragRec), then the path is carried to
// its end with k_tail's per-bounce steps — the operations and radiance-update order of k_trace + k_shade
// + k_shadow — so a handed-off path adds exactly what the wavefront stages would have added.  The host
// launches it after the trace and after the shadow launch of the previous bounce (which may still add to
// these paths' radiance) and joins it before the batch's k_accum; no other kernel touches the paths in
// between.  A bounce-0 path starts from zero radiance, as k_shade<primary> does.  The handed-off ray
// itself was counted by its trace launch; the later bounces' closest-hit and the any-hit queries are
// added to the totals here (atomics: k_shadow_dyn may be updating the per-block tallies meanwhile).
#ifndef SPTR_STRAG_WAVES
#define SPTR_STRAG_WAVES SPTR_TAIL_WAVES
#endif
template <bool kW4, bool kCube>
__global__ void __launch_bounds__(kBlock, SPTR_STRAG_WAVES) k_strag(SceneView sv, ShadeView sh, FrameView f, WaveView w,
                                                                    int depth0) {
  __shared__ KernelStack<false> s_stack;
  __shared__ DevMaterial smat[32];
  __shared__ uint32_t s_rays[2], s_next;
  const uint32_t nm = stage_materials(sh, smat);
  if (threadIdx.x < 2u) s_rays[threadIdx.x] = 0u;
  if (threadIdx.x == 0u) s_next = 0u;
  const Staged sc = stage_scene<false>(sv, nullptr);
  extern __shared__ float4 lds[];
  const uint32_t ntop = walk_reads_top(kWalkU) ? sv.num_top4 : 0u;
  const uint4* top = ntop ? stage_top(sv, lds) : nullptr;
  __syncthreads();
  const uint32_t n = min(w.work[kWorkStrag + (uint32_t)depth0 * 32u], w.strag_cap);
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&w.tot[kTotStrag], (unsigned long long)n);
  const float4* in = w.strag + (size_t)depth0 * w.strag_cap * kStragRec;
  TravStack<kLdsStackG> stack;  // the resumed walks' stack (later bounces use traverse_w's own)
  stack.lds = &s_stack.e[0][threadIdx.x];
  WideWalk wk;
  float tfar0 = 0.0f;
  uint32_t ref0 = kNoHit;
  const uint32_t L = w.L, D = f.max_depth;
  Visits vc, vr;  // vr: the resumed walks' visits (the part of the handed-off rays' traversal done here)
  uint32_t n_closest = 0u, n_shadow = 0u;
  const Sched sd = block_sched(n);
  const uint32_t nb = block_items(sd, n);
  bool have = false, loaded = false, first = false;
  vec3 ro, rd, thr, radv;
  uint32_t rng = 0u, p = 0u, depth = 0u;
  for (;;) {
    const uint32_t k = block_take(&s_next, !have);
    if (!have && k < nb) {
      const float4* rec = in + (size_t)block_item(sd, k) * kStragRec;
      const float4 o4 = rec[0], d4 = rec[1], t4 = rec[2], w4 = rec[3];
      wk.cur = __float_as_uint(w4.x);
      wk.sp = (int)(__float_as_uint(w4.y) & 0xFFFFu);
      wk.hit = (__float_as_uint(w4.y) >> 16) != 0u;
      ref0 = __float_as_uint(w4.z);
      tfar0 = w4.w;
      const uint32_t* st = reinterpret_cast<const uint32_t*>(rec + 4);
      for (int q = 0; q < wk.sp; ++q) stack.put(q, st[q]);
      ro = xyz(o4);
      rd = xyz(d4);
      thr = xyz(t4);
      rng = __float_as_uint(o4.w);
      p = __float_as_uint(d4.w);
      depth = __float_as_uint(t4.w);
      loaded = depth == 0u;  // bounce 0: the path's radiance starts at zero (rad[p] holds an older batch's)
      radv = v3(0.0f, 0.0f, 0.0f);
      first = true;
      have = depth < D;
    }
    if (__ballot(have) == 0ull) break;
    if (!have) continue;
    bool fin = true;
    do {
      float tfar = __builtin_huge_valf();
      uint32_t ref = kNoHit;
      bool hit;
      if (first) {  // the handed-off ray: its walk resumes where k_trace_dyn left it (the same walk kind)
        tfar = tfar0;
        ref = ref0;
        (void)walk_steps<false, true, kW4>(wk, stack, sc, top, ntop, make_ray(ro, rd), 0.0f,
                                                                  tfar, ref, vr, 0x7FFFFFFF);
        hit = wk.hit;
      } else {
        ++n_closest;
        hit = traverse_w_top<kW4, false, false>(sc, sv, top, ntop, make_ray(ro, rd), 0.0f, tfar, ref, vc, s_stack);
      }
      first = false;
      if (sh.debug_mode == 1) {
        radv = hit ? v3(1.0f, 1.0f, 1.0f) : v3(0.0f, 0.0f, 0.0f);
        loaded = true;
        break;
      }
      if (!loaded) {
        radv = xyz(w.rad[p]);
        loaded = true;
      }
      if (!hit) {
        radv = radv + thr * env_color<kCube>(sh.env, renormalized_again(rd));
        break;
      }
      const Surface sf = surface_at(sv, sh, smat, nm, ro, rd, tfar, ref);
      const vec3 emission = v3(sf.m.emission[0], sf.m.emission[1], sf.m.emission[2]);
      if (dot(emission, emission) > 0.0f) radv = radv + thr * emission;
      const vec3 view = -rd;
      for (uint32_t li = 0; li < L; ++li) {
        vec3 so, ldir, contrib;
        float st;
        if (!light_term(sh.lights[li], sf, view, thr, so, ldir, st, contrib)) continue;
        ++n_shadow;
        uint32_t sref = kNoHit;
        if (!traverse_w_top<kW4, true, false>(sc, sv, top, ntop, make_ray(so, ldir), 1e-4f, st, sref, vc, s_stack))
          radv = radv + contrib;
      }
      vec3 no, nd;
      if (!continue_path(sf, rd, depth, thr, rng, no, nd)) break;
      ro = no;
      rd = nd;
      fin = ++depth >= D;
    } while (false);
    if (fin) {
      if (loaded) w.rad[p] = f4(radv, 0.0f);
      have = false;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    n_closest += __shfl_xor(n_closest, off);
    n_shadow += __shfl_xor(n_shadow, off);
  }
  if (lane_id() == 0u) {
    atomicAdd(&s_rays[0], n_closest);
    atomicAdd(&s_rays[1], n_shadow);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&w.tot[kTotClosest], (unsigned long long)s_rays[0]);
    atomicAdd(&w.tot[kTotShadow], (unsigned long long)s_rays[1]);
  }
  flush_visits(vr, w.tot, kTotStragNodes);
  report_stack(vc, w.tot);
  report_stack(vr, w.tot);
}

// --------------------------------------------------------------------------------- k_sky
// Path-major bounce 0 with a cull mask (f.sky_fold): the culled pixels' camera rays all miss, so
// their samples are nothing but raygen + environment.  One thread per culled pixel sums them into
// accum in sample order — the adds k_trace (rad[p] = 0 + 1 * env) and k_accum would make, in the
// same order — and marks the pixel complete (resume slot k); k_trace skips those paths and writes no
// radiance for them, k_accum no longer reads it.  Other pixels get resume slot 0.
// a culled valid pixel of a path-major batch with sky_fold: k_sky sums its samples, k_accum none
__device__ __forceinline__ bool sky_pixel(const FrameView& f, uint32_t l, int& x, int& y) {
  return pixel_culled(f, l) && local_pixel(f, l, x, y);
}
// (r04 A/B: lane groups of 8 per culled pixel fed by per-XCD queues over a list of the culled pixels
// cost C3 0.6 ms: the fold's shuffles and the queue grabs outweigh the idle lanes of mixed waves.)
// k_sky's occupancy beside the launch chain (kCapped): it claims registers up to v<SPTR_SKY_VGPR> (128
// of 512 per lane: at most 4 of its waves per SIMD), so that the latency-bound launches beside it keep
// wave slots.  Its 43 registers admit 8 waves/SIMD, and a grid that wide took every slot from C3's
// bounce chain, which then ran after the sky rather than beside it.  r05za: C3 3.54-3.55 -> 3.31-3.33
// ms/step (5 waves 3.48, 3 waves 3.50, 6 waves 3.50-3.57); C5, whose sky runs beside the tail, 7.20-7.28
// either way.  (r05zc/zd: a capped launch beside the chain plus a full-occupancy one after it, sharing
// per-XCD pixel queues, 3.38-3.39: a 64-pixel chunk is ~0.3 ms of one wave's work, so the two launches'
// last chunks end late.)  Uncapped when nothing runs beside it.
#ifndef SPTR_SKY_VGPR
#define SPTR_SKY_VGPR 127
#endif
template <bool kCube, bool kCapped>
__global__ void __launch_bounds__(kBlock) k_sky(EnvView sh, FrameView fin) {
#if SPTR_SKY_VGPR
  if constexpr (kCapped) asm volatile("; k_sky occupancy cap" ::: "v" SPTR_STR(SPTR_SKY_VGPR));
#endif
  const FrameView f = frame_dyn(fin);
  const ImageDiv idiv = image_div(f);
  for (uint32_t l = blockIdx.x * blockDim.x + threadIdx.x; l < f.P; l += grid_threads()) {
    int x, y;
    // only the culled pixels' words: k_accum sums the others (sky_pixel)
    if (sky_pixel(f, l, x, y)) {
      vec3 a = v3(0.0f, 0.0f, 0.0f);
      if (!f.reset) a = xyz(f.accum[l]);
      const uint32_t ps = (uint32_t)(y * f.W + x);
      auto sample = [&](uint32_t smp) {
        Primary pr;
        primary_at(f, idiv, x, y, ps, f.acc0 + smp, pr);
        vec3 rv = v3(0.0f, 0.0f, 0.0f);
        if (sh.debug_mode != 1) rv = v3(0.0f, 0.0f, 0.0f) + v3(1.0f, 1.0f, 1.0f) * env_color<kCube>(sh, renormalized_again(pr.d));
        return rv;
      };
      // kSkyIlp independent samples (their environment fetches in flight together), then their adds
      // in sample order
      constexpr uint32_t kSkyIlp = SPTR_SKY_ILP;
      uint32_t smp = 0;
      for (; smp + kSkyIlp <= f.k; smp += kSkyIlp) {
        vec3 rv[kSkyIlp];
#pragma unroll
        for (uint32_t j = 0; j < kSkyIlp; ++j) rv[j] = sample(smp + j);
#pragma unroll
        for (uint32_t j = 0; j < kSkyIlp; ++j) a = a + rv[j];
      }
      for (; smp < f.k; ++smp) a = a + sample(smp);
      f.accum[l] = make_float4(a.x, a.y, a.z, __uint_as_float(f.k));
    }
  }
}

// EnvironmentManager::acesToneMapping (src/EnvironmentManager.cpp:63-74)
__device__ __forceinline__ vec3 aces(vec3 c) {
  return clamp_g((c * (2.51f * c + 0.03f)) / (c * (2.43f * c + 0.59f) + 0.14f), 0.0f, 1.0f);
}
__device__ __forceinline__ uint32_t pack_rgba(vec3 c) {
  const uint32_t r = (uint32_t)(unsigned char)(c.x * 255.0f);
  const uint32_t gg = (uint32_t)(unsigned char)(c.y * 255.0f);
  const uint32_t b = (uint32_t)(unsigned char)(c.z * 255.0f);
  return r | (gg << 8) | (b << 16) | 0xFF000000u;
}
// Wavefront tile task resolve (GLRenderer.cpp:411-431): mean -> ACES -> gamma -> clamp -> 8 bit
__device__ __forceinline__ uint32_t resolve_rgba(vec3 acc, uint32_t n) {
  vec3 c = aces(acc / float(n));
  c = v3(gamma_pow(c.x), gamma_pow(c.y), gamma_pow(c.z));
  return pack_rgba(clamp_g(c, 0.0f, 1.0f));
}
// PathTracer::renderTileTask resolve (PathTracer.cpp:364-384): the frames were tonemapped as they
// were traced, so the display value is the clamped mean
__device__ __forceinline__ uint32_t resolve_rgba_pt(vec3 acc, uint32_t n) {
  return pack_rgba(clamp_g(acc / float(n), 0.0f, 1.0f));
}

// OptiX __raygen__resolve (device_programs.cu:854-899): accum / w (by reciprocal) -> exposure 2.2
// -> Reinhard -> gamma 2.2 -> clamp -> 8 bit
__device__ __forceinline__ uint32_t resolve_rgba_optix(float4 a) {
  const float inv = (a.w > 0.0f) ? (1.0f / a.w) : 0.0f;
  vec3 c = v3(fmaxf(a.x * inv, 0.0f), fmaxf(a.y * inv, 0.0f), fmaxf(a.z * inv, 0.0f));
  c = c * 2.2f;
  c = v3(c.x / (1.0f + c.x), c.y / (1.0f + c.y), c.z / (1.0f + c.z));
  const float g = 1.0f / 2.2f;
  c = v3(powf(c.x, g), powf(c.y, g), powf(c.z, g));
  return pack_rgba(v3(fminf(fmaxf(c.x, 0.0f), 1.0f), fminf(fmaxf(c.y, 0.0f), 1.0f), fminf(fmaxf(c.z, 0.0f), 1.0f)));
}

// --------------------------------------------------------------------------------- k_accum / resolve
// Per-pixel sample sums in sample order.  A folding bounce 0 (f.pixel_major: thread or lane group
// per pixel; f.sky_fold: k_sky for the culled pixels of a path-major bounce 0) began them:
// accum[l] holds the sum up to (excluding) slot accum[l].w, the pixel's first primary hit in this
// batch, and all-sky pixels are already complete (slot = k) and are not touched.  Otherwise every
// slot's radiance is summed here, onto the previous batches' sum unless the batch resets it.
// kResolve (the last batch of a wavefront call that resolves): each thread also resolves its pixel
// from the sum it holds, as k_resolve would next (one launch and one accum re-read less).
template <bool kResolve>
__global__ void __launch_bounds__(kBlock) k_accum(FrameView fin, WaveView w, float4* accum, uint32_t* tiles,
                                                  uint8_t* image) {
  const FrameView f = frame_dyn(fin);
  const uint32_t n_total = f.dyn ? f.dyn[2] : 0u;  // total frames of the accumulation (kResolve)
  // the next batch's bounce-0 trace (k_trace_dyn) takes its work from fresh queues
  if (blockIdx.x == 0) {
    if (threadIdx.x < kXcds) w.work[kWorkTraceQueue + threadIdx.x * 32u] = 0u;
    // the straggler counts of this batch's bounces (their k_strag launches were joined before this one)
    if (threadIdx.x >= 128 && threadIdx.x < 128 + kStragBounces) w.work[kWorkStrag + (threadIdx.x - 128) * 32u] = 0u;
  }
  for (uint32_t l = blockIdx.x * blockDim.x + threadIdx.x; l < f.P; l += grid_threads()) {
    uint32_t s0 = 0u;
    vec3 a = v3(0.0f, 0.0f, 0.0f);
    bool sum = true;
    if (f.pixel_major) {
      const float4 a4 = accum[l];
      s0 = __float_as_uint(a4.w);
      a = xyz(a4);
      sum = s0 < f.k;
      if (!kResolve && !sum) continue;
    } else if (f.sky_fold) {  // k_sky summed the culled pixels; the others start from the previous batch
      int x, y;
      sum = !sky_pixel(f, l, x, y);
      if (!kResolve && !sum) continue;
      if (!sum || !f.reset) a = xyz(accum[l]);
    } else if (!f.reset) {
      a = xyz(accum[l]);
    }
    if (sum) {
    // sample order is the reference's accumulation order (one add per frame); the unroll only
    // lets eight sample loads be in flight per thread before the first add
    const float4* src = w.rad + l;
    uint32_t s = s0;
    for (; s + 8u <= f.k; s += 8u) {
      float4 v[8];
#pragma unroll
      for (uint32_t j = 0; j < 8u; ++j) v[j] = src[(size_t)(s + j) * f.P];
#pragma unroll
      for (uint32_t j = 0; j < 8u; ++j) a = a + xyz(v[j]);
    }
    for (; s < f.k; ++s) a = a + xyz(w.rad[(size_t)s * f.P + l]);
    accum[l] = f4(a, __uint_as_float(f.k));
    }
    if (kResolve) {
      int x, y;
      const bool valid = local_pixel(f, l, x, y);
      const uint32_t px = valid ? resolve_rgba(a, n_total) : 0u;
      tiles[l] = px;
      if (valid && image) {
        uint8_t* o = image + ((size_t)y * f.W + x) * 3;
        o[0] = (uint8_t)(px & 0xFF);
        o[1] = (uint8_t)((px >> 8) & 0xFF);
        o[2] = (uint8_t)((px >> 16) & 0xFF);
      }
    }
  }
  if (blockIdx.x == 0) {  // fold the per-block query tallies of this batch into the totals
    unsigned long long s = 0ull, c = 0ull;
    for (uint32_t b = threadIdx.x; b < kMaxSegs; b += kBlock) {
      s += w.bstat[b];
      c += w.bstat_closest[b];
      w.bstat[b] = 0ull;
      w.bstat_closest[b] = 0ull;
    }
    for (int off = 32; off > 0; off >>= 1) {
      s += __shfl_xor(s, off);
      c += __shfl_xor(c, off);
    }
    if (lane_id() == 0u) {
      atomicAdd(&w.tot[kTotShadow], s);
      atomicAdd(&w.tot[kTotClosest], c);
      atomicAdd(&w.tot[kTotTail], c);
    }
  }
  ktime_end(w);  // (w.tslot: the end of an untimed call's span, whose start k_frame_dyn stored)
}

__global__ void __launch_bounds__(kBlock) k_resolve(FrameView f, const float4* accum, uint32_t n_arg, uint32_t* tiles,
                                                    uint8_t* image) {
  const uint32_t n = f.dyn ? f.dyn[2] : n_arg;  // total frames of the accumulation
  for (uint32_t l = blockIdx.x * blockDim.x + threadIdx.x; l < f.P; l += grid_threads()) {
    int x, y;
    const bool valid = local_pixel(f, l, x, y);
    uint32_t px = 0u;
    if (valid) {
      if (f.integrator == SPTR_INTEGRATOR_PATHTRACER) px = resolve_rgba_pt(xyz(accum[l]), n);
      else if (f.integrator == SPTR_INTEGRATOR_OPTIX) px = resolve_rgba_optix(accum[l]);
      else px = resolve_rgba(xyz(accum[l]), n);
    }
    tiles[l] = px;
    if (valid && image) {
      uint8_t* o = image + ((size_t)y * f.W + x) * 3;
      o[0] = (uint8_t)(px & 0xFF);
      o[1] = (uint8_t)((px >> 8) & 0xFF);
      o[2] = (uint8_t)((px >> 16) & 0xFF);
    }
  }
}

__global__ void __launch_bounds__(kBlock) k_unpack(const uint32_t* g, int G, uint32_t tpr, int W, int H, int ntx,
                                                   uint8_t* rgb) {
  const uint32_t N = (uint32_t)W * (uint32_t)H;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += grid_threads()) {
    const int x = (int)(i % (uint32_t)W), y = (int)(i / (uint32_t)W);
    uint32_t r, l;
    pixel_shard(W, G, x, y, r, l);
    const uint32_t px = g[(size_t)r * tpr * kTilePixels + l];
    rgb[(size_t)i * 3 + 0] = (uint8_t)(px & 0xFF);
    rgb[(size_t)i * 3 + 1] = (uint8_t)((px >> 8) & 0xFF);
    rgb[(size_t)i * 3 + 2] = (uint8_t)((px >> 16) & 0xFF);
  }
}

// --------------------------------------------------------------------------------- k_pathtracer
// The reference's default CPU integrator, PathTracer (src/PathTracer.cpp:113-391), for
// SPTR_INTEGRATOR_PATHTRACER.  Differences from the wavefront integrator, all reproduced:
//   * camera ray through the pixel corner, u = x/W, v = y/H, no jitter (renderTileTask :351-355);
//   * intersection tnear 1e-4 (intersectRay :82-100) and normal = normalize(Ng) (:131-137);
//   * continuation origins offset by 1e-4 * max(1, |P|inf) (calculateSafeRayOrigin :103-111);
//     reflection, refraction and scatter directions are not renormalised;
//   * glass: eta from cosine > 0, refract() with sin_t2 >= 1 as total internal reflection
//     (:176-206, :396-406); Fresnel pow((1 - c), 5.0f) (:391-395);
//   * diffuse: cosineHemisphereSample (:59-75, y-up local frame, phi in double), Russian roulette
//     at every bounce (:208-219);
//   * samples_per_frame samples per frame averaged, then ACES and gamma (traceRay :280-303); the
//     tonemapped frames are what accumulates.
// The recursion color = emission + direct + weight * trace(depth - 1) is evaluated forward with a
// path throughput (same terms and estimator; the rounding of the outer sums differs).  RNG: the
// reference's thread-local mt19937(random_device) is not reproducible; each (pixel, frame, sample)
// here draws from its own wang-hash stream (pt_seed), which the oracle restates.
__device__ __forceinline__ uint32_t pt_seed(uint32_t ps, uint32_t acc, uint32_t s) {
  return wang_hash(wang_hash(ps ^ (acc * 9781u)) ^ (s * 0x9E3779B9u + 0x68E31DA4u));
}

template <bool kW4, bool kCube, int N>
__device__ vec3 pt_path(const Staged& sc, const SceneView& sv, const ShadeView& sh, const DevMaterial* smat, uint32_t nm,
                        vec3 o, vec3 d, uint32_t depth, uint32_t& rng, Visits& vc, LdsStackN<N>& ls, uint32_t& n_closest,
                        uint32_t& n_shadow) {
  vec3 rad = v3(0.0f, 0.0f, 0.0f), thr = v3(1.0f, 1.0f, 1.0f);
  for (uint32_t lvl = 0; lvl < depth; ++lvl) {
    ++n_closest;
    float t = __builtin_huge_valf();
    uint32_t ref = kNoHit;
    if (!traverse_w<kW4, false, false>(sc, sv, make_ray(o, d), 1e-4f, t, ref, vc, ls)) {
      rad = rad + thr * env_color<kCube>(sh.env, renormalize_dir(d));
      break;
    }
    const vec3 P = o + t * d;
    const uint32_t idx = ref & kIndexMask;
    vec3 ng;
    uint32_t mid;
    if (ref & kSphereBit) {
      const float4 c = sc.sph[idx];
      ng = v3((P.x - c.x) / c.w, (P.y - c.y) / c.w, (P.z - c.z) / c.w);
      mid = sh.geom_mat[sv.sph_geom[idx]];
    } else {
      const float4 c = sc.tris[3 * idx + 2];
      ng = v3(c.y, c.z, c.w);
      mid = sh.geom_mat[sv.tri_geom[idx]];
    }
    vec3 n = normalize(ng);
    if (dot(n, d) > 0.0f) n = -n;
    const DevMaterial& m = (mid < nm) ? smat[mid] : sh.mats[mid];
    const vec3 albedo = v3(m.albedo[0], m.albedo[1], m.albedo[2]);
    vec3 color = v3(m.emission[0], m.emission[1], m.emission[2]);
    const vec3 view = -d;
    for (uint32_t li = 0; li < sh.num_lights; ++li) {
      vec3 ldir, Li;
      float ldist;
      light_at(sh.lights[li], P, ldir, ldist, Li);
      const float cs = fmax_g(dot(n, ldir), 0.0f);
      if (!(cs > 0.0f)) continue;
      // Light::isOccluded (Light.cpp:16-40)
      const float eps = 1e-4f * fmax_g(1.0f, fmax_g(fmax_g(fabsf(P.x), fabsf(P.y)), fabsf(P.z)));
      float st = ldist - 1e-4f;
      uint32_t sref = kNoHit;
      ++n_shadow;
      if (!traverse_w<kW4, true, false>(sc, sv, make_ray(P + n * eps, ldir), 1e-4f, st, sref, vc, ls))
        color = color + eval_brdf(m, n, view, ldir) * Li * cs;
    }
    rad = rad + thr * color;
    const float eps = 1e-4f * fmax_g(1.0f, fmax_g(fmax_g(fabsf(P.x), fabsf(P.y)), fabsf(P.z)));
    if (m.metallic > 0.5f) {
      d = reflect(d, n);
      o = P + n * eps;
      thr = (thr * albedo) * m.metallic;
      continue;
    }
    if (m.metallic < 0.1f && m.ior > 1.3f) {
      const float ior = m.ior;
      const float cosine = -dot(d, n);
      const float eta = cosine > 0.0f ? (1.0f / ior) : ior;
      const float tr = clamp_g((ior - 1.0f) / 0.7f, 0.0f, 0.95f);
      float r0 = (1.0f - ior) / (1.0f + ior);
      r0 = r0 * r0;
      const float fres = r0 + (1.0f - r0) * pow5(1.0f - fabsf(cosine));
      if (rand01(rng) < fres) {
        d = reflect(d, n);
        o = P + n * eps;
        thr = thr * (1.0f - tr);
        continue;
      }
      // PathTracer::refract (PathTracer.cpp:396-406)
      const float cos_i = -dot(d, n);
      const float sin_t2 = eta * eta * (1.0f - cos_i * cos_i);
      vec3 refr = v3(0.0f, 0.0f, 0.0f);
      if (!(sin_t2 >= 1.0f)) refr = eta * d + (eta * cos_i - sqrtf(1.0f - sin_t2)) * n;
      if (dot(refr, refr) > 0.0f) {
        o = P - n * eps;
        d = refr;
        thr = thr * tr;
      } else {
        d = reflect(d, n);
        o = P + n * eps;
      }
      continue;
    }
    // cosineHemisphereSample (PathTracer.cpp:59-75)
    const float r1 = rand01(rng);
    const float r2 = rand01(rng);
    const float cos_t = sqrtf(r1), sin_t = sqrtf(1.0f - r1);
    const float phi = (float)(2.0 * 3.14159265358979323846 * (double)r2);
    const vec3 sd = v3(sin_t * cosf(phi), cos_t, sin_t * sinf(phi));
    const vec3 up = (fabsf(n.x) < 0.9f) ? v3(1.0f, 0.0f, 0.0f) : v3(0.0f, 1.0f, 0.0f);
    const vec3 tg = normalize_dir(cross(up, n));
    const vec3 bt = cross(n, tg);
    const vec3 scatter = tg * sd.x + n * sd.y + bt * sd.z;
    o = P + n * eps;
    const float surv = fmax_g(fmax_g(albedo.x, albedo.y), albedo.z);
    if (!(rand01(rng) < surv)) break;
    thr = (thr * albedo) / surv;
    d = scatter;
  }
  return rad;
}

// Thread per local pixel: the batch's k frames in order, samples_per_frame paths each; accum.xyz
// += the frame's tonemapped colour (the reference's accumulation_buffer, GLRenderer's
// m_accumulated_samples frames).
template <bool kLds, bool kW4, bool kCube>
__global__ void __launch_bounds__(kBlock, SPTR_PT_WAVES) k_pathtracer(SceneView sv, ShadeView sh, FrameView fin, WaveView w) {
  const FrameView f = frame_dyn(fin);
  __shared__ KernelStack<kLds> s_stack;
  extern __shared__ float4 lds[];
  __shared__ DevMaterial smat[32];
  const uint32_t nm = stage_materials(sh, smat);
  const Staged sc = stage_scene<kLds>(sv, lds);
  __syncthreads();
  const ImageDiv idiv = image_div(f);
  Visits vc;
  uint32_t n_closest = 0u, n_shadow = 0u;
  const Sched sd = block_sched(f.P);
  for (uint32_t l = sd.first + threadIdx.x; l < sd.end; l += sd.step) {
    int x = 0, y = 0;
    if (!local_pixel(f, l, x, y)) continue;
    const uint32_t ps = (uint32_t)(y * f.W + x);
    // renderTileTask: u = x / W, v = y / H (no +0.5, no jitter); Camera::getRayDirection
    const vec3 dir = camera_dir(f, div_nrm(float(x), idiv.w), div_nrm(float(y), idiv.h));
    vec3 acc = f.reset ? v3(0.0f, 0.0f, 0.0f) : xyz(f.accum[l]);
    for (uint32_t fr = 0; fr < f.k; ++fr) {
      const uint32_t accn = f.acc0 + fr;
      vec3 c = v3(0.0f, 0.0f, 0.0f);
      for (uint32_t s = 0; s < f.spf; ++s) {
        uint32_t rng = pt_seed(ps, accn, s);
        c = c + pt_path<kW4, kCube>(sc, sv, sh, smat, nm, f.cam_pos, dir, f.max_depth, rng, vc, s_stack, n_closest,
                                    n_shadow);
      }
      c = c / float(f.spf);
      c = aces(c);
      const float g = 1.0f / 2.2f;
      c = v3(powf(c.x, g), powf(c.y, g), powf(c.z, g));
      acc = acc + c;
    }
    f.accum[l] = make_float4(acc.x, acc.y, acc.z, 0.0f);
  }
  unsigned long long a = n_closest, b = n_shadow;
  for (int off = 32; off > 0; off >>= 1) {
    a += __shfl_xor(a, off);
    b += __shfl_xor(b, off);
  }
  if (lane_id() == 0u) {
    atomicAdd(&w.tot[kTotClosest], a);
    atomicAdd(&w.tot[kTotShadow], b);
  }
  report_stack(vc, w.tot);
}

// --------------------------------------------------------------------------------- k_optix
// SPTR_INTEGRATOR_OPTIX: the shading of the reference's OptiX wavefront programs
// (src/optix/device_programs.cu), restated path per thread — one path per pixel per frame, its
// contributions added to accum in bounce order (the same order the reference's per-bounce
// atomicAdds take for a pixel, since a pixel has one path per frame):
//   raygen  computePrimaryRay / __raygen__gen_primary (:220-274): pixel centre, cam_u/v/w from
//           OptixBackend::render (OptixBackend.cpp:1609-1620), seed wang_hash((pixel+1) ^ (frame*9781+1))
//   trace   tmin 1e-3, tmax 1e16 (:297-309); closest-hit Ng = normalize(cross(v1-v0, v2-v0)) or
//           normalize(P - C) (:761-820)
//   shade   (:315-690) miss -> sky (w += 1); depth cap -> normal visualisation (w += 1); direct sun
//           light without a shadow ray (GGX spec for metals, Lambert otherwise, none for
//           dielectrics); delta dielectric; GGX-sampled metal with its fallbacks; cosine diffuse
// The environment is the procedural sky (or the CPU cubemap sampling when a cubemap is set: the
// reference's equirect texture fetch is not restated).  CUDA's approximate rsqrtf / sincosf /
// __powf-class functions are replaced by correctly rounded normalize and the library sin/cos/pow.
__device__ __forceinline__ vec3 ox_nrm(vec3 v) {  // f3_normalize (rsqrtf -> correctly rounded)
  return v * inv_len(dot(v, v));
}
__device__ __forceinline__ void ox_onb(vec3 n, vec3& t, vec3& b) {  // make_onb (:213-218)
  const vec3 up = (fabsf(n.z) < 0.999f) ? v3(0.0f, 0.0f, 1.0f) : v3(1.0f, 0.0f, 0.0f);
  t = ox_nrm(v3(up.y * n.z - up.z * n.y, up.z * n.x - up.x * n.z, up.x * n.y - up.y * n.x));
  b = v3(n.y * t.z - n.z * t.y, n.z * t.x - n.x * t.z, n.x * t.y - n.y * t.x);
}
__device__ __forceinline__ vec3 ox_cross(vec3 a, vec3 b) {  // f3_cross
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ vec3 ox_reflect(vec3 v, vec3 n) { return v + n * (-2.0f * dot(v, n)); }  // f3_reflect
__device__ __forceinline__ vec3 ox_fresnel(float cosVH, vec3 F0) {  // fresnelSchlick (:170-176)
  const float m = 1.0f - fminf(fmaxf(cosVH, 0.0f), 1.0f);
  const float m2 = m * m;
  const float m5 = m2 * m2 * m;
  return F0 + v3(1.0f - F0.x, 1.0f - F0.y, 1.0f - F0.z) * m5;
}
__device__ __forceinline__ float ox_smith(float cosNL, float cosNV, float alpha) {  // smithGGX (:162-168)
  const float a = alpha + 1.0f;
  const float k = (a * a) * 0.125f;
  return (cosNL / (cosNL * (1.0f - k) + k)) * (cosNV / (cosNV * (1.0f - k) + k));
}
__device__ __forceinline__ vec3 ox_fallback_reflect(vec3 d, vec3 n) {
  vec3 R = ox_reflect(d, n);
  const float l2 = dot(R, R);
  return l2 > 0.0f ? R * inv_len(l2) : n;
}

template <bool kW4, bool kCube, int N>
__device__ void ox_path(const Staged& sc, const SceneView& sv, const ShadeView& sh, const DevMaterial* smat, uint32_t nm,
                        const FrameView& f, vec3 o, vec3 d, uint32_t rng, vec3& acc, Visits& vc, LdsStackN<N>& ls,
                        uint32_t& n_closest) {
  constexpr float kPi = 3.14159265358979323846f;
  vec3 thr = v3(1.0f, 1.0f, 1.0f);
  for (uint32_t depth = 0; depth < f.max_depth; ++depth) {
    ++n_closest;
    float t = 1e16f;
    uint32_t ref = kNoHit;
    if (!traverse_w<kW4, false, false>(sc, sv, make_ray(o, d), 1e-3f, t, ref, vc, ls)) {
      const vec3 c = env_color<kCube>(sh.env, ox_nrm(d));
      acc = acc + v3(c.x * thr.x, c.y * thr.y, c.z * thr.z);
      return;
    }
    const vec3 P = o + d * t;
    const uint32_t idx = ref & kIndexMask;
    vec3 ng;
    uint32_t gid;
    if (ref & kSphereBit) {
      const float4 c = sc.sph[idx];
      ng = ox_nrm(ox_nrm(v3(P.x - c.x, P.y - c.y, P.z - c.z)));
      gid = sv.sph_geom[idx];
    } else {
      const float4 a = sc.tris[3 * idx + 0], b = sc.tris[3 * idx + 1], c = sc.tris[3 * idx + 2];
      const vec3 e1 = -v3(a.w, b.x, b.y), e2 = v3(b.z, b.w, c.x);  // v1 - v0, v2 - v0 (stored e1 = v0 - v1)
      ng = ox_nrm(ox_nrm(ox_cross(e1, e2)));
      gid = sv.tri_geom[idx];
    }
    {  // the shade program renormalises the hit record's normal, (0, 1, 0) if degenerate (:424-433, :443-449)
      const float l2 = dot(ng, ng);
      ng = l2 > 0.0f ? ng * inv_len(l2) : v3(0.0f, 1.0f, 0.0f);
    }
    // material: clamp the id into the table, baseColor clamped to [0, 1] (:343-357)
    uint32_t mid = sh.geom_mat[gid];
    if (mid >= sh.num_mats) mid = sh.num_mats - 1u;
    const DevMaterial& m = (mid < nm) ? smat[mid] : sh.mats[mid];
    const vec3 base = v3(fminf(fmaxf(m.albedo[0], 0.0f), 1.0f), fminf(fmaxf(m.albedo[1], 0.0f), 1.0f),
                         fminf(fmaxf(m.albedo[2], 0.0f), 1.0f));
    const float metallic = m.metallic, rough = m.roughness, ior = m.ior;
    const bool dielectric = m.type == 1;
    const float omm = fminf(fmaxf(1.0f - metallic, 0.0f), 1.0f);
    const vec3 diffuse = base * omm;
    if (depth + 1u >= f.max_depth) {  // depth cap: normal visualisation (:424-440)
      const vec3 nvis = (ng + v3(1.0f, 1.0f, 1.0f)) * 0.5f;
      const vec3 shd = diffuse * nvis;
      acc = acc + v3(shd.x * thr.x, shd.y * thr.y, shd.z * thr.z);
      return;
    }
    const bool entering = dot(d, ng) < 0.0f;
    const vec3 n = entering ? ng : -ng;
    if (f.ox_has_light) {  // direct light, no shadow ray (:457-496)
      const vec3 V = ox_nrm(-d);
      const vec3 L = ox_nrm(-f.ox_light_dir);
      const float NdotL = fmaxf(dot(n, L), 0.0f);
      if (NdotL > 0.0f && !dielectric) {
        vec3 fr = v3(0.0f, 0.0f, 0.0f);
        if (metallic > 0.5f) {
          const float r = fminf(fmaxf(rough, 0.02f), 1.0f);
          const float alpha = r * r;
          const vec3 H = ox_nrm(V + L);
          const float cosNV = fmaxf(dot(n, V), 0.0f), cosNL = NdotL, cosVH = fmaxf(dot(V, H), 0.0f);
          if (cosNV > 0.0f && cosNL > 0.0f) {
            const float cosNH = fmaxf(dot(n, H), 0.0f);
            const float a2 = alpha * alpha;
            const float den = cosNH * cosNH * (a2 - 1.0f) + 1.0f;
            const float D = a2 / (kPi * den * den);
            const float G = ox_smith(cosNL, cosNV, alpha);
            const vec3 F = ox_fresnel(cosVH, base);
            const float dn = fmaxf(4.0f * cosNV * cosNL, 1e-6f);
            fr = F * ((D * G) / dn);
          }
        } else {
          fr = diffuse * (1.0f / kPi);
        }
        const vec3 Li = f.ox_light_rad;
        acc = acc + ((thr * fr) * Li) * NdotL;
      }
    }
    if (dielectric) {  // delta dielectric (:499-543)
      const float xi = rand01(rng);
      const float etaI = entering ? 1.0f : ior, etaT = entering ? ior : 1.0f;
      const float eta = etaI / etaT;
      const float cosI = fminf(fmaxf(-dot(d, n), -1.0f), 1.0f);
      float R0 = (etaT - etaI) / (etaT + etaI);
      R0 = R0 * R0;
      const float mm = 1.0f - fminf(fmaxf(cosI, 0.0f), 1.0f);
      const float Fr = R0 + (1.0f - R0) * (mm * mm * mm * mm * mm);
      // f3_refract (:75-93)
      const float ci = fminf(fmaxf(-dot(n, d), -1.0f), 1.0f);
      const float sin2T = eta * eta * fmaxf(0.0f, 1.0f - ci * ci);
      const bool can = !(sin2T > 1.0f);
      vec3 refr = v3(0.0f, 0.0f, 0.0f);
      if (can) {
        const float cosT = sqrtf(fmaxf(0.0f, 1.0f - sin2T));
        refr = d * eta + n * (eta * ci - cosT);
        const float l2 = dot(refr, refr);
        if (l2 > 0.0f) refr = refr * inv_len(l2);
      }
      vec3 nd = (!can || xi < Fr) ? ox_reflect(d, n) : refr;
      nd = ox_nrm(nd);
      o = P + nd * 1e-3f;
      d = nd;
      continue;
    }
    if (metallic > 0.5f) {  // GGX-sampled metal (:547-666)
      const float r = fminf(fmaxf(rough, 0.02f), 1.0f);
      const float alpha = r * r;
      const vec3 V = ox_nrm(-d);
      const float cosNV_raw = dot(n, V);
      if (cosNV_raw <= 0.0f) {
        d = ox_fallback_reflect(d, n);
        o = P + n * 1e-3f;
        thr = thr * base;
        continue;
      }
      const float u1 = rand01(rng), u2 = rand01(rng);
      // ggx_sample_half_vector (:178-210)
      const float a2 = alpha * alpha;
      const float phi = 6.28318530717958647692f * u1;
      const float den = 1.0f + (a2 - 1.0f) * u2;
      const float cosT = sqrtf(fmaxf(0.0f, (1.0f - u2) / den));
      const float sinT = sqrtf(fmaxf(0.0f, 1.0f - cosT * cosT));
      const float sp = sinf(phi), cp = cosf(phi);
      vec3 tb, bb;
      ox_onb(n, tb, bb);
      vec3 H = tb * (sinT * cp) + bb * (sinT * sp) + n * cosT;
      const float hl2 = dot(H, H);
      H = hl2 > 0.0f ? H * inv_len(hl2) : n;
      const float cosNH_raw = dot(n, H);
      if (cosNH_raw <= 0.0f) {
        d = ox_fallback_reflect(d, n);
        o = P + n * 1e-3f;
        thr = thr * base;
        continue;
      }
      vec3 L = ox_reflect(-V, H);
      const float ll2 = dot(L, L);
      L = ll2 > 0.0f ? L * inv_len(ll2) : n;
      const float cosNL_raw = dot(n, L);
      if (cosNL_raw <= 0.0f) {
        d = ox_fallback_reflect(d, n);
        o = P + n * 1e-3f;
        thr = thr * base;
        continue;
      }
      const float cosNV = fmaxf(cosNV_raw, 1e-6f), cosNL = fmaxf(cosNL_raw, 1e-6f), cosNH = fmaxf(cosNH_raw, 1e-6f);
      const float cosVH = fmaxf(dot(V, H), 0.0f);
      const vec3 F = ox_fresnel(cosVH, base);
      const float G = ox_smith(cosNL, cosNV, alpha);
      float scale = (G * cosVH) / (cosNV * cosNH);
      scale = fminf(scale, 50.0f);
      if (scale < 0.0f) scale = 0.0f;
      o = P + n * 1e-3f;
      d = L;
      thr = thr * (F * scale);
      continue;
    }
    // Lambert, cosine-weighted (:668-689)
    const float u1 = rand01(rng), u2 = rand01(rng);
    const float rr = sqrtf(u1);
    const float phi = 2.0f * 3.14159265358979323846f * u2;
    const float sp = sinf(phi), cp = cosf(phi);
    const vec3 loc = v3(rr * cp, rr * sp, sqrtf(fmaxf(0.0f, 1.0f - u1)));
    vec3 tb, bb;
    ox_onb(n, tb, bb);
    d = ox_nrm(tb * loc.x + bb * loc.y + n * loc.z);
    o = P + n * 1e-3f;
    thr = thr * diffuse;
  }
}

template <bool kLds, bool kW4, bool kCube>
__global__ void __launch_bounds__(kBlock, SPTR_PT_WAVES) k_optix(SceneView sv, ShadeView sh, FrameView fin, WaveView w) {
  const FrameView f = frame_dyn(fin);
  __shared__ KernelStack<kLds> s_stack;
  extern __shared__ float4 lds[];
  __shared__ DevMaterial smat[32];
  const uint32_t nm = stage_materials(sh, smat);
  const Staged sc = stage_scene<kLds>(sv, lds);
  __syncthreads();
  const ImageDiv idiv = image_div(f);
  Visits vc;
  uint32_t n_closest = 0u;
  const Sched sd = block_sched(f.P);
  for (uint32_t l = sd.first + threadIdx.x; l < sd.end; l += sd.step) {
    int x = 0, y = 0;
    if (!local_pixel(f, l, x, y)) continue;
    const uint32_t pixel = (uint32_t)(y * f.W + x);
    // computePrimaryRay (:220-234)
    const float ndx = div_nrm(float(x) + 0.5f, idiv.w) * 2.0f - 1.0f;
    const float ndy = 1.0f - div_nrm(float(y) + 0.5f, idiv.h) * 2.0f;
    const vec3 dir = ox_nrm((f.ox_u * ndx + f.ox_v * ndy) + f.ox_w);
    float4 a4 = f.reset ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : f.accum[l];
    vec3 acc = xyz(a4);
    for (uint32_t fr = 0; fr < f.k; ++fr) {
      const uint32_t frame = f.acc0 + fr - 1u;  // OptixBackend's frame_index_ (0 after a reset)
      const uint32_t rng = wang_hash((pixel + 1u) ^ (frame * 9781u + 1u));
      ox_path<kW4, kCube>(sc, sv, sh, smat, nm, f, f.cam_pos, dir, rng, acc, vc, s_stack, n_closest);
      a4.w = a4.w + 1.0f;
    }
    f.accum[l] = make_float4(acc.x, acc.y, acc.z, a4.w);
  }
  unsigned long long a = n_closest;
  for (int off = 32; off > 0; off >>= 1) a += __shfl_xor(a, off);
  if (lane_id() == 0u) atomicAdd(&w.tot[kTotClosest], a);
  report_stack(vc, w.tot);
}

// --------------------------------------------------------------------------------- query kernels
__global__ void __launch_bounds__(kBlock) k_query(SceneView sv, const uint32_t* tri_orig, const uint32_t* sph_orig,
                                                  const float* rays, uint32_t n, int anyhit, uint32_t* ref_out,
                                                  float* t_out, float* ng_out, uint8_t* occ, uint32_t* stack_overflow) {
  __shared__ LdsStack s_stack;
  const Staged sg{sv.nodes, sv.nodes4, sv.prim_ref, sv.tris, sv.sph};
  Visits vc;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += grid_threads()) {
    const float* rr = rays + (size_t)i * 8;
    const Ray r = make_ray(v3(rr[0], rr[1], rr[2]), v3(rr[3], rr[4], rr[5]));
    float tfar = rr[7];
    uint32_t ref = kNoHit;
    if (anyhit) {
      occ[i] = (sv.width == (uint32_t)kWide ? traverse_w<true, true, false>(sg, sv, r, rr[6], tfar, ref, vc, s_stack)
                               : traverse_w<false, true, false>(sg, sv, r, rr[6], tfar, ref, vc, s_stack))
                   ? 1
                   : 0;
      continue;
    }
    const bool hit = sv.width == (uint32_t)kWide ? traverse_w<true, false, false>(sg, sv, r, rr[6], tfar, ref, vc, s_stack)
                                    : traverse_w<false, false, false>(sg, sv, r, rr[6], tfar, ref, vc, s_stack);
    // report (type bit | original primitive index) so the host can map to (geomID, primID)
    ref_out[i] = hit ? ((ref & kSphereBit) | ((ref & kSphereBit) ? sph_orig[ref & kIndexMask] : tri_orig[ref & kIndexMask]))
                     : kNoHit;
    t_out[i] = hit ? tfar : __builtin_huge_valf();
    vec3 ng = v3(0.0f, 0.0f, 0.0f);
    if (hit) {
      const uint32_t idx = ref & kIndexMask;
      if (ref & kSphereBit) {
        const float4 s = sv.sph[idx];
        const vec3 P = r.o + tfar * r.d;
        ng = v3((P.x - s.x) / s.w, (P.y - s.y) / s.w, (P.z - s.z) / s.w);
      } else {
        const float4 c = sv.tris[3 * idx + 2];
        ng = v3(c.y, c.z, c.w);
      }
    }
    ng_out[(size_t)i * 3 + 0] = ng.x;
    ng_out[(size_t)i * 3 + 1] = ng.y;
    ng_out[(size_t)i * 3 + 2] = ng.z;
  }
  if (__ballot(vc.stack_overflow != 0u) && lane_id() == 0u) *stack_overflow = 1u;
}

__global__ void __launch_bounds__(kBlock) k_primary(FrameView f, float* dirs, uint32_t* rng) {
  const uint32_t N = (uint32_t)f.W * (uint32_t)f.H;
  const ImageDiv idiv = image_div(f);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += grid_threads()) {
    const int x = (int)(i % (uint32_t)f.W), y = (int)(i / (uint32_t)f.W);
    const uint32_t acc = f.acc0;
    const uint32_t ps = (uint32_t)(y * f.W + x);
    uint32_t r = wang_hash(ps ^ acc * 9781u);
    const float jx = rand01(r);
    const float jy = rand01(r);
    const vec3 dir = camera_dir(f, div_nrm(float(x) + jx, idiv.w), div_nrm(float(y) + jy, idiv.h));  // as primary_path
    const vec3 d = renormalized_again(dir);
    dirs[(size_t)i * 3 + 0] = d.x;
    dirs[(size_t)i * 3 + 1] = d.y;
    dirs[(size_t)i * 3 + 2] = d.z;
    rng[i] = wang_hash((ps ^ acc) ^ 1u);
  }
}

// The device's values of the two library calls above (sptr_eval_math): fn 0, the cosine sample's
// (sin, cos) for every r1 = k / 2^24 (out: 2^25 floats, pairs by k; x unused); fn 1, gamma_pow(x[i]).
__global__ void __launch_bounds__(kBlock) k_eval_math(int fn, const float* x, uint32_t n, float* out) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += grid_threads()) {
    if (fn == 0) {
      float sp, cp;
      cosine_sincos(float(i) / float(0x01000000u), sp, cp);
      out[2u * i] = sp;
      out[2u * i + 1u] = cp;
    } else {
      out[i] = gamma_pow(x[i]);
    }
  }
}

// --------------------------------------------------------------------------------- launchers
static inline unsigned grid_for(uint64_t work) {
  const uint64_t blocks = (work + kBlock - 1) / kBlock;
  const uint64_t cap = 256ull * 8ull;  // 256 CUs x 8 resident blocks
  return (unsigned)(blocks < 1 ? 1 : (blocks > cap ? cap : blocks));
}

// Persistent-style grid for the queue kernels: exactly the blocks that are resident at once
// (CUs x occupancy), so every block of the contiguous-slice schedule runs in the first and only
// round (a grid of 8 blocks/CU where registers admit 7 would run a 1/7-occupancy tail round).
struct GridCache {
  const void* fn = nullptr;
  uint32_t lds = 0;
  unsigned blocks = 0;
};
static unsigned resident_grid(const void* fn, uint32_t lds_bytes) {
  static GridCache cache[32];
  static int cus = 0;
  int per = 0;
  for (GridCache& g : cache)
    if (g.fn == fn && g.lds == lds_bytes) return g.blocks;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, kBlock, lds_bytes) != hipSuccess || per <= 0) per = 4;
#ifdef SPTR_EXPERIMENT_KNOBS
  static int cap = -1;  // SPTR_MAX_BLOCKS_PER_CU: experiment knob (resident blocks per CU), experiment builds only
  if (cap < 0) {
    const char* e = getenv("SPTR_MAX_BLOCKS_PER_CU");
    cap = e ? atoi(e) : 0;
  }
  if (cap > 0 && per > cap) per = cap;
#endif
  unsigned blocks = (unsigned)(cus * per);
  if (blocks > kMaxSegs) blocks = kMaxSegs;  // producer grids index the segment tables
  for (GridCache& g : cache)
    if (g.fn == nullptr) {
      g = GridCache{fn, lds_bytes, blocks};
      break;
    }
  return blocks;
}

SceneView scene_view(const Context& c) {
  SceneView s;
  s.nodes = static_cast<const BvhNode*>(c.nodes.p);
  s.nodes4 = static_cast<const WideNode*>(c.nodes4.p);
  s.tris = static_cast<const float4*>(c.tris.p);
  s.sph = static_cast<const float4*>(c.sph.p);
  s.tri_geom = static_cast<const uint32_t*>(c.tri_geom.p);
  s.sph_geom = static_cast<const uint32_t*>(c.sph_geom.p);
  s.num_nodes = c.num_nodes;
  s.num_tris = c.num_tri_refs;  // triangle slots (a split triangle has one per reference)
  s.num_sph = c.num_sph;
  s.root = c.root;
  s.num_nodes4 = c.num_nodes4;
  s.root4 = c.root4;
  // width 0 = automatic: BVH2 for LDS-staged scenes (3-20 nodes: the extra slab tests of a BVH4
  // node cost more than the saved steps), BVH4 for everything traversed from L2/HBM
  const uint64_t bytes2 = (uint64_t)c.num_nodes * 64 + (uint64_t)c.num_tri_refs * 48 + (uint64_t)c.num_sph * 16 +
                          ((uint64_t)c.num_tri_refs + c.num_sph + 3) / 4 * 16;
  s.width = c.bvh_width ? c.bvh_width : (bytes2 <= kLdsSceneBytes ? 2u : (uint32_t)kWide);
  // never a width whose worst-case traversal stack exceeds kStack (build_lbvh rejects trees that
  // even BVH2 cannot traverse)
  if (s.width == (uint32_t)kWide && c.stack_need4 > (uint32_t)kStack) s.width = 2u;
  s.prim_ref = static_cast<const uint32_t*>(c.prim_ref.p);
  const uint64_t node_bytes = s.width == (uint32_t)kWide ? (uint64_t)c.num_nodes4 * sizeof(WideNode) : (uint64_t)c.num_nodes * 64;
  const uint64_t bytes = node_bytes + (uint64_t)c.num_tri_refs * 48 + (uint64_t)c.num_sph * 16 +
                         ((uint64_t)c.num_tri_refs + c.num_sph + 3) / 4 * 16;
  s.lds_bytes = bytes <= kLdsSceneBytes ? (uint32_t)bytes : 0u;
  s.scene_bytes = bytes;
  // the refilling wide-BVH kernels of L2/HBM scenes stage the top levels (4-wide nodes only)
  s.num_top4 = (s.width == (uint32_t)kWide && kWide == 4 && s.lds_bytes == 0u) ? c.num_top4 : 0u;
  return s;
}

static unsigned trace_lds(const SceneView& sv, bool lds, bool primary, uint32_t nseg) {
  return (lds ? sv.lds_bytes : 0u) + (primary ? 0u : (4u * (nseg + 1u) + 15u) / 16u * 16u);
}

// Pixel-major bounce 0 needs enough pixels to keep every resident thread busy: with fewer than
// kPixelMajorItems pixels per thread of the resident grid, the per-thread quantisation (a thread
// holds all k samples of its pixel) costs more than the radiance round trip it saves.  Measured
// on C2 (profiles/r01h_pixel_major.txt): 1 GPU, 4.5 pixels/thread: 4.17 -> 3.74 ms; 2-way shard,
// 2.3: 2.26 -> 2.24-2.28; 4-way, 1.1: 1.20 -> 1.28-1.29; 8-way: 0.72 -> 0.99.
constexpr uint32_t kPixelMajorItems = 4;
constexpr uint32_t kPixelMajorMaxK = 128;  // samples per batch above which < 8 pixels/thread go lane-group
// Lane-group bounce 0 (k_trace_wp) from this many samples per batch: 8 lanes take 8 samples of one
// pixel per round, so smaller batches would leave lanes idle.
constexpr uint32_t kWaveFoldMinK = 16;
// k_trace_wp runs at 8 waves/SIMD when the shard's pixels fill the 7-wave resident grid's 8-pixel wave
// groups fewer than this many times (1080p: G = 8 ~4.5 rounds, G = 4 ~9, G = 2 ~18)
constexpr uint64_t kWpHiOccRounds = 6;
uint32_t bounce0_pixel_major(const SceneView& sv, const FrameView& f) {
#ifdef SPTR_EXPERIMENT_KNOBS
  if (const char* e = getenv("SPTR_FOLD")) {  // timing experiments: force kFoldNone/Thread/Wave
    const uint32_t m = (uint32_t)atoi(e);
    if (m == kFoldNone || (m == kFoldWave && f.k >= kWaveFoldMinK) || (m == kFoldThread && sv.lds_bytes != 0)) return m;
  }
#endif
  if (sv.lds_bytes != 0) {
    const unsigned lb = trace_lds(sv, true, true, 0);
    const unsigned g = sv.width == (uint32_t)kWide ? resident_grid((const void*)&k_trace_pm<false, true, false>, lb)
                                      : resident_grid((const void*)&k_trace_pm<false, false, false>, lb);
    const uint64_t threads = (uint64_t)g * kBlock;
    // a thread's pixels are serial loops of k samples: with few pixels per thread and long loops the
    // last round's tail costs more than the lane-group fold (measured r02, emulated 4K shards at
    // 4.5 pixels/thread: k = 64 (C2, 1 GPU) thread 1.45 vs lanes 1.53 ms; k = 259 (C4, 4-way)
    // thread 27.9 vs lanes 22.9 ms; 9 pixels/thread, k = 129 (C4, 2-way): 41.2 vs 45.4 ms)
    if ((uint64_t)f.P >= threads * kPixelMajorItems &&
        ((uint64_t)f.P >= threads * 2u * kPixelMajorItems || f.k <= kPixelMajorMaxK))
      return kFoldThread;
  }
  // L2/HBM scenes stay path-major.  Lane groups at the BVH4 occupancy (r02, production build):
  // C3 trace0 8.07 -> 10.41 ms against k_accum 1.47 -> 0.07 ms, 12.18 -> 13.08 ms/step; C5
  // 23.3 -> 24.1 ms/step (knobs build).  The fold's per-round shuffles and fold state cost the
  // BVH4 traversal more than the radiance round trip it saves.
  return (sv.lds_bytes != 0 && f.k >= kWaveFoldMinK) ? kFoldWave : kFoldNone;
}

// Template dispatch over runtime flags: dispatch(fn, Flags<>{}, b0, b1, ...) calls
// fn(Flags<b0, b1, ...>{}) with the flags as compile-time values (one instantiation per combination).
template <bool... B>
struct Flags {};

template <class Fn, bool... B>
static unsigned dispatch(Fn&& fn, Flags<B...>) {
  return fn(Flags<B...>{});
}
template <class Fn, bool... B, class... Rest>
static unsigned dispatch(Fn&& fn, Flags<B...>, bool first, Rest... rest) {
  return first ? dispatch(fn, Flags<B..., true>{}, rest...) : dispatch(fn, Flags<B..., false>{}, rest...);
}


unsigned launch_trace(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w_in, int depth,
                      bool count, uint32_t nseg, hipStream_t s) {
  const WaveView w = with_tslot(w_in);
  const dim3 b(kBlock);
  const bool L = sv.lds_bytes != 0;
  const bool P = depth == 0;
  const bool W = sv.width == (uint32_t)kWide;
  const bool cube = sh.env.env != nullptr;
  const unsigned lb = trace_lds(sv, L, P, nseg);
  const EnvView ev = sh.env;
  if (P && f.pixel_major == kFoldWave) {
    // rounds of 8-pixel wave groups over the resident grid: few rounds (a small shard) -> 8 waves/SIMD
    const unsigned g7 = resident_grid((const void*)&k_trace_wp<true, false, false, false>, lb);
    const bool hi = L && !W && (uint64_t)f.P < (uint64_t)g7 * (kBlock / 64u) * 8u * kWpHiOccRounds;
    return dispatch(
        [&](auto fl) -> unsigned {
          return [&]<bool Lc, bool C, bool Wc, bool Cube, bool Hi>(Flags<Lc, C, Wc, Cube, Hi>) {
            if constexpr (Hi && (Wc || !Lc)) {
              return 0u;  // not instantiated: the high-occupancy form is for LDS-staged BVH2 scenes
            } else {
              if (w.tslot) {
                const unsigned g = resident_grid((const void*)&k_trace_wp<Lc, C, Wc, Cube, Hi, true>, lb);
                SPTR_TIMED_LAUNCH((k_trace_wp<Lc, C, Wc, Cube, Hi, true>), dim3(g), b, lb, s, sv, ev, f, w);
                return g;
              }
              const unsigned g = resident_grid((const void*)&k_trace_wp<Lc, C, Wc, Cube, Hi>, lb);
              SPTR_TIMED_LAUNCH((k_trace_wp<Lc, C, Wc, Cube, Hi>), dim3(g), b, lb, s, sv, ev, f, w);
              return g;
            }
          }(fl);
        },
        Flags<>{}, L, count, W, cube, hi);
  }
  if (P && L && f.pixel_major == kFoldThread) {
    return dispatch(
        [&](auto fl) -> unsigned {
          return [&]<bool C, bool Wc, bool Cube>(Flags<C, Wc, Cube>) {
            const unsigned g = resident_grid((const void*)&k_trace_pm<C, Wc, Cube>, lb);
            SPTR_TIMED_LAUNCH((k_trace_pm<C, Wc, Cube>), dim3(g), b, lb, s, sv, ev, f, w);
            return g;
          }(fl);
        },
        Flags<>{}, count, W, cube);
  }
  if (!L && W) {  // refilling lanes (scenes traversed from L2/HBM)
    const unsigned lbd = lb + (walk_reads_top(P ? kWalkPrimary : kWalkU) ? sv.num_top4 * (unsigned)sizeof(WideNode) : 0u);  // + top levels
    // per-XCD work queues for scenes larger than an XCD's L2 (as k_shadow_dyn)
    const bool queue = trace_queue_applies(sv);
    return dispatch(
        [&](auto fl) -> unsigned {
          return [&]<bool C, bool Pc, bool Cube, bool Q>(Flags<C, Pc, Cube, Q>) {
            const unsigned g = resident_grid((const void*)&k_trace_dyn<false, C, Pc, true, Cube, Q>, lbd);
            SPTR_TIMED_LAUNCH((k_trace_dyn<false, C, Pc, true, Cube, Q>), dim3(g), b, lbd, s, sv, ev, f, w, depth, nseg);
            return g;
          }(fl);
        },
        Flags<>{}, count, P, cube, queue);
  }
  return dispatch(
      [&](auto fl) -> unsigned {
        return [&]<bool Lc, bool C, bool Pc, bool Wc, bool Cube>(Flags<Lc, C, Pc, Wc, Cube>) {
          const unsigned g = resident_grid((const void*)&k_trace<Lc, C, Pc, Wc, Cube>, lb);
          SPTR_TIMED_LAUNCH((k_trace<Lc, C, Pc, Wc, Cube>), dim3(g), b, lb, s, sv, ev, f, w, depth, nseg);
          return g;
        }(fl);
      },
      Flags<>{}, L, count, P, W, cube);
}

// the any-hit stage runs as k_shadow_dyn and the bounce traces as k_trace_dyn (scenes traversed from
// L2/HBM, one light): the pair enqueue_wavefront overlaps (bounce traces defer their misses to k_shade)
bool shadow_overlaps(const SceneView& sv, const WaveView& w) {
  return sv.lds_bytes == 0 && sv.width == (uint32_t)kWide && w.L == 1u;
}

bool shade_fuses_shadows(const SceneView& sv, const ShadeView& sh, bool count) {
#ifdef SPTR_EXPERIMENT_KNOBS
  if (getenv("SPTR_NO_FUSE")) return false;
#endif
  // the visit-count pass keeps k_shadow (shadow visit tallies); several lights keep their task
  // records (in light order) in the shadow stream; the in-shade traversal is the LDS BVH2 one
  return sv.lds_bytes != 0 && sv.width == 2u && sh.num_lights == 1u && !count;
}

unsigned launch_shade(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, int depth,
                      uint32_t nseg, bool fuse, hipStream_t s) {
  const unsigned lb = (fuse ? sv.lds_bytes : 0u) + (4u * (nseg + 1u) + 15u) / 16u * 16u;
  return dispatch(
      [&](auto fl) -> unsigned {
        return [&]<bool Pc, bool Fc>(Flags<Pc, Fc>) {
          const unsigned g = resident_grid((const void*)&k_shade<Pc, Fc>, lb);
          hipLaunchKernelGGL((k_shade<Pc, Fc>), dim3(g), dim3(kBlock), lb, s, sv, sh, f, w, depth, nseg);
          return g;
        }(fl);
      },
      Flags<>{}, depth == 0, fuse);
}

uint32_t cull_depth_for(uint32_t spp) { return spp >= 16u ? (uint32_t)kCullDepthMax : 4u; }

void launch_cull(const SceneView& sv, const FrameView& f, uint32_t* mask, uint32_t* plist, hipStream_t s) {
  if (f.P == 0u) return;
  hipLaunchKernelGGL(k_cull, dim3(f.P / kTilePixels), dim3(kBlock), 0, s, sv, f, mask, plist);
}

unsigned launch_bounce(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w_in, int depth,
                       uint32_t nseg, hipStream_t s) {
  const WaveView w = with_tslot(w_in);
  const unsigned lb = sv.lds_bytes + (4u * (nseg + 1u) + 15u) / 16u * 16u;
  return dispatch(
      [&](auto fl) -> unsigned {
        return [&]<bool Cube, bool T>(Flags<Cube, T>) {
          const unsigned g = resident_grid((const void*)&k_bounce<Cube, T>, lb);
          SPTR_TIMED_LAUNCH((k_bounce<Cube, T>), dim3(g), dim3(kBlock), lb, s, sv, sh, f, w, depth, nseg);
          return g;
        }(fl);
      },
      Flags<>{}, sh.env.env != nullptr, w.tslot != nullptr);
}

unsigned launch_bounce01(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w_in, uint32_t nseg,
                         hipStream_t s) {
  const WaveView w = with_tslot(w_in);
  const unsigned lb = sv.lds_bytes + (4u * (nseg + 1u) + 15u) / 16u * 16u;
  return dispatch(
      [&](auto fl) -> unsigned {
        return [&]<bool Cube, bool T>(Flags<Cube, T>) {
          const unsigned g = resident_grid((const void*)&k_bounce01<Cube, T>, lb);
          SPTR_TIMED_LAUNCH((k_bounce01<Cube, T>), dim3(g), dim3(kBlock), lb, s, sv, sh, f, w, nseg);
          return g;
        }(fl);
      },
      Flags<>{}, sh.env.env != nullptr, w.tslot != nullptr);
}

unsigned launch_shadow(const SceneView& sv, const ShadeView& sh, const WaveView& w_in, int depth, bool count,
                       uint32_t nseg, hipStream_t s) {
  const WaveView w = with_tslot(w_in);
  const dim3 b(kBlock);
  const bool L = sv.lds_bytes != 0;
  const bool W = sv.width == (uint32_t)kWide;
  const unsigned lb = trace_lds(sv, L, false, nseg);
  unsigned g = 0;
  if (!L && W && w.L == 1u) {  // wide BVH from L2/HBM, one light: refilling lanes
    // per-XCD work queues for scenes larger than an XCD's L2 (k_shadow_dyn kQueue)
    const bool queue = sv.scene_bytes > kL2BytesPerXcd;
    const unsigned lbd = lb + (walk_reads_top(queue ? kWalkU : kWalkInline) ? sv.num_top4 * (unsigned)sizeof(WideNode) : 0u);  // + top levels
    return dispatch(
        [&](auto fl) -> unsigned {
          return [&]<bool C, bool Q>(Flags<C, Q>) {
            const unsigned gq = resident_grid((const void*)&k_shadow_dyn<C, Q>, lbd);
            SPTR_TIMED_LAUNCH((k_shadow_dyn<C, Q>), dim3(gq), b, lbd, s, sv, sh, w, depth, nseg);
            return gq;
          }(fl);
        },
        Flags<>{}, count, queue);
  }
#define SPTR_SHADOW(Lc, C, Wc)                                                                      \
  do {                                                                                              \
    g = resident_grid((const void*)&k_shadow<Lc, C, Wc>, lb);                                       \
    SPTR_TIMED_LAUNCH((k_shadow<Lc, C, Wc>), dim3(g), b, lb, s, sv, sh, w, depth, nseg);           \
  } while (0)
#define SPTR_SHADOW_W(Lc, C) \
  do {                       \
    if (W) SPTR_SHADOW(Lc, C, true); else SPTR_SHADOW(Lc, C, false); \
  } while (0)
  if (L) { if (count) SPTR_SHADOW_W(true, true); else SPTR_SHADOW_W(true, false); }
  else   { if (count) SPTR_SHADOW_W(false, true); else SPTR_SHADOW_W(false, false); }
#undef SPTR_SHADOW_W
#undef SPTR_SHADOW
  return g;
}

unsigned launch_tail(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, int depth0,
                     uint32_t nseg, hipStream_t s) {
  const bool L = sv.lds_bytes != 0;
  const bool W = sv.width == (uint32_t)kWide;
  const unsigned lb = trace_lds(sv, L, false, nseg) + ((walk_reads_top(kWalkU) && !L && W) ? sv.num_top4 * (unsigned)sizeof(WideNode) : 0u);
  return dispatch(
      [&](auto fl) -> unsigned {
        return [&]<bool Lc, bool Wc, bool Cube>(Flags<Lc, Wc, Cube>) {
          const unsigned g = resident_grid((const void*)&k_tail<Lc, Wc, Cube>, lb);
          hipLaunchKernelGGL((k_tail<Lc, Wc, Cube>), dim3(g), dim3(kBlock), lb, s, sv, sh, f, w, depth0, nseg);
          return g;
        }(fl);
      },
      Flags<>{}, L, sv.width == (uint32_t)kWide, sh.env.env != nullptr);
}

bool trace_queue_applies(const SceneView& sv) {
  return sv.lds_bytes == 0u && sv.width == (uint32_t)kWide && sv.scene_bytes > kL2BytesPerXcd;
}
bool strag_applies(const SceneView& sv) { return trace_queue_applies(sv); }
// hit-record segments per static share: twice the share where k_trace_dyn takes its rays from the per-XCD
// queues.  (r05t: the queues for C3's bounce-0 trace too, beside k_sky: 3.53-3.55 vs 3.55-3.57 ms, noise.)
uint32_t hrec_mult(const SceneView& sv) { return trace_queue_applies(sv) ? 2u : 1u; }

// a fixed grid: the number of handed-off paths is known only on the device (k_strag reads it).  Small,
// so that it holds few of the wave slots the chain's resident grids expect (r04k: 1024 blocks, 16 waves
// per CU, made C5 8.38 -> 10.17 ms/step), large enough to finish its paths before the batch's k_accum
// (r04l/m at 16 lanes: 64 / 128 / 256 / 512 blocks 13.1 / 9.6 / 7.9 / 8.1 ms)
#ifndef SPTR_STRAG_GRID
#define SPTR_STRAG_GRID 256
#endif
void launch_strag(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, int depth,
                  hipStream_t s) {
  constexpr unsigned kStragGrid = SPTR_STRAG_GRID;
  const unsigned lb = walk_reads_top(kWalkU) ? sv.num_top4 * (unsigned)sizeof(WideNode) : 0u;  // the top levels in LDS
  if (sh.env.env != nullptr) hipLaunchKernelGGL((k_strag<true, true>), dim3(kStragGrid), dim3(kBlock), lb, s, sv, sh, f, w, depth);
  else hipLaunchKernelGGL((k_strag<true, false>), dim3(kStragGrid), dim3(kBlock), lb, s, sv, sh, f, w, depth);
}

void launch_pathtracer(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, hipStream_t s) {
  const bool L = sv.lds_bytes != 0;
  const unsigned lb = L ? sv.lds_bytes : 16u;
  dispatch(
      [&](auto fl) -> unsigned {
        return [&]<bool Lc, bool Wc, bool Cube>(Flags<Lc, Wc, Cube>) {
          const unsigned g = std::min<unsigned>(resident_grid((const void*)&k_pathtracer<Lc, Wc, Cube>, lb),
                                                (unsigned)((f.P + kBlock - 1) / kBlock));
          hipLaunchKernelGGL((k_pathtracer<Lc, Wc, Cube>), dim3(g), dim3(kBlock), lb, s, sv, sh, f, w);
          return g;
        }(fl);
      },
      Flags<>{}, L, sv.width == (uint32_t)kWide, sh.env.env != nullptr);
}

void launch_optix(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, hipStream_t s) {
  const bool L = sv.lds_bytes != 0;
  const unsigned lb = L ? sv.lds_bytes : 16u;
  dispatch(
      [&](auto fl) -> unsigned {
        return [&]<bool Lc, bool Wc, bool Cube>(Flags<Lc, Wc, Cube>) {
          const unsigned g = std::min<unsigned>(resident_grid((const void*)&k_optix<Lc, Wc, Cube>, lb),
                                                (unsigned)((f.P + kBlock - 1) / kBlock));
          hipLaunchKernelGGL((k_optix<Lc, Wc, Cube>), dim3(g), dim3(kBlock), lb, s, sv, sh, f, w);
          return g;
        }(fl);
      },
      Flags<>{}, L, sv.width == (uint32_t)kWide, sh.env.env != nullptr);
}

void launch_frame_dyn(uint32_t* dyn, uint32_t frame_begin, uint32_t reset, uint32_t total, uint32_t* clear,
                      unsigned long long* t0, hipStream_t s) {
  hipLaunchKernelGGL(k_frame_dyn, dim3(1), dim3(64), 0, s, dyn, frame_begin, reset, total, clear, t0);
}
const void* frame_dyn_kernel() { return (const void*)&k_frame_dyn; }

// sptr_overlap_probe: one wave spinning on the device wall clock (s_memrealtime, a counter read)
__global__ void k_spin(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
void launch_spin(uint64_t ticks, hipStream_t s) { hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, ticks); }

void launch_sky(const ShadeView& sh, const FrameView& f, bool capped, hipStream_t s) {
#ifdef SPTR_EXPERIMENT_KNOBS
  // SPTR_SKY_BLOCKS (A/B): a smaller grid-stride grid, leaving wave slots to the launches overlapped with it
  static const unsigned cap = getenv("SPTR_SKY_BLOCKS") ? (unsigned)atoi(getenv("SPTR_SKY_BLOCKS")) : 16384u;
#else
  constexpr unsigned cap = 16384u;
#endif
  const unsigned g = std::max(1u, std::min<unsigned>((f.P + kBlock - 1u) / kBlock, cap ? cap : 16384u));
  auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(g), dim3(kBlock), 0, s, sh.env, f); };
  if (sh.env.env != nullptr) {
    if (capped) go(k_sky<true, true>); else go(k_sky<true, false>);
  } else {
    if (capped) go(k_sky<false, true>); else go(k_sky<false, false>);
  }
}

__global__ void __launch_bounds__(kBlock) k_interleave_tiles(const uint4* a, uint32_t na, const uint4* b, uint32_t nb,
                                                             uint4* dst, uint32_t n) {
  constexpr uint32_t kQuads = kTilePixels / 4u;  // uint4 words per tile
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n * kQuads; q += grid_threads()) {
    const uint32_t t = q / kQuads, r = q - t * kQuads, h = t >> 1;
    const uint4* src = (t & 1u) ? b : a;
    const uint32_t ns = (t & 1u) ? nb : na;
    dst[q] = h < ns ? src[h * kQuads + r] : make_uint4(0u, 0u, 0u, 0u);
  }
}
void launch_interleave_tiles(const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb, uint32_t* dst,
                             uint32_t n, hipStream_t s) {
  if (n == 0u) return;
  hipLaunchKernelGGL(k_interleave_tiles, dim3(grid_for(n * (kTilePixels / 4u))), dim3(kBlock), 0, s,
                     reinterpret_cast<const uint4*>(a), na, reinterpret_cast<const uint4*>(b), nb,
                     reinterpret_cast<uint4*>(dst), n);
}

void launch_accumulate(const FrameView& f, const WaveView& w_in, float4* accum, uint32_t* tiles, uint8_t* image,
                       bool resolve, hipStream_t s) {
  const WaveView w = with_tslot(w_in);  // (the call span's end: the call's last k_accum)
  if (resolve) hipLaunchKernelGGL(k_accum<true>, dim3(grid_for(f.P)), dim3(kBlock), 0, s, f, w, accum, tiles, image);
  else hipLaunchKernelGGL(k_accum<false>, dim3(grid_for(f.P)), dim3(kBlock), 0, s, f, w, accum, tiles, image);
}

void launch_resolve(const FrameView& f, const float4* accum, uint32_t n, uint32_t* tiles, uint8_t* image,
                    hipStream_t s) {
  hipLaunchKernelGGL(k_resolve, dim3(grid_for(f.P)), dim3(kBlock), 0, s, f, accum, n, tiles, image);
}

__global__ void __launch_bounds__(kBlock) k_tri_materials(const uint32_t* tri_geom, const uint32_t* geom_mat, uint32_t n,
                                                          uint32_t* tri_mat) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += grid_threads()) tri_mat[i] = geom_mat[tri_geom[i]];
}
void launch_tri_materials(const uint32_t* tri_geom, const uint32_t* geom_mat, uint32_t n, uint32_t* tri_mat, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_tri_materials, dim3(grid_for(n)), dim3(kBlock), 0, s, tri_geom, geom_mat, n, tri_mat);
}

void launch_unpack(const uint32_t* gathered, int G, uint32_t tiles_per_rank, int W, int H, uint8_t* rgb,
                   hipStream_t s) {
  const int ntx = (W + kTile - 1) / kTile;
  hipLaunchKernelGGL(k_unpack, dim3(grid_for((uint64_t)W * H)), dim3(kBlock), 0, s, gathered, G, tiles_per_rank, W,
                     H, ntx, rgb);
}

void launch_query(const SceneView& sv, const uint32_t* tri_orig, const uint32_t* sph_orig, const float* rays, uint32_t n,
                  bool anyhit, uint32_t* ref, float* t, float* ng, uint8_t* occ, uint32_t* stack_overflow, hipStream_t s) {
  hipLaunchKernelGGL(k_query, dim3(grid_for(n)), dim3(kBlock), 0, s, sv, tri_orig, sph_orig, rays, n, anyhit ? 1 : 0,
                     ref, t, ng, occ, stack_overflow);
}

void launch_eval_math(int fn, const float* x, uint32_t n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_eval_math, dim3(grid_for(n)), dim3(kBlock), 0, s, fn, x, n, out);
}
void launch_primary(const FrameView& f, float* dirs, uint32_t* rng, hipStream_t s) {
  hipLaunchKernelGGL(k_primary, dim3(grid_for((uint64_t)f.W * f.H)), dim3(kBlock), 0, s, f, dirs, rng);
}

}  // namespace sptr
