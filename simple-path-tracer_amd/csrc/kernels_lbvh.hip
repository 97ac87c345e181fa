// kernels_lbvh.hip — on-device LBVH build replacing Embree's BVH build / OptiX GAS+IAS builds
// (src/backends/EmbreeBackend.cpp:82-181, src/backends/OptixBackend.cpp:916-1308).
//
// One flat BVH2 over every world-space triangle and analytic sphere (typed leaf links):
//   k_prim_bounds : per-primitive AABB
//   k_split_count + scan + k_split_emit (L2/HBM scenes): split references — a triangle whose box is far
//                   larger than the triangle (a sliver lying across the axes) gets 2^D references, each
//                   with the tight box of one piece of the triangle clipped by D recursive midpoint splits
//                   (early split clipping); every other primitive keeps one reference with its own box
//   k_ref_bounds  : centroid bounds of the references (ordered-int atomics)
//   k_morton      : 63-bit Morton code (21 bits/axis) of a reference's box centroid, value = reference id
//   radix sort    : radix_sort_pairs_u64 on the codes (kernels_sort.hip, hand-written LSD, stable)
//   k_leaves      : scatter triangles (v0, e1, e2, Ng precomputed as Embree's TriangleM does) and
//                   spheres into sorted slots, one slot per reference (a split triangle's references
//                   each hold a copy); typed leaf links
//   k_karras      : Karras 2012 binary radix tree over the sorted codes (ties broken by index)
//   k_refit       : bottom-up box propagation; the second child to arrive at a node finishes it
//                   (write-through 8-byte box pairs, drained before one agent-scope exchange that
//                   also carries the subtree height — the fence-free hand-off of the gfx950 guide,
//                   Guideline 16 R1)
//   k_treelet     : (L2/HBM scenes) SAH treelet restructuring after k_refit, bottom-up by subtree height, 3 passes;
//                   never deepens a subtree (k_heights, k_height_count / k_height_scatter order the launches)
//   k_wide_count + scan + k_wide_emit, one wide level at a time: wide BVH (4 children) by the greedy
//                   surface-area collapse — a wide node opens its largest-area internal child until
//                   it has kWide children; single-primitive leaves become direct links, others stay
//                   ranges; wide nodes are numbered level by level (top levels first).  (r02i: the
//                   fixed collapse of every second LBVH level it replaced left nodes half empty:
//                   C5 15.58 -> 15.38 ms/step; opening by area x primitives and a host-built SAH BVH2
//                   were A/B-only experiments, removed r05.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cstring>
#include <vector>

#include "sptr_internal.h"

// treelet size (leaves) of the SAH restructuring of L2/HBM scenes' LBVH (r03u/v A/B); a restructured
// treelet never deepens its subtree
constexpr int kTreeletLeaves = 5;

namespace sptr {

namespace {

#define LB_CHECK(x)                                                   \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      c.err = std::string("lbvh: ") + #x + ": " + hipGetErrorString(e_); \
      return SPTR_ERR_HIP;                                            \
    }                                                                 \
  } while (0)

__device__ __forceinline__ uint32_t f2ord(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

__device__ __forceinline__ uint64_t expand21(uint32_t v) {
  uint64_t x = v & 0x1FFFFFu;
  x = (x | x << 32) & 0x1F00000000FFFFull;
  x = (x | x << 16) & 0x1F0000FF0000FFull;
  x = (x | x << 8) & 0x100F00F00F00F00Full;
  x = (x | x << 4) & 0x10C30C30C30C30C3ull;
  x = (x | x << 2) & 0x1249249249249249ull;
  return x;
}

struct BuildIn {
  const float* pos;
  const uint32_t* idx;
  const float4* sph;
  const uint32_t* tri_geom;
  uint32_t ntri, nsph, sph_geom_base;
};

__device__ __forceinline__ void prim_box(const BuildIn& in, uint32_t i, vec3& lo, vec3& hi) {
  if (i < in.ntri) {
    const uint32_t a = in.idx[3 * i], b = in.idx[3 * i + 1], c = in.idx[3 * i + 2];
    const vec3 p0 = v3(in.pos[3 * a], in.pos[3 * a + 1], in.pos[3 * a + 2]);
    const vec3 p1 = v3(in.pos[3 * b], in.pos[3 * b + 1], in.pos[3 * b + 2]);
    const vec3 p2 = v3(in.pos[3 * c], in.pos[3 * c + 1], in.pos[3 * c + 2]);
    lo = v3(fminf(p0.x, fminf(p1.x, p2.x)), fminf(p0.y, fminf(p1.y, p2.y)), fminf(p0.z, fminf(p1.z, p2.z)));
    hi = v3(fmaxf(p0.x, fmaxf(p1.x, p2.x)), fmaxf(p0.y, fmaxf(p1.y, p2.y)), fmaxf(p0.z, fmaxf(p1.z, p2.z)));
  } else {
    const float4 s = in.sph[i - in.ntri];
    lo = v3(s.x - s.w, s.y - s.w, s.z - s.w);
    hi = v3(s.x + s.w, s.y + s.w, s.z + s.w);
  }
}

__global__ void k_prim_bounds(BuildIn in, float4* blo, float4* bhi) {
  const uint32_t N = in.ntri + in.nsph;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) {
    vec3 lo, hi;
    prim_box(in, i, lo, hi);
    blo[i] = make_float4(lo.x, lo.y, lo.z, 0.0f);
    bhi[i] = make_float4(hi.x, hi.y, hi.z, 0.0f);
  }
}

// ------------------------------------------------------------------------------ split references
// Early split clipping (Ernst & Greiner, "Early Split Clipping for Bounding Volume Hierarchies",
// RT 2007).  A triangle lying diagonally across the axes has a box far larger than itself: the
// 1250 x 4000 sphere mesh's rows near the poles (SceneDesc.h:225-279) are slivers ~640 / k times as
// long as they are wide in row k, all fanning out of the pole, so near the pole the boxes of hundreds of
// them overlap any point and a ray crossing there visits hundreds of nodes (r03: 256-1023 visits per ray,
// the rays that set the length of every C5 trace launch).  Such a triangle is referenced 2^D times
// instead, each reference bounding one piece: the triangle clipped by D recursive splits of its
// current piece's box at the midpoint of the longest axis.  Pieces are convex polygons (<= 3 + D
// vertices) clipped in double precision — exact for the float vertices, and each piece box is rounded
// outwards to float — so the union of a triangle's reference boxes contains the triangle.  Closest-hit
// and any-hit results are those of the triangle itself (each reference tests the same triangle).
// D: the smallest depth with box area / (ratio threshold x triangle area) <= 2^D, at most log2 of the
// context's piece limit (sptr_set_split_refs).
constexpr float kSplitRatio = 8.0f;  // box half-area / triangle area above which a triangle is split
constexpr int kMaxSplitDepth = 5;

__device__ __forceinline__ uint32_t split_pieces(const BuildIn& in, uint32_t i, float4 lo, float4 hi, uint32_t max_pieces) {
  if (i >= in.ntri || max_pieces <= 1u) return 1u;
  const uint32_t a = in.idx[3 * i], b = in.idx[3 * i + 1], c = in.idx[3 * i + 2];
  const vec3 p0 = v3(in.pos[3 * a], in.pos[3 * a + 1], in.pos[3 * a + 2]);
  const vec3 p1 = v3(in.pos[3 * b], in.pos[3 * b + 1], in.pos[3 * b + 2]);
  const vec3 p2 = v3(in.pos[3 * c], in.pos[3 * c + 1], in.pos[3 * c + 2]);
  const vec3 n = cross(p1 - p0, p2 - p0);
  const float area2 = sqrtf(dot(n, n));  // twice the triangle's area
  const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
  const float box = dx * dy + dy * dz + dz * dx;  // half the box's surface area
  if (!(area2 > 0.0f) || box <= kSplitRatio * 0.5f * area2) return 1u;
  uint32_t p = 1u;
  while (p < max_pieces && box > kSplitRatio * 0.5f * area2 * (float)p) p <<= 1;
  return p;
}

__global__ void k_split_count(BuildIn in, const float4* blo, const float4* bhi, uint32_t max_pieces, uint32_t* cnt) {
  const uint32_t N = in.ntri + in.nsph;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x)
    cnt[i] = split_pieces(in, i, blo[i], bhi[i], max_pieces);
}

struct Poly {
  double v[3 + kMaxSplitDepth][3];
  int n;
};
// Sutherland-Hodgman against the half-space x_a <= m (keep_le) or x_a >= m
__device__ void clip_poly(Poly& p, int a, double m, bool keep_le) {
  Poly o;
  o.n = 0;
  for (int i = 0; i < p.n; ++i) {
    const double* A = p.v[i];
    const double* B = p.v[(i + 1) % p.n];
    const bool ina = keep_le ? A[a] <= m : A[a] >= m;
    const bool inb = keep_le ? B[a] <= m : B[a] >= m;
    if (ina && o.n < 3 + kMaxSplitDepth) {
      for (int k = 0; k < 3; ++k) o.v[o.n][k] = A[k];
      ++o.n;
    }
    if (ina != inb && o.n < 3 + kMaxSplitDepth) {
      const double t = (m - A[a]) / (B[a] - A[a]);
      for (int k = 0; k < 3; ++k) o.v[o.n][k] = k == a ? m : A[k] + t * (B[k] - A[k]);
      ++o.n;
    }
  }
  p = o;
}
__device__ __forceinline__ void poly_box(const Poly& p, double lo[3], double hi[3]) {
  for (int k = 0; k < 3; ++k) {
    lo[k] = hi[k] = p.v[0][k];
    for (int i = 1; i < p.n; ++i) {
      lo[k] = fmin(lo[k], p.v[i][k]);
      hi[k] = fmax(hi[k], p.v[i][k]);
    }
  }
}
__device__ __forceinline__ float down_f(double x) {
  const float f = (float)x;
  return (double)f > x ? nextafterf(f, -INFINITY) : f;
}
__device__ __forceinline__ float up_f(double x) {
  const float f = (float)x;
  return (double)f < x ? nextafterf(f, INFINITY) : f;
}

// references of primitive i at roff[i] ..: rprim = i, the piece boxes (or the primitive's own box)
__global__ void k_split_emit(BuildIn in, const float4* blo, const float4* bhi, const uint32_t* cnt, const uint32_t* roff,
                             float4* rlo, float4* rhi, uint32_t* rprim) {
  const uint32_t N = in.ntri + in.nsph;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) {
    const uint32_t n = cnt[i], r0 = roff[i];
    const float4 tlo = blo[i], thi = bhi[i];
    if (n == 1u) {
      rlo[r0] = tlo;
      rhi[r0] = thi;
      rprim[r0] = i;
      continue;
    }
    const uint32_t ia = in.idx[3 * i], ib = in.idx[3 * i + 1], ic = in.idx[3 * i + 2];
    const uint32_t vid[3] = {ia, ib, ic};
    const int D = __ffs((int)n) - 1;  // n = 2^D
    for (uint32_t k = 0; k < n; ++k) {
      Poly p;
      p.n = 3;
      for (int j = 0; j < 3; ++j)
        for (int a = 0; a < 3; ++a) p.v[j][a] = (double)in.pos[3 * vid[j] + a];
      for (int lev = 0; lev < D && p.n > 0; ++lev) {
        double lo[3], hi[3];
        poly_box(p, lo, hi);
        int ax = 0;
        for (int a = 1; a < 3; ++a)
          if (hi[a] - lo[a] > hi[ax] - lo[ax]) ax = a;
        if (!(hi[ax] > lo[ax])) break;  // a point: nothing left to split
        const double m = 0.5 * (lo[ax] + hi[ax]);
        clip_poly(p, ax, m, ((k >> (D - 1 - lev)) & 1u) == 0u);
      }
      float4 o_lo = tlo, o_hi = thi;
      if (p.n > 0) {
        double lo[3], hi[3];
        poly_box(p, lo, hi);
        o_lo = make_float4(fmaxf(down_f(lo[0]), tlo.x), fmaxf(down_f(lo[1]), tlo.y), fmaxf(down_f(lo[2]), tlo.z), 0.0f);
        o_hi = make_float4(fminf(up_f(hi[0]), thi.x), fminf(up_f(hi[1]), thi.y), fminf(up_f(hi[2]), thi.z), 0.0f);
      }
      rlo[r0 + k] = o_lo;
      rhi[r0 + k] = o_hi;
      rprim[r0 + k] = i;
    }
  }
}

__global__ void k_ref_bounds(uint32_t NR, const float4* blo, const float4* bhi, uint32_t* cb) {
  uint32_t mn[3] = {~0u, ~0u, ~0u}, mx[3] = {0u, 0u, 0u};
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < NR; i += gridDim.x * blockDim.x) {
    const float4 lo = blo[i], hi = bhi[i];
    const float c[3] = {0.5f * (lo.x + hi.x), 0.5f * (lo.y + hi.y), 0.5f * (lo.z + hi.z)};
    for (int k = 0; k < 3; ++k) {
      const uint32_t o = f2ord(c[k]);
      mn[k] = min(mn[k], o);
      mx[k] = max(mx[k], o);
    }
  }
  for (int k = 0; k < 3; ++k) {
    for (int off = 32; off > 0; off >>= 1) {
      mn[k] = min(mn[k], (uint32_t)__shfl_xor((int)mn[k], off));
      mx[k] = max(mx[k], (uint32_t)__shfl_xor((int)mx[k], off));
    }
  }
  if ((threadIdx.x & 63) == 0) {
    for (int k = 0; k < 3; ++k) {
      atomicMin(&cb[k], mn[k]);
      atomicMax(&cb[3 + k], mx[k]);
    }
  }
}

// Embree's precomputed geometric normal Ng = cross(e2, e1) (msub form), as k_leaves stores it
__device__ __forceinline__ vec3 tri_ng(const BuildIn& in, uint32_t prim) {
  const uint32_t a = in.idx[3 * prim], b = in.idx[3 * prim + 1], c = in.idx[3 * prim + 2];
  const vec3 v0 = v3(in.pos[3 * a], in.pos[3 * a + 1], in.pos[3 * a + 2]);
  const vec3 v1 = v3(in.pos[3 * b], in.pos[3 * b + 1], in.pos[3 * b + 2]);
  const vec3 v2 = v3(in.pos[3 * c], in.pos[3 * c + 1], in.pos[3 * c + 2]);
  const vec3 e1 = v0 - v1, e2 = v2 - v0;
  return v3(__builtin_fmaf(e2.y, e1.z, -(e2.z * e1.y)), __builtin_fmaf(e2.z, e1.x, -(e2.x * e1.z)),
            __builtin_fmaf(e2.x, e1.y, -(e2.y * e1.x)));
}
// Morton code of the centroid; a triangle whose stored Ng is exactly zero (two equal vertices: e.g.
// the 1250x4000 sphere mesh's north-pole ring, whose vertices are all (+-0, r, +-0)) gets bit 63, so
// the sort moves it behind every other primitive and the tree is built without it: the Moeller-
// Trumbore test rejects den = dot(Ng, d) = 0 for every ray (tri_hit4: den != 0), so such a triangle
// can never be a closest hit or an occluder — excluding it changes no result, and removes boxes that
// all contain the pole from the fan every polar ray crosses.
__global__ void k_morton(BuildIn in, uint32_t N, const float4* blo, const float4* bhi, const uint32_t* rprim, const uint32_t* cb,
                         uint64_t* keys, uint32_t* vals, uint32_t* ndeg) {
  float lo[3], ext[3];
  for (int k = 0; k < 3; ++k) {
    lo[k] = ord2f(cb[k]);
    ext[k] = ord2f(cb[3 + k]) - lo[k];
  }
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) {
    const float4 a = blo[i], b = bhi[i];
    const float c[3] = {0.5f * (a.x + b.x), 0.5f * (a.y + b.y), 0.5f * (a.z + b.z)};
    uint64_t code = 0;
    for (int k = 0; k < 3; ++k) {
      const float t = ext[k] > 0.0f ? (c[k] - lo[k]) / ext[k] : 0.5f;
      const float q = fminf(fmaxf(t * 2097152.0f, 0.0f), 2097151.0f);
      code |= expand21((uint32_t)q) << (2 - k);
    }
    bool deg = false;
    const uint32_t prim = rprim[i];
    if (prim < in.ntri) {
      const vec3 ng = tri_ng(in, prim);
      deg = ng.x == 0.0f && ng.y == 0.0f && ng.z == 0.0f;
    }
    const uint32_t nd = (uint32_t)__popcll(__ballot(deg));
    if (nd && __lane_id() == (uint32_t)(__ffsll(__ballot(deg)) - 1)) atomicAdd(ndeg, nd);
    keys[i] = deg ? (code | (1ull << 63)) : code;
    vals[i] = i;
  }
}

__global__ void k_is_tri(uint32_t N, uint32_t ntri, const uint32_t* vals, const uint32_t* rprim, uint32_t* flag) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x)
    flag[i] = rprim[vals[i]] < ntri ? 1u : 0u;
}

// sorted reference i -> its slot (triangle slots in reference order, then sphere slots)
__global__ void k_leaves(BuildIn in, uint32_t N, const uint32_t* vals, const uint32_t* rprim, const uint32_t* tri_slot,
                         float4* tris, uint32_t* tri_geom, uint32_t* tri_orig, float4* sph, uint32_t* sph_geom,
                         uint32_t* sph_orig, uint32_t* prim_ref) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) {
    const uint32_t prim = rprim[vals[i]];
    if (prim < in.ntri) {
      const uint32_t slot = tri_slot[i];
      const uint32_t a = in.idx[3 * prim], b = in.idx[3 * prim + 1], c = in.idx[3 * prim + 2];
      const vec3 v0 = v3(in.pos[3 * a], in.pos[3 * a + 1], in.pos[3 * a + 2]);
      const vec3 v1 = v3(in.pos[3 * b], in.pos[3 * b + 1], in.pos[3 * b + 2]);
      const vec3 v2 = v3(in.pos[3 * c], in.pos[3 * c + 1], in.pos[3 * c + 2]);
      const vec3 e1 = v0 - v1, e2 = v2 - v0;
      const vec3 ng = tri_ng(in, prim);  // Ng = cross(e2, e1) with Embree's msub (fma) evaluation
      tris[3 * slot + 0] = make_float4(v0.x, v0.y, v0.z, e1.x);
      tris[3 * slot + 1] = make_float4(e1.y, e1.z, e2.x, e2.y);
      tris[3 * slot + 2] = make_float4(e2.z, ng.x, ng.y, ng.z);
      tri_geom[slot] = in.tri_geom[prim];
      tri_orig[slot] = prim;
      prim_ref[i] = slot;
    } else {
      const uint32_t slot = i - tri_slot[i];
      const uint32_t s = prim - in.ntri;
      sph[slot] = in.sph[s];
      sph_geom[slot] = in.sph_geom_base + s;
      sph_orig[slot] = s;
      prim_ref[i] = kSphereBit | slot;
    }
  }
}

__device__ __forceinline__ int delta(const uint64_t* keys, int N, int i, int j) {
  if (j < 0 || j >= N) return -1;
  const uint64_t a = keys[i], b = keys[j];
  if (a == b) return 64 + __clz((uint32_t)(i ^ j));
  return __clzll((long long)(a ^ b));
}

// Leaf range link for sorted primitives [lo, lo+cnt).
__device__ __forceinline__ uint32_t range_link(uint32_t lo, uint32_t cnt) {
  return kLeafBit | (lo << kLeafCountBits) | (cnt - 1u);
}

// Karras 2012 hierarchy.  Child links become range leaves when the child subtree covers at most
// leaf_max primitives; `kids` keeps the binary-tree child ids (leaf i -> kLeafBit | i) for refit.
__global__ void k_karras(int N, const uint64_t* keys, uint32_t leaf_max, BvhNode* nodes, uint2* kids,
                         uint32_t* leaf_parent) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N - 1; i += gridDim.x * blockDim.x) {
    const int d = (delta(keys, N, i, i + 1) - delta(keys, N, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(keys, N, i, i - d);
    int lmax = 2;
    while (delta(keys, N, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
      if (delta(keys, N, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(keys, N, i, j);
    int s = 0;
    for (int div = 2;; div *= 2) {
      const int t = (l + div - 1) / div;
      if (delta(keys, N, i, i + (s + t) * d) > dnode) s += t;
      if (t <= 1) break;
    }
    const int gamma = i + s * d + min(d, 0);
    const int lo = min(i, j), hi = max(i, j);
    uint32_t kl, kr;  // binary-tree child ids
    if (lo == gamma) {
      kl = kLeafBit | (uint32_t)gamma;
      leaf_parent[gamma] = (uint32_t)i;
    } else {
      kl = (uint32_t)gamma;
      nodes[gamma].link.z = (uint32_t)i;
    }
    if (hi == gamma + 1) {
      kr = kLeafBit | (uint32_t)(gamma + 1);
      leaf_parent[gamma + 1] = (uint32_t)i;
    } else {
      kr = (uint32_t)(gamma + 1);
      nodes[gamma + 1].link.z = (uint32_t)i;
    }
    const uint32_t nl = (uint32_t)(gamma - lo + 1), nr = (uint32_t)(hi - gamma);
    nodes[i].link.x = nl <= leaf_max ? range_link((uint32_t)lo, nl) : kl;
    nodes[i].link.y = nr <= leaf_max ? range_link((uint32_t)(gamma + 1), nr) : kr;
    nodes[i].link.w = (uint32_t)(hi - lo + 1);  // primitives under node i (reachability test)
    kids[i] = make_uint2(kl, kr);
  }
}

// A child box travels to the parent as three 8-byte {lo, hi} pairs (x and y in the node's
// interleaved xy words, z in its z words), each stored write-through (sc1) by one agent-scope
// relaxed atomic store and read back by agent-scope loads: the hand-off form of the gfx950 guide
// (Guideline 16, R1) with every payload store sc1 and drained and every payload load sc1, so neither
// a release fence (an L2 write-back per level per thread) nor an acquire fence is needed.
__device__ __forceinline__ void st_pair(float* p, float lo, float hi) {
  const unsigned long long v = (unsigned long long)__float_as_uint(lo) | ((unsigned long long)__float_as_uint(hi) << 32);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ld_pair(const float* p, float& lo, float& hi) {
  const unsigned long long v =
      __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  lo = __uint_as_float((uint32_t)v);
  hi = __uint_as_float((uint32_t)(v >> 32));
}

// Each leaf walks up; at each node the first arriving child stops, the second merges both child
// boxes and continues.  The arrival word doubles as the height hand-off: a child arriving swaps in
// its subtree height + 1 (never 0), so the first arriver reads 0 and stops, and the second reads
// its sibling's height.  The tree height — the deepest leaf, which sizes the traversal stack — is
// the root's height, without a per-leaf walk to the root.
__global__ void k_refit(int N, const uint32_t* vals, const float4* blo, const float4* bhi, const uint2* kids,
                        const uint32_t* leaf_parent, BvhNode* nodes, uint32_t* flags, uint32_t* max_depth) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) {
    const uint32_t prim = vals[i];
    const float4 a = blo[prim], b = bhi[prim];
    float lo[3] = {a.x, a.y, a.z}, hi[3] = {b.x, b.y, b.z};
    uint32_t child = kLeafBit | (uint32_t)i;
    uint32_t par = leaf_parent[i];
    uint32_t h = 0u;  // height of the subtree rooted at `child` (a primitive: 0)
    for (;;) {
      BvhNode* nd = nodes + par;
      const bool left = (kids[par].x == child);
      // lxy = f[0..3], rxy = f[4..7], z = f[8..11]; own pairs at `m`, the sibling's at `o`
      float* f = reinterpret_cast<float*>(nd);
      float* m = f + (left ? 0 : 4);
      float* o = f + (left ? 4 : 0);
      float* mz = f + (left ? 8 : 10);
      float* oz = f + (left ? 10 : 8);
      st_pair(m, lo[0], hi[0]);
      st_pair(m + 2, lo[1], hi[1]);
      st_pair(mz, lo[2], hi[2]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // payload drained before the signal
      const uint32_t old = __hip_atomic_exchange(flags + par, h + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == 0u) break;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below
      h = max(h, old - 1u) + 1u;
      float sl[3], sh[3];
      ld_pair(o, sl[0], sh[0]);
      ld_pair(o + 2, sl[1], sh[1]);
      ld_pair(oz, sl[2], sh[2]);
      for (int k = 0; k < 3; ++k) {
        // fminf/fmaxf are symmetric, so the merged box does not depend on which child arrived last
        lo[k] = fminf(lo[k], sl[k]);
        hi[k] = fmaxf(hi[k], sh[k]);
      }
      if (par == 0u) {
        *max_depth = h;  // only the second arriver at the root gets here
        break;
      }
      child = par;
      par = nd->link.z;
    }
  }
}

// ---------------------------------------------------------------------------- treelet restructuring
// SAH optimisation of the Karras tree by treelet restructuring (Karras & Aila, "Fast Parallel
// Construction of High-Quality Bounding Volume Hierarchies", HPG 2013), for the scenes traversed from
// L2/HBM (single-primitive leaves).  Bottom-up, one launch per subtree height: every node of height h
// grows a treelet of up to kTreeletLeaves leaves below it (repeatedly opening the treelet leaf with the
// largest surface area), finds the treelet topology of least SAH cost over all subsets of its leaves
// (dynamic programming, subsets in increasing order, each split enumerated once), and rewrites the
// treelet's internal nodes if that beats the current topology.  A node's treelet lies inside its own
// subtree, whose nodes all have smaller heights and were finalised by earlier launches, and the
// treelets of one launch are disjoint, so the launches need no synchronisation beyond their order.
// Primitives do not move: only links, child boxes, parents and counts change.  SAH constants: a node
// visit 1.2, a primitive test 1 (per primitive of a leaf), areas as half surface areas.
constexpr float kSahNode = 1.2f, kSahPrim = 1.0f;
constexpr int kTreeletBlock = 64;

struct Box3 {
  float lo[3], hi[3];
};
__device__ __forceinline__ float half_area(const Box3& b) {
  const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  return dx * dy + dy * dz + dz * dx;
}
__device__ __forceinline__ Box3 node_child_box(const BvhNode& n, bool right) {
  Box3 b;
  const float4 xy = right ? n.rxy : n.lxy;
  b.lo[0] = xy.x;
  b.hi[0] = xy.y;
  b.lo[1] = xy.z;
  b.hi[1] = xy.w;
  b.lo[2] = right ? n.z.z : n.z.x;
  b.hi[2] = right ? n.z.w : n.z.y;
  return b;
}
__device__ __forceinline__ void box_merge(Box3& a, const Box3& b) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    a.lo[k] = fminf(a.lo[k], b.lo[k]);
    a.hi[k] = fmaxf(a.hi[k], b.hi[k]);
  }
}
__device__ __forceinline__ Box3 box_empty() {
  Box3 b;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    b.lo[k] = FLT_MAX;
    b.hi[k] = -FLT_MAX;
  }
  return b;
}
__device__ __forceinline__ uint32_t prims_of(uint32_t link) { return (link & kLeafRangeMask) + 1u; }

// Subtree heights of the Karras tree (the launch order of the first pass): each primitive walks up,
// the first child to arrive at a node stops, the second carries max(heights) + 1 on.  The payload is
// the value of the arrival word itself, so no other data crosses between threads.
__global__ void k_heights(int N, const uint32_t* leaf_parent, const BvhNode* nodes, uint32_t* flags, uint32_t* height) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) {
    uint32_t par = leaf_parent[i], h = 0u;
    for (;;) {
      const uint32_t old = __hip_atomic_exchange(flags + par, h + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == 0u) break;
      h = max(h, old - 1u) + 1u;
      height[par] = h;
      if (par == 0u) break;
      par = nodes[par].link.z;
    }
  }
}

// Nodes grouped by height (the launch order of a pass): a counting sort over kHeightBlocks blocks,
// each owning a contiguous range of nodes — per-block histograms (height-major table), an exclusive
// scan of the table on the host, then each block scatters its range from its own offsets with LDS
// counters.  (r03: a single global cursor per height took one atomic per height per wave, ~150 K
// atomics on the few bottom heights' words: 14 ms of a 10M-triangle build, per pass.)
constexpr uint32_t kMaxHeight = 256;
constexpr uint32_t kHeightBlocks = 512;
__global__ void k_height_count(uint32_t nn, uint32_t per, const uint32_t* label, uint32_t* bh) {
  __shared__ uint32_t s_h[kMaxHeight];
  for (uint32_t i = threadIdx.x; i < kMaxHeight; i += blockDim.x) s_h[i] = 0u;
  __syncthreads();
  const uint32_t lo = blockIdx.x * per, hi = min(nn, lo + per);
  for (uint32_t x = lo + threadIdx.x; x < hi; x += blockDim.x) atomicAdd(&s_h[min(label[x], kMaxHeight - 1u)], 1u);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < kMaxHeight; i += blockDim.x) bh[(size_t)i * gridDim.x + blockIdx.x] = s_h[i];
}
__global__ void k_height_scatter(uint32_t nn, uint32_t per, const uint32_t* label, const uint32_t* boff, uint32_t* order) {
  __shared__ uint32_t s_run[kMaxHeight];
  for (uint32_t i = threadIdx.x; i < kMaxHeight; i += blockDim.x) s_run[i] = boff[(size_t)i * gridDim.x + blockIdx.x];
  __syncthreads();
  const uint32_t lane = __lane_id();
  const uint32_t lo = blockIdx.x * per, hi = min(nn, lo + per);
  for (uint32_t base = lo; base < hi; base += blockDim.x) {
    const uint32_t x = base + threadIdx.x;
    const bool valid = x < hi;
    const uint32_t h = valid ? min(label[x], kMaxHeight - 1u) : 0u;
    unsigned long long todo = __ballot(valid);
    while (todo) {
      const int leader = __ffsll(todo) - 1;
      const uint32_t hl = __shfl(h, leader);
      const unsigned long long m = __ballot(valid && h == hl) & todo;
      uint32_t b = 0u;
      if ((int)lane == leader) b = atomicAdd(&s_run[hl], (uint32_t)__popcll(m));
      b = __shfl(b, leader);
      if ((m >> lane) & 1ull) order[b + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = x;
      todo &= ~m;
    }
  }
}

template <int K>
__global__ void __launch_bounds__(kTreeletBlock) k_treelet(const uint32_t* order, uint32_t count, BvhNode* nodes,
                                                            float* cost, uint32_t* newh, uint32_t* leaf_parent) {
  constexpr int S = 1 << K;
  __shared__ float s_copt[S][kTreeletBlock];     // least SAH cost of a subset of the treelet's leaves
  __shared__ uint16_t s_part[S][kTreeletBlock];  // its best split (low byte) and height (high byte)
  __shared__ uint8_t s_sub[K][kTreeletBlock];    // restructuring work list: subsets, node ids, parents
  __shared__ uint32_t s_id[K][kTreeletBlock];
  const int t = threadIdx.x;
  for (uint32_t i = blockIdx.x * blockDim.x + t; i < count; i += gridDim.x * blockDim.x) {
    const uint32_t x = order[i];
    const BvhNode nd = nodes[x];
    // treelet leaves (registers, fully unrolled) and internal nodes (inter[0] = x)
    uint32_t lk[K], lh[K], lc[K], inter[K];
    Box3 lb[K];
    float la[K], lcost[K];
    int nl = 2;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      lk[j] = kNoHit;
      lh[j] = lc[j] = inter[j] = 0u;
      la[j] = lcost[j] = 0.0f;
      lb[j] = box_empty();
    }
    inter[0] = x;
    lk[0] = nd.link.x;
    lk[1] = nd.link.y;
    lb[0] = node_child_box(nd, false);
    lb[1] = node_child_box(nd, true);
    la[0] = half_area(lb[0]);
    la[1] = half_area(lb[1]);
    for (int ni = 1; nl < K; ++ni) {
      int best = -1;
      float ba = -1.0f;
#pragma unroll
      for (int j = 0; j < K; ++j)
        if (j < nl && !(lk[j] & kLeafBit) && la[j] > ba) {
          ba = la[j];
          best = j;
        }
      if (best < 0) break;
      uint32_t m = 0u;
#pragma unroll
      for (int j = 0; j < K; ++j)
        if (j == best) m = lk[j];
      const BvhNode c = nodes[m];
      const Box3 bl = node_child_box(c, false), br = node_child_box(c, true);
#pragma unroll
      for (int j = 0; j < K; ++j) {
        if (j == best) {
          lk[j] = c.link.x;
          lb[j] = bl;
          la[j] = half_area(bl);
        }
        if (j == nl) {
          lk[j] = c.link.y;
          lb[j] = br;
          la[j] = half_area(br);
        }
        if (j == ni) inter[j] = m;
      }
      ++nl;
    }
    // leaf costs, heights and primitive counts
#pragma unroll
    for (int j = 0; j < K; ++j) {
      if (j >= nl) continue;
      if (lk[j] & kLeafBit) {
        lc[j] = prims_of(lk[j]);
        lcost[j] = kSahPrim * (float)lc[j] * la[j];
        lh[j] = 0u;
      } else {
        lc[j] = nodes[lk[j]].link.w;
        lcost[j] = cost[lk[j]];
        lh[j] = newh[lk[j]];
      }
    }
    const int full = (1 << nl) - 1;
    // the current topology's cost: the node over its two children
    Box3 ball = lb[0];
#pragma unroll
    for (int j = 1; j < K; ++j)
      if (j < nl) box_merge(ball, lb[j]);
    const float a_full = half_area(ball);
    float cur_l, cur_r;
    uint32_t h_l, h_r;
    if (nd.link.x & kLeafBit) {
      const Box3 b = node_child_box(nd, false);
      cur_l = kSahPrim * (float)prims_of(nd.link.x) * half_area(b);
      h_l = 0u;
    } else {
      cur_l = cost[nd.link.x];
      h_l = newh[nd.link.x];
    }
    if (nd.link.y & kLeafBit) {
      const Box3 b = node_child_box(nd, true);
      cur_r = kSahPrim * (float)prims_of(nd.link.y) * half_area(b);
      h_r = 0u;
    } else {
      cur_r = cost[nd.link.y];
      h_r = newh[nd.link.y];
    }
    const float cur = kSahNode * a_full + cur_l + cur_r;
    if (nl <= 2) {  // nothing to rearrange
      cost[x] = cur;
      newh[x] = max(h_l, h_r) + 1u;
      continue;
    }
    // dynamic programming over the leaf subsets
    for (int sb = 1; sb <= full; ++sb) {
      if ((sb & (sb - 1)) == 0) {  // one leaf
        float c = 0.0f;
        uint32_t h = 0u;
#pragma unroll
        for (int j = 0; j < K; ++j)
          if (sb == (1 << j)) {
            c = lcost[j];
            h = lh[j];
          }
        s_copt[sb][t] = c;
        s_part[sb][t] = (uint16_t)(h << 8);
        continue;
      }
      Box3 b = box_empty();
#pragma unroll
      for (int j = 0; j < K; ++j)
        if ((sb >> j) & 1) box_merge(b, lb[j]);
      const int low = sb & -sb;
      float best = FLT_MAX;
      int bp = 0;
      for (int q = (sb - 1) & sb; q > 0; q = (q - 1) & sb) {
        if (!(q & low)) continue;
        const float c = s_copt[q][t] + s_copt[sb ^ q][t];
        if (c < best) {
          best = c;
          bp = q;
        }
      }
      const uint32_t h = max(s_part[bp][t] >> 8, s_part[sb ^ bp][t] >> 8) + 1u;
      s_copt[sb][t] = kSahNode * half_area(b) + best;
      s_part[sb][t] = (uint16_t)((h << 8) | (uint32_t)bp);
    }
    const float opt = s_copt[full][t];
    // kept unless cheaper and no deeper: the traversal stacks are sized by the tree height (the wide
    // collapse of a deeper tree can exceed the BVH4 stack bound, sptr_internal.h kStack)
    const uint32_t h_old = max(h_l, h_r) + 1u, h_new = (uint32_t)(s_part[full][t] >> 8);
    if (!(opt < cur * 0.99999f) || h_new > h_old) {
      cost[x] = cur;
      newh[x] = max(h_l, h_r) + 1u;
      continue;
    }
    // rewrite the treelet's internal nodes top-down; the root keeps its id and parent
    s_sub[0][t] = (uint8_t)full;
    s_id[0][t] = x;
    int n = 1;
    const uint32_t parent_x = nd.link.z;
    for (int k = 0; k < n; ++k) {
      const int sb = s_sub[k][t];
      const uint32_t id = s_id[k][t];
      const int p = s_part[sb][t] & 0xFF, qs = sb ^ p;
      uint32_t link[2], cnt = 0u;
      Box3 bx[2];
      for (int side = 0; side < 2; ++side) {
        const int ts = side ? qs : p;
        bx[side] = box_empty();
        uint32_t c = 0u, lkj = 0u;
#pragma unroll
        for (int j = 0; j < K; ++j)
          if ((ts >> j) & 1) {
            box_merge(bx[side], lb[j]);
            c += lc[j];
            lkj = lk[j];
          }
        cnt += c;
        if ((ts & (ts - 1)) == 0) {
          link[side] = lkj;  // a treelet leaf keeps its link (and its subtree), under a new parent
          if (!(lkj & kLeafBit)) nodes[lkj].link.z = id;
          else leaf_parent[(lkj & ~kLeafBit) >> kLeafCountBits] = id;
        } else {
          uint32_t cid = 0u;
#pragma unroll
          for (int j = 0; j < K; ++j)
            if (j == n) cid = inter[j];
          s_sub[n][t] = (uint8_t)ts;
          s_id[n][t] = cid;
          ++n;
          link[side] = cid;
          nodes[cid].link.z = id;
        }
      }
      BvhNode o;
      o.lxy = make_float4(bx[0].lo[0], bx[0].hi[0], bx[0].lo[1], bx[0].hi[1]);
      o.rxy = make_float4(bx[1].lo[0], bx[1].hi[0], bx[1].lo[1], bx[1].hi[1]);
      o.z = make_float4(bx[0].lo[2], bx[0].hi[2], bx[1].lo[2], bx[1].hi[2]);
      o.link = make_uint4(link[0], link[1], k == 0 ? parent_x : nodes[id].link.z, cnt);
      nodes[id] = o;
      cost[id] = s_copt[sb][t];
      newh[id] = (uint32_t)(s_part[sb][t] >> 8);
    }
  }
}

struct WideBoxes {
  float lo[3][kWide], hi[3][kWide];
  uint32_t link[kWide];
};

// Quantise the n child boxes of one wide node (WideNode): per axis, org = the smallest lower
// plane, step 2^e the smallest power of two (e in [-100, 60]) with extent <= 255 * 2^e, qlo =
// floor((lo - org) / 2^e) and qhi = ceil((hi - org) / 2^e) evaluated in double (exact for the
// scene's float coordinates), so the decoded box always contains the child box.
__device__ __forceinline__ WideNode quantize_wide(const WideBoxes& b, int n, uint32_t parent) {
  WideNode o;
  float org[3];
  uint32_t ex = (uint32_t)n << 24;
  for (int w = 0; w < 6; ++w)
    for (int j = 0; j < kQWords; ++j) o.q[w][j] = 0u;
  for (int a = 0; a < 3; ++a) {
    float mn = b.lo[a][0], mx = b.hi[a][0];
    for (int k = 1; k < n; ++k) {
      mn = fminf(mn, b.lo[a][k]);
      mx = fmaxf(mx, b.hi[a][k]);
    }
    org[a] = mn;
    const double ext = (double)mx - (double)mn;
    int e = -100;
    if (ext > 0.0) {
      int x;
      (void)frexp(ext / 255.0, &x);  // ext / 255 in (2^(x-1), 2^x]
      e = x;
      if (ext <= 255.0 * ldexp(1.0, e - 1)) --e;
      e = e < -100 ? -100 : (e > 60 ? 60 : e);
    }
    ex |= (uint32_t)(e + 127) << (8 * a);
    const double inv_step = ldexp(1.0, -e);
    for (int k = 0; k < n; ++k) {
      double l = floor(((double)b.lo[a][k] - (double)mn) * inv_step), h = ceil(((double)b.hi[a][k] - (double)mn) * inv_step);
      l = l < 0.0 ? 0.0 : (l > 255.0 ? 255.0 : l);
      h = h < 0.0 ? 0.0 : (h > 255.0 ? 255.0 : h);
      o.q[2 * a][k / 4] |= (uint32_t)l << (8 * (k % 4));
      o.q[2 * a + 1][k / 4] |= (uint32_t)h << (8 * (k % 4));
    }
  }
  o.ox = org[0];
  o.oy = org[1];
  o.oz = org[2];
  o.ex = ex;
  for (int k = 0; k < kWide; ++k) o.link[k] = b.link[k];
  o.parent = parent;
  for (uint32_t& x : o.pad) x = 0u;
  return o;
}

// Greedy surface-area collapse, top-down one wide level per launch pair: a wide
// node's child list starts as its BVH2 node's two children and grows, up to kWide entries, by
// opening the internal entry whose box has the largest surface area (lowest slot on ties) — it is
// replaced in place by its left and right children, so the list stays in left-to-right order.
// Unlike a fixed two-level collapse this fills nodes whose grandchildren include leaves and spends
// the wide levels where the big boxes are, so deep LBVH chains give shallower wide trees.
// Its internal entries become the next level's wide nodes.
__device__ __forceinline__ float box_area(const WideBoxes& b, int e) {
  const float dx = b.hi[0][e] - b.lo[0][e], dy = b.hi[1][e] - b.lo[1][e], dz = b.hi[2][e] - b.lo[2][e];
  return dx * dy + dy * dz + dz * dx;
}
__device__ __forceinline__ void put_child(WideBoxes& b, int e, const BvhNode& nd, bool right) {
  if (!right) {
    b.link[e] = nd.link.x;
    b.lo[0][e] = nd.lxy.x; b.hi[0][e] = nd.lxy.y; b.lo[1][e] = nd.lxy.z; b.hi[1][e] = nd.lxy.w;
    b.lo[2][e] = nd.z.x;   b.hi[2][e] = nd.z.y;
  } else {
    b.link[e] = nd.link.y;
    b.lo[0][e] = nd.rxy.x; b.hi[0][e] = nd.rxy.y; b.lo[1][e] = nd.rxy.z; b.hi[1][e] = nd.rxy.w;
    b.lo[2][e] = nd.z.z;   b.hi[2][e] = nd.z.w;
  }
}
__device__ int expand_greedy(const BvhNode* nodes, uint32_t node, WideBoxes& b) {
  for (int k = 0; k < kWide; ++k) {
    b.link[k] = kNoHit;
    for (int a = 0; a < 3; ++a) b.lo[a][k] = b.hi[a][k] = 0.0f;
  }
  const BvhNode nd = nodes[node];
  put_child(b, 0, nd, false);
  put_child(b, 1, nd, true);
  int n = 2;
  while (n < kWide) {
    int best = -1;
    float ba = -1.0f;
    for (int e = 0; e < n; ++e)
      if (!(b.link[e] & kLeafBit)) {
        const float a = box_area(b, e);
        if (a > ba) {
          ba = a;
          best = e;
        }
      }
    if (best < 0) break;
    const BvhNode cn = nodes[b.link[best]];
    for (int e = n; e > best + 1; --e) {
      b.link[e] = b.link[e - 1];
      for (int a = 0; a < 3; ++a) {
        b.lo[a][e] = b.lo[a][e - 1];
        b.hi[a][e] = b.hi[a][e - 1];
      }
    }
    put_child(b, best, cn, false);
    put_child(b, best + 1, cn, true);
    ++n;
  }
  return n;
}
// pass 1: internal children per wide node of this level (cur[j] = {BVH2 node, parent wide index})
__global__ void k_wide_count(uint32_t ncur, const uint2* cur, const BvhNode* nodes, uint32_t* cnt) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < ncur; j += gridDim.x * blockDim.x) {
    WideBoxes b;
    const int n = expand_greedy(nodes, cur[j].x, b);
    uint32_t m = 0u;
    for (int e = 0; e < n; ++e) m += (b.link[e] & kLeafBit) ? 0u : 1u;
    cnt[j] = m;
  }
}
// pass 2: wide node base + j; its m-th internal child becomes next[off[j] + m] = wide node
// base + ncur + off[j] + m of the next level
// Single-primitive leaf children become direct links (the primitive's ref in the link: its test
// needs no prim_ref load; r03: C5 13.58 -> 12.29 ms/step).
__global__ void k_wide_emit(uint32_t ncur, const uint2* cur, uint32_t base, const BvhNode* nodes, const uint32_t* off,
                            uint2* next, WideNode* out, const uint32_t* prim_ref) {
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < ncur; j += gridDim.x * blockDim.x) {
    WideBoxes b;
    const int n = expand_greedy(nodes, cur[j].x, b);
    uint32_t m = off[j];
    for (int e = 0; e < n; ++e)
      if (!(b.link[e] & kLeafBit)) {
        next[m] = make_uint2(b.link[e], base + j);
        b.link[e] = base + ncur + m;
        ++m;
      } else if ((b.link[e] & kLeafRangeMask) == 0u) {
        const uint32_t ref = prim_ref[(b.link[e] & ~kLeafBit) >> kLeafCountBits];
        b.link[e] = kLeafBit | ((ref & kIndexMask) << kLeafCountBits) | kLeafDirect |
                    ((ref & kSphereBit) ? kLeafDirectSphere : 0u);
      }
    out[base + j] = quantize_wide(b, n, cur[j].y);
  }
}

struct Tmp {
  std::vector<void*> ptrs;
  ~Tmp() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  template <class T>
  hipError_t alloc(T** p, size_t n) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, n ? n * sizeof(T) : 16);
    if (e == hipSuccess) ptrs.push_back(q);
    *p = static_cast<T*>(q);
    return e;
  }
};

hipError_t realloc_buf(DevBuf& b, size_t bytes) {
  if (b.p && b.bytes >= bytes) return hipSuccess;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  hipError_t e = hipMalloc(&b.p, bytes ? bytes : 16);
  if (e == hipSuccess) b.bytes = bytes ? bytes : 16;
  return e;
}

unsigned blocks_for(size_t n) {
  size_t b = (n + 255) / 256;
  if (b < 1) b = 1;
  if (b > 4096) b = 4096;
  return (unsigned)b;
}

}  // namespace

int build_lbvh(Context& c, const float* h_pos, uint32_t nverts, const uint32_t* h_idx, uint32_t ntris,
               const float* h_sph, uint32_t nsph, const uint32_t* h_tri_geom, uint32_t sph_geom_base) {
  const auto t0 = std::chrono::steady_clock::now();
  hipStream_t s = c.stream;
  const uint32_t NP = ntris + nsph;
  c.num_tris = ntris;
  c.num_sph = nsph;
  c.bvh_depth = 0;
  if (NP == 0) {
    c.num_nodes = 0;
    c.num_tri_refs = 0;
    c.root = kNoHit;
    c.root4 = kNoHit;
    c.num_nodes4 = 0;
    c.num_top4 = 0;
    c.stack_need2 = c.stack_need4 = 0;
    return SPTR_OK;
  }
  Tmp tmp;
  float* d_pos = nullptr;
  uint32_t *d_idx = nullptr, *d_tg = nullptr;
  float4* d_sph = nullptr;
  LB_CHECK(tmp.alloc(&d_pos, (size_t)nverts * 3));
  LB_CHECK(tmp.alloc(&d_idx, (size_t)ntris * 3));
  LB_CHECK(tmp.alloc(&d_tg, (size_t)ntris));
  LB_CHECK(tmp.alloc(&d_sph, (size_t)nsph));
  if (nverts) LB_CHECK(hipMemcpyAsync(d_pos, h_pos, (size_t)nverts * 12, hipMemcpyHostToDevice, s));
  if (ntris) {
    LB_CHECK(hipMemcpyAsync(d_idx, h_idx, (size_t)ntris * 12, hipMemcpyHostToDevice, s));
    LB_CHECK(hipMemcpyAsync(d_tg, h_tri_geom, (size_t)ntris * 4, hipMemcpyHostToDevice, s));
  }
  if (nsph) LB_CHECK(hipMemcpyAsync(d_sph, h_sph, (size_t)nsph * 16, hipMemcpyHostToDevice, s));
  BuildIn in{d_pos, d_idx, d_sph, d_tg, ntris, nsph, sph_geom_base};

  // primitive boxes, then the references: one per primitive, or 2^D pieces of a split triangle.
  // Scenes small enough to be staged in LDS (C1, C2, C4) are never split (the estimate of their
  // staged bytes is the automatic leaf-size rule's, below).
  float4 *pblo = nullptr, *pbhi = nullptr;
  uint32_t *rcnt = nullptr, *roff = nullptr;
  LB_CHECK(tmp.alloc(&pblo, NP));
  LB_CHECK(tmp.alloc(&pbhi, NP));
  LB_CHECK(tmp.alloc(&rcnt, NP));
  LB_CHECK(tmp.alloc(&roff, NP));
  hipLaunchKernelGGL(k_prim_bounds, dim3(blocks_for(NP)), dim3(256), 0, s, in, pblo, pbhi);
  const bool small = ((uint64_t)(NP - 1) * 64 + (uint64_t)ntris * 48 + (uint64_t)nsph * 16 + ((uint64_t)NP + 3) / 4 * 16) <=
                     kLdsSceneBytes;
  const uint32_t max_pieces = (small || (c.leaf_size != 0 && c.leaf_size != 1))
                                  ? 1u : std::min<uint32_t>(c.split_pieces, 1u << kMaxSplitDepth);
  hipLaunchKernelGGL(k_split_count, dim3(blocks_for(NP)), dim3(256), 0, s, in, pblo, pbhi, max_pieces, rcnt);
  size_t rbytes = 0;
  LB_CHECK(scan_u32(nullptr, rbytes, rcnt, roff, NP, s));
  void* rstore = nullptr;
  LB_CHECK(tmp.alloc(reinterpret_cast<char**>(&rstore), rbytes));
  LB_CHECK(scan_u32(rstore, rbytes, rcnt, roff, NP, s));
  uint32_t last2[2] = {0u, 0u};
  LB_CHECK(hipMemcpyAsync(&last2[0], rcnt + (NP - 1), 4, hipMemcpyDeviceToHost, s));
  LB_CHECK(hipMemcpyAsync(&last2[1], roff + (NP - 1), 4, hipMemcpyDeviceToHost, s));
  LB_CHECK(hipStreamSynchronize(s));
  const uint64_t NR64 = (uint64_t)last2[0] + last2[1];
  if (NR64 >= (1ull << (31 - kLeafCountBits)))
    return (c.err = "lbvh: too many primitive references (" + std::to_string(NR64) + ")", SPTR_ERR_INVALID);
  const uint32_t NR = (uint32_t)NR64;
  const uint32_t ntri_refs = NR - nsph;  // spheres keep one reference each
  c.num_tri_refs = ntri_refs;
  c.num_nodes = NR > 1 ? NR - 1 : 0;
  // + 64 B: the unified wide walk (wide_walk_u) reads a node's 56 B from a direct leaf's primitive address
  LB_CHECK(realloc_buf(c.tris, (size_t)ntri_refs * 48 + 64));
  LB_CHECK(realloc_buf(c.tri_geom, (size_t)ntri_refs * 4));
  LB_CHECK(realloc_buf(c.tri_orig, (size_t)ntri_refs * 4));
  LB_CHECK(realloc_buf(c.sph, (size_t)nsph * 16 + 64));
  LB_CHECK(realloc_buf(c.sph_geom, (size_t)nsph * 4));
  LB_CHECK(realloc_buf(c.sph_orig, (size_t)nsph * 4));
  LB_CHECK(realloc_buf(c.nodes, (size_t)c.num_nodes * sizeof(BvhNode)));
  LB_CHECK(realloc_buf(c.prim_ref, ((size_t)NR + 3) / 4 * 16));

  float4 *blo = nullptr, *bhi = nullptr;
  uint32_t* cb = nullptr;
  uint64_t *keys = nullptr, *keys_s = nullptr;
  uint32_t *rprim = nullptr, *vals = nullptr, *vals_s = nullptr, *flag = nullptr, *slot = nullptr, *leaf_parent = nullptr,
           *rflags = nullptr, *dmax = nullptr;
  uint2* kids = nullptr;
  LB_CHECK(tmp.alloc(&blo, NR));
  LB_CHECK(tmp.alloc(&bhi, NR));
  LB_CHECK(tmp.alloc(&rprim, NR));
  LB_CHECK(tmp.alloc(&cb, 8));
  LB_CHECK(tmp.alloc(&keys, NR));
  LB_CHECK(tmp.alloc(&keys_s, NR));
  LB_CHECK(tmp.alloc(&vals, NR));
  LB_CHECK(tmp.alloc(&vals_s, NR));
  LB_CHECK(tmp.alloc(&flag, NR));
  LB_CHECK(tmp.alloc(&slot, NR));
  LB_CHECK(tmp.alloc(&kids, NR));
  LB_CHECK(tmp.alloc(&leaf_parent, NR));
  LB_CHECK(tmp.alloc(&rflags, NR));
  LB_CHECK(tmp.alloc(&dmax, 1));
  hipLaunchKernelGGL(k_split_emit, dim3(blocks_for(NP)), dim3(256), 0, s, in, pblo, pbhi, rcnt, roff, blo, bhi, rprim);
  const uint32_t cb_init[8] = {~0u, ~0u, ~0u, 0u, 0u, 0u, 0u, 0u};
  LB_CHECK(hipMemcpyAsync(cb, cb_init, sizeof(cb_init), hipMemcpyHostToDevice, s));
  LB_CHECK(hipMemsetAsync(dmax, 0, 4, s));
  hipLaunchKernelGGL(k_ref_bounds, dim3(blocks_for(NR)), dim3(256), 0, s, NR, blo, bhi, cb);
  hipLaunchKernelGGL(k_morton, dim3(blocks_for(NR)), dim3(256), 0, s, in, NR, blo, bhi, rprim, cb, keys, vals, dmax);
  LB_CHECK(hipGetLastError());
  size_t tbytes = 0;
  LB_CHECK(radix_sort_pairs_u64(nullptr, tbytes, keys, keys_s, vals, vals_s, NR, s));
  void* tstore = nullptr;
  LB_CHECK(tmp.alloc(reinterpret_cast<char**>(&tstore), tbytes));
  LB_CHECK(radix_sort_pairs_u64(tstore, tbytes, keys, keys_s, vals, vals_s, NR, s));
  hipLaunchKernelGGL(k_is_tri, dim3(blocks_for(NR)), dim3(256), 0, s, NR, ntris, vals_s, rprim, flag);
  size_t sbytes = 0;
  LB_CHECK(scan_u32(nullptr, sbytes, flag, slot, NR, s));
  void* sstore = nullptr;
  LB_CHECK(tmp.alloc(reinterpret_cast<char**>(&sstore), sbytes));
  LB_CHECK(scan_u32(sstore, sbytes, flag, slot, NR, s));
  hipLaunchKernelGGL(k_leaves, dim3(blocks_for(NR)), dim3(256), 0, s, in, NR, vals_s, rprim, slot,
                     static_cast<float4*>(c.tris.p), static_cast<uint32_t*>(c.tri_geom.p),
                     static_cast<uint32_t*>(c.tri_orig.p), static_cast<float4*>(c.sph.p),
                     static_cast<uint32_t*>(c.sph_geom.p), static_cast<uint32_t*>(c.sph_orig.p),
                     static_cast<uint32_t*>(c.prim_ref.p));
  LB_CHECK(hipGetLastError());
  // the tree covers the first N sorted primitives: all but the exactly degenerate triangles (k_morton),
  // unless every primitive is one
  uint32_t ndeg = 0;
  LB_CHECK(hipMemcpyAsync(&ndeg, dmax, 4, hipMemcpyDeviceToHost, s));
  LB_CHECK(hipStreamSynchronize(s));
  LB_CHECK(hipMemsetAsync(dmax, 0, 4, s));
  const uint32_t N = ndeg < NR ? NR - ndeg : NR;
  c.excluded_prims = NR - N;
  c.num_nodes = N > 1 ? N - 1 : 0;
  // automatic leaf size (measured, profiles/r01*, r02g_leaf.txt): ranges of 8 for scenes small enough
  // to be staged in LDS (fewer, divergence-free node steps), single primitives for meshes traversed
  // from L2/HBM (with the greedy wide collapse: C5 14.9 -> 13.9, C3 5.04 -> 4.87 ms/step vs 2)
  const uint32_t auto_leaf = ((uint64_t)(N > 1 ? N - 1 : 0) * 64 + (uint64_t)ntri_refs * 48 + (uint64_t)nsph * 16 +
                              ((uint64_t)N + 3) / 4 * 16) <= kLdsSceneBytes ? 8u : 1u;
  const uint32_t leaf_max = std::max(1u, std::min(c.leaf_size ? c.leaf_size : auto_leaf, kMaxLeafSize));
  c.leaf_used = leaf_max;
  if (N == 1) {
    c.root = kLeafBit | 0u;  // range [0, 1)
    c.root4 = c.root;
    c.num_nodes4 = 0;
    c.num_top4 = 0;
    c.bvh_depth = 0;
    c.stack_need2 = c.stack_need4 = 0;
  } else {
    BvhNode* nodes = static_cast<BvhNode*>(c.nodes.p);
    LB_CHECK(hipMemsetAsync(nodes, 0, (size_t)(N - 1) * sizeof(BvhNode), s));
    uint32_t dep = 0;
    {
      LB_CHECK(hipMemsetAsync(rflags, 0, (size_t)N * 4, s));
      hipLaunchKernelGGL(k_karras, dim3(blocks_for(N)), dim3(256), 0, s, (int)N, keys_s, leaf_max, nodes, kids,
                         leaf_parent);
      hipLaunchKernelGGL(k_refit, dim3(blocks_for(N)), dim3(256), 0, s, (int)N, vals_s, blo, bhi, kids, leaf_parent,
                         nodes, rflags, dmax);
      LB_CHECK(hipGetLastError());
      LB_CHECK(hipMemcpyAsync(&dep, dmax, 4, hipMemcpyDeviceToHost, s));
      LB_CHECK(hipStreamSynchronize(s));
      // SAH treelet restructuring (k_treelet) for the single-primitive-leaf trees of L2/HBM scenes:
      // launch h rewrites the nodes of height h; each pass's new heights order the next pass
      if (leaf_max == 1u && N >= 3u && c.treelet_passes > 0u) {
        uint32_t *lab = nullptr, *nh = nullptr, *order = nullptr, *hist = nullptr;
        float* cst = nullptr;
        LB_CHECK(tmp.alloc(&lab, N));
        LB_CHECK(tmp.alloc(&nh, N));
        LB_CHECK(tmp.alloc(&order, N));
        LB_CHECK(tmp.alloc(&hist, (size_t)kMaxHeight * kHeightBlocks));
        LB_CHECK(tmp.alloc(&cst, N));
        LB_CHECK(hipMemsetAsync(rflags, 0, (size_t)N * 4, s));
        hipLaunchKernelGGL(k_heights, dim3(blocks_for(N)), dim3(256), 0, s, (int)N, leaf_parent, nodes, rflags, lab);
        LB_CHECK(hipGetLastError());
        const uint32_t nn = N - 1u;
        std::vector<uint32_t> hh(kMaxHeight), off(kMaxHeight), bh((size_t)kMaxHeight * kHeightBlocks);
        const uint32_t per = (nn + kHeightBlocks - 1u) / kHeightBlocks;
        for (uint32_t pass = 0; pass < c.treelet_passes; ++pass) {
          hipLaunchKernelGGL(k_height_count, dim3(kHeightBlocks), dim3(256), 0, s, nn, per, lab, hist);
          LB_CHECK(hipMemcpyAsync(bh.data(), hist, bh.size() * 4, hipMemcpyDeviceToHost, s));
          LB_CHECK(hipStreamSynchronize(s));
          uint32_t run = 0u;  // exclusive scan of the height-major table: heights in order, blocks in order
          for (uint32_t h = 0; h < kMaxHeight; ++h) {
            off[h] = run;
            for (uint32_t b = 0; b < kHeightBlocks; ++b) {
              const uint32_t n = bh[(size_t)h * kHeightBlocks + b];
              bh[(size_t)h * kHeightBlocks + b] = run;
              run += n;
            }
            hh[h] = run - off[h];
          }
          LB_CHECK(hipMemcpyAsync(hist, bh.data(), bh.size() * 4, hipMemcpyHostToDevice, s));
          hipLaunchKernelGGL(k_height_scatter, dim3(kHeightBlocks), dim3(256), 0, s, nn, per, lab, hist, order);
          for (uint32_t h = 1; h < kMaxHeight; ++h)
            if (hh[h])
              hipLaunchKernelGGL(k_treelet<kTreeletLeaves>, dim3((hh[h] + kTreeletBlock - 1) / kTreeletBlock),
                                 dim3(kTreeletBlock), 0, s, order + off[h], hh[h], nodes, cst, nh, leaf_parent);
          LB_CHECK(hipGetLastError());
          LB_CHECK(hipMemcpyAsync(&dep, nh, 4, hipMemcpyDeviceToHost, s));  // the root's new height
          LB_CHECK(hipStreamSynchronize(s));
          std::swap(lab, nh);
        }
      }
    }
    c.root = N <= leaf_max ? (kLeafBit | (N - 1u)) : 0u;  // whole scene in one leaf range, or node 0
    c.bvh_depth = dep;
    // a BVH2 node at depth d holds at most d pushed entries and pushes one more; a wide node (BVH2
    // depth kWideLevels*dw) holds at most (kWide-1)*dw and pushes up to kWide-1 more; internal nodes
    // lie at BVH2 depth <= dep - 1
    c.stack_need2 = dep;
    c.stack_need4 = (uint32_t)(kWide - 1) * ((dep > 0u ? dep - 1u : 0u) / (uint32_t)kWideLevels + 1u);
    if (c.stack_need2 > (uint32_t)kStack) {
      c.err = "lbvh: tree depth " + std::to_string(dep) + " exceeds the traversal stack";
      return SPTR_ERR_INVALID;
    }
    if (c.root & kLeafBit) {
      c.num_nodes4 = 0;
      c.num_top4 = 0;
      c.root4 = c.root;
    } else {
      // wide BVH, greedy surface-area collapse, top-down: level L's wide nodes are numbered after
      // levels 0..L-1 (so the top kTopLevels levels come first); cnt -> exclusive scan -> emit
      uint2 *cur = nullptr, *nxt = nullptr;
      uint32_t* off = nullptr;
      LB_CHECK(tmp.alloc(&cur, N));
      LB_CHECK(tmp.alloc(&nxt, N));
      LB_CHECK(tmp.alloc(&off, N));
      size_t sw = 0;
      LB_CHECK(scan_u32(nullptr, sw, flag, off, N, s));
      void* stw = nullptr;
      LB_CHECK(tmp.alloc(reinterpret_cast<char**>(&stw), sw));
      LB_CHECK(realloc_buf(c.nodes4, (size_t)(N - 1) * sizeof(WideNode)));  // <= one wide node per BVH2 node
      const uint2 root2 = make_uint2(0u, kNoHit);
      LB_CHECK(hipMemcpyAsync(cur, &root2, sizeof(root2), hipMemcpyHostToDevice, s));
      uint32_t ncur = 1u, base = 0u, levels = 0u;
      c.num_top4 = 0u;
      while (ncur > 0u) {
        hipLaunchKernelGGL(k_wide_count, dim3(blocks_for(ncur)), dim3(256), 0, s, ncur, cur, nodes, flag);
        LB_CHECK(hipGetLastError());
        LB_CHECK(scan_u32(stw, sw, flag, off, ncur, s));
        hipLaunchKernelGGL(k_wide_emit, dim3(blocks_for(ncur)), dim3(256), 0, s, ncur, cur, base, nodes, off, nxt,
                           static_cast<WideNode*>(c.nodes4.p), static_cast<const uint32_t*>(c.prim_ref.p));
        LB_CHECK(hipGetLastError());
        uint32_t last[2] = {0u, 0u};  // cnt, off of the level's last node
        LB_CHECK(hipMemcpyAsync(&last[0], flag + (ncur - 1u), 4, hipMemcpyDeviceToHost, s));
        LB_CHECK(hipMemcpyAsync(&last[1], off + (ncur - 1u), 4, hipMemcpyDeviceToHost, s));
        LB_CHECK(hipStreamSynchronize(s));
        base += ncur;
        ++levels;
        if (levels == (uint32_t)kTopLevels) c.num_top4 = base;
        ncur = last[0] + last[1];
        std::swap(cur, nxt);
      }
      if (levels < (uint32_t)kTopLevels) c.num_top4 = base;
      c.num_nodes4 = base;
      // a wide node at wide depth d holds at most (kWide-1)*d stack entries and pushes up to kWide-1
      c.stack_need4 = (uint32_t)(kWide - 1) * levels;
      c.root4 = 0u;  // node 0 (depth 0) is kept and scans to index 0
    }
  }
  LB_CHECK(hipStreamSynchronize(s));
  c.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return SPTR_OK;
}

}  // namespace sptr
