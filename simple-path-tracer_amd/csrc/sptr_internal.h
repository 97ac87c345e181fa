// sptr_internal.h — device data layout and context of libsptr_hip (not part of the public ABI).
//
// HBM layout: dense SoA "float4 streams", one 16-B coalesced load per lane per stream.
//   path id      : p = sample_slot * P + local_pixel (local pixels tile-packed: 32x32 tiles of this
//                  shard, row-major inside a tile, so a wave64 covers two rows of one tile)
//   rad[p]       : radiance of path p (summed by k_accum in sample order)
//   ray streams  : rs[b] = {o.xyz|rng, d.xyz|p, thr.xyz} indexed by *queue slot*, ping-pong b = depth&1;
//                  written densely by k_shade, read densely by k_trace (no sparse gathers)
//   hit records  : hrec[slot] = (input slot or p, t bits, prim ref), written densely by k_trace
//   shadow tasks : stask[slot*L + i] = {origin.xyz, tfar} {contrib.xyz, p} [{dir.xyz}]
// Queues are *block segments*: a producer block that consumed input slice [lo, hi) writes its
// outputs densely to [lo*m, lo*m + n_b) (m = records per input) and publishes n_b in a segment
// table; consumers scan the table (one LDS scan per block) and map compacted index -> slot.  No
// global atomics on the data path, and every stream access is dense.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <utility>
#include <vector>

#include "sptr_hip.h"
#include "sptr_math.h"
#include "tile_map.h"

namespace sptr {

constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kSphereBit = 0x40000000u;
constexpr uint32_t kIndexMask = 0x3FFFFFFFu;
// Leaf link, two forms (bit kLeafDirect tells them apart):
//   range : kLeafBit | start << kLeafCountBits | (count - 1): a contiguous range of up to 16 sorted
//           primitive references (prim_ref[start .. start+count)).  Primitive ref: [kSphereBit] | slot.
//   direct: kLeafBit | slot << kLeafCountBits | kLeafDirect [| kLeafDirectSphere]: one primitive,
//           named in the link itself, so its test needs no prim_ref load.  The wide BVH's
//           single-primitive leaf children take this form (k_wide_emit); BVH2 leaves keep ranges.
constexpr uint32_t kLeafCountBits = 5;  // start / slot keep 26 bits: up to 64M primitives
constexpr uint32_t kLeafRangeMask = 0xFu;  // count - 1 of a range
constexpr uint32_t kLeafDirect = 0x10u;
constexpr uint32_t kLeafDirectSphere = 0x08u;
constexpr uint32_t kLeafCountMask = (1u << kLeafCountBits) - 1u;
constexpr uint32_t kMaxLeafSize = kLeafRangeMask + 1u;
constexpr uint32_t kNoHit = 0xFFFFFFFFu;
constexpr int kTile = 32;
constexpr int kTilePixels = kTile * kTile;
constexpr int kMaxLights = 8;
// Collapsed ("wide") BVH: 4 children per node (8-wide measured slower: C5 22.5 -> 28.6 ms/step, spills).
constexpr int kWide = 4;
constexpr int kWideLevels = 2;  // BVH2 levels per wide level
constexpr int kQWords = 1;      // u32 words per quantised plane, one byte per child
// The wide BVH's top kTopLevels levels (at most 1 + 4 + 16 = 21 nodes, 1.3 KB) take wide indices
// 0..num_top4-1, so a kernel can stage them in LDS and tell an LDS node by its index alone.
constexpr int kTopLevels = 3;
constexpr int kMaxDepth = 32;
// Traversal stack entries.  BVH2 pushes at most one entry per internal level, a wide BVH at most
// kWide - 1, so a tree of height h needs h (BVH2) or (kWide - 1) * ((h - 1) / kWideLevels + 1)
// (wide) entries; build_lbvh records both bounds, scene_view never picks a width whose bound
// exceeds kStack, and a push that would still overflow is dropped and reported
// (kTotStackOverflow), never silent.
constexpr int kStack = 96;
constexpr int kBlock = 256;
#ifndef SPTR_TREELET_PASSES
#define SPTR_TREELET_PASSES 3
#endif
constexpr uint32_t kLdsSceneBytes = 48 * 1024;  // scenes up to this size are staged whole into LDS

// BVH2 node, 64 B: both child boxes + child links.  Link: internal node index, or a leaf range.
struct BvhNode {
  float4 lxy;  // left  lo.x hi.x lo.y hi.y
  float4 rxy;  // right lo.x hi.x lo.y hi.y
  float4 z;    // left lo.z hi.z, right lo.z hi.z
  uint4 link;  // left, right, parent, pad
};
static_assert(sizeof(BvhNode) == 64, "node size");

// Wide BVH node (64 B = half a 128-B cache line): the child boxes
// quantised to 8 bits per plane on a per-node, per-axis power-of-two grid anchored at the node's
// lower corner (org).  Child k's box is [org + qlo_k * 2^e, org + qhi_k * 2^e] per axis, rounded
// outwards at build time (k_collapse_wide), so it contains the exact child box; traverse_wide
// decodes the planes in the ray's frame with an error pad, so the test stays conservative.
struct alignas(16) WideNode {
  float ox, oy, oz;
  uint32_t ex;               // biased exponent bytes of the x / y / z grid steps; byte 3: child count
  uint32_t link[kWide];      // child: internal node index | leaf range (kLeafBit) | kNoHit
  uint32_t q[6][kQWords];    // planes lo x, hi x, lo y, hi y, lo z, hi z; byte k % 4 of word k / 4
  uint32_t parent;           // wide-node index (build bookkeeping, not traversed)
  uint32_t pad[1];
};
static_assert(sizeof(WideNode) == 64, "node size");

struct DevMaterial {  // == sptr_material
  float albedo[3];
  float metallic;
  float roughness;
  float emission[3];
  float ior;
  int32_t type;
  float pad[2];
};
static_assert(sizeof(DevMaterial) == 48, "material size");

struct DevLight {  // host-precomputed per Light::getRadiance (Light.cpp:43-79)
  int32_t type;     // 0 directional, 1 point
  float v[3];       // direction TO the light (normalize(-d)), or position
  float radiance[3];  // color * intensity
  float pad;
};

struct SceneView {
  const BvhNode* nodes;
  const WideNode* nodes4;  // used when width == 4
  const uint32_t* prim_ref;  // sorted primitive refs (leaf ranges index this)
  const float4* tris;  // 3 float4 per sorted triangle: v0.xyz e1.x | e1.yz e2.xy | e2.z Ng.xyz
  const float4* sph;   // sorted spheres: c.xyz r
  const uint32_t* tri_geom;  // geomID per sorted triangle
  const uint32_t* sph_geom;  // geomID per sorted sphere
  uint32_t num_nodes, num_tris, num_sph, root;
  uint32_t num_nodes4, root4;
  uint32_t num_top4;   // wide nodes 0..num_top4-1 are the top kTopLevels levels (staged in LDS by the
                       // refilling kernels of scenes traversed from L2/HBM); 0 = none
  uint32_t width;      // 2: BVH2 traversal, 4: BVH4 traversal
  uint32_t lds_bytes;  // 0: traverse from global memory
  uint64_t scene_bytes;  // traversed nodes + triangles + spheres + refs
};

struct EnvView {
  const float4* env;  // 6*S*S texels (rgb, -) or null for the procedural sky
  int32_t env_size;
  float env_intensity, env_clamp;
  int32_t debug_mode;
};

struct ShadeView {
  const DevMaterial* mats;
  uint32_t num_mats;
  const uint32_t* geom_mat;  // geomID -> material index, resolved as MaterialManager::getMaterialFromHit
  // triangle slot -> material index (geom_mat[tri_geom[slot]], precomputed): scenes traversed from L2/HBM,
  // where the shading of a hit saves a dependent load; null elsewhere
  const uint32_t* tri_mat;
  uint32_t num_lights;
  DevLight lights[kMaxLights];
  EnvView env;
  int32_t debug_mode;
};

struct FrameView {
  int32_t W, H, ntx, G, R;
  FastDiv div_P, div_ntx;
  uint32_t P;   // local pixels (local tiles * 1024)
  uint32_t k;   // samples in this wave
  uint32_t acc0;  // accumulation index of sample slot 0
  uint32_t max_depth;
  uint32_t valid;  // pixels of this shard inside the image
  vec3 cam_pos, cam_f, cam_r, cam_u;
  float half_w, half_h;
  uint32_t ablate;  // SPTR_ABLATE environment variable: timing experiments only (0 in normal use)
  float4* accum;    // per local pixel: running sample sum (xyz) + resume slot (w bits), see k_accum
  uint32_t reset;   // this batch starts the accumulation (frame_begin == 1, first batch)
  const uint32_t* dyn;  // device {frame_begin, reset, total} of the call (k_frame_dyn); see frame_dyn
  uint32_t pixel_major;  // kFold*: bounce 0 folds each pixel's leading misses into accum (bounce0_pixel_major)
  uint32_t integrator;   // sptr_integrator
  uint32_t spf;          // PathTracer mode: samples per frame
  vec3 ox_u, ox_v, ox_w; // OptiX mode: LaunchParams cam_u / cam_v / cam_w (OptixBackend.cpp:1609-1620)
  vec3 ox_light_dir, ox_light_rad;  // OptiX mode: first directional light (direction FROM the light)
  uint32_t ox_has_light;
  const uint32_t* cull;  // bit l: camera rays through local pixel l cannot hit the scene (k_cull); may be null
  uint32_t sky_fold;     // path-major bounce 0 with a cull mask: k_sky sums culled pixels into accum
  uint32_t cull_depth;   // BVH2 levels k_cull tests (<= kCullDepthMax)
  const uint32_t* plist; // with sky_fold: the unculled local pixels (count at plist[P]), bounce 0's paths
  const uint32_t* unculled;  // with cull: the number of unculled valid local pixels (k_cull's plist[P])
};
// FrameView::dyn words: {frame_begin, reset, total} of the call (k_frame_dyn).
constexpr size_t kDynBytes = 2048;

// Bounce-0 modes (FrameView::pixel_major): path-major (thread per path slot, every miss writes
// rad[p]); thread per pixel (k_trace_pm); wave per pixel (k_trace_wp).  The last two fold each
// pixel's leading misses into accum and record the resume slot for k_accum.
enum : uint32_t { kFoldNone = 0, kFoldThread = 1, kFoldWave = 2 };

// work-queue counters (WaveView::work), 8 XCDs 128 B apart per slot: k_shadow_dyn's two bounce slots
// (words 0 and 256), k_trace_dyn's (kWorkTraceQueue); then the straggler counts of bounces
// 0..kStragBounces-1 (kWorkStrag, 128 B apart; zeroed by k_accum)
constexpr uint32_t kWorkTraceQueue = 512;
constexpr uint32_t kWorkStrag = 768;
constexpr uint32_t kStragBounces = 4;  // bounces whose trace may hand long rays off (k_trace_dyn -> k_strag)
constexpr uint32_t kWorkWords = kWorkStrag + 32u * kStragBounces;
// Straggler hand-off (k_trace_dyn, k_strag): records per bounce, each {o, rng} {d, path} {thr, depth}
// {walk: node, depth | hit << 16, ref, tfar} and the walk's stack entries (kStragRec float4s), and the
// default lane threshold (a drained wave hands its rays off once this few lanes are still busy)
constexpr uint32_t kStragCap = 1u << 17;
constexpr uint32_t kStragRec = 4u + (uint32_t)kStack / 4u;
static_assert(kStragRec * 4u - 16u >= (uint32_t)kStack, "a straggler record holds the whole traversal stack");
constexpr uint32_t kStragLanesDefault = 12;  // C5, grid 256, bounce 0: r04n 0/8/16/32 lanes 8.03/7.76/7.95/8.48 ms; r04zb 4/8/12 lanes 7.96/7.83/7.73
// bounces whose traces hand off (<= kStragBounces): a handed-off path must be finished before the
// batch's k_accum, so the later a bounce, the less time its stragglers have beside the chain (r04n,
// C5 at 8 lanes: bounce 0 / 0-1 / 0-2: 7.76 / 7.82 / 7.94 ms)
#ifndef SPTR_STRAG_MAXD
#define SPTR_STRAG_MAXD 1
#endif
constexpr uint32_t kStragHandoffBounces = SPTR_STRAG_MAXD;
constexpr uint32_t kMaxSegs = 2048;  // max producer grid (256 CUs x 8 blocks)

// 64-bit totals block
enum : int {
  kTotClosest = 0,  // closest-hit queries (k_trace + k_tail)
  kTotShadow,       // any-hit queries
  kTotNodes, kTotTris, kTotSph,  // k_trace visit counts (SPTR_FRAME_COUNT_VISITS)
  kTotShNodes, kTotShPrims,      // k_shadow visit counts
  kTotOverflow,
  kTotTail,         // closest-hit queries traced by k_tail
  kTotStackOverflow,  // a traversal push was dropped (cannot happen within the build's stack bound)
  kTotTracedP,      // bounce-0 camera rays the trace kernels traversed (unculled pixel samples)
  kTotTracedB,      // queued rays of bounces >= 1 traversed by k_trace / k_trace_dyn
  kTotNodesP, kTotTrisP, kTotSphP,  // bounce-0 part of kTotNodes / kTotTris / kTotSph
  kTotTracedD,                       // [kStatDepths] rays the trace kernels traversed, by bounce
  kTotNodesD = kTotTracedD + 8,      // [kStatDepths] their node visits (SPTR_FRAME_COUNT_VISITS)
  kTotHistT = kTotNodesD + 8,        // [kHistBins] closest-hit rays by node visits, log2 bins (COUNT_VISITS)
  kTotHistS = kTotHistT + 16,        // [kHistBins] any-hit queries of the shadow stage, likewise
  kTotHitP = kTotHistS + 16,         // closest hits found by the bounce-0 trace kernels (COUNT_VISITS)
  kTotHitB,                          // closest hits found by the later trace kernels (COUNT_VISITS)
  kTotStrag,                         // paths k_trace_dyn handed off to k_strag
  kTotStragNodes, kTotStragTris, kTotStragSph,  // the handed-off walks' visits made by k_strag (every call)
  kTotTracedF,                       // queued rays of bounces >= 1 traced by the fused k_bounce (every call)
  kTotWords
};

constexpr int kStatDepths = 8;  // per-bounce statistics: bounces 0..6, and 7 = every later one
constexpr int kHistBins = 16;   // per-ray visit histograms: bin b holds 2^(b-1) <= visits < 2^b (bin 0: none)
static_assert(kTotWords == kTotTracedD + 8 + 8 + 16 + 16 + 7, "totals layout");

// Segment table of one block-segmented queue: producer block b wrote cnt[b] records at slots
// [b*per*mult, ...) where per (written by producer block 0) is the producer's input slice size.
struct SegTable {
  uint32_t* cnt;  // [kMaxSegs]
  uint32_t* per;  // [1]
};

// Hit records: per hit of a trace stage, the ray's input slot (bounce 0: its path id), its t bits and
// the primitive ref, 12 B in two dense arrays — {t, ref} (8 B, one dwordx2 per lane) and the slot (4 B,
// one dword) — so every access is a naturally aligned coalesced stream.  (r03: this split form replaced
// a 16-B uint4 record; a packed 12-B uint3 record, one dwordx3 per lane, measured 2 % slower on C2.)
constexpr size_t kHitBytes = 12;
struct HitStream {
  uint2* tr;     // {t bits, prim ref}
  uint32_t* id;  // input slot or path id
  __device__ __forceinline__ void put(uint32_t j, uint32_t i, uint32_t tb, uint32_t ref) const {
    tr[j] = make_uint2(tb, ref);
    id[j] = i;
  }
  __device__ __forceinline__ void get(uint32_t j, uint32_t& i, uint32_t& tb, uint32_t& ref) const {
    const uint2 v = tr[j];
    i = id[j];
    tb = v.x;
    ref = v.y;
  }
};

struct RayStream {
  float4* o;    // origin.xyz, rng state bits
  float4* d;    // direction.xyz, path id bits
  float4* thr;  // throughput.xyz
};

struct WaveView {
  RayStream rs[2];  // ping-pong by depth parity: bounce d traces rs[d&1], shade d writes rs[(d+1)&1]
  HitStream hrec;   // per hit: slot or path id, t bits, prim ref
  float4* rad;      // per path id
  float4* stask;    // per shade slot: L tasks of tstride float4
  SegTable segN, segH, segS;  // next rays, hits, shadow tasks
  unsigned long long* tot;
  unsigned long long* bstat;          // [kMaxSegs] per-block any-hit tallies (k_shadow, k_tail), folded by k_accum
  unsigned long long* bstat_closest;  // [kMaxSegs] per-block closest-hit tallies of k_tail
  uint32_t* work;    // [kWorkWords] work-queue counters of k_shadow_dyn, one per bounce (zeroed by k_shade)
  uint32_t seg_cap;  // records allocated per segmented stream (bounds guard)
  uint32_t hrec_cap;  // hit records allocated (bounce 0 segments span k samples per pixel slot)
  uint32_t L;        // lights (tasks per shaded path)
  uint32_t tstride;  // float4 slots per shadow task: 2, or 3 when a point light is present
  // bounce traces (k_trace_dyn, d >= 1) defer a miss's radiance update to the next k_shade: the ray
  // slot's throughput becomes thr * env and a record with prim kNoHit is queued, so that no kernel of
  // the bounce but k_shade writes rad[] and k_shadow_dyn(d - 1) may run beside it (enqueue_wavefront)
  uint32_t defer_miss;
  // straggler hand-off (k_trace_dyn of scenes beyond an XCD's L2): once a wave's share of rays is used
  // up and at most strag_lanes of its lanes are still tracing, those rays are written to strag (bounce
  // d's region, strag_cap records of 3 float4) and the paths are finished by k_strag beside the chain;
  // strag_lanes = 0: no hand-off
  float4* strag;
  uint32_t strag_cap, strag_lanes;
  // shadow carry (r05; scenes whose shadow rays have launches of their own, one light, a path-per-thread
  // tail): k_shade(carry_depth) hands the shadow task of every path that continues to the tail's
  // kernel (the continuation's thr.w = task slot + 1, the task's tag 0 so k_shadow_dyn skips it); k_tail
  // traces that shadow ray before the path's next bounce, so shadow(carry_depth) no longer has to end
  // before the tail starts.  kNoHit: no carry.
  uint32_t carry_depth;
  // launch timing (ktime_begin / ktime_end): this launch's slot of Context::tslots, or null (untimed)
  unsigned long long* tslot = nullptr;
};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};
// One lane's path-state streams: ray streams, hit records, radiance, shadow tasks, and
// the segment tables / per-block tallies / work counters (seg).
struct WaveBufs {
  uint64_t cap = 0;  // paths
  uint32_t L = 0, ts = 0;
  DevBuf rs[2][3], hrec, rad, stask, seg, strag;
};

struct StageMark {
  int stage;
  size_t b, e;                 // begin / end event indices in Context::events (stages timed by events)
  uint32_t slot = UINT32_MAX;  // the launch's Context::tslots slot (one-chain launches timed by the kernel)
};
constexpr uint32_t kTimeSlots = 4096;  // slot-timed launches per collection window (the rest run untimed)
// a slot: the start word, then kTimeEndLines end words, each on a 64-B line of its own (ktime_end)
constexpr uint32_t kTimeLineWords = 8, kTimeEndLines = 16, kTimeSlotWords = kTimeLineWords * (1 + kTimeEndLines);

// Events the next trace, fused-bounce or shadow launch of this thread records its own start and end
// into (hipExtLaunchKernelGGL: the timestamps of the dispatch itself, so no marker packet sits between
// two launches — a hipEventRecord there idled the GPU for 5-10 us).  Set by the stage timer right
// before the launch, taken (and cleared) by SPTR_TIMED_LAUNCH.
struct LaunchTiming {
  hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local LaunchTiming g_launch_timing;
// Or the timing slot (Context::tslots) of the next such launch: set by the stage timer, taken by the
// launcher (with_tslot) and filled by the kernel itself (ktime_begin / ktime_end: the device's wall
// clock, and not even a dispatch event).  One launch chain is timed this way; the pixel lanes' calls by
// dispatch events (Context::time_by_events), see kernels_wavefront.hip "launch timing".
extern thread_local unsigned long long* g_tslot;
WaveView with_tslot(const WaveView& w);

// Launch-graph cache of one render-call shape (sptr_api.cpp run_graph).  The key is every input of
// the call's launch sequence except the per-call device words (FrameView::dyn): the state epoch (bumped
// by every scene/state upload and buffer reallocation), the frame with frame_begin zeroed and the
// timing flags kept, and the batch plan.
struct GraphKey {
  uint64_t epoch;
  sptr_frame frame;
  uint32_t k, tail;
};
struct GraphCache {
  bool valid = false;
  GraphKey key{};
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipGraphNode_t dyn_node = nullptr;  // k_frame_dyn: its arguments are the per-call values
  hipKernelNodeParams dyn_params{};
  uint32_t waves = 0;
  // shape of the captured graph (check_graph): nodes, dependency edges, nodes on the longest path
  uint32_t nodes = 0, edges = 0, depth = 0;
};

struct Context {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t cap_stream = nullptr;  // launch-graph capture (a pixel lane's: created on its first capture)
  // side streams for launches that overlap the main sequence: the shadow launches (side) and k_sky /
  // k_strag (side2; k_sky beside the tail of scenes beyond an XCD's L2 runs on side after the last
  // shadow join), for direct launches and inside a capture (cap_*).  Star-shaped fork/join only: a side
  // stream waits on events of the call's main stream and the main stream on the side streams', never
  // one side stream on another (enqueue_wavefront, DESIGN.md §3 "Launch graphs").
  hipStream_t side_stream = nullptr, cap_side = nullptr, side2_stream = nullptr, cap_side2 = nullptr;
  // fork to a side stream, shadow join, k_sky join.  The direct launches and the captures each have
  // their own set (dev[0] direct, dev[1] captured), so an event recorded inside a capture is never
  // waited on by a direct launch.
  struct DepEvents {
    hipEvent_t fork = nullptr, join = nullptr, sky = nullptr;
  } dev[2];
  int prio_lo = 0, prio_hi = 0;  // stream priority range (hipDeviceGetStreamPriorityRange)
  hipEvent_t quiet_ev[2] = {nullptr, nullptr};  // dispatch events of untimed two-lane launches (StageTimer::quiet)
  // 0: replay a captured graph for repeated call shapes that fork no side-stream launch (run_call);
  // 1: direct launches; 2: direct, one stream; 3: graph for every repeated shape
  uint32_t launch_mode = 0;
  uint8_t* image_out = nullptr;  // a pixel lane's resolve target: its parent context's image (sptr_render)
  // a pixel lane's parent: the lane reads the parent's shading state (materials, geomID -> material
  // table, lights, environment, debug mode) instead of holding copies (shading(), sptr_api.cpp)
  const Context* parent = nullptr;
  bool last_forked = false;          // the last direct launch sequence forked launches to a side stream
  uint32_t strag_lanes = kStragLanesDefault;  // sptr_set_stragglers (0: no hand-off)
  uint64_t epoch = 1;                // bumped by every state change a captured graph depends on
  DevBuf dyn;                        // per-call {frame_begin, reset, total} (k_frame_dyn)
  DevBuf tslots;                     // [kTimeSlots][kTimeSlotWords] launch timing slots, zeroed
  uint32_t tslots_used = 0;          // slots handed out in this collection window
  double wall_khz = 0.0;             // the device wall clock's rate (wall_clock64 ticks per ms)
  bool time_by_events = false;       // one-launch stages timed by dispatch events, not slots (pixel lanes)
  GraphCache graph;
  int32_t capture_status = 0;        // hipError_t of the last capture that fell back to direct launches (0: none)
  std::string capture_error;         // ... and the call that returned it
  uint32_t captures = 0;             // graphs captured and instantiated
  GraphKey last_key{};               // the previous call's shape: a graph is captured when it repeats
  bool have_last_key = false;
  GraphKey bad_key{};                // a shape whose capture failed or was rejected: launched directly from then on
  bool have_bad_key = false;
  std::string err;
  int debug_mode = 0;
  uint64_t wave_paths = 0;  // 0 = default
  uint32_t tail_depth = 0;  // first bounce traced path-per-thread by k_tail (0 = automatic)
  // scene
  DevBuf nodes, prim_ref, tris, sph, tri_geom, sph_geom, tri_orig, sph_orig, geom_mat;
  DevBuf tri_mat;  // ShadeView::tri_mat (resolve_geom_materials)
  uint32_t leaf_size = 0;  // max primitives per BVH leaf range (1..16); 0 = automatic
  uint32_t bvh_width = 0;  // traversal width: 2 (LBVH as built), 4 (collapsed), 0 = automatic
  uint32_t leaf_used = 0;  // leaf size the current BVH was built with
  uint32_t treelet_passes = SPTR_TREELET_PASSES;  // SAH treelet passes over L2/HBM scenes' LBVH (kernels_lbvh.hip)
  uint32_t num_nodes = 0, num_tris = 0, num_sph = 0, root = 0, bvh_depth = 0;
  uint32_t num_tri_refs = 0;     // triangle references = triangle slots (split references, kernels_lbvh.hip)
  uint32_t split_pieces = 1;     // most references per split triangle (sptr_set_split_refs; 1 = no splits, the default)
  uint32_t num_nodes4 = 0, root4 = 0;
  uint32_t excluded_prims = 0;  // exactly degenerate triangles left out of the BVH (never hit; k_morton)
  uint32_t num_top4 = 0;  // wide nodes numbered first: the top kTopLevels levels
  uint32_t stack_need2 = 0, stack_need4 = 0;  // traversal stack entries the BVH2 / BVH4 can need
  DevBuf nodes4;
  uint32_t num_tri_geoms = 0;
  std::vector<uint32_t> geom_first;     // host copy for primID derivation
  std::vector<uint32_t> geom_material;  // host copy
  bool have_scene = false;
  double build_ms = 0.0;
  // shading state
  std::vector<DevMaterial> mats_host;
  DevBuf mats;
  std::vector<DevLight> lights_host;
  DevBuf env;
  int32_t env_size = 0;
  float env_intensity = 0.8f, env_clamp = 5.0f;
  WaveBufs wb;  // wavefront path state
  DevBuf w_tot;
  // pixel buffers
  int32_t W = 0, H = 0, G = 1, R = 0;
  uint32_t P = 0, local_tiles = 0;
  DevBuf accum, tiles, image;
  DevBuf cull;   // bounce-0 pixel-frustum cull mask, 1 bit per local pixel (k_cull)
  DevBuf plist;  // the local pixels k_cull did not cull, each tile's run in pixel order; their count at [P]
  // what the mask was computed for (state epoch, camera): k_cull reruns only when these change
  uint64_t cull_epoch = 0;
  sptr_camera cull_cam{};
  uint32_t cull_depth = 0;  // depth the cached mask was computed with
  uint32_t last_samples = 0;  // accumulation count after the last render
  // query scratch
  DevBuf qbuf;
  // Render calls whose counters and events are not yet collected (SPTR_FRAME_ASYNC): the device
  // totals accumulate across them and the stage events stay in the pool until sptr_collect_stats.
  std::vector<hipEvent_t> events;               // event pool
  std::vector<StageMark> marks;                 // recorded stage spans (event pool indices)
  size_t events_used = 0;
  uint32_t pending = 0;                         // render calls since the last collection
  hipStream_t pending_stream = nullptr;
  uint64_t pending_samples = 0, pending_waves = 0, pending_culls = 0;
};

// kernels_lbvh.hip
int build_lbvh(Context& c, const float* h_pos, uint32_t nverts, const uint32_t* h_idx, uint32_t ntris,
               const float* h_sph, uint32_t nsph, const uint32_t* h_tri_geom, uint32_t sph_geom_base);

// kernels_sort.hip: the build's device primitives (temp == nullptr: set temp_bytes only)
hipError_t scan_u32(void* temp, size_t& temp_bytes, const uint32_t* in, uint32_t* out, uint32_t n, hipStream_t s);
hipError_t radix_sort_pairs_u64(void* temp, size_t& temp_bytes, const uint64_t* keys_in, uint64_t* keys_out,
                                const uint32_t* vals_in, uint32_t* vals_out, uint32_t n, hipStream_t s);

// kernels_wavefront.hip
SceneView scene_view(const Context& c);
// Stage launchers return their (resident) grid size: the segment count their consumer scans.
unsigned launch_trace(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, int depth, bool count,
                  uint32_t nseg_in, hipStream_t s);
// k_shade traces the shadow ray in place (LDS-staged one-light scenes outside the visit-count pass)
bool shade_fuses_shadows(const SceneView& sv, const ShadeView& sh, bool count);
bool shadow_overlaps(const SceneView& sv, const WaveView& w);
unsigned launch_shade(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, int depth,
                      uint32_t nseg, bool fuse, hipStream_t s);
// bounce 0's shading and bounce 1 in one launch (k_bounce01): bounce 0's hit records of w.segH in, the rays
// of bounce 2 out in w.segN / rs[0]
unsigned launch_bounce01(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, uint32_t nseg,
                         hipStream_t s);
// one fused bounce (k_bounce): rays of w.segN in, continuation rays of w.segH out
unsigned launch_bounce(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, int depth,
                       uint32_t nseg, hipStream_t s);
unsigned launch_tail(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, int depth0,
                     uint32_t nseg_in, hipStream_t s);
unsigned launch_shadow(const SceneView& sv, const ShadeView& sh, const WaveView& w, int depth, bool count, uint32_t nseg_in,
                   hipStream_t s);
// the paths bounce d's trace handed off (k_strag), each carried to its end path-per-thread
void launch_strag(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, int depth,
                  hipStream_t s);
// whether bounce traces of this scene hand their stragglers off (wide BVH beyond an XCD's L2)
// k_trace_dyn of scenes beyond an XCD's L2 takes its rays from per-XCD work queues (r04l: with
// k_strag's blocks resident beside it a static share leaves late-starting blocks a tail; C5 8.68 ->
// 8.49 ms at 8 lanes, grid 128); its hit-record segments then hold twice the static shares.
bool trace_queue_applies(const SceneView& sv);
uint32_t hrec_mult(const SceneView& sv);
bool strag_applies(const SceneView& sv);
uint32_t bounce0_pixel_major(const SceneView& sv, const FrameView& f);
// resolve: also tone-map the sums into tiles (+ image) in the same launch (the call's last batch)
void launch_accumulate(const FrameView& f, const WaveView& w, float4* accum, uint32_t* tiles, uint8_t* image,
                       bool resolve, hipStream_t s);
// BVH2 levels the bounce-0 pixel cull tests for a call of spp samples per pixel
uint32_t cull_depth_for(uint32_t spp);
void launch_cull(const SceneView& sv, const FrameView& f, uint32_t* mask, uint32_t* plist, hipStream_t s);
// capped: at most 4 waves per SIMD (beside the launch chain); else full occupancy
void launch_sky(const ShadeView& sh, const FrameView& f, bool capped, hipStream_t s);
// dst local tile i <- a's tile i / 2 (i even) or b's tile i / 2 (i odd): two pixel lanes' tiles in the
// tile order of the shard they split
void launch_interleave_tiles(const uint32_t* a, uint32_t na, const uint32_t* b, uint32_t nb, uint32_t* dst,
                             uint32_t n, hipStream_t s);
void launch_resolve(const FrameView& f, const float4* accum, uint32_t n, uint32_t* tiles, uint8_t* image,
                    hipStream_t s);
// Head of every render call: the per-call values kernels read through FrameView::dyn.
void launch_frame_dyn(uint32_t* dyn, uint32_t frame_begin, uint32_t reset, uint32_t total, uint32_t* clear,
                      unsigned long long* t0, hipStream_t s);
const void* frame_dyn_kernel();
// PathTracer-mode frames (the k frames of f from f.acc0), one launch: accum += tonemapped frames.
void launch_pathtracer(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, hipStream_t s);
// OptiX-compatible frames (the k frames of f from f.acc0), one launch: accum.xyz += contributions,
// accum.w += samples.
void launch_optix(const SceneView& sv, const ShadeView& sh, const FrameView& f, const WaveView& w, hipStream_t s);
void launch_unpack(const uint32_t* gathered, int G, uint32_t tiles_per_rank, int W, int H, uint8_t* rgb,
                   hipStream_t s);
// tri_mat[i] = geom_mat[tri_geom[i]], i < n
void launch_tri_materials(const uint32_t* tri_geom, const uint32_t* geom_mat, uint32_t n, uint32_t* tri_mat, hipStream_t s);
void launch_query(const SceneView& sv, const uint32_t* tri_orig, const uint32_t* sph_orig, const float* rays, uint32_t n,
                  bool anyhit, uint32_t* ref, float* t, float* ng, uint8_t* occ, uint32_t* stack_overflow, hipStream_t s);
void launch_primary(const FrameView& f, float* dirs, uint32_t* rng, hipStream_t s);
void launch_eval_math(int fn, const float* x, uint32_t n, float* out, hipStream_t s);
// one wave spinning for `ticks` of the device wall clock (sptr_overlap_probe)
void launch_spin(uint64_t ticks, hipStream_t s);

}  // namespace sptr
