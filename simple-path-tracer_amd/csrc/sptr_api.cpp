// sptr_api.cpp — C ABI of libsptr_hip (include/sptr_hip.h): context, uploads, and the per-call
// wavefront schedule.  This is the replacement for OptixBackend::render's orchestration
// (src/backends/OptixBackend.cpp:1506-1850): where the reference does three blocking host round
// trips per bounce (queue counter readbacks + a LaunchParams upload), here every stage reads its
// queue length from device memory, so a whole render call is enqueued without a host sync.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "sptr_internal.h"

#include <dlfcn.h>
#include <execinfo.h>
#include <csignal>
#include <ucontext.h>
#include <unistd.h>

struct sptr_ctx {
  sptr::Context c;
  // Pixel lanes (sptr_set_pixel_lanes): a second context, with its own buffers and streams, renders the
  // odd half of this context's tiles beside this one's launch chain, so that each chain's launch tails
  // run beside the other's work.  Only for scenes staged into LDS (the lane holds a copy of the scene).
  sptr_ctx* lane = nullptr;
  bool is_lane = false;
  uint32_t lanes_req = 0;   // 0: automatic, 1: one chain, 2: two lanes
  bool lane_scene = false;  // the lane context holds this context's scene
  bool split = false;       // the current accumulation runs in two lanes
  hipEvent_t lane_fork = nullptr, lane_join = nullptr;
  sptr::DevBuf tiles_full;  // with split: this context's tiles, interleaved from the two lanes'
  uint32_t full_tiles = 0;
  int full_G = 1, full_R = 0;
  // sptr_read_rgb8_lagged: two device snapshots of the RGB8 image, alternately written; a copy stream and
  // the registered host destination (created / registered on first use)
  struct Snap {
    sptr::DevBuf buf;
    hipEvent_t ready = nullptr;
    int W = 0, H = 0;
    bool valid = false;
  } snap[2];
  uint32_t snap_cur = 0;
  hipStream_t copy_stream = nullptr;
  hipEvent_t copy_done = nullptr;
  void* reg_ptr = nullptr;
  size_t reg_bytes = 0;
};

namespace sptr {
namespace {

int fail(Context& c, int code, const std::string& msg) {
  c.err = msg;
  return code;
}
int sync_pending(Context& c);

#define API_HIP(x)                                                                          \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) return fail(c, SPTR_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

hipError_t ensure_buf(DevBuf& b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.p && b.bytes >= bytes) return hipSuccess;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  hipError_t e = hipMalloc(&b.p, bytes);
  if (e == hipSuccess) b.bytes = bytes;
  return e;
}
void free_buf(DevBuf& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

// The context whose shading state (materials and their device table, the geomID -> material table,
// lights, environment, debug mode) a render of c uses: a pixel lane reads its parent's (ADVICE r05:
// a copy per lane put the HDR cubemap into HBM twice, also for scenes the lane never renders).
inline const Context& shading(const Context& c) { return c.parent ? *c.parent : c; }

// One wavefront batch holds up to 2^29 paths (160 B of path state each with one light: 86 GB, under
// a third of the 288 GB of HBM).  Every batch pays the secondary bounces' latency floor once: their
// queues are short (C3: ~1% of the primary rays survive) and each launch lasts as long as its
// longest traversal (~0.2-0.3 ms in the rattan chair), so fewer, larger batches win.  Measured on
// MI355X (C3, 1080p x 256 spp; profiles/r01d_wave_sweep.txt): 2^24 paths/batch 9.8 Grays/s, 2^25
// 15.2, 2^26 22.1, 2^27 29.4, 2^28 37.1, 2^29 42.8.  The default is further capped by free memory.
constexpr uint64_t kDefaultWavePaths = 1ull << 29;
constexpr double kWaveMemFraction = 0.5;  // at most this share of the free HBM for the default batch
// Bounces 0 .. T-1 run as wavefront stages (trace, shade, shadow launches over dense queues); from
// bounce T on, k_tail carries each surviving path to its end in one launch.
// Automatic policy (tail_depth 0), measured on MI355X (C2, profiles/r01d_shards_c2.txt): with a
// full 2^27-path batch the deep-bounce launches are large enough to pay for themselves and the
// wavefront wins (no tail: 4.20 ms vs 4.34 ms with a tail from bounce 4); in the small per-rank
// batches of a sharded frame the fixed cost of the 3 launches per deep bounce dominates, and the
// tail from bounce 4 wins (8-way shard: 0.723 ms vs 0.794; 4-way: 1.208 vs 1.238).
// Scenes traversed from L2/HBM (wide BVH): the late bounces hold few rays, but every wavefront launch
// lasts as long as its longest traversal (the 64-255-visit grazing rays of a 10M-triangle mesh: ~0.25
// ms per trace or shadow launch however few rays it holds), so the tail takes over early whatever
// the batch size.  Measured r03 (SPTR_TAIL_WAVES 4): C3 (L2-resident) tail from bounce 2 4.22 vs 5.07
// ms/step without a tail (from 3: 4.58); C5 (HBM) from bounce 3 10.67 vs 11.58 (from 2: 12.12).  LDS
// scenes keep the batch-size rule (C2 1 GPU: no tail 3.21, from 4 3.31, from 3 3.48 ms).
constexpr uint32_t kSmallBatchTailDepth = 4;
constexpr uint64_t kSmallBatchPaths = 1ull << 25;  // batches up to this many paths take the tail
uint32_t auto_tail_depth(uint64_t batch_paths, const SceneView& sv) {
  if (sv.lds_bytes == 0u) return sv.scene_bytes <= (4ull << 20) ? 2u : 3u;
  return batch_paths <= kSmallBatchPaths ? kSmallBatchTailDepth : (uint32_t)kMaxDepth;
}

// MaterialManager::getMaterialFromHit (src/MaterialManager.cpp:91-103): the geomID's mapped
// material when it is in range, else MaterialManager::getMaterialByID(geomID) (:79-89).
int resolve_geom_materials(Context& c) {
  const uint32_t nm = (uint32_t)c.mats_host.size();
  const uint32_t ng = c.num_tri_geoms + c.num_sph;
  if (!c.have_scene || nm == 0) return SPTR_OK;
  std::vector<uint32_t> t(ng ? ng : 1, 0u);
  for (uint32_t g = 0; g < ng; ++g) {
    uint32_t m = ~0u;
    if (g < c.geom_material.size() && c.geom_material[g] < nm) m = c.geom_material[g];
    else m = (g < nm) ? g : g % nm;
    t[g] = m;
  }
  API_HIP(ensure_buf(c.geom_mat, t.size() * 4));
  API_HIP(hipMemcpy(c.geom_mat.p, t.data(), t.size() * 4, hipMemcpyHostToDevice));
  // scenes traversed from L2/HBM: the material of every triangle slot, so that shading a hit loads it
  // directly instead of the slot's geomID and then its material
#ifndef SPTR_TRI_MAT
#define SPTR_TRI_MAT 1
#endif
  free_buf(c.tri_mat);
  if (SPTR_TRI_MAT && scene_view(c).lds_bytes == 0u && c.num_tri_refs) {
    API_HIP(ensure_buf(c.tri_mat, (size_t)c.num_tri_refs * 4));
    launch_tri_materials(static_cast<const uint32_t*>(c.tri_geom.p), static_cast<const uint32_t*>(c.geom_mat.p),
                         c.num_tri_refs, static_cast<uint32_t*>(c.tri_mat.p), c.stream);
    API_HIP(hipGetLastError());
    API_HIP(hipStreamSynchronize(c.stream));
  }
  return SPTR_OK;
}

inline bool host_local_pixel(const Context& c, uint32_t l, int& x, int& y) {
  return shard_pixel(c.W, c.H, c.G, c.R, l, x, y);
}

// segment tables (3 x (kMaxSegs + 4) u32), per-block tallies (2 x kMaxSegs u64), work counters
size_t seg_table_bytes() { return 3 * (kMaxSegs + 4) * 4 + 2 * kMaxSegs * 8 + kWorkWords * 4; }

// device bytes per path slot of a wave: ray streams 2 x (o, d, thr), hit record(s), radiance, and
// L shadow tasks of ts float4s.  hrec_mult: hit-record segments per static share (2 when the trace
// takes its rays from the per-XCD queues, trace_queue_applies; else 1).
uint64_t wave_path_bytes(uint32_t L, uint32_t ts, uint32_t hrec_mult) {
  return 2 * 3 * 16 + hrec_mult * kHitBytes + 16 + (uint64_t)L * ts * 16;
}
// fixed segment slack of a wave's streams (see ensure_wave); k_slack = hit-record slack multiplier
uint64_t wave_slack_bytes(uint32_t L, uint32_t ts, uint32_t k_slack, uint32_t hrec_mult) {
  const uint64_t recs = (uint64_t)kMaxSegs * kBlock;
  return recs * (2 * 3 * 16 + (uint64_t)(L ? L : 1u) * ts * 16) + hrec_mult * recs * k_slack * kHitBytes;
}

// k_slack: the pixel-major bounce-0 trace gives each block a hit-record segment of k records per
// pixel slot of its static share, so the hit records span cap + kMaxSegs * kBlock * k (k_slack = k);
// every other producer needs cap + kMaxSegs * kBlock (k_slack = 1).  hrec_mult: see wave_path_bytes.
int ensure_wave(Context& c, uint64_t cap, uint32_t L, uint32_t ts, uint32_t k_slack, uint32_t hrec_mult) {
  WaveBufs& b = c.wb;
  L = L ? L : 1u;
  const size_t hrec_bytes = ((size_t)cap + (size_t)kMaxSegs * kBlock * k_slack) * kHitBytes * hrec_mult;
  const bool grow = b.hrec.bytes < hrec_bytes || !(b.cap >= cap && b.L * b.ts >= L * ts && b.rad.p) || !b.seg.p;
  if (grow && sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;  // pending renders may still use the old streams
  if (grow) ++c.epoch;
  if (!b.seg.p) {  // segment tables, per-block tallies and work counters, zeroed once
    API_HIP(ensure_buf(b.seg, seg_table_bytes()));
    API_HIP(hipMemset(b.seg.p, 0, seg_table_bytes()));
  }
  // straggler records (k_trace_dyn -> k_strag, scenes beyond an XCD's L2): kStragCap per bounce
  if (strag_applies(scene_view(c))) API_HIP(ensure_buf(b.strag, (size_t)kStragHandoffBounces * kStragCap * kStragRec * 16u));
  API_HIP(ensure_buf(b.hrec, hrec_bytes));
  if (b.cap >= cap && b.L * b.ts >= L * ts && b.rad.p) return SPTR_OK;
  // Segmented streams: a stage with G blocks writes block b's outputs at [b*per, b*per + count)
  // with per = ceil(n / (G*kBlock)) * kBlock, so the segment space G*per can exceed n by up to
  // G*kBlock - 1 records: every segmented stream carries kMaxSegs*kBlock records of slack.
  const size_t n = (size_t)cap, ns = n + (size_t)kMaxSegs * kBlock;
  for (auto& r : b.rs)
    for (DevBuf& x : r) API_HIP(ensure_buf(x, ns * 16));
  API_HIP(ensure_buf(b.rad, n * 16));
  API_HIP(ensure_buf(b.stask, ns * L * ts * 16));
  b.cap = cap;
  b.L = L;
  b.ts = ts;
  return SPTR_OK;
}

uint32_t task_stride(const Context& c) {
  for (const DevLight& l : shading(c).lights_host)
    if (l.type != 0) return 3u;
  return 2u;
}

WaveView wave_view(Context& c) {
  const WaveBufs& wb = c.wb;
  WaveView w;
  for (int b = 0; b < 2; ++b) {
    w.rs[b].o = static_cast<float4*>(wb.rs[b][0].p);
    w.rs[b].d = static_cast<float4*>(wb.rs[b][1].p);
    w.rs[b].thr = static_cast<float4*>(wb.rs[b][2].p);
  }
  const uint64_t hcap = std::min<uint64_t>(wb.hrec.bytes / kHitBytes, 0xFFFFFFFFull);
  w.hrec.tr = static_cast<uint2*>(wb.hrec.p);
  w.hrec.id = reinterpret_cast<uint32_t*>(static_cast<char*>(wb.hrec.p) + hcap * 8u);
  w.rad = static_cast<float4*>(wb.rad.p);
  w.stask = static_cast<float4*>(wb.stask.p);
  uint32_t* seg = static_cast<uint32_t*>(wb.seg.p);  // 3 tables of kMaxSegs counts + 1 stride
  w.segN = SegTable{seg, seg + kMaxSegs};
  w.segH = SegTable{seg + (kMaxSegs + 4), seg + (kMaxSegs + 4) + kMaxSegs};
  w.segS = SegTable{seg + 2 * (kMaxSegs + 4), seg + 2 * (kMaxSegs + 4) + kMaxSegs};
  w.bstat = reinterpret_cast<unsigned long long*>(seg + 3 * (kMaxSegs + 4));
  w.bstat_closest = w.bstat + kMaxSegs;
  w.work = reinterpret_cast<uint32_t*>(w.bstat_closest + kMaxSegs);
  w.tot = static_cast<unsigned long long*>(c.w_tot.p);
  w.L = (uint32_t)shading(c).lights_host.size();
  w.tstride = task_stride(c);
  w.defer_miss = 0u;
  w.seg_cap = (uint32_t)(wb.cap + (uint64_t)kMaxSegs * kBlock);
  w.hrec_cap = (uint32_t)hcap;
  w.strag = static_cast<float4*>(wb.strag.p);
  w.strag_cap = wb.strag.p ? kStragCap : 0u;
  w.strag_lanes = 0u;  // set per trace launch (enqueue_wavefront)
  w.carry_depth = kNoHit;
  return w;
}

FrameView frame_view(const Context& c, const sptr_frame& f) {
  FrameView v;
  v.W = f.width;
  v.H = f.height;
  v.ntx = (f.width + kTile - 1) / kTile;
  v.G = c.G;
  v.R = c.R;
  v.P = c.P;
  v.k = 1;
  v.acc0 = f.frame_begin;
  v.max_depth = f.max_depth;
  v.div_P = make_fastdiv(c.P ? c.P : 1u);
  v.div_ntx = make_fastdiv((uint32_t)v.ntx);
  v.valid = 0;
  {
    const int ntx = (c.W + kTile - 1) / kTile;
    for (uint32_t lt = 0; lt < c.local_tiles; ++lt) {
      const uint32_t t = lt * (uint32_t)c.G + (uint32_t)c.R;
      const int x0 = (int)(t % (uint32_t)ntx) * kTile, y0 = (int)(t / (uint32_t)ntx) * kTile;
      v.valid += (uint32_t)(std::min(kTile, c.W - x0) * std::min(kTile, c.H - y0));
    }
  }
  const sptr_camera& k = f.camera;
  v.cam_pos = v3(k.pos[0], k.pos[1], k.pos[2]);
  v.cam_f = v3(k.forward[0], k.forward[1], k.forward[2]);
  v.cam_r = v3(k.right[0], k.right[1], k.right[2]);
  v.cam_u = v3(k.up[0], k.up[1], k.up[2]);
  v.half_w = k.half_width;
  v.half_h = k.half_height;
#ifdef SPTR_EXPERIMENT_KNOBS
  // SPTR_ABLATE (timing experiments only: wrong images by design); experiment builds only
  static const uint32_t ablate = getenv("SPTR_ABLATE") ? (uint32_t)atoi(getenv("SPTR_ABLATE")) : 0u;
  v.ablate = ablate;
#else
  v.ablate = 0u;
#endif
  v.accum = static_cast<float4*>(c.accum.p);
  v.reset = 0;
  v.pixel_major = 0;
  v.dyn = nullptr;
  v.cull = nullptr;
  v.cull_depth = 4u;
  v.sky_fold = 0u;
  v.plist = nullptr;
  v.unculled = nullptr;
  v.integrator = f.integrator;
  v.spf = f.samples_per_frame ? f.samples_per_frame : 4u;
  return v;
}

ShadeView shade_view(const Context& cc) {
  const Context& c = shading(cc);
  ShadeView s{};
  s.mats = static_cast<const DevMaterial*>(c.mats.p);
  s.num_mats = (uint32_t)c.mats_host.size();
  s.geom_mat = static_cast<const uint32_t*>(c.geom_mat.p);
  s.tri_mat = cc.parent ? nullptr : static_cast<const uint32_t*>(c.tri_mat.p);  // (slots are the owner's)
  s.num_lights = (uint32_t)c.lights_host.size();
  for (uint32_t i = 0; i < s.num_lights; ++i) s.lights[i] = c.lights_host[i];
  s.env.env = static_cast<const float4*>(c.env.p);
  s.env.env_size = c.env_size;
  s.env.env_intensity = c.env_intensity;
  s.env.env_clamp = c.env_clamp;
  s.env.debug_mode = c.debug_mode;
  s.debug_mode = c.debug_mode;
  return s;
}

// Stage events on the render stream, kept in the context's pool until collected.  Stages: 0 whole
// render call, 1 trace (bounce >= 1), 2 shade (>= 1), 3 shadow, 4 accum + resolve, 5 trace bounce 0
// (raygen fused), 6 shade bounce 0, 7 tail, 8 pixel cull, 9 fused bounce (k_bounce: the trace and the
// shading of a bounce in one launch, counted with the trace launches); 0-9 with SPTR_FRAME_TIMING,
// 1, 3, 5 and 9 with SPTR_FRAME_TIMING_TRACE.
constexpr int kStages = 10;
#ifndef SPTR_CALL_SPAN
#define SPTR_CALL_SPAN 1  // untimed direct calls' span: 0 = event records, 1 = dispatch events, 2 = none (A/B)
#endif
struct StageTimer {
  Context& c;
  bool on;                  // SPTR_FRAME_TIMING or SPTR_FRAME_TIMING_TRACE
  bool trace_only;          // SPTR_FRAME_TIMING_TRACE alone: the trace (1, 5) and shadow (3) launches only
  hipStream_t s;
  hipError_t err = hipSuccess;
  std::string what;         // the call that set err
  size_t open = SIZE_MAX;   // index in c.marks of the stage being recorded
  size_t call = SIZE_MAX;   // index in c.marks of this call's stage-0 span
  size_t alloc() {  // a pool event for this call (not recorded)
    if (c.events_used == c.events.size()) {
      hipEvent_t e = nullptr;
      const hipError_t r = hipEventCreate(&e);
      if (r != hipSuccess) {
        if (err == hipSuccess) {
          err = r;
          what = "stage event create";
        }
        return SIZE_MAX;
      }
      c.events.push_back(e);
    }
    return c.events_used++;
  }
  bool capturing = false;  // inside a graph capture: no stage events (run_call), the streams are the cap_* ones
  size_t next() {
    const size_t i = alloc();
    if (i != SIZE_MAX && err == hipSuccess) {
      err = hipEventRecord(c.events[i], s);
      if (err != hipSuccess) what = "stage event record";
    }
    return i;
  }
  // the stages that are exactly one launch: timed by the launch itself (g_launch_timing), the others
  // by events recorded on s around them (an event record between two launches idles the GPU for
  // ~5-10 us: r05 8-way C2 shard, 6 records per step -> 2 without the cull and call spans)
  static bool one_launch(int stage) { return stage == 1 || stage == 5 || stage == 9 || stage == 3; }
  bool launch_timed = false;
  bool quiet = false, quiet_open = false;  // untimed launch with dispatch events (run_call)
  void begin(int stage) {
    if (quiet && !on && !capturing && one_launch(stage)) {
      g_launch_timing = LaunchTiming{c.quiet_ev[0], c.quiet_ev[1]};
      quiet_open = true;
      return;
    }
    if (!on || capturing || (trace_only && !one_launch(stage))) return;
    // timed by the dispatch's events (g_launch_timing): the pixel lanes' launches, and the shadow launches,
    // which run on a side stream beside the bounce traces and may wait there after their dispatch for
    // the CUs: a slot's start (block 0 running) leaves that wait out, a dispatch event and rocprofv3's
    // kernel trace count it (C5 r05i: shadow frac 0.48 from slots vs 0.29 from the kernel trace)
    if (one_launch(stage) && (c.time_by_events || stage == 3)) {
      const size_t b = alloc(), e = alloc();
      if (b == SIZE_MAX || e == SIZE_MAX) return;
      open = c.marks.size();
      c.marks.push_back(StageMark{stage, b, e});
      g_launch_timing = LaunchTiming{c.events[b], c.events[e]};
      launch_timed = true;
      return;
    }
    if (one_launch(stage)) {  // timed by the kernel itself (g_tslot -> WaveView::tslot)
      if (!c.tslots.p || c.tslots_used >= kTimeSlots) return;
      open = c.marks.size();
      c.marks.push_back(StageMark{stage, SIZE_MAX, SIZE_MAX, c.tslots_used});
      g_tslot = static_cast<unsigned long long*>(c.tslots.p) + (size_t)kTimeSlotWords * c.tslots_used++;
      launch_timed = true;
      return;
    }
    open = c.marks.size();
    c.marks.push_back(StageMark{stage, next(), SIZE_MAX});
  }
  void end() {
    if (quiet_open) {
      quiet_open = false;
      g_launch_timing = LaunchTiming{};  // (taken by the launch; cleared if there was none)
      return;
    }
    if (open == SIZE_MAX) return;
    if (launch_timed) {
      launch_timed = false;
      if (g_tslot || g_launch_timing.start) {  // nothing was launched: nothing recorded, no mark
        if (g_tslot) --c.tslots_used;
        g_tslot = nullptr;
        g_launch_timing = LaunchTiming{};
        c.marks.erase(c.marks.begin() + (std::ptrdiff_t)open);
      }
      open = SIZE_MAX;
      return;
    }
    c.marks[open].e = next();
    open = SIZE_MAX;
  }
  // The call span of an untimed direct wavefront call: a timing slot whose start the call's first launch
  // (k_frame_dyn) stores and whose end its last (k_accum) takes, like a slot-timed launch's, instead of
  // two event records, each of which idled the GPU for ~5 us (r06, kernel trace of the 8-way C2 shard:
  // 475 us per step with them, 463 without; dispatch events on those two launches left the same gaps).
  uint32_t call_slot = UINT32_MAX;
  bool stop_set = false;
  unsigned long long* slot_ptr(uint32_t i) const {
    return static_cast<unsigned long long*>(c.tslots.p) + (size_t)kTimeSlotWords * i;
  }
  unsigned long long* pre_call(bool wavefront) {  // right before the call's first launch: its t0 word
    if (SPTR_CALL_SPAN != 1 || !wavefront || on || capturing || !c.tslots.p || c.tslots_used >= kTimeSlots)
      return nullptr;
    call_slot = c.tslots_used++;
    return slot_ptr(call_slot);
  }
  void begin_call() {  // (a replayed graph's call span is recorded around its launch: run_call)
    if (capturing || (on && trace_only)) return;  // SPTR_FRAME_TIMING_TRACE: the trace spans only
    if (SPTR_CALL_SPAN == 2 && !on) return;
    call = c.marks.size();
    if (call_slot != UINT32_MAX) c.marks.push_back(StageMark{0, SIZE_MAX, SIZE_MAX, call_slot});
    else c.marks.push_back(StageMark{0, next(), SIZE_MAX});
  }
  void last_launch() {  // right before the call's last launch on s (k_accum)
    if (call_slot == UINT32_MAX || call == SIZE_MAX) return;
    g_tslot = slot_ptr(call_slot);
    stop_set = true;
  }
  void end_call() {
    if (call == SIZE_MAX) return;
    if (call_slot != UINT32_MAX) {  // (a slot whose end was not taken reads as 0 ms)
      if (stop_set) g_tslot = nullptr;
      return;
    }
    c.marks[call].e = next();
  }
};

// The launch intervals [start, end] (device wall-clock ticks) of the context's slot-timed launches in
// this collection window, by slot; {0, 0} for a slot whose launch left no time.
std::vector<std::pair<uint64_t, uint64_t>> read_slots(Context& c) {
  std::vector<std::pair<uint64_t, uint64_t>> iv(c.tslots_used, {0, 0});
  if (c.tslots_used == 0) return iv;
  std::vector<unsigned long long> w((size_t)kTimeSlotWords * c.tslots_used);
  if (hipMemcpy(w.data(), c.tslots.p, w.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return iv;
  for (uint32_t i = 0; i < c.tslots_used; ++i) {
    const unsigned long long* sl = w.data() + (size_t)kTimeSlotWords * i;
    uint64_t t1 = 0;
    for (uint32_t j = 1; j <= kTimeEndLines; ++j) t1 = std::max<uint64_t>(t1, sl[kTimeLineWords * j]);
    const uint64_t t0 = sl[0];
    if (t0 != 0 && t1 >= t0) iv[i] = {t0, t1};
  }
  return iv;
}

// Length of the union of intervals.
template <typename T>
double union_length(std::vector<std::pair<T, T>>& iv) {
  if (iv.empty()) return 0.0;
  std::sort(iv.begin(), iv.end());
  double busy = 0.0;
  T lo = iv[0].first, hi = iv[0].second;
  for (size_t i = 1; i < iv.size(); ++i) {
    if (iv[i].first > hi) {
      busy += (double)(hi - lo);
      lo = iv[i].first;
      hi = iv[i].second;
    } else {
      hi = std::max(hi, iv[i].second);
    }
  }
  return busy + (double)(hi - lo);
}

// Busy time of the trace stage over the pending calls of contexts cs[0..n): the union of the trace
// launches' intervals (stages 1, 5 and 9).  Slot-timed launches are placed on the device's wall clock,
// event-timed ones (the pixel lanes' calls) by their events' offsets from the first such event; both
// clocks are shared by every stream and both lanes, whose trace launches overlap.  (A window holding
// calls of both kinds adds the two unions: such calls run one after the other on the render stream.)
// 0 when a stream fails (collect_pending reports that failure).
double trace_busy_ms(Context* const* cs, int n) {
  std::vector<std::pair<uint64_t, uint64_t>> iv;
  std::vector<std::pair<float, float>> ev;
  double khz = 0.0;
  hipEvent_t ref = nullptr;
  for (int k = 0; k < n; ++k) {
    Context& c = *cs[k];
    if (c.pending == 0) continue;
    if (hipStreamSynchronize(c.pending_stream) != hipSuccess) return 0.0;
    const auto sl = read_slots(c);
    khz = c.wall_khz;
    for (const StageMark& m : c.marks) {
      if (m.stage != 1 && m.stage != 5 && m.stage != 9) continue;
      if (m.slot != UINT32_MAX) {
        if (m.slot < sl.size() && sl[m.slot].second) iv.push_back(sl[m.slot]);
      } else if (m.b < c.events.size() && m.e < c.events.size()) {
        if (!ref) ref = c.events[m.b];
        float b = 0.0f, e = 0.0f;
        if (hipEventElapsedTime(&b, ref, c.events[m.b]) == hipSuccess &&
            hipEventElapsedTime(&e, ref, c.events[m.e]) == hipSuccess)
          ev.emplace_back(b, e);
      }
    }
  }
  return (khz > 0.0 ? union_length(iv) / khz : 0.0) + union_length(ev);
}

// Wait for the pending render calls, fold their device counters and stage events into *stats
// (may be null) and start a new collection window.
int collect_pending(Context& c, sptr_stats* stats) {
  if (stats) std::memset(stats, 0, sizeof(*stats));
  if (c.pending == 0) return SPTR_OK;
  // (the side streams' work is joined into pending_stream: complete once it is)
  const hipError_t se = hipStreamSynchronize(c.pending_stream);
  Context* self = &c;
  const double busy = se == hipSuccess && stats ? trace_busy_ms(&self, 1) : 0.0;
  double ms[kStages] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t trace_launches = 0, shadow_launches = 0;
  const auto slots = se == hipSuccess ? read_slots(c) : std::vector<std::pair<uint64_t, uint64_t>>();
  for (const StageMark& m : c.marks) {
    float t = 0.0f;
    if (m.slot != UINT32_MAX) {  // timed by the launch itself
      if (m.slot < slots.size()) t = (float)((double)(slots[m.slot].second - slots[m.slot].first) / c.wall_khz);
    } else if (se == hipSuccess && m.b < c.events.size() && m.e < c.events.size()) {
      (void)hipEventElapsedTime(&t, c.events[m.b], c.events[m.e]);
    }
    ms[m.stage] += t;
    if (m.stage == 1 || m.stage == 5 || m.stage == 9) ++trace_launches;
    if (m.stage == 3) ++shadow_launches;
  }
  c.marks.clear();
  c.events_used = 0;
  if (c.tslots_used) {  // the slots this window used, zeroed for the next one (the streams are idle)
    if (se == hipSuccess) (void)hipMemset(c.tslots.p, 0, (size_t)c.tslots_used * kTimeSlotWords * 8);
    c.tslots_used = 0;
  }
  const uint64_t samples = c.pending_samples, waves = c.pending_waves, culls = c.pending_culls;
  c.pending = 0;
  c.pending_samples = c.pending_waves = c.pending_culls = 0;
  if (se != hipSuccess) return fail(c, SPTR_ERR_HIP, std::string("render: ") + hipGetErrorString(se));
  unsigned long long tot[kTotWords];
  API_HIP(hipMemcpy(tot, c.w_tot.p, sizeof(tot), hipMemcpyDeviceToHost));
  if (tot[kTotOverflow]) return fail(c, SPTR_ERR_HIP, "render: segmented stream overflow (internal error)");
  if (tot[kTotStackOverflow]) return fail(c, SPTR_ERR_HIP, "render: BVH traversal stack overflow (internal error)");
  if (!stats) return SPTR_OK;
  stats->ms_total = ms[0];
  stats->ms_raygen = 0.0;  // raygen is fused into the bounce-0 trace (ms_trace0)
  stats->ms_trace = ms[1] + ms[5] + ms[9];
  stats->ms_shade = ms[2] + ms[6];
  stats->ms_trace0 = ms[5];
  stats->ms_shade0 = ms[6];
  stats->ms_shadow = ms[3];
  stats->ms_accum = ms[4];
  stats->trace_launches = trace_launches;
  stats->rays_closest = tot[kTotClosest];
  stats->rays_shadow = tot[kTotShadow];
  stats->rays_tail = tot[kTotTail];
  stats->ms_tail = ms[7];
  stats->samples = samples;
  stats->waves = waves;
  stats->node_visits = tot[kTotNodes];
  stats->tri_tests = tot[kTotTris];
  stats->sphere_tests = tot[kTotSph];
  stats->shadow_node_visits = tot[kTotShNodes];
  stats->shadow_prim_tests = tot[kTotShPrims];
  stats->traced_primary = tot[kTotTracedP];
  stats->traced_bounce = tot[kTotTracedB];
  stats->node_visits_primary = tot[kTotNodesP];
  stats->tri_tests_primary = tot[kTotTrisP];
  stats->sphere_tests_primary = tot[kTotSphP];
  stats->ms_cull = ms[8];
  stats->shadow_launches = shadow_launches;
  for (int d = 0; d < kStatDepths; ++d) {
    stats->traced_by_depth[d] = tot[kTotTracedD + d];
    stats->nodes_by_depth[d] = tot[kTotNodesD + d];
  }
  for (int b = 0; b < kHistBins; ++b) {
    stats->trace_visit_hist[b] = tot[kTotHistT + b];
    stats->shadow_visit_hist[b] = tot[kTotHistS + b];
  }
  stats->hits_primary = tot[kTotHitP];
  stats->hits_bounce = tot[kTotHitB];
  stats->paths_handed_off = tot[kTotStrag];
  for (int i = 0; i < 3; ++i) stats->strag_visits[i] = tot[kTotStragNodes + i];
  stats->cull_launches = culls;
  stats->ms_trace_busy = busy;
  stats->traced_fused = tot[kTotTracedF];
  return SPTR_OK;
}

// Device work of the pending render calls must be complete before a host read of their results.
int sync_pending(Context& c) {
  if (c.pending) API_HIP(hipStreamSynchronize(c.pending_stream));
  return SPTR_OK;
}

// Pixel buffers of a (W, H, shard) configuration.  A pending asynchronous render may still use the
// old buffers, so it is waited for before they are reallocated, and the clears are enqueued on the
// render stream (ordered before this call's kernels).
int ensure_pixels(Context& c, int W, int H, int G, int R, hipStream_t s, bool& resized) {
  resized = false;
  if (c.W == W && c.H == H && c.G == G && c.R == R && c.accum.p) return SPTR_OK;
  if (sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;
  const uint32_t local_tiles = shard_tiles(W, H, G, R);
  c.W = W;
  c.H = H;
  c.G = G;
  c.R = R;
  c.local_tiles = local_tiles;
  c.P = local_tiles * (uint32_t)kTilePixels;
  API_HIP(ensure_buf(c.accum, (size_t)c.P * 16));
  API_HIP(ensure_buf(c.tiles, (size_t)c.P * 4));
  API_HIP(ensure_buf(c.image, (size_t)W * H * 3));
  API_HIP(ensure_buf(c.cull, (size_t)c.P / 32u * 4u + 4u));
  API_HIP(ensure_buf(c.plist, ((size_t)c.P + 2u) * 4u));
  ++c.epoch;
  API_HIP(hipMemsetAsync(c.accum.p, 0, (size_t)c.P * 16, s));
  API_HIP(hipMemsetAsync(c.tiles.p, 0, (size_t)c.P * 4, s));
  API_HIP(hipMemsetAsync(c.image.p, 0, (size_t)W * H * 3, s));
  c.last_samples = 0;
  resized = true;
  return SPTR_OK;
}

// OptiX-compatible camera and light (OptixBackend::render, src/backends/OptixBackend.cpp:1515-1620):
// cam_u / cam_v scaled from Camera::getRayDirection at the image edges, the first directional light
// as direction FROM the light and colour * intensity.  Host float arithmetic in the reference's order.
void optix_frame_params(const Context& c, const sptr_frame& f, FrameView& v) {
  const sptr_camera& k = f.camera;
  const vec3 fwd = normalize(v3(k.forward[0], k.forward[1], k.forward[2]));
  const vec3 right = normalize(v3(k.right[0], k.right[1], k.right[2]));
  const vec3 up = normalize(v3(k.up[0], k.up[1], k.up[2]));
  const vec3 cf = v3(k.forward[0], k.forward[1], k.forward[2]), cr = v3(k.right[0], k.right[1], k.right[2]),
             cu = v3(k.up[0], k.up[1], k.up[2]);
  auto ray_dir = [&](float u, float vv) {  // Camera::getRayDirection (Camera.cpp:95-106)
    const float nx = (u - 0.5f) * 2.0f, ny = -(vv - 0.5f) * 2.0f;
    return normalize(cf + nx * k.half_width * cr + ny * k.half_height * cu);
  };
  const vec3 dx = ray_dir(1.0f, 0.5f), dy = ray_dir(0.5f, 0.0f);
  const float den_x = dot(dx, fwd), den_y = dot(dy, fwd);
  const float hw = den_x != 0.0f ? dot(dx, right) / den_x : 0.0f;
  const float hh = den_y != 0.0f ? dot(dy, up) / den_y : 0.0f;
  v.ox_u = right * hw;
  v.ox_v = up * hh;
  v.ox_w = fwd;
  v.ox_has_light = 0u;
  v.ox_light_dir = v3(0.0f, -1.0f, 0.0f);
  v.ox_light_rad = v3(0.0f, 0.0f, 0.0f);
  for (const DevLight& l : shading(c).lights_host)
    if (l.type == 0) {  // DevLight keeps the direction TO the light
      v.ox_light_dir = -v3(l.v[0], l.v[1], l.v[2]);
      v.ox_light_rad = v3(l.radiance[0], l.radiance[1], l.radiance[2]);
      v.ox_has_light = 1u;
      break;
    }
}

// Path-per-thread render calls (SPTR_INTEGRATOR_PATHTRACER / _OPTIX): no wavefront streams.
// Frames are launched kPtFramesPerLaunch at a time (bounded launch length); the accumulation order
// is the frame order either way.
constexpr uint32_t kPtFramesPerLaunch = 4;
// Launch sequence of a path-per-thread call on stream s (timer tm on s); returns the launch count.
uint32_t enqueue_path_per_thread(Context& c, const sptr_frame& f, hipStream_t s, StageTimer& tm) {
  const SceneView sv = scene_view(c);
  const ShadeView sh = shade_view(c);
  WaveView w = wave_view(c);
  FrameView fv = frame_view(c, f);
  fv.dyn = static_cast<const uint32_t*>(c.dyn.p);
  const bool optix = f.integrator == SPTR_INTEGRATOR_OPTIX;
  if (optix) optix_frame_params(c, f, fv);
  tm.begin_call();
  uint32_t done = 0, launches = 0;
  while (done < f.spp) {
    fv.k = std::min<uint32_t>(kPtFramesPerLaunch, f.spp - done);
    fv.acc0 = done;                  // offset from the call's frame_begin (frame_dyn)
    fv.reset = done == 0 ? 1u : 0u;  // and the call's reset flag applies to its first batch only
    tm.begin(7);
    if (optix) launch_optix(sv, sh, fv, w, s);
    else launch_pathtracer(sv, sh, fv, w, s);
    tm.end();
    done += fv.k;
    ++launches;
  }
  if (!(f.flags & SPTR_FRAME_NO_RESOLVE)) {
    tm.begin(4);
    launch_resolve(fv, static_cast<const float4*>(c.accum.p), 0u, static_cast<uint32_t*>(c.tiles.p),
                   c.image_out ? c.image_out : static_cast<uint8_t*>(c.image.p), s);
    tm.end();
  }
  tm.end_call();
  return launches;
}


// launches overlapped on the side streams (launch mode 2: everything on one stream)
bool overlap_enabled(const Context& c) {
#ifdef SPTR_EXPERIMENT_KNOBS
  static const bool env = [] {  // SPTR_OVERLAP=0: experiment builds only
    const char* e = getenv("SPTR_OVERLAP");
    return !(e && e[0] == '0');
  }();
  if (!env) return false;
#endif
  return c.launch_mode != 2 && c.side_stream && c.side2_stream;  // (a pixel lane has no side streams)
}

// Launch sequence of a wavefront call (batches of k samples, tail from bounce T) on stream s (the
// caller's stream, or the capture stream inside a graph capture).
//
// Side streams, star-shaped: a launch that overlaps the main sequence is forked from s (an event
// recorded on s, waited on by the side stream) and joined back into s (an event recorded on the side
// stream, waited on by s); a side stream never waits on an event of the other side stream.  Any
// other shape breaks the HIP runtime torch ships (ROCm 7.0): a capture in which one forked stream
// waits on an event recorded by another forked (non-origin) stream — a fork from a fork, or two side
// streams ordered against each other — ends in an endless recursion inside hipStreamEndCapture, which
// overflows the host stack (the r03 libamdhip64+0x2d34a8 crash of the two-lane calls;
// tools/micro/capture_events.hip reproduces it with three streams).  run_call checks every captured
// graph (check_graph) before instantiating it.
uint32_t enqueue_wavefront(Context& c, const sptr_frame& f, uint32_t k, int T, hipStream_t s, StageTimer& tm) {
  const SceneView sv = scene_view(c);
  const ShadeView sh = shade_view(c);
  WaveView w = wave_view(c);
  FrameView fv = frame_view(c, f);
  fv.dyn = static_cast<const uint32_t*>(c.dyn.p);
  const bool count = (f.flags & SPTR_FRAME_COUNT_VISITS) != 0;
  const bool fuse = shade_fuses_shadows(sv, sh, count);
#ifdef SPTR_EXPERIMENT_KNOBS
  static const bool no_bounce = getenv("SPTR_NO_BOUNCE") != nullptr;
  // SPTR_FUSE_FROM: first fused bounce of a large batch (A/B; 0 = none)
  static const int fuse_from_env = getenv("SPTR_FUSE_FROM") ? atoi(getenv("SPTR_FUSE_FROM")) : 0;
#else
  constexpr bool no_bounce = false;
  constexpr int fuse_from_env = 0;
#endif
  // bounce-0 pixel-frustum cull mask of this call's camera (every batch of the call shares it): made
  // current by refresh_cull ahead of this launch sequence, or, with SPTR_FRAME_RECULL, computed as the
  // sequence's first launch (inside a captured graph, whose key includes the camera and the flag)
  if (!(f.flags & SPTR_FRAME_NO_CULL)) {
    fv.cull_depth = cull_depth_for(f.spp);
    fv.cull = static_cast<const uint32_t*>(c.cull.p);
    fv.unculled = static_cast<const uint32_t*>(c.plist.p) + c.P;
  }
  tm.begin_call();
  if (fv.cull && (f.flags & SPTR_FRAME_RECULL)) {  // the count at plist[P] was zeroed by k_frame_dyn
    tm.begin(8);
    launch_cull(sv, fv, static_cast<uint32_t*>(c.cull.p), static_cast<uint32_t*>(c.plist.p), s);
    tm.end();
  }
  uint32_t done = 0, waves = 0;
  const int D = (int)f.max_depth;
  const bool overlap = overlap_enabled(c);
  const bool cap = tm.capturing;
  const hipStream_t ss = cap ? c.cap_side : c.side_stream;   // k_shadow_dyn(d)
  const hipStream_t ks = cap ? c.cap_side2 : c.side2_stream;  // k_sky (apart from the shadow launches it outlasts)
  const Context::DepEvents& ev = c.dev[cap ? 1 : 0];
  auto check = [&](hipError_t e, const char* what) {
    if (e != hipSuccess && tm.err == hipSuccess) {
      tm.err = e;
      tm.what = what;
    }
  };
  auto fork_to = [&](hipStream_t side) {  // side's next launches start after everything enqueued on s so far
    if (!cap) c.last_forked = true;
    check(hipEventRecord(ev.fork, s), "shadow fork record");
    check(hipStreamWaitEvent(side, ev.fork, 0), "shadow fork wait");
  };
  // pending side-stream work: shadow(d) (ev.join) and k_sky (ev.sky)
  bool join = false, join_sky = false;
  auto join_shadow = [&]() {
    if (join) check(hipStreamWaitEvent(s, ev.join, 0), "shadow join wait");
    join = false;
  };
  // any-hit launches of their own (k_shadow_dyn: scenes traversed from L2/HBM) run on the side stream
  // beside the next bounce's trace: shadow(d) only adds to rad[], which the bounce traces then leave
  // alone (misses deferred to k_shade, WaveView::defer_miss); k_shade(d + 1) overwrites the shadow
  // tasks and updates rad[], so it, the tail and k_accum wait for shadow(d) (ev.join)
  const bool shadow_side = overlap && !fuse && shadow_overlaps(sv, w);
  const bool strag = c.strag_lanes != 0u && !count && w.strag != nullptr && strag_applies(sv);
  w.defer_miss = shadow_side ? 1u : 0u;
  // shadow carry (WaveView::carry_depth): the last wavefront bounce before the tail hands its continuing
  // paths' shadow rays to k_tail, so that the tail need not wait for that bounce's shadow launch (which
  // then traces only the shadow rays of paths ending there, beside the tail, joined before k_accum).
  // Not in the visit-count pass (its k_shadow tallies every query).  Only for scenes resident in an
  // XCD's L2 (r05p/q: C3 3.70 -> 3.57 ms/step; C5, traversed from HBM, 7.38-7.44 -> 7.46-7.52: there the
  // tail, path per thread at 4 waves/SIMD, traces the carried rays slower than the refilling
  // k_shadow_dyn, 816 -> 1318 us, and the launch it shortens was 374 us).
  w.carry_depth = (shadow_side && !count && T < D && w.L == 1u && !trace_queue_applies(sv)) ? (uint32_t)(T - 1) : kNoHit;
  StageTimer tside{c, tm.on, tm.trace_only, ss};
  tside.capturing = tm.capturing;
  while (done < f.spp) {
    const uint32_t kk = std::min<uint32_t>(k, f.spp - done);
    fv.k = kk;
    fv.acc0 = done;                  // offset from the call's frame_begin (frame_dyn)
    fv.reset = done == 0 ? 1u : 0u;  // and the call's reset flag applies to its first batch only
    fv.pixel_major = bounce0_pixel_major(sv, fv);
    // culled pixels summed by k_sky (beside the trace when launches overlap): path-major batches.
    // (r04s: handing them to k_sky beside the thread-per-pixel bounce 0 too: C2 3.09-3.20 -> 3.54-3.57 ms)
    fv.sky_fold = (fv.cull != nullptr && fv.pixel_major == kFoldNone) ? 1u : 0u;
    fv.plist = fv.sky_fold ? static_cast<const uint32_t*>(c.plist.p) : nullptr;
    // fused bounces (k_bounce), in batches of every size since r06: r02 measured them on C2 only where
    // launches are short (8-way shard 0.627 -> 0.590 ms, 2-way 1.887 -> 1.822, but 1 GPU (133 M paths) 3.39
    // -> 3.46 ms: the traversal at the shading kernel's occupancy); after k_bounce01 they gain on the large
    // batches too (r06s: C4, 535 M-path batches, 122.2-122.6 -> 119.2-119.4 ms/step; C2 unchanged)
    const bool fuse_bounce = fuse && !no_bounce;
    // larger batches could fuse only their late bounces, whose queues are short: no gain measured
    // (r03zx, SPTR_FUSE_FROM 2/3/4 on C2: 3.16-3.25 vs 3.17 ms/step)
    const int fuse_from = fuse_bounce ? 1 : ((fuse && !no_bounce && fuse_from_env > 0) ? fuse_from_env : D + 1);
    // segment-table chain: trace(d) -> shade(d) -> {shadow(d), trace(d+1)}; each launcher returns
    // its grid size = the number of segments its consumers scan
    uint32_t g_shade = 0;
    // k_sky beside the tail instead of beside the bounce-0 trace, for scenes beyond an XCD's L2: there the
    // chain's traces are long and latency-bound, and the sky's VALU-bound grid beside bounce 0 took the
    // wave slots of the trace on the critical path (r05t: C5 7.34-7.37 -> 7.08-7.13 ms/step).  C3's
    // cubemap sky outlasts the whole chain (2.5 of 3.6 ms), so it keeps forking at bounce 0.
    const bool sky_late = fv.sky_fold && overlap && shadow_side && T < D && trace_queue_applies(sv);
    // fused bounces alternate the ray tables: the table holding the current rays, and the other
    SegTable rays_tab = w.segN, spare_tab = w.segH;
    for (int d = 0; d < D; ++d) {
      if (d >= T) {  // the remaining bounces, path per thread
        // (shadow(d - 1) adds to rad[], which the tail reads — unless the tail carries those shadow rays
        // itself (w.carry_depth); k_sky only to the culled pixels' accum, joined before k_accum, so the
        // tail runs beside it: C3's k_sky outlasts the whole bounce chain)
        if (w.carry_depth == kNoHit) join_shadow();
        WaveView wt = w;
        wt.segN = rays_tab;
        if (sky_late) {  // k_sky beside the tail, on the (joined) shadow stream, joined before k_accum
          fork_to(ss);
          launch_sky(sh, fv, true, ss);
          check(hipEventRecord(ev.join, ss), "sky join record");
          join = true;
        }
        tm.begin(7);
        launch_tail(sv, sh, fv, wt, d, g_shade, s);
        tm.end();
        break;
      }
      if (d >= fuse_from) {  // trace + shade (+ shadow) of this bounce in one launch
        WaveView wf = w;
        wf.segN = rays_tab;
        wf.segH = spare_tab;
        tm.begin(9);  // (a trace launch that also shades: ms_trace, trace_launches)
        g_shade = launch_bounce(sv, sh, fv, wf, d, g_shade, s);
        tm.end();
        std::swap(rays_tab, spare_tab);
        continue;
      }
      const bool sky = d == 0 && fv.sky_fold && !sky_late;  // the culled pixels' environment sums: accumulation, not k_trace
      const bool sky_side = sky && overlap;
      if (sky && !sky_side) {
        tm.begin(4);
        launch_sky(sh, fv, false, s);
        tm.end();
      }
      // k_sky forks at the same point as the bounce-0 trace (it writes only the culled pixels' accum
      // words, which nothing reads before this batch's k_accum, the join point): its VALU-bound blocks
      // fill the CUs the latency-bound trace leaves idle, above all in the trace's tail.  Enqueued
      // after the trace, so that the trace's grid is dispatched first.  (sky_late: beside the tail.)
      if (sky_side) {
        if (!cap) c.last_forked = true;
        check(hipEventRecord(ev.fork, s), "sky fork record");
      }
      // straggler hand-off of this bounce's trace (scenes beyond an XCD's L2; not the visit-count pass)
      WaveView wt = w;
      wt.strag_lanes = (strag && (uint32_t)d < kStragHandoffBounces) ? c.strag_lanes : 0u;
      tm.begin(d == 0 ? 5 : 1);
      const uint32_t g_trace = launch_trace(sv, sh, fv, wt, d, count, g_shade, s);
      tm.end();
      if (sky_side) {
        check(hipStreamWaitEvent(ks, ev.fork, 0), "sky fork wait");
        launch_sky(sh, fv, true, ks);
        check(hipEventRecord(ev.sky, ks), "sky join record");
        join_sky = true;
      }
      join_shadow();  // shadow(d - 1) before shade(d)
      if (wt.strag_lanes) {
        // k_strag(d) after trace(d) and shadow(d - 1) (both may have updated the handed-off paths'
        // radiance), on the k_sky stream, joined before k_accum with k_sky (ev.sky)
        if (overlap) {
          fork_to(ks);
          launch_strag(sv, sh, fv, w, d, ks);
          check(hipEventRecord(ev.sky, ks), "straggler join record");
          join_sky = true;
        } else {
          launch_strag(sv, sh, fv, w, d, s);
        }
      }
      if (d == 0 && fuse && !no_bounce && T >= 2 && D >= 2) {
        // bounce 0's shading and bounce 1 in one launch (k_bounce01), in batches of every size: its rays of
        // bounce 2 go to w.segN, where the fused bounces from 2 on (or k_trace(2)) take them.  r06 A/B on one
        // box: C2 (two lanes, fused bounces) 2.58-2.60 -> 2.36 ms/step, 8-way shard 0.52 -> 0.49; C4 (batches
        // of 535 M paths, separate stages from bounce 2) 136.6 -> 122.4 ms, C2 as one chain 3.01 -> 2.76
        // (gpurun_out/r06p, r06q)
        tm.begin(9);
        g_shade = launch_bounce01(sv, sh, fv, w, g_trace, s);
        tm.end();
        rays_tab = w.segN;
        spare_tab = w.segH;
        d = 1;
        continue;
      }
      tm.begin(d == 0 ? 6 : 2);
      g_shade = launch_shade(sv, sh, fv, w, d, g_trace, fuse, s);
      tm.end();
      if (!fuse && shadow_side) {
        fork_to(ss);
        tside.begin(3);
        launch_shadow(sv, sh, w, d, count, g_shade, ss);
        tside.end();
        check(hipEventRecord(ev.join, ss), "shadow join record");
        join = true;
      } else if (!fuse) {
        tm.begin(3);
        launch_shadow(sv, sh, w, d, count, g_shade, s);
        tm.end();
      }
    }
    // the call's last batch resolves in the same launch (k_accum<true>: each thread resolves the
    // sum it holds, as k_resolve would next)
    const bool resolve = done + kk >= f.spp && !(f.flags & SPTR_FRAME_NO_RESOLVE);
    join_shadow();
    if (join_sky) check(hipStreamWaitEvent(s, ev.sky, 0), "sky join wait");
    join_sky = false;
    tm.begin(4);
    if (done + kk >= f.spp) tm.last_launch();
    launch_accumulate(fv, w, static_cast<float4*>(c.accum.p), static_cast<uint32_t*>(c.tiles.p),
                      c.image_out ? c.image_out : static_cast<uint8_t*>(c.image.p), resolve, s);
    tm.end();
    done += kk;
    ++waves;
  }
  if (tside.err != hipSuccess && tm.err == hipSuccess) {
    tm.err = tside.err;
    tm.what = tside.what;
  }
  tm.end_call();
  return waves;
}

// The bounce-0 pixel-frustum cull mask (and unculled-pixel list) of a wavefront call's camera.  It is
// launched directly on the render stream ahead of the call's launch sequence, never inside it: a
// captured launch graph therefore holds no k_cull, and whichever camera a replayed graph was
// captured for, it runs against the mask of the camera of its own call (a graph key includes the
// camera; the mask is recomputed here whenever the camera, the cull depth or the state epoch differ
// from the cached mask's, and on SPTR_FRAME_RECULL).
int refresh_cull(Context& c, const sptr_frame& f, hipStream_t s, bool timing) {
  if (f.flags & SPTR_FRAME_NO_CULL) return SPTR_OK;
  const uint32_t depth = cull_depth_for(f.spp);
  if (f.flags & SPTR_FRAME_RECULL) {  // the call's own launch sequence computes the mask (enqueue_wavefront)
    c.cull_epoch = 0;  // the cached key is set once that sequence is enqueued (sptr_render)
    return SPTR_OK;
  }
  if (!(f.flags & SPTR_FRAME_RECULL) && c.cull_epoch == c.epoch && c.cull_depth == depth &&
      std::memcmp(&c.cull_cam, &f.camera, sizeof(sptr_camera)) == 0)
    return SPTR_OK;
  FrameView fv = frame_view(c, f);
  fv.cull_depth = depth;
  StageTimer tm{c, timing, true, s};
  tm.begin(8);
  API_HIP(hipMemsetAsync(static_cast<uint32_t*>(c.plist.p) + c.P, 0, 8, s));
  launch_cull(scene_view(c), fv, static_cast<uint32_t*>(c.cull.p), static_cast<uint32_t*>(c.plist.p), s);
  tm.end();
  API_HIP(hipGetLastError());
  if (tm.err != hipSuccess) return fail(c, SPTR_ERR_HIP, std::string("render: cull events: ") + hipGetErrorString(tm.err));
  c.cull_epoch = c.epoch;
  c.cull_cam = f.camera;
  c.cull_depth = depth;
  ++c.pending_culls;
  return SPTR_OK;
}

bool same_key(const GraphKey& a, const GraphKey& b) { return std::memcmp(&a, &b, sizeof(GraphKey)) == 0; }

// A captured launch graph is accepted only if it is a DAG of bounded depth: nodes, dependency
// edges and the number of nodes on its longest path (Kahn's algorithm over hipGraphGetEdges).  The
// fork/join plan of enqueue_wavefront yields ~10-200 nodes whose longest path is the main sequence;
// a cycle, or a path longer than the node count, means a broken plan.
struct GraphShape {
  uint32_t nodes = 0, edges = 0, depth = 0;
};
constexpr size_t kMaxGraphNodes = 4096;
bool check_graph(hipGraph_t g, GraphShape& out, std::string& why) {
  size_t n = 0, ne = 0;
  if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess || hipGraphGetEdges(g, nullptr, nullptr, &ne) != hipSuccess) {
    why = "hipGraphGetNodes/Edges failed";
    return false;
  }
  if (n == 0 || n > kMaxGraphNodes) {
    why = std::to_string(n) + " nodes";
    return false;
  }
  std::vector<hipGraphNode_t> nodes(n), from(ne), to(ne);
  if (hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess ||
      (ne && hipGraphGetEdges(g, from.data(), to.data(), &ne) != hipSuccess)) {
    why = "hipGraphGetNodes/Edges failed";
    return false;
  }
  std::vector<std::pair<hipGraphNode_t, uint32_t>> index(n);
  for (size_t i = 0; i < n; ++i) index[i] = {nodes[i], (uint32_t)i};
  std::sort(index.begin(), index.end());
  auto id_of = [&](hipGraphNode_t x) -> int64_t {
    const auto it = std::lower_bound(index.begin(), index.end(), std::make_pair(x, 0u));
    return (it != index.end() && it->first == x) ? (int64_t)it->second : -1;
  };
  std::vector<uint32_t> indeg(n, 0), level(n, 1);
  std::vector<std::vector<uint32_t>> succ(n);
  for (size_t e = 0; e < ne; ++e) {
    const int64_t a = id_of(from[e]), b = id_of(to[e]);
    if (a < 0 || b < 0) {
      why = "edge to an unknown node";
      return false;
    }
    succ[(size_t)a].push_back((uint32_t)b);
    ++indeg[(size_t)b];
  }
  std::vector<uint32_t> ready;
  for (uint32_t i = 0; i < n; ++i)
    if (indeg[i] == 0) ready.push_back(i);
  size_t seen = 0;
  uint32_t depth = 0;
  while (!ready.empty()) {
    const uint32_t v = ready.back();
    ready.pop_back();
    ++seen;
    depth = std::max(depth, level[v]);
    for (uint32_t w : succ[v]) {
      level[w] = std::max(level[w], level[v] + 1);
      if (--indeg[w] == 0) ready.push_back(w);
    }
  }
  out.nodes = (uint32_t)n;
  out.edges = (uint32_t)ne;
  out.depth = depth;
  if (seen != n) {
    why = "dependency cycle (" + std::to_string(n - seen) + " of " + std::to_string(n) + " nodes)";
    return false;
  }
  return true;
}

void drop_graph(Context& c) {
  if (c.graph.exec) (void)hipGraphExecDestroy(c.graph.exec);
  if (c.graph.graph) (void)hipGraphDestroy(c.graph.graph);
  c.graph = GraphCache{};
}

// Enqueue one render call's launch sequence on s.  A call shape seen twice in a row is captured
// once into a hipGraph (on the context's capture stream) and replayed from then on: one graph
// launch instead of ~20 kernel launches, with the per-call values (frame_begin, reset, total) passed
// as the arguments of the graph's k_frame_dyn node.  The launch sequence itself is the same code
// either way.  A replay's call span (stage 0) is recorded around its hipGraphLaunch; calls with stage
// timing (SPTR_FRAME_TIMING*) always run as direct launches: a stage span inside a graph would need
// external event-record nodes, which torch's HIP 7.0 runtime (the one bench.py and any process that
// imports torch first binds libsptr_hip to) refuses inside a capture (hipErrorInvalidValue, r04g).
constexpr uint64_t kGraphMinSamples = 1ull << 24;  // launch mode 0 captures calls of at least this many samples
template <class Enqueue>
int run_call(Context& c, const GraphKey& key, uint32_t frame_begin, uint32_t reset, uint32_t total, uint64_t samples, uint32_t* clear,
             bool timing, bool trace_only, hipStream_t s, Enqueue&& enqueue, uint32_t& waves) {
  const bool repeat = c.have_last_key && same_key(key, c.last_key);
  c.last_key = key;
  c.have_last_key = true;
  // mode 0 captures a call whose launches fork nothing to the side streams: the runtime's graph executor
  // does not run a graph's parallel branches concurrently, so a call with side-stream launches replays
  // slower than it launches directly, at every size measured (r04h: C5 8.70 vs 8.18 ms, C3 3.80 vs 3.75;
  // r05i, 1-spp frames, C5 at 256x144 / 512x288 / 960x540 / 1920x1080: 1.87 / 2.21 / 2.52 / 3.11 vs
  // 1.23 / 1.50 / 1.72 / 2.22 ms, C3 0.46 / 0.61 / 0.78 / 0.96 vs 0.44 / 0.57 / 0.73 / 0.92 ms; r05k, the
  // default scene's 1-spp 1080p frame, which forks only k_sky: 0.47 vs 0.41 ms).  C2's 64-spp call forks
  // nothing: 3.07 graph vs 3.10 ms direct.  Mode 3 captures every repeated shape.
  // Nor does mode 0 capture small calls: the default scene's 1-spp frames (r05zh, sptr_cli, 400 frames,
  // two repetitions; mean wall / device ms, graph vs direct) 640x360 0.42/0.18 and 0.31/0.18 vs 0.38/0.19
  // and 0.30/0.20; 800x600 0.33/0.21 vs 0.31/0.22; 1280x720 0.37-0.38/0.22 vs 0.35/0.24; 1920x1080 (whose
  // pixel-major bounce 0 forks nothing) 0.46/0.25 vs 0.41-0.42/0.23 — the replays' device time is at best
  // 10 us shorter and their wall time has spikes.  Calls from kGraphMinSamples on (C2: 2.98 vs 3.02 ms).
  // Nor the halves of a two-lane call (time_by_events marks them): the two lanes' graphs replayed beside
  // each other measured slower than their direct launches (r05i, C2: 2.865 vs 2.528 ms per call).
  const bool graphable = c.launch_mode == 3 ||
                         (c.launch_mode == 0 && !c.last_forked && !c.time_by_events && samples >= kGraphMinSamples);
  const bool bad = c.have_bad_key && same_key(key, c.bad_key);  // this shape failed to capture before
  auto direct = [&]() -> int {
    c.last_forked = false;  // (set by the launch sequence if it forks)
    StageTimer tm{c, timing, trace_only, s};
    // untimed two-lane calls launch their trace and fused-bounce kernels with dispatch events all the same
    // (two events reused by every such launch, never read): r06l, C2 2.512-2.531 vs 2.548-2.565 ms per step
    // with plain launches, on one box
    tm.quiet = !timing && c.time_by_events && c.quiet_ev[1] != nullptr;
    unsigned long long* t0 = tm.pre_call(key.frame.integrator == SPTR_INTEGRATOR_WAVEFRONT);
    launch_frame_dyn(static_cast<uint32_t*>(c.dyn.p), frame_begin, reset, total, clear, t0, s);
    waves = enqueue(s, tm);
    API_HIP(hipGetLastError());
    if (tm.err != hipSuccess) return fail(c, SPTR_ERR_HIP, "render: " + tm.what + ": " + hipGetErrorString(tm.err));
    return SPTR_OK;
  };
  if (!graphable || timing || bad || !(repeat || (c.graph.valid && same_key(key, c.graph.key)))) return direct();
  if (!(c.graph.valid && same_key(key, c.graph.key))) {  // capture this shape
    drop_graph(c);
    // a pixel lane's capture stream is its own, created on its first capture (only launch mode 3 captures
    // a lane's calls).  r06: with one capture stream shared by the two contexts, a parent's capture after
    // the lane's (a mode-3 two-lane shape, then direct two-lane calls, then a one-chain shape captured in
    // mode 0) was instantiated, and its first hipGraphLaunch faulted inside torch's HIP runtime (a null
    // member read at libamdhip64+0xaee41, gpurun_out/r06e); with a stream per context it does not.
    if (!c.cap_stream && hipStreamCreateWithFlags(&c.cap_stream, hipStreamNonBlocking) != hipSuccess) {
      c.cap_stream = nullptr;
      (void)hipGetLastError();
      return direct();
    }
    GraphShape gshape;
    // A shape that cannot be captured (the capture fails, leaves a forked stream capturing, or yields
    // a graph check_graph rejects or the runtime cannot instantiate) is remembered and launched
    // directly, this call and every later one: the direct launches are safe (the runtime faults
    // only while ending a capture), and a failing shape re-captured per call would never render.
    // graph_info / sptr_capture_error report why.
    auto not_capturable = [&](hipError_t status, const std::string& why) -> int {
      c.capture_status = (int32_t)(status != hipSuccess ? status : hipErrorUnknown);
      c.capture_error = why;
      c.bad_key = key;
      c.have_bad_key = true;
      (void)hipGetLastError();
      return direct();
    };
    API_HIP(hipStreamBeginCapture(c.cap_stream, hipStreamCaptureModeThreadLocal));
    StageTimer tm{c, false, false, c.cap_stream};
    tm.capturing = true;
    const uint32_t nw = enqueue(c.cap_stream, tm);
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(c.cap_stream, &g);
    // every stream the capture forked must have left capture mode with it (a stream still capturing
    // would fold the next direct launches into a dead graph): end the capture on any that did not
    bool stuck = false;
    for (hipStream_t st : {c.cap_stream, c.cap_side, c.cap_side2}) {
      if (!st) continue;
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
        stuck = true;
        hipGraph_t gs = nullptr;
        (void)hipStreamEndCapture(st, &gs);
        if (gs) (void)hipGraphDestroy(gs);
      }
    }
    if (stuck) {
      if (g) (void)hipGraphDestroy(g);
      return not_capturable(hipErrorStreamCaptureUnjoined, "graph capture: a forked stream was still capturing");
    }
    if (ec != hipSuccess || tm.err != hipSuccess || !g) {
      if (g) (void)hipGraphDestroy(g);
      return not_capturable(ec != hipSuccess ? ec : tm.err,
                            ec != hipSuccess ? std::string("hipStreamEndCapture: ") + hipGetErrorString(ec)
                                             : tm.what + ": " + hipGetErrorString(tm.err));
    }
    {
      std::string why;
      if (!check_graph(g, gshape, why)) {
        (void)hipGraphDestroy(g);
        return not_capturable(hipErrorInvalidValue, "captured graph rejected: " + why);
      }
    }
    GraphCache gc;
    gc.graph = g;
    gc.key = key;
    gc.waves = nw;
    gc.nodes = gshape.nodes + 1;  // + the k_frame_dyn head added below, ahead of every root
    gc.depth = gshape.depth + 1;
    // the k_frame_dyn node heads the graph: every captured root depends on it
    size_t nr = 0;
    API_HIP(hipGraphGetRootNodes(g, nullptr, &nr));
    std::vector<hipGraphNode_t> roots(nr);
    API_HIP(hipGraphGetRootNodes(g, roots.data(), &nr));
    void* dyn_ptr = c.dyn.p;
    uint32_t a0 = frame_begin, a1 = reset, a2 = total;
    uint32_t* a3 = clear;
    unsigned long long* a4 = nullptr;  // (a replay's call span: event records around its launch)
    void* args[6] = {&dyn_ptr, &a0, &a1, &a2, &a3, &a4};
    hipKernelNodeParams kp{};
    kp.func = const_cast<void*>(frame_dyn_kernel());
    kp.gridDim = dim3(1);
    kp.blockDim = dim3(64);
    kp.sharedMemBytes = 0;
    kp.kernelParams = args;
    kp.extra = nullptr;
    API_HIP(hipGraphAddKernelNode(&gc.dyn_node, g, nullptr, 0, &kp));
    for (hipGraphNode_t r : roots) API_HIP(hipGraphAddDependencies(g, &gc.dyn_node, &r, 1));
    gc.edges = gshape.edges + (uint32_t)nr;
    gc.dyn_params = kp;
    const hipError_t ei = hipGraphInstantiate(&gc.exec, g, nullptr, nullptr, 0);
    if (ei != hipSuccess) {
      (void)hipGraphDestroy(g);
      return not_capturable(ei, std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
    }
    gc.valid = true;
    c.graph = gc;
    ++c.captures;
  }
  // replay: the call's values into the k_frame_dyn node, the call span around the launch
  GraphCache& gc = c.graph;
  void* dyn_ptr = c.dyn.p;
  uint32_t a0 = frame_begin, a1 = reset, a2 = total;
  uint32_t* a3 = clear;
  unsigned long long* a4 = nullptr;
  void* args[6] = {&dyn_ptr, &a0, &a1, &a2, &a3, &a4};
  hipKernelNodeParams p = gc.dyn_params;
  p.kernelParams = args;
  p.extra = nullptr;
  API_HIP(hipGraphExecKernelNodeSetParams(gc.exec, gc.dyn_node, &p));
  StageTimer tm{c, false, false, s};
  tm.begin_call();
  API_HIP(hipGraphLaunch(gc.exec, s));
  tm.end_call();
  if (tm.err != hipSuccess) return fail(c, SPTR_ERR_HIP, "render: " + tm.what + ": " + hipGetErrorString(tm.err));
  waves = gc.waves;
  return SPTR_OK;
}

}  // namespace
}  // namespace sptr

namespace sptr {
namespace {
std::vector<hipEvent_t*> dep_events(Context& c) {
  std::vector<hipEvent_t*> v;
  for (Context::DepEvents& d : c.dev)
    for (hipEvent_t* e : {&d.fork, &d.join, &d.sky}) v.push_back(e);
  return v;
}
bool create_events(Context& c) {
  for (hipEvent_t* e : dep_events(c))
    if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return false;
  for (hipEvent_t& e : c.quiet_ev)
    if (hipEventCreate(&e) != hipSuccess) return false;
  return true;
}
}  // namespace
}  // namespace sptr

using namespace sptr;

extern "C" {

static void add_stats(sptr_stats& a, const sptr_stats& b);  // (pixel lanes, below)

int sptr_abi_version(void) { return SPTR_ABI_VERSION; }


// SPTR_SEGV_TRACE=1 (diagnostics only): a host SIGSEGV prints, before the default action, the fault
// address, the faulting instruction and stack pointer, each code address among the 512 words above the
// stack pointer as library + offset (a scan that needs no unwinder, so it works on an overflowed stack),
// and then the unwinder's backtrace.  Installed once per process, on the first sptr_create, for the
// thread that creates the context (its alternate signal stack).
static void segv_put(const char* s) { (void)!write(2, s, strlen(s)); }
static void segv_hex(uint64_t v) {
  char b[19] = "0x";
  for (int i = 0; i < 16; ++i) b[2 + i] = "0123456789abcdef"[(v >> (60 - 4 * i)) & 15u];
  b[18] = 0;
  segv_put(b);
}
static void segv_where(uint64_t pc) {
  Dl_info di{};
  segv_hex(pc);
  if (dladdr(reinterpret_cast<void*>(pc), &di) && di.dli_fname) {
    segv_put(" ");
    segv_put(di.dli_fname);
    segv_put("+");
    segv_hex(pc - reinterpret_cast<uint64_t>(di.dli_fbase));
    if (di.dli_sname) {
      segv_put(" ");
      segv_put(di.dli_sname);
    }
  }
  segv_put("\n");
}
static void segv_trace(int sig, siginfo_t* si, void* uc_v) {
  const ucontext_t* uc = static_cast<const ucontext_t*>(uc_v);
  const uint64_t pc = (uint64_t)uc->uc_mcontext.gregs[REG_RIP], sp = (uint64_t)uc->uc_mcontext.gregs[REG_RSP];
  segv_put("sptr SIGSEGV: addr ");
  segv_hex(reinterpret_cast<uint64_t>(si->si_addr));
  segv_put(" sp ");
  segv_hex(sp);
  segv_put("\n  pc ");
  segv_where(pc);
  const uint64_t* st = reinterpret_cast<const uint64_t*>(sp);
  for (int i = 0, shown = 0; i < 512 && shown < 96; ++i) {
    Dl_info di{};
    const uint64_t v = st[i];
    if (v > 4096 && dladdr(reinterpret_cast<void*>(v), &di) && di.dli_fname) {
      ++shown;
      segv_put("  ret? ");
      segv_where(v);
    }
  }
  void* fr[64];
  const int n = backtrace(fr, 64);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

static void install_segv_trace() {
  static std::once_flag once;
  std::call_once(once, [] {
    if (getenv("SPTR_SEGV_TRACE") == nullptr) return;
    void* prime[2];
    (void)backtrace(prime, 2);
    static char alt[1 << 20];
    stack_t ss{};
    ss.ss_sp = alt;
    ss.ss_size = sizeof(alt);
    sigaltstack(&ss, nullptr);
    struct sigaction sa{};
    sa.sa_sigaction = segv_trace;
    sa.sa_flags = SA_ONSTACK | SA_SIGINFO;
    sigaction(SIGSEGV, &sa, nullptr);
  });
}

static int create_one(int device, sptr_ctx** out, const sptr_ctx* parent);
int sptr_create(int device, sptr_ctx** out) {
  const int rc = create_one(device, out, nullptr);
  if (rc != SPTR_OK) return rc;
  sptr_ctx* x = *out;
  // the pixel lane: a context of its own (created now, given a scene and a stream only when the scene
  // is staged into LDS)
  if (create_one(device, &x->lane, x) != SPTR_OK) x->lane = nullptr;
  if (x->lane) {
    x->lane->is_lane = true;
    if (hipEventCreateWithFlags(&x->lane_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&x->lane_join, hipEventDisableTiming) != hipSuccess) {
      (void)sptr_destroy(x);
      *out = nullptr;
      return SPTR_ERR_HIP;
    }
  }
  return SPTR_OK;
}

// parent: a pixel lane's context.  It creates no stream here: it borrows the parent's capture stream
// (captures run one at a time on the calling thread), gets its render stream when it is given a scene
// (sptr_upload_scene) and has no side streams (it renders only scenes staged into LDS, whose launches
// run on one stream).  r05zw: every stream a context creates is one more for the runtime to place on
// the process's hardware queues, and a lane created with a full set of six slowed the parent's
// overlapped C5 / C3 calls from 7.23 / 3.33 to 8.48 / 3.67 ms with the lane never used.
static int create_one(int device, sptr_ctx** out, const sptr_ctx* parent) {
  if (!out) return SPTR_ERR_INVALID;
  install_segv_trace();
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return SPTR_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return SPTR_ERR_INVALID;
  sptr_ctx* x = new sptr_ctx();
  Context& c = x->c;
  c.device = device;
  if (parent) {
    c.parent = &parent->c;
    c.prio_lo = parent->c.prio_lo;
    c.prio_hi = parent->c.prio_hi;
    if (hipSetDevice(device) != hipSuccess || !create_events(c)) {
      delete x;
      return SPTR_ERR_HIP;
    }
  } else if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c.cap_stream, hipStreamNonBlocking) != hipSuccess ||
      // the side streams at the lowest priority: a priority of its own puts a stream on a hardware
      // queue of its own, so that its launches can run beside the main sequence's.  (r05t: the main
      // streams at the highest priority instead of the default changed nothing, C3 and C5.)
      hipDeviceGetStreamPriorityRange(&c.prio_lo, &c.prio_hi) != hipSuccess ||
      hipStreamCreateWithPriority(&c.side_stream, hipStreamNonBlocking, c.prio_lo) != hipSuccess ||
      hipStreamCreateWithPriority(&c.cap_side, hipStreamNonBlocking, c.prio_lo) != hipSuccess ||
      hipStreamCreateWithPriority(&c.side2_stream, hipStreamNonBlocking, c.prio_lo) != hipSuccess ||
      hipStreamCreateWithPriority(&c.cap_side2, hipStreamNonBlocking, c.prio_lo) != hipSuccess ||
      !create_events(c)) {
    delete x;
    return SPTR_ERR_HIP;
  }
  int khz = 0;
  if (ensure_buf(c.wb.seg, seg_table_bytes()) != hipSuccess || ensure_buf(c.w_tot, kTotWords * 8) != hipSuccess ||
      ensure_buf(c.dyn, kDynBytes) != hipSuccess || hipMemset(c.wb.seg.p, 0, seg_table_bytes()) != hipSuccess ||
      ensure_buf(c.tslots, (size_t)kTimeSlots * kTimeSlotWords * 8) != hipSuccess ||
      hipMemset(c.tslots.p, 0, (size_t)kTimeSlots * kTimeSlotWords * 8) != hipSuccess ||
      hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) {
    delete x;
    return SPTR_ERR_OOM;
  }
  c.wall_khz = khz;
  *out = x;
  return SPTR_OK;
}

int sptr_destroy(sptr_ctx* x) {
  if (!x) return SPTR_ERR_INVALID;
  // this context's stream first: after an asynchronous two-lane call it may still run
  // k_interleave_tiles, which reads the lane's tiles
  (void)hipSetDevice(x->c.device);
  if (x->c.pending) (void)hipStreamSynchronize(x->c.pending_stream);
  if (x->c.stream) (void)hipStreamSynchronize(x->c.stream);
  if (x->copy_stream) {  // the lagged readback's copy stream, snapshots and registered destination
    (void)hipStreamSynchronize(x->copy_stream);
    (void)hipStreamDestroy(x->copy_stream);
  }
  if (x->copy_done) (void)hipEventDestroy(x->copy_done);
  for (auto& sn : x->snap) {
    free_buf(sn.buf);
    if (sn.ready) (void)hipEventDestroy(sn.ready);
  }
  if (x->reg_ptr) (void)hipHostUnregister(x->reg_ptr);
  if (x->lane) (void)sptr_destroy(x->lane);
  x->lane = nullptr;
  for (hipEvent_t e : {x->lane_fork, x->lane_join})
    if (e) (void)hipEventDestroy(e);
  free_buf(x->tiles_full);
  Context& c = x->c;
  (void)hipSetDevice(c.device);
  if (c.pending) (void)hipStreamSynchronize(c.pending_stream);
  if (c.stream) (void)hipStreamSynchronize(c.stream);
  DevBuf* bufs[] = {&c.nodes,  &c.prim_ref, &c.tris,  &c.sph,   &c.tri_geom, &c.sph_geom, &c.tri_orig,
                    &c.sph_orig, &c.geom_mat, &c.tri_mat, &c.mats, &c.env, &c.w_tot,  &c.accum,   &c.tiles,
                    &c.image,    &c.qbuf,     &c.nodes4, &c.cull, &c.plist, &c.tslots};
  for (DevBuf* b : bufs) free_buf(*b);
  for (DevBuf* b : {&c.wb.hrec, &c.wb.rad, &c.wb.stask, &c.wb.seg, &c.wb.strag}) free_buf(*b);
  for (auto& r : c.wb.rs)
    for (DevBuf& x : r) free_buf(x);
  for (hipStream_t st : {c.side2_stream, c.cap_side2})
    if (st) (void)hipStreamDestroy(st);
  drop_graph(c);
  free_buf(c.dyn);
  for (hipEvent_t e : c.events) (void)hipEventDestroy(e);
  if (c.stream) (void)hipStreamDestroy(c.stream);
  if (c.cap_stream) (void)hipStreamDestroy(c.cap_stream);
  if (c.side_stream) (void)hipStreamDestroy(c.side_stream);
  if (c.cap_side) (void)hipStreamDestroy(c.cap_side);
  for (hipEvent_t* e : dep_events(c))
    if (*e) (void)hipEventDestroy(*e);
  for (hipEvent_t e : c.quiet_ev)
    if (e) (void)hipEventDestroy(e);
  delete x;
  return SPTR_OK;
}

const char* sptr_last_error(const sptr_ctx* x) { return x ? x->c.err.c_str() : "null context"; }

static int set_debug_mode_one(sptr_ctx* x, int mode) {
  if (!x) return SPTR_ERR_INVALID;
  x->c.debug_mode = mode;
  ++x->c.epoch;
  return SPTR_OK;
}

static int set_leaf_size_one(sptr_ctx* x, uint32_t n) {
  if (!x) return SPTR_ERR_INVALID;
  if (n > kMaxLeafSize) return fail(x->c, SPTR_ERR_INVALID, "leaf size must be 0 (automatic) or 1..16");
  x->c.leaf_size = n;
  ++x->c.epoch;
  return SPTR_OK;
}

static int set_bvh_width_one(sptr_ctx* x, uint32_t width) {
  if (!x) return SPTR_ERR_INVALID;
  if (width != 0 && width != 2 && width != (uint32_t)kWide)
    return fail(x->c, SPTR_ERR_INVALID, "bvh width must be 0 (auto), 2 or " + std::to_string(kWide));
  x->c.bvh_width = width;
  ++x->c.epoch;
  return SPTR_OK;
}

static int set_tail_depth_one(sptr_ctx* x, uint32_t depth) {
  if (!x) return SPTR_ERR_INVALID;
  if (depth > (uint32_t)kMaxDepth) return fail(x->c, SPTR_ERR_INVALID, "tail depth must be 0 (automatic) or 1..32");
  x->c.tail_depth = depth;
  ++x->c.epoch;
  return SPTR_OK;
}

static int set_split_refs_one(sptr_ctx* x, uint32_t max_pieces) {
  if (!x) return SPTR_ERR_INVALID;
  if (max_pieces == 0u) max_pieces = 1u;
  if (max_pieces > 32u || (max_pieces & (max_pieces - 1u)))
    return fail(x->c, SPTR_ERR_INVALID, "split references: 0 (default: 1, none) or a power of two up to 32");
  x->c.split_pieces = max_pieces;
  ++x->c.epoch;
  return SPTR_OK;
}

static int set_stragglers_one(sptr_ctx* x, uint32_t lanes) {
  if (!x) return SPTR_ERR_INVALID;
  if (lanes > 64u) return fail(x->c, SPTR_ERR_INVALID, "straggler lanes: 0 (no hand-off) to 64");
  x->c.strag_lanes = lanes;
  ++x->c.epoch;  // part of every captured launch sequence's arguments
  return SPTR_OK;
}

static int set_wave_paths_one(sptr_ctx* x, uint64_t max_paths) {
  if (!x) return SPTR_ERR_INVALID;
  if (max_paths > (1ull << 30)) return fail(x->c, SPTR_ERR_INVALID, "wave paths above 2^30");
  x->c.wave_paths = max_paths;
  ++x->c.epoch;
  return SPTR_OK;
}

static int upload_scene_one(sptr_ctx* x, const sptr_scene* s) {
  if (!x || !s) return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;  // a pending render may still read the old state
  API_HIP(hipSetDevice(c.device));
  if ((s->num_tris && (!s->indices || !s->positions || !s->tri_geom_first)) || (s->num_spheres && !s->spheres) ||
      ((s->num_tri_geoms + s->num_spheres) && !s->geom_material))
    return fail(c, SPTR_ERR_INVALID, "scene: null array with nonzero count");
  // leaf links keep 32 - 1 - kLeafCountBits bits of range start
  if ((uint64_t)s->num_tris + s->num_spheres >= (1ull << (31 - kLeafCountBits)))
    return fail(c, SPTR_ERR_INVALID, "scene too large (at most 2^26 primitives)");
  if (s->num_tri_geoms && s->tri_geom_first[s->num_tri_geoms] != s->num_tris)
    return fail(c, SPTR_ERR_INVALID, "scene: tri_geom_first must end at num_tris");
  for (uint64_t i = 0; i < (uint64_t)s->num_tris * 3; ++i)
    if (s->indices[i] >= s->num_verts) return fail(c, SPTR_ERR_INVALID, "scene: vertex index out of range");
  std::vector<uint32_t> tg(s->num_tris);
  for (uint32_t g = 0; g < s->num_tri_geoms; ++g) {
    if (s->tri_geom_first[g] > s->tri_geom_first[g + 1]) return fail(c, SPTR_ERR_INVALID, "scene: geom offsets");
    for (uint32_t i = s->tri_geom_first[g]; i < s->tri_geom_first[g + 1]; ++i) tg[i] = g;
  }
  c.have_scene = false;
  c.num_tri_geoms = s->num_tri_geoms;
  c.geom_first.assign(s->tri_geom_first, s->tri_geom_first + (s->num_tri_geoms ? s->num_tri_geoms + 1 : 0));
  c.geom_material.assign(s->geom_material, s->geom_material + s->num_tri_geoms + s->num_spheres);
  const int rc = build_lbvh(c, s->positions, s->num_verts, s->indices, s->num_tris, s->spheres, s->num_spheres, tg.data(),
                            s->num_tri_geoms);
  if (rc != SPTR_OK) return rc;
  c.have_scene = true;
  ++c.epoch;
  return resolve_geom_materials(c);
}

int sptr_scene_info(const sptr_ctx* x, uint32_t* num_prims, uint32_t* num_nodes, uint32_t* depth, double* build_ms) {
  if (!x) return SPTR_ERR_INVALID;
  const Context& c = x->c;
  if (num_prims) *num_prims = c.num_tris + c.num_sph;
  if (num_nodes) *num_nodes = c.num_nodes;
  if (depth) *depth = c.bvh_depth;
  if (build_ms) *build_ms = c.build_ms;
  return SPTR_OK;
}

int sptr_scene_layout_info(const sptr_ctx* x, sptr_scene_layout* out) {
  if (!x || !out) return SPTR_ERR_INVALID;
  const Context& c = x->c;
  const SceneView sv = scene_view(c);
  out->num_tris = c.num_tris;
  out->num_spheres = c.num_sph;
  out->num_nodes = c.num_nodes;
  out->leaf_size = c.leaf_used;
  out->bvh_depth = c.bvh_depth;
  out->lds_bytes = sv.lds_bytes;
  out->bvh_width = sv.width;
  out->num_nodes = sv.width == (uint32_t)kWide ? c.num_nodes4 : c.num_nodes;
  out->node_bytes = sv.width == (uint32_t)kWide ? (uint64_t)c.num_nodes4 * sizeof(WideNode) : (uint64_t)c.num_nodes * sizeof(BvhNode);
  out->tri_bytes = (uint64_t)c.num_tri_refs * 48u;
  out->sphere_bytes = (uint64_t)c.num_sph * 16u;
  out->prim_ref_bytes = ((uint64_t)c.num_tri_refs + c.num_sph) * 4u;
  out->num_prim_refs = c.num_tri_refs + c.num_sph;
  return SPTR_OK;
}

static int set_materials_one(sptr_ctx* x, const sptr_material* m, uint32_t n) {
  if (!x || (n && !m)) return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;  // a pending render may still read the old state
  if (n == 0) return fail(c, SPTR_ERR_INVALID, "at least one material is required");
  API_HIP(hipSetDevice(c.device));
  c.mats_host.resize(n);
  std::memcpy(c.mats_host.data(), m, sizeof(DevMaterial) * n);
  API_HIP(ensure_buf(c.mats, sizeof(DevMaterial) * n));
  API_HIP(hipMemcpy(c.mats.p, c.mats_host.data(), sizeof(DevMaterial) * n, hipMemcpyHostToDevice));
  ++c.epoch;
  return resolve_geom_materials(c);
}

static int set_lights_one(sptr_ctx* x, const sptr_light* l, uint32_t n) {
  if (!x || (n && !l)) return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (n > (uint32_t)kMaxLights) return fail(c, SPTR_ERR_INVALID, "too many lights");
  c.lights_host.resize(n);
  ++c.epoch;
  for (uint32_t i = 0; i < n; ++i) {
    DevLight& d = c.lights_host[i];
    d.type = l[i].type;
    if (l[i].type == 0) {  // DirectionalLight stores normalize(-direction) (Light.cpp:43-46)
      const vec3 v = normalize(-v3(l[i].v[0], l[i].v[1], l[i].v[2]));
      d.v[0] = v.x; d.v[1] = v.y; d.v[2] = v.z;
    } else if (l[i].type == 1) {
      d.v[0] = l[i].v[0]; d.v[1] = l[i].v[1]; d.v[2] = l[i].v[2];
    } else {
      return fail(c, SPTR_ERR_INVALID, "unknown light type");
    }
    const vec3 r = v3(l[i].color[0], l[i].color[1], l[i].color[2]) * l[i].intensity;
    d.radiance[0] = r.x; d.radiance[1] = r.y; d.radiance[2] = r.z;
    d.pad = 0.0f;
  }
  return SPTR_OK;
}

static int set_environment_one(sptr_ctx* x, const sptr_environment* e) {
  if (!x) return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;  // a pending render may still read the old state
  API_HIP(hipSetDevice(c.device));
  if (!e || !e->faces) {
    free_buf(c.env);
    ++c.epoch;
    c.env_size = 0;
    if (e) {
      c.env_intensity = e->intensity;
      c.env_clamp = e->max_clamp;
    }
    return SPTR_OK;
  }
  if (e->size < 2) return fail(c, SPTR_ERR_INVALID, "environment face size must be >= 2");
  const size_t texels = (size_t)6 * e->size * e->size;
  std::vector<float> tmp(texels * 4);
  for (size_t i = 0; i < texels; ++i) {
    tmp[i * 4 + 0] = e->faces[i * 3 + 0];
    tmp[i * 4 + 1] = e->faces[i * 3 + 1];
    tmp[i * 4 + 2] = e->faces[i * 3 + 2];
    tmp[i * 4 + 3] = 0.0f;
  }
  API_HIP(ensure_buf(c.env, texels * 16));
  API_HIP(hipMemcpy(c.env.p, tmp.data(), texels * 16, hipMemcpyHostToDevice));
  c.env_size = e->size;
  ++c.epoch;
  c.env_intensity = e->intensity;
  c.env_clamp = e->max_clamp;
  return SPTR_OK;
}

static int render_one(sptr_ctx* x, const sptr_frame* f, void* stream, sptr_stats* stats) {
  if (!x || !f) return SPTR_ERR_INVALID;
  Context& c = x->c;
  API_HIP(hipSetDevice(c.device));
  if (!c.have_scene) return fail(c, SPTR_ERR_NO_SCENE, "render: no scene uploaded");
  if (shading(c).mats_host.empty()) return fail(c, SPTR_ERR_NO_SCENE, "render: no materials set");
  if (f->width <= 0 || f->height <= 0 || f->spp == 0 || f->max_depth == 0 || f->max_depth > (uint32_t)kMaxDepth ||
      f->frame_begin == 0)
    return fail(c, SPTR_ERR_INVALID, "render: bad frame parameters");
  if (f->integrator > SPTR_INTEGRATOR_OPTIX) return fail(c, SPTR_ERR_INVALID, "render: unknown integrator");
  if (f->integrator == SPTR_INTEGRATOR_PATHTRACER && f->samples_per_frame > 4096)
    return fail(c, SPTR_ERR_INVALID, "render: samples_per_frame above 4096");
  const int G = f->shard_count > 0 ? f->shard_count : 1, R = f->shard_count > 0 ? f->shard_rank : 0;
  if (R < 0 || R >= G) return fail(c, SPTR_ERR_INVALID, "render: shard_rank out of range");
  const int ntiles = ((f->width + kTile - 1) / kTile) * ((f->height + kTile - 1) / kTile);
  if (R >= ntiles) return fail(c, SPTR_ERR_INVALID, "render: more shards than tiles");
  if ((uint64_t)f->width * f->height > (1ull << 28)) return fail(c, SPTR_ERR_INVALID, "render: image too large");
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c.stream;
  if (c.pending && s != c.pending_stream)
    return fail(c, SPTR_ERR_INVALID, "render: asynchronous renders must stay on one stream until sptr_collect_stats");
  bool resized = false;
  int rc = ensure_pixels(c, f->width, f->height, G, R, s, resized);
  if (rc != SPTR_OK) return rc;
  const bool reset = f->frame_begin == 1;
  if (!reset && f->frame_begin != c.last_samples + 1)
    return fail(c, SPTR_ERR_INVALID, "render: frame_begin must continue the accumulation (last + 1) or be 1");
  const bool timing = (f->flags & SPTR_FRAME_TIMING) != 0;
  const bool trace_timing = (f->flags & SPTR_FRAME_TIMING_TRACE) != 0;
  const uint32_t total = f->frame_begin + f->spp - 1;
  GraphKey key{};
  key.epoch = c.epoch;
  key.frame = *f;
  key.frame.frame_begin = 0;
  key.frame.flags &= (SPTR_FRAME_TIMING | SPTR_FRAME_TIMING_TRACE | SPTR_FRAME_COUNT_VISITS | SPTR_FRAME_NO_RESOLVE |
                      SPTR_FRAME_NO_CULL | SPTR_FRAME_RECULL);
  uint32_t waves = 0;
  uint64_t samples = 0;
  if (f->integrator != SPTR_INTEGRATOR_WAVEFRONT) {
    if (c.pending == 0) API_HIP(hipMemsetAsync(c.w_tot.p, 0, kTotWords * 8, s));
    const uint32_t spf = f->integrator == SPTR_INTEGRATOR_PATHTRACER ? (f->samples_per_frame ? f->samples_per_frame : 4u) : 1u;
    rc = run_call(c, key, f->frame_begin, reset ? 1u : 0u, total, (uint64_t)frame_view(c, *f).valid * f->spp, nullptr,
                  timing || trace_timing, false, s,
                  [&](hipStream_t cs, StageTimer& tm) { return enqueue_path_per_thread(c, *f, cs, tm); }, waves);
    if (rc != SPTR_OK) return rc;
    samples = (uint64_t)frame_view(c, *f).valid * f->spp * spf;
  } else {
    uint64_t wave_paths = c.wave_paths;
    if (!wave_paths) {  // default: 2^29 paths, or what half of the free HBM holds (at least 2^24)
      wave_paths = kDefaultWavePaths;
      if (c.wb.cap < std::min<uint64_t>(wave_paths, (uint64_t)f->spp * c.P)) {  // would (re)allocate
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b) {
          const uint32_t hm = hrec_mult(scene_view(c));
          const uint64_t held = c.wb.cap ? c.wb.cap * wave_path_bytes(c.wb.L, c.wb.ts, hm) : 0ull;
          const uint32_t L = std::max<uint32_t>(1u, (uint32_t)shading(c).lights_host.size());
          // budget net of the streams' segment slack (worst case: pixel-major hit records, k <= spp)
          const double budget = ((double)free_b + (double)held) * kWaveMemFraction -
                                (double)wave_slack_bytes(L, task_stride(c), std::min<uint32_t>(f->spp, 1024u), hm);
          const uint64_t fit = budget > 0.0 ? (uint64_t)budget / wave_path_bytes(L, task_stride(c), hm) : 0ull;
          wave_paths = std::max<uint64_t>(1ull << 24, std::min<uint64_t>(wave_paths, fit));
        }
      }
    }
    uint32_t k = (uint32_t)std::max<uint64_t>(1, wave_paths / c.P);
    k = std::min<uint32_t>(k, f->spp);
    {
      // hit-record slack: k records per pixel slot only when some batch runs bounce 0 pixel-major
      FrameView probe = frame_view(c, *f);
      probe.k = k;
      bool pm = bounce0_pixel_major(scene_view(c), probe) != 0u;
      if (f->spp % k) {  // the call's last, partial batch
        probe.k = f->spp % k;
        pm = pm || bounce0_pixel_major(scene_view(c), probe) != 0u;
      }
      // hit-record segments hold twice the static shares when k_trace_dyn takes its rays from the per-XCD queues
      rc = ensure_wave(c, (uint64_t)k * c.P, (uint32_t)shading(c).lights_host.size(), task_stride(c), pm ? k : 1u,
                       hrec_mult(scene_view(c)));
      if (rc != SPTR_OK) return rc;
    }
    const int T = std::max(1, (int)(c.tail_depth ? c.tail_depth : auto_tail_depth((uint64_t)k * c.P, scene_view(c))));
    key.epoch = c.epoch;  // ensure_wave may have reallocated
    key.k = k;
    key.tail = (uint32_t)T;
    if (c.pending == 0) API_HIP(hipMemsetAsync(c.w_tot.p, 0, kTotWords * 8, s));
    rc = refresh_cull(c, *f, s, timing || trace_timing);
    if (rc != SPTR_OK) return rc;
    // an in-sequence cull (SPTR_FRAME_RECULL) counts its unculled pixels from zero: k_frame_dyn clears it
    uint32_t* clear = ((f->flags & SPTR_FRAME_RECULL) && !(f->flags & SPTR_FRAME_NO_CULL))
                          ? static_cast<uint32_t*>(c.plist.p) + c.P : nullptr;
    rc = run_call(c, key, f->frame_begin, reset ? 1u : 0u, total, (uint64_t)frame_view(c, *f).valid * f->spp, clear,
                  timing || trace_timing, !timing, s,
                  [&](hipStream_t cs, StageTimer& tm) { return enqueue_wavefront(c, *f, k, T, cs, tm); }, waves);
    if (rc != SPTR_OK) return rc;
    if (clear) {  // the sequence just enqueued computes this camera's mask (keyed only once enqueued)
      c.cull_epoch = c.epoch;
      c.cull_cam = f->camera;
      c.cull_depth = cull_depth_for(f->spp);
      ++c.pending_culls;
    }
    samples = (uint64_t)frame_view(c, *f).valid * f->spp;
  }
  c.last_samples = total;
  ++c.pending;
  c.pending_stream = s;
  c.pending_samples += samples;
  c.pending_waves += waves;
  if (f->flags & SPTR_FRAME_ASYNC) {
    if (stats) std::memset(stats, 0, sizeof(*stats));
    return SPTR_OK;
  }
  return collect_pending(c, stats);
}

const char* sptr_capture_error(const sptr_ctx* x) { return x ? x->c.capture_error.c_str() : "null context"; }

int sptr_graph_info(const sptr_ctx* x, uint32_t* valid, uint32_t* nodes, uint32_t* edges, uint32_t* depth,
                    uint32_t* captures, int32_t* capture_status) {
  if (!x) return SPTR_ERR_INVALID;
  const GraphCache& g = x->c.graph;
  if (captures) *captures = x->c.captures;
  if (capture_status) *capture_status = x->c.capture_status;
  if (valid) *valid = g.valid ? 1u : 0u;
  if (nodes) *nodes = g.valid ? g.nodes : 0u;
  if (edges) *edges = g.valid ? g.edges : 0u;
  if (depth) *depth = g.valid ? g.depth : 0u;
  return SPTR_OK;
}

int sptr_overlap_probe(sptr_ctx* x, double* ms) {
  if (!x || !ms) return SPTR_ERR_INVALID;
  Context& c = x->c;
  API_HIP(hipSetDevice(c.device));
  if (sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;
  int rate_khz = 0;
  API_HIP(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, c.device));
  if (rate_khz <= 0) return fail(c, SPTR_ERR_HIP, "overlap probe: no wall clock rate");
  const uint64_t ticks = (uint64_t)rate_khz / 5u;  // 200 us per spin
  // the events are destroyed on every exit path (Probe's destructor)
  struct Probe {
    hipEvent_t e0 = nullptr, e1 = nullptr, fk = nullptr, jn = nullptr;
    ~Probe() {
      for (hipEvent_t e : {e0, e1, fk, jn})
        if (e) (void)hipEventDestroy(e);
    }
  } pe;
  hipError_t err = hipSuccess;
  auto ck = [&](hipError_t e) {
    if (e != hipSuccess && err == hipSuccess) err = e;
  };
  ck(hipEventCreate(&pe.e0));
  ck(hipEventCreate(&pe.e1));
  ck(hipEventCreateWithFlags(&pe.fk, hipEventDisableTiming));
  ck(hipEventCreateWithFlags(&pe.jn, hipEventDisableTiming));
  if (err != hipSuccess) return fail(c, SPTR_ERR_HIP, std::string("overlap probe: ") + hipGetErrorString(err));
  hipEvent_t e0 = pe.e0, e1 = pe.e1, fk = pe.fk, jn = pe.jn;
  const hipStream_t s = c.stream;
  launch_spin(ticks / 8u, s);  // warm the kernel
  ck(hipStreamSynchronize(s));
  const hipStream_t sides[3] = {nullptr, c.side_stream, c.side2_stream};
  for (int i = 0; i < 3; ++i) {
    const hipStream_t side = sides[i] ? sides[i] : s;
    ck(hipEventRecord(e0, s));
    if (side != s) {
      ck(hipEventRecord(fk, s));
      ck(hipStreamWaitEvent(side, fk, 0));
    }
    launch_spin(ticks, s);
    launch_spin(ticks, side);
    if (side != s) {
      ck(hipEventRecord(jn, side));
      ck(hipStreamWaitEvent(s, jn, 0));
    }
    ck(hipEventRecord(e1, s));
    ck(hipStreamSynchronize(s));
    float t = 0.0f;
    ck(hipEventElapsedTime(&t, e0, e1));
    ms[i] = t;
  }
  if (err != hipSuccess) return fail(c, SPTR_ERR_HIP, std::string("overlap probe: ") + hipGetErrorString(err));
  return SPTR_OK;
}

static int set_launch_mode_one(sptr_ctx* x, uint32_t mode) {
  if (!x) return SPTR_ERR_INVALID;
  if (mode > 3)
    return fail(x->c, SPTR_ERR_INVALID,
                "launch mode must be 0 (graphs where they pay), 1 (direct), 2 (direct, one stream) or 3 (graphs)");
  x->c.launch_mode = mode;
  return SPTR_OK;
}

int sptr_collect_stats(sptr_ctx* x, sptr_stats* stats) {
  if (!x) return SPTR_ERR_INVALID;
  Context& c = x->c;
  API_HIP(hipSetDevice(c.device));
  if (!x->lane || x->lane->c.pending == 0) return collect_pending(c, stats);
  Context* both[2] = {&c, &x->lane->c};
  const double busy = stats ? trace_busy_ms(both, 2) : 0.0;
  sptr_stats a{}, b{};
  int rc = collect_pending(c, &a);
  if (rc != SPTR_OK) return rc;
  rc = collect_pending(x->lane->c, &b);
  if (rc != SPTR_OK) return fail(c, rc, std::string("pixel lane: ") + x->lane->c.err);
  add_stats(a, b);
  a.ms_trace_busy = busy;
  if (stats) *stats = a;
  return SPTR_OK;
}

int sptr_read_rgb8(sptr_ctx* x, uint8_t* rgb) {
  if (!x || !rgb) return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;
  if (x->split && sync_pending(x->lane->c) != SPTR_OK) return SPTR_ERR_HIP;  // (it resolves into this image)
  if (!c.image.p) return fail(c, SPTR_ERR_NO_SCENE, "read_rgb8: nothing rendered");
  API_HIP(hipSetDevice(c.device));
  API_HIP(hipMemcpy(rgb, c.image.p, (size_t)c.W * c.H * 3, hipMemcpyDeviceToHost));
  return SPTR_OK;
}

int sptr_read_rgb8_lagged(sptr_ctx* x, uint8_t* rgb, uint32_t* got) {
  if (!x || !rgb || !got) return SPTR_ERR_INVALID;
  Context& c = x->c;
  *got = 0;
  if (!c.image.p || c.pending == 0)
    return fail(c, SPTR_ERR_INVALID, "read_rgb8_lagged: call after an asynchronous render (SPTR_FRAME_ASYNC)");
  API_HIP(hipSetDevice(c.device));
  if (!x->copy_stream) {
    // a priority of its own (the lowest): its own hardware queue, apart from the render stream's
    API_HIP(hipStreamCreateWithPriority(&x->copy_stream, hipStreamNonBlocking, c.prio_lo));
    API_HIP(hipEventCreateWithFlags(&x->copy_done, hipEventDisableTiming));
    for (auto& sn : x->snap) API_HIP(hipEventCreateWithFlags(&sn.ready, hipEventDisableTiming));
  }
  const size_t bytes = (size_t)c.W * c.H * 3;
  auto& cur = x->snap[x->snap_cur];
  auto& prev = x->snap[x->snap_cur ^ 1u];
  // this call's image, snapshotted on its stream after it (with two lanes, the lane's resolve into this
  // image is joined into that stream before the call's last launch).  The slot's last reader was the copy
  // two calls back, which that call waited for.
  API_HIP(ensure_buf(cur.buf, bytes));
  API_HIP(hipMemcpyAsync(cur.buf.p, c.image.p, bytes, hipMemcpyDeviceToDevice, c.pending_stream));
  API_HIP(hipEventRecord(cur.ready, c.pending_stream));
  if (prev.valid && prev.W == c.W && prev.H == c.H) {
    if (x->reg_ptr != rgb || x->reg_bytes != bytes) {  // page-lock the destination: the copy becomes a DMA
      if (x->reg_ptr) (void)hipHostUnregister(x->reg_ptr);
      x->reg_ptr = nullptr;
      x->reg_bytes = 0;
      if (hipHostRegister(rgb, bytes, hipHostRegisterDefault) == hipSuccess) {
        x->reg_ptr = rgb;
        x->reg_bytes = bytes;
      } else {
        (void)hipGetLastError();  // (a pageable destination works too, through staging)
      }
    }
    API_HIP(hipStreamWaitEvent(x->copy_stream, prev.ready, 0));
    API_HIP(hipMemcpyAsync(rgb, prev.buf.p, bytes, hipMemcpyDeviceToHost, x->copy_stream));
    API_HIP(hipEventRecord(x->copy_done, x->copy_stream));
    API_HIP(hipEventSynchronize(x->copy_done));
    *got = 1;
  }
  cur.valid = true;
  cur.W = c.W;
  cur.H = c.H;
  x->snap_cur ^= 1u;
  return SPTR_OK;
}

int sptr_read_accum(sptr_ctx* x, float* out) {
  if (!x || !out) return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;
  if (!c.accum.p) return fail(c, SPTR_ERR_NO_SCENE, "read_accum: nothing rendered");
  API_HIP(hipSetDevice(c.device));
  std::vector<float> a((size_t)c.P * 4);
  API_HIP(hipMemcpy(a.data(), c.accum.p, a.size() * 4, hipMemcpyDeviceToHost));
  std::memset(out, 0, (size_t)c.W * c.H * 3 * 4);
  auto scatter = [&](const Context& cc, const std::vector<float>& acc) {
    for (uint32_t l = 0; l < cc.P; ++l) {
      int px, py;
      if (!host_local_pixel(cc, l, px, py)) continue;
      float* o = out + ((size_t)py * cc.W + px) * 3;
      o[0] = acc[(size_t)l * 4 + 0];
      o[1] = acc[(size_t)l * 4 + 1];
      o[2] = acc[(size_t)l * 4 + 2];
    }
  };
  scatter(c, a);
  if (x->split) {  // the odd half of the tiles, from the lane
    Context& cy = x->lane->c;
    if (sync_pending(cy) != SPTR_OK) return SPTR_ERR_HIP;
    std::vector<float> b((size_t)cy.P * 4);
    API_HIP(hipMemcpy(b.data(), cy.accum.p, b.size() * 4, hipMemcpyDeviceToHost));
    scatter(cy, b);
  }
  return SPTR_OK;
}

int sptr_tiles_device(sptr_ctx* x, void** dptr, size_t* bytes) {
  if (!x || !dptr || !bytes) return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (!c.tiles.p) return fail(c, SPTR_ERR_NO_SCENE, "tiles_device: nothing rendered");
  if (x->split) {  // the two lanes' tiles, interleaved into this context's shard order by sptr_render
    *dptr = x->tiles_full.p;
    *bytes = (size_t)x->full_tiles * kTilePixels * 4;
    return SPTR_OK;
  }
  *dptr = c.tiles.p;
  *bytes = (size_t)c.P * 4;
  return SPTR_OK;
}

int sptr_unpack_tiles(sptr_ctx* x, const void* gathered, int32_t G, uint32_t tpr, int32_t W, int32_t H, void* out,
                      void* stream) {
  if (!x || !gathered || !out || G <= 0 || W <= 0 || H <= 0) return SPTR_ERR_INVALID;
  Context& c = x->c;
  API_HIP(hipSetDevice(c.device));
  const int ntiles = ((W + kTile - 1) / kTile) * ((H + kTile - 1) / kTile);
  if ((uint64_t)tpr * (uint64_t)G < (uint64_t)ntiles) return fail(c, SPTR_ERR_INVALID, "unpack: tiles_per_rank too small");
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c.stream;
  launch_unpack(static_cast<const uint32_t*>(gathered), G, tpr, W, H, static_cast<uint8_t*>(out), s);
  API_HIP(hipGetLastError());
  if (!stream) API_HIP(hipStreamSynchronize(s));  // on a caller's stream the call only enqueues
  return SPTR_OK;
}

static int run_query(sptr_ctx* x, const float* rays, uint32_t n, bool anyhit, uint32_t* geom, uint32_t* prim, float* t,
                     float* ng, uint8_t* occ) {
  if (!x || (n && !rays)) return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (!c.have_scene) return fail(c, SPTR_ERR_NO_SCENE, "query: no scene");
  if (sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;
  if (n == 0) return SPTR_OK;
  API_HIP(hipSetDevice(c.device));
  const size_t rb = (size_t)n * 32, refb = (size_t)n * 4, tb = (size_t)n * 4, nb = (size_t)n * 12, ob = (size_t)n;
  API_HIP(ensure_buf(c.qbuf, rb + refb + tb + nb + ob + 64));
  char* base = static_cast<char*>(c.qbuf.p);
  uint32_t* d_sflag = reinterpret_cast<uint32_t*>(base + (rb + refb + tb + nb + ob + 15) / 16 * 16);
  float* d_rays = reinterpret_cast<float*>(base);
  uint32_t* d_ref = reinterpret_cast<uint32_t*>(base + rb);
  float* d_t = reinterpret_cast<float*>(base + rb + refb);
  float* d_ng = reinterpret_cast<float*>(base + rb + refb + tb);
  uint8_t* d_occ = reinterpret_cast<uint8_t*>(base + rb + refb + tb + nb);
  API_HIP(hipMemcpy(d_rays, rays, rb, hipMemcpyHostToDevice));
  API_HIP(hipMemset(d_sflag, 0, 4));
  launch_query(scene_view(c), static_cast<const uint32_t*>(c.tri_orig.p), static_cast<const uint32_t*>(c.sph_orig.p),
               d_rays, n, anyhit, d_ref, d_t, d_ng, d_occ, d_sflag, c.stream);
  API_HIP(hipGetLastError());
  API_HIP(hipStreamSynchronize(c.stream));
  uint32_t sflag = 0;
  API_HIP(hipMemcpy(&sflag, d_sflag, 4, hipMemcpyDeviceToHost));
  if (sflag) return fail(c, SPTR_ERR_HIP, "query: BVH traversal stack overflow (internal error)");
  if (anyhit) {
    API_HIP(hipMemcpy(occ, d_occ, ob, hipMemcpyDeviceToHost));
    return SPTR_OK;
  }
  std::vector<uint32_t> ref(n);
  API_HIP(hipMemcpy(ref.data(), d_ref, refb, hipMemcpyDeviceToHost));
  API_HIP(hipMemcpy(t, d_t, tb, hipMemcpyDeviceToHost));
  API_HIP(hipMemcpy(ng, d_ng, nb, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t r = ref[i];
    if (r == kNoHit) {
      geom[i] = prim[i] = 0xFFFFFFFFu;
    } else if (r & kSphereBit) {
      geom[i] = c.num_tri_geoms + (r & kIndexMask);
      prim[i] = 0;
    } else {
      const uint32_t tri = r & kIndexMask;
      const auto it = std::upper_bound(c.geom_first.begin(), c.geom_first.end(), tri);
      const uint32_t g = (uint32_t)(it - c.geom_first.begin()) - 1u;
      geom[i] = g;
      prim[i] = tri - c.geom_first[g];
    }
  }
  return SPTR_OK;
}

int sptr_intersect(sptr_ctx* x, const float* rays, uint32_t n, uint32_t* geom, uint32_t* prim, float* t, float* ng) {
  if (!geom || !prim || !t || !ng) return SPTR_ERR_INVALID;
  return run_query(x, rays, n, false, geom, prim, t, ng, nullptr);
}

int sptr_occluded(sptr_ctx* x, const float* rays, uint32_t n, uint8_t* occ) {
  if (!occ) return SPTR_ERR_INVALID;
  return run_query(x, rays, n, true, nullptr, nullptr, nullptr, nullptr, occ);
}

int sptr_primary_rays(sptr_ctx* x, const sptr_camera* cam, int32_t W, int32_t H, uint32_t acc, float* dirs,
                      uint32_t* rng) {
  if (!x || !cam || W <= 0 || H <= 0 || !dirs || !rng) return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;
  API_HIP(hipSetDevice(c.device));
  sptr_frame f{};
  f.width = W;
  f.height = H;
  f.camera = *cam;
  f.frame_begin = acc;
  f.max_depth = 1;
  FrameView fv = frame_view(c, f);
  const size_t n = (size_t)W * H;
  API_HIP(ensure_buf(c.qbuf, n * 16 + 64));
  float* d_dirs = static_cast<float*>(c.qbuf.p);
  uint32_t* d_rng = reinterpret_cast<uint32_t*>(static_cast<char*>(c.qbuf.p) + n * 12);
  launch_primary(fv, d_dirs, d_rng, c.stream);
  API_HIP(hipGetLastError());
  API_HIP(hipStreamSynchronize(c.stream));
  API_HIP(hipMemcpy(dirs, d_dirs, n * 12, hipMemcpyDeviceToHost));
  API_HIP(hipMemcpy(rng, d_rng, n * 4, hipMemcpyDeviceToHost));
  return SPTR_OK;
}

// scratch of the primitive tests: freed on every exit path
struct DevScratch {
  std::vector<void*> p;
  ~DevScratch() {
    for (void* q : p) (void)hipFree(q);
  }
  hipError_t alloc(void** q, size_t bytes) {
    *q = nullptr;
    const hipError_t e = hipMalloc(q, bytes ? bytes : 16);
    if (e == hipSuccess) p.push_back(*q);
    return e;
  }
};

int sptr_sort_pairs_u64(sptr_ctx* x, const uint64_t* keys, const uint32_t* vals, uint32_t n, uint64_t* keys_out,
                        uint32_t* vals_out) {
  if (!x || (n && (!keys || !vals || !keys_out || !vals_out))) return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;
  API_HIP(hipSetDevice(c.device));
  DevScratch d;
  void *ki = nullptr, *ko = nullptr, *vi = nullptr, *vo = nullptr, *tmp = nullptr;
  size_t tb = 0;
  API_HIP(radix_sort_pairs_u64(nullptr, tb, nullptr, nullptr, nullptr, nullptr, n, c.stream));
  API_HIP(d.alloc(&ki, (size_t)n * 8));
  API_HIP(d.alloc(&ko, (size_t)n * 8));
  API_HIP(d.alloc(&vi, (size_t)n * 4));
  API_HIP(d.alloc(&vo, (size_t)n * 4));
  API_HIP(d.alloc(&tmp, tb));
  if (n) {
    API_HIP(hipMemcpy(ki, keys, (size_t)n * 8, hipMemcpyHostToDevice));
    API_HIP(hipMemcpy(vi, vals, (size_t)n * 4, hipMemcpyHostToDevice));
  }
  API_HIP(radix_sort_pairs_u64(tmp, tb, static_cast<const uint64_t*>(ki), static_cast<uint64_t*>(ko),
                               static_cast<const uint32_t*>(vi), static_cast<uint32_t*>(vo), n, c.stream));
  API_HIP(hipStreamSynchronize(c.stream));
  if (n) {
    API_HIP(hipMemcpy(keys_out, ko, (size_t)n * 8, hipMemcpyDeviceToHost));
    API_HIP(hipMemcpy(vals_out, vo, (size_t)n * 4, hipMemcpyDeviceToHost));
  }
  return SPTR_OK;
}

int sptr_eval_math(sptr_ctx* x, int fn, const float* in, uint32_t n, float* out) {
  if (!x || !out || (fn != SPTR_MATH_COSINE_SINCOS && fn != SPTR_MATH_GAMMA) || (fn == SPTR_MATH_GAMMA && n && !in))
    return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;
  API_HIP(hipSetDevice(c.device));
  const uint32_t m = fn == SPTR_MATH_COSINE_SINCOS ? (1u << 24) : n;
  const size_t out_n = fn == SPTR_MATH_COSINE_SINCOS ? 2u * (size_t)m : (size_t)m;
  DevScratch d;
  void *di = nullptr, *dout = nullptr;
  API_HIP(d.alloc(&di, fn == SPTR_MATH_GAMMA ? (size_t)n * 4 : 16));
  API_HIP(d.alloc(&dout, out_n * 4));
  if (fn == SPTR_MATH_GAMMA && n) API_HIP(hipMemcpy(di, in, (size_t)n * 4, hipMemcpyHostToDevice));
  if (m) launch_eval_math(fn, static_cast<const float*>(di), m, static_cast<float*>(dout), c.stream);
  API_HIP(hipGetLastError());
  API_HIP(hipStreamSynchronize(c.stream));
  if (out_n) API_HIP(hipMemcpy(out, dout, out_n * 4, hipMemcpyDeviceToHost));
  return SPTR_OK;
}

int sptr_scan_u32(sptr_ctx* x, const uint32_t* in, uint32_t n, uint32_t* out) {
  if (!x || (n && (!in || !out))) return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (sync_pending(c) != SPTR_OK) return SPTR_ERR_HIP;
  API_HIP(hipSetDevice(c.device));
  DevScratch d;
  void *di = nullptr, *dout = nullptr, *tmp = nullptr;
  size_t tb = 0;
  API_HIP(scan_u32(nullptr, tb, nullptr, nullptr, n, c.stream));
  API_HIP(d.alloc(&di, (size_t)n * 4));
  API_HIP(d.alloc(&dout, (size_t)n * 4));
  API_HIP(d.alloc(&tmp, tb));
  if (n) API_HIP(hipMemcpy(di, in, (size_t)n * 4, hipMemcpyHostToDevice));
  API_HIP(scan_u32(tmp, tb, static_cast<const uint32_t*>(di), static_cast<uint32_t*>(dout), n, c.stream));
  API_HIP(hipStreamSynchronize(c.stream));
  if (n) API_HIP(hipMemcpy(out, dout, (size_t)n * 4, hipMemcpyDeviceToHost));
  return SPTR_OK;
}


// ---- pixel lanes -------------------------------------------------------------------------------
// A setter applied to the lane context too: its failure is reported through this context's error text.
static int lane_forward(sptr_ctx* x, int rc_lane) {
  if (!x || !x->lane || rc_lane == SPTR_OK) return SPTR_OK;
  return fail(x->c, rc_lane, std::string("pixel lane: ") + x->lane->c.err);
}

int sptr_upload_scene(sptr_ctx* x, const sptr_scene* s) {
  const int rc = upload_scene_one(x, s);
  if (rc != SPTR_OK) return rc;
  if (x->split) x->c.W = 0;  // the pixel buffers describe the even lane: re-laid out for the next call
  x->split = false;
  x->lane_scene = false;
  // the lane gets a copy only of scenes staged into LDS (small by construction): the two chains of a
  // larger scene traversed from L2/HBM compete for the same memory latency (r05zs: C5 8.0 -> 7.6-7.7 ms,
  // but a second copy of a 10M-triangle scene), and C3's VALU-bound sky gains nothing (3.55-3.63 -> 3.65)
  if (x->lane && scene_view(x->c).lds_bytes != 0) {
    Context& cy = x->lane->c;
    // (a priority of its own puts the lane's stream on a hardware queue apart from the render stream's:
    // created at the default priority it shared that queue and the two chains ran one after the other,
    // r05zx, C2 3.24 ms; at the lowest priority, the side streams', 2.56-2.58; at the highest 2.67-2.69)
    if (!cy.stream && hipStreamCreateWithPriority(&cy.stream, hipStreamNonBlocking, x->c.prio_lo) != hipSuccess) {
      cy.stream = nullptr;
      return fail(x->c, SPTR_ERR_HIP, "pixel lane: stream creation failed");
    }
    const int r1 = upload_scene_one(x->lane, s);
    if (r1 != SPTR_OK) return lane_forward(x, r1);
    x->lane_scene = true;
  }
  return SPTR_OK;
}

int sptr_set_pixel_lanes(sptr_ctx* x, uint32_t lanes) {
  if (!x) return SPTR_ERR_INVALID;
  if (lanes > 2u) return fail(x->c, SPTR_ERR_INVALID, "pixel lanes: 0 (automatic), 1 or 2");
  if (x->is_lane) return fail(x->c, SPTR_ERR_INVALID, "pixel lanes: not on a lane context");
  if (lanes == 2u && !x->lane) return fail(x->c, SPTR_ERR_INVALID, "pixel lanes: no lane context");
  if (sync_pending(x->c) != SPTR_OK) return SPTR_ERR_HIP;
  if (x->lane && sync_pending(x->lane->c) != SPTR_OK) return SPTR_ERR_HIP;
  x->lanes_req = lanes;
  if (x->split) x->c.W = 0;  // (as in sptr_upload_scene)
  x->split = false;  // the next call starts an accumulation of its own (frame_begin 1)
  x->c.last_samples = 0;
  return SPTR_OK;
}

int sptr_pixel_lanes_info(const sptr_ctx* x, uint32_t* requested, uint32_t* active) {
  if (!x) return SPTR_ERR_INVALID;
  if (requested) *requested = x->lanes_req;
  if (active) *active = x->split ? 1u : 0u;
  return SPTR_OK;
}

// Two lanes for this call: an accumulation continues in the mode it started in; a new one (frame_begin 1)
// runs in two lanes when the scene is staged into LDS, the integrator is the wavefront one and the call
// is large (>= 2^24 samples: r05zs, two contexts on one GPU, C2 3.0 -> 2.47 ms, C4 158.5 -> 137.5 ms, the
// 8-way C2 shard 0.49-0.51 -> 0.46 ms; 1-spp frames keep one chain), or when asked for (lanes_req 2).
static bool lanes_for(const sptr_ctx* x, const sptr_frame* f) {
  if (!x->lane || !x->lane_scene || x->lanes_req == 1u || f->integrator != SPTR_INTEGRATOR_WAVEFRONT) return false;
  const int G = f->shard_count > 0 ? f->shard_count : 1, R = f->shard_count > 0 ? f->shard_rank : 0;
  const int ntiles = ((f->width + kTile - 1) / kTile) * ((f->height + kTile - 1) / kTile);
  if (R < 0 || R >= G || R + G >= ntiles) return false;  // the second lane would hold no tile
  if (f->frame_begin != 1) return x->split;
  if (x->lanes_req == 2u) return true;
  const uint64_t px = (uint64_t)shard_tiles(f->width, f->height, G, R) * kTilePixels;
  return px * f->spp >= (1ull << 24);
}

static void add_stats(sptr_stats& a, const sptr_stats& b) {
  // the counters add, and so do the stage times (sums of launch durations); the call spans overlap
  const double total = std::max(a.ms_total, b.ms_total);
  a.rays_closest += b.rays_closest;
  a.rays_shadow += b.rays_shadow;
  a.samples += b.samples;
  a.waves += b.waves;
  a.ms_raygen += b.ms_raygen;
  a.ms_trace += b.ms_trace;
  a.ms_shade += b.ms_shade;
  a.ms_shadow += b.ms_shadow;
  a.ms_accum += b.ms_accum;
  a.trace_launches += b.trace_launches;
  a.node_visits += b.node_visits;
  a.tri_tests += b.tri_tests;
  a.sphere_tests += b.sphere_tests;
  a.shadow_node_visits += b.shadow_node_visits;
  a.shadow_prim_tests += b.shadow_prim_tests;
  a.ms_trace0 += b.ms_trace0;
  a.ms_shade0 += b.ms_shade0;
  a.rays_tail += b.rays_tail;
  a.ms_tail += b.ms_tail;
  a.traced_primary += b.traced_primary;
  a.traced_bounce += b.traced_bounce;
  a.node_visits_primary += b.node_visits_primary;
  a.tri_tests_primary += b.tri_tests_primary;
  a.sphere_tests_primary += b.sphere_tests_primary;
  a.ms_cull += b.ms_cull;
  a.cull_launches += b.cull_launches;
  a.shadow_launches += b.shadow_launches;
  for (int i = 0; i < 8; ++i) {
    a.traced_by_depth[i] += b.traced_by_depth[i];
    a.nodes_by_depth[i] += b.nodes_by_depth[i];
  }
  for (int i = 0; i < 16; ++i) {
    a.trace_visit_hist[i] += b.trace_visit_hist[i];
    a.shadow_visit_hist[i] += b.shadow_visit_hist[i];
  }
  a.hits_primary += b.hits_primary;
  a.hits_bounce += b.hits_bounce;
  a.paths_handed_off += b.paths_handed_off;
  for (int i = 0; i < 3; ++i) a.strag_visits[i] += b.strag_visits[i];
  a.traced_fused += b.traced_fused;
  a.ms_total = total;
  a.ms_trace_busy = std::max(a.ms_trace_busy, b.ms_trace_busy);  // (the callers set the union)
}

int sptr_render(sptr_ctx* x, const sptr_frame* f, void* stream, sptr_stats* stats) {
  if (!x || !f) return SPTR_ERR_INVALID;
  Context& c = x->c;
  if (!lanes_for(x, f)) {
    if (x->split) {  // leaving a two-lane accumulation: this call must start a new one
      if (f->frame_begin != 1) return fail(c, SPTR_ERR_INVALID, "render: frame_begin must be 1 after a two-lane accumulation");
      if (sync_pending(x->lane->c) != SPTR_OK) return SPTR_ERR_HIP;
      x->split = false;
      c.W = 0;  // the pixel buffers describe the even lane: re-laid out for the whole shard
    }
    c.time_by_events = false;
    return render_one(x, f, stream, stats);
  }
  // two lanes: this context renders shard (R, 2G) — the even half of shard (R, G)'s tiles — and the
  // lane shard (R + G, 2G), the odd half, on its own stream, forked after everything enqueued on s so far
  // and joined back into s
  API_HIP(hipSetDevice(c.device));
  sptr_ctx* y = x->lane;
  Context& cy = y->c;
  const int G = f->shard_count > 0 ? f->shard_count : 1, R = f->shard_count > 0 ? f->shard_rank : 0;
  sptr_frame f0 = *f, f1 = *f;
  f0.shard_count = f1.shard_count = 2 * G;
  f0.shard_rank = R;
  f1.shard_rank = R + G;
  f0.flags |= SPTR_FRAME_ASYNC;
  f1.flags |= SPTR_FRAME_ASYNC;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : c.stream;
  const bool serial = c.launch_mode == 2u;  // one stream: the lanes one after the other
  hipStream_t sy = serial ? s : cy.stream;
  // both halves checked before either is enqueued (a change into or out of launch mode 2 between two
  // asynchronous calls moves the lane's half between its own stream and s: ADVICE r05)
  if ((c.pending && s != c.pending_stream) || (cy.pending && sy != cy.pending_stream))
    return fail(c, SPTR_ERR_INVALID, "render: asynchronous renders must stay on one stream until sptr_collect_stats");
  if (!x->split || c.W != f->width || c.H != f->height || x->full_G != G || x->full_R != R) {
    if (f->frame_begin != 1) return fail(c, SPTR_ERR_INVALID, "render: frame_begin must continue the accumulation (last + 1) or be 1");
    if (sync_pending(c) != SPTR_OK || sync_pending(cy) != SPTR_OK) return SPTR_ERR_HIP;
    x->full_G = G;
    x->full_R = R;
    x->full_tiles = shard_tiles(f->width, f->height, G, R);
    API_HIP(ensure_buf(x->tiles_full, (size_t)x->full_tiles * kTilePixels * 4));
    API_HIP(hipMemsetAsync(x->tiles_full.p, 0, (size_t)x->full_tiles * kTilePixels * 4, s));
  }
  x->split = true;
  c.time_by_events = cy.time_by_events = true;  // (LaunchTiming, sptr_internal.h)
  // this context's pixel buffers first (the image both lanes resolve into is cleared on s before the fork)
  bool resized = false;
  int rc = ensure_pixels(c, f->width, f->height, 2 * G, R, s, resized);
  if (rc != SPTR_OK) return rc;
  cy.image_out = static_cast<uint8_t*>(c.image.p);
  if (!serial) {
    API_HIP(hipEventRecord(x->lane_fork, s));
    API_HIP(hipStreamWaitEvent(sy, x->lane_fork, 0));
  }
  rc = render_one(x, &f0, s, nullptr);
  if (rc != SPTR_OK) return rc;
  rc = render_one(y, &f1, sy, nullptr);
  if (rc != SPTR_OK) return fail(c, rc, std::string("pixel lane: ") + cy.err);
  if (!serial) {
    API_HIP(hipEventRecord(x->lane_join, sy));
    API_HIP(hipStreamWaitEvent(s, x->lane_join, 0));
  }
  // this context's tiles (the multi-GPU gather's send buffer): the lanes' tiles interleaved
  launch_interleave_tiles(static_cast<const uint32_t*>(c.tiles.p), c.local_tiles, static_cast<const uint32_t*>(cy.tiles.p),
                          cy.local_tiles, static_cast<uint32_t*>(x->tiles_full.p), x->full_tiles, s);
  API_HIP(hipGetLastError());
  if (f->flags & SPTR_FRAME_ASYNC) {
    if (stats) std::memset(stats, 0, sizeof(*stats));
    return SPTR_OK;
  }
  Context* both[2] = {&c, &cy};
  const double busy = stats ? trace_busy_ms(both, 2) : 0.0;
  sptr_stats a{}, b{};
  rc = collect_pending(c, &a);
  if (rc != SPTR_OK) return rc;
  rc = collect_pending(cy, &b);
  if (rc != SPTR_OK) return fail(c, rc, std::string("pixel lane: ") + cy.err);
  add_stats(a, b);
  a.ms_trace_busy = busy;
  if (stats) *stats = a;
  return SPTR_OK;
}

// The shading setters change only this context: a pixel lane reads its parent's shading state
// (shading()).  A lane render still pending reads the parent's device buffers, so the setters that
// replace them wait for it first; every shading change drops the lane's captured graph (epoch).
static int lane_shading_sync(sptr_ctx* x) {
  if (!x || !x->lane || x->lane->c.pending == 0) return SPTR_OK;
  if (sync_pending(x->lane->c) != SPTR_OK) return fail(x->c, SPTR_ERR_HIP, std::string("pixel lane: ") + x->lane->c.err);
  return SPTR_OK;
}
static int lane_shading_changed(sptr_ctx* x, int rc) {
  if (x && x->lane) ++x->lane->c.epoch;
  return rc;
}

int sptr_set_debug_mode(sptr_ctx* x, int mode) { return lane_shading_changed(x, set_debug_mode_one(x, mode)); }

int sptr_set_leaf_size(sptr_ctx* x, uint32_t n) {
  const int rc = set_leaf_size_one(x, n);
  return rc == SPTR_OK ? lane_forward(x, set_leaf_size_one(x ? x->lane : nullptr, n)) : rc;
}

int sptr_set_bvh_width(sptr_ctx* x, uint32_t width) {
  const int rc = set_bvh_width_one(x, width);
  return rc == SPTR_OK ? lane_forward(x, set_bvh_width_one(x ? x->lane : nullptr, width)) : rc;
}

int sptr_set_tail_depth(sptr_ctx* x, uint32_t depth) {
  const int rc = set_tail_depth_one(x, depth);
  return rc == SPTR_OK ? lane_forward(x, set_tail_depth_one(x ? x->lane : nullptr, depth)) : rc;
}

int sptr_set_split_refs(sptr_ctx* x, uint32_t max_pieces) {
  const int rc = set_split_refs_one(x, max_pieces);
  return rc == SPTR_OK ? lane_forward(x, set_split_refs_one(x ? x->lane : nullptr, max_pieces)) : rc;
}

int sptr_set_stragglers(sptr_ctx* x, uint32_t lanes) {
  const int rc = set_stragglers_one(x, lanes);
  return rc == SPTR_OK ? lane_forward(x, set_stragglers_one(x ? x->lane : nullptr, lanes)) : rc;
}

int sptr_set_wave_paths(sptr_ctx* x, uint64_t max_paths) {
  const int rc = set_wave_paths_one(x, max_paths);
  return rc == SPTR_OK ? lane_forward(x, set_wave_paths_one(x ? x->lane : nullptr, max_paths)) : rc;
}

int sptr_set_materials(sptr_ctx* x, const sptr_material* m, uint32_t n) {
  const int rs = lane_shading_sync(x);
  if (rs != SPTR_OK) return rs;
  return lane_shading_changed(x, set_materials_one(x, m, n));
}

int sptr_set_lights(sptr_ctx* x, const sptr_light* l, uint32_t n) {
  return lane_shading_changed(x, set_lights_one(x, l, n));  // (by value in every launch's arguments)
}

int sptr_set_environment(sptr_ctx* x, const sptr_environment* e) {
  const int rs = lane_shading_sync(x);
  if (rs != SPTR_OK) return rs;
  return lane_shading_changed(x, set_environment_one(x, e));
}

int sptr_set_launch_mode(sptr_ctx* x, uint32_t mode) {
  const int rc = set_launch_mode_one(x, mode);
  return rc == SPTR_OK ? lane_forward(x, set_launch_mode_one(x->lane, mode)) : rc;
}

}  // extern "C"
