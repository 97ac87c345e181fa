/* sptr_hip.h — C ABI of libsptr_hip.so, the MI355X (gfx950) wavefront path-tracing backend.
 *
 * Drop-in boundary: these entry points are what a binding for the reference's GPU backend slot
 * needs.  The reference has no abstract backend interface; GLRenderer::renderLoop drives the
 * concrete OptixBackend class (/root/reference/src/GLRenderer.cpp:116-176) through the surface in
 * /root/reference/include/backends/OptixBackend.h:39-71.  Mapping (each entry cites what it replaces):
 *
 *   sptr_create / sptr_destroy   <- OptixBackend::OptixBackend / destroy()        (OptixBackend.h:41-66)
 *   sptr_upload_scene            <- OptixBackend::build(const SceneDesc&)         (OptixBackend.h:46;
 *                                   GAS/IAS builds at src/backends/OptixBackend.cpp:916-1308), fed the
 *                                   world-space flattening of EmbreeBackend::build
 *                                   (src/backends/EmbreeBackend.cpp:18-193) so geomIDs match the CPU path
 *   sptr_set_materials           <- OptixBackend::setMaterialManager              (OptixBackend.h:59)
 *   sptr_set_lights              <- OptixBackend::setLightManager                 (OptixBackend.h:63)
 *   sptr_set_environment         <- OptixBackend::setEnvironment                  (OptixBackend.h:55)
 *   sptr_render + sptr_read_rgb8 <- OptixBackend::render(uint8_t* rgb,w,h,Camera) (OptixBackend.h:51;
 *                                   src/backends/OptixBackend.cpp:1506-1850)
 *   sptr_set_debug_mode          <- OptixBackend::setDebugMode                    (OptixBackend.h:71)
 *
 * Semantics are those of the CPU Embree wavefront integrator (src/wavefront/wf_pt_cpu.cpp:61-255
 * driven by src/GLRenderer.cpp:353-435), not of the OptiX device programs.
 *
 * Conventions: 0 = OK, negative = error (sptr_last_error has the text); no exceptions, no exit()
 * across the ABI.  The caller owns every host buffer; upload calls copy.  One context per GPU, used
 * from one host thread at a time; contexts are independent.  Device pointers handed out stay valid
 * until the next render call with a different size, or sptr_destroy.
 */
#ifndef SPTR_HIP_H
#define SPTR_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPTR_ABI_VERSION 9

enum sptr_status {
  SPTR_OK = 0,
  SPTR_ERR_INVALID = -1,   /* bad argument / shape */
  SPTR_ERR_HIP = -2,       /* HIP runtime error */
  SPTR_ERR_NO_SCENE = -3,  /* render before upload / materials */
  SPTR_ERR_OOM = -4,
  SPTR_ERR_NO_DEVICE = -5
};

typedef struct sptr_ctx sptr_ctx;

/* World-space flattened scene, geomID order of EmbreeBackend::build: one triangle geometry per
 * SceneDesc instance (geomIDs 0..num_tri_geoms-1), then one geometry per analytic sphere. */
typedef struct sptr_scene {
  const float* positions; /* 3 floats per vertex, world space */
  uint32_t num_verts;
  const uint32_t* indices; /* 3 global vertex indices per triangle */
  uint32_t num_tris;
  const uint32_t* tri_geom_first; /* num_tri_geoms+1 prefix offsets into the triangle list */
  uint32_t num_tri_geoms;
  const float* spheres; /* cx, cy, cz, radius per sphere */
  uint32_t num_spheres;
  const uint32_t* geom_material; /* geomID -> material index (EmbreeBackend::geomMaterialId_) */
} sptr_scene;

/* One entry of MaterialManager's table (include/Material.h:19-39, values after the ctor clamps). */
typedef struct sptr_material {
  float albedo[3];
  float metallic;
  float roughness;
  float emission[3];
  float ior;
  int32_t type; /* 0 PBR, 1 DIELECTRIC (informational; shading follows metallic/ior) */
  float pad[2];
} sptr_material;

/* LightManager entry (include/Light.h:43-81): type 0 = directional (v = direction of the light's
 * rays, as passed to addDirectionalLight), 1 = point (v = position). */
typedef struct sptr_light {
  int32_t type;
  float v[3];
  float color[3];
  float intensity;
} sptr_light;

/* EnvironmentManager state: faces == NULL selects the procedural sky
 * (src/EnvironmentManager.cpp:35-61); otherwise 6 cube faces (+X,-X,+Y,-Y,+Z,-Z) of size*size RGB
 * floats, sampled bilinearly as Cubemap::sample (src/Cubemap.cpp:82-180). */
typedef struct sptr_environment {
  const float* faces;
  int32_t size;
  float intensity; /* 0.8 in the reference (EnvironmentManager.h:12) */
  float max_clamp; /* 5.0 */
} sptr_environment;

/* Camera basis as Camera::updateCameraVectors leaves it (src/Camera.cpp:33-50). */
typedef struct sptr_camera {
  float pos[3];
  float forward[3];
  float right[3];
  float up[3];
  float half_width;
  float half_height;
} sptr_camera;

enum sptr_frame_flags {
  SPTR_FRAME_TIMING = 1u,     /* per-stage times (adds sync at the end of the call).  The trace, fused-bounce
                                 and shadow launches time themselves (one launch chain's trace launches on
                                 the device wall clock, up to 4096 per collection window — later ones in
                                 the window go untimed; the shadow launches and the pixel lanes' launches
                                 by their dispatch events); the other stages by HIP events around them */
  SPTR_FRAME_NO_RESOLVE = 2u, /* skip the tonemap/resolve pass */
  SPTR_FRAME_COUNT_VISITS = 4u, /* one instrumented trace pass: count BVH node / primitive fetches */
  SPTR_FRAME_ASYNC = 8u, /* enqueue only: return without waiting; stats are left zero and the call's
                            counters and stage times accumulate until sptr_collect_stats */
  SPTR_FRAME_TIMING_TRACE = 16u, /* the trace and shadow launches' times only (ms_trace,
                                   ms_trace0, trace_launches, ms_shadow, shadow_launches): the other
                                   stages run back to back, and ms_total / ms_cull stay 0 */
  SPTR_FRAME_NO_CULL = 32u, /* diagnostic: bounce 0 traverses every camera ray, without the pixel-frustum
                               cull (the image is the same either way) */
  SPTR_FRAME_RECULL = 64u /* recompute the bounce-0 pixel-frustum cull mask in this call even when the
                             camera and scene are unchanged (the per-frame cost of a moving camera;
                             bench.py times its steps this way) */
};

/* Integrators (sptr_frame.integrator).  The reference selects between them per frame in
 * GLRenderer::renderLoop (src/GLRenderer.cpp:163-176):
 *   SPTR_INTEGRATOR_WAVEFRONT : WavefrontPathTracerCPU semantics (src/wavefront/wf_pt_cpu.cpp:61-255,
 *                               seeded and resolved by GLRenderer::renderWavefrontTileTask, :353-435):
 *                               one jittered sample per frame, deterministic wang-hash RNG, ACES +
 *                               gamma at resolve.  The default, and the parity / benchmark path.
 *   SPTR_INTEGRATOR_PATHTRACER: PathTracer semantics, the reference's default CPU integrator
 *                               (src/PathTracer.cpp:113-391): pixel-corner rays without jitter,
 *                               samples_per_frame recursive samples per frame averaged, ACES + gamma
 *                               per frame, tonemapped frames accumulated.  The reference draws from a
 *                               non-reproducible mt19937(random_device); this mode uses a
 *                               deterministic per-(pixel, frame, sample) wang-hash stream instead
 *                               (DESIGN.md), so it matches the reference in distribution only.
 *   SPTR_INTEGRATOR_OPTIX     : the shading of the reference's OptiX device programs
 *                               (src/optix/device_programs.cu:220-690, 854-899; the 'G' key's GPU
 *                               path): pixel-centre rays, wang_hash((pixel+1) ^ (frame*9781+1)) seeds,
 *                               tmin 1e-3, direct sun light without shadow rays, GGX-sampled metals,
 *                               delta dielectrics, depth-cap normal visualisation, exposure 2.2 +
 *                               Reinhard + gamma at resolve.  Exact functions replace CUDA's
 *                               approximate rsqrtf/sincosf. */
enum sptr_integrator { SPTR_INTEGRATOR_WAVEFRONT = 0, SPTR_INTEGRATOR_PATHTRACER = 1, SPTR_INTEGRATOR_OPTIX = 2 };

/* One render call = `spp` progressive frames starting at accumulation index frame_begin (1-based,
 * as GLRenderer::m_accumulated_samples; frame_begin == 1 clears the accumulation).  A wavefront
 * frame is one sample per pixel; a PathTracer frame is samples_per_frame samples (0 = 4, the
 * reference's setupPathTracer, src/main.cpp:105-113).  Pixels are rendered in 32x32 tiles
 * (GLRenderer.h:36); with shard_count > 1 only tiles t with t % shard_count == shard_rank are
 * rendered (interleaved multi-GPU sharding). */
typedef struct sptr_frame {
  int32_t width, height;
  sptr_camera camera;
  uint32_t frame_begin;
  uint32_t spp;
  uint32_t max_depth;
  int32_t shard_rank, shard_count;
  uint32_t flags;
  uint32_t integrator;        /* sptr_integrator */
  uint32_t samples_per_frame; /* PathTracer mode only */
} sptr_frame;

typedef struct sptr_stats {
  uint64_t rays_closest; /* closest-hit queries (primary + extension) = rtcIntersect1 calls */
  uint64_t rays_shadow;  /* any-hit queries = rtcOccluded1 calls */
  uint64_t samples;      /* pixel samples completed */
  uint64_t waves;        /* wavefront batches launched */
  double ms_total;       /* SPTR_FRAME_TIMING: wall time of the call on the device stream */
  double ms_raygen, ms_trace, ms_shade, ms_shadow, ms_accum; /* SPTR_FRAME_TIMING only; raygen is fused
                                                                into the bounce-0 trace (ms_raygen = 0);
                                                                ms_accum includes the culled pixels'
                                                                environment sums (k_sky) */
  uint64_t trace_launches;
  uint64_t node_visits, tri_tests, sphere_tests; /* SPTR_FRAME_COUNT_VISITS only */
  uint64_t shadow_node_visits, shadow_prim_tests;
  double ms_trace0, ms_shade0; /* SPTR_FRAME_TIMING: bounce-0 parts of ms_trace / ms_shade */
  uint64_t rays_tail;          /* closest-hit queries (of rays_closest) traced by the path-per-thread tail */
  double ms_tail;              /* SPTR_FRAME_TIMING: the tail launch */
  /* ABI 4: the rays the trace stage (ms_trace / trace_launches) actually traversed.  Camera rays of
   * frustum-culled pixels count as closest-hit queries (rays_closest) but never reach a traversal:
   * traced_primary = unculled pixel samples of bounce 0, traced_bounce = queued rays of bounces >= 1
   * traced by the wavefront trace kernels (not the fused bounce or path-per-thread tail kernels). */
  uint64_t traced_primary, traced_bounce;
  uint64_t node_visits_primary, tri_tests_primary, sphere_tests_primary; /* SPTR_FRAME_COUNT_VISITS: the
                                                                           bounce-0 part of node_visits,
                                                                           tri_tests, sphere_tests */
  double ms_cull;              /* SPTR_FRAME_TIMING: the pixel-cull launches (k_cull) */
  uint64_t cull_launches;      /* calls whose cull mask was (re)computed */
  uint64_t shadow_launches;    /* SPTR_FRAME_TIMING / _TIMING_TRACE: shadow-stage launches (ms_shadow) */
  /* Per bounce d (index 7: bounces >= 7): rays the wavefront trace kernels traversed (every call) and
   * their BVH node visits (SPTR_FRAME_COUNT_VISITS).  Histograms (SPTR_FRAME_COUNT_VISITS): closest-hit
   * rays of the trace kernels / any-hit queries of the shadow stage by node visits, bin b counting the
   * rays with 2^(b-1) <= visits < 2^b (bin 0: no visit, bin 15: >= 2^14). */
  uint64_t traced_by_depth[8];
  uint64_t nodes_by_depth[8];
  uint64_t trace_visit_hist[16];
  uint64_t shadow_visit_hist[16];
  uint64_t hits_primary, hits_bounce; /* SPTR_FRAME_COUNT_VISITS: closest hits the trace kernels found
                                         (of traced_primary / traced_bounce) */
  uint64_t paths_handed_off;          /* ABI 6: paths a bounce trace handed to the straggler kernel
                                         (sptr_set_stragglers) */
  uint64_t strag_visits[3];           /* ABI 6: node visits, triangle and sphere tests of the handed-off
                                         rays' walks made by the straggler kernel (every call) */
  double ms_trace_busy;               /* ABI 8, SPTR_FRAME_TIMING / _TIMING_TRACE: the trace launches'
                                         busy time, the union of their intervals (= ms_trace for one
                                         launch chain; two pixel lanes' trace launches overlap) */
  uint64_t traced_fused;              /* ABI 8: queued rays of bounces >= 1 traced by the fused bounce
                                         kernel (k_bounce: trace and shading of a bounce in one launch,
                                         LDS-staged scenes; every call).  Its launches count as trace
                                         launches (ms_trace, trace_launches, ms_trace_busy), and its rays
                                         are in traced_by_depth, not in traced_bounce */
} sptr_stats;

/* ---- context ---------------------------------------------------------------------------------- */
int sptr_abi_version(void);
int sptr_create(int device, sptr_ctx** out);
int sptr_destroy(sptr_ctx* ctx);
const char* sptr_last_error(const sptr_ctx* ctx);
int sptr_set_debug_mode(sptr_ctx* ctx, int mode);
/* Largest number of paths (pixels x samples) processed per wavefront batch (at most 2^30).
 * 0 = default: 2^29, capped by what half of the device's free memory holds (at least 2^24). */
int sptr_set_wave_paths(sptr_ctx* ctx, uint64_t max_paths);
/* First bounce traced path-per-thread (one launch carries every surviving path to its end; earlier
 * bounces run as trace/shade/shadow wavefront stages).  0 = automatic: scenes traversed from L2/HBM
 * 2 (L2-resident) or 3; LDS-staged scenes 4 for batches of at most 2^25 paths (e.g. the per-rank share
 * of a sharded 1080p frame), none for larger batches; >= max_depth = none.  The image and the query
 * counts do not depend on it. */
int sptr_set_tail_depth(sptr_ctx* ctx, uint32_t depth);
/* Maximum primitives per BVH leaf range (1..16; 0 = automatic, the default: 8 for scenes staged in
 * LDS, 1 otherwise); applies to the next sptr_upload_scene. */
int sptr_set_leaf_size(sptr_ctx* ctx, uint32_t max_prims);
/* Split references (early split clipping) for scenes traversed from L2/HBM: a triangle whose box is
 * much larger than the triangle (a sliver lying across the axes) is referenced up to max_pieces times,
 * each reference bounding one piece of it, so that rays near a fan of slivers stop testing every
 * sliver's box.  0 = default (1: no splits — measured no faster on the 10M-triangle mesh),
 * else a power of two up to 32; applies to the next sptr_upload_scene.  Results do not depend on it
 * (each reference tests the same triangle). */
int sptr_set_split_refs(sptr_ctx* ctx, uint32_t max_pieces);
/* Straggler hand-off (ABI 6) for scenes traversed from HBM (a wide BVH beyond an XCD's L2): once a
 * wave of a bounce trace has no rays left to start and at most `lanes` of its 64 lanes are still
 * tracing, those rays are handed to a path-per-thread kernel beside the launch chain, which resumes
 * each walk from the state the trace saved (node, stack, closest hit so far) and finishes the path,
 * so the launch no longer lasts as long as its longest ray.
 * 0 = off, 1..64 (default 12).  Results do not depend on it (each path makes the same operations in
 * the same order wherever it runs); sptr_stats::paths_handed_off counts the paths. */
int sptr_set_stragglers(sptr_ctx* ctx, uint32_t lanes);
/* 0 (default): a render-call shape of at least 2^24 samples seen twice in a row (same frame parameters
 * except frame_begin, same state) is captured into a hipGraph once and replayed from then on — one
 * graph launch per call instead of ~20 kernel launches, the per-call accumulation index passed as a
 * kernel-node argument — except a call whose launches fork to the side streams (the graph executor
 * runs a graph's branches one after another, so such calls launch directly; a shape whose capture
 * fails or is rejected also launches directly from then on).  Smaller calls (the 1-spp interactive
 * frames) launch directly: their replays were no faster and had wall-time spikes;
 * 1: direct kernel launches for every call; 2: direct launches, all on the render stream (no launch
 * overlapped on the context's second stream); 3: as 0 for every repeated shape, whatever its size or
 * side-stream launches.
 * Calls with stage timing (SPTR_FRAME_TIMING*) launch directly in every mode.  Results are identical
 * in every mode. */
int sptr_set_launch_mode(sptr_ctx* ctx, uint32_t mode);
/* Pixel lanes (ABI 8): 2 = a wavefront call renders the even and the odd half of its shard's tiles as
 * two launch chains on two streams of the same GPU, each with its own buffers (the context holds a
 * second, internal context with a copy of the scene), so that each chain's launch tails run beside the
 * other's work; 1 = one chain; 0 (default) = two lanes for calls of >= 2^24 samples, one chain otherwise.
 * Only scenes staged into LDS (sptr_scene_layout_info: lds_bytes > 0) and the wavefront integrator run
 * in two lanes; other calls run as one chain whatever the setting.  An accumulation keeps the lane mode
 * of its first call (frame_begin 1); a change of setting or scene starts a new one.
 * Results are identical either way (each pixel's samples are the same operations in the same order);
 * sptr_tiles_device, sptr_read_rgb8 and sptr_read_accum return the shard as one chain would. */
int sptr_set_pixel_lanes(sptr_ctx* ctx, uint32_t lanes);
/* The pixel-lane setting (0, 1 or 2) and whether the current accumulation runs in two lanes (0 / 1). */
int sptr_pixel_lanes_info(const sptr_ctx* ctx, uint32_t* requested, uint32_t* active);
/* The launch graph the context holds (launch modes 0 and 3): valid = 1 once a call shape was captured; its
 * node count, dependency edges and the nodes on its longest path; captures = graphs captured so far;
 * capture_status = the hipError_t of the last capture attempt that fell back to direct launches (0:
 * none).  Every captured graph is checked to be acyclic before it is instantiated (a rejected capture
 * falls back to direct launches for that shape, reported here and by sptr_capture_error).  Any
 * pointer may be NULL. */
int sptr_graph_info(const sptr_ctx* ctx, uint32_t* valid, uint32_t* nodes, uint32_t* edges, uint32_t* depth,
                    uint32_t* captures, int32_t* capture_status);
/* The call that made the last capture attempt fall back to direct launches, with its error text ("" if none). */
const char* sptr_capture_error(const sptr_ctx* ctx);
/* Whether the context's side streams run beside its render stream on this device: ms[0] = two 200-us
 * one-wave spins on the render stream, ms[1] = one there and one on the shadow side stream, ms[2] = one
 * there and one on the k_sky side stream (device events).  ms[1], ms[2] near ms[0] / 2: the side
 * stream has a hardware queue of its own; near ms[0]: its launches serialise with the render stream's. */
int sptr_overlap_probe(sptr_ctx* ctx, double ms[3]);
/* Traversal width: 2 (the LBVH as built), 4 (collapsed to 64-B quantised BVH4 nodes), or 0 = automatic (the
 * default: 2 for scenes staged in LDS, 4 otherwise). */
int sptr_set_bvh_width(sptr_ctx* ctx, uint32_t width);

/* ---- scene / state (OptixBackend::build and setters) -------------------------------------------- */
int sptr_upload_scene(sptr_ctx* ctx, const sptr_scene* scene); /* builds the LBVH on the device */
int sptr_set_materials(sptr_ctx* ctx, const sptr_material* mats, uint32_t count);
int sptr_set_lights(sptr_ctx* ctx, const sptr_light* lights, uint32_t count);
int sptr_set_environment(sptr_ctx* ctx, const sptr_environment* env);
int sptr_scene_info(const sptr_ctx* ctx, uint32_t* num_prims, uint32_t* num_nodes, uint32_t* bvh_depth,
                    double* build_ms);
/* Device layout of the uploaded scene (DESIGN.md "Data layout in HBM"). lds_bytes = bytes staged into
 * LDS per block by the trace/shadow kernels, 0 when the scene is traversed from HBM/L2. */
typedef struct sptr_scene_layout {
  uint32_t num_tris, num_spheres, num_nodes, leaf_size, bvh_depth, lds_bytes;
  uint64_t node_bytes, tri_bytes, sphere_bytes, prim_ref_bytes;
  uint32_t bvh_width; /* num_nodes / node_bytes describe the traversed (BVH2 or BVH4) nodes */
  uint32_t num_prim_refs; /* primitive references the BVH is built over: num_tris + num_spheres, plus the
                             extra references of split triangles (sptr_set_split_refs) */
} sptr_scene_layout;
int sptr_scene_layout_info(const sptr_ctx* ctx, sptr_scene_layout* out);

/* ---- rendering ---------------------------------------------------------------------------------- */
/* Renders on the context's stream, or on `stream` (a hipStream_t) when not NULL.  Returns after the
 * work completes, with the stats of this call and of any SPTR_FRAME_ASYNC calls still uncollected;
 * with SPTR_FRAME_ASYNC it only enqueues (consecutive asynchronous calls must use one stream).
 * OptixBackend::render blocks three times per bounce (OptixBackend.cpp:1678-1789); asynchronous
 * calls let a caller queue frames, the tile copy and the multi-GPU gather back to back. */
int sptr_render(sptr_ctx* ctx, const sptr_frame* frame, void* stream, sptr_stats* stats);
/* Wait for the uncollected render calls and return their summed stats (zero when there are none). */
int sptr_collect_stats(sptr_ctx* ctx, sptr_stats* stats);
/* Full image RGB8 (width*height*3; only this shard's tiles are written) and the accumulation sums
 * (width*height*3 floats; divide by the frame count for the mean): linear radiance in wavefront
 * mode, tonemapped per-frame colours in PathTracer mode (what GLRenderer accumulates). */
int sptr_read_rgb8(sptr_ctx* ctx, uint8_t* rgb);
/* ABI 9, the interactive loop's readback with one frame of latency (GLRenderer::renderLoop calls render()
 * once per frame, src/GLRenderer.cpp:161-176): call it after an asynchronous render (SPTR_FRAME_ASYNC).  The
 * image of that call is snapshotted on the device (a device-to-device copy ordered after it); the snapshot
 * taken by the previous sptr_read_rgb8_lagged call, if it is of the same size, is copied into rgb on a
 * copy stream of its own — beside the render just enqueued — and waited for: *got = 1.  Otherwise rgb is
 * left alone and *got = 0 (the first frame, or a resize: read that frame with sptr_read_rgb8).  rgb is
 * page-locked (hipHostRegister) while the context uses it as a destination, so the copy is a DMA that
 * overlaps the next frame's kernels; it is unregistered when another buffer takes its place and by
 * sptr_destroy.  The render stream is not waited for: sptr_collect_stats collects the calls' counters. */
int sptr_read_rgb8_lagged(sptr_ctx* ctx, uint8_t* rgb, uint32_t* got);
int sptr_read_accum(sptr_ctx* ctx, float* accum);
/* Device view of this shard's resolved tiles: RGBA8, [local tile][32][32] uint32, for the
 * multi-GPU gather.  *bytes = local_tiles * 4096. */
int sptr_tiles_device(sptr_ctx* ctx, void** dptr, size_t* bytes);
/* Scatter gathered tile buffers (rank-major: rank r's local tiles at offset r*tiles_per_rank*4096
 * bytes) into an RGB8 device image width*height*3.  With stream == NULL it runs on the context's
 * stream and waits; on a caller's stream it only enqueues. */
int sptr_unpack_tiles(sptr_ctx* ctx, const void* gathered, int32_t shard_count, uint32_t tiles_per_rank,
                      int32_t width, int32_t height, void* rgb8_out, void* stream);

/* ---- query entry points (tests / tooling) -------------------------------------------------------- */
/* Closest-hit / any-hit queries on the device BVH: rays = n*8 floats (o3, d3, tnear, tfar).
 * Outputs as rtcIntersect1 reports them: geomID (0xFFFFFFFF on miss), primID, t, unnormalised Ng. */
int sptr_intersect(sptr_ctx* ctx, const float* rays, uint32_t n, uint32_t* geom, uint32_t* prim, float* t,
                   float* ng);
int sptr_occluded(sptr_ctx* ctx, const float* rays, uint32_t n, uint8_t* occluded);
/* Primary rays of the wavefront raygen for a W x H image at accumulation index acc: directions
 * (W*H*3) and initial path RNG states (W*H), computed by the device kernel. */
int sptr_primary_rays(sptr_ctx* ctx, const sptr_camera* cam, int32_t width, int32_t height, uint32_t acc,
                      float* dirs, uint32_t* rng);
/* The LBVH build's device primitives (kernels_sort.hip), exposed for their own tests; they replace
 * the rocPRIM calls Embree's replacement would otherwise make (EmbreeBackend.cpp:82-181 builds on the
 * CPU).  Host arrays in and out, n entries each; every call allocates device scratch and waits.
 *   sptr_sort_pairs_u64: stable ascending LSD radix sort of (keys, vals) (equal keys keep their order);
 *   sptr_scan_u32: exclusive prefix sum of 32-bit counts (mod 2^32); out may equal in. */
int sptr_sort_pairs_u64(sptr_ctx* ctx, const uint64_t* keys, const uint32_t* vals, uint32_t n, uint64_t* keys_out,
                        uint32_t* vals_out);
int sptr_scan_u32(sptr_ctx* ctx, const uint32_t* in, uint32_t n, uint32_t* out);
/* The device's values of the wavefront path's two library calls, for the parity residue classifier:
 * fn SPTR_MATH_COSINE_SINCOS: (sinf, cosf) of the cosine sample's phi = 2 pi r1 for every
 *   r1 = k / 2^24 (wf_math.h:51-72), out = 2^25 floats, pairs by k; x and n are ignored;
 * fn SPTR_MATH_GAMMA: powf(x[i], 1/2.2) as the resolve computes it (GLRenderer.cpp:416-430), n values. */
enum { SPTR_MATH_COSINE_SINCOS = 0, SPTR_MATH_GAMMA = 1 };
int sptr_eval_math(sptr_ctx* ctx, int fn, const float* x, uint32_t n, float* out);

/* ---- host-side scene layer (the C++ SceneDesc / Camera / MaterialManager / LightManager mirror) ---- */
typedef struct sptr_host_scene sptr_host_scene;
/* name: "default", "default_emitter", "sphere_mesh" (p0 = stacks, p1 = slices), "test_triangle",
 * or "gltf:<path>" (p0 = material id for the mesh). */
int sptr_host_builtin_scene(const char* name, uint32_t p0, uint32_t p1, sptr_host_scene** out);
int sptr_host_scene_view(const sptr_host_scene* s, sptr_scene* view);
void sptr_host_scene_free(sptr_host_scene* s);
int sptr_host_camera_lookat(const float pos[3], const float target[3], float fov_deg, float aspect,
                            sptr_camera* out);
/* MaterialManager::setupDefaultMaterials presets; with_light appends Materials::Light() as index 9. */
int sptr_host_preset_materials(int with_light, sptr_material* out, int capacity);
/* setupLights in src/main.cpp:85-94: one directional sun. */
int sptr_host_default_lights(sptr_light* out, int capacity);
/* Cubemap::loadEquirectangular: RGB float equirect (w x h) -> 6 faces of size x size. */
int sptr_host_equirect_to_faces(const float* rgb, int32_t w, int32_t h, int32_t size, float* faces);
/* Host twins of the device tile packing (interleaved 32x32 tiles, shard R of G; see sptr_render):
 * pack this shard's pixels of an RGB8 image into RGBA8 tile-packed words, and scatter gathered
 * rank-major tile buffers back into an RGB8 image. */
int sptr_host_pack_tiles(const uint8_t* rgb, int32_t width, int32_t height, int32_t shard_count, int32_t shard_rank,
                         uint32_t* tiles);
int sptr_host_unpack_tiles(const uint32_t* gathered, int32_t shard_count, uint32_t tiles_per_rank, int32_t width,
                           int32_t height, uint8_t* rgb);
/* Radiance .hdr reader (RGBE, RLE) -> RGB float; caller frees with sptr_host_free. */
int sptr_host_load_hdr(const char* path, float** rgb, int32_t* w, int32_t* h);
void sptr_host_free(void* p);

#ifdef __cplusplus
}
#endif
#endif /* SPTR_HIP_H */
