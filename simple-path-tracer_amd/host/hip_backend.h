// hip_backend.h — backends::HipBackend, the MI355X drop-in for the reference's GPU backend slot.
// Public surface = backends::OptixBackend (include/backends/OptixBackend.h:39-71): build(SceneDesc),
// render(rgb, w, h, Camera), setEnvironment / setMaterialManager / setLightManager (non-owning;
// the pointees must outlive rendering), destroy(), setDebugMode().  Progressive accumulation is
// owned by the backend and restarts on resize or camera change, as OptixBackend::render does
// (src/backends/OptixBackend.cpp:1518-1542).  Extras: setSettings, renderLinear, stats.
// Errors: build() returns false; render() logs and leaves the buffer untouched (no exit()).
#pragma once
#include <array>
#include <cstdint>
#include <string>
#include <vector>

#include "scene_desc.h"
#include "shading.h"

namespace backends {

class HipBackend {
 public:
  struct Settings {
    uint32_t spp_per_call = 1;  // progressive frames per render() call (GLRenderer renders 1)
    uint32_t max_depth = 6;     // PathTracer::Settings::max_depth used by the wavefront tile task
    // SPTR_INTEGRATOR_WAVEFRONT (the 'T' key's wavefront CPU semantics, default) or
    // SPTR_INTEGRATOR_PATHTRACER (the default key's PathTracer semantics, src/GLRenderer.cpp:172-176)
    uint32_t integrator = SPTR_INTEGRATOR_WAVEFRONT;
    uint32_t samples_per_frame = 4;  // PathTracer::Settings::samples_per_pixel (src/main.cpp:107)
    // sptr_set_launch_mode: 0 = replay a captured graph for repeated call shapes (default), 1 = direct
    // launches, 2 = direct on one stream, 3 = a graph for every repeated shape
    uint32_t launch_mode = 0;
    // sptr_set_pixel_lanes: 0 = two concurrent launch chains for calls of >= 2^24 samples on scenes
    // staged in LDS (default), 1 = one chain, 2 = two chains; a change restarts the accumulation
    uint32_t pixel_lanes = 0;
    // render() returns the previous call's image (one frame of latency) so that the read back of one frame
    // runs beside the next frame's kernels (sptr_read_rgb8_lagged); the first frame after a reset or a
    // resize is read synchronously.  The pixel buffer stays page-locked while render() writes into it.
    // Counters (stats()) are collected every kLaggedCollect calls and by flushStats().
    bool lagged_readback = false;
  };
  static constexpr uint32_t kLaggedCollect = 32;

  explicit HipBackend(int device = 0);
  ~HipBackend();
  HipBackend(const HipBackend&) = delete;
  HipBackend& operator=(const HipBackend&) = delete;

  bool build(const scene::SceneDesc& sceneDesc);
  void render(unsigned char* pixels, int width, int height, const Camera& camera);
  void setEnvironment(const EnvironmentManager* env) { env_ = env; env_dirty_ = true; }
  void setMaterialManager(const MaterialManager* mm) { mm_ = mm; mats_dirty_ = true; }
  void setLightManager(const LightManager* lm) { lm_ = lm; lights_dirty_ = true; }
  void destroy();
  void setDebugMode(int mode);

  void setSettings(const Settings& s) { settings_ = s; }
  const Settings& getSettings() const { return settings_; }
  // linear accumulated radiance mean (width*height*3) of the current accumulation
  bool renderLinear(float* rgb32, int width, int height, const Camera& camera);
  const sptr_stats& stats() const { return stats_; }
  // the counters of every render() since the last flush, summed (waits for the pending frames)
  sptr_stats flushStats();
  uint32_t frameIndex() const { return frame_index_; }
  const std::string& lastError() const { return err_; }
  const std::vector<uint32_t>& getGeomMaterialMapping() const { return geom_material_; }

 private:
  bool ensureContext();
  bool syncState();
  bool renderInternal(int width, int height, const Camera& camera, bool async = false);
  void addStats(const sptr_stats& s);

  int device_;
  sptr_ctx* ctx_ = nullptr;
  const EnvironmentManager* env_ = nullptr;
  const MaterialManager* mm_ = nullptr;
  const LightManager* lm_ = nullptr;
  bool env_dirty_ = true, mats_dirty_ = true, lights_dirty_ = true, built_ = false;
  Settings settings_;
  sptr_stats stats_{};
  uint32_t frame_index_ = 0;
  int last_w_ = 0, last_h_ = 0;
  bool has_last_camera_ = false;
  std::array<float, 9> last_cam_{};
  std::vector<uint32_t> geom_material_;
  std::string err_;
  int debug_mode_ = 0;
  uint32_t lanes_applied_ = 0;  // the pixel-lane setting the context holds
  sptr_stats flushed_{};        // counters since the last flushStats()
  uint32_t async_calls_ = 0;    // lagged mode: render calls not yet collected
};

}  // namespace backends
