// hip_backend.cpp — backends::HipBackend over the C ABI (include/sptr_hip.h).
#include "hip_backend.h"

#include <cmath>
#include <cstdio>

namespace backends {

HipBackend::HipBackend(int device) : device_(device) {}
HipBackend::~HipBackend() { destroy(); }

bool HipBackend::ensureContext() {
  if (ctx_) return true;
  const int rc = sptr_create(device_, &ctx_);
  if (rc != SPTR_OK) {
    err_ = "HipBackend: sptr_create failed (" + std::to_string(rc) + ")";
    ctx_ = nullptr;
    return false;
  }
  sptr_set_debug_mode(ctx_, debug_mode_);
  return true;
}

void HipBackend::destroy() {
  if (ctx_) (void)flushStats();
  if (ctx_) sptr_destroy(ctx_);
  ctx_ = nullptr;
  built_ = false;
  frame_index_ = 0;
  has_last_camera_ = false;
}

void HipBackend::setDebugMode(int mode) {
  debug_mode_ = mode;
  if (ctx_) sptr_set_debug_mode(ctx_, mode);
  frame_index_ = 0;
}

bool HipBackend::build(const scene::SceneDesc& sd) {
  if (!ensureContext()) return false;
  const scene::FlatScene flat = scene::Flatten(sd);
  const sptr_scene v = flat.view();
  const int rc = sptr_upload_scene(ctx_, &v);
  if (rc != SPTR_OK) {
    err_ = std::string("HipBackend::build: ") + sptr_last_error(ctx_);
    return false;
  }
  geom_material_ = flat.geom_material;
  built_ = true;
  frame_index_ = 0;
  return true;
}

bool HipBackend::syncState() {
  if (mats_dirty_) {
    std::vector<sptr_material> m;
    if (mm_) mm_->buildDeviceMaterials(m);
    else MaterialManager().buildDeviceMaterials(m);
    if (sptr_set_materials(ctx_, m.data(), uint32_t(m.size())) != SPTR_OK) return false;
    mats_dirty_ = false;
    frame_index_ = 0;
  }
  if (lights_dirty_) {
    std::vector<sptr_light> l;
    if (lm_) lm_->buildDeviceLights(l);
    if (sptr_set_lights(ctx_, l.data(), uint32_t(l.size())) != SPTR_OK) return false;
    lights_dirty_ = false;
    frame_index_ = 0;
  }
  if (env_dirty_) {
    sptr_environment e{};
    e.intensity = 0.8f;
    e.max_clamp = 5.0f;
    if (env_) e = env_->toDevice();
    if (sptr_set_environment(ctx_, &e) != SPTR_OK) return false;
    env_dirty_ = false;
    frame_index_ = 0;
  }
  return true;
}

void HipBackend::addStats(const sptr_stats& s) {
  flushed_.rays_closest += s.rays_closest;
  flushed_.rays_shadow += s.rays_shadow;
  flushed_.samples += s.samples;
  flushed_.waves += s.waves;
  flushed_.ms_total += s.ms_total;
  flushed_.ms_trace += s.ms_trace;
  flushed_.trace_launches += s.trace_launches;
}

sptr_stats HipBackend::flushStats() {
  if (ctx_ && async_calls_) {
    sptr_stats s{};
    if (sptr_collect_stats(ctx_, &s) == SPTR_OK) {
      stats_ = s;
      addStats(s);
    }
    async_calls_ = 0;
  }
  const sptr_stats out = flushed_;
  flushed_ = sptr_stats{};
  return out;
}

bool HipBackend::renderInternal(int w, int h, const Camera& camera, bool async) {
  if (!built_ || !ctx_) {
    err_ = "HipBackend::render: build() has not succeeded";
    return false;
  }
  if (!syncState()) {
    err_ = std::string("HipBackend: state upload failed: ") + sptr_last_error(ctx_);
    return false;
  }
  // progressive reset on resize / camera change (OptixBackend.cpp:1518-1542, eps 1e-4)
  const vec3 p = camera.getPosition(), f = camera.getFront(), u = camera.getUp();
  const std::array<float, 9> cam = {p.x, p.y, p.z, f.x, f.y, f.z, u.x, u.y, u.z};
  bool changed = !has_last_camera_ || w != last_w_ || h != last_h_;
  for (int i = 0; i < 9 && !changed; ++i) changed = std::fabs(cam[size_t(i)] - last_cam_[size_t(i)]) > 1e-4f;
  if (settings_.pixel_lanes != lanes_applied_) {
    if (sptr_set_pixel_lanes(ctx_, settings_.pixel_lanes) != SPTR_OK) {
      err_ = std::string("HipBackend::render: ") + sptr_last_error(ctx_);
      return false;
    }
    lanes_applied_ = settings_.pixel_lanes;
    changed = true;  // a new accumulation in the new lane mode
  }
  if (changed) frame_index_ = 0;
  has_last_camera_ = true;
  last_cam_ = cam;
  last_w_ = w;
  last_h_ = h;

  sptr_frame fr{};
  fr.width = w;
  fr.height = h;
  fr.camera = camera.toDevice();
  fr.frame_begin = frame_index_ + 1;
  fr.spp = settings_.spp_per_call ? settings_.spp_per_call : 1;
  fr.max_depth = settings_.max_depth;
  fr.shard_rank = 0;
  fr.shard_count = 1;
  fr.integrator = settings_.integrator;
  fr.samples_per_frame = settings_.samples_per_frame;
  if (async) fr.flags |= SPTR_FRAME_ASYNC;
  if (sptr_set_launch_mode(ctx_, settings_.launch_mode) != SPTR_OK) {
    err_ = std::string("HipBackend::render: ") + sptr_last_error(ctx_);
    return false;
  }
  sptr_stats st{};
  const int rc = sptr_render(ctx_, &fr, nullptr, &st);
  if (rc != SPTR_OK) {
    err_ = std::string("HipBackend::render: ") + sptr_last_error(ctx_);
    return false;
  }
  if (async) {
    ++async_calls_;
  } else {
    stats_ = st;  // (a synchronous call also collects any pending asynchronous ones)
    addStats(st);
    async_calls_ = 0;
  }
  frame_index_ += fr.spp;
  return true;
}

void HipBackend::render(unsigned char* pixels, int width, int height, const Camera& camera) {
  const bool lagged = settings_.lagged_readback;
  if (!renderInternal(width, height, camera, lagged)) {
    std::fprintf(stderr, "%s\n", err_.c_str());
    return;
  }
  if (lagged) {
    // the previous frame's image, copied while this frame's kernels run; none yet (the first frame or a
    // resize): this frame's, synchronously
    uint32_t got = 0;
    if (sptr_read_rgb8_lagged(ctx_, pixels, &got) != SPTR_OK) {
      std::fprintf(stderr, "HipBackend: %s\n", sptr_last_error(ctx_));
      return;
    }
    if (!got && sptr_read_rgb8(ctx_, pixels) != SPTR_OK) std::fprintf(stderr, "HipBackend: %s\n", sptr_last_error(ctx_));
    if (async_calls_ >= kLaggedCollect) {  // bounded: each pending call holds its call-span events
      sptr_stats s{};
      if (sptr_collect_stats(ctx_, &s) == SPTR_OK) {
        stats_ = s;
        addStats(s);
      }
      async_calls_ = 0;
    }
    return;
  }
  if (sptr_read_rgb8(ctx_, pixels) != SPTR_OK) std::fprintf(stderr, "HipBackend: %s\n", sptr_last_error(ctx_));
}

bool HipBackend::renderLinear(float* rgb32, int width, int height, const Camera& camera) {
  if (!renderInternal(width, height, camera)) return false;
  if (sptr_read_accum(ctx_, rgb32) != SPTR_OK) return false;  // PathTracer mode: mean tonemapped colour
  const float n = float(frame_index_);
  for (size_t i = 0; i < size_t(width) * height * 3; ++i) rgb32[i] /= n;
  return true;
}

}  // namespace backends
