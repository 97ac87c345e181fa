// sptr_cli — headless harness for the HIP backend (the reference only has a GLFW window,
// src/GLRenderer.cpp:111-189).  Composes the same state as src/main.cpp (camera (0,3,8)->(0,1,0),
// fov 60, one sun, depth 6) and drives backends::HipBackend exactly as GLRenderer drives a backend:
// one render() per frame, progressive accumulation.
//   sptr_cli [--scene default|default_emitter|test_triangle|sphere_mesh:STACKS:SLICES|gltf:PATH]
//            [--w 800] [--h 600] [--spp 4] [--depth 6] [--env sky|FILE.hdr] [--out image.ppm]
//            [--warmup N] [--json] [--integrator wavefront|pathtracer|optix] [--spf 4] [--launch-mode 0-3]
//            [--lagged]
// --spp N renders N progressive frames of 1 spp each (GLRenderer's m_accumulated_samples loop);
// --warmup N renders N untimed frames first (then restarts the accumulation by a camera change);
// --json prints one line with per-frame wall-clock statistics (render + RGB8 read back, as the
// window loop pays them) for bench.py's interactive leg.  --lagged: HipBackend::Settings::lagged_readback
// (each render() returns the previous frame's image, read back beside the next frame's kernels).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "hip_backend.h"

static bool build_scene(const std::string& s, scene::SceneDesc& sd, MaterialManager& mm, std::string& err) {
  if (s == "default") sd = scene::BuildDefaultScene();
  else if (s == "default_emitter") {
    sd = scene::BuildDefaultSceneWithEmitter();
    mm.addMaterial(Materials::Light());
  } else if (s == "test_triangle") sd = scene::BuildTestTriangleScene();
  else if (s.rfind("sphere_mesh:", 0) == 0) {
    unsigned a = 0, b = 0;
    if (std::sscanf(s.c_str() + 12, "%u:%u", &a, &b) != 2) { err = "bad sphere_mesh spec"; return false; }
    sd = scene::BuildSphereMeshScene(a, b);
  } else if (s.rfind("gltf:", 0) == 0) {
    return scene::LoadGLTFScene(s.substr(5), 7, sd, &err);
  } else {
    err = "unknown scene " + s;
    return false;
  }
  return true;
}

int main(int argc, char** argv) {
  std::string scene_name = "default", env = "sky", out = "image.ppm";
  int w = 800, h = 600, spp = 4, depth = 6, warmup = 0;
  bool json = false, lagged = false;
  std::string integrator = "wavefront";
  int spf = 4, launch_mode = 0;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&](void) -> const char* { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "--scene") scene_name = next();
    else if (a == "--w") w = std::atoi(next());
    else if (a == "--h") h = std::atoi(next());
    else if (a == "--spp") spp = std::atoi(next());
    else if (a == "--depth") depth = std::atoi(next());
    else if (a == "--env") env = next();
    else if (a == "--out") out = next();
    else if (a == "--warmup") warmup = std::atoi(next());
    else if (a == "--json") json = true;
    else if (a == "--integrator") integrator = next();
    else if (a == "--spf") spf = std::atoi(next());
    else if (a == "--launch-mode") launch_mode = std::atoi(next());
    else if (a == "--lagged") lagged = true;
    else {
      std::fprintf(stderr, "usage: %s [--scene S] [--w W] [--h H] [--spp N] [--depth D] [--env sky|F.hdr] [--out F] [--warmup N] [--json]\n",
                   argv[0]);
      return 2;
    }
  }
  scene::SceneDesc sd;
  MaterialManager mm;
  std::string err;
  if (!build_scene(scene_name, sd, mm, err)) {
    std::fprintf(stderr, "scene: %s\n", err.c_str());
    return 1;
  }
  LightManager lm;
  lm.addDirectionalLight(vec3{-0.5f, -1.0f, 0.3f}, vec3{1.0f, 0.95f, 0.8f}, 2.0f);
  EnvironmentManager em;
  if (env != "sky" && !em.loadCubemap(env, &err)) {
    std::fprintf(stderr, "env: %s (using procedural sky)\n", err.c_str());
  }
  Camera cam(vec3{0.0f, 3.0f, 8.0f}, vec3{0.0f, 1.0f, 0.0f}, vec3{0.0f, 1.0f, 0.0f}, 60.0f, float(w) / float(h));
  backends::HipBackend be(0);
  be.setMaterialManager(&mm);
  be.setLightManager(&lm);
  be.setEnvironment(&em);
  backends::HipBackend::Settings st;
  st.max_depth = uint32_t(depth);
  if (integrator == "pathtracer") st.integrator = SPTR_INTEGRATOR_PATHTRACER;
  else if (integrator == "optix") st.integrator = SPTR_INTEGRATOR_OPTIX;
  else if (integrator != "wavefront") {
    std::fprintf(stderr, "unknown integrator %s\n", integrator.c_str());
    return 2;
  }
  st.samples_per_frame = uint32_t(spf);
  st.launch_mode = uint32_t(launch_mode);
  st.lagged_readback = lagged;
  be.setSettings(st);
  if (!be.build(sd)) {
    std::fprintf(stderr, "%s\n", be.lastError().c_str());
    return 1;
  }
  std::vector<unsigned char> img(size_t(w) * h * 3);
  if (warmup > 0) {
    Camera wcam(vec3{0.0f, 3.0f, 8.5f}, vec3{0.0f, 1.0f, 0.0f}, vec3{0.0f, 1.0f, 0.0f}, 60.0f, float(w) / float(h));
    for (int f = 0; f < warmup; ++f) be.render(img.data(), w, h, wcam);  // the camera change below resets
  }
  std::vector<double> frame_ms;
  frame_ms.reserve(size_t(spp));
  (void)be.flushStats();  // (the warmup's counters)
  const auto t0 = std::chrono::steady_clock::now();
  for (int f = 0; f < spp; ++f) {
    const auto f0 = std::chrono::steady_clock::now();
    be.render(img.data(), w, h, cam);
    frame_ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - f0).count());
  }
  const sptr_stats tot = be.flushStats();  // (lagged: waits for the last frames, inside the clock)
  const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  const uint64_t rays = tot.rays_closest + tot.rays_shadow;
  const double ms = tot.ms_total;
  if (json) {
    std::vector<double> s = frame_ms;
    std::sort(s.begin(), s.end());
    auto pct = [&](double q) { return s.empty() ? 0.0 : s[std::min(s.size() - 1, size_t(q * double(s.size())))]; };
    std::printf("{\"scene\": \"%s\", \"launch_mode\": %d, \"width\": %d, \"height\": %d, \"frames\": %d, \"spp_per_frame\": 1, "
                "\"depth\": %d, \"ms_per_frame_wall\": %.4f, \"ms_per_frame_p50\": %.4f, \"ms_per_frame_p99\": %.4f, "
                "\"ms_per_frame_device\": %.4f, \"fps\": %.1f, \"mrays_per_s_wall\": %.1f, "
                "\"lagged_readback\": %s, \"path\": \"backends::HipBackend::render (sptr_render + %s per frame)\"}\n",
                scene_name.c_str(), launch_mode, w, h, spp, depth, wall / spp, pct(0.5), pct(0.99), ms / spp,
                wall > 0 ? 1e3 * spp / wall : 0.0, wall > 0 ? rays / (wall * 1e3) : 0.0, lagged ? "true" : "false",
                lagged ? "sptr_read_rgb8_lagged" : "sptr_read_rgb8");
  } else {
    std::printf("scene=%s %dx%d spp=%d depth=%d: %.2f ms device, %.2f ms wall, %.1f Mrays/s (device)\n",
                scene_name.c_str(), w, h, spp, depth, ms, wall, ms > 0 ? rays / (ms * 1e3) : 0.0);
  }
  FILE* fp = std::fopen(out.c_str(), "wb");
  if (!fp) return 1;
  std::fprintf(fp, "P6\n%d %d\n255\n", w, h);
  std::fwrite(img.data(), 1, img.size(), fp);
  std::fclose(fp);
  return 0;
}
