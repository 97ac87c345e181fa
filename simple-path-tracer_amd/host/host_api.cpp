// host_api.cpp — C ABI access to the host-side scene layer (sptr_host_* in include/sptr_hip.h), so
// foreign callers (ctypes harness, CLI) build scenes, cameras and material tables with exactly the
// C++ code the HipBackend uses.
#include <cstdlib>
#include <cstring>
#include <string>

#include "../csrc/tile_map.h"
#include "scene_desc.h"
#include "shading.h"

struct sptr_host_scene {
  scene::FlatScene flat;
};

extern "C" {

int sptr_host_builtin_scene(const char* name, uint32_t p0, uint32_t p1, sptr_host_scene** out) {
  if (!name || !out) return SPTR_ERR_INVALID;
  *out = nullptr;
  const std::string n(name);
  scene::SceneDesc sd;
  if (n == "default") sd = scene::BuildDefaultScene();
  else if (n == "default_emitter") sd = scene::BuildDefaultSceneWithEmitter();
  else if (n == "test_triangle") sd = scene::BuildTestTriangleScene();
  else if (n == "sphere_mesh") {
    if (p0 == 0 || p1 == 0) return SPTR_ERR_INVALID;
    sd = scene::BuildSphereMeshScene(p0, p1);
  } else if (n.rfind("gltf:", 0) == 0) {
    std::string err;
    if (!scene::LoadGLTFScene(n.substr(5), p0, sd, &err)) return SPTR_ERR_INVALID;
  } else {
    return SPTR_ERR_INVALID;
  }
  sptr_host_scene* s = new sptr_host_scene();
  s->flat = scene::Flatten(sd);
  *out = s;
  return SPTR_OK;
}

int sptr_host_scene_view(const sptr_host_scene* s, sptr_scene* view) {
  if (!s || !view) return SPTR_ERR_INVALID;
  *view = s->flat.view();
  return SPTR_OK;
}

void sptr_host_scene_free(sptr_host_scene* s) { delete s; }

int sptr_host_camera_lookat(const float pos[3], const float target[3], float fov_deg, float aspect, sptr_camera* out) {
  if (!pos || !target || !out) return SPTR_ERR_INVALID;
  const Camera c(vec3{pos[0], pos[1], pos[2]}, vec3{target[0], target[1], target[2]}, vec3{0.0f, 1.0f, 0.0f}, fov_deg,
                 aspect);
  *out = c.toDevice();
  return SPTR_OK;
}

int sptr_host_preset_materials(int with_light, sptr_material* out, int capacity) {
  MaterialManager mm;
  if (with_light) mm.addMaterial(Materials::Light());
  std::vector<sptr_material> v;
  mm.buildDeviceMaterials(v);
  if (out)
    for (int i = 0; i < int(v.size()) && i < capacity; ++i) out[i] = v[size_t(i)];
  return int(v.size());
}

int sptr_host_default_lights(sptr_light* out, int capacity) {
  LightManager lm;  // setupLights, src/main.cpp:85-94
  lm.addDirectionalLight(vec3{-0.5f, -1.0f, 0.3f}, vec3{1.0f, 0.95f, 0.8f}, 2.0f);
  std::vector<sptr_light> v;
  lm.buildDeviceLights(v);
  if (out)
    for (int i = 0; i < int(v.size()) && i < capacity; ++i) out[i] = v[size_t(i)];
  return int(v.size());
}

int sptr_host_equirect_to_faces(const float* rgb, int32_t w, int32_t h, int32_t size, float* faces) {
  if (!rgb || !faces || w <= 0 || h <= 0 || size < 2) return SPTR_ERR_INVALID;
  EquirectToFaces(rgb, w, h, size, faces);
  return SPTR_OK;
}

int sptr_host_pack_tiles(const uint8_t* rgb, int32_t W, int32_t H, int32_t G, int32_t R, uint32_t* tiles) {
  if (!rgb || !tiles || W <= 0 || H <= 0 || G <= 0 || R < 0 || R >= G) return SPTR_ERR_INVALID;
  const uint32_t n = sptr::shard_tiles(W, H, G, R) * 1024u;
  for (uint32_t l = 0; l < n; ++l) {
    int x, y;
    if (!sptr::shard_pixel(W, H, G, R, l, x, y)) {
      tiles[l] = 0u;
      continue;
    }
    const uint8_t* p = rgb + ((size_t)y * W + x) * 3;
    tiles[l] = uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | 0xFF000000u;
  }
  return SPTR_OK;
}

int sptr_host_unpack_tiles(const uint32_t* g, int32_t G, uint32_t tpr, int32_t W, int32_t H, uint8_t* rgb) {
  if (!g || !rgb || W <= 0 || H <= 0 || G <= 0) return SPTR_ERR_INVALID;
  if ((uint64_t)tpr * (uint64_t)G < (uint64_t)sptr::tiles_total(W, H)) return SPTR_ERR_INVALID;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      uint32_t r, l;
      sptr::pixel_shard(W, G, x, y, r, l);
      const uint32_t px = g[(size_t)r * tpr * 1024u + l];
      uint8_t* o = rgb + ((size_t)y * W + x) * 3;
      o[0] = uint8_t(px & 0xFF);
      o[1] = uint8_t((px >> 8) & 0xFF);
      o[2] = uint8_t((px >> 16) & 0xFF);
    }
  return SPTR_OK;
}

int sptr_host_load_hdr(const char* path, float** rgb, int32_t* w, int32_t* h) {
  if (!path || !rgb || !w || !h) return SPTR_ERR_INVALID;
  std::vector<float> v;
  int ww = 0, hh = 0;
  if (!LoadRadianceHDR(path, v, ww, hh, nullptr)) return SPTR_ERR_INVALID;
  float* p = static_cast<float*>(std::malloc(v.size() * sizeof(float)));
  if (!p) return SPTR_ERR_OOM;
  std::memcpy(p, v.data(), v.size() * sizeof(float));
  *rgb = p;
  *w = ww;
  *h = hh;
  return SPTR_OK;
}

void sptr_host_free(void* p) { std::free(p); }

}  // extern "C"
