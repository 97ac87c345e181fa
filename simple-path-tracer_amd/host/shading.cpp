// shading.cpp — host-side camera / material / light / environment state (see shading.h for the
// reference interfaces mirrored).  Float math calls use the float overloads, as the reference's
// MSVC build resolves its unqualified calls.
#include "shading.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>

using sptr::cross;
using sptr::normalize;

namespace {
inline float deg2rad(float d) { return d * 0.01745329251994329576923690768489f; }
inline float rad2deg(float r) { return r * 57.295779513082320876798154814105f; }
inline float clampf(float x, float lo, float hi) { return sptr::clamp_g(x, lo, hi); }
}  // namespace

// ------------------------------------------------------------------------------------- Camera
Camera::Camera(const vec3& position, const vec3& target, const vec3& up, float fov, float aspect_ratio)
    : pos_(position), target_(target), world_up_(up), fov_(fov), aspect_(aspect_ratio), last_pos_(position) {
  const vec3 d = normalize(target - position);
  yaw_ = rad2deg(std::atan2(d.z, d.x));
  pitch_ = rad2deg(std::asin(d.y));
  last_yaw_ = yaw_;
  last_pitch_ = pitch_;
  update();
}

void Camera::update() {  // Camera::updateCameraVectors: yaw/pitch -> forward, right, up, half extents
  vec3 f;
  f.x = std::cos(deg2rad(yaw_)) * std::cos(deg2rad(pitch_));
  f.y = std::sin(deg2rad(pitch_));
  f.z = std::sin(deg2rad(yaw_)) * std::cos(deg2rad(pitch_));
  fwd_ = normalize(f);
  right_ = normalize(cross(fwd_, vec3{0.0f, 1.0f, 0.0f}));
  up_ = normalize(cross(right_, fwd_));
  target_ = pos_ + fwd_;
  half_h_ = std::tan(deg2rad(fov_) * 0.5f);
  half_w_ = half_h_ * aspect_;
}

vec3 Camera::getRayDirection(float x, float y) const {
  const float nx = (x - 0.5f) * 2.0f;
  const float ny = -(y - 0.5f) * 2.0f;
  return normalize(fwd_ + nx * half_w_ * right_ + ny * half_h_ * up_);
}

void Camera::processKeyboard(int direction, float dt) {
  const float v = speed_ * dt;
  if (direction == FORWARD) pos_ = pos_ + fwd_ * v;
  else if (direction == BACKWARD) pos_ = pos_ - fwd_ * v;
  else if (direction == LEFT) pos_ = pos_ - right_ * v;
  else if (direction == RIGHT) pos_ = pos_ + right_ * v;
  target_ = pos_ + fwd_;
}

void Camera::processMouseMovement(float xo, float yo, bool constrainPitch) {
  yaw_ += xo * sensitivity_;
  pitch_ += yo * sensitivity_;
  if (constrainPitch) pitch_ = std::clamp(pitch_, -89.0f, 89.0f);
  update();
}

void Camera::setPosition(const vec3& p) {
  pos_ = p;
  target_ = pos_ + fwd_;
}

void Camera::setAspectRatio(float a) {
  aspect_ = a;
  update();
}

bool Camera::hasMovedSinceLastCheck(float pth, float rth) {
  if (first_check_) {
    first_check_ = false;
    return true;
  }
  const vec3 d = pos_ - last_pos_;
  const bool moved = std::sqrt(sptr::dot(d, d)) > pth || std::fabs(yaw_ - last_yaw_) > rth ||
                     std::fabs(pitch_ - last_pitch_) > rth;
  if (moved) {
    last_pos_ = pos_;
    last_yaw_ = yaw_;
    last_pitch_ = pitch_;
  }
  return moved;
}

sptr_camera Camera::toDevice() const {
  sptr_camera c{};
  const vec3* v[4] = {&pos_, &fwd_, &right_, &up_};
  float* o[4] = {c.pos, c.forward, c.right, c.up};
  for (int i = 0; i < 4; ++i) {
    o[i][0] = v[i]->x;
    o[i][1] = v[i]->y;
    o[i][2] = v[i]->z;
  }
  c.half_width = half_w_;
  c.half_height = half_h_;
  return c;
}

// ------------------------------------------------------------------------------------- Material
Material::Material(const vec3& a, float m, float r, const vec3& e, float ior_, MaterialType t)
    : albedo(a), metallic(clampf(m, 0.0f, 1.0f)), roughness(clampf(r, 0.01f, 1.0f)), emission(e), ior(ior_),
      materialType(t) {}

float Material::getTransparency() const { return isTransparent() ? clampf((ior - 1.0f) / 0.7f, 0.0f, 0.95f) : 0.0f; }

sptr_material Material::toDevice() const {
  sptr_material d{};
  d.albedo[0] = albedo.x;
  d.albedo[1] = albedo.y;
  d.albedo[2] = albedo.z;
  d.metallic = metallic;
  d.roughness = roughness;
  d.emission[0] = emission.x;
  d.emission[1] = emission.y;
  d.emission[2] = emission.z;
  d.ior = ior;
  d.type = static_cast<int32_t>(materialType);
  return d;
}

namespace Materials {
Material Gold() { return Material(vec3{1.0f, 0.71f, 0.29f}, 1.0f, 0.05f); }
Material Silver() { return Material(vec3{0.95f, 0.93f, 0.88f}, 1.0f, 0.02f); }
Material Copper() { return Material(vec3{0.95f, 0.64f, 0.54f}, 1.0f, 0.08f); }
Material Iron() { return Material(vec3{0.56f, 0.57f, 0.58f}, 1.0f, 0.3f); }
Material Plastic() { return Material(vec3{0.8f, 0.2f, 0.2f}, 0.0f, 0.4f, vec3{0, 0, 0}, 1.2f); }
Material Rubber() { return Material(vec3{0.3f, 0.3f, 0.3f}, 0.0f, 0.8f, vec3{0, 0, 0}, 1.1f); }
Material Glass() { return Material(vec3{1.0f, 1.0f, 1.0f}, 0.0f, 0.0f, vec3{0, 0, 0}, 1.5f, MaterialType::DIELECTRIC); }
Material ClearGlass() {
  return Material(vec3{0.95f, 0.98f, 1.0f}, 0.0f, 0.02f, vec3{0, 0, 0}, 1.5f, MaterialType::DIELECTRIC);
}
Material Wood() { return Material(vec3{0.4f, 0.25f, 0.1f}, 0.0f, 0.7f, vec3{0, 0, 0}, 1.0f); }
Material Concrete() { return Material(vec3{0.6f, 0.6f, 0.6f}, 0.0f, 0.9f, vec3{0, 0, 0}, 1.0f); }
Material Light(const vec3& color, float intensity) {
  return Material(vec3{0.0f, 0.0f, 0.0f}, 0.0f, 1.0f, color * intensity);
}
}  // namespace Materials

MaterialManager::MaterialManager() {
  mats_ = {Materials::Gold(),    Materials::Silver(), Materials::Copper(), Materials::Iron(),    Materials::Glass(),
           Materials::Plastic(), Materials::Rubber(), Materials::Wood(),   Materials::Concrete()};
}

void MaterialManager::setMaterial(int i, const Material& m) {
  if (i >= 0 && i < int(mats_.size())) mats_[size_t(i)] = m;
}

const Material& MaterialManager::getMaterial(int i) const {
  return (i >= 0 && i < int(mats_.size())) ? mats_[size_t(i)] : mats_[0];
}

void MaterialManager::buildDeviceMaterials(std::vector<sptr_material>& out) const {
  out.clear();
  for (const Material& m : mats_) out.push_back(m.toDevice());
}

// ------------------------------------------------------------------------------------- lights
DirectionalLight::DirectionalLight(const vec3& direction, const vec3& color, float intensity)
    : Light(DIRECTIONAL, color, intensity), given_(direction), to_light_(normalize(-direction)) {}

sptr_light DirectionalLight::toDevice() const {
  sptr_light l{};
  l.type = 0;
  l.v[0] = given_.x;
  l.v[1] = given_.y;
  l.v[2] = given_.z;
  l.color[0] = color_.x;
  l.color[1] = color_.y;
  l.color[2] = color_.z;
  l.intensity = intensity_;
  return l;
}

sptr_light PointLight::toDevice() const {
  sptr_light l{};
  l.type = 1;
  l.v[0] = pos_.x;
  l.v[1] = pos_.y;
  l.v[2] = pos_.z;
  l.color[0] = color_.x;
  l.color[1] = color_.y;
  l.color[2] = color_.z;
  l.intensity = intensity_;
  return l;
}

void LightManager::addDirectionalLight(const vec3& d, const vec3& c, float i) {
  lights_.push_back(std::make_unique<DirectionalLight>(d, c, i));
}
void LightManager::addPointLight(const vec3& p, const vec3& c, float i) {
  lights_.push_back(std::make_unique<PointLight>(p, c, i));
}
void LightManager::buildDeviceLights(std::vector<sptr_light>& out) const {
  out.clear();
  for (const auto& l : lights_) out.push_back(l->toDevice());
}

// ------------------------------------------------------------------------------------- environment
void EquirectToFaces(const float* rgb, int w, int h, int size, float* faces) {
  const double PI = 3.14159265358979323846;
  for (int f = 0; f < 6; ++f)
    for (int y = 0; y < size; ++y)
      for (int x = 0; x < size; ++x) {
        const float u = (2.0f * x / (size - 1)) - 1.0f;
        const float v = (2.0f * y / (size - 1)) - 1.0f;
        vec3 d;
        switch (f) {
          case 0: d = vec3{1.0f, -v, -u}; break;
          case 1: d = vec3{-1.0f, -v, u}; break;
          case 2: d = vec3{u, 1.0f, v}; break;
          case 3: d = vec3{u, -1.0f, -v}; break;
          case 4: d = vec3{u, -v, 1.0f}; break;
          default: d = vec3{-u, -v, -1.0f}; break;
        }
        d = normalize(d);
        const float theta = std::atan2(d.z, d.x);
        const float phi = std::acos(d.y);
        const float uu = float((double(theta) + PI) / (2.0f * PI));
        const float vv = float(double(phi) / PI);
        const int sx = std::min(std::max(int(uu * w), 0), w - 1);
        const int sy = std::min(std::max(int(vv * h), 0), h - 1);
        const float* s = rgb + (size_t(sy) * w + sx) * 3;
        float* o = faces + ((size_t(f) * size + y) * size + x) * 3;
        o[0] = s[0];
        o[1] = s[1];
        o[2] = s[2];
      }
}

void EnvironmentManager::setEquirectangular(const float* rgb, int w, int h, int face_size) {
  size_ = face_size;
  faces_.assign(size_t(6) * face_size * face_size * 3, 0.0f);
  EquirectToFaces(rgb, w, h, face_size, faces_.data());
}

bool EnvironmentManager::loadCubemap(const std::string& filename, std::string* err) {
  std::vector<float> rgb;
  int w = 0, h = 0;
  if (!LoadRadianceHDR(filename, rgb, w, h, err)) return false;
  setEquirectangular(rgb.data(), w, h, 512);
  return true;
}

sptr_environment EnvironmentManager::toDevice() const {
  sptr_environment e{};
  e.faces = size_ > 0 ? faces_.data() : nullptr;
  e.size = size_;
  e.intensity = intensity_;
  e.max_clamp = max_clamp_;
  return e;
}

// Radiance RGBE: header lines until an empty line, "-Y h +X w", then scanlines (new RLE or flat).
bool LoadRadianceHDR(const std::string& path, std::vector<float>& rgb, int& w, int& h, std::string* err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    if (err) *err = "hdr: cannot open " + path;
    return false;
  }
  std::string line;
  std::getline(f, line);
  if (line.rfind("#?", 0) != 0) {
    if (err) *err = "hdr: bad magic";
    return false;
  }
  while (std::getline(f, line) && !line.empty()) {
    if (line.rfind("FORMAT=", 0) == 0 && line != "FORMAT=32-bit_rle_rgbe") {
      if (err) *err = "hdr: unsupported format " + line;
      return false;
    }
  }
  if (!std::getline(f, line) || std::sscanf(line.c_str(), "-Y %d +X %d", &h, &w) != 2 || w <= 0 || h <= 0) {
    if (err) *err = "hdr: unsupported resolution line";
    return false;
  }
  std::vector<uint8_t> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  size_t pos = 0;
  std::vector<uint8_t> scan(size_t(w) * 4);
  rgb.assign(size_t(w) * h * 3, 0.0f);
  for (int y = 0; y < h; ++y) {
    if (w >= 8 && w < 32768 && pos + 4 <= data.size() && data[pos] == 2 && data[pos + 1] == 2 &&
        ((data[pos + 2] << 8) | data[pos + 3]) == w) {
      pos += 4;
      for (int c = 0; c < 4; ++c) {
        int x = 0;
        while (x < w) {
          if (pos >= data.size()) { if (err) *err = "hdr: truncated"; return false; }
          int n = data[pos++];
          if (n > 128) {
            n -= 128;
            if (pos >= data.size() || x + n > w) { if (err) *err = "hdr: bad run"; return false; }
            const uint8_t v = data[pos++];
            for (int k = 0; k < n; ++k) scan[size_t(x++) * 4 + c] = v;
          } else {
            if (n == 0 || pos + n > data.size() || x + n > w) { if (err) *err = "hdr: bad literal"; return false; }
            for (int k = 0; k < n; ++k) scan[size_t(x++) * 4 + c] = data[pos++];
          }
        }
      }
    } else {
      if (pos + size_t(w) * 4 > data.size()) { if (err) *err = "hdr: truncated flat scanline"; return false; }
      std::memcpy(scan.data(), data.data() + pos, size_t(w) * 4);
      pos += size_t(w) * 4;
    }
    for (int x = 0; x < w; ++x) {
      const uint8_t* p = &scan[size_t(x) * 4];
      float* o = &rgb[(size_t(y) * w + x) * 3];
      if (p[3] == 0) {
        o[0] = o[1] = o[2] = 0.0f;
      } else {
        const float s = std::ldexp(1.0f, int(p[3]) - (128 + 8));
        o[0] = float(p[0]) * s;  // stb_image's RGBE conversion (no half-step bias)
        o[1] = float(p[1]) * s;
        o[2] = float(p[2]) * s;
      }
    }
  }
  return true;
}
