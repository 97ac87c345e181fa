// shading.h — host-side L2 state the backend consumes, mirroring the reference's interfaces:
//   Camera              include/Camera.h:6-74        (basis math: src/Camera.cpp:5-50, 95-106)
//   Material/Materials  include/Material.h:19-147    (presets used by MaterialManager)
//   MaterialManager     include/MaterialManager.h:8-48, src/MaterialManager.cpp:13-103
//   Light/LightManager  include/Light.h:8-104, src/Light.cpp:43-135
//   EnvironmentManager  include/EnvironmentManager.h:8-46 (cubemap faces from an equirect HDR:
//                       src/Cubemap.cpp:18-46, 252-345)
// Only state and host math live here; shading itself runs in the HIP kernels.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../csrc/sptr_math.h"
#include "../../include/sptr_hip.h"

using sptr::vec3;

class Camera {
 public:
  Camera(const vec3& position, const vec3& target, const vec3& up = vec3{0.0f, 1.0f, 0.0f}, float fov = 45.0f,
         float aspect_ratio = 1.0f);
  vec3 getRayDirection(float x, float y) const;
  enum Movement { FORWARD = 0, BACKWARD = 1, LEFT = 2, RIGHT = 3 };
  void processKeyboard(int direction, float deltaTime);
  void processMouseMovement(float xoffset, float yoffset, bool constrainPitch = true);
  void setPosition(const vec3& position);
  void setAspectRatio(float aspect_ratio);
  bool hasMovedSinceLastCheck(float position_threshold = 0.001f, float rotation_threshold = 0.1f);
  const vec3& getPosition() const { return pos_; }
  const vec3& getFront() const { return fwd_; }
  const vec3& getRight() const { return right_; }
  const vec3& getUp() const { return up_; }
  float getYaw() const { return yaw_; }
  float getPitch() const { return pitch_; }
  float getHalfWidth() const { return half_w_; }
  float getHalfHeight() const { return half_h_; }
  sptr_camera toDevice() const;

 private:
  void update();
  vec3 pos_, target_, world_up_;  // world_up_ kept for interface parity (the basis uses +Y)
  float fov_, aspect_;
  vec3 fwd_{0, 0, -1}, right_{1, 0, 0}, up_{0, 1, 0};
  float half_w_ = 1.0f, half_h_ = 1.0f;
  float yaw_ = 0.0f, pitch_ = 0.0f, speed_ = 2.5f, sensitivity_ = 0.1f;
  vec3 last_pos_;
  float last_yaw_ = 0.0f, last_pitch_ = 0.0f;
  bool first_check_ = true;
};

enum class MaterialType : int { PBR = 0, DIELECTRIC = 1 };

struct Material {
  vec3 albedo;
  float metallic;
  float roughness;
  vec3 emission;
  float ior;
  MaterialType materialType;
  explicit Material(const vec3& albedo_ = vec3{0.5f, 0.5f, 0.5f}, float metallic_ = 0.0f, float roughness_ = 0.5f,
                    const vec3& emission_ = vec3{0.0f, 0.0f, 0.0f}, float ior_ = 1.5f,
                    MaterialType type_ = MaterialType::PBR);
  bool isTransparent() const { return metallic < 0.1f && ior > 1.3f; }
  float getTransparency() const;
  sptr_material toDevice() const;
};

namespace Materials {
Material Gold();
Material Silver();
Material Copper();
Material Iron();
Material Plastic();
Material Rubber();
Material Glass();
Material ClearGlass();
Material Wood();
Material Concrete();
Material Light(const vec3& color = vec3{1.0f, 1.0f, 1.0f}, float intensity = 5.0f);
}  // namespace Materials

class MaterialManager {
 public:
  MaterialManager();  // the nine presets of setupDefaultMaterials
  void addMaterial(const Material& m) { mats_.push_back(m); }
  void setMaterial(int index, const Material& m);
  const Material& getMaterial(int index) const;
  int getMaterialCount() const { return int(mats_.size()); }
  void setGeomMaterialMapping(const std::vector<uint32_t>& m) { geom_mat_ = m; }
  const std::vector<uint32_t>& getGeomMaterialMapping() const { return geom_mat_; }
  void buildDeviceMaterials(std::vector<sptr_material>& out) const;

 private:
  std::vector<Material> mats_;
  std::vector<uint32_t> geom_mat_;
};

class Light {
 public:
  enum Type { DIRECTIONAL, POINT, AREA };
  Light(Type t, const vec3& color, float intensity) : type_(t), color_(color), intensity_(intensity) {}
  virtual ~Light() = default;
  Type getType() const { return type_; }
  const vec3& getColor() const { return color_; }
  float getIntensity() const { return intensity_; }
  void setColor(const vec3& c) { color_ = c; }
  void setIntensity(float i) { intensity_ = i; }
  virtual sptr_light toDevice() const = 0;

 protected:
  Type type_;
  vec3 color_;
  float intensity_;
};

class DirectionalLight : public Light {
 public:
  DirectionalLight(const vec3& direction, const vec3& color, float intensity);
  const vec3& getDirection() const { return to_light_; }  // direction TO the light
  sptr_light toDevice() const override;

 private:
  vec3 given_;     // as passed in (direction of the light's rays)
  vec3 to_light_;  // normalize(-given)
};

class PointLight : public Light {
 public:
  PointLight(const vec3& position, const vec3& color, float intensity) : Light(POINT, color, intensity), pos_(position) {}
  const vec3& getPosition() const { return pos_; }
  sptr_light toDevice() const override;

 private:
  vec3 pos_;
};

class LightManager {
 public:
  void addDirectionalLight(const vec3& direction, const vec3& color, float intensity);
  void addPointLight(const vec3& position, const vec3& color, float intensity);
  size_t getLightCount() const { return lights_.size(); }
  const Light& getLight(size_t i) const { return *lights_.at(i); }
  void clearLights() { lights_.clear(); }
  void buildDeviceLights(std::vector<sptr_light>& out) const;

 private:
  std::vector<std::unique_ptr<Light>> lights_;
};

class EnvironmentManager {
 public:
  // .hdr (Radiance RGBE) equirectangular -> six 512x512 faces (Cubemap::loadEquirectangular)
  bool loadCubemap(const std::string& filename, std::string* err = nullptr);
  // synthetic or decoded equirect RGB float data
  void setEquirectangular(const float* rgb, int w, int h, int face_size = 512);
  bool hasCubemap() const { return size_ > 0; }
  int faceSize() const { return size_; }
  const std::vector<float>& faces() const { return faces_; }
  float getEnvironmentIntensity() const { return intensity_; }
  float getEnvironmentMaxClamp() const { return max_clamp_; }
  sptr_environment toDevice() const;

 private:
  std::vector<float> faces_;
  int size_ = 0;
  float intensity_ = 0.8f, max_clamp_ = 5.0f;
};

// Radiance .hdr reader (new-style RLE and flat scanlines) -> RGB float, top row first.
bool LoadRadianceHDR(const std::string& path, std::vector<float>& rgb, int& w, int& h, std::string* err);
// Cubemap::loadEquirectangular face construction (nearest lookup)
void EquirectToFaces(const float* rgb, int w, int h, int size, float* faces);
