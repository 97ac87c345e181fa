// scene_desc.h — backend-agnostic scene description for the HIP backend, mirroring the reference's
// scene::SceneDesc (include/scene/SceneDesc.h:13-159) and its generators (:166-279), plus the
// world-space flattening EmbreeBackend::build performs (src/backends/EmbreeBackend.cpp:18-193),
// which defines the geomID order both CPU and GPU paths use.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../csrc/sptr_math.h"
#include "../../include/sptr_hip.h"

namespace scene {

using sptr::vec3;
struct vec2 {
  float x, y;
};
struct uvec3 {
  uint32_t x, y, z;
};

// Column-major 4x4 (m[col][row]) with glm's translate/scale/product evaluation order.
struct mat4 {
  float m[4][4];
  static mat4 identity();
};
mat4 translate(const mat4& a, vec3 v);
mat4 scale(const mat4& a, vec3 v);
mat4 multiply(const mat4& a, const mat4& b);
vec3 transform_point(const mat4& a, vec3 p);

constexpr uint32_t kNoMaterial = UINT32_MAX;

struct Material {  // SceneDesc.h:13-28 (carried, but shading reads MaterialManager — as in the reference)
  vec3 baseColor{0.8f, 0.8f, 0.8f};
  vec3 emission{0.0f, 0.0f, 0.0f};
  float metallic = 0.0f, roughness = 0.5f, ior = 1.5f, transparency = 0.0f;
};

struct SphereData {
  vec3 center{0.0f, 0.0f, 0.0f};
  float radius = 0.5f;
  uint32_t materialId = 0;
};

struct MeshData {
  std::vector<vec3> positions;
  std::vector<vec3> normals;
  std::vector<vec2> texcoords;
  std::vector<uvec3> indices;
  uint32_t materialId = 0;
  bool isValid() const { return !positions.empty() && !indices.empty(); }
  size_t triangleCount() const { return indices.size(); }
  size_t vertexCount() const { return positions.size(); }
};

struct InstanceData {
  uint32_t meshId = 0;
  mat4 worldFromObject = mat4::identity();
  uint32_t materialId = 0;
};

struct SceneDesc {
  std::vector<Material> materials;
  std::vector<MeshData> meshes;
  std::vector<InstanceData> instances;
  std::vector<SphereData> spheres;

  uint32_t addMaterial(const Material& m) { materials.push_back(m); return uint32_t(materials.size() - 1); }
  uint32_t addMesh(MeshData m) { meshes.push_back(std::move(m)); return uint32_t(meshes.size() - 1); }
  uint32_t addInstance(uint32_t mesh, const mat4& xf = mat4::identity(), uint32_t mat = 0) {
    instances.push_back(InstanceData{mesh, xf, mat});
    return uint32_t(instances.size() - 1);
  }
  uint32_t addSphere(vec3 c, float r, uint32_t mat = 0) {
    spheres.push_back(SphereData{c, r, mat});
    return uint32_t(spheres.size() - 1);
  }
  void clear() { materials.clear(); meshes.clear(); instances.clear(); spheres.clear(); }
  size_t totalTriangles() const;  // reference's estimate: sum(mesh tris) * instances
  size_t totalVertices() const;
};

MeshData createCubeMesh(uint32_t materialId = 0);
MeshData createGroundPlaneMesh(float size = 10.0f, uint32_t materialId = 0);
MeshData createSphereMesh(uint32_t stacks = 32, uint32_t slices = 64, float radius = 0.5f, uint32_t materialId = 0);

SceneDesc BuildDefaultScene();                   // SceneBuilder.cpp:9-121
SceneDesc BuildTestTriangleScene();              // SceneBuilder.cpp:126-159
// Benchmark variants: C2 adds an emissive sphere (material 9 = Materials::Light());
// C5 replaces the glass cube by createSphereMesh(stacks, slices, 0.75, 4) at (0,1,2).
SceneDesc BuildDefaultSceneWithEmitter();
SceneDesc BuildSphereMeshScene(uint32_t stacks, uint32_t slices);
// glTF 2.0 (.gltf + .bin) -> one MeshData per primitive, instanced with the node transforms
// (the role of the unwired GLTFLoader, src/GLTFLoader.cpp:24-65, 202-382).
bool LoadGLTFScene(const std::string& path, uint32_t materialId, SceneDesc& out, std::string* err);

// World-space flattening (EmbreeBackend::build): one triangle geometry per instance, then one per
// sphere.  Keeps the arrays; view() exposes them through the C ABI struct.
struct FlatScene {
  std::vector<float> positions;
  std::vector<uint32_t> indices;
  std::vector<uint32_t> tri_geom_first;
  std::vector<float> spheres;
  std::vector<uint32_t> geom_material;
  sptr_scene view() const;
};
FlatScene Flatten(const SceneDesc& s);

}  // namespace scene
