// scene_desc.cpp — SceneDesc generators, builtin scenes, glTF adapter and the EmbreeBackend-order
// flattening for the HIP backend's host layer.  Reference behaviour followed (file:line in the
// reference tree): generators SceneDesc.h:166-279; scenes SceneBuilder.cpp:9-159; flattening
// EmbreeBackend.cpp:32-193; glTF node/mesh walk GLTFLoader.cpp:24-65, 202-382.
#include "scene_desc.h"

#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>

namespace scene {

mat4 mat4::identity() {
  mat4 r{};
  for (int i = 0; i < 4; ++i) r.m[i][i] = 1.0f;
  return r;
}

mat4 translate(const mat4& a, vec3 v) {
  mat4 r = a;
  for (int k = 0; k < 4; ++k) r.m[3][k] = a.m[0][k] * v.x + a.m[1][k] * v.y + a.m[2][k] * v.z + a.m[3][k];
  return r;
}

mat4 scale(const mat4& a, vec3 v) {
  mat4 r = a;
  for (int k = 0; k < 4; ++k) {
    r.m[0][k] = a.m[0][k] * v.x;
    r.m[1][k] = a.m[1][k] * v.y;
    r.m[2][k] = a.m[2][k] * v.z;
  }
  return r;
}

// glm mat4 * mat4: column j of the result = a * b[j], each column product summed as
// (a0*b0 + a1*b1) + (a2*b2 + a3*b3).
mat4 multiply(const mat4& a, const mat4& b) {
  mat4 r{};
  for (int j = 0; j < 4; ++j)
    for (int k = 0; k < 4; ++k) {
      const float p0 = a.m[0][k] * b.m[j][0], p1 = a.m[1][k] * b.m[j][1];
      const float p2 = a.m[2][k] * b.m[j][2], p3 = a.m[3][k] * b.m[j][3];
      r.m[j][k] = (p0 + p1) + (p2 + p3);
    }
  return r;
}

vec3 transform_point(const mat4& a, vec3 p) {
  float o[3];
  for (int k = 0; k < 3; ++k) {
    const float m0 = a.m[0][k] * p.x, m1 = a.m[1][k] * p.y, m2 = a.m[2][k] * p.z, m3 = a.m[3][k] * 1.0f;
    o[k] = (m0 + m1) + (m2 + m3);
  }
  return vec3{o[0], o[1], o[2]};
}

size_t SceneDesc::totalTriangles() const {
  size_t t = 0;
  for (const MeshData& m : meshes) t += m.triangleCount();
  return t * instances.size();
}
size_t SceneDesc::totalVertices() const {
  size_t t = 0;
  for (const MeshData& m : meshes) t += m.vertexCount();
  return t;
}

MeshData createCubeMesh(uint32_t materialId) {
  MeshData m;
  m.materialId = materialId;
  const float h = 0.5f;
  for (int i = 0; i < 8; ++i) {
    // vertex order: bottom ring (-y) then top ring (+y), each (-,-) (+,-) (+,+) (-,+) in (x,z)
    const int ring = i >> 2, k = i & 3;
    const float x = (k == 1 || k == 2) ? h : -h, z = (k >= 2) ? h : -h;
    m.positions.push_back(vec3{x, ring ? h : -h, z});
  }
  const uint32_t tri[12][3] = {{0, 2, 1}, {0, 3, 2}, {4, 5, 6}, {4, 6, 7}, {0, 1, 5}, {0, 5, 4},
                               {2, 3, 7}, {2, 7, 6}, {3, 0, 4}, {3, 4, 7}, {1, 2, 6}, {1, 6, 5}};
  for (const auto& t : tri) m.indices.push_back(uvec3{t[0], t[1], t[2]});
  return m;
}

MeshData createGroundPlaneMesh(float size, uint32_t materialId) {
  MeshData m;
  m.materialId = materialId;
  const float h = size * 0.5f;
  m.positions = {vec3{-h, 0.0f, -h}, vec3{h, 0.0f, -h}, vec3{h, 0.0f, h}, vec3{-h, 0.0f, h}};
  m.normals.assign(4, vec3{0.0f, 1.0f, 0.0f});
  m.indices = {uvec3{0, 2, 1}, uvec3{0, 3, 2}};
  return m;
}

MeshData createSphereMesh(uint32_t stacks, uint32_t slices, float radius, uint32_t materialId) {
  MeshData m;
  m.materialId = materialId;
  const float PI = 3.14159265358979323846f;
  const size_t nv = size_t(stacks + 1) * (slices + 1);
  m.positions.reserve(nv);
  m.normals.reserve(nv);
  m.texcoords.reserve(nv);
  for (uint32_t a = 0; a <= stacks; ++a) {
    const float phi = PI * static_cast<float>(a) / static_cast<float>(stacks);
    const float sp = std::sin(phi), cp = std::cos(phi);
    for (uint32_t b = 0; b <= slices; ++b) {
      const float th = 2.0f * PI * static_cast<float>(b) / static_cast<float>(slices);
      const float st = std::sin(th), ct = std::cos(th);
      const vec3 p{radius * sp * ct, radius * cp, radius * sp * st};
      m.positions.push_back(p);
      m.normals.push_back(sptr::normalize(p));
      m.texcoords.push_back(vec2{static_cast<float>(b) / static_cast<float>(slices),
                                 static_cast<float>(a) / static_cast<float>(stacks)});
    }
  }
  m.indices.reserve(size_t(stacks) * slices * 2);
  for (uint32_t a = 0; a < stacks; ++a)
    for (uint32_t b = 0; b < slices; ++b) {
      const uint32_t p0 = a * (slices + 1) + b, p1 = p0 + slices + 1;
      m.indices.push_back(uvec3{p0, p1, p0 + 1});
      m.indices.push_back(uvec3{p1, p1 + 1, p0 + 1});
    }
  return m;
}

namespace {
Material mat_of(vec3 c, float metallic, float rough, float ior, float transp) {
  Material m;
  m.baseColor = c;
  m.metallic = metallic;
  m.roughness = rough;
  m.ior = ior;
  m.transparency = transp;
  return m;
}

// SceneBuilder.cpp:17-85 material list and :98-118 sphere row / glass instance
void default_scene_common(SceneDesc& s, bool sphere_mesh, uint32_t stacks, uint32_t slices) {
  s.addMaterial(mat_of(vec3{1.0f, 0.71f, 0.29f}, 1.0f, 0.05f, 1.5f, 0.0f));
  s.addMaterial(mat_of(vec3{0.95f, 0.93f, 0.88f}, 1.0f, 0.02f, 1.5f, 0.0f));
  s.addMaterial(mat_of(vec3{0.95f, 0.64f, 0.54f}, 1.0f, 0.08f, 1.5f, 0.0f));
  s.addMaterial(mat_of(vec3{0.56f, 0.57f, 0.58f}, 1.0f, 0.3f, 1.5f, 0.0f));
  s.addMaterial(mat_of(vec3{1.0f, 1.0f, 1.0f}, 0.0f, 0.0f, 1.5f, 0.95f));
  s.addMaterial(mat_of(vec3{0.8f, 0.2f, 0.2f}, 0.0f, 0.4f, 1.2f, 0.0f));
  s.addMaterial(mat_of(vec3{0.3f, 0.3f, 0.3f}, 0.0f, 0.8f, 1.1f, 0.0f));
  s.addMaterial(mat_of(vec3{0.4f, 0.25f, 0.1f}, 0.0f, 0.7f, 1.0f, 0.0f));
  s.addMaterial(mat_of(vec3{0.6f, 0.6f, 0.6f}, 0.0f, 0.9f, 1.0f, 0.0f));
  const uint32_t mesh = sphere_mesh ? s.addMesh(createSphereMesh(stacks, slices, 0.75f, 4)) : s.addMesh(createCubeMesh(0));
  struct Row {
    float x, z;
    uint32_t mat;
  };
  const Row row[8] = {{-3, 0, 0}, {-1, 0, 1}, {1, 0, 2}, {3, 0, 3}, {-2, -2, 5}, {0, -2, 6}, {2, -2, 7}, {0, -4, 8}};
  for (const Row& r : row) s.addSphere(vec3{r.x, 1.0f, r.z}, 1.0f, r.mat);
  mat4 xf = translate(mat4::identity(), vec3{0.0f, 1.0f, 2.0f});
  if (!sphere_mesh) xf = scale(xf, vec3{1.5f, 1.5f, 1.5f});
  s.addInstance(mesh, xf, 4);
}
}  // namespace

SceneDesc BuildDefaultScene() {
  SceneDesc s;
  default_scene_common(s, false, 0, 0);
  return s;
}

SceneDesc BuildDefaultSceneWithEmitter() {
  SceneDesc s;
  default_scene_common(s, false, 0, 0);
  Material e;
  e.baseColor = vec3{0.0f, 0.0f, 0.0f};
  e.emission = vec3{5.0f, 5.0f, 5.0f};
  e.roughness = 1.0f;
  s.addMaterial(e);
  s.addSphere(vec3{0.0f, 2.5f, 1.0f}, 0.5f, 9);
  return s;
}

SceneDesc BuildSphereMeshScene(uint32_t stacks, uint32_t slices) {
  SceneDesc s;
  default_scene_common(s, true, stacks, slices);
  return s;
}

SceneDesc BuildTestTriangleScene() {
  SceneDesc s;
  Material red;
  red.baseColor = vec3{1.0f, 0.0f, 0.0f};
  s.addMaterial(red);
  MeshData tri;
  tri.positions = {vec3{-1.0f, 0.0f, -3.0f}, vec3{1.0f, 0.0f, -3.0f}, vec3{0.0f, 1.0f, -3.0f}};
  tri.indices = {uvec3{0, 1, 2}};
  const uint32_t m = s.addMesh(tri);
  s.addInstance(m, mat4::identity(), 0);
  s.addInstance(m, scale(translate(mat4::identity(), vec3{1.2f, 0.0f, 0.0f}), vec3{0.5f, 0.5f, 0.5f}), 0);
  s.addSphere(vec3{0.0f, -0.5f, -3.0f}, 0.5f, 0);
  return s;
}

FlatScene Flatten(const SceneDesc& s) {
  FlatScene f;
  f.tri_geom_first.push_back(0);
  for (const InstanceData& in : s.instances) {
    if (in.meshId >= s.meshes.size()) continue;  // invalid mesh: skipped, no geomID consumed
    const MeshData& m = s.meshes[in.meshId];
    uint32_t mat = in.materialId;
    if (mat == kNoMaterial) mat = m.materialId;
    if (mat == kNoMaterial) mat = 0;
    const uint32_t base = uint32_t(f.positions.size() / 3);
    for (const vec3& p : m.positions) {
      const vec3 w = transform_point(in.worldFromObject, p);
      f.positions.insert(f.positions.end(), {w.x, w.y, w.z});
    }
    for (const uvec3& t : m.indices) f.indices.insert(f.indices.end(), {base + t.x, base + t.y, base + t.z});
    f.tri_geom_first.push_back(uint32_t(f.indices.size() / 3));
    f.geom_material.push_back(mat);
  }
  for (const SphereData& sp : s.spheres) {
    f.spheres.insert(f.spheres.end(), {sp.center.x, sp.center.y, sp.center.z, sp.radius});
    f.geom_material.push_back(sp.materialId);
  }
  return f;
}

sptr_scene FlatScene::view() const {
  sptr_scene v{};
  v.positions = positions.data();
  v.num_verts = uint32_t(positions.size() / 3);
  v.indices = indices.data();
  v.num_tris = uint32_t(indices.size() / 3);
  v.tri_geom_first = tri_geom_first.data();
  v.num_tri_geoms = uint32_t(tri_geom_first.size() - 1);
  v.spheres = spheres.data();
  v.num_spheres = uint32_t(spheres.size() / 4);
  v.geom_material = geom_material.data();
  return v;
}

// ------------------------------------------------------------------------------------- glTF
namespace {

struct Json {
  enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
  double num = 0.0;
  bool b = false;
  std::string str;
  std::vector<Json> arr;
  std::map<std::string, Json> obj;
  const Json* get(const std::string& k) const {
    if (kind != Obj) return nullptr;
    auto it = obj.find(k);
    return it == obj.end() ? nullptr : &it->second;
  }
  double num_or(const std::string& k, double d) const {
    const Json* j = get(k);
    return (j && j->kind == Num) ? j->num : d;
  }
};

struct JsonParser {
  const std::string& s;
  size_t i = 0;
  bool ok = true;
  explicit JsonParser(const std::string& src) : s(src) {}
  void ws() {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\r' || s[i] == '\t')) ++i;
  }
  Json parse() {
    ws();
    Json j;
    if (i >= s.size()) { ok = false; return j; }
    const char c = s[i];
    if (c == '{') {
      j.kind = Json::Obj;
      ++i;
      ws();
      if (i < s.size() && s[i] == '}') { ++i; return j; }
      while (ok) {
        ws();
        Json k = parse();
        if (k.kind != Json::Str) { ok = false; break; }
        ws();
        if (i >= s.size() || s[i] != ':') { ok = false; break; }
        ++i;
        j.obj[k.str] = parse();
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == '}') { ++i; break; }
        ok = false;
      }
    } else if (c == '[') {
      j.kind = Json::Arr;
      ++i;
      ws();
      if (i < s.size() && s[i] == ']') { ++i; return j; }
      while (ok) {
        j.arr.push_back(parse());
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == ']') { ++i; break; }
        ok = false;
      }
    } else if (c == '"') {
      j.kind = Json::Str;
      ++i;
      while (i < s.size() && s[i] != '"') {
        if (s[i] == '\\' && i + 1 < s.size()) {
          const char e = s[i + 1];
          j.str.push_back(e == 'n' ? '\n' : e == 't' ? '\t' : e);
          i += (e == 'u') ? 6 : 2;
        } else {
          j.str.push_back(s[i++]);
        }
      }
      ++i;
    } else if (s.compare(i, 4, "true") == 0) {
      j.kind = Json::Bool; j.b = true; i += 4;
    } else if (s.compare(i, 5, "false") == 0) {
      j.kind = Json::Bool; i += 5;
    } else if (s.compare(i, 4, "null") == 0) {
      i += 4;
    } else {
      j.kind = Json::Num;
      const char* b = s.c_str() + i;
      char* e = nullptr;
      j.num = std::strtod(b, &e);
      if (e == b) ok = false;
      i += size_t(e - b);
    }
    return j;
  }
};

mat4 quat_to_mat4(float w, float x, float y, float z) {  // glm::mat4_cast of a unit quaternion
  mat4 r = mat4::identity();
  const float xx = x * x, yy = y * y, zz = z * z, xz = x * z, xy = x * y, yz = y * z, wx = w * x, wy = w * y,
              wz = w * z;
  r.m[0][0] = 1.0f - 2.0f * (yy + zz);
  r.m[0][1] = 2.0f * (xy + wz);
  r.m[0][2] = 2.0f * (xz - wy);
  r.m[1][0] = 2.0f * (xy - wz);
  r.m[1][1] = 1.0f - 2.0f * (xx + zz);
  r.m[1][2] = 2.0f * (yz + wx);
  r.m[2][0] = 2.0f * (xz + wy);
  r.m[2][1] = 2.0f * (yz - wx);
  r.m[2][2] = 1.0f - 2.0f * (xx + yy);
  return r;
}

mat4 node_transform(const Json& node) {
  const Json* mx = node.get("matrix");
  if (mx && mx->kind == Json::Arr && mx->arr.size() == 16) {
    mat4 r{};
    for (int c = 0; c < 4; ++c)
      for (int k = 0; k < 4; ++k) r.m[c][k] = float(mx->arr[size_t(c * 4 + k)].num);
    return r;
  }
  vec3 t{0, 0, 0}, sc{1, 1, 1};
  float q[4] = {0, 0, 0, 1};
  if (const Json* j = node.get("translation"))
    if (j->arr.size() == 3) t = vec3{float(j->arr[0].num), float(j->arr[1].num), float(j->arr[2].num)};
  if (const Json* j = node.get("scale"))
    if (j->arr.size() == 3) sc = vec3{float(j->arr[0].num), float(j->arr[1].num), float(j->arr[2].num)};
  if (const Json* j = node.get("rotation"))
    if (j->arr.size() == 4)
      for (int k = 0; k < 4; ++k) q[k] = float(j->arr[size_t(k)].num);
  mat4 r = translate(mat4::identity(), t);
  r = multiply(r, quat_to_mat4(q[3], q[0], q[1], q[2]));
  return scale(r, sc);
}

struct Gltf {
  Json doc;
  std::vector<std::vector<uint8_t>> buffers;
  // returns pointer to element 0 of an accessor and its byte stride
  bool view(int acc, const uint8_t*& p, size_t& count, int& ctype, int comps, size_t& stride, std::string* err) const {
    const Json* accs = doc.get("accessors");
    if (!accs || acc < 0 || size_t(acc) >= accs->arr.size()) { if (err) *err = "gltf: bad accessor"; return false; }
    const Json& a = accs->arr[size_t(acc)];
    const int bv = int(a.num_or("bufferView", -1));
    const Json* bvs = doc.get("bufferViews");
    if (!bvs || bv < 0 || size_t(bv) >= bvs->arr.size()) { if (err) *err = "gltf: bad bufferView"; return false; }
    const Json& v = bvs->arr[size_t(bv)];
    const int b = int(v.num_or("buffer", 0));
    if (b < 0 || size_t(b) >= buffers.size()) { if (err) *err = "gltf: bad buffer"; return false; }
    ctype = int(a.num_or("componentType", 0));
    count = size_t(a.num_or("count", 0));
    const size_t csize = (ctype == 5126 || ctype == 5125) ? 4 : (ctype == 5123 ? 2 : 1);
    stride = size_t(v.num_or("byteStride", 0));
    if (stride == 0) stride = csize * size_t(comps);
    const size_t off = size_t(v.num_or("byteOffset", 0)) + size_t(a.num_or("byteOffset", 0));
    if (count && off + stride * (count - 1) + csize * size_t(comps) > buffers[size_t(b)].size()) {
      if (err) *err = "gltf: accessor out of buffer range";
      return false;
    }
    p = buffers[size_t(b)].data() + off;
    return true;
  }
};

bool walk_node(const Gltf& g, int ni, const mat4& parent, uint32_t material, SceneDesc& out, std::string* err, int depth) {
  const Json* nodes = g.doc.get("nodes");
  if (!nodes || ni < 0 || size_t(ni) >= nodes->arr.size() || depth > 64) return true;
  const Json& node = nodes->arr[size_t(ni)];
  const mat4 world = multiply(parent, node_transform(node));
  const int mi = int(node.num_or("mesh", -1));
  const Json* meshes = g.doc.get("meshes");
  if (mi >= 0 && meshes && size_t(mi) < meshes->arr.size()) {
    const Json* prims = meshes->arr[size_t(mi)].get("primitives");
    if (prims)
      for (const Json& pr : prims->arr) {
        if (int(pr.num_or("mode", 4)) != 4) continue;  // triangles only
        const Json* attrs = pr.get("attributes");
        const Json* pos = attrs ? attrs->get("POSITION") : nullptr;
        if (!pos) continue;
        MeshData m;
        m.materialId = material;
        const uint8_t* p;
        size_t cnt, stride;
        int ct;
        if (!g.view(int(pos->num), p, cnt, ct, 3, stride, err) || ct != 5126) {
          if (err && err->empty()) *err = "gltf: POSITION must be float";
          return false;
        }
        for (size_t i = 0; i < cnt; ++i) {
          float xyz[3];
          std::memcpy(xyz, p + i * stride, 12);
          m.positions.push_back(vec3{xyz[0], xyz[1], xyz[2]});
        }
        const int ia = int(pr.num_or("indices", -1));
        if (ia >= 0) {
          if (!g.view(ia, p, cnt, ct, 1, stride, err)) return false;
          std::vector<uint32_t> ix(cnt);
          for (size_t i = 0; i < cnt; ++i) {
            if (ct == 5125) { uint32_t v; std::memcpy(&v, p + i * stride, 4); ix[i] = v; }
            else if (ct == 5123) { uint16_t v; std::memcpy(&v, p + i * stride, 2); ix[i] = v; }
            else ix[i] = p[i * stride];
          }
          for (size_t i = 0; i + 2 < ix.size(); i += 3) m.indices.push_back(uvec3{ix[i], ix[i + 1], ix[i + 2]});
        } else {
          for (uint32_t i = 0; i + 2 < m.positions.size(); i += 3) m.indices.push_back(uvec3{i, i + 1, i + 2});
        }
        for (const uvec3& t : m.indices)
          if (t.x >= m.positions.size() || t.y >= m.positions.size() || t.z >= m.positions.size()) {
            if (err) *err = "gltf: index out of range";
            return false;
          }
        const uint32_t id = out.addMesh(std::move(m));
        out.addInstance(id, world, material);
      }
  }
  if (const Json* ch = node.get("children"))
    for (const Json& c : ch->arr)
      if (!walk_node(g, int(c.num), world, material, out, err, depth + 1)) return false;
  return true;
}

}  // namespace

bool LoadGLTFScene(const std::string& path, uint32_t materialId, SceneDesc& out, std::string* err) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    if (err) *err = "gltf: cannot open " + path;
    return false;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string text = ss.str();
  Gltf g;
  JsonParser jp(text);
  g.doc = jp.parse();
  if (!jp.ok || g.doc.kind != Json::Obj) {
    if (err) *err = "gltf: JSON parse error";
    return false;
  }
  const std::string dir = path.find('/') == std::string::npos ? std::string() : path.substr(0, path.rfind('/') + 1);
  if (const Json* bufs = g.doc.get("buffers"))
    for (const Json& b : bufs->arr) {
      const Json* uri = b.get("uri");
      if (!uri || uri->kind != Json::Str || uri->str.rfind("data:", 0) == 0) {
        if (err) *err = "gltf: only external .bin buffers are supported";
        return false;
      }
      std::ifstream bf(dir + uri->str, std::ios::binary);
      if (!bf) {
        if (err) *err = "gltf: cannot open buffer " + uri->str;
        return false;
      }
      std::vector<uint8_t> data((std::istreambuf_iterator<char>(bf)), std::istreambuf_iterator<char>());
      g.buffers.push_back(std::move(data));
    }
  // every scene's root nodes, as GLTFLoader::loadGLTF walks model.scenes (GLTFLoader.cpp:57-62)
  if (const Json* scenes = g.doc.get("scenes"))
    for (const Json& sc : scenes->arr)
      if (const Json* roots = sc.get("nodes"))
        for (const Json& r : roots->arr)
          if (!walk_node(g, int(r.num), mat4::identity(), materialId, out, err, 0)) return false;
  if (out.meshes.empty()) {
    if (err) *err = "gltf: no triangle meshes";
    return false;
  }
  return true;
}

}  // namespace scene
