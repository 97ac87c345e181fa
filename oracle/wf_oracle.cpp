// =====================================================================================================
//  oracle/wf_oracle.cpp — TEST INFRASTRUCTURE ONLY (never linked into, loaded by, or called from the
//  product library).  Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
//
//  A plain-C++ restatement of the reference's CPU "Embree" wavefront path tracer
//  (yangyonggit/simple-path-tracer), written from reading the reference sources — not copied:
//    scene    : include/scene/SceneDesc.h:166-279, src/scene/SceneBuilder.cpp:9-159
//    flatten  : src/backends/EmbreeBackend.cpp:18-193 (geomID order: instances, then spheres)
//    spheres  : src/backends/EmbreeBackend.cpp:223-314 (user-geometry intersect / occluded)
//    triangles: Embree 4 (third-party, version unpinned by the reference's vcpkg setup) default
//               Moeller-Trumbore intersector, restated from its published algorithm (see tri_hit)
//    camera   : src/Camera.cpp:5-50, 95-106 ; src/main.cpp:85-113
//    seeding  : src/GLRenderer.cpp:353-435 (renderWavefrontTileTask)
//    integrate: src/wavefront/wf_pt_cpu.cpp:28-255, include/wavefront/wf_math.h:28-100
//    BRDF     : src/Material.cpp:32-117, include/Material.h:19-147, src/MaterialManager.cpp:21-103
//    lights   : src/Light.cpp:16-55
//    env      : src/EnvironmentManager.cpp:9-74, src/Cubemap.cpp:82-180, 252-345
//    PathTracer mode: src/PathTracer.cpp:59-75, 82-111, 113-224, 280-303, 331-406 (the reference's
//               default CPU integrator; its mt19937(random_device) is replaced by the same
//               deterministic per-(pixel, frame, sample) wang-hash stream as the product's pt_seed)
//    OptiX mode: src/optix/device_programs.cu:78-218 (helpers), 220-274 (raygen), 297-309 (trace),
//               315-690 (shade), 761-820 (closest hit), 854-899 (resolve); camera basis and light from
//               src/backends/OptixBackend.cpp:1515-1620 (correctly rounded normalize for rsqrtf)
//
//  PARITY UNPINNED: the reference ships no tests, golden images or known-answer vectors for this
//  path and cannot be compiled here (Embree, glm, TBB, OptiX absent), so this
//  restatement is checked only for internal consistency (brute force vs BVH, analytic cases).
//
//  Numerics: compiled with -ffp-contract=off; glm semantics restated by hand (normalize = v*(1/sqrt),
//  reflect = I - N*dot(N,I)*2, mix = x*(1-a)+y*a, clamp = min(max)).  The reference targets MSVC,
//  whose <cmath> resolves unqualified float math calls (pow/atan2/...) to the float overloads; we do
//  the same.  Embree's triangle test uses FMA (madd/msub) in AVX2 builds; restated with fmaf.
// =====================================================================================================
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <thread>
#include <vector>

namespace orc {

// ----------------------------------------------------------------------------- vector (glm-like)
struct V3 {
  float x, y, z;
};
static inline V3 mk(float x, float y, float z) { return V3{x, y, z}; }
static inline V3 operator+(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 operator-(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 operator-(V3 a) { return mk(-a.x, -a.y, -a.z); }
static inline V3 operator*(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 operator*(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline V3 operator*(float s, V3 a) { return mk(s * a.x, s * a.y, s * a.z); }
static inline V3 operator/(V3 a, V3 b) { return mk(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline V3 operator/(V3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
static inline V3 operator+(V3 a, float s) { return mk(a.x + s, a.y + s, a.z + s); }
static inline V3 operator-(float s, V3 a) { return mk(s - a.x, s - a.y, s - a.z); }
static inline float gmax(float a, float b) { return (a < b) ? b : a; }  // glm::max / std::max
static inline float gmin(float a, float b) { return (b < a) ? b : a; }  // glm::min / std::min
static inline float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }
static inline V3 gclamp(V3 v, float lo, float hi) { return mk(gclamp(v.x, lo, hi), gclamp(v.y, lo, hi), gclamp(v.z, lo, hi)); }
static inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline V3 cross(V3 a, V3 b) { return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
static inline V3 normalize(V3 v) { return v * (1.0f / std::sqrt(dot(v, v))); }
static inline V3 safe_normalize(V3 v) {
  const float l2 = dot(v, v);
  if (l2 <= 0.0f) return mk(0, 0, 0);
  return v * (1.0f / std::sqrt(l2));
}
static inline V3 reflect(V3 i, V3 n) { return i - n * dot(n, i) * 2.0f; }
static inline V3 mix(V3 a, V3 b, float t) { return a * (1.0f - t) + b * t; }
static inline float degrees_f(float r) { return r * 57.295779513082320876798154814105f; }
static inline float radians_f(float d) { return d * 0.01745329251994329576923690768489f; }
static const float kPiF = 3.14159265358979323846264338327950288f;

// ----------------------------------------------------------------------------- RNG (wf_math.h:35-49)
static inline uint32_t wang_hash(uint32_t a) {
  a = (a ^ 61u) ^ (a >> 16u);
  a *= 9u;
  a = a ^ (a >> 4u);
  a *= 0x27d4eb2du;
  a = a ^ (a >> 15u);
  return a;
}
static inline float rand01(uint32_t& s) {
  s = wang_hash(s);
  return float(s & 0x00FFFFFFu) / float(0x01000000u);
}

// Residue diagnosis (parity tests only; off by default): the GPU's values in place of glibc's for the
// operations of the wavefront path whose last bit depends on the math library or on its form —
//   sin_cos : (sinf, cosf) of the cosine sample's phi for each of the 2^24 values r1 = k / 2^24 takes
//             (wf_math.h:51-72), as the device computes them (sptr_eval_math);
//   pow_chains: pow(x, 5) / pow(x, 8) / pow(x, 64) as the device's squaring chains in double (one
//             rounding to float; glibc's powf is correctly rounded, the chains differ from it only
//             within ~6 2^-53 of a rounding midpoint).
// With both set, a GPU/oracle pixel difference that remains is not a math-library difference.
struct DevMath {
  const float* sin_cos = nullptr;  // 2^24 pairs
  bool pow_chains = false;
};
static DevMath g_devmath;
static inline void cosine_sincos(float r1, float& sp, float& cp) {
  const float phi = 2.0f * 3.14159265358979323846f * r1;
  if (g_devmath.sin_cos) {
    const uint32_t k = uint32_t(r1 * 16777216.0f);  // exact: r1 = k / 2^24
    sp = g_devmath.sin_cos[2u * k];
    cp = g_devmath.sin_cos[2u * k + 1u];
    return;
  }
  sp = std::sin(phi);
  cp = std::cos(phi);
}
static inline float pow_int(float x, float e) {  // e in {5, 8, 64}
  if (!g_devmath.pow_chains) return std::pow(x, e);
  const double s = double(x), s2 = s * s, s4 = s2 * s2;
  if (e == 5.0f) return float(s4 * s);
  const double s8 = s4 * s4;
  if (e == 8.0f) return float(s8);
  const double s16 = s8 * s8, s32 = s16 * s16;
  return float(s32 * s32);
}

// ----------------------------------------------------------------------------- scene description
struct Mat4 {  // column-major, m[col][row]
  float m[4][4];
};
static Mat4 identity4() {
  Mat4 r{};
  for (int i = 0; i < 4; ++i) r.m[i][i] = 1.0f;
  return r;
}
static Mat4 translate4(const Mat4& a, V3 v) {  // glm::translate
  Mat4 r = a;
  for (int k = 0; k < 4; ++k) r.m[3][k] = a.m[0][k] * v.x + a.m[1][k] * v.y + a.m[2][k] * v.z + a.m[3][k];
  return r;
}
static Mat4 scale4(const Mat4& a, V3 v) {  // glm::scale
  Mat4 r = a;
  for (int k = 0; k < 4; ++k) {
    r.m[0][k] = a.m[0][k] * v.x;
    r.m[1][k] = a.m[1][k] * v.y;
    r.m[2][k] = a.m[2][k] * v.z;
  }
  return r;
}
static V3 xform_point(const Mat4& a, V3 p) {  // glm mat4*vec4 evaluation order
  float o[3];
  for (int k = 0; k < 3; ++k) {
    const float m0 = a.m[0][k] * p.x, m1 = a.m[1][k] * p.y, m2 = a.m[2][k] * p.z, m3 = a.m[3][k] * 1.0f;
    o[k] = (m0 + m1) + (m2 + m3);
  }
  return mk(o[0], o[1], o[2]);
}

struct Mesh {
  std::vector<V3> pos;
  std::vector<uint32_t> idx;  // 3 per triangle
  uint32_t material = 0;
};
struct Instance {
  uint32_t mesh;
  Mat4 xf;
  uint32_t material;
};
struct Sphere {
  V3 c;
  float r;
  uint32_t material;
};
struct SceneDesc {
  std::vector<Mesh> meshes;
  std::vector<Instance> instances;
  std::vector<Sphere> spheres;
};

static Mesh cube_mesh(uint32_t mat) {  // SceneDesc.h:166-190
  Mesh m;
  m.material = mat;
  const float h = 0.5f;
  m.pos = {mk(-h, -h, -h), mk(h, -h, -h), mk(h, -h, h), mk(-h, -h, h),
           mk(-h, h, -h),  mk(h, h, -h),  mk(h, h, h),  mk(-h, h, h)};
  m.idx = {0, 2, 1, 0, 3, 2, 4, 5, 6, 4, 6, 7, 0, 1, 5, 0, 5, 4,
           2, 3, 7, 2, 7, 6, 3, 0, 4, 3, 4, 7, 1, 2, 6, 1, 6, 5};
  return m;
}

static Mesh uv_sphere_mesh(uint32_t stacks, uint32_t slices, float radius, uint32_t mat) {  // SceneDesc.h:225-279
  Mesh m;
  m.material = mat;
  const float PI = 3.14159265358979323846f;
  m.pos.reserve(size_t(stacks + 1) * (slices + 1));
  for (uint32_t a = 0; a <= stacks; ++a) {
    const float phi = PI * static_cast<float>(a) / static_cast<float>(stacks);
    const float sp = std::sin(phi), cp = std::cos(phi);
    for (uint32_t b = 0; b <= slices; ++b) {
      const float th = 2.0f * PI * static_cast<float>(b) / static_cast<float>(slices);
      const float st = std::sin(th), ct = std::cos(th);
      m.pos.push_back(mk(radius * sp * ct, radius * cp, radius * sp * st));
    }
  }
  m.idx.reserve(size_t(stacks) * slices * 6);
  for (uint32_t a = 0; a < stacks; ++a)
    for (uint32_t b = 0; b < slices; ++b) {
      const uint32_t p0 = a * (slices + 1) + b, p1 = p0 + slices + 1;
      const uint32_t t[6] = {p0, p1, p0 + 1, p1, p1 + 1, p0 + 1};
      m.idx.insert(m.idx.end(), t, t + 6);
    }
  return m;
}

// Builtin scenes.  0 = BuildDefaultScene; 1 = default + emitter sphere (material 9 = Materials::Light);
// 2 = default with the glass cube replaced by a UV-sphere mesh (stacks, slices; r 0.75 at (0,1,2));
// 3 = BuildTestTriangleScene.
static SceneDesc builtin_scene(int which, uint32_t stacks, uint32_t slices) {
  SceneDesc s;
  if (which == 3) {  // SceneBuilder.cpp:126-159
    Mesh tri;
    tri.material = 0;
    tri.pos = {mk(-1, 0, -3), mk(1, 0, -3), mk(0, 1, -3)};
    tri.idx = {0, 1, 2};
    s.meshes.push_back(tri);
    s.instances.push_back({0, identity4(), 0});
    s.instances.push_back({0, scale4(translate4(identity4(), mk(1.2f, 0, 0)), mk(0.5f, 0.5f, 0.5f)), 0});
    s.spheres.push_back({mk(0.0f, -0.5f, -3.0f), 0.5f, 0});
    return s;
  }
  // SceneBuilder.cpp:98-118 — sphere row layout and material ids
  if (which == 2) s.meshes.push_back(uv_sphere_mesh(stacks, slices, 0.75f, 4));
  else s.meshes.push_back(cube_mesh(0));
  const float sx[8] = {-3, -1, 1, 3, -2, 0, 2, 0};
  const float sz[8] = {0, 0, 0, 0, -2, -2, -2, -4};
  const uint32_t sm[8] = {0, 1, 2, 3, 5, 6, 7, 8};
  for (int i = 0; i < 8; ++i) s.spheres.push_back({mk(sx[i], 1.0f, sz[i]), 1.0f, sm[i]});
  if (which == 2) {
    s.instances.push_back({0, translate4(identity4(), mk(0, 1, 2)), 4});
  } else {
    s.instances.push_back({0, scale4(translate4(identity4(), mk(0, 1, 2)), mk(1.5f, 1.5f, 1.5f)), 4});
  }
  if (which == 1) s.spheres.push_back({mk(0.0f, 2.5f, 1.0f), 0.5f, 9});
  return s;
}

// Flattened world-space scene, geomID order of EmbreeBackend::build (instances first, then spheres).
struct Flat {
  std::vector<float> positions;        // xyz per vertex
  std::vector<uint32_t> indices;       // 3 per triangle (global vertex ids)
  std::vector<uint32_t> tri_geom_first;  // prefix over triangle geometries (size G+1)
  std::vector<float> spheres;          // cx cy cz r
  std::vector<uint32_t> geom_material;  // per geomID
};

static Flat flatten(const SceneDesc& s) {
  Flat f;
  f.tri_geom_first.push_back(0);
  for (const Instance& in : s.instances) {
    if (in.mesh >= s.meshes.size()) continue;  // EmbreeBackend.cpp:42-46
    const Mesh& m = s.meshes[in.mesh];
    uint32_t mat = in.material;
    if (mat == UINT32_MAX) mat = m.material;
    if (mat == UINT32_MAX) mat = 0;
    const uint32_t base = uint32_t(f.positions.size() / 3);
    for (const V3& p : m.pos) {
      const V3 w = xform_point(in.xf, p);
      f.positions.push_back(w.x);
      f.positions.push_back(w.y);
      f.positions.push_back(w.z);
    }
    for (uint32_t i : m.idx) f.indices.push_back(base + i);
    f.tri_geom_first.push_back(uint32_t(f.indices.size() / 3));
    f.geom_material.push_back(mat);
  }
  for (const Sphere& sp : s.spheres) {
    f.spheres.push_back(sp.c.x);
    f.spheres.push_back(sp.c.y);
    f.spheres.push_back(sp.c.z);
    f.spheres.push_back(sp.r);
    f.geom_material.push_back(sp.material);
  }
  return f;
}

// ----------------------------------------------------------------------------- materials / lights
struct Material {
  V3 albedo;
  float metallic, roughness;
  V3 emission;
  float ior;
  int type;
};
static Material make_material(V3 a, float m, float r, V3 e = mk(0, 0, 0), float ior = 1.5f, int type = 0) {
  Material x{a, m, r, e, ior, type};  // Material.h:28-39 ctor clamps
  x.metallic = gclamp(x.metallic, 0.0f, 1.0f);
  x.roughness = gclamp(x.roughness, 0.01f, 1.0f);
  return x;
}
// MaterialManager::setupDefaultMaterials (MaterialManager.cpp:21-52) presets (Material.h:99-147)
static std::vector<Material> preset_materials(bool with_light) {
  std::vector<Material> v;
  v.push_back(make_material(mk(1.0f, 0.71f, 0.29f), 1.0f, 0.05f));            // gold
  v.push_back(make_material(mk(0.95f, 0.93f, 0.88f), 1.0f, 0.02f));           // silver
  v.push_back(make_material(mk(0.95f, 0.64f, 0.54f), 1.0f, 0.08f));           // copper
  v.push_back(make_material(mk(0.56f, 0.57f, 0.58f), 1.0f, 0.3f));            // iron
  v.push_back(make_material(mk(1, 1, 1), 0.0f, 0.0f, mk(0, 0, 0), 1.5f, 1));  // glass
  v.push_back(make_material(mk(0.8f, 0.2f, 0.2f), 0.0f, 0.4f, mk(0, 0, 0), 1.2f));  // plastic
  v.push_back(make_material(mk(0.3f, 0.3f, 0.3f), 0.0f, 0.8f, mk(0, 0, 0), 1.1f));  // rubber
  v.push_back(make_material(mk(0.4f, 0.25f, 0.1f), 0.0f, 0.7f, mk(0, 0, 0), 1.0f));  // wood
  v.push_back(make_material(mk(0.6f, 0.6f, 0.6f), 0.0f, 0.9f, mk(0, 0, 0), 1.0f));   // concrete
  if (with_light) v.push_back(make_material(mk(0, 0, 0), 0.0f, 1.0f, mk(1, 1, 1) * 5.0f));  // Materials::Light()
  return v;
}
static inline bool is_transparent(const Material& m) { return m.metallic < 0.1f && m.ior > 1.3f; }
static inline float transparency(const Material& m) {
  return is_transparent(m) ? gclamp((m.ior - 1.0f) / 0.7f, 0.0f, 0.95f) : 0.0f;
}

// Material::evaluateBRDF (Material.cpp:84-117).  M_PI is a double in the reference: the GGX
// denominator `M_PI * denom * denom` is evaluated in double and rounded once to float.
static V3 eval_brdf(const Material& m, V3 N, V3 V, V3 L) {
  const V3 H = normalize(V + L);
  const float NdotV = gmax(dot(N, V), 0.0f);
  const float NdotL = gmax(dot(N, L), 0.0f);
  const float HdotV = gmax(dot(H, V), 0.0f);
  const float r = gclamp(m.roughness, 0.02f, 1.0f);
  const float alpha = r * r;
  // D
  const float a2 = alpha * alpha;
  const float NdotH = gmax(dot(N, H), 0.0f);
  const float NdotH2 = NdotH * NdotH;
  float dden = (NdotH2 * (a2 - 1.0f) + 1.0f);
  dden = float(3.14159265358979323846 * double(dden) * double(dden));
  const float D = a2 / dden;
  // G (Smith, k from r = sqrt(alpha))
  const float rr = gclamp(std::sqrt(gmax(alpha, 0.0f)), 0.02f, 1.0f);
  const float kq = (rr + 1.0f);
  const float k = (kq * kq) / 8.0f;
  const float g_v = NdotV / (NdotV * (1.0f - k) + k);
  const float g_l = NdotL / (NdotL * (1.0f - k) + k);
  const float G = g_l * g_v;
  // F (Schlick, F0 = mix(f0_dielectric, albedo, metallic))
  float f0d = (m.ior - 1.0f) / (m.ior + 1.0f);
  f0d *= f0d;
  const V3 F0 = mix(mk(f0d, f0d, f0d), m.albedo, m.metallic);
  const float pw = pow_int(gclamp(1.0f - HdotV, 0.0f, 1.0f), 5.0f);
  const V3 F = F0 + (1.0f - F0) * pw;
  const V3 numer = (D * G) * F;
  const float denom = 4.0f * NdotV * NdotL + 0.0001f;
  const V3 spec = numer / denom;
  const V3 kD = 1.0f - F;
  const V3 diffuse = (m.albedo * (1.0f - m.metallic)) / float(3.14159265358979323846);
  return (kD * diffuse + spec) * NdotL;
}

struct Light {
  int type;  // 0 directional, 1 point
  V3 v;      // as given to LightManager::add*: direction of light rays, or position
  V3 color;
  float intensity;
};
// Light::getRadiance (Light.cpp:43-79)
static V3 light_radiance(const Light& l, V3 p, V3& to_light, float& dist) {
  if (l.type == 0) {
    to_light = normalize(-l.v);
    dist = std::numeric_limits<float>::infinity();
    return l.color * l.intensity;
  }
  const V3 lv = l.v - p;
  dist = std::sqrt(dot(lv, lv));
  to_light = lv / dist;
  const float att = 1.0f + 0.09f * dist + 0.032f * dist * dist;
  return (l.color * l.intensity) / att;
}

// ----------------------------------------------------------------------------- environment
struct Env {
  const float* faces = nullptr;  // 6 * S * S * 3, order +X,-X,+Y,-Y,+Z,-Z
  int size = 0;
  float intensity = 0.8f, max_clamp = 5.0f;
};
static V3 sky(V3 d) {  // EnvironmentManager::getSkyColor (EnvironmentManager.cpp:35-61)
  float t = 0.5f * (d.y + 1.0f);
  {
    const float u = gclamp((t - 0.0f) / (1.0f - 0.0f), 0.0f, 1.0f);
    t = u * u * (3.0f - 2.0f * u);
  }
  V3 c = mix(mk(0.7f, 0.8f, 0.9f), mk(0.2f, 0.4f, 0.8f), t);
  const V3 sd = normalize(mk(0.3f, 0.6f, -0.8f));
  const float sdot = gmax(dot(d, sd), 0.0f);
  const float si = pow_int(sdot, 64.0f);
  const float sg = pow_int(sdot, 8.0f) * 0.3f;
  c = c + mk(1.0f, 0.9f, 0.7f) * (si + sg);
  return c * 0.8f;
}
static void dir_to_face_uv(V3 dir, int& face, float& u, float& v) {  // Cubemap::directionToUV
  const V3 d = normalize(dir);
  const float ax = std::fabs(d.x), ay = std::fabs(d.y), az = std::fabs(d.z);
  float ma, uc, vc;
  if (ax >= ay && ax >= az) {
    ma = ax;
    if (d.x > 0) { face = 0; uc = -d.z; vc = -d.y; }
    else         { face = 1; uc = d.z;  vc = -d.y; }
  } else if (ay >= ax && ay >= az) {
    ma = ay;
    if (d.y > 0) { face = 2; uc = d.x; vc = d.z; }
    else         { face = 3; uc = d.x; vc = -d.z; }
  } else {
    ma = az;
    if (d.z > 0) { face = 4; uc = d.x;  vc = -d.y; }
    else         { face = 5; uc = -d.x; vc = -d.y; }
  }
  u = gclamp((uc / ma + 1.0f) * 0.5f, 0.0f, 1.0f);
  v = gclamp((vc / ma + 1.0f) * 0.5f, 0.0f, 1.0f);
}
static V3 texel(const Env& e, int face, int x, int y) {
  const float* p = e.faces + ((size_t(face) * e.size + y) * e.size + x) * 3;
  return mk(p[0], p[1], p[2]);
}
static V3 env_color(const Env& e, V3 dir) {
  if (!e.faces) return sky(dir);
  int face;
  float u, v;
  dir_to_face_uv(dir, face, u, v);
  const float fx_ = u * float(e.size - 1), fy_ = v * float(e.size - 1);
  const int x0 = int(std::floor(fx_)), y0 = int(std::floor(fy_));
  const int x1 = std::min(x0 + 1, e.size - 1), y1 = std::min(y0 + 1, e.size - 1);
  const float fx = fx_ - float(x0), fy = fy_ - float(y0);
  const V3 c0 = mix(texel(e, face, x0, y0), texel(e, face, x1, y0), fx);
  const V3 c1 = mix(texel(e, face, x0, y1), texel(e, face, x1, y1), fx);
  V3 c = mix(c0, c1, fy);
  c = mk(gmin(c.x, e.max_clamp), gmin(c.y, e.max_clamp), gmin(c.z, e.max_clamp));
  return c * e.intensity;
}

// ----------------------------------------------------------------------------- intersection
static inline float madd(float a, float b, float c) { return std::fma(a, b, c); }
static inline float msub(float a, float b, float c) { return std::fma(a, b, -c); }
static inline V3 e_cross(V3 a, V3 b) {
  return mk(msub(a.y, b.z, a.z * b.y), msub(a.z, b.x, a.x * b.z), msub(a.x, b.y, a.y * b.x));
}
static inline float e_dot(V3 a, V3 b) { return madd(a.x, b.x, madd(a.y, b.y, a.z * b.z)); }
static inline float xorsign(float x, float s) {
  uint32_t a, b;
  std::memcpy(&a, &x, 4);
  std::memcpy(&b, &s, 4);
  a ^= (b & 0x80000000u);
  std::memcpy(&x, &a, 4);
  return x;
}

// Embree's default (non-robust) Moeller-Trumbore triangle test: e1 = v0-v1, e2 = v2-v0,
// Ng = cross(e2,e1); hit iff den != 0, U,V >= 0, U+V <= |den|, tnear*|den| < T <= tfar*|den|.
static inline bool tri_hit(V3 v0, V3 v1, V3 v2, V3 O, V3 D, float tnear, float tfar, float& t, V3& Ng) {
  const V3 e1 = v0 - v1, e2 = v2 - v0;
  const V3 ng = e_cross(e2, e1);
  const V3 C = v0 - O;
  const V3 R = e_cross(C, D);
  const float den = e_dot(ng, D);
  const float aden = std::fabs(den);
  const float U = xorsign(e_dot(R, e2), den);
  const float V = xorsign(e_dot(R, e1), den);
  if (!(den != 0.0f && U >= 0.0f && V >= 0.0f && U + V <= aden)) return false;
  const float T = xorsign(e_dot(ng, C), den);
  if (!(aden * tnear < T && T <= aden * tfar)) return false;
  t = T / aden;
  Ng = ng;
  return true;
}

// sphereIntersectFunc (EmbreeBackend.cpp:223-282) — quadratic in the reference's evaluation order.
static inline bool sphere_roots(const float* s, V3 O, V3 D, float& t1, float& t2) {
  const float ox = O.x - s[0], oy = O.y - s[1], oz = O.z - s[2];
  const float a = D.x * D.x + D.y * D.y + D.z * D.z;
  const float b = 2.0f * (ox * D.x + oy * D.y + oz * D.z);
  const float c = ox * ox + oy * oy + oz * oz - s[3] * s[3];
  const float disc = b * b - 4.0f * a * c;
  if (!(disc >= 0.0f)) return false;
  const float sq = std::sqrt(disc);
  t1 = (-b - sq) / (2.0f * a);
  t2 = (-b + sq) / (2.0f * a);
  return true;
}
static inline bool sphere_hit(const float* s, V3 O, V3 D, float tnear, float tfar, float& t, V3& Ng) {
  float t1, t2;
  if (!sphere_roots(s, O, D, t1, t2)) return false;
  float tt = -1.0f;
  if (t1 > tnear && t1 < tfar) tt = t1;
  else if (t2 > tnear && t2 < tfar) tt = t2;
  if (!(tt > 0.0f && tt < tfar)) return false;
  t = tt;
  const float hx = O.x + tt * D.x, hy = O.y + tt * D.y, hz = O.z + tt * D.z;
  Ng = mk((hx - s[0]) / s[3], (hy - s[1]) / s[3], (hz - s[2]) / s[3]);
  return true;
}
static inline bool sphere_occludes(const float* s, V3 O, V3 D, float tnear, float tfar) {
  float t1, t2;
  if (!sphere_roots(s, O, D, t1, t2)) return false;
  return (t1 > tnear && t1 < tfar) || (t2 > tnear && t2 < tfar);
}

// Prepared scene: flattened arrays + a CPU BVH (binned SAH, as Embree's builders are SAH-based).
// The BVH only prunes work: the closest hit equals the brute-force result (exact ties excepted),
// which tests check.  Children of an internal node are adjacent (left, left + 1).
struct Node {
  float lo[3], hi[3];
  uint32_t left, count;  // count>0: leaf over refs[left .. left+count)
  uint32_t axis, pad;    // split axis of an internal node (front-to-back order)
};
struct Prepared {
  std::vector<float> pos;
  std::vector<uint32_t> idx, geom_first, geom_material;
  std::vector<float> sph;
  uint32_t ntri = 0, nsph = 0, ngeom_tri = 0;
  std::vector<uint32_t> tri_geom;  // per triangle geomID
  std::vector<uint32_t> refs;      // prim refs: tri index, or (1u<<31)|sphere index
  std::vector<Node> nodes;
};

static void ref_bounds(const Prepared& P, uint32_t r, float lo[3], float hi[3]) {
  if (r & 0x80000000u) {
    const float* s = &P.sph[size_t(r & 0x7fffffffu) * 4];
    for (int k = 0; k < 3; ++k) { lo[k] = s[k] - s[3]; hi[k] = s[k] + s[3]; }
    return;
  }
  for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
  for (int j = 0; j < 3; ++j) {
    const float* p = &P.pos[size_t(P.idx[size_t(r) * 3 + j]) * 3];
    for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
  }
}

static inline float half_area(const float lo[3], const float hi[3]) {
  const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
  return dx * dy + dy * dz + dz * dx;
}

// Binned SAH (16 bins per axis over the centroid bounds; leaf when splitting does not pay or at
// <= 2 primitives; traversal cost 1, intersection cost 1).
static void build_bvh(Prepared& P) {
  const uint32_t n = P.ntri + P.nsph;
  P.refs.resize(n);
  for (uint32_t i = 0; i < P.ntri; ++i) P.refs[i] = i;
  for (uint32_t i = 0; i < P.nsph; ++i) P.refs[P.ntri + i] = 0x80000000u | i;
  std::vector<float> cen(size_t(n) * 3), blo(size_t(n) * 3), bhi(size_t(n) * 3);
  for (uint32_t i = 0; i < n; ++i) {
    ref_bounds(P, P.refs[i], &blo[size_t(i) * 3], &bhi[size_t(i) * 3]);
    for (int k = 0; k < 3; ++k) cen[size_t(i) * 3 + k] = 0.5f * (blo[size_t(i) * 3 + k] + bhi[size_t(i) * 3 + k]);
  }
  std::vector<uint32_t> ord(n);  // slot -> original primitive i
  for (uint32_t i = 0; i < n; ++i) ord[i] = i;
  P.nodes.clear();
  if (n == 0) return;
  P.nodes.reserve(2 * size_t(n));
  constexpr int kBins = 16;
  constexpr uint32_t kMaxLeaf = 4;
  struct Task { uint32_t node, begin, end; };
  std::vector<Task> st;
  P.nodes.push_back(Node{});
  st.push_back({0, 0, n});
  while (!st.empty()) {
    const Task t = st.back();
    st.pop_back();
    Node nd{};
    for (int k = 0; k < 3; ++k) { nd.lo[k] = INFINITY; nd.hi[k] = -INFINITY; }
    float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = t.begin; i < t.end; ++i) {
      const uint32_t o = ord[i];
      for (int k = 0; k < 3; ++k) {
        nd.lo[k] = std::min(nd.lo[k], blo[size_t(o) * 3 + k]);
        nd.hi[k] = std::max(nd.hi[k], bhi[size_t(o) * 3 + k]);
        clo[k] = std::min(clo[k], cen[size_t(o) * 3 + k]);
        chi[k] = std::max(chi[k], cen[size_t(o) * 3 + k]);
      }
    }
    const uint32_t cnt = t.end - t.begin;
    int best_ax = -1, best_bin = 0;
    float best_cost = INFINITY;
    if (cnt > 2) {
      for (int ax = 0; ax < 3; ++ax) {
        const float ext = chi[ax] - clo[ax];
        if (!(ext > 0.0f)) continue;
        float bl[kBins][3], bh[kBins][3];
        uint32_t bc[kBins] = {};
        for (int b = 0; b < kBins; ++b)
          for (int k = 0; k < 3; ++k) { bl[b][k] = INFINITY; bh[b][k] = -INFINITY; }
        const float scale = float(kBins) / ext;
        for (uint32_t i = t.begin; i < t.end; ++i) {
          const uint32_t o = ord[i];
          const int b = std::min(kBins - 1, int((cen[size_t(o) * 3 + ax] - clo[ax]) * scale));
          ++bc[b];
          for (int k = 0; k < 3; ++k) {
            bl[b][k] = std::min(bl[b][k], blo[size_t(o) * 3 + k]);
            bh[b][k] = std::max(bh[b][k], bhi[size_t(o) * 3 + k]);
          }
        }
        float ra[kBins];
        uint32_t rc[kBins];
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        uint32_t c = 0;
        for (int b = kBins - 1; b > 0; --b) {
          c += bc[b];
          for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], bl[b][k]); hi[k] = std::max(hi[k], bh[b][k]); }
          ra[b] = c ? half_area(lo, hi) : 0.0f;
          rc[b] = c;
        }
        for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
        c = 0;
        for (int b = 0; b < kBins - 1; ++b) {
          c += bc[b];
          for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], bl[b][k]); hi[k] = std::max(hi[k], bh[b][k]); }
          if (c == 0 || rc[b + 1] == 0) continue;
          const float cost = half_area(lo, hi) * float(c) + ra[b + 1] * float(rc[b + 1]);
          if (cost < best_cost) { best_cost = cost; best_ax = ax; best_bin = b; }
        }
      }
    }
    const float leaf_cost = half_area(nd.lo, nd.hi) * float(cnt);
    const float split_cost = half_area(nd.lo, nd.hi) + best_cost;  // traversal + both children
    if (cnt <= 2 || best_ax < 0 || (cnt <= kMaxLeaf && split_cost >= leaf_cost)) {
      if (cnt > kMaxLeaf && best_ax < 0) {  // coincident centroids: split the range in half
        const uint32_t mid = t.begin + cnt / 2;
        const uint32_t l = uint32_t(P.nodes.size());
        P.nodes.push_back(Node{});
        P.nodes.push_back(Node{});
        nd.left = l;
        nd.count = 0;
        nd.axis = 0;
        P.nodes[t.node] = nd;
        st.push_back({l + 1, mid, t.end});
        st.push_back({l, t.begin, mid});
        continue;
      }
      nd.left = t.begin;
      nd.count = cnt;
      P.nodes[t.node] = nd;
      continue;
    }
    const float scale = float(kBins) / (chi[best_ax] - clo[best_ax]);
    const auto it = std::partition(ord.begin() + t.begin, ord.begin() + t.end, [&](uint32_t o) {
      return std::min(kBins - 1, int((cen[size_t(o) * 3 + best_ax] - clo[best_ax]) * scale)) <= best_bin;
    });
    const uint32_t mid = uint32_t(it - ord.begin());
    const uint32_t l = uint32_t(P.nodes.size());
    P.nodes.push_back(Node{});
    P.nodes.push_back(Node{});
    nd.left = l;
    nd.count = 0;
    nd.axis = uint32_t(best_ax);
    P.nodes[t.node] = nd;
    st.push_back({l + 1, mid, t.end});
    st.push_back({l, t.begin, mid});
  }
  std::vector<uint32_t> r2(n);
  for (uint32_t i = 0; i < n; ++i) r2[i] = P.refs[ord[i]];
  P.refs.swap(r2);
}

// Ray with its per-axis reciprocal, computed once per query (the slab test prunes only).
struct RayInv {
  float o[3], inv[3];
  bool zero[3];
  int neg[3];
};
static inline RayInv ray_inv(V3 O, V3 D) {
  RayInv r;
  const float o[3] = {O.x, O.y, O.z}, d[3] = {D.x, D.y, D.z};
  for (int k = 0; k < 3; ++k) {
    r.o[k] = o[k];
    r.zero[k] = d[k] == 0.0f;
    r.inv[k] = r.zero[k] ? 0.0f : 1.0f / d[k];
    r.neg[k] = d[k] < 0.0f;
  }
  return r;
}
// conservative slab test (padded exit distance); returns the entry distance in *tent
static inline bool box_hit(const Node& nd, const RayInv& r, float tnear, float tfar, float* tent = nullptr) {
  float t0 = tnear, t1 = tfar;
  for (int k = 0; k < 3; ++k) {
    if (r.zero[k]) {
      if (r.o[k] < nd.lo[k] || r.o[k] > nd.hi[k]) return false;
      continue;
    }
    float a = (nd.lo[k] - r.o[k]) * r.inv[k], b = (nd.hi[k] - r.o[k]) * r.inv[k];
    if (a > b) std::swap(a, b);
    b *= 1.0f + 8.0f * std::numeric_limits<float>::epsilon();
    a *= 1.0f - 8.0f * std::numeric_limits<float>::epsilon();
    if (a > t0) t0 = a;
    if (b < t1) t1 = b;
    if (t0 > t1) return false;
  }
  if (tent) *tent = t0;
  return true;
}

struct HitRec {
  float t;
  uint32_t geom, prim;
  V3 Ng;
};

static inline void test_ref(const Prepared& P, uint32_t r, V3 O, V3 D, float tnear, float& tfar, HitRec& h, bool& any) {
  float t;
  V3 ng;
  if (r & 0x80000000u) {
    const uint32_t si = r & 0x7fffffffu;
    if (sphere_hit(&P.sph[size_t(si) * 4], O, D, tnear, tfar, t, ng)) {
      tfar = t;
      h = HitRec{t, P.ngeom_tri + si, 0u, ng};
      any = true;
    }
    return;
  }
  const uint32_t* ix = &P.idx[size_t(r) * 3];
  const float* a = &P.pos[size_t(ix[0]) * 3];
  const float* b = &P.pos[size_t(ix[1]) * 3];
  const float* c = &P.pos[size_t(ix[2]) * 3];
  if (tri_hit(mk(a[0], a[1], a[2]), mk(b[0], b[1], b[2]), mk(c[0], c[1], c[2]), O, D, tnear, tfar, t, ng)) {
    tfar = t;
    const uint32_t g = P.tri_geom[r];
    h = HitRec{t, g, r - P.geom_first[g], ng};
    any = true;
  }
}

static bool closest_hit(const Prepared& P, V3 O, V3 D, float tnear, float tfar, HitRec& h, bool use_bvh) {
  bool any = false;
  if (!use_bvh || P.nodes.empty()) {
    for (uint32_t i = 0; i < P.ntri; ++i) test_ref(P, i, O, D, tnear, tfar, h, any);
    for (uint32_t i = 0; i < P.nsph; ++i) test_ref(P, 0x80000000u | i, O, D, tnear, tfar, h, any);
    return any;
  }
  // front-to-back: the child on the ray's near side of the split axis first; a popped node is
  // re-tested against the shrunk tfar
  const RayInv ri = ray_inv(O, D);
  uint32_t stack[256];
  int sp = 0;
  stack[sp++] = 0;
  while (sp) {
    const Node& nd = P.nodes[stack[--sp]];
    if (!box_hit(nd, ri, tnear, tfar)) continue;
    if (nd.count) {
      for (uint32_t i = 0; i < nd.count; ++i) test_ref(P, P.refs[nd.left + i], O, D, tnear, tfar, h, any);
    } else {
      const uint32_t near = nd.left + uint32_t(ri.neg[nd.axis]), far = nd.left + 1u - uint32_t(ri.neg[nd.axis]);
      stack[sp++] = far;
      stack[sp++] = near;
    }
  }
  return any;
}

static inline bool ref_occludes(const Prepared& P, uint32_t r, V3 O, V3 D, float tnear, float tfar) {
  if (r & 0x80000000u) return sphere_occludes(&P.sph[size_t(r & 0x7fffffffu) * 4], O, D, tnear, tfar);
  const uint32_t* ix = &P.idx[size_t(r) * 3];
  const float* a = &P.pos[size_t(ix[0]) * 3];
  const float* b = &P.pos[size_t(ix[1]) * 3];
  const float* c = &P.pos[size_t(ix[2]) * 3];
  float t;
  V3 ng;
  return tri_hit(mk(a[0], a[1], a[2]), mk(b[0], b[1], b[2]), mk(c[0], c[1], c[2]), O, D, tnear, tfar, t, ng);
}

static bool occluded(const Prepared& P, V3 O, V3 D, float tnear, float tfar, bool use_bvh) {
  if (!use_bvh || P.nodes.empty()) {
    for (uint32_t i = 0; i < P.ntri; ++i) if (ref_occludes(P, i, O, D, tnear, tfar)) return true;
    for (uint32_t i = 0; i < P.nsph; ++i) if (ref_occludes(P, 0x80000000u | i, O, D, tnear, tfar)) return true;
    return false;
  }
  const RayInv ri = ray_inv(O, D);
  uint32_t stack[256];
  int sp = 0;
  stack[sp++] = 0;
  while (sp) {
    const Node& nd = P.nodes[stack[--sp]];
    if (!box_hit(nd, ri, tnear, tfar)) continue;
    if (nd.count) {
      for (uint32_t i = 0; i < nd.count; ++i) if (ref_occludes(P, P.refs[nd.left + i], O, D, tnear, tfar)) return true;
    } else {
      stack[sp++] = nd.left + 1;
      stack[sp++] = nd.left;
    }
  }
  return false;
}

// ----------------------------------------------------------------------------- camera
struct Camera {
  V3 pos, fwd, right, up;
  float half_w, half_h;
};
static Camera make_camera(V3 pos, V3 target, float fov_deg, float aspect) {  // Camera.cpp:5-50
  Camera c;
  c.pos = pos;
  const V3 dir = normalize(target - pos);
  const float yaw = degrees_f(std::atan2(dir.z, dir.x));
  const float pitch = degrees_f(std::asin(dir.y));
  V3 f;
  f.x = std::cos(radians_f(yaw)) * std::cos(radians_f(pitch));
  f.y = std::sin(radians_f(pitch));
  f.z = std::sin(radians_f(yaw)) * std::cos(radians_f(pitch));
  c.fwd = normalize(f);
  c.right = normalize(cross(c.fwd, mk(0, 1, 0)));
  c.up = normalize(cross(c.right, c.fwd));
  c.half_h = std::tan(radians_f(fov_deg) * 0.5f);
  c.half_w = c.half_h * aspect;
  return c;
}
static V3 ray_dir(const Camera& c, float x, float y) {  // Camera::getRayDirection (Camera.cpp:95-106)
  const float nx = (x - 0.5f) * 2.0f;
  const float ny = -(y - 0.5f) * 2.0f;
  const V3 d = c.fwd + nx * c.half_w * c.right + ny * c.half_h * c.up;
  return normalize(d);
}

// ----------------------------------------------------------------------------- integrator
struct Counters {
  uint64_t closest = 0, shadow = 0, samples = 0, bounces = 0;
};
struct Ctx {
  const Prepared* P;
  const std::vector<Material>* mats;
  const std::vector<Light>* lights;
  Env env;
  uint32_t max_depth;
  bool bvh;
};

static const Material& material_of(const Ctx& x, uint32_t geom) {  // MaterialManager::getMaterialFromHit
  const std::vector<Material>& M = *x.mats;
  const std::vector<uint32_t>& G = x.P->geom_material;
  if (!G.empty() && geom < G.size()) {
    const uint32_t mid = G[geom];
    if (mid < M.size()) return M[mid];
  }
  if (geom < M.size()) return M[geom];  // getMaterialByID fallback
  return M[geom % M.size()];
}

// Residue diagnosis: when set (one thread), trace_path appends every ray it traces — 9 floats: kind
// (0 closest hit, 1 shadow), origin, direction, tnear, tfar — so a test can replay them on the GPU.
static thread_local std::vector<float>* g_raylog = nullptr;
static inline void log_ray(float kind, V3 o, V3 d, float tn, float tf) {
  if (g_raylog) g_raylog->insert(g_raylog->end(), {kind, o.x, o.y, o.z, d.x, d.y, d.z, tn, tf});
}

// WavefrontPathTracerCPU::traceRay (wf_pt_cpu.cpp:61-255) for the tile task's {spp=1}
static V3 trace_path(const Ctx& x, V3 origin, V3 direction, uint32_t pixel_seed, uint32_t spp, Counters& cnt) {
  V3 color = mk(0, 0, 0);
  const float inf = std::numeric_limits<float>::infinity();
  for (uint32_t s = 0; s < spp; ++s) {
    V3 ro = origin;
    V3 rd = safe_normalize(direction);
    V3 thr = mk(1, 1, 1);
    V3 rad = mk(0, 0, 0);
    uint32_t rng = wang_hash(pixel_seed ^ (s * 9781u + 1u));
    for (uint32_t bounce = 0; bounce < x.max_depth; ++bounce) {
      HitRec h;
      ++cnt.closest;
      ++cnt.bounces;
      log_ray(0.0f, ro, rd, 0.0f, inf);
      if (!closest_hit(*x.P, ro, rd, 0.0f, inf, h, x.bvh)) {
        rad = rad + thr * env_color(x.env, safe_normalize(rd));
        break;
      }
      const V3 p = ro + h.t * rd;
      V3 n = safe_normalize(h.Ng);
      if (dot(n, rd) > 0.0f) n = -n;
      const Material& m = material_of(x, h.geom);
      if (dot(m.emission, m.emission) > 0.0f) rad = rad + thr * m.emission;
      {
        const V3 view = -rd;
        for (const Light& L : *x.lights) {
          V3 ldir;
          float ldist = 0.0f;
          const V3 Li = light_radiance(L, p, ldir, ldist);
          const float cs = std::max(dot(n, ldir), 0.0f);
          if (cs <= 0.0f) continue;
          // Light::isOccluded (Light.cpp:16-40)
          const float eps = 1e-4f * gmax(1.0f, gmax(gmax(std::fabs(p.x), std::fabs(p.y)), std::fabs(p.z)));
          const V3 so = p + n * eps;
          ++cnt.shadow;
          log_ray(1.0f, so, ldir, 1e-4f, ldist - 1e-4f);
          if (occluded(*x.P, so, ldir, 1e-4f, ldist - 1e-4f, x.bvh)) continue;
          const V3 f = eval_brdf(m, n, view, ldir);
          rad = rad + thr * (f * Li * cs);
        }
      }
      if (m.metallic > 0.5f) {  // mirror metal
        const V3 r = reflect(rd, n);
        ro = p + n * 1e-4f;
        rd = safe_normalize(r);
        thr = thr * (m.albedo * m.metallic);
        continue;
      }
      if (is_transparent(m)) {  // glass
        const float ior = m.ior;
        const float cosine = -dot(rd, n);
        const float eta = (cosine >= 0.0f) ? (1.0f / ior) : ior;
        const float tr = transparency(m);
        float r0 = (1.0f - ior) / (1.0f + ior);
        r0 = r0 * r0;
        const float xc = 1.0f - std::clamp(std::fabs(cosine), 0.0f, 1.0f);
        const float F = r0 + (1.0f - r0) * xc * xc * xc * xc * xc;
        const float xi = rand01(rng);
        if (xi < F) {
          const V3 r = reflect(rd, n);
          ro = p + n * 1e-4f;
          rd = safe_normalize(r);
          thr = thr * mk(1.0f - tr, 1.0f - tr, 1.0f - tr);
          continue;
        }
        const float ci = -dot(n, rd);
        const float k = 1.0f - eta * eta * (1.0f - ci * ci);
        V3 refr = mk(0, 0, 0);
        if (!(k < 0.0f)) refr = eta * rd + (eta * ci - std::sqrt(k)) * n;
        if (dot(refr, refr) > 0.0f) {
          ro = p - n * 1e-4f;
          rd = safe_normalize(refr);
          thr = thr * mk(tr, tr, tr);
        } else {
          const V3 r = reflect(rd, n);
          ro = p + n * 1e-4f;
          rd = safe_normalize(r);
        }
        continue;
      }
      {  // diffuse: cosine sample (wf_math.h:51-72), then RR draw
        const float r1 = rand01(rng);
        const float r2 = rand01(rng);
        float sp, cp;
        cosine_sincos(r1, sp, cp);  // phi = 2 pi r1
        const float rr = std::sqrt(r2);
        const float lx = rr * cp, ly = rr * sp;
        const float lz = std::sqrt(std::max(0.0f, 1.0f - r2));
        const V3 nn = safe_normalize(n);
        const V3 t = (std::fabs(nn.z) < 0.999f) ? normalize(cross(nn, mk(0, 0, 1))) : normalize(cross(nn, mk(0, 1, 0)));
        const V3 b = cross(t, nn);
        const V3 nd = safe_normalize(t * lx + b * ly + nn * lz);
        const V3 no = p + n * 1e-4f;
        const float surv = gmax(gmax(m.albedo.x, m.albedo.y), m.albedo.z);
        const float xi = rand01(rng);
        if (bounce > 2) {
          if (xi >= surv) break;
          thr = thr * (m.albedo / std::max(surv, 1e-6f));
        } else {
          thr = thr * m.albedo;
        }
        ro = no;
        rd = safe_normalize(nd);
        continue;
      }
    }
    color = color + rad;
  }
  return color / float(std::max(1u, spp));
}

// EnvironmentManager::acesToneMapping + the tile task's resolve (GLRenderer.cpp:411-431)
static inline void resolve_pixel(V3 acc, uint32_t n, uint8_t* out) {
  V3 c = acc / float(n);
  const float a = 2.51f, b = 0.03f, cc = 2.43f, d = 0.59f, e = 0.14f;
  c = gclamp((c * (a * c + b)) / (c * (cc * c + d) + e), 0.0f, 1.0f);
  const float g = 1.0f / 2.2f;
  c = mk(std::pow(c.x, g), std::pow(c.y, g), std::pow(c.z, g));
  c = gclamp(c, 0.0f, 1.0f);
  out[0] = static_cast<unsigned char>(c.x * 255.0f);
  out[1] = static_cast<unsigned char>(c.y * 255.0f);
  out[2] = static_cast<unsigned char>(c.z * 255.0f);
}

// ----------------------------------------------------------------------------- PathTracer mode
// PathTracer::tracePathMonteCarlo (PathTracer.cpp:113-224) evaluated forward with a throughput (as
// the product does; the estimator is the recursion's), with the deterministic RNG stream below.
static inline uint32_t pt_seed(uint32_t ps, uint32_t acc, uint32_t s) {
  return wang_hash(wang_hash(ps ^ (acc * 9781u)) ^ (s * 0x9E3779B9u + 0x68E31DA4u));
}
static V3 pt_path(const Ctx& x, V3 o, V3 d, uint32_t& rng, Counters& cnt) {
  const float inf = std::numeric_limits<float>::infinity();
  V3 rad = mk(0, 0, 0), thr = mk(1, 1, 1);
  for (uint32_t lvl = 0; lvl < x.max_depth; ++lvl) {
    HitRec h;
    ++cnt.closest;
    if (!closest_hit(*x.P, o, d, 1e-4f, inf, h, x.bvh)) {  // intersectRay: tnear 1e-4 (:82-100)
      rad = rad + thr * env_color(x.env, normalize(d));
      break;
    }
    const V3 P = o + h.t * d;
    V3 n = normalize(h.Ng);
    if (dot(n, d) > 0.0f) n = -n;
    const Material& m = material_of(x, h.geom);
    V3 color = m.emission;
    const V3 view = -d;
    for (const Light& L : *x.lights) {
      V3 ldir;
      float ldist = 0.0f;
      const V3 Li = light_radiance(L, P, ldir, ldist);
      const float cs = std::max(dot(n, ldir), 0.0f);
      if (!(cs > 0.0f)) continue;
      const float eps = 1e-4f * gmax(1.0f, gmax(gmax(std::fabs(P.x), std::fabs(P.y)), std::fabs(P.z)));
      ++cnt.shadow;
      if (!occluded(*x.P, P + n * eps, ldir, 1e-4f, ldist - 1e-4f, x.bvh)) color = color + eval_brdf(m, n, view, ldir) * Li * cs;
    }
    rad = rad + thr * color;
    // calculateSafeRayOrigin (:103-111)
    const float eps = 1e-4f * gmax(1.0f, gmax(gmax(std::fabs(P.x), std::fabs(P.y)), std::fabs(P.z)));
    if (m.metallic > 0.5f) {
      d = reflect(d, n);
      o = P + n * eps;
      thr = (thr * m.albedo) * m.metallic;
      continue;
    }
    if (is_transparent(m)) {
      const float ior = m.ior;
      const float cosine = -dot(d, n);
      const float eta = cosine > 0.0f ? (1.0f / ior) : ior;
      const float tr = transparency(m);
      float r0 = (1.0f - ior) / (1.0f + ior);  // schlickFresnel (:391-395)
      r0 = r0 * r0;
      const float fres = r0 + (1.0f - r0) * std::pow(1.0f - std::fabs(cosine), 5.0f);
      if (rand01(rng) < fres) {
        d = reflect(d, n);
        o = P + n * eps;
        thr = thr * (1.0f - tr);
        continue;
      }
      const float cos_i = -dot(d, n);  // PathTracer::refract (:396-406)
      const float sin_t2 = eta * eta * (1.0f - cos_i * cos_i);
      V3 refr = mk(0, 0, 0);
      if (!(sin_t2 >= 1.0f)) refr = eta * d + (eta * cos_i - std::sqrt(1.0f - sin_t2)) * n;
      if (dot(refr, refr) > 0.0f) {
        o = P - n * eps;
        d = refr;
        thr = thr * tr;
      } else {
        d = reflect(d, n);
        o = P + n * eps;
      }
      continue;
    }
    const float r1 = rand01(rng);  // cosineHemisphereSample (:59-75)
    const float r2 = rand01(rng);
    const float cos_t = std::sqrt(r1), sin_t = std::sqrt(1.0f - r1);
    const float phi = float(2.0 * 3.14159265358979323846 * double(r2));
    const V3 sd = mk(sin_t * std::cos(phi), cos_t, sin_t * std::sin(phi));
    const V3 up = (std::fabs(n.x) < 0.9f) ? mk(1, 0, 0) : mk(0, 1, 0);
    const V3 tg = normalize(cross(up, n));
    const V3 bt = cross(n, tg);
    const V3 scatter = tg * sd.x + n * sd.y + bt * sd.z;
    o = P + n * eps;
    const float surv = gmax(gmax(m.albedo.x, m.albedo.y), m.albedo.z);
    if (!(rand01(rng) < surv)) break;
    thr = (thr * m.albedo) / surv;
    d = scatter;
  }
  return rad;
}

// ----------------------------------------------------------------------------- OptiX mode
static inline V3 ox_nrm(V3 v) { return v * (1.0f / std::sqrt(dot(v, v))); }  // f3_normalize
static inline V3 ox_cross(V3 a, V3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static inline V3 ox_reflect(V3 v, V3 n) { return v + n * (-2.0f * dot(v, n)); }
static inline void ox_onb(V3 n, V3& t, V3& b) {
  const V3 up = (std::fabs(n.z) < 0.999f) ? mk(0, 0, 1) : mk(1, 0, 0);
  t = ox_nrm(ox_cross(up, n));
  b = ox_cross(n, t);
}
static inline V3 ox_fresnel(float cosVH, V3 F0) {
  const float m = 1.0f - std::min(std::max(cosVH, 0.0f), 1.0f);
  const float m2 = m * m;
  const float m5 = m2 * m2 * m;
  return F0 + mk(1.0f - F0.x, 1.0f - F0.y, 1.0f - F0.z) * m5;
}
static inline float ox_smith(float cosNL, float cosNV, float alpha) {
  const float a = alpha + 1.0f;
  const float k = (a * a) * 0.125f;
  return (cosNL / (cosNL * (1.0f - k) + k)) * (cosNV / (cosNV * (1.0f - k) + k));
}
static inline V3 ox_fallback_reflect(V3 d, V3 n) {
  const V3 R = ox_reflect(d, n);
  const float l2 = dot(R, R);
  return l2 > 0.0f ? R * (1.0f / std::sqrt(l2)) : n;
}
struct OxFrame {
  V3 u, v, w, light_dir, light_rad;
  bool has_light;
};
static void ox_path(const Ctx& x, const OxFrame& F, V3 o, V3 d, uint32_t rng, V3& acc, Counters& cnt) {
  const float kPi = 3.14159265358979323846f;
  V3 thr = mk(1, 1, 1);
  for (uint32_t depth = 0; depth < x.max_depth; ++depth) {
    HitRec h;
    ++cnt.closest;
    if (!closest_hit(*x.P, o, d, 1e-3f, 1e16f, h, x.bvh)) {
      const V3 c = env_color(x.env, ox_nrm(d));
      acc = acc + mk(c.x * thr.x, c.y * thr.y, c.z * thr.z);
      return;
    }
    const V3 P = o + d * h.t;
    V3 ng;
    const bool sphere = h.geom >= x.P->ngeom_tri;
    if (sphere) {
      const float* s = &x.P->sph[size_t(h.geom - x.P->ngeom_tri) * 4];
      ng = ox_nrm(ox_nrm(mk(P.x - s[0], P.y - s[1], P.z - s[2])));
    } else {
      const uint32_t tri = x.P->geom_first[h.geom] + h.prim;
      const uint32_t* ix = &x.P->idx[size_t(tri) * 3];
      const float* a = &x.P->pos[size_t(ix[0]) * 3];
      const float* b = &x.P->pos[size_t(ix[1]) * 3];
      const float* c = &x.P->pos[size_t(ix[2]) * 3];
      const V3 v0 = mk(a[0], a[1], a[2]), v1 = mk(b[0], b[1], b[2]), v2 = mk(c[0], c[1], c[2]);
      ng = ox_nrm(ox_nrm(ox_cross(v1 - v0, v2 - v0)));
    }
    {
      const float l2 = dot(ng, ng);
      ng = l2 > 0.0f ? ng * (1.0f / std::sqrt(l2)) : mk(0, 1, 0);
    }
    const std::vector<Material>& M = *x.mats;
    uint32_t mid = x.P->geom_material[h.geom];
    if (mid >= M.size()) mid = uint32_t(M.size() - 1);
    const Material& m = M[mid];
    const V3 base = mk(std::min(std::max(m.albedo.x, 0.0f), 1.0f), std::min(std::max(m.albedo.y, 0.0f), 1.0f),
                       std::min(std::max(m.albedo.z, 0.0f), 1.0f));
    const bool dielectric = m.type == 1;
    const float omm = std::min(std::max(1.0f - m.metallic, 0.0f), 1.0f);
    const V3 diffuse = base * omm;
    if (depth + 1u >= x.max_depth) {
      const V3 nvis = (ng + mk(1, 1, 1)) * 0.5f;
      const V3 shd = diffuse * nvis;
      acc = acc + mk(shd.x * thr.x, shd.y * thr.y, shd.z * thr.z);
      return;
    }
    const bool entering = dot(d, ng) < 0.0f;
    const V3 n = entering ? ng : -ng;
    if (F.has_light) {
      const V3 V = ox_nrm(-d);
      const V3 L = ox_nrm(-F.light_dir);
      const float NdotL = std::max(dot(n, L), 0.0f);
      if (NdotL > 0.0f && !dielectric) {
        V3 fr = mk(0, 0, 0);
        if (m.metallic > 0.5f) {
          const float r = std::min(std::max(m.roughness, 0.02f), 1.0f);
          const float alpha = r * r;
          const V3 H = ox_nrm(V + L);
          const float cosNV = std::max(dot(n, V), 0.0f), cosNL = NdotL, cosVH = std::max(dot(V, H), 0.0f);
          if (cosNV > 0.0f && cosNL > 0.0f) {
            const float cosNH = std::max(dot(n, H), 0.0f);
            const float a2 = alpha * alpha;
            const float den = cosNH * cosNH * (a2 - 1.0f) + 1.0f;
            const float D = a2 / (kPi * den * den);
            const float G = ox_smith(cosNL, cosNV, alpha);
            const V3 Fr = ox_fresnel(cosVH, base);
            const float dn = std::max(4.0f * cosNV * cosNL, 1e-6f);
            fr = Fr * ((D * G) / dn);
          }
        } else {
          fr = diffuse * (1.0f / kPi);
        }
        acc = acc + ((thr * fr) * F.light_rad) * NdotL;
      }
    }
    if (dielectric) {
      const float xi = rand01(rng);
      const float etaI = entering ? 1.0f : m.ior, etaT = entering ? m.ior : 1.0f;
      const float eta = etaI / etaT;
      const float cosI = std::min(std::max(-dot(d, n), -1.0f), 1.0f);
      float R0 = (etaT - etaI) / (etaT + etaI);
      R0 = R0 * R0;
      const float mm = 1.0f - std::min(std::max(cosI, 0.0f), 1.0f);
      const float Fr = R0 + (1.0f - R0) * (mm * mm * mm * mm * mm);
      const float ci = std::min(std::max(-dot(n, d), -1.0f), 1.0f);
      const float sin2T = eta * eta * std::max(0.0f, 1.0f - ci * ci);
      const bool can = !(sin2T > 1.0f);
      V3 refr = mk(0, 0, 0);
      if (can) {
        const float cosT = std::sqrt(std::max(0.0f, 1.0f - sin2T));
        refr = d * eta + n * (eta * ci - cosT);
        const float l2 = dot(refr, refr);
        if (l2 > 0.0f) refr = refr * (1.0f / std::sqrt(l2));
      }
      V3 nd = (!can || xi < Fr) ? ox_reflect(d, n) : refr;
      nd = ox_nrm(nd);
      o = P + nd * 1e-3f;
      d = nd;
      continue;
    }
    if (m.metallic > 0.5f) {
      const float r = std::min(std::max(m.roughness, 0.02f), 1.0f);
      const float alpha = r * r;
      const V3 V = ox_nrm(-d);
      const float cosNV_raw = dot(n, V);
      if (cosNV_raw <= 0.0f) {
        d = ox_fallback_reflect(d, n);
        o = P + n * 1e-3f;
        thr = thr * base;
        continue;
      }
      const float u1 = rand01(rng), u2 = rand01(rng);
      const float a2 = alpha * alpha;
      const float phi = 6.28318530717958647692f * u1;
      const float den = 1.0f + (a2 - 1.0f) * u2;
      const float cosT = std::sqrt(std::max(0.0f, (1.0f - u2) / den));
      const float sinT = std::sqrt(std::max(0.0f, 1.0f - cosT * cosT));
      const float sp = std::sin(phi), cp = std::cos(phi);
      V3 tb, bb;
      ox_onb(n, tb, bb);
      V3 H = tb * (sinT * cp) + bb * (sinT * sp) + n * cosT;
      const float hl2 = dot(H, H);
      H = hl2 > 0.0f ? H * (1.0f / std::sqrt(hl2)) : n;
      const float cosNH_raw = dot(n, H);
      if (cosNH_raw <= 0.0f) {
        d = ox_fallback_reflect(d, n);
        o = P + n * 1e-3f;
        thr = thr * base;
        continue;
      }
      V3 L = ox_reflect(-V, H);
      const float ll2 = dot(L, L);
      L = ll2 > 0.0f ? L * (1.0f / std::sqrt(ll2)) : n;
      const float cosNL_raw = dot(n, L);
      if (cosNL_raw <= 0.0f) {
        d = ox_fallback_reflect(d, n);
        o = P + n * 1e-3f;
        thr = thr * base;
        continue;
      }
      const float cosNV = std::max(cosNV_raw, 1e-6f), cosNL = std::max(cosNL_raw, 1e-6f), cosNH = std::max(cosNH_raw, 1e-6f);
      const float cosVH = std::max(dot(V, H), 0.0f);
      const V3 Fr = ox_fresnel(cosVH, base);
      const float G = ox_smith(cosNL, cosNV, alpha);
      float scale = (G * cosVH) / (cosNV * cosNH);
      scale = std::min(scale, 50.0f);
      if (scale < 0.0f) scale = 0.0f;
      o = P + n * 1e-3f;
      d = L;
      thr = thr * (Fr * scale);
      continue;
    }
    const float u1 = rand01(rng), u2 = rand01(rng);
    const float rr = std::sqrt(u1);
    const float phi = 2.0f * 3.14159265358979323846f * u2;
    const float sp = std::sin(phi), cp = std::cos(phi);
    const V3 loc = mk(rr * cp, rr * sp, std::sqrt(std::max(0.0f, 1.0f - u1)));
    V3 tb, bb;
    ox_onb(n, tb, bb);
    d = ox_nrm(tb * loc.x + bb * loc.y + n * loc.z);
    o = P + n * 1e-3f;
    thr = thr * diffuse;
  }
}

}  // namespace orc

// ===================================================================================== C ABI
using namespace orc;

extern "C" {

struct oracle_scene_in {
  const float* positions;
  uint32_t num_verts;
  const uint32_t* indices;
  uint32_t num_tris;
  const uint32_t* tri_geom_first;  // num_tri_geoms + 1
  uint32_t num_tri_geoms;
  const float* spheres;  // cx cy cz r
  uint32_t num_spheres;
  const uint32_t* geom_material;  // num_tri_geoms + num_spheres
};

struct oracle_job {
  const float* materials;  // 12 floats each: albedo3 metallic roughness emission3 ior type pad pad
  uint32_t num_materials;
  const float* lights;  // 8 floats each: type v3 color3 intensity
  uint32_t num_lights;
  const float* env_faces;  // null: procedural sky
  int32_t env_size;
  float env_intensity, env_clamp;
  float cam[14];  // pos3 fwd3 right3 up3 half_w half_h
  int32_t width, height;
  uint32_t frame_begin, num_frames, max_depth;
  int32_t shard_rank, shard_count;
  int32_t threads, use_bvh;
  float* accum;   // width*height*3, read-modify-write
  uint8_t* rgb;   // width*height*3 (shard pixels only), may be null
  uint64_t counters[4];  // closest-hit queries, shadow queries, samples, bounces
  const uint32_t* pixels;  // oracle_render only: if not null, render just these pixels (y * width + x)
  uint32_t num_pixels;
};

int oracle_version(void) { return 5; }

// Residue diagnosis (see DevMath): sin_cos = 2^24 (sin, cos) pairs or null; pow_chains 0/1.  Global,
// set before a render and reset after it.
void oracle_set_device_math(const float* sin_cos, int pow_chains) {
  g_devmath.sin_cos = sin_cos;
  g_devmath.pow_chains = pow_chains != 0;
}

uint32_t oracle_wang_hash(uint32_t a) { return wang_hash(a); }

void oracle_rand_stream(uint32_t seed, uint32_t n, float* out, uint32_t* states) {
  uint32_t s = seed;
  for (uint32_t i = 0; i < n; ++i) {
    out[i] = rand01(s);
    if (states) states[i] = s;
  }
}

void* oracle_prepare(const oracle_scene_in* in, int want_bvh) {
  Prepared* P = new Prepared();
  P->pos.assign(in->positions, in->positions + size_t(in->num_verts) * 3);
  P->idx.assign(in->indices, in->indices + size_t(in->num_tris) * 3);
  P->geom_first.assign(in->tri_geom_first, in->tri_geom_first + in->num_tri_geoms + 1);
  P->sph.assign(in->spheres, in->spheres + size_t(in->num_spheres) * 4);
  P->ntri = in->num_tris;
  P->nsph = in->num_spheres;
  P->ngeom_tri = in->num_tri_geoms;
  P->geom_material.assign(in->geom_material, in->geom_material + in->num_tri_geoms + in->num_spheres);
  P->tri_geom.resize(P->ntri);
  for (uint32_t g = 0; g < P->ngeom_tri; ++g)
    for (uint32_t i = P->geom_first[g]; i < P->geom_first[g + 1]; ++i) P->tri_geom[i] = g;
  if (want_bvh) build_bvh(*P);
  return P;
}
void oracle_release(void* h) { delete static_cast<Prepared*>(h); }

// Builtin scene generator (oracle's own restatement; tests compare it with the product's).
struct oracle_flat {
  Flat f;
};
void* oracle_builtin_scene(int which, uint32_t stacks, uint32_t slices) {
  oracle_flat* o = new oracle_flat();
  o->f = flatten(builtin_scene(which, stacks, slices));
  return o;
}
void oracle_flat_view(void* h, oracle_scene_in* out) {
  oracle_flat* o = static_cast<oracle_flat*>(h);
  out->positions = o->f.positions.data();
  out->num_verts = uint32_t(o->f.positions.size() / 3);
  out->indices = o->f.indices.data();
  out->num_tris = uint32_t(o->f.indices.size() / 3);
  out->tri_geom_first = o->f.tri_geom_first.data();
  out->num_tri_geoms = uint32_t(o->f.tri_geom_first.size() - 1);
  out->spheres = o->f.spheres.data();
  out->num_spheres = uint32_t(o->f.spheres.size() / 4);
  out->geom_material = o->f.geom_material.data();
}
void oracle_flat_free(void* h) { delete static_cast<oracle_flat*>(h); }

int oracle_preset_materials(int with_light, float* out, int cap) {
  const std::vector<Material> v = preset_materials(with_light != 0);
  const int n = int(v.size());
  for (int i = 0; i < n && i < cap; ++i) {
    const Material& m = v[i];
    float* o = out + i * 12;
    o[0] = m.albedo.x; o[1] = m.albedo.y; o[2] = m.albedo.z; o[3] = m.metallic; o[4] = m.roughness;
    o[5] = m.emission.x; o[6] = m.emission.y; o[7] = m.emission.z; o[8] = m.ior; o[9] = float(m.type);
    o[10] = 0; o[11] = 0;
  }
  return n;
}

void oracle_camera(const float pos[3], const float target[3], float fov_deg, float aspect, float out[14]) {
  const Camera c = make_camera(mk(pos[0], pos[1], pos[2]), mk(target[0], target[1], target[2]), fov_deg, aspect);
  const float v[14] = {c.pos.x, c.pos.y, c.pos.z, c.fwd.x, c.fwd.y, c.fwd.z, c.right.x, c.right.y,
                       c.right.z, c.up.x, c.up.y, c.up.z, c.half_w, c.half_h};
  std::memcpy(out, v, sizeof(v));
}

static Camera cam_from(const float* v) {
  Camera c;
  c.pos = mk(v[0], v[1], v[2]);
  c.fwd = mk(v[3], v[4], v[5]);
  c.right = mk(v[6], v[7], v[8]);
  c.up = mk(v[9], v[10], v[11]);
  c.half_w = v[12];
  c.half_h = v[13];
  return c;
}

// Primary-ray generation of the tile task for every pixel of a W x H image at sample index `acc`:
// dirs (W*H*3) and the integrator's initial rng state wang_hash((y*W+x ^ acc) ^ 1).
void oracle_primary(const float cam[14], int W, int H, uint32_t acc, float* dirs, uint32_t* rng0) {
  const Camera c = cam_from(cam);
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      const uint32_t ps = uint32_t(y * W + x);
      uint32_t r = wang_hash(ps ^ acc * 9781u);
      const float jx = rand01(r), jy = rand01(r);
      const V3 d = ray_dir(c, (float(x) + jx) / float(W), (float(y) + jy) / float(H));
      const V3 dd = safe_normalize(d);
      const size_t p = size_t(ps);
      dirs[p * 3 + 0] = dd.x; dirs[p * 3 + 1] = dd.y; dirs[p * 3 + 2] = dd.z;
      if (rng0) rng0[p] = wang_hash((ps ^ acc) ^ 1u);
    }
}

// Closest-hit queries: rays = n * 8 floats (o3, d3, tnear, tfar). Outputs geomID (~0u on miss),
// primID, t, Ng (unnormalised, as Embree reports it).
void oracle_intersect(void* h, const float* rays, uint32_t n, int use_bvh, uint32_t* geom, uint32_t* prim, float* t,
                      float* ng) {
  const Prepared& P = *static_cast<Prepared*>(h);
  for (uint32_t i = 0; i < n; ++i) {
    const float* r = rays + size_t(i) * 8;
    HitRec hr;
    if (closest_hit(P, mk(r[0], r[1], r[2]), mk(r[3], r[4], r[5]), r[6], r[7], hr, use_bvh != 0)) {
      geom[i] = hr.geom; prim[i] = hr.prim; t[i] = hr.t;
      ng[i * 3 + 0] = hr.Ng.x; ng[i * 3 + 1] = hr.Ng.y; ng[i * 3 + 2] = hr.Ng.z;
    } else {
      geom[i] = 0xFFFFFFFFu; prim[i] = 0xFFFFFFFFu; t[i] = INFINITY;
      ng[i * 3 + 0] = ng[i * 3 + 1] = ng[i * 3 + 2] = 0.0f;
    }
  }
}
void oracle_occluded(void* h, const float* rays, uint32_t n, int use_bvh, uint8_t* out) {
  const Prepared& P = *static_cast<Prepared*>(h);
  for (uint32_t i = 0; i < n; ++i) {
    const float* r = rays + size_t(i) * 8;
    out[i] = occluded(P, mk(r[0], r[1], r[2]), mk(r[3], r[4], r[5]), r[6], r[7], use_bvh != 0) ? 1 : 0;
  }
}

// EnvironmentManager::getEnvironmentColor for n directions (faces null -> procedural sky)
void oracle_env(const float* faces, int size, float intensity, float clamp_, const float* dirs, uint32_t n, float* out) {
  Env e;
  e.faces = faces; e.size = size; e.intensity = intensity; e.max_clamp = clamp_;
  for (uint32_t i = 0; i < n; ++i) {
    const V3 c = env_color(e, mk(dirs[i * 3], dirs[i * 3 + 1], dirs[i * 3 + 2]));
    out[i * 3] = c.x; out[i * 3 + 1] = c.y; out[i * 3 + 2] = c.z;
  }
}

// Cubemap::loadEquirectangular: equirect RGB float (w x h) -> 6 faces of size x size (nearest).
void oracle_equirect_to_faces(const float* rgb, int w, int h, int size, float* faces) {
  for (int f = 0; f < 6; ++f)
    for (int y = 0; y < size; ++y)
      for (int x = 0; x < size; ++x) {
        const float u = (2.0f * x / (size - 1)) - 1.0f;
        const float v = (2.0f * y / (size - 1)) - 1.0f;
        V3 d;
        switch (f) {
          case 0: d = mk(1.0f, -v, -u); break;
          case 1: d = mk(-1.0f, -v, u); break;
          case 2: d = mk(u, 1.0f, v); break;
          case 3: d = mk(u, -1.0f, -v); break;
          case 4: d = mk(u, -v, 1.0f); break;
          default: d = mk(-u, -v, -1.0f); break;
        }
        d = normalize(d);
        const float th = std::atan2(d.z, d.x);
        const float ph = std::acos(d.y);
        const float uu = float((double(th) + 3.14159265358979323846) / (2.0f * 3.14159265358979323846));
        const float vv = float(double(ph) / 3.14159265358979323846);
        const int sx = std::min(std::max(int(uu * w), 0), w - 1);
        const int sy = std::min(std::max(int(vv * h), 0), h - 1);
        const float* s = rgb + (size_t(sy) * w + sx) * 3;
        float* o = faces + ((size_t(f) * size + y) * size + x) * 3;
        o[0] = s[0]; o[1] = s[1]; o[2] = s[2];
      }
}

// Whole-image render over 32x32 tiles (std::thread pool with a dynamic tile counter, mirroring
// tbb::parallel_for over GLRenderer::renderWavefront's tiles).  Only tiles t with
// t % shard_count == shard_rank are rendered.  Each pixel runs frames frame_begin..+num_frames-1
// (one sample each, accumulated in order), then resolves with the total sample count.
int oracle_render(void* h, oracle_job* job) {
  const Prepared& P = *static_cast<Prepared*>(h);
  std::vector<Material> mats(job->num_materials);
  for (uint32_t i = 0; i < job->num_materials; ++i) {
    const float* m = job->materials + i * 12;
    mats[i] = Material{mk(m[0], m[1], m[2]), m[3], m[4], mk(m[5], m[6], m[7]), m[8], int(m[9])};
  }
  std::vector<Light> lights(job->num_lights);
  for (uint32_t i = 0; i < job->num_lights; ++i) {
    const float* l = job->lights + i * 8;
    lights[i] = Light{int(l[0]), mk(l[1], l[2], l[3]), mk(l[4], l[5], l[6]), l[7]};
  }
  if (mats.empty()) return -1;
  Ctx x;
  x.P = &P;
  x.mats = &mats;
  x.lights = &lights;
  x.env.faces = job->env_faces;
  x.env.size = job->env_size;
  x.env.intensity = job->env_intensity;
  x.env.max_clamp = job->env_clamp;
  x.max_depth = job->max_depth;
  x.bvh = job->use_bvh != 0;
  const Camera cam = cam_from(job->cam);
  const int W = job->width, H = job->height, TS = 32;
  const int ntx = (W + TS - 1) / TS, nty = (H + TS - 1) / TS, ntiles = ntx * nty;
  const int G = job->shard_count > 0 ? job->shard_count : 1, R = job->shard_rank;
  std::atomic<int> next{0};
  std::atomic<uint64_t> c_closest{0}, c_shadow{0}, c_samples{0}, c_bounces{0};
  auto pixel = [&](int xx, int y, Counters& cnt) {
    const uint32_t ps = uint32_t(y * W + xx);
    float* acc = job->accum + size_t(ps) * 3;
    V3 a = mk(acc[0], acc[1], acc[2]);
    for (uint32_t f = 0; f < job->num_frames; ++f) {
      const uint32_t n = job->frame_begin + f;
      uint32_t r = wang_hash(ps ^ n * 9781u);
      const float jx = rand01(r), jy = rand01(r);
      const V3 d = ray_dir(cam, (float(xx) + jx) / float(W), (float(y) + jy) / float(H));
      const V3 c = trace_path(x, cam.pos, d, ps ^ n, 1, cnt);
      a = a + c;
      ++cnt.samples;
    }
    acc[0] = a.x; acc[1] = a.y; acc[2] = a.z;
    if (job->rgb) resolve_pixel(a, job->frame_begin + job->num_frames - 1, job->rgb + size_t(ps) * 3);
  };
  auto worker = [&]() {
    Counters cnt;
    if (job->pixels) {  // a pixel list (residue diagnosis): 64 pixels per grab
      for (;;) {
        const uint32_t i0 = uint32_t(next.fetch_add(64));
        if (i0 >= job->num_pixels) break;
        for (uint32_t i = i0; i < std::min(i0 + 64u, job->num_pixels); ++i) {
          const uint32_t ps = job->pixels[i];
          if (ps < uint32_t(W) * uint32_t(H)) pixel(int(ps % uint32_t(W)), int(ps / uint32_t(W)), cnt);
        }
      }
    } else {
      for (;;) {
        const int t = next.fetch_add(1);
        if (t >= ntiles) break;
        if (t % G != R) continue;
        const int tx = t % ntx, ty = t / ntx;
        const int x0 = tx * TS, y0 = ty * TS, x1 = std::min(x0 + TS, W), y1 = std::min(y0 + TS, H);
        for (int y = y0; y < y1; ++y)
          for (int xx = x0; xx < x1; ++xx) pixel(xx, y, cnt);
      }
    }
    c_closest += cnt.closest;
    c_shadow += cnt.shadow;
    c_samples += cnt.samples;
    c_bounces += cnt.bounces;
  };
  int nt = job->threads > 0 ? job->threads : int(std::thread::hardware_concurrency());
  if (nt < 1) nt = 1;
  std::vector<std::thread> pool;
  for (int i = 1; i < nt; ++i) pool.emplace_back(worker);
  worker();
  for (auto& th : pool) th.join();
  job->counters[0] = c_closest;
  job->counters[1] = c_shadow;
  job->counters[2] = c_samples;
  job->counters[3] = c_bounces;
  return 0;
}

// Residue diagnosis: the rays of pixel (px, py)'s wavefront path at accumulation index `frame` (the job's
// scene state, camera and frame size), in trace order, 9 floats each (see log_ray); returns the count
// (at most cap are written).
int oracle_path_rays(void* h, oracle_job* job, int px, int py, uint32_t frame, float* out, int cap) {
  const Prepared& P = *static_cast<Prepared*>(h);
  std::vector<Material> mats(job->num_materials);
  for (uint32_t i = 0; i < job->num_materials; ++i) {
    const float* m = job->materials + i * 12;
    mats[i] = Material{mk(m[0], m[1], m[2]), m[3], m[4], mk(m[5], m[6], m[7]), m[8], int(m[9])};
  }
  std::vector<Light> lights(job->num_lights);
  for (uint32_t i = 0; i < job->num_lights; ++i) {
    const float* l = job->lights + i * 8;
    lights[i] = Light{int(l[0]), mk(l[1], l[2], l[3]), mk(l[4], l[5], l[6]), l[7]};
  }
  if (mats.empty()) return -1;
  Ctx x;
  x.P = &P;
  x.mats = &mats;
  x.lights = &lights;
  x.env.faces = job->env_faces;
  x.env.size = job->env_size;
  x.env.intensity = job->env_intensity;
  x.env.max_clamp = job->env_clamp;
  x.max_depth = job->max_depth;
  x.bvh = job->use_bvh != 0;
  const Camera cam = cam_from(job->cam);
  const int W = job->width, H = job->height;
  const uint32_t ps = uint32_t(py * W + px);
  uint32_t r = wang_hash(ps ^ frame * 9781u);
  const float jx = rand01(r), jy = rand01(r);
  const V3 d = ray_dir(cam, (float(px) + jx) / float(W), (float(py) + jy) / float(H));
  std::vector<float> log;
  Counters cnt;
  g_raylog = &log;
  (void)trace_path(x, cam.pos, d, ps ^ frame, 1, cnt);
  g_raylog = nullptr;
  const int n = int(log.size() / 9);
  for (int i = 0; i < std::min(n, cap) * 9; ++i) out[i] = log[size_t(i)];
  return n;
}

// PathTracer-mode render (PathTracer::renderImage / renderTileTask / traceRay, PathTracer.cpp:280-389):
// per pixel the corner ray u = x/W, v = y/H; per frame `samples_per_frame` paths averaged, ACES, gamma;
// accum += frame colour; rgb = clamp(accum / frames) * 255.  Same tiles / shards / threads as
// oracle_render.
int oracle_render_pt(void* h, oracle_job* job, uint32_t samples_per_frame) {
  const Prepared& P = *static_cast<Prepared*>(h);
  std::vector<Material> mats(job->num_materials);
  for (uint32_t i = 0; i < job->num_materials; ++i) {
    const float* m = job->materials + i * 12;
    mats[i] = Material{mk(m[0], m[1], m[2]), m[3], m[4], mk(m[5], m[6], m[7]), m[8], int(m[9])};
  }
  std::vector<Light> lights(job->num_lights);
  for (uint32_t i = 0; i < job->num_lights; ++i) {
    const float* l = job->lights + i * 8;
    lights[i] = Light{int(l[0]), mk(l[1], l[2], l[3]), mk(l[4], l[5], l[6]), l[7]};
  }
  if (mats.empty() || samples_per_frame == 0) return -1;
  Ctx x;
  x.P = &P;
  x.mats = &mats;
  x.lights = &lights;
  x.env.faces = job->env_faces;
  x.env.size = job->env_size;
  x.env.intensity = job->env_intensity;
  x.env.max_clamp = job->env_clamp;
  x.max_depth = job->max_depth;
  x.bvh = job->use_bvh != 0;
  const Camera cam = cam_from(job->cam);
  const int W = job->width, H = job->height, TS = 32;
  const int ntx = (W + TS - 1) / TS, nty = (H + TS - 1) / TS, ntiles = ntx * nty;
  const int G = job->shard_count > 0 ? job->shard_count : 1, R = job->shard_rank;
  std::atomic<int> next{0};
  std::atomic<uint64_t> c_closest{0}, c_shadow{0}, c_samples{0};
  auto worker = [&]() {
    Counters cnt;
    for (;;) {
      const int t = next.fetch_add(1);
      if (t >= ntiles) break;
      if (t % G != R) continue;
      const int tx = t % ntx, ty = t / ntx;
      const int x0 = tx * TS, y0 = ty * TS, x1 = std::min(x0 + TS, W), y1 = std::min(y0 + TS, H);
      for (int y = y0; y < y1; ++y)
        for (int xx = x0; xx < x1; ++xx) {
          const uint32_t ps = uint32_t(y * W + xx);
          float* acc = job->accum + size_t(ps) * 3;
          V3 a = mk(acc[0], acc[1], acc[2]);
          const V3 dir = ray_dir(cam, float(xx) / float(W), float(y) / float(H));
          for (uint32_t f = 0; f < job->num_frames; ++f) {
            const uint32_t n = job->frame_begin + f;
            V3 c = mk(0, 0, 0);
            for (uint32_t s = 0; s < samples_per_frame; ++s) {
              uint32_t rng = pt_seed(ps, n, s);
              c = c + pt_path(x, cam.pos, dir, rng, cnt);
              ++cnt.samples;
            }
            c = c / float(samples_per_frame);
            const float ka = 2.51f, kb = 0.03f, kc = 2.43f, kd = 0.59f, ke = 0.14f;  // acesToneMapping
            c = gclamp((c * (ka * c + kb)) / (c * (kc * c + kd) + ke), 0.0f, 1.0f);
            const float g = 1.0f / 2.2f;
            c = mk(std::pow(c.x, g), std::pow(c.y, g), std::pow(c.z, g));
            a = a + c;
          }
          acc[0] = a.x; acc[1] = a.y; acc[2] = a.z;
          if (job->rgb) {
            const uint32_t frames = job->frame_begin + job->num_frames - 1;
            const V3 avg = gclamp(a / float(frames), 0.0f, 1.0f);
            uint8_t* o = job->rgb + size_t(ps) * 3;
            o[0] = static_cast<unsigned char>(avg.x * 255.0f);
            o[1] = static_cast<unsigned char>(avg.y * 255.0f);
            o[2] = static_cast<unsigned char>(avg.z * 255.0f);
          }
        }
    }
    c_closest += cnt.closest;
    c_shadow += cnt.shadow;
    c_samples += cnt.samples;
  };
  int nt = job->threads > 0 ? job->threads : int(std::thread::hardware_concurrency());
  if (nt < 1) nt = 1;
  std::vector<std::thread> pool;
  for (int i = 1; i < nt; ++i) pool.emplace_back(worker);
  worker();
  for (auto& th : pool) th.join();
  job->counters[0] = c_closest;
  job->counters[1] = c_shadow;
  job->counters[2] = c_samples;
  job->counters[3] = 0;
  return 0;
}

// OptiX-mode render (the reference's OptiX wavefront programs, restated path per thread): per pixel
// and frame one path from the pixel centre; accum.xyz += contributions, count += 1 per frame
// (accum_w: width*height floats, read-modify-write); rgb = __raygen__resolve of accum / count.
int oracle_render_optix(void* h, oracle_job* job, float* accum_w) {
  const Prepared& P = *static_cast<Prepared*>(h);
  std::vector<Material> mats(job->num_materials);
  for (uint32_t i = 0; i < job->num_materials; ++i) {
    const float* m = job->materials + i * 12;
    mats[i] = Material{mk(m[0], m[1], m[2]), m[3], m[4], mk(m[5], m[6], m[7]), m[8], int(m[9])};
  }
  if (mats.empty()) return -1;
  Ctx x;
  x.P = &P;
  x.mats = &mats;
  x.lights = nullptr;
  x.env.faces = job->env_faces;
  x.env.size = job->env_size;
  x.env.intensity = job->env_intensity;
  x.env.max_clamp = job->env_clamp;
  x.max_depth = job->max_depth;
  x.bvh = job->use_bvh != 0;
  const Camera cam = cam_from(job->cam);
  // OptixBackend::render camera basis (OptixBackend.cpp:1515-1620)
  OxFrame F;
  {
    const V3 fwd = normalize(cam.fwd), right = normalize(cam.right), up = normalize(cam.up);
    const V3 dx = ray_dir(cam, 1.0f, 0.5f), dy = ray_dir(cam, 0.5f, 0.0f);
    const float den_x = dot(dx, fwd), den_y = dot(dy, fwd);
    const float hw = den_x != 0.0f ? dot(dx, right) / den_x : 0.0f;
    const float hh = den_y != 0.0f ? dot(dy, up) / den_y : 0.0f;
    F.u = right * hw;
    F.v = up * hh;
    F.w = fwd;
    F.has_light = false;
    F.light_dir = mk(0, -1, 0);
    F.light_rad = mk(0, 0, 0);
    for (uint32_t i = 0; i < job->num_lights; ++i) {
      const float* l = job->lights + i * 8;
      if (int(l[0]) != 0) continue;
      const V3 to_light = normalize(-mk(l[1], l[2], l[3]));  // DirectionalLight stores normalize(-d)
      F.light_dir = -to_light;
      F.light_rad = mk(l[4], l[5], l[6]) * l[7];
      F.has_light = true;
      break;
    }
  }
  const int W = job->width, H = job->height, TS = 32;
  const int ntx = (W + TS - 1) / TS, nty = (H + TS - 1) / TS, ntiles = ntx * nty;
  const int G = job->shard_count > 0 ? job->shard_count : 1, R = job->shard_rank;
  std::atomic<int> next{0};
  std::atomic<uint64_t> c_closest{0}, c_samples{0};
  auto worker = [&]() {
    Counters cnt;
    for (;;) {
      const int t = next.fetch_add(1);
      if (t >= ntiles) break;
      if (t % G != R) continue;
      const int tx = t % ntx, ty = t / ntx;
      const int x0 = tx * TS, y0 = ty * TS, x1 = std::min(x0 + TS, W), y1 = std::min(y0 + TS, H);
      for (int y = y0; y < y1; ++y)
        for (int xx = x0; xx < x1; ++xx) {
          const uint32_t pixel = uint32_t(y * W + xx);
          float* acc = job->accum + size_t(pixel) * 3;
          V3 a = mk(acc[0], acc[1], acc[2]);
          float wcnt = accum_w[pixel];
          const float ndx = ((float(xx) + 0.5f) / float(W)) * 2.0f - 1.0f;
          const float ndy = 1.0f - ((float(y) + 0.5f) / float(H)) * 2.0f;
          const V3 dir = ox_nrm((F.u * ndx + F.v * ndy) + F.w);
          for (uint32_t f = 0; f < job->num_frames; ++f) {
            const uint32_t frame = job->frame_begin + f - 1u;
            const uint32_t rng = wang_hash((pixel + 1u) ^ (frame * 9781u + 1u));
            ox_path(x, F, cam.pos, dir, rng, a, cnt);
            wcnt = wcnt + 1.0f;
            ++cnt.samples;
          }
          acc[0] = a.x; acc[1] = a.y; acc[2] = a.z;
          accum_w[pixel] = wcnt;
          if (job->rgb) {  // __raygen__resolve
            const float inv = (wcnt > 0.0f) ? (1.0f / wcnt) : 0.0f;
            V3 c = mk(std::max(a.x * inv, 0.0f), std::max(a.y * inv, 0.0f), std::max(a.z * inv, 0.0f));
            c = c * 2.2f;
            c = mk(c.x / (1.0f + c.x), c.y / (1.0f + c.y), c.z / (1.0f + c.z));
            const float g = 1.0f / 2.2f;
            c = mk(std::pow(c.x, g), std::pow(c.y, g), std::pow(c.z, g));
            c = gclamp(c, 0.0f, 1.0f);
            uint8_t* o = job->rgb + size_t(pixel) * 3;
            o[0] = static_cast<unsigned char>(c.x * 255.0f);
            o[1] = static_cast<unsigned char>(c.y * 255.0f);
            o[2] = static_cast<unsigned char>(c.z * 255.0f);
          }
        }
    }
    c_closest += cnt.closest;
    c_samples += cnt.samples;
  };
  int nt = job->threads > 0 ? job->threads : int(std::thread::hardware_concurrency());
  if (nt < 1) nt = 1;
  std::vector<std::thread> pool;
  for (int i = 1; i < nt; ++i) pool.emplace_back(worker);
  worker();
  for (auto& th : pool) th.join();
  job->counters[0] = c_closest;
  job->counters[1] = 0;
  job->counters[2] = c_samples;
  job->counters[3] = 0;
  return 0;
}

// Resolve an accumulation buffer (W*H*3 floats) with n samples into RGB8 (the tile task's display path).
void oracle_resolve(const float* accum, uint32_t npix, uint32_t n, uint8_t* rgb) {
  for (uint32_t i = 0; i < npix; ++i)
    resolve_pixel(mk(accum[i * 3], accum[i * 3 + 1], accum[i * 3 + 2]), n, rgb + size_t(i) * 3);
}

}  // extern "C"
