// scene.cpp — flattening of the C++ scene mirror into yart_scene_desc, the tobj-compatible
// OBJ loader, the glass presets and the seeded scene RNG.
#include "scene.hpp"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <stdexcept>

namespace yart {

double Vec3::length() const { return std::sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]); }

Material Dielectric(double b1, double b2, double b3, double c1, double c2, double c3) {
  Material m;
  m.kind = YART_MAT_DIELECTRIC;
  m.b = {{b1, b2, b3}};
  m.c = {{c1, c2, c3}};
  return m;
}
// material.rs:121-185 (the products are the reference's own constant expressions)
const Material BAF10 = Dielectric(1.5851495, 0.143559385, 1.08521269, 0.00926681282 * 1e6, 0.0424489805 * 1e6, 105.613573 * 1e6);
const Material BK7 = Dielectric(1.03961212, 0.231792344, 1.01046945, 0.00600069867, 0.0200179144, 103.560653);
const Material SF11 = Dielectric(1.73759695, 0.313747346, 1.89878101, 0.013188707 * 1e6, 0.0623068142 * 1e6, 155.23629 * 1e6);
const Material FK51A = Dielectric(0.971247817, 0.216901417, 0.904651666, 0.00472301995, 0.0153575612, 168.68133);
const Material LASF9 = Dielectric(2.00029547, 0.298926886, 1.80691843, 0.0121426017, 0.0538736236, 156.530829);
const Material SF66 = Dielectric(2.0245976, 0.470187196, 2.59970433, 0.0147053225 * 1e6, 0.0692998276 * 1e6, 161.817601 * 1e6);

// ------------------------------------------------------------------------ flattening
static bool same_texture(const yart_texture& a, const Texture& t) {
  return a.kind == t.kind && !std::memcmp(a.rgb, t.a.e, sizeof a.rgb) && !std::memcmp(a.rgb_even, t.b.e, sizeof a.rgb_even) &&
         a.noise_type == t.noise_type && a.scale == t.scale && a.perlin == t.perlin.get() &&
         a.pixels == (t.pixels ? t.pixels->data() : nullptr);
}
uint32_t Flattener::texture(const Texture& t) {
  for (size_t i = 0; i < out_.textures.size(); ++i)
    if (same_texture(out_.textures[i], t)) return (uint32_t)i;
  yart_texture y{};
  y.kind = t.kind;
  std::memcpy(y.rgb, t.a.e, sizeof y.rgb);
  std::memcpy(y.rgb_even, t.b.e, sizeof y.rgb_even);
  y.noise_type = t.noise_type;
  y.scale = t.scale;
  if (t.perlin) {
    out_.perlins.push_back(t.perlin);
    y.perlin = t.perlin.get();
  }
  if (t.pixels) {
    out_.images.push_back(t.pixels);
    y.pixels = t.pixels->data();
    y.width = t.width;
    y.height = t.height;
  }
  out_.textures.push_back(y);
  return (uint32_t)(out_.textures.size() - 1);
}
uint32_t Flattener::material(const Material& m) {
  yart_material y{};
  y.kind = m.kind;
  y.texture = (m.kind == YART_MAT_LAMBERTIAN || m.kind == YART_MAT_METAL || m.kind == YART_MAT_DIFFUSE_LIGHT ||
               m.kind == YART_MAT_ISOTROPIC) ? texture(m.texture) : 0;
  y.fuzz = m.fuzz;
  for (int i = 0; i < 3; ++i) { y.b[i] = m.b[i]; y.c[i] = m.c[i]; }
  for (size_t i = 0; i < out_.materials.size(); ++i)
    if (!std::memcmp(&out_.materials[i], &y, sizeof y)) return (uint32_t)i;
  out_.materials.push_back(y);
  return (uint32_t)(out_.materials.size() - 1);
}
uint32_t Flattener::mesh(const std::shared_ptr<const MeshData>& m) {
  for (size_t i = 0; i < out_.mesh_data.size(); ++i)
    if (out_.mesh_data[i] == m) return (uint32_t)i;
  out_.mesh_data.push_back(m);
  yart_mesh y{};
  y.n_triangles = m->n_triangles();
  y.positions = m->positions.data();
  y.normals = m->normals.data();
  y.uvs = m->uvs.empty() ? nullptr : m->uvs.data();
  out_.meshes.push_back(y);
  return (uint32_t)(out_.meshes.size() - 1);
}
void Flattener::emit(uint32_t kind, uint32_t material, const std::vector<yart_xform>& chain, const double* p, int np,
                     uint32_t mesh) {
  if (chain.size() > YART_MAX_XFORMS) throw std::runtime_error("more than YART_MAX_XFORMS nested wrappers");
  yart_object o{};
  o.kind = kind;
  o.material = override_ ? this->material(*override_) : material;
  if (override_) override_count_++;
  o.mesh = mesh;
  o.n_xforms = (uint32_t)chain.size();
  for (size_t i = 0; i < chain.size(); ++i) o.xforms[i] = chain[i];
  for (int i = 0; i < np; ++i) o.p[i] = p[i];
  target_->push_back(o);
}

void HittableList::flatten(Flattener& f, std::vector<yart_xform>& chain) const {
  // A nested list hits as its closest member (hittable.rs:67-79); flattening it in place under
  // the same wrappers keeps both the closest hit and the later-wins tie order.
  for (const auto& o : objects) o->flatten(f, chain);
}
void StillSphere::flatten(Flattener& f, std::vector<yart_xform>& chain) const {
  double p[4] = {center.x(), center.y(), center.z(), radius};
  f.emit(YART_PRIM_SPHERE, f.material(material), chain, p, 4);
}
void MovingSphere::flatten(Flattener& f, std::vector<yart_xform>& chain) const {
  double p[9] = {center0.x(), center0.y(), center0.z(), center1.x(), center1.y(), center1.z(), time0, time1, radius};
  f.emit(YART_PRIM_MOVING_SPHERE, f.material(material), chain, p, 9);
}
void XYRect::flatten(Flattener& f, std::vector<yart_xform>& chain) const { f.emit(YART_PRIM_XY_RECT, f.material(material), chain, p, 5); }
void XZRect::flatten(Flattener& f, std::vector<yart_xform>& chain) const { f.emit(YART_PRIM_XZ_RECT, f.material(material), chain, p, 5); }
void YZRect::flatten(Flattener& f, std::vector<yart_xform>& chain) const { f.emit(YART_PRIM_YZ_RECT, f.material(material), chain, p, 5); }
void BoxEntity::flatten(Flattener& f, std::vector<yart_xform>& chain) const {
  double p[6] = {p0.x(), p0.y(), p0.z(), p1.x(), p1.y(), p1.z()};
  f.emit(YART_PRIM_BOX, f.material(material), chain, p, 6);
}
void Triangle::flatten(Flattener& f, std::vector<yart_xform>& chain) const {
  double p[24];
  for (int k = 0; k < 3; ++k)
    for (int j = 0; j < 3; ++j) { p[3 * k + j] = vertices[k].e[j]; p[9 + 3 * k + j] = normals[k].e[j]; }
  for (int k = 0; k < 3; ++k) { p[18 + 2 * k] = uv[k][0]; p[19 + 2 * k] = uv[k][1]; }
  f.emit(YART_PRIM_TRIANGLE, f.material(material), chain, p, 24);
}
void TriangleMesh::flatten(Flattener& f, std::vector<yart_xform>& chain) const {
  f.emit(YART_PRIM_MESH, f.material(material), chain, nullptr, 0, f.mesh(mesh));
}
void Translate::flatten(Flattener& f, std::vector<yart_xform>& chain) const {
  yart_xform x{};
  x.kind = YART_XF_TRANSLATE;
  x.v[0] = offset.x(); x.v[1] = offset.y(); x.v[2] = offset.z();
  chain.push_back(x);
  inner->flatten(f, chain);
  chain.pop_back();
}
void RotateY::flatten(Flattener& f, std::vector<yart_xform>& chain) const {
  yart_xform x{};
  x.kind = YART_XF_ROTATE_Y;
  x.v[0] = angle;
  chain.push_back(x);
  inner->flatten(f, chain);
  chain.pop_back();
}
void FlipFace::flatten(Flattener& f, std::vector<yart_xform>& chain) const {
  yart_xform x{};
  x.kind = YART_XF_FLIP_FACE;
  chain.push_back(x);
  inner->flatten(f, chain);
  chain.pop_back();
}

void ConstantMedium::flatten(Flattener& f, std::vector<yart_xform>& chain) const {
  if (!chain.empty()) throw std::runtime_error("ConstantMedium under another wrapper is not supported");
  yart_xform x{};
  x.kind = YART_XF_MEDIUM;
  x.v[0] = density;
  chain.push_back(x);
  f.override_material(&phase_function);
  boundary->flatten(f, chain);
  const uint32_t n = f.override_count();
  f.override_material(nullptr);
  chain.pop_back();
  if (n != 1) throw std::runtime_error("a ConstantMedium boundary must be one primitive");
}

Texture ImageTexture(const std::string& ppm_path) {
  std::ifstream in(ppm_path, std::ios::binary);
  if (!in) throw std::runtime_error("cannot open image " + ppm_path + " (decode it with tools/decode_image.py)");
  auto token = [&in]() {
    std::string t;
    char c;
    while (in.get(c)) {
      if (c == '#') { std::string skip; std::getline(in, skip); continue; }
      if (std::isspace((unsigned char)c)) { if (!t.empty()) break; continue; }
      t.push_back(c);
    }
    return t;
  };
  if (token() != "P6") throw std::runtime_error(ppm_path + ": not a binary PPM (P6)");
  const long w = std::stol(token()), h = std::stol(token()), maxv = std::stol(token());
  if (w <= 0 || h <= 0 || maxv != 255) throw std::runtime_error(ppm_path + ": unsupported PPM header");
  auto px = std::make_shared<std::vector<uint8_t>>((size_t)w * (size_t)h * 3);
  if (!in.read(reinterpret_cast<char*>(px->data()), (std::streamsize)px->size()))
    throw std::runtime_error(ppm_path + ": truncated PPM");
  Texture t;
  t.kind = YART_TEX_IMAGE;
  t.width = (uint32_t)w;
  t.height = (uint32_t)h;
  t.pixels = px;
  return t;
}

Texture NoiseTexture(uint32_t noise_type, double scale, SceneRng& rng) {
  auto P = std::make_shared<yart_perlin>();
  for (int i = 0; i < 256; ++i) P->ranfloat[i] = rng.gen_range(0.0, 1.0);  // texture.rs:99-101
  for (int i = 0; i < 256; ++i)                                             // Vec3::random(-1, 1)
    for (int k = 0; k < 3; ++k) P->ranvec[i][k] = rng.gen_range(-1.0, 1.0);
  int32_t* perms[3] = {P->perm_x, P->perm_y, P->perm_z};
  for (int32_t* p : perms) {  // perlin_generate_perm + permute (texture.rs:182-190)
    for (int i = 0; i < 256; ++i) p[i] = i;
    for (int i = 255; i >= 1; --i) {
      const uint64_t target = rng.gen_index((uint64_t)i);
      std::swap(p[i], p[target]);
    }
  }
  Texture t;
  t.kind = YART_TEX_NOISE;
  t.a = RGB(1.0, 1.0, 1.0);  // the RGB::new(1, 1, 1) it reflects (texture.rs:272-296)
  t.noise_type = noise_type;
  t.scale = scale;
  t.perlin = P;
  return t;
}

yart_scene_desc SceneDesc::desc() const {
  yart_scene_desc d{};
  d.abi_version = YART_ABI_VERSION;
  d.n_objects = (uint32_t)objects.size();
  d.n_lights = (uint32_t)lights.size();
  d.n_materials = (uint32_t)materials.size();
  d.n_textures = (uint32_t)textures.size();
  d.n_meshes = (uint32_t)meshes.size();
  d.objects = objects.data();
  d.lights = lights.data();
  d.materials = materials.data();
  d.textures = textures.data();
  d.meshes = meshes.data();
  for (int i = 0; i < 3; ++i) d.background[i] = background[i];
  return d;
}

std::unique_ptr<SceneDesc> flatten_scene(const HittableList& world, const HittableList& lights, RGB background) {
  auto out = std::make_unique<SceneDesc>();
  Flattener f(*out);
  std::vector<yart_xform> chain;
  f.begin_list(&out->objects);
  world.flatten(f, chain);
  f.begin_list(&out->lights);
  lights.flatten(f, chain);
  for (int i = 0; i < 3; ++i) out->background[i] = background.e[i];
  return out;
}

// ------------------------------------------------------------------------ OBJ loading
// tobj 4.0.2, GPU_LOAD_OPTIONS = { single_index, triangulate, ignore_points, ignore_lines }:
// "v"/"vt"/"vn" parsed as f32; every face fan-triangulated (v0, vk, vk+1) in file order; all
// models concatenated in file order (triangle.rs:433-485). Corners without a normal get the
// face normal unit((v1-v0) x (v2-v0)) computed in f64; corners without a uv get (0, 0).
namespace {
struct Corner { long v = 0, t = 0, n = 0; bool has_t = false, has_n = false; };

long resolve_index(long idx, size_t count) {  // 1-based, negative = relative to the end
  if (idx > 0) return idx - 1;
  if (idx < 0) return (long)count + idx;
  return -1;
}
bool parse_corner(const char* s, Corner& c, size_t nv, size_t nt, size_t nn) {
  char* end;
  long v = std::strtol(s, &end, 10);
  c.v = resolve_index(v, nv);
  if (*end == '/') {
    const char* q = end + 1;
    if (*q != '/') {
      long t = std::strtol(q, &end, 10);
      c.t = resolve_index(t, nt); c.has_t = true;
    } else {
      end = (char*)q;
    }
    if (*end == '/') {
      long n = std::strtol(end + 1, &end, 10);
      c.n = resolve_index(n, nn); c.has_n = true;
    }
  }
  return c.v >= 0 && (size_t)c.v < nv && (!c.has_t || (c.t >= 0 && (size_t)c.t < nt)) &&
         (!c.has_n || (c.n >= 0 && (size_t)c.n < nn));
}
}  // namespace

std::shared_ptr<const MeshData> load_obj_mesh(const std::string& path) {
  static std::mutex mu;
  static std::map<std::string, std::weak_ptr<const MeshData>> cache;  // from_obj twice on one file shares it
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(path);
    if (it != cache.end())
      if (auto sp = it->second.lock()) return sp;
  }
  std::ifstream in(path);
  if (!in) throw std::runtime_error("Failed to load OBJ file: " + path);  // triangle.rs:113
  std::vector<float> pos, tex, nrm;
  auto m = std::make_shared<MeshData>();
  m->source = path;
  std::string line;
  std::vector<Corner> face;
  while (std::getline(in, line)) {
    const char* s = line.c_str();
    while (*s == ' ' || *s == '\t') ++s;
    if (s[0] == 'v' && (s[1] == ' ' || s[1] == '\t')) {
      float a[3] = {0, 0, 0};
      char* e = (char*)s + 2;
      for (int i = 0; i < 3; ++i) a[i] = std::strtof(e, &e);
      pos.insert(pos.end(), a, a + 3);
    } else if (s[0] == 'v' && s[1] == 't' && (s[2] == ' ' || s[2] == '\t')) {
      char* e = (char*)s + 3;
      float u = std::strtof(e, &e), v = std::strtof(e, &e);
      tex.push_back(u); tex.push_back(v);
    } else if (s[0] == 'v' && s[1] == 'n' && (s[2] == ' ' || s[2] == '\t')) {
      float a[3];
      char* e = (char*)s + 3;
      for (int i = 0; i < 3; ++i) a[i] = std::strtof(e, &e);
      nrm.insert(nrm.end(), a, a + 3);
    } else if (s[0] == 'f' && (s[1] == ' ' || s[1] == '\t')) {
      face.clear();
      std::istringstream ss(s + 2);
      std::string tok;
      while (ss >> tok) {
        Corner c;
        if (!parse_corner(tok.c_str(), c, pos.size() / 3, tex.size() / 2, nrm.size() / 3))
          throw std::runtime_error("Failed to load OBJ file: bad face index in " + path);
        face.push_back(c);
      }
      for (size_t k = 1; k + 1 < face.size(); ++k) {
        const Corner* cs[3] = {&face[0], &face[k], &face[k + 1]};
        double v[3][3];
        for (int i = 0; i < 3; ++i)
          for (int j = 0; j < 3; ++j) {
            float f = pos[3 * cs[i]->v + j];
            m->positions.push_back(f);
            v[i][j] = (double)f;
          }
        // default_normal = (v1 - v0).cross(v2 - v0).unit_vector()  (triangle.rs:463-465)
        double e1[3] = {v[1][0] - v[0][0], v[1][1] - v[0][1], v[1][2] - v[0][2]};
        double e2[3] = {v[2][0] - v[0][0], v[2][1] - v[0][1], v[2][2] - v[0][2]};
        double cr[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        double len = std::sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
        for (int i = 0; i < 3; ++i) {
          if (cs[i]->has_n)
            for (int j = 0; j < 3; ++j) m->normals.push_back((double)nrm[3 * cs[i]->n + j]);
          else
            for (int j = 0; j < 3; ++j) m->normals.push_back(cr[j] / len);
          if (cs[i]->has_t) { m->uvs.push_back((double)tex[2 * cs[i]->t]); m->uvs.push_back((double)tex[2 * cs[i]->t + 1]); }
          else { m->uvs.push_back(0.0); m->uvs.push_back(0.0); }
        }
      }
    }
  }
  std::lock_guard<std::mutex> g(mu);
  cache[path] = m;
  return m;
}

std::shared_ptr<TriangleMesh> TriangleMesh::from_obj(const std::string& path, Material mat) {
  auto t = std::make_shared<TriangleMesh>();
  t->mesh = load_obj_mesh(path);
  t->material = mat;
  return t;
}

// ------------------------------------------------------------------------ scene RNG
static void philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    c0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0; c1 = (uint32_t)p1;
    c2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1; c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
SceneRng::SceneRng(uint64_t seed) {
  key_[0] = (uint32_t)seed; key_[1] = (uint32_t)(seed >> 32);
  ctr_[0] = 0; ctr_[1] = 0; ctr_[2] = 0; ctr_[3] = 1;  // stream 1 = scene construction
}
uint64_t SceneRng::next_u64() {
  if (have_ == 0) { philox(ctr_, key_, buf_); ctr_[0]++; have_ = 2; }
  int i = 2 - have_; have_--;
  return ((uint64_t)buf_[2 * i + 1] << 32) | buf_[2 * i];
}
double SceneRng::gen_f64() { return (double)(next_u64() >> 11) * 0x1.0p-53; }
uint64_t SceneRng::gen_index(uint64_t n) {  // UniformInt<usize>::sample_single(0..n): zone rejection
  const uint64_t zone = (n << __builtin_clzll(n)) - 1;
  for (;;) {
    const uint64_t v = next_u64();
    const unsigned __int128 m = (unsigned __int128)v * n;
    if ((uint64_t)m <= zone) return (uint64_t)(m >> 64);
  }
}
double SceneRng::gen_range(double low, double high) {
  double scale = high - low;
  for (;;) {
    uint64_t bits = (next_u64() >> 12) | 0x3FF0000000000000ull;
    double v12; std::memcpy(&v12, &bits, 8);
    double res = (v12 - 1.0) * scale + low;
    if (res < high) return res;
    uint64_t sb; std::memcpy(&sb, &scale, 8); sb -= 1; std::memcpy(&scale, &sb, 8);
  }
}

}  // namespace yart
