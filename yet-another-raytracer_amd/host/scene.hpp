// scene.hpp — C++ host mirror of the reference's scene-description surface.
//
// The reference builds scenes from Rust trait objects (Hittable hittable.rs:11-35, Material
// material.rs:20-31, Texture texture.rs:13-16) and hands an Arc<HittableList> to its render
// loop. This header keeps the same names and constructor arguments so that presets read like
// scenes.rs, and adds one thing the reference does not have: flatten(), which walks the
// object tree once into the plain yart_scene_desc of include/yart.h (the drop-in boundary).
#pragma once

#include <array>
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/yart.h"

namespace yart {

struct Vec3 {  // vec3.rs:13-247 (host-side values only)
  double e[3] = {0.0, 0.0, 0.0};
  Vec3() = default;
  Vec3(double x, double y, double z) : e{x, y, z} {}
  double x() const { return e[0]; }
  double y() const { return e[1]; }
  double z() const { return e[2]; }
  Vec3 operator-(const Vec3& o) const { return {e[0] - o.e[0], e[1] - o.e[1], e[2] - o.e[2]}; }
  Vec3 operator+(const Vec3& o) const { return {e[0] + o.e[0], e[1] + o.e[1], e[2] + o.e[2]}; }
  double length() const;
};
using RGB = Vec3;  // color.rs:25-28 (same layout, RGB channels)

// ------------------------------------------------------------------ textures (texture.rs)
class SceneRng;
struct Texture {
  uint32_t kind = YART_TEX_SOLID;
  RGB a, b;
  uint32_t noise_type = 0;
  double scale = 0.0;
  std::shared_ptr<const yart_perlin> perlin;  // NOISE: its own tables (Perlin::new per texture)
  uint32_t width = 0, height = 0;              // IMAGE
  std::shared_ptr<const std::vector<uint8_t>> pixels;  // IMAGE: RGB8 rows, top first
};
inline Texture SolidColor(RGB c) { Texture t; t.kind = YART_TEX_SOLID; t.a = c; return t; }       // texture.rs:18-40
inline Texture CheckerTexture(RGB odd, RGB even) { Texture t; t.kind = YART_TEX_CHECKER; t.a = odd; t.b = even; return t; }  // texture.rs:42-68
// NoiseTexture::new (texture.rs:251-260): Perlin::new draws its tables from thread_rng in the
// reference; here from the scene's seeded stream, in the same order (ranfloat, ranvec, perm_x/y/z).
Texture NoiseTexture(uint32_t noise_type, double scale, SceneRng& rng);
// ImageTexture::new (texture.rs:302-318) over a binary PPM (P6) holding the decoded texels of the
// image the reference opens (tools/decode_image.py). Throws std::runtime_error.
Texture ImageTexture(const std::string& ppm_path);

// ----------------------------------------------------------------- materials (material.rs)
struct Material {
  uint32_t kind = YART_MAT_NONE;
  Texture texture;
  double fuzz = 0.0;
  std::array<double, 3> b{{0, 0, 0}}, c{{0, 0, 0}};
};
inline Material Lambertian(Texture t) { Material m; m.kind = YART_MAT_LAMBERTIAN; m.texture = t; return m; }
inline Material Metal(Texture t, double fuzz) { Material m; m.kind = YART_MAT_METAL; m.texture = t; m.fuzz = fuzz; return m; }
inline Material DiffuseLight(Texture t) { Material m; m.kind = YART_MAT_DIFFUSE_LIGHT; m.texture = t; return m; }
inline Material NoMaterial() { return Material{}; }
inline Material Isotropic(Texture t) { Material m; m.kind = YART_MAT_ISOTROPIC; m.texture = t; return m; }  // material.rs:357-381
Material Dielectric(double b1, double b2, double b3, double c1, double c2, double c3);
// Glass presets, material.rs:121-185 (C in nm^2).
extern const Material BAF10, BK7, SF11, FK51A, LASF9, SF66;

// -------------------------------------------------------------------------- geometry
class Flattener;

class Hittable {  // hittable.rs:11-35
 public:
  virtual ~Hittable() = default;
  // Append this object's primitives to `f` under the wrapper chain `chain` (outermost first).
  virtual void flatten(Flattener& f, std::vector<yart_xform>& chain) const = 0;
};
using HittablePtr = std::shared_ptr<Hittable>;

class HittableList : public Hittable {  // hittable.rs:47-123
 public:
  std::vector<HittablePtr> objects;
  void add_object(HittablePtr o) { objects.push_back(std::move(o)); }
  size_t size() const { return objects.size(); }
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};

class StillSphere : public Hittable {  // sphere.rs:31-119
 public:
  StillSphere(Vec3 center, double radius, Material m) : center(center), radius(radius), material(m) {}
  Vec3 center; double radius; Material material;
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};

class MovingSphere : public Hittable {  // sphere.rs:121-211
 public:
  MovingSphere(Vec3 center0, Vec3 center1, double time0, double time1, double radius, Material m)
      : center0(center0), center1(center1), time0(time0), time1(time1), radius(radius), material(m) {}
  Vec3 center0, center1; double time0, time1, radius; Material material;
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};

class XYRect : public Hittable {  // aarect.rs:9-77
 public:
  XYRect(double x0, double x1, double y0, double y1, double k, Material m) : p{x0, x1, y0, y1, k}, material(m) {}
  double p[5]; Material material;
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};
class XZRect : public Hittable {  // aarect.rs:79-172
 public:
  XZRect(double x0, double x1, double z0, double z1, double k, Material m) : p{x0, x1, z0, z1, k}, material(m) {}
  double p[5]; Material material;
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};
class YZRect : public Hittable {  // aarect.rs:174-242
 public:
  YZRect(double y0, double y1, double z0, double z1, double k, Material m) : p{y0, y1, z0, z1, k}, material(m) {}
  double p[5]; Material material;
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};

class BoxEntity : public Hittable {  // box_entity.rs:9-75
 public:
  BoxEntity(Vec3 p0, Vec3 p1, Material m) : p0(p0), p1(p1), material(m) {}
  Vec3 p0, p1; Material material;
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};

class Triangle : public Hittable {  // triangle.rs:19-102
 public:
  std::array<Vec3, 3> vertices, normals;
  std::array<std::array<double, 2>, 3> uv{};
  Material material;
  Triangle(std::array<Vec3, 3> v, std::array<Vec3, 3> n, std::array<std::array<double, 2>, 3> uv, Material m)
      : vertices(v), normals(n), uv(uv), material(m) {}
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};

// Triangles as TriangleMesh::from_obj leaves them (triangle.rs:111-174).
struct MeshData {
  std::string source;           // path it was loaded from
  std::vector<float> positions; // 9 per triangle
  std::vector<double> normals;  // 9 per triangle
  std::vector<double> uvs;      // 6 per triangle
  uint32_t n_triangles() const { return (uint32_t)(positions.size() / 9); }
};
// tobj 4.0.2 load_obj with GPU_LOAD_OPTIONS (single_index + triangulate, fan triangulation,
// f32 parse), then the per-triangle defaults of triangle.rs:134-156. Throws std::runtime_error.
std::shared_ptr<const MeshData> load_obj_mesh(const std::string& path);

class TriangleMesh : public Hittable {  // triangle.rs:104-185
 public:
  static std::shared_ptr<TriangleMesh> from_obj(const std::string& path, Material m);
  std::shared_ptr<const MeshData> mesh; Material material;
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};

class Translate : public Hittable {  // hittable.rs:125-163
 public:
  Translate(HittablePtr h, Vec3 offset) : inner(std::move(h)), offset(offset) {}
  HittablePtr inner; Vec3 offset;
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};
class RotateY : public Hittable {  // hittable.rs:165-256
 public:
  RotateY(HittablePtr h, double angle) : inner(std::move(h)), angle(angle) {}
  HittablePtr inner; double angle;
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};
class FlipFace : public Hittable {  // hittable.rs:328-354
 public:
  explicit FlipFace(HittablePtr h) : inner(std::move(h)) {}
  HittablePtr inner;
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};
// ConstantMedium (hittable.rs:258-326): a boundary of ONE primitive (under its own wrappers) and
// an Isotropic phase function; flattened as that primitive with an outermost MEDIUM wrapper.
class ConstantMedium : public Hittable {
 public:
  ConstantMedium(HittablePtr boundary, double density, Texture t)
      : boundary(std::move(boundary)), density(density), phase_function(Isotropic(t)) {}
  HittablePtr boundary; double density; Material phase_function;
  void flatten(Flattener& f, std::vector<yart_xform>& chain) const override;
};

// Owns every array a yart_scene_desc points into.
class SceneDesc {
 public:
  std::vector<yart_object> objects, lights;
  std::vector<yart_material> materials;
  std::vector<yart_texture> textures;
  std::vector<std::shared_ptr<const MeshData>> mesh_data;
  std::vector<std::shared_ptr<const yart_perlin>> perlins;  // tables the noise textures point at
  std::vector<std::shared_ptr<const std::vector<uint8_t>>> images;  // texels the image textures point at
  std::vector<yart_mesh> meshes;
  double background[3] = {0, 0, 0};
  yart_scene_desc desc() const;
};

class Flattener {
 public:
  explicit Flattener(SceneDesc& out) : out_(out) {}
  void begin_list(std::vector<yart_object>* target) { target_ = target; }
  uint32_t material(const Material& m);
  uint32_t mesh(const std::shared_ptr<const MeshData>& m);
  void emit(uint32_t kind, uint32_t material, const std::vector<yart_xform>& chain, const double* p, int np,
            uint32_t mesh = 0);
  // While set, emitted primitives take this material (a medium's phase function) and are counted.
  void override_material(const Material* m) { override_ = m; override_count_ = 0; }
  uint32_t override_count() const { return override_count_; }

 private:
  const Material* override_ = nullptr;
  uint32_t override_count_ = 0;
  uint32_t texture(const Texture& t);
  SceneDesc& out_;
  std::vector<yart_object>* target_ = nullptr;
};

// Flatten a world, its light list and background into one description (the single walk of
// the Hittable tree the boundary needs; the render loop then never touches the tree).
std::unique_ptr<SceneDesc> flatten_scene(const HittableList& world, const HittableList& lights, RGB background);

// --------------------------------------------------------------- presets (main.rs:211-432)
struct RenderDefaults {  // main.rs:109-118
  uint32_t width = 1200, height = 800;
  uint64_t samples_per_pixel = 100, max_depth = 50, workers = 30;
  double vfov = 20.0, aperture = 0.0;
};
struct ScenePreset {  // main.rs:132-140
  RenderDefaults defaults;
  std::string output_filename;
  RGB background;
  Vec3 lookfrom, lookat;
  std::shared_ptr<HittableList> world;
  HittableList lights;
  std::string stand_in;  // non-empty when a missing input mesh was replaced
};
// Scene names as the reference's clap ValueEnum spells them (main.rs:61-76).
const std::vector<std::string>& scene_names();
// asset_dir holds the reference's input/*.obj; scene_seed drives random_scene's draws.
ScenePreset build_scene_preset(const std::string& name, const std::string& asset_dir, uint64_t scene_seed);

// Seeded stand-in for the reference's thread_rng in scene construction (scenes.rs:34): the same
// Philox4x32-10 stream and rand 0.8.5 mappings the renderer uses, on stream id 1.
class SceneRng {
 public:
  explicit SceneRng(uint64_t seed);
  double gen_f64();                       // rng.gen::<f64>()
  double gen_range(double low, double high);  // rng.gen_range(low..high)
  uint64_t gen_index(uint64_t n);         // rng.gen_range(0..n) for usize (rand 0.8.5 UniformInt)
 private:
  uint64_t next_u64();
  uint32_t key_[2], ctr_[4], buf_[4];
  int have_ = 0;
};

}  // namespace yart
