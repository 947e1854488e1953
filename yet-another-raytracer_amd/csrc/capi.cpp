// capi.cpp — the C ABI of include/yart.h: scene upload to HBM, launches, host conveniences.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/yart.h"
#include "../host/camera_impl.h"
#include "build_id.h"  // generated (Makefile): YART_BUILD_ID
#include "bvh_build.h"
#include "kernels.h"
#include "scene_impl.h"
#include "world_bvh.h"

using namespace yart_dev;
using namespace yart_impl;

namespace yart_impl {
thread_local std::string g_err;
int fail(int code, const std::string& m) { g_err = m; return code; }
int ok() { g_err.clear(); return YART_OK; }

// Test and tuning hooks (yart_debug_set_option): process-wide, read where the behaviour is decided
// (scene creation, frame planning). The library reads no environment variable.
static std::atomic<int64_t> g_opt[YART_OPT_COUNT] = {
    {0},        // YART_OPT_QBVH_TIES_DESC
    {0},        // YART_OPT_QBVH_THREADS (0 = hardware concurrency)
    {1},        // YART_OPT_WALK_TREE
    {0},        // YART_OPT_MESH_WALK_REF
    {-1},       // YART_OPT_WORLD_BVH
    {-1},       // YART_OPT_MESH_WAVEFRONT
    {1 << 20},  // YART_OPT_WF_POOL
    {0},        // YART_OPT_SCRATCH_BYTES (0 = auto: min(16 GiB, device memory / 8))
    {0},        // YART_OPT_UNITS_PER_WAVE (0 = auto: 64 list walk, 192 mesh / world BVH)
    {8}         // YART_OPT_MESH_PARK (busy quads at which a walk parks; 0 = never)
};
int64_t opt(int k) { return k >= 0 && k < YART_OPT_COUNT ? g_opt[k].load(std::memory_order_relaxed) : 0; }
int hip_fail(hipError_t e, const char* what) {
  return fail(YART_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}
}  // namespace yart_impl

namespace {

// Object lists at least this long get a world BVH (the random scene has ~485 spheres; the
// cornell box's 8 entries are walked linearly).
constexpr uint32_t kWorldBvhMinObjects = 16;

// Smits basis spectra (color.rs:1711-1982): white, cyan, magenta, yellow, red, green, blue.
const double kSmits[7][36] = {
#include "smits.inc"
};

// RGB::into_spectrum (color.rs:54-90) at bin i; Spectrum += is `self = rhs + self` from 0.0.
double spectrum_bin(const double rgb[3], int i) {
  enum { W, Cy, Ma, Ye, Re, Gr, Bl };
  const double red = rgb[0], green = rgb[1], blue = rgb[2];
  double s = 0.0;
  if (red <= green && red <= blue) {
    s = red * kSmits[W][i] + s;
    if (green <= blue) { s = (green - red) * kSmits[Cy][i] + s; s = (blue - green) * kSmits[Bl][i] + s; }
    else { s = (blue - red) * kSmits[Cy][i] + s; s = (green - blue) * kSmits[Gr][i] + s; }
  } else if (green <= red && green <= blue) {
    s = green * kSmits[W][i] + s;
    if (red <= blue) { s = (red - green) * kSmits[Ma][i] + s; s = (blue - red) * kSmits[Bl][i] + s; }
    else { s = (blue - green) * kSmits[Ma][i] + s; s = (red - blue) * kSmits[Re][i] + s; }
  } else {
    s = blue * kSmits[W][i] + s;
    if (red <= green) { s = (red - blue) * kSmits[Ye][i] + s; s = (green - red) * kSmits[Gr][i] + s; }
    else { s = (green - blue) * kSmits[Ye][i] + s; s = (red - green) * kSmits[Re][i] + s; }
  }
  return s;
}

template <class T>
hipError_t upload(std::vector<void*>& owned, const T* src, size_t n, const T** dst, uint64_t& bytes) {
  if (n == 0) { *dst = nullptr; return hipSuccess; }
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, sizeof(T) * n);
  if (e != hipSuccess) return e;
  owned.push_back(p);
  bytes += sizeof(T) * n;
  *dst = static_cast<const T*>(p);
  return hipMemcpy(p, src, sizeof(T) * n, hipMemcpyHostToDevice);
}

bool valid_objects(const yart_scene_desc* d, const yart_object* o, uint32_t n, bool lights, std::string& why) {
  for (uint32_t i = 0; i < n; ++i) {
    if (o[i].kind > YART_PRIM_MOVING_SPHERE) { why = "object kind out of range"; return false; }
    if (o[i].n_xforms > YART_MAX_XFORMS) { why = "too many wrappers"; return false; }
    for (uint32_t l = 0; l < o[i].n_xforms; ++l) {
      if (o[i].xforms[l].kind < YART_XF_TRANSLATE || o[i].xforms[l].kind > YART_XF_MEDIUM) { why = "bad wrapper kind"; return false; }
      if (o[i].xforms[l].kind == YART_XF_MEDIUM && l != 0) { why = "a medium must be the outermost wrapper"; return false; }
    }
    if (o[i].n_xforms && o[i].xforms[0].kind == YART_XF_MEDIUM && o[i].kind == YART_PRIM_MESH) {
      why = "a mesh as a medium boundary";
      return false;
    }
    if (o[i].kind == YART_PRIM_MESH && o[i].mesh >= d->n_meshes) { why = "mesh index out of range"; return false; }
    if (!lights && o[i].material >= d->n_materials) { why = "material index out of range"; return false; }
  }
  return true;
}

DevObject to_dev(const yart_object& o) {
  DevObject d{};
  d.kind = o.kind; d.material = o.material; d.mesh = o.mesh; d.n_xf = o.n_xforms;
  for (uint32_t l = 0; l < o.n_xforms && l < (uint32_t)kMaxXforms; ++l) {
    d.xf_kind[l] = o.xforms[l].kind;
    if (o.xforms[l].kind == YART_XF_ROTATE_Y) {  // RotateY::new (hittable.rs:173-176)
      const double radians = o.xforms[l].v[0] * 3.141592653589793 / 180.0;
      // One sincos call, as gcc builds the oracle (it joins the sin and cos of one value into glibc's
      // sincos): glibc's separate sin differs from sincos by an ulp for some angles (160.037...°:
      // 0.34141019606902406 vs ...401). This matches the oracle; whether the reference's rustc build
      // calls sincos or sin and cos is not pinned (ulp-level parity at such angles unpinned).
      double sn, cs;
      ::sincos(radians, &sn, &cs);
      d.xf[l][0] = sn;
      d.xf[l][1] = cs;
    } else if (o.xforms[l].kind == YART_XF_MEDIUM) {  // ConstantMedium::new (hittable.rs:270)
      d.xf[l][0] = -1.0 / o.xforms[l].v[0];
    } else {
      for (int k = 0; k < 3; ++k) d.xf[l][k] = o.xforms[l].v[k];
    }
  }
  for (int k = 0; k < 24; ++k) d.p[k] = o.p[k];
  return d;
}

}  // namespace

yart_scene::~yart_scene() {
  DeviceGuard g(device);
  for (void* p : owned) (void)hipFree(p);
  for (auto& kv : streams) {
    (void)hipFree(kv.second->scratch);
    if (kv.second->wf_mem) (void)hipFree(kv.second->wf_mem);
    if (kv.second->ovf) (void)hipFree(kv.second->ovf);
    if (kv.second->wf_status_host) (void)hipHostFree(kv.second->wf_status_host);
    StreamState& t = *kv.second;
    for (hipStream_t x : {t.aux, t.acc})
      if (x) (void)hipStreamDestroy(x);
    for (hipEvent_t e : {t.ev_start, t.ev_render[0], t.ev_render[1], t.ev_acc[0], t.ev_acc[1]})
      if (e) (void)hipEventDestroy(e);
  }
  for (hipStream_t st : owned_streams) (void)hipStreamDestroy(st);
  for (auto& kv : frames)
    for (auto& f : kv.second)
      for (hipEvent_t e : f) (void)hipEventDestroy(e);
  for (hipEvent_t e : event_pool) (void)hipEventDestroy(e);
}

extern "C" {

const char* yart_version(void) { return "yart-mi355x 0.1 (gfx950, f64 megakernel, ABI 1)"; }
const char* yart_build_id(void) { return YART_BUILD_ID; }  // build/gen/build_id.h (Makefile)
const char* yart_last_error(void) { return g_err.c_str(); }

int yart_device_count(int* out) {
  if (!out) return fail(YART_ERR_INVALID, "null argument");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) { *out = 0; return hip_fail(e, "hipGetDeviceCount"); }
  *out = n;
  return ok();
}

int yart_camera_init(yart_camera* cam, const double lookfrom[3], const double lookat[3], const double vup[3],
                     double vfov, double aspect, double aperture, double focus_dist, double t0, double t1) {
  int rc = yart_camera_init_impl(cam, lookfrom, lookat, vup, vfov, aspect, aperture, focus_dist, t0, t1);
  return rc ? fail(rc, "null argument") : ok();
}

static int scene_create(int device, const yart_scene_desc* d, yart_scene** out) {
  if (!d || !out) return fail(YART_ERR_INVALID, "null argument");
  if (d->abi_version != YART_ABI_VERSION) return fail(YART_ERR_INVALID, "abi_version mismatch");
  if ((d->n_objects && !d->objects) || (d->n_lights && !d->lights) || (d->n_materials && !d->materials) ||
      (d->n_textures && !d->textures) || (d->n_meshes && !d->meshes))
    return fail(YART_ERR_INVALID, "null array with non-zero count");
  std::string why;
  if (!valid_objects(d, d->objects, d->n_objects, false, why) || !valid_objects(d, d->lights, d->n_lights, true, why))
    return fail(YART_ERR_INVALID, why);
  for (uint32_t i = 0; i < d->n_materials; ++i) {
    const yart_material& m = d->materials[i];
    if (m.kind > YART_MAT_ISOTROPIC) return fail(YART_ERR_INVALID, "material kind out of range");
    bool textured = m.kind == YART_MAT_LAMBERTIAN || m.kind == YART_MAT_METAL || m.kind == YART_MAT_DIFFUSE_LIGHT ||
                    m.kind == YART_MAT_ISOTROPIC;
    if (textured && m.texture >= d->n_textures) return fail(YART_ERR_INVALID, "texture index out of range");
  }
  for (uint32_t i = 0; i < d->n_textures; ++i) {
    if (d->textures[i].kind > YART_TEX_IMAGE) return fail(YART_ERR_INVALID, "texture kind out of range");
    if (d->textures[i].kind == YART_TEX_NOISE && (!d->textures[i].perlin || d->textures[i].noise_type > YART_NOISE_NET))
      return fail(YART_ERR_INVALID, "noise texture without Perlin tables or with a bad noise type");
  }
  for (uint32_t i = 0; i < d->n_objects; ++i) {
    const yart_object& o = d->objects[i];
    if (o.kind != YART_PRIM_MESH) continue;
    const yart_material& m = d->materials[o.material];
    if (m.kind != YART_MAT_NONE && m.kind != YART_MAT_DIELECTRIC && m.texture < d->n_textures &&
        d->textures[m.texture].kind == YART_TEX_IMAGE)
      return fail(YART_ERR_UNSUPPORTED, "ImageTexture on a mesh (its texcoords are not uploaded)");
  }
  if (d->n_objects >= kMaxListObjects) return fail(YART_ERR_UNSUPPORTED, "more than 2^29 - 1 world objects");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
  if (device < 0 || device >= ndev) return fail(YART_ERR_INVALID, "device index out of range");

  // host-side preparation (no device work yet)
  std::vector<DevObject> objs, lights;
  for (uint32_t i = 0; i < d->n_objects; ++i) objs.push_back(to_dev(d->objects[i]));
  for (uint32_t i = 0; i < d->n_lights; ++i) lights.push_back(to_dev(d->lights[i]));
  std::vector<DevMaterial> mats(d->n_materials);
  for (uint32_t i = 0; i < d->n_materials; ++i) {
    const yart_material& m = d->materials[i];
    mats[i].kind = m.kind; mats[i].texture = m.texture; mats[i].fuzz = m.fuzz;
    for (int k = 0; k < 3; ++k) { mats[i].b[k] = m.b[k]; mats[i].c[k] = m.c[k]; }
  }
  std::vector<DevTexture> texs(d->n_textures);
  for (uint32_t i = 0; i < d->n_textures; ++i) {
    const yart_texture& t = d->textures[i];
    texs[i].kind = t.kind;
    texs[i].noise_type = t.noise_type;
    texs[i].scale = t.scale;
    texs[i].width = t.kind == YART_TEX_IMAGE && t.pixels ? t.width : 0;
    texs[i].height = t.kind == YART_TEX_IMAGE && t.pixels ? t.height : 0;
    for (int b = 0; b < kBins; ++b) {
      texs[i].spec[b] = spectrum_bin(t.rgb, b);
      texs[i].spec_even[b] = t.kind == YART_TEX_CHECKER ? spectrum_bin(t.rgb_even, b) : 0.0;
    }
  }
  double bg[kBins];
  for (int b = 0; b < kBins; ++b) bg[b] = spectrum_bin(d->background, b);
  std::vector<BuiltMesh> built(d->n_meshes);
  uint32_t nodes = 0, leaves = 0, depth = 0, tied_cuts = 0, tied_leaves = 0, walk_nodes = 0, walk_depth = 0;
  double build_ms = 0.0;
  QbvhOptions qopt;  // the tie-order probe (tests) and the builder's thread count
  qopt.ties_desc = opt(YART_OPT_QBVH_TIES_DESC) != 0;
  qopt.threads = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(opt(YART_OPT_QBVH_THREADS), 1024));
  for (uint32_t m = 0; m < d->n_meshes; ++m) {
    const yart_mesh& ym = d->meshes[m];
    if (!ym.positions || !ym.normals) return fail(YART_ERR_INVALID, "mesh without positions/normals");
    std::string err;
    if (!build_qbvh(ym.n_triangles, ym.positions, ym.normals, built[m], err, qopt)) return fail(YART_ERR_UNSUPPORTED, err);
    // the front-to-back walk's own tree (walk_tree.cpp); YART_OPT_WALK_TREE = 0 walks the reference
    // tree front to back instead. Depth bound: the stack the walk gets (32 slots, 64 for deep meshes).
    if (opt(YART_OPT_WALK_TREE) != 0) {
      const uint32_t slots = 3 * built[m].depth + 1 > (uint32_t)kStackSlots ? (uint32_t)kMaxStackSlots : (uint32_t)kStackSlots;
      build_walk_tree(built[m], (slots - 1) / 3);
    }
    walk_nodes += built[m].walk_nodes;
    walk_depth = std::max(walk_depth, built[m].walk_depth);
    tied_cuts += built[m].tied_cuts;
    tied_leaves += built[m].tied_leaves;
    build_ms += built[m].build_ms + built[m].walk_build_ms;
    nodes += built[m].ref_nodes;
    leaves += (uint32_t)built[m].aux.size();
    depth = std::max(depth, built[m].depth);
  }

  // World BVH (world_bvh.h): for long object lists without meshes; YART_OPT_WORLD_BVH = 0 / 1
  // forces the linear walk / the BVH (when every object has a box).
  BuiltWorld world;
  bool use_world = false;
  {
    bool any_mesh = false;
    for (uint32_t i = 0; i < d->n_objects; ++i) any_mesh |= d->objects[i].kind == YART_PRIM_MESH;
    const int64_t force = opt(YART_OPT_WORLD_BVH);
    const bool want = force == 1 || (force != 0 && d->n_objects >= kWorldBvhMinObjects);
    if (want && !any_mesh) use_world = build_world_bvh(objs, world);
  }

  auto s = std::make_unique<yart_scene>();
  s->device = device;
  DeviceGuard guard(device);
  if (hipDeviceGetAttribute(&s->cu_count, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || s->cu_count <= 0)
    s->cu_count = 256;
  {
    size_t total = 0;
    if (hipDeviceTotalMem(&total, device) == hipSuccess) s->mem_total = total;
  }
  uint64_t bytes = 0;
  DevScene& ds = s->dev;
  const auto up0 = std::chrono::steady_clock::now();
  HIP_TRY(upload(s->owned, objs.data(), objs.size(), &ds.objects, bytes), "upload objects");
  HIP_TRY(upload(s->owned, lights.data(), lights.size(), &ds.lights, bytes), "upload lights");
  HIP_TRY(upload(s->owned, mats.data(), mats.size(), &ds.materials, bytes), "upload materials");
  for (uint32_t i = 0; i < d->n_textures; ++i) {
    if (d->textures[i].kind == YART_TEX_NOISE)
      HIP_TRY(upload(s->owned, d->textures[i].perlin, 1, &texs[i].perlin, bytes), "upload Perlin tables");
    if (d->textures[i].kind == YART_TEX_IMAGE && texs[i].width && texs[i].height)
      HIP_TRY(upload(s->owned, d->textures[i].pixels, (size_t)texs[i].width * texs[i].height * 3, &texs[i].pixels, bytes),
              "upload image texels");
  }
  HIP_TRY(upload(s->owned, texs.data(), texs.size(), &ds.textures, bytes), "upload textures");
  HIP_TRY(upload(s->owned, bg, kBins, &ds.background, bytes), "upload background");
  std::vector<DevMesh> dm(d->n_meshes);
  for (uint32_t m = 0; m < d->n_meshes; ++m) {
    BuiltMesh& b = built[m];
    HIP_TRY(upload(s->owned, b.nodes.data(), b.nodes.size(), &dm[m].nodes, bytes), "upload nodes");
    HIP_TRY(upload(s->owned, b.leaves.data(), b.leaves.size(), &dm[m].leaves, bytes), "upload leaves");
    // Normals from the OBJ's vn lines are f32 values (tobj parses f32): then an f32 table holds them
    // exactly in half the bytes (read once per mesh hit, mesh_rec); computed face normals are f64.
    std::vector<float> n32(b.normals.size());
    bool exact32 = true;
    for (size_t i = 0; i < b.normals.size() && exact32; ++i) {
      n32[i] = (float)b.normals[i];
      exact32 = (double)n32[i] == b.normals[i];
    }
    if (exact32) HIP_TRY(upload(s->owned, n32.data(), n32.size(), &dm[m].normals32, bytes), "upload normals");
    else HIP_TRY(upload(s->owned, b.normals.data(), b.normals.size(), &dm[m].normals, bytes), "upload normals");
    // YART_OPT_MESH_WALK_REF: walk every ray in the reference's order (A/B and tests); default:
    // front to back with the exact fallback (kernels.hip qbvh_coop)
    if (opt(YART_OPT_MESH_WALK_REF) == 0)
      HIP_TRY(upload(s->owned, b.aux.data(), b.aux.size(), &dm[m].aux, bytes), "upload leaf records");
    dm[m].root = b.ref_nodes - 1;
    dm[m].n_nodes = (uint32_t)b.nodes.size();
    dm[m].extent = b.extent;
    dm[m].wroot = b.walk_root;
    dm[m].n_recs = (uint32_t)(b.leaves.size() / kTriFloats);
    dm[m].n_leaves = (uint32_t)b.aux.size();
    {  // the cull box: union of the non-empty child boxes of the reference root and the walk root
      float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
      for (uint32_t r : {b.ref_nodes - 1, b.walk_root}) {
        const DevNode& nd = b.nodes[r];
        for (int k = 0; k < 4; ++k) {
          const float mn[3] = {nd.lo[k][0], nd.lo[k][2], nd.hi[k][0]}, mx[3] = {nd.lo[k][1], nd.lo[k][3], nd.hi[k][1]};
          if (!(std::isfinite(mn[0]) && std::isfinite(mn[1]) && std::isfinite(mn[2]))) continue;  // empty (+inf)
          for (int j = 0; j < 3; ++j) { lo[j] = std::min(lo[j], mn[j]); hi[j] = std::max(hi[j], mx[j]); }
        }
      }
      const float bl[4] = {lo[0], hi[0], lo[1], hi[1]}, bh[4] = {lo[2], hi[2], 0.0f, 0.0f};
      std::memcpy(dm[m].box_lo, bl, sizeof bl);
      std::memcpy(dm[m].box_hi, bh, sizeof bh);
    }
  }
  HIP_TRY(upload(s->owned, dm.data(), dm.size(), &ds.meshes, bytes), "upload meshes");
  if (use_world) {
    HIP_TRY(upload(s->owned, world.nodes4.data(), world.nodes4.size(), &ds.world_nodes, bytes), "upload world nodes");
    HIP_TRY(upload(s->owned, world.objs.data(), world.objs.size(), &ds.world_objs, bytes), "upload world objects");
    HIP_TRY(upload(s->owned, world.sph.data(), world.sph.size(), &ds.world_sph, bytes), "upload world spheres");
    ds.n_world_nodes = (uint32_t)world.nodes4.size();
    if (!world.plane_dirs.empty())
      HIP_TRY(upload(s->owned, world.plane_dirs.data(), world.plane_dirs.size(), &ds.plane_dirs, bytes),
              "upload in-plane directions");
    ds.n_plane_dirs = (uint32_t)world.plane_dirs.size();
  }
  ds.n_objects = d->n_objects; ds.n_lights = d->n_lights; ds.n_materials = d->n_materials;
  ds.n_textures = d->n_textures; ds.n_meshes = d->n_meshes;
  ds.has_mesh = 0;
  for (uint32_t i = 0; i < d->n_objects; ++i) ds.has_mesh |= d->objects[i].kind == YART_PRIM_MESH;
  ds.has_ext = 0;
  for (uint32_t i = 0; i < d->n_objects; ++i) ds.has_ext |= d->objects[i].n_xforms && d->objects[i].xforms[0].kind == YART_XF_MEDIUM;
  for (uint32_t i = 0; i < d->n_materials; ++i) ds.has_ext |= d->materials[i].kind == YART_MAT_ISOTROPIC;
  ds.has_time = 0;
  for (uint32_t i = 0; i < d->n_objects; ++i) ds.has_time |= d->objects[i].kind == YART_PRIM_MOVING_SPHERE;
  ds.has_ext |= ds.has_time;
  for (uint32_t i = 0; i < d->n_textures; ++i)
    ds.has_ext |= d->textures[i].kind == YART_TEX_NOISE || d->textures[i].kind == YART_TEX_IMAGE;

  // Mesh scenes: the megakernel (A/B r03: the wavefront path is 18 % slower on david and 47 % on the
  // bunny stand-in), meshes deeper than depth 10 included since r05: their walk stacks
  // keep 32 entries in LDS and overflow into HBM up to the reference's 64 (qbvh.rs:382-384; kernels.hip
  // OVF). YART_OPT_MESH_WAVEFRONT = 1 puts every mesh scene without EXT features (media, moving spheres,
  // noise / image textures) on the wavefront path (k_wf_shade / k_wf_trace); -1 (auto) and 0 keep the
  // megakernel. A deep mesh in an EXT scene is refused (no such megakernel variant).
  {
    const int64_t force = opt(YART_OPT_MESH_WAVEFRONT);
    ds.deep = d->n_meshes && 3 * depth + 1 > (uint32_t)kStackSlots;
    s->wavefront = ds.has_mesh && !ds.has_ext && force == 1;
    if (ds.deep && ds.has_ext)
      return fail(YART_ERR_UNSUPPORTED, "a mesh deeper than depth 10 in a scene with media, moving spheres or "
                                        "noise / image textures");
    // Parked walks (kernels.hip qbvh_coop PARK): the persistent megakernel of a scene with one mesh
    // object, no EXT features and a mesh of depth <= 10 (its walk stacks in the LDS)
    uint32_t mesh_objects = 0;
    for (uint32_t i = 0; i < d->n_objects; ++i) mesh_objects += d->objects[i].kind == YART_PRIM_MESH;
    bool small = true;
    for (uint32_t m = 0; m < d->n_meshes; ++m) small = small && built[m].aux.size() < (1u << 30);
    const int64_t park = opt(YART_OPT_MESH_PARK);
    ds.park = (mesh_objects == 1 && !ds.deep && !ds.has_ext && small && park > 0) ? (uint32_t)std::min<int64_t>(park, 16) : 0u;
    const int64_t pool = opt(YART_OPT_WF_POOL);
    if (pool >= 256) s->wf_pool = (uint32_t)(std::min<int64_t>(pool, 1ll << 24) / 256 * 256);
  }

  yart_scene_info& in = s->info;
  in.device = device; in.n_objects = d->n_objects; in.n_lights = d->n_lights; in.n_meshes = d->n_meshes;
  in.bvh_nodes = nodes; in.bvh_leaves = leaves; in.bvh_max_depth = depth;
  in.bvh_max_stack = d->n_meshes ? 3 * depth + 1 : 0;
  in.device_bytes = bytes;
  in.world_nodes = use_world ? (uint32_t)world.nodes4.size() : 0;
  in.world_depth = use_world ? world.depth4 : 0;
  in.bvh_tied_cuts = tied_cuts;
  in.bvh_tied_leaves = tied_leaves;
  in.bvh_build_ms = build_ms;
  in.walk_nodes = walk_nodes;
  in.walk_depth = walk_depth;
  in.upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - up0).count();
  *out = s.release();
  return ok();
}

int yart_scene_create(int device, const yart_scene_desc* d, yart_scene** out) {
  try {  // nothing unwinds across the C ABI (host allocations of the builders)
    return scene_create(device, d, out);
  } catch (const std::bad_alloc&) {
    return fail(YART_ERR_NO_MEMORY, "host allocation failed while building the scene");
  } catch (const std::exception& e) {
    return fail(YART_ERR_DEVICE, std::string("scene creation failed: ") + e.what());
  }
}

void yart_scene_destroy(yart_scene* s) { delete s; }

int yart_qbvh_build(const float* positions, const double* normals, uint32_t n, uint32_t flags, yart_qbvh_build_info* out) {
  if (!positions || !normals || !out) return fail(YART_ERR_INVALID, "null argument");
  BuiltMesh b;
  std::string err;
  QbvhOptions opt;
  opt.ties_desc = (flags & YART_QBVH_TIES_DESC) != 0;
  opt.threads = (flags & YART_QBVH_SERIAL) ? 1u : 0u;
  if (!build_qbvh(n, positions, normals, b, err, opt)) return fail(YART_ERR_UNSUPPORTED, err);
  uint32_t walk_max = 0;
  if (flags & YART_QBVH_WALK) {  // as scene creation builds it, then its structural check
    const uint32_t slots = 3 * b.depth + 1 > (uint32_t)kStackSlots ? (uint32_t)kMaxStackSlots : (uint32_t)kStackSlots;
    walk_max = (slots - 1) / 3;
    build_walk_tree(b, walk_max);
  }
  uint64_t h = 1469598103934665603ull;  // FNV-1a 64
  auto mix = [&h](const void* p, size_t len) {
    const unsigned char* c = (const unsigned char*)p;
    for (size_t i = 0; i < len; ++i) { h ^= c[i]; h *= 1099511628211ull; }
  };
  mix(b.nodes.data(), b.nodes.size() * sizeof(DevNode));
  mix(b.leaves.data(), b.leaves.size() * sizeof(float));
  mix(b.aux.data(), b.aux.size() * sizeof(LeafAux));
  mix(b.normals.data(), b.normals.size() * sizeof(double));
  std::memset(out, 0, sizeof *out);
  out->nodes = b.ref_nodes;
  out->leaves = (uint32_t)b.aux.size();
  out->depth = b.depth;
  out->tied_cuts = b.tied_cuts;
  out->tied_leaves = b.tied_leaves;
  out->digest = h;
  out->build_ms = b.build_ms;
  out->walk_nodes = b.walk_nodes;
  out->walk_depth = b.walk_depth;
  out->walk_valid = (flags & YART_QBVH_WALK) && check_walk_tree(b, walk_max) ? 1u : 0u;
  out->walk_build_ms = b.walk_build_ms;
  return ok();
}

int yart_world_bvh_build(const yart_scene_desc* d, yart_world_bvh_info* out) {
  if (!d || !out || (d->n_objects && !d->objects)) return fail(YART_ERR_INVALID, "null argument");
  std::memset(out, 0, sizeof *out);
  std::vector<DevObject> objs;
  for (uint32_t i = 0; i < d->n_objects; ++i) objs.push_back(to_dev(d->objects[i]));
  BuiltWorld w;
  if (objs.empty() || !build_world_bvh(objs, w)) return ok();  // built = 0: the list walk
  out->built = 1;
  out->nodes = (uint32_t)w.nodes.size();
  out->depth = w.depth;
  out->nodes4 = (uint32_t)w.nodes4.size();
  out->depth4 = w.depth4;
  uint64_t h = 1469598103934665603ull;  // FNV-1a 64
  auto mix = [&h](const void* p, size_t len) {
    const unsigned char* c = (const unsigned char*)p;
    for (size_t i = 0; i < len; ++i) { h ^= c[i]; h *= 1099511628211ull; }
  };
  mix(w.nodes4.data(), w.nodes4.size() * sizeof(DevWorldNode4));
  mix(w.objs.data(), w.objs.size() * sizeof(uint32_t));
  mix(w.sph.data(), w.sph.size() * sizeof(double));
  out->digest = h;
  std::string err;
  if (!check_world4(objs, w, err)) return fail(YART_ERR_UNSUPPORTED, "world BVH check: " + err);
  out->valid = 1;
  return ok();
}

int yart_scene_get_info(const yart_scene* s, yart_scene_info* out) {
  if (!s || !out) return fail(YART_ERR_INVALID, "null argument");
  *out = s->info;
  return ok();
}

int yart_debug_set_option(int option, int64_t value) {
  if (option < 0 || option >= YART_OPT_COUNT) return fail(YART_ERR_INVALID, "unknown option");
  g_opt[option].store(value, std::memory_order_relaxed);
  return ok();
}

int yart_debug_get_option(int option, int64_t* value) {
  if (!value) return fail(YART_ERR_INVALID, "null argument");
  if (option < 0 || option >= YART_OPT_COUNT) return fail(YART_ERR_INVALID, "unknown option");
  *value = opt(option);
  return ok();
}

}  // extern "C"

namespace yart_impl {

int make_args(const yart_scene* s, const yart_camera* cam, const yart_render_params* p, double* out, RenderArgs& a) {
  if (!s || !cam || !p) return fail(YART_ERR_INVALID, "null argument");
  if (p->width == 0 || p->height == 0) return fail(YART_ERR_INVALID, "width and height must be > 0");
  if ((uint64_t)p->width * p->height > 0xFFFFFFFFull) return fail(YART_ERR_INVALID, "image too large (pixel index is 32-bit)");
  const uint32_t sc = p->shard_count ? p->shard_count : 1;
  if (p->shard_index >= sc) return fail(YART_ERR_INVALID, "shard_index >= shard_count");
  a = RenderArgs{};
  a.cam = *cam;
  a.width = p->width; a.height = p->height; a.spp = p->spp; a.max_depth = p->max_depth; a.seed = p->seed;
  a.shard_index = p->shard_index; a.shard_count = sc;
  a.blocks_x = (p->width + 7) / 8;
  a.n_blocks = shard_blocks(a.blocks_x * ((p->height + 7) / 8), p->shard_index, sc);
  a.s_begin = 0; a.s_count = p->spp; a.chunk = p->spp ? p->spp : 1; a.n_chunks = 1;
  a.out = out;
  return YART_OK;
}

uint64_t shard_pixels(uint32_t w, uint32_t h, uint32_t shard_index, uint32_t shard_count) {
  // covered columns / rows per 8-pixel block column / row (main.rs:636-647)
  const uint32_t bx = (w + 7) / 8, by = (h + 7) / 8;
  auto per_block = [](uint32_t n, uint32_t nb) {
    std::vector<uint32_t> c(nb, 0);
    const uint32_t cw = n / 8;
    for (uint32_t col = 0; col < 8; ++col) {
      const uint32_t x0 = (uint32_t)(((uint64_t)n * col) / 8);
      for (uint32_t x = x0; x < x0 + cw && x < n; ++x) c[x / 8]++;
    }
    return c;
  };
  const std::vector<uint32_t> cx = per_block(w, bx), cy = per_block(h, by);
  const uint32_t sc = shard_count ? shard_count : 1;
  uint64_t n = 0;
  for (uint64_t b = shard_index; b < (uint64_t)bx * by; b += sc) n += (uint64_t)cx[b % bx] * cy[b / bx];
  return n;
}

}  // namespace yart_impl

namespace {

// Work decomposition. A unit is one wave rendering one 8x8 block for `chunk` consecutive samples.
// With chunk = spp (one unit per block) the kernel keeps the per-pixel sums in registers (fused).
// When the shard has too few blocks to fill the device several times over (strong scaling, small
// frames) the samples are split into chunks; each sample's value then goes to HBM and
// k_accumulate adds them per pixel in sample order, so the sums do not depend on the split.
struct Plan { uint32_t chunk, pass_spp; bool overlap = false; };  // overlap: passes in two scratch halves (launch_frame)

// Sample-scratch bytes a frame may use on a stream. Auto (option 0): an eighth of the device's
// memory, at most 16 GiB. C1-C4 and a C5 shard fit in one pass; C5 on one GPU (david
// 1920x1080x1024, 49.8 MB per sample, 51 GB) renders in 7 overlapped passes over two 8 GiB halves
// at -0.3 % against one 51 GB pass (r06, profiles/r06r_ab_scratch_overlap2.log; r05 had raised the
// cap to 64 GiB when passes still ran one after another: 12 passes at 4 GiB cost 13 %).
uint64_t scratch_budget(const yart_scene* s) {
  const int64_t v = opt(YART_OPT_SCRATCH_BYTES);
  if (v > 0) return (uint64_t)v;
  const uint64_t cap = 16ull << 30;
  return s->mem_total ? std::min<uint64_t>(cap, s->mem_total / 8) : (4ull << 30);
}
Plan plan(const yart_scene* s, const RenderArgs& a, uint32_t requested) {
  const uint32_t spp = a.spp;
  if (spp == 0 || a.n_blocks == 0) return {spp ? spp : 1, spp};
  const uint64_t per_sample = (uint64_t)a.n_blocks * 64 * 3 * sizeof(double);
  const uint64_t budget = scratch_budget(s);
  // A frame whose samples do not fit the budget renders in passes over two halves of it (overlapped,
  // launch_frame); the chunks are then cut for a pass, not the frame, so each pass holds as many
  // units per wave as a one-pass frame (the frame's chunks left 4 units per wave in a C5 pass).
  const bool split = (uint64_t)spp * per_sample > budget;
  const uint32_t span = split ? (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(spp, budget / 2 / per_sample)) : spp;
  uint32_t chunk;
  if (requested) {
    if (requested >= spp) return {spp, spp};  // explicit one-unit-per-block: the fused kernel
    chunk = requested;
  } else {
    // Persistent waves (4 per SIMD x 4 SIMDs per CU) pull units from a queue; many units per
    // wave keep the end-of-frame imbalance small, each unit's start costs a little. The list walk
    // (cornell: cheap samples) is best at ~64 units per wave (r02: 4,130 Msamples/s against 3,996
    // at 32 and 2,615 at 256; r05l: 64 within 0.5 % of 32-128); mesh and world-BVH frames, whose
    // samples cost 1.5-20x more and vary more, at ~192 (r05l at BASELINE spp: C4 +4.4 %, C5 shard
    // +1.1 %, C5 +0.8 %, C3 +0.4 % over 64), but not below 2 samples per unit (C3 1200x800x31:
    // -2.8 %, C4 800x800x32: -1.9 % at one sample; profiles/r05l_units_per_wave_sweep.log).
    const bool heavy = s->dev.has_mesh || s->dev.world_nodes;
    int64_t upw = opt(YART_OPT_UNITS_PER_WAVE);
    if (upw <= 0) upw = heavy ? 192 : 64;
    const uint64_t target = (uint64_t)upw * (uint64_t)s->cu_count * 16ull;
    uint64_t chunks = (target + a.n_blocks - 1) / a.n_blocks;
    const uint32_t min_chunk = heavy && span >= 2 ? 2 : 1;
    const uint64_t max_chunks = (span + min_chunk - 1) / min_chunk;  // 31 spp: 16 units of <= 2
    if (chunks > max_chunks) chunks = max_chunks;
    chunk = (uint32_t)((span + chunks - 1) / chunks);
  }
  uint64_t pass = split ? span : budget / per_sample;
  pass = pass / chunk * chunk;
  if (pass < chunk) pass = chunk;
  if (pass > spp) pass = spp;
  Plan pl{chunk, (uint32_t)pass};
  pl.overlap = chunk < spp && pass < spp;
  return pl;
}

StreamState* stream_state(yart_scene* s, hipStream_t stream) {
  std::lock_guard<std::mutex> lk(s->mu);
  auto& e = s->streams[stream];
  if (!e) e = std::make_unique<StreamState>();
  return e.get();
}

// The walk stacks' HBM overflow of a stream (deep meshes), grown on demand like the scratch.
int stream_ovf(StreamState* st, hipStream_t stream, size_t bytes, uint32_t** out) {
  if (st->ovf_bytes < bytes) {
    if (st->ovf) {
      HIP_TRY(hipStreamSynchronize(stream), "drain the stream before growing its stack overflow");
      for (hipStream_t x : {st->aux, st->acc})
        if (x) HIP_TRY(hipStreamSynchronize(x), "drain the stream before growing its stack overflow");
      HIP_TRY(hipFree(st->ovf), "hipFree stack overflow");
    }
    st->ovf = nullptr; st->ovf_bytes = 0;
    HIP_TRY(hipMalloc(&st->ovf, bytes), "hipMalloc stack overflow");
    st->ovf_bytes = bytes;
  }
  *out = st->ovf;
  return YART_OK;
}

// Scratch of a stream for one pass of pl.pass_spp samples (+ 256 B for the unit counter), grown on
// demand. Called with st->frame_mu held: no other frame of this library is being enqueued on the
// stream; earlier frames may still run on it, so the old buffer is released only after the stream
// drained. When the device cannot hold that much (the auto budget is sized from its total memory,
// not from what is free: other scenes, streams or the caller's own allocations may hold the rest),
// the pass shrinks by halves, down to one unit (`min_spp` samples), instead of failing the frame:
// more passes, the same frame (k_accumulate adds in sample order whatever the split). The larger
// buffer is allocated BEFORE the working one is released: on a nearly full device a frame then
// costs a failed hipMalloc or two and runs in the buffer it has, with no stream drain and no
// free/re-allocate churn per frame, and grows as soon as the memory is there.
// halves = 2: two such buffers back to back (the overlapped passes of launch_frame).
int pass_scratch(StreamState* st, hipStream_t stream, const RenderArgs& a, Plan& pl, uint32_t min_spp,
                 double** out, uint32_t halves = 1) {
  for (;;) {
    const size_t bytes = halves * ((size_t)a.n_blocks * pl.pass_spp * 64 * 3 * sizeof(double) + 256);
    if (st->bytes >= bytes) { *out = st->scratch; return YART_OK; }
    double* grown = nullptr;
    const hipError_t e = hipMalloc(&grown, bytes);
    if (e == hipSuccess) {
      if (st->scratch) {
        // earlier frames may still use the old one (their overlapped passes too)
        hipError_t d = hipStreamSynchronize(stream);
        for (hipStream_t x : {st->aux, st->acc})
          if (x && d == hipSuccess) d = hipStreamSynchronize(x);
        if (d != hipSuccess) { (void)hipFree(grown); return hip_fail(d, "drain the stream before growing its scratch"); }
        HIP_TRY(hipFree(st->scratch), "hipFree scratch");
      }
      st->scratch = grown; st->bytes = bytes;
      *out = st->scratch;
      return YART_OK;
    }
    if (e != hipErrorOutOfMemory || pl.pass_spp <= min_spp) return hip_fail(e, "hipMalloc scratch");
    (void)hipGetLastError();  // clear the allocation failure and try half the pass (or the old buffer)
    uint32_t half = pl.pass_spp / 2 / min_spp * min_spp;
    pl.pass_spp = half < min_spp ? min_spp : half;
  }
}

// n timing events for one frame (copied out: the caller owns them until push_frame hands them over).
int take_events(yart_scene* s, size_t n, std::vector<hipEvent_t>& f) {
  f.clear();
  std::lock_guard<std::mutex> lk(s->mu);
  while (f.size() < n) {
    if (!s->event_pool.empty()) {
      f.push_back(s->event_pool.back());
      s->event_pool.pop_back();
    } else {
      hipEvent_t e;
      hipError_t err = hipEventCreate(&e);
      if (err != hipSuccess) {
        for (hipEvent_t x : f) s->event_pool.push_back(x);
        f.clear();
        return hip_fail(err, "hipEventCreate");
      }
      f.push_back(e);
    }
  }
  return YART_OK;
}
void push_frame(yart_scene* s, hipStream_t stream, std::vector<hipEvent_t>&& f) {
  std::lock_guard<std::mutex> lk(s->mu);
  auto& frames = s->frames[stream];
  if (frames.size() >= 4096) {  // never read: recycle the oldest frame's events
    for (hipEvent_t e : frames.front()) s->event_pool.push_back(e);
    frames.erase(frames.begin());
  }
  frames.push_back(std::move(f));
}

// The wavefront buffers of a stream: the path slots (SoA, WfSlots), the shade workgroups' job
// ranges, the pass counters (alive flags ring + job counter) and the host-mapped status ring.
// Called with frame_mu held.
constexpr uint32_t kWfStatusRing = 64, kWfSentinel = 0xFFFFFFFFu;
size_t wf_slot_bytes(uint32_t pool) { return (size_t)pool * (6 * 8 + 2 * 8 + 3 * 8 + 4 * 4) + (size_t)pool / 256 * 8; }
int stream_wf(StreamState* st, hipStream_t stream, uint32_t pool, WfSlots& q, uint32_t** counters) {
  const size_t bytes = wf_slot_bytes(pool) + 256;
  if (st->wf_bytes < bytes || st->wf_pool != pool) {
    if (st->wf_mem) {
      HIP_TRY(hipStreamSynchronize(stream), "drain the stream before growing its path slots");
      HIP_TRY(hipFree(st->wf_mem), "hipFree path slots");
    }
    st->wf_mem = nullptr; st->wf_bytes = 0; st->wf_pool = 0;
    HIP_TRY(hipMalloc(&st->wf_mem, bytes), "hipMalloc path slots");
    st->wf_bytes = bytes; st->wf_pool = pool;
  }
  if (!st->wf_status_host) {
    void* h = nullptr;
    HIP_TRY(hipHostMalloc(&h, kWfStatusRing * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocCoherent),
            "hipHostMalloc status ring");
    void* d = nullptr;
    hipError_t e = hipHostGetDevicePointer(&d, h, 0);
    if (e != hipSuccess) { (void)hipHostFree(h); return hip_fail(e, "hipHostGetDevicePointer"); }
    st->wf_status_host = static_cast<uint32_t*>(h);
    st->wf_status_dev = static_cast<uint32_t*>(d);
  }
  char* p = static_cast<char*>(st->wf_mem);
  auto take = [&](size_t n) { char* r = p; p += n; return r; };
  q.o = reinterpret_cast<double*>(take(3 * 8 * (size_t)pool));
  q.d = reinterpret_cast<double*>(take(3 * 8 * (size_t)pool));
  q.T = reinterpret_cast<double*>(take(8 * (size_t)pool));
  q.wl = reinterpret_cast<double*>(take(8 * (size_t)pool));
  q.ht = reinterpret_cast<double*>(take(8 * (size_t)pool));
  q.hu = reinterpret_cast<double*>(take(8 * (size_t)pool));
  q.hv = reinterpret_cast<double*>(take(8 * (size_t)pool));
  q.job = reinterpret_cast<uint32_t*>(take(4 * (size_t)pool));
  q.depth = reinterpret_cast<uint32_t*>(take(4 * (size_t)pool));
  q.hobj = reinterpret_cast<uint32_t*>(take(4 * (size_t)pool));
  q.hsub = reinterpret_cast<uint32_t*>(take(4 * (size_t)pool));
  q.range = reinterpret_cast<uint32_t*>(take((size_t)pool / 256 * 8));
  *counters = reinterpret_cast<uint32_t*>(p);
  return YART_OK;
}

// One pass on the wavefront path: shade/trace iterations until the pass's jobs are done. The
// number of iterations is data-dependent, so the host keeps kWfLookahead iterations queued ahead
// of the device and stops when an iteration reports that no slot holds a ray any more (the few
// iterations already queued behind it find nothing to do). A device fault shows up as a stream
// error in the poll, never as a spin without end.
constexpr uint32_t kWfLookahead = 6;
int wf_pass(yart_scene* s, StreamState* st, const RenderArgs& b, hipStream_t stream) {
  const uint64_t total = (uint64_t)b.n_blocks * b.s_count * 64;
  if (total == 0) return YART_OK;
  if (total > 0xFFFFFE00ull) return fail(YART_ERR_INVALID, "wavefront pass over 2^32 jobs");
  uint32_t pool = s->wf_pool;
  if ((uint64_t)pool > (total + 255) / 256 * 256) pool = (uint32_t)((total + 255) / 256 * 256);
  WfSlots q;
  uint32_t* cnt = nullptr;
  if (int rc = stream_wf(st, stream, pool, q, &cnt)) return rc;
  HIP_TRY(hipMemsetAsync(q.job, 0xFF, 4 * (size_t)pool, stream), "empty the path slots");
  HIP_TRY(hipMemsetAsync(q.range, 0, (size_t)pool / 256 * 8, stream), "empty the job ranges");
  HIP_TRY(hipMemsetAsync(cnt, 0, 8 * sizeof(uint32_t), stream), "zero the pass counters");
  volatile uint32_t* hs = st->wf_status_host;
  WfArgs w;
  w.q = q;
  w.jobs = cnt + 4;
  w.total_jobs = (uint32_t)total;
  w.pool = pool;
  // Status slots are numbered by the stream's iteration count, which runs on across passes and
  // frames: when a pass ends at iteration j, its iterations j+1 .. j+kWfLookahead are still queued
  // and each writes its own slot, so the next pass (which starts at the following number) never
  // re-arms a slot one of them has yet to write (with the count restarting at 0 per
  // pass, a trailing write could overwrite the next pass's sentinel and end that pass early).
  // kWfStatusRing > 2 * kWfLookahead + 1 keeps the two passes' live slots apart.
  static_assert(kWfStatusRing > 2 * kWfLookahead + 1, "status ring too small for the look-ahead");
  const uint64_t base = st->wf_iter;
  for (uint32_t k = 0;; ++k) {
    if (k > (1u << 22)) return fail(YART_ERR_DEVICE, "wavefront pass did not finish");
    const uint32_t slot = (uint32_t)((base + k) % kWfStatusRing);
    __atomic_store_n(&hs[slot], kWfSentinel, __ATOMIC_RELAXED);
    w.alive = cnt + k % 4;
    w.alive_next = cnt + (k + 1) % 4;
    w.status = st->wf_status_dev + slot;
    HIP_TRY(launch_wf_shade(s->dev, b, w, stream), "launch k_wf_shade");
    HIP_TRY(launch_wf_trace(s->dev, b, w, stream), "launch k_wf_trace");
    st->wf_iter = base + k + 1;
    if (k < kWfLookahead) continue;
    const uint32_t jslot = (uint32_t)((base + k - kWfLookahead) % kWfStatusRing);
    uint32_t v;
    for (int spin = 0;; ++spin) {
      v = __atomic_load_n(&hs[jslot], __ATOMIC_ACQUIRE);
      if (v != kWfSentinel) break;
      const hipError_t e = hipStreamQuery(stream);
      if (e != hipErrorNotReady) {
        v = __atomic_load_n(&hs[jslot], __ATOMIC_ACQUIRE);
        if (v != kWfSentinel) break;
        return e != hipSuccess ? hip_fail(e, "wavefront iteration") : fail(YART_ERR_DEVICE, "wavefront iteration did not report");
      }
      if (spin > 8) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    if (v == 0) break;
  }
  return YART_OK;
}

}  // namespace

namespace yart_impl {

int launch_frame(yart_scene* s, RenderArgs a, uint32_t requested, bool stats, hipStream_t stream, Progress* prog) {
  // stats launches take the frame's own plan (r06; fused before, which measured another kernel)
  Plan pl = plan(s, a, requested);
  StreamState* st = stream_state(s, stream);
  std::lock_guard<std::mutex> frame_lock(st->frame_mu);
  std::vector<hipEvent_t> ev;
  if (prog) { a.progress = prog->device; a.progress_count = prog->counter; }
  if (s->wavefront && !stats) {  // mesh scenes: the wavefront path, pass by pass over the scratch budget
    double* scratch = nullptr;
    if (int rc = pass_scratch(st, stream, a, pl, 1, &scratch)) return rc;
    const uint32_t passes = (a.spp + pl.pass_spp - 1) / pl.pass_spp;
    if (int rc = take_events(s, 3 * (size_t)passes, ev)) return rc;
    uint32_t k = 0;
    for (uint32_t s0 = 0; s0 < a.spp; s0 += pl.pass_spp, ++k) {
      RenderArgs b = a;
      b.s_begin = s0;
      b.s_count = a.spp - s0 < pl.pass_spp ? a.spp - s0 : pl.pass_spp;
      b.chunk = b.s_count;
      b.n_chunks = 1;
      b.scratch = scratch;
      b.n_units = b.n_blocks;
      HIP_TRY(hipEventRecord(ev[3 * k], stream), "hipEventRecord");
      if (int rc = wf_pass(s, st, b, stream)) return rc;
      HIP_TRY(hipEventRecord(ev[3 * k + 1], stream), "hipEventRecord");
      HIP_TRY(launch_accumulate(b, s0 == 0, stream), "launch k_accumulate");
      HIP_TRY(hipEventRecord(ev[3 * k + 2], stream), "hipEventRecord");
    }
    if (prog) prog->total_units = 0;
    push_frame(s, stream, std::move(ev));
    return YART_OK;
  }
  // A frame larger than the scratch budget renders in passes, and the passes overlap (r06): the
  // budget is split in two halves, the odd passes render on the stream's `aux` stream into the second
  // half while the previous pass's last waves finish, and k_accumulate adds the passes in pass order
  // on `acc`; a half is rendered into again once the accumulate two passes back has read it. The sums
  // are the same (the accumulates run in order); the frame starts and ends in the caller's stream
  // order. (One pass after another, each pass's tail idled the device: C5 on 16 GiB, 4 passes,
  // -3 %; 8 GiB, 7 passes, -5.6 %; profiles/r06r_ab_scratch_budget.log.)
  bool overlap = pl.overlap;
  uint64_t ovf_words = 0;  // one launch's overflow region (a second one for the overlapped passes)
  if (s->dev.deep || s->dev.park) {  // the walk stacks' HBM overflow (deep meshes; PARK: the re-walk's
                                     // stacks): one region per wave of the largest launch below
    const uint64_t fused_waves = (uint64_t)a.n_blocks, dyn_waves = (uint64_t)s->cu_count * 16;
    const uint64_t units = (uint64_t)a.n_blocks * ((pl.pass_spp + pl.chunk - 1) / pl.chunk);
    const uint64_t waves = (pl.chunk >= a.spp ? fused_waves : std::min(dyn_waves, units)) + 4;
    ovf_words = waves * kOvfWords;
    if (int rc = stream_ovf(st, stream, (overlap ? 2 : 1) * ovf_words * sizeof(uint32_t), &a.stack_ovf)) return rc;
  }
  if (pl.chunk >= a.spp) {  // fused: one unit per block, sums in registers
    if (prog) prog->total_units = a.n_blocks;
    if (int rc = take_events(s, 2, ev)) return rc;
    HIP_TRY(hipEventRecord(ev[0], stream), "hipEventRecord");
    HIP_TRY(launch_render(s->dev, a, stats, stream), "launch k_render");
    HIP_TRY(hipEventRecord(ev[1], stream), "hipEventRecord");
    push_frame(s, stream, std::move(ev));
    return YART_OK;
  }
  double* scratch = nullptr;
  if (int rc = pass_scratch(st, stream, a, pl, pl.chunk, &scratch, overlap ? 2u : 1u)) return rc;
  overlap = overlap && pl.pass_spp < a.spp;
  if (overlap && !st->acc) {  // the stream's first overlapped frame: its two helper streams and events
    DeviceGuard g(s->device);
    hipStream_t x[2] = {nullptr, nullptr};
    hipEvent_t e[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    hipError_t err = hipSuccess;
    for (int i = 0; i < 2 && err == hipSuccess; ++i) err = hipStreamCreateWithFlags(&x[i], hipStreamNonBlocking);
    for (int i = 0; i < 5 && err == hipSuccess; ++i) err = hipEventCreateWithFlags(&e[i], hipEventDisableTiming);
    if (err != hipSuccess) {
      for (hipStream_t y : x) if (y) (void)hipStreamDestroy(y);
      for (hipEvent_t y : e) if (y) (void)hipEventDestroy(y);
      return hip_fail(err, "create the overlapped passes' streams");
    }
    st->aux = x[0]; st->acc = x[1];
    st->ev_start = e[0]; st->ev_render[0] = e[1]; st->ev_render[1] = e[2]; st->ev_acc[0] = e[3]; st->ev_acc[1] = e[4];
  }
  const size_t half_doubles = (size_t)a.n_blocks * pl.pass_spp * 64 * 3;
  const size_t half_bytes = half_doubles * sizeof(double) + 256;
  const uint32_t passes = (a.spp + pl.pass_spp - 1) / pl.pass_spp;
  if (int rc = take_events(s, 3 * (size_t)passes, ev)) return rc;
  if (overlap) {  // the helper streams start after the caller's earlier work
    HIP_TRY(hipEventRecord(st->ev_start, stream), "hipEventRecord");
    HIP_TRY(hipStreamWaitEvent(st->aux, st->ev_start, 0), "hipStreamWaitEvent");
    HIP_TRY(hipStreamWaitEvent(st->acc, st->ev_start, 0), "hipStreamWaitEvent");
  }
  uint32_t k = 0, base = 0;
  for (uint32_t s0 = 0; s0 < a.spp; s0 += pl.pass_spp, ++k) {
    const uint32_t h = overlap ? (k & 1u) : 0u;      // the scratch half (and overflow region) of the pass
    const hipStream_t rs = h ? st->aux : stream;      // where it renders
    const hipStream_t as = overlap ? st->acc : stream;  // where it is added
    double* buf = reinterpret_cast<double*>(reinterpret_cast<char*>(scratch) + h * half_bytes);
    uint32_t* queue = reinterpret_cast<uint32_t*>(buf + half_doubles);
    RenderArgs b = a;
    b.s_begin = s0;
    b.s_count = a.spp - s0 < pl.pass_spp ? a.spp - s0 : pl.pass_spp;
    b.chunk = pl.chunk;
    b.n_chunks = (b.s_count + pl.chunk - 1) / pl.chunk;
    b.scratch = buf;
    b.queue = queue;
    b.n_units = b.n_blocks * b.n_chunks;
    b.waves = (uint32_t)s->cu_count * 16;  // 4 waves per SIMD resident
    if (a.stack_ovf) b.stack_ovf = a.stack_ovf + h * ovf_words;
    b.progress_base = base;
    base += b.n_units;
    if (overlap && k >= 2) HIP_TRY(hipStreamWaitEvent(rs, st->ev_acc[h], 0), "hipStreamWaitEvent");
    // the unit counter, and the 8 XCD-local ones of mesh frames (kernels.hip, claim of a unit)
    HIP_TRY(hipMemsetAsync(queue, 0, 9 * sizeof(uint32_t), rs), "zero the unit counters");
    HIP_TRY(hipEventRecord(ev[3 * k], rs), "hipEventRecord");
    HIP_TRY(launch_render(s->dev, b, stats, rs), "launch k_render");
    HIP_TRY(hipEventRecord(ev[3 * k + 1], rs), "hipEventRecord");
    if (overlap) {
      HIP_TRY(hipEventRecord(st->ev_render[h], rs), "hipEventRecord");
      HIP_TRY(hipStreamWaitEvent(as, st->ev_render[h], 0), "hipStreamWaitEvent");
    }
    HIP_TRY(launch_accumulate(b, s0 == 0, as), "launch k_accumulate");
    HIP_TRY(hipEventRecord(ev[3 * k + 2], as), "hipEventRecord");
    if (overlap) HIP_TRY(hipEventRecord(st->ev_acc[h], as), "hipEventRecord");
  }
  if (overlap) HIP_TRY(hipStreamWaitEvent(stream, st->ev_acc[(passes - 1) & 1u], 0), "hipStreamWaitEvent");
  if (prog) prog->total_units = base;
  push_frame(s, stream, std::move(ev));
  return YART_OK;
}

int acquire_stream(yart_scene* s, hipStream_t* out) {
  {
    std::lock_guard<std::mutex> lk(s->mu);
    if (!s->idle_streams.empty()) {
      *out = s->idle_streams.back();
      s->idle_streams.pop_back();
      return YART_OK;
    }
  }
  DeviceGuard g(s->device);
  hipStream_t st;
  HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
  std::lock_guard<std::mutex> lk(s->mu);
  s->owned_streams.push_back(st);
  *out = st;
  return YART_OK;
}
void release_stream(yart_scene* s, hipStream_t st) {
  std::lock_guard<std::mutex> lk(s->mu);
  s->idle_streams.push_back(st);
}

int alloc_progress(Progress& p) {
  void* h = nullptr;
  HIP_TRY(hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc progress word");
  p.host = static_cast<uint32_t*>(h);
  __atomic_store_n(p.host, 0u, __ATOMIC_RELAXED);
  void* d = nullptr;
  hipError_t e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess) { (void)hipHostFree(h); p.host = nullptr; return hip_fail(e, "hipHostGetDevicePointer"); }
  p.device = static_cast<uint32_t*>(d);
  void* c = nullptr;
  e = hipMalloc(&c, 4);
  if (e == hipSuccess) e = hipMemset(c, 0, 4);
  if (e != hipSuccess) {
    if (c) (void)hipFree(c);
    (void)hipHostFree(h);
    p.host = p.device = nullptr;
    return hip_fail(e, "hipMalloc progress counter");
  }
  p.counter = static_cast<uint32_t*>(c);
  return YART_OK;
}
void free_progress(Progress& p) {
  if (p.host) (void)hipHostFree(p.host);
  if (p.counter) (void)hipFree(p.counter);
  p.host = p.device = p.counter = nullptr;
}

int wait_with_progress(const std::vector<hipEvent_t>& done, const std::vector<int>& devices,
                       const std::vector<Progress*>& prog, uint64_t total_pixels, yart_progress_fn fn, void* user) {
  uint64_t reported = 0;
  for (size_t i = 0; i < done.size(); ++i) {
    DeviceGuard g(devices[i]);
    for (;;) {
      const hipError_t q = hipEventQuery(done[i]);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) return hip_fail(q, "render");
      if (fn) {
        // pixels of the frame whose units have been handed out, over all devices
        uint64_t units = 0, total = 0, px = 0;
        for (Progress* p : prog) {
          const uint32_t u = __atomic_load_n(p->host, __ATOMIC_RELAXED);
          units = u < p->total_units ? u : p->total_units;
          total = p->total_units ? p->total_units : 1;
          px += p->pixels * units / total;
        }
        if (px > reported && px < total_pixels) {
          reported = px;
          fn(px, user);
        }
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(fn ? 10 : 1));
    }
  }
  if (fn && reported < total_pixels) fn(total_pixels, user);
  return YART_OK;
}

}  // namespace yart_impl

extern "C" {

int yart_frame_timing(yart_scene* s, void* stream, double* render_ms, double* accumulate_ms, uint32_t* frames) {
  if (!s || !render_ms || !accumulate_ms || !frames) return fail(YART_ERR_INVALID, "null argument");
  DeviceGuard g(s->device);
  std::vector<std::vector<hipEvent_t>> mine;
  {
    std::lock_guard<std::mutex> lk(s->mu);
    auto it = s->frames.find((hipStream_t)stream);
    if (it != s->frames.end()) mine.swap(it->second);
  }
  double r = 0.0, acc = 0.0;
  uint32_t n_frames = 0;
  int rc = YART_OK;
  for (const auto& v : mine) {
    float ms = 0.0f;
    hipError_t e = hipSuccess;
    if (v.size() == 2) {
      if ((e = hipEventElapsedTime(&ms, v[0], v[1])) == hipSuccess) r += ms;
    } else {
      for (size_t k = 0; k + 2 < v.size() && e == hipSuccess; k += 3) {
        if ((e = hipEventElapsedTime(&ms, v[k], v[k + 1])) != hipSuccess) break;
        r += ms;
        if ((e = hipEventElapsedTime(&ms, v[k + 1], v[k + 2])) != hipSuccess) break;
        acc += ms;
      }
    }
    if (e != hipSuccess && rc == YART_OK) rc = hip_fail(e, "hipEventElapsedTime");
    ++n_frames;
  }
  {
    std::lock_guard<std::mutex> lk(s->mu);
    for (auto& v : mine)
      for (hipEvent_t e : v) s->event_pool.push_back(e);
  }
  if (rc != YART_OK) return rc;
  *render_ms = r;
  *accumulate_ms = acc;
  *frames = n_frames;
  return ok();
}

int yart_render_async(yart_scene* s, const yart_camera* cam, const yart_render_params* p, double* d_xyz_sum,
                      void* stream) {
  RenderArgs a;
  if (int rc = make_args(s, cam, p, d_xyz_sum, a)) return rc;
  if (!d_xyz_sum) return fail(YART_ERR_INVALID, "null output");
  DeviceGuard g(s->device);
  if (int rc = launch_frame(s, a, p->samples_per_unit, false, (hipStream_t)stream, nullptr)) return rc;
  return ok();
}

int yart_render_packed_async(yart_scene* s, const yart_camera* cam, const yart_render_params* p, double* d_packed,
                             void* stream) {
  RenderArgs a;
  if (int rc = make_args(s, cam, p, d_packed, a)) return rc;
  if (!d_packed) return fail(YART_ERR_INVALID, "null output");
  a.packed = 1;
  DeviceGuard g(s->device);
  if (int rc = launch_frame(s, a, p->samples_per_unit, false, (hipStream_t)stream, nullptr)) return rc;
  return ok();
}

uint64_t yart_shard_packed_len(uint32_t width, uint32_t height, uint32_t shard_index, uint32_t shard_count) {
  const uint32_t sc = shard_count ? shard_count : 1;
  return (uint64_t)shard_blocks(((width + 7) / 8) * ((height + 7) / 8), shard_index, sc) * 64 * 3;
}

}  // extern "C"

namespace {

// yart_render / yart_render_with_stats: a library-owned stream per call (so concurrent calls on
// one handle, from several host threads, never share a stream, a scratch buffer or a unit
// counter), device output on it, one copy back, progress polled on the calling thread.
int render_host(yart_scene* s, const yart_camera* cam, const yart_render_params* p, double* host_out,
                yart_render_stats* stats, yart_progress_fn progress, void* user) {
  RenderArgs a;
  if (int rc = make_args(s, cam, p, nullptr, a)) return rc;
  if (!host_out) return fail(YART_ERR_INVALID, "null output");
  DeviceGuard g(s->device);
  hipStream_t stream;
  if (int rc = acquire_stream(s, &stream)) return rc;
  struct Release {
    yart_scene* s; hipStream_t st;
    ~Release() { (void)hipStreamSynchronize(st); release_stream(s, st); }
  } release{s, stream};
  const size_t bytes = sizeof(double) * 3 * (size_t)p->width * p->height;
  double* d_out = nullptr;
  unsigned long long* d_stats = nullptr;
  HIP_TRY(hipMalloc(&d_out, bytes), "hipMalloc output");
  std::unique_ptr<double, decltype(&hipFree)> hold(d_out, &hipFree);
  HIP_TRY(hipMemsetAsync(d_out, 0, bytes, stream), "hipMemset");
  if (stats) {
    HIP_TRY(hipMalloc(&d_stats, 25 * sizeof(unsigned long long)), "hipMalloc stats");
    HIP_TRY(hipMemsetAsync(d_stats, 0, 25 * sizeof(unsigned long long), stream), "hipMemset");
  }
  std::unique_ptr<unsigned long long, decltype(&hipFree)> hold2(d_stats, &hipFree);
  a.out = d_out;
  a.stats = d_stats;
  Progress pr;
  if (progress) {
    if (int rc = alloc_progress(pr)) return rc;
    pr.pixels = shard_pixels(p->width, p->height, a.shard_index, a.shard_count);
  }
  struct FreeProgress { Progress& p; ~FreeProgress() { free_progress(p); } } free_pr{pr};
  if (int rc = launch_frame(s, a, p->samples_per_unit, stats != nullptr, stream, progress ? &pr : nullptr)) return rc;
  hipEvent_t done;
  HIP_TRY(hipEventCreateWithFlags(&done, hipEventDisableTiming), "hipEventCreate");
  std::unique_ptr<std::remove_pointer<hipEvent_t>::type, decltype(&hipEventDestroy)> hold3(done, &hipEventDestroy);
  HIP_TRY(hipEventRecord(done, stream), "hipEventRecord");
  if (int rc = wait_with_progress({done}, {s->device}, {&pr}, pr.pixels, progress, user)) return rc;
  HIP_TRY(hipMemcpyAsync(host_out, d_out, bytes, hipMemcpyDeviceToHost, stream), "copy output");
  if (stats) {
    unsigned long long v[25];
    HIP_TRY(hipMemcpyAsync(v, d_stats, sizeof v, hipMemcpyDeviceToHost, stream), "copy stats");
    HIP_TRY(hipStreamSynchronize(stream), "copy stats");
    std::memset(stats, 0, sizeof *stats);
    stats->samples = v[0]; stats->segments = v[1]; stats->prim_tests = v[2]; stats->node_visits = v[3];
    stats->leaf_visits = v[4]; stats->leaf_tris = v[5]; stats->light_tests = v[6];
    stats->mesh_rewalks = v[7];
    stats->coop_rounds = v[8]; stats->coop_leaf_rounds = v[9]; stats->coop_walks = v[10];
    stats->coop_idle_slots = v[11];
    stats->world_iters = v[12]; stats->world_leaf_iters = v[13];
    stats->ovf_pushes = v[14];
    stats->coop_node_rounds = v[15]; stats->coop_node_lanes = v[16]; stats->coop_leaf_lanes = v[17];
    stats->coop_leaf_quad_lanes = v[18]; stats->iterations = v[19]; stats->camera_lanes = v[20];
    stats->scatter_lanes = v[21]; stats->camera_iters = v[22]; stats->scatter_iters = v[23];
    stats->parked_walks = v[24];
  }
  HIP_TRY(hipStreamSynchronize(stream), "copy output");
  return ok();
}

}  // namespace

extern "C" {

int yart_render(yart_scene* s, const yart_camera* cam, const yart_render_params* p, double* xyz_sum_out,
                yart_progress_fn progress, void* user) {
  return render_host(s, cam, p, xyz_sum_out, nullptr, progress, user);
}

int yart_render_with_stats(yart_scene* s, const yart_camera* cam, const yart_render_params* p, double* xyz_sum_out,
                           yart_render_stats* stats) {
  if (!stats) return fail(YART_ERR_INVALID, "null stats");
  return render_host(s, cam, p, xyz_sum_out, stats, nullptr, nullptr);
}

int yart_finalize_rgba8_async(int device, const double* d_xyz, uint32_t w, uint32_t h, uint32_t spp, uint8_t* d_rgba,
                              void* stream) {
  if (!d_xyz || !d_rgba || !w || !h) return fail(YART_ERR_INVALID, "bad argument");
  DeviceGuard g(device);
  HIP_TRY(launch_finalize(d_xyz, w, h, spp, d_rgba, (hipStream_t)stream), "launch k_finalize");
  return ok();
}

int yart_finalize_rgba8(int device, const double* xyz, uint32_t w, uint32_t h, uint32_t spp, uint8_t* rgba) {
  if (!xyz || !rgba || !w || !h) return fail(YART_ERR_INVALID, "bad argument");
  DeviceGuard g(device);
  const size_t n = (size_t)w * h;
  double* dx = nullptr;
  uint8_t* dr = nullptr;
  HIP_TRY(hipMalloc(&dx, sizeof(double) * 3 * n), "hipMalloc");
  std::unique_ptr<double, decltype(&hipFree)> h1(dx, &hipFree);
  HIP_TRY(hipMalloc(&dr, 4 * n), "hipMalloc");
  std::unique_ptr<uint8_t, decltype(&hipFree)> h2(dr, &hipFree);
  HIP_TRY(hipMemcpy(dx, xyz, sizeof(double) * 3 * n, hipMemcpyHostToDevice), "copy in");
  HIP_TRY(launch_finalize(dx, w, h, spp, dr, nullptr), "launch k_finalize");
  HIP_TRY(hipStreamSynchronize(nullptr), "k_finalize");
  HIP_TRY(hipMemcpy(rgba, dr, 4 * n, hipMemcpyDeviceToHost), "copy out");
  return ok();
}

int yart_intersect(yart_scene* s, const double* rays, uint32_t n, double* hits, int32_t* obj) {
  if (!s || (n && (!rays || !hits || !obj))) return fail(YART_ERR_INVALID, "null argument");
  if (n == 0) return ok();
  DeviceGuard g(s->device);
  hipStream_t st;
  if (int rc = acquire_stream(s, &st)) return rc;
  struct Release {
    yart_scene* s; hipStream_t st;
    ~Release() { (void)hipStreamSynchronize(st); release_stream(s, st); }
  } release{s, st};
  double *dr = nullptr, *dh = nullptr;
  int32_t* dobj = nullptr;
  HIP_TRY(hipMalloc(&dr, sizeof(double) * 8 * (size_t)n), "hipMalloc");
  std::unique_ptr<double, decltype(&hipFree)> h1(dr, &hipFree);
  HIP_TRY(hipMalloc(&dh, sizeof(double) * 8 * (size_t)n), "hipMalloc");
  std::unique_ptr<double, decltype(&hipFree)> h2(dh, &hipFree);
  HIP_TRY(hipMalloc(&dobj, sizeof(int32_t) * (size_t)n), "hipMalloc");
  std::unique_ptr<int32_t, decltype(&hipFree)> h3(dobj, &hipFree);
  HIP_TRY(hipMemcpyAsync(dr, rays, sizeof(double) * 8 * (size_t)n, hipMemcpyHostToDevice, st), "copy rays");
  HIP_TRY(launch_intersect(s->dev, dr, n, dh, dobj, st), "launch k_intersect");
  HIP_TRY(hipMemcpyAsync(hits, dh, sizeof(double) * 8 * (size_t)n, hipMemcpyDeviceToHost, st), "copy hits");
  HIP_TRY(hipMemcpyAsync(obj, dobj, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, st), "copy obj");
  HIP_TRY(hipStreamSynchronize(st), "k_intersect");
  return ok();
}

int yart_probe_rng(int device, uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, double* out) {
  if (!out || n == 0) return fail(YART_ERR_INVALID, "bad argument");
  DeviceGuard g(device);
  double* d = nullptr;
  HIP_TRY(hipMalloc(&d, sizeof(double) * n), "hipMalloc");
  std::unique_ptr<double, decltype(&hipFree)> h(d, &hipFree);
  HIP_TRY(launch_probe_rng(seed, pixel, sample, n, d, nullptr), "launch k_probe_rng");
  HIP_TRY(hipStreamSynchronize(nullptr), "k_probe_rng");
  HIP_TRY(hipMemcpy(out, d, sizeof(double) * n, hipMemcpyDeviceToHost), "copy");
  return ok();
}

int yart_probe_math(int device, int op, const double* a, const double* b, uint32_t n, double* out) {
  if (!a || !out || n == 0 || ((op == 1 || op == 4) && !b)) return fail(YART_ERR_INVALID, "bad argument");
  DeviceGuard g(device);
  double *da = nullptr, *db = nullptr, *dout = nullptr;
  HIP_TRY(hipMalloc(&da, sizeof(double) * n), "hipMalloc");
  std::unique_ptr<double, decltype(&hipFree)> h1(da, &hipFree);
  HIP_TRY(hipMalloc(&db, sizeof(double) * n), "hipMalloc");
  std::unique_ptr<double, decltype(&hipFree)> h2(db, &hipFree);
  HIP_TRY(hipMalloc(&dout, sizeof(double) * n), "hipMalloc");
  std::unique_ptr<double, decltype(&hipFree)> h3(dout, &hipFree);
  HIP_TRY(hipMemcpy(da, a, sizeof(double) * n, hipMemcpyHostToDevice), "copy a");
  HIP_TRY(hipMemcpy(db, b ? b : a, sizeof(double) * n, hipMemcpyHostToDevice), "copy b");
  HIP_TRY(launch_probe_math(op, da, db, n, dout, nullptr), "launch k_probe_math");
  HIP_TRY(hipStreamSynchronize(nullptr), "k_probe_math");
  HIP_TRY(hipMemcpy(out, dout, sizeof(double) * n, hipMemcpyDeviceToHost), "copy out");
  return ok();
}

}  // extern "C"
