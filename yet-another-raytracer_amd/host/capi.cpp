// capi.cpp — C ABI of libyart_host.so (include/yart_host.h).
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../../include/yart_host.h"
#include "camera_impl.h"
#include "scene.hpp"

namespace {
thread_local std::string g_err;
int fail(int code, const std::string& msg) { g_err = msg; return code; }
int ok() { g_err.clear(); return YART_OK; }
void copy_str(char* dst, size_t cap, const std::string& s) {
  std::snprintf(dst, cap, "%s", s.c_str());
}
}  // namespace

struct yart_preset {
  yart::ScenePreset preset;
  std::unique_ptr<yart::SceneDesc> owned;
  yart_scene_desc desc;
};

extern "C" {

const char* yart_host_last_error(void) { return g_err.c_str(); }

int yart_preset_create(const char* scene, const char* asset_dir, uint64_t scene_seed, yart_preset** out) {
  if (!scene || !out) return fail(YART_ERR_INVALID, "null argument");
  try {
    auto p = std::make_unique<yart_preset>();
    p->preset = yart::build_scene_preset(scene, asset_dir ? asset_dir : "assets", scene_seed);
    p->owned = yart::flatten_scene(*p->preset.world, p->preset.lights, p->preset.background);
    p->desc = p->owned->desc();
    *out = p.release();
    return ok();
  } catch (const std::invalid_argument& e) {
    std::string m = e.what();
    return fail(m.find("outside this build") != std::string::npos ? YART_ERR_UNSUPPORTED : YART_ERR_INVALID, m);
  } catch (const std::exception& e) {
    return fail(YART_ERR_IO, e.what());
  }
}
void yart_preset_destroy(yart_preset* p) { delete p; }
const yart_scene_desc* yart_preset_desc(const yart_preset* p) { return p ? &p->desc : nullptr; }
const char* yart_preset_stand_in(const yart_preset* p) { return p ? p->preset.stand_in.c_str() : ""; }

int yart_preset_defaults(const yart_preset* p, yart_render_defaults* o) {
  if (!p || !o) return fail(YART_ERR_INVALID, "null argument");
  const auto& d = p->preset.defaults;
  o->width = d.width; o->height = d.height;
  o->samples_per_pixel = d.samples_per_pixel; o->max_depth = d.max_depth; o->workers = d.workers;
  o->vfov = d.vfov; o->aperture = d.aperture;
  for (int i = 0; i < 3; ++i) {
    o->lookfrom[i] = p->preset.lookfrom.e[i];
    o->lookat[i] = p->preset.lookat.e[i];
    o->background[i] = p->preset.background.e[i];
  }
  copy_str(o->output_filename, sizeof o->output_filename, p->preset.output_filename);
  return ok();
}

int yart_scene_names(const char** names, int capacity) {
  const auto& n = yart::scene_names();
  for (int i = 0; i < (int)n.size() && i < capacity; ++i) names[i] = n[i].c_str();
  return (int)n.size();
}

void yart_resolve_dimensions(uint32_t dw, uint32_t dh, uint32_t wo, uint32_t ho, uint32_t* w, uint32_t* h) {
  double aspect = (double)dw / (double)dh;  // main.rs:172
  if (wo && ho) { *w = wo; *h = ho; }
  else if (wo) { *w = wo; *h = (uint32_t)std::fmax(std::round((double)wo / aspect), 1.0); }
  else if (ho) { *h = ho; *w = (uint32_t)std::fmax(std::round((double)ho * aspect), 1.0); }
  else { *w = dw; *h = dh; }
}

// clap derive Cli (main.rs:78-107) + parse_positive_usize (main.rs:151-160).
int yart_cli_parse(int argc, const char* const* argv, yart_cli* c) {
  if (!c) return fail(YART_ERR_INVALID, "null argument");
  std::memset(c, 0, sizeof *c);
  c->vfov = NAN; c->aperture = NAN;
  bool have_scene = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i], val;
    size_t eq = a.find('=');
    std::string key = a;
    bool inline_val = false;
    if (a.rfind("--", 0) == 0 && eq != std::string::npos) { key = a.substr(0, eq); val = a.substr(eq + 1); inline_val = true; }
    auto need = [&](const char* shown) -> int {
      if (inline_val) return 0;
      if (i + 1 >= argc) return fail(YART_ERR_INVALID, std::string("a value is required for '") + shown + "' but none was supplied");
      val = argv[++i];
      return 0;
    };
    auto pos_u32 = [&](const char* shown, uint32_t* dst) -> int {
      if (need(shown)) return YART_ERR_INVALID;
      char* e; errno = 0;
      long long v = std::strtoll(val.c_str(), &e, 10);
      if (*e || e == val.c_str() || errno) return fail(YART_ERR_INVALID, "invalid value '" + val + "' for '" + shown + "': invalid digit found in string");
      if (v < 1 || v > 4294967295LL) return fail(YART_ERR_INVALID, "invalid value '" + val + "' for '" + shown + "': " + val + " is not in 1..=4294967295");
      *dst = (uint32_t)v;
      return 0;
    };
    auto pos_usize = [&](const char* shown, uint64_t* dst) -> int {
      if (need(shown)) return YART_ERR_INVALID;
      char* e; errno = 0;
      if (!val.empty() && val[0] == '-') return fail(YART_ERR_INVALID, "invalid value '" + val + "' for '" + shown + "': invalid integer `" + val + "`: invalid digit found in string");
      unsigned long long v = std::strtoull(val.c_str(), &e, 10);
      if (*e || e == val.c_str() || errno) return fail(YART_ERR_INVALID, "invalid value '" + val + "' for '" + shown + "': invalid integer `" + val + "`: invalid digit found in string");
      if (v == 0) return fail(YART_ERR_INVALID, "invalid value '" + val + "' for '" + shown + "': value must be greater than 0");
      *dst = v;
      return 0;
    };
    auto f64 = [&](const char* shown, double* dst) -> int {
      if (need(shown)) return YART_ERR_INVALID;
      char* e;
      double v = std::strtod(val.c_str(), &e);
      if (*e || e == val.c_str()) return fail(YART_ERR_INVALID, "invalid value '" + val + "' for '" + shown + "': invalid float literal");
      *dst = v;
      return 0;
    };
    int rc = 0;
    if (key == "--scene") {
      if (need("--scene <SCENE>")) return YART_ERR_INVALID;
      bool known = false;
      for (const auto& n : yart::scene_names()) known |= (n == val);
      if (!known) return fail(YART_ERR_INVALID, "invalid value '" + val + "' for '--scene <SCENE>'");
      copy_str(c->scene, sizeof c->scene, val);
      have_scene = true;
    } else if (key == "--output") {
      if (need("--output <OUTPUT>")) return YART_ERR_INVALID;
      copy_str(c->output, sizeof c->output, val);
    } else if (key == "--width") rc = pos_u32("--width <WIDTH>", &c->width);
    else if (key == "--height") rc = pos_u32("--height <HEIGHT>", &c->height);
    else if (key == "--samples") rc = pos_usize("--samples <SAMPLES>", &c->samples);
    else if (key == "--max-depth") rc = pos_usize("--max-depth <MAX_DEPTH>", &c->max_depth);
    else if (key == "--workers") rc = pos_usize("--workers <WORKERS>", &c->workers);
    else if (key == "--vfov") rc = f64("--vfov <VFOV>", &c->vfov);
    else if (key == "--aperture") rc = f64("--aperture <APERTURE>", &c->aperture);
    else if (key == "--seed") { uint64_t s = 0; if (need("--seed <SEED>")) return YART_ERR_INVALID; s = std::strtoull(val.c_str(), nullptr, 0); c->seed = s; }
    else if (key == "--gpus") { uint64_t g = 0; rc = pos_usize("--gpus <GPUS>", &g); c->gpus = (int32_t)g; }
    else if (key == "--assets") { if (need("--assets <DIR>")) return YART_ERR_INVALID; copy_str(c->assets, sizeof c->assets, val); }
    else return fail(YART_ERR_INVALID, "unexpected argument '" + a + "' found");
    if (rc) return rc;
  }
  if (!have_scene) return fail(YART_ERR_INVALID, "the following required arguments were not provided:\n  --scene <SCENE>");
  return ok();
}

int yart_resolve_render_options(const char* default_filename, const yart_render_defaults* d, const yart_cli* cli,
                                yart_render_options* o) {
  if (!default_filename || !d || !cli || !o) return fail(YART_ERR_INVALID, "null argument");
  yart_resolve_dimensions(d->width, d->height, cli->width, cli->height, &o->width, &o->height);
  if (cli->output[0]) copy_str(o->output_path, sizeof o->output_path, cli->output);
  else copy_str(o->output_path, sizeof o->output_path, std::string("output/") + default_filename);  // main.rs:162-164
  o->samples_per_pixel = cli->samples ? cli->samples : d->samples_per_pixel;
  o->max_depth = cli->max_depth ? cli->max_depth : d->max_depth;
  o->workers = cli->workers ? cli->workers : d->workers;
  o->vfov = std::isnan(cli->vfov) ? d->vfov : cli->vfov;
  o->aperture = std::isnan(cli->aperture) ? d->aperture : cli->aperture;
  return ok();
}

int yart_obj_triangle_count(const char* path, uint32_t* n) {
  try {
    *n = yart::load_obj_mesh(path)->n_triangles();
    return ok();
  } catch (const std::exception& e) {
    return fail(YART_ERR_IO, e.what());
  }
}
int yart_obj_load(const char* path, float* positions, double* normals, double* uvs, uint32_t cap) {
  try {
    auto m = yart::load_obj_mesh(path);
    uint32_t n = m->n_triangles() < cap ? m->n_triangles() : cap;
    if (positions) std::memcpy(positions, m->positions.data(), sizeof(float) * 9 * n);
    if (normals) std::memcpy(normals, m->normals.data(), sizeof(double) * 9 * n);
    if (uvs) std::memcpy(uvs, m->uvs.data(), sizeof(double) * 6 * n);
    return ok();
  } catch (const std::exception& e) {
    return fail(YART_ERR_IO, e.what());
  }
}

int yart_host_camera_init(yart_camera* cam, const double lookfrom[3], const double lookat[3], const double vup[3],
                          double vfov, double aspect, double aperture, double focus_dist, double t0, double t1) {
  int rc = yart_camera_init_impl(cam, lookfrom, lookat, vup, vfov, aspect, aperture, focus_dist, t0, t1);
  return rc ? fail(rc, "null argument") : ok();
}

}  // extern "C"
