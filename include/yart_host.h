/*
 * yart_host.h — C ABI of the host-side layer (libyart_host.so): the reference's scene
 * presets, OBJ loading, CLI option resolution and PNG output, i.e. everything above the
 * render boundary of yart.h that the reference keeps on the CPU (main.rs:61-446,
 * scenes.rs, triangle.rs:111-174). Pure C++, no GPU: the CPU test suite uses it to build the
 * same scene descriptions the device library consumes.
 */
#ifndef YART_HOST_H
#define YART_HOST_H

#include <stdint.h>
#include "yart.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct yart_preset yart_preset;

/* RenderDefaults (main.rs:109-118) + the rest of ScenePreset (main.rs:132-140). */
typedef struct yart_render_defaults {
  uint32_t width, height;
  uint64_t samples_per_pixel, max_depth, workers;
  double vfov, aperture;
  double lookfrom[3], lookat[3], background[3];
  char output_filename[64];
} yart_render_defaults;

/* build_scene_preset (main.rs:211-432). scene: the clap value name ("cornell-box", ...).
 * asset_dir: directory holding the reference input meshes (input/ in the reference). scene_seed: drives the draws that
 * random_scene takes from thread_rng (scenes.rs:34). Errors: YART_ERR_INVALID (unknown name),
 * YART_ERR_UNSUPPORTED (scene needs out-of-scope features), YART_ERR_IO (mesh missing). */
int yart_preset_create(const char* scene, const char* asset_dir, uint64_t scene_seed, yart_preset** out);
void yart_preset_destroy(yart_preset* p);
const yart_scene_desc* yart_preset_desc(const yart_preset* p);
int yart_preset_defaults(const yart_preset* p, yart_render_defaults* out);
const char* yart_preset_stand_in(const yart_preset* p); /* "" unless a missing mesh was replaced */
int yart_scene_names(const char** names, int capacity);  /* returns the count */

/* resolve_dimensions (main.rs:166-186); 0 in an override = not given. */
void yart_resolve_dimensions(uint32_t default_w, uint32_t default_h, uint32_t width_override,
                             uint32_t height_override, uint32_t* w, uint32_t* h);

/* Parsed CLI (main.rs:78-107); unset numeric options are 0 / NaN, unset strings "". */
typedef struct yart_cli {
  char scene[64];
  char output[512];
  uint32_t width, height;
  uint64_t samples, max_depth, workers;
  double vfov, aperture;
  /* extensions of this build */
  uint64_t seed;
  int32_t gpus;
  char assets[512];
} yart_cli;
/* Returns 0, or YART_ERR_INVALID with yart_host_last_error() describing the clap-style error. */
int yart_cli_parse(int argc, const char* const* argv, yart_cli* out);
/* resolve_render_options (main.rs:188-209). */
typedef struct yart_render_options {
  char output_path[512];
  uint32_t width, height;
  uint64_t samples_per_pixel, max_depth, workers;
  double vfov, aperture;
} yart_render_options;
int yart_resolve_render_options(const char* default_filename, const yart_render_defaults* d,
                                const yart_cli* cli, yart_render_options* out);

/* OBJ loader (tobj 4.0.2 GPU_LOAD_OPTIONS semantics); copies up to cap triangles' data. */
int yart_obj_triangle_count(const char* path, uint32_t* n);
int yart_obj_load(const char* path, float* positions, double* normals, double* uvs, uint32_t cap);

/* RGBA8 PNG writer (image.save in main.rs:774). */
int yart_write_png(const char* path, const uint8_t* rgba, uint32_t width, uint32_t height);

/* Camera::new (camera.rs:41-80), identical to yart_camera_init in libyart. */
int yart_host_camera_init(yart_camera* cam, const double lookfrom[3], const double lookat[3],
                          const double vup[3], double vfov_degrees, double aspect_ratio,
                          double aperture, double focus_dist, double time0, double time1);

const char* yart_host_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
