/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A scalar f64 CPU restatement of the reference's per-pixel-sample hot path
 * (themayflyman/yet-another-raytracer, raytracer/src), used as the checker in tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg. The product (libyart.so) never
 * links, loads or calls anything here.
 *
 * It consumes the same flattened scene description as the product (include/yart.h) but
 * builds its own QBVH and evaluates the reference's semantics object by object.
 * Parity status: the reference (Rust nightly + crates.io) cannot be built or run in this
 * pipeline (no cargo/rustc), so the restatement is pinned by the reference's own unit tests
 * and fixtures (main.rs:808-828, color.rs:1988-2006, qbvh.rs:801-817, qbvh.rs:1168-1246),
 * by analytic known answers (SF66 Sellmeier indices, CIE_Y integral, OBJ triangle counts),
 * and by a literal recursive form of ray_reflectance checked against the iterative one.
 * The reference's RNG (rand 0.8.5 thread_rng, ChaCha12 from OS entropy) is unseedable; both
 * sides here use Philox4x32-10 keyed by (seed, pixel, sample) with rand 0.8.5's float/int
 * mappings restated (see DESIGN.md "RNG").
 */
#ifndef YART_ORACLE_H
#define YART_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/yart.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_scene oracle_scene;

int oracle_scene_create(const yart_scene_desc* desc, oracle_scene** out);
void oracle_scene_destroy(oracle_scene* s);
/* QBVH statistics of mesh m (qbvh.rs:252-361 construct): inner nodes, leaves, max depth. */
int oracle_qbvh_stats(const oracle_scene* s, uint32_t m, uint32_t* nodes, uint32_t* leaves,
                      uint32_t* depth);

/* main.rs:628-760 with the shared counter RNG. mode 0 = iterative reflectance (the form the
 * device uses), 1 = literal recursion (main.rs:537-588); | 2 = independent-stream mode (ChaCha12,
 * the reference's generator family, one sequential stream per sample; statistical tests only).
 * xyz_sum: W*H*3, only this shard's covered pixels are written. threads <= 0: all online CPUs. */
int oracle_render(const oracle_scene* s, const yart_camera* cam, const yart_render_params* p,
                  double* xyz_sum, int threads, int mode);
void oracle_chacha_block(const uint32_t in[16], uint32_t out[16], int double_rounds);
void oracle_chacha12_block(const uint32_t in[16], uint32_t out[16]);
/* main.rs:710-718 finalize. */
int oracle_finalize_rgba8(const double* xyz_sum, uint32_t w, uint32_t h, uint32_t spp,
                          uint8_t* rgba);
/* HittableList::hit over the world (hittable.rs:67-79); same layout as yart_intersect. */
int oracle_intersect(const oracle_scene* s, const double* rays, uint32_t n, double* hits,
                     int32_t* obj);
/* Per-pixel 8x8-job coverage of main.rs:636-647 (1 = sampled). */
int oracle_coverage(uint32_t w, uint32_t h, uint8_t* mask);

/* An OBJ reader of the oracle's own (oracle_obj.c): TriangleMesh::from_obj (triangle.rs:111-174)
 * over tobj's GPU_LOAD_OPTIONS, independent of the product's loader. positions n*9 f32, normals n*9
 * and uvs n*6 (may be NULL) f64. 0 or a negative error (-4: a file mixing vertices with and
 * without vn / vt, -5: unreadable). */
int oracle_obj_count(const char* path, uint32_t* n_triangles);
int oracle_obj_load(const char* path, float* positions, double* normals, double* uvs, uint32_t n_triangles);

/* Restated unit pieces for known-answer tests. */
void oracle_sanitize_sample_xyz(const double in[3], double out[3]);       /* main.rs:448-459 */
uint8_t oracle_clamp_display_channel(double c);                          /* main.rs:461-463 */
void oracle_gamma_corrected(const double in[3], double out[3]);          /* color.rs:92-107 */
void oracle_display_bytes(const double* linear, size_t n, uint8_t* out);  /* gamma + clamp, bulk */
void oracle_xyz_into_rgb(const double in[3], double out[3]);             /* color.rs:174-214 */
void oracle_xyz_from_wavelength(double wl, double out[3]);               /* color.rs:216-228 */
double oracle_rgb_reflect(const double rgb[3], double wl);               /* color.rs:54-90,160-164,276-283 */
double oracle_sellmeier_index(const double b[3], const double c[3], double wl); /* material.rs:251-257 */
double oracle_schlick(double cosine, double ref_idx);                    /* material.rs:207-211 */
int oracle_push_hit_children(uint32_t* stack, int cursor, const uint32_t children[4],
                             const uint32_t order[4], const int hits[4]); /* qbvh.rs:18-31 */
/* The shared stream: n draws of gen::<f64>() for (seed, pixel, sample). */
void oracle_rng_f64(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, double* out);
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double oracle_gen_range_f64(uint64_t seed, uint32_t pixel, uint32_t sample, double lo, double hi);
double oracle_sin(double x); /* deterministic sin/cos shared bit-for-bit with the device */
double oracle_cos(double x);
double oracle_log(double x); /* deterministic natural log (fdlibm), shared bit-for-bit with the device */
double oracle_acos(double x); /* deterministic acos / atan2 (fdlibm), likewise */
double oracle_atan2(double y, double x);
/* Texture::value of texture `tex` at point p, texture coordinates (u, v) and wavelength wl
 * (known-answer tests). */
double oracle_texture_probe(const oracle_scene* s, uint32_t tex, double wl, const double p[3], double u, double v);

#ifdef __cplusplus
}
#endif
#endif
