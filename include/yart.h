/*
 * yart.h — C ABI of the MI355X (gfx950) path-tracing core.
 *
 * This is the drop-in boundary for the reference's per-pixel-sample render loop
 * (themayflyman/yet-another-raytracer, raytracer/src/main.rs:649-730, the closure each
 * thread-pool job runs). The reference has no FFI of its own: its path sits behind the Rust
 * traits `Hittable` (hittable.rs:11-35), `Material` (material.rs:20-31), `Texture`
 * (texture.rs:13-16), `Pdf` (pdf.rs:10-13) and `Camera::get_ray` (camera.rs:82-94). A host
 * that keeps those types (the reference's own Rust, or this repo's C++ mirror under
 * yet-another-raytracer_amd/host/) walks its scene tree once, flattens it into the plain
 * structs below and makes ONE call per frame (or per device shard). See INTEGRATION.md for
 * the Rust `extern "C"` binding a maintainer would add.
 *
 * Conventions
 *  - Every entry point returns 0 (YART_OK) or a negative yart_status; the message of the
 *    last failure on the calling thread is yart_last_error(). Nothing unwinds across the ABI
 *    (the reference panics instead: triangle.rs:113, main.rs:557, main.rs:774).
 *  - All inputs are caller-owned and copied during the call; outputs are caller-allocated.
 *  - Scene handles are immutable after yart_scene_create and may be used from several host
 *    threads at once: the host-output calls (yart_render, yart_render_with_stats,
 *    yart_intersect) each run on a library-owned stream of their own with their own scratch;
 *    the *_async calls run on the caller's stream, one frame's launches enqueued atomically.
 *    Calls on distinct devices' handles are independent.
 *  - Arithmetic is IEEE f64 throughout, as in the reference (no FMA contraction).
 */
#ifndef YART_H
#define YART_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YART_ABI_VERSION 1u

typedef enum yart_status {
  YART_OK = 0,
  YART_ERR_INVALID = -1,     /* bad argument / malformed scene description          */
  YART_ERR_DEVICE = -2,      /* HIP runtime or kernel failure                        */
  YART_ERR_NO_MEMORY = -3,   /* host or device allocation failed                     */
  YART_ERR_UNSUPPORTED = -4, /* a feature outside this build's scope                 */
  YART_ERR_IO = -5           /* file could not be read / written (host helpers only) */
} yart_status;

/* ---------------------------------------------------------------- textures (texture.rs) */
enum {
  YART_TEX_SOLID = 0,   /* SolidColor<RGB>            texture.rs:18-40   */
  YART_TEX_CHECKER = 1, /* CheckerTexture<RGB>        texture.rs:42-68   */
  YART_TEX_NOISE = 2,   /* NoiseTexture (Perlin)      texture.rs:262-300 */
  YART_TEX_IMAGE = 3    /* ImageTexture               texture.rs:302-345 */
};
enum { /* NoiseType, texture.rs:70-82 */
  YART_NOISE_SQUARE = 0,
  YART_NOISE_TRILINEAR = 1,
  YART_NOISE_SMOOTH = 2,
  YART_NOISE_MARBLE = 3,
  YART_NOISE_NET = 4
};
/* Perlin tables (texture.rs:84-112, POINT_COUNT = 256), drawn by the scene builder. */
typedef struct yart_perlin {
  double ranfloat[256];
  double ranvec[256][3];
  int32_t perm_x[256];
  int32_t perm_y[256];
  int32_t perm_z[256];
} yart_perlin;
typedef struct yart_texture {
  uint32_t kind;
  uint32_t noise_type;       /* NOISE: YART_NOISE_*                                       */
  double rgb[3];             /* SOLID: the colour.  CHECKER: the `odd` colour (sines < 0). */
  double rgb_even[3];        /* CHECKER: the `even` colour.                                */
  double scale;              /* NOISE: NoiseTexture::scale                                 */
  const yart_perlin* perlin; /* NOISE: its tables (copied by yart_scene_create)            */
  uint32_t width, height;    /* IMAGE: texel grid                                          */
  const uint8_t* pixels;     /* IMAGE: width*height RGB8 texels, rows top first (to_rgb8);
                                NULL / empty = the reference's no-data texture (value 1.0) */
} yart_texture;

/* --------------------------------------------------------------- materials (material.rs) */
enum {
  YART_MAT_NONE = 0,          /* NoMaterial          material.rs:383-386 */
  YART_MAT_LAMBERTIAN = 1,    /* Lambertian<T>       material.rs:33-61   */
  YART_MAT_METAL = 2,         /* Metal<T>            material.rs:63-95   */
  YART_MAT_DIELECTRIC = 3,    /* Dielectric          material.rs:111-301 (Sellmeier b, c in nm^2) */
  YART_MAT_DIFFUSE_LIGHT = 4, /* DiffuseLight<T>     material.rs:336-355 */
  YART_MAT_ISOTROPIC = 5      /* Isotropic<T>        material.rs:357-381 (phase function of a medium) */
};
typedef struct yart_material {
  uint32_t kind;
  uint32_t texture; /* index into yart_scene_desc.textures (LAMBERTIAN, METAL, DIFFUSE_LIGHT) */
  double fuzz;      /* METAL */
  double b[3];      /* DIELECTRIC Sellmeier B1..B3 */
  double c[3];      /* DIELECTRIC Sellmeier C1..C3 (nm^2, e.g. SF66 c1 = 0.0147053225e6) */
} yart_material;

/* ------------------------------------------------------------------------- objects */
enum {
  YART_PRIM_SPHERE = 0,   /* StillSphere      sphere.rs:31-119   p = cx, cy, cz, radius      */
  YART_PRIM_XY_RECT = 1,  /* XYRect           aarect.rs:9-77     p = x0, x1, y0, y1, k       */
  YART_PRIM_XZ_RECT = 2,  /* XZRect           aarect.rs:79-172   p = x0, x1, z0, z1, k       */
  YART_PRIM_YZ_RECT = 3,  /* YZRect           aarect.rs:174-242  p = y0, y1, z0, z1, k       */
  YART_PRIM_BOX = 4,      /* BoxEntity        box_entity.rs      p = p0 xyz, p1 xyz          */
  YART_PRIM_TRIANGLE = 5, /* Triangle         triangle.rs:19-102 p = v0 v1 v2 (9), n0 n1 n2 (9), uv0 uv1 uv2 (6) */
  YART_PRIM_MESH = 6,     /* TriangleMesh     triangle.rs:104-185 (L4QBVH, qbvh.rs:244-544); `mesh` selects the triangles */
  YART_PRIM_MOVING_SPHERE = 7 /* MovingSphere sphere.rs:121-211 p = center0 xyz, center1 xyz, time0, time1, radius;
                                 its presence makes the camera draw the shutter time (camera.rs:91) */
};
enum {
  YART_XF_TRANSLATE = 1, /* Translate  hittable.rs:125-163  v = offset            */
  YART_XF_ROTATE_Y = 2,  /* RotateY    hittable.rs:165-256  v[0] = angle, degrees */
  YART_XF_FLIP_FACE = 3, /* FlipFace   hittable.rs:328-354                        */
  YART_XF_MEDIUM = 4     /* ConstantMedium hittable.rs:258-326, v[0] = density; only as the
                            OUTERMOST wrapper: the rest of the chain + the primitive is its
                            boundary, the object's material its phase function (Isotropic) */
};
typedef struct yart_xform {
  uint32_t kind;
  uint32_t reserved;
  double v[3];
} yart_xform;

#define YART_MAX_XFORMS 4
typedef struct yart_object {
  uint32_t kind;     /* YART_PRIM_* */
  uint32_t material; /* index into materials; a MESH object's triangles all share it, as
                        TriangleMesh::from_obj gives every triangle one material (triangle.rs:111) */
  uint32_t mesh;     /* MESH: index into yart_scene_desc.meshes; two objects may share a mesh */
  uint32_t n_xforms; /* wrappers around the primitive, OUTERMOST first:
                        Translate(RotateY(Box)) = { TRANSLATE, ROTATE_Y } */
  yart_xform xforms[YART_MAX_XFORMS];
  double p[24];
} yart_object;

/* A triangle soup as TriangleMesh::from_obj produces it (triangle.rs:111-174): positions are
 * the f32 values tobj parsed, normals/uvs already defaulted (face normal / (0,0)). */
typedef struct yart_mesh {
  uint32_t n_triangles;
  uint32_t reserved;
  const float* positions; /* n_triangles * 9 : v0 xyz, v1 xyz, v2 xyz                 */
  const double* normals;  /* n_triangles * 9 : n0, n1, n2 (not normalised, as stored) */
  const double* uvs;      /* n_triangles * 6 or NULL (u/v are not read by in-scope textures) */
} yart_mesh;

typedef struct yart_scene_desc {
  uint32_t abi_version; /* = YART_ABI_VERSION */
  uint32_t n_objects;
  uint32_t n_lights;
  uint32_t n_materials;
  uint32_t n_textures;
  uint32_t n_meshes;
  const yart_object* objects;   /* the world HittableList, in insertion order (scenes.rs)   */
  const yart_object* lights;    /* the `lights` HittableList (main.rs:221), in order; only
                                   bare XZ_RECT and SPHERE entries carry a pdf (aarect.rs:148-171,
                                   sphere.rs:95-118), every other entry pdf 0 (hittable.rs:28-34) */
  const yart_material* materials;
  const yart_texture* textures;
  const yart_mesh* meshes;
  double background[3]; /* background RGB, reflected spectrally on a miss (main.rs:587) */
} yart_scene_desc;

/* Camera (camera.rs:10-23). Fill with yart_camera_init (camera.rs:41-80). */
typedef struct yart_camera {
  double lower_left_corner[3];
  double horizontal[3];
  double vertical[3];
  double origin[3];
  double u[3];
  double v[3];
  double w[3];
  double lens_radius;
  double time0;
  double time1;
} yart_camera;

/* One frame (or one shard of it). The reference renders the pixels covered by its fixed 8x8
 * grid of crop rectangles (main.rs:628-647): pixels outside every crop (e.g. row 224 of a
 * 225-row image) are never sampled, their sums stay 0 and finalize leaves them RGBA 0,0,0,0.
 * Work is dealt to devices in 8x8-pixel blocks: block b (row-major over ceil(W/8) x ceil(H/8))
 * is rendered by the shard with b % shard_count == shard_index. */
typedef struct yart_render_params {
  uint32_t width;
  uint32_t height;
  uint32_t spp;       /* samples_per_pixel */
  uint32_t max_depth; /* ray_color depth    */
  uint64_t seed;      /* counter-based RNG key (Philox4x32-10); the reference's thread_rng()
                         is unseedable, see DESIGN.md "RNG" */
  uint32_t shard_index;
  uint32_t shard_count; /* 0 or 1 = whole frame */
  /* Samples one wave renders per 8x8 block before handing over (0 = chosen by the library from
   * the device size). Below spp, each sample's value goes to an HBM scratch and a second kernel
   * adds them per pixel in sample order, so the sums are bitwise those of one sequential loop
   * (main.rs:691-708) whatever the split; it only changes how finely work spreads over CUs. */
  uint32_t samples_per_unit;
  uint32_t reserved;
} yart_render_params;

typedef struct yart_scene yart_scene; /* opaque, device resident */

typedef struct yart_scene_info {
  int device;
  uint32_t n_objects;
  uint32_t n_lights;
  uint32_t n_meshes;
  uint32_t bvh_nodes;     /* inner QBVH nodes over all meshes (qbvh.rs:547-554)        */
  uint32_t bvh_leaves;    /* leaves (<= 4 triangles each, qbvh.rs:261-279)              */
  uint32_t bvh_max_depth; /* deepest root-to-leaf path in inner nodes                   */
  uint32_t bvh_max_stack; /* traversal stack slots the deepest path can need            */
  uint64_t device_bytes;  /* HBM held by the scene                                      */
  uint32_t world_nodes;   /* 4-wide world BVH nodes over the object list (0 = linear walk) */
  uint32_t world_depth;   /* its deepest root-to-leaf path (4-wide levels)              */
  uint32_t bvh_tied_cuts; /* QBVH median cuts inside a run of equal centroid keys:
                             where Rust's unstable sort (qbvh.rs:679-685) may order differently */
  uint32_t bvh_tied_leaves; /* leaves whose triangle order rests on equal keys              */
  double bvh_build_ms;    /* host QBVH build time, all meshes                           */
  double upload_ms;       /* host -> device copies of the scene                         */
  uint32_t walk_nodes;    /* nodes of the front-to-back walk's SAH tree (0 = none)      */
  uint32_t walk_depth;    /* its deepest root-to-leaf path in inner nodes               */
} yart_scene_info;

/* Per-launch work counters (optional, for roofline accounting; they slow the kernel). */
typedef struct yart_render_stats {
  uint64_t samples;        /* camera samples completed                           */
  uint64_t segments;       /* world.hit calls on path rays (hittable.rs:67)      */
  uint64_t prim_tests;     /* analytic primitive tests (sphere/rect/triangle)    */
  uint64_t node_visits;    /* QBVH inner nodes tested (4 boxes each)             */
  uint64_t leaf_visits;    /* QBVH leaves tested (<= 4 triangles each)           */
  uint64_t leaf_tris;      /* triangles tested inside leaves                     */
  uint64_t light_tests;    /* primitive hits re-run by pdf_value (pdf.rs:452)    */
  uint64_t mesh_rewalks;   /* front-to-back QBVH walks redone in reference order */
  uint64_t coop_rounds;    /* cooperative QBVH walk: wave rounds (16 quad steps)  */
  uint64_t coop_leaf_rounds; /* ... rounds in which some quad tested a leaf      */
  uint64_t coop_walks;     /* ... wave-level walks started                       */
  uint64_t coop_idle_slots; /* ... quad slots of those rounds holding no ray (the drain) */
  uint64_t world_iters;    /* world-BVH walk: loop iterations the waves issue (per-lane visits: node_visits, prim_tests) */
  uint64_t world_leaf_iters; /* ... of them with some lane at a leaf               */
  uint64_t ovf_pushes;     /* deep meshes: walk-stack entries pushed past the LDS slots into HBM */
  /* where the waves' lane-slots go (sums of active lanes, 64 per wave-instruction slot): */
  uint64_t coop_node_rounds;    /* cooperative walk rounds whose inner-node branch runs          */
  uint64_t coop_node_lanes;     /* ... lanes in that branch (4 per quad at a node)               */
  uint64_t coop_leaf_lanes;     /* lanes testing a triangle in the leaf branch (coop_leaf_rounds) */
  uint64_t coop_leaf_quad_lanes; /* ... lanes of the quads at a leaf (4 per quad)                */
  uint64_t iterations;          /* render-loop iterations (per wave)                             */
  uint64_t camera_lanes;        /* lanes starting a camera ray, summed over iterations           */
  uint64_t scatter_lanes;       /* lanes scattering at a hit, summed over iterations             */
  uint64_t camera_iters;        /* iterations in which some lane starts a camera ray             */
  uint64_t scatter_iters;       /* iterations in which some lane scatters                        */
  uint64_t parked_walks;        /* mesh walks parked for the next bounce (YART_OPT_MESH_PARK)    */
} yart_render_stats;

typedef void (*yart_progress_fn)(uint64_t pixels_done, void* user);

/* ------------------------------------------------------------------------ entry points */
const char* yart_version(void);
/* sha256 (hex) of the sources this library was compiled from (yet-another-raytracer_amd/yart/buildid.py
 * lists them): a host can check that a prebuilt library belongs to the source tree it ships with. */
const char* yart_build_id(void);
const char* yart_last_error(void); /* thread-local; "" when the last call succeeded */

int yart_device_count(int* out);

/* Copies the description to `device` (HBM), building the mesh QBVHs (qbvh.rs:252-361). */
int yart_scene_create(int device, const yart_scene_desc* desc, yart_scene** out);
void yart_scene_destroy(yart_scene* scene);
int yart_scene_get_info(const yart_scene* scene, yart_scene_info* out);

/* camera.rs:41-80 (host arithmetic, f64). */
int yart_camera_init(yart_camera* cam, const double lookfrom[3], const double lookat[3],
                     const double vup[3], double vfov_degrees, double aspect_ratio,
                     double aperture, double focus_dist, double time0, double time1);

/* Render into a DEVICE buffer on a caller stream (hipStream_t, NULL = default stream).
 * d_xyz_sum: width*height*3 doubles on the scene's device, per-pixel sums of the sanitised
 * sample XYZ (main.rs:690-708). Only this shard's blocks are written; the caller zeroes the
 * buffer if it wants the rest to read 0. Asynchronous: returns after the launch — except on the
 * wavefront path (YART_OPT_MESH_WAVEFRONT = 1), whose number of
 * iterations is data-dependent: there the calling thread stays in the launch loop until the frame's
 * last iteration is queued (the device may still be finishing it on return), and progress words
 * move only at the end of the frame. The same holds for yart_render_packed_async and
 * yart_render_multi_async on such scenes. */
int yart_render_async(yart_scene* scene, const yart_camera* cam, const yart_render_params* p,
                      double* d_xyz_sum, void* hip_stream);

/* Device time of the kernels of every frame launched on `hip_stream` since the previous call,
 * from HIP events recorded on that stream around each launch: summed render-kernel time, summed
 * in-order accumulate time (0 for frames that ran fused) and the number of frames. Call after the
 * stream has finished those frames; the events are then recycled. */
int yart_frame_timing(yart_scene* scene, void* hip_stream, double* render_ms, double* accumulate_ms,
                      uint32_t* frames);

/* Same, with host output and an optional progress callback, called on this thread while the
 * device renders (every ~10 ms when the count moved): pixels_done is monotone, counts the covered
 * pixels of the shard whose work has been handed out (chunked plan) or finished (fused plan), and
 * the last call reports all of them. */
int yart_render(yart_scene* scene, const yart_camera* cam, const yart_render_params* p,
                double* xyz_sum_out, yart_progress_fn progress, void* user);

/* Instrumented render (same image) that also returns the work counters. Host output. */
int yart_render_with_stats(yart_scene* scene, const yart_camera* cam,
                           const yart_render_params* p, double* xyz_sum_out,
                           yart_render_stats* stats);

/* ------------------------------------------------ multi-GPU: shards + one RCCL gather
 * Replaces the reference's fan-out of 64 tile jobs over its thread pool and the stitching of
 * their results into one image (main.rs:633-660, 747-760): the frame's 8x8-pixel blocks are dealt
 * round-robin to devices (block b -> shard b % N), each device renders its blocks into a PACKED
 * buffer and ONE gather over RCCL/xGMI brings every shard to the root, which unpacks the frame.
 *
 * Packed layout of shard s of N (the gather's wire format): its blocks in local order (local
 * block j = global block s + j*N), 64 pixel slots per block (slot = (y % 8) * 8 + x % 8), 3
 * doubles (XYZ sum) per slot; slots outside the frame or the crop grid are unspecified. */
uint64_t yart_shard_packed_len(uint32_t width, uint32_t height, uint32_t shard_index,
                               uint32_t shard_count); /* doubles */

/* yart_render_async with the packed output (p->shard_index / shard_count select the shard). */
int yart_render_packed_async(yart_scene* scene, const yart_camera* cam, const yart_render_params* p,
                             double* d_packed, void* hip_stream);

/* RCCL communicator over the devices of the frame, one rank per device.
 *   one process per GPU: rank 0 calls yart_comm_unique_id, hands the 128 bytes to every rank
 *                        (torch.distributed, MPI, a file ...), each calls yart_comm_init_rank;
 *   one process, N GPUs: yart_comm_init_all (ncclCommInitAll), comms_out[d] for devices[d]. */
#define YART_COMM_ID_BYTES 128
typedef struct yart_comm yart_comm;
int yart_comm_unique_id(uint8_t id_out[YART_COMM_ID_BYTES]);
int yart_comm_init_rank(const uint8_t id[YART_COMM_ID_BYTES], int n_ranks, int rank, int device,
                        yart_comm** out);
int yart_comm_init_all(int n_devices, const int* devices, yart_comm** comms_out);
void yart_comm_destroy(yart_comm* comm);

/* Every rank's packed shard (rank r holds shard r of n_ranks, `d_packed` on its device) -> the
 * whole W x H x 3 frame in `d_frame` on `root` (ignored elsewhere; every pixel written, 0 outside
 * the crop grid): ONE ncclGather of equal-sized packets, then an unpack kernel on the root. Bitwise
 * the one-device render: each pixel has exactly one writer. `d_packed` must hold
 * yart_shard_packed_len(width, height, 0, n_ranks) doubles (the largest shard: packets are equal
 * sized). Enqueued on `hip_stream` (the rank's
 * device); collective — every rank must call it. Not for comms from yart_comm_init_all (use
 * yart_render_multi, which groups the ranks' calls). */
int yart_gather_frame_async(yart_comm* comm, const double* d_packed, uint32_t width, uint32_t height,
                            int root, double* d_frame, void* hip_stream);

/* One process driving N devices: a scene resident on each (uploaded once) and an RCCL
 * communicator over them (ncclCommInitAll). p->shard_index / shard_count are ignored (device d
 * renders shard d of N).
 *
 * yart_render_multi_async is the timed multi-GPU path (bench.py --gpus N without a launcher):
 * every device renders its shard into a packed buffer on a stream of the multi's own, the
 * grouped ncclGather is enqueued right behind each device's render (stream order, no host wait)
 * and devices[0] unpacks the frame into d_frame (width*height*3 doubles on devices[0]) after the
 * work already queued on `hip_stream` (a stream of devices[0]), which then waits for the frame.
 * Frames submitted on different caller streams overlap on the devices; their gathers run in
 * submission order on every device. Bitwise yart_render on one device: each pixel has one writer.
 * Each caller stream gets its own set of device streams and buffers, made on its first frame and
 * kept for the next; at most 8 such sets live at once, and a ninth caller stream takes over the
 * least recently used set after that set's frames have finished. All are freed by
 * yart_multi_destroy.
 *
 * yart_render_multi is the same submission with host output and an optional progress callback
 * (pixels over all devices, on the calling thread); it waits for the frame and copies it to
 * xyz_sum_out. */
typedef struct yart_multi yart_multi;
int yart_multi_create(int n_devices, const int* devices, const yart_scene_desc* desc, yart_multi** out);
int yart_render_multi_async(yart_multi* m, const yart_camera* cam, const yart_render_params* p,
                            double* d_frame, void* hip_stream);
int yart_render_multi(yart_multi* m, const yart_camera* cam, const yart_render_params* p,
                      double* xyz_sum_out, yart_progress_fn progress, void* user);
/* Device time of the frames submitted with yart_render_multi_async since the previous call (call
 * once they have finished): the slowest device's summed render-kernel time, the root's summed
 * gather + unpack time (from the root's gather launch, so it includes waiting for the slowest
 * device) and the number of frames. */
int yart_multi_frame_timing(yart_multi* m, double* render_ms, double* gather_ms, uint32_t* frames);
/* Per device, summed over the frames the latest yart_multi_frame_timing read (or the latest
 * yart_render_multi): render_ms[d] its render-kernel time, gather_ms[d] the intervals of its own
 * ncclGather (from its launch, behind its render, to its end: a device that rendered early waits
 * there for the others), *frames their number. n must be the multi's device count. The per-device
 * balance of a multi-GPU frame: render max / mean, and which device the others waited for. */
int yart_multi_device_timing(yart_multi* m, int n, double* render_ms, double* gather_ms, uint32_t* frames);
/* Device time of the last yart_render_multi: render (slowest device) and gather + unpack, ms. */
int yart_multi_last_timing(const yart_multi* m, double* render_ms, double* gather_ms);
/* Where the latest frame submitted to `m` stands, without waiting (a watchdog names the stage a
 * stalled frame is in): state[d] for each device 0 = rendering, 1 = rendered (its part of the gather
 * pending), 2 = gathered; *unpacked = 1 once devices[0] has unpacked the frame, else 0. While a
 * submission is being enqueued (or before the first), every value reads -1. */
int yart_multi_query(yart_multi* m, int32_t* state, int32_t* unpacked);
void yart_multi_destroy(yart_multi* m);

/* The root side of the gather on its own (k_unpack_shards): `shards` packets back to back in
 * d_recv, packet r (shard r's packed buffer) at r * stride doubles, stride >= the largest shard's
 * yart_shard_packed_len -> the whole frame in d_frame (0 outside the crop grid). Device buffers,
 * caller stream. Lets a caller that moves packets by other means (or a test) assemble frames. */
int yart_unpack_shards_async(int device, const double* d_recv, uint32_t shards, uint64_t stride,
                             uint32_t width, uint32_t height, double* d_frame, void* hip_stream);

/* main.rs:710-718: xyz * 360 / (CIE_Y_INTERGAL * spp) -> XYZ::into_rgb -> sRGB gamma ->
 * (256 * clamp(c, 0, 0.999)) as u8, alpha 255; pixels the tile grid never covers -> 0,0,0,0.
 * Device buffers, caller stream. */
int yart_finalize_rgba8_async(int device, const double* d_xyz_sum, uint32_t width,
                              uint32_t height, uint32_t spp, uint8_t* d_rgba, void* hip_stream);
int yart_finalize_rgba8(int device, const double* xyz_sum, uint32_t width, uint32_t height,
                        uint32_t spp, uint8_t* rgba_out); /* host buffers */

/* Batched closest hit against the world list: the `Hittable::hit` boundary
 * (hittable.rs:24, HittableList::hit hittable.rs:67-79), on the device.
 * rays: n * 8 doubles (origin xyz, direction xyz, t_min, t_max).
 * hits: n * 8 doubles (t, p xyz, normal xyz, front_face 0/1); obj: n ints, the index of the
 * world object hit or -1 (then hits[] is left as NaN). Host buffers. */
int yart_intersect(yart_scene* scene, const double* rays, uint32_t n, double* hits,
                   int32_t* obj);

/* Host-only QBVH build (no device): the L4QBVH of scene creation for one mesh, reported
 * without uploading it — build time, shape, the tie exposure and a digest of the device
 * arrays (FNV-1a 64 over node records, triangle records, leaf records, normals), so builder
 * variants can be compared byte for byte. flags: YART_QBVH_TIES_DESC orders equal centroid
 * keys by descending input index instead of ascending (the probe of sort_unstable_by's freedom,
 * qbvh.rs:679-685); YART_QBVH_SERIAL builds on one thread; YART_QBVH_WALK also builds the
 * front-to-back walk's SAH tree (as scene creation does) and checks its structure: every triangle
 * in exactly one walk leaf, every box holding what is below it, four non-empty children per inner
 * node, the depth within the 32-slot stack (walk_valid = 1). */
#define YART_QBVH_TIES_DESC 1u
#define YART_QBVH_SERIAL 2u
#define YART_QBVH_WALK 4u
typedef struct yart_qbvh_build_info {
  uint32_t nodes, leaves, depth, tied_cuts, tied_leaves, reserved;
  uint64_t digest;
  double build_ms;
  uint32_t walk_nodes, walk_depth, walk_valid, walk_reserved;
  double walk_build_ms;
} yart_qbvh_build_info;
int yart_qbvh_build(const float* positions, const double* normals, uint32_t n_triangles, uint32_t flags,
                    yart_qbvh_build_info* out);

/* The world BVH of a scene description on its own (no device): the binary SAH tree and the 4-wide
 * tree the device walks, built exactly as yart_scene_create builds them (whatever the object count;
 * built = 0 when some object has no box: meshes, media, moving spheres), then the 4-wide tree's
 * structural check (world_bvh.cpp check_world4: every object in exactly one leaf, every child box
 * holding the objects below it grown by the child's culling margin (magnitude 2^-12, the magnitude
 * bounding its coordinates), depth within the walk's stack; valid = 1, or the reason in
 * yart_last_error). digest: FNV-1a 64 over the 4-wide nodes, leaf slots and sphere records. */
typedef struct yart_world_bvh_info {
  uint32_t built, nodes, depth, nodes4, depth4, valid;
  uint64_t digest;
} yart_world_bvh_info;
int yart_world_bvh_build(const yart_scene_desc* desc, yart_world_bvh_info* out);

/* Test probes (device side of the parity tests). */
/* The per-sample random stream: n draws of gen::<f64>() for (pixel, sample). */
int yart_probe_rng(int device, uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n,
                   double* out);
/* Elementwise device math on n inputs: op 0 sqrt(a), 1 a/b, 2 sin(a), 3 cos(a), 4 pow(a,b)
 * (the vendor's; no kernel uses it), 5 ln(a), 6 acos(a), 7 atan2(a,b) (2-3, 5-7: the deterministic
 * fdlibm forms the kernels use), 8-10 the guarded fast sqrt / unit / quotient, 11 the 8-bit
 * channel k_finalize gives the linear value a (gamma_corrected + clamp_display_channel). */
int yart_probe_math(int device, int op, const double* a, const double* b, uint32_t n,
                    double* out);
/* on != 0: every mesh ray whose front-to-back walk found a hit is walked again in the reference's
 * order (the per-lane walk the exact post-walk check falls back to), for the frames rendered on
 * this device until it is called with on = 0. The result is the same; only slower. */
int yart_debug_force_rewalk(int device, int on);

/* Test and tuning hooks, process-wide. The library reads no environment variable: every switch
 * that changes how it builds or renders (never what it computes — each setting gives the same
 * bits) is one of these, read at the next yart_scene_create (build and path choices) or frame
 * (scratch budget). The defaults are the shipped behaviour; tests set them and restore them. */
enum {
  YART_OPT_QBVH_TIES_DESC = 0, /* 0 | 1: equal centroid keys in descending input order (the probe of
                                  sort_unstable_by's freedom, qbvh.rs:679-685)                      */
  YART_OPT_QBVH_THREADS = 1,   /* host builder threads, 0 = the hardware's concurrency              */
  YART_OPT_WALK_TREE = 2,      /* 1 | 0: build the SAH walk tree / walk the reference tree front to back */
  YART_OPT_MESH_WALK_REF = 3,  /* 0 | 1: every mesh ray walks in the reference's order (qbvh.rs:381-543) */
  YART_OPT_WORLD_BVH = 4,      /* -1 auto (>= 16 objects, no mesh) | 0 never | 1 whenever every object has a box */
  YART_OPT_MESH_WAVEFRONT = 5, /* -1 / 0: the megakernel for every mesh scene (deep meshes included, their walk
                                  stacks overflowing into HBM) | 1: the wavefront path for every mesh scene
                                  without media / moving spheres / noise or image textures */
  YART_OPT_WF_POOL = 6,        /* wavefront path slots, >= 256 (rounded down to a multiple of 256), default 2^20 */
  YART_OPT_SCRATCH_BYTES = 7,  /* sample-scratch budget per pass and stream in bytes; 0 (default) =
                                  auto: min(16 GiB, an eighth of the device's memory); a frame
                                  that needs more renders in overlapped passes over two halves  */
  YART_OPT_UNITS_PER_WAVE = 8, /* persistent-wave plan: work units per resident wave; 0 (default) = auto:
                                  64 for list-walk scenes, 192 with a mesh or the world BVH          */
  YART_OPT_MESH_PARK = 9,      /* mesh walks stop once their wave's queue is empty and at most this many
                                  of its 16 quads still walk, and go on at the next bounce with the
                                  new rays (one mesh object, depth <= 10); 0 = never; default 8   */
  YART_OPT_COUNT = 10
};
int yart_debug_set_option(int option, int64_t value);
int yart_debug_get_option(int option, int64_t* value);

#ifdef __cplusplus
}
#endif
#endif /* YART_H */
