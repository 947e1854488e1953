// device_types.h — HBM layout of a scene on one MI355X (shared by the host side of libyart and
// the kernels). Everything the per-sample loop reads is resident; nothing is rebuilt per frame.
//
//  DevObject   world / light list entries in list order (hittable.rs:47-123). 320 B each; a wave
//              walks the list with a wave-uniform index, so the fields come in on the scalar path.
//  DevMaterial material table (material.rs), 64 B.
//  DevTexture  36-bin spectra precomputed from RGB with the Smits basis (color.rs:54-90): the
//              reference recomputes the whole spectrum per lookup and reads one bin; the bins are
//              bitwise the values it would read.
//  Mesh BLAS   the reference's L4QBVH (qbvh.rs:244-600) with its exact topology and child order:
//              DevNode 128 B (per child: box, child id, push ranks — 32 B); leaves as 192-B blocks of
//              <= 4 triangle records (48 B: v0 v1 v2, triangle index) + the f64
//              interpolated-normal table. Every f32 here is exact: tobj parses positions as f32
//              (triangle.rs:438) and box corners are min/max of those, so the f64 arithmetic of
//              the reference is reproduced bit for bit by converting on load.
#pragma once
#include <stdint.h>

#include "../../include/yart.h"

namespace yart_dev {

constexpr int kMaxXforms = 4;
// DevScene::plane_dirs (world_bvh.h BuiltWorld::plane_dirs): the half-width of the window around
// each in-plane direction, in diamond-angle units (<= radians). A computed local component is
// exactly 0 only within ~m 1e-15 rad of it (m RotateYs), or when the x-z direction is so short that
// the products underflow (world_closest_bvh checks that too).
constexpr double kPlaneDirWindow = 1e-9;
constexpr int kBins = 36;
constexpr int kStackSlots = 32;     // per-lane LDS traversal stack; 3*depth+1 <= 32 -> depth <= 10
constexpr uint32_t kMaxListObjects = 1u << 29;  // the world pass keeps obj << 3 | sub in one word (kernels.hip HitId)
constexpr int kMaxStackSlots = 64;  // the reference's stack (qbvh.rs:382-384): depth <= 21 (wavefront path)

struct DevObject {
  uint32_t kind, material, mesh, n_xf;
  uint32_t xf_kind[kMaxXforms];
  double xf[kMaxXforms][3];  // TRANSLATE: offset; ROTATE_Y: sin, cos (hittable.rs:173-176)
  double p[24];
};

struct DevMaterial {
  uint32_t kind, texture;
  double fuzz;
  double b[3], c[3];
};

struct DevTexture {
  uint32_t kind, noise_type;
  double spec[kBins];       // SOLID / CHECKER odd / NOISE: RGB(1,1,1) (texture.rs:272-296)
  double spec_even[kBins];  // CHECKER even
  double scale;             // NOISE
  const yart_perlin* perlin;  // NOISE: device copy of the tables
  uint32_t width, height;   // IMAGE
  const uint8_t* pixels;    // IMAGE: RGB8 rows, top first (device copy)
};

// Child k of a node is two float4s, read by lane k of a quad in the cooperative traversal (one
// 64-B load per quad per float4 row): lo[k] = (min x, max x, min y, max y), hi[k] = (min z,
// max z, child id bits, push ranks) — each axis's slab as an adjacent (min, max) pair. The push rank of child k for ray octant o (bits 2o..2o+1) is
// its position in the ORDER_TABLE row of the node's split axes (qbvh.rs:14-31), precomputed so a
// lane needs one shift instead of the table walk. Empty children have +inf boxes (QBVHNode::new,
// qbvh.rs:570-572).
struct alignas(16) DevNode {
  float lo[4][4];
  float hi[4][4];  // [k][2]: inner: node index; leaf: 1<<31 | count<<27 | leaf index; [k][3]: ranks
};
static_assert(sizeof(DevNode) == 128, "DevNode must be 128 B");
// Triangle records, 12 floats (48 B, three float4s) each: v0 v1 v2 (x y z each), then three words —
// the reference leaf holding the triangle (LeafAux index), its lane in that leaf and its sorted
// index (the row of the normal table). The first n records are the reference tree's, in the
// builder's sorted order; the next n the same triangles in the walk tree's leaf order
// (walk_tree.cpp). A leaf is the run [first, first + count) its node id names
// (1<<31 | count<<27 | first); lane k of a quad reads record first + k.
constexpr int kTriFloats = 12;


// Per-leaf side record for the front-to-back walk (qbvh_coop): the leaf's box exactly as its
// parent stores it, and the leaf's position in the reference's traversal order for each of the
// 8 ray octants (the depth-first order ORDER_TABLE gives, qbvh.rs:14-31, 520-531): the tie rule
// between equal-t hits in different leaves, and the box re-test that decides whether the
// front-to-back result is provably the reference's (kernels.hip, qbvh_coop).
struct alignas(16) LeafAux {
  float lo[3], hi[3];
  uint32_t pad[2];
  uint32_t rank[8];
};
static_assert(sizeof(LeafAux) == 64, "LeafAux must be 64 B");

struct DevMesh {
  const DevNode* nodes;
  const float* leaves;        // kTriFloats per triangle: sorted order, then the walk tree's leaf order
  const double* normals;      // 9 per sorted triangle: n0 n1 n2 (null when normals32 holds them)
  const float* normals32;     // the same in f32 when every value is exactly an f32 (OBJ vn)
  const LeafAux* aux;         // per leaf; null = walk in the reference's order only
  uint32_t root;              // the last node pushed (qbvh.rs:384)
  uint32_t n_nodes;           // reference + walk tree nodes
  float extent;               // max |vertex coordinate| (error scale of the f32 box test)
  uint32_t wroot;             // the walk tree's root (front to back; = root without a walk tree)
  uint32_t n_recs;            // triangle records (sorted + walk order)
  uint32_t n_leaves;          // reference leaves (LeafAux records)
  // The union of both roots' child boxes, laid out as a DevNode child (lo = min x, max x, min y,
  // max y; hi = min z, max z): a ray whose conservative f32 test misses it cannot pass any child
  // box of either root, so it is left out of the cooperative walk (qbvh_coop).
  float box_lo[4], box_hi[4];
};

// World BVH over the object list (not in the reference, whose HittableList is a linear scan):
// binary, f32 boxes padded outward so that culling is conservative; children of an inner node
// are adjacent (first, first + 1); a leaf lists `count` object indices from `first` in
// DevScene::world_objs. The closest hit it finds is the linear scan's (see world_closest_bvh).
struct alignas(16) DevWorldNode {
  float bmin[3];
  float mag;        // max |coordinate| of the box (margin scale)
  float bmax[3];
  uint32_t count;   // 0 = inner node
  uint32_t first;   // inner: left child (right = first + 1); leaf: first slot in world_objs
  uint32_t pad[3];  // pad[0]: leaf flags (kWorldLeafSpheres); pad[1]: the node's handle (below)
};
constexpr uint32_t kWorldLeafSpheres = 1u;  // every object of the leaf is a sphere without wrappers
// A node's handle: count << 28 | (kWorldLeafSpheres ? 1 << 27) | first — everything the walk needs
// to take the node, so descending and popping cost no dependent read of the node's own record.
constexpr uint32_t kWorldHandleMaxCount = 15u;
constexpr uint32_t kWorldHandleFirstMask = 1u << 27;
static_assert(sizeof(DevWorldNode) == 48, "DevWorldNode must be 48 B");
// The 4-wide world BVH the device walks (the binary tree above collapsed, two levels per node: each
// node's four children are the binary tree's nodes two levels down, or fewer where leaves come
// earlier): per child its f32 box — rounded outward as above and grown by the child's share of the
// walk's culling margin, mag · 2^-12, rounded outward again, so the walk adds only the ray's share
// (world_closest_bvh) — its magnitude (kept for the record's 128-B layout; the walk does not read
// it) and handle, laid out per axis so one lane reads a node with seven 16-B loads. An empty child
// slot has the handle kWorld4Empty and is never tested.
struct alignas(16) DevWorldNode4 {
  float bmin[3][4];   // [axis][child]
  float bmax[3][4];
  float mag[4];
  uint32_t handle[4]; // a node handle as above: leaf count << 28 | sphere flag | first slot, or an inner node's index
};
static_assert(sizeof(DevWorldNode4) == 128, "DevWorldNode4 must be 128 B");
constexpr uint32_t kWorld4Empty = 0xFFFFFFFFu;

struct DevScene {
  const DevObject* objects;
  const DevObject* lights;
  const DevMaterial* materials;
  const DevTexture* textures;
  const DevMesh* meshes;
  const double* background;  // 36 bins
  const DevWorldNode4* world_nodes;  // the 4-wide world BVH (root = node 0); null: walk the list linearly
  const uint32_t* world_objs;
  const double* world_sph;   // per world_objs slot: centre xyz, radius (plain spheres; else 0)
  const double* plane_dirs;  // BuiltWorld::plane_dirs (n_plane_dirs, a power of two; 0: none)
  uint32_t n_objects, n_lights, n_materials, n_textures, n_meshes;
  uint32_t has_mesh;
  uint32_t has_ext;  // noise/image textures, isotropic materials, media or moving spheres (EXT kernels)
  uint32_t has_time; // a MovingSphere reads the ray's shutter time: the camera draws it
  uint32_t n_world_nodes;
  uint32_t n_plane_dirs;
  uint32_t deep;     // a mesh needs more than kStackSlots stack entries: the 64-slot walk (wavefront only)
  uint32_t park;     // the persistent mesh kernel's walks park at this many busy quads (0: never; kernels.hip PARK)
};

}  // namespace yart_dev
