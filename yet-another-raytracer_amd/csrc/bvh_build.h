// bvh_build.h — host-side construction of the reference's 4-wide QBVH for one mesh.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "device_types.h"

namespace yart_dev {

struct BuiltMesh {
  std::vector<DevNode> nodes;       // the reference tree in post-order (root = nodes[ref_nodes - 1]),
                                    // then the walk tree's nodes (root = walk_root)
  std::vector<float> leaves;        // kTriFloats per triangle: the sorted order (see DevNode), then
                                    // the same triangles in the walk tree's leaf order
  std::vector<double> normals;      // 9 per sorted triangle
  std::vector<LeafAux> aux;         // per leaf: box + reference traversal rank per ray octant
  uint32_t depth = 0;               // inner-node levels on the deepest path
  float extent = 0.0f;              // max |vertex coordinate|
  uint32_t tied_cuts = 0;           // median cuts inside a run of equal centroid keys
  uint32_t tied_leaves = 0;         // leaves whose lane order rests on equal keys
  double build_ms = 0.0;            // host build time
  uint32_t ref_nodes = 0;           // reference-tree nodes (the first ref_nodes of `nodes`)
  uint32_t walk_root = 0;           // walk tree root (= ref root when there is no walk tree)
  uint32_t walk_nodes = 0, walk_depth = 0;
  double walk_build_ms = 0.0;
};

struct QbvhOptions {
  bool ties_desc = false;  // equal centroid keys in descending input order (probe of the tie freedom)
  uint32_t threads = 0;    // 0 = hardware concurrency; 1 = sequential
};

// L4QBVH::new (qbvh.rs:252-361): recursive median split into four children per node, <= 4
// triangles per leaf, centroid-extent axis choice and sort (qbvh.rs:637-693). Rust's
// sort_unstable_by leaves the order of equal keys unspecified; this build breaks ties by the
// triangle's input index (the oracle does the same). Subtrees are built on threads into
// preassigned slots, so the output does not depend on the thread count. Returns false (with
// `err`) when the mesh cannot be traversed the way the reference does (<= 4 triangles:
// qbvh.rs:383-384 underflows).
bool build_qbvh(uint32_t n_tris, const float* positions, const double* normals, BuiltMesh& out, std::string& err,
                const QbvhOptions& opt = QbvhOptions());

// The walk tree of the front-to-back traversal (not in the reference): a 4-wide tree over the
// same triangles built by the surface-area heuristic, appended to `m` (nodes after the reference
// tree's, records after the sorted ones). Its leaf records carry each triangle's reference leaf,
// lane in that leaf and sorted index, so the walk keeps the reference's tie order and exact check
// (kernels.hip, qbvh_coop). Every inner node has four non-empty children; depth <= max_depth (the
// traversal stack holds 3 depth + 1 entries).
void build_walk_tree(BuiltMesh& m, uint32_t max_depth);
// Structural check of the walk tree (yart_qbvh_build YART_QBVH_WALK; tests): every triangle in
// exactly one walk leaf with its record intact, every box inside its parent's, four non-empty
// children per inner node, depth <= max_depth.
bool check_walk_tree(const BuiltMesh& m, uint32_t max_depth);

}  // namespace yart_dev
