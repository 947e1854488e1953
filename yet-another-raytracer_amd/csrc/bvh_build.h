// bvh_build.h — host-side construction of the reference's 4-wide QBVH for one mesh.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "device_types.h"

namespace yart_dev {

struct BuiltMesh {
  std::vector<DevNode> nodes;       // post-order; root = nodes.back()
  std::vector<float> leaves;        // kTriFloats per triangle, sorted order (see DevNode)
  std::vector<double> normals;      // 9 per sorted triangle
  std::vector<LeafAux> aux;         // per leaf: box + reference traversal rank per ray octant
  uint32_t depth = 0;               // inner-node levels on the deepest path
  float extent = 0.0f;              // max |vertex coordinate|
  uint32_t tied_cuts = 0;           // median cuts inside a run of equal centroid keys
  uint32_t tied_leaves = 0;         // leaves whose lane order rests on equal keys
  double build_ms = 0.0;            // host build time
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

}  // namespace yart_dev
