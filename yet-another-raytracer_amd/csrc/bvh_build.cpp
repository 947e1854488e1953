// bvh_build.cpp — the reference's L4QBVH construction, emitted in the device layout.
#include "bvh_build.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

namespace yart_dev {
namespace {

struct Box {
  double mn[3], mx[3];
};

// ORDER_TABLE (qbvh.rs:14-16) row for a node's split axes (top | left << 2 | right << 4) and a
// ray octant (x >= 0 | y >= 0 << 1 | z >= 0 << 2): four nibbles, the child pushed k-th in nibble k
// (push_hit_children, qbvh.rs:18-31).
uint32_t push_order(uint32_t axes, uint32_t pos) {
  const uint64_t ORDER_LO = 0x1032102301320123ull, ORDER_HI = 0x3210231032012301ull;
  const uint32_t top = axes & 3u, left = (axes >> 2) & 3u, right = (axes >> 4) & 3u;
  const uint32_t idx = 4u * ((pos >> top) & 1u) + 2u * ((pos >> left) & 1u) + ((pos >> right) & 1u);
  return (uint32_t)(((idx < 4 ? ORDER_LO : ORDER_HI) >> (16u * (idx & 3u))) & 0xFFFFu);
}

struct Builder {
  const float* pos;
  std::vector<uint32_t> perm;      // working triangle order (sorted in place by split)
  std::vector<double> key;
  std::vector<Box> tri_box;        // Triangle::bounding_box (triangle.rs:37-62)
  std::vector<double> centroid;    // Hittable::centroid (hittable.rs:12-22), 3 per triangle
  BuiltMesh* out;

  // split (qbvh.rs:637-693): axis of the widest centroid extent (x; y if wider; z if wider than
  // both), sort the range by centroid on it, cut at len/2.
  int split(uint32_t off, uint32_t n) {
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = off; i < off + n; ++i) {
      const double* c = &centroid[3 * perm[i]];
      for (int a = 0; a < 3; ++a) { mn[a] = std::fmin(mn[a], c[a]); mx[a] = std::fmax(mx[a], c[a]); }
    }
    int axis = 0;
    if (mx[1] - mn[1] > mx[0] - mn[0]) axis = 1;
    if (mx[2] - mn[2] > std::fmax(mx[1] - mn[1], mx[0] - mn[0])) axis = 2;
    for (uint32_t i = off; i < off + n; ++i) key[perm[i]] = centroid[3 * perm[i] + axis];
    std::sort(perm.begin() + off, perm.begin() + off + n, [&](uint32_t a, uint32_t b) {
      if (key[a] < key[b]) return true;
      if (key[b] < key[a]) return false;
      return a < b;
    });
    return axis;
  }

  static Box merge(const Box& a, const Box& b) {  // surrounding_box (aabb.rs:187-202)
    Box r;
    for (int i = 0; i < 3; ++i) { r.mn[i] = std::fmin(a.mn[i], b.mn[i]); r.mx[i] = std::fmax(a.mx[i], b.mx[i]); }
    return r;
  }

  struct Result { bool has; Box box; uint32_t id; };

  Result leaf(uint32_t off, uint32_t n, const double* normals) {
    Box b = tri_box[perm[off]];
    for (uint32_t i = 1; i < n; ++i) b = merge(b, tri_box[perm[off + i]]);
    const uint32_t li = (uint32_t)out->aux.size();
    for (uint32_t i = 0; i < n; ++i) {  // triangle records in sorted order: leaf = [off, off + n)
      const float* v = &pos[9 * (size_t)perm[off + i]];
      float* rec = &out->leaves[kTriFloats * (size_t)(off + i)];
      for (int c = 0; c < 9; ++c) rec[c] = v[c];
      std::memcpy(&rec[9], &li, 4);  // the leaf's index (LeafAux)
      const double* nn = &normals[9 * (size_t)perm[off + i]];
      for (int c = 0; c < 9; ++c) out->normals[9 * (size_t)(off + i) + c] = nn[c];
    }
    LeafAux a{};
    for (int k = 0; k < 3; ++k) { a.lo[k] = (float)b.mn[k]; a.hi[k] = (float)b.mx[k]; }  // exact: f32 corners
    out->aux.push_back(a);
    return {true, b, (1u << 31) | (n << 27) | off};
  }

  Result construct(uint32_t off, uint32_t n, uint32_t level, const double* normals) {  // qbvh.rs:253-347
    if (n == 0) return {false, Box{}, 0xFFFFFFFFu};
    if (n <= 4) return leaf(off, n, normals);
    out->depth = std::max(out->depth, level + 1);
    uint32_t nl = n / 2, nr = n - n / 2;
    int top = split(off, n);
    int la = split(off, nl);
    Result ll = construct(off, nl / 2, level + 1, normals);
    Result lr = construct(off + nl / 2, nl - nl / 2, level + 1, normals);
    int ra = split(off + nl, nr);
    Result rl = construct(off + nl, nr / 2, level + 1, normals);
    Result rr = construct(off + nl + nr / 2, nr - nr / 2, level + 1, normals);
    DevNode node{};
    const Result* ch[4] = {&ll, &lr, &rl, &rr};
    const uint32_t axes = (uint32_t)top | ((uint32_t)la << 2) | ((uint32_t)ra << 4);
    for (int k = 0; k < 4; ++k) {
      // QBVHNode::new fills empty lanes with f64::MAX (qbvh.rs:570-572); +inf misses the same way.
      float mn[3], mx[3];
      for (int a = 0; a < 3; ++a) {
        mn[a] = ch[k]->has ? (float)ch[k]->box.mn[a] : INFINITY;
        mx[a] = ch[k]->has ? (float)ch[k]->box.mx[a] : INFINITY;
      }
      node.lo[k][0] = mn[0]; node.lo[k][1] = mx[0]; node.lo[k][2] = mn[1]; node.lo[k][3] = mx[1];
      node.hi[k][0] = mn[2]; node.hi[k][1] = mx[2];
      std::memcpy(&node.hi[k][2], &ch[k]->id, 4);
      uint32_t code = 0;  // this child's push rank for each of the 8 ray octants, 2 bits each
      for (uint32_t pos = 0; pos < 8; ++pos) {
        const uint32_t enc = push_order(axes, pos);
        for (uint32_t r = 0; r < 4; ++r)
          if (((enc >> (4 * r)) & 0xFu) == (uint32_t)k) code |= r << (2 * pos);
      }
      std::memcpy(&node.hi[k][3], &code, 4);
    }
    out->nodes.push_back(node);
    Box lb = ll.has && lr.has ? merge(ll.box, lr.box) : (ll.has ? ll.box : lr.box);
    Box rb = rl.has && rr.has ? merge(rl.box, rr.box) : (rl.has ? rl.box : rr.box);
    return {true, merge(lb, rb), (uint32_t)(out->nodes.size() - 1)};
  }
};

// Depth-first visit order of the leaves for one ray octant, as L4QBVH::hit walks them
// (qbvh.rs:520-531): a node's hit children are pushed in ORDER_TABLE order and popped last-first,
// so siblings are visited in descending push rank. Pruning only removes subtrees; it never
// reorders, so this rank orders any two leaves the reference visits for a ray of that octant.
void rank_leaves(BuiltMesh& m, uint32_t root) {
  for (uint32_t pos = 0; pos < 8; ++pos) {
    uint32_t next = 0;
    std::vector<uint32_t> stack{root};
    while (!stack.empty()) {
      const uint32_t id = stack.back();
      stack.pop_back();
      if (id >> 31) {
        uint32_t li;
        std::memcpy(&li, &m.leaves[kTriFloats * (size_t)(id & ((1u << 27) - 1u)) + 9], 4);
        m.aux[li].rank[pos] = next++;
        continue;
      }
      const DevNode& nd = m.nodes[id];
      uint32_t by_rank[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
      for (int k = 0; k < 4; ++k) {
        uint32_t child, code;
        std::memcpy(&child, &nd.hi[k][2], 4);
        std::memcpy(&code, &nd.hi[k][3], 4);
        by_rank[(code >> (2 * pos)) & 3u] = child;
      }
      for (int r = 0; r < 4; ++r)  // pushed lowest rank first: the highest rank is popped (visited) first
        if (by_rank[r] != 0xFFFFFFFFu) stack.push_back(by_rank[r]);
    }
  }
}

}  // namespace

bool build_qbvh(uint32_t n, const float* positions, const double* normals, BuiltMesh& out, std::string& err) {
  if (n <= 4) {
    err = "mesh has <= 4 triangles: the reference's L4QBVH::hit cannot traverse it (qbvh.rs:383-384)";
    return false;
  }
  if (n >= (1u << 27)) {
    err = "mesh has >= 2^27 triangles (leaf index field, qbvh.rs:270)";
    return false;
  }
  Builder b;
  b.pos = positions;
  b.out = &out;
  b.perm.resize(n);
  b.key.resize(n);
  b.tri_box.resize(n);
  b.centroid.resize(3 * (size_t)n);
  for (uint32_t t = 0; t < n; ++t) {
    b.perm[t] = t;
    Box bx;
    for (int a = 0; a < 3; ++a) {
      bx.mn[a] = INFINITY; bx.mx[a] = -INFINITY;
      for (int k = 0; k < 3; ++k) {
        double v = (double)positions[9 * (size_t)t + 3 * k + a];
        bx.mn[a] = std::fmin(bx.mn[a], v);
        bx.mx[a] = std::fmax(bx.mx[a], v);
      }
      b.centroid[3 * (size_t)t + a] = (bx.mx[a] + bx.mn[a]) / 2.0;
    }
    b.tri_box[t] = bx;
  }
  out.normals.assign(9 * (size_t)n, 0.0);
  out.leaves.assign(kTriFloats * (size_t)n, 0.0f);
  out.extent = 0.0f;  // max |coordinate| of the mesh (the f32 box test's error scale)
  for (size_t i = 0; i < 9 * (size_t)n; ++i) out.extent = std::max(out.extent, std::fabs(positions[i]));
  b.construct(0, n, 0, normals);
  rank_leaves(out, (uint32_t)out.nodes.size() - 1);
  if (3 * out.depth + 1 > (uint32_t)kStackSlots) {
    err = "QBVH too deep for the device traversal stack (depth " + std::to_string(out.depth) + ")";
    return false;
  }
  return true;
}

}  // namespace yart_dev
