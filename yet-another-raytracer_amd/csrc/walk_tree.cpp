// walk_tree.cpp — the front-to-back walk's own 4-wide tree over a mesh's triangles (not in the
// reference). The reference's L4QBVH splits at the median triangle count (qbvh.rs:637-693), so a
// node's children often overlap and a ray walks into boxes that a better-shaped tree would skip.
// The walk tree regroups the same triangles by the surface-area heuristic; the answer stays the
// reference tree's because the walk only proposes a candidate, keyed by the reference's order, and
// the exact check at the end of each walk uses the reference leaf's box (kernels.hip, qbvh_coop).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <future>
#include <vector>
#ifdef YART_WALK_TREE_STATS
#include <cstdio>
#endif

#include "bvh_build.h"

namespace yart_dev {
namespace {

struct WItem {
  float lo[3], hi[3];  // the triangle's box (exact f32: min/max of its vertices)
  float c[3];          // centroid key (box centre), for binning only
  uint32_t tri;        // sorted (reference) index
};

struct Box3 {
  float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const WItem& t) {
    for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], t.lo[k]); hi[k] = std::max(hi[k], t.hi[k]); }
  }
  void grow(const Box3& b) {
    for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); }
  }
  double area() const {
    if (!(hi[0] >= lo[0])) return 0.0;
    const double x = (double)hi[0] - lo[0], y = (double)hi[1] - lo[1], z = (double)hi[2] - lo[2];
    return x * y + y * z + z * x;
  }
};

// Inner levels a 4-way tree over n triangles needs at least (leaves hold <= 4).
uint32_t min_levels(size_t n) {
  uint32_t l = 0;
  while (n > 4) { n = (n + 3) / 4; ++l; }
  return l;
}

// The SAH's count term: the quad steps a part's leaves take, ceil(n / 4), not its triangle count.
// A leaf step costs the walk one round for its quad whether the leaf holds 1 or 4 triangles, so
// cuts at multiples of 4 are what saves rounds (r05: leaves 2.05 -> 2.55 triangles, quad steps per
// ray through the root by surface area 18.24 -> 17.77 on david; bunny +1.0 %, david +1.9 / +2.4 %,
// same box, bitwise: profiles/r05_ab_walk_tree_quad_sah.log). YART_WALK_LEAF_QUANT=1 (make variant
// DEFS=...) builds the r03-r04 tree.
#ifndef YART_WALK_LEAF_QUANT
#define YART_WALK_LEAF_QUANT 4
#endif
// The 4-wide tree from a binary SAH tree by dynamic programming (r05, the default; 0: the greedy
// 4-way expansion of r03-r04), for meshes of at most kDpMaxTris triangles (its tables take ~100 B
// per triangle); larger meshes, or a mesh whose tree cannot fit the depth bound, take the greedy one.
#ifndef YART_WALK_DP
#define YART_WALK_DP 1
#endif
#ifndef YART_WALK_DP_CL
#define YART_WALK_DP_CL 1.0  // a leaf step's cost against an inner node step's
#endif
constexpr uint32_t kDpMaxTris = 1u << 17;
double wcount(size_t n) { return (double)((n + YART_WALK_LEAF_QUANT - 1) / YART_WALK_LEAF_QUANT); }

struct WalkBuilder {
  BuiltMesh& m;
  std::vector<WItem> items;
  uint32_t n_tris = 0, max_depth = 10, depth = 0, next_rec = 0;
#ifdef YART_WALK_TREE_STATS
  // surface-area sums (study builds, make variant DEFS=-DYART_WALK_TREE_STATS): inner nodes, leaves,
  // leaves x triangles, and the leaf count
  double s_inner = 0.0, s_leaf = 0.0, s_tris = 0.0;
  size_t n_leaves = 0;
#endif
  // SAH bins per axis; the greedy 4-way expansion splits the part of largest area x count next
  // (16 / 32 / 64 bins and count- or area-only picks were within +-2 %; r05: an exact
  // sweep below 64 / 256 triangles and picking by the SAH gain moved the surface-area estimate < 0.5 %)
  static constexpr int kBins = 32;

  // Binned SAH cut of items[b, e) (n >= 2): returns the cut position in (b, e), items partitioned.
  size_t split(size_t b, size_t e) {
    constexpr int kMaxBins = kBins;
    float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (size_t i = b; i < e; ++i)
      for (int k = 0; k < 3; ++k) { cmin[k] = std::min(cmin[k], items[i].c[k]); cmax[k] = std::max(cmax[k], items[i].c[k]); }
    double best = INFINITY;
    int best_axis = -1, best_bin = 0;
    for (int axis = 0; axis < 3; ++axis) {
      const float ext = cmax[axis] - cmin[axis];
      if (!(ext > 0.0f)) continue;
      Box3 bb[kMaxBins];
      size_t cnt[kMaxBins] = {};
      const float scale = kBins / ext;
      for (size_t i = b; i < e; ++i) {
        int k = (int)((items[i].c[axis] - cmin[axis]) * scale);
        k = std::min(std::max(k, 0), kBins - 1);
        bb[k].grow(items[i]);
        cnt[k]++;
      }
      Box3 right[kMaxBins];
      size_t rc[kMaxBins] = {};
      Box3 acc;
      size_t an = 0;
      for (int k = kBins - 1; k > 0; --k) {
        acc.grow(bb[k]);
        an += cnt[k];
        right[k] = acc;
        rc[k] = an;
      }
      Box3 left;
      size_t ln = 0;
      for (int k = 0; k < kBins - 1; ++k) {  // cut after bin k
        left.grow(bb[k]);
        ln += cnt[k];
        if (ln == 0 || rc[k + 1] == 0) continue;
        const double cost = left.area() * wcount(ln) + right[k + 1].area() * wcount(rc[k + 1]);
        if (cost < best) { best = cost; best_axis = axis; best_bin = k; }
      }
    }
    if (best_axis < 0) return b + (e - b) / 2;  // every centroid equal: any cut
    const float scale = kBins / (cmax[best_axis] - cmin[best_axis]);
    const int axis = best_axis, bin = best_bin;
    auto mid = std::partition(items.begin() + (long)b, items.begin() + (long)e, [&](const WItem& t) {
      int k = (int)((t.c[axis] - cmin[axis]) * scale);
      k = std::min(std::max(k, 0), kBins - 1);
      return k <= bin;
    });
    const size_t cut = (size_t)(mid - items.begin());
    return (cut > b && cut < e) ? cut : b + (e - b) / 2;
  }

  // Four parts of items[b, e) by count (median splits along the widest centroid axis): the
  // fallback that keeps the depth within max_depth.
  void quarter(size_t b, size_t e, size_t cut[5]) {
    float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (size_t i = b; i < e; ++i)
      for (int k = 0; k < 3; ++k) { cmin[k] = std::min(cmin[k], items[i].c[k]); cmax[k] = std::max(cmax[k], items[i].c[k]); }
    int axis = 0;
    for (int k = 1; k < 3; ++k)
      if (cmax[k] - cmin[k] > cmax[axis] - cmin[axis]) axis = k;
    const size_t n = e - b;
    for (int q = 0; q <= 4; ++q) cut[q] = b + n * (size_t)q / 4;
    auto less = [axis](const WItem& x, const WItem& y) { return x.c[axis] < y.c[axis] || (x.c[axis] == y.c[axis] && x.tri < y.tri); };
    std::nth_element(items.begin() + (long)b, items.begin() + (long)cut[2], items.begin() + (long)e, less);
    std::nth_element(items.begin() + (long)b, items.begin() + (long)cut[1], items.begin() + (long)cut[2], less);
    std::nth_element(items.begin() + (long)cut[2], items.begin() + (long)cut[3], items.begin() + (long)e, less);
  }

  uint32_t leaf(size_t b, size_t e) {
    const uint32_t first = n_tris + next_rec;  // record index in m.leaves (after the sorted ones)
    for (size_t i = b; i < e; ++i, ++next_rec) {
      const uint32_t t = items[i].tri;
      const float* src = &m.leaves[kTriFloats * (size_t)t];
      float* dst = &m.leaves[kTriFloats * (size_t)(n_tris + next_rec)];
      std::memcpy(dst, src, kTriFloats * sizeof(float));  // v0 v1 v2, reference leaf, lane, sorted index
    }
    return (1u << 31) | ((uint32_t)(e - b) << 27) | first;
  }

#if YART_WALK_DP
  // A binary SAH tree (the same binned cut) down to single triangles, collapsed into the 4-wide tree
  // by dynamic programming over the expected quad steps (surface area per node visit): each inner
  // node takes exactly four subtrees of its binary node, a leaf any subtree of <= 4 triangles, and
  // no path has more than max_depth inner nodes. r05: steps per ray through the root by surface
  // area 17.77 -> 17.16 on david (18.13 -> 17.64 sycee), leaves 2.55 -> 3.08 triangles; same box,
  // bitwise, david +0.9 .. +1.3 %, bunny +0.1 / +0.9 % (profiles/r05_ab_walk_tree_dp.log).
  struct BNode { Box3 box; size_t b, e; int l = -1, r = -1, h = 0; };  // h: binary height below
  std::vector<BNode> bn;
  // memo per (node, remaining inner levels d <= min(h, max_depth)): a 4-wide tree cut from a binary
  // subtree of height h is never deeper than h, so a larger d is the same as d = h
  std::vector<float> c1, dd;
  std::vector<signed char> c1leaf, dj;
  std::vector<size_t> off;  // per node: first memo slot
  int DL = 0;               // max_depth: the levels the root may use
  int clampd(int id, int d) const { return std::min(d, bn[id].h); }
  size_t ix(int id, int d) const { return off[id] + (size_t)d; }
  // (recursion bounded: a node cut off at level 96 with more than 4 triangles has no 4-wide form,
  // so the DP finds no tree and the greedy builder takes over). The top levels' subtrees (disjoint
  // item ranges) build concurrently into their own node lists, appended in preorder: the nodes and
  // their numbering are the serial build's.
  int bbuild(std::vector<BNode>& out, size_t b, size_t e, int level) {
    BNode nd; nd.b = b; nd.e = e;
    const int id = (int)out.size();
    out.push_back(nd);
    if (e - b <= 1 || level >= 96) {
      for (size_t i = b; i < e; ++i) out[id].box.grow(items[i]);
      return id;
    }
    const size_t c = split(b, e);
    int l, r;
    if (e - b >= 16384 && level < 3) {
      std::vector<BNode> lv, rv;
      auto right = std::async(std::launch::async, [&] { bbuild(rv, c, e, level + 1); });
      bbuild(lv, b, c, level + 1);
      right.get();
      l = (int)out.size();
      for (BNode x : lv) { if (x.l >= 0) { x.l += l; x.r += l; } out.push_back(x); }
      r = (int)out.size();
      for (BNode x : rv) { if (x.l >= 0) { x.l += r; x.r += r; } out.push_back(x); }
    } else {
      l = bbuild(out, b, c, level + 1);
      r = bbuild(out, c, e, level + 1);
    }
    BNode& me = out[id];
    me.l = l; me.r = r;
    me.h = 1 + std::max(out[l].h, out[r].h);
    me.box = out[l].box;
    me.box.grow(out[r].box);
    return id;
  }
  float D(int id, int i, int d) {
    d = clampd(id, d);
    float& v = dd[ix(id, d) * 3 + (i - 2)];
    if (v == v) return v;  // memo (NaN = unset)
    const BNode& nd = bn[id];
    v = INFINITY;
    if (nd.l < 0) return v;
    for (int j = 1; j < i; ++j) {
      const float c = (j == 1 ? C1(nd.l, d) : D(nd.l, j, d)) + (i - j == 1 ? C1(nd.r, d) : D(nd.r, i - j, d));
      if (c < v) { v = c; dj[ix(id, d) * 3 + (i - 2)] = (signed char)j; }
    }
    return v;
  }
  float C1(int id, int d) {
    d = clampd(id, d);
    float& v = c1[ix(id, d)];
    if (v == v) return v;
    const BNode& nd = bn[id];
    const size_t n = nd.e - nd.b;
    v = INFINITY;
    if (n <= 4) { v = (float)(nd.box.area() * YART_WALK_DP_CL); c1leaf[ix(id, d)] = 1; }
    if (n >= 4 && nd.l >= 0 && d >= 1) {
      const float c = (float)nd.box.area() + D(id, 4, d - 1);
      if (c < v) { v = c; c1leaf[ix(id, d)] = 0; }
    }
    return v;
  }
  void gather(int id, int i, int d, std::vector<int>& out) {
    if (i == 1) { out.push_back(id); return; }
    d = clampd(id, d);
    const int j = dj[ix(id, d) * 3 + (i - 2)];
    gather(bn[id].l, j, d, out);
    gather(bn[id].r, i - j, d, out);
  }
  uint32_t emit(int id, int d, uint32_t level, Box3& box_out) {
    const BNode& nd = bn[id];
    box_out = nd.box;
    d = clampd(id, d);
    const bool lf = c1leaf[ix(id, d)] != 0;
#ifdef YART_WALK_TREE_STATS
    if (lf) { s_leaf += box_out.area(); s_tris += box_out.area() * (double)(nd.e - nd.b); ++n_leaves; }
    else s_inner += box_out.area();
#endif
    if (lf) return leaf(nd.b, nd.e);
    depth = std::max(depth, level + 1);
    std::vector<int> sub;
    gather(id, 4, d - 1, sub);
    Box3 cb[4];
    uint32_t ch[4];
    for (int q = 0; q < 4; ++q) ch[q] = emit(sub[q], d - 1, level + 1, cb[q]);
    DevNode node{};
    for (int q = 0; q < 4; ++q) {
      node.lo[q][0] = cb[q].lo[0]; node.lo[q][1] = cb[q].hi[0]; node.lo[q][2] = cb[q].lo[1]; node.lo[q][3] = cb[q].hi[1];
      node.hi[q][0] = cb[q].lo[2]; node.hi[q][1] = cb[q].hi[2];
      std::memcpy(&node.hi[q][2], &ch[q], 4);
      const uint32_t zero = 0;
      std::memcpy(&node.hi[q][3], &zero, 4);
    }
    m.nodes.push_back(node);
    return (uint32_t)m.nodes.size() - 1;
  }
  // The tree's root, or false when no tree fits max_depth (nothing emitted then).
  bool build_dp(Box3& root_box, uint32_t& root_out) {
    DL = (int)max_depth;
    const int root = bbuild(bn, 0, items.size(), 0);
    off.resize(bn.size() + 1);
    off[0] = 0;
    for (size_t k = 0; k < bn.size(); ++k) off[k + 1] = off[k] + (size_t)std::min(bn[k].h, DL) + 1;
    c1.assign(off.back(), NAN); dd.assign(off.back() * 3, NAN);
    c1leaf.assign(off.back(), 0); dj.assign(off.back() * 3, 0);
    const bool ok = C1(root, DL) < INFINITY;
    if (ok) root_out = emit(root, DL, 0, root_box);
    std::vector<BNode>().swap(bn);
    std::vector<float>().swap(c1); std::vector<float>().swap(dd);
    std::vector<signed char>().swap(c1leaf); std::vector<signed char>().swap(dj);
    std::vector<size_t>().swap(off);
    return ok;
  }
#endif
  uint32_t build(size_t b, size_t e, uint32_t level, Box3& box_out) {
    const size_t n = e - b;
    box_out = Box3();
    for (size_t i = b; i < e; ++i) box_out.grow(items[i]);
#ifdef YART_WALK_TREE_STATS
    if (n <= 4) { s_leaf += box_out.area(); s_tris += box_out.area() * (double)n; ++n_leaves; }
    else s_inner += box_out.area();
#endif
    if (n <= 4) return leaf(b, e);
    depth = std::max(depth, level + 1);
    size_t cut[5];
    if (level + 1 + min_levels((n + 3) / 4) >= max_depth) {  // no slack left: balanced quarters
      quarter(b, e, cut);
    } else {  // greedy: split the part with the largest area x count until there are four
      struct Part { size_t b, e; double cost; };
      std::vector<Part> parts{{b, e, 0.0}};
      while (parts.size() < 4) {
        int sel = -1;
        double most = -1.0;
        for (int k = 0; k < (int)parts.size(); ++k) {
          if (parts[k].e - parts[k].b < 2) continue;
          Box3 pb;
          for (size_t i = parts[k].b; i < parts[k].e; ++i) pb.grow(items[i]);
          const double cnt = (double)(parts[k].e - parts[k].b);
          const double c = pb.area() * cnt;
          if (c > most) { most = c; sel = k; }
        }
        const size_t pb = parts[sel].b, pe = parts[sel].e, pc = split(pb, pe);
        parts[sel] = {pb, pc, 0.0};
        parts.insert(parts.begin() + sel + 1, Part{pc, pe, 0.0});
      }
      for (int q = 0; q < 4; ++q) cut[q] = parts[q].b;
      cut[4] = e;
    }
    Box3 cb[4];
    uint32_t ch[4];
    for (int q = 0; q < 4; ++q) ch[q] = build(cut[q], cut[q + 1], level + 1, cb[q]);
    DevNode node{};
    for (int q = 0; q < 4; ++q) {  // exact f32 boxes; push ranks unused by the front-to-back walk
      node.lo[q][0] = cb[q].lo[0]; node.lo[q][1] = cb[q].hi[0]; node.lo[q][2] = cb[q].lo[1]; node.lo[q][3] = cb[q].hi[1];
      node.hi[q][0] = cb[q].lo[2]; node.hi[q][1] = cb[q].hi[2];
      std::memcpy(&node.hi[q][2], &ch[q], 4);
      const uint32_t zero = 0;
      std::memcpy(&node.hi[q][3], &zero, 4);
    }
    m.nodes.push_back(node);
    return (uint32_t)m.nodes.size() - 1;
  }
};

}  // namespace

void build_walk_tree(BuiltMesh& m, uint32_t max_depth) {
  const auto t0 = std::chrono::steady_clock::now();
  WalkBuilder w{m};
  w.n_tris = (uint32_t)(m.leaves.size() / kTriFloats);
  w.max_depth = max_depth;
  // The walk tree's records follow the n sorted ones, so a leaf's first record index reaches 2n - 1,
  // and a node id holds it in 27 bits (1<<31 | count<<27 | first): a larger mesh keeps walking the
  // reference tree front to back (past that bound the index ran into the count bits).
  if (2ull * w.n_tris > (1ull << 27)) return;
  w.items.resize(w.n_tris);
  for (uint32_t t = 0; t < w.n_tris; ++t) {
    const float* r = &m.leaves[kTriFloats * (size_t)t];
    WItem& it = w.items[t];
    for (int k = 0; k < 3; ++k) {
      it.lo[k] = std::min(std::min(r[k], r[3 + k]), r[6 + k]);
      it.hi[k] = std::max(std::max(r[k], r[3 + k]), r[6 + k]);
      it.c[k] = 0.5f * (it.lo[k] + it.hi[k]);
    }
    it.tri = t;
  }
  m.leaves.resize(2 * m.leaves.size());
  Box3 root_box;
  uint32_t root = 0;
  bool built = false;
#if YART_WALK_DP
  if (w.n_tris <= kDpMaxTris) built = w.build_dp(root_box, root);
#endif
  if (!built) root = w.build(0, w.n_tris, 0, root_box);
  if (root >> 31) {  // a single leaf (<= 4 triangles): keep walking the reference tree
    m.leaves.resize(m.leaves.size() / 2);
    return;
  }
  m.walk_root = root;
  m.walk_nodes = (uint32_t)m.nodes.size() - m.ref_nodes;
  m.walk_depth = w.depth;
  m.walk_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
#ifdef YART_WALK_TREE_STATS
  // expected visits per ray through the root box, by surface area (no occlusion, no culling)
  const double ar = root_box.area();
  std::fprintf(stderr, "walk-tree n %u nodes %u depth %u inner %.3f leaf %.3f tris %.3f fill %.3f\n", w.n_tris,
               m.walk_nodes, w.depth, w.s_inner / ar, w.s_leaf / ar, w.s_tris / ar, (double)w.n_tris / (double)w.n_leaves);
#endif
}

bool check_walk_tree(const BuiltMesh& m, uint32_t max_depth) {
  if (m.walk_nodes == 0) return false;
  const uint32_t n = (uint32_t)(m.leaves.size() / kTriFloats / 2);
  std::vector<uint8_t> seen(n, 0);
  bool ok = true;
  uint32_t deepest = 0;
  struct Item { uint32_t id, level; float lo[3], hi[3]; };
  std::vector<Item> st{{m.walk_root, 0, {-INFINITY, -INFINITY, -INFINITY}, {INFINITY, INFINITY, INFINITY}}};
  while (!st.empty() && ok) {
    const Item it = st.back();
    st.pop_back();
    if (it.id >> 31) {  // a leaf: its records lie inside the box its parent stores for it
      const uint32_t count = (it.id >> 27) & 0xFu, first = it.id & ((1u << 27) - 1u);
      ok = count >= 1 && count <= 4 && first >= n && first + count <= 2 * n;
      for (uint32_t i = 0; ok && i < count; ++i) {
        const float* r = &m.leaves[kTriFloats * (size_t)(first + i)];
        uint32_t tri;
        std::memcpy(&tri, &r[11], 4);
        ok = tri < n && !seen[tri] && std::memcmp(r, &m.leaves[kTriFloats * (size_t)tri], kTriFloats * sizeof(float)) == 0;
        if (ok) seen[tri] = 1;
        for (int v = 0; ok && v < 3; ++v)
          for (int k = 0; k < 3; ++k) ok = r[3 * v + k] >= it.lo[k] && r[3 * v + k] <= it.hi[k];
      }
      continue;
    }
    ok = it.id >= m.ref_nodes && it.id < m.nodes.size();
    if (!ok) break;
    deepest = std::max(deepest, it.level + 1);
    const DevNode& nd = m.nodes[it.id];
    for (int q = 0; q < 4 && ok; ++q) {
      Item c;
      std::memcpy(&c.id, &nd.hi[q][2], 4);
      c.level = it.level + 1;
      c.lo[0] = nd.lo[q][0]; c.hi[0] = nd.lo[q][1]; c.lo[1] = nd.lo[q][2]; c.hi[1] = nd.lo[q][3];
      c.lo[2] = nd.hi[q][0]; c.hi[2] = nd.hi[q][1];
      for (int k = 0; k < 3; ++k)  // non-empty, and inside its parent's box
        ok = ok && c.lo[k] <= c.hi[k] && c.lo[k] >= it.lo[k] && c.hi[k] <= it.hi[k];
      st.push_back(c);
    }
  }
  for (uint32_t t = 0; ok && t < n; ++t) ok = seen[t] != 0;
  return ok && deepest == m.walk_depth && deepest <= max_depth;
}

}  // namespace yart_dev
