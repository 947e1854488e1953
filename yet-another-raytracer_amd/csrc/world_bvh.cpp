// world_bvh.cpp — see world_bvh.h.
#include "world_bvh.h"

#include <algorithm>
#include <cmath>
#include <numeric>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

namespace yart_dev {

bool world_bounds(const DevObject& o, double lo[3], double hi[3]) {
  // A medium's hit can land past t_max (hittable.rs:306): the list walk's replace-on-any-hit
  // order matters there, so scenes with media keep the linear walk.
  if (o.n_xf && o.xf_kind[0] == YART_XF_MEDIUM) return false;
  if (o.kind == YART_PRIM_MOVING_SPHERE) return false;  // its box depends on the shutter time
  const double* p = o.p;
  switch (o.kind) {
    case YART_PRIM_SPHERE: {  // sphere.rs:48-86 (a negative radius is the same sphere)
      const double r = std::fabs(p[3]);
      for (int k = 0; k < 3; ++k) { lo[k] = p[k] - r; hi[k] = p[k] + r; }
      break;
    }
    case YART_PRIM_XY_RECT: lo[0] = p[0]; hi[0] = p[1]; lo[1] = p[2]; hi[1] = p[3]; lo[2] = hi[2] = p[4]; break;
    case YART_PRIM_XZ_RECT: lo[0] = p[0]; hi[0] = p[1]; lo[2] = p[2]; hi[2] = p[3]; lo[1] = hi[1] = p[4]; break;
    case YART_PRIM_YZ_RECT: lo[1] = p[0]; hi[1] = p[1]; lo[2] = p[2]; hi[2] = p[3]; lo[0] = hi[0] = p[4]; break;
    case YART_PRIM_BOX:
      for (int k = 0; k < 3; ++k) { lo[k] = std::min(p[k], p[3 + k]); hi[k] = std::max(p[k], p[3 + k]); }
      break;
    case YART_PRIM_TRIANGLE:
      for (int k = 0; k < 3; ++k) {
        lo[k] = std::min({p[k], p[3 + k], p[6 + k]});
        hi[k] = std::max({p[k], p[3 + k], p[6 + k]});
      }
      break;
    default:
      return false;
  }
  for (int l = (int)o.n_xf - 1; l >= 0; --l) {
    if (o.xf_kind[l] == YART_XF_TRANSLATE) {
      for (int k = 0; k < 3; ++k) { lo[k] += o.xf[l][k]; hi[k] += o.xf[l][k]; }
    } else if (o.xf_kind[l] == YART_XF_ROTATE_Y) {  // p.x = c x + s z, p.z = -s x + c z
      const double sn = o.xf[l][0], cs = o.xf[l][1];
      double nlo[3] = {INFINITY, lo[1], INFINITY}, nhi[3] = {-INFINITY, hi[1], -INFINITY};
      for (int c = 0; c < 4; ++c) {
        const double x = (c & 1) ? hi[0] : lo[0], z = (c & 2) ? hi[2] : lo[2];
        const double rx = cs * x + sn * z, rz = -sn * x + cs * z;
        nlo[0] = std::min(nlo[0], rx); nhi[0] = std::max(nhi[0], rx);
        nlo[2] = std::min(nlo[2], rz); nhi[2] = std::max(nhi[2], rz);
      }
      for (int k = 0; k < 3; ++k) { lo[k] = nlo[k]; hi[k] = nhi[k]; }
    }
  }
  for (int k = 0; k < 3; ++k)
    if (!std::isfinite(lo[k]) || !std::isfinite(hi[k])) return false;
  return true;
}

namespace {

struct Item { double lo[3], hi[3], c[3]; uint32_t idx; };

float down(double v) {
  float f = (float)v;
  return (double)f > v ? std::nextafter(f, -INFINITY) : f;
}
float up(double v) {
  float f = (float)v;
  return (double)f < v ? std::nextafter(f, INFINITY) : f;
}

void set_box(DevWorldNode& n, const Item* it, size_t cnt) {
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (size_t i = 0; i < cnt; ++i)
    for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], it[i].lo[k]); hi[k] = std::max(hi[k], it[i].hi[k]); }
  double mag = 0.0;
  for (int k = 0; k < 3; ++k) mag = std::max({mag, std::fabs(lo[k]), std::fabs(hi[k])});
  const double pad = 1e-7 * mag + 1e-30;
  for (int k = 0; k < 3; ++k) { n.bmin[k] = down(lo[k] - pad); n.bmax[k] = up(hi[k] + pad); }
  n.mag = up(mag + pad);
}

double half_area(const double lo[3], const double hi[3]) {
  const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
  return x * y + y * z + z * x;
}

// Surface-area split of items[begin, end): the cut along one axis's centroid order that minimises
// area(L)·|L| + area(R)·|R|, or 0 to make a leaf (at most kMaxLeaf objects, when testing them all
// is cheaper than a node visit plus the children's expected tests). A sphere of the random scene's
// ground (radius 1000) gets a leaf near the root this way instead of widening every box on its
// median-split path, which every ray then visited.
// Per build (YART_WORLD_SAH is read once into the build's own copy: no shared state between
// concurrent yart_scene_create calls).
struct SahParams {
  size_t max_leaf = 4;
  double node_cost = 0.7;  // one DevWorldNode visit (two f32 box tests) vs one primitive test
  size_t median_leaf = 2;  // the median splits' leaf size (larger only to bound a huge list's depth)
};
size_t sah_split(std::vector<Item>& items, size_t begin, size_t end, const double nlo[3], const double nhi[3],
                 const SahParams& prm) {
  const size_t n = end - begin;
  const double parent = half_area(nlo, nhi);
  double best = INFINITY;
  int best_axis = -1;
  size_t best_cut = 0;
  std::vector<double> right(n + 1);
  for (int axis = 0; axis < 3; ++axis) {
    std::sort(items.begin() + begin, items.begin() + end, [axis](const Item& a, const Item& b) {
      return a.c[axis] < b.c[axis] || (a.c[axis] == b.c[axis] && a.idx < b.idx);
    });
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (size_t i = n; i-- > 1;) {  // right[i]: area of items[begin + i, end)
      for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], items[begin + i].lo[k]); hi[k] = std::max(hi[k], items[begin + i].hi[k]); }
      right[i] = half_area(lo, hi);
    }
    for (int k = 0; k < 3; ++k) { lo[k] = INFINITY; hi[k] = -INFINITY; }
    for (size_t i = 1; i < n; ++i) {  // cut before items[begin + i]
      for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], items[begin + i - 1].lo[k]); hi[k] = std::max(hi[k], items[begin + i - 1].hi[k]); }
      const double cost = half_area(lo, hi) * (double)i + right[i] * (double)(n - i);
      if (cost < best) { best = cost; best_axis = axis; best_cut = i; }
    }
  }
  if (best_axis < 0) return 0;
  if (n <= prm.max_leaf && parent > 0.0 && (double)n * parent <= prm.node_cost * parent + best) return 0;
  std::sort(items.begin() + begin, items.begin() + end, [best_axis](const Item& a, const Item& b) {
    return a.c[best_axis] < b.c[best_axis] || (a.c[best_axis] == b.c[best_axis] && a.idx < b.idx);
  });
  return best_cut;
}

void build(std::vector<Item>& items, size_t begin, size_t end, uint32_t node, uint32_t level, BuiltWorld& out,
           bool sah, const SahParams& prm) {
  out.depth = std::max(out.depth, level);
  DevWorldNode& n = out.nodes[node];
  set_box(n, items.data() + begin, end - begin);
  size_t cut = 0;
  // SAH near the root; median splits below level 16 bound the depth (the device walk keeps one
  // stack slot per level, kStackSlots)
  if (sah && level < 16 && end - begin > 1) {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (size_t i = begin; i < end; ++i)
      for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], items[i].lo[k]); hi[k] = std::max(hi[k], items[i].hi[k]); }
    cut = sah_split(items, begin, end, lo, hi, prm);
    if (cut == 0) {  // a leaf
      n.count = (uint32_t)(end - begin);
      n.first = (uint32_t)out.objs.size();
      std::vector<uint32_t> ids;
      for (size_t i = begin; i < end; ++i) ids.push_back(items[i].idx);
      std::sort(ids.begin(), ids.end());
      out.objs.insert(out.objs.end(), ids.begin(), ids.end());
      return;
    }
  }
  if (cut == 0 && end - begin <= prm.median_leaf) {
    n.count = (uint32_t)(end - begin);
    n.first = (uint32_t)out.objs.size();
    std::vector<uint32_t> ids;
    for (size_t i = begin; i < end; ++i) ids.push_back(items[i].idx);
    std::sort(ids.begin(), ids.end());
    out.objs.insert(out.objs.end(), ids.begin(), ids.end());
    return;
  }
  double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (size_t i = begin; i < end; ++i)
    for (int k = 0; k < 3; ++k) { clo[k] = std::min(clo[k], items[i].c[k]); chi[k] = std::max(chi[k], items[i].c[k]); }
  int axis = 0;
  for (int k = 1; k < 3; ++k)
    if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
  size_t mid = begin + cut;
  if (cut == 0) {
    mid = (begin + end) / 2;
    std::nth_element(items.begin() + begin, items.begin() + mid, items.begin() + end, [axis](const Item& a, const Item& b) {
      return a.c[axis] < b.c[axis] || (a.c[axis] == b.c[axis] && a.idx < b.idx);
    });
  }
  const uint32_t left = (uint32_t)out.nodes.size();
  out.nodes.emplace_back();
  out.nodes.emplace_back();
  out.nodes[node].count = 0;
  out.nodes[node].first = left;
  build(items, begin, mid, left, level + 1, out, sah, prm);
  build(items, mid, end, left + 1, level + 1, out, sah, prm);
}

// Collapse the binary tree into the 4-wide tree the device walks (out.nodes4, out.depth4). A 4-wide
// node takes a binary inner node's two children and, while it has fewer than four,
//  * by area (the default): replaces the inner one of largest box area by its own two children —
//    the best-shaped nodes, but a path may advance only one binary level per 4-wide level;
//  * two levels: replaces every inner child by its two children once, so each 4-wide level spans
//    two binary levels and depth4 = ceil(binary depth / 2) (the area rule made a deep
//    binary tree's 4-wide depth exceed the walk's stack, and the scene silently lost its BVH).
// Children keep the binary nodes' boxes (already rounded outward), so every box test is the one
// the binary walk made, and the walk's answer (min t, ties to the later object) is unchanged.
// Returns whether the walk's stack holds the tree: at most three entries per 4-wide level pushed.
bool collapse4(BuiltWorld& out, bool two_level) {
  out.nodes4.clear();
  out.depth4 = 0;
  struct Job { uint32_t bin, slot, level; };
  std::vector<Job> jobs{{0u, 0u, 1u}};
  out.nodes4.emplace_back();
  auto area = [&](uint32_t b) {
    const DevWorldNode& n = out.nodes[b];
    const double x = (double)n.bmax[0] - n.bmin[0], y = (double)n.bmax[1] - n.bmin[1], z = (double)n.bmax[2] - n.bmin[2];
    return x * y + y * z + z * x;
  };
  while (!jobs.empty()) {
    const Job j = jobs.back();
    jobs.pop_back();
    out.depth4 = std::max(out.depth4, j.level);
    if (3 * out.depth4 + 1 > (uint32_t)kStackSlots) return false;
    std::vector<uint32_t> kids{out.nodes[j.bin].first, out.nodes[j.bin].first + 1};
    if (two_level) {
      std::vector<uint32_t> next;
      for (uint32_t b : kids) {
        if (out.nodes[b].count == 0) { next.push_back(out.nodes[b].first); next.push_back(out.nodes[b].first + 1); }
        else next.push_back(b);
      }
      kids.swap(next);
    }
    while (kids.size() < 4) {
      int pick = -1;
      double most = -1.0;
      for (int k = 0; k < (int)kids.size(); ++k)
        if (out.nodes[kids[k]].count == 0 && area(kids[k]) > most) { most = area(kids[k]); pick = k; }
      if (pick < 0 || two_level) break;
      const uint32_t b = kids[pick];
      kids[pick] = out.nodes[b].first;
      kids.insert(kids.begin() + pick + 1, out.nodes[b].first + 1);
    }
    DevWorldNode4 q{};
    for (int k = 0; k < 4; ++k) {
      if (k >= (int)kids.size()) {
        for (int a = 0; a < 3; ++a) { q.bmin[a][k] = INFINITY; q.bmax[a][k] = -INFINITY; }
        q.mag[k] = 0.0f;
        q.handle[k] = kWorld4Empty;
        continue;
      }
      const DevWorldNode& c = out.nodes[kids[k]];
      // grown by the child's share of the walk's margin (mag 2^-12, world_closest_bvh), rounded outward
      const double gm = (double)c.mag * 0x1p-12;
      for (int a = 0; a < 3; ++a) { q.bmin[a][k] = down((double)c.bmin[a] - gm); q.bmax[a][k] = up((double)c.bmax[a] + gm); }
      q.mag[k] = c.mag;
      if (c.count) {
        q.handle[k] = c.pad[1];  // a leaf
      } else {
        const uint32_t slot = (uint32_t)out.nodes4.size();  // an inner node: its own 4-wide node
        if (slot >= kWorldHandleFirstMask) return false;
        out.nodes4.emplace_back();
        q.handle[k] = slot;
        jobs.push_back({kids[k], slot, j.level + 1});
      }
    }
    out.nodes4[j.slot] = q;
  }
  return 3 * out.depth4 + 1 <= (uint32_t)kStackSlots;
}

// The binary tree (SAH near the root, median splits below) and its 4-wide collapse; a tree the walk's
// stack cannot hold is collapsed two levels per node, then rebuilt by median splits with leaves of
// up to 2, 4, 8, 15 objects (depth ~ log2(n / leaf)), before the list walk is the answer.
bool build_world_bvh_with(const std::vector<DevObject>& objs, BuiltWorld& out, bool sah, size_t median_leaf);

// BuiltWorld::plane_dirs. RotateY with (s, c) maps the x-z direction (dx, dz) to (c dx - s dz,
// s dx + c dz): a rotation-scaling by theta = atan2(s, c). So a chain of them (Translate moves no
// direction) zeroes the local x component along phi = pi/2 - sum(theta) and the local z component
// along phi = -sum(theta), mod pi; away from those the computed component is far from 0 (the
// rounding of the chain is ~m 2^-52 |d| against |d| |sin(phi - phi_0)|).
double plane_diamond(double dx, double dz) {  // the device's formula (kernels.hip plane_diamond)
  if (dz < 0.0 || (dz == 0.0 && dx < 0.0)) { dx = -dx; dz = -dz; }
  const double ax = std::fabs(dx);
  return dx >= 0.0 ? dz / (dx + dz) : 1.0 + ax / (ax + dz);
}
std::vector<double> plane_directions(const std::vector<DevObject>& objs) {
  std::vector<double> v;
  for (const DevObject& o : objs) {
    if (o.kind == YART_PRIM_SPHERE || o.kind > YART_PRIM_BOX) continue;  // rects and boxes only
    double theta = 0.0;
    int rot = 0;
    for (uint32_t l = 0; l < o.n_xf; ++l)
      if (o.xf_kind[l] == YART_XF_ROTATE_Y) { theta += std::atan2(o.xf[l][0], o.xf[l][1]); ++rot; }
    if (!rot) continue;  // unrotated: its planes are world planes, caught by the zero-component test
    for (double phi : {M_PI / 2 - theta, -theta}) {
      double sn, cs;
      ::sincos(phi, &sn, &cs);  // (one call: the library imports no separate sin / cos, test_abi.py)
      const double dm = plane_diamond(cs, sn);
      v.push_back(dm);
      if (dm < 4 * kPlaneDirWindow) v.push_back(dm + 2.0);  // the diamond angle wraps at 2 (= pi)
      if (dm > 2.0 - 4 * kPlaneDirWindow) v.push_back(dm - 2.0);
    }
  }
  if (v.empty()) return v;
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  size_t n = 1;
  while (n < v.size() + 1) n <<= 1;  // at least one +inf: the device's search never runs off the end
  v.resize(n, INFINITY);
  return v;
}

}  // namespace

bool build_world_bvh(const std::vector<DevObject>& objs, BuiltWorld& out, bool sah) {
  return build_world_bvh_with(objs, out, sah, 2);
}

namespace {

bool build_world_bvh_with(const std::vector<DevObject>& objs, BuiltWorld& out, bool sah, size_t median_leaf) {
  out = BuiltWorld{};
  if (objs.empty()) return false;
  std::vector<Item> items(objs.size());
  for (size_t i = 0; i < objs.size(); ++i) {
    if (!world_bounds(objs[i], items[i].lo, items[i].hi)) return false;
    for (int k = 0; k < 3; ++k) items[i].c[k] = 0.5 * (items[i].lo[k] + items[i].hi[k]);
    items[i].idx = (uint32_t)i;
  }
  SahParams prm;  // node cost and leaf size from the r02 sweep (profiles/r02g_world_sah_sweep.txt)
  prm.median_leaf = median_leaf;
  out.nodes.reserve(2 * objs.size());
  out.nodes.emplace_back();
  build(items, 0, items.size(), 0, 0, out, sah, prm);
  // Leaves whose objects are all plain spheres (no wrapper) get kWorldLeafSpheres: the walk reads
  // their centre and radius from the compact per-slot records instead of the object records.
  out.sph.assign(4 * out.objs.size(), 0.0);
  for (size_t j = 0; j < out.objs.size(); ++j) {
    const DevObject& o = objs[out.objs[j]];
    if (o.kind == YART_PRIM_SPHERE && o.n_xf == 0)
      for (int k = 0; k < 4; ++k) out.sph[4 * j + k] = o.p[k];
  }
  for (DevWorldNode& n : out.nodes) {
    if (n.count == 0) continue;
    bool all = true;
    for (uint32_t k = 0; k < n.count; ++k) {
      const DevObject& o = objs[out.objs[n.first + k]];
      all = all && o.kind == YART_PRIM_SPHERE && o.n_xf == 0;
    }
    n.pad[0] = all ? kWorldLeafSpheres : 0u;
  }
  // Each leaf's handle (pad[1]): what the walk needs to take the node without reading its record
  // (the parent's child-box test reads the handle with the box, and the stack holds handles).
  for (DevWorldNode& n : out.nodes) {
    if (n.count > kWorldHandleMaxCount || n.first >= kWorldHandleFirstMask) return false;  // the list walk then
    n.pad[1] = (n.count << 28) | ((n.pad[0] & kWorldLeafSpheres) ? (1u << 27) : 0u) | n.first;
  }
  if (out.nodes[0].count != 0) return false;  // a single leaf: the list walk
  out.plane_dirs = plane_directions(objs);
  if (collapse4(out, false) || collapse4(out, true)) return true;
  if (sah) return build_world_bvh_with(objs, out, false, 2);
  if (median_leaf < kWorldHandleMaxCount) return build_world_bvh_with(objs, out, false, std::min<size_t>(2 * median_leaf, kWorldHandleMaxCount));
  return false;
}

}  // namespace

bool check_world4(const std::vector<DevObject>& objs, const BuiltWorld& w, std::string& err) {
  if (w.nodes4.empty()) { err = "no 4-wide nodes"; return false; }
  std::vector<int> seen(objs.size(), 0);
  struct Item { uint32_t node, level; };
  std::vector<Item> todo{{0u, 1u}};
  std::vector<char> visited(w.nodes4.size(), 0);
  uint32_t depth = 0;
  while (!todo.empty()) {
    const Item it = todo.back();
    todo.pop_back();
    if (it.node >= w.nodes4.size() || visited[it.node]) { err = "node reached twice or out of range"; return false; }
    visited[it.node] = 1;
    depth = std::max(depth, it.level);
    const DevWorldNode4& q = w.nodes4[it.node];
    int kids = 0;
    for (int k = 0; k < 4; ++k) {
      const uint32_t h = q.handle[k];
      if (h == kWorld4Empty) {
        for (int a = 0; a < 3; ++a)
          if (!(q.bmin[a][k] == INFINITY && q.bmax[a][k] == -INFINITY)) { err = "empty slot with a box"; return false; }
        continue;
      }
      ++kids;
      const uint32_t count = h >> 28, first = h & (kWorldHandleFirstMask - 1u);
      // everything below the child lies inside the child's box (the boxes the binary walk tested)
      std::vector<uint32_t> below;
      if (count) {
        if ((size_t)first + count > w.objs.size()) { err = "leaf range out of bounds"; return false; }
        for (uint32_t j = 0; j < count; ++j) below.push_back(w.objs[first + j]);
      } else {
        if (h >= w.nodes4.size()) { err = "inner handle out of range"; return false; }
        todo.push_back({h, it.level + 1});
        std::vector<uint32_t> stack{h};
        while (!stack.empty()) {
          const DevWorldNode4& c = w.nodes4[stack.back()];
          stack.pop_back();
          for (int kk = 0; kk < 4; ++kk) {
            const uint32_t hh = c.handle[kk];
            if (hh == kWorld4Empty) continue;
            if (hh >> 28) {
              for (uint32_t j = 0; j < (hh >> 28); ++j) below.push_back(w.objs[(hh & (kWorldHandleFirstMask - 1u)) + j]);
            } else {
              if (hh >= w.nodes4.size()) { err = "inner handle out of range"; return false; }
              stack.push_back(hh);
            }
          }
        }
      }
      for (uint32_t i : below) {
        if (i >= objs.size()) { err = "object index out of range"; return false; }
        double lo[3], hi[3];
        if (!world_bounds(objs[i], lo, hi)) { err = "object without a box in the tree"; return false; }
        for (int a = 0; a < 3; ++a)
          if (!((double)q.bmin[a][k] <= lo[a] && hi[a] <= (double)q.bmax[a][k])) { err = "child box does not hold an object below it"; return false; }
        // what world_closest_bvh's culling margin assumes: the magnitude bounds the child's
        // coordinates, and the stored box holds the objects grown by the child's share, mag 2^-12
        const double gm = (double)q.mag[k] * 0x1p-12;
        for (int a = 0; a < 3; ++a) {
          if (!((double)q.mag[k] >= std::fabs(lo[a]) && (double)q.mag[k] >= std::fabs(hi[a]))) { err = "child magnitude below its coordinates"; return false; }
          if (!((double)q.bmin[a][k] <= lo[a] - gm && hi[a] + gm <= (double)q.bmax[a][k])) { err = "child box not grown by its margin"; return false; }
        }
      }
      if (count) {
        const bool spheres = ((h >> 27) & 1u) != 0;
        for (uint32_t j = 0; j < count; ++j) {
          const DevObject& o = objs[w.objs[first + j]];
          ++seen[w.objs[first + j]];
          if (spheres && !(o.kind == YART_PRIM_SPHERE && o.n_xf == 0)) { err = "sphere leaf holding another kind"; return false; }
        }
      }
    }
    if (kids < 2) { err = "inner node with fewer than two children"; return false; }
  }
  for (size_t i = 0; i < seen.size(); ++i)
    if (seen[i] != 1) { err = "object " + std::to_string(i) + " in " + std::to_string(seen[i]) + " leaves"; return false; }
  if (depth != w.depth4) { err = "depth4 does not match the tree"; return false; }
  if (3 * depth + 1 > (uint32_t)kStackSlots) { err = "deeper than the walk's stack"; return false; }
  return true;
}

}  // namespace yart_dev
