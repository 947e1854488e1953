// world_bvh.cpp — see world_bvh.h.
#include "world_bvh.h"

#include <algorithm>
#include <cmath>
#include <numeric>

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

void build(std::vector<Item>& items, size_t begin, size_t end, uint32_t node, uint32_t level, BuiltWorld& out) {
  out.depth = std::max(out.depth, level);
  DevWorldNode& n = out.nodes[node];
  set_box(n, items.data() + begin, end - begin);
  if (end - begin <= 2) {
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
  const size_t mid = (begin + end) / 2;
  std::nth_element(items.begin() + begin, items.begin() + mid, items.begin() + end, [axis](const Item& a, const Item& b) {
    return a.c[axis] < b.c[axis] || (a.c[axis] == b.c[axis] && a.idx < b.idx);
  });
  const uint32_t left = (uint32_t)out.nodes.size();
  out.nodes.emplace_back();
  out.nodes.emplace_back();
  out.nodes[node].count = 0;
  out.nodes[node].first = left;
  build(items, begin, mid, left, level + 1, out);
  build(items, mid, end, left + 1, level + 1, out);
}

}  // namespace

bool build_world_bvh(const std::vector<DevObject>& objs, BuiltWorld& out) {
  out = BuiltWorld{};
  if (objs.empty()) return false;
  std::vector<Item> items(objs.size());
  for (size_t i = 0; i < objs.size(); ++i) {
    if (!world_bounds(objs[i], items[i].lo, items[i].hi)) return false;
    for (int k = 0; k < 3; ++k) items[i].c[k] = 0.5 * (items[i].lo[k] + items[i].hi[k]);
    items[i].idx = (uint32_t)i;
  }
  out.nodes.reserve(2 * objs.size());
  out.nodes.emplace_back();
  build(items, 0, items.size(), 0, 0, out);
  return true;
}

}  // namespace yart_dev
