// bvh_build.cpp — the reference's L4QBVH construction, emitted in the device layout.
#include "bvh_build.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <exception>
#include <map>
#include <thread>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>
#include <new>
#include <system_error>

namespace yart_dev {
namespace {

struct Box {
  double mn[3], mx[3];
};

// Runs tasks[0] on this thread and the others on threads of their own where the system gives one;
// a task whose thread cannot be created (std::system_error) runs here instead, so the result is the
// same either way. An exception inside a task (bad_alloc in a worker) is caught in that task, and
// the first one is rethrown here after every thread has joined — to build_qbvh's handler, so it
// becomes an error code at the C ABI instead of std::terminate.
void run_all(std::vector<std::function<void()>>& tasks) {
  std::vector<std::exception_ptr> err(tasks.size());
  auto guarded = [&tasks, &err](size_t i) {
    try {
      tasks[i]();
    } catch (...) {
      err[i] = std::current_exception();
    }
  };
  std::vector<std::thread> th;
  std::vector<size_t> inline_tasks;
  for (size_t i = 1; i < tasks.size(); ++i) {
    try {
      th.emplace_back(guarded, i);
    } catch (const std::system_error&) {
      inline_tasks.push_back(i);
    }
  }
  if (!tasks.empty()) guarded(0);
  for (size_t i : inline_tasks) guarded(i);
  for (auto& t : th) t.join();
  for (const auto& e : err)
    if (e) std::rethrow_exception(e);
}

// ORDER_TABLE (qbvh.rs:14-16) row for a node's split axes (top | left << 2 | right << 4) and a
// ray octant (x >= 0 | y >= 0 << 1 | z >= 0 << 2): four nibbles, the child pushed k-th in nibble k
// (push_hit_children, qbvh.rs:18-31).
uint32_t push_order(uint32_t axes, uint32_t pos) {
  const uint64_t ORDER_LO = 0x1032102301320123ull, ORDER_HI = 0x3210231032012301ull;
  const uint32_t top = axes & 3u, left = (axes >> 2) & 3u, right = (axes >> 4) & 3u;
  const uint32_t idx = 4u * ((pos >> top) & 1u) + 2u * ((pos >> left) & 1u) + ((pos >> right) & 1u);
  return (uint32_t)(((idx < 4 ? ORDER_LO : ORDER_HI) >> (16u * (idx & 3u))) & 0xFFFFu);
}

// Subtree sizes of the reference's split (qbvh.rs:253-347) depend only on the triangle count:
// n <= 4 is one leaf, otherwise one node over the quarters n/2/2, n/2 - n/2/2, (n - n/2)/2, ...
// The builder uses them to give every subtree its own id ranges up front (post-order nodes,
// leaves in triangle order), so subtrees can be built on different threads into disjoint slots
// and the arrays come out byte-identical to the sequential build.
struct Sizes { uint32_t nodes, leaves; };
struct SizeTable {
  std::map<uint32_t, Sizes> memo;
  Sizes get(uint32_t n) {
    if (n == 0) return {0, 0};
    if (n <= 4) return {0, 1};
    auto it = memo.find(n);
    if (it != memo.end()) return it->second;
    const uint32_t nl = n / 2, nr = n - n / 2;
    const uint32_t q[4] = {nl / 2, nl - nl / 2, nr / 2, nr - nr / 2};
    Sizes s{1, 0};
    for (uint32_t k : q) { const Sizes c = get(k); s.nodes += c.nodes; s.leaves += c.leaves; }
    memo[n] = s;
    return s;
  }
};

struct Builder {
  const float* pos;
  const double* normals;
  std::vector<uint32_t> perm;      // working triangle order (sorted in place by split)
  std::vector<double> key;         // each triangle's centroid on the axis of its last split
  std::vector<double> centroid;    // Hittable::centroid (hittable.rs:12-22), 3 per triangle
  std::vector<Box> tri_box;        // Triangle::bounding_box (triangle.rs:37-62)
  std::map<uint32_t, Sizes> sizes; // SizeTable, filled before any thread starts (read-only after)
  BuiltMesh* out;
  bool ties_desc = false;          // equal keys in descending input order (the tie-order probe)
  uint32_t par_levels = 0;         // levels whose four subtrees are built on their own threads
  uint32_t threads = 1;
  std::atomic<uint32_t> tied_cuts{0}, tied_leaves{0}, depth{0};

  Sizes size_of(uint32_t n) const {
    if (n == 0) return {0, 0};
    if (n <= 4) return {0, 1};
    return sizes.at(n);
  }

  // split (qbvh.rs:637-693): axis of the widest centroid extent (x; y if wider; z if wider than
  // both), sort the range by centroid on it, cut at len/2. Rust's sort_unstable_by leaves equal
  // keys in an unspecified order; this build puts them in input order (ties_desc: reversed) and
  // counts the cuts that fall inside a run of equal keys — where that freedom changes the tree.
  // The range is sorted as (key, index) pairs (contiguous, not an indirect sort); the tie rule
  // makes the order total, so any sorting algorithm — the chunked parallel one for large ranges
  // included — gives the same permutation.
  int split(uint32_t off, uint32_t n) {
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = off; i < off + n; ++i) {
      const double* c = &centroid[3 * (size_t)perm[i]];
      for (int a = 0; a < 3; ++a) { mn[a] = std::fmin(mn[a], c[a]); mx[a] = std::fmax(mx[a], c[a]); }
    }
    int axis = 0;
    if (mx[1] - mn[1] > mx[0] - mn[0]) axis = 1;
    if (mx[2] - mn[2] > std::fmax(mx[1] - mn[1], mx[0] - mn[0])) axis = 2;
    std::vector<std::pair<double, uint32_t>> kv(n);
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t t = perm[off + i];
      key[t] = centroid[3 * (size_t)t + axis];
      kv[i] = {key[t], ties_desc ? ~t : t};  // descending index among equal keys = ascending ~index
    }
    sort_range(kv.begin(), kv.end(), std::less<std::pair<double, uint32_t>>());
    for (uint32_t i = 0; i < n; ++i) perm[off + i] = ties_desc ? ~kv[i].second : kv[i].second;
    if (n >= 2 && kv[n / 2 - 1].first == kv[n / 2].first) tied_cuts++;
    return axis;
  }

  template <class It, class Less>
  void sort_range(It first, It last, Less less) const {
    const size_t n = (size_t)(last - first);
    const uint32_t parts = (uint32_t)std::min<size_t>(threads, n / 32768);
    if (parts < 2) { std::sort(first, last, less); return; }
    std::vector<size_t> cut(parts + 1);
    for (uint32_t p = 0; p <= parts; ++p) cut[p] = n * p / parts;
    std::vector<std::function<void()>> tasks;
    for (uint32_t p = 0; p < parts; ++p) tasks.emplace_back([&, p] { std::sort(first + cut[p], first + cut[p + 1], less); });
    run_all(tasks);
    for (uint32_t w = 1; w < parts; w *= 2) {  // pairwise merges, each round in parallel
      tasks.clear();
      for (uint32_t p = 0; p + w < parts; p += 2 * w) {
        const size_t a = cut[p], m = cut[p + w], b = cut[std::min(p + 2 * w, parts)];
        tasks.emplace_back([=] { std::inplace_merge(first + a, first + m, first + b, less); });
      }
      run_all(tasks);
    }
  }

  static Box merge(const Box& a, const Box& b) {  // surrounding_box (aabb.rs:187-202)
    Box r;
    for (int i = 0; i < 3; ++i) { r.mn[i] = std::fmin(a.mn[i], b.mn[i]); r.mx[i] = std::fmax(a.mx[i], b.mx[i]); }
    return r;
  }

  struct Result { bool has; Box box; uint32_t id; };

  // A leaf is written at its sorted triangle range and its preassigned leaf index `li`.
  Result leaf(uint32_t off, uint32_t n, uint32_t li) {
    Box b = tri_box[perm[off]];
    bool tied = false;
    for (uint32_t i = 1; i < n; ++i) {
      b = merge(b, tri_box[perm[off + i]]);
      tied |= key[perm[off + i - 1]] == key[perm[off + i]];  // lane order rests on a tie
    }
    if (tied) tied_leaves++;
    for (uint32_t i = 0; i < n; ++i) {  // triangle records in sorted order: leaf = [off, off + n)
      const float* v = &pos[9 * (size_t)perm[off + i]];
      float* rec = &out->leaves[kTriFloats * (size_t)(off + i)];
      for (int c = 0; c < 9; ++c) rec[c] = v[c];
      std::memcpy(&rec[9], &li, 4);  // the leaf's index (LeafAux)
      const uint32_t lane = i, tri = off + i;  // lane in the leaf, sorted index (the walk tree's records
      std::memcpy(&rec[10], &lane, 4);        // carry the same three words, kernels.hip qbvh_coop)
      std::memcpy(&rec[11], &tri, 4);
      const double* nn = &normals[9 * (size_t)perm[off + i]];
      for (int c = 0; c < 9; ++c) out->normals[9 * (size_t)(off + i) + c] = nn[c];
    }
    LeafAux& a = out->aux[li];
    for (int k = 0; k < 3; ++k) { a.lo[k] = (float)b.mn[k]; a.hi[k] = (float)b.mx[k]; }  // exact: f32 corners
    return {true, b, (1u << 31) | (n << 27) | off};
  }

  // construct (qbvh.rs:253-347): node ids in post-order from node_base, leaf indices from leaf_base.
  Result construct(uint32_t off, uint32_t n, uint32_t level, uint32_t node_base, uint32_t leaf_base) {
    if (n == 0) return {false, Box{}, 0xFFFFFFFFu};
    if (n <= 4) return leaf(off, n, leaf_base);
    uint32_t d = depth.load();
    while (d < level + 1 && !depth.compare_exchange_weak(d, level + 1)) {}
    uint32_t nl = n / 2, nr = n - n / 2;
    int top = split(off, n);
    int la = split(off, nl);
    int ra = split(off + nl, nr);  // independent of the left quarters' construction (disjoint range)
    const uint32_t qo[4] = {off, off + nl / 2, off + nl, off + nl + nr / 2};
    const uint32_t qn[4] = {nl / 2, nl - nl / 2, nr / 2, nr - nr / 2};
    uint32_t nb[4], lb[4];
    uint32_t nbase = node_base, lbase = leaf_base;
    for (int k = 0; k < 4; ++k) {
      nb[k] = nbase; lb[k] = lbase;
      const Sizes sz = size_of(qn[k]);
      nbase += sz.nodes; lbase += sz.leaves;
    }
    Result ch[4];
    if (level < par_levels) {
      std::vector<std::function<void()>> tasks;
      for (int k = 0; k < 4; ++k) tasks.emplace_back([&, k] { ch[k] = construct(qo[k], qn[k], level + 1, nb[k], lb[k]); });
      run_all(tasks);
    } else {
      for (int k = 0; k < 4; ++k) ch[k] = construct(qo[k], qn[k], level + 1, nb[k], lb[k]);
    }
    DevNode node{};
    const uint32_t axes = (uint32_t)top | ((uint32_t)la << 2) | ((uint32_t)ra << 4);
    for (int k = 0; k < 4; ++k) {
      // QBVHNode::new fills empty lanes with f64::MAX (qbvh.rs:570-572); +inf misses the same way.
      float mn[3], mx[3];
      for (int a = 0; a < 3; ++a) {
        mn[a] = ch[k].has ? (float)ch[k].box.mn[a] : INFINITY;
        mx[a] = ch[k].has ? (float)ch[k].box.mx[a] : INFINITY;
      }
      node.lo[k][0] = mn[0]; node.lo[k][1] = mx[0]; node.lo[k][2] = mn[1]; node.lo[k][3] = mx[1];
      node.hi[k][0] = mn[2]; node.hi[k][1] = mx[2];
      std::memcpy(&node.hi[k][2], &ch[k].id, 4);
      uint32_t code = 0;  // this child's push rank for each of the 8 ray octants, 2 bits each
      for (uint32_t pos = 0; pos < 8; ++pos) {
        const uint32_t enc = push_order(axes, pos);
        for (uint32_t r = 0; r < 4; ++r)
          if (((enc >> (4 * r)) & 0xFu) == (uint32_t)k) code |= r << (2 * pos);
      }
      std::memcpy(&node.hi[k][3], &code, 4);
    }
    const uint32_t id = nbase;  // post-order: after the four subtrees
    out->nodes[id] = node;
    Box lbx = ch[0].has && ch[1].has ? merge(ch[0].box, ch[1].box) : (ch[0].has ? ch[0].box : ch[1].box);
    Box rbx = ch[2].has && ch[3].has ? merge(ch[2].box, ch[3].box) : (ch[2].has ? ch[2].box : ch[3].box);
    return {true, merge(lbx, rbx), id};
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

static bool build_qbvh_impl(uint32_t n, const float* positions, const double* normals, BuiltMesh& out, std::string& err,
                     const QbvhOptions& opt) {
  const auto t0 = std::chrono::steady_clock::now();
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
  b.normals = normals;
  b.out = &out;
  b.ties_desc = opt.ties_desc;
  uint32_t threads = opt.threads ? opt.threads : std::max(1u, std::thread::hardware_concurrency());
  b.par_levels = 0;  // 3^... threads: level L spawns 3 new threads per node, 4^L subtrees below it
  for (uint32_t t = 4; t <= threads && b.par_levels < 4; t *= 4) b.par_levels++;
  b.threads = threads;
  b.perm.resize(n);
  b.key.resize(n);
  b.centroid.resize(3 * (size_t)n);
  b.tri_box.resize(n);
  auto prep = [&](uint32_t lo, uint32_t hi) {
    for (uint32_t t = lo; t < hi; ++t) {
      Box bx;
      for (int a = 0; a < 3; ++a) {
        bx.mn[a] = INFINITY; bx.mx[a] = -INFINITY;
        for (int k = 0; k < 3; ++k) {
          double v = (double)positions[9 * (size_t)t + 3 * k + a];
          bx.mn[a] = std::fmin(bx.mn[a], v);
          bx.mx[a] = std::fmax(bx.mx[a], v);
        }
        b.centroid[3 * (size_t)t + a] = (bx.mx[a] + bx.mn[a]) / 2.0;  // Hittable::centroid (hittable.rs:12-22)
      }
      b.perm[t] = t;
      b.tri_box[t] = bx;
    }
  };
  {
    const uint32_t parts = std::min<uint32_t>(threads, std::max<uint32_t>(1u, n / 16384u));
    std::vector<std::function<void()>> tasks;
    for (uint32_t p = 0; p < parts; ++p)
      tasks.emplace_back([&, p] { prep((uint32_t)((uint64_t)n * p / parts), (uint32_t)((uint64_t)n * (p + 1) / parts)); });
    run_all(tasks);
  }
  SizeTable st;
  const Sizes total = st.get(n);
  b.sizes = std::move(st.memo);
  out.nodes.assign(total.nodes, DevNode{});
  out.aux.assign(total.leaves, LeafAux{});
  out.normals.assign(9 * (size_t)n, 0.0);
  out.leaves.assign(kTriFloats * (size_t)n, 0.0f);
  out.extent = 0.0f;  // max |coordinate| of the mesh (the f32 box test's error scale)
  for (size_t i = 0; i < 9 * (size_t)n; ++i) out.extent = std::max(out.extent, std::fabs(positions[i]));
  b.construct(0, n, 0, 0, 0);
  out.depth = b.depth.load();
  rank_leaves(out, (uint32_t)out.nodes.size() - 1);
  out.tied_cuts = b.tied_cuts.load();
  out.tied_leaves = b.tied_leaves.load();
  out.ref_nodes = (uint32_t)out.nodes.size();
  out.walk_root = out.ref_nodes - 1;
  out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (3 * out.depth + 1 > (uint32_t)kMaxStackSlots) {  // the reference's 64-entry stack overflows too
    err = "QBVH too deep for the 64-entry traversal stack (depth " + std::to_string(out.depth) + ", qbvh.rs:382-384)";
    return false;
  }
  return true;
}

bool build_qbvh(uint32_t n, const float* positions, const double* normals, BuiltMesh& out, std::string& err,
                const QbvhOptions& opt) {
  try {  // nothing may unwind across the C ABI
    return build_qbvh_impl(n, positions, normals, out, err, opt);
  } catch (const std::bad_alloc&) {
    err = "out of host memory building the QBVH";
  } catch (const std::exception& e) {
    err = std::string("QBVH build failed: ") + e.what();
  }
  return false;
}

}  // namespace yart_dev
