# Patch for tools/build_patched.sh (an experiment, not shipped; DESIGN §3 "drain forks"): during a
# cooperative walk's drain an idle quad takes the top stack entry of a busy quad's ray and the two
# walk it as a pair, exchanging leaf-round candidates through slots at the top of their stacks.
import sys, os
p = sys.argv[1]
d = os.path.dirname(p)
s = open(p).read()

def rep(old, new, cnt=1):
    global s
    assert s.count(old) >= 1, old[:80]
    s = s.replace(old, new, cnt)

# --- state before the walk loop
rep("""  if (ray < n) take();
  if (STATS && lane == 0) st.v[ST_WALKS]++;
  for (;;) {
    const bool has = ray < n;
    if (__ballot(has) == 0) break;""",
"""  if (ray < n) take();
  if (STATS && lane == 0) st.v[ST_WALKS]++;
  // Drain forks: once the pool is exhausted, an idle quad takes the top stack entry of a busy
  // quad's ray and walks that subtree as the ray's second walker. The pair posts its leaf rounds'
  // candidates to exchange slots at the top of each quad's stack region and both keep the pair's
  // best under (t, key); the last of the two to finish writes the ray's post-check word.
  const bool kFork = kPostCheck && M.fork_ok != 0u;
  uint32_t mate = 0xFFu;  // the quad walking this quad's ray with it (0xFF: none)
  uint32_t rnd = 0;       // wave-uniform round number (exchange tags)
  auto xs = [&](uint32_t quad, int k) -> uint32_t& { return qstk[(SLOTS - 1 - k) * 16 + (int)quad]; };
  for (;;) {
    const bool has = ray < n;
    if (__ballot(has) == 0) break;
    rnd++;""")

# --- leaf branch: forked quads post their candidate instead of applying it
rep("""        if (key != 0xFFFFFFFFu) {  // the winning lane keeps its u, v, triangle; the quad keeps t and who
          const uint32_t w = key & 3u;""",
"""        if (kFork && mate != 0xFFu) {
          if (key != 0xFFFFFFFFu && c == (key & 3u)) {  // the winner posts (t, key, triangle, leaf)
            const uint64_t tbits = (uint64_t)__double_as_longlong(t);
            xs(q, 0) = (uint32_t)tbits; xs(q, 1) = (uint32_t)(tbits >> 32);
            xs(q, 2) = key; xs(q, 3) = id; xs(q, 4) = li; xs(q, 5) = (ray << 16) | (rnd & 0xFFFFu);
          }
        } else if (key != 0xFFFFFFFFu) {  // the winning lane keeps its u, v, triangle; the quad keeps t and who
          const uint32_t w = key & 3u;""")

# --- after the branches: the pair's exchange
rep("""      if (!popped) {
        for (;;) {  // front to back: entries whose box begins beyond the bound are dropped""",
"""      if (kFork && mate != 0xFFu) {  // the pair's candidates of this round: both keep the better
        const uint32_t tag = (ray << 16) | (rnd & 0xFFFFu);
        double bt = INFINITY;
        uint32_t bk = 0xFFFFFFFFu, bid = 0u, bli = 0u, from = 0xFFu;
        for (int side = 0; side < 2; ++side) {
          const uint32_t qq = side == 0 ? q : mate;
          if (xs(qq, 5) != tag) continue;
          const double ct = __longlong_as_double((long long)(((uint64_t)xs(qq, 1) << 32) | xs(qq, 0)));
          const uint32_t ck = xs(qq, 2);
          if (ct < bt || (ct == bt && ck < bk)) { bt = ct; bk = ck; bid = xs(qq, 3); bli = xs(qq, 4); from = qq; }
        }
        if (bk != 0xFFFFFFFFu && (bt < tb || bk < bkey)) {
          tb = bt; fnd = true; bleaf = bli; bkey = bk;
          if (from == q && c == (bk & 3u)) {  // the poster writes the ray's record (u, v again)
            const gfloat4p R = leaves + 3 * (size_t)bid;  // the sorted record of the triangle
            const float4 p0 = ld4(R, 0), p1 = ld4(R, 1), p2 = ld4(R, 2);
            CoopRay& s = rays[ray];
            const double ro[3] = {s.o[0], s.o[1], s.o[2]}, rd[3] = {s.d[0], s.d[1], s.d[2]};
            double rt, ru, rv;
            (void)leaf_tri_hit(p0, p1, p2, ro, rd, tmin, s.tmax, rt, ru, rv);
            coop_put_d(&s.c32[0], bt); coop_put_d(&s.c32[2], ru); coop_put_d(&s.c32[4], rv);
            s.inv32[0] = __uint_as_float(bid);
            s.inv32[1] = __uint_as_float(1u);
          }
          const double lim = bt * (1.0 + kF2bMargin), tin = rays[ray].tmax;
          const double teff = lim < tin ? lim : tin;
          teff32 = (float)(teff + teff * 0x1p-20);
          bound = (float)lim;
        }
      }
      if (!popped) {
        for (;;) {  // front to back: entries whose box begins beyond the bound are dropped""")

# --- fin: a forked walker that is not the ray's last leaves the record's words to the last one
rep("""      if (kPostCheck && fin && c == 0)  // the ray's own lane checks W after the walk (below)
        rays[ray].flags = (f2b && fnd) ? (0x80000000u | bleaf) : 0u;""",
"""      bool last = true;
      if (kFork && fin && mate != 0xFFu) {  // the walker count sits in the record's flags word
        uint32_t left = 0u;
        if (c == 0) left = atomicSub(&rays[ray].flags, 1u);
        left = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane & ~3u) << 2), (int)left);
        last = left == 1u;
        mate = 0xFFu;
      }
      if (kPostCheck && fin && last && c == 0)  // the ray's own lane checks W after the walk (below)
        rays[ray].flags = (f2b && fnd) ? (0x80000000u | bleaf) : 0u;""")

rep("""    if (fin && !fnd && c == 0) rays[ray].inv32[1] = 0.0f;  // no hit (a hit's record is already written)
    const uint64_t fm = __ballot(fin && c == 0);
    if (fm) {
      if (fin) {
        ray = next + (uint32_t)__popcll(fm & ((1ull << (4u * q)) - 1ull));
        if (ray < n) take();
      }
      next += (uint32_t)__popcll(fm);
    }
  }""",
"""    if (fin && !fnd && c == 0) rays[ray].inv32[1] = 0.0f;  // no hit (a hit's record is already written)
    const uint64_t fm = __ballot(fin && c == 0);
    if (fm) {
      if (fin) {
        ray = next + (uint32_t)__popcll(fm & ((1ull << (4u * q)) - 1ull));
        if (ray < n) take();
      }
      next += (uint32_t)__popcll(fm);
    }
    if (kFork && next >= n) {  // the pool is exhausted: idle quads fork busy quads' rays
      // a mate that has left this ray (finished, or walking another) no longer counts
      const uint32_t mray = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((mate & 15u) * 4u + c) << 2), (int)ray);
      if (mate != 0xFFu && mray != ray) mate = 0xFFu;
      const bool idle = ray >= n;
      const bool busy = ray < n && f2b && mate == 0xFFu && cursor >= 1;
      uint64_t mi = __ballot(idle && c == 0), mb = __ballot(busy && c == 0);
      if (mi != 0ull && mb != 0ull) {
        uint64_t pairs = 0ull;  // 4 bits per quad: its partner
        uint32_t helpers = 0u, helped = 0u;  // bit q: quad q is a helper / a busy quad that got one
        while (mi != 0ull && mb != 0ull) {  // wave-uniform
          const uint32_t hq = (uint32_t)__builtin_ctzll(mi) >> 2, bq = (uint32_t)__builtin_ctzll(mb) >> 2;
          mi &= mi - 1ull; mb &= mb - 1ull;
          pairs |= ((uint64_t)bq << (4u * hq)) | ((uint64_t)hq << (4u * bq));
          helpers |= 1u << hq; helped |= 1u << bq;
        }
        const uint32_t partner = (uint32_t)(pairs >> (4u * q)) & 15u;
        const bool is_helper = ((helpers >> q) & 1u) != 0u, is_helped = ((helped >> q) & 1u) != 0u;
        // the busy quad gives its top entry away (every lane of the wave takes part in the permutes)
        const int src = (int)((partner * 4u + c) << 2);
        const uint32_t p_ray = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)ray);
        const int p_cursor = __builtin_amdgcn_ds_bpermute(src, cursor);
        const uint32_t tb_lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)__double_as_longlong(tb));
        const uint32_t tb_hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)((uint64_t)__double_as_longlong(tb) >> 32));
        const uint32_t p_bkey = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)bkey);
        const uint32_t p_bleaf = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)bleaf);
        const uint32_t p_fnd = (uint32_t)__builtin_amdgcn_ds_bpermute(src, fnd ? 1 : 0);
        const float p_bound = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(bound)));
        const float p_teff = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(teff32)));
        const uint32_t p_pos = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pos);
        float p_inv[3], p_c0[3], p_c1[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          p_inv[j] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(inv32[j])));
          p_c0[j] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(c32[j][0])));
          p_c1[j] = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(c32[j][1])));
        }
        if (is_helper) {  // the helper: the busy quad's ray from its top entry
          ray = p_ray;
          node = qstk[(p_cursor - 1) * 16 + (int)partner];
          cursor = 0;
          tb = __longlong_as_double((long long)(((uint64_t)tb_hi << 32) | tb_lo));
          bkey = p_bkey; bleaf = p_bleaf; fnd = p_fnd != 0u; bound = p_bound; teff32 = p_teff; pos = p_pos;
#pragma unroll
          for (int j = 0; j < 3; ++j) { inv32[j] = p_inv[j]; c32[j] = vfloat2{p_c0[j], p_c1[j]}; }
          f2b = true;
          mate = partner;
          xs(q, 5) = 0xFFFFFFFFu;
        } else if (is_helped) {  // the busy quad: its top entry is gone, the ray has two walkers
          cursor -= 1;
          mate = partner;
          xs(q, 5) = 0xFFFFFFFFu;
          if (c == 0) rays[ray].flags = 2u;
        }
      }
    }
  }""")
open(p, 'w').write(s)

# --- DevMesh::fork_ok (device_types.h) and its host side (capi.cpp)
pt = os.path.join(d, "device_types.h")
t = open(pt).read()
old = "  float box_lo[4], box_hi[4];\n};"
assert old in t
t = t.replace(old, "  float box_lo[4], box_hi[4];\n  uint32_t fork_ok;           // the front-to-back walk's stack leaves 6 slots free (drain forks)\n  uint32_t pad_[3];\n};", 1)
open(pt, 'w').write(t)
pc = os.path.join(d, "capi.cpp")
t = open(pc).read()
old = "    dm[m].n_leaves = (uint32_t)b.aux.size();\n"
assert old in t
t = t.replace(old, old + "    {\n      const uint32_t dd = b.walk_root != b.ref_nodes - 1 ? b.walk_depth : b.depth;\n      dm[m].fork_ok = 3u * dd + 1u <= (uint32_t)kStackSlots - 6u ? 1u : 0u;\n    }\n", 1)
open(pc, 'w').write(t)
