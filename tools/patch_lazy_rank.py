import sys
p=sys.argv[1]; s=open(p).read()
old='''            kk = f2b ? (aux[li].rank[pos] << 4) | (ln << 2) | c : c;
          }
        }
        double t = cand ? tt : INFINITY;
        uint32_t key = cand ? kk : 0xFFFFFFFFu;
        if (STATS && c == 0) { st.v[ST_LEAVES]++; st.v[ST_LEAF_TRIS] += count; }
        quad_min<0xB1>(t, key);  // quad_perm [1,0,3,2]
        quad_min<0x4E>(t, key);  // quad_perm [2,3,0,1]
        if (key != 0xFFFFFFFFu) {  // the winning lane keeps its u, v, triangle; the quad keeps t and who
          const uint32_t w = key & 3u;
          // t == tb only front to back with a best already held: the reference's order decides
          const bool better = t < tb || key < bkey;
          li = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane & ~3u) | w) << 2), (int)li);  // the winner's leaf
          if (better) {
            tb = t; fnd = true; bleaf = li; bkey = key;'''
new='''            kk = f2b ? (ln << 2) | c : c;  // the leaf rank (the high bits) is read only for a tie, below
          }
        }
        double t = cand ? tt : INFINITY;
        uint32_t key = cand ? kk : 0xFFFFFFFFu;
        const double tc = t;
        if (STATS && c == 0) { st.v[ST_LEAVES]++; st.v[ST_LEAF_TRIS] += count; }
        quad_min<0xB1>(t, key);  // quad_perm [1,0,3,2]
        quad_min<0x4E>(t, key);  // quad_perm [2,3,0,1]
        // Equal t's (two lanes of the quad, or the quad's best and the best held) are ordered by the
        // reference leaf's depth-first rank for the ray's octant (LeafAux): read only then, not at
        // every candidate — a dependent global load in every leaf round with a candidate.
        bool tie = false;
        if (f2b && key != 0xFFFFFFFFu) {
          const uint64_t eq = __ballot(cand && tc == t);
          tie = __popcll(eq & (0xFull << (lane & ~3u))) > 1 || (fnd && t == tb);
        }
        uint32_t bfull = bkey;  // the best held, as a full key (valid in a tie)
        if (__ballot(tie) != 0ull) {  // rare; quad-uniform `tie`
          if (tie) {
            t = tc;
            key = cand ? (aux[li].rank[pos] << 4) | kk : 0xFFFFFFFFu;
            quad_min<0xB1>(t, key);
            quad_min<0x4E>(t, key);
            bfull = fnd ? (aux[bleaf].rank[pos] << 4) | bkey : 0xFFFFFFFFu;
          }
        }
        if (key != 0xFFFFFFFFu) {  // the winning lane keeps its u, v, triangle; the quad keeps t and who
          const uint32_t w = key & 3u;
          // t == tb only front to back with a best already held (a tie): the reference's order decides
          const bool better = t < tb || key < bfull;
          li = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane & ~3u) | w) << 2), (int)li);  // the winner's leaf
          if (better) {
            tb = t; fnd = true; bleaf = li; bkey = key & 0xFu;  // lane in leaf << 2 | quad lane'''
assert old in s; s=s.replace(old,new)
open(p,'w').write(s)
