# Patch for tools/build_patched.sh: a measurement build whose work counters also count the cooperative
# walk's rounds with the pool exhausted (into mesh_rewalks) and their idle quad slots (into
# coop_leaf_rounds); read by tools/drain_probe.py. Not a product build.
import sys
p=sys.argv[1]; s=open(p).read()
old="""      if (lane == 0) {
        st.v[ST_ROUNDS]++;
        st.v[ST_LEAF_ROUNDS] += any_leaf ? 1u : 0u;
      }"""
new="""      const uint64_t hm = __ballot(has && c == 0u);
      if (lane == 0) {
        st.v[ST_ROUNDS]++;
        (void)any_leaf;
        if (next >= n) {  // probe: rounds with the pool exhausted, and their idle quad slots
          st.v[ST_REWALK]++;
          st.v[ST_LEAF_ROUNDS] += 16u - (uint32_t)__popcll(hm);
        }
      }"""
assert old in s; s=s.replace(old,new); open(p,'w').write(s)
