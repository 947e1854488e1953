# Experiment (tools/build_patched.sh): the world-BVH walk tests ONE sphere of a leaf per loop
# iteration (the lane stays on the leaf until its spheres are done) instead of the whole leaf in an
# inner loop: an iteration with some lane at a 4-sphere leaf then costs one sphere test, not four.
import sys
p = sys.argv[1]
s = open(p).read()
old = '''  uint32_t hnd = 0u;  // the root: inner node 0
  int cursor = 0;
  for (;;) {'''
new = '''  uint32_t hnd = 0u;  // the root: inner node 0
  int cursor = 0;
  uint32_t kk = 0;  // the next sphere of the current leaf
  for (;;) {'''
assert old in s
s = s.replace(old, new)
old = '''      for (uint32_t k = 0; k < count; ++k) {
        const uint32_t i = S.world_objs[first + k];
        const double* sp = S.world_sph + 4 * (size_t)(first + k);
        if (STATS) st.v[ST_PRIM]++;
        double t;
        if (sphere_t(sp, r, tmin, closest, t) && (!found || t < closest || (i << 3) > who)) {
          closest = t;
          who = i << 3;
          found = true;
        }
      }'''
new = '''      {
        const uint32_t k = kk;
        const uint32_t i = S.world_objs[first + k];
        const double* sp = S.world_sph + 4 * (size_t)(first + k);
        if (STATS) st.v[ST_PRIM]++;
        double t;
        if (sphere_t(sp, r, tmin, closest, t) && (!found || t < closest || (i << 3) > who)) {
          closest = t;
          who = i << 3;
          found = true;
        }
        kk = k + 1u;
        if (kk < count) pop = false;  // the leaf's next sphere in the next iteration
        else kk = 0u;
      }'''
assert old in s
s = s.replace(old, new)
open(p, 'w').write(s)
