# Patch for tools/build_patched.sh (experiment): a per-wave queue of precomputed camera rays for the
# analytic list kernel. When a hand-out round gives lanes jobs of a 64-job group (one sample index
# over the block's 64 pixels) not yet formed, the whole wave forms that group's camera rays (lane k:
# pixel slot k) into LDS; a lane that takes a job reads its ray there instead of running the camera
# block divergently at the top of the iteration.
import sys
p = sys.argv[1]
s = open(p).read()
def rep(old, new):
    global s
    assert s.count(old) == 1, old[:100]
    s = s.replace(old, new, 1)
rep('''  __shared__ uint32_t s_job[JOBL ? 4 * 6 * 64 : JOBL3 ? 4 * 3 * 64 : 1];''',
'''  __shared__ uint32_t s_job[JOBL ? 4 * 6 * 64 : JOBL3 ? 4 * 3 * 64 : 1];
  constexpr bool CQ = DYN && !HAS_MESH && !BVH && !EXT;
  __shared__ double s_cam[CQ ? 4 * 2 * 7 * 64 : 1];''')
rep('''  uint32_t* stk = &s_stack[HAS_MESH ? (wave * kWaveLdsWords + lane) : BVH ? (wave * kStackSlots * 64 + lane) : 0];''',
'''  uint32_t* stk = &s_stack[HAS_MESH ? (wave * kWaveLdsWords + lane) : BVH ? (wave * kStackSlots * 64 + lane) : 0];
  double* const cq = &s_cam[CQ ? wave * 2 * 7 * 64 + lane : 0];
  uint32_t cq_have0 = 0xFFFFFFFFu, cq_have1 = 0xFFFFFFFFu;  // the group each buffer holds (wave-uniform)''')
rep('''          local_blk = u / A.n_chunks; chunk_id = u % A.n_chunks;''',
'''          local_blk = u / A.n_chunks; chunk_id = u % A.n_chunks;
          cq_have0 = 0xFFFFFFFFu; cq_have1 = 0xFFFFFFFFu;''')
rep('''        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const uint32_t avail = n_jobs - next_job;''',
'''        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const uint32_t avail = n_jobs - next_job;
        if (CQ) {  // the groups this round hands out, formed by the whole wave (lane k: slot k)
          const uint32_t given0 = (uint32_t)__popcll(m), cnt = given0 < avail ? given0 : avail;
          const uint32_t g0 = next_job >> 6, g1 = (next_job + cnt - 1u) >> 6;
          for (uint32_t grp = g0; grp <= g1; ++grp) {  // wave-uniform, at most two
            if ((grp & 1u ? cq_have1 : cq_have0) == grp) continue;
            if ((cov >> lane) & 1ull) {
              const uint32_t fx = bx0 + (lane & 7u), fy = by0 + (lane >> 3);
              Rng gf = g;
              rng_phase<true>(gf, fy * W + fx, s_lo + grp, 0u);
              const double tx = (double)fx + gen_f64(gf);
              const double u = tx / (double)(W - 1);
              const double ty = (double)fy + gen_f64(gf);
              const double v = 1.0 - ty / (double)(H - 1);
              const double wl = gen_range(gf, kMinLambda, kMaxLambda);
              const Ray cr = camera_ray(*kernarg_camera(), u, v, wl, gf, false);
              double* e = cq + (grp & 1u) * 7 * 64;
              e[0] = cr.o.x; e[64] = cr.o.y; e[128] = cr.o.z;
              e[192] = cr.d.x; e[256] = cr.d.y; e[320] = cr.d.z; e[384] = wl;
            }
            if (grp & 1u) cq_have1 = grp; else cq_have0 = grp;
          }
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }''')
rep('''          if ((cov >> slot) & 1ull) { fresh = true; need = false; }''',
'''          if ((cov >> slot) & 1ull) {
            fresh = true; need = false;
            if (CQ) {  // the job's camera ray, formed above
              const double* e = cq - lane + ((job >> 6) & 1u) * 7 * 64 + slot;
              ray.o = mk(e[0], e[64], e[128]);
              ray.d = mk(e[192], e[256], e[320]);
              ray.wl = e[384];
              ray.time = kernarg_camera()->time0;
              wbin = spectrum_bin<!HAS_MESH && !EXT>(ray.wl);
              T = 1.0;
              depth = A.max_depth;
            }
          }''')
rep('''      if (fresh) {  // main.rs:692-698
        uint32_t jx = x, jy = y;''', '''      if (CQ && fresh) {  // the ray came with the job
        fresh = false;
      } else if (fresh) {  // main.rs:692-698
        uint32_t jx = x, jy = y;''')
open(p, 'w').write(s)
