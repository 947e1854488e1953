// kernels.hip — gfx950 kernels of the path-tracing hot path.
//
// k_render is a persistent-lane megakernel: one wave64 owns one 8x8 pixel block, one lane owns
// one pixel, and each lane runs its pixel's samples back to back with the sample loop and the
// bounce loop fused into a single `while (alive)` (main.rs:690-708 around ray_reflectance,
// main.rs:537-588, unrolled front to back). A lane whose path ends starts its next sample on the
// next iteration, so the wave stays full until its pixels run out of samples: ray compaction
// without a queue, and per-pixel sums in sample order (bitwise the CPU restatement's).
//
// Arithmetic is IEEE f64 like the reference (built with -ffp-contract=off, so no operation is
// fused); the expression order of every function follows the Rust source it cites. The scene's
// world list is walked with a wave-uniform index (the objects arrive on the scalar path); the
// mesh QBVH is traversed per lane with a 32-slot stack in LDS laid out [slot][lane] so every
// stack access is bank-conflict free.
#include <hip/hip_runtime.h>
#include <math.h>
#include <type_traits>

#include "kernels.h"

namespace yart_dev {

// ------------------------------------------------------------------------ tables / constants
__constant__ double c_cie[471][3] = {  // color.rs:286-1709, rows (x, y, z) per nm from 360
#include "cie_xyz.inc"
};
constexpr double kMinLambda = 360.0, kMaxLambda = 720.0, kBinWidth = 10.0;  // color.rs:7-9
constexpr double kCieYIntegral = 106.856895;                               // color.rs:12
constexpr double kMaxLum = 20.0;                                            // main.rs:59
constexpr double kPi = 3.141592653589793;
constexpr double kEps = 2.220446049250313e-16;                              // f64::EPSILON
constexpr double kF64Max = 1.7976931348623157e308;

// ---------------------------------------------------------------------- Vec3 (vec3.rs)
struct V3 { double x, y, z; };
__device__ __forceinline__ V3 mk(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 muls(V3 a, double s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 smul(double s, V3 a) { return mk(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ double dot(V3 a, V3 b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ double len2(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ double len(V3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
__device__ __forceinline__ V3 unit(V3 a) { double l = len(a); return mk(a.x / l, a.y / l, a.z / l); }  // vec3.rs unit_vector
__device__ __forceinline__ V3 divs(V3 a, double s) {  // vec3.rs:109-122 (0 -> f64::MAX)
  if (s == 0.0) return mk(kF64Max, kF64Max, kF64Max);
  return mk(a.x / s, a.y / s, a.z / s);
}

// ------------------------------------------- exact fast cores for f64 sqrt and division
// hipcc lowers f64 `sqrt` and `/` to IEEE-correct sequences (LLVM AMDGPU):
//   sqrt: x < 2^-767 ? scale by 2^256 : x; v_rsq_f64; 2 Goldschmidt + 2 Newton fma steps; unscale;
//         zero/+inf class fixup                                          (18 VALU instructions)
//   n/d:  v_div_scale_f64 (d); v_rcp_f64; 2 Newton steps; v_div_scale_f64 (n); q = n·r;
//         rem = fma(-d, q, n); v_div_fmas_f64 (= fma(rem, r, q) unless a scale fired);
//         v_div_fixup_f64 (specials, sign)                                (11 VALU instructions)
// Inside the ranges checked below no scale step fires and the fixups pass the value through, so
// the bare cores are bitwise the full sequences. Quotients sharing a positive denominator share its
// reciprocal chain (a unit vector: one v_rcp_f64 chain, not three). n = ±0 (which v_div_scale turns
// into NaN for v_div_fixup to repair) is exact in the core's rem-negated form when d > 0:
// q = ±0·r, remn = d·q − n = +0, fma(−remn, r, q) = q.
__device__ __forceinline__ double sqrt_core(double x) {  // x in [2^-767, inf)
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}
__device__ __forceinline__ double rcp_core(double d) {  // |d| in [2^-300, 2^300]
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(r, e, r);
}
__device__ __forceinline__ double div_core_pos(double n, double d, double r) {  // d > 0, r = rcp_core(d)
  const double q = n * r;
  const double remn = __builtin_fma(d, q, -n);
  return __builtin_fma(-remn, r, q);
}

// Math policies for the blocks that can run either way (scatter, closest hit). Ieee: the
// compiler's sequences. Fast: the cores, every operand checked against its core's range with
// compares only; a failed check sets `bad` and the caller re-runs the whole block with Ieee for
// that lane (one rarely taken branch per block: with one branch per operation the cores lost,
// cornell 4,336 vs 4,436 Msamples/s). Both give the same bits wherever Fast does not flag.
struct PosDen { double d, r; };  // a positive denominator shared by several quotients
struct Ieee {
  static constexpr bool kFast = false;
  __device__ __forceinline__ double sqrt(double x) { return ::sqrt(x); }
  __device__ __forceinline__ double len(V3 a) { return ::sqrt(len2(a)); }
  __device__ __forceinline__ V3 unit(V3 a) { return yart_dev::unit(a); }
  // unit(a) and len(a) (the same sqrt) from one evaluation
  __device__ __forceinline__ V3 unit_len(V3 a, double& l) { l = len(a); return mk(a.x / l, a.y / l, a.z / l); }
  __device__ __forceinline__ PosDen den(double d) { return PosDen{d, 0.0}; }
  __device__ __forceinline__ double quo(double n, const PosDen& p) { return n / p.d; }
};
struct Fast {
  static constexpr bool kFast = true;
  bool bad = false;
  __device__ __forceinline__ double sqrt(double x) {
    bad |= !(x >= 0x1p-767 && x < INFINITY);
    return sqrt_core(x);
  }
  __device__ __forceinline__ double len(V3 a) { return sqrt(len2(a)); }
  __device__ __forceinline__ PosDen den(double d) {  // d in [2^-300, 2^300]
    bad |= !(d >= 0x1p-300 && d <= 0x1p300);
    return PosDen{d, rcp_core(d)};
  }
  // n = 0 or |n| in [2^-600, 2^400] over a checked denominator: no scale, normal quotient,
  // exponent gap < 768
  __device__ __forceinline__ double quo(double n, const PosDen& p) {
    bad |= !(n == 0.0 || (fabs(n) >= 0x1p-600 && fabs(n) <= 0x1p400));
    return div_core_pos(n, p.d, p.r);
  }
  __device__ __forceinline__ V3 unit(V3 a) {
    double l;
    return unit_len(a, l);
  }
  // l = len(a) as well: a checked l in [2^-300, 2^300] has l^2 inside the sqrt core's range, so the
  // len() check passes wherever this one does
  __device__ __forceinline__ V3 unit_len(V3 a, double& l) {
    // |a| in [2^-300, 2^300] (the den check) also covers the sqrt core's range: l2 tiny, zero,
    // infinite or NaN leave l outside it. The components are at most |a|: only the lower bound.
    l = sqrt_core(len2(a));
    bad |= !(l >= 0x1p-300 && l <= 0x1p300);
    bad |= !(a.x == 0.0 || fabs(a.x) >= 0x1p-600);
    bad |= !(a.y == 0.0 || fabs(a.y) >= 0x1p-600);
    bad |= !(a.z == 0.0 || fabs(a.z) >= 0x1p-600);
    const double r = rcp_core(l);
    return mk(div_core_pos(a.x, l, r), div_core_pos(a.y, l, r), div_core_pos(a.z, l, r));
  }
};
__device__ __forceinline__ bool flagged(const Fast& m) { return m.bad; }
__device__ __forceinline__ bool flagged(const Ieee&) { return false; }
// Policy per kernel, bitwise either way (the flagged re-run replays the draws on Ieee). r02
// measurement after the register-liveness work, the Fast policy in every kernel vs Ieee in every
// kernel: cornell (list, no EXT) 4,814 vs 4,716 Msamples/s, random-scene (world BVH) 1,464 vs
// 1,514, david (mesh) 243.4 vs 243.3. So Fast ran where it won, the plain list kernel, and the
// others kept Ieee (the second copy of the block costs them registers). Re-measured in r05 on the
// world-BVH kernel after its walk changes: +0.2..+2.1 % over five same-box runs
// (profiles/r05_ab_bvh_fast_policy_*.log), so the world-BVH kernel runs Fast too. Re-measured in r06 on
// the mesh kernel after its walk changes: david 1920x1080x64 +0.7 %, bunny 800x800x512 +1.3 %, david
// 960x540x16 +1.2 % (profiles/r06k_ab_mesh_fast_policy.log), so every kernel but EXT runs Fast.
template <bool HAS_MESH, bool BVH, bool EXT>
struct MathPolicy {
  typedef typename std::conditional<!EXT, Fast, Ieee>::type type;
};
__device__ __forceinline__ V3 ld3(const double* p) { return mk(p[0], p[1], p[2]); }

struct Ray { V3 o, d; double time, wl; };
__device__ __forceinline__ V3 at(const Ray& r, double t) { return add(r.o, smul(t, r.d)); }

struct Hit { double t; V3 p, n; bool ff; uint32_t mat; double u, v; };  // u, v: EXT kernels only

// ------------------------------------------------- deterministic sin/cos (oracle.c twin)
__device__ __forceinline__ void rem_pio2(double x, int& q, double& y0, double& y1) {
  const double INV_PIO2 = 6.36619772367581382433e-01, PIO2_1 = 1.57079632673412561417e+00,
               PIO2_2 = 6.07710050630396597660e-11, PIO2_2T = 2.02226624879595063154e-21;
  double fn = floor(x * INV_PIO2 + 0.5);
  double t = x - fn * PIO2_1;
  double w = fn * PIO2_2;
  double r = t - w;
  w = fn * PIO2_2T - ((t - r) - w);
  y0 = r - w;
  y1 = (r - y0) - w;
  q = (int)((long long)fn & 3);
}
__device__ __forceinline__ double k_sin(double x, double y) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x, v = z * x;
  double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
__device__ __forceinline__ double k_cos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double z = x * x;
  double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  double hz = 0.5 * z, w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}
__device__ __forceinline__ void sincos_det(double x, double& s, double& c) {
  int q; double y0, y1;
  rem_pio2(x, q, y0, y1);
  double ks = k_sin(y0, y1), kc = k_cos(y0, y1);
  s = (q == 0) ? ks : (q == 1) ? kc : (q == 2) ? -ks : -kc;
  c = (q == 0) ? kc : (q == 1) ? -ks : (q == 2) ? -kc : ks;
}
__device__ __forceinline__ double sin_det(double x) { double s, c; sincos_det(x, s, c); return s; }
__device__ __forceinline__ double powi5(double x) { double x2 = x * x; return x * (x2 * x2); }  // material.rs:210

// Deterministic natural log, bitwise oracle_log (oracle.c): fdlibm's __ieee754_log.
__device__ __forceinline__ double log_det(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
               Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
  uint64_t bits = (uint64_t)__double_as_longlong(x);
  int32_t hx = (int32_t)(bits >> 32);
  const uint32_t lx = (uint32_t)bits;
  int k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -INFINITY;
    if (hx < 0) return NAN;
    k -= 54; x *= two54;
    bits = (uint64_t)__double_as_longlong(x); hx = (int32_t)(bits >> 32);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  int32_t i = (hx + 0x95f64) & 0x100000;
  bits = (uint64_t)__double_as_longlong(x);
  bits = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (bits & 0xffffffffull);
  x = __longlong_as_double((long long)bits);
  k += (i >> 20);
  double f = x - 1.0, dk, R;
  if ((0x000fffff & (2 + hx)) < 3) {
    if (f == 0.0) {
      if (k == 0) return 0.0;
      dk = (double)k;
      return dk * ln2_hi + dk * ln2_lo;
    }
    R = f * f * (0.5 - 0.33333333333333333 * f);
    if (k == 0) return f - R;
    dk = (double)k;
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  const double s = f / (2.0 + f);
  dk = (double)k;
  const double z = s * s;
  i = hx - 0x6147a;
  const double w = z * z;
  const int32_t j = 0x6b851 - hx;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  R = t2 + t1;
  if (i > 0) {
    const double hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// Deterministic acos / atan2 for get_sphere_uv (sphere.rs:213-220), bitwise oracle_acos /
// oracle_atan2 (fdlibm __ieee754_acos, atan, __ieee754_atan2).
__device__ __forceinline__ int32_t hi_word(double x) { return (int32_t)((uint64_t)__double_as_longlong(x) >> 32); }
__device__ __forceinline__ uint32_t lo_word(double x) { return (uint32_t)(uint64_t)__double_as_longlong(x); }
__device__ __noinline__ double acos_det(double x) {
  const double pi = 3.14159265358979311600e+00, pio2_hi = 1.57079632679489655800e+00,
               pio2_lo = 6.12323399573676603587e-17, pS0 = 1.66666666666666657415e-01,
               pS1 = -3.25565818622400915405e-01, pS2 = 2.01212532134862925881e-01,
               pS3 = -4.00555345006794114027e-02, pS4 = 7.91534994289814532176e-04,
               pS5 = 3.47933107596021167570e-05, qS1 = -2.40339491173441421878e+00,
               qS2 = 2.02094576023350569471e+00, qS3 = -6.88283971605453293030e-01,
               qS4 = 7.70381505559019352791e-02;
  const int32_t hx = hi_word(x), ix = hx & 0x7fffffff;
  double z, p, q, r, w, s, c, df;
  if (ix >= 0x3ff00000) {
    if (((ix - 0x3ff00000) | (int32_t)lo_word(x)) == 0) return hx > 0 ? 0.0 : pi + 2.0 * pio2_lo;
    return (x - x) / (x - x);
  }
  if (ix < 0x3fe00000) {
    if (ix <= 0x3c600000) return pio2_hi + pio2_lo;
    z = x * x;
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    r = p / q;
    return pio2_hi - (x - (pio2_lo - x * r));
  } else if (hx < 0) {
    z = (1.0 + x) * 0.5;
    p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    s = sqrt(z);
    r = p / q;
    w = r * s - pio2_lo;
    return pi - 2.0 * (s + w);
  }
  z = (1.0 - x) * 0.5;
  s = sqrt(z);
  df = __longlong_as_double(__double_as_longlong(s) & (long long)0xffffffff00000000ull);
  c = (z - df * df) / (s + df);
  p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  r = p / q;
  w = r * s + c;
  return 2.0 * (df + w);
}
__device__ __forceinline__ double atan_det(double x) {
  const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                            1.57079632679489655800e+00};
  const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                            6.12323399573676603587e-17};
  const double aT[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01, 1.42857142725034663711e-01,
                         -1.11111104054623557880e-01, 9.09088713343650656196e-02, -7.69187620504482999495e-02,
                         6.66107313738753120669e-02, -5.83357013379057348645e-02, 4.97687799461593236017e-02,
                         -3.65315727442169155270e-02, 1.62858201153657823623e-02};
  const int32_t hx = hi_word(x), ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x44100000) {
    if (ix > 0x7ff00000 || (ix == 0x7ff00000 && lo_word(x) != 0)) return x + x;
    return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
  }
  if (ix < 0x3fdc0000) {
    if (ix < 0x3e200000) return x;
    id = -1;
  } else {
    x = fabs(x);
    if (ix < 0x3ff30000) {
      if (ix < 0x3fe60000) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }
      else { id = 1; x = (x - 1.0) / (x + 1.0); }
    } else {
      if (ix < 0x40038000) { id = 2; x = (x - 1.5) / (1.0 + 1.5 * x); }
      else { id = 3; x = -1.0 / x; }
    }
  }
  const double z = x * x, w = z * z;
  const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
  const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
  if (id < 0) return x - x * (s1 + s2);
  const double zz = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
  return hx < 0 ? -zz : zz;
}
__device__ __noinline__ double atan2_det(double y, double x) {
  const double tiny = 1.0e-300, pi_o_4 = 7.8539816339744827900e-01, pi_o_2 = 1.5707963267948965580e+00,
               pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
  const int32_t hx = hi_word(x), ix = hx & 0x7fffffff, hy = hi_word(y), iy = hy & 0x7fffffff;
  const uint32_t lx = lo_word(x), ly = lo_word(y);
  if ((ix | (int32_t)((lx | (0u - lx)) >> 31)) > 0x7ff00000 || (iy | (int32_t)((ly | (0u - ly)) >> 31)) > 0x7ff00000)
    return x + y;
  if (((hx - 0x3ff00000) | (int32_t)lx) == 0) return atan_det(y);
  const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if ((iy | (int32_t)ly) == 0) {
    if (m <= 1) return y;
    return m == 2 ? pi + tiny : -pi - tiny;
  }
  if ((ix | (int32_t)lx) == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7ff00000) {
    if (iy == 0x7ff00000) {
      if (m == 0) return pi_o_4 + tiny;
      if (m == 1) return -pi_o_4 - tiny;
      if (m == 2) return 3.0 * pi_o_4 + tiny;
      return -3.0 * pi_o_4 - tiny;
    }
    if (m == 0) return 0.0;
    if (m == 1) return -0.0;
    return m == 2 ? pi + tiny : -pi - tiny;
  }
  if (iy == 0x7ff00000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  const int k = (iy - ix) >> 20;
  double z;
  if (k > 60) z = pi_o_2 + 0.5 * pi_lo;
  else if (hx < 0 && k < -60) z = 0.0;
  else z = atan_det(fabs(y / x));
  if (m == 0) return z;
  if (m == 1) return -z;
  if (m == 2) return pi - (z - pi_lo);
  return (z - pi_lo) - pi;
}

// ---------------------------------------------------------------- RNG (Philox4x32-10)
// Counter (block, sample, pixel, phase << 2 | stream), key = seed; oracle.c states the stream
// layout (stream 0 path draws, 1 scene construction, 2 ConstantMedium free paths). A path's draws come in phases — phase 0 the camera ray, phase k the scatter at the k-th
// bounce — each starting at block 0, so k_render computes an iteration's first two blocks at
// ONE place for the whole wave (rng_phase) instead of at every draw site any lane reaches with
// an empty buffer. The buffer is consumed by shifting, which in straight-line code is register
// renaming; a draw past the fourth refills in place (rare: rejection loops).
struct Rng { uint32_t k0, k1, c0, c1, c2, c3, b0, b1, b2, b3, b4, b5, b6, b7; int have; };
__device__ __forceinline__ void rng_init(Rng& r, uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t stream) {
  r.k0 = (uint32_t)seed; r.k1 = (uint32_t)(seed >> 32);
  r.c0 = 0; r.c1 = sample; r.c2 = pixel; r.c3 = stream; r.have = 0;
}
__device__ __forceinline__ void philox(const Rng& r, uint32_t blk, uint32_t& o0, uint32_t& o1, uint32_t& o2, uint32_t& o3) {
  uint32_t c0 = blk, c1 = r.c1, c2 = r.c2, c3 = r.c3, k0 = r.k0, k1 = r.k1;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    c0 = hi1 ^ c1 ^ k0; c1 = lo1; c2 = hi0 ^ c3 ^ k1; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  o0 = c0; o1 = c1; o2 = c2; o3 = c3;
}
// Start `phase` of (pixel, sample) with blocks 0 and 1 in the buffer (4 draws).
template <bool LAUNDER>
__device__ __forceinline__ void rng_phase(Rng& r, uint32_t pixel, uint32_t sample, uint32_t phase) {
  r.c1 = sample; r.c2 = pixel; r.c3 = phase << 2;
  if (LAUNDER) {  // the analytic linear-list kernel: +0.5 % there, -2 % on the world-BVH kernel
    // The key is loop-invariant. Hoisted, its 20-word round schedule sat in SGPRs all kernel long and
    // was spilled to VGPR lanes (one v_readlane, a VALU instruction, per round key per iteration).
    // Made opaque here, the schedule is recomputed with scalar adds at each phase start.
    r.k0 = __builtin_amdgcn_readfirstlane(r.k0);  // uniform (the seed); says so where control diverged
    r.k1 = __builtin_amdgcn_readfirstlane(r.k1);
    asm volatile("" : "+s"(r.k0), "+s"(r.k1));
  }
  philox(r, 0u, r.b0, r.b1, r.b2, r.b3);
  philox(r, 1u, r.b4, r.b5, r.b6, r.b7);
  r.c0 = 2; r.have = 4;
}
// Out of line: the refill sites are rare now, and one shared copy keeps the kernel smaller and
// its register allocation looser (+3% on the cornell box over inlining it at ~20 sites).
__device__ __noinline__ uint4 philox_block(uint32_t blk, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
  Rng r; r.c1 = c1; r.c2 = c2; r.c3 = c3; r.k0 = k0; r.k1 = k1;
  uint4 o;
  philox(r, blk, o.x, o.y, o.z, o.w);
  return o;
}
__device__ __forceinline__ uint64_t rng_u64(Rng& r) {
  if (r.have == 0) {
    const uint4 o = philox_block(r.c0, r.c1, r.c2, r.c3, r.k0, r.k1);
    r.b0 = o.x; r.b1 = o.y; r.b2 = o.z; r.b3 = o.w; r.c0++; r.have = 2;
  }
  const uint64_t v = ((uint64_t)r.b1 << 32) | r.b0;
  r.b0 = r.b2; r.b1 = r.b3; r.b2 = r.b4; r.b3 = r.b5; r.b4 = r.b6; r.b5 = r.b7;
  r.have--;
  return v;
}
__device__ __forceinline__ double gen_f64(Rng& r) { return (double)(rng_u64(r) >> 11) * 0x1.0p-53; }

// Where a world query happens; keys ConstantMedium's draw (stream 2): one gen::<f64>() per medium
// and query, counter (object index, sample, pixel, segment << 2 | 2), so the draw does not depend
// on the order objects are tested in.
struct QueryCtx { uint32_t k0, k1, sample, pixel, seg; };
__device__ __forceinline__ double medium_draw(const QueryCtx& q, uint32_t obj) {
  Rng r;
  r.k0 = q.k0; r.k1 = q.k1; r.c1 = q.sample; r.c2 = q.pixel; r.c3 = (q.seg << 2) | 2u;
  uint32_t o0, o1, o2, o3;
  philox(r, obj, o0, o1, o2, o3);
  return (double)(((((uint64_t)o1) << 32) | o0) >> 11) * 0x1.0p-53;
}
__device__ __forceinline__ double gen_range(Rng& r, double low, double high) {  // rand 0.8.5 sample_single
  double scale = high - low;
  for (int guard = 0; guard < 64; ++guard) {
    uint64_t bits = (rng_u64(r) >> 12) | 0x3FF0000000000000ull;
    double res = (__longlong_as_double((long long)bits) - 1.0) * scale + low;
    if (res < high) return res;
    scale = __longlong_as_double(__double_as_longlong(scale) - 1);
  }
  return low;
}
__device__ __forceinline__ uint64_t gen_index(Rng& r, uint64_t n) {  // UniformInt<usize> 0..n
  if (n == 1) return 0;  // the only value; its rejection draws are unobservable (oracle.c)
  uint64_t zone = (n << __clzll(n)) - 1;
  for (int guard = 0; guard < 64; ++guard) {
    uint64_t v = rng_u64(r);
    uint64_t hi = __umul64hi(v, n), lo = v * n;
    if (lo <= zone) return hi;
  }
  return 0;
}

// ----------------------------------------------------------------------------- spectra
// x / d for a constant d through the division core with r = RN(1/d) written out (Markstein: one
// fma correction of RN(x r) is the correctly rounded quotient whenever r is within half an ulp of
// 1/d and x is neither tiny nor huge): the IEEE quotient in 3 VALU instructions instead of 11.
// The constants are made opaque at each use, so they are not hoisted into registers held through
// the render loop. YART_CONST_DIV=0 builds the plain divides.
#ifndef YART_CONST_DIV
#define YART_CONST_DIV 1
#endif
constexpr double kRcpBinWidth = 0x1.999999999999ap-4;  // RN(1 / 10)
constexpr double kRcpPi = 0x1.45f306dc9c883p-2;        // RN(1 / kPi)
__device__ __forceinline__ double div_const(double x, double d, double r) {
  asm volatile("" : "+s"(d), "+s"(r));
  return div_core_pos(x, d, r);
}
// CDIV: the constant-divisor core — in the list and world-BVH kernels without EXT features (cornell
// +0.6 %, random-scene +0.7 % same box, profiles/r06f4_ab_constdiv.log); in the mesh kernels it
// raised the spills (74 -> 112 scratch sites), in the EXT list kernel cornell-box-smoke -0.7 %
template <bool CDIV>
__device__ __forceinline__ int spectrum_bin(double wl) {  // color.rs:276-283
  // wl - 360 is 0 or at least ulp(360) ~ 6e-14 here (wl from gen_range over [360, 720)), inside
  // the core's range
  double f = (CDIV && YART_CONST_DIV) ? div_const(wl - kMinLambda, kBinWidth, kRcpBinWidth) : (wl - kMinLambda) / kBinWidth;
  if (!(f > 0.0)) return 0;
  if (f >= 36.0) return 35;
  return (int)f;
}
__device__ __forceinline__ void cie_xyz(double wl, double& x, double& y, double& z) {  // color.rs:216-228
  double f = wl - kMinLambda;
  if (f != f) f = 0.0;                                             // NaN as isize = 0
  if (!(f > -1.0) || !(f < 471.0)) { x = y = z = 0.0; return; }  // (f as isize) outside 0..471
  int i = (int)f;
  x = c_cie[i][0]; y = c_cie[i][1]; z = c_cie[i][2];
}

// ------------------------------------------------------------------- primitive hits
// Each primitive comes as a closest-hit test that only finds t (`*_t`) and a record builder
// (`*_rec`) run once for the winning primitive of a world query; `*_hit` is the two together.
// Split or not, every value is computed by the same expression on the same inputs.
template <class M = Ieee>
__device__ __forceinline__ bool sphere_t(const double* p, const Ray& r, double tmin, double tmax, double& t, M&& m = M()) {  // sphere.rs:48-86
  V3 center = mk(p[0], p[1], p[2]);
  double radius = p[3];
  V3 oc = sub(r.o, center);
  double a = len2(r.d);
  double half_b = dot(oc, r.d);
  double c = len2(oc) - radius * radius;
  double disc = half_b * half_b - a * c;
  if (disc < 0.0) return false;
  double sq = m.sqrt(disc);
  const PosDen ad = m.den(a);  // a = |d|^2 > 0 for a ray that can hit
  t = m.quo(0.0 - half_b - sq, ad);
  if (t < tmin || tmax < t) {
    t = m.quo(0.0 - half_b + sq, ad);
    if (t < tmin || tmax < t) return false;
  }
  return true;
}
template <bool UV = false, class M = Ieee>
__device__ __forceinline__ void sphere_rec(const double* p, const Ray& r, double t, Hit& h, M&& m = M()) {
  V3 center = mk(p[0], p[1], p[2]);
  double radius = p[3];
  V3 pt = at(r, t);
  V3 outward = sub(pt, center);  // (pt - center) / |radius| (vec3.rs:109-122: / 0 -> f64::MAX)
  if (radius != 0.0) {
    const PosDen rd = m.den(fabs(radius));
    outward = mk(m.quo(outward.x, rd), m.quo(outward.y, rd), m.quo(outward.z, rd));
  } else {
    outward = mk(kF64Max, kF64Max, kF64Max);
  }
  if (radius < 0.0) { h.n = neg(outward); h.ff = dot(r.d, outward) > 0.0; }
  else { h.n = outward; h.ff = dot(r.d, outward) < 0.0; }
  h.t = t; h.p = pt;
  if (UV) {  // get_sphere_uv (sphere.rs:213-220)
    const double theta = acos_det(-outward.y), phi = atan2_det(-outward.z, outward.x) + kPi;
    h.u = phi / (2.0 * kPi);
    h.v = theta / kPi;
  }
}
template <class M = Ieee>
__device__ __forceinline__ bool sphere_hit(const double* p, const Ray& r, double tmin, double tmax, Hit& h, M&& m = M()) {
  double t;
  if (!sphere_t(p, r, tmin, tmax, t, m)) return false;
  sphere_rec<false>(p, r, t, h, m);
  return true;
}

// MovingSphere::hit (sphere.rs:161-199): centre at the ray's time (sphere.rs:153-156), normal
// divided by the signed radius and faced against the ray. p = c0 xyz, c1 xyz, time0, time1, r.
__device__ __forceinline__ V3 moving_center(const double* p, double time) {
  return add(ld3(p), smul((time - p[6]) / (p[7] - p[6]), sub(ld3(p + 3), ld3(p))));
}
__device__ __forceinline__ bool moving_sphere_t(const double* p, const Ray& r, double tmin, double tmax, double& t) {
  const double radius = p[8];
  const V3 oc = sub(r.o, moving_center(p, r.time));
  const double a = len2(r.d), half_b = dot(oc, r.d), c = len2(oc) - radius * radius;
  const double disc = half_b * half_b - a * c;
  if (disc < 0.0) return false;
  const double sq = sqrt(disc);
  t = (0.0 - half_b - sq) / a;
  if (t < tmin || tmax < t) {
    t = (0.0 - half_b + sq) / a;
    if (t < tmin || tmax < t) return false;
  }
  return true;
}
template <bool UV>
__device__ __forceinline__ void moving_sphere_rec(const double* p, const Ray& r, double t, Hit& h) {
  const V3 pt = at(r, t);
  const V3 outward = divs(sub(pt, moving_center(p, r.time)), p[8]);
  if (dot(r.d, outward) < 0.0) { h.n = outward; h.ff = true; }
  else { h.n = neg(outward); h.ff = false; }
  if (UV) {
    const double theta = acos_det(-outward.y), phi = atan2_det(-outward.z, outward.x) + kPi;
    h.u = phi / (2.0 * kPi);
    h.v = theta / kPi;
  }
  h.t = t; h.p = pt;
}

// aarect.rs: A = plane axis, B/C = in-plane axes; p = b0 b1 c0 c1 k.
template <int A, int B, int CC>
__device__ __forceinline__ bool rect_t(const double* p, const Ray& r, double tmin, double tmax, double& t) {
  const double* o = &r.o.x;
  const double* d = &r.d.x;
  const double num = p[4] - o[A], den = d[A];
  t = num / den;
  if (t < tmin || t > tmax) return false;
  double x = o[B] + t * d[B];
  double y = o[CC] + t * d[CC];
  if (x < p[0] || x > p[1] || y < p[2] || y > p[3]) return false;
  return true;
}
// Record of an axis-aligned rect with plane axis `a` (0 yz, 1 xz, 2 xy); a runtime axis lets the
// rect and box-face records of a wave share one code path.
// uv (aarect.rs:52-53): the in-plane coordinates b, c computed as in rect_t, over the bounds.
__device__ __forceinline__ void rect_uv(uint32_t a, const double* bounds, const Ray& r, double t, Hit& h) {
  const double* o = &r.o.x;
  const double* d = &r.d.x;
  const uint32_t B = a == 0 ? 1u : 0u, CC = a == 2 ? 1u : 2u;
  const double x = o[B] + t * d[B], y = o[CC] + t * d[CC];
  h.u = (x - bounds[0]) / (bounds[1] - bounds[0]);
  h.v = (y - bounds[2]) / (bounds[3] - bounds[2]);
}
__device__ __forceinline__ void rect_rec(uint32_t a, const Ray& r, double t, Hit& h) {
  V3 outward = mk(a == 0 ? 1.0 : 0.0, a == 1 ? 1.0 : 0.0, a == 2 ? 1.0 : 0.0);
  h.t = t; h.p = at(r, t);
  if (dot(r.d, outward) < 0.0) { h.n = outward; h.ff = true; }
  else { h.n = neg(outward); h.ff = false; }
}
template <int A, int B, int CC>
__device__ __forceinline__ bool rect_hit(const double* p, const Ray& r, double tmin, double tmax, Hit& h) {
  double t;
  if (!rect_t<A, B, CC>(p, r, tmin, tmax, t)) return false;
  rect_rec(A, r, t, h);
  return true;
}
__device__ __forceinline__ bool xz_hit(const double* p, const Ray& r, double a, double b, Hit& h) { return rect_hit<1, 0, 2>(p, r, a, b, h); }

// Conservative f32 slab pre-test for BoxEntity (not in the reference; exact by construction): a
// face hit's computed point lies within a few f64 ulps of the box, so a ray whose parameter
// range misses the box grown by m = 2^-12 (|box| + |origin|) cannot hit any face, and the six f64
// face tests may be skipped. f32 rounding (~1e-7 relative) stays far inside m; rays with
// non-finite components, or a direction component too small for f32, are never culled.
__device__ __forceinline__ bool box_may_hit(const double* p, const Ray& r, double tmin, double tmax) {
  const float o[3] = {(float)r.o.x, (float)r.o.y, (float)r.o.z};
  const float d[3] = {(float)r.d.x, (float)r.d.y, (float)r.d.z};
  const float chk = o[0] + o[1] + o[2] + d[0] + d[1] + d[2];
  if (!(fabsf(chk) <= 3.0e38f)) return true;  // NaN / inf / near-overflow: do not cull
  // A ray lying exactly in a face's plane (d[a] == 0, o[a] == the face's k) gets t = 0 / 0 = NaN in
  // rect_t, and a NaN t passes its range and bounds tests: the reference "hits" that face wherever
  // the ray runs. Such rays (an exactly zero direction component) are never culled.
  if (r.d.x == 0.0 || r.d.y == 0.0 || r.d.z == 0.0) return true;
  const float bmn[3] = {fminf((float)p[0], (float)p[3]), fminf((float)p[1], (float)p[4]), fminf((float)p[2], (float)p[5])};
  const float bmx[3] = {fmaxf((float)p[0], (float)p[3]), fmaxf((float)p[1], (float)p[4]), fmaxf((float)p[2], (float)p[5])};
  const float B = fmaxf(fmaxf(fmaxf(fabsf(bmn[0]), fabsf(bmn[1])), fmaxf(fabsf(bmn[2]), fabsf(bmx[0]))),
                        fmaxf(fabsf(bmx[1]), fabsf(bmx[2])));
  const float O = fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fabsf(o[2]));
  const float m = (B + O) * 0x1p-12f;
  float lo = (float)tmin, hi = (float)tmax;
  if (fabsf(lo) < INFINITY) lo = lo - fabsf(lo) * 0x1p-10f;  // an infinite bound stays as it is
  if (fabsf(hi) < INFINITY) hi = hi + fabsf(hi) * 0x1p-10f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    // slab unconstrained: a NaN reciprocal, which fmaxf / fminf (maxNum / minNum) ignore
    const float inv = fabsf(d[j]) >= 1.0e-20f ? __builtin_amdgcn_rcpf(d[j]) : __builtin_nanf("");
    const float t0 = (bmn[j] - m - o[j]) * inv, t1 = (bmx[j] + m - o[j]) * inv;
    lo = fmaxf(lo, fminf(t0, t1));
    hi = fminf(hi, fmaxf(t0, t1));
  }
  return lo <= hi;
}

// BoxEntity (box_entity.rs:53-70): its six rects in order, closest first; `face` 0-1 xy, 2-3 xz,
// 4-5 yz, so the face's plane axis is 2 - face / 2.
// CULL: the f32 pre-test first. The list kernels go without it (r06): their wave runs the six face
// tests whenever one lane needs them, so the test was pure cost there — cornell 800x800x256 +2.0 %,
// cornell-box-smoke +6.9 % without it, bitwise. The mesh and world-BVH kernels keep it: without it
// their code came out slower (david -2.4 %, bunny -0.8 %, random-scene -0.6 %; same box,
// profiles/r06z_ab_nocull256.log, r06z_ab_mesh_nocull.log).
template <bool CULL = true>
__device__ __forceinline__ bool box_t(const double* p, const Ray& r, double tmin, double tmax, double& t, uint32_t& face) {
  if (CULL && !box_may_hit(p, r, tmin, tmax)) return false;
  bool found = false;
  double closest = tmax, tt;
  double s[5];
  s[0] = p[0]; s[1] = p[3]; s[2] = p[1]; s[3] = p[4];
  s[4] = p[2]; if (rect_t<2, 0, 1>(s, r, tmin, closest, tt)) { closest = tt; face = 0; found = true; }
  s[4] = p[5]; if (rect_t<2, 0, 1>(s, r, tmin, closest, tt)) { closest = tt; face = 1; found = true; }
  s[2] = p[2]; s[3] = p[5];
  s[4] = p[1]; if (rect_t<1, 0, 2>(s, r, tmin, closest, tt)) { closest = tt; face = 2; found = true; }
  s[4] = p[4]; if (rect_t<1, 0, 2>(s, r, tmin, closest, tt)) { closest = tt; face = 3; found = true; }
  s[0] = p[1]; s[1] = p[4];
  s[4] = p[0]; if (rect_t<0, 1, 2>(s, r, tmin, closest, tt)) { closest = tt; face = 4; found = true; }
  s[4] = p[3]; if (rect_t<0, 1, 2>(s, r, tmin, closest, tt)) { closest = tt; face = 5; found = true; }
  t = closest;
  return found;
}

__device__ __forceinline__ bool triangle_t(const double* p, const Ray& r, double tmin, double tmax, double& t,
                                           double& u, double& v) {  // triangle.rs:48-101
  V3 v0 = ld3(p), v1 = ld3(p + 3), v2 = ld3(p + 6);
  V3 e1 = sub(v1, v0), e2 = sub(v2, v0);
  V3 hh = cross(r.d, e2);
  double a = dot(e1, hh);
  if (a > -kEps && a < kEps) return false;
  double f = 1.0 / a;
  V3 s = sub(r.o, v0);
  u = f * dot(s, hh);
  if (u < 0.0 || u > 1.0) return false;
  V3 q = cross(s, e1);
  v = f * dot(r.d, q);
  if (v < 0.0 || u + v > 1.0) return false;
  t = f * dot(e2, q);
  if (t < tmin || t > tmax) return false;
  return true;
}
// triangle_t's u and v for a triangle it accepted (the same expressions on the same inputs): the
// world pass keeps only t and who won, and the winner's record recomputes these.
__device__ __forceinline__ void triangle_uv(const double* p, const Ray& r, double& u, double& v) {
  V3 v0 = ld3(p), v1 = ld3(p + 3), v2 = ld3(p + 6);
  V3 e1 = sub(v1, v0), e2 = sub(v2, v0);
  V3 hh = cross(r.d, e2);
  double a = dot(e1, hh);
  double f = 1.0 / a;
  V3 s = sub(r.o, v0);
  u = f * dot(s, hh);
  V3 q = cross(s, e1);
  v = f * dot(r.d, q);
}
template <bool UV = false>
__device__ __forceinline__ void triangle_rec(const double* p, const Ray& r, double t, double u, double v, Hit& h) {
  double w = 1.0 - u - v;
  if (UV) {  // triangle.rs:93-94
    h.u = p[18] * w + p[20] * u + p[22] * v;
    h.v = p[19] * w + p[21] * u + p[23] * v;
  }
  V3 outward = add(add(muls(ld3(p + 9), w), muls(ld3(p + 12), u)), muls(ld3(p + 15), v));
  h.t = t; h.p = at(r, t);
  if (dot(r.d, outward) < 0.0) { h.n = outward; h.ff = true; }
  else { h.n = neg(outward); h.ff = false; }
}

// --------------------------------------------- L4QBVH::hit (qbvh.rs:381-543)
constexpr int kNumStats = 25;
struct Stats { unsigned long long v[kNumStats]; };
enum { ST_SAMPLES, ST_SEGMENTS, ST_PRIM, ST_NODES, ST_LEAVES, ST_LEAF_TRIS, ST_LIGHT };  // ST_REWALK = 7 .. 13 below
enum { ST_OVF_PUSHES = 14 };  // deep meshes: walk-stack entries pushed past the LDS slots into the HBM region
// Where a wave's lane-slots go, counted by lane 0 from ballots: the rounds
// of the cooperative walk whose node branch runs and the lanes in it; the lanes testing a triangle in
// the leaf branch and the lanes of the quads at a leaf; the loop's iterations and the lanes starting
// a camera ray or scattering in them (and the iterations where each of those branches runs).
enum { ST_NODE_ROUNDS = 15, ST_NODE_LANES = 16, ST_LEAF_LANES = 17, ST_LEAF_QUAD_LANES = 18, ST_ITERS = 19,
       ST_CAMERA_LANES = 20, ST_SCATTER_LANES = 21, ST_CAMERA_ITERS = 22, ST_SCATTER_ITERS = 23,
       ST_PARKS = 24 };  // walks parked (qbvh_coop PARK), one per quad and stop

// Ray octant: x >= 0 | y >= 0 << 1 | z >= 0 << 2, the ORDER_TABLE column (qbvh.rs:14-31); a
// child's push rank for it is 2 bits of its node record (bvh_build.cpp).
__device__ __forceinline__ uint32_t ray_octant(const double rd[3]) {
  return (rd[0] >= 0.0 ? 1u : 0u) | (rd[1] >= 0.0 ? 2u : 0u) | (rd[2] >= 0.0 ? 4u : 0u);
}
// BLAS records are read through global (address space 1) pointers: a generic pointer makes the
// compiler emit flat loads, which also count against the LDS counter and serialize with the
// traversal stack.
typedef float vfloat4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) vfloat4* gfloat4p;
__device__ __forceinline__ float4 ld4(gfloat4p p, size_t i) {
  const vfloat4 v = p[i];
  return make_float4(v.x, v.y, v.z, v.w);
}
// One child's slab test in f64 on its f32 box (AABB::hit as qbvh.rs:430-470 evaluates it per lane).
__device__ __forceinline__ bool child_hit(float4 lo, float4 hi, const double ro[3], const double inv[3], double tmin,
                                          double tmax) {
  const float bmn[3] = {lo.x, lo.z, hi.x}, bmx[3] = {lo.y, lo.w, hi.y};  // DevNode: (min, max) per axis
  double l = tmin, h = tmax;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double t0 = ((double)bmn[j] - ro[j]) * inv[j], t1 = ((double)bmx[j] - ro[j]) * inv[j];
    l = fmax(l, fmin(t0, t1));
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double t0 = ((double)bmn[j] - ro[j]) * inv[j], t1 = ((double)bmx[j] - ro[j]) * inv[j];
    h = fmin(h, fmax(t0, t1));
  }
  return h > l;
}
// Möller–Trumbore on one leaf record (hitx4's lane, qbvh.rs:475-540): a hit needs t in
// [t_min, t_max) — strict at t_max, so an equal t later in the leaf or tree does not replace.
// A leaf record as the test uses it: v0 and the edges in f64, formed from the f32 vertices. (Records
// holding these f64 values, formed on the host by the same operations — 96 B instead of 48 —
// lost 2-3 % on david in r05: the BLAS no longer fits the L2; profiles/r05_ab_tri64.log.)
struct TriF64 { double v0x, v0y, v0z, e1x, e1y, e1z, e2x, e2y, e2z; };
constexpr int kRecF4 = kTriFloats / 4;  // float4s per triangle record
// Record `i` of a leaf run: its f64 form, and the three words (reference leaf, lane, sorted index).
__device__ __forceinline__ TriF64 tri_load(gfloat4p R, uint32_t& li, uint32_t& lane, uint32_t& sorted) {
  TriF64 g;
  float4 p0 = ld4(R, 0), p1 = ld4(R, 1), p2 = ld4(R, 2);
  // one wait for the whole record (left alone, the compiler splits it into dependent rounds)
  asm volatile("" : "+v"(p0.x), "+v"(p0.y), "+v"(p0.z), "+v"(p0.w), "+v"(p1.x), "+v"(p1.y),
               "+v"(p1.z), "+v"(p1.w), "+v"(p2.x), "+v"(p2.y), "+v"(p2.z), "+v"(p2.w));
  g.v0x = p0.x; g.v0y = p0.y; g.v0z = p0.z;
  g.e1x = (double)p0.w - g.v0x; g.e1y = (double)p1.x - g.v0y; g.e1z = (double)p1.y - g.v0z;
  g.e2x = (double)p1.z - g.v0x; g.e2y = (double)p1.w - g.v0y; g.e2z = (double)p2.x - g.v0z;
  li = __float_as_uint(p2.y); lane = __float_as_uint(p2.z); sorted = __float_as_uint(p2.w);
  return g;
}
__device__ __forceinline__ bool leaf_tri_hit(const TriF64& g, const double ro[3], const double rd[3],
                                             double tmin, double tmax, double& t, double& u, double& v) {
  const double v0x = g.v0x, v0y = g.v0y, v0z = g.v0z;
  const double e1x = g.e1x, e1y = g.e1y, e1z = g.e1z;
  const double e2x = g.e2x, e2y = g.e2y, e2z = g.e2z;
  const double hx = rd[1] * e2z - rd[2] * e2y, hy = rd[2] * e2x - rd[0] * e2z, hz = rd[0] * e2y - rd[1] * e2x;
  const double a = e1x * hx + e1y * hy + e1z * hz;
  const double f = 1.0 / a;
  const double sx = ro[0] - v0x, sy = ro[1] - v0y, sz = ro[2] - v0z;
  u = f * (sx * hx + sy * hy + sz * hz);
  const double qx = sy * e1z - sz * e1y, qy = sz * e1x - sx * e1z, qz = sx * e1y - sy * e1x;
  v = f * (rd[0] * qx + rd[1] * qy + rd[2] * qz);
  t = f * (e2x * qx + e2y * qy + e2z * qz);
  // Short-circuited on purpose: in a leaf round only the lanes of quads at a leaf test triangles,
  // and when all of them fail an early condition the wave skips the rest (branch-free: david -4.5 %).
  return !(a > -kEps && a < kEps) && u >= 0.0 && u <= 1.0 && v >= 0.0 && u + v <= 1.0 && t >= tmin && tmax > t;
}

// Per-lane walk (ConstantMedium boundaries, which hit their mesh from divergent code, and the rare
// re-walk of the cooperative walk's exact check): one lane, one ray, a 32-slot stack in LDS laid
// out [slot][lane]. Out of line, with the ray passed and the hit returned by value (in registers):
// through references, the caller's Ray and hit variables became stack objects, written to scratch
// at every mesh walk of the world pass whether or not the re-walk ran.
struct LaneHit { double t, u, v; uint32_t tri, found; };
// Deep meshes in the megakernel (OVF): the traversal stacks keep their first kStackSlots entries in
// LDS and the rest — up to the reference's 64 (qbvh.rs:382-384) — in a per-wave HBM region
// (RenderArgs::stack_ovf, kOvfWords per resident wave): the per-quad stacks of the cooperative walk
// ([slot - 32][quad] node ids, then their 16-bit entries) and the per-lane stacks of the reference-
// order walk ([slot - 32][lane]). Entries past slot 32 are pushed only by walks deeper than depth 10,
// so the LDS budget — and with it 4 waves per SIMD — is that of every other mesh (kOvf*: kernels.h).
template <bool STATS, bool OVF = false>
__device__ __noinline__ LaneHit qbvh_lane(const DevMesh* __restrict__ Mp, double ox, double oy, double oz, double dx,
                                          double dy, double dz, double tmin, double tmax, uint32_t* __restrict__ stk,
                                          unsigned long long* __restrict__ stv, uint32_t* __restrict__ ovf = nullptr) {
  const DevMesh& M = *Mp;
  const double ro[3] = {ox, oy, oz}, rd[3] = {dx, dy, dz};
  const double inv[3] = {1.0 / rd[0], 1.0 / rd[1], 1.0 / rd[2]};
  const uint32_t pos = ray_octant(rd);
  const gfloat4p nodes = (gfloat4p)M.nodes, leaves = (gfloat4p)M.leaves;
  LaneHit hit{0.0, 0.0, 0.0, 0u, 0u};
  bool found = false;
  int cursor = 0;
  stk[0] = M.root;
  for (;;) {
    uint32_t id;
    if (!OVF || cursor < kStackSlots) id = stk[cursor * 64];
    else id = ovf[(cursor - kStackSlots) * 64];  // OVF: ovf is this lane's column of the wave's lane stacks
    if (id >> 31) {
      const uint32_t count = (id >> 27) & 0xFu, first = id & ((1u << 27) - 1u);
      const gfloat4p L = leaves + kRecF4 * (size_t)first;
      if (STATS) { stv[ST_LEAVES]++; stv[ST_LEAF_TRIS] += count; }
      for (uint32_t i = 0; i < count; ++i) {  // the running t_max: the first of equal hits stays
        double t, u, v;
        uint32_t li, ln, so;
        const TriF64 g = tri_load(L + kRecF4 * i, li, ln, so);
        if (leaf_tri_hit(g, ro, rd, tmin, tmax, t, u, v)) {
          tmax = t;
          hit.t = t; hit.u = u; hit.v = v;
          hit.tri = first + i;
          found = true;
        }
      }
    } else {
      const gfloat4p N = nodes + 8 * (size_t)id;
      if (STATS) stv[ST_NODES]++;
      bool hk[4];
      uint32_t chs[4], rank[4], ordered = 0;  // ordered: bit r = the child of push rank r was hit
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 hi = ld4(N, 4 + k);
        hk[k] = child_hit(ld4(N, k), hi, ro, inv, tmin, tmax);
        chs[k] = __float_as_uint(hi.z);
        rank[k] = (__float_as_uint(hi.w) >> (2u * pos)) & 3u;
        ordered |= (hk[k] ? 1u : 0u) << rank[k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // pushed in rank order: slot = hit children of lower rank
        const int slot = cursor + (int)__popc(ordered & ((1u << rank[k]) - 1u));
        if (hk[k]) {
          if (!OVF || slot < kStackSlots) {
            stk[slot * 64] = chs[k];
          } else {
            ovf[(slot - kStackSlots) * 64] = chs[k];
            if (STATS) stv[ST_OVF_PUSHES]++;
          }
        }
      }
      cursor += (int)__popc(ordered);
    }
    if (cursor == 0) break;
    cursor -= 1;
  }
  hit.found = found ? 1u : 0u;
  return hit;
}
template <bool STATS, bool OVF = false>
__device__ __forceinline__ bool qbvh_t(const DevMesh& M, const Ray& r, double tmin, double tmax, double& t_hit,
                                       uint32_t& tri, double& u_hit, double& v_hit, uint32_t* __restrict__ stk, Stats& st,
                                       uint32_t* __restrict__ ovf = nullptr) {
  // ovf: the wave's overflow region; this lane's column of its lane stacks
  const LaneHit h = qbvh_lane<STATS, OVF>(&M, r.o.x, r.o.y, r.o.z, r.d.x, r.d.y, r.d.z, tmin, tmax, stk, STATS ? st.v : nullptr,
                                          OVF ? ovf + 2 * kOvfQuadWords + __lane_id() : nullptr);
  if (h.found) { t_hit = h.t; u_hit = h.u; v_hit = h.v; tri = h.tri; }
  return h.found != 0u;
}

// Cooperative walk: a quad of lanes (4 consecutive) walks ONE ray, lane k of the quad taking
// child k of an inner node (the QBVH's 4-wide box test, qbvh.rs:430-470, as 4 lanes) or
// triangle k of a leaf (hitx4, qbvh.rs:475-540). The wave's rays are staged in LDS and handed
// to quads as they finish (16 quads, a ballot per round), so the wave's cost is its rays' total
// step count / 16 rather than 64 x its slowest ray. Call from converged code (all 64 lanes);
// `want` selects the lanes that have a ray.
//
// Two visiting orders, one result.
//  * Reference order (qbvh.rs:381-543 as written): children pushed in ORDER_TABLE order, the box
//    test against the running t_max, a leaf hit kept only if strictly nearer. For a positive
//    direction component the table walks far children first, so little is pruned.
//  * Front to back (default when the mesh has LeafAux records): nearest child first, pruned
//    against the best hit so far. Its answer is W = the minimum over the candidate set
//    S = {triangles that pass Möller–Trumbore with t_min <= t < t_max_in, in a leaf whose box passes
//    the slab test at t_max_in} under the order (t, reference depth-first leaf rank, lane). The
//    reference's answer is W too whenever t_W >= l(leaf box of W) (the f64 slab entry the
//    reference computes for it): then every ancestor of W passes its box test at any t_max > t_W
//    (slab entries of nested f32 boxes are monotone: rounding is monotone), so the reference
//    reaches W while its t_max > t_W and keeps it, and every triangle it keeps lies in S, so nothing
//    it meets afterwards is strictly nearer. That condition is re-checked exactly at the end of
//    every front-to-back walk (one 64-B load); a ray that fails it — W's t rounded to before its
//    own box entry — walks again in the reference order. Pruning keeps equal-t candidates (a
//    child is tested against min(t_max_in, t_best (1 + 2^-8)), a popped entry dropped only if its
//    entry exceeds that), so W is always visited unless a triangle's computed t lies more than
//    2^-8 relative before its box's computed entry (a Möller–Trumbore condition number above
//    ~2^44: a ray within ~1e-13 rad of the triangle's plane). Rays with a zero, NaN or infinite
//    direction or origin component, where the monotonicity argument does not hold, walk in the
//    reference order from the start.
// The ray's f32 box-test constants are formed once, when the wave stages its rays (every lane its
// own, in parallel), not in take() by the whole wave each time a quad starts a ray. The f64 1/d
// they come from is formed again where it is needed: the exact final check and the reference
// order. flags: bit 0 front to back allowed, bits 1-3 the ray octant.
struct CoopRay { double o[3], d[3], tmax; float c32[6], inv32[3]; uint32_t flags; };
// Once its walk has started, a ray's f32 constants are in its quad's registers and the record's
// c32 / inv32 words are free: the best hit so far goes there (t, u, v as f64 in c32, the triangle in
// inv32[0], found in inv32[1]), so o and d stay intact and the post-walk check reads its ray back
// from LDS instead of the caller keeping it in registers across the walk.
__device__ __forceinline__ void coop_put_d(float* w, double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  w[0] = __uint_as_float((uint32_t)b);
  w[1] = __uint_as_float((uint32_t)(b >> 32));
}
__device__ __forceinline__ double coop_get_d(const float* w) {
  return __longlong_as_double((long long)(((uint64_t)__float_as_uint(w[1]) << 32) | __float_as_uint(w[0])));
}
typedef uint16_t CoopEnt;  // a stack entry's box entry, the upper half of the f32, rounded down
constexpr int kCoopRayBytes = 64 * (int)sizeof(CoopRay);
// Per-quad stack slots (node id + its box entry, CoopEnt): 32 for meshes of depth <= 10 (3 depth + 1
// entries at most), 64 — the reference's own stack (qbvh.rs:382-384) — for deeper ones, which only
// the wavefront trace kernel walks (k_wf_trace<64>, 3 waves per SIMD for the larger LDS).
constexpr int kCoopSlots = kStackSlots;
constexpr int kDeepSlots = kMaxStackSlots;
template <int SLOTS> constexpr int coop_bytes() { return kCoopRayBytes + SLOTS * 16 * (4 + (int)sizeof(CoopEnt)); }
template <int SLOTS> constexpr int wave_lds_words() {
  return (coop_bytes<SLOTS>() / 4 > kStackSlots * 64) ? coop_bytes<SLOTS>() / 4 : kStackSlots * 64;
}
// LDS per wave: the per-lane stack (qbvh_t, world BVH) or the cooperative walk, never both at once
// The megakernel's also holds the parked walks' queue (a lane per position, u8) and quad words (PARK).
constexpr int kParkBytes = 64 + 16 * 4;
constexpr int kWaveLdsWords = wave_lds_words<kCoopSlots>() + kParkBytes / 4;
constexpr double kF2bMargin = 0x1p-8;
// PARK: a walk parks only in calls that staged at least this many new rays (the wave is still fed)
constexpr uint32_t kParkMinRays = 16u;

template <int CTRL>
__device__ __forceinline__ uint32_t quad_perm(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float quad_perm(float x) {
  return __uint_as_float(quad_perm<CTRL>(__float_as_uint(x)));
}
template <int CTRL>
__device__ __forceinline__ double quad_perm(double x) {
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  const uint64_t lo = quad_perm<CTRL>((uint32_t)b), hi = quad_perm<CTRL>((uint32_t)(b >> 32));
  return __longlong_as_double((long long)(lo | (hi << 32)));
}
// (t, key) lexicographic minimum with the partner lane CTRL names.
template <int CTRL>
__device__ __forceinline__ void quad_min(double& t, uint32_t& key) {
  const double ot = quad_perm<CTRL>(t);
  const uint32_t ok = quad_perm<CTRL>(key);
  const bool other = (ot < t) | ((ot == t) & (ok < key));
  t = other ? ot : t;
  key = other ? ok : key;
}
// One child's slab test as child_hit, also returning its entry l.
__device__ __forceinline__ bool child_hit_l(float4 lo, float4 hi, const double ro[3], const double inv[3], double tmin,
                                            double tmax, double& l) {
  const float bmn[3] = {lo.x, lo.z, hi.x}, bmx[3] = {lo.y, lo.w, hi.y};  // DevNode: (min, max) per axis
  double h = tmax;
  l = tmin;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double t0 = ((double)bmn[j] - ro[j]) * inv[j], t1 = ((double)bmx[j] - ro[j]) * inv[j];
    l = fmax(l, fmin(t0, t1));
    h = fmin(h, fmax(t0, t1));
  }
  return h > l;
}
// Conservative f32 slab test for the front-to-back walk. The ray's constants (take() in
// qbvh_coop): inv32 = (float)(1/d), and per axis c = (-o/d -+ s·delta, -o/d +- s·delta) with
// s = sign(1/d) and delta = 2^-20 (mesh extent + max|o|) |1/d|, so that t0 = fma(min, inv32, c.x) is
// the axis's entry lowered by delta and t1 = fma(max, inv32, c.y) its exit raised by delta
// whatever the sign of d. Every f32 rounding here (inv32, o/d, the fma) is below 2^-24 (extent
// + |o|) |1/d| < delta / 5, so [l, h] contains the reference's f64 interval, and t_min / t_max come
// in rounded outward: whenever the f64 test (h > l) passes, this one (h >= l) passes — it visits a
// superset of nodes, which the front-to-back walk allows (qbvh_coop) — at half the VALU cost of
// f64 arithmetic, two axis bounds per packed fma.
typedef float vfloat2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bool child_hit_f32(float4 lo, float4 hi, const float inv32[3], const vfloat2 c[3],
                                              float tmin32, float tmax32, float& l) {
  const vfloat2 bx = {lo.x, lo.y}, by = {lo.z, lo.w}, bz = {hi.x, hi.y};
  const vfloat2 tx = __builtin_elementwise_fma(bx, (vfloat2)(inv32[0]), c[0]);
  const vfloat2 ty = __builtin_elementwise_fma(by, (vfloat2)(inv32[1]), c[1]);
  const vfloat2 tz = __builtin_elementwise_fma(bz, (vfloat2)(inv32[2]), c[2]);
  l = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fmaxf(fminf(tz.x, tz.y), tmin32));
  const float h = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fminf(fmaxf(tz.x, tz.y), tmax32));
  return h >= l;
}
// Rank of this lane's key among the quad's (ties to the lower lane); +inf keys rank last.
__device__ __forceinline__ uint32_t quad_rank(float key, uint32_t c) {
  const float k1 = quad_perm<0xB1>(key), k2 = quad_perm<0x4E>(key), k3 = quad_perm<0x1B>(key);
  return (uint32_t)((k1 < key) | ((k1 == key) & ((c ^ 1u) < c))) + (uint32_t)((k2 < key) | ((k2 == key) & ((c ^ 2u) < c))) +
         (uint32_t)((k3 < key) | ((k3 == key) & ((c ^ 3u) < c)));
}
// Test hook (yart_debug_force_rewalk): every ray the post-walk check covers walks again in the
// reference's order, so the rare path is exercised on whole frames.
__device__ uint32_t g_force_rewalk;
enum { ST_REWALK = 7, ST_ROUNDS = 8, ST_LEAF_ROUNDS = 9, ST_WALKS = 10, ST_IDLE_SLOTS = 11,  // per wave: lane 0 counts
       ST_WORLD_ITERS = 12, ST_WORLD_LEAF_ITERS = 13 };  // world-BVH walk: wave-level loop iterations (first active lane)
#ifdef YART_WALK_CHECK
// Bounds-checked build of the cooperative walk (tools: make variant DEFS=-DYART_WALK_CHECK): every
// record / node / stack index is checked before use; a violation sets a bit here (1 leaf record
// range, 2 reference leaf index, 4 node index, 8 stack slot) and the access is skipped.
__device__ unsigned int g_walk_fault;
__device__ __forceinline__ void walk_fault(unsigned int bit) { atomicOr(&g_walk_fault, bit); }
#endif
// A ray's walk record (CoopRay) formed by its own lane: the f32 box-test constants, the flags, and
// whether the ray is walked at all (the cull box). A ray whose conservative test misses the
// mesh's cull box (the union of both roots' child boxes) is left out of the walk: every child box
// of either root lies inside that box, the f32 test passes on a box whenever it passes on a box
// inside it (the fma bounds are monotone in the corners) and whenever the reference's f64 test
// passes on it (child_hit_f32), so such a ray has no hit in the reference's walk either, and it
// costs the pool no round.
struct CoopStage { float inv32[3], c32[6]; uint32_t flags; bool walk; };
__device__ __forceinline__ CoopStage coop_stage(const DevMesh& M, bool has_aux, const Ray& r, float tmin32, double tmax) {
  CoopStage s;
  double so[3] = {r.o.x, r.o.y, r.o.z}, sdir[3] = {r.d.x, r.d.y, r.d.z};
  // Opaque here: hoisted out of the world pass's object loop, these constants were spilled at
  // every segment and reloaded at every mesh (5 stack slots); recomputed here they cost a few VALU.
  asm volatile("" : "+v"(sdir[0]), "+v"(sdir[1]), "+v"(sdir[2]));
  const float extent = M.extent;
  double iv[3];
  bool ok = has_aux && extent < 1e15f;
  double O = 0.0;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    iv[j] = 1.0 / sdir[j];
    // front to back needs finite, non-zero direction components (the slab entries of nested
    // boxes are then monotone) and magnitudes the f32 test holds without overflow
    ok = ok && sdir[j] != 0.0 && fabs(so[j]) < 1e15 && fabs(iv[j]) < 1e15;
    O = fmax(O, fabs(so[j]));
  }
  const double m = ((double)extent + O) * 0x1p-20;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double a = -(so[j] * iv[j]), dl = iv[j] > 0.0 ? m * iv[j] : -(m * iv[j]);
    const double sdl = iv[j] > 0.0 ? dl : -dl;
    s.inv32[j] = (float)iv[j];
    s.c32[2 * j] = (float)(a - sdl);
    s.c32[2 * j + 1] = (float)(a + sdl);
  }
  s.flags = (ok ? 1u : 0u) | (ray_octant(sdir) << 1);
  s.walk = true;
  if (ok) {
    const vfloat2 cc[3] = {vfloat2{s.c32[0], s.c32[1]}, vfloat2{s.c32[2], s.c32[3]}, vfloat2{s.c32[4], s.c32[5]}};
    const float4 blo = make_float4(M.box_lo[0], M.box_lo[1], M.box_lo[2], M.box_lo[3]);
    const float4 bhi = make_float4(M.box_hi[0], M.box_hi[1], 0.0f, 0.0f);
    float ent;
    s.walk = child_hit_f32(blo, bhi, s.inv32, cc, tmin32, (float)(tmax + fabs(tmax) * 0x1p-20), ent);
  }
  return s;
}
__device__ __forceinline__ void coop_write(CoopRay& s, const Ray& r, double tmax, const CoopStage& g) {
  s.o[0] = r.o.x; s.o[1] = r.o.y; s.o[2] = r.o.z;
  s.d[0] = r.d.x; s.d[1] = r.d.y; s.d[2] = r.d.z;
  s.tmax = tmax;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    s.inv32[j] = g.inv32[j];
    s.c32[2 * j] = g.c32[2 * j];
    s.c32[2 * j + 1] = g.c32[2 * j + 1];
  }
  s.flags = g.flags;
}
// The exact check of a front-to-back answer (below): W's reference leaf box passes the reference's
// f64 test at t_max and W's t is not before that box's entry.
__device__ __forceinline__ bool coop_check(const __attribute__((address_space(1))) LeafAux* aux, uint32_t leaf, const Ray& r,
                                           double tmin, double tmax, double t) {
  const auto& A = aux[leaf];
  const double ro[3] = {r.o.x, r.o.y, r.o.z}, rd[3] = {r.d.x, r.d.y, r.d.z};
  double l = tmin, h = tmax;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double iv = 1.0 / rd[j];
    const double t0 = ((double)A.lo[j] - ro[j]) * iv, t1 = ((double)A.hi[j] - ro[j]) * iv;
    l = fmax(l, fmin(t0, t1));
    h = fmin(h, fmax(t0, t1));
  }
  return h > l && t >= l;
}
// Inlined: +4 % david, +11 % bunny over a call (the call site spills the caller's state).
template <bool STATS, int SLOTS = kCoopSlots, bool OVF = false, bool PARK = false>
__device__ __forceinline__ void qbvh_coop(const DevMesh& M, bool want, const Ray& r, double tmin, double tmax_in,
                                       bool& found, double& t_hit, uint32_t& tri, double& u_hit, double& v_hit,
                                       uint8_t* __restrict__ lds, Stats& st, uint32_t* __restrict__ ovf = nullptr,
                                       bool resume = false, bool* parked = nullptr, uint32_t park_quads = 0u) {
  found = false;
  if (PARK) *parked = false;
  if (__ballot(want) == 0) return;
  const uint32_t lane = __lane_id();
  CoopRay* rays = reinterpret_cast<CoopRay*>(lds);
  uint32_t* qstk = reinterpret_cast<uint32_t*>(lds + kCoopRayBytes);
  CoopEnt* qent = reinterpret_cast<CoopEnt*>(lds + kCoopRayBytes + SLOTS * 16 * 4);
  // PARK: the queue (position -> the lane whose record it is) and the parked quads' words
  uint8_t* const qtab = lds + coop_bytes<SLOTS>();
  uint32_t* const qsave = reinterpret_cast<uint32_t*>(lds + coop_bytes<SLOTS>() + 64);
  // The mesh's pointers once, in registers: read through M in the loop, they are reloaded each
  // round (M is a generic pointer the LDS stores might alias) — a dependent memory round trip.
  const gfloat4p nodes = (gfloat4p)M.nodes, leaves = (gfloat4p)M.leaves;
  const __attribute__((address_space(1))) LeafAux* aux = (const __attribute__((address_space(1))) LeafAux*)M.aux;
  const uint32_t root = M.root, wroot = M.wroot;  // reference tree / walk tree (front to back)
  // The cull test first (its constants discarded), then the record formed and written in one
  // block, as before the cull: held across the pool's ballot, the constants cost the walk loop
  // registers.
  bool walk = false;
  if (want && !(PARK && resume)) walk = coop_stage(M, aux != nullptr, r, (float)(tmin - fabs(tmin) * 0x1p-20), tmax_in).walk;
  const uint64_t act = __ballot(walk);
  const uint64_t held = PARK ? __ballot(resume) : 0ull;  // lanes whose parked walk goes on here
  if (act == 0 && held == 0) return;
  const uint32_t n = (uint32_t)__popcll(act);
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
  if (walk) {
    // PARK: a lane's record is its own (a parked ray keeps its record across calls), and the queue
    // lists the new rays' lanes in lane order; otherwise the records are the queue
    coop_write(rays[PARK ? lane : rank], r, tmax_in, coop_stage(M, aux != nullptr, r, (float)(tmin - fabs(tmin) * 0x1p-20), tmax_in));
    if (PARK) qtab[rank] = (uint8_t)lane;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const uint32_t q = lane >> 2, c = lane & 3u;
  // the quad's ray: its queue position (< n), or with PARK its record (a lane, kNoRay for none)
  constexpr uint32_t kNoRay = 64u;
  uint32_t ray = q, next = 16;
  // W's exact check after the walk, per lane (the 32-slot walks only: the per-lane re-walk,
  // qbvh_t, has a 32-slot stack; the 64-slot walks check W where the ray's walk ends)
  constexpr bool kPostCheck = SLOTS == kCoopSlots;
  // The best hit so far is written to the ray's LDS record by the lane that found it (the
  // record's inputs are in registers from take() on), so the walk keeps only its t in registers.
  // The walked ray (o, d, t_max) stays in its LDS record and is read where the f64 arithmetic
  // needs it — the leaf test, the exact checks, the reference order — not held in 14 VGPRs
  // through every round of the walk.
  double tb = 0.0;
  const float tmin32 = (float)(tmin - fabs(tmin) * 0x1p-20);
  float inv32[3], teff32 = 0.0f;  // front to back: the f32 box test (child_hit_f32)
  vfloat2 c32[3];
  float bound = INFINITY;  // front to back: a popped entry beyond this is dropped
  uint32_t pos = 0, node = 0, bleaf = 0, bkey = 0;
  int cursor = 0;
  bool fnd = false, f2b = false;
  auto restart = [&](bool front_to_back) {
    node = front_to_back ? wroot : root;
    bkey = 0xFFFFFFFFu;
    cursor = 0;
    fnd = false;
    const double tin = rays[ray].tmax;
    tb = tin;  // best so far (reference order: the running t_max, which child boxes are tested against)
    teff32 = (float)(tin + fabs(tin) * 0x1p-20);  // front to back: the f32 t_max of the child tests
    bound = INFINITY;
    f2b = front_to_back;
  };
  auto take = [&]() {
    const CoopRay& s = rays[ray];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      inv32[j] = s.inv32[j];
      c32[j] = vfloat2{s.c32[2 * j], s.c32[2 * j + 1]};
    }
    const uint32_t fl = s.flags;
    pos = fl >> 1;
    restart((fl & 1u) != 0u);
  };
  // PARK: a quad that ran out of rays while few others still walk does not wait for them. The walk
  // stops and the busy quads park: the next node goes back on the quad's stack (entry 0, never
  // dropped), the best hit's leaf, key and found flag into the ray's record (its t, u, v are there
  // already), the stack depth and the ray into the quad's word. The lane renders on with its other
  // lanes and calls again with `resume`; the same quad picks the walk up where it stopped. Every
  // value the walk carries is restored as it was (the f32 constants are formed again from the
  // record, as at staging), so each quad takes the same steps in the same order: the same answer.
  auto park = [&]() {
    if (STATS && c == 0u) st.v[ST_PARKS]++;
    if (c == 0u) {
      const int slot = cursor * 16 + (int)q;
      qstk[slot] = node;
      qent[slot] = (CoopEnt)0;
      CoopRay& s = rays[ray];
      s.flags = 0x40000000u | bleaf;  // bits 31-30 = 01: parked (a finished walk writes 1x or 00)
      s.inv32[1] = __uint_as_float(fnd ? 1u : 0u);
      s.inv32[2] = __uint_as_float(bkey);
      qsave[q] = 0x80000000u | (ray << 8) | (uint32_t)(cursor + 1);
    }
  };
  auto unpark = [&](uint32_t depth) {
    const CoopRay& s = rays[ray];
    Ray wr;
    wr.o = mk(s.o[0], s.o[1], s.o[2]);
    wr.d = mk(s.d[0], s.d[1], s.d[2]);
    wr.time = 0.0; wr.wl = 0.0;
    const double tin = s.tmax;
    const CoopStage g = coop_stage(M, aux != nullptr, wr, tmin32, tin);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      inv32[j] = g.inv32[j];
      c32[j] = vfloat2{g.c32[2 * j], g.c32[2 * j + 1]};
    }
    pos = g.flags >> 1;
    f2b = (g.flags & 1u) != 0u;
    bleaf = s.flags & 0x3FFFFFFFu;
    fnd = __float_as_uint(s.inv32[1]) != 0u;
    bkey = __float_as_uint(s.inv32[2]);
    tb = fnd ? coop_get_d(&s.c32[0]) : tin;
    if (f2b && fnd) {  // as the leaf step set them at the best hit
      const double lim = tb * (1.0 + kF2bMargin);
      const double teff = lim < tin ? lim : tin;
      teff32 = (float)(teff + teff * 0x1p-20);
      bound = (float)lim;
    } else {  // as restart() set them
      teff32 = (float)(tin + fabs(tin) * 0x1p-20);
      bound = INFINITY;
    }
    cursor = (int)depth - 1;
    node = qstk[cursor * 16 + (int)q];
  };
  if (PARK) {  // parked quads first, on their own rays; the others take the queue's
    const uint32_t sv = held ? qsave[q] : 0u;
    const bool res = (sv >> 31) != 0u;
    const uint64_t fm0 = __ballot(!res && c == 0u);
    const uint32_t idx = (uint32_t)__popcll(fm0 & ((1ull << (4u * q)) - 1ull));
    next = (uint32_t)__popcll(fm0);
    if (res) {
      ray = (sv >> 8) & 63u;
      unpark(sv & 0xFFu);
      if (c == 0u) qsave[q] = 0u;
    } else {
      ray = idx < n ? (uint32_t)qtab[idx] : kNoRay;
      if (ray != kNoRay) take();
    }
  } else if (ray < n) {
    take();
  }
  if (STATS && lane == 0) st.v[ST_WALKS]++;
  for (;;) {
    const bool has = PARK ? ray != kNoRay : ray < n;
    if (__ballot(has) == 0) break;
    if (STATS) {  // the ballots outside the lane-0 branch: they must see every quad
      const uint64_t at_node = __ballot(has && !(node >> 31));
      const uint64_t busy = __ballot(has && c == 0u);
      if (lane == 0) {
        st.v[ST_ROUNDS]++;
        st.v[ST_IDLE_SLOTS] += 16u - (uint32_t)__popcll(busy);  // the drain: quads without a ray this round
        st.v[ST_NODE_ROUNDS] += at_node ? 1u : 0u;
        st.v[ST_NODE_LANES] += (uint32_t)__popcll(at_node);
      }
    }
    bool fin = false;
    if (has) {  // quad-uniform from here on
      // A round is an inner-node step (quads at a node) followed by a leaf step (quads at a leaf,
      // including those whose node step just descended into one), then one pop for the quads whose
      // step ended without a next node: a quad descending into a leaf tests it in the same round
      // instead of the next. Each quad takes the same steps in the same order, so the walk's answer
      // is unchanged; the wave runs fewer rounds.
      bool pop_now = false;
      if (!(node >> 31)) {
#ifdef YART_WALK_CHECK
        if (node >= M.n_nodes) { walk_fault(4u); node = root; }
#endif
        const gfloat4p N = nodes + 8 * (size_t)node;
        const float4 lo = ld4(N, c);
        float4 hi = ld4(N, 4 + c);
        asm volatile("" : "+v"(hi.z), "+v"(hi.w));  // child id and ranks with the box, one round
        bool hk;
        float ent;
        if (f2b) {
          hk = child_hit_f32(lo, hi, inv32, c32, tmin32, teff32, ent);
          ent = fminf(ent, 3.0e38f);
        } else {
          double l;
          const CoopRay& s = rays[ray];  // the reference order (rare): t_max is the best so far
          const double ro[3] = {s.o[0], s.o[1], s.o[2]};
          const double inv[3] = {1.0 / s.d[0], 1.0 / s.d[1], 1.0 / s.d[2]};
          hk = child_hit_l(lo, hi, ro, inv, tmin, tb, l);
          ent = 0.0f;  // unused in the reference order
        }
        // push rank: reference order from ORDER_TABLE (precomputed per octant); front to back
        // 3 - (distance rank), so the nearest hit child is the one taken next and the farthest
        // sits deepest in the stack
        const uint32_t rk = f2b ? 3u - quad_rank(hk ? ent : INFINITY, c) : (__float_as_uint(hi.w) >> (2u * pos)) & 3u;
        uint32_t ordered = hk ? 1u << rk : 0u;  // bit r: the child of push rank r was hit
        ordered |= quad_perm<0xB1>(ordered);
        ordered |= quad_perm<0x4E>(ordered);
        if (STATS && c == 0) st.v[ST_NODES]++;
        if (ordered) {
          // The last child pushed is the next popped: it goes straight to `node` (its id OR-ed
          // across the quad); the others take stack slots in rank order.
          const uint32_t last = 31u - __clz(ordered);
          const uint32_t child = __float_as_uint(hi.z);
          uint32_t nx = (hk && rk == last) ? child : 0u;
          nx |= quad_perm<0xB1>(nx);
          nx |= quad_perm<0x4E>(nx);
          if (hk && rk != last) {
            const int depth_slot = cursor + (int)__popc(ordered & ((1u << rk) - 1u));
            const int slot = depth_slot * 16 + (int)q;
            // rounded down: a dropped entry's true entry is beyond the bound too
            const uint32_t eb = __float_as_uint(ent);
            const uint32_t e16 = (eb >> 16) + ((eb >> 31) & ((eb & 0xFFFFu) != 0u));
#ifdef YART_WALK_CHECK
            if (depth_slot >= (OVF ? kMaxStackSlots : SLOTS)) walk_fault(8u);
            else
#endif
            if (!OVF || depth_slot < SLOTS) {
              qstk[slot] = child;
              qent[slot] = (CoopEnt)e16;
            } else {  // deep meshes: entries past the LDS slots in the wave's HBM region
              ovf[slot - SLOTS * 16] = child;
              ovf[kOvfQuadWords + slot - SLOTS * 16] = e16;
              if (STATS) st.v[ST_OVF_PUSHES]++;
            }
          }
          cursor += (int)__popc(ordered) - 1;
#ifdef YART_WALK_CHECK
          if (cursor >= (OVF ? kMaxStackSlots : SLOTS)) cursor = (OVF ? kMaxStackSlots : SLOTS) - 1;
#endif
          node = nx;
        } else {
          pop_now = true;
        }
      }
      if (!pop_now && (node >> 31)) {
        if (STATS) {
          const uint64_t lq = __ballot(true), lt = __ballot(c < ((node >> 27) & 0xFu));
          if (lane == (uint32_t)__builtin_ctzll(lq)) {
            st.v[ST_LEAF_ROUNDS]++; st.v[ST_LEAF_QUAD_LANES] += (uint32_t)__popcll(lq); st.v[ST_LEAF_LANES] += (uint32_t)__popcll(lt);
          }
        }
        uint32_t count = (node >> 27) & 0xFu;
        const uint32_t first = node & ((1u << 27) - 1u);
#ifdef YART_WALK_CHECK
        if (first + count > M.n_recs || count == 0 || count > 4) { walk_fault(1u); count = 0; }
#endif
        // A candidate's key orders equal t's as the reference visits them: front to back (either
        // tree) by (the reference leaf's depth-first rank for this octant, lane in that leaf) and
        // the quad lane in the low bits; in the reference's own order the lower lane of the leaf.
        // t and key take their no-candidate values in one select after the test: set up front,
        // the defaults were copied again at every exit of the short-circuited test.
        double tt, u, v;
        uint32_t kk, id, li = 0u;  // li is read across the quad (ds_bpermute): defined in every lane
        bool cand = false;
        if (c < count) {
          const gfloat4p R = leaves + kRecF4 * (size_t)(first + c);
          uint32_t ln, so;
          const TriF64 g = tri_load(R, li, ln, so);  // li: the record's reference leaf
#ifdef YART_WALK_CHECK
          if (li >= M.n_leaves) { walk_fault(2u); li = 0u; }
#endif
          // candidates: t in [t_min, t_max_in) and nearer than the best, or as near (front to
          // back: the tie goes to the reference's visiting order)
          const CoopRay& s = rays[ray];
          const double ro[3] = {s.o[0], s.o[1], s.o[2]}, rd[3] = {s.d[0], s.d[1], s.d[2]};
          if (leaf_tri_hit(g, ro, rd, tmin, s.tmax, tt, u, v) && (tt < tb || (f2b && tt == tb))) {
            cand = true;
            id = so;  // sorted index: the normal table's row
            kk = f2b ? (aux[li].rank[pos] << 4) | (ln << 2) | c : c;
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
            tb = t; fnd = true; bleaf = li; bkey = key;
            if (c == w) {
              CoopRay& s = rays[ray];
              coop_put_d(&s.c32[0], t); coop_put_d(&s.c32[2], u); coop_put_d(&s.c32[4], v);
              s.inv32[0] = __uint_as_float(id);
              s.inv32[1] = __uint_as_float(1u);
            }
            if (f2b) {
              const double lim = t * (1.0 + kF2bMargin), tin = rays[ray].tmax;
              const double teff = lim < tin ? lim : tin;
              teff32 = (float)(teff + teff * 0x1p-20);
              bound = (float)lim;
            }
          }
        }
        pop_now = true;
      }
      if (pop_now) {
        for (;;) {  // front to back: entries whose box begins beyond the bound are dropped
          if (cursor == 0) { fin = true; break; }
          cursor -= 1;
          uint32_t e16;
          if (!OVF || cursor < SLOTS) {
            node = qstk[cursor * 16 + (int)q];
            e16 = qent[cursor * 16 + (int)q];
          } else {
            node = ovf[(cursor - SLOTS) * 16 + (int)q];
            e16 = ovf[kOvfQuadWords + (cursor - SLOTS) * 16 + (int)q];
          }
          if (!f2b || !(__uint_as_float(e16 << 16) > bound)) break;
        }
      }
      if (kPostCheck && fin && c == 0)  // the ray's own lane checks W after the walk (below)
        rays[ray].flags = (f2b && fnd) ? (0x80000000u | bleaf) : 0u;
      if (!kPostCheck && fin && f2b && fnd) {
        // W is the reference's answer if its leaf box passes the reference's f64 test at t_max_in
        // (the f32 test visits a superset) and W's t is not before that box's entry (above)
        const auto& A = aux[bleaf];
        const CoopRay& s = rays[ray];
        double l = tmin, h = s.tmax;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const double iv = 1.0 / s.d[j];  // as formed at staging: the reference's slab test
          const double t0 = ((double)A.lo[j] - s.o[j]) * iv, t1 = ((double)A.hi[j] - s.o[j]) * iv;
          l = fmax(l, fmin(t0, t1));
          h = fmin(h, fmax(t0, t1));
        }
        if (!(h > l && tb >= l)) {
          if (STATS && c == 0) st.v[ST_REWALK]++;
          restart(false);
          fin = false;
        }
      }
    }
    if (fin && !fnd && c == 0) rays[ray].inv32[1] = 0.0f;  // no hit (a hit's record is already written)
    const uint64_t fm = __ballot(fin && c == 0);
    if (fm) {
      if (fin) {
        const uint32_t idx = next + (uint32_t)__popcll(fm & ((1ull << (4u * q)) - 1ull));
        if (PARK) {
          ray = idx < n ? (uint32_t)qtab[idx] : kNoRay;
          if (ray != kNoRay) take();
        } else {
          ray = idx;
          if (ray < n) take();
        }
      }
      next += (uint32_t)__popcll(fm);
    }
    // PARK: the queue is empty and at most park_quads quads still walk (a call that staged at least
    // kParkMinRays new rays: with fewer, the lanes are running out of work and the walks finish here)
    if (PARK && park_quads != 0u && n >= kParkMinRays && next >= n) {
      const bool busy = ray != kNoRay;
      if ((uint32_t)__popcll(__ballot(busy && c == 0u)) <= park_quads) {
        if (busy) park();
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // W is the reference's answer if its leaf box passes the reference's f64 test at the walk's
  // t_max (the f32 test visits a superset) and W's t is not before that box's entry (above): each
  // lane checks its own ray once, after the walk, instead of the whole wave at every ray's end. A
  // ray that fails walks again in the reference's order, per lane (qbvh_t, a 32-slot stack in this
  // wave's LDS, free once every lane has read its record) — rare.
  bool redo = false;
  Ray wr;  // the walked ray, read back from its record (the caller's copy need not live through the walk)
  if (walk || (PARK && resume)) {
    const CoopRay& s = rays[PARK ? lane : rank];
    const uint32_t fl = s.flags;
    if (PARK && (fl >> 30) == 1u) {
      *parked = true;  // its walk goes on at the next call
    } else {
      found = __float_as_uint(s.inv32[1]) != 0u;
      t_hit = coop_get_d(&s.c32[0]); u_hit = coop_get_d(&s.c32[2]); v_hit = coop_get_d(&s.c32[4]);
      tri = __float_as_uint(s.inv32[0]);
      if (kPostCheck && (fl >> 31)) {
        wr.o = mk(s.o[0], s.o[1], s.o[2]);
        wr.d = mk(s.d[0], s.d[1], s.d[2]);
        redo = !coop_check(aux, fl & 0x3FFFFFFFu, wr, tmin, tmax_in, t_hit) || __builtin_amdgcn_readfirstlane(g_force_rewalk) != 0u;
      }
    }
  }
  if (kPostCheck && __ballot(redo) != 0ull) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (redo) {
      if (STATS) st.v[ST_REWALK]++;
      // PARK: parked walks keep their records and stacks in the LDS; the re-walk's stack is this
      // lane's column of the wave's HBM region instead
      uint32_t* const rstk = (PARK && park_quads) ? ovf + 2 * kOvfQuadWords + lane : reinterpret_cast<uint32_t*>(lds) + lane;
      found = qbvh_t<STATS, OVF>(M, wr, tmin, tmax_in, t_hit, tri, u_hit, v_hit, rstk, st, ovf);
    }
  }
}

// The QBVH leaf record (qbvh.rs:500-540): barycentric normal of the winning triangle, facing
// the ray (front face when dot <= 0).
__device__ __forceinline__ void mesh_rec(const DevMesh& M, const Ray& r, double t, uint32_t tri, double u, double v, Hit& h) {
  const double ro[3] = {r.o.x, r.o.y, r.o.z}, rd[3] = {r.d.x, r.d.y, r.d.z};
  const double w = 1.0 - u - v;
  double nn[9];
  if (M.normals32) {  // exact f32 values (OBJ vn)
    const float* f = M.normals32 + 9 * (size_t)tri;
#pragma unroll
    for (int k = 0; k < 9; ++k) nn[k] = (double)f[k];
  } else {
    const double* f = M.normals + 9 * (size_t)tri;
#pragma unroll
    for (int k = 0; k < 9; ++k) nn[k] = f[k];
  }
  const double onx = nn[0] * w + nn[3] * u + nn[6] * v;
  const double ony = nn[1] * w + nn[4] * u + nn[7] * v;
  const double onz = nn[2] * w + nn[5] * u + nn[8] * v;
  const bool ff = (rd[0] * onx + rd[1] * ony + rd[2] * onz) <= 0.0;
  const double sign = ff ? 1.0 : -1.0;
  h.t = t;
  h.p = mk(ro[0] + t * rd[0], ro[1] + t * rd[1], ro[2] + t * rd[2]);
  h.n = mk(sign * onx, sign * ony, sign * onz);
  h.ff = ff;
}

// ------------------------------------------------------------------------ world hit
// Which primitive of the world list won, and where: enough to rebuild its record exactly. In the
// list and world-BVH kernels the world pass keeps t and one word, obj << 3 | sub (sub = a box face;
// every update is then one 64-bit and one 32-bit select), and the record recomputes a triangle's
// u, v; the mesh kernels carry u, v and the triangle (a mesh hit's walk result) through the pass.
struct HitId { double t, u, v; uint32_t obj, sub; };

// CULL: the box entity's f32 pre-test (box_t); off in the list kernels (HAS_MESH false), on in the
// mesh and world-BVH kernels
template <bool HAS_MESH, bool STATS, bool OVF = false, bool CULL = HAS_MESH>
__device__ __forceinline__ bool prim_t(const DevScene& S, const DevObject& o, uint32_t kind, const Ray& r,
                                       double tmin, double tmax, double& t, uint32_t& sub, double& u, double& v,
                                       uint32_t* stk, Stats& st, uint32_t* ovf = nullptr) {
  switch (kind) {
    case YART_PRIM_SPHERE: if (STATS) st.v[ST_PRIM]++; return sphere_t(o.p, r, tmin, tmax, t);
    case YART_PRIM_XY_RECT: if (STATS) st.v[ST_PRIM]++; return rect_t<2, 0, 1>(o.p, r, tmin, tmax, t);
    case YART_PRIM_XZ_RECT: if (STATS) st.v[ST_PRIM]++; return rect_t<1, 0, 2>(o.p, r, tmin, tmax, t);
    case YART_PRIM_YZ_RECT: if (STATS) st.v[ST_PRIM]++; return rect_t<0, 1, 2>(o.p, r, tmin, tmax, t);
    case YART_PRIM_BOX: if (STATS) st.v[ST_PRIM] += 6; return box_t<CULL>(o.p, r, tmin, tmax, t, sub);
    case YART_PRIM_TRIANGLE: if (STATS) st.v[ST_PRIM]++; return triangle_t(o.p, r, tmin, tmax, t, u, v);
    case YART_PRIM_MOVING_SPHERE: if (STATS) st.v[ST_PRIM]++; return moving_sphere_t(o.p, r, tmin, tmax, t);
    case YART_PRIM_MESH:
      if constexpr (HAS_MESH) return qbvh_t<STATS, OVF>(S.meshes[o.mesh], r, tmin, tmax, t, sub, u, v, stk, st, ovf);
      return false;
  }
  return false;
}

// Translate / RotateY on the way in (hittable.rs:136-152, 217-251), outermost first.
__device__ __forceinline__ Ray to_local(const DevObject& o, uint32_t nxf, const Ray& r) {
  Ray lr = r;
  for (uint32_t l = 0; l < nxf; ++l) {
    const uint32_t k = o.xf_kind[l];
    if (k == YART_XF_TRANSLATE) {
      lr.o = sub(lr.o, ld3(o.xf[l]));
    } else if (k == YART_XF_ROTATE_Y) {
      const double sn = o.xf[l][0], cs = o.xf[l][1];
      const V3 ro = lr.o, rdd = lr.d;
      lr.o.x = cs * ro.x - sn * ro.z;
      lr.o.z = sn * ro.x + cs * ro.z;
      lr.d.x = cs * rdd.x - sn * rdd.z;
      lr.d.z = sn * rdd.x + cs * rdd.z;
    }
  }
  return lr;
}

// HittableList::hit (hittable.rs:67-79), split in two: the closest-hit search over the list
// (uniform object index: the objects arrive on the scalar path) keeps only t and the winner's
// id, and hit_record then builds the one record the reference keeps — the winner's, with its
// wrappers undone innermost first on the way out. Building a record per candidate instead
// cost every wave the selects and point/normal arithmetic of each primitive some lane hit.
// ConstantMedium::hit (hittable.rs:277-318): the boundary (the wrapper chain below the medium
// and the primitive) hit twice, the entry/exit clamped to [t_min, t_max] and 0, and a free path
// -1/density · ln(ξ) against the distance inside. xf[0][0] holds -1/density.
template <bool HAS_MESH, bool STATS, bool OVF = false>
__device__ __forceinline__ bool medium_t(const DevScene& S, const DevObject& o, uint32_t kind, const Ray& lr, const Ray& r,
                                         double tmin, double tmax, double& t, uint32_t* stk, Stats& st,
                                         const QueryCtx& q, uint32_t obj, uint32_t* ovf = nullptr) {
  double t1, t2, u, v;
  uint32_t sub;
  if (!prim_t<HAS_MESH, STATS, OVF>(S, o, kind, lr, -INFINITY, INFINITY, t1, sub, u, v, stk, st, ovf)) return false;
  if (!prim_t<HAS_MESH, STATS, OVF>(S, o, kind, lr, t1 + 0.0001, INFINITY, t2, sub, u, v, stk, st, ovf)) return false;
  if (t1 < tmin) t1 = tmin;
  if (t2 > tmax) t2 = tmax;
  if (!(t1 < t2)) return false;
  if (t1 < 0.0) t1 = 0.0;
  const double ray_length = len(r.d);
  const double distance_inside_boundary = (t2 - t1) * ray_length;
  const double hit_distance = o.xf[0][0] * log_det(medium_draw(q, obj));
  if (!(hit_distance < distance_inside_boundary)) return false;
  t = t1 + hit_distance / ray_length;
  return true;
}

// EXT: the scene has media / noise textures / isotropic materials (DevScene::has_ext); kernels
// for the other scenes are built without those paths (they cost the cornell box 12 % as
// dead-but-compiled code: registers and spills).
// HAS_MESH: called from converged code by all 64 lanes, `want` marking the lanes with a query —
// meshes are walked cooperatively (qbvh_coop) by the whole wave, the other objects per lane.
// A wave-uniform read of a scene table (the list walk's object, a light of the mixture pdf): the
// index made uniform by readfirstlane and the table read through the constant address space, so
// the record arrives by scalar loads into SGPRs. Read as a plain global, the loads after the
// loop's scratch stores were vector loads (the compiler cannot prove them unclobbered) and every
// field of the record took a VGPR.
template <class T>
__device__ __forceinline__ const T& uniform_at(const T* base, uint32_t i) {
  typedef const __attribute__((address_space(4))) T* cptr;
  return *(const T*)((cptr)base + __builtin_amdgcn_readfirstlane(i));
}

template <bool HAS_MESH, bool STATS, bool EXT, int SLOTS = kCoopSlots, bool OVF = false, bool PARK = false,
          bool CULL = HAS_MESH>
__device__ __forceinline__ bool world_closest(const DevScene& S, bool want, const Ray& r, double tmin, double tmax, HitId& id,
                                              uint32_t* stk, uint8_t* coop, Stats& st, const QueryCtx& q,
                                              uint32_t* ovf = nullptr, bool resume = false, bool* parked = nullptr) {
  bool found = false;
  if (PARK) *parked = false;
  double closest = tmax;
  uint32_t who = 0;  // obj << 3 | sub (the kernels without meshes)
  id.u = 0.0; id.v = 0.0; id.obj = 0; id.sub = 0;
  for (uint32_t i = 0; i < S.n_objects; ++i) {
    const DevObject& o = uniform_at(S.objects, i);
    const uint32_t kind = o.kind, nxf = o.n_xf;
    const bool medium = EXT && nxf != 0 && o.xf_kind[0] == YART_XF_MEDIUM;
    if (HAS_MESH && kind == YART_PRIM_MESH && !medium) {  // wave-uniform
      const Ray lr = to_local(o, nxf, r);
      bool hit;
      double t, u, v;
      uint32_t sub;
      qbvh_coop<STATS, SLOTS, OVF, PARK>(uniform_at(S.meshes, o.mesh), want, lr, tmin, closest, hit, t, sub, u, v, coop, st, ovf,
                                         resume, parked, S.park);
      if (hit) {
        closest = t;
        id.obj = i; id.sub = sub; id.u = u; id.v = v;
        found = true;
      }
    } else if (want) {
      const Ray lr = to_local(o, nxf, r);
      double t, u = 0.0, v = 0.0;
      uint32_t sub = 0;
      const bool hit = medium ? medium_t<HAS_MESH, STATS, OVF>(S, o, kind, lr, r, tmin, closest, t, stk, st, q, i, ovf)
                              : prim_t<HAS_MESH, STATS, OVF, CULL>(S, o, kind, lr, tmin, closest, t, sub, u, v, stk, st, ovf);
      if (hit) {
        closest = t;
        if (HAS_MESH) { id.obj = i; id.sub = sub; id.u = u; id.v = v; }
        else who = (i << 3) | sub;
        found = true;
      }
    }
  }
  if (!HAS_MESH) { id.obj = who >> 3; id.sub = who & 7u; }
  id.t = closest;
  return found;
}

template <bool HAS_MESH, bool EXT>
__device__ __forceinline__ void hit_record(const DevScene& S, const Ray& r, const HitId& id, Hit& h) {
  const DevObject& o = S.objects[id.obj];  // per lane
  const uint32_t kind = o.kind, nxf = o.n_xf;
  if (EXT) { h.u = 0.0; h.v = 0.0; }
  if (EXT && nxf != 0 && o.xf_kind[0] == YART_XF_MEDIUM) {  // hittable.rs:306-315: at t on the outer ray
    h.t = id.t; h.p = at(r, id.t); h.n = mk(1.0, 0.0, 0.0); h.ff = true; h.mat = o.material;
    return;
  }
  const Ray lr = to_local(o, nxf, r);
  if (kind == YART_PRIM_SPHERE) {
    sphere_rec<EXT>(o.p, lr, id.t, h);
  } else if (kind <= YART_PRIM_BOX) {  // rects and box faces
    const uint32_t a = kind == YART_PRIM_BOX ? 2u - id.sub / 2u : (kind == YART_PRIM_XY_RECT ? 2u : kind == YART_PRIM_XZ_RECT ? 1u : 0u);
    rect_rec(a, lr, id.t, h);
    if (EXT) {  // the face's rect bounds (box_entity.rs:22-36)
      const double* p = o.p;
      double bnd[4] = {p[0], p[1], p[2], p[3]};
      if (kind == YART_PRIM_BOX) {
        const uint32_t f = id.sub / 2u;
        bnd[0] = f == 2 ? p[1] : p[0]; bnd[1] = f == 2 ? p[4] : p[3];
        bnd[2] = f == 0 ? p[1] : p[2]; bnd[3] = f == 0 ? p[4] : p[5];
      }
      rect_uv(a, bnd, lr, id.t, h);
    }
  } else if (kind == YART_PRIM_TRIANGLE) {
    double u = id.u, v = id.v;  // the mesh kernels carry a triangle's u, v through the world pass
    if (!HAS_MESH) triangle_uv(o.p, lr, u, v);
    triangle_rec<EXT>(o.p, lr, id.t, u, v, h);
  } else if (kind == YART_PRIM_MOVING_SPHERE) {
    moving_sphere_rec<EXT>(o.p, lr, id.t, h);
  } else {
    if constexpr (HAS_MESH) mesh_rec(S.meshes[o.mesh], lr, id.t, id.sub, id.u, id.v, h);
  }
  for (int l = (int)nxf - 1; l >= 0; --l) {
    const uint32_t k = o.xf_kind[l];
    if (k == YART_XF_TRANSLATE) {
      h.p = add(h.p, ld3(o.xf[l]));
    } else if (k == YART_XF_ROTATE_Y) {
      const double sn = o.xf[l][0], cs = o.xf[l][1];
      const V3 p = h.p, n = h.n;
      h.p.x = cs * p.x + sn * p.z;
      h.p.z = -sn * p.x + cs * p.z;
      h.n.x = cs * n.x + sn * n.z;
      h.n.z = -sn * n.x + cs * n.z;
    } else {
      h.ff = !h.ff;  // FlipFace (hittable.rs:338-349)
    }
  }
  h.mat = o.material;
}

// World BVH walk (DevWorldNode4; scenes without meshes): per lane over the 4-wide tree — the
// binary SAH tree collapsed two levels per node (world_bvh.cpp), so a ray's chain of dependent node
// reads is half as long (the random scene's walk waited on dependencies for 55 % of its wave
// cycles) — nearest child first, 32-slot stack in LDS like the QBVH. The linear scan accepts an
// object iff its first root r_i >= t_min satisfies r_i <= closest-so-far (every kind here is
// inclusive at t_max), so it returns the minimum r_i, ties going to the LATER object; any visiting
// order that keeps (min t, max index) returns the same winner, and the record is then rebuilt from
// it as before. Node culling is an f32 slab test against the box grown by m = 2^-12 (node
// magnitude + |origin|; the node's share is stored in the box, the ray's is added per walk, r05:
// random-scene +4.4-5.8 %, profiles/r05_ab_world_fma_slab.log) — f32 rounding (~1e-7 relative,
// the fma's and the per-ray constants' included) stays far inside m — over [t_min, closest]
// widened by 2^-10, so it never drops a node holding a hit the scan would accept (ties included).
// Non-finite rays take the list walk.
// The diamond angle of the x-z direction mod pi: monotone in the angle phi with slope in [1/2, 1],
// so a window of w around a tabulated direction covers at least w radians (world_bvh.cpp holds the
// host's copy of this formula).
__device__ __forceinline__ double plane_diamond(double dx, double dz) {
  if (dz < 0.0 || (dz == 0.0 && dx < 0.0)) { dx = -dx; dz = -dz; }
  const double ax = fabs(dx);
  return dx >= 0.0 ? dz / (dx + dz) : 1.0 + ax / (ax + dz);
}
__device__ __noinline__ bool near_plane_dir(const DevScene& S, double dx, double dz) {
  if (fabs(dx) + fabs(dz) < 1e-280) return true;  // so short that the rotations' products can underflow to 0
  const double dm = plane_diamond(dx, dz), lo = dm - kPlaneDirWindow;
  const double* tab = S.plane_dirs;
  uint32_t i = 0;  // the first entry >= lo (a +inf pad entry at worst)
  for (uint32_t s = S.n_plane_dirs >> 1; s != 0; s >>= 1)
    if (tab[i + s - 1] < lo) i += s;
  return tab[i] <= dm + kPlaneDirWindow;
}

template <bool STATS>
__device__ __forceinline__ bool world_closest_bvh(const DevScene& S, const Ray& r, double tmin, double tmax, HitId& id,
                                                  uint32_t* stk, Stats& st) {
  const float o[3] = {(float)r.o.x, (float)r.o.y, (float)r.o.z};
  const float d[3] = {(float)r.d.x, (float)r.d.y, (float)r.d.z};
  const float chk = o[0] + o[1] + o[2] + d[0] + d[1] + d[2];
  // Non-finite rays, and rays with an exactly zero direction component (which can lie in a rect's
  // plane, where rect_t's NaN t "hits" it outside any box: aarect.rs:111-146), take the list walk.
  bool in_plane = r.d.x == 0.0 || r.d.y == 0.0 || r.d.z == 0.0;
  // The same in the frames of the rotated rects and boxes: there a direction component can cancel to
  // exactly 0 while no world component is 0 (cos 90° d_x == d_z). Rays near those directions
  // (DevScene::plane_dirs) take the list walk too. 0 entries in scenes without rotated planes.
  if (S.n_plane_dirs) in_plane = in_plane || near_plane_dir(S, r.d.x, r.d.z);
  if (!(fabsf(chk) <= 3.0e38f) || in_plane)
    return world_closest<false, STATS, false, kCoopSlots, false, false, true>(S, true, r, tmin, tmax, id, stk, nullptr, st, QueryCtx{});
  float inv[3];
  bool use[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    use[j] = fabsf(d[j]) >= 1.0e-20f;  // smaller: the slab does not constrain t
    // an unused axis gets a NaN reciprocal: its t0, t1 are NaN, and fmaxf / fminf (IEEE maxNum /
    // minNum: the other operand) then leave the interval as it is — the slab unconstrained without
    // a branch per child and axis
    inv[j] = use[j] ? __builtin_amdgcn_rcpf(d[j]) : __builtin_nanf("");
  }
  const float O = fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fabsf(o[2]));
  // child boxes come grown by their own margin (mag 2^-12, DevWorldNode4); the ray's share, O 2^-12,
  // goes into per-ray constants so that each slab bound is one fma: t0 = (bl - mr - o) inv =
  // fma(bl, inv, -(o + mr) inv), t1 = fma(bh, inv, (mr - o) inv). A ray whose constants could
  // overflow (|o| |1/d| near the f32 range) takes the list walk.
  const float mr = O * 0x1p-12f;
  const float imax = fmaxf(fmaxf(fabsf(inv[0]), fabsf(inv[1])), fabsf(inv[2]));
  if (!((O + mr) * imax <= 1.0e37f))
    return world_closest<false, STATS, false, kCoopSlots, false, false, true>(S, true, r, tmin, tmax, id, stk, nullptr, st, QueryCtx{});
  float ca[3], cb[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) { ca[j] = -((o[j] + mr) * inv[j]); cb[j] = (mr - o[j]) * inv[j]; }
  float tlo = (float)tmin;
  tlo = tlo - fabsf(tlo) * 0x1p-10f;
  bool found = false;
  double closest = tmax;
  uint32_t who = 0;  // obj << 3 | sub; ties go to the later object: the larger word
  id.u = 0.0; id.v = 0.0;
  // the walk carries node handles (DevWorldNode4::handle), read with the child boxes: descending
  // and popping take a node without a dependent read of its own record
  const gfloat4p nodes = (gfloat4p)S.world_nodes;
  uint32_t hnd = 0u;  // the root: inner node 0
  int cursor = 0;
  uint32_t kk = 0;  // the next sphere of the current leaf
  for (;;) {
    uint32_t count = hnd >> 28, first = hnd & (kWorldHandleFirstMask - 1u);
    if (STATS) {  // SIMT efficiency of the per-lane walk: iterations the wave issues (lane visits: ST_NODES, ST_PRIM)
      const uint64_t on = __ballot(true), lf = __ballot(count != 0u);
      if (__lane_id() == (uint32_t)__builtin_ctzll(on)) { st.v[ST_WORLD_ITERS]++; st.v[ST_WORLD_LEAF_ITERS] += lf ? 1u : 0u; }
    }
    // An iteration is a leaf step (lanes at a leaf) followed by an inner-node step (lanes at an inner
    // node, including those whose leaf step just finished the leaf and popped one): a lane leaving a
    // leaf steps its next node in the same iteration instead of the next. Each lane takes the same
    // steps in the same order, so the answer is unchanged; the wave runs fewer iterations.
    if (count) {
      bool done = true;
      if ((hnd >> 27) & 1u) {
        // a leaf of plain spheres: the compact records (32 B each, one load pair) instead of the
        // object records and the kind switch; the same sphere_t on the same values. ONE sphere per
        // iteration (the lane stays on the leaf until its spheres are done), not the whole leaf in
        // an inner loop: an iteration in which some lane sits at a 4-sphere leaf then costs the wave
        // one sphere test, not four (r05: random-scene +1.7-1.8 %, profiles/r05_ab_world_step1.log).
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
        if (kk < count) done = false;  // the leaf's next sphere in the next iteration
        else kk = 0u;
      } else {
        for (uint32_t k = 0; k < count; ++k) {
          const uint32_t i = S.world_objs[first + k];
          const DevObject& ob = S.objects[i];
          const Ray lr = to_local(ob, ob.n_xf, r);
          double t, u = 0.0, v = 0.0;
          uint32_t sub = 0;
          if (prim_t<false, STATS, false, true>(S, ob, ob.kind, lr, tmin, closest, t, sub, u, v, stk, st) &&
              (!found || t < closest || (i << 3) > who)) {
            closest = t;
            who = (i << 3) | sub;
            found = true;
          }
        }
      }
      if (done) {  // the next handle: stepped below if it is an inner node, else next iteration
        if (cursor == 0) break;
        cursor--;
        hnd = stk[cursor * 64];
      }
    }
    if ((hnd >> 28) == 0u) {  // an inner node
      first = hnd & (kWorldHandleFirstMask - 1u);
      float thi = (float)closest;
      thi = thi + fabsf(thi) * 0x1p-10f;
      const gfloat4p N = nodes + 8 * (size_t)first;
      float4 bmn[3], bmx[3];
      bmn[0] = ld4(N, 0); bmn[1] = ld4(N, 1); bmn[2] = ld4(N, 2);
      bmx[0] = ld4(N, 3); bmx[1] = ld4(N, 4); bmx[2] = ld4(N, 5);
      const float4 hd = ld4(N, 7);
      const uint32_t ch[4] = {__float_as_uint(hd.x), __float_as_uint(hd.y), __float_as_uint(hd.z), __float_as_uint(hd.w)};
      // per child: the binary tree's test of that node (the same expression on the same box). (A
      // packed-f32 form, two children per v_pk_add_f32 / v_pk_mul_f32, lost 3 % on the random scene
      // in r05: profiles/r05_ab_world_packed.log.)
      float key[4];  // entry of a hit child, +inf for a miss
      uint32_t hc[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float lo = tlo, hi = thi;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const float bl = k == 0 ? bmn[j].x : k == 1 ? bmn[j].y : k == 2 ? bmn[j].z : bmn[j].w;
          const float bh = k == 0 ? bmx[j].x : k == 1 ? bmx[j].y : k == 2 ? bmx[j].z : bmx[j].w;
          const float t0 = __builtin_fmaf(bl, inv[j], ca[j]), t1 = __builtin_fmaf(bh, inv[j], cb[j]);
          lo = fmaxf(lo, fminf(t0, t1));
          hi = fminf(hi, fmaxf(t0, t1));
        }
        const bool hit = lo <= hi && ch[k] != kWorld4Empty;
        key[k] = hit ? fminf(lo, 3.0e38f) : INFINITY;  // a hit whose entry overflowed stays a hit
        hc[k] = ch[k];
      }
      if (STATS) st.v[ST_NODES]++;
      // nearest first: sort (key, handle) ascending (a 5-comparator network), take the first hit
      // and push the other hits farthest first
      auto cx = [&](int a, int b) {
        const bool sw = key[b] < key[a];
        const float ka = key[a], kb = key[b];
        const uint32_t ha = hc[a], hb = hc[b];
        key[a] = sw ? kb : ka; key[b] = sw ? ka : kb;
        hc[a] = sw ? hb : ha; hc[b] = sw ? ha : hb;
      };
      cx(0, 1); cx(2, 3); cx(0, 2); cx(1, 3); cx(1, 2);
      if (key[0] < INFINITY) {
        if (key[3] < INFINITY) stk[(cursor++) * 64] = hc[3];
        if (key[2] < INFINITY) stk[(cursor++) * 64] = hc[2];
        if (key[1] < INFINITY) stk[(cursor++) * 64] = hc[1];
        hnd = hc[0];
      } else {
        if (cursor == 0) break;
        cursor--;
        hnd = stk[cursor * 64];
      }
    }
  }
  id.obj = who >> 3; id.sub = who & 7u;
  id.t = closest;
  return found;
}

template <bool HAS_MESH, bool BVH, bool STATS, bool EXT, int SLOTS = kCoopSlots, bool OVF = false, bool PARK = false>
__device__ __forceinline__ bool world_hit(const DevScene& S, bool want, const Ray& r, double tmin, double tmax, Hit& rec,
                                          int32_t& which, uint32_t* stk, uint8_t* coop, Stats& st, const QueryCtx& q,
                                          uint32_t* ovf = nullptr, bool resume = false, bool* parked = nullptr) {
  HitId id;
  if constexpr (BVH) {  // no media or meshes in BVH scenes (capi.cpp)
    if (!world_closest_bvh<STATS>(S, r, tmin, tmax, id, stk, st)) return false;
  } else {
    if (!world_closest<HAS_MESH, STATS, EXT, SLOTS, OVF, PARK>(S, want, r, tmin, tmax, id, stk, coop, st, q, ovf, resume, parked) ||
        !want || (PARK && *parked))
      return false;
  }
  hit_record<HAS_MESH, EXT>(S, r, id, rec);
  which = (int32_t)id.obj;
  return true;
}


// ----------------------------------------------------------------------- ONB and PDFs
// u = w × v is formed where local() needs it (the same expression on the same inputs): kept as a
// member, its three doubles were live — and spilled — through the direction sampling.
struct Onb { V3 v, w; };
template <class M>
__device__ __forceinline__ Onb onb_from_w(V3 n, M& m) {  // onb.rs:10-21
  Onb b;
  b.w = m.unit(n);
  const V3 a = fabs(b.w.x) > 0.9 ? mk(0.0, 1.0, 0.0) : mk(1.0, 0.0, 0.0);
  b.v = m.unit(cross(b.w, a));
  return b;
}
__device__ __forceinline__ V3 local(const Onb& b, V3 a) {
  const V3 u = cross(b.w, b.v);
  return add(add(smul(a.x, u), smul(a.y, b.v)), smul(a.z, b.w));
}
template <class M>
__device__ __forceinline__ V3 random_cosine_direction(Rng& g, M& m) {  // pdf.rs:15-25
  const double r1 = gen_f64(g), r2 = gen_f64(g);
  const double z = m.sqrt(1.0 - r2);
  double s, c;
  sincos_det(2.0 * kPi * r1, s, c);
  const double sr2 = m.sqrt(r2);
  return mk(c * sr2, s * sr2, z);
}
// ud = unit_vector(direction), formed once per scatter by the caller (it also feeds Lambertian's
// scatter_pdf and a rect light's pdf its length): the same values, one evaluation
// x / pi through the policy with pi's reciprocal as a constant (div_const; the Fast policy checks x's
// range and re-runs the block on the IEEE sequences outside it). (The reciprocal formed by rcp_core
// and hoisted out of the loop instead cost the cornell box 1.5 %: registers; r06x_ab_picore.log.)
template <bool CDIV, class M>
__device__ __forceinline__ double over_pi(double x, M& m) {
  if (!CDIV || !YART_CONST_DIV) return x / kPi;
  double d = kPi, r = kRcpPi;
  asm volatile("" : "+s"(d), "+s"(r));
  return m.quo(x, PosDen{d, r});
}
// ud = unit_vector(direction)
template <bool CDIV, class M>
__device__ __forceinline__ double cosine_value(const Onb& b, V3 ud, M& m) {  // pdf.rs:40-47
  const double cosine = dot(ud, b.w);
  return cosine <= 0.0 ? 0.0 : over_pi<CDIV>(cosine, m);
}

// pdf_value of a light that was hit (or not) at t over [0.001, inf) by (origin, dir).
// ldir = dir.length(), formed by the caller with unit_vector(dir) (scatter_at); LEN: formed here
template <bool LEN, class M>
__device__ __forceinline__ double light_pdf_at(const DevObject& o, V3 origin, V3 dir, double ldir, bool hit, double t, M& m) {
  if (!hit) return 0.0;
  if (o.kind == YART_PRIM_XZ_RECT) {  // aarect.rs:148-162
    Hit h;
    rect_rec(1, Ray{origin, dir, 0.0, 0.0}, t, h);
    const double area = (o.p[1] - o.p[0]) * (o.p[3] - o.p[2]);
    const double distance_squared = h.t * h.t * len2(dir);
    const double cosine = fabs(dot(dir, h.n)) / (LEN ? m.len(dir) : ldir);
    return distance_squared / (cosine * area);
  }
  // sphere.rs:95-110
  const double radius = o.p[3];
  const double cos_theta_max = m.sqrt(1.0 - radius * radius / len2(sub(ld3(o.p), origin)));
  const double solid_angle = 2.0 * kPi * (1.0 - cos_theta_max);
  return 1.0 / solid_angle;
}
template <bool STATS, bool LEN, class M>
__device__ __forceinline__ double light_pdf(const DevObject& o, V3 origin, V3 dir, double ldir, double wl, Stats& st, M& m) {
  if (o.n_xf != 0) return 0.0;  // wrappers do not override Hittable::pdf_value (hittable.rs:28-30)
  Ray r{origin, dir, 0.0, wl};
  double t = 0.0;
  bool hit;
  if (o.kind == YART_PRIM_XZ_RECT) {
    if (STATS) st.v[ST_LIGHT]++;
    hit = rect_t<1, 0, 2>(o.p, r, 0.001, INFINITY, t);
  } else if (o.kind == YART_PRIM_SPHERE) {
    if (STATS) st.v[ST_LIGHT]++;
    hit = sphere_t(o.p, r, 0.001, INFINITY, t, m);
  } else {
    return 0.0;
  }
  return light_pdf_at<LEN>(o, origin, dir, ldir, hit, t, m);
}
template <class M>
__device__ __forceinline__ V3 light_random(const DevObject& o, V3 origin, Rng& g, M& m) {
  if (o.n_xf == 0 && o.kind == YART_PRIM_XZ_RECT) {  // aarect.rs:164-171
    const double x = gen_range(g, o.p[0], o.p[1]);
    const double z = gen_range(g, o.p[2], o.p[3]);
    return sub(mk(x, o.p[4], z), origin);
  }
  if (o.n_xf == 0 && o.kind == YART_PRIM_SPHERE) {  // sphere.rs:112-118, 11-21
    const V3 direction = sub(ld3(o.p), origin);
    const double d2 = len2(direction);
    const Onb uvw = onb_from_w(direction, m);
    const double r1 = gen_f64(g), r2 = gen_f64(g);
    const double radius = o.p[3];
    const double z = 1.0 + r2 * (m.sqrt(1.0 - radius * radius / d2) - 1.0);
    double s, c;
    sincos_det(2.0 * kPi * r1, s, c);
    const double sz = m.sqrt(1.0 - z * z);
    const V3 rs = mk(c * sz, s * sz, z);
    return local(uvw, rs);
  }
  return mk(1.0, 0.0, 0.0);
}

// ---------------------------------------------------------------------- materials
// Rust `f as i32`: saturating, NaN -> 0.
__device__ __forceinline__ int32_t sat_i32(double f) {
  if (f != f) return 0;
  if (f >= 2147483647.0) return INT32_MAX;
  if (f <= -2147483648.0) return INT32_MIN;
  return (int32_t)f;
}
// Perlin::noise (texture.rs:114-180), as oracle.c's perlin_noise.
__device__ __noinline__ double perlin_noise(const yart_perlin* P, uint32_t type, V3 p) {
  if (type == YART_NOISE_SQUARE) {
    const int32_t i = sat_i32(4.0 * p.x) & 255, j = sat_i32(4.0 * p.y) & 255, k = sat_i32(4.0 * p.z) & 255;
    return P->ranfloat[P->perm_x[i] ^ P->perm_y[j] ^ P->perm_z[k]];
  }
  double u = p.x - floor(p.x), v = p.y - floor(p.y), w = p.z - floor(p.z);
  const uint32_t i = (uint32_t)sat_i32(floor(p.x)), j = (uint32_t)sat_i32(floor(p.y)), k = (uint32_t)sat_i32(floor(p.z));
  double accum = 0.0;
  if (type == YART_NOISE_TRILINEAR) {
    u = u * u * (3.0 - 2.0 * u);
    v = v * v * (3.0 - 2.0 * v);
    w = w * w * (3.0 - 2.0 * w);
    for (uint32_t di = 0; di < 2; ++di)
      for (uint32_t dj = 0; dj < 2; ++dj)
        for (uint32_t dk = 0; dk < 2; ++dk) {  // trilinear_interp texture.rs:192-207
          const double c = P->ranfloat[P->perm_x[(i + di) & 255u] ^ P->perm_y[(j + dj) & 255u] ^ P->perm_z[(k + dk) & 255u]];
          accum += ((double)di * u + (double)(1u - di) * (1.0 - u)) * ((double)dj * v + (double)(1u - dj) * (1.0 - v)) *
                   ((double)dk * w + (double)(1u - dk) * (1.0 - w)) * c;
        }
    return accum;
  }
  const double uu = u * u * (3.0 - 2.0 * u), vv = v * v * (3.0 - 2.0 * v), ww = w * w * (3.0 - 2.0 * w);
  for (uint32_t di = 0; di < 2; ++di)
    for (uint32_t dj = 0; dj < 2; ++dj)
      for (uint32_t dk = 0; dk < 2; ++dk) {  // perlin_interp texture.rs:209-228
        const double* c = P->ranvec[P->perm_x[(i + di) & 255u] ^ P->perm_y[(j + dj) & 255u] ^ P->perm_z[(k + dk) & 255u]];
        const V3 weight_v = mk(u - (double)di, v - (double)dj, w - (double)dk);
        accum += ((double)di * uu + (1.0 - (double)di) * (1.0 - uu)) * ((double)dj * vv + (1.0 - (double)dj) * (1.0 - vv)) *
                 ((double)dk * ww + (1.0 - (double)dk) * (1.0 - ww)) * dot(weight_v, ld3(c));
      }
  return accum;
}
__device__ __forceinline__ double perlin_turb(const yart_perlin* P, uint32_t type, V3 p, int depth) {  // texture.rs:230-242
  double accum = 0.0, weight = 1.0;
  V3 temp_p = p;
  for (int d = 0; d < depth; ++d) {
    accum += weight * perlin_noise(P, type, temp_p);
    weight *= 0.5;
    temp_p = muls(temp_p, 2.0);
  }
  return fabs(accum);
}

// Smits basis (color.rs:1711-1982) and RGB::into_spectrum at one bin, as capi.cpp's host copy
// (texels are reflected at run time: a spectrum per texel would be 150 MB for the earth map).
__constant__ double c_smits[7][36] = {
#include "smits.inc"
};
__device__ __forceinline__ double rgb_reflect(double red, double green, double blue, int i) {  // color.rs:54-90
  enum { W, Cy, Ma, Ye, Re, Gr, Bl };
  double s = 0.0;
  if (red <= green && red <= blue) {
    s = red * c_smits[W][i] + s;
    if (green <= blue) { s = (green - red) * c_smits[Cy][i] + s; s = (blue - green) * c_smits[Bl][i] + s; }
    else { s = (blue - red) * c_smits[Cy][i] + s; s = (green - blue) * c_smits[Gr][i] + s; }
  } else if (green <= red && green <= blue) {
    s = green * c_smits[W][i] + s;
    if (red <= blue) { s = (red - green) * c_smits[Ma][i] + s; s = (blue - red) * c_smits[Bl][i] + s; }
    else { s = (blue - green) * c_smits[Ma][i] + s; s = (red - blue) * c_smits[Re][i] + s; }
  } else {
    s = blue * c_smits[W][i] + s;
    if (red <= green) { s = (red - blue) * c_smits[Ye][i] + s; s = (green - red) * c_smits[Gr][i] + s; }
    else { s = (green - blue) * c_smits[Ye][i] + s; s = (red - green) * c_smits[Re][i] + s; }
  }
  return s;
}
// f64::clamp (NaN stays NaN) and Rust `f as u32` (saturating, NaN -> 0).
__device__ __forceinline__ double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
__device__ __forceinline__ uint32_t sat_u32(double f) {
  if (!(f > 0.0)) return 0u;
  if (f >= 4294967295.0) return 0xFFFFFFFFu;
  return (uint32_t)f;
}

// `bin` = spectrum_bin(λ) of the path's wavelength (fixed along a path: computed once per sample).
template <bool EXT>
__device__ __forceinline__ double texture_value(const DevScene& S, uint32_t ti, int bin, V3 p, double hu = 0.0,
                                                double hv = 0.0) {
  const DevTexture& t = S.textures[ti];
  if (EXT && t.kind == YART_TEX_IMAGE) {  // ImageTexture::value texture.rs:320-344
    if (!t.pixels || t.width == 0 || t.height == 0) return 1.0;
    const double uu = clampd(hu, 0.0, 1.0), vv = 1.0 - clampd(hv, 0.0, 1.0);
    uint32_t i = sat_u32(uu * (double)t.width), j = sat_u32(vv * (double)t.height);
    if (i >= t.width) i = t.width - 1;
    if (j >= t.height) j = t.height - 1;
    const double color_scale = 1.0 / 255.0;
    const uint8_t* px = t.pixels + (size_t)j * t.width * 3 + (size_t)i * 3;
    return rgb_reflect(color_scale * (double)px[0], color_scale * (double)px[1], color_scale * (double)px[2], bin);
  }
  if (EXT && t.kind == YART_TEX_NOISE) {  // NoiseTexture::value texture.rs:265-300 (spec = RGB(1,1,1))
    const double white = t.spec[bin];
    if (t.noise_type == YART_NOISE_NET) return white * perlin_turb(t.perlin, t.noise_type, muls(p, t.scale), 7);
    if (t.noise_type == YART_NOISE_MARBLE)
      return white * 0.5 * (1.0 + sin_det(t.scale * p.z + 10.0 * perlin_turb(t.perlin, t.noise_type, p, 7)));
    return white * 0.5 * (1.0 + perlin_noise(t.perlin, t.noise_type, muls(p, t.scale)));
  }
  if (t.kind == YART_TEX_CHECKER) {  // texture.rs:58-67
    const double sines = sin_det(10.0 * p.x) * sin_det(10.0 * p.y) * sin_det(10.0 * p.z);
    return sines < 0.0 ? t.spec[bin] : t.spec_even[bin];
  }
  return t.spec[bin];
}
__device__ __forceinline__ V3 reflect(V3 v, V3 n) { return sub(v, smul(2.0 * dot(v, n), n)); }  // material.rs:75-77

// --------------------------------------------------------------------------- sampling
// The camera constants, read through an opaque kernarg-segment pointer at each use (scalar loads whose
// SGPRs live only in the camera block). Hoisted out of the render loop they held ~40 SGPRs for the
// whole kernel and were spilled to VGPR lanes: 22 v_readlane (VALU) per camera ray.
constexpr size_t kKernargCam = (sizeof(DevScene) + alignof(RenderArgs) - 1) / alignof(RenderArgs) * alignof(RenderArgs) +
                               offsetof(RenderArgs, cam);  // k_render(DevScene S, RenderArgs A): A.cam
typedef const __attribute__((address_space(4))) yart_camera* kcam_ptr;
__device__ __forceinline__ kcam_ptr kernarg_camera() {
  const __attribute__((address_space(4))) char* p =
      (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return (kcam_ptr)(p + kKernargCam);
}
__device__ __forceinline__ V3 ld3(const __attribute__((address_space(4))) double* p) { return mk(p[0], p[1], p[2]); }
// The render arguments the same way (YART_KA_OPAQUE, default on): each use re-reads its field by a
// scalar load from the kernarg segment, so no field of RenderArgs holds an SGPR across the render loop.
#ifndef YART_KA_OPAQUE
#define YART_KA_OPAQUE 1
#endif
typedef const __attribute__((address_space(4))) RenderArgs* kargs_ptr;
template <bool OPAQUE>
__device__ __forceinline__ kargs_ptr kernarg_args() {
  const __attribute__((address_space(4))) char* p =
      (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr();
  if (OPAQUE) asm volatile("" : "+s"(p));  // else a fixed address: loads are hoisted as for a plain parameter
  return (kargs_ptr)(p + (kKernargCam - offsetof(RenderArgs, cam)));
}

template <class Cam>
__device__ __forceinline__ Ray camera_ray(const Cam& c, double s, double t, double wl, Rng& g,
                                          bool draw_time) {  // camera.rs:82-94
  const V3 org = ld3(c.origin);
  const V3 d0 = sub(add(add(ld3(c.lower_left_corner), smul(s, ld3(c.horizontal))), smul(t, ld3(c.vertical))), org);
  Ray r;
  r.wl = wl;
  // Pinhole (lens_radius = 0, e.g. every aperture-0 preset) with no shutter-time draw: the disk
  // sample only reaches the ray as offset = u·(0·px) + v·(0·py) = ±0 per component, and no later
  // draw of phase 0 depends on how many values the rejection loop consumed. org + ±0 and d0 − ±0
  // are org and d0 whenever those components are non-zero, so the loop (and the Philox refill
  // its fourth and fifth draws trigger) is skipped exactly; a zero component takes the full path.
  if (c.lens_radius == 0.0 && !draw_time && org.x != 0.0 && org.y != 0.0 && org.z != 0.0 && d0.x != 0.0 &&
      d0.y != 0.0 && d0.z != 0.0) {
    r.o = org;
    r.d = d0;
    r.time = c.time0;
    return r;
  }
  V3 p;
  for (int guard = 0; guard < 1024; ++guard) {  // random_in_unit_disk camera.rs:25-33
    const double x = gen_range(g, -1.0, 1.0);
    const double y = gen_range(g, -1.0, 1.0);
    p = mk(x, y, 0.0);
    if (!(len2(p) >= 1.0)) break;
  }
  const V3 rd = smul(c.lens_radius, p);
  const V3 offset = add(muls(ld3(c.u), rd.x), muls(ld3(c.v), rd.y));
  r.o = add(org, offset);
  r.d = sub(d0, offset);
  // gen_range(time0..time1) (camera.rs:91): drawn only when a MovingSphere can read it
  r.time = draw_time ? gen_range(g, c.time0, c.time1) : c.time0;
  return r;
}

__device__ __forceinline__ bool covered(uint32_t x, uint32_t w) {  // main.rs:636-647 crop grid
  // w opaque: otherwise the 8 crop starts of each axis are hoisted out of the render loop as 16
  // loop-invariant SGPRs, which the list kernels spill to VGPR lanes for the whole kernel
  asm volatile("" : "+s"(w));
  const uint32_t cw = w / 8;
#pragma unroll
  for (uint32_t col = 0; col < 8; ++col) {
    const uint32_t x0 = (uint32_t)(((uint64_t)w * col) / 8);
    if (x >= x0 && x < x0 + cw) return true;
  }
  return false;
}

// Blocks b and b+8 are dealt to one XCD (MI355X_MICROARCH.md §Workgroup dispatch): give each XCD
// a contiguous run of pixel blocks so neighbouring tiles share that XCD's L2 (speed only).
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t n) {
  const uint32_t q = n / 8, r = n % 8, xcd = b % 8, k = b / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

// Waves per SIMD: 128 VGPRs -> 4 (+5 % over 3 on the cornell box; traversal is latency-bound:
// +36 % on david over 2, and 3 or 5 lose on every kernel).
constexpr int kWavesPerEu = 4;
constexpr int kMeshWavesPerEu = 4;

// Material::scatter at the stored hit + the mixture pdf (material.rs, main.rs:548-584): the path's
// next ray and throughput, or its end. One body for both math policies (the Fast cores first; a
// lane whose operand left a core's range re-runs it on the IEEE sequences from the same inputs
// and the same draws) and for both render paths (k_render's fused loop, k_wf_shade).
template <bool EXT, bool STATS, bool SHARE, class MP>
__device__ __forceinline__ void scatter_at(const DevScene& S, MP& mp, Rng& g, const V3& hp, const V3& hn, uint32_t hmat,
                                           double hu, double hv, int wbin, const Ray& ray, double T, uint32_t depth,
                                           Stats& st, double& T_, V3& o_, V3& d_, uint32_t& depth_, double& R_,
                                           bool& term_) {
  // o_ starts at the hit point, not the incoming ray's origin: only an ended path keeps the initial
  // value, and nothing reads its ray again; the origin then dies with the world pass that used it
  // instead of living (spilled) around the loop to here.
  T_ = T; o_ = hp; d_ = ray.d; depth_ = depth; R_ = 0.0; term_ = false;
  const DevMaterial& m = S.materials[hmat];
  const uint32_t kind = m.kind;
  if (kind == YART_MAT_LAMBERTIAN) {  // material.rs:44-61, main.rs:556-581
    // the albedo is looked up where it is multiplied in: fetched here, it was held (and
    // spilled) through the direction sampling and the light pdfs
    auto att = [&]() { return texture_value<EXT>(S, m.texture, wbin, hp, hu, hv); };
    const Onb uvw = onb_from_w(hn, mp);
    V3 dir, udir;  // the scattered direction and unit_vector(dir)
    double ldir;   // dir.length()
    double pdf_val;
    if (S.n_lights == 0) {
      (void)gen_range(g, 0.0, 1.0);  // MixurePDF(cos, cos): both branches sample the cosine
      dir = local(uvw, random_cosine_direction(g, mp));
      udir = mp.unit_len(dir, ldir);
      pdf_val = 0.5 * cosine_value<SHARE && !EXT>(uvw, udir, mp) + 0.5 * cosine_value<SHARE && !EXT>(uvw, udir, mp);
    } else {
      if (gen_range(g, 0.0, 1.0) < 0.5) {
        // HittableList::random (hittable.rs:113-122): 0..len-1 never picks the last light
        if (S.n_lights <= 2) {  // k = 0 for every lane (gen_index(g, 1) draws nothing): scalar loads
          dir = light_random(uniform_at(S.lights, 0u), hp, g, mp);
        } else {
          const uint32_t k = (uint32_t)gen_index(g, S.n_lights - 1);
          dir = light_random(S.lights[k], hp, g, mp);
        }
      } else {
        dir = local(uvw, random_cosine_direction(g, mp));
      }
      // hittable.rs:103-111 (formed on the host and read from the scene record instead, it cost david
      // 0.8 %: profiles/r06x_ab_devweight.log)
      const double weight = 1.0 / (double)S.n_lights;
      double sum = -0.0;
      // SHARE: unit_vector(dir) and its length once for the cosine pdf, the scatter pdf and a rect
      // light's pdf, which evaluated them separately (the compiler did not merge them): cornell
      // +2.1 %, random-scene +1.6 %; the mesh kernels keep the separate forms (david -0.7 %:
      // registers; profiles/r06w_ab_unit_reuse.log, r06x_ab_picore.log)
      if (SHARE) udir = mp.unit_len(dir, ldir);
      else ldir = 0.0;
      for (uint32_t i = 0; i < S.n_lights; ++i)
        sum = sum + weight * light_pdf<STATS, !SHARE>(uniform_at(S.lights, i), hp, dir, ldir, ray.wl, st, mp);
      if (!SHARE) udir = mp.unit(dir);
      pdf_val = 0.5 * sum + 0.5 * cosine_value<SHARE && !EXT>(uvw, udir, mp);
    }
    if (!isfinite(pdf_val) || pdf_val <= 0.0) {
      R_ = T * 0.0;  // Lambertian::emitted is 0 (material.rs:25-27)
      term_ = true;
    } else {
      const double cosine = dot(hn, SHARE ? udir : mp.unit(dir));  // Lambertian::scatter_pdf
      const double spdf = cosine < 0.0 ? 0.0 : over_pi<SHARE && !EXT>(cosine, mp);
      T_ = ((T * att()) * spdf) / pdf_val;
      o_ = hp;
      d_ = dir;
      depth_ = depth - 1;
    }
  } else if (EXT && kind == YART_MAT_ISOTROPIC) {  // material.rs:370-381: a specular-type scatter
    const double att = texture_value<EXT>(S, m.texture, wbin, hp, hu, hv);
    V3 p;
    for (int guard = 0; guard < 1024; ++guard) {  // random_in_unit_sphere material.rs:308-324
      const double px = gen_range(g, -1.0, 1.0), py = gen_range(g, -1.0, 1.0), pz = gen_range(g, -1.0, 1.0);
      p = mk(px, py, pz);
      if (!(len2(p) >= 1.0)) break;
    }
    T_ = T * att;
    o_ = hp;
    d_ = p;
    depth_ = depth - 1;
  } else if (kind == YART_MAT_METAL) {  // material.rs:79-95
    const V3 reflected = reflect(mp.unit(ray.d), hn);
    V3 p;
    for (int guard = 0; guard < 1024; ++guard) {  // random_in_unit_sphere material.rs:308-324
      const double px = gen_range(g, -1.0, 1.0), py = gen_range(g, -1.0, 1.0), pz = gen_range(g, -1.0, 1.0);
      p = mk(px, py, pz);
      if (!(len2(p) >= 1.0)) break;
    }
    const double att = texture_value<EXT>(S, m.texture, wbin, hp, hu, hv);
    T_ = T * att;
    o_ = hp;
    d_ = add(reflected, smul(m.fuzz, p));
    depth_ = depth - 1;
  } else {  // YART_MAT_DIELECTRIC, material.rs:213-301
    const double wl2 = ray.wl * ray.wl;
    const double n2 = 1.0 + m.b[0] * wl2 / (wl2 - m.c[0]) + m.b[1] * wl2 / (wl2 - m.c[1]) + m.b[2] * wl2 / (wl2 - m.c[2]);
    const double n = mp.sqrt(n2);
    // |d| divides the incidence cosine and, in unit_vector(d), the three components
    const PosDen ld = mp.den(mp.len(ray.d));
    V3 outward;
    double ni_over_nt, cosine;
    if (dot(ray.d, hn) > 0.0) {
      outward = neg(hn); ni_over_nt = n; cosine = mp.quo(n * dot(ray.d, hn), ld);
    } else {
      outward = hn; ni_over_nt = 1.0 / n; cosine = mp.quo(-dot(ray.d, hn), ld);
    }
    const V3 uv = mk(mp.quo(ray.d.x, ld), mp.quo(ray.d.y, ld), mp.quo(ray.d.z, ld));  // refract (material.rs:195-205)
    const double dt = dot(uv, outward);
    const double disc = 1.0 - ni_over_nt * ni_over_nt * (1.0 - dt * dt);
    V3 out;
    if (disc > 0.0) {
      const V3 refracted = sub(muls(sub(uv, muls(outward, dt)), ni_over_nt), muls(outward, mp.sqrt(disc)));
      double r0 = (1.0 - n) / (1.0 + n);  // schlick (material.rs:207-211)
      r0 = r0 * r0;
      const double sch = r0 + (1.0 - r0) * powi5(1.0 - cosine);
      out = gen_f64(g) < sch ? reflect(ray.d, hn) : refracted;
    } else {
      out = reflect(ray.d, hn);
    }
    T_ = T * 1.0;
    o_ = hp;
    d_ = out;
    depth_ = depth - 1;
  }
}

// DYN (chunked path only): the unit's 64 pixels x `chunk` samples form a job list that the wave's
// lanes pull from dynamically — a lane whose path ends takes the next (pixel, sample) job, the
// wave assigning consecutive job ids to the lanes that asked with one ballot + mbcnt prefix — so
// no lane idles while another still has samples of its own pixel left. Safe because each
// (pixel, sample) owns its RNG stream and its scratch slot; k_accumulate restores sample order.
// DEEP: a mesh deeper than depth 10 (DevScene::deep) — the walk stacks overflow into HBM (OVF above).
template <bool HAS_MESH, bool BVH, bool STATS, bool DYN, bool EXT, bool DEEP = false>
__global__ __launch_bounds__(256, HAS_MESH ? kMeshWavesPerEu : kWavesPerEu) void k_render(DevScene S, RenderArgs A_) {
  // The render arguments are read where used, through the opaque kernarg pointer (kernarg_args), in
  // the list and mesh kernels: SGPR spills of the chunked list kernel 45 -> 24, mesh 80 -> 54;
  // cornell 800x800x256 29.16 -> 28.84 ms, the mesh kernels +0.2-0.4 %. The world-BVH kernels keep
  // the hoisted form (random-scene -1.8 % opaque; profiles/r05_ab_covered_ka.log, r05_ab_ka256.log).
  // YART_KA_OPAQUE=0 builds the plain form everywhere.
#if YART_KA_OPAQUE
#define A (*kernarg_args<!BVH>())
#else
#define A A_
#endif
  __shared__ uint32_t s_stack[HAS_MESH ? 4 * kWaveLdsWords : BVH ? 4 * kStackSlots * 64 : 1];
  // JOBL (the chunked list and world-BVH kernels): a lane's job identity — pixel, sample, block, slot, x, y —
  // lives in LDS ([word][lane] per wave) from its hand-out to its scratch store, read where it is
  // used, instead of six VGPRs carried through every iteration.
  // The mesh kernel's LDS is nearly full (36.9 KB of walk state per workgroup): it keeps three
  // words (pixel, sample, block) and derives x, y and the slot from the pixel where needed.
  constexpr bool JOBL = DYN && !HAS_MESH, JOBL3 = DYN && HAS_MESH;
  // PARK (qbvh_coop): the persistent mesh kernel lets a walk whose wave ran out of rays stop and go on
  // at the next iteration, with the rays the other lanes bring; S.park (the busy-quad threshold, 0 =
  // off) is set for scenes with one mesh object.
  constexpr bool PARK = HAS_MESH && DYN && !EXT && !DEEP;
  __shared__ uint32_t s_job[JOBL ? 4 * 6 * 64 : JOBL3 ? 4 * 3 * 64 : 1];
  // the wave index through readfirstlane: uniform, so the per-wave LDS bases live in SGPRs (as a
  // VGPR the mesh walk's stack base was spilled and reloaded at every pop)
  const uint32_t lane = threadIdx.x & 63u, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // With the chunk count a multiple of 8 (capi.cpp plan()), each XCD's contiguous run of work ids
  // is whole chunks of every block: equal shares per XCD. (Without chunking the remap would give
  // one XCD all the expensive glass-sphere blocks: 1,960 vs 2,507 Msamples/s measured.)
  // DYN: persistent waves — the grid is one resident wave per slot, and each wave claims units
  // from A.queue (one atomic per unit) until they run out; the wave's lanes flow from one unit's
  // jobs into the next, so no wave drains a unit's last long paths with idle lanes.
  uint32_t work = DYN ? 0u : xcd_remap(blockIdx.x, gridDim.x) * 4 + wave;
  if (!DYN && work >= A.n_blocks * A.n_chunks) return;
  uint32_t local_blk = work % A.n_blocks, chunk_id = work / A.n_blocks;
  uint32_t b = A.shard_index + local_blk * A.shard_count;
  uint32_t bx0 = (b % A.blocks_x) * 8, by0 = (b / A.blocks_x) * 8;
  uint32_t slot = lane;  // pixel slot in the 8x8 block this lane is working on
  uint32_t x = bx0 + (slot & 7u), y = by0 + (slot >> 3);
  const uint32_t W = A.width, H = A.height;
  const bool active = x < W && y < H && covered(x, W) && covered(y, H);
  uint32_t* const jl = &s_job[JOBL ? wave * 6 * 64 + lane : JOBL3 ? wave * 3 * 64 + lane : 0];
  constexpr bool JL = JOBL || JOBL3;
  uint32_t* stk = &s_stack[HAS_MESH ? (wave * kWaveLdsWords + lane) : BVH ? (wave * kStackSlots * 64 + lane) : 0];
  uint8_t* coop = reinterpret_cast<uint8_t*>(&s_stack[HAS_MESH ? wave * kWaveLdsWords : 0]);
  // DEEP: this wave's HBM stack region (one per resident wave: the grid's waves, capi.cpp launch_frame)
  uint32_t* const ovf = (DEEP || PARK) ? A.stack_ovf + (size_t)(blockIdx.x * 4u + wave) * kOvfWords : nullptr;
  if (PARK) {  // no parked quads yet
    if (lane < 16u) reinterpret_cast<uint32_t*>(coop + coop_bytes<kCoopSlots>() + 64)[lane] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  Stats st;
  if (STATS) for (int i = 0; i < kNumStats; ++i) st.v[i] = 0;

  uint32_t pixel = y * W + x;
  double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
  const uint32_t s_end = A.s_begin + A.s_count;
  uint32_t s_lo = A.s_begin + chunk_id * A.chunk;
  const uint32_t s_stop = s_lo + A.chunk < s_end ? s_lo + A.chunk : s_end;
  uint32_t smp = s_lo;
  // scratch: [local_blk][sample - s_begin][slot][xyz]; DYN lanes keep their job's block
  uint32_t lane_blk = local_blk;
  uint32_t n_jobs = 0, next_job = 0;  // the wave's current unit (DYN, wave-uniform)
  uint64_t cov = 0;                   // DYN: the unit's block slots that are rendered (wave-uniform)
  bool drained = false;               // DYN: the queue has no units left (wave-uniform)
  bool need = true;                   // DYN: this lane wants a job
  bool parked = false;                // PARK: this lane's mesh walk stopped; the same ray again
  bool alive = DYN ? true : (active && smp < s_stop);
  Rng g;
  Ray ray;
  double T = 1.0;
  uint32_t depth = 0;
  bool fresh = !DYN && alive;  // start a sample at the top of the loop
  V3 hp = mk(0.0, 0.0, 0.0), hn = hp;  // the hit to scatter at the top of the next iteration
  uint32_t hmat = 0;
  double hu = 0.0, hv = 0.0;            // its texture coordinates (EXT)
  int wbin = 0;                         // spectrum bin of the path's wavelength
  g.k0 = (uint32_t)A.seed; g.k1 = (uint32_t)(A.seed >> 32);

  // The loop exits wave-uniformly: a lane without work stays in it with `run` false, so the
  // mesh walk (qbvh_coop) is reached by all 64 lanes together.
  for (;;) {
    if (DYN) {
      uint64_t m = drained ? 0ull : __ballot(need);
      while (m) {  // wave-uniform: hand out jobs until every asking lane has one
        if (next_job >= n_jobs) {  // claim the next unit
          const uint32_t first = (uint32_t)__builtin_ctzll(__ballot(true));
          uint32_t v = 0;
          if (lane == first) {
            if (HAS_MESH) {
              // XCD-local queues (mesh frames): workgroups are dealt to the 8 XCDs round-robin, so
              // XCD x takes the units of its own eighth of the frame first (its L2 then holds that
              // patch's mesh nodes), then steals from the others in turn; a partition is empty once
              // its counter passes its size, and every claim ends with a unit or after 8 tries.
              // Same-box A/B: david +1.5 %, bunny +1.9 %; the list walk (cornell -1.2 %) and the
              // world BVH (random-scene -0.2 %) keep the one counter (profiles/r05n_ab_xcd_queues.log).
              v = 0xFFFFFFFFu;
              const uint32_t x0 = blockIdx.x & 7u;
              for (uint32_t k = 0; k < 8u; ++k) {
                const uint32_t x = (x0 + k) & 7u;
                const uint32_t lo = (uint32_t)(((uint64_t)A.n_units * x) >> 3);
                const uint32_t hi = (uint32_t)(((uint64_t)A.n_units * (x + 1u)) >> 3);
                if (hi <= lo) continue;
                const uint32_t t = atomicAdd(A.queue + 1 + x, 1u);
                if (t < hi - lo) { v = lo + t; break; }
              }
              if (A.progress) {  // the units handed out so far, counted on queue[0]
                const uint32_t c = v < A.n_units ? atomicAdd(A.queue, 1u) + 1u : A.n_units;
                __hip_atomic_store(A.progress, A.progress_base + (c < A.n_units ? c : A.n_units), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
              }
            } else {
              v = atomicAdd(A.queue, 1u);
              if (A.progress)  // yart_render's progress: the units handed out so far (host-mapped word)
                __hip_atomic_store(A.progress, A.progress_base + (v < A.n_units ? v + 1u : A.n_units), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            }
          }
          const uint32_t u = (uint32_t)__builtin_amdgcn_readlane((int)v, (int)first);
          if (u >= A.n_units) { drained = true; break; }
          // block-major: a block's sample chunks are consecutive units, so the waves in flight
          // work on a compact patch of the frame (coherent camera rays and first hits, the same
          // mesh nodes in L2): bitwise the same, +0.6 % cornell, +1.5 % david, +1.9 % random-scene,
          // +4.2 % bunny over chunk-major (profiles/r05m_ab_unit_order.log)
          local_blk = u / A.n_chunks; chunk_id = u % A.n_chunks;
          b = A.shard_index + local_blk * A.shard_count;
          bx0 = (b % A.blocks_x) * 8; by0 = (b / A.blocks_x) * 8;
          s_lo = A.s_begin + chunk_id * A.chunk;
          const uint32_t stop = s_lo + A.chunk < s_end ? s_lo + A.chunk : s_end;
          n_jobs = (stop > s_lo ? stop - s_lo : 0) * 64;
          next_job = 0;
          {  // the block's pixels inside the frame and the crop grid (main.rs:636-647), once per unit
            const uint32_t cx = bx0 + (lane & 7u), cy = by0 + (lane >> 3);
            cov = __ballot(cx < W && cy < H && covered(cx, W) && covered(cy, H));
          }
          continue;
        }
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        const uint32_t avail = n_jobs - next_job;
        if (need && rank < avail) {
          const uint32_t job = next_job + rank;
          slot = job & 63u;
          smp = s_lo + (job >> 6);
          x = bx0 + (slot & 7u);
          y = by0 + (slot >> 3);
          pixel = y * W + x;
          lane_blk = local_blk;
          if (JOBL) { jl[0] = pixel; jl[64] = smp; jl[128] = lane_blk; jl[192] = slot; jl[256] = x; jl[320] = y; }
          if (JOBL3) { jl[0] = pixel; jl[64] = smp; jl[128] = lane_blk; }
          // a pixel outside the crop grid is skipped: the lane asks again
          if ((cov >> slot) & 1ull) { fresh = true; need = false; }
        }
        const uint32_t given = (uint32_t)__popcll(m);
        next_job += given < avail ? given : avail;
        m = __ballot(need);
      }
    }
    const bool run = DYN ? !need : alive;  // DYN: a lane still asking has found the queue drained
    if (__ballot(run) == 0) break;
    // T is the path's throughput while it runs and its result R (ray_reflectance's return value)
    // once it has ended (term): one register pair for both, since no lane needs both at once.
    bool term = false, want = PARK && parked;  // a parked lane's ray, T and depth are as they were
    if (STATS) {
      const uint64_t cam = __ballot(run && fresh), sca = __ballot(run && !fresh);
      if (lane == 0) {
        st.v[ST_ITERS]++;
        st.v[ST_CAMERA_LANES] += (uint32_t)__popcll(cam);
        st.v[ST_SCATTER_LANES] += (uint32_t)__popcll(sca);
        st.v[ST_CAMERA_ITERS] += cam ? 1u : 0u;
        st.v[ST_SCATTER_ITERS] += sca ? 1u : 0u;
      }
    }
    if (run && !(PARK && parked)) {
      // One Philox site per iteration for every lane: blocks 0-1 of this iteration's phase, the
      // camera ray of a fresh sample (phase 0) or the scatter of the hit the previous iteration
      // found (phase max_depth - depth + 1, its bounce level).
      rng_phase<!HAS_MESH && !BVH>(g, JL ? jl[0] : pixel, JL ? jl[64] : smp, fresh ? 0u : A.max_depth - depth + 1u);
      if (fresh) {  // main.rs:692-698
        uint32_t jx = x, jy = y;
        if (JOBL) { jx = jl[256]; jy = jl[320]; }
        if (JOBL3) { const uint32_t p = jl[0]; jy = p / W; jx = p - jy * W; }
        // W - 1 and H - 1 opaque here: hoisted, their f64 conversions held two VGPR pairs through the
        // whole loop (the mesh kernel spilled them)
        uint32_t wm1 = W - 1, hm1 = H - 1;
        asm volatile("" : "+s"(wm1), "+s"(hm1));
        const double tx = (double)jx + gen_f64(g);
        const double u = tx / (double)wm1;
        const double ty = (double)jy + gen_f64(g);
        const double v = 1.0 - ty / (double)hm1;
        const double wl = gen_range(g, kMinLambda, kMaxLambda);  // gen_wavelength color.rs:20-23
        ray = camera_ray(*kernarg_camera(), u, v, wl, g, EXT && S.has_time);
        wbin = spectrum_bin<!HAS_MESH && !EXT>(wl);  // the path's reflectance bin (color.rs:276-283), once per sample
        T = 1.0;
        depth = A.max_depth;
        fresh = false;
      } else {  // scatter at the stored hit (material.rs), main.rs:548-584
        // One body, two math policies: the Fast cores first; a lane with an operand outside a
        // core's range re-runs it on the IEEE sequences from the same inputs and the same draws.
        auto scatter = [&](auto& mp, double& T_, V3& o_, V3& d_, uint32_t& depth_, double& R_, bool& term_) {
          scatter_at<EXT, STATS, !HAS_MESH>(S, mp, g, hp, hn, hmat, hu, hv, wbin, ray, T, depth, st, T_, o_, d_, depth_, R_, term_);
        };
        double nT, nR;
        V3 no, nd;
        uint32_t ndepth;
        bool nterm;
        typename MathPolicy<HAS_MESH, BVH, EXT>::type fm;
        scatter(fm, nT, no, nd, ndepth, nR, nterm);
        if (flagged(fm)) {  // rare: the same draws again, on the IEEE sequences
          rng_phase<!HAS_MESH && !BVH>(g, JL ? jl[0] : pixel, JL ? jl[64] : smp, A.max_depth - depth + 1u);
          Ieee im;
          scatter(im, nT, no, nd, ndepth, nR, nterm);
        }
        T = nterm ? nR : nT; ray.o = no; ray.d = nd; depth = ndepth; term = nterm;
      }
      if (!term) {
        if (depth == 0) {  // main.rs:544-546: exhausted depth reflects 1.0
          T = T * 1.0;
          term = true;
        } else {
          want = true;
        }
      }
    }
    {
      Hit h;
      int32_t which;
      bool hit = false;
      bool scat = false;
      const QueryCtx q{g.k0, g.k1, JL ? jl[64] : smp, JL ? jl[0] : pixel, A.max_depth - depth + 1u};
      if (HAS_MESH) {  // converged: every lane, `want` says which have a ray
        bool now = false;
        hit = world_hit<HAS_MESH, BVH, STATS, EXT, kCoopSlots, DEEP, PARK>(S, want, ray, 0.001, INFINITY, h, which, stk, coop, st, q,
                                                                          ovf, parked, &now);
        if (PARK) {
          parked = now;
          want = want && !now;  // its hit is not known yet: nothing more for this lane in this iteration
        }
      } else if (want) {
        hit = world_hit<HAS_MESH, BVH, STATS, EXT>(S, true, ray, 0.001, INFINITY, h, which, stk, coop, st, q);
      }
      if (want && !term) {
        if (STATS) st.v[ST_SEGMENTS]++;
        if (!hit) {
          T = T * S.background[wbin];  // background_color.reflect (main.rs:587)
          term = true;
        } else {
          const DevMaterial& m = S.materials[h.mat];
          const uint32_t kind = m.kind;
          if (kind == YART_MAT_LAMBERTIAN || kind == YART_MAT_METAL || kind == YART_MAT_DIELECTRIC ||
              (EXT && kind == YART_MAT_ISOTROPIC)) {
            scat = true;  // scattered at the top of the next iteration
          } else {  // DiffuseLight emits on its front face; NoMaterial emits 0 (material.rs:347-355)
            double emitted = 0.0;
            if (kind == YART_MAT_DIFFUSE_LIGHT && h.ff) emitted = texture_value<EXT>(S, m.texture, wbin, h.p, h.u, h.v);
            T = T * emitted;
            term = true;
          }
        }
      }
      // The hit to scatter next is (re)defined for every lane here, 0 where none follows: assigned
      // only on the scatter path, it was live — and spilled — through every world pass, since the
      // compiler cannot see that a lane which did not keep a hit starts a fresh sample instead.
      hp = scat ? h.p : mk(0.0, 0.0, 0.0);
      hn = scat ? h.n : mk(0.0, 0.0, 0.0);
      hmat = scat ? h.mat : 0u;
      if (EXT) { hu = scat ? h.u : 0.0; hv = scat ? h.v : 0.0; }
    }
    if (run && term) {  // ray_color + sanitize_sample_xyz + += (main.rs:526-535, 448-459, 700-707)
      const double R = T;
      double cx, cy, cz;
      cie_xyz(ray.wl, cx, cy, cz);
      double sx = cx * R, sy = cy * R, sz = cz * R;
      if (!isfinite(sx) || !isfinite(sy) || !isfinite(sz)) {
        sx = sy = sz = 0.0;
      } else if (!(sy <= 0.0 || sy <= kMaxLum)) {
        const double k = kMaxLum / sy;
        sx = sx * k; sy = sy * k; sz = sz * k;
      }
      if (STATS) st.v[ST_SAMPLES]++;
      if (DYN) {  // chunked: k_accumulate adds the samples in order
        const uint32_t jb = JL ? jl[128] : lane_blk, js = JL ? jl[64] : smp;
        uint32_t jsl = JOBL ? jl[192] : slot;
        if (JOBL3) {  // the 8x8 blocks start at multiples of 8
          const uint32_t p = jl[0], py = p / W, px = p - py * W;
          jsl = (py & 7u) * 8u + (px & 7u);
        }
        double* q = A.scratch + 3 * (((size_t)jb * A.s_count + (js - A.s_begin)) * 64 + jsl);
        q[0] = sx; q[1] = sy; q[2] = sz;
        need = true;
      } else {
        acc0 = acc0 + sx; acc1 = acc1 + sy; acc2 = acc2 + sz;
        smp++;
        if (smp < s_stop) fresh = true;
        else alive = false;
      }
    }
  }
  if (!DYN && active) {
    double* o = A.out + 3 * (A.packed ? (size_t)local_blk * 64 + lane : (size_t)pixel);
    o[0] = acc0; o[1] = acc1; o[2] = acc2;
  }
  if (!DYN && A.progress && lane == 0) {  // units finished so far: a counter, whatever order waves end in
    const uint32_t done = atomicAdd(A.progress_count, 1u) + 1u;
    __hip_atomic_store(A.progress, A.progress_base + done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (STATS) {
    for (int i = 0; i < kNumStats; ++i)
      if (st.v[i]) atomicAdd(&A.stats[i], st.v[i]);
  }
}

#undef A
// ------------------------------------------------------------- wavefront path (mesh scenes)
// The megakernel's loop split at the world query. k_wf_shade does, for
// every path of the pool, what k_render does around the query: the record of the hit the last
// trace found, the material's scatter (or the path's end: background, emission, depth 0) and,
// for a path that ended, the scratch store of its sample and the camera ray of the next job; the
// paths that have a ray to trace are appended to the next queue with one atomic per wave (ballot
// + mbcnt). k_wf_trace then walks the world for the queued rays alone — the cooperative QBVH walk
// with nothing else live, so it runs without the megakernel's register spills. Every draw is keyed
// by (pixel, sample, phase) and every sample has its own scratch slot, so the split changes the
// order work is done in and nothing else: the sums are bitwise the megakernel's (k_accumulate adds
// the samples in order).

// job = (local block * s_count + sample - s_begin) * 64 + slot, which is also its scratch index
__device__ __forceinline__ void wf_job(const RenderArgs& A, uint32_t job, uint32_t& pixel, uint32_t& smp, uint32_t& x,
                                       uint32_t& y) {
  const uint32_t slot = job & 63u, rest = job >> 6;
  const uint32_t blk = rest / A.s_count, s = rest - blk * A.s_count;
  const uint32_t b = A.shard_index + blk * A.shard_count;
  x = (b % A.blocks_x) * 8u + (slot & 7u);
  y = (b / A.blocks_x) * 8u + (slot >> 3);
  pixel = y * A.width + x;
  smp = A.s_begin + s;
}
// ray_color + sanitize_sample_xyz (main.rs:526-535, 448-459) into the sample's scratch slot
__device__ __forceinline__ void wf_store_sample(const RenderArgs& A, uint32_t job, double wl, double R) {
  double cx, cy, cz;
  cie_xyz(wl, cx, cy, cz);
  double sx = cx * R, sy = cy * R, sz = cz * R;
  if (!isfinite(sx) || !isfinite(sy) || !isfinite(sz)) {
    sx = sy = sz = 0.0;
  } else if (!(sy <= 0.0 || sy <= kMaxLum)) {
    const double k = kMaxLum / sy;
    sx = sx * k; sy = sy * k; sz = sz * k;
  }
  double* q = A.scratch + 3 * (size_t)job;
  q[0] = sx; q[1] = sy; q[2] = sz;
}

__global__ __launch_bounds__(256) void k_wf_shade(DevScene S, RenderArgs A, WfArgs F) {
  __shared__ uint32_t s_need[4], s_take[3];
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t P = F.pool;
  const uint32_t W = A.width, H = A.height;
  const WfSlots& Q = F.q;
  Stats st;
  Rng g;
  g.k0 = (uint32_t)A.seed; g.k1 = (uint32_t)(A.seed >> 32);
  Ray ray;
  ray.time = 0.0;  // no MovingSphere on this path (EXT scenes keep the megakernel)
  ray.wl = 0.0;
  ray.o = mk(0.0, 0.0, 0.0); ray.d = ray.o;
  double T = 0.0;
  uint32_t job = Q.job[i], depth = 0;
  bool has = false;  // a ray to trace next
  if (job != kWfNoJob) {  // the path traced last iteration: its hit (main.rs:548-587)
    depth = Q.depth[i]; T = Q.T[i]; ray.wl = Q.wl[i];
    ray.o = mk(Q.o[i], Q.o[P + i], Q.o[2 * (size_t)P + i]);
    ray.d = mk(Q.d[i], Q.d[P + i], Q.d[2 * (size_t)P + i]);
    const int wbin = spectrum_bin<false>(ray.wl);
    const uint32_t obj = Q.hobj[i];
    double R = 0.0;
    bool term = false;
    if (obj == kWfMiss) {
      R = T * S.background[wbin];  // background_color.reflect (main.rs:587)
      term = true;
    } else {
      HitId id;
      id.t = Q.ht[i]; id.u = Q.hu[i]; id.v = Q.hv[i]; id.obj = obj; id.sub = Q.hsub[i];
      Hit h;
      hit_record<true, false>(S, ray, id, h);
      const DevMaterial& m = S.materials[h.mat];
      const uint32_t kind = m.kind;
      if (kind == YART_MAT_LAMBERTIAN || kind == YART_MAT_METAL || kind == YART_MAT_DIELECTRIC) {
        uint32_t pixel, smp, x, y;
        wf_job(A, job, pixel, smp, x, y);
        rng_phase<false>(g, pixel, smp, A.max_depth - depth + 1u);
        double nT, nR;
        V3 no, nd;
        uint32_t ndepth;
        bool nterm;
        Ieee im;
        scatter_at<false, false, false>(S, im, g, h.p, h.n, h.mat, 0.0, 0.0, wbin, ray, T, depth, st, nT, no, nd, ndepth, nR, nterm);
        if (nterm) {
          R = nR;
          term = true;
        } else if (ndepth == 0) {  // main.rs:544-546: exhausted depth reflects 1.0
          R = nT * 1.0;
          term = true;
        } else {
          T = nT; ray.o = no; ray.d = nd; depth = ndepth;
          has = true;
        }
      } else {  // DiffuseLight emits on its front face; NoMaterial emits 0 (material.rs:347-355)
        double emitted = 0.0;
        if (kind == YART_MAT_DIFFUSE_LIGHT && h.ff) emitted = texture_value<false>(S, m.texture, wbin, h.p);
        R = T * emitted;
        term = true;
      }
    }
    if (term) wf_store_sample(A, job, ray.wl, R);
  }
  // A slot without a ray (its path ended, or the slot is new) starts the pass's next job. The
  // workgroup hands out consecutive job ids from its own range [next, end) and claims a fresh
  // chunk of kWfChunk with ONE atomic when the range runs dry (one atomic per 256 jobs instead of
  // one per wave and iteration: same-address atomics from every CU were the pass's bottleneck).
  // Pixels outside the crop grid (main.rs:636-647) and samples that end at once (max_depth 0)
  // make the lane ask again.
  bool need = !has;
  uint32_t next = 0, end = 0;
  if (threadIdx.x == 0) { next = Q.range[2 * blockIdx.x]; end = Q.range[2 * blockIdx.x + 1]; }
  for (;;) {
    if (!__syncthreads_or(need)) break;
    const uint64_t m = __ballot(need);
    if (lane == 0) s_need[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    const uint32_t total = s_need[0] + s_need[1] + s_need[2] + s_need[3];
    uint32_t before = 0;
    for (uint32_t w = 0; w < wave; ++w) before += s_need[w];
    if (threadIdx.x == 0) {  // [next, end), then a fresh chunk [base, base + kWfChunk) if needed
      uint32_t base = kWfNoJob;
      if (end - next < total && *(volatile uint32_t*)F.jobs < F.total_jobs) {
        base = atomicAdd(F.jobs, kWfChunk);
        if (base >= F.total_jobs) base = kWfNoJob;
      }
      s_take[0] = next; s_take[1] = base;
      const uint32_t rem = end - next;
      if (base != kWfNoJob) {
        next = base + (total - rem);
        end = base + kWfChunk < F.total_jobs ? base + kWfChunk : F.total_jobs;
        if (next > end) next = end;
      } else {
        next += rem < total ? rem : total;
      }
      s_take[2] = rem;
    }
    __syncthreads();
    const uint32_t from = s_take[0], base = s_take[1], rem = s_take[2];
    const bool dry = base == kWfNoJob && rem < total;  // some lanes go without: the pass is out of jobs
    if (need) {
      const uint32_t r = before + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      uint32_t jb = kWfNoJob;
      if (r < rem) jb = from + r;
      else if (base != kWfNoJob && base + (r - rem) < F.total_jobs) jb = base + (r - rem);
      if (jb == kWfNoJob) {
        need = false;
        job = kWfNoJob;
      } else {
        uint32_t pixel, smp, x, y;
        wf_job(A, jb, pixel, smp, x, y);
        if (x < W && y < H && covered(x, W) && covered(y, H)) {  // main.rs:692-698
          job = jb;
          rng_phase<false>(g, pixel, smp, 0u);
          const double tx = (double)x + gen_f64(g);
          const double u = tx / (double)(W - 1);
          const double ty = (double)y + gen_f64(g);
          const double v = 1.0 - ty / (double)(H - 1);
          const double wl = gen_range(g, kMinLambda, kMaxLambda);  // gen_wavelength color.rs:20-23
          ray = camera_ray(*kernarg_camera(), u, v, wl, g, false);
          ray.time = 0.0;
          T = 1.0;
          depth = A.max_depth;
          if (depth == 0) {
            wf_store_sample(A, job, ray.wl, T * 1.0);
          } else {
            has = true;
            need = false;
          }
        }
      }
    }
    if (dry) {  // every lane still asking goes without
      need = false;
      if (!has) job = kWfNoJob;
    }
    __syncthreads();  // s_need / s_take are rewritten next round
  }
  if (threadIdx.x == 0) { Q.range[2 * blockIdx.x] = next; Q.range[2 * blockIdx.x + 1] = end; }
  // the path stays in its slot: the traced ray, or an empty slot
  Q.job[i] = has ? job : kWfNoJob;
  if (has) {
    Q.o[i] = ray.o.x; Q.o[P + i] = ray.o.y; Q.o[2 * (size_t)P + i] = ray.o.z;
    Q.d[i] = ray.d.x; Q.d[P + i] = ray.d.y; Q.d[2 * (size_t)P + i] = ray.d.z;
    Q.T[i] = T; Q.wl[i] = ray.wl; Q.depth[i] = depth;
  }
  if (__syncthreads_or(has) && threadIdx.x == 0) *F.alive = 1u;
}

constexpr int kWfTraceWaves = 4;  // LDS-bound: the cooperative walk's 9.2 KB per wave
// One wave per workgroup: a wave that finishes frees its slot (LDS included) for the next one
// without waiting for slower waves of a larger workgroup.
template <int SLOTS>
__global__ __launch_bounds__(64, SLOTS == kCoopSlots ? kWfTraceWaves : 3) void k_wf_trace(DevScene S, RenderArgs A,
                                                                                            WfArgs F) {
  constexpr int kWords = wave_lds_words<SLOTS>();
  __shared__ uint32_t s_stack[kWords];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const uint32_t v = *F.alive;
    *F.alive_next = 0u;  // the next iteration's flag (nothing reads it before the next shade)
    __hip_atomic_store(F.status, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const uint32_t lane = threadIdx.x, P = F.pool;
  uint32_t* stk = &s_stack[lane];
  uint8_t* coop = reinterpret_cast<uint8_t*>(&s_stack[0]);
  // one batch of 64 slots per wave (a resident grid walking every gridDim-th batch was 11-14 %
  // slower)
  for (uint32_t bt = blockIdx.x; bt < P / 64u; bt += P) {
    const uint32_t i = bt * 64u + lane;
    const bool want = F.q.job[i] != kWfNoJob;
    if (__ballot(want) == 0) continue;  // wave-uniform: the walk needs the whole wave
    Ray r;
    r.o = mk(F.q.o[i], F.q.o[P + i], F.q.o[2 * (size_t)P + i]);
    r.d = mk(F.q.d[i], F.q.d[P + i], F.q.d[2 * (size_t)P + i]);
    r.time = 0.0; r.wl = 0.0;
    HitId id;
    Stats st;
    const QueryCtx q{0u, 0u, 0u, 0u, 0u};  // no media on this path
    const bool hit = world_closest<true, false, false, SLOTS>(S, want, r, 0.001, INFINITY, id, stk, coop, st, q);
    if (want) {
      F.q.ht[i] = id.t; F.q.hu[i] = id.u; F.q.hv[i] = id.v;
      F.q.hobj[i] = hit ? id.obj : kWfMiss;
      F.q.hsub[i] = id.sub;
    }
  }
}

// Chunked path, second kernel: pixel += sample for every sample of the pass, in sample order
// (main.rs:707), so the sums are bitwise those of the fused loop. HBM-bound (24 B per sample).
__global__ __launch_bounds__(256) void k_accumulate(RenderArgs A, int first_pass) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n_blocks * 64) return;
  const uint32_t local_blk = i >> 6, lane = i & 63u;
  const uint32_t b = A.shard_index + local_blk * A.shard_count;
  const uint32_t x = (b % A.blocks_x) * 8 + (lane & 7u), y = (b / A.blocks_x) * 8 + (lane >> 3);
  if (!(x < A.width && y < A.height && covered(x, A.width) && covered(y, A.height))) return;
  double* o = A.out + 3 * (A.packed ? (size_t)i : (size_t)y * A.width + x);
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  if (!first_pass) { a0 = o[0]; a1 = o[1]; a2 = o[2]; }
  const double* q = A.scratch + 3 * ((size_t)local_blk * A.s_count * 64 + lane);
#pragma unroll 8
  for (uint32_t s = 0; s < A.s_count; ++s) {
    a0 = a0 + q[0]; a1 = a1 + q[1]; a2 = a2 + q[2];
    q += 64 * 3;
  }
  o[0] = a0; o[1] = a1; o[2] = a2;
}

// Root side of the frame gather (yart_gather_frame_async): every shard's block-packed pixels,
// shard r at recv + r * stride, back into the W x H frame; pixel (x, y) lives in global block
// b = (y / 8) * ceil(W / 8) + x / 8, i.e. shard b % N, local block b / N, slot (y % 8) * 8 + x % 8.
// Writes every pixel (0 outside the crop grid), so the frame needs no clearing.
__global__ __launch_bounds__(256) void k_unpack_shards(const double* __restrict__ recv, uint32_t shards, size_t stride,
                                                       uint32_t w, uint32_t h, double* __restrict__ frame) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w * h) return;
  const uint32_t x = i % w, y = i / w;
  double v0 = 0.0, v1 = 0.0, v2 = 0.0;
  if (covered(x, w) && covered(y, h)) {
    const uint32_t b = (y >> 3) * ((w + 7u) >> 3) + (x >> 3);
    const double* q = recv + (size_t)(b % shards) * stride + 3 * ((size_t)(b / shards) * 64 + (y & 7u) * 8 + (x & 7u));
    v0 = q[0]; v1 = q[1]; v2 = q[2];
  }
  double* o = frame + 3 * (size_t)i;
  o[0] = v0; o[1] = v1; o[2] = v2;
}

// ------------------------------------------------------------------- batched closest hit
template <int SLOTS>
__global__ __launch_bounds__(256, SLOTS == kCoopSlots ? kMeshWavesPerEu : 3) void k_intersect(DevScene S, const double* __restrict__ rays, uint32_t n,
                                                   double* __restrict__ hits, int32_t* __restrict__ obj) {
  constexpr int kWords = wave_lds_words<SLOTS>();
  __shared__ uint32_t s_stack[4 * kWords];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const bool active = i < n;  // no early exit: the mesh walk needs the whole wave
  const double* q = rays + 8 * (size_t)(active ? i : 0);
  Ray r{mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), 0.0, 0.0};
  Hit h;
  int32_t which = -1;
  Stats st;
  uint32_t* stk = &s_stack[wave * kWords + lane];
  uint8_t* coop = reinterpret_cast<uint8_t*>(&s_stack[wave * kWords]);
  const QueryCtx qc{0u, 0u, 0u, i, 0u};  // a medium's draw for query i: seed 0, sample 0, pixel i
  bool hit = false;
  if (S.world_nodes) {
    if (active) hit = world_hit<false, true, false, false>(S, true, r, q[6], q[7], h, which, stk, coop, st, qc);
  } else {
    hit = world_hit<true, false, false, true, SLOTS>(S, active, r, q[6], q[7], h, which, stk, coop, st, qc);
  }
  if (!active) return;
  double* o = hits + 8 * (size_t)i;
  if (hit) {
    o[0] = h.t; o[1] = h.p.x; o[2] = h.p.y; o[3] = h.p.z;
    o[4] = h.n.x; o[5] = h.n.y; o[6] = h.n.z; o[7] = h.ff ? 1.0 : 0.0;
  } else {
    for (int k = 0; k < 8; ++k) o[k] = NAN;
  }
  obj[i] = which;
}

// ------------------------------------------------------------------------ finalize
// gamma_corrected (color.rs:93-101) then clamp_display_channel (main.rs:461-463) is a monotone step
// function of the linear channel, so it is its 255 steps: X_k = the least double whose byte is >= k,
// derived with glibc's pow — the function the reference's f64::powf calls — by
// tools/gen_srgb_steps.py. The byte is the count of steps at or below the value: the reference's
// byte for every double (NaN and values <= 0 count none, +inf all 255), with no vendor pow, whose
// last ulp differs from glibc's (tests/test_finalize_bytes.py checks every double within 4096 ulps
// of every step). Branchless binary search: 8 compares.
__constant__ double c_srgb_steps[255] =
#include "srgb_steps.inc"
    ;  // one brace-enclosed row of 255 hex floats
__device__ __forceinline__ uint8_t srgb_byte(double linear) {
  uint32_t n = 0;
#pragma unroll
  for (uint32_t s = 128; s != 0; s >>= 1)
    if (linear >= c_srgb_steps[n + s - 1]) n += s;
  return (uint8_t)n;
}
__global__ __launch_bounds__(256) void k_finalize(const double* __restrict__ xyz, uint32_t w, uint32_t h, uint32_t spp,
                                                  uint8_t* __restrict__ rgba) {  // main.rs:710-718
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w * h) return;
  const uint32_t x = i % w, y = i / w;
  uchar4 out = make_uchar4(0, 0, 0, 0);
  if (covered(x, w) && covered(y, h)) {
    V3 v = mk(xyz[3 * (size_t)i], xyz[3 * (size_t)i + 1], xyz[3 * (size_t)i + 2]);
    v = divs(muls(v, kMaxLambda - kMinLambda), kCieYIntegral * (double)spp);
    const double r = 2.6896552 * v.x - 1.2758621 * v.y - 0.4137931 * v.z;  // XYZ::into_rgb color.rs:209-213
    const double gg = -1.0221082 * v.x + 1.9782866 * v.y + 0.0438216 * v.z;
    const double b = 0.0612245 * v.x - 0.2244898 * v.y + 1.1632653 * v.z;
    out = make_uchar4(srgb_byte(r), srgb_byte(gg), srgb_byte(b), 255);
  }
  reinterpret_cast<uchar4*>(rgba)[i] = out;
}

// --------------------------------------------------------------------------- probes
__global__ void k_probe_rng(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, double* out) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  Rng g;
  rng_init(g, seed, pixel, sample, 0);
  for (uint32_t i = 0; i < n; ++i) out[i] = gen_f64(g);
}
__global__ void k_probe_math(int op, const double* a, const double* b, uint32_t n, double* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s, c;
  switch (op) {
    case 0: out[i] = sqrt(a[i]); break;
    case 1: out[i] = a[i] / b[i]; break;
    case 2: sincos_det(a[i], s, c); out[i] = s; break;
    case 3: sincos_det(a[i], s, c); out[i] = c; break;
    case 5: out[i] = log_det(a[i]); break;
    case 6: out[i] = acos_det(a[i]); break;
    case 7: out[i] = atan2_det(a[i], b[i]); break;
    // 8-10: the Fast policy's cores where its checks pass, the IEEE sequence where they flag —
    // what a Fast block followed by its Ieee re-run produces
    case 8: { Fast m; const double v = m.sqrt(a[i]); out[i] = m.bad ? sqrt(a[i]) : v; break; }
    case 9:  // a = n/3 vectors; out = unit(a_i)
      if (3 * i + 2 < n) {
        const V3 in = mk(a[3 * i], a[3 * i + 1], a[3 * i + 2]);
        Fast m;
        V3 u = m.unit(in);
        if (m.bad) u = unit(in);
        out[3 * i] = u.x; out[3 * i + 1] = u.y; out[3 * i + 2] = u.z;
      }
      break;
    case 10: {  // a = n/3 triples over b_i > 0
      if (3 * i + 2 < n) {
        Fast m;
        const PosDen d = m.den(b[i]);
        const double x = m.quo(a[3 * i], d), y = m.quo(a[3 * i + 1], d), z = m.quo(a[3 * i + 2], d);
        out[3 * i] = m.bad ? a[3 * i] / b[i] : x;
        out[3 * i + 1] = m.bad ? a[3 * i + 1] / b[i] : y;
        out[3 * i + 2] = m.bad ? a[3 * i + 2] / b[i] : z;
      }
      break;
    }
    case 11: out[i] = (double)srgb_byte(a[i]); break;
    default: out[i] = pow(a[i], b[i]); break;
  }
}

// ------------------------------------------------------------------------- launchers
hipError_t launch_accumulate(const RenderArgs& a, bool first_pass, hipStream_t stream) {
  const uint32_t n = a.n_blocks * 64;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_accumulate, dim3((n + 255) / 256), dim3(256), 0, stream, a, first_pass ? 1 : 0);
  return hipGetLastError();
}
hipError_t launch_render(const DevScene& s, const RenderArgs& a, bool stats, hipStream_t stream) {
  const bool dyn = a.scratch != nullptr;  // stats launches follow the same plan (r06: they were fused)
  const uint32_t units = a.n_blocks * a.n_chunks;
  const uint32_t grid = ((dyn && a.waves < units ? a.waves : units) + 3) / 4;
  if (grid == 0) return hipSuccess;
#define YART_LAUNCH(MESH, BVH, EXT)                                                                            \
  do {                                                                                                        \
    if (stats && dyn) hipLaunchKernelGGL((k_render<MESH, BVH, true, true, EXT>), dim3(grid), dim3(256), 0, stream, s, a); \
    else if (stats) hipLaunchKernelGGL((k_render<MESH, BVH, true, false, EXT>), dim3(grid), dim3(256), 0, stream, s, a);  \
    else if (dyn) hipLaunchKernelGGL((k_render<MESH, BVH, false, true, EXT>), dim3(grid), dim3(256), 0, stream, s, a); \
    else hipLaunchKernelGGL((k_render<MESH, BVH, false, false, EXT>), dim3(grid), dim3(256), 0, stream, s, a);        \
  } while (0)
  if (s.has_mesh && s.deep && !s.has_ext) {  // deep meshes: stacks overflow into a.stack_ovf (capi.cpp)
    if (!a.stack_ovf) return hipErrorInvalidValue;
    if (stats && dyn) hipLaunchKernelGGL((k_render<true, false, true, true, false, true>), dim3(grid), dim3(256), 0, stream, s, a);
    else if (stats) hipLaunchKernelGGL((k_render<true, false, true, false, false, true>), dim3(grid), dim3(256), 0, stream, s, a);
    else if (dyn) hipLaunchKernelGGL((k_render<true, false, false, true, false, true>), dim3(grid), dim3(256), 0, stream, s, a);
    else hipLaunchKernelGGL((k_render<true, false, false, false, false, true>), dim3(grid), dim3(256), 0, stream, s, a);
  } else if (s.has_mesh) {
    if (s.park && dyn && !a.stack_ovf) return hipErrorInvalidValue;  // PARK: the re-walk's HBM stacks
    if (s.has_ext) YART_LAUNCH(true, false, true); else YART_LAUNCH(true, false, false);
  } else if (s.world_nodes) {
    if (s.has_ext) YART_LAUNCH(false, true, true); else YART_LAUNCH(false, true, false);  // noise textures only
  } else {
    if (s.has_ext) YART_LAUNCH(false, false, true); else YART_LAUNCH(false, false, false);
  }
#undef YART_LAUNCH
  return hipGetLastError();
}
hipError_t launch_wf_shade(const DevScene& s, const RenderArgs& a, const WfArgs& w, hipStream_t stream) {
  hipLaunchKernelGGL(k_wf_shade, dim3(w.pool / 256), dim3(256), 0, stream, s, a, w);
  return hipGetLastError();
}
hipError_t launch_wf_trace(const DevScene& s, const RenderArgs& a, const WfArgs& w, hipStream_t stream) {
  const uint32_t batches = w.pool / 64;
  const uint32_t grid = batches;
  if (s.deep) hipLaunchKernelGGL(k_wf_trace<kDeepSlots>, dim3(grid), dim3(64), 0, stream, s, a, w);
  else hipLaunchKernelGGL(k_wf_trace<kCoopSlots>, dim3(grid), dim3(64), 0, stream, s, a, w);
  return hipGetLastError();
}
hipError_t launch_unpack_shards(const double* recv, uint32_t shards, size_t stride, uint32_t w, uint32_t h, double* frame,
                                hipStream_t stream) {
  const uint32_t n = w * h;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_unpack_shards, dim3((n + 255) / 256), dim3(256), 0, stream, recv, shards, stride, w, h, frame);
  return hipGetLastError();
}
hipError_t launch_intersect(const DevScene& s, const double* rays, uint32_t n, double* hits, int32_t* obj,
                            hipStream_t stream) {
  if (n == 0) return hipSuccess;
  if (s.deep) hipLaunchKernelGGL(k_intersect<kDeepSlots>, dim3((n + 255) / 256), dim3(256), 0, stream, s, rays, n, hits, obj);
  else hipLaunchKernelGGL(k_intersect<kCoopSlots>, dim3((n + 255) / 256), dim3(256), 0, stream, s, rays, n, hits, obj);
  return hipGetLastError();
}
hipError_t launch_finalize(const double* xyz, uint32_t w, uint32_t h, uint32_t spp, uint8_t* rgba, hipStream_t stream) {
  const uint32_t n = w * h;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_finalize, dim3((n + 255) / 256), dim3(256), 0, stream, xyz, w, h, spp, rgba);
  return hipGetLastError();
}
hipError_t launch_probe_rng(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(k_probe_rng, dim3(1), dim3(64), 0, stream, seed, pixel, sample, n, out);
  return hipGetLastError();
}
hipError_t launch_probe_math(int op, const double* a, const double* b, uint32_t n, double* out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_probe_math, dim3((n + 255) / 256), dim3(256), 0, stream, op, a, b, n, out);
  return hipGetLastError();
}

}  // namespace yart_dev

extern "C" int yart_debug_force_rewalk(int device, int on) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  const uint32_t v = on ? 1u : 0u;
  return hipMemcpyToSymbol(HIP_SYMBOL(yart_dev::g_force_rewalk), &v, sizeof v) == hipSuccess ? 0 : -1;
}

#ifdef YART_WALK_CHECK
extern "C" int yart_debug_walk_fault(int device, unsigned int* out) {  // reads and clears the fault bits
  if (hipSetDevice(device) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(yart_dev::g_walk_fault), sizeof(unsigned int)) != hipSuccess) return -1;
  const unsigned int z = 0;
  return hipMemcpyToSymbol(HIP_SYMBOL(yart_dev::g_walk_fault), &z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif
