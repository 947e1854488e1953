/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Scalar f64 restatement of themayflyman/yet-another-raytracer's per-pixel-sample hot path.
 * Every function cites the reference file:line it follows (paths relative to
 * raytracer/src/). Built with -ffp-contract=off so that, like the reference (rustc never
 * contracts), every operation rounds on its own. Expression order follows the Rust source
 * (left-associative + and -).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ------------------------------------------------------------------ constants (color.rs) */
static const double MIN_LAMBDA = 360.0;        /* color.rs:7  */
static const double MAX_LAMBDA = 720.0;        /* color.rs:8  */
static const double BIN_WIDTH = 10.0;          /* color.rs:9  */
#define BIN_COUNT 36                           /* color.rs:10 */
#define N_CIE_SAMPLES 471                      /* color.rs:11 */
static const double CIE_Y_INTERGAL = 106.856895; /* color.rs:12 */
static const double MAX_SAMPLE_LUMINANCE = 20.0; /* main.rs:59  */
static const double PI = 3.141592653589793;    /* std::f64::consts::PI */
static const double F64_EPSILON = 2.220446049250313e-16; /* f64::EPSILON */

/* CIE 1931 at 1 nm, rows (x, y, z), color.rs:286-1709 (generated from tables/). */
static const double CIE_XYZ[N_CIE_SAMPLES][3] = {
#include "cie_xyz.inc"
};
/* Smits basis spectra, color.rs:1711-1982: white, cyan, magenta, yellow, red, green, blue. */
static const double SMITS[7][BIN_COUNT] = {
#include "smits.inc"
};
enum { S_WHITE, S_CYAN, S_MAGENTA, S_YELLOW, S_RED, S_GREEN, S_BLUE };

/* ---------------------------------------------------------------------- Vec3 (vec3.rs) */
typedef struct { double x, y, z; } v3;
static inline v3 V(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); } /* vec3.rs:47-60 */
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); } /* vec3.rs:69-77 */
static inline v3 vmuls(v3 a, double s) { return V(a.x * s, a.y * s, a.z * s); } /* vec3.rs:89-97 */
static inline v3 smulv(double s, v3 a) { return V(s * a.x, s * a.y, s * a.z); } /* vec3.rs:99-107 */
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }                      /* vec3.rs:124-132 */
/* Div<f64>: a zero divisor yields f64::MAX in every lane (vec3.rs:109-122). */
static inline v3 vdivs(v3 a, double s) {
  if (s == 0.0) return V(1.7976931348623157e308, 1.7976931348623157e308, 1.7976931348623157e308);
  return V(a.x / s, a.y / s, a.z / s);
}
static inline double dot(v3 a, v3 b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); } /* vec3.rs:221-223 */
static inline v3 cross(v3 a, v3 b) {                                                   /* vec3.rs:225-233 */
  return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline double length_squared(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; } /* vec3.rs:199-201 */
static inline double length(v3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }   /* vec3.rs:195-197 */
static inline v3 unit_vector(v3 a) {                                                    /* vec3.rs:203-211 */
  return V(a.x / length(a), a.y / length(a), a.z / length(a));
}
static inline double comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

typedef struct { v3 o, d; double time, wl; } ray_t; /* ray.rs:3-9 */
static inline v3 ray_at(const ray_t* r, double t) { return vadd(r->o, smulv(t, r->d)); } /* ray.rs:33-35 */

/* ------------------------------------------------------------- deterministic sin / cos
 * The reference calls libm (f64::sin/cos). To make the device and this checker agree bit for
 * bit, both use this fdlibm-style kernel (Cody-Waite pi/2 reduction in two steps + the
 * __kernel_sin/__kernel_cos minimax polynomials) built from + - * / only. It is within 1 ulp
 * of glibc (tests/test_oracle_math.py measures it). */
static const double INV_PIO2 = 6.36619772367581382433e-01;
static const double PIO2_1 = 1.57079632673412561417e+00;  /* first 33 bits of pi/2 */
static const double PIO2_2 = 6.07710050630396597660e-11;  /* second 33 bits */
static const double PIO2_2T = 2.02226624879595063154e-21; /* pi/2 - (PIO2_1 + PIO2_2) */
static inline void rem_pio2(double x, int* q, double* y0, double* y1) {
  double fn = floor(x * INV_PIO2 + 0.5);
  double t = x - fn * PIO2_1;
  double w = fn * PIO2_2;
  double r = t - w;
  w = fn * PIO2_2T - ((t - r) - w);
  *y0 = r - w;
  *y1 = (r - *y0) - w;
  *q = (int)((long long)fn & 3);
}
static inline double k_sin(double x, double y) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x, v = z * x;
  double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
static inline double k_cos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double z = x * x;
  double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  double hz = 0.5 * z, w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}
double oracle_sin(double x) {
  int q; double y0, y1;
  rem_pio2(x, &q, &y0, &y1);
  switch (q) {
    case 0: return k_sin(y0, y1);
    case 1: return k_cos(y0, y1);
    case 2: return -k_sin(y0, y1);
    default: return -k_cos(y0, y1);
  }
}
double oracle_cos(double x) {
  int q; double y0, y1;
  rem_pio2(x, &q, &y0, &y1);
  switch (q) {
    case 0: return k_cos(y0, y1);
    case 1: return -k_sin(y0, y1);
    case 2: return -k_cos(y0, y1);
    default: return k_sin(y0, y1);
  }
}

/* Deterministic acos / atan / atan2 for get_sphere_uv (sphere.rs:213-220), bitwise the device's:
 * fdlibm's __ieee754_acos, atan and __ieee754_atan2 (Sun, 1993); + - * / and sqrt only. */
static inline int32_t hi_word(double x) { uint64_t b; memcpy(&b, &x, 8); return (int32_t)(b >> 32); }
static inline uint32_t lo_word(double x) { uint64_t b; memcpy(&b, &x, 8); return (uint32_t)b; }
static inline double with_lo_zero(double x) { uint64_t b; memcpy(&b, &x, 8); b &= 0xffffffff00000000ull; memcpy(&x, &b, 8); return x; }
double oracle_acos(double x) {
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
  df = with_lo_zero(s);
  c = (z - df * df) / (s + df);
  p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
  q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
  r = p / q;
  w = r * s + c;
  return 2.0 * (df + w);
}
static double det_atan(double x) {
  static const double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                                   1.57079632679489655800e+00};
  static const double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                                   6.12323399573676603587e-17};
  static const double aT[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01, 1.42857142725034663711e-01,
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
double oracle_atan2(double y, double x) {
  const double tiny = 1.0e-300, pi_o_4 = 7.8539816339744827900e-01, pi_o_2 = 1.5707963267948965580e+00,
               pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
  const int32_t hx = hi_word(x), ix = hx & 0x7fffffff, hy = hi_word(y), iy = hy & 0x7fffffff;
  const uint32_t lx = lo_word(x), ly = lo_word(y);
  if ((ix | (int32_t)((lx | (0u - lx)) >> 31)) > 0x7ff00000 || (iy | (int32_t)((ly | (0u - ly)) >> 31)) > 0x7ff00000)
    return x + y;
  if (((hx - 0x3ff00000) | (int32_t)lx) == 0) return det_atan(y);
  const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if ((iy | (int32_t)ly) == 0) {
    switch (m) {
      case 0: case 1: return y;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if ((ix | (int32_t)lx) == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7ff00000) {
    if (iy == 0x7ff00000) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0 * pi_o_4 + tiny;
        default: return -3.0 * pi_o_4 - tiny;
      }
    }
    switch (m) {
      case 0: return 0.0;
      case 1: return -0.0;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (iy == 0x7ff00000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  const int k = (iy - ix) >> 20;
  double z;
  if (k > 60) z = pi_o_2 + 0.5 * pi_lo;
  else if (hx < 0 && k < -60) z = 0.0;
  else z = det_atan(fabs(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;  /* the high-word sign flip of fdlibm */
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

/* Deterministic natural log shared bit for bit with the device (libm's log differs between glibc
 * and ROCm's ocml in the last ulp): fdlibm's __ieee754_log (Sun, 1993) — reduction to
 * f in [sqrt(2)/2 - 1, sqrt(2) - 1), s = f / (2 + f), and the Lg1..Lg7 minimax polynomial in s^2.
 * Only + - * / and exponent bit arithmetic. Used by ConstantMedium (hittable.rs:303). */
double oracle_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
               Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
  uint64_t bits; memcpy(&bits, &x, 8);
  int32_t hx = (int32_t)(bits >> 32);
  uint32_t lx = (uint32_t)bits;
  int k = 0;
  if (hx < 0x00100000) {                              /* x < 2^-1022 */
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -INFINITY; /* log(+-0) */
    if (hx < 0) return NAN;                          /* log(-#) */
    k -= 54; x *= two54;                             /* subnormal: scale up */
    memcpy(&bits, &x, 8); hx = (int32_t)(bits >> 32);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  int32_t i = (hx + 0x95f64) & 0x100000;
  memcpy(&bits, &x, 8);
  bits = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (bits & 0xffffffffu); /* x or x/2 in [sqrt2/2, sqrt2) */
  memcpy(&x, &bits, 8);
  k += (i >> 20);
  double f = x - 1.0, dk, R;
  if ((0x000fffff & (2 + hx)) < 3) {                 /* |f| < 2^-20 */
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
  double s = f / (2.0 + f);
  dk = (double)k;
  double z = s * s;
  i = hx - 0x6147a;
  double w = z * z;
  int32_t j = 0x6b851 - hx;
  double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  R = t2 + t1;
  if (i > 0) {
    double hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* f64::powi(x, 5) as LLVM expands it: x * ((x*x) * (x*x)) (material.rs:210). */
static inline double powi5(double x) { double x2 = x * x; return x * (x2 * x2); }

/* ------------------------------------------------------------------------ RNG
 * Philox4x32-10 (Salmon et al., SC'11; Random123) keyed by the 64-bit seed, counter
 * (block, sample, pixel, phase << 2 | stream). Each block yields two u64 draws, taken in order.
 * Streams: 0 the path's draws, 1 scene construction (host SceneRng), 2 ConstantMedium's
 * free-path draw — keyed (object index, sample, pixel, segment), one per medium per world query,
 * so it does not depend on the order the objects are visited in.
 * A path's draws are split into phases, each with its own run of blocks from block 0: phase 0
 * is the camera ray (main.rs:692-698), phase k >= 1 the scatter at the k-th bounce
 * (max_depth - depth + 1 of ray_reflectance main.rs:537). The reference draws from
 * rand::thread_rng, whose stream is not reproducible, so the stream layout is this
 * implementation's own; phases let the GPU compute each bounce's blocks at one place in its
 * loop. Draws whose value cannot reach any output are not taken (a one-element index range,
 * the ray time when no MovingSphere reads it). The mappings from u64 to the values the reference
 * asks rand 0.8.5 for are restated below. */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c0 = hi1 ^ c1 ^ k0; c1 = lo1; c2 = hi0 ^ c3 ^ k1; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* Independent-stream mode (oracle_render mode bit 2, statistical tests only): the reference's own
 * generator family — rand 0.8.5's ThreadRng is ChaCha12 (rand_chacha 0.3: 12 rounds, 64-bit block
 * counter in words 12-13, next_u64 = two consecutive u32 words, low first) — one sequential stream
 * per (seed, pixel, sample) with the key drawn by splitmix64, no phases: every draw of the path in
 * the reference's order, rejection loops included. Its images must agree with the Philox ones in
 * distribution (tests/test_statistical.py), not in bits. */
static inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
#define CHACHA_QR(a, b, c, d)                        \
  a += b; d ^= a; d = rotl32(d, 16);                 \
  c += d; b ^= c; b = rotl32(b, 12);                 \
  a += b; d ^= a; d = rotl32(d, 8);                  \
  c += d; b ^= c; b = rotl32(b, 7);
void oracle_chacha_block(const uint32_t in[16], uint32_t out[16], int double_rounds) {
  uint32_t x[16];
  memcpy(x, in, sizeof x);
  for (int i = 0; i < double_rounds; ++i) {
    CHACHA_QR(x[0], x[4], x[8], x[12]) CHACHA_QR(x[1], x[5], x[9], x[13])
    CHACHA_QR(x[2], x[6], x[10], x[14]) CHACHA_QR(x[3], x[7], x[11], x[15])
    CHACHA_QR(x[0], x[5], x[10], x[15]) CHACHA_QR(x[1], x[6], x[11], x[12])
    CHACHA_QR(x[2], x[7], x[8], x[13]) CHACHA_QR(x[3], x[4], x[9], x[14])
  }
  for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}
void oracle_chacha12_block(const uint32_t in[16], uint32_t out[16]) { oracle_chacha_block(in, out, 6); }
static inline uint64_t splitmix64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

typedef struct {
  uint32_t key[2]; uint32_t ctr[4]; uint32_t buf[4]; int have;
  int chacha; uint32_t cc_in[16]; uint32_t cc_out[16]; int cc_have;
} rng_t;
static void rng_init(rng_t* r, uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t stream) {
  r->key[0] = (uint32_t)seed; r->key[1] = (uint32_t)(seed >> 32);
  r->ctr[0] = 0; r->ctr[1] = sample; r->ctr[2] = pixel; r->ctr[3] = stream;
  r->have = 0;
  r->chacha = 0;
}
static void rng_init_chacha(rng_t* r, uint64_t seed, uint32_t pixel, uint32_t sample) {
  static const uint32_t sigma[4] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
  rng_init(r, seed, pixel, sample, 0);
  r->chacha = 1;
  uint64_t sm = seed ^ (((uint64_t)pixel << 32) | sample) * 0xD1342543DE82EF95ull;
  memcpy(r->cc_in, sigma, sizeof sigma);
  for (int i = 0; i < 4; ++i) {
    uint64_t k = splitmix64(&sm);
    r->cc_in[4 + 2 * i] = (uint32_t)k; r->cc_in[5 + 2 * i] = (uint32_t)(k >> 32);
  }
  r->cc_in[12] = r->cc_in[13] = r->cc_in[14] = r->cc_in[15] = 0;
  r->cc_have = 0;
}
static void rng_phase(rng_t* r, uint32_t phase) {
  if (r->chacha) return; /* one sequential stream, as thread_rng */
  r->ctr[0] = 0; r->ctr[3] = (phase << 2) | (r->ctr[3] & 3u);
  r->have = 0;
}
static inline uint64_t rng_u64(rng_t* r) {
  if (r->chacha) {
    if (r->cc_have < 2) { /* a u64 never straddles blocks: 16 words = 8 draws */
      oracle_chacha12_block(r->cc_in, r->cc_out);
      if (++r->cc_in[12] == 0) ++r->cc_in[13];
      r->cc_have = 16;
    }
    int i = 16 - r->cc_have; r->cc_have -= 2;
    return ((uint64_t)r->cc_out[i + 1] << 32) | r->cc_out[i];
  }
  if (r->have == 0) { oracle_philox4x32_10(r->ctr, r->key, r->buf); r->ctr[0]++; r->have = 2; }
  int i = 2 - r->have; r->have--;
  return ((uint64_t)r->buf[2 * i + 1] << 32) | r->buf[2 * i];
}
/* rand 0.8.5 Standard for f64: 53 high bits * 2^-53, [0, 1). (rng.gen::<f64>(), rand::random) */
static inline double gen_f64(rng_t* r) { return (double)(rng_u64(r) >> 11) * 0x1.0p-53; }
/* rand 0.8.5 UniformFloat::sample_single: [1,2) from 52 bits, minus 1, *scale + low; retried
 * (with scale one ulp smaller) if rounding reached `high`. (gen_range(low..high)) */
static inline double gen_range_f64(rng_t* r, double low, double high) {
  double scale = high - low;
  for (;;) {
    uint64_t bits = (rng_u64(r) >> 12) | 0x3FF0000000000000ull;
    double v12; memcpy(&v12, &bits, 8);
    double res = (v12 - 1.0) * scale + low;
    if (res < high) return res;
    uint64_t sb; memcpy(&sb, &scale, 8); sb -= 1; memcpy(&scale, &sb, 8);
  }
}
/* rand 0.8.5 UniformInt<usize>::sample_single(0..n): widening multiply, zone rejection. */
static inline uint64_t gen_range_usize(rng_t* r, uint64_t n) {
  if (n == 1) return 0; /* the only value; its rejection draws are unobservable */
  uint64_t range = n;
  uint64_t zone = (range << __builtin_clzll(range)) - 1;
  for (;;) {
    uint64_t v = rng_u64(r);
    unsigned __int128 m = (unsigned __int128)v * range;
    uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
    if (lo <= zone) return hi;
  }
}

/* ConstantMedium's rng.gen::<f64>() (hittable.rs:303) for object `obj` at world query `seg`. */
static double medium_draw(uint64_t seed, uint32_t obj, uint32_t sample, uint32_t pixel, uint32_t seg) {
  const uint32_t ctr[4] = {obj, sample, pixel, (seg << 2) | 2u}, key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t out[4];
  oracle_philox4x32_10(ctr, key, out);
  return (double)((((uint64_t)out[1] << 32) | out[0]) >> 11) * 0x1.0p-53;
}

void oracle_rng_f64(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, double* out) {
  rng_t r; rng_init(&r, seed, pixel, sample, 0);
  for (uint32_t i = 0; i < n; ++i) out[i] = gen_f64(&r);
}
double oracle_gen_range_f64(uint64_t seed, uint32_t pixel, uint32_t sample, double lo, double hi) {
  rng_t r; rng_init(&r, seed, pixel, sample, 0);
  return gen_range_f64(&r, lo, hi);
}

/* ------------------------------------------------------------------ spectral (color.rs) */
/* RGB::into_spectrum (color.rs:54-90) evaluated at one bin; Spectrum += is `self = rhs + self`
 * (color.rs:252-264) starting from 0.0. */
static double rgb_spectrum_bin(const double rgb[3], int i) {
  double red = rgb[0], green = rgb[1], blue = rgb[2], s = 0.0;
  if (red <= green && red <= blue) {
    s = red * SMITS[S_WHITE][i] + s;
    if (green <= blue) {
      s = (green - red) * SMITS[S_CYAN][i] + s;
      s = (blue - green) * SMITS[S_BLUE][i] + s;
    } else {
      s = (blue - red) * SMITS[S_CYAN][i] + s;
      s = (green - blue) * SMITS[S_GREEN][i] + s;
    }
  } else if (green <= red && green <= blue) {
    s = green * SMITS[S_WHITE][i] + s;
    if (red <= blue) {
      s = (red - green) * SMITS[S_MAGENTA][i] + s;
      s = (blue - red) * SMITS[S_BLUE][i] + s;
    } else {
      s = (blue - green) * SMITS[S_MAGENTA][i] + s;
      s = (red - blue) * SMITS[S_RED][i] + s;
    }
  } else {
    s = blue * SMITS[S_WHITE][i] + s;
    if (red <= green) {
      s = (red - blue) * SMITS[S_YELLOW][i] + s;
      s = (green - red) * SMITS[S_GREEN][i] + s;
    } else {
      s = (green - blue) * SMITS[S_YELLOW][i] + s;
      s = (red - green) * SMITS[S_RED][i] + s;
    }
  }
  return s;
}
/* Spectrum::reflect (color.rs:276-283): bin = ((wl - 360) / 10) as usize, clamped to 0..35
 * (Rust's float->usize cast saturates: negative / NaN -> 0). */
static inline int spectrum_bin(double wl) {
  double f = (wl - MIN_LAMBDA) / BIN_WIDTH;
  if (!(f > 0.0)) return 0;
  if (f >= (double)BIN_COUNT) return BIN_COUNT - 1;
  int i = (int)f;
  return i > BIN_COUNT - 1 ? BIN_COUNT - 1 : i;
}
double oracle_rgb_reflect(const double rgb[3], double wl) { /* RGB::reflect color.rs:160-164 */
  return rgb_spectrum_bin(rgb, spectrum_bin(wl));
}
void oracle_xyz_from_wavelength(double wl, double out[3]) { /* color.rs:216-228 */
  double f = wl - MIN_LAMBDA;
  long long idx = (f != f) ? 0 : (f <= -9.3e18 ? INT64_MIN : (f >= 9.3e18 ? INT64_MAX : (long long)f));
  if (idx < 0 || idx >= N_CIE_SAMPLES) { out[0] = out[1] = out[2] = 0.0; return; }
  out[0] = CIE_XYZ[idx][0]; out[1] = CIE_XYZ[idx][1]; out[2] = CIE_XYZ[idx][2];
}
void oracle_xyz_into_rgb(const double in[3], double o[3]) { /* color.rs:209-213 */
  double x = in[0], y = in[1], z = in[2];
  o[0] = 2.6896552 * x - 1.2758621 * y - 0.4137931 * z;
  o[1] = -1.0221082 * x + 1.9782866 * y + 0.0438216 * z;
  o[2] = 0.0612245 * x - 0.2244898 * y + 1.1632653 * z;
}
static double gamma_channel(double linear) { /* color.rs:93-101 */
  linear = fmax(linear, 0.0);                  /* f64::max ignores NaN like fmax */
  if (linear <= 0.0031308) return 12.92 * linear;
  return 1.055 * pow(linear, 1.0 / 2.4) - 0.055;
}
void oracle_gamma_corrected(const double in[3], double out[3]) { /* color.rs:92-107 */
  out[0] = gamma_channel(in[0]); out[1] = gamma_channel(in[1]); out[2] = gamma_channel(in[2]);
}
/* The 8-bit channel of each linear value: gamma_channel (glibc's pow, as f64::powf) then
 * clamp_display_channel, as main.rs:710-718 applies them; for tests/test_finalize_bytes.py. */
void oracle_display_bytes(const double* linear, size_t n, uint8_t* out) {
  for (size_t i = 0; i < n; ++i) out[i] = oracle_clamp_display_channel(gamma_channel(linear[i]));
}
uint8_t oracle_clamp_display_channel(double c) { /* main.rs:461-463; `as u8` saturates, NaN->0 */
  double v = c;
  if (v != v) v = 0.0; /* f64::clamp propagates NaN; 256*NaN as u8 = 0 */
  else if (v < 0.0) v = 0.0;
  else if (v > 0.999) v = 0.999;
  double m = 256.0 * v;
  if (!(m > 0.0)) return 0;
  if (m >= 255.0) return 255;
  return (uint8_t)m;
}
void oracle_sanitize_sample_xyz(const double in[3], double out[3]) { /* main.rs:448-459 */
  if (!isfinite(in[0]) || !isfinite(in[1]) || !isfinite(in[2])) {
    out[0] = out[1] = out[2] = 0.0;
    return;
  }
  double lum = in[1];
  if (lum <= 0.0 || lum <= MAX_SAMPLE_LUMINANCE) { out[0] = in[0]; out[1] = in[1]; out[2] = in[2]; return; }
  double k = MAX_SAMPLE_LUMINANCE / lum;
  out[0] = in[0] * k; out[1] = in[1] * k; out[2] = in[2] * k;
}

/* -------------------------------------------------------------------- scene (oracle form) */
typedef struct { double bmin[3][4], bmax[3][4]; uint32_t child[4]; int top_axis, left_axis, right_axis; } qnode; /* qbvh.rs:547-554 */
typedef struct { double v0[3][4], e1[3][4], e2[3][4], n0[3][4], n1[3][4], n2[3][4]; } qleaf; /* qbvh.rs:603-634 (uv unused) */
typedef struct {
  uint32_t ntris;
  v3* vert;   /* ntris*3, in the final (sorted) order */
  v3* norm;   /* ntris*3 */
  qnode* nodes; uint32_t nnodes, cap_nodes;
  qleaf* leaves; uint32_t nleaves;
  uint32_t* leaf_of_first; /* leaf slot by first triangle index (replaces the HashMap, qbvh.rs:248) */
  uint32_t depth;
} qbvh_t;

struct oracle_scene {
  yart_object* objects; uint32_t nobj;
  yart_object* lights; uint32_t nlights;
  yart_material* mats; uint32_t nmats;
  yart_texture* texs; uint32_t ntexs;
  yart_perlin* perlins; /* per texture (NOISE) */
  uint8_t** images;     /* per texture (IMAGE) */
  int has_time;         /* a MovingSphere reads the ray's shutter time */
  qbvh_t* meshes; uint32_t nmeshes;
  double background[3];
  /* per object, per wrapper: RotateY sin/cos (hittable.rs:173-176) */
  double (*obj_sc)[YART_MAX_XFORMS][2];
  double (*light_sc)[YART_MAX_XFORMS][2];
};

typedef struct { double u, v, t; v3 p, normal; int front_face; uint32_t mat; } hit_rec; /* hittable.rs:37-45 */

/* ---------------------------------------------------------- L4QBVH build (qbvh.rs:252-361) */
typedef struct { double min[3], max[3]; } aabb_t; /* aabb.rs:8-12 */
static aabb_t surrounding(aabb_t a, aabb_t b) { /* aabb.rs:187-202 */
  aabb_t r;
  for (int i = 0; i < 3; ++i) { r.min[i] = fmin(a.min[i], b.min[i]); r.max[i] = fmax(a.max[i], b.max[i]); }
  return r;
}
static aabb_t tri_bbox(const v3* v) { /* triangle.rs:37-62: folds from +-INFINITY with f64::min/max */
  aabb_t b;
  for (int i = 0; i < 3; ++i) {
    b.min[i] = INFINITY; b.max[i] = -INFINITY;
    for (int k = 0; k < 3; ++k) { b.min[i] = fmin(b.min[i], comp(v[k], i)); b.max[i] = fmax(b.max[i], comp(v[k], i)); }
  }
  return b;
}

typedef struct { const v3* vert; const v3* norm; double* key; uint32_t* perm; } build_ctx;
static int cmp_key_ctx(const void* a, const void* b, void* ctx) {
  const double* key = (const double*)ctx;
  uint32_t ia = *(const uint32_t*)a, ib = *(const uint32_t*)b;
  if (key[ia] < key[ib]) return -1;
  if (key[ia] > key[ib]) return 1;
  return ia < ib ? -1 : (ia > ib ? 1 : 0); /* sort_unstable_by's tie order is unspecified; pin it */
}
/* split (qbvh.rs:637-693): centroid extents, widest axis (x, then y if larger, then z if larger
 * than both), sort by centroid on that axis, cut at len/2. */
static int split(build_ctx* c, uint32_t off, uint32_t n) {
  double mnx = INFINITY, mxx = -INFINITY, mny = INFINITY, mxy = -INFINITY, mnz = INFINITY, mxz = -INFINITY;
  double* cen = (double*)malloc(sizeof(double) * 3 * n);
  for (uint32_t i = 0; i < n; ++i) {
    aabb_t b = tri_bbox(&c->vert[3 * c->perm[off + i]]);
    /* Hittable::centroid (hittable.rs:12-22) */
    double cx = (b.max[0] + b.min[0]) / 2.0, cy = (b.max[1] + b.min[1]) / 2.0, cz = (b.max[2] + b.min[2]) / 2.0;
    cen[3 * i] = cx; cen[3 * i + 1] = cy; cen[3 * i + 2] = cz;
    mnx = fmin(mnx, cx); mxx = fmax(mxx, cx); mny = fmin(mny, cy); mxy = fmax(mxy, cy); mnz = fmin(mnz, cz); mxz = fmax(mxz, cz);
  }
  int axis = 0;
  if (mxy - mny > mxx - mnx) axis = 1;
  if (mxz - mnz > fmax(mxy - mny, mxx - mnx)) axis = 2;
  for (uint32_t i = 0; i < n; ++i) c->key[c->perm[off + i]] = cen[3 * i + axis];
  free(cen);
  qsort_r(c->perm + off, n, sizeof(uint32_t), cmp_key_ctx, c->key);
  return axis;
}

typedef struct { int has; aabb_t box; uint32_t id; } built_t;

static void push_leaf(qbvh_t* q, build_ctx* c, uint32_t off, uint32_t n, built_t* out) {
  aabb_t box = tri_bbox(&c->vert[3 * c->perm[off]]);
  for (uint32_t i = 1; i < n; ++i) box = surrounding(box, tri_bbox(&c->vert[3 * c->perm[off + i]]));
  uint32_t id = off | (1u << 31) | (n << 27);      /* qbvh.rs:270 */
  qleaf* L = &q->leaves[q->nleaves];
  const double MX = 1.7976931348623157e308;         /* precompute_soa_triangle fills with MAX */
  for (int j = 0; j < 3; ++j)
    for (int i = 0; i < 4; ++i)
      L->v0[j][i] = L->e1[j][i] = L->e2[j][i] = L->n0[j][i] = L->n1[j][i] = L->n2[j][i] = MX;
  for (uint32_t i = 0; i < n; ++i) { /* qbvh.rs:612-623; this range's order is final here */
    const v3* v = &c->vert[3 * c->perm[off + i]];
    const v3* nn = &c->norm[3 * c->perm[off + i]];
    for (int j = 0; j < 3; ++j) {
      L->v0[j][i] = comp(v[0], j);
      L->e1[j][i] = comp(v[1], j) - comp(v[0], j);
      L->e2[j][i] = comp(v[2], j) - comp(v[0], j);
      L->n0[j][i] = comp(nn[0], j);
      L->n1[j][i] = comp(nn[1], j);
      L->n2[j][i] = comp(nn[2], j);
    }
  }
  q->leaf_of_first[off] = q->nleaves++;
  out->has = 1; out->box = box; out->id = id;
}

static void construct(qbvh_t* q, build_ctx* c, uint32_t off, uint32_t n, uint32_t level, built_t* out) {
  if (n == 0) { out->has = 0; out->id = 0xFFFFFFFFu; return; }
  if (n <= 4) { push_leaf(q, c, off, n, out); return; }
  if (level + 1 > q->depth) q->depth = level + 1;
  uint32_t nl = n / 2, nr = n - n / 2;
  int top = split(c, off, n);
  int la = split(c, off, nl);
  built_t ll, lr, rl, rr;
  construct(q, c, off, nl / 2, level + 1, &ll);
  construct(q, c, off + nl / 2, nl - nl / 2, level + 1, &lr);
  int ra = split(c, off + nl, nr);
  construct(q, c, off + nl, nr / 2, level + 1, &rl);
  construct(q, c, off + nl + nr / 2, nr - nr / 2, level + 1, &rr);
  /* QBVHNode::new (qbvh.rs:557-599) */
  if (q->nnodes == q->cap_nodes) { q->cap_nodes = q->cap_nodes ? 2 * q->cap_nodes : 64; q->nodes = (qnode*)realloc(q->nodes, sizeof(qnode) * q->cap_nodes); }
  qnode* N = &q->nodes[q->nnodes];
  const double MX = 1.7976931348623157e308;
  built_t* ch[4] = {&ll, &lr, &rl, &rr};
  for (int k = 0; k < 4; ++k) {
    for (int j = 0; j < 3; ++j) { N->bmin[j][k] = MX; N->bmax[j][k] = MX; }
    if (ch[k]->has) for (int j = 0; j < 3; ++j) { N->bmin[j][k] = ch[k]->box.min[j]; N->bmax[j][k] = ch[k]->box.max[j]; }
    N->child[k] = ch[k]->id;
  }
  N->top_axis = top; N->left_axis = la; N->right_axis = ra;
  q->nnodes++;
  aabb_t lb = ll.has && lr.has ? surrounding(ll.box, lr.box) : (ll.has ? ll.box : lr.box);
  aabb_t rb = rl.has && rr.has ? surrounding(rl.box, rr.box) : (rl.has ? rl.box : rr.box);
  out->has = 1; out->box = surrounding(lb, rb); out->id = q->nnodes - 1;
}

static int build_qbvh(qbvh_t* q, const yart_mesh* m) {
  uint32_t n = m->n_triangles;
  memset(q, 0, sizeof(*q));
  if (n <= 4) return -1; /* L4QBVH::hit underflows `nodes_len - 1` (qbvh.rs:383-384) */
  v3* vin = (v3*)malloc(sizeof(v3) * 3 * n);
  v3* nin = (v3*)malloc(sizeof(v3) * 3 * n);
  for (uint32_t t = 0; t < n; ++t)
    for (int k = 0; k < 3; ++k) {
      const float* p = &m->positions[9 * t + 3 * k];
      const double* nn = &m->normals[9 * t + 3 * k];
      vin[3 * t + k] = V((double)p[0], (double)p[1], (double)p[2]); /* f32 -> f64 (triangle.rs:438) */
      nin[3 * t + k] = V(nn[0], nn[1], nn[2]);
    }
  build_ctx c;
  c.vert = vin;
  c.norm = nin;
  c.key = (double*)malloc(sizeof(double) * n);
  c.perm = (uint32_t*)malloc(sizeof(uint32_t) * n);
  for (uint32_t i = 0; i < n; ++i) c.perm[i] = i;
  q->leaves = (qleaf*)malloc(sizeof(qleaf) * (n + 1));
  q->leaf_of_first = (uint32_t*)malloc(sizeof(uint32_t) * n);
  built_t root;
  construct(q, &c, 0, n, 0, &root);
  /* the triangles vector ends up in sorted order (qbvh.rs:349-359); normals per leaf lane */
  q->ntris = n;
  q->vert = (v3*)malloc(sizeof(v3) * 3 * n);
  q->norm = (v3*)malloc(sizeof(v3) * 3 * n);
  for (uint32_t i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) { q->vert[3 * i + k] = vin[3 * c.perm[i] + k]; q->norm[3 * i + k] = nin[3 * c.perm[i] + k]; }
  free(vin); free(nin); free(c.key); free(c.perm);
  return 0;
}

/* ------------------------------------------------------- L4QBVH::hit (qbvh.rs:381-543) */
static const uint32_t ORDER_TABLE[8] = {0x0123, 0x0132, 0x1023, 0x1032, 0x2301, 0x3201, 0x2310, 0x3210}; /* qbvh.rs:14-16 */

int oracle_push_hit_children(uint32_t* stack, int cursor, const uint32_t children[4],
                             const uint32_t order[4], const int hits[4]) { /* qbvh.rs:18-31 */
  for (int k = 0; k < 4; ++k) {
    uint32_t i = order[k];
    if (hits[i]) stack[cursor++] = children[i];
  }
  return cursor;
}

static int qbvh_hit(const qbvh_t* q, const ray_t* r, double t_min, double t_max, hit_rec* rec) {
  uint32_t stack[64];
  for (int i = 0; i < 64; ++i) stack[i] = q->nnodes - 1; /* root is the last node pushed */
  int cursor = 0, found = 0;
  int pos[3] = {r->d.x >= 0.0, r->d.y >= 0.0, r->d.z >= 0.0};
  double ro[3] = {r->o.x, r->o.y, r->o.z}, rd[3] = {r->d.x, r->d.y, r->d.z};
  double inv[3] = {1.0 / rd[0], 1.0 / rd[1], 1.0 / rd[2]};
  for (;;) {
    uint32_t id = stack[cursor];
    if (id >> 31 == 1) {
      uint32_t count = (id & (0xFu << 27)) >> 27;
      uint32_t index = id & ((1u << 27) - 1);
      const qleaf* L = &q->leaves[q->leaf_of_first[index]];
      int hitl[4]; double tl[4], px[4], py[4], pz[4], nx[4], ny[4], nz[4]; int ffl[4];
      for (int i = 0; i < 4; ++i) {
        double e1x = L->e1[0][i], e1y = L->e1[1][i], e1z = L->e1[2][i];
        double e2x = L->e2[0][i], e2y = L->e2[1][i], e2z = L->e2[2][i];
        double hx = rd[1] * e2z - rd[2] * e2y, hy = rd[2] * e2x - rd[0] * e2z, hz = rd[0] * e2y - rd[1] * e2x;
        double a = e1x * hx + e1y * hy + e1z * hz;
        int hit = !(a > -F64_EPSILON && a < F64_EPSILON);
        double f = 1.0 / a;
        double sx = ro[0] - L->v0[0][i], sy = ro[1] - L->v0[1][i], sz = ro[2] - L->v0[2][i];
        double u = f * (sx * hx + sy * hy + sz * hz);
        hit = hit && (u >= 0.0) && (u <= 1.0);
        double qx = sy * e1z - sz * e1y, qy = sz * e1x - sx * e1z, qz = sx * e1y - sy * e1x;
        double v = f * (rd[0] * qx + rd[1] * qy + rd[2] * qz);
        hit = hit && (v >= 0.0) && (u + v <= 1.0);
        double t = f * (e2x * qx + e2y * qy + e2z * qz);
        hit = hit && (t >= t_min) && (t <= t_max);
        px[i] = ro[0] + t * rd[0]; py[i] = ro[1] + t * rd[1]; pz[i] = ro[2] + t * rd[2];
        double w = 1.0 - u - v;
        double onx = L->n0[0][i] * w + L->n1[0][i] * u + L->n2[0][i] * v;
        double ony = L->n0[1][i] * w + L->n1[1][i] * u + L->n2[1][i] * v;
        double onz = L->n0[2][i] * w + L->n1[2][i] * u + L->n2[2][i] * v;
        int ff = (rd[0] * onx + rd[1] * ony + rd[2] * onz) <= 0.0;
        double sign = ff ? 1.0 : -1.0;
        nx[i] = sign * onx; ny[i] = sign * ony; nz[i] = sign * onz;
        hitl[i] = hit; tl[i] = t; ffl[i] = ff;
      }
      for (uint32_t i = 0; i < count; ++i) { /* qbvh.rs:470-490: strict t_max > t */
        if (hitl[i] && t_max > tl[i]) {
          t_max = tl[i];
          rec->t = tl[i]; rec->p = V(px[i], py[i], pz[i]); rec->normal = V(nx[i], ny[i], nz[i]);
          rec->front_face = ffl[i];
          rec->u = 0.0; rec->v = 0.0; /* mesh texcoords: no in-scope texture reads them on a mesh */
          found = 1;
        }
      }
    } else {
      const qnode* N = &q->nodes[id];
      double tmn[4], tmx[4];
      for (int k = 0; k < 4; ++k) {
        /* qbvh.rs:495-519: simd_min/simd_max ignore NaN (fmin/fmax); fold from t_min / t_max */
        double lo = t_min, hi = t_max;
        for (int j = 0; j < 3; ++j) {
          double t0 = (N->bmin[j][k] - ro[j]) * inv[j];
          double t1 = (N->bmax[j][k] - ro[j]) * inv[j];
          lo = fmax(lo, fmin(t0, t1));
        }
        for (int j = 0; j < 3; ++j) {
          double t0 = (N->bmin[j][k] - ro[j]) * inv[j];
          double t1 = (N->bmax[j][k] - ro[j]) * inv[j];
          hi = fmin(hi, fmax(t0, t1));
        }
        tmn[k] = lo; tmx[k] = hi;
      }
      uint32_t enc = ORDER_TABLE[4 * pos[N->top_axis] + 2 * pos[N->left_axis] + pos[N->right_axis]];
      uint32_t order[4] = {enc & 0xF, (enc >> 4) & 0xF, (enc >> 8) & 0xF, (enc >> 12) & 0xF};
      int hits[4] = {tmx[0] > tmn[0], tmx[1] > tmn[1], tmx[2] > tmn[2], tmx[3] > tmn[3]};
      cursor = oracle_push_hit_children(stack, cursor, N->child, order, hits);
    }
    if (cursor == 0) break;
    cursor -= 1;
  }
  return found;
}

/* ------------------------------------------------------------ primitive hits */
static int sphere_hit(const double* p, const ray_t* r, double t_min, double t_max, hit_rec* rec) { /* sphere.rs:48-86 */
  v3 center = V(p[0], p[1], p[2]);
  double radius = p[3];
  v3 oc = vsub(r->o, center);
  double a = length_squared(r->d);
  double half_b = dot(oc, r->d);
  double c = length_squared(oc) - radius * radius;
  double disc = half_b * half_b - a * c;
  if (disc < 0.0) return 0;
  double t = (0.0 - half_b - sqrt(disc)) / a;
  if (t < t_min || t_max < t) {
    t = (0.0 - half_b + sqrt(disc)) / a;
    if (t < t_min || t_max < t) return 0;
  }
  v3 pt = ray_at(r, t);
  v3 outward = vdivs(vsub(pt, center), fabs(radius));
  if (radius < 0.0) { rec->normal = vneg(outward); rec->front_face = dot(r->d, outward) > 0.0; }
  else { rec->normal = outward; rec->front_face = dot(r->d, outward) < 0.0; }
  rec->t = t; rec->p = pt;
  /* get_sphere_uv (sphere.rs:213-220) of the outward normal */
  const double theta = oracle_acos(-outward.y), phi = oracle_atan2(-outward.z, outward.x) + PI;
  rec->u = phi / (2.0 * PI);
  rec->v = theta / PI;
  return 1;
}
/* MovingSphere::hit (sphere.rs:161-199): centre at the ray's time; normal faces the ray. */
static v3 moving_center(const double* p, double time) { /* sphere.rs:153-156 */
  return vadd(V(p[0], p[1], p[2]), smulv((time - p[6]) / (p[7] - p[6]), vsub(V(p[3], p[4], p[5]), V(p[0], p[1], p[2]))));
}
static int moving_sphere_hit(const double* p, const ray_t* r, double t_min, double t_max, hit_rec* rec) {
  const double radius = p[8];
  v3 oc = vsub(r->o, moving_center(p, r->time));
  double a = length_squared(r->d);
  double half_b = dot(oc, r->d);
  double c = length_squared(oc) - radius * radius;
  double disc = half_b * half_b - a * c;
  if (disc < 0.0) return 0;
  double t = (0.0 - half_b - sqrt(disc)) / a;
  if (t < t_min || t_max < t) {
    t = (0.0 - half_b + sqrt(disc)) / a;
    if (t < t_min || t_max < t) return 0;
  }
  v3 pt = ray_at(r, t);
  v3 outward = vdivs(vsub(pt, moving_center(p, r->time)), radius);
  if (dot(r->d, outward) < 0.0) { rec->normal = outward; rec->front_face = 1; }
  else { rec->normal = vneg(outward); rec->front_face = 0; }
  const double theta = oracle_acos(-outward.y), phi = oracle_atan2(-outward.z, outward.x) + PI;
  rec->u = phi / (2.0 * PI);
  rec->v = theta / PI;
  rec->t = t; rec->p = pt;
  return 1;
}
/* aarect.rs: axis a (plane normal), in-plane axes b, c: XY a=z (b=x, c=y) :41-76;
 * XZ a=y (b=x, c=z) :111-146; YZ a=x (b=y, c=z) :206-241. p = b0, b1, c0, c1, k. */
static int rect_hit(int kind, const double* p, const ray_t* r, double t_min, double t_max, hit_rec* rec) {
  int a, b, c;
  v3 outward;
  if (kind == YART_PRIM_XY_RECT) { a = 2; b = 0; c = 1; outward = V(0.0, 0.0, 1.0); }
  else if (kind == YART_PRIM_XZ_RECT) { a = 1; b = 0; c = 2; outward = V(0.0, 1.0, 0.0); }
  else { a = 0; b = 1; c = 2; outward = V(1.0, 0.0, 0.0); }
  double t = (p[4] - comp(r->o, a)) / comp(r->d, a);
  if (t < t_min || t > t_max) return 0;
  double x = comp(r->o, b) + t * comp(r->d, b);
  double y = comp(r->o, c) + t * comp(r->d, c);
  if (x < p[0] || x > p[1] || y < p[2] || y > p[3]) return 0;
  rec->u = (x - p[0]) / (p[1] - p[0]);
  rec->v = (y - p[2]) / (p[3] - p[2]);
  rec->t = t; rec->p = ray_at(r, t);
  if (dot(r->d, outward) < 0.0) { rec->normal = outward; rec->front_face = 1; }
  else { rec->normal = vneg(outward); rec->front_face = 0; }
  return 1;
}
static int box_hit(const double* p, const ray_t* r, double t_min, double t_max, hit_rec* rec) { /* box_entity.rs:22-36, 53-70 */
  double sides[6][5] = {
    {p[0], p[3], p[1], p[4], p[2]}, {p[0], p[3], p[1], p[4], p[5]},
    {p[0], p[3], p[2], p[5], p[1]}, {p[0], p[3], p[2], p[5], p[4]},
    {p[1], p[4], p[2], p[5], p[0]}, {p[1], p[4], p[2], p[5], p[3]}};
  int kinds[6] = {YART_PRIM_XY_RECT, YART_PRIM_XY_RECT, YART_PRIM_XZ_RECT, YART_PRIM_XZ_RECT, YART_PRIM_YZ_RECT, YART_PRIM_YZ_RECT};
  int found = 0; double closest = t_max; hit_rec tmp;
  for (int i = 0; i < 6; ++i)
    if (rect_hit(kinds[i], sides[i], r, t_min, closest, &tmp)) { closest = tmp.t; *rec = tmp; found = 1; }
  return found;
}
static int triangle_hit(const double* p, const ray_t* r, double t_min, double t_max, hit_rec* rec) { /* triangle.rs:48-101 */
  v3 v0 = V(p[0], p[1], p[2]), v1 = V(p[3], p[4], p[5]), v2 = V(p[6], p[7], p[8]);
  v3 n0 = V(p[9], p[10], p[11]), n1 = V(p[12], p[13], p[14]), n2 = V(p[15], p[16], p[17]);
  v3 e1 = vsub(v1, v0), e2 = vsub(v2, v0);
  v3 h = cross(r->d, e2);
  double a = dot(e1, h);
  if (a > -F64_EPSILON && a < F64_EPSILON) return 0;
  double f = 1.0 / a;
  v3 s = vsub(r->o, v0);
  double u = f * dot(s, h);
  if (u < 0.0 || u > 1.0) return 0;
  v3 q = cross(s, e1);
  double v = f * dot(r->d, q);
  if (v < 0.0 || u + v > 1.0) return 0;
  double t = f * dot(e2, q);
  if (t < t_min || t > t_max) return 0;
  double w = 1.0 - u - v;
  v3 outward = vadd(vadd(vmuls(n0, w), vmuls(n1, u)), vmuls(n2, v));
  rec->u = p[18] * w + p[20] * u + p[22] * v; /* triangle.rs:93-94 */
  rec->v = p[19] * w + p[21] * u + p[23] * v;
  rec->t = t; rec->p = ray_at(r, t);
  if (dot(r->d, outward) < 0.0) { rec->normal = outward; rec->front_face = 1; }
  else { rec->normal = vneg(outward); rec->front_face = 0; }
  return 1;
}

static int prim_hit(const oracle_scene* s, const yart_object* o, const ray_t* r, double t_min, double t_max, hit_rec* rec) {
  switch (o->kind) {
    case YART_PRIM_SPHERE: return sphere_hit(o->p, r, t_min, t_max, rec);
    case YART_PRIM_XY_RECT: case YART_PRIM_XZ_RECT: case YART_PRIM_YZ_RECT: return rect_hit((int)o->kind, o->p, r, t_min, t_max, rec);
    case YART_PRIM_BOX: return box_hit(o->p, r, t_min, t_max, rec);
    case YART_PRIM_TRIANGLE: return triangle_hit(o->p, r, t_min, t_max, rec);
    case YART_PRIM_MESH: return qbvh_hit(&s->meshes[o->mesh], r, t_min, t_max, rec); /* triangle.rs:177-185 */
    case YART_PRIM_MOVING_SPHERE: return moving_sphere_hit(o->p, r, t_min, t_max, rec);
  }
  return 0;
}

/* Wrappers, outermost first: Translate (hittable.rs:136-152), RotateY (:217-251), FlipFace (:338-349). */
/* Where a world query happens: keys ConstantMedium's draw (stream 2, see the RNG notes). */
typedef struct { uint64_t seed; uint32_t sample, pixel, seg; } wctx_t;

static int object_hit(const oracle_scene* s, const yart_object* o, const double (*sc)[2], uint32_t level,
                      const ray_t* r, double t_min, double t_max, hit_rec* rec, const wctx_t* cx, uint32_t obj) {
  if (level == o->n_xforms) return prim_hit(s, o, r, t_min, t_max, rec);
  const yart_xform* x = &o->xforms[level];
  if (x->kind == YART_XF_MEDIUM) { /* ConstantMedium::hit hittable.rs:277-318 */
    hit_rec rec1, rec2;
    if (!object_hit(s, o, sc, level + 1, r, -INFINITY, INFINITY, &rec1, cx, obj)) return 0;
    if (!object_hit(s, o, sc, level + 1, r, rec1.t + 0.0001, INFINITY, &rec2, cx, obj)) return 0;
    if (rec1.t < t_min) rec1.t = t_min;
    if (rec2.t > t_max) rec2.t = t_max;
    if (!(rec1.t < rec2.t)) return 0;
    if (rec1.t < 0.0) rec1.t = 0.0;
    const double ray_length = length(r->d);
    const double distance_inside_boundary = (rec2.t - rec1.t) * ray_length;
    const double neg_inv_density = -1.0 / x->v[0];
    const double hit_distance = neg_inv_density * oracle_log(medium_draw(cx->seed, obj, cx->sample, cx->pixel, cx->seg));
    if (!(hit_distance < distance_inside_boundary)) return 0;
    rec->t = rec1.t + hit_distance / ray_length;
    rec->u = 0.0; rec->v = 0.0;
    rec->p = ray_at(r, rec->t);
    rec->normal = V(1.0, 0.0, 0.0);
    rec->front_face = 1;
    return 1;
  }
  if (x->kind == YART_XF_TRANSLATE) {
    v3 off = V(x->v[0], x->v[1], x->v[2]);
    ray_t moved = {vsub(r->o, off), r->d, r->time, r->wl};
    if (!object_hit(s, o, sc, level + 1, &moved, t_min, t_max, rec, cx, obj)) return 0;
    rec->p = vadd(rec->p, off);
    return 1;
  }
  if (x->kind == YART_XF_ROTATE_Y) {
    double sn = sc[level][0], cs = sc[level][1];
    ray_t rot = *r;
    rot.o.x = cs * r->o.x - sn * r->o.z;
    rot.o.z = sn * r->o.x + cs * r->o.z;
    rot.d.x = cs * r->d.x - sn * r->d.z;
    rot.d.z = sn * r->d.x + cs * r->d.z;
    if (!object_hit(s, o, sc, level + 1, &rot, t_min, t_max, rec, cx, obj)) return 0;
    v3 p = rec->p, n = rec->normal;
    rec->p.x = cs * p.x + sn * p.z;
    rec->p.z = -sn * p.x + cs * p.z;
    rec->normal.x = cs * n.x + sn * n.z;
    rec->normal.z = -sn * n.x + cs * n.z;
    return 1;
  }
  /* FLIP_FACE */
  if (!object_hit(s, o, sc, level + 1, r, t_min, t_max, rec, cx, obj)) return 0;
  rec->front_face = !rec->front_face;
  return 1;
}

static int world_hit(const oracle_scene* s, const ray_t* r, double t_min, double t_max, hit_rec* rec, int32_t* which,
                     const wctx_t* cx) { /* hittable.rs:67-79 */
  int found = 0; double closest = t_max; hit_rec tmp;
  for (uint32_t i = 0; i < s->nobj; ++i) {
    if (object_hit(s, &s->objects[i], (const double (*)[2])s->obj_sc[i], 0, r, t_min, closest, &tmp, cx, i)) {
      closest = tmp.t;
      tmp.mat = s->objects[i].material;
      *rec = tmp; found = 1;
      if (which) *which = (int32_t)i;
    }
  }
  return found;
}

/* ------------------------------------------------------------------ ONB / PDFs */
typedef struct { v3 u, v, w; } onb_t;
static onb_t onb_from_w(v3 n) { /* onb.rs:10-21 */
  onb_t b;
  b.w = unit_vector(n);
  v3 a = fabs(b.w.x) > 0.9 ? V(0.0, 1.0, 0.0) : V(1.0, 0.0, 0.0);
  b.v = unit_vector(cross(b.w, a));
  b.u = cross(b.w, b.v);
  return b;
}
static v3 onb_local(const onb_t* b, v3 a) { /* onb.rs:23-25 */
  return vadd(vadd(smulv(a.x, b->u), smulv(a.y, b->v)), smulv(a.z, b->w));
}
static v3 random_cosine_direction(rng_t* g) { /* pdf.rs:15-25 */
  double r1 = gen_f64(g), r2 = gen_f64(g);
  double z = sqrt(1.0 - r2);
  double phi = 2.0 * PI * r1;
  double x = oracle_cos(phi) * sqrt(r2);
  double y = oracle_sin(phi) * sqrt(r2);
  return V(x, y, z);
}
static double cosine_pdf_value(const onb_t* b, v3 dir) { /* pdf.rs:40-47 */
  double cosine = dot(unit_vector(dir), b->w);
  return cosine <= 0.0 ? 0.0 : cosine / PI;
}
static v3 random_to_sphere(rng_t* g, double radius, double dist2) { /* sphere.rs:11-21 */
  double r1 = gen_f64(g), r2 = gen_f64(g);
  double z = 1.0 + r2 * (sqrt(1.0 - radius * radius / dist2) - 1.0);
  double phi = 2.0 * PI * r1;
  double x = oracle_cos(phi) * sqrt(1.0 - z * z);
  double y = oracle_sin(phi) * sqrt(1.0 - z * z);
  return V(x, y, z);
}
/* Hittable::pdf_value for one light-list entry: XZRect (aarect.rs:148-162), StillSphere
 * (sphere.rs:95-110); every other entry, wrapped ones included, has the trait default 0. */
static double light_pdf_value(const yart_object* o, v3 origin, v3 dir, double wl) {
  if (o->n_xforms != 0) return 0.0;
  ray_t r = {origin, dir, 0.0, wl};
  hit_rec rec;
  if (o->kind == YART_PRIM_XZ_RECT) {
    if (!rect_hit(YART_PRIM_XZ_RECT, o->p, &r, 0.001, INFINITY, &rec)) return 0.0;
    double area = (o->p[1] - o->p[0]) * (o->p[3] - o->p[2]);
    double distance_squared = rec.t * rec.t * length_squared(dir);
    double cosine = fabs(dot(dir, rec.normal)) / length(dir);
    return distance_squared / (cosine * area);
  }
  if (o->kind == YART_PRIM_SPHERE) {
    if (!sphere_hit(o->p, &r, 0.001, INFINITY, &rec)) return 0.0;
    v3 center = V(o->p[0], o->p[1], o->p[2]);
    double radius = o->p[3];
    double cos_theta_max = sqrt(1.0 - radius * radius / length_squared(vsub(center, origin)));
    double solid_angle = 2.0 * PI * (1.0 - cos_theta_max);
    return 1.0 / solid_angle;
  }
  return 0.0;
}
/* Hittable::random: XZRect (aarect.rs:164-171), StillSphere (sphere.rs:112-118), default (1,0,0). */
static v3 light_random(const yart_object* o, v3 origin, rng_t* g) {
  if (o->n_xforms == 0 && o->kind == YART_PRIM_XZ_RECT) {
    double x = gen_range_f64(g, o->p[0], o->p[1]);
    double z = gen_range_f64(g, o->p[2], o->p[3]);
    return vsub(V(x, o->p[4], z), origin);
  }
  if (o->n_xforms == 0 && o->kind == YART_PRIM_SPHERE) {
    v3 direction = vsub(V(o->p[0], o->p[1], o->p[2]), origin);
    double d2 = length_squared(direction);
    onb_t uvw = onb_from_w(direction);
    v3 rs = random_to_sphere(g, o->p[3], d2);
    return onb_local(&uvw, rs);
  }
  return V(1.0, 0.0, 0.0);
}
static double lights_pdf_value(const oracle_scene* s, v3 origin, v3 dir, double wl) { /* hittable.rs:103-111 */
  double weight = 1.0 / (double)s->nlights;
  double sum = -0.0; /* <f64 as Sum>::sum folds from -0.0 */
  for (uint32_t i = 0; i < s->nlights; ++i) sum = sum + weight * light_pdf_value(&s->lights[i], origin, dir, wl);
  return sum;
}
static v3 lights_random(const oracle_scene* s, v3 origin, rng_t* g) { /* hittable.rs:113-122 */
  if (s->nlights == 0) return V(1.0, 0.0, 0.0);
  if (s->nlights == 1) return light_random(&s->lights[0], origin, g);
  uint64_t k = gen_range_usize(g, s->nlights - 1); /* never the last light (0..len-1) */
  return light_random(&s->lights[k], origin, g);
}

/* ------------------------------------------------------------------ textures / materials */
/* f64::clamp (propagates NaN) and Rust `f as u32` (saturating, NaN -> 0). */
static double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
static uint32_t sat_u32(double f) {
  if (!(f > 0.0)) return 0;
  if (f >= 4294967295.0) return UINT32_MAX;
  return (uint32_t)f;
}
/* Rust `f as i32`: saturating, NaN -> 0. */
static int32_t sat_i32(double f) {
  if (f != f) return 0;
  if (f >= 2147483647.0) return INT32_MAX;
  if (f <= -2147483648.0) return INT32_MIN;
  return (int32_t)f;
}
/* Perlin::noise (texture.rs:114-180) */
static double perlin_noise(const yart_perlin* P, uint32_t type, v3 p) {
  if (type == YART_NOISE_SQUARE) {
    const int32_t i = sat_i32(4.0 * p.x) & 255, j = sat_i32(4.0 * p.y) & 255, k = sat_i32(4.0 * p.z) & 255;
    return P->ranfloat[P->perm_x[i] ^ P->perm_y[j] ^ P->perm_z[k]];
  }
  double u = p.x - floor(p.x), v = p.y - floor(p.y), w = p.z - floor(p.z);
  const int32_t i = sat_i32(floor(p.x)), j = sat_i32(floor(p.y)), k = sat_i32(floor(p.z));
  double accum = 0.0;
  if (type == YART_NOISE_TRILINEAR) {
    u = u * u * (3.0 - 2.0 * u);
    v = v * v * (3.0 - 2.0 * v);
    w = w * w * (3.0 - 2.0 * w);
    for (int di = 0; di < 2; ++di)
      for (int dj = 0; dj < 2; ++dj)
        for (int dk = 0; dk < 2; ++dk) { /* trilinear_interp texture.rs:192-207 */
          const double c = P->ranfloat[P->perm_x[((uint32_t)i + (uint32_t)di) & 255u] ^ P->perm_y[((uint32_t)j + (uint32_t)dj) & 255u] ^
                                       P->perm_z[((uint32_t)k + (uint32_t)dk) & 255u]];
          accum += ((double)di * u + (double)(1 - di) * (1.0 - u)) * ((double)dj * v + (double)(1 - dj) * (1.0 - v)) *
                   ((double)dk * w + (double)(1 - dk) * (1.0 - w)) * c;
        }
    return accum;
  }
  const double uu = u * u * (3.0 - 2.0 * u), vv = v * v * (3.0 - 2.0 * v), ww = w * w * (3.0 - 2.0 * w);
  for (int di = 0; di < 2; ++di)
    for (int dj = 0; dj < 2; ++dj)
      for (int dk = 0; dk < 2; ++dk) { /* perlin_interp texture.rs:209-228 */
        const double* c = P->ranvec[P->perm_x[((uint32_t)i + (uint32_t)di) & 255u] ^ P->perm_y[((uint32_t)j + (uint32_t)dj) & 255u] ^
                                    P->perm_z[((uint32_t)k + (uint32_t)dk) & 255u]];
        const v3 weight_v = V(u - (double)di, v - (double)dj, w - (double)dk);
        accum += ((double)di * uu + (1.0 - (double)di) * (1.0 - uu)) * ((double)dj * vv + (1.0 - (double)dj) * (1.0 - vv)) *
                 ((double)dk * ww + (1.0 - (double)dk) * (1.0 - ww)) * dot(weight_v, V(c[0], c[1], c[2]));
      }
  return accum;
}
static double perlin_turb(const yart_perlin* P, uint32_t type, v3 p, int depth) { /* texture.rs:230-242 */
  double accum = 0.0, weight = 1.0;
  v3 temp_p = p;
  for (int d = 0; d < depth; ++d) {
    accum += weight * perlin_noise(P, type, temp_p);
    weight *= 0.5;
    temp_p = vmuls(temp_p, 2.0);
  }
  return fabs(accum);
}

static double texture_value(const oracle_scene* s, uint32_t ti, const ray_t* r, const hit_rec* rec) {
  const yart_texture* t = &s->texs[ti];
  if (t->kind == YART_TEX_IMAGE) { /* ImageTexture::value texture.rs:320-344 */
    if (!t->pixels || t->width == 0 || t->height == 0) return 1.0;
    const double uu = clampd(rec->u, 0.0, 1.0), vv = 1.0 - clampd(rec->v, 0.0, 1.0);
    uint32_t i = sat_u32(uu * (double)t->width), j = sat_u32(vv * (double)t->height);
    if (i >= t->width) i = t->width - 1;
    if (j >= t->height) j = t->height - 1;
    const double color_scale = 1.0 / 255.0;
    const uint8_t* px = &t->pixels[(size_t)j * t->width * 3 + (size_t)i * 3];
    const double rgb[3] = {color_scale * (double)px[0], color_scale * (double)px[1], color_scale * (double)px[2]};
    return oracle_rgb_reflect(rgb, r->wl);
  }
  if (t->kind == YART_TEX_NOISE) { /* NoiseTexture::value texture.rs:265-300 (rgb = white) */
    const double white = oracle_rgb_reflect(t->rgb, r->wl);
    if (t->noise_type == YART_NOISE_NET) return white * perlin_turb(t->perlin, t->noise_type, vmuls(rec->p, t->scale), 7);
    if (t->noise_type == YART_NOISE_MARBLE)
      return white * 0.5 * (1.0 + oracle_sin(t->scale * rec->p.z + 10.0 * perlin_turb(t->perlin, t->noise_type, rec->p, 7)));
    return white * 0.5 * (1.0 + perlin_noise(t->perlin, t->noise_type, vmuls(rec->p, t->scale)));
  }
  if (t->kind == YART_TEX_CHECKER) { /* texture.rs:58-67 */
    double sines = oracle_sin(10.0 * rec->p.x) * oracle_sin(10.0 * rec->p.y) * oracle_sin(10.0 * rec->p.z);
    return sines < 0.0 ? oracle_rgb_reflect(t->rgb, r->wl) : oracle_rgb_reflect(t->rgb_even, r->wl);
  }
  return oracle_rgb_reflect(t->rgb, r->wl); /* SolidColor texture.rs:37-39 */
}
static v3 reflect(v3 v, v3 n) { return vsub(v, smulv(2.0 * dot(v, n), n)); } /* material.rs:75-77 */
static int refract(v3 v, v3 n, double ni_over_nt, v3* out) { /* material.rs:195-205 */
  v3 uv = unit_vector(v);
  double dt = dot(uv, n);
  double disc = 1.0 - ni_over_nt * ni_over_nt * (1.0 - dt * dt);
  if (disc > 0.0) { *out = vsub(vmuls(vsub(uv, vmuls(n, dt)), ni_over_nt), vmuls(n, sqrt(disc))); return 1; }
  return 0;
}
double oracle_schlick(double cosine, double ref_idx) { /* material.rs:207-211 */
  double r0 = (1.0 - ref_idx) / (1.0 + ref_idx);
  r0 = r0 * r0;
  return r0 + (1.0 - r0) * powi5(1.0 - cosine);
}
double oracle_sellmeier_index(const double b[3], const double c[3], double wl) { /* material.rs:251-257 */
  double wl2 = wl * wl;
  double n2 = 1.0 + b[0] * wl2 / (wl2 - c[0]) + b[1] * wl2 / (wl2 - c[1]) + b[2] * wl2 / (wl2 - c[2]);
  return sqrt(n2);
}
static v3 random_in_unit_sphere(rng_t* g) { /* material.rs:308-324 */
  for (;;) {
    double x = gen_range_f64(g, -1.0, 1.0), y = gen_range_f64(g, -1.0, 1.0), z = gen_range_f64(g, -1.0, 1.0);
    v3 p = V(x, y, z);
    if (length_squared(p) >= 1.0) continue;
    return p;
  }
}
static v3 random_in_unit_disk(rng_t* g) { /* camera.rs:25-33 */
  v3 p;
  do { double x = gen_range_f64(g, -1.0, 1.0); double y = gen_range_f64(g, -1.0, 1.0); p = V(x, y, 0.0); } while (length_squared(p) >= 1.0);
  return p;
}
static ray_t camera_get_ray(const yart_camera* c, double s, double t, double wl, rng_t* g, int draw_time) { /* camera.rs:82-94 */
  v3 rd = smulv(c->lens_radius, random_in_unit_disk(g));
  v3 cu = V(c->u[0], c->u[1], c->u[2]), cv = V(c->v[0], c->v[1], c->v[2]);
  v3 offset = vadd(vmuls(cu, rd.x), vmuls(cv, rd.y));
  v3 org = V(c->origin[0], c->origin[1], c->origin[2]);
  v3 llc = V(c->lower_left_corner[0], c->lower_left_corner[1], c->lower_left_corner[2]);
  v3 hor = V(c->horizontal[0], c->horizontal[1], c->horizontal[2]);
  v3 ver = V(c->vertical[0], c->vertical[1], c->vertical[2]);
  ray_t r;
  r.o = vadd(org, offset);
  r.d = vsub(vsub(vadd(vadd(llc, smulv(s, hor)), smulv(t, ver)), org), offset);
  /* gen_range(time0..time1) (camera.rs:91): drawn only when a MovingSphere can read it */
  r.time = draw_time ? gen_range_f64(g, c->time0, c->time1) : c->time0;
  r.wl = wl;
  return r;
}

/* One bounce of ray_reflectance (main.rs:537-588). Returns 1 and sets *ray_out / factors when
 * the path continues, 0 with *terminal when it ends. kind: 0 specular (R = att * next),
 * 1 pdf branch (R = att * next * spdf / pdf). */
typedef struct { int cont; int kind; double att, spdf, pdf; double terminal; ray_t next; } bounce_t;

static void bounce(const oracle_scene* s, const ray_t* r, rng_t* g, uint32_t phase, bounce_t* b) {
  hit_rec rec;
  rng_phase(g, phase);
  b->cont = 0;
  const wctx_t cx = {((uint64_t)g->key[1] << 32) | g->key[0], g->ctr[1], g->ctr[2], phase};
  if (!world_hit(s, r, 0.001, INFINITY, &rec, NULL, &cx)) {
    b->terminal = oracle_rgb_reflect(s->background, r->wl); /* main.rs:587 */
    return;
  }
  const yart_material* m = &s->mats[rec.mat];
  double emitted = 0.0;
  if (m->kind == YART_MAT_DIFFUSE_LIGHT) /* material.rs:347-355 */
    emitted = rec.front_face ? texture_value(s, m->texture, r, &rec) : 0.0;
  switch (m->kind) {
    case YART_MAT_LAMBERTIAN: { /* material.rs:44-61 + main.rs:556-581 */
      double att = texture_value(s, m->texture, r, &rec);
      onb_t uvw = onb_from_w(rec.normal);
      v3 dir;
      double pdf_val;
      if (s->nlights == 0) { /* MixurePDF(cos, cos) */
        if (gen_range_f64(g, 0.0, 1.0) < 0.5) dir = onb_local(&uvw, random_cosine_direction(g));
        else dir = onb_local(&uvw, random_cosine_direction(g));
        pdf_val = 0.5 * cosine_pdf_value(&uvw, dir) + 0.5 * cosine_pdf_value(&uvw, dir);
      } else { /* MixurePDF(HittablePDF(lights, p), cos) */
        if (gen_range_f64(g, 0.0, 1.0) < 0.5) dir = lights_random(s, rec.p, g);
        else dir = onb_local(&uvw, random_cosine_direction(g));
        pdf_val = 0.5 * lights_pdf_value(s, rec.p, dir, r->wl) + 0.5 * cosine_pdf_value(&uvw, dir);
      }
      if (!isfinite(pdf_val) || pdf_val <= 0.0) { b->terminal = emitted; return; }
      double cosine = dot(rec.normal, unit_vector(dir)); /* Lambertian::scatter_pdf */
      double spdf = cosine < 0.0 ? 0.0 : cosine / PI;
      b->cont = 1; b->kind = 1; b->att = att; b->spdf = spdf; b->pdf = pdf_val;
      b->next.o = rec.p; b->next.d = dir; b->next.time = r->time; b->next.wl = r->wl;
      return;
    }
    case YART_MAT_METAL: { /* material.rs:79-95 */
      v3 reflected = reflect(unit_vector(r->d), rec.normal);
      v3 fz = smulv(m->fuzz, random_in_unit_sphere(g));
      double att = texture_value(s, m->texture, r, &rec);
      b->cont = 1; b->kind = 0; b->att = att;
      b->next.o = rec.p; b->next.d = vadd(reflected, fz); b->next.time = r->time; b->next.wl = r->wl;
      return;
    }
    case YART_MAT_ISOTROPIC: { /* material.rs:370-381: attenuation, then a random_in_unit_sphere direction */
      double att = texture_value(s, m->texture, r, &rec);
      v3 dir = random_in_unit_sphere(g);
      b->cont = 1; b->kind = 0; b->att = att;
      b->next.o = rec.p; b->next.d = dir; b->next.time = r->time; b->next.wl = r->wl;
      return;
    }
    case YART_MAT_DIELECTRIC: { /* material.rs:213-301 */
      double n = oracle_sellmeier_index(m->b, m->c, r->wl);
      v3 outward; double ni_over_nt, cosine;
      double dn = dot(r->d, rec.normal);
      if (dn > 0.0) { outward = vneg(rec.normal); ni_over_nt = n; cosine = n * dot(r->d, rec.normal) / length(r->d); }
      else { outward = rec.normal; ni_over_nt = 1.0 / n; cosine = -dot(r->d, rec.normal) / length(r->d); }
      v3 refracted, out;
      if (refract(r->d, outward, ni_over_nt, &refracted)) {
        if (gen_f64(g) < oracle_schlick(cosine, n)) out = reflect(r->d, rec.normal);
        else out = refracted;
      } else {
        out = reflect(r->d, rec.normal);
      }
      b->cont = 1; b->kind = 0; b->att = 1.0;
      b->next.o = rec.p; b->next.d = out; b->next.time = r->time; b->next.wl = r->wl;
      return;
    }
    default: /* DiffuseLight / NoMaterial: no scatter, R = emitted */
      b->terminal = emitted;
      return;
  }
}

static double reflectance_recursive(const oracle_scene* s, const ray_t* r, rng_t* g, uint32_t depth,
                                    uint32_t max_depth) { /* main.rs:537-588 */
  if (depth == 0) return 1.0;
  bounce_t b;
  bounce(s, r, g, max_depth - depth + 1, &b);
  if (!b.cont) return b.terminal;
  if (b.kind == 0) return b.att * reflectance_recursive(s, &b.next, g, depth - 1, max_depth);
  return b.att * reflectance_recursive(s, &b.next, g, depth - 1, max_depth) * b.spdf / b.pdf;
}
/* The same recursion unrolled front to back: T accumulates att (and * spdf / pdf); the
 * terminal value multiplies last. Equal to the recursive form up to rounding order. */
static double reflectance_iterative(const oracle_scene* s, const ray_t* r0, rng_t* g, uint32_t depth) {
  const uint32_t max_depth = depth;
  double T = 1.0;
  ray_t r = *r0;
  for (;;) {
    if (depth == 0) return T * 1.0;
    bounce_t b;
    bounce(s, &r, g, max_depth - depth + 1, &b);
    if (!b.cont) return T * b.terminal;
    if (b.kind == 0) T = T * b.att;
    else T = ((T * b.att) * b.spdf) / b.pdf;
    r = b.next;
    depth--;
  }
}

/* --------------------------------------------------------------------- render loop */
static void coverage_axes(uint32_t w, uint32_t h, uint8_t* cx, uint8_t* cy) { /* main.rs:636-647 */
  memset(cx, 0, w); memset(cy, 0, h);
  for (uint32_t col = 0; col < 8; ++col) {
    uint32_t x0 = (uint32_t)(((uint64_t)w * col) / 8), cw = w / 8;
    for (uint32_t x = x0; x < x0 + cw && x < w; ++x) cx[x] = 1;
  }
  for (uint32_t row = 0; row < 8; ++row) {
    uint32_t y0 = (uint32_t)(((uint64_t)h * row) / 8), ch = h / 8;
    for (uint32_t y = y0; y < y0 + ch && y < h; ++y) cy[y] = 1;
  }
}
int oracle_coverage(uint32_t w, uint32_t h, uint8_t* mask) {
  uint8_t* cx = (uint8_t*)malloc(w); uint8_t* cy = (uint8_t*)malloc(h);
  coverage_axes(w, h, cx, cy);
  for (uint32_t y = 0; y < h; ++y) for (uint32_t x = 0; x < w; ++x) mask[(size_t)y * w + x] = cx[x] && cy[y];
  free(cx); free(cy);
  return 0;
}

typedef struct {
  const oracle_scene* s; const yart_camera* cam; const yart_render_params* p;
  double* out; const uint8_t* cx; const uint8_t* cy; int mode; int chacha;
  volatile int next_row; pthread_mutex_t mu;
} job_t;

static void render_pixel(const job_t* j, uint32_t x, uint32_t y) {
  const yart_render_params* p = j->p;
  uint32_t W = p->width, H = p->height;
  uint32_t pixel = y * W + x;
  double acc[3] = {0.0, 0.0, 0.0};
  for (uint32_t smp = 0; smp < p->spp; ++smp) { /* main.rs:691-708 */
    rng_t g;
    if (j->chacha) rng_init_chacha(&g, p->seed, pixel, smp);
    else rng_init(&g, p->seed, pixel, smp, 0);
    double tx = (double)x + gen_f64(&g);
    double u = tx / (double)(W - 1);
    double ty = (double)y + gen_f64(&g);
    double v = 1.0 - ty / (double)(H - 1);
    double wl = gen_range_f64(&g, MIN_LAMBDA, MAX_LAMBDA); /* color.rs:20-23 */
    ray_t r = camera_get_ray(j->cam, u, v, wl, &g, j->s->has_time);
    double R = j->mode ? reflectance_recursive(j->s, &r, &g, p->max_depth, p->max_depth)
                       : reflectance_iterative(j->s, &r, &g, p->max_depth);
    double cie[3], xyz[3], san[3];
    oracle_xyz_from_wavelength(r.wl, cie); /* ray_color main.rs:526-535 */
    xyz[0] = cie[0] * R; xyz[1] = cie[1] * R; xyz[2] = cie[2] * R;
    oracle_sanitize_sample_xyz(xyz, san);
    acc[0] = acc[0] + san[0]; acc[1] = acc[1] + san[1]; acc[2] = acc[2] + san[2];
  }
  double* o = &j->out[3 * (size_t)pixel];
  o[0] = acc[0]; o[1] = acc[1]; o[2] = acc[2];
}

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  uint32_t W = j->p->width, H = j->p->height;
  uint32_t bw = (W + 7) / 8;
  uint32_t sc = j->p->shard_count ? j->p->shard_count : 1, si = j->p->shard_index;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    int y = j->next_row++;
    pthread_mutex_unlock(&j->mu);
    if ((uint32_t)y >= H) break;
    if (!j->cy[y]) continue;
    for (uint32_t x = 0; x < W; ++x) {
      if (!j->cx[x]) continue;
      uint32_t blk = ((uint32_t)y / 8) * bw + x / 8;
      if (sc > 1 && blk % sc != si) continue;
      render_pixel(j, x, (uint32_t)y);
    }
  }
  return NULL;
}

int oracle_render(const oracle_scene* s, const yart_camera* cam, const yart_render_params* p,
                  double* xyz_sum, int threads, int mode) {
  if (!s || !cam || !p || !xyz_sum || p->width == 0 || p->height == 0) return YART_ERR_INVALID;
  if (p->shard_count > 1 && p->shard_index >= p->shard_count) return YART_ERR_INVALID;
  if (threads <= 0) threads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (threads < 1) threads = 1;
  job_t j;
  j.s = s; j.cam = cam; j.p = p; j.out = xyz_sum; j.mode = mode & 1; j.chacha = (mode & 2) != 0; j.next_row = 0;
  uint8_t* cx = (uint8_t*)malloc(p->width); uint8_t* cy = (uint8_t*)malloc(p->height);
  coverage_axes(p->width, p->height, cx, cy);
  j.cx = cx; j.cy = cy;
  pthread_mutex_init(&j.mu, NULL);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
  for (int i = 0; i < threads; ++i) pthread_create(&th[i], NULL, worker, &j);
  for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
  pthread_mutex_destroy(&j.mu);
  free(th); free(cx); free(cy);
  return YART_OK;
}

int oracle_finalize_rgba8(const double* xyz_sum, uint32_t w, uint32_t h, uint32_t spp, uint8_t* rgba) { /* main.rs:710-718 */
  uint8_t* cx = (uint8_t*)malloc(w); uint8_t* cy = (uint8_t*)malloc(h);
  coverage_axes(w, h, cx, cy);
  double den = CIE_Y_INTERGAL * (double)spp;
  for (uint32_t y = 0; y < h; ++y)
    for (uint32_t x = 0; x < w; ++x) {
      size_t i = (size_t)y * w + x;
      uint8_t* o = &rgba[4 * i];
      if (!(cx[x] && cy[y])) { o[0] = o[1] = o[2] = o[3] = 0; continue; }
      v3 xyz = V(xyz_sum[3 * i], xyz_sum[3 * i + 1], xyz_sum[3 * i + 2]);
      xyz = vdivs(vmuls(xyz, MAX_LAMBDA - MIN_LAMBDA), den);
      double in[3] = {xyz.x, xyz.y, xyz.z}, rgb[3], gam[3];
      oracle_xyz_into_rgb(in, rgb);
      oracle_gamma_corrected(rgb, gam);
      o[0] = oracle_clamp_display_channel(gam[0]);
      o[1] = oracle_clamp_display_channel(gam[1]);
      o[2] = oracle_clamp_display_channel(gam[2]);
      o[3] = 255;
    }
  free(cx); free(cy);
  return YART_OK;
}

double oracle_texture_probe(const oracle_scene* s, uint32_t tex, double wl, const double p[3], double u, double v) {
  ray_t r = {V(0.0, 0.0, 0.0), V(1.0, 0.0, 0.0), 0.0, wl};
  hit_rec rec;
  memset(&rec, 0, sizeof rec);
  rec.p = V(p[0], p[1], p[2]);
  rec.u = u; rec.v = v;
  return texture_value(s, tex, &r, &rec);
}

int oracle_intersect(const oracle_scene* s, const double* rays, uint32_t n, double* hits, int32_t* obj) {
  for (uint32_t i = 0; i < n; ++i) {
    const double* q = &rays[8 * (size_t)i];
    ray_t r = {V(q[0], q[1], q[2]), V(q[3], q[4], q[5]), 0.0, 0.0};
    hit_rec rec; int32_t which = -1;
    double* h = &hits[8 * (size_t)i];
    const wctx_t cx = {0, 0, i, 0};  /* a medium's draw for query i: seed 0, sample 0, pixel i */
    if (world_hit(s, &r, q[6], q[7], &rec, &which, &cx)) {
      h[0] = rec.t; h[1] = rec.p.x; h[2] = rec.p.y; h[3] = rec.p.z;
      h[4] = rec.normal.x; h[5] = rec.normal.y; h[6] = rec.normal.z; h[7] = rec.front_face ? 1.0 : 0.0;
    } else {
      for (int k = 0; k < 8; ++k) h[k] = NAN;
    }
    obj[i] = which;
  }
  return YART_OK;
}

/* ------------------------------------------------------------------ scene lifetime */
static void rotate_sc(const yart_object* objs, uint32_t n, double (*sc)[YART_MAX_XFORMS][2]) {
  for (uint32_t i = 0; i < n; ++i)
    for (uint32_t l = 0; l < objs[i].n_xforms && l < YART_MAX_XFORMS; ++l) {
      sc[i][l][0] = sc[i][l][1] = 0.0;
      if (objs[i].xforms[l].kind == YART_XF_ROTATE_Y) { /* hittable.rs:173-176, camera.rs:35-37 */
        double radians = objs[i].xforms[l].v[0] * PI / 180.0;
        sc[i][l][0] = sin(radians);
        sc[i][l][1] = cos(radians);
      }
    }
}

static int check_objects(const yart_scene_desc* d, const yart_object* o, uint32_t n) {
  for (uint32_t i = 0; i < n; ++i) {
    if (o[i].kind > YART_PRIM_MOVING_SPHERE || o[i].n_xforms > YART_MAX_XFORMS) return 0;
    if (o[i].kind == YART_PRIM_MESH && o[i].mesh >= d->n_meshes) return 0;
    if (o[i].material >= d->n_materials && d->n_materials) return 0;
    for (uint32_t l = 0; l < o[i].n_xforms; ++l)
      if (o[i].xforms[l].kind < YART_XF_TRANSLATE || o[i].xforms[l].kind > YART_XF_MEDIUM ||
          (o[i].xforms[l].kind == YART_XF_MEDIUM && l != 0))
        return 0;
  }
  return 1;
}

int oracle_scene_create(const yart_scene_desc* d, oracle_scene** out) {
  if (!d || !out || d->abi_version != YART_ABI_VERSION) return YART_ERR_INVALID;
  if (!check_objects(d, d->objects, d->n_objects) || !check_objects(d, d->lights, d->n_lights)) return YART_ERR_INVALID;
  for (uint32_t i = 0; i < d->n_materials; ++i)
    if (d->materials[i].kind > YART_MAT_ISOTROPIC ||
        ((d->materials[i].kind == YART_MAT_LAMBERTIAN || d->materials[i].kind == YART_MAT_METAL ||
          d->materials[i].kind == YART_MAT_DIFFUSE_LIGHT || d->materials[i].kind == YART_MAT_ISOTROPIC) &&
         d->materials[i].texture >= d->n_textures))
      return YART_ERR_INVALID;
  for (uint32_t i = 0; i < d->n_textures; ++i)
    if (d->textures[i].kind > YART_TEX_IMAGE ||
        (d->textures[i].kind == YART_TEX_NOISE && (!d->textures[i].perlin || d->textures[i].noise_type > YART_NOISE_NET)))
      return YART_ERR_INVALID;
  for (uint32_t i = 0; i < d->n_objects; ++i)
    if (d->objects[i].material >= d->n_materials) return YART_ERR_INVALID;
  oracle_scene* s = (oracle_scene*)calloc(1, sizeof(oracle_scene));
  s->nobj = d->n_objects; s->nlights = d->n_lights; s->nmats = d->n_materials; s->ntexs = d->n_textures;
  s->objects = (yart_object*)malloc(sizeof(yart_object) * (s->nobj + 1));
  s->lights = (yart_object*)malloc(sizeof(yart_object) * (s->nlights + 1));
  s->mats = (yart_material*)malloc(sizeof(yart_material) * (s->nmats + 1));
  s->texs = (yart_texture*)malloc(sizeof(yart_texture) * (s->ntexs + 1));
  if (s->nobj) memcpy(s->objects, d->objects, sizeof(yart_object) * s->nobj);
  if (s->nlights) memcpy(s->lights, d->lights, sizeof(yart_object) * s->nlights);
  if (s->nmats) memcpy(s->mats, d->materials, sizeof(yart_material) * s->nmats);
  if (s->ntexs) memcpy(s->texs, d->textures, sizeof(yart_texture) * s->ntexs);
  s->perlins = (yart_perlin*)calloc(s->ntexs + 1, sizeof(yart_perlin)); /* own copies of the tables */
  s->images = (uint8_t**)calloc(s->ntexs + 1, sizeof(uint8_t*));        /* and of the texels */
  for (uint32_t i = 0; i < s->ntexs; ++i) {
    if (s->texs[i].kind == YART_TEX_NOISE) { s->perlins[i] = *d->textures[i].perlin; s->texs[i].perlin = &s->perlins[i]; }
    if (s->texs[i].kind == YART_TEX_IMAGE && s->texs[i].pixels && s->texs[i].width && s->texs[i].height) {
      const size_t n = (size_t)s->texs[i].width * s->texs[i].height * 3;
      s->images[i] = (uint8_t*)malloc(n);
      memcpy(s->images[i], d->textures[i].pixels, n);
      s->texs[i].pixels = s->images[i];
    }
  }
  memcpy(s->background, d->background, sizeof(s->background));
  for (uint32_t i = 0; i < s->nobj; ++i) s->has_time |= s->objects[i].kind == YART_PRIM_MOVING_SPHERE;
  s->obj_sc = calloc(s->nobj + 1, sizeof(*s->obj_sc));
  s->light_sc = calloc(s->nlights + 1, sizeof(*s->light_sc));
  rotate_sc(s->objects, s->nobj, s->obj_sc);
  rotate_sc(s->lights, s->nlights, s->light_sc);
  s->nmeshes = d->n_meshes;
  s->meshes = (qbvh_t*)calloc(s->nmeshes + 1, sizeof(qbvh_t));
  for (uint32_t m = 0; m < d->n_meshes; ++m) {
    if (build_qbvh(&s->meshes[m], &d->meshes[m]) != 0) { oracle_scene_destroy(s); return YART_ERR_UNSUPPORTED; }
  }
  *out = s;
  return YART_OK;
}

void oracle_scene_destroy(oracle_scene* s) {
  if (!s) return;
  for (uint32_t m = 0; m < s->nmeshes; ++m) {
    qbvh_t* q = &s->meshes[m];
    free(q->vert); free(q->norm); free(q->nodes); free(q->leaves); free(q->leaf_of_first);
  }
  for (uint32_t i = 0; s->images && i < s->ntexs; ++i) free(s->images[i]);
  free(s->meshes); free(s->objects); free(s->lights); free(s->mats); free(s->texs); free(s->perlins); free(s->images);
  free(s->obj_sc); free(s->light_sc);
  free(s);
}

int oracle_qbvh_stats(const oracle_scene* s, uint32_t m, uint32_t* nodes, uint32_t* leaves, uint32_t* depth) {
  if (!s || m >= s->nmeshes) return YART_ERR_INVALID;
  *nodes = s->meshes[m].nnodes; *leaves = s->meshes[m].nleaves; *depth = s->meshes[m].depth;
  return YART_OK;
}
