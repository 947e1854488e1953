// Issue cost of the VALU instructions the render kernel is made of, on this MI355X (gfx950).
// Each kernel runs 8 independent chains of one instruction per wave, 4 waves per SIMD (every CU
// busy), and reports SIMD cycles per wave-instruction = s_memtime delta / (waves per SIMD x
// instructions per wave). Build: hipcc --offload-arch=gfx950 -O2 -o ubench_valu ubench_valu.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 256

#define KERNEL(NAME, DECL, BODY)                                                                 \
  __global__ __launch_bounds__(256) void NAME(unsigned long long* cyc, double* sink) {           \
    DECL;                                                                                        \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                 \
    for (int it = 0; it < ITERS; ++it) { BODY; }                                                 \
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                  \
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;                 \
    sink[blockIdx.x * 256 + threadIdx.x] = SINK;                                                 \
  }

// 8 chains of f64 registers
#define D8 double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
           const double b = 1.0000001;
#define U8 uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
           const uint32_t b = 0xD2511F53u;
#define OP8(ASM, C)                                                                              \
  asm volatile(ASM : "+" C(a0) : C(b)); asm volatile(ASM : "+" C(a1) : C(b));                    \
  asm volatile(ASM : "+" C(a2) : C(b)); asm volatile(ASM : "+" C(a3) : C(b));                    \
  asm volatile(ASM : "+" C(a4) : C(b)); asm volatile(ASM : "+" C(a5) : C(b));                    \
  asm volatile(ASM : "+" C(a6) : C(b)); asm volatile(ASM : "+" C(a7) : C(b));

#define SINK (double)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7)
KERNEL(k_add_f64, D8, OP8("v_add_f64 %0, %0, %1", "v"))
KERNEL(k_mul_f64, D8, OP8("v_mul_f64 %0, %0, %1", "v"))
KERNEL(k_fma_f64, D8, OP8("v_fma_f64 %0, %0, %1, %0", "v"))
KERNEL(k_rcp_f64, D8, OP8("v_rcp_f64 %0, %0 ; %1", "v"))
KERNEL(k_sqrt_f64, D8, OP8("v_sqrt_f64 %0, %0 ; %1", "v"))
KERNEL(k_div_fixup_f64, D8, OP8("v_div_fixup_f64 %0, %0, %1, %0", "v"))
KERNEL(k_div_fmas_f64, D8, OP8("v_div_fmas_f64 %0, %0, %1, %0", "v"))
KERNEL(k_cmp_f64, D8, OP8("v_cmp_lt_f64 vcc, %0, %1", "v"))
#undef SINK
#define SINK (double)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7)
KERNEL(k_add_u32, U8, OP8("v_add_u32 %0, %0, %1", "v"))
KERNEL(k_xor_b32, U8, OP8("v_xor_b32 %0, %0, %1", "v"))
KERNEL(k_mul_lo_u32, U8, OP8("v_mul_lo_u32 %0, %0, %1", "v"))
KERNEL(k_mul_hi_u32, U8, OP8("v_mul_hi_u32 %0, %0, %1", "v"))
KERNEL(k_mul_u32_u24, U8, OP8("v_mul_u32_u24 %0, %0, %1", "v"))
KERNEL(k_mul_hi_u32_u24, U8, OP8("v_mul_hi_u32_u24 %0, %0, %1", "v"))
KERNEL(k_cndmask, U8, OP8("v_cndmask_b32 %0, %0, %1, vcc", "v"))
KERNEL(k_add_f32, U8, OP8("v_add_f32 %0, %0, %1", "v"))
KERNEL(k_rcp_f32, U8, OP8("v_rcp_f32 %0, %0 ; %1", "v"))
KERNEL(k_readlane, U8, OP8("v_readlane_b32 s0, %0, 1\n v_writelane_b32 %0, s0, 2 ; %1", "v"))
#undef SINK
#define SINK (double)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7)
// v_mad_u64_u32: 64-bit destination = 32 x 32 product (+ 64-bit addend)
#define M8 uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
           const uint32_t b = 0xD2511F53u;
#define MAD8(R)                                                                                  \
  asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a0) : "v"(b) : "s0", "s1");       \
  asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a1) : "v"(b) : "s0", "s1");       \
  asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a2) : "v"(b) : "s0", "s1");       \
  asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a3) : "v"(b) : "s0", "s1");       \
  asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a4) : "v"(b) : "s0", "s1");       \
  asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a5) : "v"(b) : "s0", "s1");       \
  asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a6) : "v"(b) : "s0", "s1");       \
  asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %1, %0" : "+v"(a7) : "v"(b) : "s0", "s1");
KERNEL(k_mad_u64_u32, M8, MAD8(0))
// empty loop: overhead baseline
KERNEL(k_empty, U8, asm volatile("" : "+v"(a0)))

typedef void (*kfn)(unsigned long long*, double*);
struct Case { const char* name; kfn f; int per_iter; };

int main() {
  const Case cases[] = {
      {"empty", k_empty, 0},         {"v_add_f64", k_add_f64, 8},     {"v_mul_f64", k_mul_f64, 8},
      {"v_fma_f64", k_fma_f64, 8},   {"v_rcp_f64", k_rcp_f64, 8},     {"v_sqrt_f64", k_sqrt_f64, 8},
      {"v_div_fixup_f64", k_div_fixup_f64, 8}, {"v_div_fmas_f64", k_div_fmas_f64, 8},
      {"v_cmp_lt_f64", k_cmp_f64, 8},
      {"v_add_u32", k_add_u32, 8},   {"v_xor_b32", k_xor_b32, 8},     {"v_mul_lo_u32", k_mul_lo_u32, 8},
      {"v_mul_hi_u32", k_mul_hi_u32, 8}, {"v_mul_u32_u24", k_mul_u32_u24, 8},
      {"v_mul_hi_u32_u24", k_mul_hi_u32_u24, 8}, {"v_cndmask_b32", k_cndmask, 8},
      {"v_add_f32", k_add_f32, 8},   {"v_rcp_f32", k_rcp_f32, 8},     {"v_readlane+v_writelane", k_readlane, 8},
      {"v_mad_u64_u32", k_mad_u64_u32, 8},
  };
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int blocks = cus * 4;  // 4 blocks x 4 waves per CU -> 4 waves per SIMD
  unsigned long long* cyc;
  double* sink;
  (void)hipMalloc(&cyc, sizeof(unsigned long long) * blocks * 4);
  (void)hipMalloc(&sink, sizeof(double) * blocks * 256);
  unsigned long long* h = new unsigned long long[blocks * 4];
  double empty = 0;
  printf("{\"cus\": %d, \"waves_per_simd\": 4, \"iters\": %d, \"results\": [\n", cus, ITERS);
  for (size_t c = 0; c < sizeof(cases) / sizeof(cases[0]); ++c) {
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(cases[c].f, dim3(blocks), dim3(256), 0, 0, cyc, sink);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks * 4, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < blocks * 4; ++i) s += (double)h[i];
    const double mean = s / (blocks * 4);
    if (c == 0) empty = mean;
    const double per = cases[c].per_iter ? (mean - empty) / (4.0 * ITERS * cases[c].per_iter) : 0.0;
    printf("  {\"op\": \"%s\", \"cycles_per_wave\": %.0f, \"simd_cycles_per_wave_instr\": %.2f}%s\n", cases[c].name, mean,
           per, c + 1 < sizeof(cases) / sizeof(cases[0]) ? "," : "");
  }
  printf("]}\n");
  return 0;
}
