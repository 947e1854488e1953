// kernels.h — launch interface between the C ABI (capi.cpp) and the HIP kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/yart.h"
#include "device_types.h"

namespace yart_dev {

struct RenderArgs {
  yart_camera cam;
  uint32_t width, height, spp, max_depth;
  uint64_t seed;
  uint32_t shard_index, shard_count;
  uint32_t blocks_x;  // ceil(width / 8)
  uint32_t n_blocks;  // 8x8-pixel blocks owned by this shard
  // Work units = n_blocks x n_chunks; unit u renders block u % n_blocks for samples
  // [s_begin + (u / n_blocks) * chunk, ... + chunk) clipped to [s_begin, s_begin + s_count).
  uint32_t s_begin, s_count, chunk, n_chunks;
  uint32_t* queue;    // chunked path: unit counter (zeroed before each launch), claimed by persistent waves
  uint32_t n_units;   // n_blocks * n_chunks
  uint32_t waves;     // chunked path: resident waves to launch (CUs x 16)
  double* out;        // width * height * 3 (fused path: final sums; written by k_accumulate otherwise)
  double* scratch;    // null = fused; else n_blocks * s_count * 64 * 3 per-sample XYZ
  unsigned long long* stats;  // 8 counters (STATS build only)
};

hipError_t launch_render(const DevScene& s, const RenderArgs& a, bool stats, hipStream_t stream);
// Adds a pass's per-sample values onto the per-pixel sums in sample order (first pass from 0).
hipError_t launch_accumulate(const RenderArgs& a, bool first_pass, hipStream_t stream);
hipError_t launch_intersect(const DevScene& s, const double* rays, uint32_t n, double* hits, int32_t* obj,
                            hipStream_t stream);
hipError_t launch_finalize(const double* xyz, uint32_t w, uint32_t h, uint32_t spp, uint8_t* rgba, hipStream_t stream);
hipError_t launch_probe_rng(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, double* out, hipStream_t stream);
hipError_t launch_probe_math(int op, const double* a, const double* b, uint32_t n, double* out, hipStream_t stream);

}  // namespace yart_dev
