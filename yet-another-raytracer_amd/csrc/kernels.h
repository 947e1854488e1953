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
                      // or, packed, n_blocks * 64 * 3 in local-block order (the gather's wire format)
  double* scratch;    // null = fused; else n_blocks * s_count * 64 * 3 per-sample XYZ
  unsigned long long* stats;  // 8 counters (STATS build only)
  uint32_t packed;    // out is block-packed: [local_blk][slot][xyz] (yart_render_packed_async)
  uint32_t progress_base;     // units of earlier passes of this frame
  uint32_t* progress;         // host-mapped word (null = none): a plain store of base + units claimed
                              // (chunked path) or finished (fused path)
  uint32_t* progress_count;   // fused path with progress: device counter of finished units (zeroed per frame)
};

// Shard s of N owns global blocks s, s + N, s + 2N, ... of the ceil(W/8) x ceil(H/8) grid.
__host__ __device__ inline uint32_t shard_blocks(uint32_t total_blocks, uint32_t shard_index, uint32_t shard_count) {
  return total_blocks > shard_index ? (total_blocks - shard_index + shard_count - 1) / shard_count : 0u;
}

hipError_t launch_render(const DevScene& s, const RenderArgs& a, bool stats, hipStream_t stream);
// Adds a pass's per-sample values onto the per-pixel sums in sample order (first pass from 0).
hipError_t launch_accumulate(const RenderArgs& a, bool first_pass, hipStream_t stream);
// Root side of the frame gather: `recv` holds every shard's packed blocks back to back
// (shard r at r * stride doubles); writes the whole W x H x 3 frame (uncovered pixels 0).
hipError_t launch_unpack_shards(const double* recv, uint32_t shards, size_t stride, uint32_t width, uint32_t height,
                                double* frame, hipStream_t stream);
hipError_t launch_intersect(const DevScene& s, const double* rays, uint32_t n, double* hits, int32_t* obj,
                            hipStream_t stream);
hipError_t launch_finalize(const double* xyz, uint32_t w, uint32_t h, uint32_t spp, uint8_t* rgba, hipStream_t stream);
hipError_t launch_probe_rng(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, double* out, hipStream_t stream);
hipError_t launch_probe_math(int op, const double* a, const double* b, uint32_t n, double* out, hipStream_t stream);

}  // namespace yart_dev
