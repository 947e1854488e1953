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
  // Work units = n_blocks x n_chunks, block-major: unit u renders block u / n_chunks for samples
  // [s_begin + (u % n_chunks) * chunk, ... + chunk) clipped to [s_begin, s_begin + s_count).
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
  uint32_t* stack_ovf;        // deep meshes: kOvfWords per wave of the grid (the walk stacks' HBM overflow)
};
// Walk-stack overflow of the megakernel for meshes deeper than depth 10 (kernels.hip, qbvh_lane): per
// wave, the cooperative walk's per-quad stacks past their 32 LDS slots (node ids, then entries) and
// the reference-order walk's per-lane stacks past theirs, up to the reference's 64 entries.
constexpr int kOvfQuadWords = (kMaxStackSlots - kStackSlots) * 16;
constexpr int kOvfLaneWords = (kMaxStackSlots - kStackSlots) * 64;
constexpr int kOvfWords = 2 * kOvfQuadWords + kOvfLaneWords;

// Shard s of N owns global blocks s, s + N, s + 2N, ... of the ceil(W/8) x ceil(H/8) grid.
__host__ __device__ inline uint32_t shard_blocks(uint32_t total_blocks, uint32_t shard_index, uint32_t shard_count) {
  return total_blocks > shard_index ? (total_blocks - shard_index + shard_count - 1) / shard_count : 0u;
}

// Wavefront path for mesh scenes (k_wf_shade / k_wf_trace): the state of `pool` path slots in
// HBM, SoA (component-major: o[k * pool + i]), so the traversal kernel runs with the registers of
// the walk alone. A slot keeps its path from bounce to bounce (no compaction: with regeneration
// every slot holds a path until the pass's jobs run out); job == kWfNoJob marks an empty slot.
struct WfSlots {
  double* o;         // 3 * pool: ray origin (x block, y block, z block)
  double* d;         // 3 * pool: ray direction
  double* T;         // pool: throughput so far
  double* wl;        // pool: the path's wavelength
  uint32_t* job;     // pool: (local block, sample - s_begin, slot) as one index = the scratch slot
  uint32_t* depth;   // pool: ray_reflectance's depth argument for the traced ray
  double* ht;        // pool: closest hit t (k_wf_trace)
  double* hu;        // pool: its u
  double* hv;        // pool: its v
  uint32_t* hobj;    // pool: world object hit, kWfMiss if none
  uint32_t* hsub;    // pool: its box face / mesh triangle
  uint32_t* range;   // pool / 256 x 2: each shade workgroup's unused job range [next, end)
};
constexpr uint32_t kWfMiss = 0xFFFFFFFFu, kWfNoJob = 0xFFFFFFFFu;
constexpr uint32_t kWfChunk = 256;  // jobs a shade workgroup claims with one atomic
struct WfArgs {
  WfSlots q;
  uint32_t* alive;       // set (plain store) by every shade workgroup left with a ray this iteration
  uint32_t* alive_next;  // the next iteration's flag: k_wf_trace clears it
  uint32_t* jobs;        // job counter of the pass (device)
  uint32_t total_jobs;   // n_blocks * s_count * 64
  uint32_t pool;         // a multiple of 256
  uint32_t* status;      // host-mapped: k_wf_trace stores this iteration's flag (0 = pass done)
};
hipError_t launch_wf_shade(const DevScene& s, const RenderArgs& a, const WfArgs& w, hipStream_t stream);
hipError_t launch_wf_trace(const DevScene& s, const RenderArgs& a, const WfArgs& w, hipStream_t stream);

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
