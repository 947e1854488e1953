// scene_impl.h — internals of a yart_scene shared by the C ABI translation units (capi.cpp:
// scene upload and single-device renders; multi.cpp: RCCL communicators and multi-device renders).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/yart.h"
#include "kernels.h"

namespace yart_impl {

int64_t opt(int option);  // yart_debug_set_option's current value (capi.cpp)
int fail(int code, const std::string& m);  // sets the thread-local message, returns code
int ok();
int hip_fail(hipError_t e, const char* what);
#define HIP_TRY(expr, what)                              \
  do {                                                   \
    hipError_t e_ = (expr);                              \
    if (e_ != hipSuccess) return yart_impl::hip_fail(e_, what); \
  } while (0)

class DeviceGuard {  // keep the caller's current device (torch tracks its own)
 public:
  explicit DeviceGuard(int dev) { (void)hipGetDevice(&old_); if (old_ != dev) (void)hipSetDevice(dev); dev_ = dev; }
  ~DeviceGuard() { if (old_ != dev_) (void)hipSetDevice(old_); }
 private:
  int old_ = 0, dev_ = 0;
};

// Per-stream render state. A frame's launches (unit-counter reset, render, accumulate per pass)
// are enqueued under `frame_mu`, so two host threads submitting to one stream cannot interleave
// their passes over the shared scratch; the stream then orders the frames on the device.
struct StreamState {
  std::mutex frame_mu;
  double* scratch = nullptr;  // per-sample XYZ of the chunked path + the unit counter at its end
  size_t bytes = 0;
  // wavefront path (mesh scenes): two path queues of `wf_pool` slots, the queue counters and the
  // host-mapped status ring the iterations report into
  void* wf_mem = nullptr;
  size_t wf_bytes = 0;
  uint32_t wf_pool = 0;
  uint32_t* wf_status_host = nullptr;
  uint32_t* wf_status_dev = nullptr;
  uint64_t wf_iter = 0;  // wavefront iterations launched on this stream so far (status-ring slot numbering)
  // deep meshes on the megakernel: the walk stacks' HBM overflow, kOvfWords per wave of a launch
  uint32_t* ovf = nullptr;
  size_t ovf_bytes = 0;
  // frames of more than one scratch pass (capi.cpp launch_frame): the odd passes render on `aux`
  // into the scratch's second half while the even ones finish on the caller's stream, and `acc`
  // adds the passes in order; created with the stream's first such frame
  hipStream_t aux = nullptr, acc = nullptr;
  hipEvent_t ev_start = nullptr, ev_render[2] = {nullptr, nullptr}, ev_acc[2] = {nullptr, nullptr};
};

// Progress of one frame (yart_render's callback): the kernels store `base + units handed out` to
// a host-mapped word; the calling thread polls it while the stream runs (main.rs:720-721 sends a
// Progress message per rendered row instead).
struct Progress {
  uint32_t* host = nullptr;    // host view (hipHostMalloc, coherent)
  uint32_t* device = nullptr;  // the kernels' view of the same word
  uint32_t* counter = nullptr; // device memory: finished units of the fused path (atomic)
  uint32_t total_units = 0;    // over all passes of the frame
  uint64_t pixels = 0;         // covered pixels of the shard
};

}  // namespace yart_impl

struct yart_scene {
  int device = 0;
  int cu_count = 256;
  uint64_t mem_total = 0;  // device memory (hipDeviceTotalMem): sizes the auto scratch budget
  bool wavefront = false;  // mesh scene without EXT features: k_wf_shade / k_wf_trace (deep meshes, YART_OPT_MESH_WAVEFRONT)
  uint32_t wf_pool = 1u << 20;  // paths in flight (YART_OPT_WF_POOL)
  yart_dev::DevScene dev{};
  std::vector<void*> owned;
  yart_scene_info info{};
  std::mutex mu;  // guards the maps and pools below (never held across a device wait)
  std::map<hipStream_t, std::unique_ptr<yart_impl::StreamState>> streams;
  std::vector<hipStream_t> idle_streams;   // library-owned streams for the host-output calls
  std::vector<hipStream_t> owned_streams;
  // kernel-boundary events of the frames launched per stream and not yet read (yart_frame_timing)
  std::map<hipStream_t, std::vector<std::vector<hipEvent_t>>> frames;
  std::vector<hipEvent_t> event_pool;
  ~yart_scene();
};

namespace yart_impl {

int make_args(const yart_scene* s, const yart_camera* cam, const yart_render_params* p, double* out,
              yart_dev::RenderArgs& a);
// Enqueue one frame (all passes) on `stream`. prog: optional progress word (fills total_units).
int launch_frame(yart_scene* s, yart_dev::RenderArgs a, uint32_t requested, bool stats, hipStream_t stream,
                 Progress* prog);
// A library-owned non-blocking stream of the scene's device, exclusively the caller's until returned.
int acquire_stream(yart_scene* s, hipStream_t* out);
void release_stream(yart_scene* s, hipStream_t st);
// Covered pixels (main.rs:636-647 crop grid) of the blocks a shard owns.
uint64_t shard_pixels(uint32_t w, uint32_t h, uint32_t shard_index, uint32_t shard_count);
// Wait for `done` on the calling thread, reporting progress from the given words (one per device).
int wait_with_progress(const std::vector<hipEvent_t>& done, const std::vector<int>& devices,
                       const std::vector<Progress*>& prog, uint64_t total_pixels, yart_progress_fn fn, void* user);
int alloc_progress(Progress& p);
void free_progress(Progress& p);

}  // namespace yart_impl
