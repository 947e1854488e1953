// multi.cpp — the multi-GPU half of the C ABI (include/yart.h): RCCL communicators, the frame
// gather, and yart_render_multi (one process driving N devices).
//
// Reference: the frame is 64 tile jobs fanned out over a thread pool and stitched back into one
// image from an mpsc channel (main.rs:633-660, 747-760). Here pixels are independent as there, so
// the devices share nothing while they render: 8x8 block b belongs to device b % N, each device
// renders its blocks straight into a packed buffer (its pixels and nothing else), and ONE gather
// over RCCL (point-to-point over xGMI: one hop per device, 1/N of the frame each) lands every
// packet on the root, where one kernel scatters them into the frame.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <system_error>
#include <thread>
#include <string>
#include <vector>

#include "../../include/yart.h"
#include "kernels.h"
#include "scene_impl.h"

using namespace yart_dev;
using namespace yart_impl;

struct yart_comm {
  ncclComm_t comm = nullptr;
  int device = 0, rank = 0, n_ranks = 1;
  // root-side receive buffer (n_ranks packets) and send staging, grown on demand
  double* recv = nullptr;
  size_t recv_bytes = 0;
  ~yart_comm() {
    if (recv) { (void)hipSetDevice(device); (void)hipFree(recv); }
    if (comm) (void)ncclCommDestroy(comm);
  }
};

namespace {

int nccl_fail(ncclResult_t r, const char* what) {
  return fail(YART_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}
#define NCCL_TRY(expr, what)                         \
  do {                                               \
    ncclResult_t r_ = (expr);                        \
    if (r_ != ncclSuccess) return nccl_fail(r_, what); \
  } while (0)

uint64_t packet_len(uint32_t w, uint32_t h, uint32_t n) {  // doubles per rank: the largest shard (shard 0)
  return yart_shard_packed_len(w, h, 0, n);
}

int ensure_recv(yart_comm* c, size_t bytes) {
  if (c->recv_bytes >= bytes) return YART_OK;
  if (c->recv) HIP_TRY(hipFree(c->recv), "hipFree");
  c->recv = nullptr; c->recv_bytes = 0;
  HIP_TRY(hipMalloc(&c->recv, bytes), "hipMalloc gather buffer");
  c->recv_bytes = bytes;
  return YART_OK;
}

// The gather of one rank (inside a group for single-process communicators). Packets are equal
// sized (ncclGather's contract): a shard with fewer blocks sends the tail of its buffer too, which
// the unpack never reads. The send buffer must therefore hold packet_len doubles.
int enqueue_gather(yart_comm* c, const double* d_packed, uint32_t w, uint32_t h, int root, hipStream_t st) {
  const uint64_t n = packet_len(w, h, (uint32_t)c->n_ranks);
  if (c->rank == root)
    if (int rc = ensure_recv(c, sizeof(double) * n * (size_t)c->n_ranks)) return rc;
  NCCL_TRY(ncclGather(d_packed, c->rank == root ? c->recv : nullptr, n, ncclFloat64, root, c->comm, st), "ncclGather");
  return YART_OK;
}

}  // namespace

extern "C" {

int yart_comm_unique_id(uint8_t id_out[YART_COMM_ID_BYTES]) {
  if (!id_out) return fail(YART_ERR_INVALID, "null argument");
  static_assert(sizeof(ncclUniqueId) == YART_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::memcpy(id_out, &id, sizeof id);
  return ok();
}

int yart_comm_init_rank(const uint8_t id[YART_COMM_ID_BYTES], int n_ranks, int rank, int device, yart_comm** out) {
  if (!id || !out || n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(YART_ERR_INVALID, "bad argument");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
  if (device < 0 || device >= ndev) return fail(YART_ERR_INVALID, "device index out of range");
  DeviceGuard g(device);
  auto c = std::make_unique<yart_comm>();
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof uid);
  NCCL_TRY(ncclCommInitRank(&c->comm, n_ranks, uid, rank), "ncclCommInitRank");
  c->device = device; c->rank = rank; c->n_ranks = n_ranks;
  *out = c.release();
  return ok();
}

int yart_comm_init_all(int n, const int* devices, yart_comm** comms_out) {
  if (n < 1 || !devices || !comms_out) return fail(YART_ERR_INVALID, "bad argument");
  std::vector<ncclComm_t> comms((size_t)n, nullptr);
  NCCL_TRY(ncclCommInitAll(comms.data(), n, devices), "ncclCommInitAll");
  for (int d = 0; d < n; ++d) {
    comms_out[d] = new yart_comm();
    comms_out[d]->comm = comms[(size_t)d];
    comms_out[d]->device = devices[d]; comms_out[d]->rank = d; comms_out[d]->n_ranks = n;
  }
  return ok();
}

void yart_comm_destroy(yart_comm* c) { delete c; }

int yart_gather_frame_async(yart_comm* c, const double* d_packed, uint32_t w, uint32_t h, int root, double* d_frame,
                            void* stream) {
  if (!c || !d_packed || w == 0 || h == 0 || root < 0 || root >= c->n_ranks) return fail(YART_ERR_INVALID, "bad argument");
  if (c->rank == root && !d_frame) return fail(YART_ERR_INVALID, "null frame on the root");
  DeviceGuard g(c->device);
  hipStream_t st = (hipStream_t)stream;
  if (int rc = enqueue_gather(c, d_packed, w, h, root, st)) return rc;
  if (c->rank == root)
    HIP_TRY(launch_unpack_shards(c->recv, (uint32_t)c->n_ranks, packet_len(w, h, (uint32_t)c->n_ranks), w, h, d_frame, st),
            "launch k_unpack_shards");
  return ok();
}

}  // extern "C"


// ------------------------------------------------------------ one process, N devices
// A slot is what the frames submitted on one caller stream use: a stream, a packed shard and a
// gather event per device, and the root's receive buffer. Frames on different caller streams
// overlap (the next frame's renders take the SIMD slots the previous frame's drain leaves idle);
// the gathers still run in submission order on every device (each waits for the previous
// submission's gather on its device), which is the order RCCL needs on a communicator.
struct MultiSlot {
  std::vector<hipStream_t> streams;   // per device, library-owned, non-blocking
  std::vector<double*> packed;        // per device, packet_len doubles
  std::vector<size_t> packed_bytes;
  std::vector<hipEvent_t> gathered;   // per device: its ncclGather of the latest frame
  std::vector<hipEvent_t> rendered;   // per device: its render of the latest frame (yart_multi_query)
  hipEvent_t start = nullptr;         // devices[0]: the caller stream's work before the frame
  hipEvent_t done = nullptr;          // devices[0]: the frame unpacked
  double* recv = nullptr;             // devices[0]: every shard's packet
  size_t recv_bytes = 0;
  // devices[0]: the root's gather + unpack interval of each frame not yet read (timing)
  std::vector<std::pair<hipEvent_t, hipEvent_t>> gather_events;
  // per device: its ncclGather's interval (from its launch, after its render and the previous
  // submission's gather, to its end) for each frame not yet read — the per-device balance of the
  // first N-GPU runs (which device waited in the gather for which)
  std::vector<std::vector<std::pair<hipEvent_t, hipEvent_t>>> dev_gather_events;
  uint64_t last_use = 0;              // submission number of its latest frame (eviction order)
};

struct yart_multi {
  int n = 0;
  std::vector<int> devices;
  std::vector<yart_scene*> scenes;
  std::vector<yart_comm*> comms;
  std::mutex mu;                                   // submissions are enqueued one at a time
  std::map<hipStream_t, std::unique_ptr<MultiSlot>> slots;  // by caller stream (devices[0]), at most kMaxSlots
  uint64_t submissions = 0;
  MultiSlot* latest = nullptr;  // the slot of the latest submission (yart_multi_query)
  std::vector<hipEvent_t> last_gather;             // per device: the latest submission's gather
  hipStream_t host_stream = nullptr;               // devices[0]: yart_render_multi's caller stream
  double* frame = nullptr;                         // devices[0]: yart_render_multi's frame
  size_t frame_bytes = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> gather_pool;  // devices[0]: recycled timing pairs
  std::vector<std::vector<std::pair<hipEvent_t, hipEvent_t>>> dev_pool;  // per device: recycled timing pairs
  double render_ms = 0.0, gather_ms = 0.0;  // yart_render_multi's last frame
  // per device, summed over the frames of the latest timing read (yart_multi_frame_timing or
  // yart_render_multi): render-kernel time and its own gather time (yart_multi_device_timing)
  std::vector<double> dev_render_ms, dev_gather_ms;
  uint32_t dev_frames = 0;
  // Drains a slot's streams and frees what it holds (the destructor; eviction of the least recently
  // used slot when a new caller stream would exceed kMaxSlots, so a caller that makes a stream per
  // frame does not grow device memory without bound — ADVICE r03).
  void release_slot(MultiSlot& s) {
    for (int d = 0; d < n && d < (int)devices.size(); ++d) {
      (void)hipSetDevice(devices[(size_t)d]);
      if ((size_t)d < s.streams.size() && s.streams[(size_t)d]) (void)hipStreamSynchronize(s.streams[(size_t)d]);
    }
    for (int d = 0; d < n && d < (int)devices.size(); ++d) {
      (void)hipSetDevice(devices[(size_t)d]);
      // the scene's unread frame-timing events of this stream: read and recycled now, or a later
      // stream that happens to get the same handle would report these frames as its own
      if ((size_t)d < s.streams.size() && s.streams[(size_t)d] && (size_t)d < scenes.size()) {
        double r = 0.0, a = 0.0;
        uint32_t f = 0;
        (void)yart_frame_timing(scenes[(size_t)d], s.streams[(size_t)d], &r, &a, &f);
      }
      if ((size_t)d < s.packed.size() && s.packed[(size_t)d]) (void)hipFree(s.packed[(size_t)d]);
      if ((size_t)d < s.gathered.size() && s.gathered[(size_t)d]) (void)hipEventDestroy(s.gathered[(size_t)d]);
      if ((size_t)d < s.rendered.size() && s.rendered[(size_t)d]) (void)hipEventDestroy(s.rendered[(size_t)d]);
      if ((size_t)d < s.streams.size() && s.streams[(size_t)d]) (void)hipStreamDestroy(s.streams[(size_t)d]);
      if ((size_t)d < s.dev_gather_events.size() && (size_t)d < dev_pool.size())
        for (auto& e : s.dev_gather_events[(size_t)d]) dev_pool[(size_t)d].push_back(e);  // unread: dropped
      if (d == 0) {
        for (auto& e : s.gather_events) gather_pool.push_back(e);  // unread timings are dropped
        s.gather_events.clear();
        if (s.recv) (void)hipFree(s.recv);
        if (s.start) (void)hipEventDestroy(s.start);
        if (s.done) (void)hipEventDestroy(s.done);
      }
    }
    s = MultiSlot{};
  }
  ~yart_multi() {
    for (auto& kv : slots) release_slot(*kv.second);
    for (int d = 0; d < n && d < (int)devices.size(); ++d) {
      (void)hipSetDevice(devices[(size_t)d]);
      if ((size_t)d < dev_pool.size())
        for (auto& e : dev_pool[(size_t)d]) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
      if (d == 0) {
        for (auto& e : gather_pool) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
        if (frame) (void)hipFree(frame);
        if (host_stream) { (void)hipStreamSynchronize(host_stream); (void)hipStreamDestroy(host_stream); }
      }
    }
    for (yart_comm* c : comms) delete c;
    for (yart_scene* s : scenes) yart_scene_destroy(s);
  }
};

namespace {

struct RestoreDevice {
  int d = 0;
  RestoreDevice() { (void)hipGetDevice(&d); }
  ~RestoreDevice() { (void)hipSetDevice(d); }
};

// The slot of a caller stream, created on first use (streams and events made once, reused). At
// most kMaxSlots live at once: a new caller stream beyond that takes the place of the least
// recently used slot, after that slot's frames have finished (its streams are drained).
constexpr size_t kMaxSlots = 8;
int multi_slot(yart_multi* m, hipStream_t caller, MultiSlot** out) {
  if (!m->slots.count(caller) && m->slots.size() >= kMaxSlots) {
    auto lru = m->slots.begin();
    for (auto it = m->slots.begin(); it != m->slots.end(); ++it)
      if (it->second->last_use < lru->second->last_use) lru = it;
    if (m->latest == lru->second.get()) m->latest = nullptr;
    m->release_slot(*lru->second);
    m->slots.erase(lru);
  }
  auto& e = m->slots[caller];
  if (!e) {
    auto s = std::make_unique<MultiSlot>();
    s->streams.assign((size_t)m->n, nullptr);
    s->packed.assign((size_t)m->n, nullptr);
    s->packed_bytes.assign((size_t)m->n, 0);
    s->gathered.assign((size_t)m->n, nullptr);
    s->rendered.assign((size_t)m->n, nullptr);
    s->dev_gather_events.assign((size_t)m->n, {});
    for (int d = 0; d < m->n; ++d) {
      HIP_TRY(hipSetDevice(m->devices[(size_t)d]), "hipSetDevice");
      HIP_TRY(hipStreamCreateWithFlags(&s->streams[(size_t)d], hipStreamNonBlocking), "hipStreamCreate");
      HIP_TRY(hipEventCreateWithFlags(&s->gathered[(size_t)d], hipEventDisableTiming), "hipEventCreate");
      HIP_TRY(hipEventCreateWithFlags(&s->rendered[(size_t)d], hipEventDisableTiming), "hipEventCreate");
      if (d == 0) {
        HIP_TRY(hipEventCreateWithFlags(&s->start, hipEventDisableTiming), "hipEventCreate");
        HIP_TRY(hipEventCreateWithFlags(&s->done, hipEventDisableTiming), "hipEventCreate");
      }
    }
    e = std::move(s);
  }
  e->last_use = ++m->submissions;
  *out = e.get();
  return YART_OK;
}

// A pair of timing events from `pool` (recycled) or new ones, on the current device.
int event_pair(std::vector<std::pair<hipEvent_t, hipEvent_t>>& pool, std::pair<hipEvent_t, hipEvent_t>& out) {
  if (!pool.empty()) {
    out = pool.back();
    pool.pop_back();
    return YART_OK;
  }
  HIP_TRY(hipEventCreate(&out.first), "hipEventCreate");
  if (hipError_t e = hipEventCreate(&out.second)) { (void)hipEventDestroy(out.first); return hip_fail(e, "hipEventCreate"); }
  return YART_OK;
}

// Enqueue one frame: every device renders its shard into its packed buffer on the slot's stream,
// the grouped ncclGather follows each render in stream order, and devices[0] unpacks into
// d_frame after the caller stream's earlier work; the caller stream then waits for the frame.
// No host wait. prog: one progress word per device, or null.
int multi_submit(yart_multi* m, const yart_camera* cam, const yart_render_params* p, double* d_frame, hipStream_t caller,
                 std::vector<Progress>* prog) {
  if (!cam || !p || !d_frame) return fail(YART_ERR_INVALID, "null argument");
  if (p->width == 0 || p->height == 0) return fail(YART_ERR_INVALID, "width and height must be > 0");
  const int n = m->n;
  const uint32_t W = p->width, H = p->height;
  const uint64_t stride = packet_len(W, H, (uint32_t)n);
  const size_t pk_bytes = sizeof(double) * stride;
  RestoreDevice restore;
  MultiSlot* S = nullptr;
  if (int rc = multi_slot(m, caller, &S)) return rc;
  // the latest submission from here on, even one that fails partway (yart_multi_query then
  // describes it, not an older frame whose slot events this one is about to re-record)
  m->latest = S;
  // 1. renders, one per device, each straight into its packed shard. A wavefront (mesh) frame keeps
  // the host in its launch loop until the frame's last iterations are queued, so those devices are
  // driven from a host thread each, all at once.
  auto render_one = [&](int d) -> int {
    const size_t di = (size_t)d;
    HIP_TRY(hipSetDevice(m->devices[di]), "hipSetDevice");
    hipStream_t st = S->streams[di];
    if (S->packed_bytes[di] < pk_bytes) {
      if (S->packed[di]) {
        HIP_TRY(hipStreamSynchronize(st), "drain");
        HIP_TRY(hipFree(S->packed[di]), "hipFree");
      }
      S->packed[di] = nullptr; S->packed_bytes[di] = 0;
      HIP_TRY(hipMalloc(&S->packed[di], pk_bytes), "hipMalloc packed shard");
      // a smaller shard sends its tail too (equal-sized packets); zeroed once, never read
      HIP_TRY(hipMemsetAsync(S->packed[di], 0, pk_bytes, st), "hipMemset");
      S->packed_bytes[di] = pk_bytes;
    }
    RenderArgs a;
    yart_render_params q = *p;
    q.shard_index = (uint32_t)d;
    q.shard_count = (uint32_t)n;
    if (int rc = make_args(m->scenes[di], cam, &q, S->packed[di], a)) return rc;
    a.packed = 1;
    Progress* pr = prog ? &(*prog)[di] : nullptr;
    if (int rc = launch_frame(m->scenes[di], a, p->samples_per_unit, false, st, pr)) return rc;
    HIP_TRY(hipEventRecord(S->rendered[di], st), "hipEventRecord");
    return YART_OK;
  };
  if (n > 1 && m->scenes[0]->wavefront) {
    std::vector<int> rcs((size_t)n, YART_OK);
    std::vector<std::string> errs((size_t)n);
    std::vector<std::thread> th;
    std::vector<int> here;
    for (int d = 1; d < n; ++d) {
      try {
        th.emplace_back([&, d] { rcs[(size_t)d] = render_one(d); errs[(size_t)d] = yart_last_error(); });
      } catch (const std::system_error&) {
        here.push_back(d);
      }
    }
    rcs[0] = render_one(0);
    errs[0] = yart_last_error();
    for (int d : here) { rcs[(size_t)d] = render_one(d); errs[(size_t)d] = yart_last_error(); }
    for (auto& t : th) t.join();
    for (int d = 0; d < n; ++d)
      if (rcs[(size_t)d] != YART_OK) return fail(rcs[(size_t)d], errs[(size_t)d]);  // the message was thread-local
  } else {
    for (int d = 0; d < n; ++d)
      if (int rc = render_one(d)) return rc;
  }
  // 2. the root's receive buffer (per slot: a later slot's gather may land while this one unpacks)
  HIP_TRY(hipSetDevice(m->devices[0]), "hipSetDevice");
  if (S->recv_bytes < pk_bytes * (size_t)n) {
    if (S->recv) {
      HIP_TRY(hipStreamSynchronize(S->streams[0]), "drain");
      HIP_TRY(hipFree(S->recv), "hipFree");
    }
    S->recv = nullptr; S->recv_bytes = 0;
    HIP_TRY(hipMalloc(&S->recv, pk_bytes * (size_t)n), "hipMalloc gather buffer");
    S->recv_bytes = pk_bytes * (size_t)n;
  }
  // The frame's timing pairs join the slot's lists only once both ends are recorded (below): a
  // submission that fails half way returns them to their pools instead of leaving a pair that
  // multi_timing cannot read.
  std::pair<hipEvent_t, hipEvent_t> gev;
  if (int rc = event_pair(m->gather_pool, gev)) return rc;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> dev_ev;
  dev_ev.reserve((size_t)n);
  struct Pending {
    yart_multi* m;
    std::pair<hipEvent_t, hipEvent_t>& gev;
    std::vector<std::pair<hipEvent_t, hipEvent_t>>& dev_ev;
    bool handed_over = false;
    ~Pending() {
      if (handed_over) return;
      m->gather_pool.push_back(gev);
      for (size_t d = 0; d < dev_ev.size(); ++d) m->dev_pool[d].push_back(dev_ev[d]);
    }
  } pending{m, gev, dev_ev};
  // 3. ONE gather to devices[0], each device's part right behind its render; in submission order
  for (int d = 0; d < n; ++d) {
    const size_t di = (size_t)d;
    HIP_TRY(hipSetDevice(m->devices[di]), "hipSetDevice");
    if (m->last_gather[di] && m->last_gather[di] != S->gathered[di])
      HIP_TRY(hipStreamWaitEvent(S->streams[di], m->last_gather[di], 0), "hipStreamWaitEvent");
    if (d == 0) HIP_TRY(hipEventRecord(gev.first, S->streams[0]), "hipEventRecord");
    std::pair<hipEvent_t, hipEvent_t> pr;
    if (int rc = event_pair(m->dev_pool[di], pr)) return rc;
    dev_ev.push_back(pr);
    HIP_TRY(hipEventRecord(pr.first, S->streams[di]), "hipEventRecord");
  }
  NCCL_TRY(ncclGroupStart(), "ncclGroupStart");
  for (int d = 0; d < n; ++d) {
    const size_t di = (size_t)d;
    (void)hipSetDevice(m->devices[di]);
    ncclResult_t r = ncclGather(S->packed[di], d == 0 ? S->recv : nullptr, stride, ncclFloat64, 0, m->comms[di]->comm,
                                S->streams[di]);
    if (r != ncclSuccess) { (void)ncclGroupEnd(); return nccl_fail(r, "ncclGather"); }
  }
  NCCL_TRY(ncclGroupEnd(), "ncclGroupEnd");
  for (int d = 0; d < n; ++d) {
    const size_t di = (size_t)d;
    HIP_TRY(hipSetDevice(m->devices[di]), "hipSetDevice");
    HIP_TRY(hipEventRecord(dev_ev[di].second, S->streams[di]), "hipEventRecord");
    HIP_TRY(hipEventRecord(S->gathered[di], S->streams[di]), "hipEventRecord");
    m->last_gather[di] = S->gathered[di];
  }
  // 4. unpack on the root, after whatever the caller stream had queued (it may still read d_frame)
  HIP_TRY(hipSetDevice(m->devices[0]), "hipSetDevice");
  HIP_TRY(hipEventRecord(S->start, caller), "hipEventRecord");
  HIP_TRY(hipStreamWaitEvent(S->streams[0], S->start, 0), "hipStreamWaitEvent");
  HIP_TRY(launch_unpack_shards(S->recv, (uint32_t)n, stride, W, H, d_frame, S->streams[0]), "launch k_unpack_shards");
  HIP_TRY(hipEventRecord(gev.second, S->streams[0]), "hipEventRecord");
  S->gather_events.push_back(gev);
  for (int d = 0; d < n; ++d) S->dev_gather_events[(size_t)d].push_back(dev_ev[(size_t)d]);
  pending.handed_over = true;
  HIP_TRY(hipEventRecord(S->done, S->streams[0]), "hipEventRecord");
  HIP_TRY(hipStreamWaitEvent(caller, S->done, 0), "hipStreamWaitEvent");
  return YART_OK;
}

// Summed kernel times of the frames submitted since the last read, over every slot or one
// (their streams idle by then): render = the slowest device's summed k_render time,
// gather = the root's gather + unpack intervals, which include the root's wait for the slowest
// device's render to finish. Per device (m->dev_*): its summed render time and the summed
// intervals of its own ncclGather.
int multi_timing(yart_multi* m, MultiSlot* only, double* render_ms, double* gather_ms, uint32_t* frames) {
  RestoreDevice restore;
  double worst = 0.0;
  uint32_t nf = 0;
  m->dev_render_ms.assign((size_t)m->n, 0.0);
  m->dev_gather_ms.assign((size_t)m->n, 0.0);
  for (int d = 0; d < m->n; ++d) {
    double r = 0.0, dg = 0.0;
    for (auto& kv : m->slots) {
      if (only && kv.second.get() != only) continue;
      double rr = 0.0, acc = 0.0;
      uint32_t f = 0;
      if (int rc = yart_frame_timing(m->scenes[(size_t)d], kv.second->streams[(size_t)d], &rr, &acc, &f)) return rc;
      r += rr;
      if (d == 0) nf += f;
      HIP_TRY(hipSetDevice(m->devices[(size_t)d]), "hipSetDevice");
      // taken out of the slot first and recycled whatever happens: a failed read does not leave
      // pairs behind for every later call to trip over
      std::vector<std::pair<hipEvent_t, hipEvent_t>> evs;
      evs.swap(kv.second->dev_gather_events[(size_t)d]);
      hipError_t bad = hipSuccess;
      for (auto& e : evs) {
        float ms = 0.0f;
        if (bad == hipSuccess) bad = hipEventElapsedTime(&ms, e.first, e.second);
        if (bad == hipSuccess) dg += ms;
        m->dev_pool[(size_t)d].push_back(e);
      }
      if (bad != hipSuccess) return hip_fail(bad, "hipEventElapsedTime");
    }
    m->dev_render_ms[(size_t)d] = r;
    m->dev_gather_ms[(size_t)d] = dg;
    if (r > worst) worst = r;
  }
  m->dev_frames = nf;
  HIP_TRY(hipSetDevice(m->devices[0]), "hipSetDevice");
  double g = 0.0;
  for (auto& kv : m->slots) {
    if (only && kv.second.get() != only) continue;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> evs;
    evs.swap(kv.second->gather_events);
    hipError_t bad = hipSuccess;
    for (auto& e : evs) {
      float ms = 0.0f;
      if (bad == hipSuccess) bad = hipEventElapsedTime(&ms, e.first, e.second);
      if (bad == hipSuccess) g += ms;
      m->gather_pool.push_back(e);
    }
    if (bad != hipSuccess) return hip_fail(bad, "hipEventElapsedTime");
  }
  *render_ms = worst;
  *gather_ms = g;
  *frames = nf;
  return YART_OK;
}

}  // namespace

extern "C" {

int yart_multi_create(int n, const int* devices, const yart_scene_desc* desc, yart_multi** out) {
  if (n < 1 || !devices || !desc || !out) return fail(YART_ERR_INVALID, "bad argument");
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
  for (int d = 0; d < n; ++d) {
    if (devices[d] < 0 || devices[d] >= ndev) return fail(YART_ERR_INVALID, "device index out of range");
    for (int e = 0; e < d; ++e)
      if (devices[e] == devices[d]) return fail(YART_ERR_INVALID, "a device listed twice");
  }
  auto m = std::make_unique<yart_multi>();
  m->n = n;
  m->devices.assign(devices, devices + n);
  m->last_gather.assign((size_t)n, nullptr);
  m->dev_pool.assign((size_t)n, {});
  RestoreDevice restore;
  for (int d = 0; d < n; ++d) {  // the scene is uploaded once per device, here
    yart_scene* s = nullptr;
    if (int rc = yart_scene_create(devices[d], desc, &s)) return rc;
    m->scenes.push_back(s);
  }
  HIP_TRY(hipSetDevice(devices[0]), "hipSetDevice");
  HIP_TRY(hipStreamCreateWithFlags(&m->host_stream, hipStreamNonBlocking), "hipStreamCreate");
  m->comms.assign((size_t)n, nullptr);
  if (int rc = yart_comm_init_all(n, devices, m->comms.data())) return rc;
  *out = m.release();
  return ok();
}

int yart_render_multi_async(yart_multi* m, const yart_camera* cam, const yart_render_params* p, double* d_frame,
                            void* stream) {
  if (!m) return fail(YART_ERR_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(m->mu);
  if (int rc = multi_submit(m, cam, p, d_frame, (hipStream_t)stream, nullptr)) return rc;
  return ok();
}

int yart_multi_frame_timing(yart_multi* m, double* render_ms, double* gather_ms, uint32_t* frames) {
  if (!m || !render_ms || !gather_ms || !frames) return fail(YART_ERR_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(m->mu);
  if (int rc = multi_timing(m, nullptr, render_ms, gather_ms, frames)) return rc;
  return ok();
}

int yart_render_multi(yart_multi* m, const yart_camera* cam, const yart_render_params* p, double* xyz_sum_out,
                      yart_progress_fn progress, void* user) {
  if (!m || !cam || !p || !xyz_sum_out) return fail(YART_ERR_INVALID, "null argument");
  if (p->width == 0 || p->height == 0) return fail(YART_ERR_INVALID, "width and height must be > 0");
  std::lock_guard<std::mutex> lk(m->mu);
  const int n = m->n;
  const size_t frame_bytes = sizeof(double) * 3 * (size_t)p->width * p->height;
  RestoreDevice restore;
  HIP_TRY(hipSetDevice(m->devices[0]), "hipSetDevice");
  hipStream_t hs = m->host_stream;
  if (m->frame_bytes < frame_bytes) {
    if (m->frame) {
      HIP_TRY(hipStreamSynchronize(hs), "drain");
      HIP_TRY(hipFree(m->frame), "hipFree");
    }
    m->frame = nullptr; m->frame_bytes = 0;
    HIP_TRY(hipMalloc(&m->frame, frame_bytes), "hipMalloc frame");
    m->frame_bytes = frame_bytes;
  }
  std::vector<Progress> pr((size_t)(progress ? n : 0));
  struct FreeAll { std::vector<Progress>& v; ~FreeAll() { for (auto& x : v) free_progress(x); } } free_all{pr};
  uint64_t total_px = 0;
  std::vector<Progress*> pp;
  for (int d = 0; d < (int)pr.size(); ++d) {
    HIP_TRY(hipSetDevice(m->devices[(size_t)d]), "hipSetDevice");
    if (int rc = alloc_progress(pr[(size_t)d])) return rc;
    pr[(size_t)d].pixels = shard_pixels(p->width, p->height, (uint32_t)d, (uint32_t)n);
    total_px += pr[(size_t)d].pixels;
    pp.push_back(&pr[(size_t)d]);
  }
  // everything (renders, gather, unpack) is enqueued before the host waits
  if (int rc = multi_submit(m, cam, p, m->frame, hs, progress ? &pr : nullptr)) return rc;
  HIP_TRY(hipSetDevice(m->devices[0]), "hipSetDevice");
  hipEvent_t done;
  HIP_TRY(hipEventCreateWithFlags(&done, hipEventDisableTiming), "hipEventCreate");
  std::unique_ptr<std::remove_pointer<hipEvent_t>::type, decltype(&hipEventDestroy)> hold(done, &hipEventDestroy);
  HIP_TRY(hipEventRecord(done, hs), "hipEventRecord");
  if (int rc = wait_with_progress({done}, {m->devices[0]}, pp, total_px, progress, user)) return rc;
  HIP_TRY(hipSetDevice(m->devices[0]), "hipSetDevice");
  HIP_TRY(hipMemcpyAsync(xyz_sum_out, m->frame, frame_bytes, hipMemcpyDeviceToHost, hs), "copy frame");
  HIP_TRY(hipStreamSynchronize(hs), "copy frame");
  uint32_t frames = 0;
  // the host stream's slot is idle now: the timing of its frame
  double r = 0.0, g = 0.0;
  if (int rc = multi_timing(m, m->slots[hs].get(), &r, &g, &frames)) return rc;
  m->render_ms = frames ? r / frames : 0.0;
  m->gather_ms = frames ? g / frames : 0.0;
  return ok();
}

int yart_multi_last_timing(const yart_multi* m, double* render_ms, double* gather_ms) {
  if (!m || !render_ms || !gather_ms) return fail(YART_ERR_INVALID, "null argument");
  *render_ms = m->render_ms;
  *gather_ms = m->gather_ms;
  return ok();
}

int yart_multi_device_timing(yart_multi* m, int n, double* render_ms, double* gather_ms, uint32_t* frames) {
  if (!m || !render_ms || !gather_ms || !frames) return fail(YART_ERR_INVALID, "null argument");
  if (n != m->n) return fail(YART_ERR_INVALID, "n must be the multi's device count");
  std::lock_guard<std::mutex> lk(m->mu);
  for (int d = 0; d < n; ++d) {
    render_ms[d] = (size_t)d < m->dev_render_ms.size() ? m->dev_render_ms[(size_t)d] : 0.0;
    gather_ms[d] = (size_t)d < m->dev_gather_ms.size() ? m->dev_gather_ms[(size_t)d] : 0.0;
  }
  *frames = m->dev_frames;
  return ok();
}

int yart_multi_query(yart_multi* m, int32_t* state, int32_t* unpacked) {
  if (!m || !state || !unpacked) return fail(YART_ERR_INVALID, "null argument");
  // never waits: a submission in progress (its thread may be blocked in the gather's setup) holds the
  // lock, and then every device reads -1
  std::unique_lock<std::mutex> lk(m->mu, std::try_to_lock);
  *unpacked = -1;
  for (int d = 0; d < m->n; ++d) state[d] = -1;
  if (!lk.owns_lock() || !m->latest) return ok();
  RestoreDevice restore;
  MultiSlot& S = *m->latest;
  auto done = [](hipEvent_t e) { return e && hipEventQuery(e) == hipSuccess; };
  for (int d = 0; d < m->n; ++d) {
    (void)hipSetDevice(m->devices[(size_t)d]);
    state[d] = done(S.gathered[(size_t)d]) ? 2 : done(S.rendered[(size_t)d]) ? 1 : 0;
  }
  (void)hipSetDevice(m->devices[0]);
  *unpacked = done(S.done) ? 1 : 0;
  return ok();
}

void yart_multi_destroy(yart_multi* m) { delete m; }

int yart_unpack_shards_async(int device, const double* d_recv, uint32_t shards, uint64_t stride, uint32_t width,
                             uint32_t height, double* d_frame, void* stream) {
  if (!d_recv || !d_frame || shards == 0 || width == 0 || height == 0) return fail(YART_ERR_INVALID, "bad argument");
  if (stride < packet_len(width, height, shards)) return fail(YART_ERR_INVALID, "stride below the largest shard's packet");
  DeviceGuard g(device);
  HIP_TRY(launch_unpack_shards(d_recv, shards, stride, width, height, d_frame, (hipStream_t)stream), "launch k_unpack_shards");
  return ok();
}

}  // extern "C"
