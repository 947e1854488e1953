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
#include <memory>
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

struct yart_multi {
  int n = 0;
  std::vector<int> devices;
  std::vector<yart_scene*> scenes;
  std::vector<yart_comm*> comms;
  std::vector<hipStream_t> streams;
  std::vector<double*> packed;  // per device, packet_len doubles (grown on demand)
  std::vector<size_t> packed_bytes;
  double* frame = nullptr;      // on devices[0]
  size_t frame_bytes = 0;
  double render_ms = 0.0, gather_ms = 0.0;
  ~yart_multi() {
    for (int d = 0; d < n; ++d) {
      (void)hipSetDevice(devices[(size_t)d]);
      if ((size_t)d < streams.size() && streams[(size_t)d]) (void)hipStreamSynchronize(streams[(size_t)d]);
      if ((size_t)d < packed.size() && packed[(size_t)d]) (void)hipFree(packed[(size_t)d]);
      if (d == 0 && frame) (void)hipFree(frame);
      if ((size_t)d < streams.size() && streams[(size_t)d]) (void)hipStreamDestroy(streams[(size_t)d]);
    }
    for (yart_comm* c : comms) delete c;
    for (yart_scene* s : scenes) yart_scene_destroy(s);
  }
};

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
  int old = 0;
  (void)hipGetDevice(&old);
  for (int d = 0; d < n; ++d) {  // the scene is uploaded once per device, here
    yart_scene* s = nullptr;
    if (int rc = yart_scene_create(devices[d], desc, &s)) return rc;
    m->scenes.push_back(s);
    hipStream_t st;
    (void)hipSetDevice(devices[d]);
    hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    (void)hipSetDevice(old);
    if (e != hipSuccess) return hip_fail(e, "hipStreamCreate");
    m->streams.push_back(st);
  }
  m->comms.assign((size_t)n, nullptr);
  if (int rc = yart_comm_init_all(n, devices, m->comms.data())) return rc;
  m->packed.assign((size_t)n, nullptr);
  m->packed_bytes.assign((size_t)n, 0);
  *out = m.release();
  return ok();
}

int yart_render_multi(yart_multi* m, const yart_camera* cam, const yart_render_params* p, double* xyz_sum_out,
                      yart_progress_fn progress, void* user) {
  if (!m || !cam || !p || !xyz_sum_out) return fail(YART_ERR_INVALID, "null argument");
  if (p->width == 0 || p->height == 0) return fail(YART_ERR_INVALID, "width and height must be > 0");
  const int n = m->n;
  const uint32_t W = p->width, H = p->height;
  const size_t pk_bytes = sizeof(double) * packet_len(W, H, (uint32_t)n);
  const size_t frame_bytes = sizeof(double) * 3 * (size_t)W * H;
  int old = 0;
  (void)hipGetDevice(&old);
  struct Restore { int d; ~Restore() { (void)hipSetDevice(d); } } restore{old};

  std::vector<Progress> pr((size_t)n);
  struct FreeAll { std::vector<Progress>& v; ~FreeAll() { for (auto& p : v) free_progress(p); } } free_all{pr};
  std::vector<hipEvent_t> t0((size_t)n), t1((size_t)n), done((size_t)n);
  struct Events {
    std::vector<hipEvent_t>* v[3];
    ~Events() { for (auto* x : v) for (hipEvent_t e : *x) if (e) (void)hipEventDestroy(e); }
  } events{{&t0, &t1, &done}};
  hipEvent_t g1 = nullptr;

  // 1. every device renders its shard, packed, on its own stream
  for (int d = 0; d < n; ++d) {
    HIP_TRY(hipSetDevice(m->devices[(size_t)d]), "hipSetDevice");
    hipStream_t st = m->streams[(size_t)d];
    if (m->packed_bytes[(size_t)d] < pk_bytes) {
      if (m->packed[(size_t)d]) {
        HIP_TRY(hipStreamSynchronize(st), "drain");
        HIP_TRY(hipFree(m->packed[(size_t)d]), "hipFree");
      }
      m->packed[(size_t)d] = nullptr; m->packed_bytes[(size_t)d] = 0;
      HIP_TRY(hipMalloc(&m->packed[(size_t)d], pk_bytes), "hipMalloc packed shard");
      HIP_TRY(hipMemsetAsync(m->packed[(size_t)d], 0, pk_bytes, st), "hipMemset");
      m->packed_bytes[(size_t)d] = pk_bytes;
    }
    if (d == 0 && m->frame_bytes < frame_bytes) {
      if (m->frame) {
        HIP_TRY(hipStreamSynchronize(st), "drain");
        HIP_TRY(hipFree(m->frame), "hipFree");
      }
      m->frame = nullptr; m->frame_bytes = 0;
      HIP_TRY(hipMalloc(&m->frame, frame_bytes), "hipMalloc frame");
      m->frame_bytes = frame_bytes;
    }
    HIP_TRY(hipEventCreate(&t0[(size_t)d]), "hipEventCreate");
    HIP_TRY(hipEventCreate(&t1[(size_t)d]), "hipEventCreate");
    HIP_TRY(hipEventCreateWithFlags(&done[(size_t)d], hipEventDisableTiming), "hipEventCreate");
    RenderArgs a;
    yart_render_params q = *p;
    q.shard_index = (uint32_t)d;
    q.shard_count = (uint32_t)n;
    if (int rc = make_args(m->scenes[(size_t)d], cam, &q, m->packed[(size_t)d], a)) return rc;
    a.packed = 1;
    if (progress) {
      if (int rc = alloc_progress(pr[(size_t)d])) return rc;
      pr[(size_t)d].pixels = shard_pixels(W, H, (uint32_t)d, (uint32_t)n);
    }
    HIP_TRY(hipEventRecord(t0[(size_t)d], st), "hipEventRecord");
    if (int rc = launch_frame(m->scenes[(size_t)d], a, p->samples_per_unit, false, st, progress ? &pr[(size_t)d] : nullptr))
      return rc;
    HIP_TRY(hipEventRecord(t1[(size_t)d], st), "hipEventRecord");
    HIP_TRY(hipEventRecord(done[(size_t)d], st), "hipEventRecord");
  }
  // 2. progress on this thread while the devices render
  std::vector<Progress*> pp;
  uint64_t total_px = 0;
  for (auto& x : pr) { pp.push_back(&x); total_px += x.pixels; }
  if (int rc = wait_with_progress(done, m->devices, pp, total_px, progress, user)) return rc;
  // 3. ONE gather to devices[0] (one group over the single-process communicators), then unpack
  HIP_TRY(hipSetDevice(m->devices[0]), "hipSetDevice");
  if (int rc = ensure_recv(m->comms[0], pk_bytes * (size_t)n)) return rc;
  NCCL_TRY(ncclGroupStart(), "ncclGroupStart");
  for (int d = 0; d < n; ++d) {
    (void)hipSetDevice(m->devices[(size_t)d]);
    yart_comm* c = m->comms[(size_t)d];
    ncclResult_t r = ncclGather(m->packed[(size_t)d], d == 0 ? c->recv : nullptr, pk_bytes / sizeof(double), ncclFloat64, 0,
                                c->comm, m->streams[(size_t)d]);
    if (r != ncclSuccess) { (void)ncclGroupEnd(); return nccl_fail(r, "ncclGather"); }
  }
  NCCL_TRY(ncclGroupEnd(), "ncclGroupEnd");
  HIP_TRY(hipSetDevice(m->devices[0]), "hipSetDevice");
  hipStream_t st0 = m->streams[0];
  HIP_TRY(launch_unpack_shards(m->comms[0]->recv, (uint32_t)n, pk_bytes / sizeof(double), W, H, m->frame, st0),
          "launch k_unpack_shards");
  HIP_TRY(hipEventCreate(&g1), "hipEventCreate");
  std::unique_ptr<std::remove_pointer<hipEvent_t>::type, decltype(&hipEventDestroy)> hold(g1, &hipEventDestroy);
  HIP_TRY(hipEventRecord(g1, st0), "hipEventRecord");
  HIP_TRY(hipMemcpyAsync(xyz_sum_out, m->frame, frame_bytes, hipMemcpyDeviceToHost, st0), "copy frame");
  HIP_TRY(hipStreamSynchronize(st0), "gather");
  for (int d = 1; d < n; ++d) {
    HIP_TRY(hipSetDevice(m->devices[(size_t)d]), "hipSetDevice");
    HIP_TRY(hipStreamSynchronize(m->streams[(size_t)d]), "gather");
  }
  // timing: slowest device's render; gather + unpack on the root after its render
  double r = 0.0;
  for (int d = 0; d < n; ++d) {
    float ms = 0.0f;
    HIP_TRY(hipSetDevice(m->devices[(size_t)d]), "hipSetDevice");
    HIP_TRY(hipEventElapsedTime(&ms, t0[(size_t)d], t1[(size_t)d]), "hipEventElapsedTime");
    if (ms > r) r = ms;
  }
  float gms = 0.0f;
  HIP_TRY(hipSetDevice(m->devices[0]), "hipSetDevice");
  HIP_TRY(hipEventElapsedTime(&gms, t1[0], g1), "hipEventElapsedTime");
  m->render_ms = r;
  m->gather_ms = gms;
  return ok();
}

int yart_multi_last_timing(const yart_multi* m, double* render_ms, double* gather_ms) {
  if (!m || !render_ms || !gather_ms) return fail(YART_ERR_INVALID, "null argument");
  *render_ms = m->render_ms;
  *gather_ms = m->gather_ms;
  return ok();
}

void yart_multi_destroy(yart_multi* m) { delete m; }

}  // extern "C"
