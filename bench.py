"""bench.py — BASELINE.json's headline metric on MI355X.

Metric: Msamples/s (W x H x spp / s) for cornell-box 800x800, 256 spp, depth 50 (configs[1]);
ms_per_step is the wall-clock of one frame. A step = one frame of the hot path: the frame's 8x8
pixel blocks are dealt to the N GPUs (block b -> GPU b % N), each GPU renders its blocks with the
HIP megakernel through the C ABI, and the frame is finalized (XYZ -> sRGB RGBA8) on GPU 0. For
N > 1 each GPU renders straight into its block-packed shard and ONE RCCL gather over xGMI issued
by libyart itself assembles GPU 0's frame. Two ways to run N GPUs, one data path:

  python bench.py --gpus N          one process drives N GPUs (yart_render_multi_async: every
                                    device's render, the grouped ncclGather behind it and the
                                    unpack are stream-ordered, no host wait or copy per frame)
  torchrun --nproc-per-node N bench.py --gpus N
                                    one process per GPU (yart_render_packed_async +
                                    yart_gather_frame_async); torch.distributed (gloo) is only the
                                    control plane (communicator id, barriers, max-over-ranks time)

--gpus N must match the launch: N > 1 without torchrun needs N visible GPUs, and under torchrun
WORLD_SIZE must equal N; otherwise bench.py exits non-zero rather than report another N.
Inputs (scene, BVH, camera) are resident in HBM before the timed region. Scaling is strong: the
frame is fixed as N grows.

Also reported on the same line:
  roofline      the render kernel's average launch duration (HIP events the library records on
                the stream it launches on) against the f64 VALU peak, with ALGORITHMIC FLOPs =
                the kernel's own work counters (an untimed instrumented launch of the same frame)
                x the per-operation FLOP model in DESIGN.md ("achieved_kind": modelled, not a
                counter reading); HBM traffic from the committed rocprofv3 PMC snapshot, reported
                only while it belongs to the current kernel source (sha256 of csrc/kernels.hip).
  cpu_baseline  the CPU restatement (oracle/) on this host's cores, rank 0 only, on a bounded
                sample of the same workload (same frame at fewer spp; Msamples/s is ~spp-invariant),
                with the host's nproc, usable CPUs and CPU model.
  david         BASELINE configs[4] (david 1920x1080, depth 50, the config BASELINE assigns to 8
                GPUs) at --david-spp (default 64 = 1/16 of its 1024 spp), through the same N-GPU data
                path: one warm-up and --david-frames timed frames after the headline's, ms per frame,
                Msamples/s and the per-device render / gather times. A sub-record: `value` stays C2's.
"""
import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import torch  # first: libyart.so binds to the HIP runtime torch loaded (shared device pointers)
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
import yart  # noqa: E402
from yart.shard import PackedGather  # noqa: E402
from yart.watchdog import Watchdog, wait_events  # noqa: E402

WORKLOAD = dict(scene="cornell-box", width=800, height=800, spp=256, max_depth=50)
METRIC = "Msamples/sec (WxHxspp/sec), cornell-box 800x800x256spp depth 50"

# Stage deadlines (yart/watchdog.py): a stage that waits on device work gets 20x
# the one-GPU frame time per frame it waits for, plus a fixed allowance (120 s; the
# YART_BENCH_DEADLINE_S environment variable of this script overrides it, for tests), so a hang in a
# communicator's setup, a render or a gather ends with one JSON line naming the stage and exit 3.
ONE_GPU_FRAME_S = 0.05  # the C2 frame on one MI355X: 29 ms measured (profiles/r03q_bench_cornell.log), rounded up
BASE_DEADLINE_S = float(os.environ.get("YART_BENCH_DEADLINE_S", "120"))


def frames_deadline(n_frames):
    return BASE_DEADLINE_S + 20.0 * ONE_GPU_FRAME_S * n_frames

# f64 FLOPs per counted operation (DESIGN.md "Roofline"): add/sub/mul/div/sqrt = 1, compares 0.
FLOPS = {
    "sample": 40,        # jitter, wavelength, camera ray, CIE lookup, sanitize, accumulate
    "segment": 150,      # hit-record wrappers + material scatter + mixture pdf + ONB
    "prim": 14,          # average analytic primitive test (rect 8, sphere 28)
    "node": 96,          # QBVH inner node: 4 children x 3 axes slab (sub, mul) x 2 + min/max
    "leaf_tri": 45,      # Moller-Trumbore in f64
    "light": 30,         # pdf_value re-test of a light (rect 20, sphere 38)
}
F64_VALU_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (spec, FMA = 2 FLOPs)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-spp", type=int, default=128, help="spp of the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads for the CPU baseline (0 = the CPUs this process may use, at most 16: "
                         "the GPU box's share per GPU)")
    ap.add_argument("--no-stats", action="store_true", help="skip the instrumented launch (roofline = null)")
    ap.add_argument("--spu", type=int, default=0, help="samples per work unit (0 = library's choice)")
    ap.add_argument("--david-spp", type=int, default=64,
                    help="spp of the david (configs[4]) sub-record (0 = skip it)")
    ap.add_argument("--david-frames", type=int, default=2, help="timed frames of the david sub-record")
    ap.add_argument("--streams", type=int, default=2,
                    help="frames alternate over this many HIP streams (2: the next frame's render fills the SIMD "
                         "slots the previous frame's last paths leave idle; 1: strictly one after another)")
    return ap.parse_args()


def host_cpus():
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:  # cgroup v2 CPU quota, if any ("max 100000" = none)
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = round(int(q) / int(period), 2)
    except Exception:
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {"nproc": os.cpu_count(), "usable": usable, "cgroup_quota": quota, "model": model}


def cpu_baseline(preset, cam, w, h, spp, depth, threads):
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O
    hc = host_cpus()
    if threads <= 0:
        threads = min(16, hc["usable"], int(hc["cgroup_quota"]) if hc["cgroup_quota"] else 1 << 30)
        threads = max(1, threads)
    scene = O.OracleScene(preset.desc)
    prm = yart.render_params(w, h, spp, depth)
    t0 = time.perf_counter()
    scene.render(cam, prm, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": round(w * h * spp / dt / 1e6, 3), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{WORKLOAD['scene']} {w}x{h}x{spp}spp depth {depth} (full frame, reduced spp), "
                      f"{dt:.2f} s on {threads} threads, oracle/ C restatement (reference-semantics, not the Rust binary)",
            "host": hc}


def kernels_sha256():
    return hashlib.sha256((ROOT / "yet-another-raytracer_amd" / "csrc" / "kernels.hip").read_bytes()).hexdigest()


def pmc_snapshot(build_id):
    """The committed rocprofv3 PMC summary of the render kernel (tools/profile.sh +
    tools/summarize_profiles.py), if it was taken on the library this run loaded (its build id,
    the sha256 of every libyart.so source) — or, for a snapshot older than build ids, on the
    current kernels.hip."""
    p = ROOT / "profiles" / "pmc_render_cornell.json"
    if not p.exists():
        return {}, "no profile"
    try:
        pmc = json.loads(p.read_text())
    except Exception:
        return {}, "unreadable profile"
    if "build_id" in pmc:
        if pmc["build_id"] != build_id:
            return {}, "stale: profiles/pmc_render_cornell.json was taken on another libyart.so build"
        return pmc, "profiles/pmc_render_cornell.json (rocprofv3 --pmc snapshot of this libyart.so build)"
    if pmc.get("kernels_sha256") != kernels_sha256():
        return {}, "stale: profiles/pmc_render_cornell.json was taken on another kernels.hip"
    return pmc, "profiles/pmc_render_cornell.json (rocprofv3 --pmc snapshot of this kernel source)"


def device_balance(render_ms, gather_ms):
    """Per-device render / gather times of an N-GPU frame (ms, one frame): the fields that say,
    when a scaling run falls short, whether load imbalance or the gather is the cause (VERDICT r04
    item 5). gather_ms[d] is device d's own gather interval (it includes waiting for the others)."""
    n = len(render_ms)
    mean = sum(render_ms) / n if n else 0.0
    return {"per_device_render_ms": [round(x, 3) for x in render_ms],
            "per_device_gather_ms": [round(x, 3) for x in gather_ms] if gather_ms is not None else None,
            "render_max_over_mean": round(max(render_ms) / mean, 4) if mean > 0 else None,
            "slowest_device": int(max(range(n), key=lambda d: render_ms[d])) if n else None}


def valu_issue(pmc):
    """Fraction of SIMD cycles with a VALU instruction executing: SQ_ACTIVE_INST_VALU counts
    quad-cycles per wave, summed over the chip's 1,024 SIMDs; GRBM_GUI_ACTIVE is summed over
    the 8 XCDs."""
    try:
        simd_cycles = pmc["GRBM_GUI_ACTIVE"] / 8 * 1024
        return round(4 * pmc["SQ_ACTIVE_INST_VALU"] / simd_cycles, 4)
    except (KeyError, ZeroDivisionError):
        return None


def valu_lanes(pmc):
    """Active lanes per VALU instruction of the render kernel:
    SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU, and the same ratio of k_accumulate from the same
    pass (full 64-lane waves), which calibrates the two counters' units; `active_lanes` = 64 x the
    kernel's ratio / k_accumulate's."""
    r, c = pmc.get("valu_thread_per_active_inst"), pmc.get("calib_k_accumulate_thread_per_active_inst")
    if r is None:
        return None
    return {"thread_cycles_per_active_inst": round(r, 3), "k_accumulate_ratio": round(c, 3) if c else None,
            "active_lanes": round(64.0 * r / c, 2) if c else None,
            "source": "SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU (PMC snapshot)"}


def fp64_issue(pmc, kern_ms):
    """Hardware-counted FP64 work of the snapshot: SQ_INSTS_VALU_FLOPS_FP64 counts FLOPs per wave
    instruction (add/mul/trans 1, FMA 2); x 64 lanes, exec mask not applied, so an upper bound on
    the FP64 pipe's useful work. Plus the VALU instruction mix behind the issue-bound roofline."""
    try:
        lane_flops = pmc["SQ_INSTS_VALU_FLOPS_FP64"] * 64
        f64 = sum(pmc[k] for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                   "SQ_INSTS_VALU_TRANS_F64"))
        valu = pmc["SQ_INSTS_VALU"]
    except KeyError:
        return None
    tf = lane_flops / (kern_ms * 1e-3) / 1e12
    return {"lane_flops_per_launch": int(lane_flops), "tflops": round(tf, 3),
            "frac": round(tf / F64_VALU_PEAK_TFLOPS, 4),
            "valu_mix": {"f64_arith": round(f64 / valu, 4), "int32": round(pmc["SQ_INSTS_VALU_INT32"] / valu, 4),
                         "other": round(1 - (f64 + pmc["SQ_INSTS_VALU_INT32"]) / valu, 4)},
            "kind": "counted (PMC snapshot): f64 wave instructions x 64 lanes, inactive lanes included"}


def launch_mode(a):
    """(mode, world, rank, local): 'single' (one GPU), 'multi' (one process, N GPUs) or 'ranks' (one
    process per GPU under torch.distributed.run). Exits non-zero when --gpus and the launch disagree."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and int(env_world) > 1 or (env_world is not None and a.gpus > 1):
        world = int(env_world)
        if world != a.gpus:
            sys.exit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
                     f"(torch.distributed.run --nproc-per-node {a.gpus}) or run without a launcher")
        return "ranks", world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus < 1:
        sys.exit(f"bench.py: --gpus {a.gpus}")
    if a.gpus > 1:
        have = torch.cuda.device_count()  # counts devices without initialising the GPU
        if have < a.gpus:
            sys.exit(f"bench.py: --gpus {a.gpus} but {have} GPU(s) visible; refusing to report another N")
        return "multi", a.gpus, 0, 0
    return "single", 1, 0, 0


DAVID = dict(scene="david", width=1920, height=1080, max_depth=50)
DAVID_FRAME_S = 0.5  # one GPU, 64 spp: ~0.41 s measured (r05m C5 324.5 Msamples/s), rounded up


def david_record(a, mode, world, rank, local, dev, wd, comm, nccl_group, rehearse):
    """The david sub-record (BASELINE configs[4] at --david-spp) over the launch's N-GPU path, after
    the headline measurement: scene upload, one warm-up frame, a barrier, --david-frames frames
    timed (max over ranks), per-device render / gather times, and for N > 1 the assembled frame
    checked bitwise against a one-device render of the same frame."""
    W, H, depth, spp = DAVID["width"], DAVID["height"], DAVID["max_depth"], a.david_spp
    nfr = max(1, a.david_frames)
    per_frame = DAVID_FRAME_S * spp / 64.0
    deadline = lambda k: BASE_DEADLINE_S + 20.0 * per_frame * k  # noqa: E731
    preset = yart.Preset(DAVID["scene"])
    cam = preset.camera(W, H)
    st = torch.cuda.current_stream(dev)
    frame = torch.zeros((H, W, 3), dtype=torch.float64, device=dev)
    scene = multi = None
    with wd.stage(f"david: scene upload ({mode})", BASE_DEADLINE_S + 10.0 * world):
        if mode == "multi":
            multi = yart.MultiScene(preset, list(range(world)))
        else:
            scene = yart.DeviceScene(preset.desc, device=local)
    if mode == "ranks":
        prm = yart.render_params(W, H, spp, depth, shard_index=rank, shard_count=world)
        packed = torch.zeros(yart.shard_packed_len(W, H, 0, world), dtype=torch.float64, device=dev)
        pg = None if comm is not None else PackedGather(W, H, world, rank, torch.device("cpu") if rehearse else dev)
    else:
        prm = yart.render_params(W, H, spp, depth)
    gtimes = []

    def one():
        if mode == "single":
            scene.render_async(cam, prm, frame.data_ptr(), st.cuda_stream)
        elif mode == "multi":
            multi.render_async(cam, prm, frame.data_ptr(), st.cuda_stream)
        else:
            scene.render_packed_async(cam, prm, packed.data_ptr(), st.cuda_stream)
            g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            g0.record(st)
            if comm is not None:
                comm.gather_frame_async(packed.data_ptr(), W, H, frame.data_ptr(), st.cuda_stream)
            elif rehearse:
                ph, fh = packed.cpu(), torch.zeros_like(frame, device="cpu")
                pg(ph, fh, dist)
                if rank == 0:
                    frame.copy_(fh)
            else:
                pg(packed, frame, dist, group=nccl_group)
            g1.record(st)
            gtimes.append((g0, g1))

    def timing():
        if mode == "multi":
            return multi.frame_timing()
        return scene.frame_timing(st.cuda_stream)

    with wd.stage("david: warm-up frame", deadline(1)):
        one()
        wait_events([_event(st)])
    timing()
    gtimes.clear()
    if mode == "ranks":
        with wd.stage("david: barrier before the timed frames", BASE_DEADLINE_S):
            dist.barrier()
    with wd.stage("david: timed frames", deadline(nfr)):
        t0 = time.perf_counter()
        for _ in range(nfr):
            one()
        wait_events([_event(st)])
    if mode == "ranks":
        with wd.stage("david: barrier after the timed frames", BASE_DEADLINE_S):
            dist.barrier()
    elapsed = time.perf_counter() - t0
    if mode == "ranks":
        with wd.stage("david: max-over-ranks time", BASE_DEADLINE_S):
            t = torch.tensor([elapsed], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
    render_ms, _, n = timing()
    balance = None
    if mode == "multi":
        dr, dg, dn = multi.device_timing()
        balance = device_balance([x / max(1, dn) for x in dr], [x / max(1, dn) for x in dg])
    elif mode == "ranks":
        mine = torch.tensor([render_ms / max(1, n), sum(x.elapsed_time(y) for x, y in gtimes) / max(1, len(gtimes))],
                            dtype=torch.float64)
        every = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
        with wd.stage("david: per-rank timings", BASE_DEADLINE_S):
            dist.all_gather(every, mine)
        balance = device_balance([float(t[0]) for t in every], [float(t[1]) for t in every])
    else:
        balance = device_balance([render_ms / max(1, n)], None)
    check = None
    if rank == 0 and world > 1:
        with wd.stage("david: frame check (one-device render)", deadline(world)):
            one_dev = scene if scene is not None else yart.DeviceScene(preset.desc, device=local)
            full = torch.zeros_like(frame)
            one_dev.render_async(cam, yart.render_params(W, H, spp, depth), full.data_ptr(), st.cuda_stream)
            wait_events([_event(st)])
        assert torch.equal(full, frame), "david: assembled frame differs from the one-device render"
        check = "assembled frame bitwise equal to the one-device render"
    if multi is not None:
        multi.close()
    samples = W * H * spp
    return {"workload": f"david {W}x{H}x{spp}spp depth {depth} (BASELINE configs[4] at {spp}/1024 of its spp)",
            "spp": spp, "warmup": 1, "frames": nfr, "n_gpus": world,
            "ms_per_frame": round(elapsed / nfr * 1e3, 3),
            "msamples_per_s": round(samples * nfr / elapsed / 1e6, 3),
            "kernel_ms": round(render_ms / max(1, n), 3), "device_balance": balance, "frame_check": check}


def _event(st):
    ev = torch.cuda.Event()
    ev.record(st)
    return ev


def main():
    a = parse()
    mode, world, rank, local = launch_mode(a)
    wd = Watchdog(METRIC, rank=rank)
    # Rehearsal of the per-rank N>1 path on a 1-GPU box (RCCL refuses two ranks on one device): every
    # rank on device 0, the packed shards gathered over gloo on host copies. Never set for a real run.
    rehearse = mode == "ranks" and os.environ.get("YART_BENCH_SAME_DEVICE") == "1"
    if rehearse:
        local = 0
    if mode == "ranks":
        with wd.stage("process group init (gloo control plane)", BASE_DEADLINE_S):
            dist.init_process_group("gloo")  # control plane only
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    W, H, spp, depth = WORKLOAD["width"], WORKLOAD["height"], WORKLOAD["spp"], WORKLOAD["max_depth"]

    preset = yart.Preset(WORKLOAD["scene"])
    cam = preset.camera(W, H)
    shard_index, shard_count = (rank, world) if mode == "ranks" else (0, 1)
    prm = yart.render_params(W, H, spp, depth, shard_index=shard_index, shard_count=shard_count, samples_per_unit=a.spu)
    with wd.stage(f"scene upload (device {local})", BASE_DEADLINE_S):
        scene = yart.DeviceScene(preset.desc, device=local)
    multi = None
    if mode == "multi":
        with wd.stage(f"communicator init (yart_multi_create: {world} scene uploads + ncclCommInitAll)",
                      BASE_DEADLINE_S + 10.0 * world):
            multi = yart.MultiScene(preset, list(range(world)))
    # Frames alternate over S streams, each with its own frame / packed / RGBA buffers (and, inside
    # libyart, its own sample scratch and unit counter): frame k+1's persistent waves start in the
    # SIMD slots frame k's last long paths leave idle. Every frame is still rendered, gathered and
    # finalized whole; for N > 1 the collectives stay in step order on every rank (each gather waits
    # for the previous step's, an event across the streams; in the one-process path libyart orders
    # them itself).
    S = max(1, a.streams)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(S - 1)]
    stream = streams[0]
    frames = [torch.zeros((H, W, 3), dtype=torch.float64, device=dev) for _ in range(S)]  # rank 0: assembled
    rgbas = [torch.zeros((H, W, 4), dtype=torch.uint8, device=dev) for _ in range(S)]
    frame = frames[0]
    L = yart.load_device()  # refuses a libyart.so not built from this tree (yart.StaleLibraryError)
    build_id = L.yart_build_id().decode()

    # N > 1, one process per GPU: the data-plane collective, chosen ONCE and identically on every rank
    collective, comm, gather, nccl_group = None, None, None, None
    if mode == "multi":
        collective = "ncclGather (libyart yart_render_multi_async, one process, ncclCommInitAll)"
    if mode == "ranks":
        packeds = [torch.zeros(yart.shard_packed_len(W, H, 0, world), dtype=torch.float64, device=dev)
                   for _ in range(S)]
        if rehearse:
            collective = "gather (gloo rehearsal, host copies)"
            packed_h, frame_h = torch.zeros_like(packeds[0], device="cpu"), torch.zeros_like(frame, device="cpu")
            gather = PackedGather(W, H, world, rank, torch.device("cpu"))
        else:
            with wd.stage(f"communicator init (ncclCommInitRank, rank {rank} of {world})", BASE_DEADLINE_S + 10.0 * world):
                uid = [yart.Comm.unique_id() if rank == 0 else None]
                dist.broadcast_object_list(uid, src=0)
                ok = 1
                try:
                    comm = yart.Comm(uid[0], world, rank, local)
                except yart.YartError as e:
                    print(f"rank {rank}: libyart RCCL communicator failed ({e})", file=sys.stderr, flush=True)
                    ok = 0
                t = torch.tensor([ok], dtype=torch.int32)
                dist.all_reduce(t, op=dist.ReduceOp.MIN)
                if t.item():
                    collective = "ncclGather (libyart yart_gather_frame_async, RCCL, one rank per GPU)"
                else:  # the same packets through torch's RCCL process group
                    if comm is not None:
                        comm.close()
                        comm = None
                    nccl_group = dist.new_group(backend="nccl", device_id=dev)
                    gather = PackedGather(W, H, world, rank, dev)
                    collective = "gather (torch.distributed nccl, fallback)"

    coll_done = [None]  # the previous step's collective (ranks, N > 1): the next one waits for it
    gather_evs = []     # ranks, N > 1: this rank's (start, end) timing events around each step's gather
    last = {}           # the latest step's stage events (single / ranks): where a stalled frame stands

    def mark(key, st):
        ev = torch.cuda.Event()
        ev.record(st)
        last[key] = ev

    def where():
        """The watchdog's diagnosis: the stage the latest frame is stuck in."""
        if mode == "multi":
            state, unpacked = multi.query()
            if min(state) < 0:
                return {"frame": "being enqueued (a host call into RCCL or the render launch has not returned)"}
            waiting = [d for d, v in enumerate(state) if v == 0]
            if waiting:
                return {"frame": f"render on device(s) {waiting}", "device_state": state}
            waiting = [d for d, v in enumerate(state) if v == 1]
            if waiting:
                return {"frame": f"gather (device(s) {waiting} not through ncclGather)", "device_state": state}
            return {"frame": "unpack on device 0" if unpacked == 0 else "finalize on device 0", "device_state": state}
        for key in ("render", "gather", "end"):
            if key in last and not last[key].query():
                return {"frame": f"{key} on device {local}" + ("" if key != "gather" else f" (rank {rank} of {world})")}
        return {"frame": "host side (no device work pending)"}

    def step(i, streams=streams):
        k = i % len(streams)
        st, frame, rgba = streams[k], frames[k], rgbas[k]
        with torch.cuda.stream(st):
            if mode == "single":
                scene.render_async(cam, prm, frame.data_ptr(), st.cuda_stream)
                mark("render", st)
            elif mode == "multi":
                multi.render_async(cam, prm, frame.data_ptr(), st.cuda_stream)
            else:
                packed = packeds[k]
                scene.render_packed_async(cam, prm, packed.data_ptr(), st.cuda_stream)
                mark("render", st)
                if coll_done[0] is not None:
                    st.wait_event(coll_done[0])
                g0 = torch.cuda.Event(enable_timing=True)
                g0.record(st)
                if comm is not None:
                    comm.gather_frame_async(packed.data_ptr(), W, H, frame.data_ptr(), st.cuda_stream)
                elif rehearse:
                    packed_h.copy_(packed)
                    gather(packed_h, frame_h, dist)
                    if rank == 0:
                        frame.copy_(frame_h)
                else:
                    gather(packed, frame, dist, group=nccl_group)
                mark("gather", st)
                g1 = torch.cuda.Event(enable_timing=True)
                g1.record(st)
                gather_evs.append((g0, g1))
                coll_done[0] = last["gather"]
            if rank == 0:
                rc = L.yart_finalize_rgba8_async(local, yart.C.c_void_p(frame.data_ptr()), W, H, spp,
                                                 yart.C.c_void_p(rgba.data_ptr()), yart.C.c_void_p(st.cuda_stream))
                if rc != 0:
                    raise RuntimeError(L.yart_last_error().decode())
            mark("end", st)

    def drain_timing():
        """(render_ms, accumulate_ms or gather_ms, frames) summed over the frames since the last call."""
        if mode == "multi":
            return multi.frame_timing()
        r = acc = n = 0
        for st in streams:
            r1, a1, n1 = scene.frame_timing(st.cuda_stream)
            r, acc, n = r + r1, acc + a1, n + n1
        return r, acc, n

    def sync_all():
        """Every stream's queued work done, by polling an event on each (in the one-process N-GPU
        path each frame's unpack waits for every device's render and gather, and the caller stream
        waits for the unpack, so the caller streams' events cover all devices)."""
        evs = []
        for st in streams:
            ev = torch.cuda.Event()
            ev.record(st)
            evs.append(ev)
        wait_events(evs)

    # warm-up: W steps, and at least one frame on every stream (its scratch is allocated then)
    prep = max(0, S - a.warmup)
    with wd.stage("warm-up frames", frames_deadline(a.warmup + prep), where):
        for i in range(a.warmup + prep):
            step(i)
        sync_all()
    drain_timing()  # drop the warm-up frames' events
    if mode == "ranks":
        with wd.stage("barrier before the timed frames", BASE_DEADLINE_S):
            dist.barrier()
    gather_evs.clear()  # per-rank gather times: the timed frames (then, with S > 1, the one-stream frames)
    with wd.stage("timed frames", frames_deadline(a.steps), where):
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(i)
        sync_all()
    if mode == "ranks":
        with wd.stage("barrier after the timed frames", BASE_DEADLINE_S):
            dist.barrier()
    elapsed = time.perf_counter() - t0
    if mode == "ranks":
        with wd.stage("max-over-ranks time (all_reduce)", BASE_DEADLINE_S):
            t = torch.tensor([elapsed], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
    render_ms, accum_ms, nfr = drain_timing()
    overlap_ms = render_ms / max(1, nfr)  # k_render launch durations in the timed loop (overlapping for S > 1)
    # The roofline's kernel time: k_render alone. With S > 1 the launches in the timed loop overlap
    # (a launch's events bracket its wait for the slots the previous frame still holds), so the
    # kernel's own duration is taken from 3 frames on one stream right after the timed region.
    if S > 1:
        gather_evs.clear()
        with wd.stage("kernel-time frames (one stream)", frames_deadline(3), where):
            for i in range(3):
                step(i, streams=streams[:1])
            sync_all()
        render_ms, accum_ms, nfr = drain_timing()
    # per-device balance of the same frames (N > 1): render-kernel and own-gather time per device
    balance = None
    if mode == "multi":
        dr, dg, dn = multi.device_timing()
        balance = device_balance([x / max(1, dn) for x in dr], [x / max(1, dn) for x in dg])
    elif mode == "ranks":
        my_gather = (sum(a.elapsed_time(b) for a, b in gather_evs) / len(gather_evs)) if gather_evs else 0.0
        with wd.stage("per-rank timings (all_gather)", BASE_DEADLINE_S):
            mine = torch.tensor([render_ms / max(1, nfr), my_gather], dtype=torch.float64)
            every = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(every, mine)
        balance = device_balance([float(t[0]) for t in every], [float(t[1]) for t in every])
    kern_ms = render_ms / max(1, nfr)      # k_render average launch duration (one stream; multi: slowest GPU)
    accum_ms = accum_ms / max(1, nfr)      # k_accumulate (chunked path); multi: the root's gather + unpack
    if mode == "multi":
        gather_ms, accum_ms = accum_ms, None
    frame = frames[(a.steps - 1) % S]      # the last timed frame

    frame_check = None
    if rank == 0:  # the image really is the frame: finite, non-zero, and for N > 1 bitwise one device's
        f = frame.float()
        assert torch.isfinite(f).all() and f.abs().sum() > 0
        if world > 1:
            full = torch.zeros_like(frame)
            with wd.stage("frame check (one-device render of the whole frame)", frames_deadline(1)):
                scene.render_async(cam, yart.render_params(W, H, spp, depth), full.data_ptr(), stream.cuda_stream)
                sync_all()
            assert torch.equal(full, frame), "assembled frame differs from the one-device render"
            frame_check = "assembled frame bitwise equal to the one-device render"
            print(frame_check, file=sys.stderr, flush=True)
            scene.frame_timing(stream.cuda_stream)

    roofline = None
    cpu = None
    if rank == 0 and not a.no_stats:
        # shard 0's counted work (the whole frame at N = 1) over its kernel time
        with wd.stage("work counters (instrumented launch)", frames_deadline(10)):
            _, st = scene.render_with_stats(cam, yart.render_params(W, H, spp, depth, shard_index=0, shard_count=world))
        flops = (st.samples * FLOPS["sample"] + st.segments * FLOPS["segment"] + st.prim_tests * FLOPS["prim"] +
                 st.node_visits * FLOPS["node"] + st.leaf_tris * FLOPS["leaf_tri"] + st.light_tests * FLOPS["light"])
        achieved = flops / (kern_ms * 1e-3) / 1e12
        pmc, pmc_source = pmc_snapshot(build_id)
        traffic = pmc.get("hbm_bytes_per_launch") if world == 1 else None
        chunked = mode == "multi" or (accum_ms or 0) > 0
        roofline = {"bound": "valu", "achieved": round(achieved, 3), "peak": F64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / F64_VALU_PEAK_TFLOPS, 4), "traffic": traffic,
                    "achieved_kind": "modelled: algorithmic f64 FLOPs (kernel work counters x DESIGN.md FLOP model) "
                                     "/ HIP-event kernel time" + ("" if world == 1 else
                                                                   " (shard 0's work / the slowest GPU's kernel time)"),
                    "traffic_source": pmc_source if world == 1 else "not measured for a shard",
                    # k_render<HAS_MESH, BVH, STATS, DYN, EXT, DEEP>: the chunked (DYN) list kernel for this frame
                    "kernel": ("k_render<false,false,false,true,false,false>" if chunked
                               else "k_render<false,false,false,false,false,false>"),
                    "kernel_ms": round(kern_ms, 3),
                    "accumulate_ms": round(accum_ms, 3) if accum_ms is not None else None,
                    "kernel_ms_source": ("HIP events, 3 frames on one stream after the timed region" if S > 1
                                         else "HIP events over the timed steps"),
                    "timed_launch_ms": round(overlap_ms, 3),
                    "algorithmic_flops_per_launch": int(flops),
                    "counts": {"samples": st.samples, "segments": st.segments, "prim_tests": st.prim_tests,
                               "light_tests": st.light_tests, "node_visits": st.node_visits,
                               "leaf_tris": st.leaf_tris},
                    "hbm_frac": (round(traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6) if traffic else None),
                    # the sample scratch k_render writes (24 B of XYZ per sample)
                    "algorithmic_bytes_per_launch": st.samples * 24 if chunked else None,
                    # SURVEY §8(d)'s record bytes (24 B per rect / box-face / light re-test, 128 B per
                    # QBVH node, 36 B per leaf triangle): an algorithmic byte RATE served from the
                    # scalar / L1 caches (the scene is < 4 KB), not HBM traffic — reported beside the
                    # VALU bound, which is this kernel's roofline
                    "record_bytes_per_launch": int(24 * (st.prim_tests + st.light_tests) + 128 * st.node_visits +
                                                   36 * st.leaf_tris),
                    "record_byte_rate_of_hbm_peak": round((24 * (st.prim_tests + st.light_tests) + 128 * st.node_visits +
                                                           36 * st.leaf_tris) / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                    "valu_issue_busy": valu_issue(pmc) if world == 1 else None,
                    "valu_active_lanes": valu_lanes(pmc) if world == 1 else None,
                    "fp64_issued": fp64_issue(pmc, kern_ms) if world == 1 else None,
                    # wave-level VALU instructions (SQ_INSTS_VALU of the snapshot) per path segment
                    "valu_insts_per_segment": (round(pmc["SQ_INSTS_VALU"] / st.segments, 2)
                                               if world == 1 and pmc.get("SQ_INSTS_VALU") and st.segments else None)}
        if mode == "multi":
            roofline["gather_ms"] = round(gather_ms, 3)
        if balance is not None:
            roofline.update(balance)
    david = None
    if a.david_spp > 0:
        david = david_record(a, mode, world, rank, local, dev, wd, comm, nccl_group, rehearse)
    if rank == 0 and a.cpu_spp > 0 and world == 1:
        with wd.stage("cpu baseline (oracle on the host cores)", 900.0):
            cpu = cpu_baseline(preset, cam, W, H, a.cpu_spp, depth, a.cpu_threads)

    if rank == 0:
        samples = W * H * spp
        value = samples * a.steps / elapsed / 1e6
        line = {
            "metric": METRIC,
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic (reference scene preset, seeded Philox RNG)",
            "config": {"workload": "cornell-box 800x800x256spp depth 50 (BASELINE configs[1])", "width": W,
                       "height": H, "spp": spp, "max_depth": depth, "parallelism": f"pixel-blocks x{world}",
                       "launch": {"single": "one process, one GPU", "multi": "one process, N GPUs",
                                  "ranks": "one process per GPU (torch.distributed.run)"}[mode],
                       "streams": S, "prep_frames": prep,
                       "collective": collective, "frame_check": frame_check, "seed": yart.DEFAULT_SEED,
                       "build_id": build_id},
            "roofline": roofline, "cpu_baseline": cpu,
            # N > 1: per-device render / own-gather ms and render max / mean (also in roofline)
            "device_balance": balance,
            # BASELINE configs[4] (david, the 8-GPU config) at reduced spp on the same N-GPU path
            "david": david,
        }
        print(json.dumps(line), flush=True)
    with wd.stage("teardown (communicators, process group)", BASE_DEADLINE_S):
        if comm is not None:
            comm.close()
        if multi is not None:
            multi.close()
        if mode == "ranks":
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
