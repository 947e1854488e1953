"""Timeline of the bench's two-stream frames (study tool for the bimodal bench line).

Renders the bench frame (cornell-box 800x800x256) K times alternating over S streams, as bench.py's
timed loop does, `loops` times in one process with a synchronize between loops, and prints per loop
the time per frame and, per frame, when its stream reached it and when it finished (ms from the
loop's first event):

    python tools/stream_timeline.py [--loops 8 --frames 20 --streams 2]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
import torch  # noqa: E402
import yart  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loops", type=int, default=8)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--spp", type=int, default=256)
    a = ap.parse_args()
    W = H = 800
    p = yart.Preset("cornell-box")
    cam = p.camera(W, H)
    prm = yart.render_params(W, H, a.spp, 50)
    s = yart.DeviceScene(p)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(a.streams - 1)]
    outs = [torch.zeros((H, W, 3), dtype=torch.float64, device="cuda:0") for _ in streams]
    for k in range(2 * a.streams):  # warm-up
        st = streams[k % a.streams]
        s.render_async(cam, prm, outs[k % a.streams].data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    for loop in range(a.loops):
        t0 = torch.cuda.Event(enable_timing=True)
        t0.record(streams[0])
        for st in streams[1:]:
            st.wait_event(t0)
        evs = []
        w0 = time.perf_counter()
        for i in range(a.frames):
            st = streams[i % a.streams]
            b, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b.record(st)
            s.render_async(cam, prm, outs[i % a.streams].data_ptr(), st.cuda_stream)
            e.record(st)
            evs.append((i % a.streams, b, e))
        torch.cuda.synchronize()
        wall = (time.perf_counter() - w0) * 1e3
        rows = [(k, round(t0.elapsed_time(b), 2), round(t0.elapsed_time(e), 2)) for k, b, e in evs]
        ends = [r[2] for r in rows]
        print(json.dumps({"loop": loop, "ms_per_frame": round(wall / a.frames, 3),
                          "last_end_ms": max(ends), "frames": rows}), flush=True)
    for st in streams:
        r, acc, n = s.frame_timing(st.cuda_stream)
        print(json.dumps({"stream_render_ms_per_frame": round(r / max(1, n), 3), "frames": n}))


if __name__ == "__main__":
    main()
