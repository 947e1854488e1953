"""Predict strong scaling on one GPU: time the render of shard 0 of N (what each of N GPUs does,
before the reduce) for the cornell bench frame. Prints Msamples/s the N-GPU job would reach if the
reduce were free, and the per-shard kernel time.
    python tools/shard_sim.py [--n 1,2,4,8] [--spu 0]"""
import argparse
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
import yart  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="1,2,4,8")
    ap.add_argument("--spu", type=int, default=0)
    ap.add_argument("--scene", default="cornell-box")
    ap.add_argument("--w", type=int, default=800)
    ap.add_argument("--h", type=int, default=800)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--all", action="store_true", help="time every shard of each N (load balance), not only shard 0")
    a = ap.parse_args()
    p = yart.Preset(a.scene)
    cam = p.camera(a.w, a.h)
    s = yart.DeviceScene(p)
    out = torch.zeros((a.h, a.w, 3), dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream()
    for n, k in [(n, k) for n in map(int, a.n.split(",")) for k in (range(n) if a.all else [0])]:
        prm = yart.render_params(a.w, a.h, a.spp, 50, shard_index=k, shard_count=n, samples_per_unit=a.spu)
        s.render_async(cam, prm, out.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        best = 1e30
        s.frame_timing(st.cuda_stream)  # reset the per-stream kernel times
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            s.render_async(cam, prm, out.data_ptr(), st.cuda_stream)
            e1.record(st)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        r_ms, acc_ms, frames = s.frame_timing(st.cuda_stream)
        print(json.dumps({"n": n, "shard": k, "spu": a.spu, "shard_ms": round(best, 3),
                          "k_render_ms": round(r_ms / max(frames, 1), 3), "k_accumulate_ms": round(acc_ms / max(frames, 1), 3),
                          "predicted_Msamples_per_s": round(a.w * a.h * a.spp / (best * 1e-3) / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
