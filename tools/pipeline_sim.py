"""Frames back to back on one stream vs alternating over two or three streams (the next frame's render fills
the SIMD slots the previous frame's drain leaves idle), for the full frame and for shard 0 of N.
    python tools/pipeline_sim.py [--n 1,8] [--frames 20]"""
import argparse
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
import yart  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="1,8")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--scene", default="cornell-box")
    ap.add_argument("--w", type=int, default=800)
    ap.add_argument("--h", type=int, default=800)
    ap.add_argument("--spp", type=int, default=256)
    a = ap.parse_args()
    p = yart.Preset(a.scene)
    cam = p.camera(a.w, a.h)
    s = yart.DeviceScene(p)
    streams = [torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.zeros((a.h, a.w, 3), dtype=torch.float64, device="cuda:0") for _ in streams]
    for n in map(int, a.n.split(",")):
        prm = yart.render_params(a.w, a.h, a.spp, 50, shard_index=0, shard_count=n)
        res = {"n": n}
        for ns in (1, 2, 3, 1, 2, 3):
            for i in range(2 * ns):  # warm-up: scratch of every stream allocated
                s.render_async(cam, prm, outs[i % ns].data_ptr(), streams[i % ns].cuda_stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.frames):
                s.render_async(cam, prm, outs[i % ns].data_ptr(), streams[i % ns].cuda_stream)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.frames
            k = f"streams{ns}_ms"
            res[k] = round(min(ms, res.get(k, 1e30)), 3)
        assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
