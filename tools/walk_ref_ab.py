"""Default (front-to-back) mesh walk vs the reference-order walk (option mesh_walk_ref = 1) on one
GPU, same process, same frames (qbvh.rs:427-429, 492-531):
  * timing: each scene is created once per option value and rendered `reps` times alternately,
    best of the reps per option;
  * full frames: the same frame rendered both ways, compared value by value (XYZ sums, f64) and
    as finalized RGBA8 pixels.
    python tools/walk_ref_ab.py [--frames C4,C5] [--reps 3] [--full]
--full renders the BASELINE sizes (C4 bunny 800x800x512, C5 david 1920x1080x1024); without it the
timing frames only (C4 800x800x32, C5 1920x1080x64)."""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
import yart  # noqa: E402

FRAMES = {"C4": ("bunny", 800, 800, 32, 512), "C5": ("david", 1920, 1080, 64, 1024)}


def render(scene, p, w, h, spp):
    cam = p.camera(w, h)
    out = torch.zeros((h, w, 3), dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream()
    scene.frame_timing(st.cuda_stream)
    t0 = time.perf_counter()
    scene.render_async(cam, yart.render_params(w, h, spp, 50), out.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    r, _, n = scene.frame_timing(st.cuda_stream)
    return out, (r / n if n else wall * 1e3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", default="C4,C5")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--full", action="store_true")
    a = ap.parse_args()
    for key in a.frames.split(","):
        name, w, h, spp_t, spp_full = FRAMES[key]
        p = yart.Preset(name)
        scenes = {}
        for ref in (0, 1):
            with yart.option("mesh_walk_ref", ref):
                scenes[ref] = yart.DeviceScene(p)
        for ref in (0, 1):  # warm-up (code object load, scratch)
            render(scenes[ref], p, 64, 64, 1)
        ms = {0: [], 1: []}
        for _ in range(a.reps):
            for ref in (0, 1):
                _, t = render(scenes[ref], p, w, h, spp_t)
                ms[ref].append(t)
        best = {k: min(v) for k, v in ms.items()}
        print(json.dumps({"frame": key, "scene": name, "w": w, "h": h, "spp": spp_t, "ms_default": ms[0],
                          "ms_walk_ref": ms[1], "best_default": best[0], "best_walk_ref": best[1],
                          "walk_ref_cost_pct": round(100.0 * (best[1] / best[0] - 1.0), 2)}), flush=True)
        spp_c = spp_full if a.full else spp_t
        imgs = {}
        for ref in (0, 1):
            img, t = render(scenes[ref], p, w, h, spp_c)
            imgs[ref] = (img.cpu().numpy(), t)
        d0, d1 = imgs[0][0], imgs[1][0]
        diff_vals = int(np.count_nonzero(d0.view(np.uint64) != d1.view(np.uint64)))
        diff_px = int(np.count_nonzero((d0.view(np.uint64) != d1.view(np.uint64)).any(axis=2)))
        rgba = [yart.finalize_rgba8(imgs[r][0], spp_c) for r in (0, 1)]
        diff_rgba = int(np.count_nonzero((rgba[0] != rgba[1]).any(axis=2)))
        print(json.dumps({"frame": key, "scene": name, "w": w, "h": h, "spp": spp_c, "full_size": bool(a.full),
                          "ms_default": imgs[0][1], "ms_walk_ref": imgs[1][1],
                          "xyz_values_differing": diff_vals, "pixels_differing_xyz": diff_px,
                          "pixels_differing_rgba8": diff_rgba, "pixels": w * h}), flush=True)
        for s in scenes.values():
            s.close()


if __name__ == "__main__":
    main()
