"""Render one preset frame on cuda:0 through the C ABI (for rocprofv3 runs of scenes other than
bench.py's cornell box).
    python tools/render_once.py david 960 540 16 [frames]"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
import yart  # noqa: E402


def main():
    scene, w, h, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    frames = int(sys.argv[5]) if len(sys.argv) > 5 else 2
    p = yart.Preset(scene)
    cam = p.camera(w, h)
    s = yart.DeviceScene(p)
    out = torch.zeros((h, w, 3), dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream()
    for _ in range(frames):
        s.render_async(cam, yart.render_params(w, h, spp, 50), out.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    r, a, n = s.frame_timing(st.cuda_stream)
    print(f"{scene} {w}x{h}x{spp}: {n} frames, k_render {r / n:.2f} ms, k_accumulate {a / n:.3f} ms, "
          f"{w * h * spp / (r / n) / 1e3:.1f} Msamples/s")


if __name__ == "__main__":
    main()
