"""Unit size (samples_per_unit) against render time for one preset frame, interleaved over reps on
one box: the persistent-wave plan's ~64 units per wave (capi.cpp `plan`) was tuned on the cornell
box; this checks it on other frames at their BASELINE spp.
    python tools/plan_sweep.py david 1920 1080 1024 0,32,64,u128,u256 [reps] [shard/count]
N = samples_per_unit N (0: the library's own plan); uN = the library's plan with the option
units_per_wave = N. Prints k_render + k_accumulate ms per frame."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
import yart  # noqa: E402


def main():
    scene, w, h, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    spus = sys.argv[5].split(",")
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 2
    si, sc = (int(x) for x in (sys.argv[7] if len(sys.argv) > 7 else "0/1").split("/"))
    p = yart.Preset(scene)
    cam = p.camera(w, h)
    s = yart.DeviceScene(p)
    out = torch.zeros((h, w, 3), dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream()
    prm = {u: yart.render_params(w, h, spp, 50, shard_index=si, shard_count=sc,
                                 samples_per_unit=0 if u.startswith("u") else int(u)) for u in spus}
    upw = {u: int(u[1:]) if u.startswith("u") else 0 for u in spus}
    s.render_async(cam, prm[spus[0]], out.data_ptr(), st.cuda_stream)  # warm-up (code object, scratch)
    torch.cuda.synchronize()
    s.frame_timing(st.cuda_stream)
    res = {u: [] for u in spus}
    for rep in range(reps):
        for u in spus:
            yart.set_option("units_per_wave", upw[u])
            s.render_async(cam, prm[u], out.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            r, a, n = s.frame_timing(st.cuda_stream)
            res[u].append(r + a)
            print(f"rep {rep} spu {u}: {r:.2f} + {a:.2f} ms, {w * h * spp / sc / (r + a) / 1e3:.1f} Msamples/s", flush=True)
    for u in spus:
        best = min(res[u])
        print(f"{scene} {w}x{h}x{spp} shard {si}/{sc} spu {u}: best {best:.2f} ms, {w * h * spp / sc / best / 1e3:.1f} Msamples/s")


if __name__ == "__main__":
    main()
