"""Marginal cost of one k_render region (needs a -DYART_DUP=k build:
`make variant NAME=dup1 DEFS="-DYART_DUP=1"`; 1 camera, 2 scatter, 3 world pass, 4 sample end).
The region runs n times per execution (n = 1, 2, 3); the frame must not change, and the slope of
the frame time in n is the time one execution of the region costs the kernel. Usage on the GPU box:
    YART_DEVICE_LIB=.../libyart_dup1.so python tools/dup_cost.py cornell-box 800 800 64
"""
import ctypes as C
import json
import os
import sys
import time

import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, "yet-another-raytracer_amd")
import yart  # noqa: E402

REGIONS = {1: "camera", 2: "scatter", 3: "world", 4: "sample_end"}


def main():
    scene, w, h, spp = sys.argv[1], *map(int, sys.argv[2:5])
    reps = 3
    L = yart.load_device()
    fn = getattr(L, "yart_debug_set_dup", None)  # absent from the default build: its time at n = 1 only
    if fn is not None:
        fn.argtypes = [C.c_int, C.c_uint]
    p = yart.Preset(scene)
    s = yart.DeviceScene(p)
    cam, prm = p.camera(w, h), yart.render_params(w, h, spp, 50)
    lib = os.path.basename(os.environ.get("YART_DEVICE_LIB", "libyart.so"))
    k = int(lib.split("dup")[1].split(".")[0]) if "dup" in lib else 0
    ms, ref = {}, None
    for n in ((1, 2, 3) if fn is not None else (1,)):
        if fn is not None:
            assert fn(0, n) == 0
        s.render(cam, prm)  # warm-up
        best = float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            img = s.render(cam, prm)
            best = min(best, (time.perf_counter() - t0) * 1e3)
        if ref is None:
            ref = img
        assert (img == ref).all(), f"frame changed at n={n}"
        ms[n] = round(best, 3)
    if fn is None:
        print(json.dumps({"lib": lib, "region": None, "scene": scene, "w": w, "h": h, "spp": spp, "ms": ms}), flush=True)
        return
    fn(0, 1)
    slope = ((ms[2] - ms[1]) + (ms[3] - ms[2])) / 2
    print(json.dumps({"lib": lib, "region": REGIONS.get(k, "?"), "scene": scene, "w": w, "h": h, "spp": spp, "ms": ms,
                      "slope_ms": round(slope, 3), "share_of_frame": round(slope / ms[1], 4)}), flush=True)


if __name__ == "__main__":
    main()
