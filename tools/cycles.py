"""Shader-clock cycles per region of k_render (needs a -DYART_PROF build:
`make variant NAME=prof DEFS="-DYART_PROF"`). Usage on the GPU box:
    YART_DEVICE_LIB=.../libyart_prof.so python tools/cycles.py cornell-box 800 800 16
Prints, per region, the wave-cycles spent in it (summed over waves; a divergent region counts once
per wave execution) and its share of the loop's cycles. Regions nest: lamb / metal / diel are
inside scatter. The probe itself costs time (an s_memtime and an LDS add per region execution).
"""
import ctypes as C
import json
import sys
import time

import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, "yet-another-raytracer_amd")
import yart  # noqa: E402

NAMES = ["loop", "assign", "rng", "camera", "scatter", "lamb", "metal", "diel", "world", "shade", "term"]
WAVES = len(NAMES)


def main():
    scene, w, h, spp = sys.argv[1], *map(int, sys.argv[2:5])
    L = yart.load_device()
    fn = L.yart_debug_cycles
    fn.argtypes = [C.c_int, C.POINTER(C.c_ulonglong)]
    buf = (C.c_ulonglong * 16)()
    p = yart.Preset(scene)
    s = yart.DeviceScene(p)
    cam, prm = p.camera(w, h), yart.render_params(w, h, spp, 50)
    s.render(cam, prm)  # warm-up
    fn(0, buf)  # reset
    t0 = time.perf_counter()
    s.render(cam, prm)
    ms = (time.perf_counter() - t0) * 1e3
    assert fn(0, buf) == 0
    loop = buf[0] or 1
    regions = {n: {"cycles": buf[i], "share_of_loop": round(buf[i] / loop, 4)} for i, n in enumerate(NAMES)}
    inner = sum(buf[i] for i in (1, 2, 3, 4, 8, 9, 10))
    regions["other"] = {"cycles": loop - inner, "share_of_loop": round((loop - inner) / loop, 4)}
    print(json.dumps({"scene": scene, "w": w, "h": h, "spp": spp, "waves": buf[WAVES], "host_ms": round(ms, 2),
                      "regions": regions}, indent=1))


if __name__ == "__main__":
    main()
