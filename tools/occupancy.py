"""Lane occupancy per region of k_render (needs a -DYART_OCC build, e.g.
`make variant NAME=occ DEFS="-DYART_OCC"`). Usage on the GPU box:
    YART_DEVICE_LIB=.../libyart_occ.so python tools/occupancy.py cornell-box 800 800 16
Prints, per region, wave executions, mean active lanes and the share of all region executions.
"""
import ctypes as C
import json
import sys

import torch  # noqa: F401  (HIP runtime first)

sys.path.insert(0, "yet-another-raytracer_amd")
import yart  # noqa: E402

NAMES = ["iter", "fresh", "lamb", "lamb_light", "lamb_cos", "diel", "metal", "walk", "term", "assign"]


def main():
    scene, w, h, spp = sys.argv[1], *map(int, sys.argv[2:5])
    L = yart.load_device()
    fn = L.yart_debug_occupancy
    fn.argtypes = [C.c_int, C.POINTER(C.c_ulonglong)]
    buf = (C.c_ulonglong * 32)()
    p = yart.Preset(scene)
    s = yart.DeviceScene(p)
    fn(0, buf)  # reset
    s.render(p.camera(w, h), yart.render_params(w, h, spp, 50))
    assert fn(0, buf) == 0
    out = {}
    for i, n in enumerate(NAMES):
        waves, lanes = buf[2 * i], buf[2 * i + 1]
        out[n] = {"wave_execs": waves, "mean_lanes": round(lanes / waves, 2) if waves else 0,
                  "per_iter": round(waves / buf[0], 3) if buf[0] else 0}
    print(json.dumps({"scene": scene, "w": w, "h": h, "spp": spp, "regions": out}, indent=1))


if __name__ == "__main__":
    main()
