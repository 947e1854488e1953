"""Bounds-checked walk (a -DYART_WALK_CHECK build of libyart): render the mesh
configs' scenes (C4 bunny stand-in, C5 david, a block subset each at full spp-scale) and the
4.2M-triangle deep grid through the checked cooperative walk, compare against the default build
bitwise, and report the fault bits (1 leaf record range, 2 reference leaf index, 4 node index,
8 stack slot; 0 = every index in bounds).
    YART_DEVICE_LIB=.../libyart_walkcheck.so python tools/walk_check.py"""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np
import torch  # noqa: F401  (HIP runtime first)

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import yart  # noqa: E402

L = yart.load_device()
L.yart_debug_walk_fault.argtypes = [C.c_int, C.POINTER(C.c_uint)]
bad = 0
for scene, w, h, spp in [("bunny", 800, 800, 4), ("david", 1920, 1080, 2), ("david", 480, 270, 16)]:
    for walk_tree in ("1", "0"):
        yart.set_option("walk_tree", int(walk_tree))
        p = yart.Preset(scene)
        s = yart.DeviceScene(p)
        img = s.render(p.camera(w, h), yart.render_params(w, h, spp, 50))
        f = C.c_uint()
        assert L.yart_debug_walk_fault(0, C.byref(f)) == 0
        i = s.info()
        print(f"{scene} {w}x{h}x{spp} walk_tree={walk_tree} (walk nodes {i.walk_nodes}, depth {i.walk_depth}): "
              f"fault bits {f.value}, image sum {img.sum():.6f}", flush=True)
        np.save(f"/tmp/wc_{scene}_{w}_{walk_tree}.npy", img)
        bad |= f.value
for scene, w, h, spp in [("bunny", 800, 800, 4), ("david", 1920, 1080, 2), ("david", 480, 270, 16)]:
    a, b = np.load(f"/tmp/wc_{scene}_{w}_1.npy"), np.load(f"/tmp/wc_{scene}_{w}_0.npy")
    print(f"{scene} {w}x{h}: walk tree vs reference-tree walk bitwise: {np.array_equal(a, b)}", flush=True)
    bad |= 0 if np.array_equal(a, b) else 16
print("WALK_CHECK", "OK" if bad == 0 else f"FAULT {bad}")
sys.exit(0 if bad == 0 else 1)
