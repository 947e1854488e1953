"""Divergences of the mesh walk on near-coplanar rays (tests/test_gpu_parity.py
test_mesh_walk_near_coplanar_rays_match_oracle): the same rays through the default walk (front to
back + exact check) and the reference-order walk (option mesh_walk_ref = 1) on the GPU, each against
the oracle; every mismatching ray is written to gpurun_out/coplanar_<scene>.npz for offline study.
    python tools/coplanar_debug.py david 120 [n]"""
import sys
from pathlib import Path

import numpy as np
import torch  # noqa: F401  (the HIP runtime first)

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import oracle_lib as O  # noqa: E402
import yart  # noqa: E402
from test_gpu_parity import _mesh_triangles, _near_coplanar_rays  # noqa: E402

scene, reach = sys.argv[1], float(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 200000
p = yart.Preset(scene)
rays = _near_coplanar_rays(_mesh_triangles(p), n, seed=41, reach=reach)
h2, o2 = O.OracleScene(p.desc).intersect(rays)
out = {"rays": rays}
for name, opt in (("f2b", 0), ("ref", 1)):
    with yart.option("mesh_walk_ref", opt):
        s = yart.DeviceScene(p)
        h, o = s.intersect(rays)
    bad = np.flatnonzero((o != o2) | ((o >= 0) & np.any(h != h2, axis=1)))
    print(f"{scene} {name}: {len(bad)} of {n} differ from the oracle", flush=True)
    for i in bad[:20]:
        print(f"  ray {i}: gpu obj {o[i]} t {h[i, 0]!r}  oracle obj {o2[i]} t {h2[i, 0]!r}", flush=True)
    out[name + "_bad"] = bad
    out[name + "_h"], out[name + "_o"] = h[bad], o[bad]
out["oracle_h"], out["oracle_o"] = h2, o2
(ROOT / "gpurun_out").mkdir(exist_ok=True)
np.savez(ROOT / "gpurun_out" / f"coplanar_{scene}.npz", **out)
