"""Which hit-record fields differ between the device (world BVH forced on) and the oracle on the
mixed lists of test_world_bvh_4wide_mixed_lists_match_linear_scan: per differing ray the object
kind, its wrappers and the differing columns (t, p xyz, n xyz, front face).
    python tools/world_mixed_debug.py 257"""
import sys
from pathlib import Path

import numpy as np
import torch  # noqa: F401

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import oracle_lib as O  # noqa: E402
import yart  # noqa: E402
from test_gpu_parity import _random_rays  # noqa: E402

n = int(sys.argv[1])
d = O.mixed_list_desc(n, seed=31 + n, spread=12.0).desc()
rays = np.concatenate([_random_rays(50000, -15, 15, seed=n), _random_rays(50000, -60, 60, seed=n + 1)])
h2, o2 = O.OracleScene(d).intersect(rays)
for opt in (1, 0):
    with yart.option("world_bvh", opt):
        s = yart.DeviceScene(d)
        h, o = s.intersect(rays)
    m = (o2 >= 0) & (o == o2)
    bad = np.flatnonzero(m & np.any(h.view(np.uint64) != h2.view(np.uint64), axis=1))
    print(f"world_bvh={opt}: {len(bad)} rays differ in the record, {(o != o2).sum()} in the object")
    kinds = {}
    for i in bad[:2000]:
        ob = d.contents.objects[o2[i]]
        key = (int(ob.kind), int(ob.n_xforms), tuple(np.flatnonzero(h[i].view(np.uint64) != h2[i].view(np.uint64))))
        kinds[key] = kinds.get(key, 0) + 1
    for k, v in sorted(kinds.items(), key=lambda kv: -kv[1])[:12]:
        print("  kind %d xforms %d columns %s: %d" % (k[0], k[1], k[2], v))
    for i in bad[:3]:
        print("  ray", i, "obj", o2[i], "dev", h[i].tolist(), "oracle", h2[i].tolist())
