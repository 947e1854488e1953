"""World-BVH walk probe: renders a no-mesh frame with the work counters (STATS kernel) and prints
the per-lane walk's SIMT efficiency — the loop iterations the waves issue against the node visits
and primitive tests their lanes make (is the random scene's per-lane walk worth
a quad-cooperative form?).
    python tools/world_probe.py random-scene 1200 800 8"""
import sys
from pathlib import Path

import torch  # noqa: F401

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
import yart  # noqa: E402

scene, W, H, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
p = yart.Preset(scene)
s = yart.DeviceScene(p)
print(f"world nodes {s.info().world_nodes}, depth {s.info().world_depth}")
img, st = s.render_with_stats(p.camera(W, H), yart.render_params(W, H, spp, 50))
seg = st.segments
print(f"{scene} {W}x{H}x{spp}: samples {st.samples}, segments {seg} ({seg / st.samples:.2f} per sample)")
print(f"  per segment: node visits {st.node_visits / seg:.2f}, primitive tests {st.prim_tests / seg:.2f}, "
      f"light re-tests {st.light_tests / seg:.2f}")
print(f"  wave loop iterations {st.world_iters} ({st.world_leaf_iters / max(1, st.world_iters):.1%} with a lane at a leaf); "
      f"lane node visits per wave iteration {st.node_visits / max(1, st.world_iters):.1f} of 64")
