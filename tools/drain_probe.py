"""Walk-drain probe: renders a mesh frame with the work counters (the instrumented STATS kernel) on
the tree's libyart (or YART_DEVICE_LIB) and prints the cooperative walk's rounds and the quad
slots of those rounds that held no ray — the drain: a round runs for the whole wave however few
quads still walk. Since r05 the STATS kernel counts idle slots itself (coop_idle_slots); r04's
patched probe build counted only the rounds with the wave's own pool exhausted (profiles/
r04_drain_probe.log), which with per-wave pools were the same slots.
    python tools/drain_probe.py david 960 540 16"""
import sys
from pathlib import Path

import torch  # noqa: F401

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
import yart  # noqa: E402

scene, W, H, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
p = yart.Preset(scene)
s = yart.DeviceScene(p)
img, st = s.render_with_stats(p.camera(W, H), yart.render_params(W, H, spp, 50))
rounds, walks, idle = st.coop_rounds, st.coop_walks, st.coop_idle_slots
steps = st.node_visits + st.leaf_visits
print(f"{scene} {W}x{H}x{spp}: walks {walks}, rounds {rounds} ({rounds / walks:.1f} per walk), quad steps {steps} "
      f"({steps / (16 * rounds):.1%} of quad slots)")
print(f"  segments {st.segments}, wave walks per 64 segments {64 * walks / st.segments:.2f}")
print(f"  idle quad slots {idle} ({idle / (16 * rounds):.1%} of all quad slots)")
