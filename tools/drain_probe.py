"""Walk-drain probe (a measurement build, tools/build_patched.sh with the drain patch): renders a
mesh frame with the work counters on a given libyart and prints the cooperative walk's rounds, the
rounds run with the wave's ray pool exhausted (every quad's next ray taken) and their idle quad
slots. The probe build reuses the rewalk / leaf-round counters for these two numbers.
    YART_DEVICE_LIB=yet-another-raytracer_amd/lib/variants/libyart_drain.so python tools/drain_probe.py david 960 540 16"""
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
rounds, walks = st.coop_rounds, st.coop_walks
drain, idle = st.mesh_rewalks, st.coop_leaf_rounds
steps = st.node_visits + st.leaf_visits
print(f"{scene} {W}x{H}x{spp}: walks {walks}, rounds {rounds} ({rounds / walks:.1f} per walk), quad steps {steps} "
      f"({steps / (16 * rounds):.1%} of quad slots)")
print(f"  segments {st.segments}, wave walks per 64 segments {64 * walks / st.segments:.2f} (a wave walks each mesh "
      f"instance a segment's rays may hit)")
print(f"  rounds with the pool exhausted: {drain} ({drain / rounds:.1%}); their idle quad slots {idle} "
      f"({idle / (16 * rounds):.1%} of all quad slots)")
