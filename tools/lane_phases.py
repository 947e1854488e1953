"""Where the render kernel's lane-slots go, by phase.

The instrumented kernel (yart_render_with_stats, on the frame's own plan: the persistent waves for
chunked frames since r06) counts, from ballots, how many of a wave's 64 lanes
work each time a phase's code runs: the cooperative mesh walk's node branch and leaf branch (and the
quads idle in each walk's drain), the camera-ray branch and the scatter branch of the render loop.
Prints one JSON line per frame:

    python tools/lane_phases.py david 960 540 16 [cornell-box 800 800 16 ...]
(library options through YART_OPTIONS, e.g. YART_OPTIONS=mesh_park=0)
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
import yart  # noqa: E402


def phases(scene, w, h, spp, depth=50):
    p = yart.Preset(scene)
    s = yart.DeviceScene(p)
    _, st = s.render_with_stats(p.camera(w, h), yart.render_params(w, h, spp, depth))
    frac = lambda num, den: round(num / den, 4) if den else None  # noqa: E731
    r = {"scene": scene, "frame": f"{w}x{h}x{spp}", "segments": st.segments, "iterations": st.iterations,
         # render loop: lanes busy when the branch runs
         "camera_branch_lanes": frac(st.camera_lanes, 64 * st.camera_iters),
         "scatter_branch_lanes": frac(st.scatter_lanes, 64 * st.scatter_iters),
         "camera_iters_share": frac(st.camera_iters, st.iterations),
         "scatter_iters_share": frac(st.scatter_iters, st.iterations),
         "lanes_with_a_path": frac(st.camera_lanes + st.scatter_lanes, 64 * st.iterations)}
    if st.coop_rounds:
        r.update({
            "walk_rounds": st.coop_rounds,
            "walk_rounds_per_iteration": frac(st.coop_rounds, st.iterations),
            "node_branch_rounds_share": frac(st.coop_node_rounds, st.coop_rounds),
            "leaf_branch_rounds_share": frac(st.coop_leaf_rounds, st.coop_rounds),
            "node_branch_lanes": frac(st.coop_node_lanes, 64 * st.coop_node_rounds),
            "leaf_branch_quad_lanes": frac(st.coop_leaf_quad_lanes, 64 * st.coop_leaf_rounds),
            "leaf_branch_triangle_lanes": frac(st.coop_leaf_lanes, 64 * st.coop_leaf_rounds),
            "drain_idle_quad_slots": frac(st.coop_idle_slots, 16 * st.coop_rounds),
            "walk_calls": st.coop_walks, "walk_rounds_per_call": frac(st.coop_rounds, st.coop_walks),
            "mesh_segments_per_call": frac(st.segments, st.coop_walks),
            "parked_walks": st.parked_walks})
    if st.world_iters:
        r["world_walk_iterations"] = st.world_iters
    return r


def main(argv):
    if len(argv) < 5 or (len(argv) - 1) % 4:
        sys.exit(__doc__)
    for i in range(1, len(argv), 4):
        print(json.dumps(phases(argv[i], int(argv[i + 1]), int(argv[i + 2]), int(argv[i + 3]))), flush=True)


if __name__ == "__main__":
    main(sys.argv)
