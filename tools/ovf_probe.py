"""Work counters of the deep-mesh walks on the stacked-layers mesh of
test_deep_mesh_overflow_stack_is_used_and_exact: per walk mode, node / leaf visits, walk rounds and
the stack entries pushed past the LDS slots (ovf_pushes). GPU only.

    python tools/ovf_probe.py
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import yart  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def main():
    b, d, _ = T._layer_stack()
    L = yart.load_device()
    cam = yart.make_camera((5400.0, 0.4, 0.4), (0.0, 0.4, 0.4), 0.02, 1.0, 0.0)
    prm = yart.render_params(8, 8, 1, 2)
    for mode in ("default", "reference_order", "lane_rewalk"):
        with yart.option("mesh_walk_ref", 1 if mode == "reference_order" else 0):
            s = yart.DeviceScene(d)
        i = s.info()
        if mode == "lane_rewalk":
            L.yart_debug_force_rewalk(0, 1)
        try:
            _, st = s.render_with_stats(cam, prm)
        finally:
            L.yart_debug_force_rewalk(0, 0)
        print(json.dumps({"mode": mode, "depth": i.bvh_max_depth, "max_stack": i.bvh_max_stack,
                          **{k: getattr(st, k) for k, _ in st._fields_ if k != "reserved"}}), flush=True)


if __name__ == "__main__":
    main()
