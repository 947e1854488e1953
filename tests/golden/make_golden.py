"""Regenerate the committed golden fixtures (tests/golden/*.npz) from the CPU restatement.

    python tests/golden/make_golden.py

Each fixture is data: the inputs that define it (preset, size, spp, depth, seed, camera) and the
oracle's per-pixel f64 XYZ sums and RGBA8 output. They pin the restatement against regressions
(tests/test_golden.py, CPU) and give the device path a fixed target (GPU). The reference itself
cannot be run here (no Rust toolchain), so these are NOT reference outputs; see DESIGN.md §2."""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE.parent.parent / "yet-another-raytracer_amd"))
import oracle_lib as O  # noqa: E402
import yart  # noqa: E402

CASES = [
    # name, scene, W, H, spp, depth
    ("cornell_48x48x8", "cornell-box", 48, 48, 8, 50),
    ("two_spheres_100x56x4_d8", "two-spheres", 100, 56, 4, 8),  # C1 shape (row 55 unrendered)
    ("random_scene_36x24x4", "random-scene", 36, 24, 4, 50),
    ("bunny_standin_24x24x2", "bunny", 24, 24, 2, 50),
    ("david_32x18x2", "david", 32, 18, 2, 50),
    ("two_perlin_spheres_40x24x4", "two-perlin-spheres", 40, 24, 4, 50),  # Perlin marble
    ("simple_light_40x24x4", "simple-light", 40, 24, 4, 50),
    ("cornell_smoke_32x32x4", "cornell-box-smoke", 32, 32, 4, 50),  # ConstantMedium + Isotropic
]


def main():
    for name, scene, w, h, spp, depth in CASES:
        p = yart.Preset(scene)
        cam = p.camera(w, h)
        prm = yart.render_params(w, h, spp, depth)
        xyz = O.OracleScene(p.desc).render(cam, prm, threads=0)
        rgba = O.finalize(xyz, spp)
        np.savez_compressed(HERE / f"{name}.npz", scene=scene, width=w, height=h, spp=spp, depth=depth,
                            seed=yart.DEFAULT_SEED, xyz=xyz, rgba=rgba)
        print(name, xyz.mean())


if __name__ == "__main__":
    main()
