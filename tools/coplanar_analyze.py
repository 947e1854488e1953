"""Offline study of the near-coplanar divergences tools/coplanar_debug.py collected on the GPU
(gpurun_out/coplanar_<scene>.npz): for every ray whose GPU answer differs from the oracle's, the
ray is taken into each mesh instance's local frame exactly as the oracle does (oracle.c
object_hit: translate / rotate_y wrappers, outermost first), and Moller-Trumbore is run in numpy,
in the reference's operation order (qbvh.rs:420-450), against every triangle of the mesh. Printed
per ray: the oracle's and the GPU's t, every triangle with a valid hit, and where each hit's t lies
against the slab interval [entry, exit] of that triangle's own bounding box along the ray.
    python tools/coplanar_analyze.py david"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import mt_numpy as MT  # noqa: E402
import yart  # noqa: E402


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "david"
    z = np.load(ROOT / "gpurun_out" / f"coplanar_{scene}.npz")
    p = yart.Preset(scene)
    desc = p.desc.contents
    meshes = {k: MT.mesh_triangles(desc, k) for k in range(int(desc.n_meshes))}
    objs = [(i, desc.objects[i]) for i in range(int(desc.n_objects)) if desc.objects[i].kind == yart.abi.PRIM_MESH]
    rays, oh, oo = z["rays"], z["oracle_h"], z["oracle_o"]
    for name in ("f2b", "ref"):
        bad = z[name + "_bad"]
        print(f"== {name}: {len(bad)} rays differ")
        for j, i in enumerate(bad):
            r = rays[i]
            print(f"ray {i}: oracle obj {oo[i]} t {oh[i, 0]!r}; gpu obj {z[name + '_o'][j]} t {z[name + '_h'][j, 0]!r}")
            for oi, obj in objs:
                o, d = MT.local_ray(obj, r[0:3], r[3:6])
                tris = meshes[int(obj.mesh)]
                idx, t, a = MT.mt_all(tris, o, d, r[6], r[7])
                if len(idx) == 0:
                    print(f"   obj {oi}: no triangle hit")
                    continue
                ent, ext = MT.own_box_interval(tris, idx, o, d, r[6])
                order = np.argsort(t[idx])
                for k in order[:6]:
                    tt = t[idx[k]]
                    where = "inside" if ent[k] <= tt <= ext[k] else ("BEFORE" if tt < ent[k] else "AFTER")
                    print(f"   obj {oi} tri {idx[k]}: t {tt!r} box [{ent[k]!r}, {ext[k]!r}] {where}  a {a[idx[k]]:.3e}")


if __name__ == "__main__":
    main()
