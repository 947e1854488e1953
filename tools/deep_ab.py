"""A mesh deeper than depth 10 on one GPU: the megakernel with the walk stacks' HBM overflow (the
r05 default) against the wavefront path (mesh_wavefront = 1, the r02-r04 default for such meshes),
same process, alternating reps; the frames must be bitwise equal.
    python tools/deep_ab.py [W H spp reps]"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import yart  # noqa: E402
import oracle_lib as O  # noqa: E402
from yart import abi  # noqa: E402
from test_gpu_parity import _deep_grid  # noqa: E402

W, H, spp, reps = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (320, 320, 16, 3)))
pos, nrm = _deep_grid()
b = O.DescBuilder(background=(0.7, 0.8, 1.0))
w = b.material(abi.MAT_LAMBERTIAN, b.texture((0.6, 0.5, 0.4)))
g = b.material(abi.MAT_DIELECTRIC, 0, b=(1.62153902, 0.256287842, 1.64447552), c=(0.0122241457e6, 0.0595736775e6, 147.468793e6))
li = b.material(abi.MAT_DIFFUSE_LIGHT, b.texture((4.0, 4.0, 4.0)))
b.mesh(pos, nrm)
b.obj(abi.PRIM_MESH, w, mesh=0)
b.obj(abi.PRIM_MESH, g, mesh=0, xforms=[(abi.XF_TRANSLATE, (0.0, 0.3, 0.0))])
b.obj(abi.PRIM_SPHERE, li, (0.0, 2.0, 0.0, 0.5))
b.obj(abi.PRIM_SPHERE, li, (0.0, 2.0, 0.0, 0.5), light=True)
desc = b.desc()
scenes = {}
for name, wf in (("megakernel", -1), ("wavefront", 1)):
    with yart.option("mesh_wavefront", wf):
        scenes[name] = yart.DeviceScene(desc)
cam = yart.make_camera((0.3, 1.5, 2.0), (0.0, 0.0, 0.0), 40.0, W / H, 0.0)
prm = yart.render_params(W, H, spp, 50)
st = torch.cuda.current_stream()
ms, img = {k: [] for k in scenes}, {}
for rep in range(reps + 1):
    for k, s in scenes.items():
        out = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda:0")
        s.frame_timing(st.cuda_stream)
        s.render_async(cam, prm, out.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        r, _, n = s.frame_timing(st.cuda_stream)
        if rep:
            ms[k].append(r / max(1, n))
        img[k] = out.cpu().numpy()
best = {k: min(v) for k, v in ms.items()}
print(json.dumps({"mesh": "height field, 4,199,202 triangles, QBVH depth 11 (34 stack entries)", "frame": [W, H, spp],
                  "ms": ms, "best_ms": best, "megakernel_over_wavefront": round(best["wavefront"] / best["megakernel"], 3),
                  "bitwise_equal": bool(np.array_equal(img["megakernel"], img["wavefront"]))}))
