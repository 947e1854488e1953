"""A/B timing of libyart.so builds on one GPU: each library in its own process (so each binds its
own code object), same frame, interleaved repeats. Usage (on the GPU box):
    python tools/ab.py LIB1 LIB2[@opt=v,...] ... [--scene cornell-box --w 800 --h 800 --spp 64 --reps 3]
"""
import argparse
import json
import os
import subprocess
import sys

CHILD = r'''
import json, sys, time, torch
sys.path.insert(0, "yet-another-raytracer_amd"); sys.path.insert(0, "tests")
import yart
scene, w, h, spp, depth, check = sys.argv[1], *map(int, sys.argv[2:7])
p = yart.Preset(scene); cam = p.camera(w, h)
import os, ctypes
if os.environ.get("AB_DROP"):  # experiments: the preset without the listed objects (indices into its list)
    d = p.desc.contents
    keep = [i for i in range(d.n_objects) if str(i) not in os.environ["AB_DROP"].split(":")]
    kept = (type(d.objects[0]) * len(keep))(*[d.objects[i] for i in keep])
    d.objects = ctypes.cast(kept, type(d.objects)); d.n_objects = len(keep)
s = yart.DeviceScene(p)
out = torch.zeros((h, w, 3), dtype=torch.float64, device="cuda:0"); st = torch.cuda.current_stream()
prm = yart.render_params(w, h, spp, depth)
s.render_async(cam, yart.render_params(w, h, 1, depth), out.data_ptr(), st.cuda_stream); torch.cuda.synchronize()
ms = []
for _ in range(2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st); s.render_async(cam, prm, out.data_ptr(), st.cuda_stream); e1.record(st); torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1))
res = {"ms": min(ms), "Msps": w * h * spp / min(ms) / 1e3}
if check:
    import numpy as np, oracle_lib as O
    cw, ch = 64, 48
    g = s.render(p.camera(cw, ch), yart.render_params(cw, ch, 4, depth))
    c = O.OracleScene(p.desc).render(p.camera(cw, ch), yart.render_params(cw, ch, 4, depth))
    res["bitwise_equal_64x48x4"] = bool(np.array_equal(g, c))
print("RESULT " + json.dumps(res))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--scene", default="cornell-box")
    ap.add_argument("--w", type=int, default=800)
    ap.add_argument("--h", type=int, default=800)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    results = {lib: [] for lib in a.libs}
    for rep in range(a.reps):
        for lib in a.libs:
            # LIB@opt=v,opt=v: the same library under library options (yart YART_OPTIONS)
            path, _, opts = lib.partition("@")
            env = dict(os.environ, YART_DEVICE_LIB=os.path.abspath(path))
            if opts:
                env["YART_OPTIONS"] = opts
            r = subprocess.run([sys.executable, "-c", CHILD, a.scene, str(a.w), str(a.h), str(a.spp), str(a.depth),
                                "1" if rep == 0 else "0"], env=env, capture_output=True, text=True, timeout=600)
            line = [l for l in r.stdout.splitlines() if l.startswith("RESULT ")]
            if r.returncode != 0 or not line:
                print(f"{lib}: FAILED rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
                sys.exit(1)
            res = json.loads(line[0][7:])
            results[lib].append(res)
            print(f"{a.scene} rep{rep} {os.path.basename(path)}{'@' + opts if opts else ''}: {res}", flush=True)
    for lib, rs in results.items():
        print(json.dumps({"lib": os.path.basename(lib.split("@")[0]) + ("@" + lib.split("@", 1)[1] if "@" in lib else ""), "scene": a.scene, "best_ms": min(r["ms"] for r in rs),
                          "Msamples_per_s": max(r["Msps"] for r in rs),
                          "bitwise": rs[0].get("bitwise_equal_64x48x4")}), flush=True)


if __name__ == "__main__":
    main()
