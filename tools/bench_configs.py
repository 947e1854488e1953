"""Time every BASELINE.json config on one MI355X (bench.py covers only the headline C2).

    python tools/bench_configs.py [--configs C2,C3,C4,C5] [--spp-scale 1.0] [--cpu]
    python tools/bench_configs.py --configs E1,E2,E3,E4,E5   # the feature presets (EXT kernels)

One untimed warm-up launch at 1 spp, then one timed frame (HIP events on the launch stream),
then an instrumented launch (work counters) of the same frame. Prints one JSON line per config.
C5 (david 1920x1080x1024, quoted on 8 GPUs) is timed here on one GPU and as one shard of 8."""
import argparse
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
sys.path.insert(0, str(ROOT / "tests"))
import yart  # noqa: E402
sys.path.insert(0, str(ROOT))
from bench import FLOPS, F64_VALU_PEAK_TFLOPS, HBM_PEAK_GBS  # noqa: E402  (the FLOP model of DESIGN.md)

CONFIGS = {
    "C1": ("two-spheres", 400, 225, 16, 8),
    "C2": ("cornell-box", 800, 800, 256, 50),
    "C3": ("random-scene", 1200, 800, 500, 50),
    "C4": ("bunny", 800, 800, 512, 50),
    "C5": ("david", 1920, 1080, 1024, 50),
    # not BASELINE configs: the SURVEY 8(f)1 feature presets (EXT kernels: Perlin noise, image
    # texture, area lights in the dark, a ConstantMedium, MovingSphere) and the list-walk three
    # spheres, at a common 64 spp, so each has a throughput figure
    "E1": ("two-perlin-spheres", 800, 450, 64, 50),
    "E2": ("earth", 800, 450, 64, 50),
    "E3": ("simple-light", 800, 450, 64, 50),
    "E4": ("cornell-box-smoke", 800, 800, 64, 50),
    "E5": ("three-spheres", 800, 450, 64, 50),
}


def run(name, scene_name, w, h, spp, depth, shard=(0, 1), stats=True, cpu=False, pmc=None):
    p = yart.Preset(scene_name)
    cam = p.camera(w, h)
    ts = time.perf_counter()
    s = yart.DeviceScene(p)
    scene_s = time.perf_counter() - ts  # host build (QBVH, world BVH) + upload, once per scene
    out = torch.zeros((h, w, 3), dtype=torch.float64, device="cuda:0")
    st = torch.cuda.current_stream()
    s.render_async(cam, yart.render_params(w, h, 1, depth, shard_index=shard[0], shard_count=shard[1]),
                   out.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    prm = yart.render_params(w, h, spp, depth, shard_index=shard[0], shard_count=shard[1])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(st)
    s.render_async(cam, prm, out.data_ptr(), st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1)
    n = w * h * spp // shard[1]
    line = {"config": name, "scene": scene_name, "stand_in": p.stand_in or None, "size": f"{w}x{h}x{spp}",
            "depth": depth, "shard": f"{shard[0]}/{shard[1]}", "kernel_ms": round(ms, 2), "wall_s": round(wall, 3),
            "Msamples_per_s": round(n / (ms * 1e-3) / 1e6, 2), "scene_create_s": round(scene_s, 3),
            # end to end: scene creation (build + upload) + the frame
            "Msamples_per_s_with_scene": round(n / (ms * 1e-3 + scene_s) / 1e6, 2)}
    if stats:
        _, c = s.render_with_stats(cam, prm)
        line["counts"] = {"samples": c.samples, "segments": c.segments, "prim_tests": c.prim_tests,
                          "node_visits": c.node_visits, "leaf_visits": c.leaf_visits, "leaf_tris": c.leaf_tris,
                          "light_tests": c.light_tests, "mesh_rewalks": c.mesh_rewalks, "coop_rounds": c.coop_rounds, "coop_leaf_rounds": c.coop_leaf_rounds, "coop_walks": c.coop_walks}
        info = s.info()
        line["scene_build_ms"] = round(info.bvh_build_ms, 2)   # host QBVH build (threaded), all meshes
        line["scene_upload_ms"] = round(info.upload_ms, 2)     # host -> device copies
        if info.bvh_nodes:
            line["bvh_tied_cuts"] = info.bvh_tied_cuts
            # algorithmic bytes of the traversal: 128 B per inner node visit,
            # 48 B per tested triangle record, at most 72 B of normals per segment
            b = 128 * c.node_visits + 48 * c.leaf_tris + 72 * c.segments
            line["traversal_bytes"] = b
            line["traversal_GBps"] = round(b / (ms * 1e-3) / 1e9, 1)
        # Both rooflines. FLOP side: the work counters x bench.py's per-operation FLOP
        # model (modelled). Byte side: SURVEY's algorithmic bytes of the records the walk reads —
        # mesh 128 B per inner node visit + 36 B per tested triangle + 60 B of closest-hit
        # attributes per segment (an upper bound: every segment counted), world-BVH 48 B per node,
        # list primitives 24 B per test and per light re-test — plus 48 B per sample of
        # chunked-path scratch (written by k_render, read by k_accumulate; 0 when fused). For the
        # mesh configs the bound is the larger fraction (SURVEY: HBM-bound traversal); the list
        # scenes' records are a few KB that live in the scalar/L1 caches, so their bound is VALU
        # issue whatever the byte fraction says (SURVEY: "unattainable by construction").
        flops = (c.samples * FLOPS["sample"] + c.segments * FLOPS["segment"] + c.prim_tests * FLOPS["prim"] +
                 c.node_visits * FLOPS["node"] + c.leaf_tris * FLOPS["leaf_tri"] + c.light_tests * FLOPS["light"])
        mesh = bool(info.bvh_nodes)
        nbytes = 128 * c.node_visits + 36 * c.leaf_tris + 60 * c.segments if mesh else 48 * c.node_visits
        nbytes += 24 * (c.prim_tests + c.light_tests)
        _, a_ms, frames = s.frame_timing(st.cuda_stream)  # warm-up + timed frame: accumulate time > 0 iff chunked
        nbytes += 48 * n if frames and a_ms > 0 else 0
        tf = flops / (ms * 1e-3) / 1e12
        gbs = nbytes / (ms * 1e-3) / 1e9
        ff, bf = tf / F64_VALU_PEAK_TFLOPS, gbs / HBM_PEAK_GBS
        line["roofline"] = {"flop_tflops_modelled": round(tf, 3), "flop_frac": round(ff, 4),
                            "alg_bytes": int(nbytes), "alg_GBps": round(gbs, 1), "alg_bytes_frac_of_hbm": round(bf, 4),
                            "alg_bytes_note": "SURVEY 8(d) record bytes; for meshes served from L2 / Infinity Cache, "
                                              "not HBM (see hbm_counter)",
                            "bound": ("hbm (algorithmic bytes)" if bf > ff else "valu (f64)") if mesh else "valu (f64)"}
        if pmc:  # HBM bytes the counters saw for a render of this same frame (rocprofv3, tools/gpu_round_end.sh)
            pm = json.loads(Path(pmc).read_text())
            hb = pm.get("hbm_bytes_per_launch")
            if hb:
                line["hbm_counter"] = {"bytes_per_launch": int(hb), "GBps": round(hb / (ms * 1e-3) / 1e9, 1),
                                       "frac_of_hbm": round(hb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                       "over_alg_bytes": round(hb / nbytes, 3), "kernel": pm.get("kernel"),
                                       "source": f"{pmc} (FETCH_SIZE x 2 + WRITE_SIZE per launch, MI355X_MICROARCH.md HBM)"}
    if cpu:
        import oracle_lib as O
        cspp = max(1, spp // 64)
        t0 = time.perf_counter()
        O.OracleScene(p.desc).render(cam, yart.render_params(w, h, cspp, depth), threads=16)
        dt = time.perf_counter() - t0
        line["cpu_Msamples_per_s_16thr"] = round(w * h * cspp / dt / 1e6, 3)
        line["cpu_sample"] = f"{w}x{h}x{cspp}"
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1,C2,C3,C4,C5")
    ap.add_argument("--spp-scale", type=float, default=1.0)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--pmc", action="append", default=[],
                    help="CFG=path: rocprofv3 PMC summary (tools/summarize_profiles.py) of a render of that config's frame")
    a = ap.parse_args()
    pmc = dict(x.split("=", 1) for x in a.pmc)
    for c in a.configs.split(","):
        scene, w, h, spp, depth = CONFIGS[c]
        spp = max(1, int(spp * a.spp_scale))
        if c == "C5":
            run(c + "-shard", scene, w, h, spp, depth, shard=(0, 8), stats=not a.no_stats, cpu=False)
        run(c, scene, w, h, spp, depth, stats=not a.no_stats, cpu=a.cpu, pmc=pmc.get(c))


if __name__ == "__main__":
    main()
