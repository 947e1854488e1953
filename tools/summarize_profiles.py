"""Summarize a tools/profile.sh run (gpurun_out/prof_*) into profiles/ (committed evidence).

    python tools/summarize_profiles.py <round-tag> [kernel-substring]

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats of the bench command),
profiles/<tag>_pmc.json (per-launch PMC values of the render kernel, HBM bytes with the gfx950
correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) x 1024 x 2 + WRITE_SIZE (KiB) x 1024)
and profiles/pmc_render_cornell.json (what bench.py reads for roofline.traffic).
"""
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OUT = ROOT / "gpurun_out"
PROF = ROOT / "profiles"


def per_launch(pass_dir, kernel):
    rows = list(csv.DictReader(open(OUT / pass_dir / "run_counter_collection.csv")))
    vals = {}
    for r in rows:
        if kernel in r["Kernel_Name"]:
            vals.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in vals.items()}, rows


def kernels_sha256():
    import hashlib
    return hashlib.sha256((ROOT / "yet-another-raytracer_amd" / "csrc" / "kernels.hip").read_bytes()).hexdigest()


def main():
    tag = sys.argv[1]
    kernel = sys.argv[2] if len(sys.argv) > 2 else "k_render<false, false, true>"
    pfx = sys.argv[3] if len(sys.argv) > 3 else ""  # tools/profile.sh PFX= of the run
    PROF.mkdir(exist_ok=True)
    shutil.copy(OUT / (pfx + "prof_trace") / "run_kernel_stats.csv", PROF / f"{tag}_kernel_stats.csv")
    summary = {"kernel": kernel, "source": "tools/profile.sh (rocprofv3 --pmc, one counter block per pass)"}
    t_trace = (OUT / (pfx + "prof_trace") / "run_kernel_trace.csv").stat().st_mtime
    for p in ("prof_fetch", "prof_write", "prof_valu", "prof_stall", "prof_mix", "prof_mem", "prof_icache"):
        f = OUT / (pfx + p) / "run_counter_collection.csv"
        # only the passes of the same run as the trace (a pass left under gpurun_out/ by an earlier
        # call would otherwise overwrite this run's counters)
        if f.exists() and abs(f.stat().st_mtime - t_trace) < 1800:
            v, rows = per_launch(pfx + p, kernel)
            summary.update(v)
            for r in rows:
                if kernel in r["Kernel_Name"]:
                    summary.setdefault("vgpr", int(r["VGPR_Count"]))
                    summary.setdefault("sgpr", int(r["SGPR_Count"]))
                    summary.setdefault("lds_bytes", int(r["LDS_Block_Size"]))
                    summary.setdefault("grid", int(r["Grid_Size"]))
                    break
    # the VALU active-lane ratio SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU of this kernel, and of
    # k_accumulate in the same pass: a streaming kernel whose waves run full (64 lanes) except at
    # the grid's end, so its ratio calibrates the counters' units
    if summary.get("SQ_THREAD_CYCLES_VALU") and summary.get("SQ_ACTIVE_INST_VALU"):
        summary["valu_thread_per_active_inst"] = summary["SQ_THREAD_CYCLES_VALU"] / summary["SQ_ACTIVE_INST_VALU"]
        if (OUT / (pfx + "prof_valu") / "run_counter_collection.csv").exists():
            cal, _ = per_launch(pfx + "prof_valu", "k_accumulate")
            if cal.get("SQ_THREAD_CYCLES_VALU") and cal.get("SQ_ACTIVE_INST_VALU"):
                summary["calib_k_accumulate_thread_per_active_inst"] = cal["SQ_THREAD_CYCLES_VALU"] / cal["SQ_ACTIVE_INST_VALU"]
    stats = list(csv.DictReader(open(PROF / f"{tag}_kernel_stats.csv")))
    for s in stats:
        if kernel in s["Name"]:
            summary["avg_duration_ns"] = float(s["AverageNs"])
            summary["calls"] = int(s["Calls"])
    fetch = summary.get("FETCH_SIZE")
    write = summary.get("WRITE_SIZE")
    if fetch is not None and write is not None:
        summary["hbm_bytes_per_launch"] = int(fetch * 1024 * 2 + write * 1024)
        summary["hbm_bytes_note"] = "FETCH_SIZE x2 (gfx950 reports half of wide reads) + WRITE_SIZE, KiB -> B"
    # which kernel source the counters belong to: bench.py reports the traffic only while
    # csrc/kernels.hip still hashes to this value
    summary["kernels_sha256"] = kernels_sha256()
    # and the library's build id (the sha256 of every source libyart.so is built from; the profiled
    # process refused to load a library whose id was not the tree's, yart/buildid.py)
    sys.path.insert(0, str(ROOT / "yet-another-raytracer_amd"))
    from yart import buildid
    summary["build_id"] = buildid.build_id()
    (PROF / f"{tag}_pmc.json").write_text(json.dumps(summary, indent=1) + "\n")
    if "cornell" in tag or tag.endswith("_render"):
        (PROF / "pmc_render_cornell.json").write_text(json.dumps(summary, indent=1) + "\n")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
