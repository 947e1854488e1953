"""Per-launch HBM bytes of k_render from rocprofv3 --pmc pass directories (one counter per pass):
    python tools/pmc_summary.py <fetch-pass-dir> <write-pass-dir> [--label L] [--kernel k_render]
Prints one JSON line: FETCH_SIZE / WRITE_SIZE per launch in GB (the counters are KiB), HBM bytes as
MI355X_MICROARCH.md's HBM section corrects them for gfx950 (FETCH x 2 + WRITE), and the average
kernel duration from the same passes."""
import argparse
import csv
import json
from pathlib import Path


def per_launch(d, kernel):
    vals, dur = {}, {}
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            vals.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for f in Path(d).rglob("*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                dur[r.get("Dispatch_Id", len(dur))] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    return {k: sum(v.values()) / len(v) for k, v in vals.items()}, (sum(dur.values()) / len(dur) if dur else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--label", default="")
    ap.add_argument("--kernel", default="k_render")
    a = ap.parse_args()
    f, fd = per_launch(a.fetch, a.kernel)
    w, wd = per_launch(a.write, a.kernel)
    fetch_gb = f.get("FETCH_SIZE", 0.0) * 1024 / 1e9
    write_gb = w.get("WRITE_SIZE", 0.0) * 1024 / 1e9
    print(json.dumps({"label": a.label, "kernel": a.kernel, "fetch_gb": round(fetch_gb, 3), "write_gb": round(write_gb, 3),
                      "hbm_gb_fetch2_plus_write": round(2 * fetch_gb + write_gb, 3),
                      "kernel_ms_fetch_pass": round(fd, 3) if fd else None, "kernel_ms_write_pass": round(wd, 3) if wd else None}))


if __name__ == "__main__":
    main()
