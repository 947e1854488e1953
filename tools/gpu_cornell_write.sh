#!/bin/bash
# k_render WRITE_SIZE per launch for several libyart builds on bench.py's frame (one rocprofv3
# --pmc pass each), then an interleaved A/B of the same builds: LIBS="a.so b.so".
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$REPO/gpurun_out; mkdir -p "$OUT"; cd "$REPO"
i=0
for lib in ${LIBS}; do
  i=$((i+1))
  YART_DEVICE_LIB=$REPO/$lib PFX=w${i}_ PASSES="write" bash tools/profile.sh > /dev/null || exit 1
  python3 - "$OUT/w${i}_prof_write" "$lib" <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f)) if "k_render" in r["Kernel_Name"]]
print(sys.argv[2], "k_render WRITE_SIZE GB per launch", round(sum(v) / len(v) * 1024 / 1e9, 3), "launches", len(v))
PY
done
timeout -k 10 600 python tools/ab.py ${LIBS} --scene cornell-box --w 800 --h 800 --spp 64 --reps 3 > "$OUT/ab_write.log" 2>&1 || exit 1
grep '^{' "$OUT/ab_write.log"
