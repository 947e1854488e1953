#!/bin/bash
# One gpurun call: the cycle breakdown of k_render per region (the -DYART_PROF build) on the
# scenes given (default cornell-box, random-scene, bunny, david), each step under its own limit.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
LIB=$REPO/yet-another-raytracer_amd/lib/variants/libyart_prof.so
for c in ${CASES:-"cornell-box:800:800:16" "random-scene:600:400:8" "bunny:800:800:8" "david:960:540:4"}; do
  IFS=: read -r sc w h spp <<< "$c"
  YART_DEVICE_LIB=$LIB timeout -k 10 120 python3 tools/cycles.py "$sc" "$w" "$h" "$spp" > "$OUT/cycles_$sc.json" 2> "$OUT/cycles_$sc.err"
  rc=$?
  echo "== $sc rc=$rc"; cat "$OUT/cycles_$sc.json"
  [ $rc -eq 0 ] || { tail -5 "$OUT/cycles_$sc.err"; exit $rc; }
done
echo ALL_OK
