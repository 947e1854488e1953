#!/bin/bash
# One gpurun call: marginal cost per k_render region (tools/dup_cost.py over the -DYART_DUP=k
# builds) on the scenes given; each step under its own limit, stop at the first failure.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
for c in ${CASES:-"cornell-box:800:800:64" "random-scene:600:400:16" "bunny:800:800:16"}; do
  IFS=: read -r sc w h spp <<< "$c"
  for k in ${REGIONS:-0 1 2 3 4 5}; do
    lib=$REPO/yet-another-raytracer_amd/lib/variants/libyart_dup$k.so
    [ "$k" = 0 ] && lib=$REPO/yet-another-raytracer_amd/lib/libyart.so
    YART_DEVICE_LIB=$lib \
      timeout -k 10 180 python3 tools/dup_cost.py "$sc" "$w" "$h" "$spp" >> "$OUT/dup_cost.jsonl" 2> "$OUT/dup_${sc}_${k}.err"
    rc=$?
    echo "== $sc dup$k rc=$rc"; tail -1 "$OUT/dup_cost.jsonl"
    [ $rc -eq 0 ] || { tail -5 "$OUT/dup_${sc}_${k}.err"; exit $rc; }
  done
done
echo ALL_OK
