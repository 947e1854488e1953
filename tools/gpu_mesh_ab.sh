#!/bin/bash
# Variant A/B (one gpurun call): default libyart.so vs lib/variants/libyart_<v>.so for v in VARS,
# on the frames in SCENES ("name w h spp;..."; default the bunny stand-in and david frames).
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$REPO/gpurun_out; mkdir -p "$OUT"; cd "$REPO"
L=yet-another-raytracer_amd/lib
VARS=${VARS:-"ldsray mesh3"}
SCENES=${SCENES:-"bunny 800 800 32;david 1920 1080 16"}
libs="$L/libyart.so"; for v in $VARS; do libs="$libs $L/variants/libyart_$v.so"; done
IFS=';' read -ra list <<< "$SCENES"
for sc in "${list[@]}"; do
  set -- $sc
  timeout -k 10 600 python3 tools/ab.py $libs --scene $1 --w $2 --h $3 --spp $4 --reps 3 > "$OUT/ab_$1.log" 2>&1 || { echo "fail $1"; tail -20 "$OUT/ab_$1.log"; exit 1; }
  grep '"lib"' "$OUT/ab_$1.log"
done
echo ALL_OK
