#!/bin/bash
# Walk-tree builder knobs A/B (one gpurun call): SAH bins and the 4-way expansion choice.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$REPO/gpurun_out; mkdir -p "$OUT"; cd "$REPO"
L=yet-another-raytracer_amd/lib
if [ -f $L/variants/libyart_sort.so ]; then
  timeout -k 10 400 python3 tools/ab.py $L/libyart.so $L/variants/libyart_sort.so --scene cornell-box --w 800 --h 800 --spp 64 --reps 3 > "$OUT/ab_sort.log" 2>&1 || { echo "sort A/B failed"; tail -20 "$OUT/ab_sort.log"; exit 1; }
  tail -n 2 "$OUT/ab_sort.log"
fi
for sc in "bunny 800 800 32" "david 1920 1080 16"; do
  set -- $sc
  for cfg in "32 0" "16 0" "64 0" "32 1" "32 2"; do
    set -- $sc; b=${cfg% *}; p=${cfg#* }
    YART_WALK_BINS=$b YART_WALK_PICK=$p timeout -k 10 300 python3 tools/ab.py $L/libyart.so --scene $1 --w $2 --h $3 --spp $4 --reps 2 > "$OUT/tune_${1}_${b}_${p}.log" 2>&1 || { echo "fail $1 $b $p"; exit 1; }
    echo "$1 bins=$b pick=$p: $(tail -n 1 $OUT/tune_${1}_${b}_${p}.log)"
  done
done
echo ALL_OK
