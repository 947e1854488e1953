#!/bin/bash
# Mesh-kernel spill traffic A/B (one gpurun call): for the default library and
# each lib/variants/libyart_<v>.so in VARS,
#   * tools/ab.py timings on the david and bunny frames (interleaved, bitwise check vs the oracle),
#   * rocprofv3 FETCH_SIZE and WRITE_SIZE passes (one counter block per pass) over one david
#     960x540x16 frame (tools/render_once.py), summarized per k_render launch by tools/pmc_summary.py.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$REPO/gpurun_out; mkdir -p "$OUT"; cd "$REPO"
L=yet-another-raytracer_amd/lib
VARS=${VARS:-""}
TAG=${TAG:-spill}
FRAME=${FRAME:-"david 960 540 16"}
SCENES=${SCENES:-"david 1920 1080 16;bunny 800 800 32"}
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-4} "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after rc=$rc"; exit $rc; }
}
libs="$L/libyart.so"; for v in $VARS; do libs="$libs $L/variants/libyart_$v.so"; done
IFS=';' read -ra list <<< "$SCENES"
for sc in "${list[@]}"; do
  set -- $sc
  run ${TAG}_ab_$1 900 python3 tools/ab.py $libs --scene $1 --w $2 --h $3 --spp $4 --reps 3
done
for lib in $libs; do
  n=$(basename $lib .so)
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && YART_DEVICE_LIB=$REPO/$lib timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv \
      -d "$OUT/${TAG}_pmc_${n}_$c" -o run -- python3 $REPO/tools/render_once.py $FRAME 1 > "$OUT/${TAG}_pmc_${n}_$c.log" 2>&1) \
      || { echo "rocprof $n $c failed"; tail -5 "$OUT/${TAG}_pmc_${n}_$c.log"; exit 1; }
  done
  python3 tools/pmc_summary.py "$OUT/${TAG}_pmc_${n}_FETCH_SIZE" "$OUT/${TAG}_pmc_${n}_WRITE_SIZE" --label "$n $FRAME" | tee -a "$OUT/${TAG}_pmc_summary.jsonl"
done
echo ALL_OK
