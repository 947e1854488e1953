#!/bin/bash
# Wavefront-path diagnostics (one gpurun call): the host's per-pass iteration log, rocprofv3
# kernel traces of a bunny and a david frame (wavefront vs megakernel) and an A/B of variants.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$REPO/gpurun_out; mkdir -p "$OUT"; cd "$REPO"
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-4} "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after rc=$rc"; exit $rc; }
}
export TMPDIR=/tmp
L=yet-another-raytracer_amd/lib
run wf_log_bunny 300 env YART_WF_LOG=1 python3 tools/render_once.py bunny 800 800 32 1
run wf_log_david 300 env YART_WF_LOG=1 python3 tools/render_once.py david 960 540 16 1
for sc in "bunny 800 800 32" "david 960 540 16"; do
  set -- $sc
  run wf_trace_$1 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wf_prof_$1" -o run -- python3 $REPO/tools/render_once.py $sc 2
done
for sc in "bunny 800 800 32" "david 1920 1080 16"; do
  set -- $sc
  run ab_$1 600 python3 tools/ab.py $L/libyart.so $L/variants/libyart_wf3.so --scene $1 --w $2 --h $3 --spp $4 --reps 2
  YART_MESH_WF=0 run ab_mega_$1 600 python3 tools/ab.py $L/libyart.so --scene $1 --w $2 --h $3 --spp $4 --reps 2
done
run ab_cornell 600 python3 tools/ab.py $L/libyart.so $L/variants/libyart_regen16.so $L/variants/libyart_regen32.so $L/variants/libyart_rectcull.so --scene cornell-box --w 800 --h 800 --spp 64 --reps 3
echo ALL_OK
