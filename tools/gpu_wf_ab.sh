#!/bin/bash
# Wavefront path A/B (one gpurun call): the wavefront / deep-mesh GPU tests, then david and bunny
# frames on the default library, a variant and the megakernel (YART_OPTIONS=mesh_wavefront=0).
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
VAR=${VAR:-persist}
run wf_tests 600 python3 -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "${PYTEST_K:-deep or wavefront}"
for sc in "bunny 800 800 32" "david 1920 1080 16"; do
  set -- $sc
  run ab_$1 600 python3 tools/ab.py $L/libyart.so $L/variants/libyart_$VAR.so --scene $1 --w $2 --h $3 --spp $4 --reps 2
  YART_OPTIONS=mesh_wavefront=0 run ab_mega_$1 600 python3 tools/ab.py $L/libyart.so --scene $1 --w $2 --h $3 --spp $4 --reps 2
done
echo ALL_OK
