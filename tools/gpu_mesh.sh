#!/bin/bash
# One gpurun call for the mesh walk: mesh parity tests, C4/C5 timings with work counters (front
# to back and reference order), and an A/B of variant builds on the david scene. Each GPU step
# has its own time limit; the script stops at the first failure.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-12} "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after rc=$rc"; exit $rc; }
}
STEPS=${STEPS:-"pytest configs ab"}
for s in $STEPS; do
  case $s in
    pytest) run mesh_pytest 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread \
              -k "${PYTEST_K:-david or sycee or bunny or qbvh or C4 or C5}" ;;
    configs) run mesh_configs 600 python tools/bench_configs.py --configs ${CONFIGS:-C4,C5} --spp-scale ${SPP_SCALE:-0.0625} ;;
    configs_ref) YART_OPTIONS=mesh_walk_ref=1 run mesh_configs_ref 600 python tools/bench_configs.py --configs ${CONFIGS:-C4,C5} --spp-scale ${SPP_SCALE:-0.0625} ;;
    ab) run mesh_ab 900 python tools/ab.py yet-another-raytracer_amd/lib/libyart.so ${AB_LIBS:-} --scene ${AB_SCENE:-david} \
          --w ${AB_W:-1920} --h ${AB_H:-1080} --spp ${AB_SPP:-16} --reps 2 ;;
  esac
done
echo ALL_OK
