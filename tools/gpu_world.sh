#!/bin/bash
# One gpurun call for the world BVH: its parity tests, C3 timings with work counters for the SAH
# and the median-split trees, and an A/B against a baseline library on random-scene.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-6} "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after rc=$rc"; exit $rc; }
}
run world_pytest 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "${PYTEST_K:-world_bvh or random or C3 or three-spheres}"
run world_c3_sah 300 python tools/bench_configs.py --configs C3 --spp-scale ${SPP_SCALE:-0.0625}
run world_ab 600 python tools/ab.py yet-another-raytracer_amd/lib/libyart.so ${AB_LIBS:-} --scene random-scene --w 1200 --h 800 --spp 16 --reps 2
echo ALL_OK
