#!/bin/bash
# One development iteration on the GPU box (one gpurun call): the -m gpu suite, an A/B of the
# default build against variant builds (VARS, tools/ab.py via gpu_mesh_ab.sh on SCENES) and the
# work counters of CONFIGS (tools/bench_configs.py). Every GPU step has its own time limit and the
# script stops at the first failure.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$REPO/gpurun_out; mkdir -p "$OUT"; cd "$REPO"
TAG=${TAG:-iter}
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-6} "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after rc=$rc"; exit $rc; }
}
for s in ${STEPS:-pytest ab configs}; do
  case $s in
    pytest) run ${TAG}_gpu_tests 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    ab) run ${TAG}_ab 1100 bash tools/gpu_mesh_ab.sh ;;
    configs) run ${TAG}_configs 600 python3 tools/bench_configs.py --configs ${CONFIGS:-C4,C5} --spp-scale 0.0625 ;;
    bench) run ${TAG}_bench 300 python3 bench.py --steps 20 --warmup 5 ;;
  esac
done
echo ALL_OK
