#!/bin/bash
# One gpurun call for a round's evidence at HEAD: the -m gpu suite, bench.py (the driver's
# command), rocprofv3 passes over bench.py (cornell) and over a david frame, and the other
# BASELINE configs. Every GPU step has its own time limit; the script stops at the first failure.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$REPO/gpurun_out; mkdir -p "$OUT"; cd "$REPO"
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-4} "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after rc=$rc"; exit $rc; }
}
TAG=${TAG:-round}
STEPS=${STEPS:-"pytest bench prof_cornell prof_david configs"}
for s in $STEPS; do
  case $s in
    pytest) run ${TAG}_gpu_tests 900 python3 -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bench) run ${TAG}_bench_cornell 600 python3 bench.py --steps 20 --warmup 5 ;;
    prof_cornell) PASSES="trace fetch write valu" bash tools/profile.sh || exit 1 ;;
    prof_david) PFX=david_ PROG="tools/render_once.py david 960 540 16" PASSES="trace fetch write valu" bash tools/profile.sh || exit 1 ;;
    configs) run ${TAG}_bench_configs 900 python3 tools/bench_configs.py --spp-scale 0.0625 ;;
  esac
done
echo ALL_OK
