#!/bin/bash
# One gpurun call: GPU parity tests and an A/B of variant builds. Each GPU step has its own time
# limit; the script stops at the first failure. (PC sampling is not run on this GPU pool; the
# per-region cycle probe, tools/gpu_cycles.sh, answers where the time goes.)
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out
mkdir -p "$OUT"
cd "$REPO"
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 8 "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after rc=$rc"; exit $rc; }
}
STEPS=${STEPS:-"pytest ab"}
for s in $STEPS; do
  case $s in
    pytest) run pytest 900 python3 -m pytest tests -m gpu -x -q ;;
    ab)     run ab 900 python3 tools/ab.py yet-another-raytracer_amd/lib/libyart.so ${AB_LIBS:-} --spp 64 --reps 2 ;;
  esac
done
echo ALL_OK
