#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench. Every GPU step has its own time limit; a
# fault / abort / timeout ends the script (no further GPU work in that call).
set -u
mkdir -p gpurun_out
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  case $rc in 124|137|134|139|-6|-11) echo "fatal rc=$rc: stopping"; exit $rc;; esac
  return 0
}
STEPS=${STEPS:-"pytest smoke bench"}
for s in $STEPS; do
  case $s in
    pytest) run pytest 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
    smoke)  run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py --steps 3 --warmup 1 ;;
  esac
done
