#!/bin/bash
# One gpurun call: GPU parity tests, A/B of variant builds, and a host-trap PC-sampling profile
# of the render kernel (the -g build, so samples map to source lines). Each GPU step has its own
# time limit; the script stops at the first failure.
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
STEPS=${STEPS:-"pytest ab pcsamp"}
for s in $STEPS; do
  case $s in
    pytest) run pytest 900 python3 -m pytest tests -m gpu -x -q ;;
    ab)     run ab 900 python3 tools/ab.py yet-another-raytracer_amd/lib/libyart.so ${AB_LIBS:-} --spp 64 --reps 2 ;;
    pcsamp)
      cd /tmp && export TMPDIR=/tmp
      YART_DEVICE_LIB=$REPO/yet-another-raytracer_amd/lib/variants/libyart_g.so \
        run pcsamp 600 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
        --pc-sampling-unit time --pc-sampling-interval ${PCS_INTERVAL:-1} --output-format csv \
        -d "$OUT/pcsamp" -o run -- python3 "$REPO/bench.py" --steps 1 --warmup 0 --cpu-spp 0 --no-stats
      cd "$REPO" ;;
  esac
done
echo ALL_OK
