#!/bin/bash
# Walk-tree evidence (one gpurun call): the bounds-checked walk over the mesh scenes, the -m gpu
# suite, and an A/B of the SAH walk tree against the reference-tree front-to-back walk.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$REPO/gpurun_out; mkdir -p "$OUT"; cd "$REPO"
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-8} "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after rc=$rc"; exit $rc; }
}
export TMPDIR=/tmp
L=yet-another-raytracer_amd/lib
STEPS=${STEPS:-"check pytest ab"}
for s in $STEPS; do
  case $s in
    check) YART_DEVICE_LIB=$L/variants/libyart_walkcheck.so run walk_check 600 python3 tools/walk_check.py ;;
    pytest) run gpu_tests 900 python3 -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    ab)
      for sc in "bunny 800 800 32" "david 1920 1080 16"; do
        set -- $sc
        run ab_walk_$1 600 python3 tools/ab.py $L/libyart.so --scene $1 --w $2 --h $3 --spp $4 --reps 3
        YART_OPTIONS=walk_tree=0 run ab_refwalk_$1 600 python3 tools/ab.py $L/libyart.so --scene $1 --w $2 --h $3 --spp $4 --reps 3
      done ;;
  esac
done
echo ALL_OK
