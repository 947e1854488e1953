#!/bin/bash
# One gpurun call: GPU parity tests, then A/B of libyart builds on several scenes.
#   AB_LIBS="lib1 lib2" AB_SCENES="cornell-box:800:800:64 random-scene:1200:800:16" bash tools/gpu_ab2.sh
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO"; mkdir -p gpurun_out
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after rc=$rc"; exit $rc; }
}
if [ "${PYTEST:-1}" = 1 ]; then run pytest 900 python3 -m pytest tests -m gpu -x -q -p no:cacheprovider; fi
for sc in ${AB_SCENES:-cornell-box:800:800:64}; do
  IFS=: read -r name w h spp <<< "$sc"
  run "ab_$name" 900 python3 tools/ab.py yet-another-raytracer_amd/lib/libyart.so ${AB_LIBS:-} --scene "$name" --w "$w" --h "$h" --spp "$spp" --reps 2
done
echo ALL_OK
