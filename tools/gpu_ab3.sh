#!/bin/bash
# One gpurun call: (optional) GPU parity tests, then A/B of libyart builds on several scenes, with
# per-scene env overrides. AB_LIBS="lib1 lib2" AB_SCENES="cornell-box:800:800:64" bash tools/gpu_ab3.sh
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$REPO"; mkdir -p gpurun_out
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-8} "gpurun_out/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after rc=$rc"; exit $rc; }
}
if [ "${PYTEST:-1}" = 1 ]; then
  run pytest 900 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
fi
for sc in ${AB_SCENES:-cornell-box:800:800:64}; do
  IFS=: read -r name w h spp <<< "$sc"
  run "ab_$name" 900 python3 tools/ab.py yet-another-raytracer_amd/lib/libyart.so ${AB_LIBS:-} --scene "$name" --w "$w" --h "$h" --spp "$spp" --reps ${REPS:-3}
done
echo ALL_OK
