#!/bin/bash
# Generic same-box A/B (one gpurun call): optional GPU test suite on the tree's library, then
# tools/ab.py over LIBS on each scene of SCENES ("name w h spp;...").
set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
T=${TAG:-ab}
L=yet-another-raytracer_amd/lib
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_tests.log; exit 1; }
  tail -1 gpurun_out/${T}_tests.log
fi
IFS=';' read -ra list <<< "${SCENES:-cornell-box 800 800 64;random-scene 1200 800 16;david 960 540 16;bunny 800 800 32}"
for sc in "${list[@]}"; do
  set -- $sc
  timeout -k 10 900 python3 tools/ab.py $LIBS --scene $1 --w $2 --h $3 --spp $4 --reps ${REPS:-3} > gpurun_out/${T}_ab_$1.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/${T}_ab_$1.log; exit 1; }
  grep '"lib"' gpurun_out/${T}_ab_$1.log
done
echo ALL_OK
