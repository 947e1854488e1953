#!/bin/bash
# r05 shared-pool check (one gpurun call): a small mesh render first (a hang ends it early), the
# GPU parity suite, drain probe, then the A/B against the round's start (lib/variants/libyart_head.so).
set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
T=${TAG:-r05p}
timeout -k 10 120 python3 tools/render_once.py david 64 64 2 1 > gpurun_out/${T}_tiny.log 2>&1 || { echo TINY_FAIL; cat gpurun_out/${T}_tiny.log; exit 1; }
cat gpurun_out/${T}_tiny.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for f in "david 1920 1080 4" "david 960 540 16" "bunny 800 800 16"; do
  timeout -k 10 300 python3 tools/drain_probe.py $f >> gpurun_out/${T}_drain.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/${T}_drain.log
L=yet-another-raytracer_amd/lib
for sc in "bunny 800 800 32" "david 1920 1080 16" "david 1920 1080 64"; do
  set -- $sc
  timeout -k 10 600 python3 tools/ab.py $L/variants/libyart_head.so $L/libyart.so --scene $1 --w $2 --h $3 --spp $4 --reps 3 > gpurun_out/${T}_ab_$1_$4.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/${T}_ab_$1_$4.log; exit 1; }
  grep '"lib"' gpurun_out/${T}_ab_$1_$4.log
done
echo ALL_OK
