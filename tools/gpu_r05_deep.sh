#!/bin/bash
# r05: GPU suite, the deep-mesh megakernel vs wavefront A/B, and same-box A/Bs against the round start.
set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
T=${TAG:-r05d}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 600 python3 tools/deep_ab.py 320 320 16 3 > gpurun_out/${T}_deep_ab.log 2>&1 || { echo DEEP_FAIL; tail -20 gpurun_out/${T}_deep_ab.log; exit 1; }
grep '^{' gpurun_out/${T}_deep_ab.log
L=yet-another-raytracer_amd/lib
LIBS="$L/variants/libyart_head.so $L/libyart.so $L/variants/libyart_tri64.so" TAG=${T}m REPS=3 SCENES="david 960 540 16;bunny 800 800 32;david 1920 1080 16" bash tools/gpu_ab.sh || exit 1
LIBS="$L/variants/libyart_head.so $L/libyart.so" TAG=${T}w REPS=4 SCENES="random-scene 1200 800 16;random-scene 1200 800 64;cornell-box 800 800 64" bash tools/gpu_ab.sh
