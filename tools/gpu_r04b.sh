#!/bin/bash
# r04 check-and-A/B call: the GPU suite at the working tree, then the working tree's library against
# lib/variants (VARS) on the BASELINE frames (tools/gpu_mesh_ab.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r04b}_gpu_tests.log 2>&1
rc=$?; tail -6 gpurun_out/${TAG:-r04b}_gpu_tests.log
grep -E "FAILED|ERROR" gpurun_out/${TAG:-r04b}_gpu_tests.log | head -20
if [ $rc -ne 0 ] && [ -z "${AB_ANYWAY:-}" ]; then exit $rc; fi
VARS="${VARS:-head}" SCENES="${SCENES:-cornell-box 800 800 64;random-scene 1200 800 16;bunny 800 800 32;david 1920 1080 16}" bash tools/gpu_mesh_ab.sh
if [ -n "${COPLANAR:-}" ]; then
  timeout -k 10 300 python3 -u tools/coplanar_debug.py david 120 > gpurun_out/${TAG:-r04b}_coplanar.log 2>&1; cat gpurun_out/${TAG:-r04b}_coplanar.log
fi
