set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_boundary.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "multi" > gpurun_out/r05_multi_tests.log 2>&1 || { echo MULTI_FAIL; tail -30 gpurun_out/r05_multi_tests.log; exit 1; }
tail -1 gpurun_out/r05_multi_tests.log
L=yet-another-raytracer_amd/lib
LIBS="$L/libyart.so $L/variants/libyart_wstep1.so" TAG=r05ws REPS=4 SCENES="random-scene 1200 800 16;random-scene 600 400 64" bash tools/gpu_ab.sh || exit 1
bash tools/gpu_r05_plan.sh || exit 1
STEPS="prof_david prof_c4 prof_c5" bash tools/gpu_round_end.sh
