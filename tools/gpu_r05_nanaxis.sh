set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
L=yet-another-raytracer_amd/lib
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread -k "world_bvh or random" > gpurun_out/r05na_tests_main.log 2>&1 || { echo MAIN_FAIL; tail -30 gpurun_out/r05na_tests_main.log; exit 1; }
tail -1 gpurun_out/r05na_tests_main.log
YART_DEVICE_LIB=$L/variants/libyart_nanaxis.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_full_size_parity.py -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread -k "world_bvh or random or C3" > gpurun_out/r05na_tests_var.log 2>&1 || { echo VAR_FAIL; tail -30 gpurun_out/r05na_tests_var.log; exit 1; }
tail -1 gpurun_out/r05na_tests_var.log
LIBS="$L/libyart.so $L/variants/libyart_nanaxis.so" TAG=r05na REPS=4 SCENES="random-scene 1200 800 16;random-scene 600 400 64" bash tools/gpu_ab.sh
