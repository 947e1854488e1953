# r05: fma-slab world walk (child boxes pre-grown) and NaN-axis box cull: parity on each variant, then A/B
set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
L=yet-another-raytracer_amd/lib
YART_DEVICE_LIB=$L/variants/libyart_wfma.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_full_size_parity.py -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread -k "world_bvh or random or C3" > gpurun_out/r05wf_tests_wfma.log 2>&1 || { echo WFMA_FAIL; tail -30 gpurun_out/r05wf_tests_wfma.log; exit 1; }
tail -1 gpurun_out/r05wf_tests_wfma.log
YART_DEVICE_LIB=$L/variants/libyart_boxnan.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_full_size_parity.py -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread -k "cornell or box or C2" > gpurun_out/r05wf_tests_boxnan.log 2>&1 || { echo BOXNAN_FAIL; tail -30 gpurun_out/r05wf_tests_boxnan.log; exit 1; }
tail -1 gpurun_out/r05wf_tests_boxnan.log
LIBS="$L/libyart.so $L/variants/libyart_wfma.so" TAG=r05wf REPS=4 SCENES="random-scene 1200 800 16;random-scene 600 400 64" bash tools/gpu_ab.sh && \
LIBS="$L/libyart.so $L/variants/libyart_boxnan.so" TAG=r05bn REPS=4 SCENES="cornell-box 800 800 64" bash tools/gpu_ab.sh
