set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r05_head_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r05_head_tests.log; exit 1; }
tail -2 gpurun_out/r05_head_tests.log
timeout -k 10 600 python3 -u tools/walk_ref_ab.py --full --reps 3 > gpurun_out/r05_walk_ref_ab.log 2>&1 || { echo AB_FAIL; tail -30 gpurun_out/r05_walk_ref_ab.log; exit 1; }
cat gpurun_out/r05_walk_ref_ab.log
for f in "david 1920 1080 4" "david 960 540 16" "bunny 800 800 16"; do
  YART_DEVICE_LIB=yet-another-raytracer_amd/lib/variants/libyart_drain.so timeout -k 10 300 python3 tools/drain_probe.py $f >> gpurun_out/r05_drain_head.log 2>&1 || exit 1
done
cat gpurun_out/r05_drain_head.log
