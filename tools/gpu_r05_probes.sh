set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
timeout -k 10 300 python3 tools/world_probe.py random-scene 1200 800 8 > gpurun_out/r05_world_probe.log 2>&1 || { cat gpurun_out/r05_world_probe.log; exit 1; }
timeout -k 10 300 python3 tools/world_probe.py random-scene 600 400 32 >> gpurun_out/r05_world_probe.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r05_world_probe.log
for f in "david 1920 1080 4" "david 960 540 16" "bunny 800 800 16"; do
  timeout -k 10 300 python3 tools/drain_probe.py $f >> gpurun_out/r05_drain_kept.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r05_drain_kept.log
L=yet-another-raytracer_amd/lib
timeout -k 10 900 python3 tools/ab.py $L/libyart.so $L/variants/libyart_ka.so --scene cornell-box --w 800 --h 800 --spp 256 --reps 5 > gpurun_out/r05_ab_ka256.log 2>&1 || exit 1
grep '"lib"' gpurun_out/r05_ab_ka256.log
