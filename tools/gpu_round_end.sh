#!/bin/bash
# Round evidence at HEAD (one gpurun call; every GPU step under its own time limit, the script
# stops at the first failure):
#   pytest   the -m gpu suite
#   smoke    __graft_entry__.smoke()
#   bench    bench.py with the driver's arguments
#   prof_cornell  rocprofv3 trace + FETCH / WRITE / VALU / mix passes over bench.py (cornell, C2)
#   prof_cornell_s1  the trace pass over bench.py --streams 1 (one frame in flight: the kernel's
#            duration with no second stream's frame overlapping it)
#   prof_cornell_more  stall / memory-instruction passes over bench.py (not in the default steps)
#   prof_c4 / prof_c5  trace + FETCH / WRITE passes over the C4 / C5 frames tools/bench_configs.py
#            times at --spp-scale 0.0625 (bunny 800x800x32, david 1920x1080x64)
#   rehearse bench.py's per-rank N = 2 path on one GPU (both ranks on device 0, gloo gather)
#   configs  tools/bench_configs.py over every BASELINE config; with PMC summaries of the C4 / C5
#            frames present in profiles/ (tools/summarize_profiles.py), the counter HBM bytes too
#   configs_full  every BASELINE config at its full spp (no work counters)
# Raw outputs under gpurun_out/; tools/summarize_profiles.py turns them into profiles/ files.
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$REPO/gpurun_out; mkdir -p "$OUT"; cd "$REPO"
TAG=${TAG:-r06}
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-4} "$OUT/$name.log"
  [ $rc -eq 0 ] || { echo "stopping after rc=$rc"; exit $rc; }
}
STEPS=${STEPS:-"pytest smoke bench prof_cornell prof_cornell_s1 prof_david prof_c4 prof_c5 configs"}
for s in $STEPS; do
  case $s in
    pytest) run ${TAG}_gpu_tests 900 python3 -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    pytest_k) run ${TAG}_gpu_tests_k 600 python3 -u -m pytest tests -m gpu -k "$PYTEST_K" -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    ab) run ${TAG}_ab 1200 bash tools/gpu_mesh_ab.sh ;;
    probe) run ${TAG}_ovf_probe 300 python3 tools/ovf_probe.py ;;
    lanes) run ${TAG}_lane_phases 300 python3 tools/lane_phases.py david 960 540 16 bunny 800 800 16 cornell-box 800 800 16 random-scene 600 400 16 ;;
    bench_s3) run ${TAG}_bench_cornell_s3 600 python3 bench.py --steps 20 --warmup 5 --streams 3 --cpu-spp 0 --david-spp 0 ;;
    configs_ext) run ${TAG}_bench_configs_ext 600 python3 tools/bench_configs.py --configs E1,E2,E3,E4,E5 ;;
    smoke) run ${TAG}_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run ${TAG}_bench_cornell 600 python3 bench.py --steps 20 --warmup 5 ;;
    prof_cornell) PASSES="trace fetch write valu mix" bash tools/profile.sh || exit 1 ;;
    prof_cornell_s1) PFX=cornell_s1_ BENCH_ARGS="--steps 3 --warmup 1 --cpu-spp 0 --no-stats --streams 1 --david-spp 0" PASSES="trace" bash tools/profile.sh || exit 1 ;;
    prof_cornell_more) PFX=cornell_ PASSES="stall mem" bash tools/profile.sh || exit 1 ;;
    prof_david) PFX=david_ PROG="tools/render_once.py david 960 540 16 2" PASSES="trace fetch write valu mix" bash tools/profile.sh || exit 1 ;;
    prof_c4) PFX=c4_ PROG="tools/render_once.py bunny 800 800 32 1" PASSES="trace fetch write" bash tools/profile.sh || exit 1 ;;
    prof_c5) PFX=c5_ PROG="tools/render_once.py david 1920 1080 64 1" PASSES="trace fetch write" bash tools/profile.sh || exit 1 ;;
    rehearse) run ${TAG}_rehearse_n2 300 env YART_BENCH_SAME_DEVICE=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-spp 0 ;;
    configs)
      PM=""
      [ -f profiles/${TAG}_c4_pmc.json ] && PM="$PM --pmc C4=profiles/${TAG}_c4_pmc.json"
      [ -f profiles/${TAG}_c5_pmc.json ] && PM="$PM --pmc C5=profiles/${TAG}_c5_pmc.json"
      run ${TAG}_bench_configs 900 python3 tools/bench_configs.py --spp-scale 0.0625 $PM ;;
    configs_full) run ${TAG}_bench_configs_full 600 python3 tools/bench_configs.py --spp-scale 1.0 --no-stats ;;
  esac
done
echo ALL_OK
