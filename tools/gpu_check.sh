#!/bin/bash
# One gpurun call: GPU parity tests, smoke, bench. Every GPU step has its own time limit; a
# fault / abort / timeout ends the script (no further GPU work in that call).
set -u
mkdir -p gpurun_out
run() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  case $rc in 124|137|134|139|-6|-11) echo "fatal rc=$rc: stopping"; exit $rc;; esac
  return 0
}
STEPS=${STEPS:-"pytest smoke bench"}
for s in $STEPS; do
  case $s in
    pytest) run pytest 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 150 --timeout-method thread ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} ;;
    smoke)  run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py --steps 20 --warmup 5 ;;
    rehearse) YART_BENCH_SAME_DEVICE=1 run rehearse 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 2 --warmup 1 --no-stats --cpu-spp 0 ;;
    configs) run configs 600 python tools/bench_configs.py --spp-scale ${SPP_SCALE:-0.125} ${CONFIG_ARGS:-} ;;
    configs_ref) YART_OPTIONS=mesh_walk_ref=1 run configs_ref 600 python tools/bench_configs.py --spp-scale ${SPP_SCALE:-0.125} ${CONFIG_ARGS:-} ;;
    configs_mega) YART_OPTIONS=mesh_wavefront=0 run configs_mega 600 python tools/bench_configs.py --spp-scale ${SPP_SCALE:-0.125} ${CONFIG_ARGS:-} ;;
  esac
done
