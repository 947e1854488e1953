#!/bin/bash
# SAH parameter sweep for the world BVH on C3 (YART_WORLD_SAH=node_cost,max_leaf).
set -u
REPO=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$REPO/gpurun_out; mkdir -p "$OUT"; cd "$REPO"
for v in ${SWEEP:-0.3,2 0.7,2 0.7,4 1.2,4 0.7,8 1.5,8}; do
  YART_WORLD_SAH=$v timeout -k 10 300 python tools/bench_configs.py --configs C3 --spp-scale 0.0625 > "$OUT/sweep_$v.log" 2>&1 || { echo "fail $v"; exit 1; }
  echo "$v $(grep -o '"kernel_ms": [0-9.]*, "wall_s": [0-9.]*, "Msamples_per_s": [0-9.]*' "$OUT/sweep_$v.log") $(grep -o '"prim_tests": [0-9]*, "node_visits": [0-9]*' "$OUT/sweep_$v.log")"
done
