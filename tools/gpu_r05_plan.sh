#!/bin/bash
# bench.py's headline frame under other unit sizes (--spu) and stream counts, same box, alternating.
set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r05pl}_plan.log; : > $OUT
for rep in 1 2; do
  for cfg in "--spu 0 --streams 2" "--spu 16 --streams 2" "--spu 32 --streams 2" "--spu 0 --streams 3" "--spu 6 --streams 2"; do
    echo "== rep $rep $cfg" >> $OUT
    timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-spp 0 --no-stats $cfg 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" >> $OUT || exit 1
  done
done
cat $OUT
