#!/bin/bash
# Sweep samples-per-unit (work-unit size of the chunked path) with bench.py on one GPU.
#   SPUS="8 16 32 64 128" bash tools/sweep_spu.sh
set -u
mkdir -p gpurun_out
for s in ${SPUS:-8 16 32 64 128}; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-spp 0 --spu "$s" --no-stats > gpurun_out/spu_$s.log 2>&1 || { echo "spu=$s failed"; exit 1; }
  grep "^{" gpurun_out/spu_$s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('spu=$s', d['value'], d['ms_per_step'])"
done
