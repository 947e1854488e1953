#!/bin/bash
# units_per_wave A/B (tools/plan_sweep.py): the library's auto plan (u0) against the r05k plan's
# 64 units per wave (u64) over the BASELINE frames at full and 1/16 spp; one gpurun call.
set -u
U=${U:-u0,u64}
timeout -k 10 100 python3 tools/plan_sweep.py bunny 800 800 512 $U 3 > gpurun_out/upw_c4.log 2>&1 &&
timeout -k 10 100 python3 tools/plan_sweep.py random-scene 1200 800 500 $U 3 > gpurun_out/upw_c3.log 2>&1 &&
timeout -k 10 100 python3 tools/plan_sweep.py bunny 800 800 32 $U 5 > gpurun_out/upw_c4_32.log 2>&1 &&
timeout -k 10 100 python3 tools/plan_sweep.py david 1920 1080 64 $U 3 > gpurun_out/upw_c5_64.log 2>&1 &&
timeout -k 10 100 python3 tools/plan_sweep.py random-scene 1200 800 31 $U 5 > gpurun_out/upw_c3_31.log 2>&1 &&
timeout -k 10 100 python3 tools/plan_sweep.py cornell-box 800 800 256 $U 3 > gpurun_out/upw_c2.log 2>&1 &&
timeout -k 10 150 python3 tools/plan_sweep.py david 1920 1080 1024 $U 2 0/8 > gpurun_out/upw_c5s.log 2>&1 &&
timeout -k 10 200 python3 tools/plan_sweep.py david 1920 1080 1024 $U 1 > gpurun_out/upw_c5.log 2>&1
rc=$?; grep -h best gpurun_out/upw_*.log; exit $rc
