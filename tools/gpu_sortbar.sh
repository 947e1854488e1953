#!/bin/bash
# A/B: workgroup-sorted shading vs its barriers alone vs the default (cornell, 64 spp).
L=yet-another-raytracer_amd/lib
mkdir -p gpurun_out
timeout -k 10 500 python3 tools/ab.py $L/libyart.so $L/variants/libyart_sortbar.so $L/variants/libyart_sort.so --scene cornell-box --w 800 --h 800 --spp 64 --reps 3 > gpurun_out/ab_sortbar.log 2>&1; rc=$?; tail -n 3 gpurun_out/ab_sortbar.log; exit $rc
