#!/bin/bash
# r05 shared-pool steal-threshold sweep (one gpurun call): drain probe per library, then A/B.
set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
T=${TAG:-r05s}
L=yet-another-raytracer_amd/lib
LIBS="$L/variants/libyart_head.so $L/libyart.so ${EXTRA:-$L/variants/libyart_steal17.so $L/variants/libyart_steal12.so $L/variants/libyart_steal4.so}"
for lib in $LIBS; do
  echo "== $lib" >> gpurun_out/${T}_drain.log
  YART_DEVICE_LIB=$lib timeout -k 10 300 python3 tools/drain_probe.py david 960 540 16 >> gpurun_out/${T}_drain.log 2>&1 || { echo DRAIN_FAIL $lib; tail gpurun_out/${T}_drain.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/${T}_drain.log
for sc in ${SCENES:-"david 960 540 16" "bunny 800 800 32" "david 1920 1080 16"}; do :; done
IFS=';' read -ra list <<< "${SCENES:-david 960 540 16;bunny 800 800 32;david 1920 1080 16}"
for sc in "${list[@]}"; do
  set -- $sc
  timeout -k 10 900 python3 tools/ab.py $LIBS --scene $1 --w $2 --h $3 --spp $4 --reps 3 > gpurun_out/${T}_ab_$1_$2.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/${T}_ab_$1_$2.log; exit 1; }
  grep '"lib"' gpurun_out/${T}_ab_$1_$2.log
done
echo ALL_OK
