set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
L=yet-another-raytracer_amd/lib
for rep in 1 2; do
  timeout -k 10 600 python3 tools/ab.py $L/libyart.so --scene cornell-box --w 800 --h 800 --spp 64 --reps 2 | grep '"lib"' | sed 's/^/default: /'
  YART_OPTIONS=world_bvh=1 timeout -k 10 600 python3 tools/ab.py $L/libyart.so --scene cornell-box --w 800 --h 800 --spp 64 --reps 2 | grep '"lib"' | sed 's/^/world_bvh=1: /'
done
