set -u
cd $GRAFT_REPO_ROOT
for spu in 0 4 6; do
  PFX=spu${spu}_ PASSES="write" BENCH_ARGS="--steps 3 --warmup 1 --cpu-spp 0 --no-stats --spu $spu" bash tools/profile.sh || exit 1
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-spp 0 --no-stats --spu $spu > gpurun_out/spu${spu}_bench.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*' gpurun_out/spu${spu}_bench.log
done
