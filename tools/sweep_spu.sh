mkdir -p gpurun_out
for lib in noremap remap; do for s in 256 64 32 16; do
YART_DEVICE_LIB=yet-another-raytracer_amd/lib/variants/libyart_$lib.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-spp 0 --spu $s --no-stats 2>&1 | grep "^{" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"$lib spu=$s\", d[\"value\"], d[\"ms_per_step\"])"
done; done
