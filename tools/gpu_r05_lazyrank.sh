set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
L=yet-another-raytracer_amd/lib
LIBS="$L/libyart.so $L/variants/libyart_lazyrank.so" TAG=r05lr REPS=3 SCENES="david 960 540 16;bunny 800 800 32;david 1920 1080 16" bash tools/gpu_ab.sh || exit 1
LIBS="$L/libyart.so $L/variants/libyart_rngpeel.so" TAG=r05rp REPS=4 SCENES="cornell-box 800 800 64;random-scene 1200 800 16" bash tools/gpu_ab.sh || exit 1
LIBS="$L/variants/libyart_head.so $L/libyart.so" TAG=r05rs REPS=4 SCENES="random-scene 1200 800 16;random-scene 1200 800 64" bash tools/gpu_ab.sh || exit 1
STEPS="rehearse" bash tools/gpu_round_end.sh
