set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
L=yet-another-raytracer_amd/lib
LIBS="$L/libyart.so $L/variants/libyart_wstep1.so" TAG=r05ws REPS=4 SCENES="random-scene 1200 800 16;random-scene 600 400 64" bash tools/gpu_ab.sh || exit 1
STEPS="prof_david prof_c4 prof_c5" bash tools/gpu_round_end.sh
