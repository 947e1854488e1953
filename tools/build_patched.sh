#!/bin/bash
# Build libyart.so of the working tree with a python patch applied to kernels.hip into
# lib/variants/libyart_<name>.so, for same-box A/B runs (tools/gpu_mesh_ab.sh VARS=<name>):
#   tools/build_patched.sh <name> <patch.py>   (patch.py rewrites the file given as argv[1] in place)
set -eu
REPO=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; PATCH=$2
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
tar -C "$REPO" -cf - Makefile include yet-another-raytracer_amd/csrc yet-another-raytracer_amd/host tables tools/gen_tables_inc.py yet-another-raytracer_amd/yart/buildid.py | tar -x -C "$TMP"
python3 "$PATCH" "$TMP/yet-another-raytracer_amd/csrc/kernels.hip"
make -C "$TMP" -j8 device > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
mkdir -p "$REPO/yet-another-raytracer_amd/lib/variants"
cp "$TMP/yet-another-raytracer_amd/lib/libyart.so" "$REPO/yet-another-raytracer_amd/lib/variants/libyart_$NAME.so"
echo "built working tree + $PATCH -> lib/variants/libyart_$NAME.so"
