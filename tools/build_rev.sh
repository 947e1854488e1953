#!/bin/bash
# Build libyart.so of a git revision into lib/variants/libyart_<name>.so, for A/B runs against the
# working tree (tools/ab.py, tools/gpu_spill_ab.sh): tools/build_rev.sh <rev> <name>
set -eu
REPO=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
git -C "$REPO" archive "$REV" Makefile include yet-another-raytracer_amd/csrc yet-another-raytracer_amd/host tables tools/gen_tables_inc.py $(git -C "$REPO" cat-file -e "$REV":yet-another-raytracer_amd/yart/buildid.py 2>/dev/null && echo yet-another-raytracer_amd/yart/buildid.py) | tar -x -C "$TMP"
make -C "$TMP" -j8 device > "$TMP/build.log" 2>&1 || { tail -20 "$TMP/build.log"; exit 1; }
mkdir -p "$REPO/yet-another-raytracer_amd/lib/variants"
cp "$TMP/yet-another-raytracer_amd/lib/libyart.so" "$REPO/yet-another-raytracer_amd/lib/variants/libyart_$NAME.so"
echo "built $REV -> lib/variants/libyart_$NAME.so"
