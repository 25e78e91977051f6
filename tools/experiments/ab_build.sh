#!/usr/bin/env bash
# Build a variant of the library for same-box A/B runs (tools/experiments/ab.sh): objects and .so under
# _var/ab/<name>/ (git-ignored, but it travels to the GPU box).
#   tools/experiments/ab_build.sh <name> "<-DFLAG=value ...>"
set -eu
cd "$(dirname "$0")/../../icp-4dradar_amd"
NAME=$1; FLAGS=${2:-}
OUT=../_var/ab/$NAME
mkdir -p "$OUT"
make -j8 OUT="$OUT" EXTRA="$FLAGS" "$OUT/libicp4r.so" > "$OUT/build.txt" 2>&1 || { tail -20 "$OUT/build.txt"; exit 1; }
echo "_var/ab/$NAME/libicp4r.so"
