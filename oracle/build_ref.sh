#!/bin/bash
# Builds the pieces of the reference that compile from their own sources here (test
# infrastructure, outputs only into oracle/_ref/, git-ignored):
#   libref_glm.so  -- the reference's vendored glm 0.9.9.8 (header-only) behind oracle/ref_glm.cpp.
# The rest of the reference's path (main_raytracing.cu, Random.cu, Scene.cpp, BVH.cpp) needs
# cuda_runtime.h / curand_kernel.h / assimp / Windows headers that this image lacks; it is not
# built (no stand-ins), see DESIGN.md section 3.
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
ref="${REFERENCE_ROOT:-/root/reference}"
[ -d "$ref/include/glm" ] || { echo "no reference glm at $ref/include/glm: skipped"; exit 0; }
mkdir -p "$here/_ref"
g++ -O2 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -isystem "$ref/include" \
    "$here/ref_glm.cpp" -o "$here/_ref/libref_glm.so.tmp"
mv "$here/_ref/libref_glm.so.tmp" "$here/_ref/libref_glm.so"
echo "built $here/_ref/libref_glm.so"
