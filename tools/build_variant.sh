#!/bin/bash
# Build a librt_hip.so variant with extra compile definitions for the production family only:
#   bash tools/build_variant.sh NAME "-DFOO=1"  ->  cuda-raytracing_amd/variants/v_NAME.so
# (the other product objects are the current build's; A/B with VARS="current NAME" bash tools/gpu_ab.sh)
# CODEGEN="..." replaces build.py's codegen options for this unit, e.g. round 4's set, which miscompiled
# the 6-wave leaf-tree kernel (tools/w6_repro.sh):  CODEGEN="-mllvm -structurizecfg-skip-uniform-regions=1"
set -e
cd "$(dirname "$0")/.."
name="$1"; shift
B=cuda-raytracing_amd/build; V=cuda-raytracing_amd/variants
mkdir -p "$V" /tmp/rtvar
CODEGEN=${CODEGEN:-"-mllvm -structurizecfg-skip-uniform-regions=1 -mllvm -amdgpu-remove-redundant-endcf=0"}
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -fno-slp-vectorize $CODEGEN "$@" \
  -I include -I cuda-raytracing_amd/csrc -c cuda-raytracing_amd/csrc/rt_fast_prod.hip -o /tmp/rtvar/prod_$name.o
objs=""
for o in $B/*.o; do
  case "$o" in
    *rt_fast_prod.hip.o) objs="$objs /tmp/rtvar/prod_$name.o";;
    *rt_fast_ab*|*rt_fast_refill*|*rt_fast_screen*|*rt_lone*|*rt_wavefront*|*rt_exp*) ;;  # the plugin's (librt_hip_exp.so)
    *) objs="$objs $o";;
  esac
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs -L/opt/rocm/lib -lrccl -o "$V/v_$name.so"
echo "built $V/v_$name.so"
