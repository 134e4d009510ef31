#!/bin/bash
# Build a librt_hip.so variant with extra compile definitions for the production family only:
#   bash tools/build_variant.sh NAME "-DFOO=1"  ->  cuda-raytracing_amd/variants/v_NAME.so
# (the other objects are the current build's; run tools/gpu_variants.sh VARS="NAME new" to A/B)
set -e
cd "$(dirname "$0")/.."
name="$1"; shift
B=cuda-raytracing_amd/build; V=cuda-raytracing_amd/variants
mkdir -p "$V" /tmp/rtvar
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -fno-slp-vectorize -mllvm -structurizecfg-skip-uniform-regions=1 "$@" \
  -I include -I cuda-raytracing_amd/csrc -c cuda-raytracing_amd/csrc/rt_fast_prod.hip -o /tmp/rtvar/prod_$name.o
objs=""
for o in $B/*.o; do
  case "$o" in *rt_fast_prod.hip.o) objs="$objs /tmp/rtvar/prod_$name.o";; *) objs="$objs $o";; esac
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs -L/opt/rocm/lib -lrccl -o "$V/v_$name.so"
echo "built $V/v_$name.so"
