#!/bin/bash
# Diagnostic variant: the timing family built with -DRT_LANE_HIST (rt_fast.h) -> cuda-raytracing_amd/variants/v_lanehist.so.
# Its timing frames report wave cycles of small-step iterations with 1-4 / 5-16 active lanes
# (stats tree_nodes / tree_tri_tests), of all small-step iterations (cycles_tree_clusters) and of the
# lone-lane traversals (cycles_tree_tris).  Run: tools/lane_hist.py on the GPU box.
set -e
cd "$(dirname "$0")/.."
B=cuda-raytracing_amd/build; V=cuda-raytracing_amd/variants
mkdir -p "$V" /tmp/rtvar
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -fno-slp-vectorize -mllvm -structurizecfg-skip-uniform-regions=1 -mllvm -amdgpu-remove-redundant-endcf=0 \
  -DRT_LANE_HIST=1 -I include -I cuda-raytracing_amd/csrc -c cuda-raytracing_amd/csrc/rt_fast_timing.hip -o /tmp/rtvar/timing_hist.o
objs=""
for o in $B/*.o; do
  case "$o" in *rt_fast_timing.hip.o) objs="$objs /tmp/rtvar/timing_hist.o";; *) objs="$objs $o";; esac
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs -L/opt/rocm/lib -lrccl -o "$V/v_lanehist.so"
echo "built $V/v_lanehist.so"
