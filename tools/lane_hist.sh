#!/bin/bash
# Diagnostic variant: the timing family built with -DRT_LANE_HIST (rt_fast.h) -> cuda-raytracing_amd/variants/v_lanehist.so.
# Its timing frames report wave cycles of small-step iterations with 1-4 / 5-16 active lanes
# (stats tree_nodes / tree_tri_tests), of all small-step iterations (cycles_tree_clusters) and of the
# lone-lane traversals (cycles_tree_tris).  Run: tools/lane_hist.py on the GPU box.
# LIVE=1: instead -DRT_LIVE_HIST -> v_livehist.so: segment-loop wave cycles by live pixels of the wave
# (1-8 / 9-16 / 17-32 / all in tree_nodes / tree_tri_tests / cycles_tree_clusters / cycles_tree_tris);
# run tools/live_hist.py.
set -e
cd "$(dirname "$0")/.."
B=cuda-raytracing_amd/build; V=cuda-raytracing_amd/variants
mkdir -p "$V" /tmp/rtvar
if [ -n "${LIVE:-}" ]; then DEF=-DRT_LIVE_HIST=1; OUT="$V/v_livehist.so"; else DEF=-DRT_LANE_HIST=1; OUT="$V/v_lanehist.so"; fi
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -fno-slp-vectorize -mllvm -structurizecfg-skip-uniform-regions=1 -mllvm -amdgpu-remove-redundant-endcf=0 \
  $DEF -I include -I cuda-raytracing_amd/csrc -c cuda-raytracing_amd/csrc/rt_fast_timing.hip -o /tmp/rtvar/timing_hist.o
objs=""
for o in $B/*.o; do
  case "$o" in *rt_fast_timing.hip.o) objs="$objs /tmp/rtvar/timing_hist.o";; *) objs="$objs $o";; esac
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs -L/opt/rocm/lib -lrccl -o "$OUT"
echo "built $OUT"
