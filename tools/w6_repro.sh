#!/bin/bash
# The 6-wave mis-render of round 4 (rt_fast_body.h RT_FAST_FAMILY): render a 4-bunny frame
# at 6 waves per SIMD through the production family built with round 4's codegen options (variant
# r4codegen: -structurizecfg-skip-uniform-regions with LLVM's redundant-END_CF removal on), built by
#   CODEGEN="-mllvm -structurizecfg-skip-uniform-regions=1" bash tools/build_variant.sh r4codegen
# and through the shipped build, each against the CPU oracle, for RT_TUNE values that switch whole code
# paths off at run time (same machine code, different paths taken):
#   0x100000 twins off, 0x1 no cooperative rounds, 0x4000000 no lone traversal, 0x40000000 per-lane
#   leaf-tree walk instead of coop_tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
LIB=cuda-raytracing_amd/librt_hip.so
cp $LIB gpurun_out/librt_hip.so.orig
restore() { cp gpurun_out/librt_hip.so.orig $LIB; }
TUNES=${TUNES:-"0 0x100000 0x100001 0x4100000 0x40100000"}
for v in ${VARS:-r4codegen current}; do
  [ "$v" = current ] && restore || cp cuda-raytracing_amd/variants/v_$v.so $LIB
  echo "== $v" | tee -a gpurun_out/w6_repro.log
  ORACLE=1 timeout -k 10 ${TIMEOUT:-300} python -u tools/variant_agree.py ${SCENE:-bunny4} ${W:-256} ${H:-144} "$TUNES" "${WPS:-6}" \
    >> gpurun_out/w6_repro.log 2>&1
  rc=$?
  [ $rc = 0 ] || { echo "exit $rc"; restore; tail -20 gpurun_out/w6_repro.log; exit $rc; }
done
restore
cat gpurun_out/w6_repro.log
