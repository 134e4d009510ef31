#!/bin/bash
# Same-box A/B of prebuilt librt_hip.so variants (cuda-raytracing_amd/variants/v_*.so): each is
# copied into place in turn and the bench runs per config.  usage: VARS="old new" CFGS="cfg2" bash tools/gpu_variants.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
cp cuda-raytracing_amd/librt_hip.so cuda-raytracing_amd/variants/current.so.bak
for rep in ${REPS:-1}; do
for v in ${VARS:-old new}; do
  if [ "$v" = new ]; then cp cuda-raytracing_amd/variants/current.so.bak cuda-raytracing_amd/librt_hip.so; else cp "cuda-raytracing_amd/variants/v_$v.so" cuda-raytracing_amd/librt_hip.so; fi
  for c in ${CFGS:-cfg2}; do
    timeout -k 10 240 python bench.py --config $c --no-pmc --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/var_${v}_$c.log 2>&1
    rc=$?
    echo "rep $rep $v $c exit $rc: $(tail -1 gpurun_out/var_${v}_$c.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["plan"].get("occupancy",{}).get("probe_ms"))' 2>&1 | tail -1)"
    case $rc in 0) ;; *) cp cuda-raytracing_amd/variants/current.so.bak cuda-raytracing_amd/librt_hip.so; exit $rc;; esac
  done
done
done
cp cuda-raytracing_amd/variants/current.so.bak cuda-raytracing_amd/librt_hip.so
