#!/bin/bash
# Same-box A/B of prebuilt librt_hip.so variants on the shard-by-shard strong-scaling timing.
# usage: VARS="e0.45 e0.6" NS="4,8" LANES="48000:1.0" bash tools/gpu_variants_shards.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
cp cuda-raytracing_amd/librt_hip.so cuda-raytracing_amd/variants/current.so.bak
for v in current ${VARS}; do
  if [ "$v" = current ]; then cp cuda-raytracing_amd/variants/current.so.bak cuda-raytracing_amd/librt_hip.so; else cp "cuda-raytracing_amd/variants/v_$v.so" cuda-raytracing_amd/librt_hip.so; fi
  timeout -k 10 300 python tools/shard_timing.py --config ${CFG:-cfg2} --plans cost --reps 3 --ns ${NS:-4,8} --lanes "${LANES:-48000:1.0}" > gpurun_out/vs_$v.log 2>&1
  rc=$?
  echo "$v exit $rc: $(grep "lane\": \[" gpurun_out/vs_$v.log | python3 -c "import sys,json; print([(json.loads(l)[\"n\"], json.loads(l)[\"max_ms\"]) for l in sys.stdin])")"
  case $rc in 0) ;; *) cp cuda-raytracing_amd/variants/current.so.bak cuda-raytracing_amd/librt_hip.so; exit $rc;; esac
done
cp cuda-raytracing_amd/variants/current.so.bak cuda-raytracing_amd/librt_hip.so
