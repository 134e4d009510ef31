#!/bin/bash
# Round 3: lane-plan refinement A/B on one box -- shard by shard (tools/shard_timing.py, frames 1-2
# after a warm-up frame), the model's lane plan alone vs + bench.refine_lane_map (3 rounds), N = 8 / 4 / 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp SKIP_NO_LANE=1
for rf in ${REFINES:-0 3}; do
  timeout -k 10 500 python -u tools/shard_timing.py --config ${CFG:-cfg2} --plans cost --reps ${REPS:-3} --ns ${NS:-8,4,2} \
      --lanes "48000:1" --wps ${WPS:-6} --refine $rf --theta ${THETA:-0.75} > gpurun_out/r03e_refine${rf}_shards.log 2>&1
  rc=$?; echo "refine $rf:"; grep -E '"max_ms"' gpurun_out/r03e_refine${rf}_shards.log | grep -v '"lane": null' | cut -c1-200
  [ $rc = 0 ] || exit $rc
done
