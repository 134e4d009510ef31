#!/bin/bash
# Round 3: sweep of the measured lane-plan refinement (bench.refine_lane_map) shard by shard on one
# box: theta, rounds, occupancy (6 = the 6-wave build, 3 / 4 = the 5-wave build capped by LDS) and
# the model plan's parallel units.  COMBOS: "theta:rounds:wps:units ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp SKIP_NO_LANE=1
for c in ${COMBOS:-0.75:3:6:48000 0.85:5:6:48000 0.75:3:4:48000 0.75:5:6:24000 0.65:3:6:48000}; do
  IFS=: read th rd w u <<< "$c"
  timeout -k 10 300 python -u tools/shard_timing.py --config ${CFG:-cfg2} --plans cost --reps 3 --ns ${NS:-8,4} \
      --lanes "$u:1" --wps $w --refine $rd --theta $th > gpurun_out/sweep_$c.log 2>&1
  rc=$?; echo "$c: $(grep '"max_ms"' gpurun_out/sweep_$c.log | python3 -c 'import sys,json; print([(d["n"], d["max_ms"]) for d in map(json.loads, sys.stdin)])' 2>&1 | tail -1)"
  [ $rc = 0 ] || exit $rc
done
