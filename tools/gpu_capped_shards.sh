#!/bin/bash
# Round 3: shard-by-shard timing (tools/shard_timing.py, cost plan + lane plan) with the render
# kernel's residency capped by dynamic LDS (rt_render_params.waves_per_simd 1-4) against the
# uncapped 5- and 6-wave builds.  The question: does a strong-scaled shard (N = 4 / 8) finish
# sooner when its latency-bound long waves share their SIMD with fewer co-resident waves?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WPS_LIST:-6 4 3 2}; do
  timeout -k 10 300 python -u tools/shard_timing.py --config ${CFG:-cfg2} --plans cost --reps 2 --ns ${NS:-8,4} \
      --lanes "${LANES:-48000:1}" --wps $w > gpurun_out/capped_w$w.log 2>&1
  rc=$?
  echo "wps $w exit $rc: $(grep '"max_ms"' gpurun_out/capped_w$w.log | python3 -c 'import sys,json; print([(d["n"], d["max_ms"]) for d in map(json.loads, sys.stdin)])' 2>&1 | tail -1)"
  case $rc in 0) ;; *) exit $rc;; esac
done
