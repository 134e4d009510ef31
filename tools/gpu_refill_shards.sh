#!/bin/bash
# Round 3: a pull queue on a strong-scaled shard -- refill_lanes (a wave takes the next entries of the
# lane order once that many of its lanes are done) with the resident grid capped (waves_per_simd 2-4:
# the rest of the order is the queue), shard by shard at N = 8 (tools/shard_timing.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for c in ${COMBOS:-6:0 6:16 4:16 2:16 2:32 1:32}; do
  IFS=: read w rf <<< "$c"
  timeout -k 10 300 python -u tools/shard_timing.py --config cfg2 --plans cost --reps 3 --ns ${NS:-8} --lanes "48000:1" \
      --wps $w --refill $rf > gpurun_out/refill_$c.log 2>&1
  rc=$?; echo "wps:refill $c: $(grep '"max_ms"' gpurun_out/refill_$c.log | python3 -c 'import sys,json; print([(d["n"], "lanes" if d["lane"] else "plain", d["max_ms"]) for d in map(json.loads, sys.stdin)])' 2>&1 | tail -1)"
  [ $rc = 0 ] || exit $rc
done
