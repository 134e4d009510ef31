#!/bin/bash
# A/B of rt_render refill_lanes on the bench (usage: CFGS="cfg2" REFILLS="0 16" bash tools/gpu_refill_ab.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for c in ${CFGS:-cfg2}; do
  for r in ${REFILLS:-0 16}; do
    timeout -k 10 240 python bench.py --config $c --refill $r --no-pmc --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/rf_${c}_$r.log 2>&1
    rc=$?
    echo "$c refill=$r exit $rc: $(tail -1 gpurun_out/rf_${c}_$r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["value"], d["roofline"].get("lane_utilization"))' 2>&1 | tail -1)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
