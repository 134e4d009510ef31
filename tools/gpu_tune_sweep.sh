#!/bin/bash
# Production-kernel RT_TUNE sweep (values in TUNES, REPS interleaved rounds), config CFG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for t in ${TUNES:-0}; do
    timeout -k 10 200 python bench.py --config ${CFG:-cfg2} --tune $t --no-pmc --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS} > gpurun_out/ts_$t.log 2>&1
    rc=$?
    echo "rep $rep tune $t exit $rc: $(tail -1 gpurun_out/ts_$t.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])' 2>&1 | tail -1)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
