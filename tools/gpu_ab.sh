#!/bin/bash
# A/B timing of the render kernel under bench.py --tune variants (bench only, no tests).
# usage: AB="0 1 2 3" bash tools/gpu_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in ${AB:-0}; do
  timeout -k 10 240 python bench.py --tune $t --no-pmc --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$t.log 2>&1
  rc=$?; echo "tune $t exit $rc: $(tail -1 gpurun_out/ab_$t.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])' 2>&1)"
  case $rc in 0) ;; *) exit $rc;; esac
done
