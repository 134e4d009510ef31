#!/bin/bash
# Wavefront tracer knob sweep (RT_TUNE values in TUNES), config CFG (default cfg2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for t in ${TUNES:-0}; do
  timeout -k 10 200 python bench.py --config ${CFG:-cfg2} --tracer wavefront --tune $t --no-pmc --no-cpu-baseline --steps ${STEPS:-5} --warmup 2 > gpurun_out/wfs_$t.log 2>&1
  rc=$?
  echo "tune $t exit $rc: $(tail -1 gpurun_out/wfs_$t.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])' 2>&1 | tail -1)"
  case $rc in 0) ;; *) exit $rc;; esac
done
