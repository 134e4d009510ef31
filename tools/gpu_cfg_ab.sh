#!/bin/bash
# Timing of configs under --tune variants: CFGS="cfg2 cfg4" TUNES="0 4" bash tools/gpu_cfg_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in ${TUNES:-0}; do
  for c in ${CFGS:-cfg2}; do
    timeout -k 10 240 python bench.py --tune $t --no-pmc --config $c --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/ab_${c}_$t.log 2>&1
    rc=$?; echo "tune $t $c exit $rc: $(tail -1 gpurun_out/ab_${c}_$t.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])' 2>&1)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
