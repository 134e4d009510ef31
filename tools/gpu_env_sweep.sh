#!/bin/bash
# cfg timing under environment settings: SWEEP="RT_SPLIT_ANGLE=0.3 RT_SPLIT_ANGLE=0.6" CFG=cfg4 bash tools/gpu_env_sweep.sh
# (comma-separated assignments apply together)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for kv in ${SWEEP:-X=0}; do
  i=$((i+1))
  env $(echo "$kv" | tr ',' ' ') timeout -k 10 240 python bench.py --config ${CFG:-cfg4} --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > gpurun_out/sw_$i.log 2>&1
  rc=$?; echo "$kv exit $rc: $(tail -1 gpurun_out/sw_$i.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])' 2>&1)"
  case $rc in 0) ;; *) exit $rc;; esac
done
