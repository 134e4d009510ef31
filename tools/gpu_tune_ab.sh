#!/bin/bash
# Same-box A/B of diagnostic tune values: bench per (tune, occupancy, config), REPS times interleaved.
# usage: TUNES="0 0x8000000" OCCS="5 6" CFGS="cfg2" REPS=2 bash tools/gpu_tune_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-1}); do
for c in ${CFGS:-cfg2}; do
for o in ${OCCS:-auto}; do
for t in ${TUNES:-0}; do
  log=gpurun_out/tab_${c}_${o}_${t}_$rep.log
  timeout -k 10 240 python bench.py --config $c --no-pmc --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 --occupancy $o --tune $t > $log 2>&1
  rc=$?
  echo "rep $rep $c occ $o tune $t exit $rc: $(tail -1 $log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])' 2>&1 | tail -1)"
  [ $rc = 0 ] || exit $rc
done; done; done; done
