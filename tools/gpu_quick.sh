#!/bin/bash
# Quick A/B on the GPU box: parity subset, then bench per --tune value and config.
# usage: TESTS="tests/test_gpu_parity.py" TUNES="0 0x200000" CFGS="cfg2 cfg4" bash tools/gpu_quick.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > gpurun_out/quick_tests.log 2>&1
  rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/quick_tests.log; case $rc in 0) ;; *) exit $rc;; esac
fi
for c in ${CFGS:-cfg2}; do
  for t in ${TUNES:-0}; do
    timeout -k 10 240 python bench.py --config $c --tune $t --no-pmc --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/q_${c}_$t.log 2>&1
    rc=$?
    echo "$c tune=$t exit $rc: $(tail -1 gpurun_out/q_${c}_$t.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel_ms"], d["value"])' 2>&1 | tail -1)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
