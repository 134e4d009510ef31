#!/bin/bash
# Same-box A/B of bench.py argument sets (and optionally of prebuilt library variants), interleaved
# REPS times, one line per run: ms per frame, kernel ms, check, chosen occupancy, refinement frames.
#   ARGSETS  bench argument sets separated by ';'   e.g. "--tune 0;--tune 0x4000000" or "--lanes off;--lanes on"
#   CFGS     configs (cfg1..cfg5)                   default cfg2
#   VARS     library variants cuda-raytracing_amd/variants/v_<name>.so ("current" = the built one)
#   TESTS    pytest paths run first (e.g. tests/test_gpu_parity.py), stops on failure
#   SHARDS   set: run tools/shard_timing.py with each ARGSET instead of bench.py (strong-scaling shards)
#   REPS STEPS TIMEOUT
# usage: ARGSETS="--occupancy 6;--occupancy 7" REPS=2 bash tools/gpu_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests exit $rc"; tail -3 gpurun_out/ab_tests.log; [ $rc = 0 ] || exit $rc
fi
LIB=cuda-raytracing_amd/librt_hip.so
[ -n "${VARS:-}" ] && cp $LIB cuda-raytracing_amd/variants/current.so.bak
restore() { [ -n "${VARS:-}" ] && cp cuda-raytracing_amd/variants/current.so.bak $LIB; }
IFS=';' read -ra SETS <<< "${ARGSETS:-}"
[ ${#SETS[@]} = 0 ] && SETS=("")
n=0
for rep in $(seq 1 ${REPS:-1}); do
for v in ${VARS:-current}; do
  if [ -n "${VARS:-}" ]; then
    if [ "$v" = current ]; then cp cuda-raytracing_amd/variants/current.so.bak $LIB; else cp "cuda-raytracing_amd/variants/v_$v.so" $LIB; fi
  fi
  for c in ${CFGS:-cfg2}; do
  for a in "${SETS[@]}"; do
    n=$((n + 1)); log=gpurun_out/ab_${n}.log
    if [ -n "${SHARDS:-}" ]; then
      timeout -k 10 ${TIMEOUT:-300} python -u tools/shard_timing.py --config $c $a > $log 2>&1
      rc=$?
      echo "rep $rep $v $c [$a] exit $rc: $(grep '"max_ms"' $log | python3 -c 'import sys,json; print([(d["n"], d.get("lane"), d["max_ms"]) for d in map(json.loads, sys.stdin)])' 2>&1 | tail -1)"
    else
      timeout -k 10 ${TIMEOUT:-300} python bench.py --config $c --no-pmc --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 $a > $log 2>&1
      rc=$?
      echo "rep $rep $v $c [$a] exit $rc: $(tail -1 $log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); p=d.get("plan") or {}; print(d["ms_per_step"], d["roofline"]["kernel_ms"], "check", d.get("check_equal"), "occ", (p.get("occupancy") or {}).get("waves_per_simd"), "refine", ((p.get("lanes") or {}).get("refine") or {}).get("frame_ms"))' 2>&1 | tail -1)"
    fi
    case $rc in 0) ;; *) restore; exit $rc;; esac
  done; done
done; done
restore
exit 0
