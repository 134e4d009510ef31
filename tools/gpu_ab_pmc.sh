#!/bin/bash
# Same-box A/B of prebuilt library variants with the bench's in-run PMC pass (VALU / SALU instructions,
# lane utilisation, HBM bytes per launch) -- one line per run.
#   VARS  variants cuda-raytracing_amd/variants/v_<name>.so ("current" = the built one)   CFGS (default cfg2)
#   ARGS  extra bench arguments (e.g. "--occupancy 7")   REPS (default 2)   TIMEOUT (default 300)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=cuda-raytracing_amd/librt_hip.so
cp $LIB /tmp/current.so.bak
n=0
for rep in $(seq 1 ${REPS:-2}); do
for c in ${CFGS:-cfg2}; do
for v in ${VARS:-current}; do
  if [ "$v" = current ]; then cp /tmp/current.so.bak $LIB; else cp "cuda-raytracing_amd/variants/v_$v.so" $LIB; fi
  n=$((n + 1)); log=gpurun_out/abp_${n}.log
  timeout -k 10 ${TIMEOUT:-300} python bench.py --config $c --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 ${ARGS:-} > $log 2>&1
  rc=$?
  echo "rep $rep $c $v exit $rc: $(tail -1 $log | python3 -c '
import sys, json
d = json.loads(sys.stdin.read()); r = d["roofline"]; p = d.get("config", {}).get("plan") or d.get("plan") or {}
print(d["ms_per_step"], "kernel", r.get("kernel_ms"), "valu", r.get("valu_wave_instructions_per_launch"),
      "salu", r.get("salu_instructions_per_launch"), "lanes", r.get("lane_utilization"), "traffic", r.get("traffic"),
      "check", d.get("check_equal"), r.get("kernel"), "issue", json.dumps(r.get("issue")))' 2>&1 | tail -1)"
  [ $rc = 0 ] || { cp /tmp/current.so.bak $LIB; exit $rc; }
done; done; done
cp /tmp/current.so.bak $LIB
