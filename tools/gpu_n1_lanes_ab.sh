#!/bin/bash
# Round 3: the single-GPU frame with and without the lane plan + measured refinement (bench.py
# --lanes on / off), interleaved on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2 3; do
  for l in off on; do
    timeout -k 10 240 python bench.py --config ${CFG:-cfg2} --lanes $l --no-pmc --no-cpu-baseline --steps ${STEPS:-20} --warmup 2 > gpurun_out/n1lanes_${l}_$rep.log 2>&1
    rc=$?
    echo "rep $rep lanes $l exit $rc: $(tail -1 gpurun_out/n1lanes_${l}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); p=d.get("plan",{}); print(d["ms_per_step"], p.get("occupancy",{}).get("waves_per_simd"), p.get("occupancy",{}).get("probe_ms"), p.get("lanes",{}).get("refine",{}).get("frame_ms"))' 2>&1 | tail -1)"
    [ $rc = 0 ] || exit $rc
  done
done
