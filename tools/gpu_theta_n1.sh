#!/bin/bash
# Round 3: refinement theta at N = 1 (bench.py --lane-theta), interleaved on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
for rep in 1 2; do
  for th in 0.85 0.95 0.7; do
    timeout -k 10 240 python bench.py --lane-theta $th --no-pmc --no-cpu-baseline --steps 20 --warmup 2 > gpurun_out/theta_${th}_$rep.log 2>&1
    rc=$?
    echo "rep $rep theta $th exit $rc: $(tail -1 gpurun_out/theta_${th}_$rep.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["plan"]["lanes"].get("refine",{}); print(d["ms_per_step"], r.get("frame_ms"), r.get("plain_ms"))' 2>&1 | tail -1)"
    [ $rc = 0 ] || exit $rc
  done
done
