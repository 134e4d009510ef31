#!/bin/bash
# Round-3 first pass on the GPU box: the default bench line (PMC passes + CPU baseline), the host
# CPU probe, and the N = 8 shard timeline of config 2.  Each GPU step has its own time limit; a
# fatal exit (fault / abort / time limit) ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal exit $1 in $2"; exit "$1";; esac; }
timeout -k 10 420 python bench.py --steps 10 --warmup 3 --pmc-dir gpurun_out/pmc > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; tail -c 600 gpurun_out/bench.json; stop_if_fatal $rc bench
timeout -k 10 240 python tools/cpu_probe.py > gpurun_out/cpu_probe.log 2>&1
echo "cpu probe exit $?"
for r in ${RANKS:-0}; do
  timeout -k 10 240 python -u tools/wave_timeline.py --config cfg2 --n 8 --rank $r > gpurun_out/timeline_r$r.log 2>&1
  rc=$?; echo "timeline r$r exit $rc"; head -1 gpurun_out/timeline_r$r.log | cut -c1-700; stop_if_fatal $rc timeline
done
exit 0
