#!/bin/bash
# Kernel trace of the wavefront tracer's frames (per-dispatch durations by generation).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$PWD"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/wf_trace" -o run -- python3 "$R/bench.py" --config ${CFG:-cfg2} --tracer wavefront --steps 2 --warmup 1 --no-pmc --no-cpu-baseline ${BENCH_ARGS} > "$R/gpurun_out/wf_trace.log" 2>&1
rc=$?; echo "wf trace exit $rc"; exit $rc
