#!/bin/bash
# One GPU-box pass: parity tests, smoke, a short bench.  Every GPU step has its own time
# limit; a step that faults / aborts / times out ends the script (exit codes 124/134/137/139).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal exit $1 in $2"; exit "$1";; esac; }

timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; tail -5 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -3 gpurun_out/smoke.log; stop_if_fatal $rc smoke
timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-5} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench exit $rc"; tail -3 gpurun_out/bench.log; stop_if_fatal $rc bench
if [ -n "${PROFILE:-}" ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-pmc > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  rc=$?; echo "rocprof exit $rc"; cd "$GRAFT_REPO_ROOT"; stop_if_fatal $rc rocprof
fi
exit 0
