#!/bin/bash
# Round 3, second pass: the GPU test suite (with the full-size config-3 shard test), the default
# bench line after the kernel translation-unit split, the foreign-scene (reference Scene::Upload)
# bench line + its rocprof kernel trace, and the N = 8 contention probe of config 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal exit $1 in $2"; exit "$1";; esac; }
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; tail -3 gpurun_out/pytest_gpu.log; stop_if_fatal $rc pytest
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 420 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_own.json 2> gpurun_out/bench_own.err
rc=$?; echo "bench own exit $rc"; tail -c 300 gpurun_out/bench_own.json; stop_if_fatal $rc bench
timeout -k 10 420 python bench.py --steps 10 --warmup 3 --foreign > gpurun_out/bench_foreign.json 2> gpurun_out/bench_foreign.err
rc=$?; echo "bench foreign exit $rc"; tail -c 300 gpurun_out/bench_foreign.json; stop_if_fatal $rc bench_foreign
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_foreign" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --foreign --no-cpu-baseline --no-pmc > "$R/gpurun_out/prof_foreign.log" 2>&1
rc=$?; echo "rocprof foreign exit $rc"; cd "$R"; stop_if_fatal $rc rocprof_foreign
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_own" -o run -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-pmc > "$R/gpurun_out/prof_own.log" 2>&1
rc=$?; echo "rocprof own exit $rc"; cd "$R"; stop_if_fatal $rc rocprof_own
timeout -k 10 300 python -u tools/contention_probe.py --config cfg2 --n 8 --rank 0 > gpurun_out/contention_n8.log 2>&1
rc=$?; echo "contention exit $rc"; tail -c 800 gpurun_out/contention_n8.log; stop_if_fatal $rc contention
timeout -k 10 300 python -u tools/contention_probe.py --config cfg2 --n 4 --rank 0 > gpurun_out/contention_n4.log 2>&1
rc=$?; echo "contention4 exit $rc"; tail -c 800 gpurun_out/contention_n4.log; stop_if_fatal $rc contention4
exit 0
