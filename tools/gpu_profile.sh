#!/bin/bash
# rocprofv3 passes on the GPU box: kernel-trace stats, then PMC counters (own run, no tracing
# domains besides the kernel trace).  Outputs land in gpurun_out/prof_*/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$PWD"
ARGS="${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline} --no-pmc"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_trace" -o run -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/prof_trace.log" 2>&1
rc=$?; echo "trace exit $rc"; case $rc in 124|134|137|139) exit $rc;; esac
if [ -n "${PMC:-1}" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace -i "$R/tools/pmc_counters.txt" --output-format csv -d "$R/gpurun_out/prof_pmc" -o run -- python3 "$R/bench.py" ${PMC_ARGS:---steps 1 --warmup 0 --no-cpu-baseline} --no-pmc > "$R/gpurun_out/prof_pmc.log" 2>&1
  rc=$?; echo "pmc exit $rc"; case $rc in 124|134|137|139) exit $rc;; esac
fi
exit 0
