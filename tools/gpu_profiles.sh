#!/bin/bash
# Round profiles on the GPU box: per BASELINE config the bench line with its in-run PMC pass
# (raw rocprofv3 output kept under gpurun_out/pmc_<cfg>), a rocprofv3 kernel-trace --stats run of
# the default bench, and a HIP API trace of the --foreign path (host synchronisation check).
# usage: TAG=r02 CFGS="cfg1 cfg2 cfg3 cfg4 cfg5" bash tools/gpu_profiles.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$PWD"
TAG="${TAG:-r02}"
fatal() { case "$1" in 0) ;; *) echo "exit $1 in $2"; exit "$1";; esac; }
for c in ${CFGS:-cfg1 cfg2 cfg3 cfg4 cfg5}; do
  extra="--no-cpu-baseline"
  [ "$c" = "cfg2" ] && extra=""
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-5} --warmup 2 --pmc-dir "$R/gpurun_out/pmc_$c" $extra > gpurun_out/bench_${TAG}_$c.log 2>&1
  rc=$?; echo "bench $c exit $rc: $(tail -1 gpurun_out/bench_${TAG}_$c.log | cut -c1-200)"; fatal $rc "bench $c"
  rm -f "$R/gpurun_out/pmc_$c/lane_map.npy"  # the plan's lane map (33 MB for config 3): not a profile
done
if [ -z "${NO_TRACE:-}" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/trace_cfg2" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-pmc --no-cpu-baseline > "$R/gpurun_out/trace_cfg2.log" 2>&1
  rc=$?; echo "kernel trace cfg2 exit $rc"; fatal $rc trace_cfg2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/trace_cfg4" -o run -- python3 "$R/bench.py" --config cfg4 --steps 5 --warmup 1 --no-pmc --no-cpu-baseline > "$R/gpurun_out/trace_cfg4.log" 2>&1
  rc=$?; echo "kernel trace cfg4 exit $rc"; fatal $rc trace_cfg4
  timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$R/gpurun_out/hiptrace_foreign" -o run -- python3 "$R/bench.py" --foreign --steps 10 --warmup 2 --no-pmc --no-cpu-baseline > "$R/gpurun_out/hiptrace_foreign.log" 2>&1
  rc=$?; echo "hip trace foreign exit $rc"; fatal $rc hiptrace
  cd "$R"
fi
exit 0
