#!/bin/bash
# PC sampling (rocprofv3 beta) of the production render kernel on config 2: which instructions the
# waves sit at.  Lists the device's PC-sampling configurations first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 60 rocprofv3 -L > "$R/gpurun_out/pcs_list.txt" 2>&1; echo "list exit $?"
grep -i -A12 "pc_sampl\|PC Sampl" "$R/gpurun_out/pcs_list.txt" | head -40
cd /tmp && timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-stochastic} --pc-sampling-unit ${UNIT:-cycles} --pc-sampling-interval ${INTERVAL:-1048576} --output-format csv -d "$R/gpurun_out/pcs" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-pmc --occupancy 6 > "$R/gpurun_out/pcs.log" 2>&1
rc=$?; echo "pc sampling exit $rc"; tail -5 "$R/gpurun_out/pcs.log"; ls -la "$R/gpurun_out/pcs" 2>/dev/null | head; find "$R/gpurun_out/pcs" -name "*.csv" | head
exit 0
