#!/bin/bash
# Round-5 profile of the production kernel's own work (GPU box): the default bench line (config 2, its
# frame0_production block: timing-variant phase clocks, small-step iterations, big-leaf tests by twins),
# config 4 likewise, phase clocks at each occupancy, and the small phase's cycles by active-lane count
# (the RT_LANE_HIST timing build of tools/lane_hist.sh in place of librt_hip.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "exit $1 in $2"; cp gpurun_out/r05/librt_hip.so.orig cuda-raytracing_amd/librt_hip.so 2>/dev/null; exit "$1";; esac; }
timeout -k 10 400 python bench.py > gpurun_out/r05/bench_cfg2.json 2> gpurun_out/r05/bench_cfg2.err; fatal $? bench_cfg2
timeout -k 10 400 python bench.py --config cfg4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r05/bench_cfg4.json 2> gpurun_out/r05/bench_cfg4.err; fatal $? bench_cfg4
for w in 5 6 7; do timeout -k 10 120 python tools/phase_clocks.py cfg2 $w >> gpurun_out/r05/phase_clocks.jsonl; fatal $? phase_cfg2; done
for w in 5 7; do timeout -k 10 200 python tools/phase_clocks.py cfg4 $w >> gpurun_out/r05/phase_clocks.jsonl; fatal $? phase_cfg4; done
cp cuda-raytracing_amd/librt_hip.so gpurun_out/r05/librt_hip.so.orig
cp cuda-raytracing_amd/variants/v_lanehist.so cuda-raytracing_amd/librt_hip.so
timeout -k 10 200 python tools/lane_hist.py cfg2 > gpurun_out/r05/lane_hist.jsonl; rc=$?
timeout -k 10 300 python tools/lane_hist.py cfg4 >> gpurun_out/r05/lane_hist.jsonl; rc2=$?
cp gpurun_out/r05/librt_hip.so.orig cuda-raytracing_amd/librt_hip.so; rm -f gpurun_out/r05/librt_hip.so.orig
fatal $rc lane_hist_cfg2; fatal $rc2 lane_hist_cfg4
echo done
