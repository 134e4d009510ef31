#!/bin/bash
# Round 3: strong scaling with lone pixels -- shard-by-shard timings of config 2 at N = 1, 2, 4, 8
# for several lone-pixel counts per shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/shard_timing.py --config ${CFG:-cfg2} --plans cost --ns ${NS:-1,2,4,8} --reps 2 --lanes "${LANES:-48000:1}" --lone "${LONES:-0,256,1024,2048,4096}" > gpurun_out/lone_sweep_${CFG:-cfg2}.log 2>&1
rc=$?; echo "sweep exit $rc"; grep -v amdgpu gpurun_out/lone_sweep_${CFG:-cfg2}.log | grep '"n"' | cut -c1-250
exit $rc
