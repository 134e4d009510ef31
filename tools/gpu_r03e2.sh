cd "${GRAFT_REPO_ROOT}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_parity.py -k "lane_map or occupancy" > gpurun_out/r03e_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03e_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 500 python -u tools/shard_timing.py --config cfg2 --plans cost --reps 2 --ns 8,4,2 --lanes "48000:1" --wps 6 --refine 3 --theta 0.75 > gpurun_out/r03e_refine_shards.log 2>&1; rc=$?; grep -E '"max_ms"|refine' gpurun_out/r03e_refine_shards.log | cut -c1-220; [ $rc = 0 ] || exit $rc
NS=2 timeout -k 10 500 bash tools/gpu_dist_rehearse.sh
