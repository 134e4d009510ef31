#!/bin/bash
# Round 3 final: the C++ host tests (split path with rt_lane_refine), then the round profiles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_cpp_host.py tests/test_gpu_multi.py > gpurun_out/r03f_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03f_tests.log; [ $rc = 0 ] || exit $rc
TAG=r03e CFGS="${CFGS:-cfg2 cfg4}" STEPS=10 bash tools/gpu_profiles.sh
