#!/bin/bash
# Round 3: the lone-pixel kernel -- its parity tests, then the long-wave scaling probe with it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal exit $1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -v -x --timeout 300 --timeout-method thread -k "${TESTK:-lone or one_pixel}" > gpurun_out/pytest_lone.log 2>&1
rc=$?; echo "lone tests exit $rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_lone.log | tail -15; stop_if_fatal $rc tests
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u tools/lone_scaling.py --ks ${KS:-1,1024,2048,4096} > gpurun_out/lone_scaling2.log 2>&1
rc=$?; echo "lone scaling exit $rc"; grep -v amdgpu gpurun_out/lone_scaling2.log | cut -c1-400; stop_if_fatal $rc lone
exit 0
