#!/bin/bash
# GPU parity tests, then A/B bench timings: AB="0 8" bash tools/gpu_test_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest -m gpu exit $rc"; tail -3 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
bash tools/gpu_ab.sh
