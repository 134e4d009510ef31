#!/bin/bash
# Round 3, third pass: VALU/SALU issue microbenchmark, the long-wave scaling probe (K copies of
# the heaviest pixel's / sub-tile's wave), and a same-box A/B of prebuilt library variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal exit $1 in $2"; exit "$1";; esac; }
timeout -k 10 120 ./tools/valu_microbench > gpurun_out/valu_microbench.log 2>&1
rc=$?; echo "microbench exit $rc"; grep -E "v_add_f32|s_add" gpurun_out/valu_microbench.log | head -20; stop_if_fatal $rc microbench
timeout -k 10 300 python -u tools/lone_scaling.py > gpurun_out/lone_scaling.log 2>&1
rc=$?; echo "lone scaling exit $rc"; tail -12 gpurun_out/lone_scaling.log | cut -c1-300; stop_if_fatal $rc lone
REPS=2 VARS="${VARS:-base new}" CFGS="${CFGS:-cfg2}" bash tools/gpu_variants.sh
exit 0
