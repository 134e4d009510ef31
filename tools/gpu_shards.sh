#!/bin/bash
# Shard-by-shard timing of the multi-GPU plans on one GPU (tools/shard_timing.py), per config.
# usage: CFGS="cfg2 cfg3" bash tools/gpu_shards.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for c in ${CFGS:-cfg2}; do
  timeout -k 10 ${SHARD_TIMEOUT:-300} python -u tools/shard_timing.py --config $c ${SHARD_ARGS:-} > gpurun_out/shards_$c.log 2>&1
  rc=$?; echo "shards $c exit $rc"; tail -1 gpurun_out/shards_$c.log | cut -c1-600
  case $rc in 0) ;; *) exit $rc;; esac
done
