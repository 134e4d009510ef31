#!/bin/bash
# The driver's multi-GPU launch shapes rehearsed on a one-GPU box: torchrun N = 1 (RCCL), torchrun
# N = 2 with both ranks on GPU 0 (gloo gather, --check: sharded frame == unsharded bit for bit), and
# bench.py spawning its own 2 ranks.  Same-device times are not scaling numbers (the ranks share a GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 2 --no-pmc --no-cpu-baseline > gpurun_out/dist_n1.log 2>&1 && tail -1 gpurun_out/dist_n1.log | cut -c1-300 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --same-device --backend gloo --check --no-pmc --no-cpu-baseline > gpurun_out/dist_n2.log 2>&1 && tail -1 gpurun_out/dist_n2.log | cut -c1-400 &&
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --same-device --backend gloo --check --no-pmc --no-cpu-baseline > gpurun_out/spawn_n2.log 2>&1 && tail -1 gpurun_out/spawn_n2.log | cut -c1-400
