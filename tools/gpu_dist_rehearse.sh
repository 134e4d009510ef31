#!/bin/bash
# The driver's multi-GPU launch shapes rehearsed on a one-GPU box: torchrun N = 1 (RCCL), torchrun
# N = 2, 4 and 8 with every rank on GPU 0 (gloo gather, --check: sharded frame == unsharded bit for
# bit), and bench.py spawning its own 2 ranks.  Same-device times are not scaling numbers (the ranks
# share a GPU); the lines carry plan.invalid_wave_clocks (probe clocks the sanitiser had to replace).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out && export TMPDIR=/tmp
show() { tail -1 "$1" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["n_gpus"], d["ms_per_step"], "check", d.get("check_equal"), "invalid clocks", d.get("plan",{}).get("invalid_wave_clocks"), "waves/SIMD", d.get("plan",{}).get("occupancy",{}).get("waves_per_simd"))'; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 2 --no-pmc --no-cpu-baseline > gpurun_out/dist_n1.log 2>&1 && tail -1 gpurun_out/dist_n1.log | cut -c1-200 || exit $?
for n in ${NS:-2 4 8}; do
  timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29510 + n)) bench.py --gpus $n --steps 5 --warmup 2 --same-device --backend gloo --check --no-pmc --no-cpu-baseline > gpurun_out/dist_n$n.log 2>&1 && show gpurun_out/dist_n$n.log || exit $?
done
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --same-device --backend gloo --check --no-pmc --no-cpu-baseline > gpurun_out/spawn_n2.log 2>&1 && show gpurun_out/spawn_n2.log
