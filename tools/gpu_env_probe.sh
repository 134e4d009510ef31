#!/bin/bash
# Host facts of the GPU box (CPU model, usable cores, cgroup quota) and the PMC counter list.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
{
  echo "nproc: $(nproc)"
  python3 -c "import os; print('affinity:', len(os.sched_getaffinity(0)), 'cpu_count:', os.cpu_count())"
  echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
  grep -m1 "model name" /proc/cpuinfo
  lscpu | grep -E "Socket|Core|Thread|NUMA node\(s\)" 
  env | grep -E "OMP_NUM_THREADS|MAX_JOBS" 
} > gpurun_out/env_probe.txt 2>&1
cd /tmp && timeout -k 10 60 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/counters.txt" 2>&1
echo "probe done rc=$?"
