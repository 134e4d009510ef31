"""Child of tests/test_dist_gloo.py::test_launcher_deadline_kills_stalled_job: a gloo rank job
whose rank 1 stalls before the collective (a stand-in for a rank stuck in communicator set-up or
in a send/recv group).  STALL_MODE=watchdog: rank 1 runs under bench.Watchdog instead."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

rank = int(os.environ["RANK"])
wd = bench.Watchdog(rank, float(os.environ.get("STALL_DEADLINE", "0")))
wd.phase = "rendezvous"
dist.init_process_group("gloo")
wd.phase = "collective"
if rank == 1:
    time.sleep(3600)  # stalled rank
t = torch.ones(1)
dist.all_reduce(t)
dist.destroy_process_group()
wd.cancel()
