"""Per-wave cost distribution of one frame (timing kernel: bench --tune 256+2048 passed to rt_render): start/end clocks of every 64-pixel wave, for load-balance analysis of the
multi-GPU split.  Records are indexed by workgroup (dispatch order); the sub-tile a workgroup
renders is rt_kernel.hip xcd_block of that index.  Writes gpurun_out/wave_costs.npz and prints a summary."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402
import bench  # noqa: E402

rt = G.load_package()

rt.load_experimental()  # A/B and lone / wavefront / refill paths (librt_hip_exp.so)
scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "cfg2"]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # shard 0 of N
torch.cuda.set_device(0)
scene = rt.Scene()
scene.setup(scene_name)
scene.set_viewport(W, H)
tiles = rt.shard_tiles(W, H, 0, N)
rng = rt.alloc_rng(tiles * 256 if N > 1 else W * H)
rt.init_rng_states(rng, W, H, bench.SEED, 0, N)
scene.upload(rng.data_ptr())
a, b = rt.alloc_surface(W, H), rt.alloc_surface(W, H)
shard = torch.zeros((tiles * 256, 4), dtype=torch.float32, device="cuda")
st = torch.zeros(rt.STAT_COUNT + 8 * tiles * 4, dtype=torch.int64, device="cuda")
if N > 1:
    rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, 0, N, out_shard=shard, stats=st, tune=256 + 2048)
else:
    rt.render(scene, a, b, W, H, SPP, BOUNCES, 0, stats=st, tune=256 + 2048)
torch.cuda.synchronize()
v = st.cpu().numpy()
t = v[rt.STAT_COUNT:].reshape(-1, 8)
dur = (t[:, 1] - t[:, 0]).astype(np.float64)
t0 = t[:, 0].min()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"wave_costs_{N}.npz"), start=t[:, 0] - t0, end=t[:, 1] - t0, small=t[:, 2], big=t[:, 3], rounds=t[:, 4], iters=t[:, 5], wsmall=t[:, 6], lsmall=t[:, 7])
q = np.percentile(dur, [50, 90, 99, 100])
top = np.argsort(dur)[::-1][:8]
for i in top:  # the heaviest waves: cycles, small-phase cycles, wave small steps, busiest lane's steps
    print(f"wave {i}: cyc {dur[i]:.3g} small {t[i, 2]:.3g} big {t[i, 3]:.3g} iters {t[i, 5]} "
          f"wave_steps {t[i, 6]} lane_max_steps {t[i, 7]} cyc/step {t[i, 2] / max(t[i, 6], 1):.0f}")
mid = np.argsort(dur)[len(dur) // 2]
print(f"median wave {mid}: cyc {dur[mid]:.3g} small {t[mid, 2]:.3g} wave_steps {t[mid, 6]} lane_max_steps {t[mid, 7]} "
      f"cyc/step {t[mid, 2] / max(t[mid, 6], 1):.0f}")
print(json.dumps({"waves": int(len(dur)), "mean": float(dur.mean()), "p50": q[0], "p90": q[1], "p99": q[2],
                  "max": q[3], "span": float(t[:, 1].max() - t0), "sum_over_max": float(dur.sum() / q[3])}))
