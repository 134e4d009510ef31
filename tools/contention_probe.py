"""Where one rank's N-way shard time goes (analysis aid, one GPU): the bench's cost plan for N
ranks, rank r's lane plan, then the shard rendered (production kernel, HIP events) with every
wave, with only the plan's long waves (E >= B/2, the first `long_waves` of the map), with only the
short ones, at 5 and 6 waves per SIMD, and with the long waves at raised priority.  If all >> long
+ short stay near the even share, the waves slow each other down; if long-only is already the
shard time, the chains themselves are the bound.

    python tools/contention_probe.py [--config cfg2] [--n 8] [--rank 0] [--units 48000]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import __graft_entry__ as G  # noqa: E402
import bench  # noqa: E402
import shard_timing as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--units", type=float, default=48000.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lone", type=lambda x: [int(v) for v in x.split(",") if v], default=[256, 1024])
    args = ap.parse_args()
    rt = G.load_package()
    rt.load_experimental()  # A/B and lone / wavefront / refill paths (librt_hip_exp.so)
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    cost = S.probe(rt, scene, W, H, SPP, BOUNCES)
    lists, counts = rt.shard_plan(W, H, args.n, cost)
    mine = torch.from_numpy(lists[args.rank, : counts[args.rank]]).cuda()
    slots = mine.numel() * 256
    rng = rt.alloc_rng(slots)
    rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
    scene.upload(rng.data_ptr())
    saved = rng.clone()
    out = torch.zeros((slots, 4), dtype=torch.float32, device="cuda")
    pc = torch.zeros(slots, dtype=torch.int32, device="cuda")
    rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, out_shard=out, tile_list=mine, lane_cost=pc)
    torch.cuda.synchronize()
    c = pc.cpu().numpy()
    lm, nlong = rt.lane_plan(c, args.units, 1.0)
    maps = {"all": lm, "long": lm[: nlong * 64], "short": lm[nlong * 64:]}
    res = {"config": args.config, "n": args.n, "rank": args.rank, "waves": int(lm.size // 64), "long_waves": int(nlong),
           "even_share_ms": None}

    def timed(m, wps, prio, lone=None):
        d = torch.from_numpy(np.ascontiguousarray(m)).cuda()
        lo = None if lone is None else torch.from_numpy(np.ascontiguousarray(lone, dtype=np.int32)).cuda()
        ms = []
        for i in range(args.reps + 1):
            rng.copy_(saved)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, out_shard=out, tile_list=mine, lane_slots=d,
                      priority_waves=prio, waves_per_simd=wps, lone_slots=lo)
            e1.record()
            torch.cuda.synchronize()
            if i:
                ms.append(e0.elapsed_time(e1))
        return round(float(np.median(ms)), 3)

    for wps in (5, 6):
        for name, m in maps.items():
            res[f"{name}_w{wps}_ms"] = timed(m, wps, 0)
        res[f"all_w{wps}_prio_long_ms"] = timed(lm, wps, nlong)
    # the unplanned shard (sub-tile waves in list order) for reference
    ident = np.arange(slots, dtype=np.int32)
    res["no_lane_plan_w6_ms"] = timed(ident, 6, 0)
    # lone pixels (rt_lone_plan): the main kernel without them, the lone kernel alone, both together
    idle = np.full(64, -1, dtype=np.int32)
    for k in args.lone:
        lone, marked = rt.lone_plan(c, k)
        lmk, nl = rt.lane_plan(marked, args.units, 1.0)
        res[f"lone{k}_main_only_ms"] = timed(lmk, 6, 0)
        res[f"lone{k}_lone_only_ms"] = timed(idle, 6, 0, lone)
        res[f"lone{k}_both_ms"] = timed(lmk, 6, 0, lone)
        res[f"lone{k}_main_waves"] = int(lmk.size // 64)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
