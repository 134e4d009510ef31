"""Cost-sorted lane maps on the single-GPU frame (analysis aid, one GPU): a wave idles the lanes whose
pixel is done until its costliest lane finishes (a lane runs its pixel's samples back to back), so
pixels of similar cost in one wave should idle less.  From one lane_cost probe frame, the slots of
every G consecutive tiles of the bench's cost-ordered tile list are sorted by probe work and dealt
into waves of 64 (costliest wave first); the frame is timed against the plain tile order and
checked bit for bit (a lane map is a permutation of the slots).

    python tools/sorted_lanes_probe.py [--config cfg2] [--groups 1,4] [--wps 7] [--frames 5]
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


def sorted_map(cost, tiles, group):
    """slots of `group` consecutive list entries sorted by cost (descending), 64 per wave"""
    rows = []
    for g0 in range(0, tiles, group):
        s = np.arange(g0 * 256, min(tiles, g0 + group) * 256)
        s = s[np.argsort(-cost[s].astype(np.int64), kind="stable")]
        rows.extend(s.reshape(-1, 64))
    return np.concatenate(rows).astype(np.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--groups", default="1,4")
    ap.add_argument("--wps", type=int, default=7)
    ap.add_argument("--frames", type=int, default=5)
    args = ap.parse_args()
    rt = G.load_package()
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    tcost = S.probe(rt, scene, W, H, SPP, BOUNCES)
    lists, counts = rt.shard_plan(W, H, 1, tcost)
    order = torch.from_numpy(lists[0, : counts[0]]).cuda()
    tiles = int(counts[0])
    rng = rt.alloc_rng(W * H)
    rt.init_rng_states(rng, W, H, bench.SEED)
    scene.upload(rng.data_ptr())
    saved = rng.clone()
    bufs = [rt.alloc_surface(W, H) for _ in range(2)]
    cost = torch.zeros(tiles * 256, dtype=torch.int32, device="cuda")
    rt.render(scene, bufs[0], None, W, H, SPP, BOUNCES, 0, tile_list=order, lane_cost=cost)
    torch.cuda.synchronize()
    rng.copy_(saved)
    c = cost.cpu().numpy()
    maps = {"tile order": None}
    for g in map(int, args.groups.split(",")):
        maps[f"sorted G={g}"] = torch.from_numpy(sorted_map(c, tiles, g)).cuda()
    ref = None
    for rep in range(2):
        for name, lm in maps.items():
            ms = []
            for i in range(args.frames):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rt.render(scene, bufs[i & 1], bufs[(i + 1) & 1], W, H, SPP, BOUNCES, i, tile_list=order, lane_slots=lm,
                          waves_per_simd=args.wps)
                e1.record()
                torch.cuda.synchronize()
                if i:
                    ms.append(e0.elapsed_time(e1))
            img = rt.surface_view(bufs[(args.frames - 1) & 1], W).cpu().numpy().copy()
            st = rng.view(-1, 12)[:, :6].cpu().numpy().copy()
            rng.copy_(saved)
            same = True
            if ref is None:
                ref = (img, st)
            else:
                same = bool(np.array_equal(img.view(np.uint32), ref[0].view(np.uint32)) and np.array_equal(st, ref[1]))
            print(json.dumps({"config": args.config, "rep": rep, "map": name, "wps": args.wps,
                              "ms_per_frame": round(float(np.mean(ms)), 3), "bit_exact": same}), flush=True)


if __name__ == "__main__":
    main()
