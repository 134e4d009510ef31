"""One rank's shard of the N-way split (cost plan), rendered alone on one GPU by the production
kernel (with the bench's lane plan) and by the wavefront tracer (csrc/rt_wavefront.hip): ms per
frame over K back-to-back frames, and whether both leave the same shard and RNG states.

    python tools/wf_shard_probe.py [--config cfg2] [--ns 1,2,4,8] [--frames 6]
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
import shard_timing as ST  # noqa: E402


def frames(rt, scene, W, H, SPP, BOUNCES, mine, r, n, k, **kw):
    rng = rt.alloc_rng(mine.numel() * 256)
    rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
    scene.upload(rng.data_ptr())
    bufs = [torch.zeros((mine.numel() * 256, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(k):
        rt.render(scene, None, bufs[(i + 1) & 1], W, H, SPP, BOUNCES, i, r, n, out_shard=bufs[i & 1], tile_list=mine, **kw)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k, bufs[(k - 1) & 1].cpu().numpy(), rng.view(-1, 12)[:, :6].cpu().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--frames", type=int, default=6)
    args = ap.parse_args()
    rt = G.load_package()
    rt.load_experimental()  # A/B and lone / wavefront / refill paths (librt_hip_exp.so)
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    cost = ST.probe(rt, scene, W, H, SPP, BOUNCES)
    for n in map(int, args.ns.split(",")):
        lists, counts = rt.shard_plan(W, H, n, cost)
        mine = torch.from_numpy(lists[0, : counts[0]]).cuda()
        rng = rt.alloc_rng(mine.numel() * 256)
        rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
        scene.upload(rng.data_ptr())
        lm, nlong, _ = ST.lane_map(rt, scene, W, H, SPP, BOUNCES, mine, rng, (48000.0, 1.0)) if n > 1 else (None, 0, None)
        res = {"config": args.config, "n": n}
        for rep in range(2):
            a = frames(rt, scene, W, H, SPP, BOUNCES, mine, 0, n, args.frames, lane_slots=lm, priority_waves=nlong)
            b = frames(rt, scene, W, H, SPP, BOUNCES, mine, 0, n, args.frames, tracer="wavefront")
            res.setdefault("production_ms", []).append(round(a[0], 3))
            res.setdefault("wavefront_ms", []).append(round(b[0], 3))
        res["bit_exact"] = bool(np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32)) and np.array_equal(a[2], b[2]))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
