"""Tile order and XCD placement of the one-GPU frame: the cost plan (heaviest tile first, runs of
8 tiles per XCD: the default) against "XCD regions" -- the tile grid cut by recursive cost
bisection into 8 compact regions of equal probe cost, region x's tiles heaviest first on XCD x
(list entry k on XCD k % 8 with RT_TUNE XCD runs of one tile, -1 padding where a region has run
out), so each XCD's L2 serves one part of the image.  Both orders render every pixel; frames and
RNG states are compared bit for bit.

    python tools/xcd_order_probe.py [--config cfg2] [--frames 10] [--reps 3]
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


def regions(cost, tx, ty, k):
    """k compact rectangles of the tile grid with equal cost (recursive bisection)."""
    grid = cost.reshape(ty, tx)

    def part(x0, x1, y0, y1, k):
        if k == 1:
            return [[y * tx + x for y in range(y0, y1) for x in range(x0, x1)]]
        sub = grid[y0:y1, x0:x1]
        horiz = (x1 - x0) >= (y1 - y0)
        line = sub.sum(0) if horiz else sub.sum(1)
        cum = np.cumsum(line)
        cut = int(np.searchsorted(cum, cum[-1] / 2.0)) + 1
        cut = min(max(cut, 1), len(line) - 1)
        if horiz:
            return part(x0, x0 + cut, y0, y1, k // 2) + part(x0 + cut, x1, y0, y1, k // 2)
        return part(x0, x1, y0, y0 + cut, k // 2) + part(x0, x1, y0 + cut, y1, k // 2)

    return part(0, tx, 0, ty, k)


def run(rt, scene, W, H, SPP, BOUNCES, order, frames, tune):
    tl = torch.from_numpy(np.asarray(order, dtype=np.int32)).cuda()
    rng = rt.alloc_rng(W * H)
    rt.init_rng_states(rng, W, H, bench.SEED)
    scene.upload(rng.data_ptr())
    bufs = [rt.alloc_surface(W, H) for _ in range(2)]
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(frames):
        rt.render(scene, bufs[i & 1], bufs[(i + 1) & 1], W, H, SPP, BOUNCES, i, tile_list=tl, tune=tune, waves_per_simd=6)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / frames, rt.surface_view(bufs[(frames - 1) & 1], W).cpu().numpy(), rng.view(-1, 12)[:, :6].cpu().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    rt = G.load_package()
    rt.load_experimental()  # A/B and lone / wavefront / refill paths (librt_hip_exp.so)
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    cost = ST.probe(rt, scene, W, H, SPP, BOUNCES)
    tx, ty = (W + 15) // 16, (H + 15) // 16
    lpt = list(np.argsort(-cost, kind="stable"))
    regs = [sorted(r, key=lambda t: -cost[t]) for r in regions(cost, tx, ty, 8)]
    m = max(len(r) for r in regs)
    inter = [regs[x][i] if i < len(regs[x]) else -1 for i in range(m) for x in range(8)]
    res = {"config": args.config, "tiles": tx * ty, "region_tiles": [len(r) for r in regs],
           "region_cost_share": [round(float(cost[r].sum() / cost.sum()), 4) for r in regs], "entries_xcd": len(inter)}
    out = {}
    for rep in range(args.reps):
        for name, order, tune in (("cost_lpt_v5", lpt, 0), ("xcd_regions_v2", inter, 2 << 16), ("cost_lpt_v2", lpt, 2 << 16)):
            t, img, st = run(rt, scene, W, H, SPP, BOUNCES, order, args.frames, tune)
            res.setdefault(name + "_ms", []).append(round(t, 3))
            out[name] = (img, st)
    res["bit_exact"] = bool(all(np.array_equal(out[k][0].view(np.uint32), out["cost_lpt_v5"][0].view(np.uint32))
                                and np.array_equal(out[k][1], out["cost_lpt_v5"][1]) for k in out))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
