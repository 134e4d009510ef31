"""Per-tile frame pipelining, measured on one GPU for one rank's shard of the N-way split: the
rank's lane plan (rt_lane_plan) is cut into its long waves and its short waves, and K frames are
rendered (a) as now, one launch per frame, frames back to back on one stream, and (b) as two
launch groups on two streams, each running its K frames back to back -- a pixel's frame f + 1
depends only on its own frame f (its RNG state and its `last` value), so the short waves of frame
f + 1 can run while the long waves of frame f finish.  Both orders render every pixel of every
frame; the final shard and RNG states are compared bit for bit.

    python tools/pipeline_probe.py [--config cfg2] [--n 8] [--rank 0] [--frames 10] [--units 48000]
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


def run(rt, scene, W, H, SPP, BOUNCES, mine, r, n, frames, groups, streams):
    """K frames of the shard; groups = [(lane map, priority waves)], one stream each."""
    rng = rt.alloc_rng(mine.numel() * 256)
    rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
    scene.upload(rng.data_ptr())
    bufs = [torch.zeros((mine.numel() * 256, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    main = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for s in streams:
        s.wait_stream(main)
    for i in range(frames):
        for (lm, pw), s in zip(groups, streams):
            rt.render(scene, None, bufs[(i + 1) & 1], W, H, SPP, BOUNCES, i, r, n, out_shard=bufs[i & 1], tile_list=mine,
                      lane_slots=lm, priority_waves=pw, stream=s)
    for s in streams:
        main.wait_stream(s)
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / frames, bufs[(frames - 1) & 1].cpu().numpy(), rng.view(-1, 12)[:, :6].cpu().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--units", type=float, default=48000.0)
    ap.add_argument("--long-frac", type=float, default=1.0, help="long group = this fraction of the plan's long waves")
    args = ap.parse_args()
    rt = G.load_package()
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    cost = ST.probe(rt, scene, W, H, SPP, BOUNCES)
    lists, counts = rt.shard_plan(W, H, args.n, cost)
    mine = torch.from_numpy(lists[args.rank, : counts[args.rank]]).cuda()
    rng = rt.alloc_rng(mine.numel() * 256)
    rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
    scene.upload(rng.data_ptr())
    lm, nlong, _ = ST.lane_map(rt, scene, W, H, SPP, BOUNCES, mine, rng, (args.units, 1.0))
    nl = int(round(nlong * args.long_frac))
    m = lm.cpu().numpy()
    long_map = torch.from_numpy(np.ascontiguousarray(m[: nl * 64])).cuda()
    short_map = torch.from_numpy(np.ascontiguousarray(m[nl * 64:])).cuda()
    res = {"config": args.config, "n": args.n, "rank": args.rank, "waves": int(m.size // 64), "long_waves": nl}
    one = [torch.cuda.current_stream()]
    two = [torch.cuda.Stream(), torch.cuda.Stream()]
    out = {}
    for rep in range(2):
        for mode in ("one_launch", "two_streams"):
            if mode == "one_launch":
                t, img, st = run(rt, scene, W, H, SPP, BOUNCES, mine, args.rank, args.n, args.frames, [(lm, nlong)], one)
            else:
                t, img, st = run(rt, scene, W, H, SPP, BOUNCES, mine, args.rank, args.n, args.frames,
                                 [(long_map, nl), (short_map, 0)], two)
            res.setdefault(mode + "_ms_per_frame", []).append(round(t, 3))
            out[mode] = (img, st)
    res["bit_exact"] = bool(np.array_equal(out["one_launch"][0].view(np.uint32), out["two_streams"][0].view(np.uint32))
                            and np.array_equal(out["one_launch"][1], out["two_streams"][1]))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
