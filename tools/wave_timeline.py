"""Timeline of one rank's frame under the multi-GPU plan (analysis aid, one GPU): the bench's cost
plan for N ranks, then rank r's lane plan, then one timing frame (RT_TUNE 256 + 2048: per-wave
start / end on the device's 100 MHz clock) of exactly that shard.  Prints where the shard's time
goes -- when the last waves start, how long the longest run, how many pixels they hold, the
probe work of their heaviest pixel -- and saves gpurun_out/timeline_<cfg>_n<N>_r<r>.npz.

    python tools/wave_timeline.py [--config cfg2] [--n 8] [--rank 0] [--units 48000]
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
    ap.add_argument("--tune", type=lambda x: int(x, 0), default=0)
    ap.add_argument("--lone", type=int, default=0, help="pixels to the lone-pixel kernel (timing frame: left out)")
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
    out = torch.zeros((slots, 4), dtype=torch.float32, device="cuda")
    pc = torch.zeros(slots, dtype=torch.int32, device="cuda")
    rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, out_shard=out, tile_list=mine, lane_cost=pc)
    torch.cuda.synchronize()
    c = pc.cpu().numpy()
    lone = None
    if args.lone:  # the costliest pixels to the lone-pixel kernel (rt_lone_plan), the rest through the lane plan
        lone_np, c = rt.lone_plan(c, args.lone)
        lone = torch.from_numpy(lone_np).cuda()
    lm, nlong = rt.lane_plan(c, args.units, 1.0)
    rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
    lmd = torch.from_numpy(lm).cuda()
    waves = lm.size // 64
    res = {}
    for label, tune in (("production", 0), ("timing", 256 + 2048)):
        rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
        st = torch.zeros(rt.STAT_COUNT + 8 * waves, dtype=torch.int64, device="cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, out_shard=out, tile_list=mine, lane_slots=lmd,
                  stats=st if tune else None, tune=tune | args.tune, lone_slots=None if tune else lone)
        e1.record()
        torch.cuda.synchronize()
        res[label] = e0.elapsed_time(e1)
    t = st.cpu().numpy()[rt.STAT_COUNT:].reshape(-1, 8)
    start, end = t[:, 0].astype(np.float64), t[:, 1].astype(np.float64)
    t0 = start.min()
    start, end = (start - t0) / 1e5, (end - t0) / 1e5  # ms
    dur = end - start
    mw = lm.reshape(-1, 64)
    npx = (mw >= 0).sum(1)
    cmax = np.array([c[r[r >= 0]].max() if (r >= 0).any() else 0 for r in mw])
    csum = np.array([c[r[r >= 0]].sum() if (r >= 0).any() else 0 for r in mw])
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"timeline_{args.config}_n{args.n}_r{args.rank}_l{args.lone}.npz"), start=start, end=end,
             npx=npx, cmax=cmax, csum=csum, small=t[:, 2], big=t[:, 3], iters=t[:, 5], wsmall=t[:, 6], lsmall=t[:, 7],
             lane_cost=c, lane_map=lm)
    top = np.argsort(-end)[:10]
    print(json.dumps({"config": args.config, "n": args.n, "rank": args.rank, "tiles": int(mine.numel()),
                      "waves": int(waves), "long_waves": int(nlong), "production_ms": round(res["production"], 3),
                      "timing_ms": round(res["timing"], 3), "span_ms": round(float(end.max()), 3),
                      "cost_max": int(c.max()), "cost_sum": int(c.sum()),
                      "start_pcts_ms": [round(float(x), 3) for x in np.percentile(start, [50, 90, 99, 100])],
                      "dur_pcts_ms": [round(float(x), 3) for x in np.percentile(dur, [50, 90, 99, 100])],
                      "waves_ending_after_half": int((end > 0.5 * end.max()).sum())}))
    for i in top:
        print(json.dumps({"wave": int(i), "start": round(float(start[i]), 3), "end": round(float(end[i]), 3),
                          "pixels": int(npx[i]), "cmax": int(cmax[i]), "csum": int(csum[i]),
                          "small_cyc": int(t[i, 2]), "big_cyc": int(t[i, 3]), "wave_small_steps": int(t[i, 6]),
                          "lane_max_steps": int(t[i, 7])}))


if __name__ == "__main__":
    main()
