"""Per-rank render time of the multi-GPU split, measured on one GPU shard by shard: for N = 1, 2,
4, 8 every shard of the frame's plan is rendered alone (its own RNG states, compact output) and
timed with HIP events; the job's compute time is the slowest shard (the gather of N-1 shards into
rank 0 and the unshard kernel come on top).  Plans: round-robin ("rr") and the bench's default
cost plan ("cost": one probe frame's per-wave clocks, longest processing time first, heaviest
tiles first on every rank).  --weak: the frame grows with N as bench.py --scaling weak renders it.

    python tools/shard_timing.py [--config cfg2] [--reps 3] [--plans rr,cost] [--ns 1,2,4,8] [--weak]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402
import bench  # noqa: E402


def probe(rt, scene, W, H, SPP, BOUNCES):
    """Per-tile cost of the whole frame from one production frame's per-wave clocks."""
    lists, counts = rt.shard_plan(W, H, 1)
    order = torch.from_numpy(lists[0, : counts[0]]).cuda()
    rng = rt.alloc_rng(int(counts[0]) * 256)
    rt.init_rng_tiles(rng, W, H, order, bench.SEED)
    scene.upload(rng.data_ptr())
    out = torch.zeros((int(counts[0]) * 256, 4), dtype=torch.float32, device="cuda")
    clk = torch.zeros(int(counts[0]) * 4, dtype=torch.int64, device="cuda")
    rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, out_shard=out, tile_list=order, wave_clock=clk)
    torch.cuda.synchronize()
    cost = np.zeros(rt.sharding.tiles_total(W, H))
    cost[lists[0, : counts[0]]] = bench.sanitize_wave_clocks(clk.cpu().numpy())[0].reshape(-1, 4).sum(1)
    return cost


TUNE, WPS, SPLIT, LONE, LONE_MIN = 0, 0, 1, 0, 1  # --tune / --wps / --split / --lone / --lone-min
SKIP_NO_LANE = bool(os.environ.get("SKIP_NO_LANE"))  # only the lane-plan rows
REFILL = 0  # --refill: rt_render refill_lanes of the timed frames
REFINE, THETA = 0, 0.85  # --refine / --theta: bench.refine_lane_map rounds after the lane plan


def lane_map(rt, scene, W, H, SPP, BOUNCES, mine, rng, lane):
    """rt_lane_plan of this shard from one probe frame's per-pixel work (lane = (ratio, budget))."""
    rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
    out = torch.zeros((mine.numel() * 256, 4), dtype=torch.float32, device="cuda")
    cost = torch.zeros(mine.numel() * 256, dtype=torch.int32, device="cuda")
    rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, 0, 1, out_shard=out, tile_list=mine, lane_cost=cost)
    torch.cuda.synchronize()
    c = cost.cpu().numpy()
    if os.environ.get("LANE_SAVE"):  # per-slot probe costs for offline plan work
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        np.save(os.path.join(ROOT, "gpurun_out", f"lanecost_{os.environ['LANE_SAVE']}_{mine.numel()}_{int(mine[0])}.npy"), c)
    lone = None
    if LONE:  # the costliest pixels to the lone-pixel kernel (rt_lone_plan), the rest through the lane plan
        lone_np, c = rt.lone_plan(c, LONE, LONE_MIN)
        lone = torch.from_numpy(lone_np).cuda() if lone_np.size else None
    m, nlong = rt.lane_plan(c, lane[0], lane[1])
    nlong = int(lane[2]) if len(lane) >= 3 else nlong  # lane[2]: the number of leading waves at raised priority
    rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
    if REFINE:  # the bench's measured refinement (rt_lane_refine), same frames, same RNG copies
        def frame(**kw):
            rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, 0, 1, out_shard=out, tile_list=mine, **kw)
        m, info = bench.refine_lane_map(rt, frame, rng, m, c, REFINE, THETA, "cuda", waves_per_simd=WPS or 6)
        print(json.dumps({"refine": info, "waves": int(m.size // 64) if m is not None else 0}), flush=True)
        nlong = 0
        if m is None:  # the plain tile order won
            return None, 0, lone
    lm = torch.from_numpy(m).cuda()
    if os.environ.get("LANE_DIAG"):  # which waves are the long ones under this plan
        clk = torch.zeros(m.size // 64, dtype=torch.int64, device="cuda")
        rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, 0, 1, out_shard=out, tile_list=mine, lane_slots=lm,
                  wave_clock=clk, priority_waves=nlong)
        torch.cuda.synchronize()
        rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
        wc = clk.cpu().numpy()
        mw = m.reshape(-1, 64)
        nh = int(np.argmax((mw >= 0).sum(1) == 64)) if ((mw >= 0).sum(1) == 64).any() else len(mw)
        top = np.argsort(-wc)[:5]
        print(json.dumps({"slots": int(c.size), "cmax": int(c.max()), "csum": int(c.sum()), "R": round(float(c.sum()) / c.max(), 1),
                          "p99": float(np.percentile(c[c > 0], 99)), "waves": int(len(mw)), "long": nlong, "first_full_wave": nh,
                          "top_waves": [[int(i), round(float(wc[i]) / 1e5, 3), int((mw[i] >= 0).sum()),
                                         int(c[mw[i][mw[i] >= 0]].max()), int(c[mw[i][mw[i] >= 0]].sum())] for i in top]}),
              flush=True)
    return lm, nlong, lone


def time_shard(rt, scene, W, H, SPP, BOUNCES, tiles, r, n, reps, lane=None):
    mine = torch.from_numpy(tiles).cuda()
    rng = rt.alloc_rng(len(tiles) * 256)
    rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
    scene.upload(rng.data_ptr())
    lm, nlong, lone = lane_map(rt, scene, W, H, SPP, BOUNCES, mine, rng, lane) if lane else (None, 0, None)
    if SPLIT > 1:  # every 8x8 wave split into SPLIT waves of 64 / SPLIT pixels (rows of the sub-tile)
        slots = np.arange(len(tiles) * 256, dtype=np.int32).reshape(-1, SPLIT, 64 // SPLIT)
        m = np.full((slots.shape[0] * SPLIT, 64), -1, dtype=np.int32)
        m[:, : 64 // SPLIT] = slots.reshape(-1, 64 // SPLIT)
        lm, nlong = torch.from_numpy(m.ravel()).cuda(), 0
    bufs = [torch.zeros((len(tiles) * 256, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
    ms = []
    for i in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rt.render(scene, None, bufs[(i + 1) & 1], W, H, SPP, BOUNCES, i, r, n, out_shard=bufs[i & 1], tile_list=mine,
                  lane_slots=lm, priority_waves=nlong, tune=TUNE, waves_per_simd=WPS, lone_slots=lone,
                  refill_lanes=REFILL)
        e1.record()
        torch.cuda.synchronize()
        if i:
            ms.append(e0.elapsed_time(e1))
    return float(np.mean(ms))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--plans", default="rr,cost")
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--weak", action="store_true", help="the frame grows with N as in bench.py --scaling weak")
    ap.add_argument("--lanes", default="", help="lane plans to try, 'ratio:budget;...' (rt_lane_plan)")
    ap.add_argument("--tune", type=lambda x: int(x, 0), default=0, help="diagnostic A/B knobs passed to rt_render")
    ap.add_argument("--wps", type=int, default=0, help="rt_render waves_per_simd (0 = default)")
    ap.add_argument("--split", type=int, default=1, help="split every 8x8 wave into this many waves (1, 2, 4)")
    ap.add_argument("--lone", default="0", help="comma list of lone-pixel counts per shard to try (rt_lone_plan)")
    ap.add_argument("--lone-min", type=int, default=1, help="rt_lone_plan min_cost")
    ap.add_argument("--refill", type=int, default=0, help="rt_render refill_lanes of the timed frames (0 = off)")
    ap.add_argument("--refine", type=int, default=0, help="rounds of measured lane-plan refinement (bench --lane-refine)")
    ap.add_argument("--theta", type=float, default=0.85, help="rt_lane_refine theta (bench --lane-theta)")
    args = ap.parse_args()
    global TUNE, WPS, SPLIT, LONE, LONE_MIN, REFINE, THETA, REFILL
    REFILL = args.refill
    TUNE, WPS, SPLIT, LONE_MIN, REFINE, THETA = args.tune, args.wps, args.split, args.lone_min, args.refine, args.theta
    lone_list = [int(x) for x in args.lone.split(",")]
    rt = G.load_package()
    rt.load_experimental()  # A/B and lone / wavefront / refill paths (librt_hip_exp.so)
    scene_name, W0, H0, SPP, BOUNCES, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    res = {"config": args.config, "weak": args.weak, "plans": {}}
    costs = {}
    lanes = [None] + [tuple(map(float, x.split(":"))) for x in args.lanes.split(";") if x]
    plans = [(p, l, k) for p in args.plans.split(",") for l in lanes for k in (lone_list if l else [0])]
    for plan, lane, lone_k in plans:
        if lane is None and SKIP_NO_LANE:
            continue
        LONE = lone_k
        per_n = {}
        for n in map(int, args.ns.split(",")):
            W, H = bench.weak_size(W0, H0, n) if args.weak else (W0, H0)
            scene = rt.Scene()
            scene.setup(scene_name)
            scene.set_viewport(W, H)
            if plan == "cost":
                if (W, H) not in costs:
                    costs[(W, H)] = probe(rt, scene, W, H, SPP, BOUNCES)
                lists, counts = rt.shard_plan(W, H, n, costs[(W, H)])
            else:
                lists, counts = rt.shard_plan(W, H, n)
            shard_ms = [time_shard(rt, scene, W, H, SPP, BOUNCES, lists[r, : counts[r]], r, n, args.reps, lane)
                        for r in range(n)]
            per_n[n] = shard_ms
            print(json.dumps({"plan": plan, "lane": lane, "lone": lone_k, "n": n, "max_ms": round(max(shard_ms), 3),
                              "shard_ms": [round(x, 3) for x in shard_ms]}), flush=True)
        t1 = max(per_n[min(per_n)])
        res["plans"][plan + ("" if lane is None else f" lane{lane}") + (f" lone{lone_k}" if lone_k else "")] = {"max_shard_ms": {str(n): round(max(v), 3) for n, v in per_n.items()},
                              "shard_ms": {str(n): [round(x, 3) for x in v] for n, v in per_n.items()},
                              "compute_speedup": {str(n): round((n if args.weak else 1) * t1 / max(v), 2)
                                                  for n, v in per_n.items()}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
