"""Measured lane-plan refinement (analysis aid, one GPU): does splitting the waves that a probe frame
MEASURES as the longest (per-wave clocks) shorten a strong-scaled shard, where rt_lane_plan's cost
model (E = max c x (sum c / max c)^0.34) alone stops?

For every rank of the bench's N-way cost plan: rt_lane_plan from one lane_cost probe frame, then
ITERS rounds of (time the shard with the production kernel; one timing frame with per-wave clocks;
split every wave whose measured duration is >= THETA x the longest into two, heaviest pixels dealt
alternately; order the waves by their expected duration, longest first).  RNG states are restored
after every probe, so each timed frame renders the same pixels bit for bit (a lane map is a
permutation of the shard's slots).  Prints the slowest rank's shard time per round.

    python tools/lane_refine_probe.py [--config cfg2] [--ns 8,4] [--iters 4] [--theta 0.7]
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


def split_waves(m, c, d, theta, ways=2):
    """m: int32 [waves, 64] lane map (-1 = idle lane); c: per-slot cost; d: per-wave measured ticks."""
    longest = float(d.max())
    rows, est = [], []
    for w in range(m.shape[0]):
        px = m[w][m[w] >= 0]
        if d[w] >= theta * longest and px.size > 1:
            px = px[np.argsort(-c[px], kind="stable")]
            for g in range(ways):
                part = px[g::ways]
                if part.size:
                    rows.append(part)
                    est.append(d[w] * 0.75)
        else:
            rows.append(px)
            est.append(float(d[w]))
    order = np.argsort(-np.asarray(est), kind="stable")
    out = np.full((len(rows), 64), -1, dtype=np.int32)
    for i, k in enumerate(order):
        out[i, : rows[k].size] = rows[k]
    return out


def shard_rounds(rt, scene, W, H, SPP, BOUNCES, tiles, iters, theta, wps, units):
    mine = torch.from_numpy(tiles).cuda()
    n_slots = len(tiles) * 256
    rng = rt.alloc_rng(n_slots)
    rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
    scene.upload(rng.data_ptr())
    out = torch.zeros((n_slots, 4), dtype=torch.float32, device="cuda")
    prev = torch.zeros_like(out)
    cost = torch.zeros(n_slots, dtype=torch.int32, device="cuda")
    saved = rng.clone()
    rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, 0, 1, out_shard=out, tile_list=mine, lane_cost=cost)
    torch.cuda.synchronize()
    rng.copy_(saved)
    c = cost.cpu().numpy().astype(np.int64)
    m0, _ = rt.lane_plan(c, units, 1.0)
    m = m0.reshape(-1, 64)
    res = []
    ref = None
    for it in range(iters + 1):
        lm = torch.from_numpy(np.ascontiguousarray(m.ravel())).cuda()
        ms = []
        for rep in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rt.render(scene, None, prev, W, H, SPP, BOUNCES, 0, 0, 1, out_shard=out, tile_list=mine, lane_slots=lm,
                      waves_per_simd=wps)
            e1.record()
            torch.cuda.synchronize()
            rng.copy_(saved)
            if rep:
                ms.append(e0.elapsed_time(e1))
        img = out.cpu().numpy()
        same = True if ref is None else bool(np.array_equal(img.view(np.uint32), ref.view(np.uint32)))
        ref = img if ref is None else ref
        clk = torch.zeros(m.shape[0], dtype=torch.int64, device="cuda")
        rt.render(scene, None, prev, W, H, SPP, BOUNCES, 0, 0, 1, out_shard=out, tile_list=mine, lane_slots=lm,
                  wave_clock=clk)
        torch.cuda.synchronize()
        rng.copy_(saved)
        d = clk.cpu().numpy().astype(np.float64)
        res.append({"iter": it, "ms": round(float(np.mean(ms)), 3), "waves": int(m.shape[0]),
                    "longest_wave_ms": round(float(d.max()) / 1e5, 3), "p90_wave_ms": round(float(np.percentile(d, 90)) / 1e5, 3),
                    "bit_exact_vs_iter0": same})
        if it < iters:
            m = split_waves(m, c, d, theta)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--ns", default="8,4")
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--theta", type=float, default=0.7)
    ap.add_argument("--wps", type=int, default=6)
    ap.add_argument("--units", type=float, default=48000.0)
    args = ap.parse_args()
    rt = G.load_package()
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    cost = S.probe(rt, scene, W, H, SPP, BOUNCES)
    for n in map(int, args.ns.split(",")):
        lists, counts = rt.shard_plan(W, H, n, cost)
        per_rank = [shard_rounds(rt, scene, W, H, SPP, BOUNCES, lists[r, : counts[r]], args.iters, args.theta, args.wps,
                                 args.units) for r in range(n)]
        for it in range(args.iters + 1):
            rows = [p[it] for p in per_rank]
            print(json.dumps({"config": args.config, "n": n, "theta": args.theta, "wps": args.wps, "iter": it,
                              "max_ms": max(r["ms"] for r in rows), "shard_ms": [r["ms"] for r in rows],
                              "waves": [r["waves"] for r in rows], "longest_wave_ms": max(r["longest_wave_ms"] for r in rows),
                              "bit_exact": all(r["bit_exact_vs_iter0"] for r in rows)}), flush=True)


if __name__ == "__main__":
    main()
