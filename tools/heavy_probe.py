"""Heavy-tile latency probe: the costliest tiles of a frame (probe-frame wave clocks) rendered
alone as one-tile / few-tile shards -- how long the heaviest waves take without contention, against
the slowest shard of an N-way split.  python tools/heavy_probe.py [--config cfg2]"""
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
    args = ap.parse_args()
    rt = G.load_package()
    rt.load_experimental()  # A/B and lone / wavefront / refill paths (librt_hip_exp.so)
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    cost = S.probe(rt, scene, W, H, SPP, BOUNCES)
    order = np.argsort(-cost)
    print(json.dumps({"top_tile_cost": [float(cost[i]) for i in order[:8]], "mean": float(cost.mean())}))
    for k in [1, 2, 8, 32, 128, 512]:
        tiles = order[:k].astype(np.int32)
        ms = S.time_shard(rt, scene, W, H, SPP, BOUNCES, tiles, 0, 1, 3)
        print(json.dumps({"top_k_tiles": k, "ms": round(ms, 3)}), flush=True)


if __name__ == "__main__" and not os.environ.get("HEAVY_BREAKDOWN") and not os.environ.get("HEAVY_LANES"):
    main()


def breakdown(rt, scene, W, H, SPP, BOUNCES, tiles):
    """Timing frame (phase clocks per wave, RT_TUNE 256 + 2048) and statistics frame of `tiles` alone."""
    mine = torch.from_numpy(np.asarray(tiles, dtype=np.int32)).cuda()
    rng = rt.alloc_rng(len(tiles) * 256)
    out = torch.zeros((len(tiles) * 256, 4), dtype=torch.float32, device="cuda")
    res = {}
    for name, tune in [("timing", 256 + 2048), ("stats", 0)]:
        rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
        scene.upload(rng.data_ptr())
        st = torch.zeros(rt.STAT_COUNT + 8 * len(tiles) * 4, dtype=torch.int64, device="cuda")
        rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, 0, 1, out_shard=out, tile_list=mine, stats=st, tune=tune)
        torch.cuda.synchronize()
        v = st.cpu().numpy()
        res[name] = [int(x) for x in v[:24]]
        if name == "timing":
            res["waves"] = [[int(x) for x in r] for r in v[rt.STAT_COUNT:].reshape(-1, 8)]
    return res


if __name__ == "__main__" and os.environ.get("HEAVY_BREAKDOWN"):
    rt = G.load_package()
    rt.load_experimental()  # A/B and lone / wavefront / refill paths (librt_hip_exp.so)
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[os.environ["HEAVY_BREAKDOWN"]]
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    cost = S.probe(rt, scene, W, H, SPP, BOUNCES)
    order = np.argsort(-cost)
    for k in [1, 512]:
        b = breakdown(rt, scene, W, H, SPP, BOUNCES, order[:k])
        if k > 1:
            b.pop("waves")
        print(json.dumps({"top_k": k, "tiles": [int(t) for t in order[:min(k, 4)]], **b}))


def lane_maps(rt, scene, W, H, SPP, BOUNCES, tile):
    """The heaviest tile alone with its 256 pixels spread q per wave (lane map)."""
    mine = torch.tensor([tile], dtype=torch.int32, device="cuda")
    rng = rt.alloc_rng(256)
    out = torch.zeros((256, 4), dtype=torch.float32, device="cuda")
    cost = torch.zeros(256, dtype=torch.int32, device="cuda")
    rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
    scene.upload(rng.data_ptr())
    rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, 0, 1, out_shard=out, tile_list=mine, lane_cost=cost)
    torch.cuda.synchronize()
    c = cost.cpu().numpy().astype(np.int64)
    ref = out.clone()
    print(json.dumps({"tile": int(tile), "lane_cost_top": sorted(c.tolist())[-8:], "lane_cost_mean": float(c.mean())}))
    order = np.argsort(-c)
    for q in [64, 32, 16, 8, 4, 2, 1]:
        nw = 256 // q
        m = -np.ones((nw, 64), dtype=np.int32)
        for i, s in enumerate(order):
            m[i % nw, i // nw] = s  # heaviest pixels spread one per wave first
        lm = torch.from_numpy(m.ravel()).cuda()
        ms = []
        for rep in range(4):
            rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, 0, 1, out_shard=out, tile_list=mine, lane_slots=lm)
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        same = bool(torch.equal(out, ref))
        print(json.dumps({"q": q, "waves": nw, "ms": round(float(np.mean(ms[1:])), 3), "bit_equal": same}), flush=True)


if __name__ == "__main__" and os.environ.get("HEAVY_LANES"):
    rt = G.load_package()
    rt.load_experimental()  # A/B and lone / wavefront / refill paths (librt_hip_exp.so)
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[os.environ["HEAVY_LANES"]]
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    cost = S.probe(rt, scene, W, H, SPP, BOUNCES)
    lane_maps(rt, scene, W, H, SPP, BOUNCES, int(np.argmax(cost)))
