"""How a long wave's time depends on how many such waves share the GPU (analysis aid, one GPU):
the heaviest pixel of config 2 (and, separately, its heaviest 8x8 sub-tile) rendered as K copies
of the same wave (a lane map repeating the slot: the copies do identical work and write identical
values), K = 1 .. 6144.  Up to K = 1024 (one wave per SIMD) the time stays the lone wave's own
chain if nothing is shared; beyond that the copies share SIMDs, and the growth says whether a
long wave is issue-bound (time ~ waves per SIMD) or latency-bound (flat until the SIMD's issue
saturates).

    python tools/lone_scaling.py [--config cfg2]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--ks", default="1,64,512,1024,1536,2048,3072,4096,6144")
    ap.add_argument("--tune", type=lambda x: int(x, 0), default=0)
    args = ap.parse_args()
    rt = G.load_package()
    rt.load_experimental()  # A/B and lone / wavefront / refill paths (librt_hip_exp.so)
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    tiles = rt.sharding.tiles_total(W, H)
    mine = torch.arange(tiles, dtype=torch.int32, device="cuda")
    rng = rt.alloc_rng(tiles * 256)
    rt.init_rng_tiles(rng, W, H, mine, bench.SEED)
    scene.upload(rng.data_ptr())
    saved = rng.clone()
    out = torch.zeros((tiles * 256, 4), dtype=torch.float32, device="cuda")
    pc = torch.zeros(tiles * 256, dtype=torch.int32, device="cuda")
    rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, out_shard=out, tile_list=mine, lane_cost=pc)
    torch.cuda.synchronize()
    c = pc.cpu().numpy()
    top = int(np.argmax(c))
    wave_of = c.reshape(-1, 64).max(1)
    topw = int(np.argmax(c.reshape(-1, 64).sum(1)))  # the 8x8 sub-tile with the most work

    def timed(m, wps=6, lone=None):
        d = torch.from_numpy(np.ascontiguousarray(m, dtype=np.int32)).cuda()
        lo = None if lone is None else torch.from_numpy(np.ascontiguousarray(lone, dtype=np.int32)).cuda()
        ms = []
        for i in range(3):
            rng.copy_(saved)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rt.render(scene, None, None, W, H, SPP, BOUNCES, 0, out_shard=out, tile_list=mine, lane_slots=d,
                      waves_per_simd=wps, tune=args.tune, lone_slots=lo)
            e1.record()
            torch.cuda.synchronize()
            if i:
                ms.append(e0.elapsed_time(e1))
        return round(float(np.min(ms)), 3)

    one = np.full(64, -1, dtype=np.int32)
    one[0] = top
    full = np.arange(topw * 64, topw * 64 + 64, dtype=np.int32)
    res = {"config": args.config, "pixel_slot": top, "pixel_work": int(c[top]), "subtile": topw,
           "subtile_work_sum": int(c[topw * 64:(topw + 1) * 64].sum()), "subtile_work_max": int(wave_of[topw])}
    idle = np.full(64, -1, dtype=np.int32)
    for k in map(int, args.ks.split(",")):
        res[f"pixel_x{k}_ms"] = timed(np.tile(one, k))
        res[f"subtile_x{k}_ms"] = timed(np.tile(full, k))
        # the same work through the lone-pixel kernel (rt_lone.hip): K copies of the pixel, and the
        # sub-tile's 64 pixels K times, one wave per pixel
        res[f"lone_pixel_x{k}_ms"] = timed(idle, lone=np.full(k, top, dtype=np.int32))
        if k <= 1024:
            res[f"lone_subtile_x{k}_ms"] = timed(idle, lone=np.tile(full, k))
        print(json.dumps({"k": k, "pixel_ms": res[f"pixel_x{k}_ms"], "subtile_ms": res[f"subtile_x{k}_ms"],
                          "lone_pixel_ms": res[f"lone_pixel_x{k}_ms"],
                          "lone_subtile_ms": res.get(f"lone_subtile_x{k}_ms")}), flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
