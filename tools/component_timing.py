"""Timings of the path's set-up and output components on one MI355X (the rows SURVEY.md §8(f) adds
around the hot path), written as one JSON object (profiles/<tag>_components.json):

  init_rng_kernel   curand_init skip-ahead per pixel (Random.cu:3-13) at 1080p and 4K
  bvh               BVH::Calculate (BVH.cpp:8-124) on the host vs rt_bvh_build_device (byte-equal)
  tonemap           viewer display transform (main.cpp:78-94) at 1080p
  unshard           8 gathered compact shards -> pitched surface at 1080p (rank 0 of an 8-GPU frame)
  frames            one progressive frame of every BASELINE config that fits one GPU

GPU times are HIP-event medians over --reps launches on the current stream.

    python tools/component_timing.py --out profiles/r01_components.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402

rt = G.load_package()


def gpu_ms(fn, reps):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
    return float(np.median(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    res = {"device": torch.cuda.get_device_name(0), "reps": a.reps}

    # init_rng
    res["init_rng_ms"] = {}
    for w, h in ((1920, 1080), (3840, 2160)):
        rng = rt.alloc_rng(w * h)
        res["init_rng_ms"][f"{w}x{h}"] = round(gpu_ms(lambda: rt.init_rng_states(rng, w, h, 0xDEADBEEF), a.reps), 3)
        del rng

    # BVH: host vs GPU
    res["bvh"] = {}
    for which in ("bunny", "bunny4", "plane1m"):
        s = rt.Scene()
        s.setup_plane(708) if which == "plane1m" else s.setup(which)
        t0 = time.perf_counter()
        s.build()
        host_ms = (time.perf_counter() - t0) * 1e3
        hh = s.host_arrays()
        v = torch.from_numpy(hh["vertices"].view(np.float32).reshape(-1, 8).copy()).cuda()
        f = torch.from_numpy(hh["faces"].view(np.int32).reshape(-1, 4).copy()).cuda()
        box = {}

        def build():
            box["r"] = rt.bvh_build_device(v, f)

        gms = gpu_ms(build, a.reps)
        nodes, fi, count, depth = box["r"]
        same = (count == len(hh["nodes"]) // 32 and
                np.array_equal(nodes[:count].cpu().numpy().view(np.uint8).ravel(), hh["nodes"]) and
                np.array_equal(fi.cpu().numpy().view(np.uint8), hh["face_indices"]))
        res["bvh"][which] = {"faces": int(f.shape[0]), "nodes": int(count), "depth": int(depth),
                             "host_ms": round(host_ms, 2), "gpu_ms": round(gms, 2), "byte_identical": bool(same)}

    # tonemap and unshard at 1080p
    w, h = 1920, 1080
    surf = rt.alloc_surface(w, h)
    surf.uniform_(0, 4)
    res["tonemap_1080p_ms"] = round(gpu_ms(lambda: rt.tonemap(surf, w, h), a.reps), 3)
    n = 8
    per = rt.shard_tiles(w, h, 0, n)
    shards = torch.rand((n, per * 256, 4), dtype=torch.float32, device="cuda")
    res["unshard_8x_1080p_ms"] = round(gpu_ms(lambda: rt.unshard(surf, w, h, n, shards, per), a.reps), 3)

    # one frame of each single-GPU config (bench.py's workloads)
    import bench  # noqa: E402
    res["frame_ms"] = {}
    for cfg in ("cfg1", "cfg2", "cfg3", "cfg4", "cfg5"):
        which, W, H, spp, bounces, _ = bench.CONFIGS[cfg]
        s = rt.Scene()
        s.setup_plane(708) if which == "plane1m" else s.setup(which)
        s.set_viewport(W, H)
        rng = rt.alloc_rng(W * H)
        rt.init_rng_states(rng, W, H, 0xDEADBEEF)
        t0 = time.perf_counter()
        s.upload(rng.data_ptr())
        torch.cuda.synchronize()
        up = time.perf_counter() - t0
        A, B = rt.alloc_surface(W, H), rt.alloc_surface(W, H)
        res["frame_ms"][cfg] = {"scene": which, "size": [W, H], "spp": spp, "bounces": bounces,
                                "upload_s": round(up, 3),
                                "ms": round(gpu_ms(lambda: rt.render(s, A, B, W, H, spp, bounces), max(2, a.reps // 2)), 3)}
        del s, rng, A, B
        torch.cuda.empty_cache()
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
