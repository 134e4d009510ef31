"""Host vs GPU BVH build time (BVH::Calculate, RayTracing/BVH.cpp:8-124) per BASELINE scene, one JSON
line per scene.  The GPU build is rt_bvh_build_device on device copies of the same arrays and is
checked byte-equal to the host result.

    python tools/bvh_timing.py [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as G  # noqa: E402

rt = G.load_package()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    for which in ("bunny", "bunny4", "plane1m"):
        s = rt.Scene()
        s.setup_plane(708) if which == "plane1m" else s.setup(which)
        t0 = time.perf_counter()
        s.build()
        host_s = time.perf_counter() - t0
        h = s.host_arrays()
        v = torch.from_numpy(h["vertices"].view(np.float32).reshape(-1, 8).copy()).cuda()
        f = torch.from_numpy(h["faces"].view(np.int32).reshape(-1, 4).copy()).cuda()
        rt.bvh_build_device(v, f)  # warm-up (module load, allocator)
        times = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            nodes, fi, count, depth = rt.bvh_build_device(v, f)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        same = (count == len(h["nodes"]) // 32 and
                np.array_equal(nodes[:count].cpu().numpy().view(np.uint8).ravel(), h["nodes"]) and
                np.array_equal(fi.cpu().numpy().view(np.uint8), h["face_indices"]))
        print(json.dumps({"scene": which, "faces": int(f.shape[0]), "nodes": count, "depth": depth,
                          "host_build_s": round(host_s, 4), "gpu_build_s": round(min(times), 4),
                          "byte_identical": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
