"""Per-rank render time of the multi-GPU split, measured on one GPU: the kernel for shard 0 of
N (every N-th 16x16 tile) alone, for N = 1, 2, 4, 8 -- the compute side of strong scaling
(the gather of N-1 shards into rank 0 and the unshard kernel come on top).  --weak: the frame
grows with N as bench.py --scaling weak renders it (speedup = N x time(1) / time(N)).

    python tools/shard_timing.py [--config cfg2] [--reps 5] [--weak]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--weak", action="store_true", help="the frame grows with N as in bench.py --scaling weak")
    args = ap.parse_args()
    rt = G.load_package()
    scene_name, W0, H0, SPP, BOUNCES, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    out = {}
    for n in (1, 2, 4, 8):
        W, H = bench.weak_size(W0, H0, n) if args.weak else (W0, H0)
        scene = rt.Scene()
        scene.setup(scene_name)
        scene.set_viewport(W, H)
        per = rt.shard_tiles(W, H, 0, n)
        rng = rt.alloc_rng(per * 256)
        rt.init_rng_states(rng, W, H, bench.SEED, 0, n)
        scene.upload(rng.data_ptr())
        bufs = [torch.zeros((per * 256, 4), dtype=torch.float32, device=dev) for _ in range(2)]
        ms = []
        for i in range(args.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rt.render(scene, None, bufs[(i + 1) & 1], W, H, SPP, BOUNCES, i, 0, n, out_shard=bufs[i & 1])
            e1.record()
            torch.cuda.synchronize()
            if i:
                ms.append(e0.elapsed_time(e1))
        out[n] = sum(ms) / len(ms)
    res = {"config": args.config, "weak": args.weak, "shard0_ms": {str(k): round(v, 3) for k, v in out.items()},
           "compute_speedup": {str(k): round((k if args.weak else 1) * out[1] / v, 2) for k, v in out.items()}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
