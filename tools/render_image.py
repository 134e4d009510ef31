"""Render progressive frames of a benchmark config on cuda:0 and save the last one:
.pfm (linear) and .ppm (the reference viewer's tonemap).

    python tools/render_image.py [--config cfg2] [--frames 4] [--out gpurun_out/cfg2]
"""
import argparse
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
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "frame"))
    args = ap.parse_args()
    rt = G.load_package()
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[args.config]
    torch.cuda.set_device(0)
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    rng = rt.alloc_rng(W * H)
    rt.init_rng_states(rng, W, H, bench.SEED)
    scene.upload(rng.data_ptr())
    bufs = [rt.alloc_surface(W, H), rt.alloc_surface(W, H)]
    for i in range(args.frames):
        rt.render(scene, bufs[i & 1], bufs[(i + 1) & 1], W, H, SPP, BOUNCES, i)
    final = bufs[(args.frames - 1) & 1]
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    rt.write_pfm(args.out + ".pfm", final, W, H)
    rt.write_ppm(args.out + ".ppm", rt.tonemap(final, W, H))
    print(f"wrote {args.out}.pfm / .ppm ({W}x{H}, {args.frames} frames x {SPP} spp)")


if __name__ == "__main__":
    main()
