"""Per-pixel and per-wave work of a frame, counted by the CPU oracle (test infrastructure; an
analysis aid, not collected by pytest): segments, BVH node visits and triangle tests per pixel,
then the 8x8 waves of the render kernel ranked by their heaviest pixel and by their total.

    python tests/pixel_costs.py [--config cfg2] [--top 10]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import rt_testlib as T  # noqa: E402

CONFIGS = {"cfg1": ("bunny", 256, 256, 1, 1), "cfg2": ("bunny", 1920, 1080, 8, 6),
           "cfg4": ("bunny4", 1920, 1080, 8, 6), "small": ("bunny", 320, 180, 8, 6)}


def pixel_costs(which, w, h, spp, bounces, threads=0):
    L = T.oracle()
    L.oracle_render_costs.restype = ctypes.c_int
    L.oracle_render_costs.argtypes = L.oracle_render.argtypes + [ctypes.c_void_p]
    s = T.OracleScene(which)
    out = np.zeros((h, w, 4), dtype=np.float32)
    st = np.zeros(8, dtype=np.uint64)
    costs = np.zeros((h, w, 3), dtype=np.uint32)
    code = L.oracle_render_costs(s.h, w, h, spp, bounces, 0, T.SEED, None, None, out.ctypes.data, 0, h, threads,
                                 st.ctypes.data, costs.ctypes.data)
    assert code == 0
    return costs, st


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--top", type=int, default=10)
    ap.add_argument("--save", default="")
    args = ap.parse_args()
    which, w, h, spp, bounces = CONFIGS[args.config]
    costs, st = pixel_costs(which, w, h, spp, bounces)
    if args.save:
        np.save(args.save, costs)
    work = costs[..., 1].astype(np.int64) + costs[..., 2]  # serial steps ~ nodes + triangle tests
    print(f"frame: segments {st[0]}, nodes {st[1]}, tri tests {st[2]}")
    print(f"pixel work (nodes+tris): mean {work.mean():.0f}, p99 {np.percentile(work, 99):.0f}, max {work.max()}")
    # waves: 8x8 blocks
    hp, wp = (h + 7) // 8 * 8, (w + 7) // 8 * 8
    pad = np.zeros((hp, wp), dtype=np.int64)
    pad[:h, :w] = work
    blk = pad.reshape(hp // 8, 8, wp // 8, 8).transpose(0, 2, 1, 3).reshape(hp // 8, wp // 8, 64)
    wmax, wsum = blk.max(-1), blk.sum(-1)
    print(f"waves: {wmax.size}; max-pixel per wave: mean {wmax.mean():.0f}, max {wmax.max()}; "
          f"wave total: mean {wsum.mean():.0f}, max {wsum.max()}")
    print(f"heaviest pixel / mean pixel = {work.max() / work.mean():.1f}; "
          f"heaviest wave max-pixel / mean wave max-pixel = {wmax.max() / wmax.mean():.1f}")
    order = np.argsort(work.ravel())[::-1][: args.top]
    for i in order:
        y, x = divmod(int(i), w)
        print(f"  pixel ({x},{y}): seg {costs[y, x, 0]}, nodes {costs[y, x, 1]}, tris {costs[y, x, 2]}")


if __name__ == "__main__":
    main()
