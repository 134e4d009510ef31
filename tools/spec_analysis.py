"""Analysis aid (CPU oracle, not collected by pytest): how predictable is a pixel's sample chain?

A camera sample started at RNG offset o draws 2 + 4 * hits numbers, so sample j of a frame
starts at o_j = 2j + 4m with m the hits of the samples before it.  For a few pixels across the
cost spectrum of config 2, tabulate every even offset over several frames' worth of draws
(oracle_sample_table), follow the real chains, and report how often each frame-relative offset
is on a chain -- the data behind choosing which (pixel, offset) samples to run speculatively.

    python tools/spec_analysis.py [--pixels 24] [--offsets 1024]
"""
import argparse
import ctypes
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import rt_testlib as T  # noqa: E402


def table(L, scene, w, h, x, y, bounces, state, n):
    out = np.zeros((n, 8), dtype=np.float32)
    st = np.ascontiguousarray(state, dtype=np.uint32)
    assert L.oracle_sample_table(scene.h, w, h, x, y, bounces, st.ctypes.data, n, out.ctypes.data) == 0
    return out


def chain(tab, spp):
    """frame-relative offsets of each frame's samples, following the real chain"""
    frames, o = [], 0
    n = tab.shape[0]
    while True:
        start, rel = o, []
        for _ in range(spp):
            if o // 2 >= n:
                return frames
            rel.append(o - start)
            o += int(tab[o // 2, 3])
        frames.append((rel, o - start))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--costs", default="/tmp/cfg2_costs.npy")
    ap.add_argument("--pixels", type=int, default=24)
    ap.add_argument("--offsets", type=int, default=1024)
    args = ap.parse_args()
    L = T.oracle()
    L.oracle_sample_table.restype = ctypes.c_int
    L.oracle_sample_table.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    w, h, spp, bounces = 1920, 1080, 8, 6
    costs = np.load(args.costs)
    work = costs[..., 1].astype(np.int64) + costs[..., 2]
    flat = work.ravel()
    order = np.argsort(flat)[::-1]
    picks = list(order[: args.pixels // 2]) + list(order[np.linspace(1000, 150000, args.pixels - args.pixels // 2).astype(int)])
    scene = T.OracleScene("bunny")
    states = []
    for p in picks:
        s = np.zeros(6, dtype=np.uint32)
        L.oracle_rng_init(T.SEED, int(p), s.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
        states.append(s)

    def job(i):
        y, x = divmod(int(picks[i]), w)
        return table(L, scene, w, h, x, y, bounces, states[i], args.offsets)

    with ThreadPoolExecutor(8) as ex:
        tabs = list(ex.map(job, range(len(picks))))
    for p, tab in zip(picks, tabs):
        y, x = divmod(int(p), w)
        fr = chain(tab, spp)
        draws = np.array([d for _, d in fr])
        hist = {}
        for rel, _ in fr:
            for j, o in enumerate(rel):
                hist.setdefault(j, []).append(o)
        k = (tab[:, 3] - 2) / 4
        spread = [f"{j}:{min(v)}-{max(v)}" for j, v in sorted(hist.items())]
        print(f"px ({x},{y}) work {flat[p]} frames {len(fr)} draws/frame {draws.mean():.0f}+-{draws.std():.0f} "
              f"P(k=6) {np.mean(k == 6):.2f} P(k=0) {np.mean(k == 0):.2f} mean k {k.mean():.2f} "
              f"sample cost {np.mean(tab[:, 5] + tab[:, 6]):.0f}  offsets {' '.join(spread)}")


if __name__ == "__main__":
    main()
