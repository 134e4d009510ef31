"""Analysis: how many big-leaf visits an exact cull screen could take off the shared big-leaf rounds.

Reads tools/bigleaf_rays.c records (rays that reach a leaf of > 8 triangles, with the closest distance
at entry) and prices screens built from the leaf tree of that leaf (leaftree.h: boxes, normal cones,
cluster_cull's proven error bound, rt_fast.h): for a ray, a screen node is "culled" when cluster_cull
proves none of its triangles can pass glm's fp32 test with 0 <= t < closest.

    python tools/bigleaf_cull.py /tmp/bl_cfg2.bin [scene]
"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
rt = importlib.import_module("cuda-raytracing_amd")

f32 = np.float32


def cull(o, nd, best, K, fast=None):
    """rt_fast.h cluster_cull vectorised over rays (float32, the same operation order; the device's
    1-ulp sqrt / rcp are covered by the bound's widening, the host uses IEEE)."""
    U = f32(2.0 ** -24)
    K0, K1, K2, K3 = (K[4 * i:4 * i + 4].astype(f32) for i in range(4))
    E1, Nmin = K0[3], K1[3]
    dota = np.abs(nd[:, 0] * K2[0] + nd[:, 1] * K2[1] + nd[:, 2] * K2[2])
    ca = np.minimum(np.maximum(dota * f32(1 - 2 ** -20) - f32(4) * U, f32(0)), f32(1))
    sa = np.sqrt(np.maximum(f32(1) - ca * ca, f32(0)) + f32(2) * U) * f32(1 + 2 ** -20)
    dlb = Nmin * ((ca * K2[3] - sa * K3[0]) - f32(4) * U) * f32(1 - 2 ** -20)
    ok = dlb > f32(36) * U * E1 * E1
    with np.errstate(all="ignore"):
        g = E1 / dlb * f32(1 + 2 ** -20)
        d = np.maximum(np.abs(o - K0[:3]), np.abs(o - K1[:3]))
        dist1 = ((d[:, 0] + d[:, 1]) + d[:, 2]) * f32(1 + 2 ** -20)
        r = U * E1 * (f32(8) + g * (f32(168) * dist1 + f32(36) * E1)) * f32(1 + 2 ** -18) + f32(2 ** -100)
        tmax = (dist1 + r) * f32(1 + 2 ** -18)
        et = U * tmax * (f32(53) * E1 * g + f32(8.125)) * f32(1 + 2 ** -18)
        send = np.minimum(best, tmax)
        m = f32(2 ** -16) * (send + et) + f32(2 ** -100)
        s0, s1 = -(et + m), send + et + m
        bmax = np.max(np.abs(np.concatenate([K0[:3], K1[:3]])))
        ex0 = (r + f32(1.01) * m) * f32(1 + 2 ** -20)
        ex = ex0 + f32(2 ** -20) * (bmax + ex0)
        rnd = f32(1) / nd
        t1 = ((K0[:3] - ex[:, None]) - o) * rnd
        t2 = ((K1[:3] + ex[:, None]) - o) * rnd
        lo = np.maximum(s0, np.max(np.minimum(t1, t2), axis=1))
        hi = np.minimum(s1, np.min(np.maximum(t1, t2), axis=1))
    res = ok & (lo > hi) & (best == best)
    return res


def main():
    path = sys.argv[1]
    scene = sys.argv[2] if len(sys.argv) > 2 else "bunny"
    raw = np.fromfile(path, dtype=np.float32).reshape(-1, 14)
    u = raw.view(np.uint32)
    o, nd, best = raw[:, 0:3].copy(), raw[:, 3:6].copy(), raw[:, 9].copy()
    node, cnt = u[:, 10], u[:, 11]
    print(f"{len(raw)} big-leaf visits; leaves {dict(zip(*np.unique(node, return_counts=True)))}")
    rt.set_build_options(leaf_tree_min=9)
    s = rt.Scene()
    s.setup(scene)
    s.build()
    tris, tree, ltris = s.mirror(trees=True)
    T = tree.view(np.uint32)
    # the tree of each big leaf: its root is the lead record's po (pf == 2)
    tri_u = tris.view(np.uint32)
    ha = s.host_arrays()
    nodes_u = ha["nodes"].view(np.uint32).reshape(-1, 8)
    for leaf in np.unique(node):
        sel = node == leaf
        first, count = nodes_u[leaf, 6], nodes_u[leaf, 7]
        root = tri_u[first, 10]
        assert tri_u[first, 11] == 2, "leaf has no tree"
        end = T[root, 13]
        # children of the root: the big triangles (never culled) and the rest's subtree
        kids = []
        c = root + 1
        while c < end:
            kids.append(c)
            c = T[c, 13]
        big = [k for k in kids if not (T[k, 15] & 1) and T[k, 14] != 0xFFFFFFFF]
        rest = [k for k in kids if k not in big]
        print(f"leaf {leaf}: {count} tris, {sum(sel)} visits, root children: {len(big)} big tris + {len(rest)} subtree(s)")
        oo, dd, bb = o[sel], nd[sel], best[sel]

        def frontier(level):
            """the subtree's nodes `level` levels below the rest-root (or clusters above)"""
            fr = list(rest)
            for _ in range(level):
                nxt = []
                for k in fr:
                    if T[k, 14] != 0xFFFFFFFF:
                        nxt.append(k)
                        continue
                    c = k + 1
                    while c < T[k, 13]:
                        nxt.append(c)
                        c = T[c, 13]
                fr = nxt
            return fr

        for level in range(0, 7):
            fr = frontier(level)
            culled = np.ones(len(oo), dtype=bool)
            ntri_left = np.zeros(len(oo))
            for k in fr:
                ck = cull(oo, dd, bb, tree[k]) if (T[k, 15] & 1) else np.zeros(len(oo), dtype=bool)
                culled &= ck
                # triangles under k
                ntri = 0
                for j in range(k, T[k, 13]):
                    if T[j, 14] != 0xFFFFFFFF:
                        ntri += T[j, 15] >> 8
                ntri_left += np.where(ck, 0, ntri)
            print(f"  screen of {len(fr):3d} nodes (level {level}): all culled for {culled.mean():.3f} of visits; "
                  f"triangles left per visit {ntri_left.mean():.1f} of {count}")


if __name__ == "__main__":
    main()
