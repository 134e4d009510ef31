"""Which kernel variants agree bit for bit: one frame of a scene at every occupancy (waves per SIMD)
x every RT_TUNE value given, frames and RNG states compared against the first combination.

    python tools/variant_agree.py bunny4 256 144 "0 0x8000000 0x10000000" "5 6 7"
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import rt_testlib as T  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "bunny4"
w, h = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (256, 144)
tunes = [int(x, 0) for x in (sys.argv[4] if len(sys.argv) > 4 else "0").split()]
occs = [int(x) for x in (sys.argv[5] if len(sys.argv) > 5 else "5 6 7").split()]
spp = int(os.environ.get("SPP", "4"))
rt = T.load_rt()
rt.load_experimental()  # A/B variants (librt_hip_exp.so)
if os.environ.get("BUILD_OPTS"):  # e.g. "leaf_screens=0" (rt_set_build_options)
    rt.set_build_options(**{k: float(v) if k == "split_angle" else int(v)
                            for k, v in (kv.split("=") for kv in os.environ["BUILD_OPTS"].split(","))})
torch.cuda.set_device(0)
res = []
for t in tunes:
    for o in occs:
        s = rt.Scene()
        s.setup(which)
        s.set_viewport(w, h)
        rng = rt.alloc_rng(w * h)
        rt.init_rng_states(rng, w, h, T.SEED)
        s.upload(rng.data_ptr())
        out, last = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
        rt.render(s, out, last, w, h, spp, 6, 0, waves_per_simd=o, tune=t)
        torch.cuda.synchronize()
        res.append(((t, o), rt.surface_view(out, w).cpu().numpy().copy(), rng.view(-1, 12)[:, :6].cpu().numpy().copy()))
if os.environ.get("ORACLE"):  # the CPU oracle's frame first (the reference for every combination)
    res.insert(0, (("oracle", 0), T.OracleScene(which).render(w, h, spp, 6), None))
_, b_img, b_st = res[0]
for k, img, st in res:
    diff = np.flatnonzero((img.view(np.uint32) != b_img.view(np.uint32)).any(-1).ravel())
    print(json.dumps({"scene": which, "tune": k[0] if isinstance(k[0], str) else hex(k[0]), "wps": k[1], "pixels_differ": int(diff.size),
                      "rng_differ": int((st != b_st).any(-1).sum()) if st is not None and b_st is not None else None,
                      "first": [[int(p % w), int(p // w)] for p in diff[:5]]}), flush=True)
