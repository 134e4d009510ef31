"""A/B parity of a diagnostic tune value: frames rendered with `tune` equal tune 0 bit for bit.
python tools/tune_parity.py TUNE [config ...]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402
import bench  # noqa: E402

rt = G.load_package()

rt.load_experimental()  # A/B and lone / wavefront / refill paths (librt_hip_exp.so)
tune = int(sys.argv[1], 0)
torch.cuda.set_device(0)
for cfg in sys.argv[2:] or ["cfg2"]:
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[cfg]
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    outs = []
    for t in (0, tune):
        rng = rt.alloc_rng(W * H)
        rt.init_rng_states(rng, W, H, bench.SEED)
        scene.upload(rng.data_ptr())
        bufs = [rt.alloc_surface(W, H), rt.alloc_surface(W, H)]
        for f in range(2):
            rt.render(scene, bufs[f & 1], bufs[(f + 1) & 1], W, H, SPP, BOUNCES, f, tune=t)
        torch.cuda.synchronize()
        outs.append((rt.surface_view(bufs[1], W).cpu().numpy().copy(), rng.cpu().numpy().copy()))
    same = np.array_equal(outs[0][0].view(np.uint32), outs[1][0].view(np.uint32)) and np.array_equal(outs[0][1], outs[1][1])
    print(f"{cfg} tune={hex(tune)} bit_equal={same}", flush=True)
    if not same:
        sys.exit(1)
