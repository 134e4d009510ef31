"""Phase clocks of one frame (timing variant of the production kernel, RT_TUNE bit 8): wave cycles
in small steps (inner nodes / small leaves), big-leaf rounds, and the rest (shading, sky, RNG,
output), summed over waves.  python tools/phase_clocks.py [cfg2] [waves per SIMD] [extra RT_TUNE bits]"""
import json
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
scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "cfg2"]
torch.cuda.set_device(0)
scene = rt.Scene()
scene.setup(scene_name)
scene.set_viewport(W, H)
rng = rt.alloc_rng(W * H)
rt.init_rng_states(rng, W, H, bench.SEED)
scene.upload(rng.data_ptr())
a, b = rt.alloc_surface(W, H), rt.alloc_surface(W, H)
st = torch.zeros(rt.STAT_COUNT, dtype=torch.int64, device="cuda")
wps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
extra = int(sys.argv[3], 0) if len(sys.argv) > 3 else 0
rt.render(scene, a, b, W, H, SPP, BOUNCES, 0, stats=st, tune=256 | ({6: 2, 7: 3}.get(wps, 0) << 9) | extra)
torch.cuda.synchronize()
v = st.cpu().numpy()
small, big, total = int(v[16]), int(v[17]), int(v[18])
print(json.dumps({"config": sys.argv[1] if len(sys.argv) > 1 else "cfg2", "waves_per_simd": wps or 5, "tune_extra": hex(extra),
                  "wave_cycles_total": total,
                  "small_frac": round(small / total, 3), "big_frac": round(big / total, 3),
                  "rest_frac": round(1 - (small + big) / total, 3), "rounds_coop": int(v[19]), "rounds_shared": int(v[20]),
                  "coop_rays": int(v[21]), "wave_small_iters": int(v[8]), "lane_small": int(v[9]),
                  "small_lanes_per_iter": round(int(v[9]) / max(1, int(v[8])), 2),
                  "tree_walk_frac": round(int(v[7]) / total, 3), "tree_cluster_frac": round(int(v[22]) / total, 3),
                  "tree_tri_frac": round(int(v[23]) / total, 3), "tree_tests": int(v[14]), "wave_big_rounds": int(v[10]),
                  "lane_big": int(v[11])}))
