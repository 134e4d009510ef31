"""Where the small phase's wave cycles go by active-lane count (diagnostic; needs the RT_LANE_HIST
build from tools/lane_hist.sh in place of librt_hip.so): one timing frame, per-wave s_memtime cycles
of small-step iterations with 1-4 / 5-16 / more active lanes and of lone-lane traversals, as fractions
of all wave cycles.  python tools/lane_hist.py [cfg2]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402
import bench  # noqa: E402

rt = G.load_package()

rt.load_experimental()  # A/B and lone / wavefront / refill paths (librt_hip_exp.so)
cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[cfg]
torch.cuda.set_device(0)
scene = rt.Scene()
scene.setup(scene_name)
scene.set_viewport(W, H)
rng = rt.alloc_rng(W * H)
rt.init_rng_states(rng, W, H, bench.SEED)
scene.upload(rng.data_ptr())
a, b = rt.alloc_surface(W, H), rt.alloc_surface(W, H)
for wps in (0, 7):
    st = torch.zeros(rt.STAT_COUNT, dtype=torch.int64, device="cuda")
    rt.render(scene, a, b, W, H, SPP, BOUNCES, 0, stats=st, tune=256, waves_per_simd=wps)
    torch.cuda.synchronize()
    v = [int(x) for x in st.cpu().numpy()]
    total, small = v[18], v[16]
    it_all, lone, le4, le16 = v[22], v[23], v[14], v[15]
    print(json.dumps({"config": cfg, "waves_per_simd": wps or 5, "wave_cycles_total": total,
                      "small_phase_frac": round(small / total, 3),
                      "iters_1_4_lanes_frac": round(le4 / total, 3), "iters_5_16_lanes_frac": round(le16 / total, 3),
                      "iters_over_16_lanes_frac": round((it_all - le4 - le16) / total, 3),
                      "lone_lane_traversal_frac": round(lone / total, 3)}), flush=True)
