"""Segment-loop wave cycles by the wave's live pixels (diagnostic; needs the RT_LIVE_HIST build from
`LIVE=1 tools/lane_hist.sh` in place of librt_hip.so): one timing frame, the share of all wave cycles
spent in segment-loop iterations (trace + shade) of waves with 1-8 / 9-16 / 17-32 / more pixels still
live.  Prices merging the tails of the waves of one workgroup: a wave with
few live pixels issues every instruction for 64 lanes.  python tools/live_hist.py [cfg2 ...]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402
import bench  # noqa: E402

rt = G.load_package()
torch.cuda.set_device(0)
for cfg in (sys.argv[1:] or ["cfg2"]):
    scene_name, W, H, SPP, BOUNCES, _ = bench.CONFIGS[cfg]
    scene = rt.Scene()
    scene.setup(scene_name)
    scene.set_viewport(W, H)
    rng = rt.alloc_rng(W * H)
    rt.init_rng_states(rng, W, H, bench.SEED)
    scene.upload(rng.data_ptr())
    a, b = rt.alloc_surface(W, H), rt.alloc_surface(W, H)
    for wps in (5, 7):
        st = torch.zeros(rt.STAT_COUNT, dtype=torch.int64, device="cuda")
        rt.render(scene, a, b, W, H, SPP, BOUNCES, 0, stats=st, tune=256, waves_per_simd=wps)
        torch.cuda.synchronize()
        t = dict(zip(rt.STAT_NAMES, (int(x) for x in st.cpu().numpy())))
        tot, seg = t["cycles_total"], t["cycles_tree_tris"]
        le8, le16, le32 = t["tree_nodes"], t["tree_tri_tests"], t["cycles_tree_clusters"]
        print(json.dumps({"config": cfg, "waves_per_simd": wps, "wave_cycles_total": tot,
                          "segment_loop_frac": round(seg / tot, 4),
                          "live_1_8_frac": round(le8 / tot, 4), "live_9_16_frac": round(le16 / tot, 4),
                          "live_17_32_frac": round(le32 / tot, 4),
                          "live_over_32_frac": round((seg - le8 - le16 - le32) / tot, 4)}), flush=True)
