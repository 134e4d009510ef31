"""Generate tests/golden/golden.json from the CPU oracle (oracle/rt_oracle.c).

The reference ships no tests or golden outputs and cannot be built here (DESIGN.md,
"Parity"), so these fixtures pin the oracle itself: any later change to the oracle, the
product host code or the kernel that moves a single bit of these outputs fails a test.
Run from the repo root after building: python tools/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import rt_testlib as T  # noqa: E402


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    g = {"seed": T.SEED}
    o = T.OracleScene("bunny")
    arr = o.arrays()
    g["bunny_scene"] = {k: sha(arr[k]) for k in ("vertices", "faces", "nodes", "face_indices", "spheres", "materials")}
    g["bunny_scene"]["counts"] = {"vertices": len(arr["vertices"]) // 32, "faces": len(arr["faces"]) // 16,
                                  "nodes": len(arr["nodes"]) // 32, "max_depth": arr["max_depth"],
                                  "spheres": len(arr["spheres"]) // 32, "materials": len(arr["materials"]) // 64}
    g["camera_1920x1080"] = [float(x) for x in o.camera(1920, 1080)]
    g["camera_256x256"] = [float(x) for x in o.camera(256, 256)]
    # RNG known answers (SURVEY.md 8(c) fixture list)
    ids = [0, 1, 2, 127, 128, 1920 * 1080 - 1, 3840 * 2160 - 1]
    g["rng_states"] = {str(i): [int(x) for x in T.oracle_rng_state(T.SEED, i)] for i in ids}
    draws = np.zeros(16, dtype=np.float32)
    st = T.oracle_rng_state(T.SEED, 0)
    T.oracle().oracle_rng_draws(st.ctypes.data_as(T.ctypes.POINTER(T.ctypes.c_uint32)), 16,
                                draws.ctypes.data_as(T.ctypes.POINTER(T.ctypes.c_float)))
    g["rng_pixel0_first16"] = [float(x) for x in draws]
    # images
    for name, (w, h, spp, b) in {"cfg1_256x256_s1_b1": (256, 256, 1, 1), "small_64x36_s8_b6": (64, 36, 8, 6),
                                 "small_48x32_s2_b6_f3": (48, 32, 2, 6)}.items():
        frames = 3 if name.endswith("_f3") else 1
        rng = T.oracle_rng_frame(T.SEED, w, h)
        last, shas = None, []
        for f in range(frames):
            img, stt = o.render(w, h, spp, b, frame_index=f, rng=rng, last=last, stats=True)
            shas.append(sha(img))
            last = img
        g[name] = {"sha256": shas, "stats": [int(x) for x in stt[:7]], "mean_rgb": [float(x) for x in img[..., :3].mean((0, 1))],
                   "crop_8x8_rgb": img[h // 2:h // 2 + 8, w // 2:w // 2 + 8, :3].round(6).tolist(),
                   "rng_sha256": sha(rng)}
    for which in ("bunny4",):
        a = T.OracleScene(which).arrays()
        g[which + "_scene"] = {"vertices": len(a["vertices"]) // 32, "faces": len(a["faces"]) // 16,
                               "nodes": len(a["nodes"]) // 32, "max_depth": a["max_depth"],
                               "nodes_sha256": sha(a["nodes"]), "face_indices_sha256": sha(a["face_indices"])}
    json.dump(g, open(os.path.join(T.GOLDEN, "golden.json"), "w"), indent=1)
    print("wrote", os.path.join(T.GOLDEN, "golden.json"))


if __name__ == "__main__":
    main()
