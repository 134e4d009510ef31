"""Full-frame oracle fixtures for the BASELINE configs the GPU tests used to check on row bands only
(configs 3 and 4; config 2 too, for completeness): the CPU oracle (oracle/rt_oracle.c, test infrastructure)
renders the whole frame here once, and tests/golden/fullframe_oracle.json keeps a SHA-256 per output row of
the float32 frame, of the final RNG states, and the frame's NaN count -- data, small enough to commit;
tests/test_gpu_fullframe.py::test_full_frame_matches_oracle_fixture renders the same frame on the GPU and
compares row by row (a mismatch names its rows).

    python tools/make_fullframe_golden.py cfg3 cfg4 [cfg2]     (minutes per config on 8 CPUs)"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import rt_testlib as T  # noqa: E402

CONFIGS = {"cfg2": ("bunny", 1920, 1080, 8, 6), "cfg3": ("bunny", 3840, 2160, 64, 6), "cfg4": ("bunny4", 1920, 1080, 8, 6)}
OUT = os.path.join(T.GOLDEN, "fullframe_oracle.json")


def row_hashes(a):
    """SHA-256 (16 hex digits) of every row; NaN values hashed as one canonical quiet NaN: the bit pattern of
    a NaN is not part of the reference's arithmetic (x86 and gfx950 produce different payloads / signs for
    the same invalid operation), its position is."""
    a = np.array(a, copy=True)
    if a.dtype == np.float32:
        a = a.view(np.uint32)
        a[(a & 0x7FFFFFFF) > 0x7F800000] = 0x7FC00000
    return [hashlib.sha256(np.ascontiguousarray(r).tobytes()).hexdigest()[:16] for r in a]


def main():
    db = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for cfg in sys.argv[1:] or ["cfg3", "cfg4"]:
        which, w, h, spp, b = CONFIGS[cfg]
        t0 = time.time()
        rng = T.oracle_rng_frame(T.SEED, w, h, threads=os.cpu_count())
        img = T.OracleScene(which).render(w, h, spp, b, rng=rng, threads=os.cpu_count())
        img = img.reshape(h, w, 4)
        db[cfg] = {"scene": which, "width": w, "height": h, "spp": spp, "bounces": b, "seed": T.SEED, "frame_index": 0,
                   "rows": row_hashes(img), "rng_rows": row_hashes(rng.reshape(h, w, 6)),
                   "nan_values": int(np.isnan(img).sum()), "oracle_s": round(time.time() - t0, 1),
                   "generator": "tools/make_fullframe_golden.py (oracle/rt_oracle.c, CPU)"}
        print(cfg, db[cfg]["oracle_s"], "s", db[cfg]["nan_values"], "NaN", flush=True)
        with open(OUT, "w") as fh:
            json.dump(db, fh, separators=(",", ":"))


if __name__ == "__main__":
    main()
