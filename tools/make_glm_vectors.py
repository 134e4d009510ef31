"""Golden vectors of the reference's own glm (oracle/_ref/libref_glm.so, built from
/root/reference/include/glm by oracle/build_ref.sh): the seeded inputs of tests/glm_cases.py and
glm's outputs for them, written to tests/golden/glm_vectors.npz -- data only (inputs and expected
outputs), so tests/test_oracle_glm.py can pin the oracle where the reference is absent.

    bash oracle/build_ref.sh && python tools/make_glm_vectors.py
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import glm_cases as G  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_glm.so"))
cases = G.make_cases()
out = G.run_all(lib, "ref_", cases)
flat = {}
for k, v in cases.items():
    for j, a in enumerate(v):
        flat[f"in_{k}_{j}"] = a
flat.update({f"out_{k}": v for k, v in out.items()})
np.savez_compressed(os.path.join(ROOT, "tests", "golden", "glm_vectors.npz"), **flat)
print({k: v.shape for k, v in flat.items()})
