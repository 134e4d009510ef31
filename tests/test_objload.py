"""OBJ input (cuda-raytracing_amd/csrc/objload.cpp) against the assimp 3.3 import of the
reference's data/stanford-bunny.obj (assets/bunny_mesh.bin, made by tools/make_assets.py):
the reference's Scene::AddLoadedScene (RayTracing/Scene.cpp:75-132) receives the same vertex
positions, vertex order and faces bit for bit, and normals within a few ulps (the smoothing
sum's order follows assimp's internal sort of tied SpatialSort entries, not reproduced).

Reads the OBJ from /root/reference (the survey container only; skipped elsewhere).  CPU only.
"""
import os

import numpy as np
import pytest

import rt_testlib as T

OBJ = "/root/reference/data/stanford-bunny.obj"
pytestmark = pytest.mark.skipif(not os.path.exists(OBJ), reason="reference data not present")


def _scene(rt, path):
    s = rt.Scene()
    s.add_loaded_scene(path, np.eye(4, dtype=np.float32).reshape(-1).tolist(), 0)
    s.build()
    a = s.host_arrays()
    v = np.frombuffer(a["vertices"].tobytes(), dtype=np.float32).reshape(-1, 8)
    f = np.frombuffer(a["faces"].tobytes(), dtype=np.uint32).reshape(-1, 4)
    return v, f


def test_obj_matches_assimp_import():
    rt = T.load_rt()
    va, fa = _scene(rt, os.path.join(T.ROOT, "assets", "bunny_mesh.bin"))
    vo, fo = _scene(rt, OBJ)
    assert va.shape == vo.shape and fa.shape == fo.shape
    # AddLoadedScene: the indexed (smooth) copy first, then the flat copies
    assert np.array_equal(fa, fo)
    assert np.array_equal(va[:, 0:3], vo[:, 0:3])  # positions (transformed) bit for bit
    assert np.array_equal(va[:, 6:8], vo[:, 6:8])
    d = np.abs(va[:, 3:6] - vo[:, 3:6])  # smooth normals (unnormalised, x the transform)
    scale = np.abs(va[:, 3:6]).max()
    assert d.max() <= 4e-7 * max(1.0, scale), d.max()
