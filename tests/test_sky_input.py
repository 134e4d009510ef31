"""Sky input: the product's C++ DDS reader (csrc/scene.cpp load_cube, which
restates utils/image/DDSLoader.cpp:135-371 and the face slicing of utils/CUDATexture.cpp:187-220)
loads the reference's own data/sunset_uncompressed.dds through rt_scene_set_environment_file, and
its level-0 texels equal assets/sunset_cube128.bin byte for byte (the asset the tests, smoke()
and the benchmark render with; made by tools/make_assets.py).

The DDS file lives in /root/reference (the development container only; skipped elsewhere).  CPU.
"""
import os

import numpy as np
import pytest

import rt_testlib as T

DDS = "/root/reference/data/sunset_uncompressed.dds"


def _env(rt, path):
    s = rt.Scene()
    s.set_environment(path)
    return s.environment()


@pytest.mark.skipif(not os.path.exists(DDS), reason="reference data not present")
def test_dds_reader_matches_asset():
    rt = T.load_rt()
    dds = _env(rt, DDS)
    asset = _env(rt, os.path.join(T.ASSETS, "sunset_cube128.bin"))
    assert dds.shape == asset.shape == (6, 128, 128, 4)
    assert np.array_equal(dds.view(np.uint32), asset.view(np.uint32))
    # faces differ from each other (+X,-X,+Y,-Y,+Z,-Z order kept, not six copies of one face)
    assert len({dds[f].tobytes() for f in range(6)}) == 6


def test_environment_file_errors():
    rt = T.load_rt()
    s = rt.Scene()
    assert s.environment() is None
    with pytest.raises(rt.RTError):
        s.set_environment(os.path.join(T.ASSETS, "does_not_exist.dds"))
    with pytest.raises(rt.RTError):
        s.set_environment(os.path.join(T.ASSETS, "bunny_mesh.bin"))  # not a cube map
