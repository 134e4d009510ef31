"""The drop-in boundary from C++: tests/cpp/host_driver.cpp links librt_hip.so through
include/rt_abi.h and drives it the way the reference's CUDARayTracer drives its kernels
(RayTracing/RayTracing.cpp:205-234: init_rng over ceil(W*H/128) blocks of 128 states, Scene::Upload,
then per frame raytracing_process + the D2D copy into the last frame).  The frames it produces are
compared with the CPU oracle bit for bit (spp 5, 6 bounces: the reference's compiled constants).
"""
import os
import subprocess

import numpy as np
import pytest

import rt_testlib as T

DRIVER = os.path.join(T.ROOT, "tests", "cpp", "host_driver")


def test_host_driver_built():
    assert os.path.exists(DRIVER), "build() compiles tests/cpp/host_driver.cpp"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["single", "split"])
def test_cpp_host_progressive_frames(tmp_path, mode):
    """single: the reference's call pattern; split: the same frames over every visible device
    (rt_shard_plan + rt_render shards + rt_gather_shards over RCCL + rt_unshard_tiles)."""
    w, h, frames = 48, 32, 2
    out = tmp_path / "frame.bin"
    r = subprocess.run([DRIVER, str(out), str(w), str(h), str(frames), os.path.join(T.ROOT, "assets"), mode],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.fromfile(out, dtype=np.float32).reshape(h, w, 4)
    o = T.OracleScene("bunny")
    rng = T.oracle_rng_frame(T.SEED, w, h)
    last = None
    for f in range(frames):
        last = o.render(w, h, 5, 6, frame_index=f, rng=rng, last=last)
    assert np.array_equal(got.view(np.uint32), last.view(np.uint32)), float(np.nanmax(np.abs(got - last)))
