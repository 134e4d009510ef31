"""The C-ABI boundary: librt_hip.so loads, exports every symbol include/rt_abi.h declares,
and its structs have the reference's sizes.  No GPU work."""
import ctypes
import os
import re

import rt_testlib as T

HEADER = os.path.join(T.ROOT, "include", "rt_abi.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w\s\*]*?\b([a-z_][a-z0-9_]*)\s*\(", text, flags=re.M)
    return sorted(set(n for n in names if n not in ("static_assert", "sizeof", "offsetof")))


def test_every_declared_symbol_is_exported():
    rt = T.load_rt()
    L = rt.lib()
    names = declared_functions()
    assert "raytracing_process" in names and "init_rng" in names and "rt_render" in names
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # and the Python binding covers the same surface
    assert not (set(names) - set(rt.SIGNATURES)), set(names) - set(rt.SIGNATURES)


def test_struct_layouts():
    rt = T.load_rt()
    assert ctypes.sizeof(rt.GPUScene) == 136
    assert rt.GPUScene.camera.offset == 72 and rt.GPUScene.rng_state.offset == 56
    assert rt.GPUScene.environment_cubemap_tex.offset == 64 and rt.GPUScene.sphere_count.offset == 48
    assert ctypes.sizeof(rt.GPUCamera) == 60
    assert ctypes.sizeof(rt.GPUMaterial) == 64 and rt.GPUMaterial.roughness.offset == 48


def test_error_paths_without_gpu():
    rt = T.load_rt()
    L = rt.lib()
    p = rt.RenderParams()
    assert L.rt_render(ctypes.byref(p), None, None) != 0
    assert b"null" in L.rt_last_error()
    p.width, p.height, p.spp, p.bounces, p.shard_count = 16, 16, 1, 1, 1
    scene = rt.GPUScene()
    assert L.rt_render(ctypes.byref(p), ctypes.byref(scene), None) != 0  # no surface
    assert L.rt_init_rng(None, 4, 4, 0, 1, 1, None) != 0
    assert L.rt_cubemap_create(None, 4) == 0


def test_shard_tiles():
    rt = T.load_rt()
    w, h = 1920, 1080
    tiles = (w // 16) * ((h + 15) // 16)
    for n in (1, 2, 3, 7, 8):
        counts = [rt.shard_tiles(w, h, r, n) for r in range(n)]
        assert sum(counts) == tiles and max(counts) - min(counts) <= 1
    assert rt.shard_tiles(w, h, 8, 8) == 0


def test_experimental_paths_live_in_the_plugin():
    """librt_hip.so carries only the kernels the production path launches; the exact alternatives
    kept for A/B measurement (wavefront tracer, refill, lone-pixel kernel, RT_TUNE A/B variants) are in
    librt_hip_exp.so, whose loading registers them (rt_experimental_loaded).  Checked in a child
    process so the registration starts from a clean slate."""
    import subprocess
    import sys

    code = ("import sys, importlib; sys.path.insert(0, %r); rt = importlib.import_module('cuda-raytracing_amd'); "
            "a = rt.lib().rt_experimental_loaded(); rt.load_experimental(); "
            "print(a, rt.lib().rt_experimental_loaded())") % T.ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split() == ["0", "1"]
    nm = lambda p: subprocess.run(["nm", "-DC", p], capture_output=True, text=True).stdout
    rt = T.load_rt()
    prod, exp = nm(rt.LIB_PATH), nm(rt.EXP_LIB_PATH)
    for k in ("launch_lone", "launch_wavefront", "launch_fast_refill", "launch_fast_ab"):
        assert f"rtk::{k}(" not in prod and f"rtk::{k}(" in exp, k
    assert "rtk::launch_fast_prod(" in prod
