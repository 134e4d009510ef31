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
