"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle, bit for bit.

Tolerance: the north star allows |delta RGB| <= 1e-4 per pixel; the kernel and the oracle use
the same IEEE fp32 operation order without contraction, so these tests expect and assert
EXACT equality wherever the oracle can run (and report the max |delta| on failure).
"""
import numpy as np
import pytest
import torch

import rt_testlib as T

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope="module")
def rt():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    torch.cuda.set_device(0)
    return T.load_rt()


def make_scene(rt, which, w, h, plane_n=None):
    s = rt.Scene()
    if plane_n:
        s.setup_plane(plane_n)
    else:
        s.setup(which)
    s.set_viewport(w, h)
    return s


def gpu_render(rt, which, w, h, spp, bounces, frames=1, plane_n=None, seed=T.SEED, stats=False, tracer="fast"):
    s = make_scene(rt, which, w, h, plane_n)
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, seed)
    s.upload(rng.data_ptr())
    a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
    st = torch.zeros(rt.STAT_COUNT, dtype=torch.int64, device="cuda") if stats else None
    outs = []
    for f in range(frames):
        cur, prev = (a, b) if f % 2 == 0 else (b, a)
        rt.render(s, cur, prev, w, h, spp, bounces, frame_index=f, stats=st, tracer=tracer)
        outs.append(rt.surface_view(cur, w).cpu().numpy().copy())
    torch.cuda.synchronize()
    res = {"frames": outs, "rng": rng.view(-1, 12)[:, :6].cpu().numpy().view(np.uint32).copy()}
    if stats:
        res["stats"] = st.cpu().numpy().astype(np.uint64)
    return res


def oracle_render(which, w, h, spp, bounces, frames=1, plane_n=708, seed=T.SEED):
    o = T.OracleScene(which, grid_n=plane_n)
    rng = T.oracle_rng_frame(seed, w, h)
    outs, last, st = [], None, None
    for f in range(frames):
        img, st = o.render(w, h, spp, bounces, frame_index=f, rng=rng, last=last, stats=True)
        outs.append(img)
        last = img
    return {"frames": outs, "rng": rng, "stats": st}


def assert_close(got, want, what):
    d = np.abs(got.astype(np.float64) - want.astype(np.float64))
    mism = int((got != want).sum())
    assert np.isfinite(got).all(), f"{what}: non-finite output"
    assert d.max() <= TOL, f"{what}: max |GPU - oracle| = {d.max():.3g} ({mism} differing values)"
    assert mism == 0, f"{what}: {mism} values differ (max {d.max():.3g}) -- expected bit-exact"


def test_init_rng_matches_oracle(rt):
    w, h = 61, 37  # ragged: not a multiple of the 16x16 tile
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    got = rng.view(-1, 12)[:, :6].cpu().numpy().view(np.uint32)
    want = T.oracle_rng_frame(T.SEED, w, h)
    assert np.array_equal(got, want)


def test_init_rng_reference_entry_point(rt):
    # init_rng(thread_block_count, thread_block_size, states, seed) -- Random.cu:10; large ids too
    blocks, bs = 40, 128
    rng = rt.alloc_rng(blocks * bs)
    rt.init_rng(blocks, bs, rng, 12345)
    torch.cuda.synchronize()
    got = rng.view(-1, 12)[:, :6].cpu().numpy().view(np.uint32)
    for i in (0, 1, 2, 127, 128, blocks * bs - 1):
        assert np.array_equal(got[i], T.oracle_rng_state(12345, i)), i


@pytest.mark.parametrize("tracer", ["fast", "flat", "ref"])
@pytest.mark.parametrize("spp,bounces", [(1, 1), (4, 6), (8, 6)])
def test_render_bunny_small(rt, spp, bounces, tracer):
    """Every kernel variant (production fast path, exact-division flat path, reference-layout
    path) against the oracle, including the traversal counts."""
    w, h = 64, 36
    g = gpu_render(rt, "bunny", w, h, spp, bounces, stats=True, tracer=tracer)
    o = oracle_render("bunny", w, h, spp, bounces)
    assert_close(g["frames"][0], o["frames"][0], f"bunny {w}x{h} spp{spp} b{bounces}")
    assert np.array_equal(g["rng"], o["rng"]), "final RNG states differ"
    assert np.array_equal(g["stats"][:7], o["stats"][:7]), (g["stats"][:7], o["stats"][:7])


def test_render_config1_vs_golden(rt):
    """BASELINE configs[0]: 256x256, 1 spp, primary rays only -- against the committed golden
    hash and traversal counts, and the live oracle."""
    import hashlib
    import json
    gold = json.load(open(T.GOLDEN + "/golden.json"))["cfg1_256x256_s1_b1"]
    g = gpu_render(rt, "bunny", 256, 256, 1, 1, stats=True)
    o = oracle_render("bunny", 256, 256, 1, 1)
    assert_close(g["frames"][0], o["frames"][0], "config 1 vs oracle")
    assert hashlib.sha256(g["frames"][0].tobytes()).hexdigest() == gold["sha256"][0]
    assert [int(x) for x in g["stats"][:7]] == gold["stats"]


def test_progressive_frames(rt):
    w, h = 48, 32
    g = gpu_render(rt, "bunny", w, h, 2, 6, frames=3)
    o = oracle_render("bunny", w, h, 2, 6, frames=3)
    for f in range(3):
        assert_close(g["frames"][f], o["frames"][f], f"frame {f}")


def test_reference_entry_point_raytracing_process(rt):
    """raytracing_process(surface, last, w, h, pitch, frame, scene): spp 5, 6 bounces."""
    w, h = 40, 24
    s = make_scene(rt, "bunny", w, h)
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
    rt.raytracing_process(a, b, w, h, 0, s)
    torch.cuda.synchronize()
    o = oracle_render("bunny", w, h, 5, 6)
    assert_close(rt.surface_view(a, w).cpu().numpy(), o["frames"][0], "raytracing_process")


def test_sharded_equals_full(rt):
    """Tile sharding over N ranks + unshard reproduces the single-GPU frame byte for byte."""
    w, h, spp, bounces = 80, 50, 2, 6
    full = gpu_render(rt, "bunny", w, h, spp, bounces)["frames"][0]
    for n in (2, 3, 8):
        s = make_scene(rt, "bunny", w, h)
        per = max(rt.shard_tiles(w, h, r, n) for r in range(n))
        shards = torch.zeros((n, per * 256, 4), dtype=torch.float32, device="cuda")
        for r in range(n):
            rng = rt.alloc_rng(per * 256)
            rt.init_rng_states(rng, w, h, T.SEED, r, n)
            s.upload(rng.data_ptr())
            last = torch.zeros((per * 256, 4), dtype=torch.float32, device="cuda")
            rt.render(s, None, last, w, h, spp, bounces, 0, r, n, out_shard=shards[r])
            torch.cuda.synchronize()
        out = rt.alloc_surface(w, h)
        rt.unshard(out, w, h, n, shards, per)
        torch.cuda.synchronize()
        assert np.array_equal(rt.surface_view(out, w).cpu().numpy(), full), f"shards={n}"


def test_four_bunnies_small(rt):
    g = gpu_render(rt, "bunny4", 40, 24, 2, 6)
    o = oracle_render("bunny4", 40, 24, 2, 6)
    assert_close(g["frames"][0], o["frames"][0], "bunny4")


def test_plane_grid_small(rt):
    g = gpu_render(rt, "plane1m", 40, 24, 1, 6, plane_n=64)
    o = oracle_render("plane1m", 40, 24, 1, 6, plane_n=64)
    assert_close(g["frames"][0], o["frames"][0], "plane grid 64")


@pytest.mark.parametrize("which,plane_n", [("bunny", None), ("bunny4", None), ("plane1m", 200)])
def test_tracers_agree_medium(rt, which, plane_n):
    """256x144, 4 spp, 6 bounces: the three kernel variants produce identical frames and RNG
    states (a larger sample of rays than the oracle comparisons above)."""
    res = {t: gpu_render(rt, which, 256, 144, 4, 6, plane_n=plane_n, stats=True, tracer=t)
           for t in ("fast", "flat", "ref")}
    for t in ("flat", "ref"):
        assert np.array_equal(res["fast"]["frames"][0], res[t]["frames"][0]), t
        assert np.array_equal(res["fast"]["rng"], res[t]["rng"]), t
        assert np.array_equal(res["fast"]["stats"][:7], res[t]["stats"][:7]), t
    # the production kernel without statistics (pair records, cooperative rounds)
    g = gpu_render(rt, which, 256, 144, 4, 6, plane_n=plane_n)
    assert np.array_equal(g["frames"][0], res["ref"]["frames"][0])
    assert np.array_equal(g["rng"], res["ref"]["rng"])


def test_full_size_config2_properties(rt):
    """Config 2 at full size: finite, alpha 1, deterministic, and oracle-exact on sampled rows."""
    w, h, spp, bounces = 1920, 1080, 8, 6
    g1 = gpu_render(rt, "bunny", w, h, spp, bounces)["frames"][0]
    g2 = gpu_render(rt, "bunny", w, h, spp, bounces)["frames"][0]
    assert np.isfinite(g1).all() and (g1[..., 3] == 1.0).all()
    assert np.array_equal(g1, g2), "render is not deterministic"
    o = T.OracleScene("bunny")
    for r0 in (0, 517, 1064):
        want = o.render(w, h, spp, bounces, rows=(r0, r0 + 16))
        assert_close(g1[r0:r0 + 16], want, f"config 2 rows {r0}..{r0 + 16}")


def _dev_copy(rt, src_ptr, nbytes):
    """A fresh hipMalloc'd copy (as the reference's CUDA::DeviceMemory would hold)."""
    import ctypes
    p = ctypes.c_void_p()
    assert rt.lib().rt_malloc(ctypes.byref(p), nbytes) == 0
    assert rt.lib().rt_memcpy_d2d(p, ctypes.c_void_p(src_ptr), nbytes) == 0
    return p


def test_foreign_gpuscene(rt):
    """A GPUScene filled by another host (the reference's own Scene::Upload) -- no mirror was
    registered for it.  No call waits for the device: the first frames render through the
    reference layout while a worker thread builds the mirror; once installed, frames whose arrays
    match its fingerprint run the production tracer; an in-place change of the arrays is caught by
    the device-side fingerprint of that very frame (reference layout again) and rebuilt."""
    import ctypes
    w, h = 64, 36
    s = make_scene(rt, "bunny", w, h)
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    rng0 = rng.clone()
    ha = s.host_arrays()
    g = s.gpu.contents
    sizes = {"gpu_bvh_nodes": ha["nodes"].nbytes, "gpu_bvh_face_indices": ha["face_indices"].nbytes,
             "gpu_vertices": ha["vertices"].nbytes, "gpu_faces": ha["faces"].nbytes,
             "gpu_spheres": 32 * g.sphere_count, "gpu_materials": 64 * g.material_count}
    f = rt.GPUScene()
    ctypes.pointer(f)[0] = g
    owned = {}
    for k, n in sizes.items():
        owned[k] = _dev_copy(rt, getattr(g, k), n)
        setattr(f, k, owned[k].value)
    frng = rng.clone()
    f.rng_state = frng.data_ptr()
    try:
        def frame(scene, rng_buf, tracer="fast"):
            rng_buf.copy_(rng0)
            a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
            rt.render(scene, a, b, w, h, 2, 6, tracer=tracer)
            torch.cuda.synchronize()
            return rt.surface_view(a, w).cpu().numpy().copy()

        ref = frame(s, rng)
        assert np.array_equal(frame(f, frng), ref)
        assert rt.foreign_last_tracer(f) == -1  # no mirror yet: reference layout
        rt.foreign_mirror_wait(f)
        assert np.array_equal(frame(f, frng), ref)  # installs the mirror, fingerprint matches
        assert rt.foreign_last_tracer(f) == 1
        assert np.array_equal(frame(f, frng), ref)
        assert rt.foreign_last_tracer(f) == 1
        # move every vertex in place (same buffer, same size): this very frame must notice
        vert = ha["vertices"].copy().view(np.float32).reshape(-1, 8)
        vert[:, 0] += np.float32(0.75)
        src = torch.from_numpy(vert.reshape(-1).copy()).cuda()
        assert rt.lib().rt_memcpy_d2d(owned["gpu_vertices"], ctypes.c_void_p(src.data_ptr()), vert.nbytes) == 0
        torch.cuda.synchronize()
        moved_ref = frame(f, frng, tracer="ref")
        moved = frame(f, frng)
        assert rt.foreign_last_tracer(f) == 0  # stale mirror: the reference layout rendered it
        assert not np.array_equal(moved, ref)
        assert np.array_equal(moved, moved_ref)
        frame(f, frng)  # the mismatch has reached the host: a rebuild starts
        rt.foreign_mirror_wait(f)
        assert np.array_equal(frame(f, frng), moved_ref)
        assert rt.foreign_last_tracer(f) == 1  # rebuilt mirror in use
    finally:
        torch.cuda.synchronize()
        for p in owned.values():
            rt.lib().rt_free(p)


def test_nan_pixel_tile(rt):
    """A pixel whose reference arithmetic yields NaN: (1062, 756) of the 2720x1530 frame (the
    2-GPU weak-scaled bench frame) goes NaN in frame 0, in the oracle as on the GPU.  Only its
    16x16 tile is rendered (a one-tile shard: shard_count = tiles, shard_index = that tile),
    two progressive frames: the same values bit for bit and NaN in the same places (a NaN's
    payload bits are the ISA's choice: x86 and the GPU differ, as the reference's would)."""
    w, h, spp, bounces, px, py = 2720, 1530, 8, 6, 1062, 756
    tiles_x = (w + 15) // 16
    n = tiles_x * ((h + 15) // 16)
    tile = (py // 16) * tiles_x + px // 16
    s = make_scene(rt, "bunny", w, h)
    rng = rt.alloc_rng(256)
    rt.init_rng_states(rng, w, h, T.SEED, tile, n)
    s.upload(rng.data_ptr())
    bufs = [torch.zeros((256, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
    o = T.OracleScene("bunny")
    orng = T.oracle_rng_frame(T.SEED, w, h)
    last = None
    y0, x0 = (py // 16) * 16, (px // 16) * 16
    xs, ys = rt.sharding.slot_pixels(w, h, tile, n)
    for f in range(2):
        rt.render(s, None, bufs[(f + 1) & 1], w, h, spp, bounces, f, tile, n, out_shard=bufs[f & 1])
        torch.cuda.synchronize()
        got = bufs[f & 1].cpu().numpy()
        img = o.render(w, h, spp, bounces, frame_index=f, rng=orng, last=last, rows=(y0, y0 + 16))
        last = img
        want = img[ys - y0, xs]
        assert not np.isfinite(want[(ys == py) & (xs == px)]).all(), "expected the reference NaN pixel"
        nan_g, nan_w = np.isnan(got), np.isnan(want)
        assert np.array_equal(nan_g, nan_w), f"frame {f}: NaN positions differ"
        assert np.array_equal(got[~nan_g].view(np.uint32), want[~nan_w].view(np.uint32)), f"frame {f}: tile differs"


def _tile_shard(rt, scene, w, h, spp, bounces, px, py, frame_index=0, last=None):
    """Render only the 16x16 tile holding pixel (px, py) of a w x h frame: a one-tile shard
    (shard_count = tiles, shard_index = that tile), fresh RNG.  Returns (slots float4 [256],
    slot x, slot y)."""
    tiles_x = (w + 15) // 16
    n = tiles_x * ((h + 15) // 16)
    tile = (py // 16) * tiles_x + px // 16
    rng = rt.alloc_rng(256)
    rt.init_rng_states(rng, w, h, T.SEED, tile, n)
    scene.upload(rng.data_ptr())
    out = torch.zeros((256, 4), dtype=torch.float32, device="cuda")
    rt.render(scene, None, last, w, h, spp, bounces, frame_index, tile, n, out_shard=out)
    torch.cuda.synchronize()
    xs, ys = rt.sharding.slot_pixels(w, h, tile, n)
    return out.cpu().numpy(), xs, ys


@pytest.mark.parametrize("cfg,which,w,h,spp,picks", [
    # BASELINE configs[2]: 4K, 64 spp -- tiles on the bunny, in the box (spheres), on the floor
    ("config3", "bunny", 3840, 2160, 64, [(900, 1400), (1920, 1300), (2600, 1950)]),
    # configs[3]: the 4-bunny scene (leaf trees in the production kernel)
    ("config4", "bunny4", 1920, 1080, 8, [(200, 700), (520, 860), (960, 540)]),
    # configs[4]: the 1M-triangle plane (708 x 708 quads)
    ("config5", "plane1m", 1920, 1080, 1, [(7, 3), (960, 540), (1900, 1070)]),
])
def test_full_size_tiles(rt, cfg, which, w, h, spp, picks):
    """Full-size BASELINE configurations, tiles rendered alone through the shard path and
    compared bit for bit with the oracle's rendering of the rows that hold them."""
    s = make_scene(rt, which, w, h)
    o = T.OracleScene(which)
    for px, py in picks:
        got, xs, ys = _tile_shard(rt, s, w, h, spp, 6, px, py)
        y0 = (py // 16) * 16
        rows = min(16, h - y0)
        want = o.render(w, h, spp, 6, rows=(y0, y0 + rows))
        ok = xs >= 0
        assert_close(got[ok], want[ys[ok] - y0, xs[ok]], f"{cfg} tile at ({px}, {py})")


@pytest.mark.parametrize("which,plane_n", [("bunny", None), ("bunny4", None)])
def test_occupancy_variants_agree(rt, which, plane_n):
    """The production kernel at 5, 6 and 7 waves per SIMD (rt_render_params.waves_per_simd: the
    compiler spills differently, the arithmetic is the same) and the 5-wave build with its residency
    capped at 2 waves per SIMD by dynamic LDS render identical frames and states."""
    w, h, res = 256, 144, {}
    for wps in (5, 6, 7, 2):
        s = make_scene(rt, which, w, h, plane_n)
        rng = rt.alloc_rng(w * h)
        rt.init_rng_states(rng, w, h, T.SEED)
        s.upload(rng.data_ptr())
        out, last = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
        rt.render(s, out, last, w, h, 4, 6, 0, waves_per_simd=wps)
        torch.cuda.synchronize()
        res[wps] = (rt.surface_view(out, w).cpu().numpy().copy(), rng.view(-1, 12)[:, :6].cpu().numpy().copy())
    for wps in (6, 7, 2):
        assert np.array_equal(res[5][0], res[wps][0]) and np.array_equal(res[5][1], res[wps][1]), wps
