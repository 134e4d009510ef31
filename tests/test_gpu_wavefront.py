"""GPU parity of the wavefront tracer (rt_render_params.flags RT_RENDER_TRACER_WAVEFRONT,
csrc/rt_wavefront.hip): against the CPU oracle on small frames, and against the production
kernel -- frames, final RNG states and segment counts, bit for bit -- at medium and full size,
for the bunny (pair records, floor leaf), the 4-bunny scene (leaf trees) and the plane grid."""
import numpy as np
import pytest
import torch

import rt_testlib as T
from test_gpu_parity import assert_close, gpu_render, make_scene, oracle_render

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    torch.cuda.set_device(0)
    rt = T.load_rt()
    rt.load_experimental()  # the wavefront tracer lives in librt_hip_exp.so
    return rt


@pytest.mark.parametrize("spp,bounces", [(1, 1), (4, 6), (8, 6)])
def test_wavefront_bunny_small_vs_oracle(rt, spp, bounces):
    w, h = 64, 36
    g = gpu_render(rt, "bunny", w, h, spp, bounces, tracer="wavefront")
    o = oracle_render("bunny", w, h, spp, bounces)
    assert_close(g["frames"][0], o["frames"][0], f"wavefront bunny {w}x{h} spp{spp} b{bounces}")
    assert np.array_equal(g["rng"], o["rng"]), "final RNG states differ"


@pytest.mark.parametrize("which,plane_n", [("bunny4", None), ("plane1m", 64)])
def test_wavefront_small_scenes_vs_oracle(rt, which, plane_n):
    g = gpu_render(rt, which, 40, 24, 2, 6, plane_n=plane_n, tracer="wavefront")
    o = oracle_render(which, 40, 24, 2, 6, plane_n=plane_n or 708)
    assert_close(g["frames"][0], o["frames"][0], f"wavefront {which}")
    assert np.array_equal(g["rng"], o["rng"])


def test_wavefront_progressive_and_no_bounce(rt):
    w, h = 48, 32
    g = gpu_render(rt, "bunny", w, h, 2, 6, frames=3, tracer="wavefront")
    o = oracle_render("bunny", w, h, 2, 6, frames=3)
    for f in range(3):
        assert_close(g["frames"][f], o["frames"][f], f"frame {f}")
    a = gpu_render(rt, "bunny", w, h, 3, 0, tracer="wavefront")
    b = gpu_render(rt, "bunny", w, h, 3, 0)
    assert np.array_equal(a["frames"][0], b["frames"][0]) and np.array_equal(a["rng"], b["rng"])


def _frame(rt, which, w, h, spp, bounces, tracer, plane_n=None):
    s = make_scene(rt, which, w, h, plane_n)
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    out, last = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
    segs = torch.zeros(1, dtype=torch.int64, device="cuda")
    rt.render(s, out, last, w, h, spp, bounces, 0, segment_counter=segs, tracer=tracer)
    torch.cuda.synchronize()
    return (rt.surface_view(out, w).cpu().numpy().copy(), rng.view(-1, 12)[:, :6].cpu().numpy().copy(),
            int(segs.item()))


@pytest.mark.parametrize("which,plane_n", [("bunny", None), ("bunny4", None), ("plane1m", 200)])
def test_wavefront_equals_production_medium(rt, which, plane_n):
    a = _frame(rt, which, 256, 144, 4, 6, "fast", plane_n)
    b = _frame(rt, which, 256, 144, 4, 6, "wavefront", plane_n)
    assert np.array_equal(a[0], b[0]), "frames differ"
    assert np.array_equal(a[1], b[1]), "final RNG states differ"
    assert a[2] == b[2], (a[2], b[2])


def test_wavefront_equals_production_config2_full(rt):
    """BASELINE configs[1] at full size: 1920x1080, 8 spp, 6 bounces (30.25 M segments)."""
    a = _frame(rt, "bunny", 1920, 1080, 8, 6, "fast")
    b = _frame(rt, "bunny", 1920, 1080, 8, 6, "wavefront")
    assert a[2] == b[2] and a[2] > 30_000_000, (a[2], b[2])
    assert np.array_equal(a[1], b[1]), "final RNG states differ"
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)), "frames differ"


def test_wavefront_shard_equals_production_shard(rt):
    """A cost-ordered shard (explicit tile list, compact out_shard) through both tracers."""
    w, h, spp, bounces, n = 96, 64, 2, 6, 3
    s = make_scene(rt, "bunny", w, h)
    tiles = ((w + 15) // 16) * ((h + 15) // 16)
    order = np.arange(tiles, dtype=np.int32)[::-1][1::n].copy()  # a sparse, reversed list
    tl = torch.from_numpy(order).cuda()
    outs = {}
    for tracer in ("fast", "wavefront"):
        rng = rt.alloc_rng(len(order) * 256)
        rt.init_rng_tiles(rng, w, h, tl, T.SEED)
        s.upload(rng.data_ptr())
        shard = torch.zeros((len(order) * 256, 4), dtype=torch.float32, device="cuda")
        rt.render(s, None, torch.zeros_like(shard), w, h, spp, bounces, 0, 0, n, out_shard=shard, tile_list=tl,
                  tracer=tracer)
        torch.cuda.synchronize()
        outs[tracer] = (shard.cpu().numpy(), rng.view(-1, 12)[:, :6].cpu().numpy())
    assert np.array_equal(outs["fast"][0], outs["wavefront"][0])
    assert np.array_equal(outs["fast"][1], outs["wavefront"][1])


def test_wavefront_misuse_is_refused(rt):
    w, h = 32, 16
    s = make_scene(rt, "bunny", w, h)
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    out = rt.alloc_surface(w, h)
    st = torch.zeros(rt.STAT_COUNT, dtype=torch.int64, device="cuda")
    with pytest.raises(RuntimeError, match="wavefront"):
        rt.render(s, out, out, w, h, 1, 1, 0, stats=st, tracer="wavefront")
    with pytest.raises(RuntimeError, match="spp x bounces"):
        rt.render(s, out, out, w, h, 300, 300, 0, tracer="wavefront")
