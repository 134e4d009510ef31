"""The multi-GPU path on one device: cost-aware tile plans, the compact
shard layout for explicit tile lists, the RCCL gather from the C-ABI, and bench.py's own rank
launcher.  Any partition of the 16x16 tiles renders the same pixels as the whole frame
(per-pixel RNG subsequences, RayTracing/Random.cu:7 + GPUScene.h:95), so every check here is
bit equality with an unsharded render of the same frames."""
import os
import json
import subprocess
import sys

import numpy as np
import pytest
import torch

import rt_testlib as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    torch.cuda.set_device(0)
    rt = T.load_rt()
    rt.load_experimental()  # refill / lone-pixel kernels (librt_hip_exp.so)
    return rt


def scene(rt, w, h, which="bunny"):
    s = rt.Scene()
    s.setup(which)
    s.set_viewport(w, h)
    return s


def full_frames(rt, w, h, spp, bounces, frames, which="bunny", tile_list=None):
    s = scene(rt, w, h, which)
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    bufs = [rt.alloc_surface(w, h), rt.alloc_surface(w, h)]
    for f in range(frames):
        rt.render(s, bufs[f & 1], bufs[(f + 1) & 1], w, h, spp, bounces, f, tile_list=tile_list)
    torch.cuda.synchronize()
    return rt.surface_view(bufs[(frames - 1) & 1], w).cpu().numpy().copy(), rng.cpu().numpy().copy()


def probe_costs(rt, s, w, h, spp, bounces, n):
    """bench.make_plan's probe: each rank's round-robin tiles rendered once with per-wave clocks."""
    rr, rc = rt.shard_plan(w, h, n)
    cost = np.zeros(rt.sharding.tiles_total(w, h))
    for r in range(n):
        mine = torch.from_numpy(rr[r, : rc[r]]).cuda()
        rng = rt.alloc_rng(int(rc[r]) * 256)
        rt.init_rng_tiles(rng, w, h, mine, T.SEED)
        s.upload(rng.data_ptr())
        out = torch.zeros((int(rc[r]) * 256, 4), dtype=torch.float32, device="cuda")
        clk = torch.zeros(int(rc[r]) * 4, dtype=torch.int64, device="cuda")
        rt.render(s, None, None, w, h, spp, bounces, 0, r, n, out_shard=out, tile_list=mine, wave_clock=clk)
        torch.cuda.synchronize()
        c = clk.view(-1, 4).cpu().numpy()
        assert (c > 0).all(), "every wave of a real tile reports its clock"
        cost[rr[r, : rc[r]]] = c.sum(1)
    return cost


@pytest.mark.parametrize("n", [2, 3, 8])
def test_cost_plan_shards_equal_full(rt, n):
    """Probe -> LPT plan -> per-rank compact shards (rt_init_rng_tiles + tile_list) over two
    progressive frames -> rt_unshard_tiles == the unsharded frames, bit for bit."""
    w, h, spp, bounces, frames = 120, 72, 2, 6, 2
    full, _ = full_frames(rt, w, h, spp, bounces, frames)
    s = scene(rt, w, h)
    cost = probe_costs(rt, s, w, h, spp, bounces, n)
    lists, counts = rt.shard_plan(w, h, n, cost)
    cap = lists.shape[1]
    shards = torch.zeros((2, n, cap * 256, 4), dtype=torch.float32, device="cuda")
    for r in range(n):
        mine = torch.from_numpy(lists[r, : counts[r]]).cuda()
        rng = rt.alloc_rng(cap * 256)
        rt.init_rng_tiles(rng, w, h, mine, T.SEED)
        s.upload(rng.data_ptr())
        for f in range(frames):
            rt.render(s, None, shards[(f + 1) & 1, r], w, h, spp, bounces, f, r, n, out_shard=shards[f & 1, r],
                      tile_list=mine)
        torch.cuda.synchronize()
    out = rt.alloc_surface(w, h)
    rt.unshard_tiles(out, w, h, shards[(frames - 1) & 1], torch.from_numpy(lists).cuda())
    torch.cuda.synchronize()
    got = rt.surface_view(out, w).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32)), f"n={n}"


def test_single_gpu_tile_order_is_free(rt):
    """N = 1 with an explicit (heaviest-first) tile list: RNG stays in the reference's y*W + x
    layout and the output in the pitched surface; only the launch order changes."""
    w, h, spp, bounces = 200, 120, 2, 6
    full, rng_full = full_frames(rt, w, h, spp, bounces, 2)
    s = scene(rt, w, h)
    cost = probe_costs(rt, s, w, h, spp, bounces, 1)
    lists, counts = rt.shard_plan(w, h, 1, cost)
    order = torch.from_numpy(lists[0, : counts[0]]).cuda()
    got, rng_got = full_frames(rt, w, h, spp, bounces, 2, tile_list=order)
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32))
    assert np.array_equal(rng_got, rng_full)


def lane_costs(rt, s, w, h, spp, bounces, mine, n, r):
    """Per-pixel work of one probe frame of a shard (rt_render_params.lane_cost)."""
    rng = rt.alloc_rng(mine.numel() * 256)
    rt.init_rng_tiles(rng, w, h, mine, T.SEED)
    s.upload(rng.data_ptr())
    out = torch.zeros((mine.numel() * 256, 4), dtype=torch.float32, device="cuda")
    cost = torch.zeros(mine.numel() * 256, dtype=torch.int32, device="cuda")
    rt.render(s, None, None, w, h, spp, bounces, 0, r, n, out_shard=out, tile_list=mine, lane_cost=cost)
    torch.cuda.synchronize()
    return cost.cpu().numpy()


@pytest.mark.parametrize("n,mode", [(1, "plan"), (4, "plan"), (2, "random"), (4, "refine")])
def test_lane_map_shards_equal_full(rt, n, mode):
    """Probe per-pixel work -> rt_lane_plan (aggressive: every sub-tile wave above the costliest
    pixel's modelled time is split; "refine": then rt_lane_refine from a timing frame's per-wave
    clocks of that map, as bench.py --lane-refine does) or a random permutation with idle lanes ->
    the sharded frames rendered through the lane map == the unsharded frames, bit for bit (pixels,
    RNG progression over two progressive frames)."""
    w, h, spp, bounces, frames = 120, 72, 2, 6, 2
    full, _ = full_frames(rt, w, h, spp, bounces, frames)
    s = scene(rt, w, h)
    cost = probe_costs(rt, s, w, h, spp, bounces, n)
    lists, counts = rt.shard_plan(w, h, n, cost)
    cap = lists.shape[1]
    shards = torch.zeros((2, n, cap * 256, 4), dtype=torch.float32, device="cuda")
    gen = np.random.default_rng(n)
    for r in range(n):
        mine = torch.from_numpy(lists[r, : counts[r]]).cuda()
        c = lane_costs(rt, s, w, h, spp, bounces, mine, n, r)
        xs, ys = rt.sharding.slot_pixels(w, h, r, n, int(counts[r]), lists[r, : counts[r]])
        inside = (xs >= 0) & (xs < w) & (ys >= 0) & (ys < h)
        assert (c[inside] > 0).all() and (c[~inside] == 0).all(), "work is reported for exactly the frame's pixels"
        if mode in ("plan", "refine"):
            m, nlong = rt.lane_plan(c, 1e12, 1.0)
            assert m.size > c.size, "the heavy sub-tile waves were split"
        if mode == "refine":
            rng = rt.alloc_rng(cap * 256)
            rt.init_rng_tiles(rng, w, h, mine, T.SEED)
            s.upload(rng.data_ptr())
            clk = torch.zeros(m.size // 64, dtype=torch.int64, device="cuda")
            rt.render(s, None, None, w, h, spp, bounces, 0, r, n, out_shard=shards[0, r], tile_list=mine,
                      lane_slots=torch.from_numpy(m).cuda(), wave_clock=clk)
            torch.cuda.synchronize()
            m2, nsplit = rt.lane_refine(m, c, np.maximum(clk.cpu().numpy(), 0), 0.5)
            assert nsplit > 0 and m2.size > m.size
            m, nlong = m2, 0
        else:
            m = np.full(c.size * 2, -1, dtype=np.int32)
            m[gen.choice(m.size, c.size, replace=False)] = gen.permutation(c.size).astype(np.int32)
            nlong = 3
        assert np.array_equal(np.sort(m[m >= 0]), np.arange(c.size))
        lm = torch.from_numpy(m).cuda()
        rng = rt.alloc_rng(cap * 256)
        rt.init_rng_tiles(rng, w, h, mine, T.SEED)
        s.upload(rng.data_ptr())
        for f in range(frames):
            rt.render(s, None, shards[(f + 1) & 1, r], w, h, spp, bounces, f, r, n, out_shard=shards[f & 1, r],
                      tile_list=mine, lane_slots=lm, priority_waves=nlong)
        torch.cuda.synchronize()
    out = rt.alloc_surface(w, h)
    rt.unshard_tiles(out, w, h, shards[(frames - 1) & 1], torch.from_numpy(lists).cuda())
    torch.cuda.synchronize()
    got = rt.surface_view(out, w).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32)), f"n={n} {mode}"


def test_lane_map_full_frame_layout(rt):
    """N = 1, reference layout (RNG y*W + x, pitched surface) through a lane map == no map."""
    w, h, spp, bounces = 200, 120, 2, 6
    full, rng_full = full_frames(rt, w, h, spp, bounces, 2)
    s = scene(rt, w, h)
    tiles = rt.sharding.tiles_total(w, h)
    mine = torch.arange(tiles, dtype=torch.int32, device="cuda")
    c = lane_costs(rt, s, w, h, spp, bounces, mine, 1, 0)
    m, nlong = rt.lane_plan(c, 1e12, 1.0)
    lm = torch.from_numpy(m).cuda()
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    bufs = [rt.alloc_surface(w, h), rt.alloc_surface(w, h)]
    for f in range(2):
        rt.render(s, bufs[f & 1], bufs[(f + 1) & 1], w, h, spp, bounces, f, tile_list=mine, lane_slots=lm,
                  priority_waves=nlong)
    torch.cuda.synchronize()
    got = rt.surface_view(bufs[1], w).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32))
    assert np.array_equal(rng.cpu().numpy(), rng_full)


@pytest.mark.parametrize("refill,mapped", [(16, False), (1, True), (64, False)])
def test_refill_equals_full(rt, refill, mapped):
    """rt_render refill_lanes: a grid of resident waves pulls the rest of the lane order from a
    queue (ballot + mbcnt over the idle lanes, one atomic per refill) -- any lane may render any
    pixel at any time, so the frames and the RNG progression equal the plain render bit for bit.
    The frame is large enough that the queue is long (8160 sub-tile waves for ~5000 resident)."""
    w, h, spp, bounces = 1920, 1080, 1, 3
    full, rng_full = full_frames(rt, w, h, spp, bounces, 2)
    s = scene(rt, w, h)
    tiles = rt.sharding.tiles_total(w, h)
    mine = torch.arange(tiles, dtype=torch.int32, device="cuda")
    lm = None
    if mapped:
        m = np.arange(tiles * 256, dtype=np.int32).reshape(-1, 64)
        m[::7, ::3] = -1  # holes in the queue are skipped
        rest = np.sort(np.arange(tiles * 256).reshape(-1, 64)[::7, ::3].ravel()).astype(np.int32)
        m = np.concatenate([m.ravel(), rest, np.full((-rest.size) % 64, -1, np.int32)])
        lm = torch.from_numpy(m).cuda()
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    bufs = [rt.alloc_surface(w, h), rt.alloc_surface(w, h)]
    for f in range(2):
        rt.render(s, bufs[f & 1], bufs[(f + 1) & 1], w, h, spp, bounces, f, tile_list=mine, lane_slots=lm,
                  refill_lanes=refill)
    torch.cuda.synchronize()
    got = rt.surface_view(bufs[1], w).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32))
    assert np.array_equal(rng.cpu().numpy(), rng_full)


def test_refill_with_leaf_trees_equals_full(rt):
    """The refill kernels of a leaf-tree scene (the 4-bunny frame: cooperative tree walks, deferred tree
    leaves and their end phase inside the refill loop) equal the plain render bit for bit."""
    w, h, spp, bounces = 640, 360, 2, 4
    full, rng_full = full_frames(rt, w, h, spp, bounces, 1, "bunny4")
    s = scene(rt, w, h, "bunny4")
    mine = torch.arange(rt.sharding.tiles_total(w, h), dtype=torch.int32, device="cuda")
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
    rt.render(s, a, b, w, h, spp, bounces, 0, tile_list=mine, refill_lanes=16)
    torch.cuda.synchronize()
    assert np.array_equal(rt.surface_view(a, w).cpu().numpy().view(np.uint32), full.view(np.uint32))
    assert np.array_equal(rng.cpu().numpy(), rng_full)


@pytest.mark.parametrize("which", ["bunny", "bunny4"])
def test_one_pixel_waves_equal_full(rt, which):
    """A lane map with ONE pixel per wave: every traversal runs through the lone-ray path
    (rt_fast.h lone_traverse: the whole wave on one ray, stack spread over the lanes) -- the frames
    and the RNG progression equal the plain render bit for bit; also with the lone path switched
    off (RT_TUNE bit 26), so both paths are pinned against each other."""
    w, h, spp, bounces = 40, 24, 2, 6
    full, rng_full = full_frames(rt, w, h, spp, bounces, 2, which)
    s = scene(rt, w, h, which)
    tiles = rt.sharding.tiles_total(w, h)
    mine = torch.arange(tiles, dtype=torch.int32, device="cuda")
    xs, ys = rt.sharding.slot_pixels(w, h, 0, 1, tiles, np.arange(tiles))
    slots = np.flatnonzero(xs >= 0).astype(np.int32)
    m = np.full((slots.size, 64), -1, dtype=np.int32)
    m[:, 0] = slots
    lm = torch.from_numpy(m.ravel()).cuda()
    for tune in (0, 1 << 26):
        rng = rt.alloc_rng(w * h)
        rt.init_rng_states(rng, w, h, T.SEED)
        s.upload(rng.data_ptr())
        bufs = [rt.alloc_surface(w, h), rt.alloc_surface(w, h)]
        for f in range(2):
            rt.render(s, bufs[f & 1], bufs[(f + 1) & 1], w, h, spp, bounces, f, tile_list=mine, lane_slots=lm, tune=tune)
        torch.cuda.synchronize()
        got = rt.surface_view(bufs[1], w).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), full.view(np.uint32)), f"{which} tune={tune}"
        assert np.array_equal(rng.cpu().numpy(), rng_full)


def test_lane_map_misuse_is_refused(rt):
    w, h = 64, 64
    s = scene(rt, w, h)
    rng = rt.alloc_rng(w * h)
    s.upload(rng.data_ptr())
    a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
    with pytest.raises(rt.RTError, match="lane"):
        rt.render(s, a, b, w, h, 1, 1, tracer="ref", lane_cost=torch.zeros(w * h, dtype=torch.int32, device="cuda"))
    p = rt.RenderParams()
    p.surface, p.width, p.height, p.pitch, p.spp, p.bounces, p.shard_count = a.data_ptr(), w, h, w * 16, 1, 1, 1
    lm = torch.zeros(100, dtype=torch.int32, device="cuda")
    p.lane_slots, p.lane_slot_count = lm.data_ptr(), 100  # not a multiple of 64
    import ctypes
    assert rt.lib().rt_render(ctypes.byref(p), ctypes.cast(s.gpu, ctypes.c_void_p), None) != 0
    with pytest.raises(rt.RTError, match="refill"):
        rt.render(s, a, b, w, h, 1, 1, refill_lanes=65)
    with pytest.raises(rt.RTError, match="without refill"):
        rt.render(s, a, b, w, h, 1, 1, refill_lanes=8, lane_cost=torch.zeros(w * h, dtype=torch.int32, device="cuda"))
    torch.cuda.synchronize()


def test_rccl_gather_one_rank(rt):
    """rt_gather_shards through the C-ABI (RCCL) with a one-rank communicator: the root's own
    shard lands at its stride offset (the other ranks' path is the same send/recv group)."""
    uid = rt.Comm.unique_id()
    comm = rt.Comm(1, 0, uid)
    try:
        shard = torch.arange(4096 * 3, dtype=torch.float32, device="cuda")
        gathered = torch.full((2, 4096 * 4), -1.0, dtype=torch.float32, device="cuda")
        comm.gather(shard, shard.numel() * 4, gathered, gathered.shape[1] * 4, [shard.numel() * 4])
        torch.cuda.synchronize()
        assert torch.equal(gathered[0, : shard.numel()], shard)
        assert (gathered[0, shard.numel():] == -1).all() and (gathered[1] == -1).all()
    finally:
        comm.close()


def test_bench_two_ranks_without_launcher(tmp_path):
    """bench.py --gpus 2 --backend gloo --same-device --check: bench starts both ranks itself
    (no torchrun), deals tiles by the probe's costs, gathers, and rank 0's frame equals an
    unsharded render of the same frames bit for bit.  --lane-refine 0: the model's lane map is
    rendered as planned (with refinement, config 1's tiny frame keeps the plain tile order, which
    the default bench runs cover)."""
    cmd = [sys.executable, os.path.join(T.ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--same-device",
           "--check", "--steps", "2", "--warmup", "1", "--config", "cfg1", "--no-cpu-baseline", "--lane-refine", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2 and res["check_equal"] is True, res
    assert res["plan"]["kind"].startswith("cost") and sum(res["plan"]["tiles_per_rank"]) == 256
    assert res["plan"]["lanes"]["waves"] >= 4 * 128, "the lane plan is rendered (bench --lanes auto)"
    assert len(res["rank_kernel_ms"]) == 2
    assert res["gather_ms"] > 0 and res["gather_ms_slowest_rank"] > 0, "per-frame gather time in the line"


def test_short_buffers_are_refused(rt):
    """rt_render / rt_init_rng_tiles / rt_unshard_tiles check every device buffer against what the
    launch would touch and return an error instead of faulting the GPU.  (The check sees the
    whole device allocation a pointer lies in -- torch's caching allocator hands out sub-blocks
    of up to 2 MB segments -- so the frame here is large enough to overrun any segment.)"""
    w, h = 1920, 1088
    s = scene(rt, w, h)
    small = rt.alloc_rng(256)  # one tile's states for an 8160-tile frame
    s.upload(small.data_ptr())
    a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
    with pytest.raises(rt.RTError, match="rng_state"):
        rt.render(s, a, b, w, h, 1, 1)
    lists, counts = rt.shard_plan(w, h, 2)
    mine = torch.from_numpy(lists[0, : counts[0]]).cuda()
    with pytest.raises(rt.RTError):
        rt.init_rng_tiles(small, w, h, mine, T.SEED)  # 4080 tiles into one tile's states
    out = torch.zeros((256, 4), dtype=torch.float32, device="cuda")
    with pytest.raises(rt.RTError, match="out_shard|rng_state"):
        rt.render(s, None, None, w, h, 1, 1, 0, 0, 2, out_shard=out, tile_list=mine)
    with pytest.raises(rt.RTError):
        rt.unshard_tiles(a, w, h, torch.zeros((2, 256, 4), device="cuda"), torch.from_numpy(lists).cuda())
    torch.cuda.synchronize()


@pytest.mark.parametrize("which,frac", [("bunny", 0.25), ("bunny", 1.0), ("bunny4", 0.3)])
def test_lone_pixels_equal_full(rt, which, frac):
    """rt_lone_plan + the lone-pixel kernel (rt_lone.hip: one wave per pixel, the BVH walked as
    treelets by ballots over their preorder slots) beside the production kernel's lane map: the
    frames and the RNG progression over two progressive frames equal the plain render bit for bit.
    frac = the share of the frame's pixels (heaviest first) that go to the lone-pixel kernel; the
    4-bunny scene brings leaf trees (coop_tree) into the lone walk."""
    w, h, spp, bounces = 120, 72, 2, 6
    full, rng_full = full_frames(rt, w, h, spp, bounces, 2, which)
    s = scene(rt, w, h, which)
    tiles = rt.sharding.tiles_total(w, h)
    mine = torch.arange(tiles, dtype=torch.int32, device="cuda")
    c = lane_costs(rt, s, w, h, spp, bounces, mine, 1, 0)
    inside = int((c > 0).sum())
    lone, marked = rt.lone_plan(c, max(1, int(frac * inside)))
    assert lone.size == max(1, int(frac * inside)) and (c[lone] >= np.sort(c[c > 0])[::-1][lone.size - 1]).all()
    m, nlong = rt.lane_plan(marked, 48000.0, 1.0)
    assert not np.isin(m, lone).any(), "the lane map leaves the lone pixels out"
    assert np.array_equal(np.sort(np.concatenate([m[m >= 0], lone])), np.sort(np.flatnonzero(np.arange(c.size) >= 0)))
    lm = torch.from_numpy(m if m.size else np.full(64, -1, np.int32)).cuda()
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    bufs = [rt.alloc_surface(w, h), rt.alloc_surface(w, h)]
    lo = torch.from_numpy(lone).cuda()
    for f in range(2):
        rt.render(s, bufs[f & 1], bufs[(f + 1) & 1], w, h, spp, bounces, f, tile_list=mine, lane_slots=lm,
                  priority_waves=nlong, lone_slots=lo)
    torch.cuda.synchronize()
    got = rt.surface_view(bufs[1], w).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32)), f"{which} frac={frac}"
    assert np.array_equal(rng.cpu().numpy(), rng_full)


def test_lone_pixels_config2_full_frame(rt):
    """Config 2 at full size (1920x1080, 8 spp, 6 bounces) with its 4096 costliest pixels in the
    lone-pixel kernel: bit-identical to the plain production frame, RNG states included."""
    w, h, spp, bounces = 1920, 1080, 8, 6
    full, rng_full = full_frames(rt, w, h, spp, bounces, 1)
    s = scene(rt, w, h)
    tiles = rt.sharding.tiles_total(w, h)
    mine = torch.arange(tiles, dtype=torch.int32, device="cuda")
    c = lane_costs(rt, s, w, h, spp, bounces, mine, 1, 0)
    lone, marked = rt.lone_plan(c, 4096)
    m, nlong = rt.lane_plan(marked, 48000.0, 1.0)
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
    rt.render(s, a, b, w, h, spp, bounces, 0, tile_list=mine, lane_slots=torch.from_numpy(m).cuda(),
              priority_waves=nlong, lone_slots=torch.from_numpy(lone).cuda())
    torch.cuda.synchronize()
    got = rt.surface_view(a, w).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32))
    assert np.array_equal(rng.cpu().numpy(), rng_full)


def test_lone_pixels_many_spheres(rt):
    """More than 64 spheres (rt_scene_add_sphere has no limit): the lone-pixel kernel walks the
    spheres in strides of 64 lanes and keeps the (distance, index) minimum, so its lone pixels equal
    the production kernel's sequential sphere loop (main_raytracing.cu:89-103) bit for bit."""
    w, h, spp, bounces = 64, 48, 2, 4

    def many(s):
        m = s.add_material(albedo=(0.6, 0.5, 0.4), roughness=0.3, specular_percent=0.2, specular=(0.9, 0.9, 0.9))
        for i in range(150):  # a cloud of small spheres in front of the bunny, some overlapping
            s.add_sphere((8.0 + 1.7 * (i % 15), -10.0 + 1.9 * (i // 15), 6.0 + 0.5 * (i % 7)), 1.1, m)

    def fresh():
        s = scene(rt, w, h)
        many(s)
        return s

    s = fresh()
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    bufs = [rt.alloc_surface(w, h), rt.alloc_surface(w, h)]
    rt.render(s, bufs[0], bufs[1], w, h, spp, bounces, 0)
    torch.cuda.synchronize()
    full, rng_full = rt.surface_view(bufs[0], w).cpu().numpy().copy(), rng.cpu().numpy().copy()
    assert s.gpu.contents.sphere_count > 64
    s2 = fresh()
    tiles = rt.sharding.tiles_total(w, h)
    mine = torch.arange(tiles, dtype=torch.int32, device="cuda")
    c = lane_costs(rt, s2, w, h, spp, bounces, mine, 1, 0)
    lone, marked = rt.lone_plan(c, c.size // 2)
    m, nlong = rt.lane_plan(marked, 48000.0, 1.0)
    rng2 = rt.alloc_rng(w * h)
    rt.init_rng_states(rng2, w, h, T.SEED)
    s2.upload(rng2.data_ptr())
    out = [rt.alloc_surface(w, h), rt.alloc_surface(w, h)]
    rt.render(s2, out[0], out[1], w, h, spp, bounces, 0, tile_list=mine, lane_slots=torch.from_numpy(m).cuda(),
              priority_waves=nlong, lone_slots=torch.from_numpy(lone).cuda())
    torch.cuda.synchronize()
    got = rt.surface_view(out[0], w).cpu().numpy()
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32))
    assert np.array_equal(rng2.cpu().numpy(), rng_full)


@pytest.mark.parametrize("wps", [5, 6, 7])
def test_big_leaf_screens_equal_plain(rt, wps):
    """The big-leaf screen variants (librt_hip_exp.so, rt_build_options.leaf_screens; rt_fast.h
    screen_leaf: a lane whose ray provably misses a leaf's core tests only its outliers) render the
    4-bunny frame and RNG states bit for bit as the production kernel without screens, at every
    occupancy (a per-lane bool for the screened state once mis-rendered at 6 waves per SIMD)."""
    w, h, spp, bounces = 256, 144, 4, 6
    res = {}
    rt.set_build_options(leaf_screens=1)
    try:
        for tune in (0, 1 << 28):  # bit 28: screens off
            s = scene(rt, w, h, "bunny4")
            rng = rt.alloc_rng(w * h)
            rt.init_rng_states(rng, w, h, T.SEED)
            s.upload(rng.data_ptr())
            a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
            rt.render(s, a, b, w, h, spp, bounces, 0, waves_per_simd=wps, tune=tune)
            torch.cuda.synchronize()
            res[tune] = (rt.surface_view(a, w).cpu().numpy().copy(), rng.cpu().numpy().copy())
    finally:
        rt.set_build_options()
    assert np.array_equal(res[0][0].view(np.uint32), res[1 << 28][0].view(np.uint32))
    assert np.array_equal(res[0][1], res[1 << 28][1])


@pytest.mark.parametrize("wps,base", [(5, 0), (6, 0), (7, 0), (5, 1 << 27)])
def test_deferred_tree_leaves_equal_reference_order(rt, wps, base):
    """Deferred leaf trees (rt_fast.h defer_leaf: a lane's first tree leaf walked at the end of its
    traversal, with the bound the rest of the scene left and ties decided by DFS order) render the
    4-bunny frame and RNG states bit for bit as the walk at the leaf (RT_TUNE bit 24), at every
    occupancy; the full-frame oracle fixture of config 4 (test_gpu_fullframe.py) covers the default.
    base = bit 27 traverses the reference's node array, where the guard's face -> leaf table (private
    node indices) must not be used (rt_render drops it: ADVICE round 5)."""
    w, h, spp, bounces = 256, 144, 4, 6
    res = {}
    if base:
        rt.load_experimental()
    for tune in (0, 1 << 24):  # bit 24: deferral off
        s = scene(rt, w, h, "bunny4")
        rng = rt.alloc_rng(w * h)
        rt.init_rng_states(rng, w, h, T.SEED)
        s.upload(rng.data_ptr())
        a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
        rt.render(s, a, b, w, h, spp, bounces, 0, waves_per_simd=wps, tune=tune | base)
        torch.cuda.synchronize()
        res[tune] = (rt.surface_view(a, w).cpu().numpy().copy(), rng.cpu().numpy().copy())
    assert np.array_equal(res[0][0].view(np.uint32), res[1 << 24][0].view(np.uint32))
    assert np.array_equal(res[0][1], res[1 << 24][1])
    if wps == 5 and not base:
        # the guard's second walk (END2) runs on this frame: the timing variant counts it;
        # its redo branch is rarer still (0 of 250,700 sampled config-4 segments, tests/test_defer_rule.py)
        s = scene(rt, w, h, "bunny4")
        rng = rt.alloc_rng(w * h)
        rt.init_rng_states(rng, w, h, T.SEED)
        s.upload(rng.data_ptr())
        a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
        st = torch.zeros(rt.STAT_COUNT, dtype=torch.int64, device="cuda")
        rt.render(s, a, b, w, h, spp, bounces, 0, waves_per_simd=wps, stats=st, tune=256)
        torch.cuda.synchronize()
        t = dict(zip(rt.STAT_NAMES, st.cpu().tolist()))
        print("deferral guard: END2 walks", t["defer_end2"], "redos", t["defer_redo"])
        assert t["defer_end2"] > 0
        assert np.array_equal(rt.surface_view(a, w).cpu().numpy().view(np.uint32), res[0][0].view(np.uint32))


def test_lone_and_lane_overlap_is_caught(rt):
    """A slot in both lone_slots and lane_slots would be rendered twice at once (undefined results,
    rt_abi.h); RT_RENDER_VALIDATE finds it on the device before anything is launched."""
    w, h = 64, 64
    s = scene(rt, w, h)
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
    mine = torch.arange(rt.sharding.tiles_total(w, h), dtype=torch.int32, device="cuda")
    lanes = torch.arange(w * h, dtype=torch.int32, device="cuda")
    lanes[5] = -1
    lone = torch.tensor([5], dtype=torch.int32, device="cuda")
    rt.render(s, a, b, w, h, 1, 2, tile_list=mine, lane_slots=lanes, lone_slots=lone, validate=True)  # disjoint
    torch.cuda.synchronize()
    lone_bad = torch.tensor([5, 17], dtype=torch.int32, device="cuda")  # 17 is also a lane's slot
    with pytest.raises(rt.RTError, match="also in lone_slots"):
        rt.render(s, a, b, w, h, 1, 2, tile_list=mine, lane_slots=lanes, lone_slots=lone_bad, validate=True)
    with pytest.raises(rt.RTError, match="lone_slots entries"):
        rt.render(s, a, b, w, h, 1, 2, tile_list=mine, lane_slots=lanes, validate=True,
                  lone_slots=torch.tensor([5, 5], dtype=torch.int32, device="cuda"))
    torch.cuda.synchronize()


def test_experimental_paths_need_the_plugin():
    """Without librt_hip_exp.so, rt_render refuses refill / lone / wavefront / A/B frames with an
    error naming the plugin, before launching anything (child process: this one has it loaded)."""
    code = """
import sys, importlib, torch
sys.path.insert(0, %r); sys.path.insert(0, %r)
import rt_testlib as T
rt = T.load_rt()
w = h = 32
s = rt.Scene(); s.setup("bunny"); s.set_viewport(w, h)
rng = rt.alloc_rng(w * h); rt.init_rng_states(rng, w, h, T.SEED); s.upload(rng.data_ptr())
a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
rt.render(s, a, b, w, h, 1, 2)
n = 0
for kw in (dict(refill_lanes=8), dict(tracer="wavefront"), dict(tune=4096)):
    try:
        rt.render(s, a, b, w, h, 1, 2, **kw)
    except rt.RTError as e:
        n += "librt_hip_exp.so" in str(e)
torch.cuda.synchronize()
print("refused", n)
""" % (T.ROOT, os.path.join(T.ROOT, "tests"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "refused 3" in r.stdout, r.stdout


def test_lone_misuse_is_refused(rt):
    w, h = 64, 64
    s = scene(rt, w, h)
    rng = rt.alloc_rng(w * h)
    rt.init_rng_states(rng, w, h, T.SEED)
    s.upload(rng.data_ptr())
    a, b = rt.alloc_surface(w, h), rt.alloc_surface(w, h)
    lo = torch.zeros(4, dtype=torch.int32, device="cuda")
    with pytest.raises(rt.RTError, match="lone"):
        rt.render(s, a, b, w, h, 1, 1, lone_slots=lo)  # no lane map
    with pytest.raises(rt.RTError, match="production tracer"):
        rt.render(s, a, b, w, h, 1, 1, tracer="ref", lone_slots=lo, lane_slots=torch.full((64,), -1, dtype=torch.int32, device="cuda"))
    torch.cuda.synchronize()
