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
    return T.load_rt()


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
    unsharded render of the same frames bit for bit."""
    cmd = [sys.executable, os.path.join(T.ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--same-device",
           "--check", "--steps", "2", "--warmup", "1", "--config", "cfg1", "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2 and res["check_equal"] is True, res
    assert res["plan"]["kind"].startswith("cost") and sum(res["plan"]["tiles_per_rank"]) == 256
    assert len(res["rank_kernel_ms"]) == 2


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
