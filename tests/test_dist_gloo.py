"""World-size-2 (and 3) CPU rehearsal of the multi-GPU path with the gloo backend.

The GPU box runs the same code with RCCL: bench.py renders each rank's tiles into a compact
shard (rt_render shard mode), gathers the shards to rank 0 with sharding.gather_shards, and
unshards them there.  Here the shards are cut from a frame the oracle rendered (the kernels
need a GPU; tests/test_gpu_parity.py checks rt_render's shards and rt_unshard bit for bit),
so this covers the tile deal, the compact-shard slot order, the collective and the
reassembly.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import rt_testlib as T

W, H = 72, 40  # ragged: neither side is a multiple of the 16-pixel tile


def unshard_host(shards, width, height, tile_lists=None):
    """numpy restatement of rt_unshard / rt_unshard_tiles (the checker of the gloo rehearsal):
    [world, per_shard*256, 4] -> [H, W, 4]."""
    sh = T.load_rt().sharding
    world, n, c = shards.shape
    per_shard = n // sh.TILE_PIXELS
    img = np.zeros((height, width, c), dtype=shards.dtype)
    seen = np.zeros((height, width), dtype=np.int64)
    for r in range(world):
        xs, ys = sh.slot_pixels(width, height, r, world, per_shard, None if tile_lists is None else tile_lists[r])
        ok = xs >= 0
        img[ys[ok], xs[ok]] = shards[r][ok]
        np.add.at(seen, (ys[ok], xs[ok]), 1)
    return img, seen


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _tile_cost(frame):
    """A deterministic stand-in for the probe frame's per-tile clocks: the tile's summed RGB."""
    th, tw = (H + 15) // 16, (W + 15) // 16
    pad = np.zeros((th * 16, tw * 16), dtype=np.float64)
    pad[:H, :W] = np.nan_to_num(frame[..., :3].sum(-1), nan=1.0, posinf=1.0)
    return pad.reshape(th, 16, tw, 16).sum((1, 3)).reshape(-1) + 1.0


def _worker(rank, world, port, frame, result_q, plan):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rt = T.load_rt()
        sh = rt.sharding
        if plan == "rr":
            per_shard = max(sh.tiles_of_shard(W, H, r, world) for r in range(world))
            assert rt.shard_tiles(W, H, rank, world) == sh.tiles_of_shard(W, H, rank, world)
            lists = None
            xs, ys = sh.slot_pixels(W, H, rank, world, per_shard)
        else:
            # bench.py's cost plan: each rank measures its round-robin tiles, the costs are summed
            # over ranks (the set-up collective), and every rank computes the same LPT plan
            rr, rc = rt.shard_plan(W, H, world)
            cost = np.zeros(sh.tiles_total(W, H))
            cost[rr[rank, : rc[rank]]] = _tile_cost(frame)[rr[rank, : rc[rank]]]
            t = torch.from_numpy(cost)
            dist.all_reduce(t)
            lists, counts = rt.shard_plan(W, H, world, t.numpy())
            per_shard = lists.shape[1]
            xs, ys = sh.slot_pixels(W, H, rank, world, per_shard, lists[rank, : counts[rank]])
        shard = np.zeros((per_shard * sh.TILE_PIXELS, 4), dtype=np.float32)
        ok = xs >= 0
        shard[ok] = frame[ys[ok], xs[ok]]
        got = sh.gather_shards(torch.from_numpy(shard), rank, world)
        if rank == 0:
            img, seen = unshard_host(got.numpy(), W, H, lists)
            result_q.put((img, seen))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,plan", [(2, "rr"), (3, "rr"), (2, "cost"), (3, "cost")])
def test_gather_reassembles_frame(world, plan):
    osc = T.OracleScene("bunny")
    frame = osc.render(W, H, 1, 2, rng=T.oracle_rng_frame(0xDEADBEEF, W, H, 4), threads=4)
    frame = np.ascontiguousarray(frame.reshape(H, W, 4), dtype=np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, frame, q, plan)) for r in range(world)]
    for p in procs:
        p.start()
    img, seen = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert (seen == 1).all(), "every pixel is owned by exactly one rank"
    assert np.array_equal(img, frame)


def test_tile_deal_balanced_and_complete():
    from itertools import chain
    rt = T.load_rt()
    sh = rt.sharding
    for (w, h) in [(1920, 1080), (256, 256), (17, 1), (3840, 2160)]:
        total = sh.tiles_total(w, h)
        for n in (1, 2, 3, 8):
            counts = [rt.shard_tiles(w, h, r, n) for r in range(n)]
            assert sum(counts) == total
            assert max(counts) - min(counts) <= 1
            assert counts == [sh.tiles_of_shard(w, h, r, n) for r in range(n)]
    # slot -> pixel map is a bijection onto the frame
    n = 3
    per = max(sh.tiles_of_shard(40, 24, r, n) for r in range(n))
    pix = list(chain.from_iterable(zip(*[a[a >= 0] for a in sh.slot_pixels(40, 24, r, n, per)]) for r in range(n)))
    assert len(pix) == 40 * 24 == len(set(pix))


def test_weak_scaling_frame_sizes():
    """bench.py --scaling weak: sqrt(N) x resolution per axis, tile-aligned width, 16:9 kept."""
    import bench

    assert bench.weak_size(1920, 1080, 1) == (1920, 1080)
    assert bench.weak_size(1920, 1080, 4) == (3840, 2160)
    for n in (2, 4, 8):
        w, h = bench.weak_size(1920, 1080, n)
        assert w % 16 == 0 and abs(w / h - 16 / 9) < 2e-3
        assert abs(w * h / (1920 * 1080 * n) - 1.0) < 0.01


def test_shard_plan_round_robin_is_the_deal():
    rt = T.load_rt()
    for (w, h, n) in [(1920, 1080, 8), (72, 40, 3), (17, 1, 2), (256, 256, 1)]:
        lists, counts = rt.shard_plan(w, h, n)
        assert lists.shape[1] == rt.lib().rt_shard_plan_capacity(w, h, n)
        for r in range(n):
            assert counts[r] == rt.shard_tiles(w, h, r, n)
            assert list(lists[r, : counts[r]]) == list(range(r, rt.sharding.tiles_total(w, h), n))
            assert (lists[r, counts[r]:] == -1).all()


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_shard_plan_lpt(n):
    """Longest processing time first: every tile exactly once, within capacity, each rank's list
    heaviest first, loads within one tile's cost of each other, deterministic."""
    rt = T.load_rt()
    w, h = 1920, 1080
    tiles = rt.sharding.tiles_total(w, h)
    rng = np.random.default_rng(n)
    cost = rng.gamma(0.5, 1.0, tiles) * np.where(rng.random(tiles) < 0.05, 20.0, 1.0)
    lists, counts = rt.shard_plan(w, h, n, cost)
    cap = lists.shape[1]
    assert (counts <= cap).all() and counts.sum() == tiles
    got = np.concatenate([lists[r, : counts[r]] for r in range(n)])
    assert np.array_equal(np.sort(got), np.arange(tiles))
    loads = np.array([cost[lists[r, : counts[r]]].sum() for r in range(n)])
    assert loads.max() - loads.min() <= cost.max() + 1e-9
    for r in range(n):
        c = cost[lists[r, : counts[r]]]
        assert (np.diff(c) <= 0).all()
    again, _ = rt.shard_plan(w, h, n, cost)
    assert np.array_equal(again, lists)


def test_shard_plan_rejects_bad_costs():
    rt = T.load_rt()
    cost = np.ones(rt.sharding.tiles_total(64, 64))
    cost[3] = np.nan
    with pytest.raises(rt.RTError):
        rt.shard_plan(64, 64, 2, cost)
    cost[3] = -1.0
    with pytest.raises(rt.RTError):
        rt.shard_plan(64, 64, 2, cost)


def test_wave_clock_sanitizer_feeds_a_valid_plan():
    """bench.py's probe-frame clocks (s_memrealtime deltas, one 100 MHz time base): the sanitiser
    stays as a guard.  A wrapped (negative) delta, one longer than the probe frame's wall time and
    an inflated positive outlier (> 4096x the median) all become the median of the others, so
    rt_shard_plan (which rejects costs < 0) still deals the tiles and no outlier skews it."""
    import bench

    rt = T.load_rt()
    tiles = rt.sharding.tiles_total(64, 64)
    clocks = np.arange(1, 4 * tiles + 1, dtype=np.int64) * 1000
    clocks[5] = -(1 << 40)      # wrapped
    clocks[9] = 1 << 40         # beyond the probe's wall time
    clocks[11] = 1000 * 4 * tiles * 10000  # inflated: > 4096x the median, still inside the wall time
    wall_s = float(clocks[11]) / bench.CLOCK_HZ * 2
    c, nbad = bench.sanitize_wave_clocks(clocks, wall_s=wall_s)
    assert nbad == 3 and (c >= 0).all()
    med = np.median(np.delete(clocks, [5, 9, 11]).astype(np.float64))
    assert c[5] == c[9] == c[11] == med
    ok, n0 = bench.sanitize_wave_clocks(clocks[12:], wall_s=wall_s)
    assert n0 == 0 and np.array_equal(ok, clocks[12:].astype(np.float64))
    lists, counts = rt.shard_plan(64, 64, 2, c.reshape(-1, 4).sum(1))
    assert sorted(np.concatenate([lists[r, : counts[r]] for r in range(2)]).tolist()) == list(range(tiles))


def test_launcher_deadline_kills_stalled_job():
    """bench.launch_ranks: a job whose rank 1 stalls before a collective is killed whole at the
    deadline and the launcher returns 124 (instead of holding the driver until its own timeout)."""
    import subprocess
    import sys
    import time

    import bench

    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers", "stall_rank.py")
    t0 = time.monotonic()
    rc = bench.launch_ranks(2, cmd=[sys.executable, script], deadline_s=20.0)
    assert rc == 124 and time.monotonic() - t0 < 60
    # the per-rank watchdog (launches under torch.distributed.run): rank 1 ends itself with 124,
    # rank 0 then fails its collective or reaches its own deadline
    env = dict(os.environ, STALL_DEADLINE="15")
    t0 = time.monotonic()
    procs = []
    port = str(_free_port())
    for r in range(2):
        e = dict(env, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, script], env=e, stderr=subprocess.PIPE, text=True))
    out = [p.communicate(timeout=90)[1] for p in procs]
    assert procs[1].returncode == 124 and "deadline exceeded in phase 'collective'" in out[1]
    assert procs[0].returncode != 0
    assert time.monotonic() - t0 < 90


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gather_bookkeeping_uneven_shards(world):
    """The RCCL gather's byte bookkeeping without a transfer (the multi-rank send/recv group itself
    has only run with one rank and in same-GPU rehearsals): bench.gather_layout's recv_bytes and
    stride for an LPT plan with uneven tile counts, rt_gather_shards' copy rule restated (rank r's
    first recv_bytes[r] bytes land at r * stride; the rest of row r keeps whatever the buffer held),
    then the unshard -- the frame comes back exactly, and no slot past a rank's counts[r] tiles is
    ever read (they hold NaN here)."""
    import bench

    rt = T.load_rt()
    sh = rt.sharding
    w, h = 200, 120
    rng = np.random.default_rng(world)
    frame = rng.random((h, w, 4), dtype=np.float32)
    tiles = sh.tiles_total(w, h)
    cost = rng.gamma(0.3, 1.0, tiles) * np.where(rng.random(tiles) < 0.1, 30.0, 1.0)
    lists, counts = rt.shard_plan(w, h, world, cost)
    cap = lists.shape[1]
    assert len(set(counts.tolist())) > 1 or world == 1, "the plan should be uneven for this test"
    recv_bytes, stride = bench.gather_layout(counts, cap)
    assert stride == cap * 256 * 16 and all(rb <= stride for rb in recv_bytes)
    gathered = np.full((world, stride // 4), np.nan, dtype=np.float32)  # the root's buffer, never cleared
    for r in range(world):
        shard = np.full((cap * 256, 4), np.nan, dtype=np.float32)  # a rank's whole shard buffer
        xs, ys = sh.slot_pixels(w, h, r, world, cap, lists[r, : counts[r]])
        ok = xs >= 0
        shard[ok] = frame[ys[ok], xs[ok]]
        n = recv_bytes[r] // 4
        gathered[r, :n] = shard.reshape(-1)[:n]  # rt_gather_shards: recv_bytes[r] bytes at r * stride
    img, seen = unshard_host(gathered.reshape(world, cap * 256, 4), w, h, lists)
    assert (seen == 1).all()
    assert np.array_equal(img, frame)


def _occ_worker(rank, world, port, maps, times, plain_times, result_q):
    """One rank of bench.settle_occupancy: `maps[rank]` says whether this rank kept its lane map;
    the fake probe max-reduces its per-candidate times over ranks exactly as bench's does."""
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cands = (3, 4, 5, 6, 7)
        calls = []

        def probe(ls):
            calls.append("map" if ls is not None else "plain")
            src = times if ls is not None else plain_times
            t = torch.tensor([src[rank][w] for w in cands], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            best = {w: float(x) for w, x in zip(cands, t.tolist())}
            return min(best, key=best.get), best

        lane_slots = np.arange(64, dtype=np.int32) if maps[rank] else None
        wps, best, ls, note = bench.settle_occupancy(probe, lane_slots, 6, world, torch.device("cpu"))
        dist.barrier()
        result_q.put((rank, wps, ls is not None, note, calls))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("plain_wins", [True, False])
def test_occupancy_settles_when_one_rank_dropped_its_map(plain_wins):
    """refine_lane_map keeps or drops a rank's lane map on that rank alone, so
    ranks can disagree on `lane_slots is not None`; the plain-order re-probe (a collective) must then
    run on EVERY rank or the job hangs.  Rank 0 keeps a map, rank 1 dropped its own; the job's
    occupancy (7, max over ranks) differs from the one the map was refined at (6), so the plain order
    is probed again on both ranks, and both take the same decision."""
    world = 2
    slow = {3: 9.0, 4: 9.0, 5: 8.0}
    map0 = {**slow, 6: 7.5, 7: 7.0}     # rank 0 with its map
    plain1 = {**slow, 6: 6.4, 7: 7.2}   # rank 1 (no map): its plain order, first probe and re-probe
    plain0 = {**slow, **({6: 6.5, 7: 7.9} if plain_wins else {6: 7.8, 7: 7.9})}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_occ_worker, args=(r, world, port, [True, False], [map0, plain1], [plain0, plain1], q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, w0, m0, n0, c0), (r1, w1, m1, n1, c1) = got
    assert c0 == ["map", "plain"] and c1 == ["plain", "plain"], "both ranks make the same collective calls"
    assert w0 == w1 == (6 if plain_wins else 7)
    if plain_wins:
        assert not m0 and not m1 and n0 and "dropped" in n0 and n1 == n0
    else:
        assert m0 and not m1 and n0 is None and n1 is None
