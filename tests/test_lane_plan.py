"""rt_lane_plan (shard.cpp), the host side of the lane map: the plan is a permutation of the
slots into waves of at most 64 lanes, keeps cheap sub-tile waves whole and in list order, splits
the waves whose modelled time max c x (sum c / max c)^0.34 exceeds the target into sub-waves
within it (a pixel's sub-tile neighbours stay together), and launches the long waves first.  No
GPU needed: the plan is pure host code behind the C-ABI."""
import numpy as np
import pytest

import rt_testlib as T


@pytest.fixture(scope="module")
def rt():
    return T.load_rt()


def waves_of(m, cost):
    mw = m.reshape(-1, 64)
    out = []
    for row in mw:
        s = row[row >= 0]
        c = cost[s].astype(np.float64)
        mx = c.max() if c.size else 0.0
        e = mx * (c.sum() / mx) ** 0.34 if mx > 0 else 0.0
        out.append((s, e))
    return out


def check_perm(m, slots):
    assert m.size % 64 == 0
    v = m[m >= 0]
    assert np.array_equal(np.sort(v), np.arange(slots)), "every slot exactly once"


def test_identity_without_parallelism(rt):
    cost = np.random.default_rng(0).integers(1, 100, 64 * 40).astype(np.uint32)
    m, nlong = rt.lane_plan(cost, 0.0, 1.0)
    assert np.array_equal(m, np.arange(cost.size)) and nlong == 0


def test_uniform_work_is_not_split(rt):
    """Equal pixels: a 64-lane wave models to 50 x 64^0.34 = 206 units; with the rank's work
    over parallel_units above that (320,000 / 1,000 = 320) every sub-tile wave stays whole."""
    cost = np.full(64 * 100, 50, dtype=np.uint32)
    m, nlong = rt.lane_plan(cost, 1000.0, 1.0)
    assert np.array_equal(m, np.arange(cost.size)) and nlong == 100  # all long (>= half the target)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_heavy_pixels_are_split_out(rt, seed):
    g = np.random.default_rng(seed)
    slots = 64 * 300
    cost = g.integers(10, 60, slots).astype(np.uint32)
    heavy = g.choice(slots, 40, replace=False)
    cost[heavy] = g.integers(2000, 4000, heavy.size)
    units = 2000.0
    m, nlong = rt.lane_plan(cost, units, 1.0)
    check_perm(m, slots)
    B = max(cost.max(), cost.sum() / units)
    ws = waves_of(m, cost)
    for s, e in ws:
        assert len(s) <= 64 and len(set(s // 64)) == 1, "a wave holds pixels of one sub-tile"
        if len(s) > 1:
            assert e <= B * (1 + 1e-9)
    # long waves first, longest first, then the rest in list order
    es = [e for _, e in ws]
    assert all(e >= 0.5 * B for e in es[:nlong]) and all(e < 0.5 * B for e in es[nlong:])
    assert es[:nlong] == sorted(es[:nlong], reverse=True)
    firsts = [int(s.min() // 64) for s, _ in ws[nlong:]]
    assert firsts == sorted(firsts)
    assert nlong > 0 and len(ws) > slots // 64


def test_zero_cost_slots_ride_along(rt):
    cost = np.zeros(64 * 4, dtype=np.uint32)
    cost[:10] = 1000  # a partial edge tile: only 10 pixels in the frame
    m, _ = rt.lane_plan(cost, 1e12, 1.0)
    check_perm(m, cost.size)


def test_capacity_caps_the_split(rt):
    cost = np.full(64 * 8, 1000, dtype=np.uint32)
    m, _ = rt.lane_plan(cost, 1e12, 0.01)  # a target below one pixel: every pixel alone ...
    check_perm(m, cost.size)
    assert m.size <= rt.lib().rt_lane_plan_capacity(cost.size)  # ... until the plan's capacity


def test_bad_arguments(rt):
    with pytest.raises(rt.RTError, match="lane_plan"):
        rt.lane_plan(np.ones(100, dtype=np.uint32), 1.0, 1.0)  # not a multiple of 64
    with pytest.raises(rt.RTError, match="lane_plan"):
        rt.lane_plan(np.ones(64, dtype=np.uint32), 1.0, 0.0)  # slack must be > 0


def test_lone_plan_takes_the_heaviest_and_lane_plan_skips_them(rt):
    """rt_lone_plan picks the costliest slots (heaviest first, ties by slot), at least min_cost,
    at most max_lone, and marks them UINT32_MAX; rt_lane_plan then maps every other slot exactly
    once and none of the lone ones (sub-tile waves emptied by it disappear)."""
    gen = np.random.default_rng(3)
    cost = gen.integers(1, 1000, 64 * 50).astype(np.uint32)
    cost[64 * 7: 64 * 8] = 5000  # a sub-tile taken whole
    lone, marked = rt.lone_plan(cost, 100, 1)
    assert lone.size == 100 and (marked[lone] == 0xFFFFFFFF).all()
    assert list(cost[lone]) == sorted(cost[lone], reverse=True)
    assert cost[lone].min() >= np.delete(cost, lone).max()
    assert set(range(64 * 7, 64 * 8)) <= set(lone.tolist())
    rest = np.setdiff1d(np.arange(cost.size), lone)
    for units in (0.0, 48000.0, 1e12):
        m, _ = rt.lane_plan(marked, units, 1.0)
        v = m[m >= 0]
        assert np.array_equal(np.sort(v), rest), units
        assert not (m.reshape(-1, 64) < 0).all(axis=1).any(), "no empty waves"
    few, _ = rt.lone_plan(cost, 10, 4000)
    assert few.size == 10 and (cost[few] == 5000).all()
    none, same = rt.lone_plan(cost, 10, 6000)
    assert none.size == 0 and np.array_equal(same, cost)


def test_lane_refine_splits_the_measured_tail(rt):
    """rt_lane_refine: the waves whose measured clock is within theta of the longest (and hold more
    than one pixel) become two waves, their pixels in decreasing work dealt alternately; every slot
    stays mapped exactly once and the waves come out longest first (a half at 3/4 of its parent)."""
    gen = np.random.default_rng(5)
    slots = 64 * 40
    cost = gen.integers(1, 1000, slots).astype(np.uint32)
    m, _ = rt.lane_plan(cost, 1e12, 1.0)
    nw = m.size // 64
    ticks = gen.integers(100, 1000, nw).astype(np.int64)
    ticks[3], ticks[7] = 5000, 4000  # the measured tail: waves 3 and 7 (within 0.75 of the longest)
    lone = np.flatnonzero((m.reshape(-1, 64) >= 0).sum(1) == 1)
    if lone.size:  # a one-pixel wave in the tail stays whole
        ticks[lone[0]] = 4500
    out, nsplit = rt.lane_refine(m, cost, ticks, 0.75)
    check_perm(out, slots)
    assert nsplit == 4 and out.size == m.size + 2 * 64
    rows = [r[r >= 0] for r in out.reshape(-1, 64)]
    for w in (3, 7):
        px = m.reshape(-1, 64)[w]
        px = px[px >= 0]
        by = px[np.argsort(-cost[px].astype(np.int64), kind="stable")]
        halves = [list(by[0::2]), list(by[1::2])]
        assert sum(list(r) in halves for r in rows) == 2, w
    # waves kept whole come out longest first (the lone-pixel wave at 4,500 ticks ahead of all)
    est = {}
    mw = m.reshape(-1, 64)
    for w in range(nw):
        px = tuple(sorted(mw[w][mw[w] >= 0]))
        est[px] = float(ticks[w])
    got = [est.get(tuple(sorted(r)), None) for r in rows]
    whole = [g for g in got if g is not None]
    assert whole == sorted(whole, reverse=True)
    if lone.size:
        assert got[0] == 4500.0


def test_lane_refine_bad_arguments(rt):
    m = np.arange(128, dtype=np.int32)
    cost = np.ones(128, dtype=np.uint32)
    with pytest.raises(rt.RTError, match="lane_refine"):
        rt.lane_refine(m, cost, np.array([1, -1]), 0.75)  # negative clock
    with pytest.raises(rt.RTError, match="lane_refine"):
        rt.lane_refine(m, cost, np.array([1, 2]), 0.0)  # theta must be > 0
    bad = m.copy()
    bad[5] = 128
    with pytest.raises(rt.RTError, match="lane_refine"):
        rt.lane_refine(bad, cost, np.array([1, 2]), 0.75)  # slot outside the shard
    same, nsplit = rt.lane_refine(m, cost, np.zeros(2, dtype=np.int64), 0.75)  # nothing measured: no split
    assert nsplit == 0 and np.array_equal(same, m)
