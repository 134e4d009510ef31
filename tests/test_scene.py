"""Product host code (C++ Scene/BVH/Camera mirror) against the independent C oracle:
byte-identical scene arrays, BVH and camera basis.  No GPU work."""
import hashlib
import json
import os

import numpy as np
import pytest

import rt_testlib as T

GOLD = json.load(open(os.path.join(T.GOLDEN, "golden.json")))


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("which", ["bunny", "bunny4"])
def test_scene_arrays_match_oracle(which):
    p = T.product_scene(which).host_arrays()
    o = T.OracleScene(which).arrays()
    for k in ("vertices", "faces", "nodes", "face_indices"):
        assert p[k].shape == o[k].shape and np.array_equal(p[k], o[k]), k


def test_bunny4_counts():
    g = GOLD["bunny4_scene"]
    assert g["faces"] == 555622  # 277,804 geometric triangles x2 + 14
    p = T.product_scene("bunny4").host_arrays()
    assert sha(p["nodes"]) == g["nodes_sha256"] and sha(p["face_indices"]) == g["face_indices_sha256"]


def test_plane_grid_matches_oracle():
    rt = T.load_rt()
    s = rt.Scene()
    s.setup_plane(40)
    s.set_viewport(64, 36)
    s.build()
    p = s.host_arrays()
    o = T.OracleScene("plane1m", grid_n=40).arrays()
    assert len(p["faces"]) // 16 == 2 * 40 * 40
    for k in ("vertices", "faces", "nodes", "face_indices"):
        assert np.array_equal(p[k], o[k]), k


@pytest.mark.parametrize("w,h,ax,ay,pos", [(1920, 1080, 0, 180, (0, 0, 0)), (256, 256, 0, 180, (0, 0, 0)),
                                           (61, 37, 12.5, -33.0, (1.5, -2.0, 3.25))])
def test_camera_matches_oracle(w, h, ax, ay, pos):
    rt = T.load_rt()
    s = rt.Scene()
    s.setup("bunny")
    s.set_camera(pos, ax, ay)
    s.set_viewport(w, h)
    s.build()
    cam = np.frombuffer(bytes(s.camera()), dtype=np.float32)
    o = T.OracleScene("bunny")
    import ctypes
    o_pos = (ctypes.c_float * 3)(*pos)
    T.oracle().oracle_set_camera(o.h, o_pos, ax, ay)
    assert np.array_equal(cam, o.camera(w, h))
    if (w, h, ax, ay) == (1920, 1080, 0, 180):
        assert [float(x) for x in cam] == GOLD["camera_1920x1080"]


def test_bvh_invariants():
    s = T.product_scene("bunny")
    a = s.host_arrays()
    nodes = a["nodes"].view(np.float32).reshape(-1, 8)
    ints = a["nodes"].view(np.uint32).reshape(-1, 8)
    first, count = ints[:, 6], ints[:, 7]
    fi = a["face_indices"].view(np.uint32)
    assert np.array_equal(np.sort(fi), np.arange(len(fi), dtype=np.uint32))  # a permutation
    leaves = count > 0
    assert count[leaves].sum() == len(fi)
    inner = np.where(~leaves)[0]
    for c in (first[inner], first[inner] + 1):  # children inside the parent box
        assert (nodes[c, :3] >= nodes[inner, :3]).all() and (nodes[c, 3:6] <= nodes[inner, 3:6]).all()
    assert s.max_depth() == 25


def test_triangle_mirror_records():
    """The kernel's leaf-ordered mirror (mirror.h): record i = faces[face_indices[i]] with the
    fp32 edges glm forms (v1 - v0, v2 - v0; GPUFace field order v0, v2, v1) and the face id."""
    s = T.product_scene("bunny")
    tris = s.mirror()
    a = s.host_arrays()
    fi = np.frombuffer(a["face_indices"].tobytes(), dtype=np.uint32)
    faces = np.frombuffer(a["faces"].tobytes(), dtype=np.uint32).reshape(-1, 4)
    pos = np.frombuffer(a["vertices"].tobytes(), dtype=np.float32).reshape(-1, 8)[:, 0:3]
    f = faces[fi]
    v0, v2, v1 = pos[f[:, 0]], pos[f[:, 1]], pos[f[:, 2]]
    assert tris.shape == (len(fi), 12)
    assert np.array_equal(tris[:, 0:3], v0)
    assert np.array_equal(tris[:, 3:6], v1 - v0)
    assert np.array_equal(tris[:, 6:9], v2 - v0)
    assert np.array_equal(tris[:, 9].view(np.uint32), fi)


@pytest.mark.parametrize("which", ["bunny", "bunny4"])
def test_private_node_array(which):
    """The traversal's private node array (mirror.h nodes): the reference's tree renumbered, node for
    node the same boxes and leaf ranges, every sibling pair on a 64-B boundary, pairs numbered in the
    right-first pre-order of BVHRayHit's DFS (main_raytracing.cu:75-76), so the DFS's visit sequence
    over the private array equals the reference's node by node."""
    rt = T.load_rt()
    s = rt.Scene()
    s.setup(which)
    s.build()
    ref = s.host_arrays()["nodes"].view(np.float32).reshape(-1, 8)
    refu = ref.view(np.uint32)
    prv = s.mirror_nodes()
    prvu = prv.view(np.uint32)
    # walk both trees in the reference's DFS order (push left, push right, pop right first)
    st = [(0, 0)]
    seen, pairs_in_order = 0, []
    while st:
        a, b = st.pop()
        seen += 1
        assert np.array_equal(ref[a, :6].view(np.uint32), prv[b, :6].view(np.uint32)), (a, b)
        assert refu[a, 7] == prvu[b, 7]
        if refu[a, 7] > 0:
            assert refu[a, 6] == prvu[b, 6], "a leaf keeps its triangle range"
            continue
        fa, fb = int(refu[a, 6]), int(prvu[b, 6])
        assert fb % 2 == 0 and (fb * 32) % 64 == 0, "sibling pairs start on a 64-B boundary"
        pairs_in_order.append(fb)
        st.append((fa, fb))
        st.append((fa + 1, fb + 1))
    assert seen == prv.shape[0] - 1, "every private slot but the padding is reached once"
    # the pairs are numbered in the order the DFS first reaches them (right-first pre-order)
    assert pairs_in_order == sorted(pairs_in_order)
    assert pairs_in_order[0] == 2 and pairs_in_order[-1] == prv.shape[0] - 2


def test_big_leaf_screen_records():
    """With rt_build_options.leaf_screens, big leaves whose core (all but the few big "outlier"
    triangles) has a normal cone narrow enough for cluster_cull get a screen record (mirror.h pf = 3;
    rt_fast.h screen_leaf): the 4-bunny scene's 21-triangle leaf does; the bunny scene's 345-triangle
    floor leaf does not (its core's cone spans ~90 degrees, so no ray could ever be culled)."""
    rt = T.load_rt()
    counts = {}
    rt.set_build_options(leaf_screens=1)  # an opt-in A/B (measured slower on config 4)
    try:
        for which in ("bunny", "bunny4"):
            counts[which] = _big_leaf_flags(rt, which)
        assert _big_leaf_flags(rt, "bunny4")[21] == 3
    finally:
        rt.set_build_options()
    assert _big_leaf_flags(rt, "bunny4")[21] == 1, "off by default"
    assert counts["bunny"] == {345: 1}
    assert counts["bunny4"][21] == 3 and counts["bunny4"][12318] == 2 and counts["bunny4"][903] == 1


def _big_leaf_flags(rt, which):
    """{leaf size: pf} of a scene's big leaves (mirror.h lead records)."""
    if True:
        s = rt.Scene()
        s.setup(which)
        s.build()
        tris = s.mirror().view(np.uint32)
        nodes = s.host_arrays()["nodes"].view(np.uint32).reshape(-1, 8)
        big = nodes[(nodes[:, 7] > 8)]
        return {int(n[7]): int(tris[n[6], 11]) for n in big}


@pytest.mark.parametrize("which", ["bunny", "bunny4"])
def test_twin_quads_and_bound(which):
    """mirror.h quads: every big leaf (pair records) lists each of its triangles exactly once, as a
    quad member or as the twin (same v0, e1 and e2 swapped, bit for bit) of one -- nearly all of them
    are twins, the reference adds every loaded face twice (Scene.cpp:103-127).  And the twin test
    (rt_fast.h twin_rejected, run here on the host by the same code): over rays aimed at the edges and
    vertices, grazing the plane and random, a twin it declares rejected never passes glm's predicate,
    while it does decide most rays."""
    import ctypes
    rt = T.load_rt()
    s = rt.Scene()
    s.setup(which)
    s.build()
    tris = s.mirror()
    tu = tris.view(np.uint32).reshape(-1, 12)
    leads = [i for i in range(tu.shape[0]) if tu[i, 11] in (1, 3)]
    assert leads
    nodes = s.host_arrays()["nodes"].view(np.uint32).reshape(-1, 8)
    counts = {int(n[6]): int(n[7]) for n in nodes if n[7] > 0}
    twins = 0
    for f in leads:
        c = counts[f]
        nq = int(tu[f + 1, 11])
        keys = {}
        for i in range(c):
            r = tu[f + i]
            keys.setdefault((r[:3].tobytes(), r[3:6].tobytes(), r[6:9].tobytes()), []).append(i)
        tw = sum(1 for i in range(c) if (tu[f + i, :3].tobytes(), tu[f + i, 6:9].tobytes(), tu[f + i, 3:6].tobytes()) in keys)
        twins += tw
        assert (c + 3) // 4 <= nq <= (c + 1) // 2, "two units (a triangle and its twin, or a lone triangle) per quad"
    assert twins > 0.9 * sum(counts[f] for f in leads), "big leaves are twins (Scene.cpp:103-127)"
    lib = rt.lib()
    gen = np.random.default_rng(7)
    f = max(leads, key=lambda x: counts[x])
    rec = tris[f:f + counts[f]]
    bad = decided = total = 0
    for k in range(min(counts[f], 120)):
        r = np.ascontiguousarray(rec[k], dtype=np.float32)
        v0, e1, e2 = r[:3], r[3:6], r[6:9]
        pts = [v0, v0 + e1, v0 + e2, v0 + 0.5 * e1, v0 + 0.5 * e2, v0 + 0.5 * (e1 + e2)]
        nrm = np.cross(e1.astype(np.float64), e2.astype(np.float64))
        nrm /= np.linalg.norm(nrm) + 1e-300
        for trial in range(60):
            target = pts[trial % len(pts)] + gen.normal(size=3) * 10.0 ** gen.uniform(-7, -1) * np.abs(e1).max()
            o = (target + gen.normal(size=3) * 10.0 ** gen.uniform(-1, 2)).astype(np.float32)
            d = (target - o).astype(np.float64)
            if trial % 3 == 1:  # grazing: nearly in the triangle's plane
                d -= nrm * (d @ nrm) * (1 - 10.0 ** gen.uniform(-7, -1))
            if trial % 5 == 4:
                d = gen.normal(size=3)
            nd = (d / np.linalg.norm(d)).astype(np.float32)
            b = lib.rt_twin_check_host(r.ctypes.data, o.ctypes.data, nd.ctypes.data)
            total += 1
            decided += b & 1
            bad += (b & 1) and (b & 2)
    assert bad == 0, f"{bad} twins declared rejected but accepted by glm's predicate"
    assert decided > 0.5 * total, (decided, total)


@pytest.mark.parametrize("which", ["bunny", "bunny4"])
def test_twin_records_cover_every_triangle_once(which):
    """mirror.h quads / units of every big leaf with pair records: each leaf position appears exactly
    once, as a unit's triangle or as its twin; a unit record is the leaf's record with the twin's face
    and packed positions, a twin record is the same v0 with e1 and e2 swapped bit for bit; kd < 0
    exactly when there is no twin; quads hold the units two by two in the packed-pair layout."""
    rt = T.load_rt()
    s = rt.Scene()
    s.setup(which)
    s.build()
    tris = s.mirror()
    tu = tris.view(np.uint32).reshape(-1, 12)
    quads, units = s.mirror_twins()
    qu, uu = quads.view(np.uint32), units.view(np.uint32)
    nodes = s.host_arrays()["nodes"].view(np.uint32).reshape(-1, 8)
    counts = {int(n[6]): int(n[7]) for n in nodes if n[7] > 0}
    leads = [i for i in range(tu.shape[0]) if tu[i, 11] in (1, 3)]
    assert leads
    for f in leads:
        c = counts[f]
        qb, nq, ub, nu = int(tu[f + 1, 10]), int(tu[f + 1, 11]), int(tu[f + 2, 10]), int(tu[f + 2, 11])
        assert nq == (nu + 1) // 2
        seen = []
        for k in range(nu):
            r, w = units[ub + k], int(uu[ub + k, 11])
            pos, twin = w & 0xFFFF, w >> 16
            assert np.array_equal(uu[ub + k, :10], tu[f + pos, :10])
            seen.append(pos)
            if twin != 0xFFFF:
                seen.append(twin)
                assert np.array_equal(tu[f + twin, 0:3], uu[ub + k, 0:3])
                assert np.array_equal(tu[f + twin, 3:6], uu[ub + k, 6:9]) and np.array_equal(tu[f + twin, 6:9], uu[ub + k, 3:6])
                assert uu[ub + k, 10] == tu[f + twin, 9] and r[12] >= 0
            else:
                assert r[12] < 0
            # the quad holding this unit: half k % 2 of quad k // 2 (pairs layout, mirror.h)
            q, h = qb + k // 2, k % 2
            assert qu[q, 0 + h] == uu[ub + k, 0] and qu[q, 18 + h] == uu[ub + k, 9]
            assert qu[q, 24 + h] == uu[ub + k, 11] and (quads[q, 20 + h] < 0) == (r[12] < 0)
        assert sorted(seen) == list(range(c)), "every position once"


def test_overlapping_big_leaves_get_no_twins():
    """a big leaf's twin metadata sits in words 10-11 of its second and third records.  A
    foreign BVH whose big-leaf ranges overlap with different starts would let one leaf's metadata overwrite
    another's first record; rt_build_mirror then builds no twins at all (pairs only, exact either way), and
    every big leaf's first record keeps its own (first pair, kind).  The reference's own tree builds twins."""
    rt = T.load_rt()
    s = rt.Scene()
    s.setup("bunny")
    s.build()
    arr = s.host_arrays()
    nodes = arr["nodes"].view(np.uint32).reshape(-1, 8).copy()
    fi = arr["face_indices"].view(np.uint32)
    faces = arr["faces"].view(np.uint32).reshape(-1, 4)
    verts = arr["vertices"].view(np.float32).reshape(-1, 8)
    meta, twins = rt.mirror_build_check(nodes, fi, faces, verts)
    assert twins
    assert np.array_equal(meta, s.mirror().view(np.uint32).reshape(-1, 12)[:, 10:12])
    big = [int(n[6]) for n in nodes if n[7] > 8]
    assert big
    f = big[0]
    # a small leaf re-pointed at [f + 1, f + 21): a second big leaf starting at the first one's second record
    small = next(i for i, n in enumerate(nodes) if 0 < n[7] <= 8)
    nodes[small, 6], nodes[small, 7] = f + 1, 20
    meta2, twins2 = rt.mirror_build_check(nodes, fi, faces, verts)
    assert not twins2
    for lead in (f, f + 1):
        assert meta2[lead, 1] in (1, 3), f"big leaf at {lead} lost its first-record kind"
    assert meta2[f, 0] != meta2[f + 1, 0], "each big leaf points at its own pairs"


def test_face_leaf_table():
    """The deferred leaves' guard table (mirror.h face_leaf, rt_fast.h): for a scene with big leaves, every
    face maps to the private node of the one leaf that holds it -- whose box is then the box the reference
    tests before that face (main_raytracing.cu:43-71) -- checked against the reference arrays walked
    independently."""
    rt = T.load_rt()
    for which in ("bunny", "bunny4"):
        _check_face_leaf(rt, which)


def _check_face_leaf(rt, which):
    s = rt.Scene()
    s.setup(which)
    s.build()
    fl = s.mirror_face_leaf()
    arrays = s.host_arrays()
    ref = arrays["nodes"].view(np.float32).reshape(-1, 8)
    refu = ref.view(np.uint32)
    fidx = arrays["face_indices"].view(np.uint32)
    prv = s.mirror_nodes()
    prvu = prv.view(np.uint32)
    assert fl.size == arrays["faces"].size // 16
    # the reference's leaf of every face, through the same paired DFS as test_private_node_array
    want = np.full(fl.size, 0xFFFFFFFF, dtype=np.uint64)
    st = [(0, 0)]
    while st:
        a, b = st.pop()
        if refu[a, 7] > 0:
            f0, n = int(refu[a, 6]), int(refu[a, 7])
            faces = fidx[f0:f0 + n]
            assert np.all(want[faces] == 0xFFFFFFFF), "a face in two leaves"
            want[faces] = b
            assert np.array_equal(ref[a, :6].view(np.uint32), prv[b, :6].view(np.uint32))
            continue
        fa, fb = int(refu[a, 6]), int(prvu[b, 6])
        st.append((fa, fb))
        st.append((fa + 1, fb + 1))
    assert np.array_equal(fl.astype(np.uint64), want)
    assert np.count_nonzero(fl == 0xFFFFFFFF) == 0
