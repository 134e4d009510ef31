"""The oracle's restatement of glm (oracle/rt_oracle.c: intersectRayTriangle, intersectRaySphere,
normalize / cross / dot / reflect / mix / min / max / clamp, quat * vec3, the camera's
quat / mat4_cast / translate / scale / perspectiveRH / inverse chain, rotate, mat4 * vec4) pinned
bit for bit against the reference's OWN vendored glm 0.9.9.8 (/root/reference/include/glm),
compiled here by oracle/build_ref.sh (oracle/ref_glm.cpp; no other reference file, no stand-in):

  * test_oracle_matches_glm_vectors: against tests/golden/glm_vectors.npz, the glm outputs
    tools/make_glm_vectors.py recorded for the seeded inputs of tests/glm_cases.py (runs anywhere);
  * test_oracle_matches_reference_glm_live: against the live library on 16x as many fresh inputs
    (where /root/reference was present for build())."""
import ctypes
import os

import numpy as np
import pytest

import glm_cases as G
import rt_testlib as T

REF_LIB = os.path.join(T.ROOT, "oracle", "_ref", "libref_glm.so")
VECTORS = os.path.join(T.GOLDEN, "glm_vectors.npz")


def _bits_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype == np.float32:
        return np.array_equal(a.view(np.uint32), b.view(np.uint32)) or np.array_equal(a, b, equal_nan=True)
    return np.array_equal(a, b)


_LIBM = ctypes.CDLL("libm.so.6")
_LIBM.cosf.restype = _LIBM.sinf.restype = ctypes.c_float
_LIBM.cosf.argtypes = _LIBM.sinf.argtypes = [ctypes.c_float]


def camera_libm_agrees(ang):
    """glm's quat(vec3(radians(ax), radians(ay), 0)) calls std::cos / std::sin on floats (glibc
    cosf / sinf here; MSVC's in the reference build); the oracle rounds the double-precision
    functions.  Where the two libms differ by an ulp the camera differs by a few ulps: those
    cases pin nothing about the restatement, so they are compared within 8 ulps instead."""
    import math
    ok = []
    for ax, ay in ang:
        good = True
        for deg in (ax, ay, 0.0):
            r = np.float32(np.float32(deg) * np.float32(0.01745329251994329576923690768489)) * np.float32(0.5)
            good &= _LIBM.cosf(float(r)) == np.float32(math.cos(float(r))) and _LIBM.sinf(float(r)) == np.float32(math.sin(float(r)))
        ok.append(bool(good))
    return np.array(ok)


def _compare(got, want, cam_ok=None):
    if cam_ok is not None:  # libm-dependent cameras: within 8 ulps, the rest bit for bit
        g, w = got["camera_out"], want["camera_out"]
        ulps = np.abs(g.view(np.int32).astype(np.int64) - w.view(np.int32).astype(np.int64))
        assert (ulps[~cam_ok] <= 8).all(), ulps[~cam_ok].max()
        got = dict(got, camera_out=g[cam_ok])
        want = dict(want, camera_out=w[cam_ok])
    bad = {}
    for k, w in want.items():
        g = got[k]
        if not _bits_equal(g, w):
            diff = np.flatnonzero(~((g == w) | (np.isnan(g) & np.isnan(w))).reshape(len(w), -1).all(1)) \
                if g.dtype == np.float32 else np.flatnonzero(g != w)
            bad[k] = diff[:5].tolist()
    return bad


def test_oracle_matches_glm_vectors():
    z = np.load(VECTORS)  # data only: no pickle
    cases = {}
    for k in ("tri", "sphere", "vec", "quat", "camera", "trs"):
        cases[k] = [z[f"in_{k}_{j}"] for j in range(10) if f"in_{k}_{j}" in z]
    got = G.run_all(T.oracle(), "oracle_glm_", cases)
    want = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    cam_ok = camera_libm_agrees(cases["camera"][1])
    assert cam_ok.sum() >= len(cam_ok) - 4 and cam_ok[0]
    bad = _compare(got, want, cam_ok)
    assert not bad, f"oracle != reference glm at (first indices): {bad}"
    # the cases exercise both outcomes of every test
    assert 0 < want["tri_hit"].sum() < len(want["tri_hit"]) and 0 < want["sphere_hit"].sum() < len(want["sphere_hit"])


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="oracle/_ref/libref_glm.so not built (needs /root/reference)")
def test_oracle_matches_reference_glm_live():
    ref = ctypes.CDLL(REF_LIB)
    cases = G.make_cases(scale=16)
    cases["tri"] = G.tri_cases(4096 * 16, seed=101)
    want = G.run_all(ref, "ref_", cases)
    got = G.run_all(T.oracle(), "oracle_glm_", cases)
    bad = _compare(got, want, camera_libm_agrees(cases["camera"][1]))
    assert not bad, f"oracle != reference glm at (first indices): {bad}"
