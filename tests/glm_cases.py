"""Seeded inputs for pinning the oracle's glm restatement (oracle/rt_oracle.c) against the
reference's vendored glm (oracle/ref_glm.cpp): rays aimed at triangle interiors, edges and
vertices, grazing and parallel rays, degenerate and tiny/huge triangles, signed zeros, NaN and
infinite components -- the cases where a restatement could differ by operation order."""
import numpy as np

F = np.float32


def _ulp_jitter(g, x, k=4):
    return np.nextafter(x, np.where(g.random(x.shape) < 0.5, -np.inf, np.inf).astype(F)) if k else x


def tri_cases(n, seed=1):
    g = np.random.default_rng(seed)
    scale = F(10.0) ** g.integers(-3, 4, (n, 1)).astype(F)
    v0 = (g.standard_normal((n, 3)) * scale).astype(F)
    v1 = (v0 + g.standard_normal((n, 3)) * scale * F(0.3)).astype(F)
    v2 = (v0 + g.standard_normal((n, 3)) * scale * F(0.3)).astype(F)
    o = (g.standard_normal((n, 3)) * scale * F(5)).astype(F)
    # aim: barycentric target inside, on an edge / vertex, or just outside
    w = g.random((n, 3)).astype(F)
    kind = g.integers(0, 6, n)
    w[kind == 1, 0] = 0  # edge
    w[kind == 2, 0:2] = 0  # vertex
    w[kind == 3, 0] = -1e-6  # just outside
    w = w / np.where(np.abs(w.sum(1, keepdims=True)) > 0, w.sum(1, keepdims=True), 1)
    target = (w[:, :1] * v0 + w[:, 1:2] * v1 + w[:, 2:3] * v2).astype(F)
    d = (target - o).astype(F)
    # grazing: direction almost in the triangle's plane
    gz = kind == 4
    nrm = np.cross(v1 - v0, v2 - v0)
    nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-30)
    d[gz] = (d[gz] - (np.sum(d[gz] * nrm[gz], 1, keepdims=True) * (1 - 1e-6)) * nrm[gz]).astype(F)
    # degenerate triangles
    dg = kind == 5
    v2[dg] = v1[dg]
    # random rays for the rest of the variety
    rnd = g.random(n) < 0.15
    d[rnd] = g.standard_normal((rnd.sum(), 3)).astype(F)
    # specials: signed zeros, NaN, inf, zero direction
    sp = g.choice(n, max(1, n // 50), replace=False)
    for j, i in enumerate(sp):
        c = j % 5
        if c == 0:
            d[i, g.integers(0, 3)] = F(-0.0)
        elif c == 1:
            o[i, g.integers(0, 3)] = F(np.nan)
        elif c == 2:
            v1[i, g.integers(0, 3)] = F(np.inf)
        elif c == 3:
            d[i] = 0
        else:
            o[i] = v0[i]
    return [np.ascontiguousarray(x, dtype=F) for x in (o, d, v0, v1, v2)]


def sphere_cases(n, seed=2):
    g = np.random.default_rng(seed)
    c = (g.standard_normal((n, 3)) * 50).astype(F)
    r = (np.abs(g.standard_normal(n)) * 10 + 1e-3).astype(F)
    o = (g.standard_normal((n, 3)) * 80).astype(F)
    aim = (c + g.standard_normal((n, 3)) * r[:, None] * F(1.1)).astype(F)
    d = (aim - o).astype(F)
    inside = g.random(n) < 0.1
    o[inside] = c[inside]
    tang = g.random(n) < 0.05
    d[tang] = np.cross(c[tang] - o[tang], g.standard_normal((tang.sum(), 3))).astype(F)
    return [np.ascontiguousarray(x, dtype=F) for x in (o, d, c, r)]


def vec_cases(n, seed=3):
    g = np.random.default_rng(seed)
    a = (g.standard_normal((n, 3)) * F(10.0) ** g.integers(-2, 3, (n, 1))).astype(F)
    b = g.standard_normal((n, 3)).astype(F)
    b /= np.linalg.norm(b, axis=1, keepdims=True).astype(F)
    s = g.random(n).astype(F)
    sp = g.choice(n, max(1, n // 20), replace=False)
    a[sp[::3], 0] = F(np.nan)
    b[sp[1::3], 0] = F(np.nan)
    a[sp[2::3]] = F(-0.0)
    a[g.random(n) < 0.05] *= F(100)  # over the clamp
    return [np.ascontiguousarray(x, dtype=F) for x in (a, b, s)]


def quat_cases(n, seed=4):
    g = np.random.default_rng(seed)
    q = g.standard_normal((n, 4)).astype(F)
    q /= np.linalg.norm(q, axis=1, keepdims=True).astype(F)
    q[0] = (F(-4.371139e-08), 0, 1, 0)  # quat(vec3(0, PI, 0)) of the sky (main_raytracing.cu:151)
    v = g.standard_normal((n, 3)).astype(F)
    return [np.ascontiguousarray(x, dtype=F) for x in (q, v)]


def camera_cases(n, seed=5):
    g = np.random.default_rng(seed)
    pos = (g.standard_normal((n, 3)) * 50).astype(F)
    ang = (g.random((n, 2)) * 360 - 180).astype(F)
    wh = g.integers(16, 4096, (n, 2)).astype(np.int32)
    pos[0], ang[0], wh[0] = (0, 0, 0), (0, 0), (1920, 1080)
    return pos, ang, wh


def trs_cases(n, seed=6):
    g = np.random.default_rng(seed)
    pos = (g.standard_normal((n, 3)) * 50).astype(F)
    ang = (g.random(n) * 7 - 3.5).astype(F)
    axis = g.standard_normal((n, 3)).astype(F)
    scl = (np.abs(g.standard_normal((n, 3))) * 100 + 0.1).astype(F)
    ang[0], axis[0] = F(-3.14159265358979323846), (0, 1, 0)  # the bunny's set-up rotations
    ang[1], axis[1] = F(3.14159265358979323846 / 2), (1, 0, 0)
    return pos, ang, axis, scl


def _p(a):
    import ctypes
    return a.ctypes.data_as(ctypes.c_void_p)


def run_all(lib, prefix, cases):
    """Evaluate every case set through `lib` (ref_* of libref_glm.so or oracle_glm_* of
    liboracle.so: same signatures).  Returns a dict of output arrays."""
    import ctypes
    I64 = ctypes.c_int64
    out = {}
    o, d, v0, v1, v2 = cases["tri"]
    n = len(o)
    hit, res = np.zeros(n, np.int32), np.zeros((n, 3), F)
    getattr(lib, prefix + "tri_batch")(I64(n), _p(o), _p(d), _p(v0), _p(v1), _p(v2), _p(hit), _p(res))
    out["tri_hit"], out["tri_out"] = hit, np.where(hit[:, None] != 0, res, F(0))
    o, d, c, r = cases["sphere"]
    n = len(o)
    hit, dist = np.zeros(n, np.int32), np.zeros(n, F)
    getattr(lib, prefix + "sphere_batch")(I64(n), _p(o), _p(d), _p(c), _p(r), _p(hit), _p(dist))
    out["sphere_hit"], out["sphere_dist"] = hit, np.where(hit != 0, dist, F(0))
    a, b, s = cases["vec"]
    n = len(a)
    res = np.zeros((n, 18), F)
    getattr(lib, prefix + "vec_batch")(I64(n), _p(a), _p(b), _p(s), _p(res))
    out["vec_out"] = res
    q, v = cases["quat"]
    res = np.zeros((len(q), 3), F)
    getattr(lib, prefix + "quat_rotate_batch")(I64(len(q)), _p(q), _p(v), _p(res))
    out["quat_out"] = res
    pos, ang, wh = cases["camera"]
    res = np.zeros((len(pos), 12), F)
    for i in range(len(pos)):
        buf = np.zeros(12, F)
        if prefix == "ref_":
            lib.ref_camera(_p(pos[i]), ctypes.c_float(ang[i, 0]), ctypes.c_float(ang[i, 1]), ctypes.c_float(90.0),
                           ctypes.c_float(float(wh[i, 0])), ctypes.c_float(float(wh[i, 1])), _p(buf))
        else:
            lib.oracle_glm_camera(_p(pos[i]), ctypes.c_float(ang[i, 0]), ctypes.c_float(ang[i, 1]), int(wh[i, 0]),
                                  int(wh[i, 1]), _p(buf))
        res[i] = buf
    out["camera_out"] = res
    pos, ang, axis, scl = cases["trs"]
    trs, inv = np.zeros((len(pos), 16), F), np.zeros((len(pos), 16), F)
    for i in range(len(pos)):
        getattr(lib, prefix + "trs")(_p(pos[i]), ctypes.c_float(ang[i]), _p(axis[i]), _p(scl[i]), _p(trs[i]))
        getattr(lib, prefix + "inverse")(_p(trs[i]), _p(inv[i]))
    out["trs_out"], out["inv_out"] = trs, inv
    pts = np.ascontiguousarray(cases["vec"][0][:256])
    app = np.zeros((len(pts), 6), F)
    m1, m2 = np.ascontiguousarray(trs[0]), np.ascontiguousarray(trs[1])
    getattr(lib, prefix + "mat_apply_batch")(I64(len(pts)), _p(m1), _p(m2), _p(pts), _p(app))
    out["apply_out"] = app
    return out


def make_cases(scale=1):
    return {"tri": tri_cases(4096 * scale), "sphere": sphere_cases(2048 * scale), "vec": vec_cases(2048 * scale),
            "quat": quat_cases(512 * scale), "camera": camera_cases(64), "trs": trs_cases(64)}
