// rt_fast.h -- the fast traversal of the MI355X render kernel (included by rt_kernel.hip).
//
// Same decisions as BVHRayHit (main_raytracing.cu:33-81), bit for bit, re-organised for a
// wave64 SIMD machine:
//
// 1. Filtered-exact slab tests.  IntersectAABB (Math.h:50-61) divides (b - o) / d six
//    times per node; a correctly rounded fp32 division is ~10 instructions on gfx950.
//    Here q' = RN((b - o) * RN(1/d)) is used instead, whose relative error is below
//    2^-22.9 (two roundings of 2^-24).  Every decision the test makes is decided from q'
//    when it is further than 2^-20 (relative) from its threshold -- then it provably equals
//    the decision on the exact quotients -- and re-done with the exact IEEE quotients
//    otherwise (a ray grazing a box face; rare).  Signs and zeros of q' equal those of the
//    exact quotient, so `tmax > 0` is always decided exactly.  Rays and scenes outside the
//    range where the bound holds (|d| outside [2^-40, 2^20], origin or bound components
//    outside {0} u [2^-60, 2^62]) use the exact quotients throughout.
// 2. Branch-free triangle tests.  glm::intersectRayTriangle's accept predicate is
//    evaluated with selects (NaN-safe: the same `!(x < 0 || x > det)` forms); only an
//    accepted triangle pays the 1/det division and the distance (a rare, divergent branch).
// 3. Big-leaf synchronisation.  Leaves with more than BIG triangles (the bunny scene's
//    345-triangle floor leaf gets 96 % of all tests) are not entered until every lane of
//    the wave is either done or waiting at a big leaf; the waiting lanes then run their
//    leaves together, reading the triangles with scalar loads when they all wait at the
//    same one.  Each lane still processes its nodes and leaves in the reference's DFS order.
#pragma once

namespace rtfast {

constexpr int BIG = 8;  // leaves above this size wait for the wave

using rtm::f3;

struct Ray {
    f3 o, d, nd, r;  // origin, direction (unnormalised), normalised direction, RN(1/d)
    bool fast;       // the q' error bound applies to this ray
};

__device__ __forceinline__ bool in_range_or_zero(float v, float lo, float hi) {
    const float a = fabsf(v);
    return v == 0.0f || (a >= lo && a <= hi);
}

__device__ __forceinline__ Ray make_ray(f3 o, f3 d, f3 nd, bool scene_fast) {
    Ray R;
    R.o = o, R.d = d, R.nd = nd;
    R.r = rtm::mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    const float dlo = 0x1p-40f, dhi = 0x1p20f;
    const bool dok = fabsf(d.x) >= dlo && fabsf(d.x) <= dhi && fabsf(d.y) >= dlo && fabsf(d.y) <= dhi &&
                     fabsf(d.z) >= dlo && fabsf(d.z) <= dhi;
    const bool ook = in_range_or_zero(o.x, 0x1p-60f, 0x1p62f) && in_range_or_zero(o.y, 0x1p-60f, 0x1p62f) &&
                     in_range_or_zero(o.z, 0x1p-60f, 0x1p62f);
    R.fast = scene_fast && dok && ook;
    return R;
}

// Node as two float4: lo = (bmin.xyz, bmax.x), hi = (bmax.yz, first, count).
// Exact slab quantities (reference arithmetic: fminf/fmaxf of IEEE quotients).
__device__ __forceinline__ void slab_exact(const Ray& R, float4 lo, float4 hi, float* tmin_o, float* tmax_o) {
    float tx1 = (lo.x - R.o.x) / R.d.x, tx2 = (lo.w - R.o.x) / R.d.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    float ty1 = (lo.y - R.o.y) / R.d.y, ty2 = (hi.x - R.o.y) / R.d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2)), tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (lo.z - R.o.z) / R.d.z, tz2 = (hi.y - R.o.z) / R.d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2)), tmax = fminf(tmax, fmaxf(tz1, tz2));
    *tmin_o = tmin;
    *tmax_o = tmax;
}

// Approximate slab: same numerators (b - o, exact as in the reference), quotients by
// multiplication with RN(1/d).  Only called when R.fast (no NaN / inf / subnormal).
__device__ __forceinline__ void slab_approx(const Ray& R, float4 lo, float4 hi, float* tmin_o, float* tmax_o) {
    const float tx1 = (lo.x - R.o.x) * R.r.x, tx2 = (lo.w - R.o.x) * R.r.x;
    const float ty1 = (lo.y - R.o.y) * R.r.y, ty2 = (hi.x - R.o.y) * R.r.y;
    const float tz1 = (lo.z - R.o.z) * R.r.z, tz2 = (hi.y - R.o.z) * R.r.z;
    *tmin_o = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    *tmax_o = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
}

enum : int { NO = 0, YES = 1, UNSURE = 2 };

// `tmax >= tmin && tmax > 0` from approximations with relative error < 2^-22.9 each.
__device__ __forceinline__ int classify_ok(float tmin, float tmax) {
    if (!(tmax > 0.0f)) return NO;  // sign of tmax' == sign of tmax
    const float diff = tmax - tmin;
    const float m = (fabsf(tmax) + fabsf(tmin)) * 0x1p-20f;
    return diff > m ? YES : (diff < -m ? NO : UNSURE);
}

// `tmin < best` (best exact) from tmin' with relative error < 2^-22.9.
__device__ __forceinline__ int classify_lt(float tmin, float best) {
    const float m = fabsf(tmin) * 0x1p-20f;
    return (tmin + m < best) ? YES : ((tmin - m >= best) ? NO : UNSURE);
}

struct Hit {
    float best;
    int kind;     // 0 none, 1 sphere, 2 triangle
    uint32_t id;  // sphere index or face index
    float bx, by;
};

// Triangle records: A = (v0.xyz, e1.x), B = (e1.yz, e2.xy), C = (e2.z, face, -, -).
// glm::intersectRayTriangle (gtx/intersect.inl:29-94) as a predicate + the rare accept.
template <bool STATS, class C>
__device__ __forceinline__ void test_triangle(const Ray& R, float4 A, float4 B, float4 Cc, Hit& h, C& c) {
    const float eps = 1.1920928955078125e-07f;
    const f3 e1 = rtm::mk(A.w, B.x, B.y), e2 = rtm::mk(B.z, B.w, Cc.x);
    const f3 p = rtm::cross(R.nd, e2);
    const float det = rtm::dot(e1, p);
    const f3 dist = rtm::sub(R.o, rtm::mk(A.x, A.y, A.z));
    const float u = rtm::dot(dist, p);
    const f3 perp = rtm::cross(dist, e1);
    const float v = rtm::dot(R.nd, perp);
    const float uv = u + v;
    // det > eps: !(u < 0 || u > det) && !(v < 0 || u+v > det); det < -eps: the same with every
    // inequality reversed.  Flipping the signs of u, v, u+v and det by det's sign bit maps the
    // second case onto the first exactly (negation is exact; NaN compares stay false).
    const uint32_t sgn = __float_as_uint(det) & 0x80000000u;
    const float adet = fabsf(det);
    const float su = __uint_as_float(__float_as_uint(u) ^ sgn);
    const float sv = __uint_as_float(__float_as_uint(v) ^ sgn);
    const float suv = __uint_as_float(__float_as_uint(uv) ^ sgn);
    const bool ok = adet > eps && !(su < 0.0f || su > adet) && !(sv < 0.0f || suv > adet);
    if (STATS) c.tri++;
    if (ok) {
        const float inv_det = 1.0f / det;
        const float t = rtm::dot(e2, perp) * inv_det;
        if (!(t >= h.best || t < 0.0f)) {
            h.best = t;
            h.kind = 2;
            h.id = __float_as_uint(Cc.y);
            h.bx = u * inv_det;
            h.by = v * inv_det;
            if (STATS) c.tacc++;
        }
    }
}

typedef float f4v __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(4))) f4v* ConstF4;  // scalar-load (SMEM) view
__device__ __forceinline__ float4 ldc(ConstF4 p, uint32_t i) {
    const f4v v = p[i];
    return make_float4(v.x, v.y, v.z, v.w);
}

// Pop stack entries until one passes `tmin < closest` (the reference's pop-time test).
// SW == 2: entry = {node index | (tmin is exact) << 31, tmin bits}.
// SW == 1: entry = node index; tmin is recomputed from the node (the same slab arithmetic gives
// the same value, so the decision is the reference's), halving the LDS per lane.
template <int WAVE, int SW>
__device__ __forceinline__ bool pop(const float4* nodes4, uint32_t* stk, int& sp, const Ray& R, float best,
                                    uint32_t& first, uint32_t& count) {
    while (sp > 0) {
        sp--;
        const uint32_t w0 = stk[(sp * SW) * WAVE];
        const uint32_t idx = w0 & 0x7fffffffu;
        bool pass;
        if (SW == 1) {
            const float4 lo = nodes4[2 * idx], hi = nodes4[2 * idx + 1];
            int cl = UNSURE;
            float te, tx;
            if (R.fast) {
                slab_approx(R, lo, hi, &te, &tx);
                cl = classify_lt(te, best);
            }
            if (cl == UNSURE) {
                slab_exact(R, lo, hi, &te, &tx);
                pass = te < best;
            } else {
                pass = cl == YES;
            }
            if (pass) {
                first = __float_as_uint(hi.z), count = __float_as_uint(hi.w);
                return true;
            }
            continue;
        }
        const float t = __uint_as_float(stk[(sp * SW + 1) * WAVE]);
        if (w0 >> 31) {
            pass = t < best;
        } else {
            const int cl = classify_lt(t, best);
            if (cl == UNSURE) {
                float te, tx;
                slab_exact(R, nodes4[2 * idx], nodes4[2 * idx + 1], &te, &tx);
                pass = te < best;
            } else {
                pass = cl == YES;
            }
        }
        if (pass) {
            const float4 nh = nodes4[2 * idx + 1];
            first = __float_as_uint(nh.z), count = __float_as_uint(nh.w);
            return true;
        }
    }
    return false;
}

// One inner-node step: both children (adjacent in the node array) tested, the right child
// continued in registers, the left one continued or pushed, exactly as the reference's
// push(first), push(first+1), pop order.  Returns false when the lane must pop.
template <int WAVE, int SW, bool STATS, class C>
__device__ __forceinline__ bool inner_step(const float4* nodes4, uint32_t* stk, int& sp, const Ray& R, float best,
                                           uint32_t& first, uint32_t& count, C& c) {
    const float4 l0 = nodes4[2 * first], l1 = nodes4[2 * first + 1];
    const float4 r0 = nodes4[2 * first + 2], r1 = nodes4[2 * first + 3];
    if (STATS) c.node += 2;
    float tl = 0.0f, tlx = 0.0f, tr = 0.0f, trx = 0.0f;
    int okl = UNSURE, okr = UNSURE, rlt = UNSURE;
    if (R.fast) {
        slab_approx(R, l0, l1, &tl, &tlx);
        slab_approx(R, r0, r1, &tr, &trx);
        okl = classify_ok(tl, tlx);
        okr = classify_ok(tr, trx);
        rlt = okr == YES ? classify_lt(tr, best) : NO;
    }
    bool exact_l = false;
    if (okl == UNSURE || okr == UNSURE || rlt == UNSURE) {
        slab_exact(R, l0, l1, &tl, &tlx);
        slab_exact(R, r0, r1, &tr, &trx);
        okl = (tlx >= tl && tlx > 0.0f) ? YES : NO;
        okr = (trx >= tr && trx > 0.0f) ? YES : NO;
        rlt = (okr == YES && tr < best) ? YES : NO;
        exact_l = true;
    }
    if (rlt == YES) {
        if (okl == YES) {
            if (SW == 1) {
                stk[sp * WAVE] = first;
            } else {
                stk[(sp * 2) * WAVE] = first | (exact_l ? 0x80000000u : 0u);
                stk[(sp * 2 + 1) * WAVE] = __float_as_uint(tl);
            }
            sp++;
        }
        first = __float_as_uint(r1.z), count = __float_as_uint(r1.w);
        return true;
    }
    if (okl == YES) {
        bool llt;
        if (exact_l) {
            llt = tl < best;
        } else {
            const int cl = classify_lt(tl, best);
            if (cl == UNSURE) {
                float te, tx;
                slab_exact(R, l0, l1, &te, &tx);
                llt = te < best;
            } else {
                llt = cl == YES;
            }
        }
        if (llt) {
            first = __float_as_uint(l1.z), count = __float_as_uint(l1.w);
            return true;
        }
    }
    return false;
}

// A leaf kept resident in LDS by the workgroup (the scene's largest leaf; SoA records).
struct HotLeaf {
    const float4* a;  // LDS
    const float4* b;
    const float4* c;
    uint32_t first, count;  // count 0: none
};

// glm::intersectRayTriangle + BVHRayHit's accept test (`!(t >= best || t < 0)`) for one
// candidate; returns whether it would be accepted against threshold `best`, and reports a
// NaN distance of an otherwise accepted triangle (the sequential reference accepts a NaN t;
// a min-reduction would not, so such a ray is redone sequentially).
__device__ __forceinline__ bool tri_accept(f3 o, f3 nd, float4 A, float4 B, float4 Cc, float best, float* t_o,
                                           float* bx, float* by, bool* nan) {
    const float eps = 1.1920928955078125e-07f;
    const f3 e1 = rtm::mk(A.w, B.x, B.y), e2 = rtm::mk(B.z, B.w, Cc.x);
    const f3 p = rtm::cross(nd, e2);
    const float det = rtm::dot(e1, p);
    const f3 dist = rtm::sub(o, rtm::mk(A.x, A.y, A.z));
    const float u = rtm::dot(dist, p);
    const f3 perp = rtm::cross(dist, e1);
    const float v = rtm::dot(nd, perp);
    const float uv = u + v;
    const uint32_t sgn = __float_as_uint(det) & 0x80000000u;
    const float adet = fabsf(det);
    const float su = __uint_as_float(__float_as_uint(u) ^ sgn);
    const float sv = __uint_as_float(__float_as_uint(v) ^ sgn);
    const float suv = __uint_as_float(__float_as_uint(uv) ^ sgn);
    const bool ok = adet > eps && !(su < 0.0f || su > adet) && !(sv < 0.0f || suv > adet);
    if (!ok) return false;
    const float inv_det = 1.0f / det;
    const float t = rtm::dot(e2, perp) * inv_det;
    *nan = *nan || (t != t);
    if (t >= best || t < 0.0f) return false;
    *t_o = t;
    *bx = u * inv_det;
    *by = v * inv_det;
    return true;
}

__device__ __forceinline__ float bcast(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Cooperative big-leaf round: the waiting lanes (mask `big`) all wait at leaf [f0, f0+c0).
// Rays are taken one at a time; the 64 lanes split the leaf's triangles (lane l tests
// l, l+64, ...), each keeping its first strictly-closer candidate, and a (t, index)
// lexicographic arg-min over the wave gives exactly the triangle the sequential loop
// would end on (the first index attaining the minimum t below the ray's closest distance).
template <class C>
__device__ __forceinline__ void coop_leaf(const float4* tris, const HotLeaf& hot, unsigned long long big, uint32_t f0,
                                          uint32_t c0, const Ray& R, Hit& h, C& c) {
    const uint32_t lane = threadIdx.x & 63u;
    const bool resident = hot.count != 0 && f0 == hot.first && c0 == hot.count;
    unsigned long long m = big;
    while (m) {
        const int r = __ffsll((long long)m) - 1;
        m &= m - 1;
        const f3 rox = rtm::mk(bcast(R.o.x, r), bcast(R.o.y, r), bcast(R.o.z, r));
        const f3 nd = rtm::mk(bcast(R.nd.x, r), bcast(R.nd.y, r), bcast(R.nd.z, r));
        const float best0 = bcast(h.best, r);
        float bt = best0, bx = 0.0f, by = 0.0f;
        uint32_t bi = 0xffffffffu;
        bool nan = false;
        for (uint32_t j = lane; j < c0; j += 64u) {
            float4 A, B, Cc;
            if (resident) {
                A = hot.a[j], B = hot.b[j], Cc = hot.c[j];
            } else {
                A = tris[3 * (f0 + j)], B = tris[3 * (f0 + j) + 1], Cc = tris[3 * (f0 + j) + 2];
            }
            float t, x, y;
            if (tri_accept(rox, nd, A, B, Cc, bt, &t, &x, &y, &nan)) bt = t, bx = x, by = y, bi = j;
        }
        if (__ballot(nan)) {
            // sequential fallback for this ray (never taken for finite scenes)
            if ((int)lane == r) {
                float t, x, y;
                bool dummy = false;
                for (uint32_t j = 0; j < c0; j++) {
                    const float4 A = tris[3 * (f0 + j)], B = tris[3 * (f0 + j) + 1], Cc = tris[3 * (f0 + j) + 2];
                    if (tri_accept(R.o, R.nd, A, B, Cc, h.best, &t, &x, &y, &dummy)) {
                        h.best = t, h.kind = 2, h.bx = x, h.by = y;
                        h.id = __float_as_uint(Cc.y);
                    }
                }
            }
            continue;
        }
        // arg-min of (t, index) across the wave
        float mt = bt;
        uint32_t mi = bi;
        for (int off = 32; off > 0; off >>= 1) {
            const float ot = __shfl_xor(mt, off);
            const uint32_t oi = (uint32_t)__shfl_xor((int)mi, off);
            const bool take = ot < mt || (ot == mt && oi < mi);
            mt = take ? ot : mt;
            mi = take ? oi : mi;
        }
        mi = __builtin_amdgcn_readfirstlane(mi);
        if (mi != 0xffffffffu) {
            const int wl = (int)(mi & 63u);
            const float wbx = bcast(bx, wl), wby = bcast(by, wl), wt = bcast(bt, wl);
            if ((int)lane == r) {
                const float4 Cc = resident ? hot.c[mi] : tris[3 * (f0 + mi) + 2];
                h.best = wt, h.kind = 2, h.bx = wbx, h.by = wby;
                h.id = __float_as_uint(Cc.y);
            }
        }
    }
    (void)c;
}

// BVHRayHit for one lane (`live` = the lane has a segment to trace).  Every lane of the wave
// must call it (it synchronises big leaves across the wave).  STRIDE: the stack's lane stride.
template <int STRIDE, int SW, bool STATS, class C>
__device__ __forceinline__ void trace(const float4* nodes4, const float4* tris, const HotLeaf& hot, uint32_t tune,
                                      uint32_t* stk,
                                      const Ray& R, Hit& h, bool live, C& c) {
    bool active = false;
    uint32_t first = 0, count = 0;
    int sp = 0;
    if (live) {
        // root: IntersectAABB against the closest sphere distance
        const float4 lo = nodes4[0], hi = nodes4[1];
        if (STATS) c.node++;
        float tmin, tmax;
        slab_exact(R, lo, hi, &tmin, &tmax);
        active = tmax >= tmin && tmin < h.best && tmax > 0.0f;
        first = __float_as_uint(hi.z), count = __float_as_uint(hi.w);
    }
    for (;;) {
        const bool small = active && count <= (uint32_t)BIG;
        if (__ballot(small)) {
            if (STATS) {
                c.w_small += (threadIdx.x & 63) == 0;
                c.l_small += small;
            }
            if (small) {
                if (count > 0) {
                    for (uint32_t i = first; i < first + count; i++)
                        test_triangle<STATS>(R, tris[3 * i], tris[3 * i + 1], tris[3 * i + 2], h, c);
                    active = pop<STRIDE, SW>(nodes4, stk, sp, R, h.best, first, count);
                } else if (!inner_step<STRIDE, SW, STATS>(nodes4, stk, sp, R, h.best, first, count, c)) {
                    active = pop<STRIDE, SW>(nodes4, stk, sp, R, h.best, first, count);
                }
            }
            continue;
        }
        const unsigned long long big = __ballot(active);
        if (!big) break;
        // every waiting lane is at a big leaf: run them together
        // the leaf of the lowest waiting lane (not lane 0: it may be done, with stale state)
        const int l0 = __ffsll((long long)big) - 1;
        const uint32_t f0 = __builtin_amdgcn_readlane(first, l0);
        const uint32_t c0 = __builtin_amdgcn_readlane(count, l0);
        if (STATS) {
            uint32_t mx = active ? count : 0u;
            for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
            c.w_big += (threadIdx.x & 63) == 0 ? mx : 0;
            c.l_big += active ? count : 0;
        }
        if (__ballot(active && first == f0) == big) {
            const uint32_t k = (uint32_t)__popcll(big);
            const uint32_t chunks = (c0 + 63u) / 64u;
            if (!STATS && (tune & 1u) == 0 && k * (60u * chunks + 50u) < 50u * c0) {
                // cost model (VALU instructions): cooperative ~ k * (60 * chunks + 50), lane-parallel ~ 50 * c0
                coop_leaf(tris, hot, big, f0, c0, R, h, c);
            } else if (hot.count != 0 && f0 == hot.first && c0 == hot.count) {
                for (uint32_t i = 0; i < c0; i++) {
                    const float4 A = hot.a[i], B = hot.b[i], Cc = hot.c[i];
                    if (active) test_triangle<STATS>(R, A, B, Cc, h, c);
                }
            } else {
                // all waiting lanes share one leaf: scalar loads, next record prefetched
                ConstF4 st = (ConstF4)(tris + 3 * (size_t)f0);
                ConstF4 const last = st + 3 * (c0 - 1);
                float4 A = ldc(st, 0), B = ldc(st, 1), Cc = ldc(st, 2);
                for (uint32_t i = 0; i < c0; i++) {
                    st = st == last ? st : st + 3;
                    const float4 An = ldc(st, 0), Bn = ldc(st, 1), Cn = ldc(st, 2);
                    if (active) test_triangle<STATS>(R, A, B, Cc, h, c);
                    A = An, B = Bn, Cc = Cn;
                }
            }
        } else if (active) {
            for (uint32_t i = first; i < first + count; i++)
                test_triangle<STATS>(R, tris[3 * i], tris[3 * i + 1], tris[3 * i + 2], h, c);
        }
        if (active) active = pop<STRIDE, SW>(nodes4, stk, sp, R, h.best, first, count);
    }
}

}  // namespace rtfast
