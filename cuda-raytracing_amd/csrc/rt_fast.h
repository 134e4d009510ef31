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

constexpr int BIG = 8;     // leaves above this size wait for the wave (and have pair records)
constexpr int WAVE = 64;  // lane stride of the LDS stack

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

// float4 `i` of `base` through a 32-bit byte offset (i < 2^28): the load then takes the SGPR base + VGPR
// offset form (global_load ... v_off, s[base]) instead of a 64-bit address computed per lane
// (v_lshl_add_u64 / v_mad_u64_u32 on every node, pair and record load of the traversal loop).
__device__ __forceinline__ float4 ldo(const float4* base, uint32_t i) {
#if defined(RT_ADDR64)
    return base[i];
#else
    return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(base) + (i << 4));
#endif
}
typedef const __attribute__((address_space(4))) f4v* ConstF4;  // scalar-load (SMEM) view
__device__ __forceinline__ float4 ldc(ConstF4 p, uint32_t i) {
    const f4v v = p[i];
    return make_float4(v.x, v.y, v.z, v.w);
}

// The traversal stack of one lane: node indices, the first SL entries in LDS (lane stride WGL, the
// workgroup's lanes), deeper ones in a private per-lane array (scratch memory).  Deep stacks are rare -- no
// ray of a config-2 frame goes past 15 entries -- so a 16-entry LDS stack (4 KB per wave) costs nothing
// and leaves registers, not LDS, as the occupancy limit.
template <int SL, int WGL = WAVE>
struct Stack {
    static constexpr int LDS_ENTRIES = SL;
    static constexpr int LANES = WGL;  // lanes sharing the LDS rows (one wave, or a wave pair: trace)
    // A lane's stack pointer is ENCODED as the byte offset of its next entry from lane 0's entry 0:
    // sp = 4 * column + 4 WGL * depth (entry i of column l at lds0[l + i * WGL]).  The LDS address of an entry
    // is then lds0 + sp, one uniform base and the pointer the lane already holds: no per-lane column
    // address to keep live beside it (the 7-wave build spilled that address and reloaded it on every pop).
    // The column is the workgroup lane that started the ray; a ray handed to another lane of the workgroup
    // (wave pairs, trace) keeps its column and so its entries.
    uint32_t* lds0;  // column 0's entry 0 (workgroup-uniform)
    uint32_t* ovf;   // this lane's entries SL, SL + 1, ...
    static constexpr int STEP = 4 * WGL;  // sp per entry
    static __device__ __forceinline__ int depth(int sp) { return (int)((uint32_t)sp / (uint32_t)STEP); }  // sp >= 0: a shift
    static __device__ __forceinline__ int column(int sp) { return (sp & (STEP - 1)) >> 2; }
    static __device__ __forceinline__ int empty(int col) { return 4 * col; }  // sp of an empty stack
    __device__ __forceinline__ uint32_t* at(int sp) const {
        return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(lds0) + sp);
    }
    // the overflow entries as a rare branch of their own
    __device__ __forceinline__ void put(int sp, uint32_t v) const {
        if (__builtin_expect(depth(sp) >= SL, 0)) ovf[depth(sp) - SL] = v;
        else *at(sp) = v;
    }
    __device__ __forceinline__ uint32_t get(int sp) const {
        if (__builtin_expect(depth(sp) >= SL, 0)) return ovf[depth(sp) - SL];
        return *at(sp);
    }
    // the LDS word of entry sp, or the lane's word of the pad row SL (STACK_PAD_ROWS) past the LDS entries:
    // a store that need not happen (an entry above the top) goes there without a branch
    __device__ __forceinline__ uint32_t* at_clamped(int sp) const {
        return at(sp < SL * STEP ? sp : (sp & (STEP - 1)) + SL * STEP);
    }
};
constexpr int STACK_PAD_ROWS = 1;  // LDS rows allocated past a Stack's SL entries (at_clamped)

// Pop stack entries until one passes `tmin < closest` (the reference's pop-time test).  An
// entry is a node index (lane stride WAVE in LDS); tmin is recomputed from the node with the same
// slab arithmetic, so the decision is the reference's, at one word of LDS per entry.
template <class S>
__device__ __forceinline__ bool pop(const float4* nodes4, const S& stk, int& sp, const Ray& R, float best,
                                    uint32_t& first, uint32_t& count) {
    // One rare branch per entry: the approximate test runs for every ray (R.fast false only routes the entry
    // to the IEEE test) and the entry is read from LDS unless it lies in the overflow part (round 6: VALU and
    // SALU per launch -1.4 % each against the same loop with the R.fast, UNSURE and overflow branches apart)
    while (sp >= S::STEP) {
        sp -= S::STEP;
        uint32_t idx = *stk.at_clamped(sp);
        if (__builtin_expect(S::depth(sp) >= S::LDS_ENTRIES, 0)) idx = stk.ovf[S::depth(sp) - S::LDS_ENTRIES];
        const float4 lo = ldo(nodes4, 2 * idx), hi = ldo(nodes4, 2 * idx + 1);
        float te, tx;
        slab_approx(R, lo, hi, &te, &tx);
        const int cl = classify_lt(te, best);
        bool pass = cl == YES;
        if (!R.fast || cl == UNSURE) {
            slab_exact(R, lo, hi, &te, &tx);
            pass = te < best;
        }
        if (pass) {
            first = __float_as_uint(hi.z), count = __float_as_uint(hi.w);
            return true;
        }
    }
    return false;
}

// One inner-node step: both children (adjacent in the node array) tested, the right child
// continued in registers, the left one continued or pushed, exactly as the reference's
// push(first), push(first+1), pop order.  Returns false when the lane must pop.
template <bool STATS, class S, class C>
__device__ __forceinline__ bool inner_step(const float4* nodes4, const S& stk, int& sp, const Ray& R, float best,
                                           uint32_t& first, uint32_t& count, C& c) {
    const float4 l0 = ldo(nodes4, 2 * first), l1 = ldo(nodes4, 2 * first + 1);
    const float4 r0 = ldo(nodes4, 2 * first + 2), r1 = ldo(nodes4, 2 * first + 3);
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
            stk.put(sp, first);
            sp += S::STEP;
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

// glm's accept predicate from the four quantities (det, u, v, u + v), as test_triangle.
__device__ __forceinline__ bool tri_ok(float det, float u, float v, float uv) {
    const float eps = 1.1920928955078125e-07f;
    const uint32_t sgn = __float_as_uint(det) & 0x80000000u;
    const float adet = fabsf(det);
    const float su = __uint_as_float(__float_as_uint(u) ^ sgn);
    const float sv = __uint_as_float(__float_as_uint(v) ^ sgn);
    const float suv = __uint_as_float(__float_as_uint(uv) ^ sgn);
    return adet > eps && !(su < 0.0f || su > adet) && !(sv < 0.0f || suv > adet);
}

// glm::intersectRayTriangle + BVHRayHit's accept test (`!(t >= best || t < 0)`) for one
// candidate; returns whether it would be accepted against threshold `best`, and reports a
// NaN distance of an otherwise accepted triangle (the sequential reference accepts a NaN t;
// a min-reduction would not, so such a ray is redone sequentially).
__device__ __forceinline__ bool tri_accept(f3 o, f3 nd, float4 A, float4 B, float4 Cc, float best, float* t_o,
                                           float* bx, float* by, bool* nan) {
    const f3 e1 = rtm::mk(A.w, B.x, B.y), e2 = rtm::mk(B.z, B.w, Cc.x);
    const f3 p = rtm::cross(nd, e2);
    const float det = rtm::dot(e1, p);
    const f3 dist = rtm::sub(o, rtm::mk(A.x, A.y, A.z));
    const float u = rtm::dot(dist, p);
    const f3 perp = rtm::cross(dist, e1);
    const float v = rtm::dot(nd, perp);
    const float uv = u + v;
    if (!tri_ok(det, u, v, uv)) return false;
    const float inv_det = 1.0f / det;
    const float t = rtm::dot(e2, perp) * inv_det;
    *nan = *nan || (t != t);
    if (t >= best || t < 0.0f) return false;
    *t_o = t;
    *bx = u * inv_det;
    *by = v * inv_det;
    return true;
}

// ---------------------------------------------------------------------------------------
// Big leaves in packed pairs.  For every leaf above BIG triangles the mirror also holds the
// triangles two by two, each component interleaved (mirror.h), so one packed fp32 instruction
// (v_pk_mul_f32 / v_pk_add_f32) does the same IEEE operation for two triangles -- per half
// exactly the scalar result, so the decisions are the reference's.  An odd leaf is padded with
// an all-zero triangle (det = 0 is never accepted).
// ---------------------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));

struct Pair {
    f2 v0x, v0y, v0z, e1x, e1y, e1z, e2x, e2y, e2z;
    uint32_t fa, fb;  // face ids
};

__device__ __forceinline__ Pair make_pair(f4v q0, f4v q1, f4v q2, f4v q3, f4v q4) {
    Pair P;
    P.v0x = q0.xy, P.v0y = q0.zw, P.v0z = q1.xy;
    P.e1x = q1.zw, P.e1y = q2.xy, P.e1z = q2.zw;
    P.e2x = q3.xy, P.e2y = q3.zw, P.e2z = q4.xy;
    P.fa = __float_as_uint(q4.z), P.fb = __float_as_uint(q4.w);
    return P;
}
__device__ __forceinline__ Pair ld_pair_scalar(ConstF4 base, uint32_t p) {
    return make_pair(base[5 * p], base[5 * p + 1], base[5 * p + 2], base[5 * p + 3], base[5 * p + 4]);
}
__device__ __forceinline__ Pair ld_pair(const float4* base, uint32_t p) {
#if defined(RT_ADDR64)
    const f4v* q = reinterpret_cast<const f4v*>(base) + 5 * (size_t)p;
#else
    const f4v* q = reinterpret_cast<const f4v*>(reinterpret_cast<const char*>(base) + p * 80u);  // 32-bit offset
#endif
    return make_pair(q[0], q[1], q[2], q[3], q[4]);
}

// det, u, v, u + v and perp of glm::intersectRayTriangle for both triangles (same operation
// order as test_triangle: p = cross(nd, e2), det = dot(e1, p), dist = o - v0, u = dot(dist, p),
// perp = cross(dist, e1), v = dot(nd, perp)).
struct PairEval {
    f2 det, u, v, uv, qx, qy, qz;  // q = perp
    f2 dn;                         // |o - v0|_1 (computed; the twin test's bound, twin_rejected)
};
__device__ __forceinline__ PairEval pair_eval(f3 o, f3 nd, const Pair& P) {
    const f2 ndx = nd.x, ndy = nd.y, ndz = nd.z;
    const f2 px = ndy * P.e2z - P.e2y * ndz;
    const f2 py = ndz * P.e2x - P.e2z * ndx;
    const f2 pz = ndx * P.e2y - P.e2x * ndy;
    PairEval E;
    E.det = (P.e1x * px + P.e1y * py) + P.e1z * pz;
    const f2 dx = o.x - P.v0x, dy = o.y - P.v0y, dz = o.z - P.v0z;
    E.u = (dx * px + dy * py) + dz * pz;
    E.qx = dy * P.e1z - P.e1y * dz;
    E.qy = dz * P.e1x - P.e1z * dx;
    E.qz = dx * P.e1y - P.e1x * dy;
    E.v = (ndx * E.qx + ndy * E.qy) + ndz * E.qz;
    E.uv = E.u + E.v;
    E.dn = f2{(fabsf(dx.x) + fabsf(dy.x)) + fabsf(dz.x), (fabsf(dx.y) + fabsf(dy.y)) + fabsf(dz.y)};
    return E;
}

// The distance of an accepted pair member (rare path, scalar).
__device__ __forceinline__ float pair_t(const Pair& P, const PairEval& E, int k, float* inv) {
    const float det = k ? E.det.y : E.det.x;
    *inv = 1.0f / det;
    const f3 e2 = k ? rtm::mk(P.e2x.y, P.e2y.y, P.e2z.y) : rtm::mk(P.e2x.x, P.e2y.x, P.e2z.x);
    const f3 q = k ? rtm::mk(E.qx.y, E.qy.y, E.qz.y) : rtm::mk(E.qx.x, E.qy.x, E.qz.x);
    return rtm::dot(e2, q) * *inv;
}

// BVHRayHit's sequential leaf step for triangles 2p, 2p+1 (in that order) on this lane's ray.
__device__ __forceinline__ void pair_test(const Ray& R, const Pair& P, Hit& h) {
    const PairEval E = pair_eval(R.o, R.nd, P);
    const bool oka = tri_ok(E.det.x, E.u.x, E.v.x, E.uv.x);
    const bool okb = tri_ok(E.det.y, E.u.y, E.v.y, E.uv.y);
    if (oka) {
        float inv;
        const float t = pair_t(P, E, 0, &inv);
        if (!(t >= h.best || t < 0.0f)) h.best = t, h.kind = 2, h.id = P.fa, h.bx = E.u.x * inv, h.by = E.v.x * inv;
    }
    if (okb) {
        float inv;
        const float t = pair_t(P, E, 1, &inv);
        if (!(t >= h.best || t < 0.0f)) h.best = t, h.kind = 2, h.id = P.fb, h.bx = E.u.y * inv, h.by = E.v.y * inv;
    }
}

// device-library wave reduction (DPP), over the active lanes
extern "C" __device__ uint32_t __ockl_wfred_min_u32(uint32_t);

// ---------------------------------------------------------------------------------------
// Twins (mirror.h quads / units).  Every loaded face is in the scene twice (Scene.cpp:103-127), and a
// big leaf holds both records: A = (v0, e1, e2) and its twin A' = (v0, e2, e1), so the sequential loop
// (main_raytracing.cu:51-71) runs glm's test on each triangle twice, wound both ways.  In real
// arithmetic the twin's det, u, v are -det, -v, -u of A's, and the fp32 values stay within bounds the
// mirror precomputes (mirror.cpp rt_twin_bounds): |det + det'| <= kd, |u + v'|, |v + u'| <= ke |o - v0|_1.
// So A's own values decide the twin whenever they reject it with margin; only the rest (a ray within
// a few ulps of an edge, or nearly parallel to the plane, or a hit) test the twin itself.  Quads pack
// two triangles (packed fp32, as the pairs) and their twins for the shared-leaf loop, units one
// triangle and its twin for the cooperative rounds, so a leaf costs about half its records.
// Triangles are then visited out of leaf order, so a candidate is kept by the sequential loop's own
// rule restated in (t, position) order: below the entry distance, the smallest t, the lowest position
// among equal t (a NaN distance: the leaf is redone sequentially).
// ---------------------------------------------------------------------------------------
constexpr uint32_t NO_POS = 0xffffffffu;

// Whether glm's test certainly rejects the twin of a triangle whose own test computed (det, u, v, uv)
// at |o - v0|_1 = dn.  With the twin's det' within kd of -det, u' within m of -v and v' within m of -u
// (m = ke dn), the twin's sign-folded quantities (test_triangle) are su' = sv +- m, sv' = su +- m,
// suv' = suv (1 +- 2.0001 U) +- 2.0001 m and |det'| = |det| +- kd once |det| > kd fixes det's sign; it
// fails `|det'| > eps && 0 <= su' <= |det'| && 0 <= sv' && suv' <= |det'|` if any bound already does.
// Every threshold is widened by 2^-20 (> the rounding of these few operations) and by 2^-90 (underflow);
// NaN, infinities and huge values are never decided here.
RT_HD bool twin_rejected(float det, float u, float v, float uv, float dn, float kd, float ke) {
    const bool neg = signbit(det);  // the sign fold of test_triangle (negation is exact)
    const float ad = fabsf(det);
    const float su = neg ? -u : u, sv = neg ? -v : v, suv = neg ? -uv : uv;
    if (!(ad + fabsf(su) + fabsf(sv) + dn < 0x1p100f)) return false;
    const float m = ke * dn + 0x1p-90f;
    const float kdd = kd + 0x1p-90f;
    const float top = (ad + kdd) * (1.0f + 0x1p-20f);
    if (top <= 1.1920928955078125e-07f) return true;  // |det'| <= eps
    if (!(ad > kdd * (1.0f + 0x1p-20f))) return false;  // det' may have either sign
    if (sv < -m || su < -m) return true;                // su' < 0 or sv' < 0
    if (sv > (ad + kdd + m) * (1.0f + 0x1p-20f)) return true;  // su' > |det'|
    return suv * (1.0f - 0x1p-20f) > (ad + kdd + 2.001f * m) * (1.0f + 0x1p-20f);  // suv' > |det'|
}

// A candidate under the sequential loop's rule in (t, position) order (h.best is the entry distance
// while bpos == NO_POS).
__device__ __forceinline__ void offer(float t, uint32_t pos, uint32_t id, float bx, float by, Hit& h, uint32_t& bpos,
                                      bool& nan) {
    if (t != t) {
        nan = true;
        return;
    }
    if (t >= 0.0f && (t < h.best || (t == h.best && bpos != NO_POS && pos < bpos)))
        h.best = t, h.kind = 2, h.id = id, h.bx = bx, h.by = by, bpos = pos;
}

// glm's test of triangle (v0, e1, e2) (test_triangle's operation order) offered at `pos`.
__device__ __forceinline__ void tri_offer(f3 o, f3 nd, f3 v0, f3 e1, f3 e2, uint32_t pos, uint32_t face, Hit& h,
                                          uint32_t& bpos, bool& nan) {
    const f3 p = rtm::cross(nd, e2);
    const float det = rtm::dot(e1, p);
    const f3 dist = rtm::sub(o, v0);
    const float u = rtm::dot(dist, p);
    const f3 perp = rtm::cross(dist, e1);
    const float v = rtm::dot(nd, perp);
    if (tri_ok(det, u, v, u + v)) {
        const float inv_det = 1.0f / det;
        offer(rtm::dot(e2, perp) * inv_det, pos, face, u * inv_det, v * inv_det, h, bpos, nan);
    }
}

// Quads (mirror.h): 7 float4 -- the pair layout (x5), the twin bounds (kd_a, kd_b, ke_a, ke_b; kd < 0:
// no twin), and (pos_a | twin_a << 16, pos_b | twin_b << 16, twin face a, twin face b), read only on a
// hit or a twin test.  One quad for one ray (the shared-leaf loop: scalar loads).
template <bool TIMING, class C>
__device__ __forceinline__ void quad_test(f3 o, f3 nd, const Pair& P, f4v bnd, ConstF4 q6, Hit& h, uint32_t& bpos,
                                          bool& nan, C& c) {
    const PairEval E = pair_eval(o, nd, P);
    const bool oka = tri_ok(E.det.x, E.u.x, E.v.x, E.uv.x), okb = tri_ok(E.det.y, E.u.y, E.v.y, E.uv.y);
    const bool twa = bnd.x >= 0.0f && !twin_rejected(E.det.x, E.u.x, E.v.x, E.uv.x, E.dn.x, bnd.x, bnd.z);
    const bool twb = bnd.y >= 0.0f && !twin_rejected(E.det.y, E.u.y, E.v.y, E.uv.y, E.dn.y, bnd.y, bnd.w);
    if (TIMING) {  // timing frames: the production kernel's own big-leaf work (RT_STAT_BIG_TESTS, ...)
        c.big_tests += 2;
        c.tw_test += (uint32_t)twa + (uint32_t)twb;
        c.tw_dec += (uint32_t)(bnd.x >= 0.0f && !twa) + (uint32_t)(bnd.y >= 0.0f && !twb);
    }
    if (oka || okb || twa || twb) {  // rare: a hit, or a twin too close to call
        const f4v W = *q6;
        const uint32_t wa = __float_as_uint(W.x), wb = __float_as_uint(W.y);
        if (oka) {
            float inv;
            const float t = pair_t(P, E, 0, &inv);
            offer(t, wa & 0xffffu, P.fa, E.u.x * inv, E.v.x * inv, h, bpos, nan);
        }
        if (okb) {
            float inv;
            const float t = pair_t(P, E, 1, &inv);
            offer(t, wb & 0xffffu, P.fb, E.u.y * inv, E.v.y * inv, h, bpos, nan);
        }
        if (twa)
            tri_offer(o, nd, rtm::mk(P.v0x.x, P.v0y.x, P.v0z.x), rtm::mk(P.e2x.x, P.e2y.x, P.e2z.x),
                      rtm::mk(P.e1x.x, P.e1y.x, P.e1z.x), wa >> 16, __float_as_uint(W.z), h, bpos, nan);
        if (twb)
            tri_offer(o, nd, rtm::mk(P.v0x.y, P.v0y.y, P.v0z.y), rtm::mk(P.e2x.y, P.e2y.y, P.e2z.y),
                      rtm::mk(P.e1x.y, P.e1y.y, P.e1z.y), wb >> 16, __float_as_uint(W.w), h, bpos, nan);
    }
}

// Units (mirror.h): 4 float4 -- a triangle record (v0, e1, e2, face) with (twin face, pos | twin << 16)
// in its last two words, and (kd, ke, 0, 0); kd < 0: no twin.  One unit for one ray (cooperative
// rounds: a lane per unit).
template <bool TIMING, class C>
__device__ __forceinline__ void unit_test(f3 o, f3 nd, float4 A, float4 B, float4 Cc, float4 D, Hit& h, uint32_t& bpos,
                                          bool& nan, C& c) {
    const f3 v0 = rtm::mk(A.x, A.y, A.z), e1 = rtm::mk(A.w, B.x, B.y), e2 = rtm::mk(B.z, B.w, Cc.x);
    const f3 p = rtm::cross(nd, e2);
    const float det = rtm::dot(e1, p);
    const f3 dist = rtm::sub(o, v0);
    const float u = rtm::dot(dist, p);
    const f3 perp = rtm::cross(dist, e1);
    const float v = rtm::dot(nd, perp);
    const float uv = u + v;
    const uint32_t w = __float_as_uint(Cc.w);
    if (tri_ok(det, u, v, uv)) {
        const float inv_det = 1.0f / det;
        offer(rtm::dot(e2, perp) * inv_det, w & 0xffffu, __float_as_uint(Cc.y), u * inv_det, v * inv_det, h, bpos, nan);
    }
    const float dn = (fabsf(dist.x) + fabsf(dist.y)) + fabsf(dist.z);
    const bool tw = D.x >= 0.0f && !twin_rejected(det, u, v, uv, dn, D.x, D.y);
    if (TIMING) c.big_tests++, c.tw_test += (uint32_t)tw, c.tw_dec += (uint32_t)(D.x >= 0.0f && !tw);
    if (tw) tri_offer(o, nd, v0, e2, e1, w >> 16, __float_as_uint(Cc.z), h, bpos, nan);
}

// BVHRayHit's sequential loop over big leaf [f0, f0 + c0) for this lane (the NaN fallback).
__device__ __forceinline__ void leaf_sequential(const float4* tris, uint32_t f0, uint32_t c0, f3 o, f3 nd, Hit& h) {
    for (uint32_t j = 0; j < c0; j++) {
        const float4 A = tris[3 * (f0 + j)], B = tris[3 * (f0 + j) + 1], Cc = tris[3 * (f0 + j) + 2];
        float t, x, y;
        bool dummy = false;
        if (tri_accept(o, nd, A, B, Cc, h.best, &t, &x, &y, &dummy)) {
            h.best = t, h.kind = 2, h.bx = x, h.by = y;
            h.id = __float_as_uint(Cc.y);
        }
    }
}

// Order-preserving key of a distance t >= 0 (found candidates only): +-0 share key 0, so a tie
// between them is decided by position, as the float comparison `t == best` does.
__device__ __forceinline__ uint32_t tkey(float t) { return t == 0.0f ? 0u : __float_as_uint(t); }

__device__ __forceinline__ float bcast(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// Cooperative big-leaf round: the waiting lanes (mask `big`) all wait at leaf [f0, f0+c0),
// whose pairs start at `pairs`.  Rays are taken one at a time; lane l tests pairs l, l+64, ...
// keeping its first strictly-closer candidate, and a (t, index) lexicographic arg-min over the
// wave gives exactly the triangle the sequential loop ends on (the first index attaining the
// minimum t below the ray's closest distance).  A NaN distance sends the ray to the sequential
// loop.
__device__ __forceinline__ void coop_leaf(const float4* tris, const float4* pairs, unsigned long long big, uint32_t f0,
                                          uint32_t c0, const Ray& R, Hit& h) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t np = (c0 + 1u) / 2u;
    unsigned long long m = big;
    while (m) {
        const int r = __ffsll((long long)m) - 1;
        m &= m - 1;
        const f3 rox = rtm::mk(bcast(R.o.x, r), bcast(R.o.y, r), bcast(R.o.z, r));
        const f3 nd = rtm::mk(bcast(R.nd.x, r), bcast(R.nd.y, r), bcast(R.nd.z, r));
        float bt = bcast(h.best, r), bx = 0.0f, by = 0.0f;
        uint32_t bi = 0xffffffffu, bid = 0;
        bool nan = false;
        for (uint32_t p = lane; p < np; p += 64u) {
            const Pair P = ld_pair(pairs, p);
            const PairEval E = pair_eval(rox, nd, P);
            if (tri_ok(E.det.x, E.u.x, E.v.x, E.uv.x)) {
                float inv;
                const float t = pair_t(P, E, 0, &inv);
                nan = nan || (t != t);
                if (!(t >= bt || t < 0.0f)) bt = t, bx = E.u.x * inv, by = E.v.x * inv, bi = 2 * p, bid = P.fa;
            }
            if (tri_ok(E.det.y, E.u.y, E.v.y, E.uv.y)) {
                float inv;
                const float t = pair_t(P, E, 1, &inv);
                nan = nan || (t != t);
                if (!(t >= bt || t < 0.0f)) bt = t, bx = E.u.y * inv, by = E.v.y * inv, bi = 2 * p + 1, bid = P.fb;
            }
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
        // arg-min of (t, index) across the wave (DPP wave reductions)
        const bool has = bi != 0xffffffffu;
        const uint32_t mk = __ockl_wfred_min_u32(has ? tkey(bt) : 0xffffffffu);
        const uint32_t mi = __ockl_wfred_min_u32(has && tkey(bt) == mk ? bi : 0xffffffffu);
        if (mi != 0xffffffffu) {
            const int wl = (int)((mi >> 1) & 63u);  // lane that tested pair mi / 2
            const float wbx = bcast(bx, wl), wby = bcast(by, wl), wt = bcast(bt, wl);
            const uint32_t wid = (uint32_t)__builtin_amdgcn_readlane((int)bid, wl);
            if ((int)lane == r) h.best = wt, h.kind = 2, h.bx = wbx, h.by = wby, h.id = wid;
        }
    }
}

// coop_leaf on a leaf's units (mirror.h): lane l tests units l, l + 64, ... for the one ray, keeping
// its (t, position)-first candidate (offer); the wave's (t, position) arg-min is the sequential loop's
// result.  A NaN distance, or a NaN entry distance, runs the sequential loop.
template <bool TIMING, class C>
__device__ __forceinline__ void coop_units(const float4* tris, const float4* un, uint32_t nu, unsigned long long big,
                                           uint32_t f0, uint32_t c0, const Ray& R, Hit& h, C& c) {
    const uint32_t lane = threadIdx.x & 63u;
    unsigned long long m = big;
    while (m) {
        const int r = __ffsll((long long)m) - 1;
        m &= m - 1;
        const f3 rox = rtm::mk(bcast(R.o.x, r), bcast(R.o.y, r), bcast(R.o.z, r));
        const f3 nd = rtm::mk(bcast(R.nd.x, r), bcast(R.nd.y, r), bcast(R.nd.z, r));
        Hit L;
        L.best = bcast(h.best, r), L.kind = 0, L.id = 0, L.bx = L.by = 0.0f;
        uint32_t bpos = NO_POS;
        bool nan = !(L.best == L.best);
        for (uint32_t q = lane; q < nu; q += 64u)
            unit_test<TIMING>(rox, nd, un[4 * q], un[4 * q + 1], un[4 * q + 2], un[4 * q + 3], L, bpos, nan, c);
        if (TIMING && lane == 0) c.big_iters += (nu + 63u) / 64u;
        if (__ballot(nan)) {
            if ((int)lane == r) leaf_sequential(tris, f0, c0, R.o, R.nd, h);
            continue;
        }
        const bool has = bpos != NO_POS;
        const uint32_t mk = __ockl_wfred_min_u32(has ? tkey(L.best) : 0xffffffffu);
        const uint32_t mi = __ockl_wfred_min_u32(has && tkey(L.best) == mk ? bpos : 0xffffffffu);
        if (mi != 0xffffffffu) {
            const int wl = __ffsll((long long)__ballot(has && bpos == mi)) - 1;
            const float wt = bcast(L.best, wl), wbx = bcast(L.bx, wl), wby = bcast(L.by, wl);
            const uint32_t wid = (uint32_t)__builtin_amdgcn_readlane((int)L.id, wl);
            if ((int)lane == r) h.best = wt, h.kind = 2, h.bx = wbx, h.by = wby, h.id = wid;
        }
    }
}

// coop_leaf on the scalar records (lane l tests triangles l, l+64, ...).
__device__ __forceinline__ void coop_leaf_scalar(const float4* tris, unsigned long long big, uint32_t f0, uint32_t c0,
                                                 const Ray& R, Hit& h) {
    const uint32_t lane = threadIdx.x & 63u;
    unsigned long long m = big;
    while (m) {
        const int r = __ffsll((long long)m) - 1;
        m &= m - 1;
        const f3 rox = rtm::mk(bcast(R.o.x, r), bcast(R.o.y, r), bcast(R.o.z, r));
        const f3 nd = rtm::mk(bcast(R.nd.x, r), bcast(R.nd.y, r), bcast(R.nd.z, r));
        float bt = bcast(h.best, r), bx = 0.0f, by = 0.0f;
        uint32_t bi = 0xffffffffu;
        bool nan = false;
        for (uint32_t j = lane; j < c0; j += 64u) {
            const float4 A = tris[3 * (f0 + j)], B = tris[3 * (f0 + j) + 1], Cc = tris[3 * (f0 + j) + 2];
            float t, x, y;
            if (tri_accept(rox, nd, A, B, Cc, bt, &t, &x, &y, &nan)) bt = t, bx = x, by = y, bi = j;
        }
        if (__ballot(nan)) {
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
        // (t, index) arg-min over the lanes holding a candidate (DPP wave reductions)
        const bool has = bi != 0xffffffffu;
        const uint32_t mk = __ockl_wfred_min_u32(has ? tkey(bt) : 0xffffffffu);
        const uint32_t mi = __ockl_wfred_min_u32(has && tkey(bt) == mk ? bi : 0xffffffffu);
        if (mi != 0xffffffffu) {
            const int wl = (int)(mi & 63u);
            const float wbx = bcast(bx, wl), wby = bcast(by, wl), wt = bcast(bt, wl);
            if ((int)lane == r) {
                const float4 Cc = tris[3 * (f0 + mi) + 2];
                h.best = wt, h.kind = 2, h.bx = wbx, h.by = wby;
                h.id = __float_as_uint(Cc.y);
            }
        }
    }
}

// BVHRayHit for one lane (`live` = the lane has a segment to trace).  Every lane of the wave
// must call it (it synchronises big leaves across the wave).  STRIDE: the stack's lane stride.
// ---------------------------------------------------------------------------------------
// Leaf trees (leaftree.h).  BVHRayHit tests a leaf's triangles in order and keeps a triangle
// iff `!(t >= best || t < 0)`; for a finite `best` and finite distances the result is the
// first index attaining the minimum distance below the entry `best`.  tree_leaf computes
// exactly that -- candidates compared by (t, index) -- testing only the clusters cluster_cull
// cannot exclude, and redoes the leaf sequentially when a NaN shows up.
// ---------------------------------------------------------------------------------------
struct LeafBest {
    float t;       // running minimum (starts at the entry `best`)
    uint32_t j;    // its position inside the leaf (valid when found)
    uint32_t id;   // face id
    float bx, by;
    bool found, nan;
};

// glm::intersectRayTriangle as in test_triangle, candidate kept by (t, index).
__device__ __forceinline__ void leaf_candidate(const Ray& R, float4 A, float4 B, float4 Cc, LeafBest& L) {
    const f3 e1 = rtm::mk(A.w, B.x, B.y), e2 = rtm::mk(B.z, B.w, Cc.x);
    const f3 p = rtm::cross(R.nd, e2);
    const float det = rtm::dot(e1, p);
    const f3 dist = rtm::sub(R.o, rtm::mk(A.x, A.y, A.z));
    const float u = rtm::dot(dist, p);
    const f3 perp = rtm::cross(dist, e1);
    const float v = rtm::dot(R.nd, perp);
    if (tri_ok(det, u, v, u + v)) {
        const float inv_det = 1.0f / det;
        const float t = rtm::dot(e2, perp) * inv_det;
        const uint32_t j = __float_as_uint(Cc.z);
        L.nan = L.nan || (t != t);
        if (t >= 0.0f && (t < L.t || (t == L.t && L.found && j < L.j))) {
            L.t = t, L.j = j, L.id = __float_as_uint(Cc.y);
            L.bx = u * inv_det, L.by = v * inv_det;
            L.found = true;
        }
    }
}

// true => no triangle under the node can pass the fp32 test with 0 <= t < best for this ray.
//
// Why (U = 2^-24; every error term is bounded with the standard error model of the glm
// operation order, constants rounded up and then doubled): if the computed test accepts
// triangle (v0, e1, e2), then with D = |det| (exact) the exact barycentrics of the line/plane
// intersection X violate [b1 >= 0, b2 >= 0, b1 + b2 <= 1] by at most
//   d = 2U + U*N1*(24.1*|o - v0|_1*E1 + 5.1*E1^2)/D,   N1 = |nd|_1 <= 1.7321,
// so X lies within r = 4*d*E1 of the triangle, and X's exact ray parameter lies within Et of the
// computed t (once D >= 4x the det error, required below).  D >= Dlb comes from the node's
// normal cone (K2, K3.x) and Nmin, |o - v0|_1 <= Dist1 from its box.  The slab test then checks
// the ray segment [-Et, min(best, Tmax) + Et] against the box grown by r, with a margin m
// (2^-16 relative) that absorbs the rounding of the test itself.  Rays outside the filtered
// range (R.fast false) are never culled.  tests/test_leaf_tree.py checks the bound on the host.
// Upper bounds may come from the hardware's 1-ulp sqrt / reciprocal on the device: every use below
// is followed by a (1 + 2^-20) widening, which covers their error (the host uses IEEE sqrt / divide).
RT_HD float cull_sqrt(float x) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_sqrtf(x);
#else
    return sqrtf(x);
#endif
}
RT_HD float cull_div(float a, float b) {
#ifdef __HIP_DEVICE_COMPILE__
    return a * __builtin_amdgcn_rcpf(b);
#else
    return a / b;
#endif
}

RT_HD bool cluster_cull(const Ray& R, f3 rnd, float best, float4 K0, float4 K1, float4 K2, float4 K3) {
    const float U = 0x1p-24f;
    if (!(best == best)) return false;
    const float E1 = K0.w, Nmin = K1.w;
    const float dota = fabsf(R.nd.x * K2.x + R.nd.y * K2.y + R.nd.z * K2.z);
    const float ca = fminf(fmaxf(dota * (1.0f - 0x1p-20f) - 4.0f * U, 0.0f), 1.0f);  // <= cos(angle(nd, axis))
    const float sa = cull_sqrt(fmaxf(1.0f - ca * ca, 0.0f) + 2.0f * U) * (1.0f + 0x1p-20f);  // >= its sine
    const float dlb = Nmin * ((ca * K2.w - sa * K3.x) - 4.0f * U) * (1.0f - 0x1p-20f);  // <= min |det|
    if (!(dlb > 36.0f * U * E1 * E1)) return false;
    const float g = cull_div(E1, dlb) * (1.0f + 0x1p-20f);
    const float dx = fmaxf(fabsf(R.o.x - K0.x), fabsf(R.o.x - K1.x));
    const float dy = fmaxf(fabsf(R.o.y - K0.y), fabsf(R.o.y - K1.y));
    const float dz = fmaxf(fabsf(R.o.z - K0.z), fabsf(R.o.z - K1.z));
    const float dist1 = ((dx + dy) + dz) * (1.0f + 0x1p-20f);
    const float r = U * E1 * (8.0f + g * (168.0f * dist1 + 36.0f * E1)) * (1.0f + 0x1p-18f) + 0x1p-100f;
    const float tmax = (dist1 + r) * (1.0f + 0x1p-18f);
    const float et = U * tmax * (53.0f * E1 * g + 8.125f) * (1.0f + 0x1p-18f);
    const float send = fminf(best, tmax);
    const float m = 0x1p-16f * (send + et) + 0x1p-100f;
    const float s0 = -(et + m), s1 = send + et + m;
    const float bmax = fmaxf(fmaxf(fmaxf(fabsf(K0.x), fabsf(K1.x)), fmaxf(fabsf(K0.y), fabsf(K1.y))),
                             fmaxf(fabsf(K0.z), fabsf(K1.z)));
    const float ex0 = (r + 1.01f * m) * (1.0f + 0x1p-20f);
    const float ex = ex0 + 0x1p-20f * (bmax + ex0);
    const float tx1 = ((K0.x - ex) - R.o.x) * rnd.x, tx2 = ((K1.x + ex) - R.o.x) * rnd.x;
    const float ty1 = ((K0.y - ex) - R.o.y) * rnd.y, ty2 = ((K1.y + ex) - R.o.y) * rnd.y;
    const float tz1 = ((K0.z - ex) - R.o.z) * rnd.z, tz2 = ((K1.z + ex) - R.o.z) * rnd.z;
    const float lo = fmaxf(s0, fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2)));
    const float hi = fminf(s1, fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2)));
    return lo > hi;
}

// Leaf [f0, f0 + c0) through its tree (root `root`), this lane alone (stackless: pre-order
// with skip pointers).
template <bool STATS, class C>
__device__ __forceinline__ void tree_leaf(const float4* tris, const float4* tree, const float4* ltris, uint32_t root,
                                          uint32_t f0, uint32_t c0, const Ray& R, Hit& h, C& c) {
    if (STATS) c.tri += c0;  // the reference's work (tri_tests); node visits / tests run below
    LeafBest L;
    L.t = h.best, L.j = 0, L.id = 0, L.bx = 0.0f, L.by = 0.0f, L.found = false;
    L.nan = !(h.best == h.best);
    const bool cull_ok = R.fast;
    const f3 rnd = cull_ok ? rtm::mk(1.0f / R.nd.x, 1.0f / R.nd.y, 1.0f / R.nd.z) : rtm::mk(0.0f, 0.0f, 0.0f);
    const float4 KR = tree[4 * (size_t)root + 3];
    const uint32_t end = __float_as_uint(KR.y);
    const size_t ln = __float_as_uint(KR.x);  // leaf-tree triangles, field-major (leaftree.h)
    uint32_t k = root;
    while (k < end) {
        const float4* kp = tree + 4 * (size_t)k;
        const float4 K3 = kp[3];
        const uint32_t skip = __float_as_uint(K3.y), info = __float_as_uint(K3.w);
        if (STATS) c.ktest++;
        if (cull_ok && !L.nan && (info & 1u) && cluster_cull(R, rnd, L.t, kp[0], kp[1], kp[2], K3)) {
            k = skip;
            continue;
        }
        const uint32_t b = __float_as_uint(K3.z);
        if (b != 0xffffffffu) {
            const uint32_t n = info >> 8;
            if (STATS) c.ktri += n;
            for (uint32_t i = b; i < b + n; i++) leaf_candidate(R, ltris[i], ltris[ln + i], ltris[2 * ln + i], L);
            k = skip;
        } else {
            k++;
        }
    }
    if (L.nan) {
        for (uint32_t i = f0; i < f0 + c0; i++) {
            float t, x, y;
            bool dummy = false;
            const float4 A = tris[3 * i], B = tris[3 * i + 1], Cc = tris[3 * i + 2];
            if (tri_accept(R.o, R.nd, A, B, Cc, h.best, &t, &x, &y, &dummy)) {
                h.best = t, h.kind = 2, h.bx = x, h.by = y;
                h.id = __float_as_uint(Cc.y);
            }
        }
    } else if (L.found) {
        h.best = L.t, h.kind = 2, h.id = L.id, h.bx = L.bx, h.by = L.by;
        if (STATS) c.tacc++;
    }
}

// Traversal state of one lane between steps: the node (or leaf) it is at and its stack depth.
struct Trav {
    uint32_t first, count;
    int sp;  // stack pointer, encoded (Stack: 4 * lane + 256 * depth); bit SCREENED: at a big leaf whose screen has run
};
// Trav::sp flag (screen variants): the lane's big leaf has been screened and it waits for the wave's
// big-leaf round.  Kept in the depth word rather than in a bool of its own (a per-lane bool lives in a
// lane mask, and the 6-wave build of the screen variants mis-rendered with one: tools/variant_agree.py).
constexpr int SCREENED = 1 << 30;

// Cooperative walk of the leaf trees through their flat lists (leaftree.h) for the lanes `m`
// waiting at tree leaves, one ray at a time: the whole wave screens the cut subtrees (a lane per
// subtree), then the clusters of the surviving subtrees (a lane per cluster, two subtrees per
// round), then the triangles of the surviving clusters (kClusterMax lanes per cluster); the cull bound drops to the best candidate found so far.  cluster_cull excludes only what provably cannot pass the fp32 test with
// 0 <= t < best; every lane keeps the (t, position) minimum of what it tested (leaf_candidate),
// and the wave's (t, position) arg-min is exactly the sequential loop's result.  A NaN distance
// sends the ray to the sequential loop.  The per-lane walk (tree_leaf) runs each lane's ray on
// one lane, at a few percent lane utilisation; here all 64 lanes work on one ray.
__device__ __forceinline__ f3 bcast3(f3 v, int lane) {
    return rtm::mk(bcast(v.x, lane), bcast(v.y, lane), bcast(v.z, lane));
}

template <bool TIMING, class C>
__device__ __forceinline__ void coop_tree(const float4* tris, const float4* tree, const float4* ltris, const float4* flat,
                                          unsigned long long m, uint32_t root_l, const Ray& R, Hit& h, const Trav& T,
                                          uint32_t* scratch, uint32_t tune, C& c) {
    const uint32_t lane = threadIdx.x & 63u;
    // RT_TUNE bit 31: visit surviving subtrees nearest box first (costs more than it saves here:
    // 117 vs 111 ms on the 4-bunny frame), else in tree order
    const bool order = (tune & 0x80000000u) != 0;
    const f3 rnd_l = rtm::mk(1.0f / R.nd.x, 1.0f / R.nd.y, 1.0f / R.nd.z);  // cluster_cull's reciprocals
    while (m) {
        const int r = __ffsll((long long)m) - 1;
        m &= m - 1;
        if (TIMING && lane == 0) c.r_coop++;
        const uint32_t root = (uint32_t)__builtin_amdgcn_readlane((int)root_l, r);
        const uint32_t f0 = (uint32_t)__builtin_amdgcn_readlane((int)T.first, r);
        const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)T.count, r);
        Ray B;
        B.o = bcast3(R.o, r);
        B.nd = bcast3(R.nd, r);
        B.d = B.nd, B.r = B.nd;  // unused by cluster_cull / leaf_candidate
        B.fast = __builtin_amdgcn_readlane(R.fast ? 1 : 0, r) != 0;
        const f3 rnd = bcast3(rnd_l, r);
        const float best = bcast(h.best, r);
        const f4v K2 = ((ConstF4)(tree + 4 * (size_t)root))[2];
        const f4v KR = ((ConstF4)(tree + 4 * (size_t)root))[3];
        const uint32_t cb = __float_as_uint(K2.x), nc = __float_as_uint(K2.y), kb = __float_as_uint(K2.z),
                       nk = __float_as_uint(K2.w);
        const size_t ln = __float_as_uint(KR.x);
        // field-major lists (leaftree.h): field f of cluster i at cl[f * nc + i], of cut k at ct[f * nk + k]
        const float4* cl = flat + cb;
        const float4* ct = flat + kb;
        LeafBest L;
        L.t = best, L.j = 0, L.id = 0, L.bx = 0.0f, L.by = 0.0f, L.found = false;
        L.nan = !(best == best);
        const bool cull_ok = B.fast && !L.nan;
        float cbest = best;  // cull bound: next float above the best candidate found so far
        for (uint32_t kbase = 0; kbase < nk; kbase += 64u) {
            const uint32_t k = kbase + lane;
            bool need = false;
            uint32_t s0 = 0, s1 = 0;
            float te = 0.0f;
            if (k < nk) {
                const float4 K0 = ct[k], K1 = ct[nk + k], K3 = ct[3 * nk + k];
                s0 = __float_as_uint(K3.y), s1 = __float_as_uint(K3.z);
                need = !(cull_ok && (__float_as_uint(K3.w) & 1u) && cluster_cull(B, rnd, cbest, K0, K1, ct[2 * nk + k], K3));
                if (order) {  // box entry distance along the ray, only to order the subtrees
                    const float tx1 = (K0.x - B.o.x) * rnd.x, tx2 = (K1.x - B.o.x) * rnd.x;
                    const float ty1 = (K0.y - B.o.y) * rnd.y, ty2 = (K1.y - B.o.y) * rnd.y;
                    const float tz1 = (K0.z - B.o.z) * rnd.z, tz2 = (K1.z - B.o.z) * rnd.z;
                    te = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
                    te = te == te ? te : 0.0f;
                }
            }
            const unsigned long long mk = __ballot(need);
            const uint32_t ns = (uint32_t)__popcll(mk);
            if (TIMING && lane == 0) c.ktest += min(64u, nk - kbase), c.r_shared += ns;
            // near-first order of the surviving subtrees: rank by (entry distance, lane)
            uint32_t rank = 0;
            if (order) {
                for (unsigned long long w = mk; w; w &= w - 1) {
                    const int b = __ffsll((long long)w) - 1;
                    const float tb = bcast(te, b);
                    rank += (tb < te || (tb == te && b < (int)lane)) ? 1u : 0u;
                }
            } else {
                rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
            }
            for (uint32_t q = 0; q < ns; q += 2) {
                // two subtrees per round (<= 32 clusters each): lanes 0-31 and 32-63
                const int a = __ffsll((long long)__ballot(need && rank == q)) - 1;
                const int b = q + 1 < ns ? __ffsll((long long)__ballot(need && rank == q + 1)) - 1 : -1;
                const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)s0, a);
                const uint32_t a1 = (uint32_t)__builtin_amdgcn_readlane((int)s1, a);
                uint32_t b0 = 0, b1 = 0;
                if (b >= 0) {
                    b0 = (uint32_t)__builtin_amdgcn_readlane((int)s0, b);
                    b1 = (uint32_t)__builtin_amdgcn_readlane((int)s1, b);
                }
                const unsigned long long tc0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
                const uint32_t ci = lane < 32u ? a0 + lane : b0 + (lane - 32u);
                const bool has = lane < 32u ? ci < a1 : ci < b1;
                bool need2 = false;
                uint32_t tb = 0, n = 0;
                if (has) {
                    const float4 Q3 = cl[3 * nc + ci];
                    const uint32_t info = __float_as_uint(Q3.w);
                    tb = __float_as_uint(Q3.z), n = info >> 8;
                    need2 = !(cull_ok && (info & 1u) && cluster_cull(B, rnd, cbest, cl[ci], cl[nc + ci], cl[2 * nc + ci], Q3));
                }
                const unsigned long long mc = __ballot(need2);
                const uint32_t nsc = (uint32_t)__popcll(mc);
                if (TIMING && lane == 0) c.l_big++, c.ktest += __popcll(__ballot(has)), c.coop_rays += nsc;
                const unsigned long long tc1 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
                if (TIMING) c.cy_tcl += tc1 - tc0;
                // surviving clusters, compacted in order through the wave's LDS scratch
                if (need2) {
                    const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(mc >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mc, 0u));
                    scratch[rk] = tb | ((n - 1u) << 26);  // 1 <= n <= kClusterMax <= 64; records < 2^26
                }
                __builtin_amdgcn_wave_barrier();
                constexpr uint32_t CL = kClusterMax, PER = 64u / kClusterMax;  // lanes per cluster, clusters per round
                for (uint32_t base = 0; base < nsc; base += PER) {
                    if (TIMING && lane == 0) c.w_big++;
                    const uint32_t slot = base + lane / CL, i = lane % CL;
                    if (slot < nsc) {
                        const uint32_t w = scratch[slot], my_tb = w & 0x03ffffffu, my_n = (w >> 26) + 1u;
                        if (i < my_n) {
                            const size_t t = (size_t)(my_tb + i);
                            leaf_candidate(B, ltris[t], ltris[ln + t], ltris[2 * ln + t], L);
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
                if (TIMING) c.cy_ttri += __builtin_amdgcn_s_memtime() - tc1;
                // tighten the cull bound to just above the best candidate so far (ties on t are
                // decided by position, so a triangle at exactly that distance must stay in)
                if (__ballot(L.found)) {
                    const uint32_t mk2 = __ockl_wfred_min_u32(L.found ? tkey(L.t) : 0xffffffffu);
                    const float up = __uint_as_float(mk2 + 1u);  // next float above the best (>= 0, finite)
                    cbest = fminf(cbest, up);
                }
            }
        }
        if (__ballot(L.nan)) {
            // sequential fallback for this ray (never taken for finite scenes)
            if ((int)lane == r) {
                for (uint32_t q = f0; q < f0 + c0; q++) {
                    float t, x, y;
                    bool dummy = false;
                    const float4 A = tris[3 * q], Bq = tris[3 * q + 1], Cc = tris[3 * q + 2];
                    if (tri_accept(R.o, R.nd, A, Bq, Cc, h.best, &t, &x, &y, &dummy)) {
                        h.best = t, h.kind = 2, h.bx = x, h.by = y;
                        h.id = __float_as_uint(Cc.y);
                    }
                }
            }
            continue;
        }
        // arg-min of (t, position) over the lanes holding a candidate: smallest t, then position
        const uint32_t mt = __ockl_wfred_min_u32(L.found ? tkey(L.t) : 0xffffffffu);
        const uint32_t mj = __ockl_wfred_min_u32(L.found && tkey(L.t) == mt ? L.j : 0xffffffffu);
        if (mt != 0xffffffffu) {
            const int wl = __ffsll((long long)__ballot(L.found && L.j == mj)) - 1;
            const float wt = bcast(L.t, wl), wbx = bcast(L.bx, wl), wby = bcast(L.by, wl);
            const uint32_t wid = (uint32_t)__builtin_amdgcn_readlane((int)L.id, wl);
            if ((int)lane == r) h.best = wt, h.kind = 2, h.id = wid, h.bx = wbx, h.by = wby;
        }
    }
}


// IntersectAABB of the root against the closest sphere distance (main_raytracing.cu:37-45):
// whether the lane has anything to traverse.
template <bool STATS, class C>
__device__ __forceinline__ bool trav_begin(const float4* nodes4, const Ray& R, const Hit& h, Trav& T, C& c) {
    const float4 lo = nodes4[0], hi = nodes4[1];
    if (STATS) c.node++;
    float tmin, tmax;
    slab_exact(R, lo, hi, &tmin, &tmax);
    T.first = __float_as_uint(hi.z), T.count = __float_as_uint(hi.w), T.sp = (int)threadIdx.x * 4;  // empty, own column
    return tmax >= tmin && tmin < h.best && tmax > 0.0f;
}

// A big leaf's screen (mirror.h pf = 3, leaftree.h rt_build_leaf_screen), run by a lane when it
// reaches the leaf: when cluster_cull proves that none of the leaf's core triangles can pass glm's
// fp32 test with 0 <= t < closest for this ray, the sequential loop over the leaf
// (main_raytracing.cu:51-71) can accept only the few outlier triangles (the big ones the core's box
// leaves out), so the lane tests those, in leaf order, and moves on without waiting for the wave's
// big-leaf round.  Returns true when the leaf is done that way.
template <bool STATS, class C>
__device__ __forceinline__ bool screen_leaf(const float4* tris, const float4* pairs, const Ray& R, Hit& h, const Trav& T,
                                            C& c) {
    if (!R.fast || !pairs) return false;
    const float4 lead = tris[3 * (size_t)T.first + 2];
    if (__float_as_uint(lead.w) != 3u) return false;
    const float4* S = pairs + 5 * ((size_t)__float_as_uint(lead.z) - 1);
    const float4 K0 = S[0], K1 = S[1], K2 = S[2], K3 = S[3];
    const f3 rnd = rtm::mk(1.0f / R.nd.x, 1.0f / R.nd.y, 1.0f / R.nd.z);
    if (!cluster_cull(R, rnd, h.best, K0, K1, K2, K3)) return false;
    const float4 P = S[4];
    const uint32_t n = __float_as_uint(K3.y);
    const uint32_t pos[4] = {__float_as_uint(P.x), __float_as_uint(P.y), __float_as_uint(P.z), __float_as_uint(P.w)};
    for (uint32_t k = 0; k < n && k < 4u; k++) {
        const size_t i = (size_t)T.first + pos[k];
        test_triangle<STATS>(R, tris[3 * i], tris[3 * i + 1], tris[3 * i + 2], h, c);
    }
    return true;
}

// Deferred big leaves (RT_TUNE bit 24 turns them off).  BVHRayHit tests a leaf when it pops it
// (main_raytracing.cu:51-71), so what a big leaf hits culls the rest of the traversal, and here a lane at a
// big leaf would wait for the wave's big-leaf round while the others step on.  Instead a lane's first big
// leaf is remembered the moment the lane reaches it (an inner step landing on it, a pop returning it, or
// the big-leaf round for a lone-traversal exit), the lane steps on, and when every lane of the wave is
// done the remembered leaves run through the ordinary big-leaf rounds (twin quads / units, leaf trees) from
// the bound the rest of the scene left.  Priced and checked on the CPU first (tools/defer_probe.c, tests/
// test_defer_rule.py: 0 differences from the reference order; config 4's tree leaf: the bound finite for
// 77 % of its visits instead of 43 %).  Why the result is the reference's: the end phase in trace.
constexpr uint32_t DEFER_NONE = 0xffffffffu, DEFER_OFF = 0xfffffffeu, DEFER_END1 = 0xfffffffdu, DEFER_END2 = 0xfffffffcu;
// Per lane, 5 words of wave-private LDS (tree kernels keep coop_tree's 64-word compaction area first):
// D[0] the deferred leaf's first index, or DEFER_NONE / DEFER_OFF (after a redo) / DEFER_END1 / DEFER_END2
// (its rounds are running), D[64] its count, D[128] `closest` when it was reached, D[192] `closest` at the
// end of the rest, D[256] the leaf's first index during END1, then the guard's bound.
constexpr int DEFER_WORDS = 5 * 64;
template <int MODE>
__device__ __forceinline__ uint32_t* defer_words(uint32_t* scratch) {
    return scratch + ((MODE & 4) ? 64 : 0) + (threadIdx.x & 63u);
}

__device__ __forceinline__ float next_up(float t) {  // the next float above t >= 0 (or -0)
    return __uint_as_float((__float_as_uint(t) & 0x7fffffffu) + 1u);
}

// Only rays and scenes inside +-2^16 defer (the ray's origin; the scene's root box, scalar loads): every
// product of the slab and triangle tests is then finite, so no NaN distance -- whose place in the order of
// accepts would matter -- can arise after the deferral.  D = the lane's words, or null: deferral off.
__device__ __forceinline__ bool defer_leaf(uint32_t* D, const float4* nodes4, const Trav& T, const Ray& R, const Hit& h) {
    if (!D || D[0] != DEFER_NONE || !(h.best <= 1e30f) || !R.fast) return false;
    const f4v lo = ((ConstF4)nodes4)[0], hi = ((ConstF4)nodes4)[1];
    const float sc = fmaxf(fmaxf(fmaxf(fabsf(lo.x), fabsf(lo.y)), fmaxf(fabsf(lo.z), fabsf(lo.w))),
                           fmaxf(fabsf(hi.x), fabsf(hi.y)));
    const float ro = fmaxf(fmaxf(fabsf(R.o.x), fabsf(R.o.y)), fabsf(R.o.z));
    if (!(sc < 0x1p16f && ro < 0x1p16f)) return false;
    D[0] = T.first, D[64] = T.count, D[128] = __float_as_uint(h.best);
    return true;
}

// pop, then: a big leaf popped as the lane's first is deferred (defer_leaf) and popping goes on
template <bool DEFER, class S>
__device__ __forceinline__ bool pop_d(const float4* nodes4, uint32_t* D, const S& stk, const Ray& R, const Hit& h, Trav& T) {
    for (;;) {
        if (!pop(nodes4, stk, T.sp, R, h.best, T.first, T.count)) return false;
        if (!DEFER || T.count <= (uint32_t)BIG || !defer_leaf(D, nodes4, T, R, h)) return true;
    }
}

// One small step of a lane at a small leaf or an inner node; false when the traversal is over.
// (Testing a small leaf in the same step as the inner node that entered it was measured slower:
// 22.2 vs 20.6 ms, the extra divergence costs more than the saved iterations.)
// DEF (deferred big leaves, D non-null): a big leaf the lane reaches as its first is deferred at once
// (defer_leaf), so the lane steps on instead of waiting for the wave's big-leaf round.
template <bool STATS, bool SCR = false, bool DEF = false, class S, class C>
__device__ __forceinline__ bool small_step(const float4* nodes4, const float4* tris, const float4* spairs, const S& stk,
                                           const Ray& R, Hit& h, Trav& T, C& c, const float4* pairs = nullptr,
                                           uint32_t* D = nullptr) {
    if constexpr (SCR) {
        if (T.count > (uint32_t)BIG) {  // a big leaf just reached: its screen, else wait for the round
            if (!screen_leaf<STATS>(tris, pairs, R, h, T, c)) {
                T.sp |= SCREENED;
                return true;
            }
            return pop(nodes4, stk, T.sp, R, h.best, T.first, T.count);
        }
    }
    if (T.count > 0) {
        if (!STATS && spairs) {
            // two triangles per packed pair record (mirror.h spairs), in leaf order
            for (uint32_t i = T.first; i < T.first + T.count; i += 2) pair_test(R, ld_pair(spairs, i), h);
        } else {
            for (uint32_t i = T.first; i < T.first + T.count; i++)
                test_triangle<STATS>(R, tris[3 * i], tris[3 * i + 1], tris[3 * i + 2], h, c);
        }
        return pop_d<DEF>(nodes4, D, stk, R, h, T);
    }
    if (inner_step<STATS>(nodes4, stk, T.sp, R, h.best, T.first, T.count, c)) {
        if (!DEF || T.count <= (uint32_t)BIG || !defer_leaf(D, nodes4, T, R, h)) return true;
    }
    return pop_d<DEF>(nodes4, D, stk, R, h, T);
}

// One big-leaf round, called by all lanes of the wave in converged control flow.  `big` = the
// lanes waiting at a big leaf (`waiting` on this lane).  The lanes at the leaf of the lowest
// waiting lane run it together (pairs / cooperative rounds / scalar loads); if every waiting
// lane is at that leaf, or each lane alone otherwise (MODE: see trace).  Returns whether this
// lane ran its leaf (it then pops; the others keep waiting).
template <bool STATS, int MODE, class C>
__device__ __forceinline__ bool big_round(const float4* tris, const float4* pairs, const float4* quads, const float4* units,
                                          const float4* tree,
                                          const float4* ltris, const float4* flat, uint32_t* scratch, uint32_t tune,
                                          unsigned long long big, bool waiting,
                                          const Ray& R, Hit& h, const Trav& T, C& c) {
    if ((MODE & 4) && tree) {  // MODE bit 2: the scene has leaf trees
        // lanes at leaves with a leaf tree (mirror.h: lead record pf == 2) walk it on their own
        bool at_tree = false;
        uint32_t root = 0;
        if (waiting) {
            const float4 lead = tris[3 * (size_t)T.first + 2];
            at_tree = __float_as_uint(lead.w) == 2u;
            root = __float_as_uint(lead.z);
        }
        const unsigned long long mt = __ballot(at_tree);
        if (mt) {
            if (!STATS && flat && (tune & 0x40000000u) == 0)  // RT_TUNE bit 30: per-lane walk instead
            {
                const unsigned long long tt0 = (MODE & 8) ? __builtin_amdgcn_s_memtime() : 0;
                coop_tree<(MODE & 8) != 0>(tris, tree, ltris, flat, mt, root, R, h, T, scratch, tune, c);
                if (MODE & 8) c.cy_tree += __builtin_amdgcn_s_memtime() - tt0;
            }
            else if (at_tree)
                tree_leaf<STATS>(tris, tree, ltris, root, T.first, T.count, R, h, c);
            return at_tree;
        }
    }
    const int l0 = __ffsll((long long)big) - 1;
    const uint32_t f0 = __builtin_amdgcn_readlane(T.first, l0);
    const uint32_t c0 = __builtin_amdgcn_readlane(T.count, l0);
    if (STATS) {
        uint32_t mx = waiting ? T.count : 0u;
        for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
        c.w_big += (threadIdx.x & 63) == 0 ? mx : 0;
        c.l_big += waiting ? T.count : 0;
    }
    if (__ballot(waiting && T.first == f0) == big) {
        // the first record of a big leaf says where its pairs are, the second where its twin quads are (mirror.h)
        const f4v lead = ((ConstF4)(tris + 3 * (size_t)f0))[2];
        const uint32_t k = (uint32_t)__popcll(big);
        if (!STATS && (MODE & 3) < 2 && quads && (__float_as_uint(lead.w) & 1u)) {
            // the second record: the leaf's first quad and quad count, the third: first unit and count
            const f4v l2 = ((ConstF4)(tris + 3 * (size_t)f0 + 3))[2];
            const f4v l3 = ((ConstF4)(tris + 3 * (size_t)f0 + 6))[2];
            const uint32_t nq = __float_as_uint(l2.w), nu = __float_as_uint(l3.w);
            // cost model (VALU instructions): cooperative ~ k * (70 * chunks + 70) over the units,
            // shared ~ 95 * nq over the quads for all waiting lanes at once
            // RT_TUNE bits 21-23: the cooperative side's weight in quarters (0 = 4, the default)
            const uint32_t cw = (tune >> 21) & 7u;
            if (nu && (tune & 1u) == 0 && k * (70u * ((nu + 63u) / 64u) + 70u) * (cw ? cw : 4u) < 4u * 95u * nq) {
                coop_units<(MODE & 8) != 0>(tris, units + 4 * (size_t)__float_as_uint(l3.z), nu, big, f0, c0, R, h, c);
                if (MODE & 8) c.r_coop++, c.coop_rays += k;
                return waiting;
            }
            if (nq) {
                if (MODE & 8) c.r_shared++;
                const Hit h0 = h;
                uint32_t bpos = NO_POS;
                bool nan = !(h.best == h.best);
                ConstF4 qs = (ConstF4)(quads + 7 * (size_t)__float_as_uint(l2.z));
                for (uint32_t q = 0; q < nq; q++, qs += 7) {
                    const Pair P = make_pair(qs[0], qs[1], qs[2], qs[3], qs[4]);
                    const f4v bnd = qs[5];
                    if (waiting) quad_test<(MODE & 8) != 0>(R.o, R.nd, P, bnd, qs + 6, h, bpos, nan, c);
                }
                if (MODE & 8) c.big_iters += nq;
                if (waiting && nan) {  // the sequential loop from the entry distance (never taken for finite scenes)
                    h = h0;
                    leaf_sequential(tris, f0, c0, R.o, R.nd, h);
                }
                return waiting;
            }
        }
        if (!STATS && (MODE & 3) < 2 && pairs && (__float_as_uint(lead.w) & 1u)) {
            const float4* lp = pairs + 5 * (size_t)__float_as_uint(lead.z);
            const uint32_t np = (c0 + 1u) / 2u, chunks = (np + 63u) / 64u;
            // cost model (VALU instructions per pair ~40): cooperative ~ k * (40 * chunks + 60),
            // shared-leaf ~ 40 * np for all waiting lanes at once
            const uint32_t cchunks = (c0 + 63u) / 64u;
            if ((MODE & 3) == 0 && (tune & 1u) == 0 && k * (40u * chunks + 60u) < 40u * np) {
                coop_leaf(tris, lp, big, f0, c0, R, h);
                if (MODE & 8) c.r_coop++, c.coop_rays += k;
            } else if ((MODE & 3) == 1 && (tune & 1u) == 0 && k * (60u * cchunks + 50u) < 40u * np) {
                coop_leaf_scalar(tris, big, f0, c0, R, h);
                if (MODE & 8) c.r_coop++, c.coop_rays += k;
            } else {
                if (MODE & 8) c.r_shared++;
                ConstF4 ps = (ConstF4)lp;
                for (uint32_t q = 0; q < np; q++, ps += 5) {
                    const Pair P = ld_pair_scalar(ps, 0);
                    if (waiting) pair_test(R, P, h);
                }
            }
        } else if (!STATS && (tune & 1u) == 0 && k * (60u * ((c0 + 63u) / 64u) + 50u) < 50u * c0) {
            // cost model (VALU instructions): cooperative ~ k * (60 * chunks + 50), lane-parallel ~ 50 * c0
            coop_leaf_scalar(tris, big, f0, c0, R, h);
        } else {
            // all waiting lanes share one leaf: scalar loads, next record prefetched
            ConstF4 st = (ConstF4)(tris + 3 * (size_t)f0);
            ConstF4 const last = st + 3 * (c0 - 1);
            float4 A = ldc(st, 0), B = ldc(st, 1), Cc = ldc(st, 2);
            for (uint32_t i = 0; i < c0; i++) {
                st = st == last ? st : st + 3;
                const float4 An = ldc(st, 0), Bn = ldc(st, 1), Cn = ldc(st, 2);
                if (waiting) test_triangle<STATS>(R, A, B, Cc, h, c);
                A = An, B = Bn, Cc = Cn;
            }
        }
        return waiting;
    }
    if (waiting) {
        for (uint32_t i = T.first; i < T.first + T.count; i++)
            test_triangle<STATS>(R, tris[3 * i], tris[3 * i + 1], tris[3 * i + 2], h, c);
    }
    return waiting;
}

// big_round for the lanes waiting at a big leaf, after deferring the lanes for which it is the first (D
// non-null; lanes that reach a big leaf through the lone traversal defer here, the others at arrival).
template <bool STATS, int MODE, class C>
__device__ __forceinline__ bool big_round_d(const float4* nodes4, uint32_t* D, const float4* tris, const float4* pairs,
                                            const float4* quads, const float4* units, const float4* tree,
                                            const float4* ltris, const float4* flat, uint32_t* scratch, uint32_t tune,
                                            unsigned long long big, bool waiting, const Ray& R, Hit& h, const Trav& T, C& c) {
    const bool dfr = waiting && defer_leaf(D, nodes4, T, R, h);
    if (__ballot(dfr)) {
        waiting = waiting && !dfr;
        big = __ballot(waiting);
        if (!big) return dfr;
    }
    return big_round<STATS, MODE>(tris, pairs, quads, units, tree, ltris, flat, scratch, tune, big, waiting, R, h, T, c) || dfr;
}

// ---------------------------------------------------------------------------------------
// Lone-ray traversal.  When a single lane of the wave is still in the small phase (the others
// are done or parked at big leaves -- the tail of a wave, and most of the time of the one-pixel
// waves a lane plan makes for the costliest pixels), that lane's steps are a chain of dependent
// loads at ~1.4 K cycles each.  Here the whole wave runs that one ray's DFS instead:
//   * the node to visit and the ray are wave-uniform: children come in through scalar loads and
//     the slab tests run once, on uniform operands;
//   * the traversal stack is distributed over the lanes' registers -- lane j holds entry j:
//     node index, the node's EXACT slab tmin (IntersectAABB's, computed when the entry arrives),
//     first, count -- so a pop is a ballot of `j < sp && tmin_j < closest` and the highest such
//     lane: the entries above it are exactly the ones the reference pops and rejects
//     (main_raytracing.cu:45), with no reload;
//   * a small leaf's triangles are tested one per lane against the entry `closest`, and the
//     (t, index) lexicographic minimum is the sequential loop's result (coop_leaf); a NaN
//     distance sends the leaf to the sequential loop.
// Same visit order, same decisions, bit for bit.  The lone lane's LDS stack entries move into
// the lanes on entry (only when they all live in LDS) and back on exit (a big leaf: the wave's
// big-leaf round takes over).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bcastu(uint32_t v, int lane) { return (uint32_t)__builtin_amdgcn_readlane((int)v, lane); }

template <class S>
__device__ __forceinline__ void lone_traverse(const float4* nodes4, const float4* tris, const S& stk, int r,
                                              const Ray& R, Hit& h, Trav& T, bool& active) {
    constexpr int SL = S::LDS_ENTRIES;
    const int lane = (int)(threadIdx.x & 63u);
    const int sp0 = (int)bcastu((uint32_t)T.sp, r);
    const int rc = S::column(sp0);           // lane r's ray's LDS stack column (its own lane, or its donor's)
    uint32_t* const col = stk.lds0 + rc;
    int sp = S::depth(sp0);  // lane r's depth
    uint32_t cf = bcastu(T.first, r), cc = bcastu(T.count, r);
    Ray U;  // the lone ray, wave-uniform
    U.o = bcast3(R.o, r), U.d = bcast3(R.d, r), U.nd = bcast3(R.nd, r), U.r = bcast3(R.r, r);
    U.fast = __builtin_amdgcn_readlane(R.fast ? 1 : 0, r) != 0;
    float best = bcast(h.best, r);
    int kind = __builtin_amdgcn_readlane(h.kind, r);
    uint32_t id = bcastu(h.id, r);
    float bx = bcast(h.bx, r), by = bcast(h.by, r);
    // the distributed stack: lane j = entry j (tmin filtered as in pop: e_exact = tmin is the
    // IEEE slab value, else q' with relative error < 2^-22.9, decided by classify_lt)
    uint32_t e_idx = 0, e_first = 0, e_count = 0;
    float e_tmin = 0.0f;
    bool e_exact = false;
    if (lane < sp) {
        e_idx = col[lane * S::LANES];
        const float4 lo = nodes4[2 * e_idx], hi = nodes4[2 * e_idx + 1];
        float tx;
        if (U.fast) {
            slab_approx(U, lo, hi, &e_tmin, &tx);
        } else {
            slab_exact(U, lo, hi, &e_tmin, &tx);
            e_exact = true;
        }
        e_first = __float_as_uint(hi.z), e_count = __float_as_uint(hi.w);
    }
    bool done = false;
    for (;;) {
        bool do_pop = false;
        if (cc == 0) {
            // inner node: both children (uniform), the reference's push(first), push(first + 1), pop
            const f4v a0 = ((ConstF4)nodes4)[2 * cf], a1 = ((ConstF4)nodes4)[2 * cf + 1];
            const f4v b0 = ((ConstF4)nodes4)[2 * cf + 2], b1 = ((ConstF4)nodes4)[2 * cf + 3];
            const float4 l0 = make_float4(a0.x, a0.y, a0.z, a0.w), l1 = make_float4(a1.x, a1.y, a1.z, a1.w);
            const float4 r0 = make_float4(b0.x, b0.y, b0.z, b0.w), r1 = make_float4(b1.x, b1.y, b1.z, b1.w);
            // inner_step's filtered-exact decisions, on uniform operands
            float tl = 0.0f, tlx = 0.0f, tr = 0.0f, trx = 0.0f;
            int okl = UNSURE, okr = UNSURE, rlt = UNSURE;
            if (U.fast) {
                slab_approx(U, l0, l1, &tl, &tlx);
                slab_approx(U, r0, r1, &tr, &trx);
                okl = classify_ok(tl, tlx);
                okr = classify_ok(tr, trx);
                rlt = okr == YES ? classify_lt(tr, best) : NO;
            }
            bool exact_l = false;
            if (__builtin_amdgcn_readfirstlane((okl == UNSURE || okr == UNSURE || rlt == UNSURE) ? 1 : 0)) {
                slab_exact(U, l0, l1, &tl, &tlx);
                slab_exact(U, r0, r1, &tr, &trx);
                okl = (tlx >= tl && tlx > 0.0f) ? YES : NO;
                okr = (trx >= tr && trx > 0.0f) ? YES : NO;
                rlt = (okr == YES && tr < best) ? YES : NO;
                exact_l = true;
            }
            if (__builtin_amdgcn_readfirstlane(rlt == YES ? 1 : 0)) {
                if (__builtin_amdgcn_readfirstlane(okl == YES ? 1 : 0)) {
                    if (lane == sp) {
                        e_idx = cf, e_tmin = tl, e_exact = exact_l;
                        e_first = __float_as_uint(l1.z), e_count = __float_as_uint(l1.w);
                    }
                    sp++;
                }
                cf = __float_as_uint(r1.z), cc = __float_as_uint(r1.w);
            } else {
                bool llt = false;
                if (__builtin_amdgcn_readfirstlane(okl == YES ? 1 : 0)) {
                    int cl = exact_l ? (tl < best ? YES : NO) : classify_lt(tl, best);
                    if (__builtin_amdgcn_readfirstlane(cl == UNSURE ? 1 : 0)) {
                        float te, tx;
                        slab_exact(U, l0, l1, &te, &tx);
                        cl = te < best ? YES : NO;
                    }
                    llt = __builtin_amdgcn_readfirstlane(cl == YES ? 1 : 0) != 0;
                }
                if (llt) cf = __float_as_uint(l1.z), cc = __float_as_uint(l1.w);
                else do_pop = true;
            }
        } else if (cc <= (uint32_t)BIG) {
            // small leaf: one triangle per lane against the entry `closest`, (t, index) minimum
            float t = 0.0f, x = 0.0f, y = 0.0f;
            bool nan = false, acc = false;
            if ((uint32_t)lane < cc) {
                const uint32_t i = cf + (uint32_t)lane;
                acc = tri_accept(U.o, U.nd, tris[3 * i], tris[3 * i + 1], tris[3 * i + 2], best, &t, &x, &y, &nan);
            }
            if (__ballot(nan)) {  // the sequential loop (never taken for finite scenes)
                if (lane == 0) {
                    for (uint32_t i = cf; i < cf + cc; i++) {
                        float tt, xx, yy;
                        bool dummy = false;
                        if (tri_accept(U.o, U.nd, tris[3 * i], tris[3 * i + 1], tris[3 * i + 2], best, &tt, &xx, &yy, &dummy)) {
                            best = tt, kind = 2, bx = xx, by = yy, id = __float_as_uint(tris[3 * i + 2].y);
                        }
                    }
                }
                best = bcast(best, 0), kind = __builtin_amdgcn_readlane(kind, 0), id = bcastu(id, 0);
                bx = bcast(bx, 0), by = bcast(by, 0);
            } else if (__ballot(acc)) {
                const uint32_t mk = __ockl_wfred_min_u32(acc ? tkey(t) : 0xffffffffu);
                const uint32_t mi = __ockl_wfred_min_u32(acc && tkey(t) == mk ? (uint32_t)lane : 0xffffffffu);
                const int wl = (int)mi;
                best = bcast(t, wl), bx = bcast(x, wl), by = bcast(y, wl), kind = 2;
                id = __float_as_uint(tris[3 * (cf + mi) + 2].y);
            }
            do_pop = true;
        } else {
            break;  // a big leaf: the wave's big-leaf round takes over
        }
        if (do_pop) {
            // pop-time `tmin < closest` of every entry at once; an entry too close to call is
            // re-tested with the IEEE slab (its node reloaded)
            int cl = NO;
            if (lane < sp) cl = e_exact ? (e_tmin < best ? YES : NO) : classify_lt(e_tmin, best);
            if (__ballot(cl == UNSURE)) {
                if (cl == UNSURE) {
                    const float4 lo = nodes4[2 * e_idx], hi = nodes4[2 * e_idx + 1];
                    float tx;
                    slab_exact(U, lo, hi, &e_tmin, &tx);
                    e_exact = true;
                    cl = e_tmin < best ? YES : NO;
                }
            }
            const unsigned long long m = __ballot(cl == YES);
            if (!m) {
                done = true;
                sp = 0;
                break;
            }
            const int j = 63 - __clzll((long long)m);
            cf = bcastu(e_first, j), cc = bcastu(e_count, j);
            sp = j;
        }
    }
    // back to lane r: its traversal state, hit, and (when it stops at a big leaf) its stack
    if (lane == r) {
        T.first = cf, T.count = cc, T.sp = S::empty(rc) + sp * S::STEP;
        h.best = best, h.kind = kind, h.id = id, h.bx = bx, h.by = by;
        active = !done;
    }
    if (!done) {
        if (lane < sp && lane < SL) col[lane * S::LANES] = e_idx;
        for (int j = SL; j < sp; j++) {
            const uint32_t v = bcastu(e_idx, j);
            if (lane == r) stk.put(S::empty(rc) + j * S::STEP, v);
        }
    }
}

// ---------------------------------------------------------------------------------------
// Wave pairs (RT_PAIR = K, experiment: two waves per workgroup).  A wave's traversal ends with a tail: a
// few lanes still stepping while the rest wait (config 2, 7 waves per SIMD: small-step iterations with 1-4
// active lanes are 13 % of wave cycles, lone-lane traversals 4 %), and every one of those iterations is
// issued for 64 lanes.  Here a wave whose small phase is down to <= K rays (no lane waiting at a big leaf)
// hands them to the other wave of its workgroup, which runs them in its FREE lanes -- lanes with no segment
// this call (their pixel is done), whose ray, hit and traversal registers are dead -- beside its own rays;
// the donor sleeps until their hits come back.  Exact by construction: a ray's traversal is the same
// sequence of steps whichever lane runs it; its LDS stack stays where it is (Stack: the stack pointer
// carries the ray's column), only rays whose entries all live in LDS move, and an adopted ray finishes where
// it was adopted.  The exchange goes through an LDS mailbox: word 0 the protocol word, then field f of ray k
// at 1 + f PAIR_K + k of the posting wave's region (21 fields: o, d, nd, 1/d, fast, hit, first, count, sp), the hit coming back in its own
// fields.  Protocol word: bit w = wave w is in trace and may be handed rays, bits 8 + 8w.. = its free lanes,
// bits 24-25 = phase (EMPTY, POSTED, ADOPTED, DONE), bit 26 = the posting wave, bits 27-31 = ray count.  Only
// lane 0 of a wave changes it (compare-and-swap); the posting wave waits for DONE, the other one adopts a
// POSTED hand-over before it may leave trace, so nothing is left behind and nothing waits on a wave that
// cannot answer.
// ---------------------------------------------------------------------------------------
#if defined(RT_PAIR)
constexpr int PAIR_K = RT_PAIR;
constexpr uint32_t PH_EMPTY = 0u, PH_POSTED = 1u, PH_ADOPTED = 2u, PH_DONE = 3u;
constexpr int PAIR_FIELDS = 21;
constexpr int PAIR_MAIL_WORDS = 1 + 2 * PAIR_FIELDS * PAIR_K;  // the protocol word + one region per posting wave
// the region wave w posts its rays in (and gets their hits back in): a wave never writes into the region of a
// hand-over it did not post
__device__ __forceinline__ uint32_t* pair_region(uint32_t* mail, uint32_t w) { return mail + w * PAIR_FIELDS * PAIR_K; }
__device__ __forceinline__ uint32_t pair_phase(uint32_t st) { return (st >> 24) & 3u; }
__device__ __forceinline__ uint32_t pair_free(uint32_t st, uint32_t w) { return (st >> (8u + 8u * w)) & 127u; }
__device__ __forceinline__ uint32_t pair_load(uint32_t* mail) {
    return (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)__hip_atomic_load(mail, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
// lane 0 replaces the protocol word by f(old) while f accepts old; returns (wave-uniform) whether it did
template <class F>
__device__ __forceinline__ bool pair_update(uint32_t* mail, F f) {
    int ok = 0;
    if ((threadIdx.x & 63u) == 0) {
        uint32_t old = __hip_atomic_load(mail, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP), nw;
        while (f(old, nw)) {
            if (__hip_atomic_compare_exchange_strong(mail, &old, nw, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP)) {
                ok = 1;
                break;
            }
        }
    }
    return __builtin_amdgcn_readfirstlane(ok) != 0;
}
__device__ __forceinline__ void pair_put_hit(uint32_t* mail, int k, const Hit& h) {
    uint32_t* m = mail + 1 + k;
    m[13 * PAIR_K] = __float_as_uint(h.best), m[14 * PAIR_K] = (uint32_t)h.kind, m[15 * PAIR_K] = h.id;
    m[16 * PAIR_K] = __float_as_uint(h.bx), m[17 * PAIR_K] = __float_as_uint(h.by);
}
__device__ __forceinline__ void pair_get_hit(const uint32_t* mail, int k, Hit& h) {
    const uint32_t* m = mail + 1 + k;
    h.best = __uint_as_float(m[13 * PAIR_K]), h.kind = (int)m[14 * PAIR_K], h.id = m[15 * PAIR_K];
    h.bx = __uint_as_float(m[16 * PAIR_K]), h.by = __uint_as_float(m[17 * PAIR_K]);
}
__device__ __forceinline__ void pair_put_ray(uint32_t* mail, int k, const Ray& R, const Hit& h, const Trav& T) {
    uint32_t* m = mail + 1 + k;
    const float v[12] = {R.o.x, R.o.y, R.o.z, R.d.x, R.d.y, R.d.z, R.nd.x, R.nd.y, R.nd.z, R.r.x, R.r.y, R.r.z};
    for (int f = 0; f < 12; f++) m[f * PAIR_K] = __float_as_uint(v[f]);
    m[12 * PAIR_K] = R.fast ? 1u : 0u;
    pair_put_hit(mail, k, h);
    m[18 * PAIR_K] = T.first, m[19 * PAIR_K] = T.count, m[20 * PAIR_K] = (uint32_t)T.sp;
}
__device__ __forceinline__ void pair_get_ray(const uint32_t* mail, int k, Ray& R, Hit& h, Trav& T) {
    const uint32_t* m = mail + 1 + k;
    R.o = rtm::mk(__uint_as_float(m[0]), __uint_as_float(m[PAIR_K]), __uint_as_float(m[2 * PAIR_K]));
    R.d = rtm::mk(__uint_as_float(m[3 * PAIR_K]), __uint_as_float(m[4 * PAIR_K]), __uint_as_float(m[5 * PAIR_K]));
    R.nd = rtm::mk(__uint_as_float(m[6 * PAIR_K]), __uint_as_float(m[7 * PAIR_K]), __uint_as_float(m[8 * PAIR_K]));
    R.r = rtm::mk(__uint_as_float(m[9 * PAIR_K]), __uint_as_float(m[10 * PAIR_K]), __uint_as_float(m[11 * PAIR_K]));
    R.fast = m[12 * PAIR_K] != 0u;
    pair_get_hit(mail, k, h);
    T.first = m[18 * PAIR_K], T.count = m[19 * PAIR_K], T.sp = (int)m[20 * PAIR_K];
}
#endif

#if defined(RT_GROUP)
// ---------------------------------------------------------------------------------------
// Group traversal (experiment, -DRT_GROUP = most rays): lone_traverse for 2-4 rays at
// once.  When the small phase is down to n = 2..RT_GROUP rays and every other lane is done (no lane waits at a
// big leaf), the wave splits into n groups: each ray's own lane (its OWNER) plus the done lanes dealt round
// robin (MEMBERS; their ray and traversal registers are dead, their hit is not and is left alone).  Every
// lane of a group holds the group's ray (copied once from the owner), current node, depth and closest
// distance, and runs the inner steps' filtered-exact decisions itself; the group's stack is spread over its
// members (member e holds entry e with its filtered tmin, as in lone_traverse), so a pop is one ballot and
// the highest passing member of the group; the owner alone tests a small leaf (pair_test, its own hit) and
// the group's distance follows by a permute.  Any group reaching a big leaf, or a push its members cannot
// hold, ends group mode for all: stacks go back to the owners' LDS columns, the big-leaf rounds take over.
// The same steps in the same order per ray: bit-exact by construction.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bperm(uint32_t v, int src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
__device__ __forceinline__ float bpermf(float v, int src) { return __uint_as_float(bperm(__float_as_uint(v), src)); }
__device__ __forceinline__ uint32_t rank_in(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

#if defined(RT_GROUP_CALL)  // a real call: the trace loop's register allocation stays the production one
#define RT_GROUP_INLINE __attribute__((noinline))
#else
#define RT_GROUP_INLINE __forceinline__
#endif
template <class S>
__device__ RT_GROUP_INLINE void group_traverse(const float4* nodes4, const float4* spairs, const S& stk,
                                               unsigned long long mS, Ray& R, Hit& h, Trav& T, bool& active) {
    constexpr int SL = S::LDS_ENTRIES;
    const int lane = (int)(threadIdx.x & 63u);
    const uint32_t n = (uint32_t)__popcll(mS);
    const bool owner = ((mS >> lane) & 1ull) != 0;
    const uint32_t mrank = rank_in(~mS);
    const uint32_t gid = owner ? rank_in(mS) : mrank % n;
    const int eidx = owner ? -1 : (int)(mrank / n);
    const int cap = min((int)((64u - n) / n), SL);  // entries every group's members can hold, all in LDS at exit
    // the owners' lanes (wave-uniform), then this lane's group owner and group mask
    unsigned long long rest = mS, gm = 0;
    int ol = lane;
    for (uint32_t k = 0; k < n; k++) {
        const int lk = __ffsll((long long)rest) - 1;
        rest &= rest - 1;
        const unsigned long long mk = __ballot(gid == k);
        if (gid == k) ol = lk, gm = mk;
    }
    // the group's ray, node, depth and closest distance from its owner (members' ray registers are dead)
    R.o = rtm::mk(bpermf(R.o.x, ol), bpermf(R.o.y, ol), bpermf(R.o.z, ol));
    R.d = rtm::mk(bpermf(R.d.x, ol), bpermf(R.d.y, ol), bpermf(R.d.z, ol));
    R.nd = rtm::mk(bpermf(R.nd.x, ol), bpermf(R.nd.y, ol), bpermf(R.nd.z, ol));
    R.r = rtm::mk(bpermf(R.r.x, ol), bpermf(R.r.y, ol), bpermf(R.r.z, ol));
    R.fast = bperm(R.fast ? 1u : 0u, ol) != 0u;
    uint32_t cf = bperm(T.first, ol), cc = bperm(T.count, ol);
    const int osp = (int)bperm((uint32_t)T.sp, ol);
    const int ocol = S::column(osp);
    int gd = S::depth(osp);
    float gb = bpermf(h.best, ol);
    uint32_t* const col = stk.lds0 + ocol;
    // member e: entry e of its group's stack, with its filtered tmin (lone_traverse's entry state)
    uint32_t e_idx = 0, e_first = 0, e_count = 0;
    float e_tmin = 0.0f;
    bool e_exact = false;
    if (eidx >= 0 && eidx < gd) {
        e_idx = col[eidx * S::LANES];
        const float4 lo = ldo(nodes4, 2 * e_idx), hi = ldo(nodes4, 2 * e_idx + 1);
        float tx;
        if (R.fast) {
            slab_approx(R, lo, hi, &e_tmin, &tx);
        } else {
            slab_exact(R, lo, hi, &e_tmin, &tx);
            e_exact = true;
        }
        e_first = __float_as_uint(hi.z), e_count = __float_as_uint(hi.w);
    }
    bool gdone = false;  // this lane's group: its ray's traversal is over
    for (;;) {
        bool do_pop = false, leave = false;
        if (!gdone) {
            if (cc == 0) {
                if (gd >= cap) {
                    leave = true;  // a push might not fit the members: back to per-lane steps
                } else {
                    const float4 l0 = ldo(nodes4, 2 * cf), l1 = ldo(nodes4, 2 * cf + 1);
                    const float4 r0 = ldo(nodes4, 2 * cf + 2), r1 = ldo(nodes4, 2 * cf + 3);
                    float tl = 0.0f, tlx = 0.0f, tr = 0.0f, trx = 0.0f;
                    int okl = UNSURE, okr = UNSURE, rlt = UNSURE;
                    if (R.fast) {
                        slab_approx(R, l0, l1, &tl, &tlx);
                        slab_approx(R, r0, r1, &tr, &trx);
                        okl = classify_ok(tl, tlx);
                        okr = classify_ok(tr, trx);
                        rlt = okr == YES ? classify_lt(tr, gb) : NO;
                    }
                    bool exact_l = false;
                    if (okl == UNSURE || okr == UNSURE || rlt == UNSURE) {
                        slab_exact(R, l0, l1, &tl, &tlx);
                        slab_exact(R, r0, r1, &tr, &trx);
                        okl = (tlx >= tl && tlx > 0.0f) ? YES : NO;
                        okr = (trx >= tr && trx > 0.0f) ? YES : NO;
                        rlt = (okr == YES && tr < gb) ? YES : NO;
                        exact_l = true;
                    }
                    if (rlt == YES) {
                        if (okl == YES) {
                            if (eidx == gd) e_idx = cf, e_tmin = tl, e_exact = exact_l, e_first = __float_as_uint(l1.z),
                                            e_count = __float_as_uint(l1.w);
                            gd++;
                        }
                        cf = __float_as_uint(r1.z), cc = __float_as_uint(r1.w);
                    } else {
                        bool llt = false;
                        if (okl == YES) {
                            int cl = exact_l ? (tl < gb ? YES : NO) : classify_lt(tl, gb);
                            if (cl == UNSURE) {
                                float te, tx;
                                slab_exact(R, l0, l1, &te, &tx);
                                cl = te < gb ? YES : NO;
                            }
                            llt = cl == YES;
                        }
                        if (llt) cf = __float_as_uint(l1.z), cc = __float_as_uint(l1.w);
                        else do_pop = true;
                    }
                }
            } else if (cc <= (uint32_t)BIG) {
                if (owner)  // the small leaf, in leaf order, on the owner's own hit
                    for (uint32_t i = cf; i < cf + cc; i += 2) pair_test(R, ld_pair(spairs, i), h);
                do_pop = true;
            } else {
                leave = true;  // a big leaf: the wave's big-leaf rounds
            }
        }
        gb = bpermf(h.best, ol);  // (owners' distances; members' own hits untouched)
        if (__ballot(leave)) break;
        // pops: members holding live entries test them; the group continues at its highest passing entry
        int cl = NO;
        if (!gdone && do_pop && eidx >= 0 && eidx < gd) {
            cl = e_exact ? (e_tmin < gb ? YES : NO) : classify_lt(e_tmin, gb);
            if (cl == UNSURE) {
                const float4 lo = ldo(nodes4, 2 * e_idx), hi = ldo(nodes4, 2 * e_idx + 1);
                float tx;
                slab_exact(R, lo, hi, &e_tmin, &tx);
                e_exact = true;
                cl = e_tmin < gb ? YES : NO;
            }
        }
        const unsigned long long P = __ballot(cl == YES) & gm;
        const int w = P ? 63 - __clzll((long long)P) : lane;
        const uint32_t wf = bperm(e_first, w), wc = bperm(e_count, w), we = bperm((uint32_t)eidx, w);
        if (!gdone && do_pop) {
            if (P) {
                cf = wf, cc = wc, gd = (int)we;
            } else {
                gdone = true;
                if (owner) active = false;
            }
        }
        if (!__ballot(!gdone)) break;
    }
    // back to per-lane state: the owners of unfinished rays take the group's node and depth, the members
    // put their entries back into the owner's LDS column (gd <= cap <= the LDS rows)
    if (!gdone) {
        if (owner) T.first = cf, T.count = cc, T.sp = S::empty(ocol) + gd * S::STEP;
        if (eidx >= 0 && eidx < gd) col[eidx * S::LANES] = e_idx;
    }
}
#endif

// BVHRayHit for one lane (`live` = the lane has a segment to trace), every lane of the wave
// calling.  Small steps run while any lane has one; big leaves wait until every lane is done
// or waiting at one.  MODE & 3 -- 0: big leaves through pair records (shared-leaf loop and
// cooperative rounds); 1: pairs in the shared-leaf loop, scalar cooperative rounds; 2: scalar
// records only.  MODE & 4: leaves with a leaf tree walk it (a statistics frame then counts the
// reference's triangle tests plus the tree's own work).
template <bool STATS, int MODE, class S, class C>
__device__ __forceinline__ void trace(const float4* nodes4, const float4* tris, const float4* pairs,
                                      const float4* tree, const float4* ltris, const float4* flat,
                                      const float4* spairs, uint32_t tune, const S& stk, uint32_t* scratch,
                                      Ray& R, Hit& h, bool live, C& c, const float4* quads = nullptr,
                                      const float4* units = nullptr, const uint32_t* face_leaf = nullptr,
                                      uint32_t* mail = nullptr) {
    Trav T{0, 0, 0};
    bool active = live && trav_begin<STATS>(nodes4, R, h, T, c);
#if defined(RT_PAIR)
    // wave pairs (above): the production split-step kernels without leaf trees, screens or refill
#if defined(RT_PAIR_NOEXCH)  // A/B: the pair workgroups without the exchange
    constexpr bool PAIR = false;
#else
    constexpr bool PAIR = !STATS && (MODE & 8) == 0 && (MODE & 4) == 0 && (MODE & 16) != 0 && (MODE & 32) == 0 &&
                          (MODE & 64) == 0;
#endif
#ifndef RT_PAIR_EVERY
#define RT_PAIR_EVERY 1  // iterations between two looks at the mailbox
#endif
    uint32_t pair_tick = 0;
    const uint32_t pw = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // this wave of the pair
    const uint32_t po = 1u - pw;
    int adopted = -1;         // mail slot of the other wave's ray this lane runs, or -1
    uint32_t n_adopted = 0;   // rays adopted (wave-uniform)
    if (PAIR && mail) {       // in trace: may be handed up to (free lanes) rays
        const uint32_t nfree = min((uint32_t)__popcll(__ballot(!live)), 127u);
        pair_update(mail, [&](uint32_t o, uint32_t& nw) {
            nw = (o & ~(127u << (8u + 8u * pw))) | (1u << pw) | (nfree << (8u + 8u * pw));
            return true;
        });
    }
    auto pair_publish = [&]() {  // every adopted ray done: their hits back, DONE
        if (adopted >= 0) pair_put_hit(pair_region(mail, po), adopted, h);
        adopted = -1, n_adopted = 0;
        pair_update(mail, [](uint32_t o, uint32_t& nw) {
            nw = (o & ~(3u << 24)) | (PH_DONE << 24);
            return true;
        });
    };
#endif
    // big-leaf screens (screen_leaf, MODE bit 5): split-step variants for scenes that have them
    constexpr bool scr_on = !STATS && (MODE & 16) != 0 && (MODE & 32) != 0;
    constexpr bool TIMING = (MODE & 8) != 0;
    // deferred big leaves (defer_leaf): production, timing and refill variants, not the screen ones; D = this
    // lane's words, or null when deferral is off (RT_TUNE bit 24)
#if defined(RT_DEFER_ALL)  // experiment: every kernel defers (config 2's floor leaf too)
    constexpr bool DEFER = !STATS && (MODE & 32) == 0;
#else  // the leaf-tree kernels (config 2's 7-wave kernel spills 53 -> 186 dwords with the deferral compiled in)
    constexpr bool DEFER = !STATS && (MODE & 32) == 0 && (MODE & 4) != 0;
#endif
    uint32_t* const D = (DEFER && (tune & (1u << 24)) == 0) ? defer_words<MODE>(scratch) : nullptr;
    if (D) D[0] = DEFER_NONE;
    unsigned long long t0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
    for (;;) {
#if defined(RT_PAIR)
        if (PAIR && mail && (RT_PAIR_EVERY == 1 || (++pair_tick % RT_PAIR_EVERY) == 0)) {
            const uint32_t st = pair_load(mail);
            const uint32_t ph = pair_phase(st);
            if (ph == PH_POSTED && ((st >> 26) & 1u) != pw) {  // rays handed to this wave: free lanes take them
                const uint32_t n = st >> 27;
                const bool fr = !live && adopted < 0;
                const unsigned long long fm = __ballot(fr);
                const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
                if (fr && k < n) {
                    pair_get_ray(pair_region(mail, po), (int)k, R, h, T);
                    adopted = (int)k;
                    active = true;
                }
                n_adopted = n;
                pair_update(mail, [](uint32_t o, uint32_t& nw) {
                    nw = (o & ~(3u << 24)) | (PH_ADOPTED << 24);
                    return true;
                });
                continue;
            }
            if (n_adopted && !__ballot(adopted >= 0 && active)) pair_publish();
            const bool mine = active && T.count <= (uint32_t)BIG;  // this wave's small-phase rays
            const unsigned long long mS = __ballot(mine);
            const uint32_t nS = (uint32_t)__popcll(mS);
            if (!n_adopted && ph == PH_EMPTY && nS && nS <= (uint32_t)PAIR_K && mS == __ballot(active) &&
                ((st >> po) & 1u) && pair_free(st, po) >= nS && !__ballot(mine && S::depth(T.sp) > S::LDS_ENTRIES)) {
                const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(mS >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mS, 0u));
                if (mine) pair_put_ray(pair_region(mail, pw), (int)k, R, h, T);
                if (pair_update(mail, [&](uint32_t o, uint32_t& nw) {
                        if (pair_phase(o) != PH_EMPTY || !((o >> po) & 1u) || pair_free(o, po) < nS) return false;
                        nw = (o & 0x00ffffffu) | (PH_POSTED << 24) | (pw << 26) | (nS << 27);
                        return true;
                    })) {
                    // (bounded: a protocol error renders wrong pixels -- the parity tests catch those -- instead of
                    // hanging the device; ~2^22 sleeps is far beyond any traversal)
                    for (uint32_t spin = 0; pair_phase(pair_load(mail)) != PH_DONE && spin < (1u << 22); spin++)
                        __builtin_amdgcn_s_sleep(2);
                    if (mine) {
                        pair_get_hit(pair_region(mail, pw), (int)k, h);
                        active = false;
                    }
                    pair_update(mail, [](uint32_t o, uint32_t& nw) {
                        nw = o & 0x00ffffffu;  // EMPTY
                        return true;
                    });
                    continue;
                }
            }
        }
#endif
        if constexpr ((MODE & 16) != 0) {
            // split small steps: inner-node steps and small-leaf steps run in separate wave
            // iterations (a lane at a small leaf waits until at least half as many lanes are at
            // one as at inner nodes), so an iteration pays for one of the two code paths instead
            // of both: 19.8 -> 18.3 ms/frame.  (A three-way split with pops as a third kind, the
            // wave picking the kind with the most lanes per unit of cost, measured the same.)
            const bool inner = active && T.count == 0;
            const bool leafs = active && T.count > 0 && (T.count <= (uint32_t)BIG || (scr_on && !(T.sp & SCREENED)));
            const unsigned long long mI = __ballot(inner), mL = __ballot(leafs);
            if (mI | mL) {
                const uint32_t nI = (uint32_t)__popcll(mI), nL = (uint32_t)__popcll(mL);
#if defined(RT_GROUP)
                if constexpr (!STATS && !scr_on && (MODE & 4) == 0) {
                    const uint32_t ng = nI + nL;
                    if (ng >= 2 && ng <= (uint32_t)RT_GROUP && (mI | mL) == __ballot(active) && spairs &&
                        !__ballot((inner || leafs) && S::depth(T.sp) >= min((int)((64u - ng) / ng), S::LDS_ENTRIES))) {
                        group_traverse(nodes4, spairs, stk, mI | mL, R, h, T, active);
                        continue;
                    }
                }
#endif
                if constexpr (!STATS) {
                    // one lane left in the small phase: the whole wave runs its DFS (lone_traverse),
                    // when its stack lives in LDS (RT_TUNE bit 26 turns this off); a lane that must
                    // screen a big leaf first takes an ordinary step
#ifndef RT_LONE_MAX
#define RT_LONE_MAX 1  // most small-phase lanes for which the wave runs one of them as a lone ray
#endif
                    if (nI + nL <= (uint32_t)RT_LONE_MAX && (tune & (1u << 26)) == 0) {
                        const int r = __ffsll((long long)(mI | mL)) - 1;
                        if (S::depth(__builtin_amdgcn_readlane(T.sp, r)) <= S::LDS_ENTRIES &&
                            (!scr_on || (uint32_t)__builtin_amdgcn_readlane((int)T.count, r) <= (uint32_t)BIG)) {
#ifdef RT_LANE_HIST  // diagnostic build (tools/lane_hist.sh): wave cycles of the lone-lane tails
                            const unsigned long long tl0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
#endif
                            lone_traverse(nodes4, tris, stk, r, R, h, T, active);
#ifdef RT_LANE_HIST
                            if (TIMING) c.cy_ttri += __builtin_amdgcn_s_memtime() - tl0;
#endif
                            continue;
                        }
                    }
                }
                // leaf step when nL * 4 >= nI * (q + 1); q = 1 measured best (RT_TUNE bits 13-15: q + 1)
                const uint32_t qv = (tune >> 13) & 7u, q = qv ? qv - 1u : 1u;
                if (TIMING) c.w_small++, c.l_small += inner || leafs;
#ifdef RT_LANE_HIST  // diagnostic build: wave cycles of small-step iterations by active-lane count
                const unsigned long long th0 = TIMING ? __builtin_amdgcn_s_memtime() : 0;
#endif
#ifdef RT_COMBINE_T
                // few lanes of both kinds: one iteration serves both (their loads overlap; the split
                // exists to gather lanes per kind, which matters little when both groups are small)
                if (!scr_on && mI && mL && nI + nL <= (uint32_t)RT_COMBINE_T) {
                    if (inner || leafs) {
                        active = small_step<STATS, false, DEFER>(nodes4, tris, spairs, stk, R, h, T, c, nullptr, D);
                        if (TIMING) c.lane_work++;
                    }
                } else
#endif
                if (!mI || nL * 4u >= nI * (q + 1u)) {
                    if (leafs) {
                        active = small_step<STATS, scr_on>(nodes4, tris, spairs, stk, R, h, T, c, pairs);
                        if (TIMING) c.lane_work++;
                    }
                } else if (inner) {
                    active = small_step<STATS, false, DEFER>(nodes4, tris, spairs, stk, R, h, T, c, nullptr, D);
                    if (TIMING) c.lane_work++;
                }
#ifdef RT_LANE_HIST
                if (TIMING) {
                    const unsigned long long dt = __builtin_amdgcn_s_memtime() - th0;
                    const uint32_t n = nI + nL;
                    c.ktest += n <= 4u ? dt : 0ull;            // 1-4 active lanes
                    c.ktri += (n > 4u && n <= 16u) ? dt : 0ull;  // 5-16
                    c.cy_tcl += dt;                            // every small-step iteration
                    c.r_shared += n <= 4u;                     // iterations with 1-4 lanes
                }
#endif
                continue;
            }
        }
        const bool small = active && T.count <= (uint32_t)BIG;
        if (__ballot(small)) {
            if (STATS) {
                c.w_small += (threadIdx.x & 63) == 0;
                c.l_small += small;
            } else if (TIMING) {
                c.w_small++;
                c.l_small += small;
            }
            if (small) {
                active = small_step<STATS>(nodes4, tris, spairs, stk, R, h, T, c);
                if (TIMING) c.lane_work++;
            }
            continue;
        }
        if (TIMING) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            c.cy_small += t1 - t0;
            t0 = t1;
        }
        const unsigned long long big = __ballot(active);  // every active lane waits at a big leaf
        if (!big) {
            if (DEFER && D) {
                // Every lane's rest is done: the deferred leaves' rounds, through the loop's own big-leaf round.
                // END1 runs the leaf from the bound the rest left: just above a hit found after the leaf (the
                // leaf came first in DFS order and wins that tie), or the hit it was entered with (strict <).
                // When it finds nothing there, the rest's best hit F stands -- if the reference, having run the
                // leaf first, still reaches F's leaf P: P's ancestors contain its box, so their rounded slab tmin
                // is at most tmin_P, and it does iff the leaf holds nothing at or below tmin_P.  tmin_P <= t_F:
                // shown by END1.  tmin_P > t_F (a rounded distance below its own box's rounded entry: a triangle
                // on a box face, or an ill-conditioned grazing hit): END2 runs the leaf up to tmin_P, and if it
                // finds anything the lane is redone from the root in the reference order with `closest` = the
                // distance it had at the leaf (the leaf then accepts a hit, so the fields of the hit it had at the
                // leaf never survive, and nothing before the leaf in DFS order lies below that distance).
                const uint32_t st = D[0];
                bool go = false;
                if (st < DEFER_END2) {  // deferred: END1
                    const uint32_t entry = D[128], h1 = __float_as_uint(h.best);
                    D[192] = h1, D[256] = st, D[0] = DEFER_END1;  // D[256]: the leaf until END2 needs the word
                    h.best = h1 != entry ? next_up(h.best) : h.best;
                    T.first = st, T.count = D[64];
                    go = true;
                } else if (st == DEFER_END1) {
                    const uint32_t entry = D[128], h1 = D[192];
                    const float bnd = h1 != entry ? next_up(__uint_as_float(h1)) : __uint_as_float(h1);
                    D[0] = DEFER_NONE;
                    if (__float_as_uint(h.best) == __float_as_uint(bnd)) {  // nothing in the leaf at or below F
                        h.best = __uint_as_float(h1);
                        if (h1 != entry) {  // F came after the leaf: the guard
                            const uint32_t P = face_leaf ? face_leaf[h.id] : 0xffffffffu;
                            float tp = INFINITY, tx;
                            if (P < 0xfffffffeu) slab_exact(R, ldo(nodes4, 2 * P), ldo(nodes4, 2 * P + 1), &tp, &tx);
                            if (tp > h.best) {  // (F's leaf unknown: tp = inf, the whole leaf below the entry)
                                const float b2 = P < 0xfffffffeu ? next_up(tp) : __uint_as_float(entry);
                                T.first = D[256], T.count = D[64];
                                D[256] = __float_as_uint(b2), D[0] = DEFER_END2;
                                h.best = b2;
                                if (TIMING) c.end2++;
                                go = true;
                            }
                        }
                    }
                } else if (st == DEFER_END2) {
                    if (__float_as_uint(h.best) != D[256]) {  // the leaf holds a hit at or below tmin_P: redo
                        h.best = __uint_as_float(D[128]);
                        D[0] = DEFER_OFF;
                        if (TIMING) c.redo++;
                        active = trav_begin<STATS>(nodes4, R, h, T, c);
                    } else {
                        h.best = __uint_as_float(D[192]);
                        D[0] = DEFER_NONE;
                    }
                }
                if (go) active = true;
                if (__ballot(active)) continue;
            }
#if defined(RT_PAIR)
            if (PAIR && mail) {
                if (n_adopted) pair_publish();
                // leave trace: no more rays for this wave, unless a hand-over to it is already POSTED
                if (!pair_update(mail, [&](uint32_t o, uint32_t& nw) {
                        if (pair_phase(o) == PH_POSTED && ((o >> 26) & 1u) != pw) return false;
                        nw = o & ~(1u << pw) & ~(127u << (8u + 8u * pw));
                        return true;
                    }))
                    continue;  // adopt it first
            }
#endif
            break;
        }
        if (big_round_d<STATS, MODE>(nodes4, D, tris, pairs, quads, units, tree, ltris, flat, scratch, tune, big, active, R, h,
                                     T, c)) {
            // a big leaf run alone (cooperative round) costs about as much as 3 small steps
            if (TIMING) c.lane_work += 3;
            if constexpr (scr_on) T.sp &= ~SCREENED;
            active = pop_d<DEFER>(nodes4, D, stk, R, h, T);
        }
        if (TIMING) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            c.cy_big += t1 - t0;
            t0 = t1;
        }
    }
}

}  // namespace rtfast
