// rt_ref.hip -- the two straight restatements of BVHRayHit the production tracer is checked
// against and falls back to: the reference-layout tracer (the reference's own arrays, literally:
// foreign scenes before their mirror exists, and the gated second grid of a foreign frame) and the
// exact-division flat tracer (A/B).  One 64-lane workgroup per 8x8 sub-tile.
#include <hip/hip_runtime.h>

#include "rt_abi.h"
#include "rt_device.h"
#include "rt_math.h"
#include "rt_common.h"
#include "leaftree.h"
#include "rt_fast.h"
#include "rt_render.h"

namespace rtk {
namespace {

using rtfast::Hit;

// The sphere loop of GetRayHit (main_raytracing.cu:88-103): strict `<` replaces.
template <bool STATS>
__device__ __forceinline__ void trace_spheres(const RenderArgs& a, rtm::f3 ro, rtm::f3 nd, Hit& h, Counters& c) {
    for (int i = 0; i < a.sphere_count; i++) {
        const GeometrySphere& sp = a.spheres[i];
        float dist;
        if (rtd::intersect_sphere(ro, nd, ld3(sp.position), sp.radius * sp.radius, &dist)) {
            if (dist >= h.best) continue;
            h.best = dist;
            h.kind = 1;
            h.id = (uint32_t)i;
            if (STATS) c.sacc++;
        }
    }
}

// BVHRayHit (main_raytracing.cu:33-81) on the reference arrays, literally: uint32 stack,
// pop, AABB test against the current closest distance, leaf -> face_indices -> faces ->
// vertices, inner -> push first, first+1 (right child popped first).  Used for scenes
// whose buffers were not uploaded through rt_scene_upload (no leaf-ordered mirror).
struct RefTracer {
    static constexpr int WORDS = 1;
    template <int STACK, bool STATS>
    __device__ static void trace(const RenderArgs& a, uint32_t* stk, rtm::f3 ro, rtm::f3 rd, rtm::f3 nd, Hit& h,
                                 Counters& c) {
        int sp = 0;
        stk[0] = 0u;
        sp = 1;
        while (sp) {
            const GPUBVHNode& node = a.nodes[stk[(--sp) * WAVE]];
            if (STATS) c.node++;
            if (!rtd::intersect_aabb(ro, rd, node.bmin, node.bmax, h.best)) continue;
            if (node.prim_count > 0) {
                for (uint32_t i = 0; i < node.prim_count; i++) {
                    const uint32_t fi = a.face_indices[node.first_index + i];
                    const GPUFace f = a.faces[fi];
                    float bx, by, dist;
                    if (STATS) c.tri++;
                    if (rtd::intersect_triangle(ro, nd, ld3(a.vertices[f.v0].position), ld3(a.vertices[f.v1].position),
                                                ld3(a.vertices[f.v2].position), &bx, &by, &dist)) {
                        if (dist >= h.best || dist < 0.0f) continue;
                        h.best = dist;
                        h.kind = 2;
                        h.id = fi;
                        h.bx = bx;
                        h.by = by;
                        if (STATS) c.tacc++;
                    }
                }
            } else {
                stk[(sp++) * WAVE] = node.first_index;
                stk[(sp++) * WAVE] = node.first_index + 1;
            }
        }
    }
};

// The slab part of IntersectAABB (Math.h:50-61) that does not depend on the closest
// distance: returns tmin and whether tmax >= tmin && tmax > 0.  The remaining clause,
// tmin < ray_length, is evaluated when the reference would pop the node.
__device__ __forceinline__ bool slab(rtm::f3 o, rtm::f3 d, float4 lo, float4 hi, float* tmin_out) {
    // lo = (bmin.x, bmin.y, bmin.z, bmax.x), hi = (bmax.y, bmax.z, first, count)
    float tx1 = (lo.x - o.x) / d.x, tx2 = (lo.w - o.x) / d.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    float ty1 = (lo.y - o.y) / d.y, ty2 = (hi.x - o.y) / d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2)), tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (lo.z - o.z) / d.z, tz2 = (hi.y - o.z) / d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2)), tmax = fminf(tmax, fmaxf(tz1, tz2));
    *tmin_out = tmin;
    return tmax >= tmin && tmax > 0;
}

// The same traversal, re-associated for the GPU without changing a single decision:
//  * siblings are adjacent (children of an inner node at first, first+1), so an inner node
//    loads both children (64 contiguous bytes) and runs both slab tests at once; the right
//    child -- the one the reference pops next -- continues in registers, the left child is
//    pushed with its tmin, and `tmin < closest` is checked when it is popped, against the
//    closest distance at that moment, exactly as the reference's pop-time test;
//  * leaves read the leaf-ordered FlatTri mirror (one 48-byte record per test instead of
//    the index -> face -> 3 vertex dependent-load chain);
//  * node visit order, tested triangles and their order, and every comparison are the
//    reference's, so the closest hit (including ties between coincident faces) is identical.
// Stack entries: (node index, tmin bits) in LDS, [entry][lane].
struct FlatTracer {
    static constexpr int WORDS = 2;
    template <int STACK, bool STATS>
    __device__ static void trace(const RenderArgs& a, uint32_t* stk, rtm::f3 ro, rtm::f3 rd, rtm::f3 nd, Hit& h,
                                 Counters& c) {
        const float4* nodes4 = reinterpret_cast<const float4*>(a.nodes);
        // root (node 0), tested against the closest sphere distance
        float4 lo = nodes4[0], hi = nodes4[1];
        float tmin;
        if (STATS) c.node++;
        if (!slab(ro, rd, lo, hi, &tmin) || !(tmin < h.best)) return;
        uint32_t first = __float_as_uint(hi.z), count = __float_as_uint(hi.w);
        int sp = 0;
        for (;;) {
            if (count > 0) {
                // leaf: the reference's per-triangle loop over face_indices[first .. first+count)
                for (uint32_t i = first; i < first + count; i++) {
                    const FlatTri t = a.tris[i];
                    if (STATS) c.tri++;
                    const rtm::f3 v0 = rtm::mk(t.a.x, t.a.y, t.a.z);
                    const rtm::f3 e1 = rtm::mk(t.a.w, t.b.x, t.b.y);
                    const rtm::f3 e2 = rtm::mk(t.b.z, t.b.w, t.c.x);
                    float bx, by, dist;
                    if (rtd::intersect_triangle_e(ro, nd, v0, e1, e2, &bx, &by, &dist)) {
                        if (dist >= h.best || dist < 0.0f) continue;
                        h.best = dist;
                        h.kind = 2;
                        h.id = __float_as_uint(t.c.y);
                        h.bx = bx;
                        h.by = by;
                        if (STATS) c.tacc++;
                    }
                }
            } else {
                const float4 l0 = nodes4[2 * first], l1 = nodes4[2 * first + 1];
                const float4 r0 = nodes4[2 * first + 2], r1 = nodes4[2 * first + 3];
                if (STATS) c.node += 2;
                float tl, tr;
                const bool okl = slab(ro, rd, l0, l1, &tl);
                const bool okr = slab(ro, rd, r0, r1, &tr);
                if (okr && tr < h.best) {
                    if (okl) {
                        stk[(sp * 2) * WAVE] = first;
                        stk[(sp * 2 + 1) * WAVE] = __float_as_uint(tl);
                        sp++;
                    }
                    first = __float_as_uint(r1.z), count = __float_as_uint(r1.w);
                    continue;
                }
                if (okl && tl < h.best) {
                    first = __float_as_uint(l1.z), count = __float_as_uint(l1.w);
                    continue;
                }
            }
            // pop until an entry passes tmin < closest
            bool found = false;
            while (sp > 0) {
                sp--;
                const uint32_t idx = stk[(sp * 2) * WAVE];
                const float t = __uint_as_float(stk[(sp * 2 + 1) * WAVE]);
                if (t < h.best) {
                    const float4 nh = nodes4[2 * idx + 1];
                    first = __float_as_uint(nh.z), count = __float_as_uint(nh.w);
                    found = true;
                    break;
                }
            }
            if (!found) break;
        }
    }
};

// The per-pixel path tracer: raytracing_kernel_main + ray_color (main_raytracing.cu:111-200).
template <class Tracer, int STACK, bool STATS>
__device__ __forceinline__ void shade_pixel(const RenderArgs& a, uint32_t* stk, int x, int y, size_t rng_index,
                                            size_t out_slot, Counters& c) {
    rt_rng_state* rs = a.rng + rng_index;
    rtm::Xorwow rng{rs->d, rs->v[0], rs->v[1], rs->v[2], rs->v[3], rs->v[4]};
    const rtm::f3 cam_o = ld3(a.cam.origin), cam_h = ld3(a.cam.horizontal), cam_v = ld3(a.cam.vertical),
                  cam_ll = ld3(a.cam.lower_left_corner);
    float acc_r = 0.0f, acc_g = 0.0f, acc_b = 0.0f, acc_a = 0.0f;

    for (int sample = 0; sample < a.spp; sample++) {
        // main_raytracing.cu:190: uv = (pixel + vec2(rng(), rng())) / vec2(W, H), u drawn first
        const float ru = rng.uniform();
        const float rv = rng.uniform();
        const float uvx = ((float)x + ru) / (float)a.width;
        const float uvy = ((float)y + rv) / (float)a.height;
        // GPUCamera::GetRay (GPUScene.h:13): llc + u*h + v*v - origin (not normalized)
        rtm::f3 ro = cam_o;
        rtm::f3 rd = rtm::sub(rtm::add(rtm::add(cam_ll, rtm::muls(cam_h, uvx)), rtm::muls(cam_v, uvy)), cam_o);

        rtm::f3 color = rtm::mk(0, 0, 0), thr = rtm::mk(1, 1, 1);
        for (int bounce = 0; bounce < a.bounces; bounce++) {
            c.seg++;
            // GetRayHit (main_raytracing.cu:83-109)
            const rtm::f3 nd = rtm::normalize(rd);
            Hit h;
            h.best = 1e30f;
            h.kind = 0;
            h.id = 0;
            h.bx = h.by = 0.0f;
            trace_spheres<STATS>(a, ro, nd, h, c);
            Tracer::template trace<STACK, STATS>(a, stk, ro, rd, nd, h, c);

            // GetRayHit returns `result.distance < max_distance` (main_raytracing.cu:108): a hit whose
            // accepted distance is NaN counts as a miss, as in the reference
            if (h.kind != 0 && h.best < 1e30f) {
                if (STATS) c.hit++;
                // Attributes of the final closest hit (the reference recomputes them on every
                // accept; only the last accept survives, so computing them once is identical).
                const rtm::f3 pos = rtm::add(ro, rtm::muls(nd, h.best));
                rtm::f3 nrm;
                uint32_t mat;
                if (h.kind == 1) {
                    const GeometrySphere& sp = a.spheres[h.id];
                    nrm = rtm::divs(rtm::sub(pos, ld3(sp.position)), sp.radius);
                    mat = (uint32_t)sp.material;
                } else {
                    const GPUFace f = a.faces[h.id];
                    const float bz = (1.0f - h.bx) - h.by;
                    nrm = rtm::normalize(rtm::add(rtm::add(rtm::muls(ld3(a.vertices[f.v0].normal), h.bx),
                                                           rtm::muls(ld3(a.vertices[f.v1].normal), h.by)),
                                                  rtm::muls(ld3(a.vertices[f.v2].normal), bz)));
                    if (rtm::dot(nd, nrm) >= 0.0f) nrm = rtm::neg(nrm);
                    mat = f.material;
                }
                const GPUMaterial& m = a.materials[mat];
                const float do_spec = (rng.uniform() < m.specular_percent) ? 1.0f : 0.0f;
                color = rtm::add(color, rtm::mul(thr, ld3(m.emissive)));
                const float om = 1.0f - do_spec;
                thr = rtm::mul(thr, rtm::mk(m.albedo[0] * om + m.specular[0] * do_spec,
                                            m.albedo[1] * om + m.specular[1] * do_spec,
                                            m.albedo[2] * om + m.specular[2] * do_spec));
                // GetRandomPointOnSphere (Random.h:23-46)
                const float zz = rng.uniform() * 2.0f - 1.0f;
                const float ang = rng.uniform() * 3.141592654f * 2.0f;
                const float rr = sqrtf(1.0f - zz * zz);
                const rtm::f3 sph = rtm::mk(rr * rtm::rt_cosf(ang), rr * rtm::rt_sinf(ang), zz);
                const rtm::f3 diffuse = rtm::normalize(rtm::add(nrm, sph));
                rtm::f3 spec = rtm::normalize(rtm::reflect(rd, nrm));
                spec = rtm::normalize(rtm::mix(spec, diffuse, m.roughness * m.roughness));
                const rtm::f3 ndir = rtm::normalize(rtm::add(rtm::muls(diffuse, om), rtm::muls(spec, do_spec)));
                ro = rtm::add(pos, rtm::muls(nrm, 0.01f));
                rd = ndir;
                // Russian roulette (main_raytracing.cu:140-148)
                const float p = rtm::gmax(thr.x, rtm::gmax(thr.y, thr.z));
                if (rng.uniform() > p) break;
                thr = rtm::muls(thr, 1.0f / p);
            } else {
                if (STATS) c.miss++;
                if (a.sky) {
                    const rtm::f3 dir = rtd::quat_rotate(a.qw, a.qx, a.qy, a.qz, rd);
                    const rtm::f3 cs = rtd::cube_sample(a.sky, a.sky_n, dir);
                    const rtm::f3 cl = rtm::mk(rtm::gmin(rtm::gmax(cs.x, 0.0f), 50.0f), rtm::gmin(rtm::gmax(cs.y, 0.0f), 50.0f),
                                               rtm::gmin(rtm::gmax(cs.z, 0.0f), 50.0f));
                    color = rtm::add(color, rtm::mul(thr, cl));
                }
                break;
            }
        }
        acc_r += color.x;
        acc_g += color.y;
        acc_b += color.z;
        acc_a += 1.0f;
    }

    // main_raytracing.cu:195-199
    const float fs = (float)a.spp;
    const rtm::f4 res{acc_r / fs, acc_g / fs, acc_b / fs, acc_a / fs};
    const float lerp = a.frame_index > 0 ? 1.0f / (float)(a.frame_index + 1) : 1.0f;
    float4 prev;
    float4* out;
    if (a.out_shard) {
        prev = a.last ? reinterpret_cast<const float4*>(a.last)[out_slot] : make_float4(0, 0, 0, 0);
        out = a.out_shard + out_slot;
    } else {
        prev = a.last ? *reinterpret_cast<const float4*>(a.last + (size_t)y * a.pitch + (size_t)x * 16)
                      : make_float4(0, 0, 0, 0);
        out = reinterpret_cast<float4*>(a.surface + (size_t)y * a.pitch + (size_t)x * 16);
    }
    const rtm::f4 o = rtm::mix4(rtm::f4{prev.x, prev.y, prev.z, prev.w}, res, lerp);
    *out = make_float4(o.x, o.y, o.z, 1.0f);

    rs->d = rng.d;
    rs->v[0] = rng.v0;
    rs->v[1] = rng.v1;
    rs->v[2] = rng.v2;
    rs->v[3] = rng.v3;
    rs->v[4] = rng.v4;
}

// One wave per workgroup; wave g renders the 8x8 sub-tile (g & 3) of shard tile (g >> 2).
// The hardware dispatcher hands out the next sub-tile as soon as a wave retires, which
// balances cheap (sky) against expensive (floor leaf) tiles.
template <class Tracer, int STACK, bool STATS>
__global__ __launch_bounds__(WAVE) void render_kernel(RenderArgs a) {
    if (a.gate && *a.gate != a.gate_value) return;  // foreign scenes: the other tracer renders this frame
    __shared__ uint32_t stack_lds[STACK * Tracer::WORDS * WAVE];
    uint32_t* const stk = stack_lds + threadIdx.x;
    const int g = (int)blockIdx.x;
    const int k = g >> 2;
    const int tid = ((g & 3) << 6) | (int)threadIdx.x;  // thread index within the 16x16 tile
    const int tile = shard_tile(a, k);
    int lx, ly;
    tile_pixel(tid, &lx, &ly);
    const int x = (tile % a.tiles_x) * TILE + lx;
    const int y = (tile / a.tiles_x) * TILE + ly;
    Counters c;
    if (tile >= 0 && x < a.width && y < a.height) {  // off-frame lanes stay for the wave reduction
        const size_t slot = (size_t)(k >= 0 ? k : 0) * (TILE * TILE) + tid;
        const size_t rng_index = a.out_shard ? slot : (size_t)y * a.width + x;
        shade_pixel<Tracer, STACK, STATS>(a, stk, x, y, rng_index, slot, c);
    }
    // Segment count (always on: the Mrays/s numerator), one atomic per wave.
    if (a.seg_counter) {
        unsigned long long v = c.seg;
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (threadIdx.x == 0) atomicAdd(a.seg_counter, v);
    }
    if (STATS) {
        atomicAdd(a.stats + RT_STAT_SEGMENTS, c.seg);
        atomicAdd(a.stats + RT_STAT_NODES, c.node);
        atomicAdd(a.stats + RT_STAT_TRI_TESTS, c.tri);
        atomicAdd(a.stats + RT_STAT_TRI_ACCEPTS, c.tacc);
        atomicAdd(a.stats + RT_STAT_SPHERE_ACCEPTS, c.sacc);
        atomicAdd(a.stats + RT_STAT_HITS, c.hit);
        atomicAdd(a.stats + RT_STAT_MISSES, c.miss);
    }
}

template <class Tracer, int STACK, bool STATS>
hipError_t launch(const RenderArgs& args, int waves, hipStream_t stream) {
    hipLaunchKernelGGL((render_kernel<Tracer, STACK, STATS>), dim3(waves), dim3(WAVE), 0, stream, args);
    return hipGetLastError();
}


template <class Tracer>
hipError_t launch_variant(const RenderArgs& args, int waves, int depth, bool stats, hipStream_t s) {
    // The DFS holds at most depth + 1 entries (one pending sibling per level).  Depth is known
    // when the scene came through rt_scene_upload; otherwise use the reference's 64
    // (main_raytracing.cu:35).
    if (depth >= 0 && depth + 2 <= 28)
        return stats ? launch<Tracer, 28, true>(args, waves, s) : launch<Tracer, 28, false>(args, waves, s);
    if (depth >= 0 && depth + 2 <= 40)
        return stats ? launch<Tracer, 40, true>(args, waves, s) : launch<Tracer, 40, false>(args, waves, s);
    return stats ? launch<Tracer, 64, true>(args, waves, s) : launch<Tracer, 64, false>(args, waves, s);
}

}  // namespace

hipError_t launch_ref_tracer(bool flat, const RenderArgs& a, int waves, int depth, bool stats, hipStream_t s) {
    return flat ? launch_variant<FlatTracer>(a, waves, depth, stats, s) : launch_variant<RefTracer>(a, waves, depth, stats, s);
}

}  // namespace rtk
