// rt_wavefront.hip -- the wavefront tracer (rt_render_params.flags RT_RENDER_TRACER_WAVEFRONT).
//
// The production kernel (rt_fast_body.h) keeps a pixel on a lane for the whole frame: a wave
// traces one segment of each of its 64 pixels, and every lane waits for the wave's longest
// traversal -- 27 % lane utilisation in the small phase, which is 62 % of the frame (DESIGN.md
// §4.1).  Here a frame is a sequence of generations, each a pair of launches:
//
//   shade(g)  one lane per pixel still rendering (the generation's active list): shade the hit of
//             segment g - 1 (shade_segment), end the path or the sample as the reference does,
//             start the next camera sample (u, v draws), write the finished pixel; for the next
//             segment: the sphere loop, the root test, and the ray appended to trace queue g;
//   trace(g)  one wave per region over the rays its shade wave queued: a lane whose traversal
//             ends writes its hit and takes the region's next ray, so the lanes stay busy until the
//             region's queue drains; big leaves run in rounds once enough lanes wait at one.
//
// Per pixel the order of operations is the production kernel's: the same draws in the same order
// (main_raytracing.cu:188-193, 118-148), and each segment's DFS is rt_fast.h's -- only the lane
// and the moment a ray is traced change, so frames and RNG states are bit-identical
// (tests/test_gpu_wavefront.py).  Between launches a pixel's state lives in HBM: 64 B of pixel
// state, 32 B of ray, 16 B of hit per pixel (WfBuf); at most spp x bounces + 1 generations.
#include "rt_fast_body.h"

namespace rtk {
namespace {

// Wave w of both launches owns region w of the lists (C entries): the pixels it started in
// generation 0 (chunks w, w + W, w + 2W, ... of 64 lane-order entries, so a region samples the
// whole frame; RT_TUNE bit 18: C / 64 consecutive chunks instead -- coherent rays, but the regions
// over the bunny's base take 2.3x the frame: 68 vs 29 ms) stay with it, and
// trace wave w traces the rays shade wave w queued -- no atomics, no cross-wave hand-off (one
// atomic counter per list measured 0.75 ms per generation).  Both launches deal wave w to XCD
// w % 8, so a region's state stays in one L2.
struct WfBuf {
    uint4* pst;       // [P][4]: (d, v0, v1, v2), (v3, v4, color.xy), (color.z, thr), (acc.rgb, meta)
    float4* ray;      // [P][2]: (ro.xyz, rd.x), (rd.yz, -, -)
    float4* hit;      // [P]: (best, kind << 30 | id, bx, by)
    uint32_t* alist;  // [2][W * C]: active entries per region, generations g and g + 1 (ping-pong)
    float4* tq;       // [W * C][3]: the generation's rays to trace, per region: (ro.xyz, rd.x),
                      // (rd.yz, sphere best, kind << 30 | id), (entry, -, -, -)
    uint32_t* acnt;   // [G + 2][W]: active entries of region w in generation g
    uint32_t* tcnt;   // [G + 1][W]: rays queued by region w in generation g
    long long P;      // lane-order entries (a.entry_count)
    int W;            // regions = waves of both launches
    int C;            // entries per region (multiple of 64)
};

constexpr uint32_t META_PATH = 1u << 24;

__device__ __forceinline__ float4 pack_hit(const rtfast::Hit& h) {
    return make_float4(h.best, __uint_as_float(((uint32_t)h.kind << 30) | h.id), h.bx, h.by);
}
__device__ __forceinline__ rtfast::Hit unpack_hit(float4 v) {
    rtfast::Hit h;
    const uint32_t k = __float_as_uint(v.y);
    h.best = v.x, h.kind = (int)(k >> 30), h.id = k & 0x3fffffffu, h.bx = v.z, h.by = v.w;
    return h;
}

// Entry i of the launch's lane order -> pixel (render_fast_body's bind_entry).
__device__ __forceinline__ bool wf_bind(const RenderArgs& a, long long i, int& x, int& y, size_t& slot,
                                        rt_rng_state*& rs) {
    const long long s = a.lane_slots ? (long long)a.lane_slots[i] : i;
    const bool ok = s >= 0 && s < a.slot_count;
    const int k = ok ? (int)(s >> 8) : -1, tid = (int)(s & 255);
    const int tile = k >= 0 ? shard_tile(a, k) : -1;
    int lx, ly;
    tile_pixel(tid, &lx, &ly);
    x = (tile % a.tiles_x) * TILE + lx;
    y = (tile / a.tiles_x) * TILE + ly;
    const bool pixel = tile >= 0 && x < a.width && y < a.height;
    slot = (size_t)(k >= 0 ? k : 0) * (TILE * TILE) + tid;
    rs = a.rng + (a.out_shard ? slot : (size_t)(pixel ? y : 0) * a.width + (pixel ? x : 0));
    return pixel;
}

// Rank of this lane among the lanes of `m` below it.
__device__ __forceinline__ uint32_t lane_rank(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__global__ __launch_bounds__(WAVE) void wf_shade_kernel(RenderArgs a, WfBuf b, int g) {
    const int w = blockIdx.x;
    const size_t region = (size_t)w * (size_t)b.C;
    // generation 0: chunks w, w + W, ... of the lane order; later: the region's active entries
    const long long n = g == 0 ? (long long)b.C : (long long)b.acnt[(size_t)g * b.W + w];
    if (n == 0) {
        if (threadIdx.x == 0) b.acnt[(size_t)(g + 1) * b.W + w] = 0u, b.tcnt[(size_t)g * b.W + w] = 0u;
        return;
    }
    const uint32_t* list = b.alist + (size_t)(g & 1) * (size_t)b.W * b.C + region;
    uint32_t* next = b.alist + (size_t)((g + 1) & 1) * (size_t)b.W * b.C + region;
    float4* tq = b.tq + 3 * region;
    const bool strided = (a.tune & (1u << 18)) == 0;
    const float4* nodes4 = reinterpret_cast<const float4*>(a.nodes);
    const rtm::f3 cam_o = ld3(a.cam.origin), cam_h = ld3(a.cam.horizontal), cam_v = ld3(a.cam.vertical),
                  cam_ll = ld3(a.cam.lower_left_corner);
    Counters c;
    unsigned long long segs = 0;
    uint32_t na = 0, nt = 0;  // entries appended to the region's next active list / trace queue
    for (long long base = 0; base < n; base += WAVE) {
        const long long j = base + threadIdx.x;
        long long i = 0;
        if (g == 0) i = (strided ? (long long)w + (base / WAVE) * b.W : (long long)w * (b.C / WAVE) + base / WAVE) * WAVE + threadIdx.x;
        const bool valid = g == 0 ? i < b.P : j < n;
        const uint32_t e = valid ? (g == 0 ? (uint32_t)i : list[j]) : 0u;
        int x = 0, y = 0;
        size_t slot = 0;
        rt_rng_state* rs = a.rng;
        const bool pixel = valid && wf_bind(a, e, x, y, slot, rs);
        rtm::Xorwow rng{0, 0, 0, 0, 0, 0};
        rtm::f3 color = rtm::mk(0, 0, 0), thr = rtm::mk(1, 1, 1), acc = rtm::mk(0, 0, 0), ro = cam_o, rd = cam_o;
        int sample = 0, bounce = 0;
        bool path = false;
        if (pixel) {
            if (g == 0) {
                rng = rtm::Xorwow{rs->d, rs->v[0], rs->v[1], rs->v[2], rs->v[3], rs->v[4]};
            } else {
                const uint4 q0 = b.pst[4 * (size_t)e], q1 = b.pst[4 * (size_t)e + 1], q2 = b.pst[4 * (size_t)e + 2],
                            q3 = b.pst[4 * (size_t)e + 3];
                rng = rtm::Xorwow{q0.x, q0.y, q0.z, q0.w, q1.x, q1.y};
                color = rtm::mk(__uint_as_float(q1.z), __uint_as_float(q1.w), __uint_as_float(q2.x));
                thr = rtm::mk(__uint_as_float(q2.y), __uint_as_float(q2.z), __uint_as_float(q2.w));
                acc = rtm::mk(__uint_as_float(q3.x), __uint_as_float(q3.y), __uint_as_float(q3.z));
                sample = (int)(q3.w & 0xffffu), bounce = (int)((q3.w >> 16) & 0xffu), path = (q3.w & META_PATH) != 0;
            }
        }
        if (pixel && path) {
            // ray_color's tail for segment g - 1 (main_raytracing.cu:118-158), as render_fast_body
            const float4 r0 = b.ray[2 * (size_t)e], r1 = b.ray[2 * (size_t)e + 1];
            ro = rtm::mk(r0.x, r0.y, r0.z), rd = rtm::mk(r0.w, r1.x, r1.y);
            const rtfast::Hit h = unpack_hit(b.hit[e]);
            const rtm::f3 nd = rtm::normalize(rd);
            bool end = shade_segment<false>(a, h, ro, rd, nd, rng, color, thr, c);
            if (++bounce >= a.bounces) end = true;
            if (end) {
                acc = rtm::add(acc, color);
                sample++;
                path = false;
            }
        }
        bool done = false;
        if (pixel && !path) {
            for (;;) {
                if (sample < a.spp) {
                    // main_raytracing.cu:190: uv = (pixel + vec2(rng(), rng())) / vec2(W, H), u first
                    const float ru = rng.uniform();
                    const float rv = rng.uniform();
                    const float uvx = ((float)x + ru) / (float)a.width;
                    const float uvy = ((float)y + rv) / (float)a.height;
                    ro = cam_o;
                    rd = rtm::sub(rtm::add(rtm::add(cam_ll, rtm::muls(cam_h, uvx)), rtm::muls(cam_v, uvy)), cam_o);
                    color = rtm::mk(0, 0, 0);
                    thr = rtm::mk(1, 1, 1);
                    bounce = 0;
                    path = true;
                    if (a.bounces == 0) {  // an empty bounce loop: the sample contributes (0,0,0,1)
                        sample++;
                        path = false;
                        continue;
                    }
                    break;
                }
                done = true;
                break;
            }
        }
        if (done) {
            // main_raytracing.cu:195-199 (the production kernel's output, alpha = samples / spp)
            const float fs = (float)a.spp;
            const rtm::f4 res{acc.x / fs, acc.y / fs, acc.z / fs, (float)sample / fs};
            const float lerp = a.frame_index > 0 ? 1.0f / (float)(a.frame_index + 1) : 1.0f;
            float4 prev;
            float4* out;
            if (a.out_shard) {
                prev = a.last ? reinterpret_cast<const float4*>(a.last)[slot] : make_float4(0, 0, 0, 0);
                out = a.out_shard + slot;
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
        // the next segment: GetRayHit's sphere loop and the BVH root test (main_raytracing.cu:83-109)
        bool need = false;
        float4 qh = make_float4(0, 0, 0, 0);
        const bool go = pixel && path;
        if (go) {
            segs++;
            rtfast::Hit h;
            h.best = 1e30f, h.kind = 0, h.id = 0, h.bx = h.by = 0.0f;
            const rtm::f3 nd = rtm::normalize(rd);
            for (int k = 0; k < a.sphere_count; k++) {
                const GeometrySphere& sp = a.spheres[k];
                float dist;
                if (rtd::intersect_sphere(ro, nd, ld3(sp.position), sp.radius * sp.radius, &dist)) {
                    if (dist >= h.best) continue;
                    h.best = dist;
                    h.kind = 1;
                    h.id = (uint32_t)k;
                }
            }
            const rtfast::Ray R = rtfast::make_ray(ro, rd, nd, a.scene_fast != 0);
            rtfast::Trav T{0, 0, 0};
            need = rtfast::trav_begin<false>(nodes4, R, h, T, c);
            b.ray[2 * (size_t)e] = make_float4(ro.x, ro.y, ro.z, rd.x);
            b.ray[2 * (size_t)e + 1] = make_float4(rd.y, rd.z, 0.0f, 0.0f);
            qh = pack_hit(h);
            if (!need) b.hit[e] = qh;  // no BVH traversal: the sphere loop's hit is the segment's
            b.pst[4 * (size_t)e] = make_uint4(rng.d, rng.v0, rng.v1, rng.v2);
            b.pst[4 * (size_t)e + 1] = make_uint4(rng.v3, rng.v4, __float_as_uint(color.x), __float_as_uint(color.y));
            b.pst[4 * (size_t)e + 2] = make_uint4(__float_as_uint(color.z), __float_as_uint(thr.x), __float_as_uint(thr.y),
                                                  __float_as_uint(thr.z));
            b.pst[4 * (size_t)e + 3] = make_uint4(__float_as_uint(acc.x), __float_as_uint(acc.y), __float_as_uint(acc.z),
                                                  (uint32_t)sample | ((uint32_t)bounce << 16) | META_PATH);
        }
        const unsigned long long ma = __ballot(go), mt = __ballot(need);
        if (go) next[na + lane_rank(ma)] = e;
        if (need) {
            float4* q = tq + 3 * (size_t)(nt + lane_rank(mt));
            q[0] = make_float4(ro.x, ro.y, ro.z, rd.x);
            q[1] = make_float4(rd.y, rd.z, qh.x, qh.y);
            q[2] = make_float4(__uint_as_float(e), 0.0f, 0.0f, 0.0f);
        }
        na += (uint32_t)__popcll(ma), nt += (uint32_t)__popcll(mt);
    }
    if (threadIdx.x == 0) b.acnt[(size_t)(g + 1) * b.W + w] = na, b.tcnt[(size_t)g * b.W + w] = nt;
    if (a.seg_counter) {
        for (int off = 32; off > 0; off >>= 1) segs += __shfl_xor(segs, off);
        if ((threadIdx.x & 63) == 0 && segs) atomicAdd(a.seg_counter, segs);
    }
}

// RT_TUNE bits 20-22 (x4): refill when at least this many lanes are free (default 4); bits 23-25
// (x8): lanes waiting at big leaves that start a big round while others are still in small steps
// (default 32).  Swept on config 2: refill at 1 / 4 / 8 / 16 / 32 / 63 free lanes 32.9 / 29.9 /
// 30.3 / 30.4 / 31.8 / 33.8 ms, big rounds at 16 / 32 / 48 / 62 waiting 32.2 / 30.1 / 30.4 / 32.5.
template <int STACK, int MODE>
__device__ __forceinline__ void wf_trace_body(const RenderArgs& a, const WfBuf& b, int g) {
    const uint32_t n = b.tcnt[(size_t)g * b.W + blockIdx.x];
    if (n == 0) return;
    const float4* tq = b.tq + 3 * (size_t)blockIdx.x * b.C;
    uint32_t cursor = 0;  // rays of the region handed out so far
    // every queued ray passed the root test in its shade launch: it starts at the root's children
    const rtfast::f4v root_hi = ((rtfast::ConstF4)a.nodes)[1];
    const uint32_t root_first = __float_as_uint(root_hi.z), root_count = __float_as_uint(root_hi.w);
    constexpr int SL = STACK < 16 ? STACK : 16;
    __shared__ uint32_t stack_lds[(SL + rtfast::STACK_PAD_ROWS) * WAVE];
    __shared__ uint32_t scratch_lds[(MODE & 4) ? 64 : 1];
    uint32_t ovf[STACK > SL ? STACK - SL : 1];
    const rtfast::Stack<SL> stk{stack_lds, ovf};
    const float4* nodes4 = reinterpret_cast<const float4*>(a.nodes);
    const float4* tris = reinterpret_cast<const float4*>(a.tris);
    const uint32_t tv = (a.tune >> 20) & 7u, refill_min = tv ? 4u * tv : 4u;
    const uint32_t bw = (a.tune >> 23) & 7u, big_wait = bw ? 8u * bw : 32u;
    const uint32_t lane = threadIdx.x & 63u;
    Counters c;
    rtfast::Ray R;
    R.o = R.d = R.nd = R.r = rtm::mk(0, 0, 0);
    R.fast = false;
    rtfast::Hit h;
    h.best = 1e30f, h.kind = 0, h.id = 0, h.bx = h.by = 0.0f;
    rtfast::Trav T{0, 0, 0};
    uint32_t e = 0;
    bool has = false, active = false, exhausted = false;
    for (;;) {
        // a lane whose traversal is over hands its hit to the next shade
        if (has && !active) {
            b.hit[e] = pack_hit(h);
            has = false;
        }
        if (!exhausted) {
            const unsigned long long fm = __ballot(!has);
            const uint32_t nf = (uint32_t)__popcll(fm);
            if (nf >= refill_min || (nf && !__ballot(has))) {
                const uint32_t base = cursor;
                cursor += nf;
                if (!has) {
                    const uint32_t idx = base + lane_rank(fm);
                    if (idx < n) {
                        const float4 q0 = tq[3 * (size_t)idx], q1 = tq[3 * (size_t)idx + 1], q2 = tq[3 * (size_t)idx + 2];
                        e = __float_as_uint(q2.x);
                        const rtm::f3 ro = rtm::mk(q0.x, q0.y, q0.z), rd = rtm::mk(q0.w, q1.x, q1.y);
                        R = rtfast::make_ray(ro, rd, rtm::normalize(rd), a.scene_fast != 0);
                        h = unpack_hit(make_float4(q1.z, q1.w, 0.0f, 0.0f));
                        T.first = root_first, T.count = root_count, T.sp = rtfast::Stack<SL>::empty((int)(threadIdx.x & 63u));
                        active = true;
                        has = true;
                    }
                }
                if (cursor >= n) exhausted = true;
            }
        }
        if (!__ballot(has)) {
            if (exhausted) break;
            continue;
        }
        // one traversal iteration (rt_fast.h trace, split small steps), big rounds once big_wait
        // lanes wait at big leaves or no lane is left in the small phase
        const bool inner = active && T.count == 0;
        const bool leafs = active && T.count > 0 && T.count <= (uint32_t)rtfast::BIG;
        const bool waiting = active && T.count > (uint32_t)rtfast::BIG;
        const unsigned long long mI = __ballot(inner), mL = __ballot(leafs), mW = __ballot(waiting);
        if ((mI | mL) && (uint32_t)__popcll(mW) < big_wait) {
            const uint32_t nI = (uint32_t)__popcll(mI), nL = (uint32_t)__popcll(mL);
            if (exhausted && nI + nL == 1 && (a.tune & (1u << 26)) == 0) {
                const int r = __ffsll((long long)(mI | mL)) - 1;
                if (rtfast::Stack<SL>::depth(__builtin_amdgcn_readlane(T.sp, r)) <= rtfast::Stack<SL>::LDS_ENTRIES) {
                    rtfast::lone_traverse(nodes4, tris, stk, r, R, h, T, active);
                    continue;
                }
            }
            const uint32_t qv = (a.tune >> 13) & 7u, q = qv ? qv - 1u : 1u;
            if (a.tune & 4096u) {  // RT_TUNE bit 12: inner-node and small-leaf steps in one iteration
                if (inner || leafs) active = rtfast::small_step<false>(nodes4, tris, a.spairs, stk, R, h, T, c);
            } else if (!mI || nL * 4u >= nI * (q + 1u)) {
                if (leafs) active = rtfast::small_step<false>(nodes4, tris, a.spairs, stk, R, h, T, c);
            } else if (inner) {
                active = rtfast::small_step<false>(nodes4, tris, a.spairs, stk, R, h, T, c);
            }
            continue;
        }
        if (!mW) continue;
        if (rtfast::big_round<false, MODE>(tris, a.pairs, a.quads, a.units, a.tree, a.ltris, a.flat, scratch_lds, a.tune, mW, waiting, R, h,
                                           T, c))
            active = rtfast::pop(nodes4, stk, T.sp, R, h.best, T.first, T.count);
    }
}

template <int STACK, int MODE>
__global__ __launch_bounds__(WAVE) void wf_trace_kernel(RenderArgs a, WfBuf b, int g) {
    wf_trace_body<STACK, MODE>(a, b, g);
}

// Per-(device, stream) buffers, grown to the largest lane order rendered so far: frames queued on
// different streams of one device each have their own pixel state and queues (a frame reuses its
// stream's block only after the previous frame on that stream, by stream order).
struct WfCache {
    WfBuf b{};
    size_t bytes = 0;
};

hipError_t wf_buffers(long long P, int W, int gens, hipStream_t s, WfBuf* out) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, WfCache> per_stream;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const int C = (int)(((P + WAVE - 1) / WAVE + W - 1) / W) * WAVE;
    const size_t L = (size_t)W * C;
    const size_t need = (size_t)P * 112 + L * 56 + (size_t)(2 * gens + 3) * W * 4;
    std::lock_guard<std::mutex> lock(mu);
    WfCache& wc = per_stream[std::make_pair(dev, s)];
    if (wc.bytes < need) {
        if (wc.b.pst) (void)hipFree(wc.b.pst);
        wc = WfCache{};
        char* p = nullptr;
        if ((e = hipMalloc(&p, need)) != hipSuccess) return e;
        wc.b.pst = (uint4*)p;
        wc.bytes = need;
    }
    char* p = (char*)wc.b.pst;
    WfBuf& b = *out;
    b.pst = (uint4*)p, p += (size_t)P * 64;
    b.ray = (float4*)p, p += (size_t)P * 32;
    b.hit = (float4*)p, p += (size_t)P * 16;
    b.alist = (uint32_t*)p, p += L * 8;
    b.tq = (float4*)p, p += L * 48;
    b.acnt = (uint32_t*)p, p += (size_t)(gens + 2) * W * 4;
    b.tcnt = (uint32_t*)p;
    b.P = P, b.W = W, b.C = C;
    return hipSuccess;
}

template <int STACK>
hipError_t wf_launch_trace(const RenderArgs& a, const WfBuf& b, int g, hipStream_t s) {
    if (a.tree) hipLaunchKernelGGL((wf_trace_kernel<STACK, 21>), dim3(b.W), dim3(WAVE), 0, s, a, b, g);
    else hipLaunchKernelGGL((wf_trace_kernel<STACK, 17>), dim3(b.W), dim3(WAVE), 0, s, a, b, g);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_wavefront(const RenderArgs& a, int depth, hipStream_t s) {
    const long long P = a.entry_count;
    if (P <= 0 || P > (1ll << 31)) return hipErrorInvalidValue;
    const int gens = a.spp * a.bounces;  // segments per pixel at most: spp x bounces
    const int stack = (depth >= 0 && depth + 2 <= 30) ? 30 : (depth >= 0 && depth + 2 <= 40) ? 40 : 64;
    // regions = the trace launch's resident waves, so every region's trace wave runs at once
    int W = stack == 30 ? resident_waves(a.tree ? wf_trace_kernel<30, 21> : wf_trace_kernel<30, 17>)
                  : stack == 40 ? resident_waves(a.tree ? wf_trace_kernel<40, 21> : wf_trace_kernel<40, 17>)
                                : resident_waves(a.tree ? wf_trace_kernel<64, 21> : wf_trace_kernel<64, 17>);
    if (W <= 0) return hipErrorInvalidValue;
    // RT_TUNE bits 16-17: regions = 2^v x the resident waves (the dispatcher then balances the
    // regions over the waves as they finish; measured 29.4 / 29.9 / 31.6 / 32.4 ms for v = 0-3)
    W <<= (a.tune >> 16) & 3u;
    WfBuf b;
    hipError_t e = wf_buffers(P, W, gens, s, &b);
    if (e != hipSuccess) return e;
    for (int g = 0; g <= gens; g++) {
        hipLaunchKernelGGL(wf_shade_kernel, dim3(b.W), dim3(WAVE), 0, s, a, b, g);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (g == gens) break;
        e = stack == 30 ? wf_launch_trace<30>(a, b, g, s) : stack == 40 ? wf_launch_trace<40>(a, b, g, s) : wf_launch_trace<64>(a, b, g, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace rtk
