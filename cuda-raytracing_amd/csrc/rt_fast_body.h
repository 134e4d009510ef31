// rt_fast_body.h -- the production render kernel (rt_fast.h traversal + the per-lane segment loop)
// and its launch helpers, included by the kernel translation units rt_fast_*.hip.  Each of those
// instantiates one family of variants (production, timing, statistics, A/B, refill), so the
// families compile in parallel; rt_kernel.hip picks the family and mode (rt_render.h).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <utility>

#include "rt_abi.h"
#include "rt_device.h"
#include "rt_math.h"
#include "rt_common.h"
#include "leaftree.h"
#include "rt_fast.h"
#include "rt_render.h"

namespace rtk {

// ray_color's per-segment tail (main_raytracing.cu:118-158) for the segment whose closest hit is
// `h`: emission, throughput, the next direction from 4 draws, Russian roulette; or the sky on a
// miss.  Updates the path (ro, rd, color, thr); returns true when the path ends here.
template <bool STATS>
__device__ __forceinline__ bool shade_segment(const RenderArgs& a, const rtfast::Hit& h, rtm::f3& ro, rtm::f3& rd,
                                              const rtm::f3 nd, rtm::Xorwow& rng, rtm::f3& color, rtm::f3& thr,
                                              Counters& c) {
    bool end = false;
    // GetRayHit returns `result.distance < max_distance` (main_raytracing.cu:108): a hit whose
    // accepted distance is NaN counts as a miss, as in the reference
    if (h.kind != 0 && h.best < 1e30f) {
        if (STATS) c.hit++;
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
        if (rng.uniform() > p) {
            end = true;
        } else {
            thr = rtm::muls(thr, 1.0f / p);
        }
    } else {
        if (STATS) c.miss++;
        if (a.sky) {
            const rtm::f3 dir = rtd::quat_rotate(a.qw, a.qx, a.qy, a.qz, rd);
            const rtm::f3 cs = rtd::cube_sample(a.sky, a.sky_n, dir);
            const rtm::f3 cl = rtm::mk(rtm::gmin(rtm::gmax(cs.x, 0.0f), 50.0f), rtm::gmin(rtm::gmax(cs.y, 0.0f), 50.0f),
                                       rtm::gmin(rtm::gmax(cs.z, 0.0f), 50.0f));
            color = rtm::add(color, rtm::mul(thr, cl));
        }
        end = true;
    }
    return end;
}

// Logical sub-tile of this workgroup.  The dispatcher deals workgroups round-robin over the 8
// XCDs (workgroup g -> XCD g % 8), so consecutive sub-tiles would land in different L2s.
// Instead XCD x takes runs of S = 2^v consecutive sub-tiles: its i-th workgroup renders
// sub-tile ((i / S) * 8 + x) * S + i % S (a permutation of the first multiple of 8S workgroups;
// the rest keep their index), so neighbouring pixels share an L2.  v = 5 (runs of 8 tiles,
// 128x16 px) in plain tile order: config 2 18.29 -> 17.73 ms; v = 4 17.8, v = 6 18.1, v = 1-3 18.1-18.3.
// Round 6, on the final kernel with the cost-ordered lane map (whose consecutive waves are no longer
// neighbours): v = 3 (runs of 8 sub-tiles) config 2 13.23-13.26 vs 13.41-13.49 ms, config 4 79.7-79.9 vs
// 80.4-80.6 ms; v = 2 / 4 / the dispatcher's order in between (profiles/r06_ab_log.txt item 8).
// RT_TUNE bits 16-19 override v; 15 keeps the dispatcher's order.
__device__ __forceinline__ int xcd_block(uint32_t tune) {
    const uint32_t g = blockIdx.x, tv = (tune >> 16) & 15u, v = tv ? tv : 3u;
    if (v == 15u) return (int)g;
    const uint32_t S = 1u << v, full = gridDim.x / (8u * S) * (8u * S);
    if (g >= full) return (int)g;
    const uint32_t i = g >> 3, x = g & 7u;
    return (int)((((i / S) << 3) + x) * S + i % S);
}

// The production kernel: rt_fast.h traversal + a flat per-lane segment loop.
// raytracing_kernel_main / ray_color (main_raytracing.cu:111-200) nest `for sample { for
// bounce { ... break } }`; on a SIMD machine that makes every lane wait at the end of each
// sample for the longest path of the wave.  Here each lane runs a small state machine --
// start a camera sample, trace a segment, shade, end the path on a miss / Russian roulette /
// the bounce limit, start its next sample -- so a lane only idles once its whole pixel is
// done.  The per-pixel draw order (u, v, then 4 draws per hit) is the reference's.
#ifndef RT_LDS_SL
#define RT_LDS_SL 16  // stack entries in LDS (4 KB per wave)
#endif
#if defined(RT_PAIR)  // experiment (rt_fast.h wave pairs): two waves per workgroup, tails handed over
constexpr int WG_WAVES = 2;
#else
constexpr int WG_WAVES = 1;
#endif
constexpr int WGL = WG_WAVES * WAVE;  // lanes per workgroup (the LDS stack's column count)

template <int STACK, bool STATS, int MODE>
__device__ __forceinline__ void render_fast_body(const RenderArgs& a,
                                                 const rtfast::Stack<(STACK < RT_LDS_SL ? STACK : RT_LDS_SL), WGL>& stk,
                                                 uint32_t* const scratch, uint32_t* const mail = nullptr) {
    if (a.gate && *a.gate != a.gate_value) return;  // foreign scenes: the other tracer renders this frame
    const float4* nodes4 = reinterpret_cast<const float4*>(a.nodes);
    const float4* tris = reinterpret_cast<const float4*>(a.tris);
    // this lane's pixel: slot k*256 + tid of the launch's list (k < 0: none)
    int x = 0, y = 0;
    bool pixel = false;
    // Path state is kept small: it is live across every trace call, where the 7-wave build spills it
    // (32-bit slot, no RNG pointer: rng_slot() recomputes it; the alpha sum is the sample count)
    uint32_t slot = 0;  // < 2^32 (rt_render checks slot_count)
    rtm::Xorwow rng{0, 0, 0, 0, 0, 0};
    auto rng_slot = [&]() { return a.rng + (a.out_shard ? (size_t)slot : (size_t)y * a.width + x); };
    auto bind = [&](int k, int tid) {
        const int tile = k >= 0 ? shard_tile(a, k) : -1;
        int lx, ly;
        tile_pixel(tid, &lx, &ly);
        x = (tile % a.tiles_x) * TILE + lx;
        y = (tile / a.tiles_x) * TILE + ly;
        pixel = tile >= 0 && x < a.width && y < a.height;
        slot = (uint32_t)(k >= 0 ? k : 0) * (TILE * TILE) + (uint32_t)tid;
        if (pixel) {
            const rt_rng_state* rs = rng_slot();
            rng = rtm::Xorwow{rs->d, rs->v[0], rs->v[1], rs->v[2], rs->v[3], rs->v[4]};
        }
    };
    // entry i of the launch's lane order: the lane map, or slot i (wave i / 64 = 8x8 sub-tile)
    auto bind_entry = [&](long long i) {
        const long long s = (WG_WAVES > 1 && i >= a.entry_count) ? -1 : a.lane_slots ? (long long)a.lane_slots[i] : i;
        const bool ok = s >= 0 && s < a.slot_count;  // a bad map entry renders nothing
        bind(ok ? (int)(s >> 8) : -1, (int)(s & 255));
    };
    // one 64-lane workgroup per 8x8 sub-tile: tile k = lb / 4, sub-tile lb % 4
    // (wave pairs: the two waves of workgroup g take sub-tiles 2g, 2g + 1)
    const int lane = (int)(threadIdx.x & 63u);
    const int lb = xcd_block(a.tune) * WG_WAVES + (WG_WAVES > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0);
    bind_entry((long long)lb * WAVE + lane);
    if (a.lane_slots && lb < a.priority_waves) __builtin_amdgcn_s_setprio(3);  // the frame's long waves
    // Refill (rt_render_params.refill_lanes): the grid holds only as many waves as fit the GPU at
    // once; entries [grid x 64, entries) form a queue, and a wave whose idle lanes reach
    // refill_lanes takes that many entries with one atomic (ballot + mbcnt rank the idle lanes), so
    // lanes stay busy until the queue drains instead of idling once their own pixel is done.
    // Waves that start less than half full (split waves of a lane plan) are not refilled.
    constexpr bool REFILL = (MODE & 64) != 0;  // refill is compiled into its own kernel variants only
    bool drained = !REFILL || a.queue_head == nullptr || __popcll(__ballot(pixel)) < 32;
    const long long qbase = (long long)gridDim.x * WGL;
    Counters c;
    const rtm::f3 cam_o = ld3(a.cam.origin), cam_h = ld3(a.cam.horizontal), cam_v = ld3(a.cam.vertical),
                  cam_ll = ld3(a.cam.lower_left_corner);
    float acc_r = 0.0f, acc_g = 0.0f, acc_b = 0.0f;
    int sample = 0, bounce = 0;
    bool path = false;
    rtm::f3 ro = cam_o, rd = cam_o, color = rtm::mk(0, 0, 0), thr = rtm::mk(1, 1, 1);
    const bool scene_fast = a.scene_fast != 0;
    const unsigned long long t_start = (MODE & 8) ? __builtin_amdgcn_s_memtime() : 0;
    // wave_clock and the per-wave (start, end) diagnostics use the device's constant 100 MHz clock
    // (s_memrealtime): one time base for every wave, also for a wave saved and restored by another
    // process sharing the GPU (the shader-cycle counter s_memtime is not)
    const unsigned long long rt_start = (a.wave_clock || ((MODE & 8) && (a.tune & 2048u))) ? __builtin_amdgcn_s_memrealtime() : 0;

#ifdef RT_LIVE_HIST
    unsigned long long lh_t = 0;
    uint32_t lh_n = 0;
#endif
    for (;;) {
        if (!drained) {
            const unsigned long long idle = __ballot(!pixel && !path);
            const uint32_t ni = (uint32_t)__popcll(idle);
            if (ni && (ni >= (uint32_t)a.refill_lanes || !__ballot(path))) {
                const int lead = __ffsll((long long)idle) - 1;
                unsigned long long base = 0;
                if (lane == lead) base = atomicAdd(a.queue_head, (unsigned long long)ni);
                base = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(base >> 32), lead) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)base, lead);
                const long long qn = a.entry_count - qbase;
                if (!pixel && !path) {
                    const unsigned long long i =
                        base + __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                    if ((long long)i < qn) {
                        bind_entry(qbase + (long long)i);
                        acc_r = acc_g = acc_b = 0.0f;
                        sample = 0;
                    }
                }
                if ((long long)(base + ni) >= qn) drained = true;
            }
        }
        if (pixel && !path) {
            if (sample < a.spp) {
                // main_raytracing.cu:190: uv = (pixel + vec2(rng(), rng())) / vec2(W, H), u first
                const float ru = rng.uniform();
                const float rv = rng.uniform();
                const float uvx = ((float)x + ru) / (float)a.width;
                const float uvy = ((float)y + rv) / (float)a.height;
                ro = cam_o;  // GPUCamera::GetRay (GPUScene.h:13), not normalized
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
            } else {
                pixel = false;
                // main_raytracing.cu:195-199
                const float fs = (float)a.spp;
                // the reference's alpha sum adds 1.0f per sample: (float)sample exactly, and stuck at 2^24
                // from there on (2^24 + 1 rounds back to 2^24 in fp32)
                const rtm::f4 res{acc_r / fs, acc_g / fs, acc_b / fs, (float)min(sample, 1 << 24) / fs};
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
                rt_rng_state* rs = rng_slot();
                rs->d = rng.d;
                rs->v[0] = rng.v0;
                rs->v[1] = rng.v1;
                rs->v[2] = rng.v2;
                rs->v[3] = rng.v3;
                rs->v[4] = rng.v4;
                // per-pixel work for rt_lane_plan: traversal steps + 3 per big leaf + 1 per segment
                if ((MODE & 8) && a.lane_cost) a.lane_cost[slot] = c.lane_work + (uint32_t)c.seg;
            }
        }
#ifdef RT_LIVE_HIST  // diagnostic build (tools/lane_hist.sh LIVE=1): segment-loop wave cycles by live pixels
        if (MODE & 8) {
            const unsigned long long tn = __builtin_amdgcn_s_memtime();
            if (lh_t) {
                const unsigned long long dt = tn - lh_t;
                c.ktest += lh_n <= 8u ? dt : 0ull;                    // 1-8 live pixels
                c.ktri += (lh_n > 8u && lh_n <= 16u) ? dt : 0ull;     // 9-16
                c.cy_tcl += (lh_n > 16u && lh_n <= 32u) ? dt : 0ull;  // 17-32
                c.cy_ttri += dt;                                      // every segment-loop iteration
            }
            lh_t = tn;
            lh_n = (uint32_t)__popcll(__ballot(pixel || path));
        }
#endif
        if (!__ballot(path)) {
            if (drained) break;
            continue;  // every lane idle: refill at the top
        }
        if (MODE & 8) c.w_iter++;
        if (STATS) {
            c.w_seg += (threadIdx.x & 63) == 0;
            c.l_seg += path;
        }

        // GetRayHit (main_raytracing.cu:83-109)
        rtfast::Hit h;
        h.best = 1e30f, h.kind = 0, h.id = 0, h.bx = h.by = 0.0f;
        const rtm::f3 nd = rtm::normalize(rd);
        if (path) {
            c.seg++;
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
        rtfast::Ray R = rtfast::make_ray(ro, rd, nd, scene_fast);
        rtfast::trace<STATS, MODE>(nodes4, tris, a.pairs, a.tree, a.ltris, a.flat, a.spairs, a.tune, stk, scratch, R, h,
                                   path, c, a.quads, a.units, a.face_leaf, mail);
        if (!path) continue;

        bool end = shade_segment<STATS>(a, h, ro, rd, nd, rng, color, thr, c);
        if (++bounce >= a.bounces) end = true;
        if (end) {
            acc_r += color.x;
            acc_g += color.y;
            acc_b += color.z;
            sample++;
            path = false;
        }
    }

    if (a.seg_counter) {
        unsigned long long v = c.seg;
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if ((threadIdx.x & 63) == 0) atomicAdd(a.seg_counter, v);
    }
    // per-wave cost for cost-aware shard plans (rt_render_params.wave_clock; one store per wave)
    if (a.wave_clock && lane == 0) a.wave_clock[lb] = __builtin_amdgcn_s_memrealtime() - rt_start;
    unsigned long long lane_max = c.l_small;  // the busiest lane's small steps (timing frame)
    if (MODE & 8)
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(lane_max, off);
            lane_max = o > lane_max ? o : lane_max;
        }
    unsigned long long lane_sum = c.l_small;  // the wave's lane-steps in small-step iterations (timing frame)
    unsigned long long big_sum[5] = {c.big_tests, c.tw_dec, c.tw_test, c.end2, c.redo};  // per lane -> the wave's
    if ((MODE & 8) && a.stats)
        for (int off = 32; off > 0; off >>= 1) {
            lane_sum += __shfl_xor(lane_sum, off);
            for (int k = 0; k < 5; k++) big_sum[k] += __shfl_xor(big_sum[k], off);
        }
    if ((MODE & 8) && a.stats && lane == 0) {  // timing frame: per-wave phase clocks
        atomicAdd(a.stats + RT_STAT_CYCLES_SMALL, c.cy_small);
        atomicAdd(a.stats + RT_STAT_CYCLES_BIG, c.cy_big);
        atomicAdd(a.stats + RT_STAT_CYCLES_TOTAL, __builtin_amdgcn_s_memtime() - t_start);
        atomicAdd(a.stats + RT_STAT_ROUNDS_COOP, c.r_coop);
        atomicAdd(a.stats + RT_STAT_ROUNDS_SHARED, c.r_shared);
        atomicAdd(a.stats + RT_STAT_COOP_RAYS, c.coop_rays);
        atomicAdd(a.stats + RT_STAT_WAVE_SMALL_ITERS, c.w_small);  // small-step wave iterations
        atomicAdd(a.stats + RT_STAT_LANE_SMALL, lane_sum);          // lane-steps in them
        atomicAdd(a.stats + RT_STAT_BIG_TESTS, big_sum[0]);
        atomicAdd(a.stats + RT_STAT_TWIN_DECIDED, big_sum[1]);
        atomicAdd(a.stats + RT_STAT_TWIN_TESTS, big_sum[2]);
        atomicAdd(a.stats + RT_STAT_WAVE_BIG_ITERS, c.big_iters);
        atomicAdd(a.stats + RT_STAT_DEFER_END2, big_sum[3]);
        atomicAdd(a.stats + RT_STAT_DEFER_REDO, big_sum[4]);
        // cooperative leaf-tree walk (wave-level): rays, subtree + cluster tests, triangle rounds
        atomicAdd(a.stats + RT_STAT_TREE_NODES, c.ktest);
        atomicAdd(a.stats + RT_STAT_TREE_TRI_TESTS, c.ktri);
        atomicAdd(a.stats + RT_STAT_WAVE_BIG_TRIS, c.w_big);
        atomicAdd(a.stats + RT_STAT_LANE_BIG_TRIS, c.l_big);
        atomicAdd(a.stats + RT_STAT_CYCLES_TREE_CLUSTERS, c.cy_tcl);
        atomicAdd(a.stats + RT_STAT_CYCLES_TREE_CUT, c.cy_tree);
        atomicAdd(a.stats + RT_STAT_CYCLES_TREE_TRIS, c.cy_ttri);
        // RT_TUNE bit 11: per-wave clocks (start, end) after the counters, for load-balance analysis
        if (a.tune & 2048u) {
            unsigned long long* w = a.stats + RT_STAT_COUNT + 8 * (size_t)lb;
            w[0] = rt_start;  // 100 MHz device clock (one time base across waves)
            w[1] = __builtin_amdgcn_s_memrealtime();
            w[2] = c.cy_small;
            w[3] = c.cy_big;
            w[4] = c.r_coop + c.r_shared;
            w[5] = c.w_iter;
            w[6] = c.w_small;
            w[7] = lane_max;
        }
    }
    if (STATS) {
        atomicAdd(a.stats + RT_STAT_SEGMENTS, c.seg);
        atomicAdd(a.stats + RT_STAT_NODES, c.node);
        atomicAdd(a.stats + RT_STAT_TRI_TESTS, c.tri);
        atomicAdd(a.stats + RT_STAT_TRI_ACCEPTS, c.tacc);
        atomicAdd(a.stats + RT_STAT_SPHERE_ACCEPTS, c.sacc);
        atomicAdd(a.stats + RT_STAT_HITS, c.hit);
        atomicAdd(a.stats + RT_STAT_MISSES, c.miss);
        atomicAdd(a.stats + RT_STAT_WAVE_SMALL_ITERS, c.w_small);
        atomicAdd(a.stats + RT_STAT_LANE_SMALL, c.l_small);
        atomicAdd(a.stats + RT_STAT_WAVE_BIG_TRIS, c.w_big);
        atomicAdd(a.stats + RT_STAT_LANE_BIG_TRIS, c.l_big);
        atomicAdd(a.stats + RT_STAT_CYCLES_TREE_CLUSTERS, c.cy_tcl);
        atomicAdd(a.stats + RT_STAT_CYCLES_TREE_CUT, c.cy_tree);
        atomicAdd(a.stats + RT_STAT_CYCLES_TREE_TRIS, c.cy_ttri);
        atomicAdd(a.stats + RT_STAT_WAVE_SEGMENT_ITERS, c.w_seg);
        atomicAdd(a.stats + RT_STAT_LANE_SEGMENTS, c.l_seg);
        atomicAdd(a.stats + RT_STAT_TREE_NODES, c.ktest);
        atomicAdd(a.stats + RT_STAT_TREE_TRI_TESTS, c.ktri);
    }
}

// The production kernel.  The _w5 / _w6 / _w7 variants ask the compiler for 5 / 6 / 7 waves per
// SIMD (fewer registers, more spilled) -- an occupancy / spill trade-off (RT_TUNE bits 9-10:
// 0 = _w5, the default; 1 = unconstrained; 2 = _w6; 3 = _w7).
#if defined(RT_PAIR)  // the pair's mailbox (rt_fast.h), cleared before either wave can use it
#define RT_PAIR_MAIL                                                \
    __shared__ uint32_t pair_mail[rtfast::PAIR_MAIL_WORDS];        \
    if (threadIdx.x == 0) pair_mail[0] = 0u;                        \
    __syncthreads();
#define RT_PAIR_MAIL_ARG pair_mail
#else
#define RT_PAIR_MAIL
#define RT_PAIR_MAIL_ARG nullptr
#endif
template <int STACK, bool STATS, int MODE>
__global__ __launch_bounds__(WGL) void render_fast_kernel(RenderArgs a) {
    constexpr int SL = STACK < RT_LDS_SL ? STACK : RT_LDS_SL;  // LDS entries; deeper ones in `ovf` (rt_fast.h Stack)
    __shared__ uint32_t stack_lds[(SL + rtfast::STACK_PAD_ROWS) * WGL];  // one word per entry (rt_fast.h pop)
    __shared__ uint32_t scratch_lds[((MODE & 4) ? 64 : 0) + rtfast::DEFER_WORDS];  // coop_tree's compaction, deferred leaves
    uint32_t ovf[STACK > SL ? STACK - SL : 1];
    RT_PAIR_MAIL
    render_fast_body<STACK, STATS, MODE>(a, rtfast::Stack<SL, WGL>{stack_lds, ovf}, scratch_lds, RT_PAIR_MAIL_ARG);
}
template <int STACK, bool STATS, int MODE>
__global__ __launch_bounds__(WGL) __attribute__((amdgpu_waves_per_eu(5))) void render_fast_kernel_w5(RenderArgs a) {
    constexpr int SL = STACK < RT_LDS_SL ? STACK : RT_LDS_SL;  // LDS entries; deeper ones in `ovf` (rt_fast.h Stack)
    __shared__ uint32_t stack_lds[(SL + rtfast::STACK_PAD_ROWS) * WGL];  // one word per entry (rt_fast.h pop)
    __shared__ uint32_t scratch_lds[((MODE & 4) ? 64 : 0) + rtfast::DEFER_WORDS];  // coop_tree's compaction, deferred leaves
    uint32_t ovf[STACK > SL ? STACK - SL : 1];
    RT_PAIR_MAIL
    render_fast_body<STACK, STATS, MODE>(a, rtfast::Stack<SL, WGL>{stack_lds, ovf}, scratch_lds, RT_PAIR_MAIL_ARG);
}
template <int STACK, bool STATS, int MODE>
__global__ __launch_bounds__(WGL) __attribute__((amdgpu_waves_per_eu(6))) void render_fast_kernel_w6(RenderArgs a) {
    constexpr int SL = STACK < RT_LDS_SL ? STACK : RT_LDS_SL;  // LDS entries; deeper ones in `ovf` (rt_fast.h Stack)
    __shared__ uint32_t stack_lds[(SL + rtfast::STACK_PAD_ROWS) * WGL];  // one word per entry (rt_fast.h pop)
    __shared__ uint32_t scratch_lds[((MODE & 4) ? 64 : 0) + rtfast::DEFER_WORDS];  // coop_tree's compaction, deferred leaves
    uint32_t ovf[STACK > SL ? STACK - SL : 1];
    RT_PAIR_MAIL
    render_fast_body<STACK, STATS, MODE>(a, rtfast::Stack<SL, WGL>{stack_lds, ovf}, scratch_lds, RT_PAIR_MAIL_ARG);
}
template <int STACK, bool STATS, int MODE>
__global__ __launch_bounds__(WGL) __attribute__((amdgpu_waves_per_eu(7))) void render_fast_kernel_w7(RenderArgs a) {
    constexpr int SL = STACK < RT_LDS_SL ? STACK : RT_LDS_SL;  // LDS entries; deeper ones in `ovf` (rt_fast.h Stack)
    __shared__ uint32_t stack_lds[(SL + rtfast::STACK_PAD_ROWS) * WGL];  // one word per entry (rt_fast.h pop)
    __shared__ uint32_t scratch_lds[((MODE & 4) ? 64 : 0) + rtfast::DEFER_WORDS];  // coop_tree's compaction, deferred leaves
    uint32_t ovf[STACK > SL ? STACK - SL : 1];
    RT_PAIR_MAIL
    render_fast_body<STACK, STATS, MODE>(a, rtfast::Stack<SL, WGL>{stack_lds, ovf}, scratch_lds, RT_PAIR_MAIL_ARG);
}

// Waves of `kernel` the device holds at once (refill launches size their grid to it).
template <class K>
int resident_waves(K kernel) {
    static std::mutex mu;
    static std::map<std::pair<int, const void*>, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    std::lock_guard<std::mutex> lock(mu);
    const auto key = std::make_pair(dev, (const void*)kernel);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    // waves per SIMD from the kernel's registers and LDS (the occupancy query over-counts here)
    hipFuncAttributes fa;
    int cus = 0;
    if (hipFuncGetAttributes(&fa, (const void*)kernel) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    const int vgpr_waves = fa.numRegs > 0 ? std::min(8, 512 / ((fa.numRegs + 7) / 8 * 8)) : 8;
    const int lds_waves = fa.sharedSizeBytes > 0 ? (int)(160 * 1024 / fa.sharedSizeBytes) / 4 : 8;
    return cache[key] = std::max(1, std::min(vgpr_waves, lds_waves)) * 4 * std::max(cus, 1);
}

// Dynamic LDS that caps `kernel` at `cap` (1-4) resident waves per SIMD: each wave then holds
// 160 KB / (4 cap) of its CU's LDS (rounded down to 1 KB), so 4 cap waves fit a CU and one more
// does not.  0 when uncapped.
template <class K>
size_t cap_lds_bytes(K kernel, int cap) {
    if (cap < 1 || cap > 4) return 0;
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, (const void*)kernel) != hipSuccess) return 0;
    const size_t per_wave = (size_t)(160 * 1024 / (4 * cap)) & ~(size_t)1023;
    return per_wave > fa.sharedSizeBytes ? per_wave - fa.sharedSizeBytes : 0;
}

template <class K>
hipError_t launch_grid(K kernel, const RenderArgs& args, int waves, bool refill, hipStream_t stream, size_t lds = 0,
                       int cap = 0) {
    int grid = waves;
    if (refill && args.queue_head) {  // refill variants: one grid of resident waves, the rest through the queue
        int res = resident_waves(kernel);
        int dev = 0, cus = 0;
        if (cap > 0 && hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
            res = std::min(res, cap * 4 * cus);  // the residency cap holds fewer
        if (res > 0) grid = std::min(waves, res);
    }
    hipLaunchKernelGGL(kernel, dim3((grid + WG_WAVES - 1) / WG_WAVES), dim3(WGL), lds, stream, args);
    return hipGetLastError();
}

// One (STACK, STATS, MODE) variant at the occupancy rt_render_params asks for: statistics frames run
// the unconstrained kernel; the others 5 waves per SIMD (default), 6 or 7 (waves_per_simd, or
// RT_TUNE bits 9-10 = 2 / 3).  rt_render rejects the retired RT_TUNE override 1 (compiler's choice).
template <int STACK, bool STATS, int MODE>
hipError_t launch_occ(const RenderArgs& args, int waves, hipStream_t stream) {
    constexpr bool refill = (MODE & 64) != 0;  // only these variants drain a refill queue
    if constexpr (STATS) {
        return launch_grid(render_fast_kernel<STACK, true, MODE>, args, waves, refill, stream);
    } else {
        const uint32_t t = (args.tune >> 9) & 3u;
        const int w = t == 2u ? 6 : t == 3u ? 7 : args.waves_per_simd;
        if (w >= 1 && w <= 4) {  // the 5-wave build, residency capped by dynamic LDS
            const auto k = render_fast_kernel_w5<STACK, false, MODE>;
            return launch_grid(k, args, waves, refill, stream, cap_lds_bytes(k, w), w);
        }
        if (w == 7) return launch_grid(render_fast_kernel_w7<STACK, false, MODE>, args, waves, refill, stream);
        if (w == 6) return launch_grid(render_fast_kernel_w6<STACK, false, MODE>, args, waves, refill, stream);
        return launch_grid(render_fast_kernel_w5<STACK, false, MODE>, args, waves, refill, stream);
    }
}

// A family's entry point: the stack size (30 / 40 / 64 entries) picks the instantiation.
//
// Every unit is compiled with -structurizecfg-skip-uniform-regions AND -amdgpu-remove-redundant-endcf=0
// (build.py).  Round 4 found the 6-wave leaf-tree kernel rendering wrong pixels under the first option;
// round 5 traced it (tools/w6_repro.sh): LLVM's redundant-END_CF removal lowered the
// divergent early return of cluster_cull (`if (!(dlb > ...)) return false`) inside coop_tree as
// `s_and_b64 exec, exec, vcc` with no saved mask, the parent if's `s_or_b64 exec` restoring it; the
// register allocator, running after that lowering, then put a live-range copy of the lane's ray origin
// (v[60:63] <- v[74:77]) into the flow block behind it, which the lanes that failed the test skip -- and
// bb.406 had just loaded the cluster record into v[60:63] for them.  A uniform branch left unstructurized
// by the first option (cluster_cull's `best == best` test) added the second path into the join that made
// the copy necessary.  build.py's guard rejects any object with vector instructions in such a narrowed
// flow block.
#define RT_FAST_FAMILY(NAME, DISPATCH) \
    hipError_t NAME(int stack, int mode, const RenderArgs& a, int waves, hipStream_t s) { \
        switch (stack) { \
            case 30: return DISPATCH<30>(mode, a, waves, s); \
            case 40: return DISPATCH<40>(mode, a, waves, s); \
            default: return DISPATCH<64>(mode, a, waves, s); \
        } \
    }

}  // namespace rtk
