// rt_persist.hip -- the production render kernel: one persistent launch per frame.
//
// raytracing_kernel_main (main_raytracing.cu:162-200) gives every thread one pixel and
// loops samples x bounces.  On a wave64 SIMD machine that leaves most lanes idle: paths end
// at different bounces, and 96 % of the bunny scene's triangle tests sit in ONE
// 345-triangle leaf that the lanes of a wave reach at different times.
//
// Here a wave is a small scheduler over its 64 lanes.  Each lane is in one of four states:
//   IDLE      needs a pixel (pixels are handed out from a global counter, in 8x8-tile order)
//   TRAVERSE  walking the BVH (inner nodes and small leaves: cheap steps)
//   BIG       waiting at a leaf with more than rtfast::BIG triangles
//   SHADE     traversal done: ray_color's hit/miss step, then the next segment or sample
// Every loop iteration the wave picks ONE phase by ballot -- shade, refill, one traversal
// step, or a big-leaf round -- so that each phase runs with as many lanes as possible: the
// expensive big-leaf round waits until most lanes are there, shading and refills are batched.
// Each lane still processes its own pixel strictly in the reference's order (samples,
// bounces, draws, DFS traversal), so every pixel is bit-identical to the reference
// semantics; only the interleaving of different pixels' work changes.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>

#include "rt_common.h"
#include "rt_device.h"
#include "rt_fast.h"
#include "rt_persist.h"

namespace rtp {

using namespace rtk;
using rtfast::Hit;

enum : int { IDLE = 0, TRAVERSE = 1, SHADE = 2, DONE = 3 };

struct Pixel {
    int x, y;
    bool valid;
    size_t rng_index;
};

__device__ __forceinline__ Pixel slot_pixel(const RenderArgs& a, uint32_t s) {
    const int k = (int)(s >> 8), tid = (int)(s & 255u);
    const int tile = a.shard_index + k * a.shard_count;
    int lx, ly;
    tile_pixel(tid, &lx, &ly);
    Pixel r;
    r.x = (tile % a.tiles_x) * TILE + lx;
    r.y = (tile / a.tiles_x) * TILE + ly;
    r.valid = r.x < a.width && r.y < a.height;
    r.rng_index = a.shard_count == 1 ? (size_t)r.y * a.width + r.x : (size_t)s;
    return r;
}

template <int STACK, bool STATS>
__global__ __launch_bounds__(64) void render_persistent_kernel(RenderArgs a, uint32_t* next_slot, uint32_t n_slots) {
    __shared__ uint32_t stack_lds[STACK * 2 * 64];
    uint32_t* const stk = stack_lds + threadIdx.x;
    const uint32_t lane = threadIdx.x;
    const unsigned long long below = (1ull << lane) - 1ull;
    const float4* nodes4 = reinterpret_cast<const float4*>(a.nodes);
    const float4* tris = reinterpret_cast<const float4*>(a.tris);
    const bool scene_fast = a.scene_fast != 0;
    const rtm::f3 cam_o = ld3(a.cam.origin), cam_h = ld3(a.cam.horizontal), cam_v = ld3(a.cam.vertical),
                  cam_ll = ld3(a.cam.lower_left_corner);

    // pixel state
    int state = IDLE;
    uint32_t slot = 0;
    Pixel px;
    px.x = px.y = 0, px.valid = false, px.rng_index = 0;
    rtm::Xorwow rng{0, 0, 0, 0, 0, 0};
    float acc_r = 0.0f, acc_g = 0.0f, acc_b = 0.0f, acc_a = 0.0f;
    int sample = 0, bounce = 0;
    // path state
    rtm::f3 ro = cam_o, rd = cam_o, color = rtm::mk(0, 0, 0), thr = rtm::mk(1, 1, 1);
    // traversal state
    rtfast::Ray R;
    R.o = R.d = R.nd = R.r = rtm::mk(1, 1, 1);
    R.fast = false;
    Hit h;
    h.best = 1e30f, h.kind = 0, h.id = 0, h.bx = h.by = 0.0f;
    bool active = false;
    uint32_t first = 0, cnt = 0;
    int sp = 0;
    bool pixels_left = true;  // wave-uniform
    Counters c;

    for (;;) {
        const bool trav = state == TRAVERSE;
        const unsigned long long small_m = __ballot(trav && cnt <= (uint32_t)rtfast::BIG);
        const unsigned long long big_m = __ballot(trav && cnt > (uint32_t)rtfast::BIG);
        const unsigned long long shade_m = __ballot(state == SHADE);
        const unsigned long long idle_m = __ballot(state == IDLE);
        const int n_small = __popcll(small_m), n_big = __popcll(big_m), n_shade = __popcll(shade_m);
        const int n_idle = pixels_left ? __popcll(idle_m) : 0;

        int phase;  // 0 shade, 1 refill, 2 small step, 3 big round, 4 exit
        if (n_shade >= 32 || (n_shade > 0 && n_small == 0))
            phase = 0;
        else if (n_idle >= 32 || (n_idle > 0 && n_small == 0 && n_big < 48))
            phase = 1;
        else if (n_small > 0)
            phase = 2;
        else if (n_big > 0)
            phase = 3;
        else if (n_idle > 0)
            phase = 1;
        else
            phase = 4;
        if (phase == 4) break;

        bool start_segment = false;  // lanes that must set up a new ray this iteration
        if (phase == 1) {
            // ---- hand pixels to idle lanes: consecutive slots (an 8x8 sub-tile per 64) ----
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(next_slot, (uint32_t)__popcll(idle_m));
            base = __builtin_amdgcn_readfirstlane(base);
            if (base + (uint32_t)__popcll(idle_m) >= n_slots) pixels_left = false;
            if (state == IDLE) {
                const uint32_t s = base + (uint32_t)__popcll(idle_m & below);
                px = slot_pixel(a, s);
                if (s >= n_slots || !px.valid) {
                    state = s >= n_slots ? DONE : IDLE;
                } else {
                    slot = s;
                    const rt_rng_state* rs = a.rng + px.rng_index;
                    rng = rtm::Xorwow{rs->d, rs->v[0], rs->v[1], rs->v[2], rs->v[3], rs->v[4]};
                    acc_r = acc_g = acc_b = acc_a = 0.0f;
                    sample = -1;
                    state = SHADE;  // the next shade phase draws sample 0's camera ray
                }
            }
        } else if (phase == 0) {
            // ---- shade: ray_color's per-segment step (main_raytracing.cu:119-158) ----
            if (state == SHADE) {
                bool end = sample < 0;  // a fresh pixel has no path yet
                if (!end) {
                    if (h.kind != 0) {
                        if (STATS) c.hit++;
                        const rtm::f3 pos = rtm::add(ro, rtm::muls(R.nd, h.best));
                        rtm::f3 nrm;
                        uint32_t mat;
                        if (h.kind == 1) {
                            const GeometrySphere& sph = a.spheres[h.id];
                            nrm = rtm::divs(rtm::sub(pos, ld3(sph.position)), sph.radius);
                            mat = (uint32_t)sph.material;
                        } else {
                            const GPUFace f = a.faces[h.id];
                            const float bz = (1.0f - h.bx) - h.by;
                            nrm = rtm::normalize(rtm::add(rtm::add(rtm::muls(ld3(a.vertices[f.v0].normal), h.bx),
                                                                   rtm::muls(ld3(a.vertices[f.v1].normal), h.by)),
                                                          rtm::muls(ld3(a.vertices[f.v2].normal), bz)));
                            if (rtm::dot(R.nd, nrm) >= 0.0f) nrm = rtm::neg(nrm);
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
                            const rtm::f3 cl =
                                rtm::mk(rtm::gmin(rtm::gmax(cs.x, 0.0f), 50.0f), rtm::gmin(rtm::gmax(cs.y, 0.0f), 50.0f),
                                        rtm::gmin(rtm::gmax(cs.z, 0.0f), 50.0f));
                            color = rtm::add(color, rtm::mul(thr, cl));
                        }
                        end = true;
                    }
                    if (++bounce >= a.bounces) end = true;
                    if (end) {
                        acc_r += color.x;
                        acc_g += color.y;
                        acc_b += color.z;
                        acc_a += 1.0f;
                    }
                }
                if (end) {
                    // next camera sample (main_raytracing.cu:188-193); an empty bounce loop
                    // (bounces == 0) makes a sample contribute (0, 0, 0, 1) without a ray
                    sample++;
                    while (sample < a.spp && a.bounces == 0) {
                        rng.uniform();
                        rng.uniform();
                        acc_a += 1.0f;
                        sample++;
                    }
                    if (sample < a.spp) {
                        const float ru = rng.uniform();
                        const float rv = rng.uniform();
                        const float uvx = ((float)px.x + ru) / (float)a.width;
                        const float uvy = ((float)px.y + rv) / (float)a.height;
                        ro = cam_o;  // GPUCamera::GetRay (GPUScene.h:13), not normalized
                        rd = rtm::sub(rtm::add(rtm::add(cam_ll, rtm::muls(cam_h, uvx)), rtm::muls(cam_v, uvy)), cam_o);
                        color = rtm::mk(0, 0, 0);
                        thr = rtm::mk(1, 1, 1);
                        bounce = 0;
                        start_segment = true;
                    } else {
                        // main_raytracing.cu:195-199
                        const float fs = (float)a.spp;
                        const rtm::f4 res{acc_r / fs, acc_g / fs, acc_b / fs, acc_a / fs};
                        const float lerp = a.frame_index > 0 ? 1.0f / (float)(a.frame_index + 1) : 1.0f;
                        float4 prev;
                        float4* out;
                        if (a.out_shard) {
                            prev = a.last ? reinterpret_cast<const float4*>(a.last)[slot] : make_float4(0, 0, 0, 0);
                            out = a.out_shard + slot;
                        } else {
                            prev = a.last ? *reinterpret_cast<const float4*>(a.last + (size_t)px.y * a.pitch + (size_t)px.x * 16)
                                          : make_float4(0, 0, 0, 0);
                            out = reinterpret_cast<float4*>(a.surface + (size_t)px.y * a.pitch + (size_t)px.x * 16);
                        }
                        const rtm::f4 o = rtm::mix4(rtm::f4{prev.x, prev.y, prev.z, prev.w}, res, lerp);
                        *out = make_float4(o.x, o.y, o.z, 1.0f);
                        rt_rng_state* rs = a.rng + px.rng_index;
                        rs->d = rng.d;
                        rs->v[0] = rng.v0, rs->v[1] = rng.v1, rs->v[2] = rng.v2, rs->v[3] = rng.v3, rs->v[4] = rng.v4;
                        state = IDLE;
                    }
                } else {
                    start_segment = true;
                }
            }
        } else if (phase == 2) {
            // ---- one traversal step for every lane that can make cheap progress ----
            if (STATS) {
                c.w_small += lane == 0;
                c.l_small += (small_m >> lane) & 1ull;
            }
            if ((small_m >> lane) & 1ull) {
                if (cnt > 0) {
                    for (uint32_t i = first; i < first + cnt; i++)
                        rtfast::test_triangle<STATS>(R, tris[3 * i], tris[3 * i + 1], tris[3 * i + 2], h, c);
                    active = rtfast::pop<64>(nodes4, stk, sp, R, h.best, first, cnt);
                } else if (!rtfast::inner_step<64, STATS>(nodes4, stk, sp, R, h.best, first, cnt, c)) {
                    active = rtfast::pop<64>(nodes4, stk, sp, R, h.best, first, cnt);
                }
            }
        } else {
            // ---- big-leaf round: every waiting lane runs its leaf together ----
            const bool mine = (big_m >> lane) & 1ull;
            const int l0 = __ffsll((long long)big_m) - 1;
            const uint32_t f0 = __builtin_amdgcn_readlane(first, l0);
            const uint32_t c0 = __builtin_amdgcn_readlane(cnt, l0);
            if (STATS) {
                uint32_t mx = mine ? cnt : 0u;
                for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
                c.w_big += lane == 0 ? mx : 0;
                c.l_big += mine ? cnt : 0;
            }
            if (__ballot(mine && first == f0) == big_m) {
                rtfast::ConstF4 st = (rtfast::ConstF4)(tris + 3 * (size_t)f0);
                rtfast::ConstF4 const last = st + 3 * (c0 - 1);
                float4 A = rtfast::ldc(st, 0), B = rtfast::ldc(st, 1), Cc = rtfast::ldc(st, 2);
                for (uint32_t i = 0; i < c0; i++) {
                    st = st == last ? st : st + 3;
                    const float4 An = rtfast::ldc(st, 0), Bn = rtfast::ldc(st, 1), Cn = rtfast::ldc(st, 2);
                    if (mine) rtfast::test_triangle<STATS>(R, A, B, Cc, h, c);
                    A = An, B = Bn, Cc = Cn;
                }
            } else if (mine) {
                for (uint32_t i = first; i < first + cnt; i++)
                    rtfast::test_triangle<STATS>(R, tris[3 * i], tris[3 * i + 1], tris[3 * i + 2], h, c);
            }
            if (mine) active = rtfast::pop<64>(nodes4, stk, sp, R, h.best, first, cnt);
        }

        if (start_segment) {
            // ---- GetRayHit set-up: sphere loop + root box (main_raytracing.cu:83-109) ----
            const rtm::f3 nd = rtm::normalize(rd);
            c.seg++;
            h.best = 1e30f, h.kind = 0, h.id = 0, h.bx = h.by = 0.0f;
            for (int i = 0; i < a.sphere_count; i++) {
                const GeometrySphere& sph = a.spheres[i];
                float dist;
                if (rtd::intersect_sphere(ro, nd, ld3(sph.position), sph.radius * sph.radius, &dist)) {
                    if (dist >= h.best) continue;
                    h.best = dist;
                    h.kind = 1;
                    h.id = (uint32_t)i;
                    if (STATS) c.sacc++;
                }
            }
            R = rtfast::make_ray(ro, rd, nd, scene_fast);
            const float4 lo = nodes4[0], hi = nodes4[1];
            if (STATS) c.node++;
            float tmin, tmax;
            rtfast::slab_exact(R, lo, hi, &tmin, &tmax);
            active = tmax >= tmin && tmin < h.best && tmax > 0.0f;
            first = __float_as_uint(hi.z), cnt = __float_as_uint(hi.w);
            sp = 0;
            state = TRAVERSE;
        }
        if (state == TRAVERSE && !active) state = SHADE;
    }

    if (a.seg_counter) {
        unsigned long long v = c.seg;
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0 && v) atomicAdd(a.seg_counter, v);
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
    }
}

// Per (device, stream) 4-byte pixel counter, zeroed on the stream before each launch.
std::mutex g_mutex;
std::map<std::pair<int, void*>, uint32_t*> g_counters;

hipError_t counter_for(hipStream_t s, uint32_t** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(g_mutex);
    uint32_t*& p = g_counters[{dev, (void*)s}];
    if (!p) {
        e = hipMalloc(&p, 256);
        if (e != hipSuccess) {
            p = nullptr;
            return e;
        }
    }
    *out = p;
    return hipSuccess;
}

template <int STACK, bool STATS>
hipError_t run_t(const RenderArgs& a, int tiles, hipStream_t s) {
    uint32_t* counter = nullptr;
    hipError_t e = counter_for(s, &counter);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(counter, 0, 4, s);
    if (e != hipSuccess) return e;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    const uint32_t slots = (uint32_t)tiles * 256u;
    // Waves resident per CU are limited by the LDS stack (STACK*2*64*4 bytes per wave).
    const int per_cu = (160 * 1024) / (STACK * 2 * 64 * 4);
    int waves = cus * (per_cu < 16 ? per_cu : 16);
    const int max_waves = (int)((slots + 63) / 64);
    if (waves > max_waves) waves = max_waves;
    hipLaunchKernelGGL((render_persistent_kernel<STACK, STATS>), dim3(waves), dim3(64), 0, s, a, counter, slots);
    return hipGetLastError();
}

}  // namespace rtp

hipError_t rt_persistent_render(const rtk::RenderArgs& a, int tiles, int depth, bool stats, hipStream_t stream) {
    if (depth >= 0 && depth + 2 <= 28)
        return stats ? rtp::run_t<28, true>(a, tiles, stream) : rtp::run_t<28, false>(a, tiles, stream);
    if (depth >= 0 && depth + 2 <= 40)
        return stats ? rtp::run_t<40, true>(a, tiles, stream) : rtp::run_t<40, false>(a, tiles, stream);
    return stats ? rtp::run_t<64, true>(a, tiles, stream) : rtp::run_t<64, false>(a, tiles, stream);
}
