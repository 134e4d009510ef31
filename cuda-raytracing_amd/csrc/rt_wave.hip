// rt_wave.hip -- wavefront form of the render path (the production path for uploaded scenes).
//
// raytracing_kernel_main (main_raytracing.cu:162-200) is one thread per pixel looping
// samples x bounces.  On a wave64 machine that wastes most lanes: paths end at different
// bounces, and 96 % of the triangle tests of the bunny scene sit in one 345-triangle leaf
// that the lanes of a wave reach at different times.  Here a frame is a sequence of
// segment iterations over a queue of pixel slots:
//
//   begin_kernel   per pixel: load its RNG state, draw sample 0's camera ray, enqueue
//   trace_kernel   persistent waves pull slots from the queue; a lane that finishes its
//                  ray takes the next one, so the wave keeps all 64 lanes busy and gathers
//                  nearly all of them at the big leaf before running it (rt_fast.h)
//   shade_kernel   per queued slot: ray_color's hit / miss / Russian-roulette step; a path
//                  that ends adds its colour and starts the pixel's next sample; a pixel
//                  whose samples are done writes its progressive-lerped output and RNG state
//
// Each pixel has at most one ray in flight, and its draws happen in the reference order
// (u, v per sample, then 4 per hit), so every pixel's result is bit-identical to the
// per-pixel kernel's.  Path state lives in HBM as SoA arrays indexed by pixel slot.
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <mutex>

#include "rt_common.h"
#include "rt_device.h"
#include "rt_fast.h"
#include "rt_wave.h"

namespace rtwave {

using namespace rtk;
using rtfast::Hit;

constexpr uint32_t POOL = 128;  // per-wave ring of queued slots (LDS)
constexpr uint32_t HIT_NONE = 0xffffffffu;
constexpr uint32_t HIT_SPHERE = 0x80000000u;

struct Slot {
    int x, y;
    bool valid;
    size_t rng_index;
};

__device__ __forceinline__ Slot slot_pixel(const RenderArgs& a, uint32_t s) {
    const int k = (int)(s >> 8), tid = (int)(s & 255u);
    const int tile = a.shard_index + k * a.shard_count;
    int lx, ly;
    tile_pixel(tid, &lx, &ly);
    Slot r;
    r.x = (tile % a.tiles_x) * TILE + lx;
    r.y = (tile / a.tiles_x) * TILE + ly;
    r.valid = r.x < a.width && r.y < a.height;
    r.rng_index = a.shard_count == 1 ? (size_t)r.y * a.width + r.x : (size_t)s;
    return r;
}

__device__ __forceinline__ rtm::Xorwow load_rng(const WaveWS& w, uint32_t s) {
    const size_t n = w.n;
    return rtm::Xorwow{w.rng[s], w.rng[n + s], w.rng[2 * n + s], w.rng[3 * n + s], w.rng[4 * n + s], w.rng[5 * n + s]};
}
__device__ __forceinline__ void store_rng(const WaveWS& w, uint32_t s, const rtm::Xorwow& r) {
    const size_t n = w.n;
    w.rng[s] = r.d, w.rng[n + s] = r.v0, w.rng[2 * n + s] = r.v1, w.rng[3 * n + s] = r.v2, w.rng[4 * n + s] = r.v3,
    w.rng[5 * n + s] = r.v4;
}
__device__ __forceinline__ rtm::f3 ld3s(const float* p, size_t n, uint32_t s) { return rtm::mk(p[s], p[n + s], p[2 * n + s]); }
__device__ __forceinline__ void st3s(float* p, size_t n, uint32_t s, rtm::f3 v) {
    p[s] = v.x, p[n + s] = v.y, p[2 * n + s] = v.z;
}

// Wave-aggregated append of `slot` (lanes with `want`) to queue q.
__device__ __forceinline__ void enqueue(const WaveWS& w, int q, bool want, uint32_t slot) {
    const unsigned long long m = __ballot(want);
    if (!m) return;
    const uint32_t n = (uint32_t)__popcll(m);
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(w.ctl + q, n);
    base = __shfl(base, leader);
    if (want) {
        const uint32_t rank = (uint32_t)__popcll(m & ((1ull << (threadIdx.x & 63)) - 1ull));
        w.queue[q][base + rank] = slot;
    }
}

// main_raytracing.cu:195-199 for a finished pixel + the RNG state back to the caller's array.
__device__ __forceinline__ void finalize(const RenderArgs& a, const WaveWS& w, uint32_t s, const Slot& p,
                                         const rtm::Xorwow& rng) {
    const size_t n = w.n;
    const float fs = (float)a.spp;
    const rtm::f4 res{w.acc[s] / fs, w.acc[n + s] / fs, w.acc[2 * n + s] / fs, w.acc[3 * n + s] / fs};
    const float lerp = a.frame_index > 0 ? 1.0f / (float)(a.frame_index + 1) : 1.0f;
    float4 prev;
    float4* out;
    if (a.out_shard) {
        prev = a.last ? reinterpret_cast<const float4*>(a.last)[s] : make_float4(0, 0, 0, 0);
        out = a.out_shard + s;
    } else {
        prev = a.last ? *reinterpret_cast<const float4*>(a.last + (size_t)p.y * a.pitch + (size_t)p.x * 16)
                      : make_float4(0, 0, 0, 0);
        out = reinterpret_cast<float4*>(a.surface + (size_t)p.y * a.pitch + (size_t)p.x * 16);
    }
    const rtm::f4 o = rtm::mix4(rtm::f4{prev.x, prev.y, prev.z, prev.w}, res, lerp);
    *out = make_float4(o.x, o.y, o.z, 1.0f);
    rt_rng_state* rs = a.rng + p.rng_index;
    rs->d = rng.d;
    rs->v[0] = rng.v0, rs->v[1] = rng.v1, rs->v[2] = rng.v2, rs->v[3] = rng.v3, rs->v[4] = rng.v4;
}

// Start the pixel's next camera sample (main_raytracing.cu:188-193); returns false when the
// pixel has no samples left (it is finalized).  An empty bounce loop (bounces == 0) makes a
// sample contribute (0, 0, 0, 1) without a ray.
__device__ __forceinline__ bool next_sample(const RenderArgs& a, const WaveWS& w, uint32_t s, const Slot& p,
                                            rtm::Xorwow& rng, int sample) {
    const size_t n = w.n;
    while (sample < a.spp) {
        const float ru = rng.uniform();
        const float rv = rng.uniform();
        if (a.bounces == 0) {
            w.acc[3 * n + s] += 1.0f;
            sample++;
            continue;
        }
        const float uvx = ((float)p.x + ru) / (float)a.width;
        const float uvy = ((float)p.y + rv) / (float)a.height;
        const rtm::f3 cam_o = ld3(a.cam.origin), cam_h = ld3(a.cam.horizontal), cam_v = ld3(a.cam.vertical),
                      cam_ll = ld3(a.cam.lower_left_corner);
        st3s(w.ro, n, s, cam_o);
        st3s(w.rd, n, s, rtm::sub(rtm::add(rtm::add(cam_ll, rtm::muls(cam_h, uvx)), rtm::muls(cam_v, uvy)), cam_o));
        st3s(w.thr, n, s, rtm::mk(1, 1, 1));
        st3s(w.col, n, s, rtm::mk(0, 0, 0));
        w.bounce[s] = 0;
        w.sample[s] = sample;
        return true;
    }
    w.sample[s] = sample;
    finalize(a, w, s, p, rng);
    return false;
}

__global__ __launch_bounds__(256) void begin_kernel(RenderArgs a, WaveWS w) {
    const uint32_t s = blockIdx.x * 256u + threadIdx.x;
    bool want = false;
    if (s < w.n) {
        const Slot p = slot_pixel(a, s);
        if (p.valid) {
            const rt_rng_state* rs = a.rng + p.rng_index;
            rtm::Xorwow rng{rs->d, rs->v[0], rs->v[1], rs->v[2], rs->v[3], rs->v[4]};
            const size_t n = w.n;
            w.acc[s] = w.acc[n + s] = w.acc[2 * n + s] = w.acc[3 * n + s] = 0.0f;
            want = next_sample(a, w, s, p, rng, 0);
            store_rng(w, s, rng);
        }
    }
    enqueue(w, 0, want, s);
}

// ---------------------------------------------------------------------------------------
// trace: persistent waves with lane refill from the slot queue
// ---------------------------------------------------------------------------------------
template <int STACK, bool STATS>
__global__ __launch_bounds__(64) void trace_kernel(RenderArgs a, WaveWS w, int cur) {
    __shared__ uint32_t stack_lds[STACK * 2 * 64];
    __shared__ uint32_t pool[POOL];
    uint32_t* const stk = stack_lds + threadIdx.x;
    const uint32_t lane = threadIdx.x;
    if (blockIdx.x == 0 && lane == 0) {  // reset the other queue for this iteration's shade pass
        w.ctl[1 - cur] = 0;
        w.ctl[3 - cur] = 0;
    }
    const uint32_t count = __builtin_amdgcn_readfirstlane(w.ctl[cur]);
    if (count == 0) return;
    const uint32_t* queue = w.queue[cur];
    const float4* nodes4 = reinterpret_cast<const float4*>(a.nodes);
    const float4* tris = reinterpret_cast<const float4*>(a.tris);
    const size_t n = w.n;
    const bool scene_fast = a.scene_fast != 0;

    uint32_t ph = 0, pt = 0;  // pool ring head / tail (wave-uniform)
    bool exhausted = false;
    bool has = false, active = false;
    uint32_t slot = 0, first = 0, cnt = 0;
    int sp = 0;
    rtfast::Ray R;
    R.o = R.d = R.nd = R.r = rtm::mk(1, 1, 1);
    R.fast = false;
    Hit h;
    h.best = 1e30f, h.kind = 0, h.id = 0, h.bx = h.by = 0.0f;
    Counters c;

    for (;;) {
        const unsigned long long idle_m = __ballot(!has);
        const unsigned long long small_m = __ballot(has && active && cnt <= (uint32_t)rtfast::BIG);
        const uint32_t n_idle = (uint32_t)__popcll(idle_m);
        if ((!exhausted || pt != ph) && n_idle > 0 && (n_idle >= 16 || small_m == 0)) {
            // ---- refill idle lanes from the queue (via the LDS ring) ----
            if (!exhausted && pt - ph < n_idle) {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(w.ctl + 2 + cur, 64u);
                base = __builtin_amdgcn_readfirstlane(base);
                const uint32_t idx = base + lane;
                const bool ok = idx < count;
                if (ok) pool[(pt + lane) & (POOL - 1)] = queue[idx];
                const uint32_t got = (uint32_t)__popcll(__ballot(ok));
                pt += got;
                if (base + 64u >= count) exhausted = true;
                __syncthreads();
            }
            const uint32_t avail = pt - ph;
            const uint32_t rank = (uint32_t)__popcll(idle_m & ((1ull << lane) - 1ull));
            if (!has && rank < avail) {
                slot = pool[(ph + rank) & (POOL - 1)];
                has = true;
                // ---- segment setup: GetRayHit's sphere loop + the root box (main_raytracing.cu:83-109)
                const rtm::f3 ro = ld3s(w.ro, n, slot), rd = ld3s(w.rd, n, slot);
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
            }
            ph += avail < n_idle ? avail : n_idle;
        } else if (small_m) {
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
            // ---- every busy lane waits at a big leaf (or the queue is drained) ----
            const unsigned long long big = __ballot(has && active);
            if (big) {
                const bool mine = (big >> lane) & 1ull;
                const int l0 = __ffsll((long long)big) - 1;
                const uint32_t f0 = __builtin_amdgcn_readlane(first, l0);
                const uint32_t c0 = __builtin_amdgcn_readlane(cnt, l0);
                if (STATS) {
                    uint32_t mx = mine ? cnt : 0u;
                    for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
                    c.w_big += lane == 0 ? mx : 0;
                    c.l_big += mine ? cnt : 0;
                }
                if (__ballot(mine && first == f0) == big) {
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
            } else {
                break;  // no lane busy, queue and pool drained
            }
        }
        // ---- lanes whose traversal ended: publish the closest hit ----
        if (has && !active) {
            w.hit_t[slot] = h.best;
            w.hit_id[slot] = h.kind == 0 ? HIT_NONE : (h.kind == 1 ? (HIT_SPHERE | h.id) : h.id);
            w.hit_bx[slot] = h.bx;
            w.hit_by[slot] = h.by;
            has = false;
        }
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
        atomicAdd(a.stats + RT_STAT_WAVE_SMALL_ITERS, c.w_small);
        atomicAdd(a.stats + RT_STAT_LANE_SMALL, c.l_small);
        atomicAdd(a.stats + RT_STAT_WAVE_BIG_TRIS, c.w_big);
        atomicAdd(a.stats + RT_STAT_LANE_BIG_TRIS, c.l_big);
    }
}

// ---------------------------------------------------------------------------------------
// shade: ray_color's per-segment step (main_raytracing.cu:119-158)
// ---------------------------------------------------------------------------------------
template <bool STATS>
__global__ __launch_bounds__(256) void shade_kernel(RenderArgs a, WaveWS w, int cur) {
    const uint32_t count = w.ctl[cur];
    const uint32_t* queue = w.queue[cur];
    const size_t n = w.n;
    unsigned long long n_hit = 0, n_miss = 0;
    const uint32_t stride = gridDim.x * 256u;
    const uint32_t rounds = (count + stride - 1) / stride;
    for (uint32_t r = 0; r < rounds; r++) {
        const uint32_t qi = r * stride + blockIdx.x * 256u + threadIdx.x;
        bool want = false;
        uint32_t s = 0;
        if (qi < count) {
            s = queue[qi];
            const Slot p = slot_pixel(a, s);
            rtm::Xorwow rng = load_rng(w, s);
            rtm::f3 ro = ld3s(w.ro, n, s), rd = ld3s(w.rd, n, s), thr = ld3s(w.thr, n, s), color = ld3s(w.col, n, s);
            int bounce = w.bounce[s];
            const uint32_t hid = w.hit_id[s];
            bool end = false;
            if (hid != HIT_NONE) {
                if (STATS) n_hit++;
                const float best = w.hit_t[s];
                const rtm::f3 nd = rtm::normalize(rd);
                const rtm::f3 pos = rtm::add(ro, rtm::muls(nd, best));
                rtm::f3 nrm;
                uint32_t mat;
                if (hid & HIT_SPHERE) {
                    const GeometrySphere& sp = a.spheres[hid & ~HIT_SPHERE];
                    nrm = rtm::divs(rtm::sub(pos, ld3(sp.position)), sp.radius);
                    mat = (uint32_t)sp.material;
                } else {
                    const GPUFace f = a.faces[hid];
                    const float bx = w.hit_bx[s], by = w.hit_by[s];
                    const float bz = (1.0f - bx) - by;
                    nrm = rtm::normalize(rtm::add(rtm::add(rtm::muls(ld3(a.vertices[f.v0].normal), bx),
                                                           rtm::muls(ld3(a.vertices[f.v1].normal), by)),
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
                const float pr = rtm::gmax(thr.x, rtm::gmax(thr.y, thr.z));
                if (rng.uniform() > pr) {
                    end = true;
                } else {
                    thr = rtm::muls(thr, 1.0f / pr);
                }
            } else {
                if (STATS) n_miss++;
                if (a.sky) {
                    const rtm::f3 dir = rtd::quat_rotate(a.qw, a.qx, a.qy, a.qz, rd);
                    const rtm::f3 cs = rtd::cube_sample(a.sky, a.sky_n, dir);
                    const rtm::f3 cl = rtm::mk(rtm::gmin(rtm::gmax(cs.x, 0.0f), 50.0f), rtm::gmin(rtm::gmax(cs.y, 0.0f), 50.0f),
                                               rtm::gmin(rtm::gmax(cs.z, 0.0f), 50.0f));
                    color = rtm::add(color, rtm::mul(thr, cl));
                }
                end = true;
            }
            if (++bounce >= a.bounces) end = true;
            if (end) {
                w.acc[s] += color.x;
                w.acc[n + s] += color.y;
                w.acc[2 * n + s] += color.z;
                w.acc[3 * n + s] += 1.0f;
                want = next_sample(a, w, s, p, rng, w.sample[s] + 1);
            } else {
                st3s(w.ro, n, s, ro);
                st3s(w.rd, n, s, rd);
                st3s(w.thr, n, s, thr);
                st3s(w.col, n, s, color);
                w.bounce[s] = bounce;
                want = true;
            }
            store_rng(w, s, rng);
        }
        enqueue(w, 1 - cur, want, s);
    }
    if (STATS) {
        atomicAdd(a.stats + RT_STAT_HITS, n_hit);
        atomicAdd(a.stats + RT_STAT_MISSES, n_miss);
    }
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
struct Workspace {
    void* mem = nullptr;
    size_t bytes = 0;
};

std::mutex g_ws_mutex;
std::map<std::pair<int, void*>, Workspace> g_ws;  // (device, stream) -> workspace

hipError_t get_workspace(uint32_t slots, hipStream_t stream, WaveWS* out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    // floats: ro 3, rd 3, thr 3, col 3, acc 4, hit t/bx/by 3; ints: bounce, sample, hit id, 2 queues; rng 6
    const size_t per_slot = 4 * (3 + 3 + 3 + 3 + 4 + 3 + 1 + 1 + 1 + 2 + 6);
    const size_t need = per_slot * (size_t)slots + 256;
    std::lock_guard<std::mutex> lock(g_ws_mutex);
    Workspace& ws = g_ws[{dev, (void*)stream}];
    if (ws.bytes < need) {
        if (ws.mem) (void)hipFree(ws.mem);
        ws.mem = nullptr;
        ws.bytes = 0;
        e = hipMalloc(&ws.mem, need);
        if (e != hipSuccess) return e;
        ws.bytes = need;
    }
    char* p = (char*)ws.mem;
    const size_t n = slots;
    out->n = slots;
    out->ctl = (uint32_t*)p;
    p += 256;
    auto take = [&](size_t count) {
        char* q = p;
        p += 4 * count;
        return q;
    };
    out->ro = (float*)take(3 * n);
    out->rd = (float*)take(3 * n);
    out->thr = (float*)take(3 * n);
    out->col = (float*)take(3 * n);
    out->acc = (float*)take(4 * n);
    out->hit_t = (float*)take(n);
    out->hit_bx = (float*)take(n);
    out->hit_by = (float*)take(n);
    out->bounce = (int*)take(n);
    out->sample = (int*)take(n);
    out->hit_id = (uint32_t*)take(n);
    out->queue[0] = (uint32_t*)take(n);
    out->queue[1] = (uint32_t*)take(n);
    out->rng = (uint32_t*)take(6 * n);
    return hipSuccess;
}

template <int STACK, bool STATS>
hipError_t run_t(const RenderArgs& a, const WaveWS& w, int tiles, hipStream_t s) {
    hipError_t e = hipMemsetAsync(w.ctl, 0, 256, s);
    if (e != hipSuccess) return e;
    const uint32_t slots = (uint32_t)tiles * 256u;
    hipLaunchKernelGGL(begin_kernel, dim3((slots + 255) / 256), dim3(256), 0, s, a, w);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    const int trace_waves = cus * 12;
    const int iters = a.spp * a.bounces;
    for (int it = 0; it < iters; it++) {
        const int cur = it & 1;
        hipLaunchKernelGGL((trace_kernel<STACK, STATS>), dim3(trace_waves), dim3(64), 0, s, a, w, cur);
        hipLaunchKernelGGL((shade_kernel<STATS>), dim3(cus * 8), dim3(256), 0, s, a, w, cur);
    }
    return hipGetLastError();
}

}  // namespace rtwave

hipError_t rt_wave_render(const rtk::RenderArgs& a, int tiles, int depth, bool stats, hipStream_t stream) {
    rtwave::WaveWS w;
    hipError_t e = rtwave::get_workspace((uint32_t)tiles * 256u, stream, &w);
    if (e != hipSuccess) return e;
    if (depth >= 0 && depth + 2 <= 28)
        return stats ? rtwave::run_t<28, true>(a, w, tiles, stream) : rtwave::run_t<28, false>(a, w, tiles, stream);
    if (depth >= 0 && depth + 2 <= 40)
        return stats ? rtwave::run_t<40, true>(a, w, tiles, stream) : rtwave::run_t<40, false>(a, w, tiles, stream);
    return stats ? rtwave::run_t<64, true>(a, w, tiles, stream) : rtwave::run_t<64, false>(a, w, tiles, stream);
}
