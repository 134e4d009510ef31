// rt_lone.hip -- the lone-pixel kernel: one wave renders ONE pixel's whole frame (all its camera
// samples, every segment), all 64 lanes on that pixel's single ray at a time.
//
// Why.  A strong-scaled frame ends with its costliest pixels: a pixel's samples run one after the
// other on one RNG stream (RayTracing/main_raytracing.cu:188-193, Random.cu:7), so its chain of
// traversal steps cannot be split, and one wave issues a VALU instruction only every ~8 cycles
// (profiles/r03a_valu_microbench.txt): a lone ray stepping through BVHRayHit's DFS
// (main_raytracing.cu:43-78) one node at a time is bound by the instruction latency of each step.
// Here the wave spends its 64 lanes on the tree instead of on other rays:
//
//  * the BVH is read as TREELETS (mirror.h): subtrees of up to 63 nodes stored in right-first
//    preorder, so lane j holds the node the reference's DFS would reach j-th if nothing were pruned
//    (the subtree of lane j is lanes [j, j + size)).  One load round and ONE exact IntersectAABB
//    (Math.h:50-61, IEEE divisions) per lane test all of a treelet's nodes at once;
//  * the DFS itself is then a few ballots per leaf: with `best` the current closest distance,
//    a node is visited iff it and every ancestor passed `tmax >= tmin && tmin < best && tmax > 0`
//    at the moment the reference popped it -- ancestors' decisions are frozen when the walk passes
//    them (best only shrinks at leaves), later ones use the live best -- and the next leaf (or
//    the next frontier node, whose subtree is another treelet) in preorder is the lowest set bit
//    of one ballot.  The visit order, every decision and the leaves' triangle loops are the
//    reference's, so the hit is bit-identical;
//  * leaves: a small leaf's triangles one per lane, the (t, index) minimum below the entry best is
//    the sequential loop's result (rt_fast.h lone_traverse); big leaves through the wave's
//    cooperative rounds (coop_leaf / coop_tree); a NaN distance runs the leaf's sequential loop;
//  * spheres (main_raytracing.cu:90-103) one per lane, (distance, index) minimum; shading, Russian
//    roulette and the RNG draws are the production kernel's (shade_segment), computed uniformly.
//
// The pixels come from a list (rt_render_params.lone_slots, rt_lone_plan); the production kernel
// renders the others concurrently (rt_kernel.hip).  Same outputs as the production kernel: RNG
// state write-back, pitched surface or compact shard, segment counter.
#include "rt_fast_body.h"

namespace rtk {
namespace {

constexpr uint32_t TL_EMPTY = 0xffffffffu;  // treelet slot without a node (mirror.h)
constexpr int TL_FRAMES = 16;               // nested treelets: BVH depth <= 6 * 16 - 1

// This lane's slot of the current treelet: its ancestor slots, its subtree size (in slots, itself
// included) and whether it is a frontier (an inner node whose subtree is another treelet).
struct TLSlot {
    unsigned long long anc;
    uint32_t size;
    bool frontier;
};

__device__ __forceinline__ TLSlot tl_geom(const float4* tl, uint32_t T, uint32_t lane) {
    const float4 C = tl[(size_t)T * 192u + 3u * lane + 2u];
    TLSlot g;
    g.anc = (unsigned long long)__float_as_uint(C.x) | ((unsigned long long)__float_as_uint(C.y) << 32);
    g.size = __float_as_uint(C.z);
    g.frontier = __float_as_uint(C.w) != 0u;
    return g;
}

__device__ __forceinline__ unsigned long long bits(uint32_t lo, uint32_t hi) {  // [lo, hi), hi <= 64
    const unsigned long long top = hi >= 64u ? ~0ull : ((1ull << hi) - 1ull);
    const unsigned long long bot = lo >= 64u ? ~0ull : ((1ull << lo) - 1ull);
    return top & ~bot;
}

// IntersectAABB's box part for this lane's slot of treelet T: key = tmin when `tmax >= tmin &&
// tmax > 0`, +inf otherwise (so `key < best` is the reference's whole test); X, cnt as stored.
__device__ __forceinline__ void tl_load(const float4* tl, uint32_t T, uint32_t lane, const rtfast::Ray& R, float& key,
                                        uint32_t& X, uint32_t& cnt) {
    const float4 lo = tl[(size_t)T * 192u + 3u * lane], hi = tl[(size_t)T * 192u + 3u * lane + 1u];
    key = __int_as_float(0x7f800000);
    cnt = __float_as_uint(hi.w);
    X = __float_as_uint(hi.z);
    if (cnt != TL_EMPTY) {
        float tmin, tmax;
        rtfast::slab_exact(R, lo, hi, &tmin, &tmax);
        if (tmax >= tmin && tmax > 0.0f) key = tmin;
    }
}

struct Frames {  // suspended treelets (LDS): per lane key / X / cnt, per frame the walk state
    float key[TL_FRAMES][64];
    uint32_t x[TL_FRAMES][64], cnt[TL_FRAMES][64];
    uint32_t t[TL_FRAMES], e[TL_FRAMES], cur[TL_FRAMES];
    unsigned long long fz[TL_FRAMES];
};

// A leaf of the walk: the reference's triangle loop over [f0, f0 + c0) (main_raytracing.cu:51-71).
template <int MODE>
__device__ __forceinline__ void lone_leaf(const RenderArgs& a, const float4* tris, uint32_t lane, uint32_t f0, uint32_t c0,
                                          const rtfast::Ray& R, rtfast::Hit& h, uint32_t* scratch, Counters& c) {
    using namespace rtfast;
    if (c0 <= (uint32_t)BIG) {
        float t = 0.0f, x = 0.0f, y = 0.0f;
        bool nan = false, acc = false;
        if (lane < c0) {
            const uint32_t i = f0 + lane;
            acc = tri_accept(R.o, R.nd, tris[3 * i], tris[3 * i + 1], tris[3 * i + 2], h.best, &t, &x, &y, &nan);
        }
        if (__ballot(nan)) {  // the sequential loop, every lane alike (never taken for finite scenes)
            for (uint32_t i = f0; i < f0 + c0; i++) {
                float tt, xx, yy;
                bool dummy = false;
                if (tri_accept(R.o, R.nd, tris[3 * i], tris[3 * i + 1], tris[3 * i + 2], h.best, &tt, &xx, &yy, &dummy))
                    h.best = tt, h.kind = 2, h.bx = xx, h.by = yy, h.id = __float_as_uint(tris[3 * i + 2].y);
            }
        } else if (__ballot(acc)) {
            const uint32_t mk = rtfast::__ockl_wfred_min_u32(acc ? tkey(t) : 0xffffffffu);
            const uint32_t mi = rtfast::__ockl_wfred_min_u32(acc && tkey(t) == mk ? lane : 0xffffffffu);
            h.best = bcast(t, (int)mi), h.bx = bcast(x, (int)mi), h.by = bcast(y, (int)mi), h.kind = 2;
            h.id = __float_as_uint(tris[3 * (f0 + mi) + 2].y);
        }
        return;
    }
    // big leaf: the wave's cooperative round for the one ray (lane 0 holds it, like every lane)
    const float4 lead = tris[3 * (size_t)f0 + 2];
    const uint32_t pf = __float_as_uint(lead.w), po = __float_as_uint(lead.z);
    if ((MODE & 4) && pf == 2u && a.tree && a.flat) {
        Trav T{f0, c0, 0};
        coop_tree<false>(tris, a.tree, a.ltris, a.flat, 1ull, po, R, h, T, scratch, a.tune, c);
    } else if ((pf & 1u) && a.pairs) {  // pf 3: a screen record precedes the pairs (mirror.h)
        coop_leaf(tris, a.pairs + 5 * (size_t)po, 1ull, f0, c0, R, h);
    } else {
        coop_leaf_scalar(tris, 1ull, f0, c0, R, h);
    }
    // the round wrote the result on lane 0: make it uniform again
    h.best = bcast(h.best, 0), h.bx = bcast(h.bx, 0), h.by = bcast(h.by, 0);
    h.kind = __builtin_amdgcn_readlane(h.kind, 0), h.id = bcastu(h.id, 0);
}

// BVHRayHit (main_raytracing.cu:33-81) for the wave's one ray through the treelets; h enters with
// the closest sphere distance and leaves with the reference's closest hit.  Uniform in all lanes.
template <int MODE>
__device__ __forceinline__ void lone_bvh(const RenderArgs& a, const float4* tl, uint32_t lane,
                                         const rtfast::Ray& R, rtfast::Hit& h, Frames& F, uint32_t* scratch,
                                         bool& overflow, Counters& c) {
    using namespace rtfast;
    const float4* nodes4 = reinterpret_cast<const float4*>(a.nodes);
    const float4* tris = reinterpret_cast<const float4*>(a.tris);
    {  // the root, popped first and tested against the sphere distance (main_raytracing.cu:41-47)
        float tmin, tmax;
        slab_exact(R, nodes4[0], nodes4[1], &tmin, &tmax);
        if (!(tmax >= tmin && tmin < h.best && tmax > 0.0f)) return;
    }
    const uint32_t root_cnt = __float_as_uint(nodes4[1].w);
    if (root_cnt > 0u) {  // the root is a leaf
        lone_leaf<MODE>(a, tris, lane, __float_as_uint(nodes4[1].z), root_cnt, R, h, scratch, c);
        return;
    }
    float key;
    uint32_t X, cnt;
    uint32_t T = 0u, e = 0u, cur = 1u;
    unsigned long long fz = 0ull;
    int depth = 0;
    tl_load(tl, T, lane, R, key, X, cnt);
    TLSlot g = tl_geom(tl, T, lane);
    for (;;) {
        const uint32_t esize = (uint32_t)__builtin_amdgcn_readlane((int)g.size, (int)e);
        const unsigned long long in_sub = bits(e + 1u, e + esize);
        const unsigned long long below = bits(0u, cur);
        const unsigned long long live = __ballot(key < h.best);
        const unsigned long long pm = (fz & below) | (live & ~below);
        const bool blocked = (g.anc & in_sub & ~pm) != 0ull;
        const bool is_event = cnt != TL_EMPTY && (cnt > 0u || g.frontier);
        const unsigned long long ev =
            __ballot(((in_sub & ~below & pm) >> lane & 1ull) != 0ull && is_event && !blocked);
        if (!ev) {
            if (depth == 0) break;
            depth--;  // back to the treelet this one hangs from; its walk continues after the frontier
            T = F.t[depth], e = F.e[depth], cur = F.cur[depth], fz = F.fz[depth];
            key = F.key[depth][lane], X = F.x[depth][lane], cnt = F.cnt[depth][lane];
            g = tl_geom(tl, T, lane);
            continue;
        }
        const uint32_t nr = (uint32_t)__ffsll((long long)ev) - 1u;
        fz = (fz & below) | (pm & bits(cur, nr + 1u));  // the decisions up to the event are made
        cur = nr + 1u;
        const uint32_t ex = bcastu(X, (int)nr), ec = bcastu(cnt, (int)nr);
        if (ec == 0u) {
            // a frontier: its subtree is treelet ex (entered at its root, slot 0, which passed)
            if (depth >= TL_FRAMES) {
                overflow = true;
                return;
            }
            F.key[depth][lane] = key, F.x[depth][lane] = X, F.cnt[depth][lane] = cnt;
            F.t[depth] = T, F.e[depth] = e, F.cur[depth] = cur, F.fz[depth] = fz;
            depth++;
            T = ex, e = 0u, cur = 1u, fz = 0ull;
            tl_load(tl, T, lane, R, key, X, cnt);
            g = tl_geom(tl, T, lane);
        } else {
            lone_leaf<MODE>(a, tris, lane, ex, ec, R, h, scratch, c);
        }
    }
}

template <int MODE>
__global__ __launch_bounds__(WAVE) void render_lone_kernel(RenderArgs a, const int32_t* __restrict__ lone_slots,
                                                           int lone_count, const float4* __restrict__ tl) {
    using namespace rtfast;
    __shared__ Frames F;
    __shared__ uint32_t scratch[64];  // coop_tree's cluster compaction
    const uint32_t lane = threadIdx.x;
    if ((int)blockIdx.x >= lone_count) return;
    const long long s = lone_slots[blockIdx.x];
    if (s < 0 || s >= a.slot_count) return;
    const int k = (int)(s >> 8), tid = (int)(s & 255);
    const int tile = shard_tile(a, k);
    int lx, ly;
    tile_pixel(tid, &lx, &ly);
    const int x = (tile % a.tiles_x) * TILE + lx, y = (tile / a.tiles_x) * TILE + ly;
    if (tile < 0 || x >= a.width || y >= a.height) return;
    const size_t slot = (size_t)k * (TILE * TILE) + tid;
    rt_rng_state* rs = a.rng + (a.out_shard ? slot : (size_t)y * a.width + x);
    rtm::Xorwow rng{rs->d, rs->v[0], rs->v[1], rs->v[2], rs->v[3], rs->v[4]};
    const rtm::f3 cam_o = ld3(a.cam.origin), cam_h = ld3(a.cam.horizontal), cam_v = ld3(a.cam.vertical),
                  cam_ll = ld3(a.cam.lower_left_corner);
    const bool scene_fast = a.scene_fast != 0;
    Counters c;
    float acc_r = 0.0f, acc_g = 0.0f, acc_b = 0.0f, acc_a = 0.0f;
    bool overflow = false;
    for (int sample = 0; sample < a.spp; sample++) {
        // main_raytracing.cu:190: uv = (pixel + vec2(rng(), rng())) / vec2(W, H), u drawn first
        const float ru = rng.uniform();
        const float rv = rng.uniform();
        const float uvx = ((float)x + ru) / (float)a.width;
        const float uvy = ((float)y + rv) / (float)a.height;
        rtm::f3 ro = cam_o;  // GPUCamera::GetRay (GPUScene.h:13), not normalized
        rtm::f3 rd = rtm::sub(rtm::add(rtm::add(cam_ll, rtm::muls(cam_h, uvx)), rtm::muls(cam_v, uvy)), cam_o);
        rtm::f3 color = rtm::mk(0, 0, 0), thr = rtm::mk(1, 1, 1);
        for (int bounce = 0; bounce < a.bounces; bounce++) {
            c.seg++;
            // GetRayHit (main_raytracing.cu:83-109): spheres one per lane, strict `<` keeps the first
            const rtm::f3 nd = rtm::normalize(rd);
            Hit h;
            h.best = 1e30f, h.kind = 0, h.id = 0, h.bx = h.by = 0.0f;
            {
                // lane l tests spheres l, l + 64, ... keeping its first strictly closer one (the
                // sequential loop's rule within its own stride); the (distance, index) minimum over
                // the lanes is then the sequential loop's result
                float dist = 1e30f;
                uint32_t idx = 0xffffffffu;
                bool nan = false;
                for (int i = (int)lane; i < a.sphere_count; i += WAVE) {
                    const GeometrySphere& sp = a.spheres[i];
                    float d;
                    if (rtd::intersect_sphere(ro, nd, ld3(sp.position), sp.radius * sp.radius, &d)) {
                        nan = nan || !(d == d);
                        if (d < dist) dist = d, idx = (uint32_t)i;
                    }
                }
                const bool hit = idx != 0xffffffffu;
                if (__ballot(nan)) {  // a NaN distance: the sequential loop
                    for (int i = 0; i < a.sphere_count; i++) {
                        const GeometrySphere& sp = a.spheres[i];
                        float d2;
                        if (rtd::intersect_sphere(ro, nd, ld3(sp.position), sp.radius * sp.radius, &d2)) {
                            if (d2 >= h.best) continue;
                            h.best = d2, h.kind = 1, h.id = (uint32_t)i;
                        }
                    }
                } else {
                    const bool cand = hit && dist < 1e30f;  // dist > eps > 0: its bits order like the value
                    const uint32_t mk = rtfast::__ockl_wfred_min_u32(cand ? __float_as_uint(dist) : 0xffffffffu);
                    if (mk != 0xffffffffu) {
                        const uint32_t mi = rtfast::__ockl_wfred_min_u32(cand && __float_as_uint(dist) == mk ? idx : 0xffffffffu);
                        h.best = __uint_as_float(mk), h.kind = 1, h.id = mi;
                    }
                }
            }
            const Ray R = make_ray(ro, rd, nd, scene_fast);
            lone_bvh<MODE>(a, tl, lane, R, h, F, scratch, overflow, c);
            bool end = shade_segment<false>(a, h, ro, rd, nd, rng, color, thr, c);
            if (bounce + 1 >= a.bounces) end = true;
            if (end) break;
        }
        acc_r += color.x;
        acc_g += color.y;
        acc_b += color.z;
        acc_a += 1.0f;
    }
    if (overflow) __builtin_trap();  // a BVH deeper than the frame stack: rt_render refuses such scenes first
    if (lane == 0) {
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
        if (a.seg_counter) atomicAdd(a.seg_counter, c.seg);
    }
}

}  // namespace

hipError_t launch_lone(const RenderArgs& a, const int32_t* lone_slots, int lone_count, const void* treelets, hipStream_t s) {
    if (lone_count <= 0) return hipSuccess;
    const float4* tl = reinterpret_cast<const float4*>(treelets);
    if (a.tree)
        hipLaunchKernelGGL(render_lone_kernel<5>, dim3(lone_count), dim3(WAVE), 0, s, a, lone_slots, lone_count, tl);
    else
        hipLaunchKernelGGL(render_lone_kernel<1>, dim3(lone_count), dim3(WAVE), 0, s, a, lone_slots, lone_count, tl);
    return hipGetLastError();
}

}  // namespace rtk
