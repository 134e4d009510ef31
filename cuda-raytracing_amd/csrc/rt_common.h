// rt_common.h -- types shared by the render kernels (rt_kernel.hip, rt_wave.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "rt_abi.h"
#include "rt_math.h"

namespace rtk {

constexpr int TILE = 16;   // shard / tile granularity (16x16 pixels)
constexpr int BLOCK = 256; // threads of the tile-shaped helper kernels
constexpr int WAVE = 64;

// Leaf-ordered triangle record (product-side mirror of the reference arrays, built by
// Scene::Upload): A = (v0.xyz, e1.x), B = (e1.yz, e2.xy), C = (e2.z, face id, 0, 0) with
// e1 = v1 - v0 and e2 = v2 - v0 computed exactly as glm::intersectRayTriangle does
// (gtx/intersect.inl:37-38), so the test below is bit-identical to the reference's.
struct FlatTri {
    float4 a, b, c;
};

struct RenderArgs {
    const GeometrySphere* spheres;
    const GPUMaterial* materials;
    const GPUBVHNode* nodes;  // traversal kernels: the mirror's private node array (mirror.h); reference tracers: the scene's
    const uint32_t* face_indices;
    const GPUVertex* vertices;
    const GPUFace* faces;
    const FlatTri* tris;  // null -> reference-layout tracer
    rt_rng_state* rng;
    const float* sky;  // float4 [6][n][n] or null
    int sky_n;
    int sphere_count;
    GPUCamera cam;
    float qw, qx, qy, qz;  // quat(vec3(0, PI, 0)) for the sky lookup (main_raytracing.cu:151)
    char* surface;
    const char* last;
    float4* out_shard;
    uint64_t pitch;
    int width, height, frame_index, spp, bounces;
    int shard_index, shard_count, tiles_x;
    const int32_t* tile_list;        // tile of list entry k (rt_render_params.tile_list) or null: round-robin
    unsigned long long* wave_clock;  // per-wave elapsed clock ticks, [list entry][4 sub-tiles] (or [wave] with a lane map), or null
    const int32_t* lane_slots;       // lane map: wave w lane l renders slot lane_slots[64w + l] (< 0 idle), or null
    long long slot_count;            // slots of the launch's list (tiles x 256): larger map entries are idle lanes
    long long entry_count;           // entries of the lane order (lane map length, or slot_count)
    unsigned long long* queue_head;  // refill: entries taken from the queue so far (zeroed per launch), or null
    int refill_lanes;                // refill: idle lanes that trigger a refill
    int waves_per_simd;              // production tracer occupancy: 5 (default) or 6
    uint32_t* lane_cost;             // per-slot work of a probe frame (timing kernel), or null
    int priority_waves;              // lane map: waves below this index run at raised priority
    const int* gate;                 // foreign scenes: the kernel runs only if *gate == gate_value
    int gate_value;
    unsigned long long* stats;
    unsigned long long* seg_counter;
    int scene_fast;  // all node bounds inside the filtered-slab range (rt_fast.h)
    int screens;     // the mirror has big-leaf screen records (mirror.h pf = 3; rt_fast.h screen_leaf)
    const float4* pairs;  // big leaves' triangles in packed pairs (mirror.h) or null
    const float4* quads;  // big leaves' triangles by twins, two triangles a record (mirror.h quads) or null
    const float4* units;  // ... one triangle a record (mirror.h units)
    const float4* tree;   // leaf trees of huge leaves (leaftree.h) or null
    const float4* ltris;  // their triangle records
    const float4* spairs; // small leaves' triangles in packed pairs, pair (i, i+1) at record i, or null
    const float4* flat;   // leaf trees' flat cluster / cut lists (leaftree.h) or null
    const uint32_t* face_leaf;  // scenes with leaf trees: each face's leaf (mirror.h MirrorHost::face_leaf) or null
    // Diagnostic A/B knobs (rt_render_params.tune; 0 = the production path, every setting exact):
    //   bit 0 no cooperative leaf rounds, 1 no pair records, 2 no leaf trees, 3 no small-leaf pairs,
    //   4-5 big-leaf mode (launch_fast_t), 7 statistics through the leaf trees, 8 timing frame (phase
    //   clocks), 9-10 occupancy override (1 compiler's choice, 2 = 6, 3 = 7 waves per SIMD),
    //   11 per-wave clock records, 12 no split small steps, 13-15 split threshold, 16-19 XCD run
    //   length (xcd_block), 20 no twin quads, 21-23 twin rounds' cooperative weight, 24 no deferred leaf trees, 26 no lone-ray traversal, 27 the reference's node array instead of the
    //   mirror's private one (rt_kernel.hip), 28 no big-leaf screens, 30 per-lane leaf-tree walk,
    //   31 subtree order.
    uint32_t tune;
};

struct Counters {
    unsigned long long seg = 0, node = 0, tri = 0, tacc = 0, sacc = 0, hit = 0, miss = 0;
    unsigned long long w_small = 0, l_small = 0, w_big = 0, l_big = 0, w_seg = 0, l_seg = 0;
    unsigned long long ktest = 0, ktri = 0;  // leaf-tree node visits / triangle tests
    unsigned long long cy_small = 0, cy_big = 0, r_coop = 0, r_shared = 0, coop_rays = 0, w_iter = 0;  // timing
    unsigned long long cy_tcl = 0, cy_ttri = 0, cy_tree = 0;  // timing: leaf-tree cluster / triangle rounds, whole walk
    uint32_t lane_work = 0;  // timing: this lane's own traversal steps (+3 per big leaf), rt_render_params.lane_cost
    unsigned long long big_tests = 0, tw_test = 0, tw_dec = 0, big_iters = 0;  // timing: big-leaf work by twins
    uint32_t end2 = 0, redo = 0;  // timing: this lane's deferral guard walks and redos (rt_fast.h trace)
};

__device__ __forceinline__ rtm::f3 ld3(const float* p) { return rtm::f3{p[0], p[1], p[2]}; }

// Tile rendered by list entry k of a shard: an explicit tile list (cost-ordered plans,
// rt_shard_plan) or the round-robin deal t = shard_index + k * shard_count.  Entries < 0 are
// padding (no pixels).
__device__ __forceinline__ int shard_tile(const RenderArgs& a, int k) {
    const int t = a.tile_list ? a.tile_list[k] : a.shard_index + k * a.shard_count;
    return (t >= 0 && t < a.tiles_x * ((a.height + TILE - 1) / TILE)) ? t : -1;  // out of the frame: no pixels
}

// Tile-local pixel of tile-thread `tid` (0..255): wave w covers the 8x8 sub-tile
// ((w&1)*8, (w>>1)*8), lane l the pixel (l&7, l>>3) of it.  The compact shard layout and
// unshard_kernel use the same map.
__device__ __forceinline__ void tile_pixel(int tid, int* lx, int* ly) {
    const int w = tid >> 6, l = tid & 63;
    *lx = (w & 1) * 8 + (l & 7);
    *ly = (w >> 1) * 8 + (l >> 3);
}

}  // namespace rtk
