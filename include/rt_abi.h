/*
 * rt_abi.h -- the C-ABI drop-in boundary of the MI355X ray tracer (librt_hip.so).
 *
 * Everything here is plain C: POD structs, raw pointers, sizes, integer status codes.
 * No HIP, torch or C++ types appear in a signature, so the same header serves a C++ host
 * (the reference's Scene.cpp / BVH.cpp / RayTracing.cpp), Python ctypes and any other FFI.
 *
 * Reference interfaces replaced (paths relative to the reference repository root):
 *   raytracing_process ...... RayTracing/main_raytracing.cu:202-220 (declared by the caller
 *                             at RayTracing/RayTracing.cpp:12)
 *   init_rng ................ RayTracing/Random.cu:10-13 (caller RayTracing/RayTracing.cpp:13,220)
 *   rt_malloc / rt_free ..... CUDA::DeviceMemory, utils/CUDAHelper.h:114-156
 *   rt_memcpy_* ............. CUDA_CHECK(cudaMemcpy(...)) at RayTracing/Scene.cpp:195-230 and
 *                             RayTracing/RayTracing.cpp:233
 *   rt_cubemap_* ............ CUDA::Texture + Loader::LoadDDSFromFile,
 *                             utils/CUDATexture.cpp:112-172,187-249
 *   GPU data contract ....... RayTracing/GPUScene.h:11-96, RayTracing/Math.h:25-37
 *
 * Error behaviour: every rt_* function returns 0 on success and a nonzero code on
 * failure, with a message available from rt_last_error().  The two reference entry points
 * keep the reference's void signature; like main_raytracing.cu:215-219 they print a launch
 * failure, and additionally record it for rt_last_error().
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__cplusplus)
#define RT_ALIGNAS(n) alignas(n)
#else
#define RT_ALIGNAS(n) _Alignas(n)
#endif

/* ---------------------------------------------------------------------------------------
 * Data contract.  Field order, sizes and alignment are those of the reference structs
 * (GPUScene.h), so buffers built by the reference's Scene::Upload are consumed unchanged.
 * ------------------------------------------------------------------------------------- */

/* GPUScene.h:11-23.  60 bytes. */
typedef struct GPUCamera {
    float origin[3];
    float viewport_worldspace_size[2];
    float aspect;
    float horizontal[3];
    float vertical[3];
    float lower_left_corner[3];
} GPUCamera;

/* GPUScene.h:25-30.  32 bytes. */
typedef struct GPUVertex {
    RT_ALIGNAS(16) float position[3];
    float normal[3];
    float uv[2];
} GPUVertex;

/* GPUScene.h:32-38.  16 bytes.  NOTE the reference's field order v0, v2, v1: the aggregate
 * initialiser GPUFace{i0, i0+1, i0+2} in Scene::AddTriangle (Scene.cpp:65) therefore lands
 * as v0=i0, v2=i0+1, v1=i0+2, and the kernel reads v1/v2 by name. */
typedef struct GPUFace {
    RT_ALIGNAS(16) uint32_t v0;
    uint32_t v2;
    uint32_t v1;
    uint32_t material;
} GPUFace;

/* GPUScene.h:40-50 + Math.h:25-37 (AABB).  32 bytes.  Leaf iff prim_count > 0; an inner
 * node's children are at first_index and first_index + 1. */
typedef struct GPUBVHNode {
    RT_ALIGNAS(32) float bmin[3];
    float bmax[3];
    uint32_t first_index;
    uint32_t prim_count;
} GPUBVHNode;

/* GPUScene.h:59-64.  32 bytes. */
typedef struct GeometrySphere {
    RT_ALIGNAS(16) float position[3];
    float radius;
    int32_t material;
} GeometrySphere;

/* GPUScene.h:66-74.  64 bytes. */
typedef struct GPUMaterial {
    RT_ALIGNAS(16) float albedo[4];
    float emissive[4];
    float specular[4];
    float roughness;
    float specular_percent;
    float IOR;
} GPUMaterial;

/* GPUScene.h:76-96.  136 bytes.  All pointers are non-owning device pointers.
 * rng_state points at a caller-owned array of rt_rng_state (48 B each, the size of the
 * reference's curandState), one per pixel, indexed y*width + x (GPUScene.h:95).
 * environment_cubemap_tex is a handle from rt_cubemap_create (0 = black sky). */
typedef struct GPUScene {
    const GeometrySphere* gpu_spheres;
    const GPUMaterial* gpu_materials;
    const GPUBVHNode* gpu_bvh_nodes;
    const uint32_t* gpu_bvh_face_indices;
    const GPUVertex* gpu_vertices;
    const GPUFace* gpu_faces;
    int32_t sphere_count;
    int32_t material_count;
    void* rng_state;
    uint64_t environment_cubemap_tex;
    GPUCamera camera;
} GPUScene;

/* Per-pixel XORWOW state.  Same size and the same first 24 bytes as the reference's
 * curandStateXORWOW (d, v[5]); the Box-Muller fields are never used by this path. */
typedef struct rt_rng_state {
    RT_ALIGNAS(8) uint32_t d;
    uint32_t v[5];
    uint32_t unused[6];
} rt_rng_state;

#if defined(__cplusplus)
static_assert(sizeof(GPUCamera) == 60, "GPUCamera");
static_assert(sizeof(GPUVertex) == 32, "GPUVertex");
static_assert(sizeof(GPUFace) == 16 && offsetof(GPUFace, v2) == 4 && offsetof(GPUFace, v1) == 8, "GPUFace");
static_assert(sizeof(GPUBVHNode) == 32 && offsetof(GPUBVHNode, first_index) == 24, "GPUBVHNode");
static_assert(sizeof(GeometrySphere) == 32, "GeometrySphere");
static_assert(sizeof(GPUMaterial) == 64 && offsetof(GPUMaterial, roughness) == 48, "GPUMaterial");
static_assert(sizeof(GPUScene) == 136 && offsetof(GPUScene, sphere_count) == 48 &&
              offsetof(GPUScene, rng_state) == 56 && offsetof(GPUScene, environment_cubemap_tex) == 64 &&
              offsetof(GPUScene, camera) == 72, "GPUScene");
static_assert(sizeof(rt_rng_state) == 48, "rt_rng_state");
#endif

/* ---------------------------------------------------------------------------------------
 * Reference entry points (exact signatures).
 * ------------------------------------------------------------------------------------- */

/* main_raytracing.cu:202.  Renders one progressive frame into the pitched float4 surface:
 * reference constants sample_count = 5 (main_raytracing.cu:166-170, Release) and
 * num_bounces = 6 (:115), on the null stream, asynchronous. */
void raytracing_process(void* surface, void* surface_last_frame, int width, int height, size_t pitch,
                        int frame_index, GPUScene* scene);

/* Random.cu:10.  curand_init(seed, tid, 0) for tid in [0, count*size): XORWOW seeding
 * plus a skip-ahead of tid * 2^67 draws.  Null stream, asynchronous. */
void init_rng(uint32_t thread_block_count, uint32_t thread_block_size, void* rngStates, unsigned int seed);

/* ---------------------------------------------------------------------------------------
 * Extended entry points (runtime parameters the reference hard-codes, streams, shards).
 * ------------------------------------------------------------------------------------- */

typedef struct rt_render_params {
    void* surface;                 /* pitched float4 output (or NULL when out_shard is set) */
    const void* surface_last_frame;/* pitched float4 history, same pitch */
    int32_t width, height;
    uint64_t pitch;                /* bytes per row of both surfaces */
    int32_t frame_index;
    int32_t spp;                   /* reference: 5 (Release) / 1 (Debug) */
    int32_t bounces;               /* reference: 6 */
    int32_t shard_index;           /* tile sharding: this rank renders 16x16 tiles */
    int32_t shard_count;           /*   t = shard_index + k * shard_count (row-major tiles) */
    int32_t flags;                 /* RT_RENDER_* */
    void* out_shard;               /* if non-NULL: compact [k][16*16] float4 shard output */
    uint64_t* stats;               /* RT_RENDER_STATS: RT_STAT_COUNT uint64 counters (zeroed by caller) */
    uint64_t* segment_counter;     /* optional: += ray segments traced (GetRayHit calls) */
    /* Explicit tile list (cost-aware plans, rt_shard_plan): list entry k renders the row-major
     * 16x16 tile tile_list[k] (DEVICE int32 array, tile_count entries, < 0 = padding) instead of
     * the round-robin tile shard_index + k * shard_count.  NULL = round-robin. */
    const int32_t* tile_list;
    int64_t tile_count;
    /* Optional DEVICE uint64 [entries][4]: elapsed ticks of the device's constant 100 MHz clock
     * (s_memrealtime) of each 8x8 sub-tile wave of the production tracer (the cost input of
     * rt_shard_plan). */
    uint64_t* wave_clock;
    uint32_t tune;                 /* diagnostic A/B knobs (tools/); 0 = the production path */
    /* Optional lane map (production tracer only): wave w, lane l renders slot lane_slots[64w + l]
     * (slot k*256 + t = thread t of list entry k, as in the layout rule below; < 0 = idle lane)
     * instead of slot 64w + l.  lane_slot_count (a multiple of 64) sets the number of waves.  Any
     * permutation renders the same pixels bit for bit; rt_lane_plan builds one that isolates the
     * costliest pixels (the serial tail of a strong-scaled frame). */
    const int32_t* lane_slots;
    int64_t lane_slot_count;
    /* Optional DEVICE uint32 [slots]: per-pixel work of the frame, counted deterministically by the
     * timing variant of the production tracer (its own traversal steps + 3 per big-leaf visit + 1
     * per segment; no clock involved) -- the cost input of rt_lane_plan. */
    uint32_t* lane_cost;
    /* With a lane map: the first priority_waves waves (rt_lane_plan's long waves) issue at raised
     * wave priority, so the frame's serial tail does not queue behind the short waves. */
    int64_t priority_waves;
    /* Refill (production tracer; needs librt_hip_exp.so, rt_experimental_loaded): 0 = off.  n in [1, 64]: the launch holds only as many waves as
     * the GPU runs at once; the rest of the lane order (the lane map, or the sub-tile waves) is a
     * queue, and a wave takes the next n entries as soon as n of its lanes have finished their
     * pixels (waves that start less than half full keep their lanes to themselves). */
    int32_t refill_lanes;
    /* Occupancy of the production tracer: 0 = the default (5 waves per SIMD, 96 registers);
     * 6 = 6 waves per SIMD (80 registers, more spills), 7 = 7 (72 registers) -- faster on some
     * scenes (config 2: 16.2 / 15.3 vs 16.9 ms), slower on others (config 4: 95 vs 90 ms at 6);
     * bench.py picks it per configuration by timing one untimed probe frame of each.  1-4 = the
     * 5-wave build with its residency capped at that many waves per SIMD by dynamic LDS (each
     * wave reserves 160 KB / (4 x cap) of its CU's LDS): fewer co-resident waves for the
     * latency-bound long waves of a strong-scaled shard.  Any other value is an error. */
    int32_t waves_per_simd;
    /* Lone pixels (production tracer; rt_lone.hip, needs librt_hip_exp.so): DEVICE int32 slots (the
     * lane_slots numbering) that the lone-pixel kernel renders one per wave -- all 64 lanes on the
     * pixel's one ray, the BVH read as treelets -- concurrently with the production kernel on a second
     * stream joined back into `stream`.  Requires lane_slots, which must not hold these slots
     * (rt_lone_plan picks them and marks them for rt_lane_plan): a slot in both lists is rendered twice
     * at the same time into the same RNG state and pixel -- UNDEFINED results.  RT_RENDER_VALIDATE
     * checks this (and slot ranges) before launching.  Bit-identical pixels either way; it shortens
     * the chains of a strong-scaled frame's costliest pixels.  lone_count 0 = none. */
    const int32_t* lone_slots;
    int64_t lone_count;
} rt_render_params;

/* Layout rule: with out_shard set, RNG state s and output s are compact in list order
 * (state/slot k*256 + t for thread t of list entry k); without it, RNG states are indexed
 * y*width + x (the reference's layout) and the output goes to the pitched surface, whatever the
 * tile order. */

#define RT_RENDER_STATS 1          /* count traversal work (slower kernel variant) */
#define RT_RENDER_TRACER_REF 2     /* force the reference-layout tracer (A/B, tests) */
#define RT_RENDER_TRACER_FLAT 4    /* force the exact-division flat tracer (A/B, tests) */
#define RT_RENDER_TRACER_WAVEFRONT 8 /* wavefront tracer (needs librt_hip_exp.so): a shade launch and a
                                        persistent trace launch per segment generation, rays refilled
                                        lane by lane (same results; rt_scene_upload scenes, no
                                        statistics / lane_cost / wave_clock / refill / lone frames) */
#define RT_RENDER_VALIDATE 16      /* debug: before launching, check on the device that lone_slots and
                                      lane_slots are disjoint (synchronises; an error if they are not) */

enum {
    RT_STAT_SEGMENTS = 0,   /* GetRayHit calls */
    RT_STAT_NODES = 1,      /* BVH nodes popped (AABB tests) */
    RT_STAT_TRI_TESTS = 2,  /* ray/triangle tests */
    RT_STAT_TRI_ACCEPTS = 3,/* triangle hits accepted as the new closest */
    RT_STAT_SPHERE_ACCEPTS = 4,
    RT_STAT_HITS = 5,       /* segments that hit something */
    RT_STAT_MISSES = 6,     /* segments that sampled the sky */
    /* SIMD-efficiency counters of the fast kernel (wave-level iterations, active lanes) */
    RT_STAT_WAVE_SMALL_ITERS = 8,   /* traversal steps (inner nodes / small leaves) */
    RT_STAT_LANE_SMALL = 9,
    RT_STAT_WAVE_BIG_TRIS = 10,     /* big-leaf triangle iterations */
    RT_STAT_LANE_BIG_TRIS = 11,
    RT_STAT_WAVE_SEGMENT_ITERS = 12,/* segment-loop iterations */
    RT_STAT_LANE_SEGMENTS = 13,
    RT_STAT_TREE_NODES = 14,        /* leaf-tree nodes visited (leaftree.h; statistics frames with RT_TUNE bit 7) */
    RT_STAT_TREE_TRI_TESTS = 15,    /* triangle tests run inside leaf trees */
    RT_STAT_CYCLES_SMALL = 16,      /* RT_TUNE bit 8 timing frames: wave clock cycles in small steps */
    RT_STAT_CYCLES_BIG = 17,        /* ... in big-leaf rounds */
    RT_STAT_CYCLES_TOTAL = 18,      /* ... in the whole kernel */
    RT_STAT_ROUNDS_COOP = 19,       /* cooperative big-leaf rounds */
    RT_STAT_ROUNDS_SHARED = 20,     /* shared-leaf (pair / scalar-load) rounds */
    RT_STAT_COOP_RAYS = 21,         /* rays run through cooperative rounds */
    RT_STAT_CYCLES_TREE_CUT = 7,    /* timing frames, cooperative leaf-tree walk: whole walk (all rounds) */
    RT_STAT_CYCLES_TREE_CLUSTERS = 22, /* ... cluster screening rounds */
    RT_STAT_CYCLES_TREE_TRIS = 23,  /* ... triangle rounds */
    /* timing frames: the production kernel's own big-leaf work with twin records (mirror.h quads / units) */
    RT_STAT_BIG_TESTS = 24,         /* glm tests of a big leaf's unit triangles (quad halves, units), summed over rays */
    RT_STAT_TWIN_DECIDED = 25,      /* twins rejected from their partner's values without a test (rt_fast.h twin_rejected) */
    RT_STAT_TWIN_TESTS = 26,        /* twins tested themselves (too close to call, or a hit) */
    RT_STAT_WAVE_BIG_ITERS = 27,    /* wave iterations of those tests (shared-leaf quads, cooperative unit chunks) */
    /* timing frames of the leaf-tree kernels: deferred big leaves (rt_fast.h defer_leaf) */
    RT_STAT_DEFER_END2 = 28,        /* guard walks (END2: the leaf re-run up to tmin of the hit's own leaf) */
    RT_STAT_DEFER_REDO = 29,        /* lanes redone from the root after END2 found a hit */
    RT_STAT_COUNT = 32
};

/* Render on `stream` (a hipStream_t, NULL = null stream).  Returns 0 or an error code.
 * A GPUScene filled by another host (the reference's own Scene::Upload) is rendered without any
 * host synchronisation: each frame's arrays are fingerprinted on the device, and the frame runs the
 * production tracer when a private mirror built from exactly those arrays is installed, the
 * reference-layout tracer otherwise, while a worker thread (re)builds the mirror in the background. */
int rt_render(const rt_render_params* params, const GPUScene* scene, void* stream);
/* Foreign scenes: block until the background mirror build started by the last rt_render of this
 * scene has finished (the next rt_render installs it).  For tests and benchmarks; 0 or an error. */
int rt_foreign_mirror_wait(const GPUScene* scene);
/* Foreign scenes, for tests: the tracer of the last frame -- 1 production (mirror matched the
 * frame's fingerprint), 0 reference layout (mismatch), -1 no mirror installed yet.  Synchronises. */
int rt_foreign_last_tracer(const GPUScene* scene);

/* 1 when librt_hip_exp.so is loaded: its constructor registers the exact alternatives kept for A/B
 * measurement (wavefront tracer, refill, lone-pixel kernel, RT_TUNE A/B kernel variants) with this
 * library; rt_render refuses frames that ask for them otherwise.  0 otherwise. */
int rt_experimental_loaded(void);

/* init_rng for the pixels of one shard: state index s of shard (shard_index, shard_count)
 * of a width x height frame gets curand_init(seed, pixel_id(s), 0).  With shard_count == 1
 * the states are in y*width + x order (reference layout); otherwise they are compact in the
 * shard's tile order.  Returns 0 or an error code. */
int rt_init_rng(void* rng_states, int width, int height, int shard_index, int shard_count, uint32_t seed,
                void* stream);

/* Number of pixels of a shard (tiles of 16x16, partial edge tiles counted as rendered
 * pixels of the tile: the compact shard always holds whole tiles). */
int64_t rt_shard_tiles(int width, int height, int shard_index, int shard_count);

/* Un-permute gathered compact shards [shard_count][tiles_per_shard_max][256] float4 into a
 * pitched surface.  Returns 0 or an error code. */
int rt_unshard(void* surface, uint64_t pitch, int width, int height, int shard_count, const void* shards,
               int64_t tiles_per_shard_max, void* stream);

/* ---------------------------------------------------------------------------------------
 * Multi-GPU split (the reference renders one frame on one device,
 * RayTracing/RayTracing.cpp:205-234).  Plans deal 16x16 tiles to ranks; each rank renders a
 * compact shard; one gather per frame; the root un-permutes.
 * ------------------------------------------------------------------------------------- */
/* Entries per rank a plan may use (the row length of tile_lists below). */
int64_t rt_shard_plan_capacity(int width, int height, int shard_count);
/* Fill HOST tile_lists [shard_count][capacity] (-1 padded) and counts [shard_count].
 * tile_cost (HOST, one per row-major tile) NULL = round-robin (rank r: tiles r, r+N, ...);
 * otherwise longest-processing-time-first: heaviest tile first, each to the least-loaded rank
 * below capacity; every rank's list comes out heaviest first.  Deterministic.  0 or error. */
int rt_shard_plan(int width, int height, int shard_count, const double* tile_cost, int64_t capacity,
                  int32_t* tile_lists, int64_t* counts);
/* Lane plans (rt_render_params.lane_slots; shard.cpp).  Entries a plan for `slots` slots (a
 * multiple of 64: 256 per list entry) may use. */
int64_t rt_lane_plan_capacity(int64_t slots);
/* Fill HOST lane_slots from HOST per-slot work `cost` (rt_render_params.lane_cost of a probe
 * frame of the same list, zero for slots without a pixel).  A wave's time is modelled as
 * max c x (sum c / max c)^0.34 work units; every 8x8 sub-tile wave above the target
 * slack x max(max c, sum c / parallel_units) is split (first fit, heaviest pixels first) into
 * sub-waves within it.  Waves of at least half the target go first, longest first; the rest keep
 * list order.  Slots whose cost is UINT32_MAX (rt_lone_plan's lone pixels) are left out of the map.  parallel_units <= 0: the identity map.  MI355X: 48000 (bench.py --lane-units; measured
 * best for configs 2 and 3 at N = 2-8).
 * *long_waves (optional) receives the number of those leading waves (rt_render_params.
 * priority_waves).  Returns the entries written (a multiple of 64), or -1 on bad arguments. */
int64_t rt_lane_plan(const uint32_t* cost, int64_t slots, double parallel_units, double slack,
                     int32_t* lane_slots, int64_t capacity, int64_t* long_waves);
/* Measured refinement of a HOST lane map of `entries` entries over `slots` slots: with wave_ticks
 * [entries / 64] the per-wave clocks of a timing frame of that map (rt_render_params.wave_clock),
 * every wave of more than one pixel whose clock is at least theta (0 < theta <= 1) x the longest is
 * split in two (its pixels in decreasing `cost` dealt alternately), and all waves are written to
 * HOST `out` (capacity >= 2 * entries) ordered by expected duration, longest first.  A map is a
 * permutation of the slots, so the frame is bit-identical; the caller keeps the refined map only if
 * a timed frame of it is faster (bench.py refine_lane_map).  *split_waves (optional) receives the
 * number of waves made by splitting.  Returns the entries written, or -1 on bad arguments. */
int64_t rt_lane_refine(const int32_t* lane_slots, int64_t entries, const uint32_t* cost, int64_t slots,
                       const int64_t* wave_ticks, double theta, int32_t* out, int64_t capacity, int64_t* split_waves);
/* Lone-pixel plans: write to HOST lone_slots (up to max_lone entries) the slots whose probe work
 * `cost` is at least min_cost, heaviest first (ties: lower slot first), and mark each of them in
 * `cost` with UINT32_MAX -- the value rt_lane_plan treats as "not in this map".  Returns the number
 * written, or -1 on bad arguments. */
int64_t rt_lone_plan(uint32_t* cost, int64_t slots, int64_t max_lone, uint32_t min_cost, int32_t* lone_slots);
/* rt_init_rng for an explicit tile list (DEVICE int32): state k*256 + t <- curand_init(seed,
 * pixel id of thread t of tile tile_list[k]). */
int rt_init_rng_tiles(void* rng_states, int width, int height, const int32_t* tile_list, int64_t tile_count,
                      uint32_t seed, void* stream);
/* rt_unshard with explicit plans: tile_lists is the DEVICE copy of rt_shard_plan's output. */
int rt_unshard_tiles(void* surface, uint64_t pitch, int width, int height, int shard_count, const void* shards,
                     int64_t tiles_per_shard_max, const int32_t* tile_lists, void* stream);

/* RCCL communicator for the frame-end gather (csrc/comm.hip).  One process per GPU: rank 0 makes
 * an id, the host passes it to every rank by its own means, each rank calls rt_comm_init_rank on
 * its current device.  One process driving N devices: rt_comm_init_all. */
#define RT_COMM_ID_BYTES 128
typedef struct rt_comm rt_comm;
int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]);
int rt_comm_init_rank(rt_comm** comm, int nranks, int rank, const uint8_t id[RT_COMM_ID_BYTES]);
int rt_comm_init_all(rt_comm** comms, int ndev, const int* devices);
int rt_comm_destroy(rt_comm* comm);
int rt_comm_rank(const rt_comm* comm);
int rt_comm_size(const rt_comm* comm);
/* Bracket the per-device gathers of a one-process, N-device host (RCCL group semantics). */
int rt_comm_group_start(void);
int rt_comm_group_end(void);
/* The frame's gather on `stream`: every rank passes its shard (shard_bytes); the root receives
 * rank r's bytes at gathered + r * stride (recv_bytes[r] bytes, or shard_bytes for every rank
 * when recv_bytes is NULL; the root's own shard is copied on the stream).  Asynchronous. */
int rt_gather_shards(rt_comm* comm, const void* shard, size_t shard_bytes, void* gathered, size_t stride,
                     const size_t* recv_bytes, int root, void* stream);

/* ---------------------------------------------------------------------------------------
 * Frame output (the viewer path: main.cpp:66-94 draws the surface with exposure 0.5 + ACES film
 * into an sRGB back buffer, main.cpp:438).  For looking at frames; not on the render path.
 * ------------------------------------------------------------------------------------- */
/* Tonemap a pitched float4 surface into width*height*3 bytes of DEVICE memory, rows top to
 * bottom (display order): sRGB8(ACESFilm(0.5 * rgb)), IEC sRGB encode.  Returns 0 or nonzero. */
int rt_tonemap_srgb8(const void* surface, uint64_t pitch, int width, int height, uint8_t* out_rgb, void* stream);
/* Host files: PFM of a HOST copy of the surface (linear RGB, rows bottom to top as PFM
 * stores them = the surface's row order), and binary PPM of top-to-bottom RGB8 rows. */
int rt_write_pfm(const char* path, const float* rgba, uint64_t pitch, int width, int height);
int rt_write_ppm(const char* path, const uint8_t* rgb, int width, int height);

/* ---------------------------------------------------------------------------------------
 * Device memory / texture shim (replaces utils/CUDAHelper.h and utils/CUDATexture.*).
 * ------------------------------------------------------------------------------------- */
int rt_set_device(int device);
/* Visible HIP devices (0 when none or on error). */
int rt_device_count(void);
int rt_malloc(void** ptr, size_t bytes);
int rt_malloc_pitch(void** ptr, size_t* pitch, size_t width_bytes, size_t height);
int rt_free(void* ptr);
int rt_memcpy_h2d(void* dst, const void* src, size_t bytes);
int rt_memcpy_d2h(void* dst, const void* src, size_t bytes);
int rt_memcpy_d2d(void* dst, const void* src, size_t bytes);
int rt_memset(void* dst, int value, size_t bytes);
int rt_synchronize(void);
const char* rt_last_error(void);

/* Cube map from level-0 fp32 RGBA faces [6][size][size][4] (host memory), face order
 * +X,-X,+Y,-Y,+Z,-Z.  Sampled in software (bilinear, seamless).  Returns 0 on failure. */
uint64_t rt_cubemap_create(const float* rgba_level0, int size);
int rt_cubemap_destroy(uint64_t handle);

/* ---------------------------------------------------------------------------------------
 * Host scene (C++ mirror of RayTracing::Scene / BVH / Camera, RayTracing/Scene.{h,cpp},
 * RayTracing/BVH.{h,cpp}) exposed for non-C++ hosts.  rt_scene is opaque.
 * ------------------------------------------------------------------------------------- */
typedef struct rt_scene rt_scene;

rt_scene* rt_scene_create(void);
void rt_scene_destroy(rt_scene* scene);
uint32_t rt_scene_add_material(rt_scene* scene, const GPUMaterial* material);
void rt_scene_add_triangle(rt_scene* scene, const float a[3], const float b[3], const float c[3], int material);
void rt_scene_add_quad(rt_scene* scene, const float a[3], const float b[3], const float c[3], const float d[3],
                       int material);
void rt_scene_add_sphere(rt_scene* scene, const float position[3], float radius, int material);
/* Scene::AddLoadedScene with a mesh file -- a Wavefront .obj (imported like the reference's
 * assimp post-processing, objload.cpp) or a mesh asset (assets/bunny_mesh.bin format) -- and a
 * column-major 4x4 transform.  Returns 0 or an error code.
 * PARITY NOTE: a scene built from an .obj is NOT a parity scene.  Positions, vertex order and
 * faces are bit-identical to an assimp 3.3 import, but the smoothed normals differ from it in
 * the last ulps (assimp's summation order over coincident corners follows its SpatialSort's
 * unstable sort, and the reference pins no assimp version: vcpkg.json:4-7), so frames rendered
 * from it can diverge from the reference's.  The parity scenes (rt_scene_setup, the tests and
 * the benchmark) load the mesh asset, which holds the assimp 3.3 import verbatim. */
int rt_scene_add_mesh_file(rt_scene* scene, const char* path, const float transform[16], int material);
/* Environment cube map from an asset (assets/sunset_cube128.bin) or a legacy fp32 DDS. */
int rt_scene_set_environment_file(rt_scene* scene, const char* path);
/* Host view of the scene's level-0 cube texels [6][size][size][4] (NULL / 0 when none). */
int rt_scene_environment(const rt_scene* scene, const float** texels, int* size);
void rt_scene_set_camera(rt_scene* scene, const float position[3], float angle_x_deg, float angle_y_deg);
void rt_scene_set_viewport(rt_scene* scene, int width, int height);
/* Scene::Upload: builds the BVH when dirty, uploads dirty buffers, fills the GPUScene. */
int rt_scene_upload(rt_scene* scene, void* rng_state);
const GPUScene* rt_scene_gpu(const rt_scene* scene);
/* The host half of Scene::Upload without any device work: camera basis + BVH build. */
void rt_scene_build(rt_scene* scene);
/* The camera basis as of the last build/upload. */
void rt_scene_camera(const rt_scene* scene, GPUCamera* out);
/* CUDARayTracer::SetupCornellBox + SetupStanfordBunny (RayTracing.cpp:79-203, 33-69);
 * which = 0: Cornell box + bunny (configs 1-3), 1: 4x bunny (config 4), 2: 1M-tri plane
 * (config 5). */
int rt_scene_setup(rt_scene* scene, int which, const char* assets_dir);
/* Config-5 scene with an n x n quad grid (n = 708 for the benchmark). */
int rt_scene_setup_plane(rt_scene* scene, int n, const char* assets_dir);
/* Host views of the scene arrays (valid until the next modification). */
size_t rt_scene_host_arrays(const rt_scene* scene, const GPUBVHNode** nodes, size_t* node_count,
                            const uint32_t** face_indices, size_t* face_count, const GPUVertex** vertices,
                            size_t* vertex_count, const GPUFace** faces);
int rt_scene_bvh_max_depth(const rt_scene* scene);

/* Build options (process-wide; affect later rt_scene_upload / mirror builds and
 * rt_bvh_build_device calls).  None of them changes a rendered bit -- the leaf trees and the GPU
 * BVH builder are exact -- only speed; they replace environment knobs so that nothing in the
 * shipped path reads the environment.  rt_get_build_options fills the current values (defaults
 * on first use); rt_set_build_options(NULL) restores the defaults. */
typedef struct rt_build_options {
    uint32_t leaf_tree_min;   /* leaves with at least this many triangles get a leaf tree (1024) */
    uint32_t cut_clusters;    /* leaf trees: clusters per subtree of the flat cut, 1..32 (32) */
    uint32_t cluster_max;     /* leaf trees: triangles per tree leaf, 1..16 (16) */
    float split_angle;        /* leaf trees: split by normals while the cone half-angle exceeds this, rad (0.03) */
    uint32_t bvh_small;       /* GPU BVH builder: nodes this small build their subtree in one thread, 2..64 (16) */
    int32_t host_bvh;         /* 1: rt_scene_upload always builds the BVH on the host (0: GPU from 65,536 faces) */
    int32_t leaf_screens;     /* 1: big leaves whose core can be culled get a screen record (mirror.h pf = 3),
                                 rendered by the screen variants of librt_hip_exp.so (A/B, measured slower) (0) */
} rt_build_options;
void rt_get_build_options(rt_build_options* out);
int rt_set_build_options(const rt_build_options* options);  /* 0, or an error for out-of-range values */

/* The reference's BVH builder (BVH::Calculate, RayTracing/BVH.cpp:8-124) run on the GPU over
 * device arrays: nodes and face indices byte-identical to the host builder (depth-first node
 * numbering, the swap partition's permutation including failed axes).  nodes_out holds
 * 2 * face_count - 1 nodes; *node_count_out receives nodes_used, *max_depth_out the deepest level.
 * Vertex positions must be finite.  Synchronises `stream`.  Returns 0 or an error code. */
int rt_bvh_build_device(const GPUVertex* vertices, uint32_t vertex_count, const GPUFace* faces, uint32_t face_count,
                        GPUBVHNode* nodes_out, uint32_t* face_indices_out, uint32_t* node_count_out,
                        int* max_depth_out, void* stream);

/* Diagnostics for the tests: the kernel's private triangle mirror (cuda-raytracing_amd/csrc/
   mirror.h: leaf-ordered records, 12 floats; leaf-tree nodes, 16 floats; leaf-tree triangle
   records, 12 floats) built on the host from the scene's host arrays, and the render kernel's
   leaf-tree cull predicate (rt_fast.h cluster_cull) evaluated on the host by the same code.
   Returns 0 (cull: 1 = culled), or -1 with rt_last_error(). */
int rt_scene_mirror_info(rt_scene* scene, size_t* tri_records, size_t* tree_nodes, size_t* tree_tri_records);
int rt_scene_mirror_copy(rt_scene* scene, float* tris, float* tree, float* tree_tris);
int rt_cluster_cull_host(const float origin[3], const float nd[3], float best, const float node[16]);
/* The twin test of the big-leaf quads (rt_fast.h twin_rejected, mirror.h quads) on the host: bit 0
   the twin of triangle record `rec` (v0, e2, e1) is proven rejected from rec's own glm values for the
   ray (origin, nd), bit 1 the twin passes glm's predicate, bit 2 rec does.  For tests. */
int rt_twin_check_host(const float rec[12], const float origin[3], const float nd[3]);
/* The traversal's private node array (mirror.h nodes: GPUBVHNode records, sibling pairs 64-B
   aligned in right-first pre-order), built on the host: *count receives the node count; nodes (may
   be NULL) receives the records.  0 or -1 with rt_last_error(). */
int rt_scene_mirror_nodes(rt_scene* scene, GPUBVHNode* nodes, size_t* count);
/* The big leaves' twin records (mirror.h quads: 28 floats each, units: 16 floats each), built on the
   host: counts first, then the arrays when the pointers are not NULL.  0 or -1. */
int rt_scene_mirror_twins(rt_scene* scene, float* quads, size_t* quad_count, float* units, size_t* unit_count);
/* Scenes with big leaves: the leaf of every face (mirror.h face_leaf: the private node index, 0xffffffff
   in no leaf, 0xfffffffe in two), which the deferred leaves' guard reads (rt_fast.h).  *count receives
   the face count (0 for scenes without big leaves); leaf (may be NULL) the table.  0 or -1. */
int rt_scene_mirror_face_leaf(rt_scene* scene, uint32_t* leaf, size_t* count);

/* Test hook: the private mirror built on the host from raw reference arrays (the foreign-scene path,
   rt_render on a GPUScene not uploaded by rt_scene_upload): words 10-11 of every leaf-ordered record --
   a big leaf's first record (first pair, kind), second and third (its twin quads, its units) -- as
   2 x index_count uint32 in `meta`, and whether twin records were built (0 when big-leaf ranges overlap
   so that their metadata records would collide).  0 or -1 (rt_last_error). */
int rt_mirror_build_check(const GPUBVHNode* nodes, size_t node_count, const uint32_t* face_indices, size_t index_count,
                          const GPUFace* faces, size_t face_count, const GPUVertex* vertices, size_t vertex_count,
                          uint32_t* meta, int* twins);

/* XORWOW jump matrix A^(4^k * 2^67) (k < 32) as 800 uint32 words in rocrand's layout
 * m[i*160 + j*5 + w] (input word i, bit j, output word w).  For tests. */
int rt_xorwow_jump_matrix(int k, uint32_t out[800]);
/* Host-side curand_init(seed, subsequence, 0) for tests. */
void rt_xorwow_init_host(uint32_t seed, uint64_t subsequence, rt_rng_state* out);

#ifdef __cplusplus
}
#endif

#endif /* RT_ABI_H */
