// rt_kernel.hip -- MI355X (gfx950) render path behind the C-ABI of include/rt_abi.h: the memory /
// cube-map shim, rt_render (argument checks, foreign-scene gating, the choice of kernel variant),
// the RNG set-up and the multi-GPU unshard.
//
// Kernels here
//   init_rng_kernel              curand_init(seed, pixel, 0) with GF(2) jump matrices.
//   unshard_kernel               scatter gathered tile shards back into a pitched surface.
//   fingerprint_kernel (+ gate)  content fingerprint of a foreign scene's arrays, per frame.
// The render kernels live in their own translation units (rt_render.h): rt_fast_*.hip (the
// production tracer, rt_fast_body.h + rt_fast.h, per variant family) and rt_ref.hip (the
// reference-layout and flat tracers).
//
// Numerics: compiled with -ffp-contract=off and IEEE fp32 division/sqrt, so every value
// matches the CPU oracle bit for bit ("Parity").
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>
#include <map>
#include <atomic>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include "rt_abi.h"
#include "rt_device.h"
#include "rt_math.h"
#include "xorwow.h"
#include "rt_common.h"
#include "leaftree.h"
#include "rt_fast.h"

#include "mirror.h"

static_assert(MIRROR_BIG_LEAF == (uint32_t)rtfast::BIG, "pair records exist for exactly the big leaves");

// ---------------------------------------------------------------------------------------
// error state
// ---------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

static int set_error(const std::string& msg, int code = 1) {
    g_last_error = msg;
    return code;
}
static int check(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    return set_error(std::string(what) + ": " + hipGetErrorString(e), (int)e);
}

extern "C" const char* rt_last_error(void) { return g_last_error.c_str(); }

// Bytes of the device allocation holding p from p to its end (0 if p is not device memory).
static size_t bytes_from(const void* p) {
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (!p || hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) != hipSuccess) return 0;
    return size - (size_t)((const char*)p - (const char*)base);
}

void rt_internal_set_error(const char* msg) { set_error(msg); }

// ---------------------------------------------------------------------------------------
// memory shim (utils/CUDAHelper.h:114-156)
// ---------------------------------------------------------------------------------------
extern "C" int rt_set_device(int device) { return check(hipSetDevice(device), "hipSetDevice"); }
extern "C" int rt_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}
extern "C" int rt_malloc(void** ptr, size_t bytes) { return check(hipMalloc(ptr, bytes), "hipMalloc"); }
extern "C" int rt_malloc_pitch(void** ptr, size_t* pitch, size_t width_bytes, size_t height) {
    return check(hipMallocPitch(ptr, pitch, width_bytes, height), "hipMallocPitch");
}
extern "C" int rt_free(void* ptr) { return check(hipFree(ptr), "hipFree"); }
extern "C" int rt_memcpy_h2d(void* dst, const void* src, size_t n) {
    return check(hipMemcpy(dst, src, n, hipMemcpyHostToDevice), "hipMemcpy H2D");
}
extern "C" int rt_memcpy_d2h(void* dst, const void* src, size_t n) {
    return check(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost), "hipMemcpy D2H");
}
extern "C" int rt_memcpy_d2d(void* dst, const void* src, size_t n) {
    return check(hipMemcpy(dst, src, n, hipMemcpyDeviceToDevice), "hipMemcpy D2D");
}
extern "C" int rt_memset(void* dst, int value, size_t n) { return check(hipMemset(dst, value, n), "hipMemset"); }
extern "C" int rt_synchronize(void) { return check(hipDeviceSynchronize(), "hipDeviceSynchronize"); }

// ---------------------------------------------------------------------------------------
// cube maps (utils/CUDATexture.cpp): a handle is the device address of float4[6][n][n]
// ---------------------------------------------------------------------------------------
static std::mutex g_cube_mutex;
static std::map<uint64_t, int> g_cube_size;

extern "C" uint64_t rt_cubemap_create(const float* rgba, int size) {
    if (!rgba || size <= 0) {
        set_error("rt_cubemap_create: bad arguments");
        return 0;
    }
    void* p = nullptr;
    const size_t bytes = (size_t)6 * size * size * 16;
    if (rt_malloc(&p, bytes) || rt_memcpy_h2d(p, rgba, bytes)) return 0;
    std::lock_guard<std::mutex> lock(g_cube_mutex);
    g_cube_size[(uint64_t)p] = size;
    return (uint64_t)p;
}

extern "C" int rt_cubemap_destroy(uint64_t handle) {
    {
        std::lock_guard<std::mutex> lock(g_cube_mutex);
        if (!g_cube_size.erase(handle)) return set_error("rt_cubemap_destroy: unknown handle");
    }
    return rt_free((void*)handle);
}

static int cube_size(uint64_t handle) {
    std::lock_guard<std::mutex> lock(g_cube_mutex);
    auto it = g_cube_size.find(handle);
    return it == g_cube_size.end() ? -1 : it->second;
}

// ---------------------------------------------------------------------------------------
// render kernel
// ---------------------------------------------------------------------------------------
#include "rt_render.h"

namespace {

using namespace rtk;

// ---------------------------------------------------------------------------------------
// init_rng (Random.cu:3-13): state s <- curand_init(seed, pixel(s), 0)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void init_rng_kernel(rt_rng_state* states, const uint32_t* __restrict__ jump,
                                                         uint32_t seed, int64_t count, int width, int height,
                                                         int shard_index, int shard_count, int tiles_x,
                                                         const int32_t* __restrict__ tile_list) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= count) return;
    uint64_t sub;
    if (shard_count <= 0) {
        sub = (uint64_t)s;  // reference layout: thread id == state index
    } else {
        const int64_t k = s / BLOCK;
        const int tile = tile_list ? tile_list[k] : shard_index + (int)k * shard_count;
        if (tile < 0 || tile >= tiles_x * ((height + TILE - 1) / TILE)) return;
        int lx, ly;
        tile_pixel((int)(s % BLOCK), &lx, &ly);
        const int x = (tile % tiles_x) * TILE + lx, y = (tile / tiles_x) * TILE + ly;
        if (x >= width || y >= height) return;
        sub = (uint64_t)y * (uint64_t)width + (uint64_t)x;
    }
    uint32_t st[6];
    rt_xorwow_seed(seed, st);
    uint32_t v[5] = {st[1], st[2], st[3], st[4], st[5]};
    for (int k = 0; sub && k < RT_XORWOW_JUMPS; k++, sub >>= 2) {
        const uint32_t reps = (uint32_t)(sub & 3u);
        const uint32_t* m = jump + (size_t)k * 800;
        for (uint32_t r = 0; r < reps; r++) {
            uint32_t o[5] = {0, 0, 0, 0, 0};
            for (int i = 0; i < 5; i++) {
                const uint32_t word = v[i];
                for (int j = 0; j < 32; j++) {
                    const uint32_t mask = 0u - ((word >> j) & 1u);
                    const uint32_t* row = m + i * 160 + j * 5;
                    o[0] ^= row[0] & mask;
                    o[1] ^= row[1] & mask;
                    o[2] ^= row[2] & mask;
                    o[3] ^= row[3] & mask;
                    o[4] ^= row[4] & mask;
                }
            }
            for (int w = 0; w < 5; w++) v[w] = o[w];
        }
    }
    rt_rng_state* out = states + s;
    out->d = st[0];
    for (int i = 0; i < 5; i++) out->v[i] = v[i];
    for (int i = 0; i < 6; i++) out->unused[i] = 0;
}

__global__ __launch_bounds__(BLOCK) void unshard_kernel(char* surface, uint64_t pitch, int width, int height,
                                                        int shard_count, const float4* shards, int64_t per_shard,
                                                        int tiles_x, const int32_t* __restrict__ tile_lists) {
    const int rank = blockIdx.y;
    const int64_t k = blockIdx.x;
    const int tile = tile_lists ? tile_lists[(size_t)rank * per_shard + k] : rank + (int)k * shard_count;
    int lx, ly;
    tile_pixel(threadIdx.x, &lx, &ly);
    const int x = (tile % tiles_x) * TILE + lx, y = (tile / tiles_x) * TILE + ly;
    if (tile < 0 || tile >= tiles_x * ((height + TILE - 1) / TILE) || x >= width || y >= height) return;
    const float4 v = shards[((size_t)rank * per_shard + k) * BLOCK + threadIdx.x];
    *reinterpret_cast<float4*>(surface + (size_t)y * pitch + (size_t)x * 16) = v;
}

const uint32_t* device_jump_table() {
    static std::mutex mu;
    static std::map<int, uint32_t*> per_device;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lock(mu);
    auto it = per_device.find(dev);
    if (it != per_device.end()) return it->second;
    uint32_t* d = nullptr;
    const size_t bytes = (size_t)RT_XORWOW_JUMPS * 800 * 4;
    if (hipMalloc(&d, bytes) != hipSuccess) return nullptr;
    if (hipMemcpy(d, rt_xorwow_jump_table(), bytes, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    per_device[dev] = d;
    return d;
}

// The render kernel variant of a frame: the traversal stack of the scene's BVH depth (the DFS holds
// at most depth + 1 entries; 30 entries -- 7.5 KB of LDS per wave -- still fits 5 waves per SIMD and
// covers the 4-bunny scene's depth 28), then the MODE bits (rt_fast_body.h render_fast_body), then
// the translation unit that holds that family (rt_render.h).
std::atomic<const ExperimentalKernels*> g_experimental{nullptr};

// Whether a frame asks for a kernel of librt_hip_exp.so (rt_render.h): the non-split / big-leaf
// A/B variants (RT_TUNE bits 12, 4-5), refill, the lone-pixel kernel, the wavefront tracer.
bool needs_experimental(const rt_render_params* p, bool has_tree, bool screens) {
    const bool stats = (p->flags & RT_RENDER_STATS) != 0;
    if ((p->flags & RT_RENDER_TRACER_WAVEFRONT) || p->refill_lanes || p->lone_count > 0) return true;
    if (screens && (p->tune & 4096u) == 0 && (!stats || (p->tune & 256u))) return true;  // big-leaf screen variants
    if (stats || p->lane_cost) return false;  // statistics / timing families are in the product
    const uint32_t mode = (p->tune >> 4) & 3u;
    return (p->tune & 4096u) != 0 || (!has_tree && (mode == 2u || mode == 3u));
}

hipError_t launch_fast(const RenderArgs& args, int waves, int depth, bool stats, hipStream_t s) {
    const int stack = (depth >= 0 && depth + 2 <= 30) ? 30 : (depth >= 0 && depth + 2 <= 40) ? 40 : 64;
    // statistics: the reference's work on scalar records (RT_TUNE bit 7: through the leaf trees);
    // RT_TUNE bit 8: a timing frame of the production kernel instead (phase clocks, no counts)
    const ExperimentalKernels* x = g_experimental.load();  // rt_render refused these frames without it
    // MODE bit 5 (librt_hip_exp.so): big-leaf screens, for scenes whose mirror has screen records
    const bool scr = args.screens != 0 && (args.tune & 4096u) == 0;
    if (stats && (args.tune & 256u)) {
        if (scr) return x ? x->fast_screen(stack, args.tree ? 61 : 57, args, waves, s) : hipErrorNotSupported;
        return launch_fast_timing(stack, args.tree ? 29 : (args.tune & 4096u) ? 9 : 25, args, waves, s);
    }
    // per-pixel work (rt_render_params.lane_cost): the timing variant of the production kernel
    if (!stats && args.lane_cost) {
        if (scr) return x ? x->fast_screen(stack, args.tree ? 61 : 57, args, waves, s) : hipErrorNotSupported;
        return launch_fast_timing(stack, args.tree ? 29 : 25, args, waves, s);
    }
    if (stats) return launch_fast_stats(stack, (args.tree && (args.tune & 128u)) ? 6 : 2, args, waves, s);
    // MODE bit 4: inner-node and small-leaf steps in separate iterations (rt_fast.h trace); RT_TUNE
    // bit 12 turns it off (A/B).  Big leaves: packed pairs in the shared-leaf loop, scalar records in
    // cooperative rounds (MODE 1, measured best); leaf trees compiled in only for scenes that have
    // them (MODE bit 2); A/B: RT_TUNE bits 4-5 = 2 scalar only, 3 pairs everywhere.
    const bool split = (args.tune & 4096u) == 0;
    if (args.queue_head) return x ? x->fast_refill(stack, args.tree ? 85 : 81, args, waves, s) : hipErrorNotSupported;
    if (scr && split && (args.tree || ((args.tune >> 4) & 3u) < 2u))
        return x ? x->fast_screen(stack, args.tree ? 53 : 49, args, waves, s) : hipErrorNotSupported;
    if (args.tree) {
        if (split) return launch_fast_prod(stack, 21, args, waves, s);
        return x ? x->fast_ab(stack, 5, args, waves, s) : hipErrorNotSupported;
    }
    const uint32_t mode = (args.tune >> 4) & 3u;
    if (split && mode < 2) return launch_fast_prod(stack, 17, args, waves, s);
    if (!x) return hipErrorNotSupported;
    if (mode == 2) return x->fast_ab(stack, 2, args, waves, s);
    if (mode == 3) return x->fast_ab(stack, 0, args, waves, s);
    return x->fast_ab(stack, 1, args, waves, s);
}

}  // namespace

void rtk::register_experimental_kernels(const rtk::ExperimentalKernels* k, uint32_t abi) {
    if (k && abi != rtk::kExperimentalAbi) {  // a plugin built against another RenderArgs / table layout
        char msg[160];
        std::snprintf(msg, sizeof msg, "librt_hip_exp.so refused: its ABI stamp 0x%08x is not librt_hip.so's 0x%08x "
                      "(rebuild both)", abi, rtk::kExperimentalAbi);
        set_error(msg);
        return;
    }
    g_experimental.store(k);
}
const rtk::ExperimentalKernels* rtk::experimental_kernels() { return g_experimental.load(); }

namespace {
// Per-(device, stream) side stream of the lone-pixel kernel and its fork / join events.
struct LoneStreams {
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
};
LoneStreams* lone_streams(hipStream_t s) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, LoneStreams> all;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lock(mu);
    LoneStreams& l = all[std::make_pair(dev, s)];
    if (!l.side && (hipStreamCreateWithFlags(&l.side, hipStreamNonBlocking) != hipSuccess ||
                    hipEventCreateWithFlags(&l.fork, hipEventDisableTiming) != hipSuccess ||
                    hipEventCreateWithFlags(&l.join, hipEventDisableTiming) != hipSuccess)) {
        l = LoneStreams{};
        return nullptr;
    }
    return &l;
}

// Per-(device, stream) queue counter of refill launches, zeroed on the stream before each launch.
unsigned long long* queue_counter(hipStream_t s) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, unsigned long long*> counters;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lock(mu);
    auto& c = counters[std::make_pair(dev, s)];
    if (!c && hipMalloc(&c, sizeof(unsigned long long)) != hipSuccess) c = nullptr;
    return c;
}

int tiles_of_shard(int width, int height, int shard_index, int shard_count) {
    const int tiles = ((width + TILE - 1) / TILE) * ((height + TILE - 1) / TILE);
    if (shard_index >= tiles) return 0;
    return (tiles - shard_index + shard_count - 1) / shard_count;
}

// quat(vec3(0, PI, 0)) with PI = 3.1415926536f (main_raytracing.cu:7,151), glm
// qua(eulerAngle) (type_quat.inl:204-213) using the RT deterministic sin/cos.
void sky_quat(float* w, float* x, float* y, float* z) {
    const float ex = 0.0f, ey = 3.1415926536f, ez = 0.0f;
    const float cx = rtm::rt_cosf(ex * 0.5f), cy = rtm::rt_cosf(ey * 0.5f), cz = rtm::rt_cosf(ez * 0.5f);
    const float sx = rtm::rt_sinf(ex * 0.5f), sy = rtm::rt_sinf(ey * 0.5f), sz = rtm::rt_sinf(ez * 0.5f);
    *w = cx * cy * cz + sx * sy * sz;
    *x = sx * cy * cz - cx * sy * sz;
    *y = cx * sy * cz + sx * cy * sz;
    *z = cx * cy * sz - sx * sy * cz;
}

}  // namespace

extern "C" int64_t rt_shard_tiles(int width, int height, int shard_index, int shard_count) {
    if (width <= 0 || height <= 0 || shard_count <= 0 || shard_index < 0 || shard_index >= shard_count) return 0;
    return tiles_of_shard(width, height, shard_index, shard_count);
}

// ---------------------------------------------------------------------------------------
// Foreign scenes.  A GPUScene filled by another host (the reference's own Scene::Upload,
// Scene.cpp:182-234) never registers a mirror.  raytracing_process keeps the reference's
// asynchronous contract (main_raytracing.cu:202-220): no call waits for the device.
//
//   * Every frame enqueues, on the render stream, a content fingerprint of the four arrays the
//     mirror derives from (~15 MB read, a few microseconds) and a one-thread kernel that sets a
//     device flag: 1 when it equals the fingerprint of the installed mirror.  The production
//     kernel is launched gated on flag == 1 and the reference-layout tracer (which reads the AoS
//     arrays directly, no mirror) gated on flag == 0: exactly one of them renders the frame, and
//     the other's waves exit at their first instruction.
//   * The fingerprint is also copied (async) to pinned host memory.  A later call that finds it
//     different from the installed mirror's -- or a first call, with no mirror yet -- starts a
//     rebuild: async copies of the arrays to pinned host buffers, then a worker thread waits for
//     them, builds the mirror exactly as rt_scene_upload does, uploads it on its own stream and
//     hands it over; the next call installs it.  Until then frames render through the reference
//     layout, bit-identical by construction.
//   * A replaced mirror is freed stream-ordered after the frames that may still read it.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

struct HashArrays {
    const uint32_t* w[4];
    unsigned long long n[4];  // words
};

__global__ __launch_bounds__(BLOCK) void fingerprint_kernel(HashArrays h, unsigned long long* out) {
    unsigned long long acc = 0;
    const unsigned long long stride = (unsigned long long)gridDim.x * BLOCK;
    for (int k = 0; k < 4; k++) {
        for (unsigned long long i = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x; i < h.n[k]; i += stride)
            acc += mix64(((unsigned long long)k << 60) ^ (i << 32) ^ h.w[k][i]);
    }
    // one atomic per workgroup (the per-wave atomics on one word serialised: 55 us per frame)
    __shared__ unsigned long long part[BLOCK / 64];
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < BLOCK / 64; w++) t += part[w];
        atomicAdd(out, t);
    }
}

// flag = (fingerprint == expected) for the gated launches; then clears the accumulator for the
// next frame (kernels on one stream run in order).
__global__ void fingerprint_gate_kernel(unsigned long long* acc, unsigned long long salt, unsigned long long expected,
                                        int have, int* flag, unsigned long long* out) {
    const unsigned long long fp = *acc ^ salt;
    *flag = (have && fp == expected) ? 1 : 0;
    *out = fp;
    *acc = 0;
}

static uint64_t host_fingerprint(const std::vector<const uint32_t*>& w, const std::vector<size_t>& n, uint64_t salt) {
    auto mix = [](unsigned long long x) {
        x ^= x >> 30;
        x *= 0xbf58476d1ce4e5b9ull;
        x ^= x >> 27;
        x *= 0x94d049bb133111ebull;
        x ^= x >> 31;
        return x;
    };
    unsigned long long acc = 0;
    for (int k = 0; k < 4; k++)
        for (size_t i = 0; i < n[k]; i++) acc += mix(((unsigned long long)k << 60) ^ ((unsigned long long)i << 32) ^ w[k][i]);
    return acc ^ salt;
}

namespace {
struct ForeignBuild {  // one background rebuild
    std::thread worker;
    std::atomic<int> state{0};  // 1 running, 2 done (ok), 3 failed
    std::vector<char> host[4];
    char* pinned[4] = {nullptr, nullptr, nullptr, nullptr};
    size_t bytes[4] = {0, 0, 0, 0};
    hipEvent_t copied = nullptr;
    uint64_t fingerprint = 0;
    void* block = nullptr;
    MirrorDevice dev;
    std::string error;
    ~ForeignBuild() {
        if (worker.joinable()) worker.join();
    }
};

struct ForeignEntry {
    int device = 0;
    unsigned long long* d_acc = nullptr;  // fingerprint accumulator, fingerprint of the frame
    unsigned long long* d_fp = nullptr;
    int* d_flag = nullptr;
    unsigned long long* h_fp = nullptr;   // pinned copy of the last fingerprint
    hipEvent_t fp_ready = nullptr;
    bool fp_pending = false;
    bool have = false;      // a mirror is installed
    uint64_t fp_mirror = 0;  // fingerprint of the arrays it was built from
    MirrorDevice dev;
    void* block = nullptr;
    std::unique_ptr<ForeignBuild> build;
    std::vector<void*> retired;  // freed stream-ordered at the next call
};

std::mutex g_foreign_mutex;
std::map<const void*, std::unique_ptr<ForeignEntry>> g_foreign;  // keyed by the BVH node array

void upload_mirror(ForeignBuild* b) {
    try {
        const GPUBVHNode* nodes = reinterpret_cast<const GPUBVHNode*>(b->pinned[0]);
        const uint32_t* fi = reinterpret_cast<const uint32_t*>(b->pinned[1]);
        const GPUFace* faces = reinterpret_cast<const GPUFace*>(b->pinned[2]);
        const GPUVertex* verts = reinterpret_cast<const GPUVertex*>(b->pinned[3]);
        if (hipEventSynchronize(b->copied) != hipSuccess) throw std::runtime_error("array read-back failed");
        const std::vector<const uint32_t*> w = {(const uint32_t*)nodes, fi, (const uint32_t*)faces, (const uint32_t*)verts};
        const std::vector<size_t> n = {b->bytes[0] / 4, b->bytes[1] / 4, b->bytes[2] / 4, b->bytes[3] / 4};
        b->fingerprint = host_fingerprint(w, n, (unsigned long long)b->bytes[0] << 1 ^ (unsigned long long)b->bytes[3] << 33);
        MirrorHost mh;
        rt_build_mirror(nodes, b->bytes[0] / sizeof(GPUBVHNode), fi, b->bytes[1] / 4, faces, b->bytes[2] / sizeof(GPUFace),
                        verts, b->bytes[3] / sizeof(GPUVertex), &mh);
        const std::vector<float> lt = rt_ltris_device_layout(mh.ltris);
        const std::vector<float>* parts[11] = {&mh.tris, &mh.pairs, &mh.tree, &lt, &mh.spairs, &mh.flat, &mh.treelets, &mh.nodes,
                                               &mh.quads, &mh.units, &mh.face_leaf};
        size_t total = 256;  // each part on a 256-B boundary (mirror.h: cache-line aligned pairs)
        for (auto* v : parts) total += (v->size() * 4 + 255) & ~(size_t)255;
        hipStream_t st;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) throw std::runtime_error("stream");
        void* block = nullptr;
        if (hipMallocAsync(&block, total, st) != hipSuccess) throw std::runtime_error("mirror allocation failed");
        char* p = static_cast<char*>(block);
        const void* where[11];
        for (int i = 0; i < 11; i++) {
            const size_t nb = parts[i]->size() * 4;
            where[i] = nb ? p : nullptr;
            if (nb && hipMemcpyAsync(p, parts[i]->data(), nb, hipMemcpyHostToDevice, st) != hipSuccess)
                throw std::runtime_error("mirror upload failed");
            p += (nb + 255) & ~(size_t)255;
        }
        const hipError_t e = hipStreamSynchronize(st);  // this worker thread only
        hipStreamDestroy(st);
        if (e != hipSuccess) throw std::runtime_error("mirror upload failed");
        b->block = block;
        b->dev.tris = where[0], b->dev.pairs = where[1], b->dev.tree = where[2], b->dev.ltris = where[3];
        b->dev.spairs = where[4], b->dev.flat = where[5], b->dev.treelets = where[6], b->dev.nodes = where[7];
        b->dev.quads = where[8], b->dev.units = where[9], b->dev.face_leaf = where[10];
        b->dev.depth = mh.depth, b->dev.fast = mh.fast, b->dev.owned = false, b->dev.fingerprint = b->fingerprint;
        b->dev.screens = mh.screens;
        b->state = 2;
    } catch (const std::exception& e) {
        b->error = e.what();
        b->state = 3;
    }
}

void free_build(ForeignBuild* b) {
    if (b->worker.joinable()) b->worker.join();
    for (auto* p : b->pinned)
        if (p) hipHostFree(p);
    if (b->copied) hipEventDestroy(b->copied);
}

// Start a rebuild from the arrays as they are on `st` now.
int start_build(ForeignEntry& fe, const GPUScene* scene, hipStream_t st, const size_t bytes[4]) {
    auto b = std::make_unique<ForeignBuild>();
    const void* src[4] = {scene->gpu_bvh_nodes, scene->gpu_bvh_face_indices, scene->gpu_faces, scene->gpu_vertices};
    for (int i = 0; i < 4; i++) {
        b->bytes[i] = bytes[i];
        if (hipHostMalloc((void**)&b->pinned[i], bytes[i] ? bytes[i] : 16) != hipSuccess ||
            hipMemcpyAsync(b->pinned[i], src[i], bytes[i], hipMemcpyDeviceToHost, st) != hipSuccess) {
            free_build(b.get());
            return set_error("rt_render: foreign scene read-back failed");
        }
    }
    if (hipEventCreateWithFlags(&b->copied, hipEventDisableTiming) != hipSuccess || hipEventRecord(b->copied, st) != hipSuccess) {
        free_build(b.get());
        return set_error("rt_render: foreign scene event");
    }
    b->state = 1;
    ForeignBuild* raw = b.get();
    b->worker = std::thread([raw, dev = fe.device]() {
        hipSetDevice(dev);
        upload_mirror(raw);
    });
    fe.build = std::move(b);
    return 0;
}

ForeignEntry* foreign_entry(const GPUScene* scene) {
    std::lock_guard<std::mutex> lock(g_foreign_mutex);
    auto& slot = g_foreign[scene->gpu_bvh_nodes];
    if (!slot) {
        auto fe = std::make_unique<ForeignEntry>();
        hipGetDevice(&fe->device);
        if (hipMalloc(&fe->d_acc, 16) != hipSuccess || hipMalloc(&fe->d_fp, 8) != hipSuccess ||
            hipMalloc(&fe->d_flag, 4) != hipSuccess || hipMemset(fe->d_acc, 0, 16) != hipSuccess ||
            hipHostMalloc((void**)&fe->h_fp, 8) != hipSuccess ||
            hipEventCreateWithFlags(&fe->fp_ready, hipEventDisableTiming) != hipSuccess) {
            set_error("rt_render: foreign scene state");
            return nullptr;
        }
        slot = std::move(fe);
    }
    return slot.get();
}
}  // namespace

// Per frame for a foreign scene: install a finished rebuild, enqueue the fingerprint gate,
// start a rebuild when the arrays no longer match.  *mir receives the installed mirror (if any);
// *gate the device flag the two launches are gated on.
static int foreign_frame(const GPUScene* scene, hipStream_t st, MirrorDevice* mir, bool* have, int** gate) {
    const size_t bytes[4] = {bytes_from(scene->gpu_bvh_nodes), bytes_from(scene->gpu_bvh_face_indices),
                             bytes_from(scene->gpu_faces), bytes_from(scene->gpu_vertices)};
    if (!bytes[0] || !bytes[1] || !bytes[2] || !bytes[3]) return set_error("rt_render: scene arrays are not device allocations");
    ForeignEntry* fe = foreign_entry(scene);
    if (!fe) return 1;
    for (void* p : fe->retired) hipFreeAsync(p, st);  // after every frame already enqueued
    fe->retired.clear();
    if (fe->build && fe->build->state >= 2) {
        ForeignBuild* b = fe->build.get();
        if (b->worker.joinable()) b->worker.join();
        if (b->state == 2) {
            if (fe->block) fe->retired.push_back(fe->block);
            fe->block = b->block;
            fe->dev = b->dev;
            fe->fp_mirror = b->fingerprint;
            fe->have = true;
        }
        free_build(b);
        fe->build.reset();
    }
    const unsigned long long salt = (unsigned long long)bytes[0] << 1 ^ (unsigned long long)bytes[3] << 33;
    // the previous frame's fingerprint, if it has landed: a mismatch starts a rebuild
    bool stale = !fe->have;
    if (fe->fp_pending && hipEventQuery(fe->fp_ready) == hipSuccess) {
        fe->fp_pending = false;
        stale = stale || *fe->h_fp != fe->fp_mirror;
    }
    if (stale && !fe->build && start_build(*fe, scene, st, bytes) != 0) return 1;
    HashArrays h;
    h.w[0] = (const uint32_t*)scene->gpu_bvh_nodes, h.n[0] = bytes[0] / 4;
    h.w[1] = scene->gpu_bvh_face_indices, h.n[1] = bytes[1] / 4;
    h.w[2] = (const uint32_t*)scene->gpu_faces, h.n[2] = bytes[2] / 4;
    h.w[3] = (const uint32_t*)scene->gpu_vertices, h.n[3] = bytes[3] / 4;
    hipLaunchKernelGGL(fingerprint_kernel, dim3(512), dim3(BLOCK), 0, st, h, fe->d_acc);
    hipLaunchKernelGGL(fingerprint_gate_kernel, dim3(1), dim3(1), 0, st, fe->d_acc, salt, (unsigned long long)fe->fp_mirror,
                       fe->have ? 1 : 0, fe->d_flag, fe->d_fp);
    if (!fe->fp_pending) {
        if (hipMemcpyAsync(fe->h_fp, fe->d_fp, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipEventRecord(fe->fp_ready, st) != hipSuccess)
            return set_error("rt_render: fingerprint read-back");
        fe->fp_pending = true;
    }
    if (hipGetLastError() != hipSuccess) return set_error("rt_render: fingerprint launch");
    *have = fe->have;
    *mir = fe->dev;
    *gate = fe->d_flag;
    return 0;
}

// Tests: which tracer rendered this foreign scene's last frame -- 1 the production tracer (its
// mirror matched the frame's fingerprint), 0 the reference layout (mismatch), -1 no mirror was
// installed (reference layout, ungated).  Synchronises the device.
extern "C" int rt_foreign_last_tracer(const GPUScene* scene) {
    ForeignEntry* fe = nullptr;
    {
        std::lock_guard<std::mutex> lock(g_foreign_mutex);
        auto it = g_foreign.find(scene->gpu_bvh_nodes);
        if (it == g_foreign.end()) return -2;
        fe = it->second.get();
    }
    if (!fe->have) return -1;
    int flag = -3;
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&flag, fe->d_flag, 4, hipMemcpyDeviceToHost) != hipSuccess) return -3;
    return flag;
}

// Tests and benchmarks: wait (host) until a rebuild for this foreign scene has finished, then let
// the next frame install it.  Returns 0 when a mirror is or will be installed, 1 on failure.
extern "C" int rt_foreign_mirror_wait(const GPUScene* scene) {
    ForeignEntry* fe = nullptr;
    {
        std::lock_guard<std::mutex> lock(g_foreign_mutex);
        auto it = g_foreign.find(scene->gpu_bvh_nodes);
        if (it == g_foreign.end()) return set_error("rt_foreign_mirror_wait: scene never rendered");
        fe = it->second.get();
    }
    if (fe->build) {
        if (fe->build->worker.joinable()) fe->build->worker.join();
        if (fe->build->state != 2) return set_error(std::string("rt_foreign_mirror_wait: ") + fe->build->error);
        return 0;
    }
    return fe->have ? 0 : set_error("rt_foreign_mirror_wait: no mirror");
}

// RT_RENDER_VALIDATE: lone_slots and lane_slots must be disjoint (a slot in both is rendered twice
// at once into the same RNG state and pixel).  Marks the lone slots in a bitmap, then counts lane
// entries that hit a mark or lie outside [0, slots) (< 0 = idle lane, allowed).
__global__ __launch_bounds__(BLOCK) void mark_slots_kernel(const int32_t* list, long long n, long long slots,
                                                           uint32_t* bits, unsigned int* bad) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const int32_t v = list[i];
    if (v < 0 || v >= slots) {
        atomicAdd(bad, 1u);
        return;
    }
    if (atomicOr(bits + (v >> 5), 1u << (v & 31)) & (1u << (v & 31))) atomicAdd(bad, 1u);  // listed twice
}
__global__ __launch_bounds__(BLOCK) void check_lanes_kernel(const int32_t* lanes, long long n, long long slots,
                                                            const uint32_t* bits, unsigned int* bad) {
    const long long i = (long long)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const int32_t v = lanes[i];
    if (v < 0) return;
    if (v >= slots || (bits[v >> 5] >> (v & 31) & 1u)) atomicAdd(bad, 1u);
}

static int validate_lone(const int32_t* lone, long long nl, const int32_t* lanes, long long nm, long long slots,
                         hipStream_t s) {
    const size_t words = (size_t)(slots + 31) / 32;
    uint32_t* bits = nullptr;
    unsigned int* bad = nullptr;
    if (hipMallocAsync((void**)&bits, words * 4 + 8, s) != hipSuccess) return set_error("rt_render: validate allocation");
    bad = reinterpret_cast<unsigned int*>(bits + words);
    unsigned int h[2] = {0, 0};
    int rc = 0;
    if (hipMemsetAsync(bits, 0, words * 4 + 8, s) != hipSuccess) rc = set_error("rt_render: validate memset");
    if (!rc) {
        hipLaunchKernelGGL(mark_slots_kernel, dim3((unsigned)((nl + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, lone, nl, slots, bits, bad);
        hipLaunchKernelGGL(check_lanes_kernel, dim3((unsigned)((nm + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, lanes, nm, slots, bits,
                           bad + 1);
        if (hipMemcpyAsync(h, bad, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            rc = set_error("rt_render: validate read-back");
    }
    (void)hipFreeAsync(bits, s);
    if (rc) return rc;
    if (h[0]) return set_error("rt_render: RT_RENDER_VALIDATE: " + std::to_string(h[0]) + " lone_slots entries out of range or repeated");
    if (h[1]) return set_error("rt_render: RT_RENDER_VALIDATE: " + std::to_string(h[1]) +
                               " lane_slots entries are out of range or also in lone_slots");
    return 0;
}

extern "C" int rt_render(const rt_render_params* p, const GPUScene* scene, void* stream) {
    if (!p || !scene) return set_error("rt_render: null argument");
    if (p->width <= 0 || p->height <= 0 || p->spp <= 0 || p->bounces < 0)
        return set_error("rt_render: bad frame size / spp / bounces");
    if (p->shard_count <= 0 || p->shard_index < 0 || p->shard_index >= p->shard_count)
        return set_error("rt_render: bad shard");
    if (!p->out_shard && (!p->surface || p->pitch < (uint64_t)p->width * 16))
        return set_error("rt_render: need a surface with pitch >= 16*width, or out_shard");
    if (p->shard_count > 1 && !p->out_shard) return set_error("rt_render: sharded render needs out_shard");
    if (!scene->rng_state || !scene->gpu_bvh_nodes || !scene->gpu_materials)
        return set_error("rt_render: scene not uploaded (rng_state / bvh / materials missing)");
    if ((p->flags & RT_RENDER_STATS) && !p->stats) return set_error("rt_render: stats flag without buffer");

    RenderArgs a;
    std::memset(&a, 0, sizeof(a));
    a.spheres = scene->gpu_spheres;
    a.materials = scene->gpu_materials;
    a.nodes = scene->gpu_bvh_nodes;
    a.face_indices = scene->gpu_bvh_face_indices;
    a.vertices = scene->gpu_vertices;
    a.faces = scene->gpu_faces;
    a.rng = (rt_rng_state*)scene->rng_state;
    a.sphere_count = scene->sphere_count;
    a.cam = scene->camera;
    if (scene->environment_cubemap_tex) {
        const int n = cube_size(scene->environment_cubemap_tex);
        if (n <= 0) return set_error("rt_render: unknown environment cube map handle");
        a.sky = (const float*)scene->environment_cubemap_tex;
        a.sky_n = n;
    }
    sky_quat(&a.qw, &a.qx, &a.qy, &a.qz);
    a.surface = (char*)p->surface;
    a.last = (const char*)p->surface_last_frame;
    a.out_shard = (float4*)p->out_shard;
    a.pitch = p->pitch;
    a.width = p->width, a.height = p->height;
    a.frame_index = p->frame_index, a.spp = p->spp, a.bounces = p->bounces;
    a.shard_index = p->shard_index, a.shard_count = p->shard_count;
    a.tiles_x = (p->width + TILE - 1) / TILE;
    a.stats = (unsigned long long*)p->stats;
    a.seg_counter = (unsigned long long*)p->segment_counter;

    if (p->tile_list && (p->tile_count <= 0 || p->tile_count > (int64_t)1 << 28))
        return set_error("rt_render: tile_list needs 0 < tile_count < 2^28");
    if (p->tile_list && !p->out_shard && p->shard_count > 1) return set_error("rt_render: sharded render needs out_shard");
    a.tile_list = p->tile_list;
    a.wave_clock = (unsigned long long*)p->wave_clock;
    const int tiles = p->tile_list ? (int)p->tile_count : tiles_of_shard(p->width, p->height, p->shard_index, p->shard_count);
    if (tiles == 0) return 0;
    if (p->lane_slots && (p->lane_slot_count <= 0 || p->lane_slot_count % WAVE != 0 || p->lane_slot_count > (int64_t)1 << 30))
        return set_error("rt_render: lane_slots needs a positive multiple of 64 entries (< 2^30)");
    a.lane_slots = p->lane_slots;
    a.slot_count = (long long)tiles * TILE * TILE;
    if (a.slot_count > (1LL << 32)) return set_error("rt_render: more than 2^32 pixel slots in one launch");
    a.lane_cost = p->lane_cost;
    a.priority_waves = p->lane_slots ? (int)std::min<int64_t>(std::max<int64_t>(p->priority_waves, 0), 1 << 30) : 0;
    const int waves = p->lane_slots ? (int)(p->lane_slot_count / WAVE) : tiles * 4;  // production tracer's grid
    a.entry_count = (long long)waves * WAVE;
    if (p->refill_lanes < 0 || p->refill_lanes > 64) return set_error("rt_render: refill_lanes must be in [0, 64]");
    if (p->waves_per_simd < 0 || p->waves_per_simd > 7)
        return set_error("rt_render: waves_per_simd must be 0 (default), 1-4 (LDS-capped residency), 5, 6 or 7");
    if (((p->tune >> 9) & 3u) == 1u)
        return set_error("rt_render: RT_TUNE occupancy override 1 (compiler's choice) is not built");
    a.waves_per_simd = p->waves_per_simd;
    a.refill_lanes = p->refill_lanes;
    // Every device buffer must cover what the launch touches: a short buffer would fault the GPU.
    {
        const bool compact = p->out_shard != nullptr;
        const size_t slots = (size_t)tiles * TILE * TILE;
        const size_t frame = (size_t)p->pitch * (size_t)(p->height - 1) + (size_t)p->width * 16;
        const size_t rng_need = (compact ? slots : (size_t)p->width * p->height) * sizeof(rt_rng_state);
        if (bytes_from(scene->rng_state) < rng_need) return set_error("rt_render: rng_state is smaller than the frame / shard");
        if (compact && bytes_from(p->out_shard) < slots * 16) return set_error("rt_render: out_shard too small");
        if (compact && p->surface_last_frame && bytes_from(p->surface_last_frame) < slots * 16)
            return set_error("rt_render: surface_last_frame (shard) too small");
        if (!compact && bytes_from(p->surface) < frame) return set_error("rt_render: surface too small");
        if (!compact && p->surface_last_frame && bytes_from(p->surface_last_frame) < frame)
            return set_error("rt_render: surface_last_frame too small");
        if (p->tile_list && bytes_from(p->tile_list) < (size_t)tiles * 4) return set_error("rt_render: tile_list too small");
        if (p->wave_clock && bytes_from(p->wave_clock) < (size_t)waves * 8)
            return set_error("rt_render: wave_clock too small");
        if (p->lane_slots && bytes_from(p->lane_slots) < (size_t)p->lane_slot_count * 4)
            return set_error("rt_render: lane_slots too small");
        if (p->lane_cost && bytes_from(p->lane_cost) < slots * 4) return set_error("rt_render: lane_cost too small");
        const size_t stats_need = (RT_STAT_COUNT + ((p->tune & 2048u) ? (size_t)waves * 8 : 0)) * 8;
        if (p->stats && bytes_from(p->stats) < stats_need) return set_error("rt_render: stats too small");
    }
    const bool want_ref = (p->flags & RT_RENDER_TRACER_REF) != 0;
    MirrorDevice mir;
    int* gate = nullptr;  // foreign scenes: device flag selecting production (1) or reference-layout (0) tracer
    bool foreign_fast = false;
    if ((!rt_internal_lookup_mirror(scene, &mir) || !mir.owned) && !want_ref) {
        // not uploaded through rt_scene_upload: fingerprint-gated private mirror, no host sync
        if (foreign_frame(scene, (hipStream_t)stream, &mir, &foreign_fast, &gate) != 0) return 1;
        if (!foreign_fast) gate = nullptr, mir = MirrorDevice{};  // no mirror yet: reference layout, ungated
    }
    const void* tris = mir.tris;
    const int depth = mir.depth;
    const bool scene_fast = mir.fast;
    a.tune = p->tune;  // diagnostic A/B knobs; 0 = the production path
    a.pairs = (a.tune & 2u) ? nullptr : (const float4*)mir.pairs;
    a.quads = (a.tune & ((1u << 20) | 2u)) ? nullptr : (const float4*)mir.quads;  // RT_TUNE bit 20: no twins
    a.units = (const float4*)mir.units;
    a.tree = (a.tune & 4u) ? nullptr : (const float4*)mir.tree;
    a.ltris = (const float4*)mir.ltris;
    a.spairs = (a.tune & 8u) ? nullptr : (const float4*)mir.spairs;
    a.flat = (const float4*)mir.flat;
    a.face_leaf = (const uint32_t*)mir.face_leaf;
    a.tris = want_ref ? nullptr : (const FlatTri*)tris;
    const bool stats = (p->flags & RT_RENDER_STATS) != 0;
    hipStream_t s = (hipStream_t)stream;
    const bool want_flat = (p->flags & RT_RENDER_TRACER_FLAT) != 0;
    if ((p->lane_slots || p->lane_cost || p->refill_lanes) && (gate || !a.tris || want_flat))
        return set_error("rt_render: lane_slots / lane_cost / refill_lanes need the production tracer on an rt_scene_upload scene");
    if (p->lane_cost && p->refill_lanes) return set_error("rt_render: lane_cost probes run without refill");
    const bool want_wf = (p->flags & RT_RENDER_TRACER_WAVEFRONT) != 0;
    if (want_wf && (gate || !a.tris || want_flat || stats || p->lane_cost || p->refill_lanes || p->wave_clock ||
                    p->lone_count))
        return set_error("rt_render: the wavefront tracer needs an rt_scene_upload scene and no statistics / lane_cost / "
                         "wave_clock / refill / lone frames");
    // its pixel state packs the sample count in 16 bits and the bounce in 8; a generation per segment
    if (want_wf && (p->spp > 65535 || p->bounces > 255 || (int64_t)p->spp * p->bounces > 65536))
        return set_error("rt_render: the wavefront tracer needs spp <= 65535, bounces <= 255, spp x bounces <= 65536");
    a.screens = (mir.screens > 0 && (a.tune & (1u << 28)) == 0 && a.tris && !(p->flags & RT_RENDER_TRACER_FLAT)) ? 1 : 0;
    if (!g_experimental.load() && needs_experimental(p, a.tree != nullptr, a.screens != 0))
        return set_error("rt_render: this frame asks for an experimental render path (wavefront tracer, refill, lone-pixel "
                         "kernel or an RT_TUNE A/B variant), which lives in librt_hip_exp.so -- load it first "
                         "(rt.load_experimental())");
    const bool lone = p->lone_count > 0;
    if (p->lone_count < 0 || p->lone_count > (int64_t)1 << 28 || (lone && !p->lone_slots))
        return set_error("rt_render: lone_count must be in [0, 2^28] with lone_slots");
    if (lone && (!p->lane_slots || gate || !a.tris || want_flat || stats || p->lane_cost || p->refill_lanes))
        return set_error("rt_render: lone_slots need lane_slots and the production tracer on an rt_scene_upload scene "
                         "(no statistics / lane_cost / refill frames)");
    if (lone && (!mir.treelets || depth < 0 || depth > 75))
        return set_error("rt_render: lone_slots need the scene's treelets (a BVH of depth <= 75 with an inner root)");
    if (lone && bytes_from(p->lone_slots) < (size_t)p->lone_count * 4) return set_error("rt_render: lone_slots too small");
    if ((p->flags & RT_RENDER_VALIDATE) && lone && validate_lone(p->lone_slots, p->lone_count, p->lane_slots,
                                                                  p->lane_slot_count, a.slot_count, s) != 0)
        return 1;
    if (p->refill_lanes) {  // the queue counter, zeroed on the launch stream
        a.queue_head = queue_counter(s);
        if (!a.queue_head) return set_error("rt_render: cannot allocate the refill queue counter");
        if (check(hipMemsetAsync(a.queue_head, 0, sizeof(unsigned long long), s), "hipMemsetAsync") != 0) return 1;
    }
    a.scene_fast = scene_fast ? 1 : 0;
    // the traversal kernels read the mirror's private node array (mirror.h: 64-B aligned sibling
    // pairs in right-first pre-order; RT_TUNE bit 27: the reference's array instead, A/B); the
    // reference-layout tracers keep the reference's
    const GPUBVHNode* const trav_nodes =
        (mir.nodes && (a.tune & (1u << 27)) == 0) ? (const GPUBVHNode*)mir.nodes : scene->gpu_bvh_nodes;
    auto trav = [&](const RenderArgs& x) {  // the arguments as they stand at launch, traversal nodes
        RenderArgs f = x;
        f.nodes = trav_nodes;
        // the face -> leaf table holds private-array node indices: with the reference's array (bit 27) the
        // deferral guard must not look them up there -- without a table it walks the leaf up to the entry
        if (trav_nodes != (const GPUBVHNode*)mir.nodes) f.face_leaf = nullptr;
        return f;
    };
    hipError_t e;
    if (gate) {  // foreign scene with a mirror: exactly one of the two runs, by the frame's fingerprint
        a.gate = gate, a.gate_value = 1;
        e = want_flat ? launch_ref_tracer(true, a, tiles * 4, depth, stats, s) : launch_fast(trav(a), waves, depth, stats, s);
        if (e == hipSuccess) {
            RenderArgs r = a;
            r.tris = nullptr, r.gate_value = 0;
            e = launch_ref_tracer(false, r, tiles * 4, -1, stats, s);
        }
    } else if (!a.tris)
        e = launch_ref_tracer(false, a, tiles * 4, depth, stats, s);
    else if (want_flat)
        e = launch_ref_tracer(true, a, tiles * 4, depth, stats, s);
    else if (want_wf)
        e = g_experimental.load()->wavefront(trav(a), depth, s);
    else if (lone) {
        // the lone-pixel kernel on a side stream forked from and joined back into the caller's
        LoneStreams* ls = lone_streams(s);
        if (!ls) return set_error("rt_render: cannot create the lone-pixel stream");
        if (check(hipEventRecord(ls->fork, s), "hipEventRecord") || check(hipStreamWaitEvent(ls->side, ls->fork, 0), "hipStreamWaitEvent"))
            return 1;
        e = g_experimental.load()->lone(a, p->lone_slots, (int)p->lone_count, mir.treelets, ls->side);
        if (e == hipSuccess) e = launch_fast(trav(a), waves, depth, stats, s);
        if (check(hipEventRecord(ls->join, ls->side), "hipEventRecord") || check(hipStreamWaitEvent(s, ls->join, 0), "hipStreamWaitEvent"))
            return 1;
    } else
        e = launch_fast(trav(a), waves, depth, stats, s);
    return check(e, "render_kernel launch");
}

// 1 when librt_hip_exp.so's render paths are registered (rt_render.h ExperimentalKernels).
extern "C" int rt_experimental_loaded() { return rtk::experimental_kernels() ? 1 : 0; }

extern "C" int rt_init_rng(void* states, int width, int height, int shard_index, int shard_count, uint32_t seed,
                           void* stream) {
    if (!states || width <= 0 || height <= 0 || shard_count <= 0 || shard_index < 0 || shard_index >= shard_count)
        return set_error("rt_init_rng: bad arguments");
    const uint32_t* jump = device_jump_table();
    if (!jump) return set_error("rt_init_rng: jump table upload failed");
    const int tiles_x = (width + TILE - 1) / TILE;
    int64_t count;
    int sc;
    if (shard_count == 1) {
        count = (int64_t)width * height;
        sc = 0;
    } else {
        count = (int64_t)tiles_of_shard(width, height, shard_index, shard_count) * BLOCK;
        sc = shard_count;
    }
    if (count == 0) return 0;
    if (bytes_from(states) < (size_t)count * sizeof(rt_rng_state)) return set_error("rt_init_rng: rng_states too small");
    const int blocks = (int)((count + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(init_rng_kernel, dim3(blocks), dim3(BLOCK), 0, (hipStream_t)stream, (rt_rng_state*)states, jump,
                       seed, count, width, height, shard_index, sc, tiles_x, (const int32_t*)nullptr);
    return check(hipGetLastError(), "init_rng_kernel launch");
}

extern "C" int rt_init_rng_tiles(void* states, int width, int height, const int32_t* tile_list, int64_t tile_count,
                                 uint32_t seed, void* stream) {
    if (!states || !tile_list || width <= 0 || height <= 0 || tile_count <= 0 || tile_count > ((int64_t)1 << 28))
        return set_error("rt_init_rng_tiles: bad arguments");
    const uint32_t* jump = device_jump_table();
    if (!jump) return set_error("rt_init_rng_tiles: jump table upload failed");
    const int64_t count = tile_count * BLOCK;
    if (bytes_from(states) < (size_t)count * sizeof(rt_rng_state) || bytes_from(tile_list) < (size_t)tile_count * 4)
        return set_error("rt_init_rng_tiles: rng_states or tile_list too small");
    hipLaunchKernelGGL(init_rng_kernel, dim3((unsigned)tile_count), dim3(BLOCK), 0, (hipStream_t)stream,
                       (rt_rng_state*)states, jump, seed, count, width, height, 0, 1, (width + TILE - 1) / TILE,
                       tile_list);
    return check(hipGetLastError(), "init_rng_kernel launch");
}

extern "C" int rt_unshard(void* surface, uint64_t pitch, int width, int height, int shard_count, const void* shards,
                          int64_t per_shard, void* stream) {
    if (!surface || !shards || shard_count <= 0 || per_shard <= 0 || width <= 0 || height <= 0)
        return set_error("rt_unshard: bad arguments");
    if (bytes_from(shards) < (size_t)shard_count * per_shard * BLOCK * 16 ||
        bytes_from(surface) < pitch * (size_t)(height - 1) + (size_t)width * 16)
        return set_error("rt_unshard: shards or surface too small");
    const int tiles_x = (width + TILE - 1) / TILE;
    hipLaunchKernelGGL(unshard_kernel, dim3((unsigned)per_shard, shard_count), dim3(BLOCK), 0, (hipStream_t)stream,
                       (char*)surface, pitch, width, height, shard_count, (const float4*)shards, per_shard, tiles_x,
                       (const int32_t*)nullptr);
    return check(hipGetLastError(), "unshard_kernel launch");
}

extern "C" int rt_unshard_tiles(void* surface, uint64_t pitch, int width, int height, int shard_count,
                                const void* shards, int64_t per_shard, const int32_t* tile_lists, void* stream) {
    if (!surface || !shards || !tile_lists || shard_count <= 0 || per_shard <= 0 || width <= 0 || height <= 0)
        return set_error("rt_unshard_tiles: bad arguments");
    if (bytes_from(shards) < (size_t)shard_count * per_shard * BLOCK * 16 ||
        bytes_from(tile_lists) < (size_t)shard_count * per_shard * 4 ||
        bytes_from(surface) < pitch * (size_t)(height - 1) + (size_t)width * 16)
        return set_error("rt_unshard_tiles: shards, tile_lists or surface too small");
    hipLaunchKernelGGL(unshard_kernel, dim3((unsigned)per_shard, shard_count), dim3(BLOCK), 0, (hipStream_t)stream,
                       (char*)surface, pitch, width, height, shard_count, (const float4*)shards, per_shard,
                       (width + TILE - 1) / TILE, tile_lists);
    return check(hipGetLastError(), "unshard_kernel launch");
}

// ---------------------------------------------------------------------------------------
// reference entry points
// ---------------------------------------------------------------------------------------
extern "C" void raytracing_process(void* surface, void* surface_last_frame, int width, int height, size_t pitch,
                                   int frame_index, GPUScene* scene) {
    rt_render_params p;
    std::memset(&p, 0, sizeof(p));
    p.surface = surface;
    p.surface_last_frame = surface_last_frame;
    p.width = width, p.height = height, p.pitch = pitch;
    p.frame_index = frame_index;
    p.spp = 5;      // main_raytracing.cu:166-170 (Release)
    p.bounces = 6;  // main_raytracing.cu:115
    p.shard_index = 0, p.shard_count = 1;
    if (rt_render(&p, scene, nullptr) != 0)
        std::printf("(raytracing_kernel_main) failed to launch error = %s\n", rt_last_error());
}

extern "C" void init_rng(uint32_t thread_block_count, uint32_t thread_block_size, void* states, unsigned int seed) {
    const uint32_t* jump = device_jump_table();
    const int64_t count = (int64_t)thread_block_count * thread_block_size;
    if (bytes_from(states) < (size_t)count * sizeof(rt_rng_state)) {
        set_error("init_rng: rngStates is smaller than thread_block_count * thread_block_size states");
        std::printf("(init_rng) failed: %s\n", rt_last_error());
        return;
    }
    if (!jump || count == 0) {
        set_error("init_rng: jump table upload failed");
        std::printf("(init_rng) failed: %s\n", rt_last_error());
        return;
    }
    hipLaunchKernelGGL(init_rng_kernel, dim3(thread_block_count), dim3(thread_block_size), 0, nullptr,
                       (rt_rng_state*)states, jump, seed, count, 0, 0, 0, 0, 0, (const int32_t*)nullptr);
    if (check(hipGetLastError(), "init_rng_kernel launch")) std::printf("(init_rng) failed: %s\n", rt_last_error());
}


// Diagnostics: the leaf-tree cull predicate of the render kernel, evaluated on the host by the
// same code (tests/test_leaf_tree.py).
// The twin test (rt_fast.h twin_rejected) on the host, for tests/test_scene.py: triangle record `rec`
// (mirror.h tris) and its twin (v0, e2, e1) under glm's test (test_triangle's operation order) for the
// ray (o, nd); bit 0: twin_rejected, bit 1: the twin passes glm's predicate, bit 2: A passes it.
extern "C" int rt_twin_check_host(const float rec[12], const float o[3], const float nd[3]) {
    using rtm::f3;
    const f3 O = rtm::mk(o[0], o[1], o[2]), N = rtm::mk(nd[0], nd[1], nd[2]), v0 = rtm::mk(rec[0], rec[1], rec[2]);
    const f3 e1 = rtm::mk(rec[3], rec[4], rec[5]), e2 = rtm::mk(rec[6], rec[7], rec[8]);
    auto glm = [&](f3 a, f3 b, float* det, float* u, float* v, float* uv) {  // (e1, e2) = (a, b)
        const f3 p = rtm::cross(N, b);
        *det = rtm::dot(a, p);
        const f3 dist = rtm::sub(O, v0);
        *u = rtm::dot(dist, p);
        *v = rtm::dot(N, rtm::cross(dist, a));
        *uv = *u + *v;
    };
    auto ok = [](float det, float u, float v, float uv) {
        const bool neg = signbit(det);
        const float ad = fabsf(det), su = neg ? -u : u, sv = neg ? -v : v, suv = neg ? -uv : uv;
        return ad > 1.1920928955078125e-07f && !(su < 0.0f || su > ad) && !(sv < 0.0f || suv > ad);
    };
    float d, u, v, uv, d2, u2, v2, uv2;
    glm(e1, e2, &d, &u, &v, &uv);
    glm(e2, e1, &d2, &u2, &v2, &uv2);
    const f3 dist = rtm::sub(O, v0);
    const float dn = (fabsf(dist.x) + fabsf(dist.y)) + fabsf(dist.z);
    float kd, ke;
    rt_twin_bounds(rec, &kd, &ke);
    return (rtfast::twin_rejected(d, u, v, uv, dn, kd, ke) ? 1 : 0) | (ok(d2, u2, v2, uv2) ? 2 : 0) | (ok(d, u, v, uv) ? 4 : 0);
}

extern "C" int rt_cluster_cull_host(const float origin[3], const float nd[3], float best, const float node[16]) {
    rtfast::Ray R;
    R.o = rtm::mk(origin[0], origin[1], origin[2]);
    R.nd = rtm::mk(nd[0], nd[1], nd[2]);
    R.d = R.nd;
    R.r = rtm::mk(1.0f / nd[0], 1.0f / nd[1], 1.0f / nd[2]);
    R.fast = true;
    const float4 K0 = make_float4(node[0], node[1], node[2], node[3]);
    const float4 K1 = make_float4(node[4], node[5], node[6], node[7]);
    const float4 K2 = make_float4(node[8], node[9], node[10], node[11]);
    const float4 K3 = make_float4(node[12], node[13], node[14], node[15]);
    return rtfast::cluster_cull(R, R.r, best, K0, K1, K2, K3) ? 1 : 0;
}
