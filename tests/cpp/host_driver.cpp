// host_driver.cpp -- a C++ host driving librt_hip.so through include/rt_abi.h the way the
// reference's CUDARayTracer drives its CUDA kernels (RayTracing/RayTracing.cpp:205-234,
// 216-221): init_rng over ceil(W*H/128) blocks of 128 states, Scene::Upload, then per frame
// raytracing_process(surface, last, ...) followed by the D2D copy of surface into last.
// Writes the final frame (W*H float4, rows bottom-up, pitch removed) to argv[1].
//
// With a sixth argument "split", the same frames are split over every visible device by the
// C-ABI's multi-GPU path (one host thread, N devices): rt_shard_plan deals the 16x16 tiles,
// each device renders its compact shard (spp 5, 6 bounces as raytracing_process), and
// rt_gather_shards (RCCL, communicators from rt_comm_init_all) brings the shards to device 0,
// where rt_unshard_tiles writes the pitched surface.  Before the first frame every device runs
// one probe frame of per-pixel work (rt_render_params.lane_cost, on a copy of its RNG states)
// and renders through the lane map rt_lane_plan builds from it, refined once by rt_lane_refine from
// the per-wave clocks of a timing frame of that map (bench.py's N > 1 default).
//
//   g++ -std=c++17 -Iinclude tests/cpp/host_driver.cpp -Lcuda-raytracing_amd -lrt_hip -o host_driver
//   ./host_driver out.bin W H frames assets_dir [split]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rt_abi.h"

#define CHECK(x)                                                              \
    do {                                                                      \
        if ((x) != 0) {                                                       \
            std::fprintf(stderr, "%s failed: %s\n", #x, rt_last_error());     \
            std::exit(1);                                                     \
        }                                                                     \
    } while (0)

static void write_frame(const char* path, const void* surface, size_t pitch, int w, int h) {
    std::vector<char> img(pitch * h);
    CHECK(rt_memcpy_d2h(img.data(), surface, img.size()));
    FILE* out = std::fopen(path, "wb");
    if (!out) std::exit(1);
    for (int y = 0; y < h; y++) std::fwrite(img.data() + (size_t)y * pitch, 16, (size_t)w, out);
    std::fclose(out);
}

static int run_single(const char* path, int w, int h, int frames, const char* assets) {
    rt_scene* scene = rt_scene_create();
    CHECK(rt_scene_setup(scene, 0, assets));  // Cornell box + bunny, RayTracing.cpp:24-25
    rt_scene_set_viewport(scene, w, h);
    // RayTracing.cpp:216-221: the RNG states, seeded per pixel
    const uint32_t block = 128, blocks = (uint32_t)((w * h + block - 1) / block);
    void* rng = nullptr;
    CHECK(rt_malloc(&rng, (size_t)blocks * block * 48));
    init_rng(blocks, block, rng, 0xDEADBEEFu);  // errors are printed, as in the reference
    CHECK(rt_scene_upload(scene, rng));  // Scene::Upload
    const GPUScene* gpu = rt_scene_gpu(scene);
    void *surface = nullptr, *last = nullptr;
    size_t pitch = 0, pitch2 = 0;
    CHECK(rt_malloc_pitch(&surface, &pitch, (size_t)w * 16, h));
    CHECK(rt_malloc_pitch(&last, &pitch2, (size_t)w * 16, h));
    CHECK(rt_memset(last, 0, pitch2 * h));
    for (int f = 0; f < frames; f++) {
        raytracing_process(surface, last, w, h, pitch, f, const_cast<GPUScene*>(gpu));  // RayTracing.cpp:232
        CHECK(rt_memcpy_d2d(last, surface, pitch * h));  // RayTracing.cpp:233
    }
    CHECK(rt_synchronize());
    write_frame(path, surface, pitch, w, h);
    rt_free(surface);
    rt_free(last);
    rt_free(rng);
    rt_scene_destroy(scene);
    std::printf("ok %dx%d frames=%d pitch=%zu\n", w, h, frames, pitch);
    return 0;
}

struct Rank {
    rt_scene* scene = nullptr;
    void *rng = nullptr, *shard[2] = {nullptr, nullptr}, *tiles = nullptr, *lane_map = nullptr;
    int64_t count = 0, lanes = 0;
};

static int run_split(const char* path, int w, int h, int frames, const char* assets) {
    const int n = rt_device_count();
    if (n <= 0) {
        std::fprintf(stderr, "no HIP device\n");
        return 1;
    }
    std::vector<int> devs(n);
    for (int d = 0; d < n; d++) devs[d] = d;
    std::vector<rt_comm*> comms(n, nullptr);
    CHECK(rt_comm_init_all(comms.data(), n, devs.data()));
    const int64_t cap = rt_shard_plan_capacity(w, h, n);
    std::vector<int32_t> lists((size_t)cap * n);
    std::vector<int64_t> counts(n);
    CHECK(rt_shard_plan(w, h, n, nullptr, cap, lists.data(), counts.data()));
    const size_t shard_bytes = (size_t)cap * 256 * 16;
    std::vector<Rank> ranks(n);
    std::vector<size_t> recv_bytes(n);
    for (int d = 0; d < n; d++) {
        Rank& r = ranks[d];
        CHECK(rt_set_device(d));
        r.count = counts[d];
        recv_bytes[d] = (size_t)r.count * 256 * 16;
        r.scene = rt_scene_create();
        CHECK(rt_scene_setup(r.scene, 0, assets));
        rt_scene_set_viewport(r.scene, w, h);
        CHECK(rt_malloc(&r.tiles, (size_t)cap * 4));
        CHECK(rt_memcpy_h2d(r.tiles, lists.data() + (size_t)d * cap, (size_t)cap * 4));
        CHECK(rt_malloc(&r.rng, (size_t)cap * 256 * 48));
        CHECK(rt_init_rng_tiles(r.rng, w, h, (const int32_t*)r.tiles, r.count, 0xDEADBEEFu, nullptr));
        CHECK(rt_scene_upload(r.scene, r.rng));
        for (int b = 0; b < 2; b++) {
            CHECK(rt_malloc(&r.shard[b], shard_bytes));
            CHECK(rt_memset(r.shard[b], 0, shard_bytes));
        }
        // lane plan: probe frame of per-pixel work on a copy of the states, then rt_lane_plan
        const int64_t slots = r.count * 256;
        void *rng_copy = nullptr, *cost_dev = nullptr;
        CHECK(rt_malloc(&rng_copy, (size_t)slots * 48));
        CHECK(rt_memcpy_d2d(rng_copy, r.rng, (size_t)slots * 48));
        CHECK(rt_malloc(&cost_dev, (size_t)slots * 4));
        CHECK(rt_memset(cost_dev, 0, (size_t)slots * 4));
        rt_render_params p;
        std::memset(&p, 0, sizeof(p));
        p.width = w, p.height = h, p.spp = 5, p.bounces = 6;
        p.shard_index = d, p.shard_count = n;
        p.out_shard = r.shard[0];
        p.tile_list = (const int32_t*)r.tiles;
        p.tile_count = r.count;
        p.lane_cost = (uint32_t*)cost_dev;
        CHECK(rt_render(&p, rt_scene_gpu(r.scene), nullptr));
        std::vector<uint32_t> cost((size_t)slots);
        CHECK(rt_memcpy_d2h(cost.data(), cost_dev, cost.size() * 4));  // synchronising copy
        CHECK(rt_memcpy_d2d(r.rng, rng_copy, (size_t)slots * 48));
        CHECK(rt_memset(r.shard[0], 0, shard_bytes));
        std::vector<int32_t> map((size_t)rt_lane_plan_capacity(slots));
        int64_t nlong = 0;
        r.lanes = rt_lane_plan(cost.data(), slots, 48000.0, 1.0, map.data(), (int64_t)map.size(), &nlong);
        if (r.lanes <= 0) CHECK(1);
        CHECK(rt_malloc(&r.lane_map, (size_t)r.lanes * 4));
        CHECK(rt_memcpy_h2d(r.lane_map, map.data(), (size_t)r.lanes * 4));
        // one round of measured refinement (bench.py refine_lane_map): per-wave clocks of a timing
        // frame of the map, rt_lane_refine, and the refined map kept only if a frame of it is faster
        {
            const int64_t waves = r.lanes / 64;
            void* clk_dev = nullptr;
            CHECK(rt_malloc(&clk_dev, (size_t)waves * 8));
            p.lane_cost = nullptr;
            p.lane_slots = (const int32_t*)r.lane_map, p.lane_slot_count = r.lanes;
            p.wave_clock = (uint64_t*)clk_dev;
            CHECK(rt_render(&p, rt_scene_gpu(r.scene), nullptr));
            std::vector<int64_t> ticks((size_t)waves);
            CHECK(rt_memcpy_d2h(ticks.data(), clk_dev, ticks.size() * 8));
            CHECK(rt_memcpy_d2d(r.rng, rng_copy, (size_t)slots * 48));
            for (int64_t& t : ticks) t = t < 0 ? 0 : t;  // device-clock deltas: never negative, guarded anyway
            std::vector<int32_t> map2((size_t)(2 * r.lanes));
            int64_t nsplit = 0;
            const int64_t n2 = rt_lane_refine(map.data(), r.lanes, cost.data(), slots, ticks.data(), 0.85, map2.data(),
                                              (int64_t)map2.size(), &nsplit);
            if (n2 <= 0) CHECK(1);
            void* map2_dev = nullptr;
            CHECK(rt_malloc(&map2_dev, (size_t)n2 * 4));
            CHECK(rt_memcpy_h2d(map2_dev, map2.data(), (size_t)n2 * 4));
            p.wave_clock = nullptr;
            auto frame_s = [&](void* m, int64_t entries) {
                p.lane_slots = (const int32_t*)m, p.lane_slot_count = entries;
                CHECK(rt_synchronize());
                const auto t0 = std::chrono::steady_clock::now();
                CHECK(rt_render(&p, rt_scene_gpu(r.scene), nullptr));
                CHECK(rt_synchronize());
                const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                CHECK(rt_memcpy_d2d(r.rng, rng_copy, (size_t)slots * 48));
                return s;
            };
            if (nsplit > 0 && frame_s(map2_dev, n2) < frame_s(r.lane_map, r.lanes)) {
                rt_free(r.lane_map);
                r.lane_map = map2_dev, r.lanes = n2;
            } else {
                rt_free(map2_dev);
            }
            rt_free(clk_dev);
            CHECK(rt_memset(r.shard[0], 0, shard_bytes));
        }
        rt_free(rng_copy);
        rt_free(cost_dev);
    }
    CHECK(rt_set_device(0));
    void *gathered = nullptr, *surface = nullptr, *lists_dev = nullptr;
    size_t pitch = 0;
    CHECK(rt_malloc(&gathered, shard_bytes * n));
    CHECK(rt_malloc(&lists_dev, lists.size() * 4));
    CHECK(rt_memcpy_h2d(lists_dev, lists.data(), lists.size() * 4));
    CHECK(rt_malloc_pitch(&surface, &pitch, (size_t)w * 16, h));
    for (int f = 0; f < frames; f++) {
        for (int d = 0; d < n; d++) {
            Rank& r = ranks[d];
            CHECK(rt_set_device(d));
            rt_render_params p;
            std::memset(&p, 0, sizeof(p));
            p.surface_last_frame = r.shard[(f + 1) & 1];
            p.width = w, p.height = h, p.frame_index = f;
            p.spp = 5, p.bounces = 6;  // raytracing_process's constants (main_raytracing.cu:115,166-170)
            p.shard_index = d, p.shard_count = n;
            p.out_shard = r.shard[f & 1];
            p.tile_list = (const int32_t*)r.tiles;
            p.tile_count = r.count;
            p.lane_slots = (const int32_t*)r.lane_map;
            p.lane_slot_count = r.lanes;
            CHECK(rt_render(&p, rt_scene_gpu(r.scene), nullptr));
        }
        CHECK(rt_comm_group_start());
        for (int d = 0; d < n; d++) {
            CHECK(rt_set_device(d));
            CHECK(rt_gather_shards(comms[d], ranks[d].shard[f & 1], recv_bytes[d], d == 0 ? gathered : nullptr,
                                   shard_bytes, d == 0 ? recv_bytes.data() : nullptr, 0, nullptr));
        }
        CHECK(rt_comm_group_end());
        CHECK(rt_set_device(0));
        CHECK(rt_unshard_tiles(surface, pitch, w, h, n, gathered, cap, (const int32_t*)lists_dev, nullptr));
    }
    for (int d = 0; d < n; d++) {
        CHECK(rt_set_device(d));
        CHECK(rt_synchronize());
    }
    CHECK(rt_set_device(0));
    write_frame(path, surface, pitch, w, h);
    for (int d = 0; d < n; d++) {
        Rank& r = ranks[d];
        CHECK(rt_set_device(d));
        rt_free(r.rng);
        rt_free(r.tiles);
        rt_free(r.shard[0]);
        rt_free(r.shard[1]);
        rt_free(r.lane_map);
        rt_scene_destroy(r.scene);
        CHECK(rt_comm_destroy(comms[d]));
    }
    CHECK(rt_set_device(0));
    rt_free(gathered);
    rt_free(lists_dev);
    rt_free(surface);
    std::printf("ok split %dx%d frames=%d devices=%d\n", w, h, frames, n);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s out.bin W H frames assets_dir [split]\n", argv[0]);
        return 2;
    }
    const int w = std::atoi(argv[2]), h = std::atoi(argv[3]), frames = std::atoi(argv[4]);
    if (argc > 6 && std::strcmp(argv[6], "split") == 0) return run_split(argv[1], w, h, frames, argv[5]);
    return run_single(argv[1], w, h, frames, argv[5]);
}
