// host_driver.cpp -- a C++ host driving librt_hip.so through include/rt_abi.h the way the
// reference's CUDARayTracer drives its CUDA kernels (RayTracing/RayTracing.cpp:205-234,
// 216-221): init_rng over ceil(W*H/128) blocks of 128 states, Scene::Upload, then per frame
// raytracing_process(surface, last, ...) followed by the D2D copy of surface into last.
// Writes the final frame (W*H float4, rows bottom-up, pitch removed) to argv[1].
//
//   g++ -std=c++17 -Iinclude tests/cpp/host_driver.cpp -Lcuda-raytracing_amd -lrt_hip -o host_driver
//   ./host_driver out.bin W H frames assets_dir
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rt_abi.h"

#define CHECK(x)                                                              \
    do {                                                                      \
        if ((x) != 0) {                                                       \
            std::fprintf(stderr, "%s failed: %s\n", #x, rt_last_error());     \
            std::exit(1);                                                     \
        }                                                                     \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s out.bin W H frames assets_dir\n", argv[0]);
        return 2;
    }
    const int w = std::atoi(argv[2]), h = std::atoi(argv[3]), frames = std::atoi(argv[4]);
    rt_scene* scene = rt_scene_create();
    CHECK(rt_scene_setup(scene, 0, argv[5]));  // Cornell box + bunny, RayTracing.cpp:24-25
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
    std::vector<char> img(pitch * h);
    CHECK(rt_memcpy_d2h(img.data(), surface, img.size()));
    FILE* out = std::fopen(argv[1], "wb");
    if (!out) return 1;
    for (int y = 0; y < h; y++) std::fwrite(img.data() + (size_t)y * pitch, 16, (size_t)w, out);
    std::fclose(out);
    rt_free(surface);
    rt_free(last);
    rt_free(rng);
    rt_scene_destroy(scene);
    std::printf("ok %dx%d frames=%d pitch=%zu\n", w, h, frames, pitch);
    return 0;
}
