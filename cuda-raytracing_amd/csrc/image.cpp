// image.cpp -- frame files: PFM (linear RGB, the surface itself) and binary PPM (the viewer's
// tonemapped 8-bit image, image.hip).  Host code; buffers are host memory.
#include <cstdint>
#include <cstdio>
#include <vector>

#include "mirror.h"  // rt_internal_set_error
#include "rt_abi.h"

// Portable float map: "PF", width height, scale -1 (little-endian), rows bottom to top --
// the surface's own row order (row 0 = the bottom scanline, GPUScene.h:13).
extern "C" int rt_write_pfm(const char* path, const float* rgba, uint64_t pitch, int width, int height) {
    if (!path || !rgba || width <= 0 || height <= 0 || pitch < (uint64_t)width * 16) {
        rt_internal_set_error("rt_write_pfm: bad arguments");
        return 1;
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        rt_internal_set_error("rt_write_pfm: cannot open the file");
        return 2;
    }
    std::fprintf(f, "PF\n%d %d\n-1.0\n", width, height);
    std::vector<float> row((size_t)width * 3);
    bool ok = true;
    for (int y = 0; y < height && ok; y++) {
        const float* src = reinterpret_cast<const float*>(reinterpret_cast<const char*>(rgba) + (size_t)y * pitch);
        for (int x = 0; x < width; x++)
            for (int c = 0; c < 3; c++) row[(size_t)x * 3 + c] = src[(size_t)x * 4 + c];
        ok = std::fwrite(row.data(), sizeof(float), row.size(), f) == row.size();
    }
    if (std::fclose(f) != 0 || !ok) {
        rt_internal_set_error("rt_write_pfm: write failed");
        return 3;
    }
    return 0;
}

// Binary PPM (P6) of top-to-bottom RGB8 rows (rt_tonemap_srgb8's output).
extern "C" int rt_write_ppm(const char* path, const uint8_t* rgb, int width, int height) {
    if (!path || !rgb || width <= 0 || height <= 0) {
        rt_internal_set_error("rt_write_ppm: bad arguments");
        return 1;
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        rt_internal_set_error("rt_write_ppm: cannot open the file");
        return 2;
    }
    std::fprintf(f, "P6\n%d %d\n255\n", width, height);
    const size_t n = (size_t)width * height * 3;
    const bool ok = std::fwrite(rgb, 1, n, f) == n;
    if (std::fclose(f) != 0 || !ok) {
        rt_internal_set_error("rt_write_ppm: write failed");
        return 3;
    }
    return 0;
}
