// image.hip -- the display transform of the reference's viewer, for looking at frames.
//
// main.cpp draws the float4 surface as a full-screen quad (main.cpp:66-76, quad rect at
// main.cpp:723) through a pixel shader that scales by exposure 0.5 and applies the ACES film
// curve with saturate (main.cpp:78-94), into a DXGI_FORMAT_R8G8B8A8_UNORM_SRGB back buffer
// (main.cpp:438): the output merger encodes linear -> sRGB on write.  At a 1:1 window the
// linear sampler reads texel centres, so the transform is per pixel.  Texture row 0 (the
// surface's row 0, the bottom scanline: GPUScene.h:13) lands at the bottom of the screen; this
// kernel writes rows top to bottom, the order image files and displays use.  Viewing only: the
// sRGB encode here is the IEC formula in fp32, not any GPU's hardware conversion.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mirror.h"  // rt_internal_set_error
#include "rt_abi.h"

namespace {

__device__ __forceinline__ float saturate(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }  // NaN -> 0

__device__ __forceinline__ float aces_film(float x) {  // main.cpp:81-89
    const float a = 2.51f, b = 0.03f, c = 2.43f, d = 0.59f, e = 0.14f;
    return saturate((x * (a * x + b)) / (x * (c * x + d) + e));
}

__device__ __forceinline__ uint8_t srgb8(float l) {
    const float s = l <= 0.0031308f ? 12.92f * l : 1.055f * powf(l, 1.0f / 2.4f) - 0.055f;
    return (uint8_t)(saturate(s) * 255.0f + 0.5f);
}

// one thread per pixel; a row of the surface is read with 16-byte loads (coalesced)
__global__ __launch_bounds__(256) void tonemap_kernel(const char* surface, uint64_t pitch, int width, int height,
                                                      uint8_t* out) {
    const int x = blockIdx.x * 256 + threadIdx.x, row = blockIdx.y;
    if (x >= width) return;
    const float4 c = *reinterpret_cast<const float4*>(surface + (size_t)(height - 1 - row) * pitch + (size_t)x * 16);
    const float exposure = 0.5f;
    uint8_t* o = out + ((size_t)row * width + x) * 3;
    o[0] = srgb8(aces_film(c.x * exposure));
    o[1] = srgb8(aces_film(c.y * exposure));
    o[2] = srgb8(aces_film(c.z * exposure));
}

}  // namespace

extern "C" int rt_tonemap_srgb8(const void* surface, uint64_t pitch, int width, int height, uint8_t* out_rgb,
                                void* stream) {
    if (!surface || !out_rgb || width <= 0 || height <= 0 || pitch < (uint64_t)width * 16) {
        rt_internal_set_error("rt_tonemap_srgb8: bad arguments");
        return 1;
    }
    hipLaunchKernelGGL(tonemap_kernel, dim3((width + 255) / 256, height), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const char*>(surface), pitch, width, height, out_rgb);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        rt_internal_set_error(hipGetErrorString(e));
        return 2;
    }
    return 0;
}
