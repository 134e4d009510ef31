// rt_wave.h -- wavefront render path (rt_wave.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "rt_common.h"

namespace rtwave {

// Per-frame path state, SoA arrays of n pixel slots (device memory, cached per stream).
struct WaveWS {
    uint32_t n;
    uint32_t* ctl;  // [0..1] queue counts, [2..3] queue read heads
    float *ro, *rd, *thr, *col;  // [3][n]
    float* acc;                  // [4][n]
    float *hit_t, *hit_bx, *hit_by;
    int *bounce, *sample;
    uint32_t* hit_id;
    uint32_t* queue[2];
    uint32_t* rng;  // [6][n]: d, v0..v4
};

}  // namespace rtwave

// Render one frame (or shard) with the wavefront kernels on `stream`.
hipError_t rt_wave_render(const rtk::RenderArgs& a, int tiles, int depth, bool stats, hipStream_t stream);
