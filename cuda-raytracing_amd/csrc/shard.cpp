// shard.cpp -- tile plans for the multi-GPU split of one frame.
//
// The reference renders the whole frame on one device (raytracing_process,
// RayTracing/main_raytracing.cu:202-220, 16x16 blocks over W x H).  Every pixel owns its RNG
// subsequence (curand_init(seed, y*W + x), Random.cu:7 + GPUScene.h:95), so any partition of the
// 16x16 tiles over ranks renders bit-identical pixels.  Two plans:
//
//   * round-robin: rank r renders tiles r, r + N, r + 2N, ... (no costs needed; sky and floor
//     rows interleave, so ranks balance to within a few percent);
//   * cost-aware (longest processing time first): tiles sorted by a measured cost (the
//     production kernel's per-wave clocks of one probe frame, rt_render_params.wave_clock),
//     each dealt to the rank with the least cost so far among ranks below the capacity, so each
//     rank's list comes out heaviest tile first -- the expensive waves start at t = 0 and the
//     cheap ones fill the tail.
//
// A plan is [shard_count][capacity] int32 tile ids, -1 padded, identical on every rank that
// computes it from the same costs (deterministic ties: cost, then tile id, then rank).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <numeric>
#include <vector>

#include "rt_abi.h"

void rt_internal_set_error(const char* msg);

static int64_t frame_tiles(int width, int height) {
    return (int64_t)((width + 15) / 16) * (int64_t)((height + 15) / 16);
}

extern "C" int64_t rt_shard_plan_capacity(int width, int height, int shard_count) {
    if (width <= 0 || height <= 0 || shard_count <= 0) return 0;
    const int64_t tiles = frame_tiles(width, height);
    const int64_t even = (tiles + shard_count - 1) / shard_count;
    return std::min<int64_t>(tiles, even + (even + 3) / 4);  // 25 % headroom for uneven cost splits
}

extern "C" int rt_shard_plan(int width, int height, int shard_count, const double* tile_cost, int64_t capacity,
                             int32_t* tile_lists, int64_t* counts) {
    if (width <= 0 || height <= 0 || shard_count <= 0 || !tile_lists || !counts) {
        rt_internal_set_error("rt_shard_plan: bad arguments");
        return 1;
    }
    const int64_t tiles = frame_tiles(width, height);
    if (tiles > ((int64_t)1 << 28) || capacity * shard_count < tiles) {
        rt_internal_set_error("rt_shard_plan: capacity * shard_count < tiles of the frame");
        return 1;
    }
    std::fill(tile_lists, tile_lists + capacity * shard_count, -1);
    std::fill(counts, counts + shard_count, 0);
    if (!tile_cost) {
        for (int64_t t = 0; t < tiles; t++) {
            const int r = (int)(t % shard_count);
            tile_lists[r * capacity + counts[r]++] = (int32_t)t;
        }
        return 0;
    }
    for (int64_t t = 0; t < tiles; t++)
        if (!std::isfinite(tile_cost[t]) || tile_cost[t] < 0) {
            rt_internal_set_error("rt_shard_plan: tile costs must be finite and >= 0");
            return 1;
        }
    std::vector<int32_t> order(tiles);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(),
                     [&](int32_t a, int32_t b) { return tile_cost[a] > tile_cost[b]; });
    std::vector<double> load(shard_count, 0.0);
    for (int32_t t : order) {
        int best = -1;
        for (int r = 0; r < shard_count; r++)
            if (counts[r] < capacity && (best < 0 || load[r] < load[best])) best = r;
        load[best] += tile_cost[t];
        tile_lists[best * capacity + counts[best]++] = t;
    }
    return 0;
}
