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

// ---------------------------------------------------------------------------------------
// Lane plans (rt_render_params.lane_slots).  A wave takes as long as the union of its lanes'
// traversal steps, so a 64-pixel wave of expensive pixels (rays trapped between the bunny's base
// and the floor leaf) runs ~4x longer than its costliest pixel alone: the heaviest 16x16 tile of
// config 2 renders in 9.6 ms as 4 waves of 64 pixels, 6.8 ms as 16 waves of 16, 3.9 ms as 64
// waves of 4 and 2.4 ms as 256 one-pixel waves (bit-identical; tools/heavy_probe.py) -- about
// max x (pixels)^0.34.  Once a frame is split over enough ranks, those waves are each rank's
// whole frame time.
//
// Model: a wave of pixels with probe-frame work c_i (rt_render_params.lane_cost) takes about
// E = max c x (sum c / max c)^0.34 work units, a lone lane running one unit per unit of time;
// the whole rank needs about sum c / P units of time when the GPU is full, P = the lanes' worth
// of work the device does in parallel (MI355X, config 2: 16.4 ms for 634 M units, 2.4 ms for the
// 3,970-unit pixel alone: P ~ 24,000 by this estimate; swept on the device, P = 48,000 gave the
// fastest shards for configs 2 and 3 at N = 2-8, and bench.py --lane-units ships that).  The plan keeps every 8x8 sub-tile wave whose E is within
// the target B = slack x max(max c, sum c / P) and splits the others (their pixels in decreasing
// work, first fit into sub-waves of E <= B: pixels of one sub-tile stay together, so their rays
// stay coherent).  Waves with E >= B / 2 go first, longest first (the tail starts at t = 0), the
// rest follow in list order (cost-ordered plans put the heaviest tiles first).
// ---------------------------------------------------------------------------------------
namespace {
constexpr double kLaneExp = 0.34;  // wave time ~ max x (sum / max)^0.34 (measured, see above)

double wave_units(double mx, double sum) { return mx > 0 ? mx * std::pow(sum / mx, kLaneExp) : 0.0; }
}  // namespace

extern "C" int64_t rt_lane_plan_capacity(int64_t slots) {
    if (slots <= 0 || slots % 64 != 0) return 0;
    return 4 * slots;  // splitting stops once the plan holds four times the sub-tile waves
}

extern "C" int64_t rt_lane_plan(const uint32_t* cost, int64_t slots, double parallel_units, double slack,
                                int32_t* lane_slots, int64_t capacity, int64_t* long_waves) {
    if (!cost || !lane_slots || slots <= 0 || slots % 64 != 0 || slots > ((int64_t)1 << 30) ||
        capacity < rt_lane_plan_capacity(slots) || !(slack > 0) || !(parallel_units == parallel_units)) {
        rt_internal_set_error("rt_lane_plan: bad arguments (slots must be a positive multiple of 64, capacity >= "
                              "rt_lane_plan_capacity(slots), slack > 0)");
        return -1;
    }
    const int64_t nw = slots / 64, max_waves = capacity / 64;
    constexpr uint32_t LONE = 0xffffffffu;  // rt_lone_plan: rendered by the lone-pixel kernel, not here
    auto cst = [&](int32_t s) { return cost[s] == LONE ? 0.0 : (double)cost[s]; };
    double cmax = 0, csum = 0;
    for (int64_t s = 0; s < slots; s++) cmax = std::max(cmax, cst((int32_t)s)), csum += cst((int32_t)s);
    const double B = parallel_units > 0 ? slack * std::max(cmax, csum / parallel_units) : 0.0;
    struct Wave {
        std::vector<int32_t> lanes;
        double mx = 0, sum = 0;
        int64_t order = 0;
    };
    // sub-tile waves, split longest first (so a capped plan leaves only the shortest ones whole)
    std::vector<Wave> tile(nw);
    std::vector<double> e0(nw);
    for (int64_t w = 0; w < nw; w++) {
        tile[w].order = w;
        for (int l = 0; l < 64; l++) {
            const int32_t s = (int32_t)(w * 64 + l);
            if (cost[s] == LONE) continue;
            tile[w].lanes.push_back(s);
            tile[w].mx = std::max(tile[w].mx, cst(s)), tile[w].sum += cst(s);
        }
        e0[w] = wave_units(tile[w].mx, tile[w].sum);
    }
    std::vector<int64_t> by_e(nw);
    std::iota(by_e.begin(), by_e.end(), 0);
    std::stable_sort(by_e.begin(), by_e.end(), [&](int64_t a, int64_t b) { return e0[a] > e0[b]; });
    std::vector<std::vector<Wave>> split(nw);
    int64_t total = nw;
    for (int64_t w : by_e) {
        if (B <= 0 || e0[w] <= B) break;
        std::vector<int32_t> by = tile[w].lanes;
        std::stable_sort(by.begin(), by.end(), [&](int32_t a, int32_t b) { return cst(a) > cst(b); });
        std::vector<Wave> sub;
        for (int32_t s : by) {
            const double c = cst(s);
            bool placed = false;
            for (Wave& v : sub)
                if (v.lanes.size() < 64 && (c == 0 || wave_units(v.mx, v.sum + c) <= B)) {  // v.mx >= c (decreasing)
                    v.lanes.push_back(s), v.sum += c, placed = true;
                    break;
                }
            if (!placed) {
                Wave v;
                v.order = w, v.mx = c, v.sum = c;
                v.lanes.push_back(s);
                sub.push_back(std::move(v));
            }
        }
        if (total + (int64_t)sub.size() - 1 > max_waves) break;  // no room: the rest stay whole
        total += (int64_t)sub.size() - 1;
        split[w] = std::move(sub);
    }
    std::vector<Wave> out;
    out.reserve(total);
    for (int64_t w = 0; w < nw; w++) {
        if (!split[w].empty())
            for (Wave& v : split[w]) out.push_back(std::move(v));
        else if (!tile[w].lanes.empty())  // a sub-tile whose pixels all went to the lone-pixel kernel
            out.push_back(std::move(tile[w]));
    }
    // long waves (E >= B / 2) first, longest first; then the others in list order
    std::vector<double> e(out.size());
    for (size_t i = 0; i < out.size(); i++) e[i] = wave_units(out[i].mx, out[i].sum);
    std::vector<int64_t> idx(out.size());
    std::iota(idx.begin(), idx.end(), 0);
    int64_t nlong = 0;
    for (size_t i = 0; i < out.size(); i++) nlong += (B > 0 && e[i] >= 0.5 * B) ? 1 : 0;
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) {
        const bool la = B > 0 && e[a] >= 0.5 * B, lb = B > 0 && e[b] >= 0.5 * B;
        if (la != lb) return la;
        if (la) return e[a] > e[b];
        return out[a].order < out[b].order;
    });
    int64_t n = 0;
    for (int64_t i : idx) {
        const Wave& v = out[i];
        for (int l = 0; l < 64; l++) lane_slots[n + l] = l < (int)v.lanes.size() ? v.lanes[l] : -1;
        n += 64;
    }
    if (long_waves) *long_waves = nlong;
    return n;
}

// Measured refinement of a lane map.  The model above prices a wave from its pixels' probe work;
// on the device, multi-pixel waves at the target take about twice as long as the single costliest
// pixel (which runs its DFS with the whole wave, rt_fast.h lone_traverse), so at N = 8 the plan's
// long waves are each rank's frame.  Here the waves a timing frame of the map itself MEASURED
// within `theta` of the longest (wave_ticks: rt_render_params.wave_clock) are split in two -- their
// pixels in decreasing probe work dealt alternately, so each half keeps every other of the
// costliest -- and all waves are ordered by expected duration, longest first (a half at 3/4 of its
// parent's clock).  The caller times the new map and keeps it only if the frame got faster
// (bench.py refine_lane_map).  A lane map is a permutation of the shard's slots, so any refinement
// renders the same pixels bit for bit.
extern "C" int64_t rt_lane_refine(const int32_t* lane_slots, int64_t entries, const uint32_t* cost, int64_t slots,
                                  const int64_t* wave_ticks, double theta, int32_t* out, int64_t capacity,
                                  int64_t* split_waves) {
    if (!lane_slots || !cost || !wave_ticks || !out || entries <= 0 || entries % 64 != 0 || slots <= 0 ||
        slots > ((int64_t)1 << 30) || entries > ((int64_t)1 << 32) || capacity < 2 * entries || !(theta > 0) ||
        !(theta <= 1)) {
        rt_internal_set_error("rt_lane_refine: bad arguments (entries a positive multiple of 64, capacity >= 2 * entries, "
                              "0 < theta <= 1)");
        return -1;
    }
    const int64_t nw = entries / 64;
    int64_t longest = 0;
    for (int64_t w = 0; w < nw; w++) {
        if (wave_ticks[w] < 0) {
            rt_internal_set_error("rt_lane_refine: negative wave clock");
            return -1;
        }
        longest = std::max(longest, wave_ticks[w]);
    }
    for (int64_t i = 0; i < entries; i++)
        if (lane_slots[i] < -1 || lane_slots[i] >= slots) {
            rt_internal_set_error("rt_lane_refine: lane map entry outside [-1, slots)");
            return -1;
        }
    const double cut = theta * (double)longest;
    struct Wave {
        std::vector<int32_t> lanes;
        double est;
    };
    std::vector<Wave> waves;
    waves.reserve(2 * nw);
    int64_t nsplit = 0;
    for (int64_t w = 0; w < nw; w++) {
        Wave v;
        for (int l = 0; l < 64; l++)
            if (lane_slots[w * 64 + l] >= 0) v.lanes.push_back(lane_slots[w * 64 + l]);
        if (v.lanes.empty()) continue;
        v.est = (double)wave_ticks[w];
        if (longest > 0 && v.est >= cut && v.lanes.size() > 1) {
            std::vector<int32_t> by = v.lanes;
            std::stable_sort(by.begin(), by.end(), [&](int32_t a, int32_t b) { return cost[a] > cost[b]; });
            Wave h[2];
            for (size_t i = 0; i < by.size(); i++) h[i & 1].lanes.push_back(by[i]);
            for (Wave& x : h) {
                x.est = 0.75 * v.est;
                waves.push_back(std::move(x));
            }
            nsplit += 2;
        } else {
            waves.push_back(std::move(v));
        }
    }
    std::vector<int64_t> idx(waves.size());
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return waves[a].est > waves[b].est; });
    int64_t n = 0;
    for (int64_t i : idx) {
        const Wave& v = waves[i];
        for (int l = 0; l < 64; l++) out[n + l] = l < (int)v.lanes.size() ? v.lanes[l] : -1;
        n += 64;
    }
    if (split_waves) *split_waves = nsplit;
    return n;
}

// Lone-pixel plans (rt_render_params.lone_slots, rt_lone.hip): the costliest pixels of the probe
// frame, each to be rendered by a wave of its own, are taken out of the lane plan.
extern "C" int64_t rt_lone_plan(uint32_t* cost, int64_t slots, int64_t max_lone, uint32_t min_cost, int32_t* lone_slots) {
    if (!cost || slots <= 0 || slots > ((int64_t)1 << 30) || max_lone < 0 || (max_lone > 0 && !lone_slots)) {
        rt_internal_set_error("rt_lone_plan: bad arguments");
        return -1;
    }
    std::vector<int32_t> cand;
    for (int64_t s = 0; s < slots; s++)
        if (cost[s] != 0xffffffffu && cost[s] >= min_cost && cost[s] > 0) cand.push_back((int32_t)s);
    std::stable_sort(cand.begin(), cand.end(), [&](int32_t a, int32_t b) { return cost[a] > cost[b]; });
    const int64_t n = std::min<int64_t>(max_lone, (int64_t)cand.size());
    for (int64_t i = 0; i < n; i++) {
        lone_slots[i] = cand[i];
        cost[cand[i]] = 0xffffffffu;
    }
    return n;
}
