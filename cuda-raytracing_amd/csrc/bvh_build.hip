// bvh_build.hip -- the reference's BVH builder (RayTracing/BVH.cpp:8-124) on the GPU, byte-identical
// to the host restatement (scene.cpp BVH::Calculate): same nodes in the same order, same face
// index permutation.
//
// BVH::Subdivide is sequential by construction: a node's triangles are partitioned with a
// two-pointer swap loop (i scans from the front; a triangle whose centroid is not left of the
// split is swapped with the one at j, j--), failed axes leave their permutation behind, and
// children are numbered in the order of the depth-first recursion.  Here every level of the tree
// is built at once:
//
//  * Partition.  The swap loop's result has a closed form.  Let n elements have L "left" ones,
//    take p = L if L == n or element L is left, else L + 1 (elements [0, p) are the ones the
//    front pointer reads, [p, n) the ones the back pointer pulls in, in reverse).  Then element y
//      y < p,  left        -> y
//      y < p,  m-th right  -> n - 1 (m = 1), else (position of the (m-1)-th left counted from
//                             the back among [p, n)) - 1
//      y >= p, m-th left counted from the back -> position of the m-th right in [0, p)
//      y >= p, right       -> y - 1
//    (derivation in DESIGN.md §4.4; tests/test_gpu_bvh.py checks it against the swap loop on
//    random patterns).  Ranks are tile prefix sums; the two "position of the m-th" lookups are
//    scatter tables.  Every node of a level and every tile of a node run in parallel.
//  * Numbering.  BVH::Subdivide allocates a node's two children when it is entered, in
//    pre-order, so the children of inner node v sit at 1 + 2 * (inner nodes before v in
//    pre-order).  That count comes from subtree inner-node counts (bottom-up over the levels)
//    and a top-down pass.
//
// Nodes of at most SMALL triangles build their whole subtree in one thread with the loop itself
// (k_small_subtrees), which removes the deep levels' launches.
//
// Node bounds (UpdateBounds, glm::min / max from +-1e30) are tile reductions; min / max are
// order-independent for finite coordinates, so the result is the sequential one.  Non-finite
// vertex positions are rejected (the host builder handles those scenes).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_abi.h"
#include "rt_math.h"

void rt_internal_set_error(const char* msg);

namespace {

constexpr int TS = 256;  // elements per tile = threads per workgroup
constexpr uint32_t SMALL = 64;  // largest node that may build its whole subtree in one thread

struct BNode {
    uint32_t first, count;
    float bmin[3], bmax[3];
    int32_t left;          // tid of the left child (right = left + 1), -1 for a leaf
    uint32_t inner;        // inner nodes in the subtree (numbering)
    uint32_t before;       // inner nodes before this one in pre-order (numbering)
    uint32_t final_index;  // index in the output array
    // per-level split state
    int32_t axes[3];
    float split;
    uint32_t nleft, p;
    int32_t found;   // 0: still splitting, 1: split found, 2: leaf (one triangle), 3: small subtree
};

// element: centroid.xyz, face index bits
__global__ void k_centroids(const GPUVertex* __restrict__ v, const GPUFace* __restrict__ f, uint32_t n,
                            float4* __restrict__ e) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* p0 = v[f[i].v0].position;
    const float* p1 = v[f[i].v1].position;
    const float* p2 = v[f[i].v2].position;
    // (v0 + v1 + v2) / 3.0f  (BVH.cpp:21), glm component order
    const float cx = ((p0[0] + p1[0]) + p2[0]) / 3.0f;
    const float cy = ((p0[1] + p1[1]) + p2[1]) / 3.0f;
    const float cz = ((p0[2] + p1[2]) + p2[2]) / 3.0f;
    e[i] = make_float4(cx, cy, cz, __uint_as_float(i));
}

__global__ void k_finite(const GPUVertex* __restrict__ v, uint32_t nv, int* bad) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nv) return;
    const float* p = v[i].position;
    if (!(fabsf(p[0]) <= 3.4e38f && fabsf(p[1]) <= 3.4e38f && fabsf(p[2]) <= 3.4e38f)) atomicOr(bad, 1);
}

// tiles of the level's nodes: tile_start = exclusive scan of ceil(count / TS)
__global__ void k_tile_counts(const BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl, uint32_t nl,
                              uint32_t* __restrict__ ntiles) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    ntiles[i] = (nodes[lvl[i]].count + TS - 1) / TS;
}

// which (level slot, tile of node) this workgroup handles; false when past the end
__device__ __forceinline__ bool tile_of(const uint32_t* __restrict__ tile_start, uint32_t nl, uint32_t total,
                                        uint32_t t, uint32_t* slot, uint32_t* k) {
    if (t >= total) return false;
    uint32_t lo = 0, hi = nl;  // last slot with tile_start <= t
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tile_start[mid] <= t) lo = mid;
        else hi = mid;
    }
    *slot = lo;
    *k = t - tile_start[lo];
    return true;
}

// ---------------------------------------------------------------------------------------
// bounds (BVH::UpdateBounds): per tile partial min / max, then per node
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(TS) void k_bounds_tiles(const BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl,
                                                     uint32_t nl, const uint32_t* __restrict__ tile_start,
                                                     uint32_t total, const float4* __restrict__ e,
                                                     const GPUVertex* __restrict__ v, const GPUFace* __restrict__ f,
                                                     float* __restrict__ part) {
    __shared__ float red[6][TS];
    uint32_t slot, k;
    if (!tile_of(tile_start, nl, total, blockIdx.x, &slot, &k)) return;
    const BNode& nd = nodes[lvl[slot]];
    const uint32_t y = k * TS + threadIdx.x;
    float mn[3] = {1e30f, 1e30f, 1e30f}, mx[3] = {-1e30f, -1e30f, -1e30f};
    if (y < nd.count) {
        const uint32_t fi = __float_as_uint(e[nd.first + y].w);
        const uint32_t vi[3] = {f[fi].v0, f[fi].v1, f[fi].v2};
        for (uint32_t q : vi)
            for (int d = 0; d < 3; d++) {
                const float c = v[q].position[d];
                mn[d] = rtm::gmin(mn[d], c);
                mx[d] = rtm::gmax(mx[d], c);
            }
    }
    for (int d = 0; d < 3; d++) red[d][threadIdx.x] = mn[d], red[3 + d][threadIdx.x] = mx[d];
    __syncthreads();
    for (int s = TS / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s)
            for (int d = 0; d < 3; d++) {
                red[d][threadIdx.x] = rtm::gmin(red[d][threadIdx.x], red[d][threadIdx.x + s]);
                red[3 + d][threadIdx.x] = rtm::gmax(red[3 + d][threadIdx.x], red[3 + d][threadIdx.x + s]);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) part[(size_t)blockIdx.x * 6 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void k_bounds_nodes(BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl, uint32_t nl,
                               const uint32_t* __restrict__ tile_start, const float* __restrict__ part, uint32_t small) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    BNode& nd = nodes[lvl[i]];
    float mn[3] = {1e30f, 1e30f, 1e30f}, mx[3] = {-1e30f, -1e30f, -1e30f};
    const uint32_t t0 = tile_start[i], nt = (nd.count + TS - 1) / TS;
    for (uint32_t t = t0; t < t0 + nt; t++)
        for (int d = 0; d < 3; d++) {
            mn[d] = rtm::gmin(mn[d], part[(size_t)t * 6 + d]);
            mx[d] = rtm::gmax(mx[d], part[(size_t)t * 6 + 3 + d]);
        }
    for (int d = 0; d < 3; d++) nd.bmin[d] = mn[d], nd.bmax[d] = mx[d];
    // axis order (BVH.cpp:61-70)
    const float ext[3] = {nd.bmax[0] - nd.bmin[0], nd.bmax[1] - nd.bmin[1], nd.bmax[2] - nd.bmin[2]};
    int a1 = 0;
    if (ext[1] > ext[0]) a1 = 1;
    if (ext[2] > ext[a1]) a1 = 2;
    int a2 = (a1 + 1) % 3, a3 = (a2 + 1) % 3;
    if (ext[a3] > ext[a2]) {
        const int t = a2;
        a2 = a3, a3 = t;
    }
    nd.axes[0] = a1, nd.axes[1] = a2, nd.axes[2] = a3;
    // single triangles never split (and never move); small nodes finish in k_small_subtrees
    nd.found = nd.count < 2 ? 2 : (nd.count <= small ? 3 : 0);
    nd.left = -1;
}

// ---------------------------------------------------------------------------------------
// partition attempt (one axis) for every node of the level that has not split yet
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float comp(float4 c, int a) { return a == 0 ? c.x : (a == 1 ? c.y : c.z); }

// block-wide exclusive prefix of a 0/1 flag and the total (TS threads, wave64)
__device__ __forceinline__ uint32_t block_prefix(bool flag, uint32_t* total, uint32_t* sh) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const unsigned long long b = __ballot(flag);
    const uint32_t in_wave = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    if (lane == 0) sh[w] = (uint32_t)__popcll(b);
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t q = 0; q < TS / 64; q++) {
        before += q < w ? sh[q] : 0u;
        all += sh[q];
    }
    __syncthreads();
    *total = all;
    return before + in_wave;
}

__global__ void k_split_pos(BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl, uint32_t nl, int attempt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    BNode& nd = nodes[lvl[i]];
    if (nd.found) return;
    const int a = nd.axes[attempt];
    const float ext = nd.bmax[a] - nd.bmin[a];
    nd.split = nd.bmin[a] + ext * 0.5f;  // BVH.cpp:82
}

__global__ __launch_bounds__(TS) void k_count_left(const BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl,
                                                   uint32_t nl, const uint32_t* __restrict__ tile_start, uint32_t total,
                                                   const float4* __restrict__ e, int attempt, uint32_t* __restrict__ tl) {
    __shared__ uint32_t sh[TS / 64];
    uint32_t slot, k;
    if (!tile_of(tile_start, nl, total, blockIdx.x, &slot, &k)) return;
    const BNode& nd = nodes[lvl[slot]];
    if (nd.found) return;  // uniform per workgroup
    const uint32_t y = k * TS + threadIdx.x;
    const bool left = y < nd.count && comp(e[nd.first + y], nd.axes[attempt]) < nd.split;
    uint32_t all;
    block_prefix(left, &all, sh);
    if (threadIdx.x == 0) tl[blockIdx.x] = all;
}

// per node: tile offsets of the left counts, L, p, and whether this axis splits
__global__ void k_left_scan(BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl, uint32_t nl,
                            const uint32_t* __restrict__ tile_start, uint32_t* __restrict__ tl,
                            const float4* __restrict__ e, int attempt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    BNode& nd = nodes[lvl[i]];
    if (nd.found) return;
    const uint32_t t0 = tile_start[i], nt = (nd.count + TS - 1) / TS;
    uint32_t run = 0;
    for (uint32_t t = t0; t < t0 + nt; t++) {
        const uint32_t c = tl[t];
        tl[t] = run;  // exclusive
        run += c;
    }
    nd.nleft = run;
    const bool at_l = run < nd.count && comp(e[nd.first + run], nd.axes[attempt]) < nd.split;
    nd.p = (run == nd.count || at_l) ? run : run + 1;
}

// rank tables: rpos[m] = node position of the (m+1)-th right element in [0, p);
// lpos[m] = node position of the (m+1)-th left element counted from the back in [p, n)
__global__ __launch_bounds__(TS) void k_rank_tables(const BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl,
                                                    uint32_t nl, const uint32_t* __restrict__ tile_start,
                                                    uint32_t total, const uint32_t* __restrict__ tl,
                                                    const float4* __restrict__ e, int attempt,
                                                    uint32_t* __restrict__ rpos, uint32_t* __restrict__ lpos) {
    __shared__ uint32_t sh[TS / 64];
    uint32_t slot, k;
    if (!tile_of(tile_start, nl, total, blockIdx.x, &slot, &k)) return;
    const BNode& nd = nodes[lvl[slot]];
    if (nd.found) return;
    const uint32_t y = k * TS + threadIdx.x;
    const bool in = y < nd.count;
    const bool left = in && comp(e[nd.first + y], nd.axes[attempt]) < nd.split;
    uint32_t all;
    const uint32_t lbefore = tl[blockIdx.x] + block_prefix(left, &all, sh);  // lefts in [0, y)
    if (!in) return;
    if (y < nd.p) {
        if (!left) rpos[nd.first + (y - lbefore)] = y;  // rights in [0, y] = y + 1 - lbefore
    } else if (left) {
        lpos[nd.first + (nd.nleft - lbefore - 1)] = y;  // lefts in [y, n) = nleft - lbefore
    }
}

__global__ __launch_bounds__(TS) void k_scatter(const BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl,
                                                uint32_t nl, const uint32_t* __restrict__ tile_start, uint32_t total,
                                                const uint32_t* __restrict__ tl, const float4* __restrict__ e,
                                                int attempt, const uint32_t* __restrict__ rpos,
                                                const uint32_t* __restrict__ lpos, float4* __restrict__ tmp) {
    __shared__ uint32_t sh[TS / 64];
    uint32_t slot, k;
    if (!tile_of(tile_start, nl, total, blockIdx.x, &slot, &k)) return;
    const BNode& nd = nodes[lvl[slot]];
    if (nd.found) return;
    const uint32_t y = k * TS + threadIdx.x;
    const bool in = y < nd.count;
    const float4 c = in ? e[nd.first + y] : make_float4(0, 0, 0, 0);
    const bool left = in && comp(c, nd.axes[attempt]) < nd.split;
    uint32_t all;
    const uint32_t lbefore = tl[blockIdx.x] + block_prefix(left, &all, sh);
    if (!in) return;
    const uint32_t n = nd.count;
    uint32_t out;
    if (y < nd.p) {
        if (left) {
            out = y;
        } else {
            const uint32_t m = y + 1 - lbefore;  // this is the m-th right
            out = m == 1 ? n - 1 : lpos[nd.first + m - 2] - 1;
        }
    } else {
        out = left ? rpos[nd.first + (nd.nleft - lbefore - 1)] : y - 1;
    }
    tmp[nd.first + out] = c;
}

__global__ __launch_bounds__(TS) void k_copy_back(const BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl,
                                                  uint32_t nl, const uint32_t* __restrict__ tile_start, uint32_t total,
                                                  const float4* __restrict__ tmp, float4* __restrict__ e) {
    uint32_t slot, k;
    if (!tile_of(tile_start, nl, total, blockIdx.x, &slot, &k)) return;
    const BNode& nd = nodes[lvl[slot]];
    if (nd.found) return;
    const uint32_t y = k * TS + threadIdx.x;
    if (y < nd.count) e[nd.first + y] = tmp[nd.first + y];
}

__global__ void k_mark_found(BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl, uint32_t nl) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    BNode& nd = nodes[lvl[i]];
    if (!nd.found && nd.nleft != 0 && nd.nleft != nd.count) nd.found = 1;
}

// children (BVH.cpp:110-121) of the nodes that split; append them to the next level
__global__ void k_children(BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl, uint32_t nl,
                           uint32_t* __restrict__ counters, uint32_t* __restrict__ next) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    BNode& nd = nodes[lvl[i]];
    if (nd.found != 1) return;
    const uint32_t l = atomicAdd(&counters[0], 2u);
    const uint32_t s = atomicAdd(&counters[1], 2u);
    nd.left = (int32_t)l;
    BNode& a = nodes[l];
    BNode& b = nodes[l + 1];
    a.first = nd.first, a.count = nd.nleft;
    b.first = nd.first + nd.nleft, b.count = nd.count - nd.nleft;
    next[s] = l, next[s + 1] = l + 1;
}

// ---------------------------------------------------------------------------------------
// small nodes: BVH::Subdivide literally, one thread per subtree (its element range is its own).
// Children come from a block of 2 (count - 1) node slots; `inner` is set for every node of the
// subtree (post-order), the numbering pass below walks it top-down.
// ---------------------------------------------------------------------------------------
__device__ void small_bounds(BNode& nd, const float4* __restrict__ e, const GPUVertex* __restrict__ v,
                             const GPUFace* __restrict__ f) {
    for (int d = 0; d < 3; d++) nd.bmin[d] = 1e30f, nd.bmax[d] = -1e30f;
    for (uint32_t y = 0; y < nd.count; y++) {
        const uint32_t fi = __float_as_uint(e[nd.first + y].w);
        const uint32_t vi[3] = {f[fi].v0, f[fi].v1, f[fi].v2};
        for (uint32_t q : vi)
            for (int d = 0; d < 3; d++) {
                const float c = v[q].position[d];
                nd.bmin[d] = rtm::gmin(nd.bmin[d], c);
                nd.bmax[d] = rtm::gmax(nd.bmax[d], c);
            }
    }
}

__global__ void k_small_subtrees(BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl, uint32_t nl,
                                 float4* __restrict__ e, const GPUVertex* __restrict__ v,
                                 const GPUFace* __restrict__ f, uint32_t* __restrict__ counters, int level) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    const uint32_t root = lvl[i];
    if (nodes[root].found != 3) return;
    uint32_t next = atomicAdd(&counters[0], 2u * (nodes[root].count - 1u));
    const uint32_t block_end = next + 2u * (nodes[root].count - 1u);
    uint32_t stack[2 * SMALL];
    int depth_of[2 * SMALL];
    uint32_t order[2 * SMALL];  // pre-order of the subtree, for the post-order inner counts
    uint32_t sp = 0, no = 0;
    int maxd = level;
    stack[sp] = root, depth_of[sp++] = level;
    while (sp) {
        sp--;
        const uint32_t k = stack[sp];
        const int dk = depth_of[sp];
        maxd = max(maxd, dk);
        order[no++] = k;
        BNode& nd = nodes[k];
        nd.left = -1;
        if (nd.count < 2) continue;
        const float ext[3] = {nd.bmax[0] - nd.bmin[0], nd.bmax[1] - nd.bmin[1], nd.bmax[2] - nd.bmin[2]};
        int a1 = 0;
        if (ext[1] > ext[0]) a1 = 1;
        if (ext[2] > ext[a1]) a1 = 2;
        int a2 = (a1 + 1) % 3, a3 = (a2 + 1) % 3;
        if (ext[a3] > ext[a2]) {
            const int t = a2;
            a2 = a3, a3 = t;
        }
        const int axes[3] = {a1, a2, a3};
        bool found = false;
        int ii = 0, left_count = 0;
        for (int q = 0; q < 3 && !found; q++) {
            const int ax = axes[q];
            const float split = nd.bmin[ax] + ext[ax] * 0.5f;
            ii = (int)nd.first;
            int jj = ii + (int)nd.count - 1;
            while (ii <= jj) {
                if (comp(e[ii], ax) < split) {
                    ii++;
                } else {
                    const float4 t = e[ii];
                    e[ii] = e[jj];
                    e[jj--] = t;
                }
            }
            left_count = ii - (int)nd.first;
            found = left_count != 0 && left_count != (int)nd.count;
        }
        if (!found) continue;
        const uint32_t l = next;
        next += 2;
        nd.left = (int32_t)l;
        BNode& a = nodes[l];
        BNode& b = nodes[l + 1];
        a.first = nd.first, a.count = (uint32_t)left_count;
        b.first = (uint32_t)ii, b.count = nd.count - (uint32_t)left_count;
        small_bounds(a, e, v, f);
        small_bounds(b, e, v, f);
        stack[sp] = l + 1, depth_of[sp++] = dk + 1;  // left popped first (pre-order)
        stack[sp] = l, depth_of[sp++] = dk + 1;
    }
    for (uint32_t u = next; u < block_end; u++) nodes[u].final_index = ~0u;  // unused slots
    for (uint32_t q = no; q-- > 0;) {  // reverse pre-order: children before parents
        BNode& nd = nodes[order[q]];
        nd.inner = nd.left < 0 ? 0u : 1u + nodes[nd.left].inner + nodes[nd.left + 1].inner;
    }
    atomicMax(&counters[2], (uint32_t)maxd);
}

__global__ void k_small_number(BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl, uint32_t nl) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    const uint32_t root = lvl[i];
    if (nodes[root].found != 3) return;
    uint32_t stack[2 * SMALL];
    uint32_t sp = 0;
    stack[sp++] = root;
    while (sp) {
        const BNode& nd = nodes[stack[--sp]];
        if (nd.left < 0) continue;
        BNode& a = nodes[nd.left];
        BNode& b = nodes[nd.left + 1];
        const uint32_t c = 1u + 2u * nd.before;
        a.final_index = c, b.final_index = c + 1;
        a.before = nd.before + 1u;
        b.before = a.before + a.inner;
        stack[sp++] = nd.left + 1;
        stack[sp++] = nd.left;
    }
}

// numbering: inner-node counts bottom-up, pre-order ranks top-down
__global__ void k_inner_up(BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl, uint32_t nl) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    BNode& nd = nodes[lvl[i]];
    nd.inner = nd.left < 0 ? 0u : 1u + nodes[nd.left].inner + nodes[nd.left + 1].inner;
}

__global__ void k_rank_down(BNode* __restrict__ nodes, const uint32_t* __restrict__ lvl, uint32_t nl) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    const BNode& nd = nodes[lvl[i]];
    if (nd.left < 0) return;
    BNode& a = nodes[nd.left];
    BNode& b = nodes[nd.left + 1];
    const uint32_t c = 1u + 2u * nd.before;  // children slots allocated when nd was subdivided
    a.final_index = c, b.final_index = c + 1;
    a.before = nd.before + 1u;
    b.before = a.before + a.inner;
}

__global__ void k_emit(const BNode* __restrict__ nodes, uint32_t count, GPUBVHNode* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const BNode& nd = nodes[i];
    if (nd.final_index == ~0u) return;  // a small subtree's unused slot
    GPUBVHNode o;
    for (int d = 0; d < 3; d++) o.bmin[d] = nd.bmin[d], o.bmax[d] = nd.bmax[d];
    if (nd.left >= 0) {
        o.first_index = 1u + 2u * nd.before;
        o.prim_count = 0;
    } else {
        o.first_index = nd.first;
        o.prim_count = nd.count;
    }
    out[nd.final_index] = o;
}

__global__ void k_indices(const float4* __restrict__ e, uint32_t n, uint32_t* __restrict__ fi) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) fi[i] = __float_as_uint(e[i].w);
}

struct Dev {
    std::vector<void*> ptrs;
    ~Dev() {
        for (void* p : ptrs) (void)hipFree(p);
    }
    template <class T>
    T* alloc(size_t n) {
        void* p = nullptr;
        if (hipMalloc(&p, n * sizeof(T) + 16) != hipSuccess) return nullptr;
        ptrs.push_back(p);
        return static_cast<T*>(p);
    }
};

int fail(const std::string& m) {
    rt_internal_set_error(m.c_str());
    return 1;
}

inline unsigned blocks(size_t n, unsigned b = 256) { return (unsigned)((n + b - 1) / b); }

}  // namespace

extern "C" int rt_bvh_build_device(const GPUVertex* vertices, uint32_t vertex_count, const GPUFace* faces,
                                   uint32_t face_count, GPUBVHNode* nodes_out, uint32_t* face_indices_out,
                                   uint32_t* node_count_out, int* max_depth_out, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    rt_build_options opt;
    rt_get_build_options(&opt);  // rt_build_options.bvh_small, 2..SMALL
    const uint32_t small = opt.bvh_small < 2u ? 2u : (opt.bvh_small > SMALL ? SMALL : opt.bvh_small);
    if (!vertices || !faces || !nodes_out || !face_indices_out || face_count == 0)
        return fail("rt_bvh_build_device: bad arguments");
    const uint32_t n = face_count;
    Dev d;
    float4* e = d.alloc<float4>(n);
    float4* tmp = d.alloc<float4>(n);
    uint32_t* rpos = d.alloc<uint32_t>(n);
    uint32_t* lpos = d.alloc<uint32_t>(n);
    BNode* nodes = d.alloc<BNode>(2 * (size_t)n);
    uint32_t* lvlbuf = d.alloc<uint32_t>(2 * (size_t)n);  // all levels' node lists, back to back
    const size_t max_tiles = (size_t)n / TS + 2 * (size_t)n + 1;  // generous: <= n / TS + nodes
    uint32_t* ntiles = d.alloc<uint32_t>(2 * (size_t)n + 1);
    uint32_t* tile_start = d.alloc<uint32_t>(2 * (size_t)n + 1);
    uint32_t* tl = d.alloc<uint32_t>(max_tiles);
    float* part = d.alloc<float>(max_tiles * 6);
    uint32_t* counters = d.alloc<uint32_t>(4);
    int* bad = d.alloc<int>(1);
    if (!e || !tmp || !rpos || !lpos || !nodes || !lvlbuf || !ntiles || !tile_start || !tl || !part || !counters || !bad)
        return fail("rt_bvh_build_device: out of device memory");

    hipMemsetAsync(bad, 0, sizeof(int), st);
    hipLaunchKernelGGL(k_finite, dim3(blocks(vertex_count)), dim3(256), 0, st, vertices, vertex_count, bad);
    hipLaunchKernelGGL(k_centroids, dim3(blocks(n)), dim3(256), 0, st, vertices, faces, n, e);
    // root: tid 0, level 0 = [0]
    BNode root{};
    root.first = 0, root.count = n, root.left = -1, root.before = 0, root.final_index = 0;
    hipMemcpyAsync(nodes, &root, sizeof(BNode), hipMemcpyHostToDevice, st);
    const uint32_t zero_lvl = 0;
    hipMemcpyAsync(lvlbuf, &zero_lvl, 4, hipMemcpyHostToDevice, st);
    uint32_t cnt[3] = {1, 0, 0};  // nodes allocated, next-level size, deepest small-subtree node
    hipMemcpyAsync(counters, cnt, 12, hipMemcpyHostToDevice, st);

    // temp storage for the tile scan
    size_t scan_bytes = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, ntiles, tile_start, (int)(2 * (size_t)n), st);
    void* scan_tmp = d.alloc<char>(scan_bytes);
    if (!scan_tmp) return fail("rt_bvh_build_device: out of device memory");

    std::vector<uint32_t> level_off{0}, level_n{1};
    uint32_t nl = 1, off = 0;
    int depth = 0;
    while (nl > 0) {
        uint32_t* lvl = lvlbuf + off;
        hipLaunchKernelGGL(k_tile_counts, dim3(blocks(nl)), dim3(256), 0, st, nodes, lvl, nl, ntiles);
        hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, ntiles, tile_start, (int)nl, st);
        uint32_t last[2];
        hipMemcpyAsync(&last[0], tile_start + nl - 1, 4, hipMemcpyDeviceToHost, st);
        hipMemcpyAsync(&last[1], ntiles + nl - 1, 4, hipMemcpyDeviceToHost, st);
        if (hipStreamSynchronize(st) != hipSuccess) return fail("rt_bvh_build_device: level sync failed");
        const uint32_t total = last[0] + last[1];
        hipLaunchKernelGGL(k_bounds_tiles, dim3(total), dim3(TS), 0, st, nodes, lvl, nl, tile_start, total, e, vertices,
                           faces, part);
        hipLaunchKernelGGL(k_bounds_nodes, dim3(blocks(nl)), dim3(256), 0, st, nodes, lvl, nl, tile_start, part, small);
        for (int attempt = 0; attempt < 3; attempt++) {
            hipLaunchKernelGGL(k_split_pos, dim3(blocks(nl)), dim3(256), 0, st, nodes, lvl, nl, attempt);
            hipLaunchKernelGGL(k_count_left, dim3(total), dim3(TS), 0, st, nodes, lvl, nl, tile_start, total, e, attempt,
                               tl);
            hipLaunchKernelGGL(k_left_scan, dim3(blocks(nl)), dim3(256), 0, st, nodes, lvl, nl, tile_start, tl, e,
                               attempt);
            hipLaunchKernelGGL(k_rank_tables, dim3(total), dim3(TS), 0, st, nodes, lvl, nl, tile_start, total, tl, e,
                               attempt, rpos, lpos);
            hipLaunchKernelGGL(k_scatter, dim3(total), dim3(TS), 0, st, nodes, lvl, nl, tile_start, total, tl, e, attempt,
                               rpos, lpos, tmp);
            hipLaunchKernelGGL(k_copy_back, dim3(total), dim3(TS), 0, st, nodes, lvl, nl, tile_start, total, tmp, e);
            hipLaunchKernelGGL(k_mark_found, dim3(blocks(nl)), dim3(256), 0, st, nodes, lvl, nl);
        }
        hipLaunchKernelGGL(k_small_subtrees, dim3(blocks(nl, 64)), dim3(64), 0, st, nodes, lvl, nl, e, vertices, faces,
                           counters, depth);
        const uint32_t next_off = off + nl;
        hipMemsetAsync(counters + 1, 0, 4, st);
        hipLaunchKernelGGL(k_children, dim3(blocks(nl)), dim3(256), 0, st, nodes, lvl, nl, counters, lvlbuf + next_off);
        uint32_t nn = 0;
        hipMemcpyAsync(&nn, counters + 1, 4, hipMemcpyDeviceToHost, st);
        if (hipStreamSynchronize(st) != hipSuccess) return fail("rt_bvh_build_device: level sync failed");
        if (hipGetLastError() != hipSuccess) return fail("rt_bvh_build_device: kernel launch failed");
        off = next_off;
        nl = nn;
        if (nl) {
            level_off.push_back(off);
            level_n.push_back(nl);
            depth++;
        }
    }
    int badv = 0;
    hipMemcpyAsync(&badv, bad, sizeof(int), hipMemcpyDeviceToHost, st);
    uint32_t total_nodes = 0, small_depth = 0;
    hipMemcpyAsync(&total_nodes, counters, 4, hipMemcpyDeviceToHost, st);
    hipMemcpyAsync(&small_depth, counters + 2, 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) return fail("rt_bvh_build_device: sync failed");
    if (badv) return fail("rt_bvh_build_device: non-finite vertex positions (use the host builder)");
    // numbering: bottom-up inner counts, top-down pre-order ranks
    for (size_t L = level_off.size(); L-- > 0;)
        hipLaunchKernelGGL(k_inner_up, dim3(blocks(level_n[L])), dim3(256), 0, st, nodes, lvlbuf + level_off[L],
                           level_n[L]);
    for (size_t L = 0; L < level_off.size(); L++)
        hipLaunchKernelGGL(k_rank_down, dim3(blocks(level_n[L])), dim3(256), 0, st, nodes, lvlbuf + level_off[L],
                           level_n[L]);
    for (size_t L = 0; L < level_off.size(); L++)
        hipLaunchKernelGGL(k_small_number, dim3(blocks(level_n[L], 64)), dim3(64), 0, st, nodes, lvlbuf + level_off[L],
                           level_n[L]);
    hipLaunchKernelGGL(k_emit, dim3(blocks(total_nodes)), dim3(256), 0, st, nodes, total_nodes, nodes_out);
    uint32_t root_inner = 0;
    hipMemcpyAsync(&root_inner, &nodes[0].inner, 4, hipMemcpyDeviceToHost, st);
    hipLaunchKernelGGL(k_indices, dim3(blocks(n)), dim3(256), 0, st, e, n, face_indices_out);
    if (hipStreamSynchronize(st) != hipSuccess || hipGetLastError() != hipSuccess)
        return fail("rt_bvh_build_device: numbering failed");
    if (node_count_out) *node_count_out = 1u + 2u * root_inner;  // nodes_used
    if (max_depth_out) *max_depth_out = depth > (int)small_depth ? depth : (int)small_depth;
    return 0;
}
