// leaftree.h -- acceleration inside huge BVH leaves.
//
// The reference's midpoint builder (BVH.cpp:60-124) can leave very large leaves -- the 4-bunny
// scene (BASELINE configs[3]) has one of 12,318 triangles -- and BVHRayHit tests every
// triangle of a leaf in order.  For such a leaf the mirror also holds a small tree over its
// triangles; the kernel walks it (rt_fast.h tree_leaf) and skips a subtree only when
// cluster_cull PROVES that none of its triangles can pass the reference's fp32 triangle test
// with 0 <= t < closest.  What is tested gives exactly the sequential result: candidates are
// compared by (t, position in the leaf), and a NaN distance sends the ray back to the
// sequential loop.
//
// Node record, 64 B (pre-order; a node's first child follows it, `skip` = the node after its
// subtree):
//   K0 = (box.lo.xyz, E1)      E1   = max over the subtree of max(|e1|_1, |e2|_1)
//   K1 = (box.hi.xyz, Nmin)    Nmin = min |e2 x e1| (exact, rounded down)
//   K2 = (axis.xyz, cos)       normal cone: every triangle normal's LINE is within acos(cos)
//   K3 = (sin, skip, tri_begin, info)         of the fp32 axis; info bit 0 = cullable,
//                                             bits 8.. = triangle count of a cluster
// Boxes and cones are rounded outward, so they bound the exact fp32 triangles.  tri_begin
// indexes the leaf-tree triangle records (FlatTri with C.z = position in the leaf), ~0 for
// inner nodes.
//
// Flat lists for the cooperative walk (rt_fast.h coop_tree), appended to a separate array:
//   clusters  copies of the tree's cluster nodes in pre-order (K3.y = own index + 1);
//   cuts      a cut of the tree into subtrees of at most LeafTreeParams::cut_clusters clusters:
//             copies of those nodes with K3.y = first cluster, K3.z = end cluster (the
//             subtree's clusters are contiguous in pre-order).
// Both lists are stored field-major: field Kf of record i of a list of n records at float4
// index base + f * n + i.  The walk reads one field of 32-64 consecutive records per load
// instruction, so an instruction touches 4-8 cache lines instead of 32 (the CU's load path
// spends about a cycle per line beyond 16 per instruction; tools/td_microbench.hip).
// The root records where they are: K2 = (cluster base, cluster count, cut base, cut count) in
// float4 units of the flat array (uint bits) and info bit 1 set; the root is never culled, so
// its cone fields are free: K3.x holds the record count of the leaf-tree triangle array, which the
// device holds field-major too (record i: A at i, B at n + i, C at 2n + i; mirror.cpp).
#pragma once

#include <cstdint>
#include <vector>

// Largest cluster (tree leaf) the cooperative walk handles: it deals kClusterMax lanes per
// surviving cluster (rt_fast.h coop_tree).
constexpr uint32_t kClusterMax = 16;

struct LeafTreeParams {
    uint32_t cluster_max = 16;    // triangles per tree leaf (<= kClusterMax; 8 -> 16: 111 -> 103 ms)
    double split_angle = 0.03;    // split by normals while the cone half-angle exceeds this (rad; 0.6 -> 0.03: 4-bunny 195 -> 140 ms)
    double min_cull_cos = 0.05;   // nodes with a wider cone are never tested (always entered)
    double big_fraction = 0.25;   // triangles spanning this much of the leaf sit apart, untested
    uint32_t cut_clusters = 32;   // clusters per subtree of the flat cut list (<= 32: rt_fast.h coop_tree)
};

// Appends the tree for `count` FlatTri records (12 floats each) to `nodes` (16 floats per
// node) and the reordered records to `ltris`; returns the root's node index.
uint32_t rt_build_leaf_tree(const float* recs, uint32_t count, const LeafTreeParams& prm, std::vector<float>& nodes,
                            std::vector<float>& ltris);

// Screen record of a big leaf (rt_fast.h screen_leaf, mirror.h pf = 3): the leaf's triangles split
// into at most kScreenOutliers "outliers" (the big / degenerate ones the tree root keeps apart) and a
// core whose one node record (box, E1, Nmin, normal cone -- the fields cluster_cull reads) proves for a
// ray that none of the core can pass the fp32 test.  20 floats: K0, K1, K2, (sin, outlier count, 0, 0),
// (outlier positions in the leaf, ascending; ~0 unused).  Returns false (no record) when the core's
// cone is too wide to ever cull (cluster_cull needs cos > min_cull_cos) or there are too many outliers.
constexpr uint32_t kScreenOutliers = 4;
bool rt_build_leaf_screen(const float* recs, uint32_t count, const LeafTreeParams& prm, float out[20]);

// Appends the flat cluster and cut lists of the tree rooted at `root` to `flat` (16 floats per
// record) and records their place in the root (see above).
void rt_build_leaf_flat(std::vector<float>& nodes, uint32_t root, const LeafTreeParams& prm, std::vector<float>& flat);
