// mirror.h -- the render kernel's private, read-only view of a GPUScene's triangles.
//
// The reference arrays (GPUBVHNode / face_indices / GPUFace / GPUVertex, GPUScene.h:25-74)
// stay authoritative; from them the host derives once per geometry upload:
//
//  * tris   leaf-ordered FlatTri records, 48 B: (v0.xyz, e1.x), (e1.yz, e2.xy), (e2.z, face, po, pf)
//           -- record i is faces[face_indices[i]] with the edges glm::intersectRayTriangle forms
//           (v1 - v0, v2 - v0 in fp32, gtx/intersect.inl:37-38), so a leaf's triangles are one
//           contiguous, 16-B aligned run instead of three dependent gathers per triangle;
//  * pairs  for every leaf of more than BIG (= rtfast::BIG) triangles, the same triangles two by
//           two with each component interleaved, 80 B per pair: (v0x_a, v0x_b, v0y_a, v0y_b),
//           (v0z, e1x), (e1y, e1z), (e2x, e2y), (e2z_a, e2z_b, face_a, face_b) -- the operand
//           layout of packed fp32 instructions; an odd leaf ends with an all-zero triangle.  The
//           leaf's first tris record holds po = its first pair, pf = 1 (0 for other leaves), or
//           pf = 3 when a screen record (leaftree.h rt_build_leaf_screen: the cull record of the
//           leaf's core and the positions of its few big "outlier" triangles) sits in the 80-B slot
//           just before the pairs, at po - 1 (rt_fast.h screen_leaf);
//  * quads / units  for the same leaves, their triangles by TWINS.  The reference adds every loaded
//           face twice (Scene.cpp:103-127: the indexed face and AddTriangle's flat copy), and the two
//           records share v0 with e1 and e2 swapped -- the same triangle, wound the other way -- so a
//           twin's glm test computes, in real arithmetic, det' = -det, u' = -v, v' = -u.  A unit is a
//           triangle of the leaf and its twin (if the leaf holds one), in leaf order of the first;
//           a unit record (64 B) is the triangle record with (twin face, pos | twin pos << 16) in its
//           last two words, then (kd, ke, 0, 0) (rt_twin_bounds; kd = -1: no twin).  A quad (112 B)
//           packs two units for packed fp32: the pairs layout (x5), (kd_a, kd_b, ke_a, ke_b),
//           (pos_a | twin_a << 16, pos_b | twin_b << 16, twin face a, twin face b).  A twin is tested
//           only when its partner's own values cannot prove it rejected (rt_fast.h twin_rejected).
//           The leaf's second / third tris record hold (first quad, quad count) / (first unit, unit
//           count) in their last two words (0 quads: positions do not fit 16 bits, pairs only);
//  * spairs for every leaf of at most BIG triangles, its triangles two by two in the pairs layout,
//           the pair of triangles (i, i + 1) stored at record i (i = first, first + 2, ...; an
//           odd leaf ends with an all-zero triangle), so a small leaf needs no index of its own;
//           records at other positions are unused;
//  * tree / ltris  for leaves of at least MIRROR_TREE_LEAF triangles, a leaf tree instead
//           (leaftree.h): the first record holds po = the root node, pf = 2; ltris goes to the
//           device field-major (rt_ltris_device_layout);
//  * flat   the leaf trees' flat cluster and cut lists (leaftree.h, cooperative walk);
//  * treelets  the BVH cut into subtrees of at most 63 nodes for the lone-pixel kernel
//           (rt_lone.hip): from a root, nodes are taken breadth first while they fit; the nodes of
//           a treelet sit in 64 slots of 48 B in right-first preorder (the reference's DFS order,
//           main_raytracing.cu:75-76): (bmin.xyz, bmax.x), (bmax.yz, X, count), (ancestor-slot
//           mask lo, hi, subtree size in slots, frontier) -- X = the leaf's first triangle, or for
//           a frontier (an inner node whose children were not taken) the treelet rooted at it,
//           which holds the same node again in its slot 0; unused slots have count = ~0u;
//  * nodes  the traversal's private copy of the BVH nodes (rt_fast.h reads only this one): the
//           reference's nodes renumbered so that every sibling pair starts on a 64-B boundary (the
//           reference's 32-B root shifts half its pairs across two cache lines) and pairs follow the
//           DFS's right-first pre-order (main_raytracing.cu:75-76), so a descending ray's next pair
//           often shares the 128-B line of the pair it just tested.  Slot 0 = root, slot 1 padding,
//           pair p at slots 2 + 2p, 3 + 2p; an inner node's first_index is its left child's slot, a
//           leaf's is unchanged.  Same boxes and visit order: the same decisions;
//  * depth  the deepest leaf (sizes the traversal stack) and whether every node bound lies in
//           the range where the filtered slab test is proven (rt_fast.h).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "rt_abi.h"

constexpr uint32_t MIRROR_BIG_LEAF = 8;     // leaves above this get pair records (== rtfast::BIG)
constexpr uint32_t MIRROR_TREE_LEAF = 1024;  // ... and leaves this large a leaf tree (leaftree.h) instead
constexpr uint32_t FACE_NO_LEAF = 0xffffffffu, FACE_TWO_LEAVES = 0xfffffffeu;  // MirrorHost::face_leaf

struct MirrorHost {
    std::vector<float> nodes;     // 8 floats per private node (GPUBVHNode layout)
    std::vector<float> tris;      // 12 floats per record
    std::vector<float> pairs;     // 20 floats per pair
    std::vector<float> quads;     // 28 floats per twin quad
    std::vector<float> units;     // 16 floats per twin unit
    std::vector<float> spairs;    // 20 floats per triangle position (small leaves' pairs)
    std::vector<float> tree;      // 16 floats per leaf-tree node
    std::vector<float> ltris;     // 12 floats per leaf-tree triangle record
    std::vector<float> flat;      // 16 floats per record: leaf trees' flat cluster / cut lists
    std::vector<float> treelets;  // 64 slots x 12 floats per treelet (rt_lone.hip)
    std::vector<float> face_leaf; // scenes with big leaves: uint32 per face, the private node index of the leaf
                                  // holding it (FACE_NO_LEAF / FACE_TWO_LEAVES); rt_fast.h deferred leaves' guard
    int depth = 0;                // deepest leaf (root = 0) reachable from node 0
    bool fast = true;             // node bounds inside the filtered-slab range (rt_fast.h)
    int screens = 0;              // big leaves with a screen record (pf = 3)
    bool twins = true;            // false: big-leaf metadata records would collide (overlapping leaves), no twins
};

// Build from host copies of the reference arrays.  node_count / face_count / vertex_count
// bound the indices (out-of-range references throw std::runtime_error).
void rt_build_mirror(const GPUBVHNode* nodes, size_t node_count, const uint32_t* face_indices, size_t index_count,
                     const GPUFace* faces, size_t face_count, const GPUVertex* vertices, size_t vertex_count,
                     MirrorHost* out);

// The twin test's bounds of a triangle record (12 floats, mirror.h tris): kd bounds |det_A + det_twin|
// (the computed values), ke x |o - v0|_1 bounds |u_A + v_twin| and |v_A + u_twin| (rt_fast.h
// twin_rejected).
void rt_twin_bounds(const float* rec, float* kd, float* ke);

// The device copy of MirrorHost::ltris: field-major (record i: A at float4 i, B at n + i, C at
// 2n + i), so a load instruction of a cluster's 16 lanes touches 2 cache lines instead of 6.
std::vector<float> rt_ltris_device_layout(const std::vector<float>& ltris);

// The private node array alone (also called by rt_build_mirror).
void rt_build_private_nodes(const GPUBVHNode* nodes, size_t node_count, std::vector<float>& out);

// The treelets alone (also called by rt_build_mirror).
void rt_build_treelets(const GPUBVHNode* nodes, size_t node_count, std::vector<float>& out);

// Registry: device copies of a mirror, keyed by the GPUScene's BVH node pointer and valid
// while the scene's face_indices / faces / vertices pointers are the ones it was built from.
struct MirrorDevice {
    const void* nodes = nullptr;  // private node array (128-B aligned)
    const void* tris = nullptr;
    const void* pairs = nullptr;
    const void* quads = nullptr;
    const void* units = nullptr;
    const void* spairs = nullptr;
    const void* tree = nullptr;
    const void* ltris = nullptr;
    const void* flat = nullptr;
    const void* treelets = nullptr;
    const void* face_leaf = nullptr;
    int depth = -1;
    bool fast = false;
    int screens = 0;
    bool owned = true;         // built by rt_scene_upload, which forgets it before freeing the arrays
    uint64_t fingerprint = 0;  // foreign scenes: content hash of the arrays it was built from
};
// owned = false: a GPUScene filled by another host (the reference's Scene.cpp); the mirror is
// then revalidated against `fingerprint` at every use (rt_kernel.hip foreign_mirror).
int rt_internal_install_mirror(const GPUScene* scene, const MirrorHost& m, bool owned = true,
                               uint64_t fingerprint = 0);  // 0 or -1 (rt_last_error)
void rt_internal_forget_mirror(const void* gpu_nodes);
bool rt_internal_lookup_mirror(const GPUScene* scene, MirrorDevice* out);

void rt_internal_set_error(const char* msg);  // rt_last_error() text (rt_kernel.hip)
