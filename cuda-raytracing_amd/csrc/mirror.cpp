// mirror.cpp -- host construction and device registry of the kernel's triangle mirror
// (see mirror.h for the layout).
#include "mirror.h"

#include <cstdlib>
#include <functional>

#include "leaftree.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>

namespace {
void put_flat(float* o, const float* p0, const float* p1, const float* p2, uint32_t face) {
    o[0] = p0[0], o[1] = p0[1], o[2] = p0[2];
    o[3] = p1[0] - p0[0], o[4] = p1[1] - p0[1], o[5] = p1[2] - p0[2];  // fp32, as glm forms them
    o[6] = p2[0] - p0[0], o[7] = p2[1] - p0[1], o[8] = p2[2] - p0[2];
    std::memcpy(&o[9], &face, 4);
    o[10] = o[11] = 0.0f;
}
// Two FlatTri records a, b (b null: an all-zero triangle, never accepted) as one pair record.
void put_pair(float* q, const float* a, const float* b) {
    static const float zero[12] = {};
    if (!b) b = zero;
    for (int c = 0; c < 9; c++) q[2 * c] = a[c], q[2 * c + 1] = b[c];
    std::memcpy(&q[18], &a[9], 4);
    std::memcpy(&q[19], &b[9], 4);
}
}  // namespace

// Error bounds of glm::intersectRayTriangle's fp32 evaluation (gtx/intersect.inl:29-94, the operation
// order of rt_fast.h test_triangle) for a triangle A = (v0, e1, e2) and its twin A' = (v0, e2, e1),
// with U = 2^-24 and round-to-nearest, every product / sum rounding once:
//   cross component: |c - c_R| <= (2U + U^2) T, T = the sum of the two products' magnitudes;
//   3-term dot with computed second operand y: |d - x.y_R| <= gamma_3 sum |x_i y_i| + sum |x_i| |dy_i|.
// det = e1.(nd x e2): |det - det_R| <= 5.000001 U S, S = sum over distinct (i, j, k) of |e1_i nd_j e2_k|
// <= |e1|_1 |e2|_1 (|nd_j| <= 1 + 3U); S is symmetric in e1 and e2, and det'_R = -det_R exactly, so
// |det + det'| <= 10.0001 U |e1|_1 |e2|_1 = kd.  With dist = o - v0 (the same computed value for both):
// u = dist.(nd x e2) and v' = nd.(dist x e2) satisfy v'_R = -u_R, each within 5.000003 U |dist|_1 |e2|_1,
// so |u + v'| <= 10.00001 U |dist|_1 |e2|_1; likewise |v + u'| <= 10.00001 U |dist|_1 |e1|_1.  ke =
// 10.0001 U max(|e1|_1, |e2|_1), so ke |dist|_1 bounds both.  Computed in double, then widened by
// 2^-20 before rounding to float (tests/test_scene.py checks the bound on sampled rays).
void rt_twin_bounds(const float* r, float* kd, float* ke) {
    const double U = std::ldexp(1.0, -24);
    const double n1 = std::fabs((double)r[3]) + std::fabs((double)r[4]) + std::fabs((double)r[5]);
    const double n2 = std::fabs((double)r[6]) + std::fabs((double)r[7]) + std::fabs((double)r[8]);
    const double w = 1.0 + std::ldexp(1.0, -20);
    *kd = (float)(10.0001 * U * n1 * n2 * w * w);
    *ke = (float)(10.0001 * U * std::max(n1, n2) * w * w);
}

namespace {
// The twins of big leaf [first, first + count) (mirror.h quads / units): units in leaf order, each a
// triangle and (when the leaf holds one) its twin -- same v0, e1 and e2 swapped, bit for bit; a quad
// packs two units.  Appends the leaf's quads and units; returns false (nothing appended) for a leaf
// whose positions do not fit 16 bits.
bool build_twins(const float* tris, uint32_t first, uint32_t count, std::vector<float>& quads,
                 std::vector<float>& units, uint32_t* nq, uint32_t* nu) {
    if (count >= 0xffffu) return false;
    auto key = [&](uint32_t i, bool swapped) {
        const float* r = &tris[(size_t)(first + i) * 12];
        std::string k(reinterpret_cast<const char*>(r), 12);
        k.append(reinterpret_cast<const char*>(r + (swapped ? 6 : 3)), 12);
        k.append(reinterpret_cast<const char*>(r + (swapped ? 3 : 6)), 12);
        return k;
    };
    std::map<std::string, std::vector<uint32_t>> by;
    for (uint32_t i = 0; i < count; i++) by[key(i, false)].push_back(i);
    std::vector<char> used(count, 0);
    std::vector<std::pair<uint32_t, uint32_t>> un;  // (position, twin position or ~0u)
    for (uint32_t i = 0; i < count; i++) {
        if (used[i]) continue;
        used[i] = 1;
        uint32_t twin = ~0u;
        auto it = by.find(key(i, true));
        if (it != by.end())
            for (uint32_t j : it->second)
                if (!used[j]) {
                    twin = j;
                    used[j] = 1;
                    break;
                }
        un.push_back({i, twin});
    }
    static const float zero[12] = {};
    const uint32_t none = ~0u;
    auto face = [&](uint32_t pos) { return pos == none ? none : *reinterpret_cast<const uint32_t*>(&tris[(size_t)(first + pos) * 12 + 9]); };
    auto packed = [&](uint32_t pos, uint32_t twin) { return (pos & 0xffffu) | ((twin == none ? 0xffffu : twin) << 16); };
    for (const auto& [pos, twin] : un) {  // units: 16 floats
        float q[16] = {};
        std::memcpy(q, &tris[(size_t)(first + pos) * 12], 10 * 4);
        const uint32_t ft = face(twin), w = packed(pos, twin);
        std::memcpy(&q[10], &ft, 4);
        std::memcpy(&q[11], &w, 4);
        rt_twin_bounds(&tris[(size_t)(first + pos) * 12], &q[12], &q[13]);
        if (twin == none) q[12] = -1.0f;
        units.insert(units.end(), q, q + 16);
    }
    for (size_t u = 0; u < un.size(); u += 2) {  // quads: 28 floats
        const bool hb = u + 1 < un.size();
        const float* ra = &tris[(size_t)(first + un[u].first) * 12];
        const float* rb = hb ? &tris[(size_t)(first + un[u + 1].first) * 12] : zero;
        float q[28] = {};
        put_pair(q, ra, rb);
        float kd, ke;
        rt_twin_bounds(ra, &kd, &ke);
        q[20] = un[u].second == none ? -1.0f : kd, q[22] = ke;
        rt_twin_bounds(rb, &kd, &ke);
        q[21] = (!hb || un[u + 1].second == none) ? -1.0f : kd, q[23] = ke;
        const uint32_t wa = packed(un[u].first, un[u].second), wb = hb ? packed(un[u + 1].first, un[u + 1].second) : none;
        const uint32_t fa = face(un[u].second), fb = hb ? face(un[u + 1].second) : none;
        std::memcpy(&q[24], &wa, 4);
        std::memcpy(&q[25], &wb, 4);
        std::memcpy(&q[26], &fa, 4);
        std::memcpy(&q[27], &fb, 4);
        quads.insert(quads.end(), q, q + 28);
    }
    *nq = (uint32_t)((un.size() + 1) / 2);
    *nu = (uint32_t)un.size();
    return true;
}
}  // namespace

void rt_build_mirror(const GPUBVHNode* nodes, size_t node_count, const uint32_t* fi, size_t index_count,
                     const GPUFace* faces, size_t face_count, const GPUVertex* verts, size_t vertex_count,
                     MirrorHost* out) {
    auto bad = [](const char* what) { throw std::runtime_error(std::string("mirror: ") + what); };
    out->tris.assign(index_count * 12, 0.0f);
    for (size_t i = 0; i < index_count; i++) {
        const uint32_t f = fi[i];
        if (f >= face_count) bad("face index out of range");
        const GPUFace& fc = faces[f];
        if (fc.v0 >= vertex_count || fc.v1 >= vertex_count || fc.v2 >= vertex_count) bad("vertex index out of range");
        put_flat(&out->tris[i * 12], verts[fc.v0].position, verts[fc.v1].position, verts[fc.v2].position, f);
    }

    // walk the tree from the root: depth, filtered-slab range, big leaves
    out->pairs.clear();
    out->quads.clear();
    out->units.clear();
    out->tree.clear();
    out->ltris.clear();
    out->flat.clear();
    out->depth = 0;
    out->fast = true;
    out->screens = 0;
    std::vector<uint32_t> big;
    out->spairs.assign(index_count * 20, 0.0f);
    if (node_count == 0) return;
    std::vector<std::pair<uint32_t, int>> st{{0u, 0}};
    size_t visited = 0;
    while (!st.empty()) {
        const auto [n, d] = st.back();
        st.pop_back();
        if (n >= node_count) bad("node index out of range");
        if (++visited > node_count) bad("node graph is not a tree");
        const GPUBVHNode& nd = nodes[n];
        for (int k = 0; k < 3; k++) {
            const float lo = std::fabs(nd.bmin[k]), hi = std::fabs(nd.bmax[k]);
            if ((lo != 0.0f && (lo < 0x1p-60f || lo > 0x1p62f)) || (hi != 0.0f && (hi < 0x1p-60f || hi > 0x1p62f)))
                out->fast = false;
        }
        if (nd.prim_count > 0) {
            if ((size_t)nd.first_index + nd.prim_count > index_count) bad("leaf range out of range");
            out->depth = std::max(out->depth, d);
            if (nd.prim_count > MIRROR_BIG_LEAF)
                big.push_back(n);
            else
                for (uint32_t j = 0; j < nd.prim_count; j += 2)
                    put_pair(&out->spairs[((size_t)nd.first_index + j) * 20], &out->tris[((size_t)nd.first_index + j) * 12],
                             j + 1 < nd.prim_count ? &out->tris[((size_t)nd.first_index + j + 1) * 12] : nullptr);
        } else {
            st.push_back({nd.first_index, d + 1});
            st.push_back({nd.first_index + 1, d + 1});
        }
    }
    std::sort(big.begin(), big.end());
    big.erase(std::unique(big.begin(), big.end()), big.end());
    // A big leaf's metadata lives in words 10-11 of its records: the first (po, pf), the second and third
    // (its quads, its units: the twins).  The kernel reads the second and third of every big leaf with pair
    // records, so they must belong to that leaf alone -- neither another big leaf's first record nor its
    // second / third.  A BVH from the reference's builder never violates this (a leaf range is one node's),
    // but a foreign BVH whose big-leaf ranges overlap with different starts could: such a scene gets no
    // twins at all (pairs only, exact either way) instead of records that overwrite each other.
    bool twins_ok = true;
    {
        std::vector<uint8_t> role(index_count, 0);  // 1: a big leaf's first record, 2: a big leaf's second / third
        for (uint32_t n : big) role[nodes[n].first_index] = 1;
        std::vector<uint32_t> firsts;
        for (uint32_t n : big) firsts.push_back(nodes[n].first_index);
        std::sort(firsts.begin(), firsts.end());
        firsts.erase(std::unique(firsts.begin(), firsts.end()), firsts.end());
        for (uint32_t f : firsts)
            for (size_t r = (size_t)f + 1; r <= (size_t)f + 2 && twins_ok; r++) {
                if (r >= index_count || role[r] != 0) twins_ok = false;
                else role[r] = 2;
            }
    }
    out->twins = twins_ok;
    std::vector<uint32_t> roots;
    for (uint32_t n : big) {
        const GPUBVHNode& nd = nodes[n];
        float* lead = &out->tris[(size_t)nd.first_index * 12];
        uint32_t po;
        std::memcpy(&po, &lead[10], 4);
        uint32_t pf;
        std::memcpy(&pf, &lead[11], 4);
        if (pf) continue;  // two nodes sharing one leaf range
        rt_build_options opt;
        rt_get_build_options(&opt);
        if (nd.prim_count >= opt.leaf_tree_min) {
            LeafTreeParams prm;
            prm.cut_clusters = opt.cut_clusters;
            prm.split_angle = opt.split_angle;
            prm.cluster_max = opt.cluster_max;
            po = rt_build_leaf_tree(&out->tris[(size_t)nd.first_index * 12], nd.prim_count, prm, out->tree, out->ltris);
            rt_build_leaf_flat(out->tree, po, prm, out->flat);
            if (out->ltris.size() / 12 >= (1u << 26)) bad("leaf trees too large (record index >= 2^26)");
            roots.push_back(po);
            pf = 2;
            std::memcpy(&lead[10], &po, 4);
            std::memcpy(&lead[11], &pf, 4);
            continue;
        }
        // a screen record right before the pairs when the leaf has one (pf = 3, rt_fast.h screen_leaf)
        float scr[20];
        rt_build_options so;
        rt_get_build_options(&so);
        LeafTreeParams sp;
        sp.split_angle = so.split_angle;
        pf = 1;
        if (so.leaf_screens && rt_build_leaf_screen(&out->tris[(size_t)nd.first_index * 12], nd.prim_count, sp, scr)) {
            out->pairs.insert(out->pairs.end(), scr, scr + 20);
            pf = 3;
            out->screens++;
        }
        po = (uint32_t)(out->pairs.size() / 20);
        std::memcpy(&lead[10], &po, 4);
        std::memcpy(&lead[11], &pf, 4);
        for (uint32_t j = 0; j < nd.prim_count; j += 2) {
            float q[20];
            put_pair(q, &out->tris[((size_t)nd.first_index + j) * 12],
                     j + 1 < nd.prim_count ? &out->tris[((size_t)nd.first_index + j + 1) * 12] : nullptr);
            out->pairs.insert(out->pairs.end(), q, q + 20);
        }
        // the twins; the leaf's second / third record say where its quads / units are (mirror.h)
        const uint32_t qb = (uint32_t)(out->quads.size() / 28), ub = (uint32_t)(out->units.size() / 16);
        uint32_t nq = 0, nu = 0;
        if (twins_ok && build_twins(out->tris.data(), nd.first_index, nd.prim_count, out->quads, out->units, &nq, &nu)) {
            float* second = &out->tris[((size_t)nd.first_index + 1) * 12];
            float* third = &out->tris[((size_t)nd.first_index + 2) * 12];
            std::memcpy(&second[10], &qb, 4);
            std::memcpy(&second[11], &nq, 4);
            std::memcpy(&third[10], &ub, 4);
            std::memcpy(&third[11], &nu, 4);
        }
    }
    // every root's K3.x: the leaf-tree triangle count, the stride of their field-major device copy
    const uint32_t nl = (uint32_t)(out->ltris.size() / 12);
    for (uint32_t r : roots) std::memcpy(&out->tree[(size_t)r * 16 + 12], &nl, 4);
    rt_build_treelets(nodes, node_count, out->treelets);
    rt_build_private_nodes(nodes, node_count, out->nodes);
    // scenes with big leaves: the leaf (private node) of every face, for the deferred leaves' guard (rt_fast.h)
    out->face_leaf.clear();
    if (!out->pairs.empty() || !out->tree.empty()) {
        std::vector<uint32_t> fl(face_count, FACE_NO_LEAF);
        const size_t nn = out->nodes.size() / 8;
        for (size_t k = 0; k < nn; k++) {
            uint32_t first, count;
            std::memcpy(&first, &out->nodes[k * 8 + 6], 4);
            std::memcpy(&count, &out->nodes[k * 8 + 7], 4);
            if (count == 0 || (size_t)first + count > index_count) continue;
            for (uint32_t i = first; i < first + count; i++) {
                uint32_t f;
                std::memcpy(&f, &out->tris[(size_t)i * 12 + 9], 4);
                if (f >= face_count) continue;
                fl[f] = fl[f] == FACE_NO_LEAF || fl[f] == (uint32_t)k ? (uint32_t)k : FACE_TWO_LEAVES;
            }
        }
        out->face_leaf.resize(face_count);
        std::memcpy(out->face_leaf.data(), fl.data(), face_count * 4);
    }
}

// The traversal's private node array (mirror.h nodes): the reference's BVH nodes renumbered so
// that (1) every sibling pair -- the two children an inner step loads together -- starts on a
// 64-B boundary (the reference puts the 32-B root first, so half of its pairs straddle two cache
// lines), and (2) pairs follow the DFS's own order, right child first (main_raytracing.cu:75-76):
// pair p of node v, then the pair of v's right child, so the next pair a descending ray needs
// sits in the same 128-B line.  Slot 0 is the root, slot 1 padding, pair p at slots 2 + 2p and
// 3 + 2p; an inner node's first_index is its left child's slot, a leaf's is unchanged (the
// triangle range the tris / pair records are indexed by).  Same boxes, same visit order: the
// traversal's decisions are the reference's.
void rt_build_private_nodes(const GPUBVHNode* nodes, size_t node_count, std::vector<float>& out) {
    out.clear();
    if (node_count == 0) return;
    std::vector<uint32_t> slot(node_count, ~0u);  // private slot of every reachable node
    slot[0] = 0;
    uint32_t pairs = 0;
    std::vector<uint32_t> st{0u};
    while (!st.empty()) {  // pre-order, right child first: the order pairs are numbered in
        const uint32_t v = st.back();
        st.pop_back();
        const GPUBVHNode& nd = nodes[v];
        if (nd.prim_count > 0) continue;
        const uint32_t l = nd.first_index, r = nd.first_index + 1;
        slot[l] = 2 + 2 * pairs, slot[r] = 3 + 2 * pairs;
        pairs++;
        st.push_back(l);
        st.push_back(r);  // popped first
    }
    out.assign((size_t)(2 + 2 * pairs) * 8, 0.0f);
    for (size_t v = 0; v < node_count; v++) {
        if (slot[v] == ~0u) continue;
        GPUBVHNode nd = nodes[v];
        if (nd.prim_count == 0) nd.first_index = slot[nd.first_index];
        std::memcpy(&out[(size_t)slot[v] * 8], &nd, sizeof nd);
    }
}

std::vector<float> rt_ltris_device_layout(const std::vector<float>& ltris) {
    const size_t n = ltris.size() / 12;
    std::vector<float> d(ltris.size());
    for (size_t i = 0; i < n; i++)
        for (int f = 0; f < 3; f++) std::memcpy(&d[(f * n + i) * 4], &ltris[i * 12 + 4 * f], 16);
    return d;
}

// ---------------------------------------------------------------------------------------
// Treelets (mirror.h, rt_lone.hip).  From treelet root r, nodes are taken breadth first while two
// more fit into 63 slots; an inner node whose children were not taken is a frontier and roots
// its own treelet.  Within a treelet the nodes are stored in right-first preorder (first + 1
// before first, the reference's pop order), so a slot's subtree is the run of slots after it.
// ---------------------------------------------------------------------------------------
void rt_build_treelets(const GPUBVHNode* nodes, size_t node_count, std::vector<float>& out) {
    out.clear();
    if (node_count == 0 || nodes[0].prim_count > 0) return;  // a leaf root: nothing to walk
    constexpr uint32_t EMPTY = 0xffffffffu;
    const float inf = INFINITY;
    std::vector<uint32_t> roots{0u};
    for (size_t k = 0; k < roots.size(); k++) {
        // breadth-first selection
        std::vector<uint32_t> taken{roots[k]};
        std::map<uint32_t, bool> expanded;
        for (size_t q = 0; q < taken.size(); q++) {
            const GPUBVHNode& nd = nodes[taken[q]];
            if (nd.prim_count > 0) continue;
            if (taken.size() + 2 > 63) break;
            expanded[taken[q]] = true;
            taken.push_back(nd.first_index + 1);
            taken.push_back(nd.first_index);
        }
        // right-first preorder over the taken subtree: slot, parent slot, subtree size
        struct Slot { uint32_t node; int parent; uint32_t size; unsigned long long anc; };
        std::vector<Slot> slots;
        std::function<uint32_t(uint32_t, int, unsigned long long)> place = [&](uint32_t n, int parent,
                                                                                unsigned long long anc) -> uint32_t {
            const uint32_t me = (uint32_t)slots.size();
            slots.push_back({n, parent, 1u, anc});
            if (expanded.count(n)) {
                const unsigned long long a2 = anc | (1ull << me);
                const uint32_t s1 = place(nodes[n].first_index + 1, (int)me, a2);
                const uint32_t s2 = place(nodes[n].first_index, (int)me, a2);
                slots[me].size = 1u + s1 + s2;
            }
            return slots[me].size;
        };
        place(roots[k], -1, 0ull);
        const size_t base = out.size();
        out.resize(base + 64 * 12, 0.0f);
        for (uint32_t p = 0; p < 64; p++) {
            float* o = &out[base + p * 12];
            if (p >= slots.size()) {
                o[0] = o[1] = o[2] = inf, o[3] = o[4] = o[5] = -inf;
                std::memcpy(&o[7], &EMPTY, 4);
                continue;
            }
            const GPUBVHNode& nd = nodes[slots[p].node];
            o[0] = nd.bmin[0], o[1] = nd.bmin[1], o[2] = nd.bmin[2], o[3] = nd.bmax[0], o[4] = nd.bmax[1], o[5] = nd.bmax[2];
            uint32_t X = nd.first_index, cnt = nd.prim_count, frontier = 0u;
            if (cnt == 0 && !expanded.count(slots[p].node)) {
                X = (uint32_t)roots.size();
                roots.push_back(slots[p].node);
                frontier = 1u;
            }
            std::memcpy(&o[6], &X, 4);
            std::memcpy(&o[7], &cnt, 4);
            const uint32_t lo = (uint32_t)slots[p].anc, hi = (uint32_t)(slots[p].anc >> 32);
            std::memcpy(&o[8], &lo, 4);
            std::memcpy(&o[9], &hi, 4);
            std::memcpy(&o[10], &slots[p].size, 4);
            std::memcpy(&o[11], &frontier, 4);
        }
    }
}

// ---------------------------------------------------------------------------------------
// registry
// ---------------------------------------------------------------------------------------
namespace {
struct Entry {
    const void* face_indices;
    const void* vertices;
    const void* faces;
    void* block;  // device copy of the tris and pair records
    MirrorDevice dev;
};
std::mutex g_mutex;
std::map<const void*, Entry> g_mirrors;  // keyed by the device BVH node array

void release(Entry& e) {
    if (e.block) rt_free(e.block);
    e.block = nullptr;
}
}  // namespace

int rt_internal_install_mirror(const GPUScene* s, const MirrorHost& m, bool owned, uint64_t fingerprint) {
    const std::vector<float> lt = rt_ltris_device_layout(m.ltris);
    // the parts in one block, each starting on a 256-B boundary (pairs of nodes and records on
    // cache-line boundaries: mirror.h)
    const std::vector<float>* parts[11] = {&m.nodes, &m.tris, &m.pairs, &m.tree, &lt, &m.spairs, &m.flat, &m.treelets, &m.quads,
                                           &m.units, &m.face_leaf};
    size_t off[11], total = 0;
    for (int i = 0; i < 11; i++) {
        off[i] = total;
        total += (parts[i]->size() * 4 + 255) & ~(size_t)255;
    }
    void* block = nullptr;
    if (rt_malloc(&block, total + 256) != 0) return -1;
    char* b = static_cast<char*>(block);
    for (int i = 0; i < 11; i++)
        if (!parts[i]->empty() && rt_memcpy_h2d(b + off[i], parts[i]->data(), parts[i]->size() * 4) != 0) {
            rt_free(block);
            return -1;
        }
    auto at = [&](int i) -> const void* { return parts[i]->empty() ? nullptr : b + off[i]; };
    Entry e{s->gpu_bvh_face_indices, s->gpu_vertices, s->gpu_faces, block, {}};
    e.dev.nodes = at(0);
    e.dev.tris = b + off[1];
    e.dev.pairs = at(2);
    e.dev.tree = at(3);
    e.dev.ltris = at(4);
    e.dev.spairs = at(5);
    e.dev.flat = at(6);
    e.dev.treelets = at(7);
    e.dev.quads = at(8);
    e.dev.units = at(9);
    e.dev.face_leaf = at(10);
    e.dev.depth = m.depth;
    e.dev.fast = m.fast;
    e.dev.screens = m.screens;
    e.dev.owned = owned;
    e.dev.fingerprint = fingerprint;
    std::lock_guard<std::mutex> lock(g_mutex);
    auto it = g_mirrors.find(s->gpu_bvh_nodes);
    if (it != g_mirrors.end()) {
        release(it->second);
        g_mirrors.erase(it);
    }
    g_mirrors.emplace(s->gpu_bvh_nodes, e);
    return 0;
}

void rt_internal_forget_mirror(const void* gpu_nodes) {
    std::lock_guard<std::mutex> lock(g_mutex);
    auto it = g_mirrors.find(gpu_nodes);
    if (it == g_mirrors.end()) return;
    release(it->second);
    g_mirrors.erase(it);
}

// The mirror is used only while ALL the reference arrays it was built from are still the
// ones the GPUScene points at (and, for a foreign scene, the caller checks the fingerprint);
// otherwise only the depth (stack sizing) is reported.
bool rt_internal_lookup_mirror(const GPUScene* s, MirrorDevice* out) {
    std::lock_guard<std::mutex> lock(g_mutex);
    *out = MirrorDevice{};
    auto it = g_mirrors.find(s->gpu_bvh_nodes);
    if (it == g_mirrors.end()) return false;
    const Entry& e = it->second;
    if (e.face_indices != s->gpu_bvh_face_indices || e.vertices != s->gpu_vertices || e.faces != s->gpu_faces) {
        out->depth = e.dev.depth;
        return false;
    }
    *out = e.dev;
    return true;
}

// ---------------------------------------------------------------------------------------
// Build options (rt_abi.h rt_build_options): process-wide, exact-preserving speed knobs.
// ---------------------------------------------------------------------------------------
namespace {
std::mutex g_opt_mutex;
rt_build_options default_options() {
    rt_build_options o;
    const LeafTreeParams p;
    o.leaf_tree_min = MIRROR_TREE_LEAF;
    o.cut_clusters = p.cut_clusters;
    o.cluster_max = p.cluster_max;
    o.split_angle = (float)p.split_angle;
    o.bvh_small = 16;
    o.host_bvh = 0;
    o.leaf_screens = 0;  // measured slower (config 4), an opt-in A/B
    return o;
}
rt_build_options g_options = default_options();
}  // namespace

extern "C" int rt_mirror_build_check(const GPUBVHNode* nodes, size_t node_count, const uint32_t* face_indices,
                                     size_t index_count, const GPUFace* faces, size_t face_count,
                                     const GPUVertex* vertices, size_t vertex_count, uint32_t* meta, int* twins) {
    try {
        MirrorHost m;
        rt_build_mirror(nodes, node_count, face_indices, index_count, faces, face_count, vertices, vertex_count, &m);
        for (size_t i = 0; i < index_count; i++) std::memcpy(&meta[2 * i], &m.tris[i * 12 + 10], 8);
        *twins = m.twins && !m.quads.empty() ? 1 : 0;
        return 0;
    } catch (const std::exception& e) {
        rt_internal_set_error(e.what());
        return -1;
    }
}

extern "C" void rt_get_build_options(rt_build_options* out) {
    if (!out) return;
    std::lock_guard<std::mutex> lock(g_opt_mutex);
    *out = g_options;
}

extern "C" int rt_set_build_options(const rt_build_options* o) {
    const rt_build_options v = o ? *o : default_options();
    if (v.leaf_tree_min < 2 || v.cut_clusters < 1 || v.cut_clusters > 32 || v.cluster_max < 1 || v.cluster_max > kClusterMax ||
        !(v.split_angle >= 0.0f && v.split_angle < 3.2f) || v.bvh_small < 2 || v.bvh_small > 64 || (v.host_bvh != 0 && v.host_bvh != 1) ||
        (v.leaf_screens != 0 && v.leaf_screens != 1)) {
        rt_internal_set_error("rt_set_build_options: value out of range");
        return 1;
    }
    std::lock_guard<std::mutex> lock(g_opt_mutex);
    g_options = v;
    return 0;
}
