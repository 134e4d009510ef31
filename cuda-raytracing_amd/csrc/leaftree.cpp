// leaftree.cpp -- acceleration inside huge BVH leaves (see leaftree.h).
#include "leaftree.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <numeric>

namespace {

struct Tri {
    const float* rec;  // FlatTri record (12 floats)
    uint32_t j;        // position inside the leaf
    double p[3][3];    // exact corners v0, v0 + e1, v0 + e2 of the fp32 triangle
    double n[3], nlen; // e2 x e1 (the normal det is taken against) and its length
    double el1;        // max(|e1|_1, |e2|_1)
    double c[3];       // centroid (splitting only)
};

float round_down(double v) {
    float f = (float)v;
    if ((double)f > v) f = std::nextafterf(f, -INFINITY);
    return f;
}
float round_up(double v) {
    float f = (float)v;
    if ((double)f < v) f = std::nextafterf(f, INFINITY);
    return f;
}

// Normal cone of the triangles' normal LINES (the test is two-sided): the fp32 axis as stored
// and the cosine of the half-angle measured against that stored axis.
void normal_cone(const std::vector<Tri>& t, const std::vector<uint32_t>& ids, float axis[3], double* cos_out) {
    double a[3] = {0, 0, 0};
    const Tri& r = t[ids[0]];
    for (int pass = 0; pass < 2; pass++) {
        const double ref[3] = {pass ? a[0] : r.n[0], pass ? a[1] : r.n[1], pass ? a[2] : r.n[2]};
        double s[3] = {0, 0, 0};
        for (uint32_t i : ids) {
            const Tri& q = t[i];
            const double d = q.n[0] * ref[0] + q.n[1] * ref[1] + q.n[2] * ref[2];
            const double sg = d < 0 ? -1.0 : 1.0;
            for (int k = 0; k < 3; k++) s[k] += sg * q.n[k] / q.nlen;
        }
        const double l = std::sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
        for (int k = 0; k < 3; k++) a[k] = l > 0 ? s[k] / l : r.n[k] / r.nlen;
    }
    for (int k = 0; k < 3; k++) axis[k] = (float)a[k];
    const double al = std::sqrt((double)axis[0] * axis[0] + (double)axis[1] * axis[1] + (double)axis[2] * axis[2]);
    double cmin = 1.0;
    for (uint32_t i : ids) {
        const Tri& q = t[i];
        cmin = std::min(cmin, std::fabs(q.n[0] * axis[0] + q.n[1] * axis[1] + q.n[2] * axis[2]) / (q.nlen * al));
    }
    *cos_out = std::max(0.0, cmin - 1e-9);
}

struct Builder {
    const std::vector<Tri>& t;
    const LeafTreeParams& prm;
    std::vector<float>& nodes;
    std::vector<float>& ltris;

    uint32_t alloc() {
        nodes.resize(nodes.size() + 16, 0.0f);
        return (uint32_t)(nodes.size() / 16 - 1);
    }

    // record of node k over `ids`; tri_begin = ~0u for an inner node
    void fill(uint32_t k, const std::vector<uint32_t>& ids, bool cone_ok, uint32_t tri_begin) {
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300}, e1 = 0, nmin = 1e300;
        for (uint32_t i : ids) {
            const Tri& q = t[i];
            for (int v = 0; v < 3; v++)
                for (int d = 0; d < 3; d++) lo[d] = std::min(lo[d], q.p[v][d]), hi[d] = std::max(hi[d], q.p[v][d]);
            e1 = std::max(e1, q.el1);
            nmin = std::min(nmin, q.nlen);
        }
        float axis[3] = {0, 0, 1};
        double cs = 0.0;
        if (cone_ok && nmin > 0.0) normal_cone(t, ids, axis, &cs);
        const bool cullable = cone_ok && nmin > 0.0 && cs > prm.min_cull_cos;
        float* K = &nodes[(size_t)k * 16];
        for (int d = 0; d < 3; d++) {
            // pad by 2^-40 relative before rounding outward: covers the double rounding of the corners
            K[d] = round_down(lo[d] - std::fabs(lo[d]) * 0x1p-40);
            K[4 + d] = round_up(hi[d] + std::fabs(hi[d]) * 0x1p-40);
            K[8 + d] = axis[d];
        }
        K[3] = round_up(e1 * (1.0 + 0x1p-40));
        K[7] = round_down(nmin * (1.0 - 0x1p-30));
        K[11] = round_down(cs);
        K[12] = round_up(std::sqrt(std::max(0.0, 1.0 - (double)K[11] * K[11])) + 1e-9);
        const uint32_t skip = (uint32_t)(nodes.size() / 16);
        const uint32_t info = (cullable ? 1u : 0u) | ((uint32_t)(tri_begin == ~0u ? 0 : ids.size()) << 8);
        std::memcpy(&K[13], &skip, 4);
        std::memcpy(&K[14], &tri_begin, 4);
        std::memcpy(&K[15], &info, 4);
    }

    void emit_tris(const std::vector<uint32_t>& ids) {
        for (uint32_t i : ids) {
            const size_t o = ltris.size();
            ltris.insert(ltris.end(), t[i].rec, t[i].rec + 12);
            std::memcpy(&ltris[o + 10], &t[i].j, 4);
            ltris[o + 11] = 0.0f;
        }
    }

    void build(std::vector<uint32_t> ids) {
        const uint32_t k = alloc();
        if (ids.size() <= prm.cluster_max) {
            const uint32_t begin = (uint32_t)(ltris.size() / 12);
            emit_tris(ids);
            fill(k, ids, true, begin);
            return;
        }
        float axis[3];
        double cs;
        normal_cone(t, ids, axis, &cs);
        std::vector<uint32_t> a, b;
        if (cs < std::cos(prm.split_angle)) split_normals(ids, axis, a, b);
        if (a.empty() || b.empty()) split_space(ids, a, b);
        build(a);
        build(b);
        fill(k, ids, true, ~0u);
    }

    // median split on the coordinate of largest spread of the sign-canonical unit normals
    void split_normals(const std::vector<uint32_t>& ids, const float axis[3], std::vector<uint32_t>& a,
                       std::vector<uint32_t>& b) {
        std::vector<std::array<double, 3>> cn(ids.size());
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        for (size_t i = 0; i < ids.size(); i++) {
            const Tri& q = t[ids[i]];
            const double d = q.n[0] * axis[0] + q.n[1] * axis[1] + q.n[2] * axis[2];
            const double sg = d < 0 ? -1.0 : 1.0;
            for (int c = 0; c < 3; c++) {
                cn[i][c] = sg * q.n[c] / q.nlen;
                lo[c] = std::min(lo[c], cn[i][c]);
                hi[c] = std::max(hi[c], cn[i][c]);
            }
        }
        int c = 0;
        for (int m = 1; m < 3; m++)
            if (hi[m] - lo[m] > hi[c] - lo[c]) c = m;
        if (!(hi[c] - lo[c] > 1e-6)) return;
        std::vector<size_t> ord(ids.size());
        std::iota(ord.begin(), ord.end(), 0);
        std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return cn[x][c] < cn[y][c]; });
        const size_t h = ord.size() / 2;
        for (size_t i = 0; i < ord.size(); i++) (i < h ? a : b).push_back(ids[ord[i]]);
    }

    // median split along the longest axis of the centroid bounds
    void split_space(const std::vector<uint32_t>& ids, std::vector<uint32_t>& a, std::vector<uint32_t>& b) {
        a.clear(), b.clear();
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        for (uint32_t i : ids)
            for (int d = 0; d < 3; d++) lo[d] = std::min(lo[d], t[i].c[d]), hi[d] = std::max(hi[d], t[i].c[d]);
        int d = 0;
        for (int m = 1; m < 3; m++)
            if (hi[m] - lo[m] > hi[d] - lo[d]) d = m;
        std::vector<uint32_t> s = ids;
        std::stable_sort(s.begin(), s.end(), [&](uint32_t x, uint32_t y) { return t[x].c[d] < t[y].c[d]; });
        const size_t h = s.size() / 2;
        a.assign(s.begin(), s.begin() + h);
        b.assign(s.begin() + h, s.end());
    }
};

}  // namespace

namespace {
// corners, normal and edge lengths of the fp32 triangles (double)
std::vector<Tri> leaf_tris(const float* recs, uint32_t count, double* ext_out) {
    std::vector<Tri> t(count);
    double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
    for (uint32_t j = 0; j < count; j++) {
        Tri& q = t[j];
        q.rec = recs + (size_t)j * 12;
        q.j = j;
        const float* r = q.rec;
        for (int d = 0; d < 3; d++) {
            q.p[0][d] = r[d];
            q.p[1][d] = (double)r[d] + (double)r[3 + d];
            q.p[2][d] = (double)r[d] + (double)r[6 + d];
            q.c[d] = (q.p[0][d] + q.p[1][d] + q.p[2][d]) / 3.0;
            for (int v = 0; v < 3; v++) lo[d] = std::min(lo[d], q.p[v][d]), hi[d] = std::max(hi[d], q.p[v][d]);
        }
        const double a[3] = {r[6], r[7], r[8]}, b[3] = {r[3], r[4], r[5]};  // e2, e1
        q.n[0] = a[1] * b[2] - a[2] * b[1];
        q.n[1] = a[2] * b[0] - a[0] * b[2];
        q.n[2] = a[0] * b[1] - a[1] * b[0];
        q.nlen = std::sqrt(q.n[0] * q.n[0] + q.n[1] * q.n[1] + q.n[2] * q.n[2]);
        q.el1 = std::max(std::fabs(b[0]) + std::fabs(b[1]) + std::fabs(b[2]), std::fabs(a[0]) + std::fabs(a[1]) + std::fabs(a[2]));
    }
    *ext_out = std::max({hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]});
    return t;
}
}  // namespace

bool rt_build_leaf_screen(const float* recs, uint32_t count, const LeafTreeParams& prm, float out[20]) {
    double ext = 0;
    const std::vector<Tri> t = leaf_tris(recs, count, &ext);
    std::vector<uint32_t> big, rest;
    for (uint32_t j = 0; j < count; j++) (t[j].nlen == 0.0 || t[j].el1 > prm.big_fraction * ext ? big : rest).push_back(j);
    if (big.size() > kScreenOutliers || rest.empty()) return false;
    std::vector<float> nodes, ltris;
    Builder B{t, prm, nodes, ltris};
    const uint32_t k = B.alloc();
    B.fill(k, rest, true, ~0u);
    uint32_t info;
    std::memcpy(&info, &nodes[15], 4);
    if (!(info & 1u)) return false;  // the core's cone is too wide: cluster_cull could never prove it
    std::memcpy(out, nodes.data(), 12 * 4);
    out[12] = nodes[12];  // sin of the cone
    const uint32_t nb = (uint32_t)big.size(), none = ~0u, zero = 0;
    std::memcpy(&out[13], &nb, 4);
    std::memcpy(&out[14], &zero, 4);
    std::memcpy(&out[15], &zero, 4);
    for (uint32_t i = 0; i < kScreenOutliers; i++) std::memcpy(&out[16 + i], i < nb ? &big[i] : &none, 4);
    return true;
}

uint32_t rt_build_leaf_tree(const float* recs, uint32_t count, const LeafTreeParams& prm, std::vector<float>& nodes,
                            std::vector<float>& ltris) {
    double ext = 0;
    const std::vector<Tri> t = leaf_tris(recs, count, &ext);
    Builder B{t, prm, nodes, ltris};
    // root: a non-culled node whose children are the big / degenerate triangles one by one (never
    // culled: their bound would be useless) and a tree over the rest
    std::vector<uint32_t> big, rest, all(count);
    std::iota(all.begin(), all.end(), 0u);
    for (uint32_t j = 0; j < count; j++) (t[j].nlen == 0.0 || t[j].el1 > prm.big_fraction * ext ? big : rest).push_back(j);
    const uint32_t root = B.alloc();
    for (uint32_t j : big) {
        const uint32_t k = B.alloc();
        const uint32_t begin = (uint32_t)(ltris.size() / 12);
        B.emit_tris({j});
        B.fill(k, {j}, false, begin);
    }
    if (!rest.empty()) B.build(rest);
    B.fill(root, all, false, ~0u);
    return root;
}

void rt_build_leaf_flat(std::vector<float>& nodes, uint32_t root, const LeafTreeParams& prm, std::vector<float>& flat) {
    auto u32 = [&](uint32_t k, int f) {
        uint32_t v;
        std::memcpy(&v, &nodes[(size_t)k * 16 + f], 4);
        return v;
    };
    auto put = [](float* rec, int f, uint32_t v) { std::memcpy(&rec[f], &v, 4); };
    const uint32_t end = u32(root, 13);
    // clusters in pre-order; first_cluster[k - root] = clusters before node k
    std::vector<uint32_t> first_cluster(end - root + 1, 0);
    // records are appended field-major (leaftree.h): field f of record i of a list of n at
    // float4 index base + f * n + i
    auto append_soa = [&](const std::vector<float>& recs) {
        const size_t n = recs.size() / 16;
        for (int f = 0; f < 4; f++)
            for (size_t i = 0; i < n; i++) flat.insert(flat.end(), &recs[i * 16 + 4 * f], &recs[i * 16 + 4 * f] + 4);
    };
    const uint32_t cbase = (uint32_t)(flat.size() / 4);
    uint32_t nc = 0;
    std::vector<float> crec;
    for (uint32_t k = root; k < end; k++) {
        first_cluster[k - root] = nc;
        if (u32(k, 14) != ~0u) {
            const size_t o = crec.size();
            crec.insert(crec.end(), &nodes[(size_t)k * 16], &nodes[(size_t)k * 16] + 16);
            put(&crec[o], 13, nc + 1);
            nc++;
        }
    }
    append_soa(crec);
    first_cluster[end - root] = nc;
    const uint32_t kbase = (uint32_t)(flat.size() / 4);
    uint32_t nk = 0;
    std::vector<uint32_t> todo{root};
    std::vector<uint32_t> cuts;
    while (!todo.empty()) {  // pre-order cut: subtrees of at most cut_clusters clusters
        const uint32_t k = todo.back();
        todo.pop_back();
        const uint32_t skip = u32(k, 13);
        const uint32_t c0 = first_cluster[k - root], c1 = first_cluster[skip - root];
        if (c1 == c0) continue;
        if (c1 - c0 <= prm.cut_clusters || u32(k, 14) != ~0u) {
            cuts.push_back(k);
            continue;
        }
        std::vector<uint32_t> ch;
        for (uint32_t c = k + 1; c < skip; c = u32(c, 13)) ch.push_back(c);
        for (auto it = ch.rbegin(); it != ch.rend(); ++it) todo.push_back(*it);
    }
    std::vector<float> krec;
    for (uint32_t k : cuts) {
        const size_t o = krec.size();
        krec.insert(krec.end(), &nodes[(size_t)k * 16], &nodes[(size_t)k * 16] + 16);
        put(&krec[o], 13, first_cluster[k - root]);
        put(&krec[o], 14, first_cluster[u32(k, 13) - root]);
        nk++;
    }
    append_soa(krec);
    float* R = &nodes[(size_t)root * 16];
    put(R, 8, cbase);
    put(R, 9, nc);
    put(R, 10, kbase);
    put(R, 11, nk);
    put(R, 15, u32(root, 15) | 2u);
}
