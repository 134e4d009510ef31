// leaftree_eval.hip -- analysis tool: a leaf tree's build parameters priced on real rays, on the host.
//
// Reads the records of one huge BVH leaf (the mirror's 12-float FlatTri records in leaf order) and the
// rays that walk it (tools/defer_probe.c rays.bin: origin, normalised direction, bound at the leaf,
// bound at the end of the traversal, whether it changed after the leaf), builds the leaf tree and its
// flat lists with leaftree.cpp for each parameter set, and replays the cooperative walk of rt_fast.h
// coop_tree ray by ray with the kernel's own cluster_cull: cut screening rounds (64 cut records per
// round), cluster rounds (two surviving subtrees per round), triangle rounds (64 / kClusterMax clusters
// per round), and the result, which must be the sequential loop's (checked against it for every ray).
// The walk starts from the deferred bound (rt_fast.h defer_leaf): just above the end bound when it
// changed after the leaf, else the bound itself.
//
//   hipcc -O2 -std=c++17 -ffp-contract=off -I include -I cuda-raytracing_amd/csrc \
//     tools/leaftree_eval.hip cuda-raytracing_amd/csrc/leaftree.cpp -o /tmp/leaftree_eval
//   /tmp/leaftree_eval leaf.bin rays.bin [cluster_max split_angle min_cull_cos cut_clusters] ...
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rt_abi.h"
#include "rt_device.h"
#include "rt_math.h"
#include "xorwow.h"
#include "rt_common.h"
#include "leaftree.h"
#include "rt_fast.h"

static std::vector<float> load(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) { perror(path); exit(1); }
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<float> v(n / 4);
    if (fread(v.data(), 4, v.size(), f) != v.size()) exit(1);
    fclose(f);
    return v;
}
static uint32_t U(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float F(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

struct Cand { float t; uint32_t j; bool found; };

// Why cluster_cull (rt_fast.h) keeps a node, restated step for step with the same arithmetic:
// 0 culled, 1 the cone precondition (dlb > 36 U E1^2) fails, 2 the segment reaches the grown box but
// not the node's own box, 3 the segment reaches the node's own box (below the bound), 4 not cullable.
static int keep_reason(const rtfast::Ray& R, float best, float4 K0, float4 K1, float4 K2, float4 K3) {
    if (!(U(K3.w) & 1u)) return 4;
    if (!rtfast::cluster_cull(R, R.r, best, K0, K1, K2, K3)) {
        const float U_ = 0x1p-24f;
        const float E1 = K0.w, Nmin = K1.w;
        const float dota = fabsf(R.nd.x * K2.x + R.nd.y * K2.y + R.nd.z * K2.z);
        const float ca = fminf(fmaxf(dota * (1.0f - 0x1p-20f) - 4.0f * U_, 0.0f), 1.0f);
        const float sa = sqrtf(fmaxf(1.0f - ca * ca, 0.0f) + 2.0f * U_) * (1.0f + 0x1p-20f);
        const float dlb = Nmin * ((ca * K2.w - sa * K3.x) - 4.0f * U_) * (1.0f - 0x1p-20f);
        if (!(dlb > 36.0f * U_ * E1 * E1)) {
            const float cone = (ca * K2.w - sa * K3.x) - 4.0f * U_;
            return cone <= 0.0f ? 1 : (Nmin / (E1 * E1) < 1e-3f ? 5 : 6);
        }
        const float tx1 = (K0.x - R.o.x) * R.r.x, tx2 = (K1.x - R.o.x) * R.r.x;
        const float ty1 = (K0.y - R.o.y) * R.r.y, ty2 = (K1.y - R.o.y) * R.r.y;
        const float tz1 = (K0.z - R.o.z) * R.r.z, tz2 = (K1.z - R.o.z) * R.r.z;
        const float lo = fmaxf(0.0f, fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2)));
        const float hi = fminf(best, fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2)));
        return lo <= hi ? 3 : 2;
    }
    return 0;
}

// glm's fp32 test of a leaf-tree record and the (t, position) rule of leaf_candidate (rt_fast.h)
static void candidate(const rtfast::Ray& R, const float* r, Cand& L) {
    const float4 A = make_float4(r[0], r[1], r[2], r[3]), B = make_float4(r[4], r[5], r[6], r[7]),
                 C = make_float4(r[8], r[9], r[10], r[11]);
    const rtm::f3 e1 = rtm::mk(A.w, B.x, B.y), e2 = rtm::mk(B.z, B.w, C.x);
    const rtm::f3 p = rtm::cross(R.nd, e2);
    const float det = rtm::dot(e1, p);
    const rtm::f3 dist = rtm::sub(R.o, rtm::mk(A.x, A.y, A.z));
    const float u = rtm::dot(dist, p);
    const rtm::f3 perp = rtm::cross(dist, e1);
    const float v = rtm::dot(R.nd, perp);
    const float uv = u + v;
    const uint32_t sg = U(det) & 0x80000000u;
    const float ad = fabsf(det), su = F(U(u) ^ sg), sv = F(U(v) ^ sg), suv = F(U(uv) ^ sg);
    if (!(ad > 1.1920928955078125e-07f && !(su < 0.0f || su > ad) && !(sv < 0.0f || suv > ad))) return;
    const float t = rtm::dot(e2, perp) * (1.0f / det);
    const uint32_t j = U(C.z);
    if (t >= 0.0f && (t < L.t || (t == L.t && L.found && j < L.j))) L.t = t, L.j = j, L.found = true;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s leaf.bin rays.bin [cluster_max split_angle min_cull_cos cut_clusters]...\n", argv[0]);
        return 2;
    }
    const std::vector<float> recs = load(argv[1]), rays = load(argv[2]);
    const uint32_t n = (uint32_t)(recs.size() / 12), nr = (uint32_t)(rays.size() / 9);
    std::vector<std::vector<double>> sets;
    for (int a = 3; a + 3 < argc + 0 || a + 3 == argc - 0; a += 4) {
        if (a + 3 >= argc) break;
        sets.push_back({atof(argv[a]), atof(argv[a + 1]), atof(argv[a + 2]), atof(argv[a + 3])});
    }
    if (sets.empty()) sets.push_back({16, 0.03, 0.05, 32});
    for (const auto& ps : sets) {
        LeafTreeParams prm;
        prm.cluster_max = (uint32_t)ps[0], prm.split_angle = ps[1], prm.min_cull_cos = ps[2], prm.cut_clusters = (uint32_t)ps[3];
        std::vector<float> nodes, ltris, flat;
        const uint32_t root = rt_build_leaf_tree(recs.data(), n, prm, nodes, ltris);
        rt_build_leaf_flat(nodes, root, prm, flat);
        const float* K = &nodes[(size_t)root * 16];
        const uint32_t cb = U(K[8]), nc = U(K[9]), kb = U(K[10]), nk = U(K[11]);
        auto fld = [&](uint32_t base, uint32_t cnt, uint32_t i, int f) {
            const float* q = &flat[4 * ((size_t)base + (size_t)f * cnt + i)];
            return make_float4(q[0], q[1], q[2], q[3]);
        };
        uint64_t reason[7] = {0, 0, 0, 0, 0, 0, 0};
        uint64_t all_cl = 0, all_rounds = 0, prounds = 0, screen = 0, crounds = 0, trounds = 0, ctests = 0, surv_sub = 0, surv_cl = 0, mism = 0, tris_tested = 0;
        for (uint32_t ri = 0; ri < nr; ri++) {
            const float* q = &rays[(size_t)ri * 9];
            rtfast::Ray R;
            R.o = rtm::mk(q[0], q[1], q[2]);
            R.nd = rtm::mk(q[3], q[4], q[5]);
            R.d = R.nd;
            R.r = rtm::mk(1.0f / q[3], 1.0f / q[4], 1.0f / q[5]);
            R.fast = true;
            const float bend = q[7];
            const bool changed = U(q[8]) != 0;
            const float b0 = changed ? F((U(bend) & 0x7fffffffu) + 1u) : bend;
            Cand L{b0, 0, false};
            float cbest = b0;
            for (uint32_t kbase = 0; kbase < nk; kbase += 64) {
                screen++;
                std::vector<uint32_t> subs;
                for (uint32_t k = kbase; k < nk && k < kbase + 64; k++) {
                    const float4 K3 = fld(kb, nk, k, 3);
                    const bool need = !((U(K3.w) & 1u) && rtfast::cluster_cull(R, R.r, cbest, fld(kb, nk, k, 0), fld(kb, nk, k, 1),
                                                                            fld(kb, nk, k, 2), K3));
                    if (need) subs.push_back(k);
                }
                surv_sub += subs.size();
                for (size_t s = 0; s < subs.size(); s += 2) {
                    crounds++;
                    std::vector<uint32_t> cls;
                    for (size_t w = s; w < s + 2 && w < subs.size(); w++) {
                        const float4 K3 = fld(kb, nk, subs[w], 3);
                        for (uint32_t ci = U(K3.y); ci < U(K3.z); ci++) {
                            const float4 Q3 = fld(cb, nc, ci, 3);
                            ctests++;
                            reason[keep_reason(R, cbest, fld(cb, nc, ci, 0), fld(cb, nc, ci, 1), fld(cb, nc, ci, 2), Q3)]++;
                            if (!((U(Q3.w) & 1u) &&
                                  rtfast::cluster_cull(R, R.r, cbest, fld(cb, nc, ci, 0), fld(cb, nc, ci, 1), fld(cb, nc, ci, 2), Q3)))
                                cls.push_back(ci);
                        }
                    }
                    surv_cl += cls.size();
                    trounds += (cls.size() + (64 / kClusterMax) - 1) / (64 / kClusterMax);
                    uint32_t ntri = 0;
                    for (uint32_t ci : cls) ntri += U(fld(cb, nc, ci, 3).w) >> 8;
                    prounds += (ntri + 63) / 64;  // the same triangles packed 64 to a round
                    for (uint32_t ci : cls) {
                        const float4 Q3 = fld(cb, nc, ci, 3);
                        const uint32_t tb = U(Q3.z), cnt = U(Q3.w) >> 8;
                        for (uint32_t i = tb; i < tb + cnt; i++) candidate(R, &ltris[(size_t)i * 12], L), tris_tested++;
                    }
                    if (L.found) cbest = fminf(cbest, F(U(L.t) + 1u));
                }
            }
            {  // variant: every surviving cluster of the ray first (bound not tightened), then its triangles packed
                uint32_t ntri = 0, ncl = 0;
                for (uint32_t k = 0; k < nk; k++) {
                    const float4 K3 = fld(kb, nk, k, 3);
                    if ((U(K3.w) & 1u) && rtfast::cluster_cull(R, R.r, b0, fld(kb, nk, k, 0), fld(kb, nk, k, 1), fld(kb, nk, k, 2), K3))
                        continue;
                    for (uint32_t ci = U(K3.y); ci < U(K3.z); ci++) {
                        const float4 Q3 = fld(cb, nc, ci, 3);
                        if ((U(Q3.w) & 1u) &&
                            rtfast::cluster_cull(R, R.r, b0, fld(cb, nc, ci, 0), fld(cb, nc, ci, 1), fld(cb, nc, ci, 2), Q3))
                            continue;
                        ncl++, ntri += U(Q3.w) >> 8;
                    }
                }
                all_cl += ncl, all_rounds += (ntri + 63) / 64;
            }
            // the sequential loop over the leaf from the same bound (rt_fast.h leaf order = record j)
            if (ri % 16 == 0) {
                Cand S{b0, 0, false};
                for (uint32_t i = 0; i < (uint32_t)(ltris.size() / 12); i++) candidate(R, &ltris[(size_t)i * 12], S);
                if (S.found != L.found || (S.found && (U(S.t) != U(L.t) || S.j != L.j))) mism++;
            }
        }
        printf("{\"cluster_max\": %u, \"split_angle\": %g, \"min_cull_cos\": %g, \"cut_clusters\": %u, \"clusters\": %u, "
               "\"cuts\": %u, \"rays\": %u, \"screen_rounds\": %.3f, \"cluster_rounds\": %.3f, \"tri_rounds\": %.3f, "
               "\"cluster_tests\": %.2f, \"surviving_subtrees\": %.2f, \"surviving_clusters\": %.2f, \"tris_tested\": %.1f, "
               "\"checked_mismatches\": %llu, \"kept_cone\": %.2f, \"kept_grown_box\": %.2f, \"kept_box\": %.2f, "
               "\"kept_uncullable\": %.2f, \"kept_cone_sliver\": %.2f, \"kept_cone_other\": %.2f, \"packed_tri_rounds\": %.3f, \"untightened_clusters\": %.2f, \"untightened_packed_rounds\": %.3f}\n",
               prm.cluster_max, prm.split_angle, prm.min_cull_cos, prm.cut_clusters, nc, nk, nr, (double)screen / nr,
               (double)crounds / nr, (double)trounds / nr, (double)ctests / nr, (double)surv_sub / nr, (double)surv_cl / nr,
               (double)tris_tested / nr, (unsigned long long)mism, (double)reason[1] / nr, (double)reason[2] / nr,
               (double)reason[3] / nr, (double)reason[4] / nr, (double)reason[5] / nr, (double)reason[6] / nr, (double)prounds / nr, (double)all_cl / nr, (double)all_rounds / nr);
        fflush(stdout);
    }
    return 0;
}
