/* defer_probe.c -- analysis tool (test infrastructure, includes the oracle): what deferring a ray's
 * giant BVH leaf to the end of its own traversal would change.
 *
 * BVHRayHit (main_raytracing.cu:43-71) tests a leaf's triangles when it pops the leaf, so the rest of
 * the traversal is culled by whatever the leaf hits.  Deferred: the first leaf of >= GIANT triangles a
 * ray reaches is skipped and remembered; the traversal goes on with the distance it had (it visits a
 * superset of the reference's nodes); at the end the leaf is tested against the bound the rest of the
 * scene left.  The result is the reference's if the leaf wins ties against a hit found after the leaf
 * in DFS order (the reference would have tested the leaf first, and an equal distance later is not
 * accepted) and loses them against one found before it, PROVIDED the reference still reaches the leaf of
 * that later hit: when the hit's rounded distance lies below its own leaf box's rounded entry tmin, the
 * leaf must hold nothing at or below that tmin (the guard, as rt_fast.h: a second walk; otherwise the
 * reference order); a NaN distance anywhere after the leaf falls back to the reference order too.  This tool checks that rule against the oracle's own traversal on
 * every segment of sampled rows and prices it: node visits, and the giant leaf's triangles whose own
 * bounding box the ray enters below the bound (a proxy for the leaf tree's cull) at the leaf's entry
 * distance vs at the end-of-traversal bound.
 *
 *   gcc -O2 -fopenmp -ffp-contract=off -o /tmp/defer_probe tools/defer_probe.c -lm
 *   /tmp/defer_probe assets [scene 0|1] [width height spp row_step giant rays.bin]
 */
#include "../oracle/rt_oracle.c"

static uint32_t GIANT = 1024u;  /* leaves deferred: >= GIANT triangles (argv[7]) */
static FILE* g_rays;            /* argv[8]: per giant-leaf visit origin, nd, entry bound, end bound, changed (9 floats) */

typedef struct {
    uint64_t segs, giant_segs, nodes_ref, nodes_def, boxes_entry, boxes_end, mism, nan_fallback, leaf_won, tris_ref,
        tris_def, end_finite, entry_finite, cl_entry, cl_end, leaf_culled_end;
} Acc;

/* 16-triangle clusters of the giant leaves in Morton order of their centroids (a stand-in for the leaf
   tree's clusters, leaftree.h) */
typedef struct { uint32_t leaf; uint32_t n; ONode* box; } Clusters;
static Clusters g_cl[8];
static int g_ncl;
static uint32_t spread10(uint32_t v) {
    v &= 1023u;
    v = (v | (v << 16)) & 0x030000FFu; v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u; v = (v | (v << 2)) & 0x09249249u;
    return v;
}
typedef struct { uint32_t key, fi; } KF;
static int kf_cmp(const void* a, const void* b) {
    const uint32_t x = ((const KF*)a)->key, y = ((const KF*)b)->key;
    return x < y ? -1 : x > y;
}
static void build_clusters(const OScene* s) {
    for (uint32_t ni = 0; ni < s->nnodes && g_ncl < 8; ni++) {
        const ONode* n = &s->nodes[ni];
        if (n->count < GIANT) continue;
        KF* k = (KF*)malloc(n->count * sizeof(KF));
        for (uint32_t i = 0; i < n->count; i++) {
            const OFace* f = &s->faces[s->face_idx[n->first + i]];
            const OVertex *a = &s->verts[f->v0], *b = &s->verts[f->v1], *c = &s->verts[f->v2];
            uint32_t q[3];
            for (int d = 0; d < 3; d++) {
                const float cen = (a->p[d] + b->p[d] + c->p[d]) / 3.0f, ext = n->bmax[d] - n->bmin[d];
                q[d] = (uint32_t)(ext > 0 ? 1023.0f * (cen - n->bmin[d]) / ext : 0);
            }
            k[i].key = spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2);
            k[i].fi = s->face_idx[n->first + i];
        }
        qsort(k, n->count, sizeof(KF), kf_cmp);
        Clusters* C = &g_cl[g_ncl++];
        C->leaf = ni, C->n = (n->count + 15) / 16, C->box = (ONode*)calloc(C->n, sizeof(ONode));
        for (uint32_t c = 0; c < C->n; c++) {
            ONode* B = &C->box[c];
            for (int d = 0; d < 3; d++) B->bmin[d] = 1e30f, B->bmax[d] = -1e30f;
            for (uint32_t i = 16 * c; i < n->count && i < 16 * c + 16; i++) {
                const OFace* f = &s->faces[k[i].fi];
                const OVertex* v[3] = {&s->verts[f->v0], &s->verts[f->v1], &s->verts[f->v2]};
                for (int j = 0; j < 3; j++)
                    for (int d = 0; d < 3; d++) B->bmin[d] = fminf(B->bmin[d], v[j]->p[d]), B->bmax[d] = fmaxf(B->bmax[d], v[j]->p[d]);
            }
        }
        free(k);
    }
}

typedef struct { float t; int kind; uint32_t id; } Res;  /* kind 0 none, 1 sphere, 2 triangle */

/* IntersectAABB's rounded entry parameter (Math.h:50-61 arithmetic, as aabb_hit) */
static float aabb_tmin(v3 o, v3 d, const ONode* n) {
    float tx1 = (n->bmin[0] - o.x) / d.x, tx2 = (n->bmax[0] - o.x) / d.x;
    float tmin = fminf(tx1, tx2);
    float ty1 = (n->bmin[1] - o.y) / d.y, ty2 = (n->bmax[1] - o.y) / d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2));
    float tz1 = (n->bmin[2] - o.z) / d.z, tz2 = (n->bmax[2] - o.z) / d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2));
    return tmin;
}
static uint64_t g_again, g_redo;  /* the guard (rt_fast.h): second walks, and lanes redone in reference order */

static int tri_box_hit(const OScene* s, uint32_t fi, v3 ro, v3 rd, float bound) {
    const OFace* f = &s->faces[fi];
    const OVertex *a = &s->verts[f->v0], *b = &s->verts[f->v1], *c = &s->verts[f->v2];
    ONode n;
    for (int k = 0; k < 3; k++) {
        n.bmin[k] = fminf(fminf(a->p[k], b->p[k]), c->p[k]);
        n.bmax[k] = fmaxf(fmaxf(a->p[k], b->p[k]), c->p[k]);
    }
    return aabb_hit(ro, rd, &n, bound);
}

static int tri_t(const OScene* s, uint32_t fi, v3 ro, v3 nd, float* t) {
    const OFace* f = &s->faces[fi];
    const OVertex *v0 = &s->verts[f->v0], *v1 = &s->verts[f->v1], *v2 = &s->verts[f->v2];
    float bx, by;
    return tri_hit(ro, nd, V(v0->p[0], v0->p[1], v0->p[2]), V(v1->p[0], v1->p[1], v1->p[2]), V(v2->p[0], v2->p[1], v2->p[2]), &bx,
                   &by, t);
}

static void spheres(const OScene* s, v3 ro, v3 nd, Res* r) {
    r->t = 1e30f, r->kind = 0, r->id = 0;
    for (int i = 0; i < s->nspheres; i++) {
        const OSphere* sp = &s->spheres[i];
        float dist;
        if (sphere_hit(ro, nd, V(sp->p[0], sp->p[1], sp->p[2]), sp->r * sp->r, &dist)) {
            if (dist >= r->t) continue;
            r->t = dist, r->kind = 1, r->id = (uint32_t)i;
        }
    }
}

/* the reference order (main_raytracing.cu:43-71); entry = closest when the first giant leaf is reached */
static Res ref_hit(const OScene* s, v3 ro, v3 rd, uint64_t* nodes, uint64_t* tris, float* entry, uint32_t* giant) {
    const v3 nd = vnorm(rd);
    Res r;
    spheres(s, ro, nd, &r);
    *giant = UINT32_MAX;
    uint32_t stack[64];
    int top = 0;
    stack[top++] = 0;
    while (top) {
        const uint32_t ni = stack[--top];
        const ONode* n = &s->nodes[ni];
        (*nodes)++;
        if (!aabb_hit(ro, rd, n, r.t)) continue;
        if (n->count > 0) {
            if (n->count >= GIANT && *giant == UINT32_MAX) *giant = ni, *entry = r.t;
            for (uint32_t i = 0; i < n->count; i++) {
                float t;
                (*tris)++;
                if (tri_t(s, s->face_idx[n->first + i], ro, nd, &t)) {
                    if (t >= r.t || t < 0.0f) continue;
                    r.t = t, r.kind = 2, r.id = s->face_idx[n->first + i];
                }
            }
        } else {
            stack[top++] = n->first;
            stack[top++] = n->first + 1;
        }
    }
    return r;
}

/* deferred: the first giant leaf skipped, tested at the end against the remaining bound */
static Res def_hit(const OScene* s, v3 ro, v3 rd, uint64_t* nodes, uint64_t* tris, float* bound_end, int* nan_fb,
                   int* leaf_won) {
    const v3 nd = vnorm(rd);
    Res r;
    spheres(s, ro, nd, &r);
    uint32_t giant = UINT32_MAX, leaf_f = UINT32_MAX;
    int changed = 0, nan_after = 0;
    uint32_t stack[64];
    int top = 0;
    stack[top++] = 0;
    *nan_fb = 0, *leaf_won = 0;
    while (top) {
        const uint32_t ni = stack[--top];
        const ONode* n = &s->nodes[ni];
        (*nodes)++;
        if (!aabb_hit(ro, rd, n, r.t)) continue;
        if (n->count > 0) {
            if (n->count >= GIANT && giant == UINT32_MAX) {
                giant = ni;
                continue;
            }
            for (uint32_t i = 0; i < n->count; i++) {
                float t;
                (*tris)++;
                if (tri_t(s, s->face_idx[n->first + i], ro, nd, &t)) {
                    if (t >= r.t || t < 0.0f) continue;
                    r.t = t, r.kind = 2, r.id = s->face_idx[n->first + i];
                    if (giant != UINT32_MAX) changed = 1, nan_after |= (t != t), leaf_f = ni;
                }
            }
        } else {
            stack[top++] = n->first;
            stack[top++] = n->first + 1;
        }
    }
    *bound_end = r.t;
    if (giant == UINT32_MAX) return r;
    /* the leaf in its own order: strict < against the bound, except that the first accept may equal a
       bound set after the leaf (the leaf came first in DFS order) */
    const ONode* n = &s->nodes[giant];
    float cur = r.t;
    int incl = changed;
    for (uint32_t i = 0; i < n->count; i++) {
        float t;
        (*tris)++;
        if (tri_t(s, s->face_idx[n->first + i], ro, nd, &t)) {
            if (t != t) nan_after = 1;
            const int acc = incl ? !(t > cur || t < 0.0f) : !(t >= cur || t < 0.0f);
            if (!acc) continue;
            cur = t, incl = 0;
            r.t = t, r.kind = 2, r.id = s->face_idx[n->first + i];
            *leaf_won = 1;
        }
    }
    if (nan_after) *nan_fb = 1;
    /* the guard: the leaf found nothing and the rest's best came after it -- the reference reaches that
       best's leaf only if the deferred leaf holds nothing at or below the leaf's rounded entry tmin */
    if (changed && !*leaf_won && leaf_f != UINT32_MAX) {
        const float tp = aabb_tmin(ro, rd, &s->nodes[leaf_f]);
        if (tp > r.t) {
#pragma omp atomic
            g_again++;
            for (uint32_t i = 0; i < n->count; i++) {
                float t;
                if (tri_t(s, s->face_idx[n->first + i], ro, nd, &t) && !(t > tp || t < 0.0f)) {
                    *nan_fb = 1;  /* redone in the reference order */
#pragma omp atomic
                    g_redo++;
                    break;
                }
            }
        }
    }
    return r;
}

/* the oracle's path (main_raytracing.cu:111-160) driven by the reference hit, no colour kept */
static void probe_path(const OScene* s, v3 ro, v3 rd, ORng* rng, int bounces, Acc* acc) {
    v3 thr = V(1, 1, 1);
    for (int b = 0; b < bounces; b++) {
        uint64_t nr = 0, nd_ = 0, tr = 0, td = 0;
        float entry = 1e30f, bend = 1e30f;
        uint32_t giant;
        int nan_fb, leaf_won;
        const Res R = ref_hit(s, ro, rd, &nr, &tr, &entry, &giant);
        const Res D = def_hit(s, ro, rd, &nd_, &td, &bend, &nan_fb, &leaf_won);
        acc->segs++;
        acc->nodes_ref += nr, acc->nodes_def += nd_, acc->tris_ref += tr, acc->tris_def += td;
        if (giant != UINT32_MAX) {
            acc->giant_segs++;
            acc->entry_finite += entry < 1e30f;
            acc->end_finite += bend < 1e30f;
            acc->leaf_won += leaf_won;
            acc->leaf_culled_end += !aabb_hit(ro, rd, &s->nodes[giant], bend);
            if (g_rays) {
                const v3 ndn = vnorm(rd);
                uint32_t ch = memcmp(&entry, &bend, 4) != 0;
                float rec[9] = {ro.x, ro.y, ro.z, ndn.x, ndn.y, ndn.z, entry, bend, 0};
                memcpy(&rec[8], &ch, 4);
#pragma omp critical
                fwrite(rec, 4, 9, g_rays);
            }
            for (int c = 0; c < g_ncl; c++)
                if (g_cl[c].leaf == giant)
                    for (uint32_t j = 0; j < g_cl[c].n; j++) {
                        acc->cl_entry += aabb_hit(ro, rd, &g_cl[c].box[j], entry);
                        acc->cl_end += aabb_hit(ro, rd, &g_cl[c].box[j], bend);
                    }
            const ONode* n = &s->nodes[giant];
            for (uint32_t i = 0; i < n->count; i++) {
                const uint32_t fi = s->face_idx[n->first + i];
                acc->boxes_entry += tri_box_hit(s, fi, ro, rd, entry);
                acc->boxes_end += tri_box_hit(s, fi, ro, rd, bend);
            }
        }
        if (nan_fb) acc->nan_fallback++;
        else if (memcmp(&R.t, &D.t, 4) != 0 || R.kind != D.kind || R.id != D.id) acc->mism++;
        if (R.kind == 0) break;
        /* continue the path from the reference hit, as the oracle does */
        OHit h;
        OStats st;
        memset(&st, 0, sizeof st);
        if (!get_ray_hit(s, ro, rd, &h, &st)) break;
        const OMaterial* m = h.mat;
        float ds = (rng_uniform(rng) < m->spec_pct) ? 1.0f : 0.0f;
        float om = 1.0f - ds;
        thr = vmul(thr, V(m->albedo[0] * om + m->specular[0] * ds, m->albedo[1] * om + m->specular[1] * ds,
                          m->albedo[2] * om + m->specular[2] * ds));
        float zz = rng_uniform(rng) * 2.0f - 1.0f;
        float ang = rng_uniform(rng) * 3.141592654f * 2.0f;
        float rr = sqrtf(1.0f - zz * zz);
        v3 sp = V(rr * o_cos(ang), rr * o_sin(ang), zz);
        v3 diffuse = vnorm(vadd(h.nrm, sp));
        v3 spec = vnorm(vreflect(rd, h.nrm));
        spec = vnorm(vmix(spec, diffuse, m->rough * m->rough));
        v3 ndir = vnorm(vadd(vscale(diffuse, om), vscale(spec, ds)));
        ro = vadd(h.pos, vscale(h.nrm, 0.01f));
        rd = ndir;
        float p = gmax(thr.x, gmax(thr.y, thr.z));
        if (rng_uniform(rng) > p) break;
        thr = vscale(thr, 1.0f / p);
    }
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s assets [scene width height spp row_step]\n", argv[0]);
        return 2;
    }
    const int which = argc > 2 ? atoi(argv[2]) : 1;
    const int w = argc > 3 ? atoi(argv[3]) : 1920, hgt = argc > 4 ? atoi(argv[4]) : 1080;
    const int spp = argc > 5 ? atoi(argv[5]) : 8, step = argc > 6 ? atoi(argv[6]) : 64;
    if (argc > 7) GIANT = (uint32_t)atoi(argv[7]);
    if (argc > 8) g_rays = fopen(argv[8], "wb");
    OScene* s = oracle_scene_create(which, argv[1], 0);
    if (!s) return 1;
    OCamera cam;
    o_camera(s, w, hgt, &cam);
    v3 co = V(cam.origin[0], cam.origin[1], cam.origin[2]), ch = V(cam.horizontal[0], cam.horizontal[1], cam.horizontal[2]);
    v3 cv = V(cam.vertical[0], cam.vertical[1], cam.vertical[2]), cl = V(cam.llc[0], cam.llc[1], cam.llc[2]);
    jump_init();
    build_clusters(s);
    Acc tot;
    memset(&tot, 0, sizeof tot);
#pragma omp parallel
    {
        Acc a;
        memset(&a, 0, sizeof a);
#pragma omp for schedule(dynamic, 1)
        for (int y = step / 2; y < hgt; y += step) {
            for (int x = 0; x < w; x++) {
                const uint32_t pid = (uint32_t)(y * w + x);
                ORng r;
                rng_init(0xDEADBEEFu, pid, &r);
                for (int smp = 0; smp < spp; smp++) {
                    float ru = rng_uniform(&r), rv = rng_uniform(&r);
                    float ux = ((float)x + ru) / (float)w, uy = ((float)y + rv) / (float)hgt;
                    v3 rd = vsub(vadd(vadd(cl, vscale(ch, ux)), vscale(cv, uy)), co);
                    probe_path(s, co, rd, &r, 6, &a);
                }
            }
        }
#pragma omp critical
        {
            uint64_t* d = (uint64_t*)&tot;
            const uint64_t* q = (const uint64_t*)&a;
            for (size_t i = 0; i < sizeof(Acc) / 8; i++) d[i] += q[i];
        }
    }
    printf("{\"scene\": %d, \"width\": %d, \"height\": %d, \"spp\": %d, \"row_step\": %d, \"segments\": %llu, "
           "\"giant_segments\": %llu, \"mismatches\": %llu, \"nan_fallbacks\": %llu, \"leaf_won\": %llu, "
           "\"entry_bound_finite\": %llu, \"end_bound_finite\": %llu, \"nodes_ref\": %llu, \"nodes_deferred\": %llu, "
           "\"tris_ref\": %llu, \"tris_deferred\": %llu, \"leaf_boxes_at_entry\": %llu, \"leaf_boxes_at_end\": %llu, \"giant_leaves\": %d, \"clusters_at_entry\": %llu, \"clusters_at_end\": %llu, \"leaf_box_culled_at_end\": %llu, \"guard_second_walks\": %llu, \"guard_redone\": %llu}\n",
           which, w, hgt, spp, step, (unsigned long long)tot.segs, (unsigned long long)tot.giant_segs,
           (unsigned long long)tot.mism, (unsigned long long)tot.nan_fallback, (unsigned long long)tot.leaf_won,
           (unsigned long long)tot.entry_finite, (unsigned long long)tot.end_finite, (unsigned long long)tot.nodes_ref,
           (unsigned long long)tot.nodes_def, (unsigned long long)tot.tris_ref, (unsigned long long)tot.tris_def,
           (unsigned long long)tot.boxes_entry, (unsigned long long)tot.boxes_end, g_ncl, (unsigned long long)tot.cl_entry,
           (unsigned long long)tot.cl_end, (unsigned long long)tot.leaf_culled_end, (unsigned long long)g_again,
           (unsigned long long)g_redo);
    if (g_rays) fclose(g_rays);
    oracle_scene_destroy(s);
    return 0;
}
