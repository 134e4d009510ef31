/* order_probe.c -- analysis tool (test infrastructure, includes the oracle): what a nearest-child-first
 * traversal would save over BVHRayHit's fixed DFS order (main_raytracing.cu:43-78: push left, push right,
 * pop -- right first), and how often its result could differ from the reference's.
 *
 * Ordered: at an inner node both children are tested against `closest` and the nearer (rounded slab
 * tmin) is visited first; a candidate is kept by the reference's own rule restated in (t, DFS position)
 * order (position = the leaf's rank in the reference's right-first DFS, then the triangle's index in the
 * leaf), so ties go to the triangle the reference would have found first.  The result can still differ
 * where the reference culls a node because a hit found before it lies at or below the node's ROUNDED
 * entry tmin while one of its triangles has a ROUNDED distance below that tmin; the tool counts the
 * segments where the final hit's leaf box has tmin_P > t_F (where such a difference is possible) and the
 * segments whose hit actually differs.
 *
 *   gcc -O2 -fopenmp -ffp-contract=off -o /tmp/order_probe tools/order_probe.c -lm
 *   /tmp/order_probe assets [scene 0|1] [width height spp row_step]
 */
#include "../oracle/rt_oracle.c"

typedef struct { uint64_t segs, nodes_ref, nodes_ord, tris_ref, tris_ord, mism, anomaly; } Acc;
typedef struct { float t; int kind; uint32_t id; uint64_t pos; uint32_t leaf; } Res;

static uint32_t* g_rank;  /* DFS rank of every leaf node (right-first, as the reference pops) */

static float slab_tmin(v3 o, v3 d, const ONode* n, float* tmax_o) {
    float tx1 = (n->bmin[0] - o.x) / d.x, tx2 = (n->bmax[0] - o.x) / d.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    float ty1 = (n->bmin[1] - o.y) / d.y, ty2 = (n->bmax[1] - o.y) / d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2)), tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (n->bmin[2] - o.z) / d.z, tz2 = (n->bmax[2] - o.z) / d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2)), tmax = fminf(tmax, fmaxf(tz1, tz2));
    *tmax_o = tmax;
    return tmin;
}

static void rank_leaves(const OScene* s) {
    g_rank = (uint32_t*)calloc(s->nnodes, 4);
    uint32_t stack[128], r = 0;
    int top = 0;
    stack[top++] = 0;
    while (top) {
        const uint32_t ni = stack[--top];
        const ONode* n = &s->nodes[ni];
        if (n->count > 0) { g_rank[ni] = r++; continue; }
        stack[top++] = n->first;
        stack[top++] = n->first + 1;
    }
}

static int tri_t(const OScene* s, uint32_t fi, v3 ro, v3 nd, float* t) {
    const OFace* f = &s->faces[fi];
    const OVertex *v0 = &s->verts[f->v0], *v1 = &s->verts[f->v1], *v2 = &s->verts[f->v2];
    float bx, by;
    return tri_hit(ro, nd, V(v0->p[0], v0->p[1], v0->p[2]), V(v1->p[0], v1->p[1], v1->p[2]), V(v2->p[0], v2->p[1], v2->p[2]), &bx,
                   &by, t);
}

static void spheres(const OScene* s, v3 ro, v3 nd, Res* r) {
    r->t = 1e30f, r->kind = 0, r->id = 0, r->pos = 0, r->leaf = UINT32_MAX;
    for (int i = 0; i < s->nspheres; i++) {
        const OSphere* sp = &s->spheres[i];
        float dist;
        if (sphere_hit(ro, nd, V(sp->p[0], sp->p[1], sp->p[2]), sp->r * sp->r, &dist)) {
            if (dist >= r->t) continue;
            r->t = dist, r->kind = 1, r->id = (uint32_t)i;
        }
    }
}

static Res ref_hit(const OScene* s, v3 ro, v3 rd, uint64_t* nodes, uint64_t* tris) {
    const v3 nd = vnorm(rd);
    Res r;
    spheres(s, ro, nd, &r);
    uint32_t stack[128];
    int top = 0;
    stack[top++] = 0;
    while (top) {
        const uint32_t ni = stack[--top];
        const ONode* n = &s->nodes[ni];
        (*nodes)++;
        float tmax;
        const float tmin = slab_tmin(ro, rd, n, &tmax);
        if (!(tmax >= tmin && tmin < r.t && tmax > 0)) continue;
        if (n->count > 0) {
            for (uint32_t i = 0; i < n->count; i++) {
                float t;
                (*tris)++;
                if (tri_t(s, s->face_idx[n->first + i], ro, nd, &t)) {
                    if (t >= r.t || t < 0.0f) continue;
                    r.t = t, r.kind = 2, r.id = s->face_idx[n->first + i], r.leaf = ni;
                }
            }
        } else {
            stack[top++] = n->first;
            stack[top++] = n->first + 1;
        }
    }
    return r;
}

static Res ord_hit(const OScene* s, v3 ro, v3 rd, uint64_t* nodes, uint64_t* tris) {
    const v3 nd = vnorm(rd);
    Res r;
    spheres(s, ro, nd, &r);
    uint32_t stack[128];
    int top = 0;
    stack[top++] = 0;
    int bpos_valid = 0;  /* a triangle candidate holds r.pos */
    while (top) {
        const uint32_t ni = stack[--top];
        const ONode* n = &s->nodes[ni];
        (*nodes)++;
        float tmax;
        const float tmin = slab_tmin(ro, rd, n, &tmax);
        /* ties on t stay in (position decides them): cull only when tmin > closest */
        if (!(tmax >= tmin && tmax > 0) || tmin > r.t || (tmin == r.t && !bpos_valid)) continue;
        if (n->count > 0) {
            for (uint32_t i = 0; i < n->count; i++) {
                float t;
                (*tris)++;
                if (!tri_t(s, s->face_idx[n->first + i], ro, nd, &t) || t < 0.0f) continue;
                const uint64_t pos = ((uint64_t)g_rank[ni] << 32) | i;
                if (t < r.t || (t == r.t && bpos_valid && pos < r.pos))
                    r.t = t, r.kind = 2, r.id = s->face_idx[n->first + i], r.pos = pos, r.leaf = ni, bpos_valid = 1;
            }
        } else {
            float ta, tb, xa, xb;
            ta = slab_tmin(ro, rd, &s->nodes[n->first], &xa);
            tb = slab_tmin(ro, rd, &s->nodes[n->first + 1], &xb);
            /* nearer child on top */
            if (ta <= tb) stack[top++] = n->first + 1, stack[top++] = n->first;
            else stack[top++] = n->first, stack[top++] = n->first + 1;
        }
    }
    return r;
}

static void probe_path(const OScene* s, v3 ro, v3 rd, ORng* rng, int bounces, Acc* acc) {
    v3 thr = V(1, 1, 1);
    for (int b = 0; b < bounces; b++) {
        uint64_t nr = 0, no = 0, tr = 0, to = 0;
        const Res R = ref_hit(s, ro, rd, &nr, &tr);
        const Res O = ord_hit(s, ro, rd, &no, &to);
        acc->segs++, acc->nodes_ref += nr, acc->nodes_ord += no, acc->tris_ref += tr, acc->tris_ord += to;
        if (memcmp(&R.t, &O.t, 4) != 0 || R.kind != O.kind || R.id != O.id) acc->mism++;
        if (O.kind == 2) {
            float tmax;
            if (slab_tmin(ro, rd, &s->nodes[O.leaf], &tmax) > O.t) acc->anomaly++;
        }
        if (R.kind == 0) break;
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
    const int which = argc > 2 ? atoi(argv[2]) : 0;
    const int w = argc > 3 ? atoi(argv[3]) : 1920, hgt = argc > 4 ? atoi(argv[4]) : 1080;
    const int spp = argc > 5 ? atoi(argv[5]) : 8, step = argc > 6 ? atoi(argv[6]) : 64;
    OScene* s = oracle_scene_create(which, argv[1], 0);
    if (!s) return 1;
    rank_leaves(s);
    OCamera cam;
    o_camera(s, w, hgt, &cam);
    v3 co = V(cam.origin[0], cam.origin[1], cam.origin[2]), ch = V(cam.horizontal[0], cam.horizontal[1], cam.horizontal[2]);
    v3 cv = V(cam.vertical[0], cam.vertical[1], cam.vertical[2]), cl = V(cam.llc[0], cam.llc[1], cam.llc[2]);
    jump_init();
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
           "\"nodes_ref\": %llu, \"nodes_ordered\": %llu, \"tris_ref\": %llu, \"tris_ordered\": %llu, "
           "\"hit_differs\": %llu, \"hit_below_its_leaf_entry\": %llu}\n",
           which, w, hgt, spp, step, (unsigned long long)tot.segs, (unsigned long long)tot.nodes_ref,
           (unsigned long long)tot.nodes_ord, (unsigned long long)tot.tris_ref, (unsigned long long)tot.tris_ord,
           (unsigned long long)tot.mism, (unsigned long long)tot.anomaly);
    oracle_scene_destroy(s);
    return 0;
}
