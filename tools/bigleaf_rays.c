/* bigleaf_rays.c -- analysis tool: the rays that reach the big BVH leaves of a scene.
 *
 * Renders rows of a frame with the oracle's arithmetic (the oracle source is included, test
 * infrastructure) and, for every visit of a leaf of more than 8 triangles that passes its box test
 * (BVHRayHit, main_raytracing.cu:43-71), writes one record of 12 floats:
 *   origin.xyz, normalised direction.xyz, direction.xyz, closest distance at entry, leaf node (bits),
 *   leaf size (bits), pixel (bits), segment index in the sample (bits).
 * tools/bigleaf_cull.py reads the records to price exact cull screens for those leaves.
 *
 *   gcc -O2 -fopenmp -ffp-contract=off -o /tmp/bigleaf_rays tools/bigleaf_rays.c -lm
 *   /tmp/bigleaf_rays assets out.bin [scene 0|1] [width height spp row_step frame_rows]
 */
#include "../oracle/rt_oracle.c"

static FILE* g_out;

/* get_ray_hit with the big-leaf record hook (same decisions) */
static int probe_hit(const OScene* s, v3 ro, v3 rd, OHit* h, uint32_t pix, uint32_t seg) {
    v3 nd = vnorm(rd);
    h->dist = 1e30f;
    for (int i = 0; i < s->nspheres; i++) {
        const OSphere* sp = &s->spheres[i];
        float dist;
        if (sphere_hit(ro, nd, V(sp->p[0], sp->p[1], sp->p[2]), sp->r * sp->r, &dist)) {
            if (dist >= h->dist) continue;
            h->dist = dist;
            h->pos = vadd(ro, vscale(nd, dist));
            h->nrm = V((h->pos.x - sp->p[0]) / sp->r, (h->pos.y - sp->p[1]) / sp->r, (h->pos.z - sp->p[2]) / sp->r);
            h->mat = &s->mats[sp->mat];
        }
    }
    uint32_t stack[64];
    int top = 0;
    stack[top++] = 0;
    while (top) {
        const uint32_t ni = stack[--top];
        const ONode* n = &s->nodes[ni];
        if (!aabb_hit(ro, rd, n, h->dist)) continue;
        if (n->count > 0) {
            if (n->count > 8) {
                float rec[12] = {ro.x, ro.y, ro.z, nd.x, nd.y, nd.z, rd.x, rd.y, rd.z, h->dist, 0, 0};
                uint32_t u[4] = {ni, n->count, pix, seg};
                memcpy(&rec[10], u, 8);
#pragma omp critical
                {
                    fwrite(rec, 4, 12, g_out);
                    fwrite(&u[2], 4, 2, g_out);
                }
            }
            for (uint32_t i = 0; i < n->count; i++) {
                const OFace* f = &s->faces[s->face_idx[n->first + i]];
                const OVertex *v0 = &s->verts[f->v0], *v1 = &s->verts[f->v1], *v2 = &s->verts[f->v2];
                float bx, by, dist;
                if (tri_hit(ro, nd, V(v0->p[0], v0->p[1], v0->p[2]), V(v1->p[0], v1->p[1], v1->p[2]), V(v2->p[0], v2->p[1], v2->p[2]), &bx, &by, &dist)) {
                    if (dist >= h->dist || dist < 0.0f) continue;
                    float bz = (1.0f - bx) - by;
                    h->dist = dist;
                    h->pos = vadd(ro, vscale(nd, dist));
                    h->nrm = vnorm(vadd(vadd(vscale(V(v0->n[0], v0->n[1], v0->n[2]), bx), vscale(V(v1->n[0], v1->n[1], v1->n[2]), by)), vscale(V(v2->n[0], v2->n[1], v2->n[2]), bz)));
                    h->mat = &s->mats[f->mat];
                    if (vdot(nd, h->nrm) >= 0.0f) h->nrm = V(-h->nrm.x, -h->nrm.y, -h->nrm.z);
                }
            }
        } else {
            stack[top++] = n->first;
            stack[top++] = n->first + 1;
        }
    }
    return h->dist < 1e30f;
}

/* ray_color's path (main_raytracing.cu:111-160), no colour kept */
static void probe_path(const OScene* s, v3 ro, v3 rd, ORng* rng, int bounces, uint32_t pix) {
    v3 thr = V(1, 1, 1);
    for (int b = 0; b < bounces; b++) {
        OHit h;
        if (!probe_hit(s, ro, rd, &h, pix, (uint32_t)b)) break;
        const OMaterial* m = h.mat;
        float ds = (rng_uniform(rng) < m->spec_pct) ? 1.0f : 0.0f;
        float om = 1.0f - ds;
        thr = vmul(thr, V(m->albedo[0] * om + m->specular[0] * ds, m->albedo[1] * om + m->specular[1] * ds, m->albedo[2] * om + m->specular[2] * ds));
        float zz = rng_uniform(rng) * 2.0f - 1.0f;
        float ang = rng_uniform(rng) * 3.141592654f * 2.0f;
        float rr = sqrtf(1.0f - zz * zz);
        v3 sp = V(rr * o_cos(ang), rr * o_sin(ang), zz);
        v3 diffuse = vnorm(vadd(h.nrm, sp));
        v3 spec = vnorm(vreflect(rd, h.nrm));
        spec = vnorm(vmix(spec, diffuse, m->rough * m->rough));
        v3 nd = vnorm(vadd(vscale(diffuse, om), vscale(spec, ds)));
        ro = vadd(h.pos, vscale(h.nrm, 0.01f));
        rd = nd;
        float p = gmax(thr.x, gmax(thr.y, thr.z));
        if (rng_uniform(rng) > p) break;
        thr = vscale(thr, 1.0f / p);
    }
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s assets out.bin [scene width height spp row_step]\n", argv[0]);
        return 2;
    }
    const int which = argc > 3 ? atoi(argv[3]) : 0;
    const int w = argc > 4 ? atoi(argv[4]) : 1920, hgt = argc > 5 ? atoi(argv[5]) : 1080;
    const int spp = argc > 6 ? atoi(argv[6]) : 8, step = argc > 7 ? atoi(argv[7]) : 16;
    OScene* s = oracle_scene_create(which, argv[1], 0);
    if (!s) return 1;
    g_out = fopen(argv[2], "wb");
    OCamera cam;
    o_camera(s, w, hgt, &cam);
    v3 co = V(cam.origin[0], cam.origin[1], cam.origin[2]), ch = V(cam.horizontal[0], cam.horizontal[1], cam.horizontal[2]);
    v3 cv = V(cam.vertical[0], cam.vertical[1], cam.vertical[2]), cl = V(cam.llc[0], cam.llc[1], cam.llc[2]);
    jump_init();
#pragma omp parallel for schedule(dynamic, 1)
    for (int y = step / 2; y < hgt; y += step) {
        for (int x = 0; x < w; x++) {
            const uint32_t pid = (uint32_t)(y * w + x);
            ORng r;
            rng_init(0xDEADBEEFu, pid, &r);
            for (int smp = 0; smp < spp; smp++) {
                float ru = rng_uniform(&r), rv = rng_uniform(&r);
                float ux = ((float)x + ru) / (float)w, uy = ((float)y + rv) / (float)hgt;
                v3 rd = vsub(vadd(vadd(cl, vscale(ch, ux)), vscale(cv, uy)), co);
                probe_path(s, co, rd, &r, 6, pid);
            }
        }
    }
    fclose(g_out);
    oracle_scene_destroy(s);
    return 0;
}
