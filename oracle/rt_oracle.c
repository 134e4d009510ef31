/*
 * rt_oracle.c -- CPU restatement of the reference's hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker (or as the timed CPU baseline) -- never as part of the
 * product path.  It is written independently of the product sources (plain C, its own
 * scene builder, BVH builder, camera, RNG seeding with its own jump tables, renderer and
 * sky sampler) so that agreement between the two is evidence, not tautology.
 *
 * Parity status (see DESIGN.md "Parity"):
 *   - The reference cannot be built here (MSBuild + CUDA 11.7 + Windows headers; building
 *     its kernel would need stand-ins for cuda_runtime.h / curand_kernel.h, which the rules
 *     forbid), and it ships no tests, fixtures or golden outputs.  Parity against the
 *     reference's own outputs is therefore UNPINNED.
 *   - Partial pins: every glm operation this file restates (intersectRayTriangle,
 *     intersectRaySphere, normalize / cross / dot / reflect / mix / min / max / clamp,
 *     quat * vec3, the camera's quat / mat4_cast / translate / scale / perspectiveRH / inverse
 *     chain, rotate, mat4 * vec4) is checked bit for bit against the reference's OWN vendored
 *     glm 0.9.9.8 compiled here (oracle/ref_glm.cpp + oracle/build_ref.sh -> oracle/_ref/;
 *     tests/test_oracle_glm.py, vectors in tests/golden/glm_vectors.npz); the XORWOW jump
 *     matrices against rocrand's published table (same recurrence); the bunny mesh is the
 *     assimp 3.3 import (assets/bunny_mesh.bin).  Still unpinned: curand's seeding constants,
 *     the scene / BVH builder's control flow, the texture unit's filtering, CUDA's sinf/cosf.
 *   - Semantics restated: the reference's arithmetic in IEEE fp32 WITHOUT contraction
 *     (nvcc contracts by default; not reproducible), curand's published XORWOW seeding and
 *     uniform mapping, the RT deterministic sin/cos and cube sampler definitions.
 *
 * Each function cites the reference file:line it restates (paths relative to the
 * reference repository root).  Build: gcc -O2 -fopenmp -ffp-contract=off (see
 * cuda-raytracing_amd/build.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------ */
/* data layout (RayTracing/GPUScene.h:25-74)                                             */
/* ------------------------------------------------------------------------------------ */
typedef struct { float p[3], n[3], uv[2]; } OVertex;                     /* GPUVertex */
typedef struct { uint32_t v0, v2, v1, mat; } OFace;                      /* GPUFace (v0, v2, v1!) */
typedef struct { float bmin[3], bmax[3]; uint32_t first, count; } ONode; /* GPUBVHNode */
typedef struct { float p[3]; float r; int32_t mat; int32_t pad[3]; } OSphere;
typedef struct { float albedo[4], emissive[4], specular[4], rough, spec_pct, ior, pad; } OMaterial;
typedef struct { float origin[3], vws[2], aspect, horizontal[3], vertical[3], llc[3]; } OCamera;

typedef struct {
    OVertex* verts; size_t nverts, cap_verts;
    OFace* faces; size_t nfaces, cap_faces;
    OSphere spheres[64]; int nspheres;
    OMaterial mats[64]; int nmats;
    ONode* nodes; size_t nnodes;
    uint32_t* face_idx;
    int max_depth;
    float* sky; int sky_n;
    float cam_pos[3], cam_ax, cam_ay;
} OScene;

/* ------------------------------------------------------------------------------------ */
/* glm restatements (include/glm/detail/func_geometric.inl, func_common.inl)             */
/* ------------------------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;
static v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static v3 vscale(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
/* func_geometric.inl:46-53 */
static float vdot(v3 a, v3 b) { float x = a.x * b.x, y = a.y * b.y, z = a.z * b.z; return (x + y) + z; }
/* func_geometric.inl:66-77 */
static v3 vcross(v3 a, v3 b) { return V(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
/* func_geometric.inl:82-90 + func_exponential.inl:44-49 */
static v3 vnorm(v3 a) { float k = 1.0f / sqrtf(vdot(a, a)); return vscale(a, k); }
/* func_geometric.inl:104-110 */
static v3 vreflect(v3 i, v3 n) { return vsub(i, vscale(vscale(n, vdot(n, i)), 2.0f)); }
/* func_common.inl:104-112 */
static v3 vmix(v3 x, v3 y, float a) { float o = 1.0f - a; return vadd(vscale(x, o), vscale(y, a)); }
static float gmax(float x, float y) { return (x < y) ? y : x; } /* func_common.inl:25-30 */
static float gmin(float x, float y) { return (y < x) ? y : x; } /* func_common.inl:17-21 */

/* RT deterministic sin/cos: rint(x*2/pi) quadrant, 3-part Cody-Waite, cephes. */
static float o_reduce(float x, int* q) {
    float k = rintf(x * 0.636619746685028076171875f);
    *q = (int)k;
    float r = fmaf(k, -0x1.921fb6p+0f, x);
    r = fmaf(k, 0x1.777a5cp-25f, r);
    r = fmaf(k, 0x1.ee59dap-50f, r);
    return r;
}
static float o_sinp(float r) {
    float z = r * r;
    float p = fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f);
    p = fmaf(z, p, -1.6666654611e-1f);
    return fmaf(r * z, p, r);
}
static float o_cosp(float r) {
    float z = r * r;
    float p = fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
    p = fmaf(z, p, 4.166664568298827e-2f);
    return fmaf(z * z, p, fmaf(-0.5f, z, 1.0f));
}
static float o_sin(float x) { int q; float r = o_reduce(x, &q); switch (q & 3) { case 0: return o_sinp(r); case 1: return o_cosp(r); case 2: return -o_sinp(r); default: return -o_cosp(r); } }
static float o_cos(float x) { int q; float r = o_reduce(x, &q); switch (q & 3) { case 0: return o_cosp(r); case 1: return -o_sinp(r); case 2: return -o_cosp(r); default: return o_sinp(r); } }

/* host-side trig of the scene builder: correctly rounded via double (stands in for the
 * reference host compiler's sinf/cosf/tanf) */
static float h_sin(float x) { return (float)sin((double)x); }
static float h_cos(float x) { return (float)cos((double)x); }
static float h_tan(float x) { return (float)tan((double)x); }

/* ------------------------------------------------------------------------------------ */
/* 4x4 matrices, glm column-major m[col][row]                                            */
/* ------------------------------------------------------------------------------------ */
typedef struct { float m[4][4]; } M4;
static M4 m_ident(void) { M4 r; memset(&r, 0, sizeof r); for (int i = 0; i < 4; i++) r.m[i][i] = 1.0f; return r; }
/* type_mat4x4.inl:630-648 */
static M4 m_mul(M4 a, M4 b) {
    M4 r;
    for (int c = 0; c < 4; c++) for (int i = 0; i < 4; i++)
        r.m[c][i] = ((a.m[0][i] * b.m[c][0] + a.m[1][i] * b.m[c][1]) + a.m[2][i] * b.m[c][2]) + a.m[3][i] * b.m[c][3];
    return r;
}
/* type_mat4x4.inl:536-575 */
static void m_vec(const M4* a, const float v[4], float o[4]) {
    for (int i = 0; i < 4; i++) o[i] = (a->m[0][i] * v[0] + a->m[1][i] * v[1]) + (a->m[2][i] * v[2] + a->m[3][i] * v[3]);
}
/* ext/matrix_transform.inl:10-15 */
static M4 m_translate(M4 m, v3 v) {
    for (int i = 0; i < 4; i++) m.m[3][i] = ((m.m[0][i] * v.x + m.m[1][i] * v.y) + m.m[2][i] * v.z) + m.m[3][i];
    return m;
}
/* ext/matrix_transform.inl:78-86 */
static M4 m_scale(M4 m, v3 v) {
    for (int i = 0; i < 4; i++) { m.m[0][i] *= v.x; m.m[1][i] *= v.y; m.m[2][i] *= v.z; }
    return m;
}
/* ext/matrix_transform.inl:17-45 */
static M4 m_rotate(M4 m, float angle, v3 v) {
    float c = h_cos(angle), s = h_sin(angle);
    v3 ax = vnorm(v), t = vscale(ax, 1.0f - c);
    float R[3][3] = {
        {c + t.x * ax.x, t.x * ax.y + s * ax.z, t.x * ax.z - s * ax.y},
        {t.y * ax.x - s * ax.z, c + t.y * ax.y, t.y * ax.z + s * ax.x},
        {t.z * ax.x + s * ax.y, t.z * ax.y - s * ax.x, c + t.z * ax.z}};
    M4 r;
    for (int k = 0; k < 3; k++) for (int i = 0; i < 4; i++)
        r.m[k][i] = (m.m[0][i] * R[k][0] + m.m[1][i] * R[k][1]) + m.m[2][i] * R[k][2];
    for (int i = 0; i < 4; i++) r.m[3][i] = m.m[3][i];
    return r;
}
/* detail/func_matrix.inl:294-351 */
static M4 m_inverse(M4 M) {
    float (*m)[4] = M.m;
    float c00 = m[2][2] * m[3][3] - m[3][2] * m[2][3], c02 = m[1][2] * m[3][3] - m[3][2] * m[1][3], c03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float c04 = m[2][1] * m[3][3] - m[3][1] * m[2][3], c06 = m[1][1] * m[3][3] - m[3][1] * m[1][3], c07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float c08 = m[2][1] * m[3][2] - m[3][1] * m[2][2], c10 = m[1][1] * m[3][2] - m[3][1] * m[1][2], c11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float c12 = m[2][0] * m[3][3] - m[3][0] * m[2][3], c14 = m[1][0] * m[3][3] - m[3][0] * m[1][3], c15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float c16 = m[2][0] * m[3][2] - m[3][0] * m[2][2], c18 = m[1][0] * m[3][2] - m[3][0] * m[1][2], c19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float c20 = m[2][0] * m[3][1] - m[3][0] * m[2][1], c22 = m[1][0] * m[3][1] - m[3][0] * m[1][1], c23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    float F0[4] = {c00, c00, c02, c03}, F1[4] = {c04, c04, c06, c07}, F2[4] = {c08, c08, c10, c11};
    float F3[4] = {c12, c12, c14, c15}, F4[4] = {c16, c16, c18, c19}, F5[4] = {c20, c20, c22, c23};
    float A0[4] = {m[1][0], m[0][0], m[0][0], m[0][0]}, A1[4] = {m[1][1], m[0][1], m[0][1], m[0][1]};
    float A2[4] = {m[1][2], m[0][2], m[0][2], m[0][2]}, A3[4] = {m[1][3], m[0][3], m[0][3], m[0][3]};
    static const float SA[4] = {1, -1, 1, -1}, SB[4] = {-1, 1, -1, 1};
    M4 inv;
    for (int k = 0; k < 4; k++) {
        inv.m[0][k] = ((A1[k] * F0[k] - A2[k] * F1[k]) + A3[k] * F2[k]) * SA[k];
        inv.m[1][k] = ((A0[k] * F0[k] - A2[k] * F3[k]) + A3[k] * F4[k]) * SB[k];
        inv.m[2][k] = ((A0[k] * F1[k] - A1[k] * F3[k]) + A3[k] * F5[k]) * SA[k];
        inv.m[3][k] = ((A0[k] * F2[k] - A1[k] * F4[k]) + A2[k] * F5[k]) * SB[k];
    }
    float d0 = m[0][0] * inv.m[0][0], d1 = m[0][1] * inv.m[1][0], d2 = m[0][2] * inv.m[2][0], d3 = m[0][3] * inv.m[3][0];
    float det = (d0 + d1) + (d2 + d3);
    float od = 1.0f / det;
    for (int c = 0; c < 4; c++) for (int k = 0; k < 4; k++) inv.m[c][k] *= od;
    return inv;
}

/* ------------------------------------------------------------------------------------ */
/* Camera::Update (RayTracing/Scene.cpp:15-36)                                            */
/* ------------------------------------------------------------------------------------ */
static float o_radians(float d) { return d * 0.01745329251994329576923690768489f; }

static void o_camera(const OScene* s, int w, int h, OCamera* cam) {
    float aspect = (float)w / (float)h;
    /* quat(vec3 euler) (type_quat.inl:204-213) with host trig */
    float ex = o_radians(s->cam_ax) * 0.5f, ey = o_radians(s->cam_ay) * 0.5f, ez = 0.0f * 0.5f;
    float cx = h_cos(ex), cy = h_cos(ey), cz = h_cos(ez), sx = h_sin(ex), sy = h_sin(ey), sz = h_sin(ez);
    float qw = cx * cy * cz + sx * sy * sz, qx = sx * cy * cz - cx * sy * sz;
    float qy = cx * sy * cz + sx * cy * sz, qz = cx * cy * sz - sx * sy * cz;
    /* mat4_cast (gtc/quaternion.inl:41-72) */
    M4 R = m_ident();
    float qxx = qx * qx, qyy = qy * qy, qzz = qz * qz, qxz = qx * qz, qxy = qx * qy, qyz = qy * qz;
    float qwx = qw * qx, qwy = qw * qy, qwz = qw * qz;
    R.m[0][0] = 1.0f - 2.0f * (qyy + qzz); R.m[0][1] = 2.0f * (qxy + qwz); R.m[0][2] = 2.0f * (qxz - qwy);
    R.m[1][0] = 2.0f * (qxy - qwz); R.m[1][1] = 1.0f - 2.0f * (qxx + qzz); R.m[1][2] = 2.0f * (qyz + qwx);
    R.m[2][0] = 2.0f * (qxz + qwy); R.m[2][1] = 2.0f * (qyz - qwx); R.m[2][2] = 1.0f - 2.0f * (qxx + qyy);
    /* Math::ComposeMatrix (RayTracing/Math.h:63-70) */
    M4 T = m_translate(m_ident(), V(s->cam_pos[0], s->cam_pos[1], s->cam_pos[2]));
    T = m_scale(m_mul(T, R), V(1, 1, 1));
    /* perspectiveRH_NO (ext/matrix_clip_space.inl:249-262), fov 90, near 1, far 1000 */
    float fovy = o_radians(90.0f), th = h_tan(fovy / 2.0f), zf = 1000.0f, zn = 1.0f;
    M4 P;
    memset(&P, 0, sizeof P);
    P.m[0][0] = 1.0f / (aspect * th);
    P.m[1][1] = 1.0f / th;
    P.m[2][2] = -(zf + zn) / (zf - zn);
    P.m[2][3] = -1.0f;
    P.m[3][2] = -(2.0f * zf * zn) / (zf - zn);
    M4 IP = m_inverse(P);
    float llv[4] = {-1, -1, -1, 1}, urv[4] = {1, 1, -1, 1}, ll4[4], ur4[4];
    m_vec(&IP, llv, ll4);
    m_vec(&IP, urv, ur4);
    float ll[3] = {ll4[0] / ll4[3], ll4[1] / ll4[3], ll4[2] / ll4[3]};
    float ur[3] = {ur4[0] / ur4[3], ur4[1] / ur4[3], ur4[2] / ur4[3]};
    cam->vws[0] = ur[0] - ll[0];
    cam->vws[1] = ur[1] - ll[1];
    float hv[4] = {cam->vws[0], 0, 0, 0}, vv[4] = {0, cam->vws[1], 0, 0}, lv[4] = {ll[0], ll[1], ll[2], 1}, o[4];
    m_vec(&T, hv, o); memcpy(cam->horizontal, o, 12);
    m_vec(&T, vv, o); memcpy(cam->vertical, o, 12);
    m_vec(&T, lv, o); memcpy(cam->llc, o, 12);
    memcpy(cam->origin, s->cam_pos, 12);
    cam->aspect = aspect;
}

/* ------------------------------------------------------------------------------------ */
/* scene building (RayTracing/Scene.cpp:46-139)                                          */
/* ------------------------------------------------------------------------------------ */
static void push_vert(OScene* s, v3 p, v3 n) {
    if (s->nverts == s->cap_verts) {
        s->cap_verts = s->cap_verts ? 2 * s->cap_verts : 1024;
        s->verts = (OVertex*)realloc(s->verts, s->cap_verts * sizeof(OVertex));
    }
    OVertex* v = &s->verts[s->nverts++];
    v->p[0] = p.x; v->p[1] = p.y; v->p[2] = p.z;
    v->n[0] = n.x; v->n[1] = n.y; v->n[2] = n.z;
    v->uv[0] = v->uv[1] = 0.0f;
}
static void push_face(OScene* s, uint32_t v0, uint32_t v1, uint32_t v2, uint32_t mat) {
    if (s->nfaces == s->cap_faces) {
        s->cap_faces = s->cap_faces ? 2 * s->cap_faces : 1024;
        s->faces = (OFace*)realloc(s->faces, s->cap_faces * sizeof(OFace));
    }
    OFace* f = &s->faces[s->nfaces++];
    f->v0 = v0; f->v1 = v1; f->v2 = v2; f->mat = mat;
}
/* Scene::AddTriangle (Scene.cpp:46-67): GPUFace{i0, i0+1, i0+2} -> v0=i0, v2=i0+1, v1=i0+2 */
static void add_triangle(OScene* s, v3 a, v3 b, v3 c, int mat) {
    v3 n = vnorm(vcross(vsub(c, b), vsub(a, b)));
    uint32_t i0 = (uint32_t)s->nverts;
    push_vert(s, a, n); push_vert(s, b, n); push_vert(s, c, n);
    push_face(s, i0, i0 + 2, i0 + 1, (uint32_t)mat);
}
static void add_quad(OScene* s, v3 a, v3 b, v3 c, v3 d, int mat) { add_triangle(s, a, b, c, mat); add_triangle(s, c, d, a, mat); }
static void add_sphere(OScene* s, v3 p, float r, int mat) {
    OSphere* o = &s->spheres[s->nspheres++];
    memset(o, 0, sizeof *o);
    o->p[0] = p.x; o->p[1] = p.y; o->p[2] = p.z; o->r = r; o->mat = mat;
}
/* Material(albedo, emissive) (Scene.h:76-80) + GPUMaterial defaults (GPUScene.h:66-74) */
static int add_material(OScene* s, v3 albedo, v3 emissive, float spec_pct, v3 spec, float rough) {
    OMaterial* m = &s->mats[s->nmats];
    memset(m, 0, sizeof *m);
    m->albedo[0] = albedo.x; m->albedo[1] = albedo.y; m->albedo[2] = albedo.z; m->albedo[3] = 1.0f;
    m->emissive[0] = emissive.x; m->emissive[1] = emissive.y; m->emissive[2] = emissive.z; m->emissive[3] = 1.0f;
    m->specular[0] = spec.x; m->specular[1] = spec.y; m->specular[2] = spec.z; m->specular[3] = 0.0f;
    m->rough = rough; m->spec_pct = spec_pct; m->ior = 1.0f;
    return s->nmats++;
}
static int add_plain_material(OScene* s, v3 albedo, v3 emissive) { return add_material(s, albedo, emissive, 0.0f, V(0, 0, 0), 0.9f); }

typedef struct { float* pos; float* nrm; uint32_t* idx; uint32_t nv, nf; M4 node; } OMesh;

/* assets/bunny_mesh.bin = the assimp import the reference receives (tools/make_assets.py);
 * node transform = aiMatrix4x4::RotationX(-(float)M_PI/2) * identity * identity, transposed
 * into glm order (utils/AssimpLoader.cpp:8-27,47-48). */
static int load_mesh(const char* path, OMesh* m) {
    FILE* f = fopen(path, "rb");
    if (!f) return 1;
    char magic[8];
    if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "RTMESH01", 8) || fread(&m->nv, 4, 1, f) != 1 || fread(&m->nf, 4, 1, f) != 1) { fclose(f); return 2; }
    m->pos = (float*)malloc((size_t)m->nv * 12); m->nrm = (float*)malloc((size_t)m->nv * 12); m->idx = (uint32_t*)malloc((size_t)m->nf * 12);
    size_t ok = fread(m->pos, 12, m->nv, f) + fread(m->nrm, 12, m->nv, f) + fread(m->idx, 12, m->nf, f);
    fclose(f);
    if (ok != (size_t)m->nv * 2 + m->nf) return 3;
    /* aiMatrix4x4 row-major: RotationX(a): b2 = c3 = cos a, c2 = sin a, b3 = -sin a */
    float a = -3.14159265358979323846f / 2, rx[4][4] = {{1, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 1}};
    rx[1][1] = rx[2][2] = h_cos(a);
    rx[2][1] = h_sin(a);
    rx[1][2] = -rx[2][1];
    /* two products with identity node transforms, assimp's operator*= order */
    for (int rep = 0; rep < 2; rep++) {
        float o[4][4];
        for (int r = 0; r < 4; r++) for (int c = 0; c < 4; c++) {
            float i0 = (0 == c), i1 = (1 == c), i2 = (2 == c), i3 = (3 == c);
            o[r][c] = ((i0 * rx[r][0] + i1 * rx[r][1]) + i2 * rx[r][2]) + i3 * rx[r][3];
        }
        memcpy(rx, o, sizeof o);
    }
    for (int c = 0; c < 4; c++) for (int r = 0; r < 4; r++) m->node.m[c][r] = rx[r][c];
    return 0;
}

/* Scene::AddLoadedScene (Scene.cpp:75-132) */
static void add_loaded(OScene* s, const OMesh* mesh, M4 transform, int mat) {
    M4 mt = m_mul(transform, mesh->node);
    uint32_t off = (uint32_t)s->nverts;
    for (uint32_t v = 0; v < mesh->nv; v++) {
        float p[4] = {mesh->pos[3 * v], mesh->pos[3 * v + 1], mesh->pos[3 * v + 2], 1.0f}, n[4] = {mesh->nrm[3 * v], mesh->nrm[3 * v + 1], mesh->nrm[3 * v + 2], 0.0f}, po[4], no[4];
        m_vec(&mt, p, po);
        m_vec(&mt, n, no);
        push_vert(s, V(po[0], po[1], po[2]), V(no[0], no[1], no[2]));
    }
    for (uint32_t f = 0; f < mesh->nf; f++) {
        const uint32_t* id = &mesh->idx[3 * f];
        push_face(s, id[0] + off, id[1] + off, id[2] + off, (uint32_t)mat);
        v3 q[3];
        for (int k = 0; k < 3; k++) {
            float p[4] = {mesh->pos[3 * id[k]], mesh->pos[3 * id[k] + 1], mesh->pos[3 * id[k] + 2], 1.0f}, po[4];
            m_vec(&mt, p, po);
            q[k] = V(po[0], po[1], po[2]);
        }
        add_triangle(s, q[0], q[1], q[2], mat);
    }
}

/* CUDARayTracer::SetupCornellBox (RayTracing/RayTracing.cpp:79-203) */
static void setup_cornell(OScene* s) {
    v3 g = V(0.7f, 0.7f, 0.7f), z = V(0, 0, 0), w9 = V(0.9f, 0.9f, 0.9f), green = V(0.3f, 1.0f, 0.3f);
    int m;
    m = add_plain_material(s, g, z); add_quad(s, V(-12.6f, -12.6f, 25.0f), V(12.6f, -12.6f, 25.0f), V(12.6f, 12.6f, 25.0f), V(-12.6f, 12.6f, 25.0f), m);
    m = add_plain_material(s, g, z); add_quad(s, V(-12.6f, -12.45f, 25.0f), V(12.6f, -12.45f, 25.0f), V(12.6f, -12.45f, 15.0f), V(-12.6f, -12.45f, 15.0f), m);
    m = add_plain_material(s, g, z); add_quad(s, V(-12.6f, 12.5f, 25.0f), V(12.6f, 12.5f, 25.0f), V(12.6f, 12.5f, 15.0f), V(-12.6f, 12.5f, 15.0f), m);
    m = add_plain_material(s, V(0.1f, 0.7f, 0.1f), z); add_quad(s, V(-12.5f, -12.6f, 25.0f), V(-12.5f, -12.6f, 15.0f), V(-12.5f, 12.6f, 15.0f), V(-12.5f, 12.6f, 25.0f), m);
    m = add_plain_material(s, V(0.7f, 0.1f, 0.1f), z); add_quad(s, V(12.5f, -12.6f, 25.0f), V(12.5f, -12.6f, 15.0f), V(12.5f, 12.6f, 15.0f), V(12.5f, 12.6f, 25.0f), m);
    m = add_plain_material(s, z, vscale(V(1.0f, 0.9f, 0.7f), 20.0f)); add_quad(s, V(-5.0f, 12.4f, 22.5f), V(5.0f, 12.4f, 22.5f), V(5.0f, 12.4f, 17.5f), V(-5.0f, 12.4f, 17.5f), m);
    add_sphere(s, V(-9.0f, -9.5f, 20.0f), 3, add_material(s, V(0.9f, 0.9f, 0.50f), z, 0.5f, w9, 0.2f));
    add_sphere(s, V(0.0f, -9.5f, 20.0f), 3, add_material(s, V(0.9f, 0.5f, 0.90f), z, 0.3f, w9, 0.2f));
    add_sphere(s, V(9.0f, -9.5f, 20.0f), 3, add_material(s, V(0.0f, 0.0f, 1.0f), z, 0.5f, V(1.0f, 0.0f, 0.0f), 0.4f));
    s->cam_ay = 180.0f;
    add_sphere(s, V(-10.0f, 0.0f, 23.0f), 1.75f, add_material(s, V(1, 1, 1), z, 1.0f, green, 0.0f));
    add_sphere(s, V(-5.0f, 0.0f, 23.0f), 1.75f, add_material(s, V(1, 1, 1), z, 1.0f, green, 0.25f));
    add_sphere(s, V(0.0f, 0.0f, 23.0f), 1.75f, add_material(s, V(1, 1, 1), z, 1.0f, green, 0.5f));
    add_sphere(s, V(5.0f, 0.0f, 23.0f), 1.75f, add_material(s, V(1, 1, 1), z, 1.0f, green, 0.75f));
    add_sphere(s, V(10.0f, 0.0f, 23.0f), 1.75f, add_material(s, V(1, 1, 1), z, 1.0f, green, 0.97f));
}

/* RayTracing.cpp:42-46 */
static M4 bunny_xform(v3 t) {
    M4 m = m_translate(m_ident(), t);
    m = m_rotate(m, -3.14159265358979323846f, V(0, 1, 0));
    m = m_rotate(m, 3.14159265358979323846f / 2, V(1, 0, 0));
    return m_scale(m, V(150.0f, 150.0f, 150.0f));
}

/* RayTracing.cpp:52-68 */
static void bunny_floor_light(OScene* s) {
    v3 off = V(20, 0, 0), sc = V(50, 1, 50);
    v3 A = vadd(vmul(sc, V(-1.0f, -12.45f, 1.0f)), off), B = vadd(vmul(sc, V(1.0f, -12.45f, 1.0f)), off);
    v3 C = vadd(vmul(sc, V(1.0f, -12.45f, -1.0f)), off), D = vadd(vmul(sc, V(-1.0f, -12.45f, -1.0f)), off);
    add_quad(s, A, B, C, D, add_plain_material(s, V(0.7f, 0.7f, 0.7f), V(0, 0, 0)));
    add_sphere(s, V(30, 10, 40), 8, add_plain_material(s, V(0, 0, 0), vscale(V(0.3f, 0.9f, 0.7f), 10.0f)));
}

/* ------------------------------------------------------------------------------------ */
/* BVH (RayTracing/BVH.cpp:8-124)                                                         */
/* ------------------------------------------------------------------------------------ */
typedef struct { float c[3]; uint32_t index; } OTri;
typedef struct { OScene* s; OTri* tris; size_t used; } OBuild;

static void bvh_bounds(OBuild* b, uint32_t ni) {  /* BVH.cpp:45-57 */
    ONode* n = &b->s->nodes[ni];
    for (int k = 0; k < 3; k++) { n->bmin[k] = 1e30f; n->bmax[k] = -1e30f; }
    for (uint32_t i = 0; i < n->count; i++) {
        const OFace* f = &b->s->faces[b->tris[n->first + i].index];
        uint32_t vs[3] = {f->v0, f->v1, f->v2};
        for (int q = 0; q < 3; q++) for (int k = 0; k < 3; k++) {
            float p = b->s->verts[vs[q]].p[k];
            n->bmin[k] = gmin(n->bmin[k], p);
            n->bmax[k] = gmax(n->bmax[k], p);
        }
    }
}

static void bvh_subdivide(OBuild* b, uint32_t ni, int depth) {  /* BVH.cpp:59-124 */
    if (depth > b->s->max_depth) b->s->max_depth = depth;
    ONode* n = &b->s->nodes[ni];
    float ext[3] = {n->bmax[0] - n->bmin[0], n->bmax[1] - n->bmin[1], n->bmax[2] - n->bmin[2]};
    int a1 = 0;
    if (ext[1] > ext[0]) a1 = 1;
    if (ext[2] > ext[a1]) a1 = 2;
    int a2 = (a1 + 1) % 3, a3 = (a2 + 1) % 3;
    if (ext[a3] > ext[a2]) { int t = a2; a2 = a3; a3 = t; }
    int axes[3] = {a1, a2, a3}, found = 0, i = 0, left = 0;
    for (int q = 0; q < 3; q++) {
        int axis = axes[q];
        float split = n->bmin[axis] + ext[axis] * 0.5f;
        i = (int)n->first;
        int j = i + (int)n->count - 1;
        while (i <= j) {
            if (b->tris[i].c[axis] < split) i++;
            else { OTri t = b->tris[i]; b->tris[i] = b->tris[j]; b->tris[j] = t; j--; }
        }
        left = i - (int)n->first;
        if (left != 0 && left != (int)n->count) { found = 1; break; }
    }
    if (!found) return;
    uint32_t L = (uint32_t)b->used++, R = (uint32_t)b->used++;
    ONode* nodes = b->s->nodes;
    nodes[L].first = n->first;
    n->first = L;
    nodes[L].count = (uint32_t)left;
    nodes[R].first = (uint32_t)i;
    nodes[R].count = n->count - (uint32_t)left;
    n->count = 0;
    bvh_bounds(b, L);
    bvh_bounds(b, R);
    bvh_subdivide(b, L, depth + 1);
    bvh_subdivide(b, R, depth + 1);
}

static void bvh_build(OScene* s) {  /* BVH.cpp:8-43 */
    size_t nf = s->nfaces;
    s->nodes = (ONode*)calloc(nf * 2, sizeof(ONode));
    OBuild b = {s, (OTri*)malloc(nf * sizeof(OTri)), 1};
    for (size_t i = 0; i < nf; i++) {
        const OVertex *p0 = &s->verts[s->faces[i].v0], *p1 = &s->verts[s->faces[i].v1], *p2 = &s->verts[s->faces[i].v2];
        for (int k = 0; k < 3; k++) b.tris[i].c[k] = ((p0->p[k] + p1->p[k]) + p2->p[k]) / 3.0f;
        b.tris[i].index = (uint32_t)i;
    }
    s->nodes[0].first = 0;
    s->nodes[0].count = (uint32_t)nf;
    s->max_depth = 0;
    bvh_bounds(&b, 0);
    bvh_subdivide(&b, 0, 0);
    s->nnodes = b.used;
    s->face_idx = (uint32_t*)malloc(nf * sizeof(uint32_t));
    for (size_t i = 0; i < nf; i++) s->face_idx[i] = b.tris[i].index;
    free(b.tris);
}

static int load_sky(OScene* s, const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) return 1;
    char magic[8];
    uint32_t n;
    if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "RTCUBE01", 8) || fread(&n, 4, 1, f) != 1) { fclose(f); return 2; }
    s->sky = (float*)malloc((size_t)6 * n * n * 16);
    size_t got = fread(s->sky, 16, (size_t)6 * n * n, f);
    fclose(f);
    s->sky_n = (int)n;
    return got == (size_t)6 * n * n ? 0 : 3;
}

/* which: 0 Cornell + bunny (RayTracing.cpp:24-25), 1 four bunnies, 2 plane grid of n x n quads */
OScene* oracle_scene_create(int which, const char* assets, int grid_n) {
    OScene* s = (OScene*)calloc(1, sizeof(OScene));
    char path[4096];
    if (which == 2) {
        int m = add_plain_material(s, V(0.7f, 0.7f, 0.7f), V(0.2f, 0.2f, 0.2f));
        float* xs = (float*)malloc((grid_n + 1) * sizeof(float));
        float* ys = (float*)malloc((grid_n + 1) * sizeof(float));
        for (int i = 0; i <= grid_n; i++) { xs[i] = -60.0f + 120.0f * (float)i / (float)grid_n; ys[i] = -34.0f + 68.0f * (float)i / (float)grid_n; }
        for (int j = 0; j < grid_n; j++) for (int i = 0; i < grid_n; i++)
            add_quad(s, V(xs[i], ys[j], 30.0f), V(xs[i + 1], ys[j], 30.0f), V(xs[i + 1], ys[j + 1], 30.0f), V(xs[i], ys[j + 1], 30.0f), m);
        free(xs); free(ys);
        s->cam_ay = 180.0f;
    } else {
        OMesh mesh;
        snprintf(path, sizeof path, "%s/bunny_mesh.bin", assets);
        if (load_mesh(path, &mesh)) { free(s); return NULL; }
        setup_cornell(s);
        int m = add_material(s, V(1, 1, 1), V(0, 0, 0), 0.5f, V(0.3f, 1.0f, 0.3f), 0.8f);
        if (which == 0) {
            add_loaded(s, &mesh, bunny_xform(V(30, -18, 20)), m);
        } else {
            v3 t[4] = {V(17, -18, 7), V(43, -18, 7), V(17, -18, 33), V(43, -18, 33)};
            for (int k = 0; k < 4; k++) add_loaded(s, &mesh, bunny_xform(t[k]), m);
        }
        bunny_floor_light(s);
        free(mesh.pos); free(mesh.nrm); free(mesh.idx);
    }
    snprintf(path, sizeof path, "%s/sunset_cube128.bin", assets);
    if (load_sky(s, path)) { free(s); return NULL; }
    bvh_build(s);
    return s;
}

void oracle_scene_destroy(OScene* s) {
    if (!s) return;
    free(s->verts); free(s->faces); free(s->nodes); free(s->face_idx); free(s->sky); free(s);
}

/* host views for tests */
void oracle_scene_arrays(const OScene* s, const void** verts, size_t* nv, const void** faces, size_t* nf,
                         const void** nodes, size_t* nn, const uint32_t** face_idx, int* max_depth,
                         const void** spheres, int* ns, const void** mats, int* nm) {
    *verts = s->verts; *nv = s->nverts; *faces = s->faces; *nf = s->nfaces; *nodes = s->nodes; *nn = s->nnodes;
    *face_idx = s->face_idx; *max_depth = s->max_depth; *spheres = s->spheres; *ns = s->nspheres; *mats = s->mats; *nm = s->nmats;
}
void oracle_camera(const OScene* s, int w, int h, float out[15]) { o_camera(s, w, h, (OCamera*)out); }
void oracle_set_camera(OScene* s, const float pos[3], float ax, float ay) { memcpy(s->cam_pos, pos, 12); s->cam_ax = ax; s->cam_ay = ay; }

/* ------------------------------------------------------------------------------------ */
/* XORWOW / curand_init (RayTracing/Random.cu:3-8; curand_kernel.h restated)              */
/* ------------------------------------------------------------------------------------ */
typedef struct { uint32_t d, v[5]; } ORng;

static uint32_t rng_next(ORng* r) {  /* curand(): xorwow step + Weyl */
    uint32_t t = r->v[0] ^ (r->v[0] >> 2);
    r->v[0] = r->v[1]; r->v[1] = r->v[2]; r->v[2] = r->v[3]; r->v[3] = r->v[4];
    r->v[4] = (r->v[4] ^ (r->v[4] << 4)) ^ (t ^ (t << 1));
    r->d += 362437u;
    return r->v[4] + r->d;
}
static float rng_uniform(ORng* r) { return (float)rng_next(r) * 0x1p-32f + 0x1p-33f; } /* curand_uniform */

/* Jump tables: J[k][d-1] = A^(d * 4^k * 2^67), d = 1..3, each stored as 20 byte-indexed
 * tables of 256 x 5 words (byte b of the 160-bit state -> contribution). */
#define OJ 32
static uint32_t (*g_jt)[3][20][256][5];
static uint32_t g_mat[OJ][160][5]; /* A^(4^k 2^67) as rows: input bit -> 5 output words */

static void mat_apply(uint32_t m[160][5], const uint32_t in[5], uint32_t out[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int b = 0; b < 160; b++)
        if ((in[b >> 5] >> (b & 31)) & 1u) for (int w = 0; w < 5; w++) r[w] ^= m[b][w];
    memcpy(out, r, sizeof r);
}
static void mat_mul(uint32_t a[160][5], uint32_t b[160][5], uint32_t out[160][5]) { /* out = b o a */
    uint32_t t[160][5];
    for (int i = 0; i < 160; i++) mat_apply(b, a[i], t[i]);
    memcpy(out, t, sizeof t);
}

static void jump_init(void) {
    if (g_jt) return;
#pragma omp critical(oracle_jump_init)
    if (!g_jt) {
        static uint32_t m[160][5];
        for (int b = 0; b < 160; b++) {
            ORng r = {0, {0, 0, 0, 0, 0}};
            r.v[b >> 5] = 1u << (b & 31);
            rng_next(&r);
            memcpy(m[b], r.v, 20);
        }
        for (int s = 0; s < 67; s++) mat_mul(m, m, m);
        uint32_t (*jt)[3][20][256][5] = malloc(sizeof(*jt) * OJ);
        for (int k = 0; k < OJ; k++) {
            if (k) { mat_mul(m, m, m); mat_mul(m, m, m); }
            memcpy(g_mat[k], m, sizeof m);
            static uint32_t pw[3][160][5];
            memcpy(pw[0], m, sizeof m);
            mat_mul(pw[0], m, pw[1]);
            mat_mul(pw[1], m, pw[2]);
            for (int d = 0; d < 3; d++)
                for (int byte = 0; byte < 20; byte++)
                    for (int val = 0; val < 256; val++) {
                        uint32_t acc[5] = {0, 0, 0, 0, 0};
                        for (int bit = 0; bit < 8; bit++)
                            if ((val >> bit) & 1) for (int w = 0; w < 5; w++) acc[w] ^= pw[d][byte * 8 + bit][w];
                        memcpy(jt[k][d][byte][val], acc, 20);
                    }
        }
        g_jt = jt;
    }
}

/* curand_init(seed (32-bit, widened), subsequence, 0) */
static void rng_init(uint32_t seed, uint64_t sub, ORng* r) {
    uint32_t s0 = seed ^ 0xaad26b49u, s1 = 0u ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0, t1 = 2591861531u * s1;
    r->d = 6615241u + t1 + t0;
    r->v[0] = 123456789u + t0; r->v[1] = 362436069u ^ t0; r->v[2] = 521288629u + t1;
    r->v[3] = 88675123u ^ t1; r->v[4] = 5783321u + t0;
    jump_init();
    for (int k = 0; sub && k < OJ; k++, sub >>= 2) {
        int d = (int)(sub & 3);
        if (!d) continue;
        uint32_t acc[5] = {0, 0, 0, 0, 0};
        const uint8_t* bytes = (const uint8_t*)r->v;
        for (int byte = 0; byte < 20; byte++) {
            const uint32_t* e = g_jt[k][d - 1][byte][bytes[byte]];
            for (int w = 0; w < 5; w++) acc[w] ^= e[w];
        }
        memcpy(r->v, acc, 20);
    }
}

void oracle_rng_init(uint32_t seed, uint64_t subsequence, uint32_t out[6]) {
    ORng r;
    rng_init(seed, subsequence, &r);
    out[0] = r.d;
    memcpy(out + 1, r.v, 20);
}
/* per-pixel states of a whole frame (6 words each, y*width + x), OpenMP-parallel */
void oracle_rng_init_frame(uint32_t seed, int width, int height, uint32_t* out, int threads) {
    jump_init();
    long n = (long)width * height;
#ifdef _OPENMP
    int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nt)
#endif
    for (long i = 0; i < n; i++) {
        ORng r;
        rng_init(seed, (uint64_t)i, &r);
        out[6 * i] = r.d;
        memcpy(out + 6 * i + 1, r.v, 20);
    }
}
void oracle_rng_draws(const uint32_t state[6], int n, float* out) {
    ORng r = {state[0], {state[1], state[2], state[3], state[4], state[5]}};
    for (int i = 0; i < n; i++) out[i] = rng_uniform(&r);
}
/* matrix A^(4^k 2^67) in rocrand's layout m[i*160 + j*5 + w] */
int oracle_jump_matrix(int k, uint32_t out[800]) {
    if (k < 0 || k >= OJ) return 1;
    jump_init();
    for (int b = 0; b < 160; b++) memcpy(out + b * 5, g_mat[k][b], 20);
    return 0;
}
float oracle_sin(float x) { return o_sin(x); }
float oracle_cos(float x) { return o_cos(x); }

/* ------------------------------------------------------------------------------------ */
/* sky lookup (DESIGN.md "cube sampler"; stands in for texCubemapLod, main_raytracing.cu:152) */
/* ------------------------------------------------------------------------------------ */
static void cube_coords(float x, float y, float z, int* face, float* s, float* t) {
    float ax = fabsf(x), ay = fabsf(y), az = fabsf(z), ma, sc, tc;
    if (ax >= ay && ax >= az) { ma = ax; *face = x >= 0.0f ? 0 : 1; sc = x >= 0.0f ? -z : z; tc = -y; }
    else if (ay >= az) { ma = ay; *face = y >= 0.0f ? 2 : 3; sc = x; tc = y >= 0.0f ? z : -z; }
    else { ma = az; *face = z >= 0.0f ? 4 : 5; sc = z >= 0.0f ? x : -x; tc = -y; }
    *s = (sc / ma + 1.0f) * 0.5f;
    *t = (tc / ma + 1.0f) * 0.5f;
}
static const float* cube_texel(const float* tex, int n, int face, int i, int j) {
    if (i >= 0 && i < n && j >= 0 && j < n) return tex + 4 * ((size_t)(face * n + j) * n + i);
    float sc = (float)(2 * i + 1) / (float)n - 1.0f, tc = (float)(2 * j + 1) / (float)n - 1.0f, x, y, z;
    switch (face) {
        case 0: x = 1.0f; y = -tc; z = -sc; break;
        case 1: x = -1.0f; y = -tc; z = sc; break;
        case 2: x = sc; y = 1.0f; z = tc; break;
        case 3: x = sc; y = -1.0f; z = -tc; break;
        case 4: x = sc; y = -tc; z = 1.0f; break;
        default: x = -sc; y = -tc; z = -1.0f; break;
    }
    int f2; float s2, t2;
    cube_coords(x, y, z, &f2, &s2, &t2);
    int i2 = (int)floorf(s2 * (float)n), j2 = (int)floorf(t2 * (float)n);
    if (i2 < 0) i2 = 0; if (i2 > n - 1) i2 = n - 1;
    if (j2 < 0) j2 = 0; if (j2 > n - 1) j2 = n - 1;
    return tex + 4 * ((size_t)(f2 * n + j2) * n + i2);
}
static v3 cube_sample(const float* tex, int n, v3 d) {
    int face; float s, t;
    cube_coords(d.x, d.y, d.z, &face, &s, &t);
    float u = s * (float)n - 0.5f, v = t * (float)n - 0.5f, fu = floorf(u), fv = floorf(v);
    int i0 = (int)fu, j0 = (int)fv;
    float a = rintf((u - fu) * 256.0f) * 0.00390625f, b = rintf((v - fv) * 256.0f) * 0.00390625f;
    float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    const float *t00 = cube_texel(tex, n, face, i0, j0), *t10 = cube_texel(tex, n, face, i0 + 1, j0);
    const float *t01 = cube_texel(tex, n, face, i0, j0 + 1), *t11 = cube_texel(tex, n, face, i0 + 1, j0 + 1);
    float o[3];
    for (int c = 0; c < 3; c++) o[c] = ((w00 * t00[c] + w10 * t10[c]) + w01 * t01[c]) + w11 * t11[c];
    return V(o[0], o[1], o[2]);
}

/* ------------------------------------------------------------------------------------ */
/* renderer (RayTracing/main_raytracing.cu:33-200)                                        */
/* ------------------------------------------------------------------------------------ */
typedef struct { uint64_t seg, nodes, tris, tacc, sacc, hits, misses, pad; } OStats;

/* Math.h:50-61 with CUDA_MIN/MAX = fminf/fmaxf (CUDAHelper.h:31-32, __NVCC__ branch) */
static int aabb_hit(v3 o, v3 d, const ONode* n, float len) {
    float tx1 = (n->bmin[0] - o.x) / d.x, tx2 = (n->bmax[0] - o.x) / d.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    float ty1 = (n->bmin[1] - o.y) / d.y, ty2 = (n->bmax[1] - o.y) / d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2)); tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (n->bmin[2] - o.z) / d.z, tz2 = (n->bmax[2] - o.z) / d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2)); tmax = fminf(tmax, fmaxf(tz1, tz2));
    return tmax >= tmin && tmin < len && tmax > 0;
}

/* glm::intersectRayTriangle (gtx/intersect.inl:29-94) */
static int tri_hit(v3 o, v3 d, v3 a, v3 b, v3 c, float* bx, float* by, float* dist) {
    const float eps = 1.1920928955078125e-07f;
    v3 e1 = vsub(b, a), e2 = vsub(c, a), p = vcross(d, e2), q;
    float det = vdot(e1, p), u, v;
    if (det > eps) {
        v3 t = vsub(o, a);
        u = vdot(t, p);
        if (u < 0.0f || u > det) return 0;
        q = vcross(t, e1);
        v = vdot(d, q);
        if (v < 0.0f || u + v > det) return 0;
    } else if (det < -eps) {
        v3 t = vsub(o, a);
        u = vdot(t, p);
        if (u > 0.0f || u < det) return 0;
        q = vcross(t, e1);
        v = vdot(d, q);
        if (v > 0.0f || u + v < det) return 0;
    } else return 0;
    float inv = 1.0f / det;
    *dist = vdot(e2, q) * inv;
    *bx = u * inv;
    *by = v * inv;
    return 1;
}

/* glm::intersectRaySphere (gtx/intersect.inl:135-153) */
static int sphere_hit(v3 o, v3 d, v3 c, float r2, float* dist) {
    const float eps = 1.1920928955078125e-07f;
    v3 diff = vsub(c, o);
    float t0 = vdot(diff, d), d2 = vdot(diff, diff) - t0 * t0;
    if (d2 > r2) return 0;
    float t1 = sqrtf(r2 - d2);
    *dist = t0 > t1 + eps ? t0 - t1 : t0 + t1;
    return *dist > eps;
}

/* quat * vec3 (type_quat.inl:343-350), q = (w, x, y, z) */
static v3 q_rotate(const float* q, v3 v) {
    v3 qv = V(q[1], q[2], q[3]), uv = vcross(qv, v), uuv = vcross(qv, uv);
    return vadd(v, vscale(vadd(vscale(uv, q[0]), uuv), 2.0f));
}

/* glm::clamp(c, vec3(0), vec3(50)) (main_raytracing.cu:153; func_common.inl clamp = min(max)) */
static v3 vclamp050(v3 c) {
    return V(gmin(gmax(c.x, 0.0f), 50.0f), gmin(gmax(c.y, 0.0f), 50.0f), gmin(gmax(c.z, 0.0f), 50.0f));
}

typedef struct {
    int hit; float dist; v3 pos, nrm; const OMaterial* mat;
} OHit;

/* GetRayHit + BVHRayHit (main_raytracing.cu:33-109), attributes recomputed on every accept
 * exactly as the reference does */
static int get_ray_hit(const OScene* s, v3 ro, v3 rd, OHit* h, OStats* st) {
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
            st->sacc++;
        }
    }
    uint32_t stack[64];
    int top = 0;
    stack[top++] = 0;
    while (top) {
        const ONode* n = &s->nodes[stack[--top]];
        st->nodes++;
        if (!aabb_hit(ro, rd, n, h->dist)) continue;
        if (n->count > 0) {
            for (uint32_t i = 0; i < n->count; i++) {
                const OFace* f = &s->faces[s->face_idx[n->first + i]];
                const OVertex *v0 = &s->verts[f->v0], *v1 = &s->verts[f->v1], *v2 = &s->verts[f->v2];
                float bx, by, dist;
                st->tris++;
                if (tri_hit(ro, nd, V(v0->p[0], v0->p[1], v0->p[2]), V(v1->p[0], v1->p[1], v1->p[2]), V(v2->p[0], v2->p[1], v2->p[2]), &bx, &by, &dist)) {
                    if (dist >= h->dist || dist < 0.0f) continue;
                    float bz = (1.0f - bx) - by;
                    h->dist = dist;
                    h->pos = vadd(ro, vscale(nd, dist));
                    h->nrm = vnorm(vadd(vadd(vscale(V(v0->n[0], v0->n[1], v0->n[2]), bx), vscale(V(v1->n[0], v1->n[1], v1->n[2]), by)), vscale(V(v2->n[0], v2->n[1], v2->n[2]), bz)));
                    h->mat = &s->mats[f->mat];
                    if (vdot(nd, h->nrm) >= 0.0f) h->nrm = V(-h->nrm.x, -h->nrm.y, -h->nrm.z);
                    st->tacc++;
                }
            }
        } else {
            stack[top++] = n->first;
            stack[top++] = n->first + 1;
        }
    }
    return h->dist < 1e30f;
}

/* ray_color (main_raytracing.cu:111-160) */
static v3 ray_color(const OScene* s, v3 ro, v3 rd, ORng* rng, int bounces, float q[4], OStats* st) {
    v3 color = V(0, 0, 0), thr = V(1, 1, 1);
    for (int b = 0; b < bounces; b++) {
        OHit h;
        st->seg++;
        if (get_ray_hit(s, ro, rd, &h, st)) {
            st->hits++;
            const OMaterial* m = h.mat;
            float ds = (rng_uniform(rng) < m->spec_pct) ? 1.0f : 0.0f;
            color = vadd(color, vmul(thr, V(m->emissive[0], m->emissive[1], m->emissive[2])));
            float om = 1.0f - ds;
            thr = vmul(thr, V(m->albedo[0] * om + m->specular[0] * ds, m->albedo[1] * om + m->specular[1] * ds, m->albedo[2] * om + m->specular[2] * ds));
            /* GetRandomPointOnSphere (Random.h:23-46) */
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
        } else {
            st->misses++;
            if (s->sky) {
                v3 c = vclamp050(cube_sample(s->sky, s->sky_n, q_rotate(q, rd)));
                color = vadd(color, vmul(thr, c));
            }
            break;
        }
    }
    return color;
}

/*
 * Render rows [row_begin, row_end) of a width x height frame into out (float4 per pixel,
 * row-major, width pixels per row, row 0 = row_begin).  rng: if non-NULL, per-pixel states
 * (6 words each, y*width + x of the FULL frame) read and written back; else states are
 * seeded with curand_init(seed, y*width + x, 0).  last: float4 history in out's layout, or
 * NULL (zeros).  threads <= 0: OpenMP default.  stats: OStats (8 uint64) or NULL.
 */
static int render_rows(const OScene* s, int width, int height, int spp, int bounces, int frame_index, uint32_t seed,
                       uint32_t* rng, const float* last, float* out, int row_begin, int row_end, int threads,
                       uint64_t* stats, uint32_t* costs) {
    if (!s || width <= 0 || height <= 0 || row_begin < 0 || row_end > height || row_begin > row_end) return 1;
    OCamera cam;
    o_camera(s, width, height, &cam);
    /* quat(vec3(0, PI, 0)), PI = 3.1415926536f (main_raytracing.cu:7,151), RT sin/cos */
    float ey = 3.1415926536f * 0.5f, e0 = 0.0f * 0.5f;
    float cx = o_cos(e0), cy = o_cos(ey), cz = o_cos(e0), sx = o_sin(e0), sy = o_sin(ey), sz = o_sin(e0);
    float q[4] = {cx * cy * cz + sx * sy * sz, sx * cy * cz - cx * sy * sz, cx * sy * cz + sx * cy * sz, cx * cy * sz - sx * sy * cz};
    v3 co = V(cam.origin[0], cam.origin[1], cam.origin[2]), ch = V(cam.horizontal[0], cam.horizontal[1], cam.horizontal[2]);
    v3 cv = V(cam.vertical[0], cam.vertical[1], cam.vertical[2]), cl = V(cam.llc[0], cam.llc[1], cam.llc[2]);
    if (!rng) jump_init();
    OStats total = {0};
#ifdef _OPENMP
    int nt = threads > 0 ? threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
#endif
    for (int y = row_begin; y < row_end; y++) {
        OStats st = {0};
        for (int x = 0; x < width; x++) {
            size_t pid = (size_t)y * width + x;
            ORng r;
            if (rng) { r.d = rng[6 * pid]; memcpy(r.v, rng + 6 * pid + 1, 20); }
            else rng_init(seed, pid, &r);
            float acc[4] = {0, 0, 0, 0};
            const OStats st0 = st;
            for (int smp = 0; smp < spp; smp++) {
                float ru = rng_uniform(&r), rv = rng_uniform(&r);
                float ux = ((float)x + ru) / (float)width, uy = ((float)y + rv) / (float)height;
                v3 rd = vsub(vadd(vadd(cl, vscale(ch, ux)), vscale(cv, uy)), co);
                v3 c = ray_color(s, co, rd, &r, bounces, q, &st);
                acc[0] += c.x; acc[1] += c.y; acc[2] += c.z; acc[3] += 1.0f;
            }
            float fs = (float)spp, res[4] = {acc[0] / fs, acc[1] / fs, acc[2] / fs, acc[3] / fs};
            float l = frame_index > 0 ? 1.0f / (float)(frame_index + 1) : 1.0f, om = 1.0f - l;
            size_t o = ((size_t)(y - row_begin) * width + x) * 4;
            for (int c = 0; c < 4; c++) {
                float prev = last ? last[o + c] : 0.0f;
                out[o + c] = prev * om + res[c] * l;
            }
            out[o + 3] = 1.0f;
            if (rng) { rng[6 * pid] = r.d; memcpy(rng + 6 * pid + 1, r.v, 20); }
            if (costs) {
                uint32_t* c = costs + 3 * ((size_t)(y - row_begin) * width + x);
                c[0] = (uint32_t)(st.seg - st0.seg), c[1] = (uint32_t)(st.nodes - st0.nodes), c[2] = (uint32_t)(st.tris - st0.tris);
            }
        }
#ifdef _OPENMP
#pragma omp critical(oracle_stats)
#endif
        {
            total.seg += st.seg; total.nodes += st.nodes; total.tris += st.tris; total.tacc += st.tacc;
            total.sacc += st.sacc; total.hits += st.hits; total.misses += st.misses;
        }
    }
    if (stats) memcpy(stats, &total, sizeof total);
    return 0;
}
int oracle_render(const OScene* s, int width, int height, int spp, int bounces, int frame_index, uint32_t seed,
                  uint32_t* rng, const float* last, float* out, int row_begin, int row_end, int threads,
                  uint64_t* stats) {
    return render_rows(s, width, height, spp, bounces, frame_index, seed, rng, last, out, row_begin, row_end, threads,
                       stats, NULL);
}
/* oracle_render plus per-pixel work: costs[3 * pixel] = (segments, node visits, triangle tests) */
int oracle_render_costs(const OScene* s, int width, int height, int spp, int bounces, int frame_index, uint32_t seed,
                        uint32_t* rng, const float* last, float* out, int row_begin, int row_end, int threads,
                        uint64_t* stats, uint32_t* costs) {
    return render_rows(s, width, height, spp, bounces, frame_index, seed, rng, last, out, row_begin, row_end, threads,
                       stats, costs);
}

/*
 * One camera sample of pixel (x, y) started at every even RNG offset: the reference's sample
 * body (main_raytracing.cu:188-193: u, v, GetRay, ray_color) run from `state` advanced by
 * o = 2i draws, i < n.  A sample draws 2 + 4 * (hits) numbers, so o_{j+1} = o_j + draws(o_j)
 * from o_0 = 0 is the pixel's real sample chain and the table answers "what would sample j
 * return if it started at o" for every o.  out[8 * i] = color r, g, b, draws consumed,
 * segments, node visits, triangle tests, 0 (floats; counts exact below 2^24).
 */
int oracle_sample_table(const OScene* s, int width, int height, int x, int y, int bounces, const uint32_t state[6],
                        int n, float* out) {
    if (!s || width <= 0 || height <= 0 || n < 0) return 1;
    OCamera cam;
    o_camera(s, width, height, &cam);
    float ey = 3.1415926536f * 0.5f, e0 = 0.0f * 0.5f;
    float cx = o_cos(e0), cy = o_cos(ey), cz = o_cos(e0), sx = o_sin(e0), sy = o_sin(ey), sz = o_sin(e0);
    float q[4] = {cx * cy * cz + sx * sy * sz, sx * cy * cz - cx * sy * sz, cx * sy * cz + sx * cy * sz, cx * cy * sz - sx * sy * cz};
    v3 co = V(cam.origin[0], cam.origin[1], cam.origin[2]), ch = V(cam.horizontal[0], cam.horizontal[1], cam.horizontal[2]);
    v3 cv = V(cam.vertical[0], cam.vertical[1], cam.vertical[2]), cl = V(cam.llc[0], cam.llc[1], cam.llc[2]);
    ORng base = {state[0], {state[1], state[2], state[3], state[4], state[5]}};
    for (int i = 0; i < n; i++) {
        ORng r = base;
        uint32_t d0 = r.d;
        OStats st = {0};
        float ru = rng_uniform(&r), rv = rng_uniform(&r);
        float ux = ((float)x + ru) / (float)width, uy = ((float)y + rv) / (float)height;
        v3 rd = vsub(vadd(vadd(cl, vscale(ch, ux)), vscale(cv, uy)), co);
        v3 c = ray_color(s, co, rd, &r, bounces, q, &st);
        float* o = out + 8 * (size_t)i;
        o[0] = c.x; o[1] = c.y; o[2] = c.z;
        o[3] = (float)((r.d - d0) / 362437u);
        o[4] = (float)st.seg; o[5] = (float)st.nodes; o[6] = (float)st.tris; o[7] = 0.0f;
        rng_next(&base);
        rng_next(&base);
    }
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* The glm pieces of the restatement, exported so tests/test_oracle_glm.py can pin them     */
/* bit for bit against the reference's own vendored glm (oracle/ref_glm.cpp, built from   */
/* /root/reference/include/glm by oracle/build_ref.sh).  Same signatures as ref_glm.cpp.  */
/* ------------------------------------------------------------------------------------ */
static v3 ldv(const float* p) { return V(p[0], p[1], p[2]); }
static void stv(float* p, v3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }

void oracle_glm_tri_batch(int64_t n, const float* o, const float* d, const float* v0, const float* v1, const float* v2,
                          int32_t* hit, float* out) {
    for (int64_t i = 0; i < n; i++) {
        float bx = 0.0f, by = 0.0f, t = 0.0f;
        hit[i] = tri_hit(ldv(o + 3 * i), vnorm(ldv(d + 3 * i)), ldv(v0 + 3 * i), ldv(v1 + 3 * i), ldv(v2 + 3 * i), &bx, &by, &t);
        out[3 * i] = bx; out[3 * i + 1] = by; out[3 * i + 2] = t;
    }
}

void oracle_glm_sphere_batch(int64_t n, const float* o, const float* d, const float* c, const float* r, int32_t* hit,
                             float* dist) {
    for (int64_t i = 0; i < n; i++) {
        float t = 0.0f;
        hit[i] = sphere_hit(ldv(o + 3 * i), vnorm(ldv(d + 3 * i)), ldv(c + 3 * i), r[i] * r[i], &t);
        dist[i] = t;
    }
}

void oracle_glm_vec_batch(int64_t n, const float* a, const float* b, const float* s, float* out) {
    for (int64_t i = 0; i < n; i++) {
        v3 x = ldv(a + 3 * i), y = ldv(b + 3 * i);
        float* o = out + 18 * i;
        stv(o, vnorm(x));
        stv(o + 3, vcross(x, y));
        o[6] = vdot(x, y);
        stv(o + 7, vreflect(x, y));
        stv(o + 10, vmix(x, y, s[i]));
        o[13] = gmax(x.x, y.x);
        o[14] = gmin(x.x, y.x);
        stv(o + 15, vclamp050(x));
    }
}

void oracle_glm_quat_rotate_batch(int64_t n, const float* q, const float* v, float* out) {
    for (int64_t i = 0; i < n; i++) stv(out + 3 * i, q_rotate(q + 4 * i, ldv(v + 3 * i)));
}

/* Camera::Update (Scene.cpp:15-36) as o_camera computes it (fov 90) */
int oracle_glm_camera(const float* pos, float ax, float ay, int w, int h, float* out) {
    OScene* s = (OScene*)calloc(1, sizeof(OScene));
    OCamera cam;
    if (!s) return 1;
    memcpy(s->cam_pos, pos, 12);
    s->cam_ax = ax; s->cam_ay = ay;
    o_camera(s, w, h, &cam);
    free(s);
    memcpy(out, cam.origin, 12); memcpy(out + 3, cam.horizontal, 12);
    memcpy(out + 6, cam.vertical, 12); memcpy(out + 9, cam.llc, 12);
    return 0;
}

static M4 m_load(const float* m) { M4 r; for (int c = 0; c < 4; c++) for (int k = 0; k < 4; k++) r.m[c][k] = m[4 * c + k]; return r; }
static void m_store(M4 a, float* m) { for (int c = 0; c < 4; c++) for (int k = 0; k < 4; k++) m[4 * c + k] = a.m[c][k]; }

void oracle_glm_trs(const float* pos, float angle, const float* axis, const float* scl, float* out) {
    M4 m = m_translate(m_ident(), ldv(pos));
    m = m_rotate(m, angle, ldv(axis));
    m_store(m_scale(m, ldv(scl)), out);
}

void oracle_glm_inverse(const float* m, float* out) { m_store(m_inverse(m_load(m)), out); }

void oracle_glm_mat_apply_batch(int64_t n, const float* m1, const float* m2, const float* p, float* out) {
    M4 t = m_mul(m_load(m1), m_load(m2));
    for (int64_t i = 0; i < n; i++) {
        float v1[4] = {p[3 * i], p[3 * i + 1], p[3 * i + 2], 1.0f}, v0[4] = {p[3 * i], p[3 * i + 1], p[3 * i + 2], 0.0f}, o[4];
        m_vec(&t, v1, o); out[6 * i] = o[0]; out[6 * i + 1] = o[1]; out[6 * i + 2] = o[2];
        m_vec(&t, v0, o); out[6 * i + 3] = o[0]; out[6 * i + 4] = o[1]; out[6 * i + 5] = o[2];
    }
}
