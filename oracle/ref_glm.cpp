// ref_glm.cpp -- TEST INFRASTRUCTURE (parity pin, never shipped, never on the product path).
//
// The reference's own vendored glm 0.9.9.8 (/root/reference/include/glm, header-only) compiled
// here with g++ -- no other reference file and no stand-in header -- exporting the glm operations
// the hot path uses, so tests/test_oracle_glm.py can check oracle/rt_oracle.c's C restatement of
// them bit for bit on millions of inputs.  Each function names the reference call site it
// mirrors.  Built by oracle/build_ref.sh into oracle/_ref/libref_glm.so (git-ignored); the
// vectors it produced are also committed (tests/golden/glm_vectors.npz, tools/make_glm_vectors.py)
// so the pin holds where /root/reference is absent.
//
// Floating point: -ffp-contract=off, as the oracle and the product (nvcc's default FMA
// contraction of the reference build is not reproducible here).
#define GLM_ENABLE_EXPERIMENTAL
#include <glm/glm.hpp>
#include <glm/gtc/quaternion.hpp>
#include <glm/gtx/compatibility.hpp>
#include <glm/gtx/intersect.hpp>

#include <cstdint>

using glm::vec2;
using glm::vec3;
using glm::vec4;

static vec3 ld(const float* p) { return vec3(p[0], p[1], p[2]); }
static void st(float* p, vec3 v) { p[0] = v.x, p[1] = v.y, p[2] = v.z; }

extern "C" {

// BVHRayHit's triangle test (main_raytracing.cu:58-60): intersectRayTriangle(origin,
// normalize(direction), v0, v1, v2, bary, distance).  out[i] = (bary.x, bary.y, distance) when hit.
void ref_tri_batch(int64_t n, const float* o, const float* d, const float* v0, const float* v1, const float* v2,
                   int32_t* hit, float* out) {
    for (int64_t i = 0; i < n; i++) {
        const vec3 nd = glm::normalize(ld(d + 3 * i));
        vec2 bary(0.0f);
        float dist = 0.0f;
        hit[i] = glm::intersectRayTriangle(ld(o + 3 * i), nd, ld(v0 + 3 * i), ld(v1 + 3 * i), ld(v2 + 3 * i), bary, dist);
        out[3 * i] = bary.x, out[3 * i + 1] = bary.y, out[3 * i + 2] = dist;
    }
}

// GetRayHit's sphere test (main_raytracing.cu:92): intersectRaySphere(origin, normalize(direction),
// center, radius * radius, distance).
void ref_sphere_batch(int64_t n, const float* o, const float* d, const float* c, const float* r, int32_t* hit,
                      float* dist) {
    for (int64_t i = 0; i < n; i++) {
        const vec3 nd = glm::normalize(ld(d + 3 * i));
        float t = 0.0f;
        hit[i] = glm::intersectRaySphere(ld(o + 3 * i), nd, ld(c + 3 * i), r[i] * r[i], t);
        dist[i] = t;
    }
}

// The vector operations of ray_color's shading (main_raytracing.cu:118-148): normalize, cross,
// dot, reflect, mix, min / max (NaN order), clamp.  out per input: 3 normalize(a), 3 cross(a, b),
// 1 dot(a, b), 3 reflect(a, b), 3 mix(a, b, s), 1 max(a.x, b.x), 1 min(a.x, b.x), 3 clamp(a, 0, 50).
void ref_vec_batch(int64_t n, const float* a, const float* b, const float* s, float* out) {
    for (int64_t i = 0; i < n; i++) {
        const vec3 x = ld(a + 3 * i), y = ld(b + 3 * i);
        float* o = out + 18 * i;
        st(o, glm::normalize(x));
        st(o + 3, glm::cross(x, y));
        o[6] = glm::dot(x, y);
        st(o + 7, glm::reflect(x, y));
        st(o + 10, glm::mix(x, y, s[i]));
        o[13] = glm::max(x.x, y.x);
        o[14] = glm::min(x.x, y.x);
        st(o + 15, glm::clamp(x, vec3(0), vec3(50)));
    }
}

// The sky direction (main_raytracing.cu:151): quat * vec3 for a given quaternion (w, x, y, z).
void ref_quat_rotate_batch(int64_t n, const float* q, const float* v, float* out) {
    for (int64_t i = 0; i < n; i++) {
        const glm::quat r(q[4 * i], q[4 * i + 1], q[4 * i + 2], q[4 * i + 3]);
        st(out + 3 * i, r * ld(v + 3 * i));
    }
}

// Camera::Update (Scene.cpp:15-36) in glm calls, for a camera at `pos` with angles (ax, ay) in
// degrees, fov_y degrees, viewport w x h.  out: origin(3) horizontal(3) vertical(3) llc(3).
void ref_camera(const float* pos, float ax, float ay, float fov_y, float w, float h, float* out) {
    const float aspect = w / h;
    glm::mat4 transform = glm::identity<glm::mat4>();  // Math::ComposeMatrix (Math.h:63-70)
    transform = glm::translate(transform, ld(pos));
    transform *= glm::mat4_cast(glm::quat(vec3(glm::radians(ax), glm::radians(ay), 0)));
    transform = glm::scale(transform, vec3(1));
    const glm::mat4 projection = glm::perspectiveRH(glm::radians(fov_y), aspect, 1.0f, 1000.0f);
    const glm::mat4 inv_proj = glm::inverse(projection);
    const vec4 ll4 = inv_proj * vec4(-1, -1, -1, 1);
    const vec4 ur4 = inv_proj * vec4(1, 1, -1, 1);
    vec3 llc = ll4 / ll4.w;
    const vec3 urc = ur4 / ur4.w;
    const vec3 size = urc - llc;
    st(out, ld(pos));
    st(out + 3, vec3(transform * vec4(size.x, 0, 0, 0)));
    st(out + 6, vec3(transform * vec4(0, size.y, 0, 0)));
    st(out + 9, vec3(transform * vec4(llc, 1)));
}

// AddLoadedScene's vertex transform (Scene.cpp:89-98): (transform * mesh.transform) * vec4(p, 1)
// and * vec4(n, 0), with transform = translate/rotate(axis, angle)/scale composed as the scene
// set-up does.  m = 16 floats (column-major) of the first matrix, second = 16 more.
void ref_mat_apply_batch(int64_t n, const float* m1, const float* m2, const float* p, float* out) {
    glm::mat4 a, b;
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) a[c][r] = m1[4 * c + r], b[c][r] = m2[4 * c + r];
    const glm::mat4 t = a * b;
    for (int64_t i = 0; i < n; i++) {
        st(out + 6 * i, vec3(t * vec4(ld(p + 3 * i), 1.0f)));
        st(out + 6 * i + 3, vec3(t * vec4(ld(p + 3 * i), 0.0f)));
    }
}

// glm::rotate / translate / scale / inverse as the scene set-up composes them (RayTracing.cpp
// SetupStanfordBunny: translate, rotate about an axis, scale).  out = 16 floats column-major.
void ref_trs(const float* pos, float angle, const float* axis, const float* scl, float* out) {
    glm::mat4 m = glm::identity<glm::mat4>();
    m = glm::translate(m, ld(pos));
    m = glm::rotate(m, angle, ld(axis));
    m = glm::scale(m, ld(scl));
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) out[4 * c + r] = m[c][r];
}

void ref_inverse(const float* m, float* out) {
    glm::mat4 a;
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) a[c][r] = m[4 * c + r];
    const glm::mat4 v = glm::inverse(a);
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) out[4 * c + r] = v[c][r];
}

}  // extern "C"
