// rt_host_math.h -- host-only 4x4 matrix / quaternion routines used to build scene inputs
// (camera basis, mesh transforms).  Each follows the glm 0.9.9.8 routine the reference calls,
// in glm's operation order (column-major storage, m[column][row]).  Trigonometry on the host
// is std::sin/cos/tan evaluated in double and rounded to float (correctly rounded in
// practice), standing in for the reference host compiler's sinf/cosf/tanf.
#pragma once

#include <cmath>
#include <cstring>

#include "rt_math.h"

namespace rth {

struct mat4 {
    float m[4][4];  // m[col][row]
};

inline float hsin(float x) { return (float)std::sin((double)x); }
inline float hcos(float x) { return (float)std::cos((double)x); }
inline float htan(float x) { return (float)std::tan((double)x); }

inline mat4 identity() {
    mat4 r;
    std::memset(&r, 0, sizeof(r));
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.0f;
    return r;
}

// glm::radians: degrees * 0.01745329251994329576923690768489 (trigonometric.inl)
inline float radians(float deg) { return deg * 0.01745329251994329576923690768489f; }

// col = a*s componentwise
inline void col_muls(float out[4], const float a[4], float s) {
    for (int i = 0; i < 4; i++) out[i] = a[i] * s;
}

// glm mat4 * mat4 (detail/type_mat4x4.inl:630-648): Result[c] = ((A0*B[c][0] + A1*B[c][1]) +
// A2*B[c][2]) + A3*B[c][3]
inline mat4 mul(const mat4& a, const mat4& b) {
    mat4 r;
    for (int c = 0; c < 4; c++)
        for (int i = 0; i < 4; i++)
            r.m[c][i] = ((a.m[0][i] * b.m[c][0] + a.m[1][i] * b.m[c][1]) + a.m[2][i] * b.m[c][2]) +
                        a.m[3][i] * b.m[c][3];
    return r;
}

// glm mat4 * vec4 (type_mat4x4.inl:536-575): (m0*v0 + m1*v1) + (m2*v2 + m3*v3)
inline rtm::f4 mulv(const mat4& a, rtm::f4 v) {
    float in[4] = {v.x, v.y, v.z, v.w};
    float o[4];
    for (int i = 0; i < 4; i++)
        o[i] = (a.m[0][i] * in[0] + a.m[1][i] * in[1]) + (a.m[2][i] * in[2] + a.m[3][i] * in[3]);
    return rtm::f4{o[0], o[1], o[2], o[3]};
}

// glm::translate (ext/matrix_transform.inl:10-15): Result[3] = ((m0*v0 + m1*v1) + m2*v2) + m3
inline mat4 translate(const mat4& m, rtm::f3 v) {
    mat4 r = m;
    for (int i = 0; i < 4; i++) r.m[3][i] = ((m.m[0][i] * v.x + m.m[1][i] * v.y) + m.m[2][i] * v.z) + m.m[3][i];
    return r;
}

// glm::scale (ext/matrix_transform.inl:78-86)
inline mat4 scale(const mat4& m, rtm::f3 v) {
    mat4 r;
    col_muls(r.m[0], m.m[0], v.x);
    col_muls(r.m[1], m.m[1], v.y);
    col_muls(r.m[2], m.m[2], v.z);
    for (int i = 0; i < 4; i++) r.m[3][i] = m.m[3][i];
    return r;
}

// glm::rotate (ext/matrix_transform.inl:17-45)
inline mat4 rotate(const mat4& m, float angle, rtm::f3 v) {
    const float c = hcos(angle), s = hsin(angle);
    rtm::f3 axis = rtm::normalize(v);
    rtm::f3 temp = rtm::muls(axis, 1.0f - c);
    float R[3][3];
    R[0][0] = c + temp.x * axis.x;
    R[0][1] = temp.x * axis.y + s * axis.z;
    R[0][2] = temp.x * axis.z - s * axis.y;
    R[1][0] = temp.y * axis.x - s * axis.z;
    R[1][1] = c + temp.y * axis.y;
    R[1][2] = temp.y * axis.z + s * axis.x;
    R[2][0] = temp.z * axis.x + s * axis.y;
    R[2][1] = temp.z * axis.y - s * axis.x;
    R[2][2] = c + temp.z * axis.z;
    mat4 r;
    for (int c2 = 0; c2 < 3; c2++)
        for (int i = 0; i < 4; i++)
            r.m[c2][i] = (m.m[0][i] * R[c2][0] + m.m[1][i] * R[c2][1]) + m.m[2][i] * R[c2][2];
    for (int i = 0; i < 4; i++) r.m[3][i] = m.m[3][i];
    return r;
}

struct quat {
    float w, x, y, z;
};

// glm qua(vec3 eulerAngle) (detail/type_quat.inl:204-213)
inline quat quat_from_euler(rtm::f3 e, float (*cosf_)(float) = hcos, float (*sinf_)(float) = hsin) {
    float cx = cosf_(e.x * 0.5f), cy = cosf_(e.y * 0.5f), cz = cosf_(e.z * 0.5f);
    float sx = sinf_(e.x * 0.5f), sy = sinf_(e.y * 0.5f), sz = sinf_(e.z * 0.5f);
    quat q;
    q.w = cx * cy * cz + sx * sy * sz;
    q.x = sx * cy * cz - cx * sy * sz;
    q.y = cx * sy * cz + sx * cy * sz;
    q.z = cx * cy * sz - sx * sy * cz;
    return q;
}

// glm mat4_cast(quat) via mat3_cast (gtc/quaternion.inl:41-72)
inline mat4 mat4_cast(const quat& q) {
    float qxx = q.x * q.x, qyy = q.y * q.y, qzz = q.z * q.z;
    float qxz = q.x * q.z, qxy = q.x * q.y, qyz = q.y * q.z;
    float qwx = q.w * q.x, qwy = q.w * q.y, qwz = q.w * q.z;
    mat4 r = identity();
    r.m[0][0] = 1.0f - 2.0f * (qyy + qzz);
    r.m[0][1] = 2.0f * (qxy + qwz);
    r.m[0][2] = 2.0f * (qxz - qwy);
    r.m[1][0] = 2.0f * (qxy - qwz);
    r.m[1][1] = 1.0f - 2.0f * (qxx + qzz);
    r.m[1][2] = 2.0f * (qyz + qwx);
    r.m[2][0] = 2.0f * (qxz + qwy);
    r.m[2][1] = 2.0f * (qyz - qwx);
    r.m[2][2] = 1.0f - 2.0f * (qxx + qyy);
    return r;
}

// glm::perspectiveRH_NO (ext/matrix_clip_space.inl:249-262)
inline mat4 perspective_rh_no(float fovy, float aspect, float znear, float zfar) {
    const float tan_half = htan(fovy / 2.0f);
    mat4 r;
    std::memset(&r, 0, sizeof(r));
    r.m[0][0] = 1.0f / (aspect * tan_half);
    r.m[1][1] = 1.0f / tan_half;
    r.m[2][2] = -(zfar + znear) / (zfar - znear);
    r.m[2][3] = -1.0f;
    r.m[3][2] = -(2.0f * zfar * znear) / (zfar - znear);
    return r;
}

// glm compute_inverse<4,4> (detail/func_matrix.inl:294-351)
inline mat4 inverse(const mat4& M) {
    const float(*m)[4] = M.m;
    float c00 = m[2][2] * m[3][3] - m[3][2] * m[2][3];
    float c02 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
    float c03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float c04 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float c06 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float c07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float c08 = m[2][1] * m[3][2] - m[3][1] * m[2][2];
    float c10 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
    float c11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float c12 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float c14 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
    float c15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float c16 = m[2][0] * m[3][2] - m[3][0] * m[2][2];
    float c18 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
    float c19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float c20 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float c22 = m[1][0] * m[3][1] - m[3][0] * m[1][1];
    float c23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    float f0[4] = {c00, c00, c02, c03}, f1[4] = {c04, c04, c06, c07}, f2[4] = {c08, c08, c10, c11};
    float f3_[4] = {c12, c12, c14, c15}, f4_[4] = {c16, c16, c18, c19}, f5[4] = {c20, c20, c22, c23};
    float v0[4] = {m[1][0], m[0][0], m[0][0], m[0][0]};
    float v1[4] = {m[1][1], m[0][1], m[0][1], m[0][1]};
    float v2[4] = {m[1][2], m[0][2], m[0][2], m[0][2]};
    float v3[4] = {m[1][3], m[0][3], m[0][3], m[0][3]};
    float i0[4], i1[4], i2[4], i3[4];
    for (int k = 0; k < 4; k++) {
        i0[k] = (v1[k] * f0[k] - v2[k] * f1[k]) + v3[k] * f2[k];
        i1[k] = (v0[k] * f0[k] - v2[k] * f3_[k]) + v3[k] * f4_[k];
        i2[k] = (v0[k] * f1[k] - v1[k] * f3_[k]) + v3[k] * f5[k];
        i3[k] = (v0[k] * f2[k] - v1[k] * f4_[k]) + v2[k] * f5[k];
    }
    const float sa[4] = {1, -1, 1, -1}, sb[4] = {-1, 1, -1, 1};
    mat4 inv;
    for (int k = 0; k < 4; k++) {
        inv.m[0][k] = i0[k] * sa[k];
        inv.m[1][k] = i1[k] * sb[k];
        inv.m[2][k] = i2[k] * sa[k];
        inv.m[3][k] = i3[k] * sb[k];
    }
    float row0[4] = {inv.m[0][0], inv.m[1][0], inv.m[2][0], inv.m[3][0]};
    float d0[4];
    for (int k = 0; k < 4; k++) d0[k] = m[0][k] * row0[k];
    float d1 = (d0[0] + d0[1]) + (d0[2] + d0[3]);
    float one_over = 1.0f / d1;
    mat4 r;
    for (int c = 0; c < 4; c++)
        for (int k = 0; k < 4; k++) r.m[c][k] = inv.m[c][k] * one_over;
    return r;
}

}  // namespace rth
