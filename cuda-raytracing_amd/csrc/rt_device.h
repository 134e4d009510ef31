// rt_device.h -- per-ray math of the render kernel, written once for host and device.
// Each routine restates the reference function it cites, in its floating-point operation
// order (no contraction; IEEE division and sqrt).
#pragma once

#include "rt_math.h"

namespace rtd {

using rtm::f3;

// Math.h:50-61 IntersectAABB with the device CUDA_MIN/CUDA_MAX = fminf/fmaxf
// (utils/CUDAHelper.h:31-32).  `d` is the UNNORMALIZED ray direction; ray_length is the
// current closest distance measured along the normalized direction.
RT_HD bool intersect_aabb(f3 o, f3 d, const float* bmin, const float* bmax, float ray_length) {
    float tx1 = (bmin[0] - o.x) / d.x, tx2 = (bmax[0] - o.x) / d.x;
    float tmin = fminf(tx1, tx2), tmax = fmaxf(tx1, tx2);
    float ty1 = (bmin[1] - o.y) / d.y, ty2 = (bmax[1] - o.y) / d.y;
    tmin = fmaxf(tmin, fminf(ty1, ty2)), tmax = fminf(tmax, fmaxf(ty1, ty2));
    float tz1 = (bmin[2] - o.z) / d.z, tz2 = (bmax[2] - o.z) / d.z;
    tmin = fmaxf(tmin, fminf(tz1, tz2)), tmax = fminf(tmax, fmaxf(tz1, tz2));
    return tmax >= tmin && tmin < ray_length && tmax > 0;
}

// glm::intersectRayTriangle (include/glm/gtx/intersect.inl:29-94) with the two edges
// edge1 = vert1 - vert0, edge2 = vert2 - vert0 already formed; `dir` is normalized.
// On success writes bary (scaled by 1/det) and distance.
RT_HD bool intersect_triangle_e(f3 orig, f3 dir, f3 v0, f3 edge1, f3 edge2, float* bx, float* by, float* distance) {
    const float eps = 1.1920928955078125e-07f;  // std::numeric_limits<float>::epsilon()
    const f3 p = rtm::cross(dir, edge2);
    const float det = rtm::dot(edge1, p);
    f3 perp;
    float u, v;
    if (det > eps) {
        const f3 dist = rtm::sub(orig, v0);
        u = rtm::dot(dist, p);
        if (u < 0.0f || u > det) return false;
        perp = rtm::cross(dist, edge1);
        v = rtm::dot(dir, perp);
        if (v < 0.0f || (u + v) > det) return false;
    } else if (det < -eps) {
        const f3 dist = rtm::sub(orig, v0);
        u = rtm::dot(dist, p);
        if (u > 0.0f || u < det) return false;
        perp = rtm::cross(dist, edge1);
        v = rtm::dot(dir, perp);
        if (v > 0.0f || (u + v) < det) return false;
    } else {
        return false;
    }
    const float inv_det = 1.0f / det;
    *distance = rtm::dot(edge2, perp) * inv_det;
    *bx = u * inv_det;
    *by = v * inv_det;
    return true;
}

RT_HD bool intersect_triangle(f3 orig, f3 dir, f3 v0, f3 v1, f3 v2, float* bx, float* by, float* distance) {
    return intersect_triangle_e(orig, dir, v0, rtm::sub(v1, v0), rtm::sub(v2, v0), bx, by, distance);
}

// glm::intersectRaySphere (intersect.inl:135-153) with the squared radius.
RT_HD bool intersect_sphere(f3 start, f3 ndir, f3 center, float r2, float* distance) {
    const float eps = 1.1920928955078125e-07f;
    const f3 diff = rtm::sub(center, start);
    const float t0 = rtm::dot(diff, ndir);
    const float d2 = rtm::dot(diff, diff) - t0 * t0;
    if (d2 > r2) return false;
    const float t1 = sqrtf(r2 - d2);
    const float dist = t0 > t1 + eps ? t0 - t1 : t0 + t1;
    *distance = dist;
    return dist > eps;
}

// glm qua * vec3 (detail/type_quat.inl:343-350)
RT_HD f3 quat_rotate(float qw, float qx, float qy, float qz, f3 v) {
    const f3 qv = rtm::mk(qx, qy, qz);
    const f3 uv = rtm::cross(qv, v);
    const f3 uuv = rtm::cross(qv, uv);
    return rtm::add(v, rtm::muls(rtm::add(rtm::muls(uv, qw), uuv), 2.0f));
}

// ---------------------------------------------------------------------------------------
// Cube map lookup standing in for texCubemapLod<float4>(tex, x, y, z, 0) with
// cudaFilterModeLinear + seamlessCubemap (utils/CUDATexture.cpp:160-171,
// main_raytracing.cu:152).  The NVIDIA texture unit is not reproducible here (parity
// unpinned); this DEFINES the lookup: D3D/GL major-axis face selection, bilinear filtering
// at texel centres with 8-bit fractional weights (the CUDA guide's 9-bit fixed-point
// format), and seamless filtering by re-projecting off-face texels onto the neighbouring
// face.  Texels: float4 [6][n][n], face order +X,-X,+Y,-Y,+Z,-Z, row 0 = t 0.
// ---------------------------------------------------------------------------------------
RT_HD void cube_coords(float x, float y, float z, int* face, float* s, float* t) {
    const float ax = fabsf(x), ay = fabsf(y), az = fabsf(z);
    float ma, sc, tc;
    if (ax >= ay && ax >= az) {
        ma = ax;
        *face = x >= 0.0f ? 0 : 1;
        sc = x >= 0.0f ? -z : z;
        tc = -y;
    } else if (ay >= az) {
        ma = ay;
        *face = y >= 0.0f ? 2 : 3;
        sc = x;
        tc = y >= 0.0f ? z : -z;
    } else {
        ma = az;
        *face = z >= 0.0f ? 4 : 5;
        sc = z >= 0.0f ? x : -x;
        tc = -y;
    }
    *s = (sc / ma + 1.0f) * 0.5f;
    *t = (tc / ma + 1.0f) * 0.5f;
}

RT_HD int cube_texel_index(int face, int i, int j, int n) {
    if (i >= 0 && i < n && j >= 0 && j < n) return (face * n + j) * n + i;
    const float sc = (float)(2 * i + 1) / (float)n - 1.0f;
    const float tc = (float)(2 * j + 1) / (float)n - 1.0f;
    float x, y, z;
    switch (face) {
        case 0: x = 1.0f, y = -tc, z = -sc; break;
        case 1: x = -1.0f, y = -tc, z = sc; break;
        case 2: x = sc, y = 1.0f, z = tc; break;
        case 3: x = sc, y = -1.0f, z = -tc; break;
        case 4: x = sc, y = -tc, z = 1.0f; break;
        default: x = -sc, y = -tc, z = -1.0f; break;
    }
    int f2;
    float s2, t2;
    cube_coords(x, y, z, &f2, &s2, &t2);
    int i2 = (int)floorf(s2 * (float)n), j2 = (int)floorf(t2 * (float)n);
    i2 = i2 < 0 ? 0 : (i2 > n - 1 ? n - 1 : i2);
    j2 = j2 < 0 ? 0 : (j2 > n - 1 ? n - 1 : j2);
    return (f2 * n + j2) * n + i2;
}

// texels: float RGBA, 4 floats per texel.
RT_HD f3 cube_sample(const float* texels, int n, f3 dir) {
    int face;
    float s, t;
    cube_coords(dir.x, dir.y, dir.z, &face, &s, &t);
    const float u = s * (float)n - 0.5f, v = t * (float)n - 0.5f;
    const float fu = floorf(u), fv = floorf(v);
    const int i0 = (int)fu, j0 = (int)fv;
    const float a = rintf((u - fu) * 256.0f) * 0.00390625f;
    const float b = rintf((v - fv) * 256.0f) * 0.00390625f;
    const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    const float* t00 = texels + 4 * cube_texel_index(face, i0, j0, n);
    const float* t10 = texels + 4 * cube_texel_index(face, i0 + 1, j0, n);
    const float* t01 = texels + 4 * cube_texel_index(face, i0, j0 + 1, n);
    const float* t11 = texels + 4 * cube_texel_index(face, i0 + 1, j0 + 1, n);
    f3 r;
    r.x = ((w00 * t00[0] + w10 * t10[0]) + w01 * t01[0]) + w11 * t11[0];
    r.y = ((w00 * t00[1] + w10 * t10[1]) + w01 * t01[1]) + w11 * t11[1];
    r.z = ((w00 * t00[2] + w10 * t10[2]) + w01 * t01[2]) + w11 * t11[2];
    return r;
}

}  // namespace rtd
