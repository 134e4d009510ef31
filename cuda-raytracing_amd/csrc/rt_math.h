// rt_math.h -- deterministic fp32 vector math shared by the host scene code and the HIP
// kernels.  Every function evaluates in the operation order of the glm 0.9.9.8 routine it
// replaces (the reference's include/glm), with no contraction: the library is compiled
// with -ffp-contract=off and IEEE division/sqrt on both sides, so the CPU and the GPU give
// bit-identical results.  Citations are relative to the reference repository root.
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

namespace rtm {

struct f3 {
    float x, y, z;
};
struct f4 {
    float x, y, z, w;
};

RT_HD f3 mk(float x, float y, float z) { return f3{x, y, z}; }
RT_HD f3 add(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_HD f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_HD f3 mul(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
RT_HD f3 muls(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
RT_HD f3 divs(f3 a, float s) { return f3{a.x / s, a.y / s, a.z / s}; }
RT_HD f3 neg(f3 a) { return f3{-a.x, -a.y, -a.z}; }

// glm compute_dot<vec3> (include/glm/detail/func_geometric.inl:46-53): tmp = a*b; tmp.x+tmp.y+tmp.z
RT_HD float dot(f3 a, f3 b) {
    float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
    return (tx + ty) + tz;
}
// glm compute_cross (func_geometric.inl:66-77)
RT_HD f3 cross(f3 x, f3 y) {
    return f3{x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y};
}
// glm normalize = v * inversesqrt(dot(v,v)); inversesqrt = 1/sqrt (func_geometric.inl:82-90,
// func_exponential.inl:44-49)
RT_HD f3 normalize(f3 v) {
    float inv = 1.0f / sqrtf(dot(v, v));
    return muls(v, inv);
}
// glm reflect = I - N * dot(N, I) * 2 (func_geometric.inl:104-110)
RT_HD f3 reflect(f3 i, f3 n) { return sub(i, muls(muls(n, dot(n, i)), 2.0f)); }
// glm mix with a scalar weight: x * (1 - a) + y * a (func_common.inl:104-112)
RT_HD f3 mix(f3 x, f3 y, float a) {
    float oma = 1.0f - a;
    return add(muls(x, oma), muls(y, a));
}
RT_HD f4 mix4(f4 x, f4 y, float a) {
    float oma = 1.0f - a;
    return f4{x.x * oma + y.x * a, x.y * oma + y.y * a, x.z * oma + y.z * a, x.w * oma + y.w * a};
}
// glm max/min for scalars: (x < y) ? y : x  /  (y < x) ? y : x  (func_common.inl)
RT_HD float gmax(float x, float y) { return (x < y) ? y : x; }
RT_HD float gmin(float x, float y) { return (y < x) ? y : x; }

// ---------------------------------------------------------------------------------------
// RT deterministic sin/cos.  The reference calls CUDA's sinf/cosf inside
// GetRandomPointOnSphere (RayTracing/Random.h:26-31); their exact ulps are not
// reproducible outside nvcc, so this path DEFINES sin/cos as: quadrant k = rint(x*2/pi),
// three-part Cody-Waite reduction with fmaf, then the cephes single-precision minimax
// polynomials on [-pi/4, pi/4], every step an explicit fmaf/mul/add.  Max error ~2 ulp.
// The oracle (oracle/rt_oracle.c) restates the same definition.
// ---------------------------------------------------------------------------------------
RT_HD float rt_sin_poly(float r) {
    float z = r * r;
    float p = fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f);
    p = fmaf(z, p, -1.6666654611e-1f);
    return fmaf(r * z, p, r);
}
RT_HD float rt_cos_poly(float r) {
    float z = r * r;
    float p = fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
    p = fmaf(z, p, 4.166664568298827e-2f);
    float t = fmaf(-0.5f, z, 1.0f);
    return fmaf(z * z, p, t);
}
RT_HD float rt_reduce(float x, int* quadrant) {
    float k = rintf(x * 0.636619746685028076171875f);
    *quadrant = (int)k;
    float r = fmaf(k, -0x1.921fb6p+0f, x);
    r = fmaf(k, 0x1.777a5cp-25f, r);
    r = fmaf(k, 0x1.ee59dap-50f, r);
    return r;
}
RT_HD float rt_sinf(float x) {
    int q;
    float r = rt_reduce(x, &q);
    float s = rt_sin_poly(r), c = rt_cos_poly(r);
    switch (q & 3) {
        case 0: return s;
        case 1: return c;
        case 2: return -s;
        default: return -c;
    }
}
RT_HD float rt_cosf(float x) {
    int q;
    float r = rt_reduce(x, &q);
    float s = rt_sin_poly(r), c = rt_cos_poly(r);
    switch (q & 3) {
        case 0: return c;
        case 1: return -s;
        case 2: return -c;
        default: return s;
    }
}

// ---------------------------------------------------------------------------------------
// XORWOW as used through curand: curand() and curand_uniform() (CUDA 11.7 curand_kernel.h,
// not vendored by the reference; restated from the published algorithm -- parity unpinned
// against nvcc, step function pinned by ROCm's rocrand_xorwow.h which uses the same step).
// ---------------------------------------------------------------------------------------
struct Xorwow {
    uint32_t d, v0, v1, v2, v3, v4;
    RT_HD uint32_t next() {
        uint32_t t = v0 ^ (v0 >> 2);
        v0 = v1;
        v1 = v2;
        v2 = v3;
        v3 = v4;
        v4 = (v4 ^ (v4 << 4)) ^ (t ^ (t << 1));
        d += 362437u;
        return v4 + d;
    }
    // curand_uniform: x * 2^-32 + 2^-33 -> (0, 1]
    RT_HD float uniform() { return (float)next() * 2.3283064365386963e-10f + 1.16415321826934814453125e-10f; }
};

}  // namespace rtm
