// xorwow.cpp -- host side of the per-pixel RNG seeding (RayTracing/Random.cu:3-13).
//
// curand_init(seed, subsequence, 0) (CUDA curand_kernel.h, not vendored by the reference) =
//   1. salt and mix the 64-bit seed into the XORWOW state (constants restated from the
//      published curand source: 0xaad26b49, 0xf7dcefdd, 1099087573, 2591861531 and the
//      Marsaglia bases 123456789, 362436069, 521288629, 88675123, 5783321, 6615241);
//   2. advance the 160-bit xorshift part by subsequence * 2^67 steps (the Weyl counter d is
//      unchanged because 2^67 * 362437 = 0 mod 2^32).
// Step 2 is the linear map A^(subsequence * 2^67) over GF(2).  The jump matrices
// M_k = A^(4^k * 2^67) are computed here from A by repeated squaring (no tables are
// copied); tests pin them against rocrand's independently published table
// (rocrand_xorwow_precomputed.h, h_xorwow_sequence_jump_matrices), which describes the
// same recurrence.
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "rt_abi.h"
#include "rt_math.h"
#include "xorwow.h"

namespace {

// Matrix layout (rocrand's): m[i*160 + j*5 + w] = output word w of A applied to the unit
// vector with bit j of input word i set.
using Mat = std::vector<uint32_t>;

void apply(const uint32_t* m, const uint32_t in[5], uint32_t out[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 5; i++)
        for (int j = 0; j < 32; j++) {
            const uint32_t mask = 0u - ((in[i] >> j) & 1u);
            const uint32_t* row = m + i * 160 + j * 5;
            for (int w = 0; w < 5; w++) r[w] ^= row[w] & mask;
        }
    std::memcpy(out, r, sizeof(r));
}

Mat one_step() {
    Mat a(800);
    for (int i = 0; i < 5; i++)
        for (int j = 0; j < 32; j++) {
            rtm::Xorwow x{0, 0, 0, 0, 0, 0};
            uint32_t* v[5] = {&x.v0, &x.v1, &x.v2, &x.v3, &x.v4};
            *v[i] = 1u << j;
            x.next();
            const uint32_t o[5] = {x.v0, x.v1, x.v2, x.v3, x.v4};
            for (int w = 0; w < 5; w++) a[i * 160 + j * 5 + w] = o[w];
        }
    return a;
}

Mat square(const Mat& m) {
    Mat r(800);
    for (int i = 0; i < 5; i++)
        for (int j = 0; j < 32; j++) apply(m.data(), &m[i * 160 + j * 5], &r[i * 160 + j * 5]);
    return r;
}

std::once_flag g_once;
std::vector<Mat> g_jump;  // g_jump[k] = A^(4^k * 2^67), k < RT_XORWOW_JUMPS

void build() {
    Mat m = one_step();
    for (int s = 0; s < 67; s++) m = square(m);
    g_jump.push_back(m);
    for (int k = 1; k < RT_XORWOW_JUMPS; k++) {
        m = square(square(m));
        g_jump.push_back(m);
    }
}

}  // namespace

const uint32_t* rt_xorwow_jump_table() {
    std::call_once(g_once, build);
    static std::vector<uint32_t> flat;
    static std::once_flag flat_once;
    std::call_once(flat_once, [] {
        flat.resize((size_t)RT_XORWOW_JUMPS * 800);
        for (int k = 0; k < RT_XORWOW_JUMPS; k++) std::memcpy(&flat[(size_t)k * 800], g_jump[k].data(), 800 * 4);
    });
    return flat.data();
}

extern "C" int rt_xorwow_jump_matrix(int k, uint32_t out[800]) {
    if (k < 0 || k >= RT_XORWOW_JUMPS) return 1;
    std::memcpy(out, rt_xorwow_jump_table() + (size_t)k * 800, 800 * 4);
    return 0;
}

extern "C" void rt_xorwow_init_host(uint32_t seed, uint64_t subsequence, rt_rng_state* out) {
    uint32_t st[6];
    rt_xorwow_seed(seed, st);
    uint32_t v[5] = {st[1], st[2], st[3], st[4], st[5]};
    const uint32_t* table = rt_xorwow_jump_table();
    for (int k = 0; subsequence && k < RT_XORWOW_JUMPS; k++, subsequence >>= 2)
        for (uint32_t t = 0; t < (subsequence & 3u); t++) apply(table + (size_t)k * 800, v, v);
    std::memset(out, 0, sizeof(*out));
    out->d = st[0];
    for (int i = 0; i < 5; i++) out->v[i] = v[i];
}
