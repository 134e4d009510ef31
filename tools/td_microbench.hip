// td_microbench.hip -- cost of a vector-memory load instruction in the CU's load path (TA
// address unit, TCP L1, TD data return) on gfx950, as a function of how many lanes of the wave
// are active, the load width and the address pattern.  Every CU runs WAVES waves; each wave
// issues ITERS x 8 independent loads of an L1-resident 16 KB table.  Output: CU cycles per
// wave-instruction (in-kernel clock: s_memtime ticks / s_memrealtime ticks x 100 MHz).
//
// The render kernel's small-step loop is a gather of 16-B node records by a partially active
// wave (tools/gpu_pmc_mem.sh: TD busy ~85 % of the kernel's cycles); this measures whether such a
// load costs the data path per active lane or per wave.
//
//   hipcc --offload-arch=gfx950 -O3 tools/td_microbench.hip -o tools/td_microbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                   \
            return 1;                                                             \
        }                                                                         \
    } while (0)

constexpr int ITERS = 512;
constexpr int TABLE = 1024;  // float4 entries (16 KB)

// pattern 0: every lane the same address; 1: lane l reads entry l (1 KB contiguous);
// 2: lane l reads its own 128-B line (64 distinct lines per instruction)
template <int WIDTH>
__global__ __launch_bounds__(64) void loads(const float4* __restrict__ tab, float* out, unsigned long long* clk,
                                            int active, int pattern) {
    const int lane = threadIdx.x & 63;
    const uint32_t off = pattern == 0 ? 0u : (pattern == 1 ? (uint32_t)lane : (uint32_t)lane * 8u);
    const uint32_t step = pattern == 2 ? 1u : 64u;
    float acc = 0.0f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if (lane < active) {
        for (int i = 0; i < ITERS; i++) {
            float s = 0.0f;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t idx = (off + (uint32_t)(i * 8 + u) * step) & (TABLE - 1);
                if constexpr (WIDTH == 16) {
                    const float4 v = tab[idx];
                    s += (v.x + v.y) + (v.z + v.w);
                } else {
                    s += reinterpret_cast<const float*>(tab)[idx * 4];
                }
            }
            acc += s;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 64 + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0, clk[1] = r1 - r0;
}

int main() {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    float4* tab;
    float* out;
    unsigned long long* clk;
    CHECK(hipMalloc(&tab, TABLE * sizeof(float4)));
    CHECK(hipMemset(tab, 0, TABLE * sizeof(float4)));
    const int max_waves = 32;
    CHECK(hipMalloc(&out, (size_t)cus * max_waves * 64 * sizeof(float)));
    CHECK(hipMalloc(&clk, 2 * sizeof(unsigned long long)));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::printf("cus %d; per CU: cycles per wave-instruction (TA/TCP/TD path)\n", cus);
    for (int width : {16, 4})
        for (int pattern : {0, 1, 2})
            for (int waves : {8, 24})
                for (int active : {64, 32, 16, 4, 1}) {
                    const int grid = cus * waves;
                    for (int rep = 0; rep < 2; rep++) {
                        CHECK(hipEventRecord(e0));
                        if (width == 16)
                            hipLaunchKernelGGL(loads<16>, dim3(grid), dim3(64), 0, 0, tab, out, clk, active, pattern);
                        else
                            hipLaunchKernelGGL(loads<4>, dim3(grid), dim3(64), 0, 0, tab, out, clk, active, pattern);
                        CHECK(hipGetLastError());
                        CHECK(hipEventRecord(e1));
                        CHECK(hipEventSynchronize(e1));
                        if (rep == 0) continue;
                        float ms = 0;
                        CHECK(hipEventElapsedTime(&ms, e0, e1));
                        unsigned long long c[2];
                        CHECK(hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost));
                        const double ghz = c[1] ? (double)c[0] / ((double)c[1] * 10.0) : 2.4;  // memrealtime: 100 MHz
                        const double instr_per_cu = (double)waves * ITERS * 8;
                        const double cyc = ms * 1e-3 * ghz * 1e9 / instr_per_cu;
                        std::printf("width %2d pattern %d waves/CU %2d active %2d: %7.2f cycles/instr  (%.3f ms, clock %.2f GHz)\n",
                                    width, pattern, waves, active, cyc, ms, ghz);
                    }
                }
    return 0;
}
