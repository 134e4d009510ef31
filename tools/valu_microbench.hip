// valu_microbench.hip -- issue cost of the VALU instruction kinds the render kernel is made of,
// on gfx950: every SIMD runs WAVES waves, each wave a long unrolled stream of independent
// instructions of one kind (8 accumulators, no dependence between consecutive instructions).
// Output: cycles per wave-instruction per SIMD for each kind, relative to wall time x clock
// (in-kernel clock from s_memtime / s_memrealtime, MI355X_MICROARCH.md "DVFS give-back").
//
//   hipcc --offload-arch=gfx950 -O3 tools/valu_microbench.hip -o /tmp/valu_microbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                   \
            return 1;                                                             \
        }                                                                         \
    } while (0)

constexpr int ITERS = 256;  // outer iterations
constexpr int UNROLL = 16;  // inner: UNROLL x 8 instructions

#define OP8(OPSTR)                                                                                       \
    asm volatile(OPSTR : "+v"(a0) : "v"(b) : "vcc");                                                     \
    asm volatile(OPSTR : "+v"(a1) : "v"(b) : "vcc");                                                     \
    asm volatile(OPSTR : "+v"(a2) : "v"(b) : "vcc");                                                     \
    asm volatile(OPSTR : "+v"(a3) : "v"(b) : "vcc");                                                     \
    asm volatile(OPSTR : "+v"(a4) : "v"(b) : "vcc");                                                     \
    asm volatile(OPSTR : "+v"(a5) : "v"(b) : "vcc");                                                     \
    asm volatile(OPSTR : "+v"(a6) : "v"(b) : "vcc");                                                     \
    asm volatile(OPSTR : "+v"(a7) : "v"(b) : "vcc");
typedef float f2 __attribute__((ext_vector_type(2)));
#define PK8(OPSTR)                                                                                       \
    asm volatile(OPSTR : "+v"(p0) : "v"(q));                                                             \
    asm volatile(OPSTR : "+v"(p1) : "v"(q));                                                             \
    asm volatile(OPSTR : "+v"(p2) : "v"(q));                                                             \
    asm volatile(OPSTR : "+v"(p3) : "v"(q));                                                             \
    asm volatile(OPSTR : "+v"(p4) : "v"(q));                                                             \
    asm volatile(OPSTR : "+v"(p5) : "v"(q));                                                             \
    asm volatile(OPSTR : "+v"(p6) : "v"(q));                                                             \
    asm volatile(OPSTR : "+v"(p7) : "v"(q));

template <int K>
__global__ __launch_bounds__(64) void bench(float* out, unsigned long long* clk, float seed) {
    float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7, b = seed * 0.5f;
    f2 p0 = {a0, a1}, p1 = {a1, a2}, p2 = {a2, a3}, p3 = {a3, a4}, p4 = {a4, a5}, p5 = {a5, a6}, p6 = {a6, a7},
       p7 = {a7, a0}, q = {b, b};
    uint32_t sreg = (uint32_t)__builtin_amdgcn_readfirstlane((int)blockIdx.x);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int u = 0; u < UNROLL; u++) {
            if constexpr (K == 0) { OP8("v_add_f32 %0, %0, %1") }
            if constexpr (K == 1) { OP8("v_fma_f32 %0, %0, %1, %1") }
            if constexpr (K == 2) { OP8("v_min_f32 %0, %0, %1") }
            if constexpr (K == 3) { OP8("v_max3_f32 %0, %0, %1, %1") }
            if constexpr (K == 4) { OP8("v_and_b32 %0, %0, %1") }
            if constexpr (K == 5) { OP8("v_add_u32 %0, %0, %1") }
            if constexpr (K == 6) { OP8("v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc") }
            if constexpr (K == 7) { OP8("v_cndmask_b32 %0, %0, %1, vcc") }
            if constexpr (K == 8) { PK8("v_pk_mul_f32 %0, %0, %1") }
            if constexpr (K == 9) { OP8("v_rcp_f32 %0, %0") }
            if constexpr (K == 10) { OP8("v_mul_f32 %0, %0, %1") }
            if constexpr (K == 11) { OP8("v_sub_f32 %0, %0, %1") }
            if constexpr (K == 12) { OP8("v_xor_b32 %0, %0, %1") }
            if constexpr (K == 13) { OP8("v_cmp_lt_f32 vcc, %0, %1") }
            if constexpr (K == 14) { OP8("v_lshlrev_b32 %0, 2, %0") }
            if constexpr (K == 15) { OP8("v_mov_b32 %0, %1") }
            if constexpr (K == 16) {  // one VALU + one independent SALU per slot (do they co-issue?)
                asm volatile("v_add_f32 %0, %0, %2\n s_add_u32 %1, %1, 1" : "+v"(a0), "+s"(sreg) : "v"(b) : "scc");
                asm volatile("v_add_f32 %0, %0, %2\n s_add_u32 %1, %1, 1" : "+v"(a1), "+s"(sreg) : "v"(b) : "scc");
                asm volatile("v_add_f32 %0, %0, %2\n s_add_u32 %1, %1, 1" : "+v"(a2), "+s"(sreg) : "v"(b) : "scc");
                asm volatile("v_add_f32 %0, %0, %2\n s_add_u32 %1, %1, 1" : "+v"(a3), "+s"(sreg) : "v"(b) : "scc");
                asm volatile("v_add_f32 %0, %0, %2\n s_add_u32 %1, %1, 1" : "+v"(a4), "+s"(sreg) : "v"(b) : "scc");
                asm volatile("v_add_f32 %0, %0, %2\n s_add_u32 %1, %1, 1" : "+v"(a5), "+s"(sreg) : "v"(b) : "scc");
                asm volatile("v_add_f32 %0, %0, %2\n s_add_u32 %1, %1, 1" : "+v"(a6), "+s"(sreg) : "v"(b) : "scc");
                asm volatile("v_add_f32 %0, %0, %2\n s_add_u32 %1, %1, 1" : "+v"(a7), "+s"(sreg) : "v"(b) : "scc");
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    const f2 ps = p0 + p1 + p2 + p3 + p4 + p5 + p6 + p7;
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + ps.x + ps.y + (float)sreg;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int K>
int run(const char* name, int waves_per_simd, int cus) {
    const int blocks = cus * 4 * waves_per_simd;
    float* out;
    unsigned long long* clk;
    CHECK(hipMalloc(&out, (size_t)blocks * 64 * 4));
    CHECK(hipMalloc(&clk, (size_t)blocks * 16));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(bench<K>, dim3(blocks), dim3(64), 0, 0, out, clk, 1.0f);  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(bench<K>, dim3(blocks), dim3(64), 0, 0, out, clk, 1.0f);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> c(2 * blocks);
    CHECK(hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost));
    double cyc = 0, real = 0;
    for (int i = 0; i < blocks; i++) cyc += c[2 * i], real += c[2 * i + 1];
    cyc /= blocks, real /= blocks;
    const double ghz = cyc / (real / 100e6) / 1e9;  // s_memrealtime ticks at 100 MHz
    const int per_op = (K == 6) ? 2 : 1;  // K == 16 counts the VALU instructions only
    const double instr_per_wave = (double)ITERS * UNROLL * 8 * per_op;
    // per SIMD: waves_per_simd waves, each instr_per_wave instructions, in `cyc` cycles
    std::printf("%-24s waves/SIMD %d  %.2f cycles per wave-instruction per SIMD (wave clock %.3g cyc, %.2f GHz, %.3f ms)\n",
                name, waves_per_simd, cyc / (instr_per_wave * waves_per_simd), cyc, ghz, ms);
    hipFree(out);
    hipFree(clk);
    return 0;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int w : {1, 2, 3, 4, 6, 8}) {
        run<16>("v_add_f32 + s_add_u32", w, cus);
        run<0>("v_add_f32", w, cus);
        run<1>("v_fma_f32", w, cus);
        run<10>("v_mul_f32", w, cus);
        run<11>("v_sub_f32", w, cus);
        run<2>("v_min_f32", w, cus);
        run<3>("v_max3_f32", w, cus);
        run<4>("v_and_b32", w, cus);
        run<12>("v_xor_b32", w, cus);
        run<5>("v_add_u32", w, cus);
        run<14>("v_lshlrev_b32", w, cus);
        run<15>("v_mov_b32", w, cus);
        run<13>("v_cmp_lt_f32 (vcc)", w, cus);
        run<7>("v_cndmask_b32", w, cus);
        run<6>("v_cmp + v_cndmask (avg)", w, cus);
        run<8>("v_pk_mul_f32", w, cus);
        run<9>("v_rcp_f32", w, cus);
    }
    return 0;
}
