// rt_render.h -- launchers of the render kernels, one family per translation unit (rt_kernel.hip
// dispatches; the families compile in parallel).  `stack` is the traversal stack size of the
// instantiation (30, 40 or 64 entries: the scene's BVH depth + 2 rounded up), `mode` the MODE bits of
// render_fast_body (rt_fast_body.h).  Each returns hipErrorInvalidValue for a mode it does not hold.
#pragma once

#include <hip/hip_runtime.h>

#include "rt_common.h"

namespace rtk {

// In librt_hip.so (the product): the kernels the production path launches.
hipError_t launch_fast_prod(int stack, int mode, const RenderArgs& a, int waves, hipStream_t s);    // 17, 21
hipError_t launch_fast_timing(int stack, int mode, const RenderArgs& a, int waves, hipStream_t s);  // 25, 29, 9
hipError_t launch_fast_stats(int stack, int mode, const RenderArgs& a, int waves, hipStream_t s);   // 2, 6 (counting)
// The reference-layout tracer (flat = false) or the exact-division flat tracer (rt_ref.hip).
hipError_t launch_ref_tracer(bool flat, const RenderArgs& a, int waves, int depth, bool stats, hipStream_t s);

// In librt_hip_exp.so (rt_exp.hip): exact alternatives kept for A/B measurement and their parity
// tests, none of which serves the benchmark -- loading the library registers them (rt_render then
// accepts the flags / knobs that select them; without it those requests are refused).
hipError_t launch_fast_ab(int stack, int mode, const RenderArgs& a, int waves, hipStream_t s);      // 1, 5, 2, 0
hipError_t launch_fast_refill(int stack, int mode, const RenderArgs& a, int waves, hipStream_t s);  // 81, 85
hipError_t launch_fast_screen(int stack, int mode, const RenderArgs& a, int waves, hipStream_t s);  // 49, 53, 57, 61
// The lone-pixel kernel (rt_lone.hip): one wave per slot of `lone_slots`, through the treelets.
hipError_t launch_lone(const RenderArgs& a, const int32_t* lone_slots, int lone_count, const void* treelets, hipStream_t s);
// The wavefront tracer (rt_wavefront.hip): shade / trace launches per segment generation.
hipError_t launch_wavefront(const RenderArgs& a, int depth, hipStream_t s);

struct ExperimentalKernels {
    decltype(&launch_fast_ab) fast_ab;
    decltype(&launch_fast_refill) fast_refill;
    decltype(&launch_lone) lone;
    decltype(&launch_wavefront) wavefront;
    decltype(&launch_fast_screen) fast_screen;
};
// Layout stamp of what the plugin shares with librt_hip.so (RenderArgs by reference, this table): a
// version bumped by hand when a field changes meaning, and the two sizes.  A plugin built against another
// layout is refused at registration instead of reading a different struct (rt_exp_abi_version).
constexpr uint32_t kExperimentalAbi = (2u << 24) ^ ((uint32_t)sizeof(RenderArgs) << 8) ^ (uint32_t)sizeof(ExperimentalKernels);
// rt_kernel.hip: the registered table (nullptr until librt_hip_exp.so is loaded); a table whose `abi` is
// not this library's kExperimentalAbi is refused (rt_last_error says so, rt_experimental_loaded stays 0).
void register_experimental_kernels(const ExperimentalKernels* k, uint32_t abi);
const ExperimentalKernels* experimental_kernels();

}  // namespace rtk
