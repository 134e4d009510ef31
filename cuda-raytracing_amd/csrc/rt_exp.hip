// rt_exp.hip -- librt_hip_exp.so: registers the experimental render paths with librt_hip.so when the
// library is loaded (rt_render.h ExperimentalKernels).  The product library carries only the kernels
// the production path launches; these stay exact and tested (tests load this library through
// rt.load_experimental()), and measured slower or neutral for the benchmark.
#include "rt_render.h"

namespace rtk {
namespace {
const ExperimentalKernels kTable{launch_fast_ab, launch_fast_refill, launch_lone, launch_wavefront, launch_fast_screen};
struct Registrar {
    Registrar() { register_experimental_kernels(&kTable, kExperimentalAbi); }
    ~Registrar() { register_experimental_kernels(nullptr, kExperimentalAbi); }
} registrar;
}  // namespace
}  // namespace rtk

extern "C" int rt_exp_abi_version() { return (int)rtk::kExperimentalAbi; }
