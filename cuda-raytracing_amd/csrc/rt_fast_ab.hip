// rt_fast_ab.hip -- A/B variants behind RT_TUNE bit 12 (tools/): 1 (no split small steps) and 5 (the
// same with leaf trees).  The big-leaf mode A/B variants are in rt_fast_ab2.hip.
#include "rt_fast_body.h"

namespace rtk {
namespace {
template <int STACK>
hipError_t dispatch(int mode, const RenderArgs& a, int waves, hipStream_t s) {
    switch (mode) {
        case 1: return launch_occ<STACK, false, 1>(a, waves, s);
        case 5: return launch_occ<STACK, false, 5>(a, waves, s);
    }
    return hipErrorInvalidValue;
}
}  // namespace

hipError_t launch_fast_ab2(int stack, int mode, const RenderArgs& a, int waves, hipStream_t s);
hipError_t launch_fast_ab1(int stack, int mode, const RenderArgs& a, int waves, hipStream_t s);
RT_FAST_FAMILY(launch_fast_ab1, dispatch)

hipError_t launch_fast_ab(int stack, int mode, const RenderArgs& a, int waves, hipStream_t s) {
    return (mode == 2 || mode == 0) ? launch_fast_ab2(stack, mode, a, waves, s) : launch_fast_ab1(stack, mode, a, waves, s);
}

}  // namespace rtk
