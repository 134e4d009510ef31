// rt_fast_timing.hip -- timing variants of the production kernel (MODE bit 3: phase clocks, per-pixel
// work for rt_lane_plan, per-wave clock records): 25 (= 17 + timing), 29 (= 21 + timing), 9 (no split).
#include "rt_fast_body.h"

namespace rtk {
namespace {
template <int STACK>
hipError_t dispatch(int mode, const RenderArgs& a, int waves, hipStream_t s) {
    switch (mode) {
        case 25: return launch_occ<STACK, false, 25>(a, waves, s);
        case 29: return launch_occ<STACK, false, 29>(a, waves, s);
        case 9: return launch_occ<STACK, false, 9>(a, waves, s);
    }
    return hipErrorInvalidValue;
}
}  // namespace

RT_FAST_FAMILY(launch_fast_timing, dispatch)

}  // namespace rtk
