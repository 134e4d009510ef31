// rt_fast_screen.hip -- big-leaf screen variants (MODE bit 5; rt_fast.h screen_leaf, mirror.h pf = 3):
// 49 / 53 (= 17 / 21 + screens), 57 / 61 (their timing variants).  Exact, and measured slower on the
// one BASELINE scene that has screenable leaves (config 4: 85.2-85.4 vs 82.5-82.9 ms), so
// they live in librt_hip_exp.so and the mirror builds screen records only when rt_build_options
// leaf_screens asks for them.
#include "rt_fast_body.h"

namespace rtk {
namespace {
template <int STACK>
hipError_t dispatch(int mode, const RenderArgs& a, int waves, hipStream_t s) {
    switch (mode) {
        case 49: return launch_occ<STACK, false, 49>(a, waves, s);
        case 53: return launch_occ<STACK, false, 53>(a, waves, s);
        case 57: return launch_occ<STACK, false, 57>(a, waves, s);
        case 61: return launch_occ<STACK, false, 61>(a, waves, s);
    }
    return hipErrorInvalidValue;
}
}  // namespace

RT_FAST_FAMILY(launch_fast_screen, dispatch)

}  // namespace rtk
