// rt_fast_tl.hip -- the production and timing kernels with lone rays walked through the treelets
// (MODE bit 7, rt_fast.h lone_treelet; RT_TUNE bit 20): 145 / 149 (= 17 / 21 + 128) and their timing
// variants 153 / 157 (= 25 / 29 + 128).  Reached through launch_fast_tl (librt_hip_exp.so).
#include "rt_fast_body.h"

namespace rtk {
namespace {
template <int STACK>
hipError_t dispatch(int mode, const RenderArgs& a, int waves, hipStream_t s) {
    switch (mode) {
        case 145: return launch_occ<STACK, false, 145>(a, waves, s);
        case 149: return launch_occ<STACK, false, 149>(a, waves, s);
        case 153: return launch_occ<STACK, false, 153>(a, waves, s);
        case 157: return launch_occ<STACK, false, 157>(a, waves, s);
    }
    return hipErrorInvalidValue;
}
}  // namespace

RT_FAST_FAMILY(launch_fast_tl, dispatch)

}  // namespace rtk
