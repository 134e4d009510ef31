// rt_fast_refill.hip -- refill variants (rt_render_params.refill_lanes: lanes take new pixels from a
// queue; measured slower, opt-in): MODE 81 and 85 (with leaf trees).
#include "rt_fast_body.h"

namespace rtk {
namespace {
template <int STACK>
hipError_t dispatch(int mode, const RenderArgs& a, int waves, hipStream_t s) {
    switch (mode) {
        case 81: return launch_occ<STACK, false, 81>(a, waves, s);
        case 85: return launch_occ<STACK, false, 85>(a, waves, s);
    }
    return hipErrorInvalidValue;
}
}  // namespace

RT_FAST_FAMILY(launch_fast_refill, dispatch)

}  // namespace rtk
