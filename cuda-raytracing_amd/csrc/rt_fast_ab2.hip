// rt_fast_ab2.hip -- A/B variants behind RT_TUNE bits 4-5 (tools/): big leaves 2 (scalar records only)
// and 0 (pair records in every big-leaf mode); reached through launch_fast_ab.
#include "rt_fast_body.h"

namespace rtk {
namespace {
template <int STACK>
hipError_t dispatch(int mode, const RenderArgs& a, int waves, hipStream_t s) {
    switch (mode) {
        case 2: return launch_occ<STACK, false, 2>(a, waves, s);
        case 0: return launch_occ<STACK, false, 0>(a, waves, s);
    }
    return hipErrorInvalidValue;
}
}  // namespace

RT_FAST_FAMILY(launch_fast_ab2, dispatch)

}  // namespace rtk
