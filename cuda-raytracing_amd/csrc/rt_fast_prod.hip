// rt_fast_prod.hip -- the production variants of the render kernel: MODE 17 (split small steps, pair
// records; scenes without leaf trees) and 21 (the same with leaf trees), at 5 and 6 waves per SIMD.
#include "rt_fast_body.h"

namespace rtk {
namespace {
template <int STACK>
hipError_t dispatch(int mode, const RenderArgs& a, int waves, hipStream_t s) {
    switch (mode) {
        case 17: return launch_occ<STACK, false, 17>(a, waves, s);
        case 21: return launch_occ<STACK, false, 21>(a, waves, s);
    }
    return hipErrorInvalidValue;
}
}  // namespace

RT_FAST_FAMILY(launch_fast_prod, dispatch)

}  // namespace rtk
