// rt_fast_stats.hip -- statistics variants (exact counts of the reference's traversal work on scalar
// records): MODE 2, and 6 through the leaf trees.
#include "rt_fast_body.h"

namespace rtk {
namespace {
template <int STACK>
hipError_t dispatch(int mode, const RenderArgs& a, int waves, hipStream_t s) {
    switch (mode) {
        case 2: return launch_occ<STACK, true, 2>(a, waves, s);
        case 6: return launch_occ<STACK, true, 6>(a, waves, s);
    }
    return hipErrorInvalidValue;
}
}  // namespace

RT_FAST_FAMILY(launch_fast_stats, dispatch)

}  // namespace rtk
