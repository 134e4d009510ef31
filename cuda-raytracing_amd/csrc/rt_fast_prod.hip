// rt_fast_prod.hip -- the production variants of the render kernel: MODE 17 (split small steps, pair
// records; scenes without leaf trees) and 21 (the same with leaf trees), each built for 5, 6 and 7 waves
// per SIMD (rt_fast_body.h render_fast_kernel_w5 / _w6 / _w7; bench.py's occupancy probe picks one --
// config 2 runs render_fast_kernel_w7<30, false, 17>).
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
