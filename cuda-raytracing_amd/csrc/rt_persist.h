// rt_persist.h -- the persistent render kernel (rt_persist.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "rt_common.h"

// Render one frame (or shard) with the persistent wave-scheduled kernel on `stream`.
hipError_t rt_persistent_render(const rtk::RenderArgs& a, int tiles, int depth, bool stats, hipStream_t stream);
