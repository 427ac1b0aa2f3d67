// opk_shim.hpp -- what the drop-in translation units (openpose_hip_shim.cpp, arrayCpuGpuHip.cpp)
// share: the calling thread's libopk context (one per Wrapper GPU worker thread, bound to the GPU
// that thread's NetHip / extractors initialised on; device 0 until one does).
#pragma once
#include "opk.h"

namespace op
{
    opk_ctx* opkShimThreadContext();
}
