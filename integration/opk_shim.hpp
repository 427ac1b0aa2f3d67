// opk_shim.hpp -- what the drop-in translation units (openpose_hip_shim.cpp, arrayCpuGpuHip.cpp)
// share: the calling thread's libopk context (one per Wrapper GPU worker thread, bound to the GPU
// that thread's NetHip / extractors initialised on; device 0 until one does).
//
// Contexts are shared-owned: the thread keeps one reference (released when the thread exits or
// re-binds to another GPU) and every object that allocated device memory or created a libopk
// object on a context keeps another, so the context outlives them all.  The reference's Wrapper
// joins its GPU worker threads BEFORE it destroys their PoseExtractor / Net objects
// (wrapperAuxiliary.hpp), so objects regularly die on another thread than the one that made them.
#pragma once
#include <memory>

#include "opk.h"

namespace op
{
    using OpkContext = std::shared_ptr<opk_ctx>;
    // the calling thread's context; device >= 0 binds the thread to that GPU (a new context when it
    // differs from the thread's current one -- objects holding the old one keep it alive)
    OpkContext opkShimThreadContext(int device = -2);
}
