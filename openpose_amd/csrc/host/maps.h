// maps.h -- heat-map semantics (resize + NMS) of the reference's two builds (internal).
#pragma once
#include "../kernels/kernels.h"

namespace opk {

constexpr int kMapsCpu = 0;    // resizeAndMergeCpu + nmsCpu (OpenCV cubic A = -0.75, nmsCpu borders)
constexpr int kMapsCuda = 1;   // resizeAndMergeGpu + nmsGpu (Catmull-Rom, strict interior)

// The lazy HeatMap of resizeAndMergeGpu over `nsrc` net outputs [planes][sh[i]][sw[i]] at target
// th x tw, with its sanity checks and geometry (src/openpose/net/resizeAndMergeBase.cu):
//   one source: identity when the sizes agree (fillKernel), else only x8 (resize8TimesKernel,
//   source coordinate (x + 0.5) / ceil(th / sh) - 0.5 on both axes; other ratios are the
//   reference's "Kernel only implemented for 8x resize" error);
//   several: resizeAndAddAndAverageKernel, source i scaled by (tw / sw[0]) / (r[i] / r[0])
//   (r = scaleInputToNetInputs), at most 8 sources.
HeatMap cuda_heat_map(const float* const* src, const int* sh, const int* sw, int nsrc,
                      int channels, int th, int tw, const float* scale_ratios);

}  // namespace opk
