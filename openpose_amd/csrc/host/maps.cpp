// maps.cpp -- resizeAndMergeGpu's geometry for the CUDA-semantics heat maps (maps.h).
#include "maps.h"

#include <cmath>
#include <string>

#include "../common.h"

namespace opk {

HeatMap cuda_heat_map(const float* const* src, const int* sh, const int* sw, int nsrc,
                      int channels, int th, int tw, const float* scale_ratios)
{
    // resizeAndMergeBase.cu:276-282
    OPK_CHECK_ARG(nsrc >= 1, "sourceSizes cannot be empty.");
    OPK_CHECK_ARG(nsrc <= kMaxResizeSources,
                  "More than 8 scales are not implemented (yet). Notify us to implement it.");
    OPK_CHECK_ARG(th > 0 && tw > 0 && channels > 0, "empty target");
    HeatMap m{};
    m.channels = channels;
    m.h = th;
    m.w = tw;
    m.nsrc = nsrc;
    m.inv_n = (float)(1. / (double)nsrc);
    m.cuda = 1;
    for (int i = 0; i < nsrc; ++i) {
        OPK_CHECK_ARG(src[i] != nullptr && sh[i] > 0 && sw[i] > 0, "empty source");
        m.src[i].src = src[i];
        m.src[i].sh = sh[i];
        m.src[i].sw = sw[i];
    }
    if (nsrc == 1) {
        if (tw / sw[0] == 1 && th / sh[0] == 1) {   // fillKernel: a plain copy
            OPK_CHECK_ARG(tw == sw[0] && th == sh[0],
                          "identity resize with different source and target sizes");
            m.src[0].sx = m.src[0].sy = 1.f;
        } else {
            OPK_CHECK_ARG(tw / sw[0] == 8 && th / sh[0] == 8,
                          "Kernel only implemented for 8x resize. Notify us if this error appears.");
            const float r = (float)(unsigned)std::ceil(th / (float)sh[0]);
            m.src[0].sx = m.src[0].sy = r;
        }
        return m;
    }
    OPK_CHECK_ARG(scale_ratios != nullptr, "multi-scale merge needs scaleInputToNetInputs");
    const float main_w = tw / (float)sw[0], main_h = th / (float)sh[0];
    for (int i = 0; i < nsrc; ++i) {
        const float s = scale_ratios[i] / scale_ratios[0];
        OPK_CHECK_ARG(s > 0.f && std::isfinite(s), "scale ratio " + std::to_string(i) + " invalid");
        m.src[i].sx = main_w / s;
        m.src[i].sy = main_h / s;
    }
    return m;
}

}  // namespace opk
