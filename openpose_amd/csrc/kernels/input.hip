// input.hip -- frame -> net input on the GPU (op::CvMatToOpInput::createArray, CPU branch,
// src/openpose/core/cvMatToOpInput.cpp:63-98): resizeFixedAspectRatio's cv::warpAffine
// (openCvPrivate.cpp:34-52; INTER_AREA -> INTER_LINEAR for scales <= 1, INTER_CUBIC above, constant
// 0 border) followed by uCharCvMatToFloatPtr (openCv.cpp:57-150: BGR HWC uint8 -> CHW float,
// u / 256 - 0.5).
//
// OpenCV's 8-bit warp is integer arithmetic once the per-axis source taps / 5-bit fractions and the
// fixed-point 2-D weight table are known; the host builds both exactly as OpenCV does
// (host/input.cpp) and this kernel only gathers taps and sums integers, so the result is
// bit-identical to the CPU path by construction.  HBM-bound: 2.76 MB read + 2.90 MB written per
// 1280x720 -> 656x368 frame.
#include "kernels.h"
#include "../common.h"

namespace opk {

namespace {

// one workgroup per (frame, destination row); lanes stride the row, every channel plane is written
// with coalesced 4-byte stores
// Output image f reads source frame frame_of[f] (f when frame_of is NULL) with the tables at
// xtab + f * tab_stride, ytab + f * tab_stride (tab_stride 0: one table pair for every image).
template <int K>
__global__ __launch_bounds__(256) void cvmat_to_input_kernel(
    float* __restrict__ dst, const uint8_t* __restrict__ src, int sh, int sw, size_t src_step,
    size_t src_frame, int dh, int dw, const int2* __restrict__ xtab, const int2* __restrict__ ytab,
    const short* __restrict__ wtab, int normalize, const int* __restrict__ frame_of, int tab_stride)
{
    const int y = blockIdx.x % dh;
    const int f = blockIdx.x / dh;
    xtab += (size_t)f * tab_stride;
    ytab += (size_t)f * tab_stride;
    const int2 yt = ytab[y];                      // (first tap row, fraction index)
    const uint8_t* fsrc = src + (size_t)(frame_of ? frame_of[f] : f) * src_frame;
    const size_t plane = (size_t)dh * dw;
    float* out = dst + (size_t)f * 3 * plane + (size_t)y * dw;
    for (int x = threadIdx.x; x < dw; x += blockDim.x) {
        const int2 xt = xtab[x];
        const short* w = wtab + (yt.y * 32 + xt.y) * K * K;
        int acc[3] = {0, 0, 0};
#pragma unroll
        for (int ky = 0; ky < K; ++ky) {
            const int yy = yt.x + ky;
            const bool yin = yy >= 0 && yy < sh;
            const uint8_t* row = fsrc + (size_t)(yin ? yy : 0) * src_step;
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const int xx = xt.x + kx;
                const int wk = w[ky * K + kx];
                if (yin && xx >= 0 && xx < sw) {   // constant border: outside taps read 0
                    const uint8_t* p = row + (size_t)xx * 3;
                    acc[0] += (int)p[0] * wk;
                    acc[1] += (int)p[1] * wk;
                    acc[2] += (int)p[2] * wk;
                }
            }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            int u = (acc[c] + (1 << 14)) >> 15;   // FixedPtCast<int, uchar, 15>
            u = u < 0 ? 0 : (u > 255 ? 255 : u);
            float v = (float)u;
            if (normalize) v = v * (1.f / 256.f) - 0.5f;   // exact for u in [0, 255]
            out[(size_t)c * plane + x] = v;
        }
    }
}

}  // namespace

void launch_cvmat_to_input(float* dst, const uint8_t* src, int n, int sh, int sw, size_t src_step,
                           int dh, int dw, const int* xtab, const int* ytab, const short* wtab,
                           int ksize, int normalize, hipStream_t stream, const int* frame_of,
                           int tab_stride)
{
    OPK_CHECK_ARG(n > 0 && sh > 0 && sw > 0 && dh > 0 && dw > 0, "empty frame");
    OPK_CHECK_ARG(src_step >= (size_t)sw * 3, "row step shorter than the row");
    OPK_CHECK_ARG(ksize == 2 || ksize == 4, "linear or cubic");
    OPK_CHECK_ARG((long)n * dh < (1L << 31), "too many rows");
    const dim3 grid((unsigned)(n * dh));
    const int threads = dw >= 256 ? 256 : (dw >= 128 ? 128 : 64);
    const auto* xt = reinterpret_cast<const int2*>(xtab);
    const auto* yt = reinterpret_cast<const int2*>(ytab);
    const size_t frame = src_step * sh;
    if (ksize == 2)
        hipLaunchKernelGGL(cvmat_to_input_kernel<2>, grid, dim3(threads), 0, stream, dst, src, sh,
                           sw, src_step, frame, dh, dw, xt, yt, wtab, normalize, frame_of,
                           tab_stride);
    else
        hipLaunchKernelGGL(cvmat_to_input_kernel<4>, grid, dim3(threads), 0, stream, dst, src, sh,
                           sw, src_step, frame, dh, dw, xt, yt, wtab, normalize, frame_of,
                           tab_stride);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
