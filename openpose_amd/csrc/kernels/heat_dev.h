// heat_dev.h -- device side of HeatMap (kernels.h): one full-resolution heat-map value, read from
// HBM or evaluated on the fly with the resize/merge arithmetic of resize.hip.
//
// cv::resize INTER_CUBIC numerics (resizeAndMergeBase.cpp:9-113 -> OpenCV 4.x): horizontal pass of
// the four source rows around the target row ((t0 + t1) + t2) + t3 with the column's coefficients
// (HResizeCubic), then the vertical combination of VResizeCubic: columns inside the whole 4-float
// vectors of OpenCV's SIMD kernel sum h0 b0 + (h1 b1 + (h2 b2 + h3 b3)) (VResizeCubicVec_32f,
// v_fma = mul + add on the SSE baseline), the tail columns (w % 4 of them) left to right;
// sources merged in order as v + acc, and the sum times (float)(1/N) for N > 1 (oracle/resize.c
// states the OpenCV text this follows).  Compiled with -ffp-contract=off everywhere it is used,
// so resize_merge_kernel, the NMS and the PAF scorer all produce the same bits for a pixel.
#pragma once
#include "kernels.h"

namespace opk {

__device__ __forceinline__ int heat_clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// horizontal pass of one source row at the output column whose first tap is x0
__device__ __forceinline__ float cubic_hpass(const float* row, int sw, int x0, const float* a)
{
    const float v0 = row[heat_clampi(x0 - 1, 0, sw - 1)];
    const float v1 = row[heat_clampi(x0, 0, sw - 1)];
    const float v2 = row[heat_clampi(x0 + 1, 0, sw - 1)];
    const float v3 = row[heat_clampi(x0 + 2, 0, sw - 1)];
    return v0 * a[0] + v1 * a[1] + v2 * a[2] + v3 * a[3];
}

// OpenCV's vertical SIMD width on the x86-64 SSE baseline (v_float32::nlanes of CV_SIMD128)
constexpr int kCvVResizeLanes = 4;

// VResizeCubic of one column: x < vec_end (= w - w % 4) is inside OpenCV's SIMD body
__device__ __forceinline__ float cubic_vpass(const float h[4], float b0, float b1, float b2, float b3,
                                             bool simd)
{
    if (simd) {
        const float t3 = h[3] * b3;
        const float t2 = h[2] * b2 + t3;
        const float t1 = h[1] * b1 + t2;
        return h[0] * b0 + t1;
    }
    return h[0] * b0 + h[1] * b1 + h[2] * b2 + h[3] * b3;
}

__device__ __forceinline__ bool cubic_simd_column(int x, int w)
{
    return x < w - w % kCvVResizeLanes;
}

// ---- CUDA-build semantics (HeatMap::cuda) ------------------------------------------------------
// cubicInterpolate (include/openpose_private/gpu/cuda.hu:111-123), the expression as written,
// every operation rounded separately (-ffp-contract=off; nvcc's own contraction is not pinned)
__device__ __forceinline__ float cuda_cubic(float v0, float v1, float v2, float v3, float dx)
{
    return (-0.5f * v0 + 1.5f * v1 - 1.5f * v2 + 0.5f * v3) * dx * dx * dx +
           (v0 - 2.5f * v1 + 2.f * v2 - 0.5f * v3) * dx * dx - 0.5f * (v0 - v2) * dx + v1;
}

// bicubicInterpolate with cubicSequentialData's clamped base (cuda.hu:92-109,125-145); the x8
// kernel resize8TimesKernel (resizeAndMergeBase.cu:105-140) reads the same four clamped rows and
// columns through its 5x5 shared window, so one function serves both
__device__ __forceinline__ float cuda_bicubic(const float* src, float xs, float ys, int sw, int sh)
{
    const int x1 = heat_clampi((int)floorf(xs), 0, sw - 1);
    const int xi[4] = {max(0, x1 - 1), x1, min(sw - 1, x1 + 1), min(sw - 1, min(sw - 1, x1 + 1) + 1)};
    const float dx = xs - (float)x1;
    const int y1 = heat_clampi((int)floorf(ys), 0, sh - 1);
    const int yi[4] = {max(0, y1 - 1), y1, min(sh - 1, y1 + 1), min(sh - 1, min(sh - 1, y1 + 1) + 1)};
    const float dy = ys - (float)y1;
    float t[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float* r = src + (size_t)yi[i] * sw;
        t[i] = cuda_cubic(r[xi[0]], r[xi[1]], r[xi[2]], r[xi[3]], dx);
    }
    return cuda_cubic(t[0], t[1], t[2], t[3], dy);
}

// one target pixel of resizeAndMergeGpu: x8 single source (resize8TimesKernel, source coordinate
// (x + 0.5f) / 8 - 0.5f), identity (fillKernel) or the multi-scale resizeAndAddAndAverageKernel
// (resizeAndMergeBase.cu:142-162: sum over sources in order, then / counter)
__device__ __forceinline__ float heat_at_cuda(const HeatMap& M, int plane, int x, int y)
{
    float acc = 0.f;
    for (int n = 0; n < M.nsrc; ++n) {
        const ResizeSource& S = M.src[n];
        const float* src = S.src + (size_t)plane * S.sh * S.sw;
        if (S.sx == 1.f && S.sy == 1.f && M.nsrc == 1) return src[(size_t)y * S.sw + x];
        const float xs = ((float)x + 0.5f) / S.sx - 0.5f;
        const float ys = ((float)y + 0.5f) / S.sy - 0.5f;
        acc += cuda_bicubic(src, xs, ys, S.sw, S.sh);
    }
    return M.nsrc > 1 ? acc / (float)M.nsrc : acc;
}

// value of plane `plane` (= frame * channels + channel) at full-resolution pixel (x, y)
__device__ __forceinline__ float heat_at(const HeatMap& M, int plane, int x, int y)
{
    if (M.heat) return M.heat[((size_t)plane * M.h + y) * M.w + x];
    if (M.cuda) return heat_at_cuda(M, plane, x, y);
    float acc = 0.f;
    for (int n = 0; n < M.nsrc; ++n) {
        const ResizeSource& S = M.src[n];
        const float* src = S.src + (size_t)plane * S.sh * S.sw;
        const int x0 = S.xofs[x];
        const float4 c = *reinterpret_cast<const float4*>(S.xcoef + 4 * x);
        const float a[4] = {c.x, c.y, c.z, c.w};
        const float4 b = *reinterpret_cast<const float4*>(S.ycoef + 4 * y);
        const int yb = S.yofs[y] - 1;
        float h[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            h[k] = cubic_hpass(src + (size_t)heat_clampi(yb + k, 0, S.sh - 1) * S.sw, S.sw, x0, a);
        const float v = cubic_vpass(h, b.x, b.y, b.z, b.w, cubic_simd_column(x, M.w));
        acc = (n == 0) ? v : v + acc;
    }
    return M.nsrc > 1 ? acc * M.inv_n : acc;
}

}  // namespace opk
