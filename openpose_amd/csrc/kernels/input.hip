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

// The same warp with everything a workgroup reads staged in LDS first: the K source rows its
// destination row reads, over the column span the taps cover ([lo, hi) from the two ends of the
// affine x table), with 16-byte loads (A16: source, row step and frame step 16-byte aligned) or
// byte loads (out-of-image rows are not staged); the row's x table; and the 32 weight sets of its
// y fraction.  All of those loads are issued together behind one barrier, after which the taps
// read only LDS.  The direct kernel above chains two dependent global loads (x table, then
// weights) before each pixel's 3K^2 byte loads and reaches ~2.2 TB/s.  Same integer sums in the
// same order, so the output is bit-identical.
template <int K, bool A16>
__global__ __launch_bounds__(256) void cvmat_to_input_lds_kernel(
    float* __restrict__ dst, const uint8_t* __restrict__ src, int sh, int sw, size_t src_step,
    size_t src_frame, int dh, int dw, const int2* __restrict__ xtab, const int2* __restrict__ ytab,
    const short* __restrict__ wtab, int normalize, const int* __restrict__ frame_of, int tab_stride,
    int lds_row, int rows_at)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int2* xs = reinterpret_cast<int2*>(smem);                      // [dw]
    short* ws = reinterpret_cast<short*>(smem + (size_t)dw * 8);   // [32][K][K]
    uint8_t* rows = smem + rows_at;                                // [K][lds_row]
    const int y = blockIdx.x % dh;
    const int f = blockIdx.x / dh;
    xtab += (size_t)f * tab_stride;
    ytab += (size_t)f * tab_stride;
    const int2 yt = ytab[y];
    const int x_a = xtab[0].x, x_b = xtab[dw - 1].x;
    for (int x = threadIdx.x; x < dw; x += blockDim.x) xs[x] = xtab[x];
    for (int i = threadIdx.x; i < 32 * K * K; i += blockDim.x) ws[i] = wtab[yt.y * 32 * K * K + i];
    const int lo = max(min(x_a, x_b), 0), hi = min(max(x_a, x_b) + K, sw);   // source columns
    const uint8_t* fsrc = src + (size_t)(frame_of ? frame_of[f] : f) * src_frame;
    const int b0 = A16 ? (lo * 3) & ~15 : lo * 3;          // first staged byte of a row
    const int b1 = hi > lo ? hi * 3 : b0;                  // one past the last needed byte
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
        const int yy = yt.x + ky;
        if (yy < 0 || yy >= sh) continue;   // never read: the taps test the row below
        uint8_t* l = rows + ky * lds_row;
        const uint8_t* row = fsrc + (size_t)yy * src_step;
        if (A16) {
            const int full = (b1 - b0) >> 4;   // whole 16-byte pieces (b1 <= 3 sw: inside the row)
            const uint4* g = reinterpret_cast<const uint4*>(row + b0);
            uint4* d = reinterpret_cast<uint4*>(l);
            for (int i = threadIdx.x; i < full; i += blockDim.x) d[i] = g[i];
            for (int j = b0 + full * 16 + threadIdx.x; j < b1; j += blockDim.x) l[j - b0] = row[j];
        } else {
            for (int j = b0 + threadIdx.x; j < b1; j += blockDim.x) l[j - b0] = row[j];
        }
    }
    __syncthreads();
    const size_t plane = (size_t)dh * dw;
    float* out = dst + (size_t)f * 3 * plane + (size_t)y * dw;
    for (int x = threadIdx.x; x < dw; x += blockDim.x) {
        const int2 xt = xs[x];
        const short* w = ws + xt.y * K * K;
        int acc[3] = {0, 0, 0};
#pragma unroll
        for (int ky = 0; ky < K; ++ky) {
            const int yy = yt.x + ky;
            const bool yin = yy >= 0 && yy < sh;
            const uint8_t* l = rows + ky * lds_row - b0;
#pragma unroll
            for (int kx = 0; kx < K; ++kx) {
                const int xx = xt.x + kx;
                const int wk = w[ky * K + kx];
                if (yin && xx >= 0 && xx < sw) {   // constant border: outside taps read 0
                    const uint8_t* p = l + xx * 3;
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
    // staged rows: the column span plus the 16-byte alignment slack, padded to a 4-byte multiple
    const int lds_row = ((sw * 3 + 32) + 15) & ~15;
    const size_t rows_at = ((size_t)dw * 8 + 64 * ksize * ksize + 15) & ~(size_t)15;
    const size_t lds = rows_at + (size_t)ksize * lds_row;   // x table, weight sets, source rows
    if (lds <= 64 * 1024) {
        const bool a16 = ((uintptr_t)src % 16 == 0) && src_step % 16 == 0 && frame % 16 == 0;
#define OPK_WARP_LDS(K_, A_)                                                                   \
    hipLaunchKernelGGL((cvmat_to_input_lds_kernel<K_, A_>), grid, dim3(threads), lds, stream, dst, \
                       src, sh, sw, src_step, frame, dh, dw, xt, yt, wtab, normalize, frame_of,  \
                       tab_stride, lds_row, (int)rows_at)
        if (ksize == 2) {
            if (a16) OPK_WARP_LDS(2, true); else OPK_WARP_LDS(2, false);
        } else {
            if (a16) OPK_WARP_LDS(4, true); else OPK_WARP_LDS(4, false);
        }
#undef OPK_WARP_LDS
        OPK_LAUNCH_CHECK();
        return;
    }
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
