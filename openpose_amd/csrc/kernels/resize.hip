// resize.hip -- bicubic resize + multi-scale merge for gfx950 with resizeAndMergeCpu numerics.
//
// Replaces op::resizeAndMergeGpu (src/openpose/net/resizeAndMergeBase.cu:274-528) but computes
// what the CPU path computes (resizeAndMergeBase.cpp:9-113 -> cv::resize INTER_CUBIC, A = -0.75,
// replicate border, horizontal pass then vertical pass; multi-scale: sum of per-source resizes
// in source order, times (float)(1/N)).  Tap offsets/coefficients come from host tables built
// exactly like OpenCV's (host/resize_tables.cpp), so every output equals the oracle's bit for bit
// (file compiled with -ffp-contract=off: every mul/add rounds separately, as on the x86 CPU path).
//
// HBM-bound: per frame (config 2) 1.18 MB read, 75.3 MB written.  One workgroup = 16 output rows
// x 256 output columns of one plane; each lane owns one column: it evaluates the horizontal pass
// once per source row of the tile's footprint (<= 6 rows at x8), parks those values in its own
// LDS column, then forms the 16 vertical combinations.  Stores are row-contiguous (1 KiB per wave
// instruction); source reads hit L1/L2 (the net output is 1.2 MB per frame).
#include "kernels.h"
#include "heat_dev.h"
#include "../common.h"

namespace opk {

namespace {

constexpr int TX = 256;     // output columns per workgroup (one per lane)
constexpr int TY = 16;      // output rows per workgroup
constexpr int MAXR = 16;    // footprint rows kept in LDS

struct ResizeArgs {
    ResizeSource s[kMaxResizeSources];
    int nsrc;
    int dh, dw;
    float inv_n;
};

__global__ __launch_bounds__(TX) void resize_merge_kernel(float* __restrict__ dst, ResizeArgs args)
{
    __shared__ float hbuf[MAXR * TX];
    const int tx = threadIdx.x;
    const int x = blockIdx.x * TX + tx;
    const int y0 = blockIdx.y * TY;
    const int plane = blockIdx.z;
    const int dh = args.dh, dw = args.dw;
    const int y1 = min(y0 + TY, dh);
    float acc[TY];

    for (int n = 0; n < args.nsrc; ++n) {
        const ResizeSource& S = args.s[n];
        const float* src = S.src + (size_t)plane * S.sh * S.sw;
        const int r_lo = heat_clampi(S.yofs[y0] - 1, 0, S.sh - 1);
        const int r_hi = heat_clampi(S.yofs[y1 - 1] + 2, 0, S.sh - 1);
        const int nrows = r_hi - r_lo + 1;
        int x0 = 0;
        float a[4] = {0.f, 0.f, 0.f, 0.f};
        if (x < dw) {
            x0 = S.xofs[x];
            const float4 c = *reinterpret_cast<const float4*>(S.xcoef + 4 * x);
            a[0] = c.x; a[1] = c.y; a[2] = c.z; a[3] = c.w;
        }
        const bool tiled = nrows <= MAXR;   // block-uniform
        if (tiled && x < dw)
            for (int r = 0; r < nrows; ++r)
                hbuf[r * TX + tx] = cubic_hpass(src + (size_t)(r_lo + r) * S.sw, S.sw, x0, a);
#pragma unroll
        for (int j = 0; j < TY; ++j) {
            const int y = y0 + j;
            float v = 0.f;
            if (y < y1 && x < dw) {
                const float4 b = *reinterpret_cast<const float4*>(S.ycoef + 4 * y);
                const int yb = S.yofs[y] - 1;
                float h[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int r = heat_clampi(yb + k, 0, S.sh - 1);
                    h[k] = tiled ? hbuf[(r - r_lo) * TX + tx]
                                 : cubic_hpass(src + (size_t)r * S.sw, S.sw, x0, a);
                }
                v = cubic_vpass(h, b.x, b.y, b.z, b.w, cubic_simd_column(x, dw));
            }
            acc[j] = (n == 0) ? v : v + acc[j];
        }
    }
    if (x >= dw) return;
    float* out = dst + (size_t)plane * dh * dw + x;
#pragma unroll
    for (int j = 0; j < TY; ++j) {
        const int y = y0 + j;
        if (y < y1) out[(size_t)y * dw] = (args.nsrc > 1) ? acc[j] * args.inv_n : acc[j];
    }
}

// CUDA-build semantics (HeatMap::cuda): one lane per target pixel, heat_at_cuda
__global__ __launch_bounds__(256) void resize_merge_cuda_kernel(float* __restrict__ dst, const HeatMap M)
{
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int plane = blockIdx.z;
    if (x >= M.w || y >= M.h) return;
    dst[((size_t)plane * M.h + y) * M.w + x] = heat_at_cuda(M, plane, x, y);
}

}  // namespace

void launch_resize_merge_cuda(float* dst, const HeatMap& M, int planes, hipStream_t stream)
{
    OPK_CHECK_ARG(M.cuda && !M.heat && M.nsrc >= 1 && M.nsrc <= kMaxResizeSources,
                  "CUDA-semantics resize: 1..8 lazy sources");
    OPK_CHECK_ARG(planes > 0 && M.h > 0 && M.w > 0, "empty target");
    dim3 grid((M.w + 63) / 64, (M.h + 3) / 4, planes);
    hipLaunchKernelGGL(resize_merge_cuda_kernel, grid, dim3(256), 0, stream, dst, M);
    OPK_LAUNCH_CHECK();
}

void launch_resize_merge(float* dst, const ResizeSource* srcs, int nsrc, int planes, int dh,
                         int dw, hipStream_t stream)
{
    OPK_CHECK_ARG(nsrc >= 1 && nsrc <= kMaxResizeSources, "1..8 sources supported");
    OPK_CHECK_ARG(planes > 0 && dh > 0 && dw > 0, "empty target");
    ResizeArgs a{};
    for (int i = 0; i < nsrc; ++i) a.s[i] = srcs[i];
    a.nsrc = nsrc;
    a.dh = dh;
    a.dw = dw;
    a.inv_n = (float)(1. / (double)nsrc);
    dim3 grid((dw + TX - 1) / TX, (dh + TY - 1) / TY, planes);
    hipLaunchKernelGGL(resize_merge_kernel, grid, dim3(TX), 0, stream, dst, a);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
