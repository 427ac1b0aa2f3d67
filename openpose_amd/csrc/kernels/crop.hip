// crop.hip -- the MaximumCaffe stage of face / hand keypoint extraction on gfx950.
//
// op::FaceExtractorCaffe / op::HandExtractorCaffe (faceExtractorCaffe.cpp:210-280,
// handExtractorCaffe.cpp:140-200) resize each crop's net output x8 (ResizeAndMergeCaffe, CPU path =
// cv::resize INTER_CUBIC) and take, per part channel, the location and value of its maximum
// (MaximumCaffe -> maximumCpu, maximumBase.cpp:8-42: cv::minMaxLoc, the first maximum in raster
// order).  Here the resized values are evaluated lazily (heat_dev.h, bit-identical to resize.hip)
// and reduced in the same kernel: one workgroup per (crop, part), lanes stride the pixels, ties go
// to the smaller raster index.  VALU-bound (16-tap cubic per pixel), no HBM stack is written.
#include "kernels.h"
#include "heat_dev.h"
#include "../common.h"

namespace opk {

namespace {

__device__ __forceinline__ bool better(float v, int i, float bv, int bi)
{
    return v > bv || (v == bv && i < bi);
}

__global__ __launch_bounds__(256) void heat_argmax_kernel(float* __restrict__ peaks, HeatMap M,
                                                          int parts)
{
    __shared__ float sv[256];
    __shared__ int si[256];
    const int crop = blockIdx.x / parts, part = blockIdx.x - (blockIdx.x / parts) * parts;
    const int plane = crop * M.channels + part;
    const int hw = M.h * M.w;
    float bv = -__builtin_inff();
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < hw; i += blockDim.x) {
        const int y = i / M.w, x = i - y * M.w;
        const float v = heat_at(M, plane, x, y);
        if (better(v, i, bv, bi)) {
            bv = v;
            bi = i;
        }
    }
    sv[threadIdx.x] = bv;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int off = blockDim.x / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off && better(sv[threadIdx.x + off], si[threadIdx.x + off], sv[threadIdx.x],
                                             si[threadIdx.x])) {
            sv[threadIdx.x] = sv[threadIdx.x + off];
            si[threadIdx.x] = si[threadIdx.x + off];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        float* p = peaks + ((size_t)crop * parts + part) * 3;
        const int i = si[0];
        p[0] = (float)(i % M.w);
        p[1] = (float)(i / M.w);
        p[2] = sv[0];
    }
}

}  // namespace

// per-crop heat maps of FaceExtractorCaffe / HandExtractorCaffe (updateFaceHeatMapsForPerson,
// faceExtractorCaffe.cpp:42-75; updateHandHeatMapsForPerson, handExtractorCaffe.cpp:126-160): the
// first `parts` channels of the crop's x8 resize, through the heat-map ScaleMode -- PlusMinusOne(
// FixedAspect): fastTruncate(v) * 2 - 1; UnsignedChar: (float)positiveIntRound(fastTruncate(v) *
// 255); any other mode: fastTruncate(v) -- into dst[slot[crop]]; crops with slot -1 are skipped
__global__ __launch_bounds__(256) void crop_heatmaps_kernel(float* __restrict__ dst, const HeatMap M,
                                                            const int* __restrict__ slot, int parts,
                                                            int scale_mode)
{
    const int crop = blockIdx.z, part = blockIdx.y;
    const int sl = slot[crop];
    if (sl < 0) return;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int hw = M.h * M.w;
    if (i >= hw) return;
    const int y = i / M.w, x = i - y * M.w;
    const float v = heat_at(M, crop * M.channels + part, x, y);
    const float m = 0.f > v ? 0.f : v;           // fastTruncate(v, 0, 1) = fastMin(1, fastMax(0, v))
    const float t = 1.f < m ? 1.f : m;
    float o;
    if (scale_mode == 5 || scale_mode == 6) o = t * 2.f - 1.f;
    else if (scale_mode == 7) o = (float)(int)(t * 255.f + 0.5f);
    else o = t;
    dst[((size_t)sl * parts + part) * hw + i] = o;
}

void launch_crop_heatmaps(float* dst, const HeatMap& heat, const int* slot_dev, int crops, int parts,
                          int scale_mode, hipStream_t stream)
{
    OPK_CHECK_ARG(crops > 0 && parts > 0 && parts <= heat.channels, "bad crops / parts");
    const long hw = (long)heat.h * heat.w;
    OPK_CHECK_ARG(hw < (1L << 31), "heat map too large");
    hipLaunchKernelGGL(crop_heatmaps_kernel, dim3((unsigned)((hw + 255) / 256), parts, crops), dim3(256),
                       0, stream, dst, heat, slot_dev, parts, scale_mode);
    OPK_LAUNCH_CHECK();
}

void launch_heat_argmax(float* peaks, const HeatMap& heat, int crops, int parts, hipStream_t stream)
{
    OPK_CHECK_ARG(crops > 0 && parts > 0 && parts <= heat.channels, "bad crops / parts");
    OPK_CHECK_ARG((long)heat.h * heat.w < (1L << 31), "heat map too large");
    hipLaunchKernelGGL(heat_argmax_kernel, dim3((unsigned)(crops * parts)), dim3(256), 0, stream,
                       peaks, heat, parts);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
