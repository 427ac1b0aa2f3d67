// pool.hip -- Caffe PoolingLayer MAX 2x2 / stride 2 (ceil sizing) on the padded NHWC fp16 images
// of the net (netCaffe.cpp:248 runs it inside caffe::Net::ForwardFrom; BODY_25 pool1_stage1,
// pool2_stage1, pool3_stage1).  HBM-bound: each lane reads up to four 16-byte pieces (8 channels)
// and writes one; no LDS.
#include "conv.h"

#include "../common.h"

namespace opk {

namespace {

// max of two fp16 pairs, first operand kept on ties / NaN (Caffe's `>` comparison)
__device__ __forceinline__ uint32_t hmax2(uint32_t a, uint32_t b)
{
    const _Float16 a0 = __builtin_bit_cast(_Float16, (uint16_t)(a & 0xffff));
    const _Float16 a1 = __builtin_bit_cast(_Float16, (uint16_t)(a >> 16));
    const _Float16 b0 = __builtin_bit_cast(_Float16, (uint16_t)(b & 0xffff));
    const _Float16 b1 = __builtin_bit_cast(_Float16, (uint16_t)(b >> 16));
    const uint16_t r0 = __builtin_bit_cast(uint16_t, (float)b0 > (float)a0 ? b0 : a0);
    const uint16_t r1 = __builtin_bit_cast(uint16_t, (float)b1 > (float)a1 ? b1 : a1);
    return r0 | ((uint32_t)r1 << 16);
}

__global__ __launch_bounds__(256) void maxpool2_kernel(uint16_t* __restrict__ out,
                                                       const uint16_t* __restrict__ in,
                                                       int frames, int H, int W, int C, int OH,
                                                       int OW, int B)
{
    const int c8 = C / 8;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)frames * OH * OW * c8;
    if (idx >= total) return;
    const int g = (int)(idx % c8);
    const int ox = (int)((idx / c8) % OW);
    const int oy = (int)((idx / ((size_t)c8 * OW)) % OH);
    const int f = (int)(idx / ((size_t)c8 * OW * OH));
    const int y0 = 2 * oy, x0 = 2 * ox;
    const int y1 = min(y0 + 2, H), x1 = min(x0 + 2, W);
    uint4 m;
    bool first = true;
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            const size_t pos = ((size_t)f * (H + 2 * B) + y + B) * (W + 2 * B) + x + B;
            const uint4 v = *reinterpret_cast<const uint4*>(in + pos * C + g * 8);
            if (first) { m = v; first = false; }
            else {
                m.x = hmax2(m.x, v.x);
                m.y = hmax2(m.y, v.y);
                m.z = hmax2(m.z, v.z);
                m.w = hmax2(m.w, v.w);
            }
        }
    const size_t opos = ((size_t)f * (OH + 2 * B) + oy + B) * (OW + 2 * B) + ox + B;
    *reinterpret_cast<uint4*>(out + opos * C + g * 8) = m;
}

// split precision: per channel the (hi, lo) pair of the pixel with the largest hi + lo (the
// first on ties, as Caffe's ordered `>`); hi + lo of an fp16 pair is exact in fp32
__global__ __launch_bounds__(256) void maxpool2_split_kernel(uint16_t* __restrict__ out,
                                                             uint16_t* __restrict__ out_lo,
                                                             const uint16_t* __restrict__ in,
                                                             const uint16_t* __restrict__ in_lo,
                                                             int frames, int H, int W, int C, int OH,
                                                             int OW, int B)
{
    const int c8 = C / 8;
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)frames * OH * OW * c8;
    if (idx >= total) return;
    const int g = (int)(idx % c8);
    const int ox = (int)((idx / c8) % OW);
    const int oy = (int)((idx / ((size_t)c8 * OW)) % OH);
    const int f = (int)(idx / ((size_t)c8 * OW * OH));
    const int y0 = 2 * oy, x0 = 2 * ox;
    const int y1 = min(y0 + 2, H), x1 = min(x0 + 2, W);
    uint16_t mh[8], ml[8];
    float mv[8];
    bool first = true;
    for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) {
            const size_t pos = ((size_t)f * (H + 2 * B) + y + B) * (W + 2 * B) + x + B;
            const uint4 vh = *reinterpret_cast<const uint4*>(in + pos * C + g * 8);
            const uint4 vl = *reinterpret_cast<const uint4*>(in_lo + pos * C + g * 8);
            const uint16_t* h = reinterpret_cast<const uint16_t*>(&vh);
            const uint16_t* l = reinterpret_cast<const uint16_t*>(&vl);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float v = (float)__builtin_bit_cast(_Float16, h[e]) + (float)__builtin_bit_cast(_Float16, l[e]);
                if (first || v > mv[e]) {
                    mv[e] = v;
                    mh[e] = h[e];
                    ml[e] = l[e];
                }
            }
            first = false;
        }
    const size_t opos = ((size_t)f * (OH + 2 * B) + oy + B) * (OW + 2 * B) + ox + B;
    *reinterpret_cast<uint4*>(out + opos * C + g * 8) = *reinterpret_cast<const uint4*>(mh);
    *reinterpret_cast<uint4*>(out_lo + opos * C + g * 8) = *reinterpret_cast<const uint4*>(ml);
}

}  // namespace

void launch_maxpool2_split(uint16_t* out, uint16_t* out_lo, const uint16_t* in, const uint16_t* in_lo,
                           int frames, int H, int W, int C, int OH, int OW, hipStream_t stream,
                           int border)
{
    OPK_CHECK_ARG(border >= 1, "border >= 1");
    OPK_CHECK_ARG(C % 8 == 0, "pool channels must be a multiple of 8");
    const size_t total = (size_t)frames * OH * OW * (C / 8);
    note_launch("maxpool2_split_kernel");
    hipLaunchKernelGGL(maxpool2_split_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       stream, out, out_lo, in, in_lo, frames, H, W, C, OH, OW, border);
    OPK_LAUNCH_CHECK();
}

void launch_maxpool2(uint16_t* out, const uint16_t* in, int frames, int H, int W, int C, int OH,
                     int OW, hipStream_t stream, int border)
{
    OPK_CHECK_ARG(border >= 1, "border >= 1");
    OPK_CHECK_ARG(C % 8 == 0, "pool channels must be a multiple of 8");
    const size_t total = (size_t)frames * OH * OW * (C / 8);
    note_launch("maxpool2_kernel");
    hipLaunchKernelGGL(maxpool2_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream,
                       out, in, frames, H, W, C, OH, OW, border);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
