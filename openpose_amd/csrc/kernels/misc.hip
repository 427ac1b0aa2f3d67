// misc.hip -- small elementwise helpers.
#include "kernels.h"
#include "../common.h"

namespace opk {

namespace {
__global__ __launch_bounds__(256) void add_inplace_kernel(float* __restrict__ dst,
                                                          const float* __restrict__ src, size_t n)
{
    const size_t n4 = n / 4;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        float4 a = reinterpret_cast<float4*>(dst)[i];
        const float4 b = reinterpret_cast<const float4*>(src)[i];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        reinterpret_cast<float4*>(dst)[i] = a;
    }
    for (size_t i = n4 * 4 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        dst[i] += src[i];
}
// dev hook (POST_DELAY_US): one wave that holds its stream for `ticks` of the 100 MHz constant
// clock, so stream-ordering tests see a slow post-processing every time (bounded: the loop ends
// when the clock has advanced that far)
__global__ __launch_bounds__(64) void delay_kernel(unsigned long long ticks)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}
// element type conversion for the plugin functions' double instantiations (opk_convert): one
// rounding per element (double -> float round to nearest even, float -> double exact)
template <typename D, typename S>
__global__ __launch_bounds__(256) void convert_kernel(D* __restrict__ dst, const S* __restrict__ src, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        dst[i] = (D)src[i];
}
// getHeatMapsCopy's scaling (poseExtractorNet.cpp:106-244); ScaleMode values of
// include/openpose/core/enumClasses.hpp:6-17
constexpr int kZeroToOne = 3, kZeroToOneFixed = 4, kPlusMinusOne = 5, kPlusMinusOneFixed = 6,
              kUnsignedChar = 7, kNoScale = 8;

__device__ __forceinline__ float trunc01(float v, float lo)   // fastTruncate(v, lo, 1)
{
    const float m = lo > v ? lo : v;
    return 1.f < m ? 1.f : m;
}

// dst [frames][nsel][hw] <- heat [frames][channels][hw] at channels sel[c] (sel[nsel + c]: 0 = part or
// background, 1 = PAF), scaled as the reference does on the host
__global__ __launch_bounds__(256) void heat_copy_kernel(float* __restrict__ dst,
                                                        const float* __restrict__ heat,
                                                        const int* __restrict__ sel, int nsel,
                                                        int channels, size_t hw, int mode)
{
    const int c = blockIdx.y, f = blockIdx.z;
    const int src_c = sel[c], paf = sel[nsel + c];
    const float* s = heat + ((size_t)f * channels + src_c) * hw;
    float* d = dst + ((size_t)f * nsel + c) * hw;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < hw;
         i += (size_t)gridDim.x * blockDim.x) {
        float v = s[i];
        if (mode != kNoScale) {
            if (!paf) {
                const float t = trunc01(v, 0.f);
                if (mode == kPlusMinusOne || mode == kPlusMinusOneFixed) v = t * 2.f - 1.f;
                else if (mode == kUnsignedChar) v = (float)(int)(t * 255.f + 0.5f);
                else v = t;
            } else {
                const float t = trunc01(v, -1.f);
                if (mode == kZeroToOne || mode == kZeroToOneFixed) v = t * 0.5f + 0.5f;
                else if (mode == kUnsignedChar) v = (float)(int)(t * 128.5f + 128.5f + 0.5f);
                else v = t;
            }
        }
        d[i] = v;
    }
}
}  // namespace

void launch_heat_copy(float* dst, const float* heat, const int* sel_dev, int nsel, int frames,
                      int channels, size_t hw, int scale_mode, hipStream_t stream)
{
    if (nsel == 0 || frames == 0) return;
    const unsigned bx = (unsigned)std::min<size_t>((hw + 255) / 256, 64);
    hipLaunchKernelGGL(heat_copy_kernel, dim3(bx, nsel, frames), dim3(256), 0, stream, dst, heat,
                       sel_dev, nsel, channels, hw, scale_mode);
    OPK_LAUNCH_CHECK();
}

void launch_delay(int microseconds, hipStream_t stream)
{
    OPK_CHECK_ARG(microseconds >= 0 && microseconds <= 1000000, "delay: 0 .. 1 s");
    hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, stream, (unsigned long long)microseconds * 100ull);
    OPK_LAUNCH_CHECK();
}

void launch_add_inplace(float* dst, const float* src, size_t n, hipStream_t stream)
{
    if (n == 0) return;
    const size_t blocks = std::min<size_t>((n / 4 + 255) / 256 + 1, 4096);
    hipLaunchKernelGGL(add_inplace_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, dst, src, n);
    OPK_LAUNCH_CHECK();
}

template <typename D, typename S>
static void launch_convert(D* dst, const S* src, size_t n, hipStream_t stream)
{
    if (n == 0) return;
    const size_t blocks = std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL((convert_kernel<D, S>), dim3((unsigned)blocks), dim3(256), 0, stream, dst, src, n);
    OPK_LAUNCH_CHECK();
}

void launch_f64_to_f32(float* dst, const double* src, size_t n, hipStream_t stream)
{
    launch_convert(dst, src, n, stream);
}

void launch_f32_to_f64(double* dst, const float* src, size_t n, hipStream_t stream)
{
    launch_convert(dst, src, n, stream);
}

}  // namespace opk
