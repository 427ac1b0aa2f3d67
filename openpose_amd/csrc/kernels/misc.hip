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
}  // namespace

void launch_add_inplace(float* dst, const float* src, size_t n, hipStream_t stream)
{
    if (n == 0) return;
    const size_t blocks = std::min<size_t>((n / 4 + 255) / 256 + 1, 4096);
    hipLaunchKernelGGL(add_inplace_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, dst, src, n);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
