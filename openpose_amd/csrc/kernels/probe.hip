// probe.hip -- measured ceilings behind bench.py's rooflines (no reference counterpart; SURVEY.md
// §8d asks for the vendor peaks to be confirmed on the box).
//
// mfma_peak_kernel: v_mfma_f32_16x16x32_f16 -- the conv kernels' instruction -- from registers, 8
// independent accumulator chains per wave, consecutive MFMAs on different operand pairs (as in the
// conv loops), 4 waves per SIMD; operands uniform random or all zero.  The random / zero gap is the
// clock the chip holds under switching load.
// hbm_read_kernel: 16-byte non-temporal streaming reads over a buffer far larger than the caches.
#include "kernels.h"
#include "../common.h"

namespace opk {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float vf4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void mfma_peak_kernel(const half8_t* __restrict__ in,
                                                        float* __restrict__ out, int iters)
{
    const int lane = threadIdx.x & 63;
    half8_t a[4], b[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = in[k * 64 + lane];
#pragma unroll
    for (int k = 0; k < 2; ++k) b[k] = in[(4 + k) * 64 + lane];
    vf4 acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = vf4{0.f, 0.f, 0.f, 0.f};
    // hand-placed: the loop is the 16 MFMAs and the branch
    for (int i = 0; i < iters; i += 2) {
        asm volatile(
            "v_mfma_f32_16x16x32_f16 %0, %8, %12, %0\n"
            "v_mfma_f32_16x16x32_f16 %1, %9, %12, %1\n"
            "v_mfma_f32_16x16x32_f16 %2, %10, %12, %2\n"
            "v_mfma_f32_16x16x32_f16 %3, %11, %12, %3\n"
            "v_mfma_f32_16x16x32_f16 %4, %8, %13, %4\n"
            "v_mfma_f32_16x16x32_f16 %5, %9, %13, %5\n"
            "v_mfma_f32_16x16x32_f16 %6, %10, %13, %6\n"
            "v_mfma_f32_16x16x32_f16 %7, %11, %13, %7\n"
            "v_mfma_f32_16x16x32_f16 %0, %9, %13, %0\n"
            "v_mfma_f32_16x16x32_f16 %1, %10, %13, %1\n"
            "v_mfma_f32_16x16x32_f16 %2, %11, %13, %2\n"
            "v_mfma_f32_16x16x32_f16 %3, %8, %13, %3\n"
            "v_mfma_f32_16x16x32_f16 %4, %9, %12, %4\n"
            "v_mfma_f32_16x16x32_f16 %5, %10, %12, %5\n"
            "v_mfma_f32_16x16x32_f16 %6, %11, %12, %6\n"
            "v_mfma_f32_16x16x32_f16 %7, %8, %12, %7\n"
            : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
              "+v"(acc[6]), "+v"(acc[7])
            : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(b[0]), "v"(b[1]));
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void hbm_read_kernel(const vf4* __restrict__ p, size_t n,
                                                       float* __restrict__ out)
{
    vf4 s = {0.f, 0.f, 0.f, 0.f};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        s += __builtin_nontemporal_load(p + i);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y + s.z + s.w;
}

}  // namespace

void launch_mfma_peak(const void* operands, float* out, int blocks, int iters, hipStream_t stream)
{
    OPK_CHECK_ARG(iters > 0 && iters % 2 == 0 && blocks > 0, "mfma probe: even iters, blocks > 0");
    mfma_peak_kernel<<<blocks, 256, 0, stream>>>(static_cast<const half8_t*>(operands), out, iters);
    OPK_LAUNCH_CHECK();
}

void launch_hbm_read(const void* buf, size_t bytes, float* out, int blocks, hipStream_t stream)
{
    hbm_read_kernel<<<blocks, 256, 0, stream>>>(static_cast<const vf4*>(buf), bytes / 16, out);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
