// conv.hip -- BODY_25 convolution layers on gfx950 matrix cores.
//
// Replaces the Caffe ConvolutionLayer + PReLULayer/ReLULayer + ConcatLayer work that
// op::NetCaffe::forwardPass runs (src/openpose/net/netCaffe.cpp:248, Caffe im2col + SGEMM / cuDNN)
// with one implicit-GEMM kernel per conv: no im2col buffer, bias + PReLU/ReLU fused in the
// epilogue, concat realised by writing into channel slices of the consumer's buffer (up to six
// destinations), optional fp32 NCHW copy for the net_output blob.
//
// Tiling (MFMA v_mfma_f32_16x16x32_f16, fp32 accumulate):
//   workgroup 256 lanes = 4 waves as 2 (M) x 2 (N); tile BM = 128 positions x BN channels;
//   BK = 64 (two 32-channel chunks of the tap-major K axis) per step, double-buffered LDS,
//   register-staged global loads of step s+1 in flight while step s runs on the MFMAs, one
//   barrier per step.  LDS rows are 128 B (64 fp16 of K); 16-byte pieces are XOR-swizzled by
//   (row & 7) so every ds_read_b128 fragment read is bank-conflict free (row-interleaved
//   8-piece permutation, MI355X_MICROARCH.md §LDS lane groups).
// Every 3x3 tap is a constant shift of the GEMM row index because M enumerates the padded image's
// positions (conv.h), so the A loads are plain contiguous 16-byte NHWC reads.
#include "conv.h"

#include "../common.h"

namespace opk {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float float4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int swz(int row, int piece) { return row * 8 + (piece ^ (row & 7)); }

__device__ __forceinline__ uint16_t f2h_bits(float v)
{
    const _Float16 h = (_Float16)v;
    return __builtin_bit_cast(uint16_t, h);
}

template <int BN>
__global__ __launch_bounds__(256, 2) void conv_kernel(const ConvArgs a)
{
    constexpr int BM = kConvBM;
    constexpr int WN = BN / 2;
    constexpr int NF = WN / 16;
    constexpr int MF = 4;
    constexpr int BP = BN / 32;            // B pieces per lane per step
    __shared__ uint4 lds[2][(BM + BN) * 8];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int p = tid & 7;
    const int rsub = tid >> 3;

    const int Wp = a.W + 2;
    const int per_frame = a.H * Wp;
    int abase[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int m = m0 + rsub + 32 * i;
        if (m >= a.M) m = a.M - 1;
        const int f = m / per_frame;
        abase[i] = m + f * 2 * Wp;
    }
    const int cpt = a.cin_pad >> 5;        // chunks per tap
    const int nchunks = a.ntaps * cpt;
    const int kpad = a.ksteps * 64;
    const uint16_t* in = a.in + a.in_coff + (p & 3) * 8;
    const uint16_t* wrow = a.w + (size_t)(n0 + rsub) * kpad + p * 8;

    uint4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3;
#define OPK_GLOAD(s_)                                                                         \
    do {                                                                                      \
        int c_ = 2 * (s_) + (p >> 2);                                                         \
        if (c_ >= nchunks) c_ = 0; /* zero weights cover the padded tail of K */              \
        const int tap_ = c_ / cpt;                                                            \
        const uint16_t* src_ = in + (c_ - tap_ * cpt) * 32 + (size_t)a.tapoff[tap_] * a.in_cs; \
        ra0 = *reinterpret_cast<const uint4*>(src_ + (size_t)abase[0] * a.in_cs);             \
        ra1 = *reinterpret_cast<const uint4*>(src_ + (size_t)abase[1] * a.in_cs);             \
        ra2 = *reinterpret_cast<const uint4*>(src_ + (size_t)abase[2] * a.in_cs);             \
        ra3 = *reinterpret_cast<const uint4*>(src_ + (size_t)abase[3] * a.in_cs);             \
        const uint16_t* w_ = wrow + (s_) * 64;                                                \
        rb0 = *reinterpret_cast<const uint4*>(w_);                                            \
        if constexpr (BP > 1) rb1 = *reinterpret_cast<const uint4*>(w_ + (size_t)32 * kpad);  \
        if constexpr (BP > 2) rb2 = *reinterpret_cast<const uint4*>(w_ + (size_t)64 * kpad);  \
        if constexpr (BP > 3) rb3 = *reinterpret_cast<const uint4*>(w_ + (size_t)96 * kpad);  \
    } while (0)
#define OPK_SWRITE(buf_)                                                                      \
    do {                                                                                      \
        lds[buf_][swz(rsub, p)] = ra0;                                                        \
        lds[buf_][swz(rsub + 32, p)] = ra1;                                                   \
        lds[buf_][swz(rsub + 64, p)] = ra2;                                                   \
        lds[buf_][swz(rsub + 96, p)] = ra3;                                                   \
        lds[buf_][BM * 8 + swz(rsub, p)] = rb0;                                               \
        if constexpr (BP > 1) lds[buf_][BM * 8 + swz(rsub + 32, p)] = rb1;                    \
        if constexpr (BP > 2) lds[buf_][BM * 8 + swz(rsub + 64, p)] = rb2;                    \
        if constexpr (BP > 3) lds[buf_][BM * 8 + swz(rsub + 96, p)] = rb3;                    \
    } while (0)

    float4_t acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

    OPK_GLOAD(0);
    OPK_SWRITE(0);
    __syncthreads();
    const int r16 = lane & 15, q = lane >> 4;
    for (int s = 0; s < a.ksteps; ++s) {
        const int cur = s & 1;
        if (s + 1 < a.ksteps) OPK_GLOAD(s + 1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            half8_t af[MF], bf[NF];
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                const uint4 v = lds[cur][swz(wm * 64 + i * 16 + r16, kk * 4 + q)];
                af[i] = __builtin_bit_cast(half8_t, v);
            }
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                const uint4 v = lds[cur][BM * 8 + swz(wn * WN + j * 16 + r16, kk * 4 + q)];
                bf[j] = __builtin_bit_cast(half8_t, v);
            }
#pragma unroll
            for (int i = 0; i < MF; ++i)
#pragma unroll
                for (int j = 0; j < NF; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0,
                                                                       0, 0);
        }
        if (s + 1 < a.ksteps) OPK_SWRITE(cur ^ 1);
        __syncthreads();
    }

#undef OPK_GLOAD
#undef OPK_SWRITE

    // ---- epilogue: bias + activation, fp16 NHWC stores (+ fp32 NCHW net_output) -----------
    float bias[NF], slope[NF];
    int co[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        co[j] = n0 + wn * WN + j * 16 + r16;
        const bool ok = co[j] < a.cout;
        bias[j] = ok ? a.bias[co[j]] : 0.f;
        slope[j] = (ok && a.act == 2) ? a.slope[co[j]] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * 64 + i * 16 + q * 4 + r;
            if (m >= a.M) continue;
            const int f = m / per_frame;
            const int rem = m - f * per_frame;
            const int y = rem / Wp;
            const int x = rem - y * Wp;
            if (x >= a.W) continue;
            const size_t pos = (size_t)m + (size_t)f * 2 * Wp + Wp + 1;
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                if (co[j] >= a.cout) continue;
                float v = acc[i][j][r] + bias[j];
                if (a.act == 1) v = v > 0.f ? v : 0.f;
                else if (a.act == 2) v = v > 0.f ? v : v * slope[j];
                const uint16_t hb = f2h_bits(v);
                for (int d = 0; d < a.ndst; ++d)
                    a.dst[d][pos * a.dst_cs[d] + a.dst_coff[d] + co[j]] = hb;
                if (a.out32)
                    a.out32[(((size_t)f * a.out32_c + a.out32_coff + co[j]) * a.H + y) * a.W + x] = v;
            }
        }
}

__global__ __launch_bounds__(256) void im2col3_kernel(uint16_t* __restrict__ out,
                                                      const float* __restrict__ in, int frames,
                                                      int H, int W)
{
    const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t total = (size_t)frames * H * W;
    if (idx >= total) return;
    const int x = (int)(idx % W);
    const int y = (int)((idx / W) % H);
    const int f = (int)(idx / ((size_t)W * H));
    const size_t plane = (size_t)H * W;
    const float* src = in + (size_t)f * 3 * plane;
    uint16_t v[32];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int yy = y + ky - 1, xx = x + kx - 1;
                const float s = (yy >= 0 && yy < H && xx >= 0 && xx < W)
                                    ? src[c * plane + (size_t)yy * W + xx] : 0.f;
                v[(ky * 3 + kx) * 3 + c] = f2h_bits(s);
            }
#pragma unroll
    for (int i = 27; i < 32; ++i) v[i] = 0;
    const size_t pos = ((size_t)f * (H + 2) + y + 1) * (W + 2) + x + 1;
    uint4* dst = reinterpret_cast<uint4*>(out + pos * 32);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint4 u;
        u.x = v[8 * k] | ((uint32_t)v[8 * k + 1] << 16);
        u.y = v[8 * k + 2] | ((uint32_t)v[8 * k + 3] << 16);
        u.z = v[8 * k + 4] | ((uint32_t)v[8 * k + 5] << 16);
        u.w = v[8 * k + 6] | ((uint32_t)v[8 * k + 7] << 16);
        dst[k] = u;
    }
}

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

}  // namespace

void launch_conv(const ConvArgs& a, int bn, hipStream_t stream)
{
    OPK_CHECK_ARG(a.cin_pad % 32 == 0 && a.cin_pad > 0, "cin_pad must be a multiple of 32");
    OPK_CHECK_ARG(a.in_cs % 8 == 0 && a.in_coff % 8 == 0, "input slice must be 16-byte aligned");
    OPK_CHECK_ARG(a.in_coff + a.cin_pad <= a.in_cs, "input slice exceeds the buffer");
    OPK_CHECK_ARG(a.ntaps == 1 || a.ntaps == 9, "1 or 9 taps");
    OPK_CHECK_ARG(a.ksteps * 64 >= a.ntaps * a.cin_pad, "ksteps too small");
    OPK_CHECK_ARG(a.M > 0 && a.cout > 0 && a.ndst >= 0 && a.ndst <= kConvMaxDst, "bad sizes");
    dim3 grid((a.M + kConvBM - 1) / kConvBM, (a.cout + bn - 1) / bn);
    switch (bn) {
        case 32: hipLaunchKernelGGL(conv_kernel<32>, grid, dim3(256), 0, stream, a); break;
        case 64: hipLaunchKernelGGL(conv_kernel<64>, grid, dim3(256), 0, stream, a); break;
        case 96: hipLaunchKernelGGL(conv_kernel<96>, grid, dim3(256), 0, stream, a); break;
        case 128: hipLaunchKernelGGL(conv_kernel<128>, grid, dim3(256), 0, stream, a); break;
        default: throw Error(1, "launch_conv: unsupported BN " + std::to_string(bn));
    }
    OPK_LAUNCH_CHECK();
}

void launch_im2col3(uint16_t* out, const float* in, int frames, int H, int W, hipStream_t stream)
{
    const size_t total = (size_t)frames * H * W;
    hipLaunchKernelGGL(im2col3_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream,
                       out, in, frames, H, W);
    OPK_LAUNCH_CHECK();
}

void launch_maxpool2(uint16_t* out, const uint16_t* in, int frames, int H, int W, int C, int OH,
                     int OW, hipStream_t stream, int border)
{
    OPK_CHECK_ARG(border >= 1, "border >= 1");
    OPK_CHECK_ARG(C % 8 == 0, "pool channels must be a multiple of 8");
    const size_t total = (size_t)frames * OH * OW * (C / 8);
    hipLaunchKernelGGL(maxpool2_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream,
                       out, in, frames, H, W, C, OH, OW, border);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
