// conv_image.hip -- the first 3x3 convolution (3 -> <=64 channels) read straight from the fp32
// NCHW network input (the blob op::Net::forwardPass receives, netCaffe.cpp:248 / the Caffe
// "image" input), fused with bias + activation, written as padded NHWC fp16.
//
// K = 27 (3 taps x 3 taps x 3 channels) fits one 16x16x32 MFMA step, so the layer is pure data
// movement: read 12 B and write 128 B per pixel.  A block stages a (4+2) x (64+2) x 3 fp32 input
// tile in LDS; each lane gathers the 8 K-values of its MFMA operand from it (K order
// (ky*3 + kx)*3 + ci, zero past 27), the weights of all 64 output channels stay in registers,
// and the MFMAs compute C^T so each lane stores 4 consecutive output channels (8 bytes) of one
// pixel.  Replaces the im2col image + 1-step GEMM of conv.hip (two passes over HBM).
// SPLIT (ConvArgs::split, net.h kPrecisionSplit): the weight rows carry w_lo = fp16(w - w_hi) in
// their second 32 halves, each input value is split as x_hi = fp16(x), x_lo = fp16(x - x_hi) in
// the gather, the three products x_hi w_hi, x_lo w_hi, x_hi w_lo accumulate in that order (the
// pass order of conv3_kernel's split K loop), and the epilogue scales the sums by wscale (the
// weights are packed times 2^e, conv.h) and writes hi = fp16(v) and lo = fp16(v - hi) to dst / dst_lo.
#include "conv.h"

#include "../common.h"

namespace opk {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float float4_t __attribute__((ext_vector_type(4)));

constexpr int TH = 4;            // output rows per block (one per wave)
constexpr int TW = 64;           // output columns per block
constexpr int LW = TW + 2;       // staged columns
constexpr int NG = 4;            // 16-channel groups (cout <= 64)

__device__ __forceinline__ uint16_t f2h_bits_i(float v)
{
    const _Float16 h = (_Float16)v;
    return __builtin_bit_cast(uint16_t, h);
}

// WIDE: cout % 32 == 0 and 16-byte aligned slices -- fragment pairs (g, g+1) exchanged between
// lane rows q and q^1 by v_permlane16_swap (as conv3.hip's epilogues), so each lane stores 8
// consecutive channels (16 bytes) and a store instruction covers 64 contiguous bytes of 16 pixels
// instead of 32 (half the store instructions; same values)
// STAGE (WIDE only): each 16-pixel group's 16-byte pieces go through a per-wave LDS image first
// (piece column XOR-swizzled by the pixel) and leave as stores of 1 KiB contiguous per instruction
// -- 8 whole pixels of 128 bytes -- instead of 16 half lines of 64 bytes (CONV_IMAGE_STAGE, A/B)
template <bool SPLIT, bool WIDE, bool STAGE>
__global__ __launch_bounds__(256) void conv_image_kernel(const ConvArgs a, const float* __restrict__ img)
{
    __shared__ float tile[3 * (TH + 2) * LW];
    __shared__ uint4 ostage[STAGE ? TH : 1][SPLIT ? 2 : 1][STAGE ? 128 : 1];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // (uniform: row pointers in SGPRs)
    const int H = a.H, W = a.W, B = a.border > 0 ? a.border : 1;
    const int tiles_x = (W + TW - 1) / TW, tiles_y = (H + TH - 1) / TH;
    int b = blockIdx.x;
    const int tx = b % tiles_x;
    b /= tiles_x;
    const int ty = b % tiles_y;
    const int f = b / tiles_y;
    const int x0 = tx * TW, y0 = ty * TH;

    // stage the input tile (zero outside the image = the conv's zero padding)
    const size_t plane = (size_t)H * W;
    const float* src = img + (size_t)f * 3 * plane;
    for (int i = tid; i < 3 * (TH + 2) * LW; i += 256) {
        const int ci = i / ((TH + 2) * LW);
        const int rem = i - ci * (TH + 2) * LW;
        const int r = rem / LW, c = rem - (rem / LW) * LW;
        const int y = y0 + r - 1, x = x0 + c - 1;
        tile[i] = (y >= 0 && y < H && x >= 0 && x < W) ? src[ci * plane + (size_t)y * W + x] : 0.f;
    }

    const int r16 = lane & 15, q = lane >> 4;
    // weights (A operand of C^T): rows = output channels g*16 + r16, K = 8q .. 8q+7; row stride 64
    half8_t wf[NG], wl[NG];
    const float neg = a.act == 1 ? 0.f : 1.f;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int co = g * 16 + r16;
        wf[g] = co < a.cout ? *reinterpret_cast<const half8_t*>(a.w + (size_t)co * 64 + 8 * q)
                            : half8_t{0, 0, 0, 0, 0, 0, 0, 0};
        if constexpr (SPLIT)
            wl[g] = co < a.cout ? *reinterpret_cast<const half8_t*>(a.w + (size_t)co * 64 + 32 + 8 * q)
                                : half8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
    // bias / negative-side multipliers in LDS, read per fragment (in registers they held 32 VGPRs
    // and the split kernel to 3 waves per SIMD; bias/slope arrays are zero-padded to 128 channels)
    __shared__ float4_t sbias[16 * NG / 4], smul[16 * NG / 4];
    if (tid < 16 * NG / 4) {
        sbias[tid] = *reinterpret_cast<const float4_t*>(a.bias + 4 * tid);
        const float4_t sl = *reinterpret_cast<const float4_t*>(a.slope + 4 * tid);
        smul[tid] = a.act == 2 ? sl : float4_t{neg, neg, neg, neg};
    }
    // this lane's 8 K values: LDS offset of (ci, ky, kx) for k = 8q + e, or -1 past k = 26
    int off[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int k = 8 * q + e;
        const int t = k / 3, ci = k - 3 * (k / 3);
        off[e] = k < 27 ? (ci * (TH + 2) + t / 3) * LW + (t - 3 * (t / 3)) : -1;
    }
    __syncthreads();

    const int y = y0 + wave;
    if (y >= H) return;
    uint16_t* dbase[kConvMaxDst];
    uint16_t* dlo[kConvMaxDst];
    for (int d = 0; d < a.ndst; ++d) {
        const size_t o = ((size_t)f * (H + 2 * B) + y + B) * (W + 2 * B) * a.dst_cs[d] + a.dst_coff[d];
        dbase[d] = a.dst[d] + o;
        dlo[d] = SPLIT ? a.dst_lo[d] + o : nullptr;
    }
#pragma unroll
    for (int grp = 0; grp < TW / 16; ++grp) {
        const int xl = grp * 16 + r16;
        half8_t xf, xl8;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float xv = off[e] >= 0 ? tile[off[e] + wave * LW + xl] : 0.f;
            xf[e] = (_Float16)xv;
            if constexpr (SPLIT) xl8[e] = (_Float16)(xv - (float)xf[e]);
        }
        float4_t acc[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[g], xf, float4_t{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            if constexpr (SPLIT) {
                acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wf[g], xl8, acc[g], 0, 0, 0);
                acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[g], xf, acc[g], 0, 0, 0);
            }
        }
        const int x = x0 + xl;
        if constexpr (WIDE) {
            // lanes (r16, q) and (r16, q ^ 1) hold the same pixel: a column past W skips both
            // (STAGE: every lane writes its pieces; the stores skip the columns past W)
            if (!STAGE && x >= W) continue;
            const int cw = 16 * (q & 1) + 8 * (q >> 1);
#pragma unroll
            for (int g = 0; g < NG; g += 2) {
                if (g * 16 >= a.cout) break;
                uint32_t pk[2][2], pl[2][2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    float v[4];
                    const float4_t bq = sbias[(g + h) * 4 + q], mq = smul[(g + h) * 4 + q];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float t = (SPLIT ? acc[g + h][r] * a.wscale : acc[g + h][r]) + bq[r];
                        v[r] = t > 0.f ? t : t * mq[r];
                    }
                    pk[h][0] = (uint32_t)f2h_bits_i(v[0]) | ((uint32_t)f2h_bits_i(v[1]) << 16);
                    pk[h][1] = (uint32_t)f2h_bits_i(v[2]) | ((uint32_t)f2h_bits_i(v[3]) << 16);
                    if constexpr (SPLIT) {
                        uint16_t r[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const uint16_t hb = f2h_bits_i(v[e]);
                            r[e] = f2h_bits_i(v[e] - (float)__builtin_bit_cast(_Float16, hb));
                        }
                        pl[h][0] = (uint32_t)r[0] | ((uint32_t)r[1] << 16);
                        pl[h][1] = (uint32_t)r[2] | ((uint32_t)r[3] << 16);
                    }
                }
                const auto sl = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
                const auto sh = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
                const uint4 val = make_uint4(sl[0], sh[0], sl[1], sh[1]);
                // (STAGE: piece (g * 16 + cw) / 8 of pixel r16, column swizzled by the pixel)
                const int sp = r16 * 8 + (((g * 16 + cw) >> 3) ^ (r16 & 7));
                if constexpr (STAGE) ostage[wave][0][sp] = val;
                else
                    for (int d = 0; d < a.ndst; ++d)
                        *reinterpret_cast<uint4*>(dbase[d] + (size_t)(x + B) * a.dst_cs[d] + g * 16 + cw) = val;
                if constexpr (SPLIT) {
                    const auto ll = __builtin_amdgcn_permlane16_swap(pl[0][0], pl[1][0], false, false);
                    const auto lh = __builtin_amdgcn_permlane16_swap(pl[0][1], pl[1][1], false, false);
                    const uint4 lv = make_uint4(ll[0], lh[0], ll[1], lh[1]);
                    if constexpr (STAGE) ostage[wave][SPLIT ? 1 : 0][sp] = lv;
                    else
                        for (int d = 0; d < a.ndst; ++d)
                            *reinterpret_cast<uint4*>(dlo[d] + (size_t)(x + B) * a.dst_cs[d] + g * 16 + cw) = lv;
                }
            }
            if constexpr (STAGE) {
                // (one wave writes and reads its own image: LDS operations of a wave stay in order)
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");
                const int npc = a.cout / 8;   // 16-byte pieces per pixel (4 or 8)
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int idx = k * 64 + lane, pp = idx >> 3, pc = idx & 7;
                    const int xs = x0 + grp * 16 + pp;
                    const int rd = pp * 8 + (pc ^ (pp & 7));
                    const uint4 hv = ostage[wave][0][rd];
                    uint4 lv2 = hv;
                    if constexpr (SPLIT) lv2 = ostage[wave][SPLIT ? 1 : 0][rd];
                    if (xs < W && pc < npc) {
                        for (int d = 0; d < a.ndst; ++d) {
                            const size_t o = (size_t)(xs + B) * a.dst_cs[d] + pc * 8;
                            *reinterpret_cast<uint4*>(dbase[d] + o) = hv;
                            if constexpr (SPLIT) *reinterpret_cast<uint4*>(dlo[d] + o) = lv2;
                        }
                    }
                }
                asm volatile("" ::: "memory");
                __builtin_amdgcn_wave_barrier();   // the next group's pieces after these reads
            }
            continue;
        }
        if (x >= W) continue;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            const int ch = g * 16 + 4 * q;
            if (ch >= a.cout) continue;
            float v[4];
            const float4_t bq = sbias[g * 4 + q], mq = smul[g * 4 + q];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                // (split: the sums of the 2^e-scaled weights times 2^-e, exact; ConvArgs::wscale)
                const float t = (SPLIT ? acc[g][r] * a.wscale : acc[g][r]) + bq[r];
                v[r] = t > 0.f ? t : t * mq[r];
            }
            const uint32_t lo = (uint32_t)f2h_bits_i(v[0]) | ((uint32_t)f2h_bits_i(v[1]) << 16);
            const uint32_t hi = (uint32_t)f2h_bits_i(v[2]) | ((uint32_t)f2h_bits_i(v[3]) << 16);
            for (int d = 0; d < a.ndst; ++d)
                *reinterpret_cast<uint2*>(dbase[d] + (size_t)(x + B) * a.dst_cs[d] + ch) = make_uint2(lo, hi);
            if constexpr (SPLIT) {   // the residues of the stored halves
                uint16_t r[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint16_t hb = f2h_bits_i(v[e]);
                    r[e] = f2h_bits_i(v[e] - (float)__builtin_bit_cast(_Float16, hb));
                }
                const uint2 lv = make_uint2((uint32_t)r[0] | ((uint32_t)r[1] << 16),
                                            (uint32_t)r[2] | ((uint32_t)r[3] << 16));
                for (int d = 0; d < a.ndst; ++d)
                    *reinterpret_cast<uint2*>(dlo[d] + (size_t)(x + B) * a.dst_cs[d] + ch) = lv;
            }
        }
    }
}

}  // namespace

void launch_conv_image(const ConvArgs& a, const float* image, hipStream_t stream)
{
    OPK_CHECK_ARG(image != nullptr && a.w != nullptr, "image and weights required");
    OPK_CHECK_ARG(a.cout > 0 && a.cout <= 16 * NG && a.cout % 4 == 0, "conv_image: cout <= 64, % 4");
    OPK_CHECK_ARG(a.ndst >= 1 && a.ndst <= kConvMaxDst && a.out32 == nullptr, "conv_image: outputs");
    for (int d = 0; d < a.ndst; ++d)
        OPK_CHECK_ARG(((a.dst_cs[d] | a.dst_coff[d]) & 3) == 0, "conv_image: 8-byte aligned slices");
    const long blocks = (long)a.frames * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW);
    OPK_CHECK_ARG(blocks > 0 && blocks < (1L << 31), "conv_image: bad sizes");
    // 16-byte stores (CONV_IMAGE_WIDE=0: the 8-byte epilogue, dev A/B; same values)
    bool wide = a.cout % 32 == 0 && dev_switch("CONV_IMAGE_WIDE", 1) != 0;
    for (int d = 0; d < a.ndst; ++d) wide = wide && ((a.dst_cs[d] | a.dst_coff[d]) & 7) == 0;
    // whole-pixel stores through the per-wave LDS image (CONV_IMAGE_STAGE=0: direct, dev A/B)
    const bool stage = wide && dev_switch("CONV_IMAGE_STAGE", 1) != 0;
#define OPKI_LAUNCH(SP_, WI_, ST_)                                                               \
    hipLaunchKernelGGL((conv_image_kernel<SP_, WI_, ST_>), dim3((unsigned)blocks), dim3(256), 0, stream, a, image)
    if (a.split) {
        for (int d = 0; d < a.ndst; ++d) OPK_CHECK_ARG(a.dst_lo[d] != nullptr, "conv_image: split needs dst_lo");
        note_launch("conv_image_kernel<split>");
        if (stage) OPKI_LAUNCH(true, true, true);
        else if (wide) OPKI_LAUNCH(true, true, false);
        else OPKI_LAUNCH(true, false, false);
    } else {
        note_launch("conv_image_kernel");
        if (stage) OPKI_LAUNCH(false, true, true);
        else if (wide) OPKI_LAUNCH(false, true, false);
        else OPKI_LAUNCH(false, false, false);
    }
#undef OPKI_LAUNCH
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
