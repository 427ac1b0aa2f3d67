// conv.h -- implicit-GEMM convolution on gfx950 MFMA (fp16 operands, fp32 accumulate).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace opk {

// Activation layout everywhere in the net: NHWC fp16 with a one-pixel zero border,
// [frames][H+2][W+2][cs] ("padded image"), cs = channel stride of the buffer.
// GEMM view of a conv over such images:
//   M = frames * H * (W+2) virtual positions (the two extra columns per row are computed and
//       discarded: every 3x3 tap is then a constant shift of the whole tile),
//   N = output channels, K = taps * cin_pad (tap-major, channels inner, 32-channel chunks).
constexpr int kConvMaxDst = 6;
constexpr int kConvBK = 64;

struct ConvArgs {
    const uint16_t* in;   // fp16 bits, padded image
    int in_cs, in_coff;   // channel stride and first channel of the input slice
    int cin_pad;          // channels read per tap (multiple of 32)
    int ntaps;            // 9 (3x3) or 1 (1x1 / pre-packed)
    int tapoff[9];        // position offset of each tap from the window's top-left position
    int ksteps;           // ceil(ntaps * cin_pad / 64)
    const uint16_t* w;    // [cout_pad][ksteps*64] fp16 bits
    const float* bias;    // [cout]
    const float* slope;   // [cout] PReLU slopes (act == 2)
    int act;              // 0 none, 1 ReLU, 2 PReLU
    int frames, H, W;     // interior size (input and output share it)
    int M;                // frames * H * (W+2)
    int cout;
    int ndst;
    uint16_t* dst[kConvMaxDst];
    int dst_cs[kConvMaxDst], dst_coff[kConvMaxDst];
    float* out32;         // optional NCHW fp32 [frames][out32_c][H][W]
    int out32_c, out32_coff;
    int sw, nstrips;      // conv3 only: strip width and count (conv3_shape)
    float rcp[3];         // conv3 only, set by launch_conv3: 1/((H+2)(sw+2)), 1/(sw+2), 1/nstrips
    int wide;             // conv3 only, set by launch_conv3: 16-byte epilogue stores allowed (CONV3_WIDE)
    int prio;             // conv3 persistent: s_setprio(1) around each unit's MFMAs (CONV3P_PRIO)
    void* sink;           // conv3 persistent variant: >= kConv3SinkBytes of scratch (masked stores)
    int cus;              // conv3 persistent variant: compute units (grid size); 0 disables it
    int border;           // zero border of the padded images (conv3 / conv_image; 0 means 1)
    int actmax;           // conv3w / conv3w8: every negative-side multiplier (1 none, 0 ReLU, the
                          // PReLU slopes) lies in [0, 1], so t > 0 ? t : t*m == max(t, t*m) for
                          // every finite t (the epilogue's 2 VALU per value become 1); set by the host
    int bufst;            // conv3w: one destination whose extent is < 2^31 bytes -- epilogue stores
                          // through a buffer resource (set by launch_conv3w)
    int pool;             // conv3w8: 2x2/2 max pool fused into the epilogue; dst[0] is the pooled
                          // padded image [frames][H/2+2][W/2+2][cs] (conv3w8_pool_supported)
    int nbx;              // conv3w8, several n-blocks: XCD x computes n-block x % NB only, so an
                          // XCD's L2 holds one n-block's weights (set by launch_conv3w8)
    // Split precision (NetHip precision OPK_PRECISION_SPLIT; conv3_kernel only): every activation
    // x is held as two fp16 images, hi = fp16(x) and lo = fp16(x - hi) (in_lo / dst_lo: the lo
    // twins, same layout and offsets), and every weight w as w_hi = fp16(w), w_lo = fp16(w - w_hi).
    // The K loop runs three products per 32-channel input chunk, chunk-major -- x_hi * w_lo,
    // x_hi * w_hi (the same staged hi halo), x_lo * w_hi (the w_hi tap rows of the product
    // before, still in their weight slots: conv3w8 stages no weights for it) (weights packed
    // [cout_pad/BN][2 * cin_pad/32][ky][kx][BN][32]: the w_hi chunks, then the w_lo chunks) --
    // each product exact in fp32, so only the fp32 summation and the dropped x_lo * w_lo term
    // (~2^-22 relative) separate the result from an fp32 convolution.  The weights are packed
    // scaled by a power of two per layer, w' = w * 2^e with max |w'| in [2^14, 2^15), so w_lo is
    // a normal fp16 number (a He-init weight of ~0.03 would otherwise leave w - w_hi in fp16's
    // subnormal range, ~8 bits); the epilogue multiplies the sums by wscale = 2^-e before the
    // bias (exact: a power of two).  Kernels: conv3_kernel, conv3w8_kernel and conv_image_kernel
    // (SPLIT instantiations; the fp16 instantiations ignore wscale).
    int split;
    const uint16_t* in_lo;
    uint16_t* dst_lo[kConvMaxDst];
    float wscale;
};
// the product of a split virtual chunk (3c + k) that reads w_lo: k = 0 (the order above; dev A/B
// builds: OPK_SPLIT_WLO_K=1, the round-6 order x_hi w_hi, x_hi w_lo, x_lo w_hi, every product
// staging its weights)
#ifndef OPK_SPLIT_WLO_K
#define OPK_SPLIT_WLO_K 0
#endif

// conv3.hip: 7x7, 3x3 and 1x1, input halo staged once per 32-channel chunk over a "virtual image" of
// column strips (sw interior columns each).  Tile BM x BN = 256 x 128 / 96 (<= 80 KB LDS, two
// workgroups per CU, or 136 KB, one), 512 x 64 for cout <= 64; optional fp32 NCHW output (out32).
// Weights packed [cout_pad/BN][cin_pad/32][ky][kx][BN][32] (BN = conv3_shape(...).bn).  Reads padded positions down to -1
// and the whole row past the last one: buffers carry zeroed guards (kConvGuardTail positions).
constexpr int kConvGuardTail = 1024;   // positions
constexpr size_t kConv3SinkBytes = (size_t)1024 * 1024 * 16;   // 1024 lanes x 1024 workgroups x 16 B
struct Conv3Shape {
    int ks;                       // 7, 3 or 1
    int border;                   // zero border of the net's padded images
    int bm, bn, hr, tapu, minb;   // tile, halo rows, taps per K unit, workgroups per CU
    int nw;                       // waves per workgroup
    int sw, nstrips;
    bool persist;                 // 16-wave tiles: persistent kernel (conv3p) when the launch allows
};
// w8: the conv may run on conv3w8 (conv3_w8_eligible): 64-output 3x3 layers of >= 768 tiles then
// take the persistent 512-position geometry of the 8-wave kernel
Conv3Shape conv3_shape(int frames, int H, int W, int cout, int ks, int border = 1, bool w8 = false);
// a 64-output 3x3 conv that conv3w8's BN = 64 instantiation can run (one aligned destination, no
// fp32 output, a persistent sink): the planner and the launchers decide the same way from it
bool conv3_w8_eligible(int cout, int ntaps, int ndst, const int* dst_cs, const int* dst_coff, bool out32);
inline bool conv3_w8_eligible(const ConvArgs& a)
{
    return a.sink && a.cus > 0 && conv3_w8_eligible(a.cout, a.ntaps, a.ndst, a.dst_cs, a.dst_coff, a.out32 != nullptr);
}
void launch_conv3(const ConvArgs& a, hipStream_t stream);
// conv3w.hip: the persistent 512 x {128, 96} 3x3 variant with one mid-unit barrier per K unit
// (launched by launch_conv3 for single-n-block layers on the persistent path)
bool conv3w_supported(const ConvArgs& a);
void launch_conv3w(const ConvArgs& a, hipStream_t stream);
// conv3w8.hip: the same tile with 8 waves of 64 x BN (fewer LDS fragment reads per MFMA)
bool conv3w8_supported(const ConvArgs& a);
bool conv3w8_pool_supported(const ConvArgs& a);
void launch_conv3w8(const ConvArgs& a, hipStream_t stream);

// conv_head.hip: Mconv6 (1x1, n1 = 256 / 512 outputs, act6) -> Mconv7 (1x1, n2 <= 64 outputs) in
// one kernel; the Mconv6 activations never leave the chip.  Input / outputs as ConvArgs (padded
// NHWC fp16 slices, optional fp32 NCHW out32).  w6: [cin_pad/32][n1][32] fp16; w7: packed by
// conv_head_pack_w7 ([n2 <= 32 ? 32 : 64][n1], K permuted within 32-channel blocks); b7 zero-padded
// to 64 floats; b6 / s6 [n1].
struct HeadArgs {
    const uint16_t* in;
    int in_cs, in_coff, cin_pad;
    const uint16_t* w6;
    const float *b6, *s6;
    int act6;
    const uint16_t* w7;
    const float* b7;
    int n1, n2;
    int frames, H, W;
    int ndst;
    uint16_t* dst[kConvMaxDst];
    int dst_cs[kConvMaxDst], dst_coff[kConvMaxDst];
    float* out32;
    int out32_c, out32_coff;
    int cus;              // > 0: persistent grid of this many workgroups (conv_head.hip)
    int actmax;           // Mconv6's negative-side multipliers all in [0, 1] (ConvArgs::actmax)
    // split precision (ConvArgs::split): the input as (in, in_lo) fp16 pairs, w6 packed
    // [2][cin_pad/32][n1][32] (w_hi block, then w_lo), w7 [2][n2p][n1] (each K-permuted), both
    // scaled by 2^e per layer (sums times wscale6 / wscale7 before the bias); Mconv6's activation
    // is split into (hi, lo) on chip and Mconv7 runs x_hi w_hi + x_lo w_hi + x_hi w_lo; outputs
    // hi to dst, lo to dst_lo
    int split;
    const uint16_t* in_lo;
    uint16_t* dst_lo[kConvMaxDst];
    float wscale6, wscale7;
};
bool conv_head_supported(int n1, int n2, int cin_pad);
void conv_head_pack_w7(uint16_t* dst, const uint16_t* w7 /* [n2][n1] */, int n1, int n2);
void launch_conv_head(const HeadArgs& a, hipStream_t stream);

// First conv (3 input channels, 3x3, cout <= 64) straight from the fp32 NCHW input [frames][3][H][W]
// (conv_image.hip); weights [cout_pad][64], K order (ky*3 + kx)*3 + ci.
void launch_conv_image(const ConvArgs& a, const float* image, hipStream_t stream);

// conv1_1 (3 -> 64) + act -> conv1_2 (64 -> 64) + act -> 2x2/2 max pool in one persistent kernel
// (conv1_fused.hip).  img: fp32 NCHW [frames][3][H][W]; w1: [64][64] (K order (ky*3+kx)*3+ci);
// w2: conv3 packing for BN = 64; bias/slope arrays zero-padded to 128; out: the pooled padded NHWC
// fp16 image [frames][OH+2][OW+2][out_cs] (slice at out_coff).  H and W even.
struct Conv1FusedArgs {
    const float* img;
    int frames, H, W;
    const uint16_t* w1;
    const float *b1, *s1;
    int act1;
    const uint16_t* w2;
    const float *b2, *s2;
    int act2;
    uint16_t* out;
    int out_cs, out_coff, OH, OW;
    int actmax;           // both convs' negative-side multipliers in [0, 1] (ConvArgs::actmax)
};
bool conv1_fused_supported(int H, int W, int cout1, int cout2);
void launch_conv1_fused(const Conv1FusedArgs& a, int workgroups, hipStream_t stream);

// 2x2 stride-2 max pool with Caffe ceil sizing, padded NHWC fp16 -> padded NHWC fp16.
// split precision: the lo twins of input and output; the pooled pair is the (hi, lo) pair of the
// largest hi + lo (exact in fp32)
void launch_maxpool2_split(uint16_t* out, uint16_t* out_lo, const uint16_t* in, const uint16_t* in_lo,
                           int frames, int H, int W, int C, int OH, int OW, hipStream_t stream,
                           int border);
void launch_maxpool2(uint16_t* out, const uint16_t* in, int frames, int H, int W, int C, int OH,
                     int OW, hipStream_t stream, int border = 1);

}  // namespace opk
