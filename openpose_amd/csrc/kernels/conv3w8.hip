// conv3w8.hip -- 3x3 convolution: the persistent 512 x {128, 96} halo implicit GEMM of conv3w.hip
// with 8 waves of 64 positions x ALL output channels instead of 16 waves of 64 x 64.
//
// Why: the conv3w K loop is bound by LDS fragment reads, not by the MFMAs or the barrier
// (tools/conv3w_probe.hip ablations, 64 frames x 46x82, cin 384: 197 us as built, 194 without the
// mid-unit barrier, 174 without MFMAs, 138 without fragment reads).  With 16 waves of 64 x 64 every
// weight (B) fragment is read by 8 waves and every halo (A) fragment by 2: 8 ds_read_b128 per 16
// MFMAs.  Here a wave owns 64 positions x BN channels (acc 128 VGPRs at 2 waves per SIMD): per tap
// MF = 4 A + NF = 8 B fragments for 32 MFMAs, 25 % fewer LDS reads per MFMA, and the next tap's
// B fragments stream in during taps 0 and 1 of a K unit (fbE / fbO alternate; tap 2 re-reads the
// next unit's tap-0 B into fbE after its last MFMAs), the A fragments two steps ahead.
//
// Same tile, operands, LDS layout, K order and epilogue arithmetic as conv3w_kernel / conv3p_kernel,
// so outputs are bit-identical to them.  Schedule per K unit u = (chunk c, tap row ky), as conv3w:
//     tap 0, tap 1, [wait own DMA of unit u+1; s_barrier], tap 2, [issue DMA of unit u+2];
// fragments of unit u+1 are read during tap 2 (certified by the mid-unit barrier).
//
// lgkmcnt: per tap, step i (position fragment i) issues A(t, i+2) (for i >= 2: the next tap's A
// fragments 0 / 1) and, in taps 0 / 1, the next tap's B fragments 2i, 2i+1; the waits (kWait) are
// counted from that fixed issue order (no other LDS traffic inside the K loop).
#include "conv.h"

#include <algorithm>

#include "../common.h"
#include "conv3_dev.h"

namespace opk {

namespace {

using namespace conv3dev;

constexpr int k8_BM = 512, k8_HR = 688, k8_NW = 8;

// Unit u+2's DMA right after the mid-unit barrier (a third of a unit more lead) instead of after
// tap 2: the split 96- and 64-output tiles (measured 3-3.5 % faster per launch, round 6,
// profiles/round6/split_dma_early/); the 128-output tiles spill 26-30 VGPRs with it (1.5x slower)
// and the fp16 tiles keep their measured schedule.  Dev A/B builds: OPK8_DMA_EARLY 0 never, 1 always.
#ifndef OPK8_DMA_EARLY
#define OPK8_DMA_EARLY 2
#endif
#ifndef OPK8_ABLATE   // dev probe only (tools/conv3w_probe.hip): 1 no mid-unit barrier, 2 no MFMAs,
#define OPK8_ABLATE 0  // 3 no fragment reads, 4 no DMA after the prologue, 5 no MFMAs in tap 1 of
                       // each unit (a third fewer, replaced by VALU adds), 6 the same with nothing
                       // issued in their place, 7 no halo DMA / 8 no weight DMA after the
                       // prologue (timing only, wrong results)
#endif
#if OPK8_ABLATE == 3
#define OPK8_DSR(dst_, addr_, off_) asm volatile("; no read %1" : "=v"(dst_) : "v"(addr_))
#else
#define OPK8_DSR(dst_, addr_, off_)                                                           \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst_) : "v"(addr_), "i"(off_))
#endif

// POOL: the 2x2 / stride-2 max pool that follows the conv (pool2 / pool3 of BODY_25,
// pose_deploy.prototxt:70-87,149-166) fused into the epilogue: a tile is 6 virtual rows starting
// at an odd row, one position in (p0 = (6m + 1) VW + 1), so every pooling window lies inside one
// tile with its column pair in lanes (2k, 2k+1) of a fragment; the lanes take the horizontal max
// through a DPP swap, the first row of each window stores it into the pooled image, and after a
// workgroup barrier the second row's lanes read it back, take the max and store.  The full-size
// conv output is never written.
// MX: the activation as max(t, t*m) (ConvArgs::actmax; conv3_dev.h act_pick)
// BST: one destination, epilogue stores through a buffer resource (ConvArgs::bufst)
typedef unsigned int opk8_u4 __attribute__((ext_vector_type(4)));
#ifndef OPK_FAULT_POOL
#define OPK_FAULT_POOL 0
#endif

// SPLIT: split precision (ConvArgs::split, conv.h): K runs chunk-major over three products per
// input chunk c -- virtual chunk 3c + k: k = 0 x_hi w_lo, 1 x_hi w_hi, 2 x_lo w_hi -- so the hi
// halo of a chunk is staged once for two products (k = 1 issues no halo DMA and reads k = 0's
// slot; hi halos live in slot 0, lo halos in slot 1) and the w_hi tap rows once for two (k = 2
// stages no weights: k = 1 left them in its slots), in the order of conv3_kernel<..., SPLIT>;
// the epilogue writes hi = fp16(v) and lo = fp16(v - hi) of v = act(acc * wscale + bias) --
// bit-identical to conv3_kernel's split instantiations.
// split-precision pooling (POOL && SPLIT): of two (hi, lo) fp16 pairs of 8 channels, keep per
// channel the one with the larger hi + lo (exact in fp32), the first (h1, l1) on ties -- the rule
// of maxpool2_split_kernel (pool.hip), whose raster-order scan this reproduces window-wise
__device__ __forceinline__ void opk8_pair_max(uint4& h1, uint4& l1, const uint4& h2, const uint4& l2)
{
    uint32_t* a = reinterpret_cast<uint32_t*>(&h1);
    uint32_t* al = reinterpret_cast<uint32_t*>(&l1);
    const uint32_t* b = reinterpret_cast<const uint32_t*>(&h2);
    const uint32_t* bl = reinterpret_cast<const uint32_t*>(&l2);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const float2_t fa = __builtin_convertvector(__builtin_bit_cast(half2_t, a[w]), float2_t) +
                            __builtin_convertvector(__builtin_bit_cast(half2_t, al[w]), float2_t);
        const float2_t fb = __builtin_convertvector(__builtin_bit_cast(half2_t, b[w]), float2_t) +
                            __builtin_convertvector(__builtin_bit_cast(half2_t, bl[w]), float2_t);
        const uint32_t m = (fb.x > fa.x ? 0x0000ffffu : 0u) | (fb.y > fa.y ? 0xffff0000u : 0u);
        a[w] = (a[w] & ~m) | (b[w] & m);
        al[w] = (al[w] & ~m) | (bl[w] & m);
    }
}

template <int BN, int NB, bool POOL, bool MX, bool BST, bool SPLIT>
__global__ __launch_bounds__(64 * k8_NW, 1) void conv3w8_kernel(const ConvArgs a)
{
    constexpr int NW = k8_NW, BM = k8_BM, HR = k8_HR;
    constexpr int WROWS = BM / NW, MF = WROWS / 16, NF = BN / 16;
    static_assert(WROWS == 64 && (NF == 8 || NF == 6 || NF == 4), "wave tiles 64 x 128 / 96 / 64");
    constexpr int API = HR / 16, AIW = (API + NW - 1) / NW;
    constexpr int BROWS = 3 * BN, BPI = BROWS / 16, BIW = (BPI + NW - 1) / NW;
    constexpr int ASLOT = HR * 4, BSLOT = BROWS * 4;   // 16-byte pieces
    constexpr int LDS_PIECES = 2 * ASLOT + 3 * BSLOT + BN / 2;
    static_assert(LDS_PIECES * 16 <= 160 * 1024, "LDS budget");
    // counted lgkmcnt waits of steps 0..3 per tap kind (-1: none needed), from the issue order
    // (see OPK8_TAP): step 0 waits for the tap's last B fragment and everything older
    // (NF = 4: taps 0 / 1 stream the next tap's B fragments in steps 0 and 1 only)
    constexpr int kWait[3][4] = {
        {3, -1, NF == 4 ? 6 : 8, NF == 8 ? 8 : (NF == 6 ? 6 : 4)},                               // tap 0
        {NF == 8 ? 3 : 4, NF == 8 ? -1 : 6, NF == 4 ? 6 : 8, NF == 8 ? 8 : (NF == 6 ? 6 : 4)},   // tap 1
        {NF == 8 ? 1 : 2, NF == 8 ? -1 : 2, 2, 2}};                                              // tap 2
    __shared__ uint4 lds[LDS_PIECES];
    float* lbias = reinterpret_cast<float*>(lds + 2 * ASLOT + 3 * BSLOT);
    float* lmul = lbias + BN;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const Strips g(a);
    // POOL tiles: 6 rows of VW positions from row 6m + 1, position 1 (the 512 computed positions
    // overlap the next tile's first 512 - 6 VW, which are not stored)
    const int BMP = POOL ? 6 * g.VW : BM;
    const int ntm = POOL ? (g.total / g.VW - 1 + 5) / 6 : (g.total + BM - 1) / BM;
#define OPK8_P0(mt_) (POOL ? (6 * (mt_) + 1) * g.VW + 1 : (mt_) * BM)
    // output-channel blocks of BN: tile t = (m-tile t / NB, n-block t % NB);
    // the grid is a multiple
    // of NB (host), so a block keeps one n-block -- its weights and bias -- for the whole launch
    // and walks the m-tiles m0, m0 + G / NB, ...; the NB n-blocks of one m-tile sit on one XCD
    static_assert(NB == 1 || NB == 2 || NB == 4, "1, 2 or 4 n-blocks");
    constexpr int LGNB = NB == 4 ? 2 : NB - 1;
    const int G = gridDim.x, GM = G >> LGNB;
    const int xcd = blockIdx.x & 7, qq = G >> 3, rr = G & 7;
    int nblk, m;
    if (NB > 1 && a.nbx) {
        // (G % 8 == 0, host) the blocks of XCD x (blocks b = x mod 8, observed placement; speed
        // only) all take n-block x % NB: an XCD's L2 then holds one n-block's weights instead of
        // all NB (split precision: 1.8 MB per n-block of a 256-input layer, 3.5 MB at 512 inputs,
        // against 4 MB of L2); the n-block's 8 / NB XCDs share its m-tiles, each XCD a contiguous
        // range per round
        nblk = xcd & (NB - 1);
        m = (xcd >> LGNB) * qq + (blockIdx.x >> 3);
    } else {
        const int tix = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (blockIdx.x >> 3);
        nblk = tix & (NB - 1);
        m = tix >> LGNB;
    }
    if (m >= ntm) return;

    // bias / negative-side multiplier of the n-block: registers now, LDS after the prologue's
    // DMA wait (which covers these older loads), so they do not delay the first DMA issue
    float bias_v = 0.f, mul_v = 0.f;
    if (tid < BN) {
        const float neg = a.act == 1 ? 0.f : 1.f;
        bias_v = a.bias[nblk * BN + tid];
        mul_v = a.act == 2 ? a.slope[nblk * BN + tid] : neg;
    }

    const int lrow = lane >> 2, phys = lane & 3;
    const int cpt = a.cin_pad >> 5;
    const int cptk = SPLIT ? 3 * cpt : cpt;   // K (virtual) chunks (split: three per input chunk)
    constexpr bool kDmaEarly = OPK8_DMA_EARLY == 1 || (OPK8_DMA_EARLY == 2 && SPLIT && BN <= 96);
    const int U = 3 * cptk;
    // the n-block's first K unit in the packed weights (split: w_hi and w_lo, 2 cpt chunks of 3
    // units; virtual chunk 3c + k reads w_lo chunk c (cpt + c) for k = OPK_SPLIT_WLO_K, w_hi chunk
    // c otherwise)
    const int ublk = nblk * 3 * (SPLIT ? 2 * cpt : cpt);
    const int bi = (BPI - wave + NW - 1) / NW;
    // weight piece of B DMA instruction j (recomputed at each issue: registers)
#define OPK8_BOFF(j_)                                                                         \
    ({                                                                                        \
        int rb_ = ((j_) * NW + wave) * 16 + lrow;                                             \
        asm volatile("" : "+v"(rb_));                                                         \
        rb_ * 32 + (phys ^ (((rb_ >> 2) & 1) << 1)) * 8;                                      \
    })
    const char* abase = reinterpret_cast<const char*>(a.in + a.in_coff - a.in_cs);
    const char* abase_lo = SPLIT ? reinterpret_cast<const char*>(a.in_lo + a.in_coff - a.in_cs) : abase;
    uint32_t aoff[AIW];
#define OPK8_AROW1(mt_, i_)                                                                   \
    ({                                                                                        \
        const int hr_ = ((i_) * NW + wave) * 16 + lrow;                                       \
        const int lp_ = phys ^ (((hr_ >> 2) & 1) << 1);                                       \
        int f_, yy_, xx_, s_;                                                                 \
        const long pos_ = g.map(OPK8_P0(mt_) - g.VW - 1 + hr_, f_, yy_, xx_, s_);             \
        (uint32_t)(((pos_ + 1) * a.in_cs + lp_ * 8) * 2);                                     \
    })
#define OPK8_AROW(dst_, mt_)                                                                  \
    do {                                                                                      \
        _Pragma("unroll") for (int i_ = 0; i_ < AIW; ++i_) dst_[i_] = OPK8_AROW1(mt_, i_);     \
    } while (0)
    // K unit (virtual chunk of product k_ over input chunk dc_, tap row ky_); split: k_ = 1
    // reuses k_ = 0's hi halo (no DMA), k_ = 2 stages the lo twin's; fp16: k_ = 0, dc_ = chunk.
    // Split, k_ = 2 (x_lo w_hi) with k_ = 1 the w_hi product (OPK_SPLIT_WLO_K 0): its tap row's
    // weight slot ((u + 2) % 3 = (u - 1) % 3, written last by unit u - 3, k_ = 1 at the same ky)
    // still holds exactly these w_hi rows, so no weights are staged for it
#define OPK8_ISSUE(k_, dc_, ky_, aslot_, bslot_, nt_)                                         \
    do {                                                                                      \
        if ((ky_) == 0 && (k_) != 1 && (OPK8_ABLATE != 7 || !dma_ab)) {                       \
            const int as_ = (aslot_) * ASLOT;                                                 \
            const char* ab_ = (k_) == 2 ? abase_lo : abase;                                   \
            _Pragma("unroll") for (int i_ = 0; i_ < AIW; ++i_)                                \
                if (API % NW == 0 || i_ * NW + wave < API)                                    \
                    __builtin_amdgcn_global_load_lds(                                         \
                        (const void*)(ab_ + (dc_) * 64 +                                      \
                                      ((nt_) ? OPK8_AROW1(m + GM, i_) : aoff[i_])),            \
                        (__attribute__((address_space(3))) void*)(&lds[as_ + (i_ * NW + wave) * 64]), \
                        16, 0, 0);                                                            \
        }                                                                                     \
        const int bs_ = 2 * ASLOT + (bslot_) * BSLOT;                                         \
        const int wc_ = (SPLIT && (k_) == OPK_SPLIT_WLO_K) ? cpt + (dc_) : (dc_);            \
        const uint16_t* ub_ = a.w + (size_t)(ublk + wc_ * 3 + (ky_)) * BROWS * 32;            \
        _Pragma("unroll") for (int j_ = 0; j_ < BIW; ++j_)                                    \
            if ((BPI % NW == 0 || j_ * NW + wave < BPI) && (OPK8_ABLATE != 8 || !dma_ab) &&   \
                !(SPLIT && OPK_SPLIT_WLO_K == 0 && (k_) == 2)) {                              \
                const int bo_ = OPK8_BOFF(j_);                                                \
                __builtin_amdgcn_global_load_lds(                                             \
                    (const void*)(ub_ + bo_),                                                 \
                    (__attribute__((address_space(3))) void*)(&lds[bs_ + (j_ * NW + wave) * 64]), \
                    16, 0, 0);                                                                \
            }                                                                                 \
    } while (0)

    // fragment bases: A row wave*64 + r16 + ky*VW + kx of a halo slot; B row kx*BN + r16 of a
    // weight slot (fragment j at +1 KiB j)
    const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
    const int arow0 = wave * WROWS + r16;
    const uint32_t bswz = (uint32_t)swz64(r16, q) * 16;
#define OPK8_ABASE(slot_, ky_, kx_)                                                            \
    ({                                                                                        \
        int r_ = arow0 + (ky_) * g.VW + (kx_);                                                \
        asm volatile("" : "+v"(r_));                                                          \
        lds0 + (uint32_t)((slot_) * ASLOT * 16) + (uint32_t)swz64(r_, q) * 16;                \
    })
#define OPK8_BBASE(slot_)                                                                     \
    ({                                                                                        \
        uint32_t b_ = bswz;                                                                   \
        asm volatile("" : "+v"(b_));                                                          \
        lds0 + (uint32_t)((2 * ASLOT + (slot_) * BSLOT) * 16) + b_;                           \
    })

    half8_t fbE[NF], fbO[NF], fa[4];
    float4_t acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

    // B fragment j of a tap (weight base bb_ + tap offset)
#define OPK8_RB(dst_, bb_, toff_, j_)                                                         \
    do {                                                                                      \
        switch (j_) {                                                                         \
        case 0: OPK8_DSR(dst_, bb_, (toff_) + 0); break;                                      \
        case 1: OPK8_DSR(dst_, bb_, (toff_) + 1024); break;                                   \
        case 2: OPK8_DSR(dst_, bb_, (toff_) + 2048); break;                                   \
        case 3: OPK8_DSR(dst_, bb_, (toff_) + 3072); break;                                   \
        case 4: OPK8_DSR(dst_, bb_, (toff_) + 4096); break;                                   \
        case 5: OPK8_DSR(dst_, bb_, (toff_) + 5120); break;                                   \
        case 6: OPK8_DSR(dst_, bb_, (toff_) + 6144); break;                                   \
        default: OPK8_DSR(dst_, bb_, (toff_) + 7168); break;                                  \
        }                                                                                     \
    } while (0)
#define OPK8_RA(dst_, ab_, i_)                                                                \
    do {                                                                                      \
        switch (i_) {                                                                         \
        case 0: OPK8_DSR(dst_, ab_, 0); break;                                                \
        case 1: OPK8_DSR(dst_, ab_, 1024); break;                                             \
        case 2: OPK8_DSR(dst_, ab_, 2048); break;                                             \
        default: OPK8_DSR(dst_, ab_, 3072); break;                                            \
        }                                                                                     \
    } while (0)
#define OPK8_WAIT(n_, cur_, ...)                                                              \
    asm volatile("s_waitcnt lgkmcnt(%c[n])" : "+v"(cur_), ##__VA_ARGS__ : [n] "n"(n_))
    // one tap of kind K on B fragments FC and A fragments fa[]: K 0 / 1 (a unit's taps 0 / 1)
    // stream the next tap's B fragments into FN during the steps; K 2 (tap 2) reads the next
    // unit's tap-0 B fragments back into FC after its last MFMAs.  A fragments of the next tap
    // come from base nab_ (steps 2, 3), B fragments from nbb_ + nbo_.
#define OPK8_STEP(K, I, ab_, nab_, nbb_, nbo_, FC, FN)                                        \
    do {                                                                                      \
        if constexpr (I < 2) OPK8_RA(fa[I + 2], ab_, I + 2);                                  \
        else OPK8_RA(fa[I - 2], nab_, I - 2);                                                 \
        if constexpr (K != 2)                                                                 \
            _Pragma("unroll") for (int k_ = 0; k_ < 2; ++k_)                                  \
                if (2 * I + k_ < NF) OPK8_RB(FN[2 * I + k_], nbb_, nbo_, 2 * I + k_);          \
        constexpr int w_ = kWait[K][I];                                                       \
        if constexpr (I == 0) {                                                               \
            if constexpr (NF == 8)                                                            \
                OPK8_WAIT(w_, fa[0], "+v"(fa[1]), "+v"(FC[0]), "+v"(FC[1]), "+v"(FC[2]),      \
                          "+v"(FC[3]), "+v"(FC[4]), "+v"(FC[5]), "+v"(FC[6 % NF]),            \
                          "+v"(FC[7 % NF]));                                                  \
            else if constexpr (NF == 6)                                                       \
                OPK8_WAIT(w_, fa[0], "+v"(FC[0]), "+v"(FC[1]), "+v"(FC[2]), "+v"(FC[3]),      \
                          "+v"(FC[4 % NF]), "+v"(FC[5 % NF]));                                \
            else                                                                              \
                OPK8_WAIT(w_, fa[0], "+v"(FC[0]), "+v"(FC[1]), "+v"(FC[2]), "+v"(FC[3]));     \
        } else if constexpr (w_ >= 0) {                                                       \
            OPK8_WAIT(w_ < 0 ? 0 : w_, fa[I]);                                                \
        }                                                                                     \
        _Pragma("unroll") for (int j_ = 0; j_ < NF; ++j_)                                     \
            if constexpr (OPK8_ABLATE == 6 && K == 1)                                         \
                asm volatile("; mfma skipped" : "+v"(acc[I][j_]) : "v"(FC[j_]), "v"(fa[I]));  \
            else                                                                              \
            acc[I][j_] = (OPK8_ABLATE == 2 || (OPK8_ABLATE == 5 && K == 1))                  \
                ? acc[I][j_] + (float)fa[I][j_]                                               \
                : __builtin_amdgcn_mfma_f32_16x16x32_f16(FC[j_], fa[I], acc[I][j_], 0, 0, 0);   \
        __builtin_amdgcn_sched_barrier(0);                                                    \
    } while (0)
#define OPK8_TAP(K, ab_, nab_, nbb_, nbo_, FC, FN)                                            \
    do {                                                                                      \
        OPK8_STEP(K, 0, ab_, nab_, nbb_, nbo_, FC, FN);                                       \
        OPK8_STEP(K, 1, ab_, nab_, nbb_, nbo_, FC, FN);                                       \
        OPK8_STEP(K, 2, ab_, nab_, nbb_, nbo_, FC, FN);                                       \
        OPK8_STEP(K, 3, ab_, nab_, nbb_, nbo_, FC, FN);                                       \
        if constexpr (K == 2)                                                                 \
            _Pragma("unroll") for (int j_ = 0; j_ < NF; ++j_) OPK8_RB(FC[j_], nbb_, nbo_, j_); \
    } while (0)

    // ---- prologue: units 0 and 1 of the first tile in flight, unit 0 visible, tap 0 read ------
    OPK8_AROW(aoff, m);
    bool dma_ab = false;   // (dev ablations 7 / 8: set after the prologue)
    OPK8_ISSUE(0, 0, 0, 0, 0, false);
    OPK8_ISSUE(0, 0, 1, 0, 1, false);
    dma_ab = true;
    (void)dma_ab;
    vm_wait_rt(bi);
    if (tid < BN) {
        lbias[tid] = bias_v;
        lmul[tid] = mul_v;
    }
    __builtin_amdgcn_s_barrier();
    {
        const uint32_t bb0 = OPK8_BBASE(0);
        const uint32_t ab0 = OPK8_ABASE(0, 0, 0);
#pragma unroll
        for (int j = 0; j < NF; ++j) OPK8_RB(fbE[j], bb0, 0, j);
        OPK8_RA(fa[0], ab0, 0);
        OPK8_RA(fa[1], ab0, 1);
    }

    int gc = 0;   // running chunk index of this tile's chunk 0 (halo slot parity)
    for (;;) {
        const int mn = m + GM;
        const bool has_next = mn < ntm;
        // split: the unit's product k (vk) and input chunk (dcc), advanced by compares -- no
        // division by 3 in the loop (a % 3 slot rule cost the kernel 3 spilled VGPRs)
        int vk = 0, dcc = 0;
        for (int u = 0; u < U; ++u) {
            const int c = u / 3, ky = u - 3 * (u / 3);
            // halo slot: split -- hi halos in 0, lo halos in 1; fp16 -- chunk parity
            const int aslot = SPLIT ? (vk == 2 ? 1 : 0) : ((gc + c) & 1);
            const uint32_t bb_u = OPK8_BBASE(u % 3);
            const uint32_t ab0 = OPK8_ABASE(aslot, ky, 0);
            const uint32_t ab1 = OPK8_ABASE(aslot, ky, 1);
            const uint32_t ab2 = OPK8_ABASE(aslot, ky, 2);
            // next unit's tap 0 (unit u+1, or the next tile's unit 0): halo slot, tap row, weights
            const bool nt = u + 1 >= U;
            const int u1 = nt ? 0 : u + 1;
            const int c1 = u1 / 3, ky1 = u1 - 3 * (u1 / 3);
            // (split: unit u+1 is the same virtual chunk unless this is its tap row 2)
            const int vk1 = nt ? 0 : (ky < 2 ? vk : (vk == 2 ? 0 : vk + 1));
            const int aslot1 = SPLIT ? (vk1 == 2 ? 1 : 0) : ((gc + (nt ? cptk : 0) + c1) & 1);
            const uint32_t nab = OPK8_ABASE(aslot1, ky1, 0);
            const uint32_t nbb = OPK8_BBASE((u + 1) % 3);
            constexpr int S1 = MF * (NF / 2) * (SPLIT ? 2 : 1);   // epilogue stores per wave
#define OPK8_DMA_U2()                                                                         \
    do {                                                                                      \
        const bool nt_ = u + 2 >= U;                                                          \
        const int u2_ = nt_ ? u + 2 - U : u + 2;                                              \
        const int c2_ = u2_ / 3;                                                              \
        if constexpr (SPLIT) {   /* unit u+2: this virtual chunk at ky 0, else the next */    \
            const bool same_ = ky == 0 && !nt_;                                               \
            const int k2_ = nt_ ? 0 : (same_ ? vk : (vk == 2 ? 0 : vk + 1));                  \
            const int d2_ = nt_ ? 0 : (same_ || vk < 2 ? dcc : dcc + 1);                      \
            OPK8_ISSUE(k2_, d2_, u2_ - 3 * c2_, k2_ == 2 ? 1 : 0, (u + 2) % 3, nt_);          \
        } else {                                                                              \
            OPK8_ISSUE(0, c2_, u2_ - 3 * c2_, (gc + (nt_ ? cptk : 0) + c2_) & 1, (u + 2) % 3, nt_); \
        }                                                                                     \
    } while (0)
            OPK8_TAP(0, ab0, ab1, bb_u, BN * 64, fbE, fbO);
            OPK8_TAP(1, ab1, ab2, bb_u, 2 * BN * 64, fbO, fbE);
            // (several destinations: S1 stores per destination -- wait for all, rare layers)
            if (u == 0 && gc > 0 && (BST || a.ndst == 1)) vm_wait<S1>();   // (BST: one destination)
            else vm_wait<0>();
            if (OPK8_ABLATE != 1) __builtin_amdgcn_s_barrier();
            if (kDmaEarly && (OPK8_ABLATE != 4 || u + 2 >= U)) OPK8_DMA_U2();
            OPK8_TAP(2, ab2, nab, nbb, 0, fbE, fbO);
            if (!kDmaEarly && (OPK8_ABLATE != 4 || u + 2 >= U)) OPK8_DMA_U2();
#undef OPK8_DMA_U2
            if (SPLIT && ky == 2) {   // next virtual chunk
                dcc += vk == 2 ? 1 : 0;
                vk = vk == 2 ? 0 : vk + 1;
            }
        }

        // ---- epilogue: bias + activation + fp16 pack, 16-byte stores (border lanes to the sink)
        int el = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        asm volatile("" : "+v"(el));   // recomputed per tile: nothing lane-dependent kept (spilled)
        const int er16 = el & 15, eq = el >> 4;
        const int sidx = blockIdx.x * 64 * NW + wave * 64 + el;
        uint4* sink4 = reinterpret_cast<uint4*>(a.sink) + sidx;
        const int cw = 16 * (eq & 1) + 8 * (eq >> 1);   // channel of a lane's 16-byte store
        int prow[MF];
        bool pok[MF];
        if (g.nstrips == 1 && !POOL) {   // (conv3_dev.h Strips::rows1)
            g.rows1<MF>(OPK8_P0(m) + wave * WROWS + er16, a.W, prow, pok);
        } else {
            const int pbase = OPK8_P0(m) + wave * WROWS + er16;
            int f, yy, xx, s;
            prow[0] = (int)g.map(pbase, f, yy, xx, s);
            pok[0] = g.interior(yy, xx, s, a.W);
#pragma unroll
            for (int i = 1; i < MF; ++i) {
                xx += 16;
                if (xx >= g.VW) {
                    xx -= g.VW;
                    if (++yy == g.Hp) {
                        yy = 0;
                        if (++s == g.nstrips) {
                            s = 0;
                            ++f;
                        }
                    }
                }
                const bool in = pbase + i * 16 < g.total;
                prow[i] = in ? (f * g.Hp + yy) * g.Wp + s * g.sw + xx : 0;
                pok[i] = in && g.interior(yy, xx, s, a.W);
            }
        }
        const char* lb = reinterpret_cast<const char*>(lbias) + 4 * eq * 4;
        const int nd = a.ndst;
        uint16_t* const d0 = a.dst[0] + a.dst_coff[0] + nblk * BN;
        const int cs0 = a.dst_cs[0];
        const __amdgpu_buffer_rsrc_t rs0 = buf_rsrc(d0);
        // split: the lo twin of the destination (same layout and offsets)
        uint16_t* const d0lo = SPLIT ? a.dst_lo[0] + a.dst_coff[0] + nblk * BN : d0;
        const __amdgpu_buffer_rsrc_t rs0lo = buf_rsrc(d0lo);
        if constexpr (POOL) {
            // pooled position of each fragment's lane pair; phase 1 = the window's first row
            int qrow[MF];
            bool qok[MF], first[MF];
            {
                const int OWp = (a.W >> 1) + 2, OHp = (a.H >> 1) + 2;
                const int pb = OPK8_P0(m) + wave * WROWS + er16;
#pragma unroll
                for (int i = 0; i < MF; ++i) {
                    int f, yy, xx, s;
                    (void)g.map(pb + i * 16, f, yy, xx, s);
                    const int k = wave * WROWS + i * 16 + er16;   // tile-local position
                    qok[i] = pok[i] && (er16 & 1) == 0 && k < BMP;
                    first[i] = (yy & 1) != 0;
                    qrow[i] = qok[i] ? (f * OHp + ((yy - 1) >> 1) + 1) * OWp + ((s * g.sw + xx - 1) >> 1) + 1 : 0;
                }
            }
            // (BST) byte offsets of the window's second-row lanes (which store the pooled value), the
            // other lanes out of range
            uint32_t qo2[MF];
#pragma unroll
            for (int i = 0; i < MF; ++i)
                qo2[i] = qok[i] && !first[i] ? ((uint32_t)qrow[i] * (uint32_t)cs0 + cw) * 2 : kBufOOB;
            // The window's two rows meet in LDS: the halo slot of the tile's last chunk is free once
            // every wave has passed its last reads of it (the barrier below), and the next write into
            // it is the next tile's chunk-1 DMA, issued after that tile's mid-unit-1 barrier.  First-
            // row lanes leave their column-pair max there, second-row lanes read it back -- instead
            // of a store to the pooled image, vmcnt(0), a barrier and a load of the same bytes.
            // Window slot = (local row / 2) x (VW / 2) + (column - 1) / 2 of the tile's 6 x VW
            // positions (< 3 x 43 slots of 256 bytes), the 16 16-byte pieces of a slot rotated by the
            // slot so that neighbouring windows' pieces fall on different banks.
            __builtin_amdgcn_s_barrier();
            // (the slot bases are 256-byte aligned, so fragment pair j's piece is the lane's piece
            // for j = 0 with bits 6-7 flipped by 32 j: one XOR per access, four address registers)
            // (split: the lo-halo slot 1; the next tile's first DMA fills the hi slot 0)
            char* const xch = reinterpret_cast<char*>(lds + (SPLIT ? 1 : ((gc + cptk - 1) & 1)) * ASLOT);
            uint32_t xoff[MF];
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                const int k1 = wave * WROWS + i * 16 + er16 + 1;   // tile-local position + 1
                const int lr = fdiv(k1, g.VW, g.rv), xx = k1 - lr * g.VW;
                const int slot = (lr >> 1) * (g.VW >> 1) + ((xx - 1) >> 1);
                xoff[i] = qok[i] ? (uint32_t)(slot * 256 + (((cw >> 3) ^ slot) & 15) * 16) : 0u;
            }
#define OPK8_XCH(i_, j_) reinterpret_cast<uint4*>(xch + (xoff[i_] ^ (uint32_t)((j_) * 2)))
            if constexpr (SPLIT) {
                // Split precision: the window's winner is a (hi, lo) pair.  Per column pair the
                // even lane (the left column) keeps its own pair unless the right one's hi + lo is
                // larger; the first-row lanes leave the winner's hi and lo in the window slot, the
                // second-row lanes take the larger of the two rows (the first on ties) -- bit for
                // bit maxpool2_split_kernel over the stored pairs.  A slot holds hi and lo of four
                // of the eight 16-channel fragments, so the fragment pairs go in two halves, with
                // a barrier before the second half reuses the slots.
                static_assert(NF == 8 || NF == 4, "split pooled epilogue: 128 / 64-channel n-blocks");
#pragma unroll
                for (int hh = 0; hh < NF / 4; ++hh) {
                    uint4 kh[MF][2], kl[MF][2];
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj) {
                        const int j = 4 * hh + 2 * jj;
                        float4_t bq[2], mq[2];
#pragma unroll
                        for (int k = 0; k < 2; ++k) {
                            bq[k] = *reinterpret_cast<const float4_t*>(lb + (j + k) * 64);
                            mq[k] = *reinterpret_cast<const float4_t*>(lb + BN * 4 + (j + k) * 64);
                        }
#pragma unroll
                        for (int i = 0; i < MF; ++i) {
                            uint32_t ph[2][2], pl[2][2];
#pragma unroll
                            for (int h = 0; h < 2; ++h) {
                                const float4_t t = acc[i][j + h] * a.wscale + bq[h];
                                const float4_t tm = t * mq[h];
                                _Float16 wh[4], wl[4];
#pragma unroll
                                for (int r = 0; r < 4; ++r) {
                                    const float v = act_pick<MX>(t[r], tm[r]);
                                    const float o = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
                                        __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
                                    const _Float16 hv = (_Float16)v, ho = (_Float16)o;
                                    const _Float16 lv = (_Float16)(v - (float)hv), lo = (_Float16)(o - (float)ho);
                                    const bool right = (float)ho + (float)lo > (float)hv + (float)lv;
                                    wh[r] = right ? ho : hv;
                                    wl[r] = right ? lo : lv;
                                }
                                ph[h][0] = __builtin_bit_cast(uint32_t, (half2_t){wh[0], wh[1]});
                                ph[h][1] = __builtin_bit_cast(uint32_t, (half2_t){wh[2], wh[3]});
                                pl[h][0] = __builtin_bit_cast(uint32_t, (half2_t){wl[0], wl[1]});
                                pl[h][1] = __builtin_bit_cast(uint32_t, (half2_t){wl[2], wl[3]});
                            }
                            const auto sl = __builtin_amdgcn_permlane16_swap(ph[0][0], ph[1][0], false, false);
                            const auto sh = __builtin_amdgcn_permlane16_swap(ph[0][1], ph[1][1], false, false);
                            const auto ll = __builtin_amdgcn_permlane16_swap(pl[0][0], pl[1][0], false, false);
                            const auto lh = __builtin_amdgcn_permlane16_swap(pl[0][1], pl[1][1], false, false);
                            kh[i][jj] = make_uint4(sl[0], sh[0], sl[1], sh[1]);
                            kl[i][jj] = make_uint4(ll[0], lh[0], ll[1], lh[1]);
                            if (qok[i] && first[i]) {   // hi at pieces ^ {0, 4}, lo at ^ {8, 12}
                                *OPK8_XCH(i, 2 * jj * 16) = kh[i][jj];
                                *OPK8_XCH(i, (2 * jj + 4) * 16) = kl[i][jj];
                            }
                        }
                    }
                    __syncthreads();   // (the first rows' pairs are in LDS)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                        for (int i = 0; i < MF; ++i) {
                            const int j = 4 * hh + 2 * jj;
                            uint4 h1 = *OPK8_XCH(i, 2 * jj * 16), l1 = *OPK8_XCH(i, (2 * jj + 4) * 16);
                            opk8_pair_max(h1, l1, kh[i][jj], kl[i][jj]);   // (second-row lanes)
                            if constexpr (BST) {
                                __builtin_amdgcn_raw_buffer_store_b128((opk8_u4){h1.x, h1.y, h1.z, h1.w}, rs0,
                                                                       (int)(qo2[i] + j * 32), 0, 0);
                                __builtin_amdgcn_raw_buffer_store_b128((opk8_u4){l1.x, l1.y, l1.z, l1.w}, rs0lo,
                                                                       (int)(qo2[i] + j * 32), 0, 0);
                            } else {
                                const size_t o = cw + j * 16 + (size_t)qrow[i] * cs0;
                                const bool st = qok[i] && !first[i];
                                *(st ? reinterpret_cast<uint4*>(d0 + o) : sink4) = h1;
                                *(st ? reinterpret_cast<uint4*>(d0lo + o) : sink4) = l1;
                            }
                        }
                    if (hh + 1 < NF / 4) __syncthreads();   // (every wave read the first half: slots reused)
                }
            } else {
            uint4 keep[MF][NF / 2];
#pragma unroll
            for (int j = 0; j < NF; j += 2) {
                float4_t bq[2], mq[2];
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    bq[k] = *reinterpret_cast<const float4_t*>(lb + (j + k) * 64);
                    mq[k] = *reinterpret_cast<const float4_t*>(lb + BN * 4 + (j + k) * 64);
                }
#pragma unroll
                for (int i = 0; i < MF; ++i) {
                    uint32_t pk[2][2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const float4_t t = acc[i][j + h] + bq[h];
                        const float4_t tm = t * mq[h];
                        float v[4], o[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            v[r] = act_pick<MX>(t[r], tm[r]);
                            // the column pair's max: lane ^ 1 holds the next position
                            o[r] = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(
                                __builtin_bit_cast(int, v[r]), 0xB1, 0xF, 0xF, false));
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r)   // (OPK_FAULT_POOL: a dev variant that
                            // reproduces round 3's miscompile -- element 0's partner for all four
                            // -- to show the per-layer test catches it; never built for the product)
                            v[r] = fmaxf(v[r], o[OPK_FAULT_POOL ? 0 : r]);
                        pk[h][0] = __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_t){v[0], v[1]}, half2_t));
                        pk[h][1] = __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_t){v[2], v[3]}, half2_t));
                    }
                    const auto sl = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
                    const auto sh = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
                    keep[i][j / 2] = make_uint4(sl[0], sh[0], sl[1], sh[1]);
                    if (qok[i] && first[i]) *OPK8_XCH(i, j * 16) = keep[i][j / 2];
                }
            }
            __syncthreads();   // (lgkmcnt(0) + barrier: the first rows are in LDS)
            uint4 got[MF][NF / 2];
#pragma unroll
            for (int j = 0; j < NF; j += 2)
#pragma unroll
                for (int i = 0; i < MF; ++i)
                    got[i][j / 2] = *OPK8_XCH(i, j * 16);   // (used by the second-row lanes only)
#pragma unroll
            for (int j = 0; j < NF; j += 2)
#pragma unroll
                for (int i = 0; i < MF; ++i) {
                    const uint4 x = keep[i][j / 2], y = got[i][j / 2];
                    uint4 r;
                    r.x = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(half2_t, x.x), __builtin_bit_cast(half2_t, y.x)));
                    r.y = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(half2_t, x.y), __builtin_bit_cast(half2_t, y.y)));
                    r.z = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(half2_t, x.z), __builtin_bit_cast(half2_t, y.z)));
                    r.w = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(half2_t, x.w), __builtin_bit_cast(half2_t, y.w)));
                    if constexpr (BST) {
                        __builtin_amdgcn_raw_buffer_store_b128((opk8_u4){r.x, r.y, r.z, r.w}, rs0,
                                                               (int)(qo2[i] + j * 32), 0, 0);
                    } else {
                        uint4* p = reinterpret_cast<uint4*>(d0 + cw + j * 16 + (size_t)qrow[i] * cs0);
                        *(qok[i] && !first[i] ? p : sink4) = r;
                    }
                }
            }   // (fp16 pooled epilogue)
#undef OPK8_XCH
        } else {
        // one destination under 2 GiB (BST, host): buffer stores, masked lanes out of range
#pragma unroll
        for (int j = 0; j < NF; j += 2) {
            float4_t bq[2], mq[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                bq[k] = *reinterpret_cast<const float4_t*>(lb + (j + k) * 64);
                mq[k] = *reinterpret_cast<const float4_t*>(lb + BN * 4 + (j + k) * 64);
            }
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                uint32_t pk[2][2], pl[2][2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    // (split: the sums of the 2^e-scaled weights times 2^-e, exact; conv.h)
                    const float4_t t = (SPLIT ? acc[i][j + h] * a.wscale : acc[i][j + h]) + bq[h];
                    const float4_t v = act_pick4<MX>(t, t * mq[h]);
                    const half2_t h01 = __builtin_convertvector(v.xy, half2_t);
                    const half2_t h23 = __builtin_convertvector(v.zw, half2_t);
                    pk[h][0] = __builtin_bit_cast(uint32_t, h01);
                    pk[h][1] = __builtin_bit_cast(uint32_t, h23);
                    if constexpr (SPLIT) {   // lo = fp16(v - hi) (v - hi is exact in fp32)
                        pl[h][0] = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                            v.xy - __builtin_convertvector(h01, float2_t), half2_t));
                        pl[h][1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                            v.zw - __builtin_convertvector(h23, float2_t), half2_t));
                    }
                }
                const auto sl = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
                const auto sh = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
                const uint4 val = make_uint4(sl[0], sh[0], sl[1], sh[1]);
                uint4 lval = make_uint4(0, 0, 0, 0);
                if constexpr (SPLIT) {
                    const auto ll = __builtin_amdgcn_permlane16_swap(pl[0][0], pl[1][0], false, false);
                    const auto lh = __builtin_amdgcn_permlane16_swap(pl[0][1], pl[1][1], false, false);
                    lval = make_uint4(ll[0], lh[0], ll[1], lh[1]);
                }
                const int ch = cw + j * 16;
                if constexpr (BST) {
                    const uint32_t off = pok[i] ? (__umul24((uint32_t)prow[i], (uint32_t)cs0) + ch) * 2 : kBufOOB;
                    __builtin_amdgcn_raw_buffer_store_b128((opk8_u4){val.x, val.y, val.z, val.w}, rs0,
                                                           (int)off, 0, 0);
                    if constexpr (SPLIT)
                        __builtin_amdgcn_raw_buffer_store_b128((opk8_u4){lval.x, lval.y, lval.z, lval.w},
                                                               rs0lo, (int)off, 0, 0);
                } else if (nd == 1) {
                    const size_t o = ch + (size_t)prow[i] * cs0;
                    *(pok[i] ? reinterpret_cast<uint4*>(d0 + o) : sink4) = val;
                    if constexpr (SPLIT) *(pok[i] ? reinterpret_cast<uint4*>(d0lo + o) : sink4) = lval;
                } else {
                    for (int d = 0; d < nd; ++d) {
                        const size_t o = a.dst_coff[d] + nblk * BN + ch + (size_t)prow[i] * a.dst_cs[d];
                        *(pok[i] ? reinterpret_cast<uint4*>(a.dst[d] + o) : sink4) = val;
                        if constexpr (SPLIT)
                            *(pok[i] ? reinterpret_cast<uint4*>(a.dst_lo[d] + o) : sink4) = lval;
                    }
                }
            }
        }
        }
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < NF; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
        if (!has_next) break;
        m = mn;
        gc += cptk;
        OPK8_AROW(aoff, m);
    }
#undef OPK8_TAP
#undef OPK8_STEP
#undef OPK8_WAIT
#undef OPK8_RA
#undef OPK8_RB
#undef OPK8_ABASE
#undef OPK8_BBASE
#undef OPK8_ISSUE
#undef OPK8_AROW
#undef OPK8_AROW1
#undef OPK8_P0
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

#undef OPK8_DSR

}  // namespace

bool conv3w8_supported(const ConvArgs& a)
{
    // one 16-byte store per (fragment pair, destination), 16-byte aligned slices; several
    // destinations (conv4_4_CPM's five concat slices) wait for every store at a tile's first
    // mid-unit instead of counting them
    bool aligned = a.ndst >= 1 && a.ndst <= kConvMaxDst;
    for (int d = 0; d < a.ndst; ++d) aligned = aligned && ((a.dst_coff[d] | a.dst_cs[d]) & 7) == 0;
    // 64, 96 or 128 channels, or several 128-channel blocks (the VGG 256 / 512-channel layers)
    const bool nb_ok = a.cout == 64 || a.cout == 96 || a.cout == 128 || a.cout == 256 || a.cout == 512;
    return a.ntaps == 9 && nb_ok && a.sink && a.cus > 0 && !a.out32 && aligned &&
           a.sw + 2 * a.border > 16;
}

bool conv3w8_pool_supported(const ConvArgs& a)
{
    // windows never straddle a strip or a 6-row tile: even sizes, even strips, 1-pixel border;
    // the pooled image is dst[0] (one destination)
    return conv3w8_supported(a) && (a.cout % 128 == 0 || a.cout == 64) && a.ndst == 1 && a.border == 1 &&
           a.H % 2 == 0 && a.W % 2 == 0 && a.sw % 2 == 0 && 6 * (a.sw + 2) <= k8_BM;
}

void launch_conv3w8(const ConvArgs& a, hipStream_t stream)
{
    OPK_CHECK_ARG(conv3w8_supported(a), "conv3w8: 96 or k x 128 output channels, 3x3, one aligned slice");
    const long total = (long)a.frames * a.nstrips * (a.H + 2 * a.border) * (a.sw + 2 * a.border);
    const int VW = a.sw + 2 * a.border;
    const bool pool = a.pool != 0;
    if (pool)
        OPK_CHECK_ARG(conv3w8_pool_supported(a), "conv3w8 + pool: even H, W and strips, 64 / 128k outputs, border 1");
    const long ntm = pool ? (total / VW - 1 + 5) / 6 : (total + k8_BM - 1) / k8_BM;
    const int nb = a.cout <= 128 ? 1 : a.cout / 128;
    // a multiple of the n-block count (each block keeps one n-block)
    const unsigned G = (unsigned)(std::min<long>(a.cus / nb, ntm) * nb);
    OPK_CHECK_ARG(G >= 1 && G <= 1024, "persistent grid exceeds the sink");
    // buffer-resource epilogue stores (BUFST=0: pointer stores, A/B): one destination whose
    // positions x channel stride fit the 31-bit offsets of the raw buffer range check
    ConvArgs b = a;
    const long extent = ((long)a.frames * (a.H + 2 * a.border) * (a.W + 2 * a.border) + kConvGuardTail) *
                        a.dst_cs[0] * 2;
    const long pextent = ((long)a.frames * (a.H / 2 + 2) * (a.W / 2 + 2) + kConvGuardTail) * a.dst_cs[0] * 2;
    b.bufst = a.ndst == 1 && (pool ? pextent : extent) < (1L << 31) - 4096 && dev_switch("BUFST", 1) != 0;
    // n-blocks by XCD (W8_NBX=1, dev A/B): measured neutral in both precisions (round 6,
    // profiles/round6/r6c: split 104.0 vs 104.1 ms, fp16 33.6 vs 33.6 ms per 130-frame forward),
    // so the m-tile-major order stays the default
    b.nbx = nb > 1 && G % 8 == 0 && dev_switch("W8_NBX", 0) != 0;
#define OPK8_LAUNCH3(BN_, NB_, P_, MX_, SP_)                                                     \
    do {                                                                                        \
        note_launch("conv3w8_kernel<%d,%d,%d,%d,%d%s>", BN_, NB_, (int)P_, (int)MX_, b.bufst,     \
                    SP_ ? ",split" : "");                                                       \
        if (b.bufst)                                                                            \
            hipLaunchKernelGGL((conv3w8_kernel<BN_, NB_, P_, MX_, true, SP_>), dim3(G), dim3(64 * k8_NW), 0, stream, b); \
        else                                                                                    \
            hipLaunchKernelGGL((conv3w8_kernel<BN_, NB_, P_, MX_, false, SP_>), dim3(G), dim3(64 * k8_NW), 0, stream, b); \
    } while (0)
#define OPK8_LAUNCH2(BN_, NB_, P_, MX_)                                                          \
    do {                                                                                        \
        if (a.split) OPK8_LAUNCH3(BN_, NB_, P_, MX_, true);                                     \
        else OPK8_LAUNCH3(BN_, NB_, P_, MX_, false);                                            \
    } while (0)
#define OPK8_LAUNCH(BN_, NB_, P_)                                                                \
    do {                                                                                        \
        if (a.actmax) OPK8_LAUNCH2(BN_, NB_, P_, true);                                         \
        else OPK8_LAUNCH2(BN_, NB_, P_, false);                                                 \
    } while (0)
    OPK_CHECK_ARG(!a.split || (a.in_lo && a.dst_lo[0]), "conv3w8 split: lo twins");
    if (pool) {
        if (nb == 4) OPK8_LAUNCH(128, 4, true);
        else if (nb == 2) OPK8_LAUNCH(128, 2, true);
        else if (a.cout == 64) OPK8_LAUNCH(64, 1, true);
        else OPK8_LAUNCH(128, 1, true);
    } else if (nb == 4) OPK8_LAUNCH(128, 4, false);
    else if (nb == 2) OPK8_LAUNCH(128, 2, false);
    else if (a.cout == 128) OPK8_LAUNCH(128, 1, false);
    else if (a.cout == 96) OPK8_LAUNCH(96, 1, false);
    else OPK8_LAUNCH(64, 1, false);
#undef OPK8_LAUNCH
#undef OPK8_LAUNCH2
#undef OPK8_LAUNCH3
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
