// conv3.hip -- 3x3 convolutions on gfx950 MFMA with the input halo staged ONCE per channel chunk.
//
// Role: Caffe ConvolutionLayer + fused PReLU/ReLU + concat-by-slice (netCaffe.cpp:248) for every
// 3x3 layer of the net except conv1_1 (which reads the 3-channel image).  The implicit GEMM of
// conv2.hip re-reads each input row nine times (once per tap) and is bound by the per-CU LDS fill
// rate (profiles/round1); here each input row is staged once per 32-channel chunk.
//
// Row space ("virtual image").  The padded NHWC image [frames][H+2][W+2] is cut into vertical
// strips of sw interior columns (nstrips = ceil(W / sw); sw = W for narrow images).  Each strip is
// a padded image of width VW = sw + 2 that shares its two border columns with its neighbours; the
// virtual image is [frames][nstrips][H+2][VW] in row-major order.  The GEMM row space M is that
// virtual image (border rows/columns are computed and discarded), so every 3x3 tap is a constant
// shift ky*VW + kx of the whole tile, and a tile of BM consecutive virtual positions needs, for a
// 32-channel chunk, the virtual range [p0 - VW - 1, p0 + BM + VW + 1): one "halo" of HR rows x
// 64 B.  Strips keep the halo short (HR = BM + 256) for any image width.
//
// The K loop runs chunk-major, tap-minor in units (chunk c, ky):
//   * unit (c, 0) stages the halo of chunk c (A slot c & 1) and the 3 kx-taps' weights;
//   * units (c, 1), (c, 2) stage only their 3 taps' weights (B slot u % 3);
//   * every tap reads its A fragments from the SAME halo at row offset ky*VW + kx.
// Staging is global_load_lds_dwordx4 (lane-linear LDS) with the swizzle applied on the source
// address; 64-byte rows use piece ^ (((row >> 2) & 1) << 1), conflict-free for the unaligned row
// windows the taps read (brute-forced over all ds_read_b128 lane groups and window offsets).
//
// Tiles: BM x BN = 256 x 128 (8 waves as 4 x 2) or 512 x 64 (8 x 1); every wave owns 64 x 64.
// The MFMAs compute C^T (weights are the A operand) so each lane ends with 4 consecutive output
// channels of one position: the epilogue packs them to 8 fp16 bytes and stores straight from
// registers (no LDS pass).
#include "conv.h"

#include <algorithm>
#include <cstdlib>

#include "../common.h"
#include "conv3_dev.h"

namespace opk {

namespace {

using namespace conv3dev;

#ifndef OPK3_ABLATE
#define OPK3_ABLATE 0
#endif

#ifdef OPK3_STAMPS   // dev probe (tools/conv3_probe.hip): per-block phase timestamps
__device__ unsigned long long* opk3_stamps;
#define OPK3_STAMP(k_)                                                                        \
    do {                                                                                      \
        if (threadIdx.x == 0) {                                                               \
            opk3_stamps[blockIdx.x * 8 + (k_)] = __builtin_amdgcn_s_memtime();                \
            if ((k_) == 0) opk3_stamps[blockIdx.x * 8 + 6] = __builtin_amdgcn_s_memrealtime(); \
            if ((k_) == 5) opk3_stamps[blockIdx.x * 8 + 7] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                     \
    } while (0)
#else
#define OPK3_STAMP(k_) do {} while (0)
#endif


// TAPU: taps per K unit (3 = one ky row of taps, 1 = a single tap); MINB: workgroups per CU the
// LDS budget allows (2 -> 80 KB: the other workgroup's MFMAs cover this one's prologue, barrier
// and epilogue stalls).
// KS: 3 (3x3, pad 1) or 1 (1x1: the "halo" is the tile itself, one tap per chunk).
// NW: waves per workgroup (8, or 16 for the 512-row tiles of the one-per-CU variant).
// SPLIT: split precision (ConvArgs::split, conv.h) -- a separate instantiation, so the fp16 path
// is unchanged
template <int BM, int BN, int HR, int TAPU, int MINB, int KS, int NW = 8, bool SPLIT = false>
__global__ __launch_bounds__(64 * NW, MINB) __attribute__((amdgpu_waves_per_eu(NW / 4 * MINB)))
void conv3_kernel(const ConvArgs a)
{
    constexpr int WAVES_N = BN % 64 == 0 ? BN / 64 : 2, WAVES_M = NW / WAVES_N;
    constexpr int WROWS = BM / WAVES_M;            // wave tile WROWS x WN
    constexpr int WN = BN / WAVES_N;
    static_assert(WROWS % 16 == 0 && WROWS <= 128 && WN % 16 == 0 && WN <= 64, "wave tiles");
    static_assert(TAPU == 1 || TAPU == 3, "taps per unit");
    static_assert(KS == 3 || (KS == 7 && TAPU == 1) || (KS == 1 && TAPU == 1 && HR == BM),
                  "3x3, 7x7 (single-tap units) or 1x1 (one tap, halo = tile)");
    constexpr int MF = WROWS / 16, NF = WN / 16;
    constexpr int KT = KS * KS;                   // taps
    constexpr int UPC = KT / TAPU;                // units per 32-channel chunk
    constexpr int API = HR / 16;                  // halo DMA instructions per block (16 rows each)
    constexpr int AIW = (API + NW - 1) / NW;      // ... per wave, at most
    constexpr int BROWS = TAPU * BN;              // B rows per unit: tap-major, then channel n
    constexpr int BPI = BROWS / 16;               // B DMA instructions per block per unit
    constexpr int ASLOT = HR * 4;                 // 16-byte pieces per halo slot
    constexpr int NAS = UPC >= 2 ? 2 : 3;         // halo slots: unit u+2 may start chunk c+2 if UPC == 1
    constexpr int BSLOT = BROWS * 4;
    constexpr int LDS_PIECES = NAS * ASLOT + 3 * BSLOT;
    static_assert(HR % 16 == 0 && BROWS % 16 == 0, "DMA granularity");
    static_assert(LDS_PIECES * 16 * MINB <= 160 * 1024, "LDS budget");
    __shared__ uint4 lds[LDS_PIECES];

    OPK3_STAMP(0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave - (wave / WAVES_N) * WAVES_N;
    const Strips g(a);
    const int nn = (a.cout + BN - 1) / BN;
    // XCD-aware bijective tile order (see conv2.hip)
    const int nblk = gridDim.x;
    const int xcd = blockIdx.x & 7, qq = nblk >> 3, rr = nblk & 7;
    const int tix = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (blockIdx.x >> 3);
    const int p0 = (tix / nn) * BM;
    const int nb = tix - (tix / nn) * nn;
    const int n0 = nb * BN;

    // ---- DMA lane geometry: 16 rows x 4 pieces per wave instruction --------------------------
    const int lrow = lane >> 2, phys = lane & 3;
    const int cpt = a.cin_pad >> 5;               // 32-channel chunks of the input
    // split precision: three products per input chunk c, chunk-major -- virtual chunk 3c + k,
    // k = 0 x_hi w_lo, 1 x_hi w_hi (the hi halo of k = 0 again: no DMA), 2 x_lo w_hi (the lo
    // twin's halo; conv.h OPK_SPLIT_WLO_K); hi halos in slot 0 (UPC == 1: slots 0 / 2 by chunk
    // parity), lo halos in slot 1
    const int cptk = SPLIT ? 3 * cpt : cpt;       // K (virtual) chunks
    const int U = UPC * cptk;                     // units (chunk, taps)
    const ptrdiff_t dlo = SPLIT ? a.in_lo - a.in : 0;   // hi -> lo twin (elements)
    // halo row hr = (i*8 + wave)*16 + lrow holds virtual position p0 - VW - 1 + hr; its image
    // address (chunk 0, swizzled piece) is fixed for the whole tile
    const uint16_t* arow[AIW];
#pragma unroll
    for (int i = 0; i < AIW; ++i) {
        const int hr = (i * NW + wave) * 16 + lrow;
        const int lp = phys ^ (((hr >> 2) & 1) << 1);
        int yy, xx, s;
        int f;
        const long pos = g.template map<false>(p0 - (KS / 2) * (g.VW + 1) + hr, f, yy, xx, s);
        arow[i] = a.in + a.in_coff + pos * a.in_cs + lp * 8;
    }
    // this wave issues halo instructions i*8 + wave < API and B instructions j*8 + wave < BPI
    const int ai = (API - wave + NW - 1) / NW;
    const int bi = (BPI - wave + NW - 1) / NW;
    // split: the packed weights hold w_hi and w_lo (2 cpt chunks per n-block); virtual chunk
    // 3c + k reads w_lo chunk c (cpt + c) for k = OPK_SPLIT_WLO_K (conv.h), w_hi chunk c
    // otherwise -- OPK3_WUNIT (the order of conv3w8_kernel, so the two stay bit-identical)
    const uint16_t* wbase = a.w + (size_t)nb * (SPLIT ? 2 * cpt : cpt) * KT * BN * 32;
#define OPK3_WUNIT(u_)                                                                        \
    (!SPLIT ? (u_) : ({                                                                       \
        const int cc_ = (u_) / UPC;                                                           \
        const int wc_ = cc_ % 3 == OPK_SPLIT_WLO_K ? cpt + cc_ / 3 : cc_ / 3;                 \
        wc_ * UPC + ((u_) - cc_ * UPC);                                                       \
    }))
    // halo slot of virtual chunk c_ and whether its first unit issues a halo DMA
#define OPK3_ASLOT(c_) (!SPLIT ? (c_) % NAS : ((c_) % 3 == 2 ? 1 : (UPC == 1 ? 2 * (((c_) / 3) & 1) : 0)))
#define OPK3_HALO(c_) (!SPLIT || (c_) % 3 != 1)

#define OPK3_ISSUE(u_)                                                                        \
    do {                                                                                      \
        const int c_ = (u_) / UPC;                                                            \
        /* dev probe only: 6 = no halo DMA, 7 = no weight DMA after the prologue */           \
        if ((u_) - c_ * UPC == 0 && OPK3_HALO(c_) && (OPK3_ABLATE != 6 || (u_) < 2)) {       \
            const int as_ = OPK3_ASLOT(c_) * ASLOT;                                           \
            /* split: k = 2 reads the lo twin, k = 0 the hi image */                          \
            const ptrdiff_t ao_ = !SPLIT ? (ptrdiff_t)c_ * 32                                  \
                                         : (ptrdiff_t)(c_ / 3) * 32 + (c_ % 3 == 2 ? dlo : 0); \
            _Pragma("unroll") for (int i_ = 0; i_ < AIW; ++i_)                                \
                if (API % NW == 0 || i_ * NW + wave < API)                                    \
                    __builtin_amdgcn_global_load_lds(                                         \
                        (const void*)(arow[i_] + ao_),                                        \
                        (__attribute__((address_space(3))) void*)(&lds[as_ + (i_ * NW + wave) * 64]), \
                        16, 0, 0);                                                            \
        }                                                                                     \
        const int bs_ = NAS * ASLOT + ((u_) % 3) * BSLOT;                                     \
        const uint16_t* ub_ = wbase + (size_t)OPK3_WUNIT(u_) * BROWS * 32;                    \
        _Pragma("unroll") for (int j_ = 0; j_ < (BPI + NW - 1) / NW; ++j_) {                  \
            if ((BPI % NW == 0 || j_ * NW + wave < BPI) && (OPK3_ABLATE != 7 || (u_) < 2)) {  \
                const int rb_ = (j_ * NW + wave) * 16 + lrow;                                 \
                const int lp_ = phys ^ (((rb_ >> 2) & 1) << 1);                               \
                __builtin_amdgcn_global_load_lds(                                             \
                    (const void*)(ub_ + rb_ * 32 + lp_ * 8),                                  \
                    (__attribute__((address_space(3))) void*)(&lds[bs_ + (j_ * NW + wave) * 64]), \
                    16, 0, 0);                                                                \
            }                                                                                 \
        }                                                                                     \
    } while (0)

    float4_t acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

    const int r16 = lane & 15, q = lane >> 4;
    // bias and negative-side multiplier (1: identity, 0: ReLU, slope: PReLU) of this lane's
    // output channels; fetched before the K loop when registers allow (MINB == 1)
    float4_t bv[NF], mv[NF];
    const float neg = a.act == 1 ? 0.f : 1.f;
#define OPK3_BIAS()                                                                           \
    do {                                                                                      \
        _Pragma("unroll") for (int j_ = 0; j_ < NF; ++j_) {                                   \
            /* bias/slope arrays are zero-padded to a multiple of 128 channels */             \
            const int ch_ = n0 + wn * WN + j_ * 16 + 4 * q;                                   \
            bv[j_] = *reinterpret_cast<const float4_t*>(a.bias + ch_);                        \
            const float4_t sl_ = *reinterpret_cast<const float4_t*>(a.slope + ch_);           \
            mv[j_] = a.act == 2 ? sl_ : float4_t{neg, neg, neg, neg};                         \
        }                                                                                     \
    } while (0)
    // registers to spare across the K loop
    constexpr bool BIAS_EARLY = MINB == 1 && NW == 8 && MF * NF <= 16;
    if constexpr (BIAS_EARLY) OPK3_BIAS();

    OPK3_ISSUE(0);
    if (U > 1) OPK3_ISSUE(1);
    for (int u = 0; u < U; ++u) {
        const int c = u / UPC, t = u - (u / UPC) * UPC;
        // this wave's loads of unit u have landed once only unit u+1's may still be in flight
        // (unit u+1 carries a halo DMA when it starts a virtual chunk that stages one)
        vm_wait_rt(u + 1 < U ? bi + (t == UPC - 1 && OPK3_HALO(c + 1) ? ai : 0) : 0);
#if OPK3_ABLATE != 3   // dev probe only (3): no block barrier
        __builtin_amdgcn_s_barrier();
#endif
        if (u == 0) OPK3_STAMP(1);
#if OPK3_ABLATE == 2   // dev probe only: no DMA after the prologue (MFMA + LDS-read floor)
        if (u + 2 < U && u + 2 < 3) OPK3_ISSUE(u + 2);
#else
        if (u + 2 < U) OPK3_ISSUE(u + 2);
#endif
        const uint4* As = lds + OPK3_ASLOT(c) * ASLOT;
        const uint4* Bs = lds + NAS * ASLOT + (u % 3) * BSLOT;
#pragma unroll
        for (int k = 0; k < TAPU; ++k) {
            const int tap = t * TAPU + k;         // ky*KS + kx
            const int ky = tap / KS, kx = tap - KS * (tap / KS);
            half8_t fa[MF], fb[NF];
            const int hoff = ky * g.VW + kx;
#if OPK3_ABLATE == 4   // dev probe only: no fragment reads (register operands)
#pragma unroll
            for (int i = 0; i < MF; ++i) fa[i] = (half8_t)(_Float16)(hoff + i);
#pragma unroll
            for (int j = 0; j < NF; ++j) fb[j] = (half8_t)(_Float16)(k + j);
#else
#pragma unroll
            for (int i = 0; i < MF; ++i)
                fa[i] = __builtin_bit_cast(half8_t, As[swz64(wm * WROWS + i * 16 + r16 + hoff, q)]);
#pragma unroll
            for (int j = 0; j < NF; ++j)
                fb[j] = __builtin_bit_cast(half8_t, Bs[swz64(k * BN + wn * WN + j * 16 + r16, q)]);
#endif
#pragma unroll
            for (int i = 0; i < MF; ++i)
#pragma unroll
                for (int j = 0; j < NF; ++j)
#if OPK3_ABLATE == 1   // dev probe only: no MFMAs (data movement + sync floor)
                    acc[i][j][0] += (float)fb[j][0] * (float)fa[i][0];
#else
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa[i], acc[i][j], 0, 0, 0);
#endif
        }
    }
#undef OPK3_ISSUE
#undef OPK3_WUNIT
#undef OPK3_ASLOT
#undef OPK3_HALO
    OPK3_STAMP(2);
    if constexpr (!BIAS_EARLY) OPK3_BIAS();   // 128-VGPR variants: not kept across the K loop
#undef OPK3_BIAS

    // ---- epilogue straight from registers ------------------------------------------------------
    // lane (q, r16) of fragment (i, j) holds output channels ch..ch+3 (ch = n0 + wn*64 + j*16 + 4q)
    // of virtual position p0 + wm*64 + i*16 + r16; border and out-of-image positions are dropped.
    long prow[MF];
    bool pok[MF];
    int pbase = p0 + wm * WROWS + r16;
    asm volatile("" : "+v"(pbase));   // keep the position math after the K loop (register pressure)
    {   // fragment i is 16 virtual positions after fragment i-1: step the coordinates
        int f, yy, xx, s;
        prow[0] = g.map(pbase, f, yy, xx, s);
        pok[0] = g.interior(yy, xx, s, a.W);
#pragma unroll
        for (int i = 1; i < MF; ++i) {
            if (g.VW > 16) {
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
                prow[i] = in ? (long)(f * g.Hp + yy) * g.Wp + s * g.sw + xx : -1;
                pok[i] = in && g.interior(yy, xx, s, a.W);
            } else {
                int f2, yy2, xx2, s2;
                prow[i] = g.map(pbase + i * 16, f2, yy2, xx2, s2);
                pok[i] = g.interior(yy2, xx2, s2, a.W);
            }
        }
    }
    const int chl = n0 + wn * WN + 4 * q;   // this lane's first channel (fragment j adds 16 j)
    const bool vec = (a.cout & 3) == 0;
    // 16-byte stores (see conv3p_kernel): fragment pairs exchanged between lane rows q and q^1 by
    // v_permlane16_swap, each lane then holds 8 consecutive channels of its position.  Needs whole
    // 8-channel groups and 16-byte aligned destination slices; CONV3_WIDE=0 (opk_dev_set) disables.
    bool wide = NF % 2 == 0 && (a.cout & 7) == 0 && !a.out32 && a.wide;
    for (int d = 0; d < a.ndst; ++d) wide = wide && ((a.dst_coff[d] | a.dst_cs[d]) & 7) == 0;
    if (wide) {
        const int cw = n0 + wn * WN + 16 * (q & 1) + 8 * (q >> 1);
#pragma unroll
        for (int j = 0; j + 1 < NF; j += 2) {
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                uint32_t pk[2][2], pl[2][2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    // (split: the sums of the 2^e-scaled weights times 2^-e, exact; conv.h)
                    const float4_t t = (SPLIT ? acc[i][j + h] * a.wscale : acc[i][j + h]) + bv[j + h];
                    const float4_t tm = t * mv[j + h];
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = t[r] > 0.f ? t[r] : tm[r];
                    const half2_t h01 = __builtin_convertvector((float2_t){v[0], v[1]}, half2_t);
                    const half2_t h23 = __builtin_convertvector((float2_t){v[2], v[3]}, half2_t);
                    pk[h][0] = __builtin_bit_cast(uint32_t, h01);
                    pk[h][1] = __builtin_bit_cast(uint32_t, h23);
                    // split precision: lo = fp16(v - hi) (v - hi is exact in fp32)
                    pl[h][0] = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                        (float2_t){v[0], v[1]} - __builtin_convertvector(h01, float2_t), half2_t));
                    pl[h][1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                        (float2_t){v[2], v[3]} - __builtin_convertvector(h23, float2_t), half2_t));
                }
                // every lane takes part in the swap; masked lanes store nothing afterwards
                const auto sl = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
                const auto sh = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
                uint4 lval = make_uint4(0, 0, 0, 0);
                if constexpr (SPLIT) {
                    const auto ll = __builtin_amdgcn_permlane16_swap(pl[0][0], pl[1][0], false, false);
                    const auto lh = __builtin_amdgcn_permlane16_swap(pl[0][1], pl[1][1], false, false);
                    lval = make_uint4(ll[0], lh[0], ll[1], lh[1]);
                }
                if (!pok[i] || cw + j * 16 >= a.cout) continue;
                const uint4 val = make_uint4(sl[0], sh[0], sl[1], sh[1]);
                for (int d = 0; d < a.ndst; ++d) {
                    const size_t o = a.dst_coff[d] + cw + j * 16 + prow[i] * a.dst_cs[d];
                    *reinterpret_cast<uint4*>(a.dst[d] + o) = val;
                    if constexpr (SPLIT) *reinterpret_cast<uint4*>(a.dst_lo[d] + o) = lval;
                }
            }
        }
        OPK3_STAMP(5);
        return;
    }
    // fragment column j outer, row i inner: each (i, j) is activated, packed and stored at once
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        const float4_t bj = bv[j], mj = mv[j];
        const int ch = chl + j * 16;
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            // packed f32 math (v_pk_add/v_pk_mul) and v_cvt_pk_f16_f32 (round to nearest even)
            const float4_t t = (SPLIT ? acc[i][j] * a.wscale : acc[i][j]) + bj;
            const float4_t tm = t * mj;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = t[r] > 0.f ? t[r] : tm[r];
            if (!pok[i] || ch >= a.cout) continue;
            const half2_t h01 = __builtin_convertvector((float2_t){v[0], v[1]}, half2_t);
            const half2_t h23 = __builtin_convertvector((float2_t){v[2], v[3]}, half2_t);
            const uint32_t lo = __builtin_bit_cast(uint32_t, h01);
            const uint32_t hi = __builtin_bit_cast(uint32_t, h23);
            // split precision: the lo halves fp16(v - hi)
            const uint32_t llo = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                (float2_t){v[0], v[1]} - __builtin_convertvector(h01, float2_t), half2_t));
            const uint32_t lhi = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                (float2_t){v[2], v[3]} - __builtin_convertvector(h23, float2_t), half2_t));
            for (int d = 0; d < a.ndst; ++d) {
                const int cs = a.dst_cs[d];
                const size_t o = a.dst_coff[d] + ch + prow[i] * cs;
                uint16_t* p = a.dst[d] + o;
                if (vec && ((a.dst_coff[d] | cs) & 3) == 0) {
#if OPK3_ABLATE == 5   // dev probe only: no output stores
                    asm volatile("" ::"v"(lo), "v"(hi), "v"(p));
#else
                    *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
                    if constexpr (SPLIT) *reinterpret_cast<uint2*>(a.dst_lo[d] + o) = make_uint2(llo, lhi);
#endif
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (ch + e < a.cout) {
                            p[e] = (uint16_t)((e < 2 ? lo : hi) >> (16 * (e & 1)));
                            if constexpr (SPLIT) a.dst_lo[d][o + e] = (uint16_t)((e < 2 ? llo : lhi) >> (16 * (e & 1)));
                        }
                }
            }
            if (a.out32) {   // fp32 NCHW net output (the activations before fp16)
                int f, yy, xx, sx;
                (void)g.map(pbase + i * 16, f, yy, xx, sx);
                float* o = a.out32 + (((size_t)f * a.out32_c + a.out32_coff + ch) * a.H + yy - g.B) *
                                         a.W + sx * g.sw + xx - g.B;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (ch + r < a.cout) o[(size_t)r * a.H * a.W] = v[r];
            }
        }
    }
    OPK3_STAMP(5);
}

// ---- persistent 16-wave variant ---------------------------------------------------------------
// conv3p_kernel: the 512 x BN (128 or 96) tile with 3-tap K units of conv3_kernel<..., 16>, made
// persistent: one workgroup per CU walks its tiles and issues the next tile's first two K units
// during the current tile's last two, so every prologue (halo + weight DMA latency) overlaps the
// previous tile's epilogue.  Bias/slopes live in LDS for the whole launch.
//
// vmcnt counts stores as well as loads on gfx950 and retires in issue order, so the counted waits
// must know how many stores an epilogue issued: every (fragment pair, destination) issues exactly
// one 16-byte store, plus one 8-byte store per odd last fragment (lanes of border positions write
// to a scratch "sink"), S = MF*(NF/2 + NF%2)*ndst.

constexpr int kP_BM = 512, kP_HR = 688, kP_NW = 16;

// LDS fragment reads with explicit counters (ASMR): the compiler streams one fragment at a time
// behind s_waitcnt lgkmcnt(0) at the 128-VGPR budget (one LDS round trip per 4 MFMAs per wave);
// here the next A fragment is always in flight while the current one's MFMAs issue.  The wait is
// an asm statement that takes the fragments it covers as in/out operands, so every MFMA using
// them is ordered after it; inside the K loop no other LGKM traffic is outstanding (no SMEM, no
// compiler-issued LDS access), so the counts are exact.
#define OPK3_DSR(dst_, addr_, off_)                                                           \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst_) : "v"(addr_), "i"(off_))
template <int BN, bool ASMR, bool WIDE>
__global__ __launch_bounds__(64 * kP_NW, 1) void conv3p_kernel(const ConvArgs a)
{
    constexpr int NW = kP_NW, BM = kP_BM, HR = kP_HR;
    constexpr int WAVES_N = 2, WAVES_M = NW / WAVES_N;
    constexpr int WROWS = BM / WAVES_M, WN = BN / WAVES_N;
    static_assert(WROWS == 64 && WN % 16 == 0 && WN <= 64, "wave tiles");
    constexpr int MF = WROWS / 16, NF = WN / 16;
    constexpr int API = HR / 16, AIW = (API + NW - 1) / NW;
    constexpr int BROWS = 3 * BN, BPI = BROWS / 16, BIW = (BPI + NW - 1) / NW;
    constexpr int ASLOT = HR * 4, BSLOT = BROWS * 4;
    constexpr int LDS_PIECES = 2 * ASLOT + 3 * BSLOT + BN / 2;   // + bias and slope floats
    static_assert(LDS_PIECES * 16 <= 160 * 1024, "LDS budget");
    __shared__ uint4 lds[LDS_PIECES];
    float* lbias = reinterpret_cast<float*>(lds + 2 * ASLOT + 3 * BSLOT);
    float* lmul = lbias + BN;

    OPK3_STAMP(0);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave - (wave / WAVES_N) * WAVES_N;
    const int r16 = lane & 15, q = lane >> 4;
    const Strips g(a);
    const int nn = a.cout / BN;                   // cout % BN == 0 (host)
    const int ntm = (g.total + BM - 1) / BM;
    // XCD-aware bijective order; block -> (n-block, first m-tile); m-tiles stride by G / nn
    const int G = gridDim.x;
    const int xcd = blockIdx.x & 7, qq = G >> 3, rr = G & 7;
    const int tix = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (blockIdx.x >> 3);
    const int per_n = G / nn;
    const int nb = tix % nn;
    int m = tix / nn;
    const int n0 = nb * BN;
    if (m >= ntm) return;

    // bias and negative-side multiplier of this n-block, for the whole launch
    if (tid < BN) {
        const float neg = a.act == 1 ? 0.f : 1.f;
        lbias[tid] = a.bias[n0 + tid];
        lmul[tid] = a.act == 2 ? a.slope[n0 + tid] : neg;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    const int lrow = lane >> 2, phys = lane & 3;
    const int cpt = a.cin_pad >> 5;
    const int U = 3 * cpt;
    const int ai = (API - wave + NW - 1) / NW, bi = (BPI - wave + NW - 1) / NW;
    const uint16_t* wbase = a.w + (size_t)nb * cpt * 9 * BN * 32;
    int boff[BIW];
#pragma unroll
    for (int j = 0; j < BIW; ++j) {
        const int rb = (j * NW + wave) * 16 + lrow;
        boff[j] = rb * 32 + (phys ^ (((rb >> 2) & 1) << 1)) * 8;
    }
    // halo rows as 32-bit byte offsets from the position before the image (map() >= -1; buffers
    // hold < 2^31 elements): one VGPR each, SGPR base + VGPR offset addressing (measured faster on
    // the BODY_25 layers than 64-bit per-lane addresses)
    const char* abase = reinterpret_cast<const char*>(a.in + a.in_coff - a.in_cs);
    uint32_t aoff[AIW];
#define OPK3P_AROW(mt_)                                                                       \
    do {                                                                                      \
        _Pragma("unroll") for (int i_ = 0; i_ < AIW; ++i_) {                                  \
            const int hr_ = (i_ * NW + wave) * 16 + lrow;                                     \
            const int lp_ = phys ^ (((hr_ >> 2) & 1) << 1);                                   \
            int f_, yy_, xx_, s_;                                                             \
            const long pos_ = g.map((mt_) * BM - g.VW - 1 + hr_, f_, yy_, xx_, s_);           \
            aoff[i_] = (uint32_t)(((pos_ + 1) * a.in_cs + lp_ * 8) * 2);                      \
        }                                                                                     \
    } while (0)
    // K unit (chunk c_, tap row ky_) of the tile whose halo rows arow points at
#define OPK3P_ISSUE(c_, ky_, aslot_, bslot_)                                                  \
    do {                                                                                      \
        if ((ky_) == 0) {                                                                     \
            const int as_ = (aslot_) * ASLOT;                                                 \
            _Pragma("unroll") for (int i_ = 0; i_ < AIW; ++i_)                                \
                if (API % NW == 0 || i_ * NW + wave < API)                                    \
                    __builtin_amdgcn_global_load_lds(                                         \
                        (const void*)(abase + (c_) * 64 + aoff[i_]),                          \
                        (__attribute__((address_space(3))) void*)(&lds[as_ + (i_ * NW + wave) * 64]), \
                        16, 0, 0);                                                            \
        }                                                                                     \
        const int bs_ = 2 * ASLOT + (bslot_) * BSLOT;                                         \
        const uint16_t* ub_ = wbase + (size_t)((c_) * 3 + (ky_)) * BROWS * 32;                \
        _Pragma("unroll") for (int j_ = 0; j_ < BIW; ++j_)                                    \
            if (BPI % NW == 0 || j_ * NW + wave < BPI)                                        \
                __builtin_amdgcn_global_load_lds(                                             \
                    (const void*)(ub_ + boff[j_]),                                            \
                    (__attribute__((address_space(3))) void*)(&lds[bs_ + (j_ * NW + wave) * 64]), \
                    16, 0, 0);                                                                \
    } while (0)

    const int S = (WIDE ? MF * (NF / 2 + NF % 2) : MF * NF) * a.ndst;   // store instructions per epilogue and wave
    const bool exact = S + ai + bi <= 63;

    OPK3P_AROW(m);
    OPK3P_ISSUE(0, 0, 0, 0);
    OPK3P_ISSUE(0, 1, 0, 1);
    int gc = 0;                                   // running chunk index of this tile's chunk 0
    for (int it = 0;; ++it) {
        const int mn = m + per_n;
        const bool has_next = mn < ntm;
        const int p0 = m * BM;
        float4_t acc[MF][NF];
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < NF; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
        for (int u = 0; u < U; ++u) {
            const int c = u / 3, ky = u - 3 * (u / 3);
            // outstanding VMEM ops younger than unit u's loads: unit u+1's loads (this tile or the
            // next tile's unit 0), plus the previous epilogue's stores for units 0 and 1
            int younger = u + 1 < U ? bi + ((u + 1) % 3 == 0 ? ai : 0) : (has_next ? bi + ai : 0);
            if (it > 0 && u < 2 && exact) younger += S;
            vm_wait_rt64(younger);
            __builtin_amdgcn_s_barrier();
            if (u == 0 && it == 0) OPK3_STAMP(1);
            if (u == 0 && it == 1) OPK3_STAMP(3);
#define OPK3P_PREFETCH()                                                                      \
    do {                                                                                      \
        if (u + 2 < U) {                                                                      \
            const int c2 = (u + 2) / 3;                                                       \
            OPK3P_ISSUE(c2, (u + 2) - 3 * c2, (gc + c2) & 1, (u + 2) % 3);                    \
        } else if (has_next) {                                                                \
            if (u + 2 == U) OPK3P_AROW(mn);                                                   \
            OPK3P_ISSUE(0, u + 2 - U, (gc + cpt) & 1, (u + 2) % 3);                           \
        }                                                                                     \
    } while (0)
            OPK3P_PREFETCH();
            const uint4* As = lds + ((gc + c) & 1) * ASLOT;
            const uint4* Bs = lds + 2 * ASLOT + (u % 3) * BSLOT;
            if constexpr (ASMR) {
                static_assert(MF == 4 && NF >= 2 && NF <= 4, "ASMR fragment schedule");
                // rows i*16 / j*16 / kx*BN keep row bit 2, hence the swizzle: one lane base per
                // tap and operand, constant offsets (1 KiB per 16 rows)
                const uint32_t bb = (uint32_t)(uintptr_t)(Bs + swz64(wn * WN + r16, q));
                const int arow = wm * WROWS + r16 + ky * g.VW;
                uint32_t ab = (uint32_t)(uintptr_t)(As + swz64(arow, q));
                half8_t fb[4], fa0, fa1;
                OPK3_DSR(fb[0], bb, 0);
                OPK3_DSR(fb[1], bb, 1024);
                if (NF > 2) OPK3_DSR(fb[2], bb, 2048);
                if (NF > 3) OPK3_DSR(fb[3], bb, 3072);
                OPK3_DSR(fa0, ab, 0);
                if (a.prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
#pragma unroll
                    for (int i = 0; i < MF; ++i) {
                        half8_t& cur = (i & 1) ? fa1 : fa0;
                        half8_t& nxt = (i & 1) ? fa0 : fa1;
                        if (i + 1 < MF) {
                            switch (i) {
                            case 0: OPK3_DSR(nxt, ab, 1024); break;
                            case 1: OPK3_DSR(nxt, ab, 2048); break;
                            default: OPK3_DSR(nxt, ab, 3072); break;
                            }
                            // everything but the fragment just issued has landed
                            if (i == 0)
                                asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(cur), "+v"(fb[0]), "+v"(fb[1]), "+v"(fb[2]), "+v"(fb[3]));
                            else
                                asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(cur));
                        } else {
                            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cur));
                        }
#pragma unroll
                        for (int j = 0; j < NF; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], cur, acc[i][j], 0, 0, 0);
                        __builtin_amdgcn_sched_barrier(0);   // keep the issue order as written
                    }
                    if (kx < 2) {   // next tap: its weights and first A fragment
                        ab = (uint32_t)(uintptr_t)(As + swz64(arow + kx + 1, q));
                        const int bo = (kx + 1) * BN * 64;
                        OPK3_DSR(fa0, ab, 0);
                        switch (kx) {
                        case 0:
                            OPK3_DSR(fb[0], bb, BN * 64);
                            OPK3_DSR(fb[1], bb, BN * 64 + 1024);
                            if (NF > 2) OPK3_DSR(fb[2], bb, BN * 64 + 2048);
                            if (NF > 3) OPK3_DSR(fb[3], bb, BN * 64 + 3072);
                            break;
                        default:
                            OPK3_DSR(fb[0], bb, 2 * BN * 64);
                            OPK3_DSR(fb[1], bb, 2 * BN * 64 + 1024);
                            if (NF > 2) OPK3_DSR(fb[2], bb, 2 * BN * 64 + 2048);
                            if (NF > 3) OPK3_DSR(fb[3], bb, 2 * BN * 64 + 3072);
                            break;
                        }
                        (void)bo;
                    }
                }
                if (a.prio) __builtin_amdgcn_s_setprio(0);
            } else {
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                half8_t fa[MF], fb[NF];
                const int hoff = ky * g.VW + kx;
#pragma unroll
                for (int i = 0; i < MF; ++i)
                    fa[i] = __builtin_bit_cast(half8_t, As[swz64(wm * WROWS + i * 16 + r16 + hoff, q)]);
#pragma unroll
                for (int j = 0; j < NF; ++j)
                    fb[j] = __builtin_bit_cast(half8_t, Bs[swz64(kx * BN + wn * WN + j * 16 + r16, q)]);
#pragma unroll
                for (int i = 0; i < MF; ++i)
#pragma unroll
                    for (int j = 0; j < NF; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa[i], acc[i][j], 0, 0, 0);
            }
            }
        }
#undef OPK3P_PREFETCH
        if (it == 0) OPK3_STAMP(2);
        if (it == 1) OPK3_STAMP(4);

        // ---- epilogue: one 8-byte store per (fragment, destination), border lanes to the sink ----
        long prow[MF];
        bool pok[MF];
        {
            int pbase = p0 + wm * WROWS + r16;
            asm volatile("" : "+v"(pbase));
            int f, yy, xx, s;
            prow[0] = g.map(pbase, f, yy, xx, s);
            pok[0] = g.interior(yy, xx, s, a.W);
#pragma unroll
            for (int i = 1; i < MF; ++i) {   // VW > 16 (host): step 16 positions
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
                prow[i] = in ? (long)(f * g.Hp + yy) * g.Wp + s * g.sw + xx : 0;
                pok[i] = in && g.interior(yy, xx, s, a.W);
            }
        }
        const int chl = n0 + wn * WN + 4 * q;
        int sidx = blockIdx.x * 64 * NW + tid;    // this lane's sink slot
        asm volatile("" : "+v"(sidx));
        uint2* sink = reinterpret_cast<uint2*>(a.sink) + sidx;
        uint4* sink4 = reinterpret_cast<uint4*>(a.sink) + sidx;
        // bias + activation + fp16 pack of fragment (i, j): 4 channels of one position
#define OPK3P_ACT(i_, j_, lo_, hi_)                                                           \
    do {                                                                                      \
        const int cl_ = wn * WN + (j_) * 16 + 4 * q;   /* channel within the n-block */       \
        const float4_t t_ = acc[i_][j_] + *reinterpret_cast<const float4_t*>(lbias + cl_);    \
        const float4_t tm_ = t_ * *reinterpret_cast<const float4_t*>(lmul + cl_);             \
        float v_[4];                                                                          \
        _Pragma("unroll") for (int r_ = 0; r_ < 4; ++r_) v_[r_] = t_[r_] > 0.f ? t_[r_] : tm_[r_]; \
        lo_ = __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_t){v_[0], v_[1]}, half2_t)); \
        hi_ = __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_t){v_[2], v_[3]}, half2_t)); \
    } while (0)
        // fragment pairs (j, j+1): v_permlane16_swap of lane rows q <-> q^1 leaves every lane 8
        // consecutive channels of its position, 16 (j + (q & 1)) + 8 (q >> 1) .. + 7: one dwordx4
        // store per pair instead of two dwordx2 (the epilogue is store-issue bound)
        const int cw = n0 + wn * WN + 16 * (q & 1) + 8 * (q >> 1);
#pragma unroll
        for (int j = 0; WIDE && j + 1 < NF; j += 2) {
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                uint32_t lo0, hi0, lo1, hi1;
                OPK3P_ACT(i, j, lo0, hi0);
                OPK3P_ACT(i, j + 1, lo1, hi1);
                const auto sl = __builtin_amdgcn_permlane16_swap(lo0, lo1, false, false);
                const auto sh = __builtin_amdgcn_permlane16_swap(hi0, hi1, false, false);
                const uint4 val = make_uint4(sl[0], sh[0], sl[1], sh[1]);
                for (int d = 0; d < a.ndst; ++d) {
                    uint4* p = reinterpret_cast<uint4*>(a.dst[d] + a.dst_coff[d] + cw + j * 16 +
                                                        prow[i] * a.dst_cs[d]);
                    *(pok[i] ? p : sink4) = val;
                }
            }
        }
        // odd fragment count (96 channels): the last one as dwordx2; !WIDE (dev A/B): all of them
#pragma unroll
        for (int j = WIDE ? NF - NF % 2 : 0; j < NF; ++j) {
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                uint32_t lo, hi;
                OPK3P_ACT(i, j, lo, hi);
                for (int d = 0; d < a.ndst; ++d) {
                    uint2* p = reinterpret_cast<uint2*>(a.dst[d] + a.dst_coff[d] + chl + j * 16 +
                                                        prow[i] * a.dst_cs[d]);
                    *(pok[i] ? p : sink) = make_uint2(lo, hi);
                }
            }
        }
#undef OPK3P_ACT
        if (!has_next) break;
        m = mn;
        gc += cpt;
    }
#undef OPK3P_ISSUE
#undef OPK3P_AROW
    OPK3_STAMP(5);
}


}  // namespace

bool conv3_w8_eligible(int cout, int ntaps, int ndst, const int* dst_cs, const int* dst_coff, bool out32)
{
    return cout == 64 && ntaps == 9 && ndst == 1 && !out32 && ((dst_cs[0] | dst_coff[0]) & 7) == 0 &&
           dev_switch("CONV3W8_64", 1) != 0;
}

Conv3Shape conv3_shape(int frames, int H, int W, int cout, int ks, int border, bool w8)
{
    // variant switches (opk_dev_set; read per call so tests can compare variants in one process):
    // CONV3_SMALL=0 -> no two-per-CU tiles, CONV3_W16=0 -> no 16-wave tiles,
    // CONV3_PERSIST=0 -> 16-wave tiles without the persistent kernel
    const bool small = dev_switch("CONV3_SMALL", 1) != 0;
    const int big16 = dev_switch("CONV3_W16", 1);
    OPK_CHECK_ARG(ks == 1 || ks == 3 || ks == 7, "conv3: 1x1, 3x3 or 7x7");
    OPK_CHECK_ARG(border >= 1 && border >= ks / 2, "conv3: the zero border must cover the pad");
    Conv3Shape s;
    s.ks = ks;
    s.border = border;
    s.persist = false;
    s.bn = cout <= 64 ? 64 : (cout <= 96 ? 96 : 128);
    if (ks == 1) {   // no halo: small LDS (three tile slots), two workgroups per CU
        s.nw = 8;
        s.bm = 256;
        s.hr = s.bm;
        s.tapu = 1;
        s.minb = 2;
        s.nstrips = 1;
        s.sw = W;
        // dev A/B: CONV1_TILE=1 -> 512x128 tiles of 16 waves, 2 -> 256x256 tiles of 16 waves
        // (cout % 256 == 0): fewer tile rows staged per MFMA than 256x128
        // (default 2: measured -10..-20 % on the 384->512 and 288->256 layers)
        const int t1 = dev_switch("CONV1_TILE", 2);
        if (t1 == 1 && s.bn == 128) {
            s.bm = 512; s.hr = 512; s.nw = 16; s.minb = 1;
        } else if (t1 == 2 && cout % 256 == 0) {
            s.bn = 256; s.nw = 16; s.minb = 1;
        } else if (s.bn == 64 && dev_switch("CONV1_N64W16", 0) != 0) {   // dev A/B: 512x64, 16 waves
            s.bm = 512; s.hr = 512; s.nw = 16; s.minb = 1;
        }
        return s;
    }
    s.nw = 8;
    if (ks == 7) {   // 7x7 (COCO / MPI / face / hand stages): single-tap units, 1024-row halo
        s.bm = 256; s.hr = 1024; s.tapu = 1; s.minb = 1;
    } else {
        // two workgroups per CU pay off once every CU gets at least two 256-position tiles
        // (measured: +10-17 % on the 92x164 / 184x328 / 512-channel layers, -20 % at one tile per
        // CU)
        const long tiles = ((long)frames * (H + 2 * border) * (W + 2 * border) / 256) *
                           ((cout + s.bn - 1) / s.bn);
        // (measured, round 1: 4-wave 256x128 two-per-CU tiles and 8-wave 512x128 tiles of 128x64
        // wave tiles were both slower than these on every BODY_25 layer)
        if ((s.bn != 64 || w8) && big16 && tiles >= 3 * 256) {   // 512 x {128,96} tiles, 16 waves
            // (64 outputs: only for conv3w8's 8 waves of 64 x 64, conv3_w8_eligible)
            s.persist = dev_switch("CONV3_PERSIST", 1) != 0;
            // the persistent kernel keeps bias/slopes in LDS: 688 halo rows
            s.bm = 512; s.hr = s.persist ? kP_HR : 704; s.tapu = 3; s.minb = 1; s.nw = 16;
        } else if (small && tiles >= 2 * 256) {   // <= 80 KB of LDS
            s.bm = 256; s.hr = 448; s.tapu = 1; s.minb = 2;
        } else if (s.bn != 64) {
            s.bm = 256; s.hr = 512; s.tapu = 3; s.minb = 1;
        } else {
            s.bm = 512; s.hr = 768; s.tapu = 3; s.minb = 1;
        }
    }
    // halo: BM + (ks - 1) * (VW + 1) rows, VW = sw + 2 * border
    const int max_vw = (s.hr - s.bm - (ks - 1)) / (ks - 1);
    const int max_strip = max_vw - 2 * border;
    OPK_CHECK_ARG(max_strip >= 8, "conv3: border too wide for the halo");
    s.nstrips = (W + max_strip - 1) / max_strip;
    s.sw = (W + s.nstrips - 1) / s.nstrips;
    return s;
}

void launch_conv3(const ConvArgs& args, hipStream_t stream)
{
    ConvArgs a = args;   // + the reciprocals of the strip geometry (Strips::map, kernel arguments)
    if (a.border <= 0) a.border = 1;
    a.wide = dev_switch("CONV3_WIDE", 1);
    a.prio = dev_switch("CONV3P_PRIO", 0);
    const int B = a.border;
    a.rcp[0] = (float)(1.0 / ((double)(a.H + 2 * B) * (a.sw + 2 * B)));
    a.rcp[1] = (float)(1.0 / (double)(a.sw + 2 * B));
    a.rcp[2] = (float)(1.0 / (double)(a.nstrips > 0 ? a.nstrips : 1));
    const int ks = a.ntaps == 49 ? 7 : (a.ntaps == 9 ? 3 : 1);
    OPK_CHECK_ARG((a.ntaps == 49 || a.ntaps == 9 || a.ntaps == 1) && a.cin_pad % 32 == 0 &&
                      a.cin_pad > 0,
                  "7x7, 3x3 or 1x1, cin_pad % 32 == 0");
    OPK_CHECK_ARG(a.in_cs % 8 == 0 && a.in_coff % 8 == 0, "input slice must be 16-byte aligned");
    OPK_CHECK_ARG(a.in_coff + a.cin_pad <= a.in_cs, "input slice exceeds the buffer");
    OPK_CHECK_ARG(a.M > 0 && a.cout > 0 && a.ndst <= kConvMaxDst, "bad sizes");
    const bool w8 = conv3_w8_eligible(a);
    const Conv3Shape s = conv3_shape(a.frames, a.H, a.W, a.cout, ks, B, w8);
    OPK_CHECK_ARG(a.sw == s.sw && a.nstrips == s.nstrips, "strip geometry differs from conv3_shape");
    const int VW = s.sw + 2 * B;
    OPK_CHECK_ARG(ks == 1 || s.bm + (ks - 1) * (VW + 1) <= s.hr, "strip too wide for the halo");
    const long total = (long)a.frames * s.nstrips * (a.H + 2 * B) * VW;
    OPK_CHECK_ARG(total + s.bm + (long)(ks - 1) * (VW + 1) < (1L << 24), "too many positions per launch");
    const int nn = (a.cout + s.bn - 1) / s.bn;
    const long ntiles = ((total + s.bm - 1) / s.bm) * nn;
    dim3 grid((unsigned)ntiles);
    bool lo_ok = !a.split || a.in_lo;
    for (int d = 0; d < a.ndst && a.split; ++d) lo_ok = lo_ok && a.dst_lo[d];
    OPK_CHECK_ARG(lo_ok, "split precision: lo twins required");
    // conv + 2x2 max pool in one persistent kernel (conv3w8.hip POOL epilogue); the planner only
    // asks for it where conv3w8_pool_supported holds
    if (a.pool) {
        OPK_CHECK_ARG(s.nw == 16 && s.persist && VW > 16 && conv3w8_pool_supported(a),
                      "pool fusion requested for an unsupported conv");
        launch_conv3w8(a, stream);
        return;
    }
    // (a Winograd F(2,3)-along-x variant of the persistent kernel measured 15-50 % slower on every
    // BODY_25 layer -- LDS-read bound: 4 accumulators per output pair halve the wave tile, doubling
    // the fragment reads per MFMA; removed, source and numbers in profiles/round3/wino/)
    // several 128-channel n-blocks (the VGG 256 / 512-channel layers): conv3w8 with one n-block
    // per persistent block (bit-identical; CONV3W8N=0: the 16-wave conv3_kernel)
    // 64-output layers in the persistent geometry (both precisions): conv3w8's BN = 64 tile
    if (w8 && s.persist && s.bn == 64) {
        OPK_CHECK_ARG(s.nw == 16 && VW > 16 && conv3w8_supported(a), "conv3w8<64>: unsupported conv");
        launch_conv3w8(a, stream);
        return;
    }
    // split precision: every 512-position 96 / 128 / 256 / 512-channel 3x3 layer on conv3w8's split
    // instantiation (bit-identical to conv3_kernel's; SPLIT_W8=0: conv3_kernel, A/B) -- its three
    // times longer K loop is the regime where conv3w8 keeps the MFMA pipe busiest; the rest
    // (several destinations, the 64-channel full-resolution layer, 1x1 heads) on conv3_kernel
    if (a.split && s.nw == 16 && s.persist && s.bn != 64 && a.sink && !a.out32 && VW > 16 &&
        dev_switch("SPLIT_W8", 1) != 0 && conv3w8_supported(a)) {
        launch_conv3w8(a, stream);
        return;
    }
    if (!a.split && s.nw == 16 && s.persist && nn > 1 && s.bn == 128 && a.sink && !a.out32 && VW > 16 &&
        dev_switch("CONV3W8N", 1) != 0 && conv3w8_supported(a)) {
        launch_conv3w8(a, stream);
        return;
    }
    // measured: +3-10 % on the single-n-block layers, 3-8 % slower with 2-4 n-blocks (kept 16-wave)
    if (!a.split && s.nw == 16 && s.persist && nn == 1 && a.sink && a.cus >= nn && a.cout % s.bn == 0 &&
        !a.out32 && VW > 16) {
        bool aligned = true;
        // 16-byte stores of 8-channel groups
        for (int d = 0; d < a.ndst; ++d) aligned = aligned && ((a.dst_coff[d] | a.dst_cs[d]) & 7) == 0;
        // mid-unit-barrier schedule (conv3w.hip, bit-identical; CONV3W=0: conv3p_kernel)
        if (aligned && nn == 1 && dev_switch("CONV3W", 1) != 0 && conv3w_supported(a)) {
            // 8 waves of 64 x 128 (conv3w8.hip, bit-identical): 25 % fewer LDS fragment reads,
            // measured 2-4 % faster from cin 384 up and 4 % slower at cin 128 (tile transitions
            // weigh more there); CONV3W8=0 disables, 2 forces it for 128 outputs, 3 also for 96
            const int w8 = dev_switch("CONV3W8", 1);
            if (w8 != 0 && conv3w8_supported(a) &&
                ((a.cout == 128 && (a.cin_pad >= 384 || w8 >= 2)) || (a.cout == 96 && w8 == 3))) {
                launch_conv3w8(a, stream);
                return;
            }
            launch_conv3w(a, stream);
            return;
        }
        if (aligned) {   // one workgroup per CU, n-blocks spread evenly over the grid
            const long per_n = std::min<long>(a.cus / nn, (ntiles + nn - 1) / nn);
            const unsigned G = (unsigned)(per_n * nn);
            OPK_CHECK_ARG(G <= 1024, "persistent grid exceeds the sink");
            // (measured, round 1: a 32x32x16-MFMA version of this kernel with double-buffered
            // fragments ran 20 % slower on the 128-channel layers; a pipelined 16x16x32 fragment
            // schedule spilled at the 128-VGPR budget and ran 4 % slower; the explicit-counter
            // fragment schedule measured 1.5 % faster over the whole CNN, bit-identical)
            const bool asmr = dev_switch("CONV3P_ASMR", 1) != 0;
            // 16-byte epilogue stores (measured in tools/ab_asmr.sh; CONV3P_WIDE=0: dwordx2)
            const bool wide = dev_switch("CONV3P_WIDE", 1) != 0;
#define OPK3P_LAUNCH(BN_, ASMR_, WIDE_)                                                        \
    do {                                                                                       \
        note_launch("conv3p_kernel<%d,%d,%d>", BN_, (int)ASMR_, (int)WIDE_);                   \
        hipLaunchKernelGGL((conv3p_kernel<BN_, ASMR_, WIDE_>), dim3(G), dim3(1024), 0, stream, a); \
    } while (0)
            if (s.bn == 96) {
                if (asmr) { if (wide) OPK3P_LAUNCH(96, true, true); else OPK3P_LAUNCH(96, true, false); }
                else OPK3P_LAUNCH(96, false, true);
            } else {
                if (asmr) { if (wide) OPK3P_LAUNCH(128, true, true); else OPK3P_LAUNCH(128, true, false); }
                else OPK3P_LAUNCH(128, false, true);
            }
#undef OPK3P_LAUNCH
            OPK_LAUNCH_CHECK();
            return;
        }
    }
#define OPK3_LAUNCH(BM_, BN_, HR_, TAPU_, MINB_, KS_)                                          \
    do {                                                                                       \
        note_launch("conv3_kernel<%d,%d,%d,%d,%d,%d%s>", BM_, BN_, HR_, TAPU_, MINB_, KS_,      \
                    a.split ? ",8,split" : "");                                                \
        if (a.split)                                                                           \
            hipLaunchKernelGGL((conv3_kernel<BM_, BN_, HR_, TAPU_, MINB_, KS_, 8, true>), grid,  \
                               dim3(512), 0, stream, a);                                       \
        else                                                                                   \
            hipLaunchKernelGGL((conv3_kernel<BM_, BN_, HR_, TAPU_, MINB_, KS_>), grid, dim3(512), 0, \
                               stream, a);                                                     \
    } while (0)
#define OPK3_LAUNCH16(BM_, BN_, HR_, TAPU_, KS_)                                                \
    do {                                                                                       \
        note_launch("conv3_kernel<%d,%d,%d,%d,1,%d,16%s>", BM_, BN_, HR_, TAPU_, KS_,          \
                    a.split ? ",split" : "");                                                  \
        if (a.split)                                                                           \
            hipLaunchKernelGGL((conv3_kernel<BM_, BN_, HR_, TAPU_, 1, KS_, 16, true>), grid,     \
                               dim3(1024), 0, stream, a);                                      \
        else                                                                                   \
            hipLaunchKernelGGL((conv3_kernel<BM_, BN_, HR_, TAPU_, 1, KS_, 16>), grid, dim3(1024), 0, \
                               stream, a);                                                     \
    } while (0)
    if (ks == 7) {
        if (s.bn == 64) OPK3_LAUNCH(256, 64, 1024, 1, 1, 7);
        else if (s.bn == 96) OPK3_LAUNCH(256, 96, 1024, 1, 1, 7);
        else OPK3_LAUNCH(256, 128, 1024, 1, 1, 7);
    } else if (ks == 1) {
        if (s.nw == 16 && s.bn == 256) OPK3_LAUNCH16(256, 256, 256, 1, 1);
        else if (s.nw == 16 && s.bn == 64) OPK3_LAUNCH16(512, 64, 512, 1, 1);
        else if (s.nw == 16) OPK3_LAUNCH16(512, 128, 512, 1, 1);
        else if (s.bn == 64) OPK3_LAUNCH(256, 64, 256, 1, 2, 1);
        else if (s.bn == 96) OPK3_LAUNCH(256, 96, 256, 1, 2, 1);
        else OPK3_LAUNCH(256, 128, 256, 1, 2, 1);
    } else if (s.bn == 64) {
        if (s.minb == 2) OPK3_LAUNCH(256, 64, 448, 1, 2, 3);
        else OPK3_LAUNCH(512, 64, 768, 3, 1, 3);
    } else if (s.bn == 96) {
        if (s.nw == 16) OPK3_LAUNCH16(512, 96, 704, 3, 3);
        else if (s.minb == 2) OPK3_LAUNCH(256, 96, 448, 1, 2, 3);
        else OPK3_LAUNCH(256, 96, 512, 3, 1, 3);
    } else {
        if (s.nw == 16) OPK3_LAUNCH16(512, 128, 704, 3, 3);
        else if (s.minb == 2) OPK3_LAUNCH(256, 128, 448, 1, 2, 3);
        else OPK3_LAUNCH(256, 128, 512, 3, 1, 3);
    }
#undef OPK3_LAUNCH
#undef OPK3_LAUNCH16
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
