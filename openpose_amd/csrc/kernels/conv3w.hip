// conv3w.hip -- 3x3 convolution: the persistent 16-wave halo implicit GEMM (conv3p_kernel,
// conv3.hip) with a K loop that never restarts its MFMAs from an empty pipeline.
//
// Role: Caffe ConvolutionLayer + fused PReLU/ReLU + concat-by-slice (netCaffe.cpp:248) for the
// single-n-block 3x3 layers of BODY_25's refinement stages (96 / 128 output channels at 46x82:
// ~45 % of the net's time at 64 frames).  Same tile (512 x BN, 16 waves of 64 x BN/2), operands,
// LDS layout and K order as conv3p_kernel, so the outputs are bit-identical; the schedule differs.
//
// conv3p_kernel, per K unit u = (chunk c, tap row ky):
//     wait own DMA of unit u; s_barrier; issue DMA of unit u+2; read tap 0's fragments; 3 taps.
// Every unit therefore starts with all 16 waves leaving a barrier together and waiting on their
// first LDS reads (the MFMA pipes idle meanwhile), and every tile starts behind a barrier that
// waits for the slowest wave's epilogue.  Round-1 PMC: MFMA busy 42 %, waves parked on
// waitcnt/barrier 43 %.
//
// Here, per unit:
//     tap 0, tap 1, [wait own DMA of unit u+1; s_barrier; issue DMA of unit u+2], tap 2,
//     and tap 2 ends by issuing the NEXT unit's tap-0 fragment reads.
// The barrier certifies unit u+1 one tap before it is needed (its DMA was issued a unit and a
// half earlier), so a wave reads the next unit's fragments as soon as its last MFMA of this unit
// is issued and continues without a barrier; the only barrier of a unit sits where 16 MFMAs per
// wave (a third of the unit) are still to come.  At a tile's last unit the epilogue (bias,
// ReLU/PReLU from LDS, fp16 pack, v_permlane16_swap pairs, 16-byte stores) runs after tap 2 with
// the next tile's first fragments already in flight, and no barrier separates it from the next
// tile's first two taps: waves leave their epilogue at different times and the early ones keep
// the MFMA pipe busy while the late ones still pack and store.
//
// WAR/RAW: the DMA issued at mid-unit u writes weight slot (u+2)%3 = that of unit u-1 and, when
// u+2 starts chunk c', halo slot of chunk c'-2 (last read in unit u-2); every wave passed the
// barrier only after issuing all its MFMAs of unit u-1.  Unit u+1's data is read after the
// barrier of mid-unit u, which every wave reaches after waiting for its own part of that DMA.
// vmcnt: loads, LDS-DMA and stores retire in issue order; the epilogue's S stores are the only
// VMEM ops younger than the DMA waited for at the next tile's mid-unit 0 (vmcnt(min(S, 63))).
#include "conv.h"

#include <algorithm>

#include "../common.h"
#include "conv3_dev.h"

namespace opk {

namespace {

using namespace conv3dev;

constexpr int kW_BM = 512, kW_HR = 688, kW_NW = 16;

#ifdef OPKW_STAMPS   // dev probe (tools/conv3w_probe.hip): per-block phase timestamps of wave 0
__device__ unsigned long long* opkw_stamps;
#define OPKW_STAMP(k_)                                                                        \
    do {                                                                                      \
        if (threadIdx.x == 0) opkw_stamps[blockIdx.x * 16 + (k_)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
// per-unit stamps of the block's second tile: [2u] before the mid-unit DMA wait, [2u+1] after
// the barrier
__device__ unsigned long long* opkw_ustamps;
#define OPKW_USTAMP(k_)                                                                       \
    do {                                                                                      \
        if (threadIdx.x == 0 && (k_) < 32) opkw_ustamps[blockIdx.x * 32 + (k_)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#define OPKW_RTSTAMP(k_)                                                                      \
    do {                                                                                      \
        if (threadIdx.x == 0) opkw_stamps[blockIdx.x * 16 + (k_)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define OPKW_STAMP(k_) do {} while (0)
#define OPKW_RTSTAMP(k_) do {} while (0)
#endif

#ifndef OPKW_STORE_MODE   // dev probe: 0 plain epilogue stores, 1 non-temporal
#define OPKW_STORE_MODE 0
#endif
typedef unsigned int opkw_u4 __attribute__((ext_vector_type(4)));
typedef unsigned int opkw_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void opkw_st(uint4* p, const uint4& v)
{
    if (OPKW_STORE_MODE == 1) __builtin_nontemporal_store((opkw_u4){v.x, v.y, v.z, v.w}, reinterpret_cast<opkw_u4*>(p));
    else *p = v;
}
__device__ __forceinline__ void opkw_st(uint2* p, const uint2& v)
{
    if (OPKW_STORE_MODE == 1) __builtin_nontemporal_store((opkw_u2){v.x, v.y}, reinterpret_cast<opkw_u2*>(p));
    else *p = v;
}

#ifndef OPKW_SPOL   // dev probe: cache policy bits of the epilogue buffer stores
#define OPKW_SPOL 0
#endif
// epilogue buffer stores (conv3_dev.h buf_rsrc: lanes at kBufOOB are dropped)
__device__ __forceinline__ void opkw_bst(const uint4& v, __amdgpu_buffer_rsrc_t r, uint32_t off)
{
    __builtin_amdgcn_raw_buffer_store_b128((opkw_u4){v.x, v.y, v.z, v.w}, r, (int)off, 0, OPKW_SPOL);
}
__device__ __forceinline__ void opkw_bst(const uint2& v, __amdgpu_buffer_rsrc_t r, uint32_t off)
{
    __builtin_amdgcn_raw_buffer_store_b64((opkw_u2){v.x, v.y}, r, (int)off, 0, OPKW_SPOL);
}

#ifndef OPKW_APOL   // dev probe: cache policy bits of the halo / weight DMA (gfx950: 1 sc0, 2 nt, 16 sc1)
#define OPKW_APOL 0
#endif
#ifndef OPKW_BPOL
#define OPKW_BPOL 0
#endif
#ifndef OPKW_ABLATE   // dev probe only (tools/conv3w_probe.hip): 1 no mid-unit barrier, 2 no MFMAs,
#define OPKW_ABLATE 0  // 3 no fragment reads, 4 no DMA after the prologue (timing only, wrong results)
#endif
#ifndef OPKW_HALO_SAME   // dev probe only: every chunk's halo DMA reads chunk 0's bytes (L2-warm
#define OPKW_HALO_SAME 0  // halo for chunks 1..: is the halo's HBM/MALL traffic the stall? wrong results)
#endif
#ifndef OPKW_DESYNC       // dev probe: workgroup group g = (blockIdx.x >> 3) % OPKW_DESYNC_N starts
#define OPKW_DESYNC 0     // g * OPKW_DESYNC cycles late, so the CUs' halo bursts fall apart in time
#endif
#ifndef OPKW_DESYNC_N
#define OPKW_DESYNC_N 2
#endif
#if OPKW_ABLATE == 3
#define OPKW_DSR(dst_, addr_, off_)                                                           \
    asm volatile("; no read %1" : "=v"(dst_) : "v"(addr_))
#else
#define OPKW_DSR(dst_, addr_, off_)                                                           \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst_) : "v"(addr_), "i"(off_))
#endif

// DMA_END (the default): issue unit u+2's DMA after tap 2 instead of right after the mid-unit
// barrier -- fewer registers live at the issue point (no spills), two thirds of a unit less lead
// time; measured 2-3 % faster on the stage layers.  CONV3W=2 selects the other placement (A/B).
// MX: the activation as max(t, t*m) (ConvArgs::actmax; conv3_dev.h act_pick)
// BST: one destination, epilogue stores through a buffer resource (ConvArgs::bufst)
template <int BN, bool DMA_END, bool MX, bool BST>
__global__ __launch_bounds__(64 * kW_NW, 1) void conv3w_kernel(const ConvArgs a)
{
    constexpr int NW = kW_NW, BM = kW_BM, HR = kW_HR;
    constexpr int WAVES_N = 2, WAVES_M = NW / WAVES_N;
    constexpr int WROWS = BM / WAVES_M, WN = BN / WAVES_N;
    static_assert(WROWS == 64 && (WN == 64 || WN == 48), "wave tiles 64 x 64 / 64 x 48");
    constexpr int MF = WROWS / 16, NF = WN / 16;
    constexpr int API = HR / 16, AIW = (API + NW - 1) / NW;
    constexpr int BROWS = 3 * BN, BPI = BROWS / 16, BIW = (BPI + NW - 1) / NW;
    constexpr int ASLOT = HR * 4, BSLOT = BROWS * 4;   // 16-byte pieces
    constexpr int LDS_PIECES = 2 * ASLOT + 3 * BSLOT + BN / 2;   // + bias and slope floats
    static_assert(LDS_PIECES * 16 <= 160 * 1024, "LDS budget");
    __shared__ uint4 lds[LDS_PIECES];
    float* lbias = reinterpret_cast<float*>(lds + 2 * ASLOT + 3 * BSLOT);
    float* lmul = lbias + BN;

    OPKW_STAMP(0);
    OPKW_RTSTAMP(14);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WAVES_N, wn = wave - (wave / WAVES_N) * WAVES_N;
    const int r16 = lane & 15, q = lane >> 4;
    const Strips g(a);
    const int ntm = (g.total + BM - 1) / BM;
    // XCD-aware bijective order of the persistent grid; block b walks m-tiles tix, tix + G, ...
    const int G = gridDim.x;
    const int xcd = blockIdx.x & 7, qq = G >> 3, rr = G & 7;
    const int tix = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (blockIdx.x >> 3);
    int m = tix;
    if (m >= ntm) return;
    if (OPKW_DESYNC > 0) {
        const unsigned long long d = (unsigned long long)(((blockIdx.x >> 3) % OPKW_DESYNC_N) * OPKW_DESYNC);
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        while (__builtin_amdgcn_s_memtime() - t0 < d) __builtin_amdgcn_s_sleep(2);
    }

    // bias and negative-side multiplier (1 none, 0 ReLU, slope PReLU) for the whole launch:
    // loaded into registers here, stored to LDS once the prologue's DMA wait has covered them
    // (a cold global load no longer delays the first DMA issue)
    float bias_v = 0.f, mul_v = 0.f;
    if (tid < BN) {
        const float neg = a.act == 1 ? 0.f : 1.f;
        bias_v = a.bias[tid];
        mul_v = a.act == 2 ? a.slope[tid] : neg;
    }

    const int lrow = lane >> 2, phys = lane & 3;
    const int cpt = a.cin_pad >> 5;
    const int U = 3 * cpt;
    const int bi = (BPI - wave + NW - 1) / NW;
    int boff[BIW];
#pragma unroll
    for (int j = 0; j < BIW; ++j) {
        const int rb = (j * NW + wave) * 16 + lrow;
        boff[j] = rb * 32 + (phys ^ (((rb >> 2) & 1) << 1)) * 8;
    }
    const char* abase = reinterpret_cast<const char*>(a.in + a.in_coff - a.in_cs);
    // halo row addresses (byte offsets from the position before the image) of this tile (aoff)
    // and of the block's next tile (aoffn; a tile past the end maps to the zeroed guard)
    uint32_t aoff[AIW], aoffn[AIW];
#define OPKW_AROW(dst_, mt_)                                                                  \
    do {                                                                                      \
        _Pragma("unroll") for (int i_ = 0; i_ < AIW; ++i_) {                                  \
            const int hr_ = (i_ * NW + wave) * 16 + lrow;                                     \
            const int lp_ = phys ^ (((hr_ >> 2) & 1) << 1);                                   \
            const long pos_ = g.pos((mt_) * BM - g.VW - 1 + hr_);                              \
            dst_[i_] = (uint32_t)(((pos_ + 1) * a.in_cs + lp_ * 8) * 2);                      \
        }                                                                                     \
    } while (0)
    // DMA of K unit (chunk c_, tap row ky_) into halo slot aslot_ / weight slot bslot_; the
    // halo rows of the current (nt_ = false) or the next tile
#define OPKW_ISSUE(c_, ky_, aslot_, bslot_, nt_)                                              \
    do {                                                                                      \
        if ((ky_) == 0) {                                                                     \
            const int as_ = (aslot_) * ASLOT;                                                 \
            _Pragma("unroll") for (int i_ = 0; i_ < AIW; ++i_)                                \
                if (API % NW == 0 || i_ * NW + wave < API)                                    \
                    __builtin_amdgcn_global_load_lds(                                         \
                        (const void*)(abase + (OPKW_HALO_SAME ? 0 : (c_)) * 64 + ((nt_) ? aoffn[i_] : aoff[i_])), \
                        (__attribute__((address_space(3))) void*)(&lds[as_ + (i_ * NW + wave) * 64]), \
                        16, 0, OPKW_APOL);                                                            \
        }                                                                                     \
        const int bs_ = 2 * ASLOT + (bslot_) * BSLOT;                                         \
        const uint16_t* ub_ = a.w + (size_t)((c_) * 3 + (ky_)) * BROWS * 32;                  \
        _Pragma("unroll") for (int j_ = 0; j_ < BIW; ++j_)                                    \
            if (BPI % NW == 0 || j_ * NW + wave < BPI) {                                      \
                int bo_ = boff[j_];                                                           \
                asm volatile("" : "+v"(bo_));                                                 \
                __builtin_amdgcn_global_load_lds(                                             \
                    (const void*)(ub_ + bo_),                                                 \
                    (__attribute__((address_space(3))) void*)(&lds[bs_ + (j_ * NW + wave) * 64]), \
                    16, 0, OPKW_BPOL);                                                                \
            }                                                                                 \
    } while (0)


    // fragment read bases: A row wm*64 + r16 + ky*VW + kx of a halo slot, B row kx*BN + wn*WN +
    // r16 of a weight slot; rows i*16 / j*16 / kx*BN keep row bit 2 (the swizzle bit), so the
    // fragments of one tap are constant offsets (1 KiB per 16 rows) from one base
    const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
    const int arow0 = wm * WROWS + r16;
    const uint32_t bswz = (uint32_t)swz64(wn * WN + r16, q) * 16;
    // (computed where used from a row the compiler cannot see through, so it does not hoist the
    // nine tap bases and three slot bases out of the loop into registers it would then spill)
#define OPKW_ABASE(slot_, ky_, kx_)                                                            \
    ({                                                                                        \
        int r_ = arow0 + (ky_) * g.VW + (kx_);                                                \
        asm volatile("" : "+v"(r_));                                                          \
        lds0 + (uint32_t)((slot_) * ASLOT * 16) + (uint32_t)swz64(r_, q) * 16;                \
    })
#define OPKW_BBASE(slot_)                                                                     \
    ({                                                                                        \
        uint32_t b_ = bswz;                                                                   \
        asm volatile("" : "+v"(b_));                                                          \
        lds0 + (uint32_t)((2 * ASLOT + (slot_) * BSLOT) * 16) + b_;                           \
    })

    half8_t fb[4], fa0, fa1;
    // the fragments of a tap's first step: NF B fragments, then A fragment 0
#define OPKW_READ_TAP0(ab_, bb_, boff_)                                                       \
    do {                                                                                      \
        OPKW_DSR(fb[0], bb_, (boff_) + 0);                                                    \
        OPKW_DSR(fb[1], bb_, (boff_) + 1024);                                                 \
        OPKW_DSR(fb[2], bb_, (boff_) + 2048);                                                 \
        if (NF > 3) OPKW_DSR(fb[3], bb_, (boff_) + 3072);                                     \
        OPKW_DSR(fa0, ab_, 0);                                                                \
    } while (0)
    // one tap: fragments of step 0 in flight; step i reads A fragment i+1 and waits for its own
    // (lgkmcnt(1): only the one just issued may still be outstanding; the last step waits for
    // all); then the next tap's step-0 fragments are issued (base nab_, nbb_ + nboff_)
#define OPKW_TAP(ab_, nab_, nbb_, nboff_, PF_, ZC_)                                           \
    do {                                                                                      \
        _Pragma("unroll") for (int i_ = 0; i_ < MF; ++i_) {                                   \
            half8_t& cur_ = (i_ & 1) ? fa1 : fa0;                                             \
            half8_t& nxt_ = (i_ & 1) ? fa0 : fa1;                                             \
            if (i_ + 1 < MF) {                                                                \
                switch (i_) {                                                                 \
                case 0: OPKW_DSR(nxt_, ab_, 1024); break;                                     \
                case 1: OPKW_DSR(nxt_, ab_, 2048); break;                                     \
                default: OPKW_DSR(nxt_, ab_, 3072); break;                                    \
                }                                                                             \
                if (i_ == 0)                                                                  \
                    asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(cur_), "+v"(fb[0]), "+v"(fb[1]), "+v"(fb[2]), "+v"(fb[3])); \
                else                                                                          \
                    asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(cur_));                        \
            } else {                                                                          \
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cur_));                            \
            }                                                                                 \
            _Pragma("unroll") for (int j_ = 0; j_ < NF; ++j_)                                 \
                acc[i_][j_] = OPKW_ABLATE == 2 ? acc[i_][j_] + (float)cur_[j_]                  \
                    : __builtin_amdgcn_mfma_f32_16x16x32_f16(                                   \
                          fb[j_], cur_, (ZC_) ? float4_t{0.f, 0.f, 0.f, 0.f} : acc[i_][j_], 0, 0, 0); \
            __builtin_amdgcn_sched_barrier(0);   /* keep the issue order as written */       \
        }                                                                                     \
        if (PF_) OPKW_READ_TAP0(nab_, nbb_, nboff_);                                          \
    } while (0)

    float4_t acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

    // ---- prologue: units 0 and 1 of the first tile in flight, unit 0 visible ----------------
    OPKW_AROW(aoff, m);
    OPKW_AROW(aoffn, m + G);
    OPKW_ISSUE(0, 0, 0, 0, false);
    OPKW_ISSUE(0, 1, 0, 1, false);
    vm_wait_rt(bi);   // (the bias loads are older than unit 0's DMA)
    if (tid < BN) {
        lbias[tid] = bias_v;
        lmul[tid] = mul_v;
    }
    __builtin_amdgcn_s_barrier();
    OPKW_STAMP(1);
    int tcount = 0;   // (dev probe) tiles done
    (void)tcount;

    int gc = 0;   // running chunk index of this tile's chunk 0 (halo slot parity)
    for (;;) {
        const int mn = m + G;
        const bool has_next = mn < ntm;
        const int p0 = m * BM;
        for (int u = 0; u < U; ++u) {
            const int c = u / 3, ky = u - 3 * (u / 3);
            const int aslot = (gc + c) & 1;
            const uint32_t bb_u = OPKW_BBASE(u % 3);
            const uint32_t ab0 = OPKW_ABASE(aslot, ky, 0);
            // tap 0's fragments: unit u was certified at mid-unit u-1 (no barrier here)
            OPKW_READ_TAP0(ab0, bb_u, 0);
            const uint32_t ab1 = OPKW_ABASE(aslot, ky, 1);
            // a tile's first tap starts its accumulators from the MFMA's zero C operand (no
            // per-tile zeroing of the 4 x NF accumulators after the epilogue; bit-identical)
            if (OPK_ZC && u == 0) OPKW_TAP(ab0, ab1, bb_u, BN * 64, true, OPK_ZC);
            else OPKW_TAP(ab0, ab1, bb_u, BN * 64, true, 0);
            const uint32_t ab2 = OPKW_ABASE(aslot, ky, 2);
            OPKW_TAP(ab1, ab2, bb_u, 2 * BN * 64, true, 0);
            // mid-unit: unit u+1's DMA landed (own part; vmcnt(0) also covers the previous
            // tile's epilogue stores, the only younger VMEM ops), then visible to all (barrier);
            // then the DMA of unit u+2 (into the slots of unit u-1 / chunk c-1) -- the next
            // tile's units 0 / 1 at a tile's last two units (after the block's last tile they
            // reload a guard region into free slots; never read)
#define OPKW_DMA_U2()                                                                         \
    do {                                                                                      \
        const bool nt_ = u + 2 >= U;                                                          \
        const int u2_ = nt_ ? u + 2 - U : u + 2;                                              \
        const int c2_ = u2_ / 3;                                                              \
        OPKW_ISSUE(c2_, u2_ - 3 * c2_, (gc + (nt_ ? cpt : 0) + c2_) & 1, (u + 2) % 3, nt_);  \
    } while (0)
#ifdef OPKW_STAMPS
            if (tcount == 0 && u == 3) OPKW_STAMP(8);
            if (tcount == 1) OPKW_USTAMP(2 * u);
#endif
            // DMA_END: at a tile's unit 0 the previous tile's epilogue stores (at least S1 of
            // them) are the only VMEM ops younger than unit 1's DMA -- leave them draining
            constexpr int S1 = MF * (NF / 2 + NF % 2);
            if (DMA_END && u == 0 && gc > 0) vm_wait<S1>();
            else vm_wait<0>();
#ifdef OPKW_STAMPS
            if (tcount == 0 && u == 3) OPKW_STAMP(9);
#endif
            if (OPKW_ABLATE != 1) __builtin_amdgcn_s_barrier();
#ifdef OPKW_STAMPS
            if (tcount == 0 && u == 3) OPKW_STAMP(10);
            if (tcount == 0 && u == 4) OPKW_STAMP(11);
            if (tcount == 1 && u == 0) OPKW_STAMP(12);
            if (tcount == 1) OPKW_USTAMP(2 * u + 1);
#endif
            if (!DMA_END && (OPKW_ABLATE != 4 || u + 2 >= U)) OPKW_DMA_U2();
            OPKW_TAP(ab2, ab2, bb_u, 0, false, 0);
            if (DMA_END && (OPKW_ABLATE != 4 || u + 2 >= U)) OPKW_DMA_U2();
#undef OPKW_DMA_U2
        }

#ifdef OPKW_STAMPS
        if (tcount < 2) OPKW_STAMP(2 + 2 * tcount);
#endif
        // ---- epilogue: bias + activation + fp16 pack, 16-byte stores (border lanes to the sink)
        // Per-lane constants are recomputed here from the lane id (v_mbcnt: no input register),
        // so no lane-dependent value lives across the K loop only to be spilled and reloaded --
        // a scratch reload's vmcnt(0) would wait for the next tile's DMA and these stores.
        const int el = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        const int er16 = el & 15, eq = el >> 4;
        int sidx = blockIdx.x * 64 * NW + wave * 64 + el;       // this lane's sink slot
        uint2* sink = reinterpret_cast<uint2*>(a.sink) + sidx;
        uint4* sink4 = reinterpret_cast<uint4*>(a.sink) + sidx;
        const int cw = wn * WN + 16 * (eq & 1) + 8 * (eq >> 1);  // channel of a lane's 16-byte store
        const int chl = wn * WN + 4 * eq;                        // first channel of a lane's fragment
        int prow[MF];   // padded-image positions (< 2^24, launch_conv3 checks)
        bool pok[MF];
        if (g.nstrips == 1) {   // (conv3_dev.h Strips::rows1)
            g.rows1<MF>(p0 + wm * WROWS + er16, a.W, prow, pok);
        } else {
            const int pbase = p0 + wm * WROWS + er16;
            int f, yy, xx, s;
            prow[0] = (int)g.map(pbase, f, yy, xx, s);
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
                // one strip: the virtual image is the padded image (no multiplies)
                prow[i] = !in ? 0 : g.nstrips == 1 ? pbase + i * 16 : (f * g.Hp + yy) * g.Wp + s * g.sw + xx;
                pok[i] = in && g.interior(yy, xx, s, a.W);
            }
        }
        // bias / negative-side multiplier of this lane's channel quads, read per fragment pair
        // with the pair's four LDS reads in flight at once (the compiler otherwise waits for each
        // read before its fragment); j0 = the pair's first fragment
        float4_t bq[2], mq[2];
        const char* lb = reinterpret_cast<const char*>(lbias) + (wn * WN + 4 * eq) * 4;
#define OPKW_BIAS(j0_, n_)                                                                    \
    do {                                                                                      \
        _Pragma("unroll") for (int k_ = 0; k_ < (n_); ++k_) {                                 \
            bq[k_] = *reinterpret_cast<const float4_t*>(lb + ((j0_) + k_) * 64);              \
            mq[k_] = *reinterpret_cast<const float4_t*>(lb + BN * 4 + ((j0_) + k_) * 64);     \
        }                                                                                     \
    } while (0)
#define OPKW_ACT(i_, j_, lo_, hi_)                                                            \
    do {                                                                                      \
        const float4_t t_ = acc[i_][j_] + bq[(j_) & 1];                                       \
        const float4_t v_ = act_pick4<MX>(t_, t_ * mq[(j_) & 1]);                             \
        lo_ = __builtin_bit_cast(uint32_t, __builtin_convertvector(v_.xy, half2_t));          \
        hi_ = __builtin_bit_cast(uint32_t, __builtin_convertvector(v_.zw, half2_t));          \
    } while (0)
        // destinations: one concat slice (every stage layer but conv4_4_CPM) with its pointer and
        // stride in SGPRs; a loop over the slices otherwise
        const int nd = a.ndst;
        uint16_t* const d0 = a.dst[0] + a.dst_coff[0];
        const int cs0 = a.dst_cs[0];
#ifndef OPKW_SINK_ONLY   // dev probe: every store to the sink (tile-transition store-burst test)
#define OPKW_SINK_ONLY 0
#endif
        // one destination under 2 GiB (host): buffer stores, masked lanes out of range
        const __amdgpu_buffer_rsrc_t rs0 = buf_rsrc(d0);
        uint32_t vrow[MF];
#pragma unroll
        for (int i = 0; i < MF; ++i)
            vrow[i] = BST && pok[i] && !OPKW_SINK_ONLY ? __umul24((uint32_t)prow[i], (uint32_t)(cs0 * 2)) : kBufOOB;
#define OPKW_STORE(T_, sink_, ch_, i_, val_)                                                  \
    do {                                                                                      \
        if constexpr (BST) {                                                                  \
            opkw_bst(val_, rs0, vrow[i_] + (ch_) * 2);                                        \
        } else if (nd == 1) {                                                                 \
            T_* p_ = reinterpret_cast<T_*>(d0 + (ch_) + (size_t)prow[i_] * cs0);              \
            opkw_st(pok[i_] && !OPKW_SINK_ONLY ? p_ : sink_, val_);                           \
        } else {                                                                              \
            for (int d_ = 0; d_ < nd; ++d_) {                                                 \
                T_* p_ = reinterpret_cast<T_*>(a.dst[d_] + a.dst_coff[d_] + (ch_) +           \
                                               (size_t)prow[i_] * a.dst_cs[d_]);              \
                opkw_st(pok[i_] ? p_ : sink_, val_);                                          \
            }                                                                                 \
        }                                                                                     \
    } while (0)
#pragma unroll
        for (int j = 0; j + 1 < NF; j += 2) {
            OPKW_BIAS(j, 2);
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                uint32_t lo0, hi0, lo1, hi1;
                OPKW_ACT(i, j, lo0, hi0);
                OPKW_ACT(i, j + 1, lo1, hi1);
                const auto sl = __builtin_amdgcn_permlane16_swap(lo0, lo1, false, false);
                const auto sh = __builtin_amdgcn_permlane16_swap(hi0, hi1, false, false);
                const uint4 val = make_uint4(sl[0], sh[0], sl[1], sh[1]);
                OPKW_STORE(uint4, sink4, cw + j * 16, i, val);
            }
        }
        if (NF % 2) {   // 96 channels: the last fragment as dwordx2
            OPKW_BIAS(NF - 1, 1);
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                uint32_t lo, hi;
                OPKW_ACT(i, NF - 1, lo, hi);
                const uint2 val = make_uint2(lo, hi);
                OPKW_STORE(uint2, sink, chl + (NF - 1) * 16, i, val);
            }
        }
#undef OPKW_STORE
#undef OPKW_BIAS
#undef OPKW_ACT
        if (!OPK_ZC) {
#pragma unroll
            for (int i = 0; i < MF; ++i)
#pragma unroll
                for (int j = 0; j < NF; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
        }
#ifdef OPKW_STAMPS
        if (tcount < 2) OPKW_STAMP(3 + 2 * tcount);
        ++tcount;
#endif
        if (!has_next) break;
        m = mn;
        gc += cpt;
#pragma unroll
        for (int i = 0; i < AIW; ++i) aoff[i] = aoffn[i];
        OPKW_AROW(aoffn, m + G);
    }
#undef OPKW_TAP
#undef OPKW_READ_TAP0
#undef OPKW_ABASE
#undef OPKW_BBASE
#undef OPKW_ISSUE
#undef OPKW_AROW
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    OPKW_STAMP(6);
    OPKW_RTSTAMP(15);
}

#undef OPKW_DSR

}  // namespace

bool conv3w_supported(const ConvArgs& a)
{
    bool aligned = true;   // 16-byte stores of 8-channel groups
    for (int d = 0; d < a.ndst; ++d) aligned = aligned && ((a.dst_coff[d] | a.dst_cs[d]) & 7) == 0;
    return a.ntaps == 9 && (a.cout == 128 || a.cout == 96) && a.sink && a.cus > 0 && !a.out32 &&
           aligned && a.sw + 2 * a.border > 16;
}

void launch_conv3w(const ConvArgs& a, hipStream_t stream)
{
    OPK_CHECK_ARG(conv3w_supported(a), "conv3w: 96 / 128 output channels, 3x3, aligned slices");
    const long total = (long)a.frames * a.nstrips * (a.H + 2 * a.border) * (a.sw + 2 * a.border);
    const long ntm = (total + kW_BM - 1) / kW_BM;
    const unsigned G = (unsigned)std::min<long>(a.cus, ntm);
    OPK_CHECK_ARG(G <= 1024, "persistent grid exceeds the sink");
    const bool dma_end = dev_switch("CONV3W", 1) != 2;   // 2: DMA right after the barrier (A/B)
    // buffer-resource epilogue stores (BUFST=0: pointer stores, A/B): one destination whose
    // positions x channel stride fit the 31-bit offsets of the raw buffer range check
    ConvArgs b = a;
    const long extent = ((long)a.frames * (a.H + 2 * a.border) * (a.W + 2 * a.border) + kConvGuardTail) *
                        a.dst_cs[0] * 2;
    b.bufst = a.ndst == 1 && extent < (1L << 31) - 4096 && dev_switch("BUFST", 1) != 0;
    // (the DMA-after-barrier A/B variant only with the select activation)
#define OPKW_LAUNCH(BN_, DE_, MX_)                                                                 \
    do {                                                                                          \
        note_launch("conv3w_kernel<%d,%d,%d,%d>", BN_, (int)DE_, (int)MX_, b.bufst);              \
        if (b.bufst)                                                                              \
            hipLaunchKernelGGL((conv3w_kernel<BN_, DE_, MX_, true>), dim3(G), dim3(64 * kW_NW), 0, stream, b); \
        else                                                                                      \
            hipLaunchKernelGGL((conv3w_kernel<BN_, DE_, MX_, false>), dim3(G), dim3(64 * kW_NW), 0, stream, b); \
    } while (0)
    if (a.cout == 128) {
        if (!dma_end) OPKW_LAUNCH(128, false, false);
        else if (a.actmax) OPKW_LAUNCH(128, true, true);
        else OPKW_LAUNCH(128, true, false);
    } else {
        if (!dma_end) OPKW_LAUNCH(96, false, false);
        else if (a.actmax) OPKW_LAUNCH(96, true, true);
        else OPKW_LAUNCH(96, true, false);
    }
#undef OPKW_LAUNCH
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
