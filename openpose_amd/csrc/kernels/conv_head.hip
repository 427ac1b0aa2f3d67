// conv_head.hip -- a refinement stage's 1x1 head pair in one kernel: Mconv6 (1x1, N1 = 256 / 512
// outputs, PReLU/ReLU) -> Mconv7 (1x1, <= 64 outputs, no activation).
//
// Reference layers: models/pose/body_25/pose_deploy.prototxt Mconv6_stage*_L* / Mconv7_stage*_L*
// (run by NetCaffe::forwardPass, netCaffe.cpp:248).  Unfused, Mconv6 writes its N1-channel fp16
// output (264 MB per 64 frames at 46x82 for N1 = 512) and Mconv7 reads it back at HBM speed
// (profiles/round2: Mconv7 0.1-0.15 TF/s, 6 % of the CNN with Mconv6).  Here the Mconv6 tile never
// leaves the chip:
//   phase 1  Mconv6 as the usual implicit GEMM of a 128-position tile (1x1: the tile is its own
//            halo) x all N1 channels, 8 waves of 64 (or 32) positions x 128 channels, 32-channel K
//            steps through a 3-slot LDS ring (global_load_lds, swizzled 64-byte rows);
//   phase 2  bias + activation, fp16, and each wave's 64 x 128 block turned straight into MFMA
//            B operands: v_permlane16_swap of fragment pairs (j, j+1) gives a lane the 8 channels
//            16(q&1) + 8(q>>1) .. +7 of a 32-channel block -- a fixed permutation of the K order,
//            which the host applies to Mconv7's weights instead (conv_head_pack_w7) -- and
//            Mconv7's weights for the wave's 128 channels come from L2 into registers (per-tile
//            grid: from LDS, staged by one DMA at the last K step -- W7LDS below);
//   phase 3  the N1/128 partial products of a position block (one per wave column) are summed
//            through LDS in a fixed order (deterministic), + bias, fp16 into every concat slice and
//            the fp32 NCHW net output when requested.
// PERSIST: one workgroup per CU walks tiles (XCD-aware order): no workgroup turnover, the bias
// read once; the next tile's first two K steps are issued into the ring (which the partials
// alias) as soon as every wave has read its partial sums and issued its stores.
// SPLIT (split precision, HeadArgs::split): phase 1 runs three K steps per 32-channel chunk --
// x_hi w_hi, x_lo w_hi, x_hi w_lo, each a plain ring step with its own A and B sources -- into one
// fp32 accumulator; phase 2 scales by 2^-e6, activates and splits the Mconv6 value v into
// hi = fp16(v), lo = fp16(v - hi) (the pair the unfused layer would have stored) and runs Mconv7 as
// v_hi w7_hi + v_hi w7_lo + v_lo w7_hi; phase 3 scales by 2^-e7, adds the bias and stores the
// (hi, lo) pair.  Mconv7's weights come from L2 in both grids (no W7LDS: hi + lo fill the ring).
// MFMA f32_16x16x32_f16, C^T arrangement (weights as the A operand) as in conv3.hip.
#include "conv.h"

#include <algorithm>

#include "../common.h"
#include "conv3_dev.h"

namespace opk {

namespace {

using namespace conv3dev;

constexpr int kH_BM = 128, kH_NW = 8;

// MX: Mconv6's activation as max(t, t*m) (HeadArgs::actmax; conv3_dev.h act_pick4)
#ifndef OPKH_ABLATE   // dev probe only: 1 no Mconv6 weight DMA after a tile's first two K steps,
#define OPKH_ABLATE 0  // 2 no phase 2/3 work beyond the partial-sum barrier, 3 no phase 3 (timing
#endif                 // only, wrong results; profiles/round3/head_ablations/)
// W7LDS (per-tile grid, N1 = 256): Mconv7's weights reach phase 2 through LDS -- one DMA per tile
// into the two ring B slots that are free during the last K step, then one barrier -- instead of
// per-wave flat loads from L2 whose latency every 32-channel block of phase 2 waited for (4 exposed
// L2 round trips per tile; each fragment fetched by both waves of a wave column).  Measured
// (profiles/round3/head_w7/): N1 = 256 heads -12 % / -6 % (the CU's second workgroup covers the
// barrier); the persistent N1 = 512 heads +3.5 % / +6.6 % (one workgroup per CU: the DMA wait and
// barrier are exposed), so those keep the flat loads.  KSCHED (dev, off): a K step's fragment
// reads in consumption order with counted lgkmcnt waits -- measured neutral to +1 %.  Both only
// reorder data movement (bit-identical: tools/ab_outputs.py).
#ifndef OPKH_W7LDS
#define OPKH_W7LDS 1
#endif
#ifndef OPKH_KSCHED
#define OPKH_KSCHED 0
#endif
template <int N1, int NF2, bool PERSIST, bool MX, bool SPLIT>
__global__ __launch_bounds__(64 * kH_NW, 1) void conv_head_kernel(const HeadArgs a)
{
    constexpr int NW = kH_NW, BM = kH_BM;
    constexpr int WN1 = N1 / 128, WM = NW / WN1, WROWS = BM / WM, MF = WROWS / 16, NF = 8;
    constexpr int N2P = NF2 * 16;
    constexpr int ASLOT = BM * 4, BSLOT = N1 * 4;            // 16-byte pieces per ring slot
    constexpr int RING = 3 * (ASLOT + BSLOT);
    // partial products (float4 pieces), N2P / 4 pieces a row, the piece column XOR-swizzled by the
    // row (OPKH_PART): unswizzled, the 16 rows of a fragment fall on the same banks (round 2 PMC:
    // 60 % of the LDS cycles were bank conflicts); padded by one piece (round 2-5) the writes were
    // conflict-free but every read instruction paid one extra LDS cycle (round-5 PMC: 0.071 of the
    // LDS cycles at <512, 4>); with the XOR both are conflict-free in the lane-group model of
    // MI355X_MICROARCH.md §LDS (tools/lds_conflicts.py head_partials)
    constexpr int PSTRIDE = N2P / 4;
    constexpr int PART = NW * WROWS * PSTRIDE;
    constexpr int MAIN = RING > PART ? RING : PART;
    constexpr int LDS_PIECES = MAIN + N1 / 2;                 // + bias / multiplier of Mconv6
    static_assert(LDS_PIECES * 16 <= 160 * 1024, "LDS budget");
    static_assert(MF >= 1 && WROWS % 16 == 0, "wave tile");
    __shared__ uint4 lds[LDS_PIECES];
    float* lbias = reinterpret_cast<float*>(lds + MAIN);
    float* lmul = lbias + N1;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / WN1, wn = wave - (wave / WN1) * WN1;
    const int r16 = lane & 15, q = lane >> 4;
    const int Hp = a.H + 2, Wp = a.W + 2;
    const int total = a.frames * Hp * Wp;
    const int ntiles = (total + BM - 1) / BM;
    // tile order: blockIdx.x, or (PERSIST) the XCD-aware bijection of conv3w.hip, G apart
    const int G = gridDim.x;
    int tile = blockIdx.x;
    if constexpr (PERSIST) {
        const int xcd = blockIdx.x & 7, qq = G >> 3, rr = G & 7;
        tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (blockIdx.x >> 3);
        if (tile >= ntiles) return;
    }

    for (int i = tid; i < N1; i += 64 * NW) {
        const float neg = a.act6 == 1 ? 0.f : 1.f;
        lbias[i] = a.b6[i];
        lmul[i] = a.act6 == 2 ? a.s6[i] : neg;
    }

    // ---- phase 1: Mconv6 K loop ------------------------------------------------------------------
    const int lrow = lane >> 2, phys = lane & 3;
    const int KS = a.cin_pad >> 5;
    const int KV = SPLIT ? 3 * KS : KS;                       // ring steps (split: 3 per chunk)
    constexpr int BIW = N1 / 16 / NW;                         // B DMA instructions per wave per step
    // A DMA: instruction `wave` covers tile rows wave*16 .. +15 (positions past the end read the
    // zeroed guard after the last frame, conv.h kConvGuardTail)
    const int arow = wave * 16 + lrow;
#define OPKH_ASRC(p0_) (a.in + a.in_coff + (size_t)((p0_) + arow) * a.in_cs + (phys ^ (((arow >> 2) & 1) << 1)) * 8)
    const uint16_t* asrc = OPKH_ASRC(tile * BM);
    // (split: the lo twin has the hi buffer's layout)
    const ptrdiff_t lo_off = SPLIT ? a.in_lo - a.in : 0;
    // step s_: chunk c_, product k_ (split: 0 x_hi w_hi, 1 x_lo w_hi, 2 x_hi w_lo)
#define OPKH_ISSUE(s_)                                                                        \
    do {                                                                                      \
        const int sl_ = (s_) % 3;                                                             \
        const int c_ = SPLIT ? (s_) / 3 : (s_), k_ = SPLIT ? (s_) - 3 * ((s_) / 3) : 0;        \
        __builtin_amdgcn_global_load_lds((const void*)(asrc + (k_ == 1 ? lo_off : 0) + c_ * 32), \
                                         (__attribute__((address_space(3))) void*)(&lds[sl_ * ASLOT + wave * 64]), \
                                         16, 0, 0);                                           \
        const uint16_t* wb_ = a.w6 + (size_t)((k_ == 2 ? KS : 0) + c_) * N1 * 32;             \
        _Pragma("unroll") for (int j_ = 0; j_ < (OPKH_ABLATE == 1 && (s_) > 1 ? 0 : BIW); ++j_) { \
            const int rb_ = (j_ * NW + wave) * 16 + lrow;                                     \
            __builtin_amdgcn_global_load_lds(                                                 \
                (const void*)(wb_ + rb_ * 32 + (phys ^ (((rb_ >> 2) & 1) << 1)) * 8),         \
                (__attribute__((address_space(3))) void*)(&lds[3 * ASLOT + sl_ * BSLOT + (j_ * NW + wave) * 64]), \
                16, 0, 0);                                                                    \
        }                                                                                     \
    } while (0)

    // Mconv7's packed weights [N2P][N1] as ring rows: row r = K block (r / N2P) x output channel
    // (r % N2P), 64 bytes, swizzled like a B slot; rows [h*N1, (h+1)*N1) fill B slot (KS + h) % 3
    // (NF2 / 2 slots: the ones of K steps KS-2 and KS-3, free once every wave passed step KS-1's
    // barrier; the next tile's DMA goes into the ring only after phase 3's barrier)
    constexpr bool W7LDS = OPKH_W7LDS && !PERSIST && !SPLIT;
    constexpr int W7ROWS = (N1 / 32) * N2P, W7IW = W7ROWS / 16 / NW;
    static_assert(W7ROWS <= 2 * N1 && W7ROWS % (16 * NW) == 0, "Mconv7 weights fit two B slots");
#define OPKH_ISSUE_W7()                                                                       \
    do {                                                                                      \
        _Pragma("unroll") for (int k_ = 0; k_ < W7IW; ++k_) {                                 \
            const int inst_ = k_ * NW + wave;                                                 \
            const int r_ = inst_ * 16 + lrow;                                                 \
            const int kb_ = r_ / N2P, o_ = r_ - (r_ / N2P) * N2P;                             \
            const int sl_ = (KV + (inst_ * 16) / N1) % 3;                                     \
            __builtin_amdgcn_global_load_lds(                                                 \
                (const void*)(a.w7 + (size_t)o_ * N1 + kb_ * 32 + (phys ^ (((r_ >> 2) & 1) << 1)) * 8), \
                (__attribute__((address_space(3))) void*)(&lds[3 * ASLOT + sl_ * BSLOT + ((inst_ * 16) % N1) * 4]), \
                16, 0, 0);                                                                    \
        }                                                                                     \
    } while (0)
    const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
    (void)lds0;

    OPKH_ISSUE(0);
    if (KV > 1) OPKH_ISSUE(1);
    for (;;) {
    const int p0 = tile * BM;
    // lane terms re-derived per tile (opaque): nothing lane-dependent is hoisted out of the tile
    // loop and kept live through phase 2's registers
    int lane_t = lane;
    asm volatile("" : "+v"(lane_t));
    const int r16 = lane_t & 15, q = lane_t >> 4, lrow = lane_t >> 2, phys = lane_t & 3;
    const int arow = wave * 16 + lrow;
    (void)arow;
    float4_t acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

    for (int s = 0; s < KV; ++s) {
        // own DMA of step s landed once only step s+1's (1 + BIW instructions) may be in flight
        // (a previous tile's output stores are older)
        if (s + 1 < KV) vm_wait<1 + BIW>();
        else vm_wait<0>();
        __builtin_amdgcn_s_barrier();
        if (s + 2 < KV) OPKH_ISSUE(s + 2);
        if (W7LDS && s == KV - 1) OPKH_ISSUE_W7();
        half8_t fa[MF], fb[NF];
        if constexpr (OPKH_KSCHED) {
            // rows i*16 / j*16 keep the swizzle bit: fragment i (j) is base + 1 KiB * i (j)
            int ar = wm * WROWS + r16, br = wn * 128 + r16;
            asm volatile("" : "+v"(ar), "+v"(br));
            const uint32_t ab = lds0 + (uint32_t)(((s % 3) * ASLOT + swz64(ar, q)) * 16);
            const uint32_t bb = lds0 + (uint32_t)(((3 * ASLOT + (s % 3) * BSLOT) + swz64(br, q)) * 16);
            // reads in consumption order: fa[0], fb[0..NF-1], fa[1..MF-1] (R = MF + NF <= 15)
            constexpr int R = MF + NF;
            static_assert(R <= 15, "lgkmcnt range");
#define OPKH_DSR(dst_, addr_, off_) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst_) : "v"(addr_), "i"(off_))
            OPKH_DSR(fa[0], ab, 0);
            OPKH_DSR(fb[0], bb, 0);
            OPKH_DSR(fb[1], bb, 1024);
            OPKH_DSR(fb[2], bb, 2048);
            OPKH_DSR(fb[3], bb, 3072);
            OPKH_DSR(fb[4], bb, 4096);
            OPKH_DSR(fb[5], bb, 5120);
            OPKH_DSR(fb[6], bb, 6144);
            OPKH_DSR(fb[7], bb, 7168);
            if (MF > 1) OPKH_DSR(fa[MF > 1 ? 1 : 0], ab, 1024);
            if (MF > 2) OPKH_DSR(fa[MF > 2 ? 2 : 0], ab, 2048);
            if (MF > 3) OPKH_DSR(fa[MF > 3 ? 3 : 0], ab, 3072);
#undef OPKH_DSR
            static_assert(NF == 8 && MF <= 4, "read list above");
            // row 0 of the tile: MFMA j waits for read 1 + j (fa[0] is read 0)
#define OPKH_WAIT(n_, r_) asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(r_) : "n"(n_))
#define OPKH_ROW0(j_)                                                                         \
    do {                                                                                      \
        if ((j_) == 0) asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(fa[0]), "+v"(fb[0]) : "n"(R - 2)); \
        else OPKH_WAIT(R - 2 - (j_), fb[j_]);                                                 \
        acc[0][j_] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j_], fa[0], acc[0][j_], 0, 0, 0); \
        __builtin_amdgcn_sched_barrier(0);                                                    \
    } while (0)
            OPKH_ROW0(0); OPKH_ROW0(1); OPKH_ROW0(2); OPKH_ROW0(3);
            OPKH_ROW0(4); OPKH_ROW0(5); OPKH_ROW0(6); OPKH_ROW0(7);
#undef OPKH_ROW0
#pragma unroll
            for (int i = 1; i < MF; ++i) {
                // fa[i] is read NF + i
                switch (i) {
                case 1: OPKH_WAIT(R - NF - 2 < 0 ? 0 : R - NF - 2, fa[i]); break;
                case 2: OPKH_WAIT(R - NF - 3 < 0 ? 0 : R - NF - 3, fa[i]); break;
                default: OPKH_WAIT(0, fa[i]); break;
                }
#pragma unroll
                for (int j = 0; j < NF; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa[i], acc[i][j], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
#undef OPKH_WAIT
        } else {
            const uint4* As = lds + (s % 3) * ASLOT;
            const uint4* Bs = lds + 3 * ASLOT + (s % 3) * BSLOT;
#pragma unroll
            for (int i = 0; i < MF; ++i)
                fa[i] = __builtin_bit_cast(half8_t, As[swz64(wm * WROWS + i * 16 + r16, q)]);
#pragma unroll
            for (int j = 0; j < NF; ++j)
                fb[j] = __builtin_bit_cast(half8_t, Bs[swz64(wn * 128 + j * 16 + r16, q)]);
#pragma unroll
            for (int i = 0; i < MF; ++i)
#pragma unroll
                for (int j = 0; j < NF; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[j], fa[i], acc[i][j], 0, 0, 0);
        }
    }
    if (W7LDS) {   // Mconv7's weights landed (own DMA) and visible to every wave
        vm_wait<0>();
        __builtin_amdgcn_s_barrier();
    }

    if constexpr (OPKH_ABLATE == 2) {   // dev probe: keep the accumulators, skip phases 2 and 3
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < NF; ++j) asm volatile("" :: "v"(acc[i][j]));
        __syncthreads();
    } else {
    // ---- phase 2: activated Mconv6 block -> Mconv7 partial over this wave's 128 channels -------
    // lane (r16, q) of acc[i][j] holds channels wn*128 + 16j + 4q .. +3 of tile row
    // wm*WROWS + 16i + r16; after the swap of pair (2kb, 2kb+1) it holds channels
    // 32kb + 16(q&1) + 8(q>>1) .. +7 = B-operand K elements 8q .. 8q+7 of block kb
    float4_t acc2[MF][NF2];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int f = 0; f < NF2; ++f) acc2[i][f] = float4_t{0.f, 0.f, 0.f, 0.f};
    const float* lb = lbias + wn * 128 + 4 * q;
    const float* lm = lmul + wn * 128 + 4 * q;
    // (read per tile, not hoisted out of the persistent loop into registers it has not got)
    const uint16_t* w7o = a.w7;
    asm volatile("" : "+s"(w7o));
    // (global address space again: through the opaque copy the loads would be flat_load, which
    // also count in lgkmcnt -- every wait for them drained the LDS reads as well)
    typedef const __attribute__((address_space(1))) half8_t* gh8p;
    const __attribute__((address_space(1))) uint16_t* w7 =
        (const __attribute__((address_space(1))) uint16_t*)w7o;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        half8_t a7[NF2], a7l[SPLIT ? NF2 : 1];
#pragma unroll
        for (int f = 0; f < NF2; ++f) {
            if constexpr (W7LDS) {   // ring row (K block wn*4 + kb) x N2P + f*16 + r16
                const int r = (wn * 4 + kb) * N2P + f * 16 + r16;
                const int sl = (KV + r / N1) % 3;
                a7[f] = __builtin_bit_cast(half8_t, lds[3 * ASLOT + sl * BSLOT + swz64(r % N1, q)]);
            } else {
                a7[f] = *reinterpret_cast<gh8p>(w7 + (size_t)(f * 16 + r16) * N1 + wn * 128 +
                                                          kb * 32 + q * 8);
                if constexpr (SPLIT)   // w7_lo: the second [N2P][N1] block
                    a7l[f] = *reinterpret_cast<gh8p>(w7 + (size_t)(N2P + f * 16 + r16) * N1 +
                                                     wn * 128 + kb * 32 + q * 8);
            }
        }
        float4_t bq[2], mq[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            bq[h] = *reinterpret_cast<const float4_t*>(lb + (2 * kb + h) * 16);
            mq[h] = *reinterpret_cast<const float4_t*>(lm + (2 * kb + h) * 16);
        }
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            uint32_t pk[2][2], pl[2][2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float4_t t = (SPLIT ? acc[i][2 * kb + h] * a.wscale6 : acc[i][2 * kb + h]) + bq[h];
                const float4_t v = act_pick4<MX>(t, t * mq[h]);
                const half2_t h01 = __builtin_convertvector(v.xy, half2_t);
                const half2_t h23 = __builtin_convertvector(v.zw, half2_t);
                pk[h][0] = __builtin_bit_cast(uint32_t, h01);
                pk[h][1] = __builtin_bit_cast(uint32_t, h23);
                if constexpr (SPLIT) {   // lo = fp16(v - hi) (v - hi exact in fp32)
                    pl[h][0] = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                        v.xy - __builtin_convertvector(h01, float2_t), half2_t));
                    pl[h][1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                        v.zw - __builtin_convertvector(h23, float2_t), half2_t));
                }
            }
            const auto sl = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
            const auto sh = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
            const half8_t b2 = __builtin_bit_cast(half8_t, make_uint4(sl[0], sh[0], sl[1], sh[1]));
#pragma unroll
            for (int f = 0; f < NF2; ++f)
                acc2[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a7[f], b2, acc2[i][f], 0, 0, 0);
            if constexpr (SPLIT) {
                const auto ll = __builtin_amdgcn_permlane16_swap(pl[0][0], pl[1][0], false, false);
                const auto lh = __builtin_amdgcn_permlane16_swap(pl[0][1], pl[1][1], false, false);
                const half8_t b2l = __builtin_bit_cast(half8_t, make_uint4(ll[0], lh[0], ll[1], lh[1]));
#pragma unroll
                for (int f = 0; f < NF2; ++f) {
                    acc2[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a7l[f], b2, acc2[i][f], 0, 0, 0);
                    acc2[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a7[f], b2l, acc2[i][f], 0, 0, 0);
                }
            }
        }
    }

    if constexpr (OPKH_ABLATE == 3) {   // dev probe: phase 2 kept, phase 3 skipped
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int f = 0; f < NF2; ++f) asm volatile("" :: "v"(acc2[i][f]));
        __syncthreads();
    } else {
    // ---- phase 3: sum the wave columns' partials in order, + bias, outputs ---------------------
    __syncthreads();   // every wave is past its last ring read
    float4_t* part = reinterpret_cast<float4_t*>(lds);
    // partial of wave w: [WROWS positions][N2P channels] fp32; piece (row, c) at OPKH_PART
#define OPKH_PART(row_, c_) ((row_) * PSTRIDE + ((c_) ^ ((row_) & (PSTRIDE - 1))))
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int f = 0; f < NF2; ++f)
            part[OPKH_PART(wave * WROWS + i * 16 + r16, f * 4 + q)] = acc2[i][f];
    __syncthreads();
    // this lane's sums: output fragments f = wn, wn + WN1, ... of its wave row
    constexpr int NFO = (NF2 + WN1 - 1) / WN1;
    float4_t outv[NFO][MF];
#pragma unroll
    for (int k = 0; k < NFO; ++k) {
        const int f = wn + k * WN1;
        if (f >= NF2) continue;
        const float4_t b7 = *reinterpret_cast<const float4_t*>(a.b7 + f * 16 + 4 * q);   // zero-padded to N2P
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            float4_t v = part[OPKH_PART((wm * WN1) * WROWS + i * 16 + r16, f * 4 + q)];
            for (int w = 1; w < WN1; ++w)
                v = v + part[OPKH_PART((wm * WN1 + w) * WROWS + i * 16 + r16, f * 4 + q)];
            outv[k][i] = (SPLIT ? v * a.wscale7 : v) + b7;
        }
    }
    // positions of this lane's MF rows: padded-image coordinates by float-reciprocal division
    // (exact below 2^24, conv3_dev.h fdiv) instead of the integer division sequences
    const int HW = Hp * Wp;
    const float rHW = 1.f / (float)HW, rW = 1.f / (float)Wp;
    int pos[MF], fri[MF], yyi[MF], xxi[MF];
    bool ok[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
        const int p = p0 + wm * WROWS + i * 16 + r16;
        const int fr = fdiv(p, HW, rHW), rem = p - fr * HW;
        const int yy = fdiv(rem, Wp, rW), xx = rem - yy * Wp;
        pos[i] = p;
        fri[i] = fr;
        yyi[i] = yy;
        xxi[i] = xx;
        ok[i] = p < total && yy >= 1 && yy <= a.H && xx >= 1 && xx <= a.W;   // not a border position
    }
#pragma unroll
    for (int k = 0; k < NFO; ++k) {
        const int f = wn + k * WN1;
        const int ch = f * 16 + 4 * q;   // this lane's 4 output channels
        if (f >= NF2 || ch >= a.n2) continue;
        const int nv = min(4, a.n2 - ch);
        // (lo / hi: channels 0-1 / 2-3 of the lane's four; split: the pair's second halves in
        // lo2 / hi2)
        uint32_t lo[MF], hi[MF], lo2[SPLIT ? MF : 1], hi2[SPLIT ? MF : 1];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            const float4_t v = outv[k][i];
            const half2_t h01 = __builtin_convertvector(v.xy, half2_t);
            const half2_t h23 = __builtin_convertvector(v.zw, half2_t);
            lo[i] = __builtin_bit_cast(uint32_t, h01);
            hi[i] = __builtin_bit_cast(uint32_t, h23);
            if constexpr (SPLIT) {
                lo2[i] = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                    v.xy - __builtin_convertvector(h01, float2_t), half2_t));
                hi2[i] = __builtin_bit_cast(uint32_t, __builtin_convertvector(
                    v.zw - __builtin_convertvector(h23, float2_t), half2_t));
            }
        }
        for (int d = 0; d < a.ndst; ++d) {
            const int cs = a.dst_cs[d];
#pragma unroll
            for (int pass = 0; pass < (SPLIT ? 2 : 1); ++pass) {
                uint16_t* const od = (pass ? a.dst_lo[d] : a.dst[d]) + a.dst_coff[d] + ch;
                const uint32_t* const pa = pass ? lo2 : lo;
                const uint32_t* const pb = pass ? hi2 : hi;
                if (nv == 4 && ((a.dst_coff[d] | cs) & 3) == 0) {
#pragma unroll
                    for (int i = 0; i < MF; ++i)
                        if (ok[i]) *reinterpret_cast<uint2*>(od + (size_t)pos[i] * cs) = make_uint2(pa[i], pb[i]);
                } else {
#pragma unroll
                    for (int i = 0; i < MF; ++i)
                        if (ok[i])
                            for (int e = 0; e < nv; ++e)
                                od[(size_t)pos[i] * cs + e] = (uint16_t)((e < 2 ? pa[i] : pb[i]) >> (16 * (e & 1)));
                }
            }
        }
        if (a.out32) {
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                if (!ok[i]) continue;
                const float4_t v = outv[k][i];
                float* o = a.out32 + (((size_t)fri[i] * a.out32_c + a.out32_coff + ch) * a.H + yyi[i] - 1) * a.W + xxi[i] - 1;
                for (int e = 0; e < nv; ++e) o[(size_t)e * a.H * a.W] = v[e];
            }
        }
    }
    }   // OPKH_ABLATE != 3
    }   // OPKH_ABLATE != 2
    int next = -1;
    if constexpr (PERSIST) {
        // the ring (aliased by the partials) is free once every wave has read its sums: the
        // next tile's first two K steps (older than nothing but these stores)
        __syncthreads();
        next = tile + G;
        if (next < ntiles) {
            asrc = OPKH_ASRC(next * BM);
            OPKH_ISSUE(0);
            if (KV > 1) OPKH_ISSUE(1);
        }
    }
    if (!PERSIST || next >= ntiles) break;
    tile = next;
    }   // tiles
#undef OPKH_ISSUE
#undef OPKH_ASRC
#undef OPKH_PART
}

}  // namespace

bool conv_head_supported(int n1, int n2, int cin_pad)
{
    return (n1 == 256 || n1 == 512) && n2 >= 1 && n2 <= 64 && cin_pad >= 32 && cin_pad % 32 == 0;
}

void conv_head_pack_w7(uint16_t* dst, const uint16_t* w7, int n1, int n2)
{
    // dst [N2P][N1]: within each 32-channel block, K element 8q + e = channel 16(q&1) + 8(q>>1) + e
    const int n2p = n2 <= 32 ? 32 : 64;
    for (int o = 0; o < n2p; ++o)
        for (int k = 0; k < n1; ++k) {
            const int blk = k / 32, e = k % 8, qq = (k % 32) / 8;
            const int c = blk * 32 + 16 * (qq & 1) + 8 * (qq >> 1) + e;
            dst[(size_t)o * n1 + k] = o < n2 ? w7[(size_t)o * n1 + c] : 0;
        }
}

void launch_conv_head(const HeadArgs& a, hipStream_t stream)
{
    OPK_CHECK_ARG(conv_head_supported(a.n1, a.n2, a.cin_pad), "conv_head: N1 256/512, N2 <= 64");
    OPK_CHECK_ARG(a.ndst <= kConvMaxDst, "conv_head: too many destinations");
    if (a.split) {
        OPK_CHECK_ARG(a.in_lo != nullptr, "conv_head: split precision needs the input's lo twin");
        for (int d = 0; d < a.ndst; ++d)
            OPK_CHECK_ARG(a.dst_lo[d] != nullptr, "conv_head: split precision: lo twins required");
    }
    const long total = (long)a.frames * (a.H + 2) * (a.W + 2);
    // phase 3 decodes positions by float-reciprocal division, exact below 2^24 (conv3_dev.h)
    OPK_CHECK_ARG(total < (1L << 24), "conv_head: too many positions (split the batch)");
    const long ntiles = (total + kH_BM - 1) / kH_BM;
    // persistent at N1 = 512 (one 143 KB workgroup per CU: 4-5 % faster than one workgroup per
    // tile); at N1 = 256 two per-tile workgroups share a CU and the persistent grid measured
    // 23 % slower (one per CU) or unchanged-slow (two per CU) -- profiles/round3/head/
    // Split precision: per-tile at both N1 (the persistent <512, 4, split> spills 10-14 VGPRs per
    // tile; measured 98.5 against 98.7 ms per 130-frame split forward, profiles/round6/split_head/)
    const bool persist = a.cus > 0 && a.n1 == 512 && !a.split;
    const unsigned G = (unsigned)(persist ? std::min<long>(a.cus, ntiles) : ntiles);
    const dim3 blk(64 * kH_NW);
#define OPKH_LAUNCH3(N1_, NF2_, MX_, SP_)                                                       \
    do {                                                                                       \
        note_launch("conv_head_kernel<%d,%d,%d,%d%s>", N1_, NF2_, (int)persist, (int)MX_, SP_ ? ",split" : ""); \
        if (persist) hipLaunchKernelGGL((conv_head_kernel<N1_, NF2_, true, MX_, SP_>), dim3(G), blk, 0, stream, a); \
        else hipLaunchKernelGGL((conv_head_kernel<N1_, NF2_, false, MX_, SP_>), dim3(G), blk, 0, stream, a); \
    } while (0)
#define OPKH_LAUNCH2(N1_, NF2_, MX_)                                                            \
    do {                                                                                       \
        if (a.split) OPKH_LAUNCH3(N1_, NF2_, MX_, true);                                       \
        else OPKH_LAUNCH3(N1_, NF2_, MX_, false);                                              \
    } while (0)
#define OPKH_LAUNCH(N1_, NF2_)                                                                 \
    do {                                                                                       \
        if (a.actmax) OPKH_LAUNCH2(N1_, NF2_, true);                                           \
        else OPKH_LAUNCH2(N1_, NF2_, false);                                                   \
    } while (0)
    if (a.n1 == 512) {
        if (a.n2 <= 32) OPKH_LAUNCH(512, 2);
        else OPKH_LAUNCH(512, 4);
    } else {
        if (a.n2 <= 32) OPKH_LAUNCH(256, 2);
        else OPKH_LAUNCH(256, 4);
    }
#undef OPKH_LAUNCH
#undef OPKH_LAUNCH2
#undef OPKH_LAUNCH3
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
