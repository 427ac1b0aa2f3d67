// conv3wg.hip -- 3x3 convolution as Winograd F(2,3) along x on the persistent halo implicit GEMM.
//
// Why: the stage layers of conv3w8 run at their MFMA floor under the clock the chip holds on random
// operands: the lever left is fewer MFMAs.  F(2,3) computes two neighbouring
// outputs of one row from four inputs with four products instead of six:
//     d0..d3 = in[x-1 .. x+2]             (one tap row ky, 32 input channels)
//     t0 = d0 - d2, t1 = d1 + d2, t2 = d2 - d1, t3 = d1 - d3      (fp16, v_pk_add_f16)
//     U0 = g0, U1 = (g0 + g1 + g2) / 2, U2 = (g0 - g1 + g2) / 2, U3 = g2   (host, fp32 -> fp16)
//     M_t = sum over (ky, ci) U_t . t_t                            (MFMA, fp32 accumulate)
//     out(x) = M0 + M1 + M2,  out(x+1) = M1 - M2 - M3
// so a K unit (32-channel chunk, tap row ky) is 4 "terms" of 16x16x32 MFMAs over 16 output pairs
// instead of 3 taps over 16 outputs each: 2/3 of the MFMAs of conv3w8 for the same outputs.  The
// transforms cost one extra fp16 rounding of the input differences and of the weight sums
// (tools/wino_numerics.py: BODY_25 rel-L2 2.8e-3 vs 2.2-2.5e-3 direct at 368x656, tolerance 5e-3).
//
// Tile: 256 virtual positions (128 output pairs; the virtual row width VW = sw + 2 is even, so a
// pair never crosses a row) x BN output channels, 8 waves = 4 position groups of 32 pairs x 2
// channel groups of BN/2.  The four accumulators of a pair take twice the registers of direct
// outputs, hence half conv3w8's positions per wave.  The halo of a 32-channel chunk (positions
// p0 - VW - 1 .. p0 + 256 + VW) is DMA'd into two parity planes (even / odd virtual positions,
// EP rows each) so that the stride-2 reads d0..d3 of 16 consecutive pairs are 16 consecutive rows
// of one plane -- conflict-free with the 64-byte-row swizzle of conv3w.  Weights of a unit:
// [term][BN][32] fp16 (32 KB at BN 128) through the 3-slot ring of conv3w8, halo through 2 slots.
// Schedule per unit (one mid-unit barrier, as conv3w8):
//     term 0 (reads B term 1), term 1 (reads B term 2), [own DMA of unit u+1 landed; s_barrier],
//     term 2 (reads B term 3 and the d's of unit u+1), term 3 (reads B term 0 of unit u+1,
//     transforms the next d's between its MFMAs), issue the DMA of unit u+2.
#include "conv.h"

#include <algorithm>
#include <utility>

#include "../common.h"
#include "conv3_dev.h"

namespace opk {

namespace {

using namespace conv3dev;

constexpr int kg_BM = 256, kg_NW = 8, kg_EP = 224;   // positions per tile, waves, rows per plane

template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
// f(integral_constant<0>) ... f(integral_constant<N-1>), fully unrolled with constant indices
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f)
{
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}

template <int OFF>
__device__ __forceinline__ void dsr(half8_t& d, uint32_t addr)
{
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}

template <int N>
__device__ __forceinline__ void lgkm_wait()
{
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

// a - b and a + b on 8 fp16 lanes as four v_pk_add_f16 (the compiler splits a vector subtraction
// into scalar halves); correctly rounded, as the fp32 difference rounded to fp16 would be
__device__ __forceinline__ half8_t pk_sub(half8_t a, half8_t b)
{
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const u4 x = __builtin_bit_cast(u4, a), y = __builtin_bit_cast(u4, b);
    u4 r;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        asm("v_pk_add_f16 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r[k]) : "v"(x[k]), "v"(y[k]));
    return __builtin_bit_cast(half8_t, r);
}
__device__ __forceinline__ half8_t pk_add(half8_t a, half8_t b)
{
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const u4 x = __builtin_bit_cast(u4, a), y = __builtin_bit_cast(u4, b);
    u4 r;
#pragma unroll
    for (int k = 0; k < 4; ++k) asm("v_pk_add_f16 %0, %1, %2" : "=v"(r[k]) : "v"(x[k]), "v"(y[k]));
    return __builtin_bit_cast(half8_t, r);
}

// pins a register to this point: its later uses cannot be hoisted above the preceding wait
__device__ __forceinline__ void pin(half8_t& v) { asm volatile("" : "+v"(v)); }

template <int BN, int NB>
__global__ __launch_bounds__(64 * kg_NW, 1) void conv3wg_kernel(const ConvArgs a)
{
    constexpr int NW = kg_NW, BM = kg_BM, EP = kg_EP;
    constexpr int NFW = BN / 32;                // output-channel fragments per wave
    constexpr int CG = BN / 2;                  // output channels per channel group
    constexpr int PF = 2;                       // pair fragments per wave (32 pairs)
    constexpr int HROWS = 2 * EP;               // halo rows per slot: even plane, odd plane
    constexpr int API = HROWS / 16, AIW = (API + NW - 1) / NW;
    constexpr int BROWS = 4 * BN, BPI = BROWS / 16, BIW = (BPI + NW - 1) / NW;
    constexpr int ASLOT = HROWS * 4, BSLOT = BROWS * 4;   // 16-byte pieces
    constexpr int LDS_PIECES = 2 * ASLOT + 3 * BSLOT + BN / 2;
    static_assert(LDS_PIECES * 16 <= 160 * 1024, "LDS budget");
    static_assert(NFW == 4 || NFW == 3, "BN 128 or 96");
    static_assert(NB == 1 || NB == 2 || NB == 4, "1, 2 or 4 n-blocks");
    __shared__ uint4 lds[LDS_PIECES];
    float* lbias = reinterpret_cast<float*>(lds + 2 * ASLOT + 3 * BSLOT);
    float* lmul = lbias + BN;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int pg = wave & 3, cg = wave >> 2;   // position group (32 pairs), channel group
    const int r16 = lane & 15, q = lane >> 4;
    const Strips g(a);
    const int VW2 = g.VW >> 1;
    const int ntm = (g.total + BM - 1) / BM;
    // n-blocks as conv3w8: the grid is a multiple of NB, a block keeps one n-block
    constexpr int LGNB = NB == 4 ? 2 : NB - 1;
    const int G = gridDim.x, GM = G >> LGNB;
    const int xcd = blockIdx.x & 7, qq = G >> 3, rr = G & 7;
    const int tix = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (blockIdx.x >> 3);
    const int nblk = tix & (NB - 1);
    int m = tix >> LGNB;
    if (m >= ntm) return;

    if (tid < BN) {
        const float neg = a.act == 1 ? 0.f : 1.f;
        lbias[tid] = a.bias[nblk * BN + tid];
        lmul[tid] = a.act == 2 ? a.slope[nblk * BN + tid] : neg;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    const int lrow = lane >> 2, phys = lane & 3;
    const int cpt = a.cin_pad >> 5;
    const int U = 3 * cpt;
    const int ublk = nblk * U;
    int bi = 0;   // B DMA instructions of this wave per unit
    for (int j = 0; j < BIW; ++j) bi += (BPI % NW == 0 || j * NW + wave < BPI) ? 1 : 0;

    const char* abase = reinterpret_cast<const char*>(a.in + a.in_coff - a.in_cs);
    uint32_t aoff[AIW];
    // halo DMA instruction i: LDS row L = (i*NW + wave)*16 + lrow of a slot holds virtual
    // position p0 - VW - 1 + R, R = 2 (L mod EP) + (L >= EP)
    auto arow = [&](int mt, int i) -> uint32_t {
        const int L = (i * NW + wave) * 16 + lrow;
        const int lp = phys ^ (((L >> 2) & 1) << 1);
        const int pl = L >= EP ? 1 : 0;
        const int R = 2 * (L - pl * EP) + pl;
        int f, yy, xx, s;
        const long pos = g.map(mt * BM - g.VW - 1 + R, f, yy, xx, s);
        return (uint32_t)(((pos + 1) * a.in_cs + lp * 8) * 2);
    };
    auto issue = [&](int c, int ky, int aslot, int bslot, bool nt) {
        if (ky == 0) {
            const int as = aslot * ASLOT;
#pragma unroll
            for (int i = 0; i < AIW; ++i)
                if (API % NW == 0 || i * NW + wave < API)
                    __builtin_amdgcn_global_load_lds(
                        (const void*)(abase + c * 64 + (nt ? arow(m + GM, i) : aoff[i])),
                        (__attribute__((address_space(3))) void*)(&lds[as + (i * NW + wave) * 64]), 16, 0,
                        0);
        }
        const int bs = 2 * ASLOT + bslot * BSLOT;
        const uint16_t* ub = a.w + (size_t)(ublk + c * 3 + ky) * BROWS * 32;
#pragma unroll
        for (int j = 0; j < BIW; ++j)
            if (BPI % NW == 0 || j * NW + wave < BPI) {
                int rb = (j * NW + wave) * 16 + lrow;
                asm volatile("" : "+v"(rb));
                const int bo = rb * 32 + (phys ^ (((rb >> 2) & 1) << 1)) * 8;
                __builtin_amdgcn_global_load_lds(
                    (const void*)(ub + bo),
                    (__attribute__((address_space(3))) void*)(&lds[bs + (j * NW + wave) * 64]), 16, 0, 0);
            }
    };

    const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
    // A (pair) row bases of unit (slot, ky): even plane row pg*32 + r16 + ky*VW/2 (+1); the odd
    // plane is EP rows on (EP % 8 == 0 keeps the swizzle), pair fragment i 16 rows on
    auto abase_row = [&](int slot, int ky, int plus) -> uint32_t {
        int r = pg * 32 + r16 + ky * VW2 + plus;
        asm volatile("" : "+v"(r));
        return lds0 + (uint32_t)(slot * ASLOT * 16) + (uint32_t)swz64(r, q) * 16;
    };
    const uint32_t bswz = (uint32_t)swz64(r16, q) * 16 + (uint32_t)(cg * CG * 64);
    auto bbase = [&](int slot) -> uint32_t {
        uint32_t b = bswz;
        asm volatile("" : "+v"(b));
        return lds0 + (uint32_t)((2 * ASLOT + slot * BSLOT) * 16) + b;
    };

    float4_t acc[PF][NFW][4];
    // transformed inputs of the current unit; the next unit's d0 / d1 land in tc[0] / tc[1] once
    // terms 0 and 1 are done with them, d2 / d3 in e[0] / e[1], and the transforms are written
    // back into tc after term 3 (no copies)
    half8_t tc[4][PF];
    half8_t e[2][PF];
    half8_t fb0[NFW], fb1[NFW];
    sfor<PF>([&](auto I) {
        sfor<NFW>([&](auto J) {
            sfor<4>([&](auto T) { acc[I][J][T] = float4_t{0.f, 0.f, 0.f, 0.f}; });
        });
    });

    // B fragments of term T of the unit in weight slot base bb
    auto read_b = [&](half8_t* fb, uint32_t bb, auto T) {
        sfor<NFW>([&](auto J) { dsr<(decltype(T)::value * BN + decltype(J)::value * 16) * 64>(fb[J], bb); });
    };
    auto read_d = [&](uint32_t a0, uint32_t a1) {
        sfor<PF>([&](auto I) {
            constexpr int o = decltype(I)::value * 1024;
            dsr<o>(tc[0][I], a0);               // d0: even plane, row r
            dsr<o + EP * 64>(tc[1][I], a0);     // d1: odd plane, row r
            dsr<o>(e[0][I], a1);                // d2: even plane, row r + 1
            dsr<o + EP * 64>(e[1][I], a1);      // d3: odd plane, row r + 1
        });
    };
    auto pin_d = [&]() {
        sfor<PF>([&](auto I) {
            pin(tc[0][I]);
            pin(tc[1][I]);
            pin(e[0][I]);
            pin(e[1][I]);
        });
    };
    auto transform = [&]() {   // fp16 differences, one rounding each (v_pk_add_f16)
        sfor<PF>([&](auto I) {
            const half8_t d0 = tc[0][I], d1 = tc[1][I], d2 = e[0][I], d3 = e[1][I];
            tc[2][I] = pk_sub(d2, d1);
            tc[3][I] = pk_sub(d1, d3);
            tc[1][I] = pk_add(d1, d2);
            tc[0][I] = pk_sub(d0, d2);
        });
    };
    auto mfmas = [&](auto T, half8_t* fb) {
        constexpr int t = decltype(T)::value;
        sfor<PF>([&](auto I) {
            sfor<NFW>([&](auto J) {
                acc[I][J][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[J], tc[t][I], acc[I][J][t], 0, 0, 0);
            });
        });
    };
    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    using C2 = std::integral_constant<int, 2>;
    using C3 = std::integral_constant<int, 3>;

    // ---- prologue: units 0 and 1 of the first tile in flight, unit 0 visible ----------------
#pragma unroll
    for (int i = 0; i < AIW; ++i) aoff[i] = arow(m, i);
    issue(0, 0, 0, 0, false);
    issue(0, 1, 0, 1, false);
    vm_wait_rt(bi);
    __builtin_amdgcn_s_barrier();
    read_d(abase_row(0, 0, 0), abase_row(0, 0, 1));
    read_b(fb0, bbase(0), C0{});
    lgkm_wait<NFW>();
    pin_d();
    transform();

    const int nd = a.ndst;
    const int S1 = PF * 2 * ((NFW + 1) / 2) * nd;   // epilogue stores per wave
    int gc = 0;   // running chunk index of this tile's chunk 0 (halo slot parity)
    for (;;) {
        const int mn = m + GM;
        const bool has_next = mn < ntm;
        for (int u = 0; u < U; ++u) {
            const uint32_t bb_u = bbase(u % 3);
            const bool nt = u + 1 >= U;
            const int u1 = nt ? 0 : u + 1;
            const int c1 = u1 / 3, ky1 = u1 - 3 * c1;
            const int aslot1 = (gc + (nt ? cpt : 0) + c1) & 1;
            // term 0: B of term 1 streams in
            read_b(fb1, bb_u, C1{});
            lgkm_wait<NFW>();
            sfor<NFW>([&](auto J) { pin(fb0[J]); });
            mfmas(C0{}, fb0);
            __builtin_amdgcn_sched_barrier(0);
            // term 1: B of term 2
            read_b(fb0, bb_u, C2{});
            lgkm_wait<NFW>();
            sfor<NFW>([&](auto J) { pin(fb1[J]); });
            mfmas(C1{}, fb1);
            __builtin_amdgcn_sched_barrier(0);
            // unit u+1's DMA (own part) landed, then everyone's
            if (u == 0 && gc > 0) vm_wait_rt64(S1);
            else vm_wait<0>();
            __builtin_amdgcn_s_barrier();
            // term 2: B of term 3 and the next unit's inputs
            read_b(fb1, bb_u, C3{});
            read_d(abase_row(aslot1, ky1, 0), abase_row(aslot1, ky1, 1));
            lgkm_wait<NFW + 4 * PF>();
            sfor<NFW>([&](auto J) { pin(fb0[J]); });
            mfmas(C2{}, fb0);
            __builtin_amdgcn_sched_barrier(0);
            // term 3: B of the next unit's term 0; the next unit's transforms
            read_b(fb0, bbase((u + 1) % 3), C0{});
            lgkm_wait<NFW>();
            sfor<NFW>([&](auto J) { pin(fb1[J]); });
            pin_d();
            mfmas(C3{}, fb1);
            transform();
            __builtin_amdgcn_sched_barrier(0);
            {   // DMA of unit u+2
                const bool nt2 = u + 2 >= U;
                const int u2 = nt2 ? u + 2 - U : u + 2;
                const int c2 = u2 / 3;
                issue(c2, u2 - 3 * c2, (gc + (nt2 ? cpt : 0) + c2) & 1, (u + 2) % 3, nt2);
            }
        }

        // ---- epilogue: output transform + bias + activation + fp16 pack, 16-byte stores -------
        int el = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        asm volatile("" : "+v"(el));
        const int er16 = el & 15, eq = el >> 4;
        const int sidx = blockIdx.x * 64 * NW + wave * 64 + el;
        uint4* sink4 = reinterpret_cast<uint4*>(a.sink) + sidx;
        const int cw = 16 * (eq & 1) + 8 * (eq >> 1);   // channel of a lane's 16-byte store
        const char* lb = reinterpret_cast<const char*>(lbias) + (cg * CG + 4 * eq) * 4;
        sfor<PF>([&](auto I) {
            constexpr int i = decltype(I)::value;
            // the pair's even position and its row
            const int v0 = m * BM + 2 * (pg * 32 + i * 16 + er16);
            int f, yy, xx, s;
            const long pe = g.map(v0, f, yy, xx, s);
            const bool in0 = v0 < g.total;
            const bool oke = in0 && g.interior(yy, xx, s, a.W);
            const bool oko = in0 && g.interior(yy, xx + 1, s, a.W);
            const size_t prow[2] = {(size_t)(in0 ? pe : 0), (size_t)(in0 ? pe + 1 : 0)};
            const bool pok[2] = {oke, oko};
            float4_t o[2][NFW];
            sfor<NFW>([&](auto J) {
                constexpr int j = decltype(J)::value;
                o[0][j] = acc[i][j][0] + acc[i][j][1] + acc[i][j][2];
                o[1][j] = acc[i][j][1] - acc[i][j][2] - acc[i][j][3];
            });
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int j = 0; j + 1 < NFW; j += 2) {
                    uint32_t pk[2][2];
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const float4_t bq = *reinterpret_cast<const float4_t*>(lb + (j + k) * 64);
                        const float4_t mq = *reinterpret_cast<const float4_t*>(lb + BN * 4 + (j + k) * 64);
                        const float4_t t = o[h][j + k] + bq;
                        const float4_t tm = t * mq;
                        float v[4];
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] = t[r] > 0.f ? t[r] : tm[r];
                        pk[k][0] = __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_t){v[0], v[1]}, half2_t));
                        pk[k][1] = __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_t){v[2], v[3]}, half2_t));
                    }
                    const auto sl = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
                    const auto sh = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
                    const uint4 val = make_uint4(sl[0], sh[0], sl[1], sh[1]);
                    const int ch = nblk * BN + cg * CG + cw + j * 16;
                    for (int d = 0; d < nd; ++d) {
                        uint4* p = reinterpret_cast<uint4*>(a.dst[d] + a.dst_coff[d] + ch + prow[h] * a.dst_cs[d]);
                        *(pok[h] ? p : sink4) = val;
                    }
                }
                if constexpr (NFW % 2 == 1) {   // last fragment alone: 4 channels, 8-byte stores
                    constexpr int j = NFW - 1;
                    const float4_t bq = *reinterpret_cast<const float4_t*>(lb + j * 64);
                    const float4_t mq = *reinterpret_cast<const float4_t*>(lb + BN * 4 + j * 64);
                    const float4_t t = o[h][j] + bq;
                    const float4_t tm = t * mq;
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = t[r] > 0.f ? t[r] : tm[r];
                    const uint2 val = make_uint2(
                        __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_t){v[0], v[1]}, half2_t)),
                        __builtin_bit_cast(uint32_t, __builtin_convertvector((float2_t){v[2], v[3]}, half2_t)));
                    const int ch = nblk * BN + cg * CG + j * 16 + 4 * eq;
                    for (int d = 0; d < nd; ++d) {
                        uint2* p = reinterpret_cast<uint2*>(a.dst[d] + a.dst_coff[d] + ch + prow[h] * a.dst_cs[d]);
                        *(pok[h] ? p : reinterpret_cast<uint2*>(sink4)) = val;
                    }
                }
            }
        });
        sfor<PF>([&](auto I) {
            sfor<NFW>([&](auto J) {
                sfor<4>([&](auto T) { acc[I][J][T] = float4_t{0.f, 0.f, 0.f, 0.f}; });
            });
        });
        if (!has_next) break;
        m = mn;
        gc += cpt;
#pragma unroll
        for (int i = 0; i < AIW; ++i) aoff[i] = arow(m, i);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

}  // namespace

size_t conv3wg_packed_elems(int cout, int cin_pad)
{
    const int BN = cout == 96 ? 96 : 128;
    const int nb = (cout + BN - 1) / BN;
    return (size_t)nb * (cin_pad / 32) * 3 * 4 * BN * 32;
}

void conv3wg_pack(uint16_t* dst, const float* w, int cout, int cin, int cin_pad)
{
    const int BN = cout == 96 ? 96 : 128;
    const int cpt = cin_pad / 32;
    std::fill(dst, dst + conv3wg_packed_elems(cout, cin_pad), (uint16_t)0);
    auto h = [](float v) { const _Float16 x = (_Float16)v; return __builtin_bit_cast(uint16_t, x); };
    for (int co = 0; co < cout; ++co)
        for (int ci = 0; ci < cin; ++ci)
            for (int ky = 0; ky < 3; ++ky) {
                const float* gr = w + (((size_t)co * cin + ci) * 3 + ky) * 3;
                const float g0 = gr[0], g1 = gr[1], g2 = gr[2];
                const float U[4] = {g0, (g0 + g1 + g2) * 0.5f, (g0 - g1 + g2) * 0.5f, g2};
                for (int t = 0; t < 4; ++t) {
                    const size_t idx =
                        (((((size_t)(co / BN) * cpt + ci / 32) * 3 + ky) * 4 + t) * BN + co % BN) * 32 + ci % 32;
                    dst[idx] = h(U[t]);
                }
            }
}

bool conv3wg_supported(const ConvArgs& a)
{
    bool aligned = a.ndst >= 1;
    for (int d = 0; d < a.ndst; ++d) aligned = aligned && ((a.dst_coff[d] | a.dst_cs[d]) & 7) == 0;
    const int VW = a.sw + 2 * a.border;
    const bool nb_ok = a.cout == 96 || a.cout == 128 || a.cout == 256 || a.cout == 512;
    // pairs stay inside a virtual row (VW even); the halo plane holds 128 + VW + 1 rows
    return a.ntaps == 9 && a.border == 1 && nb_ok && a.wg && a.sink && a.cus > 0 && !a.out32 &&
           aligned && VW % 2 == 0 && kg_BM / 2 + VW + 1 <= kg_EP && VW > 16 && a.ndst <= kConvMaxDst;
}

void launch_conv3wg(const ConvArgs& args, hipStream_t stream)
{
    OPK_CHECK_ARG(conv3wg_supported(args), "conv3wg: 96 or k x 128 outputs, 3x3, even strip rows");
    ConvArgs a = args;
    a.w = a.wg;   // the Winograd weight layout
    const long total = (long)a.frames * a.nstrips * (a.H + 2 * a.border) * (a.sw + 2 * a.border);
    const long ntm = (total + kg_BM - 1) / kg_BM;
    const int nb = a.cout == 96 ? 1 : a.cout / 128;
    const unsigned G = (unsigned)(std::min<long>(a.cus / nb, ntm) * nb);
    OPK_CHECK_ARG(G >= 1 && G <= 1024, "persistent grid exceeds the sink");
    if (nb == 4) hipLaunchKernelGGL((conv3wg_kernel<128, 4>), dim3(G), dim3(64 * kg_NW), 0, stream, a);
    else if (nb == 2) hipLaunchKernelGGL((conv3wg_kernel<128, 2>), dim3(G), dim3(64 * kg_NW), 0, stream, a);
    else if (a.cout == 128) hipLaunchKernelGGL((conv3wg_kernel<128, 1>), dim3(G), dim3(64 * kg_NW), 0, stream, a);
    else hipLaunchKernelGGL((conv3wg_kernel<96, 1>), dim3(G), dim3(64 * kg_NW), 0, stream, a);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
