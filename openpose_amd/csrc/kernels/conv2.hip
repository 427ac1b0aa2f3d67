// conv2.hip -- BODY_25 convolutions on gfx950 matrix cores, LDS-DMA pipelined implicit GEMM.
//
// Replaces the Caffe ConvolutionLayer (+ in-place PReLU/ReLU, + Concat) work of
// op::NetCaffe::forwardPass (src/openpose/net/netCaffe.cpp:248) -- see conv.h for the padded-NHWC
// GEMM view.  Structure (one workgroup = 512 lanes = 8 waves as 4 (M) x 2 (N)):
//   * tile 256 positions x BN channels, wave tile 64 x BN/2, v_mfma_f32_16x16x32_f16;
//   * K advances 64 fp16 (two 32-channel chunks) per step; operands reach LDS by
//     global_load_lds_dwordx4 (no VGPR staging, no ds_write), three-slot ring, two steps in
//     flight, each wave waiting only for its own loads of the step it is about to read
//     (counted s_waitcnt vmcnt) followed by one raw s_barrier per step;
//   * LDS rows are 128 B; pieces are XOR-swizzled by (row & 7) through the per-lane SOURCE address
//     (the DMA writes lane-linear), the fragment reads apply the same XOR: conflict-free
//     ds_read_b128 (cdna_hip_programming.md §5.4 rule 21, T2);
//   * epilogue: bias + ReLU/PReLU in registers, fp16 tile transposed through LDS, 16-byte NHWC
//     stores to every destination slice (concat-by-offset), fp32 NCHW copy for net_output.
#include "conv.h"

#include "../common.h"

namespace opk {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float float4_t __attribute__((ext_vector_type(4)));

constexpr int BM2 = 256;

__device__ __forceinline__ uint16_t f2h_bits2(float v)
{
    const _Float16 h = (_Float16)v;
    return __builtin_bit_cast(uint16_t, h);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt()
{
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BN, int STAGES>
__global__ __launch_bounds__(512, 2) void conv2_kernel(const ConvArgs a)
{
    constexpr int BM = BM2;
    constexpr int WN = BN / 2;
    constexpr int NF = WN / 16;
    constexpr int MF = 4;
    constexpr int BROWS = (BN + 63) / 64 * 64;    // B rows staged (multiple of 64)
    constexpr int AI = BM / 64;                   // A DMA instructions per wave per step (4)
    constexpr int BI = BROWS / 64;                // B DMA instructions per wave per step
    constexpr int LOADS = AI + BI;
    constexpr int STAGE = (BM + BROWS) * 8;       // 16-byte pieces per ring slot
    constexpr int TSTRIDE = BN == 256 ? BN : BN + 8;   // epilogue tile row stride (fp16)
    static_assert(STAGES * STAGE * 16 <= 160 * 1024, "LDS budget");
    static_assert(BM * TSTRIDE * 2 <= STAGES * STAGE * 16, "epilogue tile must fit the ring");
    __shared__ uint4 lds[STAGES * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // XCD-aware tile order (cdna_hip_programming.md T1, bijective form): the dispatcher deals
    // workgroups round-robin over the 8 XCDs, so give each XCD a contiguous range of tiles, N-tiles
    // of one M-tile adjacent: the 3x3 halo rows and the shared A rows then hit that XCD's L2.
    const int nblk = gridDim.x, nn = (a.cout + BN - 1) / BN;
    const int xcd = blockIdx.x & 7, qq = nblk >> 3, rr = nblk & 7;
    const int tix = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (blockIdx.x >> 3);
    const int m0 = (tix / nn) * BM;
    const int n0 = (tix - (tix / nn) * nn) * BN;
    const int Wp = a.W + 2;
    const int per_frame = a.H * Wp;

    // ---- DMA geometry: lane -> (row in an 8-row group, physical piece) -> logical piece -------
    const int lrow = lane >> 3, phys = lane & 7;
    // A rows handled by this wave: wave*32 + i*8 + lrow; (row & 7) == lrow
    const int lp = phys ^ lrow;                   // logical 16-byte piece this lane fetches
    const int half = lp >> 2;                     // which 32-channel chunk of the 64-wide step
    const int cofs = (lp & 3) * 8;                // channel offset inside the chunk
    static_assert(AI == 4 && BI <= 4, "tile geometry");
    auto arow = [&](int i) {
        int m = m0 + wave * (BM / 8) + i * 8 + lrow;
        if (m >= a.M) m = a.M - 1;
        return m + (m / per_frame) * 2 * Wp;
    };
    const int abase0 = arow(0), abase1 = arow(1), abase2 = arow(2), abase3 = arow(3);
    const int kpad = a.ksteps * 64;
    const int rmax = (a.cout + BN - 1) / BN * BN - 1;   // packed weights have cout_pad rows
    auto brow = [&](int j) {
        const int r = n0 + wave * (BROWS / 8) + j * 8 + lrow;
        return a.w + (size_t)(r > rmax ? rmax : r) * kpad + lp * 8;
    };
    const uint16_t* bsrc0 = brow(0);
    const uint16_t* bsrc1 = BI > 1 ? brow(1) : bsrc0;
    const uint16_t* bsrc2 = BI > 2 ? brow(2) : bsrc0;
    const uint16_t* bsrc3 = BI > 3 ? brow(3) : bsrc0;
    const uint16_t* ain = a.in + a.in_coff + cofs;
    const int cpt = a.cin_pad >> 5;
    const int nchunks = a.ntaps * cpt;
    // this lane's chunk cursor: chunk = 2*s + half, tracked as (tap, chunk-in-tap)
    int ctap = 0, cin = half;
    while (cin >= cpt) { cin -= cpt; ++ctap; }

#define lds_ptr(slot_, piece_) ((__attribute__((address_space(3))) void*)(&lds[(slot_) * STAGE + (piece_)]))

    // issue the DMA of step s into ring slot `slot`
#define OPK_ISSUE(s_, slot_)                                                                  \
    do {                                                                                      \
        const int chunk_ = 2 * (s_) + half;                                                   \
        int tap_ = ctap, ci_ = cin;                                                           \
        if (chunk_ >= nchunks) { tap_ = 0; ci_ = 0; } /* zero weights cover the K tail */     \
        const int toff_ = a.ntaps == 9 ? (tap_ / 3) * Wp + (tap_ % 3) : Wp + 1;                \
        const uint16_t* src_ = ain + ci_ * 32 + (size_t)toff_ * a.in_cs;                     \
        const int ab_ = (wave * (BM / 8)) * 8;                                                \
        __builtin_amdgcn_global_load_lds((const void*)(src_ + (size_t)abase0 * a.in_cs),      \
                                         lds_ptr(slot_, ab_), 16, 0, 0);                      \
        __builtin_amdgcn_global_load_lds((const void*)(src_ + (size_t)abase1 * a.in_cs),      \
                                         lds_ptr(slot_, ab_ + 64), 16, 0, 0);                 \
        __builtin_amdgcn_global_load_lds((const void*)(src_ + (size_t)abase2 * a.in_cs),      \
                                         lds_ptr(slot_, ab_ + 128), 16, 0, 0);                \
        __builtin_amdgcn_global_load_lds((const void*)(src_ + (size_t)abase3 * a.in_cs),      \
                                         lds_ptr(slot_, ab_ + 192), 16, 0, 0);                \
        const int bb_ = BM * 8 + (wave * (BROWS / 8)) * 8;                                    \
        __builtin_amdgcn_global_load_lds((const void*)(bsrc0 + (s_) * 64),                    \
                                         lds_ptr(slot_, bb_), 16, 0, 0);                      \
        if constexpr (BI > 1)                                                                 \
            __builtin_amdgcn_global_load_lds((const void*)(bsrc1 + (s_) * 64),                \
                                             lds_ptr(slot_, bb_ + 64), 16, 0, 0);             \
        if constexpr (BI > 2)                                                                 \
            __builtin_amdgcn_global_load_lds((const void*)(bsrc2 + (s_) * 64),                \
                                             lds_ptr(slot_, bb_ + 128), 16, 0, 0);            \
        if constexpr (BI > 3)                                                                 \
            __builtin_amdgcn_global_load_lds((const void*)(bsrc3 + (s_) * 64),                \
                                             lds_ptr(slot_, bb_ + 192), 16, 0, 0);            \
        ci_ = cin + 2;                                                                        \
        while (ci_ >= cpt) { ci_ -= cpt; ++ctap; }                                            \
        cin = ci_;                                                                            \
    } while (0)

    float4_t acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

    const int S = a.ksteps;
    const int r16 = lane & 15, q = lane >> 4, x7 = r16 & 7;
    OPK_ISSUE(0, 0);
    if (S > 1) OPK_ISSUE(1, 1 % STAGES);
    int slot = 0;
    for (int s = 0; s < S; ++s) {
        if (STAGES >= 3) {
            if (s + 1 < S) wait_vmcnt<LOADS>(); else wait_vmcnt<0>();
        } else {
            wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        if (STAGES >= 3) {
            if (s + 2 < S) {
                int ns = slot + 2;
                if (ns >= STAGES) ns -= STAGES;
                OPK_ISSUE(s + 2, ns);
            }
        }
        const uint4* As = lds + slot * STAGE;
        const uint4* Bs = As + BM * 8;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            half8_t af[MF], bf[NF];
            const int pc = (kk * 4 + q) ^ x7;
#pragma unroll
            for (int i = 0; i < MF; ++i)
                af[i] = __builtin_bit_cast(half8_t, As[(wm * 64 + i * 16 + r16) * 8 + pc]);
#pragma unroll
            for (int j = 0; j < NF; ++j)
                bf[j] = __builtin_bit_cast(half8_t, Bs[(wn * WN + j * 16 + r16) * 8 + pc]);
#pragma unroll
            for (int i = 0; i < MF; ++i)
#pragma unroll
                for (int j = 0; j < NF; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0,
                                                                       0, 0);
        }
        if (STAGES < 3) {   // two slots: refill the slot just read after everyone is done with it
            __builtin_amdgcn_s_barrier();
            if (s + 2 < S) OPK_ISSUE(s + 2, slot);
        }
        if (++slot == STAGES) slot = 0;
    }
#undef OPK_ISSUE
#undef lds_ptr
    wait_vmcnt<0>();
    __syncthreads();

    // ---- epilogue --------------------------------------------------------------------------
    uint16_t* tile = reinterpret_cast<uint16_t*>(lds);
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
            const int ml = wm * 64 + i * 16 + q * 4 + r;
            int f = 0, y = 0, x = 0;
            bool valid = false;
            if (a.out32) {
                const int m = m0 + ml;
                f = m / per_frame;
                const int rem = m - f * per_frame;
                y = rem / Wp;
                x = rem - y * Wp;
                valid = m < a.M && x < a.W;
            }
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                float v = acc[i][j][r] + bias[j];
                if (a.act == 1) v = v > 0.f ? v : 0.f;
                else if (a.act == 2) v = v > 0.f ? v : v * slope[j];
                tile[ml * TSTRIDE + wn * WN + j * 16 + r16] = f2h_bits2(v);
                if (valid && co[j] < a.cout)
                    a.out32[(((size_t)f * a.out32_c + a.out32_coff + co[j]) * a.H + y) * a.W + x] = v;
            }
        }
    __syncthreads();
    if (a.ndst == 0) return;
    constexpr int CPR = BN / 8;   // 16-byte chunks per tile row
    for (int c = tid; c < BM * CPR; c += 512) {
        const int row = c / CPR, col = (c - row * CPR) * 8;
        const int m = m0 + row;
        if (m >= a.M) continue;
        const int f = m / per_frame;
        const int rem = m - f * per_frame;
        const int x = rem - (rem / Wp) * Wp;
        if (x >= a.W) continue;
        const int n = n0 + col;
        if (n >= a.cout) continue;
        const size_t pos = (size_t)m + (size_t)f * 2 * Wp + Wp + 1;
        const uint4 v = *reinterpret_cast<const uint4*>(tile + row * TSTRIDE + col);
        const bool full = n + 8 <= a.cout;
        for (int d = 0; d < a.ndst; ++d) {
            uint16_t* dst = a.dst[d] + pos * a.dst_cs[d] + a.dst_coff[d] + n;
            if (full && ((a.dst_coff[d] | a.dst_cs[d]) & 7) == 0) {
                *reinterpret_cast<uint4*>(dst) = v;
            } else {
                const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    if (n + e < a.cout) dst[e] = (uint16_t)(wv[e >> 1] >> (16 * (e & 1)));
            }
        }
    }
}

}  // namespace

void launch_conv2(const ConvArgs& a, int bn, hipStream_t stream)
{
    OPK_CHECK_ARG(a.cin_pad % 32 == 0 && a.cin_pad > 0, "cin_pad must be a multiple of 32");
    OPK_CHECK_ARG(a.in_cs % 8 == 0 && a.in_coff % 8 == 0, "input slice must be 16-byte aligned");
    OPK_CHECK_ARG(a.in_coff + a.cin_pad <= a.in_cs, "input slice exceeds the buffer");
    OPK_CHECK_ARG(a.ntaps == 1 || a.ntaps == 9, "1 or 9 taps");
    OPK_CHECK_ARG(a.ksteps * 64 >= a.ntaps * a.cin_pad, "ksteps too small");
    OPK_CHECK_ARG(a.M > 0 && a.cout > 0 && a.ndst >= 0 && a.ndst <= kConvMaxDst, "bad sizes");
    dim3 grid(((a.M + BM2 - 1) / BM2) * ((a.cout + bn - 1) / bn));   // 1-D, remapped in-kernel
    switch (bn) {
        case 32: hipLaunchKernelGGL((conv2_kernel<32, 3>), grid, dim3(512), 0, stream, a); break;
        case 64: hipLaunchKernelGGL((conv2_kernel<64, 3>), grid, dim3(512), 0, stream, a); break;
        case 96: hipLaunchKernelGGL((conv2_kernel<96, 3>), grid, dim3(512), 0, stream, a); break;
        case 128: hipLaunchKernelGGL((conv2_kernel<128, 3>), grid, dim3(512), 0, stream, a); break;
        case 256: hipLaunchKernelGGL((conv2_kernel<256, 2>), grid, dim3(512), 0, stream, a); break;
        default: throw Error(1, "launch_conv2: unsupported BN " + std::to_string(bn));
    }
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
