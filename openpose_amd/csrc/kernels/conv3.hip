// conv3.hip -- 3x3 convolutions on gfx950 MFMA with the input halo staged ONCE per channel chunk.
//
// Same role as conv2.hip (Caffe ConvolutionLayer + fused PReLU/ReLU + concat-by-slice,
// netCaffe.cpp:248) for the 3x3 layers whose image rows are short enough (W <= 164: the 46x82
// stage layers and conv3_x/conv4_x), where the implicit GEMM of conv2 re-reads every input row
// nine times (once per tap) and is bound by the per-CU LDS fill rate (profiles/round1).
//
// Here the GEMM row space M is the padded image itself ([frames][H+2][W+2] positions; border
// rows/columns are computed and discarded), so a tile of 256 consecutive positions needs, for a
// 32-channel chunk, the contiguous position range [p0 - Wp - 1, p0 + 256 + Wp + 1): one "halo"
// of HR rows x 64 B.  The K loop runs chunk-major, tap-minor in units (chunk, ky):
//   * unit (c, 0) stages the halo of chunk c (A slot c & 1) and the 3 kx-taps' weights;
//   * units (c, 1), (c, 2) stage only their 3 taps' weights (B slot u % 3, 24 KB each);
//   * every tap reads its A fragments from the SAME halo at row offset ky*Wp + kx.
// A traffic drops ~5x, B is unchanged (weights are L2-resident and shared by every tile).
// Staging is global_load_lds_dwordx4 (lane-linear LDS) with the swizzle applied on the source
// address; 64-byte rows use piece ^ (((row >> 2) & 1) << 1), conflict-free for the unaligned row
// windows the taps read (brute-forced over all ds_read_b128 lane groups and window offsets).
#include "conv.h"

#include "../common.h"

namespace opk {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float float4_t __attribute__((ext_vector_type(4)));

constexpr int BM3 = 256;
constexpr int BN3 = 128;

__device__ __forceinline__ int swz64(int row, int piece) { return row * 4 + (piece ^ (((row >> 2) & 1) << 1)); }

__device__ __forceinline__ uint16_t f2h_bits3(float v)
{
    const _Float16 h = (_Float16)v;
    return __builtin_bit_cast(uint16_t, h);
}

template <int N>
__device__ __forceinline__ void vm_wait()
{
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int HR>
__global__ __launch_bounds__(512, 2) void conv3_kernel(const ConvArgs a)
{
    constexpr int BM = BM3, BN = BN3;
    constexpr int WN = BN / 2, NF = WN / 16, MF = 4;
    constexpr int AI = HR / 128;                  // halo DMA instructions per wave (16 rows each)
    constexpr int BROWS = 3 * BN;                 // B rows per unit: kx-major, then channel n
    constexpr int BI = BROWS / 128;               // B DMA instructions per wave per unit (3)
    constexpr int ASLOT = HR * 4;                 // 16-byte pieces per halo slot
    constexpr int BSLOT = BROWS * 4;
    constexpr int LDS_PIECES = 2 * ASLOT + 3 * BSLOT;
    constexpr int TSTRIDE = BN + 8;
    static_assert(LDS_PIECES * 16 <= 160 * 1024, "LDS budget");
    static_assert(BM * TSTRIDE * 2 <= LDS_PIECES * 16, "epilogue tile fits");
    __shared__ uint4 lds[LDS_PIECES];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int Wp = a.W + 2;
    const int fpos = (a.H + 2) * Wp;              // positions per padded frame
    const int total = a.frames * fpos;
    const int ntile_m = (total + BM - 1) / BM;
    const int nn = (a.cout + BN - 1) / BN;
    // XCD-aware bijective tile order (see conv2.hip)
    const int nblk = gridDim.x;
    const int xcd = blockIdx.x & 7, qq = nblk >> 3, rr = nblk & 7;
    const int tix = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (blockIdx.x >> 3);
    const int p0 = (tix / nn) * BM;
    const int nb = tix - (tix / nn) * nn;
    const int n0 = nb * BN;
    (void)ntile_m;

    // ---- DMA lane geometry: 16 rows x 4 pieces per wave instruction --------------------------
    const int lrow = lane >> 2, phys = lane & 3;
    const int cpt = a.cin_pad >> 5;               // 32-channel chunks
    const int U = 3 * cpt;                        // units (chunk, ky)
    // halo row hr = (i*8 + wave)*16 + lrow, position p0 - Wp - 1 + hr
    const uint16_t* ain = a.in + a.in_coff;
    // packed weights: [nb][c][ky][kx][n 128][32 ch]; a unit is 3*128 rows of 64 B
    const uint16_t* wbase = a.w + (size_t)nb * cpt * 3 * BROWS * 32;

#define OPK3_ISSUE(u_)                                                                        \
    do {                                                                                      \
        const int c_ = (u_) / 3, ky_ = (u_) - 3 * ((u_) / 3);                                 \
        if (ky_ == 0) {                                                                       \
            const int as_ = (c_ & 1) * ASLOT;                                                 \
            _Pragma("unroll") for (int i_ = 0; i_ < AI; ++i_) {                               \
                const int hr_ = (i_ * 8 + wave) * 16 + lrow;                                  \
                const int lp_ = phys ^ (((hr_ >> 2) & 1) << 1);                               \
                const long pos_ = (long)p0 - Wp - 1 + hr_;                                    \
                __builtin_amdgcn_global_load_lds(                                             \
                    (const void*)(ain + pos_ * a.in_cs + c_ * 32 + lp_ * 8),                 \
                    (__attribute__((address_space(3))) void*)(&lds[as_ + (i_ * 8 + wave) * 64]), \
                    16, 0, 0);                                                                \
            }                                                                                 \
        }                                                                                     \
        const int bs_ = 2 * ASLOT + ((u_) % 3) * BSLOT;                                       \
        const uint16_t* ub_ = wbase + (size_t)(u_) * BROWS * 32;                              \
        _Pragma("unroll") for (int j_ = 0; j_ < BI; ++j_) {                                   \
            const int rb_ = (j_ * 8 + wave) * 16 + lrow;                                      \
            const int lp_ = phys ^ (((rb_ >> 2) & 1) << 1);                                   \
            __builtin_amdgcn_global_load_lds(                                                 \
                (const void*)(ub_ + rb_ * 32 + lp_ * 8),                                      \
                (__attribute__((address_space(3))) void*)(&lds[bs_ + (j_ * 8 + wave) * 64]),  \
                16, 0, 0);                                                                    \
        }                                                                                     \
    } while (0)

    float4_t acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};

    const int r16 = lane & 15, q = lane >> 4;
    OPK3_ISSUE(0);
    if (U > 1) OPK3_ISSUE(1);
    for (int u = 0; u < U; ++u) {
        const int ky = u - 3 * (u / 3);
        // wait for this wave's loads of unit u: units 0..u+1 have been issued, so only unit u+1's
        // loads (B, plus the next halo when u+1 starts a chunk) may stay in flight
        if (ky != 2) {
            vm_wait<BI>();
        } else {
            if (u + 1 < U) vm_wait<AI + BI>(); else vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();
        if (u + 2 < U) OPK3_ISSUE(u + 2);
        const uint4* As = lds + ((u / 3) & 1) * ASLOT;
        const uint4* Bs = lds + 2 * ASLOT + (u % 3) * BSLOT;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            half8_t af[MF], bf[NF];
            const int hoff = ky * Wp + kx;
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                const int hr = wm * 64 + i * 16 + r16 + hoff;
                af[i] = __builtin_bit_cast(half8_t, As[swz64(hr, q)]);
            }
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                const int rb = kx * BN + wn * WN + j * 16 + r16;
                bf[j] = __builtin_bit_cast(half8_t, Bs[swz64(rb, q)]);
            }
#pragma unroll
            for (int i = 0; i < MF; ++i)
#pragma unroll
                for (int j = 0; j < NF; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i], bf[j], acc[i][j], 0,
                                                                       0, 0);
        }
    }
#undef OPK3_ISSUE
    vm_wait<0>();
    __syncthreads();

    // ---- epilogue (padded-position rows; border positions are discarded) -----------------------
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
                const int pos = p0 + ml;
                f = pos / fpos;
                const int rem = pos - f * fpos;
                y = rem / Wp - 1;
                x = rem - (y + 1) * Wp - 1;
                valid = pos < total && y >= 0 && y < a.H && x >= 0 && x < a.W;
            }
#pragma unroll
            for (int j = 0; j < NF; ++j) {
                float v = acc[i][j][r] + bias[j];
                if (a.act == 1) v = v > 0.f ? v : 0.f;
                else if (a.act == 2) v = v > 0.f ? v : v * slope[j];
                tile[ml * TSTRIDE + wn * WN + j * 16 + r16] = f2h_bits3(v);
                if (valid && co[j] < a.cout)
                    a.out32[(((size_t)f * a.out32_c + a.out32_coff + co[j]) * a.H + y) * a.W + x] = v;
            }
        }
    __syncthreads();
    if (a.ndst == 0) return;
    constexpr int CPR = BN / 8;
    for (int c = tid; c < BM * CPR; c += 512) {
        const int row = c / CPR, col = (c - row * CPR) * 8;
        const int pos = p0 + row;
        if (pos >= total) continue;
        const int f = pos / fpos;
        const int rem = pos - f * fpos;
        const int y = rem / Wp;
        const int x = rem - y * Wp;
        if (y < 1 || y > a.H || x < 1 || x > a.W) continue;
        const int n = n0 + col;
        if (n >= a.cout) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(tile + row * TSTRIDE + col);
        const bool full = n + 8 <= a.cout;
        for (int d = 0; d < a.ndst; ++d) {
            uint16_t* dst = a.dst[d] + (size_t)pos * a.dst_cs[d] + a.dst_coff[d] + n;
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

int conv3_halo_rows(int W)
{
    const int need = BM3 + 2 * (W + 2) + 2;
    if (need <= 512) return 512;
    if (need <= 640) return 640;
    return 0;
}

void launch_conv3(const ConvArgs& a, hipStream_t stream)
{
    OPK_CHECK_ARG(a.ntaps == 9 && a.cin_pad % 32 == 0 && a.cin_pad > 0, "3x3, cin_pad % 32 == 0");
    OPK_CHECK_ARG(a.in_cs % 8 == 0 && a.in_coff % 8 == 0, "input slice must be 16-byte aligned");
    OPK_CHECK_ARG(a.in_coff + a.cin_pad <= a.in_cs, "input slice exceeds the buffer");
    OPK_CHECK_ARG(a.M > 0 && a.cout > 0 && a.ndst <= kConvMaxDst, "bad sizes");
    const int hr = conv3_halo_rows(a.W);
    OPK_CHECK_ARG(hr > 0, "row too long for the halo kernel");
    const int total = a.frames * (a.H + 2) * (a.W + 2);
    dim3 grid(((total + BM3 - 1) / BM3) * ((a.cout + BN3 - 1) / BN3));
    if (hr == 512) hipLaunchKernelGGL(conv3_kernel<512>, grid, dim3(512), 0, stream, a);
    else hipLaunchKernelGGL(conv3_kernel<640>, grid, dim3(512), 0, stream, a);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
