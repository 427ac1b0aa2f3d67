// conv1_fused.hip -- conv1_1 -> ReLU -> conv1_2 -> ReLU -> pool1 of the VGG front end in ONE kernel.
//
// Reference layers (models/pose/body_25/pose_deploy.prototxt, run by NetCaffe::forwardPass,
// netCaffe.cpp:248): conv1_1 (3 -> 64, 3x3) + relu1_1, conv1_2 (64 -> 64, 3x3) + relu1_2,
// pool1_stage1 (2x2/2 max).  At 368x656 these are the only full-resolution layers; unfused they
// write and re-read two 64-channel fp16 images (2 x 31 MB per frame) and are bound by that
// traffic (profiles/round1: conv_image + conv1_2 + pool1 = 3.4 ms per 64 frames).
//
// Here a persistent workgroup per CU keeps conv1_2's weights (72 KB) resident in LDS and walks
// tiles of TR x TC output pixels.  Per tile:
//   1. the fp32 NCHW image patch (TR+4) x (TC+4) x 3 is staged in LDS (prefetched in registers
//      during the previous tile's conv1_2);
//   2. conv1_1 is evaluated for the (TR+2) x (TC+2) halo conv1_2 needs, as MFMAs with K = 27
//      gathered from the patch; bias + activation, fp16, zero outside the image, written to LDS
//      in the swizzled 64-byte-row layout conv3.hip uses for its A operand;
//   3. conv1_2 is an implicit GEMM over the halo's "virtual image" of row width VW = 64
//      (TR x 64 rows, columns >= TC discarded): 2 channel chunks x 9 taps, no barrier inside;
//   4. bias + activation, fp16 tile to LDS, 2x2 max, one 16-byte store per 8 pooled channels.
// LDS writes of fp16 results go through v_permlane16_swap of fragment pairs so that every lane
// writes 16 consecutive bytes (ds_write_b128) instead of 8 (fewer instructions, fewer conflicts).
// Only the image is read and only pool1's output is written.
#include "conv.h"

#include <algorithm>

#include "../common.h"
#include "conv3_dev.h"

namespace opk {

namespace {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef float float2_t __attribute__((ext_vector_type(2)));

#ifndef OPK1_ABLATE   // dev probe only (variant builds): 1 no conv1_1 gather / MFMAs, 2 no conv1_2
#define OPK1_ABLATE 0  // MFMAs, 3 no epilogue + pooling (timing only, wrong results)
#endif

constexpr int TR = 6, TC = 62, VW = 64;       // tile rows / columns; virtual row width
constexpr int MT = TR * VW;                   // GEMM rows per tile (384)
constexpr int HROWS = (TR + 2) * VW + 8;      // halo rows (+ overflow of the last taps)
constexpr int PR = TR + 4, PCW = TC + 4;      // image patch rows / columns
constexpr int PATCH = 3 * PR * PCW;           // patch floats
// LDS patch layout, chosen so that conv1_1's K gathers are free of bank conflicts: row stride PC
// and plane stride PS with PS = 11, PC = 3 (mod 32) give every K pair (k, k + 8) of a lane pair
// q, q + 1 the same offset difference (24 mod 32), and lane rows q = 1, 3 read a second copy of
// the patch at D = 24 (mod 32) -- so the 16-float runs of the two lane rows of a ds_read_b32 group
// fall on opposite bank halves (tools/lds_conflicts.py models it)
constexpr int PC = 67, PS = 683, PD = 2072;
static_assert(PC >= PCW && PS >= PR * PC && PC % 32 == 3 && PS % 32 == 11 && PD % 32 == 24, "patch layout");
constexpr int PATCH_LDS = PD + 3 * PS;        // floats, both copies
constexpr int NT = 512;                       // lanes per workgroup (8 waves)
constexpr int PPL = (PATCH + NT - 1) / NT;    // patch floats per lane
constexpr int TSTRIDE = 72;                   // epilogue tile row stride in halves (16-B rows)
constexpr int W2_PIECES = 18 * 64 * 4;        // 2 chunks x 9 taps x 64 rows x 4 x 16 B
constexpr int HALO_PIECES = 2 * HROWS * 4;
constexpr int LDS_BYTES = (W2_PIECES + HALO_PIECES) * 16 + (PATCH_LDS * 4 + 15) / 16 * 16;
static_assert(MT * TSTRIDE * 2 <= HALO_PIECES * 16, "epilogue tile fits in the halo");
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");

// conv1_2's weights: the conv3 packing's swizzle (DMA'd as packed on the host)
__device__ __forceinline__ int swz64(int row, int piece) { return row * 4 + (piece ^ (((row >> 2) & 1) << 1)); }
// the halo (written by conv1_1's epilogue, read as conv1_2's A fragments): piece ^ ((row >> 1) & 3)
// keeps the fragment reads conflict-free and also the epilogue's ds_write_b128 (8 consecutive rows
// of one piece per lane group land on 8 distinct 16-byte bank slots)
__device__ __forceinline__ int swzh(int row, int piece) { return row * 4 + (piece ^ ((row >> 1) & 3)); }

__device__ __forceinline__ uint32_t hmax4(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
    const half2_t m = __builtin_elementwise_max(
        __builtin_elementwise_max(__builtin_bit_cast(half2_t, a), __builtin_bit_cast(half2_t, b)),
        __builtin_elementwise_max(__builtin_bit_cast(half2_t, c), __builtin_bit_cast(half2_t, d)));
    return __builtin_bit_cast(uint32_t, m);
}

// MX: activations as max(t, t*m) (Conv1FusedArgs::actmax, conv3_dev.h act_pick)
template <bool MX>
__global__ __launch_bounds__(NT, 1) void conv1_fused_kernel(const Conv1FusedArgs a)
{
    __shared__ uint4 lds[LDS_BYTES / 16];
    uint4* W2 = lds;
    uint4* HALO = lds + W2_PIECES;
    float* patch = reinterpret_cast<float*>(lds + W2_PIECES + HALO_PIECES);
    uint16_t* T = reinterpret_cast<uint16_t*>(HALO);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r16 = lane & 15, q = lane >> 4;
    const int H = a.H, W = a.W;
    const int tiles_x = (W + TC - 1) / TC, tiles_y = (H + TR - 1) / TR;
    const int ntiles = a.frames * tiles_x * tiles_y;

    // ---- resident conv1_2 weights: conv3 packing [c][ky][kx][64 n][32 ci], swizzled rows ------
    {
        const int lrow = lane >> 2, phys = lane & 3;
#pragma unroll
        for (int k = 0; k < W2_PIECES / NT; ++k) {
            const int inst = k * 8 + wave;            // 1 KiB = 16 rows of one unit
            const int row = inst * 16 + lrow;         // global row over all 18 units
            const int lp = phys ^ (((row >> 2) & 1) << 1);
            __builtin_amdgcn_global_load_lds((const void*)(a.w2 + (size_t)row * 32 + lp * 8),
                                             (__attribute__((address_space(3))) void*)(&W2[inst * 64]),
                                             16, 0, 0);
        }
    }
    // conv1_1 weights as MFMA A operand (rows = output channels g*16 + r16, K = 8q .. 8q+7)
    half8_t w1f[4];
    float4_t b1[4], m1[4], b2[4], m2[4];
    const float neg1 = a.act1 == 1 ? 0.f : 1.f, neg2 = a.act2 == 1 ? 0.f : 1.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        w1f[g] = *reinterpret_cast<const half8_t*>(a.w1 + (size_t)(g * 16 + r16) * 64 + 8 * q);
        const int ch = g * 16 + 4 * q;   // bias/slope arrays are zero-padded to 128 channels
        b1[g] = *reinterpret_cast<const float4_t*>(a.b1 + ch);
        const float4_t s1 = *reinterpret_cast<const float4_t*>(a.s1 + ch);
        m1[g] = a.act1 == 2 ? s1 : float4_t{neg1, neg1, neg1, neg1};
        b2[g] = *reinterpret_cast<const float4_t*>(a.b2 + ch);
        const float4_t s2 = *reinterpret_cast<const float4_t*>(a.s2 + ch);
        m2[g] = a.act2 == 2 ? s2 : float4_t{neg2, neg2, neg2, neg2};
    }
    // this lane's 8 conv1_1 K values: patch offset of (ci, ky, kx) for k = 8q + e (lane rows
    // q = 1, 3 in the second copy); K padding (k > 26, lane row 3) reads a dummy word 16 banks from
    // its lane-row-2 partner's and is zeroed after the read, so the eight reads issue back to back
    auto poff = [](int k) {
        const int t = k / 3, ci = k - 3 * (k / 3);
        return ci * PS + (t / 3) * PC + (t - 3 * (t / 3));
    };
    int off[8];
    unsigned kvalid = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int k = 8 * q + e;
        off[e] = k < 27 ? poff(k) + (q & 1) * PD : poff(k - 8) + 16;
        kvalid |= (k < 27 ? 1u : 0u) << e;
    }

#define OPK1_ORIGIN(tile_, f_, y0_, x0_)                                                       \
    do {                                                                                      \
        const int tx_ = (tile_) % tiles_x;                                                    \
        const int rest_ = (tile_) / tiles_x;                                                  \
        y0_ = (rest_ % tiles_y) * TR;                                                         \
        f_ = rest_ / tiles_y;                                                                 \
        x0_ = tx_ * TC;                                                                       \
    } while (0)
    // image patch of a tile: rows y0-2 .. y0+TR+1, columns x0-2 .. x0+TC+1, zero outside
    float pre[PPL];
#define OPK1_LOAD_PATCH(tile_)                                                                \
    do {                                                                                      \
        int f_, y0_, x0_;                                                                     \
        OPK1_ORIGIN(tile_, f_, y0_, x0_);                                                     \
        const float* src_ = a.img + (size_t)f_ * 3 * H * W;                                   \
        _Pragma("unroll") for (int k_ = 0; k_ < PPL; ++k_) {                                  \
            const int i_ = tid + k_ * NT;                                                     \
            float v_ = 0.f;                                                                   \
            if (i_ < PATCH && (tile_) < ntiles) {                                             \
                const int ci_ = i_ / (PR * PCW);                                              \
                const int rem_ = i_ - ci_ * (PR * PCW);                                       \
                const int r_ = rem_ / PCW, c_ = rem_ - (rem_ / PCW) * PCW;                    \
                const int y_ = y0_ - 2 + r_, x_ = x0_ - 2 + c_;                               \
                if (y_ >= 0 && y_ < H && x_ >= 0 && x_ < W)                                   \
                    v_ = src_[((size_t)ci_ * H + y_) * W + x_];                               \
            }                                                                                 \
            pre[k_] = v_;                                                                     \
        }                                                                                     \
    } while (0)

    // pool pass lane roles: ds_read_b128 lane group g (0-3) of this lane and its index k in the
    // group -> pixel g + 4 (k >> 3), channel group k & 7
    int pool_dp, pool_cg;
    {
        const unsigned g1m = 0xF00F0FF0u;          // lanes {4-11, 16-19, 28-31} of each half
        const int lo = lane & 31;
        const bool g1 = (g1m >> lo) & 1u;
        const unsigned same = g1 ? g1m : ~g1m;
        const int k = __popc(same & ((1u << lo) - 1u));
        pool_dp = (g1 ? 1 : 0) + 2 * (lane >> 5) + 4 * (k >> 3);
        pool_cg = k & 7;
    }

    // LDS index of this lane's patch floats (element tid + k * NT of [3][PR][PCW]), -1 past the end
    int pli[PPL];
#pragma unroll
    for (int k = 0; k < PPL; ++k) {
        const int i = tid + k * NT;
        const int ci = i / (PR * PCW), rem = i - ci * (PR * PCW);
        const int r = rem / PCW, cc = rem - r * PCW;
        pli[k] = i < PATCH ? ci * PS + r * PC + cc : -1;
    }

    int tile = blockIdx.x;
    OPK1_LOAD_PATCH(tile);
    for (; tile < ntiles; tile += gridDim.x) {
        int f, y0, x0;
        OPK1_ORIGIN(tile, f, y0, x0);
        __syncthreads();   // previous tile's pooling reads of T (aliasing the halo) are done
#pragma unroll
        for (int k = 0; k < PPL; ++k)
            if (pli[k] >= 0) {
                patch[pli[k]] = pre[k];
                patch[PD + pli[k]] = pre[k];
            }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // resident weights (first tile)
        __syncthreads();

        // ---- conv1_1 over the (TR+2) x 64 halo: 32 groups of 16 positions, 4 per wave ------
        // all 32 patch reads of the wave's 4 groups first (one LDS round trip), then the MFMAs
        float xv[4][8];
#pragma unroll
        for (int gi = 0; gi < 4; ++gi) {
            const int mh = (wave * 4 + gi) * 16 + r16;
            const int base = (mh >> 6) * PC + (mh & 63);   // patch row / column of the halo position
#pragma unroll
            for (int e = 0; e < 8; ++e) xv[gi][e] = patch[off[e] + base];
        }
        // the 16 MFMAs of the wave's 4 groups, then their epilogues (no MFMA result is waited
        // for right after its issue)
        float4_t c1[4][4];
#pragma unroll
        for (int gi = 0; gi < 4; ++gi) {
            half8_t xf;
#pragma unroll
            for (int e = 0; e < 8; ++e)
                xf[e] = OPK1_ABLATE == 1 ? (_Float16)0.f
                        : ((kvalid >> e) & 1u) ? (_Float16)xv[gi][e] : (_Float16)0.f;
#pragma unroll
            for (int g = 0; g < 4; ++g)
                c1[gi][g] = OPK1_ABLATE == 1 ? float4_t{(float)xf[0], 0.f, 0.f, 0.f}
                    : __builtin_amdgcn_mfma_f32_16x16x32_f16(w1f[g], xf, float4_t{0.f, 0.f, 0.f, 0.f},
                                                             0, 0, 0);
        }
#pragma unroll
        for (int gi = 0; gi < 4; ++gi) {
            const int mh = (wave * 4 + gi) * 16 + r16;       // halo position
            const int hr = mh >> 6, hc = mh & 63;
            const int y = y0 - 1 + hr, x = x0 - 1 + hc;
            const bool in = y >= 0 && y < H && x >= 0 && x < W;
            uint32_t pk[4][2];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4_t t = c1[gi][g] + b1[g];
                const float4_t a_ = conv3dev::act_pick4<MX>(t, t * m1[g]);   // packed add / mul
                const float4_t v = in ? a_ : float4_t{0.f, 0.f, 0.f, 0.f};
                pk[g][0] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v.xy, half2_t));
                pk[g][1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v.zw, half2_t));
            }
            // chunk c = channels 32c .. 32c+31 (groups 2c, 2c+1): v_permlane16_swap between lane
            // rows q and q^1 leaves lane row q channels 16 (q & 1) + 8 (q >> 1) .. +7 of the chunk,
            // i.e. 16-byte piece 2 (q & 1) + (q >> 1): one ds_write_b128 per chunk (8-lane groups,
            // at most 2-way bank conflicts) instead of two 4-way conflicting ds_write_b64
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const auto sl = __builtin_amdgcn_permlane16_swap(pk[2 * c][0], pk[2 * c + 1][0], false, false);
                const auto sh = __builtin_amdgcn_permlane16_swap(pk[2 * c][1], pk[2 * c + 1][1], false, false);
                HALO[c * HROWS * 4 + swzh(mh, 2 * (q & 1) + (q >> 1))] = make_uint4(sl[0], sh[0], sl[1], sh[1]);
            }
        }
        __syncthreads();

        // ---- prefetch the next tile's patch; conv1_2 from LDS only -----------------------------
        OPK1_LOAD_PATCH(tile + gridDim.x);
        float4_t acc[3][4];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = float4_t{0.f, 0.f, 0.f, 0.f};
        // 18 K steps (2 channel chunks x 9 taps); step s+1's fragments are read while step s's
        // MFMAs issue (two register sets, the issue order pinned by sched_barrier)
        half8_t fa[2][3], fb[2][4];
#define OPK1_READ(buf_, st_)                                                                  \
    do {                                                                                      \
        const int c_ = (st_) / 9, tap_ = (st_) - 9 * ((st_) / 9);                             \
        const int ky_ = tap_ / 3, kx_ = tap_ - 3 * (tap_ / 3);                                \
        const uint4* As_ = HALO + c_ * HROWS * 4;                                             \
        const uint4* Bs_ = W2 + (c_ * 9 + tap_) * 256;                                        \
        _Pragma("unroll") for (int i_ = 0; i_ < 3; ++i_)                                      \
            fa[buf_][i_] = __builtin_bit_cast(                                                \
                half8_t, As_[swzh(wave * 48 + i_ * 16 + r16 + ky_ * VW + kx_, q)]);             \
        _Pragma("unroll") for (int j_ = 0; j_ < 4; ++j_)                                      \
            fb[buf_][j_] = __builtin_bit_cast(half8_t, Bs_[swz64(j_ * 16 + r16, q)]);           \
    } while (0)
        OPK1_READ(0, 0);
#pragma unroll
        for (int st = 0; st < 18; ++st) {
            const int cur = st & 1;
            if (st + 1 < 18) OPK1_READ(cur ^ 1, st + 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (OPK1_ABLATE == 2)
                        asm volatile("; mfma skipped" : "+v"(acc[i][j]) : "v"(fb[cur][j]), "v"(fa[cur][i]));
                    else
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[cur][j], fa[cur][i],
                                                                           acc[i][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
#undef OPK1_READ
        __syncthreads();   // every wave is done reading the halo: T may overwrite it

        if (OPK1_ABLATE == 3) {   // keep the accumulators alive, skip epilogue and pooling
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) asm volatile("" :: "v"(acc[i][j]));
            continue;
        }
        // ---- bias + activation -> fp16 tile [m][64 ch] -----------------------------------------
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int m = wave * 48 + i * 16 + r16;
            uint32_t pk[4][2];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float4_t t = acc[i][j] + b2[j];
                const float4_t v = conv3dev::act_pick4<MX>(t, t * m2[j]);   // packed add / mul
                pk[j][0] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v.xy, half2_t));
                pk[j][1] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v.zw, half2_t));
            }
            // fragment pairs as in the halo write: 8 consecutive channels per lane, ds_write_b128
#pragma unroll
            for (int j = 0; j < 4; j += 2) {
                const auto sl = __builtin_amdgcn_permlane16_swap(pk[j][0], pk[j + 1][0], false, false);
                const auto sh = __builtin_amdgcn_permlane16_swap(pk[j][1], pk[j + 1][1], false, false);
                *reinterpret_cast<uint4*>(T + m * TSTRIDE + j * 16 + 16 * (q & 1) + 8 * (q >> 1)) =
                    make_uint4(sl[0], sh[0], sl[1], sh[1]);
            }
        }
        __syncthreads();

        // ---- 2x2 max pool: (TR/2) x (TC/2) pooled pixels x 8 channel groups ---------------------
        // A wave takes 8 pixels of one pooled row at a time (slots of 32 per row, the 32nd unused);
        // each 16-lane group of ds_read_b128 (MI355X_MICROARCH.md §LDS) reads pixels p and p + 4,
        // 8 channel groups each: 2 x 128 contiguous bytes 8 positions (= 32 banks mod 64) apart,
        // so the reads are free of bank conflicts (tools/lds_conflicts.py)
        for (int it = wave; it < (TR / 2) * 4; it += NT / 64) {
            const int slot = it * 8 + pool_dp;
            const int cg = pool_cg;
            const int pr = slot >> 5, pc = slot & 31;
            const int oy = y0 / 2 + pr, ox = x0 / 2 + pc;
            if (pc >= TC / 2 || 2 * oy + 1 >= H || 2 * ox + 1 >= W) continue;
            const int m0 = (2 * pr) * VW + 2 * pc;
            const uint16_t* s0 = T + m0 * TSTRIDE + cg * 8;
            uint4 v0 = *reinterpret_cast<const uint4*>(s0);
            const uint4 v1 = *reinterpret_cast<const uint4*>(s0 + TSTRIDE);
            const uint4 v2 = *reinterpret_cast<const uint4*>(s0 + VW * TSTRIDE);
            const uint4 v3 = *reinterpret_cast<const uint4*>(s0 + (VW + 1) * TSTRIDE);
            // packed fp16 max (v_pk_max_f16): the window's maximum; it may differ from Caffe's
            // ordered comparison only in the sign of a zero, which no later conv or pool
            // distinguishes (products of +-0 are zeros, and sums start at +0)
            v0.x = hmax4(v0.x, v1.x, v2.x, v3.x);
            v0.y = hmax4(v0.y, v1.y, v2.y, v3.y);
            v0.z = hmax4(v0.z, v1.z, v2.z, v3.z);
            v0.w = hmax4(v0.w, v1.w, v2.w, v3.w);
            uint16_t* dst = a.out + (((size_t)f * (a.OH + 2) + oy + 1) * (a.OW + 2) + ox + 1) * a.out_cs +
                            a.out_coff + cg * 8;
            *reinterpret_cast<uint4*>(dst) = v0;
        }
    }
#undef OPK1_LOAD_PATCH
#undef OPK1_ORIGIN
}

}  // namespace

bool conv1_fused_supported(int H, int W, int cout1, int cout2)
{
    return cout1 == 64 && cout2 == 64 && H % 2 == 0 && W % 2 == 0 && H >= 2 && W >= 2;
}

void launch_conv1_fused(const Conv1FusedArgs& a, int workgroups, hipStream_t stream)
{
    OPK_CHECK_ARG(a.img && a.w1 && a.w2 && a.out && a.b1 && a.b2 && a.s1 && a.s2, "NULL argument");
    OPK_CHECK_ARG(a.frames > 0 && conv1_fused_supported(a.H, a.W, 64, 64), "conv1 fusion: sizes");
    OPK_CHECK_ARG(a.OH == a.H / 2 && a.OW == a.W / 2, "conv1 fusion: pooled size");
    OPK_CHECK_ARG(a.out_cs % 8 == 0 && a.out_coff % 8 == 0 && a.out_coff + 64 <= a.out_cs,
                  "conv1 fusion: 16-byte aligned output slice");
    const long tiles = (long)a.frames * ((a.W + TC - 1) / TC) * ((a.H + TR - 1) / TR);
    OPK_CHECK_ARG(tiles < (1L << 31), "conv1 fusion: too many tiles");
    const int grid = (int)std::min<long>(tiles, workgroups > 0 ? workgroups : 256);
    note_launch("conv1_fused_kernel<%d>", a.actmax ? 1 : 0);
    if (a.actmax) hipLaunchKernelGGL(conv1_fused_kernel<true>, dim3(grid), dim3(NT), 0, stream, a);
    else hipLaunchKernelGGL(conv1_fused_kernel<false>, dim3(grid), dim3(NT), 0, stream, a);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
