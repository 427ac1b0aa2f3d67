// conv3_dev.h -- device helpers shared by the halo implicit-GEMM conv kernels (conv3.hip,
// conv3w.hip): vector types, the LDS swizzle of 64-byte rows, counted vmcnt waits, the
// "virtual image" strip geometry (see conv3.hip's header comment).
#pragma once
#include "conv.h"

// OPK_ZC: a tile's first K step takes the MFMA's zero C operand instead of accumulators zeroed
// after the previous tile's epilogue (conv3w; 0 = the zeroing, dev A/B builds).  Measured
// (profiles/round3/zc/): conv3w<96> -1.5 %, conv3w<128> -0.3 %; in conv3w8 +0.6 %, so not there
#ifndef OPK_ZC
#define OPK_ZC 1
#endif

namespace opk {
namespace conv3dev {

typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef float float2_t __attribute__((ext_vector_type(2)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));

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

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (0..15)
__device__ __forceinline__ void vm_wait_rt(int n)
{
    switch (n) {
    case 0: vm_wait<0>(); break;
    case 1: vm_wait<1>(); break;
    case 2: vm_wait<2>(); break;
    case 3: vm_wait<3>(); break;
    case 4: vm_wait<4>(); break;
    case 5: vm_wait<5>(); break;
    case 6: vm_wait<6>(); break;
    case 7: vm_wait<7>(); break;
    case 8: vm_wait<8>(); break;
    case 9: vm_wait<9>(); break;
    case 10: vm_wait<10>(); break;
    case 11: vm_wait<11>(); break;
    case 12: vm_wait<12>(); break;
    case 13: vm_wait<13>(); break;
    case 14: vm_wait<14>(); break;
    case 15: vm_wait<15>(); break;
    default: vm_wait<0>(); break;
    }
}

// n / d for 0 <= n < 2^24, 0 < d (float reciprocal estimate, then one correction step): a few VALU
// instead of the ~40-instruction integer division sequence
__device__ __forceinline__ int fdiv(int n, int d, float rd)
{
    int q = (int)((float)n * rd);
    const int r = n - (int)__umul24((unsigned)q, (unsigned)d);   // q, d < 2^24
    q += (r >= d) ? 1 : 0;
    q -= (r < 0) ? 1 : 0;
    return q;
}

// virtual-image geometry (see the header comment)
// B = the zero border of every activation buffer of the net (1 for BODY_25; the pad of its widest
// convolution in general, 3 for the 7x7 stages of COCO / MPI / face / hand)
struct Strips {
    int H, B, Hp, Wp, sw, VW, nstrips, fposV, total;
    float rf, rv, rs;   // reciprocals of fposV, VW, nstrips
    __device__ Strips(const ConvArgs& a)
        : H(a.H), B(a.border), Hp(a.H + 2 * a.border), Wp(a.W + 2 * a.border), sw(a.sw),
          VW(a.sw + 2 * a.border), nstrips(a.nstrips), fposV((a.H + 2 * a.border) * (a.sw + 2 * a.border)),
          total(a.frames * a.nstrips * (a.H + 2 * a.border) * (a.sw + 2 * a.border)),
          rf(a.rcp[0]), rv(a.rcp[1]), rs(a.rcp[2])
    {
    }
    // virtual position (yy, xx) of strip s is an output pixel of the image
    __device__ bool interior(int yy, int xx, int s, int W) const
    {
        return yy >= B && yy < H + B && xx >= B && xx < sw + B && s * sw + xx - B < W;
    }
    // padded-image position of virtual position v (any v; outside the image -> -1, a zeroed guard)
    template <bool FAST = true>
    __device__ long map(int v, int& f, int& yy, int& xx, int& s) const
    {
        if (v < 0 || v >= total) {
            f = 0;
            yy = -1;
            xx = -1;
            s = 0;
            return -1;
        }
        const int vf = FAST ? fdiv(v, fposV, rf) : v / fposV;
        const int rem = v - vf * fposV;
        yy = FAST ? fdiv(rem, VW, rv) : rem / VW;
        xx = rem - yy * VW;
        f = FAST ? fdiv(vf, nstrips, rs) : vf / nstrips;
        s = vf - f * nstrips;
        return (long)(f * Hp + yy) * Wp + s * sw + xx;
    }
    // one strip (the virtual image is the padded image): the MF epilogue rows p0 + 16 i of a lane
    // -- their padded positions (0 past the end) and whether they are output pixels -- with one
    // float-reciprocal division pair for row 0 and branch-free 16-position steps after it, 24-bit
    // multiplies (positions < 2^24, launch checks) instead of the divergent per-row carries of map()
    template <int MF>
    __device__ void rows1(int p0, int W, int (&prow)[MF], bool (&pok)[MF]) const
    {
        const int fr = fdiv(p0, fposV, rf);
        const int rem = p0 - (int)__umul24((unsigned)fr, (unsigned)fposV);
        int yy = fdiv(rem, VW, rv);
        int xx = rem - (int)__umul24((unsigned)yy, (unsigned)VW);
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            if (i > 0) {   // VW > 16 (host): at most one row carry per step
                xx += 16;
                const bool w = xx >= VW;
                xx = w ? xx - VW : xx;
                yy += w ? 1 : 0;
                yy = yy == Hp ? 0 : yy;
            }
            const int p = p0 + 16 * i;
            const bool in = p < total;
            prow[i] = in ? p : 0;
            pok[i] = in && (unsigned)(yy - B) < (unsigned)H && (unsigned)(xx - B) < (unsigned)W;
        }
    }
    // padded-image position of virtual position v only (halo rows): with one strip the virtual
    // image IS the padded image (sw = W, VW = Wp), so no division is needed
    __device__ long pos(int v) const
    {
        if (nstrips == 1) return v >= 0 && v < total ? v : -1;
        int f, yy, xx, s;
        return map(v, f, yy, xx, s);
    }
};

// epilogue activation of t = acc + bias with tm = t * m (m = 1 none, 0 ReLU, slope PReLU):
// MX (ConvArgs::actmax, every m in [0, 1]) -> max(t, tm), which equals the select for every finite t
template <bool MX>
__device__ __forceinline__ float act_pick(float t, float tm)
{
    return MX ? __builtin_fmaxf(t, tm) : (t > 0.f ? t : tm);
}

// the same on a fragment's four values, kept as vector operations so that the bias add and the
// multiply before it stay packed (v_pk_add_f32 / v_pk_mul_f32) instead of being scalarised
template <bool MX>
__device__ __forceinline__ float4_t act_pick4(float4_t t, float4_t tm)
{
    if constexpr (MX) return __builtin_elementwise_max(t, tm);
    float4_t r;
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = t[k] > 0.f ? t[k] : tm[k];
    return r;
}

// 16-byte / 8-byte buffer stores through a raw buffer resource over a destination slice: lanes
// whose byte offset is kOOB (>= num_records) are dropped by the range check, so a masked-off lane
// needs neither a branch nor a sink address, and the address is one 32-bit VGPR per position
constexpr uint32_t kBufOOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

#define OPK3_VM_CASE(n_) case n_: vm_wait<n_>(); break;
__device__ __forceinline__ void vm_wait_rt64(int n)
{
    switch (n) {
        OPK3_VM_CASE(0) OPK3_VM_CASE(1) OPK3_VM_CASE(2) OPK3_VM_CASE(3) OPK3_VM_CASE(4)
        OPK3_VM_CASE(5) OPK3_VM_CASE(6) OPK3_VM_CASE(7) OPK3_VM_CASE(8) OPK3_VM_CASE(9)
        OPK3_VM_CASE(10) OPK3_VM_CASE(11) OPK3_VM_CASE(12) OPK3_VM_CASE(13) OPK3_VM_CASE(14)
        OPK3_VM_CASE(15) OPK3_VM_CASE(16) OPK3_VM_CASE(17) OPK3_VM_CASE(18) OPK3_VM_CASE(19)
        OPK3_VM_CASE(20) OPK3_VM_CASE(21) OPK3_VM_CASE(22) OPK3_VM_CASE(23) OPK3_VM_CASE(24)
        OPK3_VM_CASE(25) OPK3_VM_CASE(26) OPK3_VM_CASE(27) OPK3_VM_CASE(28) OPK3_VM_CASE(29)
        OPK3_VM_CASE(30) OPK3_VM_CASE(31) OPK3_VM_CASE(32) OPK3_VM_CASE(33) OPK3_VM_CASE(34)
        OPK3_VM_CASE(35) OPK3_VM_CASE(36) OPK3_VM_CASE(37) OPK3_VM_CASE(38) OPK3_VM_CASE(39)
        OPK3_VM_CASE(40) OPK3_VM_CASE(41) OPK3_VM_CASE(42) OPK3_VM_CASE(43) OPK3_VM_CASE(44)
        OPK3_VM_CASE(45) OPK3_VM_CASE(46) OPK3_VM_CASE(47) OPK3_VM_CASE(48) OPK3_VM_CASE(49)
        OPK3_VM_CASE(50) OPK3_VM_CASE(51) OPK3_VM_CASE(52) OPK3_VM_CASE(53) OPK3_VM_CASE(54)
        OPK3_VM_CASE(55) OPK3_VM_CASE(56) OPK3_VM_CASE(57) OPK3_VM_CASE(58) OPK3_VM_CASE(59)
        OPK3_VM_CASE(60) OPK3_VM_CASE(61) OPK3_VM_CASE(62) OPK3_VM_CASE(63)
    default: vm_wait<0>(); break;
    }
}
#undef OPK3_VM_CASE

}  // namespace conv3dev
}  // namespace opk
