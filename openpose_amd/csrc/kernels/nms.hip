// nms.hip -- body-part peak extraction for gfx950 with nmsCpu numerics.
//
// Replaces op::nmsGpu (src/openpose/net/nmsBase.cu:251-351: register kernel + thrust scan over all
// channels + write kernel) computing what op::nmsCpu computes (src/openpose/net/nmsBase.cpp:7-170):
//   * interior pixels (1 < x < w-2, 1 < y < h-2): v > th and v > all 8 neighbours;
//   * pixels on row/column 1 or w-2 / h-2 (outer-border pixels of those rows/columns included):
//     v > th and v >= all 8 neighbours, neighbours outside the map read as th;
//   * any other pixel: never a peak;
//   * peaks kept in raster order, the first maxPeaks-1 only; position refined by the 7x7
//     score-weighted centroid in float (dy outer, dx inner), + offset; score = v.
//
// Two launches:
//   1. detect: every pixel of every (part, frame) plane in parallel, 4 per lane (HBM-bound pass);
//      a peak appends its raster index to its plane's candidate list (one atomic per peak --
//      peaks are rare) -- no int peak map and no global scan (the reference's 6 M-int thrust
//      scan, nmsBase.cu:327-329);
//   2. finalize: one workgroup per plane sorts its candidates (bitonic, LDS), keeps the first
//      maxPeaks-1 in raster order, refines them, and resets the plane's counter for the next
//      call.  A plane with more than kNmsCandidates peaks (noise, not poses) is re-scanned in
//      raster order by its workgroup, so the result never depends on the candidate capacity.
// -ffp-contract=off keeps the centroid sums bit-identical to the CPU.
#include <cstdlib>
#include <type_traits>
#include "kernels.h"
#include "heat_dev.h"
#include "../common.h"

namespace opk {

namespace {

typedef float float2_t __attribute__((ext_vector_type(2)));

constexpr int DT = 256;   // detect lanes per block
constexpr int FT = 256;   // finalize lanes per block
constexpr int CAP = kNmsCandidates;

// peak rules of nmsCpu for pixel (x, y) of value v; GET_(x, y) reads an in-map neighbour.
// cuda: nmsRegisterKernel's (nmsBase.cu:50-90) -- interior pixels only (0 < x < w-1, 0 < y < h-1),
// v > th and v > all 8 neighbours
#define OPK_PEAK_RULES(GET_)                                                                  \
    do {                                                                                      \
        if (!(v > th)) return false;                                                          \
        if (cuda) {                                                                           \
            if (!(x > 0 && x < w - 1 && y > 0 && y < h - 1)) return false;                    \
            return v > GET_(x - 1, y - 1) && v > GET_(x, y - 1) && v > GET_(x + 1, y - 1) &&  \
                   v > GET_(x - 1, y) && v > GET_(x + 1, y) && v > GET_(x - 1, y + 1) &&      \
                   v > GET_(x, y + 1) && v > GET_(x + 1, y + 1);                              \
        }                                                                                     \
        if (x > 1 && x < w - 2 && y > 1 && y < h - 2) {                                       \
            return v > GET_(x - 1, y - 1) && v > GET_(x, y - 1) && v > GET_(x + 1, y - 1) &&  \
                   v > GET_(x - 1, y) && v > GET_(x + 1, y) && v > GET_(x - 1, y + 1) &&      \
                   v > GET_(x, y + 1) && v > GET_(x + 1, y + 1);                              \
        }                                                                                     \
        if (x == 1 || x == w - 2 || y == 1 || y == h - 2) {                                   \
            bool ok = true;                                                                   \
            _Pragma("unroll") for (int dy = -1; dy <= 1; ++dy)                                \
            _Pragma("unroll") for (int dx = -1; dx <= 1; ++dx) {                              \
                if (dx == 0 && dy == 0) continue;                                             \
                const int xx = x + dx, yy = y + dy;                                           \
                const float nb = (xx >= 0 && xx < w && yy >= 0 && yy < h) ? GET_(xx, yy) : th; \
                ok = ok && (v >= nb);                                                         \
            }                                                                                 \
            return ok;                                                                        \
        }                                                                                     \
        return false;                                                                         \
    } while (0)

template <typename Get>
__device__ __forceinline__ bool peak_at(Get get, int w, int h, float th, int x, int y, float v,
                                        bool cuda = false)
{
    OPK_PEAK_RULES(get);
}

// the same rules on the lazily evaluated heat map itself.  Not a lambda over M: a closure holding
// a reference to the by-value kernel argument made the compiler copy the whole HeatMap to scratch
// at every nms_finalize_kernel start (496 B per lane, 203 MB of writes per 64-frame launch)
__device__ __forceinline__ bool peak_at_heat(const HeatMap& M, int pln, int w, int h, float th, int x,
                                             int y, float v, bool cuda)
{
#define OPK_HEAT_GET(xx_, yy_) heat_at(M, pln, xx_, yy_)
    OPK_PEAK_RULES(OPK_HEAT_GET);
#undef OPK_HEAT_GET
}

__device__ __forceinline__ void push_candidate(int* plane, int idx)
{
    const int slot = atomicAdd(plane, 1);
    if (slot < CAP) plane[1 + slot] = idx;
}

// scratch per plane: [0] candidate count, [1 .. CAP] raster indices
__global__ __launch_bounds__(DT) void nms_detect_kernel(int* __restrict__ scratch,
                                                        const float* __restrict__ heat,
                                                        int channels, int parts, int h, int w,
                                                        float th, int cuda)
{
    const int c = blockIdx.y, b = blockIdx.z;
    const float* s = heat + ((size_t)b * channels + c) * h * w;
    const int quads = (w + 3) >> 2;
    const int item = blockIdx.x * DT + threadIdx.x;
    if (item >= h * quads) return;
    const int y = item / quads;
    const int x0 = (item - y * quads) << 2;
    const float* row = s + (size_t)y * w;
    int* plane = scratch + ((size_t)b * parts + c) * (CAP + 1);
    auto get = [s, w](int xx, int yy) { return s[(size_t)yy * w + xx]; };
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int x = x0 + k;
        if (x < w && peak_at(get, w, h, th, x, y, row[x], cuda != 0)) push_candidate(plane, y * w + x);
    }
}

// Lazy heat map: a workgroup of LT lanes (one wave) owns LT consecutive columns (x0-1 .. x0+LT-2) of a
// (LOY+2)-row window of the resized plane (tile + 1-pixel halo; pixels outside the map = th).
// Each lane runs resize.hip's two passes down its own column -- horizontal pass of the window's
// source rows into its LDS column, vertical combinations with the row's (block-uniform, scalar)
// coefficients -- then the LT-2 x LOY tile pixels are tested from LDS.  The full-resolution stack
// is never written.
constexpr int LMAXR = 16;         // source rows per window kept in LDS (x8 upsampling of a
                                  // 34-row window needs 9)

// LOY = tile rows (window rows LOY + 2).  Measured per 64-frame launch (round 1): 16 rows 638 us,
// 32 rows 774 us, 48 rows 938 us (more, shorter workgroups win); 16 is the one compiled
template <int LOY, int LT>
__global__ __launch_bounds__(LT) void nms_detect_lazy_kernel(int* __restrict__ scratch,
                                                             const HeatMap M, int parts, float th)
{
    constexpr int LOX = LT - 2;       // tile columns
    constexpr int LWR = LOY + 2;      // window rows
    // hb (horizontal-pass rows) and win (window values) share LDS: a lane only ever touches its
    // own column of either before the barrier, and win is written after the last hb read
    constexpr int HBR = LWR < LMAXR ? LWR : LMAXR;   // horizontal-pass rows that fit in win
    __shared__ float win[LWR * LT];
    float* hb = win;
    const int tid = threadIdx.x;
    const int c = blockIdx.z % parts, b = blockIdx.z / parts;
    const int plane = b * M.channels + c;
    const int H = M.h, W = M.w;
    const int xw0 = blockIdx.x * LOX - 1;          // window column of lane 0
    const int x = xw0 + tid;
    const int y0 = blockIdx.y * LOY - 1;           // window row 0
    const bool xin = x >= 0 && x < W;
    const bool simd_col = cubic_simd_column(x, W);   // OpenCV's vertical SIMD body (heat_dev.h)
    const int ry_lo = max(y0, 0), ry_hi = min(y0 + LWR - 1, H - 1);
    __shared__ float4 rcoef[LWR];          // vertical coefficients of the window rows
    __shared__ int4 rofs[LWR];             // their 4 source rows as offsets into hb
    float acc[LWR];
#pragma unroll
    for (int rr = 0; rr < LWR; ++rr) acc[rr] = 0.f;
    if (M.cuda) {   // CUDA-build resize arithmetic: pixel by pixel (no shared passes)
#pragma unroll
        for (int rr = 0; rr < LWR; ++rr) {
            const int y = y0 + rr;
            win[rr * LT + tid] = (y >= 0 && y < H && xin) ? heat_at_cuda(M, plane, x, y) : th;
        }
    }
    for (int n = 0; n < (M.cuda ? 0 : M.nsrc); ++n) {
        const ResizeSource& S = M.src[n];
        const float* src = S.src + (size_t)plane * S.sh * S.sw;
        const int r_lo = heat_clampi(S.yofs[ry_lo] - 1, 0, S.sh - 1);
        const int r_hi = heat_clampi(S.yofs[ry_hi] + 2, 0, S.sh - 1);
        const int nrows = r_hi - r_lo + 1;
        const bool tiled = nrows <= HBR;     // block-uniform
        if (n > 0) __syncthreads();          // previous source's row tables fully read
        if (tid < LWR) {
            const int y = heat_clampi(y0 + tid, 0, H - 1);
            rcoef[tid] = *reinterpret_cast<const float4*>(S.ycoef + 4 * y);
            const int yb = S.yofs[y] - 1;
            int4 o;
            o.x = heat_clampi(yb, 0, S.sh - 1);
            o.y = heat_clampi(yb + 1, 0, S.sh - 1);
            o.z = heat_clampi(yb + 2, 0, S.sh - 1);
            o.w = heat_clampi(yb + 3, 0, S.sh - 1);
            if (tiled) {
                o.x = (o.x - r_lo) * LT;
                o.y = (o.y - r_lo) * LT;
                o.z = (o.z - r_lo) * LT;
                o.w = (o.w - r_lo) * LT;
            }
            rofs[tid] = o;
        }
        int xo = 0;
        float a[4] = {0.f, 0.f, 0.f, 0.f};
        if (xin) {
            xo = S.xofs[x];
            const float4 cf = *reinterpret_cast<const float4*>(S.xcoef + 4 * x);
            a[0] = cf.x; a[1] = cf.y; a[2] = cf.z; a[3] = cf.w;
        }
        if (tiled && xin)
            for (int r = 0; r < nrows; ++r)
                hb[r * LT + tid] = cubic_hpass(src + (size_t)(r_lo + r) * S.sw, S.sw, xo, a);
        __syncthreads();                     // row tables visible (hb columns are lane-private)
#pragma unroll
        for (int rr = 0; rr < LWR; ++rr) {
            const int y = y0 + rr;
            float v = 0.f;
            if (y >= 0 && y < H && xin) {
                const float4 bq = rcoef[rr];
                const int4 o = rofs[rr];
                float hv[4];
                if (tiled) {
                    hv[0] = hb[o.x + tid];
                    hv[1] = hb[o.y + tid];
                    hv[2] = hb[o.z + tid];
                    hv[3] = hb[o.w + tid];
                } else {
                    hv[0] = cubic_hpass(src + (size_t)o.x * S.sw, S.sw, xo, a);
                    hv[1] = cubic_hpass(src + (size_t)o.y * S.sw, S.sw, xo, a);
                    hv[2] = cubic_hpass(src + (size_t)o.z * S.sw, S.sw, xo, a);
                    hv[3] = cubic_hpass(src + (size_t)o.w * S.sw, S.sw, xo, a);
                }
                v = cubic_vpass(hv, bq.x, bq.y, bq.z, bq.w, simd_col);
            }
            acc[rr] = (n == 0) ? v : v + acc[rr];
        }
    }
    if (!M.cuda) {
#pragma unroll
        for (int rr = 0; rr < LWR; ++rr) {
            const int y = y0 + rr;
            win[rr * LT + tid] = (y >= 0 && y < H && xin) ? (M.nsrc > 1 ? acc[rr] * M.inv_n : acc[rr]) : th;
        }
    }
    __syncthreads();
    if (tid == 0 || tid == LT - 1 || !xin) return;
    int* pl = scratch + ((size_t)b * parts + c) * (CAP + 1);
    auto get = [xw0, y0](int xx, int yy) { return win[(yy - y0) * LT + (xx - xw0)]; };
    for (int ty = 0; ty < LOY; ++ty) {
        const int y = y0 + 1 + ty;
        if (y >= H) break;
        if (peak_at(get, W, H, th, x, y, win[(ty + 1) * LT + tid], M.cuda != 0)) push_candidate(pl, y * W + x);
    }
}

__device__ __forceinline__ void refine_write(float* __restrict__ out, const HeatMap& M, int plane, int idx,
                             int rank, float offx, float offy)
{
    const int w = M.w, h = M.h;
    const int py = idx / w, px = idx - py * w;
    float xa = 0.f, ya = 0.f, sa = 0.f;
    for (int dy = -3; dy <= 3; ++dy) {
        const int yy = py + dy;
        if (yy < 0 || yy >= h) continue;
        for (int dx = -3; dx <= 3; ++dx) {
            const int xx = px + dx;
            if (xx < 0 || xx >= w) continue;
            const float sc = heat_at(M, plane, xx, yy);
            if (sc > 0) {
                if (M.cuda) {   // nvcc contracts xAcc += x*score (default --fmad=true)
                    xa = fmaf((float)xx, sc, xa);
                    ya = fmaf((float)yy, sc, ya);
                } else {
                    xa += (float)xx * sc;
                    ya += (float)yy * sc;
                }
                sa += sc;
            }
        }
    }
    float* o = out + (size_t)(rank + 1) * 3;
    o[0] = xa / sa + offx;
    o[1] = ya / sa + offy;
    o[2] = heat_at(M, plane, px, py);
}

// refine_write for the peaks key[0 .. found) with the 7x7 windows' heat values evaluated by the whole
// workgroup first (one lazy evaluation per lane instead of 49 in a row per peak-owning lane), then
// summed by the peak's lane in refine_write's order with its arithmetic: bit-identical to it
constexpr int RP = 64;   // peaks per round
__device__ __forceinline__ void refine_peaks(float* __restrict__ out, const HeatMap& M, int plane,
                                             const int* key, int found, float offx, float offy,
                                             float* win)
{
    const int w = M.w, h = M.h, tid = threadIdx.x;
    for (int r0 = 0; r0 < found; r0 += RP) {
        const int np = min(RP, found - r0);
        __syncthreads();   // the previous round's windows are summed
        for (int i = tid; i < np * 49; i += FT) {
            const int p = i / 49, k = i - (i / 49) * 49;
            const int idx = key[r0 + p];
            const int py = idx / w, px = idx - py * w;
            const int yy = py + k / 7 - 3, xx = px + k % 7 - 3;
            win[i] = (yy >= 0 && yy < h && xx >= 0 && xx < w) ? heat_at(M, plane, xx, yy) : 0.f;
        }
        __syncthreads();
        if (tid < np) {
            const int idx = key[r0 + tid];
            const int py = idx / w, px = idx - py * w;
            const float* v = win + tid * 49;
            float xa = 0.f, ya = 0.f, sa = 0.f;
            for (int dy = -3; dy <= 3; ++dy) {
                const int yy = py + dy;
                if (yy < 0 || yy >= h) continue;
                for (int dx = -3; dx <= 3; ++dx) {
                    const int xx = px + dx;
                    if (xx < 0 || xx >= w) continue;
                    const float sc = v[(dy + 3) * 7 + dx + 3];
                    if (sc > 0) {
                        if (M.cuda) {
                            xa = fmaf((float)xx, sc, xa);
                            ya = fmaf((float)yy, sc, ya);
                        } else {
                            xa += (float)xx * sc;
                            ya += (float)yy * sc;
                        }
                        sa += sc;
                    }
                }
            }
            float* o = out + (size_t)(r0 + tid + 1) * 3;
            o[0] = xa / sa + offx;
            o[1] = ya / sa + offy;
            o[2] = v[24];   // heat_at(px, py)
        }
    }
}

#ifndef OPK_NMS_PAR_REFINE   // dev A/B: 0 = one peak per lane, refine_write
#define OPK_NMS_PAR_REFINE 1
#endif

__global__ __launch_bounds__(FT) void nms_finalize_kernel(float* __restrict__ peaks,
                                                          int* __restrict__ scratch,
                                                          const HeatMap M, int parts,
                                                          int max_peaks1, float th, float offx,
                                                          float offy)
{
    __shared__ int key[CAP];
    __shared__ int wave_tot[FT / 64];
    __shared__ float win[OPK_NMS_PAR_REFINE ? RP * 49 : 1];
    const int c = blockIdx.x, b = blockIdx.y;
    const int pln = b * M.channels + c;
    const int h = M.h, w = M.w;
    float* out = peaks + ((size_t)b * parts + c) * max_peaks1 * 3;
    int* plane = scratch + ((size_t)b * parts + c) * (CAP + 1);
    const int tid = threadIdx.x;
    const int cap = max_peaks1 - 1;
    const int n = plane[0];
    int found;
    if (n <= CAP) {
        for (int i = tid; i < CAP; i += FT) key[i] = i < n ? plane[1 + i] : 0x7fffffff;
        __syncthreads();
        int len = 1;   // smallest power of two >= n (>= 2)
        while (len < n) len <<= 1;
        if (len < 2) len = 2;
        for (int k = 2; k <= len; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = tid; i < len; i += FT) {
                    const int p = i ^ j;
                    if (p > i) {
                        const int a = key[i], bb = key[p];
                        const bool up = (i & k) == 0;
                        if ((a > bb) == up) {
                            key[i] = bb;
                            key[p] = a;
                        }
                    }
                }
                __syncthreads();
            }
        found = n < cap ? n : cap;
        if (OPK_NMS_PAR_REFINE) refine_peaks(out, M, pln, key, found, offx, offy, win);
        else
            for (int r = tid; r < found; r += FT) refine_write(out, M, pln, key[r], r, offx, offy);
    } else {
        // overflow: ordered raster scan of the plane by this workgroup
        const int lane = tid & 63, wave = tid >> 6;
        const int quads = (w + 3) >> 2;
        const int items = h * quads;
        int count = 0;   // block-uniform
        for (int base = 0; base < items && count < cap; base += FT) {
            const int item = base + tid;
            unsigned mask = 0;
            int y = 0, x0 = 0;
            if (item < items) {
                y = item / quads;
                x0 = (item - y * quads) << 2;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int x = x0 + k;
                    if (x < w && peak_at_heat(M, pln, w, h, th, x, y, heat_at(M, pln, x, y), M.cuda != 0))
                        mask |= 1u << k;
                }
            }
            const int cnt = __popc(mask);
            if (!__syncthreads_or(cnt)) continue;
            int incl = cnt;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int t = __shfl_up(incl, off, 64);
                if (lane >= off) incl += t;
            }
            if (lane == 63) wave_tot[wave] = incl;
            __syncthreads();
            int before = 0, total = 0;
            for (int i = 0; i < FT / 64; ++i) {
                const int t = wave_tot[i];
                before += (i < wave) ? t : 0;
                total += t;
            }
            int rank = count + before + incl - cnt;
            for (int k = 0; k < 4; ++k) {
                if (!(mask & (1u << k))) continue;
                if (rank < cap) refine_write(out, M, pln, y * w + x0 + k, rank, offx, offy);
                ++rank;
            }
            count += total;
            __syncthreads();
        }
        found = count < cap ? count : cap;
    }
    // slot 0 = {count, 0, 0}; unused slots zeroed (the reference leaves them stale)
    for (int i = tid; i < (max_peaks1 - 1 - found) * 3; i += FT) out[found * 3 + 3 + i] = 0.f;
    __syncthreads();
    if (tid == 0) {
        out[0] = (float)found;
        out[1] = 0.f;
        out[2] = 0.f;
        plane[0] = 0;   // ready for the next call
    }
}

// Lazy map of NS sources (1..4), CPU semantics (the pose pipeline's maps): one wave owns LT
// columns (x0-1 .. x0+LT-2, LT-2 tested) of RC consecutive map rows and walks down them once.
// Per source, the horizontal passes are kept as a rolling register window h0..h3 (source rows
// yofs[y]-1 .. yofs[y]+2, clamped) that advances one source row at a time, with the next source
// row's four taps loaded one advance ahead; each map row is one vertical combination per source
// (summed in source order, then * 1/NS as resize_merge does), written into a 4-row LDS ring, and
// the row above it is tested once the ring holds its lower neighbours.  Against the windowed
// kernel above, every source row's horizontal pass is computed once per column instead of once
// per 16-row window it touches (2.5x at x8), and the row tables are read from LDS.  Same
// hpass/vpass arithmetic and peak rules, so the candidate set is identical (the finalize kernel
// orders it).
//
// FL (variant flags, dev switch NMS_WALK):
//   bit 0 (parallel test): the row above is tested with all of its side neighbours' ring reads in
//     flight at once (6 ds_reads, one wait; the lane's own column above / below from registers)
//     and only when some lane of the wave holds a candidate (v > th on a testable pixel); without
//     it the test is nmsCpu's short-circuit chain (peak_at): one LDS round trip per neighbour;
//   bit 1 (with bit 0): no wait after the ring write -- one wave's LDS operations execute in
//     order, so a compiler barrier replaces the workgroup barrier;
//   bit 2 (staged sources): the walk's source footprint (the rows and columns its taps reach, e.g.
//     13 x 12 floats of a 46 x 82 source at x8) is copied to LDS once, and every advance reads
//     its four taps from there instead of from L2 / HBM (sources whose footprint exceeds kNmsFP
//     floats keep the global reads).
// Same rules and values in every variant, so the same candidates.
constexpr int kNmsFP = 256;
template <int LT, int RC, int NS, int FL>
__global__ __launch_bounds__(LT) void nms_detect_stream_kernel(int* __restrict__ scratch,
                                                               const HeatMap M, int parts, float th)
{
    constexpr bool PT = (FL & 1) != 0, NOWAIT = (FL & 3) == 3, ST = (FL & 4) != 0;
    static_assert(RC + 2 <= LT, "one lane per window row loads the row tables");
    __shared__ float ring[4 * LT];
    __shared__ float4 rcoef[NS][RC + 2];
    __shared__ int rsrc[NS][RC + 2];
    const int tid = threadIdx.x;
    const int c = blockIdx.z % parts, b = blockIdx.z / parts;
    const int plane = b * M.channels + c;
    const int H = M.h, W = M.w;
    const int xw0 = blockIdx.x * (LT - 2) - 1;          // map column of lane 0
    const int x = xw0 + tid;
    const bool xin = x >= 0 && x < W;
    const bool simd_col = cubic_simd_column(x, W);
    const float inv_n = M.inv_n;
    const int ys = blockIdx.y * RC, ye = min(ys + RC, H);   // tested rows [ys, ye)
    const int wy0 = ys - 1;                                  // window row of table entry 0
    // per source: locals only in the closures (one referring to the by-value kernel argument
    // makes the compiler copy the HeatMap to scratch, see peak_at_heat)
    const float* src[NS];
    int ssh[NS], ssw[NS], t[NS][4];
    float a[NS][4];
#pragma unroll
    for (int n = 0; n < NS; ++n) {
        const ResizeSource& S = M.src[n];
        if (tid < RC + 2) {
            const int y = heat_clampi(wy0 + tid, 0, H - 1);
            rcoef[n][tid] = *reinterpret_cast<const float4*>(S.ycoef + 4 * y);
            rsrc[n][tid] = S.yofs[y];
        }
        src[n] = S.src + (size_t)plane * S.sh * S.sw;
        ssh[n] = S.sh;
        ssw[n] = S.sw;
        int xo = 0;
        a[n][0] = a[n][1] = a[n][2] = a[n][3] = 0.f;
        if (xin) {
            xo = S.xofs[x];
            const float4 cf = *reinterpret_cast<const float4*>(S.xcoef + 4 * x);
            a[n][0] = cf.x; a[n][1] = cf.y; a[n][2] = cf.z; a[n][3] = cf.w;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) t[n][k] = heat_clampi(xo - 1 + k, 0, ssw[n] - 1);
    }
    __shared__ float fp[ST ? NS : 1][ST ? kNmsFP : 1];
    int fr0[NS], fc0[NS], fcn[NS];
    bool stg[NS];
    auto taps = [&](int n, int r, float v[4]) {   // source row r's taps
        if (ST && stg[n]) {
            const float* row = fp[n] + (heat_clampi(r, 0, ssh[n] - 1) - fr0[n]) * fcn[n] - fc0[n];
            v[0] = row[t[n][0]]; v[1] = row[t[n][1]]; v[2] = row[t[n][2]]; v[3] = row[t[n][3]];
            return;
        }
        const float* row = src[n] + (size_t)heat_clampi(r, 0, ssh[n] - 1) * ssw[n];
        v[0] = row[t[n][0]]; v[1] = row[t[n][1]]; v[2] = row[t[n][2]]; v[3] = row[t[n][3]];
    };
    // cubic_hpass's sum, in its order
    auto hsum = [&a](int n, const float v[4]) {
        return v[0] * a[n][0] + v[1] * a[n][1] + v[2] * a[n][2] + v[3] * a[n][3];
    };
    __syncthreads();                                         // row tables
    int cur[NS];
    float h[NS][4], nv[NS][4];
#pragma unroll
    for (int n = 0; n < NS; ++n) {
        cur[n] = rsrc[n][wy0 < 0 ? 1 : 0];                   // source row of the first map row
        stg[n] = false;
        if constexpr (ST) {
            // rows cur-1 .. (last map row's source row)+3 (the prefetch), columns of the first and
            // last in-map lanes' outer taps (xofs is non-decreasing), all clamped as the taps are
            const int r0 = heat_clampi(cur[n] - 1, 0, ssh[n] - 1);
            const int r1 = heat_clampi(rsrc[n][min(ye, H - 1) - wy0] + 3, 0, ssh[n] - 1);
            const int c0 = __shfl(t[n][0], max(xw0, 0) - xw0, LT);
            const int c1 = __shfl(t[n][3], min(xw0 + LT - 1, W - 1) - xw0, LT);
            fr0[n] = r0;
            fc0[n] = c0;
            fcn[n] = c1 - c0 + 1;
            const int cnt = (r1 - r0 + 1) * fcn[n];
            stg[n] = cnt <= kNmsFP;
            if (stg[n])
                for (int i = tid; i < cnt; i += LT) {
                    const int rr = i / fcn[n];
                    fp[n][i] = src[n][(size_t)(r0 + rr) * ssw[n] + c0 + (i - rr * fcn[n])];
                }
        }
    }
    if constexpr (ST) __syncthreads();                       // staged footprints
#pragma unroll
    for (int n = 0; n < NS; ++n) {
#pragma unroll
        for (int k = 0; k < 4; ++k) h[n][k] = nv[n][k] = 0.f;
        if (xin) {
            float v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                taps(n, cur[n] - 1 + k, v);
                h[n][k] = hsum(n, v);
            }
            taps(n, cur[n] + 3, nv[n]);                      // next advance's row, in flight
        }
    }
    int* pl = scratch + ((size_t)b * parts + c) * (CAP + 1);
    float vprev = th, vprev2 = th;
    // PT: side-neighbour lanes (clamped at the window's first / last lane, whose tests never run)
    const int tl = tid > 0 ? tid - 1 : 0, tr = tid < LT - 1 ? tid + 1 : LT - 1;
    const bool xtest = tid > 0 && tid < LT - 1 && xin;
    const bool xinner = x > 1 && x < W - 2, xedge = x == 1 || x == W - 2;
    for (int y = wy0; y <= ye; ++y) {
        float v = th;
        if (y >= 0 && y < H) {
            float acc = 0.f;
#pragma unroll
            for (int n = 0; n < NS; ++n) {
                const int tr = rsrc[n][y - wy0];
                while (cur[n] < tr) {                        // block-uniform
                    h[n][0] = h[n][1]; h[n][1] = h[n][2]; h[n][2] = h[n][3];
                    ++cur[n];
                    if (xin) {
                        h[n][3] = hsum(n, nv[n]);
                        taps(n, cur[n] + 3, nv[n]);
                    }
                }
                const float4 bq = rcoef[n][y - wy0];
                const float vn = cubic_vpass(h[n], bq.x, bq.y, bq.z, bq.w, simd_col);
                acc = (n == 0) ? vn : vn + acc;
            }
            if (xin) v = NS > 1 ? acc * inv_n : acc;
        }
        ring[(y & 3) * LT + tid] = v;                        // y >= -1: (y & 3) is y mod 4
        const int ty = y - 1;                                // row tested now
        if constexpr (PT) {
            // nmsCpu's rules (OPK_PEAK_RULES): interior pixels strictly above all 8 neighbours;
            // pixels on row / column 1 or h-2 / w-2 at least equal, neighbours outside the map = th
            // (the ring holds th there); any other pixel never
            const bool inner = xinner && ty > 1 && ty < H - 2;
            const bool cand = ty >= ys && xtest && vprev > th &&
                              (inner || xedge || ty == 1 || ty == H - 2);
            if constexpr (NOWAIT)
                asm volatile("" ::: "memory");   // the ring reads stay after the write (one wave:
                                                 // its LDS operations execute in order)
            else
                __syncthreads();
            if (__ballot(cand) != 0) {                                // wave-uniform
                const float* r0 = ring + ((ty - 1) & 3) * LT;
                const float* r1 = ring + (ty & 3) * LT;
                const float* r2 = ring + (y & 3) * LT;
                const float n0 = r0[tl], n1 = r0[tr], n2 = r1[tl], n3 = r1[tr], n4 = r2[tl], n5 = r2[tr];
                const float p = vprev;
                const bool gt = (p > n0) & (p > n1) & (p > n2) & (p > n3) & (p > n4) & (p > n5) &
                                (p > vprev2) & (p > v);
                const bool ge = (p >= n0) & (p >= n1) & (p >= n2) & (p >= n3) & (p >= n4) &
                                (p >= n5) & (p >= vprev2) & (p >= v);
                if (cand && (inner ? gt : ge)) push_candidate(pl, ty * W + x);
            }
            if constexpr (NOWAIT) asm volatile("" ::: "memory");   // next write after these reads
        } else {
            __syncthreads();                                 // rows y-2 .. y visible
            if (ty >= ys && tid > 0 && tid < LT - 1 && xin) {
                auto get = [xw0](int xx, int yy) { return ring[(yy & 3) * LT + (xx - xw0)]; };
                if (peak_at(get, W, H, th, x, ty, vprev, false)) push_candidate(pl, ty * W + x);
            }
        }
        vprev2 = vprev;
        vprev = v;
        // the ring slot written next ((y+1) & 3) was last read when row y-4 was tested
    }
}


// Two columns per lane, no LDS ring (NMS_WALK 8 / the default below): one wave owns the 128 map
// columns xw0 .. xw0 + 127 (126 tested) of RC rows and walks down them.  A lane keeps its two
// columns' horizontal passes as float2 registers, so every pass, vertical combination and merge
// is one packed v_pk_mul_f32 / v_pk_add_f32 per two pixels with resize.hip's operations in its
// order (-ffp-contract=off: the same bits).  The three rows a test needs (row above, the tested
// row, row below) stay in registers; the two side columns of the neighbouring lanes come by
// wave-wide DPP shifts, and only on rows where some lane holds a candidate (v > th on a testable
// pixel).  Measured on the ring walk: its cost is the instruction stream, not LDS latency (a test
// with all its reads in flight but more instructions ran 30 % slower: profiles/round4/nms_walk/),
// so this walk spends ~10 instructions per pixel row on the common path instead of ~30.
// A pixel passes the nmsCpu rules as peak_at: interior pixels strictly above, row / column 1 or
// h-2 / w-2 pixels at least equal to, all 8 neighbours (th outside the map); the neighbours are
// compared through their maximum, which is the same test for NaN-free maps.
__device__ __forceinline__ float dpp_from_left(float v)    // lane i gets lane i-1's value
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float dpp_from_right(float v)   // lane i gets lane i+1's value
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xF, 0xF, false));
}

template <int RC, int NS>
__global__ __launch_bounds__(64) void nms_detect_walk2_kernel(int* __restrict__ scratch,
                                                              const HeatMap M, int parts, float th)
{
    constexpr int LT = 64, CW = 2 * LT - 2;
    static_assert(RC + 2 <= LT, "one lane per window row holds the row tables");
    const int tid = threadIdx.x;
    const int c = blockIdx.z % parts, b = blockIdx.z / parts;
    const int plane = b * M.channels + c;
    const int H = M.h, W = M.w;
    const int xw0 = blockIdx.x * CW - 1;                     // map column of lane 0's first column
    const int xa = xw0 + 2 * tid, xb = xa + 1;
    const bool ina = xa >= 0 && xa < W, inb = xb >= 0 && xb < W;
    // OpenCV's SIMD body covers every in-map column of this wave: the one vertical order for both
    const bool wave_simd = min(xw0 + 2 * LT - 1, W - 1) < W - W % kCvVResizeLanes;
    const bool sa = cubic_simd_column(xa, W), sb = cubic_simd_column(xb, W);
    const float inv_n = M.inv_n;
    const int ys = blockIdx.y * RC, ye = min(ys + RC, H);
    const int wy0 = ys - 1;
    // row tables of the window's rows wy0 .. wy0 + RC + 1, one row per lane (read by v_readlane,
    // no LDS round trip per row)
    int lrsrc[NS];
    float lrc[NS][4];
    const float* src[NS];
    int ssh[NS], ssw[NS], ta[NS][4], tb[NS][4];
    float2_t A[NS][4];
#pragma unroll
    for (int n = 0; n < NS; ++n) {
        const ResizeSource& S = M.src[n];
        {
            const int y = heat_clampi(wy0 + tid, 0, H - 1);
            const float4 cq = *reinterpret_cast<const float4*>(S.ycoef + 4 * y);
            lrc[n][0] = cq.x; lrc[n][1] = cq.y; lrc[n][2] = cq.z; lrc[n][3] = cq.w;
            lrsrc[n] = S.yofs[y];
        }
        src[n] = S.src + (size_t)plane * S.sh * S.sw;
        ssh[n] = S.sh;
        ssw[n] = S.sw;
        int xo_a = 0, xo_b = 0;
        float4 ca = make_float4(0.f, 0.f, 0.f, 0.f), cb = ca;
        if (ina) {
            xo_a = S.xofs[xa];
            ca = *reinterpret_cast<const float4*>(S.xcoef + 4 * xa);
        }
        if (inb) {
            xo_b = S.xofs[xb];
            cb = *reinterpret_cast<const float4*>(S.xcoef + 4 * xb);
        }
        A[n][0] = float2_t{ca.x, cb.x};
        A[n][1] = float2_t{ca.y, cb.y};
        A[n][2] = float2_t{ca.z, cb.z};
        A[n][3] = float2_t{ca.w, cb.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ta[n][k] = heat_clampi(xo_a - 1 + k, 0, ssw[n] - 1);
            tb[n][k] = heat_clampi(xo_b - 1 + k, 0, ssw[n] - 1);
        }
    }
    auto taps = [&](int n, int r, float2_t v[4]) {   // source row r's taps of both columns
        const float* row = src[n] + (size_t)heat_clampi(r, 0, ssh[n] - 1) * ssw[n];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = float2_t{row[ta[n][k]], row[tb[n][k]]};
    };
    auto hsum = [&A](int n, const float2_t v[4]) {   // cubic_hpass's sum, in its order
        return v[0] * A[n][0] + v[1] * A[n][1] + v[2] * A[n][2] + v[3] * A[n][3];
    };
    auto rdl_i = [](int v, int l) { return __builtin_amdgcn_readlane(v, l); };
    auto rdl_f = [](float v, int l) {
        return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
    };
    int cur[NS];
    float2_t h[NS][4], nv[NS][4];
#pragma unroll
    for (int n = 0; n < NS; ++n) {
        cur[n] = rdl_i(lrsrc[n], wy0 < 0 ? 1 : 0);
        float2_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            taps(n, cur[n] - 1 + k, v);
            h[n][k] = hsum(n, v);
        }
        taps(n, cur[n] + 3, nv[n]);                          // next advance's row, in flight
    }
    int* pl = scratch + ((size_t)b * parts + c) * (CAP + 1);
    const float2_t thv = float2_t{th, th};
    // which lanes test a column, by the row's kind in nmsCpu's rules (testable: not the window's
    // halo columns, inside the map): an inner row tests inner and edge columns, an edge row (1,
    // h-2) every in-map column, an outer row (0, h-1) the edge columns only -- as wave masks.
    // Out-of-map COLUMNS need no value: no tested pixel has one as a neighbour (x = 0 and w-1 are
    // never tested); out-of-map ROWS hold th (the border rule's outside value).
    const bool ta_ok = tid > 0 && ina, tb_ok = tid < LT - 1 && inb;
    const bool a_inner = xa > 1 && xa < W - 2, b_inner = xb > 1 && xb < W - 2;
    const bool a_edge = xa == 1 || xa == W - 2, b_edge = xb == 1 || xb == W - 2;
    const uint64_t Ma_in = __ballot(ta_ok && (a_inner || a_edge)), Mb_in = __ballot(tb_ok && (b_inner || b_edge));
    const uint64_t Ma_ok = __ballot(ta_ok), Mb_ok = __ballot(tb_ok);
    const uint64_t Ma_out = __ballot(ta_ok && a_edge), Mb_out = __ballot(tb_ok && b_edge);
    // The walk with the vertical order fixed (WS: SIMD order for every column of the wave) and no
    // per-row range checks: rows wy0 (above the first tested row) and ys are computed before the
    // loop, the loop covers y = ys + 1 .. ye - 1 (inside the map), row ye after it -- most of a
    // row's scalar work is gone (the SALU, one per CU cycle, had set the pace).
    auto walk = [&](auto ws) {
        constexpr bool WS = decltype(ws)::value;
        auto row = [&](int y) {                              // merged value of map row y (in the map)
            float2_t acc;
#pragma unroll
            for (int n = 0; n < NS; ++n) {
                const int tr = rdl_i(lrsrc[n], y - wy0);
                while (cur[n] < tr) {                        // uniform
                    h[n][0] = h[n][1]; h[n][1] = h[n][2]; h[n][2] = h[n][3];
                    ++cur[n];
                    h[n][3] = hsum(n, nv[n]);
                    taps(n, cur[n] + 3, nv[n]);
                }
                const float b0 = rdl_f(lrc[n][0], y - wy0), b1 = rdl_f(lrc[n][1], y - wy0);
                const float b2 = rdl_f(lrc[n][2], y - wy0), b3 = rdl_f(lrc[n][3], y - wy0);
                float2_t vn;
                if constexpr (WS) {   // cubic_vpass, SIMD order
                    const float2_t t3 = h[n][3] * b3;
                    const float2_t t2 = h[n][2] * b2 + t3;
                    const float2_t t1 = h[n][1] * b1 + t2;
                    vn = h[n][0] * b0 + t1;
                } else {
                    const float ha[4] = {h[n][0].x, h[n][1].x, h[n][2].x, h[n][3].x};
                    const float hb[4] = {h[n][0].y, h[n][1].y, h[n][2].y, h[n][3].y};
                    vn = float2_t{cubic_vpass(ha, b0, b1, b2, b3, sa), cubic_vpass(hb, b0, b1, b2, b3, sb)};
                }
                acc = (n == 0) ? vn : vn + acc;
            }
            return NS > 1 ? acc * inv_n : acc;
        };
        // test row ty (values mid) with its neighbour rows up / dn
        auto test = [&](int ty, float2_t up, float2_t mid, float2_t dn) {
            uint64_t ma = Ma_in, mb = Mb_in;
            const bool row_inner = (unsigned)(ty - 2) < (unsigned)(H - 4);
            if (!row_inner) {                                // rows 0, 1, h-2, h-1 (uniform, rare)
                const bool row_edge = ty == 1 || ty == H - 2;
                ma = row_edge ? Ma_ok : Ma_out;
                mb = row_edge ? Mb_ok : Mb_out;
            }
            const uint64_t ca = ma & __ballot(mid.x > th), cb = mb & __ballot(mid.y > th);
            if ((ca | cb) == 0) return;                      // uniform
            // side neighbours from the adjacent lanes: left of column a, right of column b
            const float la0 = dpp_from_left(up.y), la1 = dpp_from_left(mid.y), la2 = dpp_from_left(dn.y);
            const float rb0 = dpp_from_right(up.x), rb1 = dpp_from_right(mid.x), rb2 = dpp_from_right(dn.x);
            const float na = fmaxf(fmaxf(fmaxf(la0, up.x), fmaxf(up.y, la1)),
                                   fmaxf(fmaxf(mid.y, la2), fmaxf(dn.x, dn.y)));
            const float nb = fmaxf(fmaxf(fmaxf(up.x, up.y), fmaxf(rb0, mid.x)),
                                   fmaxf(fmaxf(rb1, dn.x), fmaxf(dn.y, rb2)));
            const bool pa = ((ca >> tid) & 1) && ((a_inner && row_inner) ? mid.x > na : mid.x >= na);
            const bool pb = ((cb >> tid) & 1) && ((b_inner && row_inner) ? mid.y > nb : mid.y >= nb);
            if (pa) push_candidate(pl, ty * W + xa);
            if (pb) push_candidate(pl, ty * W + xb);
        };
        float2_t up = wy0 >= 0 ? row(wy0) : thv;             // row ys - 1
        float2_t mid = row(ys);                              // ys < ye <= H
        for (int y = ys + 1; y < ye; ++y) {
            const float2_t v = row(y);
            test(y - 1, up, mid, v);
            up = mid;
            mid = v;
        }
        test(ye - 1, up, mid, ye < H ? row(ye) : thv);
    };
    if (wave_simd) walk(std::true_type{});
    else walk(std::false_type{});
}

}  // namespace

size_t nms_scratch_ints(int frames, int parts) { return (size_t)frames * parts * (CAP + 1); }

void launch_nms(float* peaks, int* scratch, const HeatMap& heat_in, int frames, int parts,
                int max_peaks1, float threshold, float offx, float offy, hipStream_t stream,
                bool cuda)
{
    // the peak rules and centroid follow `cuda`; so does the resize arithmetic of a lazy map
    HeatMap heat = heat_in;
    heat.cuda = cuda ? 1 : 0;
    const int h = heat.h, w = heat.w;
    OPK_CHECK_ARG(frames > 0 && parts > 0 && parts <= heat.channels, "bad channel counts");
    OPK_CHECK_ARG(h > 0 && w > 0 && max_peaks1 >= 1, "bad sizes");
    OPK_CHECK_ARG(heat.heat != nullptr || (heat.nsrc >= 1 && heat.nsrc <= kMaxResizeSources),
                  "heat map: materialised or 1..8 lazy sources");
    OPK_CHECK_ARG(scratch != nullptr, "NMS scratch required (zeroed once, nms_scratch_ints)");
    OPK_CHECK_ARG((long)h * w < (1L << 31), "plane too large");
    if (heat.heat) {
        const int quads = (w + 3) >> 2;
        dim3 g1((h * quads + DT - 1) / DT, parts, frames);
        hipLaunchKernelGGL(nms_detect_kernel, g1, dim3(DT), 0, stream, scratch, heat.heat,
                           heat.channels, parts, h, w, threshold, heat.cuda);
    } else if (!cuda && heat.nsrc <= 4 && dev_switch("NMS_STREAM", 1) != 0) {   // 0: dev A/B
        // 62 x 62 walks, one wave (measured: 30-row walks, two-wave 126 / 46-row walks 4-10 %
        // slower; loading the taps two advances ahead instead of one: no change)
        constexpr int lt = 64, rc = 62;
        // (four walks per workgroup, each wave on its own ring with only lgkmcnt waits between
        // rows, measured 5-9 % slower on configs 2, 4 and 5: profiles/round3/nms_wpb/)
        const dim3 grid((w + lt - 3) / (lt - 2), (h + rc - 1) / rc, frames * parts);
        const dim3 grid2((w + 2 * lt - 3) / (2 * lt - 2), (h + rc - 1) / rc, frames * parts);
        // NMS_WALK (dev A/B): the walk's variant flags (nms_detect_stream_kernel FL)
        const int fl = dev_switch("NMS_WALK", 0);
#define OPK_NMS_WALK(NS_, FL_)                                                                 \
    hipLaunchKernelGGL((nms_detect_stream_kernel<lt, rc, NS_, FL_>), grid, dim3(lt), 0, stream, \
                       scratch, heat, parts, threshold)
#define OPK_NMS_STREAM(NS_)                                                                    \
    do {                                                                                       \
        switch (fl) {                                                                          \
        case 8:                                                                                \
            hipLaunchKernelGGL((nms_detect_walk2_kernel<rc, NS_>), grid2, dim3(64), 0, stream,  \
                               scratch, heat, parts, threshold);                               \
            break;                                                                             \
        case 1: OPK_NMS_WALK(NS_, 1); break;                                                   \
        case 3: OPK_NMS_WALK(NS_, 3); break;                                                   \
        case 4: OPK_NMS_WALK(NS_, 4); break;                                                   \
        case 5: OPK_NMS_WALK(NS_, 5); break;                                                   \
        case 7: OPK_NMS_WALK(NS_, 7); break;                                                   \
        default: OPK_NMS_WALK(NS_, 0); break;                                                  \
        }                                                                                      \
    } while (0)
        switch (heat.nsrc) {
        case 1: OPK_NMS_STREAM(1); break;
        case 2: OPK_NMS_STREAM(2); break;
        case 3: OPK_NMS_STREAM(3); break;
        default: OPK_NMS_STREAM(4); break;
        }
#undef OPK_NMS_STREAM
#undef OPK_NMS_WALK
    } else {
        constexpr int loy = 16;
        // one-wave workgroups (64 columns, 62 tested): no workgroup barrier holds four waves on
        // each other and a CU keeps ~4x more windows' loads in flight (measured 752 -> 650-672 us
        // per 64-frame launch against 256-lane workgroups; 8 / 32-row windows 711 / 700 us)
        hipLaunchKernelGGL((nms_detect_lazy_kernel<loy, 64>),
                           dim3((w + 61) / 62, (h + loy - 1) / loy, frames * parts), dim3(64), 0,
                           stream, scratch, heat, parts, threshold);
    }
    OPK_LAUNCH_CHECK();
    dim3 g2(parts, frames);
    hipLaunchKernelGGL(nms_finalize_kernel, g2, dim3(FT), 0, stream, peaks, scratch, heat, parts,
                       max_peaks1, threshold, offx, offy);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
