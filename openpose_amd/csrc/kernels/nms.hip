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

// OPK_NMS_JUMP (dev A/B builds: 1): the walk leaves a cold source window in one jump.  Measured
// slower (round 6, profiles/round6/nms_jump_paf_exit/: nms_detect_walk2 980 -> 1,498 us per
// 64-frame BODY_135 step; 88 VGPRs instead of 76, one wave per SIMD fewer), so off
#ifndef OPK_NMS_JUMP
#define OPK_NMS_JUMP 0
#endif

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
// Round 4 measured three variants of this walk, bit-identical, none kept (profiles/round4/
// nms_walk/): the peak test with all neighbour reads in flight at once (+30 %: more instructions
// per tested row), without the wait after the ring write (the same), the walk's source footprint
// staged in LDS (neutral).  nms_detect_walk2_kernel below replaced it for 1-4 sources.
template <int LT, int RC, int NS>
__global__ __launch_bounds__(LT) void nms_detect_stream_kernel(int* __restrict__ scratch,
                                                               const HeatMap M, int parts, float th)
{
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
    auto taps = [&src, &ssh, &ssw, &t](int n, int r, float v[4]) {   // source row r's taps
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
    float vprev = th;
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
        __syncthreads();                                     // rows y-2 .. y visible
        const int ty = y - 1;                                // row tested now
        if (ty >= ys && tid > 0 && tid < LT - 1 && xin) {
            auto get = [xw0](int xx, int yy) { return ring[(yy & 3) * LT + (xx - xw0)]; };
            if (peak_at(get, W, H, th, x, ty, vprev, false)) push_candidate(pl, ty * W + x);
        }
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

// COLD (one source, the pose pipeline's single-scale maps): source windows whose rows cannot reach
// the threshold are not evaluated.  A map row is sum_k b_k h_k over the window's four horizontal
// passes h_k, with OpenCV's cubic weights (A = -0.75: sum_k |b_k| = 1 + 2|A| t (1 - t) <= 1.375
// for every phase t), so max |h_k| * 1.375 (+ a rounding margin) <= th bounds every row of the
// window by th: none of them holds a pixel > th, so none is a peak, and as a neighbour of a tested
// pixel p (p > th) any value <= th compares as -inf does.  Such rows are set to -inf instead of
// evaluated (the candidate set is unchanged for NaN-free maps, as the neighbour maximum is).
constexpr float kCubicAbsSumBound = 1.3751f;
template <int RC, int NS, int CPL, bool COLD = false>
__global__ __launch_bounds__(64) void nms_detect_walk2_kernel(int* __restrict__ scratch,
                                                              const HeatMap M, int parts, float th)
{
    // (CPL 4 measured 1.5x slower than 2 on config 5: 136 VGPRs, and the wider test costs more
    // than the halved scalar work saves -- profiles/round4/nms_walk/ r4i)
    static_assert(CPL == 2 || CPL == 4, "columns per lane");
    constexpr int LT = 64, CW = CPL * LT - 2, NP = CPL / 2;   // NP column pairs per lane
    const int tid = threadIdx.x;
    const int c = blockIdx.z % parts, b = blockIdx.z / parts;
    const int plane = b * M.channels + c;
    const int H = M.h, W = M.w;
    const int xw0 = blockIdx.x * CW - 1;                     // map column of lane 0's first column
    const int x0 = xw0 + CPL * tid;                          // this lane's columns x0 .. x0 + CPL-1
    // OpenCV's SIMD body covers every in-map column of this wave: the one vertical order for all
    const bool wave_simd = min(xw0 + CPL * LT - 1, W - 1) < W - W % kCvVResizeLanes;
    const float inv_n = M.inv_n;
    const int ys = blockIdx.y * RC, ye = min(ys + RC, H);
    const int wy0 = ys - 1;
    // per source: the plane as a buffer resource (taps: a row's byte offset in an SGPR, the lane's
    // column offsets in VGPRs -- no address arithmetic per advance), the row tables as plain
    // pointers (uniform rows: scalar loads), the lane's column coefficients as column pairs
    __amdgpu_buffer_rsrc_t rs[NS];
    const int* yofs[NS];
    const float* ycoef[NS];
    int ssh[NS], ssw[NS], off[NS][CPL][4];
    float2_t A[NS][NP][4];
#pragma unroll
    for (int n = 0; n < NS; ++n) {
        const ResizeSource& S = M.src[n];
        yofs[n] = S.yofs;
        ycoef[n] = S.ycoef;
        ssh[n] = S.sh;
        ssw[n] = S.sw;
        rs[n] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(S.src + (size_t)plane * S.sh * S.sw), 0,
                                                  S.sh * S.sw * 4, 0x00020000);
        float cf[CPL][4];
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const int x = x0 + k;
            int xo = 0;
            float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
            if (x >= 0 && x < W) {
                xo = S.xofs[x];
                q = *reinterpret_cast<const float4*>(S.xcoef + 4 * x);
            }
            cf[k][0] = q.x; cf[k][1] = q.y; cf[k][2] = q.z; cf[k][3] = q.w;
#pragma unroll
            for (int t = 0; t < 4; ++t) off[n][k][t] = heat_clampi(xo - 1 + t, 0, ssw[n] - 1) * 4;
        }
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int t = 0; t < 4; ++t) A[n][p][t] = float2_t{cf[2 * p][t], cf[2 * p + 1][t]};
    }
    auto taps = [&](int n, int r, float2_t v[NP][4]) {   // source row r's taps of every column
        const int so = heat_clampi(r, 0, ssh[n] - 1) * ssw[n] * 4;
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int t = 0; t < 4; ++t)
                v[p][t] = float2_t{
                    __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs[n], off[n][2 * p][t], so, 0)),
                    __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs[n], off[n][2 * p + 1][t], so, 0))};
    };
    auto hsum = [&A](int n, int p, const float2_t v[4]) {   // cubic_hpass's sum, in its order
        return v[0] * A[n][p][0] + v[1] * A[n][p][1] + v[2] * A[n][p][2] + v[3] * A[n][p][3];
    };
    int cur[NS];
    float2_t h[NS][NP][4], nv[NS][NP][4];
#pragma unroll
    for (int n = 0; n < NS; ++n) {
        cur[n] = yofs[n][heat_clampi(wy0 < 0 ? 0 : wy0, 0, H - 1)];
        float2_t v[NP][4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            taps(n, cur[n] - 1 + k, v);
#pragma unroll
            for (int p = 0; p < NP; ++p) h[n][p][k] = hsum(n, p, v[p]);
        }
        taps(n, cur[n] + 3, nv[n]);                          // next advance's row, in flight
    }
    // (COLD) wave-uniform: the current source window bounds all its rows by th
    auto window_cold = [&]() -> bool {
        if constexpr (!COLD || NS != 1) {
            return false;
        } else {
            float m = 0.f;
#pragma unroll
            for (int p = 0; p < NP; ++p)
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    m = fmaxf(m, fmaxf(fabsf(h[0][p][k].x), fabsf(h[0][p][k].y)));
            return __ballot(m * kCubicAbsSumBound > th) == 0;
        }
    };
    bool cold = window_cold();
    int* pl = scratch + ((size_t)b * parts + c) * (CAP + 1);
    // which lanes test a column, by the row's kind in nmsCpu's rules (testable: not the window's
    // halo columns, inside the map): an inner row tests inner and edge columns, an edge row (1,
    // h-2) every in-map column, an outer row (0, h-1) the edge columns only -- as wave masks.
    // Out-of-map ROWS hold th (the border rule's outside value).  Out-of-map COLUMNS (neighbours
    // of x = 0 and x = w-1, tested on the edge rows 1 and h-2) read 0 from zero coefficients
    // where nmsCpu compares with th: the same outcome, since a tested value is > th >= 0 (both
    // comparisons hold) -- a negative threshold is rejected as nmsCpu rejects it
    // ("threshold value invalid.", nmsBase.cpp:121-122; api.cpp opk_nms, pose.cpp).
    uint64_t Min[CPL], Mok[CPL], Mout[CPL];
    bool cinner[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int x = x0 + k;
        const bool ok = x >= 0 && x < W && !(tid == 0 && k == 0) && !(tid == LT - 1 && k == CPL - 1);
        cinner[k] = x > 1 && x < W - 2;
        const bool edge = x == 1 || x == W - 2;
        Min[k] = __ballot(ok && (cinner[k] || edge));
        Mok[k] = __ballot(ok);
        Mout[k] = __ballot(ok && edge);
    }
    typedef float2_t Row[NP];
    // The walk with the vertical order fixed (WS: SIMD order for every column of the wave), no
    // per-row range checks and the row kind hoisted: rows wy0 (above the first tested row) and ys
    // are computed before the loops; the tested rows 2 .. h-3 (inner rows, almost all of them) run
    // in a loop of two rows per trip that tests only against the inner-row masks; the few rows at
    // the map's top and bottom take the generic test.  The row tables come by scalar loads one
    // trip ahead.  (PMC, round 4: the SALU, one instruction per CU cycle, had set the walk's pace
    // -- two scalar instructions per vector one -- so this keeps a row's scalar work small.)
    auto walk = [&](auto ws) {
        constexpr bool WS = decltype(ws)::value;
        // merged values of map row y (in the map) from its table entries tr (source row per
        // source) and bq (vertical coefficients per source)
        // (returns true when the row was not evaluated: a cold window, every value <= th)
        auto row = [&](const int tr[NS], const float4 bq[NS], Row out) -> bool {
            float2_t acc[NP];
            if constexpr (COLD && NS == 1) {
                if (cur[0] < tr[0]) {                        // uniform
                    do {
#pragma unroll
                        for (int p = 0; p < NP; ++p) {
                            h[0][p][0] = h[0][p][1]; h[0][p][1] = h[0][p][2]; h[0][p][2] = h[0][p][3];
                            h[0][p][3] = hsum(0, p, nv[0][p]);
                        }
                        ++cur[0];
                        taps(0, cur[0] + 3, nv[0]);
                    } while (cur[0] < tr[0]);
                    cold = window_cold();
                }
                if (cold) {
#pragma unroll
                    for (int p = 0; p < NP; ++p) out[p] = float2_t{-INFINITY, -INFINITY};
                    return true;
                }
            }
#pragma unroll
            for (int n = 0; n < NS; ++n) {
                while (cur[n] < tr[n]) {                     // uniform
#pragma unroll
                    for (int p = 0; p < NP; ++p) {
                        h[n][p][0] = h[n][p][1]; h[n][p][1] = h[n][p][2]; h[n][p][2] = h[n][p][3];
                        h[n][p][3] = hsum(n, p, nv[n][p]);
                    }
                    ++cur[n];
                    taps(n, cur[n] + 3, nv[n]);
                }
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    float2_t vn;
                    if constexpr (WS) {   // cubic_vpass, SIMD order
                        const float2_t t3 = h[n][p][3] * bq[n].w;
                        const float2_t t2 = h[n][p][2] * bq[n].z + t3;
                        const float2_t t1 = h[n][p][1] * bq[n].y + t2;
                        vn = h[n][p][0] * bq[n].x + t1;
                    } else {
                        const float ha[4] = {h[n][p][0].x, h[n][p][1].x, h[n][p][2].x, h[n][p][3].x};
                        const float hb[4] = {h[n][p][0].y, h[n][p][1].y, h[n][p][2].y, h[n][p][3].y};
                        vn = float2_t{cubic_vpass(ha, bq[n].x, bq[n].y, bq[n].z, bq[n].w, cubic_simd_column(x0 + 2 * p, W)),
                                      cubic_vpass(hb, bq[n].x, bq[n].y, bq[n].z, bq[n].w, cubic_simd_column(x0 + 2 * p + 1, W))};
                    }
                    acc[p] = (n == 0) ? vn : vn + acc[p];
                }
            }
#pragma unroll
            for (int p = 0; p < NP; ++p) out[p] = NS > 1 ? acc[p] * inv_n : acc[p];
            return false;
        };
        auto rowy = [&](int y, Row out) -> bool {            // table entries loaded here
            int tr[NS];
            float4 bq[NS];
#pragma unroll
            for (int n = 0; n < NS; ++n) {
                tr[n] = yofs[n][y];
                bq[n] = *reinterpret_cast<const float4*>(ycoef[n] + 4 * y);
            }
            return row(tr, bq, out);
        };
        auto val = [](const Row r, int k) { return r[k >> 1][k & 1]; };
        // test row ty (values mid) with its neighbour rows up / dn; INNER: ty in 2 .. h-3
        auto test = [&](auto inner, int ty, const Row up, const Row mid, const Row dn) {
            constexpr bool INNER = decltype(inner)::value;
            const bool row_inner = INNER || (unsigned)(ty - 2) < (unsigned)(H - 4);
            const bool row_edge = !INNER && (ty == 1 || ty == H - 2);
            uint64_t cand[CPL], any = 0;
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const uint64_t m = INNER ? Min[k] : row_inner ? Min[k] : row_edge ? Mok[k] : Mout[k];
                cand[k] = m & __ballot(val(mid, k) > th);
                any |= cand[k];
            }
            if (any == 0) return;                            // uniform
            // side neighbours from the adjacent lanes: left of column 0, right of column CPL-1
            const float lu = dpp_from_left(val(up, CPL - 1)), lm = dpp_from_left(val(mid, CPL - 1));
            const float ld = dpp_from_left(val(dn, CPL - 1));
            const float ru = dpp_from_right(val(up, 0)), rm = dpp_from_right(val(mid, 0));
            const float rd = dpp_from_right(val(dn, 0));
            bool pk[CPL], anyp = false;
#pragma unroll
            for (int k = 0; k < CPL; ++k) {
                const float L0 = k > 0 ? val(up, k - 1) : lu, L1 = k > 0 ? val(mid, k - 1) : lm;
                const float L2 = k > 0 ? val(dn, k - 1) : ld;
                const float R0 = k < CPL - 1 ? val(up, k + 1) : ru, R1 = k < CPL - 1 ? val(mid, k + 1) : rm;
                const float R2 = k < CPL - 1 ? val(dn, k + 1) : rd;
                const float nm = fmaxf(fmaxf(fmaxf(L0, val(up, k)), fmaxf(R0, L1)),
                                       fmaxf(fmaxf(R1, L2), fmaxf(val(dn, k), R2)));
                const float p = val(mid, k);
                pk[k] = ((cand[k] >> tid) & 1) && ((cinner[k] && row_inner) ? p > nm : p >= nm);
                anyp = anyp || pk[k];
            }
            if (anyp) {
#pragma unroll
                for (int k = 0; k < CPL; ++k)
                    if (pk[k]) push_candidate(pl, ty * W + x0 + k);
            }
        };
        const auto G = std::false_type{};                    // generic row kind
        const auto I = std::true_type{};                     // inner row
        Row up, mid, v, w;
        if (wy0 >= 0) rowy(wy0, up);                         // row ys - 1
        else
#pragma unroll
            for (int p = 0; p < NP; ++p) up[p] = float2_t{th, th};
        bool cmid = rowy(ys, mid);                           // ys < ye <= H
        int y = ys + 1;
        // rows y whose tested row y - 1 is 0 or 1 (top window only)
        for (; y < ye && y < 3; ++y) {
            cmid = rowy(y, v);                               // (v becomes mid)
            test(G, y - 1, up, mid, v);
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                up[p] = mid[p];
                mid[p] = v[p];
            }
        }
        // inner tested rows: y - 1 <= h - 3, two per trip, tables loaded a trip ahead through
        // pointers that step two rows a trip (immediate offsets).  The last trip's look-ahead reads
        // rows up to h: one entry past yofs / ycoef, still inside the context's table buffer
        // (ycoef | xcoef | yofs | xofs, Context::tables), and never used
        const int ylast = min(ye - 1, H - 2);                // last y of the inner loop
        if (y + 1 <= ylast) {
            const int* yp[NS];
            const float4* cp[NS];
            int tr0[NS], tr1[NS];
            float4 bq0[NS], bq1[NS];
#pragma unroll
            for (int n = 0; n < NS; ++n) {
                yp[n] = yofs[n] + y;
                cp[n] = reinterpret_cast<const float4*>(ycoef[n]) + y;
                tr0[n] = yp[n][0]; tr1[n] = yp[n][1];
                bq0[n] = cp[n][0]; bq1[n] = cp[n][1];
            }
            while (y + 1 <= ylast) {
                if constexpr (COLD && NS == 1 && OPK_NMS_JUMP) {
                    // rows y .. of a cold window below a cold row: none is evaluated or tested,
                    // so jump past all of them at once (their count from one load of the next 8
                    // table entries)
                    if (cold && cmid && tr0[0] == cur[0] && y + 8 <= ylast) {
                        int k = 1;
#pragma unroll
                        for (int i = 1; i < 8; ++i) k += (k == i && yp[0][i] == cur[0]) ? 1 : 0;
                        // (mid, the cold row above, already holds -inf; up is not read before
                        // the next trip overwrites it: that trip skips the test of mid)
                        y += k;
                        yp[0] = yofs[0] + y;
                        cp[0] = reinterpret_cast<const float4*>(ycoef[0]) + y;
                        tr0[0] = yp[0][0]; tr1[0] = yp[0][1];
                        bq0[0] = cp[0][0]; bq1[0] = cp[0][1];
                        continue;
                    }
                }
                int ntr0[NS], ntr1[NS];
                float4 nbq0[NS], nbq1[NS];
#pragma unroll
                for (int n = 0; n < NS; ++n) {
                    ntr0[n] = yp[n][2]; ntr1[n] = yp[n][3];
                    nbq0[n] = cp[n][2]; nbq1[n] = cp[n][3];
                    yp[n] += 2;
                    cp[n] += 2;
                }
                // a cold row (every value <= th) holds no candidate: its test is skipped
                const bool cv = row(tr0, bq0, v);
                if (!cmid) test(I, y - 1, up, mid, v);
                const bool cw = row(tr1, bq1, w);
                if (!cv) test(I, y, mid, v, w);
                cmid = cw;
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    up[p] = v[p];
                    mid[p] = w[p];
                }
#pragma unroll
                for (int n = 0; n < NS; ++n) {
                    tr0[n] = ntr0[n]; tr1[n] = ntr1[n];
                    bq0[n] = nbq0[n]; bq1[n] = nbq1[n];
                }
                y += 2;
            }
        }
        for (; y < ye; ++y) {                                // the rest (tested rows h-2, h-1 among them)
            rowy(y, v);
            if (y - 1 >= 2 && y - 1 <= H - 3) test(I, y - 1, up, mid, v);
            else test(G, y - 1, up, mid, v);
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                up[p] = mid[p];
                mid[p] = v[p];
            }
        }
        if (ye < H) rowy(ye, v);
        else
#pragma unroll
            for (int p = 0; p < NP; ++p) v[p] = float2_t{th, th};
        test(G, ye - 1, up, mid, v);
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
        // the two-columns-per-lane walk (nms_detect_walk2_kernel) for 1-4 sources: nms_detect
        // 2.2-2.4x faster than the ring walk on configs 2 and 5, +0.8 % frames/s on config 4
        // (profiles/round4/nms_walk2/); NMS_WALK=0 (dev A/B): the ring walk
        const bool walk2 = dev_switch("NMS_WALK", 8) != 0;
        // sub-threshold source windows skipped (one source; NMS_COLD=0: every row evaluated, A/B)
        const bool cold = dev_switch("NMS_COLD", 1) != 0;
        const dim3 grid2((w + 2 * lt - 3) / (2 * lt - 2), (h + rc - 1) / rc, frames * parts);
#define OPK_NMS_STREAM(NS_)                                                                    \
    do {                                                                                       \
        if (walk2 && cold && NS_ == 1)                                                         \
            hipLaunchKernelGGL((nms_detect_walk2_kernel<rc, NS_, 2, true>), grid2, dim3(64), 0, stream, \
                               scratch, heat, parts, threshold);                               \
        else if (walk2)                                                                        \
            hipLaunchKernelGGL((nms_detect_walk2_kernel<rc, NS_, 2>), grid2, dim3(64), 0, stream, \
                               scratch, heat, parts, threshold);                               \
        else                                                                                   \
            hipLaunchKernelGGL((nms_detect_stream_kernel<lt, rc, NS_>), grid, dim3(lt), 0, stream, \
                               scratch, heat, parts, threshold);                               \
    } while (0)
        switch (heat.nsrc) {
        case 1: OPK_NMS_STREAM(1); break;
        case 2: OPK_NMS_STREAM(2); break;
        case 3: OPK_NMS_STREAM(3); break;
        default: OPK_NMS_STREAM(4); break;
        }
#undef OPK_NMS_STREAM
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
