// paf.hip -- PAF line-integral scores for every candidate connection, gfx950.
//
// Replaces pafScoreKernel/process (src/openpose/net/bodyPartConnectorBase.cu:14-145) but with the
// CPU path's getScoreAB numerics (src/openpose/net/bodyPartConnectorBase.cpp:12-75):
//   n = max(5, min(25, int(sqrtf(5*max(|dx|,|dy|)) + 0.5f)));  samples at int(A + s*step + 0.5f)
//   clamped to [0, W-1] x [0, H-1];  PAF . unit(AB) > interTh counted;  score = sum/count if
//   count/n > interMinAbove, else (|AB| < sqrt(W*H)/150 ? defaultNmsTh + 1e-6 : 0).
// The "near" threshold is computed on the host in double (std::sqrt(int) in the reference) and
// the fallback score precomputed as float(defaultNmsTh + 1e-6).  -ffp-contract=off: each
// mul/add rounds separately, as on the CPU; sqrtf and '/' are correctly rounded (hipcc default).
// Work is tiny (<= 26*127*127 line integrals of <= 25 samples; ~650 for 5 people) and latency-
// bound: one workgroup per (pair, frame), lanes over (i, j).
#include "kernels.h"
#include "heat_dev.h"
#include "../common.h"

// OPK_PAF_EXIT (dev A/B builds: 0): a line leaves its sample loop once it can no longer pass
// (round 6, profiles/round6/nms_jump_paf_exit/: paf_compact 643 -> 450 us per 64-frame BODY_135
// step, bit-identical scores)
#ifndef OPK_PAF_EXIT
#define OPK_PAF_EXIT 1
#endif

namespace opk {

namespace {

__device__ __forceinline__ int round_pos(float a) { return int(a + 0.5f); }

// heat_at's cv::resize arithmetic (heat_dev.h, the M.nsrc lazy sources, CPU semantics) for the x
// and y PAF planes at once, their source images read from the interleaved LDS copy (src + 2 *
// loff[n]: source n's sh x sw pixels as (x, y) float pairs): one ds_read_b64 per tap serves both
// planes, each plane's arithmetic is heat_at's, operation for operation (bit-identical)
__device__ __forceinline__ float2 heat_at_lds2(const HeatMap& M, const float* src, const int* loff,
                                               int x, int y)
{
    float accx = 0.f, accy = 0.f;
    for (int n = 0; n < M.nsrc; ++n) {
        const ResizeSource& S = M.src[n];
        const float2* pl = reinterpret_cast<const float2*>(src) + loff[n];
        const int x0 = S.xofs[x];
        const float4 c = *reinterpret_cast<const float4*>(S.xcoef + 4 * x);
        const float4 b = *reinterpret_cast<const float4*>(S.ycoef + 4 * y);
        const int yb = S.yofs[y] - 1;
        const int c0 = heat_clampi(x0 - 1, 0, S.sw - 1), c1 = heat_clampi(x0, 0, S.sw - 1);
        const int c2 = heat_clampi(x0 + 1, 0, S.sw - 1), c3 = heat_clampi(x0 + 2, 0, S.sw - 1);
        float hx[4], hy[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float2* row = pl + heat_clampi(yb + k, 0, S.sh - 1) * S.sw;
            const float2 v0 = row[c0], v1 = row[c1], v2 = row[c2], v3 = row[c3];
            hx[k] = v0.x * c.x + v1.x * c.y + v2.x * c.z + v3.x * c.w;   // cubic_hpass
            hy[k] = v0.y * c.x + v1.y * c.y + v2.y * c.z + v3.y * c.w;
        }
        const bool simd = cubic_simd_column(x, M.w);
        const float vx = cubic_vpass(hx, b.x, b.y, b.z, b.w, simd);
        const float vy = cubic_vpass(hy, b.x, b.y, b.z, b.w, simd);
        accx = (n == 0) ? vx : vx + accx;
        accy = (n == 0) ? vy : vy + accy;
    }
    return M.nsrc > 1 ? make_float2(accx * M.inv_n, accy * M.inv_n) : make_float2(accx, accy);
}

// the fewest samples above inter_th with which the count test (float)c / (float)n > inter_min_above
// passes (n + 1: never); the test is monotonic in c
__device__ __forceinline__ int samples_needed(int n, float inter_min_above)
{
    int c = (int)fminf(fmaxf(inter_min_above * (float)n, 0.f), (float)n);
    while (c > 0 && (float)(c - 1) / (float)n > inter_min_above) --c;
    while (c <= n && !((float)c / (float)n > inter_min_above)) ++c;
    return c;
}

// LDS: the x and y PAF planes' sources staged once per (pair, frame) workgroup (interleaved, see
// heat_at_lds2); every sample of every candidate line then reads LDS instead of the L2/HBM source rows (dependent loads that set
// the kernel's pace: ~2.4 ms per 64 BODY_135 frames, 152 pairs of ~20 x 20 candidates)
template <bool LDS>
__device__ __forceinline__ float score_ab(const float* a, const float* b, const HeatMap& M,
                                          int plane_x, int plane_y, float inter_th,
                                          float inter_min_above, float reject_score,
                                          double near_dist, const float* lxy,
                                          const int* loff)
{
    const int W = M.w, H = M.h;
    const float vx = b[0] - a[0];
    const float vy = b[1] - a[1];
    const float vmax = fmaxf(fabsf(vx), fabsf(vy));
    const int n = max(5, min(25, round_pos(sqrtf(5 * vmax))));
    const float norm = sqrtf(vx * vx + vy * vy);
    if (!((double)norm > 1e-6)) return 0.f;
    const float ux = vx / norm, uy = vy / norm;
    const float stepx = vx / (float)n, stepy = vy / (float)n;
    float sum = 0.f;
    unsigned count = 0;
    // a line with more than n - samples_needed() samples at or below inter_th cannot pass the
    // count test below, whatever its other samples: it leaves the loop there (its result is the
    // fallback, which does not depend on them) -- most candidate lines join parts of different
    // people and fail within their first samples
    const int maxfail = OPK_PAF_EXIT ? n - samples_needed(n, inter_min_above) : n;
    int fails = 0;
    for (int s = 0; s < n; ++s) {
        const int px = max(0, min(W - 1, round_pos(a[0] + (float)s * stepx)));
        const int py = max(0, min(H - 1, round_pos(a[1] + (float)s * stepy)));
        const float2 h = LDS ? heat_at_lds2(M, lxy, loff, px, py)
                             : make_float2(heat_at(M, plane_x, px, py), heat_at(M, plane_y, px, py));
        const float v = ux * h.x + uy * h.y;
        if (v > inter_th) {
            sum += v;
            ++count;
        } else if (++fails > maxfail) {
            break;
        }
    }
    if ((float)count / (float)n > inter_min_above) return sum / (float)count;
    const float dist = sqrtf(vx * vx + vy * vy);
    return ((double)dist < near_dist) ? reject_score : 0.f;
}

// The same score with one candidate line per 32-lane half of a wave and one sample per lane
// (valid: the half has a line; s: the lane's sample index).  Neighbouring samples of a line read
// neighbouring source pixels, so a lane group's LDS reads are near-broadcasts instead of 32 random
// gathers (the per-lane-line form spent 60 % of its LDS cycles on bank conflicts, config 5 PMC).
// Bit-identical to score_ab: every lane evaluates its sample with score_ab's expressions; the
// count is the half's ballot; the sum is taken in sample order through readlane, the samples at
// or below the threshold (and the lanes past n) adding +0.0f -- exact, as the running sum starts
// at +0 and is never -0.  The return value is valid in every lane of the half.
template <bool LDS>
__device__ __forceinline__ float score_ab_spl(const float* a, const float* b, const HeatMap& M,
                                              int plane_x, int plane_y, float inter_th,
                                              float inter_min_above, float reject_score,
                                              double near_dist, const float* lxy,
                                              const int* loff, bool valid, int s, int half)
{
    const int W = M.w, H = M.h;
    float vx = 0.f, vy = 0.f, w = 0.f;
    int n = 5;
    bool degenerate = true, pass = false;
    if (valid) {
        vx = b[0] - a[0];
        vy = b[1] - a[1];
        const float vmax = fmaxf(fabsf(vx), fabsf(vy));
        n = max(5, min(25, round_pos(sqrtf(5 * vmax))));
        const float norm = sqrtf(vx * vx + vy * vy);
        degenerate = !((double)norm > 1e-6);
        if (!degenerate && s < n) {
            const float ux = vx / norm, uy = vy / norm;
            const float stepx = vx / (float)n, stepy = vy / (float)n;
            const int px = max(0, min(W - 1, round_pos(a[0] + (float)s * stepx)));
            const int py = max(0, min(H - 1, round_pos(a[1] + (float)s * stepy)));
            const float2 h = LDS ? heat_at_lds2(M, lxy, loff, px, py)
                                 : make_float2(heat_at(M, plane_x, px, py), heat_at(M, plane_y, px, py));
            const float v = ux * h.x + uy * h.y;
            pass = v > inter_th;
            w = pass ? v : 0.f;
        }
    }
    const uint64_t bal = __builtin_amdgcn_ballot_w64(pass);
    const unsigned count = (unsigned)__builtin_popcountll(half ? bal >> 32 : bal & 0xffffffffull);
    float sum0 = 0.f, sum1 = 0.f;
    const int wi = __builtin_bit_cast(int, w);
#pragma unroll
    for (int k = 0; k < 25; ++k) {   // n <= 25
        sum0 = sum0 + __builtin_bit_cast(float, __builtin_amdgcn_readlane(wi, k));
        sum1 = sum1 + __builtin_bit_cast(float, __builtin_amdgcn_readlane(wi, 32 + k));
    }
    const float sum = half ? sum1 : sum0;
    if (degenerate) return 0.f;
    if ((float)count / (float)n > inter_min_above) return sum / (float)count;
    const float dist = sqrtf(vx * vx + vy * vy);
    return ((double)dist < near_dist) ? reject_score : 0.f;
}

struct PafArgs {
    HeatMap heat;
    const float* peaks;
    int max_peaks;
    int npairs, nparts;
    const int* pairs;
    const int* mapx;
    const int* mapy;
    float inter_th, inter_min_above, reject_score;
    double near_dist;
};

__device__ __forceinline__ void pair_setup(const PafArgs& A, int b, int q, const float*& ca,
                                           const float*& cb, int& px, int& py, int& na, int& nb)
{
    const size_t stride = (size_t)(A.max_peaks + 1) * 3;
    const float* pk = A.peaks + (size_t)b * A.nparts * stride;
    ca = pk + A.pairs[2 * q] * stride;
    cb = pk + A.pairs[2 * q + 1] * stride;
    na = round_pos(ca[0]);
    nb = round_pos(cb[0]);
    px = b * A.heat.channels + A.mapx[q];
    py = b * A.heat.channels + A.mapy[q];
}

// dynamic LDS: the x and y planes of every source interleaved as (x, y) float pairs; source n's
// pixels start at pair loff[n] (host: paf_lds_floats; 0 = not staged: materialised, CUDA-semantics
// or too large maps)
extern __shared__ float paf_lds[];
constexpr int kPafLdsMinLines = 64;
template <bool LDS>
__device__ __forceinline__ void stage_planes(const PafArgs& A, int plx, int ply, int* loff,
                                             const float*& lxy)
{
    if constexpr (!LDS) return;
    const HeatMap& M = A.heat;
    int tot = 0;
    for (int n = 0; n < M.nsrc; ++n) {
        loff[n] = tot;
        tot += M.src[n].sh * M.src[n].sw;
    }
    lxy = paf_lds;
    float2* d = reinterpret_cast<float2*>(paf_lds);
    for (int n = 0; n < M.nsrc; ++n) {
        const ResizeSource& S = M.src[n];
        const int cnt = S.sh * S.sw;
        const float* gx = S.src + (size_t)plx * cnt;
        const float* gy = S.src + (size_t)ply * cnt;
        for (int i = threadIdx.x; i < cnt; i += blockDim.x) d[loff[n] + i] = make_float2(gx[i], gy[i]);
    }
    __syncthreads();
}

// SPL: pairs with few candidate lines take one line per half-wave, one sample per lane
// (score_ab_spl); otherwise one line per lane
template <bool LDS, bool SPL>
__global__ __launch_bounds__(256) void paf_dense_kernel(float* __restrict__ scores, PafArgs A)
{
    const int q = blockIdx.x, b = blockIdx.y;
    const float *ca, *cb;
    int plx, ply, na, nb;
    pair_setup(A, b, q, ca, cb, plx, ply, na, nb);
    int loff[kMaxResizeSources];
    const float* lxy = nullptr;
    const bool use = LDS && na * nb >= kPafLdsMinLines;
    if (use) stage_planes<LDS>(A, plx, ply, loff, lxy);
    float* out = scores + ((size_t)b * A.npairs + q) * A.max_peaks * A.max_peaks;
    // one sample per lane only for pairs with few candidate lines (< kPafLdsMinLines, never staged):
    // with many lines the half-waves' idle lanes and the in-order sums cost more than the
    // per-lane walks' LDS bank conflicts (config 5, 20 people: 0.82 -> 1.56 ms per step)
    if (SPL && na * nb < kPafLdsMinLines) {
        const int lane = threadIdx.x & 63, half = lane >> 5, s = lane & 31;
        const int wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
        for (int t0 = 2 * wv; t0 < na * nb; t0 += 2 * nw) {   // wave-uniform
            const int t = t0 + half;
            const bool valid = t < na * nb;
            const int i = valid ? t / nb : 0, j = valid ? t - (t / nb) * nb : 0;
            const float sc = score_ab_spl<false>(ca + 3 * (i + 1), cb + 3 * (j + 1), A.heat, plx, ply,
                                                 A.inter_th, A.inter_min_above, A.reject_score,
                                                 A.near_dist, lxy, loff, valid, s, half);
            if (valid && s == 0) out[(size_t)i * A.max_peaks + j] = sc;
        }
        return;
    }
    for (int t = threadIdx.x; t < na * nb; t += blockDim.x) {
        const int i = t / nb, j = t - (t / nb) * nb;
        out[(size_t)i * A.max_peaks + j] =
            use ? score_ab<true>(ca + 3 * (i + 1), cb + 3 * (j + 1), A.heat, plx, ply, A.inter_th,
                                 A.inter_min_above, A.reject_score, A.near_dist, lxy, loff)
                : score_ab<false>(ca + 3 * (i + 1), cb + 3 * (j + 1), A.heat, plx, ply, A.inter_th,
                                  A.inter_min_above, A.reject_score, A.near_dist, lxy, loff);
    }
}

// compact records: offset of pair q = sum over earlier pairs of nA*nB (recomputed per block from
// the 2*q peak counts it needs -- 26 pairs, cheaper than a separate scan launch).
template <bool LDS, bool SPL>
__global__ __launch_bounds__(256) void paf_compact_kernel(float* __restrict__ records,
                                                          int rec_floats, PafArgs A)
{
    const int q = blockIdx.x, b = blockIdx.y;
    const float *ca, *cb;
    int plx, ply, na, nb;
    pair_setup(A, b, q, ca, cb, plx, ply, na, nb);
    const size_t stride = (size_t)(A.max_peaks + 1) * 3;
    const float* pk = A.peaks + (size_t)b * A.nparts * stride;
    int offset = 0, total = 0;
    for (int r = 0; r < A.npairs; ++r) {
        const int m = round_pos(pk[A.pairs[2 * r] * stride]) * round_pos(pk[A.pairs[2 * r + 1] * stride]);
        offset += (r < q) ? m : 0;
        total += m;
    }
    float* rec = records + (size_t)b * rec_floats;
    const bool fits = total + 1 <= rec_floats;
    if (q == 0 && threadIdx.x == 0) rec[0] = fits ? (float)total : -1.f;
    if (!fits) return;
    int loff[kMaxResizeSources];
    const float* lxy = nullptr;
    // staged only for pairs with many candidate lines (block-uniform): a few lines read fewer
    // bytes than the two planes hold
    const bool use = LDS && na * nb >= kPafLdsMinLines;
    if (use) stage_planes<LDS>(A, plx, ply, loff, lxy);
    float* out = rec + 1 + offset;
    // one sample per lane only for pairs with few candidate lines (< kPafLdsMinLines, never staged):
    // with many lines the half-waves' idle lanes and the in-order sums cost more than the
    // per-lane walks' LDS bank conflicts (config 5, 20 people: 0.82 -> 1.56 ms per step)
    if (SPL && na * nb < kPafLdsMinLines) {
        const int lane = threadIdx.x & 63, half = lane >> 5, s = lane & 31;
        const int wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
        for (int t0 = 2 * wv; t0 < na * nb; t0 += 2 * nw) {   // wave-uniform
            const int t = t0 + half;
            const bool valid = t < na * nb;
            const int i = valid ? t / nb : 0, j = valid ? t - (t / nb) * nb : 0;
            const float sc = score_ab_spl<false>(ca + 3 * (i + 1), cb + 3 * (j + 1), A.heat, plx, ply,
                                                 A.inter_th, A.inter_min_above, A.reject_score,
                                                 A.near_dist, lxy, loff, valid, s, half);
            if (valid && s == 0) out[t] = sc;
        }
        return;
    }
    for (int t = threadIdx.x; t < na * nb; t += blockDim.x) {
        const int i = t / nb, j = t - (t / nb) * nb;
        out[t] = use ? score_ab<true>(ca + 3 * (i + 1), cb + 3 * (j + 1), A.heat, plx, ply, A.inter_th,
                                      A.inter_min_above, A.reject_score, A.near_dist, lxy, loff)
                     : score_ab<false>(ca + 3 * (i + 1), cb + 3 * (j + 1), A.heat, plx, ply, A.inter_th,
                                       A.inter_min_above, A.reject_score, A.near_dist, lxy, loff);
    }
}

PafArgs make_args(const HeatMap& heat, const float* peaks, int max_peaks, const PafPairTable& t,
                  float inter_th, float inter_min_above, float reject_score, double near_dist)
{
    PafArgs a{};
    a.heat = heat;
    a.peaks = peaks;
    a.max_peaks = max_peaks;
    a.npairs = t.npairs;
    a.nparts = t.nparts;
    a.pairs = t.pairs;
    a.mapx = t.mapx;
    a.mapy = t.mapy;
    a.inter_th = inter_th;
    a.inter_min_above = inter_min_above;
    a.reject_score = reject_score;
    a.near_dist = near_dist;
    return a;
}

// LDS bytes of a workgroup's staged x / y planes: lazy maps with CPU semantics whose sources fit
// 40 KiB (BODY_25 / BODY_135 at 368 rows: 2 x 46 x 82 floats = 30 KB); 0 = read the sources (or
// the materialised map) through heat_at (PAF_LDS=0: always, dev A/B).  Measured
// (profiles/round3/paf_lds/): BODY_135, 20 people, paf_compact 2.43 -> 0.82 ms per 64 frames;
// the four-scale map (57 KB: two workgroups per CU) ran 0.75 % slower staged, so it reads L2
size_t paf_lds_bytes(const HeatMap& M)
{
    if (M.heat || M.cuda || M.nsrc < 1 || dev_switch("PAF_LDS", 1) == 0) return 0;
    size_t n = 0;
    for (int i = 0; i < M.nsrc; ++i) n += (size_t)M.src[i].sh * M.src[i].sw;
    const size_t bytes = 2 * n * sizeof(float);
    return bytes <= 40 * 1024 ? bytes : 0;
}

}  // namespace

void launch_paf_scores(float* scores, const HeatMap& heat, const float* peaks, int frames,
                       int max_peaks, const PafPairTable& t, float inter_th,
                       float inter_min_above, float reject_score, double near_dist,
                       hipStream_t stream)
{
    OPK_CHECK_ARG(frames > 0 && t.npairs > 0 && max_peaks > 0, "bad sizes");
    PafArgs a = make_args(heat, peaks, max_peaks, t, inter_th, inter_min_above, reject_score,
                          near_dist);
    const size_t lds = paf_lds_bytes(heat);
    const bool spl = dev_switch("PAF_SPL", 1) != 0;
    if (lds && spl) hipLaunchKernelGGL((paf_dense_kernel<true, true>), dim3(t.npairs, frames), dim3(256), lds, stream, scores, a);
    else if (lds) hipLaunchKernelGGL((paf_dense_kernel<true, false>), dim3(t.npairs, frames), dim3(256), lds, stream, scores, a);
    else if (spl) hipLaunchKernelGGL((paf_dense_kernel<false, true>), dim3(t.npairs, frames), dim3(256), 0, stream, scores, a);
    else hipLaunchKernelGGL((paf_dense_kernel<false, false>), dim3(t.npairs, frames), dim3(256), 0, stream, scores, a);
    OPK_LAUNCH_CHECK();
}

void launch_paf_scores_compact(float* records, int rec_floats, const HeatMap& heat,
                               const float* peaks, int frames, int max_peaks,
                               const PafPairTable& t, float inter_th, float inter_min_above,
                               float reject_score, double near_dist, hipStream_t stream)
{
    OPK_CHECK_ARG(frames > 0 && t.npairs > 0 && max_peaks > 0 && rec_floats > 1, "bad sizes");
    PafArgs a = make_args(heat, peaks, max_peaks, t, inter_th, inter_min_above, reject_score,
                          near_dist);
    const size_t lds = paf_lds_bytes(heat);
    // PAF_SPL (dev A/B): 0 = one candidate line per lane
    const bool spl = dev_switch("PAF_SPL", 1) != 0;
    if (lds && spl)
        hipLaunchKernelGGL((paf_compact_kernel<true, true>), dim3(t.npairs, frames), dim3(256), lds, stream,
                           records, rec_floats, a);
    else if (lds)
        hipLaunchKernelGGL((paf_compact_kernel<true, false>), dim3(t.npairs, frames), dim3(256), lds, stream,
                           records, rec_floats, a);
    else if (spl)
        hipLaunchKernelGGL((paf_compact_kernel<false, true>), dim3(t.npairs, frames), dim3(256), 0, stream,
                           records, rec_floats, a);
    else
        hipLaunchKernelGGL((paf_compact_kernel<false, false>), dim3(t.npairs, frames), dim3(256), 0, stream,
                           records, rec_floats, a);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
