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

namespace opk {

namespace {

__device__ __forceinline__ int round_pos(float a) { return int(a + 0.5f); }

__device__ __forceinline__ float score_ab(const float* a, const float* b, const HeatMap& M,
                                          int plane_x, int plane_y, float inter_th,
                                          float inter_min_above, float reject_score,
                                          double near_dist)
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
    for (int s = 0; s < n; ++s) {
        const int px = max(0, min(W - 1, round_pos(a[0] + (float)s * stepx)));
        const int py = max(0, min(H - 1, round_pos(a[1] + (float)s * stepy)));
        const float v = ux * heat_at(M, plane_x, px, py) + uy * heat_at(M, plane_y, px, py);
        if (v > inter_th) {
            sum += v;
            ++count;
        }
    }
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

__global__ __launch_bounds__(256) void paf_dense_kernel(float* __restrict__ scores, PafArgs A)
{
    const int q = blockIdx.x, b = blockIdx.y;
    const float *ca, *cb;
    int plx, ply, na, nb;
    pair_setup(A, b, q, ca, cb, plx, ply, na, nb);
    float* out = scores + ((size_t)b * A.npairs + q) * A.max_peaks * A.max_peaks;
    for (int t = threadIdx.x; t < na * nb; t += blockDim.x) {
        const int i = t / nb, j = t - (t / nb) * nb;
        out[(size_t)i * A.max_peaks + j] =
            score_ab(ca + 3 * (i + 1), cb + 3 * (j + 1), A.heat, plx, ply, A.inter_th,
                     A.inter_min_above, A.reject_score, A.near_dist);
    }
}

// compact records: offset of pair q = sum over earlier pairs of nA*nB (recomputed per block from
// the 2*q peak counts it needs -- 26 pairs, cheaper than a separate scan launch).
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
    float* out = rec + 1 + offset;
    for (int t = threadIdx.x; t < na * nb; t += blockDim.x) {
        const int i = t / nb, j = t - (t / nb) * nb;
        out[t] = score_ab(ca + 3 * (i + 1), cb + 3 * (j + 1), A.heat, plx, ply, A.inter_th,
                          A.inter_min_above, A.reject_score, A.near_dist);
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

}  // namespace

void launch_paf_scores(float* scores, const HeatMap& heat, const float* peaks, int frames,
                       int max_peaks, const PafPairTable& t, float inter_th,
                       float inter_min_above, float reject_score, double near_dist,
                       hipStream_t stream)
{
    OPK_CHECK_ARG(frames > 0 && t.npairs > 0 && max_peaks > 0, "bad sizes");
    PafArgs a = make_args(heat, peaks, max_peaks, t, inter_th, inter_min_above, reject_score,
                          near_dist);
    hipLaunchKernelGGL(paf_dense_kernel, dim3(t.npairs, frames), dim3(256), 0, stream, scores, a);
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
    hipLaunchKernelGGL(paf_compact_kernel, dim3(t.npairs, frames), dim3(256), 0, stream, records,
                       rec_floats, a);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
