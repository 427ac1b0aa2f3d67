// nms.hip -- body-part peak extraction for gfx950 with nmsCpu numerics.
//
// Replaces op::nmsGpu (src/openpose/net/nmsBase.cu:251-351: register kernel + thrust scan over all
// channels + write kernel) with ONE launch computing what op::nmsCpu computes
// (src/openpose/net/nmsBase.cpp:7-170):
//   * interior pixels (1 < x < w-2, 1 < y < h-2): v > th and v > all 8 neighbours;
//   * pixels on row/column 1 or w-2 / h-2 (outer-border pixels of those rows/columns included):
//     v > th and v >= all 8 neighbours, neighbours outside the map read as th;
//   * any other pixel: never a peak;
//   * peaks kept in raster order, the first maxPeaks-1 only; position refined by the 7x7
//     score-weighted centroid in float (dy outer, dx inner), + offset; score = v.
// One workgroup of 1024 lanes per (part, frame) walks the plane in raster order, 4 pixels per
// lane per step; a block-wide OR skips peak-free steps (almost all of them), otherwise a wave
// shuffle scan + LDS wave totals give each peak its raster rank -- no global scan, no int peak
// map (the reference's 6 M-int thrust scan, nmsBase.cu:327-329).  HBM-bound: 24.1 MB read per
// frame (config 2).  -ffp-contract=off keeps the centroid sums bit-identical to the CPU.
#include "kernels.h"
#include "../common.h"

namespace opk {

namespace {

constexpr int NT = 1024;
constexpr int NWAVES = NT / 64;

__device__ __forceinline__ bool peak_at(const float* __restrict__ s, int w, int h, float th, int x,
                                        int y, float v)
{
    if (!(v > th)) return false;
    if (x > 1 && x < w - 2 && y > 1 && y < h - 2) {
        const float* r0 = s + (size_t)(y - 1) * w + x;
        const float* r1 = r0 + w;
        const float* r2 = r1 + w;
        return v > r0[-1] && v > r0[0] && v > r0[1] && v > r1[-1] && v > r1[1] && v > r2[-1] &&
               v > r2[0] && v > r2[1];
    }
    if (x == 1 || x == w - 2 || y == 1 || y == h - 2) {
        bool ok = true;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) {
                if (dx == 0 && dy == 0) continue;
                const int xx = x + dx, yy = y + dy;
                const float nb =
                    (xx >= 0 && xx < w && yy >= 0 && yy < h) ? s[(size_t)yy * w + xx] : th;
                ok = ok && (v >= nb);
            }
        return ok;
    }
    return false;
}

__global__ __launch_bounds__(NT) void nms_kernel(float* __restrict__ peaks,
                                                 const float* __restrict__ heat, int channels,
                                                 int parts, int h, int w, int max_peaks1,
                                                 float th, float offx, float offy)
{
    __shared__ int wave_tot[NWAVES];
    const int c = blockIdx.x, b = blockIdx.y;
    const float* s = heat + ((size_t)b * channels + c) * h * w;
    float* out = peaks + ((size_t)b * parts + c) * max_peaks1 * 3;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int quads = (w + 3) >> 2;
    const int items = h * quads;
    const int cap = max_peaks1 - 1;
    int count = 0;   // block-uniform

    for (int base = 0; base < items && count < cap; base += NT) {
        const int item = base + tid;
        unsigned mask = 0;
        int y = 0, x0 = 0;
        if (item < items) {
            y = item / quads;
            x0 = (item - y * quads) << 2;
            const float* row = s + (size_t)y * w;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int x = x0 + k;
                if (x < w && peak_at(s, w, h, th, x, y, row[x])) mask |= 1u << k;
            }
        }
        const int n = __popc(mask);
        if (!__syncthreads_or(n)) continue;
        // inclusive scan of n over the wave
        int incl = n;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int t = __shfl_up(incl, off, 64);
            if (lane >= off) incl += t;
        }
        if (lane == 63) wave_tot[wave] = incl;
        __syncthreads();
        int before = 0, total = 0;
        for (int i = 0; i < NWAVES; ++i) {
            const int t = wave_tot[i];
            before += (i < wave) ? t : 0;
            total += t;
        }
        int rank = count + before + incl - n;
        for (int k = 0; k < 4; ++k) {
            if (!(mask & (1u << k))) continue;
            if (rank < cap) {
                const int px = x0 + k, py = y;
                float xa = 0.f, ya = 0.f, sa = 0.f;
                for (int dy = -3; dy <= 3; ++dy) {
                    const int yy = py + dy;
                    if (yy < 0 || yy >= h) continue;
                    for (int dx = -3; dx <= 3; ++dx) {
                        const int xx = px + dx;
                        if (xx < 0 || xx >= w) continue;
                        const float sc = s[(size_t)yy * w + xx];
                        if (sc > 0) {
                            xa += (float)xx * sc;
                            ya += (float)yy * sc;
                            sa += sc;
                        }
                    }
                }
                float* o = out + (size_t)(rank + 1) * 3;
                o[0] = xa / sa + offx;
                o[1] = ya / sa + offy;
                o[2] = s[(size_t)py * w + px];
            }
            ++rank;
        }
        count += total;
        __syncthreads();   // wave_tot is rewritten by the next productive step
    }
    const int found = count < cap ? count : cap;
    // slot 0 = {count, 0, 0}; unused slots zeroed (the reference leaves them stale)
    for (int i = tid; i < (max_peaks1 - found) * 3; i += NT) {
        const int idx = found * 3 + 3 + i;
        if (idx < max_peaks1 * 3) out[idx] = 0.f;
    }
    if (tid == 0) {
        out[0] = (float)found;
        out[1] = 0.f;
        out[2] = 0.f;
    }
}

}  // namespace

void launch_nms(float* peaks, const float* heat, int frames, int channels, int parts, int h, int w,
                int max_peaks1, float threshold, float offx, float offy, hipStream_t stream)
{
    OPK_CHECK_ARG(frames > 0 && parts > 0 && parts <= channels, "bad channel counts");
    OPK_CHECK_ARG(h > 0 && w > 0 && max_peaks1 >= 1, "bad sizes");
    dim3 grid(parts, frames);
    hipLaunchKernelGGL(nms_kernel, grid, dim3(NT), 0, stream, peaks, heat, channels, parts, h, w,
                       max_peaks1, threshold, offx, offy);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
