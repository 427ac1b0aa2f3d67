/*
 * nms.c -- CPU oracle: restatement of op::nmsCpu (TEST INFRASTRUCTURE, see oracle.h).
 *
 * Reference: /root/reference/src/openpose/net/nmsBase.cpp
 *   :7-68    nmsRegisterKernelCPU -- three pixel classes
 *   :70-107  nmsAccuratePeakPosition -- 7x7 score-weighted centroid
 *   :109-170 nmsCpu -- raster scan per channel, keep the first targetPeaks-1 peaks
 * Parity status: unpinned (the reference file #includes <opencv2/opencv.hpp>, which the image
 * does not have, so it cannot be compiled here).  Known-answer tests: tests/test_oracle_nms.py.
 * Compiled with -ffp-contract=off: the accumulations below are plain float mul/add in the
 * reference's loop order.
 */
#include <math.h>

#include "oracle.h"

/* Returns 1 iff (x, y) registers as a peak (nmsBase.cpp:16-67). */
static int nms_is_peak(const float* s, int w, int h, float th, int x, int y)
{
    const float v = s[y * w + x];
    /* class 1: strictly inside the first inner ring -> strict maximum over 8 neighbours */
    if (x > 1 && x < w - 2 && y > 1 && y < h - 2) {
        if (!(v > th)) return 0;
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                if (!dx && !dy) continue;
                if (!(v > s[(y + dy) * w + (x + dx)])) return 0;
            }
        return 1;
    }
    /* class 2: any pixel on row/column 1 or w-2/h-2 (including the outer border pixels of those
     * rows/columns) -> non-strict maximum; neighbours outside the map read as `th` */
    if (x == 1 || x == w - 2 || y == 1 || y == h - 2) {
        if (!(v > th)) return 0;
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                if (!dx && !dy) continue;
                const int xx = x + dx, yy = y + dy;
                const float nb = (xx >= 0 && xx < w && yy >= 0 && yy < h) ? s[yy * w + xx] : th;
                if (!(v >= nb)) return 0;
            }
        return 1;
    }
    /* class 3: everything else (outer border away from the inner ring) never registers */
    return 0;
}

/* nmsBase.cpp:70-107 -- xAcc/yAcc/scoreAcc accumulated in float, dy outer, dx inner */
static void nms_refine(float* out, const float* s, int px, int py, int w, int h,
                       float offx, float offy)
{
    float xacc = 0.f, yacc = 0.f, sacc = 0.f;
    for (int dy = -3; dy <= 3; ++dy) {
        const int y = py + dy;
        if (y < 0 || y >= h) continue;
        for (int dx = -3; dx <= 3; ++dx) {
            const int x = px + dx;
            if (x < 0 || x >= w) continue;
            const float sc = s[y * w + x];
            if (sc > 0) {
                xacc += (float)x * sc;
                yacc += (float)y * sc;
                sacc += sc;
            }
        }
    }
    out[0] = xacc / sacc + offx;
    out[1] = yacc / sacc + offy;
    out[2] = s[py * w + px];
}

void orc_nms(float* peaks, const float* heat, float threshold, int channels, int max_peaks1,
             int h, int w, float offset_x, float offset_y)
{
    const long plane = (long)h * w;
    for (int c = 0; c < channels; ++c) {
        const float* s = heat + c * plane;
        float* t = peaks + (long)c * max_peaks1 * 3;
        int count = 1;                               /* slot 0 holds the count */
        for (int y = 0; y < h && count < max_peaks1; ++y)
            for (int x = 0; x < w && count < max_peaks1; ++x)
                if (nms_is_peak(s, w, h, threshold, x, y)) {
                    nms_refine(&t[count * 3], s, x, y, w, h, offset_x, offset_y);
                    ++count;
                }
        t[0] = (float)(count - 1);
    }
}

/* ---- nmsGpu (CUDA build) rules, src/openpose/net/nmsBase.cu --------------------------------
 *   :50-90   nmsRegisterKernel -- interior pixels (0 < x < w-1, 0 < y < h-1) with v > th and v
 *            strictly greater than all 8 neighbours; every border pixel is 0
 *   :161-240 writeResultKernel -- peaks in raster order (thrust exclusive scan), the first
 *            maxPeaks (= targetSize[2]-1) refined, count = min(peaks, maxPeaks); the centroid loop
 *            is nmsCpu's, but nvcc contracts `xAcc += x*score` into a fused multiply-add (default
 *            --fmad=true; the reference sets no nvcc math flags, CMakeLists.txt / cmake/Cuda.cmake)
 * Parity unpinned (no CUDA toolchain here). */
static int nms_is_peak_cuda(const float* s, int w, int h, float th, int x, int y)
{
    if (!(x > 0 && x < w - 1 && y > 0 && y < h - 1)) return 0;
    const float v = s[y * w + x];
    if (!(v > th)) return 0;
    for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
            if (!dx && !dy) continue;
            if (!(v > s[(y + dy) * w + (x + dx)])) return 0;
        }
    return 1;
}

static void nms_refine_cuda(float* out, const float* s, int px, int py, int w, int h,
                            float offx, float offy)
{
    float xacc = 0.f, yacc = 0.f, sacc = 0.f;
    for (int dy = -3; dy <= 3; ++dy) {
        const int y = py + dy;
        if (y < 0 || y >= h) continue;
        for (int dx = -3; dx <= 3; ++dx) {
            const int x = px + dx;
            if (x < 0 || x >= w) continue;
            const float sc = s[y * w + x];
            if (sc > 0) {
                xacc = fmaf((float)x, sc, xacc);
                yacc = fmaf((float)y, sc, yacc);
                sacc += sc;
            }
        }
    }
    out[0] = xacc / sacc + offx;
    out[1] = yacc / sacc + offy;
    out[2] = s[py * w + px];
}

void orc_nms_cuda(float* peaks, const float* heat, float threshold, int channels, int max_peaks1,
                  int h, int w, float offset_x, float offset_y)
{
    const long plane = (long)h * w;
    for (int c = 0; c < channels; ++c) {
        const float* s = heat + c * plane;
        float* t = peaks + (long)c * max_peaks1 * 3;
        int count = 1;
        for (int y = 0; y < h && count < max_peaks1; ++y)
            for (int x = 0; x < w && count < max_peaks1; ++x)
                if (nms_is_peak_cuda(s, w, h, threshold, x, y)) {
                    nms_refine_cuda(&t[count * 3], s, x, y, w, h, offset_x, offset_y);
                    ++count;
                }
        t[0] = (float)(count - 1);
    }
}
