/*
 * resize.c -- CPU oracle: bicubic resize + multi-scale merge (TEST INFRASTRUCTURE, see oracle.h).
 *
 * Reference call sites: /root/reference/src/openpose/net/resizeAndMergeBase.cpp
 *   :45-52   single scale: per channel cv::resize(src, dst, {W,H}, 0, 0, CV_INTER_CUBIC)
 *   :55-106  multi-scale: resize every source to the full target, add into scale 0, then /= N
 * The arithmetic lives in OpenCV (third-party, absent from this image; Ubuntu libopencv-dev 4.2 per
 * .github/workflows/main.yml:58-72).  Restated here: OpenCV's generic float INTER_CUBIC path
 *   scale = 1 / ((double)dsize / ssize);  f = (float)((d + 0.5) * scale - 0.5);  s0 = floor(f);
 *   t = f - s0;  taps s0-1 .. s0+2 clamped to the image (BORDER_REPLICATE);
 *   coefficients: Keys cubic with A = -0.75 (interpolateCubic);
 *   horizontal pass first (one row buffer per source row), then vertical.
 * Summation order (the source of every last-bit difference between OpenCV builds):
 *   horizontal pass (HResizeCubic, scalar in every version): ((S[x0-1]a0 + S[x0]a1) + S[x0+1]a2)
 *     + S[x0+2]a3, starting from 0 at the replicate-clamped border columns (0 + t0 == t0);
 *   vertical pass (VResizeCubic<float,...,VResizeCubicVec_32f>): OpenCV 4.x (the reference's CI:
 *     Ubuntu 20.04 libopencv-dev 4.2, Windows 4.5) writes the SIMD part with universal intrinsics,
 *       dst[x] = v_fma(S0, b0, v_fma(S1, b1, v_fma(S2, b2, S3 * b3)))
 *     for x < width rounded down to the vector width, and the scalar tail
 *       dst[x] = S0*b0 + S1*b1 + S2*b2 + S3*b3   (left to right);
 *     on the SSE2/SSE3 x86-64 baseline (no FMA3) v_fma is _mm_add_ps(_mm_mul_ps(a, b), c) and the
 *     vector width is 4 floats, so the body sums S0b0 + (S1b1 + (S2b2 + S3b3)) in float.  OpenCV
 *     3.x (Ubuntu 18.04's 3.2) used an SSE kernel that sums left to right everywhere.
 *   orc_set_resize_simd(4) (the default) restates 4.x; orc_set_resize_simd(0) restates 3.x.
 * Parity with OpenCV itself stays unpinned (OpenCV is absent); the HIP kernels follow the 4.x
 * order (kernels/heat_dev.h, resize.hip, nms.hip) and match THIS restatement bit for bit.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

static void keys_cubic(float x, float c[4])
{
    const float A = -0.75f;
    c[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
    c[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
    c[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
    c[3] = 1.f - c[0] - c[1] - c[2];
}

void orc_cubic_tables(int s, int d, int* ofs, float* coef)
{
    const double scale = 1. / ((double)d / s);
    for (int i = 0; i < d; ++i) {
        float f = (float)((i + 0.5) * scale - 0.5);
        const int s0 = (int)floorf(f);
        f -= (float)s0;
        ofs[i] = s0;
        keys_cubic(f, coef + 4 * i);
    }
}

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* vector width of OpenCV's vertical SIMD kernel: 4 (4.x on the x86-64 SSE baseline), 0 (3.x) */
static int g_simd = 4;
void orc_set_resize_simd(int lanes) { g_simd = lanes; }
int orc_resize_simd(void) { return g_simd; }

/* VResizeCubic for one output row of width dw */
static void vresize_cubic(float* o, const float* r0, const float* r1, const float* r2,
                          const float* r3, const float* be, int dw)
{
    const int vec_end = g_simd > 0 ? dw - dw % g_simd : 0;   /* whole vectors */
    int x = 0;
    for (; x < vec_end; ++x) {   /* v_fma nesting, each a mul then an add */
        const float t3 = r3[x] * be[3];
        const float t2 = r2[x] * be[2] + t3;
        const float t1 = r1[x] * be[1] + t2;
        o[x] = r0[x] * be[0] + t1;
    }
    for (; x < dw; ++x)   /* scalar tail (all of the row for 3.x) */
        o[x] = r0[x] * be[0] + r1[x] * be[1] + r2[x] * be[2] + r3[x] * be[3];
}

void orc_resize_cubic(float* dst, const float* src, int sh, int sw, int dh, int dw)
{
    int* xo = (int*)malloc(sizeof(int) * dw);
    int* yo = (int*)malloc(sizeof(int) * dh);
    float* xa = (float*)malloc(sizeof(float) * 4 * dw);
    float* yb = (float*)malloc(sizeof(float) * 4 * dh);
    float* rows = (float*)malloc(sizeof(float) * 4 * dw);
    orc_cubic_tables(sw, dw, xo, xa);
    orc_cubic_tables(sh, dh, yo, yb);
    for (int y = 0; y < dh; ++y) {
        for (int k = 0; k < 4; ++k) {
            const float* srow = src + (long)clampi(yo[y] - 1 + k, 0, sh - 1) * sw;
            float* r = rows + (long)k * dw;
            for (int x = 0; x < dw; ++x) {
                const float* a = xa + 4 * x;
                const int b = xo[x] - 1;
                r[x] = srow[clampi(b, 0, sw - 1)] * a[0] + srow[clampi(b + 1, 0, sw - 1)] * a[1]
                     + srow[clampi(b + 2, 0, sw - 1)] * a[2] + srow[clampi(b + 3, 0, sw - 1)] * a[3];
            }
        }
        vresize_cubic(dst + (long)y * dw, rows, rows + dw, rows + 2 * dw, rows + 3 * dw, yb + 4 * y,
                      dw);
    }
    free(xo); free(yo); free(xa); free(yb); free(rows);
}

void orc_resize_merge(float* dst, const float* const* srcs, int nsrc, int channels,
                      const int* src_hw, int dh, int dw)
{
    const long tplane = (long)dh * dw;
    if (nsrc == 1) {
        const long splane = (long)src_hw[0] * src_hw[1];
        for (int c = 0; c < channels; ++c)
            orc_resize_cubic(dst + c * tplane, srcs[0] + c * splane, src_hw[0], src_hw[1], dh, dw);
        return;
    }
    float* tmp = (float*)malloc(sizeof(float) * tplane);
    for (int n = 0; n < nsrc; ++n) {
        const long splane = (long)src_hw[2 * n] * src_hw[2 * n + 1];
        for (int c = 0; c < channels; ++c) {
            float* acc = dst + c * tplane;
            if (n == 0) {
                orc_resize_cubic(acc, srcs[0] + c * splane, src_hw[0], src_hw[1], dh, dw);
            } else {
                orc_resize_cubic(tmp, srcs[n] + c * splane, src_hw[2 * n], src_hw[2 * n + 1], dh, dw);
                for (long i = 0; i < tplane; ++i) acc[i] = tmp[i] + acc[i];    /* cv::add */
            }
        }
    }
    /* Mat /= N  ->  convertTo(alpha = 1/N): float multiply by (float)(1./N) */
    const float inv = (float)(1. / (double)nsrc);
    for (long i = 0; i < (long)channels * tplane; ++i) dst[i] = dst[i] * inv;
    free(tmp);
}

/* ---- resizeAndMergeGpu (CUDA build), src/openpose/net/resizeAndMergeBase.cu ----------------
 * include/openpose_private/gpu/cuda.hu:92-145: cubicSequentialData (clamped base column x1 =
 * clamp(floor(xs), 0, w-1), neighbours clamped, dx = xs - x1, possibly negative at the border),
 * cubicInterpolate (Catmull-Rom, A = -0.5, the polynomial as written), bicubicInterpolate (rows
 * first, then the column).  Single source: resize8TimesKernel (:105-140), source coordinate
 * (x + 0.5f) / r - 0.5f, r = ceil(H / h) on both axes (its 5x5 shared window reads the same clamped
 * rows and columns as bicubicInterpolate); identical sizes: fillKernel (a copy).  Several sources:
 * resizeAndAddAndAverageKernel (:142-162) with scale (W / w0) / (ratio_i / ratio_0), the sum over
 * sources in order, then / counter.  Compiled with -ffp-contract=off: every operation rounds (what
 * nvcc contracts in the polynomial is not reproducible here; parity unpinned). */
static float cuda_cubic(float v0, float v1, float v2, float v3, float dx)
{
    return (-0.5f * v0 + 1.5f * v1 - 1.5f * v2 + 0.5f * v3) * dx * dx * dx +
           (v0 - 2.5f * v1 + 2.f * v2 - 0.5f * v3) * dx * dx - 0.5f * (v0 - v2) * dx + v1;
}

static int mini(int a, int b) { return a < b ? a : b; }
static int maxi(int a, int b) { return a > b ? a : b; }

float orc_cuda_bicubic(const float* src, float xs, float ys, int sw, int sh)
{
    int xi[4], yi[4];
    xi[1] = clampi((int)floorf(xs), 0, sw - 1);
    xi[0] = maxi(0, xi[1] - 1);
    xi[2] = mini(sw - 1, xi[1] + 1);
    xi[3] = mini(sw - 1, xi[2] + 1);
    const float dx = xs - (float)xi[1];
    yi[1] = clampi((int)floorf(ys), 0, sh - 1);
    yi[0] = maxi(0, yi[1] - 1);
    yi[2] = mini(sh - 1, yi[1] + 1);
    yi[3] = mini(sh - 1, yi[2] + 1);
    const float dy = ys - (float)yi[1];
    float t[4];
    for (int i = 0; i < 4; ++i) {
        const float* r = src + (long)yi[i] * sw;
        t[i] = cuda_cubic(r[xi[0]], r[xi[1]], r[xi[2]], r[xi[3]], dx);
    }
    return cuda_cubic(t[0], t[1], t[2], t[3], dy);
}

/* dst [channels][dh][dw]; srcs[i] [channels][hw[2i]][hw[2i+1]]; ratios = scaleInputToNetInputs
 * (several sources only).  Returns 0, or -1 where the reference raises an error. */
int orc_resize_merge_cuda(float* dst, const float* const* srcs, int nsrc, int channels,
                          const int* hw, int dh, int dw, const float* ratios)
{
    float sx[8], sy[8];
    if (nsrc < 1 || nsrc > 8) return -1;
    if (nsrc == 1) {
        const int sh = hw[0], sw = hw[1];
        if (dw / sw == 1 && dh / sh == 1) {
            if (dw != sw || dh != sh) return -1;
            memcpy(dst, srcs[0], sizeof(float) * (size_t)channels * dh * dw);
            return 0;
        }
        if (dw / sw != 8 || dh / sh != 8) return -1;
        sx[0] = sy[0] = (float)(unsigned)ceilf(dh / (float)sh);
    } else {
        const float mw = dw / (float)hw[1], mh = dh / (float)hw[0];
        for (int i = 0; i < nsrc; ++i) {
            const float s = ratios[i] / ratios[0];
            sx[i] = mw / s;
            sy[i] = mh / s;
        }
    }
    for (int c = 0; c < channels; ++c)
        for (int y = 0; y < dh; ++y)
            for (int x = 0; x < dw; ++x) {
                float acc = 0.f;
                for (int i = 0; i < nsrc; ++i) {
                    const int sh = hw[2 * i], sw = hw[2 * i + 1];
                    const float xs = ((float)x + 0.5f) / sx[i] - 0.5f;
                    const float ys = ((float)y + 0.5f) / sy[i] - 0.5f;
                    acc += orc_cuda_bicubic(srcs[i] + (long)c * sh * sw, xs, ys, sw, sh);
                }
                dst[((long)c * dh + y) * dw + x] = nsrc > 1 ? acc / (float)nsrc : acc;
            }
    return 0;
}
