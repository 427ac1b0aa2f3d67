/*
 * preprocess.c -- CPU oracle for the frame -> net-input stage (TEST INFRASTRUCTURE ONLY; see
 * oracle.h).  Restates, in plain C:
 *
 *   op::ScaleAndSizeExtractor::extract       src/openpose/core/scaleAndSizeExtractor.cpp:37-105
 *   op::resizeGetScaleFactor                 src/openpose/utilities/openCv.cpp:182-195
 *   op::CvMatToOpInput::createArray (CPU)    src/openpose/core/cvMatToOpInput.cpp:63-98
 *     -> resizeFixedAspectRatio              src/openpose/utilities/openCvPrivate.cpp:34-52
 *        = cv::warpAffine(M = diag(s), INTER_AREA if s <= 1 else INTER_CUBIC, BORDER_CONSTANT 0)
 *     -> uCharCvMatToFloatPtr                src/openpose/utilities/openCv.cpp:57-150
 *
 * cv::warpAffine is third-party OpenCV (Ubuntu libopencv-dev 4.2, .github/workflows/main.yml:58-72),
 * absent from this image: PARITY UNPINNED.  What is restated is OpenCV 4.2's generic 8-bit path
 * (imgwarp.cpp, no IPP -- the Debian/Ubuntu packages are built without it):
 *   - warpAffine maps INTER_AREA to INTER_LINEAR;
 *   - M is inverted (invertAffineTransform arithmetic: D = 1/(m00*m11), A11 = m11*D, ...);
 *   - per destination pixel X = (X0(y) + adelta[x]) >> (AB_BITS - INTER_BITS) with
 *     AB_BITS = 10, INTER_BITS = 5, adelta[x] = cvRound(M00*x*1024),
 *     X0 = cvRound((M01*y + M02)*1024) + round_delta (1024/32/2 = 16), likewise Y;
 *     source tap = X >> 5, fraction index = X & 31;
 *   - remap with the fixed-point tables of initInterTab2D (INTER_REMAP_COEF_SCALE = 32768, the
 *     outer product of the 1-D float coefficients rounded, the sum corrected to 32768 on the
 *     largest / smallest of the four taps at [ksize/2, ksize/2 + 1]^2), out-of-image taps read the
 *     border value 0, result (sum + 16384) >> 15 saturated to uchar.
 * Normalisation 1 (VGG, every model but BODY_19N): float(u8) * (1/256.f) - 0.5f (exact in float,
 * so the AVX fmadd and the plain form agree); 0: float(u8).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "oracle.h"

#define INTER_BITS 5
#define INTER_TAB 32
#define AB_BITS 10
#define AB_SCALE 1024
#define COEF_SCALE 32768

/* cvRound(double) / cvRound(float): round half to even (SSE2 cvtsd2si under the default MXCSR) */
static int round_d(double v) { return (int)lrint(v); }
static int round_f(float v) { return (int)lrintf(v); }
static short sat_short(int v) { return (short)(v < -32768 ? -32768 : v > 32767 ? 32767 : v); }

static void cubic_coeffs(float x, float* c)   /* interpolateCubic, A = -0.75 */
{
    const float A = -0.75f;
    c[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
    c[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
    c[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
    c[3] = 1.f - c[0] - c[1] - c[2];
}

/* itab: zeroed, (1024 + 1) * ksize^2 shorts.  The fraction-0 entry saturates 1.0 to 32767 and
 * is corrected; for ksize 2 initInterTab2D's correction window [1, 2]^2 reaches past the entry
 * into the next, still zero, one -- restated as such ({32767, 0, 0, 1}). */
void orc_warp_tab(int cubic, short* itab)
{
    const int k = cubic ? 4 : 2;
    float t1[INTER_TAB * 4];
    for (int i = 0; i < INTER_TAB; ++i) {
        const float x = i * (1.f / INTER_TAB);
        if (cubic) {
            cubic_coeffs(x, t1 + i * 4);
        } else {
            t1[i * 2] = 1.f - x;
            t1[i * 2 + 1] = x;
        }
    }
    for (int i = 0; i < INTER_TAB; ++i)
        for (int j = 0; j < INTER_TAB; ++j) {
            short* it = itab + (i * INTER_TAB + j) * k * k;
            int isum = 0;
            for (int k1 = 0; k1 < k; ++k1) {
                const float vy = t1[i * k + k1];
                for (int k2 = 0; k2 < k; ++k2) {
                    const float v = vy * t1[j * k + k2];
                    it[k1 * k + k2] = sat_short(round_f(v * COEF_SCALE));
                    isum += it[k1 * k + k2];
                }
            }
            if (isum != COEF_SCALE) {
                const int diff = isum - COEF_SCALE, k2h = k / 2;
                int Mk1 = k2h, Mk2 = k2h, mk1 = k2h, mk2 = k2h;
                for (int k1 = k2h; k1 < k2h + 2; ++k1)
                    for (int k2 = k2h; k2 < k2h + 2; ++k2) {
                        if (it[k1 * k + k2] < it[mk1 * k + mk2]) {
                            mk1 = k1;
                            mk2 = k2;
                        } else if (it[k1 * k + k2] > it[Mk1 * k + Mk2]) {
                            Mk1 = k1;
                            Mk2 = k2;
                        }
                    }
                if (diff < 0)
                    it[Mk1 * k + Mk2] = (short)(it[Mk1 * k + Mk2] - diff);
                else
                    it[mk1 * k + mk2] = (short)(it[mk1 * k + mk2] - diff);
            }
        }
}

double orc_resize_scale_factor(int iw, int ih, int tw, int th)
{
    const double rw = (tw - 1) / (double)(iw - 1);
    const double rh = (th - 1) / (double)(ih - 1);
    return rw < rh ? rw : rh;
}

/* positiveIntRound (include/openpose/utilities/fastMath.hpp:29-32): int(a + 0.5f) in the type of a */
static int pos_round(float v) { return (int)(v + 0.5f); }
static int pos_round_d(double v) { return (int)(v + 0.5f); }

int orc_scale_and_size(int in_w, int in_h, int net_w, int net_h, float dyn, int scale_number,
                       double scale_gap, double* scales, int* sizes /* 2*scale_number: w, h */)
{
    if (in_w <= 0 || in_h <= 0 || scale_number < 1) return -1;
    if (net_w <= 0 || net_h <= 0) {
        if (net_w <= 0 && net_h <= 0) return -1;
        if (dyn > 0) {
            if (net_w <= 0) {
                const float a = net_h * dyn * 16.f / 9.f;
                const float b = net_h * in_w / (float)in_h;
                net_w = 16 * pos_round(1 / 16.f * (a < b ? a : b));
            } else {
                const float a = net_w * dyn * 9.f / 16.f;
                const float b = net_w * in_h / (float)in_w;
                net_h = 16 * pos_round(1 / 16.f * (a < b ? a : b));
            }
        } else {
            if (net_w <= 0)
                net_w = 16 * pos_round(1 / 16.f * net_h * in_w / (float)in_h);
            else
                net_h = 16 * pos_round(1 / 16.f * net_w * in_h / (float)in_w);
        }
    }
    for (int i = 0; i < scale_number; ++i) {
        const double cur = 1. - i * scale_gap;
        if (cur < 0. || 1. < cur) return -1;
        int tw = pos_round_d(net_w * cur) / 16 * 16;
        int th = pos_round_d(net_h * cur) / 16 * 16;
        /* fastTruncate(v, 1, max) = fastMin(max, fastMax(1, v)) (fastMath.hpp:85-88) */
        tw = tw < 1 ? 1 : tw;
        tw = net_w < tw ? net_w : tw;
        th = th < 1 ? 1 : th;
        th = net_h < th ? net_h : th;
        scales[i] = orc_resize_scale_factor(in_w, in_h, tw, th);
        sizes[2 * i] = tw;
        sizes[2 * i + 1] = th;
    }
    return 0;
}

/* warpAffine coordinate of destination index d along one axis (M diagonal: separable) */
static void warp_coord(double m, int d, int* s, int* frac)
{
    const int X0 = round_d(0.0 * AB_SCALE) + AB_SCALE / INTER_TAB / 2;
    const int X = (X0 + round_d(m * d * AB_SCALE)) >> (AB_BITS - INTER_BITS);
    *s = X >> INTER_BITS;
    *frac = X & (INTER_TAB - 1);
}

void orc_cvmat_to_input(float* dst, const uint8_t* src, int sw, int sh, double scale, int dw,
                        int dh, int normalize)
{
    /* invertAffineTransform of diag(scale) (imgwarp.cpp) */
    double D = scale * scale;
    D = D != 0 ? 1. / D : 0;
    const double m = scale * D;
    const int cubic = scale > 1.;
    const int k = cubic ? 4 : 2;
    static short tabs[2][(INTER_TAB * INTER_TAB + 1) * 16];   /* + the correction window's overrun */
    static int ready[2];
    if (!ready[cubic]) {
        orc_warp_tab(cubic, tabs[cubic]);
        ready[cubic] = 1;
    }
    const short* wtab = tabs[cubic];
    for (int y = 0; y < dh; ++y) {
        int sy, fy;
        warp_coord(m, y, &sy, &fy);
        for (int x = 0; x < dw; ++x) {
            int sx, fx;
            warp_coord(m, x, &sx, &fx);
            const short* w = wtab + (fy * INTER_TAB + fx) * k * k;
            const int ox = cubic ? sx - 1 : sx, oy = cubic ? sy - 1 : sy;
            for (int c = 0; c < 3; ++c) {
                int sum = 0;
                for (int ky = 0; ky < k; ++ky)
                    for (int kx = 0; kx < k; ++kx) {
                        const int yy = oy + ky, xx = ox + kx;
                        const int v = (yy >= 0 && yy < sh && xx >= 0 && xx < sw)
                                          ? src[((size_t)yy * sw + xx) * 3 + c] : 0;
                        sum += v * w[ky * k + kx];
                    }
                int u = (sum + (1 << 14)) >> 15;
                u = u < 0 ? 0 : u > 255 ? 255 : u;
                float f = (float)u;
                if (normalize) f = f * (1 / 256.f) - 0.5f;   /* exact: u / 256 - 0.5 */
                dst[((size_t)c * dh + y) * dw + x] = f;
            }
        }
    }
}

/*
 * cv::warpAffine(src, dst, M, {dw, dh}, INTER_LINEAR | WARP_INVERSE_MAP, BORDER_CONSTANT 0) for a
 * BGR uint8 image, then uCharCvMatToFloatPtr: the crop of FaceExtractorCaffe::forwardPass
 * (faceExtractorCaffe.cpp:215-232) and of the hand extractor's cropFrame
 * (handExtractorCaffe.cpp:44-73).  M is used as given (inverse map), with OpenCV's full per-pixel
 * arithmetic for any affine M:
 *   X = (cvRound((M01*y + M02)*1024) + 16 + cvRound(M00*x*1024)) >> 5
 *   Y = (cvRound((M11*y + M12)*1024) + 16 + cvRound(M10*x*1024)) >> 5
 * source tap (X >> 5, Y >> 5), weights of entry (Y & 31) * 32 + (X & 31).
 */
void orc_warp_affine_inv(float* dst, const uint8_t* src, int sw, int sh, const double* M, int dw,
                         int dh, int normalize)
{
    static short tab[(INTER_TAB * INTER_TAB + 1) * 4];
    static int ready;
    if (!ready) {
        orc_warp_tab(0, tab);
        ready = 1;
    }
    const int rd = AB_SCALE / INTER_TAB / 2;
    for (int y = 0; y < dh; ++y) {
        const int X0 = round_d((M[1] * y + M[2]) * AB_SCALE) + rd;
        const int Y0 = round_d((M[4] * y + M[5]) * AB_SCALE) + rd;
        for (int x = 0; x < dw; ++x) {
            const int X = (X0 + round_d(M[0] * x * AB_SCALE)) >> (AB_BITS - INTER_BITS);
            const int Y = (Y0 + round_d(M[3] * x * AB_SCALE)) >> (AB_BITS - INTER_BITS);
            const int sx = X >> INTER_BITS, sy = Y >> INTER_BITS;
            const short* w = tab + ((Y & (INTER_TAB - 1)) * INTER_TAB + (X & (INTER_TAB - 1))) * 4;
            for (int c = 0; c < 3; ++c) {
                int sum = 0;
                for (int ky = 0; ky < 2; ++ky)
                    for (int kx = 0; kx < 2; ++kx) {
                        const int yy = sy + ky, xx = sx + kx;
                        const int v = (yy >= 0 && yy < sh && xx >= 0 && xx < sw)
                                          ? src[((size_t)yy * sw + xx) * 3 + c] : 0;
                        sum += v * w[ky * 2 + kx];
                    }
                int u = (sum + (1 << 14)) >> 15;
                u = u < 0 ? 0 : u > 255 ? 255 : u;
                float f = (float)u;
                if (normalize) f = f * (1 / 256.f) - 0.5f;
                dst[((size_t)c * dh + y) * dw + x] = f;
            }
        }
    }
}
