/*
 * render.c -- CPU oracle of the GPU renderers (TEST INFRASTRUCTURE, see oracle.h).
 *
 * A per-pixel restatement of the reference's render kernels, loop for loop:
 *   orc_render_keypoints: renderKeypointsOld (include/openpose_private/utilities/render.hu:209-383)
 *     -- and renderKeypoints (:61-207), which differs only in reading the boxes getBoundingBoxPerPerson
 *     (:6-59) stored -- for pose (renderPose.cu:129-417), face (renderFace.cu:21-46) and hand
 *     (renderHand.cu:21-46): per pixel, per person whose box holds the pixel, every limb's ellipse
 *     test (atan2f / sinf / cosf evaluated per pixel, as the kernel does), then every part's circle
 *     (googly eyes included), each hit blended with addColorWeighted (cuda.hu:188-201).
 *     `ambiguous` (optional, [h][w]) marks pixels where some limb's judge lies within 1e-4 of the
 *     boundary 1: there the libm / device-library ulp differences of atan2f, sinf, cosf can flip
 *     the decision, so tests compare those pixels loosely (parity unpinned there).
 *     A person whose box maximum is exactly 0 gets the scale its box gives (the reference leaves
 *     the shared scale unset then); every other value is the reference's.
 *   orc_render_heat_map: renderBodyPartHeatMap (renderPose.cu:454-480) with getColorHeatMap
 *     (:44-80) and bicubicInterpolate (cuda.hu:125-145, orc_cuda_bicubic in resize.c);
 *   orc_render_heat_maps: renderBodyPartHeatMaps (:419-452), nearest sample, given colors;
 *   orc_render_pafs: renderPartAffinities (:482-527) with getColorXYAffinity / getColorAffinity
 *     (:82-119).
 * Frames are float BGR [h][w][3].  Compiled with -ffp-contract=off: every operation rounds.
 */
#include <math.h>
#include <stddef.h>

#include "oracle.h"

static float truncf_ref(float v, float lo, float hi)
{
    /* fastTruncateCuda = fastMinCuda(hi, fastMaxCuda(lo, v)) (cuda.hu:72-88) */
    const float m = lo > v ? lo : v;
    return hi < m ? hi : m;
}

static float add_weighted(float v1, float v2, float alpha)
{
    return (1.f - alpha) * v1 + alpha * v2;
}

void orc_render_keypoints(float* frame, int w, int h, const float* kp, int people, int parts,
                          const unsigned* pairs, int npairs, const float* colors, int ncolors,
                          const float* scales, int nscales, float radius, float line_width,
                          float threshold, float alpha, int blend, int eye1, int eye2,
                          unsigned char* ambiguous)
{
    float boxes[ORC_RENDER_MAX_PEOPLE][5];
    for (int p = 0; p < people && p < ORC_RENDER_MAX_PEOPLE; ++p) {
        float minx = (float)w, miny = (float)h, maxx = 0.f, maxy = 0.f;
        for (int i = 0; i < parts; ++i) {
            const float* k = kp + 3 * ((long)p * parts + i);
            if (k[2] > threshold) {
                if (k[0] < minx) minx = k[0];
                if (k[0] > maxx) maxx = k[0];
                if (k[1] < miny) miny = k[1];
                if (k[1] > maxy) maxy = k[1];
            }
        }
        const float averageX = maxx - minx, averageY = maxy - miny;
        boxes[p][4] = truncf_ref((averageX + averageY) / 400.f, 0.33f, 1.f);
        if (maxx != 0.f && maxy != 0.f) {
            maxx += 50.f;
            maxy += 50.f;
            minx -= 50.f;
            miny -= 50.f;
        }
        boxes[p][0] = minx;
        boxes[p][1] = miny;
        boxes[p][2] = maxx;
        boxes[p][3] = maxy;
    }
    const float lineWidthSquared = line_width * line_width;
    const float radiusSquared = radius * radius;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            float* px = frame + 3 * ((long)y * w + x);
            float b = px[0], g = px[1], r = px[2];
            unsigned char amb = 0;
            if (!blend) b = g = r = 0.f;
            for (int p = 0; p < people; ++p) {
                const float* B = boxes[p];
                if (!(x <= B[2] && x >= B[0] && y <= B[3] && y >= B[1])) continue;
                const float s = B[4];
                const float* K = kp + 3 * (long)p * parts;
                for (int j = 0; j < npairs; ++j) {
                    const unsigned pa = pairs[2 * j], pb = pairs[2 * j + 1];
                    const float xA = K[3 * pa], yA = K[3 * pa + 1], scoreA = K[3 * pa + 2];
                    const float xB = K[3 * pb], yB = K[3 * pb + 1], scoreB = K[3 * pb + 2];
                    if (!(scoreA > threshold && scoreB > threshold)) continue;
                    const float ks = scales[pb % nscales] * scales[pb % nscales] *
                                     scales[pb % nscales];
                    const float lineWidthScaled = lineWidthSquared * ks;
                    const float bSqrt = s * s * lineWidthScaled;
                    const float xP = (xA + xB) / 2.f, yP = (yA + yB) / 2.f;
                    const float aSqrt = (xA - xP) * (xA - xP) + (yA - yP) * (yA - yP);
                    const float angle = atan2f(yB - yA, xB - xA);
                    const float sine = sinf(angle), cosine = cosf(angle);
                    const float A = cosine * (x - xP) + sine * (y - yP);
                    const float Bq = sine * (x - xP) - cosine * (y - yP);
                    const float judge = A * A / aSqrt + Bq * Bq / bSqrt;
                    if (fabsf(judge - 1.f) <= 1e-4f) amb = 1;
                    if (0.f <= judge && judge <= 1.f) {
                        const float* c = colors + (pb % ncolors) * 3;
                        r = add_weighted(r, c[0], alpha);
                        g = add_weighted(g, c[1], alpha);
                        b = add_weighted(b, c[2], alpha);
                    }
                }
                for (int i = 0; i < parts; ++i) {
                    const float lx = K[3 * i], ly = K[3 * i + 1], score = K[3 * i + 2];
                    if (!(score > threshold)) continue;
                    const float ks = scales[i % nscales] * scales[i % nscales] * scales[i % nscales];
                    const float radiusScaled = radiusSquared * ks;
                    const float dist2 = (x - lx) * (x - lx) + (y - ly) * (y - ly);
                    if (i == eye1 || i == eye2) {
                        const float eyeRatio = 2.5f * sqrtf(radiusScaled);
                        const float minr2 = s * s * (eyeRatio - 2) * (eyeRatio - 2);
                        const float maxr2 = s * s * eyeRatio * eyeRatio;
                        if (dist2 <= maxr2) {
                            float v = 0.f;
                            if (dist2 <= minr2) v = 255.f;
                            if (dist2 <= minr2 * 0.6f) {
                                const float dist3 = (x - 4 - lx) * (x - 4 - lx) +
                                                    (y - ly + 4) * (y - ly + 4);
                                if (dist3 > 14.0625f) v = 0.f;
                            }
                            r = add_weighted(r, v, 0.9f);
                            g = add_weighted(g, v, 0.9f);
                            b = add_weighted(b, v, 0.9f);
                        }
                    } else {
                        const float maxr2 = s * s * radiusScaled;
                        if (0.f <= dist2 && dist2 <= maxr2) {
                            const float* c = colors + (i % ncolors) * 3;
                            r = add_weighted(r, c[0], alpha);
                            g = add_weighted(g, c[1], alpha);
                            b = add_weighted(b, c[2], alpha);
                        }
                    }
                }
            }
            px[0] = b;
            px[1] = g;
            px[2] = r;
            if (ambiguous) ambiguous[(long)y * w + x] = amb;
        }
}

static void color_heat(float* c, float v)
{
    const float vmin = 0.f, vmax = 1.f;
    const float t = truncf_ref(v, vmin, vmax);
    const float dv = vmax - vmin;
    if (t < (vmin + 0.125f * dv)) {
        c[0] = 256.f * (0.5f + (t * 4.f));
        c[1] = 0.f;
        c[2] = 0.f;
    } else if (t < (vmin + 0.375f * dv)) {
        c[0] = 255.f;
        c[1] = 256.f * (t - 0.125f) * 4.f;
        c[2] = 0.f;
    } else if (t < (vmin + 0.625f * dv)) {
        c[0] = 256.f * (-4.f * t + 2.5f);
        c[1] = 255.f;
        c[2] = 256.f * (4.f * (t - 0.375f));
    } else if (t < (vmin + 0.875f * dv)) {
        c[0] = 0.f;
        c[1] = 256.f * (-4.f * t + 3.5f);
        c[2] = 255.f;
    } else {
        c[0] = 0.f;
        c[1] = 0.f;
        c[2] = 256.f * (-4.f * t + 4.5f);
    }
}

static void blend_bgr(float* px, const float* c, float alpha)
{
    px[2] = add_weighted(px[2], c[0], alpha);
    px[1] = add_weighted(px[1], c[1], alpha);
    px[0] = add_weighted(px[0], c[2], alpha);
}

void orc_render_heat_map(float* frame, int w, int h, const float* heat, int hw, int hh,
                         float scale, int part, float alpha, int abs_value)
{
    const float* plane = heat + (long)part * hw * hh;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const float xs = (x + 0.5f) / scale - 0.5f;
            const float ys = (y + 0.5f) / scale - 0.5f;
            const float v = orc_cuda_bicubic(plane, xs, ys, hw, hh);
            float c[3];
            color_heat(c, abs_value ? fabsf(v) : v);
            blend_bgr(frame + 3 * ((long)y * w + x), c, alpha);
        }
}

void orc_render_heat_maps(float* frame, int w, int h, const float* heat, int hw, int hh,
                          float scale, int parts, const float* colors, int ncolors, float alpha)
{
    const long area = (long)hw * hh, last = area * parts - 1;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const float xs = (x + 0.5f) / scale - 0.5f;
            const float ys = (y + 0.5f) / scale - 0.5f;
            int xh = (int)(xs + 1e-5), yh = (int)(ys + 1e-5);   /* double add, as written */
            xh = xh > hw ? hw : (xh < 0 ? 0 : xh);
            yh = yh > hh ? hh : (yh < 0 ? 0 : yh);
            float c[3] = {0.f, 0.f, 0.f};
            for (int p = 0; p < parts; ++p) {
                long idx = p * area + (long)yh * hw + xh;
                if (idx > last) idx = last;   /* past the stack: see render.hip */
                float v = heat[idx];
                v = v != v ? 0.f : (v < 0.f ? 0.f : (v > 1.f ? 1.f : v));   /* __saturatef */
                const float* col = colors + (p % ncolors) * 3;
                c[0] += v * col[0];
                c[1] += v * col[1];
                c[2] += v * col[2];
            }
            blend_bgr(frame + 3 * ((long)y * w + x), c, alpha);
        }
}

static void color_xy_affinity(float* c, float x, float y)
{
    const float PI = 3.14159265358979323846f;
    const float len = sqrtf(x * x + y * y);
    const float rad = 1.f < len ? 1.f : len;
    const float a = atan2f(-y, -x) / PI;
    float fk = (a + 1.f) / 2.f;
    if (isnan(fk)) fk = 0.f;
    const int RY = 15, YG = 6, GC = 4, CB = 11, BM = 13, MR = 6;
    const int summed = RY + YG + GC + CB + BM + MR;
    const float v = truncf_ref(fk, 0.f, 1.f) * summed;
    if (v < RY) {
        c[0] = 255.f; c[1] = 255.f * (v / (RY)); c[2] = 0.f;
    } else if (v < RY + YG) {
        c[0] = 255.f * (1 - ((v - RY) / (YG))); c[1] = 255.f; c[2] = 0.f;
    } else if (v < RY + YG + GC) {
        c[0] = 0.f * (1 - ((v - RY) / (YG))); c[1] = 255.f; c[2] = 255.f * ((v - RY - YG) / (GC));
    } else if (v < RY + YG + GC + CB) {
        c[0] = 0.f; c[1] = 255.f * (1 - ((v - RY - YG - GC) / (CB))); c[2] = 255.f;
    } else if (v < summed - MR) {
        c[0] = 255.f * ((v - RY - YG - GC - CB) / (BM)); c[1] = 0.f; c[2] = 255.f;
    } else if (v < summed) {
        c[0] = 255.f; c[1] = 0.f; c[2] = 255.f * (1 - ((v - RY - YG - GC - CB - BM) / (MR)));
    } else {
        c[0] = 255.f; c[1] = 0.f; c[2] = 0.f;
    }
    c[0] *= rad;
    c[1] *= rad;
    c[2] *= rad;
}

void orc_render_pafs(float* frame, int w, int h, const float* heat, int hw, int hh, float scale,
                     int first, int count, float alpha)
{
    const long area = (long)hw * hh;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            const float xs = (x + 0.5f) / scale - 0.5f;
            const float ys = (y + 0.5f) / scale - 0.5f;
            float c[3] = {0.f, 0.f, 0.f};
            for (int part = first; part < first + count * 2; part += 2) {
                /* cubicSequentialData's base pixel and its right / lower neighbours */
                int x1 = (int)floorf(xs), y1 = (int)floorf(ys);
                x1 = x1 < 0 ? 0 : (x1 > hw - 1 ? hw - 1 : x1);
                y1 = y1 < 0 ? 0 : (y1 > hh - 1 ? hh - 1 : y1);
                const int x2 = hw - 1 < x1 + 1 ? hw - 1 : x1 + 1;
                const int y2 = hh - 1 < y1 + 1 ? hh - 1 : y1 + 1;
                const float dx = xs - x1, dy = ys - y1;
                const float* X = heat + part * area;
                const float* Y = heat + (part + 1) * area;
                float vx = X[(long)y1 * hw + x1], vy = Y[(long)y1 * hw + x1];
                if (count == 1) {
                    const float xB = X[(long)y1 * hw + x2], xC = X[(long)y2 * hw + x1],
                                xD = X[(long)y2 * hw + x2];
                    vx = (1 - dx) * (1 - dy) * vx + dx * (1 - dy) * xB + (1 - dx) * dy * xC +
                         dx * dy * xD;
                    const float yB = Y[(long)y1 * hw + x2], yC = Y[(long)y2 * hw + x1],
                                yD = Y[(long)y2 * hw + x2];
                    vy = (1 - dx) * (1 - dy) * vy + dx * (1 - dy) * yB + (1 - dx) * dy * yC +
                         dx * dy * yD;
                }
                float c2[3];
                color_xy_affinity(c2, vx, vy);
                c[0] += c2[0];
                c[1] += c2[1];
                c[2] += c2[2];
            }
            blend_bgr(frame + 3 * ((long)y * w + x), c, alpha);
        }
}
