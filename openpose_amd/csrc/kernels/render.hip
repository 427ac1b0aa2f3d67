// render.hip -- the GPU renderers of pose / face / hand keypoints and of heat maps, on gfx950.
//
// Keypoints: renderKeypointsOld / renderKeypoints (include/openpose_private/utilities/render.hu:61-383)
// as launched by renderPoseKeypointsGpu (src/openpose/pose/renderPose.cu:609-748),
// renderFaceKeypointsGpu (src/openpose/face/renderFace.cu:48-76) and renderHandKeypointsGpu
// (src/openpose/hand/renderHand.cu:48-76).  The reference evaluates, for every pixel of the frame,
// each person's box test and every limb's atan2f / sinf / cosf.  Here:
//   1. render_prep_kernel (one wave per person): the person's box and scale
//      (getBoundingBoxPerPerson, render.hu:6-59) and, per limb and per part, everything that does not
//      depend on the pixel -- limb centre, cos / sin of its angle, the ellipse's aSqrt / bSqrt, the
//      circle radii -- with the reference's expressions, in its operation order;
//   2. render_keypoints_kernel (one 32x8 pixel tile per workgroup): the people whose box meets the
//      tile are compacted in order into LDS (wave ballots); then, in rounds of 256, their limbs and
//      part circles -- person-major, limbs before circles, the reference's draw order -- are culled
//      against the tile (a limb survives if the tile reaches its squared-distance bound
//      1.01 * (aSqrt + bSqrt) + 4, beyond which the ellipse test cannot pass since
//      judge >= dist^2 / (aSqrt + bSqrt); a circle if the tile reaches its radius) and the survivors'
//      records staged in LDS; each pixel then runs the reference's per-pixel tests on those only and
//      blends with addColorWeighted (cuda.hu:188-201).
// The frame is the reference's float BGR [h][w][3]; each pixel is read and written once: the
// kernel is bound by those 24 bytes per pixel (HBM) plus the per-person ALU work.
//
// Heat maps: renderBodyPartHeatMap (bicubic + getColorHeatMap), renderBodyPartHeatMaps (nearest,
// COCO colors) and renderPartAffinities (getColorXYAffinity) of renderPose.cu:44-119,419-527,
// one pixel per lane.
//
// Arithmetic is the reference's expression by expression with every mul / add rounded separately
// (the library builds with -ffp-contract=off); atan2f / sinf / cosf are the device library's, so
// pixels on an ellipse boundary (|judge - 1| ~ 1e-6) and PAF colours (~1e-4 of 255) can differ
// from the CUDA build's: that part of render parity is unpinned.
#include "kernels.h"
#include "heat_dev.h"
#include "../common.h"

namespace opk {

namespace {

constexpr int kTileW = 32, kTileH = 8;
// float(pi) as renderPose.cu:10's __constant__ PI rounds
constexpr float kPi = 3.14159265358979323846f;

// fastTruncateCuda (cuda.hu:84-88): fastMin(hi, fastMax(lo, v)) with its NaN behaviour
__device__ __forceinline__ float truncate_ref(float v, float lo, float hi)
{
    const float m = lo > v ? lo : v;
    return hi < m ? hi : m;
}

__device__ __forceinline__ void blend(float& r, float& g, float& b, float cr, float cg, float cb,
                                      float alpha)
{
    // addWeighted: (1 - alpha) * value1 + alpha * value2
    r = (1.f - alpha) * r + alpha * cr;
    g = (1.f - alpha) * g + alpha * cg;
    b = (1.f - alpha) * b + alpha * cb;
}

// one wave per person: box (a lane-strided scan + wave reduction; min / max do not depend on the
// order), then lanes take limbs and parts
__global__ __launch_bounds__(64) void render_prep_kernel(RenderKeypointsArgs a)
{
    const int p = blockIdx.x, lane = threadIdx.x;
    const float* kp = a.kp + (size_t)p * a.parts * 3;
    float* box = a.geom + (size_t)p * 8;
    float* limb = a.geom + (size_t)a.people * 8 + (size_t)p * a.npairs * 8;
    float* part = a.geom + (size_t)a.people * 8 + (size_t)a.people * a.npairs * 8 +
                  (size_t)p * a.parts * 8;
    // getBoundingBoxPerPerson (render.hu:6-59 / 219-260)
    float minx = (float)a.w, miny = (float)a.h, maxx = 0.f, maxy = 0.f;
    for (int i = lane; i < a.parts; i += 64) {
        const float x = kp[3 * i], y = kp[3 * i + 1], s = kp[3 * i + 2];
        if (s > a.threshold) {
            if (x < minx) minx = x;
            if (x > maxx) maxx = x;
            if (y < miny) miny = y;
            if (y > maxy) maxy = y;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float a0 = __shfl_xor(minx, o), a1 = __shfl_xor(miny, o);
        const float a2 = __shfl_xor(maxx, o), a3 = __shfl_xor(maxy, o);
        minx = a0 < minx ? a0 : minx;
        miny = a1 < miny ? a1 : miny;
        maxx = a2 > maxx ? a2 : maxx;
        maxy = a3 > maxy ? a3 : maxy;
    }
    // the box's own scale; the reference leaves it unset when a coordinate maximum is exactly 0
    // (then only the box test decides, which rejects every pixel of an empty person)
    const float scale = truncate_ref(((maxx - minx) + (maxy - miny)) / 400.f, 0.33f, 1.f);
    if (maxx != 0.f && maxy != 0.f) {
        maxx += 50.f;
        maxy += 50.f;
        minx -= 50.f;
        miny -= 50.f;
    }
    if (lane == 0) {
        box[0] = minx;
        box[1] = miny;
        box[2] = maxx;
        box[3] = maxy;
        box[4] = scale;
    }
    const float s2 = scale * scale;
    const float lw2 = a.line_width * a.line_width;
    const float r2 = a.radius * a.radius;
    // limbs (render.hu:288-326)
    for (int j = lane; j < a.npairs; j += 64) {
        const unsigned pa = a.pairs[2 * j], pb = a.pairs[2 * j + 1];
        const float xA = kp[3 * pa], yA = kp[3 * pa + 1], sA = kp[3 * pa + 2];
        const float xB = kp[3 * pb], yB = kp[3 * pb + 1], sB = kp[3 * pb + 2];
        float* L = limb + (size_t)j * 8;
        if (sA > a.threshold && sB > a.threshold) {
            const float k = a.scales[pb % a.nscales];
            const float ks = k * k * k;
            const float bSqrt = s2 * (lw2 * ks);
            const float xP = (xA + xB) / 2.f, yP = (yA + yB) / 2.f;
            const float aSqrt = (xA - xP) * (xA - xP) + (yA - yP) * (yA - yP);
            const float angle = atan2f(yB - yA, xB - xA);
            L[0] = xP;
            L[1] = yP;
            L[2] = cosf(angle);
            L[3] = sinf(angle);
            L[4] = aSqrt;
            L[5] = bSqrt;
            L[6] = 1.01f * (aSqrt + bSqrt) + 4.f;   // squared-distance bound of the ellipse
            L[7] = (float)((pb % a.ncolors) * 3);
        } else {
            L[6] = -1.f;   // a score at or below the threshold: never drawn
        }
    }
    // part circles (render.hu:329-377)
    for (int i = lane; i < a.parts; i += 64) {
        float* C = part + (size_t)i * 8;
        const float x = kp[3 * i], y = kp[3 * i + 1], s = kp[3 * i + 2];
        if (!(s > a.threshold)) {
            C[4] = 0.f;
            continue;
        }
        const float k = a.scales[i % a.nscales];
        const float radiusScaled = r2 * (k * k * k);
        C[0] = x;
        C[1] = y;
        if (i == a.eye1 || i == a.eye2) {
            const float eyeRatio = 2.5f * sqrtf(radiusScaled);
            C[2] = s2 * eyeRatio * eyeRatio;                  // maxr2
            C[3] = s2 * (eyeRatio - 2) * (eyeRatio - 2);      // minr2
            C[4] = 2.f;
        } else {
            C[2] = s2 * radiusScaled;
            C[3] = 0.f;
            C[4] = 1.f;
        }
        C[5] = (float)((i % a.ncolors) * 3);
    }
}

// squared distance from (cx, cy) to the tile's pixel rectangle, with the per-pixel test's own
// operations at its nearest pixel: never above any pixel's dist^2 (rounding is monotonic)
__device__ __forceinline__ float rect_d2(float cx, float cy, float fx0, float fy0, float fx1,
                                         float fy1)
{
    const float dx = cx < fx0 ? fx0 - cx : (cx > fx1 ? cx - fx1 : 0.f);
    const float dy = cy < fy0 ? fy0 - cy : (cy > fy1 ? cy - fy1 : 0.f);
    return dx * dx + dy * dy;
}

// ordered compaction of one 256-candidate round: returns this thread's slot (or -1) and the
// round's total; wcount is the block's 4-entry scratch
__device__ __forceinline__ int compact(bool hit, int* wcount, int* total)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long m = __ballot(hit);
    if (lane == 0) wcount[wave] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
    for (int i = 0; i < 4; ++i) {
        off += i < wave ? wcount[i] : 0;
        tot += wcount[i];
    }
    *total = tot;
    return hit ? off + __popcll(m & ((1ull << lane) - 1ull)) : -1;
}

__global__ __launch_bounds__(256) void render_keypoints_kernel(RenderKeypointsArgs a)
{
    __shared__ unsigned short plist[kRenderMaxPeople];
    // one round's drawable items in draw order: {box}, {geometry}, {geometry, type, color}
    __shared__ float4 items[256][4];
    __shared__ int wcount[4];
    const int tx0 = blockIdx.x * kTileW, ty0 = blockIdx.y * kTileH;
    const float fx0 = (float)tx0, fy0 = (float)ty0;
    const float fx1 = (float)min(tx0 + kTileW - 1, a.w - 1), fy1 = (float)min(ty0 + kTileH - 1, a.h - 1);
    const float* __restrict__ boxes = a.geom;
    const float* __restrict__ limbs = a.geom + (size_t)a.people * 8;
    const float* __restrict__ circles = limbs + (size_t)a.people * a.npairs * 8;
    const float* __restrict__ colors = a.colors;

    // 1. the people whose box meets this tile, in person order
    int n = 0;
    for (int base = 0; base < a.people; base += 256) {
        const int p = base + threadIdx.x;
        bool hit = false;
        if (p < a.people) {
            const float* B = boxes + (size_t)p * 8;
            hit = B[2] >= fx0 && B[0] <= fx1 && B[3] >= fy0 && B[1] <= fy1;
        }
        int tot;
        const int slot = compact(hit, wcount, &tot);
        if (slot >= 0) plist[n + slot] = (unsigned short)p;
        __syncthreads();
        n += tot;
    }

    const int x = tx0 + (threadIdx.x & (kTileW - 1)), y = ty0 + threadIdx.x / kTileW;
    const bool inside = x < a.w && y < a.h;
    const size_t base = 3 * ((size_t)(inside ? y : 0) * a.w + (inside ? x : 0));
    float b = 0.f, g = 0.f, r = 0.f;
    if (inside && a.blend) {
        b = a.frame[base];
        g = a.frame[base + 1];
        r = a.frame[base + 2];
    }
    const float fx = (float)x, fy = (float)y;

    // 2. rounds of 256 (person, limb | part) candidates, person-major, limbs before parts (the
    //    reference's draw order); those whose ellipse bound / circle reaches the tile go to LDS
    const int per = a.npairs + a.parts;
    const int total = n * per;
    for (int k0 = 0; k0 < total; k0 += 256) {
        const int k = k0 + threadIdx.x;
        bool hit = false;
        float4 q0, q1, q2, q3;
        if (k < total) {
            const int s = k / per, j = k - s * per;
            const int p = plist[s];
            const float* B = boxes + (size_t)p * 8;
            q0 = make_float4(B[0], B[1], B[2], B[3]);
            if (j < a.npairs) {
                const float* L = limbs + ((size_t)p * a.npairs + j) * 8;
                const float rej = L[6];
                if (rej >= 0.f || rej != rej) {
                    hit = !(rect_d2(L[0], L[1], fx0, fy0, fx1, fy1) > rej);
                    q1 = make_float4(L[0], L[1], L[2], L[3]);
                    q2 = make_float4(L[4], L[5], rej, L[7]);
                    q3 = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            } else {
                const float* C = circles + ((size_t)p * a.parts + (j - a.npairs)) * 8;
                const float kind = C[4];
                if (kind != 0.f) {
                    hit = !(rect_d2(C[0], C[1], fx0, fy0, fx1, fy1) > C[2]);
                    q1 = make_float4(C[0], C[1], C[2], C[3]);
                    q2 = make_float4(0.f, 0.f, 0.f, C[5]);
                    q3 = make_float4(kind, 0.f, 0.f, 0.f);
                }
            }
        }
        int m;
        const int slot = compact(hit, wcount, &m);
        if (slot >= 0) {
            items[slot][0] = q0;
            items[slot][1] = q1;
            items[slot][2] = q2;
            items[slot][3] = q3;
        }
        __syncthreads();
        if (inside) {
            for (int i = 0; i < m; ++i) {
                const float4 B = items[i][0];
                if (!(fx <= B.z && fx >= B.x && fy <= B.w && fy >= B.y)) continue;
                const float4 G = items[i][1], H = items[i][2];
                const float type = items[i][3].x;
                const float dx = fx - G.x, dy = fy - G.y;
                const float d2 = dx * dx + dy * dy;
                if (type == 0.f) {   // limb (render.hu:301-325)
                    if (d2 > H.z) continue;
                    const float A = G.z * dx + G.w * dy;
                    const float Bq = G.w * dx - G.z * dy;
                    const float judge = A * A / H.x + Bq * Bq / H.y;
                    if (0.f <= judge && judge <= 1.f) {
                        const float* c = colors + (int)H.w;
                        blend(r, g, b, c[0], c[1], c[2], a.alpha);
                    }
                } else if (type == 2.f) {   // googly eye (render.hu:344-366)
                    if (d2 <= G.z) {
                        float v = 0.f;
                        if (d2 <= G.w) v = 255.f;
                        if (d2 <= G.w * 0.6f) {
                            const float ex = (float)(x - 4) - G.x, ey = fy - G.y + 4;
                            if (ex * ex + ey * ey > 14.0625f) v = 0.f;
                        }
                        blend(r, g, b, v, v, v, 0.9f);
                    }
                } else if (0.f <= d2 && d2 <= G.z) {   // part circle (render.hu:368-375)
                    const float* c = colors + (int)H.w;
                    blend(r, g, b, c[0], c[1], c[2], a.alpha);
                }
            }
        }
        __syncthreads();   // the next round rewrites items
    }
    if (inside) {
        a.frame[base] = b;
        a.frame[base + 1] = g;
        a.frame[base + 2] = r;
    }
}

// getColorHeatMap (renderPose.cu:44-80) with vmin 0, vmax 1
__device__ __forceinline__ void color_heat(float* c, float v)
{
    const float t = truncate_ref(v, 0.f, 1.f);
    if (t < 0.125f) {
        c[0] = 256.f * (0.5f + (t * 4.f));
        c[1] = 0.f;
        c[2] = 0.f;
    } else if (t < 0.375f) {
        c[0] = 255.f;
        c[1] = 256.f * (t - 0.125f) * 4.f;
        c[2] = 0.f;
    } else if (t < 0.625f) {
        c[0] = 256.f * (-4.f * t + 2.5f);
        c[1] = 255.f;
        c[2] = 256.f * (4.f * (t - 0.375f));
    } else if (t < 0.875f) {
        c[0] = 0.f;
        c[1] = 256.f * (-4.f * t + 3.5f);
        c[2] = 255.f;
    } else {
        c[0] = 0.f;
        c[1] = 0.f;
        c[2] = 256.f * (-4.f * t + 4.5f);
    }
}

// getColorAffinity (renderPose.cu:82-106) with vmin 0, vmax 1, then getColorXYAffinity's radius
__device__ __forceinline__ void color_xy_affinity(float* c, float x, float y)
{
    const float len = sqrtf(x * x + y * y);
    const float rad = 1.f < len ? 1.f : len;
    const float an = atan2f(-y, -x) / kPi;
    float fk = (an + 1.f) / 2.f;
    if (isnan(fk)) fk = 0.f;
    const float v = truncate_ref(fk, 0.f, 1.f) * 55;
    if (v < 15) {
        c[0] = 255.f; c[1] = 255.f * (v / 15); c[2] = 0.f;
    } else if (v < 15 + 6) {
        c[0] = 255.f * (1 - ((v - 15) / 6)); c[1] = 255.f; c[2] = 0.f;
    } else if (v < 15 + 6 + 4) {
        c[0] = 0.f * (1 - ((v - 15) / 6)); c[1] = 255.f; c[2] = 255.f * ((v - 15 - 6) / 4);
    } else if (v < 15 + 6 + 4 + 11) {
        c[0] = 0.f; c[1] = 255.f * (1 - ((v - 15 - 6 - 4) / 11)); c[2] = 255.f;
    } else if (v < 55 - 6) {
        c[0] = 255.f * ((v - 15 - 6 - 4 - 11) / 13); c[1] = 0.f; c[2] = 255.f;
    } else if (v < 55) {
        c[0] = 255.f; c[1] = 0.f; c[2] = 255.f * (1 - ((v - 15 - 6 - 4 - 11 - 13) / 6));
    } else {
        c[0] = 255.f; c[1] = 0.f; c[2] = 0.f;
    }
    c[0] *= rad;
    c[1] *= rad;
    c[2] *= rad;
}

__device__ __forceinline__ void blend_bgr(float* px, const float* c, float alpha)
{
    // addColorWeighted(target[+2], target[+1], target[+0], rgbColor, alpha)
    px[2] = (1.f - alpha) * px[2] + alpha * c[0];
    px[1] = (1.f - alpha) * px[1] + alpha * c[1];
    px[0] = (1.f - alpha) * px[0] + alpha * c[2];
}

// renderBodyPartHeatMap (renderPose.cu:454-480): one channel, bicubic, getColorHeatMap
__global__ __launch_bounds__(256) void render_heat_map_kernel(RenderHeatArgs a, int part, int absv)
{
    const int x = blockIdx.x * kTileW + (threadIdx.x & (kTileW - 1));
    const int y = blockIdx.y * kTileH + threadIdx.x / kTileW;
    if (x >= a.w || y >= a.h) return;
    const float xs = ((float)x + 0.5f) / a.scale - 0.5f;
    const float ys = ((float)y + 0.5f) / a.scale - 0.5f;
    const float v = cuda_bicubic(a.heat + (size_t)part * a.hw * a.hh, xs, ys, a.hw, a.hh);
    float c[3];
    color_heat(c, absv ? fabsf(v) : v);
    blend_bgr(a.frame + 3 * ((size_t)y * a.w + x), c, a.alpha);
}

// renderBodyPartHeatMaps (renderPose.cu:419-452): every part, nearest sample, COCO colors
__global__ __launch_bounds__(256) void render_heat_maps_kernel(RenderHeatArgs a, int parts,
                                                               const float* __restrict__ colors,
                                                               int ncolors)
{
    const int x = blockIdx.x * kTileW + (threadIdx.x & (kTileW - 1));
    const int y = blockIdx.y * kTileH + threadIdx.x / kTileW;
    if (x >= a.w || y >= a.h) return;
    const float xs = ((float)x + 0.5f) / a.scale - 0.5f;
    const float ys = ((float)y + 0.5f) / a.scale - 0.5f;
    // int(xSource + 1e-5): a double add; truncated into [0, width] (not width - 1)
    int xh = (int)((double)xs + 1e-5), yh = (int)((double)ys + 1e-5);
    xh = xh > a.hw ? a.hw : (xh < 0 ? 0 : xh);
    yh = yh > a.hh ? a.hh : (yh < 0 ? 0 : yh);
    const size_t area = (size_t)a.hw * a.hh;
    // the reference's index can pass the end of its last plane by up to width + 1 values (x or y
    // truncated to the size itself); those reads are clamped to the stack's last value
    const size_t last = area * parts - 1;
    float c[3] = {0.f, 0.f, 0.f};
    for (int p = 0; p < parts; ++p) {
        size_t idx = p * area + (size_t)yh * a.hw + xh;
        idx = idx > last ? last : idx;
        const float h = a.heat[idx];
        const float v = fminf(fmaxf(h, 0.f), 1.f);   // __saturatef (NaN -> 0)
        const float* col = colors + (p % ncolors) * 3;
        c[0] += v * col[0];
        c[1] += v * col[1];
        c[2] += v * col[2];
    }
    blend_bgr(a.frame + 3 * ((size_t)y * a.w + x), c, a.alpha);
}

// renderPartAffinities (renderPose.cu:482-527): `count` PAFs from channel `first`; one PAF is
// sampled bilinearly, several at the base pixel of cubicSequentialData
__global__ __launch_bounds__(256) void render_pafs_kernel(RenderHeatArgs a, int first, int count)
{
    const int x = blockIdx.x * kTileW + (threadIdx.x & (kTileW - 1));
    const int y = blockIdx.y * kTileH + threadIdx.x / kTileW;
    if (x >= a.w || y >= a.h) return;
    const float xs = ((float)x + 0.5f) / a.scale - 0.5f;
    const float ys = ((float)y + 0.5f) / a.scale - 0.5f;
    const int x1 = heat_clampi((int)floorf(xs), 0, a.hw - 1);
    const int x2 = min(a.hw - 1, x1 + 1);
    const float dx = xs - (float)x1;
    const int y1 = heat_clampi((int)floorf(ys), 0, a.hh - 1);
    const int y2 = min(a.hh - 1, y1 + 1);
    const float dy = ys - (float)y1;
    const size_t area = (size_t)a.hw * a.hh;
    float c[3] = {0.f, 0.f, 0.f};
    for (int part = first; part < first + count * 2; part += 2) {
        const float* X = a.heat + (size_t)part * area;
        const float* Y = X + area;
        float vx = X[(size_t)y1 * a.hw + x1], vy = Y[(size_t)y1 * a.hw + x1];
        if (count == 1) {
            const float xB = X[(size_t)y1 * a.hw + x2], xC = X[(size_t)y2 * a.hw + x1],
                        xD = X[(size_t)y2 * a.hw + x2];
            vx = (1 - dx) * (1 - dy) * vx + dx * (1 - dy) * xB + (1 - dx) * dy * xC + dx * dy * xD;
            const float yB = Y[(size_t)y1 * a.hw + x2], yC = Y[(size_t)y2 * a.hw + x1],
                        yD = Y[(size_t)y2 * a.hw + x2];
            vy = (1 - dx) * (1 - dy) * vy + dx * (1 - dy) * yB + (1 - dx) * dy * yC + dx * dy * yD;
        }
        float c2[3];
        color_xy_affinity(c2, vx, vy);
        c[0] += c2[0];
        c[1] += c2[1];
        c[2] += c2[2];
    }
    blend_bgr(a.frame + 3 * ((size_t)y * a.w + x), c, a.alpha);
}

dim3 tiles(int w, int h)
{
    return dim3((unsigned)((w + kTileW - 1) / kTileW), (unsigned)((h + kTileH - 1) / kTileH));
}

}  // namespace

size_t render_geom_floats(int people, int parts, int npairs)
{
    return (size_t)people * (8 + (size_t)npairs * 8 + (size_t)parts * 8);
}

void launch_render_keypoints(const RenderKeypointsArgs& a, hipStream_t stream)
{
    if (a.w <= 0 || a.h <= 0) return;
    if (a.people > 0) {
        render_prep_kernel<<<a.people, 64, 0, stream>>>(a);
        OPK_LAUNCH_CHECK();
    }
    render_keypoints_kernel<<<tiles(a.w, a.h), kTileW * kTileH, 0, stream>>>(a);
    OPK_LAUNCH_CHECK();
}

void launch_render_heat_map(const RenderHeatArgs& a, int part, bool abs_value, hipStream_t stream)
{
    if (a.w <= 0 || a.h <= 0) return;
    render_heat_map_kernel<<<tiles(a.w, a.h), kTileW * kTileH, 0, stream>>>(a, part, abs_value);
    OPK_LAUNCH_CHECK();
}

void launch_render_heat_maps(const RenderHeatArgs& a, int parts, const float* colors, int ncolors,
                             hipStream_t stream)
{
    if (a.w <= 0 || a.h <= 0) return;
    render_heat_maps_kernel<<<tiles(a.w, a.h), kTileW * kTileH, 0, stream>>>(a, parts, colors,
                                                                              ncolors);
    OPK_LAUNCH_CHECK();
}

void launch_render_pafs(const RenderHeatArgs& a, int first, int count, hipStream_t stream)
{
    if (a.w <= 0 || a.h <= 0) return;
    render_pafs_kernel<<<tiles(a.w, a.h), kTileW * kTileH, 0, stream>>>(a, first, count);
    OPK_LAUNCH_CHECK();
}

}  // namespace opk
