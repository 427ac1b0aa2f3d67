/*
 * caffe_cpu.c -- CPU oracle: Caffe layer semantics used by the BODY_25 prototxt
 * (TEST INFRASTRUCTURE + the timed CPU baseline, see oracle.h).
 *
 * Reference: the network is models/pose/body_25/pose_deploy.prototxt, run by Caffe
 * (3rdparty/caffe, CMU fork pinned at 1807aad, CMakeLists.txt:728,732; absent from the image)
 * through op::NetCaffe::forwardPass (src/openpose/net/netCaffe.cpp:212-261).  Restated layer
 * semantics (Caffe CPU): ConvolutionLayer = im2col + SGEMM (cross-correlation, zero pad, stride 1,
 * bias added after the product); PReLULayer per channel; ReLULayer; PoolingLayer MAX with ceil
 * output sizing and the window clipped to the image.  Parity with Caffe: unpinned (no Caffe here);
 * cross-checked against torch CPU fp32 in tests/test_oracle_cnn.py.
 *
 * The GEMM is blocked per 64-pixel tile (im2col of one tile at a time) and parallelised with
 * OpenMP; this file is built with -O3 -mavx2 -mfma (the only oracle file allowed to contract).
 */
#include <float.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define TILE 64

typedef float v8 __attribute__((vector_size(32)));

static void conv_tile(float* out, const float* in, const float* w, const float* bias, int ci,
                      int h, int wd, int co, int k, int pad, long p0, int np, float* col)
{
    const int K = ci * k * k;
    const long hw = (long)h * wd;
    /* im2col of pixels [p0, p0+np) into col[K][TILE] (zero padded) */
    for (int c = 0; c < ci; ++c)
        for (int ky = 0; ky < k; ++ky)
            for (int kx = 0; kx < k; ++kx) {
                float* row = col + (long)((c * k + ky) * k + kx) * TILE;
                for (int t = 0; t < TILE; ++t) {
                    float v = 0.f;
                    if (t < np) {
                        const long p = p0 + t;
                        const int y = (int)(p / wd) + ky - pad, x = (int)(p % wd) + kx - pad;
                        if (y >= 0 && y < h && x >= 0 && x < wd) v = in[(long)c * hw + (long)y * wd + x];
                    }
                    row[t] = v;
                }
            }
    int o = 0;
    for (; o + 4 <= co; o += 4) {
        const float* w0 = w + (long)o * K;
        for (int t0 = 0; t0 < TILE; t0 += 16) {
            v8 a[4][2];
            memset(a, 0, sizeof(a));
            for (int kk = 0; kk < K; ++kk) {
                v8 c0, c1;
                memcpy(&c0, col + (long)kk * TILE + t0, 32);
                memcpy(&c1, col + (long)kk * TILE + t0 + 8, 32);
                for (int r = 0; r < 4; ++r) {
                    const float s = w0[(long)r * K + kk];
                    a[r][0] += s * c0;
                    a[r][1] += s * c1;
                }
            }
            for (int r = 0; r < 4; ++r) {
                float tmp[16];
                memcpy(tmp, &a[r][0], 32);
                memcpy(tmp + 8, &a[r][1], 32);
                const float b = bias ? bias[o + r] : 0.f;
                for (int t = 0; t < 16 && t0 + t < np; ++t)
                    out[(long)(o + r) * hw + p0 + t0 + t] = tmp[t] + b;
            }
        }
    }
    for (; o < co; ++o) {
        const float* wr = w + (long)o * K;
        for (int t = 0; t < np; ++t) {
            float s = 0.f;
            for (int kk = 0; kk < K; ++kk) s += wr[kk] * col[(long)kk * TILE + t];
            out[(long)o * hw + p0 + t] = s + (bias ? bias[o] : 0.f);
        }
    }
}

void orc_conv2d(float* out, const float* in, const float* w, const float* bias, int n, int ci,
                int h, int wd, int co, int k, int pad, int nthreads)
{
    const long hw = (long)h * wd;
    const long tiles = (hw + TILE - 1) / TILE;
    const long K = (long)ci * k * k;
    if (nthreads <= 0) nthreads = 1;
    for (int b = 0; b < n; ++b) {
        const float* src = in + (long)b * ci * hw;
        float* dst = out + (long)b * co * hw;
        #pragma omp parallel num_threads(nthreads)
        {
            float* col = (float*)aligned_alloc(64, sizeof(float) * K * TILE);
            #pragma omp for schedule(dynamic, 4)
            for (long t = 0; t < tiles; ++t) {
                const long p0 = t * TILE;
                const int np = (int)((hw - p0) < TILE ? (hw - p0) : TILE);
                conv_tile(dst, src, w, bias, ci, h, wd, co, k, pad, p0, np, col);
            }
            free(col);
        }
    }
}

void orc_prelu(float* x, const float* slope, int n, int c, int hw)
{
    for (int b = 0; b < n; ++b)
        for (int ch = 0; ch < c; ++ch) {
            float* p = x + ((long)b * c + ch) * hw;
            const float s = slope[ch];
            for (int i = 0; i < hw; ++i) p[i] = p[i] > 0.f ? p[i] : p[i] * s;
        }
}

void orc_relu(float* x, long count)
{
    for (long i = 0; i < count; ++i) x[i] = x[i] > 0.f ? x[i] : 0.f;
}

void orc_maxpool(float* out, const float* in, int n, int c, int h, int w, int k, int s,
                 int oh, int ow)
{
    for (long pl = 0; pl < (long)n * c; ++pl) {
        const float* src = in + pl * h * w;
        float* dst = out + pl * oh * ow;
        for (int y = 0; y < oh; ++y)
            for (int x = 0; x < ow; ++x) {
                const int y0 = y * s, x0 = x * s;
                const int y1 = y0 + k < h ? y0 + k : h, x1 = x0 + k < w ? x0 + k : w;
                float m = -FLT_MAX;
                for (int yy = y0; yy < y1; ++yy)
                    for (int xx = x0; xx < x1; ++xx)
                        if (src[yy * w + xx] > m) m = src[yy * w + xx];
                dst[y * ow + x] = m;
            }
    }
}
