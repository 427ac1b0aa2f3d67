// input.cpp -- frame -> net input: ScaleAndSizeExtractor sizes, OpenCV warpAffine tables, launch.
//
// The reference prepares each frame on the CPU (op::CvMatToOpInput, cvMatToOpInput.cpp:63-98;
// its CUDA branch is disabled for -0.1% accuracy, :104-108).  Here the same integer arithmetic
// runs on the GPU: this file reproduces the parts of OpenCV's cv::warpAffine (third-party,
// imgwarp.cpp of OpenCV 4.2, generic non-IPP path) that decide which source pixels and which
// fixed-point weights every destination pixel uses; input.hip does the gather and the sums.
// Built with -ffp-contract=off: the tables must round exactly as the CPU build does.
#include "input.h"

#include <cmath>
#include <cstring>
#include <vector>

#include "../common.h"
#include "../kernels/kernels.h"
#include "context.h"

namespace opk {

namespace {
constexpr int kInterBits = 5, kInterTab = 1 << kInterBits;   // INTER_BITS, INTER_TAB_SIZE
constexpr int kAbBits = 10, kAbScale = 1 << kAbBits;         // AB_BITS = max(10, INTER_BITS)
constexpr int kCoefScale = 1 << 15;                          // INTER_REMAP_COEF_SCALE

int round_half_even(double v) { return (int)std::lrint(v); }   // cvRound(double)
int round_half_even(float v) { return (int)std::lrintf(v); }   // cvRound(float)

// positiveIntRound (include/openpose/utilities/fastMath.hpp:29-32): int(a + 0.5f) in a's type
int positive_round(float v) { return (int)(v + 0.5f); }
int positive_round(double v) { return (int)(v + 0.5f); }
}  // namespace

void scale_and_size(int in_w, int in_h, int net_w, int net_h, float dyn, int scale_number,
                    double scale_gap, double* scales, int* sizes)
{
    // scaleAndSizeExtractor.cpp:37-105
    OPK_CHECK_ARG(in_w > 0 && in_h > 0, "Wrong input element (empty cvInputData).");
    OPK_CHECK_ARG(scale_number >= 1, "scale_number must be >= 1");
    if (net_w <= 0 || net_h <= 0) {
        OPK_CHECK_ARG(net_w > 0 || net_h > 0,
                      "Only 1 of the dimensions of net input resolution can be <= 0.");
        if (dyn > 0) {
            if (net_w <= 0)
                net_w = 16 * positive_round(1 / 16.f * std::min(net_h * dyn * 16.f / 9.f,
                                                                 net_h * in_w / (float)in_h));
            else
                net_h = 16 * positive_round(1 / 16.f * std::min(net_w * dyn * 9.f / 16.f,
                                                                 net_w * in_h / (float)in_w));
        } else {
            if (net_w <= 0)
                net_w = 16 * positive_round(1 / 16.f * net_h * in_w / (float)in_h);
            else
                net_h = 16 * positive_round(1 / 16.f * net_w * in_h / (float)in_w);
        }
    }
    for (int i = 0; i < scale_number; ++i) {
        const double cur = 1. - i * scale_gap;
        OPK_CHECK_ARG(cur >= 0. && cur <= 1.,
                      "All scales must be in the range [0, 1], i.e., 0 <= 1-scale_number*scale_gap <= 1");
        const int tw = std::min(net_w, std::max(1, positive_round(net_w * cur) / 16 * 16));
        const int th = std::min(net_h, std::max(1, positive_round(net_h * cur) / 16 * 16));
        // resizeGetScaleFactor (openCv.cpp:182-195)
        const double rw = (tw - 1) / (double)(in_w - 1), rh = (th - 1) / (double)(in_h - 1);
        scales[i] = rw < rh ? rw : rh;
        sizes[2 * i] = tw;
        sizes[2 * i + 1] = th;
    }
}

void warp_weight_table(bool cubic, short* itab /* zeroed, (32*32 + 1) * k*k */)
{
    // initInterTab1D + initInterTab2D(method, fixpt = true)
    const int k = cubic ? 4 : 2;
    float t1[kInterTab * 4];
    for (int i = 0; i < kInterTab; ++i) {
        const float x = i * (1.f / kInterTab);
        float* c = t1 + i * k;
        if (cubic) {   // interpolateCubic, A = -0.75
            const float A = -0.75f;
            c[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
            c[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
            c[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
            c[3] = 1.f - c[0] - c[1] - c[2];
        } else {       // interpolateLinear
            c[0] = 1.f - x;
            c[1] = x;
        }
    }
    for (int i = 0; i < kInterTab; ++i)
        for (int j = 0; j < kInterTab; ++j) {
            short* w = itab + (i * kInterTab + j) * k * k;
            int isum = 0;
            for (int a = 0; a < k; ++a)
                for (int b = 0; b < k; ++b) {
                    const float v = t1[i * k + a] * t1[j * k + b];
                    const int r = round_half_even(v * kCoefScale);
                    w[a * k + b] = (short)std::min(32767, std::max(-32768, r));
                    isum += w[a * k + b];
                }
            if (isum == kCoefScale) continue;
            // make the weights sum to exactly 1.0: adjust the largest (sum too small) or the
            // smallest (sum too large) of the taps at [k/2, k/2 + 1]^2.  Reached only by the
            // fraction-0 entry (1.0 saturates to 32767); for k = 2 OpenCV's window runs past the
            // entry into the next, still zero one (the caller pads the table), so it adds the
            // missing unit to tap (1, 1): {32767, 0, 0, 1}, which rounds every pixel exactly as
            // {32768, 0, 0, 0} would
            const int diff = isum - kCoefScale, h = k / 2;
            int lo = h * k + h, hi = h * k + h;
            for (int a = h; a < h + 2; ++a)
                for (int b = h; b < h + 2; ++b) {
                    const int e = a * k + b;
                    if (w[e] < w[lo]) lo = e;
                    else if (w[e] > w[hi]) hi = e;
                }
            if (diff < 0) w[hi] = (short)(w[hi] - diff);
            else w[lo] = (short)(w[lo] - diff);
        }
}

void warp_axis_table(double scale, int d, bool cubic, int* tab)
{
    // warpAffine inverts M = diag(scale) (invertAffineTransform's arithmetic), then for every
    // destination index x: X = (X0 + adelta[x]) >> (AB_BITS - INTER_BITS) with
    // X0 = cvRound(0 * AB_SCALE) + round_delta, adelta[x] = cvRound(M00 * x * AB_SCALE);
    // source tap X >> INTER_BITS, fraction X & (INTER_TAB_SIZE - 1)
    double D = scale * scale;
    D = D != 0 ? 1. / D : 0;
    const double m = scale * D;
    const int x0 = round_half_even(0.0 * kAbScale) + kAbScale / kInterTab / 2;
    for (int x = 0; x < d; ++x) {
        const int X = (x0 + round_half_even(m * x * kAbScale)) >> (kAbBits - kInterBits);
        tab[2 * x] = (X >> kInterBits) - (cubic ? 1 : 0);   // first tap
        tab[2 * x + 1] = X & (kInterTab - 1);
    }
}

const short* Context::warp_weight_table(bool cubic)
{
    DevBuf& b = warp_weights[cubic ? 1 : 0];
    if (!b.ptr) {
        const int k = cubic ? 4 : 2;
        std::vector<short> host((size_t)(kInterTab * kInterTab + 1) * k * k);   // + window pad
        opk::warp_weight_table(cubic, host.data());
        const size_t bytes = (size_t)kInterTab * kInterTab * k * k * sizeof(short);
        b.get(bytes);
        OPK_HIP(hipMemcpyAsync(b.ptr, host.data(), bytes,
                               hipMemcpyHostToDevice, stream));
        OPK_HIP(hipStreamSynchronize(stream));
    }
    return static_cast<const short*>(b.ptr);
}

const Context::WarpAxes& Context::warp_axis_tables(double scale, int dw, int dh)
{
    uint64_t bits;
    std::memcpy(&bits, &scale, sizeof bits);
    const auto key = std::make_tuple(bits, dw, dh);
    auto it = warp_axes.find(key);
    if (it != warp_axes.end()) return *it->second;
    const bool cubic = scale > 1.;
    std::vector<int> host(2 * (size_t)(dw + dh));
    warp_axis_table(scale, dw, cubic, host.data());
    warp_axis_table(scale, dh, cubic, host.data() + 2 * dw);
    auto t = std::make_unique<WarpAxes>();
    int* dev = static_cast<int*>(t->buf.get(host.size() * sizeof(int)));
    OPK_HIP(hipMemcpyAsync(dev, host.data(), host.size() * sizeof(int), hipMemcpyHostToDevice,
                           stream));
    OPK_HIP(hipStreamSynchronize(stream));
    t->x = dev;
    t->y = dev + 2 * dw;
    auto& ref = *t;
    warp_axes.emplace(key, std::move(t));
    return ref;
}

void cvmat_to_input(Context* ctx, float* dst, const uint8_t* src, int n, int sw, int sh,
                    size_t step, double scale, int dw, int dh, int normalize, hipStream_t stream)
{
    OPK_CHECK_ARG(dst && src, "NULL buffer");
    OPK_CHECK_ARG(n > 0 && sw > 0 && sh > 0 && dw > 0 && dh > 0, "empty frame or net input");
    OPK_CHECK_ARG(scale > 0 && std::isfinite(scale), "scale must be positive");
    ctx->bind();
    // resizeFixedAspectRatio (openCvPrivate.cpp:34-52): INTER_CUBIC when enlarging, INTER_AREA
    // (which warpAffine runs as INTER_LINEAR) otherwise; scale 1 with the same size is the copy
    // that the identity warp reproduces exactly
    const bool cubic = scale > 1.;
    const short* w = ctx->warp_weight_table(cubic);
    const auto& ax = ctx->warp_axis_tables(scale, dw, dh);
    launch_cvmat_to_input(dst, src, n, sh, sw, step ? step : (size_t)sw * 3, dh, dw, ax.x, ax.y, w,
                          cubic ? 4 : 2, normalize, stream ? stream : ctx->stream);
}

}  // namespace opk
