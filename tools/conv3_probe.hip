// conv3_probe.hip -- dev tool: per-block phase timing of the conv3 halo kernel (s_memtime stamps).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o /tmp/conv3_probe tools/conv3_probe.hip
//   conv3_probe [frames H W cin cout iters]
//
// Prints, over all blocks of one launch, the mean/min/max shader cycles spent in
//   prologue (first DMA landed), main K loop, epilogue tile pass, store pass,
// plus the kernel's wall time from HIP events.  Inputs are random; only timing matters.
#define OPK3_STAMPS
#include "../openpose_amd/csrc/kernels/conv3.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

using namespace opk;

// the library's opk_dev_set table is not linked into this dev tool: variant switches come from
// OPK_<KEY> environment variables here (tools/probe_run.sh)
int opk::dev_switch(const char* key, int dflt)
{
    const char* e = std::getenv((std::string("OPK_") + key).c_str());
    return e && e[0] ? std::atoi(e) : dflt;
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

int main(int argc, char** argv)
{
    int frames = argc > 1 ? std::atoi(argv[1]) : 16;
    int H = argc > 2 ? std::atoi(argv[2]) : 46;
    int W = argc > 3 ? std::atoi(argv[3]) : 82;
    int cin = argc > 4 ? std::atoi(argv[4]) : 128;
    int cout = argc > 5 ? std::atoi(argv[5]) : 128;
    int iters = argc > 6 ? std::atoi(argv[6]) : 20;
    const int cin_pad = (cin + 31) / 32 * 32;
    const int Wp = W + 2;
    const long pos = (long)frames * (H + 2) * Wp;
    const long head = Wp + 64, tail = kConvGuardTail;
    const long in_elems = (head + pos + tail) * cin_pad;
    const long out_elems = (head + pos + tail) * cout;
    const long w_elems = (long)((cout + 63) / 64) * 128 * 9 * cin_pad;   // >= any BN packing

    std::vector<uint16_t> hin(in_elems);
    srand(1);
    for (auto& v : hin) v = (uint16_t)(0x3000 + (rand() & 0x0fff));   // small positive halves
    uint16_t *din, *dout, *dw;
    float *db, *ds;
    unsigned long long* dst;
    CK(hipMalloc(&din, in_elems * 2));
    CK(hipMalloc(&dout, out_elems * 2));
    CK(hipMalloc(&dw, w_elems * 2));
    CK(hipMalloc(&db, cout * 4));
    CK(hipMalloc(&ds, cout * 4));
    CK(hipMemcpy(din, hin.data(), in_elems * 2, hipMemcpyHostToDevice));
    CK(hipMemset(dw, 0x11, w_elems * 2));
    CK(hipMemset(db, 0, cout * 4));
    CK(hipMemset(ds, 0, cout * 4));

    ConvArgs a{};
    a.in = din + head * cin_pad;
    a.in_cs = cin_pad;
    a.in_coff = 0;
    a.cin_pad = cin_pad;
    a.ntaps = 9;
    a.ksteps = 9 * cin_pad / 64;
    a.w = dw;
    a.bias = db;
    a.slope = ds;
    a.act = 2;
    a.frames = frames;
    a.H = H;
    a.W = W;
    a.M = frames * H * Wp;
    a.cout = cout;
    a.ndst = 1;
    a.dst[0] = dout + head * cout;
    a.dst_cs[0] = cout;
    a.dst_coff[0] = 0;

    void* dsink;
    CK(hipMalloc(&dsink, kConv3SinkBytes));
    a.sink = dsink;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    a.cus = cus;
    const Conv3Shape s3 = conv3_shape(frames, H, W, cout, 3);
    a.sw = s3.sw;
    a.nstrips = s3.nstrips;
    const long vtot = (long)frames * s3.nstrips * (H + 2) * (s3.sw + 2);
    const int nblk = (int)(((vtot + s3.bm - 1) / s3.bm) * ((cout + s3.bn - 1) / s3.bn));
    CK(hipMalloc(&dst, (size_t)nblk * 8 * 8));
    CK(hipMemset(dst, 0, (size_t)nblk * 8 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(opk3_stamps), &dst, sizeof(dst)));

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) launch_conv3(a, 0);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) launch_conv3(a, 0);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    const double flops = 2.0 * frames * H * W * (double)cout * cin * 9;
    std::printf("frames=%d %dx%d cin=%d cout=%d blocks=%d: %.2f us/launch  %.1f TFLOP/s\n", frames,
                H, W, cin, cout, nblk, us, flops / us / 1e6);

    std::vector<unsigned long long> h((size_t)nblk * 8);
    CK(hipMemcpy(h.data(), dst, h.size() * 8, hipMemcpyDeviceToHost));
    // stamps: 0 start, 1 first DMA landed, 2 K loop done, 5 end; 6/7 = s_memrealtime (100 MHz);
    // persistent kernel (conv3p): 3 second tile's first unit, 4 second tile's K loop done
    const int ks[6][2] = {{0, 1}, {1, 2}, {2, 5}, {0, 5}, {2, 3}, {3, 4}};
    const char* names[6] = {"prologue", "K loop", "epilogue", "block", "tile gap", "K loop 2"};
    double ratio = 0;
    int nr = 0;
    for (int b = 0; b < nblk; ++b) {
        if (h[b * 8 + 5] == 0) continue;   // blocks of a persistent grid beyond G never ran
        ratio += (double)(h[b * 8 + 5] - h[b * 8 + 0]) / (double)(h[b * 8 + 7] - h[b * 8 + 6]);
        ++nr;
    }
    ratio /= nr;
    const double mhz = ratio * 100.0;
    std::printf("  s_memtime clock ~ %.0f MHz (vs s_memrealtime)\n", mhz);
    for (int k = 0; k < 6; ++k) {
        double sum = 0, mn = 1e30, mx = 0;
        int nb = 0;
        for (int b = 0; b < nblk; ++b) {
            if (h[b * 8 + 5] == 0 || (k >= 4 && h[b * 8 + 4] == 0)) continue;   // no such stamp
            ++nb;
            const double d = (double)(h[b * 8 + ks[k][1]] - h[b * 8 + ks[k][0]]);
            sum += d;
            mn = std::min(mn, d);
            mx = std::max(mx, d);
        }
        if (nb == 0) continue;
        std::printf("  %-9s mean %8.0f cyc = %7.2f us  (min %8.0f max %8.0f, %d blocks)\n", names[k],
                    sum / nb, sum / nb / mhz, mn, mx, nb);
    }
    // wall span of the launch seen by the realtime clock
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int b = 0; b < nblk; ++b) {
        if (h[b * 8 + 5] == 0) continue;
        t0 = std::min(t0, h[b * 8 + 6]);
        t1 = std::max(t1, h[b * 8 + 7]);
    }
    std::printf("  first block start -> last block end: %.2f us\n", (t1 - t0) / 100.0);
    return 0;
}
