// conv3w_probe.hip -- dev tool: phase timeline of the conv3w kernel (s_memtime stamps of wave 0
// of every workgroup) on one BODY_25 stage-layer shape, plus its event-timed throughput.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/conv3w_probe_bin tools/conv3w_probe.hip
//   conv3w_probe [frames H W cin cout iters dma_end zero_operands variant]
//   variant 1 (NOSTAMPS builds): conv3w8, checked bit for bit against conv3w
//   (round 4 also had variant 2 / 3: conv3w / conv3w8 with the rejected E2 and halo-early
//   schedules -- profiles/round4/stage_skeleton/)
//   OPK_<SWITCH>=<value> in the environment sets a dev switch
#ifndef NOSTAMPS
#define OPKW_STAMPS
#endif
#include "../openpose_amd/csrc/kernels/conv3w.hip"
#ifdef NOSTAMPS
#include "../openpose_amd/csrc/kernels/conv3w8.hip"
#endif

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

using namespace opk;

static int g_dma_end = 0;
void opk::note_launch(const char*, ...) {}
int opk::dev_switch(const char* key, int dflt)
{
    if (std::string(key) == "CONV3W") return g_dma_end ? 1 : 2;
    const char* e = std::getenv((std::string("OPK_") + key).c_str());
    return e ? std::atoi(e) : dflt;
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
    const int frames = argc > 1 ? std::atoi(argv[1]) : 64;
    const int H = argc > 2 ? std::atoi(argv[2]) : 46;
    const int W = argc > 3 ? std::atoi(argv[3]) : 82;
    const int cin = argc > 4 ? std::atoi(argv[4]) : 128;
    const int cout = argc > 5 ? std::atoi(argv[5]) : 128;
    const int iters = argc > 6 ? std::atoi(argv[6]) : 20;
    g_dma_end = argc > 7 ? std::atoi(argv[7]) : 1;
    const int variant = argc > 9 ? std::atoi(argv[9]) : 0;
    const int cin_pad = (cin + 31) / 32 * 32;
    const int Wp = W + 2;
    const long pos = (long)frames * (H + 2) * Wp;
    const long head = Wp + 64, tail = kConvGuardTail;
    const long in_elems = (head + pos + tail) * cin_pad;
    const long out_elems = (head + pos + tail) * cout;
    const long w_elems = (long)cout * 9 * cin_pad;
    std::vector<uint16_t> hin(in_elems), hw(w_elems);
    srand(1);
    for (auto& v : hin) v = (uint16_t)(0x3000 + (rand() & 0x0fff));
    for (auto& v : hw) v = (uint16_t)(0x2000 + (rand() & 0x0fff));
    if (argc > 8 && std::atoi(argv[8]) == 1) {   // all-zero operands (DVFS comparison)
        for (auto& v : hin) v = 0;
        for (auto& v : hw) v = 0;
    }
    uint16_t *din, *dout, *dw;
    float *db, *ds;
    CK(hipMalloc(&din, in_elems * 2));
    CK(hipMalloc(&dout, out_elems * 2));
    CK(hipMalloc(&dw, w_elems * 2));
    CK(hipMalloc(&db, 512 * 4));
    CK(hipMalloc(&ds, 512 * 4));
    CK(hipMemcpy(din, hin.data(), in_elems * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, hw.data(), w_elems * 2, hipMemcpyHostToDevice));
    CK(hipMemset(db, 0, 512 * 4));
    CK(hipMemset(ds, 0, 512 * 4));
    void* dsink;
    CK(hipMalloc(&dsink, kConv3SinkBytes));
    ConvArgs a{};
    a.in = din + head * cin_pad;
    a.in_cs = cin_pad;
    a.cin_pad = cin_pad;
    a.ntaps = 9;
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
    a.sink = dsink;
    CK(hipDeviceGetAttribute(&a.cus, hipDeviceAttributeMultiprocessorCount, 0));
    a.border = 1;
    a.sw = W;          // one strip (W + 2 <= 87 for the 688-row halo)
    a.nstrips = 1;
    a.rcp[0] = (float)(1.0 / ((double)(H + 2) * (W + 2)));
    a.rcp[1] = (float)(1.0 / (double)(W + 2));
    a.rcp[2] = 1.f;
    const long ntm = (pos + 511) / 512;
    const int G = (int)std::min<long>(a.cus, ntm);
    unsigned long long* dst;
    CK(hipMalloc(&dst, (size_t)G * 16 * 8));
    CK(hipMemset(dst, 0, (size_t)G * 16 * 8));
#ifdef OPKW_STAMPS
    CK(hipMemcpyToSymbol(HIP_SYMBOL(opkw_stamps), &dst, sizeof(dst)));
    unsigned long long* dus;
    CK(hipMalloc(&dus, (size_t)G * 32 * 8));
    CK(hipMemset(dus, 0, (size_t)G * 32 * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(opkw_ustamps), &dus, sizeof(dus)));
#endif

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto launch = [&](const ConvArgs& x) {
#ifdef NOSTAMPS
        if (variant == 1) { launch_conv3w8(x, 0); return; }
#endif
        launch_conv3w(x, 0);
    };
    CK(hipMemset(dout, 0, out_elems * 2));
    for (int i = 0; i < 5; ++i) launch(a);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) launch(a);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    const double flops = 2.0 * frames * H * W * (double)cout * cin * 9;
    if (variant == 1) {   // bit-identity against conv3w
        uint16_t* dref;
        CK(hipMalloc(&dref, out_elems * 2));
        CK(hipMemset(dref, 0, out_elems * 2));
        ConvArgs b = a;
        b.dst[0] = dref + head * cout;
        launch_conv3w(b, 0);
        CK(hipDeviceSynchronize());
        std::vector<uint16_t> h1(out_elems), h2(out_elems);
        CK(hipMemcpy(h1.data(), dout, out_elems * 2, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h2.data(), dref, out_elems * 2, hipMemcpyDeviceToHost));
        long diff = 0, nz = 0;
        for (long i = 0; i < out_elems; ++i) { diff += h1[i] != h2[i]; nz += h2[i] != 0; }
        std::printf("  variant %d vs conv3w", variant);
        std::printf(": %ld of %ld fp16 values differ (%ld nonzero)\n", diff, out_elems, nz);
    }
    std::printf("conv3w v%d dma_end=%d frames=%d %dx%d cin=%d cout=%d tiles=%ld grid=%d: %.2f us/launch %.1f TFLOP/s\n",
                variant, g_dma_end, frames, H, W, cin, cout, ntm, G, us, flops / us / 1e6);
#ifndef OPKW_STAMPS
    return 0;
#endif
    std::vector<unsigned long long> h((size_t)G * 16);
    CK(hipMemcpy(h.data(), dst, h.size() * 8, hipMemcpyDeviceToHost));
    double ratio = 0;
    for (int b = 0; b < G; ++b)
        ratio += (double)(h[b * 16 + 6] - h[b * 16 + 0]) / (double)(h[b * 16 + 15] - h[b * 16 + 14]);
    const double mhz = ratio / G * 100.0;
    std::printf("  clock ~ %.0f MHz\n", mhz);
    // phases (cycles): 0 start, 1 prologue barrier passed, 2 tile-0 K loop end, 3 tile-0 epilogue
    // end, 4 tile-1 K loop end, 5 tile-1 epilogue end, 6 kernel end (vmcnt 0); tile 0 unit 3:
    // 8 before vmcnt wait, 9 after it, 10 after the barrier, 11 unit 4's mid-unit; 12 tile 1 u0
    const int ph[][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 12}, {3, 4}, {4, 5}, {5, 6}, {0, 6}, {8, 9}, {9, 10}, {10, 11}};
    const char* nm[] = {"prologue", "K loop 0", "epilogue 0", "t1 to mid u0", "K loop 1", "epilogue 1",
                        "final drain", "block", "u3 vmcnt wait", "u3 barrier", "u3->u4 mid"};
    for (int k = 0; k < 11; ++k) {
        double sum = 0, mn = 1e30, mx = 0;
        int nb = 0;
        for (int b = 0; b < G; ++b) {
            const auto x0 = h[b * 16 + ph[k][0]], x1 = h[b * 16 + ph[k][1]];
            if (x0 == 0 || x1 == 0 || x1 < x0) continue;
            const double d = (double)(x1 - x0);
            sum += d;
            mn = std::min(mn, d);
            mx = std::max(mx, d);
            ++nb;
        }
        if (nb) std::printf("  %-14s mean %8.0f cyc = %7.2f us  (min %8.0f max %8.0f, %d blocks)\n", nm[k],
                            sum / nb, sum / nb / mhz, mn, mx, nb);
    }
#ifdef OPKW_STAMPS
    {   // per unit of the second tile: wait + barrier at the mid-unit, and the mid-to-mid period
        std::vector<unsigned long long> u((size_t)G * 32);
        CK(hipMemcpy(u.data(), dus, u.size() * 8, hipMemcpyDeviceToHost));
        const int U = 3 * (cin_pad / 32);
        std::printf("  tile 1 per unit (cycles, block means): unit  wait+barrier  mid->mid\n");
        for (int k = 0; k < U && 2 * k + 1 < 32; ++k) {
            double wb = 0, per = 0;
            int nb = 0, np = 0;
            for (int b = 0; b < G; ++b) {
                const auto x0 = u[b * 32 + 2 * k], x1 = u[b * 32 + 2 * k + 1];
                if (!x0 || !x1) continue;
                wb += (double)(x1 - x0);
                ++nb;
                if (k + 1 < U && 2 * k + 3 < 32 && u[b * 32 + 2 * k + 3]) {
                    per += (double)(u[b * 32 + 2 * k + 3] - x1);
                    ++np;
                }
            }
            if (nb) std::printf("    u%-3d %8.0f  %8.0f\n", k, wb / nb, np ? per / np : 0.0);
        }
    }
#endif
    unsigned long long t0 = ~0ull, t1 = 0;
    for (int b = 0; b < G; ++b) {
        t0 = std::min(t0, h[b * 16 + 14]);
        t1 = std::max(t1, h[b * 16 + 15]);
    }
    std::printf("  first block start -> last block end: %.2f us\n", (t1 - t0) / 100.0);
    return 0;
}
