// array_driver.cpp -- test driver for integration/arrayCpuGpuHip.cpp (op::ArrayCpuGpu on HIP memory).
//
// Built against the reference's own headers (include/openpose/core/arrayCpuGpu.hpp) by
// tests/test_array_cpu_gpu.py; op::error is the test's (it throws, like the reference's does after
// logging) and opkShimThreadContext opens one device-0 context, as the shim's first call on a
// thread would.  `array_driver cpu` checks the host-side Blob contract (no device touched),
// `array_driver gpu` the SyncedMemory transitions through libopk_hip device memory.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include <openpose/core/arrayCpuGpu.hpp>
#include <openpose/utilities/errorAndLog.hpp>

#include "opk.h"
#include "opk_shim.hpp"

namespace op
{
    void error(const std::string& message, const int line, const std::string& function,
               const std::string& file)
    {
        throw std::runtime_error(message + " (" + file + ":" + std::to_string(line) + " " + function + ")");
    }

    OpkContext opkShimThreadContext(const int)
    {
        static OpkContext ctx;
        if (!ctx) {
            opk_ctx* raw = nullptr;
            if (opk_ctx_create(0, nullptr, &raw) != OPK_OK)
                throw std::runtime_error(opk_last_error());
            ctx = OpkContext{raw, opk_ctx_destroy};
        }
        return ctx;
    }
}

#define EXPECT(c)                                                                             \
    do {                                                                                      \
        if (!(c)) {                                                                           \
            std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);               \
            return 1;                                                                         \
        }                                                                                     \
    } while (0)

static int cpu_checks()
{
    op::ArrayCpuGpu<float> a(2, 3, 4, 5);
    EXPECT(a.num_axes() == 4 && a.count() == 120 && a.num() == 2 && a.channels() == 3);
    EXPECT(a.height() == 4 && a.width() == 5 && a.shape(-1) == 5 && a.count(1) == 60);
    EXPECT(a.count(1, 3) == 12 && a.offset(1, 2, 3, 4) == 119);
    EXPECT(a.shape_string() == "2 3 4 5 (120)");
    const float* d = a.cpu_data();   // uninitialised -> zeroed host buffer
    for (int i = 0; i < a.count(); ++i) EXPECT(d[i] == 0.f);
    float* w = a.mutable_cpu_data();
    for (int i = 0; i < a.count(); ++i) w[i] = (float)i - 60.f;
    EXPECT(a.data_at(1, 2, 3, 4) == 59.f);
    EXPECT(a.asum_data() == 3600.f);                    // sum |i - 60|, i < 120
    float* g = a.mutable_cpu_diff();
    for (int i = 0; i < a.count(); ++i) g[i] = 1.f;
    a.Update();                                         // data -= diff
    EXPECT(a.data_at(0, 0, 0, 0) == -61.f && a.diff_at(0, 0, 0, 1) == 1.f);
    a.scale_data(2.f);
    EXPECT(a.data_at(0, 0, 0, 1) == -120.f && a.sumsq_diff() == 120.f);
    // Reshape within the capacity keeps the buffer; beyond it reallocates (Blob::Reshape)
    const float* before = a.cpu_data();
    a.Reshape(1, 1, 6, 10);
    EXPECT(a.count() == 60 && a.cpu_data() == before && a.LegacyShape(3) == 10);
    a.Reshape(std::vector<int>{7, 5});
    EXPECT(a.num_axes() == 2 && a.height() == 1 && a.width() == 1 && a.count() == 35);
    a.Reshape(4, 4, 4, 4);
    EXPECT(a.count() == 256 && a.cpu_data()[255] == 0.f);
    // external host data becomes the head
    std::vector<float> ext(256, 3.f);
    a.set_cpu_data(ext.data());
    EXPECT(a.cpu_data() == ext.data() && a.asum_data() == 768.f);
    bool threw = false;
    try { a.shape(4); } catch (const std::exception&) { threw = true; }
    EXPECT(threw);
    op::ArrayCpuGpu<int> k(1, 25, 8, 8);   // nmsCaffe's kernel blob type
    EXPECT(k.count() == 1600 && k.cpu_data()[1599] == 0);
    threw = false;
    try { op::ArrayCpuGpu<float> caffe((const void*)&k); } catch (const std::exception&) { threw = true; }
    EXPECT(threw);
    std::printf("cpu ok\n");
    return 0;
}

static int gpu_checks()
{
    opk_ctx* ctx = op::opkShimThreadContext().get();
    op::ArrayCpuGpu<float> a(1, 2, 3, 4);
    float* h = a.mutable_cpu_data();
    for (int i = 0; i < 24; ++i) h[i] = (float)i;
    const float* dev = a.gpu_data();                    // HEAD_AT_CPU -> copied up, SYNCED
    std::vector<float> back(24);
    EXPECT(opk_memcpy_d2h(ctx, back.data(), dev, 24 * 4) == OPK_OK);
    for (int i = 0; i < 24; ++i) EXPECT(back[i] == (float)i);
    // the device side becomes the head: cpu_data() must copy it back
    float* mdev = a.mutable_gpu_data();
    EXPECT(mdev == dev);
    std::vector<float> up(24, 7.5f);
    EXPECT(opk_memcpy_h2d(ctx, mdev, up.data(), 24 * 4) == OPK_OK);
    EXPECT(opk_sync(ctx) == OPK_OK);
    EXPECT(a.cpu_data()[23] == 7.5f && a.asum_data() == 180.f);
    // an external device buffer (NetHip's live output) as the head
    void* ext = nullptr;
    EXPECT(opk_malloc(ctx, &ext, 24 * 4) == OPK_OK);
    std::vector<float> v(24, -2.f);
    EXPECT(opk_memcpy_h2d(ctx, ext, v.data(), 24 * 4) == OPK_OK);
    a.set_gpu_data(static_cast<float*>(ext));
    EXPECT(a.gpu_data() == ext && a.cpu_data()[5] == -2.f);
    v.assign(24, 4.f);                                  // the next "forward" rewrites it
    EXPECT(opk_memcpy_h2d(ctx, ext, v.data(), 24 * 4) == OPK_OK);
    a.set_gpu_data(static_cast<float*>(ext));           // what NetHip::refreshOutput does
    EXPECT(a.cpu_data()[5] == 4.f);
    // shape on the device (gpu_shape) and a zero-initialised device-first blob
    std::vector<int> sh(4);
    EXPECT(opk_memcpy_d2h(ctx, sh.data(), a.gpu_shape(), 16) == OPK_OK);
    EXPECT(sh[0] == 1 && sh[1] == 2 && sh[2] == 3 && sh[3] == 4);
    op::ArrayCpuGpu<float> z(1, 1, 16, 16);
    EXPECT(z.gpu_data() != nullptr && z.cpu_data()[255] == 0.f);
    EXPECT(opk_free(ctx, ext) == OPK_OK);
    std::printf("gpu ok\n");
    return 0;
}

int main(int argc, char** argv)
{
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    try {
        return mode == "gpu" ? gpu_checks() : cpu_checks();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 1;
    }
}
