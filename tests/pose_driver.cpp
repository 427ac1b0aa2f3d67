// pose_driver.cpp -- runs the pose drop-in (integration/openpose_hip_shim.cpp) through the reference's
// own call sequence, linked against libopk_hip.so.  Built against the reference headers by
// tests/test_pose_shim.py (with tests/shim_backing.cpp for the reference symbols that need OpenCV);
// `pose_driver DIR` reads the inputs the test wrote into DIR and writes every result there, for the
// test to compare with the C-ABI pipeline on the same inputs:
//   1. PoseExtractorHip through a PoseExtractorNet* on a worker thread, as the Wrapper's GPU worker
//      runs it (wrapperAuxiliary.hpp:329, poseExtractor.cpp:38-55): initializationOnThread ->
//      forwardPass (1 scale; property push) -> getPoseKeypoints / getPoseScores / getHeatMapSize /
//      getHeatMapCpuConstPtr / getCandidatesCpuConstPtr / getScaleNetToOutput, then 4 scales; the
//      thread is joined and the extractor destroyed afterwards on the main thread, as the Wrapper
//      does (the context outlives the thread);
//   2. the same with --upsampling_ratio 4;
//   3. the poseNetOutput injection path (enableNet = false, poseExtractorCaffe.cpp:249-262);
//   4. makeNetHip in addCaffeNetOnThread's order (poseExtractorCaffe.cpp:82-95): the output blob is
//      taken before the first forward and read after two forwards of different shapes;
//   5. resizeAndMergeGpu -> nmsGpu -> connectBodyPartsGpu with the reference signatures, float and
//      double instantiations;
//   6. two worker threads, each with its own PoseExtractorHip (the --num_gpu N Wrapper threads, all
//      on device 0 here), forwarding concurrently.
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <execinfo.h>
#include <fstream>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <openpose/core/common.hpp>
#include <openpose/net/bodyPartConnectorBase.hpp>
#include <openpose/net/net.hpp>
#include <openpose/net/nmsBase.hpp>
#include <openpose/net/resizeAndMergeBase.hpp>
#include <openpose/pose/poseExtractorNet.hpp>

#include "opk.h"
#include "opk_shim.hpp"
#include "poseExtractorHip.hpp"

namespace op
{
    std::shared_ptr<Net> makeNetHip(const std::string& proto, const std::string& model, const int gpuId);
}

namespace
{
    std::string gDir;
    const char* gStage = "start";

    template <typename T>
    std::vector<T> load(const std::string& name)
    {
        std::ifstream f(gDir + "/" + name, std::ios::binary | std::ios::ate);
        if (!f)
            throw std::runtime_error("missing " + name);
        const size_t bytes = (size_t)f.tellg();
        std::vector<T> v(bytes / sizeof(T));
        f.seekg(0);
        f.read(reinterpret_cast<char*>(v.data()), bytes);
        return v;
    }

    template <typename T>
    void save(const std::string& name, const T* data, const size_t count)
    {
        std::ofstream f(gDir + "/" + name, std::ios::binary);
        f.write(reinterpret_cast<const char*>(data), count * sizeof(T));
    }

    op::Array<float> netInput(const std::vector<float>& data, const int h, const int w)
    {
        op::Array<float> a{{1, 3, h, w}};
        std::copy(data.begin(), data.end(), a.getPtr());
        return a;
    }

    void saveResults(op::PoseExtractorNet& ex, const std::string& tag, const bool maps)
    {
        const auto kp = ex.getPoseKeypoints();
        const auto sc = ex.getPoseScores();
        const int people = kp.empty() ? 0 : kp.getSize(0);
        const float meta[2] = {(float)people, ex.getScaleNetToOutput()};
        save(tag + "_meta.f32", meta, 2);
        if (people > 0)
        {
            save(tag + "_kp.f32", kp.getConstPtr(), kp.getVolume());
            save(tag + "_sc.f32", sc.getConstPtr(), sc.getVolume());
        }
        if (maps)
        {
            const auto size = ex.getHeatMapSize();
            save(tag + "_heatsize.i32", size.data(), size.size());
            const size_t n = (size_t)size[1] * size[2] * size[3];
            save(tag + "_heat.f32", ex.getHeatMapCpuConstPtr(), n);
            save(tag + "_cand.f32", ex.getCandidatesCpuConstPtr(), (size_t)25 * 128 * 3);
        }
    }

    std::vector<int> gMeta;   // net_h, net_w, nscales, (h_i, w_i)..., prod_w, prod_h, out_h, out_w

    std::unique_ptr<op::PoseExtractorNet> makeExtractor(const float upsampling, const bool enableNet)
    {
        return std::unique_ptr<op::PoseExtractorNet>{new op::PoseExtractorHip{
            op::PoseModel::BODY_25, "", 0, {}, op::ScaleMode::ZeroToOneFixedAspect, false, false,
            "builtin:BODY_25", gDir + "/model.caffemodel", upsampling, enableNet}};
    }

    void runExtractor(op::PoseExtractorNet& ex, const std::string& tag, const bool multi)
    {
        const int ns = gMeta[2];
        const op::Point<int> producer{gMeta[3 + 2 * ns], gMeta[4 + 2 * ns]};
        const auto scales = load<double>("scales.f64");
        std::vector<op::Array<float>> inputs;
        for (int i = 0; i < (multi ? ns : 1); i++)
            inputs.push_back(netInput(load<float>("in_s" + std::to_string(i) + ".f32"), gMeta[3 + 2 * i],
                                      gMeta[4 + 2 * i]));
        const std::vector<double> ratios(scales.begin(), scales.begin() + inputs.size());
        ex.forwardPass(inputs, producer, ratios);
        saveResults(ex, tag, !multi);
    }
}

int main(int argc, char** argv)
{
    if (argc < 2)
    {
        std::fprintf(stderr, "usage: pose_driver DIR\n");
        return 2;
    }
    gDir = argv[1];
    std::set_terminate([] {
        std::string what = "no active exception";
        if (auto e = std::current_exception())
        {
            try
            {
                std::rethrow_exception(e);
            }
            catch (const std::exception& x)
            {
                what = x.what();
            }
            catch (...)
            {
                what = "non-std exception";
            }
        }
        std::fprintf(stderr, "pose driver: std::terminate (last stage: %s; %s)\n", gStage, what.c_str());
        void* frames[64];
        backtrace_symbols_fd(frames, backtrace(frames, 64), 2);
        std::abort();
    });
    try
    {
        gMeta = load<int>("meta.i32");
        const int ns = gMeta[2];
        const op::Point<int> producer{gMeta[3 + 2 * ns], gMeta[4 + 2 * ns]};
        const int oh = gMeta[5 + 2 * ns], ow = gMeta[6 + 2 * ns];

        gStage = "extractors";
        // 1 + 2: extractors built on the main thread, run on a worker, destroyed after the join
        auto ex = makeExtractor(0.f, true);
        auto ex4 = makeExtractor(4.f, true);
        std::string failure;
        std::thread worker{[&] {
            try
            {
                gStage = "worker: init";
                ex->initializationOnThread();
                ex->set(op::PoseProperty::NMSThreshold, 0.06);   // pushed to libopk at the next forward
                gStage = "worker: single";
                runExtractor(*ex, "single", false);
                gStage = "worker: multi";
                runExtractor(*ex, "multi", true);
                gStage = "worker: up4";
                ex4->initializationOnThread();
                runExtractor(*ex4, "up4", false);
                gStage = "worker: done";
            }
            catch (const std::exception& e)
            {
                failure = e.what();
            }
            catch (...)
            {
                failure = "unknown exception";
            }
        }};
        worker.join();
        if (!failure.empty())
            throw std::runtime_error("worker: " + failure);
        gStage = "extractor destruction after the join";
        ex.reset();    // the worker thread (and its thread-local context reference) is gone
        ex4.reset();

        gStage = "inject";
        // 3: injected net output
        {
            auto inj = makeExtractor(0.f, false);
            inj->initializationOnThread();
            const auto netOut = load<float>("netout.f32");
            op::Array<float> poseNetOutput{{1, 78, oh, ow}};
            std::copy(netOut.begin(), netOut.end(), poseNetOutput.getPtr());
            std::vector<op::Array<float>> dummy{op::Array<float>{{1, 3, gMeta[0], gMeta[1]}, 0.f}};
            inj->forwardPass(dummy, producer, {1.}, poseNetOutput);
            saveResults(*inj, "inject", true);
        }

        gStage = "nethip";
        // 4: NetHip in addCaffeNetOnThread's order
        {
            auto net = op::makeNetHip("builtin:BODY_25", gDir + "/model.caffemodel", 0);
            net->initializationOnThread();
            const auto blob = net->getOutputBlobArray();   // before any forward
            const int before[4] = {blob->shape(0), blob->shape(1), blob->shape(2), blob->shape(3)};
            save("net_before.i32", before, 4);
            net->forwardPass(netInput(load<float>("in_s0.f32"), gMeta[3], gMeta[4]));
            save("net_out0.f32", blob->cpu_data(), (size_t)blob->count());
            net->forwardPass(netInput(load<float>("in_s1.f32"), gMeta[5], gMeta[6]));
            const int after[4] = {blob->shape(0), blob->shape(1), blob->shape(2), blob->shape(3)};
            save("net_after.i32", after, 4);
            save("net_out1.f32", blob->cpu_data(), (size_t)blob->count());
        }

        gStage = "gpu functions";
        // 5: the replaced CUDA functions with the reference signatures
        {
            opk_ctx* ctx = op::opkShimThreadContext().get();
            const int H = gMeta[0], W = gMeta[1];
            const auto netOut = load<float>("netout.f32");
            void *src = nullptr, *heat = nullptr, *peaks = nullptr, *kern = nullptr;
            if (opk_malloc(ctx, &src, netOut.size() * 4) || opk_malloc(ctx, &heat, (size_t)78 * H * W * 4) ||
                opk_malloc(ctx, &peaks, (size_t)25 * 128 * 3 * 4) || opk_malloc(ctx, &kern, (size_t)25 * H * W * 4) ||
                opk_memcpy_h2d(ctx, src, netOut.data(), netOut.size() * 4))
                throw std::runtime_error(opk_last_error());
            op::resizeAndMergeGpu((float*)heat, std::vector<const float*>{(const float*)src},
                                  std::array<int, 4>{1, 78, H, W}, {std::array<int, 4>{1, 78, oh, ow}},
                                  std::vector<float>{1.f});
            const float off = float(0.5 / (double)load<float>("fns_scale.f32")[0]);
            op::nmsGpu((float*)peaks, (int*)kern, (const float*)heat, 0.05f, std::array<int, 4>{1, 25, 128, 3},
                       std::array<int, 4>{1, 78, H, W}, op::Point<float>{off, off});
            std::vector<float> peaksHost((size_t)25 * 128 * 3);
            opk_memcpy_d2h(ctx, peaksHost.data(), peaks, peaksHost.size() * 4);
            save("fns_peaks.f32", peaksHost.data(), peaksHost.size());
            op::Array<float> kp, sc;
            op::connectBodyPartsGpu<float>(kp, sc, (const float*)heat, peaksHost.data(), op::PoseModel::BODY_25,
                                    op::Point<int>{W, H}, 127, 0.95f, 0.05f, 3, 0.4f, 0.05f,
                                    load<float>("fns_scale.f32")[0], false, op::Array<float>{}, nullptr,
                                    nullptr, nullptr, (const float*)peaks);
            const float people = kp.empty() ? 0.f : (float)kp.getSize(0);
            save("fns_meta.f32", &people, 1);
            if (!kp.empty())
            {
                save("fns_kp.f32", kp.getConstPtr(), kp.getVolume());
                save("fns_sc.f32", sc.getConstPtr(), sc.getVolume());
            }
            // 5b: the double instantiations on the same data (float kernels between conversions)
            const std::vector<double> netOut64(netOut.begin(), netOut.end());
            void *src64 = nullptr, *heat64 = nullptr, *peaks64 = nullptr;
            if (opk_malloc(ctx, &src64, netOut64.size() * 8) || opk_malloc(ctx, &heat64, (size_t)78 * H * W * 8) ||
                opk_malloc(ctx, &peaks64, (size_t)25 * 128 * 3 * 8) ||
                opk_memcpy_h2d(ctx, src64, netOut64.data(), netOut64.size() * 8))
                throw std::runtime_error(opk_last_error());
            op::resizeAndMergeGpu((double*)heat64, std::vector<const double*>{(const double*)src64},
                                  std::array<int, 4>{1, 78, H, W}, {std::array<int, 4>{1, 78, oh, ow}},
                                  std::vector<double>{1.});
            std::vector<double> heatHost64((size_t)78 * H * W);
            opk_memcpy_d2h(ctx, heatHost64.data(), heat64, heatHost64.size() * 8);
            save("fns64_heat.f64", heatHost64.data(), heatHost64.size());
            op::nmsGpu((double*)peaks64, (int*)kern, (const double*)heat64, 0.05, std::array<int, 4>{1, 25, 128, 3},
                       std::array<int, 4>{1, 78, H, W}, op::Point<double>{(double)off, (double)off});
            std::vector<double> peaksHost64((size_t)25 * 128 * 3);
            opk_memcpy_d2h(ctx, peaksHost64.data(), peaks64, peaksHost64.size() * 8);
            save("fns64_peaks.f64", peaksHost64.data(), peaksHost64.size());
            op::Array<double> kp64, sc64;
            op::connectBodyPartsGpu<double>(kp64, sc64, (const double*)heat64, peaksHost64.data(),
                                     op::PoseModel::BODY_25, op::Point<int>{W, H}, 127, 0.95, 0.05, 3, 0.4,
                                     0.05, (double)load<float>("fns_scale.f32")[0], false, op::Array<double>{},
                                     nullptr, nullptr, nullptr, (const double*)peaks64);
            const double people64 = kp64.empty() ? 0. : (double)kp64.getSize(0);
            save("fns64_meta.f64", &people64, 1);
            if (!kp64.empty())
            {
                save("fns64_kp.f64", kp64.getConstPtr(), kp64.getVolume());
                save("fns64_sc.f64", sc64.getConstPtr(), sc64.getVolume());
            }
            opk_free(ctx, src64);
            opk_free(ctx, heat64);
            opk_free(ctx, peaks64);
            opk_free(ctx, src);
            opk_free(ctx, heat);
            opk_free(ctx, peaks);
            opk_free(ctx, kern);
        }

        gStage = "threads";
        // 6: two Wrapper threads, each with its own extractor, forwarding concurrently
        {
            std::string fail[2];
            std::unique_ptr<op::PoseExtractorNet> exs[2] = {makeExtractor(0.f, true), makeExtractor(0.f, true)};
            std::thread ts[2];
            for (int t = 0; t < 2; t++)
                ts[t] = std::thread{[&, t] {
                    try
                    {
                        exs[t]->initializationOnThread();
                        exs[t]->set(op::PoseProperty::NMSThreshold, 0.06);
                        for (int rep = 0; rep < 3; rep++)
                            runExtractor(*exs[t], "thread" + std::to_string(t) + "_" + std::to_string(rep), false);
                    }
                    catch (const std::exception& e)
                    {
                        fail[t] = e.what();
                    }
                    catch (...)
                    {
                        fail[t] = "unknown exception";
                    }
                }};
            for (auto& t : ts)
                t.join();
            for (const auto& f : fail)
                if (!f.empty())
                    throw std::runtime_error("thread: " + f);
        }   // destroyed on the main thread, after the joins
        std::printf("pose driver ok\n");
        return 0;
    }
    catch (const std::exception& e)
    {
        std::fprintf(stderr, "pose driver failed: %s\n", e.what());
        return 1;
    }
}
