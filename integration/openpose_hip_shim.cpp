// openpose_hip_shim.cpp -- drop-in replacement of the reference's CUDA hot-path translation units,
// compiled INSIDE the reference tree (against include/openpose/...) and linked with libopk_hip.so.
//
// It defines, with the reference's exact signatures, the symbols the reference's CUDA objects
// define today:
//   op::resizeAndMergeGpu<float|double>   (include/openpose/net/resizeAndMergeBase.hpp:17-20,
//                                          replaces src/openpose/net/resizeAndMergeBase.cu)
//   op::nmsGpu<float|double>              (include/openpose/net/nmsBase.hpp:14-16,
//                                          replaces src/openpose/net/nmsBase.cu)
//   op::connectBodyPartsGpu<float|double> (include/openpose/net/bodyPartConnectorBase.hpp:17-24,
//                                          replaces src/openpose/net/bodyPartConnectorBase.cu)
// and op::NetHip, an op::Net (include/openpose/net/net.hpp:8-18) with NetCaffe's constructor shape
// whose output blob is an op::ArrayCpuGpu on HIP memory (arrayCpuGpuHip.cpp, which replaces
// src/openpose/core/arrayCpuGpu.cpp)
// (netCaffe.hpp:12-13), for PoseExtractorCaffe::addCaffeNetOnThread (poseExtractorCaffe.cpp:82-86),
// loading the .caffemodel itself; and the members of op::CvMatToOpInput
// (include/openpose/core/cvMatToOpInput.hpp:9-28, replaces src/openpose/core/cvMatToOpInput.cpp):
// the frame -> net-input warp and normalisation on the GPU with the CPU branch's numerics; and the
// members of op::FaceExtractorCaffe / op::HandExtractorCaffe (faceExtractorCaffe.hpp:13-45,
// handExtractorCaffe.hpp:13-58, replace src/openpose/{face,hand}/*ExtractorCaffe.cpp): every
// rectangle of a frame cropped, run through the face / hand net and reduced on the GPU at once.
// resizeAndMergeGpu / nmsGpu compute what the CUDA objects they replace compute (OPK_MAPS_CUDA:
// Catmull-Rom x8 resize, strict-interior NMS; include/opk.h) unless the shim is built with
// -DOPK_SHIM_MAPS=OPK_MAPS_CPU, which gives the CPU path's numerics (resizeAndMergeCpu / nmsCpu);
// everything else follows the CPU path.  The double instantiations run the float
// kernels between device conversions (AsFloat below).  Errors come back through op::error, the
// reference's convention (errorAndLog.cpp:158-233).  See INTEGRATION.md for the build lines.
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include <openpose/core/common.hpp>
#include <openpose/core/cvMatToOpInput.hpp>
#include <openpose/face/faceExtractorCaffe.hpp>
#include <openpose/face/faceParameters.hpp>
#include <openpose/hand/handExtractorCaffe.hpp>
#include <openpose/hand/handParameters.hpp>
#include <openpose/net/bodyPartConnectorBase.hpp>
#include <openpose/net/net.hpp>
#include <openpose/net/nmsBase.hpp>
#include <openpose/net/resizeAndMergeBase.hpp>
#include <openpose/pose/poseParameters.hpp>

#include "opk.h"
#include "opk_shim.hpp"
#include "poseExtractorHip.hpp"

#ifndef OPK_SHIM_MAPS
#define OPK_SHIM_MAPS OPK_MAPS_CUDA
#endif

namespace op
{
    // one context per calling thread = per GPU worker thread (wrapperAuxiliary.hpp:1050-1067);
    // the reference runs everything on the legacy default stream, so does this context.  Shared
    // ownership: see opk_shim.hpp.
    OpkContext opkShimThreadContext(const int device)
    {
        thread_local OpkContext ctx;
        thread_local int bound = -1;
        const int want = device >= 0 ? device : (bound >= 0 ? bound : 0);
        if (!ctx || want != bound)
        {
            opk_ctx* raw = nullptr;
            if (opk_ctx_create(want, nullptr, &raw) != OPK_OK)
                error(opk_last_error(), __LINE__, __FUNCTION__, __FILE__);
            ctx = OpkContext{raw, opk_ctx_destroy};
            bound = want;
        }
        return ctx;
    }

    namespace
    {
        opk_ctx* threadContext() { return opkShimThreadContext().get(); }

        // CvMatToOpInput's device buffers are members of the reference's own class
        // (cvMatToOpInput.hpp), so the context they were allocated on is kept beside it
        std::mutex gInputCtxMutex;
        std::map<const void*, OpkContext> gInputCtx;

        OpkContext inputContext(const void* owner)
        {
            std::lock_guard<std::mutex> lock{gInputCtxMutex};
            auto& c = gInputCtx[owner];
            if (!c)
                c = opkShimThreadContext();
            return c;
        }
    }

    namespace
    {
        void check(const int rc, const int line, const char* function)
        {
            if (rc != OPK_OK)
                error(std::string{"libopk_hip: "} + opk_last_error(), line, function, __FILE__);
        }

        // opk_net_create + the arithmetic the deployment asks for: OPENPOSE_HIP_PRECISION=split runs
        // every net of the process in OPK_PRECISION_SPLIT (fp16 hi/lo pairs, ~fp32 results at ~3.4x
        // the CNN time); unset or "fp16" keeps the default.  Any other value is an error, not a
        // silent default.
        opk_net* createNet(opk_ctx* ctx, const std::string& proto, const std::string& model)
        {
            opk_net* net = nullptr;
            check(opk_net_create(ctx, proto.c_str(), model.c_str(), &net), __LINE__, __FUNCTION__);
            const char* env = std::getenv("OPENPOSE_HIP_PRECISION");
            const std::string want = env ? env : "fp16";
            if (want != "fp16" && want != "split")
            {
                opk_net_destroy(net);
                error("OPENPOSE_HIP_PRECISION must be fp16 or split, not '" + want + "'.", __LINE__,
                      __FUNCTION__, __FILE__);
            }
            if (want == "split" && opk_net_set_precision(net, OPK_PRECISION_SPLIT) != OPK_OK)
            {
                const std::string msg = opk_last_error();   // (read before the destroy resets it)
                opk_net_destroy(net);   // not leaked on the error path
                error(std::string{"libopk_hip: "} + msg, __LINE__, __FUNCTION__, __FILE__);
            }
            return net;
        }

        // Conversion buffers of the double instantiations, kept per thread and reused in stream
        // order on the thread's context (an opk_malloc / opk_free per call would synchronise the
        // device at every hipFree).  The pool holds its context, so it is freed safely at thread
        // exit; a thread whose context moved to another device starts a new pool.
        struct ConvPool
        {
            OpkContext ctx;
            std::vector<std::pair<float*, size_t>> free;
            void flush()
            {
                for (const auto& b : free)
                    opk_free(ctx.get(), b.first);
                free.clear();
            }
            ~ConvPool() { flush(); }
        };
        thread_local ConvPool tConvPool;

        float* convAcquire(const size_t count, size_t& capacity)
        {
            auto& pool = tConvPool;
            const auto ctx = opkShimThreadContext();
            if (pool.ctx != ctx)
            {
                pool.flush();
                pool.ctx = ctx;
            }
            for (size_t i = 0; i < pool.free.size(); ++i)
                if (pool.free[i].second >= count)
                {
                    float* const b = pool.free[i].first;
                    capacity = pool.free[i].second;
                    pool.free.erase(pool.free.begin() + (long)i);
                    return b;
                }
            float* b = nullptr;
            check(opk_malloc(ctx.get(), (void**)&b, count * sizeof(float)), __LINE__, __FUNCTION__);
            capacity = count;
            return b;
        }

        void convRelease(float* b, const size_t capacity)
        {
            if (tConvPool.ctx.get() == threadContext())
                tConvPool.free.emplace_back(b, capacity);
            else
                opk_free(threadContext(), b);
        }

        // The double instantiations (resizeAndMergeBase.cu:575-581, nmsBase.cu:353-358,
        // bodyPartConnectorBase.cu:252-266) run the float kernels: a device array of T seen as
        // float -- the caller's pointer for float, a converted copy for double (opk_convert), so
        // a double caller gets the float kernels' results widened (float precision)
        template <typename T>
        class AsFloat
        {
        public:
            AsFloat(const T* src, const size_t count, const bool load) : mCount{count}
            {
                if (std::is_same<T, float>::value)
                {
                    mPtr = (float*)src;
                    return;
                }
                mPtr = convAcquire(count, mCapacity);
                mOwned = true;
                if (load)
                    check(opk_convert(threadContext(), mPtr, OPK_F32, src, OPK_F64, count), __LINE__,
                          __FUNCTION__);
            }
            ~AsFloat()
            {
                if (mOwned)
                    convRelease(mPtr, mCapacity);
            }
            AsFloat(const AsFloat&) = delete;
            AsFloat& operator=(const AsFloat&) = delete;
            float* get() const { return mPtr; }
            // the float results back into the caller's T array (double: widened)
            void store(T* dst) const
            {
                if (mOwned)
                    check(opk_convert(threadContext(), dst, OPK_F64, mPtr, OPK_F32, mCount), __LINE__,
                          __FUNCTION__);
            }
        private:
            float* mPtr = nullptr;
            size_t mCount, mCapacity = 0;
            bool mOwned = false;
        };

        size_t volume(const std::array<int, 4>& s)
        {
            return (size_t)s[0] * s[1] * s[2] * s[3];
        }
    }

    template <typename T>
    void resizeAndMergeGpu(
        T* targetPtr, const std::vector<const T*>& sourcePtrs, const std::array<int, 4>& targetSize,
        const std::vector<std::array<int, 4>>& sourceSizes, const std::vector<T>& scaleInputToNetInputs)
    {
        try
        {
            std::vector<int> sizes;
            for (const auto& s : sourceSizes)
                sizes.insert(sizes.end(), s.begin(), s.end());
            std::vector<float> ratios(scaleInputToNetInputs.begin(), scaleInputToNetInputs.end());
            std::vector<std::unique_ptr<AsFloat<T>>> sources;
            std::vector<const float*> sourceFloats;
            for (auto i = 0u; i < sourcePtrs.size(); i++)
            {
                sources.emplace_back(new AsFloat<T>{
                    sourcePtrs[i], i < sourceSizes.size() ? volume(sourceSizes[i]) : 0, true});
                sourceFloats.emplace_back(sources.back()->get());
            }
            const AsFloat<T> target{targetPtr, volume(targetSize), false};
            check(opk_resize_and_merge_semantics(threadContext(), target.get(), sourceFloats.data(),
                                                 (int)sourceFloats.size(), targetSize.data(),
                                                 sizes.data(), ratios.data(), OPK_SHIM_MAPS),
                  __LINE__, __FUNCTION__);
            target.store(targetPtr);
            check(opk_sync(threadContext()), __LINE__, __FUNCTION__);
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
        }
    }

    template <typename T>
    void nmsGpu(
        T* targetPtr, int* kernelPtr, const T* const sourcePtr, const T threshold,
        const std::array<int, 4>& targetSize, const std::array<int, 4>& sourceSize, const Point<T>& offset)
    {
        try
        {
            const AsFloat<T> source{sourcePtr, volume(sourceSize), true};
            const AsFloat<T> target{targetPtr, volume(targetSize), false};
            check(opk_nms_semantics(threadContext(), target.get(), kernelPtr, source.get(),
                                    (float)threshold, targetSize.data(), sourceSize.data(),
                                    (float)offset.x, (float)offset.y, OPK_SHIM_MAPS),
                  __LINE__, __FUNCTION__);
            target.store(targetPtr);
            check(opk_sync(threadContext()), __LINE__, __FUNCTION__);
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
        }
    }

    template <typename T>
    void connectBodyPartsGpu(
        Array<T>& poseKeypoints, Array<T>& poseScores, const T* const heatMapGpuPtr, const T* const peaksPtr,
        const PoseModel poseModel, const Point<int>& heatMapSize, const int maxPeaks,
        const T interMinAboveThreshold, const T interThreshold, const int minSubsetCnt, const T minSubsetScore,
        const T defaultNmsThreshold, const T scaleFactor, const bool maximizePositives, Array<T> pairScoresCpu,
        T* pairScoresGpuPtr, const unsigned int* const bodyPartPairsGpuPtr, const unsigned int* const mapIdxGpuPtr,
        const T* const peaksGpuPtr)
    {
        try
        {
            (void)peaksPtr; (void)pairScoresCpu; (void)pairScoresGpuPtr;   // owned by libopk_hip
            (void)bodyPartPairsGpuPtr; (void)mapIdxGpuPtr;
            const auto numberBodyParts = (int)getPoseNumberBodyParts(poseModel);
            const auto channels = numberBodyParts + (addBkgChannel(poseModel) ? 1 : 0)
                                + (int)getPoseMapIndex(poseModel).size();
            const AsFloat<T> heat{heatMapGpuPtr, (size_t)channels * heatMapSize.x * heatMapSize.y, true};
            const AsFloat<T> peaks{peaksGpuPtr, (size_t)numberBodyParts * (maxPeaks + 1) * 3, true};
            // the CPU path's assembly (the parity target) where the reference's CPU connector
            // exists; connectBodyPartsGpu's own global-sort assembly for the other models (BODY_135...)
            const bool cpuModel = numberBodyParts == 25 || numberBodyParts == 18 || numberBodyParts == 15;
            const int semantics = cpuModel ? OPK_CONNECT_CPU : OPK_CONNECT_GPU;
            int people = 0;
            std::vector<float> keypoints, scores;
            for (int capacity = maxPeaks * 4 + 8;; capacity = people)
            {
                keypoints.resize((size_t)capacity * numberBodyParts * 3);
                scores.resize(capacity);
                check(opk_connect_body_parts_semantics(
                          threadContext(), keypoints.data(), scores.data(), capacity, &people,
                          heat.get(), peaks.get(), (int)poseModel, channels,
                          heatMapSize.y, heatMapSize.x, maxPeaks, (float)interMinAboveThreshold,
                          (float)interThreshold, minSubsetCnt, (float)minSubsetScore,
                          (float)defaultNmsThreshold, (float)scaleFactor, maximizePositives ? 1 : 0, semantics),
                      __LINE__, __FUNCTION__);
                if (people <= capacity)
                    break;   // otherwise: more people than rows, run again with room for all
            }
            // peopleVectorToPeopleArray semantics (bodyPartConnectorBase.cpp:895-907)
            if (people > 0)
            {
                poseKeypoints.reset({people, numberBodyParts, 3}, 0.f);
                poseScores.reset(people);
                for (auto i = 0u; i < poseKeypoints.getVolume(); i++)
                    poseKeypoints[i] = T(keypoints[i]);
                for (auto i = 0; i < people; i++)
                    poseScores[i] = T(scores[i]);
            }
            else
            {
                poseKeypoints.reset();
                poseScores.reset();
            }
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
        }
    }

    template void resizeAndMergeGpu(
        float*, const std::vector<const float*>&, const std::array<int, 4>&,
        const std::vector<std::array<int, 4>>&, const std::vector<float>&);
    template void resizeAndMergeGpu(
        double*, const std::vector<const double*>&, const std::array<int, 4>&,
        const std::vector<std::array<int, 4>>&, const std::vector<double>&);
    template void nmsGpu(
        float*, int*, const float* const, const float, const std::array<int, 4>&,
        const std::array<int, 4>&, const Point<float>&);
    template void nmsGpu(
        double*, int*, const double* const, const double, const std::array<int, 4>&,
        const std::array<int, 4>&, const Point<double>&);
    template void connectBodyPartsGpu(
        Array<float>&, Array<float>&, const float* const, const float* const, const PoseModel,
        const Point<int>&, const int, const float, const float, const int, const float, const float,
        const float, const bool, Array<float>, float*, const unsigned int* const,
        const unsigned int* const, const float* const);
    template void connectBodyPartsGpu(
        Array<double>&, Array<double>&, const double* const, const double* const, const PoseModel,
        const Point<int>&, const int, const double, const double, const int, const double, const double,
        const double, const bool, Array<double>, double*, const unsigned int* const,
        const unsigned int* const, const double* const);

    // ---- op::Net on libopk_hip (the NetCaffe replacement) ---------------------------------------
    class NetHip : public Net
    {
    public:
        NetHip(const std::string& caffeProto, const std::string& caffeTrainedModel, const int gpuId = 0,
               const bool enableGoogleLogging = true, const std::string& lastBlobName = "net_output") :
            mProto{caffeProto}, mModel{caffeTrainedModel}, mGpuId{gpuId}
        {
            (void)enableGoogleLogging;
            if (lastBlobName != "net_output")
                error("NetHip exposes the net_output blob only.", __LINE__, __FUNCTION__, __FILE__);
        }

        virtual ~NetHip()
        {
            if (mInput)
                opk_free(mCtx.get(), mInput);
            if (mNet)
                opk_net_destroy(mNet);
        }   // the context itself goes when its last holder does

        void initializationOnThread()
        {
            mCtx = opkShimThreadContext(mGpuId);   // binds this thread to the GPU (netCaffe.cpp:169-170)
            mNet = createNet(mCtx.get(), mProto, mModel);
        }

        void forwardPass(const Array<float>& inputNetData) const
        {
            const auto size = inputNetData.getSize();   // {1, 3, H, W} (netCaffe.cpp:220-237)
            if (size.size() != 4 || size[1] != 3)
                error("Input must be NCHW with 3 channels.", __LINE__, __FUNCTION__, __FILE__);
            const size_t bytes = inputNetData.getVolume() * sizeof(float);
            if (bytes > mInputBytes)
            {
                if (mInput)
                    opk_free(mCtx.get(), mInput);
                mInput = nullptr;
                check(opk_malloc(mCtx.get(), &mInput, bytes), __LINE__, __FUNCTION__);
                mInputBytes = bytes;
            }
            check(opk_memcpy_h2d(mCtx.get(), mInput, inputNetData.getConstPtr(), bytes), __LINE__, __FUNCTION__);
            check(opk_net_forward(mNet, (const float*)mInput, size[0], size[2], size[3]), __LINE__,
                  __FUNCTION__);
            if (spOutput)
                refreshOutput();   // the blob handed out at init now holds this forward's output
        }

        // NetCaffe returns a live wrapper of its output blob (netCaffe.cpp:263-268), and
        // addCaffeNetOnThread takes it ONCE, right after initializationOnThread and before any
        // forward (poseExtractorCaffe.cpp:94-95), then reads it after every forward.  Here: one
        // ArrayCpuGpu per net (the HIP-backed one, arrayCpuGpuHip.cpp), valid from the first call
        // ({1, C, 1, 1} before a forward) and pointed at the net's device output by every
        // forwardPass (Reshape + set_gpu_data: gpu_data() is the live buffer, cpu_data() copies it
        // on demand, as Caffe's SyncedMemory does).
        std::shared_ptr<ArrayCpuGpu<float>> getOutputBlobArray() const
        {
            if (!spOutput)
            {
                float* out = nullptr;
                int shape[4];
                check(opk_net_output(mNet, &out, shape), __LINE__, __FUNCTION__);
                spOutput = std::make_shared<ArrayCpuGpu<float>>(1, shape[1], 1, 1);
                if (out != nullptr)
                    refreshOutput();
            }
            return spOutput;
        }

    private:
        void refreshOutput() const
        {
            float* out = nullptr;
            int shape[4];
            check(opk_net_output(mNet, &out, shape), __LINE__, __FUNCTION__);
            spOutput->Reshape(shape[0], shape[1], shape[2], shape[3]);
            spOutput->set_gpu_data(out);
        }

        const std::string mProto, mModel;
        const int mGpuId;
        OpkContext mCtx;
        opk_net* mNet = nullptr;
        mutable void* mInput = nullptr;
        mutable size_t mInputBytes = 0;
        mutable std::shared_ptr<ArrayCpuGpu<float>> spOutput;
    };

    std::shared_ptr<Net> makeNetHip(const std::string& proto, const std::string& model, const int gpuId)
    {
        return std::make_shared<NetHip>(proto, model, gpuId);
    }

    // ---- op::PoseExtractorHip: PoseExtractorNet on libopk_hip (no Caffe, no CUDA) ---------------
    struct PoseExtractorHip::ImplPoseExtractorHip
    {
        PoseModel poseModel;
        int gpuId;
        std::string proto, model;
        bool enableNet, maximizePositives;
        int parts = 0, heatChannels = 0;
        float upsamplingRatio = 0.f;
        OpkContext ctxOwner;
        opk_ctx* ctx = nullptr;             // ctxOwner.get()
        opk_net* net = nullptr;
        opk_pose* pose = nullptr;
        std::vector<void*> inputs;          // device net inputs, one per scale
        std::vector<size_t> inputBytes;
        void* injected = nullptr;           // device copy of poseNetOutput
        size_t injectedBytes = 0;
        int heatH = 0, heatW = 0;
        // host copies, made on request and valid until the next forwardPass
        mutable std::vector<float> heatHost, peaksHost;
        mutable bool heatFresh = false, peaksFresh = false;

        ~ImplPoseExtractorHip()
        {
            if (pose)
                opk_pose_destroy(pose);
            if (net)
                opk_net_destroy(net);
            if (ctx)
            {
                for (auto* p : inputs)
                    if (p)
                        opk_free(ctx, p);
                if (injected)
                    opk_free(ctx, injected);
            }
        }

        void* deviceBuffer(void*& buffer, size_t& capacity, const size_t bytes)
        {
            if (bytes > capacity)
            {
                if (buffer)
                    opk_free(ctx, buffer);
                buffer = nullptr;
                check(opk_malloc(ctx, &buffer, bytes), __LINE__, __FUNCTION__);
                capacity = bytes;
            }
            return buffer;
        }
    };

    PoseExtractorHip::PoseExtractorHip(
        const PoseModel poseModel, const std::string& modelFolder, const int gpuId,
        const std::vector<HeatMapType>& heatMapTypes, const ScaleMode heatMapScaleMode,
        const bool addPartCandidates, const bool maximizePositives, const std::string& protoTxtPath,
        const std::string& caffeModelPath, const float upsamplingRatio, const bool enableNet,
        const bool enableGoogleLogging) :
        PoseExtractorNet{poseModel, heatMapTypes, heatMapScaleMode, addPartCandidates, maximizePositives},
        upImpl{new ImplPoseExtractorHip{}}
    {
        try
        {
            (void)enableGoogleLogging;
            upImpl->upsamplingRatio = upsamplingRatio;   // --upsampling_ratio (poseExtractorCaffe.cpp:47-54,281-287)
            upImpl->poseModel = poseModel;
            upImpl->gpuId = gpuId;
            upImpl->enableNet = enableNet;
            upImpl->maximizePositives = maximizePositives;
            // the same paths addCaffeNetOnThread builds (poseExtractorCaffe.cpp:82-86)
            upImpl->proto = modelFolder + (protoTxtPath.empty() ? getPoseProtoTxt(poseModel) : protoTxtPath);
            upImpl->model = modelFolder + (caffeModelPath.empty() ? getPoseTrainedModel(poseModel) : caffeModelPath);
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
        }
    }

    PoseExtractorHip::~PoseExtractorHip()
    {
    }

    void PoseExtractorHip::netInitializationOnThread()
    {
        try
        {
            auto& impl = *upImpl;
            impl.ctxOwner = opkShimThreadContext(impl.gpuId);   // binds this thread to the GPU (netCaffe.cpp:169-170)
            impl.ctx = impl.ctxOwner.get();
            if (impl.enableNet)
                impl.net = createNet(impl.ctx, impl.proto, impl.model);
            // the connector the reference would run: the CPU path's assembly where its CPU
            // connector exists, connectBodyPartsGpu's for the other models (BODY_135, ...)
            const auto numberBodyParts = (int)getPoseNumberBodyParts(impl.poseModel);
            const bool cpuModel = numberBodyParts == 25 || numberBodyParts == 18 || numberBodyParts == 15;
            check(opk_pose_create_model(impl.ctx, impl.net, (int)impl.poseModel, impl.maximizePositives ? 1 : 0,
                                        cpuModel ? OPK_CONNECT_CPU : OPK_CONNECT_GPU, &impl.pose),
                  __LINE__, __FUNCTION__);
            check(opk_pose_model_info((int)impl.poseModel, &impl.parts, nullptr, nullptr, &impl.heatChannels,
                                      nullptr, nullptr), __LINE__, __FUNCTION__);
            check(opk_pose_set_upsampling_ratio(impl.pose, impl.upsamplingRatio), __LINE__, __FUNCTION__);
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
        }
    }

    void PoseExtractorHip::forwardPass(
        const std::vector<Array<float>>& inputNetData, const Point<int>& inputDataSize,
        const std::vector<double>& scaleInputToNetInputs, const Array<float>& poseNetOutput)
    {
        try
        {
            auto& impl = *upImpl;
            if (!impl.pose)
                error("netInitializationOnThread() was not called.", __LINE__, __FUNCTION__, __FILE__);
            // sanity checks of poseExtractorCaffe.cpp:213-231
            if (inputNetData.empty())
                error("Empty inputNetData.", __LINE__, __FUNCTION__, __FILE__);
            for (const auto& inputNetDataI : inputNetData)
                if (inputNetDataI.empty())
                    error("Empty inputNetData.", __LINE__, __FUNCTION__, __FILE__);
            if (inputNetData.size() != scaleInputToNetInputs.size())
                error("Size(inputNetData) must be same than size(scaleInputToNetInputs).",
                      __LINE__, __FUNCTION__, __FILE__);
            if (poseNetOutput.empty() != impl.enableNet)
                error("Either use OpenPose default network (`--body 1`) or fill the `poseNetOutput` argument"
                      " (only 1 of those 2, not both).", __LINE__, __FUNCTION__, __FILE__);
            // PoseProperty values (set/increase may change them between frames)
            const PoseProperty props[] = {
                PoseProperty::NMSThreshold, PoseProperty::ConnectInterMinAboveThreshold,
                PoseProperty::ConnectInterThreshold, PoseProperty::ConnectMinSubsetCnt,
                PoseProperty::ConnectMinSubsetScore};
            const int opkProps[] = {
                OPK_PROP_NMS_THRESHOLD, OPK_PROP_INTER_MIN_ABOVE_THRESHOLD, OPK_PROP_INTER_THRESHOLD,
                OPK_PROP_MIN_SUBSET_CNT, OPK_PROP_MIN_SUBSET_SCORE};
            for (auto i = 0; i < 5; i++)
                check(opk_pose_set_property(impl.pose, opkProps[i], get(props[i])), __LINE__, __FUNCTION__);

            const auto numberScales = inputNetData.size();
            const int netH = inputNetData[0].getSize(2), netW = inputNetData[0].getSize(3);
            if (impl.enableNet)
            {
                impl.inputs.resize(numberScales, nullptr);
                impl.inputBytes.resize(numberScales, 0);
                std::vector<const float*> ptrs(numberScales);
                std::vector<int> hw(2 * numberScales);
                for (auto i = 0u; i < numberScales; i++)
                {
                    const auto& in = inputNetData[i];   // {1, 3, H, W} (netCaffe.cpp:220-237)
                    if (in.getNumberDimensions() != 4 || in.getSize(1) != 3)
                        error("Input must be NCHW with 3 channels.", __LINE__, __FUNCTION__, __FILE__);
                    const size_t bytes = in.getVolume() * sizeof(float);
                    void* dev = impl.deviceBuffer(impl.inputs[i], impl.inputBytes[i], bytes);
                    check(opk_memcpy_h2d(impl.ctx, dev, in.getConstPtr(), bytes), __LINE__, __FUNCTION__);
                    ptrs[i] = static_cast<const float*>(dev);
                    hw[2 * i] = in.getSize(2);
                    hw[2 * i + 1] = in.getSize(3);
                }
                if (numberScales == 1)
                    check(opk_pose_forward(impl.pose, ptrs[0], inputNetData[0].getSize(0), netH, netW,
                                           inputDataSize.x, inputDataSize.y), __LINE__, __FUNCTION__);
                else
                    check(opk_pose_forward_multi(impl.pose, ptrs.data(), hw.data(), (int)numberScales,
                                                 inputNetData[0].getSize(0), inputDataSize.x, inputDataSize.y),
                          __LINE__, __FUNCTION__);
            }
            else
            {
                // injected net output (poseExtractorCaffe.cpp:249-262): one scale, [1][C][h][w]
                if (numberScales != 1u)
                    error("Size(inputNetData) must match the provided heatmaps batch size (1).",
                          __LINE__, __FUNCTION__, __FILE__);
                if (poseNetOutput.getNumberDimensions() != 4 || poseNetOutput.getSize(1) != impl.heatChannels)
                    error("poseNetOutput must be [1][heat channels][h][w].", __LINE__, __FUNCTION__, __FILE__);
                const size_t bytes = poseNetOutput.getVolume() * sizeof(float);
                void* dev = impl.deviceBuffer(impl.injected, impl.injectedBytes, bytes);
                check(opk_memcpy_h2d(impl.ctx, dev, poseNetOutput.getConstPtr(), bytes), __LINE__, __FUNCTION__);
                check(opk_pose_forward_net_output(impl.pose, static_cast<const float*>(dev), poseNetOutput.getSize(0),
                                                  poseNetOutput.getSize(2), poseNetOutput.getSize(3), netH, netW,
                                                  inputDataSize.x, inputDataSize.y),
                      __LINE__, __FUNCTION__);
            }
            // results of frame 0 (peopleVectorToPeopleArray, bodyPartConnectorBase.cpp:895-907)
            const int people = opk_pose_num_people(impl.pose, 0);
            if (people > 0)
            {
                mPoseKeypoints.reset({people, impl.parts, 3}, 0.f);
                mPoseScores.reset(people);
                check(opk_pose_keypoints(impl.pose, 0, mPoseKeypoints.getPtr(), mPoseScores.getPtr(), people),
                      __LINE__, __FUNCTION__);
            }
            else
            {
                mPoseKeypoints.reset();
                mPoseScores.reset();
            }
            mScaleNetToOutput = opk_pose_scale_net_to_output(impl.pose);
            // mNetOutputSize = the net input size x (ratio / decrease factor), ratio 1 without
            // --upsampling_ratio (poseExtractorCaffe.cpp:281-287)
            const auto ratio = (impl.upsamplingRatio <= 0.f
                                    ? 1.f : impl.upsamplingRatio / getPoseNetDecreaseFactor(impl.poseModel));
            mNetOutputSize = Point<int>{int(ratio * netW + 0.5f), int(ratio * netH + 0.5f)};
            int shape[4];
            check(opk_pose_heatmap_size(impl.pose, shape), __LINE__, __FUNCTION__);
            impl.heatH = shape[2];
            impl.heatW = shape[3];
            impl.heatFresh = false;
            impl.peaksFresh = false;
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
        }
    }

    const float* PoseExtractorHip::getCandidatesCpuConstPtr() const
    {
        try
        {
            checkThread();
            auto& impl = *upImpl;
            if (!impl.peaksFresh)
            {
                float* dev = nullptr;
                int shape[4];
                check(opk_pose_peaks(impl.pose, &dev, shape), __LINE__, __FUNCTION__);
                impl.peaksHost.resize((size_t)shape[1] * shape[2] * shape[3]);   // frame 0
                check(opk_memcpy_d2h(impl.ctx, impl.peaksHost.data(), dev, impl.peaksHost.size() * sizeof(float)),
                      __LINE__, __FUNCTION__);
                impl.peaksFresh = true;
            }
            return impl.peaksHost.data();
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
            return nullptr;
        }
    }

    const float* PoseExtractorHip::getCandidatesGpuConstPtr() const
    {
        try
        {
            checkThread();
            float* dev = nullptr;
            int shape[4];
            check(opk_pose_peaks(upImpl->pose, &dev, shape), __LINE__, __FUNCTION__);
            return dev;
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
            return nullptr;
        }
    }

    const float* PoseExtractorHip::getHeatMapCpuConstPtr() const
    {
        try
        {
            checkThread();
            auto& impl = *upImpl;
            if (!impl.heatFresh)
            {
                float* dev = nullptr;
                int shape[4];
                check(opk_pose_heatmaps(impl.pose, &dev, shape), __LINE__, __FUNCTION__);
                impl.heatHost.resize((size_t)shape[1] * shape[2] * shape[3]);   // frame 0
                check(opk_memcpy_d2h(impl.ctx, impl.heatHost.data(), dev, impl.heatHost.size() * sizeof(float)),
                      __LINE__, __FUNCTION__);
                impl.heatFresh = true;
            }
            return impl.heatHost.data();
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
            return nullptr;
        }
    }

    const float* PoseExtractorHip::getHeatMapGpuConstPtr() const
    {
        try
        {
            checkThread();
            float* dev = nullptr;
            int shape[4];
            check(opk_pose_heatmaps(upImpl->pose, &dev, shape), __LINE__, __FUNCTION__);
            return dev;
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
            return nullptr;
        }
    }

    std::vector<int> PoseExtractorHip::getHeatMapSize() const
    {
        try
        {
            checkThread();
            return {1, upImpl->heatChannels, upImpl->heatH, upImpl->heatW};   // spHeatMapsBlob->shape()
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
            return {};
        }
    }

    const float* PoseExtractorHip::getPoseGpuConstPtr() const
    {
        // as PoseExtractorCaffe::getPoseGpuConstPtr (poseExtractorCaffe.cpp:724-741)
        error("GPU pointer for people pose data not implemented yet.", __LINE__, __FUNCTION__, __FILE__);
        return nullptr;
    }

    // ---- op::CvMatToOpInput on libopk_hip --------------------------------------------------------
    // The reference's own members are reused: pInputImageCuda holds the frame, pOutputImageCuda the
    // net input of one scale (both device buffers of the calling thread's context).
    CvMatToOpInput::CvMatToOpInput(const PoseModel poseModel, const bool gpuResize) :
        mPoseModel{poseModel},
        mGpuResize{gpuResize},   // either way the GPU runs the CPU branch's arithmetic
        pInputImageCuda{nullptr},
        pInputImageReorderedCuda{nullptr},
        pOutputImageCuda{nullptr},
        pInputMaxSize{0ull},
        pOutputMaxSize{0ull}
    {
        if (mPoseModel == PoseModel::BODY_19N)
            error("BODY_19N (DenseNet normalisation) is not supported by libopk_hip.", __LINE__,
                  __FUNCTION__, __FILE__);
    }

    CvMatToOpInput::~CvMatToOpInput()
    {
        OpkContext owner;
        {
            std::lock_guard<std::mutex> lock{gInputCtxMutex};
            auto it = gInputCtx.find(this);
            if (it != gInputCtx.end())
            {
                owner = it->second;
                gInputCtx.erase(it);
            }
        }
        if (owner)   // the buffers belong to the context they were allocated on
        {
            if (pInputImageCuda)
                opk_free(owner.get(), pInputImageCuda);
            if (pOutputImageCuda)
                opk_free(owner.get(), pOutputImageCuda);
        }
    }

    std::vector<Array<float>> CvMatToOpInput::createArray(
        const Matrix& inputData, const std::vector<double>& scaleInputToNetInputs,
        const std::vector<Point<int>>& netInputSizes)
    {
        // sanity checks of cvMatToOpInput.cpp:68-76
        if (inputData.empty())
            error("Wrong input element (empty inputData).", __LINE__, __FUNCTION__, __FILE__);
        if (inputData.channels() != 3)
            error("Input images must be 3-channel BGR.", __LINE__, __FUNCTION__, __FILE__);
        if (scaleInputToNetInputs.size() != netInputSizes.size())
            error("scaleInputToNetInputs.size() != netInputSizes.size().", __LINE__, __FUNCTION__, __FILE__);
        const OpkContext owner = inputContext(this);   // the context of the first call, for good
        opk_ctx* ctx = owner.get();
        const size_t step = inputData.step1(0);   // bytes per row (uchar)
        const unsigned long long frameBytes = (unsigned long long)step * inputData.rows();
        if (pInputMaxSize < frameBytes)
        {
            if (pInputImageCuda)
                opk_free(ctx, pInputImageCuda);
            void* p = nullptr;
            check(opk_malloc(ctx, &p, frameBytes), __LINE__, __FUNCTION__);
            pInputImageCuda = static_cast<unsigned char*>(p);
            pInputMaxSize = frameBytes;
        }
        check(opk_memcpy_h2d(ctx, pInputImageCuda, inputData.dataConst(), frameBytes), __LINE__,
              __FUNCTION__);
        std::vector<Array<float>> inputNetData(scaleInputToNetInputs.size());
        for (auto i = 0u; i < inputNetData.size(); i++)
        {
            const auto& size = netInputSizes.at(i);
            const unsigned long long outBytes = 3ull * size.x * size.y * sizeof(float);
            if (pOutputMaxSize < outBytes)
            {
                if (pOutputImageCuda)
                    opk_free(ctx, pOutputImageCuda);
                void* p = nullptr;
                check(opk_malloc(ctx, &p, outBytes), __LINE__, __FUNCTION__);
                pOutputImageCuda = static_cast<float*>(p);
                pOutputMaxSize = outBytes;
            }
            check(opk_cvmat_to_input(ctx, pOutputImageCuda, pInputImageCuda, 1, inputData.cols(),
                                     inputData.rows(), step, scaleInputToNetInputs[i], size.x, size.y, 1),
                  __LINE__, __FUNCTION__);
            inputNetData[i].reset({1, 3, size.y, size.x});
            check(opk_memcpy_d2h(ctx, inputNetData[i].getPtr(), pOutputImageCuda, outBytes), __LINE__,
                  __FUNCTION__);
        }
        return inputNetData;
    }

    // ---- op::FaceExtractorCaffe / op::HandExtractorCaffe on libopk_hip ----------------------------
    namespace
    {
        // the net, the extractor and the frame buffer of one extractor object (its worker thread)
        struct KeypointNetHip
        {
            std::string proto, model;
            int gpuId = 0;
            OpkContext ctxOwner;
            opk_ctx* ctx = nullptr;   // ctxOwner.get()
            opk_net* net = nullptr;
            opk_extractor* ex = nullptr;
            void* frame = nullptr;
            size_t frameBytes = 0;

            ~KeypointNetHip()
            {
                if (ex)
                    opk_extractor_destroy(ex);
                if (net)
                    opk_net_destroy(net);
                if (frame && ctx)
                    opk_free(ctx, frame);
            }

            int heatMapScaleMode = -1;   // op::ScaleMode when --heatmaps_add_* asks for maps

            void initialize(const int kind, const Point<int>& netSize)
            {
                ctxOwner = opkShimThreadContext(gpuId);
                ctx = ctxOwner.get();
                net = createNet(ctx, proto, model);
                check(opk_extractor_create(ctx, net, kind, netSize.x, netSize.y, &ex), __LINE__,
                      __FUNCTION__);
                check(opk_extractor_set_heatmaps(ex, heatMapScaleMode), __LINE__, __FUNCTION__);
            }

            // the last forward's per-person heat maps of hand `h` (face: 0) into `heatMaps`
            // ({people, parts, H, W}, as updateFace/HandHeatMapsForPerson fill it)
            void copyHeatMaps(Array<float>& heatMaps, const int h)
            {
                const float* dev = nullptr;
                int shape[5];
                check(opk_extractor_heatmaps(ex, &dev, shape), __LINE__, __FUNCTION__);
                heatMaps.reset({shape[1], shape[2], shape[3], shape[4]}, 0.f);
                const size_t bytes = heatMaps.getVolume() * sizeof(float);
                if (bytes > 0)
                    check(opk_memcpy_d2h(ctx, heatMaps.getPtr(), dev + (size_t)h * heatMaps.getVolume(),
                                         bytes), __LINE__, __FUNCTION__);
            }

            // inputData (BGR uint8) -> device, rectangles -> keypoints [hands][people][parts][3]
            std::vector<float> forward(const Matrix& inputData, const std::vector<float>& rects,
                                       const int people, const int hands)
            {
                if (!ex)
                    error("netInitializationOnThread() was not called.", __LINE__, __FUNCTION__, __FILE__);
                if (inputData.empty())
                    error("Empty cvInputData.", __LINE__, __FUNCTION__, __FILE__);
                const size_t step = inputData.step1(0);
                const size_t bytes = step * inputData.rows();
                if (bytes > frameBytes)
                {
                    if (frame)
                        opk_free(ctx, frame);
                    frame = nullptr;
                    check(opk_malloc(ctx, &frame, bytes), __LINE__, __FUNCTION__);
                    frameBytes = bytes;
                }
                check(opk_memcpy_h2d(ctx, frame, inputData.dataConst(), bytes), __LINE__, __FUNCTION__);
                const int parts = opk_extractor_parts(ex);
                std::vector<float> keypoints((size_t)hands * people * parts * 3);
                check(opk_extractor_forward(ex, static_cast<const unsigned char*>(frame), 1,
                                            inputData.cols(), inputData.rows(), step, rects.data(),
                                            nullptr, people, keypoints.data()),
                      __LINE__, __FUNCTION__);
                return keypoints;
            }
        };

        void pushRectangle(std::vector<float>& out, const Rectangle<float>& r)
        {
            out.insert(out.end(), {r.x, r.y, r.width, r.height});
        }
    }

    struct FaceExtractorCaffe::ImplFaceExtractorCaffe : KeypointNetHip {};

    FaceExtractorCaffe::FaceExtractorCaffe(const Point<int>& netInputSize, const Point<int>& netOutputSize,
                                           const std::string& modelFolder, const int gpuId,
                                           const std::vector<HeatMapType>& heatMapTypes,
                                           const ScaleMode heatMapScaleMode, const bool enableGoogleLogging) :
        FaceExtractorNet{netInputSize, netOutputSize, heatMapTypes, heatMapScaleMode},
        upImpl{new ImplFaceExtractorCaffe{}}
    {
        (void)enableGoogleLogging;
        if (!heatMapTypes.empty())   // faceExtractorCaffe.cpp:196-198,290-299
            upImpl->heatMapScaleMode = (int)heatMapScaleMode;
        upImpl->proto = modelFolder + FACE_PROTOTXT;
        upImpl->model = modelFolder + FACE_TRAINED_MODEL;
        upImpl->gpuId = gpuId;
    }

    FaceExtractorCaffe::~FaceExtractorCaffe()
    {
    }

    void FaceExtractorCaffe::netInitializationOnThread()
    {
        upImpl->initialize(OPK_EXTRACT_FACE, mNetOutputSize);
    }

    void FaceExtractorCaffe::forwardPass(const std::vector<Rectangle<float>>& faceRectangles,
                                         const Matrix& inputData)
    {
        try
        {
            if (mEnabled && !faceRectangles.empty())
            {
                std::vector<float> rects;
                for (const auto& r : faceRectangles)
                    pushRectangle(rects, r);
                const int people = (int)faceRectangles.size();
                const auto keypoints = upImpl->forward(inputData, rects, people, 1);
                mFaceKeypoints.reset({people, (int)FACE_NUMBER_PARTS, 3}, 0.f);
                if (keypoints.size() != mFaceKeypoints.getVolume())
                    error("The face net does not have 70 parts.", __LINE__, __FUNCTION__, __FILE__);
                std::copy(keypoints.begin(), keypoints.end(), mFaceKeypoints.getPtr());
                if (!mHeatMapTypes.empty())
                    upImpl->copyHeatMaps(mHeatMaps, 0);
            }
            else
                mFaceKeypoints.reset();
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
        }
    }

    struct HandExtractorCaffe::ImplHandExtractorCaffe : KeypointNetHip {};

    HandExtractorCaffe::HandExtractorCaffe(const Point<int>& netInputSize, const Point<int>& netOutputSize,
                                           const std::string& modelFolder, const int gpuId,
                                           const int numberScales, const float rangeScales,
                                           const std::vector<HeatMapType>& heatMapTypes,
                                           const ScaleMode heatMapScaleMode, const bool enableGoogleLogging) :
        HandExtractorNet{netInputSize, netOutputSize, numberScales, rangeScales, heatMapTypes, heatMapScaleMode},
        upImpl{new ImplHandExtractorCaffe{}}
    {
        (void)enableGoogleLogging;
        if (!heatMapTypes.empty())   // handExtractorCaffe.cpp:327-332,433-441
            upImpl->heatMapScaleMode = (int)heatMapScaleMode;
        upImpl->proto = modelFolder + HAND_PROTOTXT;
        upImpl->model = modelFolder + HAND_TRAINED_MODEL;
        upImpl->gpuId = gpuId;
    }

    HandExtractorCaffe::~HandExtractorCaffe()
    {
    }

    void HandExtractorCaffe::netInitializationOnThread()
    {
        upImpl->initialize(OPK_EXTRACT_HAND, mNetOutputSize);
        check(opk_extractor_set_scales(upImpl->ex, mMultiScaleNumberAndRange.first,
                                       mMultiScaleNumberAndRange.second), __LINE__, __FUNCTION__);
    }

    void HandExtractorCaffe::forwardPass(const std::vector<std::array<Rectangle<float>, 2>> handRectangles,
                                         const Matrix& inputData)
    {
        try
        {
            if (mEnabled && !handRectangles.empty())
            {
                std::vector<float> rects;
                for (const auto& pair : handRectangles)
                {
                    pushRectangle(rects, pair[0]);
                    pushRectangle(rects, pair[1]);
                }
                const int people = (int)handRectangles.size();
                const auto keypoints = upImpl->forward(inputData, rects, people, 2);
                const size_t half = keypoints.size() / 2;
                for (auto hand = 0; hand < 2; hand++)
                {
                    mHandKeypoints[hand].reset({people, (int)HAND_NUMBER_PARTS, 3}, 0.f);
                    if (half != mHandKeypoints[hand].getVolume())
                        error("The hand net does not have 21 parts.", __LINE__, __FUNCTION__, __FILE__);
                    std::copy(keypoints.begin() + hand * half, keypoints.begin() + (hand + 1) * half,
                              mHandKeypoints[hand].getPtr());
                    if (!mHeatMapTypes.empty())
                        upImpl->copyHeatMaps(mHeatMaps[hand], hand);
                }
            }
            else
            {
                mHandKeypoints[0].reset();
                mHandKeypoints[1].reset();
            }
        }
        catch (const std::exception& e)
        {
            error(e.what(), __LINE__, __FUNCTION__, __FILE__);
        }
    }
}
