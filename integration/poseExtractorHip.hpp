// poseExtractorHip.hpp -- op::PoseExtractorHip: the body-pose extractor of the reference pipeline
// on libopk_hip, with no Caffe and no CUDA anywhere.
//
// The reference's only PoseExtractorNet is PoseExtractorCaffe, whose forwardPass body compiles
// only under USE_CAFFE (src/openpose/pose/poseExtractorCaffe.cpp:205) and whose Caffe layers reach
// the *Gpu functions only under USE_CUDA (resizeAndMergeCaffe.cpp:131-140, nmsCaffe.cpp:187-196,
// bodyPartConnectorCaffe.cpp:210-219).  On an MI355X box neither exists, so the pipeline's seam
// is PoseExtractorNet itself (include/openpose/pose/poseExtractorNet.hpp:10-79): this class has
// PoseExtractorCaffe's constructor (poseExtractorCaffe.hpp:17-23) and is constructed where the
// Wrapper constructs that one (include/openpose/wrapper/wrapperAuxiliary.hpp:329).  One call runs
// the net of every scale, the merged x8 resize, NMS and the connector on the GPU
// (opk_pose_forward / opk_pose_forward_multi) and fills mPoseKeypoints / mPoseScores; heat maps
// and candidates are copied out only when asked for (getHeatMapsCopy / getCandidatesCopy).
#ifndef OPENPOSE_POSE_POSE_EXTRACTOR_HIP_HPP
#define OPENPOSE_POSE_POSE_EXTRACTOR_HIP_HPP

#include <memory>
#include <string>
#include <vector>

#include <openpose/core/common.hpp>
#include <openpose/pose/poseExtractorNet.hpp>

namespace op
{
    class OP_API PoseExtractorHip : public PoseExtractorNet
    {
    public:
        PoseExtractorHip(
            const PoseModel poseModel, const std::string& modelFolder, const int gpuId,
            const std::vector<HeatMapType>& heatMapTypes = {},
            const ScaleMode heatMapScaleMode = ScaleMode::ZeroToOneFixedAspect,
            const bool addPartCandidates = false, const bool maximizePositives = false,
            const std::string& protoTxtPath = "", const std::string& caffeModelPath = "",
            const float upsamplingRatio = 0.f, const bool enableNet = true,
            const bool enableGoogleLogging = true);

        virtual ~PoseExtractorHip();

        virtual void netInitializationOnThread();

        virtual void forwardPass(
            const std::vector<Array<float>>& inputNetData, const Point<int>& inputDataSize,
            const std::vector<double>& scaleInputToNetInputs = {1.f},
            const Array<float>& poseNetOutput = Array<float>{});

        const float* getCandidatesCpuConstPtr() const;

        const float* getCandidatesGpuConstPtr() const;

        const float* getHeatMapCpuConstPtr() const;

        const float* getHeatMapGpuConstPtr() const;

        std::vector<int> getHeatMapSize() const;

        const float* getPoseGpuConstPtr() const;

    private:
        struct ImplPoseExtractorHip;
        std::unique_ptr<ImplPoseExtractorHip> upImpl;

        DELETE_COPY(PoseExtractorHip);
    };
}

#endif // OPENPOSE_POSE_POSE_EXTRACTOR_HIP_HPP
