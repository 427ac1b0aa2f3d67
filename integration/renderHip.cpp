// renderHip.cpp -- drop-in replacement of the reference's CUDA render translation units, compiled
// INSIDE the reference tree (against include/openpose/...) and linked with libopk_hip.so.
//
// Defines, with the reference's exact signatures:
//   op::renderPoseKeypointsGpu, op::renderPoseHeatMapGpu, op::renderPoseHeatMapsGpu,
//   op::renderPosePAFGpu, op::renderPosePAFsGpu, op::renderPoseDistanceGpu
//       (include/openpose/pose/renderPose.hpp:14-42, replaces src/openpose/pose/renderPose.cu)
//   op::renderFaceKeypointsGpu (include/openpose/face/renderFace.hpp:12-15, replaces
//       src/openpose/face/renderFace.cu)
//   op::renderHandKeypointsGpu (include/openpose/hand/renderHand.hpp:12-15, replaces
//       src/openpose/hand/renderHand.cu)
// so PoseGpuRenderer / FaceGpuRenderer / HandGpuRenderer (poseGpuRenderer.cpp, faceGpuRenderer.cpp,
// handGpuRenderer.cpp) draw through libopk_hip.so unchanged.  The maxPtr / minPtr / scalePtr scratch
// those renderers allocate is not needed (the boxes live in the context); it is accepted and left
// untouched.  Work runs on the calling thread's context (openpose_hip_shim.cpp) and is complete when
// the call returns; errors come back through op::error like the reference's cudaCheck.
#include <string>

#include <openpose/face/renderFace.hpp>
#include <openpose/hand/renderHand.hpp>
#include <openpose/pose/renderPose.hpp>

#include "opk.h"
#include "opk_shim.hpp"

namespace op
{
    namespace
    {
        void run(const int rc, const int line, const char* function)
        {
            if (rc != OPK_OK)
                error(std::string{"libopk_hip: "} + opk_last_error(), line, function, __FILE__);
            if (opk_sync(opkShimThreadContext().get()) != OPK_OK)
                error(std::string{"libopk_hip: "} + opk_last_error(), line, function, __FILE__);
        }
    }

    void renderPoseKeypointsGpu(
        float* framePtr, float* maxPtr, float* minPtr, float* scalePtr, const PoseModel poseModel,
        const int numberPeople, const Point<unsigned int>& frameSize, const float* const posePtr,
        const float renderThreshold, const bool googlyEyes, const bool blendOriginalFrame,
        const float alphaBlending)
    {
        (void)maxPtr;
        (void)minPtr;
        (void)scalePtr;
        run(opk_render_pose_keypoints(opkShimThreadContext().get(), framePtr, (int)poseModel, numberPeople,
                                      frameSize.x, frameSize.y, posePtr, renderThreshold,
                                      googlyEyes ? 1 : 0, blendOriginalFrame ? 1 : 0, alphaBlending),
            __LINE__, __FUNCTION__);
    }

    void renderPoseHeatMapGpu(
        float* frame, const Point<unsigned int>& frameSize, const float* const heatMapPtr,
        const Point<int>& heatMapSize, const float scaleToKeepRatio, const unsigned int part,
        const float alphaBlending)
    {
        run(opk_render_pose_heat_map(opkShimThreadContext().get(), frame, frameSize.x, frameSize.y,
                                     heatMapPtr, heatMapSize.x, heatMapSize.y, scaleToKeepRatio,
                                     part, alphaBlending),
            __LINE__, __FUNCTION__);
    }

    void renderPoseHeatMapsGpu(
        float* frame, const PoseModel poseModel, const Point<unsigned int>& frameSize,
        const float* const heatMapPtr, const Point<int>& heatMapSize, const float scaleToKeepRatio,
        const float alphaBlending)
    {
        run(opk_render_pose_heat_maps(opkShimThreadContext().get(), frame, (int)poseModel, frameSize.x,
                                      frameSize.y, heatMapPtr, heatMapSize.x, heatMapSize.y,
                                      scaleToKeepRatio, alphaBlending),
            __LINE__, __FUNCTION__);
    }

    void renderPosePAFGpu(
        float* framePtr, const PoseModel poseModel, const Point<unsigned int>& frameSize,
        const float* const heatMapPtr, const Point<int>& heatMapSize, const float scaleToKeepRatio,
        const int part, const float alphaBlending)
    {
        run(opk_render_pose_paf(opkShimThreadContext().get(), framePtr, (int)poseModel, frameSize.x,
                                frameSize.y, heatMapPtr, heatMapSize.x, heatMapSize.y,
                                scaleToKeepRatio, part, alphaBlending),
            __LINE__, __FUNCTION__);
    }

    void renderPosePAFsGpu(
        float* framePtr, const PoseModel poseModel, const Point<unsigned int>& frameSize,
        const float* const heatMapPtr, const Point<int>& heatMapSize, const float scaleToKeepRatio,
        const float alphaBlending)
    {
        run(opk_render_pose_pafs(opkShimThreadContext().get(), framePtr, (int)poseModel, frameSize.x,
                                 frameSize.y, heatMapPtr, heatMapSize.x, heatMapSize.y,
                                 scaleToKeepRatio, alphaBlending),
            __LINE__, __FUNCTION__);
    }

    void renderPoseDistanceGpu(
        float* framePtr, const Point<unsigned int>& frameSize, const float* const heatMapPtr,
        const Point<int>& heatMapSize, const float scaleToKeepRatio, const unsigned int part,
        const float alphaBlending)
    {
        run(opk_render_pose_distance(opkShimThreadContext().get(), framePtr, frameSize.x, frameSize.y,
                                     heatMapPtr, heatMapSize.x, heatMapSize.y, scaleToKeepRatio,
                                     part, alphaBlending),
            __LINE__, __FUNCTION__);
    }

    void renderFaceKeypointsGpu(
        float* framePtr, float* maxPtr, float* minPtr, float* scalePtr,
        const Point<unsigned int>& frameSize, const float* const facePtr, const int numberPeople,
        const float renderThreshold, const float alphaColorToAdd)
    {
        (void)maxPtr;
        (void)minPtr;
        (void)scalePtr;
        run(opk_render_face_keypoints(opkShimThreadContext().get(), framePtr, frameSize.x, frameSize.y,
                                      facePtr, numberPeople, renderThreshold, alphaColorToAdd),
            __LINE__, __FUNCTION__);
    }

    void renderHandKeypointsGpu(
        float* framePtr, float* maxPtr, float* minPtr, float* scalePtr,
        const Point<unsigned int>& frameSize, const float* const handsPtr, const int numberHands,
        const float renderThreshold, const float alphaColorToAdd)
    {
        (void)maxPtr;
        (void)minPtr;
        (void)scalePtr;
        run(opk_render_hand_keypoints(opkShimThreadContext().get(), framePtr, frameSize.x, frameSize.y,
                                      handsPtr, numberHands, renderThreshold, alphaColorToAdd),
            __LINE__, __FUNCTION__);
    }
}
