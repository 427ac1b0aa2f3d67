// pose_model.h -- pose tables and default thresholds (host side), mirroring op::poseParameters.
#pragma once
#include <vector>

namespace opk {

struct PoseModelInfo {
    int id;
    const char* name;
    int parts;                      // getPoseNumberBodyParts
    bool bkg;                       // addBkgChannel
    std::vector<int> pairs;         // getPosePartPairs (2 per pair)
    std::vector<int> map_idx;       // getPoseMapIndex  (2 per pair, relative to parts+bkg)
    float nms_th, inter_th;         // getPoseDefaultNmsThreshold / ConnectInterThreshold
    float nms_th_maxpos, inter_th_maxpos;   // ... with maximizePositives
    // body-part indices the face / hand detectors read (PoseKey below; -1: not in the model)
    std::vector<int> keys;
    int npairs() const { return (int)pairs.size() / 2; }
    // net output channels: heat maps, background, PAFs (the PAF channels the pairs index)
    int heat_channels() const { return parts + (bkg ? 1 : 0) + (int)map_idx.size(); }
    // connectBodyPartsCpu only accepts these (bodyPartConnectorBase.cpp:165-167)
    bool cpu_connector() const { return parts == 25 || parts == 18 || parts == 15; }
};

constexpr int kPoseModels = 15;   // PoseModel::Size (enumClasses.hpp:9-30)
// indices into PoseModelInfo::keys (faceDetector.cpp:8-15, handDetector.cpp:120-123)
enum PoseKey { kNeck, kNose, kLEar, kREar, kLEye, kREye, kLWrist, kLElbow, kLShoulder, kRWrist,
               kRElbow, kRShoulder, kDetectorKeys };

// throws opk::Error(OPK_ERR_UNSUPPORTED) for ids outside [0, kPoseModels)
const PoseModelInfo& pose_model(int id);

constexpr int kPoseMaxPeople = 127;   // poseParameters.hpp:14

}  // namespace opk
