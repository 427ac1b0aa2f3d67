// pose_model.h -- pose tables and default thresholds (host side), mirroring op::poseParameters.
#pragma once
#include <vector>

namespace opk {

struct PoseModelInfo {
    int id;
    int parts;                      // getPoseNumberBodyParts
    bool bkg;                       // addBkgChannel
    std::vector<int> pairs;         // getPosePartPairs (2 per pair)
    std::vector<int> map_idx;       // getPoseMapIndex  (2 per pair, relative to parts+bkg)
    int npairs() const { return (int)pairs.size() / 2; }
    int heat_channels() const { return parts + (bkg ? 1 : 0) + (int)map_idx.size(); }
};

// throws opk::Error(OPK_ERR_UNSUPPORTED) for models without tables here
const PoseModelInfo& pose_model(int id);

constexpr int kPoseMaxPeople = 127;   // poseParameters.hpp:14

}  // namespace opk
