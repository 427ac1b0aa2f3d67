// pose_model.cpp -- pose tables of every PoseModel (include/openpose/pose/enumClasses.hpp:9-30).
// The values are data generated from the reference's src/openpose/pose/poseParameters.cpp by
// tools/gen_pose_tables.py (pose_tables.inc) and pinned by tests/test_pose_tables.py.
#include "pose_model.h"

#include <string>

#include "../common.h"

namespace opk {

namespace {
struct PoseTableRow {
    int id;
    const char* name;
    int parts;
    bool bkg;
    const int* pairs;
    int npairs2;
    const int* map;
    int nmap;
    float nms_th, inter_th, nms_th_maxpos, inter_th_maxpos;
    const int* keys;
};
#include "pose_tables.inc"
}  // namespace

const PoseModelInfo& pose_model(int id)
{
    static const std::vector<PoseModelInfo> models = [] {
        std::vector<PoseModelInfo> v;
        for (const PoseTableRow& r : kPoseTableRows)
            v.push_back(PoseModelInfo{r.id, r.name, r.parts, r.bkg,
                                      std::vector<int>(r.pairs, r.pairs + r.npairs2),
                                      std::vector<int>(r.map, r.map + r.nmap), r.nms_th, r.inter_th,
                                      r.nms_th_maxpos, r.inter_th_maxpos,
                                      std::vector<int>(r.keys, r.keys + kDetectorKeys)});
        return v;
    }();
    if (id < 0 || id >= (int)models.size())
        throw Error(4, "pose model " + std::to_string(id) + " has no tables in libopk_hip");
    return models[id];
}

}  // namespace opk
