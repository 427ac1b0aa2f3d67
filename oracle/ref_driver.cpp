// ref_driver.cpp -- C entry points into the REFERENCE's own connector code (TEST INFRASTRUCTURE).
//
// Built by oracle/Makefile (target `ref`) together with these reference sources, compiled in
// place from /root/reference with the reference's own release flags (-O3 -fopenmp, no -march:
// CMakeLists.txt:103-137):
//   src/openpose/net/bodyPartConnectorBase.cpp  (createPeopleVector,
//                                               removePeopleBelowThresholdsAndFillFaces,
//                                               pafPtrIntoVector is NOT used: it needs Array<T>)
//   src/openpose/pose/poseParameters.cpp        (pose tables)
//   src/openpose/utilities/errorAndLog.cpp      (op::error)
//   src/openpose/core/point.cpp, core/rectangle.cpp
// Output: oracle/_ref/libref_connector.so (git-ignored).  Nothing here is copied from the
// reference; the reference files are compiled where they lie.
//
// Not built (they need OpenCV, absent from the image): core/array.cpp (op::Array<T>) and
// utilities/keypoint.cpp (getKeypointsRoi).  The library is linked with those symbols left
// unresolved; the entry points below only reach code paths that never call them for the
// BODY_25 / COCO / MPI models (Array<T> is touched only by the precomputed-score branch and by
// peopleVectorToPeopleArray, which this driver does not call; getKeypointsRoi only for >=135
// parts).  The final people -> array step (bodyPartConnectorBase.cpp:886-934) is a 10-line
// copy-out done here on the returned std::vector.
#include <cstring>
#include <vector>
#include <openpose/net/bodyPartConnectorBase.hpp>
#include <openpose/pose/poseParameters.hpp>

extern "C" int ref_connect_cpu(float* kp, float* ks, int max_people, const float* heat,
                               const float* peaks, int pose_model, int W, int H, int max_peaks,
                               float inter_min_above, float inter_th, int min_cnt, float min_score,
                               float nms_th, float scale, int maxpos)
{
    const auto model = (op::PoseModel)pose_model;
    const auto& pairs = op::getPosePartPairs(model);
    const auto nparts = op::getPoseNumberBodyParts(model);
    const auto npairs = (unsigned)(pairs.size() / 2);
    // createPeopleVector never reads its Array<T> argument when heatMapPtr != nullptr
    // (bodyPartConnectorBase.cpp:297-342); hand it inert storage instead of constructing an
    // op::Array (whose constructor lives in the OpenCV-dependent array.cpp).
    alignas(64) static unsigned char inert[4096] = {0};
    const auto& unused = *reinterpret_cast<const op::Array<float>*>(inert);
    auto people = op::createPeopleVector<float>(heat, peaks, model, op::Point<int>{W, H}, max_peaks,
                                                inter_th, inter_min_above, pairs, nparts, npairs,
                                                nms_th, unused);
    std::vector<int> valid;
    int npeople = 0;
    op::removePeopleBelowThresholdsAndFillFaces<float>(valid, npeople, people, nparts, min_cnt,
                                                       min_score, maxpos != 0, peaks);
    const float inv = 1 / float(nparts + npairs);
    for (int o = 0; o < (int)valid.size() && o < max_people; ++o) {
        const auto& pr = people[valid[o]];
        for (unsigned k = 0; k < nparts; ++k) {
            float* d = kp + ((size_t)o * nparts + k) * 3;
            const int s = pr.first[k];
            if (s > 0) { d[0] = peaks[s - 2] * scale; d[1] = peaks[s - 1] * scale; d[2] = peaks[s]; }
            else { d[0] = d[1] = d[2] = 0.f; }
        }
        ks[o] = pr.second * inv;
    }
    return (int)valid.size();
}
