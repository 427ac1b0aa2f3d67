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
// utilities/keypoint.cpp.  The library is linked with those symbols left unresolved; the entry
// points below never reach op::Array<T> (touched only by the precomputed-score branch and by
// peopleVectorToPeopleArray, which this driver does not call).  The one keypoint.cpp function the
// connector calls -- getKeypointsRoi(Rectangle, Rectangle), for the BODY_135 face-fragment merge
// (removePeopleBelowThresholdsAndFillFaces, bodyPartConnectorBase.cpp:799-866) -- is plain
// arithmetic, restated below (as pafPtrIntoVector's loop is further down), so that branch runs the
// reference's own code around it.  The final people -> array step (bodyPartConnectorBase.cpp:
// 886-934) is a 10-line copy-out done here on the returned std::vector.
#include <algorithm>
#include <cstring>
#include <functional>
#include <tuple>
#include <vector>
#include <openpose/net/bodyPartConnectorBase.hpp>
#include <openpose/pose/poseParameters.hpp>
#include <openpose/utilities/fastMath.hpp>
#include <openpose/utilities/keypoint.hpp>

namespace op
{
// getKeypointsRoi(Rectangle, Rectangle) (utilities/keypoint.cpp:586-632), restated: both rectangles
// shifted so that neither has a negative corner (the smallest negative x / y, or 0), then the
// intersection area over the union area in float; 0 when they do not overlap.  Subtracting a zero
// shift changes no value, so the shift is applied unconditionally.
template <typename T>
float getKeypointsRoi(const Rectangle<T>& a, const Rectangle<T>& b)
{
    const T sx = std::min(std::min(T{0}, a.x), b.x);
    const T sy = std::min(std::min(T{0}, a.y), b.y);
    Rectangle<T> ra = a, rb = b;
    ra.x -= sx;
    rb.x -= sx;
    ra.y -= sy;
    rb.y -= sy;
    const T left = fastMax(ra.x, rb.x), top = fastMax(ra.y, rb.y);
    const T right = fastMin(ra.x + ra.width, rb.x + rb.width);
    const T bottom = fastMin(ra.y + ra.height, rb.y + rb.height);
    if (!(left < right && top < bottom))
        return 0.f;
    const Rectangle<T> overlap{left, top, right - left, bottom - top};
    const auto areaA = ra.area(), areaB = rb.area(), inter = overlap.area();
    return float(inter) / float(areaA + areaB - inter);
}
template float getKeypointsRoi(const Rectangle<float>&, const Rectangle<float>&);
template float getKeypointsRoi(const Rectangle<double>&, const Rectangle<double>&);
}

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

// Pose tables of model `pose_model` as the reference computes them (poseParameters.cpp): writes
// up to `cap` pair entries and map entries; returns the number of pair entries (2 per pair), or
// -1 when a buffer is too small.  params: [0] parts, [1] bkg, [2] map entries, [3] NMS threshold,
// [4] inter threshold, [5] NMS threshold (maximizePositives), [6] inter threshold (maxpos).
extern "C" int ref_pose_table(int pose_model, unsigned* pairs, unsigned* map, int cap, float* params)
{
    const auto model = (op::PoseModel)pose_model;
    const auto& p = op::getPosePartPairs(model);
    const auto& m = op::getPoseMapIndex(model);
    if ((int)p.size() > cap || (int)m.size() > cap) return -1;
    std::memcpy(pairs, p.data(), p.size() * sizeof(unsigned));
    std::memcpy(map, m.data(), m.size() * sizeof(unsigned));
    params[0] = (float)op::getPoseNumberBodyParts(model);
    params[1] = op::addBkgChannel(model) ? 1.f : 0.f;
    params[2] = (float)m.size();
    params[3] = op::getPoseDefaultNmsThreshold(model, false);
    params[4] = op::getPoseDefaultConnectInterThreshold(model, false);
    params[5] = op::getPoseDefaultNmsThreshold(model, true);
    params[6] = op::getPoseDefaultConnectInterThreshold(model, true);
    return (int)p.size();
}

// the body-part indices the face and hand detectors read (faceDetector.cpp:8-15 with
// poseBodyPartMapStringToKey's name lists; handDetector.cpp:120-123, getPoseKeypoints): Neck,
// Nose|Head, LEar|Head, REar|Head, LEye|Head, REye|Head, LWrist, LElbow, LShoulder, RWrist,
// RElbow, RShoulder; -1 where the model has none of the names (the reference errors there)
extern "C" int ref_pose_keys(int pose_model, int* keys)
{
    const auto model = (op::PoseModel)pose_model;
    const std::vector<std::vector<std::string>> names = {
        {"Neck"}, {"Nose", "Head"}, {"LEar", "Head"}, {"REar", "Head"}, {"LEye", "Head"},
        {"REye", "Head"}, {"LWrist"}, {"LElbow"}, {"LShoulder"}, {"RWrist"}, {"RElbow"},
        {"RShoulder"}};
    for (size_t i = 0; i < names.size(); ++i) {
        try {
            keys[i] = (int)op::poseBodyPartMapStringToKey(model, names[i]);
        } catch (const std::exception&) {
            keys[i] = -1;
        }
    }
    return 0;
}

// pafPtrIntoVector's loop (it takes an op::Array: OpenCV-dependent array.cpp, not built), restated:
// collect (total, paf, q, i, j) for score > 1e-6 with total = paf + 0.1 sA + 0.1 sB, sort
// descending, then the reference's pafVectorIntoPeopleVector
static std::vector<std::pair<std::vector<int>, float>> gpu_people(const float* pair_scores,
                                                                  const float* peaks, int pose_model,
                                                                  int max_peaks)
{
    const auto model = (op::PoseModel)pose_model;
    const auto& pairs = op::getPosePartPairs(model);
    const auto nparts = op::getPoseNumberBodyParts(model);
    const auto npairs = (unsigned)(pairs.size() / 2);
    const int off = 3 * (max_peaks + 1);
    std::vector<std::tuple<float, float, int, int, int>> conn;
    for (unsigned q = 0; q < npairs; ++q) {
        const int pa = (int)pairs[2 * q], pb = (int)pairs[2 * q + 1];
        const int na = op::positiveIntRound(peaks[pa * off]);
        const int nb = op::positiveIntRound(peaks[pb * off]);
        for (int i = 0; i < na; ++i)
            for (int j = 0; j < nb; ++j) {
                const float s = pair_scores[((size_t)q * max_peaks + i) * max_peaks + j];
                if (s > 1e-6)
                    conn.emplace_back(s + 0.1f * peaks[pa * off + (i + 1) * 3 + 2] +
                                          0.1f * peaks[pb * off + (j + 1) * 3 + 2],
                                      s, (int)q, i + 1, j + 1);
            }
    }
    std::sort(conn.begin(), conn.end(), std::greater<std::tuple<double, double, int, int, int>>());
    return op::pafVectorIntoPeopleVector<float>(conn, peaks, max_peaks, pairs, nparts);
}

// 1 when removePeopleBelowThresholdsAndFillFaces will run its face-fragment merge (and so call
// getKeypointsRoi) on this input: a >= 135-part model with face-only fragments next to valid
// people with faces (its counting, bodyPartConnectorBase.cpp:740-798) -- the fixture generator
// checks that the BODY_135 face cases exercise that branch
extern "C" int ref_gpu_face_merge_reached(const float* pair_scores, const float* peaks,
                                          int pose_model, int max_peaks, int min_cnt,
                                          float min_score, int maxpos)
{
    const auto people = gpu_people(pair_scores, peaks, pose_model, max_peaks);
    if (op::getPoseNumberBodyParts((op::PoseModel)pose_model) < 135) return 0;
    auto disc = [](int& c, const std::vector<int>& r, int a, int b, int minimum) {
        int k = 0;
        for (int i = a; i < b; ++i) k += r[i] > 0;
        if (k > minimum) c += minimum - k;
    };
    std::function<bool(bool)> reaches = [&](bool mp) {
        int valid = 0, face_valid = 0, face_invalid = 0;
        for (const auto& p : people) {
            int c = p.first.back();
            const int before = c;
            disc(c, p.first, 65, 135, 1);
            if (c == 1) { ++face_invalid; continue; }
            if (c != before) ++face_valid;
            disc(c, p.first, 45, 65, 1);
            disc(c, p.first, 25, 45, 1);
            if (!mp) {
                const int b2 = c;
                disc(c, p.first, 19, 25, 0);
                if (c != b2 && c <= 4) continue;
            }
            if (c >= min_cnt && (p.second / c) >= min_score) ++valid;
        }
        if (valid > 0) return face_invalid > 0 && face_valid > 0;
        return !mp && reaches(true);
    };
    return reaches(maxpos != 0) ? 1 : 0;
}

// connectBodyPartsGpu's host half (bodyPartConnectorBase.cu:147-250) on host pair scores
// [npairs][max_peaks][max_peaks]: the restated pafPtrIntoVector loop, then the reference's
// pafVectorIntoPeopleVector, removePeopleBelowThresholdsAndFillFaces (face-fragment merge
// included) and the people -> array copy-out
extern "C" int ref_connect_gpu_assembly(float* kp, float* ks, int max_people,
                                        const float* pair_scores, const float* peaks,
                                        int pose_model, int max_peaks, int min_cnt,
                                        float min_score, float scale, int maxpos)
{
    const auto model = (op::PoseModel)pose_model;
    const auto nparts = op::getPoseNumberBodyParts(model);
    const auto npairs = (unsigned)(op::getPosePartPairs(model).size() / 2);
    auto people = gpu_people(pair_scores, peaks, pose_model, max_peaks);
    std::vector<int> keep;
    int npeople = 0;
    op::removePeopleBelowThresholdsAndFillFaces<float>(keep, npeople, people, nparts, min_cnt,
                                                       min_score, maxpos != 0, peaks);
    const float inv = 1 / float(nparts + npairs);
    for (int o = 0; o < (int)keep.size() && o < max_people; ++o) {
        const auto& pr = people[keep[o]];
        for (unsigned k = 0; k < nparts; ++k) {
            float* d = kp + ((size_t)o * nparts + k) * 3;
            const int s = pr.first[k];
            if (s > 0) { d[0] = peaks[s - 2] * scale; d[1] = peaks[s - 1] * scale; d[2] = peaks[s]; }
            else { d[0] = d[1] = d[2] = 0.f; }
        }
        ks[o] = pr.second * inv;
    }
    return (int)keep.size();
}
