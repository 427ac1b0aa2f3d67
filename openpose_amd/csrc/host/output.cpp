// output.cpp -- the reference's keypoint post-steps on the host: KeypointScaler and KeepTopNPeople.
//
// Both run on the small keypoint arrays the connector produced (people x parts x 3 floats), after
// the GPU work; they are restated here so a caller of libopk_hip gets the reference's output
// contract without the Wrapper.  Built with -ffp-contract=off (float operations as the CPU does).
#include "output.h"

#include <algorithm>
#include <cmath>
#include <functional>
#include <limits>
#include <vector>

#include "../common.h"

namespace opk {

namespace {
// op::ScaleMode (include/openpose/core/enumClasses.hpp:6-17)
enum { kInputResolution, kNetOutputResolution, kOutputResolution, kZeroToOne, kZeroToOneFixed,
       kPlusMinusOne, kPlusMinusOneFixed, kUnsignedChar, kNoScale };

// getKeypointsRectangle(...).area() (src/openpose/utilities/keypoint.cpp:289-340,378-389)
float keypoints_area(const float* person, int parts, float threshold)
{
    float minX = std::numeric_limits<float>::max(), maxX = std::numeric_limits<float>::lowest();
    float minY = minX, maxY = maxX;
    for (int part = 0; part < parts; ++part) {
        if (person[3 * part + 2] > threshold) {
            const float x = person[3 * part], y = person[3 * part + 1];
            if (maxX < x) maxX = x;
            if (minX > x) minX = x;
            if (maxY < y) maxY = y;
            if (minY > y) minY = y;
        }
    }
    if (maxX >= minX && maxY >= minY) return (maxX - minX) * (maxY - minY);
    return 0.f;
}
}  // namespace

void scale_keypoints(float* kp, int people, int parts, int mode, double scale_input_to_output,
                     double scale_net_to_output, int producer_w, int producer_h)
{
    // KeypointScaler::scale (src/openpose/core/keypointScaler.cpp:64-95) with getScaleAndOffset (:6-45)
    OPK_CHECK_ARG(people >= 0 && parts > 0 && (people == 0 || kp), "bad keypoint array");
    if (mode == kInputResolution) return;
    float ox = 0.f, oy = 0.f, sx, sy;
    if (mode == kOutputResolution) {
        sx = sy = float(scale_input_to_output);
    } else if (mode == kNetOutputResolution) {
        sx = sy = float(1. / scale_net_to_output);
    } else if (mode == kZeroToOne) {
        sx = 1.f / ((float)producer_w - 1.f);
        sy = 1.f / ((float)producer_h - 1.f);
    } else if (mode == kZeroToOneFixed) {
        sx = sy = 1.f / ((float)std::max(producer_w, producer_h) - 1.f);
    } else if (mode == kPlusMinusOne) {
        ox = oy = -1.f;
        sx = 2.f / ((float)producer_w - 1.f);
        sy = 2.f / ((float)producer_h - 1.f);
    } else if (mode == kPlusMinusOneFixed) {
        ox = oy = -1.f;
        sx = sy = 2.f / ((float)std::max(producer_w, producer_h) - 1.f);
    } else {
        throw Error(1, "Unknown ScaleMode selected.");
    }
    // scaleKeypoints2d (src/openpose/utilities/keypoint.cpp:106-169)
    const bool offset = !(ox == 0 && oy == 0);
    if (!offset && sx == 1.f && sy == 1.f) return;
    for (int i = 0; i < people * parts; ++i) {
        float* k = kp + 3 * (size_t)i;
        if (offset) {
            k[0] = k[0] * sx + ox;
            k[1] = k[1] * sy + oy;
        } else {
            k[0] *= sx;
            k[1] *= sy;
        }
    }
}

int keep_top_n_people(const float* kp, int people, int parts, const float* scores, int max_people,
                      float* out_kp, int* out_index)
{
    // KeepTopNPeople::keepTopPeople (src/openpose/core/keepTopNPeople.cpp:16-86)
    OPK_CHECK_ARG(people >= 0 && parts > 0 && (people == 0 || (kp && scores)), "bad arrays");
    const size_t area = (size_t)parts * 3;
    if (!(people > max_people && max_people > 0)) {   // no change
        if (out_kp && people) std::copy(kp, kp + people * area, out_kp);
        if (out_index) for (int p = 0; p < people; ++p) out_index[p] = p;
        return people;
    }
    std::vector<float> fin(scores, scores + people);
    for (int p = 0; p < people; ++p) fin[p] *= std::sqrt(keypoints_area(kp + p * area, parts, 0.05f));
    std::vector<float> sorted(fin);
    std::sort(sorted.begin(), sorted.end(), std::greater<float>());
    const float threshold = sorted[max_people - 1];
    int above = 0;
    for (int p = 0; p < people; ++p)
        if (fin[p] > threshold) ++above;
    const int on_threshold_to_add = max_people - above;
    int assigned_on_threshold = 0, next = 0;
    for (int p = 0; p < people; ++p) {
        if (fin[p] >= threshold) {
            if (fin[p] == threshold) ++assigned_on_threshold;
            if (fin[p] > threshold || assigned_on_threshold <= on_threshold_to_add) {
                if (out_kp) std::copy(kp + p * area, kp + (p + 1) * area, out_kp + next * area);
                if (out_index) out_index[next] = p;
                ++next;
            }
        }
    }
    // the reference's output array always has max_people rows (zeros beyond `next`)
    if (out_kp)
        std::fill(out_kp + next * area, out_kp + max_people * area, 0.f);
    return max_people;
}

}  // namespace opk
