// output.h -- KeypointScaler and KeepTopNPeople on host keypoint arrays (internal).
#pragma once

namespace opk {

// KeypointScaler::scale (keypointScaler.cpp:64-95): kp [people][parts][3] in place;
// mode = op::ScaleMode value (InputResolution = no change)
void scale_keypoints(float* kp, int people, int parts, int mode, double scale_input_to_output,
                     double scale_net_to_output, int producer_w, int producer_h);
// KeepTopNPeople::keepTopPeople (keepTopNPeople.cpp:16-86): returns the output row count (people
// unchanged when people <= max_people or max_people <= 0, else max_people); out_kp gets the rows,
// out_index the source person of each kept row (may be NULL)
int keep_top_n_people(const float* kp, int people, int parts, const float* scores, int max_people,
                      float* out_kp, int* out_index);

}  // namespace opk
