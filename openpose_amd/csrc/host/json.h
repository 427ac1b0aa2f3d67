// json.h -- people JSON writer (op::savePeopleJson) on host arrays (internal).
#pragma once
#include <string>

#include "../../../include/opk.h"

namespace opk {

using JsonKeypoints = opk_json_keypoints;

// The file content op::savePeopleJson writes (fileStream.cpp:306-344).  candidates: n_parts lists
// of [x, y, score] laid out back to back, candidate_counts[part] entries each (n_parts 0: no
// "part_candidates" key, as with an empty poseCandidates vector).
std::string people_json(const JsonKeypoints* arrays, int n_arrays, const float* candidates,
                        const int* candidate_counts, int n_parts, bool human_readable);
void save_people_json(const std::string& path, const std::string& text);

}  // namespace opk
