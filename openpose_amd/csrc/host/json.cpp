// json.cpp -- the reference's people JSON output (--write_json) on host keypoint arrays.
//
// Restates op::savePeopleJson (src/openpose/filestream/fileStream.cpp:306-344) with
// addKeypointsToJson (:20-85), addCandidatesToJson (:87-130) and the JsonOfstream formatting
// (src/openpose/filestream/jsonOfstream.cpp: '{' / '[' counters, "\n" + one tab per open brace or
// bracket when human readable; include/openpose/filestream/jsonOfstream.hpp:40-50: values through
// std::ostream's default float format).  The array shapes follow op::Array::getSize
// (src/openpose/core/array.cpp:421-437): a missing dimension counts 1, an empty array 0, so a
// 1-D person_id array writes one value per person and an empty array writes "[]".
#include "json.h"

#include <algorithm>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>

#include "../common.h"

namespace opk {

namespace {

class JsonWriter {
public:
    explicit JsonWriter(bool human) : human_(human) {}
    void object_open()
    {
        ++braces_;
        s_ << "{";
    }
    void object_close()
    {
        --braces_;
        enter();
        s_ << "}";
    }
    void array_open()
    {
        ++brackets_;
        s_ << "[";
        enter();
    }
    void array_close()
    {
        --brackets_;
        enter();
        s_ << "]";
    }
    void key(const std::string& k)
    {
        enter();
        s_ << "\"" << k << "\":";
    }
    void comma() { s_ << ","; }
    void value(float v) { s_ << v; }   // std::ostream default: %g, 6 significant digits
    void text(const char* t) { s_ << t; }
    void enter()
    {
        if (!human_) return;
        s_ << "\n";
        for (long long i = 0; i < braces_ + brackets_; ++i) s_ << "\t";
    }
    std::string finish()
    {
        enter();   // ~JsonOfstream (jsonOfstream.cpp:80-100)
        OPK_CHECK_ARG(braces_ == 0 && brackets_ == 0, "Json file wrongly generated");
        return s_.str();
    }

private:
    bool human_;
    long long braces_ = 0, brackets_ = 0;
    std::ostringstream s_;
};

// op::Array::getSize(index) for an array of `nd` dimensions (0 = empty array)
int array_size(const JsonKeypoints& a, int index)
{
    if (a.ndims == 0) return 0;
    if (index < a.ndims) return index == 0 ? a.people : index == 1 ? a.parts : a.dims;
    return 1;
}

}  // namespace

std::string people_json(const JsonKeypoints* arrays, int n_arrays, const float* candidates,
                        const int* candidate_counts, int n_parts, bool human_readable)
{
    OPK_CHECK_ARG(n_arrays >= 0 && (n_arrays == 0 || arrays), "people_json: NULL keypoint arrays");
    for (int v = 0; v < n_arrays; ++v) {
        const auto& a = arrays[v];
        OPK_CHECK_ARG(a.name != nullptr, "people_json: keypoint array without a name");
        // fileStream.cpp:313-317
        OPK_CHECK_ARG(a.ndims == 0 || a.ndims == 1 || a.ndims == 3,
                      "keypointVector.getNumberDimensions() != 1 && != 3.");
        OPK_CHECK_ARG(a.ndims == 0 || a.people >= 0, "people_json: negative size");
        OPK_CHECK_ARG(a.ndims == 0 || a.people == 0 || a.data, "people_json: NULL data");
    }
    OPK_CHECK_ARG(n_parts >= 0 && (n_parts == 0 || candidate_counts),
                  "people_json: candidates without counts");
    JsonWriter j(human_readable);
    j.object_open();
    j.key("version");
    j.text("1.3");
    j.comma();
    // addKeypointsToJson
    j.key("people");
    j.array_open();
    int people = 0;
    for (int v = 0; v < n_arrays; ++v) people = std::max(people, array_size(arrays[v], 0));
    for (int p = 0; p < people; ++p) {
        j.object_open();
        for (int v = 0; v < n_arrays; ++v) {
            const auto& a = arrays[v];
            const long per_row = (long)array_size(a, 1) * array_size(a, 2);
            j.key(a.name);
            j.array_open();
            if (per_row > 0) {
                // the reference indexes person*per_row without a bound check; an array with fewer
                // people than the widest one would read past its end there -- refused here
                OPK_CHECK_ARG(p < a.people, std::string("people_json: ") + a.name +
                                                " has fewer people than another keypoint array");
                const float* row = a.data + (long)p * per_row;
                for (long e = 0; e + 1 < per_row; ++e) {
                    j.value(row[e]);
                    j.comma();
                }
                j.value(row[per_row - 1]);
            }
            j.array_close();
            if (v < n_arrays - 1) j.comma();
        }
        j.object_close();
        if (p < people - 1) {
            j.comma();
            j.enter();
        }
    }
    j.array_close();
    // addCandidatesToJson (only with candidates: fileStream.cpp:332-336)
    if (n_parts > 0) {
        j.comma();
        j.key("part_candidates");
        j.array_open();
        j.object_open();
        const float* c = candidates;
        for (int part = 0; part < n_parts; ++part) {
            j.key(std::to_string(part));
            j.array_open();
            const int n = candidate_counts[part];
            OPK_CHECK_ARG(n >= 0 && (n == 0 || candidates), "people_json: bad candidate list");
            for (int k = 0; k < n; ++k, c += 3) {
                j.value(c[0]);
                j.comma();
                j.value(c[1]);
                j.comma();
                j.value(c[2]);
                if (k < n - 1) j.comma();
            }
            j.array_close();
            if (part < n_parts - 1) j.comma();
        }
        j.object_close();
        j.array_close();
    }
    j.object_close();
    return j.finish();
}

void save_people_json(const std::string& path, const std::string& text)
{
    std::ofstream f(path, std::ios::binary);
    OPK_CHECK_ARG(f.is_open(), "Json file " + path + " could not be opened.");
    f << text;
    OPK_CHECK_ARG(f.good(), "Json file " + path + " could not be written.");
}

}  // namespace opk
