// graph.h -- Caffe network description (prototxt subset used by the OpenPose pose models).
#pragma once
#include <string>
#include <vector>

namespace opk {

struct LayerDesc {
    std::string name, type;
    std::vector<std::string> bottom, top;
    int num_output = 0, kernel_size = 0, pad = 0, stride = 1;   // Convolution / Pooling
    std::string pool = "MAX";
    int concat_axis = 1;
};

// Parses the prototxt text (layer { ... } blocks; other top-level keys ignored).
std::vector<LayerDesc> parse_prototxt(const std::string& text);
std::vector<LayerDesc> load_prototxt(const std::string& path);
// models/pose/body_25/pose_deploy.prototxt, generated (261 layers)
std::vector<LayerDesc> builtin_body25();

}  // namespace opk
