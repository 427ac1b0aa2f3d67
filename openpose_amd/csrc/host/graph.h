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
// models/pose/{coco,mpi}/pose_deploy_linevec*.prototxt (pafs/heat channels, 4 or 6 stages)
std::vector<LayerDesc> builtin_cpm_pose(int pafs, int heat, int stages);
// models/{hand,face}/pose_deploy.prototxt (22 / 71 outputs)
std::vector<LayerDesc> builtin_cpm_single(int outputs, bool face);
// "builtin:BODY_25" | COCO_18 | MPI_15 | MPI_15_4 | HAND | FACE
std::vector<LayerDesc> builtin_graph(const std::string& name);

}  // namespace opk
