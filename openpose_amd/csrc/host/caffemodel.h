// caffemodel.h -- Caffe binary weight files (caffe.NetParameter wire format), internal.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace opk {

struct CaffeBlob {
    std::vector<int64_t> shape;   // BlobShape dims, or the legacy (num, channels, height, width)
    bool legacy = false;
    std::vector<float> data;      // float data (double data converted)
};
struct CaffeLayer {
    std::string name;
    std::vector<CaffeBlob> blobs;
};

// Layers that carry blobs, in file order (LayerParameter and legacy V1LayerParameter).
std::vector<CaffeLayer> parse_caffemodel(const uint8_t* data, size_t size);
std::vector<CaffeLayer> load_caffemodel(const std::string& path);
// Caffe's Blob::ShapeEquals (legacy blobs compare right-aligned in 4-D)
bool blob_shape_is(const CaffeBlob& b, const std::vector<int64_t>& want);

}  // namespace opk
