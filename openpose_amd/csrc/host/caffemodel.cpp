// caffemodel.cpp -- reader for Caffe's binary weight files (*.caffemodel).
//
// The reference loads trained weights with caffe::Net::CopyTrainedLayersFrom
// (src/openpose/net/netCaffe.cpp:163-185; Caffe is third-party: CMU fork 1807aad,
// CMakeLists.txt:728-732).  A .caffemodel is a serialized caffe.NetParameter in protobuf wire
// format; only the parts that carry weights are decoded here:
//   NetParameter     2: V1LayerParameter layers (legacy)   100: LayerParameter layer
//   LayerParameter   1: name  7: BlobProto blobs
//   V1LayerParameter 4: name  6: BlobProto blobs
//   BlobProto        1-4: num/channels/height/width (legacy shape)  5: float data
//                    7: BlobShape shape {1: int64 dim}  8: double data
// Repeated numeric fields are accepted packed or unpacked; every other field is skipped by wire
// type.  Truncated or malformed input throws (op::error in the reference: ReadProtoFromBinaryFile).
#include "caffemodel.h"

#include <cstring>
#include <fstream>
#include <iterator>

#include "../common.h"

namespace opk {

namespace {

struct Reader {
    const uint8_t* p;
    const uint8_t* end;
    bool done() const { return p >= end; }
    uint64_t varint()
    {
        uint64_t v = 0;
        for (int shift = 0; shift < 64; shift += 7) {
            OPK_CHECK_ARG(p < end, "caffemodel: truncated varint");
            const uint8_t b = *p++;
            v |= (uint64_t)(b & 0x7f) << shift;
            if (!(b & 0x80)) return v;
        }
        throw Error(1, "caffemodel: varint too long");
    }
    Reader sub()   // length-delimited payload
    {
        const uint64_t n = varint();
        OPK_CHECK_ARG(n <= (uint64_t)(end - p), "caffemodel: truncated field");
        Reader r{p, p + n};
        p += n;
        return r;
    }
    void skip(int wire)
    {
        switch (wire) {
        case 0: (void)varint(); break;
        case 1: OPK_CHECK_ARG(end - p >= 8, "caffemodel: truncated"); p += 8; break;
        case 2: (void)sub(); break;
        case 5: OPK_CHECK_ARG(end - p >= 4, "caffemodel: truncated"); p += 4; break;
        default: throw Error(1, "caffemodel: unsupported wire type " + std::to_string(wire));
        }
    }
    template <class T>
    T fixed()
    {
        OPK_CHECK_ARG((size_t)(end - p) >= sizeof(T), "caffemodel: truncated");
        T v;
        std::memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        return v;
    }
};

CaffeBlob parse_blob(Reader r)
{
    CaffeBlob b;
    int64_t legacy[4] = {0, 0, 0, 0};
    bool has_legacy = false;
    std::vector<double> dbl;
    while (!r.done()) {
        const uint64_t key = r.varint();
        const int field = (int)(key >> 3), wire = (int)(key & 7);
        if (field >= 1 && field <= 4 && wire == 0) {
            legacy[field - 1] = (int64_t)r.varint();
            has_legacy = true;
        } else if (field == 5 && wire == 2) {   // packed float data
            Reader d = r.sub();
            OPK_CHECK_ARG((d.end - d.p) % 4 == 0, "caffemodel: packed float data");
            const size_t n = (size_t)(d.end - d.p) / 4, at = b.data.size();
            b.data.resize(at + n);
            std::memcpy(b.data.data() + at, d.p, n * 4);
        } else if (field == 5 && wire == 5) {
            b.data.push_back(r.fixed<float>());
        } else if (field == 8 && wire == 2) {   // packed double data
            Reader d = r.sub();
            while (!d.done()) dbl.push_back(d.fixed<double>());
        } else if (field == 8 && wire == 1) {
            dbl.push_back(r.fixed<double>());
        } else if (field == 7 && wire == 2) {   // BlobShape
            Reader s = r.sub();
            while (!s.done()) {
                const uint64_t k = s.varint();
                if ((k >> 3) == 1 && (k & 7) == 2) {
                    Reader d = s.sub();
                    while (!d.done()) b.shape.push_back((int64_t)d.varint());
                } else if ((k >> 3) == 1 && (k & 7) == 0) {
                    b.shape.push_back((int64_t)s.varint());
                } else {
                    s.skip((int)(k & 7));
                }
            }
        } else {
            r.skip(wire);
        }
    }
    if (b.data.empty() && !dbl.empty()) b.data.assign(dbl.begin(), dbl.end());
    if (b.shape.empty() && has_legacy) {   // Blob::FromProto's legacy (num, channels, h, w)
        b.shape.assign(legacy, legacy + 4);
        b.legacy = true;
    }
    int64_t count = b.shape.empty() ? 0 : 1;
    for (int64_t d : b.shape) count *= d;
    OPK_CHECK_ARG(count == (int64_t)b.data.size(),
                  "caffemodel: blob data size " + std::to_string(b.data.size()) +
                      " differs from its shape (" + std::to_string(count) + ")");
    return b;
}

void parse_layer(Reader r, int name_field, int blobs_field, std::vector<CaffeLayer>& out)
{
    CaffeLayer L;
    while (!r.done()) {
        const uint64_t key = r.varint();
        const int field = (int)(key >> 3), wire = (int)(key & 7);
        if (field == name_field && wire == 2) {
            Reader s = r.sub();
            L.name.assign(reinterpret_cast<const char*>(s.p), (size_t)(s.end - s.p));
        } else if (field == blobs_field && wire == 2) {
            L.blobs.push_back(parse_blob(r.sub()));
        } else {
            r.skip(wire);
        }
    }
    if (!L.blobs.empty()) out.push_back(std::move(L));
}

}  // namespace

std::vector<CaffeLayer> parse_caffemodel(const uint8_t* data, size_t size)
{
    std::vector<CaffeLayer> out;
    Reader r{data, data + size};
    while (!r.done()) {
        const uint64_t key = r.varint();
        const int field = (int)(key >> 3), wire = (int)(key & 7);
        if (field == 100 && wire == 2)
            parse_layer(r.sub(), 1, 7, out);   // LayerParameter
        else if (field == 2 && wire == 2)
            parse_layer(r.sub(), 4, 6, out);   // V1LayerParameter (UpgradeV1Net keeps names/blobs)
        else
            r.skip(wire);
    }
    return out;
}

std::vector<CaffeLayer> load_caffemodel(const std::string& path)
{
    std::ifstream f(path, std::ios::binary);
    OPK_CHECK_ARG(f.good(), "cannot open caffemodel " + path);
    std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    return parse_caffemodel(bytes.data(), bytes.size());
}

bool blob_shape_is(const CaffeBlob& b, const std::vector<int64_t>& want)
{
    if (!b.legacy) return b.shape == want;
    // Blob::ShapeEquals for legacy blobs: the shape right-aligned into (num, channels, h, w)
    if (want.size() > 4) return false;
    std::vector<int64_t> l(4 - want.size(), 1);
    l.insert(l.end(), want.begin(), want.end());
    return l == b.shape;
}

}  // namespace opk
