// extract.h -- face / hand keypoint extraction: the op::FaceDetector / op::HandDetector rectangle
// rules and the op::FaceExtractorCaffe / op::HandExtractorCaffe forward passes, batched over every
// crop of a set of frames (internal).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "context.h"
#include "net.h"

namespace opk {

struct Rect {
    float x, y, width, height;
};

// FaceDetector::detectFaces (faceDetector.cpp:122-139): one square rectangle per person from the
// pose keypoints [people][parts][3] of pose model `pose_model`
void detect_faces(int pose_model, const float* keypoints, int people, int parts, Rect* out);
// HandDetector::detectHands (handDetector.cpp:135-160): out [people][2] = (left, right)
void detect_hands(int pose_model, const float* keypoints, int people, int parts, Rect* out);

// The crop -> net -> resize x8 -> per-part maximum -> frame coordinates pipeline of
// FaceExtractorCaffe::forwardPass (faceExtractorCaffe.cpp:174-280) and
// HandExtractorCaffe::forwardPass (handExtractorCaffe.cpp:306-445).  The reference runs one crop
// at a time (warpAffine on the CPU, a batch-1 net forward, MaximumCaffe); here every crop of the
// call is warped in one launch, the net runs on batches of crops, and the maxima of all crops are
// reduced on the device with one copy back.
class KeypointExtractor {
public:
    enum Kind { kFace = 0, kHand = 1 };
    // net_w x net_h: --face_net_resolution / --hand_net_resolution (the crop size)
    KeypointExtractor(Context* ctx, NetHip* net, int kind, int net_w, int net_h);
    // hand multi-scale detection (--hand_scale_number, --hand_scale_range)
    void set_scales(int number, float range);
    void set_max_batch(int b);
    // per-person heat maps (--heatmaps_add_* with --face / --hand): scale_mode = op::ScaleMode of
    // --heatmaps_scale, -1 off.  After extract(): [hands][people][parts][H][W] on device (H, W =
    // net output x 8); a rectangle the reference skips leaves zeros; with several hand scales the
    // last scale's maps are kept, as the reference's blob holds the last net run
    void set_heatmaps(int scale_mode);
    const float* heatmaps(int shape[5]) const;

    // frames: BGR uint8 [nframes][h][step] on device; rects on the host: face [people],
    // hand [people][2]; frame_of[people] (NULL: all frame 0).  keypoints (host): face
    // [people][parts][3], hand [2][people][parts][3] (left hands first); zeros for the rectangles
    // the reference skips.
    void extract(const uint8_t* frames, int nframes, int w, int h, size_t step, const Rect* rects,
                 const int* frame_of, int people, float* keypoints);

    int parts() const;
    int kind() const { return kind_; }
    int net_w() const { return net_w_; }
    int net_h() const { return net_h_; }
    // the crops of the last extract(): count, net inputs ([crops][3][net_h][net_w] device) and
    // per crop the 2x3 inverse map (frame <- crop)
    int crops() const { return (int)crop_m_.size() / 6; }
    const float* crop_inputs() const { return static_cast<const float*>(inputs_.ptr); }
    const double* crop_matrix(int i) const { return crop_m_.data() + 6 * (size_t)i; }

private:
    Context* ctx_;
    NetHip* net_;
    int kind_, net_w_, net_h_;
    int scales_ = 1;
    float range_ = 0.4f;
    int max_batch_ = 32;
    DevBuf inputs_, tabs_, peaks_;
    HostBuf hpeaks_;
    std::vector<double> crop_m_;
    int heat_mode_ = -1;
    DevBuf heat_out_, heat_slots_;
    int heat_shape_[5] = {0, 0, 0, 0, 0};
};

}  // namespace opk
