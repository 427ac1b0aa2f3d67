// pose.h -- PoseHip: the op::PoseExtractorCaffe::forwardPass replacement for a batch of frames.
#pragma once
#include <vector>

#include "connector.h"
#include "context.h"
#include "net.h"

namespace opk {

class PoseHip {
public:
    PoseHip(Context* ctx, NetHip* net, bool maximize_positives);

    void set_property(int prop, double v);
    double property(int prop) const { return props_[prop]; }
    void set_overlay(const float* overlay) { overlay_ = overlay; }

    void forward(const float* frames, int n, int net_h, int net_w, int prod_w, int prod_h);
    void forward_net_output(const float* net_out, int n, int out_h, int out_w, int net_h,
                            int net_w, int prod_w, int prod_h);

    int frames() const { return (int)people_.size(); }
    int num_people(int f) const { return people_.at(f); }
    const std::vector<float>& keypoints(int f) const { return kp_.at(f); }
    const std::vector<float>& scores(int f) const { return ks_.at(f); }
    // full-resolution heat maps of the last forward, materialised on first request (the pipeline
    // itself evaluates them lazily from the net output: HeatMap in kernels.h)
    float* heatmaps(int shape[4]);
    float* peaks(int shape[4]) const;
    float scale_net_to_output() const { return scale_net_to_output_; }

private:
    Context* ctx_;
    NetHip* net_;
    bool maximize_positives_;
    double props_[5];
    const float* overlay_ = nullptr;
    float scale_net_to_output_ = 1.f;

    int n_ = 0, hh_ = 0, hw_ = 0;
    HeatMap lazy_{};            // last forward's heat maps as resize of the net output
    bool heat_valid_ = false;   // heat_ holds them
    DevBuf heat_, peaks_, records_, dense_;
    HostBuf hpeaks_, hrecords_, hdense_;
    static constexpr int kMaxPeaks = kPoseMaxPeople;   // peaks blob [25][128][3]
    static constexpr int kRecordFloats = 16384;        // compact PAF scores per frame
    std::vector<int> people_;
    std::vector<std::vector<float>> kp_, ks_;
};

// resizeGetScaleFactor (src/openpose/utilities/openCv.cpp:182-195)
double resize_scale_factor(int iw, int ih, int tw, int th);

}  // namespace opk
