// pose.cpp -- PoseHip: net -> resizeAndMerge -> NMS -> connector for a batch of frames.
//
// Follows op::PoseExtractorCaffe::forwardPass (src/openpose/pose/poseExtractorCaffe.cpp:200-334):
//   heat-map blob = 8x the net output (ResizeAndMergeCaffe::Reshape, resizeAndMergeCaffe.cpp:80-81,
//     netFactor = getPoseNetDecreaseFactor = 8, scaleFactor = 1: poseExtractorCaffe.cpp:272-276);
//   scaleNetToOutput from resizeGetScaleFactor twice (:306-310);
//   NMS threshold = NMSThreshold, offset = float(0.5 / scaleNetToOutput) (:315-320);
//   connector with the PoseProperty thresholds and scaleNetToOutput (:324-333).
// All device stages are enqueued on the context stream for the whole batch; the connector's PAF
// integrals run on the GPU into compact per-frame records, and one D2H of peaks + records feeds the
// host assembly (connector.cpp) of every frame.
#include "pose.h"

#include <cmath>
#include <cstring>

#include "../../../include/opk.h"

namespace opk {

double resize_scale_factor(int iw, int ih, int tw, int th)
{
    const double rw = (tw - 1) / (double)(iw - 1);
    const double rh = (th - 1) / (double)(ih - 1);
    return rw < rh ? rw : rh;
}

PoseHip::PoseHip(Context* ctx, NetHip* net, bool maxpos)
    : ctx_(ctx), net_(net), maximize_positives_(maxpos)
{
    // defaults: poseParameters.cpp:677-756 (BODY_25)
    props_[OPK_PROP_NMS_THRESHOLD] = maxpos ? 0.02f : 0.05f;
    props_[OPK_PROP_INTER_MIN_ABOVE_THRESHOLD] = maxpos ? 0.75f : 0.95f;
    props_[OPK_PROP_INTER_THRESHOLD] = maxpos ? 0.01f : 0.05f;
    props_[OPK_PROP_MIN_SUBSET_CNT] = maxpos ? 2u : 3u;
    props_[OPK_PROP_MIN_SUBSET_SCORE] = maxpos ? 0.05f : 0.4f;
}

void PoseHip::set_property(int prop, double v)
{
    OPK_CHECK_ARG(prop >= 0 && prop < 5, "unknown PoseProperty");
    props_[prop] = v;
}

float* PoseHip::heatmaps(int shape[4])
{
    shape[0] = n_; shape[1] = pose_model(0).heat_channels(); shape[2] = hh_; shape[3] = hw_;
    if (n_ > 0 && !heat_valid_) {
        ctx_->bind();
        float* heat = static_cast<float*>(heat_.get((size_t)n_ * lazy_.channels * hh_ * hw_ * 4));
        launch_resize_merge(heat, lazy_.src, lazy_.nsrc, n_ * lazy_.channels, hh_, hw_, ctx_->stream);
        OPK_HIP(hipStreamSynchronize(ctx_->stream));
        heat_valid_ = true;
    }
    return static_cast<float*>(heat_.ptr);
}

float* PoseHip::peaks(int shape[4]) const
{
    shape[0] = n_; shape[1] = pose_model(0).parts; shape[2] = kMaxPeaks + 1; shape[3] = 3;
    return static_cast<float*>(peaks_.ptr);
}

void PoseHip::forward(const float* frames, int n, int net_h, int net_w, int prod_w, int prod_h)
{
    OPK_CHECK_ARG(net_ != nullptr, "no network: use forward_net_output (poseNetOutput path)");
    net_->forward(frames, n, net_h, net_w);
    forward_net_output(net_->output(), n, net_->out_h(), net_->out_w(), net_h, net_w, prod_w,
                       prod_h);
}

void PoseHip::forward_net_output(const float* net_out, int n, int oh, int ow, int net_h,
                                 int net_w, int prod_w, int prod_h)
{
    const PoseModelInfo& m = pose_model(0);
    const int C = m.heat_channels();
    OPK_CHECK_ARG(net_out && n > 0 && oh > 0 && ow > 0, "empty net output");
    ctx_->bind();
    hipStream_t s = ctx_->stream;
    const size_t out_elems = (size_t)n * C * oh * ow;
    if (overlay_) launch_add_inplace(const_cast<float*>(net_out), overlay_, out_elems, s);

    // 1. resize x8 (ResizeAndMergeCaffe::Reshape: (h*8 - 1)*1 + 1), evaluated lazily: NMS and
    //    the PAF scorer compute the resized values they touch with resize.hip's arithmetic
    //    (bit-identical), so the 75 MB/frame heat-map stack is only written if requested
    const int H = oh * 8, W = ow * 8;
    hh_ = H;
    hw_ = W;
    n_ = n;
    const auto& t = ctx_->tables(oh, ow, H, W);
    HeatMap heat{};
    heat.channels = C;
    heat.h = H;
    heat.w = W;
    heat.nsrc = 1;
    heat.inv_n = 1.f;
    heat.src[0] = ResizeSource{net_out, oh, ow, t.yofs, t.ycoef, t.xofs, t.xcoef};
    lazy_ = heat;
    heat_valid_ = false;

    // 2. scale net -> output (poseExtractorCaffe.cpp:281-310), net output size == net input size
    const double sp = resize_scale_factor(prod_w, prod_h, net_w, net_h);
    const int nw = (int)(sp * prod_w + 0.5f), nh = (int)(sp * prod_h + 0.5f);
    scale_net_to_output_ = (float)resize_scale_factor(nw, nh, prod_w, prod_h);

    // 3. NMS
    const float nms_th = (float)props_[OPK_PROP_NMS_THRESHOLD];
    const float off = float(0.5 / double(scale_net_to_output_));
    OPK_CHECK_ARG(!(nms_th < 0 || nms_th > 1.0), "threshold value invalid.");
    const int P1 = kMaxPeaks + 1;
    const size_t peak_floats = (size_t)m.parts * P1 * 3;
    float* peaks = static_cast<float*>(peaks_.get((size_t)n * peak_floats * 4));
    launch_nms(peaks, ctx_->nms_candidates(n, m.parts), heat, n, m.parts, P1, nms_th, off, off, s);

    // 4. connector: PAF integrals on the GPU (compact), assembly on the host
    const float inter_th = (float)props_[OPK_PROP_INTER_THRESHOLD];
    const float inter_min = (float)props_[OPK_PROP_INTER_MIN_ABOVE_THRESHOLD];
    const double near = std::sqrt((double)(W * H)) / 150;
    const float reject = float(nms_th + 1e-6);   // defaultNmsThreshold = NMSThreshold (:325)
    const auto& pt = ctx_->pose_table(0);
    float* rec = static_cast<float*>(records_.get((size_t)n * kRecordFloats * 4));
    launch_paf_scores_compact(rec, kRecordFloats, heat, peaks, n, kMaxPeaks, pt, inter_th,
                              inter_min, reject, near, s);
    float* hp = static_cast<float*>(hpeaks_.get((size_t)n * peak_floats * 4));
    float* hr = static_cast<float*>(hrecords_.get((size_t)n * kRecordFloats * 4));
    OPK_HIP(hipMemcpyAsync(hp, peaks, (size_t)n * peak_floats * 4, hipMemcpyDeviceToHost, s));
    OPK_HIP(hipMemcpyAsync(hr, rec, (size_t)n * kRecordFloats * 4, hipMemcpyDeviceToHost, s));
    OPK_HIP(hipStreamSynchronize(s));

    ConnectParams cp{(int)props_[OPK_PROP_MIN_SUBSET_CNT], (float)props_[OPK_PROP_MIN_SUBSET_SCORE],
                     scale_net_to_output_, maximize_positives_};
    people_.assign(n, 0);
    kp_.assign(n, {});
    ks_.assign(n, {});
    std::vector<int> offsets;
    for (int f = 0; f < n; ++f) {
        const float* fp = hp + (size_t)f * peak_floats;
        const float* fr = hr + (size_t)f * kRecordFloats;
        PairScores ps;
        if (fr[0] >= 0) {
            compact_offsets(m, fp, kMaxPeaks, offsets);
            ps.data = fr + 1;
            ps.compact = true;
            ps.offsets = offsets.data();
        } else {   // more candidates than a compact record holds: dense scores for this frame
            const size_t dense = (size_t)m.npairs() * kMaxPeaks * kMaxPeaks;
            float* d = static_cast<float*>(dense_.get(dense * 4));
            HeatMap hf = heat;   // frame f alone
            hf.src[0].src = net_out + (size_t)f * C * oh * ow;
            launch_paf_scores(d, hf, peaks + (size_t)f * peak_floats, 1, kMaxPeaks, pt, inter_th,
                              inter_min, reject, near, s);
            float* hd = static_cast<float*>(hdense_.get(dense * 4));
            OPK_HIP(hipMemcpyAsync(hd, d, dense * 4, hipMemcpyDeviceToHost, s));
            OPK_HIP(hipStreamSynchronize(s));
            ps.data = hd;
            ps.max_peaks = kMaxPeaks;
        }
        people_[f] = assemble_people(m, fp, kMaxPeaks, ps, cp, kp_[f], ks_[f]);
    }
}

}  // namespace opk
