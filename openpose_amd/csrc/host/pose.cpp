// pose.cpp -- PoseHip: net -> resizeAndMerge -> NMS -> connector for a batch of frames.
//
// Follows op::PoseExtractorCaffe::forwardPass (src/openpose/pose/poseExtractorCaffe.cpp:200-334):
//   heat-map blob = 8x the net output (ResizeAndMergeCaffe::Reshape, resizeAndMergeCaffe.cpp:80-81,
//     netFactor = getPoseNetDecreaseFactor = 8, scaleFactor = 1: poseExtractorCaffe.cpp:272-276);
//   scaleNetToOutput from resizeGetScaleFactor twice (:306-310);
//   NMS threshold = NMSThreshold, offset = float(0.5 / scaleNetToOutput) (:315-320);
//   connector with the PoseProperty thresholds and scaleNetToOutput (:324-333).
// Device stages of a batch are enqueued on the context stream (submit); the connector's PAF
// integrals run on the GPU into compact per-frame records, and collect() copies peaks + records
// on a second stream and assembles people on the host (connector.cpp) while the context stream
// may already run the next batch.
#include "pose.h"

#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <exception>
#include <string>
#include <thread>

#include "../../../include/opk.h"
#include "input.h"
#include "maps.h"

namespace opk {

double resize_scale_factor(int iw, int ih, int tw, int th)
{
    const double rw = (tw - 1) / (double)(iw - 1);
    const double rh = (th - 1) / (double)(ih - 1);
    return rw < rh ? rw : rh;
}

PoseHip::PoseHip(Context* ctx, NetHip* net, bool maxpos, int pose_model_id, int semantics)
    : ctx_(ctx), net_(net), maximize_positives_(maxpos), model_(pose_model_id), semantics_(semantics)
{
    if (net_) net_alive_ = net_->liveness();
    const PoseModelInfo& m = pose_model(model_);   // throws for unknown models
    OPK_CHECK_ARG(semantics == kConnectCpu || semantics == kConnectGpu, "unknown connector semantics");
    if (semantics == kConnectCpu && !m.cpu_connector())   // bodyPartConnectorBase.cpp:165-167
        throw Error(4, std::string("connectBodyPartsCpu supports BODY_25, COCO_18 and MPI_15 only (") +
                           m.name + "): use the GPU-path connector semantics");
    // defaults: poseParameters.cpp:677-756 (per model where they differ)
    props_[OPK_PROP_NMS_THRESHOLD] = maxpos ? m.nms_th_maxpos : m.nms_th;
    props_[OPK_PROP_INTER_MIN_ABOVE_THRESHOLD] = maxpos ? 0.75f : 0.95f;
    props_[OPK_PROP_INTER_THRESHOLD] = maxpos ? m.inter_th_maxpos : m.inter_th;
    props_[OPK_PROP_MIN_SUBSET_CNT] = maxpos ? 2u : 3u;
    props_[OPK_PROP_MIN_SUBSET_SCORE] = maxpos ? 0.05f : 0.4f;
    if (ctx_->device >= 0) {
        ctx_->bind();
        OPK_HIP(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking));
        for (auto& s : slots_) OPK_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    }
}

NetHip* PoseHip::live_net() const
{
    OPK_CHECK_ARG(net_ != nullptr, "no net: a pose extractor over injected net outputs");
    if (net_alive_.expired())
        throw Error(4, "the net was destroyed before this pose extractor (destroy the pose first)");
    return net_;
}

PoseHip::~PoseHip()
{
    if (copy_) {
        (void)hipStreamSynchronize(ctx_->stream);
        (void)hipStreamDestroy(copy_);
    }
    if (post_) {
        (void)hipStreamSynchronize(post_);
        if (net_ && !net_alive_.expired()) net_->forget_reader_events(post_done_, 2);
        ctx_->remove_side_stream(post_);
        (void)hipStreamDestroy(post_);
        (void)hipEventDestroy(nets_done_);
        for (auto& e : post_done_) (void)hipEventDestroy(e);
    }
    for (auto& s : slots_)
        if (s.done) (void)hipEventDestroy(s.done);
    for (auto& st : scale_streams_)
        if (st) (void)hipStreamDestroy(st);
    for (auto& e : join_)
        if (e) (void)hipEventDestroy(e);
    if (fork_) (void)hipEventDestroy(fork_);
}

void PoseHip::set_upsampling_ratio(float ratio)
{
    OPK_CHECK_ARG(std::isfinite(ratio), "upsampling ratio must be finite");
    upsampling_ = ratio;
}

// getPoseNetDecreaseFactor (poseParameters.cpp:630-641)
static float net_decrease_factor(int model) { return model == 5 /* BODY_19_X2 */ ? 4.f : 8.f; }

void PoseHip::set_map_semantics(int maps)
{
    OPK_CHECK_ARG(maps == kMapsCpu || maps == kMapsCuda, "unknown heat-map semantics");
    maps_ = maps;
}

void PoseHip::set_property(int prop, double v)
{
    OPK_CHECK_ARG(prop >= 0 && prop < 5, "unknown PoseProperty");
    props_[prop] = v;
}

size_t PoseHip::record_floats() const
{
    const PoseModelInfo& m = pose_model(model_);
    return 1 + (size_t)m.npairs() * kMaxPeaks * kMaxPeaks;
}

void PoseHip::heatmap_size(int shape[4]) const
{
    OPK_CHECK_ARG(last_ >= 0, "no collected batch");
    shape[0] = n_; shape[1] = slots_[last_].heat.channels; shape[2] = hh_; shape[3] = hw_;
}

float* PoseHip::heatmaps(int shape[4])
{
    OPK_CHECK_ARG(last_ >= 0, "no collected batch");
    OPK_CHECK_ARG(count_ == 0, "heat maps are kept only while no later batch is in flight");
    const Slot& s = slots_[last_];
    shape[0] = n_; shape[1] = s.heat.channels; shape[2] = hh_; shape[3] = hw_;
    if (!heat_valid_) {
        ctx_->bind();
        float* heat = static_cast<float*>(heat_.get((size_t)n_ * s.heat.channels * hh_ * hw_ * 4));
        if (s.heat.cuda)
            launch_resize_merge_cuda(heat, s.heat, n_ * s.heat.channels, ctx_->stream);
        else
            launch_resize_merge(heat, s.heat.src, s.heat.nsrc, n_ * s.heat.channels, hh_, hw_,
                                ctx_->stream);
        OPK_HIP(hipStreamSynchronize(ctx_->stream));
        heat_valid_ = true;
    }
    return static_cast<float*>(heat_.ptr);
}

void PoseHip::heatmaps_copy(int types, int scale_mode, float* dst, int shape[4])
{
    OPK_CHECK_ARG(types > 0 && types < 8, "heat-map types: bits 0 parts, 1 background, 2 PAFs");
    OPK_CHECK_ARG(scale_mode >= 0 && scale_mode <= 8, "unknown ScaleMode");
    const PoseModelInfo& m = pose_model(model_);
    std::vector<int> sel, kind;
    if (types & 1)
        for (int c = 0; c < m.parts; ++c) { sel.push_back(c); kind.push_back(0); }
    if (types & 2) {
        OPK_CHECK_ARG(m.bkg, "You enabled `--heatmaps_add_bkg` for a model that does not contain one. "
                             "Please, remove this flag for this model.");
        sel.push_back(m.parts);
        kind.push_back(0);
    }
    if (types & 4)
        for (int c = 0; c < 2 * m.npairs(); ++c) {
            sel.push_back(m.parts + (m.bkg ? 1 : 0) + c);
            kind.push_back(1);
        }
    int hs[4];
    float* heat = heatmaps(hs);   // materialised once per collected batch
    shape[0] = hs[0]; shape[1] = (int)sel.size(); shape[2] = hs[2]; shape[3] = hs[3];
    if (!dst) return;
    sel.insert(sel.end(), kind.begin(), kind.end());
    int* dsel = static_cast<int*>(heat_sel_.get(sel.size() * sizeof(int)));
    OPK_HIP(hipMemcpyAsync(dsel, sel.data(), sel.size() * sizeof(int), hipMemcpyHostToDevice,
                           ctx_->stream));
    launch_heat_copy(dst, heat, dsel, shape[1], hs[0], hs[1], (size_t)hs[2] * hs[3], scale_mode,
                     ctx_->stream);
    OPK_HIP(hipStreamSynchronize(ctx_->stream));   // `sel` dies at return
}

void PoseHip::candidates(int frame, float* out, int* counts) const
{
    OPK_CHECK_ARG(last_ >= 0, "no collected batch");
    OPK_CHECK_ARG(frame >= 0 && frame < n_, "bad frame");
    const PoseModelInfo& m = pose_model(model_);
    const size_t area = (size_t)(kMaxPeaks + 1) * 3;
    const float* p = static_cast<const float*>(slots_[last_].hpeaks.ptr) + (size_t)frame * m.parts * area;
    for (int part = 0; part < m.parts; ++part) {
        const float* pp = p + part * area;
        const int count = (int)std::round(pp[0]);
        if (counts) counts[part] = count;
        if (!out) continue;
        for (int c = 0; c < count; ++c) {
            float* o = out + ((size_t)part * kMaxPeaks + c) * 3;
            o[0] = pp[3 + 3 * c] * scale_net_to_output_;
            o[1] = pp[3 + 3 * c + 1] * scale_net_to_output_;
            o[2] = pp[3 + 3 * c + 2];
        }
    }
}

float* PoseHip::peaks(int shape[4]) const
{
    OPK_CHECK_ARG(last_ >= 0, "no collected batch");
    shape[0] = n_; shape[1] = pose_model(model_).parts; shape[2] = kMaxPeaks + 1; shape[3] = 3;
    return static_cast<float*>(slots_[last_].peaks.ptr);
}

void PoseHip::forward(const float* frames, int n, int net_h, int net_w, int prod_w, int prod_h)
{
    OPK_CHECK_ARG(count_ == 0, "batches in flight: collect them first");
    submit(frames, n, net_h, net_w, prod_w, prod_h);
    collect();
}

void PoseHip::forward_net_output(const float* net_out, int n, int oh, int ow, int net_h,
                                 int net_w, int prod_w, int prod_h)
{
    OPK_CHECK_ARG(count_ == 0, "batches in flight: collect them first");
    submit_net_output(net_out, n, oh, ow, net_h, net_w, prod_w, prod_h);
    collect();
}

void PoseHip::submit(const float* frames, int n, int net_h, int net_w, int prod_w, int prod_h)
{
    OPK_CHECK_ARG(net_ != nullptr, "no network: use forward_net_output (poseNetOutput path)");
    OPK_CHECK_ARG(count_ < 2, "two batches already in flight: collect first");
    ctx_->bind();
    next_output(n, net_h, net_w, true);
    live_net()->forward(frames, n, net_h, net_w);
    const NetOutput o{live_net()->output(), live_net()->out_h(), live_net()->out_w()};
    submit_outputs(&o, 1, n, net_h, net_w, prod_w, prod_h, true);
}

hipStream_t PoseHip::post_stream(bool own_net)
{
    if (!own_net || ctx_->device < 0 || dev_switch("POST_STREAM", 1) == 0) {
        wait_post(ctx_->stream);   // shared scratch / slots with a post-processing on post_
        return ctx_->stream;
    }
    if (!post_) {
        OPK_HIP(hipStreamCreateWithFlags(&post_, hipStreamNonBlocking));
        OPK_HIP(hipEventCreateWithFlags(&nets_done_, hipEventDisableTiming));
        for (auto& e : post_done_) OPK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx_->add_side_stream(post_);   // opk_sync covers the post-processing
    }
    // everything on the context stream so far: the caller's work and this batch's nets
    OPK_HIP(hipEventRecord(nets_done_, ctx_->stream));
    OPK_HIP(hipStreamWaitEvent(post_, nets_done_, 0));
    return post_;
}

void PoseHip::wait_post(hipStream_t s)
{
    if (post_count_ > 0) OPK_HIP(hipStreamWaitEvent(s, post_done_[(post_count_ - 1) & 1], 0));
}

void PoseHip::next_output(int n, int h, int w, bool alternate)
{
    // (the forward that writes the buffer waits for the post-processings reading it:
    // NetHip::note_reader)
    const bool alt = alternate && post_ != nullptr && dev_switch("NET_OUT_ALT", 1) != 0;
    (void)live_net()->select_output(n, h, w, alt);
}

void PoseHip::set_input(int net_w, int net_h, float dyn, int scale_number, double scale_gap)
{
    OPK_CHECK_ARG(net_w > 0 || net_h > 0,
                  "Only 1 of the dimensions of net input resolution can be <= 0.");
    OPK_CHECK_ARG(scale_number >= 1 && scale_number <= kMaxResizeSources, "1..8 scales");
    OPK_CHECK_ARG(1. - (scale_number - 1) * scale_gap >= 0. && scale_gap >= 0.,
                  "All scales must be in the range [0, 1], i.e., 0 <= 1-scale_number*scale_gap <= 1");
    in_net_w_ = net_w;
    in_net_h_ = net_h;
    dyn_ = dyn;
    scale_number_ = scale_number;
    scale_gap_ = scale_gap;
}

void PoseHip::submit_frames(const uint8_t* frames, int n, int w, int h, size_t step)
{
    OPK_CHECK_ARG(net_ != nullptr, "no network: raw frames need the net");
    OPK_CHECK_ARG(frames != nullptr && n > 0 && w > 0 && h > 0, "empty frames");
    OPK_CHECK_ARG(count_ < 2, "two batches already in flight: collect first");
    OPK_CHECK_ARG(model_ != 6, "BODY_19N (DenseNet normalisation) is not supported");
    double scales[kMaxResizeSources];
    scale_and_size(w, h, in_net_w_, in_net_h_, dyn_, scale_number_, scale_gap_, scales, input_hw_);
    const float* ptrs[kMaxResizeSources];
    int hw[2 * kMaxResizeSources];
    // the warps run on the context stream, after whatever the caller queued there (e.g. the
    // upload of these frames) and after the previous batch's nets (the readers of the input
    // buffers); the previous batch's post-processing runs beside them on post_
    ctx_->bind();
    for (int i = 0; i < scale_number_; ++i) {
        const int nw = input_hw_[2 * i], nh = input_hw_[2 * i + 1];
        float* x = static_cast<float*>(inputs_[i].get((size_t)n * 3 * nh * nw * sizeof(float)));
        cvmat_to_input(ctx_, x, frames, n, w, h, step, scales[i], nw, nh, 1, ctx_->stream);
        ptrs[i] = x;
        hw[2 * i] = nh;
        hw[2 * i + 1] = nw;
    }
    inputs_n_ = n;
    for (int i = 0; i < scale_number_; ++i) map_ratios_[i] = (float)scales[i];
    have_ratios_ = true;
    try {
        if (scale_number_ == 1)
            submit(ptrs[0], n, hw[0], hw[1], w, h);
        else
            submit_multi(ptrs, hw, scale_number_, n, w, h);
    } catch (...) {
        have_ratios_ = false;
        throw;
    }
    have_ratios_ = false;
}

void PoseHip::forward_frames(const uint8_t* frames, int n, int w, int h, size_t step)
{
    OPK_CHECK_ARG(count_ == 0, "batches in flight: collect them first");
    submit_frames(frames, n, w, h, step);
    collect();
}

const float* PoseHip::net_input(int i, int* w, int* h) const
{
    OPK_CHECK_ARG(i >= 0 && i < scale_number_ && inputs_n_ > 0, "no such scale");
    if (w) *w = input_hw_[2 * i];
    if (h) *h = input_hw_[2 * i + 1];
    return static_cast<const float*>(inputs_[i].ptr);
}

void PoseHip::submit_multi(const float* const* frames, const int* net_hw, int nscales, int n,
                           int prod_w, int prod_h)
{
    OPK_CHECK_ARG(net_ != nullptr, "no network: multi-scale needs the net");
    OPK_CHECK_ARG(frames && net_hw && nscales >= 1 && nscales <= kMaxResizeSources,
                  "1..8 scales");
    OPK_CHECK_ARG(count_ < 2, "two batches already in flight: collect first");
    // one net pass per scale (poseExtractorCaffe.cpp:240-245); every input shape keeps its own
    // plan and output buffer in NetHip, so the outputs coexist until the merge reads them
    std::vector<NetOutput> outs(nscales);
    for (int i = 0; i < nscales; ++i) OPK_CHECK_ARG(frames[i] != nullptr, "NULL scale input");
    ctx_->bind();
    // the scales' nets are independent until the merge: scales 1.. run on streams of their own
    // beside scale 0 (small nets leave most CUs idle on their own), each shape with its own plan
    // and buffers; the context stream waits for all of them before the merge.  Shapes that repeat
    // would share a plan, so those run in order.
    bool distinct = dev_switch("MULTISCALE_STREAMS", 1) != 0;
    for (int i = 0; i < nscales && distinct; ++i)
        for (int j = 0; j < i; ++j)
            distinct = distinct && !(net_hw[2 * i] == net_hw[2 * j] && net_hw[2 * i + 1] == net_hw[2 * j + 1]);
    // each output buffer the nets write: after the post-processings that read it (a repeated
    // shape shares one plan and buffer, and keeps it)
    for (int i = 0; i < nscales; ++i) next_output(n, net_hw[2 * i], net_hw[2 * i + 1], nscales == 1 || distinct);
    if (nscales == 1 || !distinct) {
        for (int i = 0; i < nscales; ++i) {
            live_net()->forward(frames[i], n, net_hw[2 * i], net_hw[2 * i + 1]);
            outs[i] = NetOutput{live_net()->output(), live_net()->out_h(), live_net()->out_w()};
        }
    } else {
        if (!fork_) {
            OPK_HIP(hipEventCreateWithFlags(&fork_, hipEventDisableTiming));
            for (int i = 0; i < kMaxResizeSources - 1; ++i) {
                OPK_HIP(hipStreamCreateWithFlags(&scale_streams_[i], hipStreamNonBlocking));
                OPK_HIP(hipEventCreateWithFlags(&join_[i], hipEventDisableTiming));
            }
        }
        for (int i = 0; i < nscales; ++i) live_net()->prepare(n, net_hw[2 * i], net_hw[2 * i + 1]);
        hipStream_t s = ctx_->stream;
        live_net()->time_begin(s);   // one timed region for all the scales' nets of the batch
        OPK_HIP(hipEventRecord(fork_, s));   // inputs warped, new plans zeroed
        live_net()->forward_on(frames[0], n, net_hw[0], net_hw[1], s, false);
        outs[0] = NetOutput{live_net()->output(), live_net()->out_h(), live_net()->out_w()};
        for (int i = 1; i < nscales; ++i) {
            OPK_HIP(hipStreamWaitEvent(scale_streams_[i - 1], fork_, 0));
            live_net()->forward_on(frames[i], n, net_hw[2 * i], net_hw[2 * i + 1], scale_streams_[i - 1],
                             false);
            outs[i] = NetOutput{live_net()->output(), live_net()->out_h(), live_net()->out_w()};
            OPK_HIP(hipEventRecord(join_[i - 1], scale_streams_[i - 1]));
        }
        for (int i = 1; i < nscales; ++i) OPK_HIP(hipStreamWaitEvent(s, join_[i - 1], 0));
        live_net()->time_end(s);
    }
    submit_outputs(outs.data(), nscales, n, net_hw[0], net_hw[1], prod_w, prod_h, true);
}

void PoseHip::submit_net_output(const float* net_out, int n, int oh, int ow, int net_h,
                                int net_w, int prod_w, int prod_h)
{
    const NetOutput o{net_out, oh, ow};
    submit_outputs(&o, 1, n, net_h, net_w, prod_w, prod_h, false);
}

void PoseHip::submit_outputs(const NetOutput* outs, int nscales, int n, int net_h, int net_w,
                             int prod_w, int prod_h, bool own_net)
{
    const PoseModelInfo& m = pose_model(model_);
    const int C = m.heat_channels();
    OPK_CHECK_ARG(n > 0 && nscales >= 1 && nscales <= kMaxResizeSources, "bad batch");
    for (int i = 0; i < nscales; ++i)
        OPK_CHECK_ARG(outs[i].ptr && outs[i].h > 0 && outs[i].w > 0, "empty net output");
    OPK_CHECK_ARG(count_ < 2, "two batches already in flight: collect first");
    ctx_->bind();
    Slot& sl = slots_[(head_ + count_) & 1];
    const hipStream_t s = post_stream(own_net);
    // dev hook: a slow post-processing, so a missing stream wait corrupts results every time
    if (const int d = dev_switch("POST_DELAY_US", 0)) launch_delay(d, s);
    timer_.begin(s);
    if (overlay_) {   // synthetic people on the first scale's output
        const size_t out_elems = (size_t)n * C * outs[0].h * outs[0].w;
        launch_add_inplace(const_cast<float*>(outs[0].ptr), overlay_, out_elems, s);
    }

    // 1. resize of the first scale's size (ResizeAndMergeCaffe::Reshape, resizeAndMergeCaffe.cpp:
    //    77-81: round((h * netFactor - 1) * 1) + 1, netFactor = --upsampling_ratio or the net's
    //    decrease factor, reshapePoseExtractorCaffe poseExtractorCaffe.cpp:47-54) and average of the
    //    scales (resizeAndMergeBase.cpp:55-106), evaluated lazily: NMS and the PAF scorer compute
    //    the merged values they touch with resize.hip's arithmetic (bit-identical), so the
    //    75 MB/frame heat-map stack is only written if requested
    const float dec = net_decrease_factor(model_);
    const float nf = upsampling_ > 0.f ? upsampling_ : dec;
    const int H = (int)std::round(((float)outs[0].h * nf - 1.f) * 1.f) + 1;
    const int W = (int)std::round(((float)outs[0].w * nf - 1.f) * 1.f) + 1;
    OPK_CHECK_ARG(H >= 1 && W >= 1, "upsampling ratio gives an empty heat map");
    HeatMap heat{};
    if (maps_ == kMapsCuda) {   // resizeAndMergeGpu's arithmetic (maps.h)
        OPK_CHECK_ARG(nscales == 1 || have_ratios_,
                      "multi-scale CUDA map semantics needs scaleInputToNetInputs (raw-frame path)");
        const float* ptr[kMaxResizeSources];
        int hs[kMaxResizeSources], ws[kMaxResizeSources];
        for (int i = 0; i < nscales; ++i) {
            ptr[i] = outs[i].ptr;
            hs[i] = outs[i].h;
            ws[i] = outs[i].w;
        }
        heat = cuda_heat_map(ptr, hs, ws, nscales, C, H, W, have_ratios_ ? map_ratios_ : nullptr);
    } else {
        heat.channels = C;
        heat.h = H;
        heat.w = W;
        heat.nsrc = nscales;
        heat.inv_n = (float)(1. / (double)nscales);
        for (int i = 0; i < nscales; ++i) {
            const auto& t = ctx_->tables(outs[i].h, outs[i].w, H, W);
            heat.src[i] = ResizeSource{outs[i].ptr, outs[i].h, outs[i].w, t.yofs, t.ycoef, t.xofs,
                                       t.xcoef};
        }
    }

    // 2. scale net -> output (poseExtractorCaffe.cpp:281-310): mNetOutputSize = the net input
    //    size x (ratio / decrease factor), ratio 1 without --upsampling_ratio
    const float ratio = upsampling_ <= 0.f ? 1.f : upsampling_ / dec;
    const int out_w = (int)(ratio * (float)net_w + 0.5f), out_h = (int)(ratio * (float)net_h + 0.5f);
    const double sp = resize_scale_factor(prod_w, prod_h, out_w, out_h);
    const int nw = (int)(sp * prod_w + 0.5f), nh = (int)(sp * prod_h + 0.5f);
    const float scale = (float)resize_scale_factor(nw, nh, prod_w, prod_h);

    // 3. NMS
    const float nms_th = (float)props_[OPK_PROP_NMS_THRESHOLD];
    const float off = float(0.5 / double(scale));
    OPK_CHECK_ARG(!(nms_th < 0 || nms_th > 1.0), "threshold value invalid.");
    const int P1 = kMaxPeaks + 1;
    const size_t peak_floats = (size_t)m.parts * P1 * 3;
    float* peaks = static_cast<float*>(sl.peaks.get((size_t)n * peak_floats * 4));
    const size_t cand_bytes = nms_scratch_ints(n, m.parts) * sizeof(int);
    if (cand_bytes > cand_.bytes) {   // the counters reset themselves after every launch
        cand_.get(cand_bytes);
        OPK_HIP(hipMemsetAsync(cand_.ptr, 0, cand_bytes, s));
    }
    launch_nms(peaks, static_cast<int*>(cand_.ptr), heat, n, m.parts, P1, nms_th, off, off, s,
               maps_ == kMapsCuda);

    // 4. connector, device half: PAF integrals of every candidate pair into compact records
    //    sized for the worst case (every pair of every limb), so no frame ever falls back
    const float inter_th = (float)props_[OPK_PROP_INTER_THRESHOLD];
    const float inter_min = (float)props_[OPK_PROP_INTER_MIN_ABOVE_THRESHOLD];
    const double near = std::sqrt((double)(W * H)) / 150;
    const float reject = float(nms_th + 1e-6);   // defaultNmsThreshold = NMSThreshold (:325)
    const auto& pt = ctx_->pose_table(model_);
    const size_t rf = record_floats();
    float* rec = static_cast<float*>(sl.records.get((size_t)n * rf * 4));
    launch_paf_scores_compact(rec, (int)rf, heat, peaks, n, kMaxPeaks, pt, inter_th, inter_min,
                              reject, near, s);
    timer_.end(s);
    OPK_HIP(hipEventRecord(sl.done, s));
    if (post_ && s == post_) {   // (the context stream may be the null stream)
        const int k = post_count_ & 1;
        OPK_HIP(hipEventRecord(post_done_[k], post_));
        // every later forward writing one of these outputs (ours or a direct opk_net_forward)
        // waits for this post-processing first
        for (int i = 0; i < nscales; ++i) live_net()->note_reader(outs[i].ptr, post_done_[k]);
        ++post_count_;
    }
    sl.n = n;
    sl.H = H;
    sl.W = W;
    sl.scale = scale;
    sl.heat = heat;
    ++count_;
}

int PoseHip::assembly_threads()
{
    // the CPUs this process may run on (its affinity mask: a rank pinned to its GPU-local cores
    // by openpose_amd.parallel.pin_rank_cpus gets only those), not the machine's count
    int cpus = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) cpus = CPU_COUNT(&set);
    if (cpus <= 0) cpus = (int)std::max(1u, std::thread::hardware_concurrency());
    return std::max(1, std::min(kAssemblyThreads, cpus));
}

void PoseHip::read_collect_times(int* count, double* wait_ms, double* assembly_ms)
{
    if (count) *count = collect_count_;
    if (wait_ms) *wait_ms = collect_wait_ms_;
    if (assembly_ms) *assembly_ms = collect_assembly_ms_;
    collect_count_ = 0;
    collect_wait_ms_ = collect_assembly_ms_ = 0.;
}

int PoseHip::collect()
{
    OPK_CHECK_ARG(count_ > 0, "no batch in flight");
    ctx_->bind();
    const int si = head_;
    Slot& sl = slots_[si];
    const PoseModelInfo& m = pose_model(model_);
    const int n = sl.n;
    const int P1 = kMaxPeaks + 1;
    const size_t peak_floats = (size_t)m.parts * P1 * 3;
    const size_t rf = record_floats();
    // Device-to-host copies sized from the previous batches (their blit kernels occupy CUs the
    // next batch's nets need): the first R rows of every part's peak block (R > the largest peak
    // count seen) and the first K floats of every frame's records; a frame with more peaks or
    // longer records is fetched whole below.  The host layouts stay the full ones.
    const size_t K = std::min<size_t>(record_head_, rf);
    const int R = std::min(peak_rows_, P1);
    float* hp = static_cast<float*>(sl.hpeaks.get((size_t)n * peak_floats * 4));
    float* hr = static_cast<float*>(sl.hrecords.get((size_t)n * K * 4));
    OPK_HIP(hipStreamWaitEvent(copy_, sl.done, 0));
    OPK_HIP(hipMemcpy2DAsync(hp, (size_t)P1 * 12, sl.peaks.ptr, (size_t)P1 * 12, (size_t)R * 12,
                             (size_t)n * m.parts, hipMemcpyDeviceToHost, copy_));
    OPK_HIP(hipMemcpy2DAsync(hr, K * 4, sl.records.ptr, rf * 4, K * 4, n, hipMemcpyDeviceToHost,
                             copy_));
    auto tw0 = std::chrono::steady_clock::now();
    OPK_HIP(hipStreamSynchronize(copy_));
    double wait_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw0).count();
    // frames with a part of R - 1 or more peaks: the whole peak block
    int max_count = 0;
    bool refetch = false;
    for (int f = 0; f < n; ++f) {
        int fmax = 0;
        for (int p = 0; p < m.parts; ++p)
            fmax = std::max(fmax, (int)std::lround(hp[(size_t)f * peak_floats + (size_t)p * P1 * 3]));
        max_count = std::max(max_count, fmax);
        if (fmax >= R - 1 && R < P1) {
            OPK_HIP(hipMemcpyAsync(hp + (size_t)f * peak_floats,
                                   static_cast<const float*>(sl.peaks.ptr) + (size_t)f * peak_floats,
                                   peak_floats * 4, hipMemcpyDeviceToHost, copy_));
            refetch = true;
        }
    }
    if (refetch) {
        tw0 = std::chrono::steady_clock::now();
        OPK_HIP(hipStreamSynchronize(copy_));
        wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw0).count();
    }
    peak_rows_ = std::min(P1, (max_count + 1 + 4 + 7) / 8 * 8);
    const auto tw1 = std::chrono::steady_clock::now();
    double over_ms = 0.;   // the long records' copy (a wait, inside tw1 .. tw2)

    ConnectParams cp{(int)props_[OPK_PROP_MIN_SUBSET_CNT], (float)props_[OPK_PROP_MIN_SUBSET_SCORE],
                     sl.scale, maximize_positives_, semantics_};
    people_.assign(n, 0);
    kp_.assign(n, {});
    ks_.assign(n, {});
    // per-frame compact-record offsets; records longer than the eagerly copied head are fetched
    // whole below
    std::vector<std::vector<int>> offsets(n);
    std::vector<size_t> over_at(n, (size_t)-1);
    std::vector<int> total(n);
    for (int f = 0; f < n; ++f) {
        total[f] = compact_offsets(m, hp + (size_t)f * peak_floats, kMaxPeaks, offsets[f]);
        OPK_CHECK_ARG((int)hr[(size_t)f * K] == total[f], "PAF record count differs from the peak counts");
    }
    // records longer than the eagerly copied head (many-people / BODY_135 frames): one 2-D copy
    // per run of consecutive long frames, at the width of the run's longest record, so frames
    // between two distant long ones are not copied
    struct Run { int f0, f1; size_t w, at; };
    std::vector<Run> runs;
    size_t over_floats = 0;
    for (int f = 0; f < n; ++f) {
        if ((size_t)total[f] + 1 <= K) continue;
        if (runs.empty() || runs.back().f1 != f - 1) runs.push_back(Run{f, f, 0, 0});
        runs.back().f1 = f;
        runs.back().w = std::max(runs.back().w, (size_t)total[f] + 1);
    }
    for (auto& r : runs) {
        r.at = over_floats;
        over_floats += (size_t)(r.f1 - r.f0 + 1) * r.w;
    }
    if (!runs.empty()) {
        float* ho = static_cast<float*>(overflow_.get(over_floats * 4));
        for (const auto& r : runs) {
            OPK_HIP(hipMemcpy2DAsync(ho + r.at, r.w * 4,
                                     static_cast<const float*>(sl.records.ptr) + (size_t)r.f0 * rf,
                                     rf * 4, r.w * 4, (size_t)(r.f1 - r.f0 + 1),
                                     hipMemcpyDeviceToHost, copy_));
            for (int f = r.f0; f <= r.f1; ++f) over_at[f] = r.at + (size_t)(f - r.f0) * r.w;
        }
        tw0 = std::chrono::steady_clock::now();
        OPK_HIP(hipStreamSynchronize(copy_));
        over_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw0).count();
    }
    int max_total = 0;
    for (int f = 0; f < n; ++f) max_total = std::max(max_total, total[f]);
    record_head_ = std::min<size_t>(kRecordHead, ((size_t)max_total + 1 + max_total / 4 + 1023) / 1024 * 1024);
    // people assembly: frames are independent (connectBodyParts* per frame), so they run on the
    // pool's kAssemblyThreads host threads; every frame's result is the single-threaded one
    if (!pool_ && n > 1) pool_ = std::make_unique<WorkerPool>(assembly_threads());
    const int workers = pool_ ? pool_->workers() : 1;
    if ((int)scratch_.size() < workers) scratch_.resize(workers);
    const float* ho = static_cast<const float*>(overflow_.ptr);
    auto frame = [&](int f, int worker) {
        PairScores ps;
        ps.data = (over_at[f] != (size_t)-1 ? ho + over_at[f] : hr + (size_t)f * K) + 1;
        ps.compact = true;
        ps.offsets = offsets[f].data();
        people_[f] = assemble_people(m, hp + (size_t)f * peak_floats, kMaxPeaks, ps, cp, kp_[f],
                                     ks_[f], &scratch_[worker]);
    };
    if (pool_) pool_->run(n, frame);
    else
        for (int f = 0; f < n; ++f) frame(f, 0);
    const auto tw2 = std::chrono::steady_clock::now();
    // (the waits for the copies: device time; the rest, from the first wait's end: assembly)
    collect_wait_ms_ += wait_ms + over_ms;
    collect_assembly_ms_ += std::chrono::duration<double, std::milli>(tw2 - tw1).count() - over_ms;
    ++collect_count_;
    head_ = (head_ + 1) & 1;
    --count_;
    last_ = si;
    n_ = n;
    hh_ = sl.H;
    hw_ = sl.W;
    scale_net_to_output_ = sl.scale;
    heat_valid_ = false;
    return n;
}

}  // namespace opk
