// pose.h -- PoseHip: the op::PoseExtractorCaffe::forwardPass replacement for a batch of frames.
#pragma once
#include <memory>
#include <vector>

#include "connector.h"
#include "context.h"
#include "net.h"
#include "pool.h"

namespace opk {

// Two-stage pipeline, the single-GPU equivalent of the reference's worker threads
// (WPoseExtractor feeding the CPU-side consumers through WQueue, wrapper/wrapperAuxiliary.hpp):
//   submit  -- enqueue the device work of a batch (net, NMS, PAF scores, D2H of the results) on
//              the context stream and return;
//   collect -- wait for the oldest submitted batch and assemble its people on the host.
// With one batch in flight, the host assembly of batch i overlaps the device work of batch i+1.
// Stream contract: every input (frames, net inputs, an injected net output, the overlay) is read
// in order after the work the caller queued on the context stream before the submit call.
// forward() = submit + collect.
class PoseHip {
public:
    // pose_model: PoseModel id (pose_model.h); semantics: kConnectCpu / kConnectGpu (connector.h)
    PoseHip(Context* ctx, NetHip* net, bool maximize_positives, int pose_model = 0,
            int semantics = kConnectCpu);
    ~PoseHip();

    void set_property(int prop, double v);
    // heat-map semantics of resize + NMS (maps.h: kMapsCpu, kMapsCuda)
    void set_map_semantics(int maps);
    int map_semantics() const { return maps_; }
    double property(int prop) const { return props_[prop]; }
    void set_overlay(const float* overlay) { overlay_ = overlay; }
    // --upsampling_ratio (flags.hpp:136): heat maps at round(ratio x net output) instead of the net
    // input size; <= 0 is the default (the net's decrease factor, poseExtractorCaffe.cpp:47-54)
    void set_upsampling_ratio(float ratio);
    float upsampling_ratio() const { return upsampling_; }

    void forward(const float* frames, int n, int net_h, int net_w, int prod_w, int prod_h);
    void forward_net_output(const float* net_out, int n, int out_h, int out_w, int net_h,
                            int net_w, int prod_w, int prod_h);
    void submit(const float* frames, int n, int net_h, int net_w, int prod_w, int prod_h);
    void submit_net_output(const float* net_out, int n, int out_h, int out_w, int net_h,
                           int net_w, int prod_w, int prod_h);
    // multi-scale (poseExtractorCaffe.cpp:240-245, resizeAndMergeBase.cpp:55-106): frames[i] is
    // the [n][3][net_hw[2i]][net_hw[2i+1]] net input of scale i; scale 0 sets the heat-map size
    void submit_multi(const float* const* frames, const int* net_hw, int nscales, int n,
                      int prod_w, int prod_h);
    // raw frames (the reference's full per-frame path: ScaleAndSizeExtractor -> CvMatToOpInput ->
    // PoseExtractorCaffe): n BGR uint8 frames [h][step bytes] on device, prepared on the GPU for
    // every scale of set_input(), then the net per scale and the merged post-processing
    void set_input(int net_w, int net_h, float dyn, int scale_number, double scale_gap);
    void submit_frames(const uint8_t* frames, int n, int w, int h, size_t step);
    void forward_frames(const uint8_t* frames, int n, int w, int h, size_t step);
    // net input of scale i of the last submit_frames ([n][3][h][w] fp32 device; w/h may be NULL)
    const float* net_input(int i, int* w, int* h) const;
    int collect();                       // frames of the collected batch
    int pending() const { return count_; }

    // results of the last collected batch
    int frames() const { return (int)people_.size(); }
    int num_people(int f) const { return people_.at(f); }
    const std::vector<float>& keypoints(int f) const { return kp_.at(f); }
    const std::vector<float>& scores(int f) const { return ks_.at(f); }
    // full-resolution heat maps of the last collected batch, materialised on first request (the
    // pipeline evaluates them lazily from the net output: HeatMap in kernels.h); only while no
    // later batch is in flight (its net forward overwrites the net output)
    float* heatmaps(int shape[4]);
    void heatmap_size(int shape[4]) const;   // the last collected batch's, nothing materialised
    float* peaks(int shape[4]) const;
    // PoseExtractorNet::getHeatMapsCopy (poseExtractorNet.cpp:106-244) for every frame of the last
    // collected batch: types bit 0 parts, bit 1 background, bit 2 PAFs (in that order), scale_mode
    // an op::ScaleMode value; dst [n][channels of the types][H][W] device (NULL: shape only)
    void heatmaps_copy(int types, int scale_mode, float* dst, int shape[4]);
    // PoseExtractorNet::getCandidatesCopy (:246-282): peaks of one frame, x/y * scaleNetToOutput;
    // out [parts][kMaxPeaks][3], counts [parts]
    void candidates(int frame, float* out, int* counts) const;
    float scale_net_to_output() const { return scale_net_to_output_; }
    // device time of the post-processing of every submitted batch (overlay add, NMS, PAF
    // integrals: the work after the net forward), HIP events on the context stream
    void set_timing(bool on) { timer_.on = on; }
    void read_timing(int* count, double* total_ms) { timer_.read(count, total_ms); }
    // host time of the collects since the last read: waiting for the batch's device results
    // (D2H copies behind its post-processing) and assembling its people on the pool's threads
    void read_collect_times(int* count, double* wait_ms, double* assembly_ms);
    int assembly_workers() const { return pool_ ? pool_->workers() : assembly_threads(); }
    int model() const { return model_; }

    static constexpr int kMaxPeaks = kPoseMaxPeople;   // peaks blob [parts][128][3]
    static constexpr int kRecordHead = 16384;          // record floats copied eagerly per frame
    // host threads assembling a batch's people: at most this many, and at most the CPUs of the
    // process's affinity mask (assembly_threads)
    static constexpr int kAssemblyThreads = 16;
    static int assembly_threads();

private:
    struct Slot {
        DevBuf peaks, records;
        HostBuf hpeaks, hrecords;
        hipEvent_t done = nullptr;
        int n = 0, H = 0, W = 0;
        float scale = 1.f;
        HeatMap heat{};
    };
    struct NetOutput {
        const float* ptr;
        int h, w;
    };
    void submit_outputs(const NetOutput* outs, int nscales, int n, int net_h, int net_w,
                        int prod_w, int prod_h, bool own_net);
    size_t record_floats() const;        // per frame: 1 + every candidate pair of the model

    Context* ctx_;
    NetHip* net_;
    std::weak_ptr<void> net_alive_;   // NetHip::liveness (the net may be destroyed first)
    NetHip* live_net() const;         // net_, or an error if it was destroyed
    // set_input(): --net_resolution, --net_resolution_dynamic, --scale_number, --scale_gap
    int in_net_w_ = -1, in_net_h_ = 368, scale_number_ = 1;
    float dyn_ = 1.f;
    double scale_gap_ = 0.25;
    DevBuf inputs_[kMaxResizeSources];
    int input_hw_[2 * kMaxResizeSources] = {};
    int inputs_n_ = 0;
    bool maximize_positives_;
    int model_, semantics_;
    int maps_ = 0;                              // kMapsCpu
    float map_ratios_[kMaxResizeSources] = {};  // scaleInputToNetInputs of the raw-frame path
    bool have_ratios_ = false;
    double props_[5];
    const float* overlay_ = nullptr;
    float upsampling_ = 0.f;
    hipStream_t copy_ = nullptr;         // D2H of collected batches (overlaps the next batch)
    // When this PoseHip runs the net itself (submit, submit_multi, submit_frames), the
    // post-processing of a batch (overlay, NMS, PAF integrals) runs on post_, ordered after the
    // batch's nets on the context stream.  Everything the caller enqueues on the context stream
    // -- frame uploads included -- stays ordered before the next batch's warp and nets, and the
    // next batch's warp overlaps this batch's post-processing.  The nets alternate between two
    // output buffers per input shape (NetHip::select_output; NET_OUT_ALT=0: one), and before a
    // forward the context stream waits for those of the last two recorded post-processings that
    // read the buffer it is about to write (NetHip::note_reader, which also orders a direct
    // opk_net_forward of the same net after them) -- so batch i+1's nets start while batch i's
    // post-processing still runs.  post_ is a side stream of the context (opk_sync waits for it).
    // POST_STREAM=0: all on the context stream.
    // The injection path (submit_net_output: a caller-owned net output) stays on the context
    // stream, so a caller may rewrite that buffer on its stream after submit.
    hipStream_t post_ = nullptr;
    hipEvent_t nets_done_ = nullptr, post_done_[2] = {};
    int post_count_ = 0;                     // post-processings recorded on post_
    hipStream_t post_stream(bool own_net);   // the stream a batch's post-processing runs on
    void wait_post(hipStream_t s);           // s after the last recorded post-processing
    // switch the shape's output buffer for its next forward (alternate) and plan the shape
    void next_output(int n, int h, int w, bool alternate);
    DevBuf cand_;                            // NMS candidate counters (zeroed once, self-resetting)
    // multi-scale: the nets of scales 1.. run on their own streams beside scale 0's
    hipStream_t scale_streams_[kMaxResizeSources - 1] = {};
    hipEvent_t fork_ = nullptr, join_[kMaxResizeSources - 1] = {};
    EventTimer timer_;

    Slot slots_[2];
    int head_ = 0, count_ = 0, last_ = -1;
    HostBuf overflow_;                   // records longer than the copied head (pinned)
    size_t record_head_ = kRecordHead;   // record floats per frame copied eagerly (adaptive)
    int peak_rows_ = kMaxPeaks + 1;      // peak rows per part copied eagerly (adaptive)
    // people assembly: worker threads (started by the first multi-frame collect) and one
    // scratch per worker
    std::unique_ptr<WorkerPool> pool_;
    int collect_count_ = 0;
    double collect_wait_ms_ = 0., collect_assembly_ms_ = 0.;
    std::vector<AssemblyScratch> scratch_;

    float scale_net_to_output_ = 1.f;
    int n_ = 0, hh_ = 0, hw_ = 0;
    bool heat_valid_ = false;
    DevBuf heat_, heat_sel_;
    std::vector<int> people_;
    std::vector<std::vector<float>> kp_, ks_;
};

// resizeGetScaleFactor (src/openpose/utilities/openCv.cpp:182-195)
double resize_scale_factor(int iw, int ih, int tw, int th);

}  // namespace opk
