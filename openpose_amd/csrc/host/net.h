// net.h -- NetHip: the op::NetCaffe replacement (graph planner + gfx950 executor).
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../kernels/conv.h"
#include "context.h"
#include "graph.h"

namespace opk {

class NetHip {
public:
    NetHip(Context* ctx, std::vector<LayerDesc> layers, const std::string& output_blob = "net_output");

    struct ConvInfo {
        std::string name;
        int cin, cout, k, act;   // act: 0 none, 1 ReLU, 2 PReLU
        std::string act_layer;   // the fused ReLU/PReLU layer (holds the PReLU slopes)
    };
    const std::vector<ConvInfo>& convs() const { return info_; }
    void set_conv(const std::string& name, const float* w, const float* b, const float* slope);
    // Arithmetic of the forward: kPrecisionFp16 (default: fp16 weights and stored activations,
    // fp32 MFMA accumulation, the tuned fused kernels) or kPrecisionSplit (every weight and
    // activation as an fp16 hi / lo pair, three MFMA passes per conv on conv3_kernel, no fused
    // kernels: ~fp32 results at ~3x the MFMA work; ConvArgs::split).  Re-plans the shapes and
    // re-packs the loaded weights.
    static constexpr int kPrecisionFp16 = 0, kPrecisionSplit = 1;
    void set_precision(int precision);
    int precision() const { return precision_; }
    bool ready() const;
    // caffe::Net::CopyTrainedLayersFrom (netCaffe.cpp:165,185): weights, bias and PReLU slopes of
    // every conv named in the file (shapes checked as Caffe does); layers the net does not have
    // are ignored.  Returns the number of convolutions loaded.
    int load_caffemodel(const std::string& path);

    // input: device NCHW fp32 [n][3][h][w].  Every input shape gets its own plan (activation
    // buffers with zeroed guards, launch arguments, net output), kept across forwards, so the
    // scales of a multi-scale pass alternate without re-planning and their outputs coexist.
    void forward(const float* input, int n, int h, int w);
    // the same on another stream, optionally untimed (concurrent scales, PoseHip::submit_multi);
    // prepare() plans a shape ahead (its buffers are zeroed on the context stream)
    void forward_on(const float* input, int n, int h, int w, hipStream_t stream, bool timed);
    void prepare(int n, int h, int w);
    void time_begin(hipStream_t s) { timer_.begin(s); }
    void time_end(hipStream_t s) { timer_.end(s); }
    // net output of the last forward ([n][out_channels][out_h][out_w] fp32, stays valid until
    // set_conv or until more than kMaxShapes other shapes have been planned; a shape forwarded by
    // the pose pipeline alternates between two output buffers, select_output)
    float* output() const { return cur_ ? cur_->out() : nullptr; }
    // plans the shape and returns the output buffer its next forward writes; alternate: switch to
    // the shape's other buffer first (PoseHip: batch i+1's nets need not wait for the
    // post-processing of batch i, which reads the first)
    float* select_output(int n, int h, int w, bool alternate);
    // Readers of an output buffer outside the forward's stream order (PoseHip's post-processing
    // stream): ev was recorded after the last such read of out.  Every later forward that writes
    // out -- through PoseHip or a direct opk_net_forward -- first makes its stream wait for ev, so
    // the forward never overwrites values a post-processing still reads.  One event per buffer
    // (the readers run in order on one stream, so the latest covers the earlier ones).
    // expires when the net is destroyed: a PoseHip holding this net detects a net destroyed
    // before it (~PoseHip's forget_reader_events on a dead net)
    std::weak_ptr<void> liveness() const { return alive_; }
    void note_reader(const float* out, hipEvent_t ev);
    void forget_reader_events(const hipEvent_t* evs, int n);   // (the owner destroys them)
    int out_channels() const { return out_c_; }
    int out_h() const { return cur_ ? cur_->lh[out_level_] : 0; }
    int out_w() const { return cur_ ? cur_->lw[out_level_] : 0; }
    int frames() const { return cur_ ? cur_->n : 0; }
    static constexpr int kMaxShapes = 8;
    double flops_per_frame(int h, int w) const;   // useful (unpadded) conv FLOPs
    int border() const { return border_; }
    ~NetHip();

    // forward timing on the context stream (HIP events around every forward while enabled);
    // read() waits for the recorded forwards and returns their count and summed milliseconds
    void set_timing(bool on);
    void read_timing(int* count, double* total_ms);

    // caffe::Net::blob_by_name for the last forward (inspection / per-layer tests): frames
    // [f0, f0 + nf) of a named conv / pool / concat top as fp32 NCHW host [nf][ch][h][w], read from
    // its padded NHWC fp16 buffer (or the fp32 net output).  Blobs the fused kernels keep on chip
    // (conv1_1 / conv1_2 in conv1_fused, a pooled conv's un-pooled output, Mconv6 in conv_head)
    // throw.  host == nullptr: shape only.
    void blob(const std::string& name, int f0, int nf, float* host, int shape[4]) const;
    // kernels launched by the last forward run while the dev switch LAUNCH_LOG was 1
    const std::vector<std::string>& launches() const { return log_.lines; }

private:
    struct Placement { int buf; int coff; };
    struct BufSpec { int level; int cs; };
    struct ConvPlan {
        ConvInfo info;
        std::string in_blob;
        int level = 0;
        bool from_image = false;
        Placement in{};
        int cin_pad = 0, ntaps = 9, ksteps = 0, bn = 128, cout_pad = 0;
        std::vector<Placement> outs;
        int out32_coff = -1;
        DevBuf w, bias, slope;
        DevBuf w3;            // halo-kernel weight layout (3x3 convs)
        DevBuf wh;            // conv_head.hip layout when this conv is half of a fused head pair
        int head = -1;        // index into heads_ (as either half), -1 none
        bool loaded = false;
        bool slope01 = true;  // PReLU slopes all in [0, 1] (ConvArgs::actmax)
        float wscale = 1.f;   // split precision: 2^-e of the packed weights' scaling (ConvArgs::wscale)
        std::vector<float> hw, hb, hs;   // host copies of the weights (re-packed per precision)
    };
    void pack(ConvPlan& c);   // device layouts of one conv's weights for the current precision
    struct PoolPlan { int in_buf, out_buf, level_in, channels; };
    struct Step { bool conv; int idx; };

    // shape-dependent state of one input shape
    struct ShapePlan {
        int n = 0, h = 0, w = 0;
        std::vector<int> lh, lw;
        std::vector<std::unique_ptr<DevBuf>> mem;
        std::vector<uint16_t*> base;   // first position of each buffer (past its head guard)
        bool split = false;            // planned for kPrecisionSplit: every buffer has a lo twin
        std::vector<std::unique_ptr<DevBuf>> mem_lo;
        std::vector<uint16_t*> base_lo;
        DevBuf out_mem, out_mem_alt;
        float* out32 = nullptr;
        float* out32_alt = nullptr;    // the second output buffer (select_output)
        bool alt = false;              // forwards write out32_alt
        float* out() const { return alt ? out32_alt : out32; }
        bool fused1 = false;           // conv1_fused_kernel runs for this shape
        bool fusedh = false;           // conv_head_kernel runs the fused head pairs
        std::vector<char> poolfused;   // per pool: run inside its conv's epilogue (conv3w8 POOL)
        std::vector<ConvArgs> args;    // per conv
        std::vector<char> use3;        // per conv: launch conv3
    };

    void plan(const std::vector<LayerDesc>& layers);
    void forward_launches(ShapePlan& S, const float* input, int n, int h, int w, hipStream_t st);
    void forward_steps(ShapePlan& S, const float* input, int n, int h, int w, hipStream_t st);
    ShapePlan* shape_plan(int n, int h, int w, hipStream_t zero_stream = nullptr);

    Context* ctx_;
    std::string output_blob_;
    std::vector<ConvInfo> info_;
    std::vector<ConvPlan> convs_;
    std::map<std::string, int> conv_by_name_;
    std::vector<PoolPlan> pools_;
    std::vector<Step> steps_;
    std::vector<BufSpec> bufs_;
    int out_level_ = 0, out_c_ = 0, nlevels_ = 1;
    int image_buf_ = -1;
    struct Fuse1 { int a = -1, b = -1, p = -1, abuf = -1, bbuf = -1; };
    Fuse1 fuse1_;                 // conv1_1 -> conv1_2 -> pool1 (conv1_fused.hip) when planned
    // Mconv6 -> Mconv7 pairs (conv_head.hip): a = 1x1 conv with 256 / 512 outputs read only by b,
    // a 1x1 conv with <= 64 outputs, consecutive steps; buf = a's output buffer
    struct FuseHead { int a = -1, b = -1, step = -1, buf = -1; };
    std::vector<FuseHead> heads_;
    // conv -> 2x2 max pool pairs (conv3w8.hip POOL epilogue), per pool: the conv that alone feeds it
    // (and nothing else reads), -1 none; per input shape it runs fused where conv3w8 supports it
    std::vector<int> pool_conv_;
    int cus_ = 256;               // compute units (persistent-kernel grid)
    int precision_ = kPrecisionFp16;
    int border_ = 1;              // zero border of every padded image (widest conv pad, >= 1)

    struct BlobLoc { int buf = -1, coff = 0, ch = 0, level = 0; bool out32 = false; };
    std::map<std::string, BlobLoc> blob_loc_;   // every named top (plan)
    LaunchLog log_;

    std::vector<std::unique_ptr<ShapePlan>> shapes_;   // oldest first
    ShapePlan* cur_ = nullptr;    // shape of the last forward
    std::vector<std::pair<const float*, hipEvent_t>> readers_;   // note_reader
    std::shared_ptr<int> alive_ = std::make_shared<int>(0);       // liveness()
    DevBuf sink_;                 // persistent conv3: target of masked-off stores
    EventTimer timer_;            // forwards bracketed by HIP events (set_timing)
};

}  // namespace opk
