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
    };
    const std::vector<ConvInfo>& convs() const { return info_; }
    void set_conv(const std::string& name, const float* w, const float* b, const float* slope);
    bool ready() const;

    // input: device NCHW fp32 [n][3][h][w]
    void forward(const float* input, int n, int h, int w);
    float* output() const { return out32_; }
    int out_channels() const { return out_c_; }
    int out_h() const { return lh_.empty() ? 0 : lh_[out_level_]; }
    int out_w() const { return lw_.empty() ? 0 : lw_[out_level_]; }
    int frames() const { return n_; }
    double flops_per_frame(int h, int w) const;   // useful (unpadded) conv FLOPs

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
        bool use3 = false;    // launch conv3 (decided per input shape)
        bool loaded = false;
        ConvArgs args{};
    };
    struct PoolPlan { int in_buf, out_buf, level_in, channels; };
    struct Step { bool conv; int idx; };

    void plan(const std::vector<LayerDesc>& layers);
    void reshape(int n, int h, int w);

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
    bool conv_v1_ = false;
    struct Fuse1 { int a = -1, b = -1, p = -1, abuf = -1, bbuf = -1; };
    Fuse1 fuse1_;                 // conv1_1 -> conv1_2 -> pool1 (conv1_fused.hip) when planned
    bool fused1_active_ = false;  // ... and the input shape allows it
    int cus_ = 256;               // compute units (persistent-kernel grid)

    // shape-dependent state
    int n_ = 0, h_ = 0, w_ = 0;
    std::vector<int> lh_, lw_;
    std::vector<std::unique_ptr<DevBuf>> mem_;
    std::vector<uint16_t*> base_;   // first position of each buffer (past its head guard)
    DevBuf out_mem_;
    DevBuf sink_;                 // persistent conv3: target of masked-off stores
    float* out32_ = nullptr;
};

}  // namespace opk
