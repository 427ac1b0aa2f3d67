// net.cpp -- NetHip: plans a Caffe pose graph onto padded-NHWC fp16 buffers and runs it with the
// gfx950 kernels of kernels/conv.hip.
//
// Reference behaviour replaced: op::NetCaffe (src/openpose/net/netCaffe.cpp:27-279): build the
// caffe::Net from the prototxt, load weights, reshape the input blob when the size changes
// (:224-228), ForwardFrom(0) (:248), expose the `net_output` blob (:193-195).
// Planning (once per graph):
//   * ReLU/PReLU layers applied in place to a conv's top are fused into that conv's epilogue;
//   * every Concat gets one buffer; its bottoms are written straight into their channel slices
//     (a conv may write up to six such slices), so Concat costs nothing at run time;
//   * the output Concat (net_output) is an fp32 NCHW buffer written by the final 1x1 convs;
//   * the first conv (3 input channels) reads a 27-value im2col image (K = 32, one GEMM step).
// Buffers are allocated per input shape (frames x h x w) and kept; borders stay zero.
#include "net.h"

#include "caffemodel.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <set>

namespace opk {

namespace {
int round_up(int v, int m) { return (v + m - 1) / m * m; }
int pick_bn(int cout)
{
    if (cout <= 32) return 32;
    if (cout <= 64) return 64;
    if (cout <= 96) return 96;
    return 128;
}
}  // namespace

NetHip::NetHip(Context* ctx, std::vector<LayerDesc> layers, const std::string& output_blob)
    : ctx_(ctx), output_blob_(output_blob)
{
    plan(layers);
    if (ctx_->device >= 0) {
        ctx_->bind();
        OPK_HIP(hipDeviceGetAttribute(&cus_, hipDeviceAttributeMultiprocessorCount, ctx_->device));
    }
}

void NetHip::plan(const std::vector<LayerDesc>& layers)
{
    struct Blob { int ch = 0; int level = 0; int conv = -1; std::vector<Placement> places; };
    std::map<std::string, Blob> blobs;
    blobs["image"] = Blob{3, 0, -1, {}};
    std::map<std::string, int> convs_reading, pools_reading;   // consumers (besides concat)
    const LayerDesc* out_concat = nullptr;

    // pass 1: shapes, fused activations, conv/pool records
    for (size_t li = 0; li < layers.size(); ++li) {
        const LayerDesc& L = layers[li];
        if (L.type == "Input") continue;
        if (L.type == "Convolution") {
            OPK_CHECK_ARG(L.bottom.size() == 1 && L.top.size() == 1, L.name + ": one bottom/top");
            auto it = blobs.find(L.bottom[0]);
            OPK_CHECK_ARG(it != blobs.end(), L.name + ": unknown bottom " + L.bottom[0]);
            OPK_CHECK_ARG(L.stride == 1, L.name + ": only stride 1 convolutions");
            OPK_CHECK_ARG((L.kernel_size == 3 && L.pad == 1) || (L.kernel_size == 1 && L.pad == 0) ||
                              (L.kernel_size == 7 && L.pad == 3),
                          L.name + ": only 3x3/pad 1, 7x7/pad 3 and 1x1/pad 0 convolutions");
            border_ = std::max(border_, L.kernel_size / 2);
            ConvPlan c;
            c.info = ConvInfo{L.name, it->second.ch, L.num_output, L.kernel_size, 0};
            c.in_blob = L.bottom[0];
            c.level = it->second.level;
            c.from_image = L.bottom[0] == "image";
            OPK_CHECK_ARG(!c.from_image || (L.kernel_size == 3 && it->second.ch == 3),
                          L.name + ": the input conv must be 3x3 over 3 channels");
            // in-place activation directly after the conv
            if (li + 1 < layers.size()) {
                const LayerDesc& A = layers[li + 1];
                if ((A.type == "ReLU" || A.type == "PReLU") && A.bottom.size() == 1 &&
                    A.bottom[0] == L.top[0] && A.top.size() == 1 && A.top[0] == L.top[0])
                    c.info.act = A.type == "ReLU" ? 1 : 2;
                if (c.info.act) c.info.act_layer = A.name;
            }
            if (!c.from_image) convs_reading[L.bottom[0]]++;
            blobs[L.top[0]] = Blob{L.num_output, c.level, (int)convs_.size(), {}};
            conv_by_name_[L.name] = (int)convs_.size();
            convs_.push_back(std::move(c));
            steps_.push_back({true, (int)convs_.size() - 1});
        } else if (L.type == "ReLU" || L.type == "PReLU") {
            auto it = blobs.find(L.bottom[0]);
            OPK_CHECK_ARG(it != blobs.end() && it->second.conv >= 0 &&
                              convs_[it->second.conv].info.act != 0 && L.top[0] == L.bottom[0],
                          L.name + ": only in-place activations directly after a conv");
        } else if (L.type == "Pooling") {
            auto it = blobs.find(L.bottom[0]);
            OPK_CHECK_ARG(it != blobs.end() && it->second.conv >= 0, L.name + ": pool of a conv");
            OPK_CHECK_ARG(L.pool == "MAX" && L.kernel_size == 2 && L.stride == 2 && L.pad == 0,
                          L.name + ": only 2x2/2 max pooling");
            pools_reading[L.bottom[0]]++;
            blobs[L.top[0]] = Blob{it->second.ch, it->second.level + 1, -1, {}};
            pools_.push_back(PoolPlan{-1, -1, it->second.level, it->second.ch});
            steps_.push_back({false, (int)pools_.size() - 1});
            nlevels_ = std::max(nlevels_, it->second.level + 2);
        } else if (L.type == "Concat") {
            OPK_CHECK_ARG(L.concat_axis == 1, L.name + ": channel concat only");
            int ch = 0, level = -1;
            for (const auto& b : L.bottom) {
                auto it = blobs.find(b);
                OPK_CHECK_ARG(it != blobs.end() && it->second.conv >= 0,
                              L.name + ": concat bottoms must be conv outputs");
                OPK_CHECK_ARG(level < 0 || level == it->second.level, L.name + ": mixed sizes");
                level = it->second.level;
                ch += it->second.ch;
            }
            blobs[L.top[0]] = Blob{ch, level, -1, {}};
            if (L.top[0] == output_blob_) out_concat = &L;
        } else {
            throw Error(4, "layer type " + L.type + " (" + L.name + ") not supported by NetHip");
        }
    }
    // the output blob is a Concat of convs (the pose nets) or one conv's top (hand / face nets)
    if (!out_concat) {
        auto it = blobs.find(output_blob_);
        OPK_CHECK_ARG(it != blobs.end() && it->second.conv >= 0,
                      "output blob " + output_blob_ + " not produced by a Concat or a Convolution");
        ConvPlan& c = convs_[it->second.conv];
        c.out32_coff = 0;
        out_level_ = it->second.level;
        out_c_ = it->second.ch;
    }

    // pass 2: concat buffers and placements
    for (const auto& L : layers) {
        if (L.type != "Concat") continue;
        const Blob& top = blobs[L.top[0]];
        int off = 0;
        if (&L == out_concat) {
            out_level_ = top.level;
            out_c_ = top.ch;
            for (const auto& b : L.bottom) {
                ConvPlan& c = convs_[blobs[b].conv];
                c.out32_coff = off;
                off += blobs[b].ch;
            }
            continue;
        }
        const int buf = (int)bufs_.size();
        bufs_.push_back(BufSpec{top.level, round_up(top.ch, 32)});
        blobs[L.top[0]].places.push_back(Placement{buf, 0});
        for (const auto& b : L.bottom) {
            blobs[b].places.push_back(Placement{buf, off});
            off += blobs[b].ch;
        }
    }
    // pass 3: conv outputs that something reads directly need a readable placement
    for (auto& kv : blobs) {
        Blob& B = kv.second;
        if (B.conv < 0) continue;
        const bool pooled = pools_reading.count(kv.first) > 0;
        const bool read = convs_reading.count(kv.first) > 0;
        const int need = round_up(B.ch, 32);
        bool have = false;
        for (const auto& p : B.places)
            if (p.coff % 8 == 0 && p.coff + need <= bufs_[p.buf].cs) have = true;
        if (pooled || (read && !have) || (B.places.empty() && convs_[B.conv].out32_coff < 0)) {
            const int buf = (int)bufs_.size();
            bufs_.push_back(BufSpec{B.level, pooled ? round_up(B.ch, 8) : need});
            B.places.insert(B.places.begin(), Placement{buf, 0});
        }
        ConvPlan& c = convs_[B.conv];
        c.outs = B.places;
        OPK_CHECK_ARG(c.outs.size() <= (size_t)kConvMaxDst, c.info.name + ": too many consumers");
    }
    // pass 4: pool output buffers, then conv inputs and GEMM geometry
    int pi = 0;
    for (const auto& L : layers) {
        if (L.type != "Pooling") continue;
        PoolPlan& p = pools_[pi++];
        p.in_buf = blobs[L.bottom[0]].places.at(0).buf;
        OPK_CHECK_ARG(bufs_[p.in_buf].cs == round_up(p.channels, 8),
                      L.name + ": pool input must own its buffer");
        const int buf = (int)bufs_.size();
        bufs_.push_back(BufSpec{p.level_in + 1, round_up(p.channels, 8)});
        blobs[L.top[0]].places.push_back(Placement{buf, 0});
        p.out_buf = buf;
    }
    image_buf_ = (int)bufs_.size();
    bufs_.push_back(BufSpec{0, 32});
    // where every named top lives (blob(): inspection and per-layer tests)
    for (const auto& kv : blobs) {
        const Blob& B = kv.second;
        BlobLoc loc;
        loc.ch = B.ch;
        loc.level = B.level;
        if (kv.first == "image") continue;
        if (out_concat && kv.first == output_blob_) {
            loc.out32 = true;
        } else if (!B.places.empty()) {
            loc.buf = B.places[0].buf;
            loc.coff = B.places[0].coff;
        } else if (B.conv >= 0 && convs_[B.conv].out32_coff >= 0) {
            loc.out32 = true;
            loc.coff = convs_[B.conv].out32_coff;
        } else {
            continue;
        }
        blob_loc_[kv.first] = loc;
    }
    for (auto& c : convs_) {
        if (c.from_image) {
            c.in = Placement{image_buf_, 0};
            c.cin_pad = 32;
            c.ntaps = 1;
        } else {
            const Blob& B = blobs[c.in_blob];
            c.cin_pad = round_up(B.ch, 32);
            c.ntaps = c.info.k * c.info.k;
            bool found = false;
            for (const auto& p : B.places)
                if (p.coff % 8 == 0 && p.coff + c.cin_pad <= bufs_[p.buf].cs) {
                    c.in = p;
                    found = true;
                    break;
                }
            OPK_CHECK_ARG(found, c.info.name + ": no readable placement of " + c.in_blob);
        }
        c.ksteps = (c.ntaps * c.cin_pad + kConvBK - 1) / kConvBK;
        c.bn = pick_bn(c.info.cout);
        c.cout_pad = round_up(c.info.cout, c.bn);
        info_.push_back(c.info);
    }
    // conv1_1 -> conv1_2 -> pool1 fusion (conv1_fused.hip): the first conv feeds only the second,
    // whose output feeds only a pool, and nothing else reads either buffer
    if (steps_.size() >= 3 && steps_[0].conv && steps_[1].conv && !steps_[2].conv) {
        const ConvPlan& a = convs_[steps_[0].idx];
        const ConvPlan& b = convs_[steps_[1].idx];
        const PoolPlan& p = pools_[steps_[2].idx];
        const int abuf = a.outs.size() == 1 ? a.outs[0].buf : -1;
        const int bbuf = b.outs.size() == 1 ? b.outs[0].buf : -1;
        int readers_a = 0, readers_b = 0;
        for (const auto& c : convs_) {
            readers_a += c.in.buf == abuf;
            readers_b += c.in.buf == bbuf;
        }
        for (const auto& q : pools_) {
            readers_a += q.in_buf == abuf;
            readers_b += q.in_buf == bbuf;
        }
        if (a.from_image && a.info.k == 3 && a.info.cout == 64 && b.info.k == 3 &&
            b.info.cin == 64 && b.info.cout == 64 && abuf >= 0 && bbuf >= 0 && abuf != bbuf &&
            b.in.buf == abuf && p.in_buf == bbuf && readers_a == 1 && readers_b == 1 &&
            a.out32_coff < 0 && b.out32_coff < 0)
            fuse1_ = {steps_[0].idx, steps_[1].idx, steps_[2].idx, abuf, bbuf};
    }
    // conv -> pool pairs whose conv output only the pool reads (pool2 after conv2_2, pool3 after
    // conv3_4 in BODY_25; pool1 after conv1_2 where conv1_fused does not run -- split precision):
    // candidates for the pool-fused conv3w8 epilogue (128k or 64 outputs)
    pool_conv_.assign(pools_.size(), -1);
    for (size_t si = 0; si + 1 < steps_.size(); ++si) {
        if (!steps_[si].conv || steps_[si + 1].conv) continue;
        const ConvPlan& c = convs_[steps_[si].idx];
        const PoolPlan& p = pools_[steps_[si + 1].idx];
        if (c.from_image || c.info.k != 3 || c.outs.size() != 1 || c.outs[0].coff != 0 ||
            c.out32_coff >= 0 || (c.info.cout % 128 != 0 && c.info.cout != 64) || border_ != 1 ||
            p.in_buf != c.outs[0].buf)
            continue;
        int readers = 0;
        for (const auto& q : convs_) readers += q.in.buf == p.in_buf;
        for (const auto& q : pools_) readers += q.in_buf == p.in_buf;
        if (readers == 1) pool_conv_[steps_[si + 1].idx] = steps_[si].idx;
    }
    // Mconv6 -> Mconv7 head pairs (conv_head.hip)
    for (size_t si = 0; si + 1 < steps_.size(); ++si) {
        if (!steps_[si].conv || !steps_[si + 1].conv) continue;
        ConvPlan& a = convs_[steps_[si].idx];
        ConvPlan& b = convs_[steps_[si + 1].idx];
        if (a.info.k != 1 || b.info.k != 1 || a.outs.size() != 1 || a.out32_coff >= 0 ||
            a.head >= 0 || a.from_image || border_ != 1)
            continue;
        const int abuf = a.outs[0].buf;
        int readers = 0;
        for (const auto& c : convs_) readers += c.in.buf == abuf;
        for (const auto& q : pools_) readers += q.in_buf == abuf;
        if (readers != 1 || b.in.buf != abuf || b.in.coff != a.outs[0].coff || a.outs[0].coff != 0 ||
            b.info.cin != a.info.cout || !conv_head_supported(a.info.cout, b.info.cout, a.cin_pad))
            continue;
        a.head = b.head = (int)heads_.size();
        heads_.push_back(FuseHead{steps_[si].idx, steps_[si + 1].idx, (int)si, abuf});
        ++si;
    }
}

void NetHip::set_conv(const std::string& name, const float* w, const float* b, const float* slope)
{
    auto it = conv_by_name_.find(name);
    OPK_CHECK_ARG(it != conv_by_name_.end(), "no convolution named " + name);
    ConvPlan& c = convs_[it->second];
    OPK_CHECK_ARG(w && b, name + ": weights and bias required");
    OPK_CHECK_ARG(c.info.act != 2 || slope, name + ": PReLU slopes required");
    c.hw.assign(w, w + (size_t)c.info.cout * c.info.cin * c.info.k * c.info.k);
    c.hb.assign(b, b + c.info.cout);
    if (slope) c.hs.assign(slope, slope + c.info.cout);
    else c.hs.clear();
    pack(c);
    c.loaded = true;
    shapes_.clear();   // re-derive launch arguments
    cur_ = nullptr;
}

void NetHip::set_precision(int precision)
{
    OPK_CHECK_ARG(precision == kPrecisionFp16 || precision == kPrecisionSplit, "unknown precision");
    if (precision == precision_) return;
    precision_ = precision;
    for (auto& c : convs_)
        if (c.loaded) pack(c);
    shapes_.clear();
    cur_ = nullptr;
}

void NetHip::pack(ConvPlan& c)
{
    const std::string& name = c.info.name;
    (void)name;
    const float* w = c.hw.data();
    const float* b = c.hb.data();
    const float* slope = c.hs.empty() ? nullptr : c.hs.data();
    const bool split = precision_ == kPrecisionSplit;
    const int K = c.ksteps * kConvBK;
    const int cin = c.info.cin, k = c.info.k;
    const bool need_packed = c.from_image;   // conv_image's layout: [cout_pad][64]
    std::vector<uint16_t> packed(need_packed ? (size_t)c.cout_pad * K : 0, 0);
    auto f2h = [](float v) { _Float16 h = (_Float16)v; return __builtin_bit_cast(uint16_t, h); };
    // split precision: the layer's weights scaled by 2^e, max |w| * 2^e in [2^14, 2^15), so that
    // w_lo = fp16(w' - w_hi) stays a normal fp16 number (ConvArgs::wscale); the kernels multiply
    // the sums by 2^-e (exact) before the bias.  fp16: unscaled.
    int wexp = 0;
    if (split) {
        float mx = 0.f;
        for (size_t e = 0; e < c.hw.size(); ++e) mx = std::max(mx, std::fabs(w[e]));
        if (mx > 0.f && std::isfinite(mx)) {
            int ex = 0;
            (void)std::frexp(mx, &ex);   // mx in [2^(ex-1), 2^ex)
            wexp = std::max(-100, std::min(100, 15 - ex));
        }
    }
    c.wscale = std::ldexp(1.f, -wexp);
    auto wsc = [&](float v) { return std::ldexp(v, wexp); };   // exact (no overflow / underflow here)
    for (int co = 0; co < c.info.cout && need_packed; ++co) {
        uint16_t* dst = packed.data() + (size_t)co * K;
        if (c.from_image) {   // K index (ky*3 + kx)*3 + ci; split: w_lo at K + 32
            for (int ci = 0; ci < 3; ++ci)
                for (int ky = 0; ky < 3; ++ky)
                    for (int kx = 0; kx < 3; ++kx) {
                        const float wv = wsc(w[(((size_t)co * 3 + ci) * 3 + ky) * 3 + kx]);
                        const int kk = (ky * 3 + kx) * 3 + ci;
                        dst[kk] = f2h(wv);
                        if (split) dst[32 + kk] = f2h(wv - (float)(_Float16)wv);
                    }
            continue;
        }
        for (int t = 0; t < c.ntaps; ++t) {
            const int ky = k == 3 ? t / 3 : 0, kx = k == 3 ? t % 3 : 0;
            for (int ci = 0; ci < cin; ++ci)
                dst[t * c.cin_pad + ci] = f2h(w[(((size_t)co * cin + ci) * k + ky) * k + kx]);
        }
    }
    // conv3.hip layout: [cout_pad/BN][cin_pad/32][ky][kx][n BN][ci 32]; split precision: two
    // blocks of chunks, [cout_pad/BN][2][cin_pad/32]..., holding w_hi and w_lo -- the K loop's
    // three products per chunk read w_hi, w_lo, w_hi (ConvArgs::split)
    std::vector<uint16_t> packed3;
    if (!c.from_image) {
        const int BN = conv3_shape(1, 1, 1, c.info.cout, k, border_).bn;   // BN depends on cout only
        const int nb = (c.info.cout + BN - 1) / BN, cpt = c.cin_pad / 32, kt = k * k;
        const int passes = split ? 2 : 1;
        packed3.assign((size_t)nb * passes * cpt * kt * BN * 32, 0);
        for (int co = 0; co < c.info.cout; ++co)
            for (int ci = 0; ci < cin; ++ci)
                for (int t = 0; t < kt; ++t) {
                    const float wv = wsc(w[(((size_t)co * cin + ci) * k + t / k) * k + t % k]);
                    const _Float16 hi = (_Float16)wv;
                    for (int ps = 0; ps < passes; ++ps) {
                        const size_t idx = ((((size_t)(co / BN) * passes * cpt + ps * cpt + ci / 32) * kt + t) *
                                                BN + co % BN) * 32 + ci % 32;
                        packed3[idx] = ps == 0 ? __builtin_bit_cast(uint16_t, hi)
                                               : f2h(wv - (float)hi);
                    }
                }
    }
    // conv_head.hip layouts: Mconv6 [cin_pad/32][n1][32]; Mconv7 K-permuted [n2 <= 32 ? 32 : 64][n1];
    // split precision: a w_hi block, then a w_lo block, of each (HeadArgs::split)
    std::vector<uint16_t> packedh;
    if (c.head >= 0) {
        const FuseHead& fh = heads_[c.head];
        const int passes = split ? 2 : 1;
        auto part = [&](float wv, int ps) {
            const _Float16 hi = (_Float16)wv;
            return ps == 0 ? __builtin_bit_cast(uint16_t, hi) : f2h(wv - (float)hi);
        };
        if (&convs_[fh.a] == &c) {
            const int n1 = c.info.cout, cpt = c.cin_pad / 32;
            packedh.assign((size_t)passes * cpt * n1 * 32, 0);
            for (int ps = 0; ps < passes; ++ps)
                for (int co = 0; co < n1; ++co)
                    for (int ci = 0; ci < cin; ++ci)
                        packedh[(((size_t)ps * cpt + ci / 32) * n1 + co) * 32 + ci % 32] =
                            part(wsc(w[(size_t)co * cin + ci]), ps);
        } else {
            const int n1 = cin, n2 = c.info.cout, n2p = n2 <= 32 ? 32 : 64;
            std::vector<uint16_t> w7((size_t)n2 * n1);
            packedh.assign((size_t)passes * n2p * n1, 0);
            for (int ps = 0; ps < passes; ++ps) {
                for (size_t e = 0; e < w7.size(); ++e) w7[e] = part(wsc(w[e]), ps);
                conv_head_pack_w7(packedh.data() + (size_t)ps * n2p * n1, w7.data(), n1, n2);
            }
        }
    }
    // bias/slope zero-padded to a multiple of 128 channels (conv3 reads whole 4-channel groups)
    const size_t cpad = (size_t)(c.info.cout + 127) / 128 * 128;
    std::vector<float> bias(cpad, 0.f), sl(cpad, 0.f);
    std::copy(b, b + c.info.cout, bias.begin());
    if (slope) std::copy(slope, slope + c.info.cout, sl.begin());
    c.slope01 = true;
    if (slope)
        for (int i = 0; i < c.info.cout; ++i) c.slope01 = c.slope01 && slope[i] >= 0.f && slope[i] <= 1.f;
    ctx_->bind();
    if (!packed3.empty()) {
        void* dw3 = c.w3.get(packed3.size() * 2);
        OPK_HIP(hipMemcpyAsync(dw3, packed3.data(), packed3.size() * 2, hipMemcpyHostToDevice,
                               ctx_->stream));
    }
    if (!packedh.empty()) {
        void* dwh = c.wh.get(packedh.size() * 2);
        OPK_HIP(hipMemcpyAsync(dwh, packedh.data(), packedh.size() * 2, hipMemcpyHostToDevice,
                               ctx_->stream));
    }
    void* db = c.bias.get(bias.size() * 4);
    void* ds = c.slope.get(sl.size() * 4);
    if (!packed.empty()) {
        void* dw = c.w.get(packed.size() * 2);
        OPK_HIP(hipMemcpyAsync(dw, packed.data(), packed.size() * 2, hipMemcpyHostToDevice,
                               ctx_->stream));
    }
    OPK_HIP(hipMemcpyAsync(db, bias.data(), bias.size() * 4, hipMemcpyHostToDevice, ctx_->stream));
    OPK_HIP(hipMemcpyAsync(ds, sl.data(), sl.size() * 4, hipMemcpyHostToDevice, ctx_->stream));
    OPK_HIP(hipStreamSynchronize(ctx_->stream));
}

bool NetHip::ready() const
{
    for (const auto& c : convs_) if (!c.loaded) return false;
    return true;
}

double NetHip::flops_per_frame(int h, int w) const
{
    std::vector<int> H(nlevels_), W(nlevels_);
    H[0] = h;
    W[0] = w;
    for (int l = 1; l < nlevels_; ++l) {
        H[l] = (H[l - 1] - 2 + 1) / 2 + 1;
        W[l] = (W[l - 1] - 2 + 1) / 2 + 1;
    }
    double f = 0;
    for (const auto& c : convs_)
        f += 2.0 * H[c.level] * W[c.level] * c.info.cout * c.info.cin * c.info.k * c.info.k;
    return f;
}

NetHip::ShapePlan* NetHip::shape_plan(int n, int h, int w, hipStream_t zero_stream)
{
    // least recently used first: a lookup moves its plan to the back, so the plans of the scales
    // of one multi-scale batch (<= kMaxShapes, prepared before it is submitted) stay resident
    for (size_t i = 0; i < shapes_.size(); ++i)
        if (shapes_[i]->n == n && shapes_[i]->h == h && shapes_[i]->w == w) {
            std::unique_ptr<ShapePlan> sp = std::move(shapes_[i]);
            shapes_.erase(shapes_.begin() + i);
            shapes_.push_back(std::move(sp));
            return shapes_.back().get();
        }
    if ((int)shapes_.size() >= kMaxShapes) {
        if (cur_ == shapes_.front().get()) cur_ = nullptr;
        shapes_.erase(shapes_.begin());
    }
    shapes_.push_back(std::make_unique<ShapePlan>());
    ShapePlan& S = *shapes_.back();
    S.n = n;
    S.h = h;
    S.w = w;
    std::vector<int>& lh_ = S.lh;
    std::vector<int>& lw_ = S.lw;
    lh_.assign(nlevels_, 0);
    lw_.assign(nlevels_, 0);
    lh_[0] = h;
    lw_[0] = w;
    for (int l = 1; l < nlevels_; ++l) {   // Caffe ceil sizing for 2x2/2 pooling
        lh_[l] = (lh_[l - 1] - 2 + 1) / 2 + 1;
        lw_[l] = (lw_[l - 1] - 2 + 1) / 2 + 1;
    }
    std::vector<uint16_t*>& ptr = S.base;
    ptr.assign(bufs_.size(), nullptr);
    // CONV1_FUSED=0 (opk_dev_set, A/B tests): the three separate kernels instead of the fusion
    S.split = precision_ == kPrecisionSplit;   // (split precision: no conv1 fusion)
    S.fused1 = !S.split && fuse1_.a >= 0 && dev_switch("CONV1_FUSED", 1) != 0 && border_ == 1 &&
               conv1_fused_supported(h, w, 64, 64);
    // HEAD_FUSE=0 (opk_dev_set, A/B tests): Mconv6 and Mconv7 as two conv3 launches
    // Positions are decoded by float-reciprocal division in conv_head_kernel, exact below 2^24:
    // larger batches run the pairs unfused.
    // (split precision: conv_head_kernel's split instantiations; HEAD_FUSE_SPLIT=0, dev A/B: the
    // unfused split pair)
    S.fusedh = (!S.split || dev_switch("HEAD_FUSE_SPLIT", 1) != 0) && !heads_.empty() &&
               dev_switch("HEAD_FUSE", 1) != 0;
    for (const auto& fh : heads_) {
        const int L = convs_[fh.a].level;
        S.fusedh = S.fusedh && (long)n * (lh_[L] + 2) * (lw_[L] + 2) < (1L << 24);
    }
    // POOL_FUSE=0 (opk_dev_set, A/B tests): the pools as their own kernels
    S.poolfused.assign(pools_.size(), 0);
    for (size_t q = 0; q < pools_.size(); ++q) {
        const int ci = pool_conv_[q];
        if (ci < 0 || dev_switch("POOL_FUSE", 1) == 0) continue;
        if (S.fused1 && (int)q == fuse1_.p) continue;   // (pool1 inside conv1_fused_kernel)
        const ConvPlan& c = convs_[ci];
        const int H = lh_[c.level], W = lw_[c.level];
        // (64 outputs: conv3w8's BN = 64 tile, when the conv may take it -- conv3_w8_eligible)
        std::vector<int> pcs, pco;
        for (const auto& o : c.outs) {
            pcs.push_back(bufs_[o.buf].cs);
            pco.push_back(o.coff);
        }
        const bool w8 = !pcs.empty() && conv3_w8_eligible(c.info.cout, c.ntaps, (int)c.outs.size(),
                                                          pcs.data(), pco.data(), c.out32_coff >= 0);
        const Conv3Shape s3 = conv3_shape(n, H, W, c.info.cout, 3, border_, w8);
        S.poolfused[q] = s3.persist && s3.nw == 16 && H % 2 == 0 && W % 2 == 0 && s3.sw % 2 == 0 &&
                         6 * (s3.sw + 2) <= 512 && s3.sw + 2 > 16 &&
                         lh_[c.level + 1] == H / 2 && lw_[c.level + 1] == W / 2;
    }
    S.base_lo.assign(bufs_.size(), nullptr);
    for (size_t i = 0; i < bufs_.size(); ++i) {
        S.mem.push_back(std::make_unique<DevBuf>());
        S.mem_lo.push_back(std::make_unique<DevBuf>());
        // conv_image reads the NCHW input itself (in both precisions)
        if ((int)i == image_buf_) continue;
        bool head_buf = false;
        for (const auto& fh : heads_) head_buf = head_buf || fh.buf == (int)i;
        if (S.fusedh && head_buf) continue;   // Mconv6 outputs live only inside conv_head_kernel
        if (S.fused1 && ((int)i == fuse1_.abuf || (int)i == fuse1_.bbuf))
            continue;   // conv1_1 / conv1_2 outputs live only inside conv1_fused_kernel
        bool pooled_away = false;
        for (size_t q = 0; q < pools_.size(); ++q)
            pooled_away = pooled_away || (S.poolfused[q] && pools_[q].in_buf == (int)i);
        if (pooled_away) continue;   // written pooled by its conv's epilogue
        // zeroed guards: the kernels read up to W+3 positions before the first frame and up to
        // kConvGuardTail positions after the last one (conv.h)
        const int L = bufs_[i].level, B = border_;
        const size_t head = (size_t)B * (lw_[L] + 2 * B) + B + 64;
        const size_t pos = head + (size_t)n * (lh_[L] + 2 * B) * (lw_[L] + 2 * B) + kConvGuardTail;
        const size_t bytes = pos * bufs_[i].cs * 2;
        OPK_CHECK_ARG(pos * bufs_[i].cs < (size_t)1 << 31, "activation buffer exceeds 2^31 elements");
        uint16_t* raw = static_cast<uint16_t*>(S.mem.back()->get(bytes));
        // zeroed on the stream whose kernels read the plan first
        OPK_HIP(hipMemsetAsync(raw, 0, bytes, zero_stream ? zero_stream : ctx_->stream));
        ptr[i] = raw + head * bufs_[i].cs;
        if (S.split) {   // the lo twin: same layout, zeroed borders and guards
            uint16_t* rl = static_cast<uint16_t*>(S.mem_lo.back()->get(bytes));
            OPK_HIP(hipMemsetAsync(rl, 0, bytes, zero_stream ? zero_stream : ctx_->stream));
            S.base_lo[i] = rl + head * bufs_[i].cs;
        }
    }
    const size_t out_bytes = (size_t)n * out_c_ * lh_[out_level_] * lw_[out_level_] * 4;
    S.out32 = static_cast<float*>(S.out_mem.get(out_bytes));
    void* sink = sink_.get(kConv3SinkBytes);
    S.args.assign(convs_.size(), ConvArgs{});
    S.use3.assign(convs_.size(), 0);
    for (size_t ci = 0; ci < convs_.size(); ++ci) {
        const ConvPlan& c = convs_[ci];
        ConvArgs& a = S.args[ci];
        const int H = lh_[c.level], W = lw_[c.level], Wp = W + 2 * border_;
        a.in = ptr[c.in.buf];
        a.in_cs = bufs_[c.in.buf].cs;
        a.in_coff = c.in.coff;
        a.cin_pad = c.cin_pad;
        a.ntaps = c.ntaps;
        if (a.ntaps == 9)
            for (int t = 0; t < 9; ++t) a.tapoff[t] = (t / 3) * Wp + (t % 3);
        else if (a.ntaps == 1)
            a.tapoff[0] = Wp + 1;
        a.border = border_;
        a.ksteps = c.ksteps;
        const bool use3 = !c.from_image;
        S.use3[ci] = use3;
        OPK_CHECK_ARG(use3 || c.w.ptr != nullptr, c.info.name + ": weights not set");
        if (use3) {
            // (conv3w8's 64-output tile: decided from the destinations as launch_conv3 decides)
            std::vector<int> dcs, dco;
            for (const auto& o : c.outs) {
                dcs.push_back(bufs_[o.buf].cs);
                dco.push_back(o.coff);
            }
            const bool w8 = !dcs.empty() && conv3_w8_eligible(c.info.cout, a.ntaps, (int)c.outs.size(),
                                                              dcs.data(), dco.data(), c.out32_coff >= 0);
            const Conv3Shape s3 = conv3_shape(n, H, W, c.info.cout, c.info.k, border_, w8);
            a.sw = s3.sw;
            a.nstrips = s3.nstrips;
            a.sink = sink;
            // GRID_CUS (opk_dev_set, dev): persistent grids of fewer CUs, e.g. two pipelines on
            // concurrent streams sharing the chip
            a.cus = std::min(cus_, std::max(1, dev_switch("GRID_CUS", cus_)));
        }
        a.w = static_cast<const uint16_t*>(use3 ? c.w3.ptr : c.w.ptr);
        a.bias = static_cast<const float*>(c.bias.ptr);
        a.slope = static_cast<const float*>(c.slope.ptr);
        a.act = c.info.act;
        a.actmax = dev_switch("EPI_MAX", 1) != 0;   // and the conv's slopes (at launch: set_conv may follow)
        a.frames = n;
        a.H = H;
        a.W = W;
        a.M = n * H * Wp;
        a.cout = c.info.cout;
        a.ndst = (int)c.outs.size();
        for (size_t d = 0; d < c.outs.size(); ++d) {
            a.dst[d] = ptr[c.outs[d].buf];
            a.dst_cs[d] = bufs_[c.outs[d].buf].cs;
            a.dst_coff[d] = c.outs[d].coff;
            a.dst_lo[d] = S.base_lo[c.outs[d].buf];
        }
        a.split = S.split ? 1 : 0;
        a.wscale = S.split ? c.wscale : 1.f;
        a.in_lo = S.base_lo[c.in.buf];
        for (size_t q = 0; q < pools_.size(); ++q)
            if (S.poolfused[q] && pool_conv_[q] == (int)ci) {   // the pooled image instead
                a.pool = 1;
                a.ndst = 1;
                a.dst[0] = ptr[pools_[q].out_buf];
                a.dst_lo[0] = S.base_lo[pools_[q].out_buf];   // (split precision: its lo twin)
                a.dst_cs[0] = bufs_[pools_[q].out_buf].cs;
                a.dst_coff[0] = 0;
            }
        if (c.out32_coff >= 0) {
            OPK_CHECK_ARG(c.level == out_level_, c.info.name + ": output at another resolution");
            a.out32 = S.out32;
            a.out32_c = out_c_;
            a.out32_coff = c.out32_coff;
        }
    }
    return &S;
}

void NetHip::forward(const float* input, int n, int h, int w)
{
    forward_on(input, n, h, w, ctx_->stream, true);
}

float* NetHip::select_output(int n, int h, int w, bool alternate)
{
    OPK_CHECK_ARG(n > 0 && h > 0 && w > 0, "empty input");
    ctx_->bind();
    ShapePlan& S = *shape_plan(n, h, w, ctx_->stream);
    if (alternate) {
        if (!S.out32_alt) {
            const size_t bytes = (size_t)n * out_c_ * S.lh[out_level_] * S.lw[out_level_] * 4;
            S.out32_alt = static_cast<float*>(S.out_mem_alt.get(bytes));
        }
        S.alt = !S.alt;
    }
    return S.out();
}

void NetHip::note_reader(const float* out, hipEvent_t ev)
{
    for (auto& r : readers_)
        if (r.first == out) {
            r.second = ev;
            return;
        }
    readers_.emplace_back(out, ev);
}

void NetHip::forget_reader_events(const hipEvent_t* evs, int n)
{
    for (size_t i = readers_.size(); i-- > 0;)
        for (int k = 0; k < n; ++k)
            if (readers_[i].second == evs[k]) {
                readers_.erase(readers_.begin() + (long)i);
                break;
            }
}

void NetHip::prepare(int n, int h, int w)
{
    OPK_CHECK_ARG(n > 0 && h > 0 && w > 0, "empty input");
    ctx_->bind();
    (void)shape_plan(n, h, w, ctx_->stream);
}

void NetHip::forward_on(const float* input, int n, int h, int w, hipStream_t st, bool timed)
{
    OPK_CHECK_ARG(input && n > 0 && h > 0 && w > 0, "empty input");
    OPK_CHECK_ARG(ready(), "weights not loaded for every convolution");
    ctx_->bind();
    ShapePlan& S = *shape_plan(n, h, w, st);
    cur_ = &S;
    for (const auto& r : readers_)   // post-processings still reading this output buffer
        if (r.first == S.out()) OPK_HIP(hipStreamWaitEvent(st, r.second, 0));
    if (timed) timer_.begin(st);
    forward_launches(S, input, n, h, w, st);
    if (timed) timer_.end(st);
}

void NetHip::blob(const std::string& name, int f0, int nf, float* host, int shape[4]) const
{
    OPK_CHECK_ARG(cur_ != nullptr, "no forward yet");
    const auto it = blob_loc_.find(name);
    OPK_CHECK_ARG(it != blob_loc_.end(), "no blob named " + name);
    const BlobLoc& L = it->second;
    const ShapePlan& S = *cur_;
    OPK_CHECK_ARG(f0 >= 0 && nf > 0 && f0 + nf <= S.n, "frames out of range");
    const int H = S.lh[L.level], W = S.lw[L.level];
    if (shape) {
        shape[0] = nf; shape[1] = L.ch; shape[2] = H; shape[3] = W;
    }
    if (!host) return;
    ctx_->bind();
    OPK_HIP(hipStreamSynchronize(ctx_->stream));
    const size_t hw = (size_t)H * W;
    if (L.out32) {
        OPK_CHECK_ARG(L.level == out_level_, name + ": not at the output resolution");
        for (int f = 0; f < nf; ++f)
            OPK_HIP(hipMemcpy(host + (size_t)f * L.ch * hw,
                              S.out() + ((size_t)(f0 + f) * out_c_ + L.coff) * hw,
                              (size_t)L.ch * hw * 4, hipMemcpyDeviceToHost));
        return;
    }
    OPK_CHECK_ARG(S.base[L.buf] != nullptr,
                  name + ": kept on chip by a fused kernel (not materialised at this shape)");
    const int B = border_, Wp = W + 2 * B, Hp = H + 2 * B, cs = bufs_[L.buf].cs;
    const size_t frame_elems = (size_t)Hp * Wp * cs;
    std::vector<uint16_t> raw(frame_elems * nf), rlo(S.split ? frame_elems * nf : 0);
    OPK_HIP(hipMemcpy(raw.data(), S.base[L.buf] + (size_t)f0 * frame_elems, raw.size() * 2,
                      hipMemcpyDeviceToHost));
    if (S.split)   // split precision: the value is hi + lo
        OPK_HIP(hipMemcpy(rlo.data(), S.base_lo[L.buf] + (size_t)f0 * frame_elems, rlo.size() * 2,
                          hipMemcpyDeviceToHost));
    for (int f = 0; f < nf; ++f)
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                const size_t at = f * frame_elems + ((size_t)(y + B) * Wp + x + B) * cs + L.coff;
                const uint16_t* src = raw.data() + at;
                for (int c = 0; c < L.ch; ++c)
                    host[((size_t)f * L.ch + c) * hw + (size_t)y * W + x] =
                        (float)__builtin_bit_cast(_Float16, src[c]) +
                        (S.split ? (float)__builtin_bit_cast(_Float16, rlo[at + c]) : 0.f);
            }
}

void NetHip::forward_launches(ShapePlan& S, const float* input, int n, int h, int w, hipStream_t st)
{
    const bool logging = dev_switch("LAUNCH_LOG", 0) != 0;
    if (logging) {
        log_.lines.clear();
        attach_launch_log(&log_);
    }
    struct Detach {
        bool on;
        ~Detach() { if (on) attach_launch_log(nullptr); }
    } detach{logging};
    forward_steps(S, input, n, h, w, st);
}

// conv3 over the frames of a batch in as few launches as its 24-bit position arithmetic allows
// (the full-resolution layers of a large batch run unfused only in split precision): each launch
// takes a run of whole frames, its pointers moved to the run's first frame -- the positions just
// before and after a run are frame borders, zero like the guards of a whole-batch launch.
//
// Runs are sized evenly (ceil(frames / runs) frames each), and each run takes the strip geometry
// conv3_shape chooses for ITS frame count: the planner's sw / nstrips were chosen for the whole
// batch, and a run with fewer tiles may fall into another tile branch (another halo, so another
// strip count) -- launch_conv3 requires the geometry of its own frame count.
static bool conv3_run_fits(const ConvArgs& a, int frames, int ks, int B)
{
    const Conv3Shape s = conv3_shape(frames, a.H, a.W, a.cout, ks, B, conv3_w8_eligible(a));
    const long total = (long)frames * s.nstrips * (a.H + 2 * B) * (s.sw + 2 * B);
    return total + s.bm + (long)(ks - 1) * (s.sw + 2 * B + 1) < (1L << 24);
}

static void launch_conv3_frames(const ConvArgs& a, hipStream_t st)
{
    const int B = a.border > 0 ? a.border : 1;
    const int ks = a.ntaps == 49 ? 7 : (a.ntaps == 9 ? 3 : 1);
    if (conv3_run_fits(a, a.frames, ks, B)) {
        launch_conv3(a, st);
        return;
    }
    int runs = 2;
    for (;; ++runs) {   // the fewest even runs whose every run fits (a run of 1 frame always does)
        const int run = (a.frames + runs - 1) / runs;
        const int last = a.frames - ((a.frames + run - 1) / run - 1) * run;
        if (conv3_run_fits(a, run, ks, B) && conv3_run_fits(a, last, ks, B)) break;
        OPK_CHECK_ARG(run > 1, "launch_conv3_frames: one frame exceeds a launch's position range");
    }
    const int run = (a.frames + runs - 1) / runs;
    const size_t frame_pos = (size_t)(a.H + 2 * B) * (a.W + 2 * B);   // padded image positions
    // a pooled destination (conv3w8 POOL epilogue) holds the pooled padded image per frame
    const size_t dst_pos = a.pool ? (size_t)(a.H / 2 + 2 * B) * (a.W / 2 + 2 * B) : frame_pos;
    for (int f0 = 0; f0 < a.frames; f0 += run) {
        ConvArgs b = a;
        b.frames = std::min(run, a.frames - f0);
        const Conv3Shape sb = conv3_shape(b.frames, a.H, a.W, a.cout, ks, B, conv3_w8_eligible(a));
        b.sw = sb.sw;
        b.nstrips = sb.nstrips;
        b.M = b.frames * a.H * (a.W + 2 * B);
        b.in = a.in + f0 * frame_pos * a.in_cs;
        if (a.in_lo) b.in_lo = a.in_lo + f0 * frame_pos * a.in_cs;
        for (int d = 0; d < a.ndst; ++d) {
            b.dst[d] = a.dst[d] + f0 * dst_pos * a.dst_cs[d];
            if (a.dst_lo[d]) b.dst_lo[d] = a.dst_lo[d] + f0 * dst_pos * a.dst_cs[d];
        }
        if (a.out32) b.out32 = a.out32 + (size_t)f0 * a.out32_c * a.H * a.W;
        launch_conv3(b, st);
    }
}

void NetHip::forward_steps(ShapePlan& S, const float* input, int n, int h, int w, hipStream_t st)
{
    LaunchLog* log = launch_log();
    float* const out32 = S.out();   // this forward's output buffer (select_output)
    const std::vector<uint16_t*>& ptr = S.base;
    const std::vector<int>& lh_ = S.lh;
    const std::vector<int>& lw_ = S.lw;
    size_t first = 0;
    if (S.fused1) {
        const ConvPlan& a = convs_[fuse1_.a];
        const ConvPlan& b = convs_[fuse1_.b];
        const PoolPlan& p = pools_[fuse1_.p];
        Conv1FusedArgs fa{};
        fa.img = input;
        fa.frames = n;
        fa.H = h;
        fa.W = w;
        fa.w1 = static_cast<const uint16_t*>(a.w.ptr);
        fa.b1 = static_cast<const float*>(a.bias.ptr);
        fa.s1 = static_cast<const float*>(a.slope.ptr);
        fa.act1 = a.info.act;
        fa.w2 = static_cast<const uint16_t*>(b.w3.ptr);
        fa.b2 = static_cast<const float*>(b.bias.ptr);
        fa.s2 = static_cast<const float*>(b.slope.ptr);
        fa.act2 = b.info.act;
        fa.out = ptr[p.out_buf];
        fa.out_cs = bufs_[p.out_buf].cs;
        fa.out_coff = 0;
        fa.OH = lh_[1];
        fa.OW = lw_[1];
        fa.actmax = a.slope01 && b.slope01 && dev_switch("EPI_MAX", 1) != 0;
        if (log) log->layer = a.info.name + "+" + b.info.name + "+pool";
        launch_conv1_fused(fa, std::min(cus_, std::max(1, dev_switch("GRID_CUS", cus_))), st);
        first = 3;
    }
    for (size_t si = first; si < steps_.size(); ++si) {
        const Step& s = steps_[si];
        if (s.conv) {
            const ConvPlan& c = convs_[s.idx];
            const ConvArgs& a = S.args[s.idx];
            if (S.fusedh && c.head >= 0 && heads_[c.head].step == (int)si) {
                const FuseHead& fh = heads_[c.head];
                const ConvPlan& cb = convs_[fh.b];
                const ConvArgs& b = S.args[fh.b];
                HeadArgs h{};
                h.in = a.in;
                h.in_cs = a.in_cs;
                h.in_coff = a.in_coff;
                h.cin_pad = a.cin_pad;
                h.w6 = static_cast<const uint16_t*>(c.wh.ptr);
                h.b6 = a.bias;
                h.s6 = a.slope;
                h.act6 = a.act;
                h.actmax = a.actmax && c.slope01;
                h.w7 = static_cast<const uint16_t*>(cb.wh.ptr);
                h.b7 = b.bias;
                h.n1 = c.info.cout;
                h.n2 = cb.info.cout;
                h.frames = n;
                h.H = a.H;
                h.W = a.W;
                h.ndst = b.ndst;
                for (int d = 0; d < b.ndst; ++d) {
                    h.dst[d] = b.dst[d];
                    h.dst_cs[d] = b.dst_cs[d];
                    h.dst_coff[d] = b.dst_coff[d];
                }
                h.out32 = b.out32 ? out32 : nullptr;
                h.out32_c = b.out32_c;
                h.out32_coff = b.out32_coff;
                // persistent grid (HEAD_PERSIST=0: one workgroup per tile, dev A/B)
                h.cus = dev_switch("HEAD_PERSIST", 1) != 0 ? a.cus : 0;
                if (S.split) {
                    h.split = 1;
                    h.in_lo = a.in_lo;
                    for (int d = 0; d < b.ndst; ++d) h.dst_lo[d] = b.dst_lo[d];
                    h.wscale6 = a.wscale;
                    h.wscale7 = b.wscale;
                }
                if (log) log->layer = c.info.name + "+" + cb.info.name;
                launch_conv_head(h, st);
                ++si;   // Mconv7 ran inside
                continue;
            }
            if (log) log->layer = c.info.name + (a.pool ? "+pool" : "");
            if (c.from_image) {
                ConvArgs ai = a;
                if (ai.out32) ai.out32 = out32;
                launch_conv_image(ai, input, st);
            } else {
                ConvArgs a3 = a;
                a3.actmax = a.actmax && c.slope01;
                if (a3.out32) a3.out32 = out32;
                launch_conv3_frames(a3, st);
            }
        } else {
            if (S.poolfused[s.idx]) continue;   // ran in its conv's epilogue
            const PoolPlan& p = pools_[s.idx];
            const int L = p.level_in;
            if (log) log->layer = "pool";
            if (S.split)
                launch_maxpool2_split(ptr[p.out_buf], S.base_lo[p.out_buf], ptr[p.in_buf],
                                      S.base_lo[p.in_buf], n, lh_[L], lw_[L], bufs_[p.in_buf].cs,
                                      lh_[L + 1], lw_[L + 1], st, border_);
            else
                launch_maxpool2(ptr[p.out_buf], ptr[p.in_buf], n, lh_[L], lw_[L],
                                bufs_[p.in_buf].cs, lh_[L + 1], lw_[L + 1], st, border_);
        }
    }
}

int NetHip::load_caffemodel(const std::string& path)
{
    const std::vector<CaffeLayer> layers = opk::load_caffemodel(path);
    std::map<std::string, const CaffeLayer*> by_name;
    for (const auto& L : layers) by_name[L.name] = &L;
    int loaded = 0;
    for (const ConvInfo& c : info_) {
        auto it = by_name.find(c.name);
        if (it == by_name.end()) continue;   // kept as set (Caffe keeps the filler's values)
        const auto& blobs = it->second->blobs;
        OPK_CHECK_ARG(blobs.size() == 2, c.name + ": expected weights and bias blobs, got " +
                                             std::to_string(blobs.size()));
        const std::vector<int64_t> wshape{c.cout, c.cin, c.k, c.k}, bshape{c.cout};
        // CopyTrainedLayersFrom's check (net.cpp: "Cannot copy param ... shape mismatch")
        OPK_CHECK_ARG(blob_shape_is(blobs[0], wshape), "Cannot copy param 0 weights from layer '" +
                                                           c.name + "'; shape mismatch.");
        OPK_CHECK_ARG(blob_shape_is(blobs[1], bshape), "Cannot copy param 1 weights from layer '" +
                                                           c.name + "'; shape mismatch.");
        const float* slope = nullptr;
        if (c.act == 2) {
            auto pt = by_name.find(c.act_layer);
            OPK_CHECK_ARG(pt != by_name.end() && pt->second->blobs.size() == 1 &&
                              blob_shape_is(pt->second->blobs[0], bshape),
                          c.act_layer + ": PReLU slopes missing or of the wrong shape");
            slope = pt->second->blobs[0].data.data();
        }
        set_conv(c.name, blobs[0].data.data(), blobs[1].data.data(), slope);
        ++loaded;
    }
    return loaded;
}

NetHip::~NetHip() = default;

void NetHip::set_timing(bool on)
{
    timer_.on = on;
}

void NetHip::read_timing(int* count, double* total_ms)
{
    timer_.read(count, total_ms);
}

}  // namespace opk
