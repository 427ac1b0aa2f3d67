// graph.cpp -- prototxt reader + the generated BODY_25 graph.
//
// The reference loads its graph with caffe::Net<float>(prototxt) (netCaffe.cpp:177-185).  Here a
// small reader covers the text-format subset the OpenPose pose prototxts use (nested message
// blocks, `key: value`, quoted strings, # comments), and builtin_body25() generates
// models/pose/body_25/pose_deploy.prototxt so the GPU box needs no model files;
// tests/test_graph.py checks the two agree layer by layer when the reference tree is present.
#include "graph.h"

#include <cctype>
#include <fstream>
#include <sstream>

#include "../common.h"

namespace opk {

namespace {

struct Tok {
    enum Kind { Id, Str, Num, LBrace, RBrace, Colon, End } kind;
    std::string text;
};

class Lexer {
public:
    explicit Lexer(const std::string& s) : s_(s) {}
    Tok next()
    {
        skip();
        if (i_ >= s_.size()) return {Tok::End, ""};
        const char c = s_[i_];
        if (c == '{') { ++i_; return {Tok::LBrace, "{"}; }
        if (c == '}') { ++i_; return {Tok::RBrace, "}"}; }
        if (c == ':') { ++i_; return {Tok::Colon, ":"}; }
        if (c == '"' || c == '\'') {
            const size_t j = s_.find(c, i_ + 1);
            if (j == std::string::npos) throw Error(1, "prototxt: unterminated string");
            Tok t{Tok::Str, s_.substr(i_ + 1, j - i_ - 1)};
            i_ = j + 1;
            return t;
        }
        size_t j = i_;
        while (j < s_.size() && !std::isspace((unsigned char)s_[j]) && s_[j] != '{' &&
               s_[j] != '}' && s_[j] != ':' && s_[j] != '#')
            ++j;
        Tok t{std::isdigit((unsigned char)c) || c == '-' || c == '.' ? Tok::Num : Tok::Id,
              s_.substr(i_, j - i_)};
        i_ = j;
        return t;
    }

private:
    void skip()
    {
        while (i_ < s_.size()) {
            if (std::isspace((unsigned char)s_[i_])) ++i_;
            else if (s_[i_] == '#') { while (i_ < s_.size() && s_[i_] != '\n') ++i_; }
            else break;
        }
    }
    const std::string& s_;
    size_t i_ = 0;
};

// generic text-format message: repeated scalar fields + nested messages
struct Msg {
    std::vector<std::pair<std::string, std::string>> fields;
    std::vector<std::pair<std::string, Msg>> subs;
    std::string get(const std::string& k, const std::string& dflt = "") const
    {
        for (const auto& f : fields) if (f.first == k) return f.second;
        return dflt;
    }
    std::vector<std::string> all(const std::string& k) const
    {
        std::vector<std::string> v;
        for (const auto& f : fields) if (f.first == k) v.push_back(f.second);
        return v;
    }
    const Msg* sub(const std::string& k) const
    {
        for (const auto& s : subs) if (s.first == k) return &s.second;
        return nullptr;
    }
};

Msg parse_msg(Lexer& lx, bool top)
{
    Msg m;
    for (;;) {
        Tok t = lx.next();
        if (t.kind == Tok::End) {
            if (!top) throw Error(1, "prototxt: unexpected end of input");
            return m;
        }
        if (t.kind == Tok::RBrace) {
            if (top) throw Error(1, "prototxt: unbalanced '}'");
            return m;
        }
        if (t.kind != Tok::Id) throw Error(1, "prototxt: expected a field name, got '" + t.text + "'");
        Tok u = lx.next();
        if (u.kind == Tok::Colon) u = lx.next();
        if (u.kind == Tok::LBrace) {
            m.subs.emplace_back(t.text, parse_msg(lx, false));
        } else if (u.kind == Tok::Str || u.kind == Tok::Num || u.kind == Tok::Id) {
            m.fields.emplace_back(t.text, u.text);
        } else {
            throw Error(1, "prototxt: bad value for '" + t.text + "'");
        }
    }
}

int to_int(const std::string& s, int dflt) { return s.empty() ? dflt : std::stoi(s); }

}  // namespace

std::vector<LayerDesc> parse_prototxt(const std::string& text)
{
    Lexer lx(text);
    const Msg root = parse_msg(lx, true);
    std::vector<LayerDesc> out;
    for (const auto& s : root.subs) {
        if (s.first != "layer" && s.first != "layers") continue;
        const Msg& l = s.second;
        LayerDesc d;
        d.name = l.get("name");
        d.type = l.get("type");
        d.bottom = l.all("bottom");
        d.top = l.all("top");
        if (const Msg* c = l.sub("convolution_param")) {
            d.num_output = to_int(c->get("num_output"), 0);
            d.kernel_size = to_int(c->get("kernel_size"), 0);
            d.pad = to_int(c->get("pad"), 0);
            d.stride = to_int(c->get("stride"), 1);
        }
        if (const Msg* p = l.sub("pooling_param")) {
            d.pool = p->get("pool", "MAX");
            d.kernel_size = to_int(p->get("kernel_size"), 0);
            d.stride = to_int(p->get("stride"), 1);
            d.pad = to_int(p->get("pad"), 0);
        }
        if (const Msg* c = l.sub("concat_param")) d.concat_axis = to_int(c->get("axis"), 1);
        out.push_back(d);
    }
    return out;
}

std::vector<LayerDesc> load_prototxt(const std::string& path)
{
    std::ifstream f(path);
    if (!f) throw Error(1, "Prototxt file not found: " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return parse_prototxt(ss.str());
}

std::vector<LayerDesc> builtin_body25()
{
    std::vector<LayerDesc> L;
    auto conv = [&](const std::string& name, const std::string& bottom, int cout, int k,
                    const std::string& act) {
        LayerDesc d;
        d.name = name; d.type = "Convolution"; d.bottom = {bottom}; d.top = {name};
        d.num_output = cout; d.kernel_size = k; d.pad = k == 3 ? 1 : 0;
        L.push_back(d);
        if (act.empty()) return;
        LayerDesc a;
        a.type = act.rfind("relu", 0) == 0 ? "ReLU" : "PReLU";
        a.name = act; a.bottom = {name}; a.top = {name};
        L.push_back(a);
    };
    auto pool = [&](const std::string& name, const std::string& bottom) {
        LayerDesc d;
        d.name = name; d.type = "Pooling"; d.bottom = {bottom}; d.top = {name};
        d.kernel_size = 2; d.stride = 2;
        L.push_back(d);
    };
    auto concat = [&](const std::string& name, const std::vector<std::string>& bottoms) {
        LayerDesc d;
        d.name = name; d.type = "Concat"; d.bottom = bottoms; d.top = {name};
        L.push_back(d);
    };
    conv("conv1_1", "image", 64, 3, "relu1_1");
    conv("conv1_2", "conv1_1", 64, 3, "relu1_2");
    pool("pool1_stage1", "conv1_2");
    conv("conv2_1", "pool1_stage1", 128, 3, "relu2_1");
    conv("conv2_2", "conv2_1", 128, 3, "relu2_2");
    pool("pool2_stage1", "conv2_2");
    conv("conv3_1", "pool2_stage1", 256, 3, "relu3_1");
    conv("conv3_2", "conv3_1", 256, 3, "relu3_2");
    conv("conv3_3", "conv3_2", 256, 3, "relu3_3");
    conv("conv3_4", "conv3_3", 256, 3, "relu3_4");
    pool("pool3_stage1", "conv3_4");
    conv("conv4_1", "pool3_stage1", 512, 3, "relu4_1");
    conv("conv4_2", "conv4_1", 512, 3, "prelu4_2");
    conv("conv4_3_CPM", "conv4_2", 256, 3, "prelu4_3_CPM");
    conv("conv4_4_CPM", "conv4_3_CPM", 128, 3, "prelu4_4_CPM");
    // one refinement stage: 5 dense blocks of three 3x3 convs (outputs concatenated),
    // then 1x1 -> PReLU -> 1x1
    auto stage = [&](const std::string& tag, const std::string& input, int width, int mid,
                     int cout) {
        std::string x = input;
        for (int b = 1; b <= 5; ++b) {
            std::vector<std::string> parts;
            for (int j = 0; j < 3; ++j) {
                const std::string nm = "Mconv" + std::to_string(b) + "_" + tag + "_" + std::to_string(j);
                conv(nm, j == 0 ? x : parts.back(), width, 3,
                     "Mprelu" + std::to_string(b) + "_" + tag + "_" + std::to_string(j));
                parts.push_back(nm);
            }
            x = "Mconv" + std::to_string(b) + "_" + tag + "_concat";
            concat(x, parts);
        }
        conv("Mconv6_" + tag, x, mid, 1, "Mprelu6_" + tag);
        conv("Mconv7_" + tag, "Mconv6_" + tag, cout, 1, "");
        return "Mconv7_" + tag;
    };
    std::string paf = stage("stage0_L2", "conv4_4_CPM", 96, 256, 52);
    for (int s = 1; s <= 3; ++s) {
        const std::string c = "concat_stage" + std::to_string(s) + "_L2";
        concat(c, {"conv4_4_CPM", paf});
        paf = stage("stage" + std::to_string(s) + "_L2", c, 128, 512, 52);
    }
    concat("concat_stage0_L1", {"conv4_4_CPM", paf});
    std::string hm = stage("stage0_L1", "concat_stage0_L1", 96, 256, 26);
    concat("concat_stage1_L1", {"conv4_4_CPM", hm, paf});
    hm = stage("stage1_L1", "concat_stage1_L1", 128, 512, 26);
    concat("net_output", {hm, paf});
    return L;
}

namespace {
struct GraphBuilder {
    std::vector<LayerDesc> L;
    void conv(const std::string& name, const std::string& bottom, int cout, int k,
              const std::string& relu, const std::string& top = "")
    {
        LayerDesc d;
        d.name = name; d.type = "Convolution"; d.bottom = {bottom}; d.top = {top.empty() ? name : top};
        d.num_output = cout; d.kernel_size = k; d.pad = k / 2;
        L.push_back(d);
        if (relu.empty()) return;
        LayerDesc a;
        a.type = "ReLU"; a.name = relu; a.bottom = d.top; a.top = d.top;
        L.push_back(a);
    }
    void pool(const std::string& name, const std::string& bottom)
    {
        LayerDesc d;
        d.name = name; d.type = "Pooling"; d.bottom = {bottom}; d.top = {name};
        d.kernel_size = 2; d.stride = 2;
        L.push_back(d);
    }
    void concat(const std::string& name, const std::vector<std::string>& bottoms,
                const std::string& top = "")
    {
        LayerDesc d;
        d.name = name; d.type = "Concat"; d.bottom = bottoms; d.top = {top.empty() ? name : top};
        L.push_back(d);
    }
    // VGG-19 front of every CPM net: conv1_1 .. conv4_2 (pool names differ per model)
    void vgg(const std::string& p1, const std::string& p2, const std::string& p3,
             const std::string& relu_suffix_style)
    {
        auto r = [&](const std::string& c) {
            return relu_suffix_style == "re" ? c + "_re" : "relu" + c.substr(4);
        };
        conv("conv1_1", "image", 64, 3, r("conv1_1"));
        conv("conv1_2", "conv1_1", 64, 3, r("conv1_2"));
        pool(p1, "conv1_2");
        conv("conv2_1", p1, 128, 3, r("conv2_1"));
        conv("conv2_2", "conv2_1", 128, 3, r("conv2_2"));
        pool(p2, "conv2_2");
        conv("conv3_1", p2, 256, 3, r("conv3_1"));
        conv("conv3_2", "conv3_1", 256, 3, r("conv3_2"));
        conv("conv3_3", "conv3_2", 256, 3, r("conv3_3"));
        conv("conv3_4", "conv3_3", 256, 3, r("conv3_4"));
        pool(p3, "conv3_4");
        conv("conv4_1", p3, 512, 3, r("conv4_1"));
        conv("conv4_2", "conv4_1", 512, 3, r("conv4_2"));
    }
};
}  // namespace

std::vector<LayerDesc> builtin_cpm_pose(int pafs, int heat, int stages)
{
    // models/pose/{coco,mpi}/pose_deploy_linevec*.prototxt: VGG front, conv4_3_CPM / conv4_4_CPM,
    // a 3x3 stage 1 and 7x7 stages 2..N, two branches (L1 PAFs, L2 heat maps) interleaved layer by
    // layer; net_output = concat(L2, L1)
    GraphBuilder g;
    g.vgg("pool1_stage1", "pool2_stage1", "pool3_stage1", "relu");
    g.conv("conv4_3_CPM", "conv4_2", 256, 3, "relu4_3_CPM");
    g.conv("conv4_4_CPM", "conv4_3_CPM", 128, 3, "relu4_4_CPM");
    const char* br[2] = {"L1", "L2"};
    for (int j = 1; j <= 5; ++j)
        for (const char* b : br) {
            const std::string nm = "conv5_" + std::to_string(j) + "_CPM_" + b;
            const std::string in = j == 1 ? "conv4_4_CPM" : "conv5_" + std::to_string(j - 1) + "_CPM_" + b;
            const int cout = j <= 3 ? 128 : (j == 4 ? 512 : (b[1] == '1' ? pafs : heat));
            g.conv(nm, in, cout, j <= 3 ? 3 : 1, j == 5 ? "" : "relu5_" + std::to_string(j) + "_CPM_" + b);
        }
    std::string l1 = "conv5_5_CPM_L1", l2 = "conv5_5_CPM_L2";
    for (int s = 2; s <= stages; ++s) {
        const std::string st = "stage" + std::to_string(s);
        const std::string cat = "concat_" + st;
        g.concat(cat, {l1, l2, "conv4_4_CPM"});
        for (int j = 1; j <= 7; ++j)
            for (const char* b : br) {
                const std::string nm = "Mconv" + std::to_string(j) + "_" + st + "_" + b;
                const std::string in = j == 1 ? cat : "Mconv" + std::to_string(j - 1) + "_" + st + "_" + b;
                const int cout = j <= 6 ? 128 : (b[1] == '1' ? pafs : heat);
                g.conv(nm, in, cout, j <= 5 ? 7 : 1,
                       j == 7 ? "" : "Mrelu" + std::to_string(j) + "_" + st + "_" + b);
            }
        l1 = "Mconv7_" + st + "_L1";
        l2 = "Mconv7_" + st + "_L2";
    }
    g.concat("concat_stage7", {l2, l1}, "net_output");
    return g.L;
}

std::vector<LayerDesc> builtin_cpm_single(int outputs, bool face)
{
    // models/{hand,face}/pose_deploy.prototxt: VGG front to conv5_2, conv5_3_CPM, a 1x1 stage 1,
    // five 7x7 stages on concat(previous, conv5_3_CPM); the last conv's top is net_output
    GraphBuilder g;
    if (face) g.vgg("pool1", "pool2", "pool3", "re");
    else g.vgg("pool1_stage1", "pool2_stage1", "pool3_stage1", "relu");
    auto r = [&](const std::string& c, const std::string& hand_name) {
        return face ? c + "_re" : hand_name;
    };
    g.conv("conv4_3", "conv4_2", 512, 3, r("conv4_3", "relu4_3"));
    g.conv("conv4_4", "conv4_3", 512, 3, r("conv4_4", "relu4_4"));
    g.conv("conv5_1", "conv4_4", 512, 3, r("conv5_1", "relu5_1"));
    g.conv("conv5_2", "conv5_1", 512, 3, r("conv5_2", "relu5_2"));
    g.conv("conv5_3_CPM", "conv5_2", 128, 3, r("conv5_3_CPM", "relu5_4_stage1_3"));
    g.conv("conv6_1_CPM", "conv5_3_CPM", 512, 1, r("conv6_1_CPM", "relu6_4_stage1_1"));
    g.conv("conv6_2_CPM", "conv6_1_CPM", outputs, 1, "");
    std::string prev = "conv6_2_CPM";
    for (int s = 2; s <= 6; ++s) {
        const std::string st = "stage" + std::to_string(s);
        const std::string cat = face ? "features_in_stage_" + std::to_string(s) : "concat_" + st;
        g.concat(cat, {prev, "conv5_3_CPM"});
        for (int j = 1; j <= 7; ++j) {
            const std::string nm = "Mconv" + std::to_string(j) + "_" + st;
            const std::string in = j == 1 ? cat : "Mconv" + std::to_string(j - 1) + "_" + st;
            const std::string relu = j == 7 ? "" : r(nm, "Mrelu1_" + std::to_string(j + 1) + "_" + st + "_" + std::to_string(j));
            g.conv(nm, in, j <= 6 ? 128 : outputs, j <= 5 ? 7 : 1, relu,
                   (j == 7 && s == 6) ? "net_output" : "");
        }
        prev = "Mconv7_" + st;
    }
    return g.L;
}

std::vector<LayerDesc> builtin_graph(const std::string& name)
{
    if (name == "builtin:BODY_25") return builtin_body25();
    if (name == "builtin:COCO_18") return builtin_cpm_pose(38, 19, 6);
    if (name == "builtin:MPI_15") return builtin_cpm_pose(28, 16, 6);
    if (name == "builtin:MPI_15_4") return builtin_cpm_pose(28, 16, 4);
    if (name == "builtin:HAND") return builtin_cpm_single(22, false);
    if (name == "builtin:FACE") return builtin_cpm_single(71, true);
    throw Error(1, "unknown builtin graph " + name +
                       " (BODY_25, COCO_18, MPI_15, MPI_15_4, HAND, FACE)");
}

}  // namespace opk
