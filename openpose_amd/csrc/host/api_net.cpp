// api_net.cpp -- C-ABI (include/opk.h): NetHip (op::NetCaffe) and PoseHip
// (op::PoseExtractorCaffe) entry points.
#include <cstring>
#include <memory>
#include <string>

#include "../../../include/opk.h"
#include "net.h"
#include "caffemodel.h"
#include "extract.h"
#include "input.h"
#include "pose.h"

namespace opk {
template <class F>
static int guarded_net(F&& f)
{
    try {
        f();
        return OPK_OK;
    } catch (const Error& e) {
        set_error(e.what());
        return e.code;
    } catch (const std::exception& e) {
        set_error(e.what());
        return OPK_ERR_STATE;
    }
}
}  // namespace opk

struct opk_ctx : opk::Context {};
struct opk_net {
    opk_ctx* ctx;
    std::unique_ptr<opk::NetHip> net;
};
struct opk_pose {
    opk_ctx* ctx;
    std::unique_ptr<opk::PoseHip> pose;
};

using opk::guarded_net;

extern "C" {

int opk_net_create(opk_ctx* ctx, const char* prototxt, const char* caffemodel, opk_net** out)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(ctx && prototxt && out, "NULL argument");
        const std::string p(prototxt);
        std::vector<opk::LayerDesc> layers =
            p.rfind("builtin:", 0) == 0 ? opk::builtin_graph(p) : opk::load_prototxt(p);
        auto n = std::make_unique<opk_net>(opk_net{ctx, std::make_unique<opk::NetHip>(ctx, std::move(layers))});
        if (caffemodel && caffemodel[0]) {
            OPK_CHECK_ARG(ctx->device >= 0, "weights need a device context");
            n->net->load_caffemodel(caffemodel);
        }
        *out = n.release();
    });
}

int opk_net_destroy(opk_net* net)
{
    return guarded_net([&] {
        if (!net) return;
        if (net->ctx->device >= 0) net->ctx->bind();
        delete net;
    });
}

int opk_net_num_convs(opk_net* net)
{
    if (!net) return -1;
    return (int)net->net->convs().size();
}

int opk_net_conv_info(opk_net* net, int i, char* name, int* cin, int* cout, int* k, int* act)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(net && i >= 0 && i < (int)net->net->convs().size(), "bad index");
        const auto& c = net->net->convs()[i];
        if (name) {
            std::strncpy(name, c.name.c_str(), 63);
            name[63] = 0;
        }
        if (cin) *cin = c.cin;
        if (cout) *cout = c.cout;
        if (k) *k = c.k;
        if (act) *act = c.act;
    });
}

int opk_net_set_conv(opk_net* net, const char* name, const float* w, const float* b,
                     const float* slope)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(net && name, "NULL argument");
        net->net->set_conv(name, w, b, slope);
    });
}

int opk_net_forward(opk_net* net, const float* input, int n, int h, int w)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(net, "NULL net");
        net->net->forward(input, n, h, w);
    });
}

int opk_net_flops_per_frame(opk_net* net, int h, int w, double* flops)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(net && flops && h > 0 && w > 0, "bad argument");
        *flops = net->net->flops_per_frame(h, w);
    });
}

int opk_net_output(opk_net* net, float** out, int shape[4])
{
    return guarded_net([&] {
        OPK_CHECK_ARG(net && out && shape, "NULL argument");
        *out = net->net->output();   // NULL (and a {0, C, 0, 0} shape) before the first forward
        shape[0] = net->net->frames();
        shape[1] = net->net->out_channels();
        shape[2] = net->net->out_h();
        shape[3] = net->net->out_w();
    });
}

int opk_net_blob(opk_net* net, const char* name, int frame0, int nframes, float* host_out,
                 int shape[4])
{
    return guarded_net([&] {
        OPK_CHECK_ARG(net && name && shape, "NULL argument");
        net->net->blob(name, frame0, nframes, host_out, shape);
    });
}

int opk_net_launch_log(opk_net* net, char* buf, size_t size, size_t* needed)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(net && needed, "NULL argument");
        std::string text;
        for (const auto& l : net->net->launches()) text += l + "\n";
        *needed = text.size() + 1;
        if (buf && size >= *needed) std::memcpy(buf, text.c_str(), text.size() + 1);
    });
}

int opk_pose_create(opk_ctx* ctx, opk_net* net, int maxpos, opk_pose** out)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(ctx && out, "NULL argument");
        *out = new opk_pose{ctx, std::make_unique<opk::PoseHip>(ctx, net ? net->net.get() : nullptr,
                                                                maxpos != 0)};
    });
}

int opk_pose_create_model(opk_ctx* ctx, opk_net* net, int pose_model, int maxpos, int semantics,
                          opk_pose** out)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(ctx && out, "NULL argument");
        *out = new opk_pose{ctx, std::make_unique<opk::PoseHip>(ctx, net ? net->net.get() : nullptr,
                                                                maxpos != 0, pose_model, semantics)};
    });
}

int opk_pose_destroy(opk_pose* p)
{
    return guarded_net([&] {
        if (!p) return;
        if (p->ctx->device >= 0) p->ctx->bind();
        delete p;
    });
}

int opk_pose_set_map_semantics(opk_pose* p, int semantics)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->set_map_semantics(semantics);
    });
}

int opk_pose_set_property(opk_pose* p, int prop, double v)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->set_property(prop, v);
    });
}

int opk_pose_forward(opk_pose* p, const float* frames, int n, int net_h, int net_w, int pw, int ph)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->forward(frames, n, net_h, net_w, pw, ph);
    });
}

int opk_pose_forward_net_output(opk_pose* p, const float* out, int n, int oh, int ow, int net_h,
                                int net_w, int pw, int ph)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->forward_net_output(out, n, oh, ow, net_h, net_w, pw, ph);
    });
}

int opk_pose_submit(opk_pose* p, const float* frames, int n, int net_h, int net_w, int pw, int ph)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->submit(frames, n, net_h, net_w, pw, ph);
    });
}

int opk_pose_submit_multi(opk_pose* p, const float* const* frames, const int* net_hw, int nscales,
                          int n, int pw, int ph)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->submit_multi(frames, net_hw, nscales, n, pw, ph);
    });
}

int opk_pose_forward_multi(opk_pose* p, const float* const* frames, const int* net_hw,
                           int nscales, int n, int pw, int ph)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        OPK_CHECK_ARG(p->pose->pending() == 0, "batches in flight: collect them first");
        p->pose->submit_multi(frames, net_hw, nscales, n, pw, ph);
        p->pose->collect();
    });
}

int opk_pose_submit_net_output(opk_pose* p, const float* out, int n, int oh, int ow, int net_h,
                               int net_w, int pw, int ph)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->submit_net_output(out, n, oh, ow, net_h, net_w, pw, ph);
    });
}

int opk_pose_collect(opk_pose* p, int* frames)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        const int n = p->pose->collect();
        if (frames) *frames = n;
    });
}

int opk_pose_pending(opk_pose* p) { return p ? p->pose->pending() : -1; }

int opk_pose_set_upsampling_ratio(opk_pose* p, float ratio)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->set_upsampling_ratio(ratio);
    });
}

int opk_pose_set_overlay(opk_pose* p, const float* overlay)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->set_overlay(overlay);
    });
}

int opk_pose_num_people(opk_pose* p, int frame)
{
    if (!p || frame < 0 || frame >= p->pose->frames()) return -1;
    return p->pose->num_people(frame);
}

int opk_pose_keypoints(opk_pose* p, int frame, float* kp, float* ks, int max_people)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p && frame >= 0 && frame < p->pose->frames(), "bad frame");
        const int n = std::min(max_people, p->pose->num_people(frame));
        const auto& k = p->pose->keypoints(frame);
        const auto& s = p->pose->scores(frame);
        const int parts = opk::pose_model(p->pose->model()).parts;
        if (kp && n > 0) std::memcpy(kp, k.data(), sizeof(float) * n * parts * 3);
        if (ks && n > 0) std::memcpy(ks, s.data(), sizeof(float) * n);
    });
}

int opk_pose_set_timing(opk_pose* p, int enable)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->set_timing(enable != 0);
    });
}

int opk_pose_read_timing(opk_pose* p, int* batches, double* total_ms)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->read_timing(batches, total_ms);
    });
}

int opk_pose_read_collect_times(opk_pose* p, int* collects, double* wait_ms, double* assembly_ms,
                                int* workers)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->read_collect_times(collects, wait_ms, assembly_ms);
        if (workers) *workers = p->pose->assembly_workers();
    });
}

int opk_pose_records(opk_pose* p, float* rec, size_t capacity, size_t* used)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p && used, "NULL argument");
        const opk::PoseHip& pose = *p->pose;
        const int parts = opk::pose_model(pose.model()).parts;
        size_t need = 0;
        for (int f = 0; f < pose.frames(); ++f) need += 1 + (size_t)pose.num_people(f) * (parts * 3 + 1);
        *used = need;
        if (!rec) return;
        OPK_CHECK_ARG(capacity >= need, "records buffer too small");
        float* o = rec;
        for (int f = 0; f < pose.frames(); ++f) {
            const int n = pose.num_people(f);
            *o++ = (float)n;
            if (n == 0) continue;
            std::memcpy(o, pose.keypoints(f).data(), sizeof(float) * n * parts * 3);
            o += (size_t)n * parts * 3;
            std::memcpy(o, pose.scores(f).data(), sizeof(float) * n);
            o += n;
        }
    });
}

int opk_pose_heatmaps(opk_pose* p, float** heat, int shape[4])
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p && heat && shape, "NULL argument");
        *heat = p->pose->heatmaps(shape);
    });
}

int opk_pose_heatmap_size(opk_pose* p, int shape[4])
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p && shape, "NULL argument");
        p->pose->heatmap_size(shape);
    });
}

int opk_pose_peaks(opk_pose* p, float** peaks, int shape[4])
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p && peaks && shape, "NULL argument");
        *peaks = p->pose->peaks(shape);
    });
}

int opk_net_load_caffemodel(opk_net* net, const char* caffemodel, int* loaded)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(net && caffemodel, "NULL argument");
        OPK_CHECK_ARG(net->ctx->device >= 0, "weights need a device context");
        const int n = net->net->load_caffemodel(caffemodel);
        if (loaded) *loaded = n;
    });
}

int opk_caffemodel_blob(const char* caffemodel, const char* layer, int index, float* data,
                        size_t capacity, int64_t* shape, int* ndim)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(caffemodel && layer && ndim, "NULL argument");
        const auto layers = opk::load_caffemodel(caffemodel);
        for (const auto& L : layers) {
            if (L.name != layer) continue;
            OPK_CHECK_ARG(index >= 0 && index < (int)L.blobs.size(), "no such blob");
            const auto& b = L.blobs[index];
            OPK_CHECK_ARG(b.shape.size() <= 8, "blob rank > 8");
            *ndim = (int)b.shape.size();
            if (shape) for (size_t i = 0; i < b.shape.size(); ++i) shape[i] = b.shape[i];
            if (data) {
                OPK_CHECK_ARG(capacity >= b.data.size(), "capacity too small");
                std::memcpy(data, b.data.data(), b.data.size() * sizeof(float));
            }
            return;
        }
        throw opk::Error(1, std::string("layer ") + layer + " has no blobs in " + caffemodel);
    });
}

int opk_net_set_precision(opk_net* net, int precision)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(net, "NULL net");
        net->net->set_precision(precision);
    });
}

int opk_net_set_timing(opk_net* net, int enable)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(net, "NULL net");
        net->net->set_timing(enable != 0);
    });
}

int opk_net_read_timing(opk_net* net, int* forwards, double* total_ms)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(net, "NULL net");
        net->net->read_timing(forwards, total_ms);
    });
}

int opk_scale_and_size(int in_w, int in_h, int net_w, int net_h, float dynamic_behavior,
                       int scale_number, double scale_gap, double* scales, int* net_sizes)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(scales && net_sizes, "NULL output");
        opk::scale_and_size(in_w, in_h, net_w, net_h, dynamic_behavior, scale_number, scale_gap,
                            scales, net_sizes);
    });
}

int opk_cvmat_to_input(opk_ctx* ctx, float* input_dev, const uint8_t* frames_dev, int n, int width,
                       int height, size_t step, double scale, int net_w, int net_h, int normalize)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(ctx, "NULL context");
        OPK_CHECK_ARG(normalize == 0 || normalize == 1,
                      "normalize: 0 (none) or 1 (VGG); DenseNet (2) is not supported");
        opk::cvmat_to_input(ctx, input_dev, frames_dev, n, width, height, step, scale, net_w, net_h,
                            normalize);
    });
}

int opk_pose_set_input(opk_pose* p, int net_w, int net_h, float dynamic_behavior, int scale_number,
                       double scale_gap)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->set_input(net_w, net_h, dynamic_behavior, scale_number, scale_gap);
    });
}

int opk_pose_submit_frames(opk_pose* p, const uint8_t* frames, int n, int width, int height,
                           size_t step)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->submit_frames(frames, n, width, height, step);
    });
}

int opk_pose_forward_frames(opk_pose* p, const uint8_t* frames, int n, int width, int height,
                            size_t step)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->forward_frames(frames, n, width, height, step);
    });
}

int opk_pose_net_input(opk_pose* p, int scale, const float** input_dev, int* net_w, int* net_h)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p && input_dev, "NULL argument");
        *input_dev = p->pose->net_input(scale, net_w, net_h);
    });
}

int opk_pose_heatmaps_copy(opk_pose* p, int types, int scale_mode, float* dst_dev, int shape[4])
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p && shape, "NULL argument");
        p->pose->heatmaps_copy(types, scale_mode, dst_dev, shape);
    });
}

int opk_pose_candidates(opk_pose* p, int frame, float* candidates_host, int* counts_host)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(p, "NULL pose");
        p->pose->candidates(frame, candidates_host, counts_host);
    });
}

float opk_pose_scale_net_to_output(opk_pose* p) { return p ? p->pose->scale_net_to_output() : 0.f; }

}  // extern "C"

// ---- face / hand keypoints (op::FaceDetector, op::HandDetector, op::FaceExtractorCaffe,
//      op::HandExtractorCaffe) ----------------------------------------------------------------
struct opk_extractor {
    opk_ctx* ctx;
    std::unique_ptr<opk::KeypointExtractor> ex;
};

extern "C" {

int opk_face_detect(int pose_model, const float* keypoints, int people, int parts, float* rects)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(people == 0 || rects, "NULL rectangles");
        opk::detect_faces(pose_model, keypoints, people, parts, reinterpret_cast<opk::Rect*>(rects));
    });
}

int opk_hand_detect(int pose_model, const float* keypoints, int people, int parts, float* rects)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(people == 0 || rects, "NULL rectangles");
        opk::detect_hands(pose_model, keypoints, people, parts, reinterpret_cast<opk::Rect*>(rects));
    });
}

int opk_extractor_create(opk_ctx* ctx, opk_net* net, int kind, int net_w, int net_h,
                         opk_extractor** out)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(ctx && net && out, "NULL argument");
        OPK_CHECK_ARG(ctx->device >= 0, "extraction needs a device context");
        *out = new opk_extractor{
            ctx, std::make_unique<opk::KeypointExtractor>(ctx, net->net.get(), kind, net_w, net_h)};
    });
}

int opk_extractor_destroy(opk_extractor* ex)
{
    return guarded_net([&] { delete ex; });
}

int opk_extractor_set_scales(opk_extractor* ex, int number, float range)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(ex, "NULL extractor");
        ex->ex->set_scales(number, range);
    });
}

int opk_extractor_set_max_batch(opk_extractor* ex, int max_batch)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(ex, "NULL extractor");
        ex->ex->set_max_batch(max_batch);
    });
}

int opk_extractor_parts(opk_extractor* ex) { return ex ? ex->ex->parts() : -1; }

int opk_extractor_set_heatmaps(opk_extractor* ex, int scale_mode)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(ex, "NULL extractor");
        ex->ex->set_heatmaps(scale_mode);
    });
}

int opk_extractor_heatmaps(opk_extractor* ex, const float** heatmaps_dev, int shape[5])
{
    return guarded_net([&] {
        OPK_CHECK_ARG(ex && heatmaps_dev && shape, "NULL argument");
        *heatmaps_dev = ex->ex->heatmaps(shape);
    });
}

int opk_extractor_forward(opk_extractor* ex, const uint8_t* frames, int nframes, int width,
                          int height, size_t step, const float* rects, const int* frame_of,
                          int people, float* keypoints)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(ex && (people == 0 || keypoints), "NULL argument");
        ex->ex->extract(frames, nframes, width, height, step,
                        reinterpret_cast<const opk::Rect*>(rects), frame_of, people, keypoints);
    });
}

int opk_extractor_crop_count(opk_extractor* ex) { return ex ? ex->ex->crops() : -1; }

int opk_extractor_crop(opk_extractor* ex, int i, double* matrix, const float** input_dev)
{
    return guarded_net([&] {
        OPK_CHECK_ARG(ex, "NULL extractor");
        OPK_CHECK_ARG(i >= 0 && i < ex->ex->crops(), "crop index out of range");
        const auto* k = ex->ex.get();
        if (matrix) std::memcpy(matrix, k->crop_matrix(i), 6 * sizeof(double));
        if (input_dev) {
            // crops are laid out [crops][3][net_h][net_w]
            *input_dev = k->crop_inputs() + (size_t)i * 3 * k->net_w() * k->net_h();
        }
    });
}

}  // extern "C"
