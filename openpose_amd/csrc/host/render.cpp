// render.cpp -- C-ABI (include/opk.h) of the GPU renderers: renderPoseKeypointsGpu and the heat-map
// renders of src/openpose/pose/renderPose.cu:609-866, renderFaceKeypointsGpu
// (src/openpose/face/renderFace.cu:48-76) and renderHandKeypointsGpu
// (src/openpose/hand/renderHand.cu:48-76).  Same argument meaning, launch conditions and error
// texts; the scratch pointers of the reference signatures (maxPtr / minPtr / scalePtr) are not
// needed: the per-person boxes live in the context's own scratch (kernels/render.hip).
#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/opk.h"
#include "context.h"

namespace opk {

namespace {

struct RenderTableRow {
    const char* name;
    const unsigned* pairs;
    int npairs;
    const float* scales;
    int nscales;
    const float* colors;
    int ncolors;
};
#include "render_tables.inc"

enum RenderTable { kRtBody25, kRtCoco, kRtMpi, kRtBody19, kRtBody23, kRtBody25B, kRtBody135,
                   kRtCar12, kRtCar22, kRtFace, kRtHand };

// renderPoseKeypointsGpu's dispatch (renderPose.cu:639-741) and the kernels it launches
// (renderPose.cu:129-417): table, part count, googly-eye parts.  MPI draws MPI pairs / colors with
// COCO_SCALES (renderPose.cu:351) and has no googly eyes.
struct PoseRender {
    int table, scales_table, parts, eye1, eye2;
};
bool pose_render(int model, PoseRender* out)
{
    switch (model) {
    case 0: case 7: case 9: *out = {kRtBody25, kRtBody25, 25, 15, 16}; return true;  // BODY_25/E/D
    case 1: *out = {kRtCoco, kRtCoco, 18, 14, 15}; return true;                       // COCO_18
    case 2: case 3: *out = {kRtMpi, kRtCoco, 15, -1, -1}; return true;                // MPI_15(_4)
    case 4: case 5: case 6: case 12:
        *out = {kRtBody19, kRtBody19, 19, 15, 16}; return true;                       // BODY_19*
    case 8: *out = {kRtCar12, kRtCar12, 12, 4, 5}; return true;                       // CAR_12
    case 10: *out = {kRtBody23, kRtBody23, 23, 13, 14}; return true;                  // BODY_23
    case 11: *out = {kRtCar22, kRtCar22, 22, 6, 7}; return true;                      // CAR_22
    case 13: *out = {kRtBody25B, kRtBody25B, 25, 1, 2}; return true;                  // BODY_25B
    case 14: *out = {kRtBody135, kRtBody135, 135, 1, 2}; return true;                 // BODY_135
    default: return false;
    }
}

void check_alpha(float alpha)
{
    // checkAlpha (renderPose.cu:529-533)
    OPK_CHECK_ARG(!(alpha < 0.f || alpha > 1.f), "Alpha must be in the range [0, 1].");
}

void render_keypoints(Context* ctx, float* frame, unsigned w, unsigned h, const float* kp,
                      int people, int parts, int table, int scales_table, float radius_div,
                      float line_div, float threshold, float alpha, bool blend, int eye1, int eye2)
{
    OPK_CHECK_ARG(people <= kRenderMaxPeople,
                  "at most " + std::to_string(kRenderMaxPeople) + " people per frame");
    OPK_CHECK_ARG(people == 0 || kp != nullptr, "NULL keypoints");
    ctx->bind();
    const auto& t = ctx->render_table(table);
    const auto& st = ctx->render_table(scales_table);
    RenderKeypointsArgs a{};
    a.frame = frame;
    a.w = (int)w;
    a.h = (int)h;
    a.kp = kp;
    a.people = people;
    a.parts = parts;
    a.pairs = t.pairs;
    a.npairs = t.npairs;
    a.colors = t.colors;
    a.ncolors = t.ncolors;
    a.scales = st.scales;
    a.nscales = t.nscales;   // sizeof(<model>_SCALES) even where another table's values are read
    // fastMinCuda(targetWidth, targetHeight) / 100.f etc. (int / float)
    const int m = (int)w < (int)h ? (int)w : (int)h;
    a.radius = (float)m / radius_div;
    a.line_width = (float)m / line_div;
    a.threshold = threshold;
    a.alpha = alpha;
    a.blend = blend ? 1 : 0;
    a.eye1 = eye1;
    a.eye2 = eye2;
    a.geom = static_cast<float*>(
        ctx->render_geom.get(std::max<size_t>(1, render_geom_floats(people, parts, t.npairs)) *
                             sizeof(float)));
    launch_render_keypoints(a, ctx->stream);
}

RenderHeatArgs heat_args(float* frame, unsigned w, unsigned h, const float* heat, int hw, int hh,
                         float scale, float alpha)
{
    OPK_CHECK_ARG(frame && heat, "NULL argument");
    OPK_CHECK_ARG(hw > 0 && hh > 0, "empty heat map");
    check_alpha(alpha);
    return RenderHeatArgs{frame, (int)w, (int)h, heat, hw, hh, scale, alpha};
}

template <class F>
int guarded_render(F&& f)
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

}  // namespace

const Context::RenderDev& Context::render_table(int which)
{
    auto it = render_dev.find(which);
    if (it != render_dev.end()) return *it->second;
    const RenderTableRow& r = kRenderTableRows[which];
    const size_t np = 2 * (size_t)r.npairs, nc = 3 * (size_t)r.ncolors;
    std::vector<char> host((np + r.nscales + nc) * 4);
    std::memcpy(host.data(), r.pairs, np * 4);
    std::memcpy(host.data() + np * 4, r.scales, r.nscales * 4);
    std::memcpy(host.data() + (np + r.nscales) * 4, r.colors, nc * 4);
    auto d = std::make_unique<RenderDev>();
    char* dev = static_cast<char*>(d->buf.get(host.size()));
    OPK_HIP(hipMemcpyAsync(dev, host.data(), host.size(), hipMemcpyHostToDevice, stream));
    OPK_HIP(hipStreamSynchronize(stream));
    d->pairs = reinterpret_cast<const unsigned*>(dev);
    d->scales = reinterpret_cast<const float*>(dev + np * 4);
    d->colors = reinterpret_cast<const float*>(dev + (np + r.nscales) * 4);
    d->npairs = r.npairs;
    d->nscales = r.nscales;
    d->ncolors = r.ncolors;
    auto& ref = *d;
    render_dev.emplace(which, std::move(d));
    return ref;
}

}  // namespace opk

struct opk_ctx : opk::Context {};

extern "C" {

int opk_render_pose_keypoints(opk_ctx* ctx, float* frame, int pose_model, int people,
                              unsigned width, unsigned height, const float* pose, float threshold,
                              int googly_eyes, int blend_original, float alpha)
{
    return opk::guarded_render([&] {
        OPK_CHECK_ARG(ctx && frame, "NULL argument");
        if (!(people > 0 || !blend_original)) return;   // renderPose.cu:616
        opk::PoseRender pr{};
        const bool known = opk::pose_render(pose_model, &pr);
        OPK_CHECK_ARG(!(googly_eyes && (pose_model == 2 || pose_model == 3)),
                      "Bool googlyEyes not compatible with MPI models.");
        OPK_CHECK_ARG(people <= 127,
                      "Rendering assumes that numberPeople <= POSE_MAX_PEOPLE = 127.");
        OPK_CHECK_ARG(known, "Invalid Model.");
        opk::render_keypoints(ctx, frame, width, height, pose, people < 0 ? 0 : people, pr.parts,
                              pr.table, pr.scales_table, 100.f, 120.f, threshold, alpha,
                              blend_original != 0, googly_eyes ? pr.eye1 : -1,
                              googly_eyes ? pr.eye2 : -1);
    });
}

int opk_render_face_keypoints(opk_ctx* ctx, float* frame, unsigned width, unsigned height,
                              const float* face, int people, float threshold, float alpha)
{
    return opk::guarded_render([&] {
        OPK_CHECK_ARG(ctx && frame, "NULL argument");
        if (people <= 0) return;   // renderFace.cu:54
        // renderFaceParts (renderFace.cu:21-46): FACE_NUMBER_PARTS 70, radius min/120, line min/250
        opk::render_keypoints(ctx, frame, width, height, face, people, 70, opk::kRtFace,
                              opk::kRtFace, 120.f, 250.f, threshold, alpha, true, -1, -1);
    });
}

int opk_render_hand_keypoints(opk_ctx* ctx, float* frame, unsigned width, unsigned height,
                              const float* hands, int hands_n, float threshold, float alpha)
{
    return opk::guarded_render([&] {
        OPK_CHECK_ARG(ctx && frame, "NULL argument");
        if (hands_n <= 0) return;   // renderHand.cu:54
        // renderHandsParts (renderHand.cu:21-46): HAND_NUMBER_PARTS 21, radius min/100, line min/80
        opk::render_keypoints(ctx, frame, width, height, hands, hands_n, 21, opk::kRtHand,
                              opk::kRtHand, 100.f, 80.f, threshold, alpha, true, -1, -1);
    });
}

int opk_render_pose_heat_map(opk_ctx* ctx, float* frame, unsigned width, unsigned height,
                             const float* heat, int heat_w, int heat_h, float scale_to_keep_ratio,
                             unsigned part, float alpha)
{
    return opk::guarded_render([&] {
        OPK_CHECK_ARG(ctx != nullptr, "NULL argument");
        const auto a = opk::heat_args(frame, width, height, heat, heat_w, heat_h,
                                      scale_to_keep_ratio, alpha);
        ctx->bind();
        opk::launch_render_heat_map(a, (int)part, false, ctx->stream);
    });
}

int opk_render_pose_heat_maps(opk_ctx* ctx, float* frame, int pose_model, unsigned width,
                              unsigned height, const float* heat, int heat_w, int heat_h,
                              float scale_to_keep_ratio, float alpha)
{
    return opk::guarded_render([&] {
        OPK_CHECK_ARG(ctx != nullptr, "NULL argument");
        const auto a = opk::heat_args(frame, width, height, heat, heat_w, heat_h,
                                      scale_to_keep_ratio, alpha);
        const auto& m = opk::pose_model(pose_model);
        ctx->bind();
        const auto& coco = ctx->render_table(opk::kRtCoco);   // COCO_COLORS (renderPose.cu:427)
        opk::launch_render_heat_maps(a, m.parts, coco.colors, coco.ncolors, ctx->stream);
    });
}

int opk_render_pose_paf(opk_ctx* ctx, float* frame, int pose_model, unsigned width,
                        unsigned height, const float* heat, int heat_w, int heat_h,
                        float scale_to_keep_ratio, int part, float alpha)
{
    return opk::guarded_render([&] {
        OPK_CHECK_ARG(ctx != nullptr, "NULL argument");
        const auto a = opk::heat_args(frame, width, height, heat, heat_w, heat_h,
                                      scale_to_keep_ratio, alpha);
        (void)opk::pose_model(pose_model);
        ctx->bind();
        opk::launch_render_pafs(a, part, 1, ctx->stream);
    });
}

int opk_render_pose_pafs(opk_ctx* ctx, float* frame, int pose_model, unsigned width,
                         unsigned height, const float* heat, int heat_w, int heat_h,
                         float scale_to_keep_ratio, float alpha)
{
    return opk::guarded_render([&] {
        OPK_CHECK_ARG(ctx != nullptr, "NULL argument");
        const auto a = opk::heat_args(frame, width, height, heat, heat_w, heat_h,
                                      scale_to_keep_ratio, alpha);
        const auto& m = opk::pose_model(pose_model);
        ctx->bind();
        // renderPosePAFsGpu (renderPose.cu:818-834): every pair, from the first PAF channel
        opk::launch_render_pafs(a, m.parts + (m.bkg ? 1 : 0), m.npairs(), ctx->stream);
    });
}

int opk_render_pose_distance(opk_ctx* ctx, float* frame, unsigned width, unsigned height,
                             const float* heat, int heat_w, int heat_h, float scale_to_keep_ratio,
                             unsigned part, float alpha)
{
    return opk::guarded_render([&] {
        OPK_CHECK_ARG(ctx != nullptr, "NULL argument");
        const auto a = opk::heat_args(frame, width, height, heat, heat_w, heat_h,
                                      scale_to_keep_ratio, alpha);
        ctx->bind();
        // renderPoseDistanceGpu (renderPose.cu:836-864): renderBodyPartHeatMap with absValue
        opk::launch_render_heat_map(a, (int)part, true, ctx->stream);
    });
}

}  // extern "C"
