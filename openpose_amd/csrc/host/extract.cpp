// extract.cpp -- face / hand detectors and the batched crop -> keypoint pipeline (extract.h).
// Built with -ffp-contract=off: the rectangles, the warp tables and the keypoint mapping round
// every float / double operation as the reference's CPU code does.
#include "extract.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "../common.h"
#include "../kernels/kernels.h"
#include "pose_model.h"

namespace opk {

namespace {

// getDistance (keypoint.cpp:12-26)
float distance(const float* p, int a, int b)
{
    const float dx = p[a * 3] - p[b * 3];
    const float dy = p[a * 3 + 1] - p[b * 3 + 1];
    return std::sqrt(dx * dx + dy * dy);
}

// getFaceFromPoseKeypoints (faceDetector.cpp:22-119)
Rect face_from_pose(const float* p, int neck, int nose, int lear, int rear, int leye, int reye)
{
    const float th = 0.25f;
    const bool neck_ok = p[neck * 3 + 2] > th, nose_ok = p[nose * 3 + 2] > th;
    const bool lear_ok = p[lear * 3 + 2] > th, rear_ok = p[rear * 3 + 2] > th;
    const bool leye_ok = p[leye * 3 + 2] > th, reye_ok = p[reye * 3 + 2] > th;
    float tx = 0.f, ty = 0.f, size = 0.f;
    int counter = 0;
    if (nose == lear && lear == rear) {   // head and neck given (MPI)
        if (neck_ok && nose_ok) {
            tx = p[nose * 3];
            ty = p[nose * 3 + 1];
            size = 1.33f * distance(p, neck, nose);
        }
    } else {
        if (neck_ok && nose_ok) {
            // profile (one eye and ear visible): average of nose, eye and ear
            if (leye_ok == lear_ok && reye_ok == rear_ok && leye_ok != reye_ok) {
                const int eye = leye_ok ? leye : reye, ear = leye_ok ? lear : rear;
                tx += (p[eye * 3] + p[ear * 3] + p[nose * 3]) / 3.f;
                ty += (p[eye * 3 + 1] + p[ear * 3 + 1] + p[nose * 3 + 1]) / 3.f;
                size += 0.85f * (distance(p, nose, eye) + distance(p, nose, ear) +
                                 distance(p, neck, nose));
            } else {
                tx += (p[neck * 3] + p[nose * 3]) / 2.f;
                ty += (p[neck * 3 + 1] + p[nose * 3 + 1]) / 2.f;
                size += 2.f * distance(p, neck, nose);
            }
            ++counter;
        }
        if (leye_ok && reye_ok) {
            tx += (p[leye * 3] + p[reye * 3]) / 2.f;
            ty += (p[leye * 3 + 1] + p[reye * 3 + 1]) / 2.f;
            size += 3.f * distance(p, leye, reye);
            ++counter;
        }
        if (lear_ok && rear_ok) {
            tx += (p[lear * 3] + p[rear * 3]) / 2.f;
            ty += (p[lear * 3 + 1] + p[rear * 3 + 1]) / 2.f;
            size += 2.f * distance(p, lear, rear);
            ++counter;
        }
        if (counter > 0) {
            tx /= (float)counter;
            ty /= (float)counter;
            size /= counter;
        }
    }
    return Rect{tx - size / 2, ty - size / 2, size, size};
}

// getHandFromPoseIndexes (handDetector.cpp:9-42)
Rect hand_from_pose(const float* p, int wrist, int elbow, int shoulder)
{
    const float th = 0.03f;
    Rect r{0.f, 0.f, 0.f, 0.f};
    if (p[wrist * 3 + 2] > th && p[elbow * 3 + 2] > th && p[shoulder * 3 + 2] > th) {
        const float ratio = 0.33f;
        r.x = p[wrist * 3] + ratio * (p[wrist * 3] - p[elbow * 3]);
        r.y = p[wrist * 3 + 1] + ratio * (p[wrist * 3 + 1] - p[elbow * 3 + 1]);
        const float we = distance(p, wrist, elbow);
        const float es = 0.9f * distance(p, elbow, shoulder);
        r.width = 1.5f * (we > es ? we : es);   // fastMax
    }
    r.height = r.width;
    r.x -= r.width / 2.f;
    r.y -= r.height / 2.f;
    return r;
}

const std::vector<int>& detector_keys(int model, bool hands)
{
    const PoseModelInfo& m = pose_model(model);
    const int first = hands ? kLWrist : kNeck, last = hands ? kRShoulder : kREye;
    for (int k = first; k <= last; ++k)
        if (m.keys[k] < 0)
            throw Error(4 /* OPK_ERR_UNSUPPORTED */, std::string("pose model ") + m.name +
                                                 " has no keypoints for the " +
                                                 (hands ? "hand" : "face") + " detector");
    return m.keys;
}

// Rectangle::recenter / op::recenter (rectangle.cpp:114-128, 216-233)
Rect recenter(const Rect& r, float w, float h)
{
    const float cx = r.x + r.width / 2, cy = r.y + r.height / 2;
    return Rect{cx - w / 2.f, cy - h / 2.f, w, h};
}

// warpAffine(INTER_LINEAR | WARP_INVERSE_MAP) of a map with M01 = M10 = 0 is separable: the
// source column depends on the destination column only, the row on the row only
// (imgwarp.cpp WarpAffineInvoker: X0 = cvRound((M01*y + M02)*AB_SCALE) + round_delta,
// adelta[x] = cvRound(M00*x*AB_SCALE), Y0 = cvRound((M11*y + M12)*AB_SCALE) + round_delta,
// bdelta = 0; coordinate >> (AB_BITS - INTER_BITS))
void crop_axis_tables(const double* M, int dw, int dh, int* xt, int* yt)
{
    const int rd = 1024 / 32 / 2;
    const int x0 = (int)std::lrint(M[2] * 1024) + rd;   // M01 * y = 0
    for (int x = 0; x < dw; ++x) {
        const int X = (x0 + (int)std::lrint(M[0] * x * 1024)) >> 5;
        xt[2 * x] = X >> 5;
        xt[2 * x + 1] = X & 31;
    }
    for (int y = 0; y < dh; ++y) {   // bdelta = cvRound(M10 * x * 1024) = 0
        const int Y = ((int)std::lrint((M[4] * y + M[5]) * 1024) + rd) >> 5;
        yt[2 * y] = Y >> 5;
        yt[2 * y + 1] = Y & 31;
    }
}

}  // namespace

void detect_faces(int model, const float* kp, int people, int parts, Rect* out)
{
    OPK_CHECK_ARG(people >= 0 && (people == 0 || kp), "NULL keypoints");
    const std::vector<int>& k = detector_keys(model, false);
    OPK_CHECK_ARG(people == 0 || parts == pose_model(model).parts, "parts != the model's");
    for (int i = 0; i < people; ++i)
        out[i] = face_from_pose(kp + (size_t)i * parts * 3, k[kNeck], k[kNose], k[kLEar],
                                k[kREar], k[kLEye], k[kREye]);
}

void detect_hands(int model, const float* kp, int people, int parts, Rect* out)
{
    OPK_CHECK_ARG(people >= 0 && (people == 0 || kp), "NULL keypoints");
    const std::vector<int>& k = detector_keys(model, true);
    OPK_CHECK_ARG(people == 0 || parts == pose_model(model).parts, "parts != the model's");
    for (int i = 0; i < people; ++i) {
        const float* p = kp + (size_t)i * parts * 3;
        out[2 * i] = hand_from_pose(p, k[kLWrist], k[kLElbow], k[kLShoulder]);
        out[2 * i + 1] = hand_from_pose(p, k[kRWrist], k[kRElbow], k[kRShoulder]);
    }
}

KeypointExtractor::KeypointExtractor(Context* ctx, NetHip* net, int kind, int net_w, int net_h)
    : ctx_(ctx), net_(net), kind_(kind), net_w_(net_w), net_h_(net_h)
{
    OPK_CHECK_ARG(ctx && net, "NULL context or net");
    OPK_CHECK_ARG(kind == kFace || kind == kHand, "kind: face (0) or hand (1)");
    // --face_net_resolution / --hand_net_resolution must be multiples of 16 (flagsToOpenPose)
    OPK_CHECK_ARG(net_w > 0 && net_h > 0 && net_w % 16 == 0 && net_h % 16 == 0,
                  "net resolution must be positive multiples of 16");
}

int KeypointExtractor::parts() const { return net_->out_channels() - 1; }

void KeypointExtractor::set_scales(int number, float range)
{
    OPK_CHECK_ARG(kind_ == kHand || number == 1, "multi-scale detection is a hand option");
    OPK_CHECK_ARG(number >= 1, "scale number must be >= 1");
    OPK_CHECK_ARG(std::isfinite(range), "scale range must be finite");
    scales_ = number;
    range_ = range;
}

void KeypointExtractor::set_max_batch(int b)
{
    OPK_CHECK_ARG(b >= 1 && b <= 256, "batch in [1, 256]");
    max_batch_ = b;
}

void KeypointExtractor::set_heatmaps(int scale_mode)
{
    OPK_CHECK_ARG(scale_mode >= -1 && scale_mode <= 8, "unknown ScaleMode");
    heat_mode_ = scale_mode;
}

const float* KeypointExtractor::heatmaps(int shape[5]) const
{
    OPK_CHECK_ARG(heat_mode_ >= 0, "heat maps not enabled (set_heatmaps)");
    for (int i = 0; i < 5; ++i) shape[i] = heat_shape_[i];
    return static_cast<const float*>(heat_out_.ptr);
}

void KeypointExtractor::extract(const uint8_t* frames, int nframes, int w, int h, size_t step,
                                const Rect* rects, const int* frame_of, int people,
                                float* keypoints)
{
    OPK_CHECK_ARG(people >= 0, "negative people");
    OPK_CHECK_ARG(nframes > 0 && w > 0 && h > 0, "Empty cvInputData.");
    OPK_CHECK_ARG(frames, "NULL frames");
    if (!step) step = (size_t)w * 3;
    OPK_CHECK_ARG(step >= (size_t)w * 3, "row step shorter than the row");
    const int hands = kind_ == kHand ? 2 : 1;
    const int P = parts();
    OPK_CHECK_ARG(P > 0, "net has no part channels");
    std::memset(keypoints, 0, sizeof(float) * (size_t)hands * people * P * 3);
    crop_m_.clear();
    for (int i = 0; i < 5; ++i) heat_shape_[i] = 0;
    if (people == 0) return;
    OPK_CHECK_ARG(rects, "NULL rectangles");

    // 1. crops: validity and inverse maps (faceExtractorCaffe.cpp:206-232,
    //    handExtractorCaffe.cpp:44-62, 345-421); order: hand, person, scale
    const int side = std::min(net_w_, net_h_);   // netInputSide
    struct Crop { int frame, hand, person, scale; };
    std::vector<Crop> crops;
    for (int hd = 0; hd < hands; ++hd)
        for (int p = 0; p < people; ++p) {
            const Rect& r = rects[(size_t)p * hands + hd];
            const int f = frame_of ? frame_of[p] : 0;
            OPK_CHECK_ARG(f >= 0 && f < nframes, "frame index out of range");
            if (r.width != r.height)
                throw Error(1 /* OPK_ERR_ARG */, std::string(kind_ == kFace ? "Face" : "Hand") +
                                             " rectangle for " + (kind_ == kFace ? "face" : "hand") +
                                             " keypoint estimation must be squared, i.e., width = height");
            const float mn = std::min(r.width, r.height);
            if (kind_ == kFace) {
                if (!(mn > 40)) continue;
                const double s = std::max(r.width, r.height) / (double)side;
                const double M[6] = {s, 0., (double)r.x, 0., s, (double)r.y};
                crop_m_.insert(crop_m_.end(), M, M + 6);
                crops.push_back(Crop{f, 0, p, 0});
            } else {
                if (!(mn > 1 && r.width * r.height > 10)) continue;
                const bool mirror = hd == 0;
                const float init = 1.f - range_ / 2.f;
                for (int i = 0; i < scales_; ++i) {
                    Rect rs = r;
                    if (scales_ > 1) {
                        const float sc = init + range_ * i / (scales_ - 1.f);
                        rs = recenter(r, (float)((int)(r.width * sc + 0.5f) / 2 * 2),
                                      (float)((int)(r.height * sc + 0.5f) / 2 * 2));
                    }
                    const float s = rs.width / (float)side;
                    const double M[6] = {mirror ? -(double)s : (double)s, 0.,
                                         mirror ? (double)(rs.x + rs.width) : (double)rs.x, 0.,
                                         (double)s, (double)rs.y};
                    crop_m_.insert(crop_m_.end(), M, M + 6);
                    crops.push_back(Crop{f, hd, p, i});
                }
            }
        }
    const int n = (int)crops.size();
    if (n == 0) return;
    ctx_->bind();
    hipStream_t s = ctx_->stream;

    // 2. every crop warped in one launch: per-crop separable tap tables + source frame index
    const int tw = net_w_ + net_h_;   // {tap, fraction} entries per crop
    std::vector<int> host((size_t)n * tw * 2 + n);
    for (int i = 0; i < n; ++i) {
        int* t = host.data() + (size_t)i * tw * 2;
        crop_axis_tables(crop_matrix(i), net_w_, net_h_, t, t + 2 * net_w_);
        host[(size_t)n * tw * 2 + i] = crops[i].frame;
    }
    int* tabs = static_cast<int*>(tabs_.get(host.size() * sizeof(int)));
    OPK_HIP(hipMemcpyAsync(tabs, host.data(), host.size() * sizeof(int), hipMemcpyHostToDevice, s));
    const size_t crop_elems = (size_t)3 * net_h_ * net_w_;
    float* in = static_cast<float*>(inputs_.get((size_t)n * crop_elems * sizeof(float)));
    launch_cvmat_to_input(in, frames, n, h, w, step, net_h_, net_w_, tabs, tabs + 2 * net_w_,
                          ctx_->warp_weight_table(false), 2, 1, s, tabs + (size_t)n * tw * 2,
                          tw);

    // 3. net on batches of crops (power-of-two sizes, so at most log2(max_batch) + 1 plans),
    //    each followed by its resize x8 + per-part maximum (evaluated lazily, heat_dev.h) and, on
    //    request, its per-person heat maps (the last scale of each rectangle)
    float* peaks = static_cast<float*>(peaks_.get((size_t)n * P * 3 * sizeof(float)));
    float* heat_out = nullptr;
    int* slots = nullptr;
    if (heat_mode_ >= 0) {
        std::vector<int> hs(n);
        for (int i = 0; i < n; ++i)
            hs[i] = crops[i].scale == scales_ - 1 ? crops[i].hand * people + crops[i].person : -1;
        slots = static_cast<int*>(heat_slots_.get((size_t)n * sizeof(int)));
        OPK_HIP(hipMemcpyAsync(slots, hs.data(), hs.size() * sizeof(int), hipMemcpyHostToDevice, s));
    }
    for (int done = 0; done < n;) {
        int b = 1;
        while (b * 2 <= std::min(max_batch_, n - done)) b *= 2;
        net_->forward(in + (size_t)done * crop_elems, b, net_h_, net_w_);
        const int oh = net_->out_h(), ow = net_->out_w();
        HeatMap heat{};
        heat.channels = net_->out_channels();
        heat.h = oh * 8;   // ResizeAndMergeCaffe::Reshape, factor 8, scale 1 (:80-81)
        heat.w = ow * 8;
        heat.nsrc = 1;
        heat.inv_n = 1.f;
        const auto& t = ctx_->tables(oh, ow, heat.h, heat.w);
        heat.src[0] = ResizeSource{net_->output(), oh, ow, t.yofs, t.ycoef, t.xofs, t.xcoef};
        launch_heat_argmax(peaks + (size_t)done * P * 3, heat, b, P, s);
        if (heat_mode_ >= 0) {
            if (!heat_out) {
                const int sh[5] = {hands, people, P, heat.h, heat.w};
                std::copy(sh, sh + 5, heat_shape_);
                const size_t bytes = (size_t)hands * people * P * heat.h * heat.w * sizeof(float);
                heat_out = static_cast<float*>(heat_out_.get(bytes));
                OPK_HIP(hipMemsetAsync(heat_out, 0, bytes, s));
            }
            launch_crop_heatmaps(heat_out, heat, slots + done, b, P, heat_mode_, s);
        }
        done += b;
    }
    float* hp = static_cast<float*>(hpeaks_.get((size_t)n * P * 3 * sizeof(float)));
    OPK_HIP(hipMemcpyAsync(hp, peaks, (size_t)n * P * 3 * sizeof(float), hipMemcpyDeviceToHost, s));
    OPK_HIP(hipStreamSynchronize(s));

    // 4. keypoints = M (x, y) in double, stored as float (faceExtractorCaffe.cpp:251-266,
    //    connectKeypoints handExtractorCaffe.cpp:75-99); multi-scale keeps the scale with the
    //    highest average score, the first on ties (:422-425)
    std::vector<float> est((size_t)P * 3);
    for (int i = 0; i < n; ++i) {
        const double* M = crop_matrix(i);
        const float* pk = hp + (size_t)i * P * 3;
        for (int q = 0; q < P; ++q) {
            const double x = pk[q * 3], y = pk[q * 3 + 1];
            est[q * 3] = (float)(M[0] * x + M[1] * y + M[2]);
            est[q * 3 + 1] = (float)(M[3] * x + M[4] * y + M[5]);
            est[q * 3 + 2] = pk[q * 3 + 2];
        }
        float* dst = keypoints + ((size_t)crops[i].hand * people + crops[i].person) * P * 3;
        bool take = crops[i].scale == 0;
        if (!take) {   // getAverageScore (keypoint.cpp:352-372)
            float a = 0.f, b = 0.f;
            for (int q = 0; q < P; ++q) {
                a += est[q * 3 + 2];
                b += dst[q * 3 + 2];
            }
            take = a / P > b / P;
        }
        if (take) std::memcpy(dst, est.data(), sizeof(float) * P * 3);
    }
}

}  // namespace opk
