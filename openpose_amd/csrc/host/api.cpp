// api.cpp -- C-ABI (include/opk.h): context, memory, resizeAndMerge, NMS, PAF scores, connector.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>

#include "../../../include/opk.h"
#include "connector.h"
#include "context.h"
#include "json.h"
#include "maps.h"
#include "output.h"

namespace opk {

static thread_local std::string g_error;
void set_error(const std::string& msg) { g_error = msg; }

template <class F>
static int guarded(F&& f)
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

using opk::Context;
using opk::guarded;

struct opk_ctx : Context {};

extern "C" {

const char* opk_last_error(void) { return opk::g_error.c_str(); }
int opk_version(void) { return 1; }

static int ctx_create(int device, void* stream, bool own, opk_ctx** out)
{
    return guarded([&] {
        OPK_CHECK_ARG(out != nullptr, "out is NULL");
        if (device == -1 && !own) {   // host-only context
            auto* c = new opk_ctx();
            c->device = -1;
            *out = c;
            return;
        }
        int n = 0;
        OPK_HIP(hipGetDeviceCount(&n));
        OPK_CHECK_ARG(device >= 0 && device < n, "device " + std::to_string(device) + " of " +
                                                     std::to_string(n));
        auto* c = new opk_ctx();
        c->device = device;
        c->bind();
        if (own) {
            OPK_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
            c->owns_stream = true;
        } else {
            c->stream = static_cast<hipStream_t>(stream);
        }
        *out = c;
    });
}

int opk_ctx_create(int device, void* stream, opk_ctx** out)
{
    return ctx_create(device, stream, false, out);
}

int opk_ctx_create_private_stream(int device, opk_ctx** out)
{
    return ctx_create(device, nullptr, true, out);
}

int opk_ctx_destroy(opk_ctx* ctx)
{
    return guarded([&] {
        if (!ctx) return;
        if (ctx->device >= 0) ctx->bind();
        if (ctx->owns_stream) (void)hipStreamDestroy(ctx->stream);
        delete ctx;
    });
}

int opk_ctx_stream(opk_ctx* ctx, void** s)
{
    return guarded([&] {
        OPK_CHECK_ARG(ctx && s, "NULL argument");
        *s = ctx->stream;
    });
}

int opk_sync(opk_ctx* ctx)
{
    return guarded([&] {
        OPK_CHECK_ARG(ctx, "NULL ctx");
        ctx->bind();
        OPK_HIP(hipStreamSynchronize(ctx->stream));
        for (hipStream_t s : ctx->side_streams) OPK_HIP(hipStreamSynchronize(s));
    });
}

int opk_malloc(opk_ctx* ctx, void** p, size_t bytes)
{
    return guarded([&] {
        OPK_CHECK_ARG(ctx && p, "NULL argument");
        ctx->bind();
        OPK_HIP(hipMalloc(p, bytes ? bytes : 1));
    });
}

int opk_free(opk_ctx* ctx, void* p)
{
    return guarded([&] {
        OPK_CHECK_ARG(ctx, "NULL ctx");
        ctx->bind();
        if (p) OPK_HIP(hipFree(p));
    });
}

int opk_convert(opk_ctx* ctx, void* dst, int dst_type, const void* src, int src_type, size_t count)
{
    return guarded([&] {
        OPK_CHECK_ARG(ctx && (count == 0 || (dst && src)), "NULL argument");
        OPK_CHECK_ARG((dst_type == OPK_F32 || dst_type == OPK_F64) &&
                          (src_type == OPK_F32 || src_type == OPK_F64),
                      "unknown element type");
        ctx->bind();
        if (dst_type == src_type) {
            OPK_HIP(hipMemcpyAsync(dst, src, count * (dst_type == OPK_F64 ? 8 : 4),
                                   hipMemcpyDeviceToDevice, ctx->stream));
        } else if (dst_type == OPK_F32) {
            opk::launch_f64_to_f32(static_cast<float*>(dst), static_cast<const double*>(src), count,
                                   ctx->stream);
        } else {
            opk::launch_f32_to_f64(static_cast<double*>(dst), static_cast<const float*>(src), count,
                                   ctx->stream);
        }
    });
}

int opk_memset(opk_ctx* ctx, void* p, int v, size_t bytes)
{
    return guarded([&] {
        OPK_CHECK_ARG(ctx && p, "NULL argument");
        ctx->bind();
        OPK_HIP(hipMemsetAsync(p, v, bytes, ctx->stream));
    });
}

int opk_memcpy_h2d(opk_ctx* ctx, void* dst, const void* src, size_t bytes)
{
    return guarded([&] {
        OPK_CHECK_ARG(ctx && dst && src, "NULL argument");
        ctx->bind();
        OPK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
        OPK_HIP(hipStreamSynchronize(ctx->stream));   // caller may free src on return
    });
}

int opk_memcpy_d2h(opk_ctx* ctx, void* dst, const void* src, size_t bytes)
{
    return guarded([&] {
        OPK_CHECK_ARG(ctx && dst && src, "NULL argument");
        ctx->bind();
        OPK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
        OPK_HIP(hipStreamSynchronize(ctx->stream));
    });
}

// resizeAndMergeCpu sanity checks (resizeAndMergeBase.cpp:21-41) + the batched HIP kernel
int opk_resize_and_merge(opk_ctx* ctx, float* target, const float* const* sources, int nsrc,
                         const int ts[4], const int* ss, const float* scale_ratios)
{
    (void)scale_ratios;   // unused by the CPU-path semantics (resizeAndMergeBase.cpp:18)
    return guarded([&] {
        OPK_CHECK_ARG(ctx && target && sources && ts && ss, "NULL argument");
        OPK_CHECK_ARG(nsrc >= 1, "sourceSizes cannot be empty.");
        OPK_CHECK_ARG(nsrc <= opk::kMaxResizeSources, "at most 8 scales");
        ctx->bind();
        opk::ResizeSource rs[opk::kMaxResizeSources];
        for (int i = 0; i < nsrc; ++i) {
            const int* s = ss + 4 * i;
            OPK_CHECK_ARG(s[0] == ts[0] && s[1] == ts[1],
                          "source " + std::to_string(i) + " frames/channels differ from target");
            OPK_CHECK_ARG(sources[i] != nullptr && s[2] > 0 && s[3] > 0, "empty source");
            const auto& t = ctx->tables(s[2], s[3], ts[2], ts[3]);
            rs[i] = opk::ResizeSource{sources[i], s[2], s[3], t.yofs, t.ycoef, t.xofs, t.xcoef};
        }
        opk::launch_resize_merge(target, rs, nsrc, ts[0] * ts[1], ts[2], ts[3], ctx->stream);
    });
}

int opk_resize_and_merge_semantics(opk_ctx* ctx, float* target, const float* const* sources,
                                   int nsrc, const int ts[4], const int* ss,
                                   const float* scale_ratios, int semantics)
{
    if (semantics == OPK_MAPS_CPU)
        return opk_resize_and_merge(ctx, target, sources, nsrc, ts, ss, scale_ratios);
    return guarded([&] {
        OPK_CHECK_ARG(semantics == OPK_MAPS_CUDA, "unknown heat-map semantics");
        OPK_CHECK_ARG(ctx && target && sources && ts && ss, "NULL argument");
        OPK_CHECK_ARG(nsrc >= 1, "sourceSizes cannot be empty.");
        int sh[opk::kMaxResizeSources], sw[opk::kMaxResizeSources];
        for (int i = 0; i < nsrc && i < opk::kMaxResizeSources; ++i) {
            const int* s = ss + 4 * i;
            OPK_CHECK_ARG(s[0] == ts[0] && s[1] == ts[1],
                          "source " + std::to_string(i) + " frames/channels differ from target");
            sh[i] = s[2];
            sw[i] = s[3];
        }
        const opk::HeatMap m = opk::cuda_heat_map(sources, sh, sw, nsrc, ts[1], ts[2], ts[3],
                                                  scale_ratios);
        ctx->bind();
        opk::launch_resize_merge_cuda(target, m, ts[0] * ts[1], ctx->stream);
    });
}

// nmsCpu sanity checks (nmsBase.cpp:116-122) + the batched HIP kernel
int opk_nms(opk_ctx* ctx, float* target, int* kernel_scratch, const float* source, float th,
            const int ts[4], const int ss[4], float offx, float offy)
{
    return opk_nms_semantics(ctx, target, kernel_scratch, source, th, ts, ss, offx, offy,
                             OPK_MAPS_CPU);
}

int opk_nms_semantics(opk_ctx* ctx, float* target, int* kernel_scratch, const float* source,
                      float th, const int ts[4], const int ss[4], float offx, float offy,
                      int semantics)
{
    (void)kernel_scratch;
    return guarded([&] {
        OPK_CHECK_ARG(ctx && target && source && ts && ss, "NULL argument");
        OPK_CHECK_ARG(!(th < 0 || th > 1.0), "threshold value invalid.");
        OPK_CHECK_ARG(ts[0] == ss[0], "frame count of target and source differ");
        OPK_CHECK_ARG(ts[3] == 3, "target peak vector must be 3 (x, y, score)");
        OPK_CHECK_ARG(ts[1] <= ss[1], "more target parts than source channels");
        ctx->bind();
        OPK_CHECK_ARG(semantics == OPK_MAPS_CPU || semantics == OPK_MAPS_CUDA,
                      "unknown heat-map semantics");
        opk::launch_nms(target, ctx->nms_candidates(ts[0], ts[1]),
                        opk::heat_materialised(source, ss[1], ss[2], ss[3]), ts[0], ts[1], ts[2],
                        th, offx, offy, ctx->stream, semantics == OPK_MAPS_CUDA);
    });
}

int opk_paf_scores(opk_ctx* ctx, float* pair_scores, const float* heat, const float* peaks,
                   int frames, int pose_model, int heat_channels, int heat_h, int heat_w,
                   int max_peaks, float inter_th, float inter_min_above, float default_nms_th)
{
    return guarded([&] {
        OPK_CHECK_ARG(ctx && pair_scores && heat && peaks, "NULL argument");
        const auto& m = opk::pose_model(pose_model);
        OPK_CHECK_ARG(heat_channels >= m.heat_channels(), "too few heat-map channels");
        ctx->bind();
        const auto& t = ctx->pose_table(pose_model);
        const double near = std::sqrt((double)(heat_w * heat_h)) / 150;
        const float reject = float(default_nms_th + 1e-6);
        opk::launch_paf_scores(pair_scores,
                               opk::heat_materialised(heat, heat_channels, heat_h, heat_w), peaks,
                               frames, max_peaks, t, inter_th, inter_min_above, reject, near,
                               ctx->stream);
    });
}

int opk_pose_model_info(int pose_model, int* parts, int* bkg, int* npairs, int* heat_channels,
                        int* pairs, int* map_idx)
{
    return guarded([&] {
        const auto& m = opk::pose_model(pose_model);
        if (parts) *parts = m.parts;
        if (bkg) *bkg = m.bkg ? 1 : 0;
        if (npairs) *npairs = m.npairs();
        if (heat_channels) *heat_channels = m.heat_channels();
        if (pairs) std::copy(m.pairs.begin(), m.pairs.end(), pairs);
        if (map_idx) std::copy(m.map_idx.begin(), m.map_idx.end(), map_idx);
    });
}

int opk_pose_default_thresholds(int pose_model, int maxpos, float* nms_threshold,
                                float* inter_threshold)
{
    return guarded([&] {
        const auto& m = opk::pose_model(pose_model);
        if (nms_threshold) *nms_threshold = maxpos ? m.nms_th_maxpos : m.nms_th;
        if (inter_threshold) *inter_threshold = maxpos ? m.inter_th_maxpos : m.inter_th;
    });
}

int opk_assemble_people(float* kp_out, float* ks_out, int max_people, int* num_people,
                        const float* pair_scores, const float* peaks, int pose_model,
                        int max_peaks, int min_cnt, float min_score, float scale, int maxpos)
{
    return opk_assemble_people_semantics(kp_out, ks_out, max_people, num_people, pair_scores, peaks,
                                         pose_model, max_peaks, min_cnt, min_score, scale, maxpos,
                                         OPK_CONNECT_CPU);
}

int opk_assemble_people_semantics(float* kp_out, float* ks_out, int max_people, int* num_people,
                                  const float* pair_scores, const float* peaks, int pose_model,
                                  int max_peaks, int min_cnt, float min_score, float scale,
                                  int maxpos, int semantics)
{
    return guarded([&] {
        OPK_CHECK_ARG(semantics == OPK_CONNECT_CPU || semantics == OPK_CONNECT_GPU,
                      "unknown connector semantics");
        OPK_CHECK_ARG(pair_scores && peaks && num_people, "NULL argument");
        const auto& m = opk::pose_model(pose_model);
        opk::PairScores ps;
        ps.data = pair_scores;
        ps.max_peaks = max_peaks;
        opk::ConnectParams p{min_cnt, min_score, scale, maxpos != 0, semantics};
        std::vector<float> kp, ks;
        const int n = opk::assemble_people(m, peaks, max_peaks, ps, p, kp, ks);
        *num_people = n;
        const int w = std::min(n, max_people);
        if (w > 0 && kp_out) std::memcpy(kp_out, kp.data(), sizeof(float) * (size_t)w * m.parts * 3);
        if (w > 0 && ks_out) std::memcpy(ks_out, ks.data(), sizeof(float) * w);
    });
}

int opk_connect_body_parts(opk_ctx* ctx, float* kp_out, float* ks_out, int max_people,
                           int* num_people, const float* heat, const float* peaks_dev,
                           int pose_model, int heat_channels, int heat_h, int heat_w,
                           int max_peaks, float inter_min_above, float inter_th, int min_cnt,
                           float min_score, float nms_th, float scale, int maxpos)
{
    return opk_connect_body_parts_semantics(ctx, kp_out, ks_out, max_people, num_people, heat,
                                            peaks_dev, pose_model, heat_channels, heat_h, heat_w,
                                            max_peaks, inter_min_above, inter_th, min_cnt,
                                            min_score, nms_th, scale, maxpos, OPK_CONNECT_CPU);
}

int opk_connect_body_parts_semantics(opk_ctx* ctx, float* kp_out, float* ks_out, int max_people,
                                     int* num_people, const float* heat, const float* peaks_dev,
                                     int pose_model, int heat_channels, int heat_h, int heat_w,
                                     int max_peaks, float inter_min_above, float inter_th,
                                     int min_cnt, float min_score, float nms_th, float scale,
                                     int maxpos, int semantics)
{
    return guarded([&] {
        OPK_CHECK_ARG(semantics == OPK_CONNECT_CPU || semantics == OPK_CONNECT_GPU,
                      "unknown connector semantics");
        OPK_CHECK_ARG(ctx && heat && peaks_dev && num_people, "NULL argument");
        const auto& m = opk::pose_model(pose_model);
        OPK_CHECK_ARG(heat_channels >= m.heat_channels(), "too few heat-map channels");
        ctx->bind();
        const size_t score_floats = (size_t)m.npairs() * max_peaks * max_peaks;
        const size_t peak_floats = (size_t)m.parts * (max_peaks + 1) * 3;
        auto* dscores = static_cast<float*>(ctx->scratch_scores.get(score_floats * sizeof(float)));
        const auto& t = ctx->pose_table(pose_model);
        const double near = std::sqrt((double)(heat_w * heat_h)) / 150;
        opk::launch_paf_scores(dscores, opk::heat_materialised(heat, heat_channels, heat_h, heat_w),
                               peaks_dev, 1, max_peaks, t, inter_th, inter_min_above,
                               float(nms_th + 1e-6), near, ctx->stream);
        auto* hpk = static_cast<float*>(ctx->host_peaks.get(peak_floats * sizeof(float)));
        auto* hsc = static_cast<float*>(ctx->host_scores.get(score_floats * sizeof(float)));
        OPK_HIP(hipMemcpyAsync(hpk, peaks_dev, peak_floats * sizeof(float), hipMemcpyDeviceToHost,
                               ctx->stream));
        OPK_HIP(hipMemcpyAsync(hsc, dscores, score_floats * sizeof(float), hipMemcpyDeviceToHost,
                               ctx->stream));
        OPK_HIP(hipStreamSynchronize(ctx->stream));
        opk::PairScores ps;
        ps.data = hsc;
        ps.max_peaks = max_peaks;
        opk::ConnectParams p{min_cnt, min_score, scale, maxpos != 0, semantics};
        std::vector<float> kp, ks;
        const int n = opk::assemble_people(m, hpk, max_peaks, ps, p, kp, ks);
        *num_people = n;
        const int w = std::min(n, max_people);
        if (w > 0 && kp_out) std::memcpy(kp_out, kp.data(), sizeof(float) * (size_t)w * m.parts * 3);
        if (w > 0 && ks_out) std::memcpy(ks_out, ks.data(), sizeof(float) * w);
    });
}

int opk_scale_keypoints(float* keypoints_host, int people, int parts, int scale_mode,
                        double scale_input_to_output, double scale_net_to_output, int producer_w,
                        int producer_h)
{
    return guarded([&] {
        opk::scale_keypoints(keypoints_host, people, parts, scale_mode, scale_input_to_output,
                             scale_net_to_output, producer_w, producer_h);
    });
}

int opk_keep_top_n_people(const float* keypoints_host, int people, int parts,
                          const float* scores_host, int max_people, float* out_keypoints_host,
                          int* out_index_host, int* out_people)
{
    return guarded([&] {
        const int n = opk::keep_top_n_people(keypoints_host, people, parts, scores_host, max_people,
                                             out_keypoints_host, out_index_host);
        if (out_people) *out_people = n;
    });
}

int opk_people_json(const opk_json_keypoints* arrays, int n_arrays, const float* candidates_host,
                    const int* candidate_counts_host, int n_parts, int human_readable,
                    char* out_host, size_t capacity, size_t* len)
{
    return guarded([&] {
        OPK_CHECK_ARG(len != nullptr, "opk_people_json: NULL len");
        const std::string t = opk::people_json(arrays, n_arrays, candidates_host,
                                               candidate_counts_host, n_parts, human_readable != 0);
        *len = t.size();
        if (out_host) {
            OPK_CHECK_ARG(capacity >= t.size() + 1, "opk_people_json: buffer too small");
            std::memcpy(out_host, t.c_str(), t.size() + 1);
        }
    });
}

int opk_save_people_json(const char* path, const opk_json_keypoints* arrays, int n_arrays,
                         const float* candidates_host, const int* candidate_counts_host,
                         int n_parts, int human_readable)
{
    return guarded([&] {
        OPK_CHECK_ARG(path != nullptr, "opk_save_people_json: NULL path");
        opk::save_people_json(path, opk::people_json(arrays, n_arrays, candidates_host,
                                                     candidate_counts_host, n_parts,
                                                     human_readable != 0));
    });
}

}  // extern "C"

extern "C" int opk_probe_peaks(opk_ctx* ctx, double* mfma_random_tflops, double* mfma_zero_tflops,
                               double* hbm_read_gbs)
{
    return guarded([&] {
        OPK_CHECK_ARG(ctx != nullptr, "NULL argument");
        ctx->bind();
        int cus = 0;
        OPK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
        const int blocks = 4 * cus, hbm_blocks = 16 * cus, iters = 20000;
        opk::DevBuf ops, out, big;
        void* dops = ops.get(6 * 64 * 16);   // 6 x 64 half8 operands
        // one float per lane of the larger of the two grids
        float* dout = static_cast<float*>(out.get((size_t)std::max(blocks, hbm_blocks) * 256 * 4));
        hipEvent_t e0, e1;
        OPK_HIP(hipEventCreate(&e0));
        OPK_HIP(hipEventCreate(&e1));
        auto timed = [&](auto&& launch, int reps) {
            launch();
            OPK_HIP(hipEventRecord(e0, ctx->stream));
            for (int r = 0; r < reps; ++r) launch();
            OPK_HIP(hipEventRecord(e1, ctx->stream));
            OPK_HIP(hipEventSynchronize(e1));
            float ms = 0.f;
            OPK_HIP(hipEventElapsedTime(&ms, e0, e1));
            return (double)ms / reps;
        };
        std::vector<uint16_t> h(6 * 64 * 8);
        uint32_t lcg = 12345u;
        for (int random = 1; random >= 0; --random) {
            for (auto& v : h) {   // fp16 bit patterns of uniform values in (-1, 1)
                lcg = lcg * 1664525u + 1013904223u;
                const uint32_t mant = (lcg >> 8) & 0x3ffu, ex = 11u + ((lcg >> 18) % 4u);
                v = random ? (uint16_t)(((lcg >> 31) << 15) | (ex << 10) | mant) : (uint16_t)0;
            }
            OPK_HIP(hipMemcpyAsync(dops, h.data(), h.size() * 2, hipMemcpyHostToDevice, ctx->stream));
            const double ms = timed([&] { opk::launch_mfma_peak(dops, dout, blocks, iters, ctx->stream); }, 3);
            const double tf = (double)blocks * 4 * iters * 8 * 16384.0 / (ms * 1e-3) / 1e12;
            if (random && mfma_random_tflops) *mfma_random_tflops = tf;
            if (!random && mfma_zero_tflops) *mfma_zero_tflops = tf;
        }
        const size_t bytes = (size_t)2 << 30;
        void* dbig = big.get(bytes);
        OPK_HIP(hipMemsetAsync(dbig, 0, bytes, ctx->stream));
        const double ms = timed([&] { opk::launch_hbm_read(dbig, bytes, dout, hbm_blocks, ctx->stream); }, 5);
        if (hbm_read_gbs) *hbm_read_gbs = bytes / (ms * 1e-3) / 1e9;
        OPK_HIP(hipEventDestroy(e0));
        OPK_HIP(hipEventDestroy(e1));
    });
}
