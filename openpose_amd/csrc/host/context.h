// context.h -- per-GPU-thread context behind opk_ctx (internal).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <tuple>
#include <vector>

#include "../common.h"
#include "../kernels/kernels.h"
#include "pose_model.h"

namespace opk {

// OpenCV-style cubic tables for one (source size -> target size) axis (host/resize_tables.cpp)
void cubic_tables(int s, int d, int* ofs, float* coef);

struct Context {
    int device = 0;
    hipStream_t stream = nullptr;
    bool owns_stream = false;

    // device copies of cubic tables, keyed by (sh, sw, dh, dw)
    struct Tables { DevBuf buf; const int* yofs; const float* ycoef; const int* xofs; const float* xcoef; };
    std::map<std::tuple<int, int, int, int>, std::unique_ptr<Tables>> resize_tables;
    const Tables& tables(int sh, int sw, int dh, int dw);

    // device pose tables for the PAF kernel
    struct PoseDev { DevBuf buf; PafPairTable t; };
    std::map<int, std::unique_ptr<PoseDev>> pose_dev;
    const PafPairTable& pose_table(int model);

    // frame -> net input (host/input.cpp): fixed-point weight tables (0 linear, 1 cubic) and the
    // per-axis tap tables of each (scale, dw, dh)
    DevBuf warp_weights[2];
    const short* warp_weight_table(bool cubic);
    struct WarpAxes { DevBuf buf; const int* x; const int* y; };
    std::map<std::tuple<uint64_t, int, int>, std::unique_ptr<WarpAxes>> warp_axes;
    const WarpAxes& warp_axis_tables(double scale, int dw, int dh);

    // renderers (host/render.cpp): device copies of the render tables (render_tables.inc) and the
    // per-person geometry scratch of launch_render_keypoints
    struct RenderDev { DevBuf buf; const unsigned* pairs; const float* scales; const float* colors;
                       int npairs, nscales, ncolors; };
    std::map<int, std::unique_ptr<RenderDev>> render_dev;
    const RenderDev& render_table(int which);
    DevBuf render_geom;

    DevBuf scratch_scores;   // dense pair scores for opk_connect_body_parts
    // NMS candidate lists (nms.hip), zeroed when (re)allocated; the kernels keep them zeroed
    DevBuf nms_scratch;
    int* nms_candidates(int frames, int parts);
    HostBuf host_peaks, host_scores;

    // streams other objects of this context run device work on besides `stream` (PoseHip's
    // post-processing stream, its multi-scale net streams): opk_sync waits for them too
    std::vector<hipStream_t> side_streams;
    void add_side_stream(hipStream_t s) { side_streams.push_back(s); }
    void remove_side_stream(hipStream_t s)
    {
        for (size_t i = 0; i < side_streams.size(); ++i)
            if (side_streams[i] == s) {
                side_streams.erase(side_streams.begin() + (long)i);
                return;
            }
    }

    // device < 0: host-only context (graph planning / host assembly; no device calls)
    void bind() const
    {
        if (device < 0) throw Error(3, "host-only context (device -1) cannot run device work");
        OPK_HIP(hipSetDevice(device));
    }
};

// Device-time measurement hook (no reference counterpart): while enabled, begin()/end() bracket a
// region of stream work with a pair of HIP events; read() waits for every recorded pair and
// returns their count and summed milliseconds.
class EventTimer {
public:
    ~EventTimer();
    bool on = false;
    void begin(hipStream_t s);
    void end(hipStream_t s);
    void read(int* count, double* total_ms);

private:
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events_, free_;
};

}  // namespace opk
