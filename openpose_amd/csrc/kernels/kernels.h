// kernels.h -- launchers of the gfx950 kernels in this directory (internal to libopk_hip.so).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace opk {

// ---- resize (resize.hip) -------------------------------------------------------------------
// One source of a resize/merge: [planes][sh][sw] fp32 and its cubic tables on device.
struct ResizeSource {
    const float* src;
    int sh, sw;
    const int* yofs;     // [dh]
    const float* ycoef;  // [dh][4]
    const int* xofs;     // [dw]
    const float* xcoef;  // [dw][4]
    // CUDA-build semantics only (HeatMap::cuda): target pixel x maps to source (x + 0.5) / sx - 0.5
    float sx, sy;
};
constexpr int kMaxResizeSources = 8;
// dst [planes][dh][dw]; planes = frames * channels; all sources share the plane count.
void launch_resize_merge(float* dst, const ResizeSource* srcs, int nsrc, int planes, int dh,
                         int dw, hipStream_t stream);

// A full-resolution heat-map stack [frames][channels][h][w], either materialised in HBM
// (heat != nullptr) or evaluated on the fly, pixel by pixel, as the resize/merge of `nsrc` net
// outputs with exactly the arithmetic of resize.hip (heat_dev.h) -- bit-identical values without
// writing the 75 MB/frame stack.  Consumers: NMS (nms.hip) and PAF scores (paf.hip).
struct HeatMap {
    const float* heat;
    int channels, h, w;
    int nsrc;
    float inv_n;
    ResizeSource src[kMaxResizeSources];
    // 1: the CUDA build's resizeAndMergeGpu arithmetic (heat_dev.h: cuda_bicubic, per-source
    // scale sx / sy, sum / N) instead of cv::resize's; the tables are then unused
    int cuda;
};
// dst [planes][M.h][M.w] = the CUDA-semantics resize/merge (M.cuda) of M's sources
void launch_resize_merge_cuda(float* dst, const HeatMap& M, int planes, hipStream_t stream);
inline HeatMap heat_materialised(const float* heat, int channels, int h, int w)
{
    HeatMap m{};
    m.heat = heat;
    m.channels = channels;
    m.h = h;
    m.w = w;
    return m;
}

// ---- NMS (nms.hip) ----------------------------------------------------------------------------
// peaks [frames][parts][maxPeaks1][3]; heat [frames][channels][h][w].  scratch: nms_scratch_ints()
// ints, zeroed once before the first call (every call leaves it zeroed again).
constexpr int kNmsCandidates = 1024;   // per plane; more peaks fall back to an ordered re-scan
size_t nms_scratch_ints(int frames, int parts);
// cuda: nmsGpu's rules (nmsBase.cu:50-90,161-240: strict interior, 8 strict neighbours, centroid
// sums contracted to fma as nvcc's default --fmad does) instead of nmsCpu's
void launch_nms(float* peaks, int* scratch, const HeatMap& heat, int frames, int parts,
                int max_peaks1, float threshold, float offx, float offy, hipStream_t stream,
                bool cuda = false);

// ---- PAF scores (paf.hip) --------------------------------------------------------------------
struct PafPairTable {
    int npairs;
    int nparts;
    const int* pairs;    // device [2*npairs] (part A, part B)
    const int* mapx;     // device [npairs] heat channel of the x PAF
    const int* mapy;     // device [npairs]
};
// dense: scores [frames][npairs][maxPeaks][maxPeaks]
void launch_paf_scores(float* scores, const HeatMap& heat, const float* peaks, int frames,
                       int max_peaks, const PafPairTable& t, float inter_th,
                       float inter_min_above, float reject_score, double near_dist,
                       hipStream_t stream);
// compact: per frame a record of `rec_floats` floats: [0] = number of scores (or -1 when it did
// not fit), then the nA*nB scores of pair 0, pair 1, ... (row-major i, j).
void launch_paf_scores_compact(float* records, int rec_floats, const HeatMap& heat,
                               const float* peaks, int frames, int max_peaks,
                               const PafPairTable& t, float inter_th, float inter_min_above,
                               float reject_score, double near_dist, hipStream_t stream);

// ---- frame -> net input (input.hip) -------------------------------------------------------------
// src: n BGR uint8 frames [sh][src_step bytes], frame stride src_step*sh; dst [n][3][dh][dw] fp32.
// xtab/ytab: per destination column/row {first source tap, 5-bit fraction index}; wtab: the
// fixed-point 2-D weight table [32*32][ksize*ksize] (host/input.cpp builds all three)
// frame_of (device, may be NULL): source frame of each output image; tab_stride: distance between
// the table pairs of consecutive images, in {tap, fraction} entries (0: one shared pair)
void launch_cvmat_to_input(float* dst, const uint8_t* src, int n, int sh, int sw, size_t src_step,
                           int dh, int dw, const int* xtab, const int* ytab, const short* wtab,
                           int ksize, int normalize, hipStream_t stream,
                           const int* frame_of = nullptr, int tab_stride = 0);

// ---- crops of face / hand keypoint extraction (crop.hip) -----------------------------------------
// peaks [crops][parts][3] = (x, y, value) of the maximum of each of the first `parts` channels of
// `heat` (frames = crops), the first in raster order among equal values (cv::minMaxLoc)
void launch_heat_argmax(float* peaks, const HeatMap& heat, int crops, int parts, hipStream_t stream);
// dst[slot[c]][parts][heat.h][heat.w] = ScaleMode-mapped first `parts` channels of crop c (slot -1:
// none), as FaceExtractorCaffe / HandExtractorCaffe store their per-person heat maps
void launch_crop_heatmaps(float* dst, const HeatMap& heat, const int* slot_dev, int crops, int parts,
                          int scale_mode, hipStream_t stream);

// ---- renderers (render.hip) -----------------------------------------------------------------
constexpr int kRenderMaxPeople = 1024;   // people (faces, hands) per frame one launch draws
// One keypoint render (renderKeypointsOld / renderKeypoints, render.hu): frame float BGR [h][w][3]
// in place; kp [people][parts][3]; pairs / colors (RGB) / scales on the device; geom scratch of
// render_geom_floats(people, parts, npairs) floats; eye1 / eye2 the googly-eye parts or -1.
struct RenderKeypointsArgs {
    float* frame;
    int w, h;
    const float* kp;
    int people, parts;
    const unsigned* pairs;
    int npairs;
    const float* colors;
    int ncolors;
    const float* scales;
    int nscales;
    float radius, line_width, threshold, alpha;
    int blend, eye1, eye2;
    float* geom;
};
size_t render_geom_floats(int people, int parts, int npairs);
void launch_render_keypoints(const RenderKeypointsArgs& a, hipStream_t stream);
// heat-map renders: frame [h][w][3] BGR; heat [channels][hh][hw]; target pixel x samples the heat
// map at (x + 0.5) / scale - 0.5
struct RenderHeatArgs {
    float* frame;
    int w, h;
    const float* heat;
    int hw, hh;
    float scale, alpha;
};
void launch_render_heat_map(const RenderHeatArgs& a, int part, bool abs_value, hipStream_t stream);
void launch_render_heat_maps(const RenderHeatArgs& a, int parts, const float* colors, int ncolors,
                             hipStream_t stream);
void launch_render_pafs(const RenderHeatArgs& a, int first, int count, hipStream_t stream);

// ---- measured ceilings (probe.hip) ------------------------------------------------------------
// operands: 6 x 64 half8 values; out: blocks * 256 floats; 4 waves per workgroup
void launch_mfma_peak(const void* operands, float* out, int blocks, int iters, hipStream_t stream);
void launch_hbm_read(const void* buf, size_t bytes, float* out, int blocks, hipStream_t stream);

// ---- elementwise helpers (misc.hip) -----------------------------------------------------------
void launch_add_inplace(float* dst, const float* src, size_t n, hipStream_t stream);
void launch_delay(int microseconds, hipStream_t stream);   // dev hook: hold a stream
void launch_f64_to_f32(float* dst, const double* src, size_t n, hipStream_t stream);
void launch_f32_to_f64(double* dst, const float* src, size_t n, hipStream_t stream);
// getHeatMapsCopy: dst [frames][nsel][hw] from heat [frames][channels][hw]; sel_dev = nsel source
// channels then nsel kinds (0 part/background, 1 PAF); scale_mode = op::ScaleMode value
void launch_heat_copy(float* dst, const float* heat, const int* sel_dev, int nsel, int frames,
                      int channels, size_t hw, int scale_mode, hipStream_t stream);

}  // namespace opk
