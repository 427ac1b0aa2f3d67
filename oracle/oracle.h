/*
 * oracle.h -- CPU oracle for the OpenPose BODY_25 hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so, and only as
 * the checker / the timed CPU baseline.  The product path (libopk_hip.so) never links it.
 *
 * Every function restates the reference CPU path (CPU_ONLY build) of zengjianping/openpose.
 * Citations are to /root/reference/<file>:<line>.
 *
 * Pinning status (see DESIGN.md "Oracle"):
 *   - connector (orc_connect_body_parts)     : pinned against the reference's own
 *     bodyPartConnectorBase.cpp compiled from source into oracle/_ref (tests/test_oracle_ref.py)
 *   - NMS (orc_nms)                          : parity unpinned (nmsBase.cpp needs OpenCV headers,
 *     absent from the image -> reference unbuildable here); restatement + known-answer tests
 *   - resize (orc_resize_cubic/merge)        : parity unpinned (OpenCV cv::resize is a third-party
 *     dependency absent from the image); restatement of OpenCV's generic float INTER_CUBIC path
 *   - frame -> net input (orc_cvmat_to_input) : parity unpinned (cv::warpAffine is OpenCV);
 *     restatement of OpenCV 4.2's fixed-point 8-bit warp
 *   - CNN layers (orc_conv2d, ...)           : parity unpinned (Caffe absent); restatement of Caffe
 *     layer semantics, cross-checked against torch CPU fp32 in tests
 *
 * Float semantics: the reference CPU build uses -O3 without -march (CMakeLists.txt:103-137,
 * INSTRUCTION_SET NONE), i.e. SSE float arithmetic, no FMA contraction.  Every file here except
 * the GEMM is compiled with -ffp-contract=off to keep that operation order.
 */
#ifndef OPK_ORACLE_H
#define OPK_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- NMS: restates op::nmsCpu (src/openpose/net/nmsBase.cpp:109-170) ----------------------
 * peaks   : [channels][max_peaks1][3]  (slot 0 = {count, -, -}; max_peaks1 = targetSize[2] = 128)
 * heat    : [channels][h][w]
 * Only the first `channels` planes of `heat` are read.                                       */
void orc_nms(float* peaks, const float* heat, float threshold, int channels, int max_peaks1,
             int h, int w, float offset_x, float offset_y);

/* ---- bicubic resize: restates cv::resize(..., INTER_CUBIC) as called by
 * op::resizeAndMergeCpu (src/openpose/net/resizeAndMergeBase.cpp:45-52) --------------------- */
void orc_resize_cubic(float* dst, const float* src, int sh, int sw, int dh, int dw);
/* CUDA-build semantics (resizeAndMergeBase.cu / nmsBase.cu; resize.c, nms.c) */
int orc_resize_merge_cuda(float* dst, const float* const* srcs, int nsrc, int channels,
                          const int* hw, int dh, int dw, const float* ratios);
void orc_nms_cuda(float* peaks, const float* heat, float threshold, int channels, int max_peaks1,
                  int h, int w, float offset_x, float offset_y);
/* multi-scale: resizeAndMergeBase.cpp:55-106 (each source to the full target, sum, average) */
void orc_resize_merge(float* dst, const float* const* srcs, int nsrc, int channels,
                      const int* src_hw /* nsrc*2 */, int dh, int dw);
/* vertical-pass summation order: lanes = 4 restates OpenCV 4.x's SIMD kernel (default), 0 the
 * left-to-right order of OpenCV 3.x (see resize.c) */
void orc_set_resize_simd(int lanes);
int orc_resize_simd(void);
/* the tables the cubic resize uses (for kernel cross-checks) */
void orc_cubic_tables(int s, int d, int* ofs /* d */, float* coef /* d*4 */);

/* ---- PAF score: restates getScoreAB (src/openpose/net/bodyPartConnectorBase.cpp:12-75) ----- */
float orc_paf_score(const float* candA, const float* candB /* (x,y,score) */,
                    const float* mapX, const float* mapY, int hm_w, int hm_h,
                    float inter_th, float inter_min_above, float default_nms_th);

/* ---- connector: restates op::connectBodyPartsCpu (bodyPartConnectorBase.cpp:1327-1377) ------
 * heat    : [nparts+1+2*npairs][hm_h][hm_w]   (BODY_25: 78 planes)
 * peaks   : [nparts][max_peaks+1][3]
 * out_keypoints: [max_people][nparts][3], out_scores [max_people]; returns number of people
 * (or -1 on error).  If the true count exceeds max_people, only max_people rows are written
 * but the true count is returned.
 * pose_model: 0 = BODY_25, 1 = COCO_18, 2 = MPI_15, 3 = MPI_15_4 (enumClasses.hpp:9-30)    */
int orc_connect_body_parts(float* out_keypoints, float* out_scores, int max_people,
                           const float* heat, const float* peaks, int pose_model,
                           int hm_w, int hm_h, int max_peaks, float inter_min_above,
                           float inter_th, int min_subset_cnt, float min_subset_score,
                           float default_nms_th, float scale_factor, int maximize_positives);
/* same, but fed by precomputed pair scores [npairs][max_peaks][max_peaks] (the reference's
 * alternate createPeopleVector input, bodyPartConnectorBase.cpp:321-340)                    */
int orc_connect_from_scores(float* out_keypoints, float* out_scores, int max_people,
                            const float* pair_scores, const float* peaks, int pose_model,
                            int max_peaks, int min_subset_cnt, float min_subset_score,
                            float scale_factor, int maximize_positives);
/* GPU-path assembly (pafPtrIntoVector + pafVectorIntoPeopleVector, bodyPartConnectorBase.cpp
 * :474-718) followed by the same threshold/array stages; used for models the CPU path rejects */
int orc_connect_gpu_semantics(float* out_keypoints, float* out_scores, int max_people,
                              const float* pair_scores, const float* peaks, int pose_model,
                              int max_peaks, int min_subset_cnt, float min_subset_score,
                              float scale_factor, int maximize_positives);
/* same, for any model given its tables (BODY_135 and the other models the CPU path rejects);
 * pairs: 2*npairs part indices (getPosePartPairs) */
int orc_connect_gpu_tables(float* out_keypoints, float* out_scores, int max_people,
                           const float* pair_scores, const float* peaks, int parts, int npairs,
                           const unsigned* pairs, int max_peaks, int min_subset_cnt,
                           float min_subset_score, float scale_factor, int maximize_positives);
/* dense pair scores [npairs][max_peaks][max_peaks] via getScoreAB (0 where no peak); mapx/mapy:
 * absolute heat channel of each pair's x/y PAF */
void orc_pair_scores(float* out, const float* heat, const float* peaks, int npairs,
                     const unsigned* pairs, const unsigned* mapx, const unsigned* mapy, int W,
                     int H, int max_peaks, float inter_th, float inter_min_above, float nms_th);
/* pose tables (poseParameters.cpp:253-256,413-419) */
int orc_pose_num_parts(int pose_model);
int orc_pose_num_pairs(int pose_model);
const unsigned* orc_pose_pairs(int pose_model);
const unsigned* orc_pose_map_idx(int pose_model);

/* ---- frame -> net input (preprocess.c): ScaleAndSizeExtractor::extract
 * (scaleAndSizeExtractor.cpp:37-105) and CvMatToOpInput::createArray's CPU branch
 * (cvMatToOpInput.cpp:63-98: warpAffine + uCharCvMatToFloatPtr).  Parity unpinned (OpenCV). */
int orc_scale_and_size(int in_w, int in_h, int net_w, int net_h, float dyn, int scale_number,
                       double scale_gap, double* scales, int* sizes);
double orc_resize_scale_factor(int iw, int ih, int tw, int th);
void orc_warp_tab(int cubic, short* itab);
void orc_cvmat_to_input(float* dst, const uint8_t* src, int sw, int sh, double scale, int dw,
                        int dh, int normalize);
/* cv::warpAffine(INTER_LINEAR | WARP_INVERSE_MAP, constant 0) + uCharCvMatToFloatPtr: the face /
 * hand crops (faceExtractorCaffe.cpp:215-232, handExtractorCaffe.cpp:44-73); M [2][3] */
void orc_warp_affine_inv(float* dst, const uint8_t* src, int sw, int sh, const double* M, int dw,
                         int dh, int normalize);

/* ---- Caffe layer semantics for the BODY_25 prototxt (NCHW fp32, batch n) ------------------ */
/* Convolution: cross-correlation, zero pad, stride 1, bias (Caffe ConvolutionLayer) */
void orc_conv2d(float* out, const float* in, const float* w /* [co][ci][k][k] */,
                const float* bias, int n, int ci, int h, int wd, int co, int k, int pad,
                int nthreads);
/* PReLU, per channel slope (Caffe PReLULayer, channel_shared=false) -- in place */
void orc_prelu(float* x, const float* slope, int n, int c, int hw);
void orc_relu(float* x, long count);
/* MaxPool kernel k stride s, pad 0, ceil sizing (Caffe PoolingLayer) */
void orc_maxpool(float* out, const float* in, int n, int c, int h, int w, int k, int s,
                 int oh, int ow);

/* ---- renderers (render.c): renderKeypointsOld / renderKeypoints, renderBodyPartHeatMap(s),
 * renderPartAffinities (render.hu, renderPose.cu).  Parity unpinned (CUDA device library
 * transcendentals); `ambiguous` marks the pixels where that can matter. */
#define ORC_RENDER_MAX_PEOPLE 1024
void orc_render_keypoints(float* frame, int w, int h, const float* kp, int people, int parts,
                          const unsigned* pairs, int npairs, const float* colors, int ncolors,
                          const float* scales, int nscales, float radius, float line_width,
                          float threshold, float alpha, int blend, int eye1, int eye2,
                          unsigned char* ambiguous);
float orc_cuda_bicubic(const float* src, float xs, float ys, int sw, int sh);
void orc_render_heat_map(float* frame, int w, int h, const float* heat, int hw, int hh,
                         float scale, int part, float alpha, int abs_value);
void orc_render_heat_maps(float* frame, int w, int h, const float* heat, int hw, int hh,
                          float scale, int parts, const float* colors, int ncolors, float alpha);
void orc_render_pafs(float* frame, int w, int h, const float* heat, int hw, int hh, float scale,
                     int first, int count, float alpha);

#ifdef __cplusplus
}
#endif
#endif
