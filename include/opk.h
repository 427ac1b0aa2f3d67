/*
 * opk.h -- C-ABI of libopk_hip.so, the MI355X (gfx950) implementation of OpenPose's per-frame
 * body hot path: BODY_25 CNN forward -> resizeAndMerge -> NMS -> bodyPartConnector.
 *
 * Plain C: pointers, sizes and int status codes, no C++ or torch types.  Every function returns
 * OPK_OK (0) or an error code; opk_last_error() returns the calling thread's message (the C++ shim
 * in include/openpose_amd/ converts it into op::error(), the reference's error convention,
 * errorAndLog.cpp:158-233).  "dev" pointers are device (HBM) pointers; "host" pointers host memory.
 * All device work is enqueued on the context's hipStream_t; functions that hand results to the host
 * synchronise that stream (the points where the reference reads cpu_data()).
 *
 * Each entry point names the reference interface it replaces (paths under /root/reference/).
 */
#ifndef OPK_H
#define OPK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OPK_OK 0
#define OPK_ERR_ARG 1      /* invalid argument (reference: op::error(...) sanity checks)       */
#define OPK_ERR_HIP 2      /* HIP runtime error (reference: cudaCheck, gpu/cuda.cpp:18-26)      */
#define OPK_ERR_STATE 3    /* call out of order (e.g. forward before weights)                   */
#define OPK_ERR_UNSUPPORTED 4

/* PoseModel values (include/openpose/pose/enumClasses.hpp:9-30); the tables of every model are
 * generated from the reference's poseParameters.cpp (tools/gen_pose_tables.py) */
#define OPK_BODY_25 0
#define OPK_COCO_18 1
#define OPK_MPI_15 2
#define OPK_MPI_15_4 3
#define OPK_BODY_19 4
#define OPK_BODY_19_X2 5
#define OPK_BODY_19N 6
#define OPK_BODY_25E 7
#define OPK_CAR_12 8
#define OPK_BODY_25D 9
#define OPK_BODY_23 10
#define OPK_CAR_22 11
#define OPK_BODY_19E 12
#define OPK_BODY_25B 13
#define OPK_BODY_135 14

/* Connector semantics.  OPK_CONNECT_CPU: connectBodyPartsCpu (bodyPartConnectorBase.cpp:1327-1377,
 * per-pair greedy matching; the reference accepts BODY_25 / COCO_18 / MPI_15(_4) only).
 * OPK_CONNECT_GPU: connectBodyPartsGpu's host assembly (bodyPartConnectorBase.cu:147-250:
 * pafPtrIntoVector's global sort + pafVectorIntoPeopleVector; every model, BODY_135 included).
 * Pair scores are the same getScoreAB integrals in both. */
#define OPK_CONNECT_CPU 0
#define OPK_CONNECT_GPU 1

const char* opk_last_error(void);
int opk_version(void);

/* ---- context: one per GPU worker thread (reference: one PoseExtractorCaffe per GPU thread,
 *      wrapperAuxiliary.hpp:328-337; device bound at init like Caffe::SetDevice, netCaffe.cpp:169) */
typedef struct opk_ctx opk_ctx;
/* device -1: host-only context (graph planning, opk_net_conv_info; no device work) */
int opk_ctx_create(int device, void* hip_stream /* used as given; NULL = the null stream */,
                   opk_ctx** out);
/* same, with a private non-blocking stream owned (and destroyed) by the context */
int opk_ctx_create_private_stream(int device, opk_ctx** out);
int opk_ctx_destroy(opk_ctx* ctx);
int opk_ctx_stream(opk_ctx* ctx, void** hip_stream);
/* waits for the context stream and for the side streams of the context's objects (a pose
 * pipeline's post-processing stream) */
int opk_sync(opk_ctx* ctx);
int opk_malloc(opk_ctx* ctx, void** dev, size_t bytes);
int opk_free(opk_ctx* ctx, void* dev);
int opk_memset(opk_ctx* ctx, void* dev, int value, size_t bytes);
int opk_memcpy_h2d(opk_ctx* ctx, void* dev_dst, const void* host_src, size_t bytes);
int opk_memcpy_d2h(opk_ctx* ctx, void* host_dst, const void* dev_src, size_t bytes); /* syncs */
/* element type conversion on the device, on the context stream: OPK_F32 <-> OPK_F64 (double -> float
 * rounds to nearest).  The plugin functions' double instantiations (resizeAndMergeBase.cu:575-581,
 * nmsBase.cu:353-358, bodyPartConnectorBase.cu:252-266, which compute in double) run the float
 * kernels between two conversions here (integration/openpose_hip_shim.cpp): the results are the
 * float instantiation's, widened. */
#define OPK_F32 0
#define OPK_F64 1
int opk_convert(opk_ctx* ctx, void* dst_dev, int dst_type, const void* src_dev, int src_type,
                size_t count);

/* ---- resizeAndMerge: replaces op::resizeAndMergeGpu<float>
 *      (include/openpose/net/resizeAndMergeBase.hpp:17-20) with resizeAndMergeCpu numerics
 *      (src/openpose/net/resizeAndMergeBase.cpp:9-113: cv::resize INTER_CUBIC per plane, then the
 *      multi-scale average).  target_size / source_sizes are NCHW {N, C, H, W}; N frames are
 *      processed as a batch (the reference merges N into one frame only for N == 1 per scale).
 *      scale_ratios is accepted for signature parity and ignored, as in the CPU path (:18). */
int opk_resize_and_merge(opk_ctx* ctx, float* target_dev, const float* const* sources_dev,
                         int num_sources, const int target_size[4], const int* source_sizes,
                         const float* scale_ratios);

/* ---- NMS: replaces op::nmsGpu<float> (include/openpose/net/nmsBase.hpp:14-16) with nmsCpu
 *      numerics (src/openpose/net/nmsBase.cpp:7-170).  target_size = {N, parts, maxPeaks+1, 3},
 *      source_size = {N, C, H, W}; only the first `parts` planes of each frame are scanned.
 *      kernel_scratch (the reference's int peak map) may be NULL: this implementation never
 *      materialises it (peaks are appended to small per-plane candidate lists owned by the
 *      context, then sorted into raster order per plane). */
int opk_nms(opk_ctx* ctx, float* target_dev, int* kernel_scratch_dev, const float* source_dev,
            float threshold, const int target_size[4], const int source_size[4],
            float offset_x, float offset_y);

/* ---- Heat-map semantics of the reference's two builds (resize + NMS).
 * OPK_MAPS_CPU (the default everywhere): resizeAndMergeCpu + nmsCpu, as above.
 * OPK_MAPS_CUDA: what a CUDA build of the reference computes --
 *   resizeAndMergeGpu (src/openpose/net/resizeAndMergeBase.cu:105-162,274-495): Catmull-Rom
 *   bicubic (cubicInterpolate/bicubicInterpolate, include/openpose_private/gpu/cuda.hu:92-145) with
 *   the clamped base, one source only at x8 (or identity; other ratios are the reference's
 *   "Kernel only implemented for 8x resize" error), several sources scaled by
 *   (W/W0) / (scale_ratios[i] / scale_ratios[0]) and averaged as sum / N (scale_ratios required);
 *   nmsGpu (src/openpose/net/nmsBase.cu:50-90,161-240): interior pixels only, strictly greater
 *   than all 8 neighbours, centroid sums fused multiply-adds (nvcc's default contraction).
 * The expressions are evaluated as written, each operation rounded (nvcc's exact contraction of the
 * cubic polynomial is not reproducible without the CUDA toolchain: parity unpinned). */
#define OPK_MAPS_CPU 0
#define OPK_MAPS_CUDA 1
int opk_resize_and_merge_semantics(opk_ctx* ctx, float* target_dev, const float* const* sources_dev,
                                   int num_sources, const int target_size[4],
                                   const int* source_sizes, const float* scale_ratios,
                                   int semantics);
int opk_nms_semantics(opk_ctx* ctx, float* target_dev, int* kernel_scratch_dev,
                      const float* source_dev, float threshold, const int target_size[4],
                      const int source_size[4], float offset_x, float offset_y, int semantics);

/* ---- PAF pair scores: the pafScoreKernel stage of op::connectBodyPartsGpu
 *      (src/openpose/net/bodyPartConnectorBase.cu:107-145) computed with the CPU path's getScoreAB
 *      numerics (bodyPartConnectorBase.cpp:12-75: clamp to the map, 0 on rejection).
 *      pair_scores_dev: [N][numPairs][maxPeaks][maxPeaks]; only i < nA, j < nB are written.
 *      heat: [N][heat_channels][heat_h][heat_w]; peaks: [N][parts][maxPeaks+1][3]. */
int opk_paf_scores(opk_ctx* ctx, float* pair_scores_dev, const float* heat_dev,
                   const float* peaks_dev, int num_frames, int pose_model, int heat_channels,
                   int heat_h, int heat_w, int max_peaks, float inter_threshold,
                   float inter_min_above_threshold, float default_nms_threshold);

/* ---- connectBodyParts: replaces op::connectBodyPartsGpu<float>
 *      (include/openpose/net/bodyPartConnectorBase.hpp:17-24) with connectBodyPartsCpu semantics
 *      (bodyPartConnectorBase.cpp:1327-1377): GPU pair scores + host people assembly.
 *      keypoints_host [max_people][parts][3], scores_host [max_people]; *num_people gets the true
 *      count (rows beyond max_people are dropped). */
int opk_connect_body_parts(opk_ctx* ctx, float* keypoints_host, float* scores_host,
                           int max_people, int* num_people, const float* heat_dev,
                           const float* peaks_dev, int pose_model, int heat_channels, int heat_h,
                           int heat_w, int max_peaks, float inter_min_above_threshold,
                           float inter_threshold, int min_subset_cnt, float min_subset_score,
                           float default_nms_threshold, float scale_factor,
                           int maximize_positives);

/* Host-only people assembly from host peaks + host dense pair scores
 * (createPeopleVector's precomputed-score input, bodyPartConnectorBase.cpp:321-340, then
 * removePeopleBelowThresholdsAndFillFaces + peopleVectorToPeopleArray :720-934). */
int opk_assemble_people(float* keypoints_host, float* scores_host, int max_people,
                        int* num_people, const float* pair_scores_host,
                        const float* peaks_host, int pose_model, int max_peaks,
                        int min_subset_cnt, float min_subset_score, float scale_factor,
                        int maximize_positives);

/* The same two with a connector semantics (OPK_CONNECT_CPU / OPK_CONNECT_GPU); the GPU
 * semantics replace op::connectBodyPartsGpu<float> for every model. */
int opk_assemble_people_semantics(float* keypoints_host, float* scores_host, int max_people,
                                  int* num_people, const float* pair_scores_host,
                                  const float* peaks_host, int pose_model, int max_peaks,
                                  int min_subset_cnt, float min_subset_score, float scale_factor,
                                  int maximize_positives, int semantics);
int opk_connect_body_parts_semantics(opk_ctx* ctx, float* keypoints_host, float* scores_host,
                                     int max_people, int* num_people, const float* heat_dev,
                                     const float* peaks_dev, int pose_model, int heat_channels,
                                     int heat_h, int heat_w, int max_peaks,
                                     float inter_min_above_threshold, float inter_threshold,
                                     int min_subset_cnt, float min_subset_score,
                                     float default_nms_threshold, float scale_factor,
                                     int maximize_positives, int semantics);

/* ---- Keypoint post-steps (host arrays [people][parts][3]).
 * opk_scale_keypoints replaces op::KeypointScaler::scale (src/openpose/core/keypointScaler.cpp:64-95;
 * getScaleAndOffset :6-45): scale_mode = op::ScaleMode (0 InputResolution = unchanged,
 * 1 NetOutputResolution, 2 OutputResolution, 3/4 ZeroToOne(FixedAspect), 5/6 PlusMinusOne(...)).
 * opk_keep_top_n_people replaces op::KeepTopNPeople::keepTopPeople (keepTopNPeople.cpp:16-86,
 * --number_people_max): people ranked by score * sqrt(keypoint box area) and the top max_people
 * kept in their original order; *out_people = rows written (people itself when no cut is needed),
 * out_index_host (may be NULL) = source person of each row. */
int opk_scale_keypoints(float* keypoints_host, int people, int parts, int scale_mode,
                        double scale_input_to_output, double scale_net_to_output, int producer_w,
                        int producer_h);
int opk_keep_top_n_people(const float* keypoints_host, int people, int parts,
                          const float* scores_host, int max_people, float* out_keypoints_host,
                          int* out_index_host, int* out_people);

/* ---- People JSON (--write_json).  One keypoint array of the reference's keypointVector
 * (WPeopleJsonSaver::workConsumer, include/openpose/filestream/wPeopleJsonSaver.hpp:75-88):
 * name ("person_id", "pose_keypoints_2d", ...), ndims 0 (empty op::Array), 1 ([people], e.g. the
 * person ids as float) or 3 ([people][parts][dims]); host data. */
typedef struct opk_json_keypoints {
    const char* name;
    const float* data;
    int ndims, people, parts, dims;
} opk_json_keypoints;
/* opk_people_json replaces op::savePeopleJson(keypointVector, candidates, fileName, humanReadable)
 * (src/openpose/filestream/fileStream.cpp:306-344, JsonOfstream formatting): writes the file's text
 * (no terminating NUL counted) into out_host when *len + 1 <= capacity (out_host may be NULL to
 * query), *len = its length.  candidates_host: n_parts lists of [x, y, score] back to back,
 * candidate_counts_host[part] each (the Datum's poseCandidates; n_parts 0 = none, no
 * "part_candidates" key).  opk_save_people_json writes the same text to path (PeopleJsonSaver::save,
 * peopleJsonSaver.cpp:15-30, with the ".json" already in path). */
int opk_people_json(const opk_json_keypoints* arrays, int n_arrays, const float* candidates_host,
                    const int* candidate_counts_host, int n_parts, int human_readable,
                    char* out_host, size_t capacity, size_t* len);
int opk_save_people_json(const char* path, const opk_json_keypoints* arrays, int n_arrays,
                         const float* candidates_host, const int* candidate_counts_host,
                         int n_parts, int human_readable);

/* Pose tables (getPoseNumberBodyParts, addBkgChannel, getPosePartPairs, getPoseMapIndex;
 * poseParameters.hpp:17-34).  Any output pointer may be NULL; pairs gets 2*npairs entries,
 * map_idx the model's map-index entries (heat_channels - parts - bkg). */
int opk_pose_model_info(int pose_model, int* parts, int* bkg, int* npairs, int* heat_channels,
                        int* pairs, int* map_idx);
/* getPoseDefaultNmsThreshold / getPoseDefaultConnectInterThreshold (poseParameters.hpp:29-31) */
int opk_pose_default_thresholds(int pose_model, int maximize_positives, float* nms_threshold,
                                float* inter_threshold);

/* ---- Frame -> net input.
 * opk_scale_and_size replaces op::ScaleAndSizeExtractor::extract
 *      (include/openpose/core/scaleAndSizeExtractor.hpp:17-18, scaleAndSizeExtractor.cpp:37-105):
 *      net_w or net_h <= 0 derives that side from the frame's aspect ratio (-1x368), bounded at
 *      16:9 times dynamic_behavior when it is > 0 (--net_resolution_dynamic); scales[i] =
 *      scaleInputToNetInputs, net_sizes[2i], [2i+1] = netInputSizes (w, h), i < scale_number.
 * opk_cvmat_to_input replaces op::CvMatToOpInput::createArray for one scale
 *      (include/openpose/core/cvMatToOpInput.hpp:17-19, cvMatToOpInput.cpp:63-98), for a batch:
 *      frames_dev = n BGR uint8 frames [height][step bytes] (step 0 = width*3), input_dev =
 *      [n][3][net_h][net_w] fp32: cv::warpAffine(diag(scale)) with OpenCV's fixed-point 8-bit
 *      arithmetic (INTER_LINEAR for scale <= 1, INTER_CUBIC above; zero border), then
 *      u/256 - 0.5 when normalize == 1 (uCharCvMatToFloatPtr, openCv.cpp:57-150). */
int opk_scale_and_size(int in_w, int in_h, int net_w, int net_h, float dynamic_behavior,
                       int scale_number, double scale_gap, double* scales, int* net_sizes);
int opk_cvmat_to_input(opk_ctx* ctx, float* input_dev, const uint8_t* frames_dev, int n, int width,
                       int height, size_t step, double scale, int net_w, int net_h, int normalize);

/* Kernel-variant switches (no reference counterpart; A/B tests and tuning only): key = one of
 * "CONV3_SMALL", "CONV3_W16", "CONV3_PERSIST", "CONV3_WIDE", "CONV3P_ASMR", "CONV3P_WIDE",
 * "CONV3P_PRIO", "CONV3W", "CONV1_TILE", "CONV1_N64W16", "CONV1_FUSED" (read when a launch is
 * planned);
 * reset != 0 removes the key (back to the product default).  Process-wide; the environment is
 * never consulted. */
int opk_dev_set(const char* key, int value, int reset);

/* ---- Net: replaces op::Net / op::NetCaffe (include/openpose/net/net.hpp:8-18,
 *      netCaffe.hpp:12-13).  prototxt: a Caffe prototxt path, or one of the reference's networks
 *      generated in the library: "builtin:BODY_25", "builtin:COCO_18", "builtin:MPI_15",
 *      "builtin:MPI_15_4", "builtin:HAND", "builtin:FACE" (models/.../pose_deploy*.prototxt).
 *      Supported layers: Convolution 3x3/pad 1, 7x7/pad 3, 1x1; ReLU/PReLU in place after a conv;
 *      MaxPool 2x2/2; channel Concat; the output blob is a Concat or a conv's top. */
typedef struct opk_net opk_net;
/* caffemodel (or NULL): trained weights, loaded as caffe::Net::CopyTrainedLayersFrom does
 * (netCaffe.cpp:163-185): every conv whose name is in the file gets its weights, bias and the
 * slopes of its PReLU layer, shapes checked; file layers the net lacks are ignored.  Convs not in
 * the file must be set with opk_net_set_conv before a forward. */
int opk_net_create(opk_ctx* ctx, const char* prototxt, const char* caffemodel, opk_net** out);
int opk_net_load_caffemodel(opk_net* net, const char* caffemodel, int* convs_loaded);
/* Host utility (no device): blob `index` of `layer` in a .caffemodel; shape gets <= 8 dims
 * (legacy 4-D shapes as stored), data (may be NULL) the float values. */
int opk_caffemodel_blob(const char* caffemodel, const char* layer, int index, float* data,
                        size_t capacity, int64_t* shape, int* ndim);
int opk_net_destroy(opk_net* net);
int opk_net_num_convs(opk_net* net);
/* name buffer >= 64 bytes; act: 0 none, 1 ReLU, 2 PReLU */
int opk_net_conv_info(opk_net* net, int index, char* name, int* cin, int* cout, int* kernel,
                      int* act);
/* Caffe layouts: weights [cout][cin][k][k], bias [cout], slope [cout] (NULL unless PReLU) */
int opk_net_set_conv(opk_net* net, const char* name, const float* weights_host,
                     const float* bias_host, const float* slope_host);
/* input NCHW fp32 on device: [n][3][h][w] (the net input blob, netCaffe.cpp:230-247) */
int opk_net_forward(opk_net* net, const float* input_dev, int n, int h, int w);
/* useful (unpadded) convolution FLOPs of one frame of h x w (2 * MACs, all conv layers) */
int opk_net_flops_per_frame(opk_net* net, int h, int w, double* flops);
/* Arithmetic of the forward (no reference counterpart: Caffe's forward is fp32).
 * OPK_PRECISION_FP16 (default): fp16 weights and stored activations, fp32 MFMA accumulation, the
 *   tuned fused kernels -- net output within rel-L2 ~2.5e-3 of fp32 on random He-initialised
 *   BODY_25 nets.
 * OPK_PRECISION_SPLIT: every weight and activation held as an fp16 hi/lo pair (x = hi + lo to
 *   ~22 bits; each layer's weights scaled by a power of two so that w_lo stays a normal fp16
 *   number), three MFMA passes per conv (x_hi w_hi + x_lo w_hi + x_hi w_lo, each product exact in
 *   fp32): fp32-level results (parity mode: as close to the exact convolution as an fp32 CPU
 *   implementation is) at 3x the MFMA work and 2x the activation bytes -- the 512-position
 *   persistent 8-wave kernel's split instantiation for every 96/128/256/512-channel 3x3 layer,
 *   conv_image's for the first conv, the generic kernel for the rest; no conv1 / head / pool
 *   fusion.  Re-plans the net's shapes; loaded weights are kept. */
#define OPK_PRECISION_FP16 0
#define OPK_PRECISION_SPLIT 1
int opk_net_set_precision(opk_net* net, int precision);
/* Forward timing (measurement hook, no reference counterpart): while enabled every forward is
 * bracketed by HIP events on the context stream; read waits for them and returns the number of
 * forwards since the last read and their summed device time in milliseconds. */
int opk_net_set_timing(opk_net* net, int enable);
int opk_net_read_timing(opk_net* net, int* forwards, double* total_ms);
/* device pointer + NCHW shape of the last forward's net_output blob.  Valid right after
 * opk_net_create, as NetCaffe::getOutputBlobArray is (poseExtractorCaffe.cpp:94-95 takes it once,
 * before any forward, and keeps it): before the first forward *output_dev is NULL and shape is
 * {0, out_channels, 0, 0}.  The buffer of one input shape is stable across direct forwards of
 * that shape (the values are the latest forward's).  A net driven by an opk_pose pipeline
 * alternates between two output buffers per input shape (batch i+1's nets write the one batch i's
 * post-processing does not read), so re-query the pointer after each forward.  A forward that
 * writes a buffer a pipeline's post-processing still reads -- including a direct opk_net_forward
 * between opk_pose_submit and opk_pose_collect -- waits for that post-processing first. */
int opk_net_output(opk_net* net, float** output_dev, int shape[4]);
/* Inspection (caffe::Net::blob_by_name, which NetCaffe does not expose; used by the per-layer
 * parity tests): frames [frame0, frame0 + nframes) of the named top of the last forward -- a
 * conv, pool or concat top, or net_output -- converted from its padded NHWC fp16 buffer (the fp32
 * output for net_output) to fp32 NCHW host memory [nframes][channels][h][w]; host_out NULL:
 * shape only.  Synchronises the context stream.  Blobs that fused kernels keep on chip
 * (conv1_1 / conv1_2 with the fused first layers, a pooled conv's un-pooled output, Mconv6 of a
 * fused head pair) fail with the "kept on chip" message. */
int opk_net_blob(opk_net* net, const char* name, int frame0, int nframes, float* host_out,
                 int shape[4]);
/* Kernels launched by the last forward run while the dev switch LAUNCH_LOG was 1, one
 * "<layer>\t<kernel instantiation>\n" line per launch.  *needed = bytes incl. the NUL; the text
 * is copied when size >= *needed. */
int opk_net_launch_log(opk_net* net, char* buf, size_t size, size_t* needed);

/* ---- Pose extractor: replaces op::PoseExtractorCaffe::forwardPass
 *      (src/openpose/pose/poseExtractorCaffe.cpp:200-334) for a batch of frames:
 *      net -> resizeAndMerge -> NMS -> connector, one result set per frame. */
typedef struct opk_pose opk_pose;
/* PoseProperty (enumClasses.hpp:32-40) */
#define OPK_PROP_NMS_THRESHOLD 0
#define OPK_PROP_INTER_MIN_ABOVE_THRESHOLD 1
#define OPK_PROP_INTER_THRESHOLD 2
#define OPK_PROP_MIN_SUBSET_CNT 3
#define OPK_PROP_MIN_SUBSET_SCORE 4
int opk_pose_create(opk_ctx* ctx, opk_net* net /* may be NULL: net output injected */,
                    int maximize_positives, opk_pose** out);
/* any pose model (the net output / injected heat maps carry its heat_channels) and connector
 * semantics; opk_pose_create = (BODY_25, OPK_CONNECT_CPU).  OPK_CONNECT_CPU with a model the
 * reference's CPU connector rejects fails with OPK_ERR_UNSUPPORTED. */
int opk_pose_create_model(opk_ctx* ctx, opk_net* net, int pose_model, int maximize_positives,
                          int semantics, opk_pose** out);
/* A pose uses its net until it is destroyed (its forwards, and the net's record of the
 * post-processing still reading each output buffer): destroy the pose before the net, as the
 * reference's PoseExtractorCaffe owns its net. */
int opk_pose_destroy(opk_pose* pose);
int opk_pose_set_property(opk_pose* pose, int property, double value);
/* heat-map semantics of the pipeline's resize + NMS (OPK_MAPS_CPU, the default, or OPK_MAPS_CUDA:
 * what the reference's CUDA build computes, see opk_nms_semantics); the lazy heat maps, the PAF
 * samples and opk_pose_heatmaps follow it.  Multi-scale with OPK_MAPS_CUDA needs the raw-frame
 * path (opk_pose_submit_frames), which knows scaleInputToNetInputs. */
int opk_pose_set_map_semantics(opk_pose* pose, int semantics);
/* --upsampling_ratio (include/openpose/flags.hpp:136; PoseExtractorCaffe's upsamplingRatio):
 * heat maps of round((out_h * ratio - 1)) + 1 rows (likewise columns) of the scale-0 net output,
 * resizeAndMergeCaffe.cpp:77-81, instead of the net input size; scaleNetToOutput then uses
 * mNetOutputSize = round(ratio / 8 x net input size) (poseExtractorCaffe.cpp:281-310).  ratio <= 0
 * (the default) = the net's decrease factor (8; 4 for BODY_19_X2).  CPU map semantics; the CUDA
 * build's resize accepts x8 only for one source (resizeAndMergeBase.cu) and so does OPK_MAPS_CUDA. */
int opk_pose_set_upsampling_ratio(opk_pose* pose, float ratio);
/* frames: [n][3][net_h][net_w] device fp32; producer_w/h: original frame size (for
 * scaleNetToOutput, poseExtractorCaffe.cpp:306-310) */
int opk_pose_forward(opk_pose* pose, const float* frames_dev, int n, int net_h, int net_w,
                     int producer_w, int producer_h);
/* heat-map injection (poseNetOutput path, poseExtractorCaffe.cpp:249-262): net output on device
 * [n][heat_channels][h][w] (78 for BODY_25, 439 for BODY_135); net_h/net_w = the net input size
 * it corresponds to */
int opk_pose_forward_net_output(opk_pose* pose, const float* net_output_dev, int n, int out_h,
                                int out_w, int net_h, int net_w, int producer_w, int producer_h);
/* Pipelined use (the reference's producer/worker/consumer threads, wrapperAuxiliary.hpp, on one
 * GPU): submit enqueues a batch's device work (net, NMS, PAF scores) and returns; collect waits
 * for the OLDEST submitted batch, assembles its people on the host and makes it the batch the
 * result accessors below refer to.  At most two batches in flight: submit(i+1) then collect(i)
 * overlaps the host assembly of batch i with the device work of batch i+1.  opk_pose_forward* =
 * submit + collect.  *frames (may be NULL) receives the collected batch's frame count.
 * Streams: the frames / net inputs / injected net output are read after the work queued on the
 * context stream before the submit.  When the pipeline runs its own net, a batch's
 * post-processing (overlay add, NMS, PAF scores) runs on a side stream after the batch's nets, so
 * work queued on the context stream after the submit is NOT ordered before it: keep the overlay
 * unchanged until collect (or opk_sync); forwards of the same net are ordered after it by the
 * net (opk_net_output).  The injection path stays on the context stream. */
int opk_pose_submit(opk_pose* pose, const float* frames_dev, int n, int net_h, int net_w,
                    int producer_w, int producer_h);
int opk_pose_submit_net_output(opk_pose* pose, const float* net_output_dev, int n, int out_h,
                               int out_w, int net_h, int net_w, int producer_w, int producer_h);
int opk_pose_collect(opk_pose* pose, int* frames);
/* Multi-scale (--scale_number > 1; poseExtractorCaffe.cpp:240-245 runs the net once per scale,
 * resizeAndMergeCpu averages the x8 resizes of every scale's output, resizeAndMergeBase.cpp:55-106):
 * frames_dev[i] = [n][3][net_hw[2i]][net_hw[2i+1]] net input of scale i (the reference's
 * inputNetData[i]); scale 0 sets the heat-map size and scaleNetToOutput.  1..8 scales. */
int opk_pose_submit_multi(opk_pose* pose, const float* const* frames_dev, const int* net_hw,
                          int num_scales, int n, int producer_w, int producer_h);
int opk_pose_forward_multi(opk_pose* pose, const float* const* frames_dev, const int* net_hw,
                           int num_scales, int n, int producer_w, int producer_h);
/* Raw frames: the whole per-frame path of the reference's Wrapper workers
 * (WScaleAndSizeExtractor -> WCvMatToOpInput -> WPoseExtractorNet, wrapperAuxiliary.hpp):
 * frames_dev = n BGR uint8 frames [height][step bytes] on device (step 0 = width*3), prepared
 * on the GPU for every scale of opk_pose_set_input (default: -1x368, dynamic 1, one scale, gap
 * 0.25 -- the reference's flag defaults), then one net pass per scale and the merged
 * post-processing.  Keypoints are in frame pixels (scaleNetToOutput for a frame-sized output). */
int opk_pose_set_input(opk_pose* pose, int net_w, int net_h, float dynamic_behavior,
                       int scale_number, double scale_gap);
int opk_pose_submit_frames(opk_pose* pose, const uint8_t* frames_dev, int n, int width,
                           int height, size_t step);
int opk_pose_forward_frames(opk_pose* pose, const uint8_t* frames_dev, int n, int width,
                            int height, size_t step);
/* net input of scale i prepared by the last opk_pose_submit_frames ([n][3][net_h][net_w]) */
int opk_pose_net_input(opk_pose* pose, int scale, const float** input_dev, int* net_w,
                       int* net_h);
int opk_pose_pending(opk_pose* pose);   /* batches in flight, -1 for NULL */
/* optional additive overlay on the net output before resize (synthetic-people workloads):
 * [n][78][out_h][out_w] device fp32, NULL to disable.  With a pipeline that runs its own net the
 * overlay is read by the post-processing stream after the batch's nets: rewrite it only after the
 * batch is collected (or after opk_sync). */
int opk_pose_set_overlay(opk_pose* pose, const float* overlay_dev);
int opk_pose_num_people(opk_pose* pose, int frame);
/* keypoints_host [max_people][parts][3], scores_host [max_people] of one collected frame */
int opk_pose_keypoints(opk_pose* pose, int frame, float* keypoints_host, float* scores_host,
                       int max_people);
/* Post-processing timing (measurement hook, no reference counterpart): while enabled the device
 * work of every submitted batch after its net forward (overlay add, NMS, PAF integrals) is
 * bracketed by HIP events on the stream it runs on -- the pipeline's post-processing stream when
 * it runs its own net (batch i's post-processing then shares the GPU with batch i+1's nets, so
 * the span includes that time-sharing), the context stream on the injection path; read waits for
 * them and returns the number of batches since the last read and their summed device time in
 * milliseconds. */
int opk_pose_set_timing(opk_pose* pose, int enable);
int opk_pose_read_timing(opk_pose* pose, int* batches, double* total_ms);
/* Host-side collect timing (measurement hook, no reference counterpart): for the collects since
 * the last read, their number and the summed milliseconds spent waiting for the batches' device
 * results and assembling their people; *workers = the assembly threads (at most 16 and at most
 * the CPUs of the process's affinity mask).  Any pointer may be NULL. */
int opk_pose_read_collect_times(opk_pose* pose, int* collects, double* wait_ms, double* assembly_ms,
                                int* workers);
/* Every frame of the last collected batch as one packed host record (the result the reference's
 * WQueueOrderer re-sequences, wQueueOrderer.hpp:62-141): for each frame f in order,
 *   [people_f, keypoints_f (people_f x parts x 3), scores_f (people_f)]  (all float).
 * *used receives the floats needed; with capacity < *used nothing is written and the call fails
 * with OPK_ERR_ARG (records may be NULL to query the size). */
int opk_pose_records(opk_pose* pose, float* records_host, size_t capacity, size_t* used);
/* device pointers of the last forward's heatmaps [n][heat_channels][H][W] and peaks
 * [n][parts][128][3].
 * The pipeline evaluates heat-map values lazily from the net output (NMS and PAF scoring compute
 * the resized values they touch, bit-identical to resizeAndMerge); opk_pose_heatmaps writes the
 * full stack on first request after a collect, while no later batch is in flight.  With
 * opk_pose_forward_net_output the net output buffer must stay unchanged until then. */
int opk_pose_heatmaps(opk_pose* pose, float** heat_dev, int shape[4]);
/* shape of the last collected batch's heat maps (spHeatMapsBlob->shape(), poseExtractorCaffe.cpp:
 * 651-663) without writing them */
int opk_pose_heatmap_size(opk_pose* pose, int shape[4]);
int opk_pose_peaks(opk_pose* pose, float** peaks_dev, int shape[4]);
float opk_pose_scale_net_to_output(opk_pose* pose);
/* PoseExtractorNet::getHeatMapsCopy (src/openpose/pose/poseExtractorNet.cpp:106-244) for every
 * frame of the last collected batch: types = OPK_HEATMAP_* bits (copied in the order parts,
 * background, PAFs, as --heatmaps_add_parts/_bkg/_PAFs), scale_mode = op::ScaleMode
 * (include/openpose/core/enumClasses.hpp:6-17; --heatmaps_scale: 5 PlusMinusOne, 3 ZeroToOne,
 * 7 UnsignedChar, 8 NoScale).  dst_dev [n][channels][H][W] device, or NULL to get the shape. */
#define OPK_HEATMAP_PARTS 1
#define OPK_HEATMAP_BACKGROUND 2
#define OPK_HEATMAP_PAFS 4
int opk_pose_heatmaps_copy(opk_pose* pose, int types, int scale_mode, float* dst_dev,
                           int shape[4]);
/* PoseExtractorNet::getCandidatesCopy (poseExtractorNet.cpp:246-282) of one collected frame:
 * candidates_host [parts][127][3] (x, y in output pixels = net pixels * scaleNetToOutput, score),
 * counts_host [parts]; either may be NULL. */
int opk_pose_candidates(opk_pose* pose, int frame, float* candidates_host, int* counts_host);


/* ---- face / hand keypoints -------------------------------------------------------------------
 * op::FaceDetector::detectFaces (include/openpose/face/faceDetector.hpp:10-27,
 * src/openpose/face/faceDetector.cpp:122-139) and op::HandDetector::detectHands
 * (include/openpose/hand/handDetector.hpp:13-45, src/openpose/hand/handDetector.cpp:135-160):
 * rectangles (x, y, width, height) from pose keypoints_host [people][parts][3] of pose_model;
 * rects_host face [people][4], hand [people][2 (left, right)][4].  A model without the detector's
 * body parts (e.g. CAR_12) fails with OPK_ERR_UNSUPPORTED, as poseBodyPartMapStringToKey errors. */
int opk_face_detect(int pose_model, const float* keypoints_host, int people, int parts,
                    float* rects_host);
int opk_hand_detect(int pose_model, const float* keypoints_host, int people, int parts,
                    float* rects_host);

/* op::FaceExtractorCaffe / op::HandExtractorCaffe (include/openpose/face/faceExtractorCaffe.hpp:
 * 14-45, include/openpose/hand/handExtractorCaffe.hpp:14-52): forwardPass(rectangles, inputData)
 * + getFaceKeypoints() / getHandKeypoints(), for every rectangle of a set of frames at once.  net:
 * the face (builtin:FACE, pose_deploy.prototxt of models/face) or hand (builtin:HAND) net;
 * net_w x net_h = --face_net_resolution / --hand_net_resolution (multiples of 16, default
 * 368x368). */
typedef struct opk_extractor opk_extractor;
#define OPK_EXTRACT_FACE 0
#define OPK_EXTRACT_HAND 1
int opk_extractor_create(opk_ctx* ctx, opk_net* net, int kind, int net_w, int net_h,
                         opk_extractor** out);
int opk_extractor_destroy(opk_extractor* ex);
/* hand only: --hand_scale_number / --hand_scale_range (HandExtractorNet, handExtractorNet.cpp) */
int opk_extractor_set_scales(opk_extractor* ex, int number, float range);
/* crops per net forward (default 32; batches run in power-of-two sizes) */
int opk_extractor_set_max_batch(opk_extractor* ex, int max_batch);
int opk_extractor_parts(opk_extractor* ex);   /* net output channels - 1; -1 for NULL */
/* per-person heat maps (--heatmaps_add_* with --face / --hand; FaceExtractorNet::getHeatMaps,
 * HandExtractorNet::getHeatMaps): scale_mode = op::ScaleMode of --heatmaps_scale (-1 off).  The
 * first `parts` channels of each rectangle's x8-resized crop output, mapped as
 * updateFaceHeatMapsForPerson / updateHandHeatMapsForPerson do (faceExtractorCaffe.cpp:42-75,
 * handExtractorCaffe.cpp:126-160): PlusMinusOne(FixedAspect) fastTruncate(v)*2-1, UnsignedChar
 * (float)positiveIntRound(fastTruncate(v)*255), any other mode fastTruncate(v).  With several hand
 * scales the last scale's maps are kept (the reference copies its blob after the last net run). */
int opk_extractor_set_heatmaps(opk_extractor* ex, int scale_mode);
/* after opk_extractor_forward: device pointer + shape {hands (1 face / 2 hand), people, parts, H,
 * W}; zeros for the rectangles the reference skips.  Valid until the next forward. */
int opk_extractor_heatmaps(opk_extractor* ex, const float** heatmaps_dev, int shape[5]);
/* frames_dev: BGR uint8 [nframes][height][step] on device (step 0: width*3); rects_host as
 * opk_face_detect / opk_hand_detect return them; frame_of_host [people] (NULL: frame 0).
 * keypoints_host: face [people][parts][3], hand [2][people][parts][3] (left hands first), in
 * frame pixels; zeros where the reference skips the rectangle (face: side <= 40; hand: side <= 1
 * or area <= 10).  A non-square rectangle fails with OPK_ERR_ARG as the reference errors. */
int opk_extractor_forward(opk_extractor* ex, const uint8_t* frames_dev, int nframes, int width,
                          int height, size_t step, const float* rects_host,
                          const int* frame_of_host, int people, float* keypoints_host);
/* crops of the last forward (order: hand, person, scale; skipped rectangles have none): the 2x3
 * inverse map (frame <- crop) and the crop's net input [3][net_h][net_w] on device */
int opk_extractor_crop_count(opk_extractor* ex);
int opk_extractor_crop(opk_extractor* ex, int i, double* matrix_host, const float** input_dev);

/* ---- Measured ceilings (no reference counterpart; SURVEY.md §8d "confirm the vendor peaks"):
 *      dense fp16 MFMA rate of v_mfma_f32_16x16x32_f16 from registers (the conv kernels'
 *      instruction; 4 waves per SIMD, 8 independent chains, consecutive MFMAs on different operand
 *      pairs) on uniform random and on all-zero operands, in TFLOP/s, and the streaming HBM read
 *      rate over 2 GiB in GB/s.  Runs ~0.1 s of device work on the context's stream; synchronous. */
int opk_probe_peaks(opk_ctx* ctx, double* mfma_random_tflops, double* mfma_zero_tflops,
                    double* hbm_read_gbs);

/* ---- Renderers (enqueued on the context's stream).  frame_dev: the reference's float BGR frame
 *      [height][width][3] (0..255), drawn in place.
 * opk_render_pose_keypoints replaces op::renderPoseKeypointsGpu
 *   (include/openpose/pose/renderPose.hpp:14-18; src/openpose/pose/renderPose.cu:609-748 with
 *   renderKeypointsOld, include/openpose_private/utilities/render.hu:209-383): pose_dev
 *   [people][parts][3] (x, y, score) in frame pixels; every PoseModel, its pairs / colors / scales
 *   (pose/poseParametersRender.hpp), radius min(w,h)/100, line width min(w,h)/120; nothing is
 *   drawn for people == 0 unless blend_original == 0 (then the frame is cleared).  Errors as the
 *   reference: googly eyes with MPI, people > 127 (POSE_MAX_PEOPLE), an unknown model.  The
 *   reference's maxPtr / minPtr / scalePtr scratch is internal here.
 * opk_render_face_keypoints / opk_render_hand_keypoints replace op::renderFaceKeypointsGpu /
 *   op::renderHandKeypointsGpu (face/renderFace.hpp:12-15, hand/renderHand.hpp:12-15): 70 / 21
 *   parts, radius min/120 / min/100, line min/250 / min/80, no-op for count <= 0.
 * Keypoint renders take up to 1024 people (faces, hands) per call.
 * Heat-map renders (alpha outside [0, 1]: "Alpha must be in the range [0, 1]."; heat_dev
 *   [channels][heat_h][heat_w]; frame pixel x samples (x + 0.5) / scale_to_keep_ratio - 0.5):
 *   opk_render_pose_heat_map  = op::renderPoseHeatMapGpu  (renderPose.hpp:20-23): channel `part`,
 *                               bicubic, getColorHeatMap;
 *   opk_render_pose_heat_maps = op::renderPoseHeatMapsGpu (:25-28): every body part, nearest
 *                               sample, COCO colors;
 *   opk_render_pose_paf       = op::renderPosePAFGpu      (:30-33): PAF channels part, part + 1,
 *                               bilinear;
 *   opk_render_pose_pafs      = op::renderPosePAFsGpu     (:35-38): every PAF, from channel
 *                               parts + background;
 *   opk_render_pose_distance  = op::renderPoseDistanceGpu (:40-42): channel `part`, |bicubic|.
 * Arithmetic follows the reference expression by expression (each operation rounded); atan2f /
 * sinf / cosf are the HIP device library's (render parity unpinned at limb edges and for PAF
 * colours). */
int opk_render_pose_keypoints(opk_ctx* ctx, float* frame_dev, int pose_model, int people,
                              unsigned width, unsigned height, const float* pose_dev,
                              float render_threshold, int googly_eyes, int blend_original,
                              float alpha);
int opk_render_face_keypoints(opk_ctx* ctx, float* frame_dev, unsigned width, unsigned height,
                              const float* face_dev, int people, float render_threshold,
                              float alpha);
int opk_render_hand_keypoints(opk_ctx* ctx, float* frame_dev, unsigned width, unsigned height,
                              const float* hands_dev, int hands, float render_threshold,
                              float alpha);
int opk_render_pose_heat_map(opk_ctx* ctx, float* frame_dev, unsigned width, unsigned height,
                             const float* heat_dev, int heat_w, int heat_h,
                             float scale_to_keep_ratio, unsigned part, float alpha);
int opk_render_pose_heat_maps(opk_ctx* ctx, float* frame_dev, int pose_model, unsigned width,
                              unsigned height, const float* heat_dev, int heat_w, int heat_h,
                              float scale_to_keep_ratio, float alpha);
int opk_render_pose_paf(opk_ctx* ctx, float* frame_dev, int pose_model, unsigned width,
                        unsigned height, const float* heat_dev, int heat_w, int heat_h,
                        float scale_to_keep_ratio, int part, float alpha);
int opk_render_pose_pafs(opk_ctx* ctx, float* frame_dev, int pose_model, unsigned width,
                         unsigned height, const float* heat_dev, int heat_w, int heat_h,
                         float scale_to_keep_ratio, float alpha);
int opk_render_pose_distance(opk_ctx* ctx, float* frame_dev, unsigned width, unsigned height,
                             const float* heat_dev, int heat_w, int heat_h,
                             float scale_to_keep_ratio, unsigned part, float alpha);

#ifdef __cplusplus
}
#endif
#endif /* OPK_H */
