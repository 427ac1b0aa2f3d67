// ref_render.cpp -- TEST INFRASTRUCTURE: exposes the reference's GPU render tables (the
// *_RENDER_GPU macros of include/openpose/pose/poseParametersRender.hpp,
// include/openpose/face/faceParameters.hpp:12-21 and include/openpose/hand/handParameters.hpp:12-39)
// as data, expanded by the reference's own headers compiled here.  tools/gen_render_tables.py reads
// them through ref_render_table() and writes openpose_amd/csrc/kernels/render_tables.inc plus the
// fixture tests/golden/render_tables.json.  Built by `make -C oracle ref` into oracle/_ref/ only.
#include <cstring>

#include <openpose/face/faceParameters.hpp>
#include <openpose/hand/handParameters.hpp>
#include <openpose/pose/poseParametersRender.hpp>

namespace {

// the tables renderPose.cu:12-39 declares, in this order, then the face and hand ones
// (renderFace.cu:9-11, renderHand.cu:9-11)
#define OPK_TABLE(P, S, C)                                                                 \
    {                                                                                      \
        static const unsigned pairs[] = {P};                                               \
        static const float scales[] = {S};                                                 \
        static const float colors[] = {C};                                                 \
        return copy(pairs, sizeof(pairs) / sizeof(pairs[0]), scales,                       \
                    sizeof(scales) / sizeof(scales[0]), colors,                            \
                    sizeof(colors) / sizeof(colors[0]), out_pairs, out_scales, out_colors, \
                    counts, cap);                                                          \
    }

int copy(const unsigned* p, int np, const float* s, int ns, const float* c, int nc, unsigned* op,
         float* os, float* oc, int* counts, int cap)
{
    if (np > cap || ns > cap || nc > cap) return -1;
    std::memcpy(op, p, np * sizeof(unsigned));
    std::memcpy(os, s, ns * sizeof(float));
    std::memcpy(oc, c, nc * sizeof(float));
    counts[0] = np;
    counts[1] = ns;
    counts[2] = nc;
    return 0;
}

}  // namespace

namespace op {
// inside op, as renderPose.cu is (the BODY_135 tables use op::H135 / op::F135)
static int table(int which, unsigned* out_pairs, float* out_scales, float* out_colors, int* counts,
                 int cap)
{
    switch (which) {
    case 0: OPK_TABLE(POSE_BODY_25_PAIRS_RENDER_GPU, POSE_BODY_25_SCALES_RENDER_GPU,
                      POSE_BODY_25_COLORS_RENDER_GPU)
    case 1: OPK_TABLE(POSE_COCO_PAIRS_RENDER_GPU, POSE_COCO_SCALES_RENDER_GPU,
                      POSE_COCO_COLORS_RENDER_GPU)
    case 2: OPK_TABLE(POSE_MPI_PAIRS_RENDER_GPU, POSE_MPI_SCALES_RENDER_GPU,
                      POSE_MPI_COLORS_RENDER_GPU)
    case 3: OPK_TABLE(POSE_BODY_19_PAIRS_RENDER_GPU, POSE_BODY_19_SCALES_RENDER_GPU,
                      POSE_BODY_19_COLORS_RENDER_GPU)
    case 4: OPK_TABLE(POSE_BODY_23_PAIRS_RENDER_GPU, POSE_BODY_23_SCALES_RENDER_GPU,
                      POSE_BODY_23_COLORS_RENDER_GPU)
    case 5: OPK_TABLE(POSE_BODY_25B_PAIRS_RENDER_GPU, POSE_BODY_25B_SCALES_RENDER_GPU,
                      POSE_BODY_25B_COLORS_RENDER_GPU)
    case 6: OPK_TABLE(POSE_BODY_135_PAIRS_RENDER_GPU, POSE_BODY_135_SCALES_RENDER_GPU,
                      POSE_BODY_135_COLORS_RENDER_GPU)
    case 7: OPK_TABLE(POSE_CAR_12_PAIRS_RENDER_GPU, POSE_CAR_12_SCALES_RENDER_GPU,
                      POSE_CAR_12_COLORS_RENDER_GPU)
    case 8: OPK_TABLE(POSE_CAR_22_PAIRS_RENDER_GPU, POSE_CAR_22_SCALES_RENDER_GPU,
                      POSE_CAR_22_COLORS_RENDER_GPU)
    case 9: OPK_TABLE(FACE_PAIRS_RENDER_GPU, FACE_SCALES_RENDER_GPU, FACE_COLORS_RENDER_GPU)
    case 10: OPK_TABLE(HAND_PAIRS_RENDER_GPU, HAND_SCALES_RENDER_GPU, HAND_COLORS_RENDER_GPU)
    default: return -2;
    }
}
}  // namespace op

// which: 0 BODY_25, 1 COCO, 2 MPI, 3 BODY_19, 4 BODY_23, 5 BODY_25B, 6 BODY_135, 7 CAR_12,
// 8 CAR_22, 9 FACE, 10 HAND.  counts = {#pair entries, #scales, #color floats}.
extern "C" int ref_render_table(int which, unsigned* out_pairs, float* out_scales, float* out_colors,
                                int* counts, int cap)
{
    return op::table(which, out_pairs, out_scales, out_colors, counts, cap);
}
