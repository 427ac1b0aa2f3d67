// input.h -- frame -> net input: ScaleAndSizeExtractor + CvMatToOpInput (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace opk {

struct Context;

// op::ScaleAndSizeExtractor::extract (src/openpose/core/scaleAndSizeExtractor.cpp:37-105):
// net input size of every scale (sizes: w, h pairs) and scaleInputToNetInputs.  net_w or net_h
// <= 0 selects the aspect-ratio-derived size (-1x368), bounded by `dyn`
// (--net_resolution_dynamic, > 0) at 16:9.
void scale_and_size(int in_w, int in_h, int net_w, int net_h, float dyn, int scale_number,
                    double scale_gap, double* scales, int* sizes);

// OpenCV's fixed-point tables behind cv::warpAffine on 8-bit images (imgwarp.cpp,
// initInterTab2D): weights [32*32][k*k] (k = 2 linear, 4 cubic; itab zeroed and one entry longer,
// OpenCV's sum correction reads past the last entry), and per destination index of one
// axis {first source tap, fraction index} for the inverse of the diagonal map diag(scale).
void warp_weight_table(bool cubic, short* itab);
void warp_axis_table(double scale, int d, bool cubic, int* tab /* 2*d */);

// op::CvMatToOpInput::createArray for one scale (cvMatToOpInput.cpp:63-98), a batch of n frames:
// src BGR uint8 [n][sh][step bytes] on device -> dst [n][3][dh][dw] fp32 on device
// (resizeFixedAspectRatio + uCharCvMatToFloatPtr with the VGG normalisation when normalize != 0).
// (stream: where the warp runs; nullptr = the context's stream)
void cvmat_to_input(Context* ctx, float* dst, const uint8_t* src, int n, int sw, int sh,
                    size_t step, double scale, int dw, int dh, int normalize, hipStream_t stream = nullptr);

}  // namespace opk
