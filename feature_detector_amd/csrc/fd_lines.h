// Host stage of fd_lsd_lines (fd_lines.cpp): region growing and rectangle fitting over the GPU's
// compact level-line lists, one frame per worker thread. Pure C++ (no HIP), built with g++ like the
// reference so its float sequence (glibc cosf / sinf / atan2f, no contraction) is the reference's.
#pragma once

#include <stdint.h>

#include "fd_hip.h"

namespace fdl {

// One frame's valid pixels in the reference's scan order (column outer, row inner): map index
// (row * (cols-1) + col), gradient norm and level-line angle.
struct FrameList {
    const int32_t *idx;
    const float *norm;
    const float *angle;
    int64_t n;
};

// FeatureLineDetector::DetectGoodFeatures (feature_line_detector.cpp:12-54) from the level-line map on,
// for `batch` frames of rows x cols. out: [batch][stride] rectangles (start/end already offset by 0.5,
// :43-44); counts: rectangles found per frame (may exceed stride; only stride are written). used0
// (optional, frame 0's list length): the final is_used flag of each listed pixel of frame 0.
// threads <= 1 runs inline.
void detect_lines(int rows, int cols, const fd_lsd_opts &o, const FrameList *frames, int batch, fd_lsd_rect *out,
                  int32_t stride, int32_t *counts, uint8_t *used0, int threads);

// min_region_size (feature_line_detector.cpp:17-20).
uint32_t min_region_size(int rows, int cols, float tol_rad);

}  // namespace fdl
