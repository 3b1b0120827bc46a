// Host stage of fd_lsd_lines (fd_lines.cpp): region growing and rectangle fitting over the GPU's
// compact level-line lists, one frame per worker thread. Pure C++ (no HIP), built with g++ like the
// reference so its float sequence (glibc cosf / sinf / atan2f, no contraction) is the reference's.
#pragma once

#include <stdint.h>

#include <functional>

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

// The seed order computed on the GPU (fd_lsd_lines: k_select_reference in push order): frame f's map
// indices in the reference's sorted order at ord + f * stride, usable when status[f] says the frame was
// resolved. wait() blocks until both are on the host; the workers call it after their first frame's
// setup, so the GPU sort overlaps that work. A frame without a usable order is sorted on the host.
struct SeedOrder {
    const uint32_t *ord;
    int64_t stride;
    const uint32_t *status;
    std::function<void()> wait;
};

// FeatureLineDetector::DetectGoodFeatures (feature_line_detector.cpp:12-54) from the level-line map on,
// for `batch` frames of rows x cols. out: [batch][stride] rectangles (start/end already offset by 0.5,
// :43-44); counts: rectangles found per frame (may exceed stride; only stride are written). used0
// (optional, frame 0's list length): the final is_used flag of each listed pixel of frame 0.
// seeds (optional): the GPU's seed orders. threads <= 1 runs inline.
void detect_lines(int rows, int cols, const fd_lsd_opts &o, const FrameList *frames, int batch, fd_lsd_rect *out,
                  int32_t stride, int32_t *counts, uint8_t *used0, int threads, const SeedOrder *seeds = nullptr);

// min_region_size (feature_line_detector.cpp:17-20).
uint32_t min_region_size(int rows, int cols, float tol_rad);

}  // namespace fdl
