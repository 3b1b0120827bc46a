// Frame loading for the drop-in API: what the reference's demos get from Visualizor2D::LoadImage
// (test/test_feature_point_detector.cpp:104; Visualizor2D is un-vendored). PNG only (8-bit gray,
// gray+alpha, RGB, RGBA, no interlace) through libfdhip's fd_png_decode; colour becomes gray with the
// BT.601 fixed-point rule of include/fd_hip.h (the reference's conversion is parity-unpinned).
#ifndef FEATURE_DETECTOR_IMAGE_IO_H_
#define FEATURE_DETECTOR_IMAGE_IO_H_

#include <string>

#include "fd_types.h"

namespace feature_detector {

// Loads `path` into `image` (which then owns a malloc'ed buffer). Returns false on a read or decode error.
bool LoadImage(const std::string &path, GrayImage &image);

}  // namespace feature_detector

#endif  // FEATURE_DETECTOR_IMAGE_IO_H_
