// FeatureLineDetector over libfdhip.so (reference: src/feature_line_detector/feature_line_detector.cpp).
//
// DetectGoodFeatures (:12-54) is one fd_lsd_lines call for the frame (staged on the device once): the
// GPU level-line map in compact form and the library's host region-growing stage (fd_lines.cpp),
// which returns the accepted rectangles (rectangles_, features). The other members the reference
// exposes are materialised on first access, as it leaves them: pixels_ and sorted_pixels_ from a dense
// GPU map of the staged frame (fd_lsd_map: bit-exact norm / validity / angle and the scan-ordered
// valid list, :56-97), with each listed pixel's final is_used flag from fd_lsd_lines_state.
#include "feature_detector/feature_line_detector.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "fd_hip.h"

namespace feature_detector {

FeatureLineDetector::FeatureLineDetector() {
    sorted_pixels_.clear();
    sorted_pixels_.reserve(10000);  // feature_line_detector.cpp:8-9
}

FeatureLineDetector::~FeatureLineDetector() {
    if (ctx_) fd_ctx_destroy(ctx_);
}

void FeatureLineDetector::set_device(int device) {
    if (ctx_ && device != device_) {
        fd_ctx_destroy(ctx_);
        ctx_ = nullptr;
    }
    device_ = device;
}

bool FeatureLineDetector::EnsureContext() {
    if (ctx_) return true;
    if (device_ < 0) {
        const char *e = std::getenv("FD_DEVICE");
        device_ = e ? std::atoi(e) : 0;
    }
    if (fd_ctx_create(device_, &ctx_) != FD_OK) {
        ctx_ = nullptr;
        error_ = "fd_ctx_create failed (no MI355X visible?)";
        std::fprintf(stderr, "[feature_detector] %s\n", error_.c_str());
        return false;
    }
    return true;
}

bool FeatureLineDetector::DetectGoodFeatures(const GrayImage &image, const uint32_t needed_feature_num,
                                             std::vector<Vec4> &features) {
    if (image.data() == nullptr || image.rows() < 2 || image.cols() < 2) return false;  // :14
    if (needed_feature_num == 0) return true;                                           // :15
    if (!EnsureContext()) return false;

    const fd_lsd_opts opts{options_.kMinValidGradientNorm, options_.kMinToleranceAngleResidualInRad,
                           options_.kMinValidLineLengthInPixel, options_.kMaxToleranceInlierRation};
    // Drop the previous call's lazy state first: staging reuses (or reallocates) the context's frame
    // buffer, so a failure below must not leave pixels()/sorted_pixels() pointing at it.
    staged_ = nullptr;
    members_valid_ = true;
    pixels_ = PixelMatrix();
    sorted_pixels_.clear();
    rectangles_.clear();
    const uint8_t *dframe = nullptr;
    if (fd_ctx_stage(ctx_, image.data(), static_cast<int64_t>(image.rows()) * image.cols(), &dframe) != FD_OK) {
        error_ = std::string("fd_ctx_stage: ") + fd_last_error(ctx_);
        std::fprintf(stderr, "[feature_detector] %s\n", error_.c_str());
        return false;
    }
    std::vector<fd_lsd_rect> rects(256);
    int32_t count = 0;
    for (;;) {
        const int rc = fd_lsd_lines(ctx_, dframe, 1, 1, image.rows(), image.cols(), &opts, needed_feature_num,
                                    rects.data(), static_cast<int32_t>(rects.size()), &count, 1);
        if (rc != FD_OK) {
            error_ = std::string("fd_lsd_lines: ") + fd_last_error(ctx_);
            std::fprintf(stderr, "[feature_detector] %s\n", error_.c_str());
            return false;
        }
        if (count <= static_cast<int32_t>(rects.size())) break;
        rects.resize(static_cast<size_t>(count));  // more segments than slots: run again with room for all
    }
    staged_ = dframe;
    last_rows_ = image.rows();
    last_cols_ = image.cols();
    last_min_norm_ = options_.kMinValidGradientNorm;
    members_valid_ = false;

    rectangles_.clear();
    for (int32_t k = 0; k < count; ++k) {
        const fd_lsd_rect &r = rects[static_cast<size_t>(k)];
        RectangleParam p;
        p.start_point = Vec2(r.start[0], r.start[1]);
        p.end_point = Vec2(r.end[0], r.end[1]);
        p.center_point = Vec2(r.center[0], r.center[1]);
        p.length = r.length;
        p.width = r.width;
        p.angle = r.angle;
        p.dir_vector = Vec2(r.dir[0], r.dir[1]);
        p.inlier_ratio = r.inlier_ratio;
        rectangles_.emplace_back(p);
    }
    features.clear();  // :49-53
    for (const auto &rect : rectangles_)
        features.emplace_back(Vec4(rect.start_point.x(), rect.start_point.y(), rect.end_point.x(), rect.end_point.y()));
    return true;
}

void FeatureLineDetector::Materialise() const {
    if (members_valid_) return;
    members_valid_ = true;
    if (!staged_) return;
    if (!ComputeLineLevelAngleMap()) return;
    // is_used as the reference's regions leave it (every listed pixel; unlisted ones are invalid)
    int64_t n = 0;
    fd_lsd_lines_state(ctx_, nullptr, nullptr, nullptr, nullptr, 0, &n);
    std::vector<int32_t> idx(static_cast<size_t>(n));
    std::vector<float> nv(static_cast<size_t>(n)), av(static_cast<size_t>(n));
    std::vector<uint8_t> used(static_cast<size_t>(n));
    if (n > 0) fd_lsd_lines_state(ctx_, idx.data(), nv.data(), av.data(), used.data(), n, &n);
    const int32_t pc = last_cols_ - 1;
    for (int64_t k = 0; k < n; ++k) pixels_(idx[k] / pc, idx[k] % pc).is_used = used[k] != 0;
}

FeatureLineDetector::PixelMatrix &FeatureLineDetector::pixels() {
    Materialise();
    return pixels_;
}
const FeatureLineDetector::PixelMatrix &FeatureLineDetector::pixels() const {
    Materialise();
    return pixels_;
}
std::vector<FeatureLineDetector::PixelParam *> &FeatureLineDetector::sorted_pixels() {
    Materialise();
    return sorted_pixels_;
}
const std::vector<FeatureLineDetector::PixelParam *> &FeatureLineDetector::sorted_pixels() const {
    Materialise();
    return sorted_pixels_;
}

// ComputeLineLevelAngleMap (feature_line_detector.cpp:56-97): map on the GPU (the frame staged by the
// last call), std::sort on the host.
bool FeatureLineDetector::ComputeLineLevelAngleMap() const {
    const int32_t rows = last_rows_, cols = last_cols_;
    const int32_t pr = rows - 1, pc = cols - 1;
    const size_t n = static_cast<size_t>(pr) * pc;
    std::vector<float> norm(n), angle(n);
    std::vector<uint8_t> valid(n);
    std::vector<int32_t> idx(n);
    int64_t count = 0;
    ++map_passes_;
    const int rc = fd_lsd_map(ctx_, staged_, 1, 1, rows, cols, last_min_norm_, norm.data(), angle.data(), valid.data(),
                              idx.data(), static_cast<int64_t>(n), &count, 0);
    if (rc != FD_OK) {
        error_ = std::string("fd_lsd_map: ") + fd_last_error(ctx_);
        std::fprintf(stderr, "[feature_detector] %s\n", error_.c_str());
        return false;
    }
    // Flags describe this call only (the reference carries is_used over between calls on a same-size
    // frame, and never clears sorted_pixels_; a fresh state per call is kept here).
    pixels_ = PixelMatrix();
    pixels_.resize(pr, pc);
    // The bottom-right boundary is invalid; the reference's writes there (:58-69), including its
    // pixels_(0, 1).col quirk (out of bounds when cols == 2: skipped).
    for (int32_t i = 0; i < pr; ++i) {
        pixels_(i, 0).row = i;
        pixels_(i, pc - 1).row = i;
        pixels_(i, pc - 1).col = pc - 1;
    }
    for (int32_t i = 0; i < pc; ++i) {
        if (pc > 1) pixels_(0, 1).col = i;
        pixels_(pr - 1, i).col = i;
        pixels_(pr - 1, i).row = pr - 1;
    }
    for (int32_t col = 1; col < cols - 2; ++col) {  // interior (:71-89)
        for (int32_t row = 1; row < rows - 2; ++row) {
            PixelParam &px = pixels_(row, col);
            const size_t i = static_cast<size_t>(row) * pc + col;
            px.row = row;
            px.col = col;
            px.gradient_norm = norm[i];
            px.is_valid = valid[i] != 0;
            if (px.is_valid) px.line_level_angle = angle[i];
        }
    }
    // sorted_pixels_ in scan order, then the reference's unstable std::sort by norm (:86, :92-94)
    sorted_pixels_.clear();
    for (int64_t k = 0; k < count; ++k) {
        const int32_t i = idx[k];
        sorted_pixels_.emplace_back(&pixels_(i / pc, i % pc));
    }
    std::sort(sorted_pixels_.begin(), sorted_pixels_.end(),
              [](PixelParam *a, PixelParam *b) { return a->gradient_norm > b->gradient_norm; });
    return true;
}

}  // namespace feature_detector
