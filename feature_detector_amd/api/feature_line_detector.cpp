// FeatureLineDetector over libfdhip.so. The level-line map (feature_line_detector.cpp:56-97) comes
// from the GPU (fd_lsd_map: bit-exact norm / validity / angle and the scan-ordered valid list); the
// sort of sorted_pixels_, region growing and rectangle fitting (feature_line_detector.cpp:12-54,
// 99-228) run on the host in the reference's order. Unpinned dependencies (un-vendored Slam_Utility):
// CircularBuffer overflow policy and Utility::AngleDiffInRad -- see DESIGN.md.
#include "feature_detector/feature_line_detector.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "fd_hip.h"

namespace feature_detector {

namespace {

// Utility::AngleDiffInRad (slam_basic_math.h, un-vendored): a - b wrapped into [-pi, pi].
float AngleDiffInRad(float a, float b) {
    float diff = a - b;
    while (diff > kPai) diff -= k2Pai;
    while (diff < -kPai) diff += k2Pai;
    return diff;
}

}  // namespace

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

// DetectGoodFeatures (feature_line_detector.cpp:12-54).
bool FeatureLineDetector::DetectGoodFeatures(const GrayImage &image, const uint32_t needed_feature_num,
                                             std::vector<Vec4> &features) {
    if (image.data() == nullptr || image.rows() < 2 || image.cols() < 2) return false;  // :14
    if (needed_feature_num == 0) return true;                                           // :15

    // Minimal number of pixels in a meaningful region (:17-20).
    const float p = options_.kMinToleranceAngleResidualInRad / kPai;
    const float log_NT = 5.0f * (std::log10(double(image.cols())) + std::log10(double(image.rows()))) / 2.0f +
                         std::log10(11.0f);
    const uint32_t min_region_size = static_cast<uint32_t>(-log_NT / std::log10(p));

    if (!ComputeLineLevelAngleMap(image)) return false;

    RegionParam region;
    rectangles_.clear();
    for (const auto &sorted_pixel : sorted_pixels_) {  // :27-46
        if (!sorted_pixel->is_valid || sorted_pixel->is_used) continue;
        GrowRegion(*sorted_pixel, region);
        if (region.pixels.size() < min_region_size) {
            for (auto &pixel : region.pixels) pixel->is_used = false;
            continue;
        }
        RectangleParam rectangle = ConvertRegionToRectangle(region);
        if (rectangle.length < options_.kMinValidLineLengthInPixel ||
            rectangle.inlier_ratio < options_.kMaxToleranceInlierRation)
            continue;
        rectangle.start_point += Vec2::Constant(0.5f);  // :41-42
        rectangle.end_point += Vec2::Constant(0.5f);
        rectangles_.emplace_back(rectangle);
    }

    features.clear();  // :49
    for (const auto &rect : rectangles_)
        features.emplace_back(Vec4(rect.start_point.x(), rect.start_point.y(), rect.end_point.x(), rect.end_point.y()));
    return true;
}

// ComputeLineLevelAngleMap (feature_line_detector.cpp:56-97): map on the GPU, std::sort on the host.
bool FeatureLineDetector::ComputeLineLevelAngleMap(const GrayImage &image) {
    if (!ctx_) {
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
    }
    const int32_t rows = image.rows(), cols = image.cols();
    const int32_t pr = rows - 1, pc = cols - 1;
    const size_t n = static_cast<size_t>(pr) * pc;
    std::vector<float> norm(n), angle(n);
    std::vector<uint8_t> valid(n);
    std::vector<int32_t> idx(n);
    int64_t count = 0;
    const int rc = fd_lsd_map(ctx_, image.data(), 0, 1, rows, cols, options_.kMinValidGradientNorm, norm.data(),
                              angle.data(), valid.data(), idx.data(), static_cast<int64_t>(n), &count, 0);
    if (rc != FD_OK) {
        error_ = std::string("fd_lsd_map: ") + fd_last_error(ctx_);
        std::fprintf(stderr, "[feature_detector] %s\n", error_.c_str());
        return false;
    }

    // The bottom-right boundary is invalid; these writes restate :58-69 verbatim in effect (including
    // its pixels_(0, 1).col quirk).
    pixels_.resize(pr, pc);
    for (int32_t i = 0; i < pixels_.rows(); ++i) {
        pixels_(i, 0).row = i;
        pixels_(i, pixels_.cols() - 1).row = i;
        pixels_(i, pixels_.cols() - 1).col = pixels_.cols() - 1;
    }
    for (int32_t i = 0; i < pixels_.cols(); ++i) {
        pixels_(0, 1).col = i;
        pixels_(pixels_.rows() - 1, i).col = i;
        pixels_(pixels_.rows() - 1, i).row = pixels_.rows() - 1;
    }
    // Interior (:71-89): every scanned pixel gets row/col/norm/valid; the angle only where valid.
    for (int32_t col = 1; col < cols - 2; ++col) {
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
    // sorted_pixels_ in scan order, then the reference's unstable std::sort by norm (:86, :92-94).
    // (The reference never clears sorted_pixels_ between calls; a fresh list per call is kept here.)
    sorted_pixels_.clear();
    for (int64_t k = 0; k < count; ++k) {
        const int32_t i = idx[k];
        sorted_pixels_.emplace_back(&pixels_(i / pc, i % pc));
    }
    std::sort(sorted_pixels_.begin(), sorted_pixels_.end(),
              [](PixelParam *a, PixelParam *b) { return a->gradient_norm > b->gradient_norm; });
    return true;
}

// GrowRegion (feature_line_detector.cpp:99-154).
void FeatureLineDetector::GrowRegion(PixelParam &seed_pixel, RegionParam &region) {
    candidates_.Clear();
    visited_pixels_.Clear();
    visited_pixels_.PushBack(&seed_pixel);
    seed_pixel.is_occupied = true;

    region.pixels.clear();
    region.angle = seed_pixel.line_level_angle;
    float sum_dx = std::cos(seed_pixel.line_level_angle);
    float sum_dy = std::sin(seed_pixel.line_level_angle);

    auto add_neighbours = [&](const PixelParam &p) {
        TryToAddPixelIntoCandidates(pixels_(p.row - 1, p.col - 1));
        TryToAddPixelIntoCandidates(pixels_(p.row - 1, p.col));
        TryToAddPixelIntoCandidates(pixels_(p.row - 1, p.col + 1));
        TryToAddPixelIntoCandidates(pixels_(p.row, p.col - 1));
        TryToAddPixelIntoCandidates(pixels_(p.row, p.col + 1));
        TryToAddPixelIntoCandidates(pixels_(p.row + 1, p.col - 1));
        TryToAddPixelIntoCandidates(pixels_(p.row + 1, p.col));
        TryToAddPixelIntoCandidates(pixels_(p.row + 1, p.col + 1));
    };
    add_neighbours(seed_pixel);

    while (!candidates_.Empty()) {
        PixelParam *pixel_ptr = candidates_.Front();
        candidates_.PopFront();
        visited_pixels_.PushBack(pixel_ptr);
        const float angle_residual = AngleDiffInRad(region.angle, pixel_ptr->line_level_angle);
        if (std::fabs(angle_residual) > options_.kMinToleranceAngleResidualInRad) continue;
        sum_dx += std::cos(pixel_ptr->line_level_angle);
        sum_dy += std::sin(pixel_ptr->line_level_angle);
        region.angle = std::atan2(sum_dy, sum_dx);
        region.pixels.emplace_back(pixel_ptr);
        pixel_ptr->is_used = true;
        add_neighbours(*pixel_ptr);
    }

    while (!visited_pixels_.Empty()) {  // clear the occupied flags (:150-153)
        visited_pixels_.Front()->is_occupied = false;
        visited_pixels_.PopFront();
    }
}

// TryToAddPixelIntoCandidates (feature_line_detector.cpp:156-161).
void FeatureLineDetector::TryToAddPixelIntoCandidates(PixelParam &neighbour) {
    if (!neighbour.is_occupied && !neighbour.is_used && neighbour.is_valid) {
        neighbour.is_occupied = true;
        candidates_.PushBack(&neighbour);
    }
}

// ConvertRegionToRectangle (feature_line_detector.cpp:163-228).
FeatureLineDetector::RectangleParam FeatureLineDetector::ConvertRegionToRectangle(const RegionParam &region) {
    RectangleParam rect;
    float sum_weight = 0.0f;
    for (const auto &pixel : region.pixels) {
        rect.center_point.x() += static_cast<float>(pixel->col) * pixel->gradient_norm;
        rect.center_point.y() += static_cast<float>(pixel->row) * pixel->gradient_norm;
        sum_weight += pixel->gradient_norm;
    }
    if (sum_weight == 0) return rect;
    rect.center_point /= sum_weight;

    float Ixx = 0.0f, Iyy = 0.0f, Ixy = 0.0f;
    for (const auto &pixel : region.pixels) {
        const float dx = pixel->col - rect.center_point.x();
        const float dy = pixel->row - rect.center_point.y();
        Ixx += dy * dy * pixel->gradient_norm;
        Iyy += dx * dx * pixel->gradient_norm;
        Ixy -= dx * dy * pixel->gradient_norm;
    }
    if (Ixx == 0 || Iyy == 0 || Ixy == 0) return rect;
    const float smallest_eigen_value = 0.5f * (Ixx + Iyy - std::sqrt((Ixx - Iyy) * (Ixx - Iyy) + 4.0f * Ixy * Ixy));
    rect.angle = std::fabs(Ixx) > std::fabs(Iyy) ? std::atan2(smallest_eigen_value - Ixx, Ixy)
                                                 : std::atan2(Ixy, smallest_eigen_value - Iyy);
    if (std::fabs(AngleDiffInRad(rect.angle, region.angle)) > options_.kMinToleranceAngleResidualInRad) {
        rect.angle += kPai;
        if (rect.angle >= kPai) rect.angle -= k2Pai;
    }
    rect.dir_vector = Vec2(std::cos(rect.angle), std::sin(rect.angle));

    Vec2 length_range = Vec2::Zero();
    Vec2 width_range = Vec2::Zero();
    for (const auto &pixel : region.pixels) {
        const float region_dx = pixel->col - rect.center_point.x();
        const float region_dy = pixel->row - rect.center_point.y();
        const float length = region_dx * rect.dir_vector.x() + region_dy * rect.dir_vector.y();
        const float width = -region_dx * rect.dir_vector.y() + region_dy * rect.dir_vector.x();
        length_range(0) = std::min(length_range(0), length);
        length_range(1) = std::max(length_range(1), length);
        width_range(0) = std::min(width_range(0), width);
        width_range(1) = std::max(width_range(1), width);
    }

    rect.start_point = rect.center_point + rect.dir_vector * length_range(0);
    rect.end_point = rect.center_point + rect.dir_vector * length_range(1);
    rect.length = length_range(1) - length_range(0);
    rect.width = width_range(1) - width_range(0);
    rect.length = std::max(rect.length, 1.0f);
    rect.width = std::max(rect.width, 1.0f);
    const float area_size = (length_range(1) - length_range(0)) * rect.width;
    rect.inlier_ratio = static_cast<float>(region.pixels.size()) / area_size;
    return rect;
}

}  // namespace feature_detector
