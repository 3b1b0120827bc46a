// FeatureLineDetector (LSD): the reference's public API (src/feature_line_detector/
// feature_line_detector.h:11-79). Segments come from fd_lsd_lines (GPU level-line map, host region
// growing in libfdhip.so); pixels() / sorted_pixels() / rectangles() hold what the reference leaves
// in its members after a call.
#ifndef FEATURE_DETECTOR_FEATURE_LINE_DETECTOR_H_
#define FEATURE_DETECTOR_FEATURE_LINE_DETECTOR_H_

#include <cstdint>
#include <string>
#include <vector>

#include "fd_types.h"

struct fd_ctx;

namespace feature_detector {

class FeatureLineDetector {
public:
    struct PixelParam {
        int32_t row = 0;
        int32_t col = 0;
        float line_level_angle = 0.0f;
        float gradient_norm = 0.0f;
        bool is_valid = false;     // Valid when gradient norm is large enough.
        bool is_used = false;      // Has been used in a region.
        bool is_occupied = false;  // Has been searched when region is growing. It will be cleared later.
    };

    struct RegionParam {
        std::vector<PixelParam *> pixels;
        float angle = 0.0f;
    };

    struct RectangleParam {
        Vec2 start_point = Vec2::Zero();
        Vec2 end_point = Vec2::Zero();
        Vec2 center_point = Vec2::Zero();
        float length = 0.0f;
        float width = 0.0f;
        float angle = 0.0f;
        Vec2 dir_vector = Vec2::Identity();
        float inlier_ratio = 0.0f;
    };

    struct Options {
        float kMinValidGradientNorm = 20.0f;
        float kMinToleranceAngleResidualInRad = 22.5f * kDegToRad;
        float kMinValidLineLengthInPixel = 20.0f;
        float kMaxToleranceInlierRation = 0.6f;
    };

    // Column-major (rows x cols) matrix of PixelParam, as the reference's
    // Eigen::Matrix<PixelParam, Dynamic, Dynamic> (feature_line_detector.h:74).
    class PixelMatrix {
    public:
        void resize(int rows, int cols) {
            if (rows != rows_ || cols != cols_) {  // Eigen keeps the data on a same-size resize
                rows_ = rows;
                cols_ = cols;
                buf_.assign(static_cast<size_t>(rows) * static_cast<size_t>(cols), PixelParam());
            }
        }
        PixelParam &operator()(int r, int c) { return buf_[static_cast<size_t>(c) * rows_ + r]; }
        const PixelParam &operator()(int r, int c) const { return buf_[static_cast<size_t>(c) * rows_ + r]; }
        int rows() const { return rows_; }
        int cols() const { return cols_; }

    private:
        int rows_ = 0, cols_ = 0;
        std::vector<PixelParam> buf_;
    };

public:
    FeatureLineDetector();
    virtual ~FeatureLineDetector();

    bool DetectGoodFeatures(const GrayImage &image, const uint32_t needed_feature_num, std::vector<Vec4> &features);

    // Reference for member variables. pixels() and sorted_pixels() are materialised on first access
    // after a call (one dense GPU map of the frame staged by that call): DetectGoodFeatures itself is a
    // single fd_lsd_lines pass.
    Options &options() { return options_; }
    PixelMatrix &pixels();
    std::vector<PixelParam *> &sorted_pixels();
    std::vector<RectangleParam> &rectangles() { return rectangles_; }

    // Const reference for member variables.
    const Options &options() const { return options_; }
    const PixelMatrix &pixels() const;
    const std::vector<PixelParam *> &sorted_pixels() const;
    const std::vector<RectangleParam> &rectangles() const { return rectangles_; }

    // MI355X extensions: GPU ordinal, last libfdhip error, and the number of dense map passes run so
    // far to materialise pixels() / sorted_pixels().
    void set_device(int device);
    const std::string &last_error() const { return error_; }
    int map_passes() const { return map_passes_; }

private:
    bool EnsureContext();
    // pixels_ / sorted_pixels_ as the reference leaves them (:56-97), from the GPU level-line map of
    // the frame staged by the last call, with each listed pixel's final is_used flag
    bool ComputeLineLevelAngleMap() const;
    void Materialise() const;

private:
    Options options_;

    mutable PixelMatrix pixels_;
    mutable std::vector<PixelParam *> sorted_pixels_;
    std::vector<RectangleParam> rectangles_;
    // state of the last call, for the lazily materialised members
    mutable bool members_valid_ = true;
    const uint8_t *staged_ = nullptr;  // device copy of the last frame (owned by the context)
    int32_t last_rows_ = 0, last_cols_ = 0;
    float last_min_norm_ = 0.0f;
    mutable int map_passes_ = 0;

    fd_ctx *ctx_ = nullptr;
    int device_ = -1;
    mutable std::string error_;
};

}  // namespace feature_detector

#endif  // FEATURE_DETECTOR_FEATURE_LINE_DETECTOR_H_
