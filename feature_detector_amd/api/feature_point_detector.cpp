// FeaturePointDetector family over libfdhip.so (include/fd_hip.h). Reference behaviour restated from
// Horizon1026/Feature_Detector src/feature_point_detector/feature_point_detector.cpp (cited per
// function); the per-pixel work, ordering and greedy selection run on the GPU.
#include "feature_detector/feature_point_detector.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "fd_hip.h"

namespace feature_detector {

namespace {

int DefaultDevice() {
    const char *e = std::getenv("FD_DEVICE");
    return e ? std::atoi(e) : 0;
}

// DrawRectangleInMask (feature_point_detector.cpp:76-88): zero the clipped (2d+1)^2 box.
void DrawBox(MatInt &mask, int32_t row, int32_t col, int32_t dist) {
    for (int32_t drow = -dist; drow <= dist; ++drow) {
        for (int32_t dcol = -dist; dcol <= dist; ++dcol) {
            const int32_t r = drow + row, c = dcol + col;
            if (r < 0 || c < 0 || r > mask.rows() - 1 || c > mask.cols() - 1) continue;
            mask(r, c) = 0;
        }
    }
}

}  // namespace

FeaturePointDetector::~FeaturePointDetector() {
    if (ctx_) fd_ctx_destroy(ctx_);
}

void FeaturePointDetector::set_device(int device) {
    if (ctx_ && device != device_) {
        fd_ctx_destroy(ctx_);
        ctx_ = nullptr;
    }
    device_ = device;
}

fd_ctx *FeaturePointDetector::Context() {
    if (!ctx_) {
        if (device_ < 0) device_ = DefaultDevice();
        if (fd_ctx_create(device_, &ctx_) != FD_OK) {
            ctx_ = nullptr;
            error_ = "fd_ctx_create failed (no MI355X visible?)";
        } else {
            // the drop-in reproduces the reference's std::sort order of equal responses (:58-60)
            (void)fd_ctx_set_tie_order(ctx_, FD_TIES_REFERENCE);
        }
    }
    return ctx_;
}

bool FeaturePointDetector::Fail(const std::string &what) {
    error_ = what + (ctx_ ? std::string(": ") + fd_last_error(ctx_) : std::string());
    std::fprintf(stderr, "[feature_detector] %s\n", error_.c_str());
    return false;
}

// DetectGoodFeatures (feature_point_detector.cpp:7-25): the mask state of :12-16 (materialised on
// access), a cleared candidate list (:19), the virtual ComputeCandidates (:20), then SelectGoodFeatures
// (:23, :54-74) on the GPU -- fused with the candidate stage when ComputeCandidates deferred to it.
bool FeaturePointDetector::DetectGoodFeatures(const GrayImage &image, const uint32_t needed_feature_num,
                                              std::vector<Vec2> &features) {
    if (image.data() == nullptr) return false;  // RETURN_FALSE_IF(image.data() == nullptr) (:9)
    fd_ctx *ctx = Context();
    if (!ctx) return Fail("no device context");
    last_prior_ = features;
    last_new_.clear();
    last_rows_ = image.rows();
    last_cols_ = image.cols();
    last_options_ = options_;
    last_reached_need_ = false;
    staged_frame_ = nullptr;
    mask_valid_ = false;
    candidates_.clear();
    candidates_valid_ = true;
    candidates_sorted_ = true;
    fused_kind_ = -1;
    in_detect_ = true;
    const bool ok = ComputeCandidates(image);
    in_detect_ = false;
    if (!ok) return false;  // RETURN_FALSE_IF_FALSE(ComputeCandidates(image)) (:20)
    if (fused_kind_ >= 0) return DetectFused(image, fused_kind_, needed_feature_num, features);
    candidates_sorted_ = false;
    return SelectOwnCandidates(needed_feature_num, features);
}

bool FeaturePointDetector::DeferCandidatesToGpu(int kind) {
    if (!in_detect_) return Fail("DeferCandidatesToGpu outside DetectGoodFeatures");
    fused_kind_ = kind;
    return true;
}

// The built-in detectors: mask, candidates and selection as one fd_points_detect on the staged frame.
bool FeaturePointDetector::DetectFused(const GrayImage &image, int kind, const uint32_t needed_feature_num,
                                       std::vector<Vec2> &features) {
    fd_ctx *ctx = ctx_;
    const int32_t rows = image.rows(), cols = image.cols();
    const uint8_t *dframe = nullptr;
    if (fd_ctx_stage(ctx, image.data(), static_cast<int64_t>(rows) * cols, &dframe) != FD_OK)
        return Fail("staging the image");

    std::vector<float> prior(2 * features.size());
    for (size_t i = 0; i < features.size(); ++i) {
        prior[2 * i] = features[i].x();
        prior[2 * i + 1] = features[i].y();
    }
    const int32_t nprior = static_cast<int32_t>(features.size());
    const fd_point_opts opts{options_.kMinFeatureDistance, options_.kMinValidResponse};
    const int32_t stride = static_cast<int32_t>(std::max<uint32_t>(needed_feature_num, 1u)) + 1;
    std::vector<float> out(2 * static_cast<size_t>(stride));
    int32_t count = 0;
    const int rc = fd_points_detect(ctx, kind, dframe, 1, 1, rows, cols, &opts,
                                    nprior ? prior.data() : nullptr, nprior ? &nprior : nullptr, needed_feature_num,
                                    out.data(), stride, &count, 0);
    if (rc != FD_OK) return Fail("fd_points_detect");

    for (int32_t i = 0; i < count; ++i) {
        features.emplace_back(Vec2(out[2 * i], out[2 * i + 1]));
        last_new_.emplace_back(Vec2(out[2 * i], out[2 * i + 1]));
    }
    staged_frame_ = dframe;
    last_reached_need_ = count > 0 && features.size() >= needed_feature_num;
    candidates_valid_ = false;
    mask_valid_ = false;
    return true;
}

// SelectGoodFeatures (:54-74) over the candidates a subclass pushed (fd_points_select, in the order
// they were pushed).
bool FeaturePointDetector::SelectOwnCandidates(const uint32_t needed_feature_num, std::vector<Vec2> &features) {
    if (candidates_.empty()) return true;  // RETURN_TRUE_IF(candidates_.empty()) (:55)
    const size_t n = candidates_.size();
    std::vector<float> resp(n);
    std::vector<int32_t> xs(n), ys(n);
    for (size_t i = 0; i < n; ++i) {
        resp[i] = candidates_[i].first;
        xs[i] = candidates_[i].second.x();
        ys[i] = candidates_[i].second.y();
    }
    std::vector<float> prior(2 * features.size());
    for (size_t i = 0; i < features.size(); ++i) {
        prior[2 * i] = features[i].x();
        prior[2 * i + 1] = features[i].y();
    }
    const int32_t nprior = static_cast<int32_t>(features.size());
    const fd_point_opts opts{options_.kMinFeatureDistance, options_.kMinValidResponse};
    const int32_t stride = static_cast<int32_t>(std::max<uint32_t>(needed_feature_num, 1u)) + 1;
    std::vector<float> out(2 * static_cast<size_t>(stride));
    const int64_t count_in = static_cast<int64_t>(n);
    int32_t count = 0;
    const int rc = fd_points_select(ctx_, 1, last_rows_, last_cols_, &opts, resp.data(), xs.data(), ys.data(),
                                    &count_in, count_in, 0, nprior ? prior.data() : nullptr,
                                    nprior ? &nprior : nullptr, needed_feature_num, out.data(), stride, &count, 0);
    if (rc != FD_OK) return Fail("fd_points_select");
    for (int32_t i = 0; i < count; ++i) {
        features.emplace_back(Vec2(out[2 * i], out[2 * i + 1]));
        last_new_.emplace_back(Vec2(out[2 * i], out[2 * i + 1]));
    }
    last_reached_need_ = count > 0 && features.size() >= needed_feature_num;
    mask_valid_ = false;
    return true;
}

// candidates() after a fused call: the raster-ordered candidates of the staged frame (the sequence the
// reference's ComputeCandidates pushes), recomputed on the GPU.
bool FeaturePointDetector::FetchCandidates() {
    candidates_.clear();
    if (fused_kind_ < 0 || !staged_frame_ || !ctx_) return false;
    const int64_t cap = static_cast<int64_t>(last_rows_) * last_cols_ / (fused_kind_ == FD_FAST ? 1 : 2) + 16;
    std::vector<float> resp(static_cast<size_t>(cap));
    std::vector<int32_t> xs(static_cast<size_t>(cap)), ys(static_cast<size_t>(cap));
    std::vector<float> prior(2 * last_prior_.size());
    for (size_t i = 0; i < last_prior_.size(); ++i) {
        prior[2 * i] = last_prior_[i].x();
        prior[2 * i + 1] = last_prior_[i].y();
    }
    const int32_t nprior = static_cast<int32_t>(last_prior_.size());
    const fd_point_opts opts{last_options_.kMinFeatureDistance, last_options_.kMinValidResponse};
    int64_t n = 0;
    const int rc = fd_points_candidates(ctx_, fused_kind_, staged_frame_, 1, 1, last_rows_, last_cols_, &opts,
                                        nprior ? prior.data() : nullptr, nprior ? &nprior : nullptr, resp.data(),
                                        xs.data(), ys.data(), cap, &n, nullptr, 0);
    if (rc != FD_OK) return Fail("fd_points_candidates");
    candidates_.reserve(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) candidates_.emplace_back(resp[i], Pixel(xs[i], ys[i]));
    return true;
}

void FeaturePointDetector::Materialise() const {
    auto *self = const_cast<FeaturePointDetector *>(this);
    // The reference leaves candidates_ sorted by its unstable std::sort (:58-60).
    auto sort_ref = [this]() {
        std::sort(candidates_.begin(), candidates_.end(),
                  [](const std::pair<float, Pixel> &a, const std::pair<float, Pixel> &b) { return a.first > b.first; });
    };
    if (!candidates_valid_) {
        candidates_valid_ = true;
        if (self->FetchCandidates()) sort_ref();
    } else if (!candidates_sorted_) {
        candidates_sorted_ = true;
        sort_ref();
    }
    if (!mask_valid_) {
        mask_valid_ = true;
        // mask_ after the call: prior boxes (:12-16, :90-98), then one box per accepted feature except
        // the one whose append reached `need` (the box is drawn after the check, :67-70).
        mask_.setConstant(last_rows_, last_cols_, 1);
        const int32_t d = last_options_.kMinFeatureDistance;
        for (const Vec2 &f : last_prior_) DrawBox(mask_, static_cast<int32_t>(f.y()), static_cast<int32_t>(f.x()), d);
        const size_t drawn = last_new_.size() - (last_reached_need_ ? 1 : 0);
        for (size_t i = 0; i < drawn; ++i)
            DrawBox(mask_, static_cast<int32_t>(last_new_[i].y()), static_cast<int32_t>(last_new_[i].x()), d);
    }
}

std::vector<std::pair<float, Pixel>> &FeaturePointDetector::candidates() {
    Materialise();
    return candidates_;
}
const std::vector<std::pair<float, Pixel>> &FeaturePointDetector::candidates() const {
    Materialise();
    return candidates_;
}
MatInt &FeaturePointDetector::mask() {
    Materialise();
    return mask_;
}
const MatInt &FeaturePointDetector::mask() const {
    Materialise();
    return mask_;
}

// SparsifyFeatures (feature_point_detector.cpp:27-52): host-side grid filter over a feature list.
void FeaturePointDetector::SparsifyFeatures(const std::vector<Vec2> &features, const int32_t image_rows,
                                            const int32_t image_cols, const uint8_t status_need_filter,
                                            const uint8_t status_after_filter, std::vector<uint8_t> &status) {
    if (features.size() != status.size()) status.assign(features.size(), 1);
    const float row_step = image_rows / (options_.kGridFilterRowDivideNumber - 1);  // integer division (:34)
    const float col_step = image_cols / (options_.kGridFilterColDivideNumber - 1);
    mask_.setConstant(options_.kGridFilterRowDivideNumber, options_.kGridFilterColDivideNumber, 1);
    for (size_t i = 0; i < features.size(); ++i) {
        const int32_t row = static_cast<int32_t>(features[i].y() / row_step);
        const int32_t col = static_cast<int32_t>(features[i].x() / col_step);
        if (row < 0 || row > mask_.rows() - 1 || col < 0 || col > mask_.cols() - 1) {
            status[i] = status_after_filter;
            continue;
        }
        if (mask_(row, col) && status[i] == status_need_filter) {
            mask_(row, col) = 0;
        } else if (!mask_(row, col) && status[i] == status_need_filter) {
            status[i] = status_after_filter;
        }
    }
    mask_valid_ = true;  // mask_ now holds the grid mask, as in the reference
}

// The built-in detectors' ComputeCandidates (feature_point_harris_detector.cpp:5-15, shi_tomas :5-15,
// fast :83-98): the whole detection runs fused on the GPU.
bool FeaturePointHarrisDetector::ComputeCandidates(const GrayImage & /*image*/) { return DeferCandidatesToGpu(FD_HARRIS); }
bool FeaturePointShiTomasDetector::ComputeCandidates(const GrayImage & /*image*/) {
    return DeferCandidatesToGpu(FD_SHI_TOMASI);
}
bool FeaturePointFastDetector::ComputeCandidates(const GrayImage & /*image*/) { return DeferCandidatesToGpu(FD_FAST); }

}  // namespace feature_detector
