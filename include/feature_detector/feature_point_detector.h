// FeaturePointDetector and its Harris / Shi-Tomasi / FAST subclasses: the reference's public API
// (src/feature_point_detector/feature_point_detector.h:12-53 and the subclass headers), backed by the
// MI355X kernels of libfdhip.so through the C ABI in include/fd_hip.h.
//
// DetectGoodFeatures keeps the reference's template method (feature_point_detector.cpp:7-25): mask,
// the pure virtual ComputeCandidates, SelectGoodFeatures. It always calls ComputeCandidates, as the
// reference does (:20). The built-in detectors' ComputeCandidates only marks the call for the fused GPU
// path (DeferCandidatesToGpu), after which mask, candidates and selection run as one fd_points_detect.
// Any other ComputeCandidates -- a direct subclass of FeaturePointDetector, or a subclass of a
// built-in detector that overrides it -- pushes (response, pixel) pairs into candidates(), as the
// reference's subclasses do, and those are selected on the GPU by fd_points_select.
// candidates() and mask() are materialised on first access after a call:
// candidates() holds the candidates sorted with the reference's std::sort comparator
// (feature_point_detector.cpp:58-60), exactly what the reference leaves there (the built-in detectors
// recompute them on the GPU for that). mask() may be read inside ComputeCandidates (prior boxes,
// :12-16); edits to it there are not seen by the selection, which builds the same mask on the GPU.
#ifndef FEATURE_DETECTOR_FEATURE_POINT_DETECTOR_H_
#define FEATURE_DETECTOR_FEATURE_POINT_DETECTOR_H_

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "fd_types.h"

struct fd_ctx;

namespace feature_detector {

/* Class FeaturePointDetector Declaration. */
class FeaturePointDetector {
public:
    struct Options {
        int32_t kMinFeatureDistance = 15;
        int32_t kGridFilterRowDivideNumber = 12;
        int32_t kGridFilterColDivideNumber = 12;
        float kMinValidResponse = 0.1f;
    };

public:
    FeaturePointDetector() = default;
    virtual ~FeaturePointDetector();
    FeaturePointDetector(const FeaturePointDetector &detecor) = delete;

    virtual std::string DetectorTypeName() const { return "None"; }

    bool DetectGoodFeatures(const GrayImage &image, const uint32_t needed_feature_num, std::vector<Vec2> &features);

    void SparsifyFeatures(const std::vector<Vec2> &features, const int32_t image_rows, const int32_t image_cols,
                          const uint8_t status_need_filter, const uint8_t status_after_filter,
                          std::vector<uint8_t> &status);

    // Reference for member variables.
    Options &options() { return options_; }
    std::vector<std::pair<float, Pixel>> &candidates();
    MatInt &mask();
    // Const reference for member variables.
    const Options &options() const { return options_; }
    const std::vector<std::pair<float, Pixel>> &candidates() const;
    const MatInt &mask() const;

    // MI355X extensions: GPU ordinal used by this instance (default: $FD_DEVICE or 0), and the last
    // libfdhip error message.
    void set_device(int device);
    int device() const { return device_; }
    const std::string &last_error() const { return error_; }

protected:
    // For the built-in detectors' ComputeCandidates: instead of pushing candidates, hand the whole
    // call to the fused GPU path for libfdhip detector kind `kind` (FD_HARRIS / FD_SHI_TOMASI /
    // FD_FAST). Valid only inside DetectGoodFeatures; returns true.
    bool DeferCandidatesToGpu(int kind);
    fd_ctx *Context();
    bool Fail(const std::string &what);

private:
    // The ComputeCandidates seam (feature_point_detector.h:44, called at feature_point_detector.cpp:20):
    // push the image's candidates into candidates() (already cleared), or DeferCandidatesToGpu.
    virtual bool ComputeCandidates(const GrayImage &image) = 0;
    bool DetectFused(const GrayImage &image, int kind, uint32_t needed_feature_num, std::vector<Vec2> &features);
    bool SelectOwnCandidates(uint32_t needed_feature_num, std::vector<Vec2> &features);
    bool FetchCandidates();
    void Materialise() const;

private:
    Options options_;
    mutable std::vector<std::pair<float, Pixel>> candidates_;
    mutable MatInt mask_;
    // state of the last DetectGoodFeatures call (for the lazily materialised accessors)
    mutable bool candidates_valid_ = true;
    mutable bool candidates_sorted_ = true;  // own candidates: sorted (:58-60) on first access
    mutable bool mask_valid_ = true;
    bool in_detect_ = false;     // inside DetectGoodFeatures' ComputeCandidates call
    int fused_kind_ = -1;        // kind of the last call's fused GPU path, -1 = own candidates
    const uint8_t *staged_frame_ = nullptr;  // device copy of the last image (owned by the context)
    int32_t last_rows_ = 0, last_cols_ = 0;
    Options last_options_;
    std::vector<Vec2> last_prior_;
    std::vector<Vec2> last_new_;
    bool last_reached_need_ = false;
    fd_ctx *ctx_ = nullptr;
    int device_ = -1;
    std::string error_;
};

/* Class FeaturePointHarrisDetector Declaration. */
class FeaturePointHarrisDetector : public FeaturePointDetector {
public:
    struct SubOptions {
        float kAlpha = 0.04f;
        int32_t kHalfPatchSize = 1;
    };

public:
    FeaturePointHarrisDetector() = default;
    virtual ~FeaturePointHarrisDetector() = default;
    virtual std::string DetectorTypeName() const override { return "Harris"; }

private:
    virtual bool ComputeCandidates(const GrayImage &image) override;

private:
    SubOptions sub_options_;
};

/* Class FeaturePointShiTomasDetector Declaration. */
class FeaturePointShiTomasDetector : public FeaturePointDetector {
public:
    struct SubOptions {
        int32_t kHalfPatchSize = 1;
    };

public:
    FeaturePointShiTomasDetector() = default;
    virtual ~FeaturePointShiTomasDetector() = default;
    virtual std::string DetectorTypeName() const override { return "Shi-Tomas"; }

private:
    virtual bool ComputeCandidates(const GrayImage &image) override;

private:
    SubOptions sub_options_;
};

/* Class FeaturePointFastDetector Declaration. */
class FeaturePointFastDetector : public FeaturePointDetector {
public:
    struct SubOptions {
        int32_t kN = 12;
        uint8_t kMinPixelDiffValue = 15;
    };

public:
    FeaturePointFastDetector() = default;
    virtual ~FeaturePointFastDetector() = default;
    virtual std::string DetectorTypeName() const override { return "Fast"; }

private:
    virtual bool ComputeCandidates(const GrayImage &image) override;

private:
    SubOptions sub_options_;
};

}  // namespace feature_detector

#endif  // FEATURE_DETECTOR_FEATURE_POINT_DETECTOR_H_
