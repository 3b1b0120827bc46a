// A FeaturePointDetector subclass with its own ComputeCandidates (the reference's extension point,
// feature_point_detector.h:44): the drop-in base class calls it from DetectGoodFeatures and selects
// its candidates on the GPU (fd_points_select). The candidates here are integer gradient magnitudes
// (many equal responses, so the reference's std::sort order of the pushed sequence decides).
//   usage: fd_demo_custom <raw u8 gray file> <rows> <cols> <order> <dist> <need> [prior] [base]
//     order: raster | reverse | twice (every candidate pushed twice, the copy right after it)
//     prior: 1 = the demo's 9x9 lattice of prior features (test_feature_point_detector.cpp:52-55)
//     base:  plain (default: derives from FeaturePointDetector) | harris (derives from
//            FeaturePointHarrisDetector and overrides only ComputeCandidates, the NVI extension point of
//            feature_point_harris_detector.h:24: its override must be the one that runs)
// Prints one JSON object: ok, the new features, the candidate count and the first 64 of candidates().
#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#include "feature_detector/feature_point_detector.h"

using namespace feature_detector;

// as in the reference, the base class is abstract (pure virtual ComputeCandidates, feature_point_detector.h:44)
static_assert(std::is_abstract<FeaturePointDetector>::value, "FeaturePointDetector must stay abstract");

template <typename Base>
class FeaturePointGradientDetector : public Base {
public:
    explicit FeaturePointGradientDetector(std::string order) : order_(std::move(order)) {}
    std::string DetectorTypeName() const override { return "Gradient"; }
    int calls = 0;

private:
    bool ComputeCandidates(const GrayImage &image) override {
        ++calls;
        const int32_t rows = image.rows(), cols = image.cols();
        const uint8_t *p = image.data();
        // the prior mask is readable here, as in the reference (mask_ is set before :20)
        const MatInt &m = this->mask();
        if (m.rows() != rows || m.cols() != cols) return false;
        std::vector<std::pair<float, Pixel>> found;
        for (int32_t r = 1; r < rows - 1; ++r) {
            for (int32_t c = 1; c < cols - 1; ++c) {
                const int gx = std::abs(p[r * cols + c + 1] - p[r * cols + c - 1]);
                const int gy = std::abs(p[(r + 1) * cols + c] - p[(r - 1) * cols + c]);
                const float v = static_cast<float>(gx + gy);
                if (v > this->options().kMinValidResponse) found.emplace_back(v, Pixel(c, r));
            }
        }
        auto &out = this->candidates();
        if (order_ == "reverse") {
            for (auto it = found.rbegin(); it != found.rend(); ++it) out.emplace_back(*it);
        } else {
            for (const auto &e : found) {
                out.emplace_back(e);
                if (order_ == "twice") out.emplace_back(e);
            }
        }
        return true;
    }

    std::string order_;
};

template <typename Base>
int Run(const GrayImage &image, const char *order, int dist, int need, bool prior) {
    FeaturePointGradientDetector<Base> detector(order);
    detector.options().kMinFeatureDistance = dist;
    detector.options().kMinValidResponse = 40.0f;
    std::vector<Vec2> features;
    if (prior)
        for (int32_t i = 1; i < 10; ++i)
            for (int32_t j = 1; j < 10; ++j) features.emplace_back(Vec2(i * 15, j * 15));
    const size_t n_prior = features.size();
    const bool ok = detector.DetectGoodFeatures(image, static_cast<uint32_t>(need), features);
    std::printf("{\"ok\": %s, \"calls\": %d, \"n_candidates\": %zu, \"features\": [", ok ? "true" : "false",
                detector.calls, detector.candidates().size());
    for (size_t i = n_prior; i < features.size(); ++i)
        std::printf("%s[%.1f, %.1f]", i == n_prior ? "" : ", ", features[i].x(), features[i].y());
    std::printf("], \"top_candidates\": [");
    const auto &c = detector.candidates();
    for (size_t i = 0; i < c.size() && i < 64; ++i)
        std::printf("%s[%.9g, %d, %d]", i ? ", " : "", c[i].first, c[i].second.x(), c[i].second.y());
    long zeros = 0;
    const MatInt &m = detector.mask();
    for (size_t i = 0; i < m.size(); ++i) zeros += m.data()[i] == 0;
    std::printf("], \"mask_zeros\": %ld}\n", zeros);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 7) {
        std::fprintf(stderr, "usage: %s <raw u8 file> <rows> <cols> <order> <dist> <need> [prior] [plain|harris]\n", argv[0]);
        return 2;
    }
    const int rows = std::atoi(argv[2]), cols = std::atoi(argv[3]);
    const int dist = std::atoi(argv[5]), need = std::atoi(argv[6]);
    const bool prior = argc > 7 && std::atoi(argv[7]) != 0;
    std::vector<uint8_t> buf(static_cast<size_t>(rows) * cols);
    FILE *f = std::fopen(argv[1], "rb");
    if (!f || std::fread(buf.data(), 1, buf.size(), f) != buf.size()) {
        std::fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    std::fclose(f);
    GrayImage image;
    image.SetImage(buf.data(), rows, cols, false);

    const bool harris = argc > 8 && std::string(argv[8]) == "harris";
    return harris ? Run<FeaturePointHarrisDetector>(image, argv[4], dist, need, prior)
                  : Run<FeaturePointDetector>(image, argv[4], dist, need, prior);
}
