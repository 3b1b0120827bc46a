// FeaturePointDetector::SparsifyFeatures (reference feature_point_detector.cpp:27-52) through the
// drop-in API: host-only (no GPU call), so it runs in the CPU test suite against the oracle.
//   usage: fd_demo_sparsify <rows> <cols> <grid_rows> <grid_cols> <need_filter> <after_filter>
//   stdin: n, then n lines "x y status" (status -1: pass a status vector of another size, which the
//   function resets to ones, :29-31). Prints {"status": [...], "mask": [...]} (mask row-major).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "feature_detector/feature_point_detector.h"

using namespace feature_detector;

int main(int argc, char **argv) {
    if (argc != 7) return 2;
    const int rows = std::atoi(argv[1]), cols = std::atoi(argv[2]);
    FeaturePointHarrisDetector detector;
    detector.options().kGridFilterRowDivideNumber = std::atoi(argv[3]);
    detector.options().kGridFilterColDivideNumber = std::atoi(argv[4]);
    const uint8_t need = static_cast<uint8_t>(std::atoi(argv[5])), after = static_cast<uint8_t>(std::atoi(argv[6]));
    int n = 0;
    if (std::scanf("%d", &n) != 1) return 2;
    std::vector<Vec2> features;
    std::vector<uint8_t> status;
    bool resize = false;
    for (int i = 0; i < n; ++i) {
        float x, y;
        int s;
        if (std::scanf("%f %f %d", &x, &y, &s) != 3) return 2;
        features.emplace_back(Vec2(x, y));
        if (s < 0) resize = true;
        status.push_back(static_cast<uint8_t>(s < 0 ? 0 : s));
    }
    if (resize) status.push_back(0);  // size mismatch -> reset to ones inside the call
    detector.SparsifyFeatures(features, rows, cols, need, after, status);
    std::printf("{\"status\": [");
    for (size_t i = 0; i < status.size(); ++i) std::printf("%s%d", i ? ", " : "", status[i]);
    std::printf("], \"mask\": [");
    const MatInt &m = detector.mask();
    for (int r = 0; r < m.rows(); ++r)
        for (int c = 0; c < m.cols(); ++c) std::printf("%s%d", (r || c) ? ", " : "", m(r, c));
    std::printf("]}\n");
    return 0;
}
