// Headless restatement of the reference demo test/test_feature_line_detector.cpp:98-129 (LSD with
// default options) against the drop-in API; prints the lines and map statistics as JSON.
//   usage: fd_demo_lines <raw u8 gray file> <rows> <cols> [lines_only]
//   lines_only = 1: the members are not read (map_passes shows that no dense map pass ran)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "feature_detector/feature_line_detector.h"

using namespace feature_detector;

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s <raw u8 file> <rows> <cols>\n", argv[0]);
        return 2;
    }
    const int rows = std::atoi(argv[2]), cols = std::atoi(argv[3]);
    uint8_t *buf = static_cast<uint8_t *>(std::malloc(static_cast<size_t>(rows) * cols));
    FILE *f = std::fopen(argv[1], "rb");
    if (!f || std::fread(buf, 1, static_cast<size_t>(rows) * cols, f) != static_cast<size_t>(rows) * cols) {
        std::fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    std::fclose(f);
    GrayImage image(buf, rows, cols, true);

    FeatureLineDetector detector;  // :100-106
    std::vector<Vec4> features;
    const bool ok = detector.DetectGoodFeatures(image, 200, features);
    if (argc > 4 && std::atoi(argv[4]) != 0) {
        std::printf("{\"ok\": %s, \"map_passes\": %d, \"lines\": [", ok ? "true" : "false", detector.map_passes());
        for (size_t i = 0; i < features.size(); ++i)
            std::printf("%s[%.6f, %.6f, %.6f, %.6f]", i ? ", " : "", features[i][0], features[i][1], features[i][2],
                        features[i][3]);
        std::printf("]}\n");
        return 0;
    }
    size_t n_valid = 0, n_used = 0;
    for (int c = 0; c < detector.pixels().cols(); ++c)
        for (int r = 0; r < detector.pixels().rows(); ++r) {
            n_valid += detector.pixels()(r, c).is_valid;
            n_used += detector.pixels()(r, c).is_used;
        }
    std::printf("{\"ok\": %s, \"n_valid\": %zu, \"n_sorted\": %zu, \"n_used\": %zu, \"map_passes\": %d, \"lines\": [",
                ok ? "true" : "false", n_valid, detector.sorted_pixels().size(), n_used, detector.map_passes());
    for (size_t i = 0; i < features.size(); ++i)
        std::printf("%s[%.6f, %.6f, %.6f, %.6f]", i ? ", " : "", features[i][0], features[i][1], features[i][2],
                    features[i][3]);
    std::printf("]}\n");
    return 0;
}
