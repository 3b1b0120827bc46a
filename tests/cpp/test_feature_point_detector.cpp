// Headless restatement of the reference demo test/test_feature_point_detector.cpp:28-114: the same
// detector calls with the same options, compiled against the drop-in API (include/feature_detector),
// minus the visualisation. Prints one JSON object per test to stdout.
//   usage: fd_demo_points <raw u8 gray file> <rows> <cols> [need]
//          fd_demo_points <image.png> [need]      (LoadImage, as the reference demo does at :104)
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "feature_detector/feature_point_detector.h"
#include "feature_detector/image_io.h"

using namespace feature_detector;

static void Print(const char *test, const FeaturePointDetector &detector, const std::vector<Vec2> &features,
                  size_t n_prior, bool ok) {
    std::printf("{\"test\": \"%s\", \"type\": \"%s\", \"ok\": %s, \"n_candidates\": %zu, \"features\": [", test,
                detector.DetectorTypeName().c_str(), ok ? "true" : "false", detector.candidates().size());
    for (size_t i = n_prior; i < features.size(); ++i)
        std::printf("%s[%.1f, %.1f]", i == n_prior ? "" : ", ", features[i].x(), features[i].y());
    std::printf("], \"top_candidates\": [");
    const auto &c = detector.candidates();
    for (size_t i = 0; i < c.size() && i < 8; ++i)
        std::printf("%s[%.9g, %d, %d]", i ? ", " : "", c[i].first, c[i].second.x(), c[i].second.y());
    std::printf("]}\n");
}

void TestHarrisFeatureDetector(GrayImage &image, int32_t feature_num_need) {  // :28-42
    FeaturePointHarrisDetector detector;
    detector.options().kMinFeatureDistance = 20;
    detector.options().kMinValidResponse = 30.0f;
    std::vector<Vec2> features;
    const bool ok = detector.DetectGoodFeatures(image, feature_num_need, features);
    Print("harris", detector, features, 0, ok);
}

void TestUpdateMaskWithDetectedFeatures(GrayImage &image, int32_t feature_num_need) {  // :44-65
    FeaturePointHarrisDetector detector;
    detector.options().kMinFeatureDistance = 20;
    detector.options().kMinValidResponse = 30.0f;
    std::vector<Vec2> features;
    features.reserve(feature_num_need);
    for (int32_t i = 1; i < 10; ++i)
        for (int32_t j = 1; j < 10; ++j) features.emplace_back(Vec2(i * 15, j * 15));
    const size_t n_prior = features.size();
    const bool ok = detector.DetectGoodFeatures(image, feature_num_need, features);
    Print("harris_prior", detector, features, n_prior, ok);
}

void TestShiTomasFeatureDetector(GrayImage &image, int32_t feature_num_need) {  // :67-81
    FeaturePointShiTomasDetector detector;
    detector.options().kMinFeatureDistance = 20;
    detector.options().kMinValidResponse = 40.0f;
    std::vector<Vec2> features;
    const bool ok = detector.DetectGoodFeatures(image, feature_num_need, features);
    Print("shi_tomasi", detector, features, 0, ok);
}

void TestFastFeatureDetector(GrayImage &image, int32_t feature_num_need) {  // :83-97
    FeaturePointFastDetector detector;
    detector.options().kMinFeatureDistance = 20;
    detector.options().kMinValidResponse = 10.0f;
    std::vector<Vec2> features;
    const bool ok = detector.DetectGoodFeatures(image, feature_num_need, features);
    Print("fast", detector, features, 0, ok);
}

int main(int argc, char **argv) {
    GrayImage image;
    int32_t feature_num_need = 200;  // :101
    const std::string path = argc > 1 ? argv[1] : "";
    if (path.size() > 4 && path.compare(path.size() - 4, 4, ".png") == 0) {
        if (!LoadImage(path, image)) {  // :103-104
            std::fprintf(stderr, "cannot load %s\n", argv[1]);
            return 2;
        }
        if (argc > 2) feature_num_need = std::atoi(argv[2]);
    } else {
        if (argc < 4) {
            std::fprintf(stderr, "usage: %s <raw u8 file> <rows> <cols> [need] | <image.png> [need]\n", argv[0]);
            return 2;
        }
        const int rows = std::atoi(argv[2]), cols = std::atoi(argv[3]);
        if (argc > 4) feature_num_need = std::atoi(argv[4]);
        uint8_t *buf = static_cast<uint8_t *>(std::malloc(static_cast<size_t>(rows) * cols));
        FILE *f = std::fopen(argv[1], "rb");
        if (!f || std::fread(buf, 1, static_cast<size_t>(rows) * cols, f) != static_cast<size_t>(rows) * cols) {
            std::fprintf(stderr, "cannot read %s\n", argv[1]);
            return 2;
        }
        std::fclose(f);
        image.SetImage(buf, rows, cols, true);
    }

    TestFastFeatureDetector(image, feature_num_need);  // :106-109
    TestHarrisFeatureDetector(image, feature_num_need);
    TestShiTomasFeatureDetector(image, feature_num_need);
    TestUpdateMaskWithDetectedFeatures(image, feature_num_need);

    // null image: DetectGoodFeatures returns false (feature_point_detector.cpp:9)
    FeaturePointHarrisDetector detector;
    GrayImage empty;
    std::vector<Vec2> features;
    std::printf("{\"test\": \"null_image\", \"ok\": %s}\n",
                detector.DetectGoodFeatures(empty, 10, features) ? "true" : "false");
    return 0;
}
