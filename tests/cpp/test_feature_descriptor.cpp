// Headless restatement of the reference demo test/test_feature_descriptor.cpp:16-72: Harris detection
// (kMinFeatureDistance 20, kMinValidResponse 20, need 10) then BriefDescriptor with kLength 128 and
// kHalfPatchSize 8, compiled against the drop-in API, minus the visualisation. Prints JSON lines.
//   usage: fd_demo_descriptor <raw u8 gray file> <rows> <cols> [sampler: 0 bilinear, 1 truncate]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "feature_detector/descriptor_brief.h"
#include "feature_detector/feature_point_detector.h"

using namespace feature_detector;

std::vector<Vec2> TestHarrisFeatureDetector(const GrayImage &image, const int32_t feature_num_need) {  // :16-35
    FeaturePointHarrisDetector detector;
    detector.options().kMinFeatureDistance = 20;
    detector.options().kMinValidResponse = 20.0f;
    std::vector<Vec2> features;
    const bool ok = detector.DetectGoodFeatures(image, feature_num_need, features);
    std::printf("{\"test\": \"harris\", \"ok\": %s, \"features\": [", ok ? "true" : "false");
    for (size_t i = 0; i < features.size(); ++i)
        std::printf("%s[%.1f, %.1f]", i ? ", " : "", features[i].x(), features[i].y());
    std::printf("]}\n");
    return features;
}

void TestBriefDescriptor(const GrayImage &image, const std::vector<Vec2> &features, int sampler) {  // :37-57
    BriefDescriptor descriptor;
    descriptor.options().kLength = 128;
    descriptor.options().kHalfPatchSize = 8;
    descriptor.set_sampler(sampler);
    std::vector<BriefType> descriptors;
    const bool ok = descriptor.Compute(image, features, descriptors);
    // the std::vector<Vec> overload (descriptor.h:42-62): bits as +1 / -1 floats
    std::vector<Vec> as_float;
    const bool ok_f = descriptor.Compute(image, features, as_float);
    bool float_match = ok_f && as_float.size() == descriptors.size();
    for (size_t i = 0; float_match && i < descriptors.size(); ++i) {
        float_match = as_float[i].size() == static_cast<int>(descriptors[i].size());
        for (size_t j = 0; float_match && j < descriptors[i].size(); ++j)
            float_match = as_float[i][static_cast<int>(j)] == (descriptors[i][j] ? 1.0f : -1.0f);
    }
    std::printf("{\"test\": \"brief\", \"ok\": %s, \"float_overload_ok\": %s, \"descriptors\": [", ok ? "true" : "false",
                float_match ? "true" : "false");
    for (size_t i = 0; i < descriptors.size(); ++i) {
        std::printf("%s\"", i ? ", " : "");
        for (const bool bit : descriptors[i]) std::printf("%d", bit ? 1 : 0);  // :50-55
        std::printf("\"");
    }
    std::printf("]}\n");
    // Compute's false cases (descriptor.h:29): no keypoints, no image
    std::vector<BriefType> none;
    GrayImage empty;
    std::printf("{\"test\": \"brief_false_cases\", \"empty_uv\": %s, \"null_image\": %s}\n",
                descriptor.Compute(image, std::vector<Vec2>{}, none) ? "true" : "false",
                descriptor.Compute(empty, features, none) ? "true" : "false");
}

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s <raw u8 file> <rows> <cols> [sampler]\n", argv[0]);
        return 2;
    }
    const int rows = std::atoi(argv[2]), cols = std::atoi(argv[3]);
    const int sampler = argc > 4 ? std::atoi(argv[4]) : 0;
    uint8_t *buf = static_cast<uint8_t *>(std::malloc(static_cast<size_t>(rows) * cols));
    FILE *f = std::fopen(argv[1], "rb");
    if (!f || std::fread(buf, 1, static_cast<size_t>(rows) * cols, f) != static_cast<size_t>(rows) * cols) {
        std::fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    std::fclose(f);
    GrayImage image(buf, rows, cols, true);
    const int32_t feature_num_need = 10;  // :63
    const std::vector<Vec2> features = TestHarrisFeatureDetector(image, feature_num_need);
    TestBriefDescriptor(image, features, sampler);
    return 0;
}
