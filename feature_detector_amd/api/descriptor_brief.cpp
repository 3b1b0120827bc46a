// BriefDescriptor over libfdhip.so (fd_brief_compute). Reference: Horizon1026/Feature_Detector
// src/feature_descriptor/descriptor_brief.cpp:8-50 (per keypoint) and descriptor.h:27-40 (the loop);
// every keypoint of an image is described by one kernel launch.
#include "feature_detector/descriptor_brief.h"

#include <cstdio>
#include <cstdlib>

#include "fd_hip.h"

namespace feature_detector {

BriefDescriptor::~BriefDescriptor() {
    if (ctx_) fd_ctx_destroy(ctx_);
}

void BriefDescriptor::set_device(int device) {
    if (ctx_ && device != device_) {
        fd_ctx_destroy(ctx_);
        ctx_ = nullptr;
    }
    device_ = device;
}

fd_ctx *BriefDescriptor::Context() const {
    if (!ctx_) {
        int dev = device_;
        if (dev < 0) {
            const char *e = std::getenv("FD_DEVICE");
            dev = e ? std::atoi(e) : 0;
        }
        if (fd_ctx_create(dev, &ctx_) != FD_OK) {
            ctx_ = nullptr;
            error_ = "fd_ctx_create failed (no MI355X visible?)";
            std::fprintf(stderr, "[feature_detector] %s\n", error_.c_str());
        }
    }
    return ctx_;
}

bool BriefDescriptor::Run(const GrayImage &image, const Vec2 *uv, size_t n, std::vector<BriefType> &out,
                          std::vector<uint8_t> *valid) const {
    fd_ctx *ctx = Context();
    if (!ctx) return false;
    const int32_t length = options_.kLength;
    // descriptor.assign(kLength, 0) (descriptor_brief.cpp:10) for every keypoint first: a failed call
    // leaves all-zero descriptors, as a keypoint outside the border does.
    for (size_t i = 0; i < n; ++i) out[i].assign(length > 0 ? static_cast<size_t>(length) : 0, false);
    if (n == 0 || length <= 0) return true;
    std::vector<float> xy(2 * n);
    for (size_t i = 0; i < n; ++i) {
        xy[2 * i] = uv[i].x();
        xy[2 * i + 1] = uv[i].y();
    }
    const int nw = (length + 31) / 32;
    std::vector<uint32_t> bits(static_cast<size_t>(nw) * n);
    std::vector<uint8_t> ok(n);
    fd_brief_opts o{length, options_.kHalfPatchSize, sampler_};
    const int rc = fd_brief_compute(ctx, image.data(), 0, 1, image.rows(), image.cols(), &o, xy.data(), nullptr,
                                    static_cast<int32_t>(n), bits.data(), ok.data(), 0);
    if (rc != FD_OK) {
        error_ = std::string("fd_brief_compute: ") + fd_last_error(ctx);
        std::fprintf(stderr, "[feature_detector] %s\n", error_.c_str());
        return false;
    }
    for (size_t i = 0; i < n; ++i) {
        const uint32_t *w = bits.data() + i * nw;
        for (int32_t j = 0; j < length; ++j) out[i][j] = ((w[j >> 5] >> (j & 31)) & 1u) != 0;
    }
    if (valid) *valid = ok;
    return true;
}

bool BriefDescriptor::ComputeForAllFeatures(const GrayImage &image, const std::vector<Vec2> &pixel_uv,
                                            std::vector<BriefType> &descriptors) const {
    return Run(image, pixel_uv.data(), pixel_uv.size(), descriptors, nullptr);
}

bool BriefDescriptor::ComputeForOneFeature(const GrayImage &image, const Vec2 &pixel_uv, BriefType &descriptor) const {
    std::vector<BriefType> one(1);
    std::vector<uint8_t> valid;
    const bool ran = Run(image, &pixel_uv, 1, one, &valid);
    descriptor.swap(one[0]);
    return ran && !valid.empty() && valid[0] != 0;
}

}  // namespace feature_detector
