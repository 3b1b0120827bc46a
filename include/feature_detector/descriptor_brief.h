// BriefDescriptor: the reference's steered BRIEF (src/feature_descriptor/descriptor_brief.h:9-37,
// descriptor_brief.cpp:8-50) over the MI355X kernel of libfdhip.so (fd_brief_compute).
//
// MI355X extensions: the float-coordinate sampler (the reference's comes from the un-vendored
// Slam_Utility GrayImage; FD_SAMPLE_BILINEAR by default, FD_SAMPLE_TRUNCATE selectable, see
// DESIGN.md), the GPU ordinal, and the last libfdhip error.
#ifndef FEATURE_DETECTOR_DESCRIPTOR_BRIEF_H_
#define FEATURE_DETECTOR_DESCRIPTOR_BRIEF_H_

#include <cstdint>
#include <string>
#include <vector>

#include "descriptor.h"

struct fd_ctx;

namespace feature_detector {

using BriefType = std::vector<bool>;

/* Class BriefDescriptor Declaration. */
class BriefDescriptor : public Descriptor<BriefType> {
public:
    struct Options {
        int32_t kLength = 256;
        int32_t kHalfPatchSize = 8;
    };

public:
    BriefDescriptor() : Descriptor<BriefType>() {}
    virtual ~BriefDescriptor();
    BriefDescriptor(const BriefDescriptor &) = delete;
    BriefDescriptor &operator=(const BriefDescriptor &) = delete;

    // Reference for member variables.
    Options &options() { return options_; }
    const Options &options() const { return options_; }

    void set_sampler(int sampler) { sampler_ = sampler; }
    int sampler() const { return sampler_; }
    void set_device(int device);
    int device() const { return device_; }
    const std::string &last_error() const { return error_; }

protected:
    virtual bool ComputeForAllFeatures(const GrayImage &image, const std::vector<Vec2> &pixel_uv,
                                       std::vector<BriefType> &descriptors) const override;

private:
    virtual bool ComputeForOneFeature(const GrayImage &image, const Vec2 &pixel_uv, BriefType &descriptor) const override;
    bool Run(const GrayImage &image, const Vec2 *uv, size_t n, std::vector<BriefType> &out,
             std::vector<uint8_t> *valid) const;
    fd_ctx *Context() const;

private:
    Options options_;
    int sampler_ = 0;  // FD_SAMPLE_BILINEAR
    mutable fd_ctx *ctx_ = nullptr;
    int device_ = -1;
    mutable std::string error_;
};

}  // namespace feature_detector

#endif  // FEATURE_DETECTOR_DESCRIPTOR_BRIEF_H_
