// Descriptor<DescriptorType>: the reference's generic descriptor interface
// (src/feature_descriptor/descriptor.h:12-62), with one addition for the GPU: a batch seam.
//
// The reference's Compute loops ComputeForOneFeature over the keypoints (descriptor.h:35-38). Here
// Compute calls ComputeForAllFeatures, whose default is that same loop; BriefDescriptor overrides it
// with one fd_brief_compute call per image (every keypoint in one kernel launch).
#ifndef FEATURE_DETECTOR_DESCRIPTOR_H_
#define FEATURE_DETECTOR_DESCRIPTOR_H_

#include <cstdint>
#include <type_traits>
#include <vector>

#include "fd_types.h"

namespace feature_detector {

/* Class Descriptor Declaration. */
template <typename DescriptorType>
class Descriptor {
public:
    Descriptor() = default;
    virtual ~Descriptor() = default;
    bool Compute(const GrayImage &image, const std::vector<Vec2> &pixel_uv, std::vector<DescriptorType> &descriptors) const;
    bool Compute(const GrayImage &image, const std::vector<Vec2> &pixel_uv, std::vector<Vec> &descriptors) const;

protected:
    // Batch seam (MI355X addition): descriptors already has pixel_uv.size() entries.
    virtual bool ComputeForAllFeatures(const GrayImage &image, const std::vector<Vec2> &pixel_uv,
                                       std::vector<DescriptorType> &descriptors) const {
        for (size_t i = 0; i < descriptors.size(); ++i) ComputeForOneFeature(image, pixel_uv[i], descriptors[i]);
        return true;
    }

private:
    virtual bool ComputeForOneFeature(const GrayImage &image, const Vec2 &pixel_uv, DescriptorType &descriptors) const = 0;
};

/* Class Descriptor Definition. */
// descriptor.h:27-40: false on no keypoints or no image; otherwise every keypoint gets a descriptor
// (ComputeForOneFeature's per-keypoint result is not reported, as in the reference).
template <typename DescriptorType>
bool Descriptor<DescriptorType>::Compute(const GrayImage &image, const std::vector<Vec2> &pixel_uv,
                                         std::vector<DescriptorType> &descriptors) const {
    if (pixel_uv.empty() || image.data() == nullptr) return false;
    if (descriptors.size() != pixel_uv.size()) descriptors.resize(pixel_uv.size());
    return ComputeForAllFeatures(image, pixel_uv, descriptors);
}

// descriptor.h:42-62: std::vector<bool> bits become +1.0f / -1.0f, other element types are cast.
template <typename DescriptorType>
bool Descriptor<DescriptorType>::Compute(const GrayImage &image, const std::vector<Vec2> &pixel_uv,
                                         std::vector<Vec> &descriptors) const {
    std::vector<DescriptorType> temp_descriptors;
    if (!Compute(image, pixel_uv, temp_descriptors)) return false;
    descriptors.resize(temp_descriptors.size());
    for (size_t i = 0; i < temp_descriptors.size(); ++i) {
        Vec &descriptor = descriptors[i];
        const auto &temp_descriptor = temp_descriptors[i];
        descriptor.setZero(static_cast<int>(temp_descriptor.size()), 1);
        for (size_t j = 0; j < temp_descriptor.size(); ++j) {
            if constexpr (std::is_same_v<DescriptorType, std::vector<bool>>) {
                descriptor[static_cast<int>(j)] = temp_descriptor[j] ? 1.0f : -1.0f;
            } else {
                descriptor[static_cast<int>(j)] = static_cast<float>(temp_descriptor[j]);
            }
        }
    }
    return true;
}

}  // namespace feature_detector

#endif  // FEATURE_DETECTOR_DESCRIPTOR_H_
