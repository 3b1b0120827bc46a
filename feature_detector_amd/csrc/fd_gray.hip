// Colour -> gray for the ingest front end (the reference's Visualizor2D::LoadImage,
// test/test_feature_point_detector.cpp:104, is un-vendored: its conversion is parity-unpinned).
// Gray = (4899 R + 9617 G + 1868 B + 8192) >> 14 (ITU-R BT.601 weights in 14-bit fixed point, rounded);
// gray + alpha and RGBA drop the alpha; 1-channel input is copied. HBM-bound: each lane converts 4
// pixels (reads 4 * channels bytes as dwords, writes one dword).
#include "fd_device.h"
#include "fd_kernels.h"

namespace fdk {

namespace {

__device__ __forceinline__ uint32_t gray_of(uint32_t r, uint32_t g, uint32_t b) {
    return (4899u * r + 9617u * g + 1868u * b + 8192u) >> 14;
}

template <int C>
__global__ __launch_bounds__(256) void k_rgb_gray(const uint8_t *src, uint8_t *dst, int64_t npx) {
    const int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;  // pixel quad
    const int64_t p0 = q * 4;
    if (p0 >= npx) return;
    const auto rs = make_rsrc(src, static_cast<uint32_t>(npx * C));  // (npx * C < 2^32: checked on the host)
    uint32_t out = 0;
    if (p0 + 4 <= npx && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 3) == 0) {
        uint32_t w[C];
#pragma unroll
        for (int k = 0; k < C; ++k) w[k] = buf_load_u32(rs, static_cast<int32_t>(p0 * C + 4 * k));
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            auto byte = [&](int i) { return (w[i >> 2] >> (8 * (i & 3))) & 0xFFu; };
            const uint32_t v = C <= 2 ? byte(m * C) : gray_of(byte(m * C), byte(m * C + 1), byte(m * C + 2));
            out |= v << (8 * m);
        }
        *reinterpret_cast<uint32_t *>(dst + p0) = out;
        return;
    }
    for (int m = 0; m < 4 && p0 + m < npx; ++m) {
        const int64_t i = (p0 + m) * C;
        dst[p0 + m] = static_cast<uint8_t>(C <= 2 ? src[i] : gray_of(src[i], src[i + 1], src[i + 2]));
    }
}

}  // namespace

hipError_t launch_rgb_gray(const uint8_t *src, int channels, uint8_t *dst, int64_t npx, hipStream_t s) {
    const int64_t quads = (npx + 3) / 4;
    const dim3 grid(static_cast<unsigned>((quads + 255) / 256)), block(256);
    switch (channels) {
        case 1: hipLaunchKernelGGL(k_rgb_gray<1>, grid, block, 0, s, src, dst, npx); break;
        case 2: hipLaunchKernelGGL(k_rgb_gray<2>, grid, block, 0, s, src, dst, npx); break;
        case 3: hipLaunchKernelGGL(k_rgb_gray<3>, grid, block, 0, s, src, dst, npx); break;
        case 4: hipLaunchKernelGGL(k_rgb_gray<4>, grid, block, 0, s, src, dst, npx); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace fdk
