// HBM copy ceiling for bench.py (`device_copy_gbs`): a float4 (16 B per lane) grid-stride streaming copy,
// the form MI355X_MICROARCH.md measures at ~6.3 TB/s (read + write bytes / time). Not part of the
// product library: bench.py loads it beside libfdhip.so to report the practical HBM ceiling of the
// byte-moving kernels (the LSD map) next to their achieved rates.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_copy16(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, size_t n16) {
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    // 4 independent 16-byte loads per thread in flight per iteration
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const u32x4 a = __builtin_nontemporal_load(src + i);
        const u32x4 b = __builtin_nontemporal_load(src + i + stride);
        const u32x4 c = __builtin_nontemporal_load(src + i + 2 * stride);
        const u32x4 d = __builtin_nontemporal_load(src + i + 3 * stride);
        __builtin_nontemporal_store(a, dst + i);
        __builtin_nontemporal_store(b, dst + i + stride);
        __builtin_nontemporal_store(c, dst + i + 2 * stride);
        __builtin_nontemporal_store(d, dst + i + 3 * stride);
    }
    for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// the plain form: one 16-byte element per thread, default cache policy, one workgroup per 4 KiB
__global__ __launch_bounds__(256) void k_copy16_flat(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, size_t n16) {
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n16) dst[i] = src[i];
}

// write-only: 16-byte nontemporal stores, grid-stride (the write half of the HBM ceiling)
__global__ __launch_bounds__(256) void k_fill16(u32x4 *__restrict__ dst, size_t n16, unsigned v) {
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    const u32x4 z = {v, v, v, v};
    for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += stride)
        __builtin_nontemporal_store(z, dst + i);
}

// the LSD map's traffic shape (fd_lsd.hip k_lsd_map, dense): per 4 pixels one 4-byte read of the frame and
// a 16-byte norm, a 16-byte angle and a 4-byte valid store (nontemporal), with a trivial computation in
// between -- 1 B read + 9 B written per pixel, the map's bytes without its arithmetic
__global__ __launch_bounds__(256) void k_lsd_shape(const unsigned *__restrict__ src, u32x4 *__restrict__ norm,
                                                   u32x4 *__restrict__ angle, unsigned *__restrict__ valid, size_t n4) {
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const unsigned p = __builtin_nontemporal_load(src + i);
        const u32x4 a = {p & 0xFFu, (p >> 8) & 0xFFu, (p >> 16) & 0xFFu, p >> 24};
        __builtin_nontemporal_store(a, norm + i);
        __builtin_nontemporal_store(a ^ 0x3F800000u, angle + i);
        __builtin_nontemporal_store(p & 0x01010101u, valid + i);
    }
}

// the flat forms: one element per thread, default cache policy
__global__ __launch_bounds__(256) void k_fill16_flat(u32x4 *__restrict__ dst, size_t n16, unsigned v) {
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n16) dst[i] = u32x4{v, v, v, v};
}
__global__ __launch_bounds__(256) void k_lsd_shape_flat(const unsigned *__restrict__ src, u32x4 *__restrict__ norm,
                                                        u32x4 *__restrict__ angle, unsigned *__restrict__ valid, size_t n4) {
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const unsigned p = src[i];
    const u32x4 a = {p & 0xFFu, (p >> 8) & 0xFFu, (p >> 16) & 0xFFu, p >> 24};
    norm[i] = a;
    angle[i] = a ^ 0x3F800000u;
    valid[i] = p & 0x01010101u;
}

}  // namespace

extern "C" int fdcal_fill16_flat(void *dst, size_t bytes, void *stream) {
    const size_t n16 = bytes / 16;
    hipLaunchKernelGGL(k_fill16_flat, dim3(static_cast<unsigned>((n16 + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), static_cast<u32x4 *>(dst), n16, 0u);
    return static_cast<int>(hipGetLastError());
}

extern "C" int fdcal_lsd_shape_flat(const void *src, void *norm, void *angle, void *valid, size_t npx, void *stream) {
    const size_t n4 = npx / 4;
    hipLaunchKernelGGL(k_lsd_shape_flat, dim3(static_cast<unsigned>((n4 + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), static_cast<const unsigned *>(src), static_cast<u32x4 *>(norm),
                       static_cast<u32x4 *>(angle), static_cast<unsigned *>(valid), n4);
    return static_cast<int>(hipGetLastError());
}

extern "C" int fdcal_fill16(void *dst, size_t bytes, void *stream) {
    hipLaunchKernelGGL(k_fill16, dim3(256u * 8u), dim3(256), 0, static_cast<hipStream_t>(stream), static_cast<u32x4 *>(dst),
                       bytes / 16, 0u);
    return static_cast<int>(hipGetLastError());
}

// src: npx bytes; norm, angle: 4 npx bytes each; valid: npx bytes (npx a multiple of 4, all 16-byte aligned)
extern "C" int fdcal_lsd_shape(const void *src, void *norm, void *angle, void *valid, size_t npx, void *stream) {
    hipLaunchKernelGGL(k_lsd_shape, dim3(256u * 8u), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<const unsigned *>(src), static_cast<u32x4 *>(norm), static_cast<u32x4 *>(angle),
                       static_cast<unsigned *>(valid), npx / 4);
    return static_cast<int>(hipGetLastError());
}

extern "C" int fdcal_copy16_flat(void *dst, const void *src, size_t bytes, void *stream) {
    const size_t n16 = bytes / 16;
    hipLaunchKernelGGL(k_copy16_flat, dim3(static_cast<unsigned>((n16 + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), static_cast<const u32x4 *>(src), static_cast<u32x4 *>(dst), n16);
    return static_cast<int>(hipGetLastError());
}

// bytes: a multiple of 16; src / dst 16-byte aligned device memory. Enqueued on `stream`.
extern "C" int fdcal_copy16(void *dst, const void *src, size_t bytes, void *stream) {
    const size_t n16 = bytes / 16;
    const unsigned blocks = 256u * 8u;  // 8 workgroups of 256 threads per CU
    hipLaunchKernelGGL(k_copy16, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<const u32x4 *>(src), static_cast<u32x4 *>(dst), n16);
    return static_cast<int>(hipGetLastError());
}
