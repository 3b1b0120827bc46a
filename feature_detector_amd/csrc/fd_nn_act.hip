// Bias + ReLU (+ 2x2 max pool) of the NN detectors' convolutions, one pass over an NHWC fp16 activation
// (gfx950). PyTorch-ROCm runs a biased convolution as the bias-free MIOpen/CK convolution, then a
// broadcast add, then the ReLU and the pooling as separate elementwise passes: three to four full
// reads and writes of the largest tensors of the network (64 x 640 x 480 x 64 halves = 2.5 GB for the
// first layers). Here the convolution runs without its bias and this kernel applies bias, ReLU and
// (for the layers a MaxPool2d(2, 2) follows) the pooling while the activation is read once.
// Arithmetic as PyTorch's half ops: x + b in float (opmath), rounded to half (round to nearest even),
// ReLU as max(v, 0) on the rounded value, pooling as the max of the four (exact).
#include "fd_device.h"
#include "fd_kernels.h"

namespace fdk {
namespace {

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

// 8 channels (16 bytes) of one pixel: relu(x + b) per half.
__device__ __forceinline__ u4 bias_relu8(u4 xv, u4 bv) {
    u4 r;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t xw = xv[k], bw = bv[k];
        _Float16 lo = static_cast<_Float16>(static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(xw))) +
                                            static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(bw))));
        _Float16 hi = static_cast<_Float16>(static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(xw >> 16))) +
                                            static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(bw >> 16))));
        lo = lo > static_cast<_Float16>(0.0f) ? lo : static_cast<_Float16>(0.0f);
        hi = hi > static_cast<_Float16>(0.0f) ? hi : static_cast<_Float16>(0.0f);
        r[k] = static_cast<uint32_t>(__builtin_bit_cast(uint16_t, lo)) | (static_cast<uint32_t>(__builtin_bit_cast(uint16_t, hi)) << 16);
    }
    return r;
}

// Elementwise max of two relu'd vectors (non-negative halves: their bit patterns order like integers).
__device__ __forceinline__ u4 max8(u4 a, u4 b) {
    u4 r;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t lo = max(a[k] & 0xFFFFu, b[k] & 0xFFFFu), hi = max(a[k] >> 16, b[k] >> 16);
        r[k] = lo | (hi << 16);
    }
    return r;
}

__global__ __launch_bounds__(256) void k_bias_relu(const u4 *x, const u4 *bias, u4 *y, int64_t nvec, int cvec) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < nvec;
         i += static_cast<int64_t>(gridDim.x) * 256)
        y[i] = bias_relu8(x[i], bias[i % cvec]);
}

// y [n][h/2][w/2][c] = max over the 2x2 window of relu(x + b); one thread per output 8-channel vector.
__global__ __launch_bounds__(256) void k_bias_relu_pool(const u4 *x, const u4 *bias, u4 *y, int n, int h, int w,
                                                        int cvec) {
    const int ho = h >> 1, wo = w >> 1;
    const int64_t total = static_cast<int64_t>(n) * ho * wo * cvec;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
         i += static_cast<int64_t>(gridDim.x) * 256) {
        const int cv = static_cast<int>(i % cvec);
        int64_t p = i / cvec;
        const int xo = static_cast<int>(p % wo);
        p /= wo;
        const int yo = static_cast<int>(p % ho);
        const int64_t b = p / ho;
        const int64_t r0 = ((b * h + 2 * yo) * w + 2 * xo) * cvec + cv;  // (2yo, 2xo)
        const int64_t r1 = r0 + static_cast<int64_t>(w) * cvec;          // (2yo + 1, 2xo)
        const u4 bv = bias[cv];
        const u4 a = bias_relu8(x[r0], bv), c = bias_relu8(x[r0 + cvec], bv);
        const u4 d = bias_relu8(x[r1], bv), e = bias_relu8(x[r1 + cvec], bv);
        y[i] = max8(max8(a, c), max8(d, e));
    }
}

}  // namespace

hipError_t launch_bias_relu(const void *x, const void *bias, void *y, int n, int h, int w, int c, int pool,
                            hipStream_t s) {
    const int cvec = c / 8;
    const int64_t nvec = static_cast<int64_t>(n) * h * w * cvec;
    const int64_t out = pool ? nvec / 4 : nvec;
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>((out + 255) / 256, 256 * 64));
    if (out == 0) return hipSuccess;
    if (pool)
        hipLaunchKernelGGL(k_bias_relu_pool, dim3(grid), dim3(256), 0, s, static_cast<const u4 *>(x),
                           static_cast<const u4 *>(bias), static_cast<u4 *>(y), n, h, w, cvec);
    else
        hipLaunchKernelGGL(k_bias_relu, dim3(grid), dim3(256), 0, s, static_cast<const u4 *>(x),
                           static_cast<const u4 *>(bias), static_cast<u4 *>(y), nvec, cvec);
    return hipGetLastError();
}

}  // namespace fdk
