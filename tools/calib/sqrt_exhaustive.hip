// Exhaustive check of fdk::sqrt_rn_rsq2 (fd_device.h, the Shi-Tomasi sqrt of k_corner) against the
// IEEE correctly rounded sqrt (f64 sqrt rounded to f32) on every float x in {0} U [2^-60, FLT_MAX].
// Prints "sqrt_rn_rsq2: <checked> values, <n> mismatches" and up to 16 mismatching inputs; exit 1 on any.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "fd_device.h"

__global__ __launch_bounds__(256) void k_check(uint32_t lo, uint32_t hi, unsigned long long *bad, uint32_t *ex) {
    const uint32_t stride = gridDim.x * blockDim.x * 2;
    for (uint32_t u = lo + 2 * (blockIdx.x * blockDim.x + threadIdx.x); u < hi; u += stride) {
        const uint32_t u1 = u + 1 < hi ? u + 1 : u;
        fdk::f2 x = {__uint_as_float(u), __uint_as_float(u1)};
        const fdk::f2 s = fdk::sqrt_rn_rsq2(x);
        // reference: the f64 square root (correctly rounded) rounded to f32; double rounding is
        // harmless for sqrt since 53 >= 2 * 24 + 2
        const float r0 = static_cast<float>(sqrt(static_cast<double>(x.x)));
        const float r1 = static_cast<float>(sqrt(static_cast<double>(x.y)));
        if (__float_as_uint(s.x) != __float_as_uint(r0)) {
            const unsigned long long k = atomicAdd(bad, 1ull);
            if (k < 16) ex[k] = u;
        }
        if (__float_as_uint(s.y) != __float_as_uint(r1)) {
            const unsigned long long k = atomicAdd(bad, 1ull);
            if (k < 16) ex[k] = u1;
        }
    }
}

int main() {
    unsigned long long *bad;
    uint32_t *ex;
    if (hipMalloc(&bad, sizeof(*bad)) != hipSuccess) return 2;
    if (hipMalloc(&ex, 16 * sizeof(uint32_t)) != hipSuccess) return 2;
    if (hipMemset(bad, 0, sizeof(*bad)) != hipSuccess) return 2;
    const float lo_f = 0x1p-60f;
    uint32_t lo;
    std::memcpy(&lo, &lo_f, 4);
    const uint32_t hi = 0x7F800000u;  // +inf (exclusive)
    k_check<<<4096, 256>>>(lo, hi, bad, ex);
    k_check<<<1, 1>>>(0u, 1u, bad, ex);  // x = 0
    unsigned long long nb = 0;
    uint32_t hx[16];
    if (hipMemcpy(&nb, bad, sizeof(nb), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    if (hipMemcpy(hx, ex, sizeof(hx), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    if (hipGetLastError() != hipSuccess) { std::printf("hip error\n"); return 2; }
    std::printf("sqrt_rn_rsq2: %llu values, %llu mismatches\n", (unsigned long long)(hi - lo) + 1ull, nb);
    for (unsigned long long i = 0; i < nb && i < 16; ++i) {
        float f;
        std::memcpy(&f, &hx[i], 4);
        std::printf("  x = %a (0x%08x)\n", f, hx[i]);
    }
    return nb ? 1 : 0;
}
