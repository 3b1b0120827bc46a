// How far the bare hardware square root (v_sqrt_f32) is from the IEEE correctly rounded sqrt on the
// Shi-Tomasi radicand's domain, {0} U [2^-60, 2^40): counts the inputs where it differs (by 1 ulp up or
// down, or more), to decide whether the k_corner_lp response may use it directly. Prints the counts and
// up to 16 differing inputs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__global__ __launch_bounds__(256) void k_check(uint32_t lo, uint32_t hi, unsigned long long *cnt, uint32_t *ex) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t u = lo + blockIdx.x * blockDim.x + threadIdx.x; u < hi; u += stride) {
        const float x = __uint_as_float(u);
        const float s = __builtin_amdgcn_sqrtf(x);  // v_sqrt_f32
        const float r = static_cast<float>(sqrt(static_cast<double>(x)));  // correctly rounded (53 >= 2*24+2)
        const int32_t d = static_cast<int32_t>(__float_as_uint(s)) - static_cast<int32_t>(__float_as_uint(r));
        if (d != 0) {
            const int slot = d == 1 ? 0 : (d == -1 ? 1 : 2);
            const unsigned long long k = atomicAdd(&cnt[slot], 1ull);
            if (k < 6) ex[slot * 6 + k] = u;
        }
    }
}

int main() {
    unsigned long long *cnt;
    uint32_t *ex;
    if (hipMalloc(&cnt, 3 * sizeof(*cnt)) != hipSuccess) return 2;
    if (hipMalloc(&ex, 18 * sizeof(uint32_t)) != hipSuccess) return 2;
    if (hipMemset(cnt, 0, 3 * sizeof(*cnt)) != hipSuccess) return 2;
    if (hipMemset(ex, 0, 18 * sizeof(uint32_t)) != hipSuccess) return 2;
    const float lo_f = 0x1p-60f, hi_f = 0x1p40f;
    uint32_t lo, hi;
    std::memcpy(&lo, &lo_f, 4);
    std::memcpy(&hi, &hi_f, 4);
    k_check<<<8192, 256>>>(lo, hi, cnt, ex);
    k_check<<<1, 1>>>(0u, 1u, cnt, ex);
    unsigned long long h[3];
    uint32_t hx[18];
    if (hipMemcpy(h, cnt, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    if (hipMemcpy(hx, ex, sizeof(hx), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    std::printf("v_sqrt_f32 vs IEEE sqrt on %llu floats: +1 ulp %llu, -1 ulp %llu, other %llu\n",
                (unsigned long long)(hi - lo) + 1ull, h[0], h[1], h[2]);
    for (int s = 0; s < 3; ++s)
        for (unsigned long long i = 0; i < h[s] && i < 6; ++i) {
            float f;
            std::memcpy(&f, &hx[s * 6 + i], 4);
            std::printf("  [%s] x = %a\n", s == 0 ? "+1" : (s == 1 ? "-1" : "other"), f);
        }
    return 0;
}
