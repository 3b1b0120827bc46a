// Device-side helpers shared by the gfx950 kernels (wave64, DPP, buffer loads, exact float math).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fdk {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Lane i receives lane i-1's value (lane 0 receives 0): DPP wave_shr:1.
__device__ __forceinline__ uint32_t from_left(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x138, 0xF, 0xF, false));
}
// Lane i receives lane i+1's value (lane 63 receives 0): DPP wave_shl:1.
__device__ __forceinline__ uint32_t from_right(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x130, 0xF, 0xF, false));
}
__device__ __forceinline__ float from_left_f(float v) { return __uint_as_float(from_left(__float_as_uint(v))); }
__device__ __forceinline__ float from_right_f(float v) { return __uint_as_float(from_right(__float_as_uint(v))); }

// Buffer resource over [base, base + bytes): out-of-range dword loads return 0 (hardware range check),
// which makes frame borders free of address clamping.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, static_cast<int>(bytes), 0x00020000);
}
__device__ __forceinline__ uint32_t buf_load_u32(__amdgpu_buffer_rsrc_t r, int32_t byte_off) {
    return static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}
__device__ __forceinline__ uint32_t buf_load_u8(__amdgpu_buffer_rsrc_t r, int32_t byte_off) {
    return static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b8(r, byte_off, 0, 0));
}

// Byte J (compile-time after unrolling) of the 12-byte window [L | M | R] = columns c0-4 .. c0+7.
__device__ __forceinline__ int win_byte(uint32_t L, uint32_t M, uint32_t R, int j) {
    const uint32_t w = j < 0 ? L : (j < 4 ? M : R);
    const int sh = 8 * (j < 0 ? j + 4 : (j < 4 ? j : j - 4));
    return static_cast<int>((w >> sh) & 0xFFu);
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int popc64(uint64_t m) { return __popcll(m); }
__device__ __forceinline__ uint64_t lanes_below() {
    const int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Order-preserving map of an IEEE float to an unsigned key (larger float -> larger key).
__device__ __forceinline__ uint32_t float_key(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

}  // namespace fdk
