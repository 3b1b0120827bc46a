// Device-side helpers shared by the gfx950 kernels (wave64, DPP, buffer loads, exact float math).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fdk {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Lane i receives lane i-1's value (lane 0 receives 0): DPP wave_shr:1 with bound_ctrl, so the
// invalid source lane reads 0 and no zeroed destination has to be prepared.
__device__ __forceinline__ uint32_t from_left(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x138, 0xF, 0xF, true));
}
// Lane i receives lane i+1's value (lane 63 receives 0): DPP wave_shl:1.
__device__ __forceinline__ uint32_t from_right(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), 0x130, 0xF, 0xF, true));
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

// max(a, b, c) as one v_max3_f32. fmaxf would first canonicalize each operand (IEEE mode quiets
// signalling NaNs), doubling the instruction count; callers only pass finite values.
__device__ __forceinline__ float max3f(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// a + b + c (mod 2^32) as one v_add3_u32. Written as asm because LLVM reassociates chains of 3-row
// sums into shared pair sums (two v_add_u32 per result instead of one v_add3).
__device__ __forceinline__ uint32_t add3u(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Inclusive prefix sum over the wave (lane i: lanes 0..i) by DPP: row_shr 1/2/4/8 within each row of
// 16 lanes, then row_bcast:15 / row_bcast:31 carry the row totals up (GFX9 DPP). Six dependent VALU
// ops instead of six ds_bpermute round trips (__shfl_up), which chain LDS latency.
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t x) {
    x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x111, 0xF, 0xF, false));  // row_shr:1
    x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x112, 0xF, 0xF, false));  // row_shr:2
    x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x114, 0xF, 0xF, false));  // row_shr:4
    x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x118, 0xF, 0xF, false));  // row_shr:8
    x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x142, 0xA, 0xF, false));  // row_bcast:15
    x += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x143, 0xC, 0xF, false));  // row_bcast:31
    return x;
}
// Max / min over the wave (unsigned), in every lane: the same DPP row_shr / row_bcast ladder as
// wave_incl_add with the identity as the value of lanes that have no source, then lane 63's result
// (instead of six ds_bpermute round trips of a __shfl_xor butterfly).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
    x = max(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x111, 0xF, 0xF, false)));
    x = max(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x112, 0xF, 0xF, false)));
    x = max(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x114, 0xF, 0xF, false)));
    x = max(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x118, 0xF, 0xF, false)));
    x = max(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x142, 0xA, 0xF, false)));
    x = max(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x143, 0xC, 0xF, false)));
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x), 63));
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    x = min(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(x), 0x111, 0xF, 0xF, false)));
    x = min(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(x), 0x112, 0xF, 0xF, false)));
    x = min(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(x), 0x114, 0xF, 0xF, false)));
    x = min(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(x), 0x118, 0xF, 0xF, false)));
    x = min(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(x), 0x142, 0xA, 0xF, false)));
    x = min(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(-1, static_cast<int>(x), 0x143, 0xC, 0xF, false)));
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(x), 63));
}
// Sum over the wave, in every lane.
__device__ __forceinline__ uint32_t wave_total_add(uint32_t x) {
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wave_incl_add(x)), 63));
}
// Inclusive suffix sum over the wave (lane i: lanes i..63) = wave total - exclusive prefix.
__device__ __forceinline__ uint32_t wave_suffix_add(uint32_t x) {
    const uint32_t p = wave_incl_add(x);
    const uint32_t tot = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(p), 63));
    return tot - p + x;
}

// A value the compiler cannot see through: an LDS address derived from it inside a loop is recomputed
// there (one VALU op) instead of being hoisted across the enclosing loops -- k_select runs at its
// 128-VGPR limit, and such hoisted addresses were spilled to scratch and reloaded (a memory round trip)
// at every sub-chunk.
__device__ __forceinline__ int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

// LDS pointer type: a noinline function taking one keeps issuing ds_* instructions (a generic pointer
// would make them flat accesses). to_lds / from_lds convert (the object must live in LDS).
template <class T>
using lds_t = __attribute__((address_space(3))) T;
template <class T>
__device__ __forceinline__ lds_t<T> *to_lds(T *p) { return (lds_t<T> *)(p); }
template <class T>
__device__ __forceinline__ T *from_lds(lds_t<T> *p) { return (T *)(p); }

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int popc64(uint64_t m) { return __popcll(m); }
__device__ __forceinline__ uint64_t lanes_below() {
    const int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// acc + number of set bits of m in lanes below this one (v_mbcnt_lo / v_mbcnt_hi).
__device__ __forceinline__ int mbcnt64(uint64_t m, int acc) {
    const uint32_t lo = __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), static_cast<uint32_t>(acc));
    return static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32), lo));
}

// Order-preserving map of an IEEE float to an unsigned key (larger float -> larger key).
__device__ __forceinline__ uint32_t float_key(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

typedef float f2 __attribute__((ext_vector_type(2)));

// Correctly rounded f32 sqrt of two values that are each 0 or >= 2^-60, in 4.5 issue slots per value
// (one transcendental + four packed ops): y = rsq(x) (v_rsq_f32, ~1 ulp), s0 = x*y, one Newton step
// s = s0 + (x - s0*s0) * y/2 with the residual exact (fma) and the correction rounded once (fma).
// Not correctly rounded by construction (the correction's error, ~2^-20 ulp, exceeds the 2^-29 ulp by
// which a float's square root can approach a rounding midpoint), so it is verified exhaustively: every
// float from 2^-60 up, and 0, against the IEEE sqrt (tools/calib/sqrt_exhaustive.hip, run by
// tests/test_gpu_points.py). The Shi-Tomasi radicand d*d + 4b*b is 0 or >= 2^-54 (b is 0 or |b| >= 1/9,
// a != c differ by at least ulp(1/9) = 2^-27). The tiny addend keeps rsq(0) finite (s0 = 0*y = 0,
// s = 0) and leaves every x >= 2^-54 unchanged.
__device__ __forceinline__ f2 sqrt_rn_rsq2(f2 x) {
    const f2 xt = x + 0x1p-110f;
    const f2 y = {__builtin_amdgcn_rsqf(xt.x), __builtin_amdgcn_rsqf(xt.y)};
    const f2 s0 = x * y;
    const f2 e = __builtin_elementwise_fma(-s0, s0, x);
    const f2 h = y * 0.5f;
    return __builtin_elementwise_fma(e, h, s0);
}

}  // namespace fdk
