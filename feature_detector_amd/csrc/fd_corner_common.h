// Shared device pieces of the corner kernels (fd_points.hip: k_corner, k_fast; fd_corner_lp.hip:
// k_corner_lp): workgroup -> tile decoding, frame loads, the LDS histogram, and the exact response
// arithmetic. Each including translation unit gets its own copy (anonymous namespace).
#pragma once

#include "fd_device.h"
#include "fd_kernels.h"

namespace fdk {
namespace {

constexpr float kInvCnt = 1.0f / 9.0f;                  // 1 / (3*3)  (:71)
constexpr float kInvCnt2 = (1.0f / 9.0f) * (1.0f / 9.0f);  // harris :72
constexpr float kHarrisAlpha = 0.04f;                  // feature_point_harris_detector.h:13

// Workgroup -> (frame, 4 consecutive tiles of that frame); returns false for the idle waves of a
// frame's last workgroup (they still take part in the workgroup barriers).
// The tile coordinates are made visibly wave-uniform (readfirstlane), so row/tile logic stays scalar.
// Logical workgroup id: workgroups are dealt round-robin over the 8 XCDs (b and b + 8 share an L2), so
// the grid is remapped to give each XCD a contiguous range of logical ids -- a band of a frame's tile
// rows, whose halo rows then come from that XCD's own L2 (for speed only: any placement is correct).
// Bijective for any grid size: XCD group x = b % 8 holds q (+1 for x < r) workgroups.
__device__ __forceinline__ int logical_block() {
    const int b = static_cast<int>(blockIdx.x), n = static_cast<int>(gridDim.x);
    const int q = n >> 3, r = n & 7, x = b & 7;
    return x * q + min(x, r) + (b >> 3);
}

__device__ __forceinline__ bool decode_tile(const PointsArgs &a, int &f, int &ty, int &tx) {
    const int lb = logical_block();
    f = lb / a.blocks_per_frame;
    const int t = __builtin_amdgcn_readfirstlane((lb % a.blocks_per_frame) * 4 + (threadIdx.x >> 6));
    tx = t % a.tiles_x;
    ty = t / a.tiles_x;
    return t < a.tiles_x * a.tiles_y;
}

// Dword of frame bytes [off, off+4). `aligned` (cols % 4 == 0) guarantees whole-dword range checks;
// otherwise assemble from byte loads so that a dword straddling the frame end still returns its bytes.
// A compile-time choice: a runtime branch here makes the waitcnt pass drain the prefetch queue.
template <bool ALIGNED>
__device__ __forceinline__ uint32_t load_px4(__amdgpu_buffer_rsrc_t r, int32_t off) {
#ifdef FD_NOLOAD  // diagnostic build only (tools/gpu_noload_ab.sh): same instruction stream, no frame reads
    return static_cast<uint32_t>(off) * 2654435761u;
#endif
    if constexpr (ALIGNED) return buf_load_u32(r, off);
    return buf_load_u8(r, off) | (buf_load_u8(r, off + 1) << 8) | (buf_load_u8(r, off + 2) << 16) |
           (buf_load_u8(r, off + 3) << 24);
}

// (the per-pixel kernels run 256-thread workgroups: a constant stride, no blockDim load -- whose wait
// would also hold for every vector-memory operation in flight, e.g. seg_flush's returning atomic)
constexpr int kPixWg = 256;
// LDS accesses all issued before any is used (the histogram loops were chains of one LDS round trip,
// and in the flush one exec-masked branch, per bin group); the clear by 16-byte stores (h is 16-byte
// aligned in every LDS layout: DetectLdsT, LpLds).
constexpr int kHistPer = kHistBins / (4 * kPixWg);  // uint4 groups per thread
__device__ __forceinline__ void hist_clear(uint32_t *h) {
    uint4 *h4 = reinterpret_cast<uint4 *>(h);
#pragma unroll
    for (int k = 0; k < kHistPer; ++k) h4[threadIdx.x + k * kPixWg] = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
}
// The flush keeps one bin per lane per atomic instruction (64 consecutive dwords: a 4-dwords-per-lane
// pattern spreads each wave instruction over 4x the 64-B atomic requests, measured +4.9 us at batch 1).
__device__ __forceinline__ void hist_flush(const uint32_t *h, uint32_t *g) {
    __syncthreads();
    constexpr int kPer = kHistBins / kPixWg;
    uint32_t v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) v[k] = h[threadIdx.x + k * kPixWg];
#pragma unroll
    for (int k = 0; k < kPer; ++k)
        if (v[k]) atomicAdd(&g[threadIdx.x + k * kPixWg], v[k]);
}

// Two pixels' float math at a time: <2 x float> arithmetic compiles to v_pk_mul_f32 / v_pk_add_f32 /
// v_pk_fma_f32, which round each lane exactly like the scalar op (the kernel is VALU-issue bound, and
// a packed op retires two pixels' worth of one reference operation per issue slot).
// sqrt_rn_rsq2 (correctly rounded sqrt on the reciprocal square root) lives in fd_device.h.

// Stored responses of two pixels (responses_ semantics: 0 unless written), from exact integer tensor
// sums. Same operations in the same order as the reference; only the issue is paired.
//
// Integer-to-float without v_cvt: every gradient product carries a bias beta (mod 2^32) chosen so that
// the nine products of a 3x3 sum carry exactly 9*beta == 0x4B000000 (the bit pattern of 2^23), or
// 0x4B400000 (2^23 + 2^22) for the signed cross term. Then for 0 <= S < 2^23 (S <= 9*255^2 here,
// |Sxy| < 2^22) the biased sum read as a float is exactly 2^23 + S, and one exact (packed)
// subtraction recovers float(S). 9 is odd, so beta = target * 9^-1 mod 2^32 exists.
constexpr uint32_t kBiasSq = 0xB3000000u;  // 9 * kBiasSq == 0x4B000000 (mod 2^32)
constexpr uint32_t kBiasXy = 0x41400000u;  // 9 * kBiasXy == 0x4B400000 (mod 2^32)
static_assert(9u * kBiasSq == 0x4B000000u && 9u * kBiasXy == 0x4B400000u, "bias");

// G1 (detect mode with thr >= 0): only the pre-check gates the stored value, so a pixel whose
// response is <= thr keeps its response instead of 0. The NMS that reads these values tests
// x > max(thr, neighbours): with thr >= 0 a kept response <= thr acts exactly like the reference's 0
// there (as a centre it fails x > thr, as a neighbour max(thr, r) == thr == max(thr, 0)), and every
// emitted candidate has x > thr, i.e. the reference's stored value. Saves a compare per pixel.
template <int KIND, bool G1>
__device__ __forceinline__ f2 corner_response2(uint32_t sxx0, uint32_t sxx1, uint32_t syy0, uint32_t syy1,
                                               uint32_t sxy0, uint32_t sxy1, float thr) {
    const f2 bxx = f2{__uint_as_float(sxx0), __uint_as_float(sxx1)};  // 2^23 + Sxx, exactly
    const f2 byy = f2{__uint_as_float(syy0), __uint_as_float(syy1)};
    const f2 fxy = f2{__uint_as_float(sxy0), __uint_as_float(sxy1)} - 12582912.0f;
    f2 res, gate, r;
    if constexpr (KIND == 0) {  // Harris, feature_point_harris_detector.cpp:95-103
        const f2 fxx = bxx - 8388608.0f, fyy = byy - 8388608.0f;
        const f2 trace = fxx + fyy;
        gate = ((trace * trace) * 0.21f) * kInvCnt2;
        r = (((fxx * fyy) - (fxy * fxy)) - ((kHarrisAlpha * trace) * trace)) * kInvCnt2;
    } else {  // Shi-Tomasi, feature_point_shi_tomas_detector.cpp:94-103
        // a = fl(Sxx * k) as one fma on the biased sum: bxx*k - 2^23*k is (bxx - 2^23)*k = Sxx*k
        // exactly before the fma's single rounding (2^23*k is exact: a power-of-two multiple of k).
        const f2 a = __builtin_elementwise_fma(bxx, f2{kInvCnt, kInvCnt}, f2{-8388608.0f * kInvCnt, -8388608.0f * kInvCnt});
        const f2 c = __builtin_elementwise_fma(byy, f2{kInvCnt, kInvCnt}, f2{-8388608.0f * kInvCnt, -8388608.0f * kInvCnt});
        gate = a + c;
        const f2 b = fxy * kInvCnt;
        const f2 d = a - c;
        // (4b)*b = 4*fl(b*b) exactly, so dd + fl(fl(4b)*b) is one fma of b*b with 4
        const f2 common = sqrt_rn_rsq2(__builtin_elementwise_fma(b * b, f2{4.0f, 4.0f}, d * d));
        r = (gate + common) * 0.5f;
    }
    if constexpr (G1) {
        res.x = gate.x > thr ? r.x : 0.0f;
        res.y = gate.y > thr ? r.y : 0.0f;
    } else {
        res.x = (gate.x > thr && r.x > thr) ? r.x : 0.0f;
        res.y = (gate.y > thr && r.y > thr) ? r.y : 0.0f;
    }
    return res;
}

}  // namespace
}  // namespace fdk
