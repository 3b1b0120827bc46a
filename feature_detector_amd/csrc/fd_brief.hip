// Steered BRIEF descriptor for gfx950.
//
// Reference: BriefDescriptor::ComputeForOneFeature (feature_descriptor/descriptor_brief.cpp:8-50),
// driven per keypoint by Descriptor<BriefType>::Compute (descriptor.h:27-40). One wave per keypoint:
//   1. border test (:13-17); out-of-border keypoints keep the all-zero descriptor (:10);
//   2. intensity-centroid moments m10, m01 over the (2h+1)^2 patch (:20-28);
//   3. m = sqrt(m01^2 + m10^2), sin = m01 / m, cos = m10 / m (:29-33); m < kZeroFloat -> zeros;
//   4. kLength rotated point pairs (:36-46): bit i = I(p1) < I(p2), 64 pairs per ballot.
// Float arithmetic keeps the reference's operation order (file built with -ffp-contract=off,
// correctly rounded sqrt and division), so everything up to the sampler is bit-exact.
//
// Sampler: the reference samples GrayImage::GetPixelValueNoCheck(float row, float col) from the
// un-vendored Slam_Utility, whose body is not available (parity unpinned). Two
// restatements are offered: FD_SAMPLE_BILINEAR (weights (1-ex)(1-ey), ex(1-ey), (1-ex)ey, ex*ey over
// the 2x2 neighbourhood, summed left to right) and FD_SAMPLE_TRUNCATE (pixel at (int)row, (int)col).
// Both read the row-major buffer as the reference's NoCheck accessor does (linear index
// row * cols + col); the only difference is that a linear index outside the frame reads 0 here
// (the reference reads out of bounds). At integer coordinates both samplers return the pixel, so
// the moments and orientation of integer keypoints (every detector output) are sampler-independent.
//
// Moments: every sample is an integer when the keypoint is integral or the sampler truncates, and
// for h <= 31 every partial sum stays below 2^24, so the reference's sequential float sums are exact
// and equal an integer wave reduction. Otherwise (fractional keypoint, bilinear, or h > 31) lane 0
// accumulates in the reference's loop order from samples staged 64 at a time in LDS.
#include "fd_device.h"
#include "fd_kernels.h"
#include "../../include/fd_hip.h"

namespace fdk {
namespace {

__constant__ uint32_t kPattern[256] = {
#include "fd_brief_pattern.inc"
};

constexpr float kZeroFloat = 1e-6f;        // Slam_Utility kZeroFloat (un-vendored; |m| is 0 or >= 1 for
                                           // integer keypoints, so any value in (0, 1) gives the same bits)
constexpr float kPatternMaxBound = 19.0f;  // descriptor_brief.cpp:13

// Pixel source. Global: one byte load per sample from the frame (a sample pattern spreads a wave's 64
// loads over ~30 rows: ~one cache line per lane, the TA's limit). Staged (STAGED = true, the usual
// case): the keypoint's patch -- every pixel a sample of this keypoint can touch -- was copied once into
// the wave's LDS with coalesced row loads, and samples read it there.
constexpr int kStageSide = 64;  // largest staged patch side (one lane per column)
constexpr int kPatchR = 20;     // sample reach: |rot(p)| <= sqrt(13^2 + 13^2) < 18.4 (pattern coordinates
                                // in [-13, 12]) plus the bilinear neighbour, around floor(u), floor(v)

struct Frame {
    __amdgpu_buffer_rsrc_t rsrc;
    int cols;
    const uint8_t *lds;  // staged patch [side][side] (null: global loads)
    int r0, c0, side;    // frame coordinates of lds[0]
};

__device__ __forceinline__ float pixel(const Frame &fr, int32_t r, int32_t c) {
    if (fr.lds) return static_cast<float>(fr.lds[(r - fr.r0) * fr.side + (c - fr.c0)]);
    // Linear index as the row-major NoCheck accessor; out of the frame -> 0 (buffer range check).
    const int32_t idx = r * fr.cols + c;
    return static_cast<float>(buf_load_u8(fr.rsrc, idx));
}

// Copy rows [r0, r0 + side) x columns [c0, c0 + side) -- as linear indices r * cols + c, exactly the bytes
// the global path would read (0 outside the frame's byte range) -- into the wave's LDS, one row per
// load instruction (lane = column).
__device__ __forceinline__ void stage_patch(Frame &fr, uint8_t *lds, int r0, int c0, int side) {
    const int lane = lane_id();
    for (int pr = 0; pr < side; ++pr)
        if (lane < side) lds[pr * side + lane] = static_cast<uint8_t>(buf_load_u8(fr.rsrc, (r0 + pr) * fr.cols + c0 + lane));
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    fr.lds = lds;
    fr.r0 = r0;
    fr.c0 = c0;
    fr.side = side;
}

template <int SAMPLER>
__device__ __forceinline__ float sample(const Frame &fr, float row, float col) {
    const int32_t r0 = static_cast<int32_t>(row);
    const int32_t c0 = static_cast<int32_t>(col);
    if constexpr (SAMPLER == FD_SAMPLE_TRUNCATE) {
        return pixel(fr, r0, c0);
    } else {
        const float ex = col - static_cast<float>(c0);
        const float ey = row - static_cast<float>(r0);
        const float ex1 = 1.0f - ex;
        const float ey1 = 1.0f - ey;
        const float p00 = pixel(fr, r0, c0), p01 = pixel(fr, r0, c0 + 1);
        const float p10 = pixel(fr, r0 + 1, c0), p11 = pixel(fr, r0 + 1, c0 + 1);
        return ex1 * ey1 * p00 + ex * ey1 * p01 + ex1 * ey * p10 + ex * ey * p11;
    }
}

// Sum over the wave (every lane gets it): DPP prefix sum + lane 63 (six dependent VALU ops instead of
// six ds_bpermute round trips).
__device__ __forceinline__ int wave_sum(int v) {
    const uint32_t p = wave_incl_add(static_cast<uint32_t>(v));
    return __builtin_amdgcn_readlane(static_cast<int>(p), 63);
}

template <int SAMPLER>
__device__ void brief_one(const BriefArgs &a, Frame &fr, float u, float v, uint32_t *out, uint8_t *valid,
                          float *stage, uint8_t *patch) {
    const int lane = lane_id();
    const int nw = (a.length + 31) >> 5;
    const int h = a.half;
    const float max_bound = fmaxf(kPatternMaxBound, static_cast<float>(h) * 2.0f);
    // descriptor_brief.cpp:14 (a NaN coordinate is treated as outside: the reference would read
    // arbitrary memory)
    const bool inside = !(u < max_bound || u > static_cast<float>(a.cols) - max_bound || v < max_bound ||
                          v > static_cast<float>(a.rows) - max_bound) &&
                        u == u && v == v;
    if (!inside) {
        if (lane < nw) out[lane] = 0u;
        if (valid && lane == 0) *valid = 0;
        return;
    }
    {  // stage the patch: moments reach h (+1 bilinear), the pattern kPatchR, around floor(u), floor(v)
        const int reach = max(kPatchR, h + 1);
        if (2 * reach + 1 <= kStageSide) {
            const int u0 = static_cast<int>(floorf(u)), v0 = static_cast<int>(floorf(v));
            stage_patch(fr, patch, v0 - reach, u0 - reach, 2 * reach + 1);
        }
    }
    const int side = 2 * h + 1;
    const int npatch = side * side;
    float m10, m01;
    const bool exact_int = h <= 31 && (SAMPLER == FD_SAMPLE_TRUNCATE || (u == floorf(u) && v == floorf(v)));
    if (exact_int) {
        int s10 = 0, s01 = 0;
        for (int s = lane; s < npatch; s += kWave) {
            const int dx = s / side - h;
            const int dy = s - (s / side) * side - h;
            const int val = static_cast<int>(sample<SAMPLER>(fr, v + static_cast<float>(dy), u + static_cast<float>(dx)));
            s10 += dx * val;
            s01 += dy * val;
        }
        m10 = static_cast<float>(wave_sum(s10));
        m01 = static_cast<float>(wave_sum(s01));
    } else {
        // descriptor_brief.cpp:20-28 in loop order (dx outer, dy inner), lane 0 accumulating.
        float a10 = 0.0f, a01 = 0.0f;
        for (int base = 0; base < npatch; base += kWave) {
            const int s = base + lane;
            if (s < npatch) {
                const int dx = s / side - h;
                const int dy = s - (s / side) * side - h;
                stage[lane] = sample<SAMPLER>(fr, v + static_cast<float>(dy), u + static_cast<float>(dx));
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane == 0) {
                const int n = min(kWave, npatch - base);
                for (int j = 0; j < n; ++j) {
                    const int sj = base + j;
                    const int dx = sj / side - h;
                    const int dy = sj - (sj / side) * side - h;
                    const float val = stage[j];
                    a10 += static_cast<float>(dx) * val;
                    a01 += static_cast<float>(dy) * val;
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        m10 = __shfl(a10, 0, 64);
        m01 = __shfl(a01, 0, 64);
    }
    const float m = sqrtf(m01 * m01 + m10 * m10);  // :29
    if (m < kZeroFloat) {                          // :30 (RETURN_FALSE_IF; descriptor stays zero)
        if (lane < nw) out[lane] = 0u;
        if (valid && lane == 0) *valid = 0;
        return;
    }
    const float sin_t = m01 / m;  // :32
    const float cos_t = m10 / m;  // :33
    const float nsin = -sin_t;
    uint64_t bits[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = k * kWave + lane;
        bool bit = false;
        if (i < a.length) {
            const uint32_t w = kPattern[i];
            const float px1 = static_cast<float>(static_cast<int8_t>(w & 0xFFu));
            const float py1 = static_cast<float>(static_cast<int8_t>((w >> 8) & 0xFFu));
            const float px2 = static_cast<float>(static_cast<int8_t>((w >> 16) & 0xFFu));
            const float py2 = static_cast<float>(static_cast<int8_t>(w >> 24));
            // rot * Vec2(px, py) + uv with rot = [cos, -sin; sin, cos] (:35-41)
            const float x1 = cos_t * px1 + nsin * py1 + u;
            const float y1 = sin_t * px1 + cos_t * py1 + v;
            const float x2 = cos_t * px2 + nsin * py2 + u;
            const float y2 = sin_t * px2 + cos_t * py2 + v;
            const float v1 = sample<SAMPLER>(fr, y1, x1);  // :42-43
            const float v2 = sample<SAMPLER>(fr, y2, x2);
            bit = v1 < v2;  // :44-46
        }
        bits[k] = ballot(bit);
    }
    if (lane < nw) {
        const uint64_t b = bits[lane >> 1];
        out[lane] = static_cast<uint32_t>((lane & 1) ? (b >> 32) : b);
    }
    if (valid && lane == 0) *valid = 1;
}

template <int SAMPLER>
__global__ __launch_bounds__(256) void k_brief(BriefArgs a) {
    __shared__ float stage[4][kWave];
    __shared__ uint8_t patch[4][kStageSide * kStageSide];
    const int wave = static_cast<int>(threadIdx.x >> 6);
    const int64_t slot = static_cast<int64_t>(blockIdx.x) * 4 + wave;
    if (slot >= static_cast<int64_t>(a.batch) * a.stride) return;
    const int f = static_cast<int>(__builtin_amdgcn_readfirstlane(static_cast<int>(slot / a.stride)));
    const int k = static_cast<int>(__builtin_amdgcn_readfirstlane(static_cast<int>(slot - static_cast<int64_t>(f) * a.stride)));
    if (a.counts) {
        const int n = static_cast<int>(static_cast<uint32_t>(a.counts[f]) & 0x01FFFFFFu);  // detect's guard flags off
        if (k >= n) return;  // Compute sizes the descriptor list to the keypoints (descriptor.h:30-32)
    }
    const float u = a.uv[2 * slot];
    const float v = a.uv[2 * slot + 1];
    const int nw = (a.length + 31) >> 5;
    Frame fr;
    fr.rsrc = make_rsrc(a.frames + static_cast<int64_t>(f) * a.rows * a.cols,
                        static_cast<uint32_t>(a.rows) * static_cast<uint32_t>(a.cols));
    fr.cols = a.cols;
    fr.lds = nullptr;
    fr.r0 = fr.c0 = fr.side = 0;
    brief_one<SAMPLER>(a, fr, u, v, a.out_bits + slot * nw, a.out_valid ? a.out_valid + slot : nullptr, stage[wave],
                       patch[wave]);
}

}  // namespace

hipError_t launch_brief(const BriefArgs &a, hipStream_t s) {
    const int64_t waves = static_cast<int64_t>(a.batch) * a.stride;
    if (waves == 0) return hipSuccess;
    const dim3 grid(static_cast<unsigned>((waves + 3) / 4)), block(256);
    if (a.sampler == FD_SAMPLE_TRUNCATE)
        hipLaunchKernelGGL(k_brief<FD_SAMPLE_TRUNCATE>, grid, block, 0, s, a);
    else
        hipLaunchKernelGGL(k_brief<FD_SAMPLE_BILINEAR>, grid, block, 0, s, a);
    return hipGetLastError();
}

}  // namespace fdk
