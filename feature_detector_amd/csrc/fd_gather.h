// First-chunk gather of the per-frame selection (SelectGoodFeatures, feature_point_detector.cpp:54-88),
// shared by k_gather (its own kernel, fd_select.hip) and the fused tail of the candidate kernels
// (fd_points.hip, small batches): G workgroups of one frame each derive the frame's first level-0
// chunk (the highest histogram bins holding <= kSelectChunk candidates) and append the 64-bit keys of
// their slice of the candidate list to pre_keys[f]; k_select then starts from those keys instead of a
// pass over the whole list by one workgroup.
#pragma once

#include "fd_device.h"
#include "fd_kernels.h"

namespace fdk {

// Selection key: the response through the frame's key map (order-preserving, injective on the
// candidates' response range; see SelectArgs::key_base), then ~idx so that equal responses order by
// ascending raster index (tie_idx_desc: idx, descending, SuperPoint's multimap walk order).
__device__ __forceinline__ uint32_t sel_key32(float resp, uint32_t key_base, int key_lz) {
    return (float_key(resp) - key_base) << key_lz;
}
__device__ __forceinline__ uint64_t sel_key64(float resp, uint32_t idx, uint32_t key_base, int key_lz, int tie_desc) {
    return (static_cast<uint64_t>(sel_key32(resp, key_base, key_lz)) << 32) | static_cast<uint64_t>(tie_desc ? idx : ~idx);
}

constexpr int kGatherPerThread = 16;  // list responses per thread and round

struct GatherView {
    const float *lresp;      // the frame's candidate list
    const uint32_t *lidx;
    int64_t n;               // candidates in it (clamped to the capacity)
    const uint32_t *hist;    // the frame's level-0 histogram (complete)
    uint32_t key_base;
    int key_lz, tie_desc;
    uint64_t *pk;            // the frame's pre_keys [kSelectChunk] (k_gather) or wide_keys [kWideKeys] (k_wide_gather)
    uint32_t *pcount;        // the frame's pre_count / wide_count
    uint32_t limit;          // keys the chunk may hold: kSelectChunk or kWideKeys
};

struct GatherLds {
    uint32_t S[kHistBins + 1];
    uint32_t wtot[16];
    uint32_t wg_base;
};

// Workgroup g of G (NT threads) for one frame. Every thread of the workgroup calls it.
template <int NT>
__device__ __forceinline__ void gather_first_chunk(const GatherView &v, int g, int G, GatherLds &L) {
    static_assert(kHistBins % NT == 0 && NT % kWave == 0 && NT / kWave <= 16, "gather shape");
    constexpr int kBpt = kHistBins / NT;  // histogram bins per thread
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const int64_t s0 = v.n * g / G, s1 = v.n * (g + 1) / G;
    // this slice's responses, in flight during the histogram scan (slices <= kGatherPerThread * NT)
    float rr[kGatherPerThread];
    const bool fits = s1 - s0 <= static_cast<int64_t>(kGatherPerThread) * NT;
#pragma unroll
    for (int k = 0; k < kGatherPerThread; ++k)
        rr[k] = (fits && s1 > s0) ? v.lresp[min(s0 + tid + static_cast<int64_t>(k) * NT, s1 - 1)] : 0.0f;
    for (int b = tid; b < kHistBins; b += NT) L.S[b] = v.hist[b];
    __syncthreads();
    {  // in-place suffix sums, kBpt contiguous bins per thread
        const int b0 = tid * kBpt;
        uint32_t val[kBpt], sacc = 0;
#pragma unroll
        for (int q = 0; q < kBpt; ++q) sacc += (val[q] = L.S[b0 + q]);
        const uint32_t incl = wave_suffix_add(sacc);
        if (lane == 0) L.wtot[wave] = incl;
        __syncthreads();
        uint32_t after = 0;
        after = wave_total_add((lane > wave && lane < NT / kWave) ? L.wtot[lane] : 0u);
        uint32_t run = incl - sacc + after;
#pragma unroll
        for (int q = kBpt - 1; q >= 0; --q) {
            run += val[q];
            L.S[b0 + q] = run;
        }
        if (tid == 0) L.S[kHistBins] = 0;
        __syncthreads();
    }
    int lo = 0, hi = kHistBins;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (L.S[mid] <= v.limit) hi = mid; else lo = mid + 1;
    }
    if (lo >= kHistBins || L.S[lo] == 0) return;  // top bin alone exceeds a chunk (k_select descends)
    const uint32_t k32lo = static_cast<uint32_t>(lo) << 20;
    __syncthreads();  // every thread has read S / wtot before they are reused
    // One reservation per workgroup and round: hits counted per thread (bit mask), placed by a block
    // prefix, then a single atomic on the frame's counter.
    auto emit = [&](const float (&r)[kGatherPerThread], int64_t base) {
        uint32_t hm = 0;
#pragma unroll
        for (int k = 0; k < kGatherPerThread; ++k) {
            const int64_t i = base + tid + static_cast<int64_t>(k) * NT;
            hm |= static_cast<uint32_t>(i < s1 && sel_key32(r[k], v.key_base, v.key_lz) >= k32lo) << k;
        }
        const uint32_t cntt = __popc(hm);
        const uint32_t incl = wave_incl_add(cntt);
        if (lane == kWave - 1) L.wtot[wave] = incl;
        __syncthreads();
        uint32_t before = 0, total = 0;
        for (int q = 0; q < NT / kWave; ++q) {
            const uint32_t wq = L.wtot[q];
            before += q < wave ? wq : 0u;
            total += wq;
        }
        if (tid == 0) L.wg_base = total ? atomicAdd(v.pcount, total) : 0u;
        __syncthreads();
        uint32_t pos = L.wg_base + before + incl - cntt;
        while (hm) {
            const int k = __builtin_ctz(hm);
            hm &= hm - 1u;
            const int64_t i = base + tid + static_cast<int64_t>(k) * NT;
            if (pos < v.limit)
                v.pk[pos] = sel_key64(r[k], v.lidx[i], v.key_base, v.key_lz, v.tie_desc);
            ++pos;
        }
        __syncthreads();  // wtot / wg_base reuse
    };
    if (fits) {
        emit(rr, s0);
    } else {
        for (int64_t base = s0; base < s1; base += static_cast<int64_t>(kGatherPerThread) * NT) {
            float r2[kGatherPerThread];
#pragma unroll
            for (int k = 0; k < kGatherPerThread; ++k)
                r2[k] = v.lresp[min(base + tid + static_cast<int64_t>(k) * NT, s1 - 1)];
            emit(r2, base);
        }
    }
}

}  // namespace fdk
