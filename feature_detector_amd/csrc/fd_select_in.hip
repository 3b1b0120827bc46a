// Caller-supplied candidates -> the selection's list format (fd_points_select, the seam of a
// FeaturePointDetector subclass whose ComputeCandidates runs outside this library,
// feature_point_detector.h:44 / feature_point_detector.cpp:20). The lists then go through the same
// k_select as the built-in detectors' candidates (SelectGoodFeatures, :54-88).
//
// Entry i of frame f lands at list position i, so the list keeps the order ComputeCandidates pushed
// the candidates in: FD_TIES_REFERENCE re-sorts exactly that sequence with the reference's std::sort.
// Each workgroup accumulates its share of the level-0 key histogram in LDS and flushes it once.
// HBM-bound: 12 B read + 8 B written per candidate. The keypoint-list models' post-processing
// (fd_nn_select_list) uses the same kernel on (u, v) int64 keypoints plus k_nn_pick for the
// descriptor rows.
#include "fd_device.h"
#include "fd_kernels.h"

namespace fdk {
namespace {

constexpr int kInBlock = 256;

__global__ __launch_bounds__(kInBlock) void k_cand_lists(CandInArgs a) {
    __shared__ uint32_t hist[kHistBins];
    const int f = blockIdx.y, tid = threadIdx.x;
    for (int b = tid; b < kHistBins; b += kInBlock) hist[b] = 0;
    __syncthreads();
    const int64_t want = a.counts[f];
    const bool count_ok = want >= 0 && want <= a.stride && want <= a.list_cap;
    const int64_t n = count_ok ? want : 0;
    const float *r = a.resp + static_cast<int64_t>(f) * a.stride;
    const int32_t *xs = a.x + static_cast<int64_t>(f) * a.stride;
    const int32_t *ys = a.y + static_cast<int64_t>(f) * a.stride;
    float *dr = a.list_resp + static_cast<int64_t>(f) * a.list_cap;
    uint32_t *di = a.list_idx + static_cast<int64_t>(f) * a.list_cap;
    bool bad = false;
    const int64_t step = static_cast<int64_t>(gridDim.x) * kInBlock;
    const bool keep_order = a.border < 0;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kInBlock + tid; i < n; i += step) {
        uint32_t u = __float_as_uint(r[i]);
        int32_t x, y;
        if (a.kp) {  // (u, v) int64 pairs; outside the int32 range is outside the frame
            const int64_t ku = a.kp[2 * (static_cast<int64_t>(f) * a.stride + i)];
            const int64_t kv = a.kp[2 * (static_cast<int64_t>(f) * a.stride + i) + 1];
            x = (ku >= 0 && ku < a.cols) ? static_cast<int32_t>(ku) : -1;
            y = (kv >= 0 && kv < a.rows) ? static_cast<int32_t>(kv) : -1;
        } else {
            x = xs[i];
            y = ys[i];
        }
        // the reference indexes mask_(row, col) with them (:64-66): they must lie inside the frame;
        // NaN has no place in the comparator's order (bit tests: no float arithmetic, denormals kept)
        const bool ok = x >= 0 && x < a.cols && y >= 0 && y < a.rows && (u & 0x7FFFFFFFu) <= 0x7F800000u;
        if ((u << 1) == 0u) u = 0u;  // -0 compares equal to +0 (:58-60): one key for both
        float v = __uint_as_float(u);
        bad = bad || !ok;
        if (!ok) v = 0.0f;
        const uint32_t idx = ok ? static_cast<uint32_t>(y) * static_cast<uint32_t>(a.cols) + static_cast<uint32_t>(x) : 0u;
        if (keep_order) {
            dr[i] = v;
            di[i] = idx;
        } else {
            // CreateMask (nn_feature_point_detector.cpp:61-67): a candidate in the border is never
            // selected and never draws a box, so it is left out of the list
            if (!ok || y < a.border || y >= a.rows - a.border || x < a.border || x >= a.cols - a.border) continue;
            const uint32_t pos = atomicAdd(&a.list_count[f], 1u);
            if (pos >= a.list_cap) continue;  // (cannot happen: list_cap >= count)
            dr[pos] = v;
            di[pos] = idx;
        }
        atomicAdd(&hist[((float_key(v) - a.key_base) << a.key_lz) >> 20], 1u);
    }
    if (__syncthreads_or(bad) && tid == 0) atomicOr(&a.bad[f], 0x80000000u);
    if (blockIdx.x == 0 && tid == 0) {
        if (keep_order) a.list_count[f] = static_cast<uint32_t>(n);
        if (!count_ok) atomicOr(&a.bad[f], 0x80000000u);
    }
    uint32_t *gh = a.hist0 + static_cast<int64_t>(f) * kHistBins;
    for (int b = tid; b < kHistBins; b += kInBlock) {
        const uint32_t c = hist[b];
        if (c) atomicAdd(&gh[b], c);
    }
}

// One wave per (frame, selected feature): the candidate at the feature's pixel that the selection
// visited first -- highest score, then highest index (scores equal at one pixel: the later one) --
// found by a scan of the frame's list, then its descriptor row copied
// (DirectlySelectGoodFeaturesWithDescriptors, nn_feature_point_detector.cpp:223-227).
__global__ __launch_bounds__(256) void k_nn_pick(NnPickArgs a) {
    const int64_t slot = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (slot >= static_cast<int64_t>(a.batch) * a.out_stride) return;
    const int f = static_cast<int>(slot / a.out_stride);
    const int k = static_cast<int>(slot - static_cast<int64_t>(f) * a.out_stride);
    if (k >= a.n_sel[f]) return;
    const int lane = lane_id();
    const int64_t fx = static_cast<int64_t>(a.xy[2 * slot]), fy = static_cast<int64_t>(a.xy[2 * slot + 1]);
    int64_t n = a.counts[f];
    n = n < 0 ? 0 : (n > a.stride_in ? a.stride_in : n);
    const int64_t *kp = a.kp + 2 * static_cast<int64_t>(f) * a.stride_in;
    const float *sc = a.scores + static_cast<int64_t>(f) * a.stride_in;
    uint64_t best = 0;  // (score key << 32) | (index + 1); 0 = none
    for (int64_t i = lane; i < n; i += kWave) {
        if (kp[2 * i] == fx && kp[2 * i + 1] == fy) {
            uint32_t u = __float_as_uint(sc[i]);
            if ((u << 1) == 0u) u = 0u;
            const uint64_t key = (static_cast<uint64_t>(float_key(__uint_as_float(u))) << 32) | static_cast<uint64_t>(i + 1);
            best = key > best ? key : best;
        }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t other = __shfl_xor(best, o);
        best = other > best ? other : best;
    }
    float *out = a.out + slot * a.dim;
    if (best == 0) {  // (cannot happen: every selected feature came from the list)
        for (int j = lane; j < a.dim; j += kWave) out[j] = 0.0f;
        return;
    }
    const int64_t i = static_cast<int64_t>(best & 0xFFFFFFFFull) - 1;
    const float *d = a.desc + (static_cast<int64_t>(f) * a.stride_in + i) * a.dim;
    for (int j = lane; j < a.dim; j += kWave) out[j] = d[j];
}

}  // namespace

hipError_t launch_nn_pick(const NnPickArgs &a, hipStream_t s) {
    const int64_t waves = static_cast<int64_t>(a.batch) * a.out_stride;
    if (waves == 0) return hipSuccess;
    hipLaunchKernelGGL(k_nn_pick, dim3(static_cast<unsigned>((waves + 3) / 4)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_cand_lists(const CandInArgs &a, int64_t max_count, hipStream_t s) {
    if (a.batch == 0) return hipSuccess;
    // ~16 candidates per thread, at least one workgroup per frame (it stores the list count)
    const int64_t g = (max_count + 16 * kInBlock - 1) / (16 * kInBlock);
    const unsigned gx = static_cast<unsigned>(g < 1 ? 1 : (g > 1024 ? 1024 : g));
    hipLaunchKernelGGL(k_cand_lists, dim3(gx, static_cast<unsigned>(a.batch)), dim3(kInBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace fdk
