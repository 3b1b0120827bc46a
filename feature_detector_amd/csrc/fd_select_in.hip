// Caller-supplied candidates -> the selection's list format (fd_points_select, the seam of a
// FeaturePointDetector subclass whose ComputeCandidates runs outside this library,
// feature_point_detector.h:44 / feature_point_detector.cpp:20). The lists then go through the same
// k_select as the built-in detectors' candidates (SelectGoodFeatures, :54-88).
//
// Entry i of frame f lands at list position i, so the list keeps the order ComputeCandidates pushed
// the candidates in: FD_TIES_REFERENCE re-sorts exactly that sequence with the reference's std::sort.
// Each workgroup accumulates its share of the level-0 key histogram in LDS and flushes it once.
// HBM-bound: 12 B read + 8 B written per candidate.
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
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kInBlock + tid; i < n; i += step) {
        uint32_t u = __float_as_uint(r[i]);
        const int32_t x = xs[i], y = ys[i];
        // the reference indexes mask_(row, col) with them (:64-66): they must lie inside the frame;
        // NaN has no place in the comparator's order (bit tests: no float arithmetic, denormals kept)
        const bool ok = x >= 0 && x < a.cols && y >= 0 && y < a.rows && (u & 0x7FFFFFFFu) <= 0x7F800000u;
        if ((u << 1) == 0u) u = 0u;  // -0 compares equal to +0 (:58-60): one key for both
        float v = __uint_as_float(u);
        bad = bad || !ok;
        if (!ok) v = 0.0f;
        dr[i] = v;
        di[i] = ok ? static_cast<uint32_t>(y) * static_cast<uint32_t>(a.cols) + static_cast<uint32_t>(x) : 0u;
        atomicAdd(&hist[((float_key(v) - a.key_base) << a.key_lz) >> 20], 1u);
    }
    if (__syncthreads_or(bad) && tid == 0) atomicOr(&a.bad[f], 0x80000000u);
    if (blockIdx.x == 0 && tid == 0) {
        a.list_count[f] = static_cast<uint32_t>(n);
        if (!count_ok) atomicOr(&a.bad[f], 0x80000000u);
    }
    uint32_t *gh = a.hist0 + static_cast<int64_t>(f) * kHistBins;
    for (int b = tid; b < kHistBins; b += kInBlock) {
        const uint32_t c = hist[b];
        if (c) atomicAdd(&gh[b], c);
    }
}

}  // namespace

hipError_t launch_cand_lists(const CandInArgs &a, int64_t max_count, hipStream_t s) {
    if (a.batch == 0) return hipSuccess;
    // ~16 candidates per thread, at least one workgroup per frame (it stores the list count)
    const int64_t g = (max_count + 16 * kInBlock - 1) / (16 * kInBlock);
    const unsigned gx = static_cast<unsigned>(g < 1 ? 1 : (g > 1024 ? 1024 : g));
    hipLaunchKernelGGL(k_cand_lists, dim3(gx, static_cast<unsigned>(a.batch)), dim3(kInBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace fdk
