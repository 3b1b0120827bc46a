// SuperPoint post-processing for gfx950, around a network that runs in
// PyTorch-ROCm (feature_detector_amd/superpoint.py).
//
// Reference: NNFeaturePointDetector, src/nn_feature_point_detector/nn_feature_point_detector.cpp
//   CreateMask (:59-73)                      -> border test here + K0 prior boxes (fd_points.hip)
//   SelectKeypointCandidatesFromHeatMap (:128-139) -> k_heat_candidates: every heatmap value
//       > kMinResponse becomes a candidate (unordered list + level-0 key histogram, as K1 emits)
//   SelectGoodFeaturesFromCandidates (:141-155)   -> K4 (fd_select.hip) with tie_idx_desc: the
//       multimap is walked from crbegin, i.e. response descending and, among equal responses,
//       raster index descending (equal keys are inserted at the upper bound of their range)
//   ExtractDescriptorsForSelectedFeatures (:163-193) -> k_nn_desc: bilinear sampling of the
//       1/8-resolution descriptor map, the reference's float sequence (-ffp-contract=off)
#include "fd_device.h"
#include "fd_kernels.h"

namespace fdk {
namespace {

constexpr int kHeatBlock = 256;
constexpr int kHeatRounds = 64;  // pixels per thread: a workgroup covers 16,384 consecutive pixels
constexpr int kHeatUnroll = 4;   // loads in flight per thread

constexpr int kHeatStage = 1024;  // candidates a wave stages in LDS before appending them to the list

// One workgroup = kHeatRounds * 256 consecutive pixels of one frame (coalesced f32 loads). Heatmap
// values cluster in few bins and a frame has many candidates, so neither the list append nor the
// level-0 histogram may use one global atomic per candidate (same-address atomics serialise): each
// wave stages its candidates in LDS and appends them with one atomic per flush, and the workgroup's
// histogram is accumulated in LDS and flushed once (one atomic per non-empty bin).
__global__ __launch_bounds__(kHeatBlock) void k_heat_candidates(HeatArgs a) {
    __shared__ uint32_t hist[kHistBins];
    __shared__ float st_r[kHeatBlock / kWave][kHeatStage];
    __shared__ uint32_t st_i[kHeatBlock / kWave][kHeatStage];
    const int f = blockIdx.y;
    const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    for (int b = tid; b < kHistBins; b += kHeatBlock) hist[b] = 0;
    __syncthreads();
    const int64_t npx = static_cast<int64_t>(a.rows) * a.cols;
    const float *h = a.heat + static_cast<int64_t>(f) * npx;
    const int64_t blk0 = static_cast<int64_t>(blockIdx.x) * (kHeatRounds * kHeatBlock);
    const uint32_t *fmask = a.mask ? a.mask + static_cast<int64_t>(f) * a.rows * a.mask_wpr : nullptr;
    float *dr = a.list_resp + static_cast<int64_t>(f) * a.list_cap;
    uint32_t *di = a.list_idx + static_cast<int64_t>(f) * a.list_cap;
    int staged = 0;  // wave-uniform
    auto flush = [&]() {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&a.list_count[f], static_cast<uint32_t>(staged));
        base = __builtin_amdgcn_readfirstlane(base);
        for (int k = lane; k < staged; k += kWave) {
            const uint64_t pos = static_cast<uint64_t>(base) + k;
            if (pos < static_cast<uint64_t>(a.list_cap)) {
                dr[pos] = st_r[w][k];
                di[pos] = st_i[w][k];
            }
        }
        staged = 0;
    };
    bool over = false;
    for (int r0 = 0; r0 < kHeatRounds; r0 += kHeatUnroll) {
        float v[kHeatUnroll];
#pragma unroll
        for (int j = 0; j < kHeatUnroll; ++j) {
            const int64_t p = blk0 + static_cast<int64_t>(r0 + j) * kHeatBlock + tid;
            v[j] = p < npx ? h[p] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < kHeatUnroll; ++j) {
            const int64_t p = blk0 + static_cast<int64_t>(r0 + j) * kHeatBlock + tid;
            bool ok = p < npx && v[j] > a.thr;  // :133-135 (NaN never passes)
            if (ok) {
                const int r = static_cast<int>(p / a.cols);
                const int c = static_cast<int>(p - static_cast<int64_t>(r) * a.cols);
                // CreateMask (:61-68): the kInvalidBoundary outermost rows/columns are 0; prior boxes (:69-71)
                ok = r >= a.border && r < a.rows - a.border && c >= a.border && c < a.cols - a.border;
                if (ok && fmask) ok = (fmask[static_cast<int64_t>(r) * a.mask_wpr + (c >> 5)] >> (c & 31)) & 1u;
            }
            const uint64_t m = ballot(ok);
            if (m == 0) continue;
            if (ok) {
                const int k = mbcnt64(m, staged);
                st_r[w][k] = v[j];
                st_i[w][k] = static_cast<uint32_t>(p);
                over = over || v[j] > a.vmax;
                atomicAdd(&hist[((float_key(v[j]) - a.key_base) << a.key_lz) >> 20], 1u);
            }
            staged += popc64(m);
            if (staged > kHeatStage - kWave) flush();
        }
    }
    if (staged) flush();
    if (__syncthreads_or(over) && tid == 0) atomicOr(&a.value_flag[f], 0x80000000u);  // outside the key map
    uint32_t *gh = a.hist0 + static_cast<int64_t>(f) * kHistBins;
    for (int b = tid; b < kHistBins; b += kHeatBlock) {
        const uint32_t n = hist[b];
        if (n) atomicAdd(&gh[b], n);
    }
}

// One wave per (frame, feature slot); lanes over descriptor channels.
__global__ __launch_bounds__(256) void k_nn_desc(NnDescArgs a) {
    const int64_t slot = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (slot >= static_cast<int64_t>(a.batch) * a.stride) return;
    const int f = static_cast<int>(slot / a.stride);
    const int k = static_cast<int>(slot - static_cast<int64_t>(f) * a.stride);
    if (a.counts && k >= static_cast<int>(static_cast<uint32_t>(a.counts[f]) & 0x01FFFFFFu)) return;
    const float x = a.xy[2 * slot], y = a.xy[2 * slot + 1];
    // :170-178
    const float row = y / 8.0f;
    const float col = x / 8.0f;
    const int32_t int_row = static_cast<int32_t>(row);
    const int32_t int_col = static_cast<int32_t>(col);
    const float sub_row = row - floorf(row);
    const float sub_col = col - floorf(col);
    const float inv_sub_row = 1.0f - sub_row;
    const float inv_sub_col = 1.0f - sub_col;
    const float w0 = inv_sub_col * inv_sub_row, w1 = sub_col * inv_sub_row, w2 = inv_sub_col * sub_row,
                w3 = sub_col * sub_row;
    // :184-187 (row / col ranges of the channel map; the last row and column are excluded)
    const bool inside = int_row >= 0 && int_row < a.map_rows - 1 && int_col >= 0 && int_col < a.map_cols - 1;
    const int64_t plane = static_cast<int64_t>(a.map_rows) * a.map_cols;
    const float *m = a.map + static_cast<int64_t>(f) * a.channels * plane;
    float *o = a.out + slot * a.channels;
    // element (channel j, row, col): NCHW j * plane + row * cols + col; NHWC (row * cols + col) * C + j
    const int64_t sj = a.nhwc ? 1 : plane;
    const int64_t sp = a.nhwc ? a.channels : 1;
    const int64_t p00 = (static_cast<int64_t>(int_row) * a.map_cols + int_col) * sp;
    const int64_t dc = sp, dr = static_cast<int64_t>(a.map_cols) * sp;
    for (int j = lane_id(); j < a.channels; j += kWave) {
        float d = 0.0f;
        if (inside) {
            const float *mp = m + j * sj + p00;
            d = w0 * mp[0] + w1 * mp[dc] + w2 * mp[dr] + w3 * mp[dr + dc];  // :188-189
        }
        o[j] = d;
    }
}

// SuperPoint's detector head after convPb (the network's own output stage: softmax over a cell's 65
// channels, the dustbin dropped, pixel_shuffle(8) into the cell's 8x8 pixels), in one pass from the fp16
// channels-last logits instead of PyTorch's float copy, softmax, slice and shuffle (four HBM passes over
// the map). A workgroup takes 32 cells of one cell row: 8 lanes per cell hold 8 channels each (lane 0 of
// the group also the dustbin), the max and the sum of exp(x - max) are reduced over the 8 lanes, and the
// probabilities go through LDS so that each of the 8 output rows is written as one contiguous run.
constexpr int kHeatCells = 32;
__global__ __launch_bounds__(256) void k_nn_heat_softmax(const _Float16 *semi, const _Float16 *bias, float *heat, int hc,
                                                         int wc) {
    __shared__ float pr[kHeatCells][65];
    __shared__ _Float16 lg[kHeatCells * 65 + 65];  // the group's logits (contiguous in memory), then the bias
    const int tid = static_cast<int>(threadIdx.x), cell = tid >> 3, part = tid & 7;
    const int j0 = static_cast<int>(blockIdx.x) * kHeatCells, i = static_cast<int>(blockIdx.y), b = static_cast<int>(blockIdx.z);
    const int cn = min(kHeatCells, wc - j0);
    // the group's cells are one contiguous run of cn * 65 halves: staged with coalesced loads
    const _Float16 *src = semi + ((static_cast<int64_t>(b) * hc + i) * wc + j0) * 65;
    for (int k = tid; k < cn * 65; k += 256) lg[k] = src[k];
    if (tid < 65) lg[kHeatCells * 65 + tid] = bias ? bias[tid] : static_cast<_Float16>(0.0f);
    __syncthreads();
    const int j = j0 + cell;
    const bool in = j < wc;
    // (bias: convPb's bias added to the bias-free convolution's half output, in half: a half add is the
    // float add rounded to half; a zero bias adds nothing)
    const _Float16 *cl = lg + (in ? cell : 0) * 65, *bl = lg + kHeatCells * 65;
    float v[9];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = static_cast<float>(static_cast<_Float16>(cl[part * 8 + k] + bl[part * 8 + k]));
    v[8] = part == 0 ? static_cast<float>(static_cast<_Float16>(cl[64] + bl[64])) : -INFINITY;
    float m = v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmaxf(m, v[k]);
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) m = fmaxf(m, __shfl_xor(m, o));
    float e[8], sum = part == 0 ? expf(v[8] - m) : 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        e[k] = expf(v[k] - m);
        sum += e[k];
    }
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) sum += __shfl_xor(sum, o);
#pragma unroll
    for (int k = 0; k < 8; ++k) pr[cell][part * 8 + k] = e[k] / sum;
    __syncthreads();
    const int64_t w = static_cast<int64_t>(wc) * 8;
    float *dst = heat + (static_cast<int64_t>(b) * hc * 8 + static_cast<int64_t>(i) * 8) * w + static_cast<int64_t>(j0) * 8;
    if (!in) return;
#pragma unroll
    for (int r = 0; r < 8; ++r) __builtin_nontemporal_store(pr[cell][r * 8 + part], &dst[r * w + tid]);
}

// SuperPoint's descriptor head after convDb: each cell's c-channel vector divided by its L2 norm
// (clamped to 1e-12), fp16 channels-last in, float channels-last out, one wave per cell (8 channels per
// lane and round).
// (bias, optional: convDb's bias added in half first, as for the heat). A cell of c <= 256 channels takes
// c / 8 lanes (several cells per wave); wider cells one wave each.
__global__ __launch_bounds__(256) void k_nn_desc_normalize(const _Float16 *x, const _Float16 *bias, float *y, int64_t cells,
                                                           int c) {
    const int groups = c >> 3;
    const int span = groups <= 8 ? 8 : groups <= 16 ? 16 : groups <= 32 ? 32 : kWave;  // lanes per cell
    const int per_wave = kWave / span, lane = lane_id(), sub = lane % span;
    const int64_t cell = (static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6)) * per_wave + lane / span;
    const bool in = cell < cells;
    typedef _Float16 h8v __attribute__((ext_vector_type(8)));
    const h8v *src = reinterpret_cast<const h8v *>(x + (in ? cell : 0) * c);
    const h8v *bv = reinterpret_cast<const h8v *>(bias);
    float ss = 0.0f;
    for (int g = sub; g < groups; g += span) {
        h8v h = src[g];
        if (bias) h = h + bv[g];
#pragma unroll
        for (int k = 0; k < 8; ++k) ss += static_cast<float>(h[k]) * static_cast<float>(h[k]);
    }
    for (int o = 1; o < span; o <<= 1) ss += __shfl_xor(ss, o);
    const float nrm = fmaxf(sqrtf(ss), 1e-12f);
    if (!in) return;
    float *dst = y + cell * c;
    for (int g = sub; g < groups; g += span) {
        h8v h = src[g];
        if (bias) h = h + bv[g];
        // (plain stores: nontemporal ones measured 92 -> 114 us here)
        float4 *dv = reinterpret_cast<float4 *>(dst);
        dv[2 * g] = make_float4(static_cast<float>(h[0]) / nrm, static_cast<float>(h[1]) / nrm, static_cast<float>(h[2]) / nrm,
                                static_cast<float>(h[3]) / nrm);
        dv[2 * g + 1] = make_float4(static_cast<float>(h[4]) / nrm, static_cast<float>(h[5]) / nrm,
                                    static_cast<float>(h[6]) / nrm, static_cast<float>(h[7]) / nrm);
    }
}

}  // namespace

hipError_t launch_nn_heat_softmax(const void *semi, const void *bias, float *heat, int n, int hc, int wc, hipStream_t s) {
    if (n <= 0 || hc <= 0 || wc <= 0) return hipSuccess;
    const dim3 grid(static_cast<unsigned>((wc + kHeatCells - 1) / kHeatCells), static_cast<unsigned>(hc),
                    static_cast<unsigned>(n));
    hipLaunchKernelGGL(k_nn_heat_softmax, grid, dim3(256), 0, s, static_cast<const _Float16 *>(semi),
                       static_cast<const _Float16 *>(bias), heat, hc, wc);
    return hipGetLastError();
}

hipError_t launch_nn_desc_normalize(const void *x, const void *bias, float *y, int64_t cells, int c, hipStream_t s) {
    if (cells <= 0) return hipSuccess;
    const int groups = c >> 3;
    const int per_wave = groups <= 8 ? 8 : groups <= 16 ? 4 : groups <= 32 ? 2 : 1;
    const int64_t waves = (cells + per_wave - 1) / per_wave;
    hipLaunchKernelGGL(k_nn_desc_normalize, dim3(static_cast<unsigned>((waves + 3) / 4)), dim3(256), 0, s,
                       static_cast<const _Float16 *>(x), static_cast<const _Float16 *>(bias), y, cells, c);
    return hipGetLastError();
}

hipError_t launch_heat_candidates(const HeatArgs &a, hipStream_t s) {
    if (a.blocks_per_frame == 0 || a.batch == 0) return hipSuccess;
    hipLaunchKernelGGL(k_heat_candidates, dim3(static_cast<unsigned>(a.blocks_per_frame), static_cast<unsigned>(a.batch)),
                       dim3(kHeatBlock), 0, s, a);
    return hipGetLastError();
}

int heat_blocks_per_frame(int64_t npx) {
    return static_cast<int>((npx + kHeatRounds * kHeatBlock - 1) / (kHeatRounds * kHeatBlock));
}

hipError_t launch_nn_desc(const NnDescArgs &a, hipStream_t s) {
    const int64_t waves = static_cast<int64_t>(a.batch) * a.stride;
    if (waves == 0) return hipSuccess;
    hipLaunchKernelGGL(k_nn_desc, dim3(static_cast<unsigned>((waves + 3) / 4)), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace fdk
