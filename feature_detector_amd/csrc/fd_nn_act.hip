// Bias + ReLU (+ 2x2 max pool) of the NN detectors' convolutions, one pass over an NHWC fp16 activation
// (gfx950). PyTorch-ROCm runs a biased convolution as the bias-free MIOpen/CK convolution, then a
// broadcast add, then the ReLU and the pooling as separate elementwise passes: three to four full
// reads and writes of the largest tensors of the network (64 x 640 x 480 x 64 halves = 2.5 GB for the
// first layers). Here the convolution runs without its bias and this kernel applies bias, ReLU and
// (for the layers a MaxPool2d(2, 2) follows) the pooling while the activation is read once.
// Arithmetic as PyTorch's half ops: x + b in float (opmath), rounded to half (round to nearest even),
// ReLU as max(v, 0) on the rounded value, pooling as the max of the four (exact).
#include "fd_device.h"
#include "fd_kernels.h"

namespace fdk {
namespace {

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

// 8 channels (16 bytes) of one pixel: relu(x + b) per half.
__device__ __forceinline__ u4 bias_relu8(u4 xv, u4 bv) {
    u4 r;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t xw = xv[k], bw = bv[k];
        _Float16 lo = static_cast<_Float16>(static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(xw))) +
                                            static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(bw))));
        _Float16 hi = static_cast<_Float16>(static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(xw >> 16))) +
                                            static_cast<float>(__builtin_bit_cast(_Float16, static_cast<uint16_t>(bw >> 16))));
        lo = lo > static_cast<_Float16>(0.0f) ? lo : static_cast<_Float16>(0.0f);
        hi = hi > static_cast<_Float16>(0.0f) ? hi : static_cast<_Float16>(0.0f);
        r[k] = static_cast<uint32_t>(__builtin_bit_cast(uint16_t, lo)) | (static_cast<uint32_t>(__builtin_bit_cast(uint16_t, hi)) << 16);
    }
    return r;
}

// Elementwise max of two relu'd vectors (non-negative halves: their bit patterns order like integers).
__device__ __forceinline__ u4 max8(u4 a, u4 b) {
    u4 r;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t lo = max(a[k] & 0xFFFFu, b[k] & 0xFFFFu), hi = max(a[k] >> 16, b[k] >> 16);
        r[k] = lo | (hi << 16);
    }
    return r;
}

__global__ __launch_bounds__(256) void k_bias_relu(const u4 *x, const u4 *bias, u4 *y, int64_t nvec, int cvec) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < nvec;
         i += static_cast<int64_t>(gridDim.x) * 256)
        y[i] = bias_relu8(x[i], bias[i % cvec]);
}

// y [n][h/2][w/2][c] = max over the 2x2 window of relu(x + b); one thread per output 8-channel vector.
__global__ __launch_bounds__(256) void k_bias_relu_pool(const u4 *x, const u4 *bias, u4 *y, int n, int h, int w,
                                                        int cvec) {
    const int ho = h >> 1, wo = w >> 1;
    const int64_t total = static_cast<int64_t>(n) * ho * wo * cvec;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < total;
         i += static_cast<int64_t>(gridDim.x) * 256) {
        const int cv = static_cast<int>(i % cvec);
        int64_t p = i / cvec;
        const int xo = static_cast<int>(p % wo);
        p /= wo;
        const int yo = static_cast<int>(p % ho);
        const int64_t b = p / ho;
        const int64_t r0 = ((b * h + 2 * yo) * w + 2 * xo) * cvec + cv;  // (2yo, 2xo)
        const int64_t r1 = r0 + static_cast<int64_t>(w) * cvec;          // (2yo + 1, 2xo)
        const u4 bv = bias[cv];
        const u4 a = bias_relu8(x[r0], bv), c = bias_relu8(x[r0 + cvec], bv);
        const u4 d = bias_relu8(x[r1], bv), e = bias_relu8(x[r1 + cvec], bv);
        y[i] = max8(max8(a, c), max8(d, e));
    }
}

// First layer of the NN encoders (SuperPoint conv1a: one input channel, 3x3, stride 1, zero padding 1)
// with its bias and ReLU, written straight to the channels-last fp16 activation. The 3x3 x 1 filter has
// 9 MACs per output, so the layer is write-bound (64 halves per pixel out, one in): the library
// convolution takes 1.3 ms per 64 640x480 frames and the bias + ReLU pass another 1 ms
// (tools/sp_miopen_probe.py); here one pass writes the 2.5 GB once. Each thread keeps one 8-channel
// group's 72 weights in registers (cv fixed per thread: the grid stride is a multiple of the channel
// groups) and produces that group for one pixel per step: 9 input halves (from the block's LDS copy of
// the three input rows; direct 2-byte global gathers left the layer bound by the address unit),
// float FMA accumulation in tap order, the sum rounded to half, then + bias in float rounded to half and
// the ReLU (as the bias-free convolution + fd_nn_bias_relu path rounds), one 16-byte store.
constexpr int kConv1MaxW = 4096;  // frame width the row staging holds
#ifndef FD_NN_NT_STORES
#define FD_NN_NT_STORES 1  // conv1a's activation written with nontemporal stores (A/B: 0): 589 -> 449 us
#endif
#ifndef FD_C64_NT_STORES
#define FD_C64_NT_STORES 1  // K10's outputs likewise (A/B: 0): conv2a / conv1b +22 / +27 us alone, but the forward
                            // 4.54-4.61 vs 4.69-4.71 ms (the layers after them find the caches unpolluted)
#endif
__device__ __forceinline__ void nn_store(u4 *p, u4 v) {
#if FD_C64_NT_STORES
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

__global__ __launch_bounds__(256) void k_conv3x3_c1_bias_relu(const _Float16 *x, const _Float16 *wt,
                                                              const _Float16 *bias, u4 *y, int n, int h, int w,
                                                              int cvec) {
    const int per = 256 / cvec;  // pixels per block step
    const int cv = static_cast<int>(threadIdx.x) % cvec;
    float wf[8][9], bf[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
        for (int t = 0; t < 9; ++t) wf[k][t] = static_cast<float>(wt[(cv * 8 + k) * 9 + t]);
        bf[k] = static_cast<float>(bias[cv * 8 + k]);
    }
    // one image row per block step (no per-pixel index division): its three input rows staged in LDS
    // (zero outside the frame) by 16-byte-per-thread loads where aligned, then the row's pixels over the
    // threads reading their 9 taps from LDS (8 threads of a pixel read the same words: broadcast)
    __shared__ _Float16 rin[3][kConv1MaxW + 2];
    const int rows = n * h;  // (< 2^31: checked on the host)
    for (int fr = static_cast<int>(blockIdx.x); fr < rows; fr += static_cast<int>(gridDim.x)) {
        const int yy = fr % h;
        const _Float16 *f = x + static_cast<int64_t>(fr - yy) * w;  // frame base
        for (int i = static_cast<int>(threadIdx.x); i < 3 * (w + 2); i += 256) {
            const int dy = i / (w + 2), c = i - dy * (w + 2) - 1, r = yy + dy - 1;
            rin[dy][c + 1] = (r >= 0 && r < h && c >= 0 && c < w) ? f[static_cast<int64_t>(r) * w + c]
                                                                   : static_cast<_Float16>(0.0f);
        }
        __syncthreads();
        u4 *yrow = y + static_cast<int64_t>(fr) * w * cvec;
        for (int xx = static_cast<int>(threadIdx.x) / cvec; xx < w; xx += per) {
            float in[9];
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) in[dy * 3 + dx] = static_cast<float>(rin[dy][xx + dx]);
            u4 o;
#pragma unroll
            for (int k2 = 0; k2 < 4; ++k2) {
                uint32_t packed = 0;
#pragma unroll
                for (int hlf = 0; hlf < 2; ++hlf) {
                    const int k = k2 * 2 + hlf;
                    float acc = 0.0f;
#pragma unroll
                    for (int t = 0; t < 9; ++t) acc = __builtin_fmaf(wf[k][t], in[t], acc);
                    _Float16 v = static_cast<_Float16>(static_cast<float>(static_cast<_Float16>(acc)) + bf[k]);
                    v = v > static_cast<_Float16>(0.0f) ? v : static_cast<_Float16>(0.0f);
                    packed |= static_cast<uint32_t>(__builtin_bit_cast(uint16_t, v)) << (16 * hlf);
                }
                o[k2] = packed;
            }
#if FD_NN_NT_STORES
            __builtin_nontemporal_store(o, &yrow[xx * cvec + cv]);  // (2.5 GB per SuperPoint batch: streamed past the caches)
#else
            yrow[xx * cvec + cv] = o;
#endif
        }
        __syncthreads();  // (rin reused by the next row)
    }
}

// 3x3 convolution, 64 -> 64 channels (SuperPoint conv1b, conv2a, conv2b: stride 1, padding 1), with its
// bias and ReLU and, for the layers a MaxPool2d(2, 2) follows, the pooling, as an implicit GEMM on the
// matrix cores: M = pixels, N = 64 output channels, K = 9 taps x 64 input channels, in
// mfma_f32_16x16x32_f16 steps (fp16 products, f32 sums). One workgroup (4 waves) per CU keeps the packed
// filter ([tap][co][ci], 72 KiB) in LDS and walks tiles of kCvRows rows x 64 columns: the tile's input
// pixels are staged in LDS (16-byte chunks of 8 channels, XOR-swizzled by column so that 16 lanes reading
// 16 pixels hit 8 distinct bank groups), each wave computes 16 columns x kCvRows rows x 64 channels
// (4 kCvRows accumulators), and the epilogue rounds the sum to half, adds the
// bias in float and rounds (as a bias-free convolution + fd_nn_bias_relu), applies the ReLU and the 2x2
// max within the lane (the accumulator rows are adjacent pixels, the four row blocks adjacent rows),
// stages the tile in LDS and writes it as whole 128-byte pixels.
#ifndef FD_C64_UNROLL
#define FD_C64_UNROLL 1  // the 9 taps unrolled (conv1b + conv2b 1.20 -> 0.96 ms, conv2a 556 -> 459 us per call)
#endif
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
#ifndef FD_C1_MFMA
#define FD_C1_MFMA 1  // fused conv1a on the matrix cores (0: the float FMA chain of k_conv3x3_c1_bias_relu, bit-equal to it)
#endif
#ifndef FD_C64_ROWREUSE
#define FD_C64_ROWREUSE 1  // K loop by (dx, channel half) with the input rows reused by the three dy taps
#endif
#ifndef FD_C64_ROWS
#define FD_C64_ROWS 8  // tile rows (with the row reuse: 4 rows 1,671 / 512 us, 8 rows 1,603 / 502 us for conv1b / conv2a)
#endif
constexpr int kCvRows = FD_C64_ROWS, kCvCols = 64, kCvInRows = kCvRows + 2, kCvInCols = kCvCols + 2;

// The epilogue on packed halves: the two sums rounded to half, the bias added in half (correctly rounded:
// equal to the float add rounded to half for every pair of finite halves, checked exhaustively), the
// ReLU as a max with +0 (a NaN gives 0) with the sign bit of a -0 cleared.
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h2v cv_pair(float a, float b, h2v bias2) {
    const h2v v = h2v{static_cast<_Float16>(a), static_cast<_Float16>(b)};
    return v + bias2;
}
__device__ __forceinline__ h2v cv_relu2(h2v v) {
    v = __builtin_elementwise_max(v, h2v{static_cast<_Float16>(0.0f), static_cast<_Float16>(0.0f)});
    uint32_t u = __builtin_bit_cast(uint32_t, v);
    const uint32_t sgn = u & 0x80008000u;
    u &= ~(sgn | (sgn - (sgn >> 15)));
    return __builtin_bit_cast(h2v, u);
}
[[maybe_unused]] __device__ __forceinline__ _Float16 cv_relu1(_Float16 v) {  // (the round-5 kernel's pool)
    v = __builtin_elementwise_max(v, static_cast<_Float16>(0.0f));
    const uint16_t u = __builtin_bit_cast(uint16_t, v);
    return __builtin_bit_cast(_Float16, static_cast<uint16_t>((u & 0x8000u) ? 0u : u));
}


// FUSED (SuperPoint conv1a + conv1b, fd_nn_conv3x3_c1c64): the tile's 64-channel input is conv1a itself
// (1 -> 64 channels, 3x3, bias, ReLU) recomputed from the one-channel frame rows the tile reaches (a
// 2-pixel halo), so the full-resolution 64-channel activation never goes to HBM (~2.5 GB written and
// read back, 1.55x with the halo, per 64 640x480 frames). Each thread keeps one 8-channel group's 72
// conv1a weights in registers and produces that group for 1/32 of the tile's 6 x 66 input pixels: the
// same float FMA chain in tap order, rounding to half, bias in float, rounding and ReLU as
// k_conv3x3_c1_bias_relu, so the staged values equal that kernel's output bit for bit (zero outside the
// frame: conv1b's own zero padding). x is then the [n][h][w] fp16 frame, w1 [64][9], b1 [64].
template <bool POOL, bool FUSED>
__global__ __launch_bounds__(256) void k_conv3x3_c64_mfma(const u4 *x, const u4 *wpk, const _Float16 *bias, u4 *y,
                                                          int n, int h, int w, int ystride, int yoff,
                                                          const _Float16 *w1 = nullptr, const _Float16 *b1 = nullptr) {
    __shared__ u4 Wl[9 * 64 * 8];
    __shared__ u4 In[kCvInRows * kCvInCols * 8];  // (also the output staging after the K loop)
    constexpr int kRawRows = kCvInRows + 2, kRawCols = kCvInCols + 2;
    __shared__ _Float16 raw[FUSED ? kRawRows : 1][FUSED ? kRawCols : 1];  // conv1a's input rows (FUSED)
    const int tid = static_cast<int>(threadIdx.x), lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < 9 * 64 * 8; i += 256) {
        const int ch = i & 7, row = i >> 3, co = row & 63;
        Wl[row * 8 + (ch ^ (co & 7))] = wpk[i];
    }
    h2v bv2[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) bv2[nb] = h2v{bias[nb * 16 + (lane & 15)], bias[nb * 16 + (lane & 15)]};
    const int th = (h + kCvRows - 1) / kCvRows, tw = (w + kCvCols - 1) / kCvCols;
    const int total = n * th * tw;  // (< 2^31: checked on the host)
#if FD_C1_MFMA
    // FUSED: conv1a on the matrix cores, D[16 channels][16 pixels] = W[16][K = 32] x P[K][16]: the 9 taps in
    // K 0..8 (zeros above), this lane's A fragment = channels 16 cb + (lane & 15), taps 8 (lane >> 4) ..;
    // the bias pairs of the 4 consecutive channels the lane's D fragment holds (16 cb + 4 (lane >> 4) ..)
    h8 w1a[4];
    h2v b1p[4][2];
    if constexpr (FUSED) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            const int c = cb * 16 + (lane & 15), g = lane >> 4;
#pragma unroll
            for (int e = 0; e < 8; ++e) w1a[cb][e] = 8 * g + e < 9 ? w1[c * 9 + 8 * g + e] : static_cast<_Float16>(0.0f);
            const int cd = cb * 16 + 4 * g;
            b1p[cb][0] = h2v{b1[cd], b1[cd + 1]};
            b1p[cb][1] = h2v{b1[cd + 2], b1[cd + 3]};
        }
    }
#else
    // FUSED: this thread's conv1a channel group (8 channels) and its weights
    const int cg = tid & 7;
    f2 w1f[4][9], b1f[4];
    if constexpr (FUSED) {
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) {
#pragma unroll
            for (int t = 0; t < 9; ++t)
                w1f[k2][t] = f2{static_cast<float>(w1[(cg * 8 + 2 * k2) * 9 + t]), static_cast<float>(w1[(cg * 8 + 2 * k2 + 1) * 9 + t])};
            b1f[k2] = f2{static_cast<float>(b1[cg * 8 + 2 * k2]), static_cast<float>(b1[cg * 8 + 2 * k2 + 1])};
        }
    }
#endif
    // the input tile goes through registers: the next tile's loads are issued before this tile's K loop
    // and stored to LDS after it, so their latency hides behind the matrix work (FUSED: the raw rows)
    constexpr int kChunks = kCvInRows * kCvInCols * 8, kPer = FUSED ? 1 : (kChunks + 255) / 256;
    constexpr int kRawN = kRawRows * kRawCols, kRawPer = (kRawN + 255) / 256;
    u4 pre[kPer];
    _Float16 praw[kRawPer];
    auto fetch = [&](int tile) {
        const int tx = tile % tw, t2 = tile / tw, ty = t2 % th, f = t2 / th;
        const int r0 = ty * kCvRows, c0 = tx * kCvCols;
        if constexpr (FUSED) {
            const _Float16 *xf = reinterpret_cast<const _Float16 *>(x);
#pragma unroll
            for (int k = 0; k < kRawPer; ++k) {
                const int i = tid + k * 256, rr = i / kRawCols, rc = i - rr * kRawCols;
                const int gy = r0 - 2 + rr, gx = c0 - 2 + rc;
                praw[k] = static_cast<_Float16>(0.0f);
                if (i < kRawN && tile < total && gy >= 0 && gy < h && gx >= 0 && gx < w)
                    praw[k] = xf[(static_cast<int64_t>(f) * h + gy) * w + gx];
            }
        } else {
            // through a buffer resource over the tile's frame: an out-of-frame chunk reads at an
            // offset past the resource and gets zeros (no zero fill, 32-bit offsets; the host checks
            // h * w * 128 < 2^31)
            const auto rs = make_rsrc(x + static_cast<int64_t>(min(f, n - 1)) * h * w * 8, static_cast<uint32_t>(h * w * 128));
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const int i = tid + k * 256;
                const int ch = i & 7, px = i >> 3, pc = px % kCvInCols, pr = px / kCvInCols;
                const int gy = r0 - 1 + pr, gx = c0 - 1 + pc;
                const bool ok = i < kChunks && tile < total && gy >= 0 && gy < h && gx >= 0 && gx < w;
                const int32_t off = ok ? ((gy * w + gx) * 8 + ch) * 16 : -1;
                pre[k] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
            }
        }
    };
    fetch(static_cast<int>(blockIdx.x));
    for (int tile = static_cast<int>(blockIdx.x); tile < total; tile += static_cast<int>(gridDim.x)) {
        const int tx = tile % tw, t2 = tile / tw, ty = t2 % th, f = t2 / th;
        const int r0 = ty * kCvRows, c0 = tx * kCvCols;
        __syncthreads();  // (the previous tile's staging is read out; the filter is in place)
        if constexpr (FUSED) {
#pragma unroll
            for (int k = 0; k < kRawPer; ++k) {
                const int i = tid + k * 256, rr = i / kRawCols;
                if (i < kRawN) raw[rr][i - rr * kRawCols] = praw[k];
            }
            __syncthreads();
            fetch(tile + static_cast<int>(gridDim.x));
#if FD_C1_MFMA
            // conv1a over the tile's input pixels, 16 at a time per wave: the lane's patch fragment (taps
            // 8 (lane >> 4) .. of pixel lane & 15) from the raw rows, one matrix step per 16 channels, the
            // sum rounded to half, the bias added in half, the ReLU, and the lane's 4 channels of the pixel
            // written as 8 bytes into its 16-byte chunk (zero outside the frame: conv1b's padding)
            constexpr int kInPx = kCvInRows * kCvInCols;
            for (int pb = wv; pb * 16 < kInPx; pb += 4) {
                const int px = pb * 16 + (lane & 15), g = lane >> 4;
                const int pxc = min(px, kInPx - 1);
                const int pr = pxc / kCvInCols, pc = pxc - pr * kCvInCols;
                h8 pt;
#pragma unroll
                for (int e = 0; e < 8; ++e) pt[e] = static_cast<_Float16>(0.0f);
                if (g == 0) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) pt[e] = raw[pr + e / 3][pc + e % 3];
                } else if (g == 1) {
                    pt[0] = raw[pr + 2][pc + 2];
                }
                const int gy = r0 - 1 + pr, gx = c0 - 1 + pc;
                const bool inframe = gy >= 0 && gy < h && gx >= 0 && gx < w;
#pragma unroll
                for (int cb = 0; cb < 4; ++cb) {
                    const f4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1a[cb], pt, f4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
                    const h2v lo = cv_relu2(cv_pair(d[0], d[1], b1p[cb][0])), hi = cv_relu2(cv_pair(d[2], d[3], b1p[cb][1]));
                    const int ch = cb * 16 + 4 * g;  // the lane's first channel: chunk ch / 8, half (ch & 4) / 4
                    uint2 v = make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
                    if (!inframe) v = make_uint2(0u, 0u);
                    if (px < kInPx)
                        reinterpret_cast<uint2 *>(In)[(pxc * 8 + ((ch >> 3) ^ (pc & 7))) * 2 + ((ch >> 2) & 1)] = v;
                }
            }
#else
            // conv1a over the tile's input pixels (6 x 66), 8 channels per item
            for (int px = tid >> 3; px < kCvInRows * kCvInCols; px += 32) {
                const int pr = px / kCvInCols, pc = px - pr * kCvInCols;
                const int gy = r0 - 1 + pr, gx = c0 - 1 + pc;
                u4 o = u4{0u, 0u, 0u, 0u};
                if (gy >= 0 && gy < h && gx >= 0 && gx < w) {
                    float in[9];
#pragma unroll
                    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                        for (int dx = 0; dx < 3; ++dx) in[dy * 3 + dx] = static_cast<float>(raw[pr + dy][pc + dx]);
#pragma unroll
                    for (int k2 = 0; k2 < 4; ++k2) {
                        f2 acc2 = f2{0.0f, 0.0f};
#pragma unroll
                        for (int t = 0; t < 9; ++t) acc2 = __builtin_elementwise_fma(w1f[k2][t], f2{in[t], in[t]}, acc2);
                        uint32_t packed = 0;
#pragma unroll
                        for (int hlf = 0; hlf < 2; ++hlf) {
                            _Float16 v = static_cast<_Float16>(static_cast<float>(static_cast<_Float16>(acc2[hlf])) + b1f[k2][hlf]);
                            v = v > static_cast<_Float16>(0.0f) ? v : static_cast<_Float16>(0.0f);
                            packed |= static_cast<uint32_t>(__builtin_bit_cast(uint16_t, v)) << (16 * hlf);
                        }
                        o[k2] = packed;
                    }
                }
                In[px * 8 + (cg ^ (pc & 7))] = o;
            }
#endif
            __syncthreads();
        } else {
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const int i = tid + k * 256;
                const int px = i >> 3, pc = px % kCvInCols;
                if (i < kChunks) In[px * 8 + ((i & 7) ^ (pc & 7))] = pre[k];
            }
            __syncthreads();
            fetch(tile + static_cast<int>(gridDim.x));
        }
        f4 acc[kCvRows][4];
#pragma unroll
        for (int m = 0; m < kCvRows; ++m)
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) acc[m][nb] = f4{0.0f, 0.0f, 0.0f, 0.0f};
#if FD_C64_ROWREUSE
        // K loop by (column shift dx, channel half) groups: the wave's A fragments for the group are the
        // kCvRows + 2 input rows at that shift, loaded once and used by the three taps dy = 0..2 of the
        // column (row m + dy), so each input fragment is read from LDS once per group instead of once
        // per tap (A traffic per tile halved: 36 instead of 72 fragment loads at 4 rows). The next
        // group's rows and the next tap's filter fragments are read ahead of the current MFMAs.
        auto rows_at = [&](int g, h8 (&A)[kCvRows + 2]) {
            const int dx = g >> 1, kh = g & 1;
            const int chunk = kh * 4 + (lane >> 4);
            const int pc = wv * 16 + (lane & 15) + dx;
#pragma unroll
            for (int r = 0; r < kCvRows + 2; ++r)
                A[r] = __builtin_bit_cast(h8, In[(r * kCvInCols + pc) * 8 + (chunk ^ (pc & 7))]);
        };
        auto filt_at = [&](int g, int dy, h8 (&B)[4]) {
            const int dx = g >> 1, kh = g & 1, tap = dy * 3 + dx;
            const int chunk = kh * 4 + (lane >> 4);
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                const int co = nb * 16 + (lane & 15);
                B[nb] = __builtin_bit_cast(h8, Wl[(tap * 64 + co) * 8 + (chunk ^ (co & 7))]);
            }
        };
        h8 Ar[2][kCvRows + 2], Bf[2][4];
        rows_at(0, Ar[0]);
        filt_at(0, 0, Bf[0]);
#pragma unroll
        for (int g = 0; g < 6; ++g) {
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                const int it = g * 3 + dy;
                if (dy == 0 && g + 1 < 6) rows_at(g + 1, Ar[(g + 1) & 1]);
                if (it + 1 < 18) filt_at(dy == 2 ? g + 1 : g, dy == 2 ? 0 : dy + 1, Bf[(it + 1) & 1]);
#pragma unroll
                for (int m = 0; m < kCvRows; ++m)
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        acc[m][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ar[g & 1][m + dy], Bf[it & 1][nb], acc[m][nb], 0, 0, 0);
            }
        }
#else
        // the 18 K steps (tap, channel half) with the next step's fragments read from LDS before this
        // step's matrix instructions, so the LDS latency hides behind them (one wave per SIMD: no other
        // wave would cover it)
        auto frag = [&](int step, h8 (&A)[kCvRows], h8 (&B)[4]) {
            const int tap = step >> 1, kh = step & 1;
            const int dy = tap / 3, dx = tap - dy * 3;
            const int chunk = kh * 4 + (lane >> 4);
            const int pc = wv * 16 + (lane & 15) + dx;
#pragma unroll
            for (int m = 0; m < kCvRows; ++m)
                A[m] = __builtin_bit_cast(h8, In[((m + dy) * kCvInCols + pc) * 8 + (chunk ^ (pc & 7))]);
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                const int co = nb * 16 + (lane & 15);
                B[nb] = __builtin_bit_cast(h8, Wl[(tap * 64 + co) * 8 + (chunk ^ (co & 7))]);
            }
        };
        h8 A0[kCvRows], B0[4], A1[kCvRows], B1[4];
        frag(0, A0, B0);
#pragma unroll
        for (int step = 0; step < 18; step += 2) {
            frag(step + 1, A1, B1);
#pragma unroll
            for (int m = 0; m < kCvRows; ++m)
#pragma unroll
                for (int nb = 0; nb < 4; ++nb)
                    acc[m][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0[m], B0[nb], acc[m][nb], 0, 0, 0);
            if (step + 2 < 18) frag(step + 2, A0, B0);
#pragma unroll
            for (int m = 0; m < kCvRows; ++m)
#pragma unroll
                for (int nb = 0; nb < 4; ++nb)
                    acc[m][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1[m], B1[nb], acc[m][nb], 0, 0, 0);
        }
#endif
        __syncthreads();  // (In is reused as the output staging)
        _Float16 *st = reinterpret_cast<_Float16 *>(In);
        const int col4 = wv * 16 + (lane >> 4) * 4;  // the accumulator's first pixel column in the tile
        if constexpr (POOL) {
            // staging [kCvRows / 2 pooled rows][32 pooled columns][64 channels]
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                const int co = nb * 16 + (lane & 15);
#pragma unroll
                for (int pr = 0; pr < kCvRows / 2; ++pr)
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        // max of the four biased sums, then the ReLU (= the max of the four ReLUs, NaN
                        // included: max skips a NaN unless all four are, and the ReLU maps that to 0)
                        const h2v m2 = __builtin_elementwise_max(cv_pair(acc[2 * pr][nb][2 * q], acc[2 * pr][nb][2 * q + 1], bv2[nb]),
                                                                 cv_pair(acc[2 * pr + 1][nb][2 * q], acc[2 * pr + 1][nb][2 * q + 1], bv2[nb]));
                        st[(pr * 32 + col4 / 2 + q) * 64 + co] = cv_relu1(__builtin_elementwise_max(m2.x, m2.y));
                    }
            }
            __syncthreads();
            const int ho = h >> 1, wo = w >> 1;
            for (int i = tid; i < kCvRows / 2 * 32 * 8; i += 256) {
                const int ch = i & 7, px = i >> 3, pc = px & 31, pr = px >> 5;
                const int gy = r0 / 2 + pr, gx = c0 / 2 + pc;
                if (gy < ho && gx < wo) nn_store(&y[((static_cast<int64_t>(f) * ho + gy) * wo + gx) * ystride + yoff + ch], In[px * 8 + ch]);
            }
        } else {
            // staging [kCvRows rows][64 columns][64 channels]
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                const int co = nb * 16 + (lane & 15);
#pragma unroll
                for (int m = 0; m < kCvRows; ++m)
#pragma unroll
                    for (int r = 0; r < 4; r += 2) {
                        const h2v v = cv_relu2(cv_pair(acc[m][nb][r], acc[m][nb][r + 1], bv2[nb]));
                        st[(m * kCvCols + col4 + r) * 64 + co] = v.x;
                        st[(m * kCvCols + col4 + r + 1) * 64 + co] = v.y;
                    }
            }
            __syncthreads();
            for (int i = tid; i < kCvRows * kCvCols * 8; i += 256) {
                const int ch = i & 7, px = i >> 3, pc = px % kCvCols, pr = px / kCvCols;
                const int gy = r0 + pr, gx = c0 + pc;
                if (gy < h && gx < w) nn_store(&y[((static_cast<int64_t>(f) * h + gy) * w + gx) * ystride + yoff + ch], In[px * 8 + ch]);
            }
        }
    }
}

// K10, two tiles in flight per CU (the default for fd_nn_conv3x3_c64; the kernel above stays for the fused
// conv1a path and as the A/B baseline, FD_C64_PP=0). With one wave per SIMD the tile's staging and epilogue
// ran between its matrix phases and the matrix cores idled half the time (rocprofv3 at conv1b:
// SQ_VALU_MFMA_BUSY_CYCLES 49.5 % of the kernel's cycles, gpurun_out k10 r06). Here a workgroup of 8 waves
// holds the packed filter once (72 KiB) and two 8 x 32-pixel input tiles (43 KiB each): waves 0-3 and 4-7
// are two groups, and in each phase (one barrier per phase) one group runs the K loop of its tile while the
// other, on the same SIMDs, writes its previous tile's outputs, stages its next tile into LDS from
// registers and issues the loads of the tile after -- vector-memory and VALU work beside the partner's
// matrix instructions. A wave computes 16 columns x 4 rows x 64 channels (16 accumulators) with the
// operands swapped relative to the kernel above (D = W x P: a lane holds 4 consecutive channels of one
// pixel), so the epilogue stores from registers: v_permlane16_swap pairs the lanes of adjacent channel
// quads into 16-byte runs of 8 channels (whole 2 KiB per 16 pixels per row, no LDS staging), and the 2x2
// pool takes its column partner by DPP. Persistent grid, one workgroup per CU, tiles dealt so that the 32
// workgroups of an XCD work on neighbouring tiles (their halo rows and columns come from that XCD's L2).
// Same arithmetic as the kernel above: fp16 products summed in f32, the sum rounded to half, the bias
// added in half (= the float add rounded), ReLU, pool = max of the four biased sums then the ReLU.
#ifndef FD_C64_PP
#define FD_C64_PP 1
#endif
#ifndef FD_C64_PRIO
#define FD_C64_PRIO 0
#endif
constexpr int kPpRows = 8, kPpCols = 32, kPpInRows = kPpRows + 2, kPpInCols = kPpCols + 2;
constexpr int kPpInChunks = kPpInRows * kPpInCols * 8;  // 16-byte chunks of a group's input tile
constexpr int kPpPer = (kPpInChunks + 255) / 256;       // per thread of a group

// FUSED (fd_nn_conv3x3_c1c64: SuperPoint conv1a + conv1b): the group's input tile is conv1a itself,
// computed in the housekeeping phase on the matrix cores (D[16 channels][16 pixels] = W1[16][K = the 9 taps
// padded to 32] x P[K][16]: 4 matrix instructions per 16 pixels of an input row, at most 36 per wave and
// tile beside the partner's 288) from the one-channel frame: a wave owns input rows q, q + 4, q + 8 of the
// tile, loads the 3 x 36 frame pixels each needs two phases ahead (two 2-byte loads per lane and row),
// and builds the patch fragments from a per-wave LDS copy of them; the sum rounded to half, the bias
// added in half, the ReLU, zero outside the frame (conv1b's padding).
// x is then the [n][h][w] fp16 frame, w1 [64][9], b1 [64]; the 64-channel activation never goes to HBM.
template <bool POOL, bool FUSED>
__global__ __launch_bounds__(512) void k_conv3x3_c64_pp(const u4 *x, const u4 *wpk, const _Float16 *bias, u4 *y,
                                                        int n, int h, int w, int ystride, int yoff,
                                                        const _Float16 *w1 = nullptr, const _Float16 *b1 = nullptr) {
    __shared__ u4 Wl[9 * 64 * 8];
    __shared__ u4 In[2][kPpInChunks];
    __shared__ uint16_t Raw[FUSED ? 4 : 1][3 * (kPpInCols + 2)];  // FUSED: a housekeeping wave's frame rows
    const int tid = static_cast<int>(threadIdx.x), lane = tid & 63, wv = tid >> 6;
    const int grp = wv >> 2, cb = wv & 1, rh = (wv >> 1) & 1, gtid = tid & 255;
    for (int i = tid; i < 9 * 64 * 8; i += 512) {
        const int ch = i & 7, row = i >> 3, co = row & 63;
        Wl[row * 8 + (ch ^ (co & 7))] = wpk[i];
    }
    // the lane's channels of block nb: nb * 16 + 4 (lane >> 4) + 0..3, as two bias pairs
    const int g4 = lane >> 4, px = lane & 15;
    h2v bz[4][2];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
        const int c = nb * 16 + 4 * g4;
        bz[nb][0] = h2v{bias[c], bias[c + 1]};
        bz[nb][1] = h2v{bias[c + 2], bias[c + 3]};
    }
    const int th = (h + kPpRows - 1) / kPpRows, tw = (w + kPpCols - 1) / kPpCols;
    const int total = n * th * tw;  // (< 2^31: checked on the host)
    const int G = static_cast<int>(gridDim.x), b = static_cast<int>(blockIdx.x);
    const int L = G == 256 ? (b & 7) * 32 + (b >> 3) : b;  // (blocks b, b + 8, ... share an XCD)
    const int K = L < total ? (total - L + G - 1) / G : 0;  // this workgroup's tiles: k G + L, k < K
    u4 *const in = In[grp];
    u4 pre[FUSED ? 1 : kPpPer];
    // FUSED: conv1a's weights as the lane's A fragments (channels 16 cb + (lane & 15), taps 8 (lane >> 4) ..),
    // its bias pairs for the lane's D channels 16 cb + 4 (lane >> 4) .., and the lane's patch fragments of
    // the wave's pixel blocks (blocks q, q + 4, ... of the tile's 10 x 34 input pixels)
    constexpr int kRawC = kPpInCols + 2, kRawN = 3 * kRawC;  // an input row's frame patch rows: 3 x 36
    constexpr int kWRows = (kPpInRows + 3) / 4;                // input rows per wave (3)
    h8 w1a[FUSED ? 4 : 1];
    uint32_t rawv[FUSED ? kWRows : 1][2];
    h2v b1p[FUSED ? 4 : 1][2];
    const int q4 = wv & 3;
    if constexpr (FUSED) {
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
            const int c = c4 * 16 + px;
#pragma unroll
            for (int e = 0; e < 8; ++e) w1a[c4][e] = 8 * g4 + e < 9 ? w1[c * 9 + 8 * g4 + e] : static_cast<_Float16>(0.0f);
            const int cd = c4 * 16 + 4 * g4;
            b1p[c4][0] = h2v{b1[cd], b1[cd + 1]};
            b1p[c4][1] = h2v{b1[cd + 2], b1[cd + 3]};
        }
    }
    auto fetch = [&](int k) {
        const int tile = k * G + L;
        const int tx = tile % tw, t2 = tile / tw, ty = t2 % th, f = t2 / th;
        const int r0 = ty * kPpRows, c0 = tx * kPpCols;
        if constexpr (FUSED) {
            // the frame pixels of the wave's input rows' patches (zero outside the frame)
            const uint16_t *xf = reinterpret_cast<const uint16_t *>(x) + static_cast<int64_t>(f) * h * w;
#pragma unroll
            for (int j = 0; j < kWRows; ++j) {
                const int pr = q4 + 4 * j;
#pragma unroll
                for (int e2 = 0; e2 < 2; ++e2) {
                    const int e = lane + 64 * e2, dyr = e / kRawC, cc = e - dyr * kRawC;
                    const int yy = r0 - 2 + pr + dyr, xx = c0 - 2 + cc;
                    rawv[j][e2] = (pr < kPpInRows && e < kRawN && yy >= 0 && yy < h && xx >= 0 && xx < w)
                                      ? static_cast<uint32_t>(xf[static_cast<int64_t>(yy) * w + xx]) : 0u;
                }
            }
            return;
        }
        // a buffer resource over the tile's frame: out-of-frame chunks read past it and get zeros
        const auto rs = make_rsrc(x + static_cast<int64_t>(f) * h * w * 8, static_cast<uint32_t>(h * w * 128));
#pragma unroll
        for (int k2 = 0; k2 < kPpPer; ++k2) {
            const int i = gtid + k2 * 256;
            const int ch = i & 7, p = i >> 3, pr = p / kPpInCols, pc = p - pr * kPpInCols;
            const int gy = r0 - 1 + pr, gx = c0 - 1 + pc;
            const bool ok = i < kPpInChunks && gy >= 0 && gy < h && gx >= 0 && gx < w;
            const int32_t off = ok ? ((gy * w + gx) * 8 + ch) * 16 : -1;
            pre[k2] = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        }
    };
    auto stage = [&](int k) {
        if constexpr (FUSED) {
            // conv1a of the wave's input rows: the row's patch rows into the wave's LDS copy, then per 16
            // pixels the lane's patch fragment (taps 8 (lane >> 4) ..), one matrix step per 16 channels, and
            // the lane's 4 channels of its pixel as 8 bytes into the pixel's (swizzled) 16-byte chunk
            const int tile = k * G + L;
            const int tx = tile % tw, t2 = tile / tw, ty = t2 % th;
            const int r0 = ty * kPpRows, c0 = tx * kPpCols;
            uint16_t *const raw = Raw[q4];
#pragma unroll
            for (int j = 0; j < kWRows; ++j) {
                const int pr = q4 + 4 * j;
                if (pr >= kPpInRows) break;  // (wave-uniform)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();  // (the previous row's fragments are read)
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int e2 = 0; e2 < 2; ++e2)
                    if (lane + 64 * e2 < kRawN) raw[lane + 64 * e2] = static_cast<uint16_t>(rawv[j][e2]);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const int gy = r0 - 1 + pr;
#pragma unroll
                for (int bk = 0; bk < (kPpInCols + 15) / 16; ++bk) {
                    const int pc = min(bk * 16 + px, kPpInCols - 1);
                    uint32_t t[4] = {0u, 0u, 0u, 0u};
                    if (g4 == 0) {
#pragma unroll
                        for (int e = 0; e < 8; ++e) t[e >> 1] |= static_cast<uint32_t>(raw[(e / 3) * kRawC + pc + e % 3]) << (16 * (e & 1));
                    } else if (g4 == 1) {
                        t[0] = raw[2 * kRawC + pc + 2];
                    }
                    const h8 pfr = __builtin_bit_cast(h8, u4{t[0], t[1], t[2], t[3]});
                    const int gx = c0 - 1 + pc;
                    const bool inframe = gy >= 0 && gy < h && gx >= 0 && gx < w;
                    const int pi = pr * kPpInCols + pc;
#pragma unroll
                    for (int c4 = 0; c4 < 4; ++c4) {
                        const f4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1a[c4], pfr, f4{0.0f, 0.0f, 0.0f, 0.0f}, 0, 0, 0);
                        const h2v lo = cv_relu2(cv_pair(d[0], d[1], b1p[c4][0])), hi = cv_relu2(cv_pair(d[2], d[3], b1p[c4][1]));
                        const int ch = c4 * 16 + 4 * g4;  // the lane's first channel: chunk ch / 8, half (ch & 4) / 4
                        uint2 v = make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
                        if (!inframe) v = make_uint2(0u, 0u);
                        if (bk * 16 + px < kPpInCols) reinterpret_cast<uint2 *>(in)[(pi * 8 + ((ch >> 3) ^ (pc & 7))) * 2 + ((ch >> 2) & 1)] = v;
                    }
                }
            }
            return;
        }
#pragma unroll
        for (int k2 = 0; k2 < kPpPer; ++k2) {
            const int i = gtid + k2 * 256;
            const int p = i >> 3, pc = p % kPpInCols;
            if (i < kPpInChunks) in[p * 8 + ((i & 7) ^ (pc & 7))] = pre[k2];
        }
    };
    f4 acc[4][4];
    // the K loop of one tile: groups (column shift dx, channel half) of the 6 input rows the wave's 4 rows
    // reach, each used by the three row taps; the next group's rows and the next tap's filter fragments
    // are read ahead of the current matrix instructions
    auto kloop = [&]() {
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) acc[m][nb] = f4{0.0f, 0.0f, 0.0f, 0.0f};
        auto rows_at = [&](int g, h8 (&A)[6]) {
            const int dx = g >> 1, kh = g & 1;
            const int chunk = kh * 4 + g4;
            const int pc = cb * 16 + px + dx;
#pragma unroll
            for (int r = 0; r < 6; ++r)
                A[r] = __builtin_bit_cast(h8, in[((rh * 4 + r) * kPpInCols + pc) * 8 + (chunk ^ (pc & 7))]);
        };
        auto filt_at = [&](int g, int dy, h8 (&B)[4]) {
            const int dx = g >> 1, kh = g & 1, tap = dy * 3 + dx;
            const int chunk = kh * 4 + g4;
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                const int co = nb * 16 + px;
                B[nb] = __builtin_bit_cast(h8, Wl[(tap * 64 + co) * 8 + (chunk ^ (co & 7))]);
            }
        };
        h8 Ar[2][6], Bf[2][4];
        rows_at(0, Ar[0]);
        filt_at(0, 0, Bf[0]);
#pragma unroll
        for (int g = 0; g < 6; ++g) {
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                const int it = g * 3 + dy;
                if (dy == 0 && g + 1 < 6) rows_at(g + 1, Ar[(g + 1) & 1]);
                if (it + 1 < 18) filt_at(dy == 2 ? g + 1 : g, dy == 2 ? 0 : dy + 1, Bf[(it + 1) & 1]);
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        acc[m][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(Bf[it & 1][nb], Ar[g & 1][m + dy], acc[m][nb], 0, 0, 0);
            }
        }
    };
    // a lane's 4 channels of block nb (row m) rounded, biased and ReLU'd, as two dwords
    auto quad = [&](int m, int nb, uint32_t &lo, uint32_t &hi) {
        lo = __builtin_bit_cast(uint32_t, cv_relu2(cv_pair(acc[m][nb][0], acc[m][nb][1], bz[nb][0])));
        hi = __builtin_bit_cast(uint32_t, cv_relu2(cv_pair(acc[m][nb][2], acc[m][nb][3], bz[nb][1])));
    };
    // channel blocks (2 pr, 2 pr + 1) of rows a lane holds as 4 dwords -> 8 consecutive channels: after the
    // swap, lane row g4 holds block 2 pr + (g4 & 1), channels 8 (g4 >> 1) .. + 7 (chunk 2 (2 pr + (g4 & 1)) + (g4 >> 1))
    auto pair_swap = [&](uint32_t (&v)[4]) {  // v = {lo(nb0), hi(nb0), lo(nb1), hi(nb1)} -> one 16-byte run
        typedef uint32_t u2v __attribute__((ext_vector_type(2)));
        const u2v s0 = __builtin_bit_cast(u2v, __builtin_amdgcn_permlane16_swap(v[0], v[2], false, false));
        const u2v s1 = __builtin_bit_cast(u2v, __builtin_amdgcn_permlane16_swap(v[1], v[3], false, false));
        v[0] = s0[0], v[2] = s0[1], v[1] = s1[0], v[3] = s1[1];
    };
    auto epilogue = [&](int k) {
        const int tile = k * G + L;
        const int tx = tile % tw, t2 = tile / tw, ty = t2 % th, f = t2 / th;
        const int r0 = ty * kPpRows + rh * 4, c0 = tx * kPpCols + cb * 16;
        if constexpr (POOL) {
            const int ho = h >> 1, wo = w >> 1;
            const int gx = (c0 + px) >> 1;
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) {
                const int gy = (r0 >> 1) + pr;
#pragma unroll
                for (int pp = 0; pp < 2; ++pp) {
                    uint32_t v[4];
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int nb = 2 * pp + j;
#pragma unroll
                        for (int hf = 0; hf < 2; ++hf) {
                            // max of the two rows' biased sums, then of the column pair (lane ^ 1), then the ReLU
                            h2v m2 = __builtin_elementwise_max(cv_pair(acc[2 * pr][nb][2 * hf], acc[2 * pr][nb][2 * hf + 1], bz[nb][hf]),
                                                               cv_pair(acc[2 * pr + 1][nb][2 * hf], acc[2 * pr + 1][nb][2 * hf + 1], bz[nb][hf]));
                            const uint32_t mu = __builtin_bit_cast(uint32_t, m2);
                            const uint32_t nbr = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(
                                static_cast<int>(mu), static_cast<int>(mu), 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
                            m2 = __builtin_elementwise_max(m2, __builtin_bit_cast(h2v, nbr));
                            v[2 * j + hf] = __builtin_bit_cast(uint32_t, cv_relu2(m2));
                        }
                    }
                    pair_swap(v);
                    const int chunk = 2 * (2 * pp + (g4 & 1)) + (g4 >> 1);
                    if (!(px & 1) && gy < ho && gx < wo)
                        nn_store(&y[((static_cast<int64_t>(f) * ho + gy) * wo + gx) * ystride + yoff + chunk],
                                 u4{v[0], v[1], v[2], v[3]});
                }
            }
        } else {
            const int gx = c0 + px;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int gy = r0 + m;
#pragma unroll
                for (int pp = 0; pp < 2; ++pp) {
                    uint32_t v[4];
                    quad(m, 2 * pp, v[0], v[1]);
                    quad(m, 2 * pp + 1, v[2], v[3]);
                    pair_swap(v);
                    const int chunk = 2 * (2 * pp + (g4 & 1)) + (g4 >> 1);
                    if (gy < h && gx < w)
                        nn_store(&y[((static_cast<int64_t>(f) * h + gy) * w + gx) * ystride + yoff + chunk], u4{v[0], v[1], v[2], v[3]});
                }
            }
        }
    };
    // prologue: group 0 stages tile 0 and holds tile 2 in registers, group 1 holds tile 1
    if (grp == 0) {
        if (K > 0) {
            fetch(0);
            stage(0);
        }
        if (K > 2) fetch(2);
    } else if (K > 1) {
        fetch(1);
    }
    __syncthreads();
    // phase p: group p & 1 computes tile p; the other group writes tile p - 1, stages tile p + 1 and loads
    // tile p + 3 (all its own tiles: k = grp mod 2). Every wave runs the K + 1 phases (one barrier each).
    for (int p = 0; p <= K; ++p) {
        if ((p & 1) == grp) {
#if FD_C64_PRIO
            __builtin_amdgcn_s_setprio(1);  // the matrix phase wins issue arbitration over the partner's
            if (p < K) kloop();
            __builtin_amdgcn_s_setprio(0);
#else
            if (p < K) kloop();
#endif
        } else {
            if (p >= 1) epilogue(p - 1);
            if (p + 1 < K) stage(p + 1);
            if (p + 3 < K) fetch(p + 3);
        }
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_conv3x3_c64(const void *x, const void *wpk, const void *bias, void *y, int n, int h, int w, int pool,
                              int y_channels, int y_offset, hipStream_t s, const void *w1, const void *b1) {
    const int ystride = y_channels / 8, yoff = y_offset / 8;
    const u4 *xv = static_cast<const u4 *>(x), *wv = static_cast<const u4 *>(wpk);
    const _Float16 *bv = static_cast<const _Float16 *>(bias), *w1h = static_cast<const _Float16 *>(w1),
                   *b1h = static_cast<const _Float16 *>(b1);
    u4 *yv = static_cast<u4 *>(y);
#if FD_C64_PP
    {  // two tiles in flight per CU, a persistent grid of one workgroup per CU (w1: conv1a fused)
        const int64_t pt = static_cast<int64_t>(n) * ((h + kPpRows - 1) / kPpRows) * ((w + kPpCols - 1) / kPpCols);
        if (pt == 0) return hipSuccess;
        const unsigned pg = static_cast<unsigned>(std::min<int64_t>(pt, 256));
        if (w1 && pool)
            hipLaunchKernelGGL((k_conv3x3_c64_pp<true, true>), dim3(pg), dim3(512), 0, s, xv, wv, bv, yv, n, h, w, ystride, yoff, w1h, b1h);
        else if (w1)
            hipLaunchKernelGGL((k_conv3x3_c64_pp<false, true>), dim3(pg), dim3(512), 0, s, xv, wv, bv, yv, n, h, w, ystride, yoff, w1h, b1h);
        else if (pool)
            hipLaunchKernelGGL((k_conv3x3_c64_pp<true, false>), dim3(pg), dim3(512), 0, s, xv, wv, bv, yv, n, h, w, ystride, yoff, nullptr, nullptr);
        else
            hipLaunchKernelGGL((k_conv3x3_c64_pp<false, false>), dim3(pg), dim3(512), 0, s, xv, wv, bv, yv, n, h, w, ystride, yoff, nullptr, nullptr);
        return hipGetLastError();
    }
#else
    // (the round-5 kernel: A/B builds with -DFD_C64_PP=0 only)
    const int64_t tiles = static_cast<int64_t>(n) * ((h + kCvRows - 1) / kCvRows) * ((w + kCvCols - 1) / kCvCols);
    if (tiles == 0) return hipSuccess;
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(tiles, 1024));
    if (w1) {  // conv1a fused into the staging (fd_nn_conv3x3_c1c64)
        if (pool)
            hipLaunchKernelGGL((k_conv3x3_c64_mfma<true, true>), dim3(grid), dim3(256), 0, s, xv, wv, bv, yv, n, h, w, ystride,
                               yoff, w1h, b1h);
        else
            hipLaunchKernelGGL((k_conv3x3_c64_mfma<false, true>), dim3(grid), dim3(256), 0, s, xv, wv, bv, yv, n, h, w, ystride,
                               yoff, w1h, b1h);
    } else if (pool) {
        hipLaunchKernelGGL((k_conv3x3_c64_mfma<true, false>), dim3(grid), dim3(256), 0, s, xv, wv, bv, yv, n, h, w, ystride,
                           yoff, nullptr, nullptr);
    } else {
        hipLaunchKernelGGL((k_conv3x3_c64_mfma<false, false>), dim3(grid), dim3(256), 0, s, xv, wv, bv, yv, n, h, w, ystride,
                           yoff, nullptr, nullptr);
    }
    return hipGetLastError();
#endif
}

hipError_t launch_conv3x3_c1_bias_relu(const void *x, const void *wt, const void *bias, void *y, int n, int h, int w,
                                       int c, hipStream_t s) {
    const int cvec = c / 8;
    const int64_t rows = static_cast<int64_t>(n) * h;
    if (rows == 0 || w == 0) return hipSuccess;
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(rows, 256 * 32));
    hipLaunchKernelGGL(k_conv3x3_c1_bias_relu, dim3(grid), dim3(256), 0, s, static_cast<const _Float16 *>(x),
                       static_cast<const _Float16 *>(wt), static_cast<const _Float16 *>(bias), static_cast<u4 *>(y), n, h,
                       w, cvec);
    return hipGetLastError();
}

hipError_t launch_bias_relu(const void *x, const void *bias, void *y, int n, int h, int w, int c, int pool,
                            hipStream_t s) {
    const int cvec = c / 8;
    const int64_t nvec = static_cast<int64_t>(n) * h * w * cvec;
    const int64_t out = pool ? nvec / 4 : nvec;
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>((out + 255) / 256, 256 * 64));
    if (out == 0) return hipSuccess;
    if (pool)
        hipLaunchKernelGGL(k_bias_relu_pool, dim3(grid), dim3(256), 0, s, static_cast<const u4 *>(x),
                           static_cast<const u4 *>(bias), static_cast<u4 *>(y), n, h, w, cvec);
    else
        hipLaunchKernelGGL(k_bias_relu, dim3(grid), dim3(256), 0, s, static_cast<const u4 *>(x),
                           static_cast<const u4 *>(bias), static_cast<u4 *>(y), nvec, cvec);
    return hipGetLastError();
}

}  // namespace fdk
