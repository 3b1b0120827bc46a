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

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

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
// K10: 3x3 convolution, 64 -> 64 channels (SuperPoint conv1b, conv2a, conv2b; conv3a as two 64-channel
// output blocks: stride 1, padding 1) with its bias and ReLU and, for the layers a MaxPool2d(2, 2) follows,
// the pooling, as an implicit GEMM on mfma_f32_16x16x32_f16 (M = 64 output channels, N = pixels, K = 9 taps
// x 64 input channels; fp16 products, f32 sums). Two tiles in flight per CU: with one wave per SIMD (the
// round-5 form) the tile's staging and epilogue ran between its matrix phases and the matrix cores idled
// half the time (rocprofv3 at conv1b: SQ_VALU_MFMA_BUSY_CYCLES 49.5 % of the kernel's cycles,
// profiles/r06_sp_k10_ab.txt). Here a workgroup of 8 waves holds the packed filter once ([tap][co][ci],
// 72 KiB) and two 8 x 32-pixel input tiles (43 KiB each, 16-byte chunks of 8 channels XOR-swizzled by
// column): waves 0-3 and 4-7 are two groups, and in each phase (one barrier per phase) one group runs the
// K loop of its tile while the other, on the same SIMDs, writes its previous tile's outputs, stages its
// next tile into LDS from registers and issues the loads of the tile after -- vector-memory and VALU work
// beside the partner's matrix instructions. A wave computes 16 columns x 4 rows x 64 channels (16
// accumulators; the K loop by (column shift, channel half) with each group's 6 input rows reused by the
// three row taps) as D = W x P (a lane holds 4 consecutive channels of one pixel), so the epilogue stores
// from registers: v_permlane16_swap pairs the lanes of adjacent channel quads into 16-byte runs of 8
// channels (whole 2 KiB per 16 pixels per row, no LDS staging), and the 2x2 pool takes its column partner
// by DPP. Persistent grid, one workgroup per CU, tiles dealt so that the 32 workgroups of an XCD work on
// neighbouring tiles (their halo rows and columns come from that XCD's L2). The epilogue rounds the sum to
// half, adds the bias in half (= the float add rounded, as a bias-free convolution + fd_nn_bias_relu),
// applies the ReLU; the pool takes the max of the four biased sums, then the ReLU.
constexpr int kPpRows = 8, kPpCols = 32, kPpInRows = kPpRows + 2, kPpInCols = kPpCols + 2;
constexpr int kPpInChunks = kPpInRows * kPpInCols * 8;  // 16-byte chunks of a group's input tile
constexpr int kPpPer = (kPpInChunks + 255) / 256;       // per thread of a group

template <bool POOL>
__global__ __launch_bounds__(512) void k_conv3x3_c64_pp(const u4 *x, const u4 *wpk, const _Float16 *bias, u4 *y,
                                                        int n, int h, int w, int ystride, int yoff) {
    __shared__ u4 Wl[9 * 64 * 8];
    __shared__ u4 In[2][kPpInChunks];
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
    u4 pre[kPpPer];
    auto fetch = [&](int k) {
        const int tile = k * G + L;
        const int tx = tile % tw, t2 = tile / tw, ty = t2 % th, f = t2 / th;
        const int r0 = ty * kPpRows, c0 = tx * kPpCols;
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
    auto stage = [&]() {
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
            stage();
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
            if (p < K) kloop();  // (s_setprio 1 here measured slower, profiles/r06_sp_fused_ab.txt)
        } else {
            if (p >= 1) epilogue(p - 1);
            if (p + 1 < K) stage();
            if (p + 3 < K) fetch(p + 3);
        }
        __syncthreads();
    }
}

}  // namespace

hipError_t launch_conv3x3_c64(const void *x, const void *wpk, const void *bias, void *y, int n, int h, int w, int pool,
                              int y_channels, int y_offset, hipStream_t s) {
    const int ystride = y_channels / 8, yoff = y_offset / 8;
    const int64_t tiles = static_cast<int64_t>(n) * ((h + kPpRows - 1) / kPpRows) * ((w + kPpCols - 1) / kPpCols);
    if (tiles == 0) return hipSuccess;
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>(tiles, 256));  // (persistent: one workgroup per CU)
    const u4 *xv = static_cast<const u4 *>(x), *wv = static_cast<const u4 *>(wpk);
    const _Float16 *bv = static_cast<const _Float16 *>(bias);
    u4 *yv = static_cast<u4 *>(y);
    if (pool)
        hipLaunchKernelGGL(k_conv3x3_c64_pp<true>, dim3(grid), dim3(512), 0, s, xv, wv, bv, yv, n, h, w, ystride, yoff);
    else
        hipLaunchKernelGGL(k_conv3x3_c64_pp<false>, dim3(grid), dim3(512), 0, s, xv, wv, bv, yv, n, h, w, ystride, yoff);
    return hipGetLastError();
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
