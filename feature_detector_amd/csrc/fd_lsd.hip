// LSD level-line map for gfx950: FeatureLineDetector::ComputeLineLevelAngleMap
// (Horizon1026/Feature_Detector src/feature_line_detector/feature_line_detector.cpp:56-97).
//
//   per pixel (row in [1, R-3], col in [1, C-3], :71-72):
//     ad = I(r+1,c+1) - I(r,c), bc = I(r,c+1) - I(r+1,c)            (:76-79)
//     gx = (ad + bc) / 2, gy = (ad - bc) / 2                          (:80-81)
//     norm = sqrt(gx^2 + gy^2), valid = norm > kMinValidGradientNorm  (:82-83)
//     angle = atan2f(gx, -gy) if valid                                (:85)
//   valid pixels listed in column-major scan order (:71-72, :86).
//
// gx, gy are half-integers, so gx^2 + gy^2 is exact and the correctly rounded sqrt makes `norm` and
// `valid` bit-exact. The angle uses the reference's libm: std::atan2(float, float) is glibc 2.35's
// atan2f, an fdlibm-derived float algorithm (sysdeps/ieee754/flt-32/e_atan2f.c + s_atanf.c). It is
// restated below from the published fdlibm algorithm; tests/test_lsd_atan2.py shows it equals the
// host atan2f bit for bit over the whole LSD input domain (every half-integer (gx, gy) pair).
#include "fd_device.h"
#include "fd_kernels.h"

namespace fdk {

namespace {

// fdlibm atanf (float), polynomial + 4 reduction intervals.
__device__ __forceinline__ float fd_atanf(float x) {
    constexpr float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    constexpr float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    constexpr float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                    aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                    aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                    aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const uint32_t hx = __float_as_uint(x);
    const uint32_t ix = hx & 0x7fffffffu;
    int id;
    if (ix >= 0x4c800000u) {  // |x| >= 2^26
        const float z = atanhi[3] + atanlo[3];
        return (hx >> 31) ? -z : z;
    }
    if (ix < 0x3ee00000u) {  // |x| < 7/16
        if (ix < 0x39800000u) return x;
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000u) {
            if (ix < 0x3f300000u) {
                id = 0;
                x = ((2.0f * x) - 1.0f) / (2.0f + x);
            } else {
                id = 1;
                x = (x - 1.0f) / (x + 1.0f);
            }
        } else if (ix < 0x401c0000u) {
            id = 2;
            x = (x - 1.5f) / (1.0f + (1.5f * x));
        } else {
            id = 3;
            x = -1.0f / x;
        }
    }
    float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    float hi = 0.0f, lo = 0.0f;
    switch (id) {
        case 0: hi = atanhi[0]; lo = atanlo[0]; break;
        case 1: hi = atanhi[1]; lo = atanlo[1]; break;
        case 2: hi = atanhi[2]; lo = atanlo[2]; break;
        default: hi = atanhi[3]; lo = atanlo[3]; break;
    }
    z = hi - ((x * (s1 + s2) - lo) - x);
    return (hx >> 31) ? -z : z;
}

// fdlibm atan2f(y, x) for finite inputs.
__device__ __forceinline__ float fd_atan2f(float y, float x) {
    constexpr float pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f,
                    tiny = 1.0e-30f;
    const uint32_t hx = __float_as_uint(x), hy = __float_as_uint(y);
    const uint32_t ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
    if (hx == 0x3f800000u) return fd_atanf(y);  // x == 1
    int m = static_cast<int>(((hy >> 31) & 1u) | ((hx >> 30) & 2u));
    if (iy == 0) {
        if (m <= 1) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (ix == 0) return (hy >> 31) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int k = (static_cast<int>(iy) - static_cast<int>(ix)) >> 23;
    float z;
    if (k > 26) {
        z = pi_o_2 + 0.5f * pi_lo;
        m &= 1;
    } else if (k < -26 && (hx >> 31)) {
        z = 0.0f;
    } else {
        z = fd_atanf(fabsf(y / x));
    }
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

__device__ __forceinline__ void lsd_tile(const LsdArgs &a, int &f, int &strip, int &chunk) {
    // wave-uniform (readfirstlane): row/column bounds derived from it stay in SGPRs, and the
    // per-row bound checks are scalar branches (no exec masking around the DPP moves)
    int w = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x * 4 + (threadIdx.x >> 6)));
    strip = w % a.strips;
    w /= a.strips;
    chunk = w % a.chunks;
    f = w / a.chunks;
}

// Pass 1: maps + per (column, row-chunk) valid counts and valid-row bitmasks. Lane = one column,
// walking chunk_h rows in groups of kLsdGroup; the next group's pixel loads are issued before the
// current group is computed (ping-pong register sets, so no copy on the back edge waits for them).
constexpr int kLsdGroup = 4;

__global__ __launch_bounds__(256) void k_lsd_map(LsdArgs a) {
    int f, strip, chunk;
    lsd_tile(a, f, strip, chunk);
    if (f >= a.batch) return;
    const int lane = lane_id();
    const int rows = a.rows, cols = a.cols, mc = cols - 1;
    const int col = strip * kWave + lane;
    const int r0 = 1 + chunk * a.chunk_h;
    const int r1 = min(r0 + a.chunk_h, rows - 2);  // rows [r0, r1) within [1, rows-3]
    const bool colv = col >= 1 && col <= cols - 3;
    const bool colw = col <= cols - 2;  // the map has columns [0, cols-2]; outside the scan they are 0
    const auto rs = make_rsrc(a.frames + static_cast<int64_t>(f) * rows * cols, static_cast<uint32_t>(rows * cols));
    const int64_t mbase = static_cast<int64_t>(f) * (rows - 1) * mc;
    uint32_t *bits_out = a.rowbits + ((static_cast<int64_t>(f) * mc + col) * a.chunks + chunk) * a.words;

    // Map rows 0 and rows-2 lie outside the scan (:71): written as zeros by the first / last chunk, so
    // every map entry is written exactly once and the host needs no memset.
    auto zero_row = [&](int r) {
        if (!colw) return;
        const int64_t i = mbase + static_cast<int64_t>(r) * mc + col;
        if (a.norm) a.norm[i] = 0.0f;
        if (a.angle) a.angle[i] = 0.0f;
        a.valid[i] = 0;
    };
    if (chunk == 0) zero_row(0);
    if (r1 == rows - 2) zero_row(rows - 2);

    // I(r, col) for this lane; lane 63 also loads I(r, col + 1) (the others take it from lane + 1).
    // Rows past the frame read 0 (buffer range check) and are never used.
    auto ld = [&](int r, uint32_t &p, uint32_t &e) {
        p = buf_load_u8(rs, r * cols + col);
        e = lane == kWave - 1 ? buf_load_u8(rs, r * cols + col + 1) : 0u;
    };
    // (the DPP move runs on every lane: under a partial exec mask lane 62 would read a disabled lane 63)
    auto right = [&](uint32_t p, uint32_t e) {
        const uint32_t x = from_right(p);
        return lane == kWave - 1 ? e : x;
    };
    int cnt = 0;
    uint32_t word = 0;
    // one group: rows r .. r+kLsdGroup-1 from pixel rows r .. r+kLsdGroup (P/E[0..kLsdGroup])
    auto group = [&](int r, const uint32_t (&P)[kLsdGroup + 1], const uint32_t (&E)[kLsdGroup + 1]) {
#pragma unroll
        for (int i = 0; i < kLsdGroup; ++i) {
            const int rr = r + i;
            if (rr >= r1) break;  // uniform
            const uint32_t t0 = P[i], t1 = right(P[i], E[i]);
            const uint32_t b0 = P[i + 1], b1 = right(P[i + 1], E[i + 1]);
            const int ad = static_cast<int>(b1) - static_cast<int>(t0);  // :76-79
            const int bc = static_cast<int>(t1) - static_cast<int>(b0);
            const float gx = static_cast<float>(ad + bc) / 2.0f;  // :80-81
            const float gy = static_cast<float>(ad - bc) / 2.0f;
            const float nrm = __builtin_sqrtf((gx * gx) + (gy * gy));  // :82
            const bool v = colv && nrm > a.min_norm;                  // :83
            float ang = 0.0f;
            if (v) ang = fd_atan2f(gx, -gy);  // :85
            if (colw) {
                const int64_t idx = mbase + static_cast<int64_t>(rr) * mc + col;
                if (a.norm) a.norm[idx] = colv ? nrm : 0.0f;
                if (a.angle) a.angle[idx] = ang;
                a.valid[idx] = v ? 1 : 0;
            }
            cnt += v ? 1 : 0;
            word |= static_cast<uint32_t>(v) << ((rr - r0) & 31);
        }
        // rows r0 + 32k .. r0 + 32k + 31 share a bitmask word (kLsdGroup divides 32)
        const int done = r + kLsdGroup - r0;
        if ((done & 31) == 0 || r + kLsdGroup >= r1) {
            if (colv) bits_out[(done - 1) >> 5] = word;
            word = 0;
        }
    };
    static_assert(32 % kLsdGroup == 0, "bitmask words hold whole groups");
    uint32_t A[kLsdGroup + 1], AE[kLsdGroup + 1], B[kLsdGroup + 1], BE[kLsdGroup + 1];
#pragma unroll
    for (int i = 0; i <= kLsdGroup; ++i) ld(r0 + i, A[i], AE[i]);
    for (int r = r0; r < r1; r += 2 * kLsdGroup) {
        // B: rows r+G .. r+2G (its first row is A's last: reloaded, a cache hit, to keep sets disjoint)
#pragma unroll
        for (int i = 0; i <= kLsdGroup; ++i) ld(r + kLsdGroup + i, B[i], BE[i]);
        group(r, A, AE);
        if (r + kLsdGroup >= r1) break;
#pragma unroll
        for (int i = 0; i <= kLsdGroup; ++i) ld(r + 2 * kLsdGroup + i, A[i], AE[i]);
        group(r + kLsdGroup, B, BE);
    }
    if (colv) a.col_cnt[(static_cast<int64_t>(f) * mc + col) * a.chunks + chunk] = cnt;
}

// Pass 2: per-frame exclusive scan of the counts in column-major order (col outer, chunk inner).
__global__ __launch_bounds__(1024) void k_lsd_scan(LsdArgs a) {
    __shared__ int64_t wsum[16];
    __shared__ int64_t carry;
    const int f = blockIdx.x;
    const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
    const int mc = a.cols - 1;
    const int64_t n = static_cast<int64_t>(mc) * a.chunks;
    const int32_t *cnt = a.col_cnt + static_cast<int64_t>(f) * n;
    int32_t *base = a.col_base + static_cast<int64_t>(f) * n;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int64_t s0 = 0; s0 < n; s0 += 1024) {
        const int64_t s = s0 + tid;
        // entries of columns outside [1, cols-3] were never written: treat them as 0
        const int col = static_cast<int>(s / a.chunks);
        const int c = (s < n && col >= 1 && col <= a.cols - 3) ? cnt[s] : 0;
        int64_t incl = c;
        for (int o = 1; o < kWave; o <<= 1) {
            const int64_t t = __shfl_up(incl, o);
            if (lane >= o) incl += t;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int64_t wpre = 0;
        for (int q = 0; q < wv; ++q) wpre += wsum[q];
        const int64_t start = carry + wpre + incl - c;
        __syncthreads();
        if (s < n) base[s] = static_cast<int32_t>(start);
        if (tid == 1023) carry = start + c;
        __syncthreads();
    }
    if (tid == 0) a.counts[f] = carry;
}

// Pass 3: scatter valid map indices in scan order, from the per-(column, chunk) row bitmasks of
// pass 1 (a few words per lane instead of re-reading the valid map row by row).
__global__ __launch_bounds__(256) void k_lsd_scatter(LsdArgs a) {
    int f, strip, chunk;
    lsd_tile(a, f, strip, chunk);
    if (f >= a.batch) return;
    const int lane = lane_id();
    const int rows = a.rows, cols = a.cols, mc = cols - 1;
    const int col = strip * kWave + lane;
    if (!(col >= 1 && col <= cols - 3)) return;
    const int r0 = 1 + chunk * a.chunk_h;
    const int r1 = min(r0 + a.chunk_h, rows - 2);
    const int64_t cc = (static_cast<int64_t>(f) * mc + col) * a.chunks + chunk;
    int64_t pos = a.col_base[cc];
    const uint32_t *bits = a.rowbits + cc * a.words;
    int32_t *out = a.idx + static_cast<int64_t>(f) * a.idx_cap;
    const int nw = (r1 - r0 + 31) >> 5;
    for (int w = 0; w < nw; ++w) {
        uint32_t m = bits[w];
        while (m) {
            const int rr = r0 + 32 * w + __builtin_ctz(m);
            m &= m - 1u;
            if (pos < a.idx_cap) out[pos] = static_cast<int32_t>(static_cast<int64_t>(rr) * mc + col);
            ++pos;
        }
    }
}

}  // namespace

hipError_t launch_lsd(const LsdArgs &a, hipStream_t s) {
    const int64_t waves = static_cast<int64_t>(a.batch) * a.chunks * a.strips;
    const dim3 grid(static_cast<unsigned>((waves + 3) / 4)), block(256);
    hipLaunchKernelGGL(k_lsd_map, grid, block, 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lsd_scan, dim3(a.batch), dim3(1024), 0, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lsd_scatter, grid, block, 0, s, a);
    return hipGetLastError();
}

}  // namespace fdk
