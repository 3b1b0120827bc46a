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
#include "fd_corner_common.h"  // logical_block

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

// Pass 1: maps + per (column, row-chunk) valid counts and valid-row bitmasks. A wave owns a strip of
// 256 map columns (4 per lane, read as one dword per lane and row; the fifth column comes from the
// right neighbour lane by DPP, lane 63 loads it) and walks chunk_h rows. Every map entry is written
// exactly once per call (dword-per-lane stores of 4 columns). Angles: the valid pixels' (gx, gy) are
// queued in LDS and atan2f runs on waves of up to 64 queued pixels (on ~3 % of the pixels of a
// structured frame a per-row branch would run the whole atan2f for most rows, VALU-bound; compacted it
// is a small fraction of the row work), writing into the group's angle rows in LDS (0 elsewhere);
// after each group of kLsdGroup rows the queue is drained and the rows go to the map as whole rows
// (scattered 4-byte stores into the map would cost partial-line writes and their read-modify-write).
// Workgroups are placed XCD-aware (logical_block): an XCD holds consecutive strips and row chunks of
// one frame, so the column (strip edge) and row (chunk edge) neighbours a wave reads come from its
// own L2.
constexpr int kLsdQueue = 64 + 256;  // queued valid pixels per wave: < 64 left + one row (256 columns)
constexpr int kLsdGroup = 4;         // rows per group (row loads in flight; angle rows buffered in LDS)

struct LsdQueue {
    uint32_t sd[4][kLsdQueue];   // (s = ad + bc, d = ad - bc) as two int16
    uint32_t idx[4][kLsdQueue];  // position in the wave's angle rows (row in group * 256 + column)
    float ang[4][kLsdGroup][256];  // the group's angle rows, stored to the map whole once drained
};

template <bool ALIGNED>
__device__ __forceinline__ uint32_t lsd_load4(__amdgpu_buffer_rsrc_t r, int32_t off) {
    if constexpr (ALIGNED) return buf_load_u32(r, off);
    return buf_load_u8(r, off) | (buf_load_u8(r, off + 1) << 8) | (buf_load_u8(r, off + 2) << 16) |
           (buf_load_u8(r, off + 3) << 24);
}

// atan2f(gx, -gy) (:85) of the queued pixels, 64 at a time while at least `keep_below` remain (0 at
// the end: all), written into the angle map. One out-of-line copy: the atan2f body (correctly rounded
// divisions included) is large, and a copy per unrolled row would not fit the instruction cache.
__device__ __noinline__ int lsd_drain(const uint32_t *qsd, const uint32_t *qidx, int qn, int keep_below, float *arow) {
    const int lane = lane_id();
    while (qn >= keep_below && qn > 0) {
        const int take = min(qn, kWave);
        if (lane < take) {
            const uint32_t e = qsd[qn - take + lane];
            const int sv = static_cast<int16_t>(e & 0xFFFFu), dv = static_cast<int16_t>(e >> 16);
            const float gx = static_cast<float>(sv) / 2.0f;  // :80-81
            const float gy = static_cast<float>(dv) / 2.0f;
            arow[qidx[qn - take + lane]] = fd_atan2f(gx, -gy);
        }
        qn -= take;
    }
    return qn;
}

// INTERIOR: every column of the strip is scanned ([1, cols-3]) and present in the map: no per-column
// masks, and the maps are written with buffer stores at 32-bit offsets (no 64-bit address math).
template <bool ALIGNED, bool INTERIOR>
__device__ __forceinline__ void lsd_map_tile(const LsdArgs &a, const int f, const int strip, const int chunk,
                                             LsdQueue &Q) {
    const int lane = lane_id(), wv = threadIdx.x >> 6;
    uint32_t *const qsd = Q.sd[wv];
    uint32_t *const qidx = Q.idx[wv];
    const int rows = a.rows, cols = a.cols, mc = cols - 1, mp = a.pitch;  // mp: map row pitch (entries)
    const int c0 = strip * 256 + 4 * lane;
    const int r0 = 1 + chunk * a.chunk_h;
    const int r1 = min(r0 + a.chunk_h, rows - 2);  // rows [r0, r1) within [1, rows-3]
    bool colv[4], colw[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        colv[m] = c0 + m >= 1 && c0 + m <= cols - 3;  // scanned columns (:72)
        colw[m] = c0 + m <= cols - 2;                 // map columns [0, cols-2]
    }
    const bool full = c0 + 3 <= cols - 2;  // all four map columns exist: one store per map
    const auto rs = make_rsrc(a.frames + static_cast<int64_t>(f) * rows * cols, static_cast<uint32_t>(rows * cols));
    const int64_t mbase = static_cast<int64_t>(f) * (rows - 1) * mp;
    float *const amap = a.angle ? a.angle + mbase : nullptr;
    const uint32_t mbytes = static_cast<uint32_t>(rows - 1) * static_cast<uint32_t>(mp);
    const auto rn = make_rsrc(a.norm ? a.norm + mbase : nullptr, a.norm ? 4 * mbytes : 0u);
    const auto ra = make_rsrc(amap, amap ? 4 * mbytes : 0u);
    const auto rv = make_rsrc(a.valid ? a.valid + mbase : nullptr, a.valid ? mbytes : 0u);

#ifndef FD_LSD_STORE_AUX
#define FD_LSD_STORE_AUX 2  // nt: streaming map stores (1.55 -> 1.43 ms at 1080p x256, profiles/r04_lsd_nt_ab.txt)
#endif
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    struct alignas(4) F4 { float x, y, z, w; };
    // one map row's 4 angle entries of this lane
    auto put_angle = [&](int r, const float (&av)[4]) {
        if constexpr (INTERIOR) {
            __builtin_amdgcn_raw_buffer_store_b128(
                u4{__float_as_uint(av[0]), __float_as_uint(av[1]), __float_as_uint(av[2]), __float_as_uint(av[3])}, ra,
                4 * (r * mp + c0), 0, FD_LSD_STORE_AUX);
            return;
        }
        if (!a.angle) return;
        const int64_t i = mbase + static_cast<int64_t>(r) * mp + c0;
        if (full) {
            *reinterpret_cast<F4 *>(a.angle + i) = F4{av[0], av[1], av[2], av[3]};
        } else {
#pragma unroll
            for (int m = 0; m < 4; ++m)
                if (colw[m]) a.angle[i + m] = av[m];
        }
    };
    // norm and valid of one map row (the angles follow per group, put_angle)
    auto put = [&](int r, const float (&nv)[4], uint32_t vb) {
        if constexpr (INTERIOR) {
            // (null maps: a zero-range resource drops the stores)
            const int o = r * mp + c0;  // < 2^31: checked on the host
            __builtin_amdgcn_raw_buffer_store_b128(
                u4{__float_as_uint(nv[0]), __float_as_uint(nv[1]), __float_as_uint(nv[2]), __float_as_uint(nv[3])}, rn,
                4 * o, 0, FD_LSD_STORE_AUX);
            __builtin_amdgcn_raw_buffer_store_b32(vb, rv, o, 0, FD_LSD_STORE_AUX);
            return;
        }
        const int64_t i = mbase + static_cast<int64_t>(r) * mp + c0;
        if (full) {
            if (a.norm) *reinterpret_cast<F4 *>(a.norm + i) = F4{nv[0], nv[1], nv[2], nv[3]};
            typedef uint32_t u32a1 __attribute__((aligned(1)));
            if (a.valid) *reinterpret_cast<u32a1 *>(a.valid + i) = vb;
        } else {
#pragma unroll
            for (int m = 0; m < 4; ++m)
                if (colw[m]) {
                    if (a.norm) a.norm[i + m] = nv[m];
                    if (a.valid) a.valid[i + m] = static_cast<uint8_t>(vb >> (8 * m));
                }
        }
    };
    // Map rows 0 and rows-2 lie outside the scan (:71): zeros, written by the first / last chunk.
    {
        const float z[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if (chunk == 0) {
            put(0, z, 0u);
            put_angle(0, z);
        }
        if (r1 == rows - 2) {
            put(rows - 2, z, 0u);
            put_angle(rows - 2, z);
        }
    }
    // I(r, c0 .. c0+3) and I(r, c0+4): lane 63 loads the next dword (the others take byte 0 of the
    // right lane's dword). Rows/columns past the frame read 0 and only feed unscanned entries.
    auto ld = [&](int r, uint32_t &p, uint32_t &e) {
        p = lsd_load4<ALIGNED>(rs, r * cols + c0);
        e = lane == kWave - 1 ? buf_load_u8(rs, r * cols + c0 + 4) : 0u;
    };
    auto fifth = [&](uint32_t p, uint32_t e) {  // DPP on every lane (lane 62 reads lane 63)
        const uint32_t x = from_right(p) & 0xFFu;
        return lane == kWave - 1 ? e : x;
    };
    int cnt[4] = {0, 0, 0, 0};
    uint32_t word[4] = {0, 0, 0, 0};
    int qn = 0;  // wave-uniform queue length
    float *const arows = &Q.ang[wv][0][0];  // [kLsdGroup][256]
    auto row = [&](int rr, int slot, uint32_t t, uint32_t te, uint32_t b, uint32_t be) {
        const uint32_t t4 = fifth(t, te), b4 = fifth(b, be);
        float nv[4];
        int sv[4], dv[4];
        bool vv[4];
        uint32_t vb = 0;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int tm = (t >> (8 * m)) & 0xFF, bm = (b >> (8 * m)) & 0xFF;
            const int tn = m < 3 ? ((t >> (8 * m + 8)) & 0xFF) : static_cast<int>(t4);
            const int bn = m < 3 ? ((b >> (8 * m + 8)) & 0xFF) : static_cast<int>(b4);
            const int ad = bn - tm, bc = tn - bm;  // :76-79
            sv[m] = ad + bc;
            dv[m] = ad - bc;
            // gx^2 + gy^2 = (s^2 + d^2) / 4 exactly (half-integers), so the reference's correctly
            // rounded sqrt (:82) is sqrt_rn(s^2 + d^2) / 2 (an exact power-of-two scaling)
            nv[m] = static_cast<float>(static_cast<uint32_t>(sv[m] * sv[m] + dv[m] * dv[m]));
        }
        const f2 q01 = sqrt_rn_rsq2(f2{nv[0], nv[1]}) * 0.5f, q23 = sqrt_rn_rsq2(f2{nv[2], nv[3]}) * 0.5f;
        nv[0] = q01.x, nv[1] = q01.y, nv[2] = q23.x, nv[3] = q23.y;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            vv[m] = (INTERIOR || colv[m]) && nv[m] > a.min_norm;  // :83
            if (!INTERIOR && !colv[m]) nv[m] = 0.0f;
            vb |= static_cast<uint32_t>(vv[m]) << (8 * m);
            cnt[m] += vv[m] ? 1 : 0;
            word[m] |= static_cast<uint32_t>(vv[m]) << ((rr - r0) & 31);
        }
        put(rr, nv, vb);
        if (amap) {  // zero angle row in LDS; queue the valid pixels' (s, d) and row position
            *reinterpret_cast<F4 *>(arows + slot * 256 + 4 * lane) = F4{0.0f, 0.0f, 0.0f, 0.0f};
            const uint64_t b0 = ballot(vv[0]), b1 = ballot(vv[1]), b2 = ballot(vv[2]), b3 = ballot(vv[3]);
            const int tot = popc64(b0) + popc64(b1) + popc64(b2) + popc64(b3);
            if (tot) {
                int pos = mbcnt64(b3, mbcnt64(b2, mbcnt64(b1, mbcnt64(b0, qn))));
                const uint32_t i0 = static_cast<uint32_t>(slot * 256 + 4 * lane);
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    if (vv[m]) {
                        qsd[pos] = (static_cast<uint32_t>(sv[m]) & 0xFFFFu) | (static_cast<uint32_t>(dv[m]) << 16);
                        qidx[pos] = i0 + m;
                        ++pos;
                    }
                qn += tot;
                if (qn >= kWave) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    qn = __builtin_amdgcn_readfirstlane(lsd_drain(qsd, qidx, qn, kWave, arows));
                }
            }
        }
    };
    // one group: rows r .. r+kLsdGroup-1 from pixel rows r .. r+kLsdGroup (P/E[0..kLsdGroup])
    auto group = [&](int r, const uint32_t (&P)[kLsdGroup + 1], const uint32_t (&E)[kLsdGroup + 1]) {
#pragma unroll
        for (int i = 0; i < kLsdGroup; ++i) {
            if (r + i >= r1) break;  // uniform
            row(r + i, i, P[i], E[i], P[i + 1], E[i + 1]);
        }
        if (amap) {  // the group's angles: drain the queue into the LDS rows, then store the rows whole
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (qn > 0) qn = __builtin_amdgcn_readfirstlane(lsd_drain(qsd, qidx, qn, 0, arows));
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int i = 0; i < kLsdGroup; ++i) {
                if (r + i >= r1) break;  // uniform
                const F4 v = *reinterpret_cast<const F4 *>(arows + i * 256 + 4 * lane);
                const float av[4] = {v.x, v.y, v.z, v.w};
                put_angle(r + i, av);
            }
        }
        // rows r0 + 32k .. r0 + 32k + 31 share a bitmask word (kLsdGroup divides 32)
        const int done = r + kLsdGroup - r0;
        if ((done & 31) == 0 || r + kLsdGroup >= r1) {
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                if (INTERIOR || colv[m])
                    a.rowbits[((static_cast<int64_t>(f) * a.chunks + chunk) * a.words + ((done - 1) >> 5)) * mc + c0 + m] =
                        word[m];
                word[m] = 0;
            }
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
#pragma unroll
    for (int m = 0; m < 4; ++m)
        if (INTERIOR || colv[m]) a.col_cnt[(static_cast<int64_t>(f) * a.chunks + chunk) * mc + c0 + m] = cnt[m];
}

template <bool ALIGNED>
__global__ __launch_bounds__(256) void k_lsd_map(LsdArgs a) {
    __shared__ LsdQueue Q;
    int w = __builtin_amdgcn_readfirstlane(logical_block() * 4 + (threadIdx.x >> 6));
    int strip, chunk;
    if (a.chunk_fastest) {
        chunk = w % a.chunks;
        w /= a.chunks;
        strip = w % a.strips4;
        w /= a.strips4;
    } else {
        strip = w % a.strips4;
        w /= a.strips4;
        chunk = w % a.chunks;
        w /= a.chunks;
    }
    const int f = w;
    if (f >= a.batch) return;
    if (strip * 256 >= 1 && strip * 256 + 255 <= a.cols - 3) lsd_map_tile<ALIGNED, true>(a, f, strip, chunk, Q);
    else lsd_map_tile<ALIGNED, false>(a, f, strip, chunk, Q);
}

// Pass 2: per column the total of its chunk counts, and their exclusive scan in column order (the
// column-major list order) into col_base's chunk-0 row: all the scatter reads, since a column's entries
// are one contiguous run, chunk after chunk. One workgroup per frame; each thread sums one column's chunk
// counts (loads coalesced across the threads). (Scanning every (column, chunk) entry in column-major
// order, gathered across the chunk rows, took 37 us at 1080p x256; this 15 us.)
__global__ __launch_bounds__(1024) void k_lsd_scan(LsdArgs a) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    const int f = blockIdx.x;
    const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
    const int cols = a.cols, mc = cols - 1, chunks = a.chunks;
    const int64_t n = static_cast<int64_t>(mc) * chunks;
    const int32_t *cnt = a.col_cnt + static_cast<int64_t>(f) * n;
    int32_t *base = a.col_base + static_cast<int64_t>(f) * n;
    if (tid == 0) carry = 0;
    __syncthreads();
    // (a frame's count < 2^29: 32-bit sums)
    for (int c0 = 0; c0 < mc; c0 += 1024) {
        const int col = c0 + tid;
        uint32_t tot = 0;
        if (col >= 1 && col <= cols - 3) {  // (other columns were never counted)
#pragma unroll 8
            for (int k = 0; k < chunks; ++k) tot += static_cast<uint32_t>(cnt[static_cast<int64_t>(k) * mc + col]);
        }
        const uint32_t incl = wave_incl_add(tot);
        if (lane == kWave - 1) wsum[wv] = incl;
        __syncthreads();
        uint32_t run = carry + incl - tot;
        for (int q = 0; q < wv; ++q) run += wsum[q];
        __syncthreads();  // everyone has read carry and wsum
        if (col < mc) base[col] = static_cast<int32_t>(run);
        if (tid == 1023) carry = run + tot;
        __syncthreads();
    }
    if (tid == 0) a.counts[f] = carry;
}

// Pass 3: scatter valid map indices in scan order, from the per-(column, chunk) row bitmasks of
// pass 1 (a few words per lane instead of re-reading the valid map row by row).
// Pass 3: the column-major valid list. The list holds each column's valid rows in order, chunk after
// chunk, so one column's entries (all chunks) are one contiguous run starting at its chunk-0 base. A wave
// owns NC columns and writes them one column at a time: its lanes take the column's (chunk, row word)
// items in row order, a wave prefix of their popcounts places every lane's entries inside the run, so
// each store instruction covers a few adjacent cache lines (a lane per column, as before, made every
// store touch 64 lines; the row-bit words of adjacent columns share lines, so the per-column loads hit
// L1 after the first column of a line).
template <int NC>
__global__ __launch_bounds__(256) void k_lsd_scatter(LsdArgs a) {
    const int w4 = static_cast<int>(blockIdx.x) * 4 + (static_cast<int>(threadIdx.x) >> 6);
    const int nstrips = (a.cols - 1 + NC - 1) / NC;
    const int strip = __builtin_amdgcn_readfirstlane(w4 % nstrips), f = __builtin_amdgcn_readfirstlane(w4 / nstrips);
    if (f >= a.batch) return;
    const int lane = lane_id();
    const int rows = a.rows, cols = a.cols, mc = cols - 1, words = a.words, chunks = a.chunks;
    const int items = chunks * words;
    const int64_t n = static_cast<int64_t>(mc) * chunks;
    const int32_t *cbase = a.col_base + static_cast<int64_t>(f) * n;  // [chunk][column] of this frame
    const uint32_t *fbits = a.rowbits + static_cast<int64_t>(f) * chunks * words * mc;
    int32_t *out = a.frame_base ? a.idx + a.frame_base[f] : a.idx + static_cast<int64_t>(f) * a.idx_cap;
    const int64_t cap = a.frame_base ? INT64_MAX : a.idx_cap;
    // the NC columns' run starts (lane = column), read once
    const int coll = lane < NC ? strip * NC + lane : -1;
    const int64_t basel = coll >= 1 && coll <= cols - 3 ? cbase[coll] : 0;
    auto put = [&](int col, int i, uint32_t m, int64_t &run) {
        const int c = i / words, w = i - c * words;
        const int r0 = 1 + c * a.chunk_h;
        const uint32_t cnt = static_cast<uint32_t>(__popc(m));
        const uint32_t incl = wave_incl_add(cnt);
        int64_t pos = run + (incl - cnt);
        while (m) {
            const int rr = r0 + 32 * w + __builtin_ctz(m);
            m &= m - 1u;
            if (pos < cap) out[pos] = static_cast<int32_t>(static_cast<int64_t>(rr) * mc + col);
            ++pos;
        }
        run += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), kWave - 1));
    };
    auto word = [&](int col, int i) -> uint32_t {
        const int c = i / words, w = i - c * words;
        const int r0 = 1 + c * a.chunk_h;
        if (col < 1 || col > cols - 3 || i >= items || r0 + 32 * w >= min(r0 + a.chunk_h, rows - 2)) return 0u;
        return fbits[(static_cast<int64_t>(c) * words + w) * mc + col];
    };
    if (items <= kWave) {
        // the wave's row-bit words, [item][column], read row by row (lane = column: 256 contiguous bytes per
        // load) into LDS, 16 loads in flight; then one item per lane and column from LDS
        __shared__ uint32_t sb[4][kWave][NC + 1];
        uint32_t(*const wb)[NC + 1] = sb[threadIdx.x >> 6];
        for (int i0 = 0; i0 < items; i0 += 16) {
            uint32_t v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = word(coll, i0 + k);
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (i0 + k < kWave && lane < NC) wb[i0 + k][lane] = v[k];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        constexpr int kG = 8;
        static_assert(NC % kG == 0, "whole column groups");
        for (int g = 0; g < NC; g += kG) {
            uint32_t mv[kG];
#pragma unroll
            for (int k = 0; k < kG; ++k) mv[k] = lane < items ? wb[lane][g + k] : 0u;
#pragma unroll
            for (int k = 0; k < kG; ++k) {
                const int col = strip * NC + g + k;
                if (col < 1 || col > cols - 3) continue;  // (wave-uniform)
                const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(basel), g + k));
                const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(basel >> 32), g + k));
                int64_t run = static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
                put(col, lane, mv[k], run);
            }
        }
        return;
    }
    for (int cc = 0; cc < NC; ++cc) {
        const int col = strip * NC + cc;
        if (col < 1 || col > cols - 3) continue;  // (wave-uniform)
        int64_t run = cbase[col];
        for (int i0 = 0; i0 < items; i0 += kWave) put(col, i0 + lane, word(col, i0 + lane), run);
    }
}

// Compact mode, after the scatter: each list entry's norm and angle, recomputed from its four pixels
// with the map pass's operations (bit-identical), one thread per entry.
__global__ __launch_bounds__(256) void k_lsd_values(LsdArgs a, int64_t total) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= total) return;
    int lo = 0, hi = a.batch - 1;  // frame of entry i: last f with frame_base[f] <= i
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.frame_base[mid] <= i) lo = mid; else hi = mid - 1;
    }
    const int f = lo, rows = a.rows, cols = a.cols, mc = cols - 1;
    const int32_t mi = a.idx[i];
    const int rr = mi / mc, col = mi - rr * mc;
    const auto rs = make_rsrc(a.frames + static_cast<int64_t>(f) * rows * cols, static_cast<uint32_t>(rows * cols));
    const int o = rr * cols + col;
    const int ad = static_cast<int>(buf_load_u8(rs, o + cols + 1)) - static_cast<int>(buf_load_u8(rs, o));  // :76-77
    const int bc = static_cast<int>(buf_load_u8(rs, o + 1)) - static_cast<int>(buf_load_u8(rs, o + cols));  // :78-79
    const int sv = ad + bc, dv = ad - bc;
    const float q = static_cast<float>(static_cast<uint32_t>(sv * sv + dv * dv));
    a.lnorm[i] = sqrt_rn_rsq2(f2{q, q}).x * 0.5f;                                          // :82 (as in the map pass)
    a.langle[i] = fd_atan2f(static_cast<float>(sv) / 2.0f, -(static_cast<float>(dv) / 2.0f));  // :80-81, :85
}

// Compact mode: frame_base[f] = valid pixels of frames [0, f) (one workgroup; batch is small).
__global__ __launch_bounds__(64) void k_lsd_frames(const int64_t *counts, int batch, int64_t *frame_base) {
    if (threadIdx.x != 0) return;
    int64_t acc = 0;
    for (int f = 0; f < batch; ++f) {
        frame_base[f] = acc;
        acc += counts[f];
    }
    frame_base[batch] = acc;
}

}  // namespace

namespace {

// k_lsd_scatter with a.scatter_cols columns per wave (32; 16 or 64 for A/B)
hipError_t launch_scatter(const LsdArgs &a, hipStream_t s) {
    const int nc = a.scatter_cols == 64 ? 64 : a.scatter_cols == 16 ? 16 : 32;
    const int64_t waves = static_cast<int64_t>(a.batch) * ((a.cols - 1 + nc - 1) / nc);
    const dim3 grid(static_cast<unsigned>((waves + 3) / 4)), block(256);
    if (nc == 64) hipLaunchKernelGGL(k_lsd_scatter<64>, grid, block, 0, s, a);
    else if (nc == 16) hipLaunchKernelGGL(k_lsd_scatter<16>, grid, block, 0, s, a);
    else hipLaunchKernelGGL(k_lsd_scatter<32>, grid, block, 0, s, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_lsd_count(const LsdArgs &a, hipStream_t s) {
    const int64_t mwaves = static_cast<int64_t>(a.batch) * a.chunks * a.strips4;
    const dim3 mgrid(static_cast<unsigned>((mwaves + 3) / 4)), block(256);
    if (a.aligned4) hipLaunchKernelGGL(k_lsd_map<true>, mgrid, block, 0, s, a);
    else hipLaunchKernelGGL(k_lsd_map<false>, mgrid, block, 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lsd_scan, dim3(a.batch), dim3(1024), 0, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lsd_frames, dim3(1), dim3(64), 0, s, a.counts, a.batch, a.frame_base);
    return hipGetLastError();
}

hipError_t launch_lsd_scatter(const LsdArgs &a, hipStream_t s) {
    hipError_t e = launch_scatter(a, s);
    if (e != hipSuccess || !a.frame_base || a.idx_cap <= 0) return e;
    // compact mode: idx_cap = the batch's total number of entries (frame_base[batch])
    hipLaunchKernelGGL(k_lsd_values, dim3(static_cast<unsigned>((a.idx_cap + 255) / 256)), dim3(256), 0, s, a, a.idx_cap);
    return hipGetLastError();
}

hipError_t launch_lsd(const LsdArgs &a, hipStream_t s) {
    const int64_t mwaves = static_cast<int64_t>(a.batch) * a.chunks * a.strips4;
    const dim3 mgrid(static_cast<unsigned>((mwaves + 3) / 4)), block(256);
    if (a.aligned4) hipLaunchKernelGGL(k_lsd_map<true>, mgrid, block, 0, s, a);
    else hipLaunchKernelGGL(k_lsd_map<false>, mgrid, block, 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lsd_scan, dim3(a.batch), dim3(1024), 0, s, a);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_scatter(a, s);
}

}  // namespace fdk
