// Point-detection kernels for gfx950 (MI355X): Harris / Shi-Tomasi response + 4-neighbour NMS,
// FAST-12 segment test, prior-feature mask, per-frame greedy min-distance selection.
//
// Reference (Horizon1026/Feature_Detector, paths relative to src/feature_point_detector/):
//   gradient + 3x3 tensor ........ feature_point_harris_detector.cpp:17-64, :66-88, :108-116
//   Harris response .............. feature_point_harris_detector.cpp:94-104
//   Shi-Tomasi response .......... feature_point_shi_tomas_detector.cpp:94-103
//   4-neighbour NMS .............. feature_point_harris_detector.cpp:120-137
//   FAST ......................... feature_point_fast_detector.cpp:11-98
//   mask / sort / greedy select .. feature_point_detector.cpp:7-25, :54-98
// See DESIGN.md for the data layout, the roofline of each kernel and the bit-exactness argument.
//
// Build flags matter: -ffp-contract=off (the reference's x86-64 build has no FMA) and correctly
// rounded f32 sqrt/div (hipcc default; never -ffast-math).
#include "fd_device.h"
#include "fd_kernels.h"

namespace fdk {

namespace {

constexpr int kStage = 512;  // per-wave LDS staging of candidates (detect mode)
constexpr float kInvCnt = 1.0f / 9.0f;                  // 1 / (3*3)  (:71)
constexpr float kInvCnt2 = (1.0f / 9.0f) * (1.0f / 9.0f);  // harris :72
constexpr float kHarrisAlpha = 0.04f;                  // feature_point_harris_detector.h:13

// Workgroup -> (frame, 4 consecutive tiles of that frame); returns false for the idle waves of a
// frame's last workgroup (they still take part in the workgroup barriers).
// The tile coordinates are made visibly wave-uniform (readfirstlane), so row/tile logic stays scalar.
__device__ __forceinline__ bool decode_tile(const PointsArgs &a, int &f, int &ty, int &tx) {
    f = blockIdx.x / a.blocks_per_frame;
    const int t = __builtin_amdgcn_readfirstlane((blockIdx.x % a.blocks_per_frame) * 4 + (threadIdx.x >> 6));
    tx = t % a.tiles_x;
    ty = t / a.tiles_x;
    return t < a.tiles_x * a.tiles_y;
}

// Dword of frame bytes [off, off+4). `aligned` (cols % 4 == 0) guarantees whole-dword range checks;
// otherwise assemble from byte loads so that a dword straddling the frame end still returns its bytes.
// A compile-time choice: a runtime branch here makes the waitcnt pass drain the prefetch queue.
template <bool ALIGNED>
__device__ __forceinline__ uint32_t load_px4(__amdgpu_buffer_rsrc_t r, int32_t off) {
    if constexpr (ALIGNED) return buf_load_u32(r, off);
    return buf_load_u8(r, off) | (buf_load_u8(r, off + 1) << 8) | (buf_load_u8(r, off + 2) << 16) |
           (buf_load_u8(r, off + 3) << 24);
}

// Per-wave candidate sink. Detect mode: stage in LDS, append to the frame's list with one atomic per
// flush. Raster mode: write the (row, tile) segment in column order.
struct Sink {
    float *resp;     // LDS staging (detect mode)
    uint32_t *idx;
    uint32_t *hist;  // LDS level-0 histogram of the workgroup's frame, or null
    int n;           // staged entries (wave-uniform)
};

__device__ __forceinline__ void sink_flush(Sink &sk, const PointsArgs &a, int f) {
    if (sk.n == 0) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&a.list_count[f], static_cast<uint32_t>(sk.n));
    base = __builtin_amdgcn_readfirstlane(base);
    float *dr = a.list_resp + static_cast<int64_t>(f) * a.list_cap;
    uint32_t *di = a.list_idx + static_cast<int64_t>(f) * a.list_cap;
    // The level-0 histogram is counted here, once per staged candidate, rather than in the per-row
    // emit path where every (row, column-of-4) slot would pay for the key computation.
    for (int i = lane_id(); i < sk.n; i += kWave) {
        const float r = sk.resp[i];
        if (sk.hist) atomicAdd(&sk.hist[float_key(r) >> 20], 1u);
        const int64_t pos = static_cast<int64_t>(base) + i;
        if (pos < a.list_cap) {
            dr[pos] = r;
            di[pos] = sk.idx[i];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // Drain the stores here (rare path) so the row loop's waitcnt state stays "loads only" and its
    // prefetch queue is not flushed at every loop header. s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15).
    __builtin_amdgcn_s_waitcnt(0x0F70);
    sk.n = 0;
}

// Emit up to 4 candidates of this lane (columns c0..c0+3 of row `row`), preserving column order.
// The lane's slot is the count of candidates in lower lanes: one v_mbcnt pair per column ballot.
// b[m] is the wave ballot of fl[m] (callers that hold it as a compare mask pass it directly).
template <bool RASTER, int SEGCAP>
__device__ __forceinline__ void emit_row(Sink &sk, const PointsArgs &a, int f, int tx, int row, int c0,
                                         const uint64_t (&b)[4], const bool (&fl)[4], const float (&v)[4]) {
    const uint64_t b0 = b[0], b1 = b[1], b2 = b[2], b3 = b[3];
    const int tot = popc64(b0) + popc64(b1) + popc64(b2) + popc64(b3);  // scalar unit
    const uint32_t id0 = static_cast<uint32_t>(row) * static_cast<uint32_t>(a.cols) + static_cast<uint32_t>(c0);
    if constexpr (RASTER) {
        int pos = mbcnt64(b3, mbcnt64(b2, mbcnt64(b1, mbcnt64(b0, 0))));
        const int64_t seg = (static_cast<int64_t>(f) * a.rows + row) * a.tiles_x + tx;
        if (lane_id() == 0) a.seg_cnt[seg] = tot;
        Cand *dst = a.seg + seg * SEGCAP;
#pragma unroll
        for (int m = 0; m < 4; ++m)
            if (fl[m]) dst[pos++] = Cand{v[m], id0 + m};
    } else {
        if (tot == 0) return;
        if (sk.n + tot > kStage) sink_flush(sk, a, f);
        int pos = mbcnt64(b3, mbcnt64(b2, mbcnt64(b1, mbcnt64(b0, sk.n))));
#pragma unroll
        for (int m = 0; m < 4; ++m)
            if (fl[m]) {
                sk.resp[pos] = v[m];
                sk.idx[pos] = id0 + m;
                ++pos;
            }
        sk.n += tot;
    }
}

__device__ __forceinline__ uint32_t mask_bits4(const PointsArgs &a, int f, int row, int c0) {
    if (c0 < 0 || c0 >= a.cols) return 0u;
    const uint32_t w = a.mask[(static_cast<int64_t>(f) * a.rows + row) * a.mask_wpr + (c0 >> 5)];
    return (w >> (c0 & 31)) & 0xFu;
}

// Workgroup-shared staging + level-0 histogram (detect mode).
struct DetectLds {
    float resp[4][kStage];
    uint32_t idx[4][kStage];
    uint32_t hist[kHistBins];
};

__device__ __forceinline__ void hist_clear(uint32_t *h) {
    for (int b = threadIdx.x; b < kHistBins; b += blockDim.x) h[b] = 0;
    __syncthreads();
}
__device__ __forceinline__ void hist_flush(const uint32_t *h, uint32_t *g) {
    __syncthreads();
    for (int b = threadIdx.x; b < kHistBins; b += blockDim.x) {
        const uint32_t v = h[b];
        if (v) atomicAdd(&g[b], v);
    }
}

// Two pixels' float math at a time: <2 x float> arithmetic compiles to v_pk_mul_f32 / v_pk_add_f32 /
// v_pk_fma_f32, which round each lane exactly like the scalar op (the kernel is VALU-issue bound, and
// a packed op retires two pixels' worth of one reference operation per issue slot).
typedef float f2 __attribute__((ext_vector_type(2)));

// Correctly rounded f32 sqrt of two values that are each 0 or normal: v_sqrt_f32 (within 1 ulp)
// followed by the two fma residual corrections of the compiler's own IEEE expansion, minus its
// denormal pre-scaling and inf/nan class fix-up. The Shi-Tomasi radicand d*d + 4b*b is either 0 or
// >= 2^-54: b is 0 or |b| >= 1/9, and a != c differ by at least ulp(1/9) = 2^-27. For x == 0 the
// s-1ulp candidate is a NaN whose residual compares false and the s+1ulp residual is -0, so 0 results.
__device__ __forceinline__ f2 sqrt_rn_normal2(f2 x) {
    const f2 s = {__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)};
    const f2 sdn = {__int_as_float(__float_as_int(s.x) - 1), __int_as_float(__float_as_int(s.y) - 1)};
    const f2 sup = {__int_as_float(__float_as_int(s.x) + 1), __int_as_float(__float_as_int(s.y) + 1)};
    const f2 rdn = __builtin_elementwise_fma(-sdn, s, x);
    const f2 rup = __builtin_elementwise_fma(-sup, s, x);
    f2 r;
    r.x = rup.x > 0.0f ? sup.x : (rdn.x <= 0.0f ? sdn.x : s.x);
    r.y = rup.y > 0.0f ? sup.y : (rdn.y <= 0.0f ? sdn.y : s.y);
    return r;
}

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

template <int KIND>
__device__ __forceinline__ f2 corner_response2(uint32_t sxx0, uint32_t sxx1, uint32_t syy0, uint32_t syy1,
                                               uint32_t sxy0, uint32_t sxy1, float thr) {
    const f2 fxx = f2{__uint_as_float(sxx0), __uint_as_float(sxx1)} - 8388608.0f;
    const f2 fyy = f2{__uint_as_float(syy0), __uint_as_float(syy1)} - 8388608.0f;
    const f2 fxy = f2{__uint_as_float(sxy0), __uint_as_float(sxy1)} - 12582912.0f;
    f2 res;
    if constexpr (KIND == 0) {  // Harris, feature_point_harris_detector.cpp:95-103
        const f2 trace = fxx + fyy;
        const f2 gate = ((trace * trace) * 0.21f) * kInvCnt2;
        const f2 r = (((fxx * fyy) - (fxy * fxy)) - ((kHarrisAlpha * trace) * trace)) * kInvCnt2;
        res.x = (gate.x > thr && r.x > thr) ? r.x : 0.0f;
        res.y = (gate.y > thr && r.y > thr) ? r.y : 0.0f;
    } else {  // Shi-Tomasi, feature_point_shi_tomas_detector.cpp:94-103
        const f2 a = fxx * kInvCnt;
        const f2 c = fyy * kInvCnt;
        const f2 ac = a + c;
        const f2 b = fxy * kInvCnt;
        const f2 d = a - c;
        const f2 common = sqrt_rn_normal2((d * d) + ((4.0f * b) * b));
        const f2 r = (ac + common) * 0.5f;
        res.x = (ac.x > thr && r.x > thr) ? r.x : 0.0f;
        res.y = (ac.y > thr && r.y > thr) ? r.y : 0.0f;
    }
    return res;
}

template <int KIND, bool RASTER, bool MASKED, bool ALIGNED>
__device__ __forceinline__ void corner_tile(const PointsArgs &a, int f, int ty, int tx, Sink &sk);

// ---------------------------------------------------------------------------------------------------
// K1: corner response + NMS. One wave per tile of kTileW columns x tile_h rows; lane l covers columns
// c0 = tx*kTileW + 4(l-1) .. c0+3 and walks the rows keeping 3-row sliding windows in registers:
// pixels (+ DPP halo dwords), horizontal tensor sums, responses.
// ---------------------------------------------------------------------------------------------------
template <int KIND, bool RASTER, bool MASKED, bool ALIGNED>
__global__ __launch_bounds__(256) void k_corner(PointsArgs a) {
    __shared__ DetectLds lds_all[1];
    int f, ty, tx;
    const bool active = decode_tile(a, f, ty, tx);
    Sink sk{nullptr, nullptr, nullptr, 0};
    if constexpr (!RASTER) {
        const int wv = threadIdx.x >> 6;
        sk = Sink{lds_all[0].resp[wv], lds_all[0].idx[wv], a.hist0 ? lds_all[0].hist : nullptr, 0};
        if (a.hist0) hist_clear(lds_all[0].hist);
    }
    if (active) corner_tile<KIND, RASTER, MASKED, ALIGNED>(a, f, ty, tx, sk);
    if constexpr (!RASTER) {
        if (active) sink_flush(sk, a, f);
        if (a.hist0) hist_flush(lds_all[0].hist, a.hist0 + static_cast<int64_t>(f) * kHistBins);
    }
}

template <int KIND, bool RASTER, bool MASKED, bool ALIGNED>
__device__ __forceinline__ void corner_tile(const PointsArgs &a, int f, int ty, int tx, Sink &sk) {
    const int lane = lane_id();
    const int rows = a.rows, cols = a.cols;
    const int c0 = tx * kTileW + 4 * (lane - 1);
    const int y0 = 2 + ty * a.tile_h;
    const int y1 = min(y0 + a.tile_h, rows - 2);  // output rows [y0, y1) within [2, rows-3]
    const auto rs = make_rsrc(a.frames + static_cast<int64_t>(f) * rows * cols, static_cast<uint32_t>(rows * cols));
    // Every lane's 4 columns inside [2, cols-3]: then only the frame's first/last rows need masking.
    const bool tile_interior = tx * kTileW - 4 >= 2 && tx * kTileW + 4 * 62 + 3 <= cols - 3;

    bool cval[4], colv[4];  // column inside [2, cols-3]; and owned by an interior lane (emitted)
    uint64_t colv_b[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        cval[m] = c0 + m >= 2 && c0 + m <= cols - 3;
        colv[m] = cval[m] && lane >= 1 && lane <= 62;
        colv_b[m] = ballot(colv[m]);
    }

    uint32_t hxx[3][4], hyy[3][4], hxy[3][4];  // biased horizontal sums (3 products, 3*beta)
    float rsp[3][4];
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int m = 0; m < 4; ++m) hxx[s][m] = hyy[s][m] = hxy[s][m] = 0, rsp[s][m] = 0.0f;

    // Row ring of 6 dwords: rows ri-2 .. ri are in use while rows ri+1 .. ri+3 are in flight (a row
    // step is about one HBM latency of wall time at full occupancy). The loop is unrolled by the ring
    // length so every slot keeps a fixed register (no copies of in-flight loads at the back edge,
    // which would force a vmcnt(0)). Rows outside the frame (including row -1) fall outside the
    // buffer resource's range and read as 0.
    const int n_in = (y1 - y0) + 6;
    uint32_t ring[6];
#pragma unroll
    for (int t = 0; t < 6; ++t) ring[t] = t < 3 ? load_px4<ALIGNED>(rs, (y0 - 3 + t) * cols + c0) : 0u;
    // Once per wave: land the preheader loads, so the loop header's waitcnt state is the back edge's
    // (three rows in flight) rather than the preheader's register order.
    __builtin_amdgcn_s_waitcnt(0x0F70);
    for (int i0 = 0; i0 < n_in; i0 += 6) {
#pragma unroll
        for (int t = 0; t < 6; ++t) {
            const int s = t % 3, su = (t + 1) % 3, sc = (t + 2) % 3;  // 3-slot roles: rows ri, ri-2, ri-1
            const int ri = y0 - 3 + i0 + t;                            // row consumed this step
            ring[(t + 3) % 6] = load_px4<ALIGNED>(rs, (ri + 3) * cols + c0);
            const uint32_t P_s = ring[t], P_su = ring[(t + 4) % 6], P_sc = ring[(t + 5) % 6];

            // Gradients of centre row ri-1 at the lane's 4 columns (feature_point_harris_detector.cpp:
            // 35-62); the two halo bytes of row ri-1 come from the neighbour lanes. Products carry the
            // float-conversion bias (v_mad_i32_i24 with a constant addend: free).
            const uint32_t Lc = from_left(P_sc), Rc = from_right(P_sc);
            uint32_t qxx[6], qyy[6], qxy[6];
            uint32_t bsq = kBiasSq, bxy = kBiasXy;
            asm volatile("" : "+s"(bsq), "+s"(bxy));  // opaque: keeps v_mad (else mul + or)  // products at columns c0-1 .. c0+4 (k = m + 1)
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int ix = win_byte(Lc, P_sc, Rc, m + 1) - win_byte(Lc, P_sc, Rc, m - 1);
                const int iy = win_byte(0, P_s, 0, m) - win_byte(0, P_su, 0, m);
                qxx[m + 1] = static_cast<uint32_t>(ix * ix) + bsq;
                qyy[m + 1] = static_cast<uint32_t>(iy * iy) + bsq;
                qxy[m + 1] = static_cast<uint32_t>(ix * iy) + bxy;
            }
            // Halo products from the neighbour lanes' edge columns (exact for lanes 0 / 63's inner
            // columns, whose neighbours are lanes 1 / 62).
            qxx[0] = from_left(qxx[4]);
            qyy[0] = from_left(qyy[4]);
            qxy[0] = from_left(qxy[4]);
            qxx[5] = from_right(qxx[1]);
            qyy[5] = from_right(qyy[1]);
            qxy[5] = from_right(qxy[1]);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                hxx[sc][m] = add3u(qxx[m], qxx[m + 1], qxx[m + 2]);
                hyy[sc][m] = add3u(qyy[m], qyy[m + 1], qyy[m + 2]);
                hxy[sc][m] = add3u(qxy[m], qxy[m + 1], qxy[m + 2]);
            }

            // Response of row rr = ri-2: vertical 3-row sums are exact integers (< 2^23).
            const int rr = ri - 2;
            const bool rowv = rr >= 2 && rr <= rows - 3;
            uint32_t sxx[4], syy[4], sxy[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                sxx[m] = add3u(hxx[s][m], hxx[su][m], hxx[sc][m]);
                syy[m] = add3u(hyy[s][m], hyy[su][m], hyy[sc][m]);
                sxy[m] = add3u(hxy[s][m], hxy[su][m], hxy[sc][m]);
            }
            const f2 r01 = corner_response2<KIND>(sxx[0], sxx[1], syy[0], syy[1], sxy[0], sxy[1], a.thr);
            const f2 r23 = corner_response2<KIND>(sxx[2], sxx[3], syy[2], syy[3], sxy[2], sxy[3], a.thr);
            const float r[4] = {r01.x, r01.y, r23.x, r23.y};
            if (!MASKED && rowv && tile_interior) {  // wave-uniform: no per-pixel masking needed
#pragma unroll
                for (int m = 0; m < 4; ++m) rsp[su][m] = r[m];
            } else {
                uint32_t mb = 0xFu;
                if constexpr (MASKED) mb = rowv ? mask_bits4(a, f, rr, c0) : 0u;
                // Lane 0's columns 2-3 and lane 63's columns 0-1 are exact and serve as the NMS
                // neighbours of the tile's edge columns.
#pragma unroll
                for (int m = 0; m < 4; ++m) rsp[su][m] = (rowv && cval[m] && ((mb >> m) & 1u)) ? r[m] : 0.0f;
            }

            // NMS of row nr = ri-3 (feature_point_harris_detector.cpp:120-137): strict, 4-neighbour.
            // x > thr and x > each neighbour  <=>  x > max(thr, neighbours)  (no NaNs; +-0 compare equal).
            const int nr = ri - 3;
            if (nr >= y0 && nr < y1) {  // wave-uniform
                const float lft = from_left_f(rsp[s][3]);
                const float rgt = from_right_f(rsp[s][0]);
                bool fl[4];
                float v[4];
                uint64_t b[4];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const float x = rsp[s][m];
                    const float xl = m == 0 ? lft : rsp[s][m - 1];
                    const float xr = m == 3 ? rgt : rsp[s][m + 1];
                    const float nb = max3f(max3f(xl, xr, a.thr), rsp[sc][m], rsp[su][m]);
                    const bool hit = x > nb;
                    v[m] = x;
                    fl[m] = colv[m] && hit;
                    b[m] = ballot(hit) & colv_b[m];  // the compare's lane mask, no bool round trip
                }
                emit_row<RASTER, kSegCorner>(sk, a, f, tx, nr, c0, b, fl, v);
                if constexpr (RASTER) {
                    if (a.resp_map != nullptr) {
                        float *mrow = a.resp_map + (static_cast<int64_t>(f) * rows + nr) * cols;
#pragma unroll
                        for (int m = 0; m < 4; ++m)
                            if (colv[m]) mrow[c0 + m] = v[m];
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// K3: FAST-12. Same tile walk with a 7-row register window (ring radius 3).
// ---------------------------------------------------------------------------------------------------
// Bresenham ring of radius 3 (kFastIndice, feature_point_fast_detector.cpp:7-8), as compile-time tables.
__device__ constexpr int ring_dx(int k) {
    constexpr int8_t t[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    return t[k];
}
__device__ constexpr int ring_dy(int k) {
    constexpr int8_t t[16] = {-3, -3, -2, -1, 0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3};
    return t[k];
}

// Longest circular run of set bits in a 16-bit ring mask (== the reference's two-pass count,
// feature_point_fast_detector.cpp:55-78; 16 when the whole ring is set).
__device__ __forceinline__ int circ_run16(uint32_t b) {
    if (b == 0xFFFFu) return 16;
    const uint32_t x = b | (b << 16);
    const uint32_t r2 = x & (x >> 1), r4 = r2 & (r2 >> 2), r8 = r4 & (r4 >> 4);
    uint32_t S = 0xFFFFFFFFu, T;
    int r = 0;
    T = S & r8;
    if (T) { S = T; r = 8; }
    T = S & (r4 >> r);
    if (T) { S = T; r += 4; }
    T = S & (r2 >> r);
    if (T) { S = T; r += 2; }
    T = S & (x >> r);
    if (T) { r += 1; }
    return r;
}

__device__ __forceinline__ float fast_offset(int nseg, const int64_t *ks, const double *os, const double *inc,
                                             int64_t k) {
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {  // last segment with k_start <= k
        const int mid = (lo + hi + 1) >> 1;
        if (ks[mid] <= k) lo = mid; else hi = mid - 1;
    }
    return static_cast<float>(os[lo] + static_cast<double>(k - ks[lo]) * inc[lo]);
}

template <bool RASTER, bool MASKED, bool ALIGNED>
__device__ __forceinline__ void fast_tile(const PointsArgs &a, const FastOffsets &off, const int64_t *seg_k,
                                          const double *seg_o, const double *seg_inc, int f, int ty, int tx, Sink &sk);

template <bool RASTER, bool MASKED, bool ALIGNED>
__global__ __launch_bounds__(256) void k_fast(PointsArgs a, FastOffsets off) {
    __shared__ DetectLds lds_all[1];
    __shared__ int64_t seg_k[kMaxOffsetSegs];
    __shared__ double seg_o[kMaxOffsetSegs], seg_inc[kMaxOffsetSegs];
    if (threadIdx.x == 0)
        for (int i = 0; i < off.nseg; ++i) {
            seg_k[i] = off.k_start[i];
            seg_o[i] = off.o_start[i];
            seg_inc[i] = off.inc[i];
        }
    __syncthreads();
    int f, ty, tx;
    const bool active = decode_tile(a, f, ty, tx);
    Sink sk{nullptr, nullptr, nullptr, 0};
    if constexpr (!RASTER) {
        const int wv = threadIdx.x >> 6;
        sk = Sink{lds_all[0].resp[wv], lds_all[0].idx[wv], a.hist0 ? lds_all[0].hist : nullptr, 0};
        if (a.hist0) hist_clear(lds_all[0].hist);
    }
    if (active) fast_tile<RASTER, MASKED, ALIGNED>(a, off, seg_k, seg_o, seg_inc, f, ty, tx, sk);
    if constexpr (!RASTER) {
        if (active) sink_flush(sk, a, f);
        if (a.hist0) hist_flush(lds_all[0].hist, a.hist0 + static_cast<int64_t>(f) * kHistBins);
    }
}

template <bool RASTER, bool MASKED, bool ALIGNED>
__device__ __forceinline__ void fast_tile(const PointsArgs &a, const FastOffsets &off, const int64_t *seg_k,
                                          const double *seg_o, const double *seg_inc, int f, int ty, int tx, Sink &sk) {
    const int lane = lane_id();
    const int rows = a.rows, cols = a.cols;
    const int c0 = tx * kTileW + 4 * (lane - 1);
    const int y0 = 3 + ty * a.tile_h;
    const int y1 = min(y0 + a.tile_h, rows - 3);  // output rows [y0, y1) within [3, rows-4]
    const auto rs = make_rsrc(a.frames + static_cast<int64_t>(f) * rows * cols, static_cast<uint32_t>(rows * cols));
    const int diff = 15;  // kMinPixelDiffValue (feature_point_fast_detector.h:14)

    bool colv[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) colv[m] = lane >= 1 && lane <= 62 && c0 + m >= 3 && c0 + m <= cols - 4;

    uint32_t P[7], L[7], R[7];
#pragma unroll
    for (int s = 0; s < 7; ++s) P[s] = L[s] = R[s] = 0;

    const int n_in = (y1 - y0) + 6;
    uint32_t nxt = load_px4<ALIGNED>(rs, (y0 - 3) * cols + c0);  // one row of prefetch
    for (int i0 = 0; i0 < n_in; i0 += 7) {
#pragma unroll
        for (int s = 0; s < 7; ++s) {
            const int ri = y0 - 3 + i0 + s;
            P[s] = nxt;
            nxt = load_px4<ALIGNED>(rs, (ri + 1) * cols + c0);
            L[s] = from_left(P[s]);
            R[s] = from_right(P[s]);
            const int orow = ri - 3;  // output row; its window rows orow-3..orow+3 are slots s+1..s (mod 7)
            if (orow < y0 || orow >= y1) continue;  // wave-uniform
#define PX(dy, j) win_byte(L[(s + 4 + (dy)) % 7], P[(s + 4 + (dy)) % 7], R[(s + 4 + (dy)) % 7], (j))
            uint32_t mb = 0xFu;
            if constexpr (MASKED) mb = mask_bits4(a, f, orow, c0);
            bool pass[4];
            int p[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                p[m] = PX(0, m);
                const int hi = p[m] + diff, lo = p[m] - diff;
                const int s4 = PX(0, m + 3), s8 = PX(3, m), s12 = PX(0, m - 3);
                // Cardinal pre-check (:20-42): samples 4, 8, 12 all brighter or all darker.
                pass[m] = colv[m] && ((mb >> m) & 1u) &&
                          ((s4 > hi && s8 > hi && s12 > hi) || (s4 < lo && s8 < lo && s12 < lo));
            }
            int score[4] = {0, 0, 0, 0};
            if (ballot(pass[0] || pass[1] || pass[2] || pass[3]) != 0ull) {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const int hi = p[m] + diff, lo = p[m] - diff;
                    uint32_t B = 0, D = 0;
#pragma unroll
                    for (int k = 0; k < 16; ++k) {
                        const int v = PX(ring_dy(k), m + ring_dx(k));
                        B |= static_cast<uint32_t>(v > hi) << k;
                        D |= static_cast<uint32_t>(v < lo) << k;
                    }
                    const int sc = max(circ_run16(B), circ_run16(D));
                    score[m] = pass[m] ? sc : 0;
                }
            }
#undef PX
            // Scan index k of each pixel among mask-true pixels (the offset counter of :85-93).
            int64_t kbase;
            uint32_t mword = 0;
            if constexpr (MASKED) {
                const int64_t rb = static_cast<int64_t>(f) * rows + orow;
                kbase = a.row_base[rb];
                if (c0 >= 0 && c0 < cols) {
                    const int w = c0 >> 5;
                    kbase += a.word_pref[rb * a.mask_wpr + w];
                    mword = a.mask[rb * a.mask_wpr + w];
                    if (w == 0) mword &= ~7u;
                }
            } else {
                kbase = static_cast<int64_t>(orow - 3) * (cols - 6) + (c0 - 3);
            }
            bool fl[4];
            float v[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                int64_t k;
                if constexpr (MASKED) {
                    k = kbase + __popc(mword & ((1u << ((c0 + m) & 31)) - 1u));  // earlier pixels in the word
                } else {
                    k = kbase + m;
                }
                const bool live = colv[m] && ((mb >> m) & 1u);
                float resp = 0.0f;
                bool cand = false;
                if (live && (score[m] > 0 || k >= off.k0)) {
                    const float o = fast_offset(off.nseg, seg_k, seg_o, seg_inc, k);
                    resp = static_cast<float>(score[m]) + o;  // :88 ComputeResponseOfPixel(...) + offset
                    cand = resp > a.thr;
                }
                fl[m] = cand;
                v[m] = resp;
            }
            const uint64_t b[4] = {ballot(fl[0]), ballot(fl[1]), ballot(fl[2]), ballot(fl[3])};
            emit_row<RASTER, kSegFast>(sk, a, f, tx, orow, c0, b, fl, v);
            if constexpr (RASTER) {
                if (a.resp_map != nullptr) {
                    float *mrow = a.resp_map + (static_cast<int64_t>(f) * rows + orow) * cols;
#pragma unroll
                    for (int m = 0; m < 4; ++m)
                        if (fl[m]) mrow[c0 + m] = v[m];
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// Prior-feature mask (feature_point_detector.cpp:90-98 + :76-88): one thread per (feature, box row)
// clears the box's bits of that row. The bitmap is preset to all ones.
// ---------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_mask_boxes(const float *prior_xy, const int32_t *prior_frame, int n_prior,
                                                    int dist, int rows, int cols, uint32_t *mask, int wpr) {
    const int span = 2 * dist + 1;
    const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= static_cast<int64_t>(n_prior) * span) return;
    const int p = static_cast<int>(t / span);
    const int dr = static_cast<int>(t % span) - dist;
    const int r0 = static_cast<int>(prior_xy[2 * p + 1]);  // static_cast<int32_t>(feature.y())
    const int cc = static_cast<int>(prior_xy[2 * p + 0]);
    const int r = r0 + dr;
    if (r < 0 || r > rows - 1) return;
    const int ca = max(cc - dist, 0), cb = min(cc + dist, cols - 1);
    if (ca > cb) return;
    uint32_t *row = mask + (static_cast<int64_t>(prior_frame[p]) * rows + r) * wpr;
    for (int w = ca >> 5; w <= (cb >> 5); ++w) {
        const int lo = max(ca - 32 * w, 0), hi = min(cb - 32 * w, 31);
        const uint32_t bits = (hi == 31 ? 0xFFFFFFFFu : ((1u << (hi + 1)) - 1u)) & ~((1u << lo) - 1u);
        atomicAnd(&row[w], ~bits);
    }
}

// Masked FAST scan index: per frame, row_base[r] = mask-true pixels of rows [3, r) in cols [3, C-4];
// word_pref[r][w] = mask-true pixels of row r in cols [3, min(32w, C-3)).
__global__ __launch_bounds__(1024) void k_fast_mask_scan(const uint32_t *mask, int wpr, int rows, int cols,
                                                         int32_t *row_base, int32_t *word_pref) {
    __shared__ int32_t tot[4096];
    const int f = blockIdx.x;
    const uint32_t *fm = mask + static_cast<int64_t>(f) * rows * wpr;
    for (int r = threadIdx.x; r < rows; r += blockDim.x) {
        int acc = 0;
        const bool rv = r >= 3 && r <= rows - 4;
        for (int w = 0; w < wpr; ++w) {
            word_pref[(static_cast<int64_t>(f) * rows + r) * wpr + w] = acc;
            uint32_t bits = rv ? fm[static_cast<int64_t>(r) * wpr + w] : 0u;
            // keep columns in [3, cols-4]
            const int lo = 3 - 32 * w, hi = (cols - 4) - 32 * w;
            if (hi < 0) bits = 0;
            else if (hi < 31) bits &= (1u << (hi + 1)) - 1u;
            if (lo > 31) bits = 0;
            else if (lo > 0) bits &= ~((1u << lo) - 1u);
            acc += __popc(bits);
        }
        if (r < 4096) tot[r] = acc;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // rows <= 4096 (checked on host); sequential scan is tiny
        int64_t acc = 0;
        for (int r = 0; r < rows; ++r) {
            row_base[static_cast<int64_t>(f) * rows + r] = static_cast<int32_t>(acc);
            acc += tot[r];
        }
    }
}

// ---------------------------------------------------------------------------------------------------
// K4: per-frame greedy selection (SelectGoodFeatures, feature_point_detector.cpp:54-88).
// Candidates are visited in (response desc, raster index asc) order without a full sort: a radix
// descent over the 64-bit key sk = (orderable response bits << 32) | ~idx cuts the frame's list into
// consecutive chunks of <= kSelectChunk keys, each gathered into LDS, bitonic-sorted and scanned by
// one wave. Accepted features live in an occupancy grid of (d+1)-sized cells: at most one accepted
// feature per cell, so a Chebyshev-distance test needs the 3x3 neighbouring cells only.
// ---------------------------------------------------------------------------------------------------
constexpr int kLevels = 8;
// digit widths per level: 12 (sign, exponent, 3 mantissa bits of the response), then 8 x 6, then 4
__device__ __forceinline__ int lvl_width(int l) { return l == 0 ? 12 : (l == 7 ? 4 : 8); }
__device__ __forceinline__ int lvl_top(int l) { return l == 7 ? 64 : 12 + 8 * l; }  // bits consumed through l
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

// Diagnostic phase clocks (only when a.stamps is set): slot 15 keeps the last clock; FD_STAMP(k)
// adds the time since then to slot k.
#define FD_STAMP(slot)                                                                  \
    do {                                                                                \
        if (a.stamps && threadIdx.x == 0) {                                             \
            const uint64_t now_ = __builtin_readcyclecounter();                         \
            uint64_t *st_ = a.stamps + blockIdx.x * 16;                                 \
            if ((slot) > 0) st_[(slot)] += now_ - st_[15];                              \
            st_[15] = now_;                                                             \
        }                                                                               \
    } while (0)

__device__ __forceinline__ uint64_t make_key(float resp, uint32_t idx) {
    return (static_cast<uint64_t>(float_key(resp)) << 32) | static_cast<uint64_t>(~idx);
}

constexpr int kPassUnroll = 8;  // independent list loads in flight per thread
constexpr int kSubChunk = 512;  // keys sorted per greedy sub-chunk

// One wave scans a sorted chunk in order (SelectGoodFeatures, feature_point_detector.cpp:62-72), a
// batch of 64 candidates at a time: occupancy-grid test against earlier batches, then the batch is
// resolved at once from cmask (per candidate: earlier candidates of its batch within distance d,
// computed beforehand by the whole workgroup).
// GRID: 0 = no distance test (d <= 0), 1 = occupancy grid in LDS, 2 = grid in global memory.
template <int GRID>
__device__ __forceinline__ void greedy_chunk(const SelectArgs &a, int f, int cnt, const uint32_t *pxy,
                                             const uint32_t *pcell, const uint64_t *cmask, uint32_t *grid, int gw2,
                                             uint32_t prior, int &s_acc, int &s_done) {
    const int lane = lane_id();
    const int d = a.dist;
    int acc = s_acc;
    bool done = false;
    for (int b0 = 0; b0 < cnt && !done; b0 += kWave) {
        const int i = b0 + lane;
        const bool in = i < cnt;
        const uint32_t e = in ? pxy[i] : kEmpty;
        bool ok = e != kEmpty;
        const int x = static_cast<int>(e & 0xFFFFu), y = static_cast<int>(e >> 16);
        int cell = gw2 + 1;
        uint64_t C = 0;
        if constexpr (GRID != 0) {
            cell = in ? static_cast<int>(pcell[i]) : gw2 + 1;
            C = in ? cmask[i] : 0ull;
            uint32_t g[9];
#pragma unroll
            for (int q = 0; q < 9; ++q) {
                const int o = cell + (q / 3 - 1) * gw2 + (q % 3 - 1);
                if constexpr (GRID == 1) g[q] = grid[o];
                else g[q] = __hip_atomic_load(&grid[o], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int q = 0; q < 9; ++q) {
                const int gx = static_cast<int>(g[q] & 0xFFFFu), gy = static_cast<int>(g[q] >> 16);
                if (g[q] != kEmpty && abs(x - gx) <= d && abs(y - gy) <= d) ok = false;
            }
        }
        const uint64_t m = ballot(ok);
        C &= m;
        // Fixed point: a lane is decided once all of C is; accepted iff none of C was accepted.
        uint64_t acc_m = 0, dec_m = ~m;
        bool mine = !ok;
        while (dec_m != ~0ull) {
            const bool can = !mine && (C & ~dec_m) == 0;
            const bool take = can && (C & acc_m) == 0;
            dec_m |= ballot(can);
            acc_m |= ballot(take);
            mine = mine || can;
        }
        // need cutoff (:67-69): features.size() >= need is checked after every append
        const uint32_t have = prior + static_cast<uint32_t>(acc);
        const int allow = have < a.need ? static_cast<int>(a.need - have) : 1;
        if (popc64(acc_m) >= allow) {
            uint64_t keep = 0, t = acc_m;
            for (int k = 0; k < allow; ++k) {
                keep |= t & (~t + 1ull);
                t &= t - 1ull;
            }
            acc_m = keep;
            done = true;
        }
        if ((acc_m >> lane) & 1ull) {
            const int pos = mbcnt64(acc_m, acc);
            if (pos < a.out_stride) {
                float2 *o = reinterpret_cast<float2 *>(a.out_xy) + static_cast<int64_t>(f) * a.out_stride + pos;
                *o = make_float2(static_cast<float>(x), static_cast<float>(y));
            }
            if constexpr (GRID != 0) {
                const uint32_t ev = (static_cast<uint32_t>(y) << 16) | static_cast<uint32_t>(x);
                if constexpr (GRID == 1) grid[cell] = ev;
                else __hip_atomic_store(&grid[cell], ev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        acc += popc64(acc_m);
        if constexpr (GRID == 2) __builtin_amdgcn_s_waitcnt(0);
    }
    if (lane == 0) {
        s_acc = acc;
        if (done) s_done = 1;
    }
}

__global__ __launch_bounds__(1024) void k_select(SelectArgs a) {
    __shared__ uint32_t suf0[kHistBins + 1];
    __shared__ uint32_t sufl[kLevels - 1][257];
    __shared__ __attribute__((aligned(16))) uint64_t sup[kSelectChunk];  // superchunk keys (unsorted)
    // sub-chunk keys (merge-sorted between buf and tmp; buf later holds the conflict masks)
    __shared__ __attribute__((aligned(16))) uint64_t buf[kSelectChunk];
    __shared__ __attribute__((aligned(16))) uint64_t tmp[kSelectChunk];
    // sorted chunk, decoded: (y << 16) | x (kEmpty when a prior masks it) and occupancy-grid cell
    __shared__ __attribute__((aligned(16))) uint32_t pxy[kSelectChunk];
    __shared__ uint32_t pcell[kSelectChunk];
    __shared__ uint32_t grid_lds[kGridLdsCells];
    __shared__ uint64_t prefix[kLevels];
    __shared__ int resume[kLevels];
    __shared__ uint32_t gcount;
    __shared__ int s_done, s_acc;

    const int f = blockIdx.x;
    const int tid = threadIdx.x, nthr = blockDim.x, lane = lane_id(), wave = tid >> 6;
    const int rows = a.rows, cols = a.cols;
    const int64_t n = min(static_cast<int64_t>(a.list_count[f]), a.list_cap);
    const float *lresp = a.list_resp + static_cast<int64_t>(f) * a.list_cap;
    const uint32_t *lidx = a.list_idx + static_cast<int64_t>(f) * a.list_cap;
    const int d = a.dist;
    const bool use_grid = d >= 1;
    // Occupancy grid of (d+1)-sized cells with a one-cell border (no bounds checks in the scan).
    const int gw2 = a.grid_w + 2;
    const int cells = gw2 * (a.grid_h + 2);
    const bool grid_in_lds = cells <= kGridLdsCells;
    uint32_t *const grid_g = a.grid_global ? a.grid_global + static_cast<int64_t>(f) * cells : nullptr;
    const uint32_t prior = a.prior_counts ? static_cast<uint32_t>(a.prior_counts[f]) : 0u;
    const uint32_t *fmask = a.mask ? a.mask + static_cast<int64_t>(f) * rows * a.mask_wpr : nullptr;
    FD_STAMP(0);

    if (use_grid) {
        if (grid_in_lds)
            for (int i = tid; i < cells; i += nthr) grid_lds[i] = kEmpty;
        else
            for (int i = tid; i < cells; i += nthr) grid_g[i] = kEmpty;
    }
    if (tid == 0) {
        s_done = 0;
        s_acc = 0;
        prefix[0] = 0;
    }
    if (n == 0) {  // RETURN_TRUE_IF(candidates_.empty()) (:55)
        if (tid == 0) a.out_counts[f] = 0;
        return;
    }

    // In-place suffix sums of S[0..nb) by the whole block; S[nb] = 0.
    __shared__ uint32_t wtot[16];
    auto suffix = [&](uint32_t *S, int nb) {
        const int ch = (nb + nthr - 1) / nthr;  // contiguous bins per thread (<= 4)
        const int b0 = min(tid * ch, nb), b1 = min(b0 + ch, nb);
        uint32_t v[4] = {0, 0, 0, 0};
        uint32_t sacc = 0;
        for (int b = b0; b < b1; ++b) {
            v[b - b0] = S[b];
            sacc += v[b - b0];
        }
        // suffix over threads: wave-level, then across the 16 waves
        uint32_t incl = sacc;
        for (int o = 1; o < kWave; o <<= 1) {
            const uint32_t t = __shfl_down(incl, o);
            if (lane + o < kWave) incl += t;
        }
        if (lane == 0) wtot[wave] = incl;
        __syncthreads();
        uint32_t after = 0;
        for (int q = wave + 1; q < nthr / kWave; ++q) after += wtot[q];
        uint32_t run = incl - sacc + after;
        for (int b = b1 - 1; b >= b0; --b) {
            run += v[b - b0];
            S[b] = run;
        }
        if (tid == 0) S[nb] = 0;
        __syncthreads();
    };
    // Histogram of digit `lvl` (>= 1) over keys in [klo, khi] (one pass over the list).
    auto build = [&](int lvl, uint64_t klo, uint64_t khi, uint32_t *S) {
        const int nb = 1 << lvl_width(lvl);
        const int rem = 64 - lvl_top(lvl);
        for (int b = tid; b <= nb; b += nthr) S[b] = 0;
        __syncthreads();
        for (int64_t b0 = tid; b0 < n; b0 += static_cast<int64_t>(kPassUnroll) * nthr) {
            float r[kPassUnroll];
            uint32_t ix[kPassUnroll];
#pragma unroll
            for (int u = 0; u < kPassUnroll; ++u) {
                const int64_t i = min(b0 + static_cast<int64_t>(u) * nthr, n - 1);
                r[u] = lresp[i];
                ix[u] = lidx[i];
            }
#pragma unroll
            for (int u = 0; u < kPassUnroll; ++u) {
                const int64_t i = b0 + static_cast<int64_t>(u) * nthr;
                const uint64_t sk = make_key(r[u], ix[u]);
                if (i < n && sk >= klo && sk <= khi) atomicAdd(&S[(sk >> rem) & static_cast<uint64_t>(nb - 1)], 1u);
            }
        }
        __syncthreads();
        suffix(S, nb);
    };
    auto suf = [&](int lvl) -> uint32_t * { return lvl == 0 ? suf0 : sufl[lvl - 1]; };

    // Level-0 histogram: accumulated by the per-pixel kernel while it emitted the candidates.
    for (int b = tid; b < kHistBins; b += nthr) suf0[b] = a.hist0[static_cast<int64_t>(f) * kHistBins + b];
    __syncthreads();
    FD_STAMP(1);
    suffix(suf0, kHistBins);
    FD_STAMP(2);
    int level = 0;
    int hi = (1 << lvl_width(0)) - 1;
    while (true) {
        if (s_done) break;
        if (hi < 0) {
            if (level == 0) break;
            --level;
            hi = resume[level];
            continue;
        }
        const uint32_t *S = suf(level);
        const uint32_t base = S[hi + 1];
        const uint32_t lim = static_cast<uint32_t>(kSelectChunk);
        // smallest lo in [0, hi] with S[lo] - base <= lim (S is non-increasing in b)
        int lo_b = 0, hi_b = hi + 1;
        while (lo_b < hi_b) {
            const int mid = (lo_b + hi_b) >> 1;
            if (S[mid] - base <= lim) hi_b = mid; else lo_b = mid + 1;
        }
        int lo = lo_b;
        const int w = lvl_width(level);
        const int rem = 64 - lvl_top(level);
        const uint64_t pre = prefix[level];
        if (lo > hi) {  // bin `hi` alone exceeds a chunk: descend into it
            __syncthreads();
            if (tid == 0) {
                resume[level] = hi - 1;
                prefix[level + 1] = (pre << w) | static_cast<uint64_t>(hi);
            }
            __syncthreads();
            const uint64_t klo = ((pre << w) | static_cast<uint64_t>(hi)) << rem;
            const uint64_t khi = klo | ((1ull << rem) - 1ull);
            ++level;
            if (a.stamps && tid == 0) a.stamps[blockIdx.x * 16 + 9] += 1;
            FD_STAMP(7);
            build(level, klo, khi, suf(level));
            FD_STAMP(6);  // descent pass
            hi = (1 << lvl_width(level)) - 1;
            continue;
        }
        const uint32_t cnt = S[lo] - base;
        FD_STAMP(7);  // loop control
        if (cnt > 0) {
            const uint64_t klo = ((pre << w) | static_cast<uint64_t>(lo)) << rem;
            const uint64_t khi = (((pre << w) | static_cast<uint64_t>(hi)) << rem) | ((1ull << rem) - 1ull);
            const uint32_t k32lo = static_cast<uint32_t>(klo >> 32), k32hi = static_cast<uint32_t>(khi >> 32);
            // gather the chunk: wave-uniform loop bounds, one LDS atomic per wave per round
            if (tid == 0) gcount = 0;
            __syncthreads();
            for (int64_t b0 = static_cast<int64_t>(wave) * kWave; b0 < n;
                 b0 += static_cast<int64_t>(kPassUnroll) * nthr) {
                float r[kPassUnroll];
                uint32_t ix[kPassUnroll];
#pragma unroll
                for (int u = 0; u < kPassUnroll; ++u) {  // unconditional (clamped) loads: all in flight
                    const int64_t i = min(b0 + static_cast<int64_t>(u) * nthr + lane, n - 1);
                    r[u] = lresp[i];
                    ix[u] = lidx[i];
                }
#pragma unroll
                for (int u = 0; u < kPassUnroll; ++u) {
                    const int64_t i = b0 + static_cast<int64_t>(u) * nthr + lane;
                    const uint32_t k32 = float_key(r[u]);
                    const bool near = i < n && k32 >= k32lo && k32 <= k32hi;  // cheap 32-bit prefilter
                    if (ballot(near) == 0ull) continue;
                    const uint64_t sk = make_key(r[u], ix[u]);
                    const bool hit = near && sk >= klo && sk <= khi;
                    const uint64_t m = ballot(hit);
                    if (m) {
                        uint32_t off = 0;
                        if (lane == 0) off = atomicAdd(&gcount, static_cast<uint32_t>(popc64(m)));
                        off = __builtin_amdgcn_readfirstlane(off);
                        if (hit) sup[mbcnt64(m, off)] = sk;
                    }
                }
            }
            __syncthreads();
            FD_STAMP(3);  // gather
            const uint32_t s1 = static_cast<uint32_t>(d + 1);
            auto place = [&](int pos, uint64_t sk) {  // decode position, prior mask, grid cell
                const uint32_t idx = ~static_cast<uint32_t>(sk);
                const uint32_t y = idx / static_cast<uint32_t>(cols);
                const uint32_t x = idx - y * static_cast<uint32_t>(cols);
                bool ok = true;
                if (fmask) ok = (fmask[static_cast<int64_t>(y) * a.mask_wpr + (x >> 5)] >> (x & 31)) & 1u;
                pxy[pos] = ok ? ((y << 16) | x) : kEmpty;
                if (use_grid) pcell[pos] = (y / s1 + 1) * static_cast<uint32_t>(gw2) + (x / s1 + 1);
            };
            // Sub-chunks of <= kSubChunk keys from the top bins of the superchunk (already in LDS):
            // the greedy usually stops within the first few hundred keys.
            int shi = hi;
            while (shi >= lo && !s_done) {
                const uint32_t sbase = S[shi + 1];
                int q0 = lo, q1 = shi + 1;
                while (q0 < q1) {
                    const int mid = (q0 + q1) >> 1;
                    if (S[mid] - sbase <= static_cast<uint32_t>(kSubChunk)) q1 = mid; else q0 = mid + 1;
                }
                const int slo = min(q0, shi);  // one bin larger than a sub-chunk is taken whole
                const uint32_t sc = S[slo] - sbase;
                if (sc > 0) {
                    const uint64_t sklo = ((pre << w) | static_cast<uint64_t>(slo)) << rem;
                    const uint64_t skhi = (((pre << w) | static_cast<uint64_t>(shi)) << rem) | ((1ull << rem) - 1ull);
                    if (tid == 0) gcount = 0;
                    __syncthreads();
                    for (int b0 = wave * kWave; b0 < static_cast<int>(cnt); b0 += nthr) {
                        const int i = b0 + lane;
                        const uint64_t sk = i < static_cast<int>(cnt) ? sup[i] : 0ull;
                        const bool hit = i < static_cast<int>(cnt) && sk >= sklo && sk <= skhi;
                        const uint64_t m = ballot(hit);
                        if (m) {
                            uint32_t off = 0;
                            if (lane == 0) off = atomicAdd(&gcount, static_cast<uint32_t>(popc64(m)));
                            off = __builtin_amdgcn_readfirstlane(off);
                            if (hit) buf[mbcnt64(m, off)] = sk;
                        }
                    }
                    __syncthreads();
                    FD_STAMP(10);  // sub-chunk extract
                {
                    // Merge sort of unique keys, descending: rank inside runs of 64 by counting larger
                    // keys (broadcast LDS reads), then log2 merge levels where each key moves to
                    // (its offset in its run) + (number of larger keys in the sibling run, by binary search).
                    const int c = static_cast<int>(sc);
                    const int c64 = (c + 63) & ~63;
                    for (int i = c + tid; i < c64; i += nthr) buf[i] = 0ull;
                    __syncthreads();
                    for (int p = tid; p < c; p += nthr) {
                        const uint64_t me = buf[p];
                        const ulonglong2 *b2 = reinterpret_cast<const ulonglong2 *>(buf + (p & ~63));
                        int lr = 0;
    #pragma unroll 8
                        for (int j = 0; j < 32; ++j) {
                            const ulonglong2 q = b2[j];
                            lr += (q.x > me) + (q.y > me);
                        }
                        tmp[(p & ~63) + lr] = me;
                    }
                    __syncthreads();
                    FD_STAMP(11);  // run sort
                    uint64_t *src = tmp, *dst = buf;
                    for (int w = 64; w < c; w <<= 1) {
                        for (int p = tid; p < c; p += nthr) {
                            const uint64_t me = src[p];
                            const int run = p / w;
                            const int pair = (run & ~1) * w;
                            const int sib = (run ^ 1) * w;
                            int lo2 = 0, hi2 = max(0, min(w, c - sib));  // larger keys in the sibling run
                            while (lo2 < hi2) {
                                const int mid = (lo2 + hi2) >> 1;
                                if (src[sib + mid] > me) lo2 = mid + 1; else hi2 = mid;
                            }
                            dst[pair + (p - run * w) + lo2] = me;
                        }
                        __syncthreads();
                        uint64_t *t2 = src;
                        src = dst;
                        dst = t2;
                    }
                    FD_STAMP(12);  // merges
                    for (int i = tid; i < c; i += nthr) place(i, src[i]);
                    __syncthreads();
                    FD_STAMP(13);  // place
                    // conflict masks: earlier candidates of the same 64-batch within distance d
                    if (use_grid) {
                        for (int p = tid; p < c; p += nthr) {
                            const uint32_t e = pxy[p];
                            const int x = static_cast<int>(e & 0xFFFFu), y = static_cast<int>(e >> 16);
                            uint64_t C = 0;
                            const int bb = p & ~63, me = p - bb;
                            const uint4 *q4 = reinterpret_cast<const uint4 *>(pxy + bb);  // broadcast reads
                            const int n4 = (me + 3) >> 2;  // only earlier entries matter
#pragma unroll 2
                            for (int j4 = 0; j4 < n4; ++j4) {
                                const uint4 e4 = q4[j4];
                                const uint32_t ev[4] = {e4.x, e4.y, e4.z, e4.w};
                                uint32_t bits = 0;
#pragma unroll
                                for (int t = 0; t < 4; ++t) {
                                    const int ex = static_cast<int>(ev[t] & 0xFFFFu), ey = static_cast<int>(ev[t] >> 16);
                                    const bool nb = j4 * 4 + t < me && ev[t] != kEmpty && abs(x - ex) <= d && abs(y - ey) <= d;
                                    bits |= static_cast<uint32_t>(nb) << t;
                                }
                                C |= static_cast<uint64_t>(bits) << (j4 * 4);
                            }
                            buf[p] = e == kEmpty ? 0ull : C;
                        }
                    }
                }
                __syncthreads();
                FD_STAMP(14);  // conflict masks
                // greedy scan in order by wave 0 (SelectGoodFeatures :62-72)
                if (tid < kWave) {
                    const int c = static_cast<int>(sc);
                    if (!use_grid)
                        greedy_chunk<0>(a, f, c, pxy, pcell, buf, grid_lds, gw2, prior, s_acc, s_done);
                    else if (grid_in_lds)
                        greedy_chunk<1>(a, f, c, pxy, pcell, buf, grid_lds, gw2, prior, s_acc, s_done);
                    else
                        greedy_chunk<2>(a, f, c, pxy, pcell, buf, grid_g, gw2, prior, s_acc, s_done);
                }
                __syncthreads();
                FD_STAMP(5);  // greedy
                }
                shi = slo - 1;
            }
            if (a.stamps && tid == 0) a.stamps[blockIdx.x * 16 + 8] += 1;
        }
        hi = lo - 1;
    }
    if (tid == 0) a.out_counts[f] = s_acc;
    FD_STAMP(7);
}

// ---------------------------------------------------------------------------------------------------
// K2: raster compaction of the per-(row, tile) segments into the reference's push order.
// ---------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_compact(CompactArgs a) {
    __shared__ int64_t wsum[16];
    __shared__ int64_t carry;
    const int f = blockIdx.x;
    const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
    const int nseg = (a.row_hi - a.row_lo) * a.tiles_x;
    const int32_t *cnt = a.seg_cnt + (static_cast<int64_t>(f) * a.rows + a.row_lo) * a.tiles_x;
    const Cand *seg = a.seg + (static_cast<int64_t>(f) * a.rows + a.row_lo) * a.tiles_x * a.seg_cap;
    float *oresp = a.out_resp + static_cast<int64_t>(f) * a.cap;
    int32_t *ox = a.out_x + static_cast<int64_t>(f) * a.cap;
    int32_t *oy = a.out_y + static_cast<int64_t>(f) * a.cap;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int s0 = 0; s0 < nseg; s0 += 1024) {
        const int s = s0 + tid;
        const int c = s < nseg ? cnt[s] : 0;
        // block exclusive scan of c
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
        if (tid == 1023) carry = start + c;
        for (int e = 0; e < c; ++e) {
            const int64_t pos = start + e;
            if (pos < a.cap) {
                const Cand cd = seg[static_cast<int64_t>(s) * a.seg_cap + e];
                const int y = static_cast<int>(cd.idx / static_cast<uint32_t>(a.cols));
                oresp[pos] = cd.resp;
                ox[pos] = static_cast<int32_t>(cd.idx - static_cast<uint32_t>(y) * a.cols);
                oy[pos] = y;
            }
        }
        __syncthreads();
    }
    if (tid == 0) a.out_counts[f] = carry;
}

}  // namespace

// ---------------------------------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------------------------------
static inline int blocks_for_waves(const PointsArgs &a) {
    return a.batch * a.blocks_per_frame;
}

hipError_t launch_corner(int kind, bool raster, const PointsArgs &a, hipStream_t s) {
    const dim3 grid(blocks_for_waves(a)), block(256);
    const bool masked = a.mask != nullptr, aligned = a.aligned4 != 0;
#define FD_CORNER(K, RS, M)                                                                  \
    do {                                                                                     \
        if (aligned) hipLaunchKernelGGL((k_corner<K, RS, M, true>), grid, block, 0, s, a);  \
        else hipLaunchKernelGGL((k_corner<K, RS, M, false>), grid, block, 0, s, a);         \
    } while (0)
    if (kind == 0) {
        if (raster) { if (masked) FD_CORNER(0, true, true); else FD_CORNER(0, true, false); }
        else { if (masked) FD_CORNER(0, false, true); else FD_CORNER(0, false, false); }
    } else {
        if (raster) { if (masked) FD_CORNER(1, true, true); else FD_CORNER(1, true, false); }
        else { if (masked) FD_CORNER(1, false, true); else FD_CORNER(1, false, false); }
    }
#undef FD_CORNER
    return hipGetLastError();
}

hipError_t launch_fast(bool raster, const PointsArgs &a, const FastOffsets &off, hipStream_t s) {
    const dim3 grid(blocks_for_waves(a)), block(256);
    const bool masked = a.mask != nullptr, aligned = a.aligned4 != 0;
#define FD_FAST(RS, M)                                                                          \
    do {                                                                                        \
        if (aligned) hipLaunchKernelGGL((k_fast<RS, M, true>), grid, block, 0, s, a, off);     \
        else hipLaunchKernelGGL((k_fast<RS, M, false>), grid, block, 0, s, a, off);            \
    } while (0)
    if (raster) { if (masked) FD_FAST(true, true); else FD_FAST(true, false); }
    else { if (masked) FD_FAST(false, true); else FD_FAST(false, false); }
#undef FD_FAST
    return hipGetLastError();
}

hipError_t launch_mask_boxes(const float *prior_xy, const int32_t *prior_frame, int n_prior, int dist, int rows,
                             int cols, uint32_t *mask, int mask_wpr, hipStream_t s) {
    if (n_prior <= 0 || dist < 0) return hipSuccess;
    const int64_t threads = static_cast<int64_t>(n_prior) * (2 * dist + 1);
    hipLaunchKernelGGL(k_mask_boxes, dim3(static_cast<unsigned>((threads + 255) / 256)), dim3(256), 0, s, prior_xy,
                       prior_frame, n_prior, dist, rows, cols, mask, mask_wpr);
    return hipGetLastError();
}

hipError_t launch_fast_mask_scan(const uint32_t *mask, int mask_wpr, int batch, int rows, int cols, int32_t *row_base,
                                 int32_t *word_pref, hipStream_t s) {
    hipLaunchKernelGGL(k_fast_mask_scan, dim3(batch), dim3(1024), 0, s, mask, mask_wpr, rows, cols, row_base,
                       word_pref);
    return hipGetLastError();
}

hipError_t launch_select(const SelectArgs &a, int batch, hipStream_t s) {
    hipLaunchKernelGGL(k_select, dim3(batch), dim3(1024), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_compact(const CompactArgs &a, int batch, hipStream_t s) {
    hipLaunchKernelGGL(k_compact, dim3(batch), dim3(1024), 0, s, a);
    return hipGetLastError();
}

}  // namespace fdk
