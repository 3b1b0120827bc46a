// K1 for fd_points_detect / fd_points_response with thr >= 0: lane-private candidate emission (see
// the kernel comment). gfx950 (MI355X). Reference (paths relative to src/feature_point_detector/):
//   gradient + 3x3 tensor ........ feature_point_harris_detector.cpp:17-64, :66-88, :108-116
//   Harris response .............. feature_point_harris_detector.cpp:94-104
//   Shi-Tomasi response .......... feature_point_shi_tomas_detector.cpp:94-103
//   4-neighbour NMS .............. feature_point_harris_detector.cpp:120-137
// Build flags matter: -ffp-contract=off and correctly rounded f32 sqrt/div (see fd_points.hip).
#include "fd_corner_common.h"

#include <type_traits>

// Shi-Tomasi's gate as a clamp (corner_response_fp; A/B switch)
#ifndef FD_LP_GFMA
#define FD_LP_GFMA 1
#endif

namespace fdk {

namespace {

// corner_response2<KIND, G1 = true> for k_corner_lp: Shi-Tomasi returns 2r = gate + sqrt(d*d + 4b*b),
// i.e. the reference's fl(fl(gate + common) * 0.5) times two (exact), one multiply fewer per pixel.
template <int KIND>
__device__ __forceinline__ f2 corner_response_lp(uint32_t sxx0, uint32_t sxx1, uint32_t syy0, uint32_t syy1,
                                                 uint32_t sxy0, uint32_t sxy1, float thr) {
    if constexpr (KIND == 0) return corner_response2<0, true>(sxx0, sxx1, syy0, syy1, sxy0, sxy1, thr);
    const f2 bxx = f2{__uint_as_float(sxx0), __uint_as_float(sxx1)};
    const f2 byy = f2{__uint_as_float(syy0), __uint_as_float(syy1)};
    const f2 fxy = f2{__uint_as_float(sxy0), __uint_as_float(sxy1)} - 12582912.0f;
    const f2 a = __builtin_elementwise_fma(bxx, f2{kInvCnt, kInvCnt}, f2{-8388608.0f * kInvCnt, -8388608.0f * kInvCnt});
    const f2 c = __builtin_elementwise_fma(byy, f2{kInvCnt, kInvCnt}, f2{-8388608.0f * kInvCnt, -8388608.0f * kInvCnt});
    const f2 gate = a + c;
    const f2 b = fxy * kInvCnt;
    const f2 d = a - c;
    const f2 r2 = gate + sqrt_rn_rsq2(__builtin_elementwise_fma(b * b, f2{4.0f, 4.0f}, d * d));
    f2 res;
    res.x = gate.x > thr ? r2.x : 0.0f;
    res.y = gate.y > thr ? r2.y : 0.0f;
    return res;
}

// Byte K of w as a float (v_cvt_f32_ubyteK; as asm so that differences of converted bytes stay float
// subtractions instead of becoming an integer subtraction plus a conversion).
template <int K>
__device__ __forceinline__ float cvt_ubyte(uint32_t w) {
    float r;
    if constexpr (K == 0) asm("v_cvt_f32_ubyte0_e32 %0, %1" : "=v"(r) : "v"(w));
    else if constexpr (K == 1) asm("v_cvt_f32_ubyte1_e32 %0, %1" : "=v"(r) : "v"(w));
    else if constexpr (K == 2) asm("v_cvt_f32_ubyte2_e32 %0, %1" : "=v"(r) : "v"(w));
    else asm("v_cvt_f32_ubyte3_e32 %0, %1" : "=v"(r) : "v"(w));
    return r;
}

// a + (lane i+1's b; 0 for lane 63) as one v_add_f32_dpp (the compiler leaves a v_mov_b32_dpp when
// the halo's source register is reused before the add)
__device__ __forceinline__ float add_from_right_f(float a, float b) {
    float r;
    asm("v_add_f32_dpp %0, %1, %2 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(r) : "v"(b), "v"(a));
    return r;
}

// The same responses from float tensor sums (exact integers < 2^24 held as floats, FD_LP_FP), G1 form,
// gate test as a sign mask (thr - gate < 0 <=> gate > thr): full-rate float ops only.
// Shi-Tomasi: sqrt_rn_rsq2 (fd_device.h), verified exhaustively. (Folding its halving into rsq's output
// modifier was tried: gfx950 does not apply div:2 to v_rsq_f32 -- 1-ulp errors.) This translation unit
// flushes f32 denormals; none occur (products and sums are integers, q is 0 or >= 2^-54).
template <int KIND>
__device__ __forceinline__ f2 corner_response_fp(f2 sxx, f2 syy, f2 sxy, float thr) {
    f2 gate, r;
    if constexpr (KIND == 0) {  // Harris, feature_point_harris_detector.cpp:95-103
        const f2 trace = sxx + syy;
        gate = ((trace * trace) * 0.21f) * kInvCnt2;
        r = (((sxx * syy) - (sxy * sxy)) - ((kHarrisAlpha * trace) * trace)) * kInvCnt2;
    } else {  // Shi-Tomasi, feature_point_shi_tomas_detector.cpp:94-103 (2r)
        const f2 a = sxx * kInvCnt, c = syy * kInvCnt, b = sxy * kInvCnt;
        gate = a + c;
        const f2 d = a - c;
        r = gate + sqrt_rn_rsq2(__builtin_elementwise_fma(b * b, f2{4.0f, 4.0f}, d * d));
#if FD_LP_GFMA
        // The gate as a clamp: min(2r, fl(66 gate - 64 thr)). gate > thr: 66g - 64t = 2g + 64(g - t) >=
        // 2g + 32 ulp(g) > 2r (the tensor is positive semidefinite, so sqrt(d^2 + 4b^2) <= gate up to ~6
        // ulp of rounding), i.e. 2r itself. gate <= thr: the value is <= 2 gate <= 2 thr, which neither
        // wins the NMS (it needs > 2 thr) nor changes a neighbour's outcome (a winner exceeds 2 thr, so it
        // exceeds this value exactly when it exceeds the reference's 0). Winners keep their exact 2r.
        const f2 cl = __builtin_elementwise_fma(gate, f2{66.0f, 66.0f}, f2{-64.0f * thr, -64.0f * thr});
        f2 res;
        res.x = __builtin_fminf(r.x, cl.x);
        res.y = __builtin_fminf(r.y, cl.y);
        return res;
#endif
    }
    const f2 g = f2{thr, thr} - gate;  // < 0 exactly when gate > thr
    f2 res;
    res.x = __int_as_float(__float_as_int(r.x) & (__float_as_int(g.x) >> 31));
    res.y = __int_as_float(__float_as_int(r.y) & (__float_as_int(g.y) >> 31));
    return res;
}

#ifndef FD_LP_FP
#define FD_LP_FP 1
#endif
#ifndef FD_LP_PKQ
#define FD_LP_PKQ 1
#endif


// ---------------------------------------------------------------------------------------------------
// K1 (list mode, lane-private emission): the per-pixel kernel of fd_points_detect / fd_points_response.
//
// Same arithmetic as corner_tile (biased exact integer tensor, the reference's float order, strict
// 4-neighbour NMS), re-shaped for the instruction stream:
//  * PX columns per lane (2, 4 or 8): the DPP halo exchanges, the NMS neighbour fetches and the loop
//    control are shared by PX pixels; the launch picks PX for its size (small launches: more waves);
//  * candidates go to lane-private LDS slots with no wave-level compaction in the row loop: the NMS
//    compare becomes the exec mask of one slot write and one address increment (lp_emit), so the row
//    loop carries no ballot, popcount or branch per candidate; the wave compacts its slots only when a
//    lane may run out (lp_flush: one slot index per store instruction, so every store is a contiguous run);
//  * Shi-Tomasi keeps 2r = gate + sqrt(...) (the reference's (gate + sqrt) * 0.5 without the halving:
//    exact, and the NMS compares 2r against 2thr identically); the halving happens at the flush;
//  * the centre-column validity (halo lanes: 0 and 63, or 0-1 and 62-63 at PX = 2) is a per-lane NMS
//    threshold of +inf: with thr >= 0 (G1) every other invalid column already holds 0, which never wins.
// Only for thr >= 0 (the single-gate form); negative thresholds use k_corner.
// ---------------------------------------------------------------------------------------------------
constexpr int kLpSlots = FD_LP_SLOTS;  // lane-private slots per lane (LDS: 8 B x 64 lanes each)
// With the selection histogram (16 KiB) the workgroup's LDS is slots + histogram: FD_LP_SLOTS_H slots
// keep it (with the sorted-segment words) under 40 KiB: 4 workgroups per CU instead of 3 at 48 KiB.
#ifndef FD_LP_SLOTS_H
#define FD_LP_SLOTS_H 11
#endif
template <bool HIST>
constexpr int lp_slots() { return HIST ? FD_LP_SLOTS_H : kLpSlots; }

// Occupancy the register allocation must allow: LDS admits 5 workgroups (20 waves) per CU without the
// histogram, 4 with it (FD_LP_SLOTS_H = 11); the allocator then keeps <= 96 / <= 128 VGPRs (8 columns
// per lane and the unaligned no-histogram variants would spill at those limits: no target).
#ifndef FD_LP_WAVES
#define FD_LP_WAVES(PX, HIST, ALIGNED) __attribute__((amdgpu_waves_per_eu((PX) == 8 ? 1 : (HIST) || !(ALIGNED) ? 4 : 5)))
#endif

template <int PX>
struct LpGeom {
    static constexpr int NW = PX >= 4 ? PX / 4 : 1;  // registers per row (PX = 2: one 16-bit load)
    static constexpr int LB = PX == 2 ? 2 : 4;       // bytes a neighbour lane supplies per side
    static constexpr int HL = lp_halo_lanes(PX);     // halo-only lanes per side
    static constexpr int TW = lp_tile_w(PX);         // output columns per wave
};

template <bool HIST>
struct alignas(16) LpLds {  // (hist is cleared and read as uint4, fd_corner_common.h)
    uint32_t slot[4][lp_slots<true>()][128];  // [wave][slot][0..63 response bits | 64..127 raster index]
    uint32_t hist[kHistBins];
    uint32_t seg_ovf;  // sorted-segment mode: a wave flushed before the end (the segment is unsorted)
};
// Without the histogram the slots alone: exactly 32 KiB at 16 slots, so 5 workgroups (20 waves) fit a
// CU's 160 KiB (one extra word made it 4).
template <>
struct alignas(16) LpLds<false> {
    uint32_t slot[4][lp_slots<false>()][128];
    static constexpr uint32_t *hist = nullptr;  // (never used: keeps L.hist well-formed)
};

// One row's pixels of the lane's PX columns (out-of-range bytes read 0 through the buffer resource).
template <int PX, bool ALIGNED>
__device__ __forceinline__ void lp_load_row(uint32_t (&w)[LpGeom<PX>::NW], __amdgpu_buffer_rsrc_t r, int32_t off) {
    if constexpr (PX == 2) {
        if constexpr (ALIGNED) w[0] = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0));
        else w[0] = buf_load_u8(r, off) | (buf_load_u8(r, off + 1) << 8);
    } else {
#pragma unroll
        for (int q = 0; q < LpGeom<PX>::NW; ++q) w[q] = load_px4<ALIGNED>(r, off + 4 * q);
    }
}

// Byte j (compile-time, -LB <= j < PX + LB) of the row window [L | P | R]: L = the left lane's last
// LB columns, R = the right lane's first LB columns.
template <int PX>
__device__ __forceinline__ int lp_byte(uint32_t L, const uint32_t (&P)[LpGeom<PX>::NW], uint32_t R, int j) {
    constexpr int LB = LpGeom<PX>::LB;
    uint32_t w;
    int b;
    if (j < 0) w = L, b = j + LB;
    else if (j < PX) w = P[j >> 2], b = j & 3;
    else w = R, b = j - PX;
    return static_cast<int>((w >> (8 * b)) & 0xFFu);
}

template <int PX>
__device__ __forceinline__ uint32_t lp_mask_bits(const PointsArgs &a, int f, int row, int c0) {
    if (c0 < 0 || c0 >= a.cols) return 0u;
    const uint32_t w = a.mask[(static_cast<int64_t>(f) * a.rows + row) * a.mask_wpr + (c0 >> 5)];
    return (w >> (c0 & 31)) & ((1u << PX) - 1u);  // c0 is a multiple of PX: the PX bits share a word
}

// Entry (j, lane) of the wave's slots as (response, raster index). Shi-Tomasi slots hold 2r.
template <int KIND>
__device__ __forceinline__ float lp_resp(const uint32_t *sl, int j) {
    const float v = __uint_as_float(sl[j * 128]);
    return KIND == 1 ? v * 0.5f : v;
}

// Append the wave's slot entries to the frame's list: one atomic for the wave, then per slot index j
// the lanes holding an entry j store it at consecutive positions (coalesced), level-0 histogram in LDS.
template <int KIND>
__device__ __forceinline__ void lp_flush(uint32_t &n, const uint32_t *sl, const PointsArgs &a, int f, uint32_t *hist) {
    int jmax = 0;
    uint32_t tot = 0;
    for (;;) {  // (uniform) total = sum over j of the lanes holding entry j
        const uint64_t b = ballot(n > static_cast<uint32_t>(jmax));
        if (b == 0) break;
        tot += static_cast<uint32_t>(popc64(b));
        ++jmax;
    }
    if (tot == 0) return;
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&a.list_count[f], tot);
    base = __builtin_amdgcn_readfirstlane(base);
    // The frame's list as two buffer resources of list_cap entries: a position past the capacity is
    // outside the range and its store is dropped by the hardware (no compare, no 64-bit address math;
    // the launch keeps list_cap * 4 < 2^32, lp_list_ok).
    const uint32_t cap_b = static_cast<uint32_t>(a.list_cap) * 4u;
    const auto rr = make_rsrc(a.list_resp + static_cast<int64_t>(f) * a.list_cap, cap_b);
    const auto ri = make_rsrc(a.list_idx + static_cast<int64_t>(f) * a.list_cap, cap_b);
    uint32_t off = base;
    for (int j = 0; j < jmax; ++j) {
        const uint64_t b = ballot(n > static_cast<uint32_t>(j));
        if (n > static_cast<uint32_t>(j)) {
            const float r = lp_resp<KIND>(sl, j);
            if (hist) atomicAdd(&hist[((float_key(r) - a.key_base) << a.key_lz) >> 20], 1u);
            const uint32_t pos4 = static_cast<uint32_t>(mbcnt64(b, static_cast<int>(off))) << 2;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r), rr, static_cast<int>(pos4), 0, FD_LIST_NT ? 2 : 0);
            __builtin_amdgcn_raw_buffer_store_b32(sl[j * 128 + 64], ri, static_cast<int>(pos4), 0, FD_LIST_NT ? 2 : 0);
        }
        off += static_cast<uint32_t>(popc64(b));
    }
    // drain here (rare path) so the row loop's waitcnt state stays "loads only"
    __builtin_amdgcn_s_waitcnt(0x0F70);
    n = 0;
}

// Sorted-segment flush of the lane-private slots (small launches, PointsArgs::segdesc): as seg_flush.
template <int KIND>
__device__ __forceinline__ void lp_seg_flush(uint32_t &n, const uint32_t *sl, const PointsArgs &a, int f, bool active,
                                             LpLds<true> &L, uint32_t *ovf, uint32_t (&wtot)[4], uint32_t &wg_base) {
    const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
    __syncthreads();
    if (*ovf) {  // part of the workgroup's list is already out unsorted: plain flush (frame marked)
        if (active) lp_flush<KIND>(n, sl, a, f, L.hist);
        hist_flush(L.hist, a.hist0 + static_cast<int64_t>(f) * kHistBins);
        return;
    }
    if (!active) n = 0;
    auto bin_of = [&](float r) { return ((float_key(r) - a.key_base) << a.key_lz) >> 20; };
    for (int j = 0; j < lp_slots<true>(); ++j) {
        if (ballot(n > static_cast<uint32_t>(j)) == 0) break;
        if (n > static_cast<uint32_t>(j)) atomicAdd(&L.hist[bin_of(lp_resp<KIND>(sl, j))], 1u);
    }
    hist_flush(L.hist, a.hist0 + static_cast<int64_t>(f) * kHistBins);  // (leads with a barrier)
    __syncthreads();
    constexpr int kPer = kHistBins / 256;
    uint32_t v[kPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) sum += (v[k] = L.hist[kHistBins - 1 - (tid * kPer + k)]);
    const uint32_t incl = wave_incl_add(sum);
    if (lane == kWave - 1) wtot[wv] = incl;
    __syncthreads();
    uint32_t run = incl - sum, total = 0;
    for (int q = 0; q < 4; ++q) {
        run += q < wv ? wtot[q] : 0u;
        total += wtot[q];
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        L.hist[kHistBins - 1 - (tid * kPer + k)] = run;
        run += v[k];
    }
    if (tid == 0) {
        wg_base = total ? atomicAdd(&a.list_count[f], total) : 0u;
        const int g = logical_block() % a.blocks_per_frame;
        a.segdesc[static_cast<int64_t>(f) * a.blocks_per_frame + g] = make_uint2(wg_base, total);
    }
    __syncthreads();
    float *dr = a.list_resp + static_cast<int64_t>(f) * a.list_cap;
    uint32_t *di = a.list_idx + static_cast<int64_t>(f) * a.list_cap;
    const int64_t base = wg_base;
    const int g = logical_block() % a.blocks_per_frame;
    uint64_t *head = a.seghead + (static_cast<int64_t>(f) * a.blocks_per_frame + g) * kSegHead;
    for (int j = 0; j < lp_slots<true>(); ++j) {
        if (ballot(n > static_cast<uint32_t>(j)) == 0) break;
        if (n > static_cast<uint32_t>(j)) {
            const float r = lp_resp<KIND>(sl, j);
            const uint32_t id = sl[j * 128 + 64];
            const uint32_t k32 = (float_key(r) - a.key_base) << a.key_lz;
            const uint32_t lp = atomicAdd(&L.hist[k32 >> 20], 1u);
            const int64_t pos = base + lp;
            if (pos < a.list_cap) {
                dr[pos] = r;
                di[pos] = id;
            }
            if (lp < static_cast<uint32_t>(kSegHead)) head[lp] = (static_cast<uint64_t>(k32) << 32) | static_cast<uint64_t>(~id);
        }
    }
    n = 0;
}

// One column's candidate: if x > nb, (x, id) goes to the lane's next slot (LDS byte address A: response
// word, index word 256 B later) and A advances one slot. Exec-masked to the hit lanes, so only
// candidates cost LDS bandwidth (an unconditional write per column halved K1's LDS-bound throughput)
// and the VALU cost per column is one full-rate add beyond the NMS compare.
__device__ __forceinline__ void lp_emit(uint32_t &A, float x, float nb, uint32_t id) {
    uint64_t hit, save;
    asm volatile(
        "v_cmp_gt_f32_e64 %1, %3, %4\n\t"
        "s_and_saveexec_b64 %2, %1\n\t"
        "ds_write2st64_b32 %0, %3, %5 offset1:1\n\t"
        "v_add_u32_e32 %0, 0x200, %0\n\t"
        "s_mov_b64 exec, %2"
        : "+v"(A), "=&s"(hit), "=&s"(save)
        : "v"(x), "v"(nb), "v"(id)
        : "memory");
}

template <int KIND, int PX, bool MASKED, bool ALIGNED, bool HIST, bool SEG>
FD_LP_WAVES(PX, HIST, ALIGNED) __global__ __launch_bounds__(256) void k_corner_lp(PointsArgs a) {
    using G = LpGeom<PX>;
    constexpr int NW = G::NW;
    __shared__ LpLds<HIST> L;
    int f, ty, tx;
    const bool active = decode_tile(a, f, ty, tx);
    const int lane = lane_id(), wv = threadIdx.x >> 6;
    uint32_t *sl = &L.slot[wv][0][lane];
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    const uint32_t sl_addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((lds_u32 *)sl));  // LDS byte address
    if constexpr (SEG) {
        if (threadIdx.x == 0) L.seg_ovf = 0;
    }
    if constexpr (HIST) hist_clear(L.hist);
    else if constexpr (SEG) __syncthreads();
    uint32_t *lhist = HIST ? L.hist : nullptr;
    uint32_t A = sl_addr;  // LDS byte address of this lane's next free slot (slot n at sl_addr + 512 n)

    if (active) {
        const int rows = a.rows, cols = a.cols;
        const int c0 = tx * G::TW + PX * (lane - G::HL);
        const int y0 = 2 + ty * a.tile_h;
        const int y1 = min(y0 + a.tile_h, rows - 2);  // output rows [y0, y1) within [2, rows-3]
        const auto rs = make_rsrc(a.frames + static_cast<int64_t>(f) * rows * cols, static_cast<uint32_t>(rows * cols));
        const bool tile_interior = tx * G::TW - PX * G::HL >= 2 && tx * G::TW + PX * (64 - G::HL) - 1 <= cols - 3;
        bool cval[PX];
#pragma unroll
        for (int m = 0; m < PX; ++m) cval[m] = c0 + m >= 2 && c0 + m <= cols - 3;
        // NMS threshold per lane: the halo lanes never emit (their columns belong to the neighbour waves'
        // interior lanes); Shi-Tomasi compares 2r against 2thr.
        const float thr_n = (KIND == 1 ? 2.0f : 1.0f) * a.thr;
        const float thrv = (lane >= G::HL && lane <= 63 - G::HL) ? thr_n : __builtin_inff();

#if FD_LP_FP
        f2 hxx[3][PX / 2], hyy[3][PX / 2], hxy[3][PX / 2];  // column pairs: the vertical sums are packed adds
        float fpx[3][PX];  // the rows in use as floats, same 3-slot roles as the sums
#else
        uint32_t hxx[3][PX], hyy[3][PX], hxy[3][PX];
#endif
        float rsp[3][PX];
#if FD_LP_FP
        // vertical pair sums shared by two consecutive output rows: an even step forms
        // h(ri-2) + h(ri-1) and adds h(ri-3), the next step adds h(ri) to the same pair (exact integers)
        f2 pxx[PX / 2], pyy[PX / 2], pxy[PX / 2];
#endif
#if FD_LP_FP
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int m = 0; m < PX; ++m) {
                if (m % 2 == 0) hxx[s][m / 2] = hyy[s][m / 2] = hxy[s][m / 2] = f2{0.0f, 0.0f};
                fpx[s][m] = rsp[s][m] = 0.0f;
            }
#else
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int m = 0; m < PX; ++m) hxx[s][m] = hyy[s][m] = hxy[s][m] = 0, rsp[s][m] = 0.0f;
#endif

        const int n_in = (y1 - y0) + 6;
        uint32_t ring[6][NW];
#pragma unroll
        for (int t = 0; t < 6; ++t) {
            if (t < 3) lp_load_row<PX, ALIGNED>(ring[t], rs, (y0 - 3 + t) * cols + c0);
            else
#pragma unroll
                for (int q = 0; q < NW; ++q) ring[t][q] = 0u;
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);
        // One row step; t (compile-time) is the step's place in the 6-row ring. Whole 6-step iterations
        // run in a loop with no exit inside the body (an exit edge per step costs the loop header a
        // vmcnt(0), i.e. the row prefetch), the tail of a short tile in a second copy with exits.
        auto step = [&](auto tc, int i0) {
                constexpr int t = decltype(tc)::value;
                const int s = t % 3, su = (t + 1) % 3, sc = (t + 2) % 3;  // rows ri, ri-2, ri-1
                const int ri = y0 - 3 + i0 + t;
                lp_load_row<PX, ALIGNED>(ring[(t + 3) % 6], rs, (ri + 3) * cols + c0);
                const uint32_t(&P_s)[NW] = ring[t];
#if !FD_LP_FP
                const uint32_t(&P_su)[NW] = ring[(t + 4) % 6];
                const uint32_t(&P_sc)[NW] = ring[(t + 5) % 6];
#endif

#if FD_LP_FP
                // row ri as floats (each row is converted once and used at three steps)
#pragma unroll
                for (int m = 0; m < PX; m += 4) {
                    fpx[s][m] = cvt_ubyte<0>(P_s[m >> 2]);
                    fpx[s][m + 1] = cvt_ubyte<1>(P_s[m >> 2]);
                    if constexpr (PX >= 4) {
                        fpx[s][m + 2] = cvt_ubyte<2>(P_s[m >> 2]);
                        fpx[s][m + 3] = cvt_ubyte<3>(P_s[m >> 2]);
                    }
                }
                // gradients of row ri-1 (feature_point_harris_detector.cpp:35-62) and products as exact
                // float integers; the halo pixels and the halo columns' products from the neighbour lanes
                const float fL = from_left_f(fpx[sc][PX - 1]), fR = from_right_f(fpx[sc][0]);
                float qxx[PX + 2], qyy[PX + 2], qxy[PX + 2];
#if FD_LP_PKQ
                // column pairs: iy and the three products as packed ops (2 results per issue slot;
                // separate full-rate ops pair up only when two waves offer them in the same cycle)
#pragma unroll
                for (int m = 0; m < PX; m += 2) {
                    const f2 ix = f2{(m + 1 < PX ? fpx[sc][m + 1] : fR) - (m > 0 ? fpx[sc][m - 1] : fL),
                                     (m + 2 < PX ? fpx[sc][m + 2] : fR) - fpx[sc][m]};
                    const f2 iy = f2{fpx[s][m], fpx[s][m + 1]} - f2{fpx[su][m], fpx[su][m + 1]};
                    const f2 pxx2 = ix * ix, pyy2 = iy * iy, pxy2 = ix * iy;
                    qxx[m + 1] = pxx2.x, qxx[m + 2] = pxx2.y;
                    qyy[m + 1] = pyy2.x, qyy[m + 2] = pyy2.y;
                    qxy[m + 1] = pxy2.x, qxy[m + 2] = pxy2.y;
                }
#else
#pragma unroll
                for (int m = 0; m < PX; ++m) {
                    const float ix = (m + 1 < PX ? fpx[sc][m + 1] : fR) - (m > 0 ? fpx[sc][m - 1] : fL);
                    const float iy = fpx[s][m] - fpx[su][m];
                    qxx[m + 1] = ix * ix;
                    qyy[m + 1] = iy * iy;
                    qxy[m + 1] = ix * iy;
                }
#endif
                qxx[0] = from_left_f(qxx[PX]);
                qyy[0] = from_left_f(qyy[PX]);
                qxy[0] = from_left_f(qxy[PX]);
                // 3-tap row sums, two columns at a time sharing the middle pair (exact: integers < 2^24)
#pragma unroll
                for (int m = 0; m < PX; m += 2) {
                    const float txx = qxx[m + 1] + qxx[m + 2], tyy = qyy[m + 1] + qyy[m + 2], txy = qxy[m + 1] + qxy[m + 2];
                    hxx[sc][m / 2].x = qxx[m] + txx;
                    hyy[sc][m / 2].x = qyy[m] + tyy;
                    hxy[sc][m / 2].x = qxy[m] + txy;
                    if (m + 3 <= PX) {
                        hxx[sc][m / 2].y = txx + qxx[m + 3];
                        hyy[sc][m / 2].y = tyy + qyy[m + 3];
                        hxy[sc][m / 2].y = txy + qxy[m + 3];
                    } else {  // the right halo column's products
                        hxx[sc][m / 2].y = add_from_right_f(txx, qxx[1]);
                        hyy[sc][m / 2].y = add_from_right_f(tyy, qyy[1]);
                        hxy[sc][m / 2].y = add_from_right_f(txy, qxy[1]);
                    }
                }
#else
                // gradients of row ri-1 (feature_point_harris_detector.cpp:35-62) and biased products at
                // the lane's columns; the halo columns' products come from the neighbour lanes
                const uint32_t Lc = from_left(P_sc[NW - 1]), Rc = from_right(P_sc[0]);
                uint32_t qxx[PX + 2], qyy[PX + 2], qxy[PX + 2];
                uint32_t bsq = kBiasSq, bxy = kBiasXy;
                asm volatile("" : "+s"(bsq), "+s"(bxy));
#pragma unroll
                for (int m = 0; m < PX; ++m) {
                    const int ix = lp_byte<PX>(Lc, P_sc, Rc, m + 1) - lp_byte<PX>(Lc, P_sc, Rc, m - 1);
                    const int iy = lp_byte<PX>(0, P_s, 0, m) - lp_byte<PX>(0, P_su, 0, m);
                    qxx[m + 1] = static_cast<uint32_t>(ix * ix) + bsq;
                    qyy[m + 1] = static_cast<uint32_t>(iy * iy) + bsq;
                    qxy[m + 1] = static_cast<uint32_t>(ix * iy) + bxy;
                }
                qxx[0] = from_left(qxx[PX]);
                qyy[0] = from_left(qyy[PX]);
                qxy[0] = from_left(qxy[PX]);
                qxx[PX + 1] = from_right(qxx[1]);
                qyy[PX + 1] = from_right(qyy[1]);
                qxy[PX + 1] = from_right(qxy[1]);
#pragma unroll
                for (int m = 0; m < PX; ++m) {
                    hxx[sc][m] = add3u(qxx[m], qxx[m + 1], qxx[m + 2]);
                    hyy[sc][m] = add3u(qyy[m], qyy[m + 1], qyy[m + 2]);
                    hxy[sc][m] = add3u(qxy[m], qxy[m + 1], qxy[m + 2]);
                }
#endif

                // response of row rr = ri-2 (Shi-Tomasi: 2r)
                const int rr = ri - 2;
                const bool rowv = rr >= 2 && rr <= rows - 3;
                float r[PX];
#pragma unroll
                for (int m = 0; m < PX; m += 2) {
#if FD_LP_FP
                    const int k = m / 2;
                    f2 sxx, syy, sxy;
                    if constexpr (t % 2 == 0) {
                        pxx[k] = hxx[su][k] + hxx[sc][k];
                        pyy[k] = hyy[su][k] + hyy[sc][k];
                        pxy[k] = hxy[su][k] + hxy[sc][k];
                        sxx = hxx[s][k] + pxx[k];
                        syy = hyy[s][k] + pyy[k];
                        sxy = hxy[s][k] + pxy[k];
                    } else {
                        sxx = pxx[k] + hxx[sc][k];
                        syy = pyy[k] + hyy[sc][k];
                        sxy = pxy[k] + hxy[sc][k];
                    }
                    const f2 v = corner_response_fp<KIND>(sxx, syy, sxy, a.thr);
#else
                    const f2 v = corner_response_lp<KIND>(
                        add3u(hxx[s][m], hxx[su][m], hxx[sc][m]), add3u(hxx[s][m + 1], hxx[su][m + 1], hxx[sc][m + 1]),
                        add3u(hyy[s][m], hyy[su][m], hyy[sc][m]), add3u(hyy[s][m + 1], hyy[su][m + 1], hyy[sc][m + 1]),
                        add3u(hxy[s][m], hxy[su][m], hxy[sc][m]), add3u(hxy[s][m + 1], hxy[su][m + 1], hxy[sc][m + 1]),
                        a.thr);
#endif
                    r[m] = v.x;
                    r[m + 1] = v.y;
                }
                if (!MASKED && rowv && tile_interior) {  // wave-uniform
#pragma unroll
                    for (int m = 0; m < PX; ++m) rsp[su][m] = r[m];
                } else {
                    uint32_t mb = (1u << PX) - 1u;
                    if constexpr (MASKED) mb = rowv ? lp_mask_bits<PX>(a, f, rr, c0) : 0u;
#pragma unroll
                    for (int m = 0; m < PX; ++m) rsp[su][m] = (rowv && cval[m] && ((mb >> m) & 1u)) ? r[m] : 0.0f;
                }

                // NMS of row nr = ri-3 (feature_point_harris_detector.cpp:120-137) + slot emission
                const int nr = ri - 3;
                if (nr >= y0 && nr < y1) {  // wave-uniform
                    // at most PX/2 hits per lane and row (adjacent columns cannot both be strict maxima)
                    if (ballot(A >= sl_addr + 512u * (lp_slots<HIST>() - PX / 2)) != 0ull) {
                        if constexpr (SEG) {  // this workgroup's segment is no longer one sorted run
                            if (lane == 0) {
                                atomicOr(&a.seg_bad[f], 1u);
                                L.seg_ovf = 1u;
                            }
                        }
                        uint32_t n = (A - sl_addr) >> 9;
                        lp_flush<KIND>(n, sl, a, f, lhist);
                        A = sl_addr;
                    }
                    const float lft = from_left_f(rsp[s][PX - 1]);
                    const float rgt = from_right_f(rsp[s][0]);
                    const uint32_t id0 = static_cast<uint32_t>(nr) * static_cast<uint32_t>(cols) + static_cast<uint32_t>(c0);
#pragma unroll
                    for (int m = 0; m < PX; ++m) {
                        const float x = rsp[s][m];
                        const float xl = m == 0 ? lft : rsp[s][m - 1];
                        const float xr = m == PX - 1 ? rgt : rsp[s][m + 1];
                        const float nb = max3f(max3f(xl, xr, thrv), rsp[sc][m], rsp[su][m]);
#if defined(FD_LP_KO) && FD_LP_KO == 1  // diagnostic build only: no emission (the knockout timing)
                        asm volatile("" : : "v"(x), "v"(nb));
#else
                        lp_emit(A, x, nb, id0 + m);
#endif
                    }
                }
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        using I3 = std::integral_constant<int, 3>;
        using I4 = std::integral_constant<int, 4>;
        using I5 = std::integral_constant<int, 5>;
        int i0 = 0;
        for (; i0 + 6 <= n_in; i0 += 6) {
            step(I0{}, i0);
            step(I1{}, i0);
            step(I2{}, i0);
            step(I3{}, i0);
            step(I4{}, i0);
            step(I5{}, i0);
        }
        if (i0 < n_in) {
            step(I0{}, i0);
            if (i0 + 1 < n_in) step(I1{}, i0);
            if (i0 + 2 < n_in) step(I2{}, i0);
            if (i0 + 3 < n_in) step(I3{}, i0);
            if (i0 + 4 < n_in) step(I4{}, i0);
        }
    }
    uint32_t n = (A - sl_addr) >> 9;  // this lane's used slots
    if constexpr (SEG) {
        __shared__ uint32_t seg_wtot[4], seg_base;
        lp_seg_flush<KIND>(n, sl, a, f, active, L, &L.seg_ovf, seg_wtot, seg_base);
    } else {
        if (active) lp_flush<KIND>(n, sl, a, f, lhist);
        if constexpr (HIST) hist_flush(L.hist, a.hist0 + static_cast<int64_t>(f) * kHistBins);
    }
}

}  // namespace

template <int KIND, int PX>
static void launch_corner_lp(const PointsArgs &a, dim3 grid, hipStream_t s) {
    const bool masked = a.mask != nullptr, aligned = a.aligned4 != 0, hist = a.hist0 != nullptr, seg = a.segdesc != nullptr;
#define FD_LP(M, AL, H, SG) hipLaunchKernelGGL((k_corner_lp<KIND, PX, M, AL, H, SG>), grid, dim3(256), 0, s, a)
#define FD_LP_A(M, H, SG)              \
    do {                               \
        if (aligned) FD_LP(M, true, H, SG); \
        else FD_LP(M, false, H, SG);   \
    } while (0)
    if (!hist) FD_LP_A(false, false, false);  // fd_points_response: no mask, no selection histogram
    else if (seg) { if (masked) FD_LP_A(true, true, true); else FD_LP_A(false, true, true); }
    else { if (masked) FD_LP_A(true, true, false); else FD_LP_A(false, true, false); }
#undef FD_LP_A
#undef FD_LP
}

hipError_t launch_corner_lp_any(int kind, const PointsArgs &a, hipStream_t s) {
    const dim3 grid(a.batch * a.blocks_per_frame);
    if (a.mask != nullptr && a.hist0 == nullptr) return hipErrorInvalidValue;
#define FD_LPK(K)                                                   \
    do {                                                            \
        if (a.px == 2) launch_corner_lp<K, 2>(a, grid, s);          \
        else if (a.px == 4) launch_corner_lp<K, 4>(a, grid, s);     \
        else if (a.px == 8) launch_corner_lp<K, 8>(a, grid, s);     \
        else return hipErrorInvalidValue;                           \
    } while (0)
    if (kind == 0) FD_LPK(0);
    else FD_LPK(1);
#undef FD_LPK
    return hipGetLastError();
}

}  // namespace fdk
