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
#include "fd_corner_common.h"

namespace fdk {

namespace {

// Per-wave LDS staging of candidates (detect mode). 508, not 512: with the few bytes of workgroup
// flags the corner kernel's LDS is exactly 32 KiB, 5 workgroups per CU (160 KiB); at 512 it was 24
// bytes over and only 4 fit.
constexpr int kStage = FD_STAGE_CORNER;
constexpr int kStageFast = FD_STAGE_FAST;  // FAST: fewer flushes (each drains the wave's stores)
#ifndef FD_FAST_PIPE
#define FD_FAST_PIPE 1  // k_fast: score-table loads consumed one row step after they are issued (0: same step, A/B)
#endif

// Per-wave candidate sink. Detect mode: stage in LDS, append to the frame's list with one atomic per
// flush. Raster mode: write the (row, tile) segment in column order.
struct Sink {
    float *resp;     // LDS staging (detect mode)
    uint32_t *idx;
    uint32_t *hist;  // LDS level-0 histogram of the workgroup's frame, or null
    int n;           // staged entries (wave-uniform)
    uint32_t *ovf;   // LDS flag: a wave of the workgroup flushed before the end (sorted-segment mode)
    uint32_t *ehist = nullptr;  // LDS level-0 histogram counted at emit time instead of at flush (FAST)
    int cap = kStage;           // staging capacity (entries)
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
        if (sk.hist) atomicAdd(&sk.hist[((float_key(r) - a.key_base) << a.key_lz) >> 20], 1u);
        const int64_t pos = static_cast<int64_t>(base) + i;
        if (pos < a.list_cap) {
#if FD_LIST_NT
            __builtin_nontemporal_store(r, &dr[pos]);
            __builtin_nontemporal_store(sk.idx[i], &di[pos]);
#else
            dr[pos] = r;
            di[pos] = sk.idx[i];
#endif
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
        if (sk.n + tot > sk.cap) {
            // (sorted-segment mode: this frame's list is no longer one sorted segment per workgroup)
            if (a.segdesc && lane_id() == 0) {
                atomicOr(&a.seg_bad[f], 1u);
                *sk.ovf = 1u;
            }
            sink_flush(sk, a, f);
        }
        int pos = mbcnt64(b3, mbcnt64(b2, mbcnt64(b1, mbcnt64(b0, sk.n))));
#pragma unroll
        for (int m = 0; m < 4; ++m)
            if (fl[m]) {
                if (sk.ehist) atomicAdd(&sk.ehist[((float_key(v[m]) - a.key_base) << a.key_lz) >> 20], 1u);
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
template <int S>
struct alignas(16) DetectLdsT {  // (16-byte aligned: hist is cleared and read as uint4, fd_corner_common.h)
    float resp[4][S];
    uint32_t idx[4][S];
    uint32_t hist[kHistBins];
};
using DetectLds = DetectLdsT<kStage>;
static_assert(sizeof(DetectLds) % 16 == 0 && offsetof(DetectLds, hist) % 16 == 0, "uint4 histogram access");

// Sorted-segment flush (PointsArgs::segdesc; small launches whose tiles never overflow the staging):
// the workgroup's candidates, all still staged in LDS, go to the frame's list as one contiguous
// segment ordered by level-0 bin, descending (a counting sort on the workgroup's LDS histogram), and
// the segment is described in segdesc[f][g]. k_select then reads only each segment's prefix at or
// above its first-chunk cut (a few entries per workgroup) instead of scanning the whole list.
template <class LdsT>
__device__ __forceinline__ void seg_flush(Sink &sk, const PointsArgs &a, int f, bool active, LdsT &L,
                                          uint32_t (&wtot)[4], uint32_t &wg_base) {
    const int tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
    const int n = active ? sk.n : 0;
    if (lane == 0) wtot[wv] = static_cast<uint32_t>(n);
    __syncthreads();
    if (*sk.ovf) {  // part of the workgroup's list is already out unsorted: plain flush (frame marked)
        if (active) sink_flush(sk, a, f);
        hist_flush(L.hist, a.hist0 + static_cast<int64_t>(f) * kHistBins);
        return;
    }
    // The segment's place in the list: one returning atomic, issued before the histogram work so that
    // its round trip overlaps the counting sort's scan (thread 0 waits for it only at its LDS store).
    uint32_t seg_base_early = 0;
    const uint32_t seg_total = wtot[0] + wtot[1] + wtot[2] + wtot[3];
    if (tid == 0 && seg_total) seg_base_early = atomicAdd(&a.list_count[f], seg_total);
    auto bin_of = [&](float r) { return ((float_key(r) - a.key_base) << a.key_lz) >> 20; };
    if (!sk.ehist)  // (FAST counted its candidates at emit time)
        for (int i = lane; i < n; i += kWave) atomicAdd(&L.hist[bin_of(sk.resp[i])], 1u);
    hist_flush(L.hist, a.hist0 + static_cast<int64_t>(f) * kHistBins);  // (leads with a barrier)
    __syncthreads();
    // in place: hist[b] = entries of bins above b (exclusive scan in descending bin order)
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
        wg_base = seg_base_early;
        const int g = logical_block() % a.blocks_per_frame;
        a.segdesc[static_cast<int64_t>(f) * a.blocks_per_frame + g] = make_uint2(wg_base, total);
    }
    __syncthreads();
    float *dr = a.list_resp + static_cast<int64_t>(f) * a.list_cap;
    uint32_t *di = a.list_idx + static_cast<int64_t>(f) * a.list_cap;
    const int64_t base = wg_base;
    const int g = logical_block() % a.blocks_per_frame;
    uint64_t *head = a.seghead + (static_cast<int64_t>(f) * a.blocks_per_frame + g) * kSegHead;
    for (int i = lane; i < n; i += kWave) {
        const float r = sk.resp[i];
        const uint32_t k32 = (float_key(r) - a.key_base) << a.key_lz;
        const uint32_t lp = atomicAdd(&L.hist[k32 >> 20], 1u);
        const int64_t pos = base + lp;
        if (pos < a.list_cap) {
#if FD_LIST_NT
            __builtin_nontemporal_store(r, &dr[pos]);
            __builtin_nontemporal_store(sk.idx[i], &di[pos]);
#else
            dr[pos] = r;
            di[pos] = sk.idx[i];
#endif
        }
        // the segment's head as selection keys (k32, ~idx): k_select's first read, no list hop
        if (lp < static_cast<uint32_t>(kSegHead)) head[lp] = (static_cast<uint64_t>(k32) << 32) | static_cast<uint64_t>(~sk.idx[i]);
    }
    sk.n = 0;
}

template <int KIND, bool RASTER, bool MASKED, bool ALIGNED, bool G1>
__device__ __forceinline__ void corner_tile(const PointsArgs &a, int f, int ty, int tx, Sink &sk);

// ---------------------------------------------------------------------------------------------------
// K1: corner response + NMS. One wave per tile of kTileW columns x tile_h rows; lane l covers columns
// c0 = tx*kTileW + 4(l-1) .. c0+3 and walks the rows keeping 3-row sliding windows in registers:
// pixels (+ DPP halo dwords), horizontal tensor sums, responses.
// ---------------------------------------------------------------------------------------------------
#ifdef FD_K1_CLOCKS  // diagnostic build only (tools/k1_wg_clock.py): per-workgroup s_memrealtime phase clocks
}  // namespace
__device__ unsigned long long g_fdk_k1_clocks[4096];
namespace {
#define FD_K1_CLOCK(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime()
#else
#define FD_K1_CLOCK(v)
#endif
template <int KIND, bool RASTER, bool MASKED, bool ALIGNED, bool G1>
__global__ __launch_bounds__(256) void k_corner(PointsArgs a) {
    FD_K1_CLOCK(t_entry);
    __shared__ DetectLds lds_all[1];
    int f, ty, tx;
    const bool active = decode_tile(a, f, ty, tx);
    __shared__ uint32_t seg_ovf;
    Sink sk{nullptr, nullptr, nullptr, 0, &seg_ovf};
    if constexpr (!RASTER) {
        const int wv = threadIdx.x >> 6;
        sk = Sink{lds_all[0].resp[wv], lds_all[0].idx[wv], a.hist0 ? lds_all[0].hist : nullptr, 0, &seg_ovf};
        if (threadIdx.x == 0) seg_ovf = 0;
        if (a.hist0) hist_clear(lds_all[0].hist);
        else __syncthreads();
    }
    FD_K1_CLOCK(t_clr);
    if (active) corner_tile<KIND, RASTER, MASKED, ALIGNED, G1>(a, f, ty, tx, sk);
    FD_K1_CLOCK(t_tile);
    if constexpr (!RASTER) {
        if (a.segdesc) {
            __shared__ uint32_t seg_wtot[4], seg_base;
            seg_flush(sk, a, f, active, lds_all[0], seg_wtot, seg_base);
#ifdef FD_K1_CLOCKS
            __syncthreads();
            FD_K1_CLOCK(t_end);
            if (threadIdx.x == 0 && blockIdx.x < 1024) {
                unsigned long long *c = g_fdk_k1_clocks + 4 * blockIdx.x;
                c[0] = t_entry;
                c[1] = t_clr;
                c[2] = t_tile;
                c[3] = t_end;
            }
#endif
        } else {
            if (active) sink_flush(sk, a, f);
            if (a.hist0) hist_flush(lds_all[0].hist, a.hist0 + static_cast<int64_t>(f) * kHistBins);
        }
    }
}

template <int KIND, bool RASTER, bool MASKED, bool ALIGNED, bool G1>
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
            if (i0 + t >= n_in) break;  // (uniform) short tiles: no steps past the tile's last NMS row
            const int s = t % 3, su = (t + 1) % 3, sc = (t + 2) % 3;  // 3-slot roles: rows ri, ri-2, ri-1
            const int ri = y0 - 3 + i0 + t;                            // row consumed this step
            ring[(t + 3) % 6] = load_px4<ALIGNED>(rs, (ri + 3) * cols + c0);
            const uint32_t P_s = ring[t], P_su = ring[(t + 4) % 6], P_sc = ring[(t + 5) % 6];
            // Pipeline fill: step i0+t computes the gradients of row y0-4+(i0+t) (needed from row y0-2:
            // steps >= 2) and the responses of row y0-5+(i0+t) (needed from row y0-1: steps >= 4). The
            // first steps only load (wave-uniform; compile-time true for i0 > 0 or the later t).
            // Short tiles (batch 1: 3 output rows in 9 steps) drop 2 of 9 gradient and 4 of 9 response
            // evaluations. Skipped slots keep their zero initialisation and are never read.
            if (!(t >= 2 || i0 > 0)) continue;

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

            if (!(t >= 4 || i0 > 0)) continue;
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
            const f2 r01 = corner_response2<KIND, G1>(sxx[0], sxx[1], syy[0], syy[1], sxy[0], sxy[1], a.thr);
            const f2 r23 = corner_response2<KIND, G1>(sxx[2], sxx[3], syy[2], syy[3], sxy[2], sxy[3], a.thr);
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
// K3: FAST-12
// ---------------------------------------------------------------------------------------------------
// Byte-parallel (SWAR) comparisons: a lane's dword holds 4 consecutive pixels of one row, and every
// ring sample of those 4 pixels is one dword too (the row's dword shifted by dx bytes), so one compare
// sequence classifies 4 pixels. Only bit 7 of each byte of a result is meaningful.
constexpr uint32_t kH = 0x80808080u;  // top bit of every byte
constexpr uint32_t kL = 0x7F7F7F7Fu;  // low 7 bits of every byte
constexpr uint32_t kOnes = 0x01010101u;

// Per byte: x > y, from the low-7-bit difference (no borrow leaves a byte: the minuend carries the top
// bit, the subtrahend is at most 0x80) and the top bits. yk = (y & kL) + kOnes, precomputed per pixel.
// The final select (x7 != y7 ? x7 : z7) is one v_bitop3_b32.
__device__ __forceinline__ uint32_t swar_gt(uint32_t x, uint32_t y, uint32_t yk) {
    const uint32_t z = (x | kH) - yk;
    return (x & ~y) | (~(x ^ y) & z);
}
// Per byte: min(p + 15, 255) (bright threshold; v > 255 never holds, like v > p + 15 for p > 240).
__device__ __forceinline__ uint32_t swar_adds15(uint32_t p) {
    const uint32_t t = (p & kL) + 0x0F0F0F0Fu;      // low 7 bits + 15: bit 7 = carry
    const uint32_t ov = p & t & kH;                  // p >= 128 and carry: the sum exceeds 255
    const uint32_t ovm = (ov - (ov >> 7)) | ov;      // 0xFF where ov
    return t | (p & kH) | ovm;
}
// Per byte: max(p - 15, 0) (dark threshold; v < 0 never holds, like v < p - 15 for p < 15).
__device__ __forceinline__ uint32_t swar_subs15(uint32_t p) {
    const uint32_t d = (p | kH) - 0x0F0F0F0Fu;       // 0x80 + (p & 0x7F) - 15 >= 0x71: no borrow
    const uint32_t un = ~p & ~d & kH;                // p < 128 and the difference below 128: p < 15
    const uint32_t unm = (un - (un >> 7)) | un;
    return (d ^ (~p & kH)) & ~unm;
}
// The 4 pixels' samples at column offset dx of a row held as [L | P | R] (compile-time dx).
template <int DX>
__device__ __forceinline__ uint32_t shifted(uint32_t L, uint32_t P, uint32_t R) {
    if constexpr (DX == 0) return P;
    else if constexpr (DX > 0) return __builtin_amdgcn_alignbyte(R, P, DX);
    else return __builtin_amdgcn_alignbyte(P, L, 4 + DX);
}

// FAST running offset o_k (feature_point_fast_detector.cpp:85,93) from the segment table: inside a
// segment o_k = o_s + (k - k_s) * inc exactly (build_offsets checks it), and one fma rounds that exact
// value once, so the float result is the reference's sum. Per-lane segment search (binary, LDS).
__device__ __forceinline__ float fast_offset(int nseg, const int32_t *ks, const float *os, const float *inc, int32_t k) {
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {  // last segment with k_start <= k
        const int mid = (lo + hi + 1) >> 1;
        if (ks[mid] <= k) lo = mid; else hi = mid - 1;
    }
    return __builtin_fmaf(static_cast<float>(k - ks[lo]), inc[lo], os[lo]);
}

template <bool RASTER, bool MASKED, bool ALIGNED>
__device__ __forceinline__ void fast_tile(const PointsArgs &a, const FastOffsets &off, const int32_t *seg_k,
                                          const float *seg_o, const float *seg_inc, int f, int ty, int tx, Sink &sk,
                                          float cut, uint32_t &skip);

template <bool RASTER, bool MASKED, bool ALIGNED>
__global__ __launch_bounds__(256) void k_fast(PointsArgs a, FastOffsets off) {
    __shared__ DetectLdsT<kStageFast> lds_all[1];
    __shared__ int32_t seg_k[kMaxOffsetSegs];
    __shared__ float seg_o[kMaxOffsetSegs], seg_inc[kMaxOffsetSegs];
    __shared__ uint32_t seg_ovf;
    __shared__ uint32_t seg_wtot[4], seg_base;
    int f, ty, tx;
    const bool active = decode_tile(a, f, ty, tx);
    if (a.emit_cut_next && blockIdx.x == 0 && threadIdx.x == 0) *a.emit_cut_next = 0x7F800000u;  // +inf
    const float cut = a.emit_cut ? __uint_as_float(*a.emit_cut) : -__builtin_inff();
    for (int i = threadIdx.x; i < off.nseg; i += blockDim.x) {
        seg_k[i] = static_cast<int32_t>(off.k_start[i]);  // frames < 2^31 px (checked on the host)
        seg_o[i] = static_cast<float>(off.o_start[i]);     // exact: a float of the sequence
        seg_inc[i] = static_cast<float>(off.inc[i]);       // exact: a difference of two nearby floats
    }
    // one frame's tile: staging, the row walk, the flush (every thread of the workgroup)
    auto run = [&](int fr) {
        uint32_t skip = 0;  // (wave-uniform) candidates below the cut
        Sink sk{nullptr, nullptr, nullptr, 0, &seg_ovf};
        if constexpr (!RASTER) {
            const int wv = threadIdx.x >> 6;
            sk = Sink{lds_all[0].resp[wv], lds_all[0].idx[wv], a.hist0 ? lds_all[0].hist : nullptr, 0, &seg_ovf};
            sk.ehist = sk.hist;  // FAST: histogram counted at emit time (measured faster than at flush)
            sk.hist = nullptr;
            sk.cap = kStageFast;
            if (threadIdx.x == 0) seg_ovf = 0;
            if (a.hist0) hist_clear(lds_all[0].hist);  // (includes the barrier for the segment table)
            else __syncthreads();
        } else {
            __syncthreads();
        }
        if (active) fast_tile<RASTER, MASKED, ALIGNED>(a, off, seg_k, seg_o, seg_inc, fr, ty, tx, sk, cut, skip);
        if (a.skipped && skip && lane_id() == 0) atomicAdd(&a.skipped[fr], skip);
        if constexpr (!RASTER) {
            if (a.segdesc) {
                seg_flush(sk, a, fr, active, lds_all[0], seg_wtot, seg_base);
            } else {
                if (active) sink_flush(sk, a, fr);
                if (a.hist0) hist_flush(lds_all[0].hist, a.hist0 + static_cast<int64_t>(fr) * kHistBins);
            }
        }
    };
    if (a.redo_status) {
        // Redo pass (kFrameRedo), launched with one frame's workgroups: this workgroup's tile of every
        // flagged frame, one frame after another (the flags of 64 frames per load and ballot; usually none)
        for (int base = 0; base < a.batch; base += kWave) {
            const int fr = base + lane_id();
            uint64_t m = ballot(fr < a.batch && (a.redo_status[min(fr, a.batch - 1)] & kFrameRedo));
            while (m) {  // (uniform)
                const int j = __builtin_ctzll(m);
                m &= m - 1ull;
                __syncthreads();  // (the previous frame's flush has read the staging)
                run(base + j);
            }
        }
        return;
    }
    run(f);
}

// K3: FAST-12 (feature_point_fast_detector.cpp:11-98). Same tile walk as K1 with a 7-row register
// window (ring radius 3). Per row step a lane classifies its 4 pixels at once:
//  * thresholds min(p+15, 255) / max(p-15, 0) per byte; the cardinal pre-check (:20-42: samples 4, 8,
//    12 all brighter or all darker) as 6 byte-parallel compares;
//  * only if a lane of the wave passes: the other 13 samples, each bright/dark bit inserted into
//    per-pixel 8-bit halves of the ring masks (bit k = sample k);
//  * the score, the longest circular run of either mask (the reference's two-pass count, :55-78), from
//    a 64 Ki-entry table indexed by the 16-bit mask (L2/L1-resident), for passing pixels only;
//  * response = score + o_k (:88) with o_k from the segment table (one fma).
template <bool RASTER, bool MASKED, bool ALIGNED>
__device__ __forceinline__ void fast_tile(const PointsArgs &a, const FastOffsets &off, const int32_t *seg_k,
                                          const float *seg_o, const float *seg_inc, int f, int ty, int tx, Sink &sk,
                                          float cut, uint32_t &skip) {
    const int lane = lane_id();
    const int rows = a.rows, cols = a.cols;
    const int c0 = tx * kTileW + 4 * (lane - 1);
    const int y0 = 3 + ty * a.tile_h;
    const int y1 = min(y0 + a.tile_h, rows - 3);  // output rows [y0, y1) within [3, rows-4]
    const auto rs = make_rsrc(a.frames + static_cast<int64_t>(f) * rows * cols, static_cast<uint32_t>(rows * cols));
    const auto lut = make_rsrc(off.run_lut, 65536u);

    bool colv[4];
    uint32_t colmask = 0;  // bit 7 of byte m: column c0+m inside [3, cols-4], owned by an interior lane
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        colv[m] = lane >= 1 && lane <= 62 && c0 + m >= 3 && c0 + m <= cols - 4;
        colmask |= colv[m] ? (0x80u << (8 * m)) : 0u;
    }
    // the tile's scan-index range per row (unmasked k = (row-3)(cols-6) + col-3) and its offset segment
    const int cmin = max(tx * kTileW, 3), cmax = min(tx * kTileW + kTileW - 1, cols - 4);
    int sg = 0;  // wave-uniform, advances with the rows

    uint32_t P[7], L[7], R[7];
#pragma unroll
    for (int s = 0; s < 7; ++s) P[s] = L[s] = R[s] = 0;

    // Scan index k of each pixel among mask-true pixels (the offset counter of :85-93), the response
    // score + o_k (:88), the candidate test (:89) and the emission, for output row `orow` whose scores
    // are known.
    auto finish_row = [&](int orow, uint32_t live, const int (&score)[4]) {
        float resp[4];
        bool fl[4];
        if constexpr (MASKED) {
            int32_t kbase = 0;
            uint32_t mword = 0;
            const int64_t rb = static_cast<int64_t>(f) * rows + orow;
            kbase = a.row_base[rb];
            if (c0 >= 0 && c0 < cols) {
                const int w = c0 >> 5;
                kbase += a.word_pref[rb * a.mask_wpr + w];
                mword = a.mask[rb * a.mask_wpr + w];
                if (w == 0) mword &= ~7u;
            }
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const bool lv = (live >> (8 * m + 7)) & 1u;
                const int32_t k = kbase + __popc(mword & ((1u << ((c0 + m) & 31)) - 1u));  // earlier pixels in the word
                resp[m] = 0.0f;
                if (lv && (score[m] > 0 || k >= off.k0))
                    resp[m] = static_cast<float>(score[m]) + fast_offset(off.nseg, seg_k, seg_o, seg_inc, k);
                fl[m] = lv && resp[m] > a.thr;
            }
        } else {
            const int32_t krow = (orow - 3) * (cols - 6) - 3;  // k = krow + column
            const int32_t kmin = krow + cmin, kmax = krow + cmax;
            while (sg + 1 < off.nseg && seg_k[sg + 1] <= kmin) ++sg;  // (uniform; rows only move forward)
            if (sg + 1 >= off.nseg || seg_k[sg + 1] > kmax) {     // the whole row step in one segment
                const float os = seg_o[sg], inc = seg_inc[sg];
                const int32_t kr = krow + c0 - seg_k[sg];
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    resp[m] = static_cast<float>(score[m]) + __builtin_fmaf(static_cast<float>(kr + m), inc, os);
                    fl[m] = colv[m] && resp[m] > a.thr;
                }
            } else {
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    resp[m] = 0.0f;
                    if (colv[m]) resp[m] = static_cast<float>(score[m]) +
                                           fast_offset(off.nseg, seg_k, seg_o, seg_inc, krow + c0 + m);
                    fl[m] = colv[m] && resp[m] > a.thr;
                }
            }
        }
        if constexpr (!RASTER) {
            // emission cut (PointsArgs::emit_cut): candidates below it are counted, not emitted
            bool em[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                em[m] = fl[m] && resp[m] >= cut;
                skip += static_cast<uint32_t>(popc64(ballot(fl[m] && !em[m])));
                fl[m] = em[m];
            }
        }
        const uint64_t b[4] = {ballot(fl[0]), ballot(fl[1]), ballot(fl[2]), ballot(fl[3])};
        emit_row<RASTER, kSegFast>(sk, a, f, tx, orow, c0, b, fl, resp);
        if constexpr (RASTER) {
            if (a.resp_map != nullptr) {
                float *mrow = a.resp_map + (static_cast<int64_t>(f) * rows + orow) * cols;
#pragma unroll
                for (int m = 0; m < 4; ++m)
                    if (fl[m]) mrow[c0 + m] = resp[m];
            }
        }
    };
#if FD_FAST_PIPE
    // Software pipeline over the rows: a row's score-table loads (L1/L2 hits, several hundred cycles) are
    // issued in the step that classifies it and consumed in the next step, after that step's own row
    // load and table loads are in flight -- not waited for at once in the step that issued them.
    bool pend = false;  // (wave-uniform) a classified row waits for its scores
    int p_orow = 0;
    uint32_t p_live = 0, p_pass = 0;
    uint32_t p_sb[4] = {0u, 0u, 0u, 0u}, p_sd[4] = {0u, 0u, 0u, 0u};
    auto finish_pending = [&]() {
        int score[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) score[m] = ((p_pass >> (8 * m + 7)) & 1u) ? static_cast<int>(max(p_sb[m], p_sd[m])) : 0;
        finish_row(p_orow, p_live, score);
    };
#endif

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
#define ROW(dy) L[(s + 4 + (dy)) % 7], P[(s + 4 + (dy)) % 7], R[(s + 4 + (dy)) % 7]
            const uint32_t p = P[(s + 4) % 7];
            const uint32_t tb = swar_adds15(p), td = swar_subs15(p);
            const uint32_t tbk = (tb & kL) + kOnes;         // bright: v > tb
            const uint32_t tdk = (td | kH) - kOnes;          // dark: td > v, i.e. v < td
            auto bright = [&](uint32_t v) { return swar_gt(v, tb, tbk); };
            auto dark = [&](uint32_t v) {
                const uint32_t z = tdk - (v & kL);
                return (td & ~v) | (~(td ^ v) & z);
            };
            uint32_t live = colmask;
            if constexpr (MASKED) {
                const uint32_t mb = mask_bits4(a, f, orow, c0);
                live &= ((mb & 1u) ? 0x80u : 0u) | ((mb & 2u) ? 0x8000u : 0u) | ((mb & 4u) ? 0x800000u : 0u) |
                        ((mb & 8u) ? 0x80000000u : 0u);
            }
            // Cardinal pre-check (:20-42): samples 4 (dx 3), 8 (dy 3), 12 (dx -3) all bright or all dark.
            const uint32_t v4 = shifted<3>(ROW(0)), v8 = P[(s + 7) % 7], v12 = shifted<-3>(ROW(0));
            const uint32_t b4 = bright(v4), b8 = bright(v8), b12 = bright(v12);
            const uint32_t d4 = dark(v4), d8 = dark(v8), d12 = dark(v12);
            const uint32_t pass = ((b4 & b8 & b12) | (d4 & d8 & d12)) & live;
            uint32_t sb[4] = {0u, 0u, 0u, 0u}, sd[4] = {0u, 0u, 0u, 0u};  // score-table entries (bright, dark)
            if (ballot(pass != 0u) != 0ull) {  // wave-uniform
                // ring masks, 8 samples per half: acc = bfi(kH, g, acc >> 1) inserts sample k at bit 7;
                // after 8 insertions sample k of the half sits at bit k - 8*half of each byte.
                uint32_t blo, bhi, dlo, dhi;
                auto put = [](uint32_t &acc, uint32_t g) { acc = (g & kH) | ((acc >> 1) & kL); };
                // kFastIndice (:7-8): k -> (dx, dy)
                const uint32_t v0 = shifted<0>(ROW(-3)), v1 = shifted<1>(ROW(-3)), v2 = shifted<2>(ROW(-2));
                const uint32_t v3 = shifted<3>(ROW(-1)), v5 = shifted<3>(ROW(1)), v6 = shifted<2>(ROW(2));
                const uint32_t v7 = shifted<1>(ROW(3));
                blo = bright(v0); dlo = dark(v0);
                put(blo, bright(v1)); put(dlo, dark(v1));
                put(blo, bright(v2)); put(dlo, dark(v2));
                put(blo, bright(v3)); put(dlo, dark(v3));
                put(blo, b4); put(dlo, d4);
                put(blo, bright(v5)); put(dlo, dark(v5));
                put(blo, bright(v6)); put(dlo, dark(v6));
                put(blo, bright(v7)); put(dlo, dark(v7));
                const uint32_t v9 = shifted<-1>(ROW(3)), v10 = shifted<-2>(ROW(2)), v11 = shifted<-3>(ROW(1));
                const uint32_t v13 = shifted<-3>(ROW(-1)), v14 = shifted<-2>(ROW(-2)), v15 = shifted<-1>(ROW(-3));
                bhi = b8; dhi = d8;
                put(bhi, bright(v9)); put(dhi, dark(v9));
                put(bhi, bright(v10)); put(dhi, dark(v10));
                put(bhi, bright(v11)); put(dhi, dark(v11));
                put(bhi, b12); put(dhi, d12);
                put(bhi, bright(v13)); put(dhi, dark(v13));
                put(bhi, bright(v14)); put(dhi, dark(v14));
                put(bhi, bright(v15)); put(dhi, dark(v15));
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    if ((pass >> (8 * m + 7)) & 1u) {
                        const uint32_t sel = 0x0C0C0000u | (static_cast<uint32_t>(4 + m) << 8) | static_cast<uint32_t>(m);
                        const uint32_t ib = __builtin_amdgcn_perm(bhi, blo, sel);  // bits 0-7 | 8-15
                        const uint32_t id = __builtin_amdgcn_perm(dhi, dlo, sel);
                        sb[m] = buf_load_u8(lut, static_cast<int32_t>(ib));
                        sd[m] = buf_load_u8(lut, static_cast<int32_t>(id));
                    }
                }
            }
#undef ROW
#if FD_FAST_PIPE
            if (pend) finish_pending();  // the previous row, its table loads issued one step ago
            pend = true;
            p_orow = orow;
            p_live = live;
            p_pass = pass;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                p_sb[m] = sb[m];
                p_sd[m] = sd[m];
            }
#else
            int score[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) score[m] = ((pass >> (8 * m + 7)) & 1u) ? static_cast<int>(max(sb[m], sd[m])) : 0;
            finish_row(orow, live, score);
#endif
        }
    }
#if FD_FAST_PIPE
    if (pend) finish_pending();
#endif
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
    if (!raster && a.px != 0) return launch_corner_lp_any(kind, a, s);  // (fd_corner_lp.hip; thr >= 0 only)
    const bool masked = a.mask != nullptr, aligned = a.aligned4 != 0;
    const bool g1 = !raster && a.thr >= 0.0f;  // single-gate stores (see corner_response2)
#define FD_CORNER_A(K, RS, M, G)                                                                \
    do {                                                                                        \
        if (aligned) hipLaunchKernelGGL((k_corner<K, RS, M, true, G>), grid, block, 0, s, a);  \
        else hipLaunchKernelGGL((k_corner<K, RS, M, false, G>), grid, block, 0, s, a);         \
    } while (0)
#define FD_CORNER(K, RS, M)                                      \
    do {                                                         \
        if (RS) FD_CORNER_A(K, RS, M, false);                    \
        else if (g1) FD_CORNER_A(K, false, M, true);             \
        else FD_CORNER_A(K, false, M, false);                    \
    } while (0)
    if (kind == 0) {
        if (raster) { if (masked) FD_CORNER(0, true, true); else FD_CORNER(0, true, false); }
        else { if (masked) FD_CORNER(0, false, true); else FD_CORNER(0, false, false); }
    } else {
        if (raster) { if (masked) FD_CORNER(1, true, true); else FD_CORNER(1, true, false); }
        else { if (masked) FD_CORNER(1, false, true); else FD_CORNER(1, false, false); }
    }
#undef FD_CORNER
#undef FD_CORNER_A
    return hipGetLastError();
}

hipError_t launch_fast(bool raster, const PointsArgs &a, const FastOffsets &off, hipStream_t s) {
    // (the redo pass: one frame's workgroups, each looping over the flagged frames)
    const dim3 grid(a.redo_status ? a.blocks_per_frame : blocks_for_waves(a)), block(256);
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

hipError_t launch_compact(const CompactArgs &a, int batch, hipStream_t s) {
    hipLaunchKernelGGL(k_compact, dim3(batch), dim3(1024), 0, s, a);
    return hipGetLastError();
}

}  // namespace fdk

#ifdef FD_K1_CLOCKS
extern "C" int fd_debug_k1_clocks(unsigned long long *out, int n) {
    return static_cast<int>(hipMemcpyFromSymbol(out, HIP_SYMBOL(fdk::g_fdk_k1_clocks), sizeof(unsigned long long) * n, 0,
                                                hipMemcpyDeviceToHost));
}
#endif
