// Greedy min-distance scan shared by the selection kernels (fd_select.hip: k_select,
// k_select_ordered; fd_select_ref.hip: k_select_reference): SelectGoodFeatures'
// (feature_point_detector.cpp:62-72) in-order walk over a chunk of candidates, one wave per chunk in
// batches of 64, against an occupancy grid of (d+1)-sized cells, with the batch's conflict masks
// computed beforehand by the whole workgroup.
#pragma once

#include "fd_device.h"
#include "fd_hip.h"
#include "fd_kernels.h"

namespace fdk {

namespace {

constexpr uint32_t kEmpty = 0xFFFFFFFFu;
// Empty occupancy-grid cell. Frames with rows, cols + 3d < 2^15 use 0x7FFF7FFF: in the packed-halves
// distance test (dt = g - (e - d) per 16-bit half, conflict iff both halves <= 2d) it lies more than d
// from every pixel without wrapping (0x7FFF - x + d is in (2d, 2^16) for x < cols), so the greedy's grid
// test needs no empty check; larger frames use 0xFFFFFFFF (coordinates stay below 65535) and check.
__device__ __forceinline__ bool grid_pk15(int rows, int cols, int d) { return rows + 3 * d < 32768 && cols + 3 * d < 32768; }
__device__ __forceinline__ uint32_t grid_empty(int rows, int cols, int d) { return grid_pk15(rows, cols, d) ? 0x7FFF7FFFu : kEmpty; }
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));  // packed (x, y) of a (y << 16) | x position

#ifndef FD_SEQ_CONFLICTS
#define FD_SEQ_CONFLICTS 0
#endif
// greedy batch: ordered scalar pass up to this many conflicted lanes, else the fixed point. Sweep at the
// headline (profiles/r03_select_rejected.txt): 0 (always the fixed point) 19.3-19.5 us, 2: 19.6-20.0,
// 4: 19.5-19.7, 12: 20.1-20.2 -- the fixed point's passes (the longest conflict chain, ~2-3) cost less
// than one ordered step per conflicted lane.
constexpr int kSeqConflicts = FD_SEQ_CONFLICTS;

// A batch's conflicted lanes (conf) decided by a fixed point on wave-uniform masks: each pass decides
// every undecided lane whose earlier ok neighbours (C, already restricted to ok lanes) are all decided
// -- accepted iff none of them was. Passes = the longest conflict chain; each decides at least the
// lowest undecided lane. acc_m holds the unconflicted ok lanes on entry.
__device__ __forceinline__ uint64_t resolve_batch(const SelectArgs &a, int f, uint64_t C, uint64_t conf,
                                                  uint64_t acc_m) {
    uint64_t dec_m = ~conf;  // decided: unconflicted lanes (accepted if ok) and the not-ok ones
    for (int pass = 0; dec_m != ~0ull; ++pass) {
        if (pass >= kWave) {  // unreachable
            if (lane_id() == 0) atomicOr(&a.status[f], 0x20000000u);
            break;
        }
        const uint64_t can_m = ballot((C & ~dec_m) == 0ull) & ~dec_m;
        const uint64_t free_m = ballot((C & acc_m) == 0ull);
        dec_m |= can_m;
        acc_m |= can_m & free_m;
    }
    return acc_m;
}

// One wave scans a sorted chunk in order (SelectGoodFeatures, feature_point_detector.cpp:62-72), a
// batch of 64 candidates at a time: occupancy-grid test against earlier batches, then the batch is
// resolved at once from cmask (per candidate: earlier candidates of its batch within distance d,
// computed beforehand by the whole workgroup).
// GRID: 0 = no distance test (d <= 0), 1 = occupancy grid in LDS, 2 = grid in global memory.
// Tie check (pk32 != null: the chunk's 32-bit response keys in scan order): FD_FRAME_TIES is raised
// when two adjacent candidates of the visited prefix, or the last visited one and the next, have
// equal responses -- the only case in which the reference's unstable std::sort (:58-60) can change the
// result. tie_prev / tie_has_prev carry the last key of the previous chunk (wave 0's LDS state).
//
// XM (cross masks, xmask[p]: bit j = candidate (p & ~63) - 64 + j of the previous batch lies within d):
// the grid test runs one batch ahead. Batch b+1's nine cells are read before batch b's grid writes (LDS
// operations of a wave complete in order), so it sees batches <= b-1; batch b's accepted candidates are
// excluded by xmask & (b's accepted lanes) once they are known. The grid reads' latency then overlaps
// a batch's resolution instead of starting the next one.
template <int GRID, bool XM = false>
__device__ __forceinline__ void greedy_chunk(const SelectArgs &a, int f, int cnt, const uint32_t *pxy,
                                             const uint32_t *pcell, const uint64_t *cmask, uint32_t *grid, int gw2,
                                             uint32_t prior, int &s_acc, int &s_done, bool ties, const uint64_t *tmask,
                                             uint32_t key0, uint32_t keylast,
                                             uint32_t &tie_prev, int &tie_has_prev, uint64_t *st = nullptr,
                                             const uint64_t *xmask = nullptr) {
    static_assert(!XM || GRID != 0, "cross masks need a grid");
    const int lane = lane_id();
    // diagnostic clocks (a.stamps): per-batch phases into slots 26-28 (st[15]: the running clock)
    auto gst = [&](int slot) {
        if (st && lane == 0) {
            const uint64_t now = __builtin_readcyclecounter();
            st[slot] += now - st[15];
            st[15] = now;
        }
    };
    const int d = a.dist;
    const bool pk16 = a.rows + 3 * d < 65536 && a.cols + 3 * d < 65536;  // no wrap-around in 16-bit halves
    const bool pk15 = grid_pk15(a.rows, a.cols, d);
    const uint32_t gempty = grid_empty(a.rows, a.cols, d);
    const uint32_t w2 = 2u * static_cast<uint32_t>(d);
    int acc = s_acc;
    bool done = false;
    uint32_t t_prev = tie_prev;
    bool t_has = tie_has_prev != 0;
    bool tied = false;
    // Software pipeline: a batch's position, cell and conflict mask are loaded during the previous
    // batch's resolution (they are read-only here; only the grid is written).
    auto fetch = [&](int b, uint32_t &e, int &cell, uint64_t &C, uint64_t &X) {
        // unconditional LDS reads at a clamped index (in the array: cnt <= kSelectChunk), masked after:
        // no exec-masked branch per array
        const int i = b + lane;
        const bool in = i < cnt;
        const int ic = min(i, kSelectChunk - 1);
        e = pxy[ic];
        cell = gw2 + 1;
        C = 0;
        X = 0;
        if constexpr (GRID != 0) {
            cell = static_cast<int>(pcell[ic]);
            C = cmask[ic];
        }
        if constexpr (XM) X = xmask[ic];
        if (!in) {
            e = kEmpty;
            cell = gw2 + 1;
            C = 0;
            X = 0;
        }
    };
    auto gload = [&](int cell, uint32_t (&g)[9]) {
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            const int o = cell + (q / 3 - 1) * gw2 + (q % 3 - 1);
            if constexpr (GRID == 1) g[q] = grid[o];
            else g[q] = __hip_atomic_load(&grid[o], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    // no grid entry within distance d of e (e != kEmpty)
    auto gfree = [&](uint32_t e, const uint32_t (&g)[9]) {
        bool ok = true;
        if (pk15) {  // packed halves; the empty cell tests far (grid_empty): min over the 9 cells
            const u16x2 base = __builtin_bit_cast(u16x2, e) - static_cast<uint16_t>(d);
            uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
            for (int q = 0; q < 9; ++q) {
                const u16x2 dt = __builtin_bit_cast(u16x2, g[q]) - base;
                mn = min(mn, static_cast<uint32_t>(dt.x > dt.y ? dt.x : dt.y));
            }
            ok = mn > w2;
        } else if (pk16) {  // packed halves, as in the conflict masks (select_frame)
            const u16x2 base = __builtin_bit_cast(u16x2, e) - static_cast<uint16_t>(d);
#pragma unroll
            for (int q = 0; q < 9; ++q) {
                const u16x2 dt = __builtin_bit_cast(u16x2, g[q]) - base;
                const uint32_t m = dt.x > dt.y ? dt.x : dt.y;
                if (g[q] != gempty && m <= w2) ok = false;
            }
        } else {
            const int x = static_cast<int>(e & 0xFFFFu), y = static_cast<int>(e >> 16);
#pragma unroll
            for (int q = 0; q < 9; ++q) {
                const int gx = static_cast<int>(g[q] & 0xFFFFu), gy = static_cast<int>(g[q] >> 16);
                if (g[q] != gempty && abs(x - gx) <= d && abs(y - gy) <= d) ok = false;
            }
        }
        return ok;
    };
    uint32_t e_n;
    int cell_n;
    uint64_t C_n, X_n;
    int stop = -1;  // position of the append that reached `need` (scan order of pxy)
    uint64_t acc_prev = 0;  // XM: the previous batch's accepted lanes
    bool gok_n = true;      // XM: the next batch's grid test
    uint32_t g_n[9];        // XM: the batch after next's grid cells (in flight)
    fetch(0, e_n, cell_n, C_n, X_n);
    if constexpr (XM) {
        uint32_t g0[9];
        gload(cell_n, g0);
        gok_n = gfree(e_n, g0);
    }
    for (int b0 = 0; b0 < cnt && !done; b0 += kWave) {
        const uint32_t e = e_n;
        const int cell = cell_n;
        uint64_t C = C_n;
        bool ok = e != kEmpty;
        const int x = static_cast<int>(e & 0xFFFFu), y = static_cast<int>(e >> 16);
        if constexpr (XM) {
            ok = ok && gok_n && (X_n & acc_prev) == 0ull;
            if (b0 + kWave < cnt) {  // the next batch: its grid cells before this batch's writes
                fetch(b0 + kWave, e_n, cell_n, C_n, X_n);
                gload(cell_n, g_n);
            }
        } else {
            if constexpr (GRID != 0) {
                uint32_t g[9];
                gload(cell, g);
                ok = ok && gfree(e, g);
            }
            if (b0 + kWave < cnt) fetch(b0 + kWave, e_n, cell_n, C_n, X_n);
        }
        const uint64_t m = ballot(ok);
        gst(26);  // grid test
        C &= m;
        // Resolution in scan order: a lane with no earlier ok neighbour in the batch is accepted; the
        // conflicted ones are decided by a fixed point, where each pass decides every lane whose earlier
        // neighbours are all decided (passes = the longest chain) -- accepted iff none of them was. (With
        // FD_SEQ_CONFLICTS > 0, up to that many conflicted lanes are instead decided one by one in
        // ascending order on the scalar unit: slower at every threshold measured, see kSeqConflicts.)
        const uint64_t conf = ballot(C != 0ull) & m;
        uint64_t acc_m = m & ~conf;
        if (popc64(conf) <= kSeqConflicts) {
            for (uint64_t rest = conf; rest; rest &= rest - 1ull) {
                const int i = __builtin_ctzll(rest);
                const uint64_t free_m = ballot((C & acc_m) == 0ull);
                acc_m |= free_m & (1ull << i);
            }
        } else {
            acc_m = resolve_batch(a, f, C, conf, acc_m);
        }
        gst(27);  // resolution
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
            stop = b0 + 63 - __builtin_clzll(acc_m);
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
        if constexpr (XM) {
            acc_prev = acc_m;
            if (b0 + kWave < cnt) gok_n = e_n != kEmpty && gfree(e_n, g_n);
        }
        gst(28);  // output + grid update
    }
    if (ties && cnt > 0) {
        // The reference's visiting order of this sub-chunk ends at the stop (or runs through it). Its
        // prefix holds a tie if any of its tie bits is set (bit i: position i equals i - 1), if its
        // first key equals the previous sub-chunk's last, or if the candidate after the stop equals the
        // stop (unknown past the sub-chunk: assumed). (Keys the prefilter dropped are always rejected
        // and cannot matter, see select_frame.)
        const int last = done ? stop : cnt - 1;
        bool t = false;
        for (int w = opaque(lane); w * kWave <= last; w += kWave) {
            uint64_t word = tmask[w];
            if (w * kWave + kWave - 1 > last) word &= (2ull << (last & (kWave - 1))) - 1ull;
            t = t || word != 0ull;
        }
        tied = ballot(t) != 0ull;
        if (t_has && key0 == t_prev) tied = true;
        if (done) {
            const int nx = last + 1;
            if (nx >= cnt || ((tmask[nx >> 6] >> (nx & (kWave - 1))) & 1ull)) tied = true;
        }
        t_prev = keylast;  // the chunk's last key, for the next chunk's first comparison
        t_has = true;
    }
    if (lane == 0) {
        s_acc = acc;
        if (done) s_done = 1;
        tie_prev = t_prev;
        tie_has_prev = t_has ? 1 : 0;
        if (tied) atomicOr(&a.status[f], FD_FRAME_TIES);
    }
}

// Near-bits of 16 candidates q16[0..15] (16-aligned LDS, broadcast reads) around position e: bit j set
// iff entry j lies within Chebyshev distance d (and j < lim). pk16: packed (x, y) halves,
// |ex - x| <= d  <=>  (ex - x + d) mod 2^16 <= 2d (no wrap-around: rows, cols + 3d < 2^16); empty
// entries then need no test (the greedy clears their bits: C &= ballot(ok), and an empty candidate is
// never accepted, so its cross bit never meets an accepted lane).
__device__ __forceinline__ uint32_t near16(uint32_t e, const uint32_t *q16, int lim, int d, bool pk16, uint32_t w2) {
    const uint4 *q4 = reinterpret_cast<const uint4 *>(q16);
    uint32_t bits = 0;
    if (pk16) {
        const u16x2 base = __builtin_bit_cast(u16x2, e) - static_cast<uint16_t>(d);
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
            const uint4 e4 = q4[j4];
            const uint32_t ev[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const u16x2 dt = __builtin_bit_cast(u16x2, ev[t]) - base;
                const uint32_t m = dt.x > dt.y ? dt.x : dt.y;
                bits |= (m <= w2 ? 1u : 0u) << (j4 * 4 + t);
            }
        }
        if (lim < 16) bits &= (1u << lim) - 1u;
    } else {
        const int x = static_cast<int>(e & 0xFFFFu), y = static_cast<int>(e >> 16);
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
            const uint4 e4 = q4[j4];
            const uint32_t ev[4] = {e4.x, e4.y, e4.z, e4.w};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int ex = static_cast<int>(ev[t] & 0xFFFFu), ey = static_cast<int>(ev[t] >> 16);
                const bool nb = j4 * 4 + t < lim && ev[t] != kEmpty && abs(x - ex) <= d && abs(y - ey) <= d;
                bits |= static_cast<uint32_t>(nb) << (j4 * 4 + t);
            }
        }
    }
    return bits;
}

// Conflict masks of a chunk in scan order: bit j of cmask[p] = candidate (p & ~63) + j, earlier in p's
// batch of 64, lies within Chebyshev distance d. One work item per (candidate, quarter of its batch)
// that holds earlier candidates: 16 entries each, no divergent trip counts; each item writes its 16
// bits of the 64-bit mask. Only those items are enumerated (157 per batch of 64 instead of 4 x 64, the
// rest were idle lanes): quarter 0 for every position me (me = 0 tests nothing) -- that item also
// zeroes the quarters past its own -- and quarter q >= 1 for me > 16q, q-major within the batch.
// xmask (optional, greedy_chunk's XM): bit j of xmask[p] = candidate (p & ~63) - 64 + j (the previous
// batch) within distance d; 4 x 64 more items per batch (zero for the first batch).
constexpr int kCmItems = 64 + 47 + 31 + 15;
__device__ __forceinline__ void conflict_masks(const uint32_t *pxy, int c, int d, int rows, int cols, uint64_t *cmask,
                                               int tid, int nthr, uint64_t *xmask = nullptr) {
    uint16_t *cm16 = reinterpret_cast<uint16_t *>(cmask);
    uint16_t *xm16 = reinterpret_cast<uint16_t *>(xmask);
    const bool pk16 = rows + 3 * d < 65536 && cols + 3 * d < 65536;
    const uint32_t w2 = 2u * static_cast<uint32_t>(d);
    const int per = xmask ? kCmItems + 4 * kWave : kCmItems;
    const int n_items = ((c + kWave - 1) / kWave) * per;
    for (int item = tid; item < n_items; item += nthr) {
        const int bi = item / per, t = item - bi * per;
        const int bb = bi * kWave;
        if (t >= kCmItems) {  // cross item: quarter q of the previous batch
            const int me = (t - kCmItems) & (kWave - 1), q = (t - kCmItems) >> 6;
            const int p = bb + me;
            if (p >= c) continue;
            const uint32_t e = pxy[p];
            uint32_t bits = 0;
            if (bi > 0 && e != kEmpty) bits = near16(e, pxy + bb - kWave + 16 * q, 16, d, pk16, w2);
            xm16[4 * p + q] = static_cast<uint16_t>(bits);
            continue;
        }
        int q, me;
        if (t < 64) {
            q = 0;
            me = t;
        } else if (t < 64 + 47) {
            q = 1;
            me = t - 64 + 17;
        } else if (t < 64 + 47 + 31) {
            q = 2;
            me = t - (64 + 47) + 33;
        } else {
            q = 3;
            me = t - (64 + 47 + 31) + 49;
        }
        const int p = bb + me;
        if (p >= c) continue;
        if (q == 0)  // quarters without an item of their own (16q >= me): no earlier candidates there
            for (int qz = max(1, (me + 15) >> 4); qz < 4; ++qz) cm16[4 * p + qz] = 0;
        const uint32_t e = pxy[p];
        uint32_t bits = 0;
        if (e != kEmpty && 16 * q < me) bits = near16(e, pxy + bb + 16 * q, me - 16 * q, d, pk16, w2);
        cm16[4 * p + q] = static_cast<uint16_t>(bits);
    }
}

// ---- k_select's pipelined scan (sorted chunks, occupancy grid in LDS, coordinates with grid_pk15) ----
//
// The greedy is one wave's chain of dependent instructions (a lone wave issues a dependent VALU op
// about every 8 core clocks: tools/calib/icache_probe.hip), so everything that need not be on it is
// moved off it: the conflict masks of batch b are computed by the other waves while wave 0 scans
// (their work items in batch order; ScanLds::cnt[b] counts the finished items of batch b), and the
// outputs and the tie check are done after the scan by the whole workgroup from the accepted lanes of
// each batch (ScanLds::accm / accb). tools/calib/greedy_probe.hip times the scan alone.
constexpr int kScanBatches = kSelectChunk / kWave;
struct ScanLds {  // (placed in the unused tail of the LDS occupancy grid)
    uint64_t accm[kScanBatches];  // accepted lanes of each scanned batch
    uint32_t accb[kScanBatches];  // features accepted before the batch (this frame)
    uint32_t cnt[kScanBatches];   // finished conflict-mask items of batch b (kCmItems: ready)
    int nbp, stop, done, pad;  // batches scanned; scan position of the stop; stopped at `need`
};
constexpr int kScanLdsWords = static_cast<int>(sizeof(ScanLds) / 4);

// Conflict masks (as conflict_masks) by waves 1.. of the workgroup (hw = wave - 1 of nh), items in
// batch order so that the first batches are ready first; each wave adds its finished items per batch
// to sl.cnt after its mask writes.
__device__ __forceinline__ void scan_masks(const uint32_t *pxy, int c, int d, int rows, int cols, uint64_t *cmask,
                                           ScanLds &sl, int hw, int nh) {
    const int lane = lane_id();
    uint16_t *cm16 = reinterpret_cast<uint16_t *>(cmask);
    const bool pk16 = rows + 3 * d < 65536 && cols + 3 * d < 65536;
    const uint32_t w2 = 2u * static_cast<uint32_t>(d);
    const int nb = (c + kWave - 1) / kWave;
    const int total = nb * kCmItems;
    for (int base = hw * kWave; base < total; base += nh * kWave) {
        const int item = base + lane;
        if (item < total) {
            const int bi = item / kCmItems, t = item - bi * kCmItems;
            int q, me;
            if (t < 64) {
                q = 0;
                me = t;
            } else if (t < 64 + 47) {
                q = 1;
                me = t - 64 + 17;
            } else if (t < 64 + 47 + 31) {
                q = 2;
                me = t - (64 + 47) + 33;
            } else {
                q = 3;
                me = t - (64 + 47 + 31) + 49;
            }
            const int bb = bi * kWave, p = bb + me;
            if (p < c) {
                if (q == 0)
                    for (int qz = max(1, (me + 15) >> 4); qz < 4; ++qz) cm16[4 * p + qz] = 0;
                const uint32_t e = pxy[p];
                uint32_t bits = 0;
                if (e != kEmpty && 16 * q < me) bits = near16(e, pxy + bb + 16 * q, me - 16 * q, d, pk16, w2);
                cm16[4 * p + q] = static_cast<uint16_t>(bits);
            } else if (q == 0) {
                cmask[p] = 0ull;  // (the last batch past c)
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) {
            const int hi = min(base + kWave, total);
            for (int b = base / kCmItems; b * kCmItems < hi; ++b)
                atomicAdd(&sl.cnt[b], static_cast<uint32_t>(min(hi, (b + 1) * kCmItems) - max(base, b * kCmItems)));
        }
    }
}

// Wave 0's scan of a sorted chunk (SelectGoodFeatures, feature_point_detector.cpp:62-72), greedy_chunk<1>'s
// semantics: per batch, the occupancy-grid test, the in-batch resolution from the conflict masks, the
// need cutoff (:67-69) and the grid update; the accepted lanes go to sl.accm. Waits for each batch's
// masks (sl.cnt[b] == kCmItems). Outputs: s_acc, s_done, sl.nbp / stop / done.
__device__ __forceinline__ void greedy_scan(const SelectArgs &a, int f, int cnt, const uint32_t *pxy,
                                            const uint32_t *pcell, const uint64_t *cmask, uint32_t *grid, int gw2,
                                            uint32_t prior, int &s_acc, int &s_done, ScanLds &sl,
                                            uint64_t *st = nullptr) {
    const int lane = lane_id();
    // diagnostic clocks (a.stamps): slot 26 the first batch, slot 27 the others (st[15]: the running clock)
    auto gst = [&](int slot) {
        if (st && lane == 0) {
            const uint64_t now = __builtin_readcyclecounter();
            st[slot] += now - st[15];
            st[15] = now;
        }
    };
    const int d = a.dist;
    const uint32_t w2 = 2u * static_cast<uint32_t>(d);
    const u16x2 dd = {static_cast<uint16_t>(d), static_cast<uint16_t>(d)};
    uint32_t acc = static_cast<uint32_t>(s_acc);
    const int nb = (cnt + kWave - 1) / kWave;
    bool done = false;
    int stop = -1, b = 0;
    // positions and cells are final before the scan starts: prefetched one batch ahead (entries past
    // cnt are replaced when used: an empty position in a valid cell); the masks once their batch is done
    uint32_t e_n = pxy[lane], cell_n = pcell[lane];
    uint32_t rdy_n = __hip_atomic_load(&sl.cnt[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (; b < nb && !done; ++b) {
        const bool in = b * kWave + lane < cnt;
        const uint32_t e = in ? e_n : kEmpty;
        const uint32_t cell = in ? cell_n : static_cast<uint32_t>(gw2 + 1);
        uint32_t rdy = rdy_n;
        for (int spin = 0; rdy != static_cast<uint32_t>(kCmItems); ++spin) {  // (the mask waves reach every batch)
            if (spin > (1 << 20)) {  // consistency guard instead of a hang
                if (lane == 0) atomicOr(&a.status[f], 0x20000000u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            rdy = __hip_atomic_load(&sl.cnt[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        uint32_t g[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) g[q] = grid[cell + (q / 3 - 1) * gw2 + (q % 3 - 1)];
        uint64_t C = cmask[b * kWave + lane];
        if (b + 1 < nb) {
            const int i = min((b + 1) * kWave + lane, kSelectChunk - 1);
            e_n = pxy[i];
            cell_n = pcell[i];
            rdy_n = __hip_atomic_load(&sl.cnt[b + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        // packed halves; the empty cell tests far (grid_empty): min over the 9 cells
        const u16x2 base = __builtin_bit_cast(u16x2, e) - dd;
        uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            const u16x2 dt = __builtin_bit_cast(u16x2, g[q]) - base;
            mn = min(mn, static_cast<uint32_t>(dt.x > dt.y ? dt.x : dt.y));
        }
        const uint64_t m = ballot(e != kEmpty && mn > w2);
        C &= m;
        const uint64_t conf = ballot(C != 0ull) & m;
        uint64_t acc_m = m & ~conf;
        if (conf) acc_m = resolve_batch(a, f, C, conf, acc_m);
        // need cutoff (:67-69): features.size() >= need is checked after every append
        const uint32_t have = prior + acc;
        const int allow = have < a.need ? static_cast<int>(a.need - have) : 1;
        if (popc64(acc_m) >= allow) {
            uint64_t keep = 0, t = acc_m;
            for (int k = 0; k < allow; ++k) {
                keep |= t & (~t + 1ull);
                t &= t - 1ull;
            }
            acc_m = keep;
            done = true;
            stop = b * kWave + 63 - __builtin_clzll(acc_m);
        }
        if ((acc_m >> lane) & 1ull) grid[cell] = e;
        if (lane == 0) {
            sl.accm[b] = acc_m;
            sl.accb[b] = acc;
        }
        acc += static_cast<uint32_t>(popc64(acc_m));
        gst(b == 0 ? 26 : 27);
    }
    if (lane == 0) {
        s_acc = static_cast<int>(acc);
        if (done) s_done = 1;
        sl.nbp = b;
        sl.stop = stop;
        sl.done = done ? 1 : 0;
    }
}

// After the scan (all threads, past a barrier): the accepted candidates' outputs in scan order, and
// greedy_chunk's tie check on the visited prefix from the 32-bit keys in scan order (pk32): equal
// adjacent keys in it, the chunk's first key equal to the previous sub-chunk's last, or (stopped) the
// candidate after the stop equal to it (unknown past the sub-chunk: assumed).
__device__ __forceinline__ void scan_outputs(const SelectArgs &a, int f, int cnt, const uint32_t *pxy,
                                             const ScanLds &sl, bool ties, const uint32_t *pk32, uint32_t &tie_prev,
                                             int &tie_has_prev, int tid, int nthr) {
    const int lane = lane_id();
    const int np = sl.nbp * kWave;
    for (int p = tid; p < np; p += nthr) {
        const uint64_t m = sl.accm[p >> 6];
        if ((m >> (p & 63)) & 1ull) {
            const int pos = static_cast<int>(sl.accb[p >> 6]) + popc64(m & ((1ull << (p & 63)) - 1ull));
            if (pos < a.out_stride) {
                const uint32_t e = pxy[p];
                float2 *o = reinterpret_cast<float2 *>(a.out_xy) + static_cast<int64_t>(f) * a.out_stride + pos;
                *o = make_float2(static_cast<float>(e & 0xFFFFu), static_cast<float>(e >> 16));
            }
        }
    }
    if (!ties || cnt <= 0) return;
    const bool done = sl.done != 0;
    const int last = done ? sl.stop : cnt - 1;
    bool t = false;
    for (int i = tid; i <= last; i += nthr)
        if (i > 0 && pk32[i] == pk32[i - 1]) t = true;
    if (tid == 0) {
        if (tie_has_prev && pk32[0] == tie_prev) t = true;
        if (done && (last + 1 >= cnt || pk32[last + 1] == pk32[last])) t = true;
    }
    if (ballot(t) != 0ull && lane == 0) atomicOr(&a.status[f], FD_FRAME_TIES);
    if (tid == 0) {  // (tie_prev was read above by this thread only)
        tie_prev = pk32[cnt - 1];
        tie_has_prev = 1;
    }
}

}  // namespace

}  // namespace fdk
