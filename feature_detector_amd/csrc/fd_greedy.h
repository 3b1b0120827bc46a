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

// One wave scans a sorted chunk in order (SelectGoodFeatures, feature_point_detector.cpp:62-72), a
// batch of 64 candidates at a time: occupancy-grid test against earlier batches, then the batch is
// resolved at once from cmask (per candidate: earlier candidates of its batch within distance d,
// computed beforehand by the whole workgroup).
// GRID: 0 = no distance test (d <= 0), 1 = occupancy grid in LDS, 2 = grid in global memory.
// Tie check (pk32 != null: the chunk's 32-bit response keys in scan order): FD_FRAME_TIES is raised
// when two adjacent candidates of the visited prefix, or the last visited one and the next, have
// equal responses -- the only case in which the reference's unstable std::sort (:58-60) can change the
// result. tie_prev / tie_has_prev carry the last key of the previous chunk (wave 0's LDS state).
template <int GRID>
__device__ __forceinline__ void greedy_chunk(const SelectArgs &a, int f, int cnt, const uint32_t *pxy,
                                             const uint32_t *pcell, const uint64_t *cmask, uint32_t *grid, int gw2,
                                             uint32_t prior, int &s_acc, int &s_done, bool ties, const uint64_t *tmask,
                                             uint32_t key0, uint32_t keylast,
                                             uint32_t &tie_prev, int &tie_has_prev, uint64_t *st = nullptr) {
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
    auto fetch = [&](int b, uint32_t &e, int &cell, uint64_t &C) {
        // unconditional LDS reads at a clamped index (in the array: cnt <= kSelectChunk), masked after:
        // no exec-masked branch per array
        const int i = b + lane;
        const bool in = i < cnt;
        const int ic = min(i, kSelectChunk - 1);
        e = pxy[ic];
        cell = gw2 + 1;
        C = 0;
        if constexpr (GRID != 0) {
            cell = static_cast<int>(pcell[ic]);
            C = cmask[ic];
        }
        if (!in) {
            e = kEmpty;
            cell = gw2 + 1;
            C = 0;
        }
    };
    uint32_t e_n;
    int cell_n;
    uint64_t C_n;
    int stop = -1;  // position of the append that reached `need` (scan order of pxy)
    fetch(0, e_n, cell_n, C_n);
    for (int b0 = 0; b0 < cnt && !done; b0 += kWave) {
        const uint32_t e = e_n;
        const int cell = cell_n;
        uint64_t C = C_n;
        bool ok = e != kEmpty;
        const int x = static_cast<int>(e & 0xFFFFu), y = static_cast<int>(e >> 16);
        if constexpr (GRID != 0) {
            uint32_t g[9];
#pragma unroll
            for (int q = 0; q < 9; ++q) {
                const int o = cell + (q / 3 - 1) * gw2 + (q % 3 - 1);
                if constexpr (GRID == 1) g[q] = grid[o];
                else g[q] = __hip_atomic_load(&grid[o], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (pk15) {  // packed halves; the empty cell tests far (grid_empty): min over the 9 cells
                const u16x2 base = __builtin_bit_cast(u16x2, e) - static_cast<uint16_t>(d);
                uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
                for (int q = 0; q < 9; ++q) {
                    const u16x2 dt = __builtin_bit_cast(u16x2, g[q]) - base;
                    mn = min(mn, static_cast<uint32_t>(dt.x > dt.y ? dt.x : dt.y));
                }
                ok = ok && mn > w2;
            } else if (pk16) {  // packed halves, as in the conflict masks (select_frame)
                const u16x2 base = __builtin_bit_cast(u16x2, e) - static_cast<uint16_t>(d);
#pragma unroll
                for (int q = 0; q < 9; ++q) {
                    const u16x2 dt = __builtin_bit_cast(u16x2, g[q]) - base;
                    const uint32_t m = dt.x > dt.y ? dt.x : dt.y;
                    if (g[q] != gempty && m <= w2) ok = false;
                }
            } else {
#pragma unroll
                for (int q = 0; q < 9; ++q) {
                    const int gx = static_cast<int>(g[q] & 0xFFFFu), gy = static_cast<int>(g[q] >> 16);
                    if (g[q] != gempty && abs(x - gx) <= d && abs(y - gy) <= d) ok = false;
                }
            }
        }
        if (b0 + kWave < cnt) fetch(b0 + kWave, e_n, cell_n, C_n);
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
            uint64_t dec_m = ~conf;  // decided: unconflicted lanes (accepted if ok) and the not-ok ones
            bool mine = ((conf >> lane) & 1ull) == 0ull;
            for (int pass = 0; dec_m != ~0ull; ++pass) {
                if (pass >= kWave) {  // each pass decides the lowest undecided lane: unreachable
                    if (lane == 0) atomicOr(&a.status[f], 0x20000000u);
                    break;
                }
                const bool can = !mine && (C & ~dec_m) == 0ull;
                const bool take = can && (C & acc_m) == 0ull;
                dec_m |= ballot(can);
                acc_m |= ballot(take);
                mine = mine || can;
            }
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

// Conflict masks of a chunk in scan order: bit j of cmask[p] = candidate (p & ~63) + j, earlier in p's
// batch of 64, lies within Chebyshev distance d. One work item per (candidate, quarter of its batch)
// that holds earlier candidates: 16 entries each, no divergent trip counts; each item writes its 16
// bits of the 64-bit mask. Only those items are enumerated (157 per batch of 64 instead of 4 x 64, the
// rest were idle lanes): quarter 0 for every position me (me = 0 tests nothing) -- that item also
// zeroes the quarters past its own -- and quarter q >= 1 for me > 16q, q-major within the batch.
constexpr int kCmItems = 64 + 47 + 31 + 15;
__device__ __forceinline__ void conflict_masks(const uint32_t *pxy, int c, int d, int rows, int cols, uint64_t *cmask,
                                               int tid, int nthr) {
    uint16_t *cm16 = reinterpret_cast<uint16_t *>(cmask);
    const bool pk16 = rows + 3 * d < 65536 && cols + 3 * d < 65536;
    const uint32_t w2 = 2u * static_cast<uint32_t>(d);
    const int n_items = ((c + kWave - 1) / kWave) * kCmItems;
    for (int item = tid; item < n_items; item += nthr) {
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
        if (p >= c) continue;
        if (q == 0)  // quarters without an item of their own (16q >= me): no earlier candidates there
            for (int qz = max(1, (me + 15) >> 4); qz < 4; ++qz) cm16[4 * p + qz] = 0;
        const uint32_t e = pxy[p];
        uint32_t bits = 0;
        if (e != kEmpty && 16 * q < me) {
            const int x = static_cast<int>(e & 0xFFFFu), y = static_cast<int>(e >> 16);
            const uint4 *q4 = reinterpret_cast<const uint4 *>(pxy + bb + 16 * q);  // broadcast
            const int lim = me - 16 * q;  // entries j < lim of this quarter are earlier
            if (pk16) {
                // packed (x, y) halves: |ex - x| <= d  <=>  (ex - x + d) mod 2^16 <= 2d
                // (no wrap-around: rows, cols + 3d < 2^16). Empty entries need no test:
                // the greedy clears their bits (C &= ballot(ok)).
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
        }
        cm16[4 * p + q] = static_cast<uint16_t>(bits);
    }
}

}  // namespace

}  // namespace fdk
