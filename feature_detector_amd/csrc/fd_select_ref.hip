// K4d k_select_reference: the reference tie order (FD_TIES_REFERENCE) on the GPU, graph-capturable.
//
// SelectGoodFeatures sorts its raster-ordered candidates with an unstable std::sort
// (feature_point_detector.cpp:58-60); among equal responses the visiting order is whatever libstdc++'s
// introsort leaves. k_select visits equal responses by raster index and flags every frame whose scanned
// prefix meets a tie (FD_FRAME_TIES); this kernel re-selects exactly those frames in libstdc++'s order.
//
// libstdc++ (GCC 11, bits/stl_algo.h) std::sort = __introsort_loop(first, last, 2 * __lg(n)) then
// __final_insertion_sort. The loop partitions a range of more than 16 elements around the median of
// (first + 1, mid, last - 1) moved to `first` (__move_median_to_first), by __unguarded_partition over
// [first + 1, last): a left scan stops at elements e with !(e > pivot) ("left stoppers", LS: resp <=
// pivot), a right scan at !(pivot > e) ("right stoppers", RS: resp >= pivot), and the k-th left stopper
// from the left swaps with the k-th right stopper from the right while l_k < r_k. With K such swaps the
// cut is min(l_{K+1}, r_K) (the left scan's last stop: the next original left stopper, or at the latest
// r_K, which now holds a left stopper). Both halves recurse with depth - 1; the loop leaves ranges of <=
// 16 elements, which the final insertion sort orders stably and never crosses (every element right of a
// cut is <= every element left of it). So the final order of any prefix follows from partitions of the
// ranges that overlap it alone: ranks of the stoppers come from prefix counts (ballots), the pairing is
// a scatter of stopper positions by rank, and K per range is where l_k < r_k stops holding (monotone).
//
// One 1024-thread workgroup per flagged frame:
//   1. the frame's candidates in push order: raster order for the built-in detectors (a bitmap of the
//      candidate pixels and its word prefix ranks the unordered list), the list order as given for
//      caller lists (fd_points_select);
//   2. windows of kSelectChunk positions from the front: every range overlapping the window is
//      partitioned, level by level, all of a level's ranges at once (flat index space over their
//      partition spans, one block of it per wave), until only leaves (<= 16) cover the window; leaves
//      are insertion-sorted by 16 lanes each into the visiting order; before the first greedy scan,
//      children of <= kRefWaveLocal elements leave the levels and are sorted to the end by one wave
//      each in LDS (ref_wave_resolve), which saves the last levels' barriers;
//   3. the greedy scan of k_select_ordered over the new positions (one wave, occupancy grid); stop at
//      `need`, else the next window (ranges right of the window wait in the range list).
// A range that reaches the depth limit takes libstdc++'s fallback, std::__partial_sort(first, last, last)
// = __make_heap + __sort_heap, emulated exactly by one wave (ref_heapsort: the heap built level by level,
// the subtrees of one level being disjoint, then the pops by one lane), in LDS when the range fits there;
// its visiting order is then final. FD_FRAME_UNRESOLVED is left only for a broken internal invariant
// (range guards), in which case the frame keeps k_select's raster-order features (the host resolves it
// when it synchronises).
#include "fd_greedy.h"

#include <algorithm>
#include <type_traits>

namespace fdk {

namespace {

constexpr int kRefThreads = 1024;
constexpr int kRefWaves = kRefThreads / kWave;
constexpr int kRefMaxRanges = 256;  // unresolved ranges (> 16) in the list; bound: DESIGN.md
constexpr int kRefLeaf = 16;        // libstdc++ _S_threshold
#ifndef FD_REF_U
#define FD_REF_U 4
#endif
constexpr int kRefU = FD_REF_U;     // 64-element rounds per wave whose global loads are issued together
constexpr uint32_t kRefRidCap = 8192;  // flat elements per level whose range index pass 1 caches for passes 2-3
// A range of <= kRefWaveLocal elements is partitioned to the end (its whole subtree) by one wave in LDS,
// with no workgroup barriers, in 12 B per element of the 96 KiB greedy span per wave (elements + stopper
// positions). A/B on the bench tie frames (tools/gpu_r04f.sh): off / 64 / 128 / 256 / 512 = headline
// 52.3 / 51.3 / 50.1 / 48.4 / 52.5 us per call, north star 1.48 / 1.54 / 1.53 / 1.52 / 1.53 ms.
#ifndef FD_REF_WL
#define FD_REF_WL 256
#endif
constexpr uint32_t kRefWaveLocal = FD_REF_WL;  // (0: off)
constexpr int kRefStack = 64;  // pending subranges per wave (depth-first: <= 2 per level)
constexpr uint32_t kNoPos = 0xFFFFFFFFu;

struct alignas(16) RefLds {
    // greedy (k_select_ordered's layout)
    uint32_t pxy[kSelectChunk];
    uint32_t pcell[kSelectChunk];
    uint64_t cmask[kSelectChunk];
    uint32_t grid_lds[kGridLdsCells];
    // sorted list of the unresolved ranges [lo, hi) (> 16 elements), double-buffered, with depth left
    uint32_t r_lo[2][kRefMaxRanges];
    uint32_t r_hi[2][kRefMaxRanges];
    uint32_t r_dep[2][kRefMaxRanges];
    // the level's active ranges (the list's prefix overlapping the window) j < m_act
    uint32_t o[kRefMaxRanges + 1];  // flat offset of range j's partition span [lo + 1, hi)
    float piv[kRefMaxRanges];
    uint32_t headL[kRefMaxRanges], headR[kRefMaxRanges], headW[kRefMaxRanges];
    uint32_t bL[kRefMaxRanges], nL[kRefMaxRanges], eR[kRefMaxRanges], nR[kRefMaxRanges];
    uint32_t cut[kRefMaxRanges];
    uint32_t waveL[kRefWaves], waveR[kRefWaves];
    // leaves produced by the level
    uint32_t leaf_lo[2 * kRefMaxRanges], leaf_hi[2 * kRefMaxRanges];
    // ranges of <= kRefWaveLocal elements handed to single waves (first window only), and the waves' stacks
    uint32_t wl_lo[kRefMaxRanges], wl_hi[kRefMaxRanges], wl_dep[kRefMaxRanges];
    uint32_t wl_ord[kRefMaxRanges];  // the list by size, largest first
    int wl_next;                     // next entry of wl_ord for a free wave
    uint32_t wstk[kRefWaves][kRefStack];
    uint32_t wsum[kRefWaves];
    uint16_t rid[kRefRidCap];  // levels with T <= kRefRidCap: each element's active range (set by pass 1)
    int cur, m_all, m_act, n_leaf, fail, n_wl, n_heap, n_hq;
    uint32_t heap_j[kRefMaxRanges];      // active ranges at depth 0 (heapsort fallback)
    uint32_t hq[2 * kRefMaxRanges];      // wave-local subranges at depth 0: absolute [lo, hi), heapsorted after the phase
    uint32_t T, fin;
    int s_done, s_acc;
    uint32_t tie_prev;
    int tie_has_prev;
};

__device__ __forceinline__ float as_f(uint32_t u) { return __uint_as_float(u); }

// Range guard of every data-dependent index (the emulation's invariants keep them in range; a broken
// invariant clamps the access, marks the frame failed and, with RefSortArgs::dbg, records the first
// violation: code, index, bound, level).
#define FD_REF_IDX(idx, bound, code) ref_idx((idx), (bound), (code), L, r, f)
__device__ __forceinline__ uint32_t ref_idx(uint32_t idx, uint32_t bound, uint32_t code, struct RefLds &L,
                                            const RefSortArgs &r, int f);

// libstdc++ __move_median_to_first(result = lo, a = lo + 1, b = mid, c = hi - 1) with comp = resp
// greater: the position whose element becomes the pivot (swapped into lo).
__device__ __forceinline__ uint32_t median_pos(float ra, float rb, float rc, uint32_t a, uint32_t b, uint32_t c) {
    if (ra > rb) {
        if (rb > rc) return b;
        if (ra > rc) return c;
        return a;
    }
    if (ra > rc) return a;
    if (rb > rc) return c;
    return b;
}

__device__ __forceinline__ uint32_t ref_idx(uint32_t idx, uint32_t bound, uint32_t code, RefLds &L,
                                            const RefSortArgs &r, int f) {
    if (idx < bound) return idx;
    L.fail = 4;
    if (r.dbg && atomicCAS(&r.dbg[static_cast<int64_t>(f) * 8], 0u, code) == 0u) {
        r.dbg[static_cast<int64_t>(f) * 8 + 1] = idx;
        r.dbg[static_cast<int64_t>(f) * 8 + 2] = bound;
        r.dbg[static_cast<int64_t>(f) * 8 + 3] = static_cast<uint32_t>(L.m_act);
        r.dbg[static_cast<int64_t>(f) * 8 + 4] = L.T;
    }
    return bound ? bound - 1u : 0u;
}

// Exclusive prefix of v over the workgroup; total in *tot. Two barriers.
__device__ __forceinline__ uint32_t block_excl(uint32_t v, uint32_t *wsum, uint32_t &tot) {
    const int lane = lane_id(), w = threadIdx.x / kWave;
    const uint32_t incl = wave_incl_add(v);
    if (lane == kWave - 1) wsum[w] = incl;
    __syncthreads();
    const uint32_t ws = lane < kRefWaves ? wsum[lane] : 0u;
    const uint32_t wincl = wave_incl_add(ws);
    const uint32_t wbase = static_cast<uint32_t>(__shfl(static_cast<int>(wincl - ws), w));
    tot = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wincl), kRefWaves - 1));
    __syncthreads();
    return wbase + incl - v;
}

// Index of the active range holding flat element e (o[j] <= e < o[j+1]), from a wave-uniform start j0
// at most 5 ranges back (every span has >= 16 elements, a round of 64 lanes meets <= 5 of them).
__device__ __forceinline__ int range_of(const uint32_t *o, int m, int j0, uint32_t e) {
    int j = j0;
    while (j + 1 < m && o[j + 1] <= e) ++j;
    return j;
}

// First active range whose span holds flat element e (binary search, wave-uniform e).
__device__ __forceinline__ int range_search(const uint32_t *o, int m, uint32_t e) {
    int lo = 0, hi = m - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (o[mid] <= e) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// Wave 0: the active prefix of the current list for window [fin, win_end) and the flat offsets of
// the active ranges' partition spans.
__device__ __forceinline__ void set_active(RefLds &L, uint32_t win_end) {
    const int lane = lane_id();
    const int c = L.cur, m = L.m_all;
    uint32_t carry = 0;
    int act = 0;
    for (int b = 0; b < m; b += kWave) {
        const int j = b + lane;
        const bool in = j < m && L.r_lo[c][j] < win_end;
        const uint64_t bal = ballot(in);
        const uint32_t span = in ? L.r_hi[c][j] - L.r_lo[c][j] - 1u : 0u;
        const uint32_t incl = wave_incl_add(span);
        if (in) L.o[j] = carry + incl - span;
        carry += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), kWave - 1));
        act += popc64(bal);
        if (bal != ~0ull) break;  // sorted list: the first range past the window ends the prefix
    }
    if (lane == 0) {
        L.m_act = act;
        L.o[act] = carry;
        L.T = carry;
    }
}

// Position of the k-th set bit (0-based) of m; m must hold more than k bits.
__device__ __forceinline__ uint32_t select_bit(uint64_t m, uint32_t k) {
    uint32_t pos = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1) {
        const uint32_t c = static_cast<uint32_t>(__popcll(m & ((1ull << step) - 1ull)));
        if (k >= c) {
            k -= c;
            m >>= step;
            pos += static_cast<uint32_t>(step);
        }
    }
    return pos;
}

// ---- std::__partial_sort(first, last, last): the introsort's depth-limit fallback ---------------------
// bits/stl_heap.h with comp = response greater (feature_point_detector.cpp:58-60): __adjust_heap sifts the
// hole down to a leaf along the child that comp does not order first, then __push_heap moves the value up
// while comp(parent, value). f is LDS or global memory (generic pointer).
__device__ __forceinline__ bool ref_gt(uint2 a, uint2 b) { return __uint_as_float(a.x) > __uint_as_float(b.x); }

__device__ void ref_adjust_heap(uint2 *f, int hole, int len, uint2 v) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (ref_gt(f[second], f[second - 1])) --second;
        f[hole] = f[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        f[hole] = f[second - 1];
        hole = second - 1;
    }
    while (hole > top) {  // __push_heap(f, hole, top, v)
        const int parent = (hole - 1) / 2;
        const uint2 pv = f[parent];
        if (!ref_gt(pv, v)) break;
        f[hole] = pv;
        hole = parent;
    }
    f[hole] = v;
}

// One wave: __make_heap then __sort_heap on f[0, len). __make_heap adjusts parents (len - 2) / 2 down to 0;
// the parents of one tree level own disjoint subtrees and the deeper levels come first, so the lanes
// adjust a level's parents at once. __sort_heap's pops depend on each other: lane 0.
__device__ __forceinline__ void ref_heapsort(uint2 *f, int len) {
    if (len < 2) return;
    const int lane = lane_id();
    const int last_parent = (len - 2) / 2;
    for (int k = 31 - __clz(last_parent + 1); k >= 0; --k) {
        const int lo = (1 << k) - 1, hi = min((1 << (k + 1)) - 2, last_parent);
        for (int p = lo + lane; p <= hi; p += kWave) ref_adjust_heap(f, p, len, f[p]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0)
        for (int l = len - 1; l >= 1; --l) {
            const uint2 v = f[l];
            f[l] = f[0];
            ref_adjust_heap(f, 0, l, v);
        }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave, one element per lane: libstdc++'s introsort on a range of 17..64 elements (E[0, len), in
// LDS) to the end, every subrange of a level partitioned at once. Lane p keeps its subrange [sa, sb);
// stopper ranks are popcounts of the subrange's ballot, the k-th stopper's position a bit select, the
// exchanges and the pivot move shuffles. Leaves: stable rank by response, descending, into ordp.
// A subrange at the depth limit (std::__partial_sort) is written back to X (xp: X at E[0]'s position) and
// queued in hq (absolute [lo, hi) pairs, count *hn) for the heapsort step; its lanes take no further part.
__device__ bool ref_wave_small(uint2 *E, uint32_t len, uint32_t dep, uint32_t *ordp, uint2 *xp, uint32_t xlo,
                               uint32_t *hq, int *hn) {
    const uint32_t p = static_cast<uint32_t>(lane_id());
    uint2 v = p < len ? E[p] : make_uint2(0u, 0u);
    uint32_t sa = 0, sb = len, dp = dep;
    bool queued = false;
    for (int it = 0; it < 64; ++it) {
        bool big = p < len && !queued && sb - sa > static_cast<uint32_t>(kRefLeaf);
        if (ballot(big) == 0ull) break;
        if (ballot(big && dp == 0u) != 0ull) {
            const bool hp = big && dp == 0u;
            if (hp) xp[p] = v;
            if (hp && p == sa) {
                const int q = atomicAdd(hn, 1);
                if (q < kRefMaxRanges) {
                    hq[2 * q] = xlo + sa;
                    hq[2 * q + 1] = xlo + sb;
                }
            }
            queued = queued || hp;
            big = big && !hp;
            if (ballot(big) == 0ull) break;
        }
        // pivot: __move_median_to_first(sa, sa + 1, mid, sb - 1)
        const uint32_t mid = sa + (sb - sa) / 2u;
        const uint32_t i1 = min(sa + 1u, 63u), i2 = min(mid, 63u), i3 = sb >= 1u ? min(sb - 1u, 63u) : 0u;
        const float ra = __uint_as_float(static_cast<uint32_t>(__shfl(static_cast<int>(v.x), static_cast<int>(i1))));
        const float rb = __uint_as_float(static_cast<uint32_t>(__shfl(static_cast<int>(v.x), static_cast<int>(i2))));
        const float rc = __uint_as_float(static_cast<uint32_t>(__shfl(static_cast<int>(v.x), static_cast<int>(i3))));
        const uint32_t ch = median_pos(ra, rb, rc, sa + 1u, mid, sb - 1u);
        uint32_t src = p;
        if (big) src = p == sa ? ch : (p == ch ? sa : p);
        v.x = static_cast<uint32_t>(__shfl(static_cast<int>(v.x), static_cast<int>(min(src, 63u))));
        v.y = static_cast<uint32_t>(__shfl(static_cast<int>(v.y), static_cast<int>(min(src, 63u))));
        const float pv = __uint_as_float(static_cast<uint32_t>(__shfl(static_cast<int>(v.x), static_cast<int>(min(sa, 63u)))));
        // stoppers of (sa, sb)
        const bool in = big && p > sa && p < sb;
        const float rv = __uint_as_float(v.x);
        const uint64_t BL = ballot(in && rv <= pv), BR = ballot(in && rv >= pv);
        const uint64_t hiMask = sb >= 64u ? ~0ull : ((1ull << sb) - 1ull);
        const uint64_t seg = hiMask & ~((2ull << min(sa, 62u)) - 1ull);  // bits (sa, sb)
        const uint64_t bl = BL & seg, br = BR & seg;
        const uint32_t nL = static_cast<uint32_t>(__popcll(bl)), nR = static_cast<uint32_t>(__popcll(br));
        // pair k = p - (sa + 1): t_k = l_k < r_k (r_k: the k-th right stopper from the right)
        const uint32_t k = p - (sa + 1u);
        const uint32_t mn = min(nL, nR);
        const bool tk = in && k < mn && select_bit(bl, k) < select_bit(br, nR - 1u - k);
        const uint64_t T = ballot(tk) & seg;
        const uint32_t K = static_cast<uint32_t>(__builtin_ctzll(~(T >> min(sa + 1u, 63u))));
        // exchanges
        const uint64_t below = (1ull << p) - 1ull;
        const uint64_t above = p >= 63u ? 0ull : ~((2ull << p) - 1ull);
        const uint32_t rankL = static_cast<uint32_t>(__popcll(bl & below));
        const uint32_t rankR = static_cast<uint32_t>(__popcll(br & above));
        const bool isL = ((bl >> p) & 1ull) != 0ull, isR = ((br >> p) & 1ull) != 0ull;
        uint32_t s2 = p;
        if (isL && rankL < K) s2 = select_bit(br, nR - 1u - rankL);
        else if (isR && rankR < K) s2 = select_bit(bl, rankR);
        v.x = static_cast<uint32_t>(__shfl(static_cast<int>(v.x), static_cast<int>(s2)));
        v.y = static_cast<uint32_t>(__shfl(static_cast<int>(v.y), static_cast<int>(s2)));
        if (big) {
            uint32_t cut = 0xFFFFFFFFu;
            if (K < nL) cut = select_bit(bl, K);
            if (K >= 1u) cut = min(cut, select_bit(br, nR - K));
            if (p < cut) sb = cut;
            else sa = cut;
            --dp;
        }
    }
    // leaves: stable rank within [sa, sb)
    const float ri = __uint_as_float(v.x);
    uint32_t rk = 0;
#pragma unroll
    for (int j = 0; j < kRefLeaf; ++j) {
        const uint32_t t = sa + static_cast<uint32_t>(j);
        const float rt = __uint_as_float(static_cast<uint32_t>(__shfl(static_cast<int>(v.x), static_cast<int>(min(t, 63u)))));
        rk += (t < sb && (rt > ri || (rt == ri && t < p))) ? 1u : 0u;
    }
    if (p < len && !queued) ordp[sa + rk] = v.y;
    return true;
}

// One wave: libstdc++'s introsort on X[lo, hi) (<= kRefWaveLocal elements, > kRefLeaf) to the end -- the
// same partitions as the workgroup levels (median of (first + 1, mid, last - 1) moved to first, left
// stoppers resp <= pivot from the left paired with right stoppers resp >= pivot from the right while
// l_k < r_k, cut = min(l_K, r_{K-1})), then the final insertion sort of every leaf (stable, response
// descending) -- with the elements in the wave's LDS. Writes the range's visiting order into ord[lo, hi).
// A subrange at the depth limit is queued for the heapsort step (hq, hn). Returns false on a broken invariant.
__device__ bool ref_wave_resolve(uint2 *X, uint32_t *ord, uint32_t lo, uint32_t hi, uint32_t dep, uint2 *E,
                                 uint16_t *Lp, uint16_t *Rp, uint32_t *stk, uint32_t *hq, int *hn) {
    const int lane = lane_id();
    const uint32_t s = hi - lo;
    for (uint32_t i = lane; i < s; i += kWave) E[i] = X[lo + i];
    // stack entries: a (10 bits) | b (11 bits) << 10 | depth left << 21, positions relative to lo
    int top = 0;
    if (lane == 0) stk[0] = 0u | (s << 10) | (dep << 21);
    top = 1;
    bool ok = true;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    while (top > 0) {
        --top;
        const uint32_t ent = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(stk[top])));
        const uint32_t a = ent & 1023u, b = (ent >> 10) & 2047u, dp = ent >> 21;
        if (b - a <= static_cast<uint32_t>(kWave) && b - a > static_cast<uint32_t>(kRefLeaf)) {
            if (!ref_wave_small(E + a, b - a, dp, ord + lo + a, X + lo + a, lo + a, hq, hn)) {
                ok = false;
                break;
            }
            continue;
        }
        if (b - a <= static_cast<uint32_t>(kRefLeaf)) {
            // leaf: stable rank by response, descending (lanes 0-15)
            const int len = static_cast<int>(b - a);
            const int q = lane & (kRefLeaf - 1);
            const uint2 v = q < len ? E[a + q] : make_uint2(0u, 0u);
            const float ri = __uint_as_float(v.x);
            uint32_t rk = 0;
#pragma unroll
            for (int t = 0; t < kRefLeaf; ++t) {
                const float rt = __uint_as_float(static_cast<uint32_t>(__shfl(static_cast<int>(v.x), t)));
                rk += (t < len && (rt > ri || (rt == ri && t < q))) ? 1u : 0u;
            }
            if (lane < kRefLeaf && q < len) ord[lo + a + rk] = v.y;
            continue;
        }
        if (dp == 0u) {  // std::__partial_sort(a, b, b): back to X and queued for the heapsort step
            for (uint32_t i = lane; i < b - a; i += kWave) X[lo + a + i] = E[a + i];
            if (lane == 0) {
                const int q = atomicAdd(hn, 1);
                if (q < kRefMaxRanges) {
                    hq[2 * q] = lo + a;
                    hq[2 * q + 1] = lo + b;
                }
            }
            continue;
        }
        // pivot: __move_median_to_first(a, a + 1, mid, b - 1)
        const uint32_t mid = a + (b - a) / 2u;
        const uint2 xa = E[a + 1], xb = E[mid], xc = E[b - 1];
        const uint32_t ch = median_pos(__uint_as_float(xa.x), __uint_as_float(xb.x), __uint_as_float(xc.x), a + 1, mid, b - 1);
        const uint2 xp = ch == a + 1 ? xa : (ch == mid ? xb : xc);
        const uint2 x0 = E[a];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0) {
            E[a] = xp;
            E[ch] = x0;
        }
        const float pv = __uint_as_float(xp.x);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // stoppers of [a + 1, b): left ones by rank from the left, right ones by rank from the left (reversed below)
        uint32_t nL = 0, nR = 0;
        for (uint32_t i0 = a + 1; i0 < b; i0 += kWave) {
            const uint32_t i = i0 + lane;
            const bool in = i < b;
            const float rv = in ? __uint_as_float(E[i].x) : 0.0f;
            const bool ls = in && rv <= pv, rs = in && rv >= pv;
            const uint64_t bl = ballot(ls), br = ballot(rs);
            if (ls) Lp[nL + mbcnt64(bl, 0)] = static_cast<uint16_t>(i);
            if (rs) Rp[nR + mbcnt64(br, 0)] = static_cast<uint16_t>(i);
            nL += popc64(bl);
            nR += popc64(br);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // K: pairs k with l_k < r_k (r_k = the k-th right stopper from the right), monotone in k
        const uint32_t mn = min(nL, nR);
        uint32_t K = 0;
        for (uint32_t k0 = 0; k0 < mn; k0 += kWave) {
            const uint32_t k = k0 + lane;
            const bool t = k < mn && Lp[k] < Rp[nR - 1u - min(k, nR - 1u)];
            const uint64_t bt = ballot(t);
            const uint32_t run = bt == ~0ull ? 64u : static_cast<uint32_t>(__builtin_ctzll(~bt));
            K += run;
            if (run < 64u) break;
        }
        // the swaps (pairs are disjoint)
        for (uint32_t k0 = 0; k0 < K; k0 += kWave) {
            const uint32_t k = k0 + lane;
            if (k < K) {
                const uint32_t pl = Lp[k], pr = Rp[nR - 1u - k];
                const uint2 vl = E[pl], vr = E[pr];
                E[pl] = vr;
                E[pr] = vl;
            }
        }
        uint32_t cut = 0xFFFFFFFFu;
        if (K < nL) cut = Lp[K];
        if (K >= 1u) cut = min(cut, static_cast<uint32_t>(Rp[nR - K]));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (cut <= a || cut >= b || top + 2 > kRefStack) {  // (cannot happen: the scans stop inside the range)
            ok = false;
            break;
        }
        // children, left one on top (depth-first; the order of resolution does not matter)
        if (lane == 0) {
            stk[top] = cut | (b << 10) | ((dp - 1u) << 21);
            stk[top + 1] = a | (cut << 10) | ((dp - 1u) << 21);
        }
        top += 2;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    return ok;
}

// Diagnostic phase clocks (SelectArgs::stamps, FD_SELECT_STAMPS): thread 0 adds the cycles since the
// previous mark to slot k of the frame's stamps (slots 16-23; k_select uses 0-15).
#define FD_REF_MARK(k)                                                                  \
    do {                                                                                \
        if (a.stamps && tid == 0) {                                                     \
            const uint64_t now_ = __builtin_readcyclecounter();                         \
            a.stamps[static_cast<int64_t>(f) * 32 + (k)] += now_ - t_mark;              \
            t_mark = now_;                                                              \
        }                                                                               \
    } while (0)
#define FD_REF_COUNT(k, v)                                                              \
    do {                                                                                \
        if (a.stamps && tid == 0) a.stamps[static_cast<int64_t>(f) * 32 + (k)] += (v);  \
    } while (0)

// Wave 0: the active ranges at the depth limit (L.heap_j) heapsorted one at a time (std::__partial_sort,
// ref_heapsort; in LDS when the range fits the free space: the greedy span before the grid exists, pxy ..
// cmask after), their visiting order written to ord (final), and the range list rebuilt without them.
// (A function of its own: the rare path stays out of k_select_reference's register allocation.)
__device__ __attribute__((noinline)) void ref_heap_step(lds_t<RefLds> *Lp, uint2 *X, uint32_t *ord, uint32_t n, int m,
                                                        bool grid_ready) {
    RefLds &L = *from_lds(Lp);
    const int lane = lane_id();
    const int c = L.cur, nh = L.n_heap;
    const uint32_t cap_lds = static_cast<uint32_t>(
        (grid_ready ? sizeof(L.pxy) + sizeof(L.pcell) + sizeof(L.cmask)
                    : sizeof(L.pxy) + sizeof(L.pcell) + sizeof(L.cmask) + sizeof(L.grid_lds)) / sizeof(uint2));
    for (int h = 0; h < nh; ++h) {
        const uint32_t j = L.heap_j[h];
        const uint32_t lo = L.r_lo[c][j], hi = min(L.r_hi[c][j], n);
        const uint32_t len = hi > lo ? hi - lo : 0u;
        uint2 *hbuf = X + lo;
        if (len <= cap_lds) {
            hbuf = reinterpret_cast<uint2 *>(L.pxy);
            for (uint32_t i = lane; i < len; i += kWave) hbuf[i] = X[lo + i];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        ref_heapsort(hbuf, static_cast<int>(len));
        for (uint32_t i = lane; i < len; i += kWave) {
            const uint2 e = hbuf[i];
            X[lo + i] = e;
            ord[lo + i] = e.y;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // the list without them (order kept), into the other buffer
    const int nc = c ^ 1;
    uint32_t at = 0;
    for (int b = 0; b < L.m_all; b += kWave) {
        const int j = b + lane;
        const bool keep = j < L.m_all && !(j < m && L.r_dep[c][j] == 0u);
        const uint64_t bk = ballot(keep);
        if (keep) {
            const uint32_t q = at + static_cast<uint32_t>(mbcnt64(bk, 0));
            L.r_lo[nc][q] = L.r_lo[c][j];
            L.r_hi[nc][q] = L.r_hi[c][j];
            L.r_dep[nc][q] = L.r_dep[c][j];
        }
        at += static_cast<uint32_t>(popc64(bk));
    }
    if (lane == 0) {
        L.m_all = static_cast<int>(at);
        L.cur = nc;
    }
    __builtin_amdgcn_s_waitcnt(0);
    set_active(L, L.fin + kSelectChunk);
}

template <int NT>
__global__ __launch_bounds__(NT) void k_select_reference(SelectArgs a, RefSortArgs r) {
    static_assert(NT == kRefThreads, "k_select_reference runs 1024 threads");
    __shared__ RefLds L;
    const int f = blockIdx.x, tid = threadIdx.x, lane = lane_id(), wv = tid / kWave;
    const uint32_t st0 = a.status[f];
    if (!(st0 & FD_FRAME_TIES) || (st0 & FD_FRAME_GUARD)) return;
    uint64_t t_mark = a.stamps && tid == 0 ? __builtin_readcyclecounter() : 0ull;
    if (a.stamps && tid == 0)
        for (int k = 0; k < 32; ++k) a.stamps[static_cast<int64_t>(f) * 32 + k] = 0;  // (after k_select's printout)
    const uint32_t n = static_cast<uint32_t>(min(static_cast<int64_t>(a.cand_n[f]), a.list_cap));
    const int rows = a.rows, cols = a.cols, d = a.dist;
    const uint32_t npx = static_cast<uint32_t>(rows) * static_cast<uint32_t>(cols);
    const float *lresp = a.list_resp + static_cast<int64_t>(f) * a.list_cap;
    const uint32_t *lidx = a.list_idx + static_cast<int64_t>(f) * a.list_cap;
    uint2 *X = r.x + static_cast<int64_t>(f) * r.cap;
    const uint32_t *Xr = reinterpret_cast<const uint32_t *>(X);  // X[p].x (response bits) = Xr[2p]
    uint32_t *lpos = r.lpos + static_cast<int64_t>(f) * r.cap;
    uint32_t *rpos = r.rpos + static_cast<int64_t>(f) * r.cap;
    uint32_t *ord = r.ord + static_cast<int64_t>(f) * r.cap;

    // ---- 1. the push order -------------------------------------------------------------------------
    // (every per-candidate loop loads kRefPush candidates' data before using any: one memory round trip
    // per kRefPush candidates instead of one or two per candidate)
    constexpr int kRefPush = 8;
    if (r.wide) {
        // (the prelude built X)
    } else if (r.push_order) {
        for (uint32_t i0 = tid; i0 < n; i0 += kRefPush * NT) {
            float rv[kRefPush];
            uint32_t qv[kRefPush];
#pragma unroll
            for (int k = 0; k < kRefPush; ++k) {
                const uint32_t i = min(i0 + k * NT, n - 1u);
                rv[k] = lresp[i];
                qv[k] = lidx[i];
            }
#pragma unroll
            for (int k = 0; k < kRefPush; ++k)
                if (i0 + k * NT < n) X[i0 + k * NT] = make_uint2(__float_as_uint(rv[k]), qv[k]);
        }
    } else {
        // Raster order of unique pixel indices, a part of the frame at a time: the part's candidate bitmap
        // in LDS (the greedy's arrays, pxy .. grid_lds, are free until the grid is initialised below; LDS
        // atomics instead of one global atomic per candidate, which one CU issues slowly), its word prefix
        // (offset by the earlier parts' candidates) in rpos, rank = prefix + set bits below.
        static_assert(offsetof(RefLds, pcell) == offsetof(RefLds, pxy) + sizeof(L.pxy) &&
                          offsetof(RefLds, cmask) == offsetof(RefLds, pcell) + sizeof(L.pcell) &&
                          offsetof(RefLds, grid_lds) == offsetof(RefLds, cmask) + sizeof(L.cmask),
                      "bitmap span: pxy .. grid_lds contiguous");
        constexpr uint32_t kPartWords = (sizeof(L.pxy) + sizeof(L.pcell) + sizeof(L.cmask) + sizeof(L.grid_lds)) / 4;
        uint32_t *const lbits = L.pxy;
        uint32_t *const wpre = rpos;
        const uint32_t words = (npx + 31u) >> 5;
        uint32_t carry = 0;  // candidates in the earlier parts
        for (uint32_t pw0 = 0; pw0 < words; pw0 += kPartWords) {
            const uint32_t pw = min(kPartWords, words - pw0);
            for (uint32_t w = tid; w < pw; w += NT) lbits[w] = 0u;
            __syncthreads();
            for (uint32_t i0 = tid; i0 < n; i0 += kRefPush * NT) {
                uint32_t qv[kRefPush];
#pragma unroll
                for (int k = 0; k < kRefPush; ++k) qv[k] = lidx[min(i0 + k * NT, n - 1u)];
#pragma unroll
                for (int k = 0; k < kRefPush; ++k) {
                    const uint32_t wl = (qv[k] >> 5) - pw0;  // (wraps past the part when below it)
                    if (i0 + k * NT < n && qv[k] < npx && wl < pw) atomicOr(&lbits[wl], 1u << (qv[k] & 31u));
                }
            }
            __syncthreads();
            // word prefix: a run of consecutive words per thread
            const uint32_t per = (pw + NT - 1) / NT;
            const uint32_t w0 = min(pw, tid * per), w1 = min(pw, w0 + per);
            uint32_t cnt = 0;
            for (uint32_t w = w0; w < w1; ++w) cnt += __popc(lbits[w]);
            uint32_t tot;
            uint32_t base = carry + block_excl(cnt, L.wsum, tot);
            for (uint32_t w = w0; w < w1; ++w) {
                wpre[pw0 + w] = base;
                base += __popc(lbits[w]);
            }
            carry += tot;
            __syncthreads();  // (the prefix stores are read back by other threads: same workgroup, L1-coherent
                              // through the barrier's release/acquire)
            for (uint32_t i0 = tid; i0 < n; i0 += kRefPush * NT) {
                uint32_t qv[kRefPush], wp[kRefPush];
                float rv[kRefPush];
#pragma unroll
                for (int k = 0; k < kRefPush; ++k) {
                    const uint32_t i = min(i0 + k * NT, n - 1u);
                    qv[k] = lidx[i];
                    rv[k] = lresp[i];
                }
#pragma unroll
                for (int k = 0; k < kRefPush; ++k) {
                    const uint32_t wl = min((qv[k] >> 5) - pw0, pw - 1u);
                    wp[k] = wpre[pw0 + wl];
                }
#pragma unroll
                for (int k = 0; k < kRefPush; ++k) {
                    const uint32_t q = qv[k], wl = (q >> 5) - pw0;
                    if (i0 + k * NT >= n || q >= npx || wl >= pw) continue;
                    const uint32_t rk = wp[k] + __popc(lbits[wl] & ((1u << (q & 31u)) - 1u));
                    X[FD_REF_IDX(rk, n, 1)] = make_uint2(__float_as_uint(rv[k]), q);
                }
            }
            __syncthreads();  // lbits reused by the next part (and the grid below)
        }
    }

    // ---- greedy state (k_select_ordered) --------------------------------------------------------------
    const bool use_grid = d >= 1 || (d == 0 && a.grid_at_d0);
    const int gw2 = a.grid_w + 2;
    const int cells = gw2 * (a.grid_h + 2);
    const bool grid_in_lds = cells <= kGridLdsCells;
    uint32_t *const grid_g = a.grid_global ? a.grid_global + static_cast<int64_t>(f) * cells : nullptr;
    uint32_t *const grid = grid_in_lds ? L.grid_lds : grid_g;
    const uint32_t prior = a.prior_counts ? static_cast<uint32_t>(a.prior_counts[f]) : 0u;
    const uint32_t *fmask = a.mask ? a.mask + static_cast<int64_t>(f) * rows * a.mask_wpr : nullptr;
    const uint32_t s1 = static_cast<uint32_t>(d + 1);
    // The grid is initialised just before the first greedy scan: until then its LDS (with pxy .. cmask)
    // holds the partition levels' element copies and stopper positions (LDS mode below).
    bool grid_ready = false;
    if (tid == 0) {
        L.s_done = 0;
        L.s_acc = 0;
        L.tie_prev = 0;
        L.tie_has_prev = 0;
        L.fail = 0;
        L.n_hq = 0;
        L.cur = 0;
        L.n_leaf = 0;
        L.fin = 0;
        L.n_wl = 0;
        // __introsort_loop(0, n, 2 * __lg(n)); n <= 16: the final insertion sort alone (one leaf)
        if (r.wide) {
            // the prelude's state: [0, h) of its last level, then the levels' right children, in position
            // order; ranges of <= 16 elements are leaves
            const RefCtl &C = r.ctl[f];
            const uint32_t nlev = min(C.nlev, static_cast<uint32_t>(kRefWideLevels));
            if (C.n != n || C.bad) L.fail = 6;
            int m = 0, nl = 0;
            auto add = [&](uint32_t lo, uint32_t hi, uint32_t dep) {
                if (hi > lo + static_cast<uint32_t>(kRefLeaf)) {
                    L.r_lo[0][m] = lo;
                    L.r_hi[0][m] = hi;
                    L.r_dep[0][m] = dep;
                    ++m;
                } else if (hi > lo) {
                    L.leaf_lo[nl] = lo;
                    L.leaf_hi[nl] = hi;
                    ++nl;
                }
            };
            add(0u, min(C.h[nlev], n), C.dep[nlev]);
            for (int l = static_cast<int>(nlev) - 1; l >= 0; --l) add(C.sib_lo[l], min(C.sib_hi[l], n), C.dep[l] - 1u);
            L.m_all = m;
            L.n_leaf = nl;
        } else if (n > static_cast<uint32_t>(kRefLeaf)) {
            L.r_lo[0][0] = 0;
            L.r_hi[0][0] = n;
            L.r_dep[0][0] = 2u * (31u - __clz(n));
            L.m_all = 1;
        } else {
            L.m_all = 0;
            if (n > 0) {
                L.leaf_lo[0] = 0;
                L.leaf_hi[0] = n;
                L.n_leaf = 1;
            }
        }
    }
    __syncthreads();
    FD_REF_MARK(16);  // push order (bitmap, ranks, scatter) + grid init
    if (wv == 0) set_active(L, kSelectChunk);
    __syncthreads();

    // windows x levels (bounded: each level halves). A frame whose emulation has not finished when the
    // bound runs out -- LSD seed orders of ~10M entries would need that many -- is failed (code 8), not
    // reported resolved with an unwritten tail of ord. (r.guard_limit: diagnostic override only.)
    const int guard_lim = r.guard_limit > 0 ? r.guard_limit : 1 << 16;
    bool finished = false;  // (uniform: set where every thread leaves the loop together)
    bool wrote = false;     // a window's greedy has written features (out_xy no longer k_select's)
    for (int guard = 0; guard < guard_lim; ++guard) {
        const int m = L.m_act;
        if (m > 0) {
            // ---- active ranges at the depth limit: std::__partial_sort(first, last, last) -----------------
            // Heapsorted one at a time by wave 0 (in LDS when the range fits the free space: the greedy
            // span before the grid exists, pxy .. cmask after), their visiting order written to ord (final),
            // and dropped from the range list; then the level runs on the rest.
            if (tid == 0) L.n_heap = 0;
            __syncthreads();
            if (tid < m && L.r_dep[L.cur][tid] == 0u) L.heap_j[atomicAdd(&L.n_heap, 1)] = static_cast<uint32_t>(tid);
            __syncthreads();
            if (L.n_heap > 0) {
                if (wv == 0) ref_heap_step(to_lds(&L), X, ord, n, m, grid_ready);
                __syncthreads();
                FD_REF_COUNT(31, 1u);
                continue;
            }
            // ---- one partition level over the active ranges ----------------------------------------------
            const int c = L.cur;
            const uint64_t t_level = a.stamps && tid == 0 ? __builtin_readcyclecounter() : 0ull;
            if (tid < m) {
                const uint32_t lo = L.r_lo[c][tid], hi = L.r_hi[c][tid];
                if (L.r_dep[c][tid] == 0u) L.fail = 1;  // invariant: depth-0 ranges were heapsorted above
                const uint32_t mid = lo + (hi - lo) / 2u;
                const uint2 xa = X[FD_REF_IDX(lo + 1, n, 2)], xb = X[FD_REF_IDX(mid, n, 2)], xc = X[FD_REF_IDX(hi - 1, n, 2)];
                const uint32_t ch = median_pos(as_f(xa.x), as_f(xb.x), as_f(xc.x), lo + 1, mid, hi - 1);
                const uint2 xp = ch == lo + 1 ? xa : (ch == mid ? xb : xc);
                const uint2 x0 = X[FD_REF_IDX(lo, n, 3)];
                X[FD_REF_IDX(lo, n, 3)] = xp;
                X[FD_REF_IDX(ch, n, 3)] = x0;
                L.piv[tid] = as_f(xp.x);
                L.cut[tid] = kNoPos;  // (written by the element where l_k < r_k stops holding)
            }
            __syncthreads();
            FD_REF_MARK(24);  // pivots
            if (L.fail) break;
            const uint32_t T = L.T;
            const bool cached = T <= kRefRidCap;  // passes 2-3 read the range index pass 1 stored
            // LDS mode (small levels before the first greedy scan): pass 1 also keeps each element's
            // response in LDS (RV) and the stopper positions live in LDS (LP, RP) instead of lpos / rpos:
            // pass 2 makes no memory round trip, pass 3 one (the swaps themselves).
            const bool ldsm = cached && !grid_ready;
            uint32_t *const RV = L.pxy;  // [kRefRidCap] x 3 over pxy .. grid_lds (96 KiB, see the push)
            uint32_t *const LP = RV + kRefRidCap;
            uint32_t *const RP = LP + kRefRidCap;
            const uint32_t blk = ((T + kRefWaves * kWave - 1) / (kRefWaves * kWave)) * kWave;
            const uint32_t e0 = min(T, wv * blk), e1 = min(T, e0 + blk);
            // pass 1: stopper counts per wave, local prefixes at the range heads. Each wave walks its block
            // kRefU rounds of 64 elements at a time: the rounds' element positions first (LDS), then all
            // their response loads at once, then the ballots in order (one global round trip per kRefU
            // rounds instead of one per round).
            {
                uint32_t cl = 0, cr = 0;
                int jw = e0 < e1 ? range_search(L.o, m, e0) : 0;
                for (uint32_t b0 = e0; b0 < e1; b0 += kRefU * kWave) {
                    uint32_t pu[kRefU];
                    int ju[kRefU];
                    bool vu[kRefU];
                    float ru[kRefU];
#pragma unroll
                    for (int u = 0; u < kRefU; ++u) {
                        const uint32_t b = b0 + u * kWave, e = b + lane;
                        vu[u] = e < e1;
                        while (jw + 1 < m && L.o[jw + 1] <= b) ++jw;
                        ju[u] = vu[u] ? range_of(L.o, m, jw, e) : jw;
                        pu[u] = L.r_lo[c][ju[u]] + 1u + (e - L.o[ju[u]]);
                    }
#pragma unroll
                    for (int u = 0; u < kRefU; ++u) ru[u] = vu[u] ? as_f(Xr[2u * FD_REF_IDX(pu[u], n, 5)]) : 0.0f;
                    if (cached) {
#pragma unroll
                        for (int u = 0; u < kRefU; ++u)
                            if (vu[u]) {
                                L.rid[b0 + u * kWave + lane] = static_cast<uint16_t>(ju[u]);
                                if (ldsm) RV[b0 + u * kWave + lane] = __float_as_uint(ru[u]);
                            }
                    }
#pragma unroll
                    for (int u = 0; u < kRefU; ++u) {
                        const uint32_t e = b0 + u * kWave + lane;
                        const int j = ju[u];
                        const float pv = L.piv[j];
                        const bool ls = vu[u] && ru[u] <= pv, rs = vu[u] && ru[u] >= pv;
                        const uint64_t bl = ballot(ls), br = ballot(rs);
                        if (vu[u] && e == L.o[j]) {
                            L.headL[j] = cl + mbcnt64(bl, 0);
                            L.headR[j] = cr + mbcnt64(br, 0);
                            L.headW[j] = wv;
                        }
                        cl += popc64(bl);
                        cr += popc64(br);
                    }
                }
                if (lane == 0) {
                    L.waveL[wv] = cl;
                    L.waveR[wv] = cr;
                }
            }
            __syncthreads();
            FD_REF_MARK(25);  // pass 1
            // per range: global stopper bases and counts
            uint32_t wbL, wbR;  // exclusive wave prefixes, lane i = wave i
            {
                const uint32_t vl = lane < kRefWaves ? L.waveL[lane] : 0u, vr = lane < kRefWaves ? L.waveR[lane] : 0u;
                wbL = wave_incl_add(vl) - vl;
                wbR = wave_incl_add(vr) - vr;
            }
            const uint32_t totL = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wbL), kRefWaves - 1)) +
                                  L.waveL[kRefWaves - 1];
            const uint32_t totR = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wbR), kRefWaves - 1)) +
                                  L.waveR[kRefWaves - 1];
            {
                // every wave computes its lanes' ranges (shuffles are per wave); ranges j = tid < m
                const int j = tid < m ? tid : 0;
                const int jn = j + 1;
                const uint32_t hw = L.headW[j], hwn = jn < m ? L.headW[jn] : 0u;
                const uint32_t bLj = static_cast<uint32_t>(__shfl(static_cast<int>(wbL), static_cast<int>(hw))) + L.headL[j];
                const uint32_t bRj = static_cast<uint32_t>(__shfl(static_cast<int>(wbR), static_cast<int>(hw))) + L.headR[j];
                // (shuffles with every lane active: ds_bpermute does not read inactive source lanes)
                const uint32_t sLn = static_cast<uint32_t>(__shfl(static_cast<int>(wbL), static_cast<int>(hwn)));
                const uint32_t sRn = static_cast<uint32_t>(__shfl(static_cast<int>(wbR), static_cast<int>(hwn)));
                const uint32_t bLn = jn < m ? sLn + L.headL[jn] : totL;
                const uint32_t bRn = jn < m ? sRn + L.headR[jn] : totR;
                if (tid < m) {
                    L.bL[tid] = bLj;
                    L.nL[tid] = bLn - bLj;
                    L.eR[tid] = bRn;
                    L.nR[tid] = bRn - bRj;
                }
            }
            __syncthreads();
            FD_REF_MARK(26);  // stopper bases
            // passes 2-3, compiled twice: stopper positions in LDS (LDS mode) or in lpos / rpos
            auto passes = [&](auto lm) {
                constexpr bool LM = decltype(lm)::value;
                auto lp_st = [&](uint32_t i, uint32_t v) {
                    if constexpr (LM) LP[i] = v;
                    else lpos[i] = v;
                };
                auto rp_st = [&](uint32_t i, uint32_t v) {
                    if constexpr (LM) RP[i] = v;
                    else rpos[i] = v;
                };
                auto lp_ld = [&](uint32_t i) -> uint32_t {
                    if constexpr (LM) return LP[i];
                    else return lpos[i];
                };
                auto rp_ld = [&](uint32_t i) -> uint32_t {
                    if constexpr (LM) return RP[i];
                    else return rpos[i];
                };
                // pass 2: scatter stopper positions by rank (left stoppers from the left, right from the right);
                // the same kRefU-round walk as pass 1
                {
                    const uint32_t mywbL = static_cast<uint32_t>(__shfl(static_cast<int>(wbL), wv));
                    const uint32_t mywbR = static_cast<uint32_t>(__shfl(static_cast<int>(wbR), wv));
                    uint32_t cl = mywbL, cr = mywbR;
                    int jw = !cached && e0 < e1 ? range_search(L.o, m, e0) : 0;
                    for (uint32_t b0 = e0; b0 < e1; b0 += kRefU * kWave) {
                        uint32_t pu[kRefU];
                        int ju[kRefU];
                        bool vu[kRefU];
                        float ru[kRefU];
    #pragma unroll
                        for (int u = 0; u < kRefU; ++u) {
                            const uint32_t b = b0 + u * kWave, e = b + lane;
                            vu[u] = e < e1;
                            if (cached) {
                                ju[u] = vu[u] ? L.rid[e] : 0;
                            } else {
                                while (jw + 1 < m && L.o[jw + 1] <= b) ++jw;
                                ju[u] = vu[u] ? range_of(L.o, m, jw, e) : jw;
                            }
                            pu[u] = L.r_lo[c][ju[u]] + 1u + (e - L.o[ju[u]]);
                        }
    #pragma unroll
                        for (int u = 0; u < kRefU; ++u)
                            ru[u] = !vu[u] ? 0.0f : (LM ? as_f(RV[b0 + u * kWave + lane]) : as_f(Xr[2u * FD_REF_IDX(pu[u], n, 6)]));
    #pragma unroll
                        for (int u = 0; u < kRefU; ++u) {
                            const int j = ju[u];
                            const uint32_t oj = L.o[j], p = pu[u];
                            const float pv = L.piv[j];
                            const bool ls = vu[u] && ru[u] <= pv, rs = vu[u] && ru[u] >= pv;
                            const uint64_t bl = ballot(ls), br = ballot(rs);
                            if (ls) {
                                const uint32_t rankL = static_cast<uint32_t>(mbcnt64(bl, 0)) + cl - L.bL[j];  // 0-based
                                lp_st(FD_REF_IDX(oj + rankL, L.T, 7), p);
                            }
                            if (rs) {
                                const uint32_t rankR = L.eR[j] - (static_cast<uint32_t>(mbcnt64(br, 0)) + cr) - 1u;  // from the right
                                rp_st(FD_REF_IDX(oj + rankR, L.T, 8), p);
                            }
                            cl += popc64(bl);
                            cr += popc64(br);
                        }
                    }
                }
                __syncthreads();
                FD_REF_MARK(27);  // pass 2
                // pass 3 (swaps and cuts in one pass): pair k is exchanged iff t_k = l_k < r_k (monotone in k,
                // so these are exactly the pairs k < K); the element where t stops holding finds K and writes
                // the range's cut -- K = k + 1 at the last true pair (cut = min(l_{K}, r_{K-1})), K = 0 at a
                // false first pair (cut = l_0). The kRefU rounds' stopper positions, then their elements,
                // loaded together.
                {
                    int jw = !cached && e0 < e1 ? range_search(L.o, m, e0) : 0;
                    for (uint32_t b0 = e0; b0 < e1; b0 += kRefU * kWave) {
                        int ju[kRefU];
                        bool vu[kRefU];
                        uint32_t l0[kRefU], r0[kRefU], l1[kRefU], r1[kRefU];
                        uint2 vl[kRefU], vr[kRefU];
    #pragma unroll
                        for (int u = 0; u < kRefU; ++u) {
                            const uint32_t b = b0 + u * kWave, e = b + lane;
                            vu[u] = e < e1;
                            if (cached) {
                                ju[u] = vu[u] ? L.rid[e] : 0;
                            } else {
                                while (jw + 1 < m && L.o[jw + 1] <= b) ++jw;
                                ju[u] = vu[u] ? range_of(L.o, m, jw, e) : jw;
                            }
                        }
    #pragma unroll
                        for (int u = 0; u < kRefU; ++u) {
                            const uint32_t e = b0 + u * kWave + lane;
                            // (clamped reads: entries past T are never used)
                            l0[u] = lp_ld(FD_REF_IDX(min(e, L.T - 1u), L.T, 9));
                            r0[u] = rp_ld(FD_REF_IDX(min(e, L.T - 1u), L.T, 9));
                            l1[u] = lp_ld(FD_REF_IDX(min(e + 1u, L.T - 1u), L.T, 10));
                            r1[u] = rp_ld(FD_REF_IDX(min(e + 1u, L.T - 1u), L.T, 10));
                        }
                        bool su[kRefU];
    #pragma unroll
                        for (int u = 0; u < kRefU; ++u) {
                            const uint32_t e = b0 + u * kWave + lane;
                            const int j = ju[u];
                            const uint32_t k = e - L.o[j];  // 0-based pair index
                            const uint32_t nLj = L.nL[j], mn = min(nLj, L.nR[j]);
                            const bool t = vu[u] && k < mn && l0[u] < r0[u];
                            const bool tn = t && k + 1 < mn && l1[u] < r1[u];
                            su[u] = t;
                            if (t && !tn) {  // K = k + 1
                                uint32_t cut = r0[u];
                                if (k + 1 < nLj) cut = min(cut, l1[u]);
                                L.cut[j] = cut;
                            } else if (vu[u] && k == 0u && !t) {  // K = 0 (nL >= 1: the median leaves a stopper)
                                L.cut[j] = l0[u];
                            }
                            if (t) {
                                l0[u] = FD_REF_IDX(l0[u], n, 12);
                                r0[u] = FD_REF_IDX(r0[u], n, 13);
                            }
                        }
    #pragma unroll
                        for (int u = 0; u < kRefU; ++u) {
                            if (su[u]) {
                                vl[u] = X[l0[u]];
                                vr[u] = X[r0[u]];
                            }
                        }
    #pragma unroll
                        for (int u = 0; u < kRefU; ++u) {
                            if (su[u]) {
                                X[l0[u]] = vr[u];
                                X[r0[u]] = vl[u];
                            }
                        }
                    }
                }
                __syncthreads();
                FD_REF_MARK(29);  // pass 3 (swaps + cuts)
            };
            if (ldsm) passes(std::true_type{});
            else passes(std::false_type{});
            // children: ranges > 16 into the next list (in order), the rest are leaves
            if (wv == 0) {
                const int nc = c ^ 1;
                uint32_t w_at = 0, l_at = 0;
                // before the first greedy scan, children of <= kRefWaveLocal elements go to the wave-local
                // list (while it has room) instead of the next level
                const bool wl_on = kRefWaveLocal > 0u && !grid_ready;
                uint32_t v_at = static_cast<uint32_t>(L.n_wl);
                for (int b = 0; b < m; b += kWave) {
                    const int j = b + lane;
                    const bool in = j < m;
                    uint32_t lo = 0, hi = 0, ct = 0, dp = 0;
                    if (in) {
                        lo = L.r_lo[c][j];
                        hi = L.r_hi[c][j];
                        ct = L.cut[j];
                        dp = L.r_dep[c][j] - 1u;
                        if (ct <= lo || ct >= hi) {  // (cannot happen: the scans stop inside the range)
                            L.fail = 2;
                            ct = lo + 1;
                        }
                    }
                    bool bigL = in && ct - lo > static_cast<uint32_t>(kRefLeaf);
                    bool bigR = in && hi - ct > static_cast<uint32_t>(kRefLeaf);
                    {
                        const bool cL = wl_on && bigL && ct - lo <= kRefWaveLocal;
                        const bool cR = wl_on && bigR && hi - ct <= kRefWaveLocal;
                        const uint32_t nv = (cL ? 1u : 0u) + (cR ? 1u : 0u);
                        const uint32_t iv = wave_incl_add(nv);
                        uint32_t pv = v_at + iv - nv;
                        if (cL && pv < static_cast<uint32_t>(kRefMaxRanges)) {
                            L.wl_lo[pv] = lo;
                            L.wl_hi[pv] = ct;
                            L.wl_dep[pv] = dp;
                            bigL = false;
                        }
                        if (cL) ++pv;
                        if (cR && pv < static_cast<uint32_t>(kRefMaxRanges)) {
                            L.wl_lo[pv] = ct;
                            L.wl_hi[pv] = hi;
                            L.wl_dep[pv] = dp;
                            bigR = false;
                        }
                        v_at += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(iv), kWave - 1));
                    }
                    const uint32_t nb = (bigL ? 1u : 0u) + (bigR ? 1u : 0u);
                    const bool leafL = in && ct - lo <= static_cast<uint32_t>(kRefLeaf);
                    const bool leafR = in && hi - ct <= static_cast<uint32_t>(kRefLeaf);
                    const uint32_t nlf = (leafL ? 1u : 0u) + (leafR ? 1u : 0u);
                    const uint32_t ib = wave_incl_add(nb), il = wave_incl_add(nlf);
                    uint32_t pb = w_at + ib - nb, pl = l_at + il - nlf;
                    if (bigL && pb < kRefMaxRanges) {
                        L.r_lo[nc][pb] = lo;
                        L.r_hi[nc][pb] = ct;
                        L.r_dep[nc][pb] = dp;
                    }
                    if (bigL) ++pb;
                    if (bigR && pb < kRefMaxRanges) {
                        L.r_lo[nc][pb] = ct;
                        L.r_hi[nc][pb] = hi;
                        L.r_dep[nc][pb] = dp;
                    }
                    if (leafL) {
                        L.leaf_lo[pl] = lo;
                        L.leaf_hi[pl] = ct;
                        ++pl;
                    }
                    if (leafR) {
                        L.leaf_lo[pl] = ct;
                        L.leaf_hi[pl] = hi;
                    }
                    w_at += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(ib), kWave - 1));
                    l_at += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(il), kWave - 1));
                }
                // the ranges right of the window follow unchanged
                const int rest = L.m_all - m;
                for (int i = lane; i < rest; i += kWave) {
                    const uint32_t q = w_at + static_cast<uint32_t>(i);
                    if (q < kRefMaxRanges) {
                        L.r_lo[nc][q] = L.r_lo[c][m + i];
                        L.r_hi[nc][q] = L.r_hi[c][m + i];
                        L.r_dep[nc][q] = L.r_dep[c][m + i];
                    }
                }
                if (lane == 0) {
                    const uint32_t tot = w_at + static_cast<uint32_t>(rest);
                    if (tot > kRefMaxRanges) L.fail = 3;
                    L.m_all = static_cast<int>(min(tot, static_cast<uint32_t>(kRefMaxRanges)));
                    L.cur = nc;
                    L.n_leaf = static_cast<int>(l_at);
                    L.n_wl = static_cast<int>(min(v_at, static_cast<uint32_t>(kRefMaxRanges)));
                }
                __builtin_amdgcn_s_waitcnt(0);
                set_active(L, L.fin + kSelectChunk);
            }
            __syncthreads();
            FD_REF_MARK(30);  // children + active prefix
            if (a.stamps && tid == 0) {  // per level (slots 0-15): T << 40 | cycles
                const uint64_t lv = a.stamps[static_cast<int64_t>(f) * 32 + 18];
                if (lv < 16u)
                    a.stamps[static_cast<int64_t>(f) * 32 + lv] =
                        (static_cast<uint64_t>(T) << 40) | (__builtin_readcyclecounter() - t_level);
            }
            FD_REF_COUNT(18, 1u);
            FD_REF_COUNT(19, T);
            if (L.fail) break;
        }
        // ---- leaves: the final insertion sort (stable, response descending) into the visiting order ---
        // 16 lanes per leaf: lane q holds element q and counts the elements that precede it
        for (int lf0 = 0; lf0 < L.n_leaf; lf0 += NT / kRefLeaf) {
            const int lf = lf0 + tid / kRefLeaf, q = tid % kRefLeaf;
            const bool have_leaf = lf < L.n_leaf;
            const uint32_t lo = have_leaf ? L.leaf_lo[lf] : 0u, hi = have_leaf ? L.leaf_hi[lf] : 0u;
            const int len = min(static_cast<int>(hi - lo), kRefLeaf);
            const bool mine = have_leaf && q < len;
            const uint2 v = mine ? X[FD_REF_IDX(lo + q, n, 16)] : make_uint2(0u, 0u);
            const float ri = as_f(v.x);
            uint32_t rk = 0;
#pragma unroll
            for (int t = 0; t < kRefLeaf; ++t) {  // lane group's element t (every lane of the wave takes part)
                const float rt = as_f(static_cast<uint32_t>(__shfl(static_cast<int>(v.x), (lane & ~(kRefLeaf - 1)) + t)));
                rk += (t < len && (rt > ri || (rt == ri && t < q))) ? 1u : 0u;
            }
            if (mine) ord[FD_REF_IDX(lo + rk, n, 17)] = v.y;
        }
        __syncthreads();
        FD_REF_MARK(20);  // leaves
        if (tid == 0) L.n_leaf = 0;
        if (L.m_act > 0) {
            __syncthreads();
            continue;
        }
        // ---- wave-local ranges: one wave each, partitioned to the end in LDS (the greedy span) -----------
        if (L.n_wl > 0) {
            constexpr uint32_t kWaveBytes = kRefWaveLocal * (8u + 2u + 2u);
            static_assert(kRefWaves * kWaveBytes <= sizeof(L.pxy) + sizeof(L.pcell) + sizeof(L.cmask) + sizeof(L.grid_lds),
                          "wave-local buffers fit the greedy span");
            unsigned char *const wb = reinterpret_cast<unsigned char *>(L.pxy) + wv * kWaveBytes;
            uint2 *const E = reinterpret_cast<uint2 *>(wb);
            uint16_t *const Lp = reinterpret_cast<uint16_t *>(wb + kRefWaveLocal * 8u);
            uint16_t *const Rp = Lp + kRefWaveLocal;
            const int nw = L.n_wl;
            // largest ranges first, each to whichever wave is free (longest-processing-time order)
            if (tid < nw) {
                const uint32_t st = L.wl_hi[tid] - L.wl_lo[tid];
                uint32_t rk = 0;
                for (int u = 0; u < nw; ++u) {
                    const uint32_t su = L.wl_hi[u] - L.wl_lo[u];
                    rk += (su > st || (su == st && u < tid)) ? 1u : 0u;
                }
                L.wl_ord[rk] = static_cast<uint32_t>(tid);
            }
            if (tid == 0) L.wl_next = kRefWaves;
            __syncthreads();
            bool ok = true;
            for (int j = wv; j < nw && ok;) {
                const uint32_t q = L.wl_ord[j];
                ok = ref_wave_resolve(X, ord, L.wl_lo[q], L.wl_hi[q], L.wl_dep[q], E, Lp, Rp, L.wstk[wv], L.hq, &L.n_hq);
                int nj = 0;
                if (lane == 0) nj = atomicAdd(&L.wl_next, 1);
                j = __builtin_amdgcn_readfirstlane(__shfl(nj, 0));
            }
            if (!ok && lane == 0) L.fail = 5;
            __syncthreads();
            if (L.n_hq > 0) {  // queued depth-limit subranges (<= kRefWaveLocal each): one wave each, in its buffer
                const int nq = min(L.n_hq, kRefMaxRanges);
                for (int q = wv; q < nq; q += kRefWaves) {
                    const uint32_t qlo = L.hq[2 * q], len = min(L.hq[2 * q + 1] - qlo, kRefWaveLocal);
                    for (uint32_t i = lane; i < len; i += kWave) E[i] = X[FD_REF_IDX(qlo + i, n, 19)];
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    ref_heapsort(E, static_cast<int>(len));
                    for (uint32_t i = lane; i < len; i += kWave) ord[FD_REF_IDX(qlo + i, n, 19)] = E[i].y;
                }
                if (tid == 0 && L.n_hq > kRefMaxRanges) L.fail = 7;
                __syncthreads();
                if (tid == 0) L.n_hq = 0;
            }
            if (tid == 0) L.n_wl = 0;
            FD_REF_MARK(23);  // wave-local ranges
            if (L.fail) break;
        }
        // ---- window final: greedy over [fin, fin_new) -------------------------------------------------
        const uint32_t fin = L.fin;
        const uint32_t fin_new = L.m_all > 0 ? L.r_lo[L.cur][0] : n;
        if (!grid_ready) {
            if (use_grid)
                for (int i = tid; i < cells; i += NT) grid[i] = grid_empty(rows, cols, d);
            grid_ready = true;
            __syncthreads();
        }
        for (uint32_t base = fin; base < fin_new && !r.order_only; base += kSelectChunk) {
            if (L.s_done) break;
            wrote = true;
            const int cn = static_cast<int>(min(static_cast<uint32_t>(kSelectChunk), fin_new - base));
            for (int i = tid; i < cn; i += NT) {
                uint32_t idx = ord[FD_REF_IDX(base + i, n, 18)];
                bool ok = true;
                if (idx >= npx) {  // consistency guard
                    ok = false;
                    idx = 0;
                    atomicOr(&a.status[f], 0x80000000u);
                }
                const uint32_t y = idx / static_cast<uint32_t>(cols), x = idx - y * static_cast<uint32_t>(cols);
                if (fmask) ok = ok && ((fmask[static_cast<int64_t>(y) * a.mask_wpr + (x >> 5)] >> (x & 31)) & 1u);
                L.pxy[i] = ok ? ((y << 16) | x) : kEmpty;
                if (use_grid) L.pcell[i] = (y / s1 + 1) * static_cast<uint32_t>(gw2) + (x / s1 + 1);
            }
            __syncthreads();
            {
                if (use_grid) conflict_masks(L.pxy, cn, d, rows, cols, L.cmask, tid, NT);
                __syncthreads();
                if (tid < kWave) {
                    if (!use_grid)
                        greedy_chunk<0>(a, f, cn, L.pxy, L.pcell, L.cmask, grid, gw2, prior, L.s_acc, L.s_done, false, nullptr,
                                        0u, 0u, L.tie_prev, L.tie_has_prev);
                    else if (grid_in_lds)
                        greedy_chunk<1>(a, f, cn, L.pxy, L.pcell, L.cmask, grid, gw2, prior, L.s_acc, L.s_done, false, nullptr,
                                        0u, 0u, L.tie_prev, L.tie_has_prev);
                    else
                        greedy_chunk<2>(a, f, cn, L.pxy, L.pcell, L.cmask, grid, gw2, prior, L.s_acc, L.s_done, false, nullptr,
                                        0u, 0u, L.tie_prev, L.tie_has_prev);
                }
            }
            __syncthreads();
        }
        FD_REF_MARK(21);  // greedy over the finished window
        FD_REF_COUNT(22, 1u);
        if (L.s_done || fin_new >= n) {
            finished = true;
            break;
        }
        if (wv == 0) {
            if (lane == 0) L.fin = fin_new;
            __builtin_amdgcn_s_waitcnt(0);
            set_active(L, fin_new + kSelectChunk);
        }
        __syncthreads();
    }
    __syncthreads();
    if (tid == 0) {
        if (!finished && !L.fail) L.fail = 8;  // the loop bound ran out
        if (L.fail) {
            // Device outputs of a failed frame: k_select's features (raster tie order) while no window
            // has been scanned; else the features the reference order accepted so far -- a prefix of the
            // reference's result, not a mix of the two orders. Host-output calls resolve it on the host.
            if (wrote) a.out_counts[f] = L.s_acc;
            atomicOr(&a.status[f], FD_FRAME_UNRESOLVED);
        } else {
            if (!r.order_only) a.out_counts[f] = L.s_acc;
            atomicOr(&a.status[f], FD_FRAME_RESOLVED);
        }
    }
}

// ---- wide prelude (frames of >= 1 Mpx) --------------------------------------------------------------
// One flagged 1080p frame holds ~10^5-10^6 candidates, and a single workgroup walks its push order and
// its first partition levels (the window's leftmost range [0, h) halves per level) through chains of
// memory round trips on one CU. The prelude spreads exactly that work over kRefWideGroups workgroups per
// frame, one kernel per step (the kernel boundary is the only cross-workgroup hand-off):
//   push: k_refw_init (state; the flagged frames into a compact list) -> k_refw_clear -> k_refw_bits (raster bitmap, global atomics) ->
//         k_refw_wcount (set bits per word slice) -> k_refw_wprefix (word prefix) -> k_refw_place
//         (X[rank] = candidate);
//   per level l while h > kRefWideMin: k_refw_lcount (pivot = median of X[1], X[h/2], X[h-1]; stopper
//         counts per block of [1, h)) -> k_refw_lscatter (stopper positions by rank) -> k_refw_lswap
//         (pairs with l_k < r_k swapped, the cut found where that stops holding, the pivot moved to 0).
// The pivot swap is applied virtually until k_refw_lswap (position ch reads the old X[0]), so no step
// writes what another workgroup of the same kernel reads. k_select_reference then starts from the state
// (RefCtl): range [0, h), the right children of the levels in position order, no push.
constexpr int kWT = 256;        // threads per prelude workgroup
constexpr int kWChunk = 8192;   // k_refw_lscatter: responses staged in LDS per chunk
constexpr int kWUnroll = 8;     // loads issued before use
constexpr uint32_t kNone = 0xFFFFFFFFu;

__device__ __forceinline__ bool wide_frame(const SelectArgs &a, int f) {
    const uint32_t st = a.status[f];
    return (st & FD_FRAME_TIES) && !(st & FD_FRAME_GUARD);
}

// [s, e) = workgroup g's share of [0, len) (blocks of ceil(len / G))
__device__ __forceinline__ void wide_share(uint32_t len, int g, uint32_t &s, uint32_t &e) {
    const uint32_t b = (len + kRefWideGroups - 1) / kRefWideGroups;
    s = min(len, static_cast<uint32_t>(g) * b);
    e = min(len, s + b);
}

// workgroup (kWT threads) sum; every thread gets it. ws: LDS [kWT / 64]
__device__ __forceinline__ uint32_t wg_sum(uint32_t v, uint32_t *ws) {
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t t = wave_incl_add(v);
    if (lane == kWave - 1) ws[w] = t;
    __syncthreads();
    uint32_t tot = 0;
#pragma unroll
    for (int i = 0; i < kWT / kWave; ++i) tot += ws[i];
    __syncthreads();
    return tot;
}

// workgroup exclusive prefix of v; total in tot. ws: LDS [kWT / 64]
__device__ __forceinline__ uint32_t wg_excl(uint32_t v, uint32_t *ws, uint32_t &tot) {
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_add(v);
    if (lane == kWave - 1) ws[w] = incl;
    __syncthreads();
    uint32_t wb = 0;
    tot = 0;
#pragma unroll
    for (int i = 0; i < kWT / kWave; ++i) {
        const uint32_t t = ws[i];
        wb += i < w ? t : 0u;
        tot += t;
    }
    __syncthreads();
    return wb + incl - v;
}

// one workgroup per frame: the state of a flagged frame, and the frame into the compact list the other
// prelude kernels walk (their grids cover min(batch, kRefWideSlots) frames x kRefWideGroups)
__global__ __launch_bounds__(kWT) void k_refw_init(SelectArgs a, RefSortArgs r) {
    const int f = blockIdx.x;
    if (!wide_frame(a, f) || threadIdx.x != 0) return;
    RefCtl &C = r.ctl[f];
    const uint32_t n = static_cast<uint32_t>(min(static_cast<int64_t>(a.cand_n[f]), a.list_cap));
    C.n = n;
    C.nlev = 0;
    C.bad = 0;
    C.h[0] = n;
    C.dep[0] = n > static_cast<uint32_t>(kRefLeaf) ? 2u * (31u - __clz(n)) : 0u;
    C.act[0] = n > kRefWideMin && C.dep[0] > 0u ? 1u : 0u;
    for (int l = 1; l <= kRefWideLevels; ++l) C.act[l] = 0u;
    const uint32_t j = atomicAdd(&r.wfr[0], 1u);
    r.wfr[1 + j] = static_cast<uint32_t>(f);
}

__device__ __forceinline__ void refw_clear(const SelectArgs &a, const RefSortArgs &r, int f, int g, int) {
    if (r.push_order) return;
    const uint32_t npx = static_cast<uint32_t>(a.rows) * static_cast<uint32_t>(a.cols);
    uint32_t s, e;
    wide_share((npx + 31u) >> 5, g, s, e);
    uint32_t *bits = r.lpos + static_cast<int64_t>(f) * r.cap;
    for (uint32_t w = s + threadIdx.x; w < e; w += kWT) bits[w] = 0u;
}

__device__ __forceinline__ void refw_bits(const SelectArgs &a, const RefSortArgs &r, int f, int g, int) {
    if (!wide_frame(a, f)) return;
    const uint32_t n = r.ctl[f].n;
    const uint32_t npx = static_cast<uint32_t>(a.rows) * static_cast<uint32_t>(a.cols);
    const float *lresp = a.list_resp + static_cast<int64_t>(f) * a.list_cap;
    const uint32_t *lidx = a.list_idx + static_cast<int64_t>(f) * a.list_cap;
    uint2 *X = r.x + static_cast<int64_t>(f) * r.cap;
    uint32_t *bits = r.lpos + static_cast<int64_t>(f) * r.cap;
    uint32_t s, e;
    wide_share(n, g, s, e);
    for (uint32_t i0 = s + threadIdx.x; i0 < e; i0 += kWUnroll * kWT) {
        uint32_t qv[kWUnroll];
        float rv[kWUnroll];
#pragma unroll
        for (int k = 0; k < kWUnroll; ++k) {
            const uint32_t i = min(i0 + k * kWT, e - 1u);
            qv[k] = lidx[i];
            rv[k] = r.push_order ? lresp[i] : 0.0f;
        }
#pragma unroll
        for (int k = 0; k < kWUnroll; ++k) {
            if (i0 + k * kWT >= e) continue;
            if (r.push_order) X[i0 + k * kWT] = make_uint2(__float_as_uint(rv[k]), qv[k]);
            else if (qv[k] < npx) atomicOr(&bits[qv[k] >> 5], 1u << (qv[k] & 31u));
        }
    }
}

__device__ __forceinline__ void refw_wcount(const SelectArgs &a, const RefSortArgs &r, int f, int g, int) {
    __shared__ uint32_t ws[kWT / kWave];
    if (!wide_frame(a, f) || r.push_order) return;
    const uint32_t npx = static_cast<uint32_t>(a.rows) * static_cast<uint32_t>(a.cols);
    const uint32_t *bits = r.lpos + static_cast<int64_t>(f) * r.cap;
    uint32_t s, e;
    wide_share((npx + 31u) >> 5, g, s, e);
    uint32_t cnt = 0;
    for (uint32_t w = s + threadIdx.x; w < e; w += kWT) cnt += __popc(bits[w]);
    const uint32_t tot = wg_sum(cnt, ws);
    if (threadIdx.x == 0) r.wcnt[(static_cast<int64_t>(f) * kRefWideGroups + g) * 2] = tot;
}

__device__ __forceinline__ void refw_wprefix(const SelectArgs &a, const RefSortArgs &r, int f, int g, int) {
    __shared__ uint32_t ws[kWT / kWave];
    if (!wide_frame(a, f) || r.push_order) return;
    const uint32_t npx = static_cast<uint32_t>(a.rows) * static_cast<uint32_t>(a.cols);
    const uint32_t *bits = r.lpos + static_cast<int64_t>(f) * r.cap;
    uint32_t *wpre = r.rpos + static_cast<int64_t>(f) * r.cap;
    uint32_t base = 0;
    for (int i = 0; i < g; ++i) base += r.wcnt[(static_cast<int64_t>(f) * kRefWideGroups + i) * 2];
    uint32_t s, e;
    wide_share((npx + 31u) >> 5, g, s, e);
    // a run of consecutive words per thread
    const uint32_t per = (e - s + kWT - 1) / kWT;
    const uint32_t w0 = min(e, s + threadIdx.x * per), w1 = min(e, w0 + per);
    uint32_t cnt = 0;
    for (uint32_t w = w0; w < w1; ++w) cnt += __popc(bits[w]);
    uint32_t tot;
    uint32_t at = base + wg_excl(cnt, ws, tot);
    for (uint32_t w = w0; w < w1; ++w) {
        wpre[w] = at;
        at += __popc(bits[w]);
    }
}

__device__ __forceinline__ void refw_place(const SelectArgs &a, const RefSortArgs &r, int f, int g, int) {
    if (!wide_frame(a, f) || r.push_order) return;
    const uint32_t n = r.ctl[f].n;
    const uint32_t npx = static_cast<uint32_t>(a.rows) * static_cast<uint32_t>(a.cols);
    const float *lresp = a.list_resp + static_cast<int64_t>(f) * a.list_cap;
    const uint32_t *lidx = a.list_idx + static_cast<int64_t>(f) * a.list_cap;
    uint2 *X = r.x + static_cast<int64_t>(f) * r.cap;
    const uint32_t *bits = r.lpos + static_cast<int64_t>(f) * r.cap;
    const uint32_t *wpre = r.rpos + static_cast<int64_t>(f) * r.cap;
    uint32_t s, e;
    wide_share(n, g, s, e);
    for (uint32_t i0 = s + threadIdx.x; i0 < e; i0 += kWUnroll * kWT) {
        uint32_t qv[kWUnroll], wp[kWUnroll], wb[kWUnroll];
        float rv[kWUnroll];
#pragma unroll
        for (int k = 0; k < kWUnroll; ++k) {
            const uint32_t i = min(i0 + k * kWT, e - 1u);
            qv[k] = lidx[i];
            rv[k] = lresp[i];
        }
#pragma unroll
        for (int k = 0; k < kWUnroll; ++k) {
            const uint32_t w = min(qv[k], npx - 1u) >> 5;
            wp[k] = wpre[w];
            wb[k] = bits[w];
        }
#pragma unroll
        for (int k = 0; k < kWUnroll; ++k) {
            const uint32_t q = qv[k];
            if (i0 + k * kWT >= e || q >= npx) continue;
            const uint32_t rk = wp[k] + __popc(wb[k] & ((1u << (q & 31u)) - 1u));
            if (rk < n) X[rk] = make_uint2(__float_as_uint(rv[k]), q);
        }
    }
}

// level l, step 1: the pivot, stopper counts of workgroup g's block of [1, h)
__device__ __forceinline__ void refw_lcount(const SelectArgs &a, const RefSortArgs &r, int f, int g, int l) {
    __shared__ uint32_t ws[kWT / kWave];
    if (!wide_frame(a, f)) return;
    RefCtl &C = r.ctl[f];
    if (!C.act[l]) return;
    const uint32_t h = C.h[l];
    const uint2 *X = r.x + static_cast<int64_t>(f) * r.cap;
    const uint32_t *Xr = reinterpret_cast<const uint32_t *>(X);
    const uint32_t mid = h / 2u;
    const uint2 xa = X[1], xb = X[mid], xc = X[h - 1u], x0 = X[0];
    const uint32_t ch = median_pos(as_f(xa.x), as_f(xb.x), as_f(xc.x), 1u, mid, h - 1u);
    const uint2 xch = ch == 1u ? xa : (ch == mid ? xb : xc);
    const float pv = as_f(xch.x);
    if (g == 0 && threadIdx.x == 0) {
        C.ch = ch;
        C.pv = xch.x;
        C.x0 = x0;
        C.xch = xch;
    }
    uint32_t s, e;
    wide_share(h - 1u, g, s, e);
    s += 1u;
    e += 1u;
    uint32_t cl = 0, cr = 0;
    for (uint32_t p0 = s + threadIdx.x; p0 < e; p0 += kWUnroll * kWT) {
        float rv[kWUnroll];
#pragma unroll
        for (int k = 0; k < kWUnroll; ++k) {
            const uint32_t p = min(p0 + k * kWT, e - 1u);
            rv[k] = p == ch ? as_f(x0.x) : as_f(Xr[2u * p]);
        }
#pragma unroll
        for (int k = 0; k < kWUnroll; ++k)
            if (p0 + k * kWT < e) {
                cl += rv[k] <= pv ? 1u : 0u;
                cr += rv[k] >= pv ? 1u : 0u;
            }
    }
    const uint32_t tl = wg_sum(cl, ws), tr = wg_sum(cr, ws);
    if (threadIdx.x == 0) {
        r.wcnt[(static_cast<int64_t>(f) * kRefWideGroups + g) * 2] = tl;
        r.wcnt[(static_cast<int64_t>(f) * kRefWideGroups + g) * 2 + 1] = tr;
    }
}

// level l, step 2: stopper positions by rank (left stoppers from the left into lpos, right stoppers from
// the right into rpos); the block is staged in LDS a chunk at a time and each thread ranks a run of it
__device__ __forceinline__ void refw_lscatter(const SelectArgs &a, const RefSortArgs &r, int f, int g, int l) {
    __shared__ uint32_t ws[kWT / kWave];
    __shared__ uint32_t sres[kWChunk];
    if (!wide_frame(a, f)) return;
    RefCtl &C = r.ctl[f];
    if (!C.act[l]) return;
    const uint32_t h = C.h[l], ch = C.ch, x0r = C.x0.x;
    const float pv = as_f(C.pv);
    const uint32_t *Xr = reinterpret_cast<const uint32_t *>(r.x + static_cast<int64_t>(f) * r.cap);
    uint32_t *lpos = r.lpos + static_cast<int64_t>(f) * r.cap;
    uint32_t *rpos = r.rpos + static_cast<int64_t>(f) * r.cap;
    // bases of this block, totals
    uint32_t bL = 0, bR = 0, nL = 0, nR = 0;
    for (int i = 0; i < kRefWideGroups; ++i) {
        const uint32_t vl = r.wcnt[(static_cast<int64_t>(f) * kRefWideGroups + i) * 2];
        const uint32_t vr = r.wcnt[(static_cast<int64_t>(f) * kRefWideGroups + i) * 2 + 1];
        bL += i < g ? vl : 0u;
        bR += i < g ? vr : 0u;
        nL += vl;
        nR += vr;
    }
    if (g == 0 && threadIdx.x == 0) {
        C.nL = nL;
        C.nR = nR;
    }
    uint32_t s, e;
    wide_share(h - 1u, g, s, e);
    s += 1u;
    e += 1u;
    for (uint32_t cs = s; cs < e; cs += kWChunk) {
        const uint32_t len = min(static_cast<uint32_t>(kWChunk), e - cs);
        for (uint32_t j0 = threadIdx.x; j0 < len; j0 += kWUnroll * kWT) {
            uint32_t v[kWUnroll];
#pragma unroll
            for (int k = 0; k < kWUnroll; ++k) {
                const uint32_t j = min(j0 + k * kWT, len - 1u);
                v[k] = cs + j == ch ? x0r : Xr[2u * (cs + j)];
            }
#pragma unroll
            for (int k = 0; k < kWUnroll; ++k)
                if (j0 + k * kWT < len) sres[j0 + k * kWT] = v[k];
        }
        __syncthreads();
        const uint32_t per = (len + kWT - 1) / kWT;
        const uint32_t j0 = min(len, threadIdx.x * per), j1 = min(len, j0 + per);
        uint32_t cl = 0, cr = 0;
        for (uint32_t j = j0; j < j1; ++j) {
            const float rv = as_f(sres[j]);
            cl += rv <= pv ? 1u : 0u;
            cr += rv >= pv ? 1u : 0u;
        }
        uint32_t tot;
        const uint32_t ex = wg_excl(cl | (cr << 16), ws, tot);  // (each field < 2^16: len <= 8192)
        uint32_t rl = bL + (ex & 0xFFFFu), rr = bR + (ex >> 16);
        for (uint32_t j = j0; j < j1; ++j) {
            const uint32_t p = cs + j;
            const float rv = as_f(sres[j]);
            const bool ls = rv <= pv, rs = rv >= pv;
            uint32_t kl = kNone, kr = kNone;
            if (ls) {
                kl = rl++;
                lpos[kl] = p;
            }
            if (rs) {
                kr = nR - 1u - rr++;
                rpos[kr] = p;
            }
            if (p == ch) {
                C.chL = kl;
                C.chR = kr;
            }
        }
        bL += tot & 0xFFFFu;
        bR += tot >> 16;
        __syncthreads();  // (sres reused by the next chunk)
    }
}

// level l, step 3: pairs k < K swapped (t_k = l_k < r_k holds exactly for k < K); the item where t
// stops holding gives K, the cut and the next level; workgroup 0 moves the pivot to position 0
__device__ __forceinline__ void refw_lswap(const SelectArgs &a, const RefSortArgs &r, int f, int g, int l) {
    if (!wide_frame(a, f)) return;
    RefCtl &C = r.ctl[f];
    if (!C.act[l]) return;
    const uint32_t h = C.h[l], ch = C.ch, nL = C.nL, nR = C.nR;
    const uint2 x0 = C.x0, xch = C.xch;
    const uint32_t mn = min(nL, nR);
    if (mn == 0u) {  // (cannot happen: the median of three leaves a stopper of each kind in [1, h))
        if (g == 0 && threadIdx.x == 0) C.bad = 1u;
        return;
    }
    uint2 *X = r.x + static_cast<int64_t>(f) * r.cap;
    const uint32_t *lpos = r.lpos + static_cast<int64_t>(f) * r.cap;
    const uint32_t *rpos = r.rpos + static_cast<int64_t>(f) * r.cap;
    uint32_t s, e;
    wide_share(mn + 1u, g, s, e);  // items k in [0, mn]
    for (uint32_t k0 = s + threadIdx.x; k0 < e; k0 += 4 * kWT) {
        uint32_t pl[4], pr[4], ql[4], qr[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t k = min(k0 + u * kWT, mn - 1u);
            const uint32_t kp = k0 + u * kWT == 0u ? 0u : min(k0 + u * kWT - 1u, mn - 1u);
            pl[u] = lpos[k];
            pr[u] = rpos[k];
            ql[u] = lpos[kp];
            qr[u] = rpos[kp];
        }
        bool t[4];
        uint2 vl[4], vr[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t k = k0 + u * kWT;
            t[u] = k < e && k < mn && pl[u] < pr[u];
            if (t[u]) {
                vl[u] = pl[u] == ch ? x0 : X[pl[u]];
                vr[u] = pr[u] == ch ? x0 : X[pr[u]];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t k = k0 + u * kWT;
            if (t[u]) {
                X[pl[u]] = vr[u];
                X[pr[u]] = vl[u];
            }
            const bool tp = k == 0u || ql[u] < qr[u];
            if (k < e && tp && !t[u]) {  // K = k
                uint32_t cut = k < nL ? lpos[k] : kNone;
                if (k >= 1u) cut = min(cut, qr[u]);
                const uint32_t d1 = C.dep[l] - 1u;
                if (cut == 0u || cut >= h) {  // (cannot happen: the scans stop inside the range)
                    C.bad = 1u;
                    cut = h;
                }
                C.sib_lo[l] = cut;
                C.sib_hi[l] = h;
                C.h[l + 1] = cut;
                C.dep[l + 1] = d1;
                C.act[l + 1] = l + 1 < kRefWideLevels && cut > kRefWideMin && d1 > 0u && !C.bad ? 1u : 0u;
                C.nlev = static_cast<uint32_t>(l + 1);
            }
        }
    }
    if (g == 0 && threadIdx.x == 0) {
        const uint32_t cl = C.chL, cr = C.chR;
        const bool swapped = (cl < mn && lpos[cl] < rpos[cl]) || (cr < mn && lpos[cr] < rpos[cr]);
        X[0] = xch;
        if (!swapped) X[ch] = x0;
    }
}

// the prelude kernels: workgroup (slot, g) takes flagged frames slot, slot + slots, ... of the list
#define FD_REFW_KERNEL(name)                                                                         \
    __global__ __launch_bounds__(kWT) void k_##name(SelectArgs a, RefSortArgs r, int l) {          \
        const int g = static_cast<int>(blockIdx.x % kRefWideGroups);                                \
        const uint32_t slots = gridDim.x / kRefWideGroups, cnt = r.wfr[0];                          \
        for (uint32_t j = blockIdx.x / kRefWideGroups; j < cnt; j += slots)                         \
            name(a, r, static_cast<int>(r.wfr[1 + j]), g, l);                                       \
    }
FD_REFW_KERNEL(refw_clear)
FD_REFW_KERNEL(refw_bits)
FD_REFW_KERNEL(refw_wcount)
FD_REFW_KERNEL(refw_wprefix)
FD_REFW_KERNEL(refw_place)
FD_REFW_KERNEL(refw_lcount)
FD_REFW_KERNEL(refw_lscatter)
FD_REFW_KERNEL(refw_lswap)
#undef FD_REFW_KERNEL

}  // namespace

hipError_t launch_select_reference(const SelectArgs &a, const RefSortArgs &r0, int batch, bool wide, hipStream_t s) {
    if (batch <= 0) return hipSuccess;
    RefSortArgs r = r0;
    r.wide = wide ? 1 : 0;
    if (wide) {
        const dim3 grid(static_cast<unsigned>(std::min(batch, kRefWideSlots)) * kRefWideGroups), blk(kWT);
        hipError_t e = hipMemsetAsync(r.wfr, 0, sizeof(uint32_t), s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_refw_init, dim3(static_cast<unsigned>(batch)), blk, 0, s, a, r);
        if (!r.push_order) hipLaunchKernelGGL(k_refw_clear, grid, blk, 0, s, a, r, 0);
        hipLaunchKernelGGL(k_refw_bits, grid, blk, 0, s, a, r, 0);
        if (!r.push_order) {
            hipLaunchKernelGGL(k_refw_wcount, grid, blk, 0, s, a, r, 0);
            hipLaunchKernelGGL(k_refw_wprefix, grid, blk, 0, s, a, r, 0);
            hipLaunchKernelGGL(k_refw_place, grid, blk, 0, s, a, r, 0);
        }
        for (int l = 0; l < kRefWideLevels; ++l) {
            hipLaunchKernelGGL(k_refw_lcount, grid, blk, 0, s, a, r, l);
            hipLaunchKernelGGL(k_refw_lscatter, grid, blk, 0, s, a, r, l);
            hipLaunchKernelGGL(k_refw_lswap, grid, blk, 0, s, a, r, l);
        }
    }
    hipLaunchKernelGGL(k_select_reference<kRefThreads>, dim3(static_cast<unsigned>(batch)), dim3(kRefThreads), 0, s, a, r);
    return hipGetLastError();
}

namespace {

// fd_lsd_lines' seed lists: frame f's compact run [frame_base[f], frame_base[f+1]) of (map index, norm)
// into the list format at [f * list_cap] (the scan order is the push order), the frame flagged for
// k_select_reference with its count.
__global__ __launch_bounds__(256) void k_lsd_seed_lists(const int64_t *frame_base, const int32_t *idx, const float *lnorm,
                                                        float *list_resp, uint32_t *list_idx, SelectArgs a) {
    const int f = blockIdx.y;
    const int64_t o = frame_base[f];
    const int64_t n = min(frame_base[f + 1] - o, a.list_cap);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.status[f] = FD_FRAME_TIES;
        a.cand_n[f] = static_cast<uint32_t>(n);
    }
    float *lr = list_resp + static_cast<int64_t>(f) * a.list_cap;
    uint32_t *li = list_idx + static_cast<int64_t>(f) * a.list_cap;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
        lr[i] = lnorm[o + i];
        li[i] = static_cast<uint32_t>(idx[o + i]);
    }
}

}  // namespace

hipError_t launch_lsd_seed_order(const int64_t *frame_base, const int32_t *idx, const float *lnorm, const SelectArgs &a,
                                 const RefSortArgs &r0, int batch, bool wide, hipStream_t s) {
    if (batch <= 0) return hipSuccess;
    // (the selection reads its lists through const pointers; these are the runtime's list buffers)
    hipLaunchKernelGGL(k_lsd_seed_lists, dim3(32, static_cast<unsigned>(batch)), dim3(256), 0, s, frame_base, idx, lnorm,
                       const_cast<float *>(a.list_resp), const_cast<uint32_t *>(a.list_idx), a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    RefSortArgs r = r0;
    r.push_order = 1;
    r.order_only = 1;
    return launch_select_reference(a, r, batch, wide, s);
}

}  // namespace fdk
