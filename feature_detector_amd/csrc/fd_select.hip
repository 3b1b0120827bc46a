// Per-frame greedy selection (SelectGoodFeatures, feature_point_detector.cpp:54-88) for gfx950,
// one 1024-thread workgroup per frame.
//
// The reference sorts every candidate by response (std::sort, :58-60) and walks the list, keeping a
// candidate unless an already kept feature lies within min_feature_distance (Chebyshev, :62-72),
// until `need` features exist (:67-69). Only the head of that order matters (640x480 noise: ~400
// of ~27k candidates), so the list is never sorted whole: a radix descent over 64-bit keys (level 0
// = the histogram the per-pixel kernel built while emitting) cuts it into chunks of
// <= kSelectChunk keys from the top, each gathered to LDS, cut into sub-chunks that are ordered
// and scanned in order by one wave in batches of 64 against an occupancy grid of (d+1)-sized cells
// (<= 1 kept feature per cell).
//
// The workgroup resets its frame's counters and histogram for the next call (no memset launches).
// Every data-dependent loop is bounded; an inconsistency trips a guard flag in the frame's status word
// (FD_FRAME_GUARD) that the host reports as an error instead of a hang or an out-of-bounds access.
// The status word also flags frames whose scan met equal responses (FD_FRAME_TIES); with
// FD_TIES_REFERENCE the host re-selects those in the reference's std::sort order (k_select_ordered).
#include "fd_device.h"
#include "fd_hip.h"
#include "fd_kernels.h"
#include "fd_gather.h"
#include "fd_greedy.h"

namespace fdk {

namespace {

// ---------------------------------------------------------------------------------------------------
// Per-frame greedy selection (SelectGoodFeatures, feature_point_detector.cpp:54-88).
// Candidates are visited in (response desc, raster index asc) order without a full sort: a radix
// descent over the 64-bit key sk = (orderable response bits << 32) | ~idx cuts the frame's list into
// consecutive chunks of <= kSelectChunk keys, each gathered into LDS, ordered (bucket placement or merge sort) and scanned by
// one wave. Accepted features live in an occupancy grid of (d+1)-sized cells: at most one accepted
// feature per cell, so a Chebyshev-distance test needs the 3x3 neighbouring cells only.
// ---------------------------------------------------------------------------------------------------
constexpr int kLevels = 8;
// digit widths per level: 12 (sign, exponent, 3 mantissa bits of the response), then 8 x 6, then 4
__device__ __forceinline__ int lvl_width(int l) { return l == 0 ? 12 : (l == 7 ? 4 : 8); }
__device__ __forceinline__ int lvl_top(int l) { return l == 7 ? 64 : 12 + 8 * l; }  // bits consumed through l

// Diagnostic phase clocks (only when a.stamps is set), accumulated by thread 0 in LDS (L.st) and
// written to a.stamps at the end: slot 15 keeps the last clock; FD_STAMP(k) adds the time since then
// to slot k. Slots 0, 4, 8, 9 are event counters (FD_COUNT).
#define FD_STAMP(slot)                                                                  \
    do {                                                                                \
        if (a.stamps && threadIdx.x == 0) {                                             \
            const uint64_t now_ = __builtin_readcyclecounter();                         \
            if ((slot) > 0 && (slot) != 4) L.st[(slot)] += now_ - L.st[15];             \
            L.st[15] = now_;                                                            \
        }                                                                               \
    } while (0)
#define FD_COUNT(slot, v)                                                               \
    do {                                                                                \
        if (a.stamps && threadIdx.x == 0) L.st[(slot)] += (v);                          \
    } while (0)

// n / d for quotients < 2^16 (every decode here: rows, cols, grid coordinates <= 65535) from the float
// reciprocal of d and one correction each way: the float estimate is within 2^16 * 2^-22 < 1 of n/d,
// so its truncation is off by at most one. (The integer division sequence costs ~30 instructions per
// division, three per decoded key.)
__device__ __forceinline__ uint32_t udiv16q(uint32_t n, uint32_t d, float rcp) {
    uint32_t q = static_cast<uint32_t>(static_cast<float>(n) * rcp);
    const int32_t r = static_cast<int32_t>(n - q * d);
    if (r < 0) --q;
    else if (r >= static_cast<int32_t>(d)) ++q;
    return q;
}

// Selection key of a candidate: the response through the frame's key map (order-preserving,
// injective on the candidates' response range; see SelectArgs::key_base), then ~idx so that equal
// responses order by ascending raster index.
__device__ __forceinline__ uint32_t map_key32(float resp, const SelectArgs &a) {
    return sel_key32(resp, a.key_base, a.key_lz);
}
// (tie_idx_desc: idx itself, so that equal responses order by descending raster index, the order in
// which SuperPoint's std::multimap is walked from crbegin, nn_feature_point_detector.cpp:144.)
__device__ __forceinline__ uint64_t make_key(float resp, uint32_t idx, const SelectArgs &a) {
    return sel_key64(resp, idx, a.key_base, a.key_lz, a.tie_idx_desc);
}

constexpr int kPassUnroll = 8;  // independent list loads in flight per thread
// Keys ordered per greedy sub-chunk: corner frames usually stop within the first few hundred; FAST's
// long scans drop most keys before ordering (grid prefilter), so there the whole superchunk is one
// sub-chunk (measured at 1280x720x64: 512 -> 190 us, 768 -> 166, 2048 -> 160; the 1080p list-mode
// corner selection prefers 512: 768 -> 78 us vs ~74).
constexpr int kSubChunk = 512;
constexpr int kSubChunkFast = kSelectChunk;
#ifndef FD_KO
#define FD_KO 0
#endif
// Phase-cost diagnostic builds only (-DFD_KO=mask; results are wrong): 1 = no greedy (the frame stops
// after its first sub-chunk), 2 = no conflict masks, 4 = no tie bits, 16 = place() without the
// position decode.
constexpr int kKnockOut = FD_KO;
#ifndef FD_EXIT
#define FD_EXIT 0
#endif
// Phase-cost diagnostic builds only (-DFD_EXIT=n; no outputs): k_select returns after phase n (1 the
// histogram scan and first cut, 2 the first gather, 3 the first sub-chunk's ordering), so that the
// differences of the kernel times are the phases' costs without clock stamps.
constexpr int kExitAt = FD_EXIT;
// FAST emission cut's margin (SelectArgs::cut_next): the proposal keeps max(FD_CUT_MUL x V, V + FD_CUT_ADD)
// emitted keys, V = the keys down to the lowest level-0 bin the frame's scan gathered
#ifndef FD_PICK_U
#define FD_PICK_U 2  // wide-scratch keys per thread in flight in wide_pick
#endif
#ifndef FD_CUT_MUL
#define FD_CUT_MUL 4
#endif
#ifndef FD_CUT_ADD
#define FD_CUT_ADD 4096
#endif
constexpr int kBucketMax = 64;  // largest bin of a sub-chunk ordered by bucket placement (else merge sort)
// k_select workgroup size (launch_select). Its phases are chains of dependent LDS operations per wave;
// with 256 threads (4x the items per wave) the headline frame's selection measured 1.3x slower.
constexpr int kSegPer = 2;  // sorted-segment entries per thread and round
constexpr int kRegGather = 16;  // list responses per thread and round in the level-0 gather

// Static LDS of the selection workgroup.
struct alignas(16) SelectLds {
    uint32_t suf0[kHistBins + 1];
    uint32_t sufl[kLevels - 1][257];
    uint64_t sup[kSelectChunk];  // superchunk keys (unsorted)
    // sub-chunk keys (merge-sorted between buf and tmp; buf later holds the conflict masks)
    uint64_t buf[kSelectChunk];
    uint64_t tmp[kSelectChunk];
    // sorted chunk, decoded: (y << 16) | x (kEmpty when a prior masks it) and occupancy-grid cell
    uint32_t pxy[kSelectChunk];
    uint32_t pcell[kSelectChunk];
    uint32_t pk32[kSelectChunk];  // 32-bit response keys in scan order (tie check)
    uint64_t tmask[kSelectChunk / kWave + 1];  // per 64-batch: bit l = candidate equals its predecessor
    uint32_t prev_min;                         // smallest 32-bit key of the previous sub-chunk (prefilter)
    int have_prev_min;
    alignas(16) uint32_t grid_lds[kGridLdsCells];  // (its tail holds the pipelined scan's ScanLds)
    uint32_t tie_prev;
    int tie_has_prev;
    uint64_t prefix[kLevels];
    int resume[kLevels];
    uint32_t wtot[16];
    uint32_t gcount;
    uint32_t seg_more[2];
    uint32_t lb_rng[2];  // local-digit bucket sort: the sub-chunk's smallest / largest 32-bit key
    int ff_res[2];  // first_le results (alternating slots)
    // placement votes (bucket / local-digit placement impossible), zero between sub-chunks: a store by
    // the voting threads and one barrier instead of __syncthreads_or (measured 858 vs 213 clocks at
    // 1024 threads, tools/calib/wg_probe.hip)
    uint32_t vote[2];
    int s_done, s_acc;
    uint64_t st[32];  // diagnostic phase clocks (a.stamps only); 16..31 free for ad-hoc probes
};

template <int NT, bool WIDE>
__device__ __forceinline__ void select_frame(const SelectArgs &a, const int f, SelectLds &L) {
    constexpr int kHistPerThread = kHistBins / NT;
    static_assert(kHistBins % NT == 0 && NT <= kSelectThreads, "histogram bins per thread");
    uint32_t(&suf0)[kHistBins + 1] = L.suf0;
    uint32_t(&sufl)[kLevels - 1][257] = L.sufl;
    uint64_t(&sup)[kSelectChunk] = L.sup;
    uint64_t(&buf)[kSelectChunk] = L.buf;
    uint64_t(&tmp)[kSelectChunk] = L.tmp;
    uint32_t(&pxy)[kSelectChunk] = L.pxy;
    uint32_t(&pcell)[kSelectChunk] = L.pcell;
    uint32_t(&grid_lds)[kGridLdsCells] = L.grid_lds;
    uint64_t(&prefix)[kLevels] = L.prefix;
    int(&resume)[kLevels] = L.resume;
    uint32_t(&wtot)[16] = L.wtot;
    uint32_t &gcount = L.gcount;
    int &s_done = L.s_done;
    int &s_acc = L.s_acc;
    const int tid = threadIdx.x, nthr = blockDim.x, lane = lane_id(), wave = tid >> 6;
    const int rows = a.rows, cols = a.cols;
    const int64_t n = min(static_cast<int64_t>(a.list_count[f]), a.list_cap);
    const float *lresp = a.list_resp + static_cast<int64_t>(f) * a.list_cap;
    const uint32_t *lidx = a.list_idx + static_cast<int64_t>(f) * a.list_cap;
    // List reads through buffer resources (list_cap < 2^30, checked on the host): a 32-bit byte offset
    // per thread plus a uniform one in an SGPR, instead of a 64-bit address per unrolled load (those were
    // hoisted out of the loops and spilled). Entries past the capacity read 0 (masked by i < n anyway).
    const auto rres = make_rsrc(lresp, static_cast<uint32_t>(a.list_cap) * 4u);
    const auto ridx = make_rsrc(lidx, static_cast<uint32_t>(a.list_cap) * 4u);
    // (the whole byte offset in the VGPR operand: the hardware range check covers the VGPR offset only,
    // an SGPR offset would be added after it, unchecked)
    auto lload = [](__amdgpu_buffer_rsrc_t r, uint32_t vbyte) -> uint32_t {
        return static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(r, static_cast<int>(vbyte), 0, 0));
    };
    const int d = a.dist;
    const bool use_grid = d >= 1 || (d == 0 && a.grid_at_d0);
    // Occupancy grid of (d+1)-sized cells with a one-cell border (no bounds checks in the scan).
    const int gw2 = a.grid_w + 2;
    const int cells = gw2 * (a.grid_h + 2);
    const bool grid_in_lds = cells <= kGridLdsCells;
    // the greedy's common case: LDS grid (with room for ScanLds in its tail) and packed coordinates
    // without an empty-cell test: the pipelined scan (greedy_scan beside scan_masks)
    const bool scan_fast = use_grid && grid_in_lds && cells <= kGridLdsCells - kScanLdsWords &&
                           grid_pk15(rows, cols, d) && nthr >= 2 * kWave;
    ScanLds &sl = *reinterpret_cast<ScanLds *>(&L.grid_lds[kGridLdsCells - kScanLdsWords]);
    static_assert((kGridLdsCells - kScanLdsWords) % 4 == 0, "ScanLds alignment");
    uint32_t *const grid_g = a.grid_global ? a.grid_global + static_cast<int64_t>(f) * cells : nullptr;
    const uint32_t prior = a.prior_counts ? static_cast<uint32_t>(a.prior_counts[f]) : 0u;
    const uint32_t *fmask = a.mask ? a.mask + static_cast<int64_t>(f) * rows * a.mask_wpr : nullptr;
    // k_wide_gather's key count (the previous kernel), loaded now: it lands during the histogram scan
    const uint32_t wide_pre_n = (WIDE && a.wide_count) ? a.wide_count[f] : 0xFFFFFFFFu;
    if (a.stamps && tid == 0)
        for (int i = 0; i < 32; ++i) L.st[i] = 0;
    FD_STAMP(0);
    // One memory round trip for everything the first phase needs: the level-0 histogram (accumulated
    // by the per-pixel kernel while it emitted the candidates) and the first round of the level-0
    // gather's list responses (clamped to the list capacity, not the count, so that these loads do
    // not wait for list_count; entries past the count are masked in the gather). Issued in this
    // order, waiting for the histogram leaves the list loads in flight.
    // The list loads go straight to LDS (global_load_lds: no VGPRs held across the histogram scan),
    // into the occupancy grid's space, which is initialised only after this first round is consumed.
    // (4 bins per thread: thread t loads bins 4t..4t+3 as one 16-byte load and forms the level-0
    // suffix sums from registers, below; other workgroup sizes load strided bins and go through LDS)
    constexpr bool kHist4 = kHistPerThread == 4;
    uint32_t hv[kHistPerThread];
    if constexpr (kHist4) {
        const uint4 h4 = reinterpret_cast<const uint4 *>(a.hist0 + static_cast<int64_t>(f) * kHistBins)[tid];
        hv[0] = h4.x;
        hv[1] = h4.y;
        hv[2] = h4.z;
        hv[3] = h4.w;
    } else {
#pragma unroll
        for (int j = 0; j < kHistPerThread; ++j) hv[j] = a.hist0[static_cast<int64_t>(f) * kHistBins + tid + j * NT];
    }
    float *const pre_lds = reinterpret_cast<float *>(grid_lds);
    static_assert(kRegGather * NT <= kGridLdsCells, "first gather round fits the grid's LDS");
    // sorted-segment mode: this frame's segment descriptors instead of the list prefetch
    const bool seg_mode = a.segdesc != nullptr;
    uint2 sd = make_uint2(0u, 0u);
    uint32_t seg_bad = 0;
    // (segment sg, slot j) of this thread in the sorted-segment gather, and its first two entries,
    // loaded now so that they land during the histogram scan
    const int segT = seg_mode ? max(1, nthr / a.nseg) : 1;
    const int seg_sg = tid / segT, seg_j = tid - seg_sg * segT;
    uint64_t pre_key[kSegPer] = {};
    if (seg_mode) {
        // unconditional (clamped) loads, so that nothing waits for them before their use
        const int sgc = min(seg_sg, a.nseg - 1);
        sd = a.segdesc[static_cast<int64_t>(f) * a.nseg + sgc];
        seg_bad = __hip_atomic_load(&a.seg_bad[f], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the first two entries of this thread, from the segment heads (entries past kSegHead or past
        // the segment's count are masked in seg_gather; the list is read there for them)
#pragma unroll
        for (int k = 0; k < kSegPer; ++k) {
            const int e = min(k * segT + seg_j, kSegHead - 1);
            pre_key[k] = a.seghead[(static_cast<int64_t>(f) * a.nseg + sgc) * kSegHead + e];
        }
    }
    // (not for a pre-gathered wide pass: its first chunk comes from the wide scratch)
    const bool list_prefetch = !a.pre_keys && !seg_mode && !(WIDE && a.wide_count);
    if (list_prefetch) {
        const uint32_t last = static_cast<uint32_t>(min(a.list_cap, static_cast<int64_t>(0xFFFFFFFF))) - 1u;
#pragma unroll
        for (int k = 0; k < kRegGather; ++k)
            __builtin_amdgcn_global_load_lds(lresp + min(static_cast<uint32_t>(tid + k * nthr), last),
                                             pre_lds + k * nthr + wave * kWave, 4, 0, 0);
    }

    if (use_grid && !grid_in_lds)
        for (int i = tid; i < cells; i += nthr) grid_g[i] = grid_empty(rows, cols, d);
    if (tid == 0) {
        s_done = 0;
        s_acc = 0;
        L.vote[0] = 0;
        L.vote[1] = 0;
        prefix[0] = 0;
        L.tie_prev = 0;
        L.tie_has_prev = 0;
        L.have_prev_min = 0;
        atomicExch(&a.status[f], 0u);  // (atomic: the flags below are atomicOr'ed)
        a.cand_n[f] = static_cast<uint32_t>(n);
        if (a.value_flag && (__hip_atomic_load(&a.pre_count[f], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 31))
            atomicOr(&a.status[f], FD_FRAME_VALUE_RANGE);  // candidate outside the key map
    }
    if (n == 0) {  // RETURN_TRUE_IF(candidates_.empty()) (:55)
        if (tid == 0) {
            a.out_counts[f] = 0;
            if (a.cut_next) {  // (FAST emission cut) candidates below the cut only: select again without it
                if (a.skipped[f]) atomicOr(&a.status[f], kFrameRedo);
                atomicMin(a.cut_next, 0u);
            }
        }
        return;
    }
    if (kExitAt == 9) return;  // (diagnostic: launch and prologue only)

    // In-place suffix sums of S[0..nb) by the whole block; S[nb] = 0.
    auto suffix = [&](uint32_t *S, int nb) {
        const int ch = (nb + nthr - 1) / nthr;  // contiguous bins per thread
        const int b0 = min(tid * ch, nb), b1 = min(b0 + ch, nb);
        uint32_t sacc = 0;
        for (int b = b0; b < b1; ++b) sacc += S[b];
        // suffix over threads: wave-level, then across the waves
        const uint32_t incl = wave_suffix_add(sacc);
        if (lane == 0) wtot[wave] = incl;
        __syncthreads();
        uint32_t after = 0;
        // the later waves' totals: one LDS read per lane and a wave sum (not a chain of up to 15 reads)
        after = wave_total_add((lane > wave && lane < nthr / kWave) ? wtot[lane] : 0u);
        uint32_t run = incl - sacc + after;
        for (int b = b1 - 1; b >= b0; --b) {  // (a thread's own bins: read before written)
            run += S[b];
            S[b] = run;
        }
        if (tid == 0) S[nb] = 0;
        __syncthreads();
    };
    // Smallest x in [lo_x, hi_x) with S[x] - base <= lim, or hi_x (S non-increasing: the predicate is a
    // step). All threads; each tests a contiguous run of bins and the one holding the step writes it:
    // two barriers instead of a dependent chain of ~12 LDS reads. Results alternate between two slots,
    // so a slot is rewritten only after every thread has passed the barrier that follows its read.
    int ff_parity = 0;
    auto first_le = [&](const uint32_t *S, int lo_x, int hi_x, uint32_t base, uint32_t lim) -> int {
        const int slot = ff_parity;
        ff_parity ^= 1;
        if (tid == 0) L.ff_res[slot] = hi_x;
        __syncthreads();
        const int n = hi_x - lo_x;
        const int per = (n + nthr - 1) / nthr;
        const int x0 = lo_x + tid * per, x1 = min(x0 + per, hi_x);
        if (x0 < x1 && !(x0 > lo_x && S[x0 - 1] - base <= lim)) {
            for (int x = x0; x < x1; ++x)
                if (S[x] - base <= lim) {
                    L.ff_res[slot] = x;
                    break;
                }
        }
        __syncthreads();
        return L.ff_res[slot];
    };
    // Wide scratch of the first list pass (see wide_gather below).
    // (WIDE = false: the code below folds away -- small frames in sorted-segment mode never need it,
    // and it would cost the hot small-frame path registers)
    uint64_t *const wk = (WIDE && a.wide_keys) ? a.wide_keys + static_cast<int64_t>(f) * kWideKeys : nullptr;
    int wide_lo = kHistBins, wide_hi = -1;  // level-0 bins [wide_lo, wide_hi] are in wk (when wide_n > 0)
    uint32_t wide_n = 0;
    auto in_wide = [&](uint64_t klo) {
        const int b = static_cast<int>(klo >> 52);
        return wide_n > 0 && b >= wide_lo && b <= wide_hi;
    };
    // Histogram of digit `lvl` (>= 1) over keys in [klo, khi] (one pass over the list).
    auto build = [&](int lvl, uint64_t klo, uint64_t khi, uint32_t *S) {
        const int nb = 1 << lvl_width(lvl);
        const int rem = 64 - lvl_top(lvl);
        for (int b = tid; b <= nb; b += nthr) S[b] = 0;
        __syncthreads();
        if (in_wide(klo)) {  // the bin's keys are all in the wide scratch
            for (uint32_t i = static_cast<uint32_t>(tid); i < wide_n; i += static_cast<uint32_t>(nthr)) {
                const uint64_t sk = wk[i];
                if (sk >= klo && sk <= khi) atomicAdd(&S[(sk >> rem) & static_cast<uint64_t>(nb - 1)], 1u);
            }
            __syncthreads();
            suffix(S, nb);
            return;
        }
        for (int64_t b0 = tid; b0 < n; b0 += static_cast<int64_t>(kPassUnroll) * nthr) {
            float r[kPassUnroll];
            uint32_t ix[kPassUnroll];
#pragma unroll
            for (int u = 0; u < kPassUnroll; ++u) {
                const uint32_t vb = 4u * static_cast<uint32_t>(b0 + static_cast<int64_t>(u) * nthr);
                r[u] = __uint_as_float(lload(rres, vb));
                ix[u] = lload(ridx, vb);
            }
#pragma unroll
            for (int u = 0; u < kPassUnroll; ++u) {
                const int64_t i = b0 + static_cast<int64_t>(u) * nthr;
                const uint64_t sk = make_key(r[u], ix[u], a);
                if (i < n && sk >= klo && sk <= khi) atomicAdd(&S[(sk >> rem) & static_cast<uint64_t>(nb - 1)], 1u);
            }
        }
        __syncthreads();
        suffix(S, nb);
    };
    auto suf = [&](int lvl) -> uint32_t * { return lvl == 0 ? suf0 : sufl[lvl - 1]; };

    if constexpr (kHist4) {
        // suffix(suf0, kHistBins) from the registers: no LDS round trip per bin, one 16-byte store
        FD_STAMP(1);
        const uint32_t sacc = hv[0] + hv[1] + hv[2] + hv[3];
        const uint32_t incl = wave_suffix_add(sacc);
        if (lane == 0) wtot[wave] = incl;
        __syncthreads();
        const uint32_t after = wave_total_add((lane > wave && lane < nthr / kWave) ? wtot[lane] : 0u);
        uint4 o;
        o.w = incl - sacc + after + hv[3];
        o.z = o.w + hv[2];
        o.y = o.z + hv[1];
        o.x = o.y + hv[0];
        reinterpret_cast<uint4 *>(suf0)[tid] = o;
        if (tid == 0) suf0[kHistBins] = 0;
        __syncthreads();
    } else {
        for (int j = 0; j < kHistPerThread; ++j) suf0[tid + j * NT] = hv[j];
        __syncthreads();
        FD_STAMP(1);
        suffix(suf0, kHistBins);
    }
    FD_STAMP(2);

    // Register-blocked gather of the keys whose 32-bit key lies in [k32lo, k32hi] (exact for chunks
    // cut at 32-bit key boundaries, e.g. level-0 bins): each thread tests kRegGather responses per
    // round, hits are placed by a block prefix and staged as (response, list index) in buf, then the
    // staged entries fetch their pixel index densely into sup. `pre` = this thread's first round,
    // already loaded. Sets gcount to the number of keys found.
    auto gather_exact = [&](uint32_t k32lo, uint32_t k32hi, const float *pre) {
        if (tid == 0) gcount = 0;
        __syncthreads();
        const uint32_t nn = static_cast<uint32_t>(n);  // list indices fit 32 bits (cap < 2^32)
        const uint32_t step = static_cast<uint32_t>(nthr);
        // One round: kRegGather responses per thread. Hits are packed densely into buf in no particular
        // order (the chunk is sorted afterwards): per k a ballot, the wave's total claimed with one LDS
        // atomic on gcount, each hit placed at that offset + the hits of lower lanes (mbcnt). No
        // barrier and no cross-lane scan inside a round.
        auto round = [&](const float (&rr)[kRegGather], uint32_t base) {
            uint32_t hm = 0;
#pragma unroll
            for (int k = 0; k < kRegGather; ++k) {
                const uint32_t k32 = map_key32(rr[k], a);
                const bool hit = base + tid + k * step < nn && k32 >= k32lo && k32 <= k32hi;
                hm |= static_cast<uint32_t>(hit) << k;
            }
            uint32_t wtotal = 0;
#pragma unroll
            for (int k = 0; k < kRegGather; ++k) wtotal += popc64(ballot((hm >> k) & 1u));
            if (wtotal == 0) return;
            uint32_t off = 0;
            if (lane == 0) off = atomicAdd(&gcount, wtotal);
            off = __builtin_amdgcn_readfirstlane(off);
#pragma unroll
            for (int k = 0; k < kRegGather; ++k) {
                const bool hit = (hm >> k) & 1u;
                const uint64_t m = ballot(hit);
                const uint32_t pos = static_cast<uint32_t>(mbcnt64(m, static_cast<int>(off)));
                if (hit && pos < static_cast<uint32_t>(kSelectChunk))
                    buf[pos] = (static_cast<uint64_t>(__float_as_uint(rr[k])) << 32) | (base + tid + k * step);
                off += popc64(m);
            }
        };
        uint32_t base = 0;
        if (pre) {
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this thread's LDS-direct loads have landed
            float rr[kRegGather];
#pragma unroll
            for (int k = 0; k < kRegGather; ++k) rr[k] = pre[tid + k * step];
            round(rr, 0);
            base = kRegGather * step;
        }
        for (; base < nn; base += kRegGather * step) {
            float rr[kRegGather];
#pragma unroll
            for (int k = 0; k < kRegGather; ++k) rr[k] = __uint_as_float(lload(rres, 4u * (base + tid + k * step)));
            round(rr, base);
        }
        __syncthreads();
        const uint32_t staged = gcount;
        const int ns = min(static_cast<int>(staged), kSelectChunk);
        for (int j = tid; j < ns; j += nthr) {
            const uint64_t e = buf[j];
            const uint32_t li = lload(ridx, 4u * static_cast<uint32_t>(e));
            sup[j] = make_key(__uint_as_float(static_cast<uint32_t>(e >> 32)), li, a);
        }
        __syncthreads();  // sup complete; gcount read by every thread before anyone reuses it
    };

    // Wide first pass (SelectArgs::wide_keys): the list pass that gathers the first chunk collects every
    // key of the top level-0 bins holding <= kWideKeys candidates into the frame's global scratch, so
    // that later chunks (and descents) inside those bins scan that scratch instead of the whole list:
    // one pass over the list instead of one per chunk (FAST on noise visits ~5k candidates of ~265k,
    // 3 chunks: 3 list passes of ~90k cycles each by this one workgroup before).
    auto wide_gather = [&](uint32_t k32lo, uint32_t k32hi) {
        if (tid == 0) gcount = 0;
        __syncthreads();
        const uint32_t nn = static_cast<uint32_t>(n);
        const uint32_t step = static_cast<uint32_t>(nthr);
        constexpr int kWideReg = 8;  // (half of gather_exact's round: the pass is not latency-critical)
        for (uint32_t base = 0; base < nn; base += kWideReg * step) {
            float rr[kWideReg];
#pragma unroll
            for (int k = 0; k < kWideReg; ++k) rr[k] = __uint_as_float(lload(rres, 4u * (base + tid + k * step)));
            uint32_t hm = 0;
#pragma unroll
            for (int k = 0; k < kWideReg; ++k) {
                const uint32_t k32 = map_key32(rr[k], a);
                hm |= static_cast<uint32_t>(base + tid + k * step < nn && k32 >= k32lo && k32 <= k32hi) << k;
            }
            uint32_t wtotal = 0;
#pragma unroll
            for (int k = 0; k < kWideReg; ++k) wtotal += popc64(ballot((hm >> k) & 1u));
            if (wtotal == 0) continue;
            uint32_t off = 0;
            if (lane == 0) off = atomicAdd(&gcount, wtotal);
            off = __builtin_amdgcn_readfirstlane(off);
#pragma unroll
            for (int k = 0; k < kWideReg; ++k) {
                const bool hit = (hm >> k) & 1u;
                const uint64_t m = ballot(hit);
                const uint32_t pos = static_cast<uint32_t>(mbcnt64(m, static_cast<int>(off)));
                if (hit && pos < static_cast<uint32_t>(kWideKeys))  // (response, list index); keyed below
                    wk[pos] = (static_cast<uint64_t>(__float_as_uint(rr[k])) << 32) | (base + tid + k * step);
                off += popc64(m);
            }
        }
        // staged entries -> selection keys: pixel indices fetched a few at a time per thread (independent
        // loads), not per hit inside the pass
        __threadfence_block();  // the scratch is read back by other threads of this workgroup
        __syncthreads();
        const uint32_t staged = min(gcount, static_cast<uint32_t>(kWideKeys));
        constexpr int kPer = 2;
        for (uint32_t i0 = static_cast<uint32_t>(tid); i0 < staged; i0 += kPer * step) {
            uint64_t e[kPer];
            uint32_t li[kPer];
#pragma unroll
            for (int k = 0; k < kPer; ++k) e[k] = i0 + k * step < staged ? wk[i0 + k * step] : 0ull;
#pragma unroll
            for (int k = 0; k < kPer; ++k) li[k] = lload(ridx, 4u * static_cast<uint32_t>(e[k]));
#pragma unroll
            for (int k = 0; k < kPer; ++k)
                if (i0 + k * step < staged)
                    wk[i0 + k * step] = make_key(__uint_as_float(static_cast<uint32_t>(e[k] >> 32)), li[k], a);
        }
        __threadfence_block();
        __syncthreads();
    };
    // Keys of wk in [klo, khi] into sup (unordered); gcount = their number.
    auto wide_pick = [&](uint64_t klo, uint64_t khi) {
        if (tid == 0) gcount = 0;
        __syncthreads();
        // kPickU keys per thread loaded before any is used: one memory round trip per kPickU x 1024 keys
        // (all 8 at once spill registers in this instance)
        constexpr int kPickU = FD_PICK_U;
        for (uint32_t i0 = static_cast<uint32_t>(wave) * kWave; i0 < wide_n; i0 += static_cast<uint32_t>(kPickU * nthr)) {
            uint64_t kv[kPickU];
#pragma unroll
            for (int u = 0; u < kPickU; ++u) {
                const uint32_t i = i0 + u * nthr + lane;
                kv[u] = i < wide_n ? wk[i] : 0ull;
            }
#pragma unroll
            for (int u = 0; u < kPickU; ++u) {
                const uint32_t i = i0 + u * nthr + lane;
                const uint64_t key = kv[u];
                const bool hit = i < wide_n && key >= klo && key <= khi;
                const uint64_t m = ballot(hit);
                if (m) {
                    uint32_t off = 0;
                    if (lane == 0) off = atomicAdd(&gcount, static_cast<uint32_t>(popc64(m)));
                    off = __builtin_amdgcn_readfirstlane(off);
                    const uint32_t pos = static_cast<uint32_t>(mbcnt64(m, static_cast<int>(off)));
                    if (hit && pos < static_cast<uint32_t>(kSelectChunk)) sup[pos] = key;
                }
            }
        }
        __syncthreads();
    };
    // Level-0 bins at and below `hi` (the highest not yet visited), as many as hold <= kWideKeys keys,
    // gathered in one list pass -- done at the first list pass the scan needs after its first chunk
    // (a frame that finishes within the first chunk never pays for it).
    auto ensure_wide = [&](int hi_bin) {
        if (!wk || wide_n > 0) return;
        const int wl = first_le(suf0, 0, hi_bin + 1, suf0[hi_bin + 1], static_cast<uint32_t>(kWideKeys));
        if (wl > hi_bin) return;  // the bin alone holds more than kWideKeys keys
        const uint32_t k32hi = hi_bin == kHistBins - 1 ? 0xFFFFFFFFu : (static_cast<uint32_t>(hi_bin + 1) << 20) - 1u;
        const uint32_t expect = suf0[wl] - suf0[hi_bin + 1];
        // k_wide_gather took the same cut from the same histogram (the top bins holding <= kWideKeys
        // keys) and already holds them in wk; a different count means it did not (e.g. the top bin alone
        // exceeds kWideKeys there): this workgroup makes the pass itself
        if (!(hi_bin == kHistBins - 1 && wide_pre_n == expect)) {
            wide_gather(static_cast<uint32_t>(wl) << 20, k32hi);
            if (tid == 0 && gcount != expect)  // consistency guard: gathered == histogram count
                atomicOr(&a.status[f], 0x04000000u);
        }
        wide_lo = wl;
        wide_hi = hi_bin;
        wide_n = min(expect, static_cast<uint32_t>(kWideKeys));
    };

    // First chunk from the sorted segments (PointsArgs::segdesc): every workgroup segment of the list
    // is ordered by level-0 bin, descending, so the keys of bins >= lo are a prefix of each segment.
    // T threads per segment read its entries T at a time while the last one read is still >= lo.
    auto seg_gather = [&](int lo, uint32_t k32hi) {  // keys of level-0 bins [lo, k32hi >> 20]
        if (tid == 0) {
            gcount = 0;
            L.seg_more[0] = 0;
            L.seg_more[1] = 0;
        }
        __syncthreads();
        FD_STAMP(25);
        const uint32_t k32lo = static_cast<uint32_t>(lo) << 20;
        for (int r = 0;; ++r) {
            bool more = false;
            bool hit[kSegPer] = {}, ge[kSegPer] = {};
            uint64_t kv[kSegPer];
#pragma unroll
            for (int k = 0; k < kSegPer; ++k) {
                const uint32_t e = static_cast<uint32_t>((kSegPer * r + k) * segT + seg_j);
                const bool in = seg_sg < a.nseg && e < sd.y && static_cast<int64_t>(sd.x) + e < a.list_cap;
                if (r == 0 && e < static_cast<uint32_t>(kSegHead)) {
                    kv[k] = pre_key[k];
                } else {
                    const uint32_t lb = 4u * (sd.x + e);
                    const uint64_t key = make_key(__uint_as_float(lload(rres, lb)), lload(ridx, lb), a);
                    kv[k] = in ? key : 0ull;
                }
                ge[k] = in && static_cast<uint32_t>(kv[k] >> 32) >= k32lo;
                hit[k] = ge[k] && static_cast<uint32_t>(kv[k] >> 32) <= k32hi;  // (later chunks: skip earlier ones)
            }
            more = ge[kSegPer - 1] && seg_j == segT - 1;
            // one LDS reservation per wave and round for all kSegPer slots
            uint64_t bm[kSegPer];
            uint32_t wtotal = 0;
#pragma unroll
            for (int k = 0; k < kSegPer; ++k) {
                bm[k] = ballot(hit[k]);
                wtotal += popc64(bm[k]);
            }
            if (wtotal) {
                uint32_t off = 0;
                if (lane == 0) off = atomicAdd(&gcount, wtotal);
                off = __builtin_amdgcn_readfirstlane(off);
#pragma unroll
                for (int k = 0; k < kSegPer; ++k) {
                    const uint32_t pos = static_cast<uint32_t>(mbcnt64(bm[k], static_cast<int>(off)));
                    if (hit[k] && pos < static_cast<uint32_t>(kSelectChunk)) sup[pos] = kv[k];
                    off += popc64(bm[k]);
                }
            }
            FD_STAMP(23);
            // one barrier per round: waves whose last slot still hits raise this round's flag
            // (alternating words: the one cleared here was last read before the previous barrier)
            if (tid == 0) L.seg_more[(r + 1) & 1] = 0;
            if (ballot(more) != 0ull && lane == 0) L.seg_more[r & 1] = 1;
            __syncthreads();
            FD_STAMP(24);
            if (L.seg_more[r & 1] == 0) break;
            if (r > kSelectChunk) {  // consistency guard (sorted prefixes hold <= kSelectChunk keys)
                if (tid == 0) atomicOr(&a.status[f], 0x04000000u);
                break;
            }
        }
        __syncthreads();
    };

    // The first level-0 chunk (the loop's first cut: the highest bins holding <= kSelectChunk keys),
    // gathered here so that the prefetched responses die before the sort and greedy code.
    bool first_ready = false;
    int first_lo = -1;  // the first chunk's cut (the main loop's first search, done here already)
    {
        // Sorted-segment frames (small, corner detectors) cut the first chunk at one sub-chunk: it is
        // then ordered in place (no sub-chunk extract), and frames whose greedy runs past it take the
        // next chunk through the main loop's list pass. FD_FIRST_SUB=0: the old cut (A/B).
        int lo_b = kHistBins;
        if (!WIDE && seg_mode && a.first_sub) lo_b = first_le(suf0, 0, kHistBins, 0u, static_cast<uint32_t>(kSubChunk));
        if (lo_b >= kHistBins)  // (or the top bin alone exceeds a sub-chunk)
            lo_b = first_le(suf0, 0, kHistBins, 0u, static_cast<uint32_t>(kSelectChunk));
        first_lo = lo_b;
        FD_STAMP(21);
        if (kExitAt == 1) return;
        if (lo_b < kHistBins && suf0[lo_b] > 0) {
            const uint32_t want = suf0[lo_b];
            if (a.pre_keys && a.pre_count[f] == want) {  // k_gather's result (previous kernel)
                const uint64_t *pk = a.pre_keys + static_cast<int64_t>(f) * kSelectChunk;
                for (int i = tid; i < static_cast<int>(want); i += nthr) sup[i] = pk[i];
                if (tid == 0) gcount = want;
                __syncthreads();
            } else if (seg_mode && seg_bad == 0) {
                seg_gather(lo_b, 0xFFFFFFFFu);
            } else if (wk && a.wide_eager) {
                // long scans expected (FAST: scores plus a slowly growing offset crowd the top bins):
                // the first list pass already collects the bins below the first chunk
                ensure_wide(kHistBins - 1);
                if (wide_n > 0 && wide_lo <= lo_b) {
                    wide_pick(static_cast<uint64_t>(lo_b) << 52, ~0ull);
                } else {
                    gather_exact(static_cast<uint32_t>(lo_b) << 20, 0xFFFFFFFFu, nullptr);
                }
            } else {
                if (a.pre_keys && tid == 0)  // consistency guard: k_gather saw a different cut
                    atomicOr(&a.status[f], 0x02000000u);
                gather_exact(static_cast<uint32_t>(lo_b) << 20, 0xFFFFFFFFu, list_prefetch ? pre_lds : nullptr);
            }
            first_ready = true;
        }
    }
    FD_STAMP(22);
    if (kExitAt == 2) return;
    if (use_grid && grid_in_lds) {  // the first round's LDS-direct loads are consumed (or never used)
        // vmcnt(0): no load still landing in this space (only if they were issued: the wait would
        // also hold for this thread's outstanding global stores and atomics, a memory round trip)
        if (list_prefetch) __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();
        for (int i = tid; i < cells; i += nthr) grid_lds[i] = grid_empty(rows, cols, d);
        __syncthreads();
    }
    FD_STAMP(3);
    if (kExitAt == 4) return;
    int level = 0;
    int hi = (1 << lvl_width(0)) - 1;
    for (int64_t iter = 0;; ++iter) {
        if (s_done) break;
        if (iter > 4 * n + 64) {  // every iteration retires a bin or descends; guards inconsistent input
            if (tid == 0) atomicOr(&a.status[f], 0x10000000u);
            break;
        }
        if (hi < 0) {
            if (level == 0) break;
            --level;
            hi = resume[level];
            continue;
        }
        const uint32_t *S = suf(level);
        const uint32_t base = S[hi + 1];
        // (sorted-segment corner frames: chunks of one sub-chunk, each a cheap segment-prefix gather)
        const uint32_t lim = static_cast<uint32_t>((!WIDE && seg_mode && a.first_sub && seg_bad == 0 && level == 0)
                                                       ? kSubChunk : kSelectChunk);
        // smallest lo in [0, hi] with S[lo] - base <= lim (S is non-increasing in b)
        // (level 0, top of the histogram: the cut computed for the first chunk above)
        int lo = (level == 0 && hi == kHistBins - 1 && first_lo >= 0) ? first_lo : first_le(S, 0, hi + 1, base, lim);
        const int w = lvl_width(level);
        const int rem = 64 - lvl_top(level);
        const uint64_t pre = prefix[level];
        if (lo > hi && level + 1 >= kLevels) {  // keys are unique: impossible with consistent input
            if (tid == 0) atomicOr(&a.status[f], 0x08000000u);
            break;
        }
        if (lo > hi) {  // bin `hi` alone exceeds a chunk: descend into it
            __syncthreads();
            if (tid == 0) {
                resume[level] = hi - 1;
                prefix[level + 1] = (pre << w) | static_cast<uint64_t>(hi);
            }
            __syncthreads();
            const uint64_t klo = ((pre << w) | static_cast<uint64_t>(hi)) << rem;
            const uint64_t khi = klo | ((1ull << rem) - 1ull);
            const uint32_t expect = S[hi] - S[hi + 1];
            if (level == 0) ensure_wide(hi);
            ++level;
            FD_COUNT(9, 1);
            FD_STAMP(7);
            build(level, klo, khi, suf(level));
            if (tid == 0 && suf(level)[0] != expect)  // consistency guard: descent histogram == parent bin
                atomicOr(&a.status[f], 0x02000000u);
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
            const bool k32_exact = rem >= 32;  // [klo, khi] == all keys whose top 32 bits are in [k32lo, k32hi]
            // gather the chunk: wave-uniform loop bounds, one LDS atomic per wave per round
            if (tid == 0) gcount = 0;
            __syncthreads();
            if (first_ready && level == 0) {  // gathered before the loop (sup holds it)
                first_ready = false;
                if (tid == 0) gcount = cnt;
            } else if (!WIDE && seg_mode && seg_bad == 0 && level == 0 && !a.pre_keys) {
                seg_gather(lo, k32hi);  // a later level-0 chunk: from the sorted segments' prefixes
            } else if (level == 0 && (ensure_wide(hi), in_wide(klo))) {
                wide_pick(klo, khi);
            } else if (in_wide(klo)) {
                wide_pick(klo, khi);
            } else if (k32_exact) {
                gather_exact(k32lo, k32hi, nullptr);
            } else
            for (int64_t b0 = static_cast<int64_t>(wave) * kWave; b0 < n;
                 b0 += static_cast<int64_t>(kPassUnroll) * nthr) {
                float r[kPassUnroll];
                uint32_t ix[kPassUnroll];
#pragma unroll
                for (int u = 0; u < kPassUnroll; ++u) {  // unconditional loads: all in flight
                    const uint32_t vb = 4u * static_cast<uint32_t>(b0 + static_cast<int64_t>(u) * nthr + lane);
                    r[u] = __uint_as_float(lload(rres, vb));
                    ix[u] = lload(ridx, vb);
                }
#pragma unroll
                for (int u = 0; u < kPassUnroll; ++u) {
                    const int64_t i = b0 + static_cast<int64_t>(u) * nthr + lane;
                    const uint32_t k32 = map_key32(r[u], a);
                    const bool near = i < n && k32 >= k32lo && k32 <= k32hi;  // 32-bit prefilter
                    const uint64_t sk = make_key(r[u], ix[u], a);
                    bool hit = near;
                    if (!k32_exact) {  // chunk bounds inside the 32-bit key: full 64-bit test
                        if (ballot(near) == 0ull) continue;
                        hit = near && sk >= klo && sk <= khi;
                    }
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
            if (tid == 0 && gcount != cnt)  // consistency guard: gathered == histogram count
                atomicOr(&a.status[f], 0x04000000u);
            FD_STAMP(3);  // gather
            const uint32_t s1 = static_cast<uint32_t>(d + 1);
            const float rcp_cols = 1.0f / static_cast<float>(cols), rcp_s1 = 1.0f / static_cast<float>(s1);
            auto place = [&](int pos, uint64_t sk) {  // decode position, prior mask, grid cell
                if (kKnockOut & 16) {  // (diagnostic build: keys only)
                    pxy[pos] = static_cast<uint32_t>(sk) & 0x00FF00FFu;
                    L.pk32[pos] = static_cast<uint32_t>(sk >> 32);
                    pcell[pos] = static_cast<uint32_t>(gw2 + 1);
                    return;
                }
                uint32_t idx = a.tie_idx_desc ? static_cast<uint32_t>(sk) : ~static_cast<uint32_t>(sk);
                bool ok = true;
                if (idx >= static_cast<uint32_t>(rows) * static_cast<uint32_t>(cols)) {  // consistency guard
                    ok = false;
                    idx = 0;
                    atomicOr(&a.status[f], 0x80000000u);
                }
                const uint32_t y = udiv16q(idx, static_cast<uint32_t>(cols), rcp_cols);
                const uint32_t x = idx - y * static_cast<uint32_t>(cols);
                if (fmask) ok = (fmask[static_cast<int64_t>(y) * a.mask_wpr + (x >> 5)] >> (x & 31)) & 1u;
                pxy[pos] = ok ? ((y << 16) | x) : kEmpty;
                L.pk32[pos] = static_cast<uint32_t>(sk >> 32);
                if (use_grid)
                    pcell[pos] = (udiv16q(y, s1, rcp_s1) + 1) * static_cast<uint32_t>(gw2) + (udiv16q(x, s1, rcp_s1) + 1);
            };
            // Sub-chunks of <= kSubChunk keys from the top bins of the superchunk (already in LDS):
            const uint32_t sub_lim = static_cast<uint32_t>((WIDE && (a.wide_eager || a.fast_sub)) ? kSubChunkFast : kSubChunk);
            // the greedy usually stops within the first few hundred keys.
            int shi = hi;
            while (shi >= lo && !s_done) {
                const uint32_t sbase = S[shi + 1];
                // (the whole remaining range fits a sub-chunk: no search)
                const int q0 = S[lo] - sbase <= sub_lim ? lo : first_le(S, lo, shi + 1, sbase, sub_lim);
                const int slo = min(q0, shi);  // one bin larger than a sub-chunk is taken whole
                const uint32_t sc = S[slo] - sbase;
                if (sc > 0) {
                    FD_COUNT(0, 1);  // diagnostics: sub-chunk count and total keys
                    FD_COUNT(4, sc);
                    const uint64_t sklo = ((pre << w) | static_cast<uint64_t>(slo)) << rem;
                    const uint64_t skhi = (((pre << w) | static_cast<uint64_t>(shi)) << rem) | ((1ull << rem) - 1ull);
                    // the sub-chunk's unsorted keys: the whole chunk in place, or extracted into buf
                    const bool whole = sc == cnt;
                    uint64_t *unsorted = whole ? sup : buf;
                    if (!whole) {
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
                    }
                    FD_STAMP(10);  // sub-chunk extract
                    // Once the grid holds features (earlier sub-chunks, priors), the keys it already
                    // rules out -- and those the prior mask rejects -- are dropped before the ordering:
                    // the reference rejects them whenever it visits them (their blocking feature has a
                    // strictly larger response, or the mask), so they never change the result and their
                    // place among equal responses does not matter. The one exception, a chain of equal
                    // responses across the sub-chunk boundary, is flagged as a tie (sc_max / prev_min).
                    // The ordering then takes the merge path (the level's suffix counts no longer
                    // describe the kept keys). WIDE instance only (FAST, list mode).
                    int c_sort = static_cast<int>(sc);
                    uint64_t *keys = unsorted;
                    bool filtered = false;
                    if (WIDE && use_grid && (s_acc > 0 || prior > 0)) {
                        uint64_t *const kbuf = reinterpret_cast<uint64_t *>(pxy);  // pxy + pcell: free until placed
                        static_assert(sizeof(L.pxy) + sizeof(L.pcell) >= kSelectChunk * sizeof(uint64_t), "kbuf");
                        const bool pk16 = rows + 3 * d < 65536 && cols + 3 * d < 65536;
                        const uint32_t w2 = 2u * static_cast<uint32_t>(d);
                        if (tid == 0) {
                            gcount = 0;
                            L.seg_more[0] = 0u;
                            L.seg_more[1] = 0xFFFFFFFFu;
                        }
                        __syncthreads();
                        uint32_t kmax = 0u, kmin = 0xFFFFFFFFu;
                        for (int b0 = wave * kWave; b0 < c_sort; b0 += nthr) {
                            const int i = b0 + lane;
                            const uint64_t sk = i < c_sort ? unsorted[i] : 0ull;
                            bool keep = false;
                            if (i < c_sort) {
                                const uint32_t k32 = static_cast<uint32_t>(sk >> 32);
                                kmax = max(kmax, k32);
                                kmin = min(kmin, k32);
                                const uint32_t idx = a.tie_idx_desc ? static_cast<uint32_t>(sk) : ~static_cast<uint32_t>(sk);
                                keep = true;  // (an out-of-range index is kept: place() raises its guard)
                                if (idx < static_cast<uint32_t>(rows) * static_cast<uint32_t>(cols)) {
                                    const uint32_t y = udiv16q(idx, static_cast<uint32_t>(cols), rcp_cols);
                                    const uint32_t x = idx - y * static_cast<uint32_t>(cols);
                                    if (fmask && !((fmask[static_cast<int64_t>(y) * a.mask_wpr + (x >> 5)] >> (x & 31)) & 1u))
                                        keep = false;
                                    const int cell = static_cast<int>((udiv16q(y, s1, rcp_s1) + 1) * static_cast<uint32_t>(gw2) +
                                                                      (udiv16q(x, s1, rcp_s1) + 1));
                                    const uint32_t e = (y << 16) | x;
                                    const u16x2 base = __builtin_bit_cast(u16x2, e) - static_cast<uint16_t>(d);
                                    if (grid_in_lds && grid_pk15(rows, cols, d)) {  // as greedy_chunk's grid test
                                        uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
                                        for (int q = 0; q < 9; ++q) {
                                            const u16x2 dt = __builtin_bit_cast(u16x2, grid_lds[cell + (q / 3 - 1) * gw2 + (q % 3 - 1)]) - base;
                                            mn = min(mn, static_cast<uint32_t>(dt.x > dt.y ? dt.x : dt.y));
                                        }
                                        if (mn <= w2) keep = false;
                                    } else
#pragma unroll
                                    for (int q = 0; q < 9; ++q) {
                                        const int o = cell + (q / 3 - 1) * gw2 + (q % 3 - 1);
                                        const uint32_t g = grid_in_lds ? grid_lds[o]
                                                                       : __hip_atomic_load(&grid_g[o], __ATOMIC_RELAXED,
                                                                                           __HIP_MEMORY_SCOPE_AGENT);
                                        if (g == grid_empty(rows, cols, d)) continue;
                                        if (pk16) {
                                            const u16x2 dt = __builtin_bit_cast(u16x2, g) - base;
                                            if ((dt.x > dt.y ? dt.x : dt.y) <= w2) keep = false;
                                        } else if (abs(static_cast<int>(x) - static_cast<int>(g & 0xFFFFu)) <= d &&
                                                   abs(static_cast<int>(y) - static_cast<int>(g >> 16)) <= d) {
                                            keep = false;
                                        }
                                    }
                                }
                            }
                            const uint64_t m = ballot(keep);
                            if (m) {
                                uint32_t off = 0;
                                if (lane == 0) off = atomicAdd(&gcount, static_cast<uint32_t>(popc64(m)));
                                off = __builtin_amdgcn_readfirstlane(off);
                                if (keep) kbuf[mbcnt64(m, off)] = sk;
                            }
                        }
                        kmax = wave_max_u32(kmax);
                        kmin = wave_min_u32(kmin);
                        if (lane == 0) {
                            atomicMax(&L.seg_more[0], kmax);
                            atomicMin(&L.seg_more[1], kmin);
                        }
                        __syncthreads();
                        c_sort = static_cast<int>(gcount);
                        keys = kbuf;
                        filtered = true;
                        if (tid == 0 && !a.tie_idx_desc && L.have_prev_min && L.seg_more[0] == L.prev_min)
                            atomicOr(&a.status[f], FD_FRAME_TIES);
                    }
                {
                    const int c = c_sort;
                    uint64_t *const unsorted = keys;

                    // Bucket placement (every bin of the sub-chunk holds <= kBucketMax keys, the usual
                    // case at the top of the list): a key of bin b belongs at (keys in the bins above b)
                    // + (larger keys of its own bin). The level's suffix counts give the first term; a
                    // bin's keys are grouped by one LDS atomic each on S[b+1] (entries not read again:
                    // the next sub-chunk starts at S[slo]), then ranked by a scan of their group.
                    uint64_t me = 0;
                    uint32_t s_b = 0, s_b1 = 0;
                    int bin = 0;
                    bool big = c > nthr || filtered;
                    if (!big && tid < c) {
                        me = unsorted[tid];
                        bin = static_cast<int>((me >> rem) & ((1ull << w) - 1ull));
                        s_b = S[bin];
                        s_b1 = S[bin + 1];
                        big = s_b - s_b1 > static_cast<uint32_t>(kBucketMax);
                    }
                    if (kExitAt == 5) return;
                    if (ballot(big) != 0ull && lane == 0) L.vote[0] = 1u;
                    if (scan_fast && tid < kScanBatches) sl.cnt[tid] = 0u;  // (the last scan's reads are barriers ago)
                    __syncthreads();
                    if (L.vote[0] == 0u) {
                        uint32_t slot = 0;
                        if (tid < c) {
                            slot = atomicAdd(const_cast<uint32_t *>(&S[bin + 1]), 1u) - sbase;
                            tmp[min(slot, static_cast<uint32_t>(kSelectChunk - 1))] = me;
                        }
                        __syncthreads();
                        FD_STAMP(11);  // bucket scatter
                        if (kExitAt == 6) return;
                        if (tid < c) {
                            const uint32_t g0 = s_b1 - sbase, gn = s_b - s_b1;
                            uint32_t r = 0;
                            if (!a.dup_keys) {
                                for (uint32_t j0 = 0; j0 < gn; j0 += 8) {  // 8 loads in flight (clamped to the group)
                                    uint64_t v[8];
#pragma unroll
                                    for (uint32_t u = 0; u < 8; ++u) v[u] = tmp[g0 + min(j0 + u, gn - 1)];
#pragma unroll
                                    for (uint32_t u = 0; u < 8; ++u) r += (j0 + u < gn && v[u] > me) ? 1u : 0u;
                                }
                            } else {  // equal keys (caller lists naming a pixel twice): ranked by group slot
                                const uint32_t mine = slot - g0;
                                for (uint32_t j = 0; j < gn; ++j) {
                                    const uint64_t v = tmp[g0 + j];
                                    r += (v > me || (v == me && j < mine)) ? 1u : 0u;
                                }
                            }
                            place(static_cast<int>(min(g0 + r, static_cast<uint32_t>(kSelectChunk - 1))), me);
                        }
                        __syncthreads();
                        FD_STAMP(13);  // bucket rank + place
                    } else {
                    // Local-digit bucket placement (the level's digit left a bin of more than kBucketMax
                    // keys, or the prefilter dropped keys: FAST's clustered top responses): the same
                    // placement on a digit of the sub-chunk's own 32-bit key range, kLocalBins buckets.
                    // Falls back to the merge sort below when a bucket still holds more than kBucketMax.
                    constexpr int kLocalBins = 1024;
                    constexpr int kPer = (kSelectChunk + NT - 1) / NT;
                    uint32_t *const lcnt = L.pk32;  // [kLocalBins + 1] counts, then suffix sums (place rewrites pk32)
                    if (tid == 0) {
                        L.lb_rng[0] = 0xFFFFFFFFu;
                        L.lb_rng[1] = 0u;
                    }
                    for (int b = tid; b <= kLocalBins; b += nthr) lcnt[b] = 0u;
                    uint64_t kk[kPer];
                    uint32_t kmn = 0xFFFFFFFFu, kmx = 0u;
#pragma unroll
                    for (int j = 0; j < kPer; ++j) {
                        const int p = tid + j * nthr;
                        kk[j] = p < c ? unsorted[p] : 0ull;
                        if (p < c) {
                            kmn = min(kmn, static_cast<uint32_t>(kk[j] >> 32));
                            kmx = max(kmx, static_cast<uint32_t>(kk[j] >> 32));
                        }
                    }
                    kmn = wave_min_u32(kmn);
                    kmx = wave_max_u32(kmx);
                    __syncthreads();  // (lb_rng, lcnt initialised)
                    if (lane == 0 && kmn <= kmx) {
                        atomicMin(&L.lb_rng[0], kmn);
                        atomicMax(&L.lb_rng[1], kmx);
                    }
                    __syncthreads();
                    const uint32_t lo32 = L.lb_rng[0], rng = L.lb_rng[1] - L.lb_rng[0];
                    const int lsh = rng < static_cast<uint32_t>(kLocalBins) ? 0 : (32 - __builtin_clz(rng)) - 10;
                    uint32_t dg[kPer], sl[kPer];
#pragma unroll
                    for (int j = 0; j < kPer; ++j) {
                        dg[j] = (static_cast<uint32_t>(kk[j] >> 32) - lo32) >> lsh;
                        sl[j] = 0;
                        if (tid + j * nthr < c) sl[j] = atomicAdd(&lcnt[dg[j]], 1u);
                    }
                    __syncthreads();
                    FD_STAMP(10);
                    suffix(lcnt, kLocalBins);  // lcnt[b] = keys of digits >= b (descending placement)
                    bool lbig = false;
#pragma unroll
                    for (int j = 0; j < kPer; ++j)
                        if (tid + j * nthr < c) lbig = lbig || lcnt[dg[j]] - lcnt[dg[j] + 1] > static_cast<uint32_t>(kBucketMax);
                    if (ballot(lbig) != 0ull && lane == 0) L.vote[1] = 1u;
                    __syncthreads();
                    if (L.vote[1] == 0u) {
#pragma unroll
                        for (int j = 0; j < kPer; ++j)
                            if (tid + j * nthr < c) tmp[min(lcnt[dg[j] + 1] + sl[j], static_cast<uint32_t>(kSelectChunk - 1))] = kk[j];
                        __syncthreads();
                        FD_STAMP(11);  // local bucket scatter
                        uint32_t pos[kPer];
#pragma unroll
                        for (int j = 0; j < kPer; ++j) {
                            pos[j] = 0;
                            if (tid + j * nthr >= c) continue;
                            const uint32_t g0 = lcnt[dg[j] + 1], gn = lcnt[dg[j]] - g0;
                            uint32_t r = 0;
                            // 8 loads in flight (clamped to the group; a group is usually a few keys):
                            // not a chain of dependent LDS round trips
                            for (uint32_t q0 = 0; q0 < gn; q0 += 8) {
                                uint64_t v[8];
#pragma unroll
                                for (uint32_t u = 0; u < 8; ++u) v[u] = tmp[g0 + min(q0 + u, gn - 1)];
#pragma unroll
                                for (uint32_t u = 0; u < 8; ++u) {
                                    const uint32_t q = q0 + u;
                                    r += (q < gn && (v[u] > kk[j] || (v[u] == kk[j] && q < sl[j]))) ? 1u : 0u;
                                }
                            }
                            pos[j] = g0 + r;
                        }
                        __syncthreads();  // lcnt (pk32) is read above, rewritten by place
#pragma unroll
                        for (int j = 0; j < kPer; ++j)
                            if (tid + j * nthr < c) place(static_cast<int>(min(pos[j], static_cast<uint32_t>(kSelectChunk - 1))), kk[j]);
                        __syncthreads();
                        FD_STAMP(13);  // local bucket rank + place
                    } else {
                    // Merge sort, descending: rank inside runs of 64 by counting larger
                    // keys (broadcast LDS reads), then log2 merge levels where each key moves to
                    // (its offset in its run) + (number of larger keys in the sibling run, by binary search).
                    const int c64 = (c + 63) & ~63;
                    for (int i = c + tid; i < c64; i += nthr) unsorted[i] = 0ull;
                    __syncthreads();
                    for (int p = tid; p < c; p += nthr) {
                        const uint64_t me = unsorted[p];
                        const ulonglong2 *b2 = reinterpret_cast<const ulonglong2 *>(unsorted + (p & ~63));
                        int lr = 0;
                        if (!a.dup_keys) {
    #pragma unroll 8
                            for (int j = 0; j < 32; ++j) {
                                const ulonglong2 q = b2[j];
                                lr += (q.x > me) + (q.y > me);
                            }
                        } else {  // equal keys: by position in the run (a stable order)
                            const int mine = p & 63;
                            for (int j = 0; j < 32; ++j) {
                                const ulonglong2 q = b2[j];
                                lr += (q.x > me || (q.x == me && 2 * j < mine)) + (q.y > me || (q.y == me && 2 * j + 1 < mine));
                            }
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
                            // larger keys in the sibling run (and, for the right run of a pair, equal
                            // ones: a stable merge when keys repeat; unique keys are unaffected)
                            const bool right = (run & 1) != 0;
                            int lo2 = 0, hi2 = max(0, min(w, c - sib));
                            while (lo2 < hi2) {
                                const int mid = (lo2 + hi2) >> 1;
                                const uint64_t o = src[sib + mid];
                                if (o > me || (right && o == me)) lo2 = mid + 1; else hi2 = mid;
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
                    }
                    }
                    if (!a.tie_idx_desc && !(kKnockOut & 4) && !scan_fast) {  // tie bits over the ordered sub-chunk (wave-aligned 64-blocks)
                        const int c64 = ((c + kWave - 1) & ~(kWave - 1)) + kWave;
                        for (int i = opaque(tid); i < c64; i += nthr) {
                            const bool t = i > 0 && i < c && L.pk32[i] == L.pk32[i - 1];
                            const uint64_t m = ballot(t);
                            if (lane == 0) L.tmask[i >> 6] = m;
                        }
                    }
                    // conflict masks: earlier candidates of the same 64-batch within distance d
                    // (the pipelined scan computes both per batch, beside the scan)
                    if (use_grid && !(kKnockOut & 2) && !scan_fast) conflict_masks(pxy, c, d, rows, cols, buf, tid, nthr);
                }
                if (!scan_fast) __syncthreads();
                if (tid == 0) {  // (read before the placement's last barrier; the next placement is barriers away)
                    L.vote[0] = 0u;
                    L.vote[1] = 0u;
                }
                FD_STAMP(14);  // conflict masks
                if (kExitAt == 3) return;
                // greedy scan in order by wave 0 (SelectGoodFeatures :62-72); ties checked unless the
                // order of equal responses is defined (SuperPoint's multimap)
                if (kKnockOut & 1) {  // (phase-cost diagnostic build: no greedy, the frame ends here)
                    if (tid == 0) s_done = 1;
                } else if (scan_fast) {
                    // wave 0 scans batch b once waves 1.. have its conflict masks in LDS
                    if (wave == 0)
                        greedy_scan(a, f, c_sort, pxy, pcell, buf, grid_lds, gw2, prior, s_acc, s_done, sl,
                                    a.stamps ? L.st : nullptr);
                    else
                        scan_masks(pxy, c_sort, d, rows, cols, buf, sl, wave - 1, nthr / kWave - 1);
                    __syncthreads();
                    scan_outputs(a, f, c_sort, pxy, sl, !a.tie_idx_desc, L.pk32, L.tie_prev, L.tie_has_prev, tid, nthr);
                } else if (tid < kWave) {
                    const bool ties = !a.tie_idx_desc;
                    const uint64_t *tm = L.tmask;
                    if (!use_grid)
                        greedy_chunk<0>(a, f, c_sort, pxy, pcell, buf, grid_lds, gw2, prior, s_acc, s_done, ties, tm,
                                        L.pk32[0], L.pk32[max(c_sort - 1, 0)], L.tie_prev, L.tie_has_prev,
                                        a.stamps ? L.st : nullptr);
                    else if (grid_in_lds)
                        greedy_chunk<1>(a, f, c_sort, pxy, pcell, buf, grid_lds, gw2, prior, s_acc, s_done, ties, tm,
                                        L.pk32[0], L.pk32[max(c_sort - 1, 0)], L.tie_prev, L.tie_has_prev,
                                        a.stamps ? L.st : nullptr);
                    else
                        greedy_chunk<2>(a, f, c_sort, pxy, pcell, buf, grid_g, gw2, prior, s_acc, s_done, ties, tm,
                                        L.pk32[0], L.pk32[max(c_sort - 1, 0)], L.tie_prev, L.tie_has_prev,
                                        a.stamps ? L.st : nullptr);
                }
                if (tid == 0 && (filtered || c_sort > 0)) {  // the sub-chunk's smallest 32-bit key
                    L.prev_min = filtered ? L.seg_more[1] : L.pk32[c_sort - 1];
                    L.have_prev_min = 1;
                }
                __syncthreads();
                FD_STAMP(5);  // greedy
                }
                shi = slo - 1;
            }
            FD_COUNT(8, 1);
        }
        hi = lo - 1;
    }
    if (a.cut_next) {
        // FAST emission cut (PointsArgs::emit_cut). Out of emitted keys before `need` with candidates left
        // below the cut: the frame runs again without it (redo pass, same call) -- the reference's scan
        // would continue past the cut. Either way, this frame's proposal for the next call's cut: the
        // lower edge of the highest level-0 bin with at least max(4 V, V + 4096) emitted keys at or above
        // it, V = the keys in the bins down to the lowest one the scan gathered (a margin for frames of the
        // same kind); with fewer emitted keys than that, 1.0 below this call's cut; 0 (no cut) for a frame
        // that ran out.
        const bool done = s_done != 0;
        uint32_t prop = 0u;
        if (done && L.have_prev_min) {
            const uint32_t vis = suf0[min(static_cast<int>(L.prev_min >> 20), kHistBins - 1)];
            const uint32_t target = max(static_cast<uint32_t>(FD_CUT_MUL) * vis, vis + static_cast<uint32_t>(FD_CUT_ADD));
            const int x0 = first_le(suf0, 0, kHistBins, 0u, target - 1u);  // (all threads: barriers)
            if (x0 > 0) {
                const uint32_t fk = a.key_base + ((static_cast<uint32_t>(x0 - 1) << 20) >> a.key_lz);
                prop = (fk & 0x80000000u) ? (fk & 0x7FFFFFFFu) : 0u;  // the bin's lowest response (a positive float)
            } else {
                const float cur = __uint_as_float(*a.cut_cur);
                prop = cur > 1.0f ? __float_as_uint(cur - 1.0f) : 0u;
            }
        }
        if (tid == 0) {
            if (!done && a.skipped[f]) atomicOr(&a.status[f], kFrameRedo);
            atomicMin(a.cut_next, prop);
        }
    }
    if (tid == 0) a.out_counts[f] = s_acc;  // (flags, if any, are in a.status[f])
    FD_STAMP(7);
    if (a.stamps && tid == 0)
        for (int i = 0; i < 32; ++i) a.stamps[static_cast<int64_t>(f) * 32 + i] = L.st[i];
}

// Resets the frame's counters and level-0 histogram for the next call (stream order puts that call's
// per-pixel kernel after this kernel).
__device__ __forceinline__ void finish_frame(const SelectArgs &a, const int f) {
    __syncthreads();
    // sc1 stores: written through and dropped from this XCD's L2, like the atomics that update these
    // words in the next call's per-pixel kernel (a kernel boundary separates the two either way).
    uint32_t *h = a.hist0 + static_cast<int64_t>(f) * kHistBins;
    for (int b = threadIdx.x; b < kHistBins; b += blockDim.x)
        __hip_atomic_store(&h[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) {
        __hip_atomic_store(&a.list_count[f], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.pre_count) __hip_atomic_store(&a.pre_count[f], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.seg_bad) __hip_atomic_store(&a.seg_bad[f], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // (wide_cut too: the control block's layout depends on the batch, so a word left non-zero here
        // could be a histogram bin of a later call with another batch size)
        if (a.wide_count) __hip_atomic_store(&a.wide_count[f], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.wide_cut) __hip_atomic_store(&a.wide_cut[f], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.skipped) __hip_atomic_store(&a.skipped[f], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the frame's final status to the host (the stream's synchronisation makes it visible; a redo
        // pass's finish_frame writes it again)
        if (a.status_host) a.status_host[f] = __hip_atomic_load(&a.status[f], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Gather kernel (small batches): G workgroups per frame each derive the frame's first level-0 chunk
// (the highest bins holding <= kSelectChunk candidates) from the histogram and append the keys of
// their slice of the list to pre_keys. k_select, the next kernel, reads them: the kernel boundary is
// the visibility point, so no hand-off happens inside either kernel.
__global__ __launch_bounds__(1024) void k_gather(SelectArgs a) {
    __shared__ GatherLds L;
    const int G = a.gather_groups;
    const int f = blockIdx.x / G, g = blockIdx.x % G;
    const GatherView v{a.list_resp + static_cast<int64_t>(f) * a.list_cap, a.list_idx + static_cast<int64_t>(f) * a.list_cap,
                       min(static_cast<int64_t>(a.list_count[f]), a.list_cap), a.hist0 + static_cast<int64_t>(f) * kHistBins,
                       a.key_base, a.key_lz, a.tie_idx_desc, a.pre_keys + static_cast<int64_t>(f) * kSelectChunk,
                       a.pre_count + f, static_cast<uint32_t>(kSelectChunk)};
    gather_first_chunk<1024>(v, g, G, L);
}

// Wide pass (FAST, SelectArgs::wide_count) in two kernels: k_wide_cut finds each frame's cut (the top
// level-0 bins holding <= kWideKeys candidates) once, from the complete histogram; k_wide_gather then
// streams the frame's list over wide_groups workgroups and appends the keys at or above the cut to the
// frame's wide scratch. In k_select one workgroup made this pass (FAST on 1280x720 noise: ~270k
// candidates, ~55k of ~130k cycles per frame); a cut per gather workgroup cost more than the pass.
__global__ __launch_bounds__(256) void k_wide_cut(SelectArgs a) {
    __shared__ uint32_t wt[4];
    __shared__ int res;
    const int f = blockIdx.x, tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    static_assert(kHistBins == 256 * 16, "16 bins per thread");
    const uint4 *h = reinterpret_cast<const uint4 *>(a.hist0 + static_cast<int64_t>(f) * kHistBins) + 4 * tid;
    uint32_t v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint4 q = h[j];
        v[4 * j] = q.x;
        v[4 * j + 1] = q.y;
        v[4 * j + 2] = q.z;
        v[4 * j + 3] = q.w;
    }
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) sum += v[j];
    const uint32_t incl = wave_suffix_add(sum);  // this thread's bins and every higher thread's in the wave
    if (lane == 0) wt[wave] = incl;
    if (tid == 0) res = kHistBins;
    __syncthreads();
    uint32_t run = incl - sum;  // keys in bins above this thread's, within the wave ...
    for (int w = wave + 1; w < 4; ++w) run += wt[w];  // ... and in the higher waves
    // smallest bin b with (keys in bins >= b) <= kWideKeys: the suffix is non-increasing in b
    int best = kHistBins;
    uint32_t best_s = 0;
#pragma unroll
    for (int j = 15; j >= 0; --j) {
        run += v[j];
        if (run <= static_cast<uint32_t>(kWideKeys)) {
            best = 16 * tid + j;
            best_s = run;
        }
    }
    if (best < kHistBins) atomicMin(&res, best);
    __syncthreads();
    __shared__ uint32_t res_s;
    if (tid == 0) res_s = 0;
    __syncthreads();
    if (best == res) res_s = best_s;  // (one thread: the bins are disjoint)
    __syncthreads();
    if (tid == 0) {
        // no keys at or above the cut (none at all, or the bin below it alone holds more than kWideKeys),
        // or the top bin alone holds more: nothing to gather (k_select descends itself), as in k_select's
        // own wide pass
        const bool none = res >= kHistBins || res_s == 0u;
        a.wide_cut[f] = none ? static_cast<uint32_t>(kHistBins) : static_cast<uint32_t>(res);
    }
}

constexpr int kWidePer = 16;      // list entries per thread and round of k_wide_gather (4 x 16-byte loads)
constexpr int kWideThreads = 1024;  // k_wide_gather workgroup
// One reservation on the frame's key counter per workgroup and round (a block prefix of the waves' hit
// counts): same-address device atomics serialise at the memory side (256-thread workgroups with one
// atomic per wave measured 41-60 us for 64 frames of 1280x720 FAST, slower with more workgroups).
__global__ __launch_bounds__(kWideThreads) void k_wide_gather(SelectArgs a) {
    __shared__ uint32_t wsum[kWideThreads / kWave];
    __shared__ uint32_t wg_base;
    const int G = a.wide_groups;
    const int f = blockIdx.x / G, g = blockIdx.x % G;
    const uint32_t cut = a.wide_cut[f];
    if (cut >= static_cast<uint32_t>(kHistBins)) return;
    const uint32_t k32lo = cut << 20;
    const int tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
    const uint32_t n = static_cast<uint32_t>(min(static_cast<int64_t>(a.list_count[f]), a.list_cap));
    const float *lresp = a.list_resp + static_cast<int64_t>(f) * a.list_cap;
    const uint32_t *lidx = a.list_idx + static_cast<int64_t>(f) * a.list_cap;
    // (list_cap < 2^30 entries, checked on the host: the byte offsets fit the resource; loads past the
    // frame's capacity read 0)
    const auto rres = make_rsrc(lresp, static_cast<uint32_t>(a.list_cap) * 4u);
    const auto ridx = make_rsrc(lidx, static_cast<uint32_t>(a.list_cap) * 4u);
    uint64_t *wk = a.wide_keys + static_cast<int64_t>(f) * kWideKeys;
    constexpr uint32_t kRound = static_cast<uint32_t>(kWideThreads) * kWidePer;
    // (the loop bounds are uniform across the workgroup: every thread reaches every barrier)
    for (uint32_t base = static_cast<uint32_t>(g) * kRound; base < n; base += static_cast<uint32_t>(G) * kRound) {
        // wave w reads the contiguous 4 KiB [base + 1024 w, +1024): its lanes' 16-byte loads side by side
        const uint32_t i0 = base + static_cast<uint32_t>(wave) * (kWave * kWidePer) + 4u * static_cast<uint32_t>(lane);
        float r[kWidePer];
#pragma unroll
        for (int j = 0; j < kWidePer / 4; ++j) {
            const auto q = __builtin_amdgcn_raw_buffer_load_b128(rres, static_cast<int>(4u * (i0 + 256u * j)), 0, 0);
            r[4 * j] = __uint_as_float(q[0]);
            r[4 * j + 1] = __uint_as_float(q[1]);
            r[4 * j + 2] = __uint_as_float(q[2]);
            r[4 * j + 3] = __uint_as_float(q[3]);
        }
        auto at = [&](int j) { return i0 + 256u * static_cast<uint32_t>(j >> 2) + static_cast<uint32_t>(j & 3); };
        uint32_t hm = 0;
#pragma unroll
        for (int j = 0; j < kWidePer; ++j)
            hm |= static_cast<uint32_t>(at(j) < n && sel_key32(r[j], a.key_base, a.key_lz) >= k32lo) << j;
        const uint32_t cnt = __popc(hm);
        const uint32_t incl = wave_incl_add(cnt);
        if (lane == kWave - 1) wsum[wave] = incl;
        __syncthreads();
        uint32_t before = 0, total = 0;
#pragma unroll
        for (int w = 0; w < kWideThreads / kWave; ++w) {
            const uint32_t v = wsum[w];
            before += w < wave ? v : 0u;
            total += v;
        }
        if (tid == 0) wg_base = total ? atomicAdd(&a.wide_count[f], total) : 0u;
        __syncthreads();
        uint32_t pos = wg_base + before + incl - cnt;
        if (hm) {
            // the pixel indices of this thread's entries in one round trip (not one dependent load per hit)
            uint32_t ix[kWidePer];
#pragma unroll
            for (int j = 0; j < kWidePer / 4; ++j) {
                const auto q = __builtin_amdgcn_raw_buffer_load_b128(ridx, static_cast<int>(4u * (i0 + 256u * j)), 0, 0);
                ix[4 * j] = q[0];
                ix[4 * j + 1] = q[1];
                ix[4 * j + 2] = q[2];
                ix[4 * j + 3] = q[3];
            }
#pragma unroll
            for (int j = 0; j < kWidePer; ++j) {
                if ((hm >> j) & 1u) {
                    if (pos < static_cast<uint32_t>(kWideKeys))
                        wk[pos] = sel_key64(r[j], ix[j], a.key_base, a.key_lz, a.tie_idx_desc);
                    ++pos;
                }
            }
        }
        __syncthreads();  // (wsum / wg_base reused by the next round)
    }
}

template <int NT, bool WIDE>
__global__ __launch_bounds__(NT) void k_select(SelectArgs a) {
    __shared__ SelectLds L;
    const int f = blockIdx.x;
    select_frame<NT, WIDE>(a, f, L);
    finish_frame(a, f);
}

// The redo pass (kFrameRedo; FAST's emission cut), a few workgroups: workgroup w owns frames w, w + G, ...
// (a static assignment: select_frame clears a frame's status word, which no other workgroup reads), their
// flags one load per lane, broadcast; usually none is set. Its own kernel: a loop around select_frame in
// k_select itself cost that kernel ~30 more spilled registers.
template <int NT>
__global__ __launch_bounds__(NT) void k_select_redo(SelectArgs a) {
    __shared__ SelectLds L;
    __shared__ uint64_t mine;
    const int G = static_cast<int>(gridDim.x), w = static_cast<int>(blockIdx.x);
    for (int base = 0; base < a.batch; base += kWave * G) {
        if (threadIdx.x < kWave) {
            const int fr = base + G * static_cast<int>(threadIdx.x) + w;
            const uint64_t b = ballot(fr < a.batch && (a.redo_status[min(fr, a.batch - 1)] & kFrameRedo));
            if (threadIdx.x == 0) mine = b;
        }
        __syncthreads();
        uint64_t m = mine;
        __syncthreads();  // (mine is rewritten by the next round)
        while (m) {
            const int f = base + G * __builtin_ctzll(m) + w;
            m &= m - 1ull;
            select_frame<NT, true>(a, f, L);
            if (threadIdx.x == 0) atomicOr(&a.status[f], FD_FRAME_REDETECTED);
            finish_frame(a, f);
            __syncthreads();  // (LDS reused by the next frame)
        }
    }
}

// Greedy selection in a given order (FD_TIES_REFERENCE): the frame's candidates as raster indices in
// the order the reference's std::sort leaves them (computed on the host for frames k_select flagged),
// visited chunk by chunk with the same greedy as k_select (SelectGoodFeatures :62-72): decode, prior
// mask, grid cell; conflict masks; one wave scans in batches of 64. Overwrites the frame's features.
struct alignas(16) OrderedLds {
    uint32_t pxy[kSelectChunk];
    uint32_t pcell[kSelectChunk];
    uint64_t cmask[kSelectChunk];
    uint32_t grid_lds[kGridLdsCells];
    int s_done, s_acc;
    uint32_t tie_prev;
    int tie_has_prev;
};

template <int NT>
__global__ __launch_bounds__(NT) void k_select_ordered(SelectArgs a, OrderedArgs o) {
    __shared__ OrderedLds L;
    const int j = blockIdx.x, tid = threadIdx.x;
    const int f = o.frame[j];
    const uint32_t *ord = o.order + o.offset[j];
    const int64_t n = o.count[j];
    const int rows = a.rows, cols = a.cols, d = a.dist;
    const bool use_grid = d >= 1 || (d == 0 && a.grid_at_d0);
    const int gw2 = a.grid_w + 2;
    const int cells = gw2 * (a.grid_h + 2);
    const bool grid_in_lds = cells <= kGridLdsCells;
    uint32_t *const grid_g = a.grid_global ? a.grid_global + static_cast<int64_t>(f) * cells : nullptr;
    uint32_t *const grid = grid_in_lds ? L.grid_lds : grid_g;
    const uint32_t prior = a.prior_counts ? static_cast<uint32_t>(a.prior_counts[f]) : 0u;
    const uint32_t *fmask = a.mask ? a.mask + static_cast<int64_t>(f) * rows * a.mask_wpr : nullptr;
    const uint32_t npx = static_cast<uint32_t>(rows) * static_cast<uint32_t>(cols);
    const uint32_t s1 = static_cast<uint32_t>(d + 1);
    if (use_grid)
        for (int i = tid; i < cells; i += NT) grid[i] = grid_empty(rows, cols, d);
    if (tid == 0) {
        L.s_done = 0;
        L.s_acc = 0;
        L.tie_prev = 0;
        L.tie_has_prev = 0;
    }
    __syncthreads();
    for (int64_t base = 0; base < n; base += kSelectChunk) {
        if (L.s_done) break;
        const int c = static_cast<int>(min(static_cast<int64_t>(kSelectChunk), n - base));
        for (int i = tid; i < c; i += NT) {
            uint32_t idx = ord[base + i];
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
        if (use_grid) conflict_masks(L.pxy, c, d, rows, cols, L.cmask, tid, NT);
        __syncthreads();
        if (tid < kWave) {
            if (!use_grid)
                greedy_chunk<0>(a, f, c, L.pxy, L.pcell, L.cmask, grid, gw2, prior, L.s_acc, L.s_done, false, nullptr, 0u, 0u,
                                L.tie_prev, L.tie_has_prev);
            else if (grid_in_lds)
                greedy_chunk<1>(a, f, c, L.pxy, L.pcell, L.cmask, grid, gw2, prior, L.s_acc, L.s_done, false, nullptr, 0u, 0u,
                                L.tie_prev, L.tie_has_prev);
            else
                greedy_chunk<2>(a, f, c, L.pxy, L.pcell, L.cmask, grid, gw2, prior, L.s_acc, L.s_done, false, nullptr, 0u, 0u,
                                L.tie_prev, L.tie_has_prev);
        }
        __syncthreads();
    }
    if (tid == 0) {
        a.out_counts[f] = L.s_acc;
        atomicAnd(&a.status[f], ~FD_FRAME_UNRESOLVED);
        atomicOr(&a.status[f], FD_FRAME_RESOLVED);
    }
}

}  // namespace

hipError_t launch_select_ordered(const SelectArgs &a, const OrderedArgs &o, int n_frames, hipStream_t s) {
    if (n_frames <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_select_ordered<256>, dim3(static_cast<unsigned>(n_frames)), dim3(256), 0, s, a, o);
    return hipGetLastError();
}

hipError_t launch_select(const SelectArgs &a, int batch, hipStream_t s) {
    if (a.pre_keys) {
        hipLaunchKernelGGL(k_gather, dim3(static_cast<unsigned>(batch * a.gather_groups)), dim3(1024), 0, s, a);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (a.redo_status) {  // (redo pass: a few workgroups loop over the flagged frames, no wide-pass kernels)
        hipLaunchKernelGGL(k_select_redo<kSelectThreads>, dim3(static_cast<unsigned>(std::min(batch, 8))),
                           dim3(kSelectThreads), 0, s, a);
        return hipGetLastError();
    }
    const unsigned sel_grid = static_cast<unsigned>(batch);
    if (a.wide_count && a.wide_keys && a.wide_groups > 0) {
        hipLaunchKernelGGL(k_wide_cut, dim3(static_cast<unsigned>(batch)), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_wide_gather, dim3(static_cast<unsigned>(batch * a.wide_groups)), dim3(kWideThreads), 0, s, a);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    // the wide pass (k_select<.., true>) for FAST and for list mode; the corner detectors' small frames
    // (sorted segments) keep the leaner instance
    if ((a.wide_keys && (a.wide_eager || !a.segdesc)) || a.fast_sub)
        hipLaunchKernelGGL((k_select<kSelectThreads, true>), dim3(sel_grid), dim3(kSelectThreads), 0, s, a);
    else
        hipLaunchKernelGGL((k_select<kSelectThreads, false>), dim3(sel_grid), dim3(kSelectThreads), 0, s, a);
    return hipGetLastError();
}

}  // namespace fdk
