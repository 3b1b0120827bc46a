// Kernel argument blocks and host-side launchers (defined in fd_points.hip / fd_select.hip / fd_lsd.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fdk {

// Tile geometry of the per-pixel kernels: one wave owns kTileW output columns (lanes 1..62, 4 px
// each; lanes 0 and 63 only supply halo data) and tile_h output rows, walked top to bottom.
constexpr int kTileW = 248;
constexpr int kSegCorner = kTileW / 2;  // strict 4-neighbour NMS: <= 1 candidate per 2 columns
constexpr int kSegFast = kTileW;        // FAST has no NMS
#ifndef FD_LIST_NT
#define FD_LIST_NT 0  // candidate list stores with the nt (streaming) cache policy
#endif
constexpr int kSelectChunk = 2048;      // candidates sorted per greedy chunk (LDS)
#ifndef FD_SELECT_THREADS
#define FD_SELECT_THREADS 1024
#endif
constexpr int kSelectThreads = FD_SELECT_THREADS;  // k_select workgroup size (sorted segments: <= this many per frame)
constexpr int kGridLdsCells = 16384;    // occupancy grid kept in LDS up to this many cells
constexpr int kMaxOffsetSegs = 48;
constexpr int kSegHead = 64;           // selection keys kept per sorted segment head (PointsArgs::seghead)
constexpr int kWideKeys = 8192;        // keys per frame of k_select's wide first pass (SelectArgs::wide_keys)
constexpr int kHistBins = 4096;         // level-0 digit of the selection key: top 12 bits of the mapped response

// k_corner_lp tiles: px columns per lane, halo-only lanes per side so that lane 0 / 63 cover the 3
// columns of reach (NMS + 3x3 sum + central difference): 2 lanes at px = 2, else 1.
constexpr int lp_halo_lanes(int px) { return px == 2 ? 2 : 1; }
constexpr int lp_tile_w(int px) { return (64 - 2 * lp_halo_lanes(px)) * px; }

// A raster-mode segment entry (fd_points_candidates only).
struct Cand {
    float resp;
    uint32_t idx;  // row * cols + col
};

// FAST running offset o_k (feature_point_fast_detector.cpp:85,93) as a piecewise-arithmetic table:
// o_k = o_start[s] + (k - k_start[s]) * inc[s], exact in double.
struct FastOffsets {
    int nseg;
    int64_t k0;  // first k with o_k > threshold (score-0 pixels before it are never candidates)
    int64_t k_start[kMaxOffsetSegs];
    double o_start[kMaxOffsetSegs];
    double inc[kMaxOffsetSegs];
    // FAST score of a 16-bit ring mask (bit k = sample k of kFastIndice): the longest circular run of
    // set bits, i.e. the reference's two-pass count (feature_point_fast_detector.cpp:55-78). 64 KiB,
    // device memory owned by the context (build_offsets fills it once).
    const uint8_t *run_lut;
};

struct PointsArgs {
    const uint8_t *frames;
    int batch, rows, cols;
    int tiles_x, tiles_y, tile_h;
    int blocks_per_frame;  // workgroups of 4 waves per frame (a workgroup never straddles frames)
    int px;  // corner detect/response: columns per lane of k_corner_lp (2, 4, 8; tile width lp_tile_w), 0 = k_corner
    int aligned4;  // cols % 4 == 0 and 4-byte aligned frames: whole-dword loads are range-exact
    float thr;
    const uint32_t *mask;  // prior-feature bitmap [batch][rows][mask_wpr], bit = mask true; null = all ones
    int mask_wpr;
    // detect mode: unordered per-frame lists (SoA) + level-0 key histogram
    float *list_resp;
    uint32_t *list_idx;
    int64_t list_cap;
    uint32_t *list_count;
    uint32_t *hist0;  // [batch][kHistBins] or null
    uint32_t key_base;  // level-0 bin = ((float_key(resp) - key_base) << key_lz) >> 20 (see SelectArgs)
    int key_lz;
    // raster mode: per (frame, row, tile_x) segments
    int32_t *seg_cnt;
    Cand *seg;
    float *resp_map;  // optional full response map (raster mode)
    // masked FAST: k = row_base[f][r] + word_pref[f][r][w] + popcount within the word
    const int32_t *row_base;
    const int32_t *word_pref;
    // Sorted-segment mode (small launches, detect mode with hist0): [batch][blocks_per_frame] (base,
    // count) of each workgroup's bin-sorted list segment; seg_bad[f] set when a tile overflowed its
    // staging (the frame's list is then unsorted). Null = off.
    uint2 *segdesc;
    uint32_t *seg_bad;
    uint64_t *seghead;  // [batch][blocks_per_frame][kSegHead] the segments' first keys (selection keys)
    // FAST emission cut (detect mode, raster tie order): a candidate whose response is
    // below the float *emit_cut (bits; null: none) is counted in skipped[f] instead of emitted; workgroup 0
    // sets *emit_cut_next to +inf, the identity of the selection's proposals for the next call. redo_status:
    // the second pass, where only the frames whose status word has kFrameRedo run (emitting everything).
    const uint32_t *emit_cut;
    uint32_t *emit_cut_next;
    uint32_t *skipped;
    const uint32_t *redo_status;
};

// Internal status bit (SelectArgs::status): the selection ran out of emitted keys of a frame whose
// per-pixel pass skipped some (FAST emission cut); the frame is detected and selected again in the same
// call (redo pass), which clears the bit.
constexpr uint32_t kFrameRedo = 0x00000100u;

struct SelectArgs {
    const float *list_resp;
    const uint32_t *list_idx;
    uint32_t *list_count;  // reset to 0 by the kernel once the frame is done
    uint32_t *hist0;       // [batch][kHistBins], reset likewise
    int64_t list_cap;
    int rows, cols;
    const uint32_t *mask;
    int mask_wpr;
    const int32_t *prior_counts;  // device, per frame (null = none)
    uint32_t need;
    int dist;
    int grid_w, grid_h;
    uint32_t *grid_global;  // [batch][grid_w * grid_h] when the grid does not fit LDS (slow path)
    float *out_xy;
    int out_stride;
    int32_t *out_counts;  // plain feature counts (no flag bits)
    // host-output calls in the raster tie order: out_xy / out_counts are pinned host memory and the final
    // status words are mirrored here by finish_frame, so no copy follows the kernel (nullptr: none)
    uint32_t *status_host;
    // [batch] per-frame status (fd_hip.h FD_FRAME_*: tie in the scanned prefix, guard flags) and
    // [batch] candidate count of the frame (kept for a tie resolution after the list count is reset)
    uint32_t *status;
    uint32_t *cand_n;
    // key map: 32-bit key = (float_key(response) - key_base) << key_lz; all candidates have
    // responses > min_valid_response, so key_base = float_key(min_valid_response) and key_lz spreads
    // the possible response range over the full 32 bits (finer level-0 bins).
    uint32_t key_base;
    int key_lz;
    int tie_idx_desc;  // equal responses by descending raster index (SuperPoint) instead of ascending
    int value_flag;    // pre_count bit 31 set by the candidate kernel -> guard flag 0x40000000 (out of key range)
    // gather kernel (k_gather, batch x gather_groups workgroups) -> first level-0 chunk per frame;
    // null pre_keys: k_select gathers it itself
    uint64_t *pre_keys;   // [batch][kSelectChunk]
    uint32_t *pre_count;  // [batch], reset by k_select
    int gather_groups;
    const uint2 *segdesc;   // the candidate kernel's sorted segments (PointsArgs::segdesc) or null
    const uint64_t *seghead;  // their first kSegHead selection keys (PointsArgs::seghead)
    uint32_t *seg_bad;      // [batch], reset by k_select
    int nseg;               // segments per frame
    uint64_t *wide_keys;  // [batch][kWideKeys] scratch of the wide pass, or null (one list pass per chunk)
    int wide_eager;       // wide pass with the first chunk (FAST) instead of at the first later list pass
    int fast_sub;         // FAST's selection shape (k_select<.., true>, whole-superchunk sub-chunks) without a wide
                          // pass (wide_keys null): the short lists of the emission cut
    // k_wide_cut + k_wide_gather (batch x wide_groups workgroups of 256 threads, before k_select): the wide pass of a
    // wide_eager frame spread over the frame's list, keys into wide_keys, their number into wide_count
    // (reset by k_select); null wide_count: k_select makes the pass itself, one workgroup per frame
    uint32_t *wide_count;
    uint32_t *wide_cut;  // [batch] k_wide_cut's level-0 bin cut (kHistBins: none), read by k_wide_gather
    int wide_groups;
    // FAST emission cut (PointsArgs::emit_cut): skipped [batch] (reset here), the cut this call used and the
    // word the frames' proposals for the next call go to (atomicMin of float bits); redo_status: the redo
    // pass, in which only frames flagged kFrameRedo run (k_wide_cut / k_wide_gather / k_select)
    uint32_t *skipped;
    const uint32_t *cut_cur;
    uint32_t *cut_next;
    const uint32_t *redo_status;
    int batch;  // frames of the call (the redo pass's workgroups loop over them)
    int first_sub;     // sorted-segment corner frames: first chunk cut at one sub-chunk (kSubChunk keys)
    int grid_at_d0;    // distance 0 still tests the grid (1-pixel cells): caller lists may name a pixel twice
    int dup_keys;      // equal selection keys possible (caller lists): the orderings rank them stably
    uint64_t *stamps;  // diagnostic only (FD_SELECT_STAMPS): per-frame phase clocks, never read back by kernels
};

// Greedy selection over candidates given in an explicit order (FD_TIES_REFERENCE: the reference's
// std::sort permutation of a frame, computed on the host), one workgroup per listed frame.
struct OrderedArgs {
    const uint32_t *order;  // raster indices (row * cols + col), each frame's run in visiting order
    const int64_t *offset;  // [n_frames] start of frame j's run in `order`
    const uint32_t *count;  // [n_frames] its length
    const int32_t *frame;   // [n_frames] frame index (into SelectArgs' per-frame arrays)
};

// Wide prelude of k_select_reference (large frames, launch_select_reference with wide): the push order
// and the first partition levels of the frame's leftmost range, each spread over kRefWideGroups
// workgroups per flagged frame, while that range has more than kRefWideMin elements.
constexpr int kRefWideLevels = 8;
constexpr int kRefWideGroups = 32;
constexpr int kRefWideSlots = 32;  // flagged frames in flight per prelude kernel (more: each workgroup loops)
constexpr uint32_t kRefWideMin = 8192;
struct RefCtl {  // per frame, written by the prelude, read by k_select_reference
    uint32_t n, nlev, bad;
    uint32_t h[kRefWideLevels + 1], dep[kRefWideLevels + 1], act[kRefWideLevels + 1];  // level l: range [0, h[l])
    uint32_t sib_lo[kRefWideLevels], sib_hi[kRefWideLevels];  // level l's right child [sib_lo, sib_hi), depth dep[l] - 1
    uint32_t ch, pv, nL, nR, chL, chR;  // the current level's pivot position / response bits, stopper counts, ranks of ch
    uint2 x0, xch;                      // its elements at 0 and ch before the pivot swap
};

// k_select_reference (FD_TIES_REFERENCE on the GPU): per-frame scratch of cap entries each (cap >= the
// list capacity and >= rows * cols / 32: the raster-order bitmap and its word prefix live in lpos / rpos).
struct RefSortArgs {
    uint2 *x;        // [batch][cap] (response bits, raster index) in push order, partitioned in place
    uint32_t *lpos;  // [batch][cap] left-stopper positions by rank (per level)
    uint32_t *rpos;  // [batch][cap] right-stopper positions by rank
    uint32_t *ord;   // [batch][cap] the reference's visiting order (raster indices) of the finalised prefix
    int64_t cap;
    int push_order;  // the list is already in push order (fd_points_select); else unique raster indices
    uint32_t *dbg;   // [batch][8] first broken invariant per frame (FD_REF_DEBUG), or null
    RefCtl *ctl;     // [batch] wide prelude state (launch_select_reference with wide), else unused
    uint32_t *wcnt;  // [batch][kRefWideGroups][2] per-workgroup counts of the prelude
    uint32_t *wfr;   // [1 + batch] the prelude's compact list: count, flagged frames
    int wide;        // set by the launcher: the prelude ran (push order and the first levels are done)
    int order_only;  // the visiting order alone (ord, every window; no greedy, no outputs): LSD seed order
    int guard_limit;  // iterations of the window x level loop before the frame is failed (0: 1 << 16); diagnostic override
};

// fd_points_select: caller candidates (response, x, y at [f * stride], counts[f]) -> list format.
struct CandInArgs {
    const float *resp;
    const int32_t *x, *y;
    const int64_t *counts;  // [batch] (device)
    int64_t stride;
    int batch, rows, cols;
    float *list_resp;
    uint32_t *list_idx;
    int64_t list_cap;
    uint32_t *list_count;
    uint32_t *hist0;
    uint32_t key_base;
    int key_lz;
    uint32_t *bad;  // [batch] bit 31: a candidate outside the frame, a NaN response or a bad count
    // keypoint-list models (fd_nn_select_list): (u, v) int64 pairs instead of x / y, and candidates
    // within `border` of the frame edge dropped (CreateMask's zero rows/cols). The list is then
    // appended to (unordered; the selection orders equal scores by raster index, tie_idx_desc).
    const int64_t *kp;
    int border;  // < 0: keep push order at list position i (fd_points_select)
};

// fd_nn_select_list: descriptor rows of the selected keypoints. Per (frame f, feature k), the
// candidate at that pixel visited first by the selection (highest score, then highest index).
struct NnPickArgs {
    const int64_t *kp;      // [batch][stride_in][2]
    const float *scores;    // [batch][stride_in]
    const int64_t *counts;  // [batch]
    int64_t stride_in;
    const float *desc;      // [batch][stride_in][dim]
    int dim;
    const float *xy;        // [batch][out_stride][2] selected features
    const int32_t *n_sel;   // [batch]
    int out_stride;
    int batch;
    float *out;             // [batch][out_stride][dim]
};

struct CompactArgs {
    const int32_t *seg_cnt;
    const Cand *seg;
    int rows, cols, tiles_x, seg_cap, row_lo, row_hi;  // segment rows [row_lo, row_hi)
    float *out_resp;
    int32_t *out_x, *out_y;
    int64_t cap;
    int64_t *out_counts;
};

struct LsdArgs {
    const uint8_t *frames;
    int batch, rows, cols;
    int strips, chunks, chunk_h;
    int strips4;   // k_lsd_map strips of 256 columns (4 per lane); strips: 64-column strips
    int aligned4;  // cols % 4 == 0 and 4-byte aligned frames: whole-dword row loads
    float min_norm;
    float *norm, *angle;
    uint8_t *valid;
    int pitch;          // dense maps: entries per map row (>= cols-1; a multiple of 4 keeps the row stores aligned)
    uint32_t *rowbits;  // [batch][chunks][words][cols-1]: valid rows of each (column, chunk), bit r - r0
                        // (column fastest: a wave's stores and loads are contiguous)
    int words;          // ceil(chunk_h / 32)
    int chunk_fastest;  // k_lsd_map wave order: chunk index fastest (else strip fastest)
    int scatter_cols;   // k_lsd_scatter columns per wave (16, 32 or 64)
    int32_t *col_cnt;   // [batch][chunks][cols-1]
    int32_t *col_base;  // same layout, exclusive scan in column-major order (column outer, chunk inner)
    int32_t *idx;
    int64_t idx_cap;
    int64_t *counts;
    // Compact mode (fd_lsd_lines): no dense maps (norm/angle/valid null); the scatter writes, per valid
    // pixel in scan order, its map index, norm and angle into one list for the whole batch, frame f's
    // run starting at frame_base[f] (exclusive scan of counts, k_lsd_frames). Null = per-frame idx_cap.
    float *lnorm;
    float *langle;
    int64_t *frame_base;
};

struct BriefArgs {
    const uint8_t *frames;
    int batch, rows, cols;
    const float *uv;        // [batch][stride][2] (x, y)
    const int32_t *counts;  // [batch] or null (= stride)
    int stride;
    int length, half, sampler;
    uint32_t *out_bits;  // [batch][stride][ceil(length / 32)]
    uint8_t *out_valid;  // [batch][stride] or null
};

// SuperPoint heatmap -> candidate lists (the K1 list format + level-0 histogram), for K4.
struct HeatArgs {
    const float *heat;  // [batch][rows][cols]
    int batch, rows, cols;
    int blocks_per_frame;
    float thr;
    int border;            // kInvalidBoundary: rows/cols within it are masked out
    const uint32_t *mask;  // prior-feature bitmap (null = none)
    int mask_wpr;
    float *list_resp;
    uint32_t *list_idx;
    int64_t list_cap;
    uint32_t *list_count;
    uint32_t *hist0;
    uint32_t key_base;
    int key_lz;
    float vmax;           // values above it set bit 31 of value_flag[f] (the key map assumes <= vmax)
    uint32_t *value_flag;  // [batch], the selection control block's pre_count words (gather disabled)
};

// Bilinear descriptor sampling from the 1/8-resolution descriptor map.
struct NnDescArgs {
    const float *map;  // [batch][channels][map_rows][map_cols], or [batch][map_rows][map_cols][channels] (nhwc)
    int batch, channels, map_rows, map_cols;
    int nhwc;
    const float *xy;        // [batch][stride][2]
    const int32_t *counts;  // [batch] or null (= stride)
    int stride;
    float *out;  // [batch][stride][channels]
};

// Launchers (stream-ordered, no allocation, no synchronisation: graph-capturable).
hipError_t launch_mask_boxes(const float *prior_xy, const int32_t *prior_frame, int n_prior, int dist, int rows,
                             int cols, uint32_t *mask, int mask_wpr, hipStream_t s);
hipError_t launch_fast_mask_scan(const uint32_t *mask, int mask_wpr, int batch, int rows, int cols, int32_t *row_base,
                                 int32_t *word_pref, hipStream_t s);
hipError_t launch_corner(int kind, bool raster, const PointsArgs &a, hipStream_t s);
hipError_t launch_corner_lp_any(int kind, const PointsArgs &a, hipStream_t s);  // k_corner_lp (a.px != 0)
hipError_t launch_fast(bool raster, const PointsArgs &a, const FastOffsets &off, hipStream_t s);
hipError_t launch_select(const SelectArgs &a, int batch, hipStream_t s);  // k_gather (a.pre_keys) / k_wide_gather (a.wide_count) + k_select
hipError_t launch_select_ordered(const SelectArgs &a, const OrderedArgs &o, int n_frames, hipStream_t s);
// libstdc++ std::sort order emulated on the GPU for the frames k_select flagged (FD_FRAME_TIES)
// wide: run the multi-workgroup prelude first (r.ctl, r.wcnt set): frames of >= 1 Mpx
hipError_t launch_select_reference(const SelectArgs &a, const RefSortArgs &r, int batch, bool wide, hipStream_t s);
// fd_lsd_lines: the reference's seed order (std::sort of the scan-ordered valid list by norm, descending,
// feature_line_detector.cpp:88-94) of every frame into r.ord: the compact lists (frame_base, idx, lnorm)
// into the list format of `a` (push order), then k_select_reference with order_only.
hipError_t launch_lsd_seed_order(const int64_t *frame_base, const int32_t *idx, const float *lnorm, const SelectArgs &a,
                                 const RefSortArgs &r, int batch, bool wide, hipStream_t s);
hipError_t launch_cand_lists(const CandInArgs &a, int64_t max_count, hipStream_t s);
hipError_t launch_nn_pick(const NnPickArgs &a, hipStream_t s);
hipError_t launch_compact(const CompactArgs &a, int batch, hipStream_t s);
hipError_t launch_lsd(const LsdArgs &a, hipStream_t s);
hipError_t launch_lsd_count(const LsdArgs &a, hipStream_t s);    // compact mode: map (counts, row bits) + scans
hipError_t launch_lsd_scatter(const LsdArgs &a, hipStream_t s);  // compact mode: the lists
hipError_t launch_brief(const BriefArgs &a, hipStream_t s);
hipError_t launch_heat_candidates(const HeatArgs &a, hipStream_t s);
int heat_blocks_per_frame(int64_t npx);
hipError_t launch_nn_desc(const NnDescArgs &a, hipStream_t s);
// SuperPoint heads: softmax + dustbin drop + pixel_shuffle(8) of the fp16 channels-last logits
// [n][hc][wc][65] into heat [n][8hc][8wc] f32; L2 normalisation of fp16 channels-last cells [cells][c]
// into f32 (c a multiple of 8)
// (bias, optional: the preceding convolution's bias added to its half output first, in half)
hipError_t launch_nn_heat_softmax(const void *semi, const void *bias, float *heat, int n, int hc, int wc, hipStream_t s);
hipError_t launch_nn_desc_normalize(const void *x, const void *bias, float *y, int64_t cells, int c, hipStream_t s);
// (w1, b1 non-null: x is the one-channel frame and conv1a -- 1 -> 64, 3x3, bias, ReLU -- is fused in)
hipError_t launch_conv3x3_c64(const void *x, const void *wpk, const void *bias, void *y, int n, int h, int w, int pool,
                              int y_channels, int y_offset, hipStream_t s);
hipError_t launch_conv3x3_c1_bias_relu(const void *x, const void *wt, const void *bias, void *y, int n, int h, int w,
                                       int c, hipStream_t s);
hipError_t launch_bias_relu(const void *x, const void *bias, void *y, int n, int h, int w, int c, int pool,
                            hipStream_t s);
// Interleaved 8-bit samples (channels 1-4) of npx pixels -> gray frames (fd_gray.hip).
hipError_t launch_rgb_gray(const uint8_t *src, int channels, uint8_t *dst, int64_t npx, hipStream_t s);

}  // namespace fdk
