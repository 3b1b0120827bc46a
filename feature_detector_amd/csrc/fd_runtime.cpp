// Host runtime of libfdhip.so: the C ABI declared in include/fd_hip.h.
// Owns the per-context stream and grow-only device workspace, stages host buffers, builds the FAST
// offset table and launches the kernels of fd_points.hip / fd_lsd.hip in stream order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fd_hip.h"
#include "fd_kernels.h"
#include "fd_lines.h"
#include "fd_png.h"

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t n = 0;
};

struct HostBuf {  // pinned host memory (hipHostMalloc), grow-only
    void *p = nullptr;
    size_t n = 0;
};

}  // namespace

struct fd_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;
    // workspace
    DevBuf frames, prior_xy, prior_frame, prior_counts, mask, row_base, word_pref;
    DevBuf list_resp, list_idx, out_xy, out_counts, grid;
    // selection control block: [batch][kHistBins] level-0 histograms, then list_count per frame.
    // Zero between calls: k_select resets what a call used. sel_dirty marks a call whose kernels may
    // not have run to the end (the next call clears the block first).
    DevBuf selctl, pre_keys, wide_keys, segdesc, seghead;
    bool sel_dirty = true;
    DevBuf seg_cnt, seg, resp_map, c_resp, c_x, c_y, c_counts;
    DevBuf l_norm, l_angle, l_valid, l_cnt, l_base, l_idx, l_counts, l_bits;
    DevBuf b_uv, b_counts, b_bits, b_valid;
    DevBuf n_heat, n_map, n_xy, n_counts, n_out;
    DevBuf dbg;
    // per-frame status of the last selection call: [batch] FD_FRAME_* flags, then [batch] candidate
    // counts (internal); status_batch = its frame count (0: no selection call yet)
    DevBuf status;
    int status_batch = 0;
    int tie_order = FD_TIES_RASTER;
    DevBuf ord, ord_meta;  // FD_TIES_REFERENCE host path: host-computed visiting orders of flagged frames
    DevBuf r_x, r_lpos, r_rpos, r_ord, r_ctl, r_wcnt, r_wfr;  // FD_TIES_REFERENCE on the GPU (k_select_reference scratch)
    DevBuf run_lut;        // FAST score per 16-bit ring mask (FastOffsets::run_lut), filled once
    DevBuf fast_cut;       // FAST emission cut: two float words, read / proposed alternately per call
    int fast_cut_parity = 0;
    // fd_lsd_lines: compact lists (device), their pinned host copies, frame 0's final state
    // (l_lists: one buffer of three sections, map index | norm | angle, copied back in one transfer)
    DevBuf l_lists, l_fbase;
    HostBuf h_lists;
    // fd_lsd_lines' seed order on the GPU: lists in the selection's format, status + counts, the orders'
    // and statuses' pinned host copies; a side stream (the sort overlaps the lists' copy and the host
    // setup) and its two events (lists ready -> sort; sort copied back)
    DevBuf l_sresp, l_sidx, l_sst;
    HostBuf h_ord, h_sst;
    hipStream_t aux = nullptr;
    hipEvent_t l_ev0 = nullptr, l_ev1 = nullptr;
    HostBuf h_png;  // fd_png_frames: decoded samples of a batch (pinned)
    // host-output selection calls: status words, counts and features come back in one copy into h_res
    // (pinned); the status words stay cached on the host (h_status) for fd_ctx_frame_status until the
    // next selection call
    HostBuf h_res;
    std::vector<uint32_t> h_status;
    bool h_status_valid = false;
    DevBuf d_png;
    std::vector<int32_t> st_idx;
    std::vector<float> st_norm, st_angle;
    std::vector<uint8_t> st_used;
    bool run_lut_ready = false;
    hipEvent_t xev = nullptr;  // orders a stream switch after the old stream's work (fd_ctx_set_stream)
    // FAST offset table cache
    int64_t off_n = -1;
    float off_thr = 0.0f;
    fdk::FastOffsets off{};
};

namespace {

// A/B and diagnostic switches (FD_PX, FD_TILE_H, FD_SELECT_STAMPS, ...) take effect only when FD_DEBUG_AB is
// set as well, so a stray variable in a user's environment cannot change the library's code path.
const char *ab_env(const char *name) {
    const char *on = std::getenv("FD_DEBUG_AB");
    if (!on || !*on || std::strcmp(on, "0") == 0) return nullptr;
    return std::getenv(name);
}

int fail(fd_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    return code;
}

#define FD_HIP_TRY(ctx, expr)                                                                                    \
    do {                                                                                                         \
        hipError_t e_ = (expr);                                                                                  \
        if (e_ != hipSuccess)                                                                                    \
            return fail((ctx), FD_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));                   \
    } while (0)

// Grow-only workspace. Growing while the context stream is being captured into a HIP graph would put
// an allocation into the capture: that fails here with hipErrorStreamCaptureUnsupported (reserve the
// shape first, fd_ctx_reserve, or run the call once before capturing).
hipError_t ensure(fd_ctx *c, DevBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.n >= bytes) return hipSuccess;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (c && c->stream && hipStreamIsCapturing(c->stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
        return hipErrorStreamCaptureUnsupported;
    if (b.p) {
        hipError_t e = hipFree(b.p);
        if (e != hipSuccess) return e;
        b.p = nullptr;
        b.n = 0;
    }
    const size_t want = bytes + 256;  // slack: whole-dword loads near the end stay inside the allocation
    hipError_t e = hipMalloc(&b.p, want);
    if (e != hipSuccess) return e;
    b.n = want;
    return hipSuccess;
}

hipError_t ensure_host(HostBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.n >= bytes) return hipSuccess;
    if (b.p) {
        hipError_t e = hipHostFree(b.p);
        if (e != hipSuccess) return e;
        b.p = nullptr;
        b.n = 0;
    }
    const size_t want = bytes + bytes / 4;  // headroom: batches vary in valid-pixel counts
    hipError_t e = hipHostMalloc(&b.p, want, hipHostMallocDefault);
    if (e != hipSuccess) return e;
    b.n = want;
    return hipSuccess;
}

void release(HostBuf &b) {
    if (b.p) (void)hipHostFree(b.p);
    b.p = nullptr;
    b.n = 0;
}

void release(DevBuf &b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.n = 0;
}

template <typename T>
T *as(DevBuf &b) {
    return static_cast<T *>(b.p);
}

// Tile height: a multiple of `period` (3 for the corner walk, 7 for FAST) that still gives the launch
// enough waves to fill 256 CUs, capped so halo rows stay a small overhead.
int choose_tile_h(int64_t batch, int tiles_x, int out_rows, int period, int max_mult) {
    int64_t target_waves = 10240;  // ~2 rounds of resident waves at 256 CUs (measured sweep)
    if (const char *e = ab_env("FD_TARGET_WAVES")) target_waves = std::max<int64_t>(1, std::atoll(e));  // tuning
    if (const char *e = ab_env("FD_TILE_MULT")) max_mult = std::max(1, std::atoi(e));                   // tuning
    int64_t h = (batch * tiles_x * static_cast<int64_t>(out_rows)) / target_waves;
    if (h < period && period == 6) {
        // small launches: the tile's serial row chain is the latency; 3 rows (9 steps of the 6-row
        // ring, the loop stops early) measured best at 640x480 batch 1 (tile_h 6/4/3/2/1: K1 11.4 /
        // 10.3 / 10.1 / 10.2 / 13.2 us, and k_select grows with the number of segments below 3)
        h = 3;
    } else {
        h = std::max<int64_t>(h, period);
        h = ((h + period - 1) / period) * period;
    }
    h = std::min<int64_t>(h, static_cast<int64_t>(period) * max_mult);
    if (const char *e = ab_env("FD_TILE_H")) h = std::max(1, std::atoi(e));  // tuning (A/B)
    return static_cast<int>(h);
}

// FAST running offset o_0 = 1e-5f, o_{k+1} = fl(o_k + 1e-5f) (feature_point_fast_detector.cpp:85,93)
// as runs of constant increment; verified exact against the recurrence before use.
// FAST score table (FastOffsets::run_lut): for every 16-bit ring mask, the reference's two-pass count
// (feature_point_fast_detector.cpp:55-78) of consecutive set bits, run over the mask twice without a
// reset between the passes (so a run may wrap around), stopping once 16 is reached.
int ensure_run_lut(fd_ctx *c) {
    if (c->run_lut_ready) return FD_OK;
    FD_HIP_TRY(c, ensure(c, c->run_lut, 65536));
    std::vector<uint8_t> table(65536);
    for (uint32_t b = 0; b < 65536; ++b) {
        int run = 0, best = 0;
        for (int pass = 0; pass < 2 && best < 16; ++pass)
            for (int k = 0; k < 16; ++k) {
                run = ((b >> k) & 1u) ? run + 1 : 0;
                best = std::max(best, run);
            }
        table[b] = static_cast<uint8_t>(std::min(best, 16));
    }
    FD_HIP_TRY(c, hipMemcpyAsync(c->run_lut.p, table.data(), 65536, hipMemcpyHostToDevice, c->stream));
    FD_HIP_TRY(c, hipStreamSynchronize(c->stream));  // the host table dies with this call
    c->run_lut_ready = true;
    return FD_OK;
}

int build_offsets(fd_ctx *c, int64_t n, float thr) {
    int rc = ensure_run_lut(c);
    if (rc) return rc;
    c->off.run_lut = as<uint8_t>(c->run_lut);
    if (c->off_n == n && c->off_thr == thr) return FD_OK;
    fdk::FastOffsets o{};
    o.nseg = 0;
    o.k0 = std::numeric_limits<int64_t>::max();
    std::vector<float> seq(static_cast<size_t>(std::max<int64_t>(n, 1)));
    float v = 1e-5f;
    double prev_inc = -1.0;
    for (int64_t k = 0; k < n; ++k) {
        seq[static_cast<size_t>(k)] = v;
        const float next = v + 1e-5f;
        const double inc = static_cast<double>(next) - static_cast<double>(v);
        if (k == 0 || inc != prev_inc) {
            if (o.nseg >= fdk::kMaxOffsetSegs) return fail(c, FD_ERR_INVALID, "FAST offset table too large");
            o.k_start[o.nseg] = k;
            o.o_start[o.nseg] = static_cast<double>(v);
            o.inc[o.nseg] = inc;
            ++o.nseg;
            prev_inc = inc;
        }
        if (o.k0 == std::numeric_limits<int64_t>::max() && v > thr) o.k0 = k;
        v = next;
    }
    if (o.nseg == 0) {
        o.nseg = 1;
        o.k_start[0] = 0;
        o.o_start[0] = 1e-5;
        o.inc[0] = 0.0;
    }
    int s = 0;
    for (int64_t k = 0; k < n; ++k) {
        while (s + 1 < o.nseg && o.k_start[s + 1] <= k) ++s;
        const float r = static_cast<float>(o.o_start[s] + static_cast<double>(k - o.k_start[s]) * o.inc[s]);
        if (r != seq[static_cast<size_t>(k)]) return fail(c, FD_ERR_INVALID, "FAST offset table not exact");
    }
    o.run_lut = as<uint8_t>(c->run_lut);
    c->off = o;
    c->off_n = n;
    c->off_thr = thr;
    return FD_OK;
}

struct PriorInfo {
    int64_t total = 0;
    const uint32_t *mask = nullptr;
    const int32_t *counts_dev = nullptr;
    int wpr = 0;
};

// Upload prior features and draw their boxes into the mask bitmap (feature_point_detector.cpp:90-98).
int setup_priors(fd_ctx *c, int batch, int rows, int cols, int dist, const float *prior_xy,
                 const int32_t *prior_counts, PriorInfo &pi) {
    pi = PriorInfo{};
    if (prior_counts == nullptr) return FD_OK;
    std::vector<int32_t> frame_of;
    for (int b = 0; b < batch; ++b) {
        if (prior_counts[b] < 0) return fail(c, FD_ERR_INVALID, "negative prior count");
        pi.total += prior_counts[b];
    }
    FD_HIP_TRY(c, ensure(c, c->prior_counts, sizeof(int32_t) * batch));
    FD_HIP_TRY(c, hipMemcpyAsync(c->prior_counts.p, prior_counts, sizeof(int32_t) * batch, hipMemcpyHostToDevice,
                                 c->stream));
    pi.counts_dev = as<int32_t>(c->prior_counts);
    if (pi.total == 0) {
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));  // prior_counts is caller-owned host memory
        return FD_OK;
    }
    if (prior_xy == nullptr) return fail(c, FD_ERR_INVALID, "prior_xy is NULL but prior_counts is not zero");
    frame_of.reserve(static_cast<size_t>(pi.total));
    for (int b = 0; b < batch; ++b)
        for (int i = 0; i < prior_counts[b]; ++i) frame_of.push_back(b);
    pi.wpr = (cols + 31) / 32;
    const size_t mbytes = sizeof(uint32_t) * static_cast<size_t>(batch) * rows * pi.wpr;
    FD_HIP_TRY(c, ensure(c, c->prior_xy, sizeof(float) * 2 * pi.total));
    FD_HIP_TRY(c, ensure(c, c->prior_frame, sizeof(int32_t) * pi.total));
    FD_HIP_TRY(c, ensure(c, c->mask, mbytes));
    FD_HIP_TRY(c, hipMemcpyAsync(c->prior_xy.p, prior_xy, sizeof(float) * 2 * pi.total, hipMemcpyHostToDevice,
                                 c->stream));
    FD_HIP_TRY(c, hipMemcpyAsync(c->prior_frame.p, frame_of.data(), sizeof(int32_t) * pi.total,
                                 hipMemcpyHostToDevice, c->stream));
    FD_HIP_TRY(c, hipMemsetAsync(c->mask.p, 0xFF, mbytes, c->stream));
    FD_HIP_TRY(c, fdk::launch_mask_boxes(as<float>(c->prior_xy), as<int32_t>(c->prior_frame),
                                         static_cast<int>(pi.total), dist, rows, cols, as<uint32_t>(c->mask), pi.wpr,
                                         c->stream));
    // The synchronous copies above read host memory that the caller may free after return.
    FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
    pi.mask = as<uint32_t>(c->mask);
    return FD_OK;
}

int check_shape(fd_ctx *c, int kind, int batch, int rows, int cols, bool points = true) {
    if (!c) return FD_ERR_INVALID;
    if (kind < FD_HARRIS || kind > FD_FAST) return fail(c, FD_ERR_INVALID, "unknown detector kind");
    if (batch < 1 || rows < 1 || cols < 1) return fail(c, FD_ERR_INVALID, "batch, rows and cols must be >= 1");
    // the selection grid packs (x, y) into 16 bits each
    if (points && (rows > 65535 || cols > 65535)) return fail(c, FD_ERR_INVALID, "rows and cols must be <= 65535");
    if (static_cast<int64_t>(rows) * cols >= (int64_t(1) << 31)) return fail(c, FD_ERR_INVALID, "frame too large");
    return FD_OK;
}

// Stage the frames on the device (or use the caller's device pointer).
int stage_frames(fd_ctx *c, const uint8_t *frames, int on_device, int batch, int rows, int cols,
                 const uint8_t *&dframes) {
    if (frames == nullptr) return fail(c, FD_ERR_INVALID, "frames is NULL");  // feature_point_detector.cpp:9
    const size_t bytes = static_cast<size_t>(batch) * rows * cols;
    if (on_device) {
        dframes = frames;
        return FD_OK;
    }
    FD_HIP_TRY(c, ensure(c, c->frames, bytes));
    FD_HIP_TRY(c, hipMemcpyAsync(c->frames.p, frames, bytes, hipMemcpyHostToDevice, c->stream));
    dframes = as<uint8_t>(c->frames);
    return FD_OK;
}

// Geometry of the per-pixel launch for a detector kind.
struct PointGeom {
    int border;    // 2 for Harris/Shi-Tomasi, 3 for FAST
    int out_rows;  // rows of the candidate region
    int tiles_x, tiles_y, tile_h;
    int blocks_per_frame;
    bool empty;
};

// Columns per lane of k_corner_lp for a corner launch in list mode (fd_points_detect /
// fd_points_response); 0 = k_corner (FAST, negative thresholds, the raster-ordered candidate stage).
// Large launches take wide lanes (the halo exchanges and loop control shared by more pixels), small
// ones narrow lanes (more waves, shorter serial row chains). FD_PX overrides (A/B).
int corner_px(int kind, int batch, int rows, int cols, float thr) {
    if (kind == FD_FAST || !(thr >= 0.0f)) return 0;
    // k_corner_lp addresses a frame's list through a buffer resource: list_cap * 4 bytes < 2^32
    if (static_cast<int64_t>(rows) * cols >= (int64_t(1) << 30)) return 0;
    if (const char *e = ab_env("FD_PX")) {
        const int v = std::atoi(e);
        if (v == 0 || v == 2 || v == 4 || v == 8) return v;
    }
    // Measured (north-star shape, 1080p x 256): 4 columns per lane 4-5 % faster than k_corner, 8 slower
    // (VGPR-limited to 3 waves per SIMD); at 640x480 x 1 k_corner is faster (11.4 vs 10.0 us).
    const int64_t px = static_cast<int64_t>(batch) * rows * cols;
    return px >= (int64_t(1) << 21) ? 4 : 0;
}

PointGeom point_geom(int kind, int batch, int rows, int cols, int px = 0) {
    PointGeom g{};
    g.border = kind == FD_FAST ? 3 : 2;
    g.out_rows = rows - 2 * g.border;
    const int out_cols = cols - 2 * g.border;
    g.empty = g.out_rows <= 0 || out_cols <= 0;
    const int tw = px ? fdk::lp_tile_w(px) : fdk::kTileW;
    g.tiles_x = std::max(1, (cols - g.border + tw - 1) / tw);
    const int period = kind == FD_FAST ? 7 : 6;  // rows per unrolled loop iteration of the kernel
    g.tile_h = choose_tile_h(batch, g.tiles_x, std::max(g.out_rows, 1), period, kind == FD_FAST ? 9 : 100);
    g.tiles_y = std::max(1, (std::max(g.out_rows, 1) + g.tile_h - 1) / g.tile_h);
    g.blocks_per_frame = (g.tiles_x * g.tiles_y + 3) / 4;
    return g;
}

int64_t detect_list_cap(int kind, int rows, int cols) {
    const int64_t px = static_cast<int64_t>(rows) * cols;
    return (kind == FD_FAST ? px : px / 2) + 64;
}

struct SelectBufs {
    uint32_t *hist0, *list_count, *pre_count, *seg_bad, *wide_count, *wide_cut, *skipped;
    uint64_t *pre_keys, *wide_keys;
    uint32_t *status, *cand_n;
};

// Candidate lists and the (self-resetting) control block for `batch` frames.
int select_buffers(fd_ctx *c, int batch, int64_t cap, SelectBufs &sb) {
    FD_HIP_TRY(c, ensure(c, c->list_resp, sizeof(float) * cap * batch));
    FD_HIP_TRY(c, ensure(c, c->list_idx, sizeof(uint32_t) * cap * batch));
    FD_HIP_TRY(c, ensure(c, c->pre_keys, sizeof(uint64_t) * fdk::kSelectChunk * batch));
    FD_HIP_TRY(c, ensure(c, c->wide_keys, sizeof(uint64_t) * fdk::kWideKeys * batch));
    const size_t ctl = sizeof(uint32_t) * static_cast<size_t>(batch) * (fdk::kHistBins + 6);
    if (c->selctl.n < ctl) {
        FD_HIP_TRY(c, ensure(c, c->selctl, ctl));
        c->sel_dirty = true;
    }
    if (c->sel_dirty) {
        FD_HIP_TRY(c, hipMemsetAsync(c->selctl.p, 0, c->selctl.n, c->stream));
        c->sel_dirty = false;
    }
    uint32_t *base = as<uint32_t>(c->selctl);
    sb.hist0 = base;
    sb.list_count = base + static_cast<size_t>(batch) * fdk::kHistBins;
    sb.pre_count = sb.list_count + batch;
    sb.seg_bad = sb.pre_count + batch;
    sb.wide_count = sb.seg_bad + batch;
    sb.wide_cut = sb.wide_count + batch;
    sb.skipped = sb.wide_cut + batch;
    sb.pre_keys = as<uint64_t>(c->pre_keys);
    sb.wide_keys = as<uint64_t>(c->wide_keys);
    FD_HIP_TRY(c, ensure(c, c->status, sizeof(uint32_t) * 2 * static_cast<size_t>(batch)));
    sb.status = as<uint32_t>(c->status);
    sb.cand_n = sb.status + batch;
    return FD_OK;
}

uint32_t host_float_key(float f) {
    uint32_t u;
    std::memcpy(&u, &f, sizeof(u));
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Key map of the selection (SelectArgs::key_base / key_lz): candidates have responses in
// (thr, rmax], rmax = +inf for the corner detectors and 16 + the largest FAST offset (+1) for FAST.
void key_map(int kind, float thr, const fdk::FastOffsets *off, int64_t n_off, uint32_t &base, int &lz) {
    base = host_float_key(thr);
    uint32_t kmax = host_float_key(std::numeric_limits<float>::infinity());
    if (kind == FD_FAST && off && off->nseg > 0 && n_off > 0) {
        const int s = off->nseg - 1;
        const double omax = off->o_start[s] + static_cast<double>(n_off - 1 - off->k_start[s]) * off->inc[s];
        kmax = std::max(base, host_float_key(static_cast<float>(16.0 + omax + 1.0)));
    }
    lz = kmax > base ? __builtin_clz(kmax - base) : 0;
}

// Inputs of the selection stage (K4) after a candidate kernel filled the lists of `sb`.
struct SelectCall {
    int batch = 0, rows = 0, cols = 0, dist = 0;
    uint32_t need = 0;
    int64_t cap = 0;
    uint32_t key_base = 0;
    int key_lz = 0;
    int tie_idx_desc = 0;  // equal responses: raster index descending (SuperPoint multimap) instead of ascending
    bool wide_eager = false;  // FAST: the wide pass comes with the first chunk (SelectArgs::wide_eager)
    bool value_flag = false;  // the candidate kernel flags out-of-range values in pre_count (gather kernel off)
    const uint2 *segdesc = nullptr;  // sorted segments of the candidate kernel (PointsArgs::segdesc)
    const uint64_t *seghead = nullptr;
    int nseg = 0;
    bool push_order = false;  // lists hold the caller's push order (fd_points_select), not raster order
    bool dup_keys = false;    // a pixel may be listed twice with one response (caller lists): equal keys
    bool grid_at_d0 = false;  // distance 0 tests the grid too (1-pixel cells; set with push_order)
    // FAST emission cut (PointsArgs::emit_cut): the per-pixel launch of this call (re-run for the frames
    // the selection flags, kFrameRedo), its offsets, the skipped counters and the cut words
    const fdk::PointsArgs *redo_points = nullptr;
    const fdk::FastOffsets *redo_off = nullptr;
    uint32_t *skipped = nullptr;
    const uint32_t *cut_cur = nullptr;
    uint32_t *cut_next = nullptr;
    const char *value_msg = "a value above the declared maximum (fd_nn_opts::max_response)";
};

// Sorted-segment lists (PointsArgs::segdesc): for launches small enough that k_select can give every
// workgroup segment of a frame its own threads (<= kSelectThreads segments per frame) and that would
// otherwise gather their first chunk inside k_select (no k_gather kernel). FD_SEG_LISTS=0: off (A/B).
bool use_seg_lists(int blocks_per_frame, int rows, int cols) {
    if (const char *e = ab_env("FD_SEG_LISTS"); e && std::atoi(e) == 0) return false;
    return blocks_per_frame <= fdk::kSelectThreads && static_cast<int64_t>(rows) * cols < (1 << 20);
}

std::string hex(uint32_t v) {
    char t[16];
    std::snprintf(t, sizeof t, "%x", v);
    return std::string(t);
}

// Scratch of k_select_reference for `batch` frames of lists of `cap` entries.
int ref_buffers(fd_ctx *c, int batch, int rows, int cols, int64_t cap, fdk::RefSortArgs &r) {
    const int64_t words = (static_cast<int64_t>(rows) * cols + 31) / 32;
    const int64_t rcap = std::max<int64_t>({cap, words, 1});
    const size_t n = static_cast<size_t>(rcap) * static_cast<size_t>(batch);
    FD_HIP_TRY(c, ensure(c, c->r_x, sizeof(uint2) * n));
    FD_HIP_TRY(c, ensure(c, c->r_lpos, sizeof(uint32_t) * n));
    FD_HIP_TRY(c, ensure(c, c->r_rpos, sizeof(uint32_t) * n));
    FD_HIP_TRY(c, ensure(c, c->r_ord, sizeof(uint32_t) * n));
    FD_HIP_TRY(c, ensure(c, c->r_ctl, sizeof(fdk::RefCtl) * static_cast<size_t>(batch)));
    FD_HIP_TRY(c, ensure(c, c->r_wcnt, sizeof(uint32_t) * 2 * fdk::kRefWideGroups * static_cast<size_t>(batch)));
    r.ctl = as<fdk::RefCtl>(c->r_ctl);
    r.wcnt = as<uint32_t>(c->r_wcnt);
    FD_HIP_TRY(c, ensure(c, c->r_wfr, sizeof(uint32_t) * (1 + static_cast<size_t>(batch))));
    r.wfr = as<uint32_t>(c->r_wfr);
    r.x = as<uint2>(c->r_x);
    r.lpos = as<uint32_t>(c->r_lpos);
    r.rpos = as<uint32_t>(c->r_rpos);
    r.ord = as<uint32_t>(c->r_ord);
    r.cap = rcap;
    // diagnostic (FD_DEBUG_AB=1): a low bound on k_select_reference's window x level loop, so that tests
    // reach its failure path (FD_FRAME_UNRESOLVED, host fallback) on small inputs
    if (const char *e = ab_env("FD_REF_GUARD")) r.guard_limit = std::max(0, std::atoi(e));
    return FD_OK;
}

// FD_TIES_REFERENCE (fd_ctx_set_tie_order): frames whose greedy scan met equal responses
// (FD_FRAME_TIES from k_select) are selected again in the reference's own order. The reference sorts
// its raster-ordered candidates with an unstable std::sort (feature_point_detector.cpp:58-60), whose
// permutation of equal responses is defined only by libstdc++'s introsort run on that exact sequence:
// the frame's candidate list (still in the workspace, unordered) is copied back, put in raster order
// (the order ComputeCandidates pushes them, feature_point_harris_detector.cpp:120-137,
// feature_point_fast_detector.cpp:83-98), sorted here with std::sort and the reference comparator,
// and the resulting visiting order goes back to the GPU for the greedy pass (k_select_ordered).
// `which` selects the frames: FD_FRAME_TIES (FD_TIES_HOST=1: the host path for every flagged frame) or
// FD_FRAME_UNRESOLVED (the frames k_select_reference left to the host).
int resolve_ties(fd_ctx *c, fdk::SelectArgs s, int batch, const SelectBufs &sb, bool push_order, uint32_t which) {
    // The status read below synchronises the stream, which a stream being captured into a graph cannot
    // do (and the host sort could not be replayed): refuse before touching the capture.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    FD_HIP_TRY(c, hipStreamIsCapturing(c->stream, &cap));
    if (cap != hipStreamCaptureStatusNone)
        return fail(c, FD_ERR_INVALID, "FD_TIES_REFERENCE synchronises (status read, host std::sort): not allowed "
                                       "during stream capture; use FD_TIES_RASTER and read FD_FRAME_TIES");
    std::vector<uint32_t> st(2 * static_cast<size_t>(batch));
    FD_HIP_TRY(c, hipMemcpyAsync(st.data(), sb.status, sizeof(uint32_t) * st.size(), hipMemcpyDeviceToHost, c->stream));
    FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
    std::vector<int32_t> frames;
    for (int b = 0; b < batch; ++b) {
        if (st[b] & FD_FRAME_GUARD)  // (read here anyway: reported for device outputs too)
            return fail(c, FD_ERR_HIP, "internal: selection consistency guard tripped (status 0x" + hex(st[b]) +
                                           ", frame " + std::to_string(b) + ")");
        if (st[b] & which) frames.push_back(b);
    }
    if (frames.empty()) return FD_OK;
    struct Cand {
        float resp;
        uint32_t idx;
    };
    std::vector<std::vector<Cand>> lists(frames.size());
    std::vector<std::vector<float>> resp(frames.size());
    std::vector<std::vector<uint32_t>> idx(frames.size());
    for (size_t j = 0; j < frames.size(); ++j) {
        const int f = frames[j];
        const size_t n = std::min<size_t>(st[batch + f], static_cast<size_t>(s.list_cap));
        resp[j].resize(n);
        idx[j].resize(n);
        const size_t o = static_cast<size_t>(f) * static_cast<size_t>(s.list_cap);
        FD_HIP_TRY(c, hipMemcpyAsync(resp[j].data(), s.list_resp + o, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
        FD_HIP_TRY(c, hipMemcpyAsync(idx[j].data(), s.list_idx + o, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, c->stream));
    }
    FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
    std::vector<uint32_t> order;
    std::vector<int64_t> offset(frames.size());
    std::vector<uint32_t> count(frames.size());
    for (size_t j = 0; j < frames.size(); ++j) {
        std::vector<Cand> &v = lists[j];
        v.resize(resp[j].size());
        for (size_t i = 0; i < v.size(); ++i) v[i] = {resp[j][i], idx[j][i]};
        // the order ComputeCandidates pushed them in -- raster order for the built-in detectors (their
        // indices are unique; the lists are unordered), the list order for caller-supplied candidates
        // (fd_points_select keeps it) -- then the reference's sort (:58-60)
        // (raster order of unique indices: any sort gives it; an LSD radix sort, 3 x 11 bits, is ~20x
        // faster than std::sort here and leaves the reference's own std::sort below as the cost)
        if (!push_order) {
            std::vector<Cand> tmp(v.size());
            for (int shift = 0; shift < 33; shift += 11) {
                uint32_t hist[2049] = {};
                for (const Cand &e : v) ++hist[((e.idx >> shift) & 2047u) + 1];
                for (int k = 0; k < 2048; ++k) hist[k + 1] += hist[k];
                for (const Cand &e : v) tmp[hist[(e.idx >> shift) & 2047u]++] = e;
                v.swap(tmp);
            }
        }
        std::sort(v.begin(), v.end(), [](const Cand &a, const Cand &b) { return a.resp > b.resp; });
        offset[j] = static_cast<int64_t>(order.size());
        count[j] = static_cast<uint32_t>(v.size());
        for (const Cand &e : v) order.push_back(e.idx);
    }
    const size_t nf = frames.size();
    const size_t meta = (sizeof(int64_t) + sizeof(uint32_t) + sizeof(int32_t)) * nf;
    FD_HIP_TRY(c, ensure(c, c->ord, sizeof(uint32_t) * std::max<size_t>(order.size(), 1)));
    FD_HIP_TRY(c, ensure(c, c->ord_meta, meta));
    std::vector<uint8_t> mbuf(meta);
    std::memcpy(mbuf.data(), offset.data(), sizeof(int64_t) * nf);
    std::memcpy(mbuf.data() + sizeof(int64_t) * nf, count.data(), sizeof(uint32_t) * nf);
    std::memcpy(mbuf.data() + (sizeof(int64_t) + sizeof(uint32_t)) * nf, frames.data(), sizeof(int32_t) * nf);
    FD_HIP_TRY(c, hipMemcpyAsync(c->ord.p, order.data(), sizeof(uint32_t) * order.size(), hipMemcpyHostToDevice, c->stream));
    FD_HIP_TRY(c, hipMemcpyAsync(c->ord_meta.p, mbuf.data(), meta, hipMemcpyHostToDevice, c->stream));
    fdk::OrderedArgs o{};
    o.order = as<uint32_t>(c->ord);
    o.offset = reinterpret_cast<const int64_t *>(c->ord_meta.p);
    o.count = reinterpret_cast<const uint32_t *>(static_cast<uint8_t *>(c->ord_meta.p) + sizeof(int64_t) * nf);
    o.frame = reinterpret_cast<const int32_t *>(static_cast<uint8_t *>(c->ord_meta.p) +
                                                (sizeof(int64_t) + sizeof(uint32_t)) * nf);
    FD_HIP_TRY(c, fdk::launch_select_ordered(s, o, static_cast<int>(nf), c->stream));
    FD_HIP_TRY(c, hipStreamSynchronize(c->stream));  // the host vectors above are the copies' sources
    return FD_OK;
}

bool host_ties_env() {  // FD_TIES_HOST=1: the round-3 host path for every flagged frame (A/B and checker)
    static const bool v = ab_env("FD_TIES_HOST") && std::atoi(ab_env("FD_TIES_HOST")) != 0;
    return v;
}

// Calls that will synchronise the context stream (host outputs, or the host tie path) cannot run while
// that stream is being captured into a graph: refuse at entry, before any work is enqueued, so that a
// failed call leaves nothing half-recorded in the capture.
int refuse_sync_under_capture(fd_ctx *c, int outputs_on_device) {
    const bool syncs = !outputs_on_device || (c->tie_order == FD_TIES_REFERENCE && host_ties_env());
    if (!syncs || !c->stream) return FD_OK;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    FD_HIP_TRY(c, hipStreamIsCapturing(c->stream, &cap));
    if (cap != hipStreamCaptureStatusNone)
        return fail(c, FD_ERR_INVALID, "this call synchronises the stream (host outputs or FD_TIES_HOST): not allowed "
                                       "during stream capture; pass device outputs");
    return FD_OK;
}

// K4 (k_gather + k_select) on the candidate lists, features into out_xy / out_counts (device, or copied
// back to the host and checked when !outputs_on_device).
int run_select(fd_ctx *c, const SelectCall &q, const PriorInfo &pi, const SelectBufs &sb, float *out_xy,
               int32_t out_stride, int32_t *out_counts, int outputs_on_device, int frames_on_device) {
    fdk::SelectArgs s{};
    const int batch = q.batch, rows = q.rows, cols = q.cols;
    if (q.cap >= (int64_t(1) << 30))  // k_select reads the lists through buffer resources (byte offsets < 2^32)
        return fail(c, FD_ERR_INVALID, "candidate list capacity must be < 2^30 entries per frame");
    s.list_resp = as<float>(c->list_resp);
    s.list_idx = as<uint32_t>(c->list_idx);
    s.list_count = sb.list_count;
    s.hist0 = sb.hist0;
    s.list_cap = q.cap;
    s.rows = rows;
    s.cols = cols;
    s.batch = batch;
    s.tie_idx_desc = q.tie_idx_desc;
    s.value_flag = q.value_flag ? 1 : 0;
    s.mask = pi.mask;
    s.mask_wpr = pi.wpr;
    s.prior_counts = pi.counts_dev;
    s.need = q.need;
    s.dist = q.dist;
    s.grid_at_d0 = (q.push_order || q.grid_at_d0) ? 1 : 0;  // caller lists may name a pixel twice: distance 0 tests it
    s.dup_keys = q.dup_keys ? 1 : 0;
    if (s.dist >= 1 || (s.dist == 0 && s.grid_at_d0)) {
        s.grid_w = (cols + s.dist) / (s.dist + 1);
        s.grid_h = (rows + s.dist) / (s.dist + 1);
        const int64_t cells = static_cast<int64_t>(s.grid_w + 2) * (s.grid_h + 2);  // bordered grid
        if (cells > fdk::kGridLdsCells) {
            FD_HIP_TRY(c, ensure(c, c->grid, sizeof(uint32_t) * cells * batch));
            s.grid_global = as<uint32_t>(c->grid);
        }
    }
    float *dxy = out_xy;
    int32_t *dcnt = out_counts;
    c->h_status_valid = false;
    // Host outputs: the counts and features are written behind the status words (status | candidate
    // counts | feature counts | features, one buffer), so that all of it returns in one copy into
    // pinned memory and one synchronisation (three pageable copies and a status read cost ~40 us more
    // per 640x480 frame).
    const size_t res_head = (sizeof(uint32_t) * 3 * static_cast<size_t>(batch) + 15) & ~size_t(15);
    const size_t res_bytes = res_head + sizeof(float) * 2 * static_cast<size_t>(out_stride) * batch;
    SelectBufs sbl = sb;
    // In the raster tie order nothing after k_select changes the outputs: the kernel writes the features
    // and counts straight into the pinned result buffer and mirrors the status words there (no copy after
    // the kernel: ~6 us per 640x480 host frame). The reference order's pass rewrites them: copied as before.
    static const bool no_direct = ab_env("FD_HOST_DIRECT") && std::atoi(ab_env("FD_HOST_DIRECT")) == 0;  // (A/B)
    const bool direct = !outputs_on_device && c->tie_order != FD_TIES_REFERENCE && !no_direct;
    if (!outputs_on_device) {
        if (c->status.n < res_bytes) {  // (grow: the selection's status words move with it)
            FD_HIP_TRY(c, ensure(c, c->status, res_bytes));
            sbl.status = as<uint32_t>(c->status);
            sbl.cand_n = sbl.status + batch;
        }
        FD_HIP_TRY(c, ensure_host(c->h_res, res_bytes));
        uint8_t *const res = static_cast<uint8_t *>(direct ? c->h_res.p : c->status.p);
        dcnt = reinterpret_cast<int32_t *>(res + sizeof(uint32_t) * 2 * static_cast<size_t>(batch));
        dxy = reinterpret_cast<float *>(res + res_head);
    }
    s.status_host = direct ? static_cast<uint32_t *>(c->h_res.p) : nullptr;
    s.out_xy = dxy;
    s.out_stride = out_stride;
    s.out_counts = dcnt;
    s.key_base = q.key_base;
    s.key_lz = q.key_lz;
    s.status = sbl.status;
    s.cand_n = sbl.cand_n;
    // Small batches of large frames: spread the first chunk's gather over ~256 workgroups in its own
    // kernel (~9 us of fixed cost: pays off once one workgroup's pass over the list costs more, i.e.
    // from about a megapixel per frame; measured at 640x480: break-even).
    const bool big = static_cast<int64_t>(rows) * cols >= (1 << 20);
    s.gather_groups = big ? std::max(1, std::min(64, 256 / std::max(batch, 1))) : 1;
    if (const char *e = ab_env("FD_GATHER_GROUPS")) s.gather_groups = std::max(1, std::atoi(e));  // A/B
    if (q.value_flag) s.gather_groups = 1;  // pre_count carries the candidate kernel's flag instead
    s.pre_count = sb.pre_count;
    s.pre_keys = s.gather_groups > 1 ? sb.pre_keys : nullptr;
    s.seg_bad = sb.seg_bad;
    s.wide_keys = ab_env("FD_NO_WIDE") ? nullptr : sb.wide_keys;  // (A/B switch)
    // FAST's top responses are scores plus a slowly growing offset: thousands of candidates share the
    // top bins and the greedy scan runs over several chunks (1280x720 noise: ~5k), so the wide pass
    // comes with the first chunk; the corner detectors usually finish within it (wide pass deferred).
    s.wide_eager = q.wide_eager ? 1 : 0;
    if (q.skipped && ab_env("FD_CUT_NO_WIDE")) {  // (A/B: the cut's short lists gathered chunk by chunk instead)
        s.wide_keys = nullptr;
        s.wide_eager = 0;
        s.fast_sub = 1;
    }
    // ... and its list pass is spread over the frame's list by k_wide_gather, ~16k entries per workgroup
    // at FAST's ~30 % candidate density on noise (one workgroup read the whole list before: 1280x720,
    // ~55k of k_select's ~130k cycles per frame). FD_WIDE_GROUPS=0: off (A/B).
    // (not under FAST's emission cut: its lists of a few tens of thousands of keys are cheaper to pass once
    // inside k_select -- 85 us vs 73 + 13 + 5 us for k_select, k_wide_gather and k_wide_cut at configs[2])
    if (s.wide_eager && s.wide_keys && !s.pre_keys && !q.value_flag && !q.skipped) {
        const int64_t est = static_cast<int64_t>(rows) * cols * 3 / 10;
        s.wide_groups = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(64, (est + 16383) / 16384)));
        if (const char *e = ab_env("FD_WIDE_GROUPS")) s.wide_groups = std::max(0, std::atoi(e));
        if (s.wide_groups > 0) {
            s.wide_count = sb.wide_count;
            s.wide_cut = sb.wide_cut;
        }
    }
    if (q.segdesc && !s.pre_keys) {
        s.segdesc = q.segdesc;
        s.seghead = q.seghead;
        s.nseg = q.nseg;
    }
    s.first_sub = 1;
    if (const char *e = ab_env("FD_FIRST_SUB")) s.first_sub = std::atoi(e) != 0;  // (A/B switch)
    static const bool stamps = ab_env("FD_SELECT_STAMPS") != nullptr;
    if (stamps) {  // diagnostic build-free switch: phase clocks of k_select for frame 0
        FD_HIP_TRY(c, ensure(c, c->dbg, sizeof(uint64_t) * 32 * batch));
        FD_HIP_TRY(c, hipMemsetAsync(c->dbg.p, 0, sizeof(uint64_t) * 32 * batch, c->stream));
        s.stamps = as<uint64_t>(c->dbg);
    }
    s.skipped = q.skipped;
    s.cut_cur = q.cut_cur;
    s.cut_next = q.cut_next;
    FD_HIP_TRY(c, fdk::launch_select(s, batch, c->stream));
    if (q.redo_points) {
        // the frames whose selection ran out of emitted keys with candidates left below the cut (kFrameRedo):
        // detected again without the cut and selected again, in stream order; every other workgroup of
        // these launches exits at once (graph-capturable: no host round trip)
        fdk::PointsArgs pr = *q.redo_points;
        pr.emit_cut = nullptr;
        pr.emit_cut_next = nullptr;
        pr.skipped = nullptr;
        pr.redo_status = s.status;
        FD_HIP_TRY(c, fdk::launch_fast(false, pr, *q.redo_off, c->stream));
        fdk::SelectArgs s2 = s;
        s2.skipped = nullptr;
        s2.cut_cur = nullptr;
        s2.cut_next = nullptr;
        s2.redo_status = s.status;
        s2.stamps = nullptr;
        FD_HIP_TRY(c, fdk::launch_select(s2, batch, c->stream));
    }
    c->sel_dirty = false;
    c->status_batch = batch;
    if (stamps) {
        uint64_t h[32];
        FD_HIP_TRY(c, hipMemcpyAsync(h, c->dbg.p, sizeof(h), hipMemcpyDeviceToHost, c->stream));
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
        std::fprintf(stderr, "k_select cycles: init %llu hist0 %llu gather %llu subkeys %llu greedy %llu descent %llu "
                             "control %llu | chunks %llu descents %llu subchunks %llu | extract %llu runsort %llu merges %llu place %llu cmask %llu\n",
                     (unsigned long long)h[1], (unsigned long long)h[2], (unsigned long long)h[3],
                     (unsigned long long)h[4], (unsigned long long)h[5], (unsigned long long)h[6],
                     (unsigned long long)h[7], (unsigned long long)h[8], (unsigned long long)h[9],
                     (unsigned long long)h[0], (unsigned long long)h[10], (unsigned long long)h[11], (unsigned long long)h[12],
                     (unsigned long long)h[13], (unsigned long long)h[14]);
        std::fprintf(stderr, "  fine:");
        for (int i = 16; i < 32; ++i) std::fprintf(stderr, " %llu", (unsigned long long)h[i]);
        std::fprintf(stderr, "\n");
        if (batch > 1) {  // spread over the frames: the kernel lasts as long as its slowest frame
            std::vector<uint64_t> all(static_cast<size_t>(batch) * 32);
            FD_HIP_TRY(c, hipMemcpyAsync(all.data(), c->dbg.p, sizeof(uint64_t) * all.size(), hipMemcpyDeviceToHost,
                                         c->stream));
            FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
            uint64_t mn = ~0ull, mx = 0, gmx = 0, grmx = 0;
            int fmx = 0;
            for (int b = 0; b < batch; ++b) {
                const uint64_t *q = all.data() + static_cast<size_t>(b) * 32;
                const uint64_t t = q[1] + q[2] + q[3] + q[4] + q[5] + q[6] + q[7];
                if (t > mx) mx = t, fmx = b;
                mn = std::min(mn, t);
                gmx = std::max(gmx, q[3]);
                grmx = std::max(grmx, q[5]);
            }
            std::fprintf(stderr, "  frames: total cycles min %llu max %llu (frame %d), max gather %llu, max greedy %llu\n",
                         (unsigned long long)mn, (unsigned long long)mx, fmx, (unsigned long long)gmx,
                         (unsigned long long)grmx);
        }
    }
    if (c->tie_order == FD_TIES_REFERENCE && !q.tie_idx_desc) {
        if (host_ties_env()) {  // the round-3 host path (A/B and checker): every flagged frame sorted on the host
            const int rc = resolve_ties(c, s, batch, sbl, q.push_order, FD_FRAME_TIES);
            if (rc) return rc;
        } else {
            fdk::RefSortArgs r{};
            const int rc = ref_buffers(c, batch, rows, cols, q.cap, r);
            if (rc) return rc;
            r.push_order = q.push_order ? 1 : 0;
            static const bool ref_debug = ab_env("FD_REF_DEBUG") != nullptr;  // diagnostic: broken invariants
            if (ref_debug) {
                FD_HIP_TRY(c, ensure(c, c->dbg, sizeof(uint32_t) * 8 * batch));
                FD_HIP_TRY(c, hipMemsetAsync(c->dbg.p, 0, sizeof(uint32_t) * 8 * batch, c->stream));
                r.dbg = as<uint32_t>(c->dbg);
            }
            // frames of >= 1 Mpx: the multi-workgroup prelude (push order, first levels); FD_REF_WIDE=0/1
            // forces it off / on (A/B)
            const char *wide_env = ab_env("FD_REF_WIDE");
            const bool wide = wide_env ? std::atoi(wide_env) != 0
                                       : static_cast<int64_t>(rows) * cols >= (int64_t{1} << 20);
            FD_HIP_TRY(c, fdk::launch_select_reference(s, r, batch, wide, c->stream));
            if (stamps) {  // k_select_reference's phase clocks (slots 16-30) of the flagged frames
                std::vector<uint64_t> all(static_cast<size_t>(batch) * 32);
                FD_HIP_TRY(c, hipMemcpyAsync(all.data(), c->dbg.p, sizeof(uint64_t) * all.size(), hipMemcpyDeviceToHost,
                                             c->stream));
                FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
                for (int b = 0; b < batch; ++b) {
                    const uint64_t *q = all.data() + static_cast<size_t>(b) * 32;
                    if (q[18])
                        std::fprintf(stderr, "k_select_reference frame %d cycles: push %llu | levels %llu sumT %llu: pivots %llu "
                                             "pass1 %llu bases %llu pass2 %llu (K) %llu pass3 %llu children %llu | leaves %llu "
                                             "wave-local %llu greedy %llu windows %llu\n", b, (unsigned long long)q[16], (unsigned long long)q[18],
                                     (unsigned long long)q[19], (unsigned long long)q[24], (unsigned long long)q[25],
                                     (unsigned long long)q[26], (unsigned long long)q[27], (unsigned long long)q[28],
                                     (unsigned long long)q[29], (unsigned long long)q[30], (unsigned long long)q[20],
                                     (unsigned long long)q[23], (unsigned long long)q[21], (unsigned long long)q[22]);
                    if (q[18]) {
                        std::fprintf(stderr, "  levels (T:cycles):");
                        for (int l = 0; l < 16 && l < static_cast<int>(q[18]); ++l)
                            std::fprintf(stderr, " %llu:%llu", (unsigned long long)(q[l] >> 40),
                                         (unsigned long long)(q[l] & ((1ull << 40) - 1)));
                        std::fprintf(stderr, "\n");
                    }
                }
            }
            if (ref_debug) {
                std::vector<uint32_t> h(static_cast<size_t>(8) * batch);
                FD_HIP_TRY(c, hipMemcpyAsync(h.data(), c->dbg.p, sizeof(uint32_t) * h.size(), hipMemcpyDeviceToHost, c->stream));
                FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
                for (int b = 0; b < batch; ++b)
                    if (h[8 * b])
                        std::fprintf(stderr, "k_select_reference frame %d: check %u idx %u bound %u m_act %u T %u\n", b, h[8 * b],
                                     h[8 * b + 1], h[8 * b + 2], h[8 * b + 3], h[8 * b + 4]);
            }
            if (!outputs_on_device) {  // the call synchronises anyway: frames left to the host
                const int rc2 = resolve_ties(c, s, batch, sbl, q.push_order, FD_FRAME_UNRESOLVED);
                if (rc2) return rc2;
            }
        }
    }
    if (!outputs_on_device) {
        if (!direct) FD_HIP_TRY(c, hipMemcpyAsync(c->h_res.p, c->status.p, res_bytes, hipMemcpyDeviceToHost, c->stream));
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
        const uint32_t *st = static_cast<const uint32_t *>(c->h_res.p);
        std::memcpy(out_counts, st + 2 * static_cast<size_t>(batch), sizeof(int32_t) * batch);
        std::memcpy(out_xy, static_cast<const uint8_t *>(c->h_res.p) + res_head,
                    sizeof(float) * 2 * static_cast<size_t>(out_stride) * batch);
        c->h_status.assign(st, st + batch);
        c->h_status_valid = true;
        for (int b = 0; b < batch; ++b) {
            if (st[b] & FD_FRAME_VALUE_RANGE)
                return fail(c, FD_ERR_INVALID, "frame " + std::to_string(b) + ": " + q.value_msg);
            if (st[b] & FD_FRAME_GUARD)
                return fail(c, FD_ERR_HIP, "internal: selection consistency guard tripped (status 0x" + hex(st[b]) +
                                               ", frame " + std::to_string(b) + ")");
            if (out_counts[b] > out_stride) return fail(c, FD_ERR_CAPACITY, "out_stride smaller than the features found");
        }
    } else if (!frames_on_device) {
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));  // the host frames must stay valid until copied
    }
    return FD_OK;
}

// Shared LSD launch geometry (fd_lsd_map and fd_lsd_lines).
void lsd_geometry(fdk::LsdArgs &a, int batch, int rows, int cols, const uint8_t *dframes) {
    const int work_rows = rows - 3;  // rows [1, rows-3]
    a.frames = dframes;
    a.batch = batch;
    a.rows = rows;
    a.cols = cols;
    a.strips = (cols - 1 + 63) / 64;  // map columns [0, cols-2]
    a.strips4 = (cols - 1 + 255) / 256;
    a.aligned4 = (cols % 4 == 0) && (reinterpret_cast<uintptr_t>(dframes) % 4 == 0);
    a.pitch = cols - 1;  // dense maps: unpitched unless the caller gives a pitch (fd_lsd_map_pitched)
    // k_lsd_map chunks of 32 rows (one row-bit word per (column, chunk)), consecutive waves taking consecutive
    // chunks of a strip: the shortest chunks whose scatter stays on its one-pass path (chunks <= 64 at 1080p);
    // 1080p x256 map + scan + scatter 1.514 -> 1.469 ms against 67-row chunks strip-fastest
    // (profiles/r06_lsd_rows.txt). 16 rows when 32 would leave fewer than 4096 waves (small batches).
    int64_t ch = static_cast<int64_t>(batch) * a.strips4 * ((work_rows + 31) / 32) < 4096 ? 16 : 32;
    a.chunk_fastest = 1;
    if (const char *e = ab_env("FD_LSD_WAVES"))  // A/B: rows per chunk from a target wave count
        ch = std::max<int64_t>(16, std::min<int64_t>(static_cast<int64_t>(batch) * a.strips4 * work_rows /
                                                         std::max<int64_t>(64, std::atoll(e)), 256));
    if (const char *e = ab_env("FD_LSD_CH")) ch = std::max(16, std::min(256, std::atoi(e)));  // A/B
    a.chunk_h = static_cast<int>(ch);
    if (const char *e = ab_env("FD_LSD_ORDER")) a.chunk_fastest = std::atoi(e);  // A/B
    a.scatter_cols = 32;  // scatter 116 -> 111 us dense, 106 -> 99 us compact vs 64 (16: 130 / 124; r06_lsd_rows.txt)
    if (const char *e = ab_env("FD_LSD_SC")) a.scatter_cols = std::atoi(e);  // A/B: 16, 32 or 64
    a.chunks = (work_rows + a.chunk_h - 1) / a.chunk_h;
    a.words = (a.chunk_h + 31) / 32;
}

// Host threads of the line stage: all hardware threads, capped by the process's thread budget
// (OMP_NUM_THREADS, e.g. a lease's CPU share); FD_LINE_THREADS overrides.
int default_line_threads() {
    int t = static_cast<int>(std::thread::hardware_concurrency());
    if (const char *e = std::getenv("OMP_NUM_THREADS"); e && std::atoi(e) > 0) t = std::min(t, std::atoi(e));
    if (const char *e = std::getenv("FD_LINE_THREADS"); e && std::atoi(e) > 0) t = std::atoi(e);
    return std::max(1, t);
}

}  // namespace

extern "C" {

const char *fd_build_info(void) {
    return "libfdhip gfx950 (MI355X); kernels: corner response+NMS, FAST-12, greedy select, LSD map; "
           "flags: -O3 -ffp-contract=off";
}

int fd_abi_version(void) { return FD_ABI_VERSION; }

int fd_ctx_create(int device, fd_ctx **out) {
    if (!out) return FD_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return FD_ERR_HIP;
    if (device < 0 || device >= n) return FD_ERR_INVALID;
    if (hipSetDevice(device) != hipSuccess) return FD_ERR_HIP;
    fd_ctx *c = new fd_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return FD_ERR_HIP;
    }
    c->stream = c->own_stream;
    *out = c;
    return FD_OK;
}

void fd_ctx_destroy(fd_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    DevBuf *bufs[] = {&c->frames,    &c->prior_xy,  &c->prior_frame, &c->prior_counts, &c->mask,       &c->row_base,
                      &c->word_pref, &c->list_resp, &c->list_idx,  &c->selctl,      &c->pre_keys,   &c->out_xy,
                      &c->out_counts, &c->grid,     &c->dbg,
                      &c->seg_cnt,  &c->seg,      &c->resp_map,    &c->c_resp,       &c->c_x,     &c->c_y,
                      &c->c_counts, &c->l_norm,   &c->l_angle,     &c->l_valid,      &c->l_cnt,   &c->l_base,
                      &c->l_idx,    &c->l_counts, &c->l_bits, &c->b_uv,     &c->b_counts,    &c->b_bits,       &c->b_valid,
                      &c->n_heat,   &c->n_map,    &c->n_xy,        &c->n_counts,     &c->n_out,
                      &c->segdesc,  &c->seghead,  &c->status,  &c->ord,   &c->ord_meta, &c->run_lut, &c->fast_cut,
                      &c->l_lists,  &c->l_fbase, &c->wide_keys, &c->r_x, &c->r_lpos,
                      &c->r_rpos,   &c->r_ord,    &c->r_ctl,       &c->r_wcnt,      &c->r_wfr,
                      &c->l_sresp,  &c->l_sidx,   &c->l_sst};
    if (c->aux) (void)hipStreamSynchronize(c->aux);
    for (HostBuf *b : {&c->h_lists, &c->h_png, &c->h_ord, &c->h_sst, &c->h_res}) release(*b);
    release(c->d_png);
    for (DevBuf *b : bufs) release(*b);
    if (c->xev) (void)hipEventDestroy(c->xev);
    if (c->l_ev0) (void)hipEventDestroy(c->l_ev0);
    if (c->l_ev1) (void)hipEventDestroy(c->l_ev1);
    if (c->aux) (void)hipStreamDestroy(c->aux);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

const char *fd_last_error(const fd_ctx *c) { return c ? c->err.c_str() : "null context"; }

// The workspace is shared by every call on the context, so a new stream must not start before the
// old one's work: the switch records an event on the old stream and makes the new one wait for it
// (skipped when the new stream is being captured: a capture may not wait on uncaptured work, so the
// caller orders it, e.g. with torch's stream.wait_stream before capturing).
static int switch_stream(fd_ctx *c, hipStream_t s) {
    FD_HIP_TRY(c, hipSetDevice(c->device));
    if (s == c->stream) return FD_OK;
    if (s) {
        int dev = -1;
        FD_HIP_TRY(c, hipStreamGetDevice(s, &dev));
        if (dev != c->device)
            return fail(c, FD_ERR_INVALID, "stream belongs to device " + std::to_string(dev) + ", the context to device " +
                                               std::to_string(c->device));
    }
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    FD_HIP_TRY(c, hipStreamIsCapturing(s, &cs));
    hipStreamCaptureStatus cs_old = hipStreamCaptureStatusNone;
    FD_HIP_TRY(c, hipStreamIsCapturing(c->stream, &cs_old));
    if (cs == hipStreamCaptureStatusNone && cs_old == hipStreamCaptureStatusNone) {
        if (!c->xev) FD_HIP_TRY(c, hipEventCreateWithFlags(&c->xev, hipEventDisableTiming));
        FD_HIP_TRY(c, hipEventRecord(c->xev, c->stream));
        FD_HIP_TRY(c, hipStreamWaitEvent(s, c->xev, 0));
    }
    c->stream = s;
    return FD_OK;
}

int fd_ctx_set_stream(fd_ctx *c, void *s) {
    if (!c) return FD_ERR_INVALID;
    return switch_stream(c, static_cast<hipStream_t>(s));
}

int fd_ctx_use_own_stream(fd_ctx *c) {
    if (!c) return FD_ERR_INVALID;
    return switch_stream(c, c->own_stream);
}

int fd_ctx_set_tie_order(fd_ctx *c, int order) {
    if (!c) return FD_ERR_INVALID;
    if (order != FD_TIES_RASTER && order != FD_TIES_REFERENCE) return fail(c, FD_ERR_INVALID, "unknown tie order");
    c->tie_order = order;
    return FD_OK;
}

int fd_ctx_frame_status(fd_ctx *c, uint32_t *dst, int batch, int async) {
    if (!c) return FD_ERR_INVALID;
    if (!dst || batch < 0) return fail(c, FD_ERR_INVALID, "bad arguments");
    if (batch > c->status_batch)
        return fail(c, FD_ERR_INVALID, "the last selection call had " + std::to_string(c->status_batch) + " frames");
    if (batch == 0) return FD_OK;
    FD_HIP_TRY(c, hipSetDevice(c->device));
    if (c->h_status_valid && static_cast<size_t>(batch) <= c->h_status.size()) {
        // the last selection call returned host outputs and left its status words here: a host
        // destination is served without a device round trip (device memory still gets a copy)
        hipPointerAttribute_t at{};
        const hipError_t e = hipPointerGetAttributes(&at, dst);
        if (e != hipSuccess) (void)hipGetLastError();  // (unregistered host memory on some runtimes)
        if (e != hipSuccess || at.type == hipMemoryTypeHost || at.type == hipMemoryTypeUnregistered) {
            std::memcpy(dst, c->h_status.data(), sizeof(uint32_t) * batch);
            return FD_OK;
        }
    }
    FD_HIP_TRY(c, hipMemcpyAsync(dst, c->status.p, sizeof(uint32_t) * batch, hipMemcpyDefault, c->stream));
    if (!async) FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
    return FD_OK;
}

void *fd_ctx_get_stream(const fd_ctx *c) { return c ? static_cast<void *>(c->stream) : nullptr; }

int fd_ctx_synchronize(fd_ctx *c) {
    if (!c) return FD_ERR_INVALID;
    FD_HIP_TRY(c, hipSetDevice(c->device));
    FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
    return FD_OK;
}

int fd_ctx_stage(fd_ctx *c, const void *host, int64_t bytes, const uint8_t **device_out) {
    if (!c || !host || bytes < 0 || !device_out) return fail(c, FD_ERR_INVALID, "bad arguments");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    FD_HIP_TRY(c, ensure(c, c->frames, static_cast<size_t>(bytes)));
    FD_HIP_TRY(c, hipMemcpyAsync(c->frames.p, host, static_cast<size_t>(bytes), hipMemcpyHostToDevice, c->stream));
    FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
    *device_out = as<uint8_t>(c->frames);
    return FD_OK;
}

int fd_ctx_reserve(fd_ctx *c, int kind, int batch, int rows, int cols, int64_t max_prior_total) {
    int rc = check_shape(c, kind, batch, rows, cols);
    if (rc) return rc;
    FD_HIP_TRY(c, hipSetDevice(c->device));
    const int64_t cap = detect_list_cap(kind, rows, cols);
    SelectBufs sb{};
    rc = select_buffers(c, batch, cap, sb);
    if (rc) return rc;
    FD_HIP_TRY(c, ensure(c, c->prior_counts, sizeof(int32_t) * batch));
    if (max_prior_total > 0) {
        FD_HIP_TRY(c, ensure(c, c->prior_xy, sizeof(float) * 2 * max_prior_total));
        FD_HIP_TRY(c, ensure(c, c->prior_frame, sizeof(int32_t) * max_prior_total));
        FD_HIP_TRY(c, ensure(c, c->mask, sizeof(uint32_t) * static_cast<size_t>(batch) * rows * ((cols + 31) / 32)));
    }
    if (kind == FD_FAST) {
        rc = build_offsets(c, std::max<int64_t>(0, static_cast<int64_t>(rows - 6) * (cols - 6)), c->off_thr);
        if (rc) return rc;
        if (!c->fast_cut.p) {  // the emission cut's words (fd_points_detect; zero: no cut)
            FD_HIP_TRY(c, ensure(c, c->fast_cut, 2 * sizeof(uint32_t)));
            FD_HIP_TRY(c, hipMemsetAsync(c->fast_cut.p, 0, c->fast_cut.n, c->stream));
        }
        if (max_prior_total > 0) {  // masked FAST: the mask scan's prefix tables
            FD_HIP_TRY(c, ensure(c, c->row_base, sizeof(int32_t) * static_cast<size_t>(batch) * rows));
            FD_HIP_TRY(c, ensure(c, c->word_pref, sizeof(int32_t) * static_cast<size_t>(batch) * rows * ((cols + 31) / 32)));
        }
    }
    FD_HIP_TRY(c, ensure(c, c->status, sizeof(uint32_t) * 2 * static_cast<size_t>(batch)));
    if (c->tie_order == FD_TIES_REFERENCE) {  // k_select_reference's scratch
        fdk::RefSortArgs r{};
        rc = ref_buffers(c, batch, rows, cols, cap, r);
        if (rc) return rc;
    }
    for (const int px : {0, corner_px(kind, batch, rows, cols, 0.0f)}) {  // (either kernel's geometry)
        const PointGeom g = point_geom(kind, batch, rows, cols, px);
        if (!g.empty && use_seg_lists(g.blocks_per_frame, rows, cols)) {
            FD_HIP_TRY(c, ensure(c, c->segdesc, sizeof(uint2) * static_cast<size_t>(batch) * g.blocks_per_frame));
            FD_HIP_TRY(c, ensure(c, c->seghead, sizeof(uint64_t) * fdk::kSegHead * static_cast<size_t>(batch) * g.blocks_per_frame));
        }
    }
    return FD_OK;
}

int fd_points_detect(fd_ctx *c, int kind, const uint8_t *frames, int frames_on_device, int batch, int rows, int cols,
                     const fd_point_opts *opts, const float *prior_xy, const int32_t *prior_counts, uint32_t need,
                     float *out_xy, int32_t out_stride, int32_t *out_counts, int outputs_on_device) {
    int rc = check_shape(c, kind, batch, rows, cols);
    if (rc) return rc;
    if (!opts || !out_xy || !out_counts || out_stride < 1) return fail(c, FD_ERR_INVALID, "bad output arguments");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    if ((rc = refuse_sync_under_capture(c, outputs_on_device))) return rc;
    const uint8_t *dframes = nullptr;
    rc = stage_frames(c, frames, frames_on_device, batch, rows, cols, dframes);
    if (rc) return rc;
    PriorInfo pi;
    rc = setup_priors(c, batch, rows, cols, opts->min_feature_distance, prior_xy, prior_counts, pi);
    if (rc) return rc;

    const int px = corner_px(kind, batch, rows, cols, opts->min_valid_response);
    const PointGeom g = point_geom(kind, batch, rows, cols, px);
    const int64_t cap = detect_list_cap(kind, rows, cols);
    SelectBufs sb{};
    rc = select_buffers(c, batch, cap, sb);
    if (rc) return rc;

    fdk::PointsArgs a{};
    a.px = px;
    a.frames = dframes;
    a.batch = batch;
    a.rows = rows;
    a.cols = cols;
    a.tiles_x = g.tiles_x;
    a.tiles_y = g.tiles_y;
    a.tile_h = g.tile_h;
    a.aligned4 = (cols % 4 == 0) && (reinterpret_cast<uintptr_t>(dframes) % 4 == 0);
    a.thr = opts->min_valid_response;
    a.blocks_per_frame = g.blocks_per_frame;
    a.mask = pi.mask;
    a.mask_wpr = pi.wpr;
    a.list_resp = as<float>(c->list_resp);
    a.list_idx = as<uint32_t>(c->list_idx);
    a.list_cap = cap;
    a.list_count = sb.list_count;
    a.hist0 = sb.hist0;
    const bool seg = !g.empty && use_seg_lists(g.blocks_per_frame, rows, cols);
    if (seg) {
        FD_HIP_TRY(c, ensure(c, c->segdesc, sizeof(uint2) * static_cast<size_t>(batch) * g.blocks_per_frame));
        a.segdesc = as<uint2>(c->segdesc);
        a.seg_bad = sb.seg_bad;
        FD_HIP_TRY(c, ensure(c, c->seghead, sizeof(uint64_t) * fdk::kSegHead * static_cast<size_t>(batch) * g.blocks_per_frame));
        a.seghead = as<uint64_t>(c->seghead);
    }
    if (kind == FD_FAST && !g.empty) {
        rc = build_offsets(c, static_cast<int64_t>(rows - 6) * (cols - 6), opts->min_valid_response);
        if (rc) return rc;
    }
    key_map(kind, opts->min_valid_response, kind == FD_FAST && !g.empty ? &c->off : nullptr,
            static_cast<int64_t>(rows - 6) * (cols - 6), a.key_base, a.key_lz);
    // FAST's emission cut (PointsArgs::emit_cut): only in the raster tie order (the
    // reference order's emulation needs every candidate in push order). FD_FAST_CUT=0: off (A/B).
    const bool fast_cut = kind == FD_FAST && !g.empty && c->tie_order == FD_TIES_RASTER &&
                          !(ab_env("FD_FAST_CUT") && std::atoi(ab_env("FD_FAST_CUT")) == 0);
    if (fast_cut && !c->fast_cut.p) {  // (zero: no cut, until a selection proposes one)
        FD_HIP_TRY(c, ensure(c, c->fast_cut, 2 * sizeof(uint32_t)));
        FD_HIP_TRY(c, hipMemsetAsync(c->fast_cut.p, 0, c->fast_cut.n, c->stream));
    }
    c->sel_dirty = true;  // until k_select is enqueued: it resets the control block
    if (!g.empty) {
        if (kind == FD_FAST) {
            if (pi.mask) {
                if (rows > 4096) return fail(c, FD_ERR_INVALID, "FAST with prior features supports rows <= 4096");
                FD_HIP_TRY(c, ensure(c, c->row_base, sizeof(int32_t) * static_cast<size_t>(batch) * rows));
                FD_HIP_TRY(c, ensure(c, c->word_pref, sizeof(int32_t) * static_cast<size_t>(batch) * rows * pi.wpr));
                FD_HIP_TRY(c, fdk::launch_fast_mask_scan(pi.mask, pi.wpr, batch, rows, cols, as<int32_t>(c->row_base),
                                                         as<int32_t>(c->word_pref), c->stream));
                a.row_base = as<int32_t>(c->row_base);
                a.word_pref = as<int32_t>(c->word_pref);
            }
            if (fast_cut) {
                // the emission cut of this call (written by the previous FAST call's selection) and the word
                // this call's selection proposes the next one in: two words, alternating per call
                const int p = c->fast_cut_parity;
                c->fast_cut_parity ^= 1;
                a.emit_cut = as<uint32_t>(c->fast_cut) + p;
                a.emit_cut_next = as<uint32_t>(c->fast_cut) + (p ^ 1);
                a.skipped = sb.skipped;
            }
            FD_HIP_TRY(c, fdk::launch_fast(false, a, c->off, c->stream));
        } else {
            FD_HIP_TRY(c, fdk::launch_corner(kind, false, a, c->stream));
        }
    }

    SelectCall sc{};
    sc.batch = batch;
    sc.rows = rows;
    sc.cols = cols;
    sc.dist = opts->min_feature_distance;
    sc.need = need;
    sc.cap = cap;
    sc.key_base = a.key_base;
    sc.key_lz = a.key_lz;
    sc.segdesc = a.segdesc;
    sc.seghead = a.seghead;
    sc.nseg = g.blocks_per_frame;
    sc.wide_eager = kind == FD_FAST;
    if (fast_cut) {
        sc.redo_points = &a;
        sc.redo_off = &c->off;
        sc.skipped = sb.skipped;
        sc.cut_cur = a.emit_cut;
        sc.cut_next = a.emit_cut_next;
    }
    return run_select(c, sc, pi, sb, out_xy, out_stride, out_counts, outputs_on_device, frames_on_device);
}

// SelectGoodFeatures (feature_point_detector.cpp:54-88) over caller-supplied candidates (the
// ComputeCandidates seam, :20): k_cand_lists puts them into the selection's list format (push order
// kept), then the same k_select as fd_points_detect, with the full float order as key map.
int fd_points_select(fd_ctx *c, int batch, int rows, int cols, const fd_point_opts *opts, const float *cand_resp,
                     const int32_t *cand_x, const int32_t *cand_y, const int64_t *cand_counts, int64_t cand_cap,
                     int cands_on_device, const float *prior_xy, const int32_t *prior_counts, uint32_t need,
                     float *out_xy, int32_t out_stride, int32_t *out_counts, int outputs_on_device) {
    int rc = check_shape(c, FD_HARRIS, batch, rows, cols);
    if (rc) return rc;
    if (!opts || !out_xy || !out_counts || out_stride < 1) return fail(c, FD_ERR_INVALID, "bad output arguments");
    if (!cand_counts || cand_cap < 0 || cand_cap > 0xFFFFFFFFll)
        return fail(c, FD_ERR_INVALID, "cand_counts is NULL or cand_cap out of range");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    if ((rc = refuse_sync_under_capture(c, outputs_on_device))) return rc;
    int64_t max_n = cand_cap;
    if (!cands_on_device) {
        max_n = 0;
        for (int b = 0; b < batch; ++b) {
            if (cand_counts[b] < 0 || cand_counts[b] > cand_cap)
                return fail(c, FD_ERR_INVALID, "frame " + std::to_string(b) + ": candidate count outside [0, cand_cap]");
            max_n = std::max(max_n, cand_counts[b]);
        }
    }
    if (max_n > 0 && (!cand_resp || !cand_x || !cand_y)) return fail(c, FD_ERR_INVALID, "candidate arrays are NULL");
    PriorInfo pi;
    rc = setup_priors(c, batch, rows, cols, opts->min_feature_distance, prior_xy, prior_counts, pi);
    if (rc) return rc;
    const int64_t cap = std::max<int64_t>(max_n, 64);
    SelectBufs sb{};
    rc = select_buffers(c, batch, cap, sb);
    if (rc) return rc;
    fdk::CandInArgs a{};
    a.stride = cands_on_device ? cand_cap : max_n;
    if (cands_on_device) {
        a.resp = cand_resp;
        a.x = cand_x;
        a.y = cand_y;
        a.counts = cand_counts;
    } else {  // pack the frames' lists at stride max_n
        const size_t tot = static_cast<size_t>(batch) * static_cast<size_t>(std::max<int64_t>(max_n, 1));
        FD_HIP_TRY(c, ensure(c, c->c_resp, sizeof(float) * tot));
        FD_HIP_TRY(c, ensure(c, c->c_x, sizeof(int32_t) * tot));
        FD_HIP_TRY(c, ensure(c, c->c_y, sizeof(int32_t) * tot));
        FD_HIP_TRY(c, ensure(c, c->c_counts, sizeof(int64_t) * batch));
        for (int b = 0; b < batch; ++b) {
            const size_t n = static_cast<size_t>(cand_counts[b]);
            if (n == 0) continue;
            const size_t src = static_cast<size_t>(b) * static_cast<size_t>(cand_cap);
            const size_t dst = static_cast<size_t>(b) * static_cast<size_t>(max_n);
            FD_HIP_TRY(c, hipMemcpyAsync(as<float>(c->c_resp) + dst, cand_resp + src, sizeof(float) * n,
                                         hipMemcpyHostToDevice, c->stream));
            FD_HIP_TRY(c, hipMemcpyAsync(as<int32_t>(c->c_x) + dst, cand_x + src, sizeof(int32_t) * n,
                                         hipMemcpyHostToDevice, c->stream));
            FD_HIP_TRY(c, hipMemcpyAsync(as<int32_t>(c->c_y) + dst, cand_y + src, sizeof(int32_t) * n,
                                         hipMemcpyHostToDevice, c->stream));
        }
        FD_HIP_TRY(c, hipMemcpyAsync(c->c_counts.p, cand_counts, sizeof(int64_t) * batch, hipMemcpyHostToDevice,
                                     c->stream));
        a.resp = as<float>(c->c_resp);
        a.x = as<int32_t>(c->c_x);
        a.y = as<int32_t>(c->c_y);
        a.counts = as<int64_t>(c->c_counts);
    }
    a.batch = batch;
    a.rows = rows;
    a.cols = cols;
    a.list_resp = as<float>(c->list_resp);
    a.list_idx = as<uint32_t>(c->list_idx);
    a.list_cap = cap;
    a.list_count = sb.list_count;
    a.hist0 = sb.hist0;
    // any float: keys from float_key(-inf) - 1 (never 0) to float_key(+inf), the whole 32-bit range
    a.key_base = host_float_key(-std::numeric_limits<float>::infinity()) - 1u;
    a.key_lz = 0;
    a.bad = sb.pre_count;
    a.border = -1;  // list position = push position
    c->sel_dirty = true;  // until k_select is enqueued: it resets the control block
    FD_HIP_TRY(c, fdk::launch_cand_lists(a, max_n, c->stream));
    if (!cands_on_device) FD_HIP_TRY(c, hipStreamSynchronize(c->stream));  // caller's host arrays were the sources
    SelectCall sc{};
    sc.batch = batch;
    sc.rows = rows;
    sc.cols = cols;
    sc.dist = opts->min_feature_distance;
    sc.need = need;
    sc.cap = cap;
    sc.key_base = a.key_base;
    sc.key_lz = a.key_lz;
    sc.value_flag = true;
    sc.push_order = true;
    sc.dup_keys = true;
    sc.value_msg = "a candidate outside the frame, a NaN response or a bad candidate count";
    return run_select(c, sc, pi, sb, out_xy, out_stride, out_counts, outputs_on_device, 1);
}

static int points_response(fd_ctx *c, int kind, const uint8_t *frames, int batch, int rows, int cols,
                           const fd_point_opts *opts, float *out_resp, uint32_t *out_idx, int64_t cand_cap,
                           uint32_t *out_counts, bool reset_counts) {
    int rc = check_shape(c, kind, batch, rows, cols);
    if (rc) return rc;
    if (!opts || !frames || !out_resp || !out_idx || !out_counts || cand_cap < 1)
        return fail(c, FD_ERR_INVALID, "bad arguments");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    // k_corner_lp addresses the caller's list through a buffer resource of cand_cap * 4 bytes and
    // 32-bit byte offsets: larger capacities take k_corner (64-bit positions against the int64 cap).
    const int px = cand_cap < (int64_t(1) << 30) ? corner_px(kind, batch, rows, cols, opts->min_valid_response) : 0;
    const PointGeom g = point_geom(kind, batch, rows, cols, px);
    if (reset_counts) FD_HIP_TRY(c, hipMemsetAsync(out_counts, 0, sizeof(uint32_t) * batch, c->stream));
    if (g.empty) return FD_OK;
    fdk::PointsArgs a{};
    a.px = px;
    a.frames = frames;
    a.batch = batch;
    a.rows = rows;
    a.cols = cols;
    a.tiles_x = g.tiles_x;
    a.tiles_y = g.tiles_y;
    a.tile_h = g.tile_h;
    a.blocks_per_frame = g.blocks_per_frame;
    a.aligned4 = (cols % 4 == 0) && (reinterpret_cast<uintptr_t>(frames) % 4 == 0);
    a.thr = opts->min_valid_response;
    a.list_resp = out_resp;
    a.list_idx = out_idx;
    a.list_cap = cand_cap;
    a.list_count = out_counts;
    if (kind == FD_FAST) {
        rc = build_offsets(c, static_cast<int64_t>(rows - 6) * (cols - 6), opts->min_valid_response);
        if (rc) return rc;
        FD_HIP_TRY(c, fdk::launch_fast(false, a, c->off, c->stream));
    } else {
        FD_HIP_TRY(c, fdk::launch_corner(kind, false, a, c->stream));
    }
    return FD_OK;
}

int fd_points_response(fd_ctx *c, int kind, const uint8_t *frames, int batch, int rows, int cols,
                       const fd_point_opts *opts, float *out_resp, uint32_t *out_idx, int64_t cand_cap,
                       uint32_t *out_counts) {
    return points_response(c, kind, frames, batch, rows, cols, opts, out_resp, out_idx, cand_cap, out_counts, true);
}

int fd_points_response_append(fd_ctx *c, int kind, const uint8_t *frames, int batch, int rows, int cols,
                              const fd_point_opts *opts, float *out_resp, uint32_t *out_idx, int64_t cand_cap,
                              uint32_t *out_counts) {
    return points_response(c, kind, frames, batch, rows, cols, opts, out_resp, out_idx, cand_cap, out_counts, false);
}

int fd_points_candidates(fd_ctx *c, int kind, const uint8_t *frames, int frames_on_device, int batch, int rows,
                         int cols, const fd_point_opts *opts, const float *prior_xy, const int32_t *prior_counts,
                         float *out_resp, int32_t *out_x, int32_t *out_y, int64_t cand_cap, int64_t *out_counts,
                         float *out_response_map, int outputs_on_device) {
    int rc = check_shape(c, kind, batch, rows, cols);
    if (rc) return rc;
    if (!opts || !out_resp || !out_x || !out_y || !out_counts || cand_cap < 0)
        return fail(c, FD_ERR_INVALID, "bad output arguments");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    const uint8_t *dframes = nullptr;
    rc = stage_frames(c, frames, frames_on_device, batch, rows, cols, dframes);
    if (rc) return rc;
    PriorInfo pi;
    rc = setup_priors(c, batch, rows, cols, opts->min_feature_distance, prior_xy, prior_counts, pi);
    if (rc) return rc;

    const PointGeom g = point_geom(kind, batch, rows, cols);
    const int segcap = kind == FD_FAST ? fdk::kSegFast : fdk::kSegCorner;
    const size_t nseg = static_cast<size_t>(batch) * rows * g.tiles_x;
    FD_HIP_TRY(c, ensure(c, c->seg_cnt, sizeof(int32_t) * nseg));
    FD_HIP_TRY(c, ensure(c, c->seg, sizeof(fdk::Cand) * nseg * segcap));
    const size_t npx = static_cast<size_t>(batch) * rows * cols;
    float *dmap = nullptr;
    if (out_response_map) {
        if (outputs_on_device) {
            dmap = out_response_map;
        } else {
            FD_HIP_TRY(c, ensure(c, c->resp_map, sizeof(float) * npx));
            dmap = as<float>(c->resp_map);
        }
        FD_HIP_TRY(c, hipMemsetAsync(dmap, 0, sizeof(float) * npx, c->stream));
    }
    float *dr = out_resp;
    int32_t *dx = out_x, *dy = out_y;
    int64_t *dc = out_counts;
    const size_t ncap = static_cast<size_t>(std::max<int64_t>(cand_cap, 1)) * batch;
    if (!outputs_on_device) {
        FD_HIP_TRY(c, ensure(c, c->c_resp, sizeof(float) * ncap));
        FD_HIP_TRY(c, ensure(c, c->c_x, sizeof(int32_t) * ncap));
        FD_HIP_TRY(c, ensure(c, c->c_y, sizeof(int32_t) * ncap));
        FD_HIP_TRY(c, ensure(c, c->c_counts, sizeof(int64_t) * batch));
        dr = as<float>(c->c_resp);
        dx = as<int32_t>(c->c_x);
        dy = as<int32_t>(c->c_y);
        dc = as<int64_t>(c->c_counts);
    }
    if (g.empty) {
        FD_HIP_TRY(c, hipMemsetAsync(dc, 0, sizeof(int64_t) * batch, c->stream));
    } else {
        fdk::PointsArgs a{};
        a.frames = dframes;
        a.batch = batch;
        a.rows = rows;
        a.cols = cols;
        a.tiles_x = g.tiles_x;
        a.tiles_y = g.tiles_y;
        a.tile_h = g.tile_h;
        a.blocks_per_frame = g.blocks_per_frame;
        a.aligned4 = (cols % 4 == 0) && (reinterpret_cast<uintptr_t>(dframes) % 4 == 0);
        a.thr = opts->min_valid_response;
        a.mask = pi.mask;
        a.mask_wpr = pi.wpr;
        a.seg_cnt = as<int32_t>(c->seg_cnt);
        a.seg = as<fdk::Cand>(c->seg);
        a.resp_map = dmap;
        if (kind == FD_FAST) {
            rc = build_offsets(c, static_cast<int64_t>(rows - 6) * (cols - 6), opts->min_valid_response);
            if (rc) return rc;
            if (pi.mask) {
                if (rows > 4096) return fail(c, FD_ERR_INVALID, "FAST with prior features supports rows <= 4096");
                FD_HIP_TRY(c, ensure(c, c->row_base, sizeof(int32_t) * static_cast<size_t>(batch) * rows));
                FD_HIP_TRY(c, ensure(c, c->word_pref, sizeof(int32_t) * static_cast<size_t>(batch) * rows * pi.wpr));
                FD_HIP_TRY(c, fdk::launch_fast_mask_scan(pi.mask, pi.wpr, batch, rows, cols, as<int32_t>(c->row_base),
                                                         as<int32_t>(c->word_pref), c->stream));
                a.row_base = as<int32_t>(c->row_base);
                a.word_pref = as<int32_t>(c->word_pref);
            }
            FD_HIP_TRY(c, fdk::launch_fast(true, a, c->off, c->stream));
        } else {
            FD_HIP_TRY(c, fdk::launch_corner(kind, true, a, c->stream));
        }
        fdk::CompactArgs k{};
        k.seg_cnt = a.seg_cnt;
        k.seg = a.seg;
        k.rows = rows;
        k.cols = cols;
        k.tiles_x = g.tiles_x;
        k.seg_cap = segcap;
        k.row_lo = g.border;
        k.row_hi = rows - g.border;
        k.out_resp = dr;
        k.out_x = dx;
        k.out_y = dy;
        k.cap = cand_cap;
        k.out_counts = dc;
        FD_HIP_TRY(c, fdk::launch_compact(k, batch, c->stream));
    }
    if (!outputs_on_device) {
        FD_HIP_TRY(c, hipMemcpyAsync(out_counts, dc, sizeof(int64_t) * batch, hipMemcpyDeviceToHost, c->stream));
        if (cand_cap > 0) {
            FD_HIP_TRY(c, hipMemcpyAsync(out_resp, dr, sizeof(float) * cand_cap * batch, hipMemcpyDeviceToHost, c->stream));
            FD_HIP_TRY(c, hipMemcpyAsync(out_x, dx, sizeof(int32_t) * cand_cap * batch, hipMemcpyDeviceToHost, c->stream));
            FD_HIP_TRY(c, hipMemcpyAsync(out_y, dy, sizeof(int32_t) * cand_cap * batch, hipMemcpyDeviceToHost, c->stream));
        }
        if (out_response_map)
            FD_HIP_TRY(c, hipMemcpyAsync(out_response_map, dmap, sizeof(float) * npx, hipMemcpyDeviceToHost, c->stream));
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
        for (int b = 0; b < batch; ++b)
            if (out_counts[b] > cand_cap) return fail(c, FD_ERR_CAPACITY, "cand_cap smaller than the candidates found");
    } else if (!frames_on_device) {
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    return FD_OK;
}

int fd_lsd_map(fd_ctx *c, const uint8_t *frames, int frames_on_device, int batch, int rows, int cols, float min_norm,
               float *norm, float *angle, uint8_t *valid, int32_t *valid_idx, int64_t idx_cap, int64_t *valid_counts,
               int outputs_on_device) {
    return fd_lsd_map_pitched(c, frames, frames_on_device, batch, rows, cols, min_norm, norm, angle, valid,
                              static_cast<int64_t>(cols) - 1, valid_idx, idx_cap, valid_counts, outputs_on_device);
}

// Row pitch of the library's own (device) dense maps: 16 entries, so every f32 map row starts on a
// 64-byte and every u8 row on a 16-byte boundary and the map kernel's dword / dwordx4 row stores are
// aligned (a 1919-entry row is misaligned on 3 of 4 rows: the vector-memory address unit then splits
// the stores).
int64_t lsd_aligned_pitch(int cols) { return (static_cast<int64_t>(cols) - 1 + 15) / 16 * 16; }

int fd_lsd_map_pitched(fd_ctx *c, const uint8_t *frames, int frames_on_device, int batch, int rows, int cols,
                       float min_norm, float *norm, float *angle, uint8_t *valid, int64_t map_pitch, int32_t *valid_idx,
                       int64_t idx_cap, int64_t *valid_counts, int outputs_on_device) {
    int rc = check_shape(c, FD_HARRIS, batch, rows, cols, false);
    if (rc) return rc;
    if (rows < 2 || cols < 2) return fail(c, FD_ERR_INVALID, "LSD needs rows >= 2 and cols >= 2");  // :14
    const int mc = cols - 1;
    if (map_pitch < mc || map_pitch > (int64_t(1) << 29)) return fail(c, FD_ERR_INVALID, "map_pitch must be >= cols-1");
    // device maps: the caller's pitch; host maps: the library's staging maps use the aligned pitch
    const int64_t dpitch = outputs_on_device ? map_pitch : lsd_aligned_pitch(cols);
    if (static_cast<int64_t>(rows - 1) * dpitch >= (int64_t(1) << 29))  // 32-bit byte offsets into a frame's maps
        return fail(c, FD_ERR_INVALID, "LSD frame too large ((rows-1)*pitch must be < 2^29)");
    if (!valid_counts || idx_cap < 0 || (idx_cap > 0 && !valid_idx))
        return fail(c, FD_ERR_INVALID, "bad output arguments");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    const uint8_t *dframes = nullptr;
    rc = stage_frames(c, frames, frames_on_device, batch, rows, cols, dframes);
    if (rc) return rc;
    const size_t nmap = static_cast<size_t>(batch) * (rows - 1) * static_cast<size_t>(dpitch);
    float *dn = nullptr, *da = nullptr;
    uint8_t *dv = nullptr;
    if (outputs_on_device) {
        dn = norm;
        da = angle;
        dv = valid;
    } else {
        if (norm) {
            FD_HIP_TRY(c, ensure(c, c->l_norm, sizeof(float) * nmap));
            dn = as<float>(c->l_norm);
        }
        if (angle) {
            FD_HIP_TRY(c, ensure(c, c->l_angle, sizeof(float) * nmap));
            da = as<float>(c->l_angle);
        }
    }
    if (dv == nullptr) {  // the valid map is needed internally for the ordered scatter
        FD_HIP_TRY(c, ensure(c, c->l_valid, nmap));
        dv = as<uint8_t>(c->l_valid);
    }

    int32_t *di = valid_idx;
    int64_t *dc = valid_counts;
    if (!outputs_on_device) {
        FD_HIP_TRY(c, ensure(c, c->l_idx, sizeof(int32_t) * static_cast<size_t>(std::max<int64_t>(idx_cap, 1)) * batch));
        FD_HIP_TRY(c, ensure(c, c->l_counts, sizeof(int64_t) * batch));
        di = as<int32_t>(c->l_idx);
        dc = as<int64_t>(c->l_counts);
    }
    const int work_rows = rows - 3;  // rows [1, rows-3]
    const int work_cols = cols - 3;  // cols [1, cols-3]
    if (work_rows <= 0 || work_cols <= 0) {  // nothing scanned: all-zero maps
        if (dn) FD_HIP_TRY(c, hipMemsetAsync(dn, 0, sizeof(float) * nmap, c->stream));
        if (da) FD_HIP_TRY(c, hipMemsetAsync(da, 0, sizeof(float) * nmap, c->stream));
        FD_HIP_TRY(c, hipMemsetAsync(dv, 0, nmap, c->stream));
        FD_HIP_TRY(c, hipMemsetAsync(dc, 0, sizeof(int64_t) * batch, c->stream));
    } else {  // k_lsd_map writes every map entry (zeros outside the scanned rows/columns; pitch padding untouched)
        fdk::LsdArgs a{};
        lsd_geometry(a, batch, rows, cols, dframes);
        a.pitch = static_cast<int>(dpitch);
        a.min_norm = min_norm;
        a.norm = dn;
        a.angle = da;
        a.valid = dv;
        const size_t ncnt = static_cast<size_t>(batch) * mc * a.chunks;
        FD_HIP_TRY(c, ensure(c, c->l_cnt, sizeof(int32_t) * ncnt));
        FD_HIP_TRY(c, ensure(c, c->l_base, sizeof(int32_t) * ncnt));
        FD_HIP_TRY(c, ensure(c, c->l_bits, sizeof(uint32_t) * ncnt * a.words));
        a.rowbits = as<uint32_t>(c->l_bits);
        a.col_cnt = as<int32_t>(c->l_cnt);
        a.col_base = as<int32_t>(c->l_base);
        a.idx = di;
        a.idx_cap = idx_cap;
        a.counts = dc;
        FD_HIP_TRY(c, fdk::launch_lsd(a, c->stream));
    }
    if (!outputs_on_device) {
        FD_HIP_TRY(c, hipMemcpyAsync(valid_counts, dc, sizeof(int64_t) * batch, hipMemcpyDeviceToHost, c->stream));
        if (idx_cap > 0)
            FD_HIP_TRY(c, hipMemcpyAsync(valid_idx, di, sizeof(int32_t) * idx_cap * batch, hipMemcpyDeviceToHost, c->stream));
        // pitched device maps -> the host's maps (row pitch map_pitch entries)
        const size_t hrows = static_cast<size_t>(batch) * (rows - 1);
        if (norm)
            FD_HIP_TRY(c, hipMemcpy2DAsync(norm, sizeof(float) * map_pitch, dn, sizeof(float) * dpitch, sizeof(float) * mc,
                                           hrows, hipMemcpyDeviceToHost, c->stream));
        if (angle)
            FD_HIP_TRY(c, hipMemcpy2DAsync(angle, sizeof(float) * map_pitch, da, sizeof(float) * dpitch, sizeof(float) * mc,
                                           hrows, hipMemcpyDeviceToHost, c->stream));
        if (valid)
            FD_HIP_TRY(c, hipMemcpy2DAsync(valid, map_pitch, dv, dpitch, mc, hrows, hipMemcpyDeviceToHost, c->stream));
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
        for (int b = 0; b < batch; ++b)
            if (valid_counts[b] > idx_cap) return fail(c, FD_ERR_CAPACITY, "idx_cap smaller than the valid pixels");
    } else if (!frames_on_device) {
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    return FD_OK;
}

namespace {

// fd_lsd_lines' seed order (sorted_pixels_, feature_line_detector.cpp:88-94) on a side stream, after
// c->l_ev0 (recorded on the context stream once the compact lists exist): k_select_reference in push
// order over each frame's (norm, map index) list, the orders and statuses copied to c->h_ord / c->h_sst,
// c->l_ev1 recorded after the copies. The context stream does not wait for it: fd_lsd_lines waits on
// l_ev1 before it returns.
int lsd_seed_order(fd_ctx *c, int batch, int map_rows, int map_cols, const std::vector<int64_t> &base,
                   const fdk::LsdArgs &la, int64_t &ord_stride) {
    int64_t cap = 1;
    for (int b = 0; b < batch; ++b) cap = std::max(cap, base[static_cast<size_t>(b) + 1] - base[static_cast<size_t>(b)]);
    if (cap >= (int64_t(1) << 30)) return fail(c, FD_ERR_INVALID, "LSD frame with >= 2^30 valid pixels");
    const size_t nb = static_cast<size_t>(batch);
    FD_HIP_TRY(c, ensure(c, c->l_sresp, sizeof(float) * static_cast<size_t>(cap) * nb));
    FD_HIP_TRY(c, ensure(c, c->l_sidx, sizeof(uint32_t) * static_cast<size_t>(cap) * nb));
    FD_HIP_TRY(c, ensure(c, c->l_sst, sizeof(uint32_t) * 2 * nb));
    fdk::RefSortArgs r{};
    const int rc = ref_buffers(c, batch, map_rows, map_cols, cap, r);
    if (rc) return rc;
    FD_HIP_TRY(c, ensure_host(c->h_ord, sizeof(uint32_t) * static_cast<size_t>(r.cap) * nb));
    FD_HIP_TRY(c, ensure_host(c->h_sst, sizeof(uint32_t) * nb));
    fdk::SelectArgs s{};
    s.list_resp = as<float>(c->l_sresp);
    s.list_idx = as<uint32_t>(c->l_sidx);
    s.list_cap = cap;
    s.rows = map_rows;
    s.cols = map_cols;
    s.need = 0xFFFFFFFFu;
    s.status = as<uint32_t>(c->l_sst);
    s.cand_n = s.status + batch;
    // (no multi-workgroup prelude: every frame is sorted, all workgroups are busy anyway, and the ~30
    // prelude launches cost more than its first levels save: seed orders 0.35-0.6 ms after the lists
    // instead of 0.58-0.87, profiles/r05_lines_seed_order.txt; FD_LSD_WIDE=1: with it, A/B)
    bool wide = false;
    if (const char *e = ab_env("FD_LSD_WIDE")) wide = std::atoi(e) != 0;
    FD_HIP_TRY(c, hipStreamWaitEvent(c->aux, c->l_ev0, 0));
    // order_only never reads ord back: the kernel may write it straight into the pinned host buffer
    // (FD_LSD_ORD_MAPPED=0: a device buffer and a copy, A/B)
    const char *mapped_env = ab_env("FD_LSD_ORD_MAPPED");
    const bool mapped = !mapped_env || std::atoi(mapped_env) != 0;
    if (mapped) {
        void *dp = nullptr;
        FD_HIP_TRY(c, hipHostGetDevicePointer(&dp, c->h_ord.p, 0));
        r.ord = static_cast<uint32_t *>(dp);
    }
    FD_HIP_TRY(c, fdk::launch_lsd_seed_order(la.frame_base, la.idx, la.lnorm, s, r, batch, wide, c->aux));
    if (!mapped)
        FD_HIP_TRY(c, hipMemcpyAsync(c->h_ord.p, r.ord, sizeof(uint32_t) * static_cast<size_t>(r.cap) * nb,
                                     hipMemcpyDeviceToHost, c->aux));
    FD_HIP_TRY(c, hipMemcpyAsync(c->h_sst.p, s.status, sizeof(uint32_t) * nb, hipMemcpyDeviceToHost, c->aux));
    FD_HIP_TRY(c, hipEventRecord(c->l_ev1, c->aux));
    ord_stride = r.cap;
    return FD_OK;
}

}  // namespace

int fd_lsd_lines(fd_ctx *c, const uint8_t *frames, int frames_on_device, int batch, int rows, int cols,
                 const fd_lsd_opts *opts, uint32_t needed, fd_lsd_rect *out_rects, int32_t rect_stride,
                 int32_t *out_counts, int threads) {
    int rc = check_shape(c, FD_HARRIS, batch, rows, cols, false);
    if (rc) return rc;
    if (rows < 2 || cols < 2) return fail(c, FD_ERR_INVALID, "LSD needs rows >= 2 and cols >= 2");  // :14
    if (static_cast<int64_t>(rows - 1) * (cols - 1) >= (int64_t(1) << 29))
        return fail(c, FD_ERR_INVALID, "LSD frame too large ((rows-1)*(cols-1) must be < 2^29)");
    if (!opts || !out_counts || rect_stride < 0 || (rect_stride > 0 && !out_rects))
        return fail(c, FD_ERR_INVALID, "bad output arguments");
    if (frames == nullptr) return fail(c, FD_ERR_INVALID, "frames is NULL");
    c->st_idx.clear();
    c->st_norm.clear();
    c->st_angle.clear();
    c->st_used.clear();
    for (int b = 0; b < batch; ++b) out_counts[b] = 0;
    if (needed == 0) return FD_OK;  // :15
    if (c->aux) FD_HIP_TRY(c, hipStreamSynchronize(c->aux));  // (a failed earlier call's seed sort: drained)
    const bool timing = ab_env("FD_LINES_TIMING") != nullptr;  // diagnostic: phase times to stderr
    // FD_LSD_HOST_SORT=1 (A/B): the seed order by std::sort on the host workers instead of the GPU
    const bool host_sort = ab_env("FD_LSD_HOST_SORT") && std::atoi(ab_env("FD_LSD_HOST_SORT")) != 0;
    bool gpu_seeds = false;
    int64_t ord_stride = 0;
    // Once the seed sort is launched on the side stream it uses the context's shared scratch (the
    // k_select_reference buffers, h_ord): every return from here on drains it first, so that no later
    // call on the context stream races it (the normal path has waited for it already).
    struct AuxDrain {
        hipStream_t s = nullptr;
        ~AuxDrain() {
            if (s) (void)hipStreamSynchronize(s);
        }
    } drain;
    const auto t_start = std::chrono::steady_clock::now();
    FD_HIP_TRY(c, hipSetDevice(c->device));
    const uint8_t *dframes = nullptr;
    rc = stage_frames(c, frames, frames_on_device, batch, rows, cols, dframes);
    if (rc) return rc;
    std::vector<int64_t> base(static_cast<size_t>(batch) + 1, 0);
    if (rows - 3 > 0 && cols - 3 > 0) {
        // GPU: validity counts + row bits and the scans (pass 1-2), then the compact lists (pass 3)
        fdk::LsdArgs a{};
        lsd_geometry(a, batch, rows, cols, dframes);
        a.min_norm = opts->min_valid_gradient_norm;
        const size_t ncnt = static_cast<size_t>(batch) * (cols - 1) * a.chunks;
        FD_HIP_TRY(c, ensure(c, c->l_cnt, sizeof(int32_t) * ncnt));
        FD_HIP_TRY(c, ensure(c, c->l_base, sizeof(int32_t) * ncnt));
        FD_HIP_TRY(c, ensure(c, c->l_bits, sizeof(uint32_t) * ncnt * a.words));
        FD_HIP_TRY(c, ensure(c, c->l_counts, sizeof(int64_t) * batch));
        FD_HIP_TRY(c, ensure(c, c->l_fbase, sizeof(int64_t) * (static_cast<size_t>(batch) + 1)));
        a.rowbits = as<uint32_t>(c->l_bits);
        a.col_cnt = as<int32_t>(c->l_cnt);
        a.col_base = as<int32_t>(c->l_base);
        a.counts = as<int64_t>(c->l_counts);
        a.frame_base = as<int64_t>(c->l_fbase);
        FD_HIP_TRY(c, fdk::launch_lsd_count(a, c->stream));
        FD_HIP_TRY(c, hipMemcpyAsync(base.data(), a.frame_base, sizeof(int64_t) * base.size(), hipMemcpyDeviceToHost,
                                     c->stream));
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
        const int64_t total = base[static_cast<size_t>(batch)];
        if (total > 0) {
            const size_t sec = (static_cast<size_t>(total) + 63) & ~size_t(63);  // section length (entries)
            FD_HIP_TRY(c, ensure(c, c->l_lists, sizeof(uint32_t) * 3 * sec));
            FD_HIP_TRY(c, ensure_host(c->h_lists, sizeof(uint32_t) * 3 * sec));
            a.idx = as<int32_t>(c->l_lists);
            a.idx_cap = total;
            a.lnorm = reinterpret_cast<float *>(a.idx + sec);
            a.langle = a.lnorm + sec;
            FD_HIP_TRY(c, fdk::launch_lsd_scatter(a, c->stream));
            if (!host_sort) {
                if (!c->aux) FD_HIP_TRY(c, hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
                if (!c->l_ev0) FD_HIP_TRY(c, hipEventCreateWithFlags(&c->l_ev0, hipEventDisableTiming));
                if (!c->l_ev1) FD_HIP_TRY(c, hipEventCreateWithFlags(&c->l_ev1, hipEventDisableTiming));
                FD_HIP_TRY(c, hipEventRecord(c->l_ev0, c->stream));  // the lists exist (k_lsd_scatter + k_lsd_values)
            }
            // the lists back in one transfer (the PCIe-bound copy is enqueued before the seed sort, which
            // runs beside it on the side stream)
            FD_HIP_TRY(c, hipMemcpyAsync(c->h_lists.p, a.idx, sizeof(uint32_t) * 3 * sec, hipMemcpyDeviceToHost, c->stream));
            if (!host_sort) {
                drain.s = c->aux;
                const int rc2 = lsd_seed_order(c, batch, rows - 1, cols - 1, base, a, ord_stride);
                if (rc2) return rc2;
                gpu_seeds = true;
            }
            FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
        }
    } else if (!frames_on_device) {
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));  // the staging copy reads the caller's buffer
    }
    const auto t_gpu = std::chrono::steady_clock::now();
    // host: region growing + rectangles, frames over worker threads
    std::vector<fdl::FrameList> fl(static_cast<size_t>(batch));
    const size_t sec = (static_cast<size_t>(base[static_cast<size_t>(batch)]) + 63) & ~size_t(63);
    const int32_t *hidx = static_cast<const int32_t *>(c->h_lists.p);
    const float *hn = reinterpret_cast<const float *>(hidx + sec), *ha = hn + sec;
    for (int b = 0; b < batch; ++b) {
        const int64_t o = base[static_cast<size_t>(b)], n = base[static_cast<size_t>(b) + 1] - o;
        fl[static_cast<size_t>(b)] = fdl::FrameList{n ? hidx + o : nullptr, n ? hn + o : nullptr, n ? ha + o : nullptr, n};
    }
    const int64_t n0 = fl[0].n;
    c->st_used.assign(static_cast<size_t>(n0), 0);
    // the workers wait for the GPU's seed orders after their first frame's setup (once per call)
    std::once_flag seeds_once;
    hipError_t seeds_err = hipSuccess;
    auto t_seeds = t_gpu;
    fdl::SeedOrder so{static_cast<const uint32_t *>(c->h_ord.p), ord_stride, static_cast<const uint32_t *>(c->h_sst.p),
                      [&]() {
                          std::call_once(seeds_once, [&]() {
                              seeds_err = hipEventSynchronize(c->l_ev1);
                              t_seeds = std::chrono::steady_clock::now();
                              if (seeds_err != hipSuccess)  // (reported below; the frames sort on the host)
                                  std::memset(c->h_sst.p, 0, sizeof(uint32_t) * static_cast<size_t>(batch));
                          });
                      }};
    fdl::detect_lines(rows, cols, *opts, fl.data(), batch, out_rects, rect_stride, out_counts, c->st_used.data(),
                      threads > 0 ? threads : default_line_threads(), gpu_seeds ? &so : nullptr);
    if (gpu_seeds) {
        so.wait();  // (every worker waited unless none ran a frame) the side stream's work is done
        FD_HIP_TRY(c, seeds_err);
    }
    if (timing) {
        const auto t_end = std::chrono::steady_clock::now();
        int on_gpu = 0;
        for (int b = 0; gpu_seeds && b < batch; ++b) {
            const uint32_t st = static_cast<const uint32_t *>(c->h_sst.p)[b];
            on_gpu += (st & FD_FRAME_RESOLVED) && !(st & (FD_FRAME_UNRESOLVED | FD_FRAME_GUARD));
        }
        std::fprintf(stderr, "[fd_lsd_lines] batch %d: gpu+d2h %.3f ms, host %.3f ms (seed orders there at %.3f), valid "
                             "%lld, seed orders from the gpu %d\n", batch,
                     std::chrono::duration<double, std::milli>(t_gpu - t_start).count(),
                     std::chrono::duration<double, std::milli>(t_end - t_gpu).count(),
                     std::chrono::duration<double, std::milli>(t_seeds - t_gpu).count(),
                     static_cast<long long>(base[static_cast<size_t>(batch)]), on_gpu);
    }
    if (n0 > 0) {
        c->st_idx.assign(fl[0].idx, fl[0].idx + n0);
        c->st_norm.assign(fl[0].norm, fl[0].norm + n0);
        c->st_angle.assign(fl[0].angle, fl[0].angle + n0);
    }
    return FD_OK;
}

int fd_lsd_lines_state(fd_ctx *c, int32_t *idx, float *norm, float *angle, uint8_t *used, int64_t cap, int64_t *n) {
    if (!c || !n || cap < 0) return FD_ERR_INVALID;
    const int64_t m = static_cast<int64_t>(c->st_idx.size());
    *n = m;
    const int64_t w = std::min(m, cap);
    if (w > 0 && (!idx || !norm || !angle || !used)) return fail(c, FD_ERR_INVALID, "bad output arguments");
    for (int64_t k = 0; k < w; ++k) {
        idx[k] = c->st_idx[static_cast<size_t>(k)];
        norm[k] = c->st_norm[static_cast<size_t>(k)];
        angle[k] = c->st_angle[static_cast<size_t>(k)];
        used[k] = c->st_used[static_cast<size_t>(k)];
    }
    return FD_OK;
}

int fd_png_info(const uint8_t *png, size_t len, int32_t *rows, int32_t *cols, int32_t *channels) {
    fdp::PngInfo in;
    if (fdp::png_info(png, len, in) != fdp::kPngOk) return FD_ERR_INVALID;
    if (rows) *rows = in.rows;
    if (cols) *cols = in.cols;
    if (channels) *channels = in.channels;
    return FD_OK;
}

int fd_png_decode(const uint8_t *png, size_t len, uint8_t *out_gray, size_t cap, int32_t *rows, int32_t *cols) {
    fdp::PngInfo in;
    if (fdp::png_info(png, len, in) != fdp::kPngOk) return FD_ERR_INVALID;
    if (rows) *rows = in.rows;
    if (cols) *cols = in.cols;
    const size_t npx = static_cast<size_t>(in.rows) * in.cols;
    if (!out_gray || cap < npx) return FD_ERR_CAPACITY;
    std::vector<uint8_t> samples(npx * in.channels);
    const int rc = fdp::png_decode(png, len, samples.data(), samples.size(), in);
    if (rc == fdp::kPngCapacity) return FD_ERR_CAPACITY;
    if (rc) return FD_ERR_INVALID;
    const int ch = in.channels;
    for (size_t i = 0; i < npx; ++i) {  // the same conversion as k_rgb_gray (fd_gray.hip)
        const uint8_t *p = samples.data() + i * ch;
        out_gray[i] = ch <= 2 ? p[0]
                              : static_cast<uint8_t>((4899u * p[0] + 9617u * p[1] + 1868u * p[2] + 8192u) >> 14);
    }
    return FD_OK;
}

int fd_png_frames(fd_ctx *c, const uint8_t *const *pngs, const size_t *lens, int n, int rows, int cols,
                  uint8_t *frames_device, int threads) {
    if (!c) return FD_ERR_INVALID;
    if (n < 1 || rows < 1 || cols < 1 || !pngs || !lens || !frames_device) return fail(c, FD_ERR_INVALID, "bad arguments");
    // every image must have the batch geometry; its channel count sets the staging layout (all equal)
    int channels = 0;
    for (int i = 0; i < n; ++i) {
        fdp::PngInfo in;
        if (fdp::png_info(pngs[i], lens[i], in) != fdp::kPngOk)
            return fail(c, FD_ERR_INVALID, "image " + std::to_string(i) + ": not a supported PNG");
        if (in.rows != rows || in.cols != cols)
            return fail(c, FD_ERR_INVALID, "image " + std::to_string(i) + ": size differs from the batch");
        if (i > 0 && in.channels != channels)
            return fail(c, FD_ERR_INVALID, "image " + std::to_string(i) + ": channel count differs from the batch");
        channels = in.channels;
    }
    const size_t per = static_cast<size_t>(rows) * cols * channels;
    if (per * n >= (size_t(1) << 32)) return fail(c, FD_ERR_INVALID, "batch too large (samples >= 4 GiB)");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    // the previous call's upload may still read the pinned staging: wait for the stream first
    FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
    FD_HIP_TRY(c, ensure_host(c->h_png, per * n));
    std::vector<fdp::PngInfo> infos(static_cast<size_t>(n));
    const int rc = fdp::png_decode_batch(pngs, lens, n, static_cast<uint8_t *>(c->h_png.p), per, infos.data(),
                                         threads > 0 ? threads : default_line_threads());
    if (rc) return fail(c, rc == fdp::kPngCapacity ? FD_ERR_CAPACITY : FD_ERR_INVALID, "PNG decode failed");
    uint8_t *src = frames_device;  // gray input: straight into the frames
    if (channels != 1) {
        FD_HIP_TRY(c, ensure(c, c->d_png, per * n));
        src = as<uint8_t>(c->d_png);
    }
    FD_HIP_TRY(c, hipMemcpyAsync(src, c->h_png.p, per * n, hipMemcpyHostToDevice, c->stream));
    if (channels != 1)
        FD_HIP_TRY(c, fdk::launch_rgb_gray(src, channels, frames_device, static_cast<int64_t>(rows) * cols * n, c->stream));
    return FD_OK;
}

int fd_brief_compute(fd_ctx *c, const uint8_t *frames, int frames_on_device, int batch, int rows, int cols,
                     const fd_brief_opts *opts, const float *uv, const int32_t *counts, int32_t stride,
                     uint32_t *out_bits, uint8_t *out_valid, int io_on_device) {
    int rc = check_shape(c, FD_HARRIS, batch, rows, cols, false);
    if (rc) return rc;
    if (!opts || !uv || !out_bits || stride < 0) return fail(c, FD_ERR_INVALID, "bad arguments");
    // pattern_idx_ holds 256 pairs (descriptor_brief.h:36): a longer kLength would read past it
    if (opts->length < 1 || opts->length > 256) return fail(c, FD_ERR_INVALID, "length must be in [1, 256]");
    if (opts->half_patch_size < 0 || opts->half_patch_size > 255)
        return fail(c, FD_ERR_INVALID, "half_patch_size must be in [0, 255]");
    if (opts->sampler != FD_SAMPLE_BILINEAR && opts->sampler != FD_SAMPLE_TRUNCATE)
        return fail(c, FD_ERR_INVALID, "unknown sampler");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    if (stride == 0) return FD_OK;
    const uint8_t *dframes = nullptr;
    rc = stage_frames(c, frames, frames_on_device, batch, rows, cols, dframes);
    if (rc) return rc;
    const size_t slots = static_cast<size_t>(batch) * stride;
    const int nw = (opts->length + 31) / 32;
    fdk::BriefArgs a{};
    a.frames = dframes;
    a.batch = batch;
    a.rows = rows;
    a.cols = cols;
    a.stride = stride;
    a.length = opts->length;
    a.half = opts->half_patch_size;
    a.sampler = opts->sampler;
    if (io_on_device) {
        a.uv = uv;
        a.counts = counts;
        a.out_bits = out_bits;
        a.out_valid = out_valid;
    } else {
        FD_HIP_TRY(c, ensure(c, c->b_uv, sizeof(float) * 2 * slots));
        FD_HIP_TRY(c, ensure(c, c->b_bits, sizeof(uint32_t) * nw * slots));
        FD_HIP_TRY(c, hipMemcpyAsync(c->b_uv.p, uv, sizeof(float) * 2 * slots, hipMemcpyHostToDevice, c->stream));
        a.uv = as<float>(c->b_uv);
        a.out_bits = as<uint32_t>(c->b_bits);
        if (counts) {
            FD_HIP_TRY(c, ensure(c, c->b_counts, sizeof(int32_t) * batch));
            FD_HIP_TRY(c, hipMemcpyAsync(c->b_counts.p, counts, sizeof(int32_t) * batch, hipMemcpyHostToDevice,
                                         c->stream));
            a.counts = as<int32_t>(c->b_counts);
        }
        if (out_valid) {
            FD_HIP_TRY(c, ensure(c, c->b_valid, slots));
            a.out_valid = as<uint8_t>(c->b_valid);
        }
    }
    FD_HIP_TRY(c, fdk::launch_brief(a, c->stream));
    if (!io_on_device) {
        // Slots past counts[b] are not written by the kernel; copy back only the written prefix of each
        // frame so the caller's buffer keeps its contents there, as the device path does.
        for (int b = 0; b < batch; ++b) {
            const int n = counts ? std::min<int64_t>(static_cast<uint32_t>(counts[b]) & 0x01FFFFFFu, stride) : stride;
            if (n <= 0) continue;
            const size_t s0 = static_cast<size_t>(b) * stride;
            FD_HIP_TRY(c, hipMemcpyAsync(out_bits + s0 * nw, a.out_bits + s0 * nw, sizeof(uint32_t) * nw * n,
                                         hipMemcpyDeviceToHost, c->stream));
            if (out_valid)
                FD_HIP_TRY(c, hipMemcpyAsync(out_valid + s0, a.out_valid + s0, n, hipMemcpyDeviceToHost, c->stream));
        }
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
    } else if (!frames_on_device) {
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));  // the host frames must stay valid until copied
    }
    return FD_OK;
}

int fd_nn_select(fd_ctx *c, const float *heatmap, int heatmap_on_device, int batch, int rows, int cols,
                 const fd_nn_opts *opts, const float *prior_xy, const int32_t *prior_counts, float *out_xy,
                 int32_t out_stride, int32_t *out_counts, int outputs_on_device) {
    int rc = check_shape(c, FD_HARRIS, batch, rows, cols);
    if (rc) return rc;
    if (!heatmap) return fail(c, FD_ERR_INVALID, "heatmap is NULL");
    if (!opts || !out_xy || !out_counts || out_stride < 1) return fail(c, FD_ERR_INVALID, "bad output arguments");
    if (opts->invalid_boundary < 0) return fail(c, FD_ERR_INVALID, "invalid_boundary must be >= 0");
    if (opts->max_features < 0) return fail(c, FD_ERR_INVALID, "max_features must be >= 0");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    if ((rc = refuse_sync_under_capture(c, outputs_on_device))) return rc;
    const int64_t npx = static_cast<int64_t>(rows) * cols;
    const float *dheat = heatmap;
    if (!heatmap_on_device) {
        FD_HIP_TRY(c, ensure(c, c->n_heat, sizeof(float) * npx * batch));
        FD_HIP_TRY(c, hipMemcpyAsync(c->n_heat.p, heatmap, sizeof(float) * npx * batch, hipMemcpyHostToDevice, c->stream));
        dheat = as<float>(c->n_heat);
    }
    PriorInfo pi;
    rc = setup_priors(c, batch, rows, cols, opts->min_feature_distance, prior_xy, prior_counts, pi);
    if (rc) return rc;
    const int64_t cap = npx + 64;
    SelectBufs sb{};
    rc = select_buffers(c, batch, cap, sb);
    if (rc) return rc;
    fdk::HeatArgs h{};
    h.heat = dheat;
    h.batch = batch;
    h.rows = rows;
    h.cols = cols;
    h.blocks_per_frame = fdk::heat_blocks_per_frame(npx);
    h.thr = opts->min_response;
    h.border = opts->invalid_boundary;
    h.mask = pi.mask;
    h.mask_wpr = pi.wpr;
    h.list_resp = as<float>(c->list_resp);
    h.list_idx = as<uint32_t>(c->list_idx);
    h.list_cap = cap;
    h.list_count = sb.list_count;
    h.hist0 = sb.hist0;
    // responses in (thr, max_response] (probabilities: max 1) or (thr, +inf]
    key_map(FD_HARRIS, opts->min_response, nullptr, 0, h.key_base, h.key_lz);
    h.vmax = std::numeric_limits<float>::infinity();
    const bool bounded = std::isfinite(opts->max_response) && opts->max_response > opts->min_response;
    if (bounded) {
        h.vmax = opts->max_response;
        const uint32_t kmax = host_float_key(opts->max_response) + 1u;
        h.key_lz = kmax > h.key_base ? __builtin_clz(kmax - h.key_base) : 0;
    }
    h.value_flag = sb.pre_count;
    c->sel_dirty = true;  // until k_select is enqueued: it resets the control block
    FD_HIP_TRY(c, fdk::launch_heat_candidates(h, c->stream));
    SelectCall sc{};
    sc.batch = batch;
    sc.rows = rows;
    sc.cols = cols;
    sc.dist = opts->min_feature_distance;
    sc.need = static_cast<uint32_t>(opts->max_features);
    sc.cap = cap;
    sc.key_base = h.key_base;
    sc.key_lz = h.key_lz;
    sc.tie_idx_desc = 1;
    sc.value_flag = true;
    return run_select(c, sc, pi, sb, out_xy, out_stride, out_counts, outputs_on_device, heatmap_on_device);
}

// DirectlySelectGoodFeaturesWithDescriptors (nn_feature_point_detector.cpp:204-230) for the
// keypoint-list models (kSuperpointNms / kDiskNms, nn_feature_point_detector_superpoint.cpp:76-112,
// nn_feature_point_detector_disk.cpp:76-112): k_cand_lists (border dropped) + k_select in descending
// (score, raster index) order + k_nn_pick for the descriptor rows.
int fd_nn_select_list(fd_ctx *c, const int64_t *keypoints, const float *scores, const int64_t *counts, int64_t cap,
                      int inputs_on_device, int batch, int rows, int cols, const fd_nn_opts *opts,
                      const float *prior_xy, const int32_t *prior_counts, const float *cand_desc, int desc_dim,
                      float *out_desc, float *out_xy, int32_t out_stride, int32_t *out_counts, int outputs_on_device) {
    int rc = check_shape(c, FD_HARRIS, batch, rows, cols);
    if (rc) return rc;
    if (!opts || !out_xy || !out_counts || out_stride < 1) return fail(c, FD_ERR_INVALID, "bad output arguments");
    if (opts->invalid_boundary < 0) return fail(c, FD_ERR_INVALID, "invalid_boundary must be >= 0");
    if (opts->max_features < 0) return fail(c, FD_ERR_INVALID, "max_features must be >= 0");
    if (!counts || cap < 0 || cap > 0x7FFFFFFFll) return fail(c, FD_ERR_INVALID, "counts is NULL or cap out of range");
    if (cand_desc && (desc_dim < 1 || !out_desc)) return fail(c, FD_ERR_INVALID, "descriptors need desc_dim >= 1 and out_desc");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    if ((rc = refuse_sync_under_capture(c, outputs_on_device))) return rc;
    if (!inputs_on_device)
        for (int b = 0; b < batch; ++b)
            if (counts[b] < 0 || counts[b] > cap)
                return fail(c, FD_ERR_INVALID, "frame " + std::to_string(b) + ": keypoint count outside [0, cap]");
    if (cap > 0 && (!keypoints || !scores)) return fail(c, FD_ERR_INVALID, "keypoints / scores are NULL");
    const int64_t *dkp = keypoints, *dcnt = counts;
    const float *dsc = scores, *ddesc = cand_desc;
    if (!inputs_on_device) {  // one upload of the whole batch
        const size_t nb = static_cast<size_t>(batch) * static_cast<size_t>(cap);
        FD_HIP_TRY(c, ensure(c, c->c_x, sizeof(int64_t) * 2 * std::max<size_t>(nb, 1)));
        FD_HIP_TRY(c, ensure(c, c->c_resp, sizeof(float) * std::max<size_t>(nb, 1)));
        FD_HIP_TRY(c, ensure(c, c->c_counts, sizeof(int64_t) * batch));
        if (nb) {
            FD_HIP_TRY(c, hipMemcpyAsync(c->c_x.p, keypoints, sizeof(int64_t) * 2 * nb, hipMemcpyHostToDevice, c->stream));
            FD_HIP_TRY(c, hipMemcpyAsync(c->c_resp.p, scores, sizeof(float) * nb, hipMemcpyHostToDevice, c->stream));
        }
        FD_HIP_TRY(c, hipMemcpyAsync(c->c_counts.p, counts, sizeof(int64_t) * batch, hipMemcpyHostToDevice, c->stream));
        if (cand_desc && nb) {
            FD_HIP_TRY(c, ensure(c, c->n_map, sizeof(float) * nb * desc_dim));
            FD_HIP_TRY(c, hipMemcpyAsync(c->n_map.p, cand_desc, sizeof(float) * nb * desc_dim, hipMemcpyHostToDevice,
                                         c->stream));
            ddesc = as<float>(c->n_map);
        }
        dkp = as<int64_t>(c->c_x);
        dsc = as<float>(c->c_resp);
        dcnt = as<int64_t>(c->c_counts);
    }
    PriorInfo pi;
    rc = setup_priors(c, batch, rows, cols, opts->min_feature_distance, prior_xy, prior_counts, pi);
    if (rc) return rc;
    const int64_t lcap = std::max<int64_t>(cap, 64);
    SelectBufs sb{};
    rc = select_buffers(c, batch, lcap, sb);
    if (rc) return rc;
    fdk::CandInArgs a{};
    a.resp = dsc;
    a.kp = dkp;
    a.counts = dcnt;
    a.stride = cap;
    a.batch = batch;
    a.rows = rows;
    a.cols = cols;
    a.border = opts->invalid_boundary;
    a.list_resp = as<float>(c->list_resp);
    a.list_idx = as<uint32_t>(c->list_idx);
    a.list_cap = lcap;
    a.list_count = sb.list_count;
    a.hist0 = sb.hist0;
    a.key_base = host_float_key(-std::numeric_limits<float>::infinity()) - 1u;
    a.key_lz = 0;
    a.bad = sb.pre_count;
    c->sel_dirty = true;  // until k_select is enqueued: it resets the control block
    FD_HIP_TRY(c, fdk::launch_cand_lists(a, cap, c->stream));
    SelectCall sc{};
    sc.batch = batch;
    sc.rows = rows;
    sc.cols = cols;
    sc.dist = opts->min_feature_distance;
    sc.need = static_cast<uint32_t>(opts->max_features);
    sc.cap = lcap;
    sc.key_base = a.key_base;
    sc.key_lz = a.key_lz;
    sc.tie_idx_desc = 1;  // equal scores: raster index descending (ArgSort walked from the back; unpinned)
    sc.dup_keys = true;
    sc.grid_at_d0 = true;
    sc.value_flag = true;
    sc.value_msg = "a keypoint outside the frame, a NaN score or a bad keypoint count";
    // selection into device buffers first when the descriptor rows are wanted on the device
    float *sel_xy = out_xy;
    int32_t *sel_cnt = out_counts;
    if (cand_desc && !outputs_on_device) {
        FD_HIP_TRY(c, ensure(c, c->n_xy, sizeof(float) * 2 * static_cast<size_t>(out_stride) * batch));
        FD_HIP_TRY(c, ensure(c, c->n_counts, sizeof(int32_t) * batch));
        sel_xy = as<float>(c->n_xy);
        sel_cnt = as<int32_t>(c->n_counts);
    }
    rc = run_select(c, sc, pi, sb, sel_xy, out_stride, sel_cnt, cand_desc ? 1 : outputs_on_device, 1);
    if (rc) return rc;
    if (cand_desc) {
        fdk::NnPickArgs k{};
        k.kp = dkp;
        k.scores = dsc;
        k.counts = dcnt;
        k.stride_in = cap;
        k.desc = ddesc;
        k.dim = desc_dim;
        k.xy = sel_xy;
        k.n_sel = sel_cnt;
        k.out_stride = out_stride;
        k.batch = batch;
        float *dout = out_desc;
        if (!outputs_on_device) {
            FD_HIP_TRY(c, ensure(c, c->n_out, sizeof(float) * static_cast<size_t>(out_stride) * batch * desc_dim));
            dout = as<float>(c->n_out);
        }
        k.out = dout;
        FD_HIP_TRY(c, fdk::launch_nn_pick(k, c->stream));
        if (!outputs_on_device) {
            std::vector<uint32_t> st(static_cast<size_t>(batch));
            FD_HIP_TRY(c, hipMemcpyAsync(out_xy, sel_xy, sizeof(float) * 2 * static_cast<size_t>(out_stride) * batch,
                                         hipMemcpyDeviceToHost, c->stream));
            FD_HIP_TRY(c, hipMemcpyAsync(out_counts, sel_cnt, sizeof(int32_t) * batch, hipMemcpyDeviceToHost, c->stream));
            FD_HIP_TRY(c, hipMemcpyAsync(out_desc, dout, sizeof(float) * static_cast<size_t>(out_stride) * batch * desc_dim,
                                         hipMemcpyDeviceToHost, c->stream));
            FD_HIP_TRY(c, hipMemcpyAsync(st.data(), sb.status, sizeof(uint32_t) * batch, hipMemcpyDeviceToHost, c->stream));
            FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
            for (int b = 0; b < batch; ++b) {
                if (st[b] & FD_FRAME_VALUE_RANGE)
                    return fail(c, FD_ERR_INVALID, "frame " + std::to_string(b) + ": " + sc.value_msg);
                if (st[b] & FD_FRAME_GUARD)
                    return fail(c, FD_ERR_HIP, "internal: selection consistency guard tripped (status 0x" + hex(st[b]) +
                                                   ", frame " + std::to_string(b) + ")");
            }
        }
    }
    if (!inputs_on_device) FD_HIP_TRY(c, hipStreamSynchronize(c->stream));  // host inputs were copy sources
    return FD_OK;
}

int fd_nn_bias_relu(fd_ctx *c, const void *x, const void *bias, int64_t bias_len, void *y, int n, int h, int w, int ch,
                    int pool) {
    if (!c) return FD_ERR_INVALID;
    if (!x || !bias || !y) return fail(c, FD_ERR_INVALID, "bad arguments");
    if (bias_len != ch) return fail(c, FD_ERR_INVALID, "bias length must equal the channel count");
    if (n < 0 || h < 0 || w < 0 || ch <= 0 || ch % 8) return fail(c, FD_ERR_INVALID, "need n, h, w >= 0, c a multiple of 8");
    if (pool && ((h | w) & 1)) return fail(c, FD_ERR_INVALID, "pooling needs even h and w");
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(bias) | reinterpret_cast<uintptr_t>(y)) & 15)
        return fail(c, FD_ERR_INVALID, "pointers must be 16-byte aligned");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    FD_HIP_TRY(c, fdk::launch_bias_relu(x, bias, y, n, h, w, ch, pool, c->stream));
    return FD_OK;
}

int fd_nn_heat_softmax(fd_ctx *c, const void *semi, const void *bias, float *heat, int n, int hc, int wc) {
    if (!c) return FD_ERR_INVALID;
    if (!semi || !heat) return fail(c, FD_ERR_INVALID, "bad arguments");
    if (n < 0 || hc < 0 || wc < 0) return fail(c, FD_ERR_INVALID, "need n, hc, wc >= 0");
    if (static_cast<int64_t>(hc) * 8 * wc * 8 >= (int64_t(1) << 31) || hc > 65535 || n > 65535)
        return fail(c, FD_ERR_INVALID, "map too large");
    if (((reinterpret_cast<uintptr_t>(semi) | reinterpret_cast<uintptr_t>(bias)) & 1) || (reinterpret_cast<uintptr_t>(heat) & 3))
        return fail(c, FD_ERR_INVALID, "pointers must be 2-byte (semi, bias) / 4-byte (heat) aligned");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    FD_HIP_TRY(c, fdk::launch_nn_heat_softmax(semi, bias, heat, n, hc, wc, c->stream));
    return FD_OK;
}

int fd_nn_desc_normalize(fd_ctx *c, const void *x, const void *bias, float *y, int64_t cells, int ch) {
    if (!c) return FD_ERR_INVALID;
    if (!x || !y) return fail(c, FD_ERR_INVALID, "bad arguments");
    if (cells < 0 || ch <= 0 || ch % 8) return fail(c, FD_ERR_INVALID, "need cells >= 0 and c a multiple of 8");
    if ((cells + 3) / 4 >= (int64_t(1) << 31)) return fail(c, FD_ERR_INVALID, "too many cells");
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(bias) | reinterpret_cast<uintptr_t>(y)) & 15)
        return fail(c, FD_ERR_INVALID, "pointers must be 16-byte aligned");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    FD_HIP_TRY(c, fdk::launch_nn_desc_normalize(x, bias, y, cells, ch, c->stream));
    return FD_OK;
}

int fd_nn_conv3x3_c1(fd_ctx *c, const void *x, const void *weight, const void *bias, int64_t channels, void *y, int n,
                     int h, int w) {
    if (!c) return FD_ERR_INVALID;
    if (!x || !weight || !bias || !y) return fail(c, FD_ERR_INVALID, "bad arguments");
    if (channels < 8 || channels > 256 || channels % 8 || 256 % (channels / 8))
        return fail(c, FD_ERR_INVALID, "channels must be 8, 16, 32, 64, 128 or 256");
    if (n < 0 || h < 0 || w < 0) return fail(c, FD_ERR_INVALID, "need n, h, w >= 0");
    if (static_cast<int64_t>(n) * h >= (int64_t(1) << 31)) return fail(c, FD_ERR_INVALID, "n * h must be < 2^31");
    if (w > 4096) return fail(c, FD_ERR_INVALID, "w must be <= 4096");
    if ((reinterpret_cast<uintptr_t>(y) & 15) || (reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(weight) |
                                                  reinterpret_cast<uintptr_t>(bias)) & 1)
        return fail(c, FD_ERR_INVALID, "y must be 16-byte aligned, x / weight / bias 2-byte aligned");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    FD_HIP_TRY(c, fdk::launch_conv3x3_c1_bias_relu(x, weight, bias, y, n, h, w, static_cast<int>(channels), c->stream));
    return FD_OK;
}

int fd_nn_conv3x3_c64(fd_ctx *c, const void *x, const void *weight_packed, const void *bias, void *y, int n, int h,
                      int w, int pool, int y_channels, int y_offset) {
    if (!c) return FD_ERR_INVALID;
    if (!x || !weight_packed || !bias || !y) return fail(c, FD_ERR_INVALID, "bad arguments");
    if (n < 0 || h < 0 || w < 0) return fail(c, FD_ERR_INVALID, "need n, h, w >= 0");
    if (pool && ((h | w) & 1)) return fail(c, FD_ERR_INVALID, "pooling needs even h and w");
    if (y_channels < 64 || y_channels % 64 || y_offset < 0 || y_offset % 64 || y_offset + 64 > y_channels)
        return fail(c, FD_ERR_INVALID, "y_channels must be a multiple of 64 holding [y_offset, y_offset + 64)");
    if (static_cast<int64_t>(n) * ((h + 7) / 8) * ((w + 31) / 32) >= (int64_t(1) << 31))  // (K10's 8 x 32 tiles)
        return fail(c, FD_ERR_INVALID, "too many tiles");
    if (static_cast<int64_t>(h) * w * 128 >= (int64_t(1) << 31))  // (one frame's input: 32-bit buffer offsets)
        return fail(c, FD_ERR_INVALID, "frame too large (h * w * 64 channels * 2 B must be < 2^31)");
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(weight_packed) | reinterpret_cast<uintptr_t>(y)) & 15 ||
        reinterpret_cast<uintptr_t>(bias) & 1)
        return fail(c, FD_ERR_INVALID, "x, weight, y must be 16-byte aligned");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    FD_HIP_TRY(c, fdk::launch_conv3x3_c64(x, weight_packed, bias, y, n, h, w, pool, y_channels, y_offset, c->stream));
    return FD_OK;
}

int fd_nn_descriptors(fd_ctx *c, const float *map, int map_on_device, int map_layout, int batch, int channels,
                      int map_rows, int map_cols, const float *xy, const int32_t *counts, int32_t stride, float *out,
                      int io_on_device) {
    if (!c) return FD_ERR_INVALID;
    if (!map || !xy || !out) return fail(c, FD_ERR_INVALID, "bad arguments");
    if (batch < 1 || channels < 1 || map_rows < 1 || map_cols < 1 || stride < 0)
        return fail(c, FD_ERR_INVALID, "batch, channels, map_rows, map_cols must be >= 1");
    FD_HIP_TRY(c, hipSetDevice(c->device));
    if (stride == 0) return FD_OK;
    const size_t mapn = static_cast<size_t>(batch) * channels * map_rows * map_cols;
    const size_t slots = static_cast<size_t>(batch) * stride;
    if (map_layout != FD_MAP_NCHW && map_layout != FD_MAP_NHWC) return fail(c, FD_ERR_INVALID, "unknown map layout");
    fdk::NnDescArgs a{};
    a.nhwc = map_layout == FD_MAP_NHWC;
    a.batch = batch;
    a.channels = channels;
    a.map_rows = map_rows;
    a.map_cols = map_cols;
    a.stride = stride;
    a.map = map;
    if (!map_on_device) {
        FD_HIP_TRY(c, ensure(c, c->n_map, sizeof(float) * mapn));
        FD_HIP_TRY(c, hipMemcpyAsync(c->n_map.p, map, sizeof(float) * mapn, hipMemcpyHostToDevice, c->stream));
        a.map = as<float>(c->n_map);
    }
    if (io_on_device) {
        a.xy = xy;
        a.counts = counts;
        a.out = out;
    } else {
        FD_HIP_TRY(c, ensure(c, c->n_xy, sizeof(float) * 2 * slots));
        FD_HIP_TRY(c, ensure(c, c->n_out, sizeof(float) * channels * slots));
        FD_HIP_TRY(c, hipMemcpyAsync(c->n_xy.p, xy, sizeof(float) * 2 * slots, hipMemcpyHostToDevice, c->stream));
        a.xy = as<float>(c->n_xy);
        a.out = as<float>(c->n_out);
        if (counts) {
            FD_HIP_TRY(c, ensure(c, c->n_counts, sizeof(int32_t) * batch));
            FD_HIP_TRY(c, hipMemcpyAsync(c->n_counts.p, counts, sizeof(int32_t) * batch, hipMemcpyHostToDevice, c->stream));
            a.counts = as<int32_t>(c->n_counts);
        }
    }
    FD_HIP_TRY(c, fdk::launch_nn_desc(a, c->stream));
    if (!io_on_device) {
        for (int b = 0; b < batch; ++b) {
            const int n = counts ? std::min<int64_t>(static_cast<uint32_t>(counts[b]) & 0x01FFFFFFu, stride) : stride;
            if (n <= 0) continue;
            const size_t s0 = static_cast<size_t>(b) * stride;
            FD_HIP_TRY(c, hipMemcpyAsync(out + s0 * channels, a.out + s0 * channels, sizeof(float) * channels * n,
                                         hipMemcpyDeviceToHost, c->stream));
        }
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
    } else if (!map_on_device) {
        FD_HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    return FD_OK;
}

}  // extern "C"
