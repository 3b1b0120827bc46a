/*
 * fd_hip.h -- C ABI of the MI355X feature-detection hot path (libfdhip.so).
 *
 * Plain C, no HIP/torch types: pointers, sizes and status codes only. A context owns one HIP stream
 * (or borrows the caller's) and all device workspace; calls on different contexts may run
 * concurrently from different host threads (one context per GPU is the multi-GPU model).
 *
 * Each entry point names the reference interface it replaces (paths relative to
 * Horizon1026/Feature_Detector/src/). The reference has no FFI of its own: its seams are the C++
 * virtual FeaturePointDetector::ComputeCandidates (feature_point_detector.h:44, called at
 * feature_point_detector.cpp:20), the whole DetectGoodFeatures (feature_point_detector.h:29), and the
 * private FeatureLineDetector::ComputeLineLevelAngleMap (feature_line_detector.h:66, called at
 * feature_line_detector.cpp:22). The C++ drop-in classes in include/feature_detector/ call these.
 *
 * Conventions: every function returns FD_OK (0) or an FD_ERR_* code; fd_last_error() describes the
 * last failure on that context. Pointers flagged "*_on_device" are HIP device pointers on the
 * context's device, otherwise host pointers. Device-pointer calls are asynchronous on the context
 * stream; host-pointer outputs are complete when the call returns.
 */
#ifndef FD_HIP_H_
#define FD_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FD_OK 0
#define FD_ERR_INVALID 1  /* bad argument */
#define FD_ERR_HIP 2      /* HIP runtime error (allocation, launch, copy) */
#define FD_ERR_CAPACITY 3 /* an output capacity was too small; counts still report true sizes */

typedef struct fd_ctx fd_ctx;

/* Detector kinds: FeaturePointHarrisDetector (feature_point_harris_detector.h:9),
 * FeaturePointShiTomasDetector (feature_point_shi_tomas_detector.h:9),
 * FeaturePointFastDetector (feature_point_fast_detector.h:9). */
enum fd_point_kind { FD_HARRIS = 0, FD_SHI_TOMASI = 1, FD_FAST = 2 };

/* FeaturePointDetector::Options (feature_point_detector.h:15-20) fields used on the hot path.
 * The SubOptions of the reference are private constants and fixed here: Harris kAlpha = 0.04 and
 * kHalfPatchSize = 1 (feature_point_harris_detector.h:12-15), Shi-Tomasi kHalfPatchSize = 1
 * (feature_point_shi_tomas_detector.h:12-14), FAST kN = 12 and kMinPixelDiffValue = 15
 * (feature_point_fast_detector.h:12-15). */
typedef struct fd_point_opts {
    int32_t min_feature_distance; /* kMinFeatureDistance, default 15 */
    float min_valid_response;     /* kMinValidResponse,  default 0.1 */
} fd_point_opts;

/* ---- context ---------------------------------------------------------------------------------- */
int fd_ctx_create(int device, fd_ctx **out);
void fd_ctx_destroy(fd_ctx *ctx);
const char *fd_last_error(const fd_ctx *ctx);
/* Run on the caller's hipStream_t from now on (NULL = the HIP null stream, e.g. PyTorch's default
 * stream). A new context runs on a non-blocking stream of its own; fd_ctx_use_own_stream restores it. */
int fd_ctx_set_stream(fd_ctx *ctx, void *hip_stream);
int fd_ctx_use_own_stream(fd_ctx *ctx);
void *fd_ctx_get_stream(const fd_ctx *ctx);
int fd_ctx_synchronize(fd_ctx *ctx);
/* Pre-size device workspace for a (kind, batch, rows, cols) shape so that later calls of that shape
 * allocate nothing (required before hipGraph capture of fd_points_detect). Not covered: the global
 * occupancy grid of very small min_feature_distance (cells > 16384 per frame, e.g. 640x480 with d <= 4)
 * -- run one call of the shape before capturing. A call that would grow the workspace while its
 * stream is being captured fails (FD_ERR_HIP, "stream capture") instead of allocating. */
int fd_ctx_reserve(fd_ctx *ctx, int kind, int batch, int rows, int cols, int64_t max_prior_total);
/*
 * Order of equal responses in the selection (SelectGoodFeatures, feature_point_detector.cpp:58-60 sorts
 * with an unstable std::sort, so equal responses have no defined order):
 *   FD_TIES_RASTER     (default) response descending, equal responses by raster index ascending: a
 *                      total order, fully asynchronous and graph-capturable.
 *   FD_TIES_REFERENCE  the reference's own permutation: every frame whose greedy scan meets two equal
 *                      responses (FD_FRAME_TIES) is re-selected, on the GPU, in the order libstdc++'s
 *                      (GCC 11) std::sort leaves the raster-ordered candidates in (its introsort is
 *                      emulated over the visited prefix; FD_FRAME_RESOLVED). Frames without such a tie
 *                      are identical in both modes. Asynchronous and graph-capturable (reserve first,
 *                      fd_ctx_reserve after fd_ctx_set_tie_order). The depth limit's heapsort is emulated
 *                      too. A frame that breaks one of the emulation's capacity guards or its loop bound
 *                      gets FD_FRAME_UNRESOLVED instead: host-output calls then resolve it on the host;
 *                      device-output calls return k_select's raster-order features for it (if no window
 *                      of the reference order was scanned) or the features the reference order selected
 *                      before the stop (a prefix of the reference's result), with the flag in
 *                      fd_ctx_frame_status.
 * SuperPoint's fd_nn_select has a defined order (std::multimap) and ignores this setting.
 */
enum fd_tie_order { FD_TIES_RASTER = 0, FD_TIES_REFERENCE = 1 };
int fd_ctx_set_tie_order(fd_ctx *ctx, int order);

/*
 * Per-frame status words of the last selection call on this context (fd_points_detect, fd_nn_select):
 * FD_FRAME_* bits. Copies `batch` words to dst on the context stream (dst: device or host memory);
 * with async = 0 the call waits for the copy. Device-output calls return plain counts and leave their
 * flags here, so a caller can check them without a host round trip per call.
 */
#define FD_FRAME_TIES 0x00000001u       /* equal responses met in the greedy scan (order defined by the mode) */
#define FD_FRAME_RESOLVED 0x00000002u   /* re-selected in the reference's std::sort order (FD_TIES_REFERENCE) */
#define FD_FRAME_UNRESOLVED 0x00000004u /* FD_TIES_REFERENCE: the GPU emulation stopped (see fd_tie_order) */
#define FD_FRAME_REDETECTED 0x00000008u /* FAST, FD_TIES_RASTER: detected and selected a second time in the same call,
                                           without the adaptive emission cut (it was too high for this frame) */
#define FD_FRAME_VALUE_RANGE 0x40000000u /* fd_nn_select: a heatmap value above fd_nn_opts::max_response */
#define FD_FRAME_GUARD 0xBE000000u      /* internal consistency guard tripped (host-output calls fail FD_ERR_HIP) */
int fd_ctx_frame_status(fd_ctx *ctx, uint32_t *dst, int batch, int async);

/* Copy `bytes` of host memory into the context's frame staging buffer; *device_out receives its device
 * address, valid until the next call that stages frames on this context. Lets a caller run several
 * entry points on one upload (frames_on_device = 1). Synchronous. */
int fd_ctx_stage(fd_ctx *ctx, const void *host, int64_t bytes, const uint8_t **device_out);

/* ---- corner / FAST points ----------------------------------------------------------------------- */
/*
 * fd_points_detect -- FeaturePointDetector::DetectGoodFeatures (feature_point_detector.cpp:7-25) on a
 * batch of independent frames: mask from prior features (:12-16, :90-98), candidates
 * (ComputeCandidates: Harris feature_point_harris_detector.cpp:5-137, Shi-Tomasi
 * feature_point_shi_tomas_detector.cpp:5-137, FAST feature_point_fast_detector.cpp:11-98), sort by
 * response and greedy min-distance selection (SelectGoodFeatures :54-88).
 *
 *   frames        batch * rows * cols u8, row-major, frame-contiguous (GrayImage layout)
 *   prior_xy      all frames' incoming `features` (x, y float pairs) concatenated, or NULL
 *   prior_counts  batch entries (number of prior features of each frame), or NULL
 *   need          needed_feature_num (counts the prior features, checked after each append, :67-69)
 *   out_xy        batch * out_stride (x, y) float pairs: the NEW features of each frame, in order
 *   out_counts    batch int32: number of new features per frame (plain counts; per-frame flags are
 *                 in fd_ctx_frame_status)
 * Candidate order: response descending; equal responses as fd_ctx_set_tie_order says (default raster
 * index ascending; FD_TIES_REFERENCE = the reference's std::sort permutation, DESIGN.md "Tie order").
 * out_stride must be >= min(need, candidates) + 1.
 */
int fd_points_detect(fd_ctx *ctx, int kind, const uint8_t *frames, int frames_on_device, int batch, int rows,
                     int cols, const fd_point_opts *opts, const float *prior_xy, const int32_t *prior_counts,
                     uint32_t need, float *out_xy, int32_t out_stride, int32_t *out_counts, int outputs_on_device);

/*
 * fd_points_candidates -- the ComputeCandidates seam (feature_point_detector.h:44): per frame, the
 * candidates in the order the reference pushes them (raster order), as (response, x, y). Mask rules
 * as above. Writes at most cand_cap per frame at [b * cand_cap]; out_counts (int64) gets the true
 * count (FD_ERR_CAPACITY if any exceeds cand_cap). Optionally also returns the response map
 * (batch * rows * cols float, 0 where not stored; NULL to skip) -- Harris/Shi-Tomasi responses_
 * (feature_point_harris_detector.cpp:74-75,100-102); for FAST the map holds score + offset of every
 * candidate pixel and 0 elsewhere.
 */
int fd_points_candidates(fd_ctx *ctx, int kind, const uint8_t *frames, int frames_on_device, int batch, int rows,
                         int cols, const fd_point_opts *opts, const float *prior_xy, const int32_t *prior_counts,
                         float *out_resp, int32_t *out_x, int32_t *out_y, int64_t cand_cap, int64_t *out_counts,
                         float *out_response_map, int outputs_on_device);

/*
 * fd_points_select -- SelectGoodFeatures (feature_point_detector.cpp:54-88) over caller-supplied
 * candidates: the ComputeCandidates seam (feature_point_detector.h:44, called at
 * feature_point_detector.cpp:20) for a FeaturePointDetector subclass whose candidates come from
 * elsewhere. Frame b's candidates are (cand_resp, cand_x, cand_y)[b * cand_cap + i], i < cand_counts[b],
 * in the order ComputeCandidates pushed them; fd_points_candidates' outputs can be passed as they are.
 * Mask from the prior features as fd_points_detect (:12-16, :90-98); then sort by response and greedy
 * min-distance scan (the reference's SelectGoodFeatures does not filter by min_valid_response, and
 * neither does this call). Equal responses as fd_ctx_set_tie_order says: FD_TIES_RASTER orders them
 * by raster index, FD_TIES_REFERENCE by libstdc++'s std::sort of the pushed order. A pixel may be
 * listed more than once. Every candidate must lie in the frame and have a non-NaN response
 * (host outputs: FD_ERR_INVALID; device outputs: FD_FRAME_VALUE_RANGE in fd_ctx_frame_status).
 * cand_* and cand_counts are device pointers when cands_on_device, host pointers otherwise;
 * out_xy / out_counts as fd_points_detect.
 */
int fd_points_select(fd_ctx *ctx, int batch, int rows, int cols, const fd_point_opts *opts, const float *cand_resp,
                     const int32_t *cand_x, const int32_t *cand_y, const int64_t *cand_counts, int64_t cand_cap,
                     int cands_on_device, const float *prior_xy, const int32_t *prior_counts, uint32_t need,
                     float *out_xy, int32_t out_stride, int32_t *out_counts, int outputs_on_device);

/*
 * fd_points_response -- the per-pixel stage alone (response + NMS for Harris/Shi-Tomasi, segment test
 * + offset for FAST), i.e. ComputeCandidates without ordering: per frame, the candidates' responses
 * at out_resp[b * cand_cap] and raster indices (row * cols + col) at out_idx[b * cand_cap], in
 * unspecified order, and their count in out_counts[b]. Device pointers only (frames and outputs).
 * Used to time the hot kernel alone and by callers that select features themselves.
 */
int fd_points_response(fd_ctx *ctx, int kind, const uint8_t *frames, int batch, int rows, int cols,
                       const fd_point_opts *opts, float *out_resp, uint32_t *out_idx, int64_t cand_cap,
                       uint32_t *out_counts);

/*
 * fd_points_response_append -- fd_points_response without resetting out_counts: each frame's
 * candidates are appended after the out_counts[b] entries already there (slots past cand_cap are
 * counted but not written). A launch is then the corner/segment-test kernel alone, so a caller can
 * issue many back to back (or capture them in a HIP graph) to time the kernel by itself.
 */
int fd_points_response_append(fd_ctx *ctx, int kind, const uint8_t *frames, int batch, int rows, int cols,
                              const fd_point_opts *opts, float *out_resp, uint32_t *out_idx, int64_t cand_cap,
                              uint32_t *out_counts);

/* ---- LSD level-line map ------------------------------------------------------------------------ */
/*
 * fd_lsd_map -- FeatureLineDetector::ComputeLineLevelAngleMap (feature_line_detector.cpp:56-97).
 * Maps are (rows-1) x (cols-1) per frame, row-major, computed for row in [1, rows-3] and col in
 * [1, cols-3] and 0 elsewhere:
 *   norm   gradient_norm (:82)          (float, NULL to skip)
 *   angle  line_level_angle (:85)       (float, 0 where not valid; NULL to skip)
 *   valid  is_valid = norm > min_norm   (u8, NULL to skip)
 * valid_idx receives, per frame at [b * idx_cap], the row-major map index (row * (cols-1) + col) of
 * every valid pixel in the reference's scan order (column outer, row inner, :71-72, :86), i.e.
 * sorted_pixels_ before its std::sort (:92). valid_counts (int64) gets the true counts.
 */
int fd_lsd_map(fd_ctx *ctx, const uint8_t *frames, int frames_on_device, int batch, int rows, int cols, float min_norm,
               float *norm, float *angle, uint8_t *valid, int32_t *valid_idx, int64_t idx_cap, int64_t *valid_counts,
               int outputs_on_device);

/*
 * fd_lsd_map_pitched -- fd_lsd_map with dense maps of row pitch map_pitch entries (>= cols-1): row r of
 * frame b's maps starts at entry (b * (rows-1) + r) * map_pitch of norm / angle / valid (entries past
 * cols-2 in a row are left untouched, except that frames too small to scan -- rows or cols < 4 -- get
 * their maps cleared whole). The map indices in valid_idx stay row * (cols-1) + col. With a
 * pitch that is a multiple of 16 entries every map row starts 64-byte (f32) / 16-byte (u8) aligned and
 * the map kernel's row stores are aligned (the faster layout for device outputs; host outputs are
 * always computed that way and copied to the caller's pitch). fd_lsd_map = map_pitch cols-1.
 */
int fd_lsd_map_pitched(fd_ctx *ctx, const uint8_t *frames, int frames_on_device, int batch, int rows, int cols,
                       float min_norm, float *norm, float *angle, uint8_t *valid, int64_t map_pitch, int32_t *valid_idx,
                       int64_t idx_cap, int64_t *valid_counts, int outputs_on_device);

/* ---- LSD line segments (level-line map on the GPU, region growing on host threads) --------------- */
/* FeatureLineDetector::Options (feature_line_detector.h:40-45). */
typedef struct fd_lsd_opts {
    float min_valid_gradient_norm;         /* kMinValidGradientNorm (20) */
    float min_tolerance_angle_residual_rad; /* kMinToleranceAngleResidualInRad (22.5 deg as float) */
    float min_valid_line_length;           /* kMinValidLineLengthInPixel (20) */
    float max_tolerance_inlier_ratio;      /* kMaxToleranceInlierRation (0.6) */
} fd_lsd_opts;

/* FeatureLineDetector::RectangleParam (feature_line_detector.h:29-38) of an accepted segment, as the
 * reference leaves it in rectangles_ (start/end offset by +0.5, feature_line_detector.cpp:43-44). */
typedef struct fd_lsd_rect {
    float start[2], end[2], center[2]; /* (x, y) */
    float length, width, angle;
    float dir[2];
    float inlier_ratio;
} fd_lsd_rect;

/*
 * fd_lsd_lines -- FeatureLineDetector::DetectGoodFeatures (feature_line_detector.cpp:12-54) for a
 * batch of frames. The level-line map runs on the GPU in compact mode (no dense maps: per valid pixel
 * its map index, norm and angle in scan order, bit-exact to fd_lsd_map); the lists come back over PCIe
 * once and region growing + rectangle fitting (:99-228) run per frame on `threads` host threads
 * (<= 0: all hardware threads). Segment k of frame b is out_rects[b * rect_stride + k]; its endpoints
 * are the reference's features[k] = (start.x, start.y, end.x, end.y). out_counts[b] = segments found
 * (may exceed rect_stride: only rect_stride are written; FD_ERR_CAPACITY is not raised for lines).
 * needed == 0 returns FD_OK with counts 0 and no work (:15). frames may be host or device memory.
 * Unpinned semantics of the un-vendored Slam_Utility (CircularBuffer overflow, AngleDiffInRad): DESIGN.md.
 */
int fd_lsd_lines(fd_ctx *ctx, const uint8_t *frames, int frames_on_device, int batch, int rows, int cols,
                 const fd_lsd_opts *opts, uint32_t needed, fd_lsd_rect *out_rects, int32_t rect_stride,
                 int32_t *out_counts, int threads);

/*
 * fd_lsd_lines_state -- the last fd_lsd_lines call's frame 0 as the reference leaves its members
 * (pixels_ / sorted_pixels_, feature_line_detector.h:74-75): the valid pixels in scan order (map index,
 * norm, angle) and each one's final is_used flag. n receives the count; at most cap are written.
 */
int fd_lsd_lines_state(fd_ctx *ctx, int32_t *idx, float *norm, float *angle, uint8_t *used, int64_t cap, int64_t *n);

/* ---- ingest front end: PNG frames ----------------------------------------------------------------- */
/*
 * The reference loads frames with Visualizor2D::LoadImage (test/test_feature_point_detector.cpp:104,
 * un-vendored). PNG files with 8-bit samples, colour type gray / gray+alpha / RGB / RGBA, no interlace.
 * Colour becomes gray as (4899 R + 9617 G + 1868 B + 8192) >> 14 (BT.601; the reference's conversion
 * is parity-unpinned); alpha is dropped. Errors: FD_ERR_INVALID (not a PNG, corrupt or
 * unsupported variant), FD_ERR_CAPACITY (output too small).
 *
 * fd_png_info   -- geometry of one PNG (no context, no GPU).
 * fd_png_decode -- one PNG to a host gray image (host decode; the C++ loader uses it).
 * fd_png_frames -- a batch of same-size PNGs to device gray frames [n][rows][cols] (the layout
 *                  fd_points_detect / fd_lsd_lines take): zlib inflate + PNG row filters on `threads`
 *                  host threads (<= 0: all, capped by OMP_NUM_THREADS) into pinned memory, one H2D copy,
 *                  colour -> gray on the GPU, stream-ordered on the context stream.
 */
int fd_png_info(const uint8_t *png, size_t len, int32_t *rows, int32_t *cols, int32_t *channels);
int fd_png_decode(const uint8_t *png, size_t len, uint8_t *out_gray, size_t cap, int32_t *rows, int32_t *cols);
int fd_png_frames(fd_ctx *ctx, const uint8_t *const *pngs, const size_t *lens, int n, int rows, int cols,
                  uint8_t *frames_device, int threads);

/* ---- steered BRIEF descriptor ------------------------------------------------------------------- */
/* BriefDescriptor::Options (descriptor_brief.h:17-20) plus the float-coordinate sampler of the
 * un-vendored GrayImage (descriptor_brief.cpp:24,42-43; see DESIGN.md: parity unpinned). */
enum fd_sampler { FD_SAMPLE_BILINEAR = 0, FD_SAMPLE_TRUNCATE = 1 };
typedef struct fd_brief_opts {
    int32_t length;          /* kLength, bits per descriptor, 1..256 (default 256) */
    int32_t half_patch_size; /* kHalfPatchSize, moment patch half size, 0..255 (default 8) */
    int32_t sampler;         /* enum fd_sampler */
} fd_brief_opts;

/*
 * fd_brief_compute -- Descriptor<BriefType>::Compute (descriptor.h:27-40) with
 * BriefDescriptor::ComputeForOneFeature (descriptor_brief.cpp:8-50) per keypoint, for a batch of frames.
 * uv: [batch][stride][2] float (x = col, y = row), the layout fd_points_detect writes, so a device-side
 * detect -> describe chain needs no host round trip. counts: keypoints per frame (int32 [batch]; NULL =
 * stride each; bits 25..31 are ignored, so fd_points_detect's device counts can be passed as they are).
 * out_bits: [batch][stride][ceil(length/32)] uint32, descriptor bit i = bit (i % 32) of word i / 32
 * (bit i set <=> I(p1_i) < I(p2_i), descriptor_brief.cpp:44-46); keypoints outside the border
 * (:13-17) or with zero moment (:30) get all-zero words and out_valid 0 (NULL to skip out_valid).
 * Slots k >= counts[b] are not written. uv, counts, out_bits and out_valid are all device pointers
 * when io_on_device, all host pointers otherwise.
 */
int fd_brief_compute(fd_ctx *ctx, const uint8_t *frames, int frames_on_device, int batch, int rows, int cols,
                     const fd_brief_opts *opts, const float *uv, const int32_t *counts, int32_t stride,
                     uint32_t *out_bits, uint8_t *out_valid, int io_on_device);

/* ---- SuperPoint post-processing (the network runs in PyTorch-ROCm) -------------------------------- */
/* NNFeaturePointDetector::Options (nn_feature_point_detector.h:22-31) fields of the heatmap path. */
typedef struct fd_nn_opts {
    int32_t invalid_boundary;     /* kInvalidBoundary, default 3 */
    int32_t min_feature_distance; /* kMinFeatureDistance, default 15 */
    int32_t max_features;         /* kMaxNumberOfDetectedFeatures, default 240 (counts prior features) */
    float min_response;           /* kMinResponse, default 0.1 */
    float max_response;           /* upper bound of the heatmap values: 1.0 for SuperPoint's softmax
                                     probabilities (finer selection keys); a larger value fails the call
                                     (FD_ERR_INVALID). <= min_response or non-finite: no bound assumed */
} fd_nn_opts;

/*
 * fd_nn_select -- CreateMask + SelectKeypointCandidatesFromHeatMap + SelectGoodFeaturesFromCandidates
 * (nn_feature_point_detector.cpp:59-73, 128-155) for a batch of full-resolution heatmaps
 * [batch][rows][cols] (float). Candidates are heatmap values > min_response outside the invalid
 * boundary and the prior boxes; they are visited in the reference's std::multimap order (response
 * descending, equal responses by raster index descending) and kept greedily with the
 * min_feature_distance box rule until max_features (including the priors) exist. out_xy / out_counts
 * as fd_points_detect (new features only, selection order).
 */
int fd_nn_select(fd_ctx *ctx, const float *heatmap, int heatmap_on_device, int batch, int rows, int cols,
                 const fd_nn_opts *opts, const float *prior_xy, const int32_t *prior_counts, float *out_xy,
                 int32_t out_stride, int32_t *out_counts, int outputs_on_device);

/*
 * fd_nn_select_list -- the keypoint-list models (kSuperpointNms / kDiskNms, whose networks run NMS
 * in-graph): CreateMask + ArgSort + DirectlySelectGoodFeaturesWithDescriptors
 * (nn_feature_point_detector.cpp:59-73, 204-230; nn_feature_point_detector_superpoint.cpp:106-109,
 * nn_feature_point_detector_disk.cpp:106-109). Per frame b, counts[b] keypoints (u = x, v = y as int64
 * pairs, [b * cap + i]) with scores [b * cap + i] and optionally descriptor rows
 * cand_desc [(b * cap + i) * desc_dim ...]. Keypoints are visited by descending score; equal scores
 * by descending raster index, then descending list index (SlamOperation::ArgSort is un-vendored: its
 * order of equal scores is parity-unpinned). Masked ones (border, prior boxes) are skipped,
 * the rest kept until max_features (priors included) with the min_feature_distance box rule.
 * out_xy / out_counts as fd_nn_select; out_desc [b * out_stride + k][desc_dim] = the descriptor row
 * of new feature k (new features only, as the reference's `descriptors`). Inputs (keypoints, scores,
 * counts, cand_desc) are device pointers when inputs_on_device; outputs when outputs_on_device.
 */
int fd_nn_select_list(fd_ctx *ctx, const int64_t *keypoints, const float *scores, const int64_t *counts, int64_t cap,
                      int inputs_on_device, int batch, int rows, int cols, const fd_nn_opts *opts,
                      const float *prior_xy, const int32_t *prior_counts, const float *cand_desc, int desc_dim,
                      float *out_desc, float *out_xy, int32_t out_stride, int32_t *out_counts, int outputs_on_device);

/*
 * fd_nn_descriptors -- ExtractDescriptorsForSelectedFeatures (nn_feature_point_detector.cpp:163-193):
 * per feature (x, y) in xy [batch][stride][2] (counts as fd_brief_compute), bilinear samples at
 * (y / 8, x / 8) of each of the `channels` planes of the descriptor map (zero outside
 * [0, map_rows-1) x [0, map_cols-1)), into out [batch][stride][channels]. map_layout
 * FD_MAP_NCHW: [batch][channels][map_rows][map_cols] (the reference's per-channel matrices);
 * FD_MAP_NHWC: [batch][map_rows][map_cols][channels] (channels-last network output, read in place).
 * xy, counts and out are all device pointers when io_on_device, host pointers otherwise.
 */
enum fd_map_layout { FD_MAP_NCHW = 0, FD_MAP_NHWC = 1 };
int fd_nn_descriptors(fd_ctx *ctx, const float *map, int map_on_device, int map_layout, int batch, int channels,
                      int map_rows, int map_cols, const float *xy, const int32_t *counts, int32_t stride, float *out,
                      int io_on_device);

/*
 * fd_nn_bias_relu -- the NN detectors' bias + ReLU after a bias-free convolution, and with pool = 1 the
 * 2x2 / stride-2 max pool that follows (nn.MaxPool2d(2, 2)), in one pass over an NHWC (channels-last)
 * fp16 activation x [n][h][w][c] on the device: y = relu(x + bias[c]) ([n][h][w][c]; may alias x), or
 * its pooled [n][h/2][w/2][c]. Arithmetic as PyTorch's separate half-precision add / ReLU / max-pool ops
 * (the add in float, rounded to half); a NaN sum becomes 0 (torch.relu would keep it).
 * bias: bias_len fp16 values on the device, bias_len == c (FD_ERR_INVALID otherwise); c a multiple of 8;
 * pool needs even h and w; 16-byte aligned pointers. Runs on the context's stream.
 */
int fd_nn_bias_relu(fd_ctx *ctx, const void *x, const void *bias, int64_t bias_len, void *y, int n, int h, int w,
                    int c, int pool);

/*
 * fd_nn_conv3x3_c1 -- the NN encoders' first layer (one input channel, 3x3 filter, stride 1, zero padding
 * 1; SuperPoint conv1a) with its bias and ReLU, in one pass: y [n][h][w][channels] (channels-last fp16) =
 * relu(conv(x) + bias) for x [n][h][w] fp16 and weight [channels][1][3][3] fp16, all on the device. The
 * convolution sums its 9 products in float (FMA, tap order) and rounds to half; the bias is then added in
 * float and rounded (as a bias-free convolution followed by fd_nn_bias_relu). channels in {8, 16, 32, 64,
 * 128, 256}; w <= 4096; y 16-byte aligned. Runs on the context's stream.
 */
int fd_nn_conv3x3_c1(fd_ctx *ctx, const void *x, const void *weight, const void *bias, int64_t channels, void *y,
                     int n, int h, int w);

/*
 * fd_nn_conv3x3_c64 -- a 3x3 convolution from 64 to 64 channels (stride 1, zero padding 1; SuperPoint
 * conv1b / conv2a / conv2b) with its bias and ReLU and, with pool = 1, the 2x2 / stride-2 max pool, on the
 * matrix cores: x [n][h][w][64] channels-last fp16 -> channels [y_offset, y_offset + 64) of y
 * [n][h][w][y_channels] (or [n][h/2][w/2][y_channels]) fp16, with weight_packed [9 taps (ky, kx)][64 out][64 in]
 * fp16 and bias [64] fp16 (that block of output channels), all on the device; wider outputs (64 -> 128,
 * SuperPoint conv3a) are one call per 64-channel block. fp16 products summed in float; the sum rounded to
 * half, the bias added in float and rounded (as a bias-free convolution followed by fd_nn_bias_relu).
 * x, weight_packed, y 16-byte aligned; y_channels a multiple of 64; pool needs even h, w.
 */
int fd_nn_conv3x3_c64(fd_ctx *ctx, const void *x, const void *weight_packed, const void *bias, void *y, int n, int h,
                      int w, int pool, int y_channels, int y_offset);

/*
 * fd_nn_heat_softmax -- SuperPoint's detector-head output (the network's last stage after convPb:
 * softmax over a cell's 65 channels, the dustbin channel dropped, pixel_shuffle by 8): semi
 * [n][hc][wc][65] channels-last fp16 logits -> heat [n][8 hc][8 wc] float, heat[8i + r][8j + c] =
 * exp(x_{8r+c} - m) / sum_k exp(x_k - m) over the cell's 65 logits x (m their max), in float. bias
 * (optional, 65 fp16): convPb's bias, added to a bias-free convolution's output in half first. All on
 * the device, semi and bias 2-byte, heat 4-byte aligned. Runs on the context's stream.
 */
int fd_nn_heat_softmax(fd_ctx *ctx, const void *semi, const void *bias, float *heat, int n, int hc, int wc);

/*
 * fd_nn_desc_normalize -- SuperPoint's descriptor-head output (after convDb): every cell's c-channel
 * vector divided by max(||x||_2, 1e-12), in float: x [cells][c] fp16 (a channels-last map) -> y
 * [cells][c] float, all on the device; bias (optional, c fp16): convDb's bias, added in half first;
 * c a multiple of 8; x, bias and y 16-byte aligned. Runs on the context's stream.
 */
int fd_nn_desc_normalize(fd_ctx *ctx, const void *x, const void *bias, float *y, int64_t cells, int c);

/* ---- build info --------------------------------------------------------------------------------- */
const char *fd_build_info(void);

/*
 * ABI version of this header: bumped whenever an entry point's parameter list changes or one is removed
 * (5: int64_t bias_len in fd_nn_bias_relu; 6: fd_nn_conv3x3_c1c64 removed -- the fused first layers
 * measured slower than fd_nn_conv3x3_c1 + fd_nn_conv3x3_c64). Bindings compare fd_abi_version() with the FD_ABI_VERSION they were
 * written for and refuse a mismatched library, instead of passing misread arguments.
 */
#define FD_ABI_VERSION 6
int fd_abi_version(void);

/* ---- ingest: pinned, pipelined host frames -> features ------------------------ */
/*
 * A streaming front end for DetectGoodFeatures on host frames (what the reference's callers do per
 * frame after Visualizor2D::LoadImage, test_feature_point_detector.cpp:104-110): `depth` slots, each
 * a pinned host buffer for `batch` frames plus device buffers. fd_ingest_submit copies a slot to the
 * GPU on the ingest's own copy stream and queues detection (fd_points_detect) and the copy-back of
 * the features on the context stream, so the upload of slot i+1 overlaps the detection of slot i.
 * The host fills a slot's frames in place (fd_ingest_frames) and collects its features with
 * fd_ingest_wait; slots are reused round-robin by the caller. One ingest per context at a time (its
 * detections share the context workspace, serialised on the context stream).
 */
typedef struct fd_ingest fd_ingest;
int fd_ingest_create(fd_ctx *ctx, int kind, int batch, int rows, int cols, int depth, uint32_t need,
                     int32_t out_stride, fd_ingest **out);
void fd_ingest_destroy(fd_ingest *ing);
/* pinned host buffer of slot `slot`: batch * rows * cols bytes (GrayImage layout) */
uint8_t *fd_ingest_frames(fd_ingest *ing, int slot);
/* queue slot `slot` (its frames written) with these options; returns without waiting */
int fd_ingest_submit(fd_ingest *ing, int slot, const fd_point_opts *opts);
/* wait for slot `slot`; *xy -> batch * out_stride (x, y) pairs, *counts -> batch new-feature counts
 * (pinned host memory owned by the ingest, valid until the slot is submitted again) */
int fd_ingest_wait(fd_ingest *ing, int slot, const float **xy, const int32_t **counts);

#ifdef __cplusplus
}
#endif

#endif /* FD_HIP_H_ */
