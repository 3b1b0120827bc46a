// =====================================================================================================
// fd_oracle.cpp -- CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and only
// as the checker (or as the timed CPU baseline). The product path (feature_detector_amd/, libfdhip.so)
// never links, loads or calls it; it fails loudly when the HIP library is missing.
//
// Reference: Horizon1026/Feature_Detector (read-only at /root/reference). Every function cites the
// reference file:line it restates. All paths are relative to /root/reference/src/.
//
// Parity pinning: PARITY UNPINNED. The reference cannot be built here without writing stand-ins for
// its un-vendored Slam_Utility headers (and Eigen), which this project does not do, so no
// oracle/_ref build exists, and the reference ships no golden vectors. The only recorded reference
// outputs are the candidate / feature / LSD counts of SURVEY.md §8c, and those came from a survey
// probe built against stand-in headers, so they do not pin anything either: tests/
// test_oracle_pinning.py reproduces them as a consistency check only. The survey's FNV digests of
// the feature lists were not reproducible (their byte format is not recorded) and are not checked.
//
// Float semantics: build with -O2 -ffp-contract=off and no -march, exactly like the reference's
// x86-64 build (CMakeLists.txt:6 has no -march, so no FMA). Every float expression below keeps the
// reference's operation order.
// =====================================================================================================
#include <algorithm>
#include <map>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct Cand {
    float response;
    int32_t x;  // col
    int32_t y;  // row
};

// Reference comparator: feature_point_detector.cpp:58-60 (unstable std::sort, response desc).
void SortCandidates(std::vector<Cand> &c, int sort_mode) {
    if (sort_mode == 0) {
        std::sort(c.begin(), c.end(), [](const Cand &a, const Cand &b) { return a.response > b.response; });
    } else {
        // Deterministic total order used by the HIP path: response desc, raster index asc.
        std::stable_sort(c.begin(), c.end(), [](const Cand &a, const Cand &b) { return a.response > b.response; });
    }
}

// Mask construction: feature_point_detector.cpp:12-16 (all ones) and :90-98 + :76-88 (boxes of
// radius kMinFeatureDistance around truncated prior features, clipped to the image).
void BuildMask(std::vector<int32_t> &mask, int rows, int cols, int dist, const float *prior_xy, int n_prior) {
    mask.assign(static_cast<size_t>(rows) * cols, 1);
    for (int i = 0; i < n_prior; ++i) {
        const int32_t r0 = static_cast<int32_t>(prior_xy[2 * i + 1]);  // :93 row = feature.y()
        const int32_t c0 = static_cast<int32_t>(prior_xy[2 * i + 0]);  // :94 col = feature.x()
        for (int32_t dr = -dist; dr <= dist; ++dr) {
            for (int32_t dc = -dist; dc <= dist; ++dc) {
                const int32_t r = r0 + dr, c = c0 + dc;
                if (r < 0 || c < 0 || r > rows - 1 || c > cols - 1) continue;  // :81-83
                mask[static_cast<size_t>(r) * cols + c] = 0;
            }
        }
    }
}

void DrawBox(std::vector<int32_t> &mask, int rows, int cols, int dist, int32_t r0, int32_t c0) {
    for (int32_t dr = -dist; dr <= dist; ++dr)
        for (int32_t dc = -dist; dc <= dist; ++dc) {
            const int32_t r = r0 + dr, c = c0 + dc;
            if (r < 0 || c < 0 || r > rows - 1 || c > cols - 1) continue;
            mask[static_cast<size_t>(r) * cols + c] = 0;
        }
}

}  // namespace

extern "C" {

int orc_version(void) { return 1; }

// -----------------------------------------------------------------------------------------------------
// Structure tensor sums (feature_point_harris_detector.cpp:17-64 horizontal pass, :66-88/:108-116
// vertical pass; byte-identical in feature_point_shi_tomas_detector.cpp). Central differences
// ix = I[r][c+1]-I[r][c-1], iy = I[r+1][c]-I[r-1][c] (:35-41); 3x3 box sums. The reference keeps
// these sums in float, but every partial sum is an integer of magnitude < 2^24, so they are exact
// and equal to the int32 sums computed here. Output is defined for r in [2,R-3], c in [2,C-3].
// -----------------------------------------------------------------------------------------------------
void orc_tensor_sums(const uint8_t *img, int rows, int cols, int32_t *sxx, int32_t *syy, int32_t *sxy) {
    const size_t n = static_cast<size_t>(rows) * cols;
    std::memset(sxx, 0, n * 4);
    std::memset(syy, 0, n * 4);
    std::memset(sxy, 0, n * 4);
    for (int r = 2; r < rows - 2; ++r) {
        for (int c = 2; c < cols - 2; ++c) {
            int32_t a = 0, b = 0, d = 0;
            for (int dr = -1; dr <= 1; ++dr) {
                for (int dc = -1; dc <= 1; ++dc) {
                    const int rr = r + dr, cc = c + dc;
                    const int32_t ix = int32_t(img[rr * cols + cc + 1]) - int32_t(img[rr * cols + cc - 1]);
                    const int32_t iy = int32_t(img[(rr + 1) * cols + cc]) - int32_t(img[(rr - 1) * cols + cc]);
                    a += ix * ix;
                    b += iy * iy;
                    d += ix * iy;
                }
            }
            sxx[r * cols + c] = a;
            syy[r * cols + c] = b;
            sxy[r * cols + c] = d;
        }
    }
}

// -----------------------------------------------------------------------------------------------------
// Response map. kind 0 = Harris (feature_point_harris_detector.cpp:66-118, response at :94-104),
// kind 1 = Shi-Tomasi (feature_point_shi_tomas_detector.cpp:66-118, response at :94-103).
// responses_ is zero-filled (:74-75) and written only where mask != 0 and res > thr, for
// r in [bound, R-bound), c in [bound, C-bound), bound = kHalfPatchSize + 1 = 2 (:89-91).
// mask may be NULL (all ones: feature_point_detector.cpp:13).
// -----------------------------------------------------------------------------------------------------
void orc_response_map(const uint8_t *img, int rows, int cols, int kind, float thr, const int32_t *mask, float *resp) {
    const size_t n = static_cast<size_t>(rows) * cols;
    std::vector<int32_t> sxx(n), syy(n), sxy(n);
    orc_tensor_sums(img, rows, cols, sxx.data(), syy.data(), sxy.data());
    std::memset(resp, 0, n * sizeof(float));
    const float inv_cnt = 1.0f / static_cast<float>(3 * 3);  // :71
    const float inv_cnt2 = inv_cnt * inv_cnt;                // harris :72
    const float k_alpha = 0.04f;                             // feature_point_harris_detector.h:13
    for (int r = 2; r < rows - 2; ++r) {
        for (int c = 2; c < cols - 2; ++c) {
            const size_t i = static_cast<size_t>(r) * cols + c;
            if (mask != nullptr && mask[i] == 0) continue;
            if (kind == 0) {
                const float fxx = static_cast<float>(sxx[i]);
                const float fyy = static_cast<float>(syy[i]);
                const float trace = fxx + fyy;
                if (trace * trace * 0.21f * inv_cnt2 > thr) {
                    const float fxy = static_cast<float>(sxy[i]);
                    const float res = (fxx * fyy - fxy * fxy - k_alpha * trace * trace) * inv_cnt2;
                    if (res > thr) resp[i] = res;
                }
            } else {
                const float a = static_cast<float>(sxx[i]) * inv_cnt;
                const float cv = static_cast<float>(syy[i]) * inv_cnt;
                if (a + cv > thr) {
                    const float b = static_cast<float>(sxy[i]) * inv_cnt;
                    const float diff = a - cv;
                    const float common = std::sqrt(diff * diff + 4.0f * b * b);
                    const float res = (a + cv + common) * 0.5f;
                    if (res > thr) resp[i] = res;
                }
            }
        }
    }
}

// -----------------------------------------------------------------------------------------------------
// 4-neighbour strict NMS + raster-order extraction (feature_point_harris_detector.cpp:120-137).
// Returns the number of candidates (writes at most cap).
// -----------------------------------------------------------------------------------------------------
int64_t orc_nms(const float *resp, int rows, int cols, float thr, float *out_resp, int32_t *out_x, int32_t *out_y,
                int64_t cap) {
    int64_t n = 0;
    for (int r = 2; r < rows - 2; ++r) {
        const float *row = resp + static_cast<size_t>(r) * cols;
        for (int c = 2; c < cols - 2; ++c) {
            const float v = row[c];
            if (v <= thr) continue;  // :130
            if (v > row[c - 1] && v > row[c + 1] && v > row[c - cols] && v > row[c + cols]) {  // :131-132
                if (n < cap) {
                    out_resp[n] = v;
                    out_x[n] = c;
                    out_y[n] = r;
                }
                ++n;
            }
        }
    }
    return n;
}

// -----------------------------------------------------------------------------------------------------
// FAST score of one pixel (feature_point_fast_detector.cpp:11-81) with kN = 12, diff = 15
// (feature_point_fast_detector.h:13-14). Ring offsets {dx, dy}: :7-8.
// -----------------------------------------------------------------------------------------------------
static const int32_t kRing[16][2] = {{0, -3}, {1, -3}, {2, -2}, {3, -1}, {3, 0},  {3, 1},   {2, 2},   {1, 3},
                                     {0, 3},  {-1, 3}, {-2, 2}, {-3, 1}, {-3, 0}, {-3, -1}, {-2, -2}, {-1, -3}};

int32_t orc_fast_score(const uint8_t *img, int cols, int row, int col, int n_arc, int diff) {
    const int32_t p = img[row * cols + col];
    const int32_t hi = p + diff, lo = p - diff;  // :13-14
    auto at = [&](int k) { return int32_t(img[(row + kRing[k][1]) * cols + col + kRing[k][0]]); };
    if (n_arc >= 12) {  // :20-42 cardinal pre-check; passes iff the trailing run over {0,4,8,12} is >= 3
        int32_t nb = 0, nd = 0;
        const int idx[4] = {0, 4, 8, 12};
        for (int k : idx) {
            const int32_t v = at(k);
            if (v > hi) { ++nb; nd = 0; }
            else if (v < lo) { ++nd; nb = 0; }
            else { nb = 0; nd = 0; }
        }
        if (nd < 3 && nb < 3) return 0;
    }
    int32_t cmp[16];
    for (int k = 0; k < 16; ++k) {  // :44-52
        const int32_t v = at(k);
        cmp[k] = v > hi ? 1 : (v < lo ? -1 : 0);
    }
    int32_t nb = 0, nd = 0, best = 0;  // :55-78, two passes, counters not reset between passes
    for (int pass = 0; pass < 2 && best < 16; ++pass) {
        for (int k = 0; k < 16; ++k) {
            if (cmp[k] == 1) { ++nb; nd = 0; }
            else if (cmp[k] == -1) { ++nd; nb = 0; }
            else { nb = 0; nd = 0; }
            if (nb > best) best = nb;
            if (nd > best) best = nd;
        }
    }
    return best;
}

// FAST candidates (feature_point_fast_detector.cpp:83-98): running float offset, no NMS.
int64_t orc_fast_candidates(const uint8_t *img, int rows, int cols, float thr, const int32_t *mask, float *out_resp,
                            int32_t *out_x, int32_t *out_y, int64_t cap) {
    const int bound = 3;  // :84 kHalfPatchSize
    float offset = 1e-5f;  // :85
    int64_t n = 0;
    for (int r = bound; r < rows - bound; ++r) {
        for (int c = bound; c < cols - bound; ++c) {
            if (mask != nullptr && mask[static_cast<size_t>(r) * cols + c] == 0) continue;
            const float response = static_cast<float>(orc_fast_score(img, cols, r, c, 12, 15)) + offset;
            if (response > thr) {
                if (n < cap) {
                    out_resp[n] = response;
                    out_x[n] = c;
                    out_y[n] = r;
                }
                ++n;
            }
            offset += 1e-5f;  // :93
        }
    }
    return n;
}

// The offset sequence o_0 = 1e-5f, o_{k+1} = fl(o_k + 1e-5f) (feature_point_fast_detector.cpp:85,93).
void orc_fast_offsets(int64_t n, float *out) {
    float o = 1e-5f;
    for (int64_t k = 0; k < n; ++k) {
        out[k] = o;
        o += 1e-5f;
    }
}

// SelectGoodFeatures (feature_point_detector.cpp:54-74) over `cand` in the order ComputeCandidates
// pushed them: sort (sort_mode 0: the reference's std::sort; 1: response desc, raster index asc --
// the HIP path's FD_TIES_RASTER order), then the greedy scan against `mask`. Returns the new features.
static int SelectGoodFeatures(std::vector<Cand> &cand, std::vector<int32_t> &mask, int rows, int cols, int dist,
                              uint32_t need, int n_prior, int sort_mode, float *out_xy, int out_cap) {
    int nout = 0;
    size_t total = static_cast<size_t>(n_prior);
    if (cand.empty()) return 0;  // :55
    if (sort_mode == 1)  // raster order first (a no-op for the built-in detectors' raster-pushed lists)
        std::stable_sort(cand.begin(), cand.end(), [cols](const Cand &a, const Cand &b) {
            return static_cast<int64_t>(a.y) * cols + a.x < static_cast<int64_t>(b.y) * cols + b.x;
        });
    SortCandidates(cand, sort_mode);
    for (const Cand &c : cand) {
        if (mask[static_cast<size_t>(c.y) * cols + c.x]) {
            if (nout < out_cap) {
                out_xy[2 * nout] = static_cast<float>(c.x);
                out_xy[2 * nout + 1] = static_cast<float>(c.y);
            }
            ++nout;
            ++total;
            if (total >= need) break;  // :67-69 checked after the append
            DrawBox(mask, rows, cols, dist, c.y, c.x);
        }
    }
    return nout;
}

// -----------------------------------------------------------------------------------------------------
// Full FeaturePointDetector::DetectGoodFeatures (feature_point_detector.cpp:7-25) for one frame.
//   kind: 0 Harris, 1 Shi-Tomasi, 2 FAST.  sort_mode: 0 reference std::sort, 1 stable.
//   prior_xy/n_prior: the incoming `features` vector (x, y pairs). New features are written to out_xy
//   (x, y pairs, at most out_cap) and their count returned via *out_n. Candidates (sorted as the
//   reference leaves candidates() after the call) go to cand_* (at most cand_cap); their total count
//   is the return value.
// -----------------------------------------------------------------------------------------------------
int64_t orc_detect(int kind, const uint8_t *img, int rows, int cols, int dist, float thr, uint32_t need,
                   const float *prior_xy, int n_prior, int sort_mode, float *out_xy, int out_cap, int *out_n,
                   float *cand_resp, int32_t *cand_x, int32_t *cand_y, int64_t cand_cap) {
    std::vector<int32_t> mask;
    BuildMask(mask, rows, cols, dist, prior_xy, n_prior);  // :12-16
    const bool all_ones = (n_prior == 0);
    const size_t np = static_cast<size_t>(rows) * cols;
    std::vector<Cand> cand;
    {
        std::vector<float> r(np / 2 + 16);
        std::vector<int32_t> cx(np / 2 + 16), cy(np / 2 + 16);
        int64_t n;
        if (kind == 2) {
            std::vector<float> fr(np);
            std::vector<int32_t> fx(np), fy(np);
            n = orc_fast_candidates(img, rows, cols, thr, all_ones ? nullptr : mask.data(), fr.data(), fx.data(),
                                    fy.data(), static_cast<int64_t>(np));
            cand.resize(static_cast<size_t>(n));
            for (int64_t i = 0; i < n; ++i) cand[i] = {fr[i], fx[i], fy[i]};
        } else {
            std::vector<float> resp(np);
            orc_response_map(img, rows, cols, kind, thr, all_ones ? nullptr : mask.data(), resp.data());
            n = orc_nms(resp.data(), rows, cols, thr, r.data(), cx.data(), cy.data(), static_cast<int64_t>(r.size()));
            cand.resize(static_cast<size_t>(n));
            for (int64_t i = 0; i < n; ++i) cand[i] = {r[i], cx[i], cy[i]};
        }
    }
    *out_n = SelectGoodFeatures(cand, mask, rows, cols, dist, need, n_prior, sort_mode, out_xy, out_cap);
    for (size_t i = 0; i < cand.size() && static_cast<int64_t>(i) < cand_cap; ++i) {
        cand_resp[i] = cand[i].response;
        cand_x[i] = cand[i].x;
        cand_y[i] = cand[i].y;
    }
    return static_cast<int64_t>(cand.size());
}

// SelectGoodFeatures alone over caller-supplied candidates (a subclass's ComputeCandidates, the
// fd_points_select seam): mask from the prior features (:12-16, :90-98), then the sort and greedy scan
// of SelectGoodFeatures. Candidates must lie inside the image. Returns the number of new features.
// sorted_* (nullable, n entries): the candidates as SelectGoodFeatures leaves them sorted (candidates()).
int orc_select(const float *resp, const int32_t *x, const int32_t *y, int64_t n, int rows, int cols, int dist,
               uint32_t need, const float *prior_xy, int n_prior, int sort_mode, float *out_xy, int out_cap,
               float *sorted_resp, int32_t *sorted_x, int32_t *sorted_y) {
    std::vector<int32_t> mask;
    BuildMask(mask, rows, cols, dist, prior_xy, n_prior);
    std::vector<Cand> cand(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) cand[i] = {resp[i], x[i], y[i]};
    const int nout = SelectGoodFeatures(cand, mask, rows, cols, dist, need, n_prior, sort_mode, out_xy, out_cap);
    if (sorted_resp)
        for (int64_t i = 0; i < n; ++i) {
            sorted_resp[i] = cand[i].response;
            sorted_x[i] = cand[i].x;
            sorted_y[i] = cand[i].y;
        }
    return nout;
}

// Tie check for the greedy scan: returns 1 if, within the prefix of sorted candidates that the greedy
// loop visits, two adjacent candidates share a response (the only place where an unstable sort can
// change the output). cand_* must be sorted (either mode); n_scanned = index of the last visited + 1.
int orc_prefix_has_ties(const float *cand_resp, int64_t n_scanned) {
    for (int64_t i = 1; i < n_scanned; ++i)
        if (cand_resp[i] == cand_resp[i - 1]) return 1;
    return 0;
}

// -----------------------------------------------------------------------------------------------------
// SparsifyFeatures (feature_point_detector.cpp:27-52). status has n entries (resized to 1s by the
// caller when its size differs, :29-31). grid_mask receives the final grid_rows x grid_cols mask.
// -----------------------------------------------------------------------------------------------------
void orc_sparsify(const float *xy, int n, int rows, int cols, int grid_rows, int grid_cols, uint8_t need_filter,
                  uint8_t after_filter, uint8_t *status, int32_t *grid_mask) {
    const float row_step = rows / (grid_rows - 1);  // :34 integer division, then float
    const float col_step = cols / (grid_cols - 1);  // :35
    for (int i = 0; i < grid_rows * grid_cols; ++i) grid_mask[i] = 1;
    for (int i = 0; i < n; ++i) {
        const int32_t r = static_cast<int32_t>(xy[2 * i + 1] / row_step);
        const int32_t c = static_cast<int32_t>(xy[2 * i] / col_step);
        if (r < 0 || r > grid_rows - 1 || c < 0 || c > grid_cols - 1) {
            status[i] = after_filter;
            continue;
        }
        int32_t &m = grid_mask[r * grid_cols + c];
        if (m && status[i] == need_filter) m = 0;
        else if (!m && status[i] == need_filter) status[i] = after_filter;
    }
}

// -----------------------------------------------------------------------------------------------------
// LSD level-line map (feature_line_detector.cpp:56-97). Maps are (R-1) x (C-1), row-major here (the
// reference's Eigen matrix is column-major; the element values are what matters). Written only for
// row in [1, R-3], col in [1, C-3] (:71-72); elsewhere 0/false. valid_colmajor receives the linear
// row-major index (row * (C-1) + col) of every valid pixel in the reference's scan order (column
// outer, row inner: :71-72, :86) -- i.e. sorted_pixels_ before the std::sort at :92.
// Returns the number of valid pixels.
// -----------------------------------------------------------------------------------------------------
int64_t orc_lsd_map(const uint8_t *img, int rows, int cols, float min_norm, float *norm, float *angle, uint8_t *valid,
                    int32_t *valid_colmajor, int64_t cap) {
    const int pr = rows - 1, pc = cols - 1;
    std::memset(norm, 0, sizeof(float) * pr * pc);
    std::memset(angle, 0, sizeof(float) * pr * pc);
    std::memset(valid, 0, static_cast<size_t>(pr) * pc);
    int64_t n = 0;
    for (int col = 1; col < cols - 2; ++col) {
        for (int row = 1; row < rows - 2; ++row) {
            const int32_t ad = int32_t(img[(row + 1) * cols + col + 1]) - int32_t(img[row * cols + col]);  // :76-77
            const int32_t bc = int32_t(img[row * cols + col + 1]) - int32_t(img[(row + 1) * cols + col]);  // :78-79
            const float gx = static_cast<float>(ad + bc) / 2.0f;  // :80
            const float gy = static_cast<float>(ad - bc) / 2.0f;  // :81
            const float nrm = std::sqrt(gx * gx + gy * gy);      // :82
            const size_t i = static_cast<size_t>(row) * pc + col;
            norm[i] = nrm;
            if (nrm > min_norm) {  // :83
                valid[i] = 1;
                angle[i] = std::atan2(gx, -gy);  // :85
                if (n < cap) valid_colmajor[n] = static_cast<int32_t>(i);
                ++n;
            }
        }
    }
    return n;
}

// sorted_pixels_ after the reference's unstable std::sort by norm desc (feature_line_detector.cpp:92-94),
// applied to the column-major scan-order list. idx is sorted in place.
void orc_lsd_sort(const float *norm, int32_t *idx, int64_t n, int sort_mode) {
    if (sort_mode == 0)
        std::sort(idx, idx + n, [&](int32_t a, int32_t b) { return norm[a] > norm[b]; });
    else
        std::stable_sort(idx, idx + n, [&](int32_t a, int32_t b) { return norm[a] > norm[b]; });
}

// LSD min_region_size (feature_line_detector.cpp:17-20).
uint32_t orc_lsd_min_region_size(int rows, int cols, float tol_rad) {
    const float pi = 3.14159265358979323846f;
    const float p = tol_rad / pi;
    const float log_nt = 5.0f * (std::log10(double(cols)) + std::log10(double(rows))) / 2.0f + std::log10(11.0f);
    return static_cast<uint32_t>(-log_nt / std::log10(p));
}

// -----------------------------------------------------------------------------------------------------
// Steered BRIEF, BriefDescriptor::ComputeForOneFeature (feature_descriptor/descriptor_brief.cpp:8-50),
// looped over keypoints as Descriptor<BriefType>::Compute (descriptor.h:27-40).
// pattern: the reference's pattern_idx_ (descriptor_brief.cpp:52-309) as int16[4 * 256]
// (dcol1, drow1, dcol2, drow2), passed in by the caller.
// sampler: GrayImage::GetPixelValueNoCheck(float row, float col) is un-vendored Slam_Utility code
// (parity unpinned): 0 = bilinear ((1-ex)(1-ey), ex(1-ey), (1-ex)ey, ex*ey, summed left to right),
// 1 = truncation. Reads use the row-major linear index row * cols + col like the NoCheck accessor;
// an index outside the frame reads 0 (the reference would read out of bounds).
// kZeroFloat (slam_basic_math.h, un-vendored) = 1e-6f: only |m| in (0, 1) could depend on it, which
// integer keypoints never produce.
// out_bits: n x ceil(length/32) words, bit i of the descriptor = bit i%32 of word i/32.
// out_valid (may be NULL): ComputeForOneFeature's return value. out_m (may be NULL): m10, m01, m.
// -----------------------------------------------------------------------------------------------------
static float BriefPixel(const uint8_t *img, int rows, int cols, int32_t r, int32_t c) {
    const int64_t idx = static_cast<int64_t>(r) * cols + c;
    if (idx < 0 || idx >= static_cast<int64_t>(rows) * cols) return 0.0f;
    return static_cast<float>(img[idx]);
}

static float BriefSample(const uint8_t *img, int rows, int cols, float row, float col, int sampler) {
    const int32_t r0 = static_cast<int32_t>(row);
    const int32_t c0 = static_cast<int32_t>(col);
    if (sampler == 1) return BriefPixel(img, rows, cols, r0, c0);
    const float ex = col - static_cast<float>(c0);
    const float ey = row - static_cast<float>(r0);
    const float ex1 = 1.0f - ex;
    const float ey1 = 1.0f - ey;
    return ex1 * ey1 * BriefPixel(img, rows, cols, r0, c0) + ex * ey1 * BriefPixel(img, rows, cols, r0, c0 + 1) +
           ex1 * ey * BriefPixel(img, rows, cols, r0 + 1, c0) + ex * ey * BriefPixel(img, rows, cols, r0 + 1, c0 + 1);
}

void orc_brief(const uint8_t *img, int rows, int cols, const float *uv, int n, int length, int half, int sampler,
               const int16_t *pattern, uint32_t *out_bits, uint8_t *out_valid, float *out_m) {
    const int nw = (length + 31) / 32;
    for (int k = 0; k < n; ++k) {
        uint32_t *bits = out_bits + static_cast<size_t>(k) * nw;
        for (int j = 0; j < nw; ++j) bits[j] = 0;  // :10 descriptor.assign(kLength, 0)
        if (out_valid) out_valid[k] = 0;
        if (out_m) out_m[3 * k] = out_m[3 * k + 1] = out_m[3 * k + 2] = 0.0f;
        const float x = uv[2 * k], y = uv[2 * k + 1];
        constexpr float kPatternMaxBound = 19.0f;  // :13
        const float max_bound = std::max(kPatternMaxBound, static_cast<float>(half) * 2.0f);  // :14
        if (x < max_bound || x > cols - max_bound || y < max_bound || y > rows - max_bound) continue;  // :15-17
        if (x != x || y != y) continue;  // NaN: outside (the reference would read arbitrary memory)
        float m01 = 0.0f;  // :20-28
        float m10 = 0.0f;
        for (int32_t dx = -half; dx <= half; ++dx) {
            for (int32_t dy = -half; dy <= half; ++dy) {
                const float value = BriefSample(img, rows, cols, y + dy, x + dx, sampler);
                m10 += dx * value;
                m01 += dy * value;
            }
        }
        const float m = std::sqrt(m01 * m01 + m10 * m10);  // :29
        if (out_m) {
            out_m[3 * k] = m10;
            out_m[3 * k + 1] = m01;
            out_m[3 * k + 2] = m;
        }
        if (m < 1e-6f) continue;  // :30
        const float sin_theta = m01 / m;  // :32-35
        const float cos_theta = m10 / m;
        const float r00 = cos_theta, r01 = -sin_theta, r10 = sin_theta, r11 = cos_theta;
        for (int32_t i = 0; i < length; ++i) {  // :38-47
            const float ax = pattern[4 * i], ay = pattern[4 * i + 1], bx = pattern[4 * i + 2], by = pattern[4 * i + 3];
            const float p1x = r00 * ax + r01 * ay + x, p1y = r10 * ax + r11 * ay + y;
            const float p2x = r00 * bx + r01 * by + x, p2y = r10 * bx + r11 * by + y;
            const float value_1 = BriefSample(img, rows, cols, p1y, p1x, sampler);
            const float value_2 = BriefSample(img, rows, cols, p2y, p2x, sampler);
            if (value_1 < value_2) bits[i >> 5] |= 1u << (i & 31);
        }
        if (out_valid) out_valid[k] = 1;
    }
}

// -----------------------------------------------------------------------------------------------------
// SuperPoint post-processing, NNFeaturePointDetector (nn_feature_point_detector/nn_feature_point_detector.cpp).
// CreateMask (:59-73): ones, kInvalidBoundary outermost rows/cols zero (topRows/bottomRows/leftCols/
// rightCols), then a (2d+1)^2 box (clipped, :75-82) around each truncated prior feature (:84-90).
// SelectKeypointCandidatesFromHeatMap (:128-139): std::multimap<float, Pixel> of every value > thr.
// SelectGoodFeaturesFromCandidates (:141-155): crbegin -> crend; skip masked; append; stop at
// max_features (priors included); draw the box.
// Returns the number of new features written to out_xy (x, y).
// -----------------------------------------------------------------------------------------------------
int orc_nn_select(const float *heat, int rows, int cols, int border, int dist, int max_features, float thr,
                  const float *prior_xy, int n_prior, float *out_xy, int out_cap) {
    std::vector<int32_t> mask(static_cast<size_t>(rows) * cols, 1);
    auto draw = [&](int32_t row, int32_t col, int32_t radius) {  // DrawRectangleInMask (:75-82)
        const int32_t r0 = std::max(0, row - radius), r1 = std::min(rows - 1, row + radius);
        const int32_t c0 = std::max(0, col - radius), c1 = std::min(cols - 1, col + radius);
        for (int32_t r = r0; r <= r1; ++r)
            for (int32_t c = c0; c <= c1; ++c) mask[static_cast<size_t>(r) * cols + c] = 0;
    };
    if (border) {
        for (int r = 0; r < rows; ++r)
            for (int c = 0; c < cols; ++c)
                if (r < border || r >= rows - border || c < border || c >= cols - border)
                    mask[static_cast<size_t>(r) * cols + c] = 0;
    }
    for (int i = 0; i < n_prior; ++i) draw(static_cast<int32_t>(prior_xy[2 * i + 1]), static_cast<int32_t>(prior_xy[2 * i]), dist);
    std::multimap<float, std::pair<int32_t, int32_t>> candidates;  // response -> (col, row)
    for (int32_t row = 0; row < rows; ++row)
        for (int32_t col = 0; col < cols; ++col) {
            const float response = heat[static_cast<size_t>(row) * cols + col];
            if (response > thr) candidates.insert(std::make_pair(response, std::make_pair(col, row)));
        }
    size_t size = static_cast<size_t>(n_prior);
    int n = 0;
    for (auto it = candidates.crbegin(); it != candidates.crend(); ++it) {
        const int32_t col = it->second.first, row = it->second.second;
        if (!mask[static_cast<size_t>(row) * cols + col]) continue;
        if (n < out_cap) {
            out_xy[2 * n] = static_cast<float>(col);
            out_xy[2 * n + 1] = static_cast<float>(row);
        }
        ++n;
        ++size;
        if (size >= static_cast<size_t>(max_features)) break;
        draw(row, col, dist);
    }
    return n;
}

// ArgSort + DirectlySelectGoodFeaturesWithDescriptors (nn_feature_point_detector.cpp:204-230) for the
// keypoint-list models (nn_feature_point_detector_superpoint.cpp:106-109): keypoints kp[i] = (u, v)
// (int64, cast to int32 as :215), scores[i]. SlamOperation::ArgSort (un-vendored) is restated as an
// ascending argsort; its order of equal scores is unpinned: taken here as ascending raster index,
// then ascending list index, so the walk from the back (:213) visits equal scores by descending
// raster index (the heatmap path's multimap order), then descending list index. Mask as
// orc_nn_select (CreateMask, :59-73). Returns the number of new features; out_index receives the
// list index of each (the descriptor rows gathered at :224-227).
int orc_nn_select_list(const int64_t *kp, const float *scores, int64_t n, int rows, int cols, int border, int dist,
                       int max_features, const float *prior_xy, int n_prior, float *out_xy, int32_t *out_index,
                       int out_cap) {
    std::vector<int32_t> mask(static_cast<size_t>(rows) * cols, 1);
    auto draw = [&](int32_t row, int32_t col, int32_t radius) {  // DrawRectangleInMask (:75-82)
        const int32_t r0 = std::max(0, row - radius), r1 = std::min(rows - 1, row + radius);
        const int32_t c0 = std::max(0, col - radius), c1 = std::min(cols - 1, col + radius);
        for (int32_t r = r0; r <= r1; ++r)
            for (int32_t c = c0; c <= c1; ++c) mask[static_cast<size_t>(r) * cols + c] = 0;
    };
    for (int r = 0; r < rows; ++r)
        for (int c = 0; c < cols; ++c)
            if (r < border || r >= rows - border || c < border || c >= cols - border) mask[static_cast<size_t>(r) * cols + c] = 0;
    for (int i = 0; i < n_prior; ++i) draw(static_cast<int32_t>(prior_xy[2 * i + 1]), static_cast<int32_t>(prior_xy[2 * i]), dist);
    std::vector<int32_t> sorted(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) sorted[i] = static_cast<int32_t>(i);
    auto raster = [&](int32_t i) { return kp[2 * i + 1] * cols + kp[2 * i]; };
    std::sort(sorted.begin(), sorted.end(), [&](int32_t a, int32_t b) {
        if (scores[a] != scores[b]) return scores[a] < scores[b];
        if (raster(a) != raster(b)) return raster(a) < raster(b);
        return a < b;
    });
    size_t size = static_cast<size_t>(n_prior);
    int nout = 0;
    for (auto it = sorted.rbegin(); it != sorted.rend(); ++it) {
        const int32_t index = *it;
        const int32_t u = static_cast<int32_t>(kp[2 * index]), v = static_cast<int32_t>(kp[2 * index + 1]);
        if (!mask[static_cast<size_t>(v) * cols + u]) continue;  // :216
        if (nout < out_cap) {
            out_xy[2 * nout] = static_cast<float>(u);
            out_xy[2 * nout + 1] = static_cast<float>(v);
            out_index[nout] = index;
        }
        ++nout;
        ++size;
        if (size >= static_cast<size_t>(max_features)) break;  // :219
        draw(v, u, dist);
    }
    return nout;
}

// ExtractDescriptorsForSelectedFeatures (:163-193): map is [channels][map_rows][map_cols].
void orc_nn_descriptors(const float *map, int channels, int map_rows, int map_cols, const float *xy, int n, float *out) {
    for (int i = 0; i < n; ++i) {
        const float row = xy[2 * i + 1] / 8.0f;
        const float col = xy[2 * i] / 8.0f;
        const int32_t int_row = static_cast<int32_t>(row);
        const int32_t int_col = static_cast<int32_t>(col);
        const float sub_row = row - std::floor(row);
        const float sub_col = col - std::floor(col);
        const float inv_sub_row = 1.0f - sub_row;
        const float inv_sub_col = 1.0f - sub_col;
        const float weights[4] = {inv_sub_col * inv_sub_row, sub_col * inv_sub_row, inv_sub_col * sub_row, sub_col * sub_row};
        for (int j = 0; j < channels; ++j) {
            float &d = out[static_cast<size_t>(i) * channels + j];
            if (int_row < 0 || int_row >= map_rows - 1 || int_col < 0 || int_col >= map_cols - 1) {
                d = 0.0f;
                continue;
            }
            const float *p = map + (static_cast<size_t>(j) * map_rows + int_row) * map_cols + int_col;
            d = weights[0] * p[0] + weights[1] * p[1] + weights[2] * p[map_cols] + weights[3] * p[map_cols + 1];
        }
    }
}

}  // extern "C"

#include <random>
// Test-input generator shared by tests/bench (identical on host and GPU box): std::mt19937(seed) drawn
// raw, one draw per pixel in raster order. This is the generator behind BASELINE.md §2's candidate
// counts ("noise" and "checker" inputs); tests/test_oracle_pinning.py reproduces those counts exactly.
//   pattern 0: noise   v = rng() % 256
//   pattern 1: checker v = clamp((((r/P)+(c/P)) odd ? 180 : 60) + int(rng() % 21) - 10, 0, 255)
extern "C" void orc_make_frame(int pattern, uint32_t seed, int rows, int cols, int period, uint8_t *out) {
    std::mt19937 rng(seed);
    for (int r = 0; r < rows; ++r) {
        for (int c = 0; c < cols; ++c) {
            int v;
            if (pattern == 0) {
                v = static_cast<int>(rng() % 256u);
            } else {
                const bool odd = (((r / period) + (c / period)) & 1) != 0;
                v = (odd ? 180 : 60) + static_cast<int>(rng() % 21u) - 10;
            }
            out[static_cast<size_t>(r) * cols + c] = static_cast<uint8_t>(std::min(255, std::max(0, v)));
        }
    }
}
