// =====================================================================================================
// fd_oracle_refflow.cpp -- CPU restatement of FeaturePointDetector::DetectGoodFeatures in the
// reference's DATA FLOW. TEST INFRASTRUCTURE ONLY (same rules as fd_oracle.cpp: loaded by tests/ and
// bench.py's cpu_baseline legs, never by the product path).
//
// fd_oracle.cpp computes the structure tensor as direct 3x3 integer sums (the clearest statement of
// the arithmetic). This file instead follows the reference's memory traffic and loop structure, so
// that the timed CPU baseline costs what the reference costs per frame:
//   * Harris / Shi-Tomasi: horizontal pass into a float R x 3C interleaved `tmp_` with 3-tap sliding
//     row sums (feature_point_harris_detector.cpp:17-64), vertical sliding sums over three float
//     vectors with the response computed in place into a zero-filled float `responses_` map
//     (:66-118), then the 4-neighbour NMS scan appending (response, Pixel) pairs (:120-137);
//   * FAST: per-pixel ComputeResponseOfPixel with its heap-allocated 16-entry compare vector
//     (feature_point_fast_detector.cpp:11-81) and the running offset (:83-98);
//   * selection: an int32 mask matrix set to all ones per call (feature_point_detector.cpp:13), the
//     unstable std::sort of the candidate pairs (:58-60), the greedy scan with (2d+1)^2 box writes
//     (:62-88).
// Every float sum here is an integer below 2^24, so the result equals fd_oracle.cpp's bit for bit
// (tests/test_oracle_refflow.py checks it).
// =====================================================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <utility>
#include <vector>

namespace {

struct RefPixel {  // Pixel(col, row): basic_type.h's Eigen int vector, x = col, y = row
    int32_t x, y;
};

// One detector instance's reusable state (the reference keeps these as members across calls).
struct RefState {
    std::vector<float> tmp;        // tmp_ rows x 3*cols (feature_point_harris_detector.h)
    std::vector<float> responses;  // responses_ rows x cols
    std::vector<int32_t> mask;     // mask_ (feature_point_detector.h:52)
    std::vector<std::pair<float, RefPixel>> candidates;  // candidates_ (feature_point_detector.h:51)
};

// feature_point_harris_detector.cpp:17-64 (byte-identical in the Shi-Tomasi detector).
void HorizontalGradientSums(RefState &s, const uint8_t *data, int rows, int cols) {
    const int half = 1, patch = 3;
    s.tmp.resize(static_cast<size_t>(rows) * 3 * cols);
    std::vector<float> ixx(cols, 0.0f), iyy(cols, 0.0f), ixy(cols, 0.0f);
    for (int r = 1; r < rows - 1; ++r) {
        const uint8_t *row = data + static_cast<size_t>(r) * cols;
        const uint8_t *prev = row - cols, *next = row + cols;
        for (int c = 1; c < cols - 1; ++c) {
            const float gx = static_cast<float>(row[c + 1]) - static_cast<float>(row[c - 1]);
            const float gy = static_cast<float>(next[c]) - static_cast<float>(prev[c]);
            ixx[c] = gx * gx;
            iyy[c] = gy * gy;
            ixy[c] = gx * gy;
        }
        float *t = s.tmp.data() + static_cast<size_t>(r) * 3 * cols;
        float a = 0, b = 0, d = 0;
        for (int c = 0; c < patch; ++c) {
            a += ixx[c];
            b += iyy[c];
            d += ixy[c];
        }
        t[half * 3] = a;
        t[half * 3 + 1] = b;
        t[half * 3 + 2] = d;
        for (int c = half + 1; c < cols - half; ++c) {
            a += ixx[c + half] - ixx[c - half - 1];
            b += iyy[c + half] - iyy[c - half - 1];
            d += ixy[c + half] - ixy[c - half - 1];
            t[c * 3] = a;
            t[c * 3 + 1] = b;
            t[c * 3 + 2] = d;
        }
    }
}

// feature_point_harris_detector.cpp:66-118 (kind 0) / feature_point_shi_tomas_detector.cpp:66-118 (kind 1).
void ResponseMap(RefState &s, int rows, int cols, int kind, float thr) {
    const int half = 1, patch = 3;
    const float inv_cnt = 1.0f / static_cast<float>(patch * patch);
    const float inv_cnt2 = inv_cnt * inv_cnt;
    s.responses.assign(static_cast<size_t>(rows) * cols, 0.0f);
    std::vector<float> sxx(cols, 0.0f), syy(cols, 0.0f), sxy(cols, 0.0f);
    for (int r = 1; r < 1 + patch && r < rows; ++r) {
        const float *t = s.tmp.data() + static_cast<size_t>(r) * 3 * cols;
        for (int c = half; c < cols - half; ++c) {
            sxx[c] += t[c * 3];
            syy[c] += t[c * 3 + 1];
            sxy[c] += t[c * 3 + 2];
        }
    }
    const int bound = half + 1;
    for (int r = bound; r < rows - bound; ++r) {
        float *out = s.responses.data() + static_cast<size_t>(r) * cols;
        const int32_t *m = s.mask.data() + static_cast<size_t>(r) * cols;
        for (int c = bound; c < cols - bound; ++c) {
            if (!m[c]) continue;
            if (kind == 0) {
                const float fxx = sxx[c], fyy = syy[c];
                const float trace = fxx + fyy;
                if (trace * trace * 0.21f * inv_cnt2 > thr) {
                    const float fxy = sxy[c];
                    const float res = (fxx * fyy - fxy * fxy - 0.04f * trace * trace) * inv_cnt2;
                    if (res > thr) out[c] = res;
                }
            } else {
                const float a = sxx[c] * inv_cnt, cc = syy[c] * inv_cnt;
                if (a + cc > thr) {
                    const float b = sxy[c] * inv_cnt;
                    const float res = (a + cc + std::sqrt((a - cc) * (a - cc) + 4.0f * b * b)) * 0.5f;
                    if (res > thr) out[c] = res;
                }
            }
        }
        if (r + half + 1 < rows - 1) {
            const float *tn = s.tmp.data() + static_cast<size_t>(r + half + 1) * 3 * cols;
            const float *tp = s.tmp.data() + static_cast<size_t>(r - half) * 3 * cols;
            for (int c = half; c < cols - half; ++c) {
                sxx[c] += tn[c * 3] - tp[c * 3];
                syy[c] += tn[c * 3 + 1] - tp[c * 3 + 1];
                sxy[c] += tn[c * 3 + 2] - tp[c * 3 + 2];
            }
        }
    }
}

// feature_point_harris_detector.cpp:120-137.
void NmsExtract(RefState &s, int rows, int cols, float thr) {
    const int bound = 2;
    for (int r = bound; r < rows - bound; ++r) {
        const float *row = s.responses.data() + static_cast<size_t>(r) * cols;
        for (int c = bound; c < cols - bound; ++c) {
            const float v = row[c];
            if (v <= thr) continue;
            if (v > row[c - 1] && v > row[c + 1] && v > row[c - cols] && v > row[c + cols])
                s.candidates.emplace_back(v, RefPixel{c, r});
        }
    }
}

const int32_t kRing[16][2] = {{0, -3}, {1, -3}, {2, -2}, {3, -1}, {3, 0},  {3, 1},   {2, 2},   {1, 3},
                              {0, 3},  {-1, 3}, {-2, 2}, {-3, 1}, {-3, 0}, {-3, -1}, {-2, -2}, {-1, -3}};

// feature_point_fast_detector.cpp:11-81 (kN 12, diff 15), including the per-call compare vector.
float FastResponse(const uint8_t *img, int cols, int row, int col) {
    const int32_t p = img[static_cast<size_t>(row) * cols + col];
    const int32_t hi = p + 15, lo = p - 15;
    auto at = [&](int k) { return int32_t(img[static_cast<size_t>(row + kRing[k][1]) * cols + col + kRing[k][0]]); };
    int32_t nb = 0, nd = 0;
    const int32_t idx[4] = {0, 4, 8, 12};
    for (int i = 0; i < 4; ++i) {
        const int32_t v = at(idx[i]);
        if (v > hi) { ++nb; nd = 0; }
        else if (v < lo) { ++nd; nb = 0; }
        else { nb = 0; nd = 0; }
    }
    if (nd < 3 && nb < 3) return 0;
    std::vector<int32_t> cmp(16, 0);
    for (int i = 0; i < 16; ++i) {
        const int32_t v = at(i);
        if (v > hi) cmp[i] = 1;
        else if (v < lo) cmp[i] = -1;
    }
    nd = nb = 0;
    int32_t best = 0;
    for (int k = 0; k < 2 && best < 16; ++k) {
        for (size_t i = 0; i < cmp.size(); ++i) {
            if (cmp[i] == 1) { ++nb; nd = 0; }
            else if (cmp[i] == -1) { ++nd; nb = 0; }
            else { nb = 0; nd = 0; }
            if (nb > best) best = nb;
            if (nd > best) best = nd;
        }
    }
    return static_cast<float>(best);
}

void FastCandidates(RefState &s, const uint8_t *img, int rows, int cols, float thr) {
    float offset = 1e-5f;
    for (int r = 3; r < rows - 3; ++r)
        for (int c = 3; c < cols - 3; ++c)
            if (s.mask[static_cast<size_t>(r) * cols + c]) {
                const float response = FastResponse(img, cols, r, c) + offset;
                if (response > thr) s.candidates.emplace_back(response, RefPixel{c, r});
                offset += 1e-5f;
            }
}

void DrawRect(RefState &s, int rows, int cols, int dist, int32_t row, int32_t col) {  // :76-88
    for (int32_t dr = -dist; dr <= dist; ++dr)
        for (int32_t dc = -dist; dc <= dist; ++dc) {
            const int32_t rr = dr + row, cc = dc + col;
            if (rr < 0 || cc < 0 || rr > rows - 1 || cc > cols - 1) continue;
            s.mask[static_cast<size_t>(rr) * cols + cc] = 0;
        }
}

}  // namespace

extern "C" {

void *orc_ref_state_new(void) { return new RefState(); }
void orc_ref_state_free(void *p) { delete static_cast<RefState *>(p); }

// DetectGoodFeatures (feature_point_detector.cpp:7-25) with an empty incoming feature list, in the
// reference's data flow. Writes up to out_cap new features (x, y) and returns their count.
int orc_detect_refflow(void *state, int kind, const uint8_t *img, int rows, int cols, int dist, float thr,
                       uint32_t need, float *out_xy, int out_cap) {
    RefState &s = *static_cast<RefState *>(state);
    s.mask.assign(static_cast<size_t>(rows) * cols, 1);  // :13
    s.candidates.clear();                                // :19
    if (kind == 2) {
        FastCandidates(s, img, rows, cols, thr);
    } else {
        HorizontalGradientSums(s, img, rows, cols);
        ResponseMap(s, rows, cols, kind, thr);
        NmsExtract(s, rows, cols, thr);
    }
    if (s.candidates.empty()) return 0;  // :55
    std::sort(s.candidates.begin(), s.candidates.end(),
              [](const std::pair<float, RefPixel> &a, const std::pair<float, RefPixel> &b) { return a.first > b.first; });
    int n = 0;
    for (const auto &cand : s.candidates) {  // :62-71
        const int32_t row = cand.second.y, col = cand.second.x;
        if (s.mask[static_cast<size_t>(row) * cols + col]) {
            if (n < out_cap) {
                out_xy[2 * n] = static_cast<float>(col);
                out_xy[2 * n + 1] = static_cast<float>(row);
            }
            ++n;
            if (static_cast<uint32_t>(n) >= need) break;
            DrawRect(s, rows, cols, dist, row, col);
        }
    }
    return n;
}

}  // extern "C"
