// =====================================================================================================
// fd_oracle_lines.cpp -- CPU restatement of the LSD line detector, TEST INFRASTRUCTURE ONLY (same
// rules as fd_oracle.cpp: loaded by tests/ and bench.py's cpu_baseline legs, never by the product).
//
// Restates FeatureLineDetector::DetectGoodFeatures (src/feature_line_detector/feature_line_detector.cpp
// :12-54) end to end on one frame, in the reference's own data structures: a column-major matrix of
// per-pixel records (PixelParam, feature_line_detector.h:14-22) filled by the level-line scan (:56-89),
// a list of record pointers sorted by gradient norm with std::sort (:92-94), breadth-first region
// growing with two 1000-entry ring buffers (:99-161, h:76-77) and the rectangle fit (:163-228).
//
// Parity unpinned (un-vendored Slam_Utility): CircularBuffer's overflow policy
// (here: a push onto a full ring drops the oldest element), Utility::AngleDiffInRad (here: a - b
// wrapped into [-pi, pi]) and kPai (3.14159265358979323846f). The reference's recorded line counts
// (40 on examples/image.png, 112 and 792 on the 64-px checker frames, tests/golden) are reproduced.
// The scan is the same restatement as orc_lsd_map (fd_oracle.cpp), repeated here so that this file
// holds the whole per-frame pipeline in the reference's layout.
// =====================================================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

namespace {

constexpr float kPai = 3.14159265358979323846f;
constexpr float k2Pai = 2.0f * kPai;

struct Px {  // PixelParam (feature_line_detector.h:14-22)
    int32_t row = 0, col = 0;
    float line_level_angle = 0.0f, gradient_norm = 0.0f;
    bool is_valid = false, is_used = false, is_occupied = false;
};

template <int N>
struct Ring {  // CircularBuffer<PixelParam *, N>, overflow drops the oldest (assumed)
    Px *buf[N];
    int head = 0, size = 0;
    void Clear() { head = size = 0; }
    bool Empty() const { return size == 0; }
    void PushBack(Px *p) {
        if (size == N) {
            buf[head] = p;
            head = (head + 1) % N;
            return;
        }
        buf[(head + size) % N] = p;
        ++size;
    }
    Px *Front() const { return buf[head]; }
    void PopFront() {
        head = (head + 1) % N;
        --size;
    }
};

float AngleDiff(float a, float b) {
    float d = a - b;
    while (d > kPai) d -= k2Pai;
    while (d < -kPai) d += k2Pai;
    return d;
}

struct Rect {  // RectangleParam (feature_line_detector.h:29-38), Vec2 as two floats
    float sx = 0, sy = 0, ex = 0, ey = 0, cx = 0, cy = 0;
    float length = 0, width = 0, angle = 0;
    float dx = 1, dy = 0;  // Vec2::Identity()
    float inlier_ratio = 0;
};

struct Lsd {
    int pr = 0, pc = 0;  // map rows/cols
    std::vector<Px> map;  // column-major, like the reference's Eigen matrix
    std::vector<Px *> sorted;
    Ring<1000> candidates, visited;
    float tol = 0, min_norm = 0, min_len = 0, min_inlier = 0;

    Px &at(int r, int c) { return map[static_cast<size_t>(c) * pr + r]; }

    // ComputeLineLevelAngleMap (:56-97)
    void Scan(const uint8_t *img, int rows, int cols) {
        pr = rows - 1;
        pc = cols - 1;
        map.assign(static_cast<size_t>(pr) * pc, Px{});
        for (int i = 0; i < pr; ++i) {  // :59-63
            at(i, 0).row = i;
            at(i, pc - 1).row = i;
            at(i, pc - 1).col = pc - 1;
        }
        for (int i = 0; i < pc; ++i) {  // :64-68 (including its at(0, 1).col quirk; out of bounds,
            if (pc > 1) at(0, 1).col = i;  // i.e. undefined, in the reference when cols == 2: skipped)
            at(pr - 1, i).col = i;
            at(pr - 1, i).row = pr - 1;
        }
        sorted.clear();
        for (int col = 1; col < cols - 2; ++col) {
            for (int row = 1; row < rows - 2; ++row) {
                Px &p = at(row, col);
                p.row = row;
                p.col = col;
                const int32_t ad = int32_t(img[(row + 1) * cols + col + 1]) - int32_t(img[row * cols + col]);
                const int32_t bc = int32_t(img[row * cols + col + 1]) - int32_t(img[(row + 1) * cols + col]);
                const float gx = static_cast<float>(ad + bc) / 2.0f;
                const float gy = static_cast<float>(ad - bc) / 2.0f;
                p.gradient_norm = std::sqrt(gx * gx + gy * gy);
                p.is_valid = p.gradient_norm > min_norm;
                if (p.is_valid) {
                    p.line_level_angle = std::atan2(gx, -gy);
                    sorted.push_back(&p);
                }
            }
        }
        std::sort(sorted.begin(), sorted.end(), [](Px *a, Px *b) { return a->gradient_norm > b->gradient_norm; });
    }

    void Offer(Px &n) {  // TryToAddPixelIntoCandidates (:156-161)
        if (!n.is_occupied && !n.is_used && n.is_valid) {
            n.is_occupied = true;
            candidates.PushBack(&n);
        }
    }
    void OfferAround(const Px &p) {  // :112-119 / :139-146
        Offer(at(p.row - 1, p.col - 1));
        Offer(at(p.row - 1, p.col));
        Offer(at(p.row - 1, p.col + 1));
        Offer(at(p.row, p.col - 1));
        Offer(at(p.row, p.col + 1));
        Offer(at(p.row + 1, p.col - 1));
        Offer(at(p.row + 1, p.col));
        Offer(at(p.row + 1, p.col + 1));
    }

    // GrowRegion (:99-154)
    float Grow(Px &seed, std::vector<Px *> &region) {
        candidates.Clear();
        visited.Clear();
        visited.PushBack(&seed);
        seed.is_occupied = true;
        region.clear();
        float angle = seed.line_level_angle;
        float sdx = std::cos(seed.line_level_angle);
        float sdy = std::sin(seed.line_level_angle);
        OfferAround(seed);
        while (!candidates.Empty()) {
            Px *p = candidates.Front();
            candidates.PopFront();
            visited.PushBack(p);
            if (std::fabs(AngleDiff(angle, p->line_level_angle)) > tol) continue;
            sdx += std::cos(p->line_level_angle);
            sdy += std::sin(p->line_level_angle);
            angle = std::atan2(sdy, sdx);
            region.push_back(p);
            p->is_used = true;
            OfferAround(*p);
        }
        while (!visited.Empty()) {
            visited.Front()->is_occupied = false;
            visited.PopFront();
        }
        return angle;
    }

    // ConvertRegionToRectangle (:163-228)
    Rect Fit(const std::vector<Px *> &region, float region_angle) const {
        Rect r;
        float sw = 0.0f;
        for (const Px *p : region) {
            r.cx += static_cast<float>(p->col) * p->gradient_norm;
            r.cy += static_cast<float>(p->row) * p->gradient_norm;
            sw += p->gradient_norm;
        }
        if (sw == 0) return r;
        r.cx /= sw;
        r.cy /= sw;
        float ixx = 0.0f, iyy = 0.0f, ixy = 0.0f;
        for (const Px *p : region) {
            const float dx = p->col - r.cx, dy = p->row - r.cy;
            ixx += dy * dy * p->gradient_norm;
            iyy += dx * dx * p->gradient_norm;
            ixy -= dx * dy * p->gradient_norm;
        }
        if (ixx == 0 || iyy == 0 || ixy == 0) return r;
        const float ev = 0.5f * (ixx + iyy - std::sqrt((ixx - iyy) * (ixx - iyy) + 4.0f * ixy * ixy));
        r.angle = std::fabs(ixx) > std::fabs(iyy) ? std::atan2(ev - ixx, ixy) : std::atan2(ixy, ev - iyy);
        if (std::fabs(AngleDiff(r.angle, region_angle)) > tol) {
            r.angle += kPai;
            if (r.angle >= kPai) r.angle -= k2Pai;
        }
        r.dx = std::cos(r.angle);
        r.dy = std::sin(r.angle);
        float l0 = 0.0f, l1 = 0.0f, w0 = 0.0f, w1 = 0.0f;
        for (const Px *p : region) {
            const float dx = p->col - r.cx, dy = p->row - r.cy;
            const float len = dx * r.dx + dy * r.dy;
            const float wid = -dx * r.dy + dy * r.dx;
            l0 = std::min(l0, len);
            l1 = std::max(l1, len);
            w0 = std::min(w0, wid);
            w1 = std::max(w1, wid);
        }
        r.sx = r.cx + l0 * r.dx;
        r.sy = r.cy + l0 * r.dy;
        r.ex = r.cx + l1 * r.dx;
        r.ey = r.cy + l1 * r.dy;
        r.length = std::max(l1 - l0, 1.0f);
        r.width = std::max(w1 - w0, 1.0f);
        r.inlier_ratio = static_cast<float>(region.size()) / ((l1 - l0) * r.width);
        return r;
    }
};

}  // namespace

extern "C" {

// DetectGoodFeatures (:12-54) on one frame. opts: kMinValidGradientNorm, kMinToleranceAngleResidualInRad,
// kMinValidLineLengthInPixel, kMaxToleranceInlierRation. out: up to cap rectangles as 12 floats each
// (start x, y, end x, y, center x, y, length, width, angle, dir x, y, inlier ratio), start/end offset
// by 0.5 (:43-44). Returns the number of segments; -1 for the reference's `false` (:14).
int64_t orc_lsd_lines(const uint8_t *img, int rows, int cols, const float *opts, uint32_t needed, float *out,
                      int64_t cap) {
    if (img == nullptr || rows < 2 || cols < 2) return -1;  // :14
    if (needed == 0) return 0;                              // :15
    Lsd L;
    L.min_norm = opts[0];
    L.tol = opts[1];
    L.min_len = opts[2];
    L.min_inlier = opts[3];
    const float p = L.tol / kPai;  // :18-20
    const float log_nt = 5.0f * (std::log10(double(cols)) + std::log10(double(rows))) / 2.0f + std::log10(11.0f);
    const uint32_t min_region_size = static_cast<uint32_t>(-log_nt / std::log10(p));
    L.Scan(img, rows, cols);
    std::vector<Px *> region;
    int64_t n = 0;
    for (Px *s : L.sorted) {  // :27-46
        if (!s->is_valid || s->is_used) continue;
        const float ang = L.Grow(*s, region);
        if (region.size() < min_region_size) {
            for (Px *q : region) q->is_used = false;
            continue;
        }
        Rect r = L.Fit(region, ang);
        if (r.length < L.min_len || r.inlier_ratio < L.min_inlier) continue;
        r.sx += 0.5f;
        r.sy += 0.5f;
        r.ex += 0.5f;
        r.ey += 0.5f;
        if (n < cap) {
            const float v[12] = {r.sx, r.sy, r.ex, r.ey, r.cx, r.cy, r.length, r.width, r.angle, r.dx, r.dy, r.inlier_ratio};
            std::copy(v, v + 12, out + 12 * n);
        }
        ++n;
    }
    return n;
}

}  // extern "C"
