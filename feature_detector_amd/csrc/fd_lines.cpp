// fd_lines.cpp -- batched host stage of the LSD line detector.
//
// Reference: FeatureLineDetector::DetectGoodFeatures / GrowRegion / TryToAddPixelIntoCandidates /
// ConvertRegionToRectangle (src/feature_line_detector/feature_line_detector.cpp:12-54, 99-228).
//
// Why on the host: a frame's regions are grown one after another from seeds in gradient-norm order,
// and every region depends on the pixels earlier regions consumed (is_used), so the work is a serial
// chain per frame with a glibc cosf / sinf / atan2f per accepted pixel (the reference's float
// sequence, which the line endpoints inherit). Frames are independent: the batch is spread over
// worker threads, each with its own scratch.
//
// Data layout (not the reference's 20-byte PixelParam matrix): the GPU hands over, per frame, the
// valid pixels in scan order as three arrays (map index, norm, angle). A frame is then
//   * a valid bitmask over the (rows-1) x (cols-1) map plus a map-index -> entry table (written only
//     at valid pixels, read only where the mask is set: never cleared),
//   * per entry: a state byte (used / occupied) and its row and column,
// and the seeds are (norm, entry) pairs in scan order, ordered by the reference's comparator with
// std::sort -- the same comparisons on the same sequence, hence the same permutation, ties included.
//
// Un-vendored Slam_Utility semantics (parity unpinned): CircularBuffer<T, 1000> on a
// full buffer drops its oldest element; Utility::AngleDiffInRad(a, b) is a - b wrapped into [-pi, pi].
#include "fd_lines.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <memory>
#include <thread>
#include <utility>
#include <vector>

namespace fdl {

namespace {

constexpr float kPi = 3.14159265358979323846f;  // kPai (slam_basic_math.h)
constexpr float k2Pi = 2.0f * kPi;               // k2Pai
constexpr uint8_t kUsed = 1, kOccupied = 2, kSeen = 4;  // (kSeen: order_seeds' permutation check only)
constexpr int kRing = 1000;  // CircularBuffer<PixelParam *, 1000> (feature_line_detector.h:76-77)
#ifdef FD_LINES_PHASES
}  // namespace
std::atomic<long long> g_phase_ns[3];  // load (incl. sort), sort, grow + fit
namespace {
#endif

float wrap_diff(float a, float b) {  // Utility::AngleDiffInRad (assumed: wrap a - b into [-pi, pi])
    float d = a - b;
    while (d > kPi) d -= k2Pi;
    while (d < -kPi) d += k2Pi;
    return d;
}

// Fixed-capacity FIFO of entry numbers; a push onto a full ring replaces the oldest entry.
struct Fifo {
    int32_t v[kRing];
    int head = 0, size = 0;
    void clear() { head = size = 0; }
    bool empty() const { return size == 0; }
    void push(int32_t e) {
        if (size == kRing) {
            v[head] = e;
            head = head + 1 == kRing ? 0 : head + 1;
            return;
        }
        int t = head + size;
        if (t >= kRing) t -= kRing;
        v[t] = e;
        ++size;
    }
    int32_t pop() {
        const int32_t e = v[head];
        head = head + 1 == kRing ? 0 : head + 1;
        --size;
        return e;
    }
};

class FrameLines {
public:
    FrameLines(int rows, int cols, const fd_lsd_opts &o)
        : pc_(cols - 1), words_((static_cast<int64_t>(rows - 1) * (cols - 1) + 63) / 64), o_(o),
          min_region_(min_region_size(rows, cols, o.min_tolerance_angle_residual_rad)),
          // read only where the frame's mask bit is set, i.e. after load() wrote it: left uninitialised
          // (a map-sized zero fill per worker per call cost more than the sparse frames touch)
          entry_of_(new int32_t[static_cast<size_t>(rows - 1) * (cols - 1)]) {
        mask_.assign(static_cast<size_t>(words_), 0ull);
    }

    // One frame: returns the number of rectangles (writes at most stride of them).
    // order: this frame's seed order from the GPU, or null (host sort); obtained through get_order after
    // the frame's setup.
    template <typename GetOrder>
    int32_t run(const FrameList &fl, fd_lsd_rect *out, int32_t stride, uint8_t *used_out, GetOrder get_order) {
#ifdef FD_LINES_PHASES  // diagnostic build only (tools/calib/lines_host_timing.cpp)
        const auto t0 = std::chrono::steady_clock::now();
#endif
        load(fl);
        order_seeds(get_order());
#ifdef FD_LINES_PHASES
        const auto t1 = std::chrono::steady_clock::now();
        g_phase_ns[0] += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
#endif
        int32_t nrect = 0;
        for (const auto &seed : seeds_) {  // :27-46
            const int32_t s = seed.second;
            if (state_[s] & kUsed) continue;
            grow(s);
            if (region_.size() < min_region_) {
                for (const int32_t e : region_) state_[e] &= static_cast<uint8_t>(~kUsed);
                continue;
            }
            fd_lsd_rect r;
            fit(r);
            if (r.length < o_.min_valid_line_length || r.inlier_ratio < o_.max_tolerance_inlier_ratio) continue;
            r.start[0] += 0.5f;  // :43-44
            r.start[1] += 0.5f;
            r.end[0] += 0.5f;
            r.end[1] += 0.5f;
            if (nrect < stride) out[nrect] = r;
            ++nrect;
        }
#ifdef FD_LINES_PHASES
        g_phase_ns[2] += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t1).count();
#endif
        if (used_out)
            for (int64_t k = 0; k < fl.n; ++k) used_out[k] = (state_[k] & kUsed) ? 1 : 0;
        for (int64_t k = 0; k < fl.n; ++k) mask_[static_cast<size_t>(fl.idx[k]) >> 6] = 0ull;  // clean for the next frame
        return nrect;
    }

private:
    void load(const FrameList &fl) {
        const size_t n = static_cast<size_t>(fl.n);
        state_.assign(n, 0);
        row_.resize(n);
        col_.resize(n);
        cos_.resize(n);
        sin_.resize(n);
        seeds_.resize(n);
        idx_ = fl.idx;
        norm_ = fl.norm;
        angle_ = fl.angle;
        for (size_t k = 0; k < n; ++k) {
            const int32_t i = fl.idx[k];
            mask_[static_cast<size_t>(i) >> 6] |= 1ull << (i & 63);
            entry_of_[static_cast<size_t>(i)] = static_cast<int32_t>(k);
            row_[k] = i / pc_;
            col_[k] = i - row_[k] * pc_;
            // glibc cosf / sinf of the angle: GrowRegion calls them whenever a pixel seeds or joins a
            // region, which happens many times per pixel (rejected regions release their pixels);
            // the same call on the same value, made once
            cos_[k] = std::cos(fl.angle[k]);
            sin_[k] = std::sin(fl.angle[k]);
        }
    }

    // sorted_pixels_: the scan-ordered list under the reference's comparator (:92-94). The GPU's order
    // (the same libstdc++ introsort permutation, emulated by k_select_reference) is taken when it is a
    // permutation of this frame's valid pixels in non-increasing norm; otherwise (a broken emulation,
    // a stale buffer), and without one, std::sort here.
    void order_seeds(const uint32_t *ord) {
#ifdef FD_LINES_PHASES
        const auto ts = std::chrono::steady_clock::now();
#endif
        const size_t n = seeds_.size();
        bool ok = ord != nullptr;
        for (size_t k = 0; ok && k < n; ++k) {
            const uint32_t i = ord[k];
            if (i >= static_cast<uint32_t>(words_ * 64) || !((mask_[i >> 6] >> (i & 63)) & 1ull)) {
                ok = false;
                break;
            }
            const int32_t e = entry_of_[i];
            if (state_[e] & kSeen) {
                ok = false;
                break;
            }
            if (k > 0 && norm_[e] > norm_[seeds_[k - 1].second]) {  // not sorted by the comparator
                ok = false;
                break;
            }
            state_[e] |= kSeen;
            seeds_[k].second = e;
        }
        for (uint8_t &v : state_) v = 0;  // (kSeen cleared; nothing else is set before the growing)
        if (!ok) {
            for (size_t k = 0; k < n; ++k) seeds_[k] = {norm_[k], static_cast<int32_t>(k)};
            std::sort(seeds_.begin(), seeds_.end(),
                      [](const std::pair<float, int32_t> &a, const std::pair<float, int32_t> &b) { return a.first > b.first; });
        }
#ifdef FD_LINES_PHASES
        g_phase_ns[1] += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - ts).count();
#endif
    }

    // TryToAddPixelIntoCandidates (:156-161) for the 8 neighbours of entry e, in the reference's order
    // (:112-119 / :139-146). Invalid neighbours are not listed; the valid ones are never on the map
    // border (valid rows/cols start at 1 and end 2 before the map edge), so no bounds checks.
    void offer_neighbours(int32_t e) {
        const int32_t r = row_[e], c = col_[e];
        static constexpr int dr[8] = {-1, -1, -1, 0, 0, 1, 1, 1};
        static constexpr int dc[8] = {-1, 0, 1, -1, 1, -1, 0, 1};
        for (int j = 0; j < 8; ++j) {
            const int64_t i = static_cast<int64_t>(r + dr[j]) * pc_ + (c + dc[j]);
            if (!((mask_[static_cast<size_t>(i) >> 6] >> (i & 63)) & 1ull)) continue;
            const int32_t k = entry_of_[static_cast<size_t>(i)];
            if (state_[k] & (kUsed | kOccupied)) continue;
            state_[k] |= kOccupied;
            cand_.push(k);
        }
    }

    // GrowRegion (:99-154): breadth-first from the seed; a candidate joins when its angle is within
    // the tolerance of the region's running mean direction, which it then updates.
    void grow(int32_t seed) {
        cand_.clear();
        seen_.clear();
        seen_.push(seed);
        state_[seed] |= kOccupied;
        region_.clear();
        float region_angle = angle_[seed];
        float sum_dx = cos_[seed];
        float sum_dy = sin_[seed];
        offer_neighbours(seed);
        while (!cand_.empty()) {
            const int32_t e = cand_.pop();
            seen_.push(e);
            if (std::fabs(wrap_diff(region_angle, angle_[e])) > o_.min_tolerance_angle_residual_rad) continue;
            sum_dx += cos_[e];
            sum_dy += sin_[e];
            region_angle = std::atan2(sum_dy, sum_dx);
            region_.push_back(e);
            state_[e] |= kUsed;
            offer_neighbours(e);
        }
        while (!seen_.empty()) state_[seen_.pop()] &= static_cast<uint8_t>(~kOccupied);
        region_angle_ = region_angle;
    }

    // ConvertRegionToRectangle (:163-228): norm-weighted centroid, principal direction from the
    // second moments, extent along / across it, inlier ratio.
    void fit(fd_lsd_rect &r) const {
        float cx = 0.0f, cy = 0.0f, wsum = 0.0f;
        r = fd_lsd_rect{{0.0f, 0.0f}, {0.0f, 0.0f}, {0.0f, 0.0f}, 0.0f, 0.0f, 0.0f, {1.0f, 0.0f}, 0.0f};
        for (const int32_t e : region_) {
            cx += static_cast<float>(col_[e]) * norm_[e];
            cy += static_cast<float>(row_[e]) * norm_[e];
            wsum += norm_[e];
        }
        r.center[0] = cx;
        r.center[1] = cy;
        if (wsum == 0) return;
        cx /= wsum;
        cy /= wsum;
        r.center[0] = cx;
        r.center[1] = cy;
        float ixx = 0.0f, iyy = 0.0f, ixy = 0.0f;
        for (const int32_t e : region_) {
            const float dx = col_[e] - cx;
            const float dy = row_[e] - cy;
            ixx += dy * dy * norm_[e];
            iyy += dx * dx * norm_[e];
            ixy -= dx * dy * norm_[e];
        }
        if (ixx == 0 || iyy == 0 || ixy == 0) return;
        const float lambda_min = 0.5f * (ixx + iyy - std::sqrt((ixx - iyy) * (ixx - iyy) + 4.0f * ixy * ixy));
        float ang = std::fabs(ixx) > std::fabs(iyy) ? std::atan2(lambda_min - ixx, ixy) : std::atan2(ixy, lambda_min - iyy);
        if (std::fabs(wrap_diff(ang, region_angle_)) > o_.min_tolerance_angle_residual_rad) {
            ang += kPi;
            if (ang >= kPi) ang -= k2Pi;
        }
        r.angle = ang;
        const float ux = std::cos(ang), uy = std::sin(ang);
        r.dir[0] = ux;
        r.dir[1] = uy;
        float lmin = 0.0f, lmax = 0.0f, wmin = 0.0f, wmax = 0.0f;  // Vec2::Zero() ranges
        for (const int32_t e : region_) {
            const float dx = col_[e] - cx;
            const float dy = row_[e] - cy;
            const float along = dx * ux + dy * uy;
            const float across = -dx * uy + dy * ux;
            lmin = std::min(lmin, along);
            lmax = std::max(lmax, along);
            wmin = std::min(wmin, across);
            wmax = std::max(wmax, across);
        }
        r.start[0] = cx + lmin * ux;
        r.start[1] = cy + lmin * uy;
        r.end[0] = cx + lmax * ux;
        r.end[1] = cy + lmax * uy;
        r.length = std::max(lmax - lmin, 1.0f);
        r.width = std::max(wmax - wmin, 1.0f);
        r.inlier_ratio = static_cast<float>(region_.size()) / ((lmax - lmin) * r.width);
    }

    const int32_t pc_;
    const int64_t words_;
    const fd_lsd_opts o_;
    const uint32_t min_region_;
    std::unique_ptr<int32_t[]> entry_of_;
    std::vector<uint64_t> mask_;
    std::vector<uint8_t> state_;
    std::vector<int32_t> row_, col_;
    std::vector<float> cos_, sin_;
    std::vector<std::pair<float, int32_t>> seeds_;
    std::vector<int32_t> region_;
    const int32_t *idx_ = nullptr;
    const float *norm_ = nullptr;
    const float *angle_ = nullptr;
    float region_angle_ = 0.0f;
    Fifo cand_, seen_;
};

}  // namespace

uint32_t min_region_size(int rows, int cols, float tol_rad) {
    const float p = tol_rad / kPi;
    const float log_nt = 5.0f * (std::log10(double(cols)) + std::log10(double(rows))) / 2.0f + std::log10(11.0f);
    return static_cast<uint32_t>(-log_nt / std::log10(p));
}

void detect_lines(int rows, int cols, const fd_lsd_opts &o, const FrameList *frames, int batch, fd_lsd_rect *out,
                  int32_t stride, int32_t *counts, uint8_t *used0, int threads, const SeedOrder *seeds) {
    threads = std::max(1, std::min(threads, batch));
    std::atomic<int> next{0};
    auto worker = [&]() {
        FrameLines fl(rows, cols, o);
        bool waited = false;
        for (int f = next.fetch_add(1); f < batch; f = next.fetch_add(1)) {
            auto get_order = [&]() -> const uint32_t * {
                if (!seeds) return nullptr;
                if (!waited) {
                    seeds->wait();
                    waited = true;
                }
                const uint32_t st = seeds->status[f];
                if (!(st & FD_FRAME_RESOLVED) || (st & (FD_FRAME_UNRESOLVED | FD_FRAME_GUARD))) return nullptr;
                return seeds->ord + static_cast<int64_t>(f) * seeds->stride;
            };
            counts[f] = fl.run(frames[f], out + static_cast<int64_t>(f) * stride, stride, f == 0 ? used0 : nullptr, get_order);
        }
    };
    if (threads == 1) {
        worker();
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve(static_cast<size_t>(threads));
    for (int t = 0; t < threads; ++t) pool.emplace_back(worker);
    for (auto &t : pool) t.join();
}

}  // namespace fdl
