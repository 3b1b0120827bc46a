// Host-stage phase timing of fd_lsd_lines (diagnostic, not part of the library): fd_lines.cpp built with
// -DFD_LINES_PHASES, fed with the level-line lists of synthetic 1920x1080 frames (64-px checker 60/180 +
// U[-10, 10] noise, the bench's configs[3] frames; the map formula of feature_line_detector.cpp:71-86
// computed here), one thread: per-frame time in load (glibc cosf / sinf per entry, seeds), std::sort of
// the seeds, region growing + rectangles. usage: lines_host_timing [frames]
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "fd_lines.h"

namespace fdl {
extern std::atomic<long long> g_phase_ns[3];
}

int main(int argc, char **argv) {
    const int frames = argc > 1 ? std::atoi(argv[1]) : 8, rows = 1080, cols = 1920;
    std::mt19937 rng(3);
    std::vector<std::vector<int32_t>> idx(frames);
    std::vector<std::vector<float>> nrm(frames), ang(frames);
    std::vector<uint8_t> img(static_cast<size_t>(rows) * cols);
    for (int f = 0; f < frames; ++f) {
        for (int r = 0; r < rows; ++r)
            for (int c = 0; c < cols; ++c) {
                const int b = ((r / 64 + c / 64) % 2) ? 180 : 60;
                const int v = b + static_cast<int>(rng() % 21) - 10;
                img[static_cast<size_t>(r) * cols + c] = static_cast<uint8_t>(v < 0 ? 0 : v > 255 ? 255 : v);
            }
        const int pc = cols - 1;
        for (int col = 1; col < cols - 2; ++col)
            for (int row = 1; row < rows - 2; ++row) {
                const int ad = int(img[(row + 1) * cols + col + 1]) - int(img[row * cols + col]);
                const int bc = int(img[row * cols + col + 1]) - int(img[(row + 1) * cols + col]);
                const float gx = static_cast<float>(ad + bc) / 2.0f, gy = static_cast<float>(ad - bc) / 2.0f;
                const float n = std::sqrt(gx * gx + gy * gy);
                if (n > 20.0f) {
                    idx[f].push_back(row * pc + col);
                    nrm[f].push_back(n);
                    ang[f].push_back(std::atan2(gx, -gy));
                }
            }
    }
    std::vector<fdl::FrameList> fl(frames);
    long long tot = 0;
    for (int f = 0; f < frames; ++f) {
        fl[f] = fdl::FrameList{idx[f].data(), nrm[f].data(), ang[f].data(), static_cast<int64_t>(idx[f].size())};
        tot += static_cast<long long>(idx[f].size());
    }
    fd_lsd_opts o{};
    o.min_valid_gradient_norm = 20.0f;
    o.min_tolerance_angle_residual_rad = 22.5f * 3.14159265358979323846f / 180.0f;
    o.min_valid_line_length = 20.0f;
    o.max_tolerance_inlier_ratio = 0.6f;
    std::vector<fd_lsd_rect> out(static_cast<size_t>(frames) * 4096);
    std::vector<int32_t> counts(frames);
    const auto t0 = std::chrono::steady_clock::now();
    fdl::detect_lines(rows, cols, o, fl.data(), frames, out.data(), 4096, counts.data(), nullptr, 1);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const double ld = fdl::g_phase_ns[0] / 1e6, so = fdl::g_phase_ns[1] / 1e6, gr = fdl::g_phase_ns[2] / 1e6;
    std::printf("%d frames, %.0f valid px/frame, %d rects/frame: %.2f ms/frame on 1 thread: load %.2f (of which std::sort %.2f, "
                "cosf/sinf + setup %.2f), grow + fit %.2f\n", frames, double(tot) / frames, counts[0], ms / frames,
                ld / frames, so / frames, (ld - so) / frames, gr / frames);
    return 0;
}
