// Walk-shape probe (gfx950): the LSD map's bytes (k_lsd_map, dense 1920x1080 x256, rows padded to 1920
// entries) moved by waves that each walk H map rows of one 256-column strip -- the map kernel's access
// pattern with no arithmetic -- against the same bytes moved flat (H = 1: consecutive waves write
// consecutive 1 KiB pieces). Per 4 pixels: one dword read, a 16-B norm, a 16-B angle and a 4-B valid store.
// usage: lsd_walk   (one line per (H, store policy, order): ms and GB/s of algorithmic bytes, best of 5)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

constexpr int kN = 256, kR = 1080, kC = 1920, kMR = kR - 1, kP = 1920, kStrips = 8;

// ORDER 0: strip fastest, then chunk, then frame (k_lsd_map's order); ORDER 1: chunk fastest, then strip
template <int AUX, int ORDER>
__global__ __launch_bounds__(256) void k_walk(const uint8_t *fr, float *norm, float *angle, uint8_t *valid, int H,
                                              int chunks) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x) * 4 + (threadIdx.x >> 6));
    int strip, chunk, f;
    if constexpr (ORDER == 0) {
        strip = w % kStrips;
        chunk = (w / kStrips) % chunks;
        f = w / (kStrips * chunks);
    } else {
        chunk = w % chunks;
        strip = (w / chunks) % kStrips;
        f = w / (kStrips * chunks);
    }
    if (f >= kN) return;
    const int c0 = strip * 256 + 4 * lane;
    if (c0 >= kC) return;
    const int r0 = chunk * H, r1 = r0 + H < kMR ? r0 + H : kMR;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(fr) + static_cast<int64_t>(f) * kR * kC, 0,
                                                      kR * kC, 0x00020000);
    const int64_t mb = static_cast<int64_t>(f) * kMR * kP;
    const auto rn = __builtin_amdgcn_make_buffer_rsrc(norm + mb, 0, kMR * kP * 4, 0x00020000);
    const auto ra = __builtin_amdgcn_make_buffer_rsrc(angle + mb, 0, kMR * kP * 4, 0x00020000);
    const auto rv = __builtin_amdgcn_make_buffer_rsrc(valid + mb, 0, kMR * kP, 0x00020000);
    for (int r = r0; r < r1; ++r) {
        const uint32_t p = __builtin_amdgcn_raw_buffer_load_b32(rs, (r + 1) * kC + c0, 0, 0);
        const u4 a = {p & 0xFFu, (p >> 8) & 0xFFu, (p >> 16) & 0xFFu, p >> 24};
        const int o = r * kP + c0;
        __builtin_amdgcn_raw_buffer_store_b128(a, rn, 4 * o, 0, AUX);
        __builtin_amdgcn_raw_buffer_store_b128(a ^ 0x3F800000u, ra, 4 * o, 0, AUX);
        __builtin_amdgcn_raw_buffer_store_b32(p & 0x01010101u, rv, o, 0, AUX);
    }
}

template <int AUX, int ORDER>
static void run(const uint8_t *fr, float *n, float *a, uint8_t *v, int H, hipEvent_t e0, hipEvent_t e1) {
    const int chunks = (kMR + H - 1) / H;
    const int64_t waves = static_cast<int64_t>(kN) * kStrips * chunks;
    const unsigned grid = static_cast<unsigned>((waves + 3) / 4);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_walk<AUX, ORDER>), dim3(grid), dim3(256), 0, 0, fr, n, a, v, H, chunks);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double bytes = 10.0 * kN * kMR * (kC - 1);  // 1 B read + 9 B written per map entry
    printf("H=%3d aux=%d order=%d  %.3f ms  %.0f GB/s\n", H, AUX, ORDER, best, bytes / best / 1e6);
}

int main() {
    uint8_t *fr, *v;
    float *n, *a;
    const size_t fb = static_cast<size_t>(kN) * kR * kC, mb = static_cast<size_t>(kN) * kMR * kP;
    if (hipMalloc(&fr, fb) || hipMalloc(&n, 4 * mb) || hipMalloc(&a, 4 * mb) || hipMalloc(&v, mb)) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(fr, 0x5A, fb);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int hs[] = {1, 2, 4, 8, 16, 32, 67};
    for (int H : hs) {
        run<2, 0>(fr, n, a, v, H, e0, e1);
        run<0, 0>(fr, n, a, v, H, e0, e1);
    }
    for (int H : {16, 67}) {
        run<2, 1>(fr, n, a, v, H, e0, e1);
        run<0, 1>(fr, n, a, v, H, e0, e1);
    }
    printf("err %d\n", static_cast<int>(hipDeviceSynchronize()));
    return 0;
}
