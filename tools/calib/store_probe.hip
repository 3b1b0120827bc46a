// Store-shape probe (gfx950): what a wave-row of map stores costs by width and alignment, the shapes of
// the LSD map's outputs (k_lsd_map: f32 norm/angle rows of (C-1) entries as dwordx4 per lane, u8 valid
// rows as one dword per lane; a (C-1)-entry row pitch leaves 3 of 4 rows misaligned). Each wave writes
// `rows` rows of 64 lanes x W bytes at a row pitch; timed with hipEvents, the best of 5 launches.
// usage: store_probe   (one line per shape: GB/s of stored bytes)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void k_store(uint8_t *p, uint32_t bytes, uint32_t pitch, int rows) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, static_cast<int>(bytes), 0x00020000);
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t strip = wave % 7, band = wave / 7;  // 7 strips of 256 columns per row, bands of rows
    const uint32_t v = wave * 2654435761u + lane;
    for (int r = 0; r < rows; ++r) {
        const uint32_t row = band * rows + r;
        if constexpr (MODE == 0 || MODE == 1) {  // f32 x4 per lane (1 KiB per wave-row)
            const uint32_t off = row * pitch + (strip * 256 + 4 * lane) * 4;
            __builtin_amdgcn_raw_buffer_store_b128(u4{v, v + 1, v + 2, v + r}, rs, static_cast<int>(off), 0, 0);
        } else if constexpr (MODE == 2 || MODE == 3) {  // u8 x4 per lane as one dword (256 B per wave-row)
            const uint32_t off = row * pitch + strip * 256 + 4 * lane;
            __builtin_amdgcn_raw_buffer_store_b32(v + r, rs, static_cast<int>(off), 0, 0);
        } else if constexpr (MODE == 4) {  // the same bytes as four byte stores
            const uint32_t off = row * pitch + strip * 256 + 4 * lane;
#pragma unroll
            for (int k = 0; k < 4; ++k) __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(v >> (8 * k)), rs, static_cast<int>(off + k), 0, 0);
        } else if constexpr (MODE == 6) {  // MODE 1's rows re-aligned: 16-B chunks shifted by the row's offset t
            // (lanes 1..63 aligned dwordx4; lane 0's head and the strip's tail as 1-2-lane partial stores)
            const uint32_t e0 = row * (pitch / 4) + strip * 256;  // first entry of the strip in this row
            const uint32_t t = e0 & 3u;                           // entries past a 16-B boundary
            const uint32_t o = 4u * (e0 + 4 * lane);              // this lane's own 4 entries
            if (t == 0) {
                __builtin_amdgcn_raw_buffer_store_b128(u4{v, v + 1, v + 2, v + r}, rs, static_cast<int>(o), 0, 0);
            } else {
                if (lane > 0) __builtin_amdgcn_raw_buffer_store_b128(u4{v, v + 1, v + 2, v + r}, rs, static_cast<int>(o - 4 * t), 0, 0);
                if (t == 2) {
                    if (lane == 0 || lane == 63) {
                        typedef uint32_t u2 __attribute__((ext_vector_type(2)));
                        __builtin_amdgcn_raw_buffer_store_b64(u2{v, v + 1}, rs, static_cast<int>(lane == 0 ? o : o + 8), 0, 0);
                    }
                } else {
                    if (lane == 0 || lane == 63)
                        __builtin_amdgcn_raw_buffer_store_b32(v, rs, static_cast<int>(lane == 0 ? o : o + 12), 0, 0);
                    if (lane == (t == 1 ? 0 : 63)) {
                        typedef uint32_t u2 __attribute__((ext_vector_type(2)));
                        __builtin_amdgcn_raw_buffer_store_b64(u2{v, v + 1}, rs, static_cast<int>(o + 4), 0, 0);
                    }
                }
            }
        } else if constexpr (MODE == 5) {  // as two aligned shorts when the row start is 2-aligned
            const uint32_t off = row * pitch + strip * 256 + 4 * lane;
            __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(v), rs, static_cast<int>(off), 0, 0);
            __builtin_amdgcn_raw_buffer_store_b16(static_cast<uint16_t>(v >> 16), rs, static_cast<int>(off + 2), 0, 0);
        }
    }
}

template <int MODE>
static float run(uint8_t *p, uint32_t bytes, uint32_t pitch, int rows, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int i = 0; i < 5; ++i) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k_store<MODE>, dim3(blocks), dim3(256), 0, 0, p, bytes, pitch, rows);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    hipEventDestroy(a);
    hipEventDestroy(b);
    return best;
}

int main() {
    const int blocks = 4096, rows = 64;  // 16384 waves: 7 strips x 2340 bands of 64 rows
    const uint32_t bands = (blocks * 4 + 6) / 7;
    const uint32_t bytes = 0xF0000000u;
    uint8_t *p;
    if (hipMalloc(&p, bytes) != hipSuccess) return 1;
    hipMemset(p, 0, bytes);
    struct S { const char *name; int mode; uint32_t pitch; int wbytes; };
    const S shapes[] = {{"f32x4 rows, pitch 7680 (16-B aligned)", 0, 7680, 16},
                        {"f32x4 rows, pitch 7676 (4-B aligned: (C-1) f32 rows)", 1, 7676, 16},
                        {"u8x4 dword, pitch 1920 (aligned)", 2, 1920, 4},
                        {"u8x4 dword, pitch 1919 (byte-misaligned: (C-1) u8 rows)", 3, 1919, 4},
                        {"u8 x 4 byte stores, pitch 1919", 4, 1919, 4},
                        {"u16 x 2 stores, pitch 1918 (2-B aligned)", 5, 1918, 4},
                        {"f32x4 rows, pitch 7676, re-aligned chunks + edge stores", 6, 7676, 16}};
    for (const S &s : shapes) {
        if (static_cast<uint64_t>(bands) * rows * s.pitch > bytes) return 2;
        float ms = 0;
        switch (s.mode) {
            case 0: ms = run<0>(p, bytes, s.pitch, rows, blocks); break;
            case 1: ms = run<1>(p, bytes, s.pitch, rows, blocks); break;
            case 2: ms = run<2>(p, bytes, s.pitch, rows, blocks); break;
            case 3: ms = run<3>(p, bytes, s.pitch, rows, blocks); break;
            case 4: ms = run<4>(p, bytes, s.pitch, rows, blocks); break;
            case 5: ms = run<5>(p, bytes, s.pitch, rows, blocks); break;
            case 6: ms = run<6>(p, bytes, s.pitch, rows, blocks); break;
        }
        const double stored = double(blocks) * 4 * rows * 64 * s.wbytes;
        std::printf("%-58s %8.3f ms  %7.1f GB/s stored\n", s.name, ms, stored / (ms * 1e6));
    }
    hipFree(p);
    return 0;
}
