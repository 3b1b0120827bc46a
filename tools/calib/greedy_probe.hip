// Greedy-scan probe (diagnostic, not part of the library): the selection kernels' wave-serial greedy
// (fd_greedy.h greedy_chunk<1>, LDS occupancy grid) alone on a synthetic sorted chunk -- c candidates at
// random positions of a 640x480 frame, distance 20, need 500 -- timed with s_memtime around the call,
// in a 64-thread and a 1024-thread workgroup (wave 0 scans, the other waves wait at the barrier, as in
// k_select). Prints core clocks per call and per 64-candidate batch. No arguments.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>

#include "fd_greedy.h"

using namespace fdk;


// Lean scan (candidate for fd_greedy.h): pk15 frames only; the chunk padded to whole batches (kEmpty /
// cell gw2 + 1 / zero masks), so the next batch's loads need no masking; no tie check, no stamps;
// DEFER: the accepted lanes of each batch go to accm[b] (written out afterwards by the whole
// workgroup) instead of a global store per batch.
template <bool DEFER, int FP>
__device__ __forceinline__ void greedy_lean(const SelectArgs &a, int f, int cnt, const uint32_t *pxy,
                                            const uint32_t *pcell, const uint64_t *cmask, uint32_t *grid, int gw2,
                                            uint32_t prior, int &s_acc, int &s_done, uint64_t *accm) {
    const int lane = lane_id();
    const int d = a.dist;
    const uint32_t w2 = 2u * static_cast<uint32_t>(d);
    const u16x2 dd = {static_cast<uint16_t>(d), static_cast<uint16_t>(d)};
    int acc = s_acc;
    const int nb = (cnt + kWave - 1) / kWave;
    uint32_t e_n = pxy[lane], cell_n = pcell[lane];
    uint64_t C_n = cmask[lane];
    bool done = false;
    for (int b = 0; b < nb && !done; ++b) {
        const uint32_t e = e_n, cell = cell_n;
        uint64_t C = C_n;
        uint32_t g[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) g[q] = grid[cell + (q / 3 - 1) * gw2 + (q % 3 - 1)];
        if (b + 1 < nb) {
            e_n = pxy[(b + 1) * kWave + lane];
            cell_n = pcell[(b + 1) * kWave + lane];
            C_n = cmask[(b + 1) * kWave + lane];
        }
        const u16x2 base = __builtin_bit_cast(u16x2, e) - dd;
        uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            const u16x2 dt = __builtin_bit_cast(u16x2, g[q]) - base;
            mn = min(mn, static_cast<uint32_t>(dt.x > dt.y ? dt.x : dt.y));
        }
        const bool ok = e != kEmpty && mn > w2;
        const uint64_t m = ballot(ok);
        C &= m;
        const uint64_t conf = ballot(C != 0ull) & m;
        uint64_t acc_m = m & ~conf;
        if constexpr (FP == 0) {
            if (conf) {
                uint64_t dec_m = ~conf;
                bool mine = ((conf >> lane) & 1ull) == 0ull;
                for (int pass = 0; dec_m != ~0ull && pass < kWave; ++pass) {
                    const bool can = !mine && (C & ~dec_m) == 0ull;
                    const bool take = can && (C & acc_m) == 0ull;
                    dec_m |= ballot(can);
                    acc_m |= ballot(take);
                    mine = mine || can;
                }
            }
        } else {
            // wave-uniform masks: a lane is decided once all its earlier ok neighbours are (its own
            // decided bit plays `mine`), accepted iff none of them was accepted
            uint64_t dec_m = ~conf;
            for (int pass = 0; dec_m != ~0ull && pass < kWave; ++pass) {
                const uint64_t can_m = ballot((C & ~dec_m) == 0ull) & ~dec_m;
                const uint64_t free_m = ballot((C & acc_m) == 0ull);
                dec_m |= can_m;
                acc_m |= can_m & free_m;
            }
        }
        const uint32_t have = prior + static_cast<uint32_t>(acc);
        const int allow = have < a.need ? static_cast<int>(a.need - have) : 1;
        if (popc64(acc_m) >= allow) {
            uint64_t keep = 0, t = acc_m;
            for (int k = 0; k < allow; ++k) {
                keep |= t & (~t + 1ull);
                t &= t - 1ull;
            }
            acc_m = keep;
            done = true;
        }
        if ((acc_m >> lane) & 1ull) {
            grid[cell] = e;
            if constexpr (!DEFER) {
                const int pos = mbcnt64(acc_m, acc);
                if (pos < a.out_stride) {
                    float2 *o = reinterpret_cast<float2 *>(a.out_xy) + static_cast<int64_t>(f) * a.out_stride + pos;
                    *o = make_float2(static_cast<float>(e & 0xFFFFu), static_cast<float>(e >> 16));
                }
            }
        }
        if constexpr (DEFER) {
            if (lane == 0) accm[b] = acc_m;
        }
        acc += popc64(acc_m);
    }
    if (lane == 0) {
        s_acc = acc;
        if (done) s_done = 1;
    }
}

constexpr int kRows = 480, kCols = 640, kD = 20;

struct alignas(16) ProbeLds {
    uint32_t pxy[kSelectChunk];
    uint32_t pcell[kSelectChunk];
    uint64_t cmask[kSelectChunk];
    uint64_t tmask[kSelectChunk / kWave + 1];
    uint64_t accm[kSelectChunk / kWave];
    ScanLds sl;
    uint32_t grid[kGridLdsCells];
    uint32_t tie_prev;
    int tie_has_prev, s_acc, s_done;
};

template <int VAR>
__global__ __launch_bounds__(1024) void k_probe(SelectArgs a, const uint32_t *pos, int c, uint64_t *out) {
    __shared__ ProbeLds L;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int gw2 = a.grid_w + 2, cells = gw2 * (a.grid_h + 2);
    const uint32_t s1 = static_cast<uint32_t>(a.dist + 1);
    for (int i = tid; i < cells; i += nthr) L.grid[i] = grid_empty(a.rows, a.cols, a.dist);
    for (int i = tid; i < kSelectChunk; i += nthr) {
        const uint32_t e = i < c ? pos[i] : kEmpty;
        L.pxy[i] = e;
        L.pcell[i] = i < c ? ((e >> 16) / s1 + 1) * static_cast<uint32_t>(gw2) + ((e & 0xFFFFu) / s1 + 1)
                           : static_cast<uint32_t>(gw2 + 1);
    }
    for (int i = tid; i <= kSelectChunk / kWave; i += nthr) L.tmask[i] = 0;
    for (int i = tid; i < kScanBatches; i += nthr) L.sl.cnt[i] = kCmItems;  // (masks all ready)
    if (tid == 0) {
        L.tie_prev = 0;
        L.tie_has_prev = 0;
        L.s_acc = 0;
        L.s_done = 0;
    }
    __syncthreads();
    conflict_masks(L.pxy, c, a.dist, a.rows, a.cols, L.cmask, tid, nthr);
    for (int i = c + tid; i < ((c + kWave - 1) & ~(kWave - 1)); i += nthr) L.cmask[i] = 0;
    __syncthreads();
    uint64_t t0 = 0, t1 = 0, r0 = 0, r1 = 0;
    if (tid < kWave) {
        r0 = __builtin_amdgcn_s_memrealtime();
        t0 = __builtin_readcyclecounter();
        if constexpr (VAR == 0)
            greedy_chunk<1>(a, 0, c, L.pxy, L.pcell, L.cmask, L.grid, gw2, 0u, L.s_acc, L.s_done, false, L.tmask, 0u,
                            0u, L.tie_prev, L.tie_has_prev, nullptr);
        else if constexpr (VAR == 1)
            greedy_chunk<1>(a, 0, c, L.pxy, L.pcell, L.cmask, L.grid, gw2, 0u, L.s_acc, L.s_done, true, L.tmask, 0u,
                            0u, L.tie_prev, L.tie_has_prev, nullptr);
        else if constexpr (VAR == 5)
            greedy_scan(a, 0, c, L.pxy, L.pcell, L.cmask, L.grid, gw2, 0u, L.s_acc, L.s_done, L.sl);
        else
            greedy_lean<VAR >= 3, VAR == 4>(a, 0, c, L.pxy, L.pcell, L.cmask, L.grid, gw2, 0u, L.s_acc, L.s_done, L.accm);
        t1 = __builtin_readcyclecounter();
        if constexpr (VAR == 0) {  // core clock calibration: a ~20 us spin against the 100 MHz real-time counter
            while (__builtin_readcyclecounter() - t1 < 50000) __builtin_amdgcn_s_sleep(1);
            t1 = __builtin_readcyclecounter();
        }
        r1 = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    if (tid == 0) {
        out[0] = t1 - t0;
        out[1] = static_cast<uint64_t>(L.s_acc);
        out[2] = r1 - r0;
    }
}

int main(int argc, char **argv) {
    // argv[1] (optional): a chunk's positions in scan order, uint32 (y << 16) | x (greedy_probe_pos.bin:
    // the top 512 Harris candidates of oracle.make_frame("noise", 7, 480, 640), threshold 30), need 200
    const int c = 509;
    std::mt19937 rng(7);
    std::vector<uint32_t> pos(512);
    for (auto &p : pos) p = (static_cast<uint32_t>(rng() % kRows) << 16) | static_cast<uint32_t>(rng() % kCols);
    uint32_t need = 500;
    if (argc > 1) {
        FILE *fp = std::fopen(argv[1], "rb");
        if (!fp || std::fread(pos.data(), 4, 512, fp) != 512) {
            std::printf("cannot read %s\n", argv[1]);
            return 1;
        }
        std::fclose(fp);
        need = 200;
    }
    uint32_t *dpos = nullptr, *status = nullptr;
    uint64_t *out = nullptr;
    float *oxy = nullptr;
    hipMalloc(&dpos, c * 4);
    hipMalloc(&status, 64);
    hipMalloc(&out, 64);
    hipMalloc(&oxy, 8 * 1024);
    hipMemcpy(dpos, pos.data(), c * 4, hipMemcpyHostToDevice);
    std::printf("%s positions, need %u\n", argc > 1 ? argv[1] : "uniform random", need);
    SelectArgs a{};
    a.rows = kRows;
    a.cols = kCols;
    a.dist = kD;
    a.need = need;
    a.grid_w = (kCols + kD) / (kD + 1);
    a.grid_h = (kRows + kD) / (kD + 1);
    a.out_xy = oxy;
    a.out_stride = 1024;
    a.status = status;
    const char *names[] = {"greedy_chunk<1> (+spin)", "greedy_chunk<1> + ties", "lean", "lean, deferred output",
                           "lean, deferred, mask fp", "greedy_scan (pipelined)"};
    for (int var = 0; var < 6; ++var)
    for (int nt : {64, 1024}) {
        uint64_t best = ~0ull, acc = 0, first = 0;
        for (int r = 0; r < 7; ++r) {
            switch (var) {
                case 0: hipLaunchKernelGGL(k_probe<0>, dim3(1), dim3(nt), 0, 0, a, dpos, c, out); break;
                case 1: hipLaunchKernelGGL(k_probe<1>, dim3(1), dim3(nt), 0, 0, a, dpos, c, out); break;
                case 2: hipLaunchKernelGGL(k_probe<2>, dim3(1), dim3(nt), 0, 0, a, dpos, c, out); break;
                case 3: hipLaunchKernelGGL(k_probe<3>, dim3(1), dim3(nt), 0, 0, a, dpos, c, out); break;
                case 4: hipLaunchKernelGGL(k_probe<4>, dim3(1), dim3(nt), 0, 0, a, dpos, c, out); break;
                default: hipLaunchKernelGGL(k_probe<5>, dim3(1), dim3(nt), 0, 0, a, dpos, c, out); break;
            }
            uint64_t h[3];
            hipMemcpy(h, out, 24, hipMemcpyDeviceToHost);
            if (var == 0 && r == 6)
                std::printf("core clock: %llu clocks in %llu real-time ticks (100 MHz): %.0f MHz\n",
                            static_cast<unsigned long long>(h[0]), static_cast<unsigned long long>(h[2]),
                            100.0 * static_cast<double>(h[0]) / static_cast<double>(h[2]));
            if (h[0] < best) best = h[0];
            if (r == 0) first = h[0];
            acc = h[1];
        }
        std::printf("%-24s threads %4d: first launch %llu, best %llu clocks for %d candidates (%d batches, %llu accepted): %.0f per batch\n",
                    names[var], nt, static_cast<unsigned long long>(first), static_cast<unsigned long long>(best), c, (c + 63) / 64, static_cast<unsigned long long>(acc),
                    static_cast<double>(best) / ((c + 63) / 64));
    }
    return 0;
}
