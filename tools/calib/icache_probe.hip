// Instruction-fetch probe (diagnostic, not part of the library): core clocks of one wave running N
// straight-line dependent FMAs (8-byte VOP3 each: N = 2048 is 16 KB of code executed once), on the
// first pass (cold instruction cache: each launch lands on another CU) and on a second pass over the
// same code in the same launch (warm), with the hardware id each launch ran on. No arguments.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

template <int N>
__global__ __launch_bounds__(64) void k_straight(uint64_t *out, float seed) {
    float x = seed + static_cast<float>(threadIdx.x);
#pragma unroll 1
    for (int rep = 0; rep < 2; ++rep) {  // the same code twice: cold, then warm instruction cache
        asm volatile("" : "+v"(x));
        const uint64_t t0 = __builtin_readcyclecounter();
        asm volatile("" : "+v"(x));
#pragma unroll
        for (int i = 0; i < N; ++i) x = __builtin_fmaf(x, 1.0001f + static_cast<float>(i) * 1e-7f, 0.5f);
        asm volatile("" : "+v"(x));
        const uint64_t t1 = __builtin_readcyclecounter();
        if (threadIdx.x == 0) out[rep] = t1 - t0;
    }
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));  // HW_REG_HW_ID
    if (threadIdx.x == 0) out[2] = hw;
    if (x == 12345.0f) out[3] = 1;
}

template <int N>
void run(uint64_t *d) {
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k_straight<N>, dim3(1), dim3(64), 0, 0, d, 1.0f);
        uint64_t h[3] = {0, 0, 0};
        (void)hipMemcpy(h, d, 24, hipMemcpyDeviceToHost);
        std::printf("N %5d (%3d KB) launch %d: cold %7llu clocks (%.2f per instruction), warm %7llu (%.2f), hw_id 0x%08llx\n",
                    N, N * 8 / 1024, r, static_cast<unsigned long long>(h[0]), static_cast<double>(h[0]) / N,
                    static_cast<unsigned long long>(h[1]), static_cast<double>(h[1]) / N,
                    static_cast<unsigned long long>(h[2]));
    }
}

int main() {
    uint64_t *d = nullptr;
    (void)hipMalloc(&d, 64);
    run<256>(d);
    run<1024>(d);
    run<2048>(d);
    run<4096>(d);
    return 0;
}
