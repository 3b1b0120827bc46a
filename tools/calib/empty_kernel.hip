// Launch-floor calibration: kernel durations of an empty kernel and of a 1-workgroup kernel that loads
// 16 KB, at the headline's grid shapes (rocprofv3 --kernel-trace --stats reports them).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int *p) {
    if (p && threadIdx.x == 1 && blockIdx.x == 0xFFFFFF) p[0] = 1;
}
__global__ __launch_bounds__(1024) void k_load16k(const unsigned *h, unsigned *o) {
    unsigned v = 0;
    for (int j = 0; j < 4; ++j) v += h[threadIdx.x + j * 1024];
    __shared__ unsigned s[1024];
    s[threadIdx.x] = v;
    __syncthreads();
    if (threadIdx.x == 0) o[0] = s[5];
}

int main() {
    unsigned *h = nullptr, *o = nullptr;
    hipMalloc(&h, 16384 * 4);
    hipMalloc(&o, 64);
    hipMemset(h, 0, 16384 * 4);
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, nullptr);
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_empty, dim3(120), dim3(256), 0, 0, nullptr);
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_load16k, dim3(1), dim3(1024), 0, 0, h, o);
    hipDeviceSynchronize();
    std::printf("done\n");
    return 0;
}
