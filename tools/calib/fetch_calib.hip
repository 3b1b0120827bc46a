// FETCH_SIZE calibration for 4-byte-per-lane buffer loads (the per-pixel kernels' access width):
// each wave streams rows of a frame-sized buffer with buffer_load_dword, like K1, and writes one
// word per workgroup. Run under rocprofv3 --pmc FETCH_SIZE; compare with the known byte count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void k_stream_dword(const uint8_t *p, uint32_t bytes, uint32_t *out) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p), 0, static_cast<int>(bytes), 0x00020000);
    const uint32_t chunk = bytes / gridDim.x;  // contiguous slice per workgroup
    const uint32_t base = blockIdx.x * chunk;
    uint32_t acc = 0;
    for (uint32_t off = threadIdx.x * 4; off < chunk; off += blockDim.x * 4)
        acc ^= static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(base + off), 0, 0));
    if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keeps the loads live
}

int main() {
    const uint32_t bytes = 512u << 20;  // 512 MiB: far beyond the Infinity Cache
    uint8_t *p;
    uint32_t *o;
    if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&o, 4096 * 4) != hipSuccess) return 1;
    hipMemset(p, 1, bytes);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_stream_dword, dim3(4096), dim3(256), 0, 0, p, bytes, o);
    hipDeviceSynchronize();
    std::printf("{\"bytes_per_launch\": %u}\n", bytes);
    hipFree(p);
    hipFree(o);
    return 0;
}
