// VALU issue-cost probe (gfx950): cycles per wave-instruction per SIMD for the instruction classes of
// the per-pixel kernels (K1 k_corner*, K3 k_fast), at 1..8 waves per SIMD. Each wave runs a loop of
// 32 instructions of one class over 8 independent register chains (so one wave alone is not bound by
// dependency latency beyond 8 instructions); cycles come from s_memtime at the wave's start and end.
// usage: valu_probe   (prints one line per class and waves/SIMD)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#include <utility>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int kIters = 2048;

#define R8(op) op(0) op(1) op(2) op(3) op(4) op(5) op(6) op(7)
#define BODY4(X) X X X X
#define BIG4(X) X X X X
#define BIG64(X) BIG4(BIG4(BIG4(X)))

template <int CLASS>
__global__ __launch_bounds__(256) void probe(uint64_t *cyc, uint32_t *sink, uint32_t seed) {
    uint32_t v0 = seed + threadIdx.x, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7, v4 = v0 * 11, v5 = v0 * 13,
             v6 = v0 * 17, v7 = v0 * 19;
    uint32_t w0 = v0 ^ 1, w1 = v1 ^ 1, w2 = v2 ^ 1, w3 = v3 ^ 1, w4 = v4 ^ 1, w5 = v5 ^ 1, w6 = v6 ^ 1, w7 = v7 ^ 1;
    uint64_t p0 = v0 | (uint64_t(v1) << 32), p1 = v1 | (uint64_t(v2) << 32), p2 = v2 | (uint64_t(v3) << 32),
             p3 = v3 | (uint64_t(v4) << 32), p4 = v4 | (uint64_t(v5) << 32), p5 = v5 | (uint64_t(v6) << 32),
             p6 = v6 | (uint64_t(v7) << 32), p7 = v7 | (uint64_t(v0) << 32);
    const uint64_t q0 = p0 ^ 3, q1 = p1 ^ 3, q2 = p2 ^ 3, q3 = p3 ^ 3, q4 = p4 ^ 3, q5 = p5 ^ 3, q6 = p6 ^ 3, q7 = p7 ^ 3;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it) {
#define A3(i) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(v##i) : "v"(w##i));
#define ADD(i) asm volatile("v_add_u32_e32 %0, %1, %0" : "+v"(v##i) : "v"(w##i));
#define MAD(i) asm volatile("v_mad_i32_i24 %0, %0, %1, %0" : "+v"(v##i) : "v"(w##i));
#define PK(i) asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(p##i) : "v"(q##i));
#define FMA(i) asm volatile("v_fma_f32 %0, %0, %1, %0" : "+v"(v##i) : "v"(w##i));
#define DPPW(i) asm volatile("v_mov_b32_dpp %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(v##i) : "v"(w##i));
#define DPPR(i) asm volatile("v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(v##i) : "v"(w##i));
#define SDWA(i) asm volatile("v_sub_u32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_3" : "+v"(v##i) : "v"(w##i));
#define RSQ(i) asm volatile("v_rsq_f32_e32 %0, %1" : "=v"(v##i) : "v"(w##i));
#define MAX3(i) asm volatile("v_max3_f32 %0, %0, %1, %0" : "+v"(v##i) : "v"(w##i));
#define CMPADDC(i) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1\n\tv_addc_co_u32_e32 %0, vcc, 0, %0, vcc" : "+v"(v##i) : "v"(w##i) : "vcc");
#define CND(i) asm volatile("v_cmp_gt_f32_e64 s[2:3], %0, %1\n\tv_cndmask_b32_e64 %0, 0, %0, s[2:3]" : "+v"(v##i) : "v"(w##i) : "s2", "s3");
#define PKMIX(i) asm volatile("v_pk_fma_f32 %0, %0, %2, %0\n\tv_add3_u32 %1, %1, %3, %1" : "+v"(p##i), "+v"(v##i) : "v"(q##i), "v"(w##i));
#define X15(i) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X16(i) asm volatile("v_pk_mad_u16 %0, %0, %1, %0" : "+v"(v##i) : "v"(w##i));
#define X17(i) asm volatile("v_pk_mul_lo_u16 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X18(i) asm volatile("v_dot2_u32_u16 %0, %1, %1, %0" : "+v"(v##i) : "v"(w##i));
#define X19(i) asm volatile("v_dot2_i32_i16 %0, %1, %1, %0" : "+v"(v##i) : "v"(w##i));
#define X20(i) asm volatile("v_dot4_u32_u8 %0, %1, %1, %0" : "+v"(v##i) : "v"(w##i));
#define X21(i) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(v##i) : "v"(w##i));
#define X22(i) asm volatile("v_bfe_u32 %0, %1, 8, 8" : "=v"(v##i) : "v"(w##i));
#define X23(i) asm volatile("v_lshl_add_u32 %0, %0, 9, %1" : "+v"(v##i) : "v"(w##i));
#define X24(i) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(v##i) : "v"(w##i));
#define X25(i) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1" : : "v"(v##i), "v"(w##i) : "vcc");
#define X26(i) asm volatile("v_max_f32_e32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X27(i) asm volatile("v_mul_f32_e32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X28(i) asm volatile("v_add_f32_e32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X29(i) asm volatile("v_mul_u32_u24_e32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X30(i) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(v##i) : "v"(w##i));
#define X31(i) asm volatile("v_addc_co_u32_e32 %0, vcc, 0, %0, vcc" : "+v"(v##i) : : "vcc");
#define X32(i) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(v##i) : "v"(w##i));
#define X33(i) asm volatile("v_mov_b32_e32 %0, %1" : "=v"(v##i) : "v"(w##i));
#define X34(i) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf" : "=v"(v##i) : "v"(w##i));
#define X35(i) asm volatile("v_add_u32_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v##i) : "v"(w##i));
#define X36(i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p##i) : "v"(q##i));
#define X37(i) asm volatile("v_sqrt_f32_e32 %0, %1" : "=v"(v##i) : "v"(w##i));
#define X38(i) asm volatile("v_rsq_f32_e32 %0, %1\n\tv_fma_f32 %2, %2, %3, %2" : "=v"(v##i), "+v"(w##i) : "v"(w##i), "v"(v##i));
#define X39(i) asm volatile("v_sad_u16 %0, %0, %1, %0" : "+v"(v##i) : "v"(w##i));
#define X40(i) asm volatile("v_add_u16_e32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X41(i) asm volatile("v_and_b32_e32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X42(i) asm volatile("v_lshrrev_b32_e32 %0, 8, %0" : "+v"(v##i));
#define X43(i) asm volatile("v_sub_u32_e32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X44(i) asm volatile("v_fmac_f32_e32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X45(i) asm volatile("v_pk_fma_f32 %0, %1, %1, %0" : "+v"(p##i) : "v"(q##i));
#define X46(i) asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(v##i) : "v"(w##i), "v"(w##i), "v"(v##i));
#define X47(i) asm volatile("v_cvt_f32_ubyte0_e32 %0, %1" : "=v"(v##i) : "v"(w##i));
#define X48(i) asm volatile("v_cvt_f32_ubyte3_e32 %0, %1" : "=v"(v##i) : "v"(w##i));
#define X49(i) asm volatile("v_cvt_f32_i32_e32 %0, %1" : "=v"(v##i) : "v"(w##i));
#define X50(i) asm volatile("v_rsq_f32_e64 %0, %1 div:2" : "=v"(v##i) : "v"(w##i));
#define X51(i) asm volatile("v_mul_f32_e64 %0, %0, %1 mul:2" : "+v"(v##i) : "v"(w##i));
#define X52(i) asm volatile("v_sub_f32_e32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X53(i) asm volatile("v_fma_f32 %0, -%0, %1, %0" : "+v"(v##i) : "v"(w##i));
#define X54(i) asm volatile("v_cndmask_b32_e64 %0, 0, %0, s[4:5]" : "+v"(v##i) : : "s4", "s5");
#define X55(i) asm volatile("v_cmp_gt_f32_e64 s[4:5], %0, %1" : : "v"(v##i), "v"(w##i) : "s4", "s5");
#define X56(i) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X57(i) asm volatile("v_min_f32_e32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X58(i) asm volatile("v_max_u32_e32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X59(i) asm volatile("v_med3_f32 %0, %0, %1, %0" : "+v"(v##i) : "v"(w##i));
#define X60(i) asm volatile("v_mul_legacy_f32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X61(i) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(v##i) : "v"(w##i) : "vcc");
#define X62(i) asm volatile("v_or3_b32 %0, %0, %1, %0" : "+v"(v##i) : "v"(w##i));
#define X63(i) asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(v##i) : "v"(w##i));
#define X64(i) asm volatile("v_cvt_f32_u32_e32 %0, %1" : "=v"(v##i) : "v"(w##i));
#define X65(i) asm volatile("v_lshlrev_b32_e32 %0, 9, %0" : "+v"(v##i));
#define X66(i) asm volatile("v_cmp_gt_f32_e32 vcc, %0, %1\n\tv_cndmask_b32_e32 %0, 0, %0, vcc" : "+v"(v##i) : "v"(w##i) : "vcc");
#define X67(i) asm volatile("v_cmp_gt_f32_e64 s[6:7], %0, %1\n\tv_cndmask_b32_e64 %2, 0, %3, s[6:7]\n\tv_add_u32_e32 %0, %0, %2" : "+v"(v##i), "=&v"(w##i) : "v"(w##i), "v"(512) : "s6", "s7");
#define X68(i) asm volatile("v_add_f32_e32 %0, %0, %1\n\tv_mov_b32_dpp %1, %0 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v##i), "+v"(w##i));
#define X69(i) asm volatile("ds_write2st64_b32 %0, %1, %1 offset1:1" : : "v"(v##i & 0x1FC), "v"(w##i) : "memory");
        if constexpr (CLASS == 0) { BODY4(R8(A3)) }
        if constexpr (CLASS == 1) { BODY4(R8(ADD)) }
        if constexpr (CLASS == 2) { BODY4(R8(MAD)) }
        if constexpr (CLASS == 3) { BODY4(R8(FMA)) }
        if constexpr (CLASS == 4) { BODY4(R8(PK)) }
        if constexpr (CLASS == 5) { BODY4(R8(DPPW)) }
        if constexpr (CLASS == 6) { BODY4(R8(DPPR)) }
        if constexpr (CLASS == 7) { BODY4(R8(SDWA)) }
        if constexpr (CLASS == 8) { BODY4(R8(RSQ)) }
        if constexpr (CLASS == 9) { BODY4(R8(MAX3)) }
        if constexpr (CLASS == 10) { BODY4(R8(CMPADDC)) }
        if constexpr (CLASS == 11) { BODY4(R8(CND)) }
        if constexpr (CLASS == 12) { BODY4(R8(PKMIX)) }
        if constexpr (CLASS == 15) { BODY4(R8(X15)) }
        if constexpr (CLASS == 16) { BODY4(R8(X16)) }
        if constexpr (CLASS == 17) { BODY4(R8(X17)) }
        if constexpr (CLASS == 18) { BODY4(R8(X18)) }
        if constexpr (CLASS == 19) { BODY4(R8(X19)) }
        if constexpr (CLASS == 20) { BODY4(R8(X20)) }
        if constexpr (CLASS == 21) { BODY4(R8(X21)) }
        if constexpr (CLASS == 22) { BODY4(R8(X22)) }
        if constexpr (CLASS == 23) { BODY4(R8(X23)) }
        if constexpr (CLASS == 24) { BODY4(R8(X24)) }
        if constexpr (CLASS == 25) { BODY4(R8(X25)) }
        if constexpr (CLASS == 26) { BODY4(R8(X26)) }
        if constexpr (CLASS == 27) { BODY4(R8(X27)) }
        if constexpr (CLASS == 28) { BODY4(R8(X28)) }
        if constexpr (CLASS == 29) { BODY4(R8(X29)) }
        if constexpr (CLASS == 30) { BODY4(R8(X30)) }
        if constexpr (CLASS == 31) { BODY4(R8(X31)) }
        if constexpr (CLASS == 32) { BODY4(R8(X32)) }
        if constexpr (CLASS == 33) { BODY4(R8(X33)) }
        if constexpr (CLASS == 34) { BODY4(R8(X34)) }
        if constexpr (CLASS == 35) { BODY4(R8(X35)) }
        if constexpr (CLASS == 36) { BODY4(R8(X36)) }
        if constexpr (CLASS == 37) { BODY4(R8(X37)) }
        if constexpr (CLASS == 38) { BODY4(R8(X38)) }
        if constexpr (CLASS == 39) { BODY4(R8(X39)) }
        if constexpr (CLASS == 40) { BODY4(R8(X40)) }
        if constexpr (CLASS == 41) { BODY4(R8(X41)) }
        if constexpr (CLASS == 42) { BODY4(R8(X42)) }
        if constexpr (CLASS == 43) { BODY4(R8(X43)) }
        if constexpr (CLASS == 44) { BODY4(R8(X44)) }
        if constexpr (CLASS == 45) { BODY4(R8(X45)) }
        if constexpr (CLASS == 46) { BODY4(R8(X46)) }
        if constexpr (CLASS == 47) { BODY4(R8(X47)) }
        if constexpr (CLASS == 48) { BODY4(R8(X48)) }
        if constexpr (CLASS == 49) { BODY4(R8(X49)) }
        if constexpr (CLASS == 50) { BODY4(R8(X50)) }
        if constexpr (CLASS == 51) { BODY4(R8(X51)) }
        if constexpr (CLASS == 52) { BODY4(R8(X52)) }
        if constexpr (CLASS == 53) { BODY4(R8(X53)) }
        if constexpr (CLASS == 54) { BODY4(R8(X54)) }
        if constexpr (CLASS == 55) { BODY4(R8(X55)) }
        if constexpr (CLASS == 56) { BODY4(R8(X56)) }
        if constexpr (CLASS == 57) { BODY4(R8(X57)) }
        if constexpr (CLASS == 58) { BODY4(R8(X58)) }
        if constexpr (CLASS == 59) { BODY4(R8(X59)) }
        if constexpr (CLASS == 60) { BODY4(R8(X60)) }
        if constexpr (CLASS == 61) { BODY4(R8(X61)) }
        if constexpr (CLASS == 62) { BODY4(R8(X62)) }
        if constexpr (CLASS == 63) { BODY4(R8(X63)) }
        if constexpr (CLASS == 64) { BODY4(R8(X64)) }
        if constexpr (CLASS == 65) { BODY4(R8(X65)) }
        if constexpr (CLASS == 66) { BODY4(R8(X66)) }
        if constexpr (CLASS == 67) { BODY4(R8(X67)) }
        if constexpr (CLASS == 68) { BODY4(R8(X68)) }
        if constexpr (CLASS == 69) { BODY4(R8(X69)) }
        // mixes: does a dual-capable op (v_add/mul_f32) issue beside a packed / 3-operand one?
#define M70(i) PK(i) X28(i)
#define M71(i) PK(i) X27(i) X28(i)
#define M72(i) MAX3(i) X28(i)
#define M73(i) X27(i) X28(i)
#define M74(i) X36(i) X28(i) X52(i)
#define M75(i) PK(i) X41(i)
        if constexpr (CLASS == 70) { BODY4(R8(M70)) }
        if constexpr (CLASS == 71) { BODY4(R8(M71)) }
        if constexpr (CLASS == 72) { BODY4(R8(M72)) }
        if constexpr (CLASS == 73) { BODY4(R8(M73)) }
        if constexpr (CLASS == 74) { BODY4(R8(M74)) }
        if constexpr (CLASS == 75) { BODY4(R8(M75)) }
        // big loop bodies (instruction-fetch test): 64x the 32-instruction block, 1/64 of the iterations
        if constexpr (CLASS == 13) { if (it % 64 == 0) { BIG64(BODY4(R8(A3))) } }
        if constexpr (CLASS == 14) { if (it % 64 == 0) { BIG64(BODY4(R8(ADD))) } }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = static_cast<uint32_t>(p0 ^ p1 ^ p2 ^ p3 ^ p4 ^ p5 ^ p6 ^ p7) ^ v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7 ^ w0 ^ w1 ^ w2 ^ w3 ^ w4 ^ w5 ^ w6 ^ w7;
}

static const char *kNames[] = {"v_add3_u32", "v_add_u32_e32", "v_mad_i32_i24", "v_fma_f32", "v_pk_fma_f32",
                               "dpp wave_shr", "dpp row_shr", "v_sub_u32_sdwa", "v_rsq_f32", "v_max3_f32",
                               "cmp+addc (2)", "cmp_e64+cndmask (2)", "pk_fma+add3 (2)",
                               "v_add3 16KB body", "v_add_e32 8KB body", "v_pk_add_u16", "v_pk_mad_u16", "v_pk_mul_lo_u16", "v_dot2_u32_u16", "v_dot2_i32_i16", "v_dot4_u32_u8", "v_perm_b32", "v_bfe_u32", "v_lshl_add_u32", "v_cndmask_b32_e32", "v_cmp_gt_f32_e32", "v_max_f32_e32", "v_mul_f32_e32", "v_add_f32_e32", "v_mul_u32_u24_e32", "v_mad_u32_u24", "v_addc_co_u32_e32", "v_alignbyte_b32", "v_mov_b32_e32", "dpp quad_perm", "v_add_u32_dpp", "v_pk_add_f32", "v_sqrt_f32", "rsq+fma (2)", "v_sad_u16", "v_add_u16_e32", "v_and_b32_e32", "v_lshrrev_b32_e32", "v_sub_u32_e32", "v_fmac_f32_e32", "v_pk_fma_f32 2-reg", "v_add3 distinct", "v_cvt_f32_ubyte0", "v_cvt_f32_ubyte3", "v_cvt_f32_i32", "v_rsq_f32 div:2", "v_mul_f32 mul:2", "v_sub_f32_e32", "v_fma_f32 neg", "cndmask_e64 s-pair", "cmp_e64 only", "v_add_u32_e64", "v_min_f32_e32", "v_max_u32_e32", "v_med3_f32", "v_mul_legacy_f32", "v_add_co_u32_e32", "v_or3_b32", "v_xor_b32_e32", "v_cvt_f32_u32", "v_lshlrev_b32_e32", "v_cndmask_e32 after cmp", "cmp_e64+cndmask+add (3)", "v_mov_b32_dpp wave_shl dep", "ds_write2st64_b32", "pk_fma+add_f32 (2)", "pk_fma+mul+add_f32 (3)", "max3+add_f32 (2)", "mul_f32+add_f32 (2)", "pk_add+add+sub_f32 (3)", "pk_fma+and_b32 (2)"};

template <int C>
static int run(int cus, uint64_t *dcyc, uint32_t *dsink) {
    for (int w : {1, 2, 4, 8}) {
        if (w != 1 && w != 8 && getenv("PROBE_QUICK")) continue;
        const int blocks = cus * w;
        hipLaunchKernelGGL(probe<C>, dim3(blocks), dim3(256), 0, 0, dcyc, dsink, 1u);  // warm
        CHECK(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        CHECK(hipEventRecord(e0));
        hipLaunchKernelGGL(probe<C>, dim3(blocks), dim3(256), 0, 0, dcyc, dsink, 2u);
        CHECK(hipEventRecord(e1));
        CHECK(hipDeviceSynchronize());
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<uint64_t> c(blocks * 4);
        CHECK(hipMemcpy(c.data(), dcyc, c.size() * 8, hipMemcpyDeviceToHost));
        std::sort(c.begin(), c.end());
        const int per_iter = (C == 67 || C == 71 || C == 74) ? 96 : (((C >= 10 && C <= 12) || C == 38 || C == 68 || C == 70 || C == 72 || C == 73 || C == 75) ? 64 : 32);  // wave-instructions per loop iteration (average)
        const double instr = double(kIters) * per_iter;
        // waves per SIMD = w (a 256-thread block puts one wave on each SIMD of its CU)
        printf("%-22s waves/SIMD %d  cycles/instr/SIMD (median wave) %.2f  (max wave) %.2f  wall %.3f ms -> %.2f GHz-equiv\n",
               kNames[C], w, double(c[c.size() / 2]) / (instr * w), double(c.back()) / (instr * w), ms,
               double(c.back()) / (ms * 1e6));
        CHECK(hipEventDestroy(e0));
        CHECK(hipEventDestroy(e1));
    }
    return 0;
}

template <int... Cs>
static int run_all(int cus, uint64_t *d, uint32_t *k, int only, std::integer_sequence<int, Cs...>) {
    int rc = 0;
    ((rc = rc ? rc : ((only < 0 || only == Cs) ? run<Cs>(cus, d, k) : 0)), ...);
    return rc;
}

int main(int argc, char **argv) {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint64_t *dcyc;
    uint32_t *dsink;
    CHECK(hipMalloc(&dcyc, sizeof(uint64_t) * cus * 8 * 4));
    CHECK(hipMalloc(&dsink, sizeof(uint32_t) * cus * 8 * 256));
    printf("CUs %d, clock %d kHz\n", cus, p.clockRate);
    const int only = argc > 1 ? atoi(argv[1]) : -1;
    if (run_all(cus, dcyc, dsink, only, std::make_integer_sequence<int, 76>())) return 1;
    printf("valu_probe done\n");
    return 0;
}
