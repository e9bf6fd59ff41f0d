// trans_rate.hip -- issue cost of transcendental and packed ops for ONE wave per SIMD on gfx950
// (the fa_fwd_w4 regime). Standalone diagnostic, not product code.
//
// The tile loop's exps cost ~11 % of C2 (profiles/r3_exp_decision_exp_cost.log: a timing build
// without v_exp_f32 runs 1316 vs 1180 TFLOP/s). This measures cycles per instruction of
// independent streams: v_exp_f32, v_exp_f16, v_exp_legacy_f32, v_fma_f32, v_pk_fma_f32,
// v_pk_mul_f32, v_cvt_pk_f16_f32, each 8 independent chains x 64 iterations, s_memtime around the
// loop, one workgroup of 4 waves per CU on every CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define BODY8(INS)                                                                                             \
    asm volatile(INS " %0, %0\n\t" INS " %1, %1\n\t" INS " %2, %2\n\t" INS " %3, %3\n\t" INS " %4, %4\n\t" INS \
                     " %5, %5\n\t" INS " %6, %6\n\t" INS " %7, %7"                                               \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));

template <int K>
__global__ __launch_bounds__(256, 1) void probe(unsigned long long *out, float seed) {
    float a0 = seed, a1 = seed * 1.1f, a2 = seed * 1.2f, a3 = seed * 1.3f, a4 = seed * 1.4f, a5 = seed * 1.5f,
          a6 = seed * 1.6f, a7 = seed * 1.7f;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < 64; ++it) {
        if constexpr (K == 0) { BODY8("v_exp_f32") }
        if constexpr (K == 1) { BODY8("v_exp_f16") }
        if constexpr (K == 2) { BODY8("v_exp_legacy_f32") }
        if constexpr (K == 3) {
            asm volatile(
                "v_fma_f32 %0, %0, %0, %0\n\tv_fma_f32 %1, %1, %1, %1\n\tv_fma_f32 %2, %2, %2, %2\n\tv_fma_f32 %3, %3, %3, %3\n\t"
                "v_fma_f32 %4, %4, %4, %4\n\tv_fma_f32 %5, %5, %5, %5\n\tv_fma_f32 %6, %6, %6, %6\n\tv_fma_f32 %7, %7, %7, %7"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        }
        if constexpr (K == 4) {  // v_exp_f16 on the high halves too (op_sel): two f16 exps per register
            asm volatile(
                "v_exp_f16 %0, %0\n\tv_exp_f16_sdwa %1, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
                "v_exp_f16 %2, %2\n\tv_exp_f16_sdwa %3, %3 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
                "v_exp_f16 %4, %4\n\tv_exp_f16_sdwa %5, %5 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1\n\t"
                "v_exp_f16 %6, %6\n\tv_exp_f16_sdwa %7, %7 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        }
        if constexpr (K == 5) {
            asm volatile(
                "v_cvt_pk_f16_f32 %0, %0, %1\n\tv_cvt_pk_f16_f32 %1, %1, %2\n\tv_cvt_pk_f16_f32 %2, %2, %3\n\tv_cvt_pk_f16_f32 %3, %3, %4\n\t"
                "v_cvt_pk_f16_f32 %4, %4, %5\n\tv_cvt_pk_f16_f32 %5, %5, %6\n\tv_cvt_pk_f16_f32 %6, %6, %7\n\tv_cvt_pk_f16_f32 %7, %7, %0"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = t1 - t0;
    if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 12345.678f) out[1] = 1;  // keep the chains live
}

int main() {
    unsigned long long *d, h[2];
    if (hipMalloc(&d, 16) != hipSuccess) return 1;
    const char *names[] = {"v_exp_f32", "v_exp_f16", "v_exp_legacy_f32", "v_fma_f32", "v_exp_f16 lo+hi (sdwa)", "v_cvt_pk_f16_f32"};
    for (int rep = 0; rep < 3; ++rep) {
        for (int k = 0; k < 6; ++k) {
            void (*kern)(unsigned long long *, float) = k == 0 ? probe<0> : k == 1 ? probe<1> : k == 2 ? probe<2>
                                                       : k == 3 ? probe<3> : k == 4 ? probe<4> : probe<5>;
            for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(kern, dim3(256), dim3(256), 0, 0, d, 0.5f);
            if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, d, 16, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            printf("rep %d %-24s %6.2f cycles per instruction (one wave per SIMD, 8 independent chains)\n", rep, names[k],
                   (double)h[0] / (64.0 * 8.0));
        }
    }
    return 0;
}
