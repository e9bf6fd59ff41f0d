// MFMA data-hazard probe for gfx950: compile with
//   hipcc --offload-arch=gfx950 -O3 -S --cuda-device-only scripts/microbench/mfma_hazard_probe.hip -o probe.s
// and read the s_nop the compiler's hazard recognizer puts between each pair (builtins, so it sees
// them): VALU write -> MFMA SrcA/B 1 wait state (s_nop 0), VALU -> SrcC 2 (s_nop 1), 32x32x16 result ->
// VALU / store 12 (s_nop 11), 16x16x32 result -> VALU 8 (s_nop 7), MFMA -> same-size SrcC 0. These are
// the counts flash_attention_cute_amd/_asm_check.hazards enforces around the inline-asm MFMAs, which
// the recognizer cannot see.
#include <hip/hip_runtime.h>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define FENCE __builtin_amdgcn_sched_barrier(0)
// (a) VALU write of an operand VGPR -> MFMA SrcA read
__global__ void valu_to_srca(f32x16 *out, const f16x8 *in, const f32x16 *c) {
    f16x8 a = in[threadIdx.x], b = in[threadIdx.x + 64];
    f32x16 acc = c[threadIdx.x];
    FENCE;
    a = a * (_Float16)1.5f;  // VALU (v_pk_mul_f16)
    FENCE;
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    FENCE;
    out[threadIdx.x] = acc;
}
// (b) VALU write of the accumulator -> MFMA SrcC read
__global__ void valu_to_srcc(f32x16 *out, const f16x8 *in, const f32x16 *c) {
    f16x8 a = in[threadIdx.x], b = in[threadIdx.x + 64];
    f32x16 acc = c[threadIdx.x];
    FENCE;
    acc = acc * 2.0f;
    FENCE;
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    FENCE;
    out[threadIdx.x] = acc;
}
// (c) MFMA write -> VALU read
__global__ void mfma_to_valu(f32x16 *out, const f16x8 *in, const f32x16 *c) {
    f16x8 a = in[threadIdx.x], b = in[threadIdx.x + 64];
    f32x16 acc = c[threadIdx.x];
    FENCE;
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    FENCE;
    float x = acc[3] * 3.0f;
    FENCE;
    out[threadIdx.x][0] = x;
}
// (d) MFMA write -> MFMA SrcA read (the result, converted, as an operand)
__global__ void mfma_to_mfma_srcc_same(f32x16 *out, const f16x8 *in, const f32x16 *c) {
    f16x8 a = in[threadIdx.x], b = in[threadIdx.x + 64];
    f32x16 acc = c[threadIdx.x];
    FENCE;
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    FENCE;
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, acc, 0, 0, 0);
    FENCE;
    out[threadIdx.x] = acc;
}
// (e) 16x16x32: VALU -> SrcA, MFMA -> VALU
typedef float f32x4v __attribute__((ext_vector_type(4)));
__global__ void mfma16_to_valu(float *out, const f16x8 *in, const f32x4v *c) {
    f16x8 a = in[threadIdx.x], b = in[threadIdx.x + 64];
    f32x4v acc = c[threadIdx.x];
    FENCE;
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc, 0, 0, 0);
    FENCE;
    out[threadIdx.x] = acc[1] * 3.0f;
}
// (f) MFMA reads SrcC (c), then VALU overwrites c's registers (WAR on SrcC)
__global__ void srcc_war(f32x16 *out, const f16x8 *in, const f32x16 *c) {
    f16x8 a = in[threadIdx.x], b = in[threadIdx.x + 64];
    f32x16 cc = c[threadIdx.x];
    f32x16 acc;
    FENCE;
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, cc, 0, 0, 0);
    FENCE;
    cc = cc * 3.0f;  // new values into the same registers if the allocator reuses them
    FENCE;
    out[threadIdx.x] = acc + cc;
}
// (g) MFMA reads SrcA, then VALU overwrites a
__global__ void srca_war(f32x16 *out, f16x8 *in, const f32x16 *c) {
    f16x8 a = in[threadIdx.x], b = in[threadIdx.x + 64];
    f32x16 acc = c[threadIdx.x];
    FENCE;
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    FENCE;
    a = a * (_Float16)3.0f;
    FENCE;
    in[threadIdx.x] = a;
    out[threadIdx.x] = acc;
}
// (h) MFMA write then VALU write of the same registers (WAW): result discarded
__global__ void mfma_waw(float *out, const f16x8 *in, const f32x16 *c) {
    f16x8 a = in[threadIdx.x], b = in[threadIdx.x + 64];
    f32x16 acc = c[threadIdx.x];
    FENCE;
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
    FENCE;
    acc[0] = 7.0f;
    FENCE;
    out[threadIdx.x] = acc[0] + acc[5];
}
