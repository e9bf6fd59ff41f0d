// rowsum_filler.hip -- cycles per v_mfma_f32_32x32x16_bf16 with the tile loop's per-gap softmax
// filler, ONE wave per SIMD on every CU (the fa_fwd_w4 regime). Standalone diagnostic, not product
// code. The question: does the row sum cost less as one v_dot2_f32_bf16 per rounded P pair (fp32
// accumulate of the two bf16 halves, the same rounded P the P.V MFMA uses) than as two v_add_f32 of
// the fp32 exps?
//   V0  bare MFMAs
//   V1  the kernel's unit per gap: v_fma_f32 + v_exp_f32 + v_add_f32, every other gap v_cvt_pk_bf16_f32
//   V2  the same with the sum as v_dot2_f32_bf16 of the packed pair, every other gap (no v_add_f32)
//   V3  V1 without any sum (the floor of both)
//   V4  V1 + one v_max3_f32 per gap (phase 2's max chains)
//   V5  V1 + phase 2's V^T reads (8 ds_read_b64_tr_b16 per 8 gaps, two per gap in the first four)
//   V6  V5 + one v_max3_f32 per gap (phase 2's mix)
//   V7  V1 + phase 1's K reads (two ds_read_b128 every 4 gaps)
//   V8  V6 with the V^T reads spread one per gap over all 8 gaps, counted waits (6/4/2/0) in gaps 0-3
//   V9  V7 with the two K reads of a 4-gap step in its first two gaps, one each
//   V10 V6 with the 8 V^T reads of a step in its first gap; V11 four in each of its first two gaps
// Each gap is one asm statement (MFMA then its fillers), 8 gaps per iteration over 4 accumulators,
// 256 iterations between s_memtime stamps.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));


template <int V>
__global__ __launch_bounds__(256, 1) void probe(unsigned long long *out, float seed) {
    __shared__ uint4 lds[2048];  // 32 KiB: LDS reads of the V5-V7 variants
    lds[threadIdx.x] = make_uint4(threadIdx.x, 1, 2, 3);
    __syncthreads();
    // conflict-free: lane i reads 8 B (tr_b16) / 16 B (b128) at 16 * i, each wave its own 1 KiB
    const uint32_t laddr = (uint32_t)(uintptr_t)lds + 16 * (threadIdx.x & 63) + 1024 * (threadIdx.x >> 6);
    float mx = seed;
    uint2 tr = make_uint2(0, 0);
    uint4 kr = make_uint4(0, 0, 0, 0);
    f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    u32x4 a = {__float_as_uint(seed), 0x3f803f80u, 0x3f003f00u, 0x3e803e80u};
    u32x4 b = {0x3f803f80u, __float_as_uint(seed * 2.f), 0x3f003f00u, 0x3e803e80u};
    float s0 = seed, s1 = seed * 0.5f, sc = 0.1275f, nm = -1.f, acc = 0.f, x0 = 0.f, x1 = 0.f, t = 0.f;
    uint32_t w = 0, ones = 0x3f803f80u;  // (1, 1) in bf16
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < 256; ++it) {
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            f32x16 &c = (g & 3) == 0 ? c0 : (g & 3) == 1 ? c1 : (g & 3) == 2 ? c2 : c3;
            // (written registers are "+v" operands; named operands: c a b t xn xo acc s sc nm w ones)
#define OPS_W [c] "+v"(c), [t] "+v"(t), [xn] "+v"((g & 1) ? x1 : x0), [acc] "+v"(acc), [w] "+v"(w)
#define OPS_R [a] "v"(a), [b] "v"(b), [xo] "v"((g & 1) ? x0 : x1), [s] "v"((g & 1) ? s1 : s0), [sc] "v"(sc), \
              [nm] "v"(nm), [ones] "v"(ones)
#define MFN "v_mfma_f32_32x32x16_bf16 %[c], %[a], %[b], %[c]\n\t"
#define UNIT "v_fma_f32 %[t], %[s], %[sc], %[nm]\n\tv_exp_f32 %[xn], %[t]\n\t"
            if constexpr (V == 0) {
                asm volatile(MFN : OPS_W : OPS_R);
            } else if constexpr (V == 1) {
                if (g & 1) asm volatile(MFN UNIT "v_add_f32 %[acc], %[acc], %[xo]\n\tv_cvt_pk_bf16_f32 %[w], %[xo], %[acc]" : OPS_W : OPS_R);
                else asm volatile(MFN UNIT "v_add_f32 %[acc], %[acc], %[xo]" : OPS_W : OPS_R);
            } else if constexpr (V == 2) {
                if (g & 1) asm volatile(MFN UNIT "v_cvt_pk_bf16_f32 %[w], %[xo], %[acc]\n\tv_dot2_f32_bf16 %[acc], %[w], %[ones], %[acc]" : OPS_W : OPS_R);
                else asm volatile(MFN UNIT : OPS_W : OPS_R);
            } else if constexpr (V == 3) {
                if (g & 1) asm volatile(MFN UNIT "v_cvt_pk_bf16_f32 %[w], %[xo], %[acc]" : OPS_W : OPS_R);
                else asm volatile(MFN UNIT : OPS_W : OPS_R);
            } else {
                // V1's unit plus the variant's extra filler
                if (g & 1) asm volatile(MFN UNIT "v_add_f32 %[acc], %[acc], %[xo]\n\tv_cvt_pk_bf16_f32 %[w], %[xo], %[acc]" : OPS_W : OPS_R);
                else asm volatile(MFN UNIT "v_add_f32 %[acc], %[acc], %[xo]" : OPS_W : OPS_R);
                if constexpr (V == 4 || V == 6) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(mx) : "v"(s0), "v"(s1));
                // LDS reads as the kernel places them: phase 2's V^T reads two per gap in the first 4 gaps
                // of each 8-gap step, waited at the next step's start; phase 1's K reads two b128 every 4
                // gaps, waited 4 gaps later
                if constexpr (V == 5 || V == 6) {
                    if (g == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (g < 4) {
                        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(tr) : "v"(laddr), "i"(g * 4096 % 16384));
                        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(tr) : "v"(laddr), "i"((g * 4096 + 512) % 16384));
                    }
                }
                if constexpr (V == 8) {
                    asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(mx) : "v"(s0), "v"(s1));
                    if (g == 0) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
                    if (g == 1) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
                    if (g == 2) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
                    if (g == 3) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(tr) : "v"(laddr), "i"(g * 2048 % 16384));
                }
                if constexpr (V == 10 || V == 11) {
                    asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(mx) : "v"(s0), "v"(s1));
                    if (g == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    constexpr int per = V == 10 ? 8 : 4;
                    if (g * per < 8) {
#pragma unroll
                        for (int r = 0; r < per; ++r)
                            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(tr) : "v"(laddr), "i"((g * per + r) * 2048 % 16384));
                    }
                }
                if constexpr (V == 9) {
                    if ((g & 3) == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if ((g & 3) < 2) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kr) : "v"(laddr), "i"((g * 4096 + 8192 * (g & 1)) % 16384));
                }
                if constexpr (V == 7) {
                    if ((g & 3) == 0) {
                        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kr) : "v"(laddr), "i"(g * 4096 % 16384));
                        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kr) : "v"(laddr), "i"((g * 4096 + 8192) % 16384));
                    }
                }
            }
        }
    }
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = t1 - t0;
    const float keep = c0[0] + c1[1] + c2[2] + c3[3] + acc + x0 + x1 + t + (float)w + mx + (float)tr.x + (float)kr.y;
    if (keep == 12345.678f) out[1] = 1;  // keep everything live
}

int main() {
    unsigned long long *d, h[2];
    if (hipMalloc(&d, 16) != hipSuccess) return 1;
    const char *names[] = {"bare MFMA", "fma+exp+add (+cvt/2)", "fma+exp (+cvt+dot2)/2", "fma+exp (+cvt/2), no sum",
                           "V1 + max3", "V1 + V^T reads (1/gap)", "V1 + max3 + V^T reads", "V1 + K reads (0.5/gap)",
                           "V6, V^T reads spread", "V7, K reads spread", "V6, V^T reads 8 in gap 0",
                           "V6, V^T reads 4+4"};
    void (*kerns[])(unsigned long long *, float) = {probe<0>, probe<1>, probe<2>, probe<3>,
                                                    probe<4>, probe<5>, probe<6>, probe<7>, probe<8>, probe<9>, probe<10>, probe<11>};
    for (int rep = 0; rep < 3; ++rep) {
        for (int k = 0; k < 12; ++k) {
            for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(kerns[k], dim3(256), dim3(256), 0, 0, d, 0.5f);
            if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h, d, 16, hipMemcpyDeviceToHost) != hipSuccess) return 1;
            printf("rep %d V%d %-28s %7.2f cycles per MFMA gap\n", rep, k, names[k], (double)h[0] / (256.0 * 8.0));
        }
    }
    return 0;
}
