// mfma_shape.hip -- measured A/B of the two bf16/f16 MFMA shapes for the attention tile loop
// (SURVEY.md section 7 hard part 1). Standalone; not part of the product.
//
// One wave per SIMD (256-thread workgroups, one per CU, persistent), random operands in registers
// (no memory traffic in the loop), the same work per KV tile as one fa_fwd_w4 wave: 64 queries x
// 64 keys x D = 128, i.e. S^T = K.Q^T then O^T += V^T.P^T (2 * 524288 MACs), plus the softmax VALU of
// the kernel per lane and tile: 64 x {fma (exp argument), v_exp_f32, add (row sum)}, 32 cvt_pk, 32
// max. Shapes:
//   32: v_mfma_f32_32x32x16_f16, 32 + 32 MFMAs per tile (32 cycles each), S 4 x f32x16 per lane
//   16: v_mfma_f32_16x16x32_f16, 64 + 64 MFMAs per tile (16 cycles each), S 16 x f32x4 per lane
// (the per-lane softmax work is the same in both shapes: each lane owns 64 scores of a tile; the
// 16x16 row max needs cross-lane steps only on the rare rescale, like the 32x32 one.)
// Modes: 0 = MFMAs only, 1 = MFMAs + softmax VALU interleaved evenly (one unit per gap group),
// 2 = as 1 without the exp-argument fma (what folding the scale / max into the MFMA would save),
// 3 = as 2 without the row-sum add as well; 4 = mode 1's VALU as one block between the MFMA phases.
// W8 rows: two waves per SIMD (512-thread workgroups), each with HALF the rows (32 queries per
// wave: 16 + 16 MFMAs and 32 softmax units per tile), waves 4-7 one phase behind waves 0-3: the
// same work per SIMD as one W4 wave, to see whether two waves interleave the VALU with the MFMAs
// better than one (a single wave issues a VALU op every 4 cycles at most; the SIMD every 2).
// Prints TFLOP/s (MFMA FLOPs), cycles per tile and the in-kernel clock, per shape and mode,
// interleaved repetitions on one device.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<N, I + 1>(f);
    }
}
#define FENCE() __builtin_amdgcn_sched_barrier(0)
__device__ __forceinline__ void pin(float &x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(uint32_t &x) { asm volatile("" : "+v"(x)); }

template <bool kFirst>
__device__ __forceinline__ void mfma32(f32x16 &c, const u32x4 &a, const u32x4 &b) {
    if constexpr (kFirst) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "v"(b));
    else asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
template <bool kFirst>
__device__ __forceinline__ void mfma16(f32x4 &c, const u32x4 &a, const u32x4 &b) {
    if constexpr (kFirst) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(c) : "v"(a), "v"(b));
    else asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma32a(f32x16 &c, const u32x4 &a, const u32x4 &b) {
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma16a(f32x4 &c, const u32x4 &a, const u32x4 &b) {
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ uint32_t pack(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){lo, hi}, f16x2));
}

// the softmax work of one score slot u (0..63): fma + exp + row-sum add; every 2nd: cvt_pk + max
struct Sm {
    float sc, msc, l, mx;
};

template <int SHAPE, int MODE, int WAVES = 4>
__global__ __launch_bounds__(64 * WAVES, 1) void tile_loop(const int tiles, const uint32_t *seed, float *sink,
                                                           unsigned long long *clk) {
    const int lane = threadIdx.x & 63;
    const uint32_t s0 = seed[(blockIdx.x * 512 + threadIdx.x) & 0xffff];
    constexpr int HALF = WAVES == 8 ? 2 : 1;  // rows per wave: 64 / HALF
    // operand fragments: random fp16 in (-1, 1) (random data: the clock the chip holds depends on the
    // operand values, MI355X_MICROARCH 'DVFS give-back'); S = K.Q^T then has a std of ~2 (D = 128)
    u32x4 kf[4], qf[4], vf[4];
    uint32_t hs = s0 | 1u;
    auto rnd = [&]() {
        hs ^= hs << 13; hs ^= hs >> 17; hs ^= hs << 5;
        const float a = (float)(hs & 0xffff) / 32768.f - 1.f, b = (float)(hs >> 16) / 32768.f - 1.f;
        return pack(a, b);
    };
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        kf[i] = (u32x4){rnd(), rnd(), rnd(), rnd()};
        qf[i] = (u32x4){rnd(), rnd(), rnd(), rnd()};
        vf[i] = (u32x4){rnd(), rnd(), rnd(), rnd()};
    }
    constexpr int NS = (SHAPE == 32 ? 4 : 16) / HALF;   // S accumulators per lane (64 floats)
    constexpr int NO = (SHAPE == 32 ? 8 : 32) / HALF;   // O accumulators per lane (128 floats)
    constexpr int NU = 32 / HALF;                       // softmax units per phase
    typedef typename std::conditional<SHAPE == 32, f32x16, f32x4>::type acc_t;
    constexpr int AL = SHAPE == 32 ? 16 : 4;
    acc_t S[2][NS], O[NO];
    uint32_t P[32 / HALF];
#pragma unroll
    for (int i = 0; i < NS; ++i) { S[0][i] = (acc_t){}; S[1][i] = (acc_t){}; }
#pragma unroll
    for (int i = 0; i < NO; ++i) O[i] = (acc_t){};
#pragma unroll
    for (int i = 0; i < 32 / HALF; ++i) P[i] = s0 + i;
    Sm st{1.0f, 0.5f, 0.f, -1e30f};  // exp2 arguments ~ N(-0.5, 2): P in a realistic range
    constexpr int G = (SHAPE == 32 ? 32 : 64) / HALF;   // MFMAs per phase
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();

    auto ph1 = [&](auto PAR) {
        constexpr int c = decltype(PAR)::value, pc = c ^ 1;
        // phase 1: S[c] = K.Q^T (G MFMAs) || softmax units 0..31 of S[pc]
        static_for<G>([&](auto GG) {
            constexpr int g = decltype(GG)::value;
            // S[c][i] accumulates over D: the first k-step of each accumulator starts from C = 0
            if constexpr (SHAPE == 32) mfma32<(g < NS)>(S[c][g % NS], kf[g & 3], qf[(g >> 2) & 3]);
            else mfma16<(g < NS)>(S[c][g % NS], kf[g & 3], qf[(g >> 2) & 3]);
            FENCE();
            if constexpr (MODE >= 1 && MODE <= 3) {
                static_for<NU>([&](auto UU) {
                    constexpr int u = decltype(UU)::value;
                    if constexpr ((u * G) / NU == g) {
                        float e = (MODE >= 2 && MODE <= 3) ? __builtin_amdgcn_exp2f(S[pc][u / AL][u % AL])
                                            : __builtin_amdgcn_exp2f(__builtin_fmaf(S[pc][u / AL][u % AL], st.sc, -st.msc));
                        pin(e);
                        if constexpr (MODE <= 2 || MODE == 4) {
                            st.l += e;
                            pin(st.l);
                        }
                        S[pc][u / AL][u % AL] = e;
                        if constexpr (u & 1) {
                            uint32_t w = pack(S[pc][(u - 1) / AL][(u - 1) % AL], e);
                            pin(w);
                            P[(u >> 1) % (32 / HALF)] = w;
                            st.mx = fmaxf(st.mx, fmaxf(S[c ^ 1][(u - 1) / AL][(u - 1) % AL], e));
                            pin(st.mx);
                        }
                    }
                });
            }
            FENCE();
        });
    };
    auto ph2 = [&](auto PAR) {
        constexpr int c = decltype(PAR)::value, pc = c ^ 1;
        // phase 2: O += V.P (G MFMAs) || softmax units 32..63 of S[pc]
        static_for<G>([&](auto GG) {
            constexpr int g = decltype(GG)::value;
            constexpr int NP_ = 32 / HALF;
            u32x4 pb = (u32x4){P[(4 * g) % NP_], P[(4 * g + 1) % NP_], P[(4 * g + 2) % NP_], P[(4 * g + 3) % NP_]};
            if constexpr (SHAPE == 32) mfma32a(O[g % NO], vf[g & 3], pb);
            else mfma16a(O[g % NO], vf[g & 3], pb);
            FENCE();
            if constexpr (MODE >= 1 && MODE <= 3) {
                static_for<NU>([&](auto UU) {
                    constexpr int u = NU + decltype(UU)::value;
                    if constexpr (((u - NU) * G) / NU == g) {
                        float e = (MODE >= 2 && MODE <= 3) ? __builtin_amdgcn_exp2f(S[pc][u / AL][u % AL])
                                            : __builtin_amdgcn_exp2f(__builtin_fmaf(S[pc][u / AL][u % AL], st.sc, -st.msc));
                        pin(e);
                        if constexpr (MODE <= 2 || MODE == 4) {
                            st.l += e;
                            pin(st.l);
                        }
                        S[pc][u / AL][u % AL] = e;
                        if constexpr (u & 1) {
                            uint32_t w = pack(S[pc][(u - 1) / AL][(u - 1) % AL], e);
                            pin(w);
                            P[(u >> 1) % (32 / HALF)] = w;
                            st.mx = fmaxf(st.mx, fmaxf(S[c ^ 1][(u - 1) / AL][(u - 1) % AL], e));
                            pin(st.mx);
                        }
                    }
                });
            }
            FENCE();
        });
    };
    // MODE 4: the same units as MODE 1, but as one VALU block between the two MFMA phases (no
    // interleaving inside a wave: with two waves per SIMD the partner's MFMAs fill the block)
    auto smblock = [&](auto PAR) {
        constexpr int c = decltype(PAR)::value, pc = c ^ 1;
        static_for<2 * NU>([&](auto UU) {
            constexpr int u = decltype(UU)::value;
            float e = __builtin_amdgcn_exp2f(__builtin_fmaf(S[pc][u / AL][u % AL], st.sc, -st.msc));
            pin(e);
            st.l += e;
            pin(st.l);
            S[pc][u / AL][u % AL] = e;
            if constexpr (u & 1) {
                uint32_t w = pack(S[pc][(u - 1) / AL][(u - 1) % AL], e);
                pin(w);
                P[(u >> 1) % (32 / HALF)] = w;
                st.mx = fmaxf(st.mx, fmaxf(S[c ^ 1][(u - 1) / AL][(u - 1) % AL], e));
                pin(st.mx);
            }
        });
    };
    if (WAVES == 8 && threadIdx.x >= 256) ph2(std::integral_constant<int, 1>{});  // stagger: one phase behind
    for (int t = 0; t < tiles; t += 2) {
        ph1(std::integral_constant<int, 0>{});
        if constexpr (MODE == 4) smblock(std::integral_constant<int, 0>{});
        ph2(std::integral_constant<int, 0>{});
        ph1(std::integral_constant<int, 1>{});
        if constexpr (MODE == 4) smblock(std::integral_constant<int, 1>{});
        ph2(std::integral_constant<int, 1>{});
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float acc = st.l + st.mx;
#pragma unroll
    for (int i = 0; i < NO; ++i)
#pragma unroll
        for (int j = 0; j < AL; ++j) acc += O[i][j];
#pragma unroll
    for (int i = 0; i < NS; ++i)
#pragma unroll
        for (int j = 0; j < AL; ++j) acc += S[0][i][j] + S[1][i][j];
    sink[blockIdx.x * 512 + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char **argv) {
    const int tiles = argc > 1 ? atoi(argv[1]) : 4096;
    const int reps = argc > 2 ? atoi(argv[2]) : 7;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int nwg = ncu;
    uint32_t *seed;
    float *sink;
    unsigned long long *clk;
    CK(hipMalloc(&seed, 65536 * 4));
    CK(hipMalloc(&sink, nwg * 512 * 4));
    CK(hipMalloc(&clk, nwg * 16));
    std::vector<uint32_t> h(65536);
    uint32_t x = 12345;
    for (auto &v : h) { x = x * 1664525u + 1013904223u; v = x; }
    CK(hipMemcpy(seed, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    typedef void (*K)(int, const uint32_t *, float *, unsigned long long *);
    constexpr int NK = 14;
    const K ks[NK] = {tile_loop<32, 0>, tile_loop<32, 1>, tile_loop<32, 2>, tile_loop<32, 3>,
                      tile_loop<16, 0>, tile_loop<16, 1>, tile_loop<16, 2>, tile_loop<16, 3>,
                      tile_loop<32, 0, 8>, tile_loop<32, 1, 8>, tile_loop<16, 0, 8>, tile_loop<16, 1, 8>,
                      tile_loop<32, 4, 4>, tile_loop<32, 4, 8>};
    const int waves[NK] = {4, 4, 4, 4, 4, 4, 4, 4, 8, 8, 8, 8, 4, 8};
    const char *names[NK] = {"32x32x16 MFMA only", "32x32x16 + softmax VALU", "32x32x16 softmax -fma",
                             "32x32x16 softmax -fma -add", "16x16x32 MFMA only", "16x16x32 + softmax VALU",
                             "16x16x32 softmax -fma", "16x16x32 softmax -fma -add", "W8 32x32x16 MFMA only",
                             "W8 32x32x16 + softmax", "W8 16x16x32 MFMA only", "W8 16x16x32 + softmax",
                             "32x32x16 softmax block", "W8 32x32x16 softmax block"};
    const double flop_per_tile = 2.0 * 2 * 64 * 64 * 128;  // S and P.V per wave
    std::vector<std::vector<double>> tf(NK), cyc(NK), ghz(NK);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    // warm-up: ~2 s of launches (the clock settles, MI355X_MICROARCH 'DVFS give-back')
    for (int w = 0; w < 8; ++w)
        for (int k = 0; k < NK; ++k) hipLaunchKernelGGL(ks[k], dim3(nwg), dim3(64 * waves[k]), 0, 0, tiles, seed, sink, clk);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> hc(nwg * 2);
    for (int r = 0; r < reps; ++r)
        for (int k = 0; k < NK; ++k) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(ks[k], dim3(nwg), dim3(64 * waves[k]), 0, 0, tiles, seed, sink, clk);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            CK(hipMemcpy(hc.data(), clk, nwg * 16, hipMemcpyDeviceToHost));
            std::vector<double> cy, gh;
            for (int i = 0; i < nwg; ++i) {
                cy.push_back((double)hc[2 * i] / tiles);
                gh.push_back((double)hc[2 * i] / (double)hc[2 * i + 1] * 0.1);  // memrealtime = 100 MHz
            }
            std::sort(cy.begin(), cy.end());
            std::sort(gh.begin(), gh.end());
            // per SIMD and tile: 64 query rows either way (W8: two waves of 32 rows)
            tf[k].push_back(flop_per_tile * tiles * 4.0 * nwg / (ms * 1e-3) / 1e12);
            cyc[k].push_back(cy[nwg / 2]);
            ghz[k].push_back(gh[nwg / 2]);
        }
    printf("tiles %d, %d workgroups x 4 waves, %d interleaved repetitions (median)\n", tiles, nwg, reps);
    for (int k = 0; k < NK; ++k) {
        std::sort(tf[k].begin(), tf[k].end());
        std::sort(cyc[k].begin(), cyc[k].end());
        std::sort(ghz[k].begin(), ghz[k].end());
        printf("  %-26s %8.1f TFLOP/s  %7.1f cycles/tile  clock %.3f GHz  (TF min %.1f max %.1f)\n", names[k],
               tf[k][reps / 2], cyc[k][reps / 2], ghz[k][reps / 2], tf[k].front(), tf[k].back());
    }
    return 0;
}
