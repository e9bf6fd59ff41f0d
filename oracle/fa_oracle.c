/*
 * fa_oracle.c -- CPU restatement of the reference FlashAttention-2 forward, fp32 arithmetic.
 * TEST INFRASTRUCTURE ONLY: called by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg, never by the product path.
 *
 * Same algorithm as oracle/fa_oracle.py (mask="inf" convention), but with the kernel's own
 * arithmetic widths: S and O accumulated in fp32, P rounded to T (RNE) before P.V, 64-key blocks.
 * It follows:
 *   reference csrc/flash_attention_api.cpp:64-135      host: Sq==1 q-head pack, scale*log2(e)
 *   reference csrc/flash_attention_template.cuh:342-528 block loop, online softmax, epilogue
 *   reference csrc/mask.cuh:37-52                        OOB + bottom-right causal mask
 * Parallelised with OpenMP over (batch, q-head, 64-row q block) so it can serve as the CPU
 * baseline ("port") on the GPU box's host cores.
 *
 * Inputs are contiguous [B, H, S, D] arrays of 16-bit values (fp16 or bf16 bit patterns).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define BN 64
#define BM 64

static float h2f(uint16_t h) {
    const uint32_t s = (uint32_t)(h & 0x8000) << 16;
    const uint32_t e = (h >> 10) & 0x1f;
    uint32_t m = h & 0x3ff;
    uint32_t u;
    if (e == 0) {
        if (m == 0) {
            u = s;
        } else { /* subnormal */
            int ee = -1;
            do { ee++; m <<= 1; } while (!(m & 0x400));
            u = s | (uint32_t)(127 - 15 - ee) << 23 | (m & 0x3ff) << 13;
        }
    } else if (e == 31) {
        u = s | 0x7f800000u | m << 13;
    } else {
        u = s | (e + 112) << 23 | m << 13;
    }
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static uint16_t f2h(float f) { /* RNE, as v_cvt_f16_f32 */
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000;
    const uint32_t ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t)(sign | 0x7c00 | (ax > 0x7f800000u ? 0x200 : 0));
    if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00); /* >= 65520 rounds to inf */
    if (ax < 0x38800000u) {                                  /* |f| < 2^-14: subnormal or zero */
        float a;
        memcpy(&a, &ax, 4);
        return (uint16_t)(sign | (uint32_t)nearbyintf(a * 16777216.0f));
    }
    const uint32_t mant = ax & 0x7fffff;
    uint32_t h = ((ax >> 23) - 112) << 10 | (mant >> 13);
    const uint32_t rem = mant & 0x1fff;
    if (rem > 0x1000 || (rem == 0x1000 && (h & 1))) h++;
    return (uint16_t)(sign | h);
}

static float b2f(uint16_t b) {
    uint32_t u = (uint32_t)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static uint16_t f2b(float f) { /* RNE */
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1)) >> 16);
}

static inline float to_f(uint16_t x, int dtype) { return dtype == 0 ? h2f(x) : b2f(x); }
static inline uint16_t from_f(float x, int dtype) { return dtype == 0 ? f2h(x) : f2b(x); }
static inline float round_t(float x, int dtype) { return to_f(from_f(x, dtype), dtype); }

/*
 * o[B,Hq,Sq,D] = attention(q[B,Hq,Sq,D], k[B,Hkv,Sk,D], v[B,Hkv,Sk,D]); softmax_scale is the user
 * scale (log2(e) is folded in here, as the host API does). dtype 0 = fp16, 1 = bf16.
 * o32 (optional) receives the unrounded fp32 output. Returns 0, or -1 on invalid shapes.
 */
/*
 * window_left >= 0: key n is also masked for query m when n < m + Sk - Sq - window_left (the local
 * window of include/fa_gfx950.h fa_fwd_gfx950_window; the reference has no such mask, so this part
 * follows transformers' sliding_window_causal_mask_function with sliding_window = window_left + 1).
 * With Sq == 1 every packed q-head row is the one query at position Sk - 1.
 */
int fa_oracle_fwd_window(const uint16_t *q, const uint16_t *k, const uint16_t *v, uint16_t *o, float *o32,
                         int64_t B, int64_t Hq, int64_t Hkv, int64_t Sq, int64_t Sk, int64_t D, float softmax_scale,
                         int causal, int dtype, int threads, int64_t window_left) {
    if (B <= 0 || Hq <= 0 || Hkv <= 0 || Sq <= 0 || Sk <= 0 || D <= 0 || Hq % Hkv) return -1;
    const int64_t group = Hq / Hkv;
    const float s2 = (float)((double)softmax_scale * 1.4426950408889634);
    /* decode q-head packing (reference csrc/flash_attention_api.cpp:72-83) */
    int64_t hq_eff = Hq, sq_eff = Sq, g_eff = group;
    if (Sq == 1) {
        hq_eff = Hkv;
        sq_eff = group;
        g_eff = 1;
        causal = 0;
    }
    const int64_t n_qb = (sq_eff + BM - 1) / BM;
    const int64_t n_items = B * hq_eff * n_qb;
    const int64_t diag = Sk - sq_eff;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel
#endif
    {
        float *qs = (float *)malloc(sizeof(float) * BM * D);
        float *ks = (float *)malloc(sizeof(float) * BN * D);
        float *vs = (float *)malloc(sizeof(float) * BN * D);
        float *acc = (float *)malloc(sizeof(float) * BM * D);
        float s[BM][BN];
        float m[BM], l[BM];
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t it = 0; it < n_items; ++it) {
            const int64_t qb = it % n_qb;
            const int64_t h = (it / n_qb) % hq_eff;
            const int64_t b = it / (n_qb * hq_eff);
            const int64_t hk = h / g_eff;
            const int64_t r0 = qb * BM;
            const int64_t nr = (sq_eff - r0) < BM ? (sq_eff - r0) : BM;
            const uint16_t *qh = q + ((b * hq_eff + h) * sq_eff) * D;
            const uint16_t *kh = k + ((b * Hkv + hk) * Sk) * D;
            const uint16_t *vh = v + ((b * Hkv + hk) * Sk) * D;
            for (int64_t r = 0; r < nr; ++r)
                for (int64_t d = 0; d < D; ++d) qs[r * D + d] = to_f(qh[(r0 + r) * D + d], dtype);
            for (int64_t r = 0; r < nr; ++r) {
                m[r] = -INFINITY;
                l[r] = 0.f;
            }
            memset(acc, 0, sizeof(float) * BM * D);
            const int64_t n_blocks = (Sk + BN - 1) / BN;
            for (int64_t j = 0; j < n_blocks; ++j) {
                const int64_t c0 = j * BN;
                const int64_t nc = (Sk - c0) < BN ? (Sk - c0) : BN;
                if (causal && c0 > r0 + nr - 1 + diag) break; /* fully masked for every row */
                for (int64_t c = 0; c < nc; ++c)
                    for (int64_t d = 0; d < D; ++d) {
                        ks[c * D + d] = to_f(kh[(c0 + c) * D + d], dtype);
                        vs[c * D + d] = to_f(vh[(c0 + c) * D + d], dtype);
                    }
                for (int64_t r = 0; r < nr; ++r) {
                    const float *qr = qs + r * D;
                    float mx = -INFINITY;
                    for (int64_t c = 0; c < BN; ++c) {
                        float sv = -INFINITY;
                        int visible = c < nc && (!causal || c0 + c <= r0 + r + diag);
                        if (window_left >= 0)
                            visible = visible && c0 + c >= (Sq == 1 ? Sk - 1 : r0 + r + diag) - window_left;
                        if (visible) {
                            const float *kr = ks + c * D;
                            float a = 0.f;
#pragma omp simd reduction(+ : a)
                            for (int64_t d = 0; d < D; ++d) a += qr[d] * kr[d];
                            sv = a;
                        }
                        s[r][c] = sv;
                        mx = sv > mx ? sv : mx;
                    }
                    const float m_new = m[r] > mx ? m[r] : mx;
                    const float m_sc = m_new == -INFINITY ? 0.f : m_new * s2;
                    const float alpha = exp2f(m[r] * s2 - m_sc);
                    m[r] = m_new;
                    float ls = 0.f;
                    float *ar = acc + r * D;
                    for (int64_t d = 0; d < D; ++d) ar[d] *= alpha;
                    for (int64_t c = 0; c < nc; ++c) {
                        const float p = exp2f(s[r][c] * s2 - m_sc);
                        ls += p;
                        const float pt = round_t(p, dtype);
                        if (pt != 0.f) {
                            const float *vr = vs + c * D;
#pragma omp simd
                            for (int64_t d = 0; d < D; ++d) ar[d] += pt * vr[d];
                        }
                    }
                    l[r] = l[r] * alpha + ls;
                }
            }
            uint16_t *oh = o + ((b * hq_eff + h) * sq_eff) * D;
            for (int64_t r = 0; r < nr; ++r) {
                const float inv = l[r] == 0.f ? 1.f : 1.f / l[r];
                for (int64_t d = 0; d < D; ++d) {
                    const float x = acc[r * D + d] * inv;
                    oh[(r0 + r) * D + d] = from_f(x, dtype);
                    if (o32) o32[((b * hq_eff + h) * sq_eff + r0 + r) * D + d] = x;
                }
            }
        }
        free(qs);
        free(ks);
        free(vs);
        free(acc);
    }
    return 0;
}

int fa_oracle_fwd(const uint16_t *q, const uint16_t *k, const uint16_t *v, uint16_t *o, float *o32, int64_t B,
                  int64_t Hq, int64_t Hkv, int64_t Sq, int64_t Sk, int64_t D, float softmax_scale, int causal,
                  int dtype, int threads) {
    return fa_oracle_fwd_window(q, k, v, o, o32, B, Hq, Hkv, Sq, Sk, D, softmax_scale, causal, dtype, threads, -1);
}

int fa_oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
