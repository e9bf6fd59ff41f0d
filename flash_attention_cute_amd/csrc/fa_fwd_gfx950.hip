// fa_fwd_gfx950.hip -- FlashAttention-2 forward for MI355X (gfx950 / CDNA4).
//
// Replaces, MI355X-first (not a translation):
//   reference csrc/flash_attention_template.cuh:138-564  flash_attention_v2 (CuTe, mma.sync, 4 warps)
//   reference csrc/mask.cuh:30-88                        Mask (OOB + bottom-right causal)
//   reference csrc/flash_attention_impl.cu:7-49          tile choice + 4 specialisations
//   reference csrc/kernel_dispatcher.h:20-52             dtype / headdim / causal dispatch
//
// Design (DESIGN.md section 3 has the numbers):
//   * one workgroup = 8 wave64s = 256 query rows of one (batch, q-head); each wave owns 32 rows;
//   * KV tiles of 64 keys are register-staged (global_load_dwordx4 issued one tile ahead)
//     into a double-buffered LDS ring (K and V, 16 KiB each per buffer, 64 KiB total);
//   * S^T = K . Q^T with v_mfma_f32_32x32x16_{f16,bf16}: A = K rows from LDS (ds_read_b128,
//     XOR-swizzled), B = Q^T held in VGPRs for the whole KV loop. Each lane then owns ONE query
//     and 32 of the tile's 64 keys, so the row max / row sum are in-lane plus a single
//     v_permlane32_swap (the reference needs a 4-lane shuffle butterfly, template.cuh:72-88);
//   * O^T += V^T . P^T with the same MFMA: the S^T accumulator, rounded to T, is directly the
//     B operand (no LDS round trip, no lane movement); V^T comes from ds_read_b64_tr_b16
//     transposed LDS reads of a row-major, XOR-swizzled V tile;
//   * O^T keeps the query on the lane, so the online-softmax rescale is a per-lane scalar;
//   * masking only on KV tiles that cross the causal diagonal or the Sk tail, and a wave skips
//     KV tiles that are fully masked for its 32 rows;
//   * workgroup ids are remapped so that the q-tiles of one kv-head group run on one XCD
//     (blocks b and b+8 share an XCD), keeping the K/V stream in that XCD's 4 MiB L2.
//
// Numerics follow the reference (Appendix A of SURVEY.md): S accumulated in fp32, max taken on
// unscaled S, P = exp2(S*s' - m*s') with s' = scale*log2(e) precomputed by the host, P rounded
// (RNE) to T before P.V, row sums of the fp32 P, O / l with l == 0 -> 1. Fully masked rows
// (causal with Sq > Sk) are defined as 0 (DESIGN.md "quirks").
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "fa_gfx950.h"

namespace fa {

constexpr int kBlockM = 256;      // query rows per workgroup
constexpr int kBlockN = 64;       // keys per KV tile
constexpr int kHeadDimPad = 128;  // head dim of the LDS image / MFMA k-steps (D <= 128, zero padded)
constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;
constexpr int kTileBytes = kBlockN * kHeadDimPad * 2;  // 16 KiB: one K or V tile
constexpr int kBufBytes = 2 * kTileBytes;              // K + V
constexpr int kLdsBytes = 2 * kBufBytes;               // double buffer, 64 KiB

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct F16 {
    static __device__ __forceinline__ f32x16 mfma(u32x4 a, u32x4 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                      __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    }
    // round-to-nearest-even pack of two fp32 into two fp16 (low element first)
    static __device__ __forceinline__ uint32_t pack(float lo, float hi) {
        f16x2 v = __builtin_convertvector((f32x2){lo, hi}, f16x2);
        return __builtin_bit_cast(uint32_t, v);
    }
};

struct BF16 {
    static __device__ __forceinline__ f32x16 mfma(u32x4 a, u32x4 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                       __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    }
    static __device__ __forceinline__ uint32_t pack(float lo, float hi) {
        bf16x2 v = __builtin_convertvector((f32x2){lo, hi}, bf16x2);
        return __builtin_bit_cast(uint32_t, v);
    }
};

// K tile image: 64 rows x 256 B; 16-B chunk c of row r lives at chunk slot c ^ (r & 15).
// The A-operand read (lane r reads row r, one chunk) then hits 16 distinct slots per
// ds_read_b128 lane group (groups cover rows {0-3,12-15,20-27} etc., distinct mod 16).
__device__ __forceinline__ int k_off(int row, int ch) { return row * 256 + 16 * (ch ^ (row & 15)); }
// V tile image: chunk slot c ^ ((r & 3) << 2). A ds_read_b64_tr_b16 half-wave reads 4 rows x
// 64 B; the XOR moves each of the 4 rows into a different 64-B quarter of the bank row.
__device__ __forceinline__ int v_off(int row, int ch) { return row * 256 + 16 * (ch ^ ((row & 3) << 2)); }

// v_permlane32_swap(vdst=x, src=x): the lower half-wave receives the upper half's x in the src
// result and keeps its own in vdst; the upper half the other way round. Combining both results
// therefore gives the (l, l^32) pair reduction with the same value in both lanes.
__device__ __forceinline__ float pair_max(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair_sum(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ u32x2 tr_read(const char *lds_ptr) {
    typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
    i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4 *)(lds_ptr));
    return __builtin_bit_cast(u32x2, v);
}

template <class DT, bool kCausal>
__global__ __launch_bounds__(kThreads) void fa_fwd_kernel(const fa_fwd_params p, const int n_qtiles) {
    __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31;
    const int h = lane >> 5;

    // ---- XCD-aware work decode ----------------------------------------------------------
    // Blocks are dealt round-robin over the 8 XCDs (b and b+8 share one). Remap so that each
    // XCD walks a contiguous range of the logical order (bijective for any grid size).
    const uint32_t nwg = gridDim.x;
    const uint32_t bid = blockIdx.x;
    const uint32_t xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const uint32_t w = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    // logical order: batch, q-head (members of one kv group adjacent), q-tile
    const uint32_t t = w % (uint32_t)n_qtiles;
    const uint32_t bh = w / (uint32_t)n_qtiles;
    const int64_t hq = bh % (uint32_t)p.num_heads_q;
    const int64_t b = bh / (uint32_t)p.num_heads_q;
    const int64_t qtile = kCausal ? (int64_t)(n_qtiles - 1 - t) : (int64_t)t;  // heavy first
    const int64_t hkv = hq / p.head_q_per_group;

    const int64_t Sq = p.seqlen_q, Sk = p.seqlen_kv, D = p.headdim;
    const float sc = p.softmax_scale;

    const char *qb = (const char *)p.q_ptr + 2 * (b * p.q_batch_stride + hq * p.q_head_stride);
    const char *kb = (const char *)p.k_ptr + 2 * (b * p.k_batch_stride + hkv * p.k_head_stride);
    const char *vb = (const char *)p.v_ptr + 2 * (b * p.v_batch_stride + hkv * p.v_head_stride);
    char *ob = (char *)p.o_ptr + 2 * (b * p.o_batch_stride + hq * p.o_head_stride);

    const int64_t m0 = qtile * kBlockM;        // first query row of the workgroup
    const int64_t mw = m0 + wave * 32;         // first query row of this wave
    const int64_t my_q = mw + r;               // this lane's query row
    const int64_t diag = Sk - Sq;              // bottom-right causal offset: key n visible iff n <= m + diag

    // ---- KV tile range ----------------------------------------------------------------
    const int64_t n_blocks = (Sk + kBlockN - 1) / kBlockN;
    int64_t n_end = n_blocks;
    if (kCausal) {
        // last valid query of the workgroup sees keys up to (min(m0+BM, Sq) - 1) + diag
        const int64_t x = diag + (m0 + kBlockM < Sq ? m0 + kBlockM : Sq);
        const int64_t nb = x <= 0 ? 0 : (x + kBlockN - 1) / kBlockN;
        n_end = nb < n_blocks ? nb : n_blocks;
    }

    // ---- Q fragments (B operand of S^T = K.Q^T), resident for the whole loop ----------
    // lane (h, r) holds Q[my_q][16*ks + 8*h + 0..7] for k-step ks
    u32x4 qf[8];
    {
        const bool q_ok = my_q < Sq;
        const char *qrow = qb + 2 * my_q * p.q_seqlen_stride;
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            const int d0 = 16 * ks + 8 * h;
            qf[ks] = (q_ok && d0 < D) ? *(const u32x4 *)(qrow + 2 * d0) : (u32x4){0, 0, 0, 0};
        }
    }

    // ---- register staging of K/V tiles ------------------------------------------------
    // thread t moves 16-B chunk (t & 15) of rows (t >> 4) and (t >> 4) + 32 of both K and V
    const int srow = tid >> 4;
    const int sch = tid & 15;
    const bool sch_ok = sch * 8 < D;
    u32x4 kst0, kst1, vst0, vst1;
    const u32x4 zero4 = {0, 0, 0, 0};

    auto stage_load = [&](int64_t j) {
        const int64_t key0 = j * kBlockN + srow;
        const int64_t key1 = key0 + 32;
        const bool ok0 = sch_ok && key0 < Sk;
        const bool ok1 = sch_ok && key1 < Sk;
        kst0 = ok0 ? *(const u32x4 *)(kb + 2 * (key0 * p.k_seqlen_stride + sch * 8)) : zero4;
        kst1 = ok1 ? *(const u32x4 *)(kb + 2 * (key1 * p.k_seqlen_stride + sch * 8)) : zero4;
        vst0 = ok0 ? *(const u32x4 *)(vb + 2 * (key0 * p.v_seqlen_stride + sch * 8)) : zero4;
        vst1 = ok1 ? *(const u32x4 *)(vb + 2 * (key1 * p.v_seqlen_stride + sch * 8)) : zero4;
    };
    auto stage_write = [&](int buf) {
        char *K = lds + buf * kBufBytes;
        char *V = K + kTileBytes;
        *(u32x4 *)(K + k_off(srow, sch)) = kst0;
        *(u32x4 *)(K + k_off(srow + 32, sch)) = kst1;
        *(u32x4 *)(V + v_off(srow, sch)) = vst0;
        *(u32x4 *)(V + v_off(srow + 32, sch)) = vst1;
    };

    // ---- per-lane constant LDS addresses ----------------------------------------------
    // K A-operand: row (kt*32 + r), chunk (2*ks + h)  -> offset k_off(r, 2ks+h) + kt*8192
    // V^T A-operand via ds_read_b64_tr_b16: lane = 16*g + 4*qq + pp supplies row (R + qq),
    // columns dt*32 + 16*(g&1) + 4*pp .. +3 where R = kt*32 + 16*s + 4*(g>>1) (+8 for the
    // second half of the fragment).
    const int g = lane >> 4;
    const int qq = (lane >> 2) & 3;
    const int pp = lane & 3;
    int v_addr[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
        const int row = 4 * (g >> 1) + qq;
        const int ch = dt * 4 + 2 * (g & 1) + (pp >> 1);
        v_addr[dt] = v_off(row, ch) + 8 * (pp & 1);
    }

    f32x16 o0 = {}, o1 = {}, o2 = {}, o3 = {};
    float m_run = -INFINITY;
    float l_run = 0.f;

    if (n_end > 0) {
        stage_load(0);
        stage_write(0);
        if (n_end > 1) stage_load(1);
    }
    __syncthreads();

    for (int64_t j = 0; j < n_end; ++j) {
        const int buf = (int)(j & 1);
        const char *K = lds + buf * kBufBytes;
        const char *V = K + kTileBytes;
        const int64_t key0 = j * kBlockN;

        bool wave_active = true;
        bool need_mask = key0 + kBlockN > Sk;
        if (kCausal) {
            wave_active = key0 <= mw + 31 + diag;           // some key visible to the wave's last row
            need_mask = need_mask || (key0 + kBlockN - 1 > mw + diag);  // some key hidden from its first row
        }

        if (wave_active) {
            // ---- S^T = K . Q^T : two 32-key sub-tiles ---------------------------------
            f32x16 s0 = {}, s1 = {};
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                const u32x4 a0 = *(const u32x4 *)(K + k_off(r, 2 * ks + h));
                const u32x4 a1 = *(const u32x4 *)(K + 8192 + k_off(r, 2 * ks + h));
                s0 = DT::mfma(a0, qf[ks], s0);
                s1 = DT::mfma(a1, qf[ks], s1);
            }

            // ---- mask (only tiles crossing the diagonal or the Sk tail) --------------
            if (need_mask) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int64_t kk0 = key0 + (i & 3) + 8 * (i >> 2) + 4 * h;
                    const int64_t kk1 = kk0 + 32;
                    bool m0k = kk0 >= Sk, m1k = kk1 >= Sk;
                    if (kCausal) {
                        m0k = m0k || (kk0 > my_q + diag);
                        m1k = m1k || (kk1 > my_q + diag);
                    }
                    if (m0k) s0[i] = -INFINITY;
                    if (m1k) s1[i] = -INFINITY;
                }
            }

            // ---- online softmax (per lane = per query row) -----------------------------
            float mx = fmaxf(s0[0], s1[0]);
#pragma unroll
            for (int i = 1; i < 16; ++i) mx = fmaxf(mx, fmaxf(s0[i], s1[i]));
            mx = pair_max(mx);
            const float m_new = fmaxf(m_run, mx);
            const float m_sc = (m_new == -INFINITY) ? 0.f : m_new * sc;
            const float alpha = __builtin_amdgcn_exp2f(m_run * sc - m_sc);
            m_run = m_new;

            float ls = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                s0[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(s0[i], sc, -m_sc));
                s1[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(s1[i], sc, -m_sc));
                ls += s0[i] + s1[i];
            }
            l_run = l_run * alpha + ls;

            if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    o0[i] *= alpha;
                    o1[i] *= alpha;
                    o2[i] *= alpha;
                    o3[i] *= alpha;
                }
            }

            // ---- P (rounded to T) as the B operand: k-step kk = (kt, s) -> regs 8s..8s+7
            u32x4 pf[4];
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                pf[s] = (u32x4){DT::pack(s0[8 * s + 0], s0[8 * s + 1]), DT::pack(s0[8 * s + 2], s0[8 * s + 3]),
                                DT::pack(s0[8 * s + 4], s0[8 * s + 5]), DT::pack(s0[8 * s + 6], s0[8 * s + 7])};
                pf[2 + s] = (u32x4){DT::pack(s1[8 * s + 0], s1[8 * s + 1]), DT::pack(s1[8 * s + 2], s1[8 * s + 3]),
                                    DT::pack(s1[8 * s + 4], s1[8 * s + 5]), DT::pack(s1[8 * s + 6], s1[8 * s + 7])};
            }

            // ---- O^T += V^T . P^T ------------------------------------------------------
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {
                const int rowoff = (kk >> 1) * 32 * 256 + (kk & 1) * 16 * 256;  // kt*32 + 16*s rows
                u32x4 a[4];
#pragma unroll
                for (int dt = 0; dt < 4; ++dt) {
                    const u32x2 lo = tr_read(V + rowoff + v_addr[dt]);
                    const u32x2 hi = tr_read(V + rowoff + 8 * 256 + v_addr[dt]);
                    a[dt] = (u32x4){lo[0], lo[1], hi[0], hi[1]};
                }
                o0 = DT::mfma(a[0], pf[kk], o0);
                o1 = DT::mfma(a[1], pf[kk], o1);
                o2 = DT::mfma(a[2], pf[kk], o2);
                o3 = DT::mfma(a[3], pf[kk], o3);
            }
        }

        if (j + 1 < n_end) stage_write(buf ^ 1);
        __syncthreads();
        if (j + 2 < n_end) stage_load(j + 2);
    }

    // ---- epilogue: O = O^T / l, row per lane, 16-B stores after a half-wave swap ----------
    const float l_tot = pair_sum(l_run);
    const float inv = (l_tot == 0.f) ? 1.f : 1.f / l_tot;
    const bool q_ok = my_q < Sq;
    char *orow = ob + 2 * my_q * p.o_seqlen_stride;
    auto store_tile = [&](const f32x16 &o, int dt) {
#pragma unroll
        for (int gp = 0; gp < 4; gp += 2) {
            // this lane holds d = dt*32 + 8*grp + 4*h + 0..3 in o[4*grp .. 4*grp+3]
            uint32_t a0 = DT::pack(o[4 * gp + 0] * inv, o[4 * gp + 1] * inv);
            uint32_t a1 = DT::pack(o[4 * gp + 2] * inv, o[4 * gp + 3] * inv);
            uint32_t b0 = DT::pack(o[4 * gp + 4] * inv, o[4 * gp + 5] * inv);
            uint32_t b1 = DT::pack(o[4 * gp + 6] * inv, o[4 * gp + 7] * inv);
            auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
            auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
            // lower half: d = dt*32 + 8*gp + 0..7 ; upper half: d = dt*32 + 8*(gp+1) + 0..7
            const int d0 = dt * 32 + 8 * (gp + h);
            if (q_ok && d0 < D) *(u32x4 *)(orow + 2 * d0) = (u32x4){x0[0], x1[0], x0[1], x1[1]};
        }
    };
    store_tile(o0, 0);
    store_tile(o1, 1);
    store_tile(o2, 2);
    store_tile(o3, 3);
}

}  // namespace fa

// ============================================================================================
// C-ABI (include/fa_gfx950.h)
// ============================================================================================
namespace {

thread_local char g_err[512] = "";

int set_err(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int set_err(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

bool aligned16(const void *ptr) { return ((uintptr_t)ptr & 15) == 0; }

int check_params(const fa_fwd_params *p, int dtype, int causal) {
    (void)causal;
    if (!p) return set_err(FA_ERR_INVALID_ARGUMENT, "params is NULL");
    if (dtype != FA_DTYPE_F16 && dtype != FA_DTYPE_BF16)
        return set_err(FA_ERR_UNSUPPORTED, "No suitable implementation for flash attention kernel (dtype %d)", dtype);
    if (!p->q_ptr || !p->k_ptr || !p->v_ptr || !p->o_ptr)
        return set_err(FA_ERR_INVALID_ARGUMENT, "q, k, v, o pointers must be non-NULL");
    if (p->batch_size <= 0 || p->num_heads_q <= 0 || p->num_heads_kv <= 0 || p->seqlen_q <= 0 ||
        p->seqlen_kv <= 0 || p->headdim <= 0)
        return set_err(FA_ERR_INVALID_ARGUMENT, "q, k, v must have at least one element");
    if (p->headdim % 8 != 0) return set_err(FA_ERR_INVALID_ARGUMENT, "hidden dimension must be multiple of 8");
    if (p->headdim > 128)
        return set_err(FA_ERR_UNSUPPORTED, "only support hidden dimension <= 128");
    if (p->head_q_per_group <= 0 || p->num_heads_q != p->num_heads_kv * p->head_q_per_group)
        return set_err(FA_ERR_INVALID_ARGUMENT,
                       "num_heads_q (%lld) must equal num_heads_kv (%lld) * head_q_per_group (%lld)",
                       (long long)p->num_heads_q, (long long)p->num_heads_kv, (long long)p->head_q_per_group);
    if (!aligned16(p->q_ptr) || !aligned16(p->k_ptr) || !aligned16(p->v_ptr) || !aligned16(p->o_ptr))
        return set_err(FA_ERR_INVALID_ARGUMENT, "q, k, v, o base pointers must be 16-byte aligned");
    const int64_t strides[12] = {p->q_batch_stride, p->k_batch_stride, p->v_batch_stride, p->o_batch_stride,
                                 p->q_head_stride,  p->k_head_stride,  p->v_head_stride,  p->o_head_stride,
                                 p->q_seqlen_stride, p->k_seqlen_stride, p->v_seqlen_stride, p->o_seqlen_stride};
    for (int i = 0; i < 12; ++i)
        if (strides[i] % 8 != 0)
            return set_err(FA_ERR_INVALID_ARGUMENT, "strides must be multiples of 8 elements (16 bytes)");
    const int64_t n_qtiles = (p->seqlen_q + fa::kBlockM - 1) / fa::kBlockM;
    const int64_t nwg = n_qtiles * p->num_heads_q * p->batch_size;
    if (nwg > 0x7fffffffLL) return set_err(FA_ERR_UNSUPPORTED, "grid too large (%lld workgroups)", (long long)nwg);
    g_err[0] = 0;
    return FA_OK;
}

template <class DT, bool C>
int launch(const fa_fwd_params &p, hipStream_t stream) {
    const int64_t n_qtiles = (p.seqlen_q + fa::kBlockM - 1) / fa::kBlockM;
    const int64_t nwg = n_qtiles * p.num_heads_q * p.batch_size;
    hipLaunchKernelGGL((fa::fa_fwd_kernel<DT, C>), dim3((uint32_t)nwg), dim3(fa::kThreads), 0, stream, p,
                       (int)n_qtiles);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(FA_ERR_LAUNCH, "HIP launch failed: %s", hipGetErrorString(e));
    return FA_OK;
}

}  // namespace

extern "C" int fa_fwd_gfx950_check(const fa_fwd_params *params, int dtype, int causal) {
    return check_params(params, dtype, causal);
}

extern "C" int fa_fwd_gfx950(const fa_fwd_params *params, int dtype, int causal, void *stream) {
    const int rc = check_params(params, dtype, causal);
    if (rc != FA_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (dtype == FA_DTYPE_F16)
        return causal ? launch<fa::F16, true>(*params, s) : launch<fa::F16, false>(*params, s);
    return causal ? launch<fa::BF16, true>(*params, s) : launch<fa::BF16, false>(*params, s);
}

extern "C" const char *fa_last_error(void) { return g_err; }

extern "C" int fa_abi_version(void) { return FA_GFX950_ABI_VERSION; }

extern "C" int fa_fwd_gfx950_geometry(const fa_fwd_params *params, int causal, int64_t *block_m,
                                      int64_t *block_n, int64_t *threads, int64_t *workgroups) {
    (void)causal;
    if (!params) return set_err(FA_ERR_INVALID_ARGUMENT, "params is NULL");
    const int64_t n_qtiles = (params->seqlen_q + fa::kBlockM - 1) / fa::kBlockM;
    if (block_m) *block_m = fa::kBlockM;
    if (block_n) *block_n = fa::kBlockN;
    if (threads) *threads = fa::kThreads;
    if (workgroups) *workgroups = n_qtiles * params->num_heads_q * params->batch_size;
    return FA_OK;
}
