#pragma once
// fa_fwd_kernels.hpp -- FlashAttention-2 forward kernels for MI355X (gfx950 / CDNA4).
//
// Device code only. Each (dtype, causal, head-dim tile, exact-D) combination is instantiated in
// its own translation unit (fa_inst.hip, compiled once per combination by _build.py, in
// parallel); fa_fwd_gfx950.hip holds the C-ABI and the runtime dispatch.
//
// Replaces, MI355X-first (not a translation):
//   reference csrc/flash_attention_template.cuh:138-564  flash_attention_v2 (CuTe, mma.sync, 4 warps)
//   reference csrc/mask.cuh:30-88                        Mask (OOB + bottom-right causal)
//   reference csrc/flash_attention_impl.cu:7-49          tile choice + 4 specialisations
//   reference csrc/kernel_dispatcher.h:20-52             dtype / headdim / causal dispatch
//
// Two prefill kernels (DESIGN.md section 4 has the numbers):
//   * fa_fwd_w4 (default): persistent grid, one workgroup per CU walking Q blocks of 256 query rows
//     of one (batch, q-head); 4 wave64s, one per SIMD, each owning 64 rows (two 32-row blocks,
//     one in each half of the Q block, so the last causal diagonal tiles run one block only)
//     with the whole 512-register file: O^T and the Q fragments in literal AGPRs (fa_agpr_asm.inc),
//     K/V tiles of 64 keys by LDS-DMA into 2-slot rings, a two-phase software pipeline per tile
//     (S = K.Q^T beside the previous tile's softmax tail; O += P.V beside this tile's max, rescale
//     decision and first exps) with every MFMA issued alone between hand-placed softmax units;
//   * fa_fwd_w8 (FA_GFX950_VARIANT=w8, cross-check): 8 wave64s x 32 rows, register-staged K/V.
// Both:
//   * S^T = K . Q^T with v_mfma_f32_32x32x16_{f16,bf16}: A = K rows from LDS (ds_read_b128,
//     XOR-swizzled), B = Q^T. Each lane then owns ONE query and 32 of the tile's 64 keys, so the
//     row max / row sum are in-lane plus a single v_permlane32_swap (the reference needs a 4-lane
//     shuffle butterfly, template.cuh:72-88);
//   * O^T += V^T . P^T with the same MFMA: the S^T accumulator, rounded to T, is directly the
//     B operand (no LDS round trip, no lane movement); V^T comes from ds_read_b64_tr_b16
//     transposed LDS reads of a row-major, XOR-swizzled V tile;
//   * O^T keeps the query on the lane, so the online-softmax rescale is a per-lane scalar;
//   * masking only on KV tiles that cross the causal diagonal or the Sk tail;
//   * Q blocks are ordered so that the q-tiles of one kv-head group run on one XCD (blocks b and
//     b+8 share an XCD), keeping the K/V stream in that XCD's 4 MiB L2; causal orders heavy-first.
//
// Numerics follow the reference (Appendix A of SURVEY.md): S accumulated in fp32, max taken on
// unscaled S, P = exp2(S*s' - m*s') with s' = scale*log2(e) precomputed by the host, P rounded
// (RNE) to T before P.V, row sums of the fp32 P, O / l with l == 0 -> 1. Fully masked rows
// (causal with Sq > Sk) are defined as 0 (DESIGN.md "quirks").
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fa_gfx950.h"
#include "fa_launch.h"

namespace fa {

// Masked / not-yet-seen scores use a large finite sentinel instead of -inf so that the kernel can
// be compiled without IEEE inf/NaN semantics (no canonicalising v_max before fmaxf, v_max3).
constexpr float kNeg = -1.0e30f;
// Deferred rescale (guide T13): the running max used for exp2 is only raised when a row's max grows
// by more than kRescaleThr (log2 units, i.e. a factor 2^8) -- P then stays <= 256, exact in fp16 /
// bf16 relative precision, and the O / l rescale pass is skipped on almost every tile.
constexpr float kRescaleThr = 8.0f;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

template <int N>
struct IC {
    static constexpr int value = N;
};
// compile-time loop: f(IC<I>{}) for I = 0 .. N-1 (every index a constant expression)
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I < N) {
        f(IC<I>{});
        static_for<N, I + 1>(f);
    }
}

struct F16 {
    static constexpr bool kIsF16 = true;
    static __device__ __forceinline__ f32x16 mfma(u32x4 a, u32x4 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                      __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    }
    // round-to-nearest-even pack of two fp32 into two fp16 (low element first): v_cvt_pk_f16_f32
    static __device__ __forceinline__ uint32_t pack(float lo, float hi) {
        f16x2 v = __builtin_convertvector((f32x2){lo, hi}, f16x2);
        return __builtin_bit_cast(uint32_t, v);
    }
    // rotate-half RoPE of 8 elements (HF apply_rotary_pos_emb, reference models/rope_attn_fwd.py:8-38):
    // x*cos + rot*sin with rot = -partner (first half) / +partner (second half), fp32, one RNE rounding
    static __device__ __forceinline__ u32x4 rope8(u32x4 v, u32x4 partner, u32x4 c, u32x4 s, bool second) {
        const f16x8 x = __builtin_bit_cast(f16x8, v), y = __builtin_bit_cast(f16x8, partner);
        const f16x8 cc = __builtin_bit_cast(f16x8, c), ss = __builtin_bit_cast(f16x8, s);
        u32x4 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float r0 = second ? (float)y[2 * i] : -(float)y[2 * i];
            const float r1 = second ? (float)y[2 * i + 1] : -(float)y[2 * i + 1];
            float a0 = __builtin_fmaf((float)x[2 * i], (float)cc[2 * i], r0 * (float)ss[2 * i]);
            float a1 = __builtin_fmaf((float)x[2 * i + 1], (float)cc[2 * i + 1], r1 * (float)ss[2 * i + 1]);
            asm volatile("" : "+v"(a0), "+v"(a1));  // fp32 rounding step kept, as csrc/fa_rope.hip
            r[i] = pack(a0, a1);
        }
        return r;
    }
};

struct BF16 {
    static constexpr bool kIsF16 = false;
    static __device__ __forceinline__ f32x16 mfma(u32x4 a, u32x4 b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                       __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    }
    // v_cvt_pk_bf16_f32 (RNE)
    static __device__ __forceinline__ uint32_t pack(float lo, float hi) {
        bf16x2 v = __builtin_convertvector((f32x2){lo, hi}, bf16x2);
        return __builtin_bit_cast(uint32_t, v);
    }
    // rotate-half RoPE of 8 elements (HF apply_rotary_pos_emb, reference models/rope_attn_fwd.py:8-38):
    // x*cos + rot*sin with rot = -partner (first half) / +partner (second half), fp32, one RNE rounding
    static __device__ __forceinline__ u32x4 rope8(u32x4 v, u32x4 partner, u32x4 c, u32x4 s, bool second) {
        const bf16x8 x = __builtin_bit_cast(bf16x8, v), y = __builtin_bit_cast(bf16x8, partner);
        const bf16x8 cc = __builtin_bit_cast(bf16x8, c), ss = __builtin_bit_cast(bf16x8, s);
        u32x4 r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float r0 = second ? (float)y[2 * i] : -(float)y[2 * i];
            const float r1 = second ? (float)y[2 * i + 1] : -(float)y[2 * i + 1];
            float a0 = __builtin_fmaf((float)x[2 * i], (float)cc[2 * i], r0 * (float)ss[2 * i]);
            float a1 = __builtin_fmaf((float)x[2 * i + 1], (float)cc[2 * i + 1], r1 * (float)ss[2 * i + 1]);
            asm volatile("" : "+v"(a0), "+v"(a1));  // fp32 rounding step kept, as csrc/fa_rope.hip
            r[i] = pack(a0, a1);
        }
        return r;
    }
};

// Per head-dim geometry. kD is the padded head dim of the LDS image and of the MFMA k-steps.
template <int kD>
struct Geo {
    static constexpr int kRowBytes = kD * 2;            // 256 / 128
    static constexpr int kChunks = kD / 8;              // 16-B chunks per row
    static constexpr int kTileBytes = kBlockN * kRowBytes;
    // LDS ring: 2 K slots + 3 V slots. V needs a third slot because waves 4-7 run their P.V of
    // tile j after the barrier that publishes tile j+1 (see "stagger" in the kernel).
    static constexpr int kLdsBytes = 5 * kTileBytes;
    static constexpr int kKSteps = kD / 16;             // k-steps of S^T = K.Q^T
    static constexpr int kDTiles = kD / 32;             // 32-row d tiles of O^T
    static constexpr int kStage = kBlockN * kChunks / kThreads;  // chunks per thread per tile (2 / 1)

    // K image: the A-operand read has lane r on row r (one 16-B chunk each). For 256-B rows the
    // chunk slot is c ^ (r & 15); for 128-B rows (two rows per 256-B bank row) c ^ ((r >> 1) & 7).
    // Both put the 16 lanes of every ds_read_b128 lane group on 16 distinct 16-B bank slots.
    static __device__ __forceinline__ int k_off(int row, int ch) {
        return kD == 128 ? row * 256 + 16 * (ch ^ (row & 15)) : row * 128 + 16 * (ch ^ ((row >> 1) & 7));
    }
    // V image, read transposed by ds_read_b64_tr_b16: a half-wave reads 4 rows R..R+3 (R % 4 == 0)
    // x 64 B; the XOR puts the four 64-B pieces into the four quarters of the 256-B bank row.
    static __device__ __forceinline__ int v_off(int row, int ch) {
        return kD == 128 ? row * 256 + 16 * (ch ^ ((row & 3) << 2))
                         : row * 128 + 16 * (ch ^ (((row >> 1) & 1) << 2));
    }
};

// v_permlane32_swap(vdst=x, src=x): the lower half-wave receives the upper half's x in the src
// result and keeps its own in vdst; the upper half the other way round. Combining both results
// therefore gives the (l, l^32) pair reduction with the same value in both lanes.
// a * fa + b * fb as two rounded products and one rounded sum, never contracted into an fma (the
// key-split combine: symmetric in its two operands, so bit-identical whichever piece is "a")
__device__ __forceinline__ float sum_of_products(float a, float fa, float b, float fb) {
    float x = a * fa, y = b * fb;
    asm volatile("" : "+v"(x), "+v"(y));
    return x + y;
}
// the same for two neighbouring elements at once (v_pk_mul_f32 x 2, v_pk_add_f32)
__device__ __forceinline__ f32x2 sum_of_products2(f32x2 a, f32x2 fa, f32x2 b, f32x2 fb) {
    f32x2 x = a * fa, y = b * fb;
    asm volatile("" : "+v"(x), "+v"(y));
    return x + y;
}
// Key-split workspace accesses. The two pieces of a block run on ONE XCD: fa_fwd_w4's work order puts
// both in the list of the XCD that blockIdx & 7 names, and the hardware deals workgroups to XCDs
// round-robin by workgroup id (MI355X_MICROARCH "Workgroup dispatch"). The hand-off relies on that
// shared L2: every record store is a 16-B write-through (sc1) store drained by its wave before the
// flag, the flag an agent-scope (sc1) store, the counter an agent-scope atomic, and every load of a
// record or statistic an sc1 load (bypasses this CU's L1) behind the poll -- with no agent-scope fence
// and no buffer_wbl2 / buffer_inv, which write back / invalidate the whole L2 of the XCD, the K/V lines
// of every other workgroup included (measured: the layout ran at half speed with them). Pieces on two
// XCDs would need them. A poll that times out is counted (fa_split_errors). Inline asm
// (the builtin forms cost the D=128 causal kernels a spilled VGPR), so: the loads and their wait in
// ONE statement with early-clobber outputs (hipcc counts no asm load), and every 16-B store ends in
// s_nop 1 (hipcc may otherwise overwrite its data registers before the store has read them).
__device__ __forceinline__ void st_ws(u32x4 *p, const u32x4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
// four records 64 x 16 B apart from each of pa and pb, landed (one round trip for two d-tiles)
__device__ __forceinline__ void ld_ws8(const u32x4 *pa, const u32x4 *pb, u32x4 (&x)[4], u32x4 (&y)[4]) {
    asm volatile("global_load_dwordx4 %0, %8, off sc1\n\tglobal_load_dwordx4 %1, %8, off offset:1024 sc1\n\t"
                 "global_load_dwordx4 %2, %8, off offset:2048 sc1\n\tglobal_load_dwordx4 %3, %8, off offset:3072 sc1\n\t"
                 "global_load_dwordx4 %4, %9, off sc1\n\tglobal_load_dwordx4 %5, %9, off offset:1024 sc1\n\t"
                 "global_load_dwordx4 %6, %9, off offset:2048 sc1\n\tglobal_load_dwordx4 %7, %9, off offset:3072 sc1\n\t"
                 "s_waitcnt vmcnt(0)"
                 : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3]), "=&v"(y[0]), "=&v"(y[1]), "=&v"(y[2]), "=&v"(y[3])
                 : "v"(pa), "v"(pb)
                 : "memory");
}
// two records (p, p + 64), landed
__device__ __forceinline__ void ld_ws2(const u32x4 *p, u32x4 &x0, u32x4 &x1) {
    asm volatile("global_load_dwordx4 %0, %2, off sc1\n\tglobal_load_dwordx4 %1, %2, off offset:1024 sc1\n\t"
                 "s_waitcnt vmcnt(0)"
                 : "=&v"(x0), "=&v"(x1)
                 : "v"(p)
                 : "memory");
}
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

// Buffer descriptor over [base, base + nbytes): loads past the end return 0 and stores past the
// end are dropped by the hardware range check, so ragged tails need no per-lane predicates.
__device__ __forceinline__ rsrc_t make_rsrc(const char *base, uint32_t nbytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)nbytes, 0x00020000);
}

// the same from values the compiler cannot prove wave-uniform (loaded from memory, carried across
// branches): readfirstlane keeps the descriptor in SGPRs (the values are uniform by construction)
__device__ __forceinline__ rsrc_t make_rsrc_u(const char *base, uint32_t nbytes) {
    const uint64_t a = (uint64_t)(uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const char *ub = (const char *)(uintptr_t)(((uint64_t)hi << 32) | lo);
    return make_rsrc(ub, __builtin_amdgcn_readfirstlane(nbytes));
}

// bytes of the first `rows` rows of a [rows, D] slab with row stride `stride` elements; 0 if
// rows <= 0. The host guarantees rows * stride * 2 + 256 < 2^31 for the slabs the kernels address
// (K / V: 64-row tiles; Q / O / RoPE: kQoSpanRows rows, fa_launch.h).
__device__ __forceinline__ uint32_t slab_bytes(int rows, int stride, int D) {
    return rows <= 0 ? 0u : (uint32_t)(((rows - 1) * stride + D) * 2);
}

// XCD-aware work decode. Workgroups are dealt round-robin over the 8 XCDs (blocks b and b+8 share
// one, MI355X_MICROARCH "Workgroup dispatch"), and an XCD starts its blocks in bid order. Each XCD is
// given a contiguous range of the logical order (batch, q-head, q-tile) -- the q-tiles of one
// (batch, head), and the q-heads of one kv group, share that XCD's 4 MiB L2 for their K/V stream.
// Causal: when the XCD's range is made of whole (batch, head) rows, it is cut into groups of hg
// heads (about 64 workgroups, two per CU of the XCD; with 16 q-tiles that is 4 heads, one GQA group
// of Llama-3) and each group is walked q-tile-major, heaviest q-tile level first across its heads
// (longest-processing-time-first, so each group ends on light tiles while the next group's heavy
// tiles fill the CUs that free up), keeping only hg heads' K/V in flight per XCD; otherwise each
// (batch, head) row is walked heavy-first.
// Bijective for any grid size; speed only, never correctness.
#ifdef FA_STAMPS
__device__ __forceinline__ unsigned long long xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return (unsigned long long)(x & 15);
}
#endif

struct Work {
    int qtile, hq, b;
    int kr = 0;  // (fa_fwd_w4 key-split launches) kind | mid << 2: 0 the whole block, 1 its key tiles
                 // [0, mid), 2 its key tiles [mid, n_end) -- a piece that meets its partner in the epilogue
};
template <bool kCausal>
__device__ __forceinline__ Work decode_work(const uint32_t nwg, const uint32_t bid, const int n_qtiles, const int Hq,
                                            const int g) {
    const uint32_t xcd = bid & 7, k = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
    const uint32_t start = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
    const uint32_t cnt = q8 + (xcd < r8 ? 1u : 0u);
    const uint32_t nq = (uint32_t)n_qtiles;
    uint32_t t, bh;
    if (kCausal && start % nq == 0 && cnt % nq == 0) {
        const uint32_t nb = cnt / nq;  // heads of this XCD
        // at least one GQA group: with many q-tiles (long sequences, local windows) the XCD's CUs
        // then run neighbouring q-tiles of the g q-heads that share one K/V stream
        uint32_t hg = 64u / nq;
        hg = hg < (uint32_t)g ? (uint32_t)g : hg;
        hg = hg < 1u ? 1u : (hg > nb ? nb : hg);
        while (nb % hg) --hg;
        const uint32_t grp = k / (hg * nq), kk = k % (hg * nq);
        t = kk / hg;
        bh = start / nq + grp * hg + kk % hg;
    } else {
        const uint32_t w = start + k;
        t = w % nq;
        bh = w / nq;
    }
    Work r;
    r.hq = (int)(bh % (uint32_t)Hq);
    r.b = (int)(bh / (uint32_t)Hq);
    r.qtile = kCausal ? (n_qtiles - 1 - (int)t) : (int)t;  // causal: heavy tiles first
    return r;
}

#ifdef FA_DEBUG_VARIANTS  // (debug / A-B library only: _build.build_abi(debug=True))
template <class DT, bool kCausal, int kD, bool kExactD>
__global__ __launch_bounds__(kThreads) void fa_fwd_w8(const fa_fwd_params p, const int n_qtiles) {
    using G = Geo<kD>;
    __shared__ __attribute__((aligned(16))) char lds[G::kLdsBytes];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31;
    const int h = lane >> 5;

    // ---- XCD-aware work decode ----------------------------------------------------------
    const Work wk = decode_work<kCausal>(gridDim.x, blockIdx.x, n_qtiles, (int)p.num_heads_q, (int)p.head_q_per_group);
    const int hq = wk.hq, b = wk.b, qtile = wk.qtile;
    const int hkv = hq / (int)p.head_q_per_group;

    const int Sq = (int)p.seqlen_q, Sk = (int)p.seqlen_kv, D = (int)p.headdim;
    const float sc = p.softmax_scale;
    const float thr_raw = kRescaleThr / sc;  // rescale threshold in unscaled score units

    const char *qb = (const char *)p.q_ptr + 2 * ((int64_t)b * p.q_batch_stride + (int64_t)hq * p.q_head_stride);
    const char *kb = (const char *)p.k_ptr + 2 * ((int64_t)b * p.k_batch_stride + (int64_t)hkv * p.k_head_stride);
    const char *vb = (const char *)p.v_ptr + 2 * ((int64_t)b * p.v_batch_stride + (int64_t)hkv * p.v_head_stride);
    char *ob = (char *)p.o_ptr + 2 * ((int64_t)b * p.o_batch_stride + (int64_t)hq * p.o_head_stride);

    const int m0 = qtile * kBlockM;   // first query row of the workgroup
    const int mw = m0 + wave * 32;    // first query row of this wave
    const int my_q = mw + r;          // this lane's query row
    const int diag = Sk - Sq;         // bottom-right causal offset: key n visible iff n <= m + diag

    // ---- KV tile range ----------------------------------------------------------------
    const int n_blocks = (Sk + kBlockN - 1) / kBlockN;
    int n_end = n_blocks;
    if (kCausal) {
        // the workgroup's last valid query sees keys up to min(m0+BM, Sq) - 1 + diag
        const int x = diag + min(m0 + kBlockM, Sq);
        const int nb = x <= 0 ? 0 : (x + kBlockN - 1) / kBlockN;
        n_end = min(nb, n_blocks);
    }

    // ---- Q fragments (B operand of S^T = K.Q^T), resident for the whole loop ----------
    // lane (h, r) holds Q[my_q][16*ks + 8*h + 0..7] for k-step ks; rows >= Sq read as 0
    u32x4 qf[G::kKSteps];
    {
        const int qs = (int)p.q_seqlen_stride;
        const rsrc_t qr = make_rsrc(qb + 2 * (int64_t)mw * qs, slab_bytes(min(Sq - mw, 32), qs, D));
        const int off = r * qs * 2 + 16 * h;
#pragma unroll
        for (int ks = 0; ks < G::kKSteps; ++ks) {
            qf[ks] = __builtin_amdgcn_raw_buffer_load_b128(qr, off + 32 * ks, 0, 0);
            if (!kExactD && 16 * ks + 8 * h >= D) qf[ks] = (u32x4){0, 0, 0, 0};
        }
    }

    // ---- register staging of K/V tiles ------------------------------------------------
    // thread t moves 16-B chunk (t % kChunks) of rows t / kChunks (+ 32 for D = 128) of K and V
    const int srow = tid / G::kChunks;
    const int sch = tid % G::kChunks;
    const int ks_ = (int)p.k_seqlen_stride, vs_ = (int)p.v_seqlen_stride;
    const int koff0 = srow * ks_ * 2 + 16 * sch;
    const int voff0 = srow * vs_ * 2 + 16 * sch;
    const int koff1 = koff0 + 32 * ks_ * 2;
    const int voff1 = voff0 + 32 * vs_ * 2;
    const bool sch_ok = kExactD || sch * 8 < D;
    u32x4 kst0, kst1, vst0, vst1;

    auto stage_load = [&](int j) {
        // descriptors rebased per tile: 32-bit lane offsets stay tile-invariant; rows >= Sk read 0
        const int key0 = j * kBlockN;
        const rsrc_t kr = make_rsrc(kb + 2 * (int64_t)key0 * ks_, slab_bytes(min(Sk - key0, kBlockN), ks_, D));
        const rsrc_t vr = make_rsrc(vb + 2 * (int64_t)key0 * vs_, slab_bytes(min(Sk - key0, kBlockN), vs_, D));
        kst0 = __builtin_amdgcn_raw_buffer_load_b128(kr, koff0, 0, 0);
        vst0 = __builtin_amdgcn_raw_buffer_load_b128(vr, voff0, 0, 0);
        if (G::kStage == 2) {
            kst1 = __builtin_amdgcn_raw_buffer_load_b128(kr, koff1, 0, 0);
            vst1 = __builtin_amdgcn_raw_buffer_load_b128(vr, voff1, 0, 0);
        }
    };
    auto stage_write = [&](int kslot, int vslot) {
        char *K = lds + kslot * G::kTileBytes;
        char *V = lds + (2 + vslot) * G::kTileBytes;
        // D < kD: K columns past D must be 0 (they meet Q's zero columns, garbage could be NaN)
        const u32x4 z = {0, 0, 0, 0};
        *(u32x4 *)(K + G::k_off(srow, sch)) = sch_ok ? kst0 : z;
        *(u32x4 *)(V + G::v_off(srow, sch)) = vst0;
        if (G::kStage == 2) {
            *(u32x4 *)(K + G::k_off(srow + 32, sch)) = sch_ok ? kst1 : z;
            *(u32x4 *)(V + G::v_off(srow + 32, sch)) = vst1;
        }
    };

    // ---- per-lane constant LDS addresses ----------------------------------------------
    // V^T A-operand via ds_read_b64_tr_b16: lane = 16*g + 4*qq + pp supplies row (R + qq),
    // columns dt*32 + 16*(g&1) + 4*pp .. +3 where R = kt*32 + 16*s + 4*(g>>1) (+8 for the
    // second half of the fragment); it receives column dt*32 + (lane & 31) of rows R..R+3.
    const int g = lane >> 4;
    const int qq = (lane >> 2) & 3;
    const int pp = lane & 3;
    int v_addr[G::kDTiles];
#pragma unroll
    for (int dt = 0; dt < G::kDTiles; ++dt)
        v_addr[dt] = G::v_off(4 * (g >> 1) + qq, dt * 4 + 2 * (g & 1) + (pp >> 1)) + 8 * (pp & 1);
    int k_addr[G::kKSteps];
#pragma unroll
    for (int ks = 0; ks < G::kKSteps; ++ks) k_addr[ks] = G::k_off(r, 2 * ks + h);

    f32x16 o[G::kDTiles];
#pragma unroll
    for (int dt = 0; dt < G::kDTiles; ++dt) o[dt] = (f32x16){};
    float m_use = kNeg;  // running max used by exp2 (unscaled score units), lags by < kRescaleThr
    float msc = 0.f;     // m_use * sc, or 0 while the row has seen no visible key
    float l_run = 0.f;   // lane-partial row sum of P (32 of the 64 keys of each tile)

    // Stagger (MI355X_MICROARCH "Two waves per SIMD"): waves w and w+4 share a SIMD. Waves 4-7
    // ("lag") run each tile's P.V after the tile's barrier, i.e. half a tile behind waves 0-3, so
    // one wave's softmax (VALU) overlaps its partner's MFMAs instead of both waves alternating
    // between all-MFMA and all-VALU phases in lockstep.
    const bool lag = wave >= 4;
    u32x4 pf[4];               // P of the last softmax (B operand of P.V), k-step kk = (kt, s)
    bool pv_pending = false;   // lag waves: P.V of the previous tile still to do
    const char *pv_v = lds;    // ... and the V slot it reads

    // S^T = K.Q^T, mask, online softmax; leaves P (rounded to T) in pf
    auto qk_softmax = [&](const char *K, const int key0, const bool need_mask) {
        f32x16 s0 = {}, s1 = {};
#pragma unroll
        for (int ks = 0; ks < G::kKSteps; ++ks) {
            const u32x4 a0 = *(const u32x4 *)(K + k_addr[ks]);
            const u32x4 a1 = *(const u32x4 *)(K + 32 * G::kRowBytes + k_addr[ks]);
            s0 = DT::mfma(a0, qf[ks], s0);
            s1 = DT::mfma(a1, qf[ks], s1);
        }
        // mask (only tiles crossing the diagonal or the Sk tail)
        if (need_mask) {
            const int lim = kCausal ? min(Sk - 1, my_q + diag) : Sk - 1;  // last visible key
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int kk = key0 + (i & 3) + 8 * (i >> 2) + 4 * h;
                if (kk > lim) s0[i] = kNeg;
                if (kk + 32 > lim) s1[i] = kNeg;
            }
        }
        // online softmax (per lane = per query row)
        float mx = fmaxf(fmaxf(s0[0], s0[1]), fmaxf(s1[0], s1[1]));
#pragma unroll
        for (int i = 2; i < 16; i += 2) mx = fmaxf(mx, fmaxf(fmaxf(s0[i], s0[i + 1]), fmaxf(s1[i], s1[i + 1])));
        // deferred rescale: taken by the whole wave when any row's max outgrows m_use; every
        // earlier P.V is already in O at this point (lag waves ran theirs first). Both lane halves
        // hold the same row's m_use, so the check needs no cross-half reduction.
        float alpha = 1.f;
        const bool grow = mx > m_use + thr_raw;
        if (__builtin_amdgcn_ballot_w64(grow)) {
            const float m_new = fmaxf(m_use, pair_max(mx));
            const float msc_new = (m_new <= kNeg) ? 0.f : m_new * sc;
            alpha = __builtin_amdgcn_exp2f(msc - msc_new);  // msc == 0 && m_use == kNeg: l, O are 0
            m_use = m_new;
            msc = msc_new;
#pragma unroll
            for (int dt = 0; dt < G::kDTiles; ++dt) o[dt] *= alpha;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            s0[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(s0[i], sc, -msc));
            s1[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(s1[i], sc, -msc));
        }
        float ls0 = s0[0], ls1 = s1[0];
#pragma unroll
        for (int i = 1; i < 16; ++i) {
            ls0 += s0[i];
            ls1 += s1[i];
        }
        l_run = l_run * alpha + (ls0 + ls1);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            pf[s] = (u32x4){DT::pack(s0[8 * s + 0], s0[8 * s + 1]), DT::pack(s0[8 * s + 2], s0[8 * s + 3]),
                            DT::pack(s0[8 * s + 4], s0[8 * s + 5]), DT::pack(s0[8 * s + 6], s0[8 * s + 7])};
            pf[2 + s] = (u32x4){DT::pack(s1[8 * s + 0], s1[8 * s + 1]), DT::pack(s1[8 * s + 2], s1[8 * s + 3]),
                                DT::pack(s1[8 * s + 4], s1[8 * s + 5]), DT::pack(s1[8 * s + 6], s1[8 * s + 7])};
        }
    };

    // O^T += V^T . P^T
    auto pv = [&](const char *V) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int rowoff = ((kk >> 1) * 32 + (kk & 1) * 16) * G::kRowBytes;  // kt*32 + 16*s
#pragma unroll
            for (int dt = 0; dt < G::kDTiles; ++dt) {
                const u32x2 lo = tr_read(V + rowoff + v_addr[dt]);
                const u32x2 hi = tr_read(V + rowoff + 8 * G::kRowBytes + v_addr[dt]);
                o[dt] = DT::mfma((u32x4){lo[0], lo[1], hi[0], hi[1]}, pf[kk], o[dt]);
            }
        }
    };

    if (n_end > 0) stage_load(0);
    // retire Q and tile 0 here; the asm barrier re-defines qf so the loop's wait analysis does not
    // see the Q loads as pending (it would otherwise wait vmcnt(0) at the top of every iteration)
    __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
    for (int ks = 0; ks < G::kKSteps; ++ks) asm volatile("" : "+v"(qf[ks]));
    if (n_end > 0) {
        stage_write(0, 0);
        if (n_end > 1) stage_load(1);
    }
    __syncthreads();

    // one KV tile; the K slot KB is a compile-time constant (loop unrolled by 2) so K addresses
    // are a per-lane base plus an immediate offset; the V slot cycles through 3
    int vslot = 0;
    auto tile = [&](const int j, auto KB) {
        constexpr int kslot = decltype(KB)::value;
        const char *K = lds + kslot * G::kTileBytes;
        const char *V = lds + (2 + vslot) * G::kTileBytes;
        const int key0 = j * kBlockN;

        bool wave_active = true;
        bool need_mask = key0 + kBlockN > Sk;
        if (kCausal) {
            wave_active = key0 <= mw + 31 + diag;                      // a key visible to the last row
            need_mask = need_mask || (key0 + kBlockN - 1 > mw + diag);  // a key hidden from the first row
        }
        if (pv_pending) {  // lag waves: previous tile's P.V (its V slot is not overwritten until j+2)
            pv(pv_v);
            pv_pending = false;
        }
        if (wave_active) {
            qk_softmax(K, key0, need_mask);
            if (lag) {
                pv_pending = true;
                pv_v = V;
            } else {
                pv(V);
            }
        }
        vslot = vslot == 2 ? 0 : vslot + 1;
        if (j + 1 < n_end) stage_write(kslot ^ 1, vslot);
        __syncthreads();
        if (j + 2 < n_end) stage_load(j + 2);
    };
    for (int j = 0; j < n_end; j += 2) {
        tile(j, IC<0>{});
        if (j + 1 < n_end) tile(j + 1, IC<1>{});
    }
    if (pv_pending) pv(pv_v);

    // ---- epilogue: O = O^T / l, row per lane, 16-B stores after a half-wave swap ----------
    const float l_tot = pair_sum(l_run);
    const float inv = (l_tot == 0.f) ? 1.f : 1.f / l_tot;
    const int os_ = (int)p.o_seqlen_stride;
    const rsrc_t orr = make_rsrc(ob + 2 * (int64_t)mw * os_, slab_bytes(min(Sq - mw, 32), os_, D));
    const int orow = r * os_ * 2;
#pragma unroll
    for (int dt = 0; dt < G::kDTiles; ++dt) {
#pragma unroll
        for (int gp = 0; gp < 4; gp += 2) {
            // this lane holds d = dt*32 + 8*grp + 4*h + 0..3 in o[dt][4*grp .. 4*grp+3]
            const uint32_t a0 = DT::pack(o[dt][4 * gp + 0] * inv, o[dt][4 * gp + 1] * inv);
            const uint32_t a1 = DT::pack(o[dt][4 * gp + 2] * inv, o[dt][4 * gp + 3] * inv);
            const uint32_t b0 = DT::pack(o[dt][4 * gp + 4] * inv, o[dt][4 * gp + 5] * inv);
            const uint32_t b1 = DT::pack(o[dt][4 * gp + 6] * inv, o[dt][4 * gp + 7] * inv);
            const auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
            const auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
            // lower half: d = dt*32 + 8*gp + 0..7 ; upper half: d = dt*32 + 8*(gp+1) + 0..7
            const int d0 = dt * 32 + 8 * (gp + h);
            if (kExactD || d0 < D)
                __builtin_amdgcn_raw_buffer_store_b128((u32x4){x0[0], x1[0], x0[1], x1[1]}, orr, orow + 2 * d0, 0,
                                                       0);
        }
    }
}


#endif  // FA_DEBUG_VARIANTS

// =============================================================================================
// fa_fwd_w4: one wave per SIMD, 64 query rows per wave (two 32-row blocks A and B), software
// pipelined so that every MFMA stretch of one block runs beside the softmax VALU of the other:
//
//   phase 1: S_A(j)  = K_j . Q_A^T        ||  softmax part 2 of B (tile j-1)
//   phase 2: O_B    += V_{j-1}^T . P_B^T  ||  softmax part 1 of A (tile j)   -> rescale O_A
//   phase 3: S_B(j)  = K_j . Q_B^T        ||  softmax part 2 of A (tile j)
//   phase 4: O_A    += V_j^T . P_A^T      ||  softmax part 1 of B (tile j)   -> rescale O_B
//
// Within a phase the MFMAs (inline asm, 2 or 4 per group) and slices of the other block's softmax
// alternate in program order, pinned by sched_barrier; operand fragments are read from LDS one
// group ahead. The O accumulators of both blocks live in AGPRs for the whole kernel (asm "+a"
// operands); S, P, Q/K/V fragments and the softmax state stay in the 256 arch VGPRs.
// K/V tiles arrive by LDS-DMA (buffer_load ... lds, 1 KiB per wave-instruction) issued one tile
// ahead into a 2-slot K / 3-slot V ring; the XOR swizzle of the LDS images is applied on the
// per-lane SOURCE offsets (the DMA destination is lane-linear). Q is DMA'd to LDS once and its
// fragments are re-read per tile. One barrier per tile.
// Tiles that need masking (causal diagonal, Sk tail) or where a block is idle run a plain,
// non-pipelined body after the pipeline has been drained.
// =============================================================================================

// wait states between an asm MFMA's result and its first non-MFMA reader (s_ready, mfma_drain, the
// AGPR rescale of fa_agpr_asm.inc): see s_ready below
#ifdef FA_DRAIN21
#define FA_DRAIN_NOPS "s_nop 7\n\ts_nop 7\n\ts_nop 4"
#else
#define FA_DRAIN_NOPS "s_nop 11"
#endif
#include "fa_agpr_asm.inc"

// one MFMA a[BASE..BASE+15] += A.B into literal AGPRs (fa_agpr_asm.inc)
// (kW4: the form that also clobbers fa_fwd_w4's Q AGPRs a128..a191, fa_agpr_asm.inc)
template <bool kF16, int BASE, bool kW4 = false>
__device__ __forceinline__ void agpr_mfma(const u32x4 &a, const u32x4 &b) {
#define FA_CASE(N)                                                    \
    if constexpr (BASE == N) {                                        \
        if constexpr (kW4 && kF16) fa_agpr_mfma_w4_f16_##N(a, b);     \
        else if constexpr (kW4) fa_agpr_mfma_w4_bf16_##N(a, b);       \
        else if constexpr (kF16) fa_agpr_mfma_f16_##N(a, b);          \
        else fa_agpr_mfma_bf16_##N(a, b);                             \
    }
    FA_CASE(0) FA_CASE(16) FA_CASE(32) FA_CASE(48) FA_CASE(64) FA_CASE(80) FA_CASE(96) FA_CASE(112)
#undef FA_CASE
}
template <int DTL, bool kBlockB>
__device__ __forceinline__ void agpr_scale(const float alpha) {
    if constexpr (DTL == 4) {
        if constexpr (kBlockB) fa_agpr_scale_4_b(alpha); else fa_agpr_scale_4_a(alpha);
    } else {
        if constexpr (kBlockB) fa_agpr_scale_2_b(alpha); else fa_agpr_scale_2_a(alpha);
    }
}
template <int BASE>
__device__ __forceinline__ void agpr_read8(float *x) {
#define FA_CASE(N) \
    if constexpr (BASE == N) fa_agpr_read8_##N(x);
    FA_CASE(0) FA_CASE(8) FA_CASE(16) FA_CASE(24) FA_CASE(32) FA_CASE(40) FA_CASE(48) FA_CASE(56)
    FA_CASE(64) FA_CASE(72) FA_CASE(80) FA_CASE(88) FA_CASE(96) FA_CASE(104) FA_CASE(112) FA_CASE(120)
#undef FA_CASE
}
template <int BASE>
__device__ __forceinline__ f32x16 agpr_read16() {
    float x[16];
    if constexpr (BASE == 0) fa_agpr_read16_0(x);
    else if constexpr (BASE == 16) fa_agpr_read16_16(x);
    else if constexpr (BASE == 32) fa_agpr_read16_32(x);
    else if constexpr (BASE == 48) fa_agpr_read16_48(x);
    else if constexpr (BASE == 64) fa_agpr_read16_64(x);
    else if constexpr (BASE == 80) fa_agpr_read16_80(x);
    else if constexpr (BASE == 96) fa_agpr_read16_96(x);
    else if constexpr (BASE == 112) fa_agpr_read16_112(x);
    else if constexpr (BASE == 128) fa_agpr_read16_128(x);
    else if constexpr (BASE == 144) fa_agpr_read16_144(x);
    else if constexpr (BASE == 160) fa_agpr_read16_160(x);
    else fa_agpr_read16_176(x);
    f32x16 v;
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = x[i];
    return v;
}

// one MFMA of S^T = K.Q^T into arch VGPRs (inline asm, so hipcc keeps it in program order among
// the softmax slices); first: C = 0
template <bool kF16>
__device__ __forceinline__ void mfma_sv(const bool first, f32x16 &acc, const u32x4 &a, const u32x4 &b) {
    if (first) {
        if constexpr (kF16) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
        else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
    } else {
        if constexpr (kF16) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
        else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
    }
}

// Q fragments pinned in AGPRs a[128 + 4*(X*KS + ks)] (fa_agpr_asm.inc): write one, and one MFMA of
// S^T = K.Q^T reading it as the B operand
template <int QB>
__device__ __forceinline__ void agpr_qset(const u32x4 &v) {
#define FA_CASE(N) \
    if constexpr (QB == N) fa_agpr_qset_##N(v[0], v[1], v[2], v[3]);
    FA_CASE(128) FA_CASE(132) FA_CASE(136) FA_CASE(140) FA_CASE(144) FA_CASE(148) FA_CASE(152) FA_CASE(156)
    FA_CASE(160) FA_CASE(164) FA_CASE(168) FA_CASE(172) FA_CASE(176) FA_CASE(180) FA_CASE(184) FA_CASE(188)
#undef FA_CASE
}
// asynchronous load of one Q fragment from rs + voff straight into a[QB .. QB+3]
template <int QB>
__device__ __forceinline__ void agpr_qload(const rsrc_t &rs, const int voff, const bool nop) {
#define FA_CASE(N) \
    if constexpr (QB == N) fa_agpr_qload_##N(rs, voff, nop);
    FA_CASE(128) FA_CASE(132) FA_CASE(136) FA_CASE(140) FA_CASE(144) FA_CASE(148) FA_CASE(152) FA_CASE(156)
    FA_CASE(160) FA_CASE(164) FA_CASE(168) FA_CASE(172) FA_CASE(176) FA_CASE(180) FA_CASE(184) FA_CASE(188)
#undef FA_CASE
}
// one Q fragment from LDS (staged there by LDS-DMA) straight into a[QB .. QB+3]
template <int QB>
__device__ __forceinline__ void agpr_qlds(const uint32_t addr) {
#define FA_CASE(N) \
    if constexpr (QB == N) fa_agpr_qlds_##N(addr);
    FA_CASE(128) FA_CASE(132) FA_CASE(136) FA_CASE(140) FA_CASE(144) FA_CASE(148) FA_CASE(152) FA_CASE(156)
    FA_CASE(160) FA_CASE(164) FA_CASE(168) FA_CASE(172) FA_CASE(176) FA_CASE(180) FA_CASE(184) FA_CASE(188)
#undef FA_CASE
}
template <bool kF16, int QB>
__device__ __forceinline__ void mfma_sq(const bool first, f32x16 &acc, const u32x4 &a) {
#define FA_CASE(N)                                                                         \
    if constexpr (QB == N) {                                                               \
        if (first) {                                                                       \
            if constexpr (kF16) fa_sq_f16_##N##_1(acc, a); else fa_sq_bf16_##N##_1(acc, a); \
        } else {                                                                           \
            if constexpr (kF16) fa_sq_f16_##N##_0(acc, a); else fa_sq_bf16_##N##_0(acc, a); \
        }                                                                                  \
    }
    FA_CASE(128) FA_CASE(132) FA_CASE(136) FA_CASE(140) FA_CASE(144) FA_CASE(148) FA_CASE(152) FA_CASE(156)
    FA_CASE(160) FA_CASE(164) FA_CASE(168) FA_CASE(172) FA_CASE(176) FA_CASE(180) FA_CASE(184) FA_CASE(188)
#undef FA_CASE
}

// An asm-issued MFMA's result is invisible to hipcc's hazard recognizer: before the first VALU
// read of S (or AGPR read of O) after its last MFMA, the wait states hipcc inserts itself after a
// builtin v_mfma_f32_32x32x16 on gfx950: 12 (8 passes + 4; scripts/microbench/mfma_hazard_probe.hip,
// enforced by _asm_check rule R3). (FA_DRAIN21: the 21 of rounds 1-3, for A/B.)
__device__ __forceinline__ void s_ready(f32x16 &s0, f32x16 &s1) { asm volatile(FA_DRAIN_NOPS : "+v"(s0), "+v"(s1)); }
__device__ __forceinline__ void mfma_drain() { asm volatile(FA_DRAIN_NOPS ::: "memory"); }
__device__ __forceinline__ void s_ready4(f32x16 &s0, f32x16 &s1, f32x16 &s2, f32x16 &s3) {
    asm volatile(FA_DRAIN_NOPS : "+v"(s0), "+v"(s1), "+v"(s2), "+v"(s3));
}

#define FA_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
// s_waitcnt lgkmcnt(0) alone (gfx9 encoding: vmcnt 63, expcnt 7, lgkmcnt 0)
constexpr int kLgkm0 = 0xC07F;

// Causal / tail mask of score I of both key halves of a block (fa_fwd_w4 `mask`): key offsets
// c = (I & 3) + 8 (I >> 2) and c + 32 against e (the lane's last visible key minus key0 + 4h);
// hidden scores become kNeg. Two independent compare -> select chains (VCC and an SGPR pair).
// (neg: kNeg in a VGPR -- gfx9 VOP3 reads one SGPR / literal at most, and the select's mask is one)
template <int I>
__device__ __forceinline__ void mask_pair(f32x16 &s0, f32x16 &s1, const int e, const float neg) {
    constexpr int c = (I & 3) + 8 * (I >> 2);
    float x0 = s0[I], x1 = s1[I];
    uint64_t m;
    asm volatile(
        "v_cmp_le_i32_e32 vcc, %4, %3\n\t"
        "v_cmp_le_i32_e64 %2, %5, %3\n\t"
        "v_cndmask_b32_e64 %0, %6, %0, vcc\n\t"
        "v_cndmask_b32_e64 %1, %6, %1, %2"
        : "+v"(x0), "+v"(x1), "=&s"(m)
        : "v"(e), "n"(c), "n"(c + 32), "v"(neg)
        : "vcc");
    s0[I] = x0;
    s1[I] = x1;
}

// The same with a local window: score c is visible iff f <= c <= e (f: the lane's first visible key
// minus key0 + 4h), so both compares and their AND per score (two chains: VCC and SGPR pairs)
template <int I>
__device__ __forceinline__ void mask_pair_win(f32x16 &s0, f32x16 &s1, const int e, const int f, const float neg) {
    constexpr int c = (I & 3) + 8 * (I >> 2);
    float x0 = s0[I], x1 = s1[I];
    uint64_t m0, m1;
    asm volatile(
        "v_cmp_le_i32_e32 vcc, %5, %4\n\t"
        "v_cmp_ge_i32_e64 %2, %5, %8\n\t"
        "v_cmp_le_i32_e64 %3, %6, %4\n\t"
        "s_and_b64 vcc, vcc, %2\n\t"
        "v_cmp_ge_i32_e64 %2, %6, %8\n\t"
        "v_cndmask_b32_e64 %0, %7, %0, vcc\n\t"
        "s_and_b64 %3, %3, %2\n\t"
        "v_cndmask_b32_e64 %1, %7, %1, %3"
        : "+v"(x0), "+v"(x1), "=&s"(m0), "=&s"(m1)
        : "v"(e), "n"(c), "n"(c + 32), "v"(neg), "v"(f)
        : "vcc", "scc");
    s0[I] = x0;
    s1[I] = x1;
}

// Opaque redefinition: ties a value to this point of the (volatile-asm ordered) instruction stream,
// so IR-level sinking / hoisting cannot move the VALU slices out of their MFMA gap.
#ifndef FA_NOPIN
__device__ __forceinline__ void pin(float &x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(u32x4 &x) { asm volatile("" : "+v"(x)); }
__device__ __forceinline__ void pin(uint32_t &x) { asm volatile("" : "+v"(x)); }
#else
__device__ __forceinline__ void pin(float &) {}
__device__ __forceinline__ void pin(u32x4 &) {}
__device__ __forceinline__ void pin(uint32_t &) {}
#endif

__device__ __forceinline__ uint32_t lds_u32(const void *ptr) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)ptr;
}

// one LDS-DMA piece (1 KiB per wave-instruction) from rs + voff to LDS address `lds`.
// Issued from asm so hipcc does not see an LDS write it cannot disambiguate (it would otherwise
// wait vmcnt(0) before the next ds_read of any slot); the caller retires it with an explicit
// s_waitcnt vmcnt(0) before the tile's barrier. M0 is an asm input ("{m0}"): hipcc materialises it
// with one s_mov_b32 and keeps its own M0 bookkeeping; the s_nop 0 is the one wait state between
// an SALU write of M0 and an LDS-DMA that reads it (what hipcc inserts for its own LDS-DMA).
// nop: 5 more wait states ahead of the descriptor read (a VALU write of those SGPRs is invisible
// to the hazard recognizer).
__device__ __forceinline__ void dma_one(const rsrc_t &rs, const uint32_t lds, const int voff, const bool nop) {
    if (nop)
        asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "{m0}"(lds)
                     : "memory");
    else
        asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "{m0}"(lds)
                     : "memory");
}
// the same to LDS address base + OFF: M0 is formed inside the asm (s_add_u32), so the kernel keeps
// one LDS base in an SGPR instead of one materialised M0 value per (slot, piece)
template <int OFF>
__device__ __forceinline__ void dma_one_at(const rsrc_t &rs, const uint32_t base, const int voff, const bool nop) {
    if (nop)
        asm volatile("s_add_u32 m0, %2, %3\n\ts_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
                     "s"(base), "i"(OFF)
                     : "memory", "m0", "scc");
    else
        asm volatile("s_add_u32 m0, %2, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
                     "s"(base), "i"(OFF)
                     : "memory", "m0", "scc");
}
// NP pieces from rs + voff[n] to LDS lds0 + n*1024
template <int NP>
__device__ __forceinline__ void dma_pieces(const rsrc_t &rs, const uint32_t lds0, const int *voff) {
#pragma unroll
    for (int n = 0; n < NP; ++n) dma_one(rs, lds0 + n * 1024, voff[n], n == 0);
}

// One LDS-DMA piece of a tile from descriptor q + voff + IOFF to LDS M0 + IOFF: gfx950 adds the
// instruction offset to the LDS destination as well as to the source (scripts/microbench/
// ldsdma_offset.hip), so the pieces n = 1.. of a tile reuse piece 0's M0 with IOFF = n * 1024 and
// voff pre-reduced by n * 1024 (same bytes, same bounds check: the offset is range-checked).
// Piece 0 (IOFF == 0) writes M0 = m0v, then 5 wait states before the LDS-DMA (1 for the SALU
// write of M0, 5 if hipcc produced the descriptor by a VALU write of SGPRs, e.g. v_readfirstlane:
// the hazard recognizer does not see this asm read them); nothing between the pieces of one tile
// may write M0 (the loop issues no other LDS-DMA in that phase).
template <int IOFF>
__device__ __forceinline__ void dma_q(const rsrc_t &q, const uint32_t m0v, const int voff) {
    if constexpr (IOFF == 0)
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(q),
                     "s"(m0v)
                     : "memory", "m0");
    else
        asm volatile("buffer_load_dwordx4 %0, %1, 0 offen offset:%2 lds" ::"v"(voff), "s"(q), "i"(IOFF) : "memory");
}
// the NP pieces of one tile outside the pipelined loop: every piece names M0 as an input (hipcc
// sets it) and carries its own wait states (5 ahead of the first: the descriptor may come from a
// v_readfirstlane, a VALU write of SGPRs that the hazard recognizer cannot see the asm read)
template <int NP, int N = 0>
__device__ __forceinline__ void dma_tile(const rsrc_t &q, const uint32_t m0v, const int *voff) {
    if constexpr (N < NP) {
        if constexpr (N == 0)
            asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff[N]), "s"(q), "{m0}"(m0v)
                         : "memory");
        else
            asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen offset:%3 lds" ::"v"(voff[N]), "s"(q),
                         "{m0}"(m0v), "i"(N * 1024)
                         : "memory");
        dma_tile<NP, N + 1>(q, m0v, voff);
    }
}
// the same with M0 = base + MOFF formed inside the asm (one LDS base SGPR for every slot)
template <int MOFF, int IOFF>
__device__ __forceinline__ void dma_q_at(const rsrc_t &q, const uint32_t base, const int voff) {
    if constexpr (IOFF == 0)
        asm volatile("s_add_u32 m0, %2, %3\n\ts_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(q),
                     "s"(base), "i"(MOFF)
                     : "memory", "m0", "scc");
    else
        asm volatile("buffer_load_dwordx4 %0, %1, 0 offen offset:%2 lds" ::"v"(voff), "s"(q), "i"(IOFF) : "memory");
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// s_waitcnt immediate for vmcnt(n) alone (gfx9 encoding: vmcnt[3:0] + vmcnt[5:4] at [15:14], expcnt
// 7, lgkmcnt 15)
constexpr int vmcnt_enc(int n) { return (n & 15) | (((n >> 4) & 3) << 14) | 0x70 | 0xF00; }

// =============================================================================================
// fa_fwd_w4: one wave per SIMD, 64 query rows per wave (two 32-row blocks A and B). Per KV tile j:
//
//   P1(j): S_A(j), S_B(j) = K_j . Q^T   (32 MFMAs, K fragments shared)  ||  softmax part 2 of j-1
//   P2(j): O += V_{j-1}^T . P^T(j-1)    (2*DTL MFMAs per 16 keys: both blocks share the V^T
//          fragments)                                                  ||  softmax part 1 of j
//          then (rarely) rescale O and the row sums of a block whose max grew past the threshold
//
// MFMAs are inline asm (S into arch VGPRs, O and row sums into literal AGPRs, fa_agpr_asm.inc),
// with slices of softmax VALU pinned between them (pin + sched_barrier). Operand fragments are
// read from LDS one k-step ahead. S and P are double-buffered by tile parity (loop unrolled by
// 2). K/V tiles arrive by LDS-DMA (asm buffer_load ... lds, 1 KiB per wave-instruction): K_{j+1}
// and V_j are issued at the top of iteration j into 2-slot rings, with the XOR swizzle of the
// LDS images applied on the per-lane SOURCE offsets; Q is DMA'd once. One barrier per tile.
// Tiles that need masking (causal diagonal, Sk tail) run a non-pipelined body after the pipeline
// has been drained.
// =============================================================================================
template <class DT, bool kCausal, int kD, bool kExactD>
__global__ __launch_bounds__(256, 1) void fa_fwd_w4(const fa_fwd_params p, const int n_qtiles, const int dbg,
                                                    unsigned long long *stamps, const PathArgs xa) {
    // Diagnostic build only (-DFA_STAMPS=1, scripts/stamps.py): per-wave s_memtime phase totals.
#ifdef FA_STAMPS
    // (32-bit cycle stamps: a block's deltas fit, and half the SGPRs of 64-bit ones keep the
    // diagnostic build's register pressure near the product's)
    uint32_t st_t0 = (uint32_t)__builtin_amdgcn_s_memtime();
    unsigned long long st_rt0 = __builtin_amdgcn_s_memrealtime();
    uint32_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define FA_STAMP(v) const uint32_t v = (uint32_t)__builtin_amdgcn_s_memtime()
#ifdef FA_STAMPS_FINE  // (finer split: phase 2 at the ends of its quarters, phase 1 at its middle)
    uint32_t st_f[4] = {0, 0, 0, 0}, st_fa[4] = {0, 0, 0, 0};
#define FA_STAMP_W 19
#else
#define FA_STAMP_W 15
#endif
#else
    (void)stamps;
#define FA_STAMP(v)
#endif
    using G = Geo<kD>;
    constexpr bool F = DT::kIsF16;
    constexpr int KS = G::kKSteps;
    constexpr int DTL = G::kDTiles;
    constexpr int RB = G::kRowBytes;
    constexpr int T = G::kTileBytes;
    constexpr int NP = T / 4 / 1024;  // LDS-DMA pieces per wave per K or V tile (4 / 2)
    constexpr int ROWS_PER_PIECE = 1024 / RB;
    constexpr int kOStores = 2 * DTL * 2;  // O stores per wave and block (epilogue)
#ifdef FA_V0
    constexpr int kV0 = FA_V0;
#else
    constexpr int kV0 = 16;  // early scores per block and tile (phase 2); the rest run in phase 1
#endif
    static_assert(kV0 >= 4 && kV0 < 32 && kV0 % 2 == 0, "kV0");
    constexpr int kNL = 2 * (32 - kV0);  // late exp units of phase 1
    constexpr int QB = 128;  // Q fragments: AGPRs a[QB + 4*(X*KS + ks)] (fa_agpr_asm.inc)
#ifndef FA_QLDS
#define FA_QLDS 1
#endif
#ifndef FA_ZERO_MFMA  // O zeroed by 2 * DTL MFMAs in the prologue (0: 32 * DTL v_accvgpr_write)
#define FA_ZERO_MFMA 1
#endif
#ifndef FA_DRAIN_OVL  // the drain's late softmax in its P.V MFMA gaps (0: all of it before the P.V)
#define FA_DRAIN_OVL 1
#endif
#ifndef FA_EPI_OVL  // a block's O stores in the MFMA gaps of the next block's first tile (0: at its end;
#define FA_EPI_OVL 0   // 1 measured -0.3 % C4, -0.8 % C5, -2 % on C4's 8-way share: profiles/r5b_ab_*.log)
#endif
#ifndef FA_SPLIT_AGPR  // key-split combine: partner records into the Q AGPRs, a block per round trip
#define FA_SPLIT_AGPR 1  // (0: one d-tile of both blocks per round trip, into VGPRs)
#endif
#ifndef FA_PAIR_SHIFT  // key-split pairs: the heavy q-tile's split point moves this many tiles towards
#define FA_PAIR_SHIFT 2  // the workgroup that runs two blocks (its extra switch and hand-off)
#endif
#ifndef FA_SPLIT_PK  // (FA_SPLIT_AGPR) packed f32 combine with 1 / l folded into the two factors:
#define FA_SPLIT_PK 1   // o * (fm / l) + p * (fo / l), still symmetric in the pieces (0: (o fm + p fo) / l)
#endif
    // Q staging (kQL): 0 = HBM -> AGPR loads issued under the previous block's drain; 1 = LDS-DMA
    // into a Q image (K's swizzle) under the drain, read into the AGPRs at the block prologue;
    // 2 = the same pieces spread over the previous block's tiles (kQPT per tile, phase 2), so the
    // block switch moves no Q bytes. 1 is the default since the round-3 instruction cut: the two
    // per-tile checks of 2 cost more than the switch's Q burst (A/B +0.4..0.5 % on C2 / C4 / C5,
    // bit-identical, profiles/r3_ab_q_staging.log; round 2 had measured 2 ahead)
    constexpr int kQL = FA_QLDS;
    constexpr int kQPT = 2;
#ifndef FA_QPH
#define FA_QPH 2
#endif
    constexpr int kQPhase = FA_QPH;  // phase of the tile that issues them
    // (phase 1's K / V pieces share one M0 per tensor, dma_q_at: no other LDS-DMA may sit between them)
    static_assert(kQL != 2 || kQPhase == 2, "Q pieces in phase 2 only");
    constexpr int NQP = T / 1024;  // Q pieces per wave (its 64 rows): 16 / 8
    // a wave's block B starts kRowB rows after its block A (rows interleaved over the waves); the
    // wave's rows span kRowSpan rows from mw
    constexpr int kRowB = kBlockM / 2, kRowSpan = kRowB + 32;
    static_assert(kBlockM == 256, "4 waves x 2 blocks of 32 rows");
    static_assert(kRowSpan == kQoSpanRows, "the host's 32-bit offset bound (check_params) covers the wave's slab");
    // LDS: K slots 0,1 | V slots 0,1 (64 KiB at D = 128), so every fragment read is a per-lane base
    // plus a 16-bit immediate offset; then (kQL) the Q image, T bytes per wave.
    constexpr int KV0 = 0;
    constexpr int QOFF = 4 * T;
    __shared__ __attribute__((aligned(1024))) char lds[(kQL ? 8 : 4) * T];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31;
    const int h = lane >> 5;

    // sequence lengths of the current Q block: fixed for a dense launch; per batch row with
    // per-sequence ranges (xa.k_rng != nullptr, PathArgs: packed varlen or padded batches;
    // p.seqlen_* = upper bounds)
    const int D = (int)p.headdim;
    int Sq = (int)p.seqlen_q, Sk = (int)p.seqlen_kv;
    const float sc = p.softmax_scale;
    const float thr_raw = kRescaleThr / sc;
    int diag = Sk - Sq;
    int n_blocks = (Sk + kBlockN - 1) / kBlockN;

    // ---- persistent schedule ----------------------------------------------------------------
    // The grid holds about one workgroup per CU; each walks Q blocks (q-tile, q-head, batch) of its
    // own XCD's range of the XCD-aware logical order (decode_work), one round per gx workgroups of
    // the XCD, snake-ordered (odd rounds reversed) so that a heavy-first causal order balances
    // without a work queue. The next block's Q fragments and first K tile are fetched while the
    // current block drains its pipeline and stores O.
    // Head-packed blocks (xa.head_pack, causal GQA with a multiple of 4 q-heads per kv-head, multi-round
    // grids; dense, RoPE, per-sequence ranges, local window): a block is (batch, 4 consecutive q-heads of one kv group, 64-row q-tile),
    // wave w runs q-head 4 u + w on those 64 rows (block A the first 32, block B the next 32). Every
    // row keeps its own 32-row group and tile order, so the output is the plain layout's bit for bit;
    // but the causal diagonal of a block is ONE tile instead of four (plain 256-row blocks: 4 masked
    // tiles, 2 of them A-dead), and no tile is A-dead. Units: (batch, q-head quad u) rows of n_qtiles
    // (the host passes Sq / 64 q-tiles); g / 4 quads share a K/V stream.
    const bool hp = kCausal && xa.head_pack != 0;
    const int heads_u = hp ? (int)p.num_heads_q / 4 : (int)p.num_heads_q;             // head rows of the work order
    const int grp_u = hp ? (int)p.head_q_per_group / 4 : (int)p.head_q_per_group;  // of them per K/V stream
    const uint32_t nwg = (uint32_t)n_qtiles * (uint32_t)heads_u * (uint32_t)p.batch_size;
    const uint32_t xcd = blockIdx.x & 7, cx = blockIdx.x >> 3;
    const uint32_t gx = (gridDim.x - xcd + 7) >> 3;  // workgroups of this XCD
    // key-split blocks (below): the XCD-aware order runs over units whose pieces meet in ONE XCD's
    // list, so they meet through that XCD's L2. Plain split: a unit is a (batch, q-head, q-tile), its
    // two pieces next to each other in the list, walked by the snake. Pairs (xa.split_pairs): a unit
    // is a (batch, q-head, pair p) of the heavy q-tile Q - 1 - p and the light q-tile p on two
    // neighbouring workgroups, in one pass: workgroup 2u runs tiles [mid, n_end) of the heavy q-tile,
    // workgroup 2u + 1 its tiles [0, mid) and then the light q-tile whole, with mid putting the same
    // work on both (a block switch and the hand-off counted as FA_PAIR_SHIFT tiles).
    const bool spl = kCausal && xa.split_ws != nullptr;
    const bool pairs = spl && xa.split_pairs != 0;
    const int nqp = n_qtiles >> 1;  // (key-split launches: the host passes twice the plain q-tiles)
    const uint32_t nunits = pairs ? (uint32_t)((nqp + 1) >> 1) * (uint32_t)heads_u * p.batch_size : spl ? nwg >> 1 : nwg;
    const uint32_t nux = (nunits - xcd + 7) >> 3;  // units of this XCD
    const uint32_t cnt = pairs ? 2 * gx : spl ? 2 * nux : (nwg - xcd + 7) >> 3;  // Q blocks of this XCD
    auto nend_of = [&](const int t) __attribute__((always_inline)) {  // a dense causal q-tile's key tiles
        const int x = diag + min((t + 1) * (hp ? 64 : kBlockM), Sq);
        return min(x <= 0 ? 0 : (x + kBlockN - 1) / kBlockN, n_blocks);
    };
    // pairs: item k = rnd * gx + c of workgroup c; false if it has none
    auto pair_item = [&](const uint32_t k, Work &w) __attribute__((always_inline)) {
        const uint32_t r = k >= gx ? 1u : 0u, c = k - r * gx;
        if (c >= 2 * nux) return false;
        w = decode_work<kCausal>(nunits, xcd + 8 * (c >> 1), (nqp + 1) >> 1, heads_u, grp_u);
        const int pl = w.qtile, hv = nqp - 1 - pl;  // light and heavy q-tile (equal: the middle one)
        const int ch = nend_of(hv);
        const int mid = hv == pl ? ch >> 1 : max(0, ((ch - nend_of(pl)) >> 1) - FA_PAIR_SHIFT);
        if (!(c & 1)) {
            w.qtile = hv;
            w.kr = mid > 0 ? 2 | (mid << 2) : 0;
            return r == 0;
        }
        const int n1 = (mid > 0 ? 1 : 0) + (hv != pl ? 1 : 0);
        if ((int)r >= n1) return false;
        const bool piece = r == 0 && mid > 0;
        w.qtile = piece ? hv : pl;
        w.kr = piece ? 1 | (mid << 2) : 0;
        return true;
    };
    auto valid = [&](const uint32_t k) __attribute__((always_inline)) {
        Work w;
        return pairs ? pair_item(k, w) : k < cnt;
    };
    auto work_of = [&](const uint32_t k) __attribute__((always_inline)) {
        if (!spl)
            return decode_work<kCausal>(nwg, xcd + 8 * k, n_qtiles, heads_u, grp_u);
        Work w;
        if (pairs) {
            pair_item(k, w);
        } else {
            const uint32_t u = xcd + 8 * (k >> 1);
            // level-major (xa.split_rr, default): unit u is q-tile level u / rows (heaviest first) of row
            // u % rows, so every XCD holds a share of every level. decode_work's XCD-contiguous ranges gave
            // the first XCD the heaviest levels of one row -- 32 CUs of long pieces on one XCD, which clocks
            // lower when fully loaded: level-major measured +1.7 to +4.6 % (head-packed pieces: up to +21 %)
            if (xa.split_rr) {
                const uint32_t rows = (uint32_t)heads_u * p.batch_size, lv = u / rows, bh = u - lv * rows;
                w.qtile = nqp - 1 - (int)lv;
                w.hq = (int)(bh % (uint32_t)heads_u);
                w.b = (int)(bh / (uint32_t)heads_u);
            } else {
                w = decode_work<kCausal>(nunits, u, nqp, heads_u, grp_u);
            }
            w.kr = (k & 1 ? 2 : 1) | ((nend_of(w.qtile) >> 1) << 2);  // piece k & 1 of the halves
        }
        // (wave-uniform: said so, or the block's buffer descriptors may land in VGPRs, which the
        // LDS-DMA asm cannot take)
        w.qtile = __builtin_amdgcn_readfirstlane(w.qtile);
        w.hq = __builtin_amdgcn_readfirstlane(w.hq);
        w.b = __builtin_amdgcn_readfirstlane(w.b);
        w.kr = __builtin_amdgcn_readfirstlane(w.kr);
        return w;
    };
    auto block_of = [&](const uint32_t rnd) {
        return pairs ? rnd * gx + cx : rnd * gx + ((rnd & 1) ? gx - 1 - cx : cx);
    };
    uint32_t rnd = 0, kblk = block_of(0);
    if (!valid(kblk)) return;

    // Zigzag Q blocks (xa.zigzag, dense causal launches whose blocks fit one round of the grid):
    // block t pairs the 128-row segment t (block A) with segment nseg - 1 - t (block B), so every
    // block carries the same causal work -- a short top segment and a long bottom one -- instead of
    // the heaviest of the 256-row blocks setting the span (the C4 rank share at N = 8: 256 blocks on
    // 256 CUs). Block A's rows are always the workgroup's first 128 rows from m0 (the A-dead tiles
    // below follow); block B's rows start rowB rows after block A's (128 for the plain layout).
    const bool zz = kCausal && xa.zigzag;
    // Key-split causal blocks (xa.split_ws, dense causal launches whose blocks fit one round; the host
    // passes twice the q-tiles): item 2t + k is piece k of plain q-tile t, over the first (k = 0) or
    // second (k = 1) half of the block's key tiles. Both pieces of a q-tile are heavy-first
    // neighbours of one XCD's list, so the persistent snake puts a heavy piece and a light one on
    // every workgroup (two rounds) and no block is longer than half the longest q-tile. Their
    // combine is in the epilogue.
    auto qtile_of = [&](const Work &wk) { return wk.qtile; };
    int split_slot = 0;  // (batch, q-head, plain q-tile) of the current block: its workspace slot
    bool blk_split = false;  // the current block is a key-split piece
    auto geom_of = [&](const int qtile, const int sq, int &m0o, int &rowbo) __attribute__((always_inline)) {
        if (zz) {
            const int nseg = (sq + 127) >> 7, sB = nseg - 1 - qtile;
            m0o = qtile << 7;
            rowbo = sB > qtile ? (sB - qtile) << 7 : (nseg - qtile) << 7;  // (no partner: rows past Sq)
        } else if (hp) {
            m0o = qtile * 64;
            rowbo = 32;
        } else {
            m0o = qtile * kBlockM;
            rowbo = kRowB;
        }
    };
    int rowB = kRowB, rowB_next = kRowB;

    // per-block geometry (set_block)
    const char *qb, *kb, *vb;
    const char *cosb = nullptr, *sinb = nullptr;  // RoPE tables of this block's sequence (xa.cos)
    char *ob;
    int m0, mw, n_end, n_pipe;
    // local window (xa.window_left >= 0): tiles [j_lo, n_end) hold the block's visible keys, and
    // tiles below j_um have a score left of some row's window (masked like the diagonal)
    const int wl = xa.window_left;
    int j_lo = 0, j_um = 0;
    auto set_block = [&](const Work wk) {
        const int hq = hp ? 4 * wk.hq + wave : wk.hq, b = wk.b;  // (hp: wk.hq is the q-head quad)
        const int hkv = hq / (int)p.head_q_per_group;
        int64_t qrow0 = (int64_t)b * p.q_batch_stride, krow0 = (int64_t)b * p.k_batch_stride;
        int64_t vrow0 = (int64_t)b * p.v_batch_stride, orow0 = (int64_t)b * p.o_batch_stride;
        if (xa.q_rng) {  // this batch row's query rows and keys: absolute rows (the host zeroes the
                         // batch strides of ranged tensors; both ranges are given together here)
            const int q0 = xa.q_rng[b], k0 = xa.k_rng[b];
            Sq = xa.q_rng[b + xa.rng_hi] - q0;
            Sk = xa.k_rng[b + xa.rng_hi] - k0;
            diag = Sk - Sq;
            n_blocks = (Sk + kBlockN - 1) / kBlockN;
            qrow0 = (int64_t)q0 * p.q_seqlen_stride;
            orow0 = (int64_t)q0 * p.o_seqlen_stride;
            krow0 = (int64_t)k0 * p.k_seqlen_stride;
            vrow0 = (int64_t)k0 * p.v_seqlen_stride;
        }
        if (kExactD && xa.cos) {  // (RoPE: dense launches of exact-D instantiations only)
            const int64_t crow0 = (int64_t)b * xa.batch_stride;
            cosb = (const char *)xa.cos + 2 * crow0;
            sinb = (const char *)xa.sin + 2 * crow0;
        }
        qb = (const char *)p.q_ptr + 2 * (qrow0 + (int64_t)hq * p.q_head_stride);
        kb = (const char *)p.k_ptr + 2 * (krow0 + (int64_t)hkv * p.k_head_stride);
        vb = (const char *)p.v_ptr + 2 * (vrow0 + (int64_t)hkv * p.v_head_stride);
        ob = (char *)p.o_ptr + 2 * (orow0 + (int64_t)hq * p.o_head_stride);
        geom_of(qtile_of(wk), Sq, m0, rowB);
        // rows interleaved over the waves: block A = rows mw..mw+31 (the workgroup's first half),
        // block B = rows mw+rowB.. (its second half), so the last causal diagonal tiles hold no
        // score of any wave's block A (A-dead tiles, below)
        mw = hp ? m0 : m0 + wave * 32;
        n_end = n_blocks;
        if (kCausal) {
            // the workgroup's last row: block B's (zigzag: block A's when B has no partner segment)
            const int last = min(m0 + rowB < Sq ? m0 + rowB + kRowB : m0 + kRowB, Sq);
            const int x = diag + (zz ? last : min(m0 + (hp ? 64 : kBlockM), Sq));
            const int nb = x <= 0 ? 0 : (x + kBlockN - 1) / kBlockN;
            n_end = min(nb, n_blocks);
        }
        if (m0 >= Sq) n_end = 0;  // varlen: a q-tile past this sequence's end is empty
        // leading tiles with no masked score for any row of the WORKGROUP (pipelined; the same
        // count for all waves keeps the LDS ring and the barriers aligned)
        n_pipe = Sk / kBlockN;
        if (kCausal) {
            const int x = m0 + diag + 1;  // keys visible to the workgroup's first row
            n_pipe = min(n_pipe, x <= 0 ? 0 : x / kBlockN);
        }
        n_pipe = min(n_pipe, n_end);
        j_lo = j_um = 0;
        if (wl >= 0) {
            const int lo0 = m0 + diag - wl;                         // the first row's first key
            const int lo1 = min(m0 + (hp ? 64 : kBlockM), Sq) - 1 + diag - wl;  // the last row's
            j_lo = min(max(lo0, 0) / kBlockN, n_end);
            j_um = min((max(lo1, 0) + kBlockN - 1) / kBlockN, n_end);
        }
        if (spl) {  // a piece: tiles [0, mid) (kind 1) or [mid, n_end) (kind 2, the diagonal tiles among them)
            const int kind = wk.kr & 3, mid = wk.kr >> 2;
            // (selects, not branches: a three-way branch here let hipcc move the K / V tile descriptors
            // into VGPRs, which the LDS-DMA asm cannot take)
            j_lo = kind == 2 ? mid : j_lo;
            j_um = kind == 2 ? mid : j_um;
            n_end = kind == 1 ? mid : n_end;
            n_pipe = min(n_pipe, n_end);
            blk_split = kind != 0;
            split_slot = (b * heads_u + wk.hq) * nqp + wk.qtile;  // (hp: wk.hq is the quad, one record per wave)
        }
    };
    set_block(work_of(kblk));

    // ---- Q: this wave's 64 rows, B-operand fragments straight from HBM into AGPRs ----------
    // lane (h, r) of block X holds Q[mw + rowB*X + r][16*ks + 8*h + 0..7]; rows >= Sq read as 0.
    // Asynchronous: retired by the vmcnt wait ahead of the block's first barrier.
    auto load_q = [&]() __attribute__((always_inline)) {
        const int qs = (int)p.q_seqlen_stride;
        const rsrc_t qr = make_rsrc(qb + 2 * (int64_t)mw * qs, slab_bytes(min(Sq - mw, rowB + 32), qs, D));
        auto qoff = [&](const int X, const int ks) {
            const bool ok = kExactD || 16 * ks + 8 * h < D;  // columns past D read as 0
            return ok ? (rowB * X + r) * qs * 2 + 32 * ks + 16 * h : 0x7ffffff0;
        };
        static_for<2 * KS>([&](auto I) {
            constexpr int i = decltype(I)::value;
            agpr_qload<QB + 4 * i>(qr, qoff(i / KS, i % KS), i == 0);
        });
    };
    // RoPE fused into the Q load (xa.cos != nullptr, exact D): Q, cos and sin of the wave's 64 rows
    // into VGPRs, rotate-half in fp32, rounded once to T, then into the Q AGPRs. The rotation partner
    // of chunk 2ks+h is chunk 2(ks +- KS/2)+h -- the same lane. Issued in the block prologue (not
    // under the previous block's drain, whose S / P registers are live) and waited for there.
    const bool rope_q = kExactD && xa.cos != nullptr;
    auto load_q_rope = [&]() __attribute__((always_inline)) {
        const int qs = (int)p.q_seqlen_stride, cs = (int)xa.seq_stride;
        const int rows = min(Sq - mw, rowB + 32);
        const rsrc_t qr = make_rsrc(qb + 2 * (int64_t)mw * qs, slab_bytes(rows, qs, D));
        const rsrc_t cr = make_rsrc(cosb + 2 * (int64_t)mw * cs, slab_bytes(rows, cs, D));
        const rsrc_t sr = make_rsrc(sinb + 2 * (int64_t)mw * cs, slab_bytes(rows, cs, D));
        static_for<2>([&](auto XX) {
            constexpr int X = decltype(XX)::value;
            u32x4 qv[KS], cv[KS], sv[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                qv[ks] = __builtin_amdgcn_raw_buffer_load_b128(qr, (rowB * X + r) * qs * 2 + 32 * ks + 16 * h, 0, 0);
                cv[ks] = __builtin_amdgcn_raw_buffer_load_b128(cr, (rowB * X + r) * cs * 2 + 32 * ks + 16 * h, 0, 0);
                sv[ks] = __builtin_amdgcn_raw_buffer_load_b128(sr, (rowB * X + r) * cs * 2 + 32 * ks + 16 * h, 0, 0);
            }
            static_for<KS>([&](auto KK) {
                constexpr int ks = decltype(KK)::value;
                constexpr int pk = ks < KS / 2 ? ks + KS / 2 : ks - KS / 2;
                agpr_qset<QB + 4 * (X * KS + ks)>(DT::rope8(qv[ks], qv[pk], cv[ks], sv[ks], ks >= KS / 2));
            });
        });
    };
    // ---- Q by LDS-DMA (kQL): piece n (0..NQP-1) holds rows n*RPP.. of this wave's 64 in K's
    // swizzled image. Lane l writes image bytes n*1024 + 16 l = row n*RPP + 16 l / RB, slot
    // (16 l % RB) / 16; its source chunk is the slot XOR the row term of Geo::k_off, which for piece
    // n is the lane's piece-0 term XOR 4 * (n mod 4) (D = 128) or 4 * (n mod 2) (D = 64).
    const int qs_ = (int)p.q_seqlen_stride;
    const int q_row_l = (16 * lane) / RB;
    const int q_ch0 = G::k_off(q_row_l, ((16 * lane) % RB) / 16) % RB / 16;
    const uint32_t q_lane_off = (uint32_t)(q_row_l * qs_ * 2);
    const uint32_t q_lds = lds_u32(lds) + QOFF + wave * T;  // this wave's Q image
    auto q_piece = [&](const rsrc_t &qr, const int n, const int rb) __attribute__((always_inline)) {
        const int ch = q_ch0 ^ (4 * (n & (RB == 256 ? 3 : 1)));
        // image rows 0..31 are block A's rows mw.., rows 32..63 block B's rows mw+rb.. (rb: that
        // block's rowB)
        const int srow = n * ROWS_PER_PIECE + (n >= NQP / 2 ? rb - 32 : 0);
        uint32_t voff = q_lane_off + (uint32_t)(srow * qs_ * 2) + 16u * (uint32_t)ch;
        if (!kExactD && ch * 8 >= D) voff = 0x7ffffff0u;  // columns past D read as 0
        dma_one(qr, q_lds + n * 1024, (int)voff, true);
    };
    // this wave's Q slab of block wk (rows past the sequence read as 0); rb: that block's rowB
    auto q_rsrc_of = [&](const Work wk, int &rb) __attribute__((always_inline)) {
        int64_t row0 = (int64_t)wk.b * p.q_batch_stride;
        int sq = (int)p.seqlen_q;
        if (xa.q_rng) {
            const int q0 = xa.q_rng[wk.b];
            sq = xa.q_rng[wk.b + xa.rng_hi] - q0;
            row0 = (int64_t)q0 * qs_;
        }
        int m0n;
        geom_of(qtile_of(wk), sq, m0n, rb);
        const int mwn = hp ? m0n : m0n + wave * 32;
        const int hqn = hp ? 4 * wk.hq + wave : wk.hq;
        const char *qbn = (const char *)p.q_ptr + 2 * (row0 + (int64_t)hqn * p.q_head_stride);
        return make_rsrc_u(qbn + 2 * (int64_t)mwn * qs_, slab_bytes(min(sq - mwn, rb + 32), qs_, D));
    };
    // the next block (decoded once, in this block's prologue) and its Q pieces: qn of qnt issued
    // (kQL == 2: during this block's tiles)
    Work wk_next = {0, 0, 0};
    rsrc_t qnr = make_rsrc(nullptr, 0u);
    int qn = 0, qnt = 0;
    auto plan_next = [&]() __attribute__((always_inline)) {
        const uint32_t kn = block_of(rnd + 1);
        qn = 0;
        qnt = 0;
        if (valid(kn)) {
            wk_next = work_of(kn);
            if (kQL && !rope_q) {
                qnr = q_rsrc_of(wk_next, rowB_next);
                qnt = NQP;
            }
        }
    };
    if (!rope_q) {
        if constexpr (kQL != 0) {
            int rb0;
            const rsrc_t qr0 = q_rsrc_of(work_of(kblk), rb0);
            static_for<NQP>([&](auto N) { q_piece(qr0, decltype(N)::value, rb0); });
        } else {
            load_q();
        }
    }

    // ---- LDS-DMA staging: this wave writes pieces (wave*NP + n) of each K and V tile --------
    const int ks_ = (int)p.k_seqlen_stride, vs_ = (int)p.v_seqlen_stride;
    int kvo[NP], vvo[NP];
#pragma unroll
    for (int n = 0; n < NP; ++n) {
        const int row = (wave * NP + n) * ROWS_PER_PIECE + (16 * lane) / RB;
        const int slot = ((16 * lane) % RB) / 16;
        const int kch = G::k_off(row, slot) % RB / 16;  // the XOR swizzles are involutions
        const int vch = G::v_off(row, slot) % RB / 16;
        // piece n is issued with instruction offset n * 1024 (dma_q): its lane offsets carry
        // -n * 1024 (row >= n * ROWS_PER_PIECE and the row stride >= D keep them >= 0)
        kvo[n] = ((kExactD || kch * 8 < D) ? row * ks_ * 2 + 16 * kch : 0x7ffffff0) - n * 1024;
        vvo[n] = ((kExactD || vch * 8 < D) ? row * vs_ * 2 + 16 * vch : 0x7ffffff0) - n * 1024;
    }
    // tile j into ring slot `slot` (the block's tiles alternate slots from j_lo on), outside the
    // pipelined loop: every piece names M0 as an input (hipcc sets it; one wait state in the asm)
    auto stage_pieces = [&](const char *base, const int stride, const int j, const uint32_t m0v, const int *voff) {
        const int key0 = j * kBlockN;
        // (make_rsrc_u: the descriptor provably in SGPRs, whatever the register pressure)
        dma_tile<NP>(make_rsrc_u(base + 2 * (int64_t)key0 * stride, slab_bytes(min(Sk - key0, kBlockN), stride, D)),
                     m0v, voff);
    };
    auto stage_k = [&](const int j, const int slot) {
        stage_pieces(kb, ks_, j, lds_u32(lds + KV0 + slot * T) + wave * NP * 1024, kvo);
    };
    auto stage_v = [&](const int j, const int slot) {
        stage_pieces(vb, vs_, j, lds_u32(lds + KV0 + (2 + slot) * T) + wave * NP * 1024, vvo);
    };

    // ---- per-lane LDS read addresses -----------------------------------------------------
    const int g = lane >> 4;
    const int qq = (lane >> 2) & 3;
    const int pp = lane & 3;
    int v_addr[DTL];
#pragma unroll
    for (int dt = 0; dt < DTL; ++dt)
        v_addr[dt] = G::v_off(4 * (g >> 1) + qq, dt * 4 + 2 * (g & 1) + (pp >> 1)) + 8 * (pp & 1);
    int k_addr[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) k_addr[ks] = G::k_off(r, 2 * ks + h);
    // a block's Q image -> the Q AGPRs (its pieces have landed: the caller waited vmcnt; the
    // caller also waits lgkmcnt before the first S MFMA). The B-operand fragment (block X, k-step
    // ks) sits where K's A-operand fragment does, 32X rows on.
    auto q_from_lds = [&]() __attribute__((always_inline)) {
        static_for<2 * KS>([&](auto I) {
            constexpr int i = decltype(I)::value;
            agpr_qlds<QB + 4 * i>(q_lds + (i / KS) * 32 * RB + k_addr[i % KS]);
        });
    };
    bool q_in_agpr = false;  // the block's Q was read into the AGPRs at the switch
    // ---- state ------------------------------------------------------------------------------
    struct Sm {               // online-softmax state of one block (per lane: one query row)
        float m, nmsc, alpha;  // running max (unscaled), -m*sc (the exp2 argument's addend: no
                               // negation per tile), alpha of the last decision
        float mt;             // m + the rescale threshold (unscaled)
        float mE, mO;         // two max chains over the tile being reduced (mE then holds m_new)
        float l, t;           // this lane's half of the row sum over finished tiles; s0 sum of the
                              // tile being reduced (new scale, added to l at the end of the tile)
        uint64_t rmask;       // the decision's ballot (rows whose max outgrew m + threshold)
    };
    Sm st[2];
    f32x16 S[2][4];  // [tile parity][2 * block + half]: half 0 = keys 0-31, 1 = keys 32-63
    u32x4 P[2][8];   // [tile parity][4 * block + k-step]

    // ---- softmax units (each a few VALU instructions, placed between single MFMAs) ----------
    // max chain unit i (0..15) of block X: scores i of both halves
    auto u_max = [&](const int c, const int X, const int i) {
#ifdef FA_EXP_NOMAX  // (timing experiment: no max chain, no decision; m fixed per block; wrong results)
        if (true) { (void)c; (void)X; (void)i; return; }
#endif
        const f32x16 &s0 = S[c][2 * X], &s1 = S[c][2 * X + 1];
        float &mm = (i & 1) ? st[X].mO : st[X].mE;
        mm = (i < 2) ? fmaxf(s0[i], s1[i]) : fmaxf(mm, fmaxf(s0[i], s1[i]));
        pin(mm);
    };
    // the rescale decision of block X in two units: the row max and m_new; then m*sc and alpha
    auto u_dec = [&](const int c, const int X, const int k) {
        Sm &Z = st[X];
#if defined(FA_EXP_NODEC) || defined(FA_EXP_NOMAX)
        if (true) { (void)c; (void)k; Z.rmask = 0; return; }  // timing only
#endif
        if (k == 0) {
            // both lane halves hold the same row's m, so the ballot over the half-row maxima
            // needs no cross-half reduction; the row max itself is only needed to rescale
            const float mx = fmaxf(Z.mE, Z.mO);
            // the mask is materialised in SGPRs here, a gap before the branches that test it (a
            // branch on vcc straight from the compare measured slower)
            uint64_t bm = __builtin_amdgcn_ballot_w64(mx > Z.mt);
            asm volatile("" : "+s"(bm));
            Z.rmask = bm;
            Z.mE = mx;
            pin(Z.mE);
        } else if (__builtin_expect(Z.rmask != 0, 0)) {  // wave-uniform and rare: the rest only then
            const float m_new = fmaxf(Z.m, pair_max(Z.mE));
            const float seen = m_new > 0.5f * kNeg ? 1.f : 0.f;  // m_new * sc, or 0 before any visible key
            const float msc_new = m_new * sc * seen;
            // a row's first visible key: O and l are still 0 and exp2(0 - m*sc) may overflow
            Z.alpha = (Z.m <= 0.5f * kNeg) ? 0.f : __builtin_amdgcn_exp2f(-Z.nmsc - msc_new);
            Z.m = m_new;
            Z.mt = m_new + thr_raw;
            Z.nmsc = -msc_new;
            pin(Z.nmsc);
            pin(Z.alpha);
        }
    };
    // P = exp2(s * sc - m * sc) of score v of half hf of block X, in place
    auto u_exp = [&](const int c, const int X, const int hf, const int v) {
        f32x16 &s = S[c][2 * X + hf];
#if defined(FA_EXP_NOEXP)
        float x = __builtin_fmaf(s[v], sc, st[X].nmsc);
#else
        float x = __builtin_amdgcn_exp2f(__builtin_fmaf(s[v], sc, st[X].nmsc));
#endif
        pin(x);
        s[v] = x;
    };
    // row sum of P (half 0 -> t, half 1 -> l) and, for odd v, the rounded pair (v-1, v) into the
    // P.V operand of its 16-key k-step
    auto u_fin = [&](const int c, const int X, const int hf, const int v) {
        const f32x16 &s = S[c][2 * X + hf];
        {
            // the late scores (run after the tile's rescale) add into l, the early ones into t
            // (t restarts every tile: seeded with s[0] + s[1] at v == 1, no copy at v == 0)
            float &acc = (16 * hf + v >= kV0) ? st[X].l : st[X].t;
            if (!(hf == 0 && v == 0)) {
                acc = (hf == 0 && v == 1) ? s[0] + s[1] : acc + s[v];
                pin(acc);
            }
        }
        if (v & 1) {
            uint32_t w = DT::pack(s[v - 1], s[v]);
            pin(w);
            P[c][4 * X + 2 * hf + (v >> 3)][(v & 7) >> 1] = w;
        }
    };
    // o_zero: O holds no P.V yet (a block's first tile, where every row takes its first reference):
    // scaling it is a no-op, so only l is updated
    auto rescale = [&](const bool o_zero) {
        // The common l += t first; the rare branch (one for both blocks: a block that did not rescale
        // has alpha = 1) an if-then that redoes it as fma(l, alpha, t) from the saved l -- the value the
        // round-4 if-else computed. hipcc structurised that if-else into two flows with phi copies of the
        // block states on the common path: 14 instructions per two tiles, A/B C4 +0.6 %, C5 +0.8 %, C3
        // +0.5 %, C2 +0.1 %, bit-identical (profiles/r5e_ab_*.log)
        const float l0 = st[0].l, l1 = st[1].l;
#pragma unroll
        for (int X = 0; X < 2; ++X) st[X].l += st[X].t;
        if (__builtin_expect((st[0].rmask | st[1].rmask) != 0, 0)) {
            if (!o_zero) {
                agpr_scale<DTL, false>(st[0].alpha);
                agpr_scale<DTL, true>(st[1].alpha);
            }
            st[0].l = __builtin_fmaf(l0, st[0].alpha, st[0].t);
            st[1].l = __builtin_fmaf(l1, st[1].alpha, st[1].t);
            st[0].alpha = 1.f;
            st[1].alpha = 1.f;
        }
    };

    const uint32_t lds_base = lds_u32(lds) + wave * NP * 1024;  // this wave's pieces of slot 0
    // O = 0 (FA_ZERO_MFMA: 2 * DTL MFMAs 0 * 0 + 0, one issue slot per 16 AGPRs, worked off by the matrix
    // pipe beside the VALU that follows; the block's first P.V MFMA, tile jb's phase 2, is the first reader)
    auto zero_o = [&]() __attribute__((always_inline)) {
#if FA_ZERO_MFMA
        u32x4 z = {0, 0, 0, 0};
        asm volatile("" : "+v"(z));
        if constexpr (DTL == 4) fa_agpr_zmfma_4(z); else fa_agpr_zmfma_2(z);
#else
        if constexpr (DTL == 4) fa_agpr_zero_4(); else fa_agpr_zero_2();
#endif
    };
    // Deferred epilogue (FA_EPI_OVL): a dense block that another block follows leaves O in the AGPRs
    // and its stores to the next block's first tile, whose phase-1 gaps are free of softmax work (no
    // tile -1): unit u is one 16-B store per lane (block X, d-tile dt, row pair gp) -- 8 AGPR reads,
    // O / l, packing and a half-wave swap, as store_block
    bool epi_pending = false;
    float epi_inv0 = 1.f, epi_inv1 = 1.f;
    rsrc_t epi_orr = make_rsrc(nullptr, 0u);
    int epi_rowb = 0;
    auto epi_unit = [&](auto U) __attribute__((always_inline)) {
        constexpr int u = decltype(U)::value;
        constexpr int X = u / (2 * DTL), dt = (u % (2 * DTL)) / 2, gp = (u & 1) * 2;
        float x[8];
        agpr_read8<16 * DTL * X + 16 * dt + 4 * gp>(x);
        const float inv = X ? epi_inv1 : epi_inv0;
        const uint32_t a0 = DT::pack(x[0] * inv, x[1] * inv), a1 = DT::pack(x[2] * inv, x[3] * inv);
        const uint32_t b0 = DT::pack(x[4] * inv, x[5] * inv), b1 = DT::pack(x[6] * inv, x[7] * inv);
        const auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
        const auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
        const int d0 = dt * 32 + 8 * (gp + h);
        const int orow = r * (int)p.o_seqlen_stride * 2 + (X ? epi_rowb : 0);
        __builtin_amdgcn_raw_buffer_store_b128((u32x4){x0[0], x1[0], x0[1], x1[1]}, epi_orr,
                                               (kExactD || d0 < D) ? orow + 2 * d0 : 0x7ffffff0, 0, 0);
    };
    // ---- softmax split: of each block's 32 scores of a tile (index q = 16 * half + v), q < kV0 are
    // exponentiated in phase 2 right after the tile's rescale decision ("early", summed into t), the
    // rest in the next phase 1 ("late", summed into l).
    struct Late {  // late unit u: block u & 1, score index q = kV0 + u / 2 (q = 16 * half + v)
        static constexpr int hf(int u) { return (kV0 + (u >> 1)) >> 4; }
        static constexpr int v(int u) { return (kV0 + (u >> 1)) & 15; }
    };
    // ---- phase 1: S[c] = K.Q^T for both blocks (4*KS single MFMAs) ----------------------------
    // gap g (after MFMA g): next k-step's K fragments (gaps 4ks, 4ks+1; Q is in AGPRs), one LDS-DMA piece
    // (gap 4ks+2: K_{j+1} pieces, then V_j pieces), and with SM2 the second softmax half of the
    // tile of parity pr (32 units: block u&1, score u>>1 of half 1).
    constexpr int G1 = 4 * KS;
    // phase 2's first-k-step V^T fragments, read in phase 1's last k-step (its K fragment buffer is
    // free there; V_{j-1}'s ring slot is not a DMA target in this tile) instead of all at the phase
    // boundary: A/B C2 +0.9 %, C4 +0.5 %, C5 +1.1 %, bit-identical (profiles/r4_ab_batch1.log)
    u32x4 va_pre[DTL];
    // AD (A-dead tiles, causal diagonal): bit 0 = block A has no visible score in this tile (its S
    // MFMAs are skipped), bit 1 = nor in the previous tile (its late softmax units are skipped);
    // bit 2 = read phase 2's first V^T fragments into va_pre (with SM2)
    auto phase1 = [&](const char *K, auto PAR, auto SM2, auto DMA, const rsrc_t &kq, const rsrc_t &vq, auto AD)
        __attribute__((always_inline)) {
        constexpr int c = decltype(PAR)::value, pr = c ^ 1;
        constexpr bool do_sm = decltype(SM2)::value, do_dma = decltype(DMA)::value;
        constexpr bool sdead = decltype(AD)::value & 1, pdead = decltype(AD)::value & 2;
        constexpr bool vpre = decltype(AD)::value & 4;
        // bit 3: a block's first tile with the previous block's deferred O stores (FA_EPI_OVL): its K / V
        // pieces go first (gaps 0 .. 2 NP - 1), so the tile's closing wait can leave the stores in flight
        constexpr bool epi = decltype(AD)::value & 8;
        u32x4 kf[2][2];  // [buffer][key half]
#pragma unroll
        for (int x = 0; x < 2; ++x) kf[0][x] = *(const u32x4 *)(K + x * 32 * RB + k_addr[0]);
        static_for<G1>([&](auto G) {
            constexpr int g = decltype(G)::value;
            constexpr int ks = g >> 2, i = g & 3, cb = ks & 1;
            // one counted wait per k-step (its two K fragments were read a whole k-step ahead)
#ifndef FA_EXP_NOLGKM1
            if constexpr (ks > 0 && i == 0) __builtin_amdgcn_s_waitcnt(kLgkm0);
#endif
            if constexpr (sdead && i < 2) {
            } else {
                mfma_sq<F, QB + 4 * ((i >> 1) * KS + ks)>(ks == 0, S[c][i], kf[cb][i & 1]);
            }
            // the MFMA alone in its scheduling region: the pre-RA scheduler would otherwise hoist
            // this gap's (independent) VALU above it, into the previous gap
            FA_SCHED_FENCE();
            if constexpr (ks + 1 < KS && i == 0) {
#if defined(FA_EXP_HALFLDS) || defined(FA_EXP_HALFK)  // (timing experiment of the stamps build only:
                                                      // half the K fragment reads, wrong results)
                if constexpr ((ks + 1) & 1) {
#ifdef FA_EXP_HALF_XOR  // the skipped fragment: the previous one with mantissa bits flipped, so the MFMA
                        // operands still toggle like real data (an opaque register is near-constant
                        // data: the chip then clocks up for the data, not for the saved LDS reads)
                    static_for<4>([&](auto E) {
                        constexpr int e = decltype(E)::value;
                        kf[cb ^ 1][0][e] = kf[cb][0][e] ^ 0x01ff01ffu;
                        kf[cb ^ 1][1][e] = kf[cb][1][e] ^ 0x01ff01ffu;
                    });
#else
                    asm volatile("" : "=v"(kf[cb ^ 1][0]), "=v"(kf[cb ^ 1][1]));
#endif
                } else
#endif
                {
#ifdef FA_EXP_NOLGKM1  // (timing experiment, stamps builds only: K reads the compiler cannot see and no
                       // k-step waits -- how much of phase 1 the per-k-step LDS waits cost; wrong results)
                    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kf[cb ^ 1][0]) : "v"(k_addr[ks + 1]), "i"(KV0 + c * T));
                    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(kf[cb ^ 1][1]) : "v"(k_addr[ks + 1]), "i"(KV0 + c * T + 32 * RB));
#else
                    kf[cb ^ 1][0] = *(const u32x4 *)(K + k_addr[ks + 1]);
                    kf[cb ^ 1][1] = *(const u32x4 *)(K + 32 * RB + k_addr[ks + 1]);
#endif
                }
            }
            if constexpr (do_sm && vpre && ks == KS - 1 && i < DTL) {
                static_for<2>([&](auto E) {
                    constexpr int n = 2 * i + decltype(E)::value;
                    const u32x2 x = tr_read(K + (2 + pr - c) * T + (n & 1) * 8 * RB + v_addr[n >> 1]);
                    va_pre[n >> 1][2 * (n & 1)] = x[0];
                    va_pre[n >> 1][2 * (n & 1) + 1] = x[1];
                });
            }
            if constexpr (do_dma && (epi ? g < 2 * NP : i == 2)) {
                constexpr int n = epi ? g : ks;  // (piece)
                if constexpr (n < NP) dma_q_at<pr * T, n * 1024>(kq, lds_base, kvo[n]);
                else dma_q_at<(2 + c) * T, (n - NP) * 1024>(vq, lds_base, vvo[n - NP]);
            }
            if constexpr (epi) {
                static_for<kOStores>([&](auto U) {
                    constexpr int u = decltype(U)::value;
                    if constexpr (2 * NP + (u * (G1 - 2 * NP)) / kOStores == g) {
                        if (epi_pending) epi_unit(U);
                    }
                });
            }
            // the next block's Q: kQPT pieces per tile, in evenly spaced gaps
            if constexpr (kQL == 2 && kQPhase == 1 && do_dma && i == 3 && (ks * kQPT) % KS == 0) {
                if (qn < qnt) {
                    q_piece(qnr, qn, rowB_next);
                    ++qn;
                }
            }
            if constexpr (do_sm) {
                static_for<kNL>([&](auto U) {
                    constexpr int u = decltype(U)::value;
                    if constexpr ((u * G1) / kNL == g && !(pdead && (u & 1) == 0)) {
                        u_exp(pr, u & 1, Late::hf(u), Late::v(u));
                        if constexpr (u >= 2) u_fin(pr, u & 1, Late::hf(u - 2), Late::v(u - 2));
                    }
                });
            }
            FA_SCHED_FENCE();
#ifdef FA_STAMPS_FINE
            if constexpr (do_sm && do_dma && g == G1 / 2 - 1) st_f[3] = (uint32_t)__builtin_amdgcn_s_memtime();
#endif
        });
        if constexpr (do_sm) {
            if constexpr (!pdead) u_fin(pr, 0, Late::hf(kNL - 2), Late::v(kNL - 2));
            u_fin(pr, 1, Late::hf(kNL - 1), Late::v(kNL - 1));
        }
    };
    // the same second softmax half without MFMAs (drain and masked tiles)
    auto sm2_all = [&](auto PAR, auto AD) __attribute__((always_inline)) {
        constexpr int c = decltype(PAR)::value;
        constexpr int X0 = (decltype(AD)::value & 2) ? 1 : 0;  // (block A dead in tile c: B only)
        static_for<32 - kV0>([&](auto VV) {  // the late scores
            constexpr int q = kV0 + decltype(VV)::value;
            static_for<2>([&](auto XX) {
                if constexpr (decltype(XX)::value >= X0) {
                    u_exp(c, decltype(XX)::value, q >> 4, q & 15);
                    u_fin(c, decltype(XX)::value, q >> 4, q & 15);
                }
            });
        });
    };

    // ---- phase 2: O^T += V^T.P^T for both blocks (8*DTL single MFMAs into the AGPRs) ----------
    // gap g (kk = g / 2DTL, i = g % 2DTL; MFMA: block i / DTL, d-tile i % DTL): V^T read i of
    // k-step kk+1, and with SM1 the first softmax half of the tile of parity cs (schedule below).
    constexpr int NPK = 2 * DTL;  // MFMAs per 16-key step
    constexpr int G2 = 4 * NPK;
    constexpr int GQ = G2 / 8;  // 4 (D=128) / 2 (D=64)
    // exp unit e (0..31) -> block / score: A0..A4, then B and A alternating, then B11..B15
    constexpr int NE = 2 * kV0;  // early exp units of phase 2
    struct Ex {  // early exp unit e (0..NE-1) -> block / score: A0..A3, then B and A alternating, then B's tail
        // head: A's units before B's first one, which waits for B's rescale decision
        static constexpr int hd() {
            int hh = 4;
            while (GQ + 2 + (hh * (G2 - GQ - 2)) / NE < 2 * GQ + 1) ++hh;
            return hh;
        }
        static constexpr int mid() { return 2 * (kV0 - hd()); }
        static constexpr int blk(int e) { return e < hd() ? 0 : (e < hd() + mid() ? (((e - hd()) & 1) ? 0 : 1) : 1); }
        static constexpr int v(int e) {  // score index q = 16 * half + v
            return e < hd() ? e
                            : (e < hd() + mid() ? (((e - hd()) & 1) ? hd() + ((e - hd()) >> 1) : (e - hd()) >> 1)
                                                : (kV0 - hd()) + (e - hd() - mid()));
        }
        static constexpr int gap(int e) { return GQ + 2 + (e * (G2 - GQ - 2)) / NE; }
        static constexpr int max_gap(int X, int m) { return X * GQ + (m * GQ) / 16; }
        static constexpr int dec_gap(int X, int k) { return (X + 1) * GQ + (GQ == 2 ? 0 : k); }
    };
    static_assert([] {  // the schedule respects max -> decision -> exp of each block, and fits
        for (int X = 0; X < 2; ++X) {
            if (Ex::dec_gap(X, 0) < Ex::max_gap(X, 15) || Ex::dec_gap(X, 1) < Ex::dec_gap(X, 0)) return false;
            if (Ex::max_gap(X, 15) >= G2) return false;
        }
        int seen[2][32] = {};
        for (int e = 0; e < NE; ++e) {
            if (Ex::gap(e) < Ex::dec_gap(Ex::blk(e), 1) || Ex::gap(e) >= G2) return false;
            if (e > 0 && Ex::gap(e) < Ex::gap(e - 1)) return false;
            if (Ex::v(e) < 0 || Ex::v(e) >= kV0 || seen[Ex::blk(e)][Ex::v(e)]++) return false;  // v: score index q
        }
        return true;
    }(), "phase-2 softmax schedule");
    // AD: bit 0 = block A has no visible score in tile cs (its early softmax units are skipped),
    // bit 1 = nor in tile cp (its P.V MFMAs are skipped: P is 0); bit 2 = the first V^T fragments
    // are in va_pre (with SM1)
    auto phase2 = [&](const char *V, auto PPV, auto PSM, auto SM1, auto AD) __attribute__((always_inline)) {
        constexpr int cp = decltype(PPV)::value, cs = decltype(PSM)::value;
        constexpr bool do_sm = decltype(SM1)::value == 1;
        constexpr bool sdead = decltype(AD)::value & 1, pdead = decltype(AD)::value & 2;
        constexpr bool vpre = decltype(AD)::value & 4;  // (phase 1 read the first V^T fragments)
        u32x4 va[2][DTL];
        auto rd = [&](const int kk, const int n, u32x4 *dst) {
            const int rowoff = ((kk >> 1) * 32 + (kk & 1) * 16) * RB + (n & 1) * 8 * RB;
#ifdef FA_EXP_NOLGKM2  // (timing experiment, as FA_EXP_NOLGKM1 for the V^T reads of phase 2)
            u32x2 x;
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(x) : "v"(v_addr[n >> 1]), "i"(KV0 + (2 + cp) * T + rowoff));
#else
            const u32x2 x = tr_read(V + rowoff + v_addr[n >> 1]);
#endif
            dst[n >> 1][2 * (n & 1)] = x[0];
            dst[n >> 1][2 * (n & 1) + 1] = x[1];
        };
        constexpr bool do_late = decltype(SM1)::value == 2;  // (the drain: tile cp's late softmax)
        if constexpr (do_sm && vpre) {  // (read in phase 1 of the same iteration)
#pragma unroll
            for (int n = 0; n < DTL; ++n) va[0][n] = va_pre[n];
        } else {
#pragma unroll
            for (int n = 0; n < 2 * DTL; ++n) rd(0, n, va[0]);
        }
        static_for<G2>([&](auto G) {
            constexpr int g = decltype(G)::value;
            constexpr int kk = g / NPK, i = g % NPK;
            constexpr int X = i / DTL, dt = i % DTL;
            // one counted wait per 16-key step: its V^T fragments were read in the first DTL gaps
            // of the previous step, two per gap
#ifndef FA_EXP_NOLGKM2
            if constexpr (kk > 0 && i == 0) __builtin_amdgcn_s_waitcnt(kLgkm0);
#endif
            if constexpr (!(pdead && X == 0)) agpr_mfma<F, X * 16 * DTL + 16 * dt, true>(va[kk & 1][dt], P[cp][4 * X + kk]);
            FA_SCHED_FENCE();  // (see phase 1)
            if constexpr (kk + 1 < 4 && i < DTL) {
#if defined(FA_EXP_HALFLDS) || defined(FA_EXP_HALFV)  // (timing experiment, as in phase 1: half the V^T reads)
                if constexpr ((kk + 1) & 1) {
#ifdef FA_EXP_HALF_XOR
                    static_for<4>([&](auto E) {
                        constexpr int e = decltype(E)::value;
                        va[(kk + 1) & 1][i][e] = va[kk & 1][i][e] ^ 0x01ff01ffu;
                    });
#else
                    asm volatile("" : "=v"(va[(kk + 1) & 1][i]));
#endif
                } else
#endif
                {
                    rd(kk + 1, 2 * i, va[(kk + 1) & 1]);
                    rd(kk + 1, 2 * i + 1, va[(kk + 1) & 1]);
                }
            }
            // (kQPhase 2) the next block's Q pieces early in phase 2, where no K/V DMA is issued
            if constexpr (kQL == 2 && kQPhase == 2 && do_sm && g % 2 == 1 && g < 2 * kQPT) {
                if (__builtin_expect(qn < qnt, 0)) {  // (out of line: the common path falls through)
                    q_piece(qnr, qn, rowB_next);
                    ++qn;
                }
            }
            if constexpr (do_late && g <= 16) {
                // late score v = g of both blocks (P of k-steps 2, 3: their MFMAs start at gap 16),
                // the row sum and pack of score g - 1 a gap after its exp
                static_for<2>([&](auto XX) {
                    constexpr int X2 = decltype(XX)::value;
                    if constexpr (!(pdead && X2 == 0)) {
                        if constexpr (g < 16) u_exp(cp, X2, 1, g);
                        if constexpr (g > 0) u_fin(cp, X2, 1, g - 1);
                    }
                });
            }
            if constexpr (do_sm) {
                static_for<32>([&](auto M) {
                    constexpr int X2 = decltype(M)::value >> 4, m = decltype(M)::value & 15;
                    if constexpr (Ex::max_gap(X2, m) == g && !(sdead && X2 == 0)) u_max(cs, X2, m);
                });
                static_for<4>([&](auto K2) {
                    constexpr int X2 = decltype(K2)::value >> 1, k = decltype(K2)::value & 1;
                    if constexpr (Ex::dec_gap(X2, k) == g && !(sdead && X2 == 0)) u_dec(cs, X2, k);
                });
                static_for<NE>([&](auto E) {
                    constexpr int e = decltype(E)::value;
                    if constexpr (!(sdead && Ex::blk(e) == 0)) {
                        if constexpr (Ex::gap(e) + 1 == g) u_fin(cs, Ex::blk(e), Ex::v(e) >> 4, Ex::v(e) & 15);
                        if constexpr (Ex::gap(e) == g) u_exp(cs, Ex::blk(e), Ex::v(e) >> 4, Ex::v(e) & 15);
                    }
                });
            }
            FA_SCHED_FENCE();
#ifdef FA_STAMPS_FINE
            if constexpr (do_sm && (g + 1) % (G2 / 4) == 0 && g + 1 < G2)
                st_f[(g + 1) / (G2 / 4) - 1] = (uint32_t)__builtin_amdgcn_s_memtime();
#endif
        });
        if constexpr (do_sm) {
            static_for<NE>([&](auto E) {
                constexpr int e = decltype(E)::value;
                if constexpr (Ex::gap(e) == G2 - 1 && !(sdead && Ex::blk(e) == 0))
                    u_fin(cs, Ex::blk(e), Ex::v(e) >> 4, Ex::v(e) & 15);
            });
        }
    };
    // the same first softmax half without MFMAs (masked tiles)
    auto sm1_all = [&](auto PAR) __attribute__((always_inline)) {
        constexpr int c = decltype(PAR)::value;
        static_for<2>([&](auto XX) {
            constexpr int X = decltype(XX)::value;
            static_for<16>([&](auto M) { u_max(c, X, decltype(M)::value); });
            u_dec(c, X, 0);
            u_dec(c, X, 1);
            static_for<kV0>([&](auto VV) {  // the early scores (the late ones: sm2_all)
                constexpr int q = decltype(VV)::value;
                u_exp(c, X, q >> 4, q & 15);
                u_fin(c, X, q >> 4, q & 15);
            });
        });
    };

    // pipelined loop: running tile pointers (no 64-bit multiply per tile) and descriptor sizes
    // without branches; a full tile spans full_k / full_v bytes, the Sk tail tile fewer, a tile
    // past Sk none. (A descriptor carried across tiles as a plain u32x4 and advanced in place
    // saved its assembly, but hipcc may then keep it in VGPRs, which an asm "s" operand cannot
    // take: rsrc_t keeps it in SGPRs.)
    const uint32_t full_k = slab_bytes(kBlockN, ks_, D), full_v = slab_bytes(kBlockN, vs_, D);
    const int64_t step_k = 2 * (int64_t)kBlockN * ks_, step_v = 2 * (int64_t)kBlockN * vs_;
    const char *kp, *vp;  // K tile j + 1 / V tile j of iteration j
    int kfe = 0;        // tiles below kfe are full (this block's Sk)
    uint32_t k_last = 0;  // the bytes of K tile kfe (the Sk tail, or 0)
    auto tile_bytes = [&](const int key0, const uint32_t full, const int stride) {
        const int rows = Sk - key0;
        return rows >= kBlockN ? full : slab_bytes(rows, stride, D);
    };

    // Tile parity: a block's first tile j_lo runs with parity 1 (its own iteration, iter_first), the
    // pipelined tiles j > j_lo with parity (j - j_lo - 1) & 1; parity c = K ring slot c, V slot c,
    // S[c], P[c].
    stage_k(j_lo, 1);  // the first block's first K tile (its Q is in flight above)
    for (;;) {
    // ---- block prologue: Q and K_0 of this block are in flight ------------------------------
#ifdef FA_STAMPS
    st_t0 = (uint32_t)__builtin_amdgcn_s_memtime();
    st_rt0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int i = 0; i < 8; ++i) st_acc[i] = 0;
#ifdef FA_STAMPS_FINE
#pragma unroll
    for (int i = 0; i < 4; ++i) st_fa[i] = 0;
#endif
#endif
    kp = kb + (j_lo + 1) * step_k;
    vp = vb + j_lo * step_v;
    kfe = Sk / kBlockN;
    k_last = tile_bytes(kfe * kBlockN, full_k, ks_);
    if (rope_q) load_q_rope();
#pragma unroll
    for (int X = 0; X < 2; ++X) {
        st[X] = {kNeg, 0.f, 1.f, kNeg + thr_raw, kNeg, kNeg, 0.f, 0.f, 0ull};
#ifdef FA_EXP_NOMAX  // (timing: a reference max that keeps N(0,1) scores' P in (0, ~2])
        st[X].nmsc = -5.77f;
#endif
    }
#if FA_EPI_OVL
    // (O is zeroed in the first tile, after the previous block's deferred epilogue has read it)
#elif FA_ZERO_MFMA
    zero_o();
#else
    if constexpr (DTL == 4) fa_agpr_zero_4(); else fa_agpr_zero_2();
#endif
    // (no pipeline fill: the block's first tile runs its own iteration without the P.V and late
    // softmax of an empty tile -1, iter FIRST below)
    // Q, K_0 landed. After the first block the previous block's O stores were issued after these
    // loads: leave them in flight (vmcnt counts stores too, in issue order)
    // (FA_EPI_OVL: a dense block defers its stores into the next block's first tile, so only a key-split
    // block's combining piece leaves stores in flight here)
#ifdef FA_STAMPS
    const uint32_t st_w0 = (uint32_t)__builtin_amdgcn_s_memtime();
#endif
    if (rnd == 0 || (FA_EPI_OVL && !spl)) dma_wait(); else __builtin_amdgcn_s_waitcnt(vmcnt_enc(kOStores));
#ifdef FA_STAMPS
    st_acc[6] = (uint32_t)__builtin_amdgcn_s_memtime() - st_w0;  // (the wait for this block's Q and K_0)
#endif
    if (kQL && !rope_q && !q_in_agpr) q_from_lds();
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    plan_next();
    __syncthreads();  // visible to every wave
    FA_STAMP(s_pro);

    // ---- pipelined tiles: iteration j = P1(S_j || softmax half 2 of j-1, DMA K_{j+1}, V_j),
    //      P2(O += P_{j-1} V_{j-1} || softmax half 1 of j), rescale, barrier -------------------
    // causal diagonal / Sk tail: scores of keys past a row's last visible key -> kNeg
    // row0: the block's first query row (wave-uniform; the lane's row is row0 + r). Score i of half
    // hf is key key0 + 32 hf + c_i + 4 h with c_i = (i & 3) + 8 (i >> 2): against the lane's last
    // visible key minus key0 + 4 h, each score is one compare with an inline constant and a select.
    // (inline asm: two independent compare -> select chains per score pair, one through VCC and one
    // through an SGPR pair, so no select waits on the compare just before it; compiled C++ turned
    // the same selects into SALU-mask chains that cost ~1.9k cycles per masked tile, stamps r3)
    auto mask = [&](f32x16 &s0, f32x16 &s1, const int row0, const int key0) __attribute__((always_inline)) {
        if (wl < 0) {
            const int e = (kCausal ? min(Sk - 1, row0 + r + diag) : Sk - 1) - key0 - 4 * h;
            float neg = kNeg;
            asm volatile("" : "+v"(neg));  // (materialised once, in a VGPR)
            static_for<16>([&](auto I) { mask_pair<decltype(I)::value>(s0, s1, e, neg); });
        } else {  // and keys left of the row's window
            const int row = row0 + r;
            const int e = (kCausal ? min(Sk - 1, row + diag) : Sk - 1) - key0 - 4 * h;
            const int f = row + diag - wl - key0 - 4 * h;
            float neg = kNeg;
            asm volatile("" : "+v"(neg));
            static_for<16>([&](auto I) { mask_pair_win<decltype(I)::value>(s0, s1, e, f, neg); });
        }
    };
    // does tile key0 hold a hidden score of rows row0..row0+31 (wave-uniform)? keys past the first
    // row's last visible key (causal diagonal, Sk tail), or left of the last row's window
    auto hides = [&](const int row0, const int key0) __attribute__((always_inline)) {
        const int lim = kCausal ? min(Sk - 1, row0 + diag) : Sk - 1;
        return key0 + kBlockN - 1 > lim || (wl >= 0 && key0 < row0 + 31 + diag - wl);
    };
    // the first softmax half of a block's first tile on its own (iter FIRST: no P.V to pair it with;
    // AD bit 0: block A dead)
    auto sm1_first = [&](auto PAR, auto AD) __attribute__((always_inline)) {
        constexpr int c = decltype(PAR)::value;
        constexpr int X0 = (decltype(AD)::value & 1) ? 1 : 0;
        static_for<2>([&](auto XX) {
            constexpr int X = decltype(XX)::value;
            if constexpr (X >= X0) {
                static_for<16>([&](auto M) { u_max(c, X, decltype(M)::value); });
                u_dec(c, X, 0);
                u_dec(c, X, 1);
                static_for<kV0>([&](auto VV) {  // the early scores (the late ones: the next tile's phase 1)
                    constexpr int q = decltype(VV)::value;
                    u_exp(c, X, q >> 4, q & 15);
                    u_fin(c, X, q >> 4, q & 15);
                });
            }
        });
    };
    // MASKED: 0 = no masked score, 1 = masked (diagonal / tail / window), 2 = masked and block A
    // dead in tile j (no row of any wave's block A sees a key of it), 3 = A dead in tiles j and j-1.
    // FIRST: the block's first tile j_lo (parity 1). The pipeline is not filled with an empty tile
    // -1: phase 1 computes S(j_lo) and issues the DMA of K_{j_lo+1} and V_{j_lo} with no late softmax
    // beside it, and "phase 2" is the first softmax half of j_lo alone (no P.V of a tile -1: 32 MFMAs
    // of zeros and their V^T reads in rounds 1-4, and the zeroed V slot behind them).
    auto iter = [&](const int j, auto PAR, auto MASKED, auto FIRST) __attribute__((always_inline)) {
        constexpr int c = decltype(PAR)::value, pr = c ^ 1;
        constexpr int mk = decltype(MASKED)::value;
        constexpr bool first = decltype(FIRST)::value;
        static_assert(!first || (c == 1 && mk != 3), "first tile: parity 1, no previous tile");
        // (bit 2: phase 2's first V^T fragments read in phase 1 -- unmasked tiles only: in a masked one
        // they would stay live through the mask step, where the causal kernels have no VGPR to spare)
        using AD = IC<(mk == 2 ? 1 : mk == 3 ? 3 : 0) | (mk == 0 ? 4 : 0) | (first && FA_EPI_OVL ? 8 : 0)>;
#if FA_EPI_OVL
        const bool had_epi = first && epi_pending;
#endif
        if constexpr (mk >= 2) {  // block A takes no decision and adds no row sum in tile j
            st[0].rmask = 0;
            st[0].t = 0.f;
        }
        FA_STAMP(sa);
        // (unmasked: j + 1 <= n_pipe <= kfe, V_j full)
        const rsrc_t kq = make_rsrc(kp, mk == 0 ? (j + 1 < kfe ? full_k : k_last) : tile_bytes((j + 1) * kBlockN, full_k, ks_));
        const rsrc_t vq = make_rsrc(vp, mk == 0 ? full_v : tile_bytes(j * kBlockN, full_v, vs_));
        // FA_EXP_*: timing experiments of the stamps build only (results are garbage)
#if defined(FA_EXP_NOSM)
        phase1(lds + KV0 + c * T, PAR, IC<0>{}, IC<1>{}, kq, vq, AD{});
#elif defined(FA_EXP_NODMA)
        phase1(lds + KV0 + c * T, PAR, IC<!first>{}, IC<0>{}, kq, vq, AD{});
#else
        phase1(lds + KV0 + c * T, PAR, IC<!first>{}, IC<1>{}, kq, vq, AD{});
#endif
        kp += step_k;
        vp += step_v;
#if FA_EPI_OVL
        if constexpr (first) {  // the previous block's O has been read: O = 0 for this block
            zero_o();
            epi_pending = false;
        }
#endif
        // the first tile's softmax reads S right after its MFMAs (no P.V MFMAs in between)
        if constexpr (first) s_ready4(S[c][0], S[c][1], S[c][2], S[c][3]);
#ifndef FA_EXP_NOMASK  // (timing experiment of the stamps build only: no mask step, wrong results)
        if constexpr (mk != 0) {  // diagonal / tail tile: mask S before phase 2
            // (per wave and block: only where some score of its 32 rows is hidden; on a causal
            // diagonal that is half of the wave-blocks of the workgroup's masked tiles)
            const int key0 = j * kBlockN;
            if constexpr (mk == 1) {
                if (hides(mw, key0)) {
                    if constexpr (!first) s_ready(S[c][0], S[c][1]);
                    mask(S[c][0], S[c][1], mw, key0);
                }
            }
            if (hides(mw + rowB, key0)) {
                if constexpr (!first) s_ready(S[c][2], S[c][3]);
                mask(S[c][2], S[c][3], mw + rowB, key0);
            }
        }
#endif
        FA_STAMP(sb);
        if constexpr (first) {
            sm1_first(PAR, AD{});
            rescale(true);  // (O holds no P.V yet: l only)
        } else {
#if defined(FA_EXP_NOSM)
            phase2(lds + KV0 + (2 + pr) * T, IC<pr>{}, PAR, IC<0>{}, AD{});
#else
            phase2(lds + KV0 + (2 + pr) * T, IC<pr>{}, PAR, IC<1>{}, AD{});
#endif
            rescale(false);
        }
        FA_STAMP(sc_);
#if FA_EPI_OVL
        // K_{j+1}, V_j landed (the first tile's pieces precede the deferred O stores: those may stay in flight)
        if (first && had_epi) __builtin_amdgcn_s_waitcnt(vmcnt_enc(kOStores)); else dma_wait();
#else
        dma_wait();  // K_{j+1}, V_j landed
#endif
        FA_STAMP(sd);
        __syncthreads();
#ifdef FA_STAMPS
        const uint32_t se = (uint32_t)__builtin_amdgcn_s_memtime();
        if constexpr (first) st_acc[5] += se - sa;  // (the first tile: its own record field)
#ifdef FA_STAMPS_MASKED  // (diagnostic: the tile columns of the record count masked tiles only)
        if constexpr (mk != 0 && !first)
#else
        if constexpr (!first)
#endif
        {
            st_acc[0] += sb - sa;
            st_acc[1] += sc_ - sb;
            st_acc[2] += sd - sc_;
            st_acc[3] += se - sd;
            st_acc[4] += 1;
#ifdef FA_STAMPS_FINE
            st_fa[0] += st_f[0] - sb;
            st_fa[1] += st_f[1] - st_f[0];
            st_fa[2] += st_f[2] - st_f[1];
            st_fa[3] += st_f[3] - sa;
#endif
        }
#endif
    };
    // every tile runs pipelined: first the tiles without a masked score, then (a second loop, so
    // the hot loop carries no mask branch) the diagonal / tail tiles with a mask step between the
    // phases. The debug variant (dbg & 1) runs all tiles through the plain body below instead.
    // The first tile j_lo runs alone (iter FIRST, parity 1); tile j > j_lo runs with parity
    // (j - jb) & 1, jb = j_lo + 1 (ring slots and S / P registers). A local window adds a leading
    // run of masked tiles [jb, j_um), rounded up to an even count so the unmasked loop starts on
    // parity 0.
#ifdef FA_DEBUG_VARIANTS
    const int n_loop = (dbg & 1) ? j_lo : n_end;
#else
    (void)dbg;  // (the product library has no debug body: every tile runs pipelined)
    const int n_loop = n_end;
#endif
    const int n_unm = min(n_pipe, n_loop);
    // causal: the tiles from jA on hold no visible score of any wave's block A (its rows are the
    // workgroup's first half, m0 .. m0 + kRowB - 1): they run B only (MASKED 2, then 3)
    int jA = n_loop;
    if (kCausal) {
        // the last visible key of block A (rows m0 .. m0 + 127 in both layouts; head-packed m0 .. m0 + 31)
        const int x = min(Sk - 1, m0 + (hp ? 31 : kRowB - 1) + diag);
        jA = x < 0 ? 0 : x / kBlockN + 1;
    }
    const int jb = j_lo + 1;
    int j = jb;  // the next tile after the first
    // (the first tile computes block A even where no row of it sees a key -- key-split second pieces
    // of the first q-tiles, Sq > Sk: its scores are masked; the A-dead tiles after it run MASKED 2, 3)
    // (one body for the first tile, masked or not: its mask step masks only the wave-blocks whose rows
    // hide a score of it, so an unmasked first tile pays the scalar tests alone -- and one body keeps
    // the block's O zeroing on every path into the tile loops)
    if (j_lo < n_loop) iter(j_lo, IC<1>{}, IC<1>{}, IC<true>{});
#if FA_EPI_OVL
    else {  // a block without tiles: the deferred stores here, then O = 0 (stored as such)
        if (epi_pending) static_for<kOStores>([&](auto U) { epi_unit(U); });
        zero_o();
        epi_pending = false;
    }
#endif
    {
        if (j_um > j) {
            const int e = min(j_um + ((j_um - j) & 1), n_loop);
            for (int t = j; t < e; t += 2) {
                iter(t, IC<0>{}, IC<1>{}, IC<false>{});
                if (t + 1 < e) iter(t + 1, IC<1>{}, IC<1>{}, IC<false>{});
            }
            j = max(j, e);
        }
        for (int t = j; t < n_unm; t += 2) {
            iter(t, IC<0>{}, IC<0>{}, IC<false>{});
            if (t + 1 < n_unm) iter(t + 1, IC<1>{}, IC<0>{}, IC<false>{});
        }
        j = max(j, n_unm);
        const int j0 = j, jm = min(max(jA, j), n_loop);
        if (((j - jb) & 1) && j < jm) iter(j++, IC<1>{}, IC<1>{}, IC<false>{});
        for (; j < jm; j += 2) {
            iter(j, IC<0>{}, IC<1>{}, IC<false>{});
            if (j + 1 < jm) iter(j + 1, IC<1>{}, IC<1>{}, IC<false>{});
        }
        j = max(j0, jm);  // (the pair loop may step past jm)
        if constexpr (kCausal) {
            // (j > jA when the first tile or a window's leading run is past jA: they computed block A)
            if (j < n_loop) {
                if ((j - jb) & 1) iter(j, IC<1>{}, IC<2>{}, IC<false>{}); else iter(j, IC<0>{}, IC<2>{}, IC<false>{});
                ++j;
            }
            for (; j < n_loop; ++j) {
                if ((j - jb) & 1) iter(j, IC<1>{}, IC<3>{}, IC<false>{}); else iter(j, IC<0>{}, IC<3>{}, IC<false>{});
            }
        }
    }
    const bool last_dead = kCausal && n_loop > max(jA, j_lo);  // the last pipelined tile is A-dead
    FA_STAMP(s_loop_end);
#ifdef FA_DEBUG_VARIANTS
    // ---- debug variant: every tile masked, not pipelined -----------------------------------
    if (n_loop < n_end) {
        stage_v(n_loop, (n_loop - j_lo + 1) & 1);  // the pipeline fetched V one tile late; catch up first
        dma_wait();
        __syncthreads();
    }
    for (int j = n_loop; j < n_end; ++j) {
        const int sl = (j - j_lo + 1) & 1;  // (K_{j_lo} is in slot 1)
        if (j + 1 < n_end) {
            stage_k(j + 1, sl ^ 1);
            stage_v(j + 1, sl ^ 1);
        }
        const char *K = lds + KV0 + sl * T;
        const char *V = lds + KV0 + (2 + sl) * T;
        const int key0 = j * kBlockN;
        phase1(K, IC<0>{}, IC<0>{}, IC<0>{}, make_rsrc(nullptr, 0u), make_rsrc(nullptr, 0u), IC<0>{});  // (no DMA)
        s_ready(S[0][0], S[0][1]);
        s_ready(S[0][2], S[0][3]);
        mask(S[0][0], S[0][1], mw, key0);
        mask(S[0][2], S[0][3], mw + rowB, key0);
        sm1_all(IC<0>{});
        rescale(j == j_lo);
        sm2_all(IC<0>{}, IC<0>{});
        phase2(V, IC<0>{}, IC<0>{}, IC<0>{}, IC<0>{});
        dma_wait();
        __syncthreads();
    }

#endif  // FA_DEBUG_VARIANTS

    // ---- next block: its Q fragments and K_0 go in flight under this block's drain and stores.
    // Every wave is past this block's last barrier: the Q AGPRs and both K slots are free (the
    // drain reads only a V slot).
    char *const ob_c = ob;
    const int mw_c = mw, sq_c = Sq, jlo_c = j_lo, rowb_c = rowB, slot_c = split_slot;
    const bool spl_c = blk_split;
#ifdef FA_STAMPS
    const uint32_t blk_c = xcd + 8 * kblk;
#endif
    kblk = block_of(++rnd);
    const bool more = valid(kblk);
    if (more) {
        set_block(wk_next);
        // kQL: when this block's tiles issued all the next block's Q pieces they have landed (each
        // tile waits vmcnt(0)), so Q goes into the AGPRs now, under the drain; else the rest is
        // issued here and read in the prologue
        q_in_agpr = kQL && qnt > 0 && qn == qnt;
        if constexpr (kQL != 0) {
            for (; qn < qnt; ++qn) q_piece(qnr, qn, rowB_next);
        } else if (!rope_q) {
            load_q();
        }
        stage_k(j_lo, 1);
        if (q_in_agpr) q_from_lds();
    }
#ifdef FA_STAMPS
    st_acc[7] = (uint32_t)__builtin_amdgcn_s_memtime() - s_loop_end;  // (the next block's Q / K_0 issue)
#endif
    // drain the last pipelined tile: softmax half 2 and P.V
    auto drain = [&](auto PAR, auto AD) __attribute__((always_inline)) {
        constexpr int c = decltype(PAR)::value;
        // the late scores of the last tile in the first two k-steps' MFMA gaps (their P feeds k-steps 2, 3);
        // at D = 64 the causal kernels have no VGPRs for it (hipcc spilled into the O AGPRs)
        if constexpr (FA_DRAIN_OVL && DTL == 4) {
            phase2(lds + KV0 + (2 + c) * T, PAR, PAR, IC<2>{}, AD);
        } else {
            sm2_all(PAR, AD);
            phase2(lds + KV0 + (2 + c) * T, PAR, PAR, IC<0>{}, AD);
        }
    };
    if (n_loop > jlo_c) {  // (set_block above moved j_lo to the next block)
        if (kCausal && last_dead) {
            if constexpr (kCausal) {
                if ((n_loop - jlo_c) & 1) drain(IC<1>{}, IC<2>{}); else drain(IC<0>{}, IC<2>{});
            }
        } else {
            if ((n_loop - jlo_c) & 1) drain(IC<1>{}, IC<0>{}); else drain(IC<0>{}, IC<0>{});
        }
    }
    FA_STAMP(s_pipe_end);

    // ---- epilogue ---------------------------------------------------------------------------
    mfma_drain();  // last asm MFMA -> AGPR reads
    const int os_ = (int)p.o_seqlen_stride;
    const rsrc_t orr = make_rsrc(ob_c + 2 * (int64_t)mw_c * os_, slab_bytes(min(sq_c - mw_c, rowb_c + 32), os_, D));
    auto store_block = [&](const int row, auto OBASE, const float l_tot) {
        constexpr int ob0 = decltype(OBASE)::value;
        f32x16 o[DTL];
        o[0] = agpr_read16<ob0>();
        o[1] = agpr_read16<ob0 + 16>();
        if constexpr (DTL == 4) {
            o[2] = agpr_read16<ob0 + 32>();
            o[3] = agpr_read16<ob0 + 48>();
        }
        const float inv = (l_tot == 0.f) ? 1.f : 1.f / l_tot;
        const int orow = row * os_ * 2;
#pragma unroll
        for (int dt = 0; dt < DTL; ++dt) {
#pragma unroll
            for (int gp = 0; gp < 4; gp += 2) {
                const uint32_t a0 = DT::pack(o[dt][4 * gp + 0] * inv, o[dt][4 * gp + 1] * inv);
                const uint32_t a1 = DT::pack(o[dt][4 * gp + 2] * inv, o[dt][4 * gp + 3] * inv);
                const uint32_t b0 = DT::pack(o[dt][4 * gp + 4] * inv, o[dt][4 * gp + 5] * inv);
                const uint32_t b1 = DT::pack(o[dt][4 * gp + 6] * inv, o[dt][4 * gp + 7] * inv);
                const auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
                const auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
                const int d0 = dt * 32 + 8 * (gp + h);
                // unconditional (columns past D go out of range and are dropped): every wave issues
                // exactly kOStores stores per block, which the next block's counted wait relies on
                __builtin_amdgcn_raw_buffer_store_b128((u32x4){x0[0], x1[0], x0[1], x1[1]}, orr,
                                                       (kExactD || d0 < D) ? orow + 2 * d0 : 0x7ffffff0, 0, 0);
            }
        }
    };
    // key-split blocks: the same stores of o * fm + pw * fo (pw: the partner piece's partial O of
    // this wave's two blocks), one d-tile of both blocks per load round trip (each round trip to the
    // write-through records costs microseconds under load: measured +1.4 to +3.2 % over one d-tile of
    // one block per trip), registers for one d-tile only. Two rounded products and their rounded
    // sum -- no fma: the same bits whichever piece arrives second.
    auto store_both_combined = [&](const float *lt, const u32x4 *pw, const float *fm, const float *fo) {
        const float inv0 = (lt[0] == 0.f) ? 1.f : 1.f / lt[0], inv1 = (lt[1] == 0.f) ? 1.f : 1.f / lt[1];
        static_for<DTL>([&](auto DD) {
            constexpr int dt = decltype(DD)::value;
            u32x4 xs[2][4];
            ld_ws8(pw + dt * 4 * 64 + lane, pw + (DTL + dt) * 4 * 64 + lane, xs[0], xs[1]);
            static_for<2>([&](auto XX) {
                constexpr int X = decltype(XX)::value;
                f32x16 od = agpr_read16<16 * DTL * X + 16 * dt>();
                const float inv = X ? inv1 : inv0;
                const int orow = (X ? r + rowb_c : r) * os_ * 2;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        od[4 * q + e] = sum_of_products(od[4 * q + e], fm[X], __uint_as_float(xs[X][q][e]), fo[X]);
                }
#pragma unroll
                for (int gp = 0; gp < 4; gp += 2) {
                    const uint32_t a0 = DT::pack(od[4 * gp + 0] * inv, od[4 * gp + 1] * inv);
                    const uint32_t a1 = DT::pack(od[4 * gp + 2] * inv, od[4 * gp + 3] * inv);
                    const uint32_t b0 = DT::pack(od[4 * gp + 4] * inv, od[4 * gp + 5] * inv);
                    const uint32_t b1 = DT::pack(od[4 * gp + 6] * inv, od[4 * gp + 7] * inv);
                    const auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
                    const auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
                    const int d0 = dt * 32 + 8 * (gp + h);
                    __builtin_amdgcn_raw_buffer_store_b128((u32x4){x0[0], x1[0], x0[1], x1[1]}, orr,
                                                           (kExactD || d0 < D) ? orow + 2 * d0 : 0x7ffffff0, 0, 0);
                }
            });
        });
    };
    // (FA_SPLIT_AGPR) one block's combine from the partner records in a[PB ..): own O * fm + partner * fo,
    // O / l, packed; the 2 * DTL store values and offsets into vals / offs
    auto combine_block = [&](auto XX, auto PB, const float fmx, const float fox, const float inv, u32x4 *vals,
                             int *offs) __attribute__((always_inline)) {
        constexpr int X = decltype(XX)::value, pb = decltype(PB)::value;
        static_for<DTL>([&](auto DD) {
            constexpr int dt = decltype(DD)::value;
            f32x16 od = agpr_read16<16 * DTL * X + 16 * dt>();
            const f32x16 pw = agpr_read16<pb + 16 * dt>();
            const int orow = (X ? r + rowb_c : r) * os_ * 2;
#if FA_SPLIT_PK
            const f32x2 fm2 = {fmx * inv, fmx * inv}, fo2 = {fox * inv, fox * inv};
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                const f32x2 c = sum_of_products2((f32x2){od[i], od[i + 1]}, fm2, (f32x2){pw[i], pw[i + 1]}, fo2);
                od[i] = c[0];
                od[i + 1] = c[1];
            }
            constexpr float sc = 1.f;
#else
#pragma unroll
            for (int i = 0; i < 16; ++i) od[i] = sum_of_products(od[i], fmx, pw[i], fox);
            const float sc = inv;
#endif
#pragma unroll
            for (int gp = 0; gp < 4; gp += 2) {
                const uint32_t a0 = DT::pack(od[4 * gp + 0] * sc, od[4 * gp + 1] * sc);
                const uint32_t a1 = DT::pack(od[4 * gp + 2] * sc, od[4 * gp + 3] * sc);
                const uint32_t b0 = DT::pack(od[4 * gp + 4] * sc, od[4 * gp + 5] * sc);
                const uint32_t b1 = DT::pack(od[4 * gp + 6] * sc, od[4 * gp + 7] * sc);
                const auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
                const auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
                const int d0 = dt * 32 + 8 * (gp + h);
                vals[2 * dt + gp / 2] = (u32x4){x0[0], x1[0], x0[1], x1[1]};
                offs[2 * dt + gp / 2] = (kExactD || d0 < D) ? orow + 2 * d0 : 0x7ffffff0;
            }
        });
    };
    FA_STAMP(s_masked_end);
    [[maybe_unused]] int split_role = 0;  // (stamps) key-split piece: 1 the first to arrive, 3 the second
    if (!spl_c) {
        // row sums: each lane half summed half of the tile's keys
        const float l0 = pair_sum(st[0].l);
        const float l1 = pair_sum(st[1].l);
#if FA_EPI_OVL
        if (more) {  // the stores go into the next block's first tile (epi_unit)
            epi_pending = true;
            epi_inv0 = (l0 == 0.f) ? 1.f : 1.f / l0;
            epi_inv1 = (l1 == 0.f) ? 1.f : 1.f / l1;
            epi_orr = orr;
            epi_rowb = rowb_c * os_ * 2;
        } else
#endif
        {
            store_block(r, IC<0>{}, l0);
            store_block(r + rowb_c, IC<16 * DTL>{}, l1);
        }
    } else {
        // ---- key-split block: the two pieces meet per wave. The first to arrive leaves its
        // unnormalised O (AGPR fragment order, 64 lanes x 16 B per record) and its (nmsc, l, m) per
        // lane in the workspace and marks them ready in the arrivals word; the second finds them
        // ready in its own arrival, or waits for the mark (the first has finished its tiles and only
        // stores), rescales both to their larger reference and stores O. The hand-off RELIES on both
        // pieces running on one XCD (work_of's order + the host's placement check, fa_launch.h
        // same_xcd_placement): its sc1 accesses meet in that XCD's L2 (see st_ws).
        constexpr int kWaveF = 64 * (32 * DTL + kSplitStatsPerLane);
        unsigned *sync = xa.split_sync + 2 * ((size_t)slot_c * 4 + wave);
        u32x4 *wsw = (u32x4 *)(xa.split_ws + ((size_t)slot_c * 4 + wave) * kWaveF);
        u32x4 *stats = wsw + 8 * DTL * 64;  // after the 2 x DTL x 4 O records
        // sync[0]: arrivals + kReady once the first piece's records are written (sync[1] is unused).
        // Within a launch the word runs 0 -> 1 -> 2 (arrivals) with + kReady at any point after 1, and
        // the combining piece zeroes it, so every launch finds it 0. A second piece whose poll times out
        // ABANDONS the pair: it swaps 2 (both arrived, not ready) for 0, so the first piece's late
        // + kReady reads 0 and takes its own add back -- no launch inherits a stale ready mark.
        constexpr uint32_t kReady = 4;
#ifdef FA_DEBUG_VARIANTS
        // (debug library, dbg & 2: force one hand-off to time out -- wave 0 of the last q-tile of
        // (batch 0, q-head 0), split in both layouts: the first piece holds its ready mark until its
        // partner has abandoned the pair, the partner polls briefly)
        const bool fault = (dbg & 2) && slot_c == nqp - 1 && wave == 0;
#else
        constexpr bool fault = false;
#endif
        uint32_t arrived = 0;
        if (lane == 0) arrived = __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        arrived = __builtin_amdgcn_readfirstlane(arrived);
        if (arrived == 0) {
            static_for<2 * DTL>([&](auto I) {
                constexpr int i = decltype(I)::value;
                const f32x16 o = agpr_read16<16 * i>();
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    st_ws(wsw + (i * 4 + q) * 64 + lane,
                          (u32x4){__float_as_uint(o[4 * q]), __float_as_uint(o[4 * q + 1]), __float_as_uint(o[4 * q + 2]),
                                  __float_as_uint(o[4 * q + 3])});
            });
            st_ws(stats + lane, (u32x4){__float_as_uint(st[0].nmsc), __float_as_uint(st[1].nmsc),
                                        __float_as_uint(st[0].l), __float_as_uint(st[1].l)});
            st_ws(stats + 64 + lane, (u32x4){__float_as_uint(st[0].m), __float_as_uint(st[1].m), 0u, 0u});
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (every lane's records written through before the flag)
            if (lane == 0) {
                if (fault)  // (debug: until the partner has arrived and abandoned the pair, bounded)
                    for (int it = 0; it < (1 << 22); ++it) {
                        __builtin_amdgcn_s_sleep(8);
                        if (it > 64 && __hip_atomic_load(sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) break;
                    }
                // ready: + kReady on the arrivals word (an add: the partner's arrival may land in between).
                // It reads 0 only if the partner abandoned the pair: then no one else touches the word in
                // this launch, and the add is taken back for the next one
                if (__hip_atomic_fetch_add(sync, kReady, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
                    __hip_atomic_store(sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            split_role = 1;
        } else {
            split_role = 3;
            // the arrival already saw the records ready (the pairs layout's usual case: the partner
            // finished long before), or a bounded poll (~1 s), so a protocol failure never hangs the
            // GPU; a timeout abandons the pair (2 -> 0, above) and is counted in the stream's error
            // counter (fa_split_errors) -- the rows it combines are wrong
            if (lane == 0) {
                bool seen = arrived >= kReady;
                const int polls = fault ? 64 : (1 << 22);
                for (int it = 0; !seen && it < polls; ++it) {
                    __builtin_amdgcn_s_sleep(8);
                    seen = __hip_atomic_load(sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= kReady;
                }
                if (!seen) {
                    unsigned expect = 2u;  // (the ready mark may land now: then the records are there)
                    seen = !__hip_atomic_compare_exchange_strong(sync, &expect, 0u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT);
                    if (!seen && xa.split_err)
                        __hip_atomic_fetch_add(xa.split_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                // both pieces are past their last access to the pair: zero it for the next launch
                if (seen) __hip_atomic_store(sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: loads stay below the poll)
#if FA_SPLIT_AGPR && FA_QLDS != 2  // (staging 2 may have read the next block's Q into those AGPRs already)
            // the partner's first 16 records (block A's at D = 128, both blocks' at D = 64) into the Q AGPRs
            // (free here: the next block's Q is read in its prologue), beside the statistics: one round trip
            const char *wb = (const char *)(wsw + lane);
            fa_agpr_ldws4_128(wb);
            fa_agpr_ldws4_144(wb + 4096);
            fa_agpr_ldws4_160(wb + 8192);
            fa_agpr_ldws4_176(wb + 12288);
#endif
            u32x4 s0, s1;
            ld_ws2(stats + lane, s0, s1);
            float fm[2], fo[2], lt[2];
#pragma unroll
            for (int X = 0; X < 2; ++X) {
                // references: -nmsc (scaled); a row that saw no key in a piece has m = kNeg, O = l = 0
                const bool sm = st[X].m > 0.5f * kNeg, so = __uint_as_float(s1[X]) > 0.5f * kNeg;
                const float mm = -st[X].nmsc, mo = -__uint_as_float(s0[X]);
                const float mt = sm && so ? fmaxf(mm, mo) : (sm ? mm : mo);
                fm[X] = sm ? __builtin_amdgcn_exp2f(mm - mt) : 0.f;
                fo[X] = so ? __builtin_amdgcn_exp2f(mo - mt) : 0.f;
                lt[X] = pair_sum(sum_of_products(st[X].l, fm[X], __uint_as_float(s0[2 + X]), fo[X]));
            }
#if FA_SPLIT_AGPR && FA_QLDS != 2
            const float inv0 = (lt[0] == 0.f) ? 1.f : 1.f / lt[0], inv1 = (lt[1] == 0.f) ? 1.f : 1.f / lt[1];
            u32x4 va_[2 * DTL], vb_[2 * DTL];
            int oa_[2 * DTL], ob_[2 * DTL];
            if constexpr (DTL == 4) {
                combine_block(IC<0>{}, IC<128>{}, fm[0], fo[0], inv0, va_, oa_);
                // block B's records into the same AGPRs, then block A's stores: the counted wait below
                // retires the loads and leaves the stores in flight
                fa_agpr_ldws4_128(wb + 16384);
                fa_agpr_ldws4_144(wb + 20480);
                fa_agpr_ldws4_160(wb + 24576);
                fa_agpr_ldws4_176(wb + 28672);
#pragma unroll
                for (int i = 0; i < 2 * DTL; ++i) __builtin_amdgcn_raw_buffer_store_b128(va_[i], orr, oa_[i], 0, 0);
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                combine_block(IC<1>{}, IC<128>{}, fm[1], fo[1], inv1, vb_, ob_);
            } else {
                combine_block(IC<0>{}, IC<128>{}, fm[0], fo[0], inv0, va_, oa_);
                combine_block(IC<1>{}, IC<160>{}, fm[1], fo[1], inv1, vb_, ob_);
#pragma unroll
                for (int i = 0; i < 2 * DTL; ++i) __builtin_amdgcn_raw_buffer_store_b128(va_[i], orr, oa_[i], 0, 0);
            }
#pragma unroll
            for (int i = 0; i < 2 * DTL; ++i) __builtin_amdgcn_raw_buffer_store_b128(vb_[i], orr, ob_[i], 0, 0);
#else
            store_both_combined(lt, wsw, fm, fo);
#endif
        }
    }
#ifdef FA_STAMPS
    {
        __builtin_amdgcn_s_waitcnt(0);
        const uint32_t s_end = (uint32_t)__builtin_amdgcn_s_memtime();
        const unsigned long long rt_end = __builtin_amdgcn_s_memrealtime();
        if (stamps && lane == 0) {
            // per Q block: [total, p1, p2+rescale, dma wait, barrier, tiles, drain (+ next block's
            //  prefetch issue), prologue, epilogue, realtime (100 MHz ticks), start time, xcc, (FINE:
            //  4 sub-phase fields), prologue wait, next-block issue, first tile]
            unsigned long long *o = stamps + ((size_t)blk_c * 4 + wave) * FA_STAMP_W;
            o[0] = s_end - st_t0;
            for (int i = 0; i < 5; ++i) o[1 + i] = st_acc[i];
            o[6] = s_pipe_end - s_loop_end;
            o[7] = s_pro - st_t0;
            o[8] = s_end - s_masked_end;
            o[9] = rt_end - st_rt0;
            o[10] = st_rt0;  // (realtime: one clock for every XCD)
            o[11] = xcc_id() | (split_role << 8);  // (key-split role: split_role)
#ifdef FA_STAMPS_FINE  // [12..14] phase 2 quarters 1-3 (the 4th: p2+rescale - their sum), [15] phase 1 half 1
#pragma unroll
            for (int i = 0; i < 4; ++i) o[12 + i] = st_fa[i];
#endif
            o[FA_STAMP_W - 3] = st_acc[6];  // the prologue's wait for Q and K_0
            o[FA_STAMP_W - 2] = st_acc[7];  // the next block's Q / K_0 issue at the block's end
            o[FA_STAMP_W - 1] = st_acc[5];  // the block's first tile (iter FIRST)
        }
    }
#endif
    if (!more) break;
    }  // persistent block loop
}
#undef FA_STAMP

#ifdef FA_DEBUG_VARIANTS
// the paired 8-wave kernel (fa_fwd_p8.hpp)
template <class DT, bool C, int kD, bool kExact>
int launch_p8(const fa_fwd_params &p, hipStream_t stream);
// the MFMA-shape A/B body (fa_fwd_mb.hpp): m16 = 16x16x32, else 32x32x16
template <class DT, bool C, int kD, bool kExact>
int launch_mb(const fa_fwd_params &p, hipStream_t stream, bool m16);
#endif

// ---- host launch of one instantiation -------------------------------------------------
template <class DT, bool C, int kD, bool kExact>
int launch_one(const fa_fwd_params &p, const PathArgs &xa, hipStream_t stream) {
    if (xa.cos && !kExact) return set_err(FA_ERR_UNSUPPORTED, "fused RoPE needs head dim 64 or 128");
    // varlen, fused RoPE and the local window run fa_fwd_w4 (w4slow under the debug variant); w8 / p8
    // have none of them
#ifdef FA_DEBUG_VARIANTS
    const bool w4_only = xa.k_rng || xa.cos || xa.window_left >= 0;
    const int variant = w4_only && variant_from_env() != 2 ? 0 : variant_from_env();
    if (variant == 3) return launch_p8<DT, C, kD, kExact>(p, stream);
    if (variant == 4 || variant == 5) return launch_mb<DT, C, kD, kExact>(p, stream, variant == 5);  // (unsplit)
#else
    constexpr int variant = 0;  // the product library: fa_fwd_w4 only
#endif
    // fa_fwd_w4 / w4slow: key-split causal blocks when the dispatcher passed their workspace
    // (xa.split_ws), else zigzag Q blocks for a causal launch that fits one round
    PathArgs xz = xa;
    if (variant == 1) xz.split_ws = nullptr;
    // (the default rules are disjoint: head-packed blocks on multi-round grids, zigzag on one-round ones;
    // the head_pack knob 2 forces them over zigzag; key-split pieces are head-packed wherever the layout
    // applies, use_head_pack_split)
    // q-tiles per (batch, q-head) or, head-packed, per (batch, q-head quad): 256 or 64 rows
    auto qtiles_of = [&](const bool hp) { return hp ? (p.seqlen_q + 63) / 64 : (p.seqlen_q + kBlockM - 1) / kBlockM; };
    auto rows_of = [&](const bool hp) { return (hp ? p.num_heads_q / 4 : p.num_heads_q) * p.batch_size; };
    auto pairs_of = [&](const bool hp) { return use_split_pairs(qtiles_of(hp) * rows_of(hp), rows_of(hp), device_cus()); };
    if (xz.split_ws) {  // head-packed pieces: under the pairs layout (knob 2: under the halves too)
        const bool hp = variant != 1 && use_head_pack_split(p, C, xa) && (knobs().head_pack == 2 || pairs_of(true));
        xz.head_pack = hp ? 1 : 0;
        xz.split_pairs = pairs_of(hp) ? 1 : 0;
    } else {
        xz.head_pack = variant != 1 && use_head_pack(p, C, xa) ? 1 : 0;
        xz.split_pairs = 0;
    }
    xz.zigzag = !xz.split_ws && !xz.head_pack && variant != 1 && use_zigzag(p, C, xa) ? 1 : 0;
    xz.split_rr = knobs().split_rr;
    const int64_t n_plain = qtiles_of(xz.head_pack != 0);
    const int64_t heads_u = xz.head_pack ? p.num_heads_q / 4 : p.num_heads_q;
    const int64_t n_pairs = (n_plain + 1) / 2 * heads_u * p.batch_size;
    const int64_t n_qtiles = xz.split_ws ? 2 * n_plain : xz.zigzag ? zigzag_qtiles(p.seqlen_q) : n_plain;
    const int64_t nwg = n_qtiles * heads_u * p.batch_size;
#ifdef FA_DEBUG_VARIANTS
    if (variant == 1)
        hipLaunchKernelGGL((fa_fwd_w8<DT, C, kD, kExact>), dim3((uint32_t)nwg), dim3(kThreads), 0, stream, p,
                           (int)n_qtiles);
    else
#endif
        // persistent: about one workgroup per CU (the kernel walks the Q blocks itself)
        hipLaunchKernelGGL((fa_fwd_w4<DT, C, kD, kExact>),
                           dim3((uint32_t)(xz.split_ws ? w4_grid_split(xz.split_pairs ? n_pairs : nwg / 2) : w4_grid(nwg))),
                           dim3(256), 0, stream, p,
                           (int)n_qtiles, (variant == 2 ? 1 : 0) | (knobs().split_fault ? 2 : 0), stamp_buffer(), xz);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(FA_ERR_LAUNCH, "HIP launch failed: %s", hipGetErrorString(e));
    set_last_path(variant == 1 ? kPathW8 : variant == 2 ? kPathW4Slow : kPathW4);
    set_last_zigzag(xz.split_ws ? (xz.head_pack ? 5 : 2) + xz.split_pairs : xz.head_pack ? 4 : xz.zigzag);
    return FA_OK;
}

}  // namespace fa
