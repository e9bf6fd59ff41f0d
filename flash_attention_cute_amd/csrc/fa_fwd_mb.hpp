#pragma once
// fa_fwd_mb.hpp -- the MFMA-shape A/B body: ONE kernel, templated on the shape of both contractions
// (debug / A-B library only; FA_GFX950_VARIANT=m16 | m32, _debug.forward(variant="m16")):
//
//   kM16 = true : v_mfma_f32_16x16x32_{f16,bf16}, the shape family north_star names (the reference's
//                 atom is SM80_16x8x16, csrc/flash_attention_template.cuh:253-257)
//   kM16 = false: v_mfma_f32_32x32x16_{f16,bf16}, the shape of the product kernel fa_fwd_w4
//
// Everything but the shape is shared by the two instantiations: the output tile per wave (64 query
// rows, blocks A / B of 32 interleaved as in fa_fwd_w4, every 64-key K/V tile), the LDS images
// (Geo<kD> swizzles, LDS-DMA pieces into 2-slot K / V rings, one barrier per tile), the persistent
// XCD-aware grid, the online softmax (max on unscaled S, deferred rescale kRescaleThr, exp2 with the
// host's scale * log2 e, P rounded to T, fp32 row sums, O / l with l == 0 -> 1) and a two-phase
// software pipeline per tile
//     phase 1: S(j) = K_j . Q^T                    (MFMA)
//     phase 2: O += V_{j-1}^T . P(j-1)^T (MFMA)  ||  softmax of tile j (VALU)
// that hipcc schedules itself (builtin MFMAs, its own register allocation). So the A/B of the two
// instantiations prices the shape alone, on random data, by wall time and in-kernel clock (guide
// cdna_hip_programming.md rule 28; MI355X_MICROARCH.md "DVFS give-back" item 7). Dense prefill only
// (no varlen, window, RoPE or key-split: those stay on fa_fwd_w4).
//
// Layouts, per lane (l = lane, r = l & 31, h = l >> 5, c = l & 15, g = l >> 4). S^T = K . Q^T puts the
// query on the lane in both shapes; the 32 scores a lane holds of a block X per tile are s[X][n]:
//   32x32x16: n = 16 hf + i (i: register of the key half hf's accumulator) -> query r,
//             key 32 hf + (i & 3) + 8 (i >> 2) + 4 h
//   16x16x32: n = 16 hf + 8 qs + 4 ks + e (query sub-tile qs, 16-key sub-tile ks, register e) ->
//             query 16 qs + c, key 32 hf + 16 ks + 4 g + e: TWO queries per lane and block, each
//             spread over the four lanes c, c + 16, c + 32, c + 48 (two cross-lane steps per row max)
// and in both the P.V B operand u (0..3) of block X is the eight rounded scores n = 8u .. 8u + 7 in
// place: the 32x32x16 k-step u (16 keys), or the 16x16x32 (qs = u & 1, key half u >> 1) operand whose
// k index 8g + j is key 32 hf + 4g + j (j < 4) / 32 hf + 16 + 4g + j - 4 (j >= 4) -- the V^T operand
// reads those rows with two ds_read_b64_tr_b16 per fragment, so no score moves between lanes.
#include "fa_fwd_kernels.hpp"

namespace fa {
namespace mb {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool kF16>
__device__ __forceinline__ f32x16 mfma32(const u32x4 &a, const u32x4 &b, const f32x16 &c) {
    if constexpr (kF16)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                       0, 0);
}
template <bool kF16>
__device__ __forceinline__ f32x4 mfma16(const u32x4 &a, const u32x4 &b, const f32x4 &c) {
    if constexpr (kF16)
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                       0, 0);
}
// S^T MFMAs as inline asm: the scores land in arch VGPRs (the softmax reads them there) and the Q
// operand stays in AGPRs (the "a" constraint), so hipcc keeps both the 256 arch VGPRs for the softmax and
// the AGPRs for O and Q; first: C = 0. Their results are read only after s_ready (below).
template <bool kF16>
__device__ __forceinline__ void mfma32_s(f32x16 &acc, const u32x4 &a, const u32x4 &b, const bool first) {
    if (first) {
        if constexpr (kF16) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
        else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
    } else {
        if constexpr (kF16) asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
        else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
    }
}
template <bool kF16>
__device__ __forceinline__ void mfma16_s(f32x4 &acc, const u32x4 &a, const u32x4 &b, const bool first) {
    if (first) {
        if constexpr (kF16) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
        else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "a"(b));
    } else {
        if constexpr (kF16) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
        else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "a"(b));
    }
}
// x = kNeg unless the constant key offset C <= E (one compare through VCC, one select)
template <int C>
__device__ __forceinline__ void mask_one(float &x, const int E, const float neg) {
    asm volatile("v_cmp_le_i32_e32 vcc, %2, %1\n\tv_cndmask_b32_e32 %0, %3, %0, vcc" : "+v"(x) : "v"(E), "n"(C), "v"(neg)
                 : "vcc");
}
// max / sum over the lanes l and l ^ 16 (v_permlane16_swap: rows of 16 lanes, odd rows of the first
// operand against even rows of the second -- with both operands x, the pair holds x_l and x_(l^16))
__device__ __forceinline__ float x16_max(float x) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float x16_sum(float x) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// key of score n of a block (relative to the tile's first key) and its query row (relative to the
// block's first row), for lane l
template <bool kM16>
__device__ __forceinline__ int key_of(const int n, const int lane) {
    if constexpr (kM16) return 32 * (n >> 4) + 16 * ((n >> 2) & 1) + 4 * (lane >> 4) + (n & 3);
    else return 32 * (n >> 4) + (n & 3) + 8 * ((n >> 2) & 3) + 4 * (lane >> 5);
}
template <bool kM16>
__device__ __forceinline__ int qrow_of(const int n, const int lane) {
    if constexpr (kM16) return 16 * ((n >> 3) & 1) + (lane & 15);
    else return lane & 31;
}

}  // namespace mb

template <class DT, bool kCausal, int kD, bool kExactD, bool kM16>
__global__ __launch_bounds__(256, 1) void fa_fwd_mb(const fa_fwd_params p, const int n_qtiles) {
    using G = Geo<kD>;
    using mb::f32x4;
    constexpr bool F = DT::kIsF16;
    constexpr int RB = G::kRowBytes, T = G::kTileBytes;
    constexpr int NP = T / 4 / 1024;  // LDS-DMA pieces per wave per K or V tile
    constexpr int ROWS_PER_PIECE = 1024 / RB;
    constexpr int DTL = kD / 32;                    // 32-row d tiles of O^T (32x32x16)
    constexpr int KQ = kM16 ? kD / 32 : kD / 16;    // k-steps of S^T = K.Q^T
    constexpr int NQF = kM16 ? 2 * KQ : KQ;          // Q fragments per block
    constexpr int NQ = kM16 ? 2 : 1;                 // queries per lane and block
    constexpr int kRowB = kBlockM / 2;
    __shared__ __attribute__((aligned(1024))) char lds[4 * T];  // K slots 0, 1 | V slots 0, 1

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, h = lane >> 5, c16 = lane & 15, g4 = lane >> 4;
    const int D = (int)p.headdim, Sq = (int)p.seqlen_q, Sk = (int)p.seqlen_kv;
    const float sc = p.softmax_scale, thr_raw = kRescaleThr / sc;
    const int diag = Sk - Sq, n_blocks = (Sk + kBlockN - 1) / kBlockN;

    // ---- persistent schedule (fa_fwd_w4's plain layout): XCD-aware order, snake rounds ----------
    const uint32_t nwg = (uint32_t)n_qtiles * (uint32_t)p.num_heads_q * (uint32_t)p.batch_size;
    const uint32_t xcd = blockIdx.x & 7, cx = blockIdx.x >> 3;
    const uint32_t gx = (gridDim.x - xcd + 7) >> 3;
    const uint32_t cnt = (nwg - xcd + 7) >> 3;
    auto block_of = [&](const uint32_t rnd) { return rnd * gx + ((rnd & 1) ? gx - 1 - cx : cx); };

    // ---- per-lane LDS addresses (both shapes; the slot / half / sub-tile offsets are immediates) --
    int k_addr[KQ], v_addr[kM16 ? 2 * DTL : DTL];
    const int qq = (lane >> 2) & 3, pp = lane & 3;
    if constexpr (kM16) {
#pragma unroll
        for (int k = 0; k < KQ; ++k) k_addr[k] = G::k_off(c16, 4 * k + g4);
#pragma unroll
        for (int dt = 0; dt < 2 * DTL; ++dt) v_addr[dt] = G::v_off(4 * g4 + qq, 2 * dt + (pp >> 1)) + 8 * (pp & 1);
    } else {
#pragma unroll
        for (int ks = 0; ks < KQ; ++ks) k_addr[ks] = G::k_off(r, 2 * ks + h);
#pragma unroll
        for (int dt = 0; dt < DTL; ++dt)
            v_addr[dt] = G::v_off(4 * (g4 >> 1) + qq, dt * 4 + 2 * (g4 & 1) + (pp >> 1)) + 8 * (pp & 1);
    }
    // LDS-DMA: this wave writes pieces wave * NP + n of each K / V tile (K's / V's swizzle applied on
    // the per-lane source offsets; columns past D read as 0)
    const int ks_ = (int)p.k_seqlen_stride, vs_ = (int)p.v_seqlen_stride, qs_ = (int)p.q_seqlen_stride;
    int kvo[NP], vvo[NP];
#pragma unroll
    for (int n = 0; n < NP; ++n) {
        const int row = (wave * NP + n) * ROWS_PER_PIECE + (16 * lane) / RB;
        const int slot = ((16 * lane) % RB) / 16;
        const int kch = G::k_off(row, slot) % RB / 16, vch = G::v_off(row, slot) % RB / 16;
        kvo[n] = ((kExactD || kch * 8 < D) ? row * ks_ * 2 + 16 * kch : 0x7ffffff0) - n * 1024;
        vvo[n] = ((kExactD || vch * 8 < D) ? row * vs_ * 2 + 16 * vch : 0x7ffffff0) - n * 1024;
    }
    const uint32_t lds_w = lds_u32(lds) + wave * NP * 1024;
    auto stage = [&](const char *base, const int stride, const int j, const uint32_t slot_off, const int *voff) {
        const int key0 = j * kBlockN;
        dma_tile<NP>(make_rsrc_u(base + 2 * (int64_t)key0 * stride, slab_bytes(min(Sk - key0, kBlockN), stride, D)),
                     lds_w + slot_off, voff);
    };

    // ---- state --------------------------------------------------------------------------------
    u32x4 q[2][NQF];                                   // Q^T B-operand fragments of blocks A, B
    float s[2][32];                                    // S / P of the current tile (layout above)
    u32x4 P[2][4];                                     // rounded P of the previous tile (P.V B operands)
    f32x16 o32[2][kM16 ? 1 : DTL];                     // O^T (32x32x16)
    f32x4 o16[2][kM16 ? 2 : 1][kM16 ? 2 * DTL : 1];     // O^T (16x16x32): [block][query sub-tile][16-d tile]
    float m_[2][NQ], msc[2][NQ], l_[2][NQ], alpha[2][NQ];
    // O^T lives in AGPRs (the P.V MFMAs accumulate there): tied to "a" after every VALU touch (zeroing,
    // rescale), or hipcc keeps a VGPR home for it and copies it to and from the AGPRs around each MFMA
    auto pin_o = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int X = 0; X < 2; ++X) {
            if constexpr (kM16) {
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int dt = 0; dt < 2 * DTL; ++dt) asm volatile("" : "+a"(o16[X][t][dt]));
            } else {
#pragma unroll
                for (int dt = 0; dt < DTL; ++dt) asm volatile("" : "+a"(o32[X][dt]));
            }
        }
    };

    for (uint32_t rnd = 0;; ++rnd) {
        const uint32_t kblk = block_of(rnd);
        if (kblk >= cnt) break;
        const Work wk = decode_work<kCausal>(nwg, xcd + 8 * kblk, n_qtiles, (int)p.num_heads_q, (int)p.head_q_per_group);
        const int qtile = __builtin_amdgcn_readfirstlane(wk.qtile), hq = __builtin_amdgcn_readfirstlane(wk.hq);
        const int b = __builtin_amdgcn_readfirstlane(wk.b);
        const int hkv = hq / (int)p.head_q_per_group;
        const char *qb = (const char *)p.q_ptr + 2 * ((int64_t)b * p.q_batch_stride + (int64_t)hq * p.q_head_stride);
        const char *kb = (const char *)p.k_ptr + 2 * ((int64_t)b * p.k_batch_stride + (int64_t)hkv * p.k_head_stride);
        const char *vb = (const char *)p.v_ptr + 2 * ((int64_t)b * p.v_batch_stride + (int64_t)hkv * p.v_head_stride);
        char *ob = (char *)p.o_ptr + 2 * ((int64_t)b * p.o_batch_stride + (int64_t)hq * p.o_head_stride);
        const int m0 = qtile * kBlockM, mw = m0 + wave * 32;  // block A rows mw.., block B rows mw + kRowB..
        int n_end = n_blocks;
        if (kCausal) {
            const int x = diag + min(m0 + kBlockM, Sq);
            n_end = min(x <= 0 ? 0 : (x + kBlockN - 1) / kBlockN, n_blocks);
        }
        // K_0 and this wave's Q fragments (rows past Sq and columns past D read as 0)
        if (n_end > 0) stage(kb, ks_, 0, 0, kvo);
        {
            const rsrc_t qr = make_rsrc_u(qb + 2 * (int64_t)mw * qs_, slab_bytes(min(Sq - mw, kRowB + 32), qs_, D));
#pragma unroll
            for (int X = 0; X < 2; ++X)
#pragma unroll
                for (int f = 0; f < NQF; ++f) {
                    int row, col;  // (query row in the wave's slab, byte column)
                    if constexpr (kM16) {
                        row = kRowB * X + 16 * (f / KQ) + c16;
                        col = 64 * (f % KQ) + 16 * g4;
                    } else {
                        row = kRowB * X + r;
                        col = 32 * f + 16 * h;
                    }
                    q[X][f] = __builtin_amdgcn_raw_buffer_load_b128(
                        qr, (kExactD || col < 2 * D) ? row * qs_ * 2 + col : 0x7ffffff0, 0, 0);
#ifndef FA_MB_Q_VGPR
                    // (Q only feeds MFMAs: parked in AGPRs, which the MFMA reads directly, so the
                    // softmax keeps the 256 arch VGPRs)
                    asm volatile("" : "+a"(q[X][f]));
#endif
                }
        }
#pragma unroll
        for (int X = 0; X < 2; ++X) {
#pragma unroll
            for (int t = 0; t < NQ; ++t) {
                m_[X][t] = kNeg;
                msc[X][t] = 0.f;
                l_[X][t] = 0.f;
                alpha[X][t] = 1.f;
            }
            if constexpr (kM16) {
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int dt = 0; dt < 2 * DTL; ++dt) o16[X][t][dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
            } else {
#pragma unroll
                for (int dt = 0; dt < DTL; ++dt)
#pragma unroll
                    for (int i = 0; i < 16; ++i) o32[X][dt][i] = 0.f;
            }
        }
        pin_o();
        dma_wait();
        __syncthreads();

        // phase 1: S(j) from K slot j & 1 in 16 steps (each: the next step's K fragment, then its 2 /
        // 4 MFMAs; a scheduling fence between steps keeps hipcc from hoisting every K read up front)
        auto phase1 = [&](const int j) __attribute__((always_inline)) {
            const char *K = lds + (j & 1) * T;
            // step st: 32x32x16 ks = st >> 1, hf = st & 1; 16x16x32 k = st >> 2, hf = (st >> 1) & 1, ks = st & 1
            auto kread = [&](const int st) __attribute__((always_inline)) {
                if constexpr (kM16) return *(const u32x4 *)(K + (32 * ((st >> 1) & 1) + 16 * (st & 1)) * RB + k_addr[st >> 2]);
                else return *(const u32x4 *)(K + 32 * (st & 1) * RB + k_addr[st >> 1]);
            };
            constexpr int NS = kM16 ? 4 * KQ : 2 * KQ;
            f32x4 acc16[2][2][2][2];  // [X][hf][qs][ks]
            f32x16 acc32[2][2];       // [X][hf]
            u32x4 kf[2];
            kf[0] = kread(0);
            static_for<NS>([&](auto S_) {
                constexpr int st = decltype(S_)::value;
                if constexpr (st + 1 < NS) kf[(st + 1) & 1] = kread(st + 1);
                if constexpr (kM16) {
                    constexpr int k = st >> 2, hf = (st >> 1) & 1, ks = st & 1;
#pragma unroll
                    for (int X = 0; X < 2; ++X)
#pragma unroll
                        for (int qs = 0; qs < 2; ++qs) mb::mfma16_s<F>(acc16[X][hf][qs][ks], kf[st & 1], q[X][qs * KQ + k], k == 0);
                } else {
                    constexpr int ks = st >> 1, hf = st & 1;
#pragma unroll
                    for (int X = 0; X < 2; ++X) mb::mfma32_s<F>(acc32[X][hf], kf[st & 1], q[X][ks], ks == 0);
                }
                FA_SCHED_FENCE();
            });
            // the asm MFMAs' results are invisible to hipcc's hazard recognizer: the wait states it puts
            // after a builtin MFMA before the first VALU read (fa_fwd_kernels.hpp s_ready), tied to S
            if constexpr (kM16) {
                asm volatile(FA_DRAIN_NOPS : "+v"(acc16[0][0][0][0]), "+v"(acc16[0][0][0][1]), "+v"(acc16[0][0][1][0]),
                             "+v"(acc16[0][0][1][1]), "+v"(acc16[0][1][0][0]), "+v"(acc16[0][1][0][1]),
                             "+v"(acc16[0][1][1][0]), "+v"(acc16[0][1][1][1]), "+v"(acc16[1][0][0][0]),
                             "+v"(acc16[1][0][0][1]), "+v"(acc16[1][0][1][0]), "+v"(acc16[1][0][1][1]),
                             "+v"(acc16[1][1][0][0]), "+v"(acc16[1][1][0][1]), "+v"(acc16[1][1][1][0]),
                             "+v"(acc16[1][1][1][1]));
            } else {
                s_ready4(acc32[0][0], acc32[0][1], acc32[1][0], acc32[1][1]);
            }
#pragma unroll
            for (int X = 0; X < 2; ++X)
#pragma unroll
                for (int n = 0; n < 32; ++n) {
                    if constexpr (kM16) s[X][n] = acc16[X][n >> 4][(n >> 3) & 1][(n >> 2) & 1][n & 3];
                    else s[X][n] = acc32[X][n >> 4][n & 15];
                }
        };
        // causal diagonal / Sk tail: scores of hidden keys -> kNeg (only where some score of the wave's
        // rows is hidden; block B's rows come after block A's, so A's test covers both)
        auto mask = [&](const int j) __attribute__((always_inline)) {
            const int key0 = j * kBlockN;
            const bool any = key0 + kBlockN > Sk || (kCausal && key0 + kBlockN - 1 > mw + diag);
            if (!any) return;
#ifdef FA_MB_ABL_NOMASK
            if (any) return;
#endif
            // score n is visible iff its key offset const_n (relative to key0 + lane part) <= E_t: the
            // row's last visible key - key0 - lane part; one compare with an inline constant and one
            // select per score, in asm (compiled C++ materialises every compare in SGPR pairs)
            float neg = kNeg;
            asm volatile("" : "+v"(neg));
            const int lp = kM16 ? 4 * g4 : 4 * h;
#pragma unroll
            for (int X = 0; X < 2; ++X)
#pragma unroll
                for (int t = 0; t < NQ; ++t) {
                    const int row = mw + kRowB * X + (kM16 ? 16 * t + c16 : r);
                    const int E = (kCausal ? min(Sk - 1, row + diag) : Sk - 1) - key0 - lp;
                    static_for<32>([&](auto N_) {
                        constexpr int n = decltype(N_)::value;
                        constexpr int cn = kM16 ? 32 * (n >> 4) + 16 * ((n >> 2) & 1) + (n & 3)
                                                : 32 * (n >> 4) + (n & 3) + 8 * ((n >> 2) & 3);
                        if constexpr (!kM16 || ((n >> 3) & 1) == 0) {
                            if (kM16 ? t == 0 : true) mb::mask_one<cn>(s[X][n], E, neg);
                        } else {
                            if (t == 1) mb::mask_one<cn>(s[X][n], E, neg);
                        }
                    });
                }
        };
        // ---- softmax of tile j as 34 units (per block: 4 max units of 8 scores, the decision, 8 exp
        // units of 4 scores, 4 pack units of 8), placed in the gaps of phase 2's 16 MFMA steps ------
        float mx[2][NQ];
        auto u_max = [&](const int X, const int k) __attribute__((always_inline)) {
#pragma unroll
            for (int n = 8 * k; n < 8 * k + 8; ++n) {
                const int t = kM16 ? (n >> 3) & 1 : 0;
                mx[X][t] = (n == 0 || (kM16 && n == 8)) ? s[X][n] : fmaxf(mx[X][t], s[X][n]);
            }
            // (pin: ties each unit's results to its place among the fenced MFMA steps -- without it, IR
            // code sinking moves the softmax below phase 2's last MFMA, past the rescale branch)
#pragma unroll
            for (int t = 0; t < NQ; ++t) pin(mx[X][t]);
        };
        // the row max across the lanes that share a row, the deferred-rescale decision of the block
        // (branch-free: m moves for every row of the block when some row outgrew m + threshold), alpha
        auto u_dec = [&](const int X) __attribute__((always_inline)) {
            bool up = false;
#pragma unroll
            for (int t = 0; t < NQ; ++t) {
                mx[X][t] = kM16 ? pair_max(mb::x16_max(mx[X][t])) : pair_max(mx[X][t]);
                up = up || mx[X][t] > m_[X][t] + thr_raw;
            }
            const bool any = __builtin_amdgcn_ballot_w64(up) != 0;
#pragma unroll
            for (int t = 0; t < NQ; ++t) {
                const float m_new = any ? fmaxf(m_[X][t], mx[X][t]) : m_[X][t];
                const float seen = m_new > 0.5f * kNeg ? 1.f : 0.f;
                const float msc_new = m_new * sc * seen;
                alpha[X][t] = (m_[X][t] <= 0.5f * kNeg) ? 0.f : __builtin_amdgcn_exp2f(msc[X][t] - msc_new);
                m_[X][t] = m_new;
                msc[X][t] = msc_new;
                l_[X][t] *= alpha[X][t];
                pin(msc[X][t]);
                pin(alpha[X][t]);
                pin(l_[X][t]);
            }
        };
        auto u_exp = [&](const int X, const int k) __attribute__((always_inline)) {
#pragma unroll
            for (int n = 4 * k; n < 4 * k + 4; ++n) {
                const int t = kM16 ? (n >> 3) & 1 : 0;
                s[X][n] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[X][n], sc, -msc[X][t]));
                pin(s[X][n]);
                l_[X][t] += s[X][n];
                pin(l_[X][t]);
            }
        };
        auto u_pack = [&](const int X, const int u) __attribute__((always_inline)) {
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                uint32_t x = DT::pack(s[X][8 * u + 2 * w], s[X][8 * u + 2 * w + 1]);
                pin(x);
                P[X][u][w] = x;
            }
        };
        // unit i: 0-3 A max, 4-7 B max, 8 A decision, 9-16 A exp, 17 B decision, 18-25 B exp, 26-29 A pack,
        // 30-33 B pack
        auto run_unit = [&](const int i) __attribute__((always_inline)) {
#ifdef FA_MB_ABL_NOSM
            if (i >= 26) u_pack(i < 30 ? 0 : 1, (i - 26) & 3);
            return;
#endif
            if (i < 8) u_max(i >> 2, i & 3);
            else if (i == 8) u_dec(0);
            else if (i < 17) u_exp(0, i - 9);
            else if (i == 17) u_dec(1);
            else if (i < 26) u_exp(1, i - 18);
            else u_pack(i < 30 ? 0 : 1, (i - 26) & 3);
        };
        constexpr int NU = 34, NS2 = 16;
        // the gap of unit i: spread evenly, a pack unit no earlier than the step after the last MFMA that
        // reads the previous tile's operand u (NS2: after the steps)
        struct Sched {
            static constexpr int last_read(int u) { return kM16 ? (u >> 1) * 2 * DTL + 2 * DTL - 1 : u * DTL + DTL - 1; }
            static constexpr int gap(int i) {
                const int g0 = (i * NS2) / NU;
                if (i < 26) return g0;
                const int lr = last_read((i - 26) & 3) + 1;
                return g0 > lr ? g0 : lr;
            }
        };
        // phase 2: O += V_{j-1}^T . P(j-1)^T (V slot vs; none for the first tile) in 16 steps, each: the
        // next step's V^T fragment (two transposed reads), its 2 / 4 MFMAs, then its softmax units
        auto phase2 = [&](const int vs, auto FIRST) __attribute__((always_inline)) {
            constexpr bool first = decltype(FIRST)::value;
            const char *V = lds + (2 + vs) * T;
            // step st: 32x32x16 kk = st / DTL, dt = st % DTL; 16x16x32 hf = st / (2 DTL), dt = st % (2 DTL)
            auto vread = [&](const int st) __attribute__((always_inline)) {
                u32x2 x0, x1;
                if constexpr (kM16) {
                    const int hf = st / (2 * DTL), dt = st % (2 * DTL);
                    x0 = tr_read(V + 32 * hf * RB + v_addr[dt]);
                    x1 = tr_read(V + (32 * hf + 16) * RB + v_addr[dt]);
                } else {
                    const int kk = st / DTL, dt = st % DTL;
                    x0 = tr_read(V + 16 * kk * RB + v_addr[dt]);
                    x1 = tr_read(V + (16 * kk + 8) * RB + v_addr[dt]);
                }
                return (u32x4){x0[0], x0[1], x1[0], x1[1]};
            };
            constexpr int NSV = 4 * DTL;  // MFMA steps (16 at D = 128, 8 at D = 64)
            u32x4 va[2];
            if constexpr (!first) va[0] = vread(0);
            static_for<NS2>([&](auto S_) {
                constexpr int st = decltype(S_)::value;
                if constexpr (!first && st < NSV) {
                    if constexpr (st + 1 < NSV) va[(st + 1) & 1] = vread(st + 1);
                    if constexpr (kM16) {
                        constexpr int hf = st / (2 * DTL), dt = st % (2 * DTL);
#pragma unroll
                        for (int X = 0; X < 2; ++X)
#pragma unroll
                            for (int qs = 0; qs < 2; ++qs)
                                o16[X][qs][dt] = mb::mfma16<F>(va[st & 1], P[X][2 * hf + qs], o16[X][qs][dt]);
                    } else {
                        constexpr int kk = st / DTL, dt = st % DTL;
#pragma unroll
                        for (int X = 0; X < 2; ++X) o32[X][dt] = mb::mfma32<F>(va[st & 1], P[X][kk], o32[X][dt]);
                    }
                }
                FA_SCHED_FENCE();
                static_for<NU>([&](auto U_) {
                    constexpr int i = decltype(U_)::value;
                    if constexpr (Sched::gap(i) == st) run_unit(i);
                });
                FA_SCHED_FENCE();
            });
            static_for<NU>([&](auto U_) {
                constexpr int i = decltype(U_)::value;
                if constexpr (Sched::gap(i) >= NS2) run_unit(i);
            });
        };
        // the last tile's P.V alone (no softmax beside it)
        auto pv_drain = [&](const int vs) __attribute__((always_inline)) {
            const char *V = lds + (2 + vs) * T;
            if constexpr (kM16) {
#pragma unroll
                for (int hf = 0; hf < 2; ++hf)
#pragma unroll
                    for (int dt = 0; dt < 2 * DTL; ++dt) {
                        const u32x2 x0 = tr_read(V + 32 * hf * RB + v_addr[dt]);
                        const u32x2 x1 = tr_read(V + (32 * hf + 16) * RB + v_addr[dt]);
                        const u32x4 va = {x0[0], x0[1], x1[0], x1[1]};
#pragma unroll
                        for (int X = 0; X < 2; ++X)
#pragma unroll
                            for (int qs = 0; qs < 2; ++qs) o16[X][qs][dt] = mb::mfma16<F>(va, P[X][2 * hf + qs], o16[X][qs][dt]);
                    }
            } else {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                    for (int dt = 0; dt < DTL; ++dt) {
                        const u32x2 x0 = tr_read(V + 16 * kk * RB + v_addr[dt]);
                        const u32x2 x1 = tr_read(V + (16 * kk + 8) * RB + v_addr[dt]);
                        const u32x4 va = {x0[0], x0[1], x1[0], x1[1]};
#pragma unroll
                        for (int X = 0; X < 2; ++X) o32[X][dt] = mb::mfma32<F>(va, P[X][kk], o32[X][dt]);
                    }
            }
        };
        auto rescale = [&]() __attribute__((always_inline)) {
            bool any = false;
#pragma unroll
            for (int X = 0; X < 2; ++X)
#pragma unroll
                for (int t = 0; t < NQ; ++t) any = any || alpha[X][t] != 1.f;
            if (__builtin_amdgcn_ballot_w64(any) == 0) return;
#pragma unroll
            for (int X = 0; X < 2; ++X) {
                if constexpr (kM16) {
#pragma unroll
                    for (int t = 0; t < 2; ++t)
#pragma unroll
                        for (int dt = 0; dt < 2 * DTL; ++dt) o16[X][t][dt] *= alpha[X][t];
                } else {
#pragma unroll
                    for (int dt = 0; dt < DTL; ++dt) o32[X][dt] *= alpha[X][0];
                }
            }
            pin_o();
        };

        // ---- tiles: iteration j issues K_{j+1} and V_j, computes S(j), then P.V of tile j - 1 beside
        // the softmax of tile j; one barrier per tile (K_{j+1} lands in the slot K_{j-1} left, V_j in
        // the slot V_{j-2} left)
        if (n_end > 0) {  // tile 0 alone: the softmax with no P.V beside it (O holds nothing yet)
            if (n_end > 1) stage(kb, ks_, 1, T, kvo);
            stage(vb, vs_, 0, 2 * T, vvo);
            phase1(0);
            mask(0);
            phase2(0, IC<true>{});
            dma_wait();
            __syncthreads();
        }
        for (int j = 1; j < n_end; ++j) {
            if (j + 1 < n_end) stage(kb, ks_, j + 1, ((j + 1) & 1) * T, kvo);
            stage(vb, vs_, j, (2 + (j & 1)) * T, vvo);
            phase1(j);
            mask(j);
            phase2((j - 1) & 1, IC<false>{});
            rescale();
            dma_wait();
            __syncthreads();
        }
        if (n_end > 0) pv_drain((n_end - 1) & 1);  // the last tile's P.V

        // ---- epilogue: O / l, rounded to T, stored (rows past Sq and columns past D are dropped by
        // the descriptor range / offset) ----------------------------------------------------------
        const int os_ = (int)p.o_seqlen_stride;
        const rsrc_t orr = make_rsrc_u(ob + 2 * (int64_t)mw * os_, slab_bytes(min(Sq - mw, kRowB + 32), os_, D));
#pragma unroll
        for (int X = 0; X < 2; ++X) {
            if constexpr (kM16) {
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const float lt = pair_sum(mb::x16_sum(l_[X][t]));
                    const float inv = lt == 0.f ? 1.f : 1.f / lt;
                    const int row = kRowB * X + 16 * t + c16;
#pragma unroll
                    for (int dt = 0; dt < 2 * DTL; ++dt) {
                        const f32x4 &x = o16[X][t][dt];
                        const int d0 = 16 * dt + 4 * g4;
                        __builtin_amdgcn_raw_buffer_store_b64(
                            (u32x2){DT::pack(x[0] * inv, x[1] * inv), DT::pack(x[2] * inv, x[3] * inv)}, orr,
                            (kExactD || d0 < D) ? row * os_ * 2 + 2 * d0 : 0x7ffffff0, 0, 0);
                    }
                }
            } else {
                const float lt = pair_sum(l_[X][0]);
                const float inv = lt == 0.f ? 1.f : 1.f / lt;
                const int row = kRowB * X + r;
#pragma unroll
                for (int dt = 0; dt < DTL; ++dt)
#pragma unroll
                    for (int gp = 0; gp < 4; gp += 2) {
                        const f32x16 &x = o32[X][dt];
                        const uint32_t a0 = DT::pack(x[4 * gp + 0] * inv, x[4 * gp + 1] * inv);
                        const uint32_t a1 = DT::pack(x[4 * gp + 2] * inv, x[4 * gp + 3] * inv);
                        const uint32_t b0 = DT::pack(x[4 * gp + 4] * inv, x[4 * gp + 5] * inv);
                        const uint32_t b1 = DT::pack(x[4 * gp + 6] * inv, x[4 * gp + 7] * inv);
                        const auto x0 = __builtin_amdgcn_permlane32_swap(a0, b0, false, false);
                        const auto x1 = __builtin_amdgcn_permlane32_swap(a1, b1, false, false);
                        const int d0 = dt * 32 + 8 * (gp + h);
                        __builtin_amdgcn_raw_buffer_store_b128((u32x4){x0[0], x1[0], x0[1], x1[1]}, orr,
                                                               (kExactD || d0 < D) ? row * os_ * 2 + 2 * d0 : 0x7ffffff0, 0,
                                                               0);
                    }
            }
        }
        // (the next block's K_0 goes into K slot 0, free since the last tile's barrier; its V_0 is
        // issued after its prologue barrier, when every wave is past this block's last V read)
    }
}

template <class DT, bool C, int kD, bool kExact>
int launch_mb(const fa_fwd_params &p, hipStream_t stream, const bool m16) {
    const int64_t n_qtiles = (p.seqlen_q + kBlockM - 1) / kBlockM;
    const int64_t nwg = n_qtiles * p.num_heads_q * p.batch_size;
    const dim3 grid((uint32_t)w4_grid(nwg));
    if (m16)
        hipLaunchKernelGGL((fa_fwd_mb<DT, C, kD, kExact, true>), grid, dim3(256), 0, stream, p, (int)n_qtiles);
    else
        hipLaunchKernelGGL((fa_fwd_mb<DT, C, kD, kExact, false>), grid, dim3(256), 0, stream, p, (int)n_qtiles);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(FA_ERR_LAUNCH, "HIP launch failed: %s", hipGetErrorString(e));
    set_last_path(m16 ? kPathM16 : kPathM32);
    return FA_OK;
}

}  // namespace fa
