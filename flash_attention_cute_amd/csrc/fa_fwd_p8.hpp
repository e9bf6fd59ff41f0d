#pragma once
// fa_fwd_p8.hpp -- fa_fwd_p8: the paired 8-wave FA2 forward (two waves per SIMD), gfx950.
//
// Same contract, work units and numerics as fa_fwd_w4 (fa_fwd_kernels.hpp; reference
// csrc/flash_attention_template.cuh:138-564): persistent XCD-aware grid over Q blocks of 256 query
// rows of one (batch, q-head), K/V tiles of 64 keys by LDS-DMA, S^T = K.Q^T and O^T += V^T.P^T on
// v_mfma_f32_32x32x16, P rounded to T before P.V, deferred rescale with a rare wave-uniform branch.
//
// What differs is the wave structure. fa_fwd_w4 runs one wave per SIMD (64 rows, 512 registers)
// and hides the softmax VALU between its own MFMAs; a single wave issues a VALU op every 4 cycles
// at most, so that loop is issue-bound. Here every SIMD holds two waves of 32
// rows each (<= 256 registers), and each wave runs fa_fwd_w4's two-phase tile for ONE 32-row block:
//   P1(j): S(j) = K_j . Q^T       16 MFMAs (D = 128) || the late softmax half of tile j - 1; the
//                                 leaders (waves 0-3) also issue the LDS-DMA of K_{j+1} and V_j
//   P2(j): O += P(j-1) . V_{j-1}  16 MFMAs || row max, rescale decision, early softmax half of j
// Leaders run P1(j) P2(j) | barrier, followers (wave w + 4, same SIMD) P2(j-1) P1(j) | barrier, so
// the SIMD has two instruction streams to fill the matrix pipe's gaps from. One barrier per tile
// publishes K_{j+1} and V_j; V has a 4-slot ring because a follower reads V_{j-2} while the
// leaders' DMA of V_j is in flight. The arithmetic (and its order) is fa_fwd_w4's: outputs are
// bit-identical.
//
// Measured (in-kernel stamps, C2): 195k cycles per Q block against 210k for
// fa_fwd_w4 (and 174k without the softmax), but the chip holds 1.62 GHz under it against 1.76:
// the denser issue is paid back by DVFS, and end to end fa_fwd_p8 is 1-4 % slower. It stays a
// cross-check variant (FA_GFX950_VARIANT=p8), in the parity sweep.
//
// Registers per wave: 256 at two waves per SIMD, which the compiler splits 128 arch / 128 AGPR once
// a kernel uses AGPRs. O^T (32 rows x D) sits in a[0 : 16 DTL) and the Q fragments in a[64 : 64 + 4
// KS), literal AGPRs only inline asm touches (fa_agpr_asm.inc; _asm_check gates it; an empty asm
// clobbering them in every MFMA gap keeps compiler spills out), a96..a127 are the compiler's. The
// arch VGPRs hold S (32), P (16: ONE tile -- phase B overwrites P(j-1) word by word with P(j), each
// 16-key k-step only after its P.V MFMAs have issued; an MFMA reads its A/B operands at issue), the
// K / V fragments and the softmax state.
#include "fa_fwd_kernels.hpp"

namespace fa {

template <int QB>
__device__ __forceinline__ void p8_qload(const rsrc_t &rs, const int voff, const bool nop) {
#define FA_CASE(N) \
    if constexpr (QB == N) fa_agpr_qload_##N(rs, voff, nop);
    FA_CASE(64) FA_CASE(68) FA_CASE(72) FA_CASE(76) FA_CASE(80) FA_CASE(84) FA_CASE(88) FA_CASE(92)
#undef FA_CASE
}
// S = K . Q^T k-step into arch VGPRs, B = the Q fragment in a[QB .. QB+3]; first: C = 0
template <bool kF16, int QB>
__device__ __forceinline__ void p8_mfma_sq(const bool first, f32x16 &acc, const u32x4 &a) {
#define FA_CASE(N)                                                                         \
    if constexpr (QB == N) {                                                               \
        if (first) {                                                                       \
            if constexpr (kF16) fa_sq_f16_##N##_1(acc, a); else fa_sq_bf16_##N##_1(acc, a); \
        } else {                                                                           \
            if constexpr (kF16) fa_sq_f16_##N##_0(acc, a); else fa_sq_bf16_##N##_0(acc, a); \
        }                                                                                  \
    }
    FA_CASE(64) FA_CASE(68) FA_CASE(72) FA_CASE(76) FA_CASE(80) FA_CASE(84) FA_CASE(88) FA_CASE(92)
#undef FA_CASE
}
// The O^T and Q AGPRs are live across the whole kernel but only inline asm touches them, so the
// compiler sees them free between two asm statements and may park a spilled VGPR there. This
// empty statement clobbers all of them; placed in every MFMA gap, no spill range can span it.
__device__ __forceinline__ void p8_reserve_agprs() {
    asm volatile("" :::
        "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15",
        "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30",
        "a31", "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45",
        "a46", "a47", "a48", "a49", "a50", "a51", "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60",
        "a61", "a62", "a63", "a64", "a65", "a66", "a67", "a68", "a69", "a70", "a71", "a72", "a73", "a74", "a75",
        "a76", "a77", "a78", "a79", "a80", "a81", "a82", "a83", "a84", "a85", "a86", "a87", "a88", "a89", "a90",
        "a91", "a92", "a93", "a94", "a95");
}

template <class DT, bool kCausal, int kD, bool kExactD>
__global__ __launch_bounds__(512, 1) void fa_fwd_p8(const fa_fwd_params p, const int n_qtiles,
                                                    unsigned long long *stamps) {
    // Diagnostic build only (-DFA_STAMPS=1, scripts/stamps.py ... p8): per-wave phase totals
#ifdef FA_STAMPS
    unsigned long long st_t0 = 0, st_rt0 = 0, st_acc[5] = {0, 0, 0, 0, 0};
#define P8_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
    (void)stamps;
#define P8_STAMP(v)
#endif
    using G = Geo<kD>;
    constexpr bool F = DT::kIsF16;
    constexpr int KS = G::kKSteps;    // k-steps of S^T = K.Q^T: 8 / 4
    constexpr int DTL = G::kDTiles;   // 32-row d tiles of O^T: 4 / 2
    constexpr int RB = G::kRowBytes;
    constexpr int T = G::kTileBytes;  // one K or V tile: 16 / 8 KiB
    constexpr int NP = T / 4 / 1024;  // LDS-DMA pieces per leader wave per K or V tile: 4 / 2
    constexpr int ROWS_PER_PIECE = 1024 / RB;
    constexpr int QB = 64;            // Q fragment of k-step ks: a[64 + 4 ks]
    constexpr int VOFF = 2 * T;       // LDS: K slots 0, 1 | V slots 0..3
    constexpr int kOStores = DTL * 2;  // O stores per wave and block
    constexpr int kVRA = 2;  // V^T reads issued this many MFMAs ahead (3: same speed)
    __shared__ __attribute__((aligned(1024))) char lds[6 * T];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool lead = wave < 4;  // waves w and w + 4 share a SIMD
    const int r = lane & 31;
    const int h = lane >> 5;

    const int D = (int)p.headdim;
    const int Sq = (int)p.seqlen_q, Sk = (int)p.seqlen_kv;
    const float sc = p.softmax_scale;
    const float thr_raw = kRescaleThr / sc;
    const int diag = Sk - Sq;
    const int n_blocks = (Sk + kBlockN - 1) / kBlockN;

    // ---- persistent schedule (fa_fwd_w4) ------------------------------------------------------
    const uint32_t nwg = (uint32_t)n_qtiles * (uint32_t)p.num_heads_q * (uint32_t)p.batch_size;
    const uint32_t xcd = blockIdx.x & 7, cx = blockIdx.x >> 3;
    const uint32_t gx = (gridDim.x - xcd + 7) >> 3;
    const uint32_t cnt = (nwg - xcd + 7) >> 3;
    auto block_of = [&](const uint32_t rnd_) { return rnd_ * gx + ((rnd_ & 1) ? gx - 1 - cx : cx); };
    uint32_t rnd = 0, kblk = block_of(0);
    if (kblk >= cnt) return;

    const char *qb, *kb, *vb;
    char *ob;
    int m0, mw, n_end, n_pipe;
    auto set_block = [&](const uint32_t k) {
        const Work wk = decode_work<kCausal>(nwg, xcd + 8 * k, n_qtiles, (int)p.num_heads_q, (int)p.head_q_per_group);
        const int hkv = wk.hq / (int)p.head_q_per_group;
        qb = (const char *)p.q_ptr + 2 * ((int64_t)wk.b * p.q_batch_stride + (int64_t)wk.hq * p.q_head_stride);
        kb = (const char *)p.k_ptr + 2 * ((int64_t)wk.b * p.k_batch_stride + (int64_t)hkv * p.k_head_stride);
        vb = (const char *)p.v_ptr + 2 * ((int64_t)wk.b * p.v_batch_stride + (int64_t)hkv * p.v_head_stride);
        ob = (char *)p.o_ptr + 2 * ((int64_t)wk.b * p.o_batch_stride + (int64_t)wk.hq * p.o_head_stride);
        m0 = wk.qtile * kBlockM;
        mw = m0 + 32 * wave;  // this wave's 32 rows
        n_end = n_blocks;
        if (kCausal) {
            const int x = diag + min(m0 + kBlockM, Sq);
            const int nb = x <= 0 ? 0 : (x + kBlockN - 1) / kBlockN;
            n_end = min(nb, n_blocks);
        }
        // leading tiles with no masked score for any row of the workgroup (same for all waves)
        n_pipe = Sk / kBlockN;
        if (kCausal) {
            const int x = m0 + diag + 1;
            n_pipe = min(n_pipe, x <= 0 ? 0 : x / kBlockN);
        }
        n_pipe = min(n_pipe, n_end);
    };
    set_block(kblk);

    // ---- Q: this wave's 32 rows straight from HBM into the Q AGPRs (retired by a vmcnt wait) ----
    // lane (h, r) holds Q[mw + r][16 ks + 8 h + 0..7] in a[64 + 4 ks]; rows >= Sq read as 0
    auto load_q = [&]() __attribute__((always_inline)) {
        const int qs = (int)p.q_seqlen_stride;
        const rsrc_t qr = make_rsrc_u(qb + 2 * (int64_t)mw * qs, slab_bytes(min(Sq - mw, 32), qs, D));
        static_for<KS>([&](auto KK) {
            constexpr int ks = decltype(KK)::value;
            const bool ok = kExactD || 16 * ks + 8 * h < D;  // columns past D read as 0
            p8_qload<QB + 4 * ks>(qr, ok ? r * qs * 2 + 32 * ks + 16 * h : 0x7ffffff0, ks == 0);
        });
    };
    load_q();

    // ---- LDS-DMA staging (leaders): wave w writes pieces w*NP + n of each K and V tile --------
    const int ks_ = (int)p.k_seqlen_stride, vs_ = (int)p.v_seqlen_stride;
    const int wl = wave & 3;
    // Per-lane source offsets of piece n, computed when issued (registers are scarce at two waves
    // per SIMD; the leaders' phase A has VALU slack): the row is (wl NP + n) RPP + 16 l / RB and the
    // chunk the slot XOR the swizzle's row term (the XOR swizzles are involutions)
    auto src_off = [&](const int n, const int stride, const bool is_k) __attribute__((always_inline)) {
        const int row = (wl * NP + n) * ROWS_PER_PIECE + (16 * lane) / RB;
        const int slot = ((16 * lane) % RB) / 16;
        const int ch = (is_k ? G::k_off(row, slot) : G::v_off(row, slot)) % RB / 16;
        return (kExactD || ch * 8 < D) ? row * stride * 2 + 16 * ch : 0x7ffffff0;
    };

    const uint32_t lds0 = lds_u32(lds);
    const uint32_t lds_w = lds0 + wl * NP * 1024;  // this leader's pieces of slot 0
    auto stage_k0 = [&]() {  // K_0 of the current block into K slot 0
        const rsrc_t kr = make_rsrc_u(kb, slab_bytes(min(Sk, kBlockN), ks_, D));
        static_for<NP>([&](auto N) {
            constexpr int n = decltype(N)::value;
            dma_one(kr, lds_w + n * 1024, src_off(n, ks_, true), n == 0);
        });
    };

    // ---- per-lane LDS read addresses (fa_fwd_w4) --------------------------------------------
    const int g = lane >> 4;
    const int qq = (lane >> 2) & 3;
    const int pp = lane & 3;
    int v_addr[DTL];
#pragma unroll
    for (int dt = 0; dt < DTL; ++dt)
        v_addr[dt] = G::v_off(4 * (g >> 1) + qq, dt * 4 + 2 * (g & 1) + (pp >> 1)) + 8 * (pp & 1);
    // K fragment of k-step ks: Geo::k_off(r, 2 ks + h) = k_off(r, h) ^ 32 ks (the k-step moves only
    // bits 5-7 of the swizzled chunk; the row term sits above them) -- one VGPR for all k-steps
    const int k_addr0 = G::k_off(r, h);
    static_assert(kD == 128 || kD == 64, "k_addr0");

    // ---- state --------------------------------------------------------------------------------
    struct Sm {
        float m, msc, alpha, mt;  // running max (unscaled), m*sc, alpha of the last decision, m + thr
        float mE, mO;             // two max chains over the tile (mE then holds the tile max)
        float l, t;               // this lane's half of the row sum: finished scores / this tile's early ones
        uint64_t rmask;
    };
    Sm st;
    // S of a tile: key half 0 (its scores are exponentiated early, in the tile's phase 2) and key
    // half 1 (late, in the next tile's phase 1, so it is double-buffered by tile parity)
    f32x16 S0;
    f32x16 S1[2];
    u32x4 P[4];  // rounded P of one tile, per 16-key k-step (see the header)

    // max chain unit i (0..15): scores i of both halves of the tile of parity c
    auto u_max = [&](const int c, const int i) {
        float &mm = (i & 1) ? st.mO : st.mE;
        mm = (i < 2) ? fmaxf(S0[i], S1[c][i]) : fmaxf(mm, fmaxf(S0[i], S1[c][i]));
        pin(mm);
    };
    // the rescale decision: the ballot (k = 0); the new reference (k = 1, rare, wave-uniform)
    auto u_dec = [&](const int k) {
        if (k == 0) {
            const float mx = fmaxf(st.mE, st.mO);
            uint64_t bm = __builtin_amdgcn_ballot_w64(mx > st.mt);
            asm volatile("" : "+s"(bm));
            st.rmask = bm;
            st.mE = mx;
            pin(st.mE);
        } else if (__builtin_expect(st.rmask != 0, 0)) {
            const float m_new = fmaxf(st.m, pair_max(st.mE));
            const float seen = m_new > 0.5f * kNeg ? 1.f : 0.f;
            const float msc_new = m_new * sc * seen;
            st.alpha = (st.m <= 0.5f * kNeg) ? 0.f : __builtin_amdgcn_exp2f(st.msc - msc_new);
            st.m = m_new;
            st.mt = m_new + thr_raw;
            st.msc = msc_new;
            pin(st.msc);
            pin(st.alpha);
        }
    };
    // P = exp2(s * sc - m * sc) of score v of half 0 (early) or of half 1 of parity c (late), in place
    auto u_exp = [&](const int c, const int hf, const int v) {
        f32x16 &s = hf ? S1[c] : S0;
        float x = __builtin_amdgcn_exp2f(__builtin_fmaf(s[v], sc, -st.msc));
        pin(x);
        s[v] = x;
    };
    // row sum (early scores -> t, late -> l) and, for odd v, the rounded pair (v - 1, v) into P
    auto u_fin = [&](const int c, const int hf, const int v) {
        const f32x16 &s = hf ? S1[c] : S0;
        float &acc = hf ? st.l : st.t;
        acc = (hf == 0 && v == 0) ? s[0] : acc + s[v];
        pin(acc);
        if (v & 1) {
            uint32_t w = DT::pack(s[v - 1], s[v]);
            pin(w);
            P[2 * hf + (v >> 3)][(v & 7) >> 1] = w;
        }
    };
    // o_zero: O holds no P.V yet (a block's first tile): only l is updated (fa_fwd_w4)
    auto rescale = [&](const bool o_zero) {
        if (__builtin_expect(st.rmask != 0, 0)) {
            if (!o_zero) agpr_scale<DTL, false>(st.alpha);
            st.l = __builtin_fmaf(st.l, st.alpha, st.t);
            st.alpha = 1.f;
        } else {
            st.l += st.t;
        }
    };

    // ---- phase 1: S(j) = K_j . Q^T into S0, S1[c] (2 KS single MFMAs) || the late softmax half of
    //      tile j - 1 (S1[c ^ 1]); leaders: the LDS-DMA of K_{j+1} and V_j ------------------------
    constexpr int G1 = 2 * KS;  // 16 / 8 MFMAs
    auto late_gap = [](const int v) { return (v * G1) / 16; };  // late unit v (0..15) -> gap
    auto phase1 = [&](const char *K, auto PAR, auto DMA, auto SM, const rsrc_t &kr, const rsrc_t &vr,
                      const uint32_t k_dst, const uint32_t v_dst) __attribute__((always_inline)) {
        constexpr int c = decltype(PAR)::value, pc = c ^ 1;
        constexpr bool dma = decltype(DMA)::value, do_sm = decltype(SM)::value;
        u32x4 kf[2][2];  // [buffer][key half]
#pragma unroll
        for (int x = 0; x < 2; ++x) kf[0][x] = *(const u32x4 *)(K + x * 32 * RB + k_addr0);
        static_for<G1>([&](auto GG) {
            constexpr int gi = decltype(GG)::value;
            constexpr int ks = gi >> 1, x = gi & 1, cb = ks & 1;
            if constexpr (ks > 0 && x == 0) __builtin_amdgcn_s_waitcnt(kLgkm0);
            if constexpr (x == 0) p8_mfma_sq<F, QB + 4 * ks>(ks == 0, S0, kf[cb][0]);
            else p8_mfma_sq<F, QB + 4 * ks>(ks == 0, S1[c], kf[cb][1]);
            p8_reserve_agprs();
            FA_SCHED_FENCE();
            if constexpr (ks + 1 < KS && x == 0) {
                const int ka = k_addr0 ^ (32 * (ks + 1));
                kf[cb ^ 1][0] = *(const u32x4 *)(K + ka);
                kf[cb ^ 1][1] = *(const u32x4 *)(K + 32 * RB + ka);
            }
            if constexpr (dma && x == 1) {  // leaders: K pieces in the first k-steps, then V
                if constexpr (ks < NP) dma_one(kr, k_dst + ks * 1024, src_off(ks, ks_, true), ks == 0);
                else if constexpr (ks - NP < NP)
                    dma_one(vr, v_dst + (ks - NP) * 1024, src_off(ks - NP, vs_, false), ks == NP);
            }
            if constexpr (do_sm) {
                static_for<16>([&](auto VV) {
                    constexpr int v = decltype(VV)::value;
                    if constexpr (late_gap(v) == gi) {
                        u_exp(pc, 1, v);
                        if constexpr (v > 0) u_fin(pc, 1, v - 1);
                    }
                });
            }
            FA_SCHED_FENCE();
        });
        if constexpr (do_sm) u_fin(pc, 1, 15);
    };
    // the late half without MFMAs (the drain)
    auto sm_late = [&](auto PAR) __attribute__((always_inline)) {
        constexpr int c = decltype(PAR)::value;
        static_for<16>([&](auto VV) {
            constexpr int v = decltype(VV)::value;
            u_exp(c, 1, v);
            u_fin(c, 1, v);
        });
    };
    // causal diagonal / Sk tail: scores of keys past a row's last visible key -> kNeg
    auto mask = [&](auto PAR, const int key0) __attribute__((always_inline)) {
        constexpr int c = decltype(PAR)::value;
        s_ready(S0, S1[c]);  // asm MFMA results -> VALU reads
        const int row = mw + r;
        const int lim = kCausal ? min(Sk - 1, row + diag) : Sk - 1;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int kk = key0 + (i & 3) + 8 * (i >> 2) + 4 * h;
            if (kk > lim) S0[i] = kNeg;
            if (kk + 32 > lim) S1[c][i] = kNeg;
        }
    };

    // ---- phase 2: O += P . V (4 DTL single MFMAs into the AGPRs) || the early softmax half of the
    //      tile of parity c: row max, rescale decision, scores 0..15 (SM; else the drain) ------------
    constexpr int G2 = 4 * DTL;  // 16 / 8 MFMAs
    // gap u = after MFMA u. Max units from gap 1 (the S MFMAs are two MFMA issues back by then), the
    // ballot, the rare branch, then the 16 early exp / fin pairs. A fin writes the P word of k-step
    // v / 8, whose DTL P.V MFMAs (gaps DTL kk .. DTL kk + DTL - 1) must have issued (an MFMA reads
    // its A / B operands at issue)
    constexpr int kMaxG0 = 1;
    constexpr int kMaxPer = G2 >= 16 ? 4 : 8;
    constexpr int kDecG = kMaxG0 + (16 + kMaxPer - 1) / kMaxPer;
    constexpr int kExpG0 = kDecG + 1;
    struct XG {
        static constexpr int base(int v) { return kExpG0 + (v * (G2 - kExpG0)) / 16; }
        static constexpr int at(int v) {  // exp gap; its fin runs one gap later
            return base(v) > DTL * (v >> 3) + DTL - 2 ? base(v) : DTL * (v >> 3) + DTL - 2;
        }
    };
    static_assert(kExpG0 < G2, "p8 softmax schedule");
    auto phase2 = [&](const char *V, auto PAR, auto SM) __attribute__((always_inline)) {
        constexpr int c = decltype(PAR)::value;
        constexpr bool do_sm = decltype(SM)::value;
        // V^T fragments of MFMA u = (kk = u / DTL, dt = u % DTL), read kVRA MFMAs ahead
        u32x4 va[kVRA + 1];
        auto rd = [&](const int u) {
            const int kk = u / DTL, dt = u % DTL;
            const int rowoff = ((kk >> 1) * 32 + (kk & 1) * 16) * RB;
            const u32x2 lo = tr_read(V + rowoff + v_addr[dt]);
            const u32x2 hi = tr_read(V + rowoff + 8 * RB + v_addr[dt]);
            va[u % (kVRA + 1)] = (u32x4){lo[0], lo[1], hi[0], hi[1]};
        };
        static_for<kVRA>([&](auto U) { rd(decltype(U)::value); });
        static_for<G2>([&](auto GG) {
            constexpr int u = decltype(GG)::value;
            constexpr int kk = u / DTL, dt = u % DTL;
            // fragments of MFMA u landed (the reads of the next kVRA - 1 MFMAs may still be in flight)
            constexpr int ahead = (G2 - 1 - u) < (kVRA - 1) ? (G2 - 1 - u) : (kVRA - 1);
            __builtin_amdgcn_s_waitcnt(kLgkm0 | ((2 * ahead) << 8));
            agpr_mfma<F, 16 * dt>(va[u % (kVRA + 1)], P[kk]);
            p8_reserve_agprs();
            FA_SCHED_FENCE();
            if constexpr (u + kVRA < G2) rd(u + kVRA);
            if constexpr (do_sm) {
                static_for<16>([&](auto M) {
                    constexpr int i = decltype(M)::value;
                    if constexpr (kMaxG0 + i / kMaxPer == u) u_max(c, i);
                });
                if constexpr (u == kDecG) u_dec(0);
                if constexpr (u == kExpG0) u_dec(1);
                static_for<16>([&](auto VV) {
                    constexpr int v = decltype(VV)::value;
                    if constexpr (XG::at(v) + 1 == u) u_fin(c, 0, v);
                });
                static_for<16>([&](auto VV) {
                    constexpr int v = decltype(VV)::value;
                    if constexpr (XG::at(v) == u) u_exp(c, 0, v);
                });
            }
            FA_SCHED_FENCE();
        });
        if constexpr (do_sm) {
            static_for<16>([&](auto VV) {
                constexpr int v = decltype(VV)::value;
                if constexpr (XG::at(v) + 1 >= G2) u_fin(c, 0, v);
            });
        }
    };

    // one pipelined iteration of tile j (PAR = j & 1). Leaders: P1(j) [mask] P2(j) | wait | barrier.
    // Followers: P2(j-1) P1(j) [mask] | barrier. (Measured alternatives, same speed or slower: a
    // second barrier between the phases; followers in lockstep with the leaders; s_setprio 1 for
    // the followers -1 to -3 %.)
#ifdef FA_P8_NOSM
    constexpr int kSm = 0;  // timing only: no softmax in the loop (results are garbage)
#else
    constexpr int kSm = 1;
#endif
    const uint32_t full_k = slab_bytes(kBlockN, ks_, D), full_v = slab_bytes(kBlockN, vs_, D);
    auto tile_rsrc = [&](const char *base, const int j, const uint32_t full, const int stride) {
        const int key0 = j * kBlockN;
        const int rows = Sk - key0;
        return make_rsrc_u(base + 2 * (int64_t)key0 * stride, rows >= kBlockN ? full : slab_bytes(rows, stride, D));
    };
    auto vslot = [&](const int j) { return lds + VOFF + ((j + 4) & 3) * T; };
    auto iter_lead = [&](const int j, auto PAR, auto MASKED, auto DMA) __attribute__((always_inline)) {
        constexpr int c = decltype(PAR)::value;
        P8_STAMP(sa);
        const rsrc_t kr = tile_rsrc(kb, j + 1, full_k, ks_);
        const rsrc_t vr = tile_rsrc(vb, j, full_v, vs_);
        const uint32_t k_dst = lds_w + (uint32_t)(c ^ 1) * T;       // K_{j+1}
        const uint32_t v_dst = lds_u32(vslot(j)) + wl * NP * 1024;  // V_j
        phase1(lds + c * T, PAR, DMA, IC<kSm>{}, kr, vr, k_dst, v_dst);
        if constexpr (decltype(MASKED)::value) mask(PAR, j * kBlockN);
        P8_STAMP(sb);
        phase2(vslot(j - 1), PAR, IC<kSm>{});
        rescale(j == 0);
        P8_STAMP(sc_);
        dma_wait();
        P8_STAMP(sd);
        __syncthreads();
#ifdef FA_STAMPS
        const unsigned long long se = __builtin_amdgcn_s_memtime();
        st_acc[0] += sb - sa;
        st_acc[1] += sc_ - sb;
        st_acc[2] += sd - sc_;
        st_acc[3] += se - sd;
        st_acc[4] += 1;
#endif
    };
    // followers: phase 2 of tile j - 1 (parity c ^ 1), then phase 1 of tile j
    auto iter_follow = [&](const int j, auto PAR, auto MASKED) __attribute__((always_inline)) {
        constexpr int c = decltype(PAR)::value;
        P8_STAMP(sa);
        phase2(vslot(j - 2), IC<c ^ 1>{}, IC<kSm>{});  // P.V of tile j - 2, early softmax of tile j - 1
        rescale(j <= 1);
        P8_STAMP(sb);
        const rsrc_t none = make_rsrc(nullptr, 0u);
        phase1(lds + c * T, PAR, IC<0>{}, IC<kSm>{}, none, none, 0u, 0u);
        if constexpr (decltype(MASKED)::value) mask(PAR, j * kBlockN);
        P8_STAMP(sc_);
        __syncthreads();
#ifdef FA_STAMPS
        const unsigned long long se = __builtin_amdgcn_s_memtime();
        st_acc[0] += sc_ - sb;  // phase 1
        st_acc[1] += sb - sa;   // phase 2
        st_acc[3] += se - sc_;
        st_acc[4] += 1;
#endif
    };

    if (lead) stage_k0();
    for (;;) {
        // ---- block prologue: Q and (leaders) K_0 in flight ----------------------------------
#ifdef FA_STAMPS
        st_t0 = __builtin_amdgcn_s_memtime();
        st_rt0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int i = 0; i < 5; ++i) st_acc[i] = 0;
#endif
        st = {kNeg, 0.f, 1.f, kNeg + thr_raw, kNeg, kNeg, 0.f, 0.f, 0ull};
        fa_agpr_zero_2();  // a0..a63: O^T (D = 128; a0..a31 at D = 64)
        // tiles -1 and -2 of the pipeline are empty: S = kNeg gives P = 0, P buffers 0, and their V
        // slots (3 and 2) are zeroed so that 0 * V stays 0
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            S0[i] = kNeg;
            S1[0][i] = kNeg;
            S1[1][i] = kNeg;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) P[k] = (u32x4){0, 0, 0, 0};
        __syncthreads();  // every wave is past the previous block's reads of V slots 2 and 3
        {
            constexpr int per_thread = 2 * T / 512 / 16;
#pragma unroll
            for (int i = 0; i < per_thread; ++i)
                *(u32x4 *)(lds + VOFF + 2 * T + (i * 512 + tid) * 16) = (u32x4){0, 0, 0, 0};
        }
        // Q, K_0 landed; the previous block's O stores (issued after them) may stay in flight
        if (rnd == 0) dma_wait(); else __builtin_amdgcn_s_waitcnt(vmcnt_enc(kOStores));
        __syncthreads();  // K_0 and the zeroed slots visible to every wave
        P8_STAMP(s_pro);

        const int n_unm = n_pipe, n_loop = n_end;
        if (lead) {
            for (int j = 0; j < n_unm; j += 2) {
                iter_lead(j, IC<0>{}, IC<0>{}, IC<1>{});
                if (j + 1 < n_unm) iter_lead(j + 1, IC<1>{}, IC<0>{}, IC<1>{});
            }
            int j = n_unm;
            if ((j & 1) && j < n_loop) iter_lead(j++, IC<1>{}, IC<1>{}, IC<1>{});
            for (; j < n_loop; j += 2) {
                iter_lead(j, IC<0>{}, IC<1>{}, IC<1>{});
                if (j + 1 < n_loop) iter_lead(j + 1, IC<1>{}, IC<1>{}, IC<1>{});
            }
        } else {
            for (int j = 0; j < n_unm; j += 2) {
                iter_follow(j, IC<0>{}, IC<0>{});
                if (j + 1 < n_unm) iter_follow(j + 1, IC<1>{}, IC<0>{});
            }
            int j = n_unm;
            if ((j & 1) && j < n_loop) iter_follow(j++, IC<1>{}, IC<1>{});
            for (; j < n_loop; j += 2) {
                iter_follow(j, IC<0>{}, IC<1>{});
                if (j + 1 < n_loop) iter_follow(j + 1, IC<1>{}, IC<1>{});
            }
        }

        P8_STAMP(s_loop_end);
        // ---- next block: Q and K_0 in flight under the drain (every wave is past the last barrier:
        // the Q AGPRs and both K slots are free; the drain reads V slots only) -------------------
        char *const ob_c = ob;
        const int mw_c = mw;
        kblk = block_of(++rnd);
        const bool more = kblk < cnt;
        const int last = n_loop - 1;
        if (more) {
            set_block(kblk);
            load_q();
            if (lead) stage_k0();
        }
        // drain: followers first run phase 2 of the last tile (its early softmax beside P.V of the
        // tile before); then everybody the late softmax half of the last tile and its P.V
        if (last & 1) {
            if (!lead) {
                phase2(vslot(last - 1), IC<1>{}, IC<1>{});
                rescale(last <= 0);
            }
            sm_late(IC<1>{});
            phase2(vslot(last), IC<1>{}, IC<0>{});
        } else {
            if (!lead) {
                phase2(vslot(last - 1), IC<0>{}, IC<1>{});
                rescale(last <= 0);
            }
            sm_late(IC<0>{});
            phase2(vslot(last), IC<0>{}, IC<0>{});
        }
        P8_STAMP(s_pipe_end);
        // ---- epilogue: O / l, row per lane, 16-B stores after a half-wave swap -------------------
        mfma_drain();  // last asm MFMA -> AGPR reads
        const int os_ = (int)p.o_seqlen_stride;
        const rsrc_t orr = make_rsrc(ob_c + 2 * (int64_t)mw_c * os_, slab_bytes(min(Sq - mw_c, 32), os_, D));
        {
            f32x16 o[DTL];
            o[0] = agpr_read16<0>();
            o[1] = agpr_read16<16>();
            if constexpr (DTL == 4) {
                o[2] = agpr_read16<32>();
                o[3] = agpr_read16<48>();
            }
            const float l_tot = pair_sum(st.l);
            const float inv = (l_tot == 0.f) ? 1.f : 1.f / l_tot;
            const int orow = r * os_ * 2;
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
                    __builtin_amdgcn_raw_buffer_store_b128((u32x4){x0[0], x1[0], x0[1], x1[1]}, orr,
                                                           (kExactD || d0 < D) ? orow + 2 * d0 : 0x7ffffff0, 0, 0);
                }
            }
        }
#ifdef FA_STAMPS
        {
            __builtin_amdgcn_s_waitcnt(0);
            const unsigned long long s_end = __builtin_amdgcn_s_memtime(), rt_end = __builtin_amdgcn_s_memrealtime();
            if (stamps && lane == 0) {  // the fa_fwd_w4 record, 8 waves per Q block
                const uint32_t blk = xcd + 8 * block_of(rnd - 1);
                unsigned long long *o = stamps + ((size_t)blk * 8 + wave) * 12;
                o[0] = s_end - st_t0;
                for (int i = 0; i < 5; ++i) o[1 + i] = st_acc[i];
                o[6] = s_pipe_end - s_loop_end;
                o[7] = s_pro - st_t0;
                o[8] = s_end - s_pipe_end;
                o[9] = rt_end - st_rt0;
                o[10] = st_t0;
                o[11] = xcc_id();
            }
        }
#endif
        if (!more) break;
    }  // persistent block loop
#undef P8_STAMP
}


template <class DT, bool C, int kD, bool kExact>
int launch_p8(const fa_fwd_params &p, hipStream_t stream) {
    const int64_t n_qtiles = (p.seqlen_q + kBlockM - 1) / kBlockM;
    const int64_t nwg = n_qtiles * p.num_heads_q * p.batch_size;
    hipLaunchKernelGGL((fa_fwd_p8<DT, C, kD, kExact>), dim3((uint32_t)w4_grid(nwg)), dim3(512), 0, stream, p,
                       (int)n_qtiles, stamp_buffer());
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(FA_ERR_LAUNCH, "HIP launch failed: %s", hipGetErrorString(e));
    set_last_path(kPathP8);
    return FA_OK;
}

}  // namespace fa
