#pragma once
// fa_decode.hpp -- split-KV ("flash-decoding") forward for few query rows per kv-head, gfx950.
//
// The reference has no split-KV kernel (TODO at reference README.md:20). Its decode path is the
// q-head pack of reference csrc/flash_attention_api.cpp:72-83: with Sq == 1 the group of q-heads
// that share one kv-head becomes the rows of one problem, and the prefill kernel then runs one
// 128-row CTA per (batch, kv-head) over the whole K/V stream -- B * Hkv CTAs, most rows empty.
// Decode is HBM-bound (every K/V byte is read once per step), so this kernel is built around the
// K/V stream instead of the MFMA:
//
//   * a row block is up to 32 (q-head, position) rows of one (batch, kv-head): rows_total =
//     head_q_per_group * Sq, row r -> q-head hkv * g + r / Sq, position r % Sq. The host's Sq == 1
//     pack (g' = 1, Sq' = g) and unpacked GQA with a few query positions (speculative decode,
//     causal per position) map onto the same rows; K/V are read once per group either way;
//   * one workgroup = 4 wave64s on one (batch, kv-head, row block, key split); each wave owns a
//     contiguous quarter of the split's 32-key tiles and streams them through its OWN 2-slot
//     LDS ring by LDS-DMA (buffer_load ... lds, 1 KiB per wave-instruction, XOR swizzle applied
//     on the source offsets as in fa_fwd_w4). No barrier in the key loop: a wave only waits for
//     its own DMA (vmcnt);
//   * per tile S^T = K.Q^T and O^T += V^T.P^T with v_mfma_f32_32x32x16 (fragment layouts of
//     fa_fwd_w8: each lane owns one row, the rounded P^T is directly the B operand); MFMA time is
//     ~1/4 of the tile's HBM time at 1 wave per SIMD, so padding rows to 32 costs nothing;
//   * the 4 wave partials are merged in LDS (log-sum-exp weights); with n_split == 1 the
//     workgroup writes O, otherwise fp32 partials (O / l and lse) go to a caller-provided
//     workspace and fa_decode_combine merges the splits.
//
// Numerics: S in fp32, P = exp2(S*s' - m*s') rounded (RNE) to T before P.V, row sums of the fp32
// P, deferred max (guide T13, as fa_fwd_w4). The split changes only which running max a P is
// rounded against, which is within the stated fp16 / bf16 tolerance (tests/test_gpu_parity.py).
// Rows that see no key are 0 (DESIGN.md quirk iii).
#include "fa_fwd_kernels.hpp"

namespace fa {

// LDS-DMA with the non-temporal policy (K/V of a decode step are read once)
__device__ __forceinline__ void dma_one_nt(const rsrc_t &rs, const uint32_t lds, const int voff, const bool nop) {
    if (nop)
        asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %1, 0 offen nt lds" ::"v"(voff), "s"(rs), "{m0}"(lds)
                     : "memory");
    else
        asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen nt lds" ::"v"(voff), "s"(rs), "{m0}"(lds)
                     : "memory");
}

template <int kD>
struct DecGeo {
    using G = Geo<kD>;
    static constexpr int RB = G::kRowBytes;
    static constexpr int kTile = kDecKeys * RB;     // bytes of one K (or V) tile: 8 / 4 KiB
    static constexpr int kPieces = kTile / 1024;    // LDS-DMA pieces per K (or V) tile
    static constexpr int kSlot = 2 * kTile;         // K + V
    static constexpr int kWaveLds = 2 * kSlot;      // 2-slot ring per wave
    static constexpr int kLds = kDecWaves * kWaveLds;
    static constexpr int kQPiecesPerWave = kDecRows * RB / 1024 / kDecWaves;  // 2 / 1
};

// Fused merge of a unit's n_split partials by the last of its workgroups (fa_decode, a.cnt): the same
// arithmetic as fa_decode_combine (weights 2^(lse - M) in split order, acc / L), spread over the
// workgroup: lse of every (split, row) into LDS, each row's weights by one thread, then a float4 of
// one valid row per thread per pass. Loads are device-scope (sc1: not from this CU's L1).
template <class DT, int kD, bool kExactD>
__device__ __forceinline__ void decode_merge(const fa_fwd_params &p, const DecArgs &a, const int unit, const int b,
                                          const int hkv, const int rb) {
    __shared__ float wt[kDecMaxSplit][kDecRows];
    __shared__ float linv[kDecRows];
    const int tid = threadIdx.x, ns = a.n_split;
    const size_t base = (size_t)unit * ns * kDecRows;  // slot of (split 0, row 0)
    const int nrow = min(a.rows - rb * kDecRows, kDecRows);  // valid rows of this unit
    const rsrc_t lr = make_rsrc((const char *)(a.ws_lse + base), (uint32_t)(ns * kDecRows * 4));
    const rsrc_t orr = make_rsrc((const char *)(a.ws_o + base * kD), (uint32_t)(ns * kDecRows * kD * 4));
    constexpr int kSc1 = 16;  // (CPol SC1: device scope, misses this CU's L1)
    for (int i = tid; i < ns * kDecRows; i += 256)
        wt[i / kDecRows][i % kDecRows] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(lr, 4 * i, 0, kSc1));
    __syncthreads();
    if (tid < nrow) {
        float M = kNeg, L = 0.f;
        for (int s = 0; s < ns; ++s) M = fmaxf(M, wt[s][tid]);
        for (int s = 0; s < ns; ++s) {
            const float ls = wt[s][tid];
            const float w = (ls <= 0.5f * kNeg) ? 0.f : __builtin_amdgcn_exp2f(ls - M);
            L += w;
            wt[s][tid] = w;
        }
        linv[tid] = L > 0.f ? 1.f / L : 0.f;
    }
    __syncthreads();
    constexpr int C4 = kD / 4;  // float4 chunks of a row
    const int Sq = (int)p.seqlen_q, D = (int)p.headdim;
    for (int it = tid; it < nrow * C4; it += 256) {
        const int row = it / C4, c = it % C4;
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
        for (int s = 0; s < ns; ++s) {
            const float w = wt[s][row];
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(orr, (((s * kDecRows) + row) * kD + 4 * c) * 4, 0, kSc1);
            acc.x += w * __uint_as_float(x[0]);
            acc.y += w * __uint_as_float(x[1]);
            acc.z += w * __uint_as_float(x[2]);
            acc.w += w * __uint_as_float(x[3]);
        }
        const float inv = linv[row];
        const int rg = rb * kDecRows + row;
        const int hq = hkv * a.g + rg / Sq, pos = rg % Sq;
        char *orow = (char *)p.o_ptr +
                     2 * ((int64_t)b * p.o_batch_stride + (int64_t)hq * p.o_head_stride + (int64_t)pos * p.o_seqlen_stride);
        const int d = 4 * c;
        if (kExactD || d < D) {
            const u32x2 w2 = {DT::pack(acc.x * inv, acc.y * inv), DT::pack(acc.z * inv, acc.w * inv)};
            *(u32x2 *)(orow + 2 * d) = w2;
        }
    }
}

// kFuse: the fused-merge body (a.cnt set; split launches only) -- a separate instantiation, so the
// unsplit launches keep the kernel without the merge code
template <class DT, bool kCausal, int kD, bool kExactD, bool kFuse = false>
__global__ __launch_bounds__(256, 1) void fa_decode(const fa_fwd_params p, const DecArgs a) {
    using G = Geo<kD>;
    using DG = DecGeo<kD>;
    constexpr int KS = G::kKSteps;
    constexpr int DTL = G::kDTiles;
    constexpr int RB = DG::RB;
    constexpr int NP = DG::kPieces;
    __shared__ __attribute__((aligned(1024))) char lds[DG::kLds];
    __shared__ __attribute__((aligned(1024))) char qlds[kDecRows * RB];
    __shared__ float ml[kDecWaves][kDecRows][2];
    __shared__ uint32_t last_wg;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31;
    const int h = lane >> 5;

    // ---- work: (unit = (b, hkv, rb), split) ----------------------------------------------------
    // fused merge (a.cnt): unit u's splits are the workgroups (u >> 3) * n_split + split of XCD u & 7
    // (the hardware deals workgroups to XCDs by id mod 8), so the last one reads the others' partials
    // through its own L2; the grid pads every XCD to the same count (the extra workgroups leave)
    int split, unit;
    if constexpr (kFuse) {
        const int k = (int)(blockIdx.x >> 3);
        unit = ((k / a.n_split) << 3) | (int)(blockIdx.x & 7);
        split = k % a.n_split;
        if (unit >= (int)p.batch_size * (int)p.num_heads_kv * a.n_rb) return;
    } else {
        split = blockIdx.x % a.n_split;
        unit = blockIdx.x / a.n_split;
    }
    const int rb = unit % a.n_rb;
    const int hkv = (unit / a.n_rb) % (int)p.num_heads_kv;
    const int b = unit / (a.n_rb * (int)p.num_heads_kv);
    const int Sq = (int)p.seqlen_q, D = (int)p.headdim;  // Sq: positions per q-head (row addressing)
    const float sc = p.softmax_scale;
    const float thr_raw = kRescaleThr / sc;
    // this batch row's keys: positions [k0, k0 + Sk) (a padded batch's key range, DecArgs); else
    // every key
    // (clamped to [0, seqlen_kv]: out-of-range positions never address outside the K / V rows)
    int k0 = 0, Sk = (int)p.seqlen_kv;
    if (a.k_lo) {
        const int sk_all = Sk;
        k0 = min(max(a.k_lo[b], 0), sk_all);
        Sk = min(max(a.k_hi[b], k0), sk_all) - k0;
    }
    const int diag = Sk - Sq;

    // this lane's row
    const int rg = rb * kDecRows + r;
    const bool row_ok = rg < a.rows;
    const int pos = row_ok ? rg % Sq : 0;
    const int lim = (kCausal && row_ok) ? min(Sk - 1, pos + diag) : Sk - 1;  // last visible key

    // ---- this wave's tiles: a contiguous quarter of the split --------------------------------
    const int n_tiles = (Sk + kDecKeys - 1) / kDecKeys;
    // splits of the plan's (maximum) length; with per-sequence key ranges every split takes an equal
    // share of THIS sequence's tiles instead, so a short sequence leaves no split empty and a long
    // one no split overfull
    const int tps = a.k_lo ? (n_tiles + a.n_split - 1) / a.n_split : a.tps;
    const int s_lo = min(split * tps, n_tiles), s_hi = min(s_lo + tps, n_tiles);
    const int per_wave = (s_hi - s_lo + kDecWaves - 1) / kDecWaves;
    const int t_lo = min(s_lo + wave * per_wave, s_hi), t_hi = min(t_lo + per_wave, s_hi);

    const int ks_ = (int)p.k_seqlen_stride, vs_ = (int)p.v_seqlen_stride;
    const char *kb = (const char *)p.k_ptr +
                     2 * ((int64_t)b * p.k_batch_stride + (int64_t)hkv * p.k_head_stride + (int64_t)k0 * ks_);
    const char *vb = (const char *)p.v_ptr +
                     2 * ((int64_t)b * p.v_batch_stride + (int64_t)hkv * p.v_head_stride + (int64_t)k0 * vs_);

    // ---- LDS-DMA source offsets (lane-linear destination, swizzle on the source) ---------------
    constexpr int ROWS_PER_PIECE = 1024 / RB;
    int kvo[NP], vvo[NP];
#pragma unroll
    for (int n = 0; n < NP; ++n) {
        const int row = n * ROWS_PER_PIECE + (16 * lane) / RB;
        const int slot = ((16 * lane) % RB) / 16;
        const int kch = G::k_off(row, slot) % RB / 16;
        const int vch = G::v_off(row, slot) % RB / 16;
        kvo[n] = (kExactD || kch * 8 < D) ? row * ks_ * 2 + 16 * kch : 0x7ffffff0;
        vvo[n] = (kExactD || vch * 8 < D) ? row * vs_ * 2 + 16 * vch : 0x7ffffff0;
    }
    char *ring = lds + wave * DG::kWaveLds;
    const uint32_t ring_u = lds_u32(ring);
    auto issue = [&](const int t) {
        const int key0 = t * kDecKeys;
        const int rows = min(Sk - key0, kDecKeys);
        const uint32_t dst = ring_u + (t & 1) * DG::kSlot;
        const rsrc_t kr = make_rsrc(kb + 2 * (int64_t)key0 * ks_, slab_bytes(rows, ks_, D));
        const rsrc_t vr = make_rsrc(vb + 2 * (int64_t)key0 * vs_, slab_bytes(rows, vs_, D));
        if (a.flags & kDecNt) {
#pragma unroll
            for (int n = 0; n < NP; ++n) dma_one_nt(kr, dst + n * 1024, kvo[n], n == 0);
#pragma unroll
            for (int n = 0; n < NP; ++n) dma_one_nt(vr, dst + DG::kTile + n * 1024, vvo[n], n == 0);
        } else {
#pragma unroll
            for (int n = 0; n < NP; ++n) dma_one(kr, dst + n * 1024, kvo[n], n == 0);
#pragma unroll
            for (int n = 0; n < NP; ++n) dma_one(vr, dst + DG::kTile + n * 1024, vvo[n], n == 0);
        }
    };
    // ---- Q: the row block's 32 rows by LDS-DMA into a shared K-swizzled image -----------------
    // (rows are scattered over q-heads / positions; a descriptor over the group's span bounds
    // them, invalid rows and columns past D read 0). Issued before the K/V tiles so that the
    // counted wait below retires it.
    {
        const int64_t qspan = ((int64_t)(a.g - 1) * p.q_head_stride + (int64_t)(Sq - 1) * p.q_seqlen_stride + D) * 2;
        const rsrc_t qr = make_rsrc((const char *)p.q_ptr + 2 * ((int64_t)b * p.q_batch_stride +
                                                                 (int64_t)hkv * a.g * p.q_head_stride),
                                    (uint32_t)qspan);
#pragma unroll
        for (int n = 0; n < DG::kQPiecesPerWave; ++n) {
            const int piece = wave * DG::kQPiecesPerWave + n;
            const int row = piece * ROWS_PER_PIECE + (16 * lane) / RB;
            const int slot = ((16 * lane) % RB) / 16;
            const int ch = G::k_off(row, slot) % RB / 16;
            const int rq = rb * kDecRows + row;
            const int off = (rq < a.rows && (kExactD || ch * 8 < D))
                                ? 2 * ((rq / Sq) * (int)p.q_head_stride + (rq % Sq) * (int)p.q_seqlen_stride) + 16 * ch
                                : 0x7ffffff0;
            dma_one(qr, lds_u32(qlds) + piece * 1024, off, n == 0);
        }
    }
    const bool has0 = t_lo < t_hi, has1 = t_lo + 1 < t_hi;
    if (has0) issue(t_lo);
    if (has1) issue(t_lo + 1);
    if (has1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * NP) : "memory");
    else if (has0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's Q pieces landed
    // B operand of S^T = K.Q^T: lane (h, r) holds Q[row r][16 ks + 8 h .. +7]
    u32x4 qf[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *(const u32x4 *)(qlds + G::k_off(r, 2 * ks + h));

    // ---- per-lane LDS fragment addresses (fa_fwd_w8 layouts) ----------------------------------
    const int g4 = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    int v_addr[DTL];
#pragma unroll
    for (int dt = 0; dt < DTL; ++dt)
        v_addr[dt] = G::v_off(4 * (g4 >> 1) + qq, dt * 4 + 2 * (g4 & 1) + (pp >> 1)) + 8 * (pp & 1);
    int k_addr[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) k_addr[ks] = G::k_off(r, 2 * ks + h);

    f32x16 o[DTL];
#pragma unroll
    for (int dt = 0; dt < DTL; ++dt) o[dt] = (f32x16){};
    float m_use = kNeg, msc = 0.f, l_run = 0.f;

    for (int t = t_lo; t < t_hi; ++t) {
        // tile t landed (the youngest 2*NP pieces, tile t+1, may still be in flight)
        if (t + 1 < t_hi) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NP) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const char *K = ring + (t & 1) * DG::kSlot;
        const char *V = K + DG::kTile;
        u32x4 kf[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) kf[ks] = *(const u32x4 *)(K + k_addr[ks]);
        u32x4 va[2][DTL];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int dt = 0; dt < DTL; ++dt) {
                const u32x2 lo = tr_read(V + kk * 16 * RB + v_addr[dt]);
                const u32x2 hi = tr_read(V + kk * 16 * RB + 8 * RB + v_addr[dt]);
                va[kk][dt] = (u32x4){lo[0], lo[1], hi[0], hi[1]};
            }
        // the slot is free once its fragments are in registers: refill it with tile t+2
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (t + 2 < t_hi) issue(t + 2);

        f32x16 s = {};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s = DT::mfma(kf[ks], qf[ks], s);

        const int key0 = t * kDecKeys;
        // lane (h, r) holds keys key0 + (i & 3) + 8 (i >> 2) + 4 h of row r
        if (__builtin_amdgcn_ballot_w64(key0 + kDecKeys - 1 > lim)) {
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (key0 + (i & 3) + 8 * (i >> 2) + 4 * h > lim) s[i] = kNeg;
        }
        float mx = fmaxf(s[0], s[1]);
#pragma unroll
        for (int i = 2; i < 16; ++i) mx = fmaxf(mx, s[i]);
        // both lane halves hold the same row's m_use: the check needs no cross-half reduction
        if (__builtin_amdgcn_ballot_w64(mx > m_use + thr_raw)) {
            const float m_new = fmaxf(m_use, pair_max(mx));
            const float msc_new = (m_new <= 0.5f * kNeg) ? 0.f : m_new * sc;
            // a row's first visible key: O and l are still 0, alpha must not overflow
            const float alpha = (m_use <= 0.5f * kNeg) ? 0.f : __builtin_amdgcn_exp2f(msc - msc_new);
            m_use = m_new;
            msc = msc_new;
            l_run *= alpha;
#pragma unroll
            for (int dt = 0; dt < DTL; ++dt) o[dt] *= alpha;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) s[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[i], sc, -msc));
        float ls = s[0];
#pragma unroll
        for (int i = 1; i < 16; ++i) ls += s[i];
        l_run += ls;
        u32x4 pf[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
            pf[kk] = (u32x4){DT::pack(s[8 * kk + 0], s[8 * kk + 1]), DT::pack(s[8 * kk + 2], s[8 * kk + 3]),
                             DT::pack(s[8 * kk + 4], s[8 * kk + 5]), DT::pack(s[8 * kk + 6], s[8 * kk + 7])};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int dt = 0; dt < DTL; ++dt) o[dt] = DT::mfma(va[kk][dt], pf[kk], o[dt]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- merge the 4 wave partials in LDS ------------------------------------------------------
    __syncthreads();  // every wave is done with its ring
    float *ow = (float *)lds;  // [wave][row][kD]
    {
        const float l_tot = pair_sum(l_run);
        if (h == 0) {
            ml[wave][r][0] = (m_use <= 0.5f * kNeg) ? kNeg : msc;
            ml[wave][r][1] = l_tot;
        }
#pragma unroll
        for (int dt = 0; dt < DTL; ++dt)
#pragma unroll
            for (int grp = 0; grp < 4; ++grp) {
                const int d = dt * 32 + 8 * grp + 4 * h;
                *(float4 *)(ow + (wave * kDecRows + r) * kD + d) =
                    make_float4(o[dt][4 * grp], o[dt][4 * grp + 1], o[dt][4 * grp + 2], o[dt][4 * grp + 3]);
            }
    }
    __syncthreads();

    constexpr int DPT = kD / 8;  // d values per thread: thread (row = tid / 8, part = tid % 8)
    const int row = tid >> 3, part = tid & 7;
    float M = kNeg;
#pragma unroll
    for (int w = 0; w < kDecWaves; ++w) M = fmaxf(M, ml[w][row][0]);
    float wgt[kDecWaves], L = 0.f;
#pragma unroll
    for (int w = 0; w < kDecWaves; ++w) {
        const float mw = ml[w][row][0];
        wgt[w] = (mw <= 0.5f * kNeg) ? 0.f : __builtin_amdgcn_exp2f(mw - M);
        L += wgt[w] * ml[w][row][1];
    }
    float acc[DPT];
#pragma unroll
    for (int i = 0; i < DPT; ++i) acc[i] = 0.f;
#pragma unroll
    for (int w = 0; w < kDecWaves; ++w) {
        const float *src = ow + (w * kDecRows + row) * kD + part * DPT;
#pragma unroll
        for (int i = 0; i < DPT; i += 4) {
            const float4 x = *(const float4 *)(src + i);
            acc[i] += wgt[w] * x.x;
            acc[i + 1] += wgt[w] * x.y;
            acc[i + 2] += wgt[w] * x.z;
            acc[i + 3] += wgt[w] * x.w;
        }
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
    const int rg2 = rb * kDecRows + row;
    if (a.n_split == 1) {
        if (rg2 < a.rows) {
            const int hq2 = hkv * a.g + rg2 / Sq, pos2 = rg2 % Sq;
            char *orow = (char *)p.o_ptr + 2 * ((int64_t)b * p.o_batch_stride + (int64_t)hq2 * p.o_head_stride +
                                                (int64_t)pos2 * p.o_seqlen_stride);
#pragma unroll
            for (int i = 0; i < DPT; i += 8) {
                const int d = part * DPT + i;
                if (kExactD || d < D) {
                    const u32x4 w4 = {DT::pack(acc[i] * inv, acc[i + 1] * inv), DT::pack(acc[i + 2] * inv, acc[i + 3] * inv),
                                      DT::pack(acc[i + 4] * inv, acc[i + 5] * inv),
                                      DT::pack(acc[i + 6] * inv, acc[i + 7] * inv)};
                    *(u32x4 *)(orow + 2 * d) = w4;
                }
            }
        }
    } else {
        if (rg2 < a.rows) {
            const size_t slot = ((size_t)unit * a.n_split + split) * kDecRows + row;
            float *dst = a.ws_o + slot * kD + part * DPT;
#pragma unroll
            for (int i = 0; i < DPT; i += 4)
                *(float4 *)(dst + i) = make_float4(acc[i] * inv, acc[i + 1] * inv, acc[i + 2] * inv, acc[i + 3] * inv);
            if (part == 0) a.ws_lse[slot] = L > 0.f ? M + __builtin_amdgcn_logf(L) : kNeg;  // log2
        }
        if constexpr (kFuse) {
            // fused merge: every thread's partials are in L2 before the workgroup arrives; the last
            // arrival merges the unit (the others' stores were drained before their arrivals, and
            // its loads bypass its CU's L1)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) {
                const uint32_t old = __hip_atomic_fetch_add(a.cnt + unit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last_wg = old + 1 == (uint32_t)a.n_split;
                if (last_wg) __hip_atomic_store(a.cnt + unit, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
            if (last_wg) decode_merge<DT, kD, kExactD>(p, a, unit, b, hkv, rb);
        }
    }
}

// Merge n_split partials (O / l and lse = m*s' + log2 l, log2 units): one wave per valid (q-head,
// position) row of a (batch, kv-head) -- a workgroup covers 4 of its a.rows rows, so the grid holds
// only valid rows (B * Hkv * ceil(rows / 4) workgroups) -- lane l owns d = 2l, 2l+1 (kD = 128) or
// d = l (kD = 64), so every partial row is one contiguous 512 / 256-B wave read.
template <class DT, int kD, bool kExactD>
__global__ __launch_bounds__(256) void fa_decode_combine(const fa_fwd_params p, const DecArgs a) {
    constexpr int DPL = kD / 64;  // d values per lane
    const int lane = threadIdx.x & 63;
    const int nb4 = (a.rows + 3) / 4;  // workgroups per (batch, kv-head)
    const int bh = blockIdx.x / nb4;
    const int rg = (blockIdx.x % nb4) * 4 + (threadIdx.x >> 6);  // row of the (batch, kv-head)
    if (bh >= (int)(p.batch_size * p.num_heads_kv) || rg >= a.rows) return;
    const int rb = rg / kDecRows, row = rg % kDecRows;
    const int unit = bh * a.n_rb + rb;
    const int hkv = bh % (int)p.num_heads_kv;
    const int b = bh / (int)p.num_heads_kv;
    const int Sq = (int)p.seqlen_q, D = (int)p.headdim;
    const size_t base = (size_t)unit * a.n_split * kDecRows + row;
    float M = kNeg;
    for (int s = 0; s < a.n_split; ++s) M = fmaxf(M, a.ws_lse[base + (size_t)s * kDecRows]);
    float acc[DPL], L = 0.f;
#pragma unroll
    for (int i = 0; i < DPL; ++i) acc[i] = 0.f;
    for (int s = 0; s < a.n_split; ++s) {
        const size_t slot = base + (size_t)s * kDecRows;
        const float ls = a.ws_lse[slot];
        const float w = (ls <= 0.5f * kNeg) ? 0.f : __builtin_amdgcn_exp2f(ls - M);
        L += w;
        const float *src = a.ws_o + slot * kD + lane * DPL;
        if constexpr (DPL == 2) {
            const float2 x = *(const float2 *)src;
            acc[0] += w * x.x;
            acc[1] += w * x.y;
        } else {
            acc[0] += w * src[0];
        }
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
    const int hq = hkv * a.g + rg / Sq, pos = rg % Sq;
    char *orow = (char *)p.o_ptr +
                 2 * ((int64_t)b * p.o_batch_stride + (int64_t)hq * p.o_head_stride + (int64_t)pos * p.o_seqlen_stride);
    const int d = lane * DPL;
    if (kExactD || d < D) {
        if constexpr (DPL == 2) {
            *(uint32_t *)(orow + 2 * d) = DT::pack(acc[0] * inv, acc[1] * inv);
        } else {
            const uint32_t w2 = DT::pack(acc[0] * inv, 0.f);
            *(uint16_t *)(orow + 2 * d) = (uint16_t)(w2 & 0xffff);
        }
    }
}

template <class DT, bool C, int kD, bool kExact>
int launch_decode(const fa_fwd_params &p, DecArgs a, void *ws, hipStream_t stream) {
    const int64_t units = decode_units(p, a);
    if (a.n_split > 1) {
        const int64_t slots = units * a.n_split * kDecRows;
        a.ws_o = (float *)ws;
        a.ws_lse = (float *)((char *)ws + slots * kD * 4);
    }
    // fused merge: the stream's zeroed per-unit counters (none under graph capture), and only where a
    // unit's splits share an XCD (same_xcd_placement)
    if (a.n_split > 1 && knobs().dec_fuse && same_xcd_placement()) {
        unsigned *err = nullptr;
        a.cnt = split_sync_area(stream, units * 4, &err);
    }
    set_last_dec_fused(a.cnt != nullptr);
    // (fused: every XCD holds ceil(units / 8) units' splits)
    const int64_t grid = a.cnt ? 8 * ((units + 7) / 8) * a.n_split : units * a.n_split;
    if (a.cnt)
        hipLaunchKernelGGL((fa_decode<DT, C, kD, kExact, true>), dim3((uint32_t)grid), dim3(256), 0, stream, p, a);
    else
        hipLaunchKernelGGL((fa_decode<DT, C, kD, kExact>), dim3((uint32_t)grid), dim3(256), 0, stream, p, a);
    if (a.n_split > 1 && !a.cnt)
        hipLaunchKernelGGL((fa_decode_combine<DT, kD, kExact>),
                           dim3((uint32_t)(p.batch_size * p.num_heads_kv * ((a.rows + 3) / 4))), dim3(256), 0, stream,
                           p, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(FA_ERR_LAUNCH, "HIP launch failed: %s", hipGetErrorString(e));
    set_last_path(a.n_split > 1 ? kPathDecodeSplit : kPathDecode);
    return FA_OK;
}

}  // namespace fa
