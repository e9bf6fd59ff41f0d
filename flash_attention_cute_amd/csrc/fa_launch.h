// fa_launch.h -- internal seam between the C-ABI dispatcher (fa_fwd_gfx950.hip) and the kernel
// instantiations (fa_inst.hip x 16, one translation unit per combination so they compile in
// parallel). Not part of the public boundary; include/fa_gfx950.h is.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "fa_gfx950.h"

namespace fa {

constexpr int kBlockM = 256;  // query rows per workgroup
constexpr int kBlockN = 64;   // keys per KV tile
// rows one wave's Q / O (and RoPE table) slab spans in fa_fwd_w4: block A's 32 rows, block B's
// 32 rows kBlockM / 2 rows later; the host bounds q / o / RoPE seqlen strides so that a slab's
// byte offsets fit 32 bits (check_params)
constexpr int kQoSpanRows = kBlockM / 2 + 32;
constexpr int kWaves = 8;     // fa_fwd_w8
constexpr int kThreads = kWaves * 64;

struct F16;
struct BF16;

// records a message for fa_last_error() and returns `code`
int set_err(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

// Tuning / debug knobs. The product dispatcher never reads the environment per launch: the values
// are taken ONCE, from the environment of the process at the first launch (A/B scripts set them on
// the command line), and can be changed afterwards only through fa_debug_set_knobs (tests).
//   variant    0 = fa_fwd_w4 (default); 1 = fa_fwd_w8 (FA_GFX950_VARIANT=w8: the 8-wave
//              register-staged kernel, A/B and cross-check); 2 = w4 without its pipelined body
//              (FA_GFX950_VARIANT=w4slow, debug); 3 = fa_fwd_p8 (FA_GFX950_VARIANT=p8: two waves per
//              SIMD, dense prefill; varlen / RoPE stay on fa_fwd_w4); 4 / 5 = fa_fwd_mb with the
//              32x32x16 / 16x16x32 MFMA (FA_GFX950_VARIANT=m32 / m16: the shape A/B body, dense
//              prefill only, fa_fwd_mb.hpp)
//   w4_grid    cap of the persistent fa_fwd_w4 grid (FA_W4_GRID; 0 = the CU count)
//   decode     split-KV decode kernel for few rows per kv-head (FA_GFX950_DECODE=0 turns it off)
//   dec_target workgroups the decode split plan aims at (FA_DEC_TARGET_WGS)
//   dec_flags  kDec* bits of the decode kernel (FA_DEC_FLAGS)
//   zigzag     causal Q-block layout: 1 = zigzag when the blocks fit one round of the persistent
//              grid (default), 0 = never, 2 = always where it applies (FA_ZIGZAG; tests)
struct Knobs {
    int variant;
    int64_t w4_grid;
    int decode;
    int64_t dec_target;
    int dec_flags;
    int zigzag;
    int split;  // key-split causal Q blocks (use_split): 0 never, 1 where measured faster (default), 2 always
    int split_pairs;  // key-split pairs (use_split_pairs): 0 never, 1 where they fit one pass (default)
    int dec_fuse;     // split-KV decode: 1 the last split of a unit merges (default), 0 fa_decode_combine
    int xccs;         // XCDs per device for the placement check (0: the device's own count; tests)
    int head_pack;    // head-packed causal GQA blocks (use_head_pack): 0 never, 1 the rule (default), 2 always
    int split_fault;  // (debug library only) force one key-split hand-off to time out (kernel dbg & 2)
    int split_rr;     // key-split halves' order: 0 XCD-contiguous decode_work ranges, 1 level-major (default)
};

const Knobs &knobs();
inline int variant_from_env() { return knobs().variant; }

// Which kernel the last fa_fwd_gfx950* call on this thread launched (fa_debug_last_path)
enum Path { kPathNone = 0, kPathW4 = 1, kPathW8 = 2, kPathW4Slow = 3, kPathDecode = 4, kPathDecodeSplit = 5, kPathP8 = 6,
            kPathM32 = 7, kPathM16 = 8 };
void set_last_path(int path);
void set_last_zigzag(int z);
void set_last_dec_fused(bool fused);  // (fa_debug_last_dec_fused: the last decode launch merged in-kernel)

// diagnostic per-wave phase stamps of fa_fwd_w4 (only a -DFA_STAMPS=1 build writes them; see
// fa_debug_set_stamps in fa_fwd_gfx950.hip and scripts/stamps.py); nullptr otherwise
unsigned long long *stamp_buffer();

// workgroups of a persistent fa_fwd_w4 launch over nwg Q blocks: nwg if it fits the cap (the CU
// count of the current device), else the cap rounded down to a multiple of 8, at least 8 (the kernel
// deals Q blocks to workgroups by bid mod 8). FA_W4_GRID=<n> overrides the cap (A/B runs, tests).
int64_t w4_grid(int64_t nwg);
// compute units of the current device (queried once per device)
int64_t device_cus();
// XCDs (XCCs) of the current device (queried once per device; the xccs knob overrides it)
int64_t device_xccs();
// Whether workgroups b and b + 8 of a launch share an XCD, the placement that the key-split hand-off
// and the fused decode merge rely on (their sc1 records meet in that XCD's L2, no L2 write-back or
// invalidate). The hardware deals a launch's workgroups to the XCDs round-robin by workgroup id
// (MI355X_MICROARCH "Workgroup dispatch"), so this holds when the XCD count divides 8: 8 (SPX, 256
// CUs), 4 (DPX), 2, 1 (CPX). Otherwise the dispatcher runs the layouts that need no hand-off (zigzag
// prefill, the separate decode combine launch).
inline bool same_xcd_placement() {
    const int64_t x = device_xccs();
    return x >= 1 && 8 % x == 0;
}



// Optional parts of a prefill launch.
// RoPE tables for the Q load (fa_fwd_gfx950_rope): cos / sin [.., Sq, D] of the q dtype, strides in
// elements (row of query m of batch b: b * batch_stride + m * seq_stride; varlen: packed row *
// seq_stride). cos == nullptr: no rotation.
// Local window (fa_fwd_gfx950_window): key n is visible to query m only if n >= m + Sk - Sq -
// window_left (the sliding window of window_left + 1 keys ending at the bottom-right diagonal);
// window_left < 0: none.
// Per-sequence ranges (device int32 arrays, or nullptr = the whole dimension): batch row b's query
// rows are [q_rng[b], q_rng[b + rng_hi]) and its keys [k_rng[b], k_rng[b + rng_hi]), ABSOLUTE rows
// (row r at base + r * seqlen stride; the host zeroes the batch strides of ranged tensors); query
// ranges come with key ranges. Packed varlen passes cu_seqlens with rng_hi = 1
// (fa_fwd_gfx950_varlen); padded batches [2, B] arrays of starts then ends with rng_hi = B
// (fa_fwd_gfx950_padded). Masks are bottom-right aligned per sequence.
// k_lo / k_hi (decode kernel only, fa_fwd_gfx950_padded): key POSITIONS [k_lo[b], k_hi[b]) within
// batch row b (its batch strides apply), or nullptr.
// zigzag (set by launch_one, never by the dispatchers): causal Q blocks pair the 128-row segments t
// and nseg - 1 - t (fa_fwd_w4 "Zigzag Q blocks"), for dense causal launches that fit one round.
// split_ws (set by the dispatcher when the caller passed a workspace, use_split): every causal Q
// block runs as two pieces over the two halves of its key tiles, on two workgroups; the piece that
// finishes first leaves its unnormalised O and row statistics in split_ws, the second combines
// them with its own and stores O (fa_fwd_w4 "Key-split causal blocks"). split_sync: per (block,
// wave) [arrivals + 4 once the first piece's records are ready, unused] words, zero at the launch;
// the combining piece zeroes its pair again
// (split_sync_area). split_err: the device's count of hand-offs that timed out (or nullptr).
// split_pairs (set by launch_one, use_split_pairs): the pieces are laid out as pairs of a heavy
// and a light q-tile on two workgroups (fa_fwd_w4 "key-split blocks").
struct PathArgs {
    const void *cos;
    const void *sin;
    int64_t batch_stride;
    int64_t seq_stride;
    int window_left;
    int rng_hi;
    const int *q_rng, *k_rng;
    const int *k_lo, *k_hi;
    int zigzag;
    float *split_ws;
    unsigned *split_sync;
    unsigned *split_err;
    int split_pairs;
    int head_pack;  // (set by launch_one, use_head_pack) head-packed causal blocks (fa_fwd_w4)
    int split_rr;   // (set by launch_one, knob split_rr) the halves' units level-major over the XCDs
};

// Whether a prefill launch runs zigzag Q blocks, and its logical q-tile count (blocks per (batch,
// q-head)): causal, dense (no per-sequence ranges, window or RoPE), more than one 128-row segment,
// the plain blocks fitting one round of the grid (knob 1) or always (knob 2), and the wave's Q / O
// slab (block B up to Sq rows past block A) inside 32-bit byte offsets.
inline bool use_zigzag(const fa_fwd_params &p, bool causal, const PathArgs &xa) {
    if (!causal || xa.k_rng || xa.cos || xa.window_left >= 0 || knobs().zigzag == 0 || p.seqlen_q <= 128) return false;
    const int64_t big = p.q_seqlen_stride > p.o_seqlen_stride ? p.q_seqlen_stride : p.o_seqlen_stride;
    if (big * 2 * (p.seqlen_q + 32) + 256 > 0x7fffffffLL) return false;
    const int64_t nwg = (p.seqlen_q + kBlockM - 1) / kBlockM * p.num_heads_q * p.batch_size;
    return knobs().zigzag == 2 || nwg <= device_cus();
}
inline int64_t zigzag_qtiles(int64_t seqlen_q) { return ((seqlen_q + 127) / 128 + 1) / 2; }

// Head-packed causal blocks (fa_fwd_w4 "Head-packed blocks"): causal GQA with a multiple of 4 q-heads
// per kv-head (4 consecutive q-heads of one kv group per block, one per wave: Llama-3-8B's g = 4 --
// C4, C5 -- or Llama-3-70B's g = 8 as two quads), more than one 64-row q-tile, when neither zigzag nor
// key-split takes the launch (multi-round grids, and one-round grids more than half full). Dense,
// fused-RoPE (the patched Llama layer),
// per-sequence-range (varlen, padded) and local-window launches. A block is (batch, q-head quad,
// 64 rows): its causal diagonal is one tile instead of the plain 256-row block's four, two of them
// A-dead (and a window's left edge spans 64 rows' keys, not 256); bit-identical to the plain layout. Knob head_pack (env FA_HEAD_PACK): 0 never, 1 by this
// rule (default), 2 whenever it applies (also one-round grids, tests).
inline bool use_head_pack(const fa_fwd_params &p, bool causal, const PathArgs &xa) {
    if (!causal || knobs().head_pack == 0) return false;
    if (p.head_q_per_group % 4 != 0 || p.seqlen_q <= 64) return false;
    if (knobs().head_pack == 2) return true;
    if (knobs().zigzag == 2 && use_zigzag(p, causal, xa)) return false;  // (a forced zigzag wins over the rule)
    // multi-round grids, and one-round grids more than half full that key-split did not take (short keys):
    // there head-packed blocks measured +4 to +6 % over zigzag (B4 Hq32 S512, B8 Hq32 S256) and tied at
    // 192 blocks; at half fill or less zigzag ties or wins (profiles/r6_ab_headpack_short.log)
    const int64_t nwg = (p.seqlen_q + kBlockM - 1) / kBlockM * p.num_heads_q * p.batch_size;
    return 2 * nwg > device_cus();
}

// Head-packed key-split pieces (fa_fwd_w4 "Head-packed blocks" + "key-split blocks"): a key-split
// launch (one-round grid, use_split) with a multiple of 4 q-heads per kv-head can run its pieces over
// (batch, q-head quad, 64-row q-tile) blocks -- the halves or pairs layout over those units, the same
// hand-off per (block, wave) (each wave one q-head's 64 rows, as a plain block's wave) -- so a piece's
// diagonal is one tile. Whether it may (launch_one decides): knob head_pack 1 (default) only under the
// pairs layout (measured +0.8 to +7 % over plain-block pairs; under the halves it lost 1.5-14 %,
// profiles/r6_split_rule_sweep.log), 2 under both, 0 never.
inline bool use_head_pack_split(const fa_fwd_params &p, bool causal, const PathArgs &xa) {
    return causal && !xa.k_rng && !xa.cos && xa.window_left < 0 && knobs().head_pack != 0 &&
           p.head_q_per_group % 4 == 0 && p.seqlen_q > 64;
}

// Key-split causal blocks: dense causal launches (no varlen, window or RoPE) when the caller passes
// the workspace. Knob 1 (default): where measured faster than zigzag (same-process A/B over one-round
// grids, profiles/r6_split_rule_sweep.log; round 4's rule, before the pairs layout, was 3072 / 2048
// keys): the plain blocks fit one round of the grid and the keys are long enough for each piece to
// carry its extra block start and combine -- at least 2048 keys (more than half the CUs: the pairs
// layout, +10 to +16 % at 2048; at 1024 MHA lost 8 %), or 1024 when the blocks fill at most half
// the CUs (the halves, +6 to +14 % at 1024; at 512-768 zigzag ties or wins). Knob 2: always (tests). Workspace: the per-(block, wave) sync counters, then per (block,
// wave) the partial O of its 64 rows (32 * DTL fp32 per lane) and two 16-byte statistic records per lane.
inline bool use_split(const fa_fwd_params &p, bool causal, const PathArgs &xa) {
    if (!causal || xa.k_rng || xa.cos || xa.window_left >= 0 || knobs().split == 0 || p.seqlen_q <= 128) return false;
    if (!same_xcd_placement()) return false;  // (the pieces' hand-off needs one XCD per pair)
    if (knobs().split == 2) return true;
    const int64_t nwg = (p.seqlen_q + kBlockM - 1) / kBlockM * p.num_heads_q * p.batch_size, cus = device_cus();
    return nwg <= cus && (p.seqlen_kv >= 2048 || (p.seqlen_kv >= 1024 && 2 * nwg <= cus));
}
constexpr int kSplitStatsPerLane = 8;  // floats: (nmsc, l) of blocks A and B, then (m_A, m_B, 0, 0)
inline int64_t split_wave_floats(int64_t headdim) {
    return 64 * ((headdim <= 64 ? 2 : 4) * 32 + kSplitStatsPerLane);  // 64 lanes x (2 blocks x DTL x 16 + stats)
}
// Key-split pairs (fa_fwd_w4 "key-split blocks"): when the split's two pieces per block would need a
// second round of the grid (more plain blocks than half the CUs), lay them out as pairs instead --
// the heavy q-tile Q - 1 - p split between two workgroups, one of which then also runs the light
// q-tile p whole -- one pass, two workgroups per pair, so the grid must hold 2 x ceil(pairs / 8) per
// XCD. Knob split_pairs (env FA_SPLIT_PAIRS): 0 never, 1 where this holds (default).
#ifndef FA_SPLIT_PAIRS
#define FA_SPLIT_PAIRS 1
#endif
#ifndef FA_HEAD_PACK  // default of Knobs::head_pack
#define FA_HEAD_PACK 1
#endif
#ifndef FA_SPLIT_RR  // default of Knobs::split_rr (level-major halves: +1.7 to +4.6 %, r6_ab_split_halves_order.log)
#define FA_SPLIT_RR 1
#endif
#ifndef FA_DEC_FUSE  // default of Knobs::dec_fuse
#define FA_DEC_FUSE 1
#endif
// workgroups of a key-split launch over `units` plain blocks (2 pieces each) or pairs: every XCD gets
// two workgroups per unit of its list when that fits the grid cap (units are dealt to XCDs, so 2 *
// units workgroups could leave some XCD short and run both pieces of a block on one workgroup)
int64_t w4_grid_split(int64_t units);
// blocks: the launch's unsplit Q blocks (q-tiles x rows of the work order); rows: its (batch, q-head)
// or, head-packed, (batch, q-head quad) rows
inline bool use_split_pairs(int64_t blocks, int64_t rows, int64_t cus) {
    if (knobs().split_pairs == 0) return false;
    const int64_t nq = blocks / rows, units = (nq + 1) / 2 * rows;
    return 2 * blocks > cus && w4_grid_split(units) == 16 * ((units + 7) / 8);
}
inline int64_t split_blocks(const fa_fwd_params &p) {
    return (p.seqlen_q + kBlockM - 1) / kBlockM * p.num_heads_q * p.batch_size;
}
inline int64_t split_sync_bytes(const fa_fwd_params &p) { return (split_blocks(p) * 4 * 2 * 4 + 255) / 256 * 256; }
inline int64_t split_ws_bytes(const fa_fwd_params &p) {
    return split_sync_bytes(p) + split_blocks(p) * 4 * split_wave_floats(p.headdim) * 4;
}

// The key-split / fused-decode counters of eager launches on `stream` of the current device: a device
// area allocated once per (device, stream) and zeroed by a memset on that stream (stream-ordered, no
// device synchronisation; the kernels leave it zeroed), or nullptr when `bytes` exceed it or the stream
// is capturing a graph -- a graph never holds the shared area (its replays could run beside eager
// launches on the stream), the caller then zeroes counters in its workspace (a memset node) or runs the
// separate decode combine. *err: the stream's hand-off error counter (under capture: the capturing
// stream's, if it has an area; else nullptr).
unsigned *split_sync_area(hipStream_t stream, int64_t bytes, unsigned **err);

// launch one (dtype, causal, head-dim tile, exact head dim) instantiation on `stream`
template <class DT, bool C, int kD, bool kExact>
int launch_one(const fa_fwd_params &p, const PathArgs &xa, hipStream_t stream);


// ---- split-KV decode (fa_decode.hpp) -------------------------------------------------------------
constexpr int kDecRows = 32;  // query rows per row block (one 32x32 MFMA column block)
constexpr int kDecKeys = 32;  // keys per tile
constexpr int kDecWaves = 4;  // waves per workgroup, each on its own contiguous key range
// decode kernel when a (batch, kv-head) has at most this many (q-head, position) rows
constexpr int kDecMaxRows = 2 * kDecRows;
// split plan: about kDecTargetWgs workgroups (the 128 KiB LDS ring admits one per CU), every wave
// at least kDecMinTilesPerWave tiles. Fewer, longer splits than one per CU measured faster (B1 Hkv8
// Sk131072 bf16: 5.2-5.5 TB/s at 160-192 workgroups vs 4.9-5.0 at 256, same run)
constexpr int kDecTargetWgs = 160;
constexpr int kDecMinTilesPerWave = 4;
constexpr int kDecMaxSplit = 64;

struct DecArgs {
    int g;          // q-heads per kv-head
    int rows;       // g * Sq: (q-head, position) rows of one (batch, kv-head)
    int n_rb;       // 32-row blocks per (batch, kv-head)
    int n_split;    // key splits (workgroups per row block)
    int tps;        // 32-key tiles per split
    float *ws_o;    // [units * n_split][32][kD] fp32 partial O / l    (n_split > 1)
    float *ws_lse;  // [units * n_split][32] fp32 m * s' + log2(l)      (n_split > 1)
    int flags;      // kDec* bits
    // per-sequence key positions [k_lo[b], k_hi[b]) within batch row b (a padded batch), or nullptr
    // (every key). Query ranges are not supported here (the dispatcher sends them to fa_fwd_w4).
    const int *k_lo, *k_hi;
    // (n_split > 1) per-unit arrival counters, zero at the launch (the stream's persistent
    // split_sync_area): the last split of a unit to finish merges the partials itself -- the unit's
    // splits then run on ONE XCD (fa_decode "fused merge"; the partials are published by stores drained
    // before a relaxed agent-scope add, with no release / acquire fence, which is enough ONLY inside one
    // XCD's L2: the host checks same_xcd_placement) -- and re-zeroes its counter; nullptr: the separate
    // fa_decode_combine launch merges them
    unsigned *cnt;
};
constexpr int kDecNt = 1;  // K/V LDS-DMA with the non-temporal cache policy

inline int64_t decode_units(const fa_fwd_params &p, const DecArgs &a) {
    return p.batch_size * p.num_heads_kv * a.n_rb;
}

inline DecArgs decode_plan(const fa_fwd_params &p, int max_split) {
    DecArgs a{};
    a.g = (int)p.head_q_per_group;
    a.rows = (int)(p.head_q_per_group * p.seqlen_q);
    a.n_rb = (a.rows + kDecRows - 1) / kDecRows;
    const int64_t units = decode_units(p, a);
    const int n_tiles = (int)((p.seqlen_kv + kDecKeys - 1) / kDecKeys);
    const int64_t target = knobs().dec_target;
    a.flags = knobs().dec_flags;
    int64_t ns = (target + units - 1) / units;
    const int64_t by_len = n_tiles / (kDecWaves * kDecMinTilesPerWave);
    ns = ns < by_len ? ns : by_len;
    ns = ns < max_split ? ns : max_split;
    ns = ns < 1 ? 1 : ns;
    a.tps = (int)((n_tiles + ns - 1) / ns);
    a.n_split = (n_tiles + a.tps - 1) / a.tps;
    return a;
}

// workspace bytes of a plan (fp32 partials + lse); 0 when it does not split
inline int64_t decode_ws_bytes(const fa_fwd_params &p, const DecArgs &a) {
    if (a.n_split <= 1) return 0;
    const int64_t slots = decode_units(p, a) * a.n_split * kDecRows;
    const int64_t dpad = p.headdim <= 64 ? 64 : 128;
    return slots * dpad * 4 + slots * 4;
}

// launch the decode kernel (+ the split combine when a.n_split > 1) of one instantiation
template <class DT, bool C, int kD, bool kExact>
int launch_decode(const fa_fwd_params &p, DecArgs a, void *ws, hipStream_t stream);

#define FA_FOR_EACH_INSTANCE(X)                                                                    \
    X(F16, false, 64, false) X(F16, false, 64, true) X(F16, false, 128, false) X(F16, false, 128, true) \
    X(F16, true, 64, false) X(F16, true, 64, true) X(F16, true, 128, false) X(F16, true, 128, true)     \
    X(BF16, false, 64, false) X(BF16, false, 64, true) X(BF16, false, 128, false)                      \
    X(BF16, false, 128, true) X(BF16, true, 64, false) X(BF16, true, 64, true)                         \
    X(BF16, true, 128, false) X(BF16, true, 128, true)

#define FA_DECLARE_EXTERN(DT, C, D, E)                                                  \
    extern template int launch_one<DT, C, D, E>(const fa_fwd_params &, const PathArgs &, hipStream_t);            \
    extern template int launch_decode<DT, C, D, E>(const fa_fwd_params &, DecArgs, void *, hipStream_t);
FA_FOR_EACH_INSTANCE(FA_DECLARE_EXTERN)
#undef FA_DECLARE_EXTERN

}  // namespace fa
