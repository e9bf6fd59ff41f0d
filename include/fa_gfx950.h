/*
 * fa_gfx950.h -- C-ABI boundary of the MI355X (gfx950 / CDNA4) FlashAttention-2
 * forward operator.
 *
 * This header is the drop-in seam that replaces the reference's C++ template
 * entry point and its parameter struct:
 *
 *   reference csrc/flash_attention.h:5-37   struct FlashAttentionParams
 *   reference csrc/flash_attention.h:39-41  template<T,kHeaddim,IsCausal>
 *                                           void run_flash_attention(Params&, cudaStream_t)
 *   reference csrc/kernel_dispatcher.h:20-52 dtype / headdim / causal dispatch
 *
 * The reference dispatches at compile time through three nested lambdas and
 * reaches the kernel through a C++ template; here the whole dispatch is one
 * plain C function taking the same parameters by pointer plus two runtime
 * enums, so it can be bound from ctypes / cgo / JNI without C++ name mangling
 * or torch types.
 *
 * Conventions (identical to the reference's FlashAttentionParams):
 *   - q [B, Hq, Sq, D], k/v [B, Hkv, Sk, D], o [B, Hq, Sq, D]; the last
 *     dimension is contiguous (stride 1), every other stride is given in
 *     ELEMENTS, not bytes;
 *   - softmax_scale is ALREADY multiplied by log2(e) (reference
 *     csrc/flash_attention_api.cpp:87), the kernel evaluates exp2;
 *   - head_q_per_group = Hq / Hkv; q-head h reads kv-head h / head_q_per_group
 *     (reference csrc/flash_attention_template.cuh:157-160);
 *   - causal masking is bottom-right aligned: key n is visible to query m iff
 *     n <= m + (Sk - Sq) (reference csrc/mask.cuh:37-39).
 *   - base pointers must be 16-byte aligned and D % 8 == 0 (every row chunk is
 *     a 16-byte vector), D <= 128.
 *
 * Return values: FA_OK (0) on success, a positive FA_ERR_* code otherwise;
 * fa_last_error() returns a human-readable message for the calling thread.
 * The reference kills the process on a CUDA error (csrc/utils.h:9-18); this
 * ABI reports it instead, and the torch binding turns it into a RuntimeError.
 */
#ifndef FA_GFX950_H
#define FA_GFX950_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 7: fa_fwd_gfx950_ws takes the key-split layout only when the workspace is large enough (a smaller one
 *    runs the zigzag layout instead of failing), its counters live in a per-(device, stream) area the
 *    library keeps zeroed (no per-call memset), and fa_split_errors() reports failed hand-offs.
 * 8: the per-stream area is zeroed by a memset on the launching stream (no device-wide
 *    synchronisation on a stream's first call), graph captures never use it (workspace counters), a
 *    timed-out hand-off leaves it zeroed, the error count is kept per stream (fa_split_errors sums the
 *    device's), and key-split / the fused decode merge run only where workgroups b and b + 8 share an
 *    XCD (the XCD count divides 8). */
#define FA_GFX950_ABI_VERSION 8

/* Field order mirrors reference csrc/flash_attention.h:5-37. */
typedef struct fa_fwd_params {
    const void *q_ptr;
    const void *k_ptr;
    const void *v_ptr;
    void *o_ptr;

    int64_t batch_size;
    int64_t num_heads_q;
    int64_t num_heads_kv;
    int64_t seqlen_q;
    int64_t seqlen_kv;
    int64_t headdim;

    int64_t head_q_per_group;

    int64_t q_batch_stride;
    int64_t k_batch_stride;
    int64_t v_batch_stride;
    int64_t o_batch_stride;

    int64_t q_head_stride;
    int64_t k_head_stride;
    int64_t v_head_stride;
    int64_t o_head_stride;

    int64_t q_seqlen_stride;
    int64_t k_seqlen_stride;
    int64_t v_seqlen_stride;
    int64_t o_seqlen_stride;

    float softmax_scale; /* scale * log2(e) */
} fa_fwd_params;

/* dtype codes (reference csrc/kernel_dispatcher.h:20-34: kHalf, kBFloat16) */
enum { FA_DTYPE_F16 = 0, FA_DTYPE_BF16 = 1 };

enum {
    FA_OK = 0,
    FA_ERR_INVALID_ARGUMENT = 1, /* shape / stride / alignment violation */
    FA_ERR_UNSUPPORTED = 2,      /* dtype or headdim with no kernel */
    FA_ERR_LAUNCH = 3,           /* HIP runtime error at launch */
};

/*
 * Launch the forward kernel on `stream` (a hipStream_t; NULL = default
 * stream). Asynchronous: no host synchronisation, no allocation, no global
 * state, safe under hipGraph capture.
 * Replaces run_flash_attention<T,128,IsCausal> (reference
 * csrc/flash_attention_impl.cu:30-49) together with the dispatch of
 * csrc/kernel_dispatcher.h:20-52.
 */
int fa_fwd_gfx950(const fa_fwd_params *params, int dtype, int causal, void *stream);

/*
 * Workspace variant. Few query rows per kv-head (the Sq == 1 q-head pack of
 * reference csrc/flash_attention_api.cpp:72-83, or head_q_per_group * Sq <=
 * 64) run a split-KV decode kernel; splitting the keys over more workgroups
 * needs `workspace_bytes` >= fa_fwd_gfx950_workspace_size() of device memory
 * for fp32 partials. A causal prefill whose 256-row blocks fit one round of the
 * persistent grid (at most one block per CU: a single long sequence, one GPU's
 * share of a multi-GPU split) with at least 2048 keys (1024 when the blocks fill
 * at most half the CUs) splits each block's keys in two pieces on two
 * workgroups instead, when the workspace holds at least
 * fa_fwd_gfx950_workspace_size() bytes (else the blocks run unsplit, in zigzag
 * order); the workspace then holds the first piece's fp32 partial O. The pieces'
 * per-block counters live in a device area the library allocates once per
 * (device, stream) on the first such eager call on that stream (hipMalloc, then
 * a memset enqueued on `stream`: no device synchronisation) and the kernel
 * leaves zeroed; under graph capture the counters go to the workspace instead,
 * zeroed by a memset node this call adds on `stream`. The split layouts need
 * workgroups b and b + 8 of a launch on one XCD (the device's XCD count divides
 * 8, MI355X deals workgroups to XCDs round-robin); elsewhere the blocks run
 * unsplit. With workspace == NULL it behaves exactly like
 * fa_fwd_gfx950 (decode kernel unsplit, causal prefill in zigzag blocks). The
 * workspace is scratch: it may be reused as soon as the launch completes in
 * stream order. 16-byte aligned.
 * No reference counterpart (split-KV is a TODO at reference README.md:20).
 */
int fa_fwd_gfx950_ws(const fa_fwd_params *params, int dtype, int causal, void *workspace,
                     int64_t workspace_bytes, void *stream);

/*
 * Bytes of workspace fa_fwd_gfx950_ws wants for these parameters (0 when the
 * launch does not split; -1 when the parameters are invalid). Host-only (it
 * queries the current device's CU count for the causal-prefill split).
 */
int64_t fa_fwd_gfx950_workspace_size(const fa_fwd_params *params, int dtype, int causal);

/*
 * Validate `params` exactly as fa_fwd_gfx950 does, without touching the
 * device. Returns FA_OK or the error code fa_fwd_gfx950 would return.
 */
int fa_fwd_gfx950_check(const fa_fwd_params *params, int dtype, int causal);

/*
 * Key-split hand-offs on the current device that timed out (a piece whose partner's
 * partial result did not arrive within ~1 s combined what was there: its rows are
 * wrong; the pair is abandoned, so later launches are unaffected), summed over the
 * device's streams and launches since the last reset; 0 when none. Synchronises
 * with the device. reset != 0 zeroes the count.
 */
int64_t fa_split_errors(int reset);

/* Message for the last non-OK return on this thread ("" if none). */
const char *fa_last_error(void);

/* FA_GFX950_ABI_VERSION of the loaded library. */
int fa_abi_version(void);

/*
 * Tile geometry of the kernel that fa_fwd_gfx950 would launch for these
 * parameters: rows of q per work unit, keys per KV tile, threads per
 * workgroup and number of work units (Q blocks; decode: row blocks x key
 * splits). The prefill kernel is persistent: it launches min(units, CUs)
 * workgroups that walk the units (FA_W4_GRID overrides the cap). Host-only
 * (touches no device), for schedulers and tests.
 */
int fa_fwd_gfx950_geometry(const fa_fwd_params *params, int causal, int64_t *block_m,
                           int64_t *block_n, int64_t *threads, int64_t *workgroups);

/*
 * Variable-length (packed) batches. No reference counterpart: varlen is a TODO at reference
 * README.md:18, and the reference's vendored models reject any attention_mask
 * (models/modeling_llama.py:296-297); this is the entry a padding mask is lowered to.
 *
 * The B sequences are packed along the row dimension: q [total_q, Hq, D], k/v [total_k, Hkv, D],
 * o [total_q, Hq, D] (any row / head strides, multiples of 8 elements; last dim contiguous).
 * Sequence b owns q rows [cu_seqlens_q[b], cu_seqlens_q[b+1]) and k/v rows
 * [cu_seqlens_k[b], cu_seqlens_k[b+1]) -- int32 prefix sums in DEVICE memory, B + 1 entries.
 * In `base`: batch_size = B; seqlen_q / seqlen_kv = upper bounds of the per-sequence lengths
 * (seqlen_q sizes the grid: a longer sequence would be cut short, so it must be at least the true
 * maximum; a larger bound only launches empty q-tiles);
 * the *_batch_stride fields are ignored; the head / seqlen strides are those of the packed tensors.
 * Causal masking is bottom-right aligned per sequence (key n visible to query m iff
 * n <= m + Sk_b - Sq_b), rows of a sequence with no visible key are 0, a sequence with Sk_b == 0
 * gives 0 rows. The prefill kernel serves every sequence (no split-KV decode path).
 */
typedef struct fa_varlen_params {
    fa_fwd_params base;
    const int32_t *cu_seqlens_q; /* [B + 1], device */
    const int32_t *cu_seqlens_k; /* [B + 1], device */
} fa_varlen_params;

int fa_fwd_gfx950_varlen(const fa_varlen_params *params, int dtype, int causal, void *stream);

/* The varlen forward with the local window of fa_fwd_gfx950_window applied per sequence (key n of
 * sequence b visible to its query m only if n >= m + Sk_b - Sq_b - window_left; < 0: none). */
int fa_fwd_gfx950_varlen_window(const fa_varlen_params *params, int dtype, int causal, int64_t window_left,
                                void *stream);

/* Host-only validation of the varlen parameters (the device arrays are not read). */
int fa_fwd_gfx950_varlen_check(const fa_varlen_params *params, int dtype, int causal);

/*
 * Padded batches: per-sequence query / key ranges inside DENSE tensors (the layout of an HF
 * padded batch and its KV cache, read in place -- no packing copy). No reference counterpart
 * (the reference drops attention_mask, models/rope_attn_fwd.py:40-64); this is the entry an HF
 * left- or right-padding mask is lowered to.
 *
 * `base` describes dense q [B, Hq, Sq, D], k/v [B, Hkv, Sk, D], o [B, Hq, Sq, D] exactly as for
 * fa_fwd_gfx950 (seqlen_q / seqlen_kv = the padded lengths). Batch row b's real keys are positions
 * [k_start[b], k_end[b]) of its Sk and its real queries positions [q_start[b], q_end[b]) of its Sq --
 * int32 arrays of B entries in DEVICE memory; q_start == q_end == NULL means every query row,
 * k_start == k_end == NULL every key. The kernels clamp every range to its dimension (start into
 * [0, Sq] / [0, Sk], end into [start, Sq] / [start, Sk]) on the device, so an out-of-range position
 * never reads or writes outside the tensors. Masks are bottom-right aligned per sequence (key n of the
 * range visible to query m of the range iff n - k_start <= m - q_start + Sk_b - Sq_b);
 * window_left >= 0 adds the local window of fa_fwd_gfx950_window per sequence (< 0: none). Output
 * rows outside the query ranges are NOT written (the torch binding zero-fills them first); rows with
 * no visible key are 0.
 * Few query rows per kv-head without query ranges or window (Sq == 1 after the q-head pack, or
 * head_q_per_group * Sq <= 64) run the split-KV decode kernel on each sequence's key positions;
 * everything else runs the prefill kernel, whose launch first converts the positions into row
 * arrays in the workspace (this needs each tensor's batch stride to be a multiple of its seqlen
 * stride, the same multiple for q and o, and for k and v). fa_fwd_gfx950_padded_workspace_size()
 * gives the bytes either path wants (decode: split-KV partials, NULL = unsplit; prefill: required).
 * Asynchronous, no host synchronisation: safe under hipGraph capture.
 */
typedef struct fa_padded_params {
    fa_fwd_params base;
    const int32_t *q_start; /* [B], device, or NULL */
    const int32_t *q_end;   /* [B], device, or NULL */
    const int32_t *k_start; /* [B], device, or NULL */
    const int32_t *k_end;   /* [B], device, or NULL */
} fa_padded_params;

int fa_fwd_gfx950_padded(const fa_padded_params *params, int dtype, int causal, int64_t window_left,
                         void *workspace, int64_t workspace_bytes, void *stream);

/* Workspace bytes fa_fwd_gfx950_padded wants (0: no split; -1: invalid parameters). Host-only. */
int64_t fa_fwd_gfx950_padded_workspace_size(const fa_padded_params *params, int dtype, int causal,
                                            int64_t window_left);

/*
 * RoPE fused into the attention forward (the reference applies RoPE with
 * elementwise torch ops before the call, reference models/rope_attn_fwd.py:14-38, :88).
 * q is given UNROTATED; the kernel rotates it (HF rotate-half convention: q * cos +
 * rotate_half(q) * sin, fp32, one rounding to T) while loading it, with the cos / sin rows of the
 * query positions: row of query m of batch b = b * rope_batch_stride + m * rope_seqlen_stride
 * (elements; cos and sin share the strides, have q's dtype and head dim). k must already be rotated
 * (fa_rope_gfx950: the KV cache stores rotated keys). Head dim 64 or 128; the prefill kernel serves
 * every shape (no split-KV decode path). FA_ERR_UNSUPPORTED otherwise.
 */
typedef struct fa_rope_fwd_params {
    fa_fwd_params base;
    const void *rope_cos;
    const void *rope_sin;
    int64_t rope_batch_stride;
    int64_t rope_seqlen_stride;
} fa_rope_fwd_params;

int fa_fwd_gfx950_rope(const fa_rope_fwd_params *params, int dtype, int causal, void *stream);

/*
 * Local (sliding-window) attention: as fa_fwd_gfx950, and key n is visible to query m only if
 * n >= m + seqlen_kv - seqlen_q - window_left, i.e. each query sees at most the window_left + 1
 * keys ending at its bottom-right diagonal (with causal; without it, every key from that one on).
 * This is transformers' sliding_window (window_left = sliding_window - 1; flash-attn
 * window_size = (window_left, -1)). The reference computes the Qwen2 sliding window and ignores it
 * (reference models/rope_attn_fwd.py:95-101). Keys left of every row's window are cut off the
 * problem; if the window then masks nothing more the call is fa_fwd_gfx950 on the rest (split-KV
 * decode included), else the prefill kernel masks it. window_left < 0: no window.
 */
int fa_fwd_gfx950_window(const fa_fwd_params *params, int dtype, int causal, int64_t window_left, void *stream);

/*
 * Standalone rotate-half RoPE, out = x * cos + rotate_half(x) * sin (same arithmetic as the fused
 * path), x / out [B, H, S, D] with element strides (out == x: in place), cos / sin rows at
 * b * cs_batch_stride + s * cs_seqlen_stride. D even. One HBM pass; asynchronous on `stream`.
 */
typedef struct fa_rope_params {
    const void *x;
    void *out;
    const void *cos;
    const void *sin;
    int64_t batch_size;
    int64_t num_heads;
    int64_t seqlen;
    int64_t headdim;
    int64_t x_batch_stride;
    int64_t x_head_stride;
    int64_t x_seqlen_stride;
    int64_t out_batch_stride;
    int64_t out_head_stride;
    int64_t out_seqlen_stride;
    int64_t cs_batch_stride;
    int64_t cs_seqlen_stride;
} fa_rope_params;

int fa_rope_gfx950(const fa_rope_params *params, int dtype, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* FA_GFX950_H */
