// fa_fwd_gfx950.hip -- C-ABI of the MI355X FlashAttention-2 forward (include/fa_gfx950.h).
//
// Host code only: parameter validation (reference csrc/flash_attention_api.cpp:17-59 restated on
// plain pointers and sizes), the runtime dtype / causal / head-dim dispatch that replaces the
// reference's compile-time dispatcher (csrc/kernel_dispatcher.h:20-52) and tile choice
// (csrc/flash_attention_impl.cu:7-49), and the error channel. The kernels live in
// fa_fwd_kernels.hpp and are instantiated by fa_inst.hip.
#include <hip/hip_runtime.h>
#include <stdarg.h>

#include <mutex>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fa_gfx950.h"
#include "fa_launch.h"

// ============================================================================================
// C-ABI (include/fa_gfx950.h)
// ============================================================================================
namespace {
thread_local char g_err[512] = "";
}  // namespace

int fa::set_err(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

namespace {
unsigned long long *g_stamps = nullptr;
thread_local int g_last_path = fa::kPathNone;

fa::Knobs knobs_from_env() {
    fa::Knobs k{0, 0, 1, fa::kDecTargetWgs, fa::kDecNt, 1, 1, FA_SPLIT_PAIRS, FA_DEC_FUSE, 0, FA_HEAD_PACK, 0, FA_SPLIT_RR};
    if (const char *v = getenv("FA_GFX950_VARIANT"))
        k.variant = !strcmp(v, "w8") ? 1 : !strcmp(v, "w4slow") ? 2 : !strcmp(v, "p8") ? 3 : !strcmp(v, "m32") ? 4
                  : !strcmp(v, "m16") ? 5 : 0;
    if (const char *e = getenv("FA_W4_GRID")) k.w4_grid = atoll(e) > 0 ? atoll(e) : 0;
    if (const char *e = getenv("FA_GFX950_DECODE")) k.decode = strcmp(e, "0") != 0;
    if (const char *e = getenv("FA_DEC_TARGET_WGS")) k.dec_target = atoll(e) > 0 ? atoll(e) : fa::kDecTargetWgs;
    if (const char *e = getenv("FA_DEC_FLAGS")) k.dec_flags = atoi(e);
    if (const char *e = getenv("FA_ZIGZAG")) k.zigzag = atoi(e);
    if (const char *e = getenv("FA_SPLIT")) k.split = atoi(e);
    if (const char *e = getenv("FA_SPLIT_PAIRS")) k.split_pairs = atoi(e);
    if (const char *e = getenv("FA_DEC_FUSE")) k.dec_fuse = atoi(e);
    if (const char *e = getenv("FA_XCCS")) k.xccs = atoi(e) > 0 ? atoi(e) : 0;
    if (const char *e = getenv("FA_HEAD_PACK")) k.head_pack = atoi(e);
    if (const char *e = getenv("FA_SPLIT_RR")) k.split_rr = atoi(e);
#ifdef FA_DEBUG_VARIANTS
    if (k.variant != 0)  // a debug / A-B body replaces the product kernel for the whole process: say so
        fprintf(stderr,
                "[fa_gfx950] FA_GFX950_VARIANT=%s: prefill launches run the %s kernel instead of fa_fwd_w4 "
                "(debug / A-B variant, not the product path)\n",
                getenv("FA_GFX950_VARIANT"),
                k.variant == 1 ? "fa_fwd_w8" : k.variant == 2 ? "w4slow" : k.variant == 3 ? "fa_fwd_p8"
                : k.variant == 4 ? "fa_fwd_mb (32x32x16)" : "fa_fwd_mb (16x16x32)");
#else
    if (k.variant != 0) {  // the product library compiles fa_fwd_w4 only
        fprintf(stderr,
                "[fa_gfx950] FA_GFX950_VARIANT=%s ignored: the debug / A-B kernel bodies are only in "
                "lib/libfa_gfx950_debug.so (built with -DFA_DEBUG_VARIANTS)\n",
                getenv("FA_GFX950_VARIANT"));
        k.variant = 0;
    }
#endif
    return k;
}
const fa::Knobs &env_defaults() {
    static const fa::Knobs d = knobs_from_env();  // once per process, at the first launch
    return d;
}
fa::Knobs &knobs_mut() {
    static fa::Knobs k = env_defaults();
    return k;
}
}  // namespace

const fa::Knobs &fa::knobs() { return knobs_mut(); }
void fa::set_last_path(int path) { g_last_path = path; }

// Diagnostic hooks (not in include/fa_gfx950.h; flash_attention_cute_amd/_debug.py):
// override the knobs for the following launches (a negative value restores that knob's
// environment/default value) and report the kernel the last call on this thread launched.
// Single-threaded test hooks: the knobs are plain process-wide fields, so setting them while
// another thread launches may let that launch see a mix of old and new values.
extern "C" void fa_debug_set_knobs(int variant, int64_t w4_grid, int decode, int64_t dec_target, int dec_flags) {
    const fa::Knobs &d = env_defaults();
    fa::Knobs &k = knobs_mut();
#ifdef FA_DEBUG_VARIANTS
    k.variant = variant < 0 ? d.variant : variant;
#else
    (void)variant;  // (fa_fwd_w4 only in the product library)
#endif
    k.w4_grid = w4_grid < 0 ? d.w4_grid : w4_grid;
    k.decode = decode < 0 ? d.decode : decode;
    k.dec_target = dec_target <= 0 ? d.dec_target : dec_target;
    k.dec_flags = dec_flags < 0 ? d.dec_flags : dec_flags;
}
extern "C" int fa_debug_last_path(void) { return g_last_path; }
// key-split knob (fa_launch.h Knobs::split, env FA_SPLIT): 0 never, 1 (default) when the caller passes
// a workspace and use_split's measured rule holds, 2 whenever a workspace is passed; < 0
// restores the environment / default value
extern "C" void fa_debug_set_split(int mode) {
    knobs_mut().split = mode < 0 ? env_defaults().split : mode;
}
// key-split pairs knob (Knobs::split_pairs, env FA_SPLIT_PAIRS): 0 never, 1 (default) where they fit
// one pass of the grid (use_split_pairs); < 0 restores the environment / default value
extern "C" void fa_debug_set_split_pairs(int mode) {
    knobs_mut().split_pairs = mode < 0 ? env_defaults().split_pairs : mode;
}
// split-KV decode merge knob (Knobs::dec_fuse, env FA_DEC_FUSE): 1 (default) the last split of a unit
// merges the partials in the decode kernel, 0 the separate fa_decode_combine launch; < 0 restores
extern "C" void fa_debug_set_dec_fuse(int mode) {
    knobs_mut().dec_fuse = mode < 0 ? env_defaults().dec_fuse : mode;
}
// placement knob (Knobs::xccs, env FA_XCCS): XCDs per device for same_xcd_placement (0 / < 0: the
// device's own count) -- tests force a count that does not divide 8 to see the fallback layouts
extern "C" void fa_debug_set_xccs(int n) { knobs_mut().xccs = n < 0 ? env_defaults().xccs : n; }
// key-split halves' work order knob (Knobs::split_rr, env FA_SPLIT_RR): 0 the XCD-contiguous
// decode_work ranges, 1 level-major (every XCD a share of every q-tile level); < 0 restores the default
extern "C" void fa_debug_set_split_rr(int mode) {
    knobs_mut().split_rr = mode < 0 ? env_defaults().split_rr : mode;
}
// (debug library only) force one key-split hand-off per launch to time out (slot 0, wave 0; fa_fwd_w4
// dbg & 2): 1 on, 0 off; the product library ignores it
extern "C" void fa_debug_set_split_fault(int on) {
#ifdef FA_DEBUG_VARIANTS
    knobs_mut().split_fault = on > 0 ? 1 : 0;
#else
    (void)on;
#endif
}
// head-packed causal blocks knob (Knobs::head_pack, env FA_HEAD_PACK): 0 never, 1 (default) the rule of
// use_head_pack, 2 wherever it applies; < 0 restores the environment / default value
extern "C" void fa_debug_set_head_pack(int mode) {
    knobs_mut().head_pack = mode < 0 ? env_defaults().head_pack : mode;
}
// zigzag knob (fa_launch.h Knobs::zigzag): 0 never, 1 when the blocks fit one round, 2 always; < 0
// restores the environment / default value. fa_debug_last_zigzag: the causal block layout of the
// last prefill launch on this thread: 0 plain, 1 zigzag, 2 key-split, 3 key-split pairs, 4 head-packed,
// 5 / 6 key-split halves / pairs over head-packed blocks.
extern "C" void fa_debug_set_zigzag(int mode) {
    knobs_mut().zigzag = mode < 0 ? env_defaults().zigzag : mode;
}
namespace {
thread_local int g_last_zigzag = 0;
}
extern "C" int fa_debug_last_zigzag(void) { return g_last_zigzag; }
void fa::set_last_zigzag(int z) { g_last_zigzag = z; }

unsigned long long *fa::stamp_buffer() { return g_stamps; }

int64_t fa::device_cus() {
    // CU count per device, queried once (a racing first query writes the same value)
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = -1;
    int n = dev >= 0 ? cus[dev] : 0;
    if (n <= 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev < 0 ? 0 : dev) != hipSuccess || n <= 0)
            n = 256;
        if (dev >= 0) cus[dev] = n;
    }
    return n;
}

int64_t fa::w4_grid_split(int64_t units) {
    int64_t cap = device_cus();
    if (fa::knobs().w4_grid > 0) cap = fa::knobs().w4_grid;
    cap = cap < 8 ? 8 : cap / 8 * 8;
    const int64_t n = 16 * ((units + 7) / 8);  // 2 pieces x ceil(units / 8) per XCD
    return n < cap ? n : cap;
}

int64_t fa::device_xccs() {
    if (fa::knobs().xccs > 0) return fa::knobs().xccs;
    // XCDs per device, queried once (a racing first query writes the same value); unknown -> 0, which
    // fails same_xcd_placement (the dispatcher then takes the layouts without a hand-off)
    static int xccs[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    if (xccs[dev] <= 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeNumberOfXccs, dev) != hipSuccess || n <= 0) return 0;
        xccs[dev] = n;
    }
    return xccs[dev];
}

// Key-split / fused-decode counter areas (fa_launch.h split_sync_area): one per (device, stream),
// allocated the first time such an eager launch runs on that stream and zeroed by a memset ON THAT
// STREAM (ordered before the launch that gets it; no hipDeviceSynchronize, which would stall every
// stream of the device and break another thread's graph capture), never freed. The kernels zero their
// counters again -- a timed-out key-split hand-off included (fa_fwd_w4 abandons the pair) -- so the
// area is zero between launches and no launch needs a memset. Each area ends in its stream's hand-off
// error counter. Launches under graph capture never get an area (split_sync_area).
namespace {
constexpr int64_t kSyncAreaBytes = 256 * 1024;  // 8192 blocks x 4 waves x 2 counters
constexpr int64_t kAreaAlloc = kSyncAreaBytes + 256;  // + the error counter
constexpr int kMaxAreas = 64;
struct SyncArea {
    int dev;
    hipStream_t stream;
    unsigned *ptr;
    unsigned *err() const { return ptr + kSyncAreaBytes / 4; }
};
std::mutex g_sync_mu;
SyncArea g_areas[kMaxAreas];
int g_n_areas = 0;
thread_local int g_last_dec_fused = 0;
}  // namespace

void fa::set_last_dec_fused(bool fused) { g_last_dec_fused = fused ? 1 : 0; }
extern "C" int fa_debug_last_dec_fused(void) { return g_last_dec_fused; }

unsigned *fa::split_sync_area(hipStream_t stream, int64_t bytes, unsigned **err) {
    *err = nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess) return nullptr;
    const bool capturing = cs != hipStreamCaptureStatusNone;
    std::lock_guard<std::mutex> lk(g_sync_mu);
    SyncArea *a = nullptr;
    for (int i = 0; i < g_n_areas && !a; ++i)
        if (g_areas[i].dev == dev && g_areas[i].stream == stream) a = &g_areas[i];
    if (capturing) {  // (a graph's replays may run beside eager launches on this stream: no shared counters)
        *err = a ? a->err() : nullptr;
        return nullptr;
    }
    if (!a) {
        if (g_n_areas >= kMaxAreas) return nullptr;
        unsigned *ptr = nullptr;
        // (this thread in relaxed capture mode for the allocation: another stream of the process may be
        // capturing a graph in global mode, which forbids hipMalloc to threads in global mode -- the
        // allocation is not part of any capture, and this stream is not capturing)
        hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
        const bool swapped = hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess;
        const hipError_t me = hipMalloc(&ptr, kAreaAlloc);
        if (swapped) (void)hipThreadExchangeStreamCaptureMode(&mode);
        if (me != hipSuccess) return nullptr;
        if (hipMemsetAsync(ptr, 0, kAreaAlloc, stream) != hipSuccess) {
            (void)hipFree(ptr);
            return nullptr;
        }
        g_areas[g_n_areas] = {dev, stream, ptr};
        a = &g_areas[g_n_areas++];
    }
    *err = a->err();
    return bytes > kSyncAreaBytes ? nullptr : a->ptr;
}

extern "C" int64_t fa_split_errors(int reset) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    unsigned *errs[kMaxAreas];
    int n_err = 0;
    {
        std::lock_guard<std::mutex> lk(g_sync_mu);
        for (int i = 0; i < g_n_areas; ++i)
            if (g_areas[i].dev == dev) errs[n_err++] = g_areas[i].err();
    }
    if (!n_err || hipDeviceSynchronize() != hipSuccess) return 0;
    int64_t total = 0;
    for (int i = 0; i < n_err; ++i) {
        unsigned n = 0;
        if (hipMemcpy(&n, errs[i], sizeof(n), hipMemcpyDeviceToHost) != hipSuccess) return total;
        total += n;
        if (reset && n) (void)hipMemset(errs[i], 0, sizeof(unsigned));
    }
    return total;
}

int64_t fa::w4_grid(int64_t nwg) {
    int64_t cap = device_cus();
    if (fa::knobs().w4_grid > 0) cap = fa::knobs().w4_grid;
    if (nwg <= cap) return nwg;  // one Q block per workgroup
    // Capped: the kernel deals Q block i to the workgroups with (bid & 7) == (i & 7), so every
    // residue class needs a workgroup -- at least 8, a multiple of 8 (equal rounds per XCD).
    cap = cap < 8 ? 8 : cap / 8 * 8;
    return nwg < cap ? nwg : cap;
}

// Diagnostic hook (not in include/fa_gfx950.h): device buffer of 15 u64 per wave (19 with FA_STAMPS_FINE) of the next
// launches; honoured only by a -DFA_STAMPS=1 build of the kernels (scripts/stamps.py).
extern "C" void fa_debug_set_stamps(void *device_buffer) { g_stamps = (unsigned long long *)device_buffer; }

namespace {
using fa::set_err;
using fa::launch_one;

bool aligned16(const void *ptr) { return ((uintptr_t)ptr & 15) == 0; }

constexpr fa::PathArgs kNoPath{nullptr, nullptr, 0, 0, -1, 0, nullptr, nullptr, nullptr, nullptr};

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
    if (p->seqlen_q > 0x3fffffffLL || p->seqlen_kv > 0x3fffffffLL)
        return set_err(FA_ERR_UNSUPPORTED, "sequence lengths must be < 2^30");
    // 32-bit lane offsets inside one 64-row K/V tile and one wave's Q/O slab: fa_fwd_w4 interleaves
    // a wave's two 32-row blocks kBlockM / 2 rows apart, so its slab spans kQoSpanRows rows
    for (int i = 8; i < 12; ++i) {
        const int64_t rows = (i == 8 || i == 11) ? fa::kQoSpanRows : fa::kBlockN;
        if (strides[i] < 0 || strides[i] * 2 * rows + 256 > 0x7fffffffLL)
            return set_err(FA_ERR_UNSUPPORTED, "sequence stride too large for 32-bit tile offsets");
    }
    const int64_t n_qtiles = (p->seqlen_q + fa::kBlockM - 1) / fa::kBlockM;
    const int64_t nwg = n_qtiles * p->num_heads_q * p->batch_size;
    if (nwg > 0x7fffffffLL) return set_err(FA_ERR_UNSUPPORTED, "grid too large (%lld workgroups)", (long long)nwg);
    g_err[0] = 0;
    return FA_OK;
}

// head-dim dispatch: D <= 64 runs the 64-wide tile, 64 < D <= 128 the 128-wide tile (the reference
// runs every D <= 128 on its 128 kernel, csrc/kernel_dispatcher.h:45-52)
template <class DT, bool C>
int launch(const fa_fwd_params &p, hipStream_t stream, const fa::PathArgs &xa = kNoPath) {
    if (p.headdim <= 64)
        return p.headdim == 64 ? launch_one<DT, C, 64, true>(p, xa, stream)
                               : launch_one<DT, C, 64, false>(p, xa, stream);
    return p.headdim == 128 ? launch_one<DT, C, 128, true>(p, xa, stream)
                            : launch_one<DT, C, 128, false>(p, xa, stream);
}
template <class DT, bool C>
int launch_dec(const fa_fwd_params &p, const fa::DecArgs &a, void *ws, hipStream_t stream) {
    if (p.headdim <= 64)
        return p.headdim == 64 ? fa::launch_decode<DT, C, 64, true>(p, a, ws, stream)
                               : fa::launch_decode<DT, C, 64, false>(p, a, ws, stream);
    return p.headdim == 128 ? fa::launch_decode<DT, C, 128, true>(p, a, ws, stream)
                            : fa::launch_decode<DT, C, 128, false>(p, a, ws, stream);
}

// Split-KV decode path (fa_decode.hpp) for few (q-head, position) rows per (batch, kv-head): the
// reference's Sq == 1 pack and short GQA query blocks. The `decode` knob (FA_GFX950_DECODE=0) sends
// them to the prefill kernel instead (A/B measurements).
bool use_decode(const fa_fwd_params &p, const fa::PathArgs &ranges = kNoPath) {
    if (ranges.q_rng) return false;  // query ranges: fa_fwd_w4
    if (!fa::knobs().decode || fa::knobs().variant != 0) return false;
    if (p.head_q_per_group * p.seqlen_q > fa::kDecMaxRows) return false;
    // the row block's q rows are addressed by 32-bit offsets from the group's first q-head
    const int64_t qspan = ((p.head_q_per_group - 1) * p.q_head_stride + (p.seqlen_q - 1) * p.q_seqlen_stride +
                           p.headdim) * 2;
    return qspan >= 0 && qspan < 0x7ff00000LL;
}

// ranges: per-sequence query / key ranges (fa_fwd_gfx950_padded), or kNoPath
int dispatch(const fa_fwd_params *params, int dtype, int causal, void *ws, int64_t ws_bytes, void *stream,
             const fa::PathArgs &ranges = kNoPath) {
    g_last_path = fa::kPathNone;
    const int rc = check_params(params, dtype, causal);
    if (rc != FA_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    const fa_fwd_params &p = *params;
    if (use_decode(p, ranges)) {
        fa::DecArgs a = fa::decode_plan(p, ws ? fa::kDecMaxSplit : 1);
        a.k_lo = ranges.k_lo;
        a.k_hi = ranges.k_hi;
        if (ws && fa::decode_ws_bytes(p, a) > ws_bytes)
            return set_err(FA_ERR_INVALID_ARGUMENT, "workspace of %lld bytes is smaller than the %lld required",
                           (long long)ws_bytes, (long long)fa::decode_ws_bytes(p, a));
        if (dtype == FA_DTYPE_F16)
            return causal ? launch_dec<fa::F16, true>(p, a, ws, s) : launch_dec<fa::F16, false>(p, a, ws, s);
        return causal ? launch_dec<fa::BF16, true>(p, a, ws, s) : launch_dec<fa::BF16, false>(p, a, ws, s);
    }
    fa::PathArgs xa = ranges;
    // key-split causal blocks (fa_launch.h use_split) when the workspace holds their partials; a
    // smaller one runs the blocks unsplit (zigzag), as without a workspace
    if (ws && fa::use_split(p, causal != 0, ranges) && fa::split_ws_bytes(p) <= ws_bytes) {
        xa.split_ws = (float *)((char *)ws + fa::split_sync_bytes(p));
        xa.split_sync = fa::split_sync_area(s, fa::split_sync_bytes(p), &xa.split_err);
        if (!xa.split_sync) {  // (graph capture before the stream's area exists: counters in the workspace)
            xa.split_sync = (unsigned *)ws;
            const hipError_t e = hipMemsetAsync(ws, 0, fa::split_sync_bytes(p), s);
            if (e != hipSuccess) return set_err(FA_ERR_LAUNCH, "hipMemsetAsync failed: %s", hipGetErrorString(e));
        }
    }
    if (dtype == FA_DTYPE_F16)
        return causal ? launch<fa::F16, true>(p, s, xa) : launch<fa::F16, false>(p, s, xa);
    return causal ? launch<fa::BF16, true>(p, s, xa) : launch<fa::BF16, false>(p, s, xa);
}

int check_varlen(const fa_varlen_params *v, int dtype, int causal) {
    if (!v) return set_err(FA_ERR_INVALID_ARGUMENT, "params is NULL");
    if (!v->cu_seqlens_q || !v->cu_seqlens_k)
        return set_err(FA_ERR_INVALID_ARGUMENT, "cu_seqlens_q and cu_seqlens_k must be non-NULL");
    if (((uintptr_t)v->cu_seqlens_q & 3) || ((uintptr_t)v->cu_seqlens_k & 3))
        return set_err(FA_ERR_INVALID_ARGUMENT, "cu_seqlens must be 4-byte aligned int32 arrays");
    // packed layout: the batch strides are not used (a sequence starts at row cu_seqlens[b])
    fa_fwd_params p = v->base;
    p.q_batch_stride = p.k_batch_stride = p.v_batch_stride = p.o_batch_stride = 0;
    return check_params(&p, dtype, causal);
}

// window_left >= 0: the local window per sequence (the kernel starts each Q block at its first
// visible tile; no host cut, the sequence bounds live on the device). The window is always passed
// to the kernel: a window longer than a sequence hides nothing there (its per-sequence first tile
// is 0), so a seqlen_kv below the true maximum cannot drop it.
int dispatch_varlen(const fa_varlen_params *v, int dtype, int causal, void *stream, int64_t window_left = -1) {
    g_last_path = fa::kPathNone;
    const int rc = check_varlen(v, dtype, causal);
    if (rc != FA_OK) return rc;
    if (window_left > 0x3fffffffLL) window_left = 0x3fffffff;  // (hides nothing either way)
    hipStream_t s = (hipStream_t)stream;
    const int *cq = v->cu_seqlens_q, *ck = v->cu_seqlens_k;
    // packed rows: sequence b is rows [cu[b], cu[b + 1]) of the tensors, no batch offset
    fa_fwd_params p = v->base;
    p.q_batch_stride = p.k_batch_stride = p.v_batch_stride = p.o_batch_stride = 0;
    const fa::PathArgs xa{nullptr, nullptr, 0, 0, window_left < 0 ? -1 : (int)window_left, 1, cq, ck, nullptr, nullptr};
    if (dtype == FA_DTYPE_F16)
        return causal ? launch<fa::F16, true>(p, s, xa) : launch<fa::F16, false>(p, s, xa);
    return causal ? launch<fa::BF16, true>(p, s, xa) : launch<fa::BF16, false>(p, s, xa);
}

int check_padded(const fa_padded_params *v, int dtype, int causal) {
    if (!v) return set_err(FA_ERR_INVALID_ARGUMENT, "params is NULL");
    if (!v->k_start != !v->k_end || !v->q_start != !v->q_end)
        return set_err(FA_ERR_INVALID_ARGUMENT, "k_start / k_end (and q_start / q_end) must be given together");
    const int32_t *arr[4] = {v->q_start, v->q_end, v->k_start, v->k_end};
    for (int i = 0; i < 4; ++i)
        if ((uintptr_t)arr[i] & 3) return set_err(FA_ERR_INVALID_ARGUMENT, "ranges must be 4-byte aligned int32 arrays");
    if (v->base.batch_size > 0x7fffffffLL) return set_err(FA_ERR_UNSUPPORTED, "batch too large");
    return check_params(&v->base, dtype, causal);
}

// The decode kernel reads per-sequence key positions as given. The prefill kernel addresses a
// ranged sequence by ABSOLUTE rows (row r at base + r * seqlen stride, batch strides unused), so the
// dispatcher converts the positions into [2, B] row arrays in the workspace: rows of batch row b =
// b * rows_per_batch + position (a missing range is the whole dimension).
__global__ void padded_rows(int32_t *q_rng, int32_t *k_rng, const int32_t *qs, const int32_t *qe, const int32_t *ks,
                            const int32_t *ke, int batch, int64_t q_rpb, int64_t k_rpb, int sq, int sk) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < batch) {
        // positions clamped to the dimension (start into [0, n], end into [start, n]): a range past
        // the tensor never addresses another batch row's rows or memory past the allocation
        const int q0 = qs ? min(max(qs[b], 0), sq) : 0, q1 = qe ? min(max(qe[b], q0), sq) : sq;
        const int k0 = ks ? min(max(ks[b], 0), sk) : 0, k1 = ke ? min(max(ke[b], k0), sk) : sk;
        q_rng[b] = (int32_t)(b * q_rpb + q0);
        q_rng[batch + b] = (int32_t)(b * q_rpb + q1);
        k_rng[b] = (int32_t)(b * k_rpb + k0);
        k_rng[batch + b] = (int32_t)(b * k_rpb + k1);
    }
}

bool padded_on_decode(const fa_padded_params *v, int64_t window_left) {
    return !v->q_start && window_left < 0 && use_decode(v->base);
}
// workspace of a prefill-kernel padded launch: the two [2, B] row arrays, 16-B aligned
int64_t padded_rows_bytes(const fa_padded_params *v) { return (4 * v->base.batch_size * 4 + 15) / 16 * 16; }

// Padded batches: per-sequence query / key positions inside dense tensors. Few rows per kv-head (no
// query ranges, no window) run the split-KV decode kernel on each sequence's key positions, all else
// fa_fwd_w4 on the row arrays built in the workspace; window_left >= 0 applies the local window per
// sequence.
int dispatch_padded(const fa_padded_params *v, int dtype, int causal, int64_t window_left, void *ws,
                    int64_t ws_bytes, void *stream) {
    g_last_path = fa::kPathNone;
    const int rc = check_padded(v, dtype, causal);
    if (rc != FA_OK) return rc;
    if (window_left > 0x3fffffffLL) window_left = 0x3fffffff;
    hipStream_t s = (hipStream_t)stream;
    if (padded_on_decode(v, window_left)) {
        fa::PathArgs xa = kNoPath;
        xa.k_lo = v->k_start;
        xa.k_hi = v->k_end;
        return dispatch(&v->base, dtype, causal, ws, ws_bytes, stream, xa);
    }
    const fa_fwd_params &b = v->base;
    auto rpb = [](int64_t bstride, int64_t sstride, int64_t nb) -> int64_t {
        if (nb == 1) return 0;
        return (sstride > 0 && bstride % sstride == 0) ? bstride / sstride : -1;
    };
    const int64_t q_rpb = rpb(b.q_batch_stride, b.q_seqlen_stride, b.batch_size);
    const int64_t k_rpb = rpb(b.k_batch_stride, b.k_seqlen_stride, b.batch_size);
    if (q_rpb < 0 || k_rpb < 0 || rpb(b.o_batch_stride, b.o_seqlen_stride, b.batch_size) != q_rpb ||
        rpb(b.v_batch_stride, b.v_seqlen_stride, b.batch_size) != k_rpb ||
        (b.batch_size - 1) * q_rpb + b.seqlen_q > 0x7fffffffLL || (b.batch_size - 1) * k_rpb + b.seqlen_kv > 0x7fffffffLL)
        return set_err(FA_ERR_INVALID_ARGUMENT,
                       "padded prefill: the batch strides of q / o (k / v) must be the same multiple of their seqlen "
                       "strides");
    const int64_t need = padded_rows_bytes(v);
    if (!ws || ws_bytes < need)
        return set_err(FA_ERR_INVALID_ARGUMENT, "workspace of %lld bytes is smaller than the %lld required",
                       (long long)ws_bytes, (long long)need);
    int32_t *q_rng = (int32_t *)ws, *k_rng = q_rng + 2 * b.batch_size;
    hipLaunchKernelGGL(padded_rows, dim3((uint32_t)((b.batch_size + 255) / 256)), dim3(256), 0, s, q_rng, k_rng,
                       v->q_start, v->q_end, v->k_start, v->k_end, (int)b.batch_size, q_rpb, k_rpb, (int)b.seqlen_q,
                       (int)b.seqlen_kv);
    fa_fwd_params p = b;
    p.q_batch_stride = p.k_batch_stride = p.v_batch_stride = p.o_batch_stride = 0;
    fa::PathArgs xa = kNoPath;
    xa.window_left = window_left < 0 ? -1 : (int)window_left;
    xa.rng_hi = (int)b.batch_size;
    xa.q_rng = q_rng;
    xa.k_rng = k_rng;
    if (dtype == FA_DTYPE_F16)
        return causal ? launch<fa::F16, true>(p, s, xa) : launch<fa::F16, false>(p, s, xa);
    return causal ? launch<fa::BF16, true>(p, s, xa) : launch<fa::BF16, false>(p, s, xa);
}

int dispatch_rope(const fa_rope_fwd_params *r, int dtype, int causal, void *stream) {
    g_last_path = fa::kPathNone;
    if (!r) return set_err(FA_ERR_INVALID_ARGUMENT, "params is NULL");
    const int rc = check_params(&r->base, dtype, causal);
    if (rc != FA_OK) return rc;
    if (!r->rope_cos || !r->rope_sin) return set_err(FA_ERR_INVALID_ARGUMENT, "rope_cos and rope_sin must be non-NULL");
    if (r->base.headdim != 64 && r->base.headdim != 128)
        return set_err(FA_ERR_UNSUPPORTED, "fused RoPE supports head dim 64 or 128 (got %lld)", (long long)r->base.headdim);
    if (!aligned16(r->rope_cos) || !aligned16(r->rope_sin) || r->rope_batch_stride % 8 || r->rope_seqlen_stride % 8)
        return set_err(FA_ERR_INVALID_ARGUMENT, "RoPE tables must be 16-byte aligned with strides multiple of 8");
    if (r->rope_seqlen_stride < 0 || r->rope_seqlen_stride * 2 * fa::kQoSpanRows + 256 > 0x7fffffffLL)
        return set_err(FA_ERR_UNSUPPORTED, "RoPE seqlen stride too large for 32-bit tile offsets");
    const fa::PathArgs ra{r->rope_cos, r->rope_sin, r->rope_batch_stride, r->rope_seqlen_stride, -1, 0, nullptr, nullptr, nullptr, nullptr};
    hipStream_t s = (hipStream_t)stream;
    if (dtype == FA_DTYPE_F16)
        return causal ? launch<fa::F16, true>(r->base, s, ra) : launch<fa::F16, false>(r->base, s, ra);
    return causal ? launch<fa::BF16, true>(r->base, s, ra) : launch<fa::BF16, false>(r->base, s, ra);
}

// Local (sliding) window: keys below the first row's window are cut off the problem (views of k /
// v, so the kernel never fetches them); if the window then cuts nothing more, the plain path runs
// (including the split-KV decode kernel), else fa_fwd_w4 with the window mask.
int dispatch_window(const fa_fwd_params *params, int dtype, int causal, int64_t window_left, void *stream) {
    g_last_path = fa::kPathNone;
    const int rc = check_params(params, dtype, causal);
    if (rc != FA_OK) return rc;
    if (window_left < 0) return dispatch(params, dtype, causal, nullptr, 0, stream);
    fa_fwd_params p = *params;
    int64_t cut = p.seqlen_kv - p.seqlen_q - window_left;
    if (cut > 0) {
        p.k_ptr = (const char *)p.k_ptr + 2 * cut * p.k_seqlen_stride;
        p.v_ptr = (const char *)p.v_ptr + 2 * cut * p.v_seqlen_stride;
        p.seqlen_kv -= cut;
    }
    // the last query row's window starts at key Sk' - 1 - window_left: at or before 0, nothing is cut
    if (p.seqlen_kv - 1 <= window_left) return dispatch(&p, dtype, causal, nullptr, 0, stream);
    const fa::PathArgs xa{nullptr, nullptr, 0, 0, (int)window_left, 0, nullptr, nullptr, nullptr, nullptr};
    hipStream_t s = (hipStream_t)stream;
    if (dtype == FA_DTYPE_F16)
        return causal ? launch<fa::F16, true>(p, s, xa) : launch<fa::F16, false>(p, s, xa);
    return causal ? launch<fa::BF16, true>(p, s, xa) : launch<fa::BF16, false>(p, s, xa);
}

}  // namespace

extern "C" int fa_fwd_gfx950_window(const fa_fwd_params *params, int dtype, int causal, int64_t window_left,
                                    void *stream) {
    return dispatch_window(params, dtype, causal, window_left, stream);
}

extern "C" int fa_fwd_gfx950_rope(const fa_rope_fwd_params *params, int dtype, int causal, void *stream) {
    return dispatch_rope(params, dtype, causal, stream);
}

extern "C" int fa_fwd_gfx950_varlen(const fa_varlen_params *params, int dtype, int causal, void *stream) {
    return dispatch_varlen(params, dtype, causal, stream);
}

extern "C" int fa_fwd_gfx950_varlen_window(const fa_varlen_params *params, int dtype, int causal,
                                           int64_t window_left, void *stream) {
    return dispatch_varlen(params, dtype, causal, stream, window_left);
}

extern "C" int fa_fwd_gfx950_padded(const fa_padded_params *params, int dtype, int causal, int64_t window_left,
                                    void *workspace, int64_t workspace_bytes, void *stream) {
    if (workspace && ((uintptr_t)workspace & 15))
        return set_err(FA_ERR_INVALID_ARGUMENT, "workspace must be 16-byte aligned");
    return dispatch_padded(params, dtype, causal, window_left, workspace_bytes > 0 ? workspace : nullptr,
                           workspace_bytes, stream);
}

extern "C" int64_t fa_fwd_gfx950_padded_workspace_size(const fa_padded_params *params, int dtype, int causal,
                                                       int64_t window_left) {
    if (check_padded(params, dtype, causal) != FA_OK) return -1;
    if (!padded_on_decode(params, window_left)) return padded_rows_bytes(params);
    return fa::decode_ws_bytes(params->base, fa::decode_plan(params->base, fa::kDecMaxSplit));
}

extern "C" int fa_fwd_gfx950_varlen_check(const fa_varlen_params *params, int dtype, int causal) {
    return check_varlen(params, dtype, causal);
}

extern "C" int fa_fwd_gfx950_check(const fa_fwd_params *params, int dtype, int causal) {
    return check_params(params, dtype, causal);
}

extern "C" int fa_fwd_gfx950(const fa_fwd_params *params, int dtype, int causal, void *stream) {
    return dispatch(params, dtype, causal, nullptr, 0, stream);
}

extern "C" int64_t fa_fwd_gfx950_workspace_size(const fa_fwd_params *params, int dtype, int causal) {
    if (check_params(params, dtype, causal) != FA_OK) return -1;
    if (!use_decode(*params)) return fa::use_split(*params, causal != 0, kNoPath) ? fa::split_ws_bytes(*params) : 0;
    return fa::decode_ws_bytes(*params, fa::decode_plan(*params, fa::kDecMaxSplit));
}

extern "C" int fa_fwd_gfx950_ws(const fa_fwd_params *params, int dtype, int causal, void *workspace,
                                int64_t workspace_bytes, void *stream) {
    if (workspace && ((uintptr_t)workspace & 15))
        return set_err(FA_ERR_INVALID_ARGUMENT, "workspace must be 16-byte aligned");
    return dispatch(params, dtype, causal, workspace_bytes > 0 ? workspace : nullptr, workspace_bytes, stream);
}

extern "C" const char *fa_last_error(void) { return g_err; }

extern "C" int fa_abi_version(void) { return FA_GFX950_ABI_VERSION; }

extern "C" int fa_fwd_gfx950_geometry(const fa_fwd_params *params, int causal, int64_t *block_m,
                                      int64_t *block_n, int64_t *threads, int64_t *workgroups) {
    if (!params) return set_err(FA_ERR_INVALID_ARGUMENT, "params is NULL");
    if (use_decode(*params)) {
        // without a workspace fa_fwd_gfx950 runs the decode kernel unsplit
        const fa::DecArgs a = fa::decode_plan(*params, 1);
        if (block_m) *block_m = fa::kDecRows;
        if (block_n) *block_n = fa::kDecKeys;
        if (threads) *threads = fa::kDecWaves * 64;
        if (workgroups) *workgroups = fa::decode_units(*params, a) * a.n_split;
        return FA_OK;
    }
    // (head-packed blocks: (batch, q-head quad, 64 rows) units of 4 q-heads x 64 rows)
    const bool hpk = fa::use_head_pack(*params, causal != 0, kNoPath);
    const bool zz = !hpk && fa::use_zigzag(*params, causal != 0, kNoPath);
    const int64_t n_qtiles = zz ? fa::zigzag_qtiles(params->seqlen_q)
                             : hpk ? (params->seqlen_q + 63) / 64 : (params->seqlen_q + fa::kBlockM - 1) / fa::kBlockM;
    if (block_m) *block_m = fa::kBlockM;
    if (block_n) *block_n = fa::kBlockN;
    if (threads) *threads = (fa::variant_from_env() == 1 || fa::variant_from_env() == 3 ? fa::kThreads : 256);
    if (workgroups) *workgroups = n_qtiles * (hpk ? params->num_heads_q / 4 : params->num_heads_q) * params->batch_size;
    return FA_OK;
}
