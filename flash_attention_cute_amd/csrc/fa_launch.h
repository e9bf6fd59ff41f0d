// fa_launch.h -- internal seam between the C-ABI dispatcher (fa_fwd_gfx950.hip) and the kernel
// instantiations (fa_inst.hip x 16, one translation unit per combination so they compile in
// parallel). Not part of the public boundary; include/fa_gfx950.h is.
#pragma once

#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include "fa_gfx950.h"

namespace fa {

constexpr int kBlockM = 256;  // query rows per workgroup
constexpr int kBlockN = 64;   // keys per KV tile
constexpr int kWaves = 8;     // fa_fwd_w8
constexpr int kThreads = kWaves * 64;

struct F16;
struct BF16;

// records a message for fa_last_error() and returns `code`
int set_err(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

// Kernel variant: 0 = fa_fwd_w4 (default), 1 = fa_fwd_w8 (FA_GFX950_VARIANT=w8: the 8-wave
// register-staged kernel, kept for A/B measurements and as a cross-check in the tests),
// 2 = w4 without its pipelined body (FA_GFX950_VARIANT=w4slow, debug).
inline int variant_from_env() {
    const char *v = getenv("FA_GFX950_VARIANT");
    if (v && strcmp(v, "w8") == 0) return 1;
    if (v && strcmp(v, "w4slow") == 0) return 2;
    return 0;
}

// diagnostic per-wave phase stamps of fa_fwd_w4 (only a -DFA_STAMPS=1 build writes them; see
// fa_debug_set_stamps in fa_fwd_gfx950.hip and scripts/stamps.py); nullptr otherwise
unsigned long long *stamp_buffer();

// launch one (dtype, causal, head-dim tile, exact head dim) instantiation on `stream`
template <class DT, bool C, int kD, bool kExact>
int launch_one(const fa_fwd_params &p, hipStream_t stream);

#define FA_FOR_EACH_INSTANCE(X)                                                                    \
    X(F16, false, 64, false) X(F16, false, 64, true) X(F16, false, 128, false) X(F16, false, 128, true) \
    X(F16, true, 64, false) X(F16, true, 64, true) X(F16, true, 128, false) X(F16, true, 128, true)     \
    X(BF16, false, 64, false) X(BF16, false, 64, true) X(BF16, false, 128, false)                      \
    X(BF16, false, 128, true) X(BF16, true, 64, false) X(BF16, true, 64, true)                         \
    X(BF16, true, 128, false) X(BF16, true, 128, true)

#define FA_DECLARE_EXTERN(DT, C, D, E) extern template int launch_one<DT, C, D, E>(const fa_fwd_params &, hipStream_t);
FA_FOR_EACH_INSTANCE(FA_DECLARE_EXTERN)
#undef FA_DECLARE_EXTERN

}  // namespace fa
