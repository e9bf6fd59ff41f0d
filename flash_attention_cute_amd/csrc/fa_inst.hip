// fa_inst.hip -- one kernel instantiation per translation unit. _build.py compiles this file once
// per combination of FA_INST_DT (F16 | BF16), FA_INST_CAUSAL (0 | 1), FA_INST_D (64 | 128) and
// FA_INST_EXACT (0 | 1), in parallel, and links the objects with fa_fwd_gfx950.hip.
#ifndef FA_INST_STUB
#include "fa_fwd_kernels.hpp"
#ifdef FA_DEBUG_VARIANTS  // (the debug / A-B library: the paired 8-wave body, the MFMA-shape A/B body)
#include "fa_fwd_p8.hpp"
#include "fa_fwd_mb.hpp"
#endif
#include "fa_decode.hpp"
#else
// diagnostic builds that only need some instantiations (_build.build_abi(only=...)): the others
// are stubs that report FA_ERR_UNSUPPORTED
#include "fa_launch.h"
namespace fa {
template <class DT, bool C, int kD, bool kExact>
int launch_one(const fa_fwd_params &, const PathArgs &, hipStream_t) { return set_err(FA_ERR_UNSUPPORTED, "stub instantiation"); }
template <class DT, bool C, int kD, bool kExact>
int launch_decode(const fa_fwd_params &, DecArgs, void *, hipStream_t) {
    return set_err(FA_ERR_UNSUPPORTED, "stub instantiation");
}
}  // namespace fa
#endif

#if !defined(FA_INST_DT) || !defined(FA_INST_CAUSAL) || !defined(FA_INST_D) || !defined(FA_INST_EXACT)
#error "fa_inst.hip needs -DFA_INST_DT= -DFA_INST_CAUSAL= -DFA_INST_D= -DFA_INST_EXACT="
#endif

namespace fa {
template int launch_one<FA_INST_DT, (FA_INST_CAUSAL != 0), FA_INST_D, (FA_INST_EXACT != 0)>(const fa_fwd_params &,
                                                                                        const PathArgs &, hipStream_t);
template int launch_decode<FA_INST_DT, (FA_INST_CAUSAL != 0), FA_INST_D, (FA_INST_EXACT != 0)>(const fa_fwd_params &,
                                                                                           DecArgs, void *,
                                                                                           hipStream_t);
}  // namespace fa
