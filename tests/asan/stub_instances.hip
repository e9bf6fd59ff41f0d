// Host-only stand-ins for the 16 kernel instantiations (csrc/fa_inst.hip), so the C-ABI dispatcher
// (csrc/fa_fwd_gfx950.hip) links into the sanitizer test driver without device code: a launch that
// gets past validation reports FA_ERR_UNSUPPORTED here instead of touching a GPU.
#include "fa_launch.h"

namespace fa {
template <class DT, bool C, int kD, bool kExact>
int launch_one(const fa_fwd_params &, const PathArgs &, hipStream_t) {
    return set_err(FA_ERR_UNSUPPORTED, "stub instantiation (sanitizer build)");
}
template <class DT, bool C, int kD, bool kExact>
int launch_decode(const fa_fwd_params &, DecArgs, void *, hipStream_t) {
    return set_err(FA_ERR_UNSUPPORTED, "stub instantiation (sanitizer build)");
}
#define FA_STUB_INSTANCE(DT, C, D, E)                                                             \
    template int launch_one<DT, C, D, E>(const fa_fwd_params &, const PathArgs &, hipStream_t); \
    template int launch_decode<DT, C, D, E>(const fa_fwd_params &, DecArgs, void *, hipStream_t);
FA_FOR_EACH_INSTANCE(FA_STUB_INSTANCE)
}  // namespace fa
