// fa_rope.hip -- standalone rotate-half RoPE for gfx950 (C-ABI fa_rope_gfx950, include/fa_gfx950.h).
//
// The caller-side half of SURVEY.md 8(f) row 3. The reference applies RoPE with six elementwise
// torch ops per tensor before the attention call (reference models/rope_attn_fwd.py:8-38, :88). Here:
//   * Q is rotated inside the attention kernel's Q load (fa_fwd_kernels.hpp, load_q_rope) -- no pass;
//   * K is rotated by this kernel in ONE HBM pass (read x, cos, sin; write out), because the rotated
//     keys must be materialised anyway (the KV cache stores them) and every K tile is re-read by
//     Sq / 256 workgroups of the attention kernel, so rotating it per tile would multiply the work.
// It also serves Q where the fused path does not apply (decode-sized query blocks, other head dims).
//
// Arithmetic as the fused path: out = fma(x, cos, rot * sin) in fp32, rot = -x[d + D/2] (d < D/2) or
// x[d - D/2], rounded once (RNE) to T. HBM-bound: 2 * |x| + |cos| + |sin| bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fa_gfx950.h"
#include "fa_launch.h"

namespace fa {
namespace {

typedef uint32_t u32x4r __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <bool kF16>
__device__ __forceinline__ float ld(const uint16_t v) {
    if constexpr (kF16) return (float)__builtin_bit_cast(_Float16, v);
    else return (float)__builtin_bit_cast(__bf16, v);
}
template <bool kF16>
__device__ __forceinline__ uint16_t st(const float f) {
    if constexpr (kF16) return __builtin_bit_cast(uint16_t, (_Float16)f);
    else return __builtin_bit_cast(uint16_t, (__bf16)f);
}
template <bool kF16>
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
    if constexpr (kF16) {
        typedef _Float16 hh2 __attribute__((ext_vector_type(2)));
        return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){lo, hi}, hh2));
    } else {
        typedef __bf16 bb2 __attribute__((ext_vector_type(2)));
        return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){lo, hi}, bb2));
    }
}

// one thread per (row, 8-element chunk of the first half): reads the chunk and its partner of x,
// cos and sin (16-B loads), writes both rotated chunks. kVec = false: one element pair per thread.
template <bool kF16, bool kVec>
__global__ __launch_bounds__(256) void fa_rope_kernel(const fa_rope_params p, const int64_t n_items) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_items) return;
    const int W = kVec ? 8 : 1;
    const int half = (int)p.headdim / 2;
    const int per_row = half / W;
    const int c = (int)(i % per_row);
    const int64_t row = i / per_row;  // (b, h, s) row-major
    const int64_t s = row % p.seqlen, bh = row / p.seqlen;
    const int64_t h = bh % p.num_heads, b = bh / p.num_heads;
    const uint16_t *x = (const uint16_t *)p.x + b * p.x_batch_stride + h * p.x_head_stride + s * p.x_seqlen_stride;
    uint16_t *o = (uint16_t *)p.out + b * p.out_batch_stride + h * p.out_head_stride + s * p.out_seqlen_stride;
    const int64_t cso = b * p.cs_batch_stride + s * p.cs_seqlen_stride;
    const uint16_t *cs = (const uint16_t *)p.cos + cso, *sn = (const uint16_t *)p.sin + cso;
    const int d0 = c * W, d1 = d0 + half;
    if constexpr (kVec) {
        const u32x4r xa = *(const u32x4r *)(x + d0), xb = *(const u32x4r *)(x + d1);
        const u32x4r ca = *(const u32x4r *)(cs + d0), cb = *(const u32x4r *)(cs + d1);
        const u32x4r sa = *(const u32x4r *)(sn + d0), sb = *(const u32x4r *)(sn + d1);
        const uint16_t *xa_ = (const uint16_t *)&xa, *xb_ = (const uint16_t *)&xb;
        const uint16_t *ca_ = (const uint16_t *)&ca, *cb_ = (const uint16_t *)&cb;
        const uint16_t *sa_ = (const uint16_t *)&sa, *sb_ = (const uint16_t *)&sb;
        u32x4r oa, ob;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float a[2], bb[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int e = 2 * j + t;
                const float u = ld<kF16>(xa_[e]), w = ld<kF16>(xb_[e]);
                a[t] = __builtin_fmaf(u, ld<kF16>(ca_[e]), -w * ld<kF16>(sa_[e]));
                bb[t] = __builtin_fmaf(w, ld<kF16>(cb_[e]), u * ld<kF16>(sb_[e]));
            }
            asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(bb[0]), "+v"(bb[1]));  // fp32 step kept (above)
            oa[j] = pack2<kF16>(a[0], a[1]);
            ob[j] = pack2<kF16>(bb[0], bb[1]);
        }
        *(u32x4r *)(o + d0) = oa;
        *(u32x4r *)(o + d1) = ob;
    } else {
        const float u = ld<kF16>(x[d0]), w = ld<kF16>(x[d1]);
        float a = __builtin_fmaf(u, ld<kF16>(cs[d0]), -w * ld<kF16>(sn[d0]));
        float bb = __builtin_fmaf(w, ld<kF16>(cs[d1]), u * ld<kF16>(sn[d1]));
        // keep the fp32 rounding step: without the pin hipcc folds fptrunc(fma(fpext ..)) into one
        // mixed-precision fma rounded straight to fp16, which differs from the 16-B path on ties
        asm volatile("" : "+v"(a), "+v"(bb));
        o[d0] = st<kF16>(a);
        o[d1] = st<kF16>(bb);
    }
}

bool al16(const void *ptr) { return ((uintptr_t)ptr & 15) == 0; }

}  // namespace

int rope_check(const fa_rope_params *p, int dtype) {
    if (!p) return set_err(FA_ERR_INVALID_ARGUMENT, "params is NULL");
    if (dtype != FA_DTYPE_F16 && dtype != FA_DTYPE_BF16)
        return set_err(FA_ERR_UNSUPPORTED, "RoPE supports fp16 / bf16 only (dtype %d)", dtype);
    if (!p->x || !p->out || !p->cos || !p->sin) return set_err(FA_ERR_INVALID_ARGUMENT, "RoPE pointers must be non-NULL");
    if (p->batch_size < 0 || p->num_heads < 0 || p->seqlen < 0 || p->headdim <= 0 || (p->headdim & 1))
        return set_err(FA_ERR_INVALID_ARGUMENT, "RoPE needs non-negative sizes and an even head dim");
    return FA_OK;
}

int rope_launch(const fa_rope_params *p, int dtype, hipStream_t stream) {
    const int rc = rope_check(p, dtype);
    if (rc != FA_OK) return rc;
    const int64_t rows = p->batch_size * p->num_heads * p->seqlen;
    if (rows == 0) return FA_OK;
    // the 16-B path needs every chunk (and its partner half) 16-B aligned
    const int64_t st[8] = {p->x_batch_stride, p->x_head_stride, p->x_seqlen_stride, p->out_batch_stride,
                           p->out_head_stride, p->out_seqlen_stride, p->cs_batch_stride, p->cs_seqlen_stride};
    bool vec = p->headdim % 16 == 0 && al16(p->x) && al16(p->out) && al16(p->cos) && al16(p->sin);
    for (int i = 0; i < 8; ++i) vec = vec && st[i] % 8 == 0;
    const int64_t items = rows * (p->headdim / 2 / (vec ? 8 : 1));
    const dim3 grid((uint32_t)((items + 255) / 256));
    if (dtype == FA_DTYPE_F16) {
        if (vec) hipLaunchKernelGGL((fa_rope_kernel<true, true>), grid, dim3(256), 0, stream, *p, items);
        else hipLaunchKernelGGL((fa_rope_kernel<true, false>), grid, dim3(256), 0, stream, *p, items);
    } else {
        if (vec) hipLaunchKernelGGL((fa_rope_kernel<false, true>), grid, dim3(256), 0, stream, *p, items);
        else hipLaunchKernelGGL((fa_rope_kernel<false, false>), grid, dim3(256), 0, stream, *p, items);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_err(FA_ERR_LAUNCH, "HIP launch failed: %s", hipGetErrorString(e));
    return FA_OK;
}

}  // namespace fa

extern "C" int fa_rope_gfx950(const fa_rope_params *params, int dtype, void *stream) {
    return fa::rope_launch(params, dtype, (hipStream_t)stream);
}
