// flash_attention_api.cpp -- torch host API of the gfx950 FlashAttention-2 forward.
//
// Host-side mirror of reference csrc/flash_attention_api.cpp:14-141 (same function name, same
// argument meaning, same TORCH_CHECK messages, same decode q-head packing and stride-preserving
// output allocation). Differences, all MI355X-side:
//   * the compute-capability check (reference :17-19) becomes a gfx950 architecture check that is
//     cached per device instead of two device-attribute queries per call;
//   * the kernel is reached through the C-ABI of include/fa_gfx950.h (fa_fwd_gfx950), not a C++
//     template dispatch (reference csrc/kernel_dispatcher.h); runtime errors come back as a
//     RuntimeError instead of exit() (reference csrc/utils.h:9-18);
//   * inputs whose base pointer or strides are not 16-byte aligned (the reference silently assumes
//     alignment, csrc/flash_attention_template.cuh:135-137) are copied to a contiguous buffer.
#include <torch/extension.h>

#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <string>
#include <vector>

#include "fa_gfx950.h"

namespace flash_attention {

namespace {

bool device_is_gfx950(int device) {
    static std::mutex mu;
    static std::vector<int> cache;  // -1 unknown, 0 no, 1 yes
    std::lock_guard<std::mutex> lock(mu);
    if ((int)cache.size() <= device) cache.resize(device + 1, -1);
    if (cache[device] < 0) {
        hipDeviceProp_t prop;
        const hipError_t e = hipGetDeviceProperties(&prop, device);
        TORCH_CHECK(e == hipSuccess, "hipGetDeviceProperties failed: ", hipGetErrorString(e));
        cache[device] = std::string(prop.gcnArchName).rfind("gfx950", 0) == 0 ? 1 : 0;
    }
    return cache[device] == 1;
}

bool aligned16(const torch::Tensor &t) {
    if (reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 != 0) return false;
    for (int i = 0; i < 3; ++i)
        if (t.stride(i) % 8 != 0 && t.size(i) > 1) return false;
    return true;
}

int64_t stride_or_zero(const torch::Tensor &t, int dim) {
    // a size-1 dimension may carry any stride; the kernel never steps along it
    return t.size(dim) == 1 ? 0 : t.stride(dim);
}

// cos / sin tables of RoPE: [B, S, D], [1, S, D] or [S, D] of x's dtype on x's device; returns the
// table as [B', S, D] with 16-B aligned rows (B' = 1: shared by every batch row, batch stride 0)
torch::Tensor rope_table(const torch::Tensor &t, const torch::Tensor &x, int64_t batch, int64_t seqlen, int64_t dim,
                         const char *name) {
    TORCH_CHECK(t.dim() == 2 || t.dim() == 3, name, " must be [B, S, D] or [S, D]");
    torch::Tensor u = t.dim() == 2 ? t.unsqueeze(0) : t;
    TORCH_CHECK(u.size(0) == batch || u.size(0) == 1, name, " batch must be 1 or ", batch);
    TORCH_CHECK(u.size(1) == seqlen && u.size(2) == dim, name, " must cover ", seqlen, " positions x ", dim);
    TORCH_CHECK(u.dtype() == x.dtype(), name, " must have the dtype of q / k");
    TORCH_CHECK(u.device() == x.device(), name, " must be on the device of q / k");
    const bool ok = reinterpret_cast<uintptr_t>(u.data_ptr()) % 16 == 0 && u.stride(2) == 1 &&
                    (u.stride(1) % 8 == 0 || u.size(1) == 1) && (u.stride(0) % 8 == 0 || u.size(0) == 1);
    return ok ? u : u.contiguous();
}

fa_rope_params rope_params(const torch::Tensor &x, const torch::Tensor &out, const torch::Tensor &cs,
                           const torch::Tensor &sn) {
    fa_rope_params r;
    r.x = x.data_ptr();
    r.out = out.data_ptr();
    r.cos = cs.data_ptr();
    r.sin = sn.data_ptr();
    r.batch_size = x.size(0);
    r.num_heads = x.size(1);
    r.seqlen = x.size(2);
    r.headdim = x.size(3);
    r.x_batch_stride = x.stride(0);
    r.x_head_stride = x.stride(1);
    r.x_seqlen_stride = x.stride(2);
    r.out_batch_stride = out.stride(0);
    r.out_head_stride = out.stride(1);
    r.out_seqlen_stride = out.stride(2);
    r.cs_batch_stride = cs.size(0) == 1 ? 0 : cs.stride(0);
    r.cs_seqlen_stride = cs.stride(1);
    return r;
}

}  // namespace

// out = x * cos + rotate_half(x) * sin for x [B, H, S, D] (fp16 / bf16, last dim contiguous); out keeps
// x's strides (HF's [B, S, H, D] projection views stay copy-free). One HIP pass (csrc/fa_rope.hip).
torch::Tensor rope_apply(torch::Tensor &x, torch::Tensor &cos, torch::Tensor &sin) {
    TORCH_CHECK(x.dim() == 4, "x must be 4-D [batch, heads, seqlen, dim]");
    TORCH_CHECK(x.dtype() == torch::kHalf || x.dtype() == torch::kBFloat16, "RoPE supports fp16 or bf16");
    TORCH_CHECK(x.is_cuda(), "x must be on CUDA device");
    TORCH_CHECK(x.stride(3) == 1, "x must be contiguous in the last dimension");
    TORCH_CHECK(x.size(3) % 2 == 0, "RoPE needs an even head dimension");
    c10::DeviceGuard device_guard(x.device());
    torch::Tensor cs = rope_table(cos, x, x.size(0), x.size(2), x.size(3), "cos");
    torch::Tensor sn = rope_table(sin, x, x.size(0), x.size(2), x.size(3), "sin");
    TORCH_CHECK(cs.size(0) == sn.size(0) && cs.strides() == sn.strides(), "cos and sin must have the same layout");
    auto out = torch::empty_like(x);
    if (x.numel() == 0) return out;
    const fa_rope_params r = rope_params(x, out, cs, sn);
    const int dtype = x.scalar_type() == torch::kHalf ? FA_DTYPE_F16 : FA_DTYPE_BF16;
    const int rc = fa_rope_gfx950(&r, dtype, c10::hip::getCurrentHIPStream(x.device().index()).stream());
    TORCH_CHECK(rc == FA_OK, "fa_rope_gfx950 failed (code ", rc, "): ", fa_last_error());
    return out;
}

// window_left >= 0 (flash_attention_window_fwd, after its cut): the local-window entry, no pack
torch::Tensor fwd_impl(torch::Tensor &q, torch::Tensor &k, torch::Tensor &v, float softmax_scale, bool causal,
                       int64_t window_left) {
    // Check input shape (reference :21-37)
    TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "q, k, v must be 4-D [batch, heads, seqlen, dim]");
    TORCH_CHECK(q.size(0) == k.size(0) && q.size(0) == v.size(0), "q, k, v must have the same batch size");
    TORCH_CHECK(k.size(1) == v.size(1), "k, v must have the same number of heads");
    TORCH_CHECK(k.size(2) == v.size(2), "k, v must have the same sequence length");
    TORCH_CHECK(q.size(3) == k.size(3) && q.size(3) == v.size(3), "q, k, v must have the same hidden dimension");
    TORCH_CHECK(q.size(0) > 0 && q.size(1) > 0 && q.size(2) > 0 && q.size(3) > 0,
                "q, k, v must have at least one element");
    TORCH_CHECK(k.size(2) > 0, "q, k, v must have at least one element");
    TORCH_CHECK(q.size(1) >= k.size(1),
                "number of heads in q must be greater or equal to number of heads in k and v");
    TORCH_CHECK(q.size(1) % k.size(1) == 0, "number of heads in q must be multiple of number of heads in k and v");

    // Check input data type (reference :39-43)
    TORCH_CHECK(q.dtype() == k.dtype() && q.dtype() == v.dtype(), "q, k, v must have the same data type");
    TORCH_CHECK(q.dtype() == torch::kHalf || q.dtype() == torch::kBFloat16,
                "q, k, v only support fp16 or bf16 data type");

    // Check input memory contiguity (reference :45-51)
    TORCH_CHECK(q.stride(3) == 1, "q must be contiguous in the last dimension");
    TORCH_CHECK(k.stride(3) == 1, "k must be contiguous in the last dimension");
    TORCH_CHECK(v.stride(3) == 1, "v must be contiguous in the last dimension");

    // Check kernel constraints (reference :53-59)
    TORCH_CHECK(q.size(3) % 8 == 0, "hidden dimension must be multiple of 8");
    TORCH_CHECK(q.size(3) <= 128, "only support hidden dimension <= 128");
    TORCH_CHECK(q.is_cuda() && k.is_cuda() && v.is_cuda(), "q, k, v must be on CUDA device");
    TORCH_CHECK(q.device() == k.device() && q.device() == v.device(), "q, k, v must be on the same CUDA device");

    c10::DeviceGuard device_guard(q.device());
    TORCH_CHECK(device_is_gfx950(q.device().index()),
                "flash attention (gfx950 build) is only supported on MI355X / gfx950 devices");

    torch::Tensor qx = aligned16(q) ? q : q.contiguous();
    torch::Tensor kx = aligned16(k) ? k : k.contiguous();
    torch::Tensor vx = aligned16(v) ? v : v.contiguous();

    int64_t bs = qx.size(0);
    int64_t head_q = qx.size(1);
    const int64_t head_kv = kx.size(1);
    int64_t seqlen_q = qx.size(2);
    const int64_t seqlen_kv = kx.size(2);
    const int64_t headdim = qx.size(3);
    const int64_t head_q_per_group = head_q / head_kv;

    // Decode q-head packing (reference :64-83): with one query row per head, the q-heads of one
    // kv group become the rows of a single (batch, kv-head) problem so one workgroup serves the
    // whole group from one K/V stream. Causal masking is dropped, as in the reference (:81).
    const bool is_pack_head_q = seqlen_q == 1 && window_left < 0;
    if (is_pack_head_q) {
        head_q = head_kv;
        seqlen_q = seqlen_q * head_q_per_group;
        causal = false;
        qx = qx.reshape({bs, head_q, seqlen_q, headdim});
        if (!aligned16(qx)) qx = qx.contiguous();
    }

    // stride-preserving output (reference :85): o inherits q's physical layout, so the
    // transpose(1, 2).reshape(...) of the HF attention caller stays copy-free
    auto o = torch::empty_like(qx);
    if (!aligned16(o)) o = torch::empty(qx.sizes(), qx.options());

    fa_fwd_params params;
    params.q_ptr = qx.data_ptr();
    params.k_ptr = kx.data_ptr();
    params.v_ptr = vx.data_ptr();
    params.o_ptr = o.data_ptr();
    params.batch_size = bs;
    params.num_heads_q = head_q;
    params.num_heads_kv = head_kv;
    params.seqlen_q = seqlen_q;
    params.seqlen_kv = seqlen_kv;
    params.headdim = headdim;
    // pack path runs as MHA over the packed rows (reference :100)
    params.head_q_per_group = is_pack_head_q ? 1 : head_q_per_group;
    params.q_batch_stride = stride_or_zero(qx, 0);
    params.k_batch_stride = stride_or_zero(kx, 0);
    params.v_batch_stride = stride_or_zero(vx, 0);
    params.o_batch_stride = stride_or_zero(o, 0);
    params.q_head_stride = stride_or_zero(qx, 1);
    params.k_head_stride = stride_or_zero(kx, 1);
    params.v_head_stride = stride_or_zero(vx, 1);
    params.o_head_stride = stride_or_zero(o, 1);
    params.q_seqlen_stride = stride_or_zero(qx, 2);
    params.k_seqlen_stride = stride_or_zero(kx, 2);
    params.v_seqlen_stride = stride_or_zero(vx, 2);
    params.o_seqlen_stride = stride_or_zero(o, 2);
    // log2(e) folded into the scale on the host (reference :87)
    // (float * double -> float, exactly as `softmax_scale *= M_LOG2E` there)
    softmax_scale *= M_LOG2E;
    params.softmax_scale = softmax_scale;

    const int dtype = qx.scalar_type() == torch::kHalf ? FA_DTYPE_F16 : FA_DTYPE_BF16;
    void *stream = c10::hip::getCurrentHIPStream(qx.device().index()).stream();
    if (window_left >= 0) {
        const int rc = fa_fwd_gfx950_window(&params, dtype, causal ? 1 : 0, window_left, stream);
        TORCH_CHECK(rc == FA_OK, "fa_fwd_gfx950_window failed (code ", rc, "): ", fa_last_error());
        if (o.sizes() != q.sizes()) o = o.reshape(q.sizes());
        return o;
    }
    // split-KV decode (few rows per kv-head) wants fp32 scratch for its partials: taken from
    // torch's caching allocator on the current stream, so it is graph-capture safe and reused
    const int64_t ws_bytes = fa_fwd_gfx950_workspace_size(&params, dtype, causal ? 1 : 0);
    TORCH_CHECK(ws_bytes >= 0, "fa_fwd_gfx950_workspace_size failed: ", fa_last_error());
    torch::Tensor ws;
    if (ws_bytes > 0) ws = torch::empty({ws_bytes}, qx.options().dtype(torch::kUInt8));
    const int rc = fa_fwd_gfx950_ws(&params, dtype, causal ? 1 : 0, ws_bytes > 0 ? ws.data_ptr() : nullptr,
                                    ws_bytes, stream);
    TORCH_CHECK(rc == FA_OK, "fa_fwd_gfx950_ws failed (code ", rc, "): ", fa_last_error());

    if (is_pack_head_q) {
        head_q = head_kv * head_q_per_group;
        seqlen_q = seqlen_q / head_q_per_group;
        o = o.reshape({bs, head_q, seqlen_q, headdim});
    }
    if (o.sizes() != q.sizes()) o = o.reshape(q.sizes());
    return o;
}

torch::Tensor flash_attention_fwd(torch::Tensor &q, torch::Tensor &k, torch::Tensor &v, float softmax_scale,
                                  bool causal) {
    return fwd_impl(q, k, v, softmax_scale, causal, -1);
}

// Local (sliding-window) attention, include/fa_gfx950.h fa_fwd_gfx950_window: key n visible to query
// m iff n >= m + Sk - Sq - window_left (and, causal, n <= m + Sk - Sq). The keys left of every row's
// window are cut off here as views of k / v; when the window masks nothing more (decode: Sq == 1)
// the plain forward runs on the rest (q-head pack and split-KV decode included).
torch::Tensor flash_attention_window_fwd(torch::Tensor &q, torch::Tensor &k, torch::Tensor &v, int64_t window_left,
                                         float softmax_scale, bool causal) {
    TORCH_CHECK(window_left >= 0, "window_left must be >= 0");
    TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "q, k, v must be 4-D [batch, heads, seqlen, dim]");
    TORCH_CHECK(k.size(2) == v.size(2), "k, v must have the same sequence length");
    const int64_t sq = q.size(2), sk = k.size(2);
    const int64_t cut = sk - sq - window_left;
    torch::Tensor kc = cut > 0 ? k.narrow(2, cut, sk - cut) : k;
    torch::Tensor vc = cut > 0 ? v.narrow(2, cut, sk - cut) : v;
    if (kc.size(2) - 1 <= window_left) return fwd_impl(q, kc, vc, softmax_scale, causal, -1);
    return fwd_impl(q, kc, vc, softmax_scale, causal, window_left);
}

// Attention with RoPE applied to q inside the kernel's Q load (fa_fwd_gfx950_rope); k is already
// rotated. Query blocks the split-KV decode kernel serves (Sq == 1 pack, g * Sq <= 64) and other head
// dims rotate q with rope_apply first and take the plain path.
torch::Tensor flash_attention_rope_fwd(torch::Tensor &q, torch::Tensor &k, torch::Tensor &v, torch::Tensor &cos,
                                       torch::Tensor &sin, float softmax_scale, bool causal) {
    TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "q, k, v must be 4-D [batch, heads, seqlen, dim]");
    TORCH_CHECK(k.size(1) > 0 && q.size(1) % k.size(1) == 0,
                "number of heads in q must be multiple of number of heads in k and v");
    const int64_t g = q.size(1) / k.size(1), sq = q.size(2), d = q.size(3);
    const bool fused = (d == 64 || d == 128) && sq > 1 && g * sq > 64 && q.is_cuda() && q.stride(3) == 1 &&
                       (q.dtype() == torch::kHalf || q.dtype() == torch::kBFloat16);
    if (!fused) {
        torch::Tensor qr = rope_apply(q, cos, sin);
        return flash_attention_fwd(qr, k, v, softmax_scale, causal);
    }
    // the checks of flash_attention_fwd on a dry run of the same tensors (no Sq == 1 pack here)
    TORCH_CHECK(q.size(0) == k.size(0) && q.size(0) == v.size(0), "q, k, v must have the same batch size");
    TORCH_CHECK(k.size(1) == v.size(1), "k, v must have the same number of heads");
    TORCH_CHECK(k.size(2) == v.size(2), "k, v must have the same sequence length");
    TORCH_CHECK(q.size(3) == k.size(3) && q.size(3) == v.size(3), "q, k, v must have the same hidden dimension");
    TORCH_CHECK(k.size(2) > 0 && q.size(0) > 0, "q, k, v must have at least one element");
    TORCH_CHECK(q.dtype() == k.dtype() && q.dtype() == v.dtype(), "q, k, v must have the same data type");
    TORCH_CHECK(k.stride(3) == 1 && v.stride(3) == 1, "k, v must be contiguous in the last dimension");
    TORCH_CHECK(k.is_cuda() && v.is_cuda() && q.device() == k.device() && q.device() == v.device(),
                "q, k, v must be on the same CUDA device");
    c10::DeviceGuard device_guard(q.device());
    TORCH_CHECK(device_is_gfx950(q.device().index()),
                "flash attention (gfx950 build) is only supported on MI355X / gfx950 devices");
    torch::Tensor cs = rope_table(cos, q, q.size(0), sq, d, "cos");
    torch::Tensor sn = rope_table(sin, q, q.size(0), sq, d, "sin");
    TORCH_CHECK(cs.size(0) == sn.size(0) && cs.strides() == sn.strides(), "cos and sin must have the same layout");
    torch::Tensor qx = aligned16(q) ? q : q.contiguous();
    torch::Tensor kx = aligned16(k) ? k : k.contiguous();
    torch::Tensor vx = aligned16(v) ? v : v.contiguous();
    auto o = torch::empty_like(qx);
    if (!aligned16(o)) o = torch::empty(qx.sizes(), qx.options());

    fa_rope_fwd_params rp;
    fa_fwd_params &params = rp.base;
    params.q_ptr = qx.data_ptr();
    params.k_ptr = kx.data_ptr();
    params.v_ptr = vx.data_ptr();
    params.o_ptr = o.data_ptr();
    params.batch_size = qx.size(0);
    params.num_heads_q = qx.size(1);
    params.num_heads_kv = kx.size(1);
    params.seqlen_q = sq;
    params.seqlen_kv = kx.size(2);
    params.headdim = d;
    params.head_q_per_group = g;
    params.q_batch_stride = stride_or_zero(qx, 0);
    params.k_batch_stride = stride_or_zero(kx, 0);
    params.v_batch_stride = stride_or_zero(vx, 0);
    params.o_batch_stride = stride_or_zero(o, 0);
    params.q_head_stride = stride_or_zero(qx, 1);
    params.k_head_stride = stride_or_zero(kx, 1);
    params.v_head_stride = stride_or_zero(vx, 1);
    params.o_head_stride = stride_or_zero(o, 1);
    params.q_seqlen_stride = stride_or_zero(qx, 2);
    params.k_seqlen_stride = stride_or_zero(kx, 2);
    params.v_seqlen_stride = stride_or_zero(vx, 2);
    params.o_seqlen_stride = stride_or_zero(o, 2);
    softmax_scale *= M_LOG2E;
    params.softmax_scale = softmax_scale;
    rp.rope_cos = cs.data_ptr();
    rp.rope_sin = sn.data_ptr();
    rp.rope_batch_stride = cs.size(0) == 1 ? 0 : cs.stride(0);
    rp.rope_seqlen_stride = cs.stride(1);
    const int dtype = qx.scalar_type() == torch::kHalf ? FA_DTYPE_F16 : FA_DTYPE_BF16;
    const int rc = fa_fwd_gfx950_rope(&rp, dtype, causal ? 1 : 0,
                                      c10::hip::getCurrentHIPStream(qx.device().index()).stream());
    TORCH_CHECK(rc == FA_OK, "fa_fwd_gfx950_rope failed (code ", rc, "): ", fa_last_error());
    if (o.sizes() != q.sizes()) o = o.reshape(q.sizes());
    return o;
}

// Variable-length (packed) batches: q [total_q, Hq, D], k / v [total_k, Hkv, D], cu_seqlens_* int32
// [B + 1] on the device (include/fa_gfx950.h fa_fwd_gfx950_varlen). No reference counterpart
// (varlen is a TODO at reference README.md:18); the checks follow flash_attention_fwd's.
torch::Tensor flash_attention_varlen_fwd(torch::Tensor &q, torch::Tensor &k, torch::Tensor &v,
                                         torch::Tensor &cu_seqlens_q, torch::Tensor &cu_seqlens_k,
                                         int64_t max_seqlen_q, int64_t max_seqlen_k, float softmax_scale,
                                         bool causal, int64_t window_left) {
    TORCH_CHECK(q.dim() == 3 && k.dim() == 3 && v.dim() == 3, "varlen q, k, v must be 3-D [total, heads, dim]");
    TORCH_CHECK(k.size(0) == v.size(0), "k, v must have the same number of rows");
    TORCH_CHECK(k.size(1) == v.size(1), "k, v must have the same number of heads");
    TORCH_CHECK(q.size(2) == k.size(2) && q.size(2) == v.size(2), "q, k, v must have the same hidden dimension");
    TORCH_CHECK(q.size(1) > 0 && k.size(1) > 0 && q.size(2) > 0, "q, k, v must have at least one head");
    TORCH_CHECK(q.size(1) % k.size(1) == 0, "number of heads in q must be multiple of number of heads in k and v");
    TORCH_CHECK(q.dtype() == k.dtype() && q.dtype() == v.dtype(), "q, k, v must have the same data type");
    TORCH_CHECK(q.dtype() == torch::kHalf || q.dtype() == torch::kBFloat16,
                "q, k, v only support fp16 or bf16 data type");
    TORCH_CHECK(q.stride(2) == 1 && k.stride(2) == 1 && v.stride(2) == 1,
                "q, k, v must be contiguous in the last dimension");
    TORCH_CHECK(q.size(2) % 8 == 0, "hidden dimension must be multiple of 8");
    TORCH_CHECK(q.size(2) <= 128, "only support hidden dimension <= 128");
    TORCH_CHECK(q.is_cuda() && k.is_cuda() && v.is_cuda(), "q, k, v must be on CUDA device");
    TORCH_CHECK(q.device() == k.device() && q.device() == v.device(), "q, k, v must be on the same CUDA device");
    TORCH_CHECK(cu_seqlens_q.dtype() == torch::kInt32 && cu_seqlens_k.dtype() == torch::kInt32,
                "cu_seqlens must be int32");
    TORCH_CHECK(cu_seqlens_q.dim() == 1 && cu_seqlens_k.dim() == 1 && cu_seqlens_q.size(0) == cu_seqlens_k.size(0) &&
                    cu_seqlens_q.size(0) >= 2,
                "cu_seqlens_q and cu_seqlens_k must be 1-D with batch_size + 1 entries");
    TORCH_CHECK(cu_seqlens_q.device() == q.device() && cu_seqlens_k.device() == q.device(),
                "cu_seqlens must be on the same device as q");
    TORCH_CHECK(max_seqlen_q >= 0 && max_seqlen_k >= 0, "max_seqlen must be non-negative");

    c10::DeviceGuard device_guard(q.device());
    TORCH_CHECK(device_is_gfx950(q.device().index()),
                "flash attention (gfx950 build) is only supported on MI355X / gfx950 devices");
    auto o = torch::empty_like(q);
    if (q.size(0) == 0 || max_seqlen_q == 0) return o;
    if (max_seqlen_k == 0) return o.zero_();  // no sequence has a key: every row is 0

    auto aligned_rows = [](const torch::Tensor &t) {
        return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && (t.stride(0) % 8 == 0 || t.size(0) <= 1) &&
               (t.stride(1) % 8 == 0 || t.size(1) <= 1);
    };
    torch::Tensor qx = aligned_rows(q) ? q : q.contiguous();
    torch::Tensor kx = aligned_rows(k) ? k : k.contiguous();
    torch::Tensor vx = aligned_rows(v) ? v : v.contiguous();
    if (!aligned_rows(o)) o = torch::empty(q.sizes(), q.options());
    torch::Tensor cq = cu_seqlens_q.contiguous(), ck = cu_seqlens_k.contiguous();

    fa_varlen_params vp;
    fa_fwd_params &params = vp.base;
    params.q_ptr = qx.data_ptr();
    params.k_ptr = kx.data_ptr();
    params.v_ptr = vx.data_ptr();
    params.o_ptr = o.data_ptr();
    params.batch_size = cq.size(0) - 1;
    params.num_heads_q = qx.size(1);
    params.num_heads_kv = kx.size(1);
    params.seqlen_q = max_seqlen_q;
    params.seqlen_kv = max_seqlen_k;
    params.headdim = qx.size(2);
    params.head_q_per_group = qx.size(1) / kx.size(1);
    params.q_batch_stride = params.k_batch_stride = params.v_batch_stride = params.o_batch_stride = 0;
    params.q_head_stride = qx.stride(1);
    params.k_head_stride = kx.stride(1);
    params.v_head_stride = vx.stride(1);
    params.o_head_stride = o.stride(1);
    params.q_seqlen_stride = qx.stride(0);
    params.k_seqlen_stride = kx.stride(0);
    params.v_seqlen_stride = vx.stride(0);
    params.o_seqlen_stride = o.stride(0);
    softmax_scale *= M_LOG2E;
    params.softmax_scale = softmax_scale;
    vp.cu_seqlens_q = cq.data_ptr<int32_t>();
    vp.cu_seqlens_k = ck.data_ptr<int32_t>();

    const int dtype = qx.scalar_type() == torch::kHalf ? FA_DTYPE_F16 : FA_DTYPE_BF16;
    void *stream = c10::hip::getCurrentHIPStream(qx.device().index()).stream();
    const int rc = window_left >= 0 ? fa_fwd_gfx950_varlen_window(&vp, dtype, causal ? 1 : 0, window_left, stream)
                                    : fa_fwd_gfx950_varlen(&vp, dtype, causal ? 1 : 0, stream);
    TORCH_CHECK(rc == FA_OK, "fa_fwd_gfx950_varlen failed (code ", rc, "): ", fa_last_error());
    return o;
}

// Padded batches (include/fa_gfx950.h fa_fwd_gfx950_padded): dense q [B, Hq, Sq, D], k / v
// [B, Hkv, Sk, D] (any strides, last dim contiguous) with the real tokens of batch row b at key
// positions [k_start[b], k_end[b]) and, optionally, query positions [q_start[b], q_end[b]) -- int32
// [B] on the device. Read in place: no packing copy, no host synchronisation (graph-capturable).
// Output rows outside the query ranges are 0. Sq == 1 without query ranges takes the q-head pack
// and the split-KV decode kernel over each sequence's key range (a window there narrows the key
// range on the device instead). No reference counterpart (the reference drops attention_mask).
torch::Tensor flash_attention_padded_fwd(torch::Tensor &q, torch::Tensor &k, torch::Tensor &v,
                                         c10::optional<torch::Tensor> q_start, c10::optional<torch::Tensor> q_end,
                                         torch::Tensor &k_start, torch::Tensor &k_end, float softmax_scale,
                                         bool causal, int64_t window_left) {
    TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "q, k, v must be 4-D [batch, heads, seqlen, dim]");
    TORCH_CHECK(q.size(0) == k.size(0) && q.size(0) == v.size(0), "q, k, v must have the same batch size");
    TORCH_CHECK(k.size(1) == v.size(1), "k, v must have the same number of heads");
    TORCH_CHECK(k.size(2) == v.size(2), "k, v must have the same sequence length");
    TORCH_CHECK(q.size(3) == k.size(3) && q.size(3) == v.size(3), "q, k, v must have the same hidden dimension");
    TORCH_CHECK(q.size(0) > 0 && q.size(1) > 0 && q.size(2) > 0 && q.size(3) > 0 && k.size(2) > 0,
                "q, k, v must have at least one element");
    TORCH_CHECK(q.size(1) % k.size(1) == 0, "number of heads in q must be multiple of number of heads in k and v");
    TORCH_CHECK(q.dtype() == k.dtype() && q.dtype() == v.dtype(), "q, k, v must have the same data type");
    TORCH_CHECK(q.dtype() == torch::kHalf || q.dtype() == torch::kBFloat16,
                "q, k, v only support fp16 or bf16 data type");
    TORCH_CHECK(q.stride(3) == 1 && k.stride(3) == 1 && v.stride(3) == 1,
                "q, k, v must be contiguous in the last dimension");
    TORCH_CHECK(q.size(3) % 8 == 0, "hidden dimension must be multiple of 8");
    TORCH_CHECK(q.size(3) <= 128, "only support hidden dimension <= 128");
    TORCH_CHECK(q.is_cuda() && k.is_cuda() && v.is_cuda(), "q, k, v must be on CUDA device");
    TORCH_CHECK(q.device() == k.device() && q.device() == v.device(), "q, k, v must be on the same CUDA device");
    TORCH_CHECK(q_start.has_value() == q_end.has_value(), "q_start and q_end must be given together");
    const int64_t bs = q.size(0);
    auto check_range = [&](const torch::Tensor &t, const char *name) {
        TORCH_CHECK(t.dtype() == torch::kInt32 && t.dim() == 1 && t.size(0) == bs, name, " must be int32 [batch]");
        TORCH_CHECK(t.device() == q.device(), name, " must be on the device of q");
    };
    check_range(k_start, "k_start");
    check_range(k_end, "k_end");
    const bool q_ranges = q_start.has_value();
    if (q_ranges) {
        check_range(*q_start, "q_start");
        check_range(*q_end, "q_end");
    }
    c10::DeviceGuard device_guard(q.device());
    TORCH_CHECK(device_is_gfx950(q.device().index()),
                "flash attention (gfx950 build) is only supported on MI355X / gfx950 devices");

    // the prefill kernel addresses a ranged sequence by absolute rows (row r at base + r * seqlen
    // stride): the batch stride must be a multiple of the seqlen stride, the same multiple for k and v
    // (q and o) -- other layouts are copied to a contiguous buffer
    auto rows_per_batch = [](const torch::Tensor &t) -> int64_t {
        if (t.size(0) == 1) return 0;
        if (t.stride(2) <= 0 || t.stride(0) % t.stride(2) != 0) return -1;
        return t.stride(0) / t.stride(2);
    };
    torch::Tensor qx = aligned16(q) ? q : q.contiguous();
    torch::Tensor kx = aligned16(k) ? k : k.contiguous();
    torch::Tensor vx = aligned16(v) ? v : v.contiguous();
    if (rows_per_batch(kx) < 0 || rows_per_batch(kx) != rows_per_batch(vx) || kx.stride(2) != vx.stride(2)) {
        kx = kx.contiguous();
        vx = vx.contiguous();
    }
    int64_t head_q = qx.size(1), seqlen_q = qx.size(2);
    const int64_t head_kv = kx.size(1), headdim = qx.size(3), g = head_q / head_kv;
    torch::Tensor ks = k_start.contiguous(), ke = k_end.contiguous(), qs, qe;
    if (q_ranges) {
        qs = q_start->contiguous();
        qe = q_end->contiguous();
    }
    // decode: one query row that sees the last window_left + 1 keys of its range -> narrow the range
    if (window_left >= 0 && seqlen_q == 1 && !q_ranges) {
        ks = torch::maximum(ks, ke - (int32_t)std::min<int64_t>(window_left + 1, 0x7fffffff));
        window_left = -1;
    }
    // Sq == 1: the q-head pack of flash_attention_fwd (reference :64-83)
    const bool pack = seqlen_q == 1 && !q_ranges && window_left < 0;
    if (pack) {
        head_q = head_kv;
        seqlen_q = g;
        causal = false;
        qx = qx.reshape({bs, head_q, seqlen_q, headdim});
        if (!aligned16(qx)) qx = qx.contiguous();
    }
    if (rows_per_batch(qx) < 0) qx = qx.contiguous();  // (the prefill path may run, also after a pack)
    auto o = torch::empty_like(qx);
    if (!aligned16(o) || o.strides() != qx.strides()) o = torch::empty(qx.sizes(), qx.options());
    // the prefill kernel addresses q and o rows with ONE rows-per-batch multiple: a q that is not
    // dense (a seqlen slice of a longer buffer, a view cut from a wider tensor) leaves empty_like with
    // a contiguous o, so q is made contiguous too
    if (rows_per_batch(o) != rows_per_batch(qx)) {
        qx = qx.contiguous();
        o = torch::empty(qx.sizes(), qx.options());
    }
    if (q_ranges) o.zero_();  // rows outside the query ranges are not written by the kernel

    fa_padded_params pp;
    fa_fwd_params &params = pp.base;
    params.q_ptr = qx.data_ptr();
    params.k_ptr = kx.data_ptr();
    params.v_ptr = vx.data_ptr();
    params.o_ptr = o.data_ptr();
    params.batch_size = bs;
    params.num_heads_q = head_q;
    params.num_heads_kv = head_kv;
    params.seqlen_q = seqlen_q;
    params.seqlen_kv = kx.size(2);
    params.headdim = headdim;
    params.head_q_per_group = pack ? 1 : g;
    params.q_batch_stride = stride_or_zero(qx, 0);
    params.k_batch_stride = stride_or_zero(kx, 0);
    params.v_batch_stride = stride_or_zero(vx, 0);
    params.o_batch_stride = stride_or_zero(o, 0);
    params.q_head_stride = stride_or_zero(qx, 1);
    params.k_head_stride = stride_or_zero(kx, 1);
    params.v_head_stride = stride_or_zero(vx, 1);
    params.o_head_stride = stride_or_zero(o, 1);
    // the seqlen strides convert rows into addresses on the prefill path, even at size 1
    params.q_seqlen_stride = pack ? stride_or_zero(qx, 2) : qx.stride(2);
    params.k_seqlen_stride = kx.stride(2);
    params.v_seqlen_stride = vx.stride(2);
    params.o_seqlen_stride = pack ? stride_or_zero(o, 2) : o.stride(2);
    softmax_scale *= M_LOG2E;
    params.softmax_scale = softmax_scale;
    pp.q_start = q_ranges ? qs.data_ptr<int32_t>() : nullptr;
    pp.q_end = q_ranges ? qe.data_ptr<int32_t>() : nullptr;
    pp.k_start = ks.data_ptr<int32_t>();
    pp.k_end = ke.data_ptr<int32_t>();

    const int dtype = qx.scalar_type() == torch::kHalf ? FA_DTYPE_F16 : FA_DTYPE_BF16;
    void *stream = c10::hip::getCurrentHIPStream(qx.device().index()).stream();
    const int64_t ws_bytes = fa_fwd_gfx950_padded_workspace_size(&pp, dtype, causal ? 1 : 0, window_left);
    TORCH_CHECK(ws_bytes >= 0, "fa_fwd_gfx950_padded_workspace_size failed: ", fa_last_error());
    torch::Tensor ws;
    if (ws_bytes > 0) ws = torch::empty({ws_bytes}, qx.options().dtype(torch::kUInt8));
    const int rc = fa_fwd_gfx950_padded(&pp, dtype, causal ? 1 : 0, window_left,
                                        ws_bytes > 0 ? ws.data_ptr() : nullptr, ws_bytes, stream);
    TORCH_CHECK(rc == FA_OK, "fa_fwd_gfx950_padded failed (code ", rc, "): ", fa_last_error());
    if (o.sizes() != q.sizes()) o = o.reshape(q.sizes());
    return o;
}

}  // namespace flash_attention

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.def("flash_attention_fwd", &flash_attention::flash_attention_fwd,
          "FlashAttention-2 forward, hand-written HIP kernel for MI355X / gfx950");
    m.def("flash_attention_varlen_fwd", &flash_attention::flash_attention_varlen_fwd,
          "FlashAttention-2 forward over packed variable-length sequences (cu_seqlens), gfx950");
    m.def("flash_attention_rope_fwd", &flash_attention::flash_attention_rope_fwd,
          "FlashAttention-2 forward with rotate-half RoPE applied to q in the kernel's Q load, gfx950");
    m.def("flash_attention_window_fwd", &flash_attention::flash_attention_window_fwd,
          "FlashAttention-2 forward with a local (sliding) window of window_left + 1 keys, gfx950");
    m.def("flash_attention_padded_fwd", &flash_attention::flash_attention_padded_fwd,
          "FlashAttention-2 forward over padded batches (per-sequence query / key ranges in dense tensors), gfx950");
    m.def("rope_apply", &flash_attention::rope_apply, "rotate-half RoPE, one HIP pass (gfx950)");
    m.def("abi_version", []() { return fa_abi_version(); });
}
