// Host-side validation of the C-ABI (include/fa_gfx950.h) under AddressSanitizer + UBSan
// (tests/test_abi.py::test_host_validation_under_asan_ubsan builds and runs it; CPU only). Every entry
// point is called with valid and invalid parameters -- NULLs, zero / negative / huge sizes, odd
// strides, misaligned pointers, mismatched ranges -- and must return the right code with no
// sanitizer report. Launches that pass validation reach the host-only stub instantiations
// (stub_instances.hip), never a device.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "fa_gfx950.h"

static int failures = 0;
#define EXPECT(cond)                                                          \
    do {                                                                      \
        if (!(cond)) {                                                        \
            fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond, fa_last_error()); \
            ++failures;                                                       \
        }                                                                     \
    } while (0)

static fa_fwd_params good(int64_t b, int64_t hq, int64_t hkv, int64_t sq, int64_t sk, int64_t d) {
    fa_fwd_params p;
    memset(&p, 0, sizeof(p));
    p.q_ptr = (const void *)0x10000;
    p.k_ptr = (const void *)0x20000;
    p.v_ptr = (const void *)0x30000;
    p.o_ptr = (void *)0x40000;
    p.batch_size = b;
    p.num_heads_q = hq;
    p.num_heads_kv = hkv;
    p.seqlen_q = sq;
    p.seqlen_kv = sk;
    p.headdim = d;
    p.head_q_per_group = hq / hkv;
    p.q_batch_stride = p.o_batch_stride = hq * sq * d;
    p.k_batch_stride = p.v_batch_stride = hkv * sk * d;
    p.q_head_stride = p.o_head_stride = sq * d;
    p.k_head_stride = p.v_head_stride = sk * d;
    p.q_seqlen_stride = p.k_seqlen_stride = p.v_seqlen_stride = p.o_seqlen_stride = d;
    p.softmax_scale = 0.1275f;
    return p;
}

int main() {
    EXPECT(fa_abi_version() == FA_GFX950_ABI_VERSION);
    fa_fwd_params p = good(2, 8, 2, 300, 300, 128);
    EXPECT(fa_fwd_gfx950_check(&p, FA_DTYPE_F16, 0) == FA_OK);
    EXPECT(fa_fwd_gfx950_check(NULL, FA_DTYPE_F16, 0) == FA_ERR_INVALID_ARGUMENT);
    EXPECT(fa_fwd_gfx950_check(&p, 7, 0) == FA_ERR_UNSUPPORTED);
    // every single-field violation: the right code, a message, no out-of-bounds access
    struct Case { int field; int64_t value; int code; } cases[] = {
        {0, 100, FA_ERR_INVALID_ARGUMENT},      // headdim not a multiple of 8
        {0, 136, FA_ERR_UNSUPPORTED},           // headdim > 128
        {0, 0, FA_ERR_INVALID_ARGUMENT},        // empty
        {0, -8, FA_ERR_INVALID_ARGUMENT},
        {1, 3, FA_ERR_INVALID_ARGUMENT},        // group does not divide
        {2, 0, FA_ERR_INVALID_ARGUMENT},        // seqlen_kv 0
        {3, INT64_C(1) << 40, FA_ERR_UNSUPPORTED},  // seqlen_q past 2^30
        {4, 132, FA_ERR_INVALID_ARGUMENT},      // stride not a multiple of 8
        {5, -128, FA_ERR_UNSUPPORTED},          // negative seqlen stride
        {5, INT64_C(1) << 33, FA_ERR_UNSUPPORTED},  // 32-bit tile offsets overflow
        {6, INT64_C(1) << 40, FA_ERR_UNSUPPORTED},  // grid too large
    };
    for (size_t i = 0; i < sizeof(cases) / sizeof(cases[0]); ++i) {
        fa_fwd_params b = good(2, 8, 2, 300, 300, 128);
        switch (cases[i].field) {
            case 0: b.headdim = cases[i].value; break;
            case 1: b.head_q_per_group = cases[i].value; break;
            case 2: b.seqlen_kv = cases[i].value; break;
            case 3: b.seqlen_q = cases[i].value; break;
            case 4: b.k_seqlen_stride = cases[i].value; break;
            case 5: b.k_seqlen_stride = cases[i].value; break;
            case 6: b.batch_size = cases[i].value; b.num_heads_q = 1 << 20; b.num_heads_kv = 1 << 20; b.head_q_per_group = 1; break;
        }
        const int rc = fa_fwd_gfx950_check(&b, FA_DTYPE_BF16, 1);
        if (rc != cases[i].code) fprintf(stderr, "case %zu: rc %d\n", i, rc);
        EXPECT(rc == cases[i].code);
        EXPECT(strlen(fa_last_error()) > 0 && strlen(fa_last_error()) < 512);
        // the launch entries validate before touching the device
        EXPECT(fa_fwd_gfx950(&b, FA_DTYPE_BF16, 1, NULL) == cases[i].code);
        EXPECT(fa_fwd_gfx950_workspace_size(&b, FA_DTYPE_BF16, 1) == -1);
    }
    fa_fwd_params mis = good(2, 8, 2, 300, 300, 128);
    mis.q_ptr = (const void *)0x10008;
    EXPECT(fa_fwd_gfx950_check(&mis, FA_DTYPE_F16, 0) == FA_ERR_INVALID_ARGUMENT);
    mis = good(2, 8, 2, 300, 300, 128);
    mis.o_ptr = NULL;
    EXPECT(fa_fwd_gfx950(&mis, FA_DTYPE_F16, 0, NULL) == FA_ERR_INVALID_ARGUMENT);
    // valid parameters reach the (stub) instantiation: dispatch + geometry + workspace sizing
    EXPECT(fa_fwd_gfx950(&p, FA_DTYPE_F16, 1, NULL) == FA_ERR_UNSUPPORTED);
    int64_t bm = 0, bn = 0, th = 0, wg = 0;
    EXPECT(fa_fwd_gfx950_geometry(&p, 1, &bm, &bn, &th, &wg) == FA_OK && bm == 256 && bn == 64 && wg == 2 * 8 * 2);
    EXPECT(fa_fwd_gfx950_geometry(NULL, 1, &bm, &bn, &th, &wg) == FA_ERR_INVALID_ARGUMENT);
    fa_fwd_params dec = good(32, 32, 8, 1, 4096, 128);
    dec.head_q_per_group = 1;  // (the torch binding packs Sq == 1: rows = group)
    dec.num_heads_q = 8;
    dec.seqlen_q = 4;
    dec.q_batch_stride = dec.o_batch_stride = 8 * 4 * 128;
    dec.q_head_stride = dec.o_head_stride = 4 * 128;
    const int64_t ws = fa_fwd_gfx950_workspace_size(&dec, FA_DTYPE_BF16, 0);
    EXPECT(ws >= 0);
    EXPECT(fa_fwd_gfx950_ws(&dec, FA_DTYPE_BF16, 0, (void *)0x100008, ws, NULL) == FA_ERR_INVALID_ARGUMENT);
    EXPECT(fa_fwd_gfx950_geometry(&dec, 0, &bm, &bn, &th, &wg) == FA_OK && bm == 32);
    // varlen
    int32_t cu[3] = {0, 100, 300};
    fa_varlen_params vp;
    memset(&vp, 0, sizeof(vp));
    vp.base = good(2, 8, 2, 300, 300, 128);
    vp.cu_seqlens_q = cu;
    vp.cu_seqlens_k = cu;
    EXPECT(fa_fwd_gfx950_varlen_check(&vp, FA_DTYPE_F16, 1) == FA_OK);
    vp.cu_seqlens_k = NULL;
    EXPECT(fa_fwd_gfx950_varlen_check(&vp, FA_DTYPE_F16, 1) == FA_ERR_INVALID_ARGUMENT);
    EXPECT(fa_fwd_gfx950_varlen(NULL, FA_DTYPE_F16, 1, NULL) == FA_ERR_INVALID_ARGUMENT);
    vp.cu_seqlens_k = (const int32_t *)((const char *)cu + 2);
    EXPECT(fa_fwd_gfx950_varlen_check(&vp, FA_DTYPE_F16, 1) == FA_ERR_INVALID_ARGUMENT);
    // padded
    fa_padded_params pp;
    memset(&pp, 0, sizeof(pp));
    pp.base = good(2, 8, 2, 300, 300, 128);
    pp.k_start = cu;
    EXPECT(fa_fwd_gfx950_padded_workspace_size(&pp, FA_DTYPE_F16, 1, -1) == -1);  // k_end missing
    pp.k_end = cu + 1;
    EXPECT(fa_fwd_gfx950_padded_workspace_size(&pp, FA_DTYPE_F16, 1, -1) > 0);
    EXPECT(fa_fwd_gfx950_padded(&pp, FA_DTYPE_F16, 1, -1, NULL, 0, NULL) == FA_ERR_INVALID_ARGUMENT);
    pp.base.q_batch_stride = 300 * 128 * 8 + 8;  // not a multiple of the seqlen stride
    EXPECT(fa_fwd_gfx950_padded(&pp, FA_DTYPE_F16, 1, -1, (void *)0x100000, 1 << 20, NULL) == FA_ERR_INVALID_ARGUMENT);
    // window / rope: validation paths
    EXPECT(fa_fwd_gfx950_window(NULL, FA_DTYPE_F16, 1, 10, NULL) == FA_ERR_INVALID_ARGUMENT);
    fa_rope_fwd_params rp;
    memset(&rp, 0, sizeof(rp));
    rp.base = good(1, 4, 4, 64, 64, 128);
    EXPECT(fa_fwd_gfx950_rope(&rp, FA_DTYPE_F16, 1, NULL) == FA_ERR_INVALID_ARGUMENT);  // no tables
    rp.base.headdim = 96;
    rp.rope_cos = rp.rope_sin = (const void *)0x50000;
    EXPECT(fa_fwd_gfx950_rope(&rp, FA_DTYPE_F16, 1, NULL) == FA_ERR_UNSUPPORTED);
    if (failures) fprintf(stderr, "%d failures\n", failures);
    else printf("abi validation ok\n");
    return failures ? 1 : 0;
}
