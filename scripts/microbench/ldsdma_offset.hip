// ldsdma_offset.hip -- what the instruction offset of an LDS-DMA load does on gfx950.
// Standalone diagnostic, not product code.
//
// buffer_load_dwordx4 v_off, s[rsrc], soff offen offset:OFF lds  moves 16 B per lane from
// rsrc.base + soff + v_off + OFF into LDS. The question for fa_fwd_w4's tile loop: does OFF also
// move the LDS destination (M0 + OFF + 16 * lane), so that the four 1-KiB pieces of a tile can share
// one M0 value? One wave, source word i = i, M0 = 4096, soff = 0 and 256; the LDS image is read back
// whole and the first lane's source word / destination are printed for each OFF.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __amdgpu_buffer_rsrc_t rsrc_t;

template <int OFF>
__global__ void probe(const uint32_t *src, uint32_t *out, int soff) {
    __shared__ __attribute__((aligned(1024))) uint32_t lds[4096];  // 16 KiB
    const int lane = threadIdx.x;
    for (int i = lane; i < 4096; i += 64) lds[i] = 0xffffffffu;
    __syncthreads();
    const rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)src, (short)0, 1 << 20, 0x00020000);
    const uint32_t m0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)lds + 4096;
    const int voff = lane * 16;
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen offset:%4 lds\n\ts_waitcnt vmcnt(0)"
                 ::"v"(voff), "s"(rs), "s"(m0), "s"(soff), "i"(OFF)
                 : "memory", "m0");
    __syncthreads();
    for (int i = lane; i < 4096; i += 64) out[i] = lds[i];
}

template <int OFF>
void run(const uint32_t *dsrc, uint32_t *dout, uint32_t *hout, int soff) {
    hipLaunchKernelGGL(probe<OFF>, dim3(1), dim3(64), 0, 0, dsrc, dout, soff);
    if (hipMemcpy(hout, dout, 4096 * 4, hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return; }
    int first = -1, n = 0;
    for (int i = 0; i < 4096; ++i)
        if (hout[i] != 0xffffffffu) { if (first < 0) first = i; ++n; }
    if (first < 0) { printf("OFF=%4d soff=%3d: nothing landed\n", OFF, soff); return; }
    // first landed word: its LDS byte address relative to the LDS array, and the source byte it holds
    printf("OFF=%4d soff=%3d: %d words landed, first at LDS byte %d (M0 = 4096), holding source byte %u; "
           "last holds source byte %u\n",
           OFF, soff, n, first * 4, hout[first] * 4, hout[first + n - 1] * 4);
}

int main() {
    uint32_t *dsrc, *dout, *hsrc = new uint32_t[1 << 18], *hout = new uint32_t[4096];
    for (int i = 0; i < (1 << 18); ++i) hsrc[i] = i;
    if (hipMalloc(&dsrc, 1 << 20) != hipSuccess || hipMalloc(&dout, 4096 * 4) != hipSuccess) return 1;
    if (hipMemcpy(dsrc, hsrc, 1 << 20, hipMemcpyHostToDevice) != hipSuccess) return 1;
    for (int soff : {0, 256}) {
        run<0>(dsrc, dout, hout, soff);
        run<1024>(dsrc, dout, hout, soff);
        run<2048>(dsrc, dout, hout, soff);
        run<3072>(dsrc, dout, hout, soff);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    printf("done\n");
    return 0;
}
