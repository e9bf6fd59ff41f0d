// pair_atomic.hip -- do two workgroups that add 1 to one counter always see {0, 1}? Standalone
// diagnostic for the key-split hand-off (not product code). Pairs on one XCD (b, b ^ 8) and across
// XCDs (b, b ^ 1); the counter add as inline asm with scope bits sc0 sc1 (return, system), sc0
// (return, CU scope) and as the HIP agent-scope builtin. Every workgroup also stamps its XCC id.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int V>
__global__ __launch_bounds__(64) void pair(unsigned *cnt, unsigned *seen, unsigned *xcc, int cross) {
    const unsigned b = blockIdx.x;
    const unsigned slot = cross ? (b >> 1) : ((b >> 4) * 8 + (b & 7));
    unsigned old = 0;
    if (threadIdx.x == 0) {
        if constexpr (V == 0)
            asm volatile("global_atomic_add %0, %1, %2, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(old) : "v"(cnt + 16 * slot), "v"(1u) : "memory");
        else if constexpr (V == 1)
            asm volatile("global_atomic_add %0, %1, %2, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"(old) : "v"(cnt + 16 * slot), "v"(1u) : "memory");
        else
            old = __hip_atomic_fetch_add(cnt + 16 * slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        seen[b] = old;
        unsigned id;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
        xcc[b] = id;
    }
}

int main() {
    const int nb = 512;
    unsigned *cnt, *seen, *xcc, h[nb], hx[nb];
    if (hipMalloc(&cnt, nb * 64) != hipSuccess || hipMalloc(&seen, nb * 4) != hipSuccess || hipMalloc(&xcc, nb * 4) != hipSuccess) return 1;
    void (*k[3])(unsigned *, unsigned *, unsigned *, int) = {pair<0>, pair<1>, pair<2>};
    const char *nm[3] = {"asm sc0 sc1", "asm sc0", "hip agent"};
    for (int v = 0; v < 3; ++v)
        for (int cross = 0; cross < 2; ++cross) {
            int bad = 0, xbad = 0;
            for (int rep = 0; rep < 200; ++rep) {
                hipMemset(cnt, 0, nb * 64);
                hipLaunchKernelGGL(k[v], dim3(nb), dim3(64), 0, 0, cnt, seen, xcc, cross);
                if (hipDeviceSynchronize() != hipSuccess) return 2;
                hipMemcpy(h, seen, nb * 4, hipMemcpyDeviceToHost);
                hipMemcpy(hx, xcc, nb * 4, hipMemcpyDeviceToHost);
                for (int b = 0; b < nb; ++b) {
                    const int p = cross ? (b ^ 1) : (b ^ 8);
                    if (h[b] + h[p] != 1) ++bad;
                    if (!cross && hx[b] != hx[p]) ++xbad;
                }
            }
            printf("%-12s %-9s pairs with a wrong count %d / %d, same-XCD pairs on two XCDs %d\n", nm[v],
                   cross ? "cross-XCD" : "same-XCD", bad / 2, 200 * nb / 2, xbad / 2);
        }
    return 0;
}
