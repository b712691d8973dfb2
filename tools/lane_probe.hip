// Probe of gfx950 v_permlane32_swap / v_permlane16_swap lane semantics (used by wave_sum9).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
    const int l = threadIdx.x;
    unsigned a = 1000 + l, b = 2000 + l;
    auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    out[l] = r[0]; out[64 + l] = r[1];
    auto q = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    out[128 + l] = q[0]; out[192 + l] = q[1];
}
int main() {
    int* d; int h[256];
    hipMalloc(&d, sizeof(h));
    k<<<1, 64>>>(d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char* nm[4] = {"swap32.r0", "swap32.r1", "swap16.r0", "swap16.r1"};
    for (int s = 0; s < 4; ++s) {
        printf("%s:", nm[s]);
        for (int l = 0; l < 64; l += 8) printf(" [%d]=%d", l, h[s * 64 + l]);
        printf("\n");
    }
    return 0;
}
