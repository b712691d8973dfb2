// Probe: does a wave64 VALU instruction on gfx950 (SIMD-32, 2 passes) get cheaper when one
// 32-lane half of EXEC is zero?  Times a dependent-free FMA block under different lane masks.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void k_probe(float *out, int iters) {
    const int lane = threadIdx.x & 63;
    bool on;
    if (MODE == 0) on = true;                  // all 64 lanes
    else if (MODE == 1) on = lane < 32;        // low half only
    else if (MODE == 2) on = (lane & 1);       // every other lane (both halves active)
    else on = lane < 16;                       // a quarter (low half partially)
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float m = 1.0000001f, c = 0.5f;
    if (__builtin_expect(on, 1)) {
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                a0 = fmaf(a0, m, c); a1 = fmaf(a1, m, c); a2 = fmaf(a2, m, c); a3 = fmaf(a3, m, c);
                a4 = fmaf(a4, m, c); a5 = fmaf(a5, m, c); a6 = fmaf(a6, m, c); a7 = fmaf(a7, m, c);
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

template <int MODE>
static float run(float *d, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k_probe<MODE><<<blocks, 256>>>(d, iters);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) k_probe<MODE><<<blocks, 256>>>(d, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    const int blocks = 256 * 8, iters = 200;
    float *d = nullptr;
    if (hipMalloc(&d, sizeof(float) * 256 * blocks) != hipSuccess) return 1;
    printf("all64 %.3f ms\n", run<0>(d, blocks, iters));
    printf("low32 %.3f ms\n", run<1>(d, blocks, iters));
    printf("odd   %.3f ms\n", run<2>(d, blocks, iters));
    printf("low16 %.3f ms\n", run<3>(d, blocks, iters));
    hipFree(d);
    return 0;
}
