// Probe: SIMD throughput of the VALU instruction kinds the render kernels use, on gfx950.
// 8 waves per SIMD, 8 independent chains per lane; prints cycles per wave64 instruction per SIMD
// (assuming the 2.4 GHz max clock; the ratios between kinds are what matters).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(256) void k_probe(float *out, int iters) {
    float a[8];
    f2 p[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a[j] = threadIdx.x + j; p[j] = f2{a[j], a[j] + 0.5f}; }
    const float m = 1.0000001f, c = 1e-7f;
    const f2 m2 = {m, m}, c2 = {c, c};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (KIND == 0) a[j] = fmaf(a[j], m, c);
                else if (KIND == 1) p[j] = __builtin_elementwise_fma(p[j], m2, c2);
                else if (KIND == 2) a[j] = __builtin_amdgcn_exp2f(a[j]) * 0.5f;  // exp + mul
                else if (KIND == 3) a[j] = __builtin_amdgcn_rcpf(a[j]) + 1.0f;   // rcp + add
                else if (KIND == 4) a[j] = a[j] + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, a[j]), 0x128, 0xF, 0xF, false));
                else if (KIND == 5) { auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[j]), __float_as_uint(a[(j + 1) & 7]), false, false);
                                      a[j] = __uint_as_float(r[0]); a[(j + 1) & 7] = __uint_as_float(r[1]); }
                else if (KIND == 6) a[j] = a[j] * m;
            }
        }
    }
    float s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] + p[j].x + p[j].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int KIND>
static void run(const char *name, float *d, int blocks, int iters, int instr_per_inner) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k_probe<KIND><<<blocks, 256>>>(d, iters);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) k_probe<KIND><<<blocks, 256>>>(d, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double waves_per_simd = blocks * 4.0 / 1024.0;
    const double instr = waves_per_simd * iters * 16.0 * 8.0 * instr_per_inner;
    printf("%-22s %8.3f ms  %6.2f cycles/instr/SIMD (at 2.4 GHz)\n", name, ms, ms * 1e-3 * 2.4e9 / instr);
}

int main() {
    const int blocks = 256 * 8, iters = 100;
    float *d = nullptr;
    if (hipMalloc(&d, sizeof(float) * 256 * blocks) != hipSuccess) return 1;
    run<0>("v_fma_f32", d, blocks, iters, 1);
    run<1>("v_pk_fma_f32 (2 fma)", d, blocks, iters, 1);
    run<2>("v_exp_f32 + v_mul", d, blocks, iters, 2);
    run<3>("v_rcp_f32 + v_add", d, blocks, iters, 2);
    run<4>("v_add_f32_dpp", d, blocks, iters, 1);
    run<5>("v_permlane32_swap", d, blocks, iters, 1);
    run<6>("v_mul_f32", d, blocks, iters, 1);
    hipFree(d);
    return 0;
}
