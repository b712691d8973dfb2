// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access shapes the rasterizer
// kernels use (MI355X_MICROARCH.md: only 16-B/lane streaming reads and stores are calibrated there).
// Every kernel touches a known number of bytes of a 1 GiB table (4x the 256 MiB Infinity Cache, so
// re-use cannot hide traffic).  Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` and
// divide the counter by the printed byte count.
//   k_stream16   coalesced float4 per lane, contiguous                 (the guide's calibrated case)
//   k_gather48   3 float4 of a random 64-B record per lane            (render staging: rec[0..2])
//   k_gather64   4 float4 of a random 64-B record per lane            (rec[0..3])
//   k_gather16   1 float4 of a random 64-B record per lane            (epilogue rec[3] re-read)
//   k_seq48      3 float4 per lane, 48-B records, lane-contiguous      (gauss_bwd part records)
//   k_scatter48  3 float4 stores per lane to random 48-B records        (render_bwd part records)
//   k_seq12      3 dwords per lane, 12-B records, lane-contiguous      ((P,3) parameter arrays)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ inline uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void k_stream16(const float4 *__restrict__ a, size_t n, float *out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

template <int NF4>
__global__ void k_gather(const float4 *__restrict__ tab, uint32_t nrec, uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = hash32(i) % nrec;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NF4; ++k) {
        const float4 v = tab[4 * (size_t)r + k];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

__global__ void k_gather16_last(const float4 *__restrict__ tab, uint32_t nrec, uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = hash32(i) % nrec;
    const float4 v = tab[4 * (size_t)r + 3];
    if (v.x + v.y + v.z + v.w == 1234.5f) out[0] = 1.f;
}

__global__ void k_seq48(const float4 *__restrict__ a, uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 x = a[3 * (size_t)i], y = a[3 * (size_t)i + 1], z = a[3 * (size_t)i + 2];
    if (x.x + y.y + z.z + x.w == 1234.5f) out[0] = 1.f;
}

__global__ void k_scatter48(float4 *__restrict__ a, uint32_t nrec, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = hash32(i) % nrec;
    const float f = (float)i;
    a[3 * (size_t)r] = make_float4(f, f, f, f);
    a[3 * (size_t)r + 1] = make_float4(f, f, f, f);
    a[3 * (size_t)r + 2] = make_float4(f, 0.f, 0.f, 0.f);
}

__global__ void k_seq12(const float *__restrict__ a, uint32_t n, float *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float s = a[3 * (size_t)i] + a[3 * (size_t)i + 1] + a[3 * (size_t)i + 2];
    if (s == 1234.5f) out[0] = 1.f;
}

int main() {
    const size_t bytes = size_t(1) << 30;
    float4 *tab = nullptr;
    float *out = nullptr;
    if (hipMalloc(&tab, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    if (hipMemset(tab, 0, bytes) != hipSuccess) return 1;
    const uint32_t nrec64 = (uint32_t)(bytes / 64), nrec48 = (uint32_t)(bytes / 48);
    const uint32_t n = 4u << 20;  // 4 Mi gathers / records per kernel
    for (int rep = 0; rep < 2; ++rep) {
        k_stream16<<<4096, 256>>>(tab, (size_t(256) << 20) / 16, out);           // 256 MiB
        k_gather<3><<<n / 256, 256>>>(tab, nrec64, n, out);
        k_gather<4><<<n / 256, 256>>>(tab, nrec64, n, out);
        k_gather16_last<<<n / 256, 256>>>(tab, nrec64, n, out);
        k_seq48<<<n / 256, 256>>>(tab, n, out);
        k_scatter48<<<n / 256, 256>>>(tab, nrec48, n);
        k_seq12<<<n / 256, 256>>>(reinterpret_cast<const float *>(tab), n, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("k_stream16     read  %zu B\n", size_t(256) << 20);
    printf("k_gather<3>    read  %zu B (48 B x %u random 64-B records)\n", size_t(48) * n, n);
    printf("k_gather<4>    read  %zu B (64 B x %u)\n", size_t(64) * n, n);
    printf("k_gather16_last read %zu B (16 B x %u)\n", size_t(16) * n, n);
    printf("k_seq48        read  %zu B\n", size_t(48) * n);
    printf("k_scatter48    write %zu B (48 B x %u random 48-B records)\n", size_t(48) * n, n);
    printf("k_seq12        read  %zu B\n", size_t(12) * n);
    hipFree(tab);
    hipFree(out);
    return 0;
}
