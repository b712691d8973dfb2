// gsr_io.hip -- the pixel side of the data path: decoded 8-bit camera frames
// and segmentation masks of one timestep, uploaded as ONE u8 batch, become the float tensors the
// reference's load_timestep_views builds (shared.py:127-171) per view with ~6 torch ops each:
//   image = torch.tensor(u8 HWC).float().cuda().permute(2, 0, 1) / 255      (shared.py:152-160)
//   mask  = torch.stack((m, zeros_like(m), 1 - m)),  m = float(u8 HW)        (shared.py:131-143,161-168)
// On the GPU torch divides by a Python scalar as a multiply by its float reciprocal
// (x * (1.0f / 255.0f)); the kernel does exactly that, so the result is bitwise the reference's.
//
// k_views_pack: grid.y = frame, one thread per 4 consecutive pixels: three dword loads give the 12
// interleaved RGB bytes (wave: 768 contiguous bytes), one dword gives 4 mask bytes; the planar
// outputs are float4 stores (coalesced per plane).  Byte work, HBM-bound: 4 B read + 24 B written per
// pixel with a mask (12 B without).
#include "gsr_common.h"
#include "gsr_internal.h"

namespace gsr {

constexpr int kPackThreads = 256;

__device__ inline float u8f(uint32_t w, int k) { return (float)((w >> (8 * k)) & 0xFFu); }

__global__ __launch_bounds__(kPackThreads) void k_views_pack(int HW, const uint8_t *__restrict__ rgb,
                                                             const uint8_t *__restrict__ seg,
                                                             float *__restrict__ img, float *__restrict__ msk) {
    const int f = blockIdx.y;
    const int p0 = 4 * (blockIdx.x * kPackThreads + threadIdx.x);
    if (p0 >= HW) return;
    const float inv = 1.0f / 255.0f;
    const uint8_t *src = rgb + (size_t)f * HW * 3;
    float *dst = img + (size_t)f * 3 * HW;
    if ((HW & 3) == 0) {  // 4 whole pixels, 4-byte aligned loads, 16-byte aligned stores
        const uint32_t *s32 = reinterpret_cast<const uint32_t *>(src + 3 * (size_t)p0);
        const uint32_t w0 = s32[0], w1 = s32[1], w2 = s32[2];  // r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
        const float4 R = make_float4(u8f(w0, 0) * inv, u8f(w0, 3) * inv, u8f(w1, 2) * inv, u8f(w2, 1) * inv);
        const float4 G = make_float4(u8f(w0, 1) * inv, u8f(w1, 0) * inv, u8f(w1, 3) * inv, u8f(w2, 2) * inv);
        const float4 B = make_float4(u8f(w0, 2) * inv, u8f(w1, 1) * inv, u8f(w2, 0) * inv, u8f(w2, 3) * inv);
        *reinterpret_cast<float4 *>(dst + p0) = R;
        *reinterpret_cast<float4 *>(dst + HW + p0) = G;
        *reinterpret_cast<float4 *>(dst + 2 * (size_t)HW + p0) = B;
        if (seg) {
            const uint32_t m = *reinterpret_cast<const uint32_t *>(seg + (size_t)f * HW + p0);
            float *md = msk + (size_t)f * 3 * HW;
            const float4 M = make_float4(u8f(m, 0), u8f(m, 1), u8f(m, 2), u8f(m, 3));
            *reinterpret_cast<float4 *>(md + p0) = M;
            *reinterpret_cast<float4 *>(md + HW + p0) = make_float4(0.f, 0.f, 0.f, 0.f);
            *reinterpret_cast<float4 *>(md + 2 * (size_t)HW + p0) =
                make_float4(1.f - M.x, 1.f - M.y, 1.f - M.z, 1.f - M.w);
        }
        return;
    }
    for (int p = p0; p < min(p0 + 4, HW); ++p) {  // ragged frame: byte loads, scalar stores
        dst[p] = (float)src[3 * (size_t)p] * inv;
        dst[HW + p] = (float)src[3 * (size_t)p + 1] * inv;
        dst[2 * (size_t)HW + p] = (float)src[3 * (size_t)p + 2] * inv;
        if (seg) {
            const float m = (float)seg[(size_t)f * HW + p];
            float *md = msk + (size_t)f * 3 * HW;
            md[p] = m;
            md[HW + p] = 0.f;
            md[2 * (size_t)HW + p] = 1.f - m;
        }
    }
}

hipError_t launch_views_pack(int frames, int HW, const uint8_t *rgb, const uint8_t *seg, float *img, float *msk,
                             hipStream_t s) {
    const dim3 grid(div_up(div_up(HW, 4), kPackThreads), frames);
    hipLaunchKernelGGL(k_views_pack, grid, dim3(kPackThreads), 0, s, HW, rgb, seg, img, msk);
    return hipGetLastError();
}

}  // namespace gsr
