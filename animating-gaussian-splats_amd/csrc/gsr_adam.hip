// gsr_adam.hip -- one-launch Adam step over every per-Gaussian parameter tensor (SURVEY.md 8(f)
// row 3), replacing torch.optim.Adam (densify.py:68-86: one named group per parameter, eps 1e-15,
// betas (0.9, 0.999), no weight decay) whose foreach path runs ~8 elementwise kernels per group, each
// streaming the parameter / gradient / moments through HBM again.
//
// k_adam: blocks walk a table of up to kAdamMaxTensors tensors (block -> tensor by a prefix of block
// counts, passed in the kernel arguments); each thread updates 4 consecutive elements (float4 when
// the tensor is 16-byte aligned) with the operation order of torch's _multi_tensor_adam:
//   m = lerp(m, g, 1 - beta1)                   = m + w (g - m)            (w < 0.5 form, fused)
//   v = v * beta2;  v = v + (1 - beta2) (g g)   (addcmul, fused)
//   d = sqrt(v) / sqrt(1 - beta2^t) + eps
//   p = p + step_size * (m / d),  step_size = -lr / (1 - beta1^t)           (addcdiv, fused)
// Per-tensor scalars are computed on the host in double exactly as torch does and rounded to float.
// Algorithmic HBM bytes: 28 per element (read p, g, m, v; write p, m, v).
#include "gsr_common.h"
#include "gsr_internal.h"

namespace gsr {

constexpr int kAdamThreads = 256;
constexpr int kAdamPerBlock = kAdamThreads * 4;

__device__ inline void adam_elem(float &p, float g, float &m, float &v, float w1, float b2, float omb2,
                                 float eps, float step_size, float bc2s) {
    m = fmaf(w1, g - m, m);
    const float vb = v * b2;
    v = fmaf(omb2, g * g, vb);  // addcmul: self + value * (t1 * t2), contracted
    const float d = sqrtf(v) / bc2s + eps;
    p = fmaf(step_size, m / d, p);
}

__global__ __launch_bounds__(kAdamThreads) void k_adam(AdamTable tab) {
    int t = 0;
    while (t + 1 < tab.n && (int)blockIdx.x >= tab.block_start[t + 1]) ++t;
    const AdamTensor &T = tab.t[t];
    const long long e0 = (long long)((int)blockIdx.x - tab.block_start[t]) * kAdamPerBlock + 4ll * threadIdx.x;
    if (e0 >= T.n) return;
    if (T.vec4 && e0 + 4 <= T.n) {
        float4 p = *reinterpret_cast<const float4 *>(T.param + e0);
        const float4 g = *reinterpret_cast<const float4 *>(T.grad + e0);
        float4 m = *reinterpret_cast<const float4 *>(T.exp_avg + e0);
        float4 v = *reinterpret_cast<const float4 *>(T.exp_avg_sq + e0);
        adam_elem(p.x, g.x, m.x, v.x, tab.w1, tab.b2, tab.omb2, tab.eps, T.step_size, T.bc2_sqrt);
        adam_elem(p.y, g.y, m.y, v.y, tab.w1, tab.b2, tab.omb2, tab.eps, T.step_size, T.bc2_sqrt);
        adam_elem(p.z, g.z, m.z, v.z, tab.w1, tab.b2, tab.omb2, tab.eps, T.step_size, T.bc2_sqrt);
        adam_elem(p.w, g.w, m.w, v.w, tab.w1, tab.b2, tab.omb2, tab.eps, T.step_size, T.bc2_sqrt);
        *reinterpret_cast<float4 *>(T.param + e0) = p;
        *reinterpret_cast<float4 *>(T.exp_avg + e0) = m;
        *reinterpret_cast<float4 *>(T.exp_avg_sq + e0) = v;
        return;
    }
    for (long long e = e0; e < e0 + 4 && e < T.n; ++e) {
        float p = T.param[e], m = T.exp_avg[e], v = T.exp_avg_sq[e];
        adam_elem(p, T.grad[e], m, v, tab.w1, tab.b2, tab.omb2, tab.eps, T.step_size, T.bc2_sqrt);
        T.param[e] = p; T.exp_avg[e] = m; T.exp_avg_sq[e] = v;
    }
}

int adam_blocks(long long n) { return (int)((n + kAdamPerBlock - 1) / kAdamPerBlock); }

hipError_t launch_adam(const AdamTable &tab, hipStream_t s) {
    const int nb = tab.block_start[tab.n];
    if (nb == 0) return hipSuccess;
    k_adam<<<nb, kAdamThreads, 0, s>>>(tab);
    return hipGetLastError();
}

}  // namespace gsr
