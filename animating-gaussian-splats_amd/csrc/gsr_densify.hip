// gsr_densify.hip -- densification statistics and clone/split/prune compaction with Adam state
// surgery, replacing the torch op chains of densify.py:154-162 and
// external.py:113-314.
//
// The reference densifies with ~60 torch ops per call (boolean-mask gathers, cat, repeat, bmm, and
// a fresh allocation of every parameter and both Adam moments three times).  Here:
//   k_dens_radii     max-radius / visibility update (densify.py:154-162), one thread per Gaussian
//   k_dens_grads     gradient-norm accumulation (external.py:113-124)
//   k_dens_flags     per Gaussian: clone / split / prune decisions of the ORIGINAL row and of its
//                    copies, block counts of the four output categories
//   k_dens_scan      one block: exclusive scan of the block counts -> output offsets, totals
//   k_dens_stds      split Gaussians' scales, the std of the reference's torch.normal draw
//   k_dens_apply     every (column, row) writes its row to its up-to-four output slots, Adam moments
//                    copied for surviving originals and zeroed for new rows, split means offset by
//                    R(q) * sample, split log-scales = log(exp(s) / 1.6)
// Output order equals the reference's: surviving originals, surviving clones, surviving first split
// copies, surviving second split copies, each in index order.
#include "gsr_common.h"
#include "gsr_internal.h"

namespace gsr {

constexpr int kDensBlock = 1024;
enum : uint32_t { kFClone = 1, kFSplit = 2, kFKeepOrig = 4, kFKeepClone = 8, kFKeepSplit = 16 };

__global__ void k_dens_radii(int P, const int *__restrict__ radii, float *__restrict__ max_radii,
                             uint8_t *__restrict__ visible) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const int r = radii[i];
    const bool vis = r > 0;
    visible[i] = vis;
    if (vis) max_radii[i] = fmaxf((float)r, max_radii[i]);
}

__global__ void k_dens_grads(int P, const uint8_t *__restrict__ visible, const float *__restrict__ m2grad,
                             float *__restrict__ grad_accum, float *__restrict__ vis_count) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P || !visible[i]) return;
    const float gx = m2grad[3 * i], gy = m2grad[3 * i + 1];
    grad_accum[i] += sqrtf(gx * gx + gy * gy);
    vis_count[i] += 1.0f;
}

__device__ inline float max_exp3(const float *ls) {
    return fmaxf(fmaxf(expf(ls[0]), expf(ls[1])), expf(ls[2]));
}
__device__ inline bool dens_pruned(float opacity_logit, float max_scale, const DensArgs &a) {
    const float o = 1.0f / (1.0f + expf(-opacity_logit));
    return o < a.remove_opacity || (a.prune_big && max_scale > a.big_scale);
}

// Category bits of row i; the split copies' scales are log(exp(s) / 1.6).
__device__ inline uint32_t dens_row_flags(int i, const DensArgs &a) {
    const float cnt = a.vis_count[i];
    float avg = a.grad_accum[i] / cnt;
    if (avg != avg) avg = 0.f;  // 0 / 0 -> nan -> 0 (external.py:229)
    const float *ls = a.log_scales + 3 * (size_t)i;
    const float ms = max_exp3(ls);
    const float ol = a.opacity_logits[i];
    const bool hot = avg >= a.grad_threshold;
    const bool clone = hot && ms <= a.small_scale;
    const bool split = hot && ms > a.small_scale;
    const bool pr = dens_pruned(ol, ms, a);
    uint32_t f = (clone ? kFClone : 0u) | (split ? kFSplit : 0u);
    if (!split && !pr) f |= kFKeepOrig;
    if (clone && !pr) f |= kFKeepClone;
    if (split) {
        float ls2[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) ls2[k] = logf(expf(ls[k]) * a.inv_split_div);
        if (!dens_pruned(ol, max_exp3(ls2), a)) f |= kFKeepSplit;
    }
    return f;
}

// categories: 0 surviving originals, 1 surviving clones, 2 all splits (sample index), 3 surviving splits
__device__ inline uint4 dens_cats(uint32_t f) {
    return make_uint4((f & kFKeepOrig) ? 1u : 0u, (f & kFKeepClone) ? 1u : 0u, (f & kFSplit) ? 1u : 0u,
                      (f & kFKeepSplit) ? 1u : 0u);
}

__global__ __launch_bounds__(kDensBlock) void k_dens_flags(DensArgs a, uint8_t *__restrict__ flags,
                                                           uint4 *__restrict__ bsum) {
    __shared__ uint32_t s_red[16];
    const int i = blockIdx.x * kDensBlock + threadIdx.x;
    uint32_t f = 0;
    if (i < a.P) {
        f = dens_row_flags(i, a);
        flags[i] = (uint8_t)f;
    }
    const uint4 c = dens_cats(f);
    uint4 t;
    block_excl_scan_u32(c.x, s_red, &t.x);
    block_excl_scan_u32(c.y, s_red, &t.y);
    block_excl_scan_u32(c.z, s_red, &t.z);
    block_excl_scan_u32(c.w, s_red, &t.w);
    if (threadIdx.x == 0) bsum[blockIdx.x] = t;
}

__global__ __launch_bounds__(1024) void k_dens_scan(int NB, const uint4 *__restrict__ bsum, uint4 *__restrict__ boff,
                                                     uint32_t *__restrict__ totals) {
    __shared__ uint32_t s_red[16];
    uint4 carry = make_uint4(0, 0, 0, 0);
    for (int base = 0; base < NB; base += blockDim.x) {
        const int b = base + threadIdx.x;
        const uint4 c = b < NB ? bsum[b] : make_uint4(0, 0, 0, 0);
        uint4 t, e;
        e.x = block_excl_scan_u32(c.x, s_red, &t.x) + carry.x;
        e.y = block_excl_scan_u32(c.y, s_red, &t.y) + carry.y;
        e.z = block_excl_scan_u32(c.z, s_red, &t.z) + carry.z;
        e.w = block_excl_scan_u32(c.w, s_red, &t.w) + carry.w;
        if (b < NB) boff[b] = e;
        carry.x += t.x; carry.y += t.y; carry.z += t.z; carry.w += t.w;
    }
    if (threadIdx.x == 0) { totals[0] = carry.x; totals[1] = carry.y; totals[2] = carry.z; totals[3] = carry.w; }
}

// Per row: output slots of its original / clone / first and second split copies (or -1), its split
// rank (sample index), from the block offsets and an in-block scan.
struct DensSlots { int orig, clone, split_a, split_b, rank; uint32_t f; };
__device__ inline DensSlots dens_slots(int i, const uint8_t *__restrict__ flags, const uint4 *__restrict__ boff,
                                       const uint32_t *__restrict__ tot, uint32_t *s_red) {
    const uint32_t f = i < 0 ? 0u : flags[i];
    const uint4 c = dens_cats(f);
    const uint4 o = boff[blockIdx.x];
    uint32_t t;
    const uint32_t ex = block_excl_scan_u32(c.x, s_red, &t) + o.x;
    const uint32_t ey = block_excl_scan_u32(c.y, s_red, &t) + o.y;
    const uint32_t ez = block_excl_scan_u32(c.z, s_red, &t) + o.z;
    const uint32_t ew = block_excl_scan_u32(c.w, s_red, &t) + o.w;
    const uint32_t n_ko = tot[0], n_kc = tot[1], n_ks = tot[3];
    DensSlots s;
    s.f = f;
    s.orig = c.x ? (int)ex : -1;
    s.clone = c.y ? (int)(n_ko + ey) : -1;
    s.split_a = c.w ? (int)(n_ko + n_kc + ew) : -1;
    s.split_b = c.w ? (int)(n_ko + n_kc + n_ks + ew) : -1;
    s.rank = c.z ? (int)ez : -1;
    return s;
}

__global__ __launch_bounds__(kDensBlock) void k_dens_stds(DensArgs a, const uint8_t *__restrict__ flags,
                                                          const uint4 *__restrict__ boff,
                                                          const uint32_t *__restrict__ tot, float *__restrict__ stds) {
    __shared__ uint32_t s_red[16];
    const int i = blockIdx.x * kDensBlock + threadIdx.x;
    const DensSlots s = dens_slots(i < a.P ? i : -1, flags, boff, tot, s_red);
    if (s.rank < 0) return;
    const int S = (int)tot[2];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float e = expf(a.log_scales[3 * (size_t)i + k]);
        stds[3 * (size_t)s.rank + k] = e;
        stds[3 * (size_t)(S + s.rank) + k] = e;
    }
}

__global__ __launch_bounds__(kDensBlock) void k_dens_apply(DensArgs a, const uint8_t *__restrict__ flags,
                                                           const uint4 *__restrict__ boff,
                                                           const uint32_t *__restrict__ tot,
                                                           const float *__restrict__ samples, DensColumns cols) {
    __shared__ uint32_t s_red[16];
    const int i = blockIdx.x * kDensBlock + threadIdx.x;
    const DensSlots s = dens_slots(i < a.P ? i : -1, flags, boff, tot, s_red);
    if (i >= a.P) return;
    const int S = (int)tot[2];
    // split-copy means offset R(q) * sample, R = build_rotation(q) (external.py:27-46)
    float off[2][3] = {{0, 0, 0}, {0, 0, 0}};
    if (s.split_a >= 0) {
        float4 q = make_float4(a.rotations[4 * (size_t)i], a.rotations[4 * (size_t)i + 1],
                               a.rotations[4 * (size_t)i + 2], a.rotations[4 * (size_t)i + 3]);
        const float n = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
        const float r = q.x / n, x = q.y / n, y = q.z / n, z = q.w / n;
        const float R[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                            2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                            2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)};
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const float *smp = samples + 3 * (size_t)(c * S + s.rank);
#pragma unroll
            for (int row = 0; row < 3; ++row)
                off[c][row] = R[3 * row] * smp[0] + R[3 * row + 1] * smp[1] + R[3 * row + 2] * smp[2];
        }
    }
    for (int ci = 0; ci < cols.n; ++ci) {
        const DensColumn &c = cols.c[ci];
        const int w = c.width;
        const float *src = c.src + (size_t)i * w;
        for (int k = 0; k < w; ++k) {
            const float val = src[k];
            if (s.orig >= 0) {
                c.dst[(size_t)s.orig * w + k] = val;
                if (c.m_dst) {
                    c.m_dst[(size_t)s.orig * w + k] = c.m_src[(size_t)i * w + k];
                    c.v_dst[(size_t)s.orig * w + k] = c.v_src[(size_t)i * w + k];
                }
            }
            if (s.clone >= 0) {
                c.dst[(size_t)s.clone * w + k] = val;
                if (c.m_dst) { c.m_dst[(size_t)s.clone * w + k] = 0.f; c.v_dst[(size_t)s.clone * w + k] = 0.f; }
            }
            if (s.split_a >= 0) {
                float va = val, vb = val;
                if (c.role == GSR_DENS_MEANS && k < 3) { va = val + off[0][k]; vb = val + off[1][k]; }
                if (c.role == GSR_DENS_LOG_SCALES) { va = vb = logf(expf(val) * a.inv_split_div); }
                c.dst[(size_t)s.split_a * w + k] = va;
                c.dst[(size_t)s.split_b * w + k] = vb;
                if (c.m_dst) {
                    c.m_dst[(size_t)s.split_a * w + k] = 0.f; c.v_dst[(size_t)s.split_a * w + k] = 0.f;
                    c.m_dst[(size_t)s.split_b * w + k] = 0.f; c.v_dst[(size_t)s.split_b * w + k] = 0.f;
                }
            }
        }
    }
}

// ==========================================================================================
hipError_t launch_dens_radii(int P, const int *radii, float *max_radii, uint8_t *visible, hipStream_t s) {
    if (P == 0) return hipSuccess;
    k_dens_radii<<<div_up(P, 256), 256, 0, s>>>(P, radii, max_radii, visible);
    return hipGetLastError();
}

hipError_t launch_dens_grads(int P, const uint8_t *visible, const float *m2grad, float *grad_accum,
                             float *vis_count, hipStream_t s) {
    if (P == 0) return hipSuccess;
    k_dens_grads<<<div_up(P, 256), 256, 0, s>>>(P, visible, m2grad, grad_accum, vis_count);
    return hipGetLastError();
}

DensWorkspace::DensWorkspace(int P) {
    NB = div_up(P > 0 ? P : 1, kDensBlock);
    size_t o = 0;
    flags = o;  o = align256(o + (size_t)NB * kDensBlock);
    bsum = o;   o = align256(o + sizeof(uint4) * NB);
    boff = o;   o = align256(o + sizeof(uint4) * NB);
    totals = o; o = align256(o + sizeof(uint32_t) * 4);
    total = o;
}

hipError_t launch_dens_plan(const DensArgs &a, char *ws, hipStream_t s) {
    const DensWorkspace L(a.P);
    k_dens_flags<<<L.NB, kDensBlock, 0, s>>>(a, (uint8_t *)(ws + L.flags), (uint4 *)(ws + L.bsum));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    k_dens_scan<<<1, 1024, 0, s>>>(L.NB, (const uint4 *)(ws + L.bsum), (uint4 *)(ws + L.boff),
                                   (uint32_t *)(ws + L.totals));
    return hipGetLastError();
}

hipError_t launch_dens_stds(const DensArgs &a, const char *ws, float *stds, hipStream_t s) {
    const DensWorkspace L(a.P);
    k_dens_stds<<<L.NB, kDensBlock, 0, s>>>(a, (const uint8_t *)(ws + L.flags), (const uint4 *)(ws + L.boff),
                                            (const uint32_t *)(ws + L.totals), stds);
    return hipGetLastError();
}

hipError_t launch_dens_apply(const DensArgs &a, const char *ws, const float *samples, const DensColumns &cols,
                             hipStream_t s) {
    const DensWorkspace L(a.P);
    k_dens_apply<<<L.NB, kDensBlock, 0, s>>>(a, (const uint8_t *)(ws + L.flags), (const uint4 *)(ws + L.boff),
                                             (const uint32_t *)(ws + L.totals), samples, cols);
    return hipGetLastError();
}

}  // namespace gsr
