// gsr_loss.hip -- fused L1 + SSIM image loss (forward and backward) for the render call sites.
//
// Replaces, at train.py:354-364 / densify.py:127-129,149-151, the pair
//     torch.nn.functional.l1_loss(img1, img2)   and   calc_ssim(img1, img2)   (external.py:68-110)
// where calc_ssim runs five grouped 11x11 conv2d (window = outer product of a normalised 1-D
// Gaussian, sigma 1.5, zero padding 5) and a dozen elementwise kernels, each with its own autograd
// node.  Here the window is applied separably out of LDS and everything else is fused:
//
//   k_ssim_fwd   one wave64 per 64-column x 32-row strip of one image plane, 4 independent waves per
//                block: rows stream through wave-private LDS (11-tap horizontal pass of
//                (x, y, x^2, y^2, xy)) into an 11-row register ring (vertical pass), then per pixel
//                the SSIM value, its three partial derivatives dS/dmu1, dS/d<x^2>, dS/d<xy> (stored
//                for the backward) and |x - y|.  Per-wave partial sums, no atomics.
//   k_ssim_sum   one block: fixed-order (double) sum of the block partials -> (mean |x-y|, mean S).
//   k_ssim_bwd   same strips: blur the three stored derivative maps (the window is symmetric, so the
//                adjoint of the zero-padded correlation is the same correlation) and combine
//                dL/dx = gS/N (blur(dS/dmu1) + 2 x blur(dS/d<x^2>) + y blur(dS/d<xy>)) + gL1/N sign(x-y)
//                with the upstream gradients gL1, gS read from device memory (no host sync).
//
// Algorithmic HBM bytes: forward 2 reads + 3 writes per pixel (20 B), backward 3 + 2 reads + 1
// write (24 B); the 10 halo rows per 32-row strip and the 10 halo columns re-read through L2.
#include "gsr_common.h"
#include "gsr_internal.h"

namespace gsr {

constexpr int kSsR = 5;                 // window radius (window_size 11)
constexpr int kSsTaps = 2 * kSsR + 1;
constexpr int kSsRH = 32;               // output rows per wave strip (64 columns = one per lane)
constexpr int kSsWaves = 4;             // independent waves per 256-thread block
constexpr int kSsRowBuf = 80;           // staged row: 64 + 2 * 5 halo columns (+ pad)
constexpr float kSsC1 = 0.01f * 0.01f, kSsC2 = 0.03f * 0.03f;

// Strip of wave `gw`: plane, first column x0, first output row y0.
struct SsStrip { int plane, x0, y0; };
__device__ inline SsStrip ss_strip(int gw, int sx, int sy) {
    SsStrip t;
    t.plane = gw / (sx * sy);
    const int r = gw - t.plane * sx * sy;
    t.y0 = (r / sx) * kSsRH;
    t.x0 = (r % sx) * 64;
    return t;
}

// Stage input row `gy` of one plane, columns [x0 - 5, x0 + 69), into the wave's LDS row (zero outside
// the image: conv2d zero padding).  Lane l holds column x0 - 5 + l, lanes 0..9 also x0 + 59 + l.
__device__ inline void ss_load_row(const float *__restrict__ src, int H, int W, int x0, int gy, int lane,
                                   float &lo, float &hi) {
    const bool row_ok = gy >= 0 && gy < H;
    const int ca = x0 - kSsR + lane, cb = x0 + 64 - kSsR + lane;
    lo = (row_ok && ca >= 0 && ca < W) ? src[(size_t)gy * W + ca] : 0.f;
    hi = (row_ok && lane < 2 * kSsR && cb < W) ? src[(size_t)gy * W + cb] : 0.f;
}

// ------------------------------------------------------------------------------------------
// Forward.  Each wave streams down a 64-column strip: per input row it stages the row (+ halo) of
// both images in wave-private LDS, forms the 5 horizontal window sums of (x, y, x^2, y^2, xy) for
// its lane's column, and keeps the last 11 rows of those sums in a register ring (slot = row mod
// 11, resolved at compile time by unrolling 2 x 11 rows; the next two rows' loads are in flight); once 11 rows are in, the vertical window gives
// mu1, mu2, <x^2>, <y^2>, <xy> of the output row 5 above.  No block barriers.
__global__ __launch_bounds__(256) void k_ssim_fwd(int planes, int H, int W, int sx, int sy,
                                                  const float *__restrict__ img1, const float *__restrict__ img2,
                                                  SsimWindow w, float *__restrict__ maps, size_t plane_stride,
                                                  float2 *__restrict__ partial) {
    __shared__ float s_row[kSsWaves][2][kSsRowBuf];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int gw = blockIdx.x * kSsWaves + wv;
    if (gw >= planes * sx * sy) return;
    const SsStrip st = ss_strip(gw, sx, sy);
    const float *a = img1 + st.plane * plane_stride, *b = img2 + st.plane * plane_stride;
    float *m0 = maps + st.plane * plane_stride;
    const size_t map_stride = plane_stride * planes;  // the three maps are [3][planes][H][W]
    float *ra = s_row[wv][0], *rb = s_row[wv][1];
    const int gx = st.x0 + lane;
    const int nin = min(kSsRH, H - st.y0) + 2 * kSsR;  // input rows this strip streams
    float h[kSsTaps][5];   // ring of horizontal sums
    float ssum = 0.f, lsum = 0.f;
    // input rows prefetched 2 ahead into statically named registers (unroll by 2 x 11)
    float pf[2][4];
#pragma unroll
    for (int d = 0; d < 2; ++d) {
        ss_load_row(a, H, W, st.x0, st.y0 - kSsR + d, lane, pf[d][0], pf[d][1]);
        ss_load_row(b, H, W, st.x0, st.y0 - kSsR + d, lane, pf[d][2], pf[d][3]);
    }
    for (int base = 0; base < nin; base += 2 * kSsTaps) {
#pragma unroll
        for (int k = 0; k < 2 * kSsTaps; ++k) {
            const int i = base + k;  // input row index within the strip (wave-uniform)
            if (i >= nin) continue;
            const int slot = k % kSsTaps, d = k & 1;
            ra[lane] = pf[d][0]; rb[lane] = pf[d][2];
            if (lane < 16) { ra[64 + lane] = pf[d][1]; rb[64 + lane] = pf[d][3]; }
            if (i + 2 < nin) {
                ss_load_row(a, H, W, st.x0, st.y0 - kSsR + i + 2, lane, pf[d][0], pf[d][1]);
                ss_load_row(b, H, W, st.x0, st.y0 - kSsR + i + 2, lane, pf[d][2], pf[d][3]);
            }
            wave_lds_sync();
#pragma unroll
            for (int q = 0; q < 5; ++q) h[slot][q] = 0.f;
#pragma unroll
            for (int t = 0; t < kSsTaps; ++t) {
                const float x = ra[lane + t], y = rb[lane + t];
                // the centre pixel of input row i lies in output row i - 5 (L1 term)
                if (t == kSsR && i >= kSsR && i < nin - kSsR && gx < W) lsum += fabsf(x - y);
                h[slot][0] = fmaf(w.w[t], x, h[slot][0]);
                h[slot][1] = fmaf(w.w[t], y, h[slot][1]);
                h[slot][2] = fmaf(w.w[t], x * x, h[slot][2]);
                h[slot][3] = fmaf(w.w[t], y * y, h[slot][3]);
                h[slot][4] = fmaf(w.w[t], x * y, h[slot][4]);
            }
            wave_lds_sync();  // the row buffer is rewritten next iteration
            if (i >= 2 * kSsR) {  // output row o = i - 10: window rows i - 10 .. i
                float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int t = 0; t < kSsTaps; ++t) {
                    const int rs = (k + 1 + t) % kSsTaps;  // ring slot of row i - 10 + t
#pragma unroll
                    for (int q = 0; q < 5; ++q) acc[q] = fmaf(w.w[t], h[rs][q], acc[q]);
                }
                const int gy = st.y0 + i - 2 * kSsR;
                if (gx < W) {
                    const float mu1 = acc[0], mu2 = acc[1];
                    const float mu1_sq = mu1 * mu1, mu2_sq = mu2 * mu2, mu1_mu2 = mu1 * mu2;
                    const float sigma1_sq = acc[2] - mu1_sq, sigma2_sq = acc[3] - mu2_sq, sigma12 = acc[4] - mu1_mu2;
                    const float A = 2.f * mu1_mu2 + kSsC1, B = 2.f * sigma12 + kSsC2;
                    const float C = mu1_sq + mu2_sq + kSsC1, D = sigma1_sq + sigma2_sq + kSsC2;
                    const float inv = 1.f / (C * D);
                    const float S = (A * B) * inv;
                    ssum += S;
                    // S = A B / (C D): dS/dmu1 = (2 mu2 (B - A) - 2 mu1 S (D - C)) / (C D),
                    // dS/d<x^2> = -S / D, dS/d<xy> = 2 A / (C D)
                    const size_t p = (size_t)gy * W + gx;
                    m0[p] = (2.f * mu2 * (B - A) - 2.f * mu1 * S * (D - C)) * inv;
                    m0[map_stride + p] = -S / D;
                    m0[2 * map_stride + p] = 2.f * A * inv;
                }
            }
        }
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        ssum += __shfl_xor(ssum, d, 64);
        lsum += __shfl_xor(lsum, d, 64);
    }
    if (lane == 0) partial[gw] = make_float2(lsum, ssum);
}

// One block: *out_l1 = mean |x - y|, *out_ssim = mean S over n pixels (double accumulation, fixed order).
__global__ __launch_bounds__(256) void k_ssim_sum(int nb, const float2 *__restrict__ partial, double inv_n,
                                                  float *__restrict__ out_l1, float *__restrict__ out_ssim) {
    __shared__ double s_l[256], s_s[256];
    double l = 0, s = 0;
    for (int i = threadIdx.x; i < nb; i += 256) { l += partial[i].x; s += partial[i].y; }
    s_l[threadIdx.x] = l; s_s[threadIdx.x] = s;
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
        if ((int)threadIdx.x < d) { s_l[threadIdx.x] += s_l[threadIdx.x + d]; s_s[threadIdx.x] += s_s[threadIdx.x + d]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) { *out_l1 = (float)(s_l[0] * inv_n); *out_ssim = (float)(s_s[0] * inv_n); }
}

// ------------------------------------------------------------------------------------------
// Backward, same strips: stream the three derivative maps through the horizontal + register-ring
// vertical window and combine at each output pixel.
__global__ __launch_bounds__(256) void k_ssim_bwd(int planes, int H, int W, int sx, int sy,
                                                  const float *__restrict__ img1, const float *__restrict__ img2,
                                                  SsimWindow w, const float *__restrict__ maps, size_t plane_stride,
                                                  const float *__restrict__ g_l1, const float *__restrict__ g_ssim,
                                                  float inv_n, float *__restrict__ dimg1) {
    __shared__ float s_row[kSsWaves][3][kSsRowBuf];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int gw = blockIdx.x * kSsWaves + wv;
    if (gw >= planes * sx * sy) return;
    const SsStrip st = ss_strip(gw, sx, sy);
    const size_t map_stride = plane_stride * planes;
    const float gs = g_ssim ? g_ssim[0] * inv_n : 0.f;
    const float gl = g_l1 ? g_l1[0] * inv_n : 0.f;
    const float *a = img1 + st.plane * plane_stride, *b = img2 + st.plane * plane_stride;
    const float *mp = maps + st.plane * plane_stride;
    float *dst = dimg1 + st.plane * plane_stride;
    const int gx = st.x0 + lane;
    const int nout = min(kSsRH, H - st.y0);
    if (!g_ssim) {  // L1 term only
        if (gx < W)
            for (int o = 0; o < nout; ++o) {
                const size_t p = (size_t)(st.y0 + o) * W + gx;
                const float d = a[p] - b[p];
                dst[p] = gl * (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f));
            }
        return;
    }
    const int nin = nout + 2 * kSsR;
    float *r0 = s_row[wv][0], *r1 = s_row[wv][1], *r2 = s_row[wv][2];
    float h[kSsTaps][3];
    float pf[2][3][2];  // map rows prefetched 2 ahead (lo, hi halo)
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            ss_load_row(mp + j * map_stride, H, W, st.x0, st.y0 - kSsR + d, lane, pf[d][j][0], pf[d][j][1]);
    for (int base = 0; base < nin; base += 2 * kSsTaps) {
#pragma unroll
        for (int k = 0; k < 2 * kSsTaps; ++k) {
            const int i = base + k;
            if (i >= nin) continue;
            const int slot = k % kSsTaps, d = k & 1;
            r0[lane] = pf[d][0][0]; r1[lane] = pf[d][1][0]; r2[lane] = pf[d][2][0];
            if (lane < 16) { r0[64 + lane] = pf[d][0][1]; r1[64 + lane] = pf[d][1][1]; r2[64 + lane] = pf[d][2][1]; }
            if (i + 2 < nin) {
#pragma unroll
                for (int j = 0; j < 3; ++j)
                    ss_load_row(mp + j * map_stride, H, W, st.x0, st.y0 - kSsR + i + 2, lane, pf[d][j][0], pf[d][j][1]);
            }
            wave_lds_sync();
#pragma unroll
            for (int q = 0; q < 3; ++q) h[slot][q] = 0.f;
#pragma unroll
            for (int t = 0; t < kSsTaps; ++t) {
                h[slot][0] = fmaf(w.w[t], r0[lane + t], h[slot][0]);
                h[slot][1] = fmaf(w.w[t], r1[lane + t], h[slot][1]);
                h[slot][2] = fmaf(w.w[t], r2[lane + t], h[slot][2]);
            }
            wave_lds_sync();
            if (i >= 2 * kSsR) {
                float acc[3] = {0.f, 0.f, 0.f};
#pragma unroll
                for (int t = 0; t < kSsTaps; ++t) {
                    const int rs = (k + 1 + t) % kSsTaps;
#pragma unroll
                    for (int q = 0; q < 3; ++q) acc[q] = fmaf(w.w[t], h[rs][q], acc[q]);
                }
                if (gx < W) {
                    const size_t p = (size_t)(st.y0 + i - 2 * kSsR) * W + gx;
                    const float x = a[p], y = b[p];
                    const float dd = x - y;
                    const float sgn = dd > 0.f ? 1.f : (dd < 0.f ? -1.f : 0.f);
                    dst[p] = gs * (acc[0] + 2.f * x * acc[1] + y * acc[2]) + gl * sgn;
                }
            }
        }
    }
}

// ==========================================================================================
size_t ssim_partials(int planes, int H, int W) {
    return (size_t)planes * div_up(W, 64) * div_up(H, kSsRH);
}

hipError_t launch_ssim_fwd(int planes, int H, int W, const float *img1, const float *img2, const SsimWindow &w,
                           float *maps, float2 *partial, float *out_l1, float *out_ssim, hipStream_t s) {
    const int sx = div_up(W, 64), sy = div_up(H, kSsRH);
    const int nw = planes * sx * sy;
    const size_t ps = (size_t)H * W;
    k_ssim_fwd<<<div_up(nw, kSsWaves), 64 * kSsWaves, 0, s>>>(planes, H, W, sx, sy, img1, img2, w, maps, ps, partial);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    k_ssim_sum<<<1, 256, 0, s>>>(nw, partial, 1.0 / ((double)planes * ps), out_l1, out_ssim);
    return hipGetLastError();
}

hipError_t launch_ssim_bwd(int planes, int H, int W, const float *img1, const float *img2, const SsimWindow &w,
                           const float *maps, const float *g_l1, const float *g_ssim, float *dimg1,
                           hipStream_t s) {
    const int sx = div_up(W, 64), sy = div_up(H, kSsRH);
    const int nw = planes * sx * sy;
    const size_t ps = (size_t)H * W;
    k_ssim_bwd<<<div_up(nw, kSsWaves), 64 * kSsWaves, 0, s>>>(planes, H, W, sx, sy, img1, img2, w, maps, ps,
                                                              g_l1, g_ssim, (float)(1.0 / ((double)planes * ps)), dimg1);
    return hipGetLastError();
}

}  // namespace gsr
