// gsr_backward.hip -- backward pass of the MI355X-native Gaussian-splat rasterizer.
//
//   k_render_bwd  1 block (4 wave64) / 16x16 tile: per-pixel reverse walk (SURVEY.md 2.1 row
//                 renderCUDA bwd).  Instead of the reference's per-pixel float atomics into
//                 per-Gaussian buffers, every wave reduces its 64 pixels' 9 partials with DPP,
//                 the 4 wave sums are added in fixed order, and one 36-byte record per sorted
//                 (tile, Gaussian) slot is stored with plain coalesced stores: no global atomics,
//                 bitwise reproducible.
//   k_gauss_bwd   1 thread / Gaussian: sums its slot records in emission order (through the
//                 emission->slot map written by k_tile_sort), then the fused per-Gaussian chain
//                 computeCov2D bwd -> projection bwd -> SH bwd -> Sigma3D bwd (SURVEY.md 2.1 rows
//                 computeCov2DCUDA + preprocessCUDA bwd).  Writes every output element.
#include "gsr_common.h"
#include "gsr_internal.h"

namespace gsr {

constexpr int kBwdBatch = 128;  // Gaussians staged per LDS batch in the reverse walk

__global__ __launch_bounds__(256) void k_render_bwd(
    int W, int H, int gx, const uint2 *__restrict__ ranges, const uint32_t *__restrict__ point_list,
    const float2 *__restrict__ xy, const float4 *__restrict__ conic_op, const float4 *__restrict__ rgbd,
    const float *__restrict__ bg, const float *__restrict__ final_Ts,
    const uint32_t *__restrict__ n_contrib, const uint32_t *__restrict__ tile_maxc,
    const float *__restrict__ dL_dpixels, float *__restrict__ partial) {
    __shared__ float2 s_xy[kBwdBatch];
    __shared__ float4 s_co[kBwdBatch];
    __shared__ float4 s_col[kBwdBatch];
    __shared__ float s_acc[4][kPartial][kBwdBatch];  // per-wave sums, summed in fixed order
    const int tile = blockIdx.x;
    const uint2 rg = ranges[tile];
    const int n = (int)(rg.y - rg.x);
    if (n <= 0) return;
    const int tx = tile % gx, ty = tile / gx;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int px = tx * kTileW + (tid & 15), py = ty * kTileH + (tid >> 4);
    const bool inside = px < W && py < H;
    const int pid = py * W + px;
    const float pfx = (float)px, pfy = (float)py;
    const int maxc = min((int)tile_maxc[tile], n);
    // slots nobody in this tile reached get zero records
    for (int p = maxc + tid; p < n; p += blockDim.x) {
        float *dst = partial + (size_t)(rg.x + p) * kPartial;
#pragma unroll
        for (int k = 0; k < kPartial; ++k) dst[k] = 0.f;
    }
    const float ddelx_dx = (float)(0.5 * W), ddely_dy = (float)(0.5 * H);
    const float T_final = inside ? final_Ts[pid] : 0.f;
    float T = T_final;
    const uint32_t last_c = inside ? n_contrib[pid] : 0u;
    float dp0 = 0.f, dp1 = 0.f, dp2 = 0.f;
    if (inside) { dp0 = dL_dpixels[pid]; dp1 = dL_dpixels[H * W + pid]; dp2 = dL_dpixels[2 * H * W + pid]; }
    float bg_dot = 0;
    bg_dot += bg[0] * dp0; bg_dot += bg[1] * dp1; bg_dot += bg[2] * dp2;
    float ar0 = 0.f, ar1 = 0.f, ar2 = 0.f;       // accum_rec
    float lc0 = 0.f, lc1 = 0.f, lc2 = 0.f;       // last_color
    float last_alpha = 0.f;

    for (int end = maxc; end > 0; end -= kBwdBatch) {
        const int start = end > kBwdBatch ? end - kBwdBatch : 0;
        const int cnt = end - start;
        __syncthreads();  // previous batch fully consumed
        if (tid < cnt) {
            const uint32_t g = point_list[rg.x + start + tid];
            s_xy[tid] = xy[g];
            s_co[tid] = conic_op[g];
            s_col[tid] = rgbd[g];
        }
        for (int k = tid; k < 4 * kPartial * kBwdBatch; k += blockDim.x) (&s_acc[0][0][0])[k] = 0.f;
        __syncthreads();
        for (int j = cnt - 1; j >= 0; --j) {
            const uint32_t p = (uint32_t)(start + j);
            float v0 = 0, v1 = 0, v2 = 0, v3 = 0, v4 = 0, v5 = 0, v6 = 0, v7 = 0, v8 = 0;
            bool contrib = false;
            if (p < last_c) {
                const float2 q = s_xy[j];
                const float dx = q.x - pfx, dy = q.y - pfy;
                const float4 co = s_co[j];
                const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                if (power <= 0.0f) {
                    const float G = expf(power);
                    const float alpha = fminf(0.99f, co.w * G);
                    if (alpha >= 1.0f / 255.0f) {
                        contrib = true;
                        T = T / (1.f - alpha);
                        const float dchannel_dcolor = alpha * T;
                        const float4 c = s_col[j];
                        float dL_dalpha = 0.0f;
                        ar0 = last_alpha * lc0 + (1.f - last_alpha) * ar0; lc0 = c.x;
                        dL_dalpha += (c.x - ar0) * dp0; v6 = dchannel_dcolor * dp0;
                        ar1 = last_alpha * lc1 + (1.f - last_alpha) * ar1; lc1 = c.y;
                        dL_dalpha += (c.y - ar1) * dp1; v7 = dchannel_dcolor * dp1;
                        ar2 = last_alpha * lc2 + (1.f - last_alpha) * ar2; lc2 = c.z;
                        dL_dalpha += (c.z - ar2) * dp2; v8 = dchannel_dcolor * dp2;
                        dL_dalpha *= T;
                        last_alpha = alpha;
                        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                        const float dL_dG = co.w * dL_dalpha;
                        const float gdx = G * dx, gdy = G * dy;
                        const float dG_ddelx = -gdx * co.x - gdy * co.y;
                        const float dG_ddely = -gdy * co.z - gdx * co.y;
                        v0 = dL_dG * dG_ddelx * ddelx_dx;
                        v1 = dL_dG * dG_ddely * ddely_dy;
                        v2 = -0.5f * gdx * dx * dL_dG;
                        v3 = -0.5f * gdx * dy * dL_dG;
                        v4 = -0.5f * gdy * dy * dL_dG;
                        v5 = G * dL_dalpha;
                    }
                }
            }
            if (__ballot(contrib)) {  // wave-uniform: skip the reduction when no lane contributed
                v0 = wave_sum_lane63(v0); v1 = wave_sum_lane63(v1); v2 = wave_sum_lane63(v2);
                v3 = wave_sum_lane63(v3); v4 = wave_sum_lane63(v4); v5 = wave_sum_lane63(v5);
                v6 = wave_sum_lane63(v6); v7 = wave_sum_lane63(v7); v8 = wave_sum_lane63(v8);
                if (lane == 63) {
                    s_acc[wid][0][j] = v0; s_acc[wid][1][j] = v1; s_acc[wid][2][j] = v2;
                    s_acc[wid][3][j] = v3; s_acc[wid][4][j] = v4; s_acc[wid][5][j] = v5;
                    s_acc[wid][6][j] = v6; s_acc[wid][7][j] = v7; s_acc[wid][8][j] = v8;
                }
            }
        }
        __syncthreads();
        if (tid < cnt) {
            float *dst = partial + (size_t)(rg.x + start + tid) * kPartial;
#pragma unroll
            for (int k = 0; k < kPartial; ++k)
                dst[k] = ((s_acc[0][k][tid] + s_acc[1][k][tid]) + s_acc[2][k][tid]) + s_acc[3][k][tid];
        }
    }
}

// ------------------------------------------------------------------------------------------
__device__ inline float3 dnormvdv(float3 v, float3 dv) {
    const float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    return make_float3(((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32,
                       (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32,
                       (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32);
}

// SH backward; writes all M coefficient rows of dL_dsh (zeros past the active degree).
__device__ inline float3 sh_backward(int deg, int M, float3 mean, const float *campos,
                                     const float *__restrict__ sh, const bool *clamped,
                                     float3 dL_dcolor, float *__restrict__ dL_dsh) {
    const float3 d0 = make_float3(mean.x - campos[0], mean.y - campos[1], mean.z - campos[2]);
    const float len = sqrtf(d0.x * d0.x + d0.y * d0.y + d0.z * d0.z);
    const float x = d0.x / len, y = d0.y / len, z = d0.z / len;
    const float dRGB[3] = {dL_dcolor.x * (clamped[0] ? 0.f : 1.f), dL_dcolor.y * (clamped[1] ? 0.f : 1.f),
                           dL_dcolor.z * (clamped[2] ? 0.f : 1.f)};
    float dx[3] = {0, 0, 0}, dy[3] = {0, 0, 0}, dz[3] = {0, 0, 0};
    for (int k = 0; k < M * 3; ++k) dL_dsh[k] = 0.f;
#define SH(i, c) sh[(i) * 3 + (c)]
#define DSH(i, c) dL_dsh[(i) * 3 + (c)]
#pragma unroll
    for (int c = 0; c < 3; ++c) DSH(0, c) = GSR_SH_C0 * dRGB[c];
    if (deg > 0) {
        const float d1 = -GSR_SH_C1 * y, d2 = GSR_SH_C1 * z, d3 = -GSR_SH_C1 * x;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            DSH(1, c) = d1 * dRGB[c]; DSH(2, c) = d2 * dRGB[c]; DSH(3, c) = d3 * dRGB[c];
            dx[c] = -GSR_SH_C1 * SH(3, c); dy[c] = -GSR_SH_C1 * SH(1, c); dz[c] = GSR_SH_C1 * SH(2, c);
        }
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            const float d4 = kSH_C2[0] * xy, d5 = kSH_C2[1] * yz, d6 = kSH_C2[2] * (2.f * zz - xx - yy);
            const float d7 = kSH_C2[3] * xz, d8 = kSH_C2[4] * (xx - yy);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                DSH(4, c) = d4 * dRGB[c]; DSH(5, c) = d5 * dRGB[c]; DSH(6, c) = d6 * dRGB[c];
                DSH(7, c) = d7 * dRGB[c]; DSH(8, c) = d8 * dRGB[c];
                dx[c] += kSH_C2[0] * y * SH(4, c) + kSH_C2[2] * 2.f * -x * SH(6, c) + kSH_C2[3] * z * SH(7, c) +
                         kSH_C2[4] * 2.f * x * SH(8, c);
                dy[c] += kSH_C2[0] * x * SH(4, c) + kSH_C2[1] * z * SH(5, c) + kSH_C2[2] * 2.f * -y * SH(6, c) +
                         kSH_C2[4] * 2.f * -y * SH(8, c);
                dz[c] += kSH_C2[1] * y * SH(5, c) + kSH_C2[2] * 2.f * 2.f * z * SH(6, c) + kSH_C2[3] * x * SH(7, c);
            }
            if (deg > 2) {
                const float d9 = kSH_C3[0] * y * (3.f * xx - yy);
                const float d10 = kSH_C3[1] * xy * z;
                const float d11 = kSH_C3[2] * y * (4.f * zz - xx - yy);
                const float d12 = kSH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
                const float d13 = kSH_C3[4] * x * (4.f * zz - xx - yy);
                const float d14 = kSH_C3[5] * z * (xx - yy);
                const float d15 = kSH_C3[6] * x * (xx - 3.f * yy);
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    DSH(9, c) = d9 * dRGB[c]; DSH(10, c) = d10 * dRGB[c]; DSH(11, c) = d11 * dRGB[c];
                    DSH(12, c) = d12 * dRGB[c]; DSH(13, c) = d13 * dRGB[c]; DSH(14, c) = d14 * dRGB[c];
                    DSH(15, c) = d15 * dRGB[c];
                    dx[c] += (kSH_C3[0] * SH(9, c) * 3.f * 2.f * xy + kSH_C3[1] * SH(10, c) * yz +
                              kSH_C3[2] * SH(11, c) * -2.f * xy + kSH_C3[3] * SH(12, c) * -3.f * 2.f * xz +
                              kSH_C3[4] * SH(13, c) * (-3.f * xx + 4.f * zz - yy) +
                              kSH_C3[5] * SH(14, c) * 2.f * xz + kSH_C3[6] * SH(15, c) * 3.f * (xx - yy));
                    dy[c] += (kSH_C3[0] * SH(9, c) * 3.f * (xx - yy) + kSH_C3[1] * SH(10, c) * xz +
                              kSH_C3[2] * SH(11, c) * (-3.f * yy + 4.f * zz - xx) +
                              kSH_C3[3] * SH(12, c) * -3.f * 2.f * yz + kSH_C3[4] * SH(13, c) * -2.f * xy +
                              kSH_C3[5] * SH(14, c) * -2.f * yz + kSH_C3[6] * SH(15, c) * -3.f * 2.f * xy);
                    dz[c] += (kSH_C3[1] * SH(10, c) * xy + kSH_C3[2] * SH(11, c) * 4.f * 2.f * yz +
                              kSH_C3[3] * SH(12, c) * 3.f * (2.f * zz - xx - yy) +
                              kSH_C3[4] * SH(13, c) * 4.f * 2.f * xz + kSH_C3[5] * SH(14, c) * (xx - yy));
                }
            }
        }
    }
#undef SH
#undef DSH
    const float3 dL_ddir = make_float3(dx[0] * dRGB[0] + dx[1] * dRGB[1] + dx[2] * dRGB[2],
                                       dy[0] * dRGB[0] + dy[1] * dRGB[1] + dy[2] * dRGB[2],
                                       dz[0] * dRGB[0] + dz[1] * dRGB[1] + dz[2] * dRGB[2]);
    return dnormvdv(d0, dL_ddir);
}

__device__ inline void cov3d_backward(float3 s3, float mod, float4 q, const float *dc, float3 &dscale,
                                      float4 &drot) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    const m3 R = rot_from_quat(q);
    const float s[3] = {mod * s3.x, mod * s3.y, mod * s3.z};
    m3 S = {{0, 0, 0, 0, 0, 0, 0, 0, 0}};
    GM(S, 0, 0) = s[0]; GM(S, 1, 1) = s[1]; GM(S, 2, 2) = s[2];
    const m3 M = m3_mul(S, R);
    const m3 dSig = {{dc[0], 0.5f * dc[1], 0.5f * dc[2], 0.5f * dc[1], dc[3], 0.5f * dc[4], 0.5f * dc[2],
                      0.5f * dc[4], dc[5]}};
    m3 M2;
#pragma unroll
    for (int k = 0; k < 9; ++k) M2.m[k] = 2.0f * M.m[k];
    const m3 dM = m3_mul(M2, dSig);
    const m3 Rt = m3_T(R);
    m3 dMt = m3_T(dM);
    float ds[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        ds[i] = GM(Rt, i, 0) * GM(dMt, i, 0) + GM(Rt, i, 1) * GM(dMt, i, 1) + GM(Rt, i, 2) * GM(dMt, i, 2);
    dscale = make_float3(ds[0], ds[1], ds[2]);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) GM(dMt, i, rr) *= s[i];
#define G(c, rr) GM(dMt, c, rr)
    drot.x = 2 * z * (G(0, 1) - G(1, 0)) + 2 * y * (G(2, 0) - G(0, 2)) + 2 * x * (G(1, 2) - G(2, 1));
    drot.y = 2 * y * (G(1, 0) + G(0, 1)) + 2 * z * (G(2, 0) + G(0, 2)) + 2 * r * (G(1, 2) - G(2, 1)) -
             4 * x * (G(2, 2) + G(1, 1));
    drot.z = 2 * x * (G(1, 0) + G(0, 1)) + 2 * r * (G(2, 0) - G(0, 2)) + 2 * z * (G(1, 2) + G(2, 1)) -
             4 * y * (G(2, 2) + G(0, 0));
    drot.w = 2 * r * (G(0, 1) - G(1, 0)) + 2 * x * (G(2, 0) + G(0, 2)) + 2 * y * (G(1, 2) + G(2, 1)) -
             4 * z * (G(1, 1) + G(0, 0));
#undef G
}

__global__ __launch_bounds__(256) void k_gauss_bwd(
    int P, int D, int M, int W, int H, float scale_modifier, float tan_fovx, float tan_fovy,
    float h_x, float h_y, const float *__restrict__ means3D, const float *__restrict__ scales,
    const float *__restrict__ rotations, const float *__restrict__ shs,
    const float *__restrict__ cov3D_precomp, const float *__restrict__ viewmatrix,
    const float *__restrict__ projmatrix, const float *__restrict__ campos,
    const int *__restrict__ radii, const uint32_t *__restrict__ goff, const uint32_t *__restrict__ inv,
    const float *__restrict__ partial, float *__restrict__ dL_dmeans2D, float *__restrict__ dL_dcolors,
    float *__restrict__ dL_dopacity, float *__restrict__ dL_dmeans3D, float *__restrict__ dL_dcov3D,
    float *__restrict__ dL_dsh, float *__restrict__ dL_dscales, float *__restrict__ dL_drot) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    if (!(radii[i] > 0)) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            dL_dmeans2D[3 * i + k] = 0.f; dL_dcolors[3 * i + k] = 0.f; dL_dmeans3D[3 * i + k] = 0.f;
            dL_dscales[3 * i + k] = 0.f;
        }
        dL_dopacity[i] = 0.f;
#pragma unroll
        for (int k = 0; k < 6; ++k) dL_dcov3D[6 * i + k] = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) dL_drot[4 * i + k] = 0.f;
        if (dL_dsh)
            for (int k = 0; k < M * 3; ++k) dL_dsh[(size_t)i * M * 3 + k] = 0.f;
        return;
    }
    // ---- sum the slot records of this Gaussian in emission order ----
    float acc[kPartial];
#pragma unroll
    for (int k = 0; k < kPartial; ++k) acc[k] = 0.f;
    const uint32_t e0 = goff[i], e1 = goff[i + 1];
    for (uint32_t e = e0; e < e1; ++e) {
        const float *src = partial + (size_t)inv[e] * kPartial;
#pragma unroll
        for (int k = 0; k < kPartial; ++k) acc[k] += src[k];
    }
    dL_dmeans2D[3 * i] = acc[0]; dL_dmeans2D[3 * i + 1] = acc[1]; dL_dmeans2D[3 * i + 2] = 0.f;
    dL_dopacity[i] = acc[5];
    dL_dcolors[3 * i] = acc[6]; dL_dcolors[3 * i + 1] = acc[7]; dL_dcolors[3 * i + 2] = acc[8];
    const float dcx = acc[2], dcy = acc[3], dcz = acc[4];

    float vm[16], pj[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) { vm[k] = viewmatrix[k]; pj[k] = projmatrix[k]; }
    const float3 mean = make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
    float c3[6];
    float3 s3 = make_float3(0, 0, 0);
    float4 q = make_float4(0, 0, 0, 0);
    if (cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; ++k) c3[k] = cov3D_precomp[6 * i + k];
    } else {
        s3 = make_float3(scales[3 * i], scales[3 * i + 1], scales[3 * i + 2]);
        q = make_float4(rotations[4 * i], rotations[4 * i + 1], rotations[4 * i + 2], rotations[4 * i + 3]);
        cov3d_from_scale_rot(s3, scale_modifier, q, c3);
    }
    // ---- computeCov2DCUDA ----
    float3 t = xform4x3(mean, vm);
    const float limx = 1.3f * tan_fovx, limy = 1.3f * tan_fovy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float x_grad_mul = txtz < -limx || txtz > limx ? 0 : 1;
    const float y_grad_mul = tytz < -limy || tytz > limy ? 0 : 1;
    const m3 J = {{h_x / t.z, 0.0f, -(h_x * t.x) / (t.z * t.z), 0.0f, h_y / t.z,
                   -(h_y * t.y) / (t.z * t.z), 0, 0, 0}};
    const m3 Wm = {{vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]}};
    const m3 V = {{c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]}};
    const m3 T = m3_mul(Wm, J);
    const m3 c2 = m3_mul(m3_mul(m3_T(T), m3_T(V)), T);
    const float a = GM(c2, 0, 0) + 0.3f, b = GM(c2, 0, 1), c = GM(c2, 1, 1) + 0.3f;
    const float denom = a * c - b * b;
    float dL_da = 0, dL_db = 0, dL_dc = 0;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    float dcov[6];
#define TT(cc, rr) GM(T, cc, rr)
    if (denom2inv != 0) {
        dL_da = denom2inv * (-c * c * dcx + 2 * b * c * dcy + (denom - a * c) * dcz);
        dL_dc = denom2inv * (-a * a * dcz + 2 * a * b * dcy + (denom - a * c) * dcx);
        dL_db = denom2inv * 2 * (b * c * dcx - (denom + 2 * b * b) * dcy + a * b * dcz);
        dcov[0] = (TT(0, 0) * TT(0, 0) * dL_da + TT(0, 0) * TT(1, 0) * dL_db + TT(1, 0) * TT(1, 0) * dL_dc);
        dcov[3] = (TT(0, 1) * TT(0, 1) * dL_da + TT(0, 1) * TT(1, 1) * dL_db + TT(1, 1) * TT(1, 1) * dL_dc);
        dcov[5] = (TT(0, 2) * TT(0, 2) * dL_da + TT(0, 2) * TT(1, 2) * dL_db + TT(1, 2) * TT(1, 2) * dL_dc);
        dcov[1] = 2 * TT(0, 0) * TT(0, 1) * dL_da + (TT(0, 0) * TT(1, 1) + TT(0, 1) * TT(1, 0)) * dL_db +
                  2 * TT(1, 0) * TT(1, 1) * dL_dc;
        dcov[2] = 2 * TT(0, 0) * TT(0, 2) * dL_da + (TT(0, 0) * TT(1, 2) + TT(0, 2) * TT(1, 0)) * dL_db +
                  2 * TT(1, 0) * TT(1, 2) * dL_dc;
        dcov[4] = 2 * TT(0, 2) * TT(0, 1) * dL_da + (TT(0, 1) * TT(1, 2) + TT(0, 2) * TT(1, 1)) * dL_db +
                  2 * TT(1, 1) * TT(1, 2) * dL_dc;
    } else {
#pragma unroll
        for (int k = 0; k < 6; ++k) dcov[k] = 0;
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) dL_dcov3D[6 * i + k] = dcov[k];
#define VV(cc, rr) GM(V, cc, rr)
    const float dT00 = 2 * (TT(0, 0) * VV(0, 0) + TT(0, 1) * VV(0, 1) + TT(0, 2) * VV(0, 2)) * dL_da +
                       (TT(1, 0) * VV(0, 0) + TT(1, 1) * VV(0, 1) + TT(1, 2) * VV(0, 2)) * dL_db;
    const float dT01 = 2 * (TT(0, 0) * VV(1, 0) + TT(0, 1) * VV(1, 1) + TT(0, 2) * VV(1, 2)) * dL_da +
                       (TT(1, 0) * VV(1, 0) + TT(1, 1) * VV(1, 1) + TT(1, 2) * VV(1, 2)) * dL_db;
    const float dT02 = 2 * (TT(0, 0) * VV(2, 0) + TT(0, 1) * VV(2, 1) + TT(0, 2) * VV(2, 2)) * dL_da +
                       (TT(1, 0) * VV(2, 0) + TT(1, 1) * VV(2, 1) + TT(1, 2) * VV(2, 2)) * dL_db;
    const float dT10 = 2 * (TT(1, 0) * VV(0, 0) + TT(1, 1) * VV(0, 1) + TT(1, 2) * VV(0, 2)) * dL_dc +
                       (TT(0, 0) * VV(0, 0) + TT(0, 1) * VV(0, 1) + TT(0, 2) * VV(0, 2)) * dL_db;
    const float dT11 = 2 * (TT(1, 0) * VV(1, 0) + TT(1, 1) * VV(1, 1) + TT(1, 2) * VV(1, 2)) * dL_dc +
                       (TT(0, 0) * VV(1, 0) + TT(0, 1) * VV(1, 1) + TT(0, 2) * VV(1, 2)) * dL_db;
    const float dT12 = 2 * (TT(1, 0) * VV(2, 0) + TT(1, 1) * VV(2, 1) + TT(1, 2) * VV(2, 2)) * dL_dc +
                       (TT(0, 0) * VV(2, 0) + TT(0, 1) * VV(2, 1) + TT(0, 2) * VV(2, 2)) * dL_db;
#undef TT
#undef VV
#define WW(cc, rr) GM(Wm, cc, rr)
    const float dJ00 = WW(0, 0) * dT00 + WW(0, 1) * dT01 + WW(0, 2) * dT02;
    const float dJ02 = WW(2, 0) * dT00 + WW(2, 1) * dT01 + WW(2, 2) * dT02;
    const float dJ11 = WW(1, 0) * dT10 + WW(1, 1) * dT11 + WW(1, 2) * dT12;
    const float dJ12 = WW(2, 0) * dT10 + WW(2, 1) * dT11 + WW(2, 2) * dT12;
#undef WW
    const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    const float dL_dtx = x_grad_mul * -h_x * tz2 * dJ02;
    const float dL_dty = y_grad_mul * -h_y * tz2 * dJ12;
    const float dL_dtz = -h_x * tz2 * dJ00 - h_y * tz2 * dJ11 + (2 * h_x * t.x) * tz3 * dJ02 +
                         (2 * h_y * t.y) * tz3 * dJ12;
    float dm0 = vm[0] * dL_dtx + vm[1] * dL_dty + vm[2] * dL_dtz;
    float dm1 = vm[4] * dL_dtx + vm[5] * dL_dty + vm[6] * dL_dtz;
    float dm2 = vm[8] * dL_dtx + vm[9] * dL_dty + vm[10] * dL_dtz;
    // ---- preprocessCUDA bwd: screen-space mean -> means3D ----
    const float4 mh = xform4x4(mean, pj);
    const float m_w = 1.0f / (mh.w + 0.0000001f);
    const float mul1 = (pj[0] * mean.x + pj[4] * mean.y + pj[8] * mean.z + pj[12]) * m_w * m_w;
    const float mul2 = (pj[1] * mean.x + pj[5] * mean.y + pj[9] * mean.z + pj[13]) * m_w * m_w;
    const float g2x = acc[0], g2y = acc[1];
    dm0 += (pj[0] * m_w - pj[3] * mul1) * g2x + (pj[1] * m_w - pj[3] * mul2) * g2y;
    dm1 += (pj[4] * m_w - pj[7] * mul1) * g2x + (pj[5] * m_w - pj[7] * mul2) * g2y;
    dm2 += (pj[8] * m_w - pj[11] * mul1) * g2x + (pj[9] * m_w - pj[11] * mul2) * g2y;
    if (shs) {
        const float *sh = shs + (size_t)i * M * 3;
        bool cl[3];
        (void)sh_to_rgb(D, mean, campos, sh, cl);  // recompute the forward's clamp mask
        const float3 d = sh_backward(D, M, mean, campos, sh, cl, make_float3(acc[6], acc[7], acc[8]),
                                     dL_dsh + (size_t)i * M * 3);
        dm0 += d.x; dm1 += d.y; dm2 += d.z;
    } else if (dL_dsh) {
        for (int k = 0; k < M * 3; ++k) dL_dsh[(size_t)i * M * 3 + k] = 0.f;
    }
    dL_dmeans3D[3 * i] = dm0; dL_dmeans3D[3 * i + 1] = dm1; dL_dmeans3D[3 * i + 2] = dm2;
    if (scales && !cov3D_precomp) {
        float3 ds; float4 dr;
        cov3d_backward(s3, scale_modifier, q, dcov, ds, dr);
        dL_dscales[3 * i] = ds.x; dL_dscales[3 * i + 1] = ds.y; dL_dscales[3 * i + 2] = ds.z;
        dL_drot[4 * i] = dr.x; dL_drot[4 * i + 1] = dr.y; dL_drot[4 * i + 2] = dr.z; dL_drot[4 * i + 3] = dr.w;
    } else {
        dL_dscales[3 * i] = 0.f; dL_dscales[3 * i + 1] = 0.f; dL_dscales[3 * i + 2] = 0.f;
        dL_drot[4 * i] = 0.f; dL_drot[4 * i + 1] = 0.f; dL_drot[4 * i + 2] = 0.f; dL_drot[4 * i + 3] = 0.f;
    }
}

// ==========================================================================================
hipError_t launch_render_bwd(const BwdArgs &a, hipStream_t s) {
    const int T = a.gx * a.gy;
    if (a.K == 0) return hipSuccess;
    k_render_bwd<<<T, kTilePix, 0, s>>>(a.W, a.H, a.gx, a.ranges, a.point_list, a.xy, a.conic_op,
                                        a.rgbd, a.bg, a.final_T, a.n_contrib, a.tile_maxc,
                                        a.dL_dcolor, a.partial);
    return hipGetLastError();
}

hipError_t launch_gauss_bwd(const BwdArgs &a, hipStream_t s) {
    if (a.P == 0) return hipSuccess;
    k_gauss_bwd<<<div_up(a.P, 256), 256, 0, s>>>(
        a.P, a.D, a.M, a.W, a.H, a.scale_modifier, a.tan_fovx, a.tan_fovy, a.focal_x, a.focal_y,
        a.means3D, a.scales, a.rotations, a.shs, a.cov3D_precomp, a.viewmatrix, a.projmatrix, a.campos,
        a.radii, a.goff, a.inv, a.partial, a.dL_dmeans2D, a.dL_dcolors, a.dL_dopacity, a.dL_dmeans3D,
        a.dL_dcov3D, a.dL_dsh, a.dL_dscales, a.dL_drot);
    return hipGetLastError();
}

}  // namespace gsr
