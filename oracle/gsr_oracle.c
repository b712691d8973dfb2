/*
 * gsr_oracle.c -- CPU restatement of the differentiable Gaussian-splat rasterizer
 * (diff-gaussian-rasterization-w-depth) that bryanboateng/animating-gaussian-splats calls.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product path (libgsr.so) never calls it.
 *
 * PARITY STATUS: the rasterizer's own source is absent from /root/reference (the git submodule
 * /root/reference/diff-gaussian-rasterization-w-depth is empty, .gitmodules:1-3) and the reference
 * ships no tests or fixtures for it, so this restatement is "parity unpinned" against the reference
 * CUDA code.  It follows the behavioural spec in SURVEY.md sections 2.1 and 8(a) (upstream graphdeco
 * design + the -w-depth depth output), the reference call sites that fix the inputs
 * (shared.py:29-42 create_render_arguments, shared.py:64-124 create_render_settings,
 * train.py:354-364 / 506-547, densify.py:114-151) and the quaternion convention of
 * external.py:27-46 (build_rotation).  Its backward is pinned independently against torch.autograd
 * of a dense per-pixel restatement (tests/test_oracle_autograd.py), and the boundary callers are
 * pinned against golden vectors produced by the reference's own Python (tests/golden/).
 *
 * Conventions (all asserted by the tests):
 *   - matrices are 16 floats, column-major (the .contiguous() of the (1,4,4) transposed tensors of
 *     shared.py:80,110,120): x' = m[0]x + m[4]y + m[8]z + m[12]
 *   - 16x16 pixel tiles; sort key = (tile << 32) | float_bits(view depth); stable => ties by
 *     Gaussian index
 *   - every float expression is evaluated in the written order, no FMA contraction
 *     (built with -ffp-contract=off); the HIP kernels use the same order so integer outputs
 *     (radii, rects, tiles touched, point lists, tile ranges) are bit-exact.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define BX 16
#define BY 16

static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

/* ---- small column-major 3x3 helpers: m[c*3+r] is column c, row r (glm storage) ---- */
typedef struct { float m[9]; } mat3;

static mat3 mat3_mul(const mat3 *a, const mat3 *b) {
    /* (A*B)[c][r] = A[0][r]*B[c][0] + A[1][r]*B[c][1] + A[2][r]*B[c][2] */
    mat3 o;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r)
            o.m[c * 3 + r] = a->m[0 * 3 + r] * b->m[c * 3 + 0] + a->m[1 * 3 + r] * b->m[c * 3 + 1] +
                             a->m[2 * 3 + r] * b->m[c * 3 + 2];
    return o;
}
static mat3 mat3_T(const mat3 *a) {
    mat3 o;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) o.m[c * 3 + r] = a->m[r * 3 + c];
    return o;
}
#define M3(A, c, r) ((A).m[(c) * 3 + (r)])

static float ndc2pix(float v, int S) { return (float)(((v + 1.0) * S - 1.0) * 0.5); }

static void get_rect(float px, float py, int max_radius, int gx, int gy, int *rmin, int *rmax) {
    int a, b;
    a = (int)((px - max_radius) / BX); if (a < 0) a = 0; if (a > gx) a = gx; rmin[0] = a;
    b = (int)((py - max_radius) / BY); if (b < 0) b = 0; if (b > gy) b = gy; rmin[1] = b;
    a = (int)((px + max_radius + BX - 1) / BX); if (a < 0) a = 0; if (a > gx) a = gx; rmax[0] = a;
    b = (int)((py + max_radius + BY - 1) / BY); if (b < 0) b = 0; if (b > gy) b = gy; rmax[1] = b;
}

static void xform4x3(const float *p, const float *m, float *o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}
static void xform4x4(const float *p, const float *m, float *o) {
    xform4x3(p, m, o);
    o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}

/* Sigma = (S R)^T (S R) with R from the UNnormalised quaternion (w,x,y,z); output upper triangle. */
static void cov3d_from_scale_rot(const float *s3, float mod, const float *q, float *cov) {
    mat3 S = {{0}};
    M3(S, 0, 0) = mod * s3[0]; M3(S, 1, 1) = mod * s3[1]; M3(S, 2, 2) = mod * s3[2];
    float r = q[0], x = q[1], y = q[2], z = q[3];
    mat3 R = {{1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
               2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
               2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)}};
    mat3 M = mat3_mul(&S, &R);
    mat3 Mt = mat3_T(&M);
    mat3 Sig = mat3_mul(&Mt, &M);
    cov[0] = M3(Sig, 0, 0); cov[1] = M3(Sig, 0, 1); cov[2] = M3(Sig, 0, 2);
    cov[3] = M3(Sig, 1, 1); cov[4] = M3(Sig, 1, 2); cov[5] = M3(Sig, 2, 2);
}

/* EWA projection: 2D covariance (a, b, c) incl. the 0.3 low-pass. */
static void cov2d(const float *mean, float fx, float fy, float tfx, float tfy, const float *c3,
                  const float *vm, float *out) {
    float t[3];
    xform4x3(mean, vm, t);
    const float limx = 1.3f * tfx, limy = 1.3f * tfy;
    const float txtz = t[0] / t[2], tytz = t[1] / t[2];
    t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
    t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];
    mat3 J = {{fx / t[2], 0.0f, -(fx * t[0]) / (t[2] * t[2]), 0.0f, fy / t[2],
               -(fy * t[1]) / (t[2] * t[2]), 0, 0, 0}};
    mat3 W = {{vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]}};
    mat3 T = mat3_mul(&W, &J);
    mat3 V = {{c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]}};
    mat3 Tt = mat3_T(&T), Vt = mat3_T(&V);
    mat3 tmp = mat3_mul(&Tt, &Vt);
    mat3 cov = mat3_mul(&tmp, &T);
    out[0] = M3(cov, 0, 0) + 0.3f;
    out[1] = M3(cov, 0, 1);
    out[2] = M3(cov, 1, 1) + 0.3f;
}

static void sh_to_rgb(int deg, int max_coeffs, const float *mean, const float *campos,
                      const float *sh, float *rgb, unsigned char *clamped) {
    float dir[3] = {mean[0] - campos[0], mean[1] - campos[1], mean[2] - campos[2]};
    float len = sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    dir[0] = dir[0] / len; dir[1] = dir[1] / len; dir[2] = dir[2] / len;
    (void)max_coeffs;
    for (int ch = 0; ch < 3; ++ch) {
#define S(i) sh[(i) * 3 + ch]
        float res = SH_C0 * S(0);
        if (deg > 0) {
            float x = dir[0], y = dir[1], z = dir[2];
            res = res - SH_C1 * y * S(1) + SH_C1 * z * S(2) - SH_C1 * x * S(3);
            if (deg > 1) {
                float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
                res = res + SH_C2[0] * xy * S(4) + SH_C2[1] * yz * S(5) +
                      SH_C2[2] * (2.0f * zz - xx - yy) * S(6) + SH_C2[3] * xz * S(7) +
                      SH_C2[4] * (xx - yy) * S(8);
                if (deg > 2) {
                    res = res + SH_C3[0] * y * (3.0f * xx - yy) * S(9) + SH_C3[1] * xy * z * S(10) +
                          SH_C3[2] * y * (4.0f * zz - xx - yy) * S(11) +
                          SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * S(12) +
                          SH_C3[4] * x * (4.0f * zz - xx - yy) * S(13) +
                          SH_C3[5] * z * (xx - yy) * S(14) + SH_C3[6] * x * (xx - 3.0f * yy) * S(15);
                }
            }
        }
#undef S
        res += 0.5f;
        clamped[ch] = res < 0;
        rgb[ch] = res < 0.0f ? 0.0f : res;
    }
}

/* ======================================================================================
 * Forward: preprocess (SURVEY 2.1 row preprocessCUDA; callers train.py:359, densify.py:124)
 * ====================================================================================== */
void ora_preprocess(int P, int D, int M, const float *means3D, const float *scales, float scale_modifier,
                    const float *rotations, const float *opacities, const float *shs,
                    const float *colors_precomp, const float *cov3D_precomp, const float *viewmatrix,
                    const float *projmatrix, const float *campos, int W, int H, float tan_fovx,
                    float tan_fovy, int prefiltered, float *depths, int *radii, float *xy,
                    float *conic_opacity, float *rgb, float *cov3Ds, unsigned char *clamped,
                    unsigned *tiles_touched, int *rects) {
    (void)prefiltered;
    const float focal_y = H / (2.0f * tan_fovy);
    const float focal_x = W / (2.0f * tan_fovx);
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; ++i) {
        radii[i] = 0;
        tiles_touched[i] = 0;
        rects[4 * i + 0] = rects[4 * i + 1] = rects[4 * i + 2] = rects[4 * i + 3] = 0;
        const float *p = means3D + 3 * i;
        float ph[4], pv[3];
        xform4x4(p, projmatrix, ph);
        xform4x3(p, viewmatrix, pv);
        if (pv[2] <= 0.2f) continue; /* frustum cull (near) */
        const float pw = 1.0f / (ph[3] + 0.0000001f);
        const float pp[3] = {ph[0] * pw, ph[1] * pw, ph[2] * pw};
        const float *c3;
        if (cov3D_precomp) {
            c3 = cov3D_precomp + 6 * i;
        } else {
            cov3d_from_scale_rot(scales + 3 * i, scale_modifier, rotations + 4 * i, cov3Ds + 6 * i);
            c3 = cov3Ds + 6 * i;
        }
        float cv[3];
        cov2d(p, focal_x, focal_y, tan_fovx, tan_fovy, c3, viewmatrix, cv);
        const float det = cv[0] * cv[2] - cv[1] * cv[1];
        if (det == 0.0f) continue;
        const float det_inv = 1.f / det;
        const float conic[3] = {cv[2] * det_inv, -cv[1] * det_inv, cv[0] * det_inv};
        const float mid = 0.5f * (cv[0] + cv[2]);
        const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
        const float my_radius = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
        const float pix[2] = {ndc2pix(pp[0], W), ndc2pix(pp[1], H)};
        int rmin[2], rmax[2];
        get_rect(pix[0], pix[1], (int)my_radius, gx, gy, rmin, rmax);
        if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) continue;
        if (!colors_precomp) sh_to_rgb(D, M, p, campos, shs + (size_t)i * M * 3, rgb + 3 * i, clamped + 3 * i);
        depths[i] = pv[2];
        radii[i] = (int)my_radius;
        xy[2 * i] = pix[0]; xy[2 * i + 1] = pix[1];
        conic_opacity[4 * i + 0] = conic[0]; conic_opacity[4 * i + 1] = conic[1];
        conic_opacity[4 * i + 2] = conic[2]; conic_opacity[4 * i + 3] = opacities[i];
        tiles_touched[i] = (unsigned)((rmax[1] - rmin[1]) * (rmax[0] - rmin[0]));
        rects[4 * i + 0] = rmin[0]; rects[4 * i + 1] = rmin[1];
        rects[4 * i + 2] = rmax[0]; rects[4 * i + 3] = rmax[1];
    }
}

/* ======================================================================================
 * Forward: binning = inclusive scan + duplicateWithKeys + stable radix sort + tile ranges
 * (SURVEY 2.1 rows DeviceScan / duplicateWithKeys / SortPairs / identifyTileRanges).
 * A stable sort by (tile<<32 | depth bits) equals a sort by (key, emission index).
 * ====================================================================================== */
typedef struct { uint64_t key; uint32_t val; uint32_t emit; } ora_pair;

static int pair_cmp(const void *a, const void *b) {
    const ora_pair *x = (const ora_pair *)a, *y = (const ora_pair *)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->emit < y->emit ? -1 : (x->emit > y->emit);
}

/* returns num_rendered; point_list must hold sum(tiles_touched) entries, ranges 2*T entries.
 * The stable sort of all K (tile << 32 | depth bits) keys is done as a stable bucketing by tile
 * (emission order kept) followed by an independent sort of every tile's bucket by
 * (depth bits, emission index) -- the same total order, with the tiles sorted in parallel. */
long ora_bin(int P, const float *depths, const int *radii, const int *rects,
             const unsigned *tiles_touched, int W, int H, unsigned *point_list, unsigned *ranges) {
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    const int T = gx * gy;
    long K = 0;
    for (int i = 0; i < P; ++i) K += tiles_touched[i];
    memset(ranges, 0, sizeof(unsigned) * 2 * (size_t)T);
    if (K == 0) return 0;
    ora_pair *pairs = (ora_pair *)malloc(sizeof(ora_pair) * K);
    long *start = (long *)calloc((size_t)T + 1, sizeof(long));
    for (int i = 0; i < P; ++i) {  /* tile histogram */
        if (radii[i] <= 0) continue;
        for (int y = rects[4 * i + 1]; y < rects[4 * i + 3]; ++y)
            for (int x = rects[4 * i + 0]; x < rects[4 * i + 2]; ++x) ++start[y * gx + x + 1];
    }
    for (int t = 0; t < T; ++t) start[t + 1] += start[t];
    long *cur = (long *)malloc(sizeof(long) * ((size_t)T + 1));
    memcpy(cur, start, sizeof(long) * ((size_t)T + 1));
    long off = 0;  /* emission index: Gaussian order, rect y-major then x (duplicateWithKeys) */
    for (int i = 0; i < P; ++i) {
        if (radii[i] <= 0) continue;
        uint32_t dbits;
        memcpy(&dbits, depths + i, 4);
        for (int y = rects[4 * i + 1]; y < rects[4 * i + 3]; ++y)
            for (int x = rects[4 * i + 0]; x < rects[4 * i + 2]; ++x) {
                const int t = y * gx + x;
                ora_pair *q = pairs + cur[t]++;
                q->key = ((uint64_t)t << 32) | dbits;
                q->val = (uint32_t)i;
                q->emit = (uint32_t)off++;
            }
    }
#pragma omp parallel for schedule(dynamic, 16)
    for (int t = 0; t < T; ++t) {
        const long a = start[t], b = start[t + 1];
        if (b > a) qsort(pairs + a, (size_t)(b - a), sizeof(ora_pair), pair_cmp);
        for (long k = a; k < b; ++k) point_list[k] = pairs[k].val;
        if (b > a) { ranges[2 * t] = (unsigned)a; ranges[2 * t + 1] = (unsigned)b; }
    }
    free(cur);
    free(start);
    free(pairs);
    return K;
}

/* The blend weight's exponential.  The reference's renderCUDA calls CUDA's single-precision exp (a few
 * ulp, not correctly rounded; no CUDA here), glibc's expf is not correctly rounded either (<= 0.502
 * ulp), so neither gives the reference's bits.  The restatement uses the correctly rounded value -- the
 * double-precision exp rounded to float -- a definition independent of the libm at hand, which the GPU's
 * exact-threshold evaluations (gsr_common.h exact_blend, k_render_tsat) reproduce bit for bit. */
static inline float ora_expf(float x) { return (float)exp((double)x); }

/* ======================================================================================
 * Forward: front-to-back alpha blend of colour and depth (SURVEY 2.1 row renderCUDA fwd)
 * ====================================================================================== */
void ora_render(const unsigned *ranges, const unsigned *point_list, int W, int H, const float *xy,
                const float *features, const float *conic_opacity, const float *depths,
                const float *bg, float *out_color, float *out_depth, float *final_T,
                unsigned *n_contrib) {
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
#pragma omp parallel for collapse(2) schedule(dynamic, 4)
    for (int ty = 0; ty < gy; ++ty)
        for (int tx = 0; tx < gx; ++tx) {
            const unsigned r0 = ranges[2 * (ty * gx + tx)], r1 = ranges[2 * (ty * gx + tx) + 1];
            for (int py = ty * BY; py < ty * BY + BY && py < H; ++py)
                for (int px = tx * BX; px < tx * BX + BX && px < W; ++px) {
                    const float pfx = (float)px, pfy = (float)py;
                    float T = 1.0f, C[3] = {0, 0, 0}, Dp = 0;
                    unsigned contributor = 0, last = 0;
                    for (unsigned k = r0; k < r1; ++k) {
                        ++contributor;
                        const unsigned g = point_list[k];
                        const float dx = xy[2 * g] - pfx, dy = xy[2 * g + 1] - pfy;
                        const float *co = conic_opacity + 4 * g;
                        const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                        if (power > 0.0f) continue;
                        const float alpha = fminf(0.99f, co[3] * ora_expf(power));
                        if (alpha < 1.0f / 255.0f) continue;
                        const float test_T = T * (1 - alpha);
                        if (test_T < 0.0001f) break;
                        for (int ch = 0; ch < 3; ++ch) C[ch] += features[3 * g + ch] * alpha * T;
                        Dp += depths[g] * alpha * T;
                        T = test_T;
                        last = contributor;
                    }
                    const int pid = py * W + px;
                    final_T[pid] = T;
                    n_contrib[pid] = last;
                    for (int ch = 0; ch < 3; ++ch) out_color[ch * H * W + pid] = C[ch] + T * bg[ch];
                    out_depth[pid] = Dp;
                }
        }
}

/* ======================================================================================
 * Backward: reverse walk per pixel (SURVEY 2.1 row renderCUDA bwd).
 * Every pixel re-walks its tile list back to front from its n_contrib, recovering the
 * transmittance in front of each contributor by division, and forms the blend's partial
 * derivatives.  dL/dmean2D is in NDC units (x 0.5W, 0.5H); dL/dconic holds (a, b/2-convention, -, c).
 * The background term enters dL/dalpha; the 0.99 clamp is ignored in the gradient; the depth image
 * carries no gradient (the -w-depth reference discards it).
 * Summation: tiles run in parallel, each accumulating its own per-slot partials (a slot belongs to
 * one tile) over its pixels in row-major order; the slots are then added into the per-Gaussian
 * gradients serially in slot (tile-major) order -- fixed order, independent of the thread count.
 * (The reference used float atomics, whose order is unspecified.)
 * ====================================================================================== */
#define ORA_SLOT 9 /* per slot: dmean2D x,y; dconic a,b,c; dopacity; dcolour r,g,b */
void ora_render_backward(const unsigned *ranges, const unsigned *point_list, int W, int H,
                         const float *bg, const float *xy, const float *conic_opacity,
                         const float *colors, const float *final_Ts, const unsigned *n_contrib,
                         const float *dL_dpixels, float *dL_dmean2D, float *dL_dconic,
                         float *dL_dopacity, float *dL_dcolors) {
    const int gx = (W + BX - 1) / BX, gy = (H + BY - 1) / BY;
    const float ndc_sx = (float)(0.5 * W), ndc_sy = (float)(0.5 * H);
    long K = 0;
    for (int t = 0; t < gx * gy; ++t)
        if ((long)ranges[2 * t + 1] > K) K = (long)ranges[2 * t + 1];
    if (K == 0) return;
    float *slot = (float *)calloc((size_t)K * ORA_SLOT, sizeof(float));
#pragma omp parallel for collapse(2) schedule(dynamic, 4)
    for (int ty = 0; ty < gy; ++ty)
        for (int tx = 0; tx < gx; ++tx) {
            const unsigned r0 = ranges[2 * (ty * gx + tx)], r1 = ranges[2 * (ty * gx + tx) + 1];
            for (int py = ty * BY; py < ty * BY + BY && py < H; ++py)
                for (int px = tx * BX; px < tx * BX + BX && px < W; ++px) {
                    const int pid = py * W + px;
                    const float pfx = (float)px, pfy = (float)py;
                    const float t_end = final_Ts[pid];
                    float trans = t_end;
                    const unsigned n_used = n_contrib[pid];
                    /* colour seen behind the current contributor, and the contributor met just before
                     * it in this back-to-front walk (its alpha and colour) */
                    float behind[3] = {0, 0, 0}, gpix[3], prev_col[3] = {0, 0, 0};
                    float prev_alpha = 0;
                    for (int ch = 0; ch < 3; ++ch) gpix[ch] = dL_dpixels[ch * H * W + pid];
                    float bg_dot = 0;
                    for (int ch = 0; ch < 3; ++ch) bg_dot += bg[ch] * gpix[ch];
                    for (unsigned k = r1; k > r0; --k) {
                        const unsigned pos = k - 1 - r0; /* 0-based position in the tile list */
                        if (pos >= n_used) continue;
                        const unsigned g = point_list[k - 1];
                        const float dx = xy[2 * g] - pfx, dy = xy[2 * g + 1] - pfy;
                        const float *co = conic_opacity + 4 * g;
                        const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                        if (power > 0.0f) continue;
                        const float G = ora_expf(power);
                        const float alpha = fminf(0.99f, co[3] * G);
                        if (alpha < 1.0f / 255.0f) continue;
                        trans = trans / (1.f - alpha);
                        const float w_col = alpha * trans; /* d(pixel colour) / d(Gaussian colour) */
                        float *o = slot + (size_t)(k - 1) * ORA_SLOT;
                        float g_alpha = 0.0f;
                        for (int ch = 0; ch < 3; ++ch) {
                            const float c = colors[3 * g + ch];
                            behind[ch] = prev_alpha * prev_col[ch] + (1.f - prev_alpha) * behind[ch];
                            prev_col[ch] = c;
                            g_alpha += (c - behind[ch]) * gpix[ch];
                            o[6 + ch] += w_col * gpix[ch];
                        }
                        g_alpha *= trans;
                        prev_alpha = alpha;
                        g_alpha += (-t_end / (1.f - alpha)) * bg_dot;
                        const float g_gauss = co[3] * g_alpha; /* dL/dG */
                        const float gdx = G * dx, gdy = G * dy;
                        const float dG_dx = -gdx * co[0] - gdy * co[1];
                        const float dG_dy = -gdy * co[2] - gdx * co[1];
                        o[0] += g_gauss * dG_dx * ndc_sx;
                        o[1] += g_gauss * dG_dy * ndc_sy;
                        o[2] += -0.5f * gdx * dx * g_gauss;
                        o[3] += -0.5f * gdx * dy * g_gauss;
                        o[4] += -0.5f * gdy * dy * g_gauss;
                        o[5] += G * g_alpha;
                    }
                }
        }
    for (long k = 0; k < K; ++k) {
        const unsigned g = point_list[k];
        const float *o = slot + (size_t)k * ORA_SLOT;
        dL_dmean2D[3 * g + 0] += o[0];
        dL_dmean2D[3 * g + 1] += o[1];
        dL_dconic[4 * g + 0] += o[2];
        dL_dconic[4 * g + 1] += o[3];
        dL_dconic[4 * g + 3] += o[4];
        dL_dopacity[g] += o[5];
        for (int ch = 0; ch < 3; ++ch) dL_dcolors[3 * g + ch] += o[6 + ch];
    }
    free(slot);
}

/* ---- backward helpers ---- */
/* Chain rule through u = v / |v|: du/dv = (|v|^2 I - v v^T) / |v|^3, applied to the gradient g. */
static void unit_vec_bwd(const float *v, const float *g, float *o) {
    const float n2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    const float inv_n3 = 1.0f / sqrtf(n2 * n2 * n2);
    o[0] = ((+n2 - v[0] * v[0]) * g[0] - v[1] * v[0] * g[1] - v[2] * v[0] * g[2]) * inv_n3;
    o[1] = (-v[0] * v[1] * g[0] + (n2 - v[1] * v[1]) * g[1] - v[2] * v[1] * g[2]) * inv_n3;
    o[2] = (-v[0] * v[2] * g[0] - v[1] * v[2] * g[1] + (n2 - v[2] * v[2]) * g[2]) * inv_n3;
}

static void sh_backward(int deg, const float *mean, const float *campos, const float *sh,
                        const unsigned char *clamped, const float *dL_dcolor, float *dL_dmean,
                        float *dL_dsh) {
    float dir_orig[3] = {mean[0] - campos[0], mean[1] - campos[1], mean[2] - campos[2]};
    const float len = sqrtf(dir_orig[0] * dir_orig[0] + dir_orig[1] * dir_orig[1] + dir_orig[2] * dir_orig[2]);
    const float x = dir_orig[0] / len, y = dir_orig[1] / len, z = dir_orig[2] / len;
    float dRGB[3];
    for (int c = 0; c < 3; ++c) dRGB[c] = dL_dcolor[c] * (clamped[c] ? 0.f : 1.f);
    float dx[3] = {0, 0, 0}, dy[3] = {0, 0, 0}, dz[3] = {0, 0, 0};
#define SH(i, c) sh[(i) * 3 + (c)]
#define DSH(i, c) dL_dsh[(i) * 3 + (c)]
    for (int c = 0; c < 3; ++c) DSH(0, c) = SH_C0 * dRGB[c];
    if (deg > 0) {
        const float d1 = -SH_C1 * y, d2 = SH_C1 * z, d3 = -SH_C1 * x;
        for (int c = 0; c < 3; ++c) {
            DSH(1, c) = d1 * dRGB[c]; DSH(2, c) = d2 * dRGB[c]; DSH(3, c) = d3 * dRGB[c];
            dx[c] = -SH_C1 * SH(3, c); dy[c] = -SH_C1 * SH(1, c); dz[c] = SH_C1 * SH(2, c);
        }
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            const float d4 = SH_C2[0] * xy, d5 = SH_C2[1] * yz, d6 = SH_C2[2] * (2.f * zz - xx - yy);
            const float d7 = SH_C2[3] * xz, d8 = SH_C2[4] * (xx - yy);
            for (int c = 0; c < 3; ++c) {
                DSH(4, c) = d4 * dRGB[c]; DSH(5, c) = d5 * dRGB[c]; DSH(6, c) = d6 * dRGB[c];
                DSH(7, c) = d7 * dRGB[c]; DSH(8, c) = d8 * dRGB[c];
                dx[c] += SH_C2[0] * y * SH(4, c) + SH_C2[2] * 2.f * -x * SH(6, c) + SH_C2[3] * z * SH(7, c) +
                         SH_C2[4] * 2.f * x * SH(8, c);
                dy[c] += SH_C2[0] * x * SH(4, c) + SH_C2[1] * z * SH(5, c) + SH_C2[2] * 2.f * -y * SH(6, c) +
                         SH_C2[4] * 2.f * -y * SH(8, c);
                dz[c] += SH_C2[1] * y * SH(5, c) + SH_C2[2] * 2.f * 2.f * z * SH(6, c) + SH_C2[3] * x * SH(7, c);
            }
            if (deg > 2) {
                const float d9 = SH_C3[0] * y * (3.f * xx - yy);
                const float d10 = SH_C3[1] * xy * z;
                const float d11 = SH_C3[2] * y * (4.f * zz - xx - yy);
                const float d12 = SH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
                const float d13 = SH_C3[4] * x * (4.f * zz - xx - yy);
                const float d14 = SH_C3[5] * z * (xx - yy);
                const float d15 = SH_C3[6] * x * (xx - 3.f * yy);
                for (int c = 0; c < 3; ++c) {
                    DSH(9, c) = d9 * dRGB[c]; DSH(10, c) = d10 * dRGB[c]; DSH(11, c) = d11 * dRGB[c];
                    DSH(12, c) = d12 * dRGB[c]; DSH(13, c) = d13 * dRGB[c]; DSH(14, c) = d14 * dRGB[c];
                    DSH(15, c) = d15 * dRGB[c];
                    dx[c] += (SH_C3[0] * SH(9, c) * 3.f * 2.f * xy + SH_C3[1] * SH(10, c) * yz +
                              SH_C3[2] * SH(11, c) * -2.f * xy + SH_C3[3] * SH(12, c) * -3.f * 2.f * xz +
                              SH_C3[4] * SH(13, c) * (-3.f * xx + 4.f * zz - yy) +
                              SH_C3[5] * SH(14, c) * 2.f * xz + SH_C3[6] * SH(15, c) * 3.f * (xx - yy));
                    dy[c] += (SH_C3[0] * SH(9, c) * 3.f * (xx - yy) + SH_C3[1] * SH(10, c) * xz +
                              SH_C3[2] * SH(11, c) * (-3.f * yy + 4.f * zz - xx) +
                              SH_C3[3] * SH(12, c) * -3.f * 2.f * yz + SH_C3[4] * SH(13, c) * -2.f * xy +
                              SH_C3[5] * SH(14, c) * -2.f * yz + SH_C3[6] * SH(15, c) * -3.f * 2.f * xy);
                    dz[c] += (SH_C3[1] * SH(10, c) * xy + SH_C3[2] * SH(11, c) * 4.f * 2.f * yz +
                              SH_C3[3] * SH(12, c) * 3.f * (2.f * zz - xx - yy) +
                              SH_C3[4] * SH(13, c) * 4.f * 2.f * xz + SH_C3[5] * SH(14, c) * (xx - yy));
                }
            }
        }
    }
#undef SH
#undef DSH
    const float dL_ddir[3] = {dx[0] * dRGB[0] + dx[1] * dRGB[1] + dx[2] * dRGB[2],
                              dy[0] * dRGB[0] + dy[1] * dRGB[1] + dy[2] * dRGB[2],
                              dz[0] * dRGB[0] + dz[1] * dRGB[1] + dz[2] * dRGB[2]};
    float dm[3];
    unit_vec_bwd(dir_orig, dL_ddir, dm);
    dL_dmean[0] += dm[0]; dL_dmean[1] += dm[1]; dL_dmean[2] += dm[2];
}

static void cov3d_backward(const float *s3, float mod, const float *q, const float *dL_dcov3D,
                           float *dL_dscale, float *dL_drot) {
    const float r = q[0], x = q[1], y = q[2], z = q[3];
    mat3 R = {{1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
               2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
               2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)}};
    const float s[3] = {mod * s3[0], mod * s3[1], mod * s3[2]};
    mat3 S = {{0}};
    M3(S, 0, 0) = s[0]; M3(S, 1, 1) = s[1]; M3(S, 2, 2) = s[2];
    mat3 M = mat3_mul(&S, &R);
    const float *d = dL_dcov3D;
    mat3 dSig = {{d[0], 0.5f * d[1], 0.5f * d[2], 0.5f * d[1], d[3], 0.5f * d[4], 0.5f * d[2],
                  0.5f * d[4], d[5]}};
    mat3 M2;
    for (int k = 0; k < 9; ++k) M2.m[k] = 2.0f * M.m[k];
    mat3 dM = mat3_mul(&M2, &dSig);
    mat3 Rt = mat3_T(&R), dMt = mat3_T(&dM);
    for (int i = 0; i < 3; ++i)
        dL_dscale[i] = M3(Rt, i, 0) * M3(dMt, i, 0) + M3(Rt, i, 1) * M3(dMt, i, 1) + M3(Rt, i, 2) * M3(dMt, i, 2);
    for (int i = 0; i < 3; ++i)
        for (int rr = 0; rr < 3; ++rr) M3(dMt, i, rr) *= s[i];
#define G(c, rr) M3(dMt, c, rr)
    dL_drot[0] = 2 * z * (G(0, 1) - G(1, 0)) + 2 * y * (G(2, 0) - G(0, 2)) + 2 * x * (G(1, 2) - G(2, 1));
    dL_drot[1] = 2 * y * (G(1, 0) + G(0, 1)) + 2 * z * (G(2, 0) + G(0, 2)) + 2 * r * (G(1, 2) - G(2, 1)) -
                 4 * x * (G(2, 2) + G(1, 1));
    dL_drot[2] = 2 * x * (G(1, 0) + G(0, 1)) + 2 * r * (G(2, 0) - G(0, 2)) + 2 * z * (G(1, 2) + G(2, 1)) -
                 4 * y * (G(2, 2) + G(0, 0));
    dL_drot[3] = 2 * r * (G(0, 1) - G(1, 0)) + 2 * x * (G(2, 0) + G(0, 2)) + 2 * y * (G(1, 2) + G(2, 1)) -
                 4 * z * (G(1, 1) + G(0, 0));
#undef G
}

/* ======================================================================================
 * Backward: per Gaussian (SURVEY 2.1 rows computeCov2DCUDA + preprocessCUDA bwd)
 * ====================================================================================== */
void ora_preprocess_backward(int P, int D, int M, const float *means3D, const int *radii,
                             const float *shs, const unsigned char *clamped, const float *scales,
                             const float *rotations, float scale_modifier, const float *cov3Ds,
                             const float *viewmatrix, const float *projmatrix, int W, int H,
                             float tan_fovx, float tan_fovy, const float *campos,
                             const float *dL_dmean2D, const float *dL_dconic, const float *dL_dcolor,
                             float *dL_dmeans3D, float *dL_dcov3D, float *dL_dsh, float *dL_dscale,
                             float *dL_drot) {
    const float h_y = H / (2.0f * tan_fovy);
    const float h_x = W / (2.0f * tan_fovx);
    const float *vm = viewmatrix, *pj = projmatrix;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; ++i) {
        if (!(radii[i] > 0)) continue;
        /* ---- dL/dconic -> dL/dSigma2D -> dL/dSigma3D and the mean's share through J (SURVEY 2.1 computeCov2DCUDA) ---- */
        const float *c3 = cov3Ds + 6 * i;
        const float *mean = means3D + 3 * i;
        const float dcx = dL_dconic[4 * i], dcy = dL_dconic[4 * i + 1], dcz = dL_dconic[4 * i + 3];
        float t[3];
        xform4x3(mean, vm, t);
        const float limx = 1.3f * tan_fovx, limy = 1.3f * tan_fovy;
        const float txtz = t[0] / t[2], tytz = t[1] / t[2];
        t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
        t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];
        const float keep_tx = txtz < -limx || txtz > limx ? 0 : 1;
        const float keep_ty = tytz < -limy || tytz > limy ? 0 : 1;
        mat3 J = {{h_x / t[2], 0.0f, -(h_x * t[0]) / (t[2] * t[2]), 0.0f, h_y / t[2],
                   -(h_y * t[1]) / (t[2] * t[2]), 0, 0, 0}};
        mat3 Wm = {{vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]}};
        mat3 V = {{c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]}};
        mat3 T = mat3_mul(&Wm, &J);
        mat3 Tt = mat3_T(&T), Vt = mat3_T(&V);
        mat3 tmp = mat3_mul(&Tt, &Vt);
        mat3 c2 = mat3_mul(&tmp, &T);
        const float a = M3(c2, 0, 0) + 0.3f, b = M3(c2, 0, 1), c = M3(c2, 1, 1) + 0.3f;
        const float denom = a * c - b * b;
        float dL_da = 0, dL_db = 0, dL_dc = 0;
        const float inv_det2 = 1.0f / ((denom * denom) + 0.0000001f);
        float *dcov = dL_dcov3D + 6 * i;
        if (inv_det2 != 0) {
            dL_da = inv_det2 * (-c * c * dcx + 2 * b * c * dcy + (denom - a * c) * dcz);
            dL_dc = inv_det2 * (-a * a * dcz + 2 * a * b * dcy + (denom - a * c) * dcx);
            dL_db = inv_det2 * 2 * (b * c * dcx - (denom + 2 * b * b) * dcy + a * b * dcz);
#define TT(cc, rr) M3(T, cc, rr)
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
            for (int k = 0; k < 6; ++k) dcov[k] = 0;
        }
#define VV(cc, rr) M3(V, cc, rr)
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
#define WW(cc, rr) M3(Wm, cc, rr)
        const float dJ00 = WW(0, 0) * dT00 + WW(0, 1) * dT01 + WW(0, 2) * dT02;
        const float dJ02 = WW(2, 0) * dT00 + WW(2, 1) * dT01 + WW(2, 2) * dT02;
        const float dJ11 = WW(1, 0) * dT10 + WW(1, 1) * dT11 + WW(1, 2) * dT12;
        const float dJ12 = WW(2, 0) * dT10 + WW(2, 1) * dT11 + WW(2, 2) * dT12;
#undef WW
        const float tz = 1.f / t[2], tz2 = tz * tz, tz3 = tz2 * tz;
        const float dL_dtx = keep_tx * -h_x * tz2 * dJ02;
        const float dL_dty = keep_ty * -h_y * tz2 * dJ12;
        const float dL_dtz = -h_x * tz2 * dJ00 - h_y * tz2 * dJ11 + (2 * h_x * t[0]) * tz3 * dJ02 +
                             (2 * h_y * t[1]) * tz3 * dJ12;
        float *dm = dL_dmeans3D + 3 * i;
        /* back through the view rotation: W^T (dL/dt) */
        dm[0] = vm[0] * dL_dtx + vm[1] * dL_dty + vm[2] * dL_dtz;
        dm[1] = vm[4] * dL_dtx + vm[5] * dL_dty + vm[6] * dL_dtz;
        dm[2] = vm[8] * dL_dtx + vm[9] * dL_dty + vm[10] * dL_dtz;

        /* ---- screen-space mean -> means3D through the projection (SURVEY 2.1 preprocessCUDA bwd) ---- */
        float mh[4];
        xform4x4(mean, pj, mh);
        const float m_w = 1.0f / (mh[3] + 0.0000001f);
        const float mul1 = (pj[0] * mean[0] + pj[4] * mean[1] + pj[8] * mean[2] + pj[12]) * m_w * m_w;
        const float mul2 = (pj[1] * mean[0] + pj[5] * mean[1] + pj[9] * mean[2] + pj[13]) * m_w * m_w;
        const float g2x = dL_dmean2D[3 * i], g2y = dL_dmean2D[3 * i + 1];
        const float dmx = (pj[0] * m_w - pj[3] * mul1) * g2x + (pj[1] * m_w - pj[3] * mul2) * g2y;
        const float dmy = (pj[4] * m_w - pj[7] * mul1) * g2x + (pj[5] * m_w - pj[7] * mul2) * g2y;
        const float dmz = (pj[8] * m_w - pj[11] * mul1) * g2x + (pj[9] * m_w - pj[11] * mul2) * g2y;
        dm[0] += dmx; dm[1] += dmy; dm[2] += dmz;
        if (shs)
            sh_backward(D, mean, campos, shs + (size_t)i * M * 3, clamped + 3 * i, dL_dcolor + 3 * i, dm,
                        dL_dsh + (size_t)i * M * 3);
        if (scales)
            cov3d_backward(scales + 3 * i, scale_modifier, rotations + 4 * i, dcov, dL_dscale + 3 * i,
                           dL_drot + 4 * i);
    }
}

/* markVisible: near-plane frustum test only (SURVEY 2.1 row checkFrustum / markVisible) */
void ora_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                      unsigned char *present) {
    (void)projmatrix;
    for (int i = 0; i < P; ++i) {
        float pv[3];
        xform4x3(means3D + 3 * i, viewmatrix, pv);
        present[i] = !(pv[2] <= 0.2f);
    }
}

/* OpenMP threads of the oracle's parallel loops (bench.py's cpu_baseline leg sets the host's core
 * count; OMP_NUM_THREADS only applies before the runtime's first parallel region).  Returns the
 * count the next parallel region will use. */
int ora_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}
