/*
 * asan_check.c -- TEST INFRASTRUCTURE: drives every entry point of gsr_oracle.c on a small
 * deterministic scene (SH3 and precomputed-colour cases, a ragged image size, a cluster of
 * Gaussians on one tile) so that `make -C oracle asan` can run the oracle under AddressSanitizer +
 * UndefinedBehaviorSanitizer ("-fsanitize=address on the CPU oracle").  Prints one
 * checksum line per case; tests/test_oracle_asan.py runs the sanitized and the plain build and
 * requires a clean exit and identical checksums.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void ora_preprocess(int P, int D, int M, const float *means3D, const float *scales, float scale_modifier,
                    const float *rotations, const float *opacities, const float *shs,
                    const float *colors_precomp, const float *cov3D_precomp, const float *viewmatrix,
                    const float *projmatrix, const float *campos, int W, int H, float tan_fovx,
                    float tan_fovy, int prefiltered, float *depths, int *radii, float *xy,
                    float *conic_opacity, float *rgb, float *cov3Ds, unsigned char *clamped,
                    unsigned *tiles_touched, int *rects);
long ora_bin(int P, const float *depths, const int *radii, const int *rects,
             const unsigned *tiles_touched, int W, int H, unsigned *point_list, unsigned *ranges);
void ora_render(const unsigned *ranges, const unsigned *point_list, int W, int H, const float *xy,
                const float *features, const float *conic_opacity, const float *depths,
                const float *bg, float *out_color, float *out_depth, float *final_T,
                unsigned *n_contrib);
void ora_render_backward(const unsigned *ranges, const unsigned *point_list, int W, int H,
                         const float *bg, const float *xy, const float *conic_opacity,
                         const float *colors, const float *final_Ts, const unsigned *n_contrib,
                         const float *dL_dpixels, float *dL_dmean2D, float *dL_dconic,
                         float *dL_dopacity, float *dL_dcolors);
void ora_preprocess_backward(int P, int D, int M, const float *means3D, const int *radii,
                             const float *shs, const unsigned char *clamped, const float *scales,
                             const float *rotations, float scale_modifier, const float *cov3Ds,
                             const float *viewmatrix, const float *projmatrix, int W, int H,
                             float tan_fovx, float tan_fovy, const float *campos,
                             const float *dL_dmean2D, const float *dL_dconic, const float *dL_dcolor,
                             float *dL_dmeans3D, float *dL_dcov3D, float *dL_dsh, float *dL_dscale,
                             float *dL_drot);
void ora_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                      unsigned char *present);
int ora_set_threads(int n);

static unsigned long long rng = 88172645463325252ull;
static float urand(void) { /* xorshift64, [0, 1) */
    rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
    return (float)((rng >> 40) * (1.0 / 16777216.0));
}
static float nrand(void) { /* Box-Muller */
    float u = urand(), v = urand();
    if (u < 1e-7f) u = 1e-7f;
    return sqrtf(-2.f * logf(u)) * cosf(6.2831853f * v);
}
static double sumf(const float *a, size_t n) { double s = 0; for (size_t i = 0; i < n; ++i) s += a[i]; return s; }
static double sumu(const unsigned *a, size_t n) { double s = 0; for (size_t i = 0; i < n; ++i) s += a[i]; return s; }

static int run_case(const char *name, int P, int W, int H, int D, int cluster) {
    const int M = D >= 0 ? (D + 1) * (D + 1) : 0;
    float *means = malloc(sizeof(float) * 3 * P), *scales = malloc(sizeof(float) * 3 * P);
    float *rots = malloc(sizeof(float) * 4 * P), *op = malloc(sizeof(float) * P);
    float *cols = malloc(sizeof(float) * 3 * P), *sh = M ? malloc(sizeof(float) * 3 * M * P) : NULL;
    for (int i = 0; i < P; ++i) {
        const int c = cluster && i % 2 == 0;
        means[3 * i] = c ? 0.01f * nrand() : 4.4f * urand() - 2.2f;
        means[3 * i + 1] = c ? 0.01f * nrand() : 2.5f * urand() - 1.25f;
        means[3 * i + 2] = 2.f * urand() - 1.f;
        for (int k = 0; k < 3; ++k) scales[3 * i + k] = 0.03f * expf(0.3f * nrand());
        float q[4], n = 0;
        for (int k = 0; k < 4; ++k) { q[k] = nrand(); n += q[k] * q[k]; }
        n = sqrtf(n);
        for (int k = 0; k < 4; ++k) rots[4 * i + k] = q[k] / n;
        op[i] = 1.f / (1.f + expf(-nrand()));
        for (int k = 0; k < 3; ++k) cols[3 * i + k] = urand();
        for (int k = 0; k < 3 * M; ++k) sh[(size_t)3 * M * i + k] = k < 3 ? (urand() - 0.5f) / 0.28209479f : 0.05f * nrand();
    }
    /* camera: identity rotation, distance 4 (look_at(0, 0, 4)), f = W, principal point centred;
     * column-major viewmatrix (w2c^T) and projmatrix = viewmatrix * proj */
    const float f = (float)W, znear = 1.f, zfar = 100.f;
    float vm[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 4, 1};
    float pr[16] = {2 * f / W, 0, 0, 0, 0, 2 * f / H, 0, 0, 0, 0, zfar / (zfar - znear), 1,
                    0, 0, -(zfar * znear) / (zfar - znear), 0};
    float pm[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) {
            float s = 0;
            for (int k = 0; k < 4; ++k) s += pr[k * 4 + r] * vm[c * 4 + k];  /* proj @ w2c */
            pm[c * 4 + r] = s;
        }
    const float campos[3] = {0, 0, -4}, bg[3] = {0.1f, 0.2f, 0.3f};
    const float tfx = W / (2.f * f), tfy = H / (2.f * f);
    const int gx = (W + 15) / 16, gy = (H + 15) / 16, N = W * H;
    float *depths = calloc(P, sizeof(float)), *xy = calloc(2 * P, sizeof(float));
    float *conic = calloc(4 * P, sizeof(float)), *rgb = calloc(3 * P, sizeof(float));
    float *cov = calloc(6 * P, sizeof(float));
    int *radii = calloc(P, sizeof(int)), *rects = calloc(4 * P, sizeof(int));
    unsigned char *clamped = calloc(3 * P, 1), *vis = calloc(P, 1);
    unsigned *tiles = calloc(P, sizeof(unsigned)), *ranges = calloc(2 * gx * gy, sizeof(unsigned));
    ora_preprocess(P, D < 0 ? 0 : D, M, means, scales, 1.f, rots, op, sh, D < 0 ? cols : NULL, NULL, vm, pm,
                   campos, W, H, tfx, tfy, 0, depths, radii, xy, conic, rgb, cov, clamped, tiles, rects);
    long K = 0;
    for (int i = 0; i < P; ++i) K += tiles[i];
    unsigned *pl = calloc(K > 0 ? K : 1, sizeof(unsigned));
    const long K2 = ora_bin(P, depths, radii, rects, tiles, W, H, pl, ranges);
    if (K2 != K) { printf("%s: K mismatch %ld vs %ld\n", name, K2, K); return 1; }
    float *color = calloc(3 * N, sizeof(float)), *depth = calloc(N, sizeof(float)), *T = calloc(N, sizeof(float));
    unsigned *nc = calloc(N, sizeof(unsigned));
    const float *feats = D < 0 ? cols : rgb;
    ora_render(ranges, pl, W, H, xy, feats, conic, depths, bg, color, depth, T, nc);
    float *dpix = malloc(sizeof(float) * 3 * N);
    for (int k = 0; k < 3 * N; ++k) dpix[k] = nrand();
    float *dm2 = calloc(3 * P, sizeof(float)), *dcon = calloc(4 * P, sizeof(float));
    float *dop = calloc(P, sizeof(float)), *dcol = calloc(3 * P, sizeof(float));
    ora_render_backward(ranges, pl, W, H, bg, xy, conic, feats, T, nc, dpix, dm2, dcon, dop, dcol);
    float *dm3 = calloc(3 * P, sizeof(float)), *dcov = calloc(6 * P, sizeof(float));
    float *dsh = M ? calloc(3 * M * P, sizeof(float)) : NULL, *dsc = calloc(3 * P, sizeof(float));
    float *drot = calloc(4 * P, sizeof(float));
    ora_preprocess_backward(P, D < 0 ? 0 : D, M, means, radii, sh, clamped, scales, rots, 1.f, cov, vm, pm, W, H,
                            tfx, tfy, campos, dm2, dcon, dcol, dm3, dcov, dsh, dsc, drot);
    ora_mark_visible(P, means, vm, pm, vis);
    double nv = 0;
    for (int i = 0; i < P; ++i) nv += vis[i];
    printf("%s K=%ld ranges=%.17g color=%.17g depth=%.17g T=%.17g nc=%.17g dm2=%.17g dop=%.17g dcol=%.17g "
           "dm3=%.17g dcov=%.17g dsh=%.17g dsc=%.17g drot=%.17g vis=%.0f\n",
           name, K, sumu(ranges, 2 * gx * gy), sumf(color, 3 * N), sumf(depth, N), sumf(T, N), sumu(nc, N),
           sumf(dm2, 3 * P), sumf(dop, P), sumf(dcol, 3 * P), sumf(dm3, 3 * P), sumf(dcov, 6 * P),
           M ? sumf(dsh, 3 * M * P) : 0.0, sumf(dsc, 3 * P), sumf(drot, 4 * P), nv);
    free(means); free(scales); free(rots); free(op); free(cols); free(sh); free(depths); free(xy); free(conic);
    free(rgb); free(cov); free(radii); free(rects); free(clamped); free(vis); free(tiles); free(ranges); free(pl);
    free(color); free(depth); free(T); free(nc); free(dpix); free(dm2); free(dcon); free(dop); free(dcol);
    free(dm3); free(dcov); free(dsh); free(dsc); free(drot);
    return 0;
}

int main(void) {
    ora_set_threads(2);
    int rc = 0;
    rc |= run_case("rgb_ragged", 3000, 200, 120, -1, 0);
    rc |= run_case("sh3", 2000, 96, 80, 3, 0);
    rc |= run_case("cluster_long_tiles", 3000, 64, 64, -1, 1);
    return rc;
}
