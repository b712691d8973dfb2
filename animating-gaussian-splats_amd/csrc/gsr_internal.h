// gsr_internal.h -- argument bundles and host launchers shared by the libgsr translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsr {

struct FwdArgs {
    // inputs
    int P, D, M, W, H, gx, gy, act;
    float scale_modifier, tan_fovx, tan_fovy, focal_x, focal_y;
    const float *means3D, *scales, *rotations, *opacities, *shs, *colors_precomp, *cov3D_precomp;
    const float *viewmatrix, *projmatrix, *campos, *bg;
    CamStrides cs;
    // geom
    float *depth; float4 *rec; uint2 *rect; uint32_t *tiles; uint32_t *goff; uint8_t *clampm;
    // image
    uint2 *ranges; float4 *pix_end; uint32_t *n_contrib; uint32_t *tile_maxc;
    uint32_t *tile_order_f; uint32_t *seg_off; uint32_t *sort_lists; uint32_t *tile_count;
    uint32_t *tile_cursor; uint32_t *block_sums; uint32_t *block_off; uint32_t *meta; uint32_t *chunk_off;
    uint32_t *items_ws; uint32_t *scan_ws; uint32_t *tile_rank;
    // exact-threshold mode: per tile, the count of near-threshold weights k_render_fwd re-evaluated, and
    // their records (kNearCap per tile: key (list position << 8 | pixel), power, G, alpha)
    uint32_t *tile_flag; float4 *near_rec;
    // exact-threshold mode: pixels whose final T lies within t_window of 1e-4, redone by k_render_tsat
    // (count in items_ws[kTSatCtr])
    uint32_t *tsat_list;
    // binning
    uint4 *pairs; uint32_t *point_list; uint32_t *slot_emit; float4 *seg_state;
    // outputs
    int *radii; float *out_color; float *out_depth;
    // speculative enqueue (gsr_forward_info with speculate): the BINNING capacity the post-scan kernels
    // were queued with before the host read K (0: exact path), and the device flag they check
    // (meta + 1, written by k_bin_scan; nullptr: exact path)
    uint32_t spec_cap; const uint32_t *spec_ok;
    uint32_t spec_sort_blocks;  // grid of the speculative k_tile_sort (<= kSpecSortBlocks; 0: that bound)
    // asynchronous forward (gsr_forward_async): the gate word the speculative render's first wave waits
    // on when the speculation failed, the value that opens it, the forward's timeout error word (set to
    // gate_seq when the gate is abandoned) and the timeout (s_memrealtime ticks, 100 MHz)
    const uint32_t *gate; uint32_t gate_seq; uint32_t *gate_err; uint64_t gate_timeout;
    // exact-threshold mode (gsr_set_exact_thresholds, on by default): near-threshold weights
    // re-evaluated in the reference's expression order
    int exact;
};
// blocks of the speculative k_tile_sort launch (they loop over the device-side list count)
constexpr int kSpecSortBlocks = 512;

struct BwdArgs {
    int P, D, M, W, H, gx, gy, K, act;
    float scale_modifier, tan_fovx, tan_fovy, focal_x, focal_y;
    const float *means3D, *scales, *rotations, *shs, *colors_precomp, *cov3D_precomp;
    const float *viewmatrix, *projmatrix, *campos, *bg;
    CamStrides cs;
    const int *radii;
    // saved state
    const float4 *rec; const uint2 *rect; const uint8_t *clampm;
    const uint32_t *goff; const uint2 *ranges; const float4 *pix_end; const uint32_t *n_contrib;
    const uint32_t *tile_maxc; const uint32_t *tile_flag; const float4 *near_rec; const uint32_t *seg_off; const uint32_t *meta; uint32_t *items_ws;
    const uint32_t *point_list; const uint32_t *slot_emit; const float4 *seg_state;
    uint2 *items; uint32_t max_items;
    // scratch
    float4 *part;
    // upstream gradient
    const float *dL_dcolor;
    // outputs
    float *dL_dmeans2D, *dL_dcolors, *dL_dopacity, *dL_dmeans3D, *dL_dcov3D, *dL_dsh, *dL_dscales,
        *dL_drot;
    int accm;  // gsr_grad_bits: outputs accumulated into instead of overwritten
    const uint32_t *spec_ok;  // speculative render half (pair count unknown): kernels return when the forward's speculation failed
};

hipError_t launch_preprocess(const FwdArgs &a, hipStream_t s);
hipError_t launch_bin_count(const FwdArgs &a, hipStream_t s);
hipError_t launch_bin_scan(const FwdArgs &a, uint32_t *host_words, hipStream_t s);
hipError_t launch_bin_emit(const FwdArgs &a, int K, hipStream_t s);
hipError_t launch_tile_sort(const FwdArgs &a, uint32_t n_mid, uint32_t n_vlong, uint32_t max_n, uint4 *tmp,
                            hipStream_t s);
hipError_t launch_render_fwd(const FwdArgs &a, hipStream_t s);
hipError_t launch_zero(float *p, size_t n, hipStream_t s);
hipError_t launch_mark_visible(int P, const float *means3D, const float *viewmatrix, uint8_t *present,
                               hipStream_t s);

hipError_t launch_bwd_items(const BwdArgs &a, hipStream_t s);
hipError_t launch_bwd_items_raw(int K, int T, int P, const uint2 *ranges, const uint32_t *tile_maxc,
                                const uint32_t *tile_flag, uint2 *items, uint32_t *ws, hipStream_t s,
                                const uint32_t *spec_ok = nullptr);
hipError_t launch_render_bwd(const BwdArgs &a, hipStream_t s);
hipError_t launch_gauss_bwd(const BwdArgs &a, hipStream_t s);
// Each Gaussian's per-pair records of one view summed in emission order into kPartial x P SoA sums
// (the deferred multi-view pass reads these instead of walking the records itself).
hipError_t launch_sum_records(int P, const uint32_t *goff, const float4 *part, float *sums, hipStream_t s,
                              const uint32_t *spec_ok, const float *viewmatrix, const float *projmatrix,
                              const float *campos, CamStrides cs, int W, int H);

// Per-Gaussian backward over several views of the same Gaussians (gsr_backward_gaussians): one
// launch reads the parameters and read-modify-writes every gradient once for up to kMultiViews views.
constexpr int kMultiViews = 8;
struct MultiView {
    const float *viewmatrix, *projmatrix, *campos;
    CamStrides cs;
    float tan_fovx, tan_fovy, focal_x, focal_y;
    const int *radii;
    const float4 *rec;      // the view's render records (GEOM): the activated opacity (sigmoid chain)
    const uint8_t *clampm;  // the view's SH clamp masks (GEOM)
    const float *sums;      // the view's per-Gaussian record sums, kPartial x P SoA (SUMS, gsr_backward_render)
    float *dL_dmeans2D;     // the view's screen-space gradient (P,3) or NULL
    int acc2;               // add into dL_dmeans2D instead of overwriting
};
struct MultiArgs {
    int P, D, M, nv, act, accm;
    float scale_modifier;
    const float *means3D, *scales, *rotations, *shs, *cov3D_precomp;
    float *dL_dcolors, *dL_dopacity, *dL_dmeans3D, *dL_dcov3D, *dL_dsh, *dL_dscales, *dL_drot;
    MultiView v[kMultiViews];
};
hipError_t launch_gauss_bwd_multi(const MultiArgs &a, hipStream_t s);

// fused L1 + SSIM (gsr_loss.hip): normalised 1-D window of calc_ssim (external.py:48-65)
struct SsimWindow { float w[11]; };
size_t ssim_partials(int planes, int H, int W);
hipError_t launch_ssim_fwd(int planes, int H, int W, const float *img1, const float *img2, const SsimWindow &w,
                           float *maps, float2 *partial, float *out_l1, float *out_ssim, hipStream_t s);
hipError_t launch_ssim_bwd(int planes, int H, int W, const float *img1, const float *img2, const SsimWindow &w,
                           const float *maps, const float *g_l1, const float *g_ssim, float *dimg1,
                           hipStream_t s);

// densification (gsr_densify.hip)
struct DensArgs {
    int P, prune_big;
    float grad_threshold, small_scale, big_scale, remove_opacity, inv_split_div;
    const float *grad_accum, *vis_count, *log_scales, *opacity_logits, *rotations;
};
struct DensColumn {
    int width, role;
    const float *src, *m_src, *v_src;
    float *dst, *m_dst, *v_dst;
};
constexpr int kDensMaxColumns = 8;
struct DensColumns { int n; DensColumn c[kDensMaxColumns]; };
struct DensWorkspace {
    int NB;
    size_t flags, bsum, boff, totals, total;
    explicit DensWorkspace(int P);
};
hipError_t launch_dens_radii(int P, const int *radii, float *max_radii, uint8_t *visible, hipStream_t s);
hipError_t launch_dens_grads(int P, const uint8_t *visible, const float *m2grad, float *grad_accum,
                             float *vis_count, hipStream_t s);
hipError_t launch_dens_plan(const DensArgs &a, char *ws, hipStream_t s);
hipError_t launch_dens_stds(const DensArgs &a, const char *ws, float *stds, hipStream_t s);
hipError_t launch_dens_apply(const DensArgs &a, const char *ws, const float *samples, const DensColumns &cols,
                             hipStream_t s);

// fused Adam (gsr_adam.hip)
struct AdamTensor {
    float *param; const float *grad; float *exp_avg; float *exp_avg_sq;
    long long n; float step_size, bc2_sqrt; int vec4;
};
constexpr int kAdamMaxTensors = 16;
struct AdamTable {
    int n; float w1, b2, omb2, eps;
    AdamTensor t[kAdamMaxTensors];
    int block_start[kAdamMaxTensors + 1];
};
int adam_blocks(long long n);
hipError_t launch_adam(const AdamTable &tab, hipStream_t s);

// camera frames -> view tensors (gsr_io.hip)
hipError_t launch_views_pack(int frames, int HW, const uint8_t *rgb, const uint8_t *seg, float *img, float *msk,
                             hipStream_t s);

}  // namespace gsr
