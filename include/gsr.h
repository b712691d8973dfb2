/*
 * gsr.h -- C ABI of the MI355X-native differentiable Gaussian-splat rasterizer (libgsr.so).
 *
 * This is the native boundary under the Python drop-in `diff_gaussian_rasterization`
 * (GaussianRasterizer / GaussianRasterizationSettings, imported by the reference at
 * train.py:16, densify.py:9, shared.py:9).  Each entry point replaces one function of the
 * reference's native extension `diff_gaussian_rasterization._C`, whose source is the (empty here)
 * submodule `diff-gaussian-rasterization-w-depth` (.gitmodules:1-3); see SURVEY.md section 2.1:
 *
 *   gsr_forward       <- _C.rasterize_gaussians           (rasterize_points.cu RasterizeGaussiansCUDA,
 *                                                          CudaRasterizer::Rasterizer::forward)
 *   gsr_backward      <- _C.rasterize_gaussians_backward  (RasterizeGaussiansBackwardCUDA,
 *                                                          CudaRasterizer::Rasterizer::backward)
 *   gsr_mark_visible  <- _C.mark_visible                  (markVisible)
 *
 * Plain pointers and sizes only; no torch types.  All tensor pointers are DEVICE pointers to
 * contiguous fp32 data in the reference's own layouts (means3D (P,3), shs (P,M,3), colors (P,3),
 * opacities (P,1), scales (P,3), rotations (P,4) = quaternion (w,x,y,z), cov3D (P,6) upper
 * triangle).  Matrices are the 16 floats of the `.contiguous()` (1,4,4) tensors built by
 * shared.py:80,110,120 (column-major: x' = m[0]x + m[4]y + m[8]z + m[12]).
 *
 * Every call is asynchronous on `stream` (a hipStream_t; NULL = legacy default stream) except for
 * the single device->host read of num_rendered inside gsr_forward, which the reference also does.
 * Functions return GSR_OK (0) or an error code; gsr_last_error() gives the thread-local message.
 */
#ifndef GSR_H
#define GSR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSR_ABI_VERSION 21

enum gsr_status {
    GSR_OK = 0,
    GSR_ERR_ARG = 1,         /* invalid argument (shape/combination); message in gsr_last_error() */
    GSR_ERR_HIP = 2,         /* HIP runtime / kernel launch error */
    GSR_ERR_ALLOC = 3,       /* the allocation callback returned NULL */
    GSR_ERR_UNSUPPORTED = 4  /* configuration outside the supported envelope */
};

/* Buffer kinds requested through the allocation callback.  They mirror the reference's
 * geometryBuffer / binningBuffer / imageBuffer resize functors (rasterize_points.cu), plus the
 * backward pass's transient scratch.  The caller owns every returned buffer; GEOM, BINNING and
 * IMAGE must be kept alive and handed back to gsr_backward. */
enum gsr_buffer { GSR_BUF_GEOM = 0, GSR_BUF_BINNING = 1, GSR_BUF_IMAGE = 2, GSR_BUF_SCRATCH = 3,
                  GSR_BUF_SUMS = 4 /* ABI >= 15: gsr_backward_render's per-Gaussian record sums */ };

/* Returns a device pointer of at least `bytes` bytes, 256-byte aligned, or NULL on failure. */
typedef void *(*gsr_alloc_fn)(void *ctx, int which, size_t bytes);

/* Camera / raster settings: the 11 fields of GaussianRasterizationSettings (shared.py:112-124). */
typedef struct gsr_camera {
    int image_width;
    int image_height;
    float tan_fovx;          /* = W / (2 fx)  (shared.py:115) */
    float tan_fovy;          /* = H / (2 fy)  (shared.py:116) */
    const float *viewmatrix; /* device, 16 floats */
    const float *projmatrix; /* device, 16 floats (= view * proj, shared.py:120) */
    const float *campos;     /* device, 3 floats */
    const float *bg;         /* device, 3 floats */
    int prefiltered;         /* accepted; the near-plane cull is applied either way */
    /* ABI >= 8: element strides of the matrices' (row, column) and of campos, so the reference's
     * views pass as they are -- its viewmatrix is the non-contiguous transpose w2c^T (shared.py:80)
     * and campos a column slice of inv(w2c) (shared.py:79).  Element k of the 16 read as m[k] (the
     * column-major convention above) is at (k / 4) * stride[0] + (k % 4) * stride[1].  Zeros mean
     * contiguous: {4, 1} and 1. */
    int viewmatrix_stride[2];
    int projmatrix_stride[2];
    int campos_stride;
} gsr_camera;

/* Fused parameter activations (bit mask, gsr_gaussians.activations).  The reference's caller
 * activates the raw parameters before every render (shared.py:33-41: rotations =
 * normalize(rotation_quaternions), opacities = sigmoid(opacity_logits), scales = exp(log_scales));
 * with a bit set the corresponding pointer holds the RAW parameter, the kernels apply the
 * activation on load, and gsr_backward returns the gradient with respect to the raw parameter
 * (the chain rule of torch's normalize(eps = 1e-12) / sigmoid / exp).  0 = inputs already activated,
 * exactly the reference's _C interface. */
enum gsr_activation {
    GSR_ACT_NONE = 0,
    GSR_ACT_SIGMOID_OPACITY = 1,
    GSR_ACT_EXP_SCALES = 2,
    GSR_ACT_NORMALIZE_ROTATIONS = 4
};

/* Per-Gaussian inputs: the render arguments of shared.py:29-42 (activated unless `activations`). */
typedef struct gsr_gaussians {
    int P;                       /* number of Gaussians (>= 0) */
    int sh_degree;               /* active SH degree D (0..3) */
    int sh_coeffs;               /* M = shs.size(1), 0 when shs is NULL */
    float scale_modifier;
    const float *means3D;        /* (P,3) required */
    const float *shs;            /* (P,M,3) or NULL -- exactly one of shs / colors_precomp */
    const float *colors_precomp; /* (P,3)   or NULL */
    const float *opacities;      /* (P,1) required */
    const float *scales;         /* (P,3)   or NULL -- scales+rotations, or cov3D_precomp */
    const float *rotations;      /* (P,4)   or NULL */
    const float *cov3D_precomp;  /* (P,6)   or NULL */
    int activations;             /* gsr_activation bit mask (ABI >= 2); 0 = activated inputs */
    /* ABI >= 12.  gsr_forward: nonzero = a backward will follow, so the forward also builds the
     * backward's work-item list (one small kernel after the blend, off the backward's critical path)
     * in gsr_backward_items_bytes() extra bytes at the end of the BINNING buffer.  gsr_backward /
     * gsr_backward_render: must equal the value the forward was called with. */
    int prepare_backward;
    /* ABI >= 14.  gsr_backward / gsr_backward_render: the BINNING layout the forward reported
     * (gsr_forward_info.binning_layout); 0 = num_rendered (gsr_forward, or a forward that did not
     * enqueue speculatively).  Ignored by the forward. */
    int binning_layout;
} gsr_gaussians;

/* Bits of gsr_grads.accumulate (ABI >= 6), one per output array. */
enum gsr_grad_bits {
    GSR_GRAD_MEANS2D = 1, GSR_GRAD_COLORS = 2, GSR_GRAD_OPACITY = 4, GSR_GRAD_MEANS3D = 8,
    GSR_GRAD_COV3D = 16, GSR_GRAD_SH = 32, GSR_GRAD_SCALES = 64, GSR_GRAD_ROTATIONS = 128
};

/* Gradient outputs of gsr_backward, in the order _C.rasterize_gaussians_backward returns them.
 * Every element of every non-NULL array is written (no pre-zeroing needed).  Any of them may be
 * NULL when the caller does not need it (ABI >= 13; before, dL_dmeans2D, dL_dopacity, dL_dmeans3D
 * and dL_dsh were required): dL_dcolors under SH colour, dL_dcov3D when scales/rotations are given,
 * and every input that does not require grad -- train.py renders frozen Gaussians
 * (train.py:155-163 sets requires_grad = False) whose only live gradients are means3D, rotations
 * and means2D.  The skipped arrays' HBM writes (and the SH coefficient rows) are not issued.
 * `accumulate` (gsr_grad_bits): the marked arrays already hold a gradient and receive
 * old + new (one fp32 add, what torch's AccumulateGrad computes) instead of new -- gradient
 * accumulation over the views of a step without a separate add pass. */
typedef struct gsr_grads {
    float *dL_dmeans2D;   /* (P,3)  NDC units, z = 0 */
    float *dL_dcolors;    /* (P,3) */
    float *dL_dopacity;   /* (P,1) */
    float *dL_dmeans3D;   /* (P,3) */
    float *dL_dcov3D;     /* (P,6) */
    float *dL_dsh;        /* (P,M,3) or NULL when M == 0 */
    float *dL_dscales;    /* (P,3) */
    float *dL_drotations; /* (P,4) */
    int accumulate;       /* gsr_grad_bits (ABI >= 6); 0 = overwrite every output */
} gsr_grads;

/* Forward: preprocess -> tile binning -> per-tile depth sort -> alpha blend (colour + depth).
 * Writes out_color (3,H,W), out_depth (1,H,W), out_radii (P) and *out_num_rendered.  The three
 * persistent buffers are requested through `alloc` (GEOM, IMAGE, then BINNING once the
 * Gaussian/tile pair count is known).  P == 0 writes zeros (no background), like the reference. */
int gsr_forward(const gsr_camera *cam, const gsr_gaussians *g, gsr_alloc_fn alloc, void *alloc_ctx,
                float *out_color, float *out_depth, int *out_radii, int *out_num_rendered,
                void *stream);

/* Speculative enqueue (ABI >= 14).  gsr_forward waits on the host for num_rendered between the
 * tile-count scan and the pair emission (the BINNING buffer is sized by it), so the stream idles while
 * the host reads K back, calls the allocator and launches the rest.  gsr_forward_info_call with
 * `speculate` set queues the post-scan kernels BEFORE that read-back, against a BINNING capacity of
 * 1.25 x the largest pair count seen for this (device, P, W, H) + 65536 (no speculation on a first
 * call, or when the last one needed the long-list merge sort); k_bin_scan checks the capacity on the
 * device and those kernels return at once when it fails, in which case the host redoes them with the
 * exact count before returning -- the outputs are the same either way (bitwise).  The call still
 * returns after num_rendered is known.  `info->binning_layout` is the pair count the BINNING buffer
 * is laid out for (the capacity, or num_rendered); pass it to the backward calls in
 * gsr_gaussians.binning_layout and to gsr_buffer_offsets. */
typedef struct gsr_forward_info {
    int num_rendered;    /* K, the reference's num_rendered (-1: pending, see gsr_forward_async) */
    int binning_layout;  /* the pair count BINNING is laid out for (>= num_rendered) */
    int speculated;      /* 1: the speculatively queued kernels stood; 0: exact path */
    unsigned long long pending;  /* ABI >= 17: nonzero = an asynchronous forward's handle */
    /* reserved (ABI 17-19: the item list's auxiliary stream, removed in round 5); always NULL */
    void *aux_stream;
} gsr_forward_info;
int gsr_forward_info_call(const gsr_camera *cam, const gsr_gaussians *g, gsr_alloc_fn alloc, void *alloc_ctx,
                          float *out_color, float *out_depth, int *out_radii, int speculate, gsr_forward_info *info,
                          void *stream);
/* Speculation counters since the last reset (stood / redone); reset != 0 also clears the history. */
int gsr_spec_stats(int *hits, int *misses, int reset);
/* Pair-count history keys held (at most 64; the least recently used key is evicted). */
int gsr_spec_keys(void);

/* Asynchronous forward (ABI >= 17).  Like gsr_forward_info_call with speculation, but when the
 * speculation has a capacity (a key with history, no long-list merge sort) the call returns as soon
 * as every kernel is queued -- the host never waits for num_rendered, so a caller that renders
 * several views from one thread (train.py:402-412) keeps queueing while the GPU works.  It then sets
 * info->num_rendered = -1 and info->pending to a handle.  The device checks the capacity after the
 * tile scan; when it did not hold, the library's resolver thread redoes the post-scan kernels with
 * the exact pair count on a stream of its own and the forward's last kernel holds `stream` until
 * that is done, so everything queued after the call sees the exact outputs (bitwise those of
 * gsr_forward).  Without a capacity it behaves as gsr_forward_info_call (pending = 0).
 *   gsr_forward_resolve  waits until the forward's pair count is known (and a redo is done) and gives
 *                        the pair count, the BINNING layout and the BINNING buffer to hand to the
 *                        backward calls (the caller's buffer, or the resolver's for a redone forward)
 *   gsr_forward_release  the caller is done with the handle (after its backward, or at once for a
 *                        forward without one); the resolver's buffer is freed stream-ordered on the
 *                        forward's stream.  Every handle must be released exactly once. */
typedef struct gsr_forward_resolution {
    int num_rendered;
    int binning_layout;
    void *binning;
    int redone;          /* 1: the speculation failed and the resolver redid the post-scan kernels */
} gsr_forward_resolution;
int gsr_forward_async(const gsr_camera *cam, const gsr_gaussians *g, gsr_alloc_fn alloc, void *alloc_ctx,
                      float *out_color, float *out_depth, int *out_radii, gsr_forward_info *info, void *stream);
/* Waits until the forward's pair count is known (and a failed speculation redone).  Fails (GSR_ERR_HIP)
 * when the forward failed, or when its render abandoned the gate (a 5 s timeout) before the redo opened
 * it -- the caller's work queued after the forward then ran on outputs that were not final, so the step
 * must not go on (the binding raises in that step's backward).  A timed-out forward released without a
 * resolution makes the next forward fail instead. */
int gsr_forward_resolve(unsigned long long handle, gsr_forward_resolution *out);
int gsr_forward_release(unsigned long long handle);
/* 1: gsr_forward_resolve would return without waiting; 0: not yet; -1: unknown handle. */
int gsr_forward_query(unsigned long long handle);
/* Asynchronous forwards since the last gsr_spec_stats reset, and handles not yet released+resolved. */
int gsr_async_stats(int *calls, int *pending);
/* Stops the resolver thread once it has no redo in flight (call at process exit, before the HIP
 * runtime is torn down; a later asynchronous forward starts it again). */
int gsr_async_shutdown(void);
/* Test hook for the asynchronous forward's failure path: the resolver keeps the NEXT redone forward's
 * gate closed for hold_next_redo_ms (0: no delay), later forwards' gates time out after gate_timeout_ms
 * (<= 0: the default 5 s); clear != 0 also drops a pending sticky error (see gsr_forward_resolve). */
int gsr_debug_async_fault(int hold_next_redo_ms, int gate_timeout_ms, int clear);

/* Backward of gsr_forward given dL/d(color) (3,H,W).  dL_ddepth is accepted and ignored: the
 * reference discards the depth output (train.py:355-361, densify.py:120-126) and its -w-depth
 * backward does not propagate it.  Requests one SCRATCH buffer through `alloc`. */
int gsr_backward(const gsr_camera *cam, const gsr_gaussians *g, const int *radii, int num_rendered,
                 const void *geom, const void *binning, const void *image, const float *dL_dcolor,
                 const float *dL_ddepth, gsr_alloc_fn alloc, void *alloc_ctx, gsr_grads *out,
                 void *stream);

/* ---- Multi-view backward (ABI >= 12) ------------------------------------------------------------
 * gsr_backward split in two so that the per-Gaussian half runs ONCE for all the views of a step
 * (train.py:753-767 sums the losses of 5 views before one backward):
 *
 *   gsr_backward_render     the per-pixel half of gsr_backward for one view: requests a SCRATCH
 *                           buffer through `alloc` for the view's per-(tile, Gaussian) gradient
 *                           records, then a SUMS buffer (gsr_sums_bytes(P), ABI >= 15) into which it
 *                           sums each Gaussian's records in emission order (9 x P floats, SoA, then
 *                           the view's camera key, one word -- a hash of its view and projection
 *                           matrices, camera position and image size: gsr_backward_gaussians sums the
 *                           views in the order of their keys, not the order they were passed in;
 *                           views with equal keys, i.e. the same camera passed twice in one launch,
 *                           keep the order they were passed in, so their sum depends on it).  Only
 *                           SUMS (and the view's GEOM, radii) must stay alive until
 *                           gsr_backward_gaussians has been queued; SCRATCH may be released once the
 *                           call returns (its last reader is queued on `stream`).
 *   gsr_backward_gaussians  the per-Gaussian half over `nviews` such views of the SAME Gaussians `g`:
 *                           every per-Gaussian gradient of `out` receives the SUM over the views
 *                           (added into the arrays marked in out->accumulate, as gsr_backward does);
 *                           each view's dL/dmeans2D goes to that view's own array.  out->dL_dmeans2D
 *                           is ignored.  All views' gsr_backward_render work must be complete on
 *                           `stream` or ordered before it by the caller (same stream or events).
 *
 * The result equals gsr_backward per view with the gradients summed, up to the order of the fp32
 * additions (views are summed in registers, then added to the arrays once).  SH needs M in
 * {1, 4, 9, 16} (GSR_ERR_UNSUPPORTED otherwise).
 *
 * ABI >= 19, speculative render half: gsr_backward_render with num_rendered < 0 and g->binning_layout =
 * the capacity an asynchronous forward reported (gsr_forward_info.binning_layout) queues the half
 * before that forward's pair count is known, against its own BINNING buffer, with SCRATCH sized for the
 * capacity (gsr_scratch_bytes(binning_layout, W, H)).  Its kernels read the device's speculation verdict
 * and return at once when it failed; the caller then learns `redone` from gsr_forward_resolve and must
 * call gsr_backward_render again with the resolved num_rendered / binning_layout / BINNING (a fresh
 * SUMS buffer) before gsr_backward_gaussians.  When the speculation stood the SUMS are final and equal
 * to those of the resolved call.  gsr_backward rejects num_rendered < 0. */
typedef struct gsr_view_grad {
    const gsr_camera *cam;   /* the view's camera (as given to its gsr_forward) */
    const int *radii;        /* the view's radii (P) */
    const void *geom;        /* the view's GEOM buffer */
    const void *scratch;     /* the view's SUMS buffer, filled by gsr_backward_render (ABI >= 15;
                                the SCRATCH buffer before) */
    int num_rendered;        /* the view's num_rendered */
    float *dL_dmeans2D;      /* (P,3) the view's screen-space gradient, or NULL */
    int accumulate_means2D;  /* nonzero: add into dL_dmeans2D instead of overwriting it */
} gsr_view_grad;

int gsr_backward_render(const gsr_camera *cam, const gsr_gaussians *g, const int *radii, int num_rendered,
                        const void *geom, const void *binning, const void *image, const float *dL_dcolor,
                        gsr_alloc_fn alloc, void *alloc_ctx, void *stream);
int gsr_backward_gaussians(int nviews, const gsr_view_grad *views, const gsr_gaussians *g, gsr_grads *out,
                           void *stream);

/* Cross-stream order of gradient writes (ABI >= 10).  gsr_backward calls that write the same
 * gradient array (any of the gsr_grads pointers, accumulated or not) from different streams are
 * ordered behind each other by the library: each write waits for the previous writer of every
 * array it touches when that writer ran on another stream.  gsr_grad_fence declares that the work
 * queued so far on `stream` also writes the `n` arrays `grads` (e.g. an all-reduce or a reset of the
 * gradient bucket they live in), so the next gsr_backward into any of them, on any stream, waits
 * for it -- and the streams themselves need not. */
int gsr_grad_fence(const void *const *grads, int n, void *stream);

/* present[i] = Gaussian i passes the near-plane frustum test (view-space z > 0.2). */
int gsr_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                     uint8_t *present, void *stream);

/* Byte sizes of the buffers gsr_forward requests (for callers that pre-allocate pools). */
size_t gsr_geom_bytes(int P);
size_t gsr_image_bytes(int width, int height, int P);
size_t gsr_binning_bytes(int num_rendered, int P);  /* ABI >= 16: the boundary states depend on P */
size_t gsr_scratch_bytes(int num_rendered, int width, int height);
size_t gsr_sums_bytes(int P);  /* ABI >= 15: the SUMS buffer of gsr_backward_render */
/* Extra BINNING bytes gsr_forward requests when gsr_gaussians.prepare_backward is set (ABI 12). */
size_t gsr_backward_items_bytes(int num_rendered, int width, int height);

/* Pre-allocated buffers (ABI >= 16).  gsr_prealloc_alloc is a gsr_alloc_fn (ctx = a gsr_prealloc)
 * that hands out ptr[which] when bytes[which] covers the request and passes every other request to
 * `fallback` (NULL: the request fails).  A caller that sizes the buffers beforehand (the functions
 * above and gsr_spec_binning_bytes) gets no call back into its own allocator on the usual path --
 * a Python caller's allocator needs the interpreter lock, which a forward otherwise re-acquires three
 * times while other threads submit their views.  `used` (output): bit k set when ptr[k] was handed
 * out. */
typedef struct gsr_prealloc {
    void *ptr[5];          /* indexed by gsr_buffer */
    size_t bytes[5];
    gsr_alloc_fn fallback;
    void *fallback_ctx;
    int used;
} gsr_prealloc;
void *gsr_prealloc_alloc(void *ctx, int which, size_t bytes);
/* The BINNING bytes a speculative gsr_forward_info_call with these sizes on the current device will
 * request (the capacity from its pair-count history, plus the backward's item list when
 * prepare_backward is set), or 0 when it will not speculate (no history, or the last forward of
 * these sizes needed the long-list merge sort).  Another thread's forward may raise the capacity
 * meanwhile: a larger request then goes to the fallback. */
size_t gsr_spec_binning_bytes(int P, int width, int height, int prepare_backward);

/* Introspection for parity tests: byte offsets of the arrays inside the three forward buffers, in
 * this order: geom {depth, rec (64-byte render records), rect, tiles, goff}, image {ranges,
 * pix_end (per pixel float4: accumulated colour without background, final transmittance),
 * n_contrib, tile_maxc}, binning {pairs (16-byte records: index, depth bits, emission, 0),
 * point_list, slot_emit}, image {seg_off}, binning {seg_state (the blend state at every interior
 * 128-entry boundary of every tile list: 256 float4 (C0, C1, C2, T) per boundary)}, image
 * {tile_flag (ABI 21: per tile, the count of near-threshold weights the forward re-evaluated inline in
 * the exact-threshold form; their records follow in IMAGE near_rec, at most 16 per tile, and a count
 * above 16 sends the tile's backward items to the re-evaluating k_render_bwd<true>)}, image {tsat_count
 * (one word: the pixels the exact saturation re-walk redid, round 6)}.  Returns the count written (16, or
 * max_out if smaller). */
int gsr_buffer_offsets(int P, int width, int height, int num_rendered, size_t *out, int max_out);

const char *gsr_last_error(void);
int gsr_abi_version(void);

/* Exact-threshold mode (ABI >= 18; process-wide; ON by default since ABI 21, GSR_EXACT_THRESHOLDS=0 at
 * load turns it off).  The render kernels evaluate the blend weight as 2^(power log2 e) with FMAs and
 * the hardware exp, which differs from the reference's expf(power) (renderCUDA, forward.cu /
 * backward.cu) by a few ulp; a (pixel, Gaussian) weight that close to 1/255 can take the other side of
 * the threshold.  With the mode on, k_render_fwd re-evaluates every weight it would take that lies
 * within 1e-5 (relative) of 1/255 inline, in the reference's expression order with a double-precision
 * exp, and appends (list position, pixel, power, G, alpha) to the tile's near records (IMAGE near_rec,
 * 16 per tile; IMAGE tile_flag = the tile's count).  The backward's walk looks those weights up in the
 * records; a tile with more than 16 re-evaluates them itself (k_render_bwd<true>).  So decisions match
 * the reference's.
 * The backward follows the flags its forward wrote, so the setting may change at any time; it applies
 * to forwards queued after the call.  Returns the previous setting. */
int gsr_set_exact_thresholds(int on);

/* ---- Fused L1 + SSIM image loss (ABI >= 3) ------------------------------
 * Replaces the loss of every render call site, train.py:362-363 / densify.py:127-129,149-151:
 *     torch.nn.functional.l1_loss(img1, img2)  and  calc_ssim(img1, img2)   (external.py:68-110:
 *     window_size 11, Gaussian sigma 1.5, zero padding 5, size_average=True)
 * with one forward and one backward kernel pair.  img1/img2/dL_dimg1: `planes` contiguous fp32
 * planes of height x width (a (3,H,W) image is 3 planes, a (B,C,H,W) batch B*C planes).  The
 * scratch buffer (gsr_ssim_scratch_bytes) carries the per-pixel SSIM derivatives from the forward to
 * the backward and must be kept alive between them. */
size_t gsr_ssim_scratch_bytes(int planes, int height, int width);
/* out_l1 = mean |img1 - img2|, out_ssim = mean SSIM: device float scalars (the values l1_loss and
 * calc_ssim return). */
int gsr_l1_ssim_forward(int planes, int height, int width, const float *img1, const float *img2,
                        void *scratch, float *out_l1, float *out_ssim, void *stream);
/* dL_dimg1 = dL_dl1 * d(l1)/d(img1) + dL_dssim * d(ssim)/d(img1); dL_dl1 / dL_dssim are DEVICE
 * scalars (either may be NULL = 0), so no host synchronisation is needed.  img2 gets no gradient. */
int gsr_l1_ssim_backward(int planes, int height, int width, const float *img1, const float *img2,
                         const void *scratch, const float *dL_dl1, const float *dL_dssim,
                         float *dL_dimg1, void *stream);

/* ---- Densification: statistics, clone / split / prune with Adam state surgery (ABI >= 4) ------
 * SURVEY.md 8(f) row 2.  Replaces update_max_2d_radii_and_visibility_mask (densify.py:154-162),
 * accumulate_mean_2d_gradients (external.py:113-124) and the body of densify_gaussians
 * (external.py:211-304 with cat_params_to_optimizer / remove_points, :144-204).  All pointers are
 * device pointers to contiguous fp32 (P, width) rows unless stated. */
enum gsr_densify_role {
    GSR_DENS_OTHER = 0,      /* copied to every output row of its Gaussian */
    GSR_DENS_MEANS = 1,      /* split copies get + build_rotation(q) * sample (external.py:262-265) */
    GSR_DENS_LOG_SCALES = 2  /* split copies get log(exp(s) / split_divisor) (external.py:266-268) */
};

typedef struct gsr_densify_settings {
    int P;
    float grad_threshold;          /* 0.0002 (external.py:224) */
    float small_scale;             /* 0.01 * scene_radius: clone if max scale <= it, split if > it */
    float big_scale;               /* 0.1 * scene_radius: pruned when prune_big (external.py:294-299) */
    float remove_opacity;          /* sigmoid(logit) below it is pruned: 0.005, or 0.25 at i == 5000 */
    int prune_big;                 /* i >= 3000 */
    float split_divisor;           /* 0.8 * n = 1.6 */
    const float *grad_accum;       /* (P) mean_2d_gradients_accumulated */
    const float *vis_count;        /* (P) visibility_count */
    const float *log_scales;       /* (P,3) */
    const float *opacity_logits;   /* (P,1) */
    const float *rotation_quaternions; /* (P,4) */
} gsr_densify_settings;

typedef struct gsr_densify_counts {
    int n_keep_orig;   /* originals surviving (not split, not pruned) */
    int n_keep_clone;  /* clones surviving */
    int n_split;       /* Gaussians split: the reference draws 2 * n_split samples */
    int n_keep_split;  /* split copies surviving, per copy */
    int P_out;         /* n_keep_orig + n_keep_clone + 2 * n_keep_split */
} gsr_densify_counts;

/* One per-Gaussian parameter and its Adam moments (exp_avg / exp_avg_sq may be NULL together when
 * the optimizer holds no state for it; dst_* likewise).  dst arrays hold P_out rows. */
typedef struct gsr_densify_column {
    int width;
    int role;                      /* gsr_densify_role */
    const float *src, *exp_avg, *exp_avg_sq;
    float *dst, *dst_exp_avg, *dst_exp_avg_sq;
} gsr_densify_column;

/* max_radii[vis] = max(radii, max_radii); visible[i] = radii[i] > 0 (u8). */
int gsr_densify_update_radii(int P, const int *radii, float *max_radii, uint8_t *visible, void *stream);
/* grad_accum[vis] += |means2D_grad[vis, :2]|; vis_count[vis] += 1.  means2D_grad is (P,3). */
int gsr_densify_accumulate_grads(int P, const uint8_t *visible, const float *means2D_grad,
                                 float *grad_accum, float *vis_count, void *stream);
size_t gsr_densify_workspace_bytes(int P);
/* Decides every row's fate and fills *counts (host struct; this call synchronises `stream`, as the
 * reference's boolean-mask indexing does). */
int gsr_densify_plan(const gsr_densify_settings *s, void *workspace, gsr_densify_counts *counts,
                     void *stream);
/* stds (2 * n_split, 3): exp(log_scales) of the split rows, twice (external.py:257-259) -- the std of
 * the caller's torch.normal draw. */
int gsr_densify_split_stds(const gsr_densify_settings *s, const void *workspace, float *stds, void *stream);
/* Writes every column's P_out output rows (and moments) in the reference's order; `counts` is what
 * gsr_densify_plan returned, `samples` the (2 * n_split, 3) normal draw (may be NULL when n_split is
 * 0).  At most 8 columns. */
int gsr_densify_apply(const gsr_densify_settings *s, const void *workspace, const gsr_densify_counts *counts,
                      const float *samples, int ncols, const gsr_densify_column *cols, void *stream);

/* ---- Fused Adam step over the per-Gaussian parameters (ABI >= 5) ---------
 * Replaces optimizer.step() of torch.optim.Adam(..., eps=1e-15) (densify.py:68-86, :247) for every
 * tensor in one launch, with torch's _multi_tensor_adam operation order.  `step` is the tensor's
 * step count after this update (torch increments it first); lr / step / betas / eps are the group's
 * Python values (bias corrections are formed in double, as torch does). */
typedef struct gsr_adam_tensor {
    float *param;
    const float *grad;
    float *exp_avg;
    float *exp_avg_sq;
    long long numel;
    double lr;
    double step;
} gsr_adam_tensor;

int gsr_adam_step(int ntensors, const gsr_adam_tensor *tensors, double beta1, double beta2, double eps,
                  void *stream);

/* ---- Camera frames of one timestep -> the reference's view tensors (ABI >= 7) ----
 * Replaces the per-view tensor formatting of load_timestep_views (shared.py:127-171) for `frames`
 * frames of H x W pixels at once.  Inputs are device pointers to the decoded 8-bit data: `rgb`
 * (frames, H, W, 3) interleaved, `seg` (frames, H, W) or NULL.  Outputs (contiguous fp32):
 * `images` (frames, 3, H, W) = rgb / 255 (as torch computes it on the GPU: x * (1.0f / 255.0f)),
 * `seg_masks` (frames, 3, H, W) = (m, 0, 1 - m) with m = float(seg), or NULL when seg is NULL. */
int gsr_views_pack(int frames, int H, int W, const uint8_t *rgb, const uint8_t *seg, float *images,
                   float *seg_masks, void *stream);

/* Per-phase device timing with HIP events recorded on the call's stream (off by default).
 * Phases: "preprocess", "bin_count", "bin_scan", "bin_emit", "tile_sort", "render_fwd",
 * "bwd_items", "render_bwd", "sum_records", "gauss_bwd", "ssim_fwd", "ssim_bwd", "densify_plan", "densify_apply", "adam", "views_pack".  gsr_profile_read synchronises on the recorded events. */
int gsr_profile_enable(int on);
/* Restrict event recording to a comma-separated list of phases (NULL or "" = every phase), so a
 * timed region can carry the events of one kernel only.  Host-side timers are unaffected. */
int gsr_profile_select(const char *phases);
int gsr_profile_reset(void);
int gsr_profile_read(const char *phase, double *total_ms, int *count);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H */
