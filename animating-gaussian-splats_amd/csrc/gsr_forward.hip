// gsr_forward.hip -- forward pass of the MI355X-native Gaussian-splat rasterizer.
//
// Pipeline (one HIP stream, one host sync for the pair count K, as the reference does):
//   k_preprocess   1 thread / Gaussian: cull, Sigma3D, EWA Sigma2D, conic, radius, tile rect, SH->RGB
//   k_bin_count    chunked over Gaussians: LDS tile histogram -> the chunk's row of a (chunk, tile)
//                  count matrix
//   k_bin_colscan  column scan of that matrix: each chunk's slab offset inside every tile, tile totals
//   k_bin_scan     1 block: exclusive scan of tile counts -> tile ranges; scan of chunk sums; K
//   k_bin_emit     chunked: slab starts into LDS (range start + column offset), scatter one 16-byte
//                  record per pair (64-bit key depth_bits << 32 | gaussian + emission index) into
//                  its tile's range; exclusive emission offsets
//   k_tile_sort    1 block / tile: sort the tile's keys by (depth bits, index) in LDS (bitonic),
//                  write the Gaussian list + the emission->slot map used by the backward reduction
//   k_render_fwd   1 block (4 wave64) / 16x16 tile: front-to-back blend of colour and depth
//
// The reference instead emits (tile<<32 | depth) keys and radix-sorts all K pairs globally
// (SURVEY.md 2.1 rows duplicateWithKeys / SortPairs / identifyTileRanges).  Bucketing by tile first
// and sorting (depth, index) inside each tile yields the identical order: a stable LSD sort on
// (tile, depth) breaks ties by emission order, and within one tile the emission order is the
// Gaussian index.  Tile ranges fall out of the bucket scan.
#include "gsr_common.h"
#include "gsr_internal.h"

#include <algorithm>
#include <type_traits>

namespace gsr {

#ifdef GSR_TRACE
__device__ uint64_t *g_trace_fwd;
#ifdef GSR_TRACE
// the forward waves' work counter: batches << 40 | ticks in the walk << 20 | evaluations
__device__ inline uint64_t trace_fwd_work(uint64_t batches, uint64_t walk, uint64_t evals) {
    return (batches << 40) | ((walk < 0xFFFFFull ? walk : 0xFFFFFull) << 20) | (evals < 0xFFFFFull ? evals : 0xFFFFFull);
}
#endif
__device__ uint64_t *g_trace_emit;  // per k_bin_emit block: start, counted, reserved, end
#define GSR_EMIT_STAMP(k)                                                                        \
    do {                                                                                         \
        if (g_trace_emit && threadIdx.x == 0)                                                    \
            g_trace_emit[4 * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime();               \
    } while (0)
#else
#define GSR_EMIT_STAMP(k) do {} while (0)
#endif

// ------------------------------------------------------------------------------------------
template <int MC>  // SH coefficient count staged through LDS (0: direct loads / no SH)
__global__ __launch_bounds__(256) void k_preprocess(
    int P, int D, int M, const float *__restrict__ means3D, const float *__restrict__ scales,
    float scale_modifier, const float *__restrict__ rotations, const float *__restrict__ opacities,
    const float *__restrict__ shs, const float *__restrict__ colors_precomp,
    const float *__restrict__ cov3D_precomp, const float *__restrict__ viewmatrix,
    const float *__restrict__ projmatrix, const float *__restrict__ campos, int W, int H,
    float tan_fovx, float tan_fovy, float focal_x, float focal_y, int gx, int gy,
    int *__restrict__ radii, float *__restrict__ depth_out, float4 *__restrict__ rec_out,
    uint2 *__restrict__ rect_out, uint32_t *__restrict__ tiles_out, int act, CamStrides cs,
    uint32_t *__restrict__ tile_count, int T, uint8_t *__restrict__ clamp_out) {
    extern __shared__ __attribute__((aligned(16))) float s_sh[];
    constexpr int RL = 3 * MC, RS = sh_row_stride(MC);
    const int i0 = blockIdx.x * kShBlock;
    const int i = i0 + threadIdx.x;
    // k_bin_count's tile histogram starts from zero: cleared here instead of by a memset launch
    for (int t = i; t < T; t += (int)gridDim.x * kShBlock) tile_count[t] = 0;
    // this Gaussian's own inputs are loaded first (clamped index for the tail lanes), so their
    // latency overlaps the SH row copy instead of following its barrier
    const int ic = min(i, P - 1);
    const float3 p = make_float3(means3D[3 * ic], means3D[3 * ic + 1], means3D[3 * ic + 2]);
    float3 s_in = make_float3(0.f, 0.f, 0.f);
    float4 q_in = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!cov3D_precomp) {
        s_in = make_float3(scales[3 * ic], scales[3 * ic + 1], scales[3 * ic + 2]);
        q_in = make_float4(rotations[4 * ic], rotations[4 * ic + 1], rotations[4 * ic + 2], rotations[4 * ic + 3]);
    }
    const float o_in = opacities[ic];
    if constexpr (MC > 0) {  // coalesced copy of this block's SH rows into LDS
        sh_rows_to_lds<MC>(shs + (size_t)i0 * RL, min(kShBlock, P - i0), s_sh);
        __syncthreads();
    }
    if (i >= P) return;
    // matrices are tiny and uniform: every lane reads the same words (scalar loads)
    float vm[16], pm[16];
    load_mat16(viewmatrix, cs.v0, cs.v1, vm);
    load_mat16(projmatrix, cs.p0, cs.p1, pm);
    radii[i] = 0;
    tiles_out[i] = 0;
    rect_out[i] = make_uint2(0, 0);
    const float4 ph = xform4x4(p, pm);
    const float3 pv = xform4x3(p, vm);
    if (pv.z <= 0.2f) return;  // near-plane cull (in_frustum)
    const float pw = 1.0f / (ph.w + 0.0000001f);
    const float ppx = ph.x * pw, ppy = ph.y * pw;
    float c3[6];
    if (cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; ++k) c3[k] = cov3D_precomp[6 * i + k];
    } else {
        float3 s = s_in;
        float4 q = q_in;
        if (act & GSR_ACT_EXP_SCALES) s = act_exp3(s);
        if (act & GSR_ACT_NORMALIZE_ROTATIONS) q = act_normalize(q, quat_norm(q));
        cov3d_from_scale_rot(s, scale_modifier, q, c3);
    }
    const float3 cv = cov2d(p, focal_x, focal_y, tan_fovx, tan_fovy, c3, vm);
    const float det = cv.x * cv.z - cv.y * cv.y;
    if (det == 0.0f) return;
    const float det_inv = 1.f / det;
    const float mid = 0.5f * (cv.x + cv.z);
    const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float my_radius = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    const float pix_x = ndc2pix(ppx, W), pix_y = ndc2pix(ppy, H);
    int x0, y0, x1, y1;
    get_rect(pix_x, pix_y, (int)my_radius, gx, gy, x0, y0, x1, y1);
    if ((x1 - x0) * (y1 - y0) == 0) return;
    float3 rgb;
    if (colors_precomp) {
        rgb = make_float3(colors_precomp[3 * i], colors_precomp[3 * i + 1], colors_precomp[3 * i + 2]);
    } else {
        bool cl[3];
        const float3 cp = load_campos(campos, cs.c0);
        if (MC > 0) rgb = sh_to_rgb(D, p, cp, s_sh + threadIdx.x * RS, cl);
        else rgb = sh_to_rgb(D, p, cp, shs + (size_t)i * M * 3, cl);
        clamp_out[i] = clamp_bits(cl);  // for the backward's SH chain
    }
    radii[i] = (int)my_radius;
    depth_out[i] = pv.z;
    const float o = (act & GSR_ACT_SIGMOID_OPACITY) ? act_sigmoid(o_in) : o_in;
    const float ca = cv.z * det_inv, cb = -cv.y * det_inv, cc = cv.x * det_inv;
    const float tau2 = o >= 1.0f / 255.0f ? 2.f * log2f(255.f * o) : -1.f;
    float4 *r = rec_out + (size_t)kRecF4 * i;
    r[0] = make_float4(pix_x, pix_y, -0.5f * GSR_LOG2E * ca, -GSR_LOG2E * cb);
    r[1] = make_float4(-0.5f * GSR_LOG2E * cc, o, pv.z, tau2);
    r[2] = make_float4(rgb.x, rgb.y, rgb.z, pv.z);  // (.w: the depth again, beside the colour for the blend)
    r[3] = make_float4(ca, cb, cc, 0.f);
    rect_out[i] = pack_rect(x0, y0, x1, y1);
    tiles_out[i] = (uint32_t)((y1 - y0) * (x1 - x0));
}

// ------------------------------------------------------------------------------------------
// Tile histogram per chunk of Gaussians.  USE_LDS (T <= kMaxLdsTiles): histogram in LDS, stored as
// the chunk's row of the (chunk, tile) count matrix (coalesced, no global atomics; k_bin_colscan
// turns the columns into slab offsets and tile totals).  Otherwise global atomics into tile_count.
template <bool USE_LDS>
__global__ __launch_bounds__(kBinThreads) void k_bin_count(int P, int CH, int T, int gx,
                                                   const uint2 *__restrict__ rects,
                                                   const uint32_t *__restrict__ tiles,
                                                   uint32_t *__restrict__ tile_count,
                                                   uint32_t *__restrict__ block_sums,
                                                   uint32_t *__restrict__ chunk_off,
                                                   uint32_t *__restrict__ items_ws,
                                                   uint32_t *__restrict__ scan_ws) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];
    __shared__ uint32_t s_red[16];
    const int b = blockIdx.x;
    if (b == 0) {  // the tile scan's and the backward item builder's workspaces start zeroed
        for (int i = threadIdx.x; i < kItemsWsWords; i += blockDim.x) items_ws[i] = 0;
        if (scan_ws)
            for (int i = threadIdx.x; i < kScanWsWords; i += blockDim.x) scan_ws[i] = 0;
    }
    const int g0 = b * CH, g1 = min(P, g0 + CH);
    if (USE_LDS) {
        for (int t = threadIdx.x; t < T; t += blockDim.x) s_hist[t] = 0;
        __syncthreads();
    }
    uint32_t my_sum = 0;
    for (int g = g0 + threadIdx.x; g < g1; g += blockDim.x) {
        const uint32_t n = tiles[g];
        if (n == 0) continue;
        my_sum += n;
        const uint2 r = rects[g];
        const int x0 = r.x & 0xFFFF, y0 = r.x >> 16, x1 = r.y & 0xFFFF, y1 = r.y >> 16;
        for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x) {
                if (USE_LDS) atomicAdd(&s_hist[y * gx + x], 1u);
                else atomicAdd(&tile_count[y * gx + x], 1u);
            }
    }
    uint32_t tot;
    block_excl_scan_u32(my_sum, s_red, &tot);
    if (threadIdx.x == 0) block_sums[b] = tot;
    if (USE_LDS) {
        __syncthreads();
        uint32_t *row = chunk_off + (size_t)b * T;
        for (int t = threadIdx.x; t < T; t += blockDim.x) row[t] = s_hist[t];
    }
}

// Column scan of the (chunk, tile) count matrix: chunk_off[b][t] <- the counts of tile t over the
// chunks before b (chunk b's slab start inside the tile's range), tile_count[t] <- the tile's total.
// kColW tile columns x kColG groups of consecutive chunks per block; a thread holds its group's
// (at most kColR) counts in registers between the two passes, so the matrix is read once.  Replaces
// one device-scope atomic per non-empty (chunk, tile) bin in k_bin_count and a returning one in
// k_bin_emit (~2 M each at C3) with 2 x NB x T x 4 bytes of coalesced traffic.
//
// The same kernel then finishes the tile scan in a single pass (what a separate one-block scan kernel
// did, ~25 us at C3 on ONE CU): blocks take their tile columns by ticket (dispatch order), publish their
// columns' pair and segment-boundary sums and look back over the earlier blocks' words (decoupled
// look-back: one wave reads 64 predecessors at a time) for their exclusive prefix, then write their
// tiles' ranges, cursors, segment offsets, list classes and LPT bucket ranks.  The last block to finish
// (done counter) turns the LPT bucket counts into offsets (k_bin_emit scatters the dispatch order),
// scans the chunk sums into chunk emission offsets and publishes K and the list classes to meta and
// the host words -- as k_bin_scan does.
constexpr int kColW = 32, kColG = 32, kColR = 16;  // tile columns x chunk groups per k_bin_colscan block
static_assert(kColG * kColR >= 512, "BinGrid makes at most 512 chunks");
static_assert(kColW <= 64 && kMaxLdsTiles <= kColW * kScanBlocksMax, "look-back: one wave per block, <= kScanBlocksMax blocks");
// Slabs inside a tile's range follow chunk order (an XCD-grouped order was faster alone but slower in
// the 3-stream step).
__global__ __launch_bounds__(kColW * kColG) void k_bin_colscan(
    int T, int NB, uint32_t *__restrict__ chunk_off, uint32_t *__restrict__ tile_count, uint2 *__restrict__ ranges,
    uint32_t *__restrict__ tile_cursor, uint32_t *__restrict__ seg_off, uint32_t *__restrict__ sort_lists,
    uint32_t *__restrict__ tile_rank, uint32_t *__restrict__ ws, const uint32_t *__restrict__ block_sums,
    uint32_t *__restrict__ block_off, uint32_t *__restrict__ meta, uint32_t *host_words, uint32_t cap, int ks) {
    __shared__ uint32_t s_part[kColG][kColW + 1];
    __shared__ uint32_t s_tile[kColW];
    __shared__ uint32_t s_blk, s_last;
    __shared__ uint32_t s_red[16];
    __shared__ uint32_t s_lpt[kOrderBuckets];  // this block's tiles per LPT bucket, then the block's base
    uint64_t *look = reinterpret_cast<uint64_t *>(ws);
    uint32_t *ctr = ws + 2 * kScanBlocksMax, *lpt = ctr + kScanCtr;
    // blocks take their columns by blockIdx: a grid is dispatched in block order, so every block a
    // look-back waits on is resident
    if (threadIdx.x == 0) s_blk = blockIdx.x;
    for (int i = threadIdx.x; i < kOrderBuckets; i += blockDim.x) s_lpt[i] = 0;
    __syncthreads();
    const int blk = (int)s_blk;
    const int col = threadIdx.x % kColW, grp = threadIdx.x / kColW;
    const int t = blk * kColW + col;
    const int R = div_up(NB, kColG);
    const int r0 = min(NB, grp * R), r1 = min(NB, r0 + R);
    uint32_t *p = chunk_off + t;
    uint32_t v[kColR];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kColR; ++k) {  // slab positions r0 .. r1 - 1 of this group
        v[k] = (t < T && r0 + k < r1) ? p[(size_t)(r0 + k) * T] : 0u;
        sum += v[k];
    }
    s_part[grp][col] = sum;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kColG; ++k) {
        const uint32_t c = s_part[k][col];
        pre += k < grp ? c : 0u;
        tot += c;
    }
    if (t < T) {
        if (grp == 0) tile_count[t] = tot;
#pragma unroll
        for (int k = 0; k < kColR; ++k) {
            if (r0 + k < r1) p[(size_t)(r0 + k) * T] = pre;
            pre += v[k];
        }
    }
    if (grp == 0) s_tile[col] = t < T ? tot : 0u;
    __syncthreads();
    if (threadIdx.x < 64) {  // wave 0: the block's prefix, then its tiles' outputs
        const int lane = threadIdx.x;
        const uint32_t cnt = lane < kColW ? s_tile[lane] : 0u, sb = seg_bounds(cnt, ks);
        const uint32_t ic = wave_incl_scan_u32(cnt), is = wave_incl_scan_u32(sb);
        const uint32_t agg_c = (uint32_t)__builtin_amdgcn_readlane((int)ic, 63);
        const uint32_t agg_s = (uint32_t)__builtin_amdgcn_readlane((int)is, 63);
        if (lane == 0)
            __hip_atomic_store(&look[blk], (blk == 0 ? kScanInc : kScanAgg) | ((uint64_t)agg_s << 32) | agg_c,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t ex_c = 0, ex_s = 0;
        for (int base = blk - 1; base >= 0; base -= 64) {  // predecessors base, base - 1, ... (lane order)
            const int j = base - lane;
            uint64_t w;
            uint64_t inc, zero;
            for (;;) {
                w = j >= 0 ? __hip_atomic_load(&look[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kScanInc;
                inc = __ballot((w >> 62) == 2u);
                zero = __ballot((w >> 62) == 0u);
                const uint64_t upto = inc ? (~0ull >> (63 - __builtin_ctzll(inc))) : ~0ull;  // lanes up to the nearest inclusive
                if (!(zero & upto)) break;
                __builtin_amdgcn_s_sleep(1);
            }
            const int first = inc ? __builtin_ctzll(inc) : 64;
            const uint32_t wc = lane <= first ? (uint32_t)w : 0u;
            const uint32_t ws_ = lane <= first ? (uint32_t)(w >> 32) & 0x3FFFFFFFu : 0u;
            ex_c += (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_u32(wc), 63);
            ex_s += (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_u32(ws_), 63);
            if (inc) break;
        }
        if (lane == 0 && blk > 0)
            __hip_atomic_store(&look[blk], kScanInc | ((uint64_t)(ex_s + agg_s) << 32) | (ex_c + agg_c),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int tl = blk * kColW + lane;
        // rank inside the tile's LPT bucket: the block's tiles of one bucket take one global reservation
        // (same-address global atomics serialise: one per tile cost ~100 us at C3)
        const uint32_t bkt = lpt_bucket(cnt);
        const bool mine = lane < kColW && tl < T;
        const uint32_t local = mine ? atomicAdd(&s_lpt[bkt], 1u) : 0u;
        wave_lds_sync();
        if (mine && local == 0) s_lpt[bkt] = atomicAdd(&lpt[bkt], s_lpt[bkt]);
        wave_lds_sync();
        if (mine) tile_rank[tl] = s_lpt[bkt] + local;
        if (mine) {
            const uint32_t ex = ex_c + ic - cnt;
            ranges[tl] = cnt ? make_uint2(ex, ex + cnt) : make_uint2(0, 0);  // empty: {0,0} like the reference
            tile_cursor[tl] = ex;
            seg_off[tl] = ex_s + is - sb;
            if (cnt > (uint32_t)kSortCap) {  // long: merge-sorted; listed from the end
                sort_lists[T - 1 - atomicAdd(&ctr[3], 1u)] = (uint32_t)tl;
                atomicMax(&ctr[4], cnt);
            } else if (cnt > (uint32_t)kFwdSortCap) {
                sort_lists[atomicAdd(&ctr[2], 1u)] = (uint32_t)tl;
            }
        }
    }
    // No agent-scope fences: the 8 XCDs' L2s are not coherent, so such a fence writes back / invalidates
    // the whole L2 (a first version with __threadfence() and acquire / release look-back words took
    // ~100 us).  Everything another block reads here is a device-scope atomic (payload and flag share
    // one word); every wave drains its own atomics (an explicit vmcnt(0): the workgroup-scope fence
    // waits for LDS only) before the block counts itself done.
    drain_vmem();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(&ctr[1], 1u) == gridDim.x - 1 ? 1u : 0u;
    __syncthreads();
    if (!s_last) return;
    // the last block: every tile is classified and ranked
    const uint64_t fin = __hip_atomic_load(&look[gridDim.x - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t K = (uint32_t)fin, n_seg = (uint32_t)(fin >> 32) & 0x3FFFFFFFu;
    {   // LPT bucket counts -> offsets (kOrderBuckets / blockDim.x per thread)
        constexpr int kPer = kOrderBuckets / (kColW * kColG);
        uint32_t h[kPer], hs = 0;
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            h[i] = __hip_atomic_load(&lpt[threadIdx.x * kPer + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            hs += h[i];
        }
        uint32_t tt;
        uint32_t e = block_excl_scan_u32(hs, s_red, &tt);
#pragma unroll
        for (int i = 0; i < kPer; ++i) {
            lpt[threadIdx.x * kPer + i] = e;
            e += h[i];
        }
    }
    {   // chunk emission offsets (NB <= 512 <= blockDim.x)
        const uint32_t bs = (int)threadIdx.x < NB ? block_sums[threadIdx.x] : 0u;
        uint32_t btot;
        const uint32_t bex = block_excl_scan_u32(bs, s_red, &btot);
        if ((int)threadIdx.x < NB) block_off[threadIdx.x] = bex;
    }
    if (threadIdx.x == 0) {
        const uint32_t n_mid = __hip_atomic_load(&ctr[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t n_long = __hip_atomic_load(&ctr[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t max_long = __hip_atomic_load(&ctr[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        seg_off[T] = n_seg;
        meta[0] = K;
        // speculative enqueue (gsr_forward_info): the kernels queued before the host read K run
        // only when the BINNING capacity holds K and no list needs the merge sort
        meta[1] = (cap && K <= cap && n_long == 0u) ? 1u : 0u;
        meta[2] = n_mid;
        if (host_words) {
            __hip_atomic_store(host_words + 1, n_mid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_words + 2, n_long, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_words + 3, max_long, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_words, K, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// ------------------------------------------------------------------------------------------
// Single block (1024 threads): exclusive scan of the T tile counts -> ranges/cursors, and of the
// NB chunk sums -> chunk emission offsets.  meta[0] = K.  Up to 16384 tiles every thread holds its
// (at most 16) consecutive counts in registers, loaded with every load in flight, so the kernel does
// one block scan instead of a chain of dependent strided load-scan rounds; larger grids take the
// strided path.
__global__ __launch_bounds__(1024) void k_bin_scan(int T, int NB, const uint32_t *__restrict__ tile_count,
                                                   uint2 *__restrict__ ranges,
                                                   uint32_t *__restrict__ tile_cursor,
                                                   const uint32_t *__restrict__ block_sums,
                                                   uint32_t *__restrict__ block_off,
                                                   uint32_t *__restrict__ meta,
                                                   uint32_t *host_words,
                                                   uint32_t *__restrict__ tile_order,
                                                   uint32_t *__restrict__ sort_lists,
                                                   uint32_t *__restrict__ seg_off, uint32_t cap, int ks) {
    __shared__ uint32_t s_red[16];
    __shared__ uint32_t s_hist[kOrderBuckets];
    __shared__ uint32_t s_cls[3];
    if (threadIdx.x < 3) s_cls[threadIdx.x] = 0;
    if (T <= kScanRegs * (int)blockDim.x && NB <= (int)blockDim.x) {
        // fast path: thread owns tiles [tid c, tid c + c); all counts loaded up front, one block scan
        const int c = div_up(T, (int)blockDim.x), t0 = threadIdx.x * c;
        uint32_t cnt[kScanRegs];
#pragma unroll
        for (int i = 0; i < kScanRegs; ++i) cnt[i] = (i < c && t0 + i < T) ? tile_count[t0 + i] : 0u;
        const uint32_t bsum = (int)threadIdx.x < NB ? block_sums[threadIdx.x] : 0u;
        uint32_t mine = 0;
#pragma unroll
        for (int i = 0; i < kScanRegs; ++i) mine += cnt[i];
        uint32_t K;
        uint32_t ex = block_excl_scan_u32(mine, s_red, &K);
#pragma unroll
        for (int i = 0; i < kScanRegs; ++i) {
            const int t = t0 + i;
            if (i < c && t < T) {
                ranges[t] = cnt[i] ? make_uint2(ex, ex + cnt[i]) : make_uint2(0, 0);  // empty: {0,0} like the reference
                tile_cursor[t] = ex;
                if (cnt[i] > (uint32_t)kSortCap) {  // long: merge-sorted; listed from the end
                    sort_lists[T - 1 - atomicAdd(&s_cls[1], 1u)] = (uint32_t)t;
                    atomicMax(&s_cls[2], cnt[i]);
                } else if (cnt[i] > (uint32_t)kFwdSortCap) {
                    sort_lists[atomicAdd(&s_cls[0], 1u)] = (uint32_t)t;
                }
            }
            ex += cnt[i];
        }
        // backward segment boundaries: exclusive prefix over tiles (index of each tile's first state)
        uint32_t nbs = 0;
#pragma unroll
        for (int i = 0; i < kScanRegs; ++i) nbs += (i < c && t0 + i < T) ? seg_bounds(cnt[i], ks) : 0u;
        uint32_t nbt;
        uint32_t sex = block_excl_scan_u32(nbs, s_red, &nbt);
#pragma unroll
        for (int i = 0; i < kScanRegs; ++i) {
            if (i < c && t0 + i < T) {
                seg_off[t0 + i] = sex;
                sex += seg_bounds(cnt[i], ks);
            }
        }
        if (threadIdx.x == 0) seg_off[T] = nbt;
        uint32_t btot;
        const uint32_t bex = block_excl_scan_u32(bsum, s_red, &btot);  // contains the barrier s_cls needs
        if ((int)threadIdx.x < NB) block_off[threadIdx.x] = bex;
        if (threadIdx.x == 0) {
            meta[0] = K;
            // speculative enqueue (gsr_forward_info): the kernels queued before the host read K run
            // only when the BINNING capacity holds K and no list needs the merge sort
            meta[1] = (cap && K <= cap && s_cls[1] == 0u) ? 1u : 0u;
            meta[2] = s_cls[0];
            if (host_words) {
                for (int q = 0; q < 3; ++q)
                    __hip_atomic_store(host_words + 1 + q, s_cls[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(host_words, K, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        lpt_order_regs<kScanRegs>(T, c, cnt, tile_order, s_hist, s_red);
        return;
    }
    uint32_t carry = 0;
    for (int base = 0; base < T; base += blockDim.x) {
        const int t = base + threadIdx.x;
        const uint32_t c = t < T ? tile_count[t] : 0;
        uint32_t tot;
        const uint32_t ex = block_excl_scan_u32(c, s_red, &tot) + carry;
        if (t < T) {
            ranges[t] = c ? make_uint2(ex, ex + c) : make_uint2(0, 0);  // empty tiles: {0,0} like the reference
            tile_cursor[t] = ex;
        }
        carry += tot;
    }
    uint32_t carry3 = 0;
    for (int base = 0; base < T; base += blockDim.x) {
        const int t = base + threadIdx.x;
        const uint32_t nb = t < T ? seg_bounds(tile_count[t], ks) : 0;
        uint32_t tot;
        const uint32_t ex = block_excl_scan_u32(nb, s_red, &tot) + carry3;
        if (t < T) seg_off[t] = ex;
        carry3 += tot;
    }
    if (threadIdx.x == 0) seg_off[T] = carry3;
    uint32_t carry2 = 0;
    for (int base = 0; base < NB; base += blockDim.x) {
        const int b = base + threadIdx.x;
        const uint32_t c = b < NB ? block_sums[b] : 0;
        uint32_t tot;
        const uint32_t ex = block_excl_scan_u32(c, s_red, &tot) + carry2;
        if (b < NB) block_off[b] = ex;
        carry2 += tot;
    }
    // tiles too long for the in-render sort (k_tile_sort launches exactly one block per such tile)
    __syncthreads();
    for (int t = threadIdx.x; t < T; t += blockDim.x) {
        const uint32_t n = tile_count[t];
        if (n == 0) continue;
        if (n > (uint32_t)kSortCap) {
            sort_lists[T - 1 - atomicAdd(&s_cls[1], 1u)] = (uint32_t)t;
            atomicMax(&s_cls[2], n);
        } else if (n > (uint32_t)kFwdSortCap) {
            sort_lists[atomicAdd(&s_cls[0], 1u)] = (uint32_t)t;
        }
    }
    lds_barrier();  // s_cls: no-return LDS atomics above
    if (threadIdx.x == 0) {
        meta[0] = carry;
        meta[1] = (cap && carry <= cap && s_cls[1] == 0u) ? 1u : 0u;
        meta[2] = s_cls[0];
        // publish straight into host-mapped pinned memory (the host spins on word 0): no copy
        // kernel, no stream synchronisation.  K goes last with system-scope release.
        if (host_words) {
            for (int c = 0; c < 3; ++c)
                __hip_atomic_store(host_words + 1 + c, s_cls[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(host_words, carry, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    // forward render dispatch order: longest tile lists first
    lpt_order(T, [&](int t) { return tile_count[t]; }, tile_order, s_hist, s_red);
}

// ------------------------------------------------------------------------------------------
// Scatter keys into tile buckets.  Each chunk re-counts its tile histogram in LDS, reserves one
// contiguous slab per non-empty tile with a single global atomic, then hands out slots from LDS.
// The order inside a tile is arbitrary here; k_tile_sort makes it canonical.
template <bool USE_LDS>
__global__ __launch_bounds__(kBinThreads) void k_bin_emit(int P, int CH, int T, int gx,
                                                  const uint2 *__restrict__ rects,
                                                  const uint32_t *__restrict__ tiles,
                                                  const float *__restrict__ depth,
                                                  const uint32_t *__restrict__ block_off,
                                                  uint32_t *__restrict__ tile_cursor,
                                                  uint32_t *__restrict__ goff,
                                                  uint4 *__restrict__ pairs, uint32_t K,
                                                  const uint32_t *__restrict__ chunk_off,
                                                  const uint32_t *__restrict__ spec_ok,
                                                  const uint32_t *__restrict__ tile_count,
                                                  const uint32_t *__restrict__ tile_rank,
                                                  const uint32_t *__restrict__ lpt_off,
                                                  uint32_t *__restrict__ tile_order) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_cur[];
    __shared__ uint32_t s_red[16];
    if (spec_ok && *spec_ok == 0u) return;  // speculative launch whose capacity failed: the host redoes it
    const int b = blockIdx.x;
    const int g0 = b * CH, g1 = min(P, g0 + CH);
    if (tile_rank) {  // the forward's dispatch order (k_bin_colscan's LPT buckets): this block's share of tiles
        const int per = div_up(T, (int)gridDim.x), t1 = min(T, (b + 1) * per);
        for (int t = b * per + (int)threadIdx.x; t < t1; t += blockDim.x)
            tile_order[lpt_off[lpt_bucket(tile_count[t])] + tile_rank[t]] = (uint32_t)t;
    }
    GSR_EMIT_STAMP(0);
    if (USE_LDS) {  // this chunk's slab in every tile: the tile's range start + the column scan
        const uint32_t *row = chunk_off + (size_t)b * T;
        for (int t = threadIdx.x; t < T; t += blockDim.x) s_cur[t] = tile_cursor[t] + row[t];
        __syncthreads();
        GSR_EMIT_STAMP(1);
        GSR_EMIT_STAMP(2);
    }
    // emission offsets (exclusive scan of tiles over Gaussian index) + key scatter
    uint32_t carry = block_off[b];
    for (int base = g0; base < g1; base += blockDim.x) {
        const int g = base + threadIdx.x;
        const uint32_t n = g < g1 ? tiles[g] : 0;
        uint32_t tot;
        const uint32_t ex = block_excl_scan_u32(n, s_red, &tot) + carry;
        carry += tot;
        if (g < g1) {
            goff[g] = ex;
            if (n) {
                const uint2 r = rects[g];
                const int x0 = r.x & 0xFFFF, y0 = r.x >> 16, x1 = r.y & 0xFFFF, y1 = r.y >> 16;
                const uint32_t dbits = __float_as_uint(depth[g]);
                uint32_t e = ex;  // emission index: y-major over the rect, as the reference emits
                for (int y = y0; y < y1; ++y)
                    for (int x = x0; x < x1; ++x, ++e) {
                        const int t = y * gx + x;
                        const uint32_t pos = USE_LDS ? atomicAdd(&s_cur[t], 1u) : atomicAdd(&tile_cursor[t], 1u);
                        pairs[pos] = make_uint4((uint32_t)g, dbits, e, 0u);
                    }
            }
        }
    }
    if (b == gridDim.x - 1 && threadIdx.x == 0) goff[P] = spec_ok ? spec_ok[-1] : K;  // meta[0] = K
#ifdef GSR_TRACE
    __syncthreads();
    GSR_EMIT_STAMP(3);
#endif
}

// ------------------------------------------------------------------------------------------
// Per-tile sort of (depth_bits << 32 | index) keys, then outputs.

// ---- wave-level register bitonic sort (gfx950 cross-lane ops) ------------------------------
// Element i = lane * R + r lives in register r of `lane`: exchanges at distance < R stay inside a
// lane, larger distances are lane xors d = dist / R, all on the VALU (no LDS round trip):
// d = 1, 2 DPP quad_perm; d = 4 DPP row_half_mirror then quad reversal; d = 8 DPP row_ror:8;
// d = 16, 32 v_permlane16_swap / v_permlane32_swap.
template <int D>
__device__ inline uint32_t lane_xor(uint32_t x) {
    if constexpr (D == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
    else if constexpr (D == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
    else if constexpr (D == 4) {
        const int m = __builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // i -> 7 - i per 8 lanes
        return (uint32_t)__builtin_amdgcn_mov_dpp(m, 0x1B, 0xF, 0xF, false);     // reverse each quad
    } else if constexpr (D == 8) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xF, 0xF, false);
    else if constexpr (D == 16) {
        auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (threadIdx.x & 16) ? r[0] : r[1];
    } else {
        auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (threadIdx.x & 32) ? r[0] : r[1];
    }
}

template <int R, int D>
__device__ inline void bitonic_xlane(uint64_t (&k)[R], uint32_t (&v)[R], bool take_min) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t plo = lane_xor<D>((uint32_t)k[r]), phi = lane_xor<D>((uint32_t)(k[r] >> 32));
        const uint32_t pv = lane_xor<D>(v[r]);
        const uint64_t pk = ((uint64_t)phi << 32) | plo;
        const bool mine = (k[r] < pk) == take_min;
        k[r] = mine ? k[r] : pk;
        v[r] = mine ? v[r] : pv;
    }
}

// Stages j = J, J/2, ..., 1 (J < 64 R) of the bitonic merge of size kk, on the wave's elements
// i = gbase + lane * R + r (ascending where (i & kk) == 0).
template <int R, int J>
__device__ inline void wave_merge_stages(uint64_t (&k)[R], uint32_t (&v)[R], int lane, uint32_t gbase, uint32_t KK) {
    if constexpr (J > 0) {
        if constexpr (J < R) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (r & J) continue;
                const int r2 = r | J;
                const bool asc = ((gbase + lane * R + r) & KK) == 0;
                if ((k[r] > k[r2]) == asc) {
                    const uint64_t t = k[r]; k[r] = k[r2]; k[r2] = t;
                    const uint32_t u = v[r]; v[r] = v[r2]; v[r2] = u;
                }
            }
        } else {
            constexpr int D = J / R;
            const bool asc = ((gbase + lane * R) & KK) == 0;
            const bool take_min = ((lane & D) == 0) == asc;
            bitonic_xlane<R, D>(k, v, take_min);
        }
        wave_merge_stages<R, J / 2>(k, v, lane, gbase, KK);
    }
}

// Full bitonic network over the wave's 64 R elements (merge sizes 2 .. 64 R); the last merge runs
// descending when (gbase & 64 R) != 0, which is what the next cross-wave merge needs.
template <int R, int KK>
__device__ inline void wave_sort_stages(uint64_t (&k)[R], uint32_t (&v)[R], int lane, uint32_t gbase) {
    if constexpr (KK <= 64 * R) {
        wave_merge_stages<R, KK / 2>(k, v, lane, gbase, KK);
        wave_sort_stages<R, 2 * KK>(k, v, lane, gbase);
    }
}

// LDS slot of sorted element i: one pad element after every 16, so that the 16 lanes of a register
// row -- elements l R + r, l = 0..15 -- land on 16 distinct 8-byte bank pairs (unpadded, lanes l,
// l + 16 / R, ... collide: a 4-way conflict at R = 4).  A lane's R elements (R | 16) stay adjacent, so
// its stores and the exchange partner's loads (i ^ j, j a multiple of 64 R) are one address plus
// immediate offsets, and consecutive elements stay conflict-free for the readers of the sorted run.
__device__ inline uint32_t sort_slot(uint32_t i) { return i + (i >> 4); }
constexpr int sort_slots(int n) { return n + n / 16; }

// One cross-wave compare-exchange stage (distance J >= 64 R) of merge size KK through LDS.
template <int R>
__device__ inline void block_xchg_stage(uint64_t (&k)[R], uint32_t (&v)[R], uint32_t ibase, int kk, int j,
                                        uint64_t *s_key, uint32_t *s_val) {
    const uint32_t sb = sort_slot(ibase), qb = sort_slot(ibase ^ (uint32_t)j);
#pragma unroll
    for (int r = 0; r < R; ++r) { s_key[sb + r] = k[r]; s_val[sb + r] = v[r]; }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t i = ibase + r;
        const uint64_t pk = s_key[qb + r];
        const uint32_t pv = s_val[qb + r];
        const bool take_min = ((i & j) == 0) == ((i & kk) == 0);
        const bool mine = (k[r] < pk) == take_min;
        k[r] = mine ? k[r] : pk;
        v[r] = mine ? v[r] : pv;
    }
    __syncthreads();
}

// Sort one tile's n <= 64 R NW (key, emission) pairs with the block's NW waves: each wave sorts its
// 64 R-element segment in registers (DPP / swizzle / permlane exchanges), then every cross-wave
// merge level exchanges through LDS for distances >= 64 R and finishes in registers.  Leaves sorted
// element i (key, emission) at s_key / s_val[sort_slot(i)], i < n (arrays of sort_slots(64 R NW)).  Keys are
// (depth_bits << 32 | index), unique inside a tile.
template <int R, int NW>
__device__ inline void block_sort_tile(int n, uint32_t start, const uint4 *__restrict__ pairs, uint64_t *s_key,
                                       uint32_t *s_val) {
    constexpr int SEG = 64 * R;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t gbase = (uint32_t)(w * SEG), ibase = gbase + lane * R;
    uint64_t k[R];
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = (int)ibase + r;
        const uint4 q = i < n ? pairs[start + i] : make_uint4(~0u, ~0u, 0u, 0u);  // +inf padding sorts last
        k[r] = pair_key(q);
        v[r] = q.z;
    }
    wave_sort_stages<R, 2>(k, v, lane, gbase);
    for (uint32_t kk = 2 * SEG; kk <= (uint32_t)(NW * SEG); kk <<= 1) {
        for (uint32_t j = kk >> 1; j >= (uint32_t)SEG; j >>= 1) block_xchg_stage<R>(k, v, ibase, kk, j, s_key, s_val);
        wave_merge_stages<R, SEG / 2>(k, v, lane, gbase, kk);
    }
    const uint32_t sb = sort_slot(ibase);
#pragma unroll
    for (int r = 0; r < R; ++r) { s_key[sb + r] = k[r]; s_val[sb + r] = v[r]; }
    __syncthreads();
}

// Tiles longer than kFwdSortCap and at most kSortCap pairs (one 512-thread block each, launched only
// for those tiles): the register + LDS hybrid of block_sort_tile over 8 waves (4 or 8 keys per lane).
// Launched with one block per such tile (nlist = n_mid known on the host), or -- speculative
// enqueue, before the host knows the count -- with a fixed grid whose blocks loop over the list
// count k_bin_scan left in meta[2] (spec_ok = meta + 1).
__global__ __launch_bounds__(512) void k_tile_sort(int gx, const uint32_t *__restrict__ tiles,
                                                    const uint2 *__restrict__ ranges,
                                                    uint4 *__restrict__ pairs,
                                                    uint32_t *__restrict__ point_list,
                                                    uint32_t *__restrict__ slot_emit, uint32_t nlist,
                                                    const uint32_t *__restrict__ spec_ok) {
    __shared__ uint64_t s_keys[sort_slots(kSortCap)];
    __shared__ uint32_t s_vals[sort_slots(kSortCap)];
    if (spec_ok) {
        if (*spec_ok == 0u) return;
        nlist = spec_ok[1];  // meta[2]: tiles of kFwdSortCap < n <= kSortCap pairs
    }
    static_assert(kSortCap == 8 * 64 * 8, "k_tile_sort: 8 waves x 64 lanes x 8 keys");
    for (uint32_t li = blockIdx.x; li < nlist; li += gridDim.x) {
        const int tile = (int)tiles[li];
        const uint2 rg = ranges[tile];
        const int n = (int)(rg.y - rg.x);
        if (n <= 4 * 64 * 8) block_sort_tile<4, 8>(n, rg.x, pairs, s_keys, s_vals);
        else block_sort_tile<8, 8>(n, rg.x, pairs, s_keys, s_vals);
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const uint32_t sl = sort_slot((uint32_t)i);
            point_list[rg.x + i] = (uint32_t)s_keys[sl];
            slot_emit[rg.x + i] = s_vals[sl];
        }
        __syncthreads();  // the LDS keys are reused by the block's next list
    }
}

// ---- lists longer than kSortCap: multi-block merge sort -------------------------------------
// (a densified scene's dense tiles: tens of thousands of pairs in one tile).  The tile's range is
// cut into kSortCap chunks, each sorted in LDS by its own block (k_chunk_sort, block_sort_tile,
// written back in place as 16-byte records), then log2(n / kSortCap) merge passes double the sorted
// run length (k_merge_pass): every block produces kSortCap outputs of one pair of runs, finding its
// share of each run by a merge-path search (64-ary, one wave per end of the window), staging that
// window in LDS and merging 8 outputs per thread.  Passes ping-pong between the pair records and a
// temporary copy; the last one writes the point list and the slot -> emission map.  Keys
// (depth bits << 32 | index) are unique inside a tile, so the order is exactly the stable (tile,
// depth) order of the reference's radix sort.  Grid: (max chunks of a long tile, long tiles).
__device__ inline uint4 key_record(uint64_t k, uint32_t emit) {
    return make_uint4((uint32_t)k, (uint32_t)(k >> 32), emit, 0u);
}

__global__ __launch_bounds__(512) void k_chunk_sort(int T, const uint32_t *__restrict__ lists,
                                                     const uint2 *__restrict__ ranges, uint4 *__restrict__ pairs) {
    __shared__ uint64_t s_keys[sort_slots(kSortCap)];
    __shared__ uint32_t s_vals[sort_slots(kSortCap)];
    const int tile = (int)lists[T - 1 - (int)blockIdx.y];  // long tiles are listed from the end
    const uint2 rg = ranges[tile];
    const int n = (int)(rg.y - rg.x);
    const int c0 = (int)blockIdx.x * kSortCap;
    if (c0 >= n) return;
    const int m = min(kSortCap, n - c0);
    block_sort_tile<8, 8>(m, rg.x + c0, pairs, s_keys, s_vals);
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const uint32_t sl = sort_slot((uint32_t)i);
        pairs[rg.x + c0 + i] = key_record(s_keys[sl], s_vals[sl]);
    }
}

// Merge-path split of diagonal d between sorted runs a (length la) and b (length lb): the number of
// a's elements among the first d outputs.  One wave, 64 probes per round.
__device__ inline uint32_t merge_split(const uint4 *__restrict__ a, uint32_t la, const uint4 *__restrict__ b,
                                       uint32_t lb, uint32_t d) {
    const int lane = threadIdx.x & 63;
    uint32_t lo = d > lb ? d - lb : 0u, hi = min(d, la);  // answer in [lo, hi]
    while (lo < hi) {
        const uint32_t span = hi - lo, step = (span + 63) / 64;
        const uint32_t x = lo + (uint32_t)lane * step;
        // P(x): a[x] precedes b[d - 1 - x] (true for a prefix of x, false after)
        const bool p = x < hi && pair_key(a[x]) < pair_key(b[d - 1 - x]);
        const uint32_t c = (uint32_t)__popcll(__ballot(p));
        const uint32_t nlo = c ? lo + (c - 1) * step + 1 : lo;
        const uint32_t nhi = min(hi, lo + c * step);
        lo = nlo;
        hi = max(nlo, nhi);
    }
    return lo;
}

__global__ __launch_bounds__(512) void k_merge_pass(int T, const uint32_t *__restrict__ lists,
                                                     const uint2 *__restrict__ ranges, uint32_t L,
                                                     const uint4 *__restrict__ src, uint4 *__restrict__ dst,
                                                     int final_pass, uint32_t *__restrict__ point_list,
                                                     uint32_t *__restrict__ slot_emit) {
    __shared__ uint64_t s_ka[kSortCap], s_kb[kSortCap];
    __shared__ uint32_t s_va[kSortCap], s_vb[kSortCap];
    __shared__ uint32_t s_split[2];
    const int tile = (int)lists[T - 1 - (int)blockIdx.y];
    const uint2 rg = ranges[tile];
    const uint32_t n = rg.y - rg.x;
    const uint32_t o0 = blockIdx.x * (uint32_t)kSortCap;
    if (o0 >= n) return;
    const uint32_t pb = o0 / (2 * L) * (2 * L);                    // this pair of runs starts here
    const uint32_t la = min(L, n - pb), lb = n - pb > L ? min(L, n - pb - L) : 0u;
    const uint4 *a = src + rg.x + pb, *b = a + la;
    const uint32_t d0 = o0 - pb, d1 = min(d0 + (uint32_t)kSortCap, la + lb);
    const int wv = threadIdx.x >> 6;
    if (wv < 2) {
        const uint32_t sp = merge_split(a, la, b, lb, wv == 0 ? d0 : d1);
        if ((threadIdx.x & 63) == 0) s_split[wv] = sp;
    }
    __syncthreads();
    const uint32_t i0 = s_split[0], i1 = s_split[1], j0 = d0 - i0, j1 = d1 - i1;
    const uint32_t na = i1 - i0, nb = j1 - j0;
    for (uint32_t i = threadIdx.x; i < na; i += blockDim.x) { const uint4 q = a[i0 + i]; s_ka[i] = pair_key(q); s_va[i] = q.z; }
    for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) { const uint4 q = b[j0 + i]; s_kb[i] = pair_key(q); s_vb[i] = q.z; }
    __syncthreads();
    // 8 consecutive outputs per thread: its diagonal's split in LDS, then a sequential merge
    constexpr uint32_t kPer = kSortCap / 512;
    const uint32_t dl = threadIdx.x * kPer;
    if (dl >= na + nb) return;
    uint32_t lo = dl > nb ? dl - nb : 0u, hi = min(dl, na);
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_ka[mid] < s_kb[dl - 1 - mid]) lo = mid + 1; else hi = mid;
    }
    uint32_t ia = lo, ib = dl - lo;
    const uint32_t e = min(dl + kPer, na + nb);
    for (uint32_t o = dl; o < e; ++o) {
        const bool take_a = ib >= nb || (ia < na && s_ka[ia] < s_kb[ib]);
        const uint64_t k = take_a ? s_ka[ia] : s_kb[ib];
        const uint32_t v = take_a ? s_va[ia] : s_vb[ib];
        ia += take_a; ib += !take_a;
        const size_t slot = (size_t)rg.x + pb + d0 + o;
        if (final_pass) { point_list[slot] = (uint32_t)k; slot_emit[slot] = v; }
        else dst[slot] = key_record(k, v);
    }
}

// ------------------------------------------------------------------------------------------
// Per-tile depth sort + front-to-back blend.  One 256-thread block per 16x16 tile, dispatched
// longest list first (tile_order).  A list of up to kFwdSortCap pairs is first depth-sorted by the
// block (block_sort_tile: registers + three LDS exchange stages), which also writes the backward's
// point_list / slot_emit; longer lists were sorted beforehand by k_tile_sort.  The blend walks the
// sorted list in batches of 64: the block stages each batch once (thread 4e + q gathers entry e's
// render record and tests it against quarter q = pixel rows 4q..4q+3 with a conservative ellipse
// bound), then wave q blends its 16x4 quarter (one pixel per lane) over the entries whose bit q is
// set; saturated quarters skip their evaluations and the walk ends when all four are saturated.
// Asynchronous forwards (gsr_forward_async): when k_bin_scan found the speculative capacity too
// small (spec_ok == 0: the queued kernels return at once), the speculative k_render_fwd's first wave
// holds the stream until the library's resolver thread has redone the post-scan kernels exactly on its
// own stream and published `seq` in the forward's gate word (host-mapped) -- everything the caller
// queues after the forward is ordered behind it.  When the speculation stood nothing waits.  A gate that
// never opens (the resolver died or is stuck) is abandoned after `timeout` ticks (5 s by default) with
// the forward's error word set, so a failure cannot hang the device; the host then fails that forward's
// resolution (gsr_forward_resolve), i.e. the backward of the step whose outputs are not final.
__device__ inline void gate_wait(const uint32_t *gate, uint32_t seq, uint32_t *err, uint64_t timeout) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while ((int32_t)(__hip_atomic_load(gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - seq) < 0) {
        __builtin_amdgcn_s_sleep(100);
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
            // the gate is read again before the error is published: a gate the resolver
            // opened during the last sleep means the redo completed first, so the outputs are final
            if (threadIdx.x == 0 &&
                (int32_t)(__hip_atomic_load(gate, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - seq) < 0)
                __hip_atomic_store(err, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
    }
}

// The exact saturation re-walk of one pixel (exact-threshold mode; round 6), by one
// kTSatThreads-thread block of k_render_tsat (below).  The pixel's final T lies within
// the drift window of 1e-4 (gsr_common.h t_window), so its stop is recomputed with the reference's
// transmittance test (SURVEY.md 2.1 row renderCUDA fwd, oracle/gsr_oracle.c ora_render): the threads take
// kTSatThreads list entries at a time -- the fast weight decides which can contribute, as in the blend (p2 <= 0,
// alpha >= kNearLo; a weight in the near window is decided by its exact value) -- and each contributor gets
// its exact weight, min(0.99, o exp(power)) with the reference's expression order and a double-precision
// exp, and the reference's 1 - alpha (one fp32 rounding), packed in list order into LDS.  Wave 0 then runs
// the reference's chain test_T = T * (1 - alpha) over them, four multiplies per LDS read (T only
// decreases: a block of four whose last value is >= 1e-4 keeps all four; the crossing block is stepped
// through), stopping below 1e-4.  So n_contrib and T are the reference's.  The walk can only end before
// the fast one (t_stop in the blend), never after it, so only the entries before the fast n_contrib are
// evaluated.  The fast colour and depth lose the contributions of the entries the fast walk kept past
// the reference's stop (a few at most, at T ~ 1e-4; their weights from the exact chain continued past
// the stop).  The pixel's outputs, its end state for the backward and its state at every segment
// boundary at or past the new n_contrib are written (the earlier boundary states are the fast walk's, as
// for every other pixel); the tile's quarter maxima stay upper bounds, and every entry the pixel keeps was
// seen by the fast walk (whose near records the backward looks up).
#ifndef GSR_TSAT_THREADS  // 64: render_fwd alone -1.2 % against 128 (and 256), profiles/r06_tsat_threads_ab.txt
#define GSR_TSAT_THREADS 64
#endif
constexpr int kTSatThreads = GSR_TSAT_THREADS;  // threads (list entries per round) of a re-walk block
struct TSatRec { float4 r0, r1, r3; };  // position + pre-scaled conic, (C2, opacity, ...), exact conic
__device__ inline TSatRec tsat_load(const float4 *__restrict__ rec, uint32_t g, bool v) {
    TSatRec t;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 *r = rec + (size_t)kRecF4 * g;
    t.r0 = v ? r[0] : z; t.r1 = v ? r[1] : z; t.r3 = v ? r[3] : z;
    return t;
}
// entries [0, nf) of the pixel's list, point list [start, start + nf): T, n_contrib and the fast walk's extra
// contributions E (wave 0's values); the list's point indices two rounds ahead, render records one ahead
__device__ inline void tsat_chain(int nf, const uint32_t *__restrict__ plist, float pfx, float pfy,
                                  const float4 *__restrict__ rec, uint32_t *s_rc, float *s_q, float *s_a,
                                  uint32_t *s_pos, float &T, uint32_t &nex, float4 &E) {
    constexpr int NT = kTSatThreads, NW = NT / 64;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    float Tc = 0.f;
    bool stopped = false;
    uint32_t g_next = t < nf ? plist[t] : 0u;
    TSatRec cur = tsat_load(rec, g_next, t < nf);
    g_next = NT + t < nf ? plist[NT + t] : 0u;
    for (int base = 0; base < nf; base += NT) {
        const int e = base + t;
        const TSatRec r = cur;
        cur = tsat_load(rec, g_next, e + NT < nf);
        g_next = e + 2 * NT < nf ? plist[e + 2 * NT] : 0u;
        bool take = false;
        float al = 0.f;
        if (e < nf) {
            const Blend eb = blend_eval<true>(r.r0, r.r1, pfx, pfy);
            if (eb.p2 <= 0.0f && eb.alpha >= kNearLo) {  // the blend's live test (exact mode)
                const ExactBlend x = exact_blend(r.r0.x, r.r0.y, r.r3, r.r1.y, pfx, pfy);
                take = eb.alpha >= kNearHi || (x.power <= 0.0f && x.alpha >= 1.0f / 255.0f);
                al = x.alpha;
            }
        }
        // pack the contributors in list order: rank = contributors before this thread in the round
        const uint64_t m = __ballot(take);
        if (lane == 0) s_rc[wv] = (uint32_t)__builtin_popcountll(m);
        __syncthreads();
        uint32_t off = 0, nc = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            off += w < wv ? s_rc[w] : 0u;
            nc += s_rc[w];
        }
        if (take) {
            const uint32_t rk = off + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            s_q[rk] = 1.0f - al;  // the reference's (1 - alpha), one fp32 rounding
            s_a[rk] = al;
            s_pos[rk] = (uint32_t)e;
        }
        if (t < 4) s_q[nc + t] = 1.0f;  // padding of the last block of four: T unchanged
        __syncthreads();
        if (wv == 0) {  // the reference's chain (wave-uniform values; every lane computes it)
            const float4 *q4 = reinterpret_cast<const float4 *>(s_q);
            for (uint32_t k = 0; k < nc; k += 4) {
                uint32_t j = 0;
                const uint32_t v = min(4u, nc - k);  // real contributors in the block
                if (!stopped) {
                    const float4 q = q4[k >> 2];
                    const float t1 = T * q.x, t2 = t1 * q.y, t3 = t2 * q.z, t4 = t3 * q.w;
                    if (t4 >= kTSat) {  // all kept (T only decreases)
                        T = t4;
                        nex = s_pos[k + v - 1] + 1u;
                        continue;
                    }
                    // the block crosses: the reference stops at the first value below 1e-4
                    const float tv[4] = {t1, t2, t3, t4};
                    while (tv[j] >= kTSat) ++j;  // (j < v: the padding keeps T >= 1e-4)
                    if (j > 0) {
                        T = tv[j - 1];
                        nex = s_pos[k + j - 1] + 1u;
                    }
                    stopped = true;
                    Tc = T;
                }
                for (; j < v; ++j) {  // the entries past the stop: the fast walk kept them (rare)
                    const float a = s_a[k + j];
                    const float4 c = rec[(size_t)kRecF4 * plist[s_pos[k + j]] + 2];  // (r, g, b, depth)
                    const float w = a * Tc;
                    E.x += c.x * w; E.y += c.y * w; E.z += c.z * w; E.w += c.w * w;
                    Tc = Tc * (1.0f - a);
                }
            }
        }
        __syncthreads();  // (the round's LDS is reused)
    }
}
// the re-walked pixel's outputs (thread 0) and its segment boundaries at or past the new n_contrib (all)
__device__ inline void tsat_store(int px, int py, int W, int H, int n, float4 pe, float dfast, float T, uint32_t nex,
                                  float4 E, const float *__restrict__ bg, float *__restrict__ out_color,
                                  float *__restrict__ out_depth, float4 *__restrict__ pix_end,
                                  uint32_t *__restrict__ n_contrib, size_t sb, float4 *__restrict__ seg_state, int ks,
                                  uint32_t *s_nex) {
    const int t = threadIdx.x;
    const int pid = py * W + px;
    const float4 fin = make_float4(pe.x - E.x, pe.y - E.y, pe.z - E.z, T);
    if (t == 0) {
        pix_end[pid] = fin;
        n_contrib[pid] = nex;
        out_color[pid] = fin.x + T * bg[0];
        out_color[H * W + pid] = fin.y + T * bg[1];
        out_color[2 * H * W + pid] = fin.z + T * bg[2];
        out_depth[pid] = dfast - E.w;
    }
    const uint32_t b0 = (nex + (1u << ks) - 1u) >> ks;  // first boundary index >= n_contrib
    const int lx = px % kTileW, ly = py % kTileH;
    const int bslot = 64 * (ly >> 2) + 16 * (ly & 3) + lx;  // the backward's pixel slot
    const uint32_t nb = n > 0 ? (uint32_t)(n - 1) >> ks : 0u;  // boundaries of the list (1..nb)
    for (uint32_t q = max(b0, 1u) + (uint32_t)t; q <= nb; q += kTSatThreads)
        seg_state[(sb + q - 1u) * kTilePix + bslot] = fin;
    (void)s_nex;
}
// 8 waves per SIMD (<= 64 VGPRs): the blend's latency is hidden by occupancy (6 waves: +17 %,
// profiles/r05_fwd_ilp_ab.txt)
#define GSR_FWD_ATTR __attribute__((amdgpu_waves_per_eu(8, 8)))
template <bool EXACT>
__global__ __launch_bounds__(256) GSR_FWD_ATTR void k_render_fwd(
    int W, int H, int gx, int T, const uint32_t *__restrict__ tile_order, const uint2 *__restrict__ ranges,
    const uint4 *__restrict__ pairs,
    uint32_t *__restrict__ point_list, uint32_t *__restrict__ slot_emit, const float4 *__restrict__ rec,
    const float *__restrict__ bg, float *__restrict__ out_color, float *__restrict__ out_depth,
    float4 *__restrict__ pix_end, uint32_t *__restrict__ n_contrib, uint32_t *__restrict__ tile_maxc,
    const uint32_t *__restrict__ seg_off, float4 *__restrict__ seg_state, const uint32_t *__restrict__ spec_ok,
    int ks, const uint32_t *gate, uint32_t gate_seq, uint32_t *gate_err, uint64_t gate_timeout,
    uint32_t *__restrict__ tile_flag, float4 *__restrict__ near_rec, uint32_t *__restrict__ tsat_n,
    uint32_t *__restrict__ tsat_list, uint32_t tsat_cap) {
    __shared__ uint64_t s_key[sort_slots(kFwdSortCap > 0 ? kFwdSortCap : 1)];
    __shared__ union {
        uint32_t val[sort_slots(kFwdSortCap > 0 ? kFwdSortCap : 1)];  // sort payload (emission index), until written out
        struct {
            // then: the staged batch of 64 render records, part q of entry e at rec[q][e]; rows padded by
            // 2 float4 so that the staging stores of one entry's 3 parts (lanes 4e + q) fall in distinct
            // banks (unpadded the rows are 1 KiB apart: a 3-way conflict in every 8-lane group)
            float4 rec[3][66];
            uint32_t q[64];         // and their quarter masks
        } st;
    } s_u;
    __shared__ uint32_t s_live;     // quarters (bits) with an unsaturated pixel
    __shared__ uint32_t s_near;     // (EXACT) near-threshold weights re-evaluated in this tile
#ifdef GSR_TRACE
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    if (spec_ok && *spec_ok == 0u) {  // speculative launch whose capacity failed: redone by the host
        if (gate && blockIdx.x == 0 && threadIdx.x < 64) gate_wait(gate, gate_seq, gate_err, gate_timeout);  // (asynchronous)
        return;
    }
    const int tile = (int)tile_order[blockIdx.x];
    const uint2 rg = ranges[tile];
    const int n = (int)(rg.y - rg.x);
    const bool sorted_here = n <= kFwdSortCap;
    if (threadIdx.x == 0) s_near = 0;  // (ordered before its atomics by the barrier ahead of the blend)
    if (n > 0 && sorted_here) {
        if (n <= 256) block_sort_tile<1, 4>(n, rg.x, pairs, s_key, s_u.val);
        else if (n <= 512) block_sort_tile<2, 4>(n, rg.x, pairs, s_key, s_u.val);
        else block_sort_tile<4, 4>(n, rg.x, pairs, s_key, s_u.val);
        for (int i = threadIdx.x; i < n; i += 256) {
            const uint32_t sl = sort_slot((uint32_t)i);
            point_list[rg.x + i] = (uint32_t)s_key[sl];
            slot_emit[rg.x + i] = s_u.val[sl];
        }
    }
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tx = tile % gx, ty = tile / gx;
    // wave q blends the 8x8 quarter (8 (q & 1), 8 (q >> 1)) of the tile: a compact footprint crosses
    // fewer quarters than a 16x4 strip (tools/contrib_stats.py: 1.54 vs 1.73 evaluated quarters per
    // list entry at C3)
    const int lx = 8 * (wv & 1) + (lane & 7), ly = 8 * (wv >> 1) + (lane >> 3);
    const int px = tx * kTileW + lx;
    const int py = ty * kTileH + ly;
    const float pfx = (float)px, pfy = (float)py;
    // this pixel's slot in the backward's layout (16x4 strip k = ly / 4, lane = 16 (ly % 4) + lx)
    const int bslot = 64 * (ly >> 2) + 16 * (ly & 3) + lx;
    // staging role: thread 4e + q handles entry e of the batch against quarter q
    const int se = threadIdx.x >> 2, sq = threadIdx.x & 3;
    const float qx0 = (float)(tx * kTileW + 8 * (sq & 1)), qy0 = (float)(ty * kTileH + 8 * (sq >> 1));
    constexpr int kQW = 8, kQH = 8;
    const bool inside = px < W && py < H;
    // The pixel's alpha threshold: 1/255 while it blends, 2 (above any alpha <= 0.99) once it is done
    // (outside the image, or saturated): a finished pixel fails the same compare instead of carrying
    // a done flag through the loop as a lane mask (its mask logic cost ~7 scalar instructions per
    // blended entry).  The decisions are those of !done && blend_ok(e).  EXACT: the live threshold is
    // the lower end of the near window, kNearLo; a weight in [kNearLo, kNearHi) is re-evaluated (and
    // compared with 1/255), any other weight is on the same side of kNearLo as of 1/255.
    constexpr float kThrDone = 2.0f;
    constexpr float kThrLive = EXACT ? kNearLo : 1.0f / 255.0f;
    float thr = inside ? kThrLive : kThrDone;
    const uint32_t pix_key = (uint32_t)(16 * ly + lx);  // near record key: (list position << 8) | pixel
    if (threadIdx.x == 0) s_live = 0;
    __syncthreads();  // sort outputs consumed / s_live cleared
#ifdef GSR_TRACE
    const uint64_t tr_sorted = __builtin_amdgcn_s_memrealtime();  // (diagnostic) the in-render sort's end
#endif
    if (__ballot(thr < kThrDone) && lane == 0) atomicOr(&s_live, 1u << wv);
    float Tt = 1.0f;
    f2v C01 = f2(0.f, 0.f), C2D = f2(0.f, 0.f);  // (C0, C1), (C2, depth): packed accumulators
    uint32_t last = 0;
    // entry se of the NEXT batch: its render record halves (x, y, conic; colour) in registers, loaded
    // one batch ahead so the gathers' latency hides behind the current batch's blend
    float4 pa = make_float4(0.f, 0.f, 0.f, 0.f), pb = pa, pr = pa;
    bool pv = false;
#define FETCH_BATCH(bse)                                                                           \
    do {                                                                                           \
        const int idx_ = (bse) + se;                                                               \
        pv = idx_ < n;                                                                             \
        if (pv) {                                                                                  \
            const uint32_t g_ = sorted_here ? (uint32_t)s_key[sort_slot(idx_)] : point_list[rg.x + idx_]; \
            const float4 *r_ = rec + (size_t)kRecF4 * g_;                                          \
            pa = r_[0];                                                                            \
            pb = r_[1];                                                                            \
            pr = r_[sq < 3 ? sq : 2];                                                              \
        }                                                                                          \
    } while (0)
    FETCH_BATCH(0);
#ifdef GSR_TRACE
    uint64_t tr_batches = 0, tr_walk = 0, tr_entries = 0;  // (diagnostic) batches, walk ticks, evaluations
#endif
    for (int base = 0; base < n; base += 64) {
        lds_barrier();  // previous batch fully consumed; s_live up to date
        const uint32_t live = s_live;
        if (!live) break;
        // segment boundary (every 2^ks entries): this quarter's blend state before entry `base`, the state a
        // backward segment's reverse walk starts from; stored while the quarter is live, i.e. for
        // every boundary below its pixels' last contributor (done pixels store their final state)
        // (8x8 quarters: every quarter stores while any is live -- the backward reads whole 16x4 strips,
        // which span two quarters; a finished pixel's state is its final one)
        if (base > 0 && (base & ((1 << ks) - 1)) == 0) {
            const size_t b = (size_t)seg_off[tile] + ((uint32_t)base >> ks) - 1u;
            seg_state[b * kTilePix + bslot] = make_float4(C01.x, C01.y, C2D.x, Tt);
        }
        // ---- stage the batch (block-wide) ----
        bool hit = false, opaque = false;
        {   // this batch's records were loaded during the previous batch's blend
            const float4 a = pa, b = pb;
            opaque = pv && b.y > 0.99f;  // alpha = min(0.99, o G) can clamp
            if (pv) {
                if (sq < 3) s_u.st.rec[sq][se] = pr;
                hit = ((live >> sq) & 1u) &&
                      !tile_cull(a.x, a.y, -2.f * a.z, -a.w, -2.f * b.x, b.y, b.w, qx0, qy0, qx0 + (kQW - 1), qy0 + (kQH - 1));
            }
            FETCH_BATCH(base + 64);
        }
        // combine the 4 quarter bits of entry se (lanes 4e..4e+3 of this wave) with DPP
        uint32_t bits = hit ? (1u << sq) : 0u;
        bits |= (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0xB1, 0xF, 0xF, false);  // xor 1
        bits |= (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0x4E, 0xF, 0xF, false);  // xor 2
        if (sq == 0) s_u.st.q[se] = bits | ((bits && opaque) ? 16u : 0u);  // bit 4: a clamping entry
        __syncthreads();
        // ---- blend this wave's quarter ----
        const uint32_t qw = s_u.st.q[lane];
        uint64_t m = __ballot((qw >> wv) & 1u);
        if (!((live >> wv) & 1u)) m = 0;
        // batch-uniform: some staged entry's opacity exceeds 0.99 (the backward takes the same variant)
        const bool clamp = __builtin_amdgcn_ballot_w64((qw & 16u) != 0u) != 0;
        // the transmittance test's bound for this batch's entries (EXACT: widened by the drift window at
        // the batch's last position, gsr_common.h t_window)
        const float t_stop = EXACT ? kTSat * (1.0f - t_window((uint32_t)base + 64u)) : kTSat;
        // one entry's blend into this pixel's state (front to back)
        auto take = [&](const Blend &e, bool ok, float4 b, float4 c, int j) {
            const float test_T = fmaf(-e.alpha, Tt, Tt);  // T (1 - alpha), one rounding
            // keep == !(test_T < 1e-4) (test_T is never NaN: T in (0, 1], alpha in [0, 0.99]); the
            // pixel finishes when it takes the entry but may not keep it.  EXACT: on while test_T >=
            // 1e-4 (1 - t_window) (this batch's bound), the pixels that end near 1e-4 are redone by k_render_tsat
            const bool use = ok && test_T >= t_stop;
            thr = (ok && !use) ? kThrDone : thr;
            if (use) {  // an exec-masked update: no selects for w, T and the last contributor (-1 %)
                const float w = e.alpha * Tt;
                C01 = fma2(f2(c.x, c.y), f2(w, w), C01);  // C0, C1 += (c.x, c.y) w
                C2D = fma2(f2(c.z, c.w), f2(w, w), C2D);  // C2, depth += (c.z, depth) w
                Tt = test_T;
                last = (uint32_t)(base + j + 1);
            }
        };
        auto walk = [&](auto clamp_c) {
            constexpr bool CL = decltype(clamp_c)::value;
            while (m) {
                const int j = __builtin_ctzll(m);
                // clear bit j: s_lshl_b64 + s_andn2_b64 instead of the 64-bit m - 1 (s_add, s_addc) + s_and
                // (render_fwd -1.5 % alone, profiles/r06_fwd_bitclr_ab.txt)
                m &= ~(1ull << j);
                const float4 a = s_u.st.rec[0][j], b = s_u.st.rec[1][j], c = s_u.st.rec[2][j];
                Blend e = blend_eval<CL>(a, b, pfx, pfy);
                bool ok = e.p2 <= 0.0f && e.alpha >= thr;  // blend_ok(e) for a live pixel
                if constexpr (EXACT) {
                    // (one compare per evaluation; the re-evaluation is rare: ~6 % of the C3 tiles have one)
                    const bool nr = ok && e.alpha < kNearHi;
                    if (nr) {  // (an exec-masked region, skipped when no lane has one)
                        const int idx = base + j;
                        const uint32_t g = sorted_here ? (uint32_t)s_key[sort_slot(idx)] : point_list[rg.x + idx];
                        const ExactBlend x = exact_blend(a.x, a.y, rec[(size_t)kRecF4 * g + 3], b.y, pfx, pfy);
                        e.p2 = x.power; e.G = x.G; e.alpha = x.alpha;
                        ok = x.power <= 0.0f && x.alpha >= 1.0f / 255.0f;
                        // the backward's walk of this tile looks the re-evaluated weight up (near_rec)
                        const uint32_t slot = atomicAdd(&s_near, 1u);
                        if (slot < kNearCap)
                            near_rec[(size_t)kNearCap * tile + slot] =
                                make_float4(__uint_as_float(((uint32_t)idx << 8) | pix_key), x.power, x.G, x.alpha);
                    }
                }
                take(e, ok, b, c, j);
            }
        };
#ifdef GSR_TRACE
        const uint64_t tr_w0 = __builtin_amdgcn_s_memrealtime();
        tr_batches += 1;
        tr_entries += (uint64_t)__builtin_popcountll(m);
#endif
        if (clamp) walk(std::true_type{});
        else walk(std::false_type{});
#ifdef GSR_TRACE
        tr_walk += __builtin_amdgcn_s_memrealtime() - tr_w0;
#endif
        if (((live >> wv) & 1u) && !__ballot(thr < kThrDone) && lane == 0) atomicAnd(&s_live, ~(1u << wv));
    }
    // EXACT: a pixel whose final T lies within the drift window of 1e-4 (gsr_common.h t_window) is redone by
    // k_render_tsat with the reference's transmittance test; its record carries what that needs
    // (pixel, list start and length, fast n_contrib, fast colour + depth), so the re-walk starts with one load
    if (EXACT && inside && Tt < kTSat * (1.0f + t_window(last))) {
        const uint32_t slot = atomicAdd(tsat_n, 1u);
        if (slot < tsat_cap) {
            uint4 *r = reinterpret_cast<uint4 *>(tsat_list) + 2 * (size_t)slot;
            r[0] = make_uint4((uint32_t)(py * W + px), rg.x, (uint32_t)n, last);
            r[1] = make_uint4(__float_as_uint(C01.x), __float_as_uint(C01.y), __float_as_uint(C2D.x), __float_as_uint(C2D.y));
        }
    }
    if (inside) {
        const int pid = py * W + px;
        pix_end[pid] = make_float4(C01.x, C01.y, C2D.x, Tt);
        n_contrib[pid] = last;
        out_color[pid] = C01.x + Tt * bg[0];
        out_color[H * W + pid] = C01.y + Tt * bg[1];
        out_color[2 * H * W + pid] = C2D.x + Tt * bg[2];
        out_depth[pid] = C2D.y;
    }
    // per 16x4 strip maximum of n_contrib (the backward's quarters): rows 4k..4k+3 = half of the lanes of
    // two waves; lanes (lane >> 3) < 4 hold strip 2 (wv >> 1), the others strip 2 (wv >> 1) + 1
    uint32_t mx = last;
#pragma unroll
    for (int d = 16; d > 0; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));  // within 32 lanes
    __syncthreads();  // every wave is past its last read of s_u
    if (threadIdx.x < 4) s_u.st.q[threadIdx.x] = 0;
    __syncthreads();
    if ((lane & 31) == 0) atomicMax(&s_u.st.q[2 * (wv >> 1) + (lane >> 5)], mx);
    lds_barrier();  // the quarter maxima: no-return LDS atomics
    if (threadIdx.x < 4) tile_maxc[4 * tile + threadIdx.x] = s_u.st.q[threadIdx.x];
    // near records of the tile (count; > kNearCap: the backward re-evaluates the tile itself)
    if (threadIdx.x == 0) tile_flag[tile] = EXACT ? s_near : 0u;
#ifdef GSR_TRACE
    trace_wave(g_trace_fwd, 4 * blockIdx.x + wv, t_start, trace_fwd_work(tr_batches, tr_walk, tr_entries));
    if (g_trace_fwd && lane == 0)  // ticks to the sort's end, above the HW_ID / XCC_ID word's 40 bits
        g_trace_fwd[4 * (4 * blockIdx.x + wv) + 2] |= (tr_sorted - t_start) << 40;
#endif
}

// The exact saturation re-walk of the pixels k_render_fwd flagged: one kTSatThreads-thread block per pixel, all in
// parallel (a fixed grid looping over the device-side count), the walk of tsat_chain / tsat_store above.
// Each pixel's record (written by k_render_fwd) holds its position, list and fast state, so a block starts
// with one load.  (A version that re-walked inside k_render_fwd's blocks, after their blend, was slower:
// the tiles with the most flagged pixels are the long ones at the head of the LPT order)
#ifndef GSR_TSAT_BLOCKS
#define GSR_TSAT_BLOCKS 4096
#endif
constexpr int kTSatBlocks = GSR_TSAT_BLOCKS;
__global__ __launch_bounds__(kTSatThreads) void k_render_tsat(
    int W, int H, const uint32_t *__restrict__ point_list, const float4 *__restrict__ rec,
    const float *__restrict__ bg, float *__restrict__ out_color, float *__restrict__ out_depth,
    float4 *__restrict__ pix_end, uint32_t *__restrict__ n_contrib, const uint32_t *__restrict__ seg_off,
    float4 *__restrict__ seg_state, const uint32_t *__restrict__ tsat_n, const uint32_t *__restrict__ tsat_list,
    uint32_t tsat_cap, const uint32_t *__restrict__ spec_ok, int ks, int gx) {
    constexpr int NT = kTSatThreads;
    __shared__ float4 s_buf[(3 * NT + 4 + 3) / 4];  // the round's contributors: 1 - alpha (+ padding), alpha, position
    __shared__ uint32_t s_rc[4];   // contributors per wave
    if (spec_ok && *spec_ok == 0u) return;  // speculative launch whose capacity failed: redone by the host
    const uint32_t cnt = min(*tsat_n, tsat_cap);
#ifdef GSR_TRACE
    const uint64_t tr_b = __builtin_amdgcn_s_memrealtime();  // (diagnostic) the block's start
#endif
    float *s_q = reinterpret_cast<float *>(s_buf), *s_a = s_q + NT + 4;
    uint32_t *s_pos = reinterpret_cast<uint32_t *>(s_a + NT);
    for (uint32_t i = blockIdx.x; i < cnt; i += gridDim.x) {
#ifdef GSR_TRACE
        const uint64_t tr_i = __builtin_amdgcn_s_memrealtime();
#endif
        const uint4 *rp = reinterpret_cast<const uint4 *>(tsat_list) + 2 * (size_t)i;
        const uint4 r0 = rp[0], r1 = rp[1];  // (pixel, list start, length, fast n_contrib), fast (C0, C1, C2, depth)
        const uint32_t pid = r0.x, start = r0.y;
        const int n = (int)r0.z, nf = (int)r0.w;
        const int px = (int)(pid % (uint32_t)W), py = (int)(pid / (uint32_t)W);
        const int tile = (py / kTileH) * gx + px / kTileW;
        float T = 1.0f;
        uint32_t nex = 0;
        float4 E = make_float4(0.f, 0.f, 0.f, 0.f);
        tsat_chain(nf, point_list + start, (float)px, (float)py, rec, s_rc, s_q, s_a, s_pos, T, nex, E);
#ifdef GSR_TRACE
        const uint64_t tr_c = __builtin_amdgcn_s_memrealtime();
#endif
        if (threadIdx.x == 0) {  // wave 0 holds the result: broadcast through LDS
            s_rc[0] = nex;
            s_rc[1] = __float_as_uint(T);
            s_q[0] = E.x; s_q[1] = E.y; s_q[2] = E.z; s_q[3] = E.w;
        }
        __syncthreads();
        tsat_store(px, py, W, H, n,
                   make_float4(__uint_as_float(r1.x), __uint_as_float(r1.y), __uint_as_float(r1.z), 0.f),
                   __uint_as_float(r1.w), __uint_as_float(s_rc[1]), s_rc[0],
                   make_float4(s_q[0], s_q[1], s_q[2], s_q[3]), bg, out_color, out_depth, pix_end, n_contrib,
                   seg_off[tile], seg_state, ks, nullptr);
        __syncthreads();  // (the LDS is reused by the next pixel)
#ifdef GSR_TRACE
        // (diagnostic, tools/tsat_trace.py) per pixel after the forward's 4T wave slots: (start, end,
        // fast n_contrib | list length << 32, chain ticks | ticks since the block's start << 32)
        const uint32_t ntile = (uint32_t)gx * (uint32_t)((H + kTileH - 1) / kTileH);
        if (g_trace_fwd && threadIdx.x == 0 && i < 4u * ntile) {
            uint64_t *o = g_trace_fwd + 16 * (size_t)ntile + 4 * (size_t)i;
            o[0] = tr_i;
            o[1] = __builtin_amdgcn_s_memrealtime();
            o[2] = (uint64_t)(uint32_t)nf | ((uint64_t)(uint32_t)n << 32);
            o[3] = (tr_c - tr_i) | ((tr_i - tr_b) << 32);
        }
#endif
    }
}

__global__ void k_zero_f32(float *p, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = 0.f;
}

__global__ void k_mark_visible(int P, const float *__restrict__ means3D,
                               const float *__restrict__ viewmatrix, uint8_t *__restrict__ present) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    float vm[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) vm[k] = viewmatrix[k];
    const float3 pv = xform4x3(make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]), vm);
    present[i] = !(pv.z <= 0.2f);
}

// ==========================================================================================
// host launchers
// ==========================================================================================
template <int MC>
static void preprocess_mc(const FwdArgs &a, hipStream_t s) {
    k_preprocess<MC><<<div_up(a.P, kShBlock), kShBlock, sizeof(float) * kShBlock * (MC ? sh_row_stride(MC) : 0), s>>>(
        a.P, a.D, a.M, a.means3D, a.scales, a.scale_modifier, a.rotations, a.opacities, a.shs,
        a.colors_precomp, a.cov3D_precomp, a.viewmatrix, a.projmatrix, a.campos, a.W, a.H, a.tan_fovx,
        a.tan_fovy, a.focal_x, a.focal_y, a.gx, a.gy, a.radii, a.depth, a.rec, a.rect, a.tiles, a.act, a.cs,
        a.tile_count, a.gx * a.gy, a.clampm);
}

hipError_t launch_preprocess(const FwdArgs &a, hipStream_t s) {
    if (a.P == 0) return hipSuccess;
    const int mc = a.shs ? a.M : 0;
    switch (mc) {
        case 16: preprocess_mc<16>(a, s); break;
        case 9: preprocess_mc<9>(a, s); break;
        case 4: preprocess_mc<4>(a, s); break;
        case 1: preprocess_mc<1>(a, s); break;
        default: preprocess_mc<0>(a, s); break;
    }
    return hipGetLastError();
}

hipError_t launch_bin_count(const FwdArgs &a, hipStream_t s) {
    const BinGrid bg(a.P);
    const int T = a.gx * a.gy;
    if (bg.NB == 0) return hipSuccess;  // (tile_count was zeroed by k_preprocess)
    if (T <= kMaxLdsTiles)
        k_bin_count<true><<<bg.NB, kBinThreads, sizeof(uint32_t) * T, s>>>(a.P, bg.CH, T, a.gx, a.rect, a.tiles, a.tile_count, a.block_sums, a.chunk_off, a.items_ws, a.scan_ws);
    else
        k_bin_count<false><<<bg.NB, kBinThreads, 0, s>>>(a.P, bg.CH, T, a.gx, a.rect, a.tiles, a.tile_count, a.block_sums, nullptr, a.items_ws, nullptr);
    return hipGetLastError();
}

// LDS binning (T <= kMaxLdsTiles): the column scan with the single-pass tile scan; otherwise the
// one-block scan over the globally counted tiles
hipError_t launch_bin_scan(const FwdArgs &a, uint32_t *host_words, hipStream_t s) {
    const BinGrid bg(a.P);
    const int T = a.gx * a.gy;
    if (T <= kMaxLdsTiles && bg.NB > 0)
        k_bin_colscan<<<div_up(T, kColW), kColW * kColG, 0, s>>>(T, bg.NB, a.chunk_off, a.tile_count, a.ranges,
                                                                a.tile_cursor, a.seg_off, a.sort_lists, a.tile_rank,
                                                                a.scan_ws, a.block_sums, a.block_off, a.meta,
                                                                host_words, a.spec_cap, seg_log2(a.P));
    else
        k_bin_scan<<<1, 1024, 0, s>>>(T, bg.NB, a.tile_count, a.ranges, a.tile_cursor,
                                      a.block_sums, a.block_off, a.meta, host_words, a.tile_order_f,
                                      a.sort_lists, a.seg_off, a.spec_cap, seg_log2(a.P));
    return hipGetLastError();
}

hipError_t launch_bin_emit(const FwdArgs &a, int K, hipStream_t s) {
    const BinGrid bg(a.P);
    const int T = a.gx * a.gy;
    if (bg.NB == 0) return hipSuccess;
    if (T <= kMaxLdsTiles)
        k_bin_emit<true><<<bg.NB, kBinThreads, sizeof(uint32_t) * T, s>>>(a.P, bg.CH, T, a.gx, a.rect, a.tiles, a.depth, a.block_off, a.tile_cursor, a.goff, a.pairs, (uint32_t)K, a.chunk_off, a.spec_ok,
                                                                           a.tile_count, a.tile_rank, a.scan_ws + 2 * kScanBlocksMax + kScanCtr, a.tile_order_f);
    else
        k_bin_emit<false><<<bg.NB, kBinThreads, 0, s>>>(a.P, bg.CH, T, a.gx, a.rect, a.tiles, a.depth, a.block_off, a.tile_cursor, a.goff, a.pairs, (uint32_t)K, a.chunk_off, a.spec_ok,
                                                        nullptr, nullptr, nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_tile_sort(const FwdArgs &a, uint32_t n_mid, uint32_t n_vlong, uint32_t max_n, uint4 *tmp,
                            hipStream_t s) {
    // lists of up to kFwdSortCap pairs are sorted inside k_render_fwd; up to kSortCap by one block
    // per tile; longer ones by chunk sorts + merge passes
    const int T = a.gx * a.gy;
    if (a.spec_ok) {  // speculative: the count is on the device; blocks loop over it (none here: n_vlong == 0)
        const int nb = a.spec_sort_blocks ? (int)a.spec_sort_blocks : kSpecSortBlocks;
        k_tile_sort<<<std::min(T, nb), 512, 0, s>>>(a.gx, a.sort_lists, a.ranges, a.pairs, a.point_list,
                                                                 a.slot_emit, 0u, a.spec_ok);
        return hipGetLastError();
    }
    if (n_mid) k_tile_sort<<<n_mid, 512, 0, s>>>(a.gx, a.sort_lists, a.ranges, a.pairs, a.point_list, a.slot_emit,
                                                 n_mid, nullptr);
    if (n_vlong) {
        const dim3 grid((unsigned)div_up((int)max_n, kSortCap), n_vlong);
        k_chunk_sort<<<grid, 512, 0, s>>>(T, a.sort_lists, a.ranges, a.pairs);
        const uint4 *src = a.pairs;
        uint4 *dst = tmp;
        for (uint32_t L = kSortCap; L < max_n; L *= 2) {
            const int final_pass = 2 * (size_t)L >= max_n;
            k_merge_pass<<<grid, 512, 0, s>>>(T, a.sort_lists, a.ranges, L, src, dst, final_pass, a.point_list,
                                              a.slot_emit);
            const uint4 *t = dst;
            dst = const_cast<uint4 *>(src);
            src = t;
        }
    }
    return hipGetLastError();
}

hipError_t launch_render_fwd(const FwdArgs &a, hipStream_t s) {
    const int T = a.gx * a.gy;
    auto k = a.exact ? k_render_fwd<true> : k_render_fwd<false>;
    k<<<T, 256, 0, s>>>(a.W, a.H, a.gx, T, a.tile_order_f, a.ranges, a.pairs,
                        a.point_list, a.slot_emit, a.rec, a.bg, a.out_color, a.out_depth, a.pix_end, a.n_contrib,
                        a.tile_maxc, a.seg_off, a.seg_state, a.spec_ok, seg_log2(a.P), a.gate, a.gate_seq,
                        a.gate_err, a.gate_timeout, a.tile_flag, a.near_rec, a.items_ws + kTSatCtr, a.tsat_list,
                        tsat_capacity(a.W * a.H));
    if (a.exact)  // the flagged pixels' exact re-walk (a fixed grid that loops over the device-side count)
        k_render_tsat<<<kTSatBlocks, kTSatThreads, 0, s>>>(a.W, a.H, a.point_list, a.rec, a.bg, a.out_color, a.out_depth,
                                                 a.pix_end, a.n_contrib, a.seg_off, a.seg_state, a.items_ws + kTSatCtr,
                                                 a.tsat_list, tsat_capacity(a.W * a.H), a.spec_ok, seg_log2(a.P),
                                                 a.gx);
    return hipGetLastError();
}

hipError_t launch_zero(float *p, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_zero_f32<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(p, n);
    return hipGetLastError();
}

hipError_t launch_mark_visible(int P, const float *means3D, const float *viewmatrix, uint8_t *present,
                               hipStream_t s) {
    if (P == 0) return hipSuccess;
    k_mark_visible<<<div_up(P, 256), 256, 0, s>>>(P, means3D, viewmatrix, present);
    return hipGetLastError();
}

}  // namespace gsr

#ifdef GSR_TRACE
extern "C" int gsr_debug_trace_fwd(void *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(gsr::g_trace_fwd), &buf, sizeof(buf)) == hipSuccess ? 0 : 2;
}
extern "C" int gsr_debug_trace_emit(void *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(gsr::g_trace_emit), &buf, sizeof(buf)) == hipSuccess ? 0 : 2;
}
#endif
