// gsr_forward.hip -- forward pass of the MI355X-native Gaussian-splat rasterizer.
//
// Pipeline (one HIP stream, one host sync for the pair count K, as the reference does):
//   k_preprocess   1 thread / Gaussian: cull, Sigma3D, EWA Sigma2D, conic, radius, tile rect, SH->RGB
//   k_bin_count    chunked over Gaussians: LDS tile histogram -> one global add per (chunk, tile)
//   k_bin_scan     1 block: exclusive scan of tile counts -> tile ranges; scan of chunk sums; K
//   k_bin_emit     chunked: re-count in LDS, reserve a (chunk, tile) slab, scatter 64-bit keys
//                  (depth_bits << 32 | gaussian) into their tile's range; exclusive emission offsets
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

namespace gsr {

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
    uint2 *__restrict__ rect_out, uint32_t *__restrict__ tiles_out, int act) {
    extern __shared__ __attribute__((aligned(16))) float s_sh[];
    constexpr int RL = 3 * MC, RS = sh_row_stride(MC);
    const int i0 = blockIdx.x * kShBlock;
    if (MC > 0) {  // coalesced copy of this block's SH rows into LDS
        const int nrow = min(kShBlock, P - i0);
        const float *src = shs + (size_t)i0 * RL;
        for (int e = threadIdx.x; e < nrow * RL; e += kShBlock) {
            const int r = e / RL;
            s_sh[r * RS + (e - r * RL)] = src[e];
        }
        __syncthreads();
    }
    const int i = i0 + threadIdx.x;
    if (i >= P) return;
    // matrices are tiny and uniform: every lane reads the same words (scalar loads)
    float vm[16], pm[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) { vm[k] = viewmatrix[k]; pm[k] = projmatrix[k]; }
    radii[i] = 0;
    tiles_out[i] = 0;
    rect_out[i] = make_uint2(0, 0);
    const float3 p = make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
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
        float3 s = make_float3(scales[3 * i], scales[3 * i + 1], scales[3 * i + 2]);
        float4 q = make_float4(rotations[4 * i], rotations[4 * i + 1], rotations[4 * i + 2],
                               rotations[4 * i + 3]);
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
        if (MC > 0) rgb = sh_to_rgb(D, p, campos, s_sh + threadIdx.x * RS, cl);
        else rgb = sh_to_rgb(D, p, campos, shs + (size_t)i * M * 3, cl);
    }
    radii[i] = (int)my_radius;
    depth_out[i] = pv.z;
    const float o = (act & GSR_ACT_SIGMOID_OPACITY) ? act_sigmoid(opacities[i]) : opacities[i];
    const float ca = cv.z * det_inv, cb = -cv.y * det_inv, cc = cv.x * det_inv;
    const float tau2 = o >= 1.0f / 255.0f ? 2.f * log2f(255.f * o) : -1.f;
    float4 *r = rec_out + (size_t)kRecF4 * i;
    r[0] = make_float4(pix_x, pix_y, -0.5f * GSR_LOG2E * ca, -GSR_LOG2E * cb);
    r[1] = make_float4(-0.5f * GSR_LOG2E * cc, o, pv.z, tau2);
    r[2] = make_float4(rgb.x, rgb.y, rgb.z, 0.f);
    r[3] = make_float4(ca, cb, cc, 0.f);
    rect_out[i] = pack_rect(x0, y0, x1, y1);
    tiles_out[i] = (uint32_t)((y1 - y0) * (x1 - x0));
}

// ------------------------------------------------------------------------------------------
// Tile histogram per chunk of Gaussians.  USE_LDS: histogram in LDS (T <= kMaxLdsTiles), then one
// global atomic per non-empty (chunk, tile) bin -- lanes of a wave add to 64 consecutive counters.
template <bool USE_LDS>
__global__ __launch_bounds__(256) void k_bin_count(int P, int CH, int T, int gx,
                                                   const uint2 *__restrict__ rects,
                                                   const uint32_t *__restrict__ tiles,
                                                   uint32_t *__restrict__ tile_count,
                                                   uint32_t *__restrict__ block_sums) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_hist[];
    __shared__ uint32_t s_red[16];
    const int b = blockIdx.x;
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
        for (int t = threadIdx.x; t < T; t += blockDim.x) {
            const uint32_t c = s_hist[t];
            if (c) atomicAdd(&tile_count[t], c);
        }
    }
}

// ------------------------------------------------------------------------------------------
// Single block (1024 threads): exclusive scan of the T tile counts -> ranges/cursors, and of the
// NB chunk sums -> chunk emission offsets.  meta[0] = K.
__global__ __launch_bounds__(1024) void k_bin_scan(int T, int NB, const uint32_t *__restrict__ tile_count,
                                                   uint2 *__restrict__ ranges,
                                                   uint32_t *__restrict__ tile_cursor,
                                                   const uint32_t *__restrict__ block_sums,
                                                   uint32_t *__restrict__ block_off,
                                                   uint32_t *__restrict__ meta,
                                                   uint32_t *host_words,
                                                   uint32_t *__restrict__ tile_order,
                                                   uint32_t *__restrict__ sort_lists) {
    __shared__ uint32_t s_red[16];
    __shared__ uint32_t s_hist[kOrderBuckets];
    __shared__ uint32_t s_cls[3];
    if (threadIdx.x < 3) s_cls[threadIdx.x] = 0;
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
    uint32_t carry2 = 0;
    for (int base = 0; base < NB; base += blockDim.x) {
        const int b = base + threadIdx.x;
        const uint32_t c = b < NB ? block_sums[b] : 0;
        uint32_t tot;
        const uint32_t ex = block_excl_scan_u32(c, s_red, &tot) + carry2;
        if (b < NB) block_off[b] = ex;
        carry2 += tot;
    }
    // tiles per sort path (exact classes, so the host launches exactly the blocks each path needs)
    __syncthreads();
    for (int t = threadIdx.x; t < T; t += blockDim.x) {
        const uint32_t n = tile_count[t];
        if (n == 0) continue;
        const int c = n <= (uint32_t)kRegSortShort ? 0 : (n <= (uint32_t)kRegSortMax ? 1 : 2);
        sort_lists[c * T + atomicAdd(&s_cls[c], 1u)] = (uint32_t)t;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        meta[0] = carry;
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
__global__ __launch_bounds__(256) void k_bin_emit(int P, int CH, int T, int gx,
                                                  const uint2 *__restrict__ rects,
                                                  const uint32_t *__restrict__ tiles,
                                                  const float *__restrict__ depth,
                                                  const uint32_t *__restrict__ block_off,
                                                  uint32_t *__restrict__ tile_cursor,
                                                  uint32_t *__restrict__ goff,
                                                  uint64_t *__restrict__ keys,
                                                  uint32_t *__restrict__ vals, uint32_t K) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_cur[];
    __shared__ uint32_t s_red[16];
    const int b = blockIdx.x;
    const int g0 = b * CH, g1 = min(P, g0 + CH);
    if (USE_LDS) {
        for (int t = threadIdx.x; t < T; t += blockDim.x) s_cur[t] = 0;
        __syncthreads();
        for (int g = g0 + threadIdx.x; g < g1; g += blockDim.x) {
            if (tiles[g] == 0) continue;
            const uint2 r = rects[g];
            const int x0 = r.x & 0xFFFF, y0 = r.x >> 16, x1 = r.y & 0xFFFF, y1 = r.y >> 16;
            for (int y = y0; y < y1; ++y)
                for (int x = x0; x < x1; ++x) atomicAdd(&s_cur[y * gx + x], 1u);
        }
        __syncthreads();
        for (int t = threadIdx.x; t < T; t += blockDim.x) {
            const uint32_t c = s_cur[t];
            s_cur[t] = c ? atomicAdd(&tile_cursor[t], c) : 0u;
        }
        __syncthreads();
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
                const uint64_t key_lo = (uint64_t)(uint32_t)g;
                const uint64_t key = ((uint64_t)__float_as_uint(depth[g]) << 32) | key_lo;
                uint32_t e = ex;  // emission index: y-major over the rect, as the reference emits
                for (int y = y0; y < y1; ++y)
                    for (int x = x0; x < x1; ++x, ++e) {
                        const int t = y * gx + x;
                        const uint32_t pos = USE_LDS ? atomicAdd(&s_cur[t], 1u) : atomicAdd(&tile_cursor[t], 1u);
                        keys[pos] = key;
                        vals[pos] = e;
                    }
            }
        }
    }
    if (b == gridDim.x - 1 && threadIdx.x == 0) goff[P] = K;
}

// ------------------------------------------------------------------------------------------
// Per-tile sort of (depth_bits << 32 | index) keys, then outputs.
__device__ inline void tile_sort_write(uint64_t key, uint32_t slot, int tx, int ty,
                                       const uint2 *__restrict__ rects,
                                       const uint32_t *__restrict__ goff,
                                       uint32_t *__restrict__ point_list, uint32_t *__restrict__ slot_emit) {
    const uint32_t g = (uint32_t)key;
    point_list[slot] = g;
    const uint2 r = rects[g];
    const int x0 = r.x & 0xFFFF, y0 = r.x >> 16, x1 = r.y & 0xFFFF;
    slot_emit[slot] = goff[g] + (uint32_t)((ty - y0) * (x1 - x0) + (tx - x0));  // y-major emission order
}

// ---- wave-level register bitonic sort (gfx950 cross-lane ops) ------------------------------
// Element i = lane * R + r lives in register r of `lane`: exchanges at distance < R stay inside a
// lane, larger distances are lane xors d = dist / R done with DPP (d = 1, 2), ds_swizzle
// (d = 4, 8, 16) or v_permlane32_swap (d = 32).
template <int D>
__device__ inline uint32_t lane_xor(uint32_t x) {
    if constexpr (D == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
    else if constexpr (D == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
    else if constexpr (D == 4 || D == 8 || D == 16) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x1F | (D << 10));
    else {
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

template <int R>
__device__ inline void wave_bitonic_kv(uint64_t (&k)[R], uint32_t (&v)[R], int lane) {
#pragma clang loop unroll(full)
    for (int kk = 2; kk <= 64 * R; kk <<= 1) {
#pragma clang loop unroll(full)
        for (int j = kk >> 1; j > 0; j >>= 1) {
            if (j < R) {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    if (r & j) continue;
                    const int r2 = r | j;
                    const bool asc = ((lane * R + r) & kk) == 0;
                    if ((k[r] > k[r2]) == asc) {
                        const uint64_t t = k[r]; k[r] = k[r2]; k[r2] = t;
                        const uint32_t u = v[r]; v[r] = v[r2]; v[r2] = u;
                    }
                }
            } else {
                const int d = j / R;
                const bool asc = ((lane * R) & kk) == 0;
                const bool lower = (lane & d) == 0;
                const bool take_min = lower == asc;
                switch (d) {
                    case 1: bitonic_xlane<R, 1>(k, v, take_min); break;
                    case 2: bitonic_xlane<R, 2>(k, v, take_min); break;
                    case 4: bitonic_xlane<R, 4>(k, v, take_min); break;
                    case 8: bitonic_xlane<R, 8>(k, v, take_min); break;
                    case 16: bitonic_xlane<R, 16>(k, v, take_min); break;
                    default: bitonic_xlane<R, 32>(k, v, take_min); break;
                }
            }
        }
    }
}

template <int R>
__device__ inline void tile_sort_regs(int n, uint32_t start, const uint64_t *__restrict__ keys,
                                      const uint32_t *__restrict__ vals, uint32_t *__restrict__ point_list,
                                      uint32_t *__restrict__ slot_emit, int lane) {
    uint64_t k[R];
    uint32_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = lane * R + r;
        k[r] = i < n ? keys[start + i] : ~0ull;  // +inf padding sorts to the end
        v[r] = i < n ? vals[start + i] : 0u;
    }
    wave_bitonic_kv<R>(k, v, lane);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int i = lane * R + r;
        if (i < n) {
            point_list[start + i] = (uint32_t)k[r];
            slot_emit[start + i] = v[r];
        }
    }
}

// One wave per tile (4 tiles per block, no barriers), lists sorted entirely in registers.
// LONG = false: tiles of 1..512 pairs (R <= 8); LONG = true: 513..1024 pairs (R = 16, more VGPRs,
// separate launch so the short-list kernel keeps its occupancy).  Longer lists: k_tile_sort.
// `tiles` holds exactly the tiles of this path (built by k_bin_scan).
template <bool LONG>
__global__ __launch_bounds__(256) void k_tile_sort_wave(int count, const uint32_t *__restrict__ tiles,
                                                        const uint2 *__restrict__ ranges,
                                                        const uint64_t *__restrict__ keys,
                                                        const uint32_t *__restrict__ vals,
                                                        uint32_t *__restrict__ point_list,
                                                        uint32_t *__restrict__ slot_emit) {
    const int w = blockIdx.x * kTilesPerBlock + (threadIdx.x >> 6);
    if (w >= count) return;
    const int lane = threadIdx.x & 63;
    const uint2 rg = ranges[tiles[w]];
    const int n = (int)(rg.y - rg.x);
    if (LONG) {
        tile_sort_regs<16>(n, rg.x, keys, vals, point_list, slot_emit, lane);
        return;
    }
    if (n <= 64) tile_sort_regs<1>(n, rg.x, keys, vals, point_list, slot_emit, lane);
    else if (n <= 128) tile_sort_regs<2>(n, rg.x, keys, vals, point_list, slot_emit, lane);
    else if (n <= 256) tile_sort_regs<4>(n, rg.x, keys, vals, point_list, slot_emit, lane);
    else tile_sort_regs<8>(n, rg.x, keys, vals, point_list, slot_emit, lane);
}

__global__ __launch_bounds__(256) void k_tile_sort(int gx, const uint32_t *__restrict__ tiles,
                                                   const uint2 *__restrict__ ranges,
                                                   uint64_t *__restrict__ keys,
                                                   const uint2 *__restrict__ rects,
                                                   const uint32_t *__restrict__ goff,
                                                   uint32_t *__restrict__ point_list,
                                                   uint32_t *__restrict__ slot_emit) {
    extern __shared__ __attribute__((aligned(16))) uint64_t s_keys[];
    const int tile = (int)tiles[blockIdx.x];
    const uint2 rg = ranges[tile];
    const int n = (int)(rg.y - rg.x);
    const int tx = tile % gx, ty = tile / gx;
    const int tid = threadIdx.x, nt = blockDim.x;
    if (n <= kSortCap) {
        int np = 1;
        while (np < n) np <<= 1;
        for (int i = tid; i < np; i += nt) s_keys[i] = i < n ? keys[rg.x + i] : ~0ull;
        __syncthreads();
        for (int k = 2; k <= np; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = tid; i < (np >> 1); i += nt) {
                    const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1)), hi = lo + j;
                    const bool asc = (lo & k) == 0;
                    const uint64_t a = s_keys[lo], c = s_keys[hi];
                    if ((a > c) == asc) { s_keys[lo] = c; s_keys[hi] = a; }
                }
                __syncthreads();
            }
        for (int i = tid; i < n; i += nt) tile_sort_write(s_keys[i], rg.x + i, tx, ty, rects, goff, point_list, slot_emit);
    } else {
        // long tile: in-place bitonic network in global memory with virtual +inf padding
        // ("flip" form: every comparator puts the minimum at the lower index).
        uint64_t *a = keys + rg.x;
        int np = 1;
        while (np < n) np <<= 1;
        for (int k = 2; k <= np; k <<= 1) {
            const int h = k >> 1;
            for (int i = tid; i < (np >> 1); i += nt) {
                const int lo = ((i & ~(h - 1)) << 1) | (i & (h - 1)), hi = lo ^ (k - 1);
                if (hi < n) {
                    const uint64_t x = a[lo], y = a[hi];
                    if (x > y) { a[lo] = y; a[hi] = x; }
                }
            }
            __syncthreads();
            for (int j = k >> 2; j > 0; j >>= 1) {
                for (int i = tid; i < (np >> 1); i += nt) {
                    const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1)), hi = lo + j;
                    if (hi < n) {
                        const uint64_t x = a[lo], y = a[hi];
                        if (x > y) { a[lo] = y; a[hi] = x; }
                    }
                }
                __syncthreads();
            }
        }
        for (int i = tid; i < n; i += nt) tile_sort_write(a[i], rg.x + i, tx, ty, rects, goff, point_list, slot_emit);
    }
}

// ------------------------------------------------------------------------------------------
// Front-to-back blend.  One 256-thread block per 16x16 tile; wave w owns pixel rows 4w..4w+3 (one
// pixel per lane) and walks the tile's list on its own: wave-private LDS staging, no block
// barriers, early exit per 64 pixels.  Tiles are dispatched longest list first (tile_order).
// Gaussians are staged one per lane in batches of 64 (one gather of the 64-byte render record) and
// a conservative ellipse test against the wave's 16x4 pixel rectangle drops pairs that cannot reach
// alpha >= 1/255 there; the per-pixel update is branch-free (selects + FMAs).
__global__ __launch_bounds__(256) void k_render_fwd(
    int W, int H, int gx, int T, const uint32_t *__restrict__ tile_order, const uint2 *__restrict__ ranges,
    const uint32_t *__restrict__ point_list, const float4 *__restrict__ rec, const float *__restrict__ bg,
    float *__restrict__ out_color, float *__restrict__ out_depth, float *__restrict__ final_T,
    uint32_t *__restrict__ n_contrib, uint32_t *__restrict__ tile_maxc, uint32_t *__restrict__ tile_cost) {
    __shared__ float4 s_rec[kTilesPerBlock][3][64];
    const int wv = threadIdx.x >> 6;
    float4(&s_a)[64] = s_rec[wv][0];
    float4(&s_b)[64] = s_rec[wv][1];
    float4(&s_c)[64] = s_rec[wv][2];
    const int tile = (int)tile_order[blockIdx.x];
    const int tx = tile % gx, ty = tile / gx;
    const int lane = threadIdx.x & 63;
    const int px = tx * kTileW + (lane & 15);
    const int py = ty * kTileH + 4 * wv + (lane >> 4);
    const float pfx = (float)px, pfy = (float)py;
    const float rx0 = (float)(tx * kTileW), ry0 = (float)(ty * kTileH + 4 * wv);
    const float rx1 = rx0 + (kTileW - 1), ry1 = ry0 + 3;
    const uint2 rg = ranges[tile];
    const int n = (int)(rg.y - rg.x);
    const bool inside = px < W && py < H;
    bool done = !inside;
    float Tt = 1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f, Dp = 0.f;
    uint32_t last = 0;
    for (int base = 0; base < n; base += 64) {
        if (!__ballot(!done)) break;
        const int idx = base + lane;
        bool live = false;
        if (idx < n) {
            const uint32_t g = point_list[rg.x + idx];
            const float4 a = rec[(size_t)kRecF4 * g], b = rec[(size_t)kRecF4 * g + 1], c = rec[(size_t)kRecF4 * g + 2];
            s_a[lane] = a; s_b[lane] = b; s_c[lane] = c;
            live = !tile_cull(a.x, a.y, -2.f * a.z, -a.w, -2.f * b.x, b.y, b.w, rx0, ry0, rx1, ry1);
        }
        uint64_t m = __ballot(live);
        wave_lds_sync();
        while (m) {
            if (!__ballot(!done)) break;
            const int j = __builtin_ctzll(m);
            m &= m - 1;
            const float4 a = s_a[j], b = s_b[j], c = s_c[j];
            const Blend e = blend_eval(a, b, pfx, pfy);
            const bool ok = !done && blend_ok(e);
            const float test_T = Tt * (1.f - e.alpha);
            const bool fin = ok && test_T < 0.0001f;
            const bool use = ok && !fin;
            done = done || fin;
            const float w = use ? e.alpha * Tt : 0.f;
            C0 = fmaf(c.x, w, C0);
            C1 = fmaf(c.y, w, C1);
            C2 = fmaf(c.z, w, C2);
            Dp = fmaf(b.z, w, Dp);
            Tt = use ? test_T : Tt;
            last = use ? (uint32_t)(base + j + 1) : last;
        }
        wave_lds_sync();
    }
    if (inside) {
        const int pid = py * W + px;
        final_T[pid] = Tt;
        n_contrib[pid] = last;
        out_color[pid] = C0 + Tt * bg[0];
        out_color[H * W + pid] = C1 + Tt * bg[1];
        out_color[2 * H * W + pid] = C2 + Tt * bg[2];
        out_depth[pid] = Dp;
    }
    uint32_t mx = last, sum = last;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
        sum += (uint32_t)__shfl_xor((int)sum, d, 64);
    }
    if (lane == 0) { tile_maxc[4 * tile + wv] = mx; tile_cost[4 * tile + wv] = sum; }
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
        a.tan_fovy, a.focal_x, a.focal_y, a.gx, a.gy, a.radii, a.depth, a.rec, a.rect, a.tiles, a.act);
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
    hipError_t e = hipMemsetAsync(a.tile_count, 0, sizeof(uint32_t) * T, s);
    if (e != hipSuccess) return e;
    if (bg.NB == 0) return hipSuccess;
    if (T <= kMaxLdsTiles)
        k_bin_count<true><<<bg.NB, 256, sizeof(uint32_t) * T, s>>>(a.P, bg.CH, T, a.gx, a.rect, a.tiles, a.tile_count, a.block_sums);
    else
        k_bin_count<false><<<bg.NB, 256, 0, s>>>(a.P, bg.CH, T, a.gx, a.rect, a.tiles, a.tile_count, a.block_sums);
    return hipGetLastError();
}

hipError_t launch_bin_scan(const FwdArgs &a, uint32_t *host_words, hipStream_t s) {
    const BinGrid bg(a.P);
    k_bin_scan<<<1, 1024, 0, s>>>(a.gx * a.gy, bg.NB, a.tile_count, a.ranges, a.tile_cursor,
                                  a.block_sums, a.block_off, a.meta, host_words, a.tile_order_f,
                                  a.sort_lists);
    return hipGetLastError();
}

hipError_t launch_bin_emit(const FwdArgs &a, int K, hipStream_t s) {
    const BinGrid bg(a.P);
    const int T = a.gx * a.gy;
    if (bg.NB == 0) return hipSuccess;
    if (T <= kMaxLdsTiles)
        k_bin_emit<true><<<bg.NB, 256, sizeof(uint32_t) * T, s>>>(a.P, bg.CH, T, a.gx, a.rect, a.tiles, a.depth, a.block_off, a.tile_cursor, a.goff, a.keys, a.vals, (uint32_t)K);
    else
        k_bin_emit<false><<<bg.NB, 256, 0, s>>>(a.P, bg.CH, T, a.gx, a.rect, a.tiles, a.depth, a.block_off, a.tile_cursor, a.goff, a.keys, a.vals, (uint32_t)K);
    return hipGetLastError();
}

hipError_t launch_tile_sort(const FwdArgs &a, const uint32_t *n_per_path, hipStream_t s) {
    const int T = a.gx * a.gy;
    const uint32_t *lists = a.sort_lists;
    if (n_per_path[0])
        k_tile_sort_wave<false><<<div_up((int)n_per_path[0], kTilesPerBlock), 256, 0, s>>>(
            (int)n_per_path[0], lists, a.ranges, a.keys, a.vals, a.point_list, a.slot_emit);
    if (n_per_path[1])
        k_tile_sort_wave<true><<<div_up((int)n_per_path[1], kTilesPerBlock), 256, 0, s>>>(
            (int)n_per_path[1], lists + T, a.ranges, a.keys, a.vals, a.point_list, a.slot_emit);
    if (n_per_path[2])
        k_tile_sort<<<n_per_path[2], 256, sizeof(uint64_t) * kSortCap, s>>>(
            a.gx, lists + 2 * T, a.ranges, a.keys, a.rect, a.goff, a.point_list, a.slot_emit);
    return hipGetLastError();
}

hipError_t launch_render_fwd(const FwdArgs &a, hipStream_t s) {
    const int T = a.gx * a.gy;
    k_render_fwd<<<T, 256, 0, s>>>(a.W, a.H, a.gx, T, a.tile_order_f, a.ranges, a.point_list, a.rec,
                                   a.bg, a.out_color, a.out_depth, a.final_T, a.n_contrib,
                                   a.tile_maxc, a.tile_cost);
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
