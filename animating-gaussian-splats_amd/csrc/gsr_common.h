// gsr_common.h -- shared device math, constants and HBM workspace layouts of libgsr.
//
// The float expressions below are evaluated in exactly the order the CPU oracle
// (oracle/gsr_oracle.c) evaluates them, and the library is compiled with -ffp-contract=off, so
// every float that feeds an integer decision (radius, tile rectangle, sort key) is bit-identical to
// the oracle.  Behavioural spec: SURVEY.md section 2.1 (upstream diff-gaussian-rasterization-w-depth,
// absent from /root/reference: .gitmodules:1-3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gsr.h"  // gsr_activation bits

namespace gsr {

constexpr int kTileW = 16;  // 16x16 pixel tiles (upstream BLOCK_X/BLOCK_Y)
constexpr int kTileH = 16;
constexpr int kTilePix = kTileW * kTileH;  // 256 = 4 wave64 per tile block
constexpr int kPartial = 9;  // per (tile, Gaussian) backward partial: dmean2D xy, dconic abc, dopacity, dcolour rgb
constexpr int kRecF = kPartial;  // floats per stored partial-gradient record (36 bytes, packed)
constexpr int kSortCap = 4096;  // per-tile list length sorted entirely in LDS (32 KiB of u64 keys)
__host__ __device__ inline uint64_t pair_key(uint4 r) { return ((uint64_t)r.y << 32) | r.x; }
#ifndef GSR_FWD_SORT_CAP
#define GSR_FWD_SORT_CAP 1024
#endif
constexpr int kFwdSortCap = GSR_FWD_SORT_CAP;  // lists up to this length are depth-sorted inside k_render_fwd
// host-mapped words published by k_bin_scan: [0] = K (written last, release), [1] = number of
// tiles with kFwdSortCap < n <= kSortCap pairs (k_tile_sort), [2] = number of longer tiles (chunk
// sort + merge passes), [3] = the longest list
constexpr int kHostWords = 4;

__host__ __device__ inline int div_up(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// ---------------------------------------------------------------------------------------------
// Workspace layouts.  One allocation per kind; every array starts 256-byte aligned.
// ---------------------------------------------------------------------------------------------
// GEOM (per Gaussian, P): written by preprocess, read by binning/render/backward.
//   rec: one 64-byte render record per Gaussian, so a (tile, Gaussian) gather touches one line:
//        [0] = (x, y, A2, B2)        [1] = (C2, opacity, depth, tau2)
//        [2] = (r, g, b, depth)      [3] = (conic_a, conic_b, conic_c, 0)
//        power * log2(e) = A2 dx^2 + B2 dx dy + C2 dy^2, i.e. (A2, B2, C2) = -log2(e) (a/2, b, c/2),
//        so the blend weight is one v_exp_f32; tau2 = 2 log2(255 opacity) bounds the alpha >= 1/255
//        footprint (culling); [3] keeps the exact conic for gradients and introspection.
//   depth/rect/tiles/goff: SoA arrays for the binning kernels.
constexpr int kRecF4 = 4;  // float4 per render record (64 B)
struct GeomLayout {
    size_t depth, rec, rect, tiles, goff, clampm, total;
    __host__ __device__ GeomLayout(int P) {
        size_t o = 0;
        depth = o;    o = align256(o + sizeof(float) * P);
        rec = o;      o = align256(o + sizeof(float4) * kRecF4 * (size_t)P);
        rect = o;     o = align256(o + sizeof(uint2) * P);
        tiles = o;    o = align256(o + sizeof(uint32_t) * P);
        goff = o;     o = align256(o + sizeof(uint32_t) * (P + 1));
        clampm = o;   o = align256(o + (size_t)P);  // SH clamp mask per Gaussian (clamp_bits)
        total = o;
    }
};

// Binning work decomposition over Gaussians: NB chunks of CH Gaussians (CH multiple of 256).
constexpr int kBinThreads = 1024;  // threads per binning block (one chunk of CH Gaussians; 256 / 512 measured)
// Tile histogram kept in LDS when T * 4 B fits in 64 KiB; larger tile grids (e.g. 4K frames)
// count straight into global memory.
constexpr int kMaxLdsTiles = 16384;
struct BinGrid {
    int CH, NB;
    __host__ __device__ BinGrid(int P) {
        int c = div_up(P, 512);  // ~512 chunks (2 per CU)
        c = div_up(c, 256) * 256;
        CH = c < 1024 ? 1024 : c;
        NB = P > 0 ? div_up(P, CH) : 0;
    }
};

// Backward segments: the backward blend walks each tile's list in independent work items of up to
// kSeg list entries (SURVEY.md 2.1 renderCUDA bwd restated as (tile, segment) items, so a long list
// spreads over several waves and no item costs more than 4 kSeg (pair, quarter) steps -- a
// longest-first dispatch then balances the launch).  The forward saves every pixel's blend state
// (front colour, transmittance) before entry kSeg, 2 kSeg, ... of its tile: the state a segment's
// reverse walk starts from.  A power of two >= the forward's 64-entry batch (k_render_fwd tests
// boundaries with a mask).  256: measured against 128 / 512 / 1024 (tools/ab_variants.sh).
constexpr int kSeg = 256;  // the longest segment
static_assert(kSeg >= 64 && (kSeg & (kSeg - 1)) == 0, "kSeg: a power of two, >= the forward's 64-entry batch");
constexpr int kSegLog2Max = __builtin_ctz(kSeg), kSegLog2Min = 6;
// The segment length of a cloud of P Gaussians, log2 (fixed before the pair count is known: the
// forward's tile scan lays out the boundary states with it).  Small clouds have short lists and few
// items per launch: the longest item then sets the backward's time (C2, 100k Gaussians at 800x800:
// render_bwd 114 us at 256-entry segments, 75 us at 64), so the segment shrinks until ~4 P >> ks
// (about the pair count) gives >= 8192 items; 1M-Gaussian clouds keep kSeg.
__host__ __device__ inline int seg_log2(int P) {
    int ks = kSegLog2Max;
    while (ks > kSegLog2Min && ((4 * (size_t)(P > 0 ? P : 0)) >> ks) < 8192) --ks;
    return ks;
}
__host__ __device__ inline uint32_t seg_bounds(uint32_t n, int ks) { return n > 0 ? (n - 1) >> ks : 0; }

// The backward's work items of a tile with n list entries and per-quarter max n_contrib mq: one per
// segment (2^ks entries) below the largest quarter maximum (at least one per non-empty tile, which
// also writes the zero records of the entries nobody reached); cost = its (pair, quarter) steps.
__host__ __device__ inline uint32_t bwd_item_count(uint32_t n, uint4 mq, int ks) {
    const uint32_t maxc = min(max(max(mq.x, mq.y), max(mq.z, mq.w)), n);
    return n == 0 ? 0u : max(1u, (maxc + (1u << ks) - 1) >> ks);
}
__host__ __device__ inline uint32_t bwd_item_cost(uint32_t j, uint4 mq, int ks) {
    const uint32_t s0 = j << ks, s1 = s0 + (1u << ks);
    const uint32_t a = mq.x > s0 ? min(mq.x, s1) - s0 : 0u, b = mq.y > s0 ? min(mq.y, s1) - s0 : 0u;
    const uint32_t c = mq.z > s0 ? min(mq.z, s1) - s0 : 0u, d = mq.w > s0 ? min(mq.w, s1) - s0 : 0u;
    return a + b + c + d;
}
// Zero-record items: a tile's list entries past every pixel's last contributor (maxc .. n) get zero
// gradient records (k_gauss_bwd sums every emission slot); the tile's last segment item writes the
// first kZeroChunk of them, every further kZeroChunk is an item of its own (seg = kZeroItem | chunk),
// so a long list whose pixels saturated early does not leave one wave storing all of them.
constexpr uint32_t kZeroChunk = 1024;
constexpr uint32_t kZeroItem = 0x80000000u;
__host__ __device__ inline uint32_t bwd_zero_items(uint32_t n, uint4 mq) {
    const uint32_t maxc = min(max(max(mq.x, mq.y), max(mq.z, mq.w)), n);
    return n - maxc > kZeroChunk ? (n - maxc - 1) / kZeroChunk : 0u;
}
// the upper bound of the item count the backward launch covers (for any segment length)
__host__ __device__ inline size_t max_bwd_items(int K, int T) {
    const size_t k = (size_t)(K > 0 ? K : 0);
    return (k >> kSegLog2Min) + k / kZeroChunk + (k < (size_t)T ? k : (size_t)T) + 1;
}

// Cost buckets of the longest-first (LPT) dispatch orders (lpt_order, the backward's item list).
constexpr int kOrderBuckets = 2048;
// The backward item builder's workspace (k_items_count / k_items_emit, IMAGE.items_ws): per-bucket item
// counts [0, kOrderBuckets), the buckets' cursors [kOrderBuckets, 2 kOrderBuckets), the builder's done
// counter [2 kOrderBuckets].  k_bin_count zeroes it in every forward; the count kernel's last block
// leaves the counts and the counter at zero again, so a second build (a repeated backward) starts clean.
constexpr int kItemsWsWords = 2 * kOrderBuckets + 64;
// items_ws word counting the pixels the exact saturation re-walk redoes (zeroed with the workspace by
// k_bin_count; the item kernels use words [0, 2 kOrderBuckets])
constexpr int kTSatCtr = 2 * kOrderBuckets + 8;
// records of the pixels the exact saturation re-walk redoes (32 B each, IMAGE tsat_list): one per 8 pixels
// (measured ~0.1 % of a C3 view's pixels; past the capacity a pixel keeps the fast walk's outputs)
__host__ __device__ constexpr uint32_t tsat_capacity(int npix) { return (uint32_t)(npix / 8 + 64); }

// The single-pass tile scan of k_bin_colscan (IMAGE.scan_ws, zeroed by k_bin_count): one look-back
// word per block of tiles (u64: flag in bits 62-63 -- kScanAgg: the block's own sums, kScanInc: the sums
// of every block up to it -- pair count in bits 0-31, segment-boundary count in bits 32-61), then
// counters (kScanCtr words: [0] block ticket, [1] done blocks, [2] mid lists, [3] long lists, [4] the
// longest list), then the forward dispatch order's bucket counts (-> offsets, kOrderBuckets words).
constexpr uint64_t kScanAgg = 1ull << 62, kScanInc = 2ull << 62;
constexpr int kScanBlocksMax = 512;  // blocks of the LDS-binning column scan (T <= kMaxLdsTiles)
constexpr int kScanCtr = 16;
constexpr int kScanWsWords = 2 * kScanBlocksMax + kScanCtr + kOrderBuckets;
// the forward's LPT dispatch bucket of a tile with c list entries (0 = longest): exact below 1024, then
// 32 buckets per power of two (a fixed map, so the tiles can be bucketed before the longest is known)
__host__ __device__ inline uint32_t lpt_bucket(uint32_t c) {
    uint32_t b = c;
    if (c >= 1024u) {
        const uint32_t e = 31u - (uint32_t)__builtin_clz(c);
        b = 1024u + ((e - 10u) << 5) + ((c >> (e - 5u)) & 31u);
    }
    return (uint32_t)kOrderBuckets - 1u - b;
}

// IMAGE (per pixel / per tile): tile ranges, blend state saved for backward, binning counters.
//   pix_end: per pixel (C0, C1, C2, T) at the end of the blend (accumulated colour without the
//            background, final transmittance);  seg_off: per tile, exclusive prefix of its interior
//            segment boundaries (seg_bounds) -> index of its first saved boundary state.
// near records per tile (IMAGE near_rec): the forward's re-evaluated (pixel, entry) weights, which the
// backward looks up instead of re-evaluating; a tile with more re-evaluates in the backward as well
constexpr uint32_t kNearCap = 16;
struct ImageLayout {
    size_t ranges, pix_end, n_contrib, tile_maxc, tile_order_f, seg_off, sort_lists,
        tile_count, tile_cursor, block_sums, block_off, meta, items_ws, scan_ws, tile_rank, tile_flag, tsat_list,
        near_rec, chunk_off, total;
    __host__ __device__ ImageLayout(int W, int H, int P) {
        const int T = div_up(W, kTileW) * div_up(H, kTileH);
        const int N = W * H;
        const int NB = BinGrid(P).NB;
        size_t o = 0;
        ranges = o;      o = align256(o + sizeof(uint2) * T);
        pix_end = o;     o = align256(o + sizeof(float4) * N);
        n_contrib = o;   o = align256(o + sizeof(uint32_t) * N);
        tile_maxc = o;   o = align256(o + sizeof(uint32_t) * 4 * T);  // per quarter tile (16x4 px)
        tile_order_f = o; o = align256(o + sizeof(uint32_t) * T);    // forward dispatch order (LPT)
        seg_off = o;     o = align256(o + sizeof(uint32_t) * (T + 1));
        sort_lists = o;  o = align256(o + sizeof(uint32_t) * T);      // tiles longer than kFwdSortCap
        tile_count = o;  o = align256(o + sizeof(uint32_t) * T);
        tile_cursor = o; o = align256(o + sizeof(uint32_t) * T);
        block_sums = o;  o = align256(o + sizeof(uint32_t) * (NB + 1));
        block_off = o;   o = align256(o + sizeof(uint32_t) * (NB + 1));
        meta = o;        o = align256(o + sizeof(uint32_t) * 16);
        items_ws = o;    o = align256(o + sizeof(uint32_t) * kItemsWsWords);
        scan_ws = o;     o = align256(o + sizeof(uint32_t) * kScanWsWords);
        tile_rank = o;   o = align256(o + sizeof(uint32_t) * T);           // rank inside its LPT bucket
        tile_flag = o;   o = align256(o + sizeof(uint32_t) * T);           // near-threshold re-evaluations
        tsat_list = o;   o = align256(o + 32 * (size_t)tsat_capacity(N));  // pixels the exact re-walk redoes
        near_rec = o;    o = align256(o + sizeof(float4) * kNearCap * T);  // and their records
        // (chunk, tile) counts, then each chunk's slab offset inside the tile's range (LDS binning)
        chunk_off = o;   o = align256(o + (T <= kMaxLdsTiles ? sizeof(uint32_t) * (size_t)NB * T : 0));
        total = o;
    }
};

// BINNING (per Gaussian-tile pair, K): sort keys + their emission index, sorted Gaussian list,
// emission index of every sorted slot (where the backward stores the slot's gradient record), the
// saved blend state at every interior segment boundary (<= K >> seg_log2(P) boundaries in total;
// each 256 float4 (C0, C1, C2, T), one per pixel of the tile in row-major order).
struct BinningLayout {
    size_t pairs, point_list, slot_emit, seg_state, total;
    __host__ __device__ BinningLayout(int K, int P) {
        size_t o = 0;
        // one 16-byte record per pair: (index, depth bits, emission index, 0) -- the 64-bit sort key
        // (depth_bits << 32 | index) in .x/.y and its payload in .z, so k_bin_emit's scatter is ONE
        // store per pair (the scatter is bound by scattered line requests, not bytes)
        pairs = o;      o = align256(o + sizeof(uint4) * (K > 0 ? K : 1));
        point_list = o; o = align256(o + sizeof(uint32_t) * (K > 0 ? K : 1));
        slot_emit = o;  o = align256(o + sizeof(uint32_t) * (K > 0 ? K : 1));  // sorted slot -> emission
        seg_state = o;  o = align256(o + sizeof(float4) * kTilePix * (size_t)(((size_t)(K > 0 ? K : 0) >> seg_log2(P)) + 1));
        total = o;
    }
};

// The backward's work-item list ([0].x = count, then (tile, segment) in dispatch order): in SCRATCH,
// or -- when the forward prepares the backward (gsr_gaussians.prepare_backward) -- right after the
// BINNING arrays (at BinningLayout(K, P).total), built by the forward.
__host__ __device__ inline size_t bwd_items_bytes(int K, int T) { return align256(sizeof(uint2) * (max_bwd_items(K, T) + 1)); }

// SCRATCH (backward): one packed 36-byte partial-gradient record per Gaussian-tile pair, stored at
// the pair's EMISSION index (Gaussian-major), so each Gaussian's records are contiguous for the
// per-Gaussian reduction: dmean2D.xy, dconic.abc, dopacity, dcolour.rgb; then the backward's work
// items ([0].x = count, then (tile, segment) in dispatch order, built by k_bwd_items).
struct ScratchLayout {
    size_t part, items, total;
    __host__ __device__ ScratchLayout(int K, int T) {
        const size_t k = size_t(K > 0 ? K : 1);
        size_t o = 0;
        // kRecF floats per record, packed; + 16 bytes: the readers' aligned float4 loads may run up
        // to 12 bytes past the last record
        part = o;  o = align256(o + sizeof(float) * kRecF * k + 16);
        items = o; o += bwd_items_bytes(K, T);
        total = o;
    }
};

// SH rows staged through LDS by the per-Gaussian kernels (coalesced global traffic): compile-time
// coefficient counts for the degrees the reference can activate; other counts use direct loads.
// Threads (= Gaussians) per block of the SH-staging kernels (k_preprocess, k_gauss_bwd): 25 KB of
// LDS at SH3, small enough to co-run with other streams' render kernels (256 was 2 % slower).
constexpr int kShBlock = 128;
__host__ __device__ constexpr int sh_row_stride(int MC) { return (3 * MC) | 1; }  // odd: no bank conflicts

// Block copy of `nrow` SH rows (3 MC floats each, contiguous in global memory) into LDS rows of
// stride sh_row_stride(MC).  The block's global span starts 16-byte aligned whenever the array does
// (kShBlock * 3 MC is a multiple of 4), so it is read as float4: every thread issues up to INFL loads
// before its first LDS store (all 12 at once for MC = 16 by default; a caller with live registers
// passes a smaller INFL and the copy runs in rounds).
template <int MC, int INFL = 16>
__device__ inline void sh_rows_to_lds(const float *__restrict__ src, int nrow, float *s) {
    constexpr int RL = 3 * MC, RS = sh_row_stride(MC);
    constexpr int IT = (kShBlock * RL / 4 + kShBlock - 1) / kShBlock;
    constexpr int B = IT < INFL ? IT : INFL;
    const int n = nrow * RL;
    if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
        const int n4 = n >> 2;
        const float4 *s4 = reinterpret_cast<const float4 *>(src);
#pragma unroll
        for (int i0 = 0; i0 < IT; i0 += B) {
            float4 v[B];
#pragma unroll
            for (int it = 0; it < B; ++it) {
                const int q = threadIdx.x + (i0 + it) * kShBlock;
                if (i0 + it < IT && q < n4) v[it] = s4[q];
            }
#pragma unroll
            for (int it = 0; it < B; ++it) {
                const int q = threadIdx.x + (i0 + it) * kShBlock;
                if (i0 + it < IT && q < n4) {
                    const float f[4] = {v[it].x, v[it].y, v[it].z, v[it].w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int e = 4 * q + j, r = e / RL;
                        s[r * RS + (e - r * RL)] = f[j];
                    }
                }
            }
        }
        for (int e = 4 * n4 + (int)threadIdx.x; e < n; e += kShBlock) {
            const int r = e / RL;
            s[r * RS + (e - r * RL)] = src[e];
        }
    } else {
        for (int e = threadIdx.x; e < n; e += kShBlock) {
            const int r = e / RL;
            s[r * RS + (e - r * RL)] = src[e];
        }
    }
}

// The reverse copy (LDS rows -> contiguous global rows), float4 stores when aligned; ACC adds the
// rows to what dst holds (gradient accumulation).
template <int MC, bool ACC = false>
__device__ inline void sh_rows_from_lds(const float *s, int nrow, float *__restrict__ dst) {
    constexpr int RL = 3 * MC, RS = sh_row_stride(MC);
    const int n = nrow * RL;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        const int n4 = n >> 2;
        float4 *d4 = reinterpret_cast<float4 *>(dst);
        constexpr int IT = (kShBlock * RL / 4 + kShBlock - 1) / kShBlock;
        float4 o[IT];  // ACC: every old float4 of this thread loaded before the first store
        if (ACC) {
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int q = threadIdx.x + it * kShBlock;
                o[it] = d4[q < n4 ? q : 0];  // clamped (n4 >= 1 whenever a row exists), unpredicated
            }
        }
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int q = threadIdx.x + it * kShBlock;
            if (q >= n4) break;
            float f[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int e = 4 * q + j, r = e / RL;
                f[j] = s[r * RS + (e - r * RL)];
            }
            float4 v = make_float4(f[0], f[1], f[2], f[3]);
            if (ACC) v = make_float4(o[it].x + v.x, o[it].y + v.y, o[it].z + v.z, o[it].w + v.w);
            d4[q] = v;
        }
        for (int e = 4 * n4 + (int)threadIdx.x; e < n; e += kShBlock) {
            const int r = e / RL;
            const float v = s[r * RS + (e - r * RL)];
            dst[e] = ACC ? dst[e] + v : v;
        }
    } else {
        for (int e = threadIdx.x; e < n; e += kShBlock) {
            const int r = e / RL;
            const float v = s[r * RS + (e - r * RL)];
            dst[e] = ACC ? dst[e] + v : v;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Device math -- same op order as oracle/gsr_oracle.c
// ---------------------------------------------------------------------------------------------
#define GSR_SH_C0 0.28209479177387814f
#define GSR_SH_C1 0.4886025119029199f
__device__ __constant__ const float kSH_C2[5] = {1.0925484305920792f, -1.0925484305920792f,
                                                 0.31539156525252005f, -1.0925484305920792f,
                                                 0.5462742152960396f};
__device__ __constant__ const float kSH_C3[7] = {-0.5900435899266435f, 2.890611442640554f,
                                                 -0.4570457994644658f, 0.3731763325901154f,
                                                 -0.4570457994644658f, 1.445305721320277f,
                                                 -0.5900435899266435f};

// column-major 3x3 (glm storage): m[c*3+r]
struct m3 { float m[9]; };
#define GM(A, c, r) ((A).m[(c) * 3 + (r)])

__device__ inline m3 m3_mul(const m3 &a, const m3 &b) {
    m3 o;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r)
            o.m[c * 3 + r] = a.m[0 * 3 + r] * b.m[c * 3 + 0] + a.m[1 * 3 + r] * b.m[c * 3 + 1] +
                             a.m[2 * 3 + r] * b.m[c * 3 + 2];
    return o;
}
__device__ inline m3 m3_T(const m3 &a) {
    m3 o;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) o.m[c * 3 + r] = a.m[r * 3 + c];
    return o;
}

__device__ inline float ndc2pix(float v, int S) { return (float)(((v + 1.0) * S - 1.0) * 0.5); }

__device__ inline void get_rect(float px, float py, int max_radius, int gx, int gy, int &x0, int &y0,
                                int &x1, int &y1) {
    x0 = min(gx, max(0, (int)((px - max_radius) / kTileW)));
    y0 = min(gy, max(0, (int)((py - max_radius) / kTileH)));
    x1 = min(gx, max(0, (int)((px + max_radius + kTileW - 1) / kTileW)));
    y1 = min(gy, max(0, (int)((py + max_radius + kTileH - 1) / kTileH)));
}

__device__ inline float3 xform4x3(float3 p, const float *m) {
    return make_float3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                       m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
__device__ inline float4 xform4x4(float3 p, const float *m) {
    return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                       m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14],
                       m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}

__device__ inline m3 rot_from_quat(float4 q) {  // q = (w, x, y, z), NOT normalised (reference quirk)
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    m3 R = {{1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
             2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
             2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y)}};
    return R;
}

__device__ inline void cov3d_from_scale_rot(float3 s3, float mod, float4 q, float *cov) {
    m3 S = {{0, 0, 0, 0, 0, 0, 0, 0, 0}};
    GM(S, 0, 0) = mod * s3.x; GM(S, 1, 1) = mod * s3.y; GM(S, 2, 2) = mod * s3.z;
    const m3 R = rot_from_quat(q);
    const m3 M = m3_mul(S, R);
    const m3 Sig = m3_mul(m3_T(M), M);
    cov[0] = GM(Sig, 0, 0); cov[1] = GM(Sig, 0, 1); cov[2] = GM(Sig, 0, 2);
    cov[3] = GM(Sig, 1, 1); cov[4] = GM(Sig, 1, 2); cov[5] = GM(Sig, 2, 2);
}

// ---- fused parameter activations (shared.py:33-41; gsr_activation bits) ----
// torch.nn.functional.normalize(q, dim=-1, eps=1e-12) = q / max(|q|, eps), |q| = sqrt(sum q_k^2)
__device__ inline float quat_norm(float4 q) { return sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w); }
__device__ inline float4 act_normalize(float4 q, float n) {
    const float c = fmaxf(n, 1e-12f);
    return make_float4(q.x / c, q.y / c, q.z / c, q.w / c);
}
// d/dq_raw of q_raw / max(|q_raw|, eps): (g - qhat (qhat . g)) / |q| when |q| > eps, else g / eps
__device__ inline float4 act_normalize_bwd(float4 qhat, float n, float4 g) {
    if (!(n > 1e-12f)) return make_float4(g.x / 1e-12f, g.y / 1e-12f, g.z / 1e-12f, g.w / 1e-12f);
    const float d = qhat.x * g.x + qhat.y * g.y + qhat.z * g.z + qhat.w * g.w;
    return make_float4((g.x - qhat.x * d) / n, (g.y - qhat.y * d) / n, (g.z - qhat.z * d) / n,
                       (g.w - qhat.w * d) / n);
}
__device__ inline float act_sigmoid(float x) { return 1.f / (1.f + expf(-x)); }
__device__ inline float3 act_exp3(float3 s) { return make_float3(expf(s.x), expf(s.y), expf(s.z)); }

__device__ inline float3 cov2d(float3 mean, float fx, float fy, float tfx, float tfy, const float *c3,
                               const float *vm) {
    float3 t = xform4x3(mean, vm);
    const float limx = 1.3f * tfx, limy = 1.3f * tfy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const m3 J = {{fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z,
                   -(fy * t.y) / (t.z * t.z), 0, 0, 0}};
    const m3 Wm = {{vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]}};
    const m3 T = m3_mul(Wm, J);
    const m3 V = {{c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]}};
    const m3 cov = m3_mul(m3_mul(m3_T(T), m3_T(V)), T);
    return make_float3(GM(cov, 0, 0) + 0.3f, GM(cov, 0, 1), GM(cov, 1, 1) + 0.3f);
}

// Element strides of the camera inputs (gsr_camera, ABI 8): matrix element k (column-major m[k] of
// the kernels) sits at (k / 4) * m0 + (k % 4) * m1; campos component c at c * c0.
struct CamStrides { int v0, v1, p0, p1, c0; };
// The camera inputs are read through the constant address space: their addresses are wave-uniform
// and no kernel writes them, so these become scalar loads into SGPRs (as plain global pointers next to
// the kernels' unrestricted output pointers, they were 35 per-lane vector loads into VGPRs per view).
typedef const __attribute__((address_space(4))) float *cam_ptr;
__device__ inline void load_mat16(const float *__restrict__ m, int s0, int s1, float (&out)[16]) {
    const cam_ptr c = (cam_ptr)m;
#pragma unroll
    for (int k = 0; k < 16; ++k) out[k] = c[(k >> 2) * s0 + (k & 3) * s1];
}
__device__ inline float3 load_campos(const float *__restrict__ c, int s) {
    const cam_ptr p = (cam_ptr)c;
    return c ? make_float3(p[0], p[s], p[2 * s]) : make_float3(0.f, 0.f, 0.f);
}

// SH -> RGB for one channel set; `sh` points at the Gaussian's (M,3) coefficients (global or LDS).
template <typename ShPtr>
__device__ inline float3 sh_to_rgb(int deg, float3 mean, float3 campos, ShPtr sh, bool *clamped) {
    float3 dir = make_float3(mean.x - campos.x, mean.y - campos.y, mean.z - campos.z);
    const float len = sqrtf(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z);
    dir.x = dir.x / len; dir.y = dir.y / len; dir.z = dir.z / len;
    float out[3];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
#define S(i) sh[(i) * 3 + ch]
        float res = GSR_SH_C0 * S(0);
        if (deg > 0) {
            const float x = dir.x, y = dir.y, z = dir.z;
            res = res - GSR_SH_C1 * y * S(1) + GSR_SH_C1 * z * S(2) - GSR_SH_C1 * x * S(3);
            if (deg > 1) {
                const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
                res = res + kSH_C2[0] * xy * S(4) + kSH_C2[1] * yz * S(5) +
                      kSH_C2[2] * (2.0f * zz - xx - yy) * S(6) + kSH_C2[3] * xz * S(7) +
                      kSH_C2[4] * (xx - yy) * S(8);
                if (deg > 2) {
                    res = res + kSH_C3[0] * y * (3.0f * xx - yy) * S(9) + kSH_C3[1] * xy * z * S(10) +
                          kSH_C3[2] * y * (4.0f * zz - xx - yy) * S(11) +
                          kSH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * S(12) +
                          kSH_C3[4] * x * (4.0f * zz - xx - yy) * S(13) +
                          kSH_C3[5] * z * (xx - yy) * S(14) + kSH_C3[6] * x * (xx - 3.0f * yy) * S(15);
                }
            }
        }
#undef S
        res += 0.5f;
        clamped[ch] = res < 0;
        out[ch] = res < 0.0f ? 0.0f : res;
    }
    return make_float3(out[0], out[1], out[2]);
}

// The forward's SH clamp mask (bit c: channel c's colour was clamped at 0), one byte per Gaussian in
// GEOM (`clampm`): the backward reads it instead of re-evaluating the SH colour in every view.
__device__ inline uint8_t clamp_bits(const bool (&cl)[3]) {
    return (uint8_t)((cl[0] ? 1u : 0u) | (cl[1] ? 2u : 0u) | (cl[2] ? 4u : 0u));
}
__device__ inline void clamp_from_mask(uint32_t m, bool (&cl)[3]) { cl[0] = m & 1u; cl[1] = m & 2u; cl[2] = m & 4u; }

// rect packing: x = x0 | y0 << 16, y = x1 | y1 << 16
__device__ inline uint2 pack_rect(int x0, int y0, int x1, int y1) {
    return make_uint2((uint32_t)x0 | ((uint32_t)y0 << 16), (uint32_t)x1 | ((uint32_t)y1 << 16));
}

// ---------------------------------------------------------------------------------------------
// wave64 / block primitives
// ---------------------------------------------------------------------------------------------
__device__ inline uint32_t wave_incl_scan_u32(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// Block-wide exclusive scan over blockDim.x (multiple of 64, <= 1024); `lds` holds >= 16 words.
// Returns the exclusive prefix; *total receives the block sum.  Contains __syncthreads().
__device__ inline uint32_t block_excl_scan_u32(uint32_t v, uint32_t *lds, uint32_t *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint32_t inc = wave_incl_scan_u32(v);
    if (lane == 63) lds[wid] = inc;
    __syncthreads();
    uint32_t woff = 0, tot = 0;
    for (int w = 0; w < nw; ++w) {
        const uint32_t s = lds[w];
        if (w < wid) woff += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return woff + inc - v;
}

// Sum of v over the 64 lanes of the wave, valid in lane 63 (gfx9 DPP row ops + row broadcasts).
__device__ inline float wave_sum_lane63(float v) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));  // quad_perm 1,0,3,2
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));  // quad_perm 2,3,0,1
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x124, 0xF, 0xF, false)); // row_ror:4
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false)); // row_ror:8
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xA, 0xF, false)); // row_bcast:15
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x143, 0xC, 0xF, false)); // row_bcast:31
    return v;
}

constexpr int kTilesPerBlock = 4;
#define GSR_LOG2E 1.4426950408889634f

// Diagnostic builds (make trace -> libgsr_trace.so): every render wave stores (start, end,
// HW_ID) with s_memrealtime (100 MHz, chip-wide) into a buffer registered by
// gsr_debug_trace_{fwd,bwd}; compiled out of libgsr.so.
#ifdef GSR_TRACE
// per wave: start, end, HW_ID | XCC_ID << 32, kernel-defined work counter
__device__ inline void trace_wave(uint64_t *buf, int slot, uint64_t t0, uint64_t work = 0) {
    if (buf && (threadIdx.x & 63) == 0) {
        buf[4 * slot] = t0;
        buf[4 * slot + 1] = __builtin_amdgcn_s_memrealtime();
        buf[4 * slot + 2] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |     // HW_REG_HW_ID
                            ((uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);  // HW_REG_XCC_ID
        buf[4 * slot + 3] = work;
    }
}
#endif

// Blend weight of one (pixel, Gaussian) pair, shared by the forward and backward kernels so that
// both take identical decisions: power2 = power * log2(e) evaluated with FMAs, G = 2^power2.
// Exponent of the Gaussian at a pixel, log2 units: p2 = A2 dx^2 + B2 dx dy + C2 dy^2 with the
// record's pre-scaled conic.  Evaluated as P0 + dy (P1 + C2 dy), P0 = (A2 dx) dx, P1 = B2 dx, so
// the backward (4 pixels of one column per lane) computes the dx-only part once per pair; forward
// and backward use this exact operation sequence, hence bitwise-identical blend decisions.
struct PairX { float dx, P0, P1; };
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ inline f2v f2(float x, float y) { return f2v{x, y}; }
__device__ inline PairX pair_x(float4 r0, float pfx) {
    PairX x;
    x.dx = r0.x - pfx;
    const f2v t = f2(r0.z, r0.w) * f2(x.dx, x.dx);  // (A2 dx, B2 dx): one packed multiply
    x.P0 = t.x * x.dx;
    x.P1 = t.y;
    return x;
}
__device__ inline float pair_power(const PairX &x, float C2, float dy) { return fmaf(dy, fmaf(C2, dy, x.P1), x.P0); }

// f2v (above): two-lane fp32 vectors -- the packed VALU forms (v_pk_add / v_pk_mul / v_pk_fma_f32) do
// two of the same IEEE operations in one instruction, so the results are bitwise the scalar code's.
__device__ inline f2v fma2(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }

struct Blend { float dx, dy, p2, G, alpha; };
// CLAMP = false: no staged opacity exceeds 0.99, so min(0.99, o G) == o G wherever p2 <= 0 (G <= 1)
template <bool CLAMP = true>
__device__ inline Blend blend_eval(float4 r0, float4 r1, float pfx, float pfy) {
    Blend e;
    // (dx, dy) and (A2 dx, B2 dx) as packed pairs: the same operations as pair_x / pair_power
    const f2v d = f2(r0.x, r0.y) - f2(pfx, pfy);
    const f2v t = f2(r0.z, r0.w) * f2(d.x, d.x);
    e.dx = d.x;
    e.dy = d.y;
    e.p2 = fmaf(e.dy, fmaf(r1.x, e.dy, t.y), t.x * d.x);
    e.G = __builtin_amdgcn_exp2f(e.p2);
    e.alpha = CLAMP ? fminf(0.99f, r1.y * e.G) : r1.y * e.G;
    return e;
}
__device__ inline bool blend_ok(const Blend &e) { return e.p2 <= 0.0f && e.alpha >= 1.0f / 255.0f; }

// Near-threshold exact blend weight (exact-threshold mode, gsr_set_exact_thresholds, VERDICT r03
// item 9): the fast weight
// 2^(p2) (FMAs on log2(e)-scaled conic terms + v_exp_f32) differs from the reference's
// expf(-0.5 (a dx^2 + c dy^2) - b dx dy) by a few ulp, so a pair whose weight lies within kNearRel of
// 1/255 can take the other branch.  Such pairs (rare: the wave branches only when a lane has one) are
// re-evaluated with the reference's expression order in fp32 (the library builds with
// -ffp-contract=off, like the oracle) and a double-precision exp rounded to float, from the exact
// conic kept in the render record's 4th float4.
constexpr float kNearRel = 1e-5f;
constexpr float kNearLo = (1.0f / 255.0f) * (1.0f - kNearRel), kNearHi = (1.0f / 255.0f) * (1.0f + kNearRel);
__device__ inline bool near_threshold(float alpha) { return alpha >= kNearLo && alpha < kNearHi; }
// The same for the transmittance test T (1 - alpha) >= 1e-4 (round 6).  The fast
// forward's T (one fmaf per contributor, v_exp_f32 weights) drifts from the reference's (two roundings
// per contributor, the exact weights) by at most t_window(L) relative after L list entries: <= 3
// roundings of 2^-24 per contributor (kTW1) plus the weights' few-ulp differences, which T accumulates
// as sum alpha / (1 - alpha) * (their relative error) <= 5e-5 (kTW0) for T >= 1e-4 -- measured at most
// 4.7e-6 over C2 / C3 / C4 views (tools/t_drift.py).  In the exact-threshold mode the fast
// walk goes on while test_T >= 1e-4 (1 - t_window), so it never stops before the reference would, and
// every pixel whose final T is below 1e-4 (1 + t_window(n_contrib)) -- the only ones whose stop can
// differ -- is redone by k_render_tsat, the reference's walk for that pixel with the exact weights.
constexpr float kTSat = 1e-4f;

constexpr float kTW0 = 5e-5f, kTW1 = 2e-7f;
__device__ inline float t_window(uint32_t L) { return kTW0 + kTW1 * (float)L; }
// exact (power, G, alpha) of the Gaussian at (gx, gy) with exact conic (ca, cb, cc) and opacity o.  Not
// inlined (the double-precision exp would hold registers in the hot loops) and returned by value (a
// by-reference output would put the caller's blend variables in scratch memory).
struct ExactBlend { float power, G, alpha; };
__device__ __attribute__((noinline)) ExactBlend exact_blend(float gx, float gy, float4 conic, float o, float pfx,
                                                            float pfy) {
    const float dx = gx - pfx, dy = gy - pfy;
    ExactBlend r;
    r.power = -0.5f * (conic.x * dx * dx + conic.z * dy * dy) - conic.y * dx * dy;
    r.G = (float)exp((double)r.power);
    r.alpha = fminf(0.99f, o * r.G);
    return r;
}

// A workgroup barrier after this wave's LDS stores / no-return LDS atomics, with an explicit
// s_waitcnt lgkmcnt(0) in front.  __syncthreads()'s release fence normally brings that wait, but the
// compiler dropped it in one build at k_render_fwd's blend-loop head (its loop-carried s_live mask,
// lowered by a no-return ds_and, was then read stale by other waves after the barrier: waves of one
// block left the loop at different batches, the tile's quarter maxima were corrupted and the backward
// went nondeterministic).  An explicit wait is kept by the compiler.
// tools/lds_lint.py (tests/test_lds_lint.py) checks every barrier of the shipped code object for the wait.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "lds_barrier(): 0xC07F is the gfx9 s_waitcnt encoding (lgkmcnt(0)); pick the target's encoding"
#endif
__device__ inline void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // gfx9 encoding: vmcnt / expcnt at maximum, lgkmcnt(0)
    __syncthreads();
}

// Wait until every vector-memory operation of this wave -- its device-scope atomics included -- has
// completed (gfx9 encoding: vmcnt(0), expcnt / lgkmcnt at maximum).  A workgroup-scope release fence
// does not wait for them (it compiles to an LDS wait only), so a block that counts itself done with
// an atomic after its other atomics puts this, then its barrier, in front of the done counter.
__device__ inline void drain_vmem() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Make this wave's LDS writes visible to its own later LDS reads (waves of a render block work
// on different tiles and never synchronise with each other).
__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Longest-processing-time-first dispatch order, computed by ONE block: order[] lists the T tiles
// by descending cost(t) (bucketed into 2048 log-free linear buckets; arbitrary order inside a bucket,
// which only affects scheduling).  `s_hist` must hold 2048 words, `s_red` 16.  All threads call it.
struct IdentityPos { __device__ uint32_t operator()(uint32_t p) const { return p; } };
template <typename CostFn, typename PosMap = IdentityPos>
__device__ inline void lpt_order(int T, CostFn cost, uint32_t *__restrict__ order, uint32_t *s_hist,
                                 uint32_t *s_red, PosMap pos = PosMap()) {
    uint32_t mx = 0;
    for (int t = threadIdx.x; t < T; t += blockDim.x) mx = max(mx, cost(t));
    for (int d = 32; d > 0; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = mx;
    for (int b = threadIdx.x; b < kOrderBuckets; b += blockDim.x) s_hist[b] = 0;
    __syncthreads();
    mx = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) mx = max(mx, s_red[w]);
    int shift = 0;
    while ((mx >> shift) >= (uint32_t)kOrderBuckets) ++shift;
    __syncthreads();
    for (int t = threadIdx.x; t < T; t += blockDim.x)
        atomicAdd(&s_hist[kOrderBuckets - 1 - (cost(t) >> shift)], 1u);  // descending cost
    __syncthreads();
    uint32_t carry = 0;
    for (int base = 0; base < kOrderBuckets; base += blockDim.x) {
        const int b = base + threadIdx.x;
        const uint32_t c = b < kOrderBuckets ? s_hist[b] : 0;
        uint32_t tot;
        const uint32_t ex = block_excl_scan_u32(c, s_red, &tot) + carry;
        if (b < kOrderBuckets) s_hist[b] = ex;
        carry += tot;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < T; t += blockDim.x)
        order[pos(atomicAdd(&s_hist[kOrderBuckets - 1 - (cost(t) >> shift)], 1u))] = (uint32_t)t;
}

// The same LPT order when every thread already holds the costs of the c consecutive tiles
// t = threadIdx.x * c + i (i < c <= C) in registers: the single-block scan kernels prefetch them with
// every load in flight instead of re-reading global memory in dependent strided loops.
template <int C, typename PosMap = IdentityPos>
__device__ inline void lpt_order_regs(int T, int c, const uint32_t (&cost)[C], uint32_t *__restrict__ order,
                                      uint32_t *s_hist, uint32_t *s_red, PosMap pos = PosMap()) {
    const int t0 = threadIdx.x * c;
    uint32_t mx = 0;
#pragma unroll
    for (int i = 0; i < C; ++i)
        if (i < c && t0 + i < T) mx = max(mx, cost[i]);
    for (int d = 32; d > 0; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = mx;
    for (int b = threadIdx.x; b < kOrderBuckets; b += blockDim.x) s_hist[b] = 0;
    __syncthreads();
    mx = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) mx = max(mx, s_red[w]);
    int shift = 0;
    while ((mx >> shift) >= (uint32_t)kOrderBuckets) ++shift;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < C; ++i)
        if (i < c && t0 + i < T) atomicAdd(&s_hist[kOrderBuckets - 1 - (cost[i] >> shift)], 1u);
    __syncthreads();
    uint32_t carry = 0;
    for (int base = 0; base < kOrderBuckets; base += blockDim.x) {
        const int b = base + threadIdx.x;
        const uint32_t h = b < kOrderBuckets ? s_hist[b] : 0;
        uint32_t tot;
        const uint32_t ex = block_excl_scan_u32(h, s_red, &tot) + carry;
        if (b < kOrderBuckets) s_hist[b] = ex;
        carry += tot;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < C; ++i)
        if (i < c && t0 + i < T)
            order[pos(atomicAdd(&s_hist[kOrderBuckets - 1 - (cost[i] >> shift)], 1u))] = (uint32_t)(t0 + i);
}
// Boustrophedon over rounds of S slots: rank p of round r = p / S lands at slot p % S in even rounds and
// at the mirrored slot in odd ones (the last, partial round mirrors within its own length).  For a
// launch whose waves are all resident at once (one wave per SIMD per round, S = SIMDs), each SIMD
// then holds one heavy and one light tile of every pair of rounds instead of the k-th heaviest of
// every round.
struct SnakePos {
    uint32_t S, T;
    __device__ uint32_t operator()(uint32_t p) const {
        const uint32_t r = p / S, j = p - r * S;
        if (!(r & 1u)) return p;
        const uint32_t L = min(S, T - r * S);
        return r * S + (L - 1u - j);
    }
};

// Tiles per thread held in registers by the single-block kernels (1024 threads): T <= 16384.
constexpr int kScanRegs = 16;

// XCD-aware bijection over T tiles: blocks b, b+8, ... (one XCD under round-robin dispatch) take a
// contiguous run of tiles, so neighbouring tiles share Gaussian records in one L2.  Speed only.
__device__ inline int remap_tile(int b, int T) {
    const int x = b & 7, i = b >> 3, q = T >> 3, r = T & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// Conservative (tile, Gaussian) cull: true only if NO pixel centre of the pixel rectangle
// [x0, x1] x [y0, y1] can reach alpha >= 1/255.  Q(d) = a dx^2 + 2 b dx dy + c dy^2 is the
// Mahalanobis form of the blend's power (power = -Q/2); its minimum over the tile rectangle is
// compared with tau = 2 ln(255 o) with a margin that dominates the fp32 rounding of the per-pixel
// evaluation (valid while |b| / sqrt(ac) < 0.999; thinner ellipses are never culled).  Culling a
// pair therefore changes no output: the per-pixel test would have skipped it everywhere.
__device__ inline bool tile_cull(float gx, float gy, float a, float b, float c, float o, float tau,
                                 float x0, float y0, float x1, float y1) {
    if (o < 1.0f / 255.0f) return true;  // alpha = min(.99, o exp(power)) <= o for power <= 0
    if (!(b * b < 0.998f * a * c)) return false;
    const float dxlo = gx - x1, dxhi = gx - x0;
    const float dylo = gy - y1, dyhi = gy - y0;
    if (dxlo <= 0.f && dxhi >= 0.f && dylo <= 0.f && dyhi >= 0.f) return false;  // centre inside
    // Each edge's minimiser uses the hardware reciprocal (1 ulp) instead of an IEEE division: a
    // slightly-off minimiser inside the clamp range can only RAISE the edge value, by O(c ddy^2),
    // ~1e-14 relative -- far inside the margin below, so the cull stays conservative.
    const float ia = __builtin_amdgcn_rcpf(a), ic = __builtin_amdgcn_rcpf(c);
    float qmin;
    {   // edges with dx fixed: minimise over dy
        float dx = dxlo;
        float dy = fminf(fmaxf(-b * dx * ic, dylo), dyhi);
        qmin = a * dx * dx + 2.f * b * dx * dy + c * dy * dy;
        dx = dxhi;
        dy = fminf(fmaxf(-b * dx * ic, dylo), dyhi);
        qmin = fminf(qmin, a * dx * dx + 2.f * b * dx * dy + c * dy * dy);
        // edges with dy fixed: minimise over dx
        dy = dylo;
        dx = fminf(fmaxf(-b * dy * ia, dxlo), dxhi);
        qmin = fminf(qmin, a * dx * dx + 2.f * b * dx * dy + c * dy * dy);
        dy = dyhi;
        dx = fminf(fmaxf(-b * dy * ia, dxlo), dxhi);
        qmin = fminf(qmin, a * dx * dx + 2.f * b * dx * dy + c * dy * dy);
    }
    return qmin > tau * 1.001f + 1e-3f;
}

// ---- cross-lane folds over a wave64 (gfx950) ----------------------------------------------
// No-return LDS float add (ds_add_f32).
__device__ inline void lds_add(float *p, float v) {
    (void)__hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ inline float fold32(float a, float b) {  // lanes 0-31: a folded, lanes 32-63: b folded
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ inline float fold16(float a, float b) {  // rows (a0+a1, b0+b1, a2+a3, b2+b3)
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
}  // namespace gsr
