// gsr_backward.hip -- backward pass of the MI355X-native Gaussian-splat rasterizer.
//
//   k_render_bwd  1 wave64 / (tile, segment of kSeg entries): per-pixel reverse walk (SURVEY.md 2.1
//                 row renderCUDA bwd) from the blend state the forward saved at the segment's end.
//                 Instead of the reference's per-pixel float atomics into per-Gaussian buffers, the
//                 wave reduces its 256 pixels' partials with permlane swaps + DPP and stores one
//                 36-byte record per (tile, Gaussian) pair at the pair's emission slot: no global
//                 atomics, bitwise reproducible.
//   k_gauss_bwd   1 thread / Gaussian: sums its slot records in emission order (through the
//                 emission->slot map written by k_tile_sort), then the fused per-Gaussian chain
//                 computeCov2D bwd -> projection bwd -> SH bwd -> Sigma3D bwd (SURVEY.md 2.1 rows
//                 computeCov2DCUDA + preprocessCUDA bwd).  Writes every output element.
#include "gsr_common.h"
#include "gsr_internal.h"

#include <algorithm>

namespace gsr {

#ifdef GSR_TRACE
__device__ uint64_t *g_trace_bwd;
#endif

constexpr uint32_t kItemStartCost = 64;  // init loads + first gathers, in (pair, quarter) steps

// The same item list built over the whole chip (the single block above runs on ONE CU: ~30 us at C3,
// 21 at C2, on the view's critical path).  k_items_count: one thread per tile counts its items per cost
// bucket in an LDS histogram, the block adds its non-zero buckets into the workspace's global counts,
// and the last block to finish (a done counter) turns the counts into the buckets' cursors (exclusive
// scan, descending cost).  k_items_emit: each block counts its tiles' items again, reserves its run in
// every bucket with one global atomic, and hands out the slots from LDS.  Order inside a bucket
// follows the atomics (scheduling only).
constexpr int kItemsBlock = 256;  // tiles (threads) per block
struct ItemBucket {  // item cost -> LPT bucket (descending cost) for segments of 2^ks entries
    uint32_t shift;
    __device__ explicit ItemBucket(int ks) {
        const uint32_t mx = (4u << ks) + kItemStartCost;
        shift = mx >= (uint32_t)kOrderBuckets ? 32 - __builtin_clz(mx / kOrderBuckets) : 0;
    }
    __device__ uint32_t operator()(uint32_t cost) const {
        return (uint32_t)kOrderBuckets - 1u - min(cost >> shift, (uint32_t)kOrderBuckets - 1u);
    }
};
// f(item code, bucket) for every item of a tile with n list entries and quarter maxima mq
template <typename F>
__device__ inline void for_tile_items(uint32_t n, uint4 mq, int ks, const ItemBucket &bk, F f) {
    const uint32_t J = bwd_item_count(n, mq, ks), Z = bwd_zero_items(n, mq);
    for (uint32_t j = 0; j < J + Z; ++j) {
        const uint32_t cost = j < J ? bwd_item_cost(j, mq, ks) + kItemStartCost : kItemStartCost;
        f(j < J ? j : kZeroItem | (j - J), bk(cost));
    }
}

__global__ __launch_bounds__(kItemsBlock) void k_items_count(int T, const uint2 *__restrict__ ranges,
                                                             const uint32_t *__restrict__ tile_maxc,
                                                             const uint32_t *__restrict__ tile_flag,
                                                             uint2 *__restrict__ items, uint32_t *__restrict__ ws,
                                                             const uint32_t *__restrict__ spec_ok, int ks) {
    __shared__ uint32_t s_hist[kOrderBuckets];
    __shared__ uint32_t s_red[16];
    __shared__ uint32_t s_last;
    if (spec_ok && *spec_ok == 0u) return;  // speculative launch whose capacity failed: redone by the host
    for (int b = threadIdx.x; b < kOrderBuckets; b += blockDim.x) s_hist[b] = 0;
    __syncthreads();
    const ItemBucket bk(ks);
    const int t = blockIdx.x * kItemsBlock + (int)threadIdx.x;
    if (t < T && tile_flag[t] <= kNearCap) {  // (near-record overflow tiles' items are listed after these)
        const uint2 rg = ranges[t];
        const uint4 mq = reinterpret_cast<const uint4 *>(tile_maxc)[t];
        for_tile_items(rg.y - rg.x, mq, ks, bk, [&](uint32_t, uint32_t b) { atomicAdd(&s_hist[b], 1u); });
    }
    lds_barrier();  // (no-return LDS atomics)
    for (int b = threadIdx.x; b < kOrderBuckets; b += blockDim.x) {
        const uint32_t h = s_hist[b];
        if (h) atomicAdd(&ws[b], h);
    }
    // (no agent-scope fence: it would write back / invalidate the XCD's whole L2; the counts are
    // device-scope atomics, drained by an explicit vmcnt(0) before the done counter)
    drain_vmem();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(&ws[2 * kOrderBuckets], 1u) == gridDim.x - 1 ? 1u : 0u;
    __syncthreads();
    if (!s_last) return;
    // the last block: every block's counts are in; cursors = exclusive scan, counts + counter reset
    constexpr int kPer = kOrderBuckets / kItemsBlock;
    const int b0 = (int)threadIdx.x * kPer;
    uint32_t h[kPer], sum = 0;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        h[i] = __hip_atomic_load(&ws[b0 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sum += h[i];
    }
    uint32_t tot;
    uint32_t ex = block_excl_scan_u32(sum, s_red, &tot);
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        ws[kOrderBuckets + b0 + i] = ex;
        ws[b0 + i] = 0;
        ex += h[i];
    }
    if (threadIdx.x == 0) {
        items[0] = make_uint2(tot, 0u);
        ws[2 * kOrderBuckets] = 0;
    }
}

__global__ __launch_bounds__(kItemsBlock) void k_items_emit(int T, const uint2 *__restrict__ ranges,
                                                            const uint32_t *__restrict__ tile_maxc,
                                                            const uint32_t *__restrict__ tile_flag,
                                                            uint2 *__restrict__ items, uint32_t *__restrict__ ws,
                                                            const uint32_t *__restrict__ spec_ok, int ks) {
    __shared__ uint32_t s_cur[kOrderBuckets];
    if (spec_ok && *spec_ok == 0u) return;
    for (int b = threadIdx.x; b < kOrderBuckets; b += blockDim.x) s_cur[b] = 0;
    __syncthreads();
    const ItemBucket bk(ks);
    const int t = blockIdx.x * kItemsBlock + (int)threadIdx.x;
    const uint2 rg = t < T ? ranges[t] : make_uint2(0, 0);
    const uint4 mq = t < T ? reinterpret_cast<const uint4 *>(tile_maxc)[t] : make_uint4(0, 0, 0, 0);
    const bool ex = t < T && tile_flag[t] > kNearCap;
    // a tile with more near-threshold records than kNearCap: its items go after the others' ([0].x of
    // them), unordered, counted in [0].y (zeroed by k_items_count), for k_render_bwd<true>
    if (ex) {
        const uint32_t base = 1u + items[0].x;
        for_tile_items(rg.y - rg.x, mq, ks, bk, [&](uint32_t code, uint32_t) {
            items[base + atomicAdd(&items[0].y, 1u)] = make_uint2((uint32_t)t, code);
        });
    }
    const uint32_t n = ex ? 0u : rg.y - rg.x;
    for_tile_items(n, mq, ks, bk, [&](uint32_t, uint32_t b) { atomicAdd(&s_cur[b], 1u); });
    lds_barrier();  // (no-return LDS atomics)
    for (int b = threadIdx.x; b < kOrderBuckets; b += blockDim.x) {  // this block's run in each bucket
        const uint32_t h = s_cur[b];
        if (h) s_cur[b] = atomicAdd(&ws[kOrderBuckets + b], h);
    }
    lds_barrier();
    for_tile_items(n, mq, ks, bk, [&](uint32_t code, uint32_t b) {
        items[1 + atomicAdd(&s_cur[b], 1u)] = make_uint2((uint32_t)t, code);
    });
}

// One wave64 per (tile, segment) item, 4 pixels per lane (pixel k of lane l: column l & 15, row
// (l >> 4) + 4 k, i.e. quarter k = rows 4k..4k+3), reverse walk over the segment's entries in
// batches of 64.  Per surviving (tile, Gaussian) pair each contributing pixel adds sG = o G dL/dalpha
// times (1, dx, dy, dx^2, dx dy, dy^2) and w dL/dpix (w = alpha T, the colour gradient); the lane
// sums its 4 pixels in registers, the wave reduces them with permlane swaps + DPP (pair_sums), and at
// the end of the batch the lane that staged Gaussian j turns its sums into the reference's per-pair
// quantities (dmeans2D in NDC units, dconic (a, b, c) in the b/2 convention, dopacity, dcolour) with
// the exact conic, storing one 36-byte record at the pair's emission slot (no atomics).
//
// A segment [s0, s0 + kSeg) starts from the blend state behind its last entry: for a quarter whose
// pixels' contributors reach past the segment, the state the forward saved at that boundary --
// transmittance T and front colour C_f, so the colour behind, projected on dL/dpixel, is
// AR = (<dL/dpix, C_all - C_f> + T_final <bg, dL/dpix>) / T -- otherwise the pixel's final state
// (T_final, AR = <bg, dL/dpix>).
// One 36-byte partial-gradient record at emission slot `em` of the packed record array: three
// 12-byte stores (4-byte aligned), the kPartial values in slot order.
struct __attribute__((packed, aligned(4))) F3 { float x, y, z; };
__device__ inline void rec_store(float4 *part, uint32_t em, float r0, float r1, float r2, float r3, float r4,
                                 float r5, float r6, float r7, float r8) {
    F3 *d = reinterpret_cast<F3 *>(reinterpret_cast<float *>(part) + (size_t)kRecF * em);
    d[0] = F3{r0, r1, r2};
    d[1] = F3{r3, r4, r5};
    d[2] = F3{r6, r7, r8};
}

// the register budget: 7 waves per SIMD (72 VGPRs, LDS 21.5 KB per 4-wave workgroup; the record's two
// tail inputs live in a register pair that the compiler parks in scratch during the walk: one store and
// one load per batch).  1 % faster alone than 6 waves (profiles/r05_bwd_waves_ab.txt; 5 -> 6 was 3 %).
// The near-overflow variant keeps 4 (its re-evaluation call site needs the registers).
#define GSR_BWD_ATTR __attribute__((amdgpu_waves_per_eu(EXACT ? 4 : 7, 8)))
constexpr int kBwdWaves = 4;  // items (one wave each) per workgroup
#ifndef GSR_EXACT_BWD_BLOCKS
#define GSR_EXACT_BWD_BLOCKS 256
#endif
constexpr int kExactBwdBlocks = GSR_EXACT_BWD_BLOCKS;  // grid of the exact-threshold tiles' k_render_bwd

// ---- the pair reduction ---------------------------------------------------------------------------
// Every lane holds, for its 4 pixels of one column, S0 = sum sG, S1 = sum sG dy, S4 = sum sG dy^2 and
// cs_c = sum w dL/dpix_c.  The rows of a column are folded first (3 permlane32 + 2 permlane16 swaps
// on the 6 raw values), the column weights dx, dx^2 applied to the 16 column sums, and each 16-lane
// row summed by 3 DPP stages into two halves (lanes of each parity: lanes 0 and 1 of the row hold
// them, both added into the pair's LDS slot).  Row totals, slot = 4 * register + row:
//   X rows: [sum dx S0, sum S4, sum S1, sum cs0]      (slots 0-3)
//   Y rows: [sum dx^2 S0, sum cs1, sum dx S1, sum cs2] (slots 4-7)
//   Z row 0: sum S0                                   (slot 8)
// Fixed tree: bitwise reproducible.
// The three row reductions of a pair, each 16-lane row summed by 3 DPP stages (row_ror 8, 4, 2) into
// halves over the lanes of each parity -- lanes 0 and 1 of the row hold them.  Written out so that every
// stage is one v_add_f32_dpp (the compiler keeps the last stage's move and add apart when the add sinks
// into the storing lanes' branch); the three registers are interleaved, so each stage reads a register
// written two instructions earlier (the VALU-write -> DPP-read hazard needs 2 wait states; the s_nop
// covers the inputs' own writes).
__device__ inline void row_halves3(float &X, float &Y, float &Z) {
    asm("s_nop 1\n\t"
        "v_add_f32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %1, %1, %1 row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %2, %2, %2 row_ror:8 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %1, %1, %1 row_ror:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %2, %2, %2 row_ror:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %0, %0, %0 row_ror:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %1, %1, %1 row_ror:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_add_f32_dpp %2, %2, %2 row_ror:2 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "+v"(X), "+v"(Y), "+v"(Z));
}
struct RowW { bool r0, r2; };  // the lane's row of the folded column sums is row 0 / row 2 (lane masks)
__device__ inline RowW row_weights(int row) { return RowW{row == 0, row == 2}; }
struct PairSums { float X, Y, Z; };
__device__ inline PairSums pair_sums(float S0, float S1, float S4, float cs0, float cs1, float cs2, float dx,
                                     const RowW &w) {
    const float pA = fold32(S0, S1), pB = fold32(S4, cs0), pC = fold32(cs1, cs2);
    const float rA = fold16(pA, pB);   // column sums, rows [S0, S4, S1, cs0]
    const float rC = fold16(0.f, pC);  // rows [0, cs1, 0, cs2]
    const float wx = w.r0 ? dx : 1.f;                           // row 0: dx, else 1
    const float wy = w.r0 ? dx * dx : (w.r2 ? dx : 0.f);        // row 0: dx^2, row 2: dx, else 0
    PairSums r{rA * wx, fmaf(rA, wy, rC), rA};
    row_halves3(r.X, r.Y, r.Z);
    return r;
}

// Per-pixel walk state of one quarter slot k.
struct PixState { float T, AR; f2v d01; float d2, fy; int lrel; };  // d01: dL/dpix channels 0, 1
// Running per-lane sums of one walked pair (packed pairs: (S1, S4), (c0, c1)).
struct LaneSums { float S0; f2v S14, c01; float c2; };

// One (pair, quarter) evaluation.  CLAMP: the pair's opacity can exceed 0.99, so alpha may be clamped
// (wave-uniform, flagged at staging); otherwise alpha = o G exactly and sG = o G T (C - AR) = w (C - AR)
// with w = alpha T, the colour weight -- the same product in fewer operations.  Branch-free: a pixel
// that does not take the pair gets alpha = 0, which makes every update an identity (r = 1, AR
// unchanged, zero sums).  The blend weight is pair_power + 2^x, the forward's exact operation
// sequence, hence bitwise-identical decisions.
// NEAR (exact-threshold mode, a tile whose forward re-evaluated near-threshold weights): kNearLook --
// a weight in the near window takes the forward's re-evaluated (power, G, alpha) from the tile's near
// records (key: list position << 8 | pixel k of the lane = lane + 64 k); kNearEval -- re-evaluated here
// as the forward did (a tile with more records than kNearCap).  Either way the forward's decisions.
constexpr int kNearNone = 0, kNearLook = 1, kNearEval = 2;
struct NearRecs { const float4 *r; uint32_t n; int start; };  // the tile's records, the batch's list start
template <bool CLAMP, int NEAR>
__device__ __forceinline__ void eval_quarter(PixState &ps, LaneSums &s, bool &any, const PairX &x, float4 a,
                                             float C2, float o, float4 c, int j, int k, float pfx,
                                             const float4 *__restrict__ rec, const uint32_t *__restrict__ pl,
                                             const NearRecs &nrs) {
    const float dy = a.y - ps.fy;  // same operation as the forward's
    float p2 = pair_power(x, C2, dy);
    float G = __builtin_amdgcn_exp2f(p2);
    float alpha = CLAMP ? fminf(0.99f, o * G) : o * G;
    const bool live = j < ps.lrel;  // the entry lies before this pixel's last contributor
    if constexpr (NEAR == kNearEval) {  // the forward's near-threshold re-evaluation: the same decisions
        // (the forward re-evaluates only a weight it would otherwise take: p2 <= 0 included)
        const bool nr = live && p2 <= 0.0f && near_threshold(alpha);
        if (nr) {  // (an exec-masked region, skipped when no lane has one)
            const ExactBlend e = exact_blend(a.x, a.y, rec[(size_t)kRecF4 * pl[j] + 3], o, pfx, ps.fy);
            p2 = e.power; G = e.G; alpha = e.alpha;
        }
    } else if constexpr (NEAR == kNearLook) {
        const bool nr = live && p2 <= 0.0f && near_threshold(alpha);
        if (nr) {  // (an exec-masked region, skipped when no lane has one)
            const uint32_t key = ((uint32_t)(nrs.start + j) << 8) | (uint32_t)((threadIdx.x & 63) + 64 * k);
            for (uint32_t i = 0; i < nrs.n; ++i) {  // (uniform loads)
                const float4 r = nrs.r[i];
                const bool hit = __float_as_uint(r.x) == key;
                p2 = hit ? r.y : p2;
                G = hit ? r.z : G;
                alpha = hit ? r.w : alpha;
            }
        }
    }
    const bool ok = live && p2 <= 0.0f && alpha >= 1.0f / 255.0f;
    any = any || ok;
    const float al = ok ? alpha : 0.f;
    ps.T = ps.T * __builtin_amdgcn_rcpf(1.f - al);  // T in front of the pair
    const float cd = fmaf(c.z, ps.d2, fmaf(c.y, ps.d01.y, c.x * ps.d01.x));  // <colour, dL/dpix>
    const float diff = cd - ps.AR;
    ps.AR = fmaf(al, diff, ps.AR);
    const float w = al * ps.T;
    float gd;  // sG = o G T (C - AR), the reference's dL/dG * G scaled by the opacity
    if constexpr (CLAMP) {
        const float tg = ps.T * diff;
        gd = ok ? (o * G) * tg : 0.f;  // the reference's alpha gradient ignores the 0.99 clamp
    } else {
        gd = w * diff;
    }
    const float u = gd * dy;
    s.S0 += gd;
    s.S14 = fma2(f2(gd, u), f2(dy, dy), s.S14);  // S1 += gd dy (fused), S4 += u dy
    s.c01 = fma2(f2(w, w), ps.d01, s.c01);
    s.c2 = fmaf(w, ps.d2, s.c2);
}

// The walk of one batch: every staged pair j (descending) over the quarters of its mask; each pair's
// sums are reduced and added into its s_out slot when any pixel of the wave took it.  CLAMP: some
// staged pair's opacity exceeds 0.99 (batch-uniform, so the pair loop itself has no variant branch).
template <bool CLAMP, int NEAR>
__device__ __forceinline__ void walk_batch(PixState (&ps)[4], uint64_t m, const float4 *s_a, float pfx,
                                           const RowW &rw, float *o_row, const float4 *__restrict__ rec,
                                           const uint32_t *__restrict__ pl, const NearRecs &nrs) {
    constexpr int kStage = 64 * kBwdWaves;
    while (m) {
        const int j = 63 - __builtin_clzll(m);
        m &= ~(1ull << j);
        const float4 a = s_a[j], b = s_a[kStage + j], c = s_a[2 * kStage + j];
        // wave-uniform quarter mask of the staged entry
        const uint32_t qm = __builtin_amdgcn_readfirstlane(__float_as_uint(c.w));
        const PairX x = pair_x(a, pfx);
        // -0 seeds: x + (-0) == x for every x, so the first contributor needs no add (the ISA folds it)
        LaneSums s{-0.f, f2(-0.f, -0.f), f2(-0.f, -0.f), -0.f};
        bool any = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!(qm & (1u << k))) continue;  // wave-uniform: quarter k cannot reach alpha >= 1/255
            eval_quarter<CLAMP, NEAR>(ps[k], s, any, x, a, b.x, b.y, c, j, k, pfx, rec, pl, nrs);
        }
        // the skip pays although only ~3 % of the walked pairs have no taker (tools/contrib_stats.py):
        // always reducing measured 0.325 vs 0.316 ms alone (profiles/r05_bwd_micro_ab.txt)
        if (__builtin_amdgcn_ballot_w64(any)) {  // some pixel of the wave took the pair
            const PairSums sm = pair_sums(s.S0, s.S14.x, s.S14.y, s.c01.x, s.c01.y, s.c2, x.dx, rw);
            if ((threadIdx.x & 14) == 0) {  // lanes 0 and 1 of each row hold its two halves
                float *o = o_row + j * kPartial;
                lds_add(o, sm.X);
                lds_add(o + 4, sm.Y);
                if ((threadIdx.x & 63) < 2) lds_add(o + 8, sm.Z);
            }
        }
    }
}

// One (tile, segment) item of k_render_bwd on one wave, with the wave's LDS slices: per staged entry
// (x, y, A2, B2); + kStage: (C2, opacity, exact conic a, b); + 2 kStage: colour + quarter mask -- the
// record's inputs wait in LDS, not in registers, while the batch is walked (but for the exact conic's
// c and the emission index, which the staging lane keeps).
template <bool EXACT>
__device__ __forceinline__ void bwd_item(
    uint2 it, uint32_t item, int W, int H, int gx, const uint2 *__restrict__ ranges,
    const uint32_t *__restrict__ point_list,
    const float4 *__restrict__ rec, const float *__restrict__ bg, const float4 *__restrict__ pix_end,
    const uint32_t *__restrict__ n_contrib, const uint32_t *__restrict__ tile_maxc,
    const uint32_t *__restrict__ seg_off, const float4 *__restrict__ seg_state,
    const uint32_t *__restrict__ slot_emit, const float *__restrict__ dL_dpixels,
    float4 *__restrict__ part, int ks, const uint32_t *__restrict__ tile_flag,
    const float4 *__restrict__ near_rec, float4 *s_a, float *s_out) {
    constexpr int kStage = 64 * kBwdWaves;
#ifdef GSR_TRACE
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    const int tile = (int)it.x;
    const uint32_t seg = it.y;
    const uint2 rg = ranges[tile];
    const int n = (int)(rg.y - rg.x);
    const int tx = tile % gx, ty = tile / gx;
    const int lane = threadIdx.x & 63;
    const int px = tx * kTileW + (lane & 15);
    const int py0 = ty * kTileH + (lane >> 4);
    const float pfx = (float)px;
    const float tx0 = (float)(tx * kTileW), ty0 = (float)(ty * kTileH);
    const float tx1 = tx0 + (kTileW - 1);
    const uint4 mq = reinterpret_cast<const uint4 *>(tile_maxc)[tile];  // per quarter-tile maxima
    const int maxc = min((int)max(max(mq.x, mq.y), max(mq.z, mq.w)), n);
    if (seg & kZeroItem) {  // zero records for one kZeroChunk of the slots past maxc (see bwd_zero_items)
        const int z0 = maxc + (int)kZeroChunk * (int)((seg & ~kZeroItem) + 1);
        for (int p = z0 + lane; p < min(n, z0 + (int)kZeroChunk); p += 64) {
            rec_store(part, slot_emit[rg.x + p], 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f);
        }
        return;
    }
    const int s0 = (int)seg << ks, s1f = s0 + (1 << ks);
    const int s1 = min(s1f, maxc);
    if (s1f >= maxc) {  // the tile's last segment item: the first kZeroChunk slots nobody reached
        for (int p = maxc + lane; p < min(n, maxc + (int)kZeroChunk); p += 64) {
            rec_store(part, slot_emit[rg.x + p], 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f);
        }
    }
    const float half_w = (float)(0.5 * W), half_h = (float)(0.5 * H);
    const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];
    // Per pixel state of the reverse walk.  The reference keeps accum_rec and last_color per channel
    // and folds the previous contributor into accum_rec when it meets the next one; dL/dalpha only
    // needs the projection of accum_rec on dL/dpixel, and folding eagerly right after each
    // contributor (AR <- AR + alpha (<c, dL/dpix> - AR)) gives the same value, while a
    // non-contributing pair (alpha = 0) leaves it untouched without a select.  The reference's
    // background term -T_final / (1 - alpha) <bg, dL/dpix> is carried inside AR: starting the
    // recurrence from the background seen through T_final gives exactly T_before (<c, dL/dpix> - AR).
    PixState ps[4];
    const uint32_t qmax[4] = {mq.x, mq.y, mq.z, mq.w};
    const bool has_bound = s1f < n;
    const size_t bidx = has_bound ? ((size_t)seg_off[tile] + seg) * kTilePix : 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int py = py0 + 4 * k;
        ps[k].fy = (float)py;
        const bool inside = px < W && py < H;
        const int pid = py * W + px;
        const float4 pe = inside ? pix_end[pid] : make_float4(0.f, 0.f, 0.f, 0.f);
        // entry p lies before the pixel's last contributor iff p < n_contrib: kept relative to the
        // batch start (lrel = n_contrib - start, advanced per batch)
        ps[k].lrel = (inside ? (int)n_contrib[pid] : 0) - s1;
        ps[k].d01 = f2(inside ? dL_dpixels[pid] : 0.f, inside ? dL_dpixels[H * W + pid] : 0.f);
        ps[k].d2 = inside ? dL_dpixels[2 * H * W + pid] : 0.f;
        float bd = 0;
        bd += bg0 * ps[k].d01.x; bd += bg1 * ps[k].d01.y; bd += bg2 * ps[k].d2;
        if (has_bound && qmax[k] >= (uint32_t)s1f) {  // wave-uniform: this quarter resumes at the boundary
            const float4 st = seg_state[bidx + 64 * k + lane];
            ps[k].T = st.w;
            const float behind = ps[k].d01.x * (pe.x - st.x) + ps[k].d01.y * (pe.y - st.y) + ps[k].d2 * (pe.z - st.z);
            ps[k].AR = st.w > 0.f ? (behind + pe.w * bd) / st.w : bd;
        } else {
            ps[k].T = pe.w;
            ps[k].AR = bd;
        }
    }
    const RowW rw = row_weights(lane >> 4);
    float *o_row = s_out + (lane >> 4);  // this lane's row slot of every pair's sums
    // the tile's near records (exact-threshold mode; none when its forward re-evaluated no weight)
    NearRecs nrs{near_rec + (size_t)kNearCap * tile, EXACT ? 0u : tile_flag[tile], 0};
    // the point list entry of each batch's slot is loaded one batch ahead (the render record gathers
    // depend on it); the records themselves are gathered at the batch start
    uint32_t g_n = 0, em_n = 0;
    auto fetch = [&](int e) {
        const int st = e - 64 > s0 ? e - 64 : s0;
        if (lane < e - st) {
            g_n = point_list[rg.x + st + lane];
            em_n = slot_emit[rg.x + st + lane];
        }
    };
    if (s1 > s0) fetch(s1);
    for (int end = s1; end > s0; end -= 64) {
        const int start = end - 64 > s0 ? end - 64 : s0;
        const int cnt = end - start;
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a, c = a, cj = a;
        float2 tl = make_float2(0.f, 0.f);
        if (lane < cnt) {
            const float4 *r = rec + (size_t)kRecF4 * g_n;
            a = r[0]; b = r[1]; c = r[2]; cj = r[3];  // cj: exact conic (a, b, c) of the staged Gaussian
            tl = make_float2(cj.z, __uint_as_float(em_n));
        }
        if (end - 64 > s0) fetch(end - 64);
#pragma unroll
        for (int q = 0; q < kPartial; ++q) s_out[lane * kPartial + q] = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) ps[k].lrel += cnt;  // n_contrib - start
        // cull per 16x4 quarter: pixel slot k of every lane lies in rows 4k..4k+3 of the tile; a
        // quarter whose pixels all precede this slot in the forward's order (p >= its max
        // n_contrib) is skipped too.  Bit 4: the opacity can be clamped (alpha = min(0.99, o G)).
        uint32_t qmask = 0;
        if (lane < cnt) {
            const uint32_t p = (uint32_t)(start + lane);
            s_a[lane] = a;
            s_a[kStage + lane] = make_float4(b.x, b.y, cj.x, cj.y);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (p < qmax[k] &&
                    !tile_cull(a.x, a.y, -2.f * a.z, -a.w, -2.f * b.x, b.y, b.w, tx0, ty0 + 4 * k, tx1, ty0 + 4 * k + 3))
                    qmask |= 1u << k;
            if (qmask && b.y > 0.99f) qmask |= 16u;  // (the batch then takes the clamping walk)
            s_a[2 * kStage + lane] = make_float4(c.x, c.y, c.z, __uint_as_float(qmask));  // .w: the quarter mask
        }
        uint64_t m = __ballot(qmask != 0);
        wave_lds_sync();
        const uint32_t *pl = point_list + rg.x + start;
        const bool clamp = __builtin_amdgcn_ballot_w64(qmask & 16u) != 0;
        if constexpr (EXACT) {
            if (clamp) walk_batch<true, kNearEval>(ps, m, s_a, pfx, rw, o_row, rec, pl, nrs);
            else walk_batch<false, kNearEval>(ps, m, s_a, pfx, rw, o_row, rec, pl, nrs);
        } else {
            nrs.start = start;
            if (nrs.n) {  // (wave-uniform: the tile's forward re-evaluated near-threshold weights)
                if (clamp) walk_batch<true, kNearLook>(ps, m, s_a, pfx, rw, o_row, rec, pl, nrs);
                else walk_batch<false, kNearLook>(ps, m, s_a, pfx, rw, o_row, rec, pl, nrs);
            } else {
                if (clamp) walk_batch<true, kNearNone>(ps, m, s_a, pfx, rw, o_row, rec, pl, nrs);
                else walk_batch<false, kNearNone>(ps, m, s_a, pfx, rw, o_row, rec, pl, nrs);
            }
        }
        wave_lds_sync();
        if (lane < cnt) {
            const float *s2 = s_out + lane * kPartial;
            float sm[kPartial];
#pragma unroll
            for (int q = 0; q < kPartial; ++q) sm[q] = s2[q];
            const float4 bj = s_a[kStage + lane];  // (C2, opacity, exact conic a, b)
            // tl: (exact conic c, emission index) of the entry this lane staged
            const float o = bj.y;
            const uint32_t em = __float_as_uint(tl.y);
            // sums of sG = o G dL/dalpha: the opacity is already in; dL/dopacity = sum G dL/dalpha
            rec_store(part, em,
                      (-bj.z * sm[0] - bj.w * sm[2]) * half_w,  // dL/dmeans2D.x (NDC)
                      (-bj.w * sm[0] - tl.x * sm[2]) * half_h,  // dL/dmeans2D.y (NDC)
                      -0.5f * sm[4],                            // dL/dconic.a
                      -0.5f * sm[6],                            // dL/dconic.b (b/2 convention)
                      -0.5f * sm[1],                            // dL/dconic.c
                      sm[8] != 0.f ? sm[8] / o : 0.f,           // dL/dopacity
                      sm[3], sm[5], sm[7]);                     // dL/dcolour
        }
    }
#ifdef GSR_TRACE
    trace_wave(g_trace_bwd, item, t_start, 0);
#endif
}


template <bool EXACT>
__global__ __launch_bounds__(64 * kBwdWaves) GSR_BWD_ATTR void k_render_bwd(
    int W, int H, int gx, const uint2 *__restrict__ items, const uint2 *__restrict__ ranges,
    const uint32_t *__restrict__ point_list,
    const float4 *__restrict__ rec, const float *__restrict__ bg, const float4 *__restrict__ pix_end,
    const uint32_t *__restrict__ n_contrib, const uint32_t *__restrict__ tile_maxc,
    const uint32_t *__restrict__ seg_off, const float4 *__restrict__ seg_state,
    const uint32_t *__restrict__ slot_emit, const float *__restrict__ dL_dpixels,
    float4 *__restrict__ part, int ks, const uint32_t *__restrict__ spec_ok,
    const uint32_t *__restrict__ tile_flag, const float4 *__restrict__ near_rec) {
    // Each wave of the workgroup takes its own item and its own LDS slice; the waves never
    // synchronise with each other.  Items are in descending cost order, so the kBwdWaves items of
    // one workgroup cost about the same: grouping them keeps the launch's workgroups coarse, which
    // leaves the CUs' free slots to the forward kernels of the other streams in a pipelined step
    // (one-wave workgroups take every slot a finishing wave frees and starve their large-LDS
    // workgroups).
    // Staging: one array, so the three record parts of entry j are at fixed offsets from one address
    // (one address VGPR per pair, the rest immediate offsets).
    constexpr int kStage = 64 * kBwdWaves;
    __shared__ float4 s_stage[3 * kStage];
    __shared__ float s_out_all[64 * kPartial * kBwdWaves];  // per staged pair: its kPartial wave sums
    if (spec_ok && *spec_ok == 0u) return;  // speculative render half whose forward was redone: redone too
    // (the wave index as a scalar: the item, its tile and everything derived from them live in SGPRs)
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float4 *s_a = s_stage + 64 * wv;
    float *s_out = s_out_all + 64 * kPartial * wv;
    const uint2 hd = items[0];  // (items, items of the tiles with more than kNearCap near records after them)
    if constexpr (EXACT) {
        // the tiles with more near-threshold weights than kNearCap (rare): every wave loops over them
        for (uint32_t i = blockIdx.x * kBwdWaves + wv; i < hd.y; i += gridDim.x * kBwdWaves)
            bwd_item<true>(items[1 + hd.x + i], hd.x + i, W, H, gx, ranges, point_list, rec, bg, pix_end, n_contrib, tile_maxc, seg_off, seg_state, slot_emit, dL_dpixels, part, ks, tile_flag, near_rec, s_a, s_out);
    } else {
        const uint32_t item = blockIdx.x * kBwdWaves + wv;
        if (item >= hd.x) return;  // the launch covers the item bound
        bwd_item<false>(items[1 + item], item, W, H, gx, ranges, point_list, rec, bg, pix_end, n_contrib, tile_maxc, seg_off, seg_state, slot_emit, dL_dpixels, part, ks, tile_flag, near_rec, s_a, s_out);
    }
}

// Gradient output write: plain store, or (accumulate bit set, gsr_grads.accumulate) add into the
// caller's existing gradient -- the same single fp32 add autograd's AccumulateGrad would do.
__device__ inline void gput(float *p, size_t idx, float v, bool acc) { p[idx] = acc ? p[idx] + v : v; }
// The same with the old value fetched beforehand (old_load): the outputs a Gaussian accumulates into
// are read in one batch instead of one load -> add -> store round trip per element.
template <int N>
__device__ inline void old_load(const float *p, size_t base, bool acc, float (&o)[N]) {
#pragma unroll
    for (int k = 0; k < N; ++k) o[k] = acc ? p[base + k] : 0.f;
}
__device__ inline void gput_old(float *p, size_t idx, float v, bool acc, float old) { p[idx] = acc ? old + v : v; }

// ------------------------------------------------------------------------------------------
// Chain rule through u = v / |v|: du/dv = (|v|^2 I - v v^T) / |v|^3 applied to the gradient g.
__device__ inline float3 unit_vec_bwd(float3 v, float3 g) {
    const float n2 = v.x * v.x + v.y * v.y + v.z * v.z;
    const float inv_n3 = 1.0f / sqrtf(n2 * n2 * n2);
    return make_float3(((+n2 - v.x * v.x) * g.x - v.y * v.x * g.y - v.z * v.x * g.z) * inv_n3,
                       (-v.x * v.y * g.x + (n2 - v.y * v.y) * g.y - v.z * v.y * g.z) * inv_n3,
                       (-v.x * v.z * g.x - v.y * v.z * g.y + (n2 - v.z * v.z) * g.z) * inv_n3);
}

// SH backward; writes all M coefficient rows of dL_dsh (zeros past the active degree).  `sh` and
// `dL_dsh` may alias (the same LDS row): phase 1 reads the coefficients (direction derivative),
// phase 2 writes the coefficient gradients, which depend only on the direction and dL/dRGB.
// Phase 1 alone: dL/d(direction) = sum_c dRGB_c d(RGB_c)/d(dir) from the coefficients (before the
// normalisation's chain rule).  (x, y, z) = the unit direction.
template <typename ShPtr>
__device__ inline float3 sh_dir_grad(int deg, float x, float y, float z, ShPtr sh, const float (&dRGB)[3]) {
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    float dx[3] = {0, 0, 0}, dy[3] = {0, 0, 0}, dz[3] = {0, 0, 0};
#define SH(i, c) sh[(i) * 3 + (c)]
    // ---- phase 1: d(RGB)/d(direction) from the coefficients ----
    if (deg > 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            dx[c] = -GSR_SH_C1 * SH(3, c); dy[c] = -GSR_SH_C1 * SH(1, c); dz[c] = GSR_SH_C1 * SH(2, c);
        }
        if (deg > 1) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                dx[c] += kSH_C2[0] * y * SH(4, c) + kSH_C2[2] * 2.f * -x * SH(6, c) + kSH_C2[3] * z * SH(7, c) +
                         kSH_C2[4] * 2.f * x * SH(8, c);
                dy[c] += kSH_C2[0] * x * SH(4, c) + kSH_C2[1] * z * SH(5, c) + kSH_C2[2] * 2.f * -y * SH(6, c) +
                         kSH_C2[4] * 2.f * -y * SH(8, c);
                dz[c] += kSH_C2[1] * y * SH(5, c) + kSH_C2[2] * 2.f * 2.f * z * SH(6, c) + kSH_C2[3] * x * SH(7, c);
            }
            if (deg > 2) {
#pragma unroll
                for (int c = 0; c < 3; ++c) {
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
    return make_float3(dx[0] * dRGB[0] + dx[1] * dRGB[1] + dx[2] * dRGB[2],
                       dy[0] * dRGB[0] + dy[1] * dRGB[1] + dy[2] * dRGB[2],
                       dz[0] * dRGB[0] + dz[1] * dRGB[1] + dz[2] * dRGB[2]);
}

// The 16 SH basis values of the unit direction (x, y, z) (degree 3 and below).
__device__ inline void sh_basis16(float x, float y, float z, float (&basis)[16]) {
    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    basis[0] = GSR_SH_C0;
    basis[1] = -GSR_SH_C1 * y; basis[2] = GSR_SH_C1 * z; basis[3] = -GSR_SH_C1 * x;
    basis[4] = kSH_C2[0] * xy; basis[5] = kSH_C2[1] * yz; basis[6] = kSH_C2[2] * (2.f * zz - xx - yy);
    basis[7] = kSH_C2[3] * xz; basis[8] = kSH_C2[4] * (xx - yy);
    basis[9] = kSH_C3[0] * y * (3.f * xx - yy);
    basis[10] = kSH_C3[1] * xy * z;
    basis[11] = kSH_C3[2] * y * (4.f * zz - xx - yy);
    basis[12] = kSH_C3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy);
    basis[13] = kSH_C3[4] * x * (4.f * zz - xx - yy);
    basis[14] = kSH_C3[5] * z * (xx - yy);
    basis[15] = kSH_C3[6] * x * (xx - 3.f * yy);
}

// The SH colour's derivative with respect to the mean (returned) and the coefficient gradients
// (written to all M rows of dL_dsh, zeros past the active degree).  `sh` and `dL_dsh` may alias (the
// same LDS row): phase 1 reads the coefficients (direction derivative), phase 2 writes the
// coefficient gradients, which depend only on the direction and dL/dRGB.
template <typename ShPtr, typename OutPtr>
__device__ inline float3 sh_backward(int deg, int M, float3 mean, float3 campos, ShPtr sh,
                                     const bool *clamped, float3 dL_dcolor, OutPtr dL_dsh, bool acc = false) {
    const float3 d0 = make_float3(mean.x - campos.x, mean.y - campos.y, mean.z - campos.z);
    const float len = sqrtf(d0.x * d0.x + d0.y * d0.y + d0.z * d0.z);
    const float x = d0.x / len, y = d0.y / len, z = d0.z / len;
    const float dRGB[3] = {dL_dcolor.x * (clamped[0] ? 0.f : 1.f), dL_dcolor.y * (clamped[1] ? 0.f : 1.f),
                           dL_dcolor.z * (clamped[2] ? 0.f : 1.f)};
    const float3 dL_ddir = sh_dir_grad(deg, x, y, z, sh, dRGB);
    float basis[16];
    sh_basis16(x, y, z, basis);
    const int active = (deg + 1) * (deg + 1);
    if (dL_dsh) {  // null: the coefficients' gradient is not requested (only the mean's)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (i < M) {
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const float v = i < active ? basis[i] * dRGB[c] : 0.f;
                    dL_dsh[i * 3 + c] = acc ? dL_dsh[i * 3 + c] + v : v;
                }
            }
        }
        for (int i = 16; i < M; ++i)
            for (int c = 0; c < 3; ++c) dL_dsh[i * 3 + c] = acc ? dL_dsh[i * 3 + c] : 0.f;
    }
    return unit_vec_bwd(d0, dL_ddir);
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

// Records summed per Gaussian, staged through LDS: the 64 Gaussians of a wave own the contiguous
// record span [goff[first], goff[last + 1]) (emission order), which the wave reads in chunks of
// kRecChunk records with lane-contiguous float4 loads (a handful of lines per load instruction instead
// of one line per lane), parks in its LDS slice, and every lane then adds its own records from LDS
// in emission order -- the same additions in the same order as a direct per-lane walk.
// kRecChunk: 256 records when the SH rows' LDS slice of a wave holds them (MC = 16), else 128.
template <int MC> constexpr int kRecChunk = 3 * 256 * 16 <= 64 * sh_row_stride(MC) * 4 ? 256 : 128;
template <int MC> constexpr int kRecStageF4 = 3 * kRecChunk<MC>;  // float4 per wave slice
// A chunk of n packed records starting at record cb, as lane-contiguous float4 loads from the
// 16-byte aligned address at or below its first float: (kRecF cb) & 3 floats of lead-in.
__host__ __device__ constexpr int rec_chunk_f4(int C) { return (kRecF * C + 3 + 3) / 4; }
// A lane's records [lo, hi) of a chunk staged at `sf` (record cb at sf[0]), added into acc in
// emission order, one record per trip (2 and 4 per trip with their LDS reads issued together measured
// slower: DESIGN 2.5).
__device__ inline void add_chunk_records(const float *sf, uint32_t cb, uint32_t lo, uint32_t hi,
                                         float (&acc)[kPartial]) {
    for (uint32_t e = lo; e < hi; ++e) {
        const float *p = sf + kRecF * (e - cb);
#pragma unroll
        for (int k = 0; k < kPartial; ++k) acc[k] += p[k];
    }
}

template <int C>  // records per staged chunk (the wave's LDS slice holds 3 C float4)
__device__ inline void sum_records_span(uint32_t e0, uint32_t e1, const float4 *__restrict__ part,
                                        float4 *stage, float (&acc)[kPartial]) {
    const int lane = threadIdx.x & 63;
    const uint32_t E0 = __builtin_amdgcn_readfirstlane(e0);
    const uint32_t E1 = __builtin_amdgcn_readlane(e1, 63);
#pragma unroll
    for (int k = 0; k < kPartial; ++k) acc[k] = 0.f;
    constexpr int NL = (rec_chunk_f4(C) + 63) / 64;  // float4 loads per lane
    static_assert(64 * NL <= 3 * C, "the staged chunk fits the wave's LDS slice");
    const float *pf = reinterpret_cast<const float *>(part);
    for (uint32_t cb = E0; cb < E1; cb += C) {
        const size_t f0 = (size_t)kRecF * cb;
        const uint32_t lead = (uint32_t)(f0 & 3u);
        const uint32_t nf4 = (lead + kRecF * min((uint32_t)C, E1 - cb) + 3u) / 4u;
        const float4 *src = reinterpret_cast<const float4 *>(pf + (f0 - lead));
        float4 v[NL];
#pragma unroll
        for (int t = 0; t < NL; ++t)  // clamped index: every load in bounds, none predicated
            v[t] = src[min(lane + 64u * t, nf4 - 1u)];
#pragma unroll
        for (int t = 0; t < NL; ++t)  // unpredicated (slots past nf4 get a copy, never read):
            stage[lane + 64 * t] = v[t];  // a predicated store would sink its load into the branch
        wave_lds_sync();
        const float *sf = reinterpret_cast<const float *>(stage) + lead;
        add_chunk_records(sf, cb, max(e0, cb), min(e1, cb + C), acc);
        wave_lds_sync();
    }
}
template <int C>
__device__ inline void sum_records_chunked(int i, int P, const uint32_t *__restrict__ goff,
                                           const float4 *__restrict__ part, float4 *stage,
                                           float (&acc)[kPartial]) {
    const uint32_t e0 = goff[min(i, P)], e1 = goff[min(i + 1, P)];  // both in flight at once
    sum_records_span<C>(e0, e1, part, stage, acc);
}
template <int MC>
__device__ inline void sum_records_wave(int i, int P, const uint32_t *__restrict__ goff,
                                        const float4 *__restrict__ part, float4 *stage,
                                        float (&acc)[kPartial]) {
    sum_records_chunked<kRecChunk<MC>>(i, P, goff, part, stage, acc);
}

// dL/dconic (acc[2..4]) and dL/dmeans2D (acc[0..1]) of one view -> dL/dcov3D (dcov, upper triangle)
// and the mean's gradient through the view's Jacobian and projection (dm): SURVEY.md 2.1 rows
// computeCov2DCUDA + preprocessCUDA bwd (the SH and cov3D chains are the callers').
__device__ inline void view_chain(float3 mean, const float (&c3)[6], const float (&vm)[16], const float (&pj)[16],
                                  float tan_fovx, float tan_fovy, float h_x, float h_y,
                                  const float (&acc)[kPartial], float (&dcov)[6], float &dm0, float &dm1,
                                  float &dm2) {
    const float dcx = acc[2], dcy = acc[3], dcz = acc[4];
    float3 t = xform4x3(mean, vm);
    const float limx = 1.3f * tan_fovx, limy = 1.3f * tan_fovy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float keep_tx = txtz < -limx || txtz > limx ? 0 : 1;
    const float keep_ty = tytz < -limy || tytz > limy ? 0 : 1;
    const m3 J = {{h_x / t.z, 0.0f, -(h_x * t.x) / (t.z * t.z), 0.0f, h_y / t.z,
                   -(h_y * t.y) / (t.z * t.z), 0, 0, 0}};
    const m3 Wm = {{vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]}};
    const m3 V = {{c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]}};
    const m3 T = m3_mul(Wm, J);
    const m3 c2 = m3_mul(m3_mul(m3_T(T), m3_T(V)), T);
    const float a = GM(c2, 0, 0) + 0.3f, b = GM(c2, 0, 1), c = GM(c2, 1, 1) + 0.3f;
    const float denom = a * c - b * b;
    // upstream: every term zero when the determinant's inverse square vanishes; selects instead of a
    // branch (a branch merging the six sums kept them in scratch memory)
    const float inv_det2 = 1.0f / ((denom * denom) + 0.0000001f);
    const bool live = inv_det2 != 0;
    const float dL_da = live ? inv_det2 * (-c * c * dcx + 2 * b * c * dcy + (denom - a * c) * dcz) : 0.f;
    const float dL_dc = live ? inv_det2 * (-a * a * dcz + 2 * a * b * dcy + (denom - a * c) * dcx) : 0.f;
    const float dL_db = live ? inv_det2 * 2 * (b * c * dcx - (denom + 2 * b * b) * dcy + a * b * dcz) : 0.f;
#define TT(cc, rr) GM(T, cc, rr)
    dcov[0] = live ? (TT(0, 0) * TT(0, 0) * dL_da + TT(0, 0) * TT(1, 0) * dL_db + TT(1, 0) * TT(1, 0) * dL_dc) : 0.f;
    dcov[3] = live ? (TT(0, 1) * TT(0, 1) * dL_da + TT(0, 1) * TT(1, 1) * dL_db + TT(1, 1) * TT(1, 1) * dL_dc) : 0.f;
    dcov[5] = live ? (TT(0, 2) * TT(0, 2) * dL_da + TT(0, 2) * TT(1, 2) * dL_db + TT(1, 2) * TT(1, 2) * dL_dc) : 0.f;
    dcov[1] = live ? 2 * TT(0, 0) * TT(0, 1) * dL_da + (TT(0, 0) * TT(1, 1) + TT(0, 1) * TT(1, 0)) * dL_db +
                         2 * TT(1, 0) * TT(1, 1) * dL_dc : 0.f;
    dcov[2] = live ? 2 * TT(0, 0) * TT(0, 2) * dL_da + (TT(0, 0) * TT(1, 2) + TT(0, 2) * TT(1, 0)) * dL_db +
                         2 * TT(1, 0) * TT(1, 2) * dL_dc : 0.f;
    dcov[4] = live ? 2 * TT(0, 2) * TT(0, 1) * dL_da + (TT(0, 1) * TT(1, 2) + TT(0, 2) * TT(1, 1)) * dL_db +
                         2 * TT(1, 1) * TT(1, 2) * dL_dc : 0.f;
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
    const float dL_dtx = keep_tx * -h_x * tz2 * dJ02;
    const float dL_dty = keep_ty * -h_y * tz2 * dJ12;
    const float dL_dtz = -h_x * tz2 * dJ00 - h_y * tz2 * dJ11 + (2 * h_x * t.x) * tz3 * dJ02 +
                         (2 * h_y * t.y) * tz3 * dJ12;
    dm0 = vm[0] * dL_dtx + vm[1] * dL_dty + vm[2] * dL_dtz;
    dm1 = vm[4] * dL_dtx + vm[5] * dL_dty + vm[6] * dL_dtz;
    dm2 = vm[8] * dL_dtx + vm[9] * dL_dty + vm[10] * dL_dtz;
    // ---- screen-space mean -> means3D through the projection ----
    const float4 mh = xform4x4(mean, pj);
    const float m_w = 1.0f / (mh.w + 0.0000001f);
    const float mul1 = (pj[0] * mean.x + pj[4] * mean.y + pj[8] * mean.z + pj[12]) * m_w * m_w;
    const float mul2 = (pj[1] * mean.x + pj[5] * mean.y + pj[9] * mean.z + pj[13]) * m_w * m_w;
    const float g2x = acc[0], g2y = acc[1];
    dm0 += (pj[0] * m_w - pj[3] * mul1) * g2x + (pj[1] * m_w - pj[3] * mul2) * g2y;
    dm1 += (pj[4] * m_w - pj[7] * mul1) * g2x + (pj[5] * m_w - pj[7] * mul2) * g2y;
    dm2 += (pj[8] * m_w - pj[11] * mul1) * g2x + (pj[9] * m_w - pj[11] * mul2) * g2y;
}

// A Gaussian's inputs that k_gauss_bwd loads before its record walk (their latency overlaps it).
struct GaussIn { int radius; float3 mean, s3; float4 q; float o; };

template <int MC>
__device__ inline void gauss_bwd_one(
    int i, int D, int M, int W, int H, float scale_modifier, float tan_fovx, float tan_fovy,
    float h_x, float h_y, const float *__restrict__ means3D, const float *__restrict__ scales,
    const float *__restrict__ rotations, const float *__restrict__ shs,
    const float *__restrict__ cov3D_precomp, const float *__restrict__ viewmatrix,
    const float *__restrict__ projmatrix, const float *__restrict__ campos, CamStrides cs,
    const int *__restrict__ radii, const float (&acc)[kPartial], float *__restrict__ dL_dmeans2D,
    float *__restrict__ dL_dcolors, float *__restrict__ dL_dopacity, float *__restrict__ dL_dmeans3D,
    float *__restrict__ dL_dcov3D, float *__restrict__ dL_dsh, float *__restrict__ dL_dscales,
    float *__restrict__ dL_drot, float *s_row, int act, const float4 *__restrict__ rec, int accm,
    const uint8_t *__restrict__ clampm, const GaussIn &gi) {
    // every output may be NULL (gradient not requested: the input does not require grad); accm:
    // gsr_grad_bits of the outputs to add into instead of overwrite
    const bool a2 = accm & GSR_GRAD_MEANS2D, ac = accm & GSR_GRAD_COLORS, ao = accm & GSR_GRAD_OPACITY,
               a3 = accm & GSR_GRAD_MEANS3D, acv = accm & GSR_GRAD_COV3D, ash = accm & GSR_GRAD_SH,
               asc = accm & GSR_GRAD_SCALES, ar = accm & GSR_GRAD_ROTATIONS;
    if (!(gi.radius > 0)) {  // zero gradient: accumulated outputs keep their content
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (dL_dmeans2D && !a2) dL_dmeans2D[3 * i + k] = 0.f;
            if (dL_dmeans3D && !a3) dL_dmeans3D[3 * i + k] = 0.f;
            if (dL_dcolors && !ac) dL_dcolors[3 * i + k] = 0.f;
            if (dL_dscales && !asc) dL_dscales[3 * i + k] = 0.f;
        }
        if (dL_dopacity && !ao) dL_dopacity[i] = 0.f;
        if (dL_dcov3D && !acv) {
#pragma unroll
            for (int k = 0; k < 6; ++k) dL_dcov3D[6 * i + k] = 0.f;
        }
        if (dL_drot && !ar) {
#pragma unroll
            for (int k = 0; k < 4; ++k) dL_drot[4 * i + k] = 0.f;
        }
        if (MC > 0) {
#pragma unroll
            for (int k = 0; k < 3 * MC; ++k) s_row[k] = 0.f;
        } else if (dL_dsh && !ash) {
            for (int k = 0; k < M * 3; ++k) dL_dsh[(size_t)i * M * 3 + k] = 0.f;
        }
        return;
    }
    {   // screen-space outputs: old values (accumulation) fetched together
        float o2[3], oo[1], oc[3];
        old_load(dL_dmeans2D, 3 * (size_t)i, dL_dmeans2D && a2, o2);
        old_load(dL_dopacity, (size_t)i, dL_dopacity && ao, oo);
        old_load(dL_dcolors, 3 * (size_t)i, dL_dcolors && ac, oc);
        if (dL_dmeans2D) {
            gput_old(dL_dmeans2D, 3 * i, acc[0], a2, o2[0]); gput_old(dL_dmeans2D, 3 * i + 1, acc[1], a2, o2[1]);
            gput_old(dL_dmeans2D, 3 * i + 2, 0.f, a2, o2[2]);
        }
        // opacity = sigmoid(logit) when fused: d/dlogit = o (1 - o), o from the forward's record
        if (!dL_dopacity) {
        } else if (act & GSR_ACT_SIGMOID_OPACITY) {
            const float o = gi.o;
            gput_old(dL_dopacity, i, acc[5] * ((1.f - o) * o), ao, oo[0]);
        } else {
            gput_old(dL_dopacity, i, acc[5], ao, oo[0]);
        }
        if (dL_dcolors) {
            gput_old(dL_dcolors, 3 * i, acc[6], ac, oc[0]); gput_old(dL_dcolors, 3 * i + 1, acc[7], ac, oc[1]);
            gput_old(dL_dcolors, 3 * i + 2, acc[8], ac, oc[2]);
        }
    }
    float vm[16], pj[16];
    load_mat16(viewmatrix, cs.v0, cs.v1, vm);
    load_mat16(projmatrix, cs.p0, cs.p1, pj);
    const float3 mean = gi.mean;
    float c3[6];
    float3 s3 = make_float3(0, 0, 0);
    float4 q = make_float4(0, 0, 0, 0);
    float qn = 0.f;
    if (cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; ++k) c3[k] = cov3D_precomp[6 * i + k];
    } else {
        s3 = gi.s3;
        q = gi.q;
        if (act & GSR_ACT_EXP_SCALES) s3 = act_exp3(s3);
        if (act & GSR_ACT_NORMALIZE_ROTATIONS) { qn = quat_norm(q); q = act_normalize(q, qn); }
        cov3d_from_scale_rot(s3, scale_modifier, q, c3);
    }
    float dcov[6], dm0, dm1, dm2;
    view_chain(mean, c3, vm, pj, tan_fovx, tan_fovy, h_x, h_y, acc, dcov, dm0, dm1, dm2);
    if (dL_dcov3D) {
#pragma unroll
        for (int k = 0; k < 6; ++k) gput(dL_dcov3D, 6 * i + k, dcov[k], acv);
    }
    if (MC > 0) {
        bool cl[3];
        const float3 cp = load_campos(campos, cs.c0);
        clamp_from_mask(clampm[i], cl);  // the forward's clamp mask
        const float3 d = sh_backward(D, MC, mean, cp, s_row, cl, make_float3(acc[6], acc[7], acc[8]), s_row);
        dm0 += d.x; dm1 += d.y; dm2 += d.z;
    } else if (shs) {
        const float *sh = shs + (size_t)i * M * 3;
        bool cl[3];
        const float3 cp = load_campos(campos, cs.c0);
        clamp_from_mask(clampm[i], cl);
        const float3 d = sh_backward(D, M, mean, cp, sh, cl, make_float3(acc[6], acc[7], acc[8]),
                                     dL_dsh ? dL_dsh + (size_t)i * M * 3 : nullptr, ash);
        dm0 += d.x; dm1 += d.y; dm2 += d.z;
    } else if (dL_dsh) {
        if (!ash) for (int k = 0; k < M * 3; ++k) dL_dsh[(size_t)i * M * 3 + k] = 0.f;
    }
    const bool has_sr = scales && !cov3D_precomp;
    float o3[3], os[3], orr[4];  // old values of the remaining accumulated outputs, fetched together
    old_load(dL_dmeans3D, 3 * (size_t)i, dL_dmeans3D && a3, o3);
    old_load(dL_dscales, 3 * (size_t)i, has_sr && dL_dscales && asc, os);
    old_load(dL_drot, 4 * (size_t)i, has_sr && dL_drot && ar, orr);
    if (dL_dmeans3D) {
        gput_old(dL_dmeans3D, 3 * i, dm0, a3, o3[0]); gput_old(dL_dmeans3D, 3 * i + 1, dm1, a3, o3[1]);
        gput_old(dL_dmeans3D, 3 * i + 2, dm2, a3, o3[2]);
    }
    if (has_sr) {
        float3 ds; float4 dr;
        cov3d_backward(s3, scale_modifier, q, dcov, ds, dr);
        if (act & GSR_ACT_EXP_SCALES) { ds.x *= s3.x; ds.y *= s3.y; ds.z *= s3.z; }
        if (act & GSR_ACT_NORMALIZE_ROTATIONS) dr = act_normalize_bwd(q, qn, dr);
        if (dL_dscales) {
            gput_old(dL_dscales, 3 * i, ds.x, asc, os[0]); gput_old(dL_dscales, 3 * i + 1, ds.y, asc, os[1]);
            gput_old(dL_dscales, 3 * i + 2, ds.z, asc, os[2]);
        }
        if (dL_drot) {
            gput_old(dL_drot, 4 * i, dr.x, ar, orr[0]); gput_old(dL_drot, 4 * i + 1, dr.y, ar, orr[1]);
            gput_old(dL_drot, 4 * i + 2, dr.z, ar, orr[2]); gput_old(dL_drot, 4 * i + 3, dr.w, ar, orr[3]);
        }
    } else {
        if (dL_dscales && !asc) { dL_dscales[3 * i] = 0.f; dL_dscales[3 * i + 1] = 0.f; dL_dscales[3 * i + 2] = 0.f; }
        if (dL_drot && !ar) { dL_drot[4 * i] = 0.f; dL_drot[4 * i + 1] = 0.f; dL_drot[4 * i + 2] = 0.f; dL_drot[4 * i + 3] = 0.f; }
    }
}

template <int MC>  // SH coefficient count staged through LDS (0: direct global access / no SH)
__global__ __launch_bounds__(256) void k_gauss_bwd(
    int P, int D, int M, int W, int H, float scale_modifier, float tan_fovx, float tan_fovy,
    float h_x, float h_y, const float *__restrict__ means3D, const float *__restrict__ scales,
    const float *__restrict__ rotations, const float *__restrict__ shs,
    const float *__restrict__ cov3D_precomp, const float *__restrict__ viewmatrix,
    const float *__restrict__ projmatrix, const float *__restrict__ campos, CamStrides cs,
    const int *__restrict__ radii, const uint32_t *__restrict__ goff,
    const float4 *__restrict__ part, float *__restrict__ dL_dmeans2D,
    float *__restrict__ dL_dcolors, float *__restrict__ dL_dopacity, float *__restrict__ dL_dmeans3D,
    float *__restrict__ dL_dcov3D, float *__restrict__ dL_dsh, float *__restrict__ dL_dscales,
    float *__restrict__ dL_drot, int act, const float4 *__restrict__ rec, int accm,
    const uint8_t *__restrict__ clampm) {
    extern __shared__ __attribute__((aligned(16))) float s_sh[];
    constexpr int RL = 3 * MC, RS = sh_row_stride(MC);
    const int i0 = blockIdx.x * kShBlock;
    const int nrow = min(kShBlock, P - i0);
    const int i = i0 + threadIdx.x;
    // the Gaussian's radius, parameters and activated opacity are loaded first (clamped index for the
    // tail lanes), so their latency overlaps the record walk instead of following it
    const int ic = min(i, P - 1);
    GaussIn gi;
    gi.radius = radii[ic];
    gi.mean = make_float3(means3D[3 * ic], means3D[3 * ic + 1], means3D[3 * ic + 2]);
    gi.s3 = make_float3(0.f, 0.f, 0.f);
    gi.q = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!cov3D_precomp) {
        gi.s3 = make_float3(scales[3 * ic], scales[3 * ic + 1], scales[3 * ic + 2]);
        gi.q = make_float4(rotations[4 * ic], rotations[4 * ic + 1], rotations[4 * ic + 2], rotations[4 * ic + 3]);
    }
    gi.o = (act & GSR_ACT_SIGMOID_OPACITY) && dL_dopacity ? rec[(size_t)kRecF4 * ic + 1].y : 0.f;
    // the record sums, each wave in its own slice of the block's LDS (which the SH rows reuse)
    float acc[kPartial];
    sum_records_wave<MC>(i, P, goff, part, reinterpret_cast<float4 *>(s_sh) + (threadIdx.x >> 6) * kRecStageF4<MC>, acc);
    if constexpr (MC > 0) {  // coalesced copy of this block's SH rows into LDS (reused for dL/dSH)
        __syncthreads();
        sh_rows_to_lds<MC>(shs + (size_t)i0 * RL, nrow, s_sh);
        __syncthreads();
    }
    if (i < P) gauss_bwd_one<MC>(i, D, M, W, H, scale_modifier, tan_fovx, tan_fovy, h_x, h_y, means3D,
                                 scales, rotations, shs, cov3D_precomp, viewmatrix, projmatrix, campos, cs,
                                 radii, acc, dL_dmeans2D, dL_dcolors, dL_dopacity,
                                 dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drot, s_sh + threadIdx.x * RS,
                                 act, rec, accm, clampm, gi);
    if constexpr (MC > 0) {  // coalesced store of the dL/dSH rows
        if (!dL_dsh) return;
        __syncthreads();
        if (accm & GSR_GRAD_SH) sh_rows_from_lds<MC, true>(s_sh, nrow, dL_dsh + (size_t)i0 * RL);
        else sh_rows_from_lds<MC, false>(s_sh, nrow, dL_dsh + (size_t)i0 * RL);
    }
}

// ---- per-view record sums (gsr_backward_render, deferred views) ---------------------------------
// One thread per Gaussian, its wave's record span staged through LDS in 128-record chunks
// (sum_records_span: lane-contiguous coalesced loads, each lane adding its own records in emission
// order -- the same additions in the same order as k_gauss_bwd's walk), stored as kPartial x P SoA:
// the multi-view pass then reads 9 coalesced words per Gaussian and view.  Few registers and 6 KB
// of LDS per wave, so the walk's LDS round trips hide behind other waves; it runs on the view's
// stream right after k_render_bwd, beside the other views' render kernels.
constexpr int kSumChunk = 128;
// The view's camera key (FNV-1a over the bits of its view matrix, projection matrix, camera position and
// image size), stored after the sums: k_gauss_bwd_multi orders a launch's views by it (view_order).  Two
// views of one launch with the same key -- the same camera rendered twice, e.g. two timesteps of one
// pose -- keep the order the backward pass queued them in (include/gsr.h, gsr_backward_gaussians).
__device__ inline uint32_t camera_key(const float *viewmatrix, const float *projmatrix, const float *campos,
                                      CamStrides cs, int W, int H) {
    float vm[16], pj[16];
    load_mat16(viewmatrix, cs.v0, cs.v1, vm);
    load_mat16(projmatrix, cs.p0, cs.p1, pj);
    const float3 cp = load_campos(campos, cs.c0);
    uint32_t x = 2166136261u;
    auto mix = [&x](uint32_t w) { x = (x ^ w) * 16777619u; };
#pragma unroll
    for (int k = 0; k < 16; ++k) mix(__float_as_uint(vm[k]));
#pragma unroll
    for (int k = 0; k < 16; ++k) mix(__float_as_uint(pj[k]));
    mix(__float_as_uint(cp.x)); mix(__float_as_uint(cp.y)); mix(__float_as_uint(cp.z));
    mix((uint32_t)W); mix((uint32_t)H);
    return x;
}
__global__ __launch_bounds__(256) void k_sum_records(int P, const uint32_t *__restrict__ goff,
                                                     const float4 *__restrict__ part, float *__restrict__ sums,
                                                     const uint32_t *__restrict__ spec_ok, const float *viewmatrix,
                                                     const float *projmatrix, const float *campos, CamStrides cs,
                                                     int W, int H) {
    __shared__ float4 s_stage[3 * kSumChunk * 4];
    if (spec_ok && *spec_ok == 0u) return;  // (as k_render_bwd)
    if (blockIdx.x == 0 && threadIdx.x == 0)
        reinterpret_cast<uint32_t *>(sums)[(size_t)kPartial * P] = camera_key(viewmatrix, projmatrix, campos, cs, W, H);
    const int i = blockIdx.x * 256 + threadIdx.x;
    float acc[kPartial];
    sum_records_chunked<kSumChunk>(i, P, goff, part, s_stage + (threadIdx.x >> 6) * 3 * kSumChunk, acc);
    if (i < P) {
#pragma unroll
        for (int k = 0; k < kPartial; ++k) sums[(size_t)k * P + i] = acc[k];
    }
}

// ---- the per-Gaussian backward of several views in one pass (gsr_backward_gaussians) -----------
// A training step's views (train.py:753-767 sums 5 view losses before ONE backward) share every
// parameter and gradient array: one thread per Gaussian reads its parameters and SH row once, walks
// the views -- each view's records summed from its own SCRATCH (staged per wave as in k_gauss_bwd),
// its cov2D / projection / SH chains with its own camera -- and keeps the running sums of the
// per-Gaussian gradients in registers (dL/dcov3D is summed before the single cov3D -> scale /
// rotation chain: that chain is linear in it), then adds them into the gradient arrays ONCE.
// Against one k_gauss_bwd per view this removes (V - 1) reads of the parameters and (V - 1)
// read-modify-writes of every gradient array: at SH3 ~ 0.6 KB of HBM traffic per Gaussian per view.
// Per view the screen-space gradient goes to that view's own dL/dmeans2D array.
#define GSR_MV_ATTR  // (the compiler's register budget: 4 waves/SIMD spilled)
template <int MC>
constexpr size_t multi_sh_floats() { return MC ? (((size_t)kShBlock * sh_row_stride(MC) + 3) & ~size_t(3)) : 0; }
template <int MC>
constexpr size_t multi_lds_bytes() { return sizeof(float) * multi_sh_floats<MC>(); }

// The order the launch sums its views in: fixed by their cameras -- the key
// k_sum_records stored after each view's sums (a hash of its view matrix and camera position), ties (the
// same camera twice) in queue order -- not by the order the backward pass queued them, so a caller whose
// threads finish their forwards in a varying order gets the same gradients bit for bit.  Position t's
// view is bits 4t..4t+3.  Wave-uniform: nv scalar loads and scalar compares.
static_assert(kMultiViews <= 8, "view order packed 4 bits per position");
__device__ inline uint32_t view_order(const MultiArgs &a) {
    typedef const __attribute__((address_space(4))) uint32_t *key_ptr;
    uint32_t h[kMultiViews];
#pragma unroll
    for (int u = 0; u < kMultiViews; ++u) h[u] = u < a.nv ? ((key_ptr)a.v[u].sums)[(size_t)kPartial * a.P] : 0u;
    uint32_t ord = 0;
#pragma unroll
    for (int u = 0; u < kMultiViews; ++u) {
        int rank = 0;
#pragma unroll
        for (int w = 0; w < kMultiViews; ++w) rank += (w < a.nv && (h[w] < h[u] || (h[w] == h[u] && w < u))) ? 1 : 0;
        if (u < a.nv) ord |= (uint32_t)u << (4 * rank);
    }
    return ord;
}

template <int MC>  // SH coefficient count (1, 4, 9, 16), or 0 without SH (colours precomputed)
__global__ __launch_bounds__(kShBlock) GSR_MV_ATTR void k_gauss_bwd_multi(const MultiArgs a) {
    extern __shared__ __attribute__((aligned(16))) float s_sh[];
    constexpr int RL = 3 * MC, RS = sh_row_stride(MC);
    const int P = a.P;
    const int i0 = blockIdx.x * kShBlock;
    const int nrow = min(kShBlock, P - i0);
    const int i = i0 + threadIdx.x;
    const bool live = i < P;
    const int ii = live ? i : i0;  // lanes past P load (and never store) row i0's parameters
    float *s_row = s_sh + threadIdx.x * RS;
    const uint32_t ord = view_order(a);
    auto vid = [ord](int t) { return (int)((ord >> (4 * t)) & 15u); };  // the view summed t-th
    // the Gaussian's own parameters and the first view's record sums and radius are loaded before the
    // SH row copy, so that their latency overlaps it instead of following its barrier
    const float3 mean = make_float3(a.means3D[3 * ii], a.means3D[3 * ii + 1], a.means3D[3 * ii + 2]);
    float c3[6];
    float3 s3 = make_float3(0, 0, 0);
    float4 q = make_float4(0, 0, 0, 0);
    float qn = 0.f;
    if (a.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; ++k) c3[k] = a.cov3D_precomp[6 * ii + k];
    } else {
        s3 = make_float3(a.scales[3 * ii], a.scales[3 * ii + 1], a.scales[3 * ii + 2]);
        q = make_float4(a.rotations[4 * ii], a.rotations[4 * ii + 1], a.rotations[4 * ii + 2], a.rotations[4 * ii + 3]);
    }
    // each view's record sums (gsr_backward_render's k_sum_records, kPartial x P SoA: coalesced) and
    // radius are loaded one view ahead, so their latency hides behind the previous view's chains
    float nx[kPartial];
#pragma unroll
    for (int k = 0; k < kPartial; ++k) nx[k] = a.v[vid(0)].sums[(size_t)k * P + ii];
    int rn = a.v[vid(0)].radii[ii];
    if constexpr (MC > 0) {  // coefficient rows, read by every view's SH chain
        sh_rows_to_lds<MC>(a.shs + (size_t)i0 * RL, nrow, s_sh);
        __syncthreads();
    }
    if (!a.cov3D_precomp) {
        if (a.act & GSR_ACT_EXP_SCALES) s3 = act_exp3(s3);
        if (a.act & GSR_ACT_NORMALIZE_ROTATIONS) { qn = quat_norm(q); q = act_normalize(q, qn); }
        cov3d_from_scale_rot(s3, a.scale_modifier, q, c3);
    }
    float gm0 = 0.f, gm1 = 0.f, gm2 = 0.f, gop = 0.f, gc0 = 0.f, gc1 = 0.f, gc2 = 0.f;
    float gcov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    bool vis = false;
    float o_act = 0.f;  // the activated opacity, from the record of a view that sees the Gaussian
    float m2[3] = {0.f, 0.f, 0.f};  // the screen-space gradient carried across views of one array
    bool m2_have = false;            // m2 holds a value (else the next view's gradient starts it)
    const int active = (a.D + 1) * (a.D + 1);
    for (int t = 0; t < a.nv; ++t) {
        const MultiView &V = a.v[vid(t)];
        const int rv = rn;
        float acc[kPartial];
#pragma unroll
        for (int k = 0; k < kPartial; ++k) acc[k] = nx[k];
        if (t + 1 < a.nv) {
            const MultiView &Vn = a.v[vid(t + 1)];
#pragma unroll
            for (int k = 0; k < kPartial; ++k) nx[k] = Vn.sums[(size_t)k * P + ii];
            rn = Vn.radii[ii];
        }
        if (!live) continue;
        const bool r = rv > 0;
        if (V.dL_dmeans2D) {
            // consecutive views writing the same array (one means2D leaf rendered from several
            // cameras) carry its value in registers: loaded at the run's first view, stored after its
            // last -- the same additions, in view order, as a read-modify-write per view.  An array some
            // view of the launch overwrites (a fresh .grad) starts empty at its first view in the
            // summing order; a later run of it reloads what the earlier one stored.
            const float *X = V.dL_dmeans2D;
            const bool cont = t > 0 && a.v[vid(t - 1)].dL_dmeans2D == X;
            const bool last = !(t + 1 < a.nv && a.v[vid(t + 1)].dL_dmeans2D == X);
            const float gx = r ? acc[0] : 0.f, gy = r ? acc[1] : 0.f;
            if (!cont) {
                bool first = true, accx = true;  // (wave-uniform scans of the launch's views)
                for (int u = 0; u < a.nv; ++u)
                    if (a.v[u].dL_dmeans2D == X) accx = accx && a.v[u].acc2;
                for (int u = 0; u < t; ++u)
                    if (a.v[vid(u)].dL_dmeans2D == X) first = false;
                m2_have = !(first && !accx);
                if (m2_have) old_load(V.dL_dmeans2D, 3 * (size_t)i, true, m2);
            }
            m2[0] = m2_have ? m2[0] + gx : gx;
            m2[1] = m2_have ? m2[1] + gy : gy;
            m2[2] = m2_have ? m2[2] + 0.f : 0.f;
            m2_have = true;
            if (last) {
                V.dL_dmeans2D[3 * i] = m2[0]; V.dL_dmeans2D[3 * i + 1] = m2[1]; V.dL_dmeans2D[3 * i + 2] = m2[2];
            }
        }
        if (!r) continue;
        // the activated opacity (sigmoid chain only): written by every view that sees the Gaussian
        if (!vis && (a.act & GSR_ACT_SIGMOID_OPACITY)) o_act = V.rec[(size_t)kRecF4 * i + 1].y;
        vis = true;
        gop += acc[5]; gc0 += acc[6]; gc1 += acc[7]; gc2 += acc[8];
        float vm[16], pj[16];
        load_mat16(V.viewmatrix, V.cs.v0, V.cs.v1, vm);
        load_mat16(V.projmatrix, V.cs.p0, V.cs.p1, pj);
        float dcov[6], dm0, dm1, dm2;
        view_chain(mean, c3, vm, pj, V.tan_fovx, V.tan_fovy, V.focal_x, V.focal_y, acc, dcov, dm0, dm1, dm2);
#pragma unroll
        for (int k = 0; k < 6; ++k) gcov[k] += dcov[k];
        if constexpr (MC > 0) {
            const float3 cp = load_campos(V.campos, V.cs.c0);
            bool cl[3];
            clamp_from_mask(V.clampm[i], cl);  // the forward's clamp mask in this view
            const float3 d0 = make_float3(mean.x - cp.x, mean.y - cp.y, mean.z - cp.z);
            const float len = sqrtf(d0.x * d0.x + d0.y * d0.y + d0.z * d0.z);
            const float x = d0.x / len, y = d0.y / len, z = d0.z / len;
            const float dRGB[3] = {acc[6] * (cl[0] ? 0.f : 1.f), acc[7] * (cl[1] ? 0.f : 1.f),
                                   acc[8] * (cl[2] ? 0.f : 1.f)};
            const float3 d = unit_vec_bwd(d0, sh_dir_grad(a.D, x, y, z, s_row, dRGB));
            dm0 += d.x; dm1 += d.y; dm2 += d.z;
        }
        gm0 += dm0; gm1 += dm1; gm2 += dm2;
    }
    if (live) {
        const int accm = a.accm;
        const bool ac = accm & GSR_GRAD_COLORS, ao = accm & GSR_GRAD_OPACITY, a3 = accm & GSR_GRAD_MEANS3D,
                   acv = accm & GSR_GRAD_COV3D, asc = accm & GSR_GRAD_SCALES, ar = accm & GSR_GRAD_ROTATIONS;
        if (!vis) {  // no view sees it: zero gradient, accumulated outputs keep their content
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                if (a.dL_dmeans3D && !a3) a.dL_dmeans3D[3 * i + k] = 0.f;
                if (a.dL_dcolors && !ac) a.dL_dcolors[3 * i + k] = 0.f;
                if (a.dL_dscales && !asc) a.dL_dscales[3 * i + k] = 0.f;
            }
            if (a.dL_dopacity && !ao) a.dL_dopacity[i] = 0.f;
            if (a.dL_dcov3D && !acv) {
#pragma unroll
                for (int k = 0; k < 6; ++k) a.dL_dcov3D[6 * i + k] = 0.f;
            }
            if (a.dL_drot && !ar) {
#pragma unroll
                for (int k = 0; k < 4; ++k) a.dL_drot[4 * i + k] = 0.f;
            }
        } else {
            float oo[1], oc[3], o3[3];
            old_load(a.dL_dopacity, (size_t)i, a.dL_dopacity && ao, oo);
            old_load(a.dL_dcolors, 3 * (size_t)i, a.dL_dcolors && ac, oc);
            old_load(a.dL_dmeans3D, 3 * (size_t)i, a.dL_dmeans3D && a3, o3);
            if (!a.dL_dopacity) {
            } else if (a.act & GSR_ACT_SIGMOID_OPACITY) {  // d/dlogit = o (1 - o), o from a forward's record
                gput_old(a.dL_dopacity, i, gop * ((1.f - o_act) * o_act), ao, oo[0]);
            } else {
                gput_old(a.dL_dopacity, i, gop, ao, oo[0]);
            }
            if (a.dL_dcolors) {
                gput_old(a.dL_dcolors, 3 * i, gc0, ac, oc[0]); gput_old(a.dL_dcolors, 3 * i + 1, gc1, ac, oc[1]);
                gput_old(a.dL_dcolors, 3 * i + 2, gc2, ac, oc[2]);
            }
            if (a.dL_dmeans3D) {
                gput_old(a.dL_dmeans3D, 3 * i, gm0, a3, o3[0]); gput_old(a.dL_dmeans3D, 3 * i + 1, gm1, a3, o3[1]);
                gput_old(a.dL_dmeans3D, 3 * i + 2, gm2, a3, o3[2]);
            }
            if (a.dL_dcov3D) {
#pragma unroll
                for (int k = 0; k < 6; ++k) gput(a.dL_dcov3D, 6 * i + k, gcov[k], acv);
            }
            const bool has_sr = a.scales && !a.cov3D_precomp;
            if (has_sr) {
                float os[3], orr[4];
                old_load(a.dL_dscales, 3 * (size_t)i, a.dL_dscales && asc, os);
                old_load(a.dL_drot, 4 * (size_t)i, a.dL_drot && ar, orr);
                float3 ds; float4 dr;
                cov3d_backward(s3, a.scale_modifier, q, gcov, ds, dr);
                if (a.act & GSR_ACT_EXP_SCALES) { ds.x *= s3.x; ds.y *= s3.y; ds.z *= s3.z; }
                if (a.act & GSR_ACT_NORMALIZE_ROTATIONS) dr = act_normalize_bwd(q, qn, dr);
                if (a.dL_dscales) {
                    gput_old(a.dL_dscales, 3 * i, ds.x, asc, os[0]); gput_old(a.dL_dscales, 3 * i + 1, ds.y, asc, os[1]);
                    gput_old(a.dL_dscales, 3 * i + 2, ds.z, asc, os[2]);
                }
                if (a.dL_drot) {
                    gput_old(a.dL_drot, 4 * i, dr.x, ar, orr[0]); gput_old(a.dL_drot, 4 * i + 1, dr.y, ar, orr[1]);
                    gput_old(a.dL_drot, 4 * i + 2, dr.z, ar, orr[2]); gput_old(a.dL_drot, 4 * i + 3, dr.w, ar, orr[3]);
                }
            } else {
                if (a.dL_dscales && !asc) { a.dL_dscales[3 * i] = 0.f; a.dL_dscales[3 * i + 1] = 0.f; a.dL_dscales[3 * i + 2] = 0.f; }
                if (a.dL_drot && !ar) { a.dL_drot[4 * i] = 0.f; a.dL_drot[4 * i + 1] = 0.f; a.dL_drot[4 * i + 2] = 0.f; a.dL_drot[4 * i + 3] = 0.f; }
            }
        }
    }
    if constexpr (MC > 0) {
        // dL/dSH = sum over the views of basis(dir_v) x dRGB_v, summed in the lane's own LDS row: the
        // coefficients it held are no longer read (every view's direction gradient is done), and the
        // 3 MC sums stay out of the registers the view loop needs (4 -> 3 waves/SIMD at SH3).  Same
        // additions in the same order as running sums over the views.  dRGB_v is reloaded from the
        // view's sums, the clamp mask and direction recomputed as in the loop.
        if (!a.dL_dsh) return;
        if (live) {
#pragma unroll
            for (int k = 0; k < RL; ++k) s_row[k] = 0.f;
            // a view's radius, clamp mask and colour sums are loaded together (none waits for the
            // radius) and one view ahead, so the loop pays one load latency instead of two per view
            const MultiView &V0 = a.v[vid(0)];
            int rv_n = V0.radii[i];
            uint8_t cm_n = V0.clampm[i];
            float g_n[3] = {V0.sums[(size_t)6 * P + i], V0.sums[(size_t)7 * P + i], V0.sums[(size_t)8 * P + i]};
            for (int t = 0; t < a.nv; ++t) {
                const MultiView &V = a.v[vid(t)];
                const int rv = rv_n;
                const uint8_t cm = cm_n;
                const float g[3] = {g_n[0], g_n[1], g_n[2]};
                if (t + 1 < a.nv) {
                    const MultiView &Vn = a.v[vid(t + 1)];
                    rv_n = Vn.radii[i];
                    cm_n = Vn.clampm[i];
#pragma unroll
                    for (int c = 0; c < 3; ++c) g_n[c] = Vn.sums[(size_t)(6 + c) * P + i];
                }
                if (!(rv > 0)) continue;
                const float3 cp = load_campos(V.campos, V.cs.c0);
                bool cl[3];
                clamp_from_mask(cm, cl);
                const float3 d0 = make_float3(mean.x - cp.x, mean.y - cp.y, mean.z - cp.z);
                const float len = sqrtf(d0.x * d0.x + d0.y * d0.y + d0.z * d0.z);
                const float x = d0.x / len, y = d0.y / len, z = d0.z / len;
                const float dRGB[3] = {g[0] * (cl[0] ? 0.f : 1.f), g[1] * (cl[1] ? 0.f : 1.f), g[2] * (cl[2] ? 0.f : 1.f)};
                float basis[16];
                sh_basis16(x, y, z, basis);
#pragma unroll
                for (int k = 0; k < MC; ++k)
                    if (k < active) {
#pragma unroll
                        for (int c = 0; c < 3; ++c) s_row[3 * k + c] += basis[k] * dRGB[c];
                    }
            }
        }
        __syncthreads();
        if (a.accm & GSR_GRAD_SH) sh_rows_from_lds<MC, true>(s_sh, nrow, a.dL_dsh + (size_t)i0 * RL);
        else sh_rows_from_lds<MC, false>(s_sh, nrow, a.dL_dsh + (size_t)i0 * RL);
    }
}


// ==========================================================================================
hipError_t launch_bwd_items_raw(int K, int T, int P, const uint2 *ranges, const uint32_t *tile_maxc,
                                const uint32_t *tile_flag, uint2 *items, uint32_t *ws, hipStream_t s,
                                const uint32_t *spec_ok) {
    if (K == 0) return hipSuccess;
    const int nb = div_up(T, kItemsBlock);
    k_items_count<<<nb, kItemsBlock, 0, s>>>(T, ranges, tile_maxc, tile_flag, items, ws, spec_ok, seg_log2(P));
    k_items_emit<<<nb, kItemsBlock, 0, s>>>(T, ranges, tile_maxc, tile_flag, items, ws, spec_ok, seg_log2(P));
    return hipGetLastError();
}
hipError_t launch_bwd_items(const BwdArgs &a, hipStream_t s) {
    return launch_bwd_items_raw(a.K, a.gx * a.gy, a.P, a.ranges, a.tile_maxc, a.tile_flag, a.items, a.items_ws, s);
}

hipError_t launch_render_bwd(const BwdArgs &a, hipStream_t s) {
    if (a.K == 0) return hipSuccess;
    // one wave per item, kBwdWaves per workgroup; the launch covers the item bound, waves without an
    // item exit at once.  Then the items of the tiles whose near-threshold records overflowed (tile_flag
    // > kNearCap; none when the exact-threshold mode is off) on a small grid that loops over their
    // device-side count.
    const int ks = seg_log2(a.P);
    k_render_bwd<false><<<div_up((int)a.max_items, kBwdWaves), 64 * kBwdWaves, 0, s>>>(
        a.W, a.H, a.gx, a.items, a.ranges, a.point_list, a.rec, a.bg, a.pix_end, a.n_contrib, a.tile_maxc, a.seg_off,
        a.seg_state, a.slot_emit, a.dL_dcolor, a.part, ks, a.spec_ok, a.tile_flag, a.near_rec);
    k_render_bwd<true><<<std::min(div_up((int)a.max_items, kBwdWaves), kExactBwdBlocks), 64 * kBwdWaves, 0, s>>>(
        a.W, a.H, a.gx, a.items, a.ranges, a.point_list, a.rec, a.bg, a.pix_end, a.n_contrib, a.tile_maxc, a.seg_off,
        a.seg_state, a.slot_emit, a.dL_dcolor, a.part, ks, a.spec_ok, a.tile_flag, a.near_rec);
    return hipGetLastError();
}

template <int MC>
static void gauss_bwd_mc(const BwdArgs &a, hipStream_t s) {
    constexpr size_t lds = std::max(sizeof(float) * kShBlock * (MC ? sh_row_stride(MC) : 0),
                                    sizeof(float4) * kRecStageF4<MC> * (kShBlock / 64));
    k_gauss_bwd<MC><<<div_up(a.P, kShBlock), kShBlock, lds, s>>>(
        a.P, a.D, a.M, a.W, a.H, a.scale_modifier, a.tan_fovx, a.tan_fovy, a.focal_x, a.focal_y,
        a.means3D, a.scales, a.rotations, a.shs, a.cov3D_precomp, a.viewmatrix, a.projmatrix, a.campos, a.cs,
        a.radii, a.goff, a.part, a.dL_dmeans2D, a.dL_dcolors, a.dL_dopacity,
        a.dL_dmeans3D, a.dL_dcov3D, a.dL_dsh, a.dL_dscales, a.dL_drot, a.act, a.rec, a.accm, a.clampm);
}

hipError_t launch_gauss_bwd(const BwdArgs &a, hipStream_t s) {
    if (a.P == 0) return hipSuccess;
    switch (a.shs ? a.M : 0) {
        case 16: gauss_bwd_mc<16>(a, s); break;
        case 9: gauss_bwd_mc<9>(a, s); break;
        case 4: gauss_bwd_mc<4>(a, s); break;
        case 1: gauss_bwd_mc<1>(a, s); break;
        default: gauss_bwd_mc<0>(a, s); break;
    }
    return hipGetLastError();
}

template <int MC>
static void gauss_bwd_multi_mc(const MultiArgs &a, hipStream_t s) {
    k_gauss_bwd_multi<MC><<<div_up(a.P, kShBlock), kShBlock, multi_lds_bytes<MC>(), s>>>(a);
}

hipError_t launch_sum_records(int P, const uint32_t *goff, const float4 *part, float *sums, hipStream_t s,
                              const uint32_t *spec_ok, const float *viewmatrix, const float *projmatrix,
                              const float *campos, CamStrides cs, int W, int H) {
    if (P == 0) return hipSuccess;
    k_sum_records<<<div_up(P, 256), 256, 0, s>>>(P, goff, part, sums, spec_ok, viewmatrix, projmatrix, campos, cs,
                                                 W, H);
    return hipGetLastError();
}

hipError_t launch_gauss_bwd_multi(const MultiArgs &a, hipStream_t s) {
    if (a.P == 0 || a.nv == 0) return hipSuccess;
    switch (a.shs ? a.M : 0) {  // the caller checked M in {1, 4, 9, 16} when shs are given
        case 16: gauss_bwd_multi_mc<16>(a, s); break;
        case 9: gauss_bwd_multi_mc<9>(a, s); break;
        case 4: gauss_bwd_multi_mc<4>(a, s); break;
        case 1: gauss_bwd_multi_mc<1>(a, s); break;
        default: gauss_bwd_multi_mc<0>(a, s); break;
    }
    return hipGetLastError();
}

}  // namespace gsr

#ifdef GSR_TRACE
extern "C" int gsr_debug_trace_bwd(void *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(gsr::g_trace_bwd), &buf, sizeof(buf)) == hipSuccess ? 0 : 2;
}
#endif
