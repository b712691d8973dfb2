// gsr_api.hip -- C ABI of libgsr (declared in include/gsr.h).
//
// Host-side orchestration of the forward/backward kernel pipelines: argument validation with the
// reference's error behaviour, workspace carving, the single num_rendered read-back per forward,
// per-phase HIP-event timing, and a thread-local error string.  Mirrors the reference's
// rasterize_points.cu glue + CudaRasterizer::Rasterizer::{forward,backward}.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <chrono>
#include <condition_variable>
#include <thread>
#include <map>
#include <memory>
#include <unordered_map>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gsr.h"
#include "gsr_common.h"
#include "gsr_internal.h"

using namespace gsr;


namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e__ = (expr);                                                               \
        if (e__ != hipSuccess) return fail(GSR_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e__)); \
    } while (0)

// ---- per-phase event profiling ----
struct ProfRec { std::string phase; hipEvent_t a, b; };
std::mutex g_prof_mu;
bool g_prof_on = false;
std::string g_prof_sel;  // ",a,b," filter; empty = every phase
std::vector<ProfRec> g_prof;
std::vector<hipEvent_t> g_evpool;
std::map<std::string, double> g_host_ms;
std::map<std::string, int> g_host_n;

hipEvent_t ev_get() {
    if (!g_evpool.empty()) { hipEvent_t e = g_evpool.back(); g_evpool.pop_back(); return e; }
    hipEvent_t e = nullptr;
    // timing only: no system-scope fence (its L2 writeback + invalidate would also slow the kernel
    // that follows the event, and the host reads the events after a stream synchronisation anyway)
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
    return e;
}

struct Phase {
    hipStream_t s; const char *name; hipEvent_t a = nullptr, b = nullptr;
    Phase(hipStream_t s_, const char *n) : s(s_), name(n) {
        if (!g_prof_on) return;
        std::lock_guard<std::mutex> lk(g_prof_mu);
        if (!g_prof_sel.empty() && g_prof_sel.find("," + std::string(n) + ",") == std::string::npos) return;
        a = ev_get(); b = ev_get();
        if (a) (void)hipEventRecord(a, s);
    }
    ~Phase() {
        if (!a || !b) return;
        (void)hipEventRecord(b, s);
        std::lock_guard<std::mutex> lk(g_prof_mu);
        g_prof.push_back({name, a, b});
    }
};

// Cross-stream order of the gradient writes.  A caller may render its views on several HIP streams
// (bench.py --streams, splat_train) so one view's memory-bound k_gauss_bwd overlaps another view's
// VALU-bound render kernels; the views' gradients still land in the same buffers.  Every gradient
// output pointer a k_gauss_bwd writes is tracked with the stream and event of its last writer; the
// next write of ANY of those pointers from another stream waits for that event first.  Additions then
// happen in call order and the result is bitwise the single-stream one.  Same-stream writes add no
// wait (stream order already holds).  Entries are dropped only once their event has completed (a
// later writer then has nothing to wait for), so no pending write is ever forgotten, however many
// gradient sets are in flight.
std::vector<hipEvent_t> g_gw_evpool;  // (g_gw_mu) events of dropped entries, re-recorded by later writes
struct GradEvent {
    hipEvent_t ev = nullptr;
    ~GradEvent() { if (ev) g_gw_evpool.push_back(ev); }  // destroyed under g_gw_mu (table updates)
};
struct GradWriter { hipStream_t s = nullptr; std::shared_ptr<GradEvent> ev; };
std::mutex g_gw_mu;
std::unordered_map<const void *, GradWriter> g_gw;
constexpr size_t kGradPruneAt = 1024;  // scan for completed entries when the table grows past this

hipError_t no_launch() { return hipSuccess; }

template <typename Launch>
hipError_t ordered_grad_write(const void *const *keys, int nkeys, hipStream_t s, Launch launch) {
    std::lock_guard<std::mutex> lk(g_gw_mu);
    const GradEvent *waited[16];
    int nw = 0;
    for (int k = 0; k < nkeys; ++k) {
        if (!keys[k]) continue;
        auto it = g_gw.find(keys[k]);
        if (it == g_gw.end() || it->second.s == s) continue;
        const GradEvent *e = it->second.ev.get();
        bool seen = false;
        for (int j = 0; j < nw; ++j) seen = seen || waited[j] == e;
        if (seen) continue;
        const hipError_t r = hipStreamWaitEvent(s, e->ev, 0);
        if (r != hipSuccess) return r;
        if (nw < 16) waited[nw++] = e;
    }
    auto ev = std::make_shared<GradEvent>();
    hipError_t r = hipSuccess;
    if (!g_gw_evpool.empty()) { ev->ev = g_gw_evpool.back(); g_gw_evpool.pop_back(); }
    else r = hipEventCreateWithFlags(&ev->ev, hipEventDisableTiming);
    if (r != hipSuccess) { ev->ev = nullptr; return r; }
    r = launch();
    if (r != hipSuccess) return r;
    r = hipEventRecord(ev->ev, s);
    if (r != hipSuccess) return r;
    for (int k = 0; k < nkeys; ++k)
        if (keys[k]) g_gw[keys[k]] = GradWriter{s, ev};
    if (g_gw.size() > kGradPruneAt) {
        for (auto it = g_gw.begin(); it != g_gw.end();)
            it = hipEventQuery(it->second.ev->ev) == hipSuccess ? g_gw.erase(it) : std::next(it);
    }
    return hipSuccess;
}

// Host-mapped, coherent pinned word per thread for the num_rendered read-back.  k_bin_scan stores
// K into it with a system-scope store; the host spins on it (no copy kernel, no runtime wait).
struct HostWord { uint32_t *h = nullptr; uint32_t *d = nullptr; };
HostWord pinned_word() {
    thread_local HostWord w;
    if (!w.h) {
        uint32_t *h = nullptr;
        if (hipHostMalloc((void **)&h, 4 * kHostWords, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return w;
        uint32_t *d = nullptr;
        if (hipHostGetDevicePointer((void **)&d, h, 0) != hipSuccess) { (void)hipHostFree(h); return w; }
        w.h = h; w.d = d;
    }
    return w;
}

constexpr uint32_t kNoValue = 0xFFFFFFFFu;

// host-side timers (profiling mode only)
using hclock = std::chrono::steady_clock;
struct HostPhase {
    const char *name; hclock::time_point t0; bool on;
    explicit HostPhase(const char *n) : name(n), t0(hclock::now()), on(g_prof_on) {}
    ~HostPhase() {
        if (!on) return;
        const double ms = std::chrono::duration<double, std::milli>(hclock::now() - t0).count();
        std::lock_guard<std::mutex> lk(g_prof_mu);
        g_host_ms[name] += ms;
        g_host_n[name] += 1;
    }
};

int check_common(const gsr_camera *cam, const gsr_gaussians *g, bool need_opacity) {
    if (!cam || !g) return fail(GSR_ERR_ARG, "null camera or gaussians");
    if (g->P < 0) return fail(GSR_ERR_ARG, "P must be >= 0");
    if (cam->image_width <= 0 || cam->image_height <= 0)
        return fail(GSR_ERR_ARG, "image size must be positive (got %dx%d)", cam->image_width, cam->image_height);
    const int gx = div_up(cam->image_width, kTileW), gy = div_up(cam->image_height, kTileH);
    if (gx > 65535 || gy > 65535) return fail(GSR_ERR_UNSUPPORTED, "tile grid too large");
    if (g->activations & ~(GSR_ACT_SIGMOID_OPACITY | GSR_ACT_EXP_SCALES | GSR_ACT_NORMALIZE_ROTATIONS))
        return fail(GSR_ERR_ARG, "unknown activation bits 0x%x", g->activations);
    if (g->P == 0) return GSR_OK;
    if (!g->means3D || (need_opacity && !g->opacities))
        return fail(GSR_ERR_ARG, "means3D and opacities are required");
    if ((g->shs == nullptr) == (g->colors_precomp == nullptr))
        return fail(GSR_ERR_ARG, "Please provide excatly one of either SHs or precomputed colors!");
    const bool sr = g->scales && g->rotations;
    if (sr == (g->cov3D_precomp != nullptr) || ((g->scales != nullptr) != (g->rotations != nullptr)))
        return fail(GSR_ERR_ARG, "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    if (g->shs && (g->sh_coeffs <= 0 || (g->sh_degree + 1) * (g->sh_degree + 1) > g->sh_coeffs || g->sh_degree > 3 || g->sh_degree < 0))
        return fail(GSR_ERR_ARG, "invalid SH configuration: degree %d with %d coefficients", g->sh_degree, g->sh_coeffs);
    if (!cam->viewmatrix || !cam->projmatrix || !cam->bg || (g->shs && !cam->campos))
        return fail(GSR_ERR_ARG, "camera matrices / bg / campos missing");
    return GSR_OK;
}

// exact-threshold mode (gsr_set_exact_thresholds): on by default, GSR_EXACT_THRESHOLDS=0 at load turns
// it off
std::atomic<int> g_exact{[] {
    const char *e = getenv("GSR_EXACT_THRESHOLDS");
    return (e && e[0] == '0') ? 0 : 1;
}()};

void fill_common(FwdArgs &a, const gsr_camera *cam, const gsr_gaussians *g) {
    memset(&a, 0, sizeof(a));
    a.exact = g_exact.load(std::memory_order_relaxed);
    a.P = g->P; a.D = g->sh_degree; a.M = g->shs ? g->sh_coeffs : 0;
    a.W = cam->image_width; a.H = cam->image_height;
    a.gx = div_up(a.W, kTileW); a.gy = div_up(a.H, kTileH);
    a.scale_modifier = g->scale_modifier;
    a.act = g->activations;
    a.tan_fovx = cam->tan_fovx; a.tan_fovy = cam->tan_fovy;
    a.focal_y = a.H / (2.0f * a.tan_fovy);
    a.focal_x = a.W / (2.0f * a.tan_fovx);
    a.means3D = g->means3D; a.scales = g->scales; a.rotations = g->rotations; a.opacities = g->opacities;
    a.shs = g->shs; a.colors_precomp = g->colors_precomp; a.cov3D_precomp = g->cov3D_precomp;
    a.viewmatrix = cam->viewmatrix; a.projmatrix = cam->projmatrix; a.campos = cam->campos; a.bg = cam->bg;
    const bool vz = !cam->viewmatrix_stride[0] && !cam->viewmatrix_stride[1];
    const bool pz = !cam->projmatrix_stride[0] && !cam->projmatrix_stride[1];
    a.cs.v0 = vz ? 4 : cam->viewmatrix_stride[0]; a.cs.v1 = vz ? 1 : cam->viewmatrix_stride[1];
    a.cs.p0 = pz ? 4 : cam->projmatrix_stride[0]; a.cs.p1 = pz ? 1 : cam->projmatrix_stride[1];
    a.cs.c0 = cam->campos_stride ? cam->campos_stride : 1;
}

void carve_geom(FwdArgs &a, char *base) {
    const GeomLayout L(a.P);
    a.depth = (float *)(base + L.depth); a.rec = (float4 *)(base + L.rec);
    a.rect = (uint2 *)(base + L.rect); a.tiles = (uint32_t *)(base + L.tiles); a.goff = (uint32_t *)(base + L.goff);
    a.clampm = (uint8_t *)(base + L.clampm);
}
void carve_image(FwdArgs &a, char *base) {
    const ImageLayout L(a.W, a.H, a.P);
    a.ranges = (uint2 *)(base + L.ranges); a.pix_end = (float4 *)(base + L.pix_end);
    a.n_contrib = (uint32_t *)(base + L.n_contrib); a.tile_maxc = (uint32_t *)(base + L.tile_maxc);
    a.tile_order_f = (uint32_t *)(base + L.tile_order_f);
    a.seg_off = (uint32_t *)(base + L.seg_off);
    a.sort_lists = (uint32_t *)(base + L.sort_lists);
    a.tile_count = (uint32_t *)(base + L.tile_count); a.tile_cursor = (uint32_t *)(base + L.tile_cursor);
    a.block_sums = (uint32_t *)(base + L.block_sums); a.block_off = (uint32_t *)(base + L.block_off);
    a.meta = (uint32_t *)(base + L.meta); a.chunk_off = (uint32_t *)(base + L.chunk_off);
    a.items_ws = (uint32_t *)(base + L.items_ws);
    a.scan_ws = (uint32_t *)(base + L.scan_ws); a.tile_rank = (uint32_t *)(base + L.tile_rank);
    a.tile_flag = (uint32_t *)(base + L.tile_flag); a.near_rec = (float4 *)(base + L.near_rec);
    a.tsat_list = (uint32_t *)(base + L.tsat_list);
}
void carve_binning(FwdArgs &a, char *base, int K) {
    const BinningLayout L(K, a.P);
    a.pairs = (uint4 *)(base + L.pairs);
    a.point_list = (uint32_t *)(base + L.point_list);
    a.slot_emit = (uint32_t *)(base + L.slot_emit);
    a.seg_state = (float4 *)(base + L.seg_state);
}

}  // namespace

extern "C" {

const char *gsr_last_error(void) { return g_err.c_str(); }

int gsr_set_exact_thresholds(int on) { return g_exact.exchange(on ? 1 : 0); }
int gsr_abi_version(void) { return GSR_ABI_VERSION; }

size_t gsr_geom_bytes(int P) { return GeomLayout(P < 0 ? 0 : P).total; }
size_t gsr_image_bytes(int W, int H, int P) { return ImageLayout(W, H, P < 0 ? 0 : P).total; }
size_t gsr_binning_bytes(int K, int P) { return BinningLayout(K, P).total; }
size_t gsr_backward_items_bytes(int K, int W, int H) {
    return bwd_items_bytes(K < 0 ? 0 : K, div_up(W < 0 ? 0 : W, kTileW) * div_up(H < 0 ? 0 : H, kTileH));
}
// kPartial x P sums, then the view's camera key (k_sum_records; the multi-view pass orders views by it)
size_t gsr_sums_bytes(int P) { return align256(sizeof(float) * (kPartial * (size_t)(P < 0 ? 0 : P) + 1)); }
size_t gsr_scratch_bytes(int K, int W, int H) {
    return ScratchLayout(K, div_up(W < 0 ? 0 : W, kTileW) * div_up(H < 0 ? 0 : H, kTileH)).total;
}

void *gsr_prealloc_alloc(void *ctx, int which, size_t bytes) {
    gsr_prealloc *pa = (gsr_prealloc *)ctx;
    if (!pa) return nullptr;
    if (which >= 0 && which < 5 && pa->ptr[which] && pa->bytes[which] >= bytes && !(pa->used & (1 << which))) {
        pa->used |= 1 << which;
        return pa->ptr[which];
    }
    return pa->fallback ? pa->fallback(pa->fallback_ctx, which, bytes) : nullptr;
}

int gsr_buffer_offsets(int P, int W, int H, int K, size_t *out, int max_out) {
    const GeomLayout g(P);
    const ImageLayout im(W, H, P);
    const BinningLayout b(K, P);
    const size_t v[16] = {g.depth, g.rec, g.rect, g.tiles, g.goff,
                          im.ranges, im.pix_end, im.n_contrib, im.tile_maxc,
                          b.pairs, b.point_list, b.slot_emit, im.seg_off, b.seg_state, im.tile_flag,
                          im.items_ws + sizeof(uint32_t) * kTSatCtr};
    int n = 0;
    for (; n < 16 && n < max_out; ++n) out[n] = v[n];
    return n;
}

}  // extern "C"

namespace {
// Pair-count history for the speculative enqueue, per (device, P, W, H): the largest K seen and
// whether a list needed the merge sort.  A forward with history queues its post-scan kernels against
// a BINNING capacity of 1.25 x that K (+ 64 K pairs) before reading K back, so the GPU never waits for
// the host between k_bin_scan and k_bin_emit; the kernels check k_bin_scan's verdict on the device
// and the host redoes the post-scan part with the exact K when it failed (a larger K, a long list).
struct SpecKey {
    int dev, P, W, H;
    bool operator==(const SpecKey &o) const { return dev == o.dev && P == o.P && W == o.W && H == o.H; }
};
struct SpecKeyHash {
    size_t operator()(const SpecKey &k) const {
        return ((size_t)k.dev * 1000003u) ^ ((size_t)k.P * 2654435761u) ^ ((size_t)k.W << 20) ^ (size_t)k.H;
    }
};
// The capacity follows the largest K of the last kSpecWindow forwards of the key (one dense close-up
// view does not inflate every later view's BINNING for good), and the table keeps the kSpecKeys most
// recently used keys (densification changes P, i.e. the key, every 100 iterations).
constexpr int kSpecWindow = 16;
constexpr size_t kSpecKeys = 64;
struct SpecStat {
    uint32_t recent[kSpecWindow] = {};
    uint32_t recent_mid[kSpecWindow] = {};  // lists sorted by k_tile_sort (1024 < n <= 4096)
    int n = 0;
    bool long_lists = false;
    uint64_t used = 0;
    uint32_t window_max() const {
        uint32_t m = 0;
        for (int k = 0; k < std::min(n, kSpecWindow); ++k) m = std::max(m, recent[k]);
        return m;
    }
};
std::mutex g_spec_mu;
std::unordered_map<SpecKey, SpecStat, SpecKeyHash> g_spec;
uint64_t g_spec_clock = 0;
int g_spec_hits = 0, g_spec_misses = 0, g_async_calls = 0;

// The speculative capacity of a key (0: no history / long lists) and, in *sort_blocks, the grid of the
// speculative k_tile_sort (its blocks loop over the device-side list count; a grid near the recent
// counts instead of kSpecSortBlocks keeps hundreds of idle 48 KB-LDS blocks out of a busy chip).
uint32_t spec_capacity(const SpecKey &key, uint32_t *sort_blocks = nullptr) {
    std::lock_guard<std::mutex> lk(g_spec_mu);
    auto it = g_spec.find(key);
    if (it == g_spec.end() || it->second.long_lists) return 0;
    it->second.used = ++g_spec_clock;
    const uint32_t mk = it->second.window_max();
    if (sort_blocks) {
        uint32_t mm = 0;
        for (int k = 0; k < std::min(it->second.n, kSpecWindow); ++k) mm = std::max(mm, it->second.recent_mid[k]);
        *sort_blocks = std::min<uint32_t>((uint32_t)kSpecSortBlocks, mm + mm / 4 + 16);
    }
    const uint64_t c = (uint64_t)mk + mk / 4 + 65536;
    return (uint32_t)std::min<uint64_t>((c + 4095) & ~uint64_t(4095), 0x7FFFFFFFu);
}
void spec_record(const SpecKey &key, uint32_t K, bool long_lists, int outcome, uint32_t n_mid) {
    std::lock_guard<std::mutex> lk(g_spec_mu);
    if (!g_spec.count(key) && g_spec.size() >= kSpecKeys) {  // evict the least recently used key
        auto lru = g_spec.begin();
        for (auto it = g_spec.begin(); it != g_spec.end(); ++it)
            if (it->second.used < lru->second.used) lru = it;
        g_spec.erase(lru);
    }
    SpecStat &st = g_spec[key];
    st.recent[st.n % kSpecWindow] = K;
    st.recent_mid[st.n % kSpecWindow] = n_mid;
    ++st.n;
    st.long_lists = long_lists;
    st.used = ++g_spec_clock;
    if (outcome > 0) ++g_spec_hits;
    if (outcome < 0) ++g_spec_misses;
}

// ---- asynchronous forwards (ABI 17, gsr_forward_async) ------------------------------------------
// A speculative forward whose capacity came from the key's history returns as soon as its kernels are
// queued, without reading num_rendered back.  Each such forward takes a slot of a host-mapped ring:
// k_bin_scan publishes K and the list-class counts into the slot's words, and the speculative
// k_render_fwd holds the caller's stream (gate_wait) only when the device found the capacity too small.
// The resolver thread (one per process, no Python, no caller locks) reads every pending slot; on a
// failed speculation it redoes the post-scan kernels exactly on its own stream, into a BINNING buffer
// it allocates stream-ordered (hipMallocAsync), and then opens the gate.  Outputs are therefore the
// exact path's in every case, and nothing downstream of the forward can run before they are final.
// gsr_forward_resolve gives the backward the pair count and the BINNING buffer to use; a forward's
// record (and the resolver's buffer, freed stream-ordered on the forward's stream) is dropped once
// the caller released it and it is resolved.
constexpr int kAsyncSlots = 4096;
constexpr int kSlotWords = 16;  // 64 bytes: [0..3] k_bin_scan's host words, [4] the gate, [5] its timeout error
constexpr int kGateWord = 4, kGateErrWord = 5;
constexpr uint64_t kGateTimeoutTicks = 500000000ull;  // 5 s of s_memrealtime (100 MHz)
// test hooks (gsr_debug_async_fault): the gate timeout of later forwards, and a delay the resolver
// holds the next redone forward's gate closed for
std::atomic<uint64_t> g_gate_timeout{kGateTimeoutTicks};
std::atomic<int> g_hold_next_redo_ms{0};

struct AsyncFwd {
    uint64_t id = 0;
    int dev = 0, slot = -1, T = 0;
    hipStream_t s = nullptr;
    uint32_t seq = 0, cap = 0;
    bool prep = false, released = false, err_reported = false;
    SpecKey key{0, 0, 0, 0};
    FwdArgs a;                  // the launch arguments (GEOM / IMAGE / outputs carved)
    void *spec_bin = nullptr;   // the caller's BINNING, laid out for `cap`
    hipEvent_t ev_scan = nullptr;  // recorded on `s` after k_bin_scan (the redo waits for it)
    int state = 0;              // 0 pending, 1 stood, 2 redo queued, 3 redone, -1 failed
    uint32_t K = 0;
    int layout = 0;
    void *bin = nullptr;        // the BINNING buffer the backward uses
    void *own = nullptr;        // the resolver's allocation (redone forwards)
    std::string err;
};

std::mutex g_as_mu;
std::condition_variable g_as_wake;  // the resolver: a forward was queued / a redo is needed
std::condition_variable g_as_done;  // resolutions
std::unordered_map<uint64_t, std::shared_ptr<AsyncFwd>> g_as;
uint64_t g_as_next_id = 1;
uint32_t g_as_seq = 0;
uint32_t *g_slot_h = nullptr, *g_slot_d = nullptr;  // kAsyncSlots * kSlotWords words + 16 (error words)
std::vector<uint8_t> g_slot_busy;
std::vector<hipEvent_t> g_as_evpool;  // k_bin_scan events of reaped forwards
int g_slot_next = 0;
std::string g_async_err;  // a failed redo, or a timed-out gate whose forward was never resolved: reported
                          // by the next forward (sticky until gsr_debug_async_fault(.., clear) or a report)
bool g_resolver_started = false, g_resolver_stop = false;
std::thread g_resolver;

uint32_t *slot_h(int k) { return g_slot_h + (size_t)k * kSlotWords; }
uint32_t *slot_d(int k) { return g_slot_d + (size_t)k * kSlotWords; }

void resolver_main();

// The resolver's stream of each device.  A failed speculation holds the forward's stream in a
// spinning wave until the redo on this stream is done, so this stream must never wait for that wave:
// (1) non-blocking (a blocking stream would wait for the legacy default stream, torch's default);
// (2) not behind it in a hardware queue -- a process's streams share GPU_MAX_HW_QUEUES queues per
// priority level, and the call-shape probe deadlocked when the resolver's normal-priority stream
// shared the held stream's queue.  The resolver's stream therefore has the highest priority, a level
// callers' streams do not use unless they ask for it.  (A CU-masked stream gets a queue of its own,
// but HIP creates it blocking: the redo then waited for the held default stream.)  Created on the
// caller's thread at the first asynchronous forward of the device (g_as_mu held).
std::map<int, hipStream_t> g_resolver_streams;
hipStream_t resolver_stream(int dev) {
    hipStream_t &h = g_resolver_streams[dev];
    if (h) return h;
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
    if (hipStreamCreateWithPriority(&h, hipStreamNonBlocking, hi) != hipSuccess) h = nullptr;
    return h;
}

// (g_as_mu held) the slot ring and the resolver thread, on first use
bool async_init() {
    if (!g_slot_h) {
        uint32_t *h = nullptr;
        const size_t bytes = sizeof(uint32_t) * ((size_t)kAsyncSlots * kSlotWords + 16);
        if (hipHostMalloc((void **)&h, bytes, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess)
            return false;
        uint32_t *d = nullptr;
        if (hipHostGetDevicePointer((void **)&d, h, 0) != hipSuccess) { (void)hipHostFree(h); return false; }
        memset(h, 0, bytes);
        g_slot_h = h; g_slot_d = d;
        g_slot_busy.assign(kAsyncSlots, 0);
    }
    if (!g_resolver_started) {  // lives until gsr_async_shutdown (the binding's atexit hook)
        g_resolver_stop = false;
        g_resolver = std::thread(resolver_main);
        g_resolver_started = true;
    }
    return true;
}

// (g_as_mu held) a free slot, or -1 when every slot has an unresolved forward
int slot_acquire() {
    for (int k = 0; k < kAsyncSlots; ++k) {
        const int j = (g_slot_next + k) % kAsyncSlots;
        if (!g_slot_busy[j]) {
            g_slot_busy[j] = 1;
            g_slot_next = (j + 1) % kAsyncSlots;
            return j;
        }
    }
    return -1;
}

// (g_as_mu held) classify a forward whose K is published: 1 = the queued kernels stood, 2 = redo needed
void async_classify(AsyncFwd &f) {
    const uint32_t *w = slot_h(f.slot);
    f.K = __atomic_load_n(w, __ATOMIC_ACQUIRE);
    const uint32_t n_vlong = __atomic_load_n(w + 2, __ATOMIC_ACQUIRE), n_mid = __atomic_load_n(w + 1, __ATOMIC_ACQUIRE);
    if (f.K <= f.cap && n_vlong == 0) {  // the device's verdict (k_bin_scan: K <= cap, no merge-sorted list)
        f.state = 1;
        f.layout = (int)f.cap;
        f.bin = f.spec_bin;
        spec_record(f.key, f.K, false, +1, n_mid);
    } else {
        f.state = 2;
        spec_record(f.key, f.K, n_vlong > 0, -1, n_mid);
    }
}

// (g_as_mu held) drop a released, resolved record: the resolver's BINNING is freed stream-ordered on
// the forward's stream (after everything the caller queued there, the backward included)
void async_reap(std::unordered_map<uint64_t, std::shared_ptr<AsyncFwd>>::iterator it) {
    AsyncFwd &f = *it->second;
    if (f.own) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (cur != f.dev) (void)hipSetDevice(f.dev);
        (void)hipFreeAsync(f.own, f.s);
        if (cur != f.dev) (void)hipSetDevice(cur);
        f.own = nullptr;
    }
    if (f.ev_scan) g_as_evpool.push_back(f.ev_scan);  // a pending record may be re-recorded later
    f.ev_scan = nullptr;
    if (f.slot >= 0 && !f.err_reported && __atomic_load_n(slot_h(f.slot) + kGateErrWord, __ATOMIC_ACQUIRE) == f.seq)
        g_async_err = "an asynchronous forward's gate timed out (seq " + std::to_string(f.seq) + "), its outputs were not final";
    if (f.slot >= 0) g_slot_busy[f.slot] = 0;
    g_as.erase(it);
}

// The exact post-scan kernels of a failed speculation, on the resolver's stream of the forward's
// device, then the gate opens.  Runs without g_as_mu.
int async_redo(AsyncFwd &f, hipStream_t H) {
    (void)hipSetDevice(f.dev);
    if (!H) return fail(GSR_ERR_HIP, "asynchronous forward: no resolver stream on device %d", f.dev);
    HIP_TRY(hipStreamWaitEvent(H, f.ev_scan, 0));
    const uint32_t *w = slot_h(f.slot);
    const uint32_t K = f.K, n_mid = w[1], n_vlong = w[2], max_n = w[3];
    FwdArgs a = f.a;
    a.spec_ok = nullptr;
    a.spec_cap = 0;
    const size_t bin_bytes = BinningLayout((int)K, a.P).total;
    const size_t item_bytes = (f.prep) ? bwd_items_bytes((int)K, f.T) : 0;
    const size_t tmp_bytes = n_vlong ? sizeof(uint4) * (size_t)K : 0;
    void *bin = nullptr;
    if (hipMallocAsync(&bin, bin_bytes + item_bytes + tmp_bytes, H) != hipSuccess || !bin)
        return fail(GSR_ERR_ALLOC, "asynchronous forward: hipMallocAsync of %zu bytes failed", bin_bytes + item_bytes + tmp_bytes);
    f.own = bin;
    carve_binning(a, (char *)bin, (int)K);
    HIP_TRY(launch_bin_emit(a, (int)K, H));
    HIP_TRY(launch_tile_sort(a, n_mid, n_vlong, max_n, (uint4 *)((char *)bin + bin_bytes + item_bytes), H));
    HIP_TRY(launch_render_fwd(a, H));
    if (f.prep)
        HIP_TRY(launch_bwd_items_raw((int)K, f.T, a.P, a.ranges, a.tile_maxc, a.tile_flag, (uint2 *)((char *)bin + bin_bytes), a.items_ws, H));
    HIP_TRY(hipStreamSynchronize(H));
    f.bin = bin;
    f.layout = (int)K;
    return GSR_OK;
}

// The resolver thread: takes the oldest unclassified forward, sleeps on its scan event (a
// blocking-sync event: no polling, no CPU burned, no lock held), classifies it from the slot's words,
// redoes it when the speculation failed, and drops released + resolved records.  Forwards whose
// backward resolved them first are skipped.
void resolver_main() {
    std::unique_lock<std::mutex> lk(g_as_mu);
    for (;;) {
        for (auto it = g_as.begin(); it != g_as.end();) {  // reap released, resolved records
            const AsyncFwd &f = *it->second;
            if (f.released && (f.state == 1 || f.state == 3 || f.state == -1)) async_reap(it++);
            else ++it;
        }
        std::shared_ptr<AsyncFwd> next;
        for (auto &kv : g_as)  // the oldest forward still to classify or redo
            if ((kv.second->state == 0 || kv.second->state == 2) && (!next || kv.second->id < next->id)) next = kv.second;
        if (!next) {
            if (g_resolver_stop) break;
            g_as_wake.wait(lk);
            continue;
        }
        if (next->state == 0) {
            hipEvent_t ev = next->ev_scan;
            const int dev = next->dev;
            lk.unlock();
            (void)hipSetDevice(dev);
            const hipError_t r = hipEventSynchronize(ev);  // k_bin_scan done: its words are published
            lk.lock();
            if (next->state == 0) {
                if (r != hipSuccess || __atomic_load_n(slot_h(next->slot), __ATOMIC_ACQUIRE) == kNoValue) {
                    next->state = -1;
                    next->err = r != hipSuccess ? std::string("stream error before num_rendered was published: ") +
                                                      hipGetErrorString(r)
                                                : std::string("num_rendered was not published");
                    __atomic_store_n(slot_h(next->slot) + kGateWord, next->seq, __ATOMIC_RELEASE);
                } else {
                    async_classify(*next);
                }
                g_as_done.notify_all();
            }
            continue;
        }
        // state 2: redo the post-scan kernels exactly, then open the gate
        hipStream_t H = g_resolver_streams.count(next->dev) ? g_resolver_streams[next->dev] : nullptr;
        lk.unlock();
        const int rc = async_redo(*next, H);
        const std::string msg = rc ? g_err : std::string();
        if (g_hold_next_redo_ms > 0) {  // test hook: the gate stays closed a while (the wave may time out)
            std::this_thread::sleep_for(std::chrono::milliseconds(g_hold_next_redo_ms));
            g_hold_next_redo_ms = 0;
        }
        __atomic_store_n(slot_h(next->slot) + kGateWord, next->seq, __ATOMIC_RELEASE);  // open the gate
        lk.lock();
        next->state = rc ? -1 : 3;
        if (rc) { next->err = msg; g_async_err = "asynchronous forward redo failed: " + msg; }
        g_as_done.notify_all();
    }
}

}  // namespace

extern "C" size_t gsr_spec_binning_bytes(int P, int W, int H, int prepare_backward) {
    if (P <= 0 || W <= 0 || H <= 0) return 0;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const uint32_t cap = spec_capacity(SpecKey{dev, P, W, H});
    if (!cap) return 0;
    const size_t items = (prepare_backward) ? bwd_items_bytes((int)cap, div_up(W, kTileW) * div_up(H, kTileH)) : 0;
    return BinningLayout((int)cap, P).total + items;
}

namespace {
// mode 0: exact (the host reads K, then queues the rest); 1: speculative, the call still returns after
// K is known; 2: asynchronous (gsr_forward_async) -- with a capacity the call returns once everything
// is queued, info->pending names the forward for gsr_forward_resolve / gsr_forward_release.
int forward_impl(const gsr_camera *cam, const gsr_gaussians *g, gsr_alloc_fn alloc, void *alloc_ctx,
                 float *out_color, float *out_depth, int *out_radii, gsr_forward_info *info, int mode,
                 void *stream) {
    HostPhase host_total("host_forward");
    int rc = check_common(cam, g, true);
    if (rc) return rc;
    if (!alloc || !out_color || !out_depth || !info || (g->P > 0 && !out_radii))
        return fail(GSR_ERR_ARG, "gsr_forward: missing output or allocator");
    {
        std::lock_guard<std::mutex> lk(g_as_mu);
        if (!g_async_err.empty()) return fail(GSR_ERR_HIP, "%s", g_async_err.c_str());
    }
    hipStream_t s = (hipStream_t)stream;
    FwdArgs a;
    fill_common(a, cam, g);
    a.radii = out_radii; a.out_color = out_color; a.out_depth = out_depth;
    const size_t npix = (size_t)a.W * a.H;
    // The three persistent buffers are always requested, so a caller can hand them back verbatim.
    char *geom = (char *)alloc(alloc_ctx, GSR_BUF_GEOM, GeomLayout(a.P).total);
    char *img = (char *)alloc(alloc_ctx, GSR_BUF_IMAGE, ImageLayout(a.W, a.H, a.P).total);
    if (!geom || !img) return fail(GSR_ERR_ALLOC, "allocation callback failed (geom/image)");
    carve_geom(a, geom);
    carve_image(a, img);
    info->num_rendered = 0;
    info->binning_layout = 0;
    info->speculated = 0;
    info->pending = 0;
    info->aux_stream = nullptr;
    if (a.P == 0) {  // reference: colour/depth stay zero (no background) when there are no Gaussians
        HIP_TRY(launch_zero(out_color, 3 * npix, s));
        HIP_TRY(launch_zero(out_depth, npix, s));
        char *bin = (char *)alloc(alloc_ctx, GSR_BUF_BINNING, BinningLayout(0, 0).total);
        if (!bin) return fail(GSR_ERR_ALLOC, "allocation callback failed (binning)");
        return GSR_OK;
    }
    int dev = 0;
    (void)hipGetDevice(&dev);
    const SpecKey key{dev, a.P, a.W, a.H};
    uint32_t sort_blocks = kSpecSortBlocks;
    const uint32_t cap = mode ? spec_capacity(key, &sort_blocks) : 0u;
    a.spec_cap = cap;
    a.spec_sort_blocks = sort_blocks;
    const int T = a.gx * a.gy;
    // where k_bin_scan publishes K: an asynchronous forward's ring slot, else this thread's word
    std::shared_ptr<AsyncFwd> af;
    uint32_t *words_h = nullptr, *words_d = nullptr;
    if (mode == 2 && cap) {
        std::lock_guard<std::mutex> lk(g_as_mu);
        if (async_init() && resolver_stream(dev)) {
            const int slot = slot_acquire();
            if (slot >= 0) {
                af = std::make_shared<AsyncFwd>();
                af->slot = slot;
                af->seq = ++g_as_seq;
                words_h = slot_h(slot);
                words_d = slot_d(slot);
                __atomic_store_n(words_h + kGateErrWord, 0u, __ATOMIC_RELAXED);
            }
        }
    }
    struct SlotGuard {  // an acquired slot goes back to the ring unless the forward got registered
        std::shared_ptr<AsyncFwd> *f;
        ~SlotGuard() {
            if (!*f || (*f)->id) return;
            std::lock_guard<std::mutex> lk(g_as_mu);
            g_slot_busy[(*f)->slot] = 0;
            if ((*f)->ev_scan) g_as_evpool.push_back((*f)->ev_scan);
        }
    } slot_guard{&af};
    if (!af) {
        HostWord hw = pinned_word();
        if (!hw.h) return fail(GSR_ERR_HIP, "hipHostMalloc(mapped) failed");
        words_h = hw.h;
        words_d = hw.d;
    }
    __atomic_store_n(words_h, kNoValue, __ATOMIC_SEQ_CST);
    { Phase ph(s, "preprocess"); HIP_TRY(launch_preprocess(a, s)); }
    { Phase ph(s, "bin_count"); HIP_TRY(launch_bin_count(a, s)); }
    { Phase ph(s, "bin_scan"); HIP_TRY(launch_bin_scan(a, words_d, s)); }
    if (af) {
        {
            std::lock_guard<std::mutex> lk(g_as_mu);
            if (!g_as_evpool.empty()) { af->ev_scan = g_as_evpool.back(); g_as_evpool.pop_back(); }
        }
        if (!af->ev_scan) HIP_TRY(hipEventCreateWithFlags(&af->ev_scan, hipEventDisableTiming | hipEventBlockingSync));
        HIP_TRY(hipEventRecord(af->ev_scan, s));
    }
    const size_t spec_item_bytes = (g->prepare_backward) ? bwd_items_bytes((int)cap, T) : 0;
    char *spec_bin = nullptr;
    if (cap) {  // speculative: the post-scan kernels are queued now, against the capacity
        spec_bin = (char *)alloc(alloc_ctx, GSR_BUF_BINNING, BinningLayout((int)cap, a.P).total + spec_item_bytes);
        if (!spec_bin) return fail(GSR_ERR_ALLOC, "allocation callback failed (binning, capacity %u)", cap);
        FwdArgs sa = a;
        carve_binning(sa, spec_bin, (int)cap);
        sa.spec_ok = sa.meta + 1;
        if (af) {  // a failed speculation holds the stream in the speculative render until it is redone
            sa.gate = words_d + kGateWord;
            sa.gate_seq = af->seq;
            sa.gate_err = words_d + kGateErrWord;
            sa.gate_timeout = g_gate_timeout;
        }
        { Phase ph(s, "bin_emit"); HIP_TRY(launch_bin_emit(sa, 0, s)); }
        { Phase ph(s, "tile_sort"); HIP_TRY(launch_tile_sort(sa, 0, 0, 0, nullptr, s)); }
        { Phase ph(s, "render_fwd"); HIP_TRY(launch_render_fwd(sa, s)); }
        if (g->prepare_backward) {
            uint2 *items = (uint2 *)(spec_bin + BinningLayout((int)cap, a.P).total);
            Phase ph(s, "bwd_items");
            HIP_TRY(launch_bwd_items_raw((int)cap, T, a.P, a.ranges, a.tile_maxc, a.tile_flag, items, a.items_ws, s, sa.spec_ok));
        }
    }
    if (af) {  // asynchronous: gate the stream on the verdict and return
        std::lock_guard<std::mutex> lk(g_as_mu);
        af->id = g_as_next_id++;
        af->dev = dev; af->s = s; af->cap = cap; af->T = T; af->key = key;
        af->prep = g->prepare_backward != 0;
        af->a = a;
        af->spec_bin = spec_bin;
        g_as[af->id] = af;
        info->num_rendered = -1;
        info->binning_layout = (int)cap;
        info->speculated = 1;
        info->pending = af->id;
        {
            std::lock_guard<std::mutex> lk2(g_spec_mu);
            ++g_async_calls;
        }
        g_as_wake.notify_one();
        return GSR_OK;
    }
    uint32_t K;
    {
        HostPhase hp("host_wait_K");
        // Spin on the host-mapped word (the scan is queued behind the caller's earlier work on this
        // stream, so this can take milliseconds).  Every ~0.5 ms ask the runtime whether the stream
        // has drained or failed, so a faulted launch cannot leave us spinning.
        auto last = hclock::now();
        while ((K = __atomic_load_n(words_h, __ATOMIC_ACQUIRE)) == kNoValue) {
            __builtin_ia32_pause();
            if (hclock::now() - last > std::chrono::microseconds(500)) {
                last = hclock::now();
                const hipError_t q = hipStreamQuery(s);
                if (q == hipErrorNotReady) continue;
                if (q != hipSuccess) return fail(GSR_ERR_HIP, "stream error while waiting for num_rendered: %s", hipGetErrorString(q));
                K = __atomic_load_n(words_h, __ATOMIC_ACQUIRE);
                if (K == kNoValue) return fail(GSR_ERR_HIP, "num_rendered was not published");
                break;
            }
        }
    }
    if (K > 0x7FFFFFFFu) return fail(GSR_ERR_UNSUPPORTED, "num_rendered overflow");
    info->num_rendered = (int)K;
    // tiles to sort outside the render: [1] up to kSortCap pairs, [2] longer (merge sort), [3] the
    // longest list (merge passes); the latter need a temporary copy of the pair records
    const uint32_t n_mid = __atomic_load_n(words_h + 1, __ATOMIC_ACQUIRE);
    const uint32_t n_vlong = __atomic_load_n(words_h + 2, __ATOMIC_ACQUIRE);
    const uint32_t max_n = __atomic_load_n(words_h + 3, __ATOMIC_ACQUIRE);
    if (cap && K <= cap && n_vlong == 0) {  // the device took the same verdict: the queued work stands
        info->binning_layout = (int)cap;
        info->speculated = 1;
        spec_record(key, K, false, +1, n_mid);
        return GSR_OK;
    }
    // exact path (also the redo of a failed speculation: its queued kernels returned at once)
    a.spec_ok = nullptr;
    // BINNING = the binning arrays, [the backward's item list], [the long-list merge buffer]
    const size_t bin_bytes = BinningLayout((int)K, a.P).total;
    const size_t item_bytes = (g->prepare_backward) ? bwd_items_bytes((int)K, T) : 0;
    const size_t tmp_bytes = n_vlong ? sizeof(uint4) * (size_t)K : 0;
    char *bin = (char *)alloc(alloc_ctx, GSR_BUF_BINNING, bin_bytes + item_bytes + tmp_bytes);
    if (!bin) return fail(GSR_ERR_ALLOC, "allocation callback failed (binning, K=%u)", K);
    carve_binning(a, bin, (int)K);
    { Phase ph(s, "bin_emit"); HIP_TRY(launch_bin_emit(a, (int)K, s)); }
    { Phase ph(s, "tile_sort"); HIP_TRY(launch_tile_sort(a, n_mid, n_vlong, max_n, (uint4 *)(bin + bin_bytes + item_bytes), s)); }
    { Phase ph(s, "render_fwd"); HIP_TRY(launch_render_fwd(a, s)); }
    if (g->prepare_backward) {  // the backward's item list, built here, off its critical path
        uint2 *items = (uint2 *)(bin + bin_bytes);
        Phase ph(s, "bwd_items");
        HIP_TRY(launch_bwd_items_raw((int)K, T, a.P, a.ranges, a.tile_maxc, a.tile_flag, items, a.items_ws, s));
    }
    info->binning_layout = (int)K;
    spec_record(key, K, n_vlong > 0, cap ? -1 : 0, n_mid);
    return GSR_OK;
}
}  // namespace

extern "C" {

int gsr_forward(const gsr_camera *cam, const gsr_gaussians *g, gsr_alloc_fn alloc, void *alloc_ctx,
                float *out_color, float *out_depth, int *out_radii, int *out_num_rendered,
                void *stream) {
    if (!out_num_rendered) return fail(GSR_ERR_ARG, "gsr_forward: missing output or allocator");
    *out_num_rendered = 0;
    gsr_forward_info info;
    const int rc = forward_impl(cam, g, alloc, alloc_ctx, out_color, out_depth, out_radii, &info, 0, stream);
    *out_num_rendered = info.num_rendered;
    return rc;
}

int gsr_forward_info_call(const gsr_camera *cam, const gsr_gaussians *g, gsr_alloc_fn alloc, void *alloc_ctx,
                          float *out_color, float *out_depth, int *out_radii, int speculate, gsr_forward_info *info,
                          void *stream) {
    if (!info) return fail(GSR_ERR_ARG, "gsr_forward_info_call: null info");
    return forward_impl(cam, g, alloc, alloc_ctx, out_color, out_depth, out_radii, info, speculate ? 1 : 0, stream);
}

int gsr_forward_async(const gsr_camera *cam, const gsr_gaussians *g, gsr_alloc_fn alloc, void *alloc_ctx,
                      float *out_color, float *out_depth, int *out_radii, gsr_forward_info *info, void *stream) {
    if (!info) return fail(GSR_ERR_ARG, "gsr_forward_async: null info");
    return forward_impl(cam, g, alloc, alloc_ctx, out_color, out_depth, out_radii, info, 2, stream);
}

int gsr_forward_resolve(unsigned long long handle, gsr_forward_resolution *out) {
    if (!out) return fail(GSR_ERR_ARG, "gsr_forward_resolve: null output");
    HostPhase hp("host_wait_K");
    std::unique_lock<std::mutex> lk(g_as_mu);
    auto it = g_as.find(handle);
    if (it == g_as.end()) return fail(GSR_ERR_ARG, "gsr_forward_resolve: unknown or released forward %llu", handle);
    std::shared_ptr<AsyncFwd> f = it->second;
    auto last = hclock::now();
    while (f->state == 0 || f->state == 2) {
        if (f->state == 0) {
            if (__atomic_load_n(slot_h(f->slot), __ATOMIC_ACQUIRE) != kNoValue) {
                async_classify(*f);
                if (f->state == 2) g_as_wake.notify_one();  // the resolver redoes it
                continue;
            }
            // K not published yet: spin outside the lock, checking the stream for faults every ~0.5 ms
            lk.unlock();
            while (__atomic_load_n(slot_h(f->slot), __ATOMIC_ACQUIRE) == kNoValue) {
                __builtin_ia32_pause();
                if (hclock::now() - last > std::chrono::microseconds(500)) {
                    last = hclock::now();
                    const hipError_t q = hipStreamQuery(f->s);
                    if (q == hipErrorNotReady) continue;
                    if (__atomic_load_n(slot_h(f->slot), __ATOMIC_ACQUIRE) != kNoValue) break;
                    lk.lock();
                    if (f->state == 0) {
                        f->state = -1;
                        f->err = q == hipSuccess ? std::string("num_rendered was not published")
                                                 : std::string("stream error: ") + hipGetErrorString(q);
                        __atomic_store_n(slot_h(f->slot) + kGateWord, f->seq, __ATOMIC_RELEASE);
                    }
                    lk.unlock();
                    break;
                }
            }
            lk.lock();
            continue;
        }
        g_as_done.wait(lk);
    }
    if (f->state < 0) return fail(GSR_ERR_HIP, "asynchronous forward %llu failed: %s", handle, f->err.c_str());
    // a gate the render abandoned (timeout) before the redo opened it: everything the caller queued after
    // the forward ran on outputs that were not final -- this forward's resolution (the step's backward) fails
    if (__atomic_load_n(slot_h(f->slot) + kGateErrWord, __ATOMIC_ACQUIRE) == f->seq) {
        f->err_reported = true;
        return fail(GSR_ERR_HIP, "asynchronous forward %llu: its gate timed out before the redo opened it; the outputs "
                    "the caller used after the forward were not final", handle);
    }
    out->num_rendered = (int)f->K;
    out->binning_layout = f->layout;
    out->binning = f->bin;
    out->redone = f->state == 3;
    return GSR_OK;
}

int gsr_forward_query(unsigned long long handle) {
    std::lock_guard<std::mutex> lk(g_as_mu);
    auto it = g_as.find(handle);
    if (it == g_as.end()) return -1;
    AsyncFwd &f = *it->second;
    if (f.state == 0 && __atomic_load_n(slot_h(f.slot), __ATOMIC_ACQUIRE) != kNoValue) {
        async_classify(f);
        if (f.state == 2) g_as_wake.notify_one();
    }
    return (f.state == 1 || f.state == 3 || f.state == -1) ? 1 : 0;
}

int gsr_forward_release(unsigned long long handle) {
    std::lock_guard<std::mutex> lk(g_as_mu);
    auto it = g_as.find(handle);
    if (it == g_as.end()) return GSR_OK;
    it->second->released = true;
    const int st = it->second->state;
    if (st == 1 || st == 3 || st == -1) async_reap(it);
    else g_as_wake.notify_one();  // reaped by the resolver once resolved
    return GSR_OK;
}

int gsr_async_shutdown(void) {
    std::thread t;
    {
        std::lock_guard<std::mutex> lk(g_as_mu);
        if (!g_resolver_started) return GSR_OK;
        g_resolver_stop = true;
        g_resolver_started = false;
        t = std::move(g_resolver);
    }
    g_as_wake.notify_all();
    if (t.joinable()) t.join();
    return GSR_OK;
}

int gsr_async_stats(int *calls, int *pending) {
    {
        std::lock_guard<std::mutex> lk(g_spec_mu);
        if (calls) *calls = g_async_calls;
    }
    std::lock_guard<std::mutex> lk(g_as_mu);
    if (pending) *pending = (int)g_as.size();
    return GSR_OK;
}

int gsr_spec_stats(int *hits, int *misses, int reset) {
    std::lock_guard<std::mutex> lk(g_spec_mu);
    if (hits) *hits = g_spec_hits;
    if (misses) *misses = g_spec_misses;
    if (reset) { g_spec.clear(); g_spec_hits = g_spec_misses = g_async_calls = 0; }
    return GSR_OK;
}

int gsr_debug_async_fault(int hold_next_redo_ms, int gate_timeout_ms, int clear) {
    std::lock_guard<std::mutex> lk(g_as_mu);
    g_hold_next_redo_ms = hold_next_redo_ms > 0 ? hold_next_redo_ms : 0;
    g_gate_timeout = gate_timeout_ms > 0 ? (uint64_t)gate_timeout_ms * 100000ull : kGateTimeoutTicks;
    if (clear) g_async_err.clear();
    return GSR_OK;
}

int gsr_spec_keys(void) {
    std::lock_guard<std::mutex> lk(g_spec_mu);
    return (int)g_spec.size();
}

}  // extern "C"


namespace {
// The per-pixel half of the backward (bwd items + k_render_bwd): BwdArgs of the view and its SCRATCH
// buffer (records at a.part) requested through `alloc`.
int backward_render(const gsr_camera *cam, const gsr_gaussians *g, const int *radii, int num_rendered,
                    const void *geom, const void *binning, const void *image, const float *dL_dcolor,
                    gsr_alloc_fn alloc, void *alloc_ctx, hipStream_t s, BwdArgs &a, bool sums = false) {
    if (!geom || !binning || !image || !dL_dcolor || !radii || !alloc)
        return fail(GSR_ERR_ARG, "gsr_backward: missing saved buffers / dL_dcolor / allocator");
    // num_rendered < 0: a speculative render half (ABI 19) -- an asynchronous forward whose pair count is
    // not known yet, queued against its capacity (binning_layout) and its own BINNING; its kernels
    // return at once when the device's speculation verdict (the forward's meta[1]) failed, and the
    // caller redoes the half once gsr_forward_resolve reports the forward redone
    const bool spec = num_rendered < 0;
    if (spec && g->binning_layout <= 0) return fail(GSR_ERR_ARG, "num_rendered < 0 without the forward's binning_layout");
    FwdArgs f;
    fill_common(f, cam, g);
    carve_geom(f, (char *)geom);
    carve_image(f, (char *)image);
    // the BINNING layout the forward used: its capacity when it enqueued speculatively (gsr_forward_info)
    const int layout = g->binning_layout > 0 ? g->binning_layout : num_rendered;
    if (layout < num_rendered) return fail(GSR_ERR_ARG, "binning_layout %d < num_rendered %d", layout, num_rendered);
    if (spec) num_rendered = layout;  // the bound every size below is taken from
    carve_binning(f, (char *)binning, layout);
    memset(&a, 0, sizeof(a));
    a.P = f.P; a.D = f.D; a.M = f.M; a.W = f.W; a.H = f.H; a.gx = f.gx; a.gy = f.gy; a.K = num_rendered;
    a.act = f.act;
    a.scale_modifier = f.scale_modifier; a.tan_fovx = f.tan_fovx; a.tan_fovy = f.tan_fovy;
    a.focal_x = f.focal_x; a.focal_y = f.focal_y;
    a.means3D = f.means3D; a.scales = f.scales; a.rotations = f.rotations; a.shs = f.shs;
    a.colors_precomp = f.colors_precomp; a.cov3D_precomp = f.cov3D_precomp;
    a.viewmatrix = f.viewmatrix; a.projmatrix = f.projmatrix; a.campos = f.campos; a.bg = f.bg; a.cs = f.cs;
    a.radii = radii;
    a.rec = f.rec; a.rect = f.rect; a.goff = f.goff; a.clampm = f.clampm;
    a.ranges = f.ranges; a.pix_end = f.pix_end; a.n_contrib = f.n_contrib; a.tile_maxc = f.tile_maxc;
    a.tile_flag = f.tile_flag; a.near_rec = f.near_rec;
    a.seg_off = f.seg_off; a.meta = f.meta; a.items_ws = f.items_ws;
    a.point_list = f.point_list; a.slot_emit = f.slot_emit; a.seg_state = f.seg_state;
    a.dL_dcolor = dL_dcolor;
    a.spec_ok = spec ? f.meta + 1 : nullptr;
    const ScratchLayout SL(num_rendered, a.gx * a.gy);
    char *scr = (char *)alloc(alloc_ctx, GSR_BUF_SCRATCH, SL.total);
    if (!scr) return fail(GSR_ERR_ALLOC, "allocation callback failed (scratch)");
    a.part = (float4 *)(scr + SL.part);
    a.max_items = (uint32_t)max_bwd_items(num_rendered, a.gx * a.gy);
    if (g->prepare_backward) {  // built by the forward, after the binning arrays
        a.items = (uint2 *)((char *)binning + BinningLayout(layout, a.P).total);
    } else {
        a.items = (uint2 *)(scr + SL.items);
        Phase ph(s, "bwd_items");
        HIP_TRY(launch_bwd_items(a, s));
    }
    { Phase ph(s, "render_bwd"); HIP_TRY(launch_render_bwd(a, s)); }
    if (sums) {  // deferred view: its per-Gaussian record sums for gsr_backward_gaussians (SUMS buffer)
        float *out = (float *)alloc(alloc_ctx, GSR_BUF_SUMS, gsr_sums_bytes(a.P));
        if (!out) return fail(GSR_ERR_ALLOC, "allocation callback failed (sums)");
        Phase ph(s, "sum_records");
        HIP_TRY(launch_sum_records(a.P, a.goff, a.part, out, s, a.spec_ok, a.viewmatrix, a.projmatrix, a.campos, a.cs, a.W, a.H));
    }
    return GSR_OK;
}
}  // namespace

extern "C" {

int gsr_backward(const gsr_camera *cam, const gsr_gaussians *g, const int *radii, int num_rendered,
                 const void *geom, const void *binning, const void *image, const float *dL_dcolor,
                 const float *dL_ddepth, gsr_alloc_fn alloc, void *alloc_ctx, gsr_grads *out,
                 void *stream) {
    (void)dL_ddepth;
    HostPhase host_total("host_backward");
    int rc = check_common(cam, g, false);
    if (rc) return rc;
    if (!out) return fail(GSR_ERR_ARG, "gsr_backward: null grads");
    if (g->P == 0) return GSR_OK;
    if (out->accumulate & ~0xFF) return fail(GSR_ERR_ARG, "gsr_backward: unknown accumulate bits 0x%x", out->accumulate);
    if (num_rendered < 0) return fail(GSR_ERR_ARG, "gsr_backward: num_rendered < 0 (resolve the forward first)");
    hipStream_t s = (hipStream_t)stream;
    BwdArgs a;
    rc = backward_render(cam, g, radii, num_rendered, geom, binning, image, dL_dcolor, alloc, alloc_ctx, s, a);
    if (rc) return rc;
    a.dL_dmeans2D = out->dL_dmeans2D; a.dL_dcolors = out->dL_dcolors; a.dL_dopacity = out->dL_dopacity;
    a.dL_dmeans3D = out->dL_dmeans3D; a.dL_dcov3D = out->dL_dcov3D; a.dL_dsh = out->dL_dsh;
    a.dL_dscales = out->dL_dscales; a.dL_drot = out->dL_drotations;
    a.accm = out->accumulate;
    const void *written[8] = {a.dL_dmeans2D, a.dL_dcolors, a.dL_dopacity, a.dL_dmeans3D,
                              a.dL_dcov3D, a.dL_dsh, a.dL_dscales, a.dL_drot};
    { Phase ph(s, "gauss_bwd"); HIP_TRY(ordered_grad_write(written, 8, s, [&] { return launch_gauss_bwd(a, s); })); }
    return GSR_OK;
}

int gsr_backward_render(const gsr_camera *cam, const gsr_gaussians *g, const int *radii, int num_rendered,
                        const void *geom, const void *binning, const void *image, const float *dL_dcolor,
                        gsr_alloc_fn alloc, void *alloc_ctx, void *stream) {
    HostPhase host_total("host_backward");
    int rc = check_common(cam, g, false);
    if (rc) return rc;
    if (g->P == 0) return GSR_OK;
    BwdArgs a;
    return backward_render(cam, g, radii, num_rendered, geom, binning, image, dL_dcolor, alloc, alloc_ctx,
                           (hipStream_t)stream, a, true);
}

int gsr_backward_gaussians(int nviews, const gsr_view_grad *views, const gsr_gaussians *g, gsr_grads *out,
                           void *stream) {
    HostPhase host_total("host_backward");
    if (nviews < 0 || (nviews > 0 && !views) || !out) return fail(GSR_ERR_ARG, "gsr_backward_gaussians: bad view list / grads");
    if (nviews == 0) return GSR_OK;
    for (int v = 0; v < nviews; ++v) {
        const int rc = check_common(views[v].cam, g, false);
        if (rc) return rc;
    }
    if (g->P == 0) return GSR_OK;
    if (g->shs && g->sh_coeffs != 1 && g->sh_coeffs != 4 && g->sh_coeffs != 9 && g->sh_coeffs != 16)
        return fail(GSR_ERR_UNSUPPORTED, "gsr_backward_gaussians: %d SH coefficients (1, 4, 9 or 16 supported)", g->sh_coeffs);
    if (out->accumulate & ~0xFF) return fail(GSR_ERR_ARG, "gsr_backward_gaussians: unknown accumulate bits 0x%x", out->accumulate);
    for (int v = 0; v < nviews; ++v)
        if (!views[v].radii || !views[v].geom || !views[v].scratch || views[v].num_rendered < 0)
            return fail(GSR_ERR_ARG, "gsr_backward_gaussians: view %d lacks radii / geom / scratch", v);
    hipStream_t s = (hipStream_t)stream;
    MultiArgs m;
    memset(&m, 0, sizeof(m));
    m.P = g->P; m.D = g->sh_degree; m.M = g->shs ? g->sh_coeffs : 0; m.act = g->activations;
    m.scale_modifier = g->scale_modifier;
    m.means3D = g->means3D; m.scales = g->scales; m.rotations = g->rotations; m.shs = g->shs;
    m.cov3D_precomp = g->cov3D_precomp;
    m.dL_dcolors = out->dL_dcolors; m.dL_dopacity = out->dL_dopacity; m.dL_dmeans3D = out->dL_dmeans3D;
    m.dL_dcov3D = out->dL_dcov3D; m.dL_dsh = out->dL_dsh; m.dL_dscales = out->dL_dscales; m.dL_drot = out->dL_drotations;
    for (int v0 = 0; v0 < nviews; v0 += kMultiViews) {  // groups of kMultiViews views; later groups add
        m.nv = std::min(kMultiViews, nviews - v0);
        m.accm = (out->accumulate | (v0 ? 0xFF : 0)) & ~GSR_GRAD_MEANS2D;
        const void *written[8 + kMultiViews] = {m.dL_dcolors, m.dL_dopacity, m.dL_dmeans3D, m.dL_dcov3D,
                                                m.dL_dsh, m.dL_dscales, m.dL_drot};
        for (int k = 0; k < m.nv; ++k) {
            const gsr_view_grad &vg = views[v0 + k];
            const gsr_camera *cam = vg.cam;
            FwdArgs f;
            fill_common(f, cam, g);
            MultiView &mv = m.v[k];
            mv.viewmatrix = cam->viewmatrix; mv.projmatrix = cam->projmatrix; mv.campos = cam->campos;
            mv.cs = f.cs;
            mv.tan_fovx = f.tan_fovx; mv.tan_fovy = f.tan_fovy; mv.focal_x = f.focal_x; mv.focal_y = f.focal_y;
            mv.radii = vg.radii;
            mv.rec = (const float4 *)((const char *)vg.geom + GeomLayout(g->P).rec);
            mv.clampm = (const uint8_t *)vg.geom + GeomLayout(g->P).clampm;
            mv.sums = (const float *)vg.scratch;  // the view's SUMS buffer (gsr_backward_render)
            mv.dL_dmeans2D = vg.dL_dmeans2D;
            mv.acc2 = vg.accumulate_means2D ? 1 : 0;
            written[7 + k] = vg.dL_dmeans2D;
        }
        { Phase ph(s, "gauss_bwd"); HIP_TRY(ordered_grad_write(written, 7 + m.nv, s, [&] { return launch_gauss_bwd_multi(m, s); })); }
    }
    return GSR_OK;
}

int gsr_grad_fence(const void *const *grads, int n, void *stream) {
    if (n < 0 || (n > 0 && !grads)) return fail(GSR_ERR_ARG, "gsr_grad_fence: bad gradient list");
    HIP_TRY(ordered_grad_write(grads, n, (hipStream_t)stream, no_launch));
    return GSR_OK;
}

int gsr_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                     uint8_t *present, void *stream) {
    (void)projmatrix;
    if (P < 0) return fail(GSR_ERR_ARG, "P must be >= 0");
    if (P > 0 && (!means3D || !viewmatrix || !present)) return fail(GSR_ERR_ARG, "null pointer");
    HIP_TRY(launch_mark_visible(P, means3D, viewmatrix, present, (hipStream_t)stream));
    return GSR_OK;
}

}  // extern "C"

// ---- fused L1 + SSIM ----------------------------------------------------------------------
namespace {
struct SsimScratch {
    size_t maps, partial, total;
    SsimScratch(int planes, int H, int W) {
        const size_t n = (size_t)planes * H * W;
        maps = 0;
        partial = align256(sizeof(float) * 3 * n);
        total = align256(partial + sizeof(float2) * ssim_partials(planes, H, W));
    }
};

// The window of calc_ssim: gaussian(11, 1.5) (external.py:48-55) evaluates exp() in double, stores
// float32 and normalises by the float32 sum.
SsimWindow ssim_window() {
    SsimWindow w;
    float sum = 0.f;
    for (int x = 0; x < 11; ++x) {
        w.w[x] = (float)std::exp(-(double)((x - 5) * (x - 5)) / (2.0 * 1.5 * 1.5));
        sum += w.w[x];
    }
    for (int x = 0; x < 11; ++x) w.w[x] = w.w[x] / sum;
    return w;
}

int check_ssim(int planes, int H, int W, const float *img1, const float *img2) {
    if (planes < 0 || H < 0 || W < 0) return fail(GSR_ERR_ARG, "l1_ssim: negative size");
    if ((size_t)planes * H * W > 0 && (!img1 || !img2)) return fail(GSR_ERR_ARG, "l1_ssim: null image");
    if ((size_t)planes * H * W >= (size_t)1 << 31) return fail(GSR_ERR_UNSUPPORTED, "l1_ssim: image too large");
    if (planes > 65535) return fail(GSR_ERR_UNSUPPORTED, "l1_ssim: more than 65535 planes");
    return GSR_OK;
}
}  // namespace

extern "C" {

size_t gsr_ssim_scratch_bytes(int planes, int H, int W) {
    return SsimScratch(planes < 0 ? 0 : planes, H < 0 ? 0 : H, W < 0 ? 0 : W).total;
}

int gsr_l1_ssim_forward(int planes, int H, int W, const float *img1, const float *img2, void *scratch,
                        float *out_l1, float *out_ssim, void *stream) {
    int rc = check_ssim(planes, H, W, img1, img2);
    if (rc) return rc;
    if (!out_l1 || !out_ssim) return fail(GSR_ERR_ARG, "l1_ssim: null output");
    if ((size_t)planes * H * W == 0) return fail(GSR_ERR_ARG, "l1_ssim: empty image (the mean is undefined)");
    if (!scratch) return fail(GSR_ERR_ARG, "l1_ssim: null scratch");
    hipStream_t s = (hipStream_t)stream;
    const SsimScratch L(planes, H, W);
    char *base = (char *)scratch;
    Phase ph(s, "ssim_fwd");
    HIP_TRY(launch_ssim_fwd(planes, H, W, img1, img2, ssim_window(), (float *)(base + L.maps),
                            (float2 *)(base + L.partial), out_l1, out_ssim, s));
    return GSR_OK;
}

int gsr_l1_ssim_backward(int planes, int H, int W, const float *img1, const float *img2, const void *scratch,
                         const float *dL_dl1, const float *dL_dssim, float *dL_dimg1, void *stream) {
    int rc = check_ssim(planes, H, W, img1, img2);
    if (rc) return rc;
    if ((size_t)planes * H * W == 0) return GSR_OK;
    if (!dL_dimg1 || !scratch) return fail(GSR_ERR_ARG, "l1_ssim: null gradient output / scratch");
    hipStream_t s = (hipStream_t)stream;
    const SsimScratch L(planes, H, W);
    Phase ph(s, "ssim_bwd");
    HIP_TRY(launch_ssim_bwd(planes, H, W, img1, img2, ssim_window(), (const float *)((const char *)scratch + L.maps),
                            dL_dl1, dL_dssim, dL_dimg1, s));
    return GSR_OK;
}

// ---- densification --------------------------------------------------------------------------
}  // extern "C"
namespace {
int dens_args(const gsr_densify_settings *st, DensArgs &a) {
    if (!st) return fail(GSR_ERR_ARG, "densify: null settings");
    if (st->P < 0) return fail(GSR_ERR_ARG, "densify: P must be >= 0");
    if (st->P > 0 && (!st->grad_accum || !st->vis_count || !st->log_scales || !st->opacity_logits ||
                      !st->rotation_quaternions))
        return fail(GSR_ERR_ARG, "densify: statistics / log_scales / opacity_logits / rotations required");
    if (!(st->split_divisor > 0.f)) return fail(GSR_ERR_ARG, "densify: split_divisor must be > 0");
    a.P = st->P; a.prune_big = st->prune_big;
    a.grad_threshold = st->grad_threshold; a.small_scale = st->small_scale; a.big_scale = st->big_scale;
    a.remove_opacity = st->remove_opacity;
    // torch evaluates tensor / python-scalar on the GPU as tensor * (1 / scalar) in float
    a.inv_split_div = 1.0f / st->split_divisor;
    a.grad_accum = st->grad_accum; a.vis_count = st->vis_count; a.log_scales = st->log_scales;
    a.opacity_logits = st->opacity_logits; a.rotations = st->rotation_quaternions;
    return GSR_OK;
}
}  // namespace
extern "C" {

int gsr_densify_update_radii(int P, const int *radii, float *max_radii, uint8_t *visible, void *stream) {
    if (P < 0) return fail(GSR_ERR_ARG, "densify: P must be >= 0");
    if (P > 0 && (!radii || !max_radii || !visible)) return fail(GSR_ERR_ARG, "densify: null pointer");
    HIP_TRY(launch_dens_radii(P, radii, max_radii, visible, (hipStream_t)stream));
    return GSR_OK;
}

int gsr_densify_accumulate_grads(int P, const uint8_t *visible, const float *means2D_grad, float *grad_accum,
                                 float *vis_count, void *stream) {
    if (P < 0) return fail(GSR_ERR_ARG, "densify: P must be >= 0");
    if (P > 0 && (!visible || !means2D_grad || !grad_accum || !vis_count))
        return fail(GSR_ERR_ARG, "densify: null pointer");
    HIP_TRY(launch_dens_grads(P, visible, means2D_grad, grad_accum, vis_count, (hipStream_t)stream));
    return GSR_OK;
}

size_t gsr_densify_workspace_bytes(int P) { return DensWorkspace(P < 0 ? 0 : P).total; }

int gsr_densify_plan(const gsr_densify_settings *st, void *workspace, gsr_densify_counts *counts, void *stream) {
    DensArgs a;
    int rc = dens_args(st, a);
    if (rc) return rc;
    if (!workspace || !counts) return fail(GSR_ERR_ARG, "densify: null workspace / counts");
    memset(counts, 0, sizeof(*counts));
    if (a.P == 0) return GSR_OK;
    hipStream_t s = (hipStream_t)stream;
    const DensWorkspace L(a.P);
    { Phase ph(s, "densify_plan"); HIP_TRY(launch_dens_plan(a, (char *)workspace, s)); }
    uint32_t tot[4];
    HIP_TRY(hipMemcpyAsync(tot, (char *)workspace + L.totals, sizeof(tot), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    counts->n_keep_orig = (int)tot[0];
    counts->n_keep_clone = (int)tot[1];
    counts->n_split = (int)tot[2];
    counts->n_keep_split = (int)tot[3];
    const long long po = (long long)tot[0] + tot[1] + 2ll * tot[3];
    if (po > 0x7FFFFFFF) return fail(GSR_ERR_UNSUPPORTED, "densify: output too large");
    counts->P_out = (int)po;
    return GSR_OK;
}

int gsr_densify_split_stds(const gsr_densify_settings *st, const void *workspace, float *stds, void *stream) {
    DensArgs a;
    int rc = dens_args(st, a);
    if (rc) return rc;
    if (a.P == 0) return GSR_OK;
    if (!workspace || !stds) return fail(GSR_ERR_ARG, "densify: null workspace / stds");
    HIP_TRY(launch_dens_stds(a, (const char *)workspace, stds, (hipStream_t)stream));
    return GSR_OK;
}

int gsr_densify_apply(const gsr_densify_settings *st, const void *workspace, const gsr_densify_counts *counts,
                      const float *samples, int ncols, const gsr_densify_column *cols, void *stream) {
    DensArgs a;
    int rc = dens_args(st, a);
    if (rc) return rc;
    if (ncols < 0 || ncols > kDensMaxColumns) return fail(GSR_ERR_ARG, "densify: 0..%d columns", kDensMaxColumns);
    if (a.P == 0 || ncols == 0) return GSR_OK;
    if (!workspace || !cols || !counts) return fail(GSR_ERR_ARG, "densify: null workspace / counts / columns");
    if (counts->n_split > 0 && !samples) return fail(GSR_ERR_ARG, "densify: %d splits need samples", counts->n_split);
    DensColumns dc;
    memset(&dc, 0, sizeof(dc));
    dc.n = ncols;
    for (int k = 0; k < ncols; ++k) {
        const gsr_densify_column &c = cols[k];
        if (c.width <= 0 || !c.src || !c.dst) return fail(GSR_ERR_ARG, "densify: column %d has no data", k);
        if ((c.exp_avg == nullptr) != (c.exp_avg_sq == nullptr) || (c.exp_avg == nullptr) != (c.dst_exp_avg == nullptr) ||
            (c.dst_exp_avg == nullptr) != (c.dst_exp_avg_sq == nullptr))
            return fail(GSR_ERR_ARG, "densify: column %d: Adam moments must be given together", k);
        if (c.role == GSR_DENS_MEANS && c.width != 3) return fail(GSR_ERR_ARG, "densify: means need width 3");
        if (c.role == GSR_DENS_LOG_SCALES && c.width != 3) return fail(GSR_ERR_ARG, "densify: log_scales need width 3");
        dc.c[k] = DensColumn{c.width, c.role, c.src, c.exp_avg, c.exp_avg_sq, c.dst, c.dst_exp_avg, c.dst_exp_avg_sq};
    }
    hipStream_t s = (hipStream_t)stream;
    Phase ph(s, "densify_apply");
    HIP_TRY(launch_dens_apply(a, (const char *)workspace, samples, dc, s));
    return GSR_OK;
}

int gsr_adam_step(int ntensors, const gsr_adam_tensor *tensors, double beta1, double beta2, double eps,
                  void *stream) {
    if (ntensors < 0 || (ntensors > 0 && !tensors)) return fail(GSR_ERR_ARG, "adam: bad tensor list");
    hipStream_t s = (hipStream_t)stream;
    for (int k = 0; k < ntensors; ++k) {  // validate everything before launching anything
        const gsr_adam_tensor &a = tensors[k];
        if (a.numel < 0) return fail(GSR_ERR_ARG, "adam: tensor %d: negative numel", k);
        if (a.numel > 0 && (!a.param || !a.grad || !a.exp_avg || !a.exp_avg_sq))
            return fail(GSR_ERR_ARG, "adam: tensor %d: null pointer", k);
        if (a.numel > 0 && !(a.step >= 1.0)) return fail(GSR_ERR_ARG, "adam: tensor %d: step must be >= 1", k);
        if (adam_blocks(a.numel) > (1 << 30)) return fail(GSR_ERR_UNSUPPORTED, "adam: tensor %d too large", k);
    }
    Phase ph(s, "adam");
    AdamTable tab;
    auto reset = [&]() {
        memset(&tab, 0, sizeof(tab));
        tab.w1 = (float)(1.0 - beta1);
        tab.b2 = (float)beta2;
        tab.omb2 = (float)(1.0 - beta2);
        tab.eps = (float)eps;
    };
    reset();
    int nb = 0;
    for (int k = 0; k < ntensors; ++k) {
        const gsr_adam_tensor &a = tensors[k];
        if (a.numel == 0) continue;
        const int b = adam_blocks(a.numel);
        if (tab.n == kAdamMaxTensors || nb + (long long)b > (1ll << 30)) {  // table full: launch it
            tab.block_start[tab.n] = nb;
            HIP_TRY(launch_adam(tab, s));
            reset();
            nb = 0;
        }
        const double bc1 = 1.0 - std::pow(beta1, a.step), bc2 = 1.0 - std::pow(beta2, a.step);
        AdamTensor &t = tab.t[tab.n];
        t.param = a.param; t.grad = a.grad; t.exp_avg = a.exp_avg; t.exp_avg_sq = a.exp_avg_sq;
        t.n = a.numel;
        t.step_size = (float)((a.lr / bc1) * -1.0);
        t.bc2_sqrt = (float)std::pow(bc2, 0.5);
        const uintptr_t al = (uintptr_t)a.param | (uintptr_t)a.grad | (uintptr_t)a.exp_avg | (uintptr_t)a.exp_avg_sq;
        t.vec4 = (al & 15) == 0;
        tab.block_start[tab.n] = nb;
        nb += b;
        ++tab.n;
    }
    if (tab.n) {
        tab.block_start[tab.n] = nb;
        HIP_TRY(launch_adam(tab, s));
    }
    return GSR_OK;
}

int gsr_views_pack(int frames, int H, int W, const uint8_t *rgb, const uint8_t *seg, float *images,
                   float *seg_masks, void *stream) {
    if (frames < 0 || H < 0 || W < 0) return fail(GSR_ERR_ARG, "views_pack: negative size");
    if (frames == 0 || H == 0 || W == 0) return GSR_OK;
    if ((long long)H * W > (1ll << 29)) return fail(GSR_ERR_UNSUPPORTED, "views_pack: frame of %d x %d too large", H, W);
    if (frames > 65535) return fail(GSR_ERR_UNSUPPORTED, "views_pack: more than 65535 frames in one call");
    if (!rgb || !images) return fail(GSR_ERR_ARG, "views_pack: null rgb / images");
    if ((seg == nullptr) != (seg_masks == nullptr))
        return fail(GSR_ERR_ARG, "views_pack: seg and seg_masks must be given together");
    const int HW = H * W;
    if (HW % 4 == 0) {  // the vector path's alignment contract
        if (((uintptr_t)rgb & 3) || (seg && ((uintptr_t)seg & 3)) || ((uintptr_t)images & 15) ||
            (seg_masks && ((uintptr_t)seg_masks & 15)))
            return fail(GSR_ERR_ARG, "views_pack: rgb / seg must be 4-byte and outputs 16-byte aligned");
    }
    hipStream_t s = (hipStream_t)stream;
    Phase ph(s, "views_pack");
    HIP_TRY(launch_views_pack(frames, HW, rgb, seg, images, seg_masks, s));
    return GSR_OK;
}

int gsr_profile_enable(int on) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_on = on != 0;
    return GSR_OK;
}

int gsr_profile_select(const char *phases) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_sel = (phases && *phases) ? "," + std::string(phases) + "," : std::string();
    return GSR_OK;
}

int gsr_profile_reset(void) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_host_ms.clear();
    g_host_n.clear();
    for (auto &r : g_prof) { g_evpool.push_back(r.a); g_evpool.push_back(r.b); }
    g_prof.clear();
    return GSR_OK;
}

int gsr_profile_read(const char *phase, double *total_ms, int *count) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    double tot = 0; int n = 0;
    if (phase && !strncmp(phase, "host_", 5)) {  // host-side wall time of the named section
        if (total_ms) *total_ms = g_host_ms.count(phase) ? g_host_ms[phase] : 0.0;
        if (count) *count = g_host_n.count(phase) ? g_host_n[phase] : 0;
        return GSR_OK;
    }
    for (auto &r : g_prof) {
        if (phase && r.phase != phase) continue;
        if (hipEventSynchronize(r.b) != hipSuccess) return fail(GSR_ERR_HIP, "hipEventSynchronize failed");
        float ms = 0;
        if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) return fail(GSR_ERR_HIP, "hipEventElapsedTime failed");
        tot += ms; ++n;
    }
    if (total_ms) *total_ms = tot;
    if (count) *count = n;
    return GSR_OK;
}

}  // extern "C"
