// api.hip -- the C ABI of libgsr.so (declared in include/gsr.h): workspace ownership,
// argument validation, stage orchestration on the caller's stream, stage timing.
//
// gsr_forward replaces upstream `_C.rasterize_gaussians` / Rasterizer::forward
// (rasterizer_impl.cu), which the viewer reaches through renderer_cuda.py:211-224.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gsr.h"
#include "gsr_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define GSR_HIP(call, what)                                                                  \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail(GSR_E_HIP, std::string(what) + ": " + hipGetErrorString(e_));        \
    } while (0)

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
};

constexpr int kStages = 7;       // the chain on the caller's stream
constexpr int kAllStages = 8;    // + "color", on the second stream (overlaps stages 1..5)
constexpr int kTimingRing = 256;  // frames whose stage events are kept
// gsr_context::frame words: view 16, proj 16, campos 3 (+1), bg 3 (+1) floats, then the frame
// tag and the device K / overflow words k_col_scatter writes
constexpr int kFrameView = 0, kFrameProj = 16, kFrameCampos = 32, kFrameBg = 36, kFrameTag = 40,
              kFrameK = 41, kFrameWords = 44;
constexpr size_t kMaxGraphs = 4;

const char *kStageNames[kAllStages] = {"preprocess", "depth_sort", "scan",  "duplicate",
                                       "tile_sort",  "ranges",     "blend", "color"};

}  // namespace

struct gsr_context {
    int device = 0;
    // per-Gaussian workspace
    DevBuf records, strip_rect, sort_keys, partials, total, hist, digit_total, bin, chunk_first,
        rect_sorted, pair_count;
    DevBuf ds_a, ds_b;  // depth sort: (key, id) pairs between passes (ping-pong)
    DevBuf block_kept;  // depth sort compaction (strips): kept keys per 256-Gaussian block
    DevBuf color_ids;   // compacted strips: the kept ids the colour pass walks (4 B x P)
    hipEvent_t compacted = nullptr;  // the compacted ids are written (main -> second stream)
    DevBuf perm;    // the depth sort's result: Gaussian ids in depth order (kept ones)
    DevBuf ds_ctl;  // depth sort control words: kept count, key bits, per-tile key stats
    DevBuf col_hist;  // column-first binning: per-(Gaussian block, column) pair counts
    // per-pair workspace
    DevBuf tile_keys, tile_vals, tile_keys_alt, tile_vals_alt;
    DevBuf ranges_local;
    DevBuf tile_diff;  // difference-array partials of the second-stream tile ranges
    // pinned: [K from the device scan (debug), unused, K from the pair count, depth key bits D]
    // [4]: (frame tag << 32) | D from the depth sort's pass 0
    uint64_t *h_total = nullptr;
    unsigned long long *d_hostK = nullptr;  // device view of h_total + 2
    unsigned long long *d_hostD = nullptr;  // device view of h_total + 4
    uint32_t sort_tag = 0;                  // frames sorted on this context (tags h_total[4])
    // state of the last forward (for gsr_get_binning)
    bool have_forward = false;
    int64_t last_K = 0;
    uint32_t last_gx = 0, last_gy = 0, last_rb = 0, last_re = 0;
    uint32_t *last_point_list = nullptr, *last_tiles_local = nullptr;
    bool last_packed = false;             // last_point_list is a packed pair list (no keys)
    uint32_t last_id_mask = 0xFFFFFFFFu;  // packed word -> Gaussian id
    // options / timing
    int cull = 1;
    int fast = 1;
    int tile_sort_shape = 3;  // 8 waves x 8 keys/lane: fastest measured
    int fused_binning = 1;    // duplicate fused with the first tile-sort pass
    // tile ranges from the rects' per-tile counts on the second stream, before the colour (1;
    // the colour then overlaps the column count and scatter rather than the depth sort: C3 with
    // two frames in flight 3,470 -> 3,600 fps, serial +0.5 %, C2 +9 %, C4 and its strips even;
    // 2 = after the colour, the round-2 default; 0 = k_ranges on the main stream).  env
    // GSR_AUX_RANGES
    int aux_ranges = 1;
    // GSR_OPT_PACKED_PAIRS: one 32-bit word per (tile, Gaussian) pair -- the tile-id bits the
    // second tile-sort pass needs above the Gaussian id -- instead of a key and a value array
    // (needs the second-stream ranges; falls back when the bits do not fit)
    int packed_pairs = 1;
    // GSR_OPT_COLUMN_PAIRS: the first tile-sort pass on (Gaussian, column) segments of the
    // depth-sorted Gaussians instead of per pair (binning.hip k_col_count / k_col_scatter)
    int column_pairs = 1;
    // grid cap of the overlapped colour pass (0 = none: one wave per 64 Gaussians).  Uncapped
    // gives the best frame rate with two frames in flight (C3: 3,186 fps vs 3,010 at 256
    // blocks); 256 the best serial frame (0.369 vs 0.386 ms): the colour then takes fewer CUs
    // from the depth sort it overlaps (env GSR_COLOR_BLOCKS)
    int color_blocks = 0;
    // k_color: colour waves per SIMD (0 = as many as fit; -1 = auto: 3 below 4M Gaussians, else
    // 4 -- GSR_COLOR_WAVES sweeps on MI355X, C3 and a C4 strip)
    int color_waves = -1;
    // host learns D before queueing the depth sort's later passes: 1 / 0, or -1 = auto: only when
    // the previous frame had >= 4M pairs.  Waiting keeps the empty third pass off the GPU (C3:
    // 3,480 vs 3,340 frames/s) but holds the host to the GPU's progress, which host-bound small
    // frames (C2, a C3 strip: ~1M pairs) feel more (7,500 vs 8,000-9,300 frames/s in flight)
    int wait_D = -1;
    uint32_t blend_xcd_group = 16;  // tuning (env GSR_BLEND_XCD_GROUP)
    int aux_low_priority = 1;  // second stream at the lowest priority
    bool serial_color = false; // tuning (env GSR_SERIAL_COLOR): join right after the fork
    bool late_K = false;       // tuning (env GSR_LATE_K): also sync on the scan's total
    bool split_color = true;   // GSR_OPT_SPLIT_COLOR
    // depth sort compaction (GSR_OPT_COMPACT_SORT, env GSR_COMPACT_SORT): 1 on, 0 off, -1 auto
    // = on for strips of >= 4M Gaussians.  A strip keeps a fraction of the Gaussians; compacting
    // them first spares pass 0 the dropped keys (C4 1/8 strip: 2,017 -> 2,097 fps), but it
    // delays the pass-0 D the host waits for, which costs more than it saves on small frames
    // (C3 1/8 strip: 9,290 -> 7,170 fps with two frames in flight)
    int compact_sort = -1;
    // Stage timing: a ring of event sets, one per forward, read back after the timed region.
    int timing = 0;  // 0 off, 1 every stage, 2 the blend only, on every 8th forward
    int64_t forwards = 0;  // forwards since gsr_set_timing (mode 2's sampling)
    int64_t timed_frames = 0;
    hipEvent_t ev[kTimingRing][kStages + 1] = {};
    hipEvent_t ev_color[kTimingRing][2] = {};
    // second stream: k_color runs there between a fork after the preprocess and a join
    // before the blend
    hipStream_t aux = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    // Captured frames (GSR_OPT_GRAPH, env GSR_GRAPH; off by default): the whole forward as
    // one hipGraph, so a frame costs the host one staging launch + one graph launch (~9 us)
    // instead of ~20 launches, ~6 event calls and two waits (~100 us).  K is not known when
    // the graph is built: the pair buffers are sized for graph_cap and the device checks K
    // against it (k_col_scatter).  Measured on MI355X it does not pay: ROCm replays only
    // linear graphs as pre-built packet batches (a fork / join graph took 63-115 us to launch,
    // tools/micro/host_cost), and a linear frame gives up the second stream's overlap (C3:
    // 3,050 vs 3,510 frames/s; C2 and C3 strips even; small frames are bound by the GPU's
    // ~2-4 us per dependent kernel, not by the host).  DESIGN.md.
    int graph = 0;
    bool capturing = false;     // forward_impl is recording into cap_stream
    hipStream_t cap_stream = nullptr;
    DevBuf frame;               // per-frame staging (kFrame* word offsets below)
    uint32_t frame_tag = 0;     // frames launched as graphs (tags h_total[5])
    int64_t graph_cap = 0;      // pair capacity of the captured frames (0: not yet known)
    uint64_t buf_gen = 0;       // bumped by every reallocation (captured pointers go stale)
    // what a captured frame leaves for gsr_get_binning (set by forward_impl while capturing)
    uint32_t *cap_point_list = nullptr, *cap_tiles_local = nullptr;
    uint32_t cap_id_mask = 0xFFFFFFFFu;
    bool cap_packed = false;
    struct Graph {
        std::vector<uint64_t> key;
        hipGraphExec_t exec = nullptr;
        uint32_t *point_list = nullptr, *tiles_local = nullptr;
        uint32_t id_mask = 0xFFFFFFFFu;
        bool packed = false;
        uint64_t used = 0;
    };
    std::vector<Graph> graphs;  // at most kMaxGraphs, least recently used evicted
    uint64_t graph_clock = 0;
    bool graph_stats = false;
    double gs_acc[3] = {};
    uint64_t gs_n = 0;
};

namespace {

// Grow-only device buffer.  The stream is drained first so no in-flight kernel still reads
// the old allocation.
int grow(gsr_context *ctx, DevBuf &b, size_t bytes, hipStream_t s) {
    if (bytes <= b.cap) return GSR_OK;
    size_t want = std::max(bytes, b.cap + b.cap / 2);
    want = (want + 255) & ~size_t(255);
    if (b.p) {
        GSR_HIP(hipStreamSynchronize(s), "hipStreamSynchronize(grow)");
        if (ctx->aux) GSR_HIP(hipStreamSynchronize(ctx->aux), "hipStreamSynchronize(grow)");
        GSR_HIP(hipFree(b.p), "hipFree");
        b.p = nullptr;
        b.cap = 0;
    }
    if (hipMalloc(&b.p, want) != hipSuccess) {
        (void)hipGetLastError();
        b.p = nullptr;
        return fail(GSR_E_NOMEM, "hipMalloc of " + std::to_string(want) + " bytes failed");
    }
    b.cap = want;
    ++ctx->buf_gen;
    return GSR_OK;
}

// Grow-only buffer whose contents must start at zero (look-back granules, ticket).
int grow_zeroed(gsr_context *ctx, DevBuf &b, size_t bytes, hipStream_t s) {
    const void *before = b.p;
    int rc = grow(ctx, b, bytes, s);
    if (rc != GSR_OK) return rc;
    if (b.p != before) GSR_HIP(hipMemsetAsync(b.p, 0, b.cap, s), "hipMemsetAsync(zero-init)");
    return GSR_OK;
}

#define GSR_TRY(expr)                 \
    do {                              \
        int rc_ = (expr);             \
        if (rc_ != GSR_OK) return rc_; \
    } while (0)

int reserve_P(gsr_context *ctx, int64_t P, hipStream_t s) {
    const size_t n = (size_t)std::max<int64_t>(P, 1);
    GSR_TRY(grow(ctx, ctx->records, n * sizeof(gsr::SplatRecord), s));
    GSR_TRY(grow(ctx, ctx->strip_rect, n * 8, s));
    GSR_TRY(grow(ctx, ctx->sort_keys, n * 4, s));
    GSR_TRY(grow(ctx, ctx->ds_a, n * 8, s));
    GSR_TRY(grow(ctx, ctx->ds_b, n * 8, s));
    GSR_TRY(grow(ctx, ctx->block_kept, 4 * ((n + 255) / 256), s));
    GSR_TRY(grow(ctx, ctx->partials, (size_t)std::max<int64_t>(gsr_scan_blocks(P), 1) * 4, s));
    GSR_TRY(grow_zeroed(ctx, ctx->total, 16, s));  // [K (u64), look-back error flag (u32)]
    // per preprocess block: its pair count (8 B) and kept-key OR / AND (8 B)
    GSR_TRY(grow(ctx, ctx->pair_count, (size_t)std::max<int64_t>((P + 255) / 256, 1) * 16, s));
    GSR_TRY(grow(ctx, ctx->hist, (size_t)std::max(gsr_radix_hist_words(P),
                                                  gsr_depth_sort_hist_words(P)) * 4, s));
    // column-first binning's per-(block, column) counts: its own buffer, since reserve_K may
    // regrow hist between the count and the scatter
    GSR_TRY(grow(ctx, ctx->col_hist, (size_t)std::max<int64_t>(gsr_col_blocks(P), 1) * 256 * 4, s));
    // 256 words per radix pass; the depth sort's 4096 digits
    GSR_TRY(grow(ctx, ctx->digit_total,
                 (size_t)std::max(256 * GSR_RADIX_MAX_PASSES, gsr_depth_sort_digit_words()) * 4, s));
    GSR_TRY(grow(ctx, ctx->perm, n * 4, s));
    GSR_TRY(grow(ctx, ctx->ds_ctl, (size_t)gsr_depth_sort_ctl_words(P) * 4, s));
    GSR_TRY(grow(ctx, ctx->bin, n * 16, s));
    GSR_TRY(grow(ctx, ctx->rect_sorted, n * 8, s));
    return GSR_OK;
}

int reserve_K(gsr_context *ctx, int64_t K, hipStream_t s) {
    const size_t n = (size_t)std::max<int64_t>(K, 1);
    GSR_TRY(grow(ctx, ctx->tile_keys, n * 4, s));
    GSR_TRY(grow(ctx, ctx->tile_vals, n * 4, s));
    GSR_TRY(grow(ctx, ctx->tile_keys_alt, n * 4, s));
    GSR_TRY(grow(ctx, ctx->tile_vals_alt, n * 4, s));
    GSR_TRY(grow(ctx, ctx->hist, (size_t)gsr_radix_hist_words(K) * 4, s));
    GSR_TRY(grow(ctx, ctx->chunk_first, (size_t)(gsr_duplicate_chunks(K) + 1) * 4, s));
    return GSR_OK;
}

int bits_for(uint64_t max_value) {  // bits needed to represent every value <= max_value
    int b = 0;
    while (b < 32 && (max_value >> b) != 0) ++b;
    return b;
}

}  // namespace

// The thread's last-error message for the other translation units (ply_loader.hip).
int gsr_set_error(int code, const std::string &msg) { return fail(code, msg); }

extern "C" {

int gsr_abi_version(void) { return GSR_ABI_VERSION; }
const char *gsr_last_error(void) { return g_err.c_str(); }
const char *gsr_stage_name(int i) { return (i >= 0 && i < kAllStages) ? kStageNames[i] : ""; }

int gsr_create(gsr_context **out) {
    if (!out) return fail(GSR_E_INVALID, "gsr_create: out is NULL");
    *out = nullptr;
    gsr_context *ctx = new gsr_context();
    if (hipGetDevice(&ctx->device) != hipSuccess) {
        (void)hipGetLastError();
        delete ctx;
        return fail(GSR_E_HIP, "gsr_create: no HIP device");
    }
    if (hipHostMalloc(reinterpret_cast<void **>(&ctx->h_total), 8 * sizeof(uint64_t),
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void **>(&ctx->d_hostK), ctx->h_total + 2, 0) !=
            hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void **>(&ctx->d_hostD), ctx->h_total + 4, 0) !=
            hipSuccess) {
        (void)hipGetLastError();
        delete ctx;
        return fail(GSR_E_HIP, "gsr_create: hipHostMalloc failed");
    }
    std::memset(ctx->h_total, 0, 8 * sizeof(uint64_t));  // tag 0 never matches a frame
    int prio_least = 0, prio_greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess) {
        (void)hipGetLastError();
        prio_least = prio_greatest = 0;
    }
    const char *env_prio = std::getenv("GSR_AUX_PRIORITY");  // tuning: "0" = default priority
    ctx->aux_low_priority = env_prio ? std::atoi(env_prio) : 1;
    const char *env_cb = std::getenv("GSR_COLOR_BLOCKS");    // tuning: grid cap, 0 = none
    if (env_cb) ctx->color_blocks = std::atoi(env_cb);
    const char *env_cw = std::getenv("GSR_COLOR_WAVES");     // tuning: 0 = no cap
    if (env_cw) ctx->color_waves = std::atoi(env_cw);
    const char *env_cp = std::getenv("GSR_COLUMN_PAIRS");
    if (env_cp) ctx->column_pairs = std::atoi(env_cp);
    const char *env_pp = std::getenv("GSR_PACKED_PAIRS");
    if (env_pp) ctx->packed_pairs = std::atoi(env_pp);
    const char *env_ar = std::getenv("GSR_AUX_RANGES");
    if (env_ar) ctx->aux_ranges = std::atoi(env_ar);
    const char *env_cs = std::getenv("GSR_COMPACT_SORT");
    if (env_cs) ctx->compact_sort = std::atoi(env_cs);
    const char *env_xg = std::getenv("GSR_BLEND_XCD_GROUP");
    if (env_xg) ctx->blend_xcd_group = (uint32_t)std::atoi(env_xg);
    ctx->serial_color = std::getenv("GSR_SERIAL_COLOR") != nullptr;
    const char *env_gr = std::getenv("GSR_GRAPH");  // 0: every frame on the stream
    if (env_gr) ctx->graph = std::atoi(env_gr) != 0;
    ctx->graph_stats = std::getenv("GSR_GRAPH_STATS") != nullptr;
    const char *env_wd = std::getenv("GSR_WAIT_D");  // tuning: 0 = queue every pass at once
    if (env_wd) ctx->wait_D = std::atoi(env_wd);
    ctx->late_K = std::getenv("GSR_LATE_K") != nullptr;
    bool ok = hipStreamCreateWithPriority(&ctx->aux, hipStreamNonBlocking,
                                          ctx->aux_low_priority ? prio_least : 0) == hipSuccess &&
              // stream-to-stream hand-offs on one device: a device-scope release suffices
              hipEventCreateWithFlags(&ctx->fork, hipEventDisableTiming | hipEventReleaseToDevice) ==
                  hipSuccess &&
              hipEventCreateWithFlags(&ctx->join, hipEventDisableTiming | hipEventReleaseToDevice) ==
                  hipSuccess &&
              hipEventCreateWithFlags(&ctx->compacted,
                                      hipEventDisableTiming | hipEventReleaseToDevice) == hipSuccess;
    // timing events only time: no system-scope fence (cache writeback) when they complete
    for (auto &set : ctx->ev)
        for (auto &e : set) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableSystemFence) == hipSuccess;
    for (auto &set : ctx->ev_color)
        for (auto &e : set) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableSystemFence) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        gsr_destroy(ctx);
        return fail(GSR_E_HIP, "gsr_create: stream / event creation failed");
    }
    *out = ctx;
    return GSR_OK;
}

void gsr_destroy(gsr_context *ctx) {
    if (!ctx) return;
    (void)hipDeviceSynchronize();
    DevBuf *bufs[] = {&ctx->records,       &ctx->strip_rect,    &ctx->sort_keys,
                      &ctx->ds_a,          &ctx->ds_b,          &ctx->block_kept,
                      &ctx->partials,      &ctx->total,         &ctx->hist,
                      &ctx->digit_total,   &ctx->bin,           &ctx->chunk_first,
                      &ctx->rect_sorted,   &ctx->pair_count,    &ctx->perm,
                      &ctx->ds_ctl,
                      &ctx->tile_keys,     &ctx->tile_vals,
                      &ctx->tile_keys_alt, &ctx->tile_vals_alt, &ctx->ranges_local,
                      &ctx->tile_diff,     &ctx->col_hist,      &ctx->frame,
                      &ctx->color_ids};
    for (auto &e : ctx->graphs) (void)hipGraphExecDestroy(e.exec);
    if (ctx->cap_stream) (void)hipStreamDestroy(ctx->cap_stream);
    for (DevBuf *b : bufs)
        if (b->p) (void)hipFree(b->p);
    for (auto &set : ctx->ev)
        for (auto &e : set)
            if (e) (void)hipEventDestroy(e);
    for (auto &set : ctx->ev_color)
        for (auto &e : set)
            if (e) (void)hipEventDestroy(e);
    if (ctx->fork) (void)hipEventDestroy(ctx->fork);
    if (ctx->join) (void)hipEventDestroy(ctx->join);
    if (ctx->compacted) (void)hipEventDestroy(ctx->compacted);
    if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
    if (ctx->h_total) (void)hipHostFree(ctx->h_total);
    delete ctx;
}

int gsr_reserve(gsr_context *ctx, int64_t P, int64_t K) {
    if (!ctx || P < 0 || K < 0) return fail(GSR_E_INVALID, "gsr_reserve: bad arguments");
    GSR_TRY(reserve_P(ctx, P, nullptr));
    GSR_TRY(reserve_K(ctx, K, nullptr));
    GSR_HIP(hipDeviceSynchronize(), "gsr_reserve");
    return GSR_OK;
}

int gsr_set_option(gsr_context *ctx, int option, int64_t value) {
    if (!ctx) return fail(GSR_E_INVALID, "gsr_set_option: NULL context");
    if (option == GSR_OPT_BLEND_CULL) {
        ctx->cull = value ? 1 : 0;
        return GSR_OK;
    }
    if (option == GSR_OPT_BLEND_FAST) {
        if (value < 0 || value > 1) return fail(GSR_E_INVALID, "gsr_set_option: fast 0..1");
        ctx->fast = (int)value;
        return GSR_OK;
    }
    if (option == GSR_OPT_SPLIT_COLOR) {
        ctx->split_color = value != 0;
        return GSR_OK;
    }
    if (option == GSR_OPT_FUSED_BINNING) {
        ctx->fused_binning = value ? 1 : 0;
        return GSR_OK;
    }
    if (option == GSR_OPT_COLUMN_PAIRS) {
        ctx->column_pairs = value ? 1 : 0;
        return GSR_OK;
    }
    if (option == GSR_OPT_PACKED_PAIRS) {
        ctx->packed_pairs = value ? 1 : 0;
        return GSR_OK;
    }
    if (option == GSR_OPT_COMPACT_SORT) {
        if (value < -1 || value > 1) return fail(GSR_E_INVALID, "gsr_set_option: compact -1..1");
        ctx->compact_sort = (int)value;
        return GSR_OK;
    }
    if (option == GSR_OPT_GRAPH) {
        ctx->graph = value ? 1 : 0;
        return GSR_OK;
    }
    if (option == GSR_OPT_TILE_SORT_SHAPE) {
        if (value < 0 || value > 5) return fail(GSR_E_INVALID, "gsr_set_option: shape 0..5");
        ctx->tile_sort_shape = (int)value;
        return GSR_OK;
    }
    return fail(GSR_E_INVALID, "gsr_set_option: unknown option " + std::to_string(option));
}

int gsr_set_timing(gsr_context *ctx, int enable) {
    if (!ctx) return fail(GSR_E_INVALID, "gsr_set_timing: NULL context");
    if (enable < 0 || enable > 2) return fail(GSR_E_INVALID, "gsr_set_timing: mode 0..2");
    ctx->timing = enable;
    ctx->forwards = 0;
    ctx->timed_frames = 0;
    return GSR_OK;
}

// Mean per-stage time (ms) over the timed forwards since gsr_set_timing(1) (the most recent
// kTimingRing of them).  Waits for the last one; returns the number of frames averaged in
// *n_frames if non-NULL.  Return value: number of stages.
int gsr_stage_times(gsr_context *ctx, float *ms, int n) {
    if (!ctx || (!ms && n > 0)) return fail(GSR_E_INVALID, "gsr_stage_times: bad arguments");
    if (ctx->timed_frames == 0) return fail(GSR_E_STATE, "gsr_stage_times: no timed forward yet");
    const int64_t frames = std::min<int64_t>(ctx->timed_frames, kTimingRing);
    const int64_t last = (ctx->timed_frames - 1) % kTimingRing;
    GSR_HIP(hipEventSynchronize(ctx->ev[last][kStages]), "hipEventSynchronize");
    const bool all = ctx->timing != 2;  // mode 2 recorded the blend's two events only
    double acc[kAllStages] = {};
    for (int64_t f = 0; f < frames; ++f) {
        const int64_t slot = (ctx->timed_frames - 1 - f) % kTimingRing;
        for (int i = all ? 0 : kStages - 1; i < kStages; ++i) {
            float t = 0.f;
            GSR_HIP(hipEventElapsedTime(&t, ctx->ev[slot][i], ctx->ev[slot][i + 1]),
                    "hipEventElapsedTime");
            acc[i] += t;
        }
        if (all) {
            float t = 0.f;
            GSR_HIP(hipEventElapsedTime(&t, ctx->ev_color[slot][0], ctx->ev_color[slot][1]),
                    "hipEventElapsedTime");
            acc[kStages] += t;
        }
    }
    for (int i = 0; i < kAllStages && i < n; ++i) ms[i] = (float)(acc[i] / (double)frames);
    return kAllStages;
}

// The forward on stream s.  ctx->capturing: s is recording a captured frame (gsr_forward):
// camera and bg come from ctx->frame, K is not waited for (the binning is sized for
// ctx->graph_cap and reads K on the device) and nothing is published for the host but K.
static int forward_impl(gsr_context *ctx, const gsr_gaussians *g, const gsr_raster_settings *st,
                        gsr_outputs *out, hipStream_t s) {
    const bool cap_mode = ctx->capturing;
    float *frame = static_cast<float *>(ctx->frame.p);
    uint32_t *d_K = cap_mode ? reinterpret_cast<uint32_t *>(frame) + kFrameK : nullptr;
    const int64_t P = g->P;
    const int W = st->image_width, H = st->image_height;
    if (P < 0 || P > (int64_t)UINT32_MAX) return fail(GSR_E_INVALID, "gsr_forward: bad P");
    if (W <= 0 || H <= 0) return fail(GSR_E_INVALID, "gsr_forward: image size must be positive");
    if (!out->color || (P > 0 && !out->radii))
        return fail(GSR_E_INVALID, "gsr_forward: color and radii outputs are required");
    if (P > 0) {
        if (!g->means3D || !g->opacities)
            return fail(GSR_E_INVALID, "gsr_forward: means3D and opacities are required");
        if ((g->shs == nullptr) == (g->colors_precomp == nullptr))
            return fail(GSR_E_INVALID,
                        "Please provide excatly one of either SHs or precomputed colors!");
        if (((g->scales == nullptr || g->rotations == nullptr) && g->cov3D_precomp == nullptr) ||
            ((g->scales != nullptr || g->rotations != nullptr) && g->cov3D_precomp != nullptr))
            return fail(GSR_E_INVALID, "Please provide exactly one of either scale/rotation pair "
                                       "or precomputed 3D covariance!");
        if (g->shs && (g->M <= 0 || g->D < 0 || g->D > 3 || (g->D + 1) * (g->D + 1) > g->M))
            return fail(GSR_E_INVALID, "gsr_forward: sh_degree " + std::to_string(g->D) +
                                           " needs (deg+1)^2 <= " + std::to_string(g->M) +
                                           " stored coefficients (deg <= 3)");
        if (!st->viewmatrix || !st->projmatrix || (g->shs && !st->campos))
            return fail(GSR_E_INVALID, "gsr_forward: camera matrices are required");
    }
    if (!st->bg) return fail(GSR_E_INVALID, "gsr_forward: bg is required");

    const uint32_t gx = (uint32_t)((W + GSR_TILE_X - 1) / GSR_TILE_X);
    const uint32_t gy = (uint32_t)((H + GSR_TILE_Y - 1) / GSR_TILE_Y);
    if (gx > 0xFFFFu || gy > 0xFFFFu)  // packed 16-bit tile rects (preprocess.hip)
        return fail(GSR_E_INVALID, "gsr_forward: image larger than 65535 tiles per side");
    uint32_t rb = 0, re = gy;
    if (st->tile_row_begin != 0 || st->tile_row_end != 0) {
        if (st->tile_row_begin < 0 || st->tile_row_end > (int)gy ||
            st->tile_row_begin >= st->tile_row_end)
            return fail(GSR_E_INVALID, "gsr_forward: bad tile row strip");
        rb = (uint32_t)st->tile_row_begin;
        re = (uint32_t)st->tile_row_end;
    }
    const uint32_t rows_tiles = re - rb;
    const int y0 = (int)(rb * GSR_TILE_Y);
    const int rows_out = std::min(H, (int)(re * GSR_TILE_Y)) - y0;
    const uint64_t T_strip = (uint64_t)gx * rows_tiles;

    ctx->have_forward = false;
    const bool dbg = st->debug != 0;
    hipEvent_t *ev = ctx->ev[ctx->timed_frames % kTimingRing];
    // this forward's timing: mode 1 every stage; mode 2 the blend, on every 8th forward
    const int tmode = ctx->timing == 1 ? 1 : (ctx->timing == 2 && ctx->forwards++ % 8 == 0) ? 2 : 0;
    auto stage_end = [&](int i) -> int {
        if (tmode == 1 || (tmode == 2 && i >= 5))
            GSR_HIP(hipEventRecord(ev[i + 1], s), "hipEventRecord");
        if (dbg) {
            GSR_HIP(hipStreamSynchronize(s), std::string("stage ") + kStageNames[i]);
            GSR_HIP(hipGetLastError(), std::string("stage ") + kStageNames[i]);
        }
        return GSR_OK;
    };

    GSR_TRY(reserve_P(ctx, P, s));
    GSR_TRY(grow(ctx, ctx->ranges_local, (size_t)std::max<uint64_t>(T_strip, 1) * 8, s));
    // tile ranges on the second stream (from the rects' per-tile counts) when the strip's
    // difference array fits in LDS; else k_ranges over the sorted keys on the main stream
    const uint32_t diff_cells = gsr_tile_diff_cells(gx, rows_tiles);
    const bool aux_ranges = ctx->split_color && ctx->fused_binning &&
                            ctx->aux_ranges && diff_cells <= kTileDiffMaxCells;
    if (aux_ranges)
        GSR_TRY(grow(ctx, ctx->tile_diff, (size_t)kTileDiffBlocks * diff_cells * 4, s));

    if (P == 0) {  // upstream returns the zero-initialised image without rendering
        GSR_HIP(hipMemsetAsync(out->color, 0, (size_t)3 * rows_out * W * sizeof(float), s),
                "hipMemsetAsync(color)");
        GSR_HIP(hipMemsetAsync(ctx->ranges_local.p, 0, T_strip * 8, s), "hipMemsetAsync");
        out->num_rendered = 0;
        ctx->last_K = 0;
        ctx->last_gx = gx; ctx->last_gy = gy; ctx->last_rb = rb; ctx->last_re = re;
        ctx->last_point_list = static_cast<uint32_t *>(ctx->tile_vals.p);
        ctx->last_id_mask = 0xFFFFFFFFu;
        ctx->last_packed = false;
        ctx->last_tiles_local = static_cast<uint32_t *>(ctx->tile_keys.p);
        ctx->have_forward = true;
        return GSR_OK;
    }

    if (tmode == 1) GSR_HIP(hipEventRecord(ev[0], s), "hipEventRecord");

    // ---- 1. preprocess -------------------------------------------------------------------
    GsrPreprocessArgs pa{};
    pa.P = P;
    pa.D = g->D;
    pa.M = g->M;
    pa.scale_modifier = g->scale_modifier;
    pa.means3D = g->means3D;
    pa.scales = g->scales;
    pa.rotations = g->rotations;
    pa.opacities = g->opacities;
    pa.shs = g->shs;
    pa.colors_precomp = g->colors_precomp;
    pa.cov3D_precomp = g->cov3D_precomp;
    pa.viewmatrix = cap_mode ? frame + kFrameView : st->viewmatrix;
    pa.projmatrix = cap_mode ? frame + kFrameProj : st->projmatrix;
    pa.campos = cap_mode ? (st->campos ? frame + kFrameCampos : nullptr) : st->campos;
    pa.frame_tag = cap_mode ? reinterpret_cast<const uint32_t *>(frame) + kFrameTag : nullptr;
    pa.tanfovx = st->tanfovx;
    pa.tanfovy = st->tanfovy;
    // rasterizer_impl.cu: focal_y = height / (2.0f * tan_fovy); focal_x likewise (float).
    pa.focal_y = (float)H / (2.0f * st->tanfovy);
    pa.focal_x = (float)W / (2.0f * st->tanfovx);
    pa.W = W;
    pa.H = H;
    pa.grid_x = gx;
    pa.grid_y = gy;
    pa.row_begin = rb;
    pa.row_end = re;
    pa.prefiltered = st->prefiltered;
    pa.sh_vec4 = (g->shs && g->M == 16 && (reinterpret_cast<uintptr_t>(g->shs) & 15) == 0) ? 1 : 0;
    pa.rot_vec4 = (g->rotations && (reinterpret_cast<uintptr_t>(g->rotations) & 15) == 0) ? 1 : 0;
    pa.radii = out->radii;
    pa.records = static_cast<gsr::SplatRecord *>(ctx->records.p);
    pa.sort_keys = static_cast<uint32_t *>(ctx->sort_keys.p);
    const bool compact_sort =
        ctx->compact_sort < 0 ? (rows_tiles < gy && P >= (4 << 20)) : ctx->compact_sort != 0;
    pa.block_kept = compact_sort ? static_cast<uint32_t *>(ctx->block_kept.p) : nullptr;
    pa.strip_rect = static_cast<uint2 *>(ctx->strip_rect.p);
    pa.block_pairs = static_cast<uint64_t *>(ctx->pair_count.p);
    pa.host_K = ctx->d_hostK;
    pa.depths = out->depths;
    pa.means2D = out->means2D;
    pa.conic_opacity = out->conic_opacity;
    pa.rgb = out->rgb;
    pa.tiles_touched = out->tiles_touched;
    if (pa.conic_opacity && (reinterpret_cast<uintptr_t>(pa.conic_opacity) & 15) != 0)
        return fail(GSR_E_INVALID, "gsr_forward: conic_opacity output must be 16-B aligned");
    const bool split_color = ctx->split_color;
    // compacted strip frames: the colour pass walks the depth sort's compacted kept ids
    // (k_color_ids) instead of every Gaussian's rect -- at a 1/8 strip of 6M Gaussians a lane
    // in ~8 had a row to read
    const bool color_ids = compact_sort && split_color && !cap_mode && gsr_color_ids_ok(pa);
    if (color_ids) GSR_TRY(grow(ctx, ctx->color_ids, (size_t)P * 4, s));
    GSR_HIP(gsr_launch_preprocess(pa, !split_color, s), "preprocess launch");
    hipEvent_t *evc = ctx->ev_color[ctx->timed_frames % kTimingRing];
    struct JoinGuard {
        hipStream_t s;
        hipEvent_t join;
        bool done = true;
        ~JoinGuard() {
            if (!done) (void)hipStreamWaitEvent(s, join, 0);
        }
    } join_guard{s, ctx->join};
    // fork point of the second stream (colour, K, tile ranges): right after the preprocess.  Its
    // work is queued after the depth sort's first pass, so the host hands the critical chain to
    // the GPU first (queueing ~10 second-stream commands first left the main queue idle ~40 us
    // on a strip frame, where the host's submission rate is the bound)
    // (a captured frame is one stream: a graph with a fork / join launches ~10x slower on the
    // host -- ROCm replays only linear graphs as pre-built packet batches, tools/micro/host_cost)
    if (split_color && !cap_mode) GSR_HIP(hipEventRecord(ctx->fork, s), "hipEventRecord(fork)");
    if (!split_color && tmode == 1) {  // no colour stage: record an empty interval
        GSR_HIP(hipEventRecord(evc[0], s), "hipEventRecord");
        GSR_HIP(hipEventRecord(evc[1], s), "hipEventRecord");
    }
    GSR_TRY(stage_end(0));

    // ---- 2. stable sort of the Gaussians by view depth (depth_sort.hip) -------------------
    // compacting: Gaussians without pairs in the strip (sentinel keys) are dropped by the first
    // pass; the count of the rest lands in ds_ctl[0] (device), the pass count is decided there
    uint32_t *hist = static_cast<uint32_t *>(ctx->hist.p);
    uint32_t *digit_total = static_cast<uint32_t *>(ctx->digit_total.p);
    uint32_t *d_valid = static_cast<uint32_t *>(ctx->ds_ctl.p);
    uint32_t *perm = static_cast<uint32_t *>(ctx->perm.p);
    uint2 *ds_a = static_cast<uint2 *>(ctx->ds_a.p), *ds_b = static_cast<uint2 *>(ctx->ds_b.p);
    // compacted keys / ids live in ds_b until pass 1 overwrites it
    uint32_t *keys_c = reinterpret_cast<uint32_t *>(ds_b), *ids_c = keys_c + P;
    const uint32_t tag = ++ctx->sort_tag;
    auto depth_sort = [&](int p0, int p1) {
        return compact_sort
                   ? gsr_depth_sort_compacted(
                         pa.sort_keys, P, pa.block_kept, keys_c, ids_c, ds_a, ds_b, perm, hist,
                         digit_total, d_valid, p0, p1, s, cap_mode ? nullptr : ctx->d_hostD, tag,
                         color_ids ? static_cast<uint32_t *>(ctx->color_ids.p) : nullptr,
                         color_ids ? ctx->compacted : nullptr)
                   : gsr_depth_sort(pa.sort_keys, P, 1, ds_a, ds_b, perm, hist, digit_total,
                                    d_valid, p0, p1, s, cap_mode ? nullptr : ctx->d_hostD, tag);
    };
    GSR_HIP(depth_sort(0, 1), "depth sort launch");
    if (split_color) {
        // second stream: colour, overlapped with the depth sort and the binning
        hipStream_t as = cap_mode ? s : ctx->aux;
        if (!cap_mode)
            GSR_HIP(hipStreamWaitEvent(ctx->aux, ctx->fork, 0), "hipStreamWaitEvent(fork)");
        // K (the pair count) first: k_publish_K sums the preprocess blocks' counts into pinned
        // memory; the host waits for it only after the depth sort and the scan are enqueued,
        // so the GPU does not idle on the host round trip
        pa.k_tag = cap_mode ? 0u : (tag ? tag : 1u);  // (launched after the preprocess)
        GSR_HIP(gsr_launch_count_pairs(pa, as), "pair count launch");
        if (tmode == 1) GSR_HIP(hipEventRecord(evc[0], as), "hipEventRecord");
        // (with the compacted ids the ranges go first: the colour waits for the compaction)
        const bool ranges_first = aux_ranges && (ctx->aux_ranges == 1 || color_ids);
        if (ranges_first) {
            uint32_t *part = static_cast<uint32_t *>(ctx->tile_diff.p);
            GSR_HIP(gsr_launch_tile_ranges_aux(pa.strip_rect, P, gx, rows_tiles, part,
                                               static_cast<uint2 *>(ctx->ranges_local.p), as),
                    "tile ranges launch");
        }
        // (in a captured frame the colour runs alone: no cap)
        const int color_waves = ctx->color_waves >= 0 ? ctx->color_waves
                                : cap_mode            ? 0
                                : P < (4 << 20)       ? 3
                                                      : 4;
        if (color_ids) {
            GSR_HIP(hipStreamWaitEvent(as, ctx->compacted, 0), "hipStreamWaitEvent(compacted)");
            GSR_HIP(gsr_launch_color_ids(pa, static_cast<const uint32_t *>(ctx->color_ids.p),
                                         d_valid, color_waves, as),
                    "color launch");
        } else {
            GSR_HIP(gsr_launch_color(pa, ctx->color_blocks, color_waves, as), "color launch");
        }
        if (aux_ranges && !ranges_first) {
            uint32_t *part = static_cast<uint32_t *>(ctx->tile_diff.p);
            GSR_HIP(gsr_launch_tile_ranges_aux(pa.strip_rect, P, gx, rows_tiles, part,
                                               static_cast<uint2 *>(ctx->ranges_local.p), as),
                    "tile ranges launch");
        }
        if (tmode == 1) GSR_HIP(hipEventRecord(evc[1], as), "hipEventRecord");
        if (!cap_mode) {
            GSR_HIP(hipEventRecord(ctx->join, ctx->aux), "hipEventRecord(join)");
            // every exit from here on (errors included) leaves the caller's stream behind the
            // join, so k_color never outlives the caller's view of its inputs
            join_guard.done = false;
        }
        if (dbg) GSR_HIP(hipStreamSynchronize(ctx->aux), "stage color");
        if (ctx->serial_color && !cap_mode)
            GSR_HIP(hipStreamWaitEvent(s, ctx->join, 0), "hipStreamWaitEvent");
    }
    // D (the bits in which the kept depth keys differ) arrives in pinned memory from pass 0's
    // scan, tagged with this frame, while pass 0's downsweep runs: the host then queues only the
    // passes D needs before the GPU reaches them.  If it does not arrive in 50 ms (a GPU still
    // busy with earlier frames), all passes are queued and the unneeded ones exit at once.
    int depth_passes = 3;
    if (!cap_mode && (ctx->wait_D > 0 || (ctx->wait_D < 0 && ctx->last_K >= (4 << 20)))) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spin = 0;; ++spin) {
            const uint64_t v = __atomic_load_n(&ctx->h_total[4], __ATOMIC_ACQUIRE);
            if ((uint32_t)(v >> 32) == tag) {
                depth_passes = gsr_depth_sort_passes((uint32_t)v);
                break;
            }
            if ((spin & 1023u) == 1023u &&
                std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50))
                break;
        }
    }
    GSR_HIP(depth_sort(1, depth_passes), "depth sort launch");
    GSR_TRY(stage_end(1));

    // ---- 3. offsets scan over depth-sorted strip tile counts; K readback --------------------
    uint32_t *partials = static_cast<uint32_t *>(ctx->partials.p);
    uint64_t *d_total = static_cast<uint64_t *>(ctx->total.p);
    uint2 *rect_sorted = static_cast<uint2 *>(ctx->rect_sorted.p);
    // column-first pair generation: packed word = strip-local tile row << col_shift | id
    const int ybits = rows_tiles > 1 ? bits_for(rows_tiles - 1) : 0;
    const int col_shift = 32 - ybits;
    const bool colpairs = ctx->column_pairs && ctx->fused_binning &&
                          aux_ranges && gx <= 256 && rows_tiles <= 256 &&
                          (col_shift == 32 || (uint64_t)P <= (1ull << col_shift));
    if (colpairs) {  // per-column pair counts of the depth-sorted Gaussians + their scan
        GSR_HIP(gsr_launch_col_pairs_count(perm, pa.strip_rect, P, d_valid, rect_sorted,
                                           static_cast<uint32_t *>(ctx->col_hist.p), digit_total,
                                           s),
                "column count launch");
    } else {
        GSR_HIP(gsr_launch_scan_reduce(perm, pa.strip_rect, P, d_valid, partials, rect_sorted, s),
                "scan launch");
        GSR_HIP(gsr_launch_scan_partials(partials, gsr_scan_blocks(P), d_total, s),
                "scan launch");
    }
    const bool check_device_total =
        !colpairs && (dbg || ctx->late_K || !split_color);
    if (check_device_total)  // K from the device (debug mode: checked against the pair count)
        GSR_HIP(hipMemcpyAsync(ctx->h_total, d_total, 16, hipMemcpyDeviceToHost, s),
                "hipMemcpyAsync(num_rendered)");
    GSR_TRY(stage_end(2));
    // K (the pair count, which sizes the binning) from the second stream's pair count,
    // published in pinned memory ~20 us after the preprocess; the host waits for it only after
    // the sort and the column counts are queued
    uint64_t K = 0;
    if (cap_mode) {
        K = (uint64_t)ctx->graph_cap;  // an upper bound; the device knows the real K
        if (!colpairs) return fail(GSR_E_STATE, "gsr_forward: frame not capturable");
    } else if (split_color) {
        // spin on the frame's K tag (pinned memory, written by k_publish_K after K): a sleeping
        // event wait adds wake-up jitter to every frame (and its record a host call); after
        // 50 ms without the tag, wait for the second stream instead (it reports a fault)
        const uint64_t want = pa.k_tag;
        const auto t0 = std::chrono::steady_clock::now();
        bool got = false;
        for (uint32_t spin = 0;; ++spin) {
            if (__atomic_load_n(&ctx->h_total[7], __ATOMIC_ACQUIRE) == want) {
                got = true;
                break;
            }
            if ((spin & 1023u) == 1023u &&
                std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50))
                break;
        }
        if (!got) GSR_HIP(hipStreamSynchronize(ctx->aux), "hipStreamSynchronize(pair count)");
        K = __atomic_load_n(&ctx->h_total[2], __ATOMIC_ACQUIRE);
        if (dbg) {  // the pair count's D and the sort's own D (pass 0) agree
            uint32_t ctl2[2];
            GSR_HIP(hipMemcpyAsync(ctl2, d_valid, 8, hipMemcpyDeviceToHost, s),
                    "hipMemcpyAsync(ctl)");
            GSR_HIP(hipStreamSynchronize(s), "hipStreamSynchronize(ctl)");
            if (ctl2[1] != (uint32_t)ctx->h_total[3])
                return fail(GSR_E_HIP, "gsr_forward: depth key bits mismatch (pair count " +
                                           std::to_string(ctx->h_total[3]) + ", sort " +
                                           std::to_string(ctl2[1]) + ")");
        }
    }
    if (check_device_total) {
        GSR_HIP(hipStreamSynchronize(s), "hipStreamSynchronize(num_rendered)");
        if (!split_color) K = ctx->h_total[0];
        if (ctx->h_total[0] != K)
            return fail(GSR_E_HIP, "gsr_forward: pair count mismatch (preprocess " +
                                       std::to_string(K) + ", scan " +
                                       std::to_string(ctx->h_total[0]) + ")");
    }
    if (K > (uint64_t)UINT32_MAX - 4096)
        return fail(GSR_E_INVALID, "gsr_forward: more than 2^32-4097 (Gaussian, tile) pairs");
    GSR_TRY(reserve_K(ctx, (int64_t)K, s));

    // ---- 4. duplicate into (tile, Gaussian) pairs, depth order, load-balanced by output ------
    const int tbits = T_strip > 1 ? bits_for(T_strip - 1) : 0;
    uint32_t *tk = static_cast<uint32_t *>(ctx->tile_keys.p);
    uint32_t *tv = static_cast<uint32_t *>(ctx->tile_vals.p);
    uint32_t *tk_alt = static_cast<uint32_t *>(ctx->tile_keys_alt.p);
    uint32_t *tv_alt = static_cast<uint32_t *>(ctx->tile_vals_alt.p);
    uint4 *bin = static_cast<uint4 *>(ctx->bin.p);
    uint32_t *chunk_first = static_cast<uint32_t *>(ctx->chunk_first.p);
    hist = static_cast<uint32_t *>(ctx->hist.p);  // may have been regrown
    const GsrRadixPlan tplan = gsr_radix_plan(0, tbits);
    const bool fused = ctx->fused_binning != 0;
    // packed pair list: word = (tile id >> first-pass bits) << pack_shift | Gaussian id; the
    // pair keys are not stored (the ranges come from the second stream)
    const int high_bits = tplan.n == 2 ? tplan.nbits[1] : 0;
    const int pack_shift = 32 - high_bits;
    const bool packed = !colpairs && ctx->packed_pairs && fused && aux_ranges && tplan.n <= 2 &&
                        (pack_shift == 32 || (uint64_t)P <= (1ull << pack_shift));
    const int word_shift = colpairs ? col_shift : pack_shift;
    const uint32_t id_mask = ((packed || colpairs) && word_shift < 32) ? (1u << word_shift) - 1u
                                                                       : 0xFFFFFFFFu;
    if (K > 0 && colpairs) {
        GSR_HIP(gsr_launch_col_pairs_scatter(perm, rect_sorted, P, d_valid,
                                             static_cast<const uint32_t *>(ctx->col_hist.p),
                                             digit_total, col_shift, tv_alt, s,
                                             cap_mode ? (uint32_t)K : 0xFFFFFFFFu, d_K),
                "column scatter launch");
        std::swap(tv, tv_alt);
    } else if (K > 0) {
        GSR_HIP(gsr_launch_scan_down(perm, rect_sorted, partials, P, d_valid, d_total, bin,
                                     chunk_first, s),
                "scan_down launch");
        if (fused) {
            // duplicate fused with the first tile-sort pass (a single pass when tbits == 0)
            GSR_HIP(gsr_launch_dup_sort_pass(bin, chunk_first, (int64_t)K, gx,
                                             tplan.n ? tplan.shift[0] : 0,
                                             tplan.n ? tplan.nbits[0] : 0, hist, digit_total,
                                             tk_alt, tv_alt,
                                             static_cast<uint2 *>(ctx->ranges_local.p),
                                             aux_ranges ? 0u : (uint32_t)T_strip, s,
                                             packed ? pack_shift : -1),
                    "duplicate launch");
            std::swap(tk, tk_alt);
            std::swap(tv, tv_alt);
        } else {
            GSR_HIP(gsr_launch_duplicate(bin, chunk_first, (int64_t)K, gx, tk, tv, s),
                    "duplicate launch");
        }
    }
    GSR_TRY(stage_end(3));

    // ---- 5. stable radix sort of the pairs by (strip-local) tile id -------------------------
    if (colpairs) {  // pass 2: the tile rows of the packed words, keys only
        uint32_t *no_vals = nullptr, *no_vals_alt = nullptr;
        if (ybits > 0)
            GSR_HIP(gsr_radix_sort_pairs(&tv, &no_vals, &tv_alt, &no_vals_alt, (int64_t)K,
                                         col_shift, 32, hist, digit_total, s,
                                         ctx->tile_sort_shape, 0, nullptr, d_K),
                    "tile sort launch");
    } else if (packed) {  // the remaining tile bits of the packed words, keys only
        uint32_t *no_vals = nullptr, *no_vals_alt = nullptr;
        if (high_bits > 0)
            GSR_HIP(gsr_radix_sort_pairs(&tv, &no_vals, &tv_alt, &no_vals_alt, (int64_t)K,
                                         pack_shift, 32, hist, digit_total, s,
                                         ctx->tile_sort_shape, 0),
                    "tile sort launch");
    } else {
        GSR_HIP(gsr_radix_sort_pairs(&tk, &tv, &tk_alt, &tv_alt, (int64_t)K, 0, tbits, hist,
                                     digit_total, s, ctx->tile_sort_shape, fused ? 1 : 0),
                "tile sort launch");
    }
    GSR_TRY(stage_end(4));

    // ---- 6. tile ranges ----------------------------------------------------------------------
    if (!aux_ranges) {  // else written on the second stream (joined below)
        if (!(fused && K > 0))  // else zeroed by k_dup_count
            GSR_HIP(hipMemsetAsync(ctx->ranges_local.p, 0, T_strip * 8, s),
                    "hipMemsetAsync(ranges)");
        GSR_HIP(gsr_launch_ranges(tk, (int64_t)K, static_cast<uint32_t *>(ctx->ranges_local.p), s),
                "ranges launch");
    }
    if (!join_guard.done) {  // the blend reads the colours: join the second stream here
        join_guard.done = true;
        GSR_HIP(hipStreamWaitEvent(s, ctx->join, 0), "hipStreamWaitEvent(join)");
    }
    GSR_TRY(stage_end(5));

    // ---- 7. blend ------------------------------------------------------------------------------
    GsrBlendArgs ba{};
    ba.ranges = static_cast<const uint2 *>(ctx->ranges_local.p);
    ba.point_list = tv;
    ba.records = pa.records;
    ba.W = W;
    ba.H = H;
    ba.grid_x = gx;
    ba.row_begin = rb;
    ba.rows_tiles = rows_tiles;
    ba.y0 = y0;
    ba.rows_out = rows_out;
    ba.bg = cap_mode ? frame + kFrameBg : st->bg;
    ba.skip = cap_mode ? d_K + 1 : nullptr;
    ba.out_color = out->color;
    ba.final_T = out->final_T;
    ba.n_contrib = out->n_contrib;
    ba.cull = ctx->cull;
    ba.fast = ctx->fast;
    ba.xcd_group = ctx->blend_xcd_group;
    ba.id_mask = id_mask;
    GSR_HIP(gsr_launch_blend(ba, s), "blend launch");
    GSR_TRY(stage_end(6));

    if (cap_mode) {  // gsr_forward publishes these once the frame's K is known
        ctx->cap_point_list = tv;
        ctx->cap_tiles_local = tk;
        ctx->cap_id_mask = id_mask;
        ctx->cap_packed = packed || colpairs;
        return GSR_OK;
    }
    out->num_rendered = (int64_t)K;
    ctx->last_K = (int64_t)K;
    ctx->last_gx = gx; ctx->last_gy = gy; ctx->last_rb = rb; ctx->last_re = re;
    ctx->last_point_list = tv;
    ctx->last_tiles_local = tk;
    ctx->last_id_mask = id_mask;
    ctx->last_packed = (packed || colpairs) && K > 0;

    ctx->have_forward = true;
    if (tmode) ++ctx->timed_frames;
    return GSR_OK;
}

}  // extern "C"

namespace {

// Camera, background and frame tag of a captured frame into ctx->frame (one small launch
// ahead of the graph: the graph's kernels read them from there, so a moving camera -- new
// tensors every frame -- replays the same graph).
__global__ void k_stage_frame(const float *__restrict__ view, const float *__restrict__ proj,
                              const float *__restrict__ campos, const float *__restrict__ bg,
                              float *__restrict__ frame, uint32_t tag) {
    const int t = threadIdx.x;
    if (t < 16)
        frame[kFrameView + t] = view[t];
    else if (t < 32)
        frame[kFrameProj + t - 16] = proj[t - 16];
    else if (t < 35)
        frame[kFrameCampos + t - 32] = campos ? campos[t - 32] : 0.0f;
    else if (t >= 36 && t < 39)
        frame[kFrameBg + t - 36] = bg[t - 36];
    else if (t == 40)
        reinterpret_cast<uint32_t *>(frame)[kFrameTag] = tag;
}

// Whether forward_impl can record the frame: the column-first binning with second-stream tile
// ranges, whose kernels all learn K on the device.  (Mirrors forward_impl's own choices.)
bool capturable(const gsr_context *ctx, const gsr_gaussians *g, const gsr_raster_settings *st,
                const gsr_outputs *out) {
    if (!ctx->graph || ctx->timing != 0 || st->debug || !ctx->split_color || g->P <= 0 ||
        g->P > (int64_t)UINT32_MAX || !st->viewmatrix || !st->projmatrix || !st->bg ||
        !out->color || !out->radii || st->image_width <= 0 || st->image_height <= 0)
        return false;
    const uint32_t gx = (uint32_t)((st->image_width + GSR_TILE_X - 1) / GSR_TILE_X);
    const uint32_t gy = (uint32_t)((st->image_height + GSR_TILE_Y - 1) / GSR_TILE_Y);
    uint32_t rb = 0, re = gy;
    if (st->tile_row_begin != 0 || st->tile_row_end != 0) {
        if (st->tile_row_begin < 0 || st->tile_row_end > (int)gy ||
            st->tile_row_begin >= st->tile_row_end)
            return false;  // forward_impl reports it
        rb = (uint32_t)st->tile_row_begin;
        re = (uint32_t)st->tile_row_end;
    }
    const uint32_t rows = re - rb;
    const bool aux_ranges = ctx->fused_binning && ctx->aux_ranges &&
                            gsr_tile_diff_cells(gx, rows) <= kTileDiffMaxCells;
    const int col_shift = 32 - (rows > 1 ? bits_for(rows - 1) : 0);
    return aux_ranges && ctx->column_pairs && gx <= 256 && rows <= 256 &&
           (col_shift == 32 || (uint64_t)g->P <= (1ull << col_shift));
}

// Everything a recorded frame bakes in besides the camera and bg (staged per frame).
std::vector<uint64_t> frame_key(const gsr_context *ctx, const gsr_gaussians *g,
                                const gsr_raster_settings *st, const gsr_outputs *out) {
    std::vector<uint64_t> k;
    k.reserve(48);
    auto u = [&](uint64_t v) { k.push_back(v); };
    auto p = [&](const void *v) { k.push_back((uint64_t)reinterpret_cast<uintptr_t>(v)); };
    auto f = [&](float x) {
        uint32_t b;
        std::memcpy(&b, &x, 4);
        k.push_back(b);
    };
    u((uint64_t)g->P), u((uint64_t)g->D), u((uint64_t)g->M), f(g->scale_modifier);
    p(g->means3D), p(g->scales), p(g->rotations), p(g->opacities), p(g->shs);
    p(g->colors_precomp), p(g->cov3D_precomp);
    u((uint64_t)st->image_width), u((uint64_t)st->image_height), f(st->tanfovx), f(st->tanfovy);
    u(st->campos != nullptr), u((uint64_t)st->tile_row_begin), u((uint64_t)st->tile_row_end);
    u((uint64_t)st->prefiltered);
    p(out->color), p(out->radii), p(out->depths), p(out->means2D), p(out->conic_opacity);
    p(out->rgb), p(out->tiles_touched), p(out->final_T), p(out->n_contrib);
    u((uint64_t)ctx->cull), u((uint64_t)ctx->fast), u((uint64_t)ctx->tile_sort_shape);
    u((uint64_t)ctx->packed_pairs), u((uint64_t)(int64_t)ctx->color_blocks);
    u((uint64_t)(int64_t)ctx->color_waves), u((uint64_t)(int64_t)ctx->compact_sort);
    u(ctx->blend_xcd_group), u(ctx->serial_color);
    u(ctx->buf_gen), u((uint64_t)ctx->graph_cap);
    return k;
}

int64_t cap_for(int64_t K) {  // pair capacity of the captured frames: K + 25 %, 64k granules
    const int64_t c = std::max<int64_t>(K + K / 4, 1 << 16);
    return (c + 65535) & ~int64_t(65535);
}

void drop_graphs(gsr_context *ctx, hipStream_t s) {
    if (ctx->graphs.empty()) return;
    (void)hipStreamSynchronize(s);  // no launch of them is still pending
    for (auto &e : ctx->graphs) (void)hipGraphExecDestroy(e.exec);
    ctx->graphs.clear();
}

// One frame as a replayed hipGraph (recorded on first use of its key).
int forward_graph(gsr_context *ctx, const gsr_gaussians *g, const gsr_raster_settings *st,
                  gsr_outputs *out, hipStream_t s) {
    const int64_t P = g->P;
    const uint32_t gx = (uint32_t)((st->image_width + GSR_TILE_X - 1) / GSR_TILE_X);
    const uint32_t gy = (uint32_t)((st->image_height + GSR_TILE_Y - 1) / GSR_TILE_Y);
    const bool strip = st->tile_row_begin != 0 || st->tile_row_end != 0;
    const uint32_t rb = strip ? (uint32_t)st->tile_row_begin : 0u;
    const uint32_t re = strip ? (uint32_t)st->tile_row_end : gy;
    const uint64_t T_strip = (uint64_t)gx * (re - rb);
    // every buffer the recorded frame touches, at its final size, before recording
    const uint64_t gen0 = ctx->buf_gen;
    GSR_TRY(reserve_P(ctx, P, s));
    GSR_TRY(grow(ctx, ctx->ranges_local, (size_t)std::max<uint64_t>(T_strip, 1) * 8, s));
    GSR_TRY(grow(ctx, ctx->tile_diff,
                 (size_t)kTileDiffBlocks * gsr_tile_diff_cells(gx, re - rb) * 4, s));
    GSR_TRY(reserve_K(ctx, ctx->graph_cap, s));
    GSR_TRY(grow(ctx, ctx->frame, kFrameWords * 4, s));
    if (ctx->buf_gen != gen0) drop_graphs(ctx, s);  // they point at freed buffers
    const std::vector<uint64_t> key = frame_key(ctx, g, st, out);
    gsr_context::Graph *hit = nullptr;
    for (auto &e : ctx->graphs)
        if (e.key == key) hit = &e;
    if (!hit) {
        if (!ctx->cap_stream)
            GSR_HIP(hipStreamCreateWithFlags(&ctx->cap_stream, hipStreamNonBlocking),
                    "hipStreamCreate(capture)");
        GSR_HIP(hipStreamBeginCapture(ctx->cap_stream, hipStreamCaptureModeThreadLocal),
                "hipStreamBeginCapture");
        ctx->capturing = true;
        const uint64_t gen1 = ctx->buf_gen;
        int rc = forward_impl(ctx, g, st, out, ctx->cap_stream);
        ctx->capturing = false;
        hipGraph_t graph = nullptr;
        const hipError_t e = hipStreamEndCapture(ctx->cap_stream, &graph);
        hipGraphExec_t exec = nullptr;
        if (rc == GSR_OK && e == hipSuccess && ctx->buf_gen == gen1 && graph)
            rc = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) == hipSuccess
                     ? GSR_OK
                     : GSR_E_HIP;
        else if (rc == GSR_OK)
            rc = GSR_E_HIP;
        if (graph) (void)hipGraphDestroy(graph);
        if (rc != GSR_OK) {  // not recordable here: this context renders on the stream
            (void)hipGetLastError();
            ctx->graph = 0;
            return forward_impl(ctx, g, st, out, s);
        }
        if (ctx->graphs.size() >= kMaxGraphs) {
            auto lru = std::min_element(ctx->graphs.begin(), ctx->graphs.end(),
                                        [](const gsr_context::Graph &a,
                                           const gsr_context::Graph &b) { return a.used < b.used; });
            (void)hipStreamSynchronize(s);
            (void)hipGraphExecDestroy(lru->exec);
            ctx->graphs.erase(lru);
        }
        gsr_context::Graph ge;
        ge.key = key;
        ge.exec = exec;
        ge.point_list = ctx->cap_point_list;
        ge.tiles_local = ctx->cap_tiles_local;
        ge.id_mask = ctx->cap_id_mask;
        ge.packed = ctx->cap_packed;
        ctx->graphs.push_back(std::move(ge));
        hit = &ctx->graphs.back();
    }
    hit->used = ++ctx->graph_clock;
    uint32_t tag = ++ctx->frame_tag;
    if (tag == 0) tag = ++ctx->frame_tag;  // 0 is the pinned word's initial value
    ctx->have_forward = false;
    const auto tl0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_stage_frame, dim3(1), dim3(64), 0, s, st->viewmatrix, st->projmatrix,
                       st->campos, st->bg, static_cast<float *>(ctx->frame.p), tag);
    GSR_HIP(hipGetLastError(), "stage launch");
    const auto tl1 = std::chrono::steady_clock::now();
    GSR_HIP(hipGraphLaunch(hit->exec, s), "hipGraphLaunch");
    // K (pair count) arrives in pinned memory from the graph's k_publish_K, tagged
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
        if ((uint32_t)__atomic_load_n(&ctx->h_total[5], __ATOMIC_ACQUIRE) == tag) break;
        if ((spin & 1023u) == 1023u &&
            std::chrono::steady_clock::now() - t0 > std::chrono::seconds(20))
            return fail(GSR_E_HIP, "gsr_forward: the frame's pair count never arrived");
    }
    const uint64_t K = __atomic_load_n(&ctx->h_total[2], __ATOMIC_ACQUIRE);
    if (ctx->graph_stats) {  // env GSR_GRAPH_STATS: host-time split of the replayed frames
        const auto t1 = std::chrono::steady_clock::now();
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        ctx->gs_acc[0] += us(tl0, tl1), ctx->gs_acc[1] += us(tl1, t0), ctx->gs_acc[2] += us(t0, t1);
        if (++ctx->gs_n % 200 == 0)
            std::fprintf(stderr, "gsr graph: %zu graphs, per frame: stage %.1f us, launch %.1f us, "
                                 "K wait %.1f us\n", ctx->graphs.size(), ctx->gs_acc[0] / 200,
                         ctx->gs_acc[1] / 200, ctx->gs_acc[2] / 200),
                ctx->gs_acc[0] = ctx->gs_acc[1] = ctx->gs_acc[2] = 0;
    }
    if (K > (uint64_t)UINT32_MAX - 4096)
        return fail(GSR_E_INVALID, "gsr_forward: more than 2^32-4097 (Gaussian, tile) pairs");
    if ((int64_t)K > ctx->graph_cap) {
        // the device skipped the binning and the blend: grow, render this frame on the stream
        ctx->graph_cap = cap_for((int64_t)K);
        return forward_impl(ctx, g, st, out, s);
    }
    out->num_rendered = (int64_t)K;
    ctx->last_K = (int64_t)K;
    ctx->last_gx = gx; ctx->last_gy = gy; ctx->last_rb = rb; ctx->last_re = re;
    ctx->last_point_list = hit->point_list;
    ctx->last_tiles_local = hit->tiles_local;
    ctx->last_id_mask = hit->id_mask;
    ctx->last_packed = hit->packed && K > 0;
    ctx->have_forward = true;
    return GSR_OK;
}

}  // namespace

extern "C" {

int gsr_forward(gsr_context *ctx, const gsr_gaussians *g, const gsr_raster_settings *st,
                gsr_outputs *out, void *stream_) {
    if (!ctx || !g || !st || !out) return fail(GSR_E_INVALID, "gsr_forward: NULL argument");
    hipStream_t s = static_cast<hipStream_t>(stream_);
    if (!capturable(ctx, g, st, out)) return forward_impl(ctx, g, st, out, s);
    if (ctx->graph_cap == 0) {  // first frame: K is learnt on the stream path
        GSR_TRY(forward_impl(ctx, g, st, out, s));
        ctx->graph_cap = cap_for(ctx->last_K);
        return GSR_OK;
    }
    return forward_graph(ctx, g, st, out, s);
}

int gsr_get_binning(gsr_context *ctx, uint32_t *point_list, uint32_t *point_tiles,
                    uint32_t *ranges, int64_t *num_rendered, int32_t *num_tiles, void *stream) {
    if (!ctx) return fail(GSR_E_INVALID, "gsr_get_binning: NULL context");
    if (!ctx->have_forward) return fail(GSR_E_STATE, "gsr_get_binning: no forward yet");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t K = ctx->last_K;
    const uint64_t T = (uint64_t)ctx->last_gx * ctx->last_gy;
    const uint64_t off = (uint64_t)ctx->last_rb * ctx->last_gx;
    const uint64_t T_strip = (uint64_t)ctx->last_gx * (ctx->last_re - ctx->last_rb);
    if (num_rendered) *num_rendered = K;
    if (num_tiles) *num_tiles = (int32_t)T;
    if (point_list && K > 0) {
        if (ctx->last_id_mask != 0xFFFFFFFFu)
            GSR_HIP(gsr_launch_unpack_ids(ctx->last_point_list, K, ctx->last_id_mask, point_list,
                                          s),
                    "unpack launch");
        else
            GSR_HIP(hipMemcpyAsync(point_list, ctx->last_point_list, (size_t)K * 4,
                                   hipMemcpyDeviceToDevice, s),
                    "hipMemcpyAsync(point_list)");
    }
    if (point_tiles && K > 0) {
        if (!ctx->last_packed)
            GSR_HIP(gsr_launch_globalize_tiles(ctx->last_tiles_local, K, (uint32_t)off,
                                               point_tiles, s),
                    "globalize launch");
        else  // packed list (no key array): the tile of every pair from the ranges
            GSR_HIP(gsr_launch_fill_tiles(static_cast<const uint2 *>(ctx->ranges_local.p),
                                          (uint32_t)T_strip, (uint32_t)off, point_tiles, s),
                    "fill_tiles launch");
    }

    if (ranges) {
        GSR_HIP(hipMemsetAsync(ranges, 0, T * 8, s), "hipMemsetAsync(ranges)");
        GSR_HIP(hipMemcpyAsync(reinterpret_cast<char *>(ranges) + off * 8, ctx->ranges_local.p,
                               T_strip * 8, hipMemcpyDeviceToDevice, s),
                "hipMemcpyAsync(ranges)");
    }
    GSR_HIP(hipStreamSynchronize(s), "gsr_get_binning");
    return GSR_OK;
}

int gsr_tile_row_pairs(gsr_context *ctx, uint32_t *row_pairs, int32_t n_rows, void *stream) {
    if (!ctx) return fail(GSR_E_INVALID, "gsr_tile_row_pairs: NULL context");
    if (!ctx->have_forward) return fail(GSR_E_STATE, "gsr_tile_row_pairs: no forward yet");
    const uint32_t rows = ctx->last_re - ctx->last_rb;
    if (n_rows != (int32_t)rows || (rows > 0 && !row_pairs))
        return fail(GSR_E_INVALID, "gsr_tile_row_pairs: n_rows must be the strip's " +
                                       std::to_string(rows) + " tile rows");
    GSR_HIP(gsr_launch_row_pairs(static_cast<const uint2 *>(ctx->ranges_local.p), ctx->last_gx,
                                 rows, row_pairs, static_cast<hipStream_t>(stream)),
            "row pairs launch");
    return GSR_OK;
}

int gsr_mark_visible(gsr_context *ctx, const float *means3D, int64_t P, const float *viewmatrix,
                     const float *projmatrix, uint8_t *visible, void *stream) {
    (void)projmatrix;  // upstream in_frustum only tests view-space depth
    if (!ctx || P < 0 || (P > 0 && (!means3D || !viewmatrix || !visible)))
        return fail(GSR_E_INVALID, "gsr_mark_visible: bad arguments");
    GSR_HIP(gsr_launch_mark_visible(means3D, P, viewmatrix, visible,
                                    static_cast<hipStream_t>(stream)),
            "mark_visible launch");
    return GSR_OK;
}

int gsr_depth_argsort(gsr_context *ctx, const float *xyz, int64_t P, const float *view_host16,
                      int32_t *out_index, float *out_depth, void *stream) {
    if (!ctx || P < 0 || !view_host16 || (P > 0 && (!xyz || !out_index)))
        return fail(GSR_E_INVALID, "gsr_depth_argsort: bad arguments");
    if (P > (int64_t)INT32_MAX) return fail(GSR_E_INVALID, "gsr_depth_argsort: P too large");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (P == 0) return GSR_OK;
    GSR_TRY(reserve_P(ctx, P, s));
    uint32_t *k = static_cast<uint32_t *>(ctx->sort_keys.p);
    GSR_HIP(gsr_launch_view_depth_keys(xyz, P, view_host16[8], view_host16[9], view_host16[10],
                                       view_host16[11], k, out_depth, s),
            "view depth launch");
    // every key is kept (no sentinel); the indices land in out_index directly (< 2^31)
    GSR_HIP(gsr_depth_sort(k, P, 0, static_cast<uint2 *>(ctx->ds_a.p),
                           static_cast<uint2 *>(ctx->ds_b.p), reinterpret_cast<uint32_t *>(out_index),
                           static_cast<uint32_t *>(ctx->hist.p),
                           static_cast<uint32_t *>(ctx->digit_total.p),
                           static_cast<uint32_t *>(ctx->ds_ctl.p), 0, 3, s),
            "depth argsort launch");
    return GSR_OK;
}

}  // extern "C"
