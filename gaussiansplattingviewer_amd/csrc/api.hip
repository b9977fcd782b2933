// api.hip -- the C ABI of libgsr.so (declared in include/gsr.h): workspace ownership,
// argument validation, stage orchestration on the caller's stream, stage timing.
//
// gsr_forward replaces upstream `_C.rasterize_gaussians` / Rasterizer::forward
// (rasterizer_impl.cu), which the viewer reaches through renderer_cuda.py:211-224.  One frame is
// a fixed sequence of stages, each its own function below:
//
//   main stream                                    second stream (fork after the preprocess)
//   1 preprocess        (preprocess.hip)           pair count K + depth-key bits -> pinned host
//   2 depth sort        (depth_sort.hip)           tile ranges from the rects (column pairs)
//   3 column counts + scan  (binning.hip)          SH -> RGB colour
//   4 column scatter    = tile-sort pass 1
//   5 row pass          = tile-sort pass 2 (radix_sort.hip)
//   6 join                                          <- join
//   7 blend             (blend.hip)
//
// Binning has two forms with identical results: the column-first form above (default), and the
// per-pair form (offsets scan -> duplicate fused with the first tile-sort pass -> the remaining
// passes -> tile ranges from the sorted keys) for the frames the column form cannot take: more
// than 256 tile columns or strip rows, a difference array larger than LDS, or more Gaussians than
// the packed pair word holds (the choice is automatic; tests reach the per-pair form with images
// wider than 256 tiles).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
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

#define GSR_TRY(expr)                  \
    do {                               \
        int rc_ = (expr);              \
        if (rc_ != GSR_OK) return rc_; \
    } while (0)

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
};

constexpr int kStages = 7;        // the chain on the caller's stream
constexpr int kAllStages = 8;     // + "color", on the second stream (overlaps stages 1..5)
constexpr int kTimingRing = 256;  // frames whose stage events are kept
// The host learns the pair count K and the depth-key bits D by spinning on pinned words the GPU
// stores (k_publish_K, the depth sort's pass 0); after this long without them it falls back to a
// blocking wait (K) or queues every depth pass (D).
constexpr auto kSpinLimit = std::chrono::milliseconds(50);
// Frames with at least this many pairs wait for D before queueing the LSD depth sort's later
// passes (an empty third pass stays off the GPU: C3 3,480 vs 3,340 frames/s); smaller frames are
// bound by the host's submission rate, which the wait would hold to the GPU (DESIGN.md §3
// decision 2).  Only while the previous frame's D left a pass to skip (<= 24 bits): a frame whose
// keys vary in more bits needs all three, and the wait only holds the host (c3r, D = 31).
constexpr int64_t kWaitDPairs = 4 << 20;
// The depth sort compacts the kept keys first on strips of at least this many Gaussians
// (GSR_OPT_DEPTH_SORT auto): a 1/8 strip of C4 keeps ~1/8 of them (DESIGN.md decision 2).
constexpr int64_t kCompactP = 4 << 20;
// The MSD depth sort for frames whose previous frame's kept depth keys spanned a range of <= this
// many bits (setup_frame).
constexpr uint32_t kMsdMaxD = 25;
// ... and of <= this many on one-stream frames (GSR_OPT_SECOND_STREAM 0, frames in flight): there
// the frame's total work counts more than its critical path, and the MSD form's single pass
// outweighs the block sorts of crowded buckets (c3r, Dr = 26, four frames in flight: 4,200 ->
// 4,420 frames/s, while a serial frame loses 0.315 -> 0.342 ms; profiles/r05z5_ab_msd26.txt)
constexpr uint32_t kMsdMaxDOneStream = kMsdMaxD + 1;
// The MSD local sort keeps its wide form (8192 LDS slots) for this many frames after one whose
// buckets crowded the narrow form's 4096 (C5: serial 0.342 -> 0.315 ms; the narrow form's
// smaller LDS keeps C3 even, profiles/r05w_ab_local_slots.txt).
constexpr uint32_t kCrowdFrames = 8;

const char *kStageNames[kAllStages] = {"preprocess", "depth_sort", "scan",  "duplicate",
                                       "tile_sort",  "ranges",     "blend", "color"};

// Frame graphs: recorded pairs of graphs kept per context (least recently used replaced), and
// executable graphs replaced while possibly in flight, kept until a synchronisation point.
constexpr size_t kGraphCache = 4;
constexpr size_t kGraphRetired = 16;
// The binning capacity of frame graphs: the list length seen so far plus a quarter, at least
// kMinListCap entries.
constexpr int64_t kMinListCap = 1 << 16;

// Everything the kernels of a frame's recorded graphs read besides the context's own
// workspace (named by its generation): a forward whose key equals a recorded one replays it.
struct GraphKey {
    uint64_t ws_gen;
    int64_t cap, P;
    const void *means3D, *shs, *colors_precomp;
    int32_t D, M, W, H;
    uint32_t gx, gy, rb, re;
    int32_t col_shift, color_waves;
    uint8_t msd, main_publish, tight, sh_vec4;
};

struct GraphEntry {
    GraphKey key;
    // the frame stream's two halves (K publish + depth sort; column counts + binning) and the
    // second stream's chain: queued in the direct path's order, sort, second stream, binning
    hipGraphExec_t sort = nullptr, bin = nullptr, aux = nullptr;
    uint32_t *point_list = nullptr;                // the list the recorded row pass leaves
    uint64_t used = 0;                             // LRU stamp
};

}  // namespace

struct gsr_context {
    int device = 0;
    // One caller at a time: every entry point that reads or changes the context's workspace,
    // options, pinned words or recorded graphs holds this (the `_C` extension renders with the
    // GIL released, so two host threads may reach one device's context together).
    std::mutex mu;
    // The stream the last call that used the workspace ran on: a call on another stream first
    // waits for the device (the workspace is stream-ordered on one stream at a time).
    hipStream_t ws_stream = nullptr;
    bool ws_stream_set = false;
    // per-Gaussian workspace
    DevBuf records, strip_rect, sort_keys, partials, total, hist, digit_total, bin, chunk_first,
        rect_sorted, pair_count;
    DevBuf strip_rc, rc_sorted;  // tight binning: {rect, span word}, by id and in depth order
    DevBuf ds_a, ds_b;   // depth sort: (key, id) pairs between passes (ping-pong)
    DevBuf block_kept;   // depth sort compaction (strips): kept keys per 256-Gaussian block
    DevBuf color_ids;    // compacted strips: the kept ids the colour pass walks (4 B x P)
    DevBuf perm;         // the depth sort's result: Gaussian ids in depth order (kept ones)
    DevBuf ds_ctl;       // depth sort control words: kept count, key bits, per-tile key stats
    DevBuf col_hist;     // column-first binning: per-(Gaussian block, column) pair counts
    // per-pair workspace
    DevBuf tile_keys, tile_vals, tile_keys_alt, tile_vals_alt;
    DevBuf ranges_local;
    DevBuf tile_diff;  // difference-array partials of the second-stream tile ranges
    DevBuf blend_order;  // the blend's tile groups, heaviest first (second stream)
    // pinned host words the GPU stores into: [0] -, [1] -, [2] K (k_publish_K), [3] its depth-key
    // bits D, [4] (frame tag << 32) | D from the depth sort's pass 0, [5] the pair count over the
    // spans (k_publish_K), [6] the bits of the kept depth keys' range (k_publish_K), [7] K's tag
    uint64_t *h_total = nullptr;
    unsigned long long *d_hostK = nullptr;  // device view of h_total + 2
    unsigned long long *d_hostD = nullptr;  // device view of h_total + 4
    unsigned long long *d_hostCrowd = nullptr;  // device view of h_total + 1
    uint32_t sort_tag = 0;                  // frames rendered on this context (the pinned tags)
    // the bits of the last frame's kept depth keys' range and the bits in which they differ
    // (wait_K); the first frame, with no history, takes the LSD sort, which any spread of depths
    // suits
    uint32_t last_Dr = UINT32_MAX, last_D = UINT32_MAX;
    // state of the last forward (gsr_get_binning, gsr_tile_row_pairs)
    bool have_forward = false;
    int64_t last_K = 0;        // upstream's num_rendered
    int64_t last_list = 0;     // pairs in the list (tight binning: fewer than last_K)
    bool last_tight = false;
    uint32_t last_gx = 0, last_gy = 0, last_rb = 0, last_re = 0;
    uint32_t *last_point_list = nullptr, *last_tiles_local = nullptr;
    bool last_packed = false;             // column pairs: packed words, no tile-key array
    uint32_t last_id_mask = 0xFFFFFFFFu;  // packed word -> Gaussian id
    // options (include/gsr.h)
    int cull = 1;
    int fast = 1;
    int depth_sort = -1;  // GSR_OPT_DEPTH_SORT
    int tight = 1;
    // stage timing: a ring of event sets, one per timed forward, read back after the timed region
    int timing = 0;        // 0 off, 1 every stage, 2 the blend only, on every 8th forward
    int64_t forwards = 0;  // forwards since gsr_set_timing (mode 2's sampling)
    int64_t timed_frames = 0;
    hipEvent_t ev[kTimingRing][kStages + 1] = {};
    hipEvent_t ev_color[kTimingRing][2] = {};
    // second stream: pair count, tile ranges and colour, between a fork after the preprocess and
    // a join before the blend.  Created on the first forward that uses it; GSR_OPT_SECOND_STREAM
    // 0 runs that work on the frame's stream and destroys it, freeing its hardware queue for
    // another frame in flight.  Normal priority, as the callers' streams: a stream's hardware
    // queue is picked when it is created among the queues of its priority, and a low-priority
    // second stream held one of the process's 4 queues apart from them, so four one-stream frame
    // streams created after it shared three (C3 depth 4: ~3,300-3,550 against ~4,090 frames/s,
    // profiles/r05y_stream_probe.txt, r05z2_ab_aux_priority.txt)
    int second_stream = 1;
    hipStream_t aux = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    hipEvent_t compacted = nullptr;  // the compacted ids are written (main -> second stream)
    // frame graphs (GSR_OPT_FRAME_GRAPHS, DESIGN.md decision 12): the frame stream's chain after
    // the preprocess and the second stream's chain, each recorded once as a linear graph and
    // replayed while the key matches; the binning is sized by a capacity instead of the host
    // waiting for K in mid-frame
    int graphs = 0;
    DevBuf frame_words;                  // [0] tag, [1] list length, [4..6] campos
    uint32_t ws_gen = 0;                 // bumped by every (re)allocation of a workspace buffer
    int64_t list_cap = 0;                // pair-list capacity of the graphs (0: none yet)
    std::vector<GraphEntry> graph_cache;
    std::vector<hipGraphExec_t> graph_retired;
    uint64_t graph_clock = 0;
    int64_t graph_frames = 0, graph_records = 0, graph_overflows = 0;  // (gsr_graph_stats)
};

namespace {

// Orders this call after the context's previous workspace user when the caller switched streams
// (rare: a pipeline gives every stream its own context; a synchronisation only then).
int order_stream(gsr_context *ctx, hipStream_t s) {
    if (ctx->ws_stream_set && s != ctx->ws_stream)
        GSR_HIP(hipDeviceSynchronize(), "hipDeviceSynchronize(stream switch)");
    ctx->ws_stream = s;
    ctx->ws_stream_set = true;
    return GSR_OK;
}

// Grow-only device buffer.  Both streams are drained first so no in-flight kernel still reads
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
    ++ctx->ws_gen;  // recorded frame graphs hold the old pointers
    if (hipMalloc(&b.p, want) != hipSuccess) {
        (void)hipGetLastError();
        b.p = nullptr;
        return fail(GSR_E_NOMEM, "hipMalloc of " + std::to_string(want) + " bytes failed");
    }
    b.cap = want;
    return GSR_OK;
}

int reserve_P(gsr_context *ctx, int64_t P, hipStream_t s) {
    const size_t n = (size_t)std::max<int64_t>(P, 1);
    GSR_TRY(grow(ctx, ctx->records, n * sizeof(gsr::SplatRecord), s));
    GSR_TRY(grow(ctx, ctx->strip_rect, n * 8, s));
    GSR_TRY(grow(ctx, ctx->sort_keys, n * 4, s));
    GSR_TRY(grow(ctx, ctx->ds_a, n * 8, s));
    GSR_TRY(grow(ctx, ctx->ds_b, n * 8, s));
    GSR_TRY(grow(ctx, ctx->block_kept, 4 * ((n + 255) / 256), s));
    GSR_TRY(grow(ctx, ctx->partials, (size_t)std::max<int64_t>(gsr_scan_blocks(P), 1) * 4, s));
    GSR_TRY(grow(ctx, ctx->total, 16, s));
    // per preprocess block: its pair count (8 B) and kept-key OR / AND (8 B)
    GSR_TRY(grow(ctx, ctx->pair_count, (size_t)std::max<int64_t>(gsr_preprocess_blocks(P), 1) * 16, s));
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
    GSR_TRY(grow(ctx, ctx->strip_rc, n * 16, s));
    GSR_TRY(grow(ctx, ctx->rc_sorted, n * 16, s));
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

// Spin on a pinned word the GPU stores (system scope) until pred(value) holds; false after
// kSpinLimit.  A sleeping event wait adds wake-up jitter to every frame (and its record a host
// call); the spin keeps one host core busy for the frame's first ~20-50 us.
template <typename Pred>
bool spin_on(const uint64_t *word, Pred pred, uint64_t &value) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
        value = __atomic_load_n(word, __ATOMIC_ACQUIRE);
        if (pred(value)) return true;
        if ((spin & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > kSpinLimit)
            return false;
    }
}

// Everything one forward derives from its arguments, shared by the stage functions.
struct Frame {
    hipStream_t s;
    int64_t P;
    int W, H;
    uint32_t gx, gy, rb, re, rows_tiles;  // tile grid; strip tile rows [rb, re)
    int y0, rows_out;                     // strip pixel rows
    uint64_t T_strip;
    bool dbg;
    int tmode;  // this forward's timing: 0 none, 1 every stage, 2 the blend
    hipEvent_t *ev, *evc;
    bool compact_sort;  // the depth sort compacts the kept keys first
    bool msd_sort;      // the depth sort's MSD pass + per-bucket local sort (else LSD passes)
    bool main_publish;  // K is published on the main stream (with the MSD sort's D), not the
                        // second
    bool color_ids;     // the colour pass walks the compacted ids
    bool colpairs;      // column-first binning (else the per-pair form)
    bool graph = false;  // this forward replays recorded frame graphs (forward_graph)
    int col_shift;      // column pairs: packed word = strip row << col_shift | Gaussian id
    uint32_t tag;       // this frame's tag for the pinned words
    bool wide_local;    // the MSD local sort's 8192-slot form (crowded buckets lately)
    GsrPreprocessArgs pa;
    bool tight;  // tight binning: pairs only over the span words (needs the column-first form)
    uint64_t K = 0;   // upstream's num_rendered
    uint64_t KL = 0;  // pairs in the list (K, or fewer with tight binning)
    // the pair list the blend reads and gsr_get_binning exports
    uint32_t *point_list = nullptr, *tiles_local = nullptr;
    uint32_t id_mask = 0xFFFFFFFFu;
};

int stage_end(gsr_context *ctx, const Frame &f, int i) {
    if (f.tmode == 1 || (f.tmode == 2 && i >= 5))
        GSR_HIP(hipEventRecord(f.ev[i + 1], f.s), "hipEventRecord");
    if (f.dbg) {
        GSR_HIP(hipStreamSynchronize(f.s), std::string("stage ") + kStageNames[i]);
        GSR_HIP(hipGetLastError(), std::string("stage ") + kStageNames[i]);
    }
    (void)ctx;
    return GSR_OK;
}

// Arguments -> Frame (upstream's argument checks and messages, rasterize_points.cu /
// __init__.py), workspace for P.
int setup_frame(gsr_context *ctx, const gsr_gaussians *g, const gsr_raster_settings *st,
                gsr_outputs *out, hipStream_t s, Frame &f) {
    const int64_t P = g->P;
    const int W = st->image_width, H = st->image_height;
    if (P < 0 || P > (int64_t)UINT32_MAX) return fail(GSR_E_INVALID, "gsr_forward: bad P");
    if (W <= 0 || H <= 0) return fail(GSR_E_INVALID, "gsr_forward: image size must be positive");
    const bool strip = st->tile_row_begin != 0 || st->tile_row_end != 0;
    const bool per_gaussian = out->depths || out->means2D || out->conic_opacity || out->rgb ||
                              out->tiles_touched;
    if (!out->color || (P > 0 && !out->radii && (!strip || per_gaussian)))
        return fail(GSR_E_INVALID, "gsr_forward: color and radii outputs are required (radii "
                                   "may be NULL only on a strip without per-Gaussian outputs)");
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
    if (out->conic_opacity && (reinterpret_cast<uintptr_t>(out->conic_opacity) & 15) != 0)
        return fail(GSR_E_INVALID, "gsr_forward: conic_opacity output must be 16-B aligned");

    f.s = s;
    f.P = P;
    f.W = W;
    f.H = H;
    f.gx = (uint32_t)((W + GSR_TILE_X - 1) / GSR_TILE_X);
    f.gy = (uint32_t)((H + GSR_TILE_Y - 1) / GSR_TILE_Y);
    if (f.gx > 0xFFFFu || f.gy > 0xFFFFu)  // packed 16-bit tile rects (preprocess.hip)
        return fail(GSR_E_INVALID, "gsr_forward: image larger than 65535 tiles per side");
    f.rb = 0;
    f.re = f.gy;
    if (st->tile_row_begin != 0 || st->tile_row_end != 0) {
        if (st->tile_row_begin < 0 || st->tile_row_end > (int)f.gy ||
            st->tile_row_begin >= st->tile_row_end)
            return fail(GSR_E_INVALID, "gsr_forward: bad tile row strip");
        f.rb = (uint32_t)st->tile_row_begin;
        f.re = (uint32_t)st->tile_row_end;
    }
    f.rows_tiles = f.re - f.rb;
    f.y0 = (int)(f.rb * GSR_TILE_Y);
    f.rows_out = std::min(H, (int)(f.re * GSR_TILE_Y)) - f.y0;
    f.T_strip = (uint64_t)f.gx * f.rows_tiles;
    f.dbg = st->debug != 0;
    f.ev = ctx->ev[ctx->timed_frames % kTimingRing];
    f.evc = ctx->ev_color[ctx->timed_frames % kTimingRing];
    f.tmode = ctx->timing == 1 ? 1 : (ctx->timing == 2 && ctx->forwards++ % 8 == 0) ? 2 : 0;

    // column-first binning: the tile ranges come from the rects' difference arrays (in LDS),
    // the column pass ranks <= 256 columns and the packed word holds the strip row and the id
    const int ybits = f.rows_tiles > 1 ? bits_for(f.rows_tiles - 1) : 0;
    f.col_shift = 32 - ybits;
    f.colpairs = f.gx <= 256 && f.rows_tiles <= 256 &&
                 gsr_tile_diff_cells(f.gx, f.rows_tiles) <= kTileDiffMaxCells &&
                 (f.col_shift == 32 || (uint64_t)P <= (1ull << f.col_shift));

    GSR_TRY(reserve_P(ctx, P, s));
    GSR_TRY(grow(ctx, ctx->ranges_local, (size_t)std::max<uint64_t>(f.T_strip, 1) * 8, s));
    if (f.colpairs) {
        GSR_TRY(grow(ctx, ctx->tile_diff,
                     (size_t)kTileDiffBlocks * gsr_tile_diff_cells(f.gx, f.rows_tiles) * 4, s));
        GSR_TRY(grow(ctx, ctx->blend_order,
                     (size_t)gsr_blend_order_groups((uint32_t)f.T_strip) * 4, s));
    }

    GsrPreprocessArgs &pa = f.pa;
    pa = GsrPreprocessArgs{};
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
    pa.viewmatrix = st->viewmatrix;
    pa.projmatrix = st->projmatrix;
    pa.campos = st->campos;
    pa.tanfovx = st->tanfovx;
    pa.tanfovy = st->tanfovy;
    // rasterizer_impl.cu: focal_y = height / (2.0f * tan_fovy); focal_x likewise (float).
    pa.focal_y = (float)H / (2.0f * st->tanfovy);
    pa.focal_x = (float)W / (2.0f * st->tanfovx);
    pa.W = W;
    pa.H = H;
    pa.grid_x = f.gx;
    pa.grid_y = f.gy;
    pa.row_begin = f.rb;
    pa.row_end = f.re;
    pa.prefiltered = st->prefiltered;
    pa.sh_vec4 = (g->shs && g->M == 16 && (reinterpret_cast<uintptr_t>(g->shs) & 15) == 0) ? 1 : 0;
    pa.rot_vec4 = (g->rotations && (reinterpret_cast<uintptr_t>(g->rotations) & 15) == 0) ? 1 : 0;
    pa.radii = out->radii;
    pa.strip_skip = out->radii == nullptr ? 1 : 0;
    pa.records = static_cast<gsr::SplatRecord *>(ctx->records.p);
    pa.sort_keys = static_cast<uint32_t *>(ctx->sort_keys.p);
    f.compact_sort = ctx->depth_sort < 0 ? (f.rows_tiles < f.gy && P >= kCompactP)
                                         : ctx->depth_sort == 1 || ctx->depth_sort == 3;
    pa.block_kept = f.compact_sort ? static_cast<uint32_t *>(ctx->block_kept.p) : nullptr;
    // the MSD sort wants buckets of a few thousand keys: its 4096 buckets split the top 12 bits of
    // the kept keys' range (key - min), which balances them while the depths span a few float
    // exponents (Dr <= 25: C2, C3, C5 -- whose near Gaussians cross depth 2.0, D = 31 but Dr =
    // 24-25; C5 in flight +4 %, profiles/r05q_ab_range_msd.txt); wider ranges crowd some buckets
    // past the LDS sort (c3r, Dr = 26: serial 0.313 -> 0.340 ms), so they keep the LSD passes --
    // except on one-stream frames in flight, where the single pass wins (kMsdMaxDOneStream).
    // The choice follows the previous frame's range (the result is the same either way, only the
    // time differs)
    f.msd_sort = ctx->depth_sort < 0
                     ? ctx->last_Dr <= (ctx->second_stream ? kMsdMaxD : kMsdMaxDOneStream)
                     : ctx->depth_sort >= 2;
    // (compacted strips keep the second stream's publish: on the C4 1/8 strip the main-stream
    // publish let the tile counts and colour start earlier, beside the depth sort, 80 -> 134 us)
    f.main_publish = f.msd_sort && !f.compact_sort;
    pa.strip_rect = static_cast<uint2 *>(ctx->strip_rect.p);
    // tight binning: the column-first form, and no n_contrib (upstream's n_contrib counts list
    // positions of the full 3-sigma pairs); span words only then (NULL: every rect full).  Full
    // frames only: on a strip the replicated preprocess writes a 16-B record for every Gaussian
    // to shorten one strip's lists (C4 3/8 strip: preprocess 97 -> 141 us, row pass 52 -> 42 us;
    // C3 3/8 strip 0.150 -> 0.157 ms per frame; DESIGN.md decision 11)
    f.tight = ctx->tight && f.colpairs && !out->n_contrib && f.rows_tiles == f.gy;
    pa.strip_rc = f.tight ? static_cast<uint4 *>(ctx->strip_rc.p) : nullptr;
    pa.block_pairs = static_cast<uint64_t *>(ctx->pair_count.p);
    pa.host_K = ctx->d_hostK;
    pa.depths = out->depths;
    pa.means2D = out->means2D;
    pa.conic_opacity = out->conic_opacity;
    pa.rgb = out->rgb;
    pa.tiles_touched = out->tiles_touched;
    // compacted strip frames: the colour pass walks the depth sort's compacted kept ids
    // (k_color_ids) instead of every Gaussian's rect -- at a 1/8 strip of 6M Gaussians a lane
    // in ~8 had a row to read
    f.color_ids = f.compact_sort && gsr_color_ids_ok(pa);
    if (f.color_ids) GSR_TRY(grow(ctx, ctx->color_ids, (size_t)P * 4, s));
    f.tag = ++ctx->sort_tag;
    if (f.tag == 0) f.tag = ++ctx->sort_tag;  // 0 is the pinned words' initial value
    pa.k_tag = f.tag;
    // the local sort's wide form while one of the last kCrowdFrames frames' sorts found buckets
    // of 513-1024 keys crowding a group past 4096 LDS slots (the flag of the frame before this
    // one may not have landed yet: the form is only a speed choice)
    {
        const uint32_t crowd = (uint32_t)__atomic_load_n(&ctx->h_total[1], __ATOMIC_ACQUIRE);
        f.wide_local = crowd != 0u && f.tag - crowd <= kCrowdFrames;
    }
    return GSR_OK;
}

// ---- 2. the stable depth sort of the Gaussians (depth_sort.hip), passes [p0, p1) ------------
int launch_depth_sort(gsr_context *ctx, const Frame &f, int p0, int p1) {
    uint32_t *hist = static_cast<uint32_t *>(ctx->hist.p);
    uint32_t *digit_total = static_cast<uint32_t *>(ctx->digit_total.p);
    uint32_t *ctl = static_cast<uint32_t *>(ctx->ds_ctl.p);
    uint32_t *perm = static_cast<uint32_t *>(ctx->perm.p);
    uint2 *ds_a = static_cast<uint2 *>(ctx->ds_a.p), *ds_b = static_cast<uint2 *>(ctx->ds_b.p);
    hipError_t e;
    const int64_t nb = gsr_preprocess_blocks(f.P);  // (their key OR / AND words)
    const uint2 *keybits = reinterpret_cast<const uint2 *>(f.pa.block_pairs + nb);
    if (f.compact_sort) {
        // the compacted keys / ids live in ds_b until pass 1 (or the MSD pass) has read them
        if (f.msd_sort && p0 != 0) return GSR_OK;  // (no later passes)
        uint32_t *keys_c = reinterpret_cast<uint32_t *>(ds_b), *ids_c = keys_c + f.P;
        e = gsr_depth_sort_compacted(f.pa.sort_keys, f.P, f.pa.block_kept, keys_c, ids_c, ds_a,
                                     ds_b, perm, hist, digit_total, ctl, p0, p1, f.s,
                                     ctx->d_hostD, f.tag,
                                     f.color_ids ? static_cast<uint32_t *>(ctx->color_ids.p)
                                                 : nullptr,
                                     f.color_ids ? ctx->compacted : nullptr, f.msd_sort ? 1 : 0,
                                     f.msd_sort && !f.main_publish ? keybits : nullptr, nb);
    } else if (f.msd_sort) {
        // MSD pass + per-bucket local sort, the whole sort at once (D from the preprocess blocks)
        if (p0 != 0) return GSR_OK;  // (no later passes)
        e = gsr_depth_sort_msd(f.pa.sort_keys, f.P, f.main_publish ? nullptr : keybits, nb,
                               ds_a, ds_b, perm, hist, digit_total, ctl, f.s,
                               f.graph ? nullptr : ctx->d_hostD, f.tag,
                               f.graph ? nullptr : ctx->d_hostCrowd, f.graph ? 0 : f.wide_local);
    } else {  // (frame graphs queue every pass; the host reads no D)
        e = gsr_depth_sort(f.pa.sort_keys, f.P, 1, ds_a, ds_b, perm, hist, digit_total, ctl, p0,
                           p1, f.s, f.graph ? nullptr : ctx->d_hostD, f.tag);
    }
    GSR_HIP(e, "depth sort launch");
    return GSR_OK;
}

// colour waves per SIMD (gsr_launch_color): 2 on a full frame, so the colour leaves the CUs
// to the binning chain it overlaps (C3 two frames in flight 3,890-3,918 -> 3,947-3,954
// frames/s, serial 0.317 -> 0.308 ms; C4 serial 2.09 -> 2.06 ms); 3 on a compacted strip
// (C4 1/8 strip 0.481 -> 0.468 ms).  profiles/r04n_ab_color_waves.txt, DESIGN.md decision 7.
// 4 on a strip that is not compacted: its waves scan every Gaussian and only ~1 lane in 8 has
// a colour to compute, so more of them hide the row loads' latency (C3 strips +2-3 %, colour
// 49 -> 44 us, profiles/r06x_ab_strip_colour_cap.txt).
constexpr int kColorWavesFull = 2, kColorWavesCompacted = 3, kColorWavesStrip = 4;
int color_waves_of(const Frame &f) {
    if (f.color_ids) return kColorWavesCompacted;
    return f.rows_tiles < f.gy ? kColorWavesStrip : kColorWavesFull;
}

// ---- the second stream: K, the tile ranges (column pairs), the colour -----------------------
// The second stream's kernels on stream `as` (a frame graph records them on its capture
// stream; d_tag then names the device word holding the frame's tag).
int aux_chain(gsr_context *ctx, const Frame &f, hipStream_t as, const uint32_t *d_tag) {
    // K first: k_publish_K sums the preprocess blocks' counts into pinned memory; the host
    // waits for it only after the depth sort and the column counts are queued (MSD frames
    // publish on the main stream instead, with the sort's D)
    if (!f.main_publish)
        GSR_HIP(gsr_launch_count_pairs(f.pa, as, nullptr, d_tag), "pair count launch");
    if (f.tmode == 1) GSR_HIP(hipEventRecord(f.evc[0], as), "hipEventRecord");
    // the tile ranges before the colour, so the colour overlaps the column count and scatter
    // rather than the depth sort (C3 two frames in flight 3,470 -> 3,600 frames/s)
    // (column pairs: the ranges, then the blend's heaviest-first order of the tile groups)
    if (f.colpairs) {
        GSR_HIP(gsr_launch_tile_ranges_aux(f.pa.strip_rect, f.pa.strip_rc, f.P, f.gx,
                                           f.rows_tiles,
                                           static_cast<uint32_t *>(ctx->tile_diff.p),
                                           static_cast<uint2 *>(ctx->ranges_local.p), as),
                "tile ranges launch");
        GSR_HIP(gsr_launch_blend_order(static_cast<const uint2 *>(ctx->ranges_local.p),
                                       (uint32_t)f.T_strip,
                                       static_cast<uint32_t *>(ctx->blend_order.p), as),
                "blend order launch");
    }
    const int color_waves = color_waves_of(f);
    if (f.color_ids) {
        GSR_HIP(hipStreamWaitEvent(as, ctx->compacted, 0), "hipStreamWaitEvent(compacted)");
        GSR_HIP(gsr_launch_color_ids(f.pa, static_cast<const uint32_t *>(ctx->color_ids.p),
                                     static_cast<const uint32_t *>(ctx->ds_ctl.p), color_waves,
                                     as),
                "color launch");
    } else {
        GSR_HIP(gsr_launch_color(f.pa, color_waves, as), "color launch");
    }
    if (f.tmode == 1) GSR_HIP(hipEventRecord(f.evc[1], as), "hipEventRecord");
    return GSR_OK;
}

int launch_second_stream(gsr_context *ctx, const Frame &f) {
    if (!ctx->second_stream) return aux_chain(ctx, f, f.s, nullptr);  // in order, same stream
    hipStream_t as = ctx->aux;
    GSR_HIP(hipStreamWaitEvent(as, ctx->fork, 0), "hipStreamWaitEvent(fork)");
    GSR_TRY(aux_chain(ctx, f, as, nullptr));
    GSR_HIP(hipEventRecord(ctx->join, as), "hipEventRecord(join)");
    if (f.dbg) GSR_HIP(hipStreamSynchronize(as), "stage color");
    return GSR_OK;
}

// ---- 3. the scan: per-column pair counts of the depth-sorted Gaussians (column pairs), or the
// offsets scan over their strip tile counts (per-pair form) --------------------------------------
int launch_scan(gsr_context *ctx, const Frame &f) {
    const uint32_t *perm = static_cast<const uint32_t *>(ctx->perm.p);
    const uint32_t *d_valid = static_cast<const uint32_t *>(ctx->ds_ctl.p);
    uint2 *rect_sorted = static_cast<uint2 *>(ctx->rect_sorted.p);
    if (f.colpairs) {
        GSR_HIP(gsr_launch_col_pairs_count(perm, f.pa.strip_rect, f.pa.strip_rc, f.P, d_valid,
                                           rect_sorted,
                                           f.tight ? static_cast<uint4 *>(ctx->rc_sorted.p)
                                                   : nullptr,
                                           static_cast<uint32_t *>(ctx->col_hist.p),
                                           static_cast<uint32_t *>(ctx->digit_total.p), f.s),
                "column count launch");
    } else {
        uint32_t *partials = static_cast<uint32_t *>(ctx->partials.p);
        GSR_HIP(gsr_launch_scan_reduce(perm, f.pa.strip_rect, f.P, d_valid, partials,
                                       rect_sorted, f.s),
                "scan launch");
        GSR_HIP(gsr_launch_scan_partials(partials, gsr_scan_blocks(f.P),
                                         static_cast<uint64_t *>(ctx->total.p), f.s),
                "scan launch");
    }
    return GSR_OK;
}

// The frame graphs' list capacity for a list of n entries (capacity cap so far): a quarter more,
// at least kMinListCap, 4096-aligned (the row pass's tiles), and at least 1.5x the old one.
int64_t list_capacity(int64_t n, int64_t cap) {
    int64_t c = std::max({n + n / 4, kMinListCap, cap + cap / 2});
    c = (c + 4095) & ~(int64_t)4095;
    return std::min<int64_t>(c, (int64_t)UINT32_MAX - 4096);
}

// K (the pair count, which sizes the binning) from k_publish_K on the second stream, published
// in pinned memory ~20 us after the preprocess.  Debug mode also checks it against the depth
// sort's own key bits and, in the per-pair form, against the offsets scan's total.
int wait_K(gsr_context *ctx, Frame &f) {
    uint64_t tagv = 0;
    if (!spin_on(&ctx->h_total[7], [&](uint64_t v) { return v == f.tag; }, tagv))
        GSR_HIP(hipStreamSynchronize(f.main_publish || !ctx->second_stream ? f.s : ctx->aux),
                "hipStreamSynchronize(pair count)");
    f.K = __atomic_load_n(&ctx->h_total[2], __ATOMIC_ACQUIRE);
    ctx->last_Dr = (uint32_t)__atomic_load_n(&ctx->h_total[6], __ATOMIC_ACQUIRE);
    ctx->last_D = (uint32_t)__atomic_load_n(&ctx->h_total[3], __ATOMIC_ACQUIRE);
    f.KL = f.tight ? __atomic_load_n(&ctx->h_total[5], __ATOMIC_ACQUIRE) : f.K;
    if (f.dbg) {
        uint32_t ctl2[2];
        uint64_t scan_K[2] = {0, 0};
        GSR_HIP(hipMemcpyAsync(ctl2, ctx->ds_ctl.p, 8, hipMemcpyDeviceToHost, f.s),
                "hipMemcpyAsync(ctl)");
        if (!f.colpairs)
            GSR_HIP(hipMemcpyAsync(scan_K, ctx->total.p, 16, hipMemcpyDeviceToHost, f.s),
                    "hipMemcpyAsync(num_rendered)");
        GSR_HIP(hipStreamSynchronize(f.s), "hipStreamSynchronize(ctl)");
        if (ctl2[1] != (uint32_t)ctx->h_total[3])
            return fail(GSR_E_HIP, "gsr_forward: depth key bits mismatch (pair count " +
                                       std::to_string(ctx->h_total[3]) + ", sort " +
                                       std::to_string(ctl2[1]) + ")");
        if (!f.colpairs && scan_K[0] != f.K)
            return fail(GSR_E_HIP, "gsr_forward: pair count mismatch (preprocess " +
                                       std::to_string(f.K) + ", scan " +
                                       std::to_string(scan_K[0]) + ")");
    }
    if (f.K > (uint64_t)UINT32_MAX - 4096)
        return fail(GSR_E_INVALID, "gsr_forward: more than 2^32-4097 (Gaussian, tile) pairs");
    // column-first frames also size the frame graphs' list capacity (before the binning, so
    // this frame's list is not reallocated under it)
    int64_t want = (int64_t)f.KL;
    if (ctx->graphs && f.colpairs && want > ctx->list_cap) {
        ctx->list_cap = list_capacity(want, ctx->list_cap);
        want = ctx->list_cap;
    }
    return reserve_K(ctx, want, f.s);
}

// ---- 4 + 5. the pairs, stably sorted by strip tile ------------------------------------------
int launch_binning(gsr_context *ctx, Frame &f) {
    const uint32_t *perm = static_cast<const uint32_t *>(ctx->perm.p);
    const uint32_t *d_valid = static_cast<const uint32_t *>(ctx->ds_ctl.p);
    const uint2 *rect_sorted = static_cast<const uint2 *>(ctx->rect_sorted.p);
    uint32_t *hist = static_cast<uint32_t *>(ctx->hist.p);  // (after reserve_K)
    uint32_t *digit_total = static_cast<uint32_t *>(ctx->digit_total.p);
    uint32_t *tk = static_cast<uint32_t *>(ctx->tile_keys.p);
    uint32_t *tv = static_cast<uint32_t *>(ctx->tile_vals.p);
    uint32_t *tk_alt = static_cast<uint32_t *>(ctx->tile_keys_alt.p);
    uint32_t *tv_alt = static_cast<uint32_t *>(ctx->tile_vals_alt.p);
    const int64_t K = (int64_t)f.KL;
    if (f.colpairs) {
        // pass 1 by column on (Gaussian, column) segments, then pass 2 on the packed words'
        // row bits, keys only
        if (K > 0)
            GSR_HIP(gsr_launch_col_pairs_scatter(perm, rect_sorted,
                                                 f.tight ? static_cast<const uint4 *>(ctx->rc_sorted.p)
                                                         : nullptr,
                                                 f.P, d_valid,
                                                 static_cast<const uint32_t *>(ctx->col_hist.p),
                                                 digit_total, f.col_shift, tv_alt, f.s),
                    "column scatter launch");
        std::swap(tv, tv_alt);
        GSR_TRY(stage_end(ctx, f, 3));
        if (K > 0 && f.col_shift < 32)
            GSR_HIP(gsr_radix_sort_keys(&tv, &tv_alt, K, f.col_shift, 32, hist, digit_total, f.s),
                    "tile sort launch");
        GSR_TRY(stage_end(ctx, f, 4));
        f.point_list = tv;
        f.tiles_local = nullptr;
        f.id_mask = f.col_shift < 32 ? (1u << f.col_shift) - 1u : 0xFFFFFFFFu;
        return GSR_OK;
    }
    // per-pair form: offsets, then the duplication fused with the first tile-sort pass (which
    // also zeroes the ranges), then the remaining passes and the ranges over the sorted keys
    const int tbits = f.T_strip > 1 ? bits_for(f.T_strip - 1) : 0;
    const GsrRadixPlan plan = gsr_radix_plan(0, tbits);
    if (K > 0) {
        GSR_HIP(gsr_launch_scan_down(perm, rect_sorted,
                                     static_cast<const uint32_t *>(ctx->partials.p), f.P, d_valid,
                                     static_cast<const uint64_t *>(ctx->total.p),
                                     static_cast<uint4 *>(ctx->bin.p),
                                     static_cast<uint32_t *>(ctx->chunk_first.p), f.s),
                "scan_down launch");
        GSR_HIP(gsr_launch_dup_sort_pass(static_cast<const uint4 *>(ctx->bin.p),
                                         static_cast<const uint32_t *>(ctx->chunk_first.p), K,
                                         f.gx, plan.n ? plan.shift[0] : 0,
                                         plan.n ? plan.nbits[0] : 0, hist, digit_total, tk_alt,
                                         tv_alt, static_cast<uint2 *>(ctx->ranges_local.p),
                                         (uint32_t)f.T_strip, f.s),
                "duplicate launch");
        std::swap(tk, tk_alt);
        std::swap(tv, tv_alt);
    }
    GSR_TRY(stage_end(ctx, f, 3));
    if (K > 1)
        GSR_HIP(gsr_radix_sort_pairs(&tk, &tv, &tk_alt, &tv_alt, K, 0, tbits, hist, digit_total,
                                     f.s, 1),
                "tile sort launch");
    GSR_TRY(stage_end(ctx, f, 4));
    if (K == 0)
        GSR_HIP(hipMemsetAsync(ctx->ranges_local.p, 0, f.T_strip * 8, f.s),
                "hipMemsetAsync(ranges)");
    GSR_HIP(gsr_launch_ranges(tk, K, static_cast<uint32_t *>(ctx->ranges_local.p), f.s),
            "ranges launch");
    f.point_list = tv;
    f.tiles_local = tk;
    f.id_mask = 0xFFFFFFFFu;
    return GSR_OK;
}

// ---- 7. blend ----------------------------------------------------------------------------------
int launch_blend(gsr_context *ctx, const Frame &f, const gsr_raster_settings *st,
                 gsr_outputs *out) {
    GsrBlendArgs ba{};
    ba.ranges = static_cast<const uint2 *>(ctx->ranges_local.p);
    ba.point_list = f.point_list;
    ba.records = f.pa.records;
    ba.W = f.W;
    ba.H = f.H;
    ba.grid_x = f.gx;
    ba.row_begin = f.rb;
    ba.rows_tiles = f.rows_tiles;
    ba.y0 = f.y0;
    ba.rows_out = f.rows_out;
    ba.bg = st->bg;
    ba.out_color = out->color;
    ba.final_T = out->final_T;
    ba.n_contrib = out->n_contrib;
    ba.cull = ctx->cull;
    ba.fast = ctx->fast;
    ba.id_mask = f.id_mask;
    ba.order = f.colpairs ? static_cast<const uint32_t *>(ctx->blend_order.p)
                          : nullptr;  // (per-pair form: row-major)
    if (f.graph) {  // the list length is on the device: a list over the capacity is not blended
        ba.list_n = static_cast<const uint32_t *>(ctx->frame_words.p) + 1;
        ba.list_cap = (uint32_t)ctx->list_cap;
    }
    GSR_HIP(gsr_launch_blend(ba, f.s), "blend launch");
    return GSR_OK;
}

// The second stream must not outlive the caller's view of its inputs: every exit after the
// fork leaves the caller's stream behind the join.
struct JoinGuard {
    hipStream_t s = nullptr;
    hipEvent_t join = nullptr;
    bool armed = false;
    ~JoinGuard() {
        if (armed) (void)hipStreamWaitEvent(s, join, 0);
    }
};

// The state gsr_get_binning / gsr_tile_row_pairs read, after a rendered frame.
void finish_frame(gsr_context *ctx, const Frame &f, gsr_outputs *out) {
    out->num_rendered = (int64_t)f.K;
    ctx->last_K = (int64_t)f.K;
    ctx->last_list = (int64_t)f.KL;
    ctx->last_tight = f.tight;
    ctx->last_gx = f.gx, ctx->last_gy = f.gy, ctx->last_rb = f.rb, ctx->last_re = f.re;
    ctx->last_point_list = f.point_list;
    ctx->last_tiles_local = f.tiles_local;
    ctx->last_id_mask = f.id_mask;
    ctx->last_packed = f.colpairs && f.KL > 0;
    ctx->have_forward = true;
    if (f.tmode) ++ctx->timed_frames;
}

// ---- frame graphs (DESIGN.md decision 12) -----------------------------------------------------
// A small frame is bound by the host: ~17 kernel launches at ~5 us each.  ROCm launches a linear
// graph as one batch of pre-built packets (a 20-kernel chain in ~6 us), so the frame stream's
// chain after the preprocess (K publish, depth sort, column counts, column scatter, row pass)
// and the second stream's chain (tile ranges, blend order, colour) are each recorded once as a
// linear graph and replayed; the preprocess (the frame's camera and outputs) and the blend (its
// image) stay direct launches, so 2 launches + 2 graph launches + the fork / join remain.  A
// graph cannot take per-frame arguments: the preprocess stores the frame's tag and camera
// position into device words the recorded kernels read, and the binning is sized by a capacity
// (the list lengths seen so far + 25 %) instead of the host waiting for K in mid-frame; the
// column scatter stores the true length on the device and the row pass and the blend do
// nothing when it exceeds the capacity.  The host reads K after queueing the whole frame (for
// num_rendered) and re-renders an overflowed frame the direct way with a larger capacity, so
// every returned image is complete.

// Eligible forwards: column-first binning, a known capacity, no debug, no per-stage timing, no
// compaction (its colour pass waits on a mid-chain event of the frame stream), no rgb output
// (the colour pass's).
// (One-stream frames too: the second stream's chain then runs in order on the frame's stream,
// as the direct path's one-stream frames do -- recorded as its own graph in mode 1.)
bool graph_eligible(const gsr_context *ctx, const Frame &f, const gsr_outputs *out) {
    return ctx->graphs && ctx->list_cap > 0 && f.colpairs && !f.dbg && f.tmode != 1 &&
           !f.compact_sort && !f.color_ids && !out->rgb && f.P > 0;
}

GraphKey graph_key(const gsr_context *ctx, const Frame &f) {
    GraphKey k;
    std::memset(&k, 0, sizeof(k));  // (padding compares equal)
    k.ws_gen = ctx->ws_gen;
    k.cap = ctx->list_cap;
    k.P = f.P;
    k.means3D = f.pa.means3D;
    k.shs = f.pa.shs;
    k.colors_precomp = f.pa.colors_precomp;
    k.D = f.pa.D;
    k.M = f.pa.M;
    k.W = f.W;
    k.H = f.H;
    k.gx = f.gx;
    k.gy = f.gy;
    k.rb = f.rb;
    k.re = f.re;
    k.col_shift = f.col_shift;
    k.color_waves = color_waves_of(f);
    k.msd = f.msd_sort;
    k.main_publish = f.main_publish;
    k.tight = f.tight;
    k.sh_vec4 = (uint8_t)f.pa.sh_vec4;
    return k;
}

// The preprocess arguments the recorded kernels see: the camera position from the frame
// words, and none of the per-frame pointers (camera matrices, outputs), which they do not read.
GsrPreprocessArgs graph_args(const gsr_context *ctx, const GsrPreprocessArgs &a) {
    GsrPreprocessArgs g = a;
    uint32_t *fw = static_cast<uint32_t *>(ctx->frame_words.p);
    g.campos = a.campos ? reinterpret_cast<const float *>(fw + 4) : nullptr;
    g.viewmatrix = g.projmatrix = nullptr;
    g.scales = g.rotations = g.opacities = g.cov3D_precomp = nullptr;
    g.radii = nullptr;
    g.depths = g.means2D = g.conic_opacity = g.rgb = nullptr;
    g.tiles_touched = nullptr;
    g.k_tag = 0;
    g.frame_words = nullptr;
    return g;
}

void retire_graph(gsr_context *ctx, GraphEntry &e) {
    for (hipGraphExec_t *ge : {&e.sort, &e.bin, &e.aux}) {
        if (*ge) ctx->graph_retired.push_back(*ge);
        *ge = nullptr;
    }
}

// Destroys the retired executable graphs once enough have gathered (they ran only on this
// context's frame stream and second stream, which are drained first).
int drain_retired(gsr_context *ctx, hipStream_t s, bool force) {
    if (ctx->graph_retired.empty() || (!force && ctx->graph_retired.size() < kGraphRetired))
        return GSR_OK;
    GSR_HIP(hipStreamSynchronize(s), "hipStreamSynchronize(graphs)");
    if (ctx->aux) GSR_HIP(hipStreamSynchronize(ctx->aux), "hipStreamSynchronize(graphs)");
    for (hipGraphExec_t ge : ctx->graph_retired) (void)hipGraphExecDestroy(ge);
    ctx->graph_retired.clear();
    return GSR_OK;
}

// Records one chain into an executable graph, captured on the context's second stream (a
// capture executes nothing; a private capture stream would take one of the process's
// GPU_MAX_HW_QUEUES = 4 hardware queues, which the frame streams and second streams of two frames
// in flight already fill: with it, every stream shares a queue and the direct path lost 20 % in
// flight).
// A context without its second stream (one-stream frames) captures on a stream made for the
// recording and destroyed right after it: it holds no hardware queue beyond the recording, which
// happens once per key.
struct CaptureStream {
    hipStream_t s = nullptr;
    bool own = false;
    ~CaptureStream() {
        if (own && s) (void)hipStreamDestroy(s);
    }
};

template <typename Chain>
int record_chain(gsr_context *ctx, Chain chain, hipGraphExec_t *out) {
    CaptureStream capture;
    capture.s = ctx->aux;
    if (!capture.s) {
        GSR_HIP(hipStreamCreateWithFlags(&capture.s, hipStreamNonBlocking),
                "hipStreamCreateWithFlags(capture)");
        capture.own = true;
    }
    hipStream_t cs = capture.s;
    GSR_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    const int rc = chain(cs);
    hipGraph_t graph = nullptr;
    const hipError_t e = hipStreamEndCapture(cs, &graph);  // (ends the capture on every path)
    if (rc != GSR_OK) {
        if (graph) (void)hipGraphDestroy(graph);
        return rc;
    }
    GSR_HIP(e, "hipStreamEndCapture");
    const hipError_t ei = hipGraphInstantiate(out, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    GSR_HIP(ei, "hipGraphInstantiate");
    return GSR_OK;
}

// The deferred-K frame's chains on stream cs (the frame graphs record them; GSR_OPT_FRAME_GRAPHS
// 2 launches them directly): g is graph_frame's copy of the frame.
Frame graph_frame(const gsr_context *ctx, const Frame &f) {
    Frame g = f;
    g.pa = graph_args(ctx, f.pa);
    g.tmode = 0;
    return g;
}

// K publish (main-stream frames) + the depth sort.
int chain_sort(gsr_context *ctx, Frame &g, hipStream_t cs) {
    g.s = cs;
    if (g.main_publish)
        GSR_HIP(gsr_launch_count_pairs(g.pa, cs, static_cast<uint32_t *>(ctx->ds_ctl.p),
                                       static_cast<const uint32_t *>(ctx->frame_words.p)),
                "pair count launch");
    return launch_depth_sort(ctx, g, 0, gsr_depth_sort_passes(32));
}

// The column counts, the column scatter and the row pass over the capacity, the list length
// read on the device; *point_list: the buffer the sorted list ends in.
int chain_bin(gsr_context *ctx, Frame &g, hipStream_t cs, uint32_t **point_list) {
    g.s = cs;
    GSR_TRY(launch_scan(ctx, g));
    const int64_t cap = ctx->list_cap;
    uint32_t *list_n = static_cast<uint32_t *>(ctx->frame_words.p) + 1;
    uint32_t *tv = static_cast<uint32_t *>(ctx->tile_vals.p);
    uint32_t *tv_alt = static_cast<uint32_t *>(ctx->tile_vals_alt.p);
    GSR_HIP(gsr_launch_col_pairs_scatter(
                static_cast<const uint32_t *>(ctx->perm.p),
                static_cast<const uint2 *>(ctx->rect_sorted.p),
                g.tight ? static_cast<const uint4 *>(ctx->rc_sorted.p) : nullptr, g.P,
                static_cast<const uint32_t *>(ctx->ds_ctl.p),
                static_cast<const uint32_t *>(ctx->col_hist.p),
                static_cast<uint32_t *>(ctx->digit_total.p), g.col_shift, tv_alt, cs,
                (uint32_t)cap, list_n),
            "column scatter launch");
    std::swap(tv, tv_alt);
    if (g.col_shift < 32)
        GSR_HIP(gsr_radix_sort_keys(&tv, &tv_alt, cap, g.col_shift, 32,
                                    static_cast<uint32_t *>(ctx->hist.p),
                                    static_cast<uint32_t *>(ctx->digit_total.p), cs, list_n),
                "tile sort launch");
    *point_list = tv;
    return GSR_OK;
}

// Records the frame's three chains (the key's) into e.
int record_frame_graphs(gsr_context *ctx, const Frame &f, GraphEntry &e) {
    Frame g = graph_frame(ctx, f);
    const uint32_t *fw = static_cast<const uint32_t *>(ctx->frame_words.p);
    GSR_TRY(record_chain(ctx, [&](hipStream_t cs) { return chain_sort(ctx, g, cs); }, &e.sort));
    GSR_TRY(record_chain(ctx, [&](hipStream_t cs) { return chain_bin(ctx, g, cs, &e.point_list); },
                         &e.bin));
    GSR_TRY(record_chain(ctx, [&](hipStream_t cs) { return aux_chain(ctx, g, cs, fw); }, &e.aux));
    ++ctx->graph_records;
    return GSR_OK;
}

// The recorded graphs of this frame's key (recording them on a miss), or nullptr on failure.
int find_graphs(gsr_context *ctx, const Frame &f, GraphEntry **out) {
    const GraphKey key = graph_key(ctx, f);
    GraphEntry *hit = nullptr;
    for (auto it = ctx->graph_cache.begin(); it != ctx->graph_cache.end();) {
        if (it->key.ws_gen != ctx->ws_gen || it->key.cap != ctx->list_cap) {  // stale pointers
            retire_graph(ctx, *it);
            it = ctx->graph_cache.erase(it);
            continue;
        }
        if (std::memcmp(&it->key, &key, sizeof(key)) == 0) hit = &*it;
        ++it;
    }
    if (!hit) {
        if (ctx->graph_cache.size() >= kGraphCache) {  // replace the least recently used
            auto lru = std::min_element(ctx->graph_cache.begin(), ctx->graph_cache.end(),
                                        [](const GraphEntry &a, const GraphEntry &b) {
                                            return a.used < b.used;
                                        });
            retire_graph(ctx, *lru);
            ctx->graph_cache.erase(lru);
        }
        GraphEntry e;
        e.key = key;
        const int rc = record_frame_graphs(ctx, f, e);
        if (rc != GSR_OK) {
            retire_graph(ctx, e);
            return rc;
        }
        ctx->graph_cache.push_back(e);
        hit = &ctx->graph_cache.back();
    }
    hit->used = ++ctx->graph_clock;
    *out = hit;
    return GSR_OK;
}

constexpr int kOverflow = 1;  // forward_graph: the list outgrew the capacity (not rendered)
constexpr int kNoGraphs = 2;  // forward_graph: recording failed before anything was queued

int forward_graph(gsr_context *ctx, Frame &f, const gsr_raster_settings *st, gsr_outputs *out) {
    GraphEntry *e = nullptr;
    const bool replay = ctx->graphs == 1;  // 2: the same chains launched directly
    // a chain that cannot be recorded or instantiated leaves the frame to the direct path
    if (replay && find_graphs(ctx, f, &e) != GSR_OK) return kNoGraphs;
    Frame g = graph_frame(ctx, f);
    const uint32_t *fw = static_cast<const uint32_t *>(ctx->frame_words.p);
    hipStream_t s = f.s;
    if (f.tmode == 1) GSR_HIP(hipEventRecord(f.ev[0], s), "hipEventRecord");
    f.pa.frame_words = static_cast<uint32_t *>(ctx->frame_words.p);
    GSR_HIP(gsr_launch_preprocess(f.pa, s), "preprocess launch");
    GSR_HIP(hipEventRecord(ctx->fork, s), "hipEventRecord(fork)");
    if (replay) GSR_HIP(hipGraphLaunch(e->sort, s), "hipGraphLaunch(depth sort)");
    else GSR_TRY(chain_sort(ctx, g, s));
    const bool two = ctx->second_stream != 0;  // (else mode 2 on one stream: in order on s)
    if (two) GSR_HIP(hipStreamWaitEvent(ctx->aux, ctx->fork, 0), "hipStreamWaitEvent(fork)");
    if (replay) GSR_HIP(hipGraphLaunch(e->aux, two ? ctx->aux : s), "hipGraphLaunch(aux chain)");
    else GSR_TRY(aux_chain(ctx, g, two ? ctx->aux : s, fw));
    if (two) GSR_HIP(hipEventRecord(ctx->join, ctx->aux), "hipEventRecord(join)");
    uint32_t *point_list = nullptr;
    if (replay) {
        GSR_HIP(hipGraphLaunch(e->bin, s), "hipGraphLaunch(binning)");
        point_list = e->point_list;
    } else {
        GSR_TRY(chain_bin(ctx, g, s, &point_list));
    }
    if (two) GSR_HIP(hipStreamWaitEvent(s, ctx->join, 0), "hipStreamWaitEvent(join)");
    GSR_TRY(stage_end(ctx, f, 5));
    f.point_list = point_list;
    f.tiles_local = nullptr;
    f.id_mask = f.col_shift < 32 ? (1u << f.col_shift) - 1u : 0xFFFFFFFFu;
    GSR_TRY(launch_blend(ctx, f, st, out));
    GSR_TRY(stage_end(ctx, f, 6));
    ++ctx->graph_frames;
    // K for num_rendered: published by the first kernel after the preprocess, long before the
    // host has queued the rest of the frame
    uint64_t tagv = 0;
    if (!spin_on(&ctx->h_total[7], [&](uint64_t v) { return v == f.tag; }, tagv))
        GSR_HIP(hipStreamSynchronize(f.main_publish || !two ? s : ctx->aux),
                "hipStreamSynchronize(pair count)");
    f.K = __atomic_load_n(&ctx->h_total[2], __ATOMIC_ACQUIRE);
    ctx->last_Dr = (uint32_t)__atomic_load_n(&ctx->h_total[6], __ATOMIC_ACQUIRE);
    ctx->last_D = (uint32_t)__atomic_load_n(&ctx->h_total[3], __ATOMIC_ACQUIRE);
    f.KL = f.tight ? __atomic_load_n(&ctx->h_total[5], __ATOMIC_ACQUIRE) : f.K;
    if (f.K > (uint64_t)UINT32_MAX - 4096)
        return fail(GSR_E_INVALID, "gsr_forward: more than 2^32-4097 (Gaussian, tile) pairs");
    if ((int64_t)f.KL > ctx->list_cap) return kOverflow;
    finish_frame(ctx, f, out);
    return GSR_OK;
}

int forward(gsr_context *ctx, const gsr_gaussians *g, const gsr_raster_settings *st,
            gsr_outputs *out, hipStream_t s) {
    Frame f;
    ctx->have_forward = false;
    GSR_TRY(setup_frame(ctx, g, st, out, s, f));
    if (ctx->second_stream && !ctx->aux)
        GSR_HIP(hipStreamCreateWithPriority(&ctx->aux, hipStreamNonBlocking, 0),
                "hipStreamCreateWithPriority(second stream)");
    f.graph = f.P > 0 && graph_eligible(ctx, f, out);
    if (f.graph) {
        GSR_TRY(drain_retired(ctx, s, false));
        int rc = forward_graph(ctx, f, st, out);
        if (rc == kNoGraphs) {
            // recording failed before anything of the frame was queued: this context launches
            // the same deferred-K chains directly from now on (GSR_OPT_FRAME_GRAPHS 2)
            ctx->graphs = 2;
            rc = forward_graph(ctx, f, st, out);
        }
        if (rc != kOverflow) return rc;
        // the list outgrew the capacity: nothing was binned or blended.  Grow the capacity and
        // render the frame again the direct way (the stream orders it after the skipped one)
        ++ctx->graph_overflows;
        ctx->list_cap = list_capacity((int64_t)f.KL, ctx->list_cap);
        GSR_TRY(reserve_K(ctx, ctx->list_cap, s));
        GSR_TRY(setup_frame(ctx, g, st, out, s, f));
        f.graph = false;
    }

    if (f.P == 0) {  // upstream returns the zero-initialised image without rendering
        GSR_HIP(hipMemsetAsync(out->color, 0, (size_t)3 * f.rows_out * f.W * sizeof(float), s),
                "hipMemsetAsync(color)");
        GSR_HIP(hipMemsetAsync(ctx->ranges_local.p, 0, f.T_strip * 8, s), "hipMemsetAsync");
        out->num_rendered = 0;
        ctx->last_K = 0;
        ctx->last_list = 0;
        ctx->last_tight = false;
        ctx->last_gx = f.gx, ctx->last_gy = f.gy, ctx->last_rb = f.rb, ctx->last_re = f.re;
        ctx->last_point_list = static_cast<uint32_t *>(ctx->tile_vals.p);
        ctx->last_tiles_local = static_cast<uint32_t *>(ctx->tile_keys.p);
        ctx->last_id_mask = 0xFFFFFFFFu;
        ctx->last_packed = false;
        ctx->have_forward = true;
        return GSR_OK;
    }

    if (f.tmode == 1) GSR_HIP(hipEventRecord(f.ev[0], s), "hipEventRecord");
    // ---- 1. preprocess
    GSR_HIP(gsr_launch_preprocess(f.pa, s), "preprocess launch");
    GSR_HIP(hipEventRecord(ctx->fork, s), "hipEventRecord(fork)");
    GSR_TRY(stage_end(ctx, f, 0));
    // MSD frames: K for the host and D for the sort from one kernel on the main stream (one
    // launch fewer than the second stream's publish plus the sort's own key-bit reduction)
    if (f.main_publish)
        GSR_HIP(gsr_launch_count_pairs(f.pa, s, static_cast<uint32_t *>(ctx->ds_ctl.p)),
                "pair count launch");

    // ---- 2. depth sort: pass 0 first, then the second stream's work (the host hands the
    // critical chain to the GPU first: queueing the ~10 second-stream commands before it left
    // the main queue idle ~40 us on a strip frame), then the later passes
    GSR_TRY(launch_depth_sort(ctx, f, 0, 1));
    JoinGuard guard{s, ctx->join, false};
    GSR_TRY(launch_second_stream(ctx, f));
    guard.armed = ctx->second_stream != 0;
    // D (the bits in which the kept depth keys differ) arrives in pinned memory from pass 0's
    // scan, tagged with this frame, while pass 0's downsweep runs: the host then queues only the
    // passes D needs.  Without it every pass is queued and the unneeded ones exit at once.
    if (!f.msd_sort) {  // the LSD sort: the passes D needs
        int depth_passes = gsr_depth_sort_passes(32);  // all
        uint64_t dv = 0;
        if (ctx->last_K >= kWaitDPairs && ctx->last_D <= 2u * 12u &&
            spin_on(&ctx->h_total[4], [&](uint64_t v) { return (uint32_t)(v >> 32) == f.tag; },
                    dv))
            depth_passes = gsr_depth_sort_passes((uint32_t)dv);
        GSR_TRY(launch_depth_sort(ctx, f, 1, depth_passes));
    }
    GSR_TRY(stage_end(ctx, f, 1));

    // ---- 3. scan
    GSR_TRY(launch_scan(ctx, f));
    GSR_TRY(stage_end(ctx, f, 2));
    GSR_TRY(wait_K(ctx, f));

    // ---- 4, 5. duplicate + tile sort (+ the per-pair form's ranges)
    GSR_TRY(launch_binning(ctx, f));

    // ---- 6. join: the blend reads the colours and the second-stream ranges
    guard.armed = false;
    if (ctx->second_stream)
        GSR_HIP(hipStreamWaitEvent(s, ctx->join, 0), "hipStreamWaitEvent(join)");
    GSR_TRY(stage_end(ctx, f, 5));

    // ---- 7. blend
    GSR_TRY(launch_blend(ctx, f, st, out));
    GSR_TRY(stage_end(ctx, f, 6));
    finish_frame(ctx, f, out);
    return GSR_OK;
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
            hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void **>(&ctx->d_hostCrowd), ctx->h_total + 1,
                                0) != hipSuccess) {
        (void)hipGetLastError();
        delete ctx;
        return fail(GSR_E_HIP, "gsr_create: hipHostMalloc failed");
    }
    std::memset(ctx->h_total, 0, 8 * sizeof(uint64_t));  // tag 0 never matches a frame
    bool ok = hipMalloc(&ctx->frame_words.p, 64) == hipSuccess &&
              hipMemset(ctx->frame_words.p, 0, 64) == hipSuccess &&
              // stream-to-stream hand-offs on one device: a device-scope release suffices
              hipEventCreateWithFlags(&ctx->fork, hipEventDisableTiming | hipEventReleaseToDevice) ==
                  hipSuccess &&
              hipEventCreateWithFlags(&ctx->join, hipEventDisableTiming | hipEventReleaseToDevice) ==
                  hipSuccess &&
              hipEventCreateWithFlags(&ctx->compacted,
                                      hipEventDisableTiming | hipEventReleaseToDevice) == hipSuccess &&
              gsr_color_setup() == hipSuccess;
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
    for (GraphEntry &e : ctx->graph_cache) retire_graph(ctx, e);
    for (hipGraphExec_t ge : ctx->graph_retired) (void)hipGraphExecDestroy(ge);
    DevBuf *bufs[] = {&ctx->records,     &ctx->strip_rect,    &ctx->sort_keys,  &ctx->ds_a,
                      &ctx->ds_b,        &ctx->block_kept,    &ctx->partials,   &ctx->total,
                      &ctx->hist,        &ctx->digit_total,   &ctx->bin,        &ctx->chunk_first,
                      &ctx->rect_sorted, &ctx->pair_count,    &ctx->perm,       &ctx->ds_ctl,
                      &ctx->tile_keys,   &ctx->tile_vals,     &ctx->tile_keys_alt,
                      &ctx->tile_vals_alt, &ctx->ranges_local, &ctx->tile_diff, &ctx->col_hist,
                      &ctx->color_ids, &ctx->blend_order, &ctx->strip_rc, &ctx->rc_sorted,
                      &ctx->frame_words};
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
    std::lock_guard<std::mutex> lock(ctx->mu);
    GSR_TRY(reserve_P(ctx, P, nullptr));
    if (K > ctx->list_cap) ctx->list_cap = std::min<int64_t>((K + 4095) & ~(int64_t)4095,
                                                             (int64_t)UINT32_MAX - 4096);
    GSR_TRY(reserve_K(ctx, std::max<int64_t>(K, ctx->list_cap), nullptr));
    GSR_HIP(hipDeviceSynchronize(), "gsr_reserve");
    return GSR_OK;
}

int gsr_set_option(gsr_context *ctx, int option, int64_t value) {
    if (!ctx) return fail(GSR_E_INVALID, "gsr_set_option: NULL context");
    std::lock_guard<std::mutex> lock(ctx->mu);
    switch (option) {
        case GSR_OPT_BLEND_CULL: ctx->cull = value ? 1 : 0; return GSR_OK;
        case GSR_OPT_BLEND_FAST:
            if (value < 0 || value > 1) return fail(GSR_E_INVALID, "gsr_set_option: fast 0..1");
            ctx->fast = (int)value;
            return GSR_OK;
        case GSR_OPT_TIGHT_BINNING: ctx->tight = value ? 1 : 0; return GSR_OK;
        case GSR_OPT_SECOND_STREAM:
            if (value < 0 || value > 1)
                return fail(GSR_E_INVALID, "gsr_set_option: second stream 0..1");
            ctx->second_stream = (int)value;
            if (!value && ctx->aux) {  // (drained first: its last frame's work may still run)
                GSR_HIP(hipStreamSynchronize(ctx->aux), "hipStreamSynchronize(second stream)");
                GSR_HIP(hipStreamDestroy(ctx->aux), "hipStreamDestroy(second stream)");
                ctx->aux = nullptr;
            }
            return GSR_OK;
        case GSR_OPT_FRAME_GRAPHS:
            if (value < 0 || value > 2) return fail(GSR_E_INVALID, "gsr_set_option: graphs 0..2");
            ctx->graphs = (int)value;
            return GSR_OK;
        case GSR_OPT_DEPTH_SORT:
            if (value < -1 || value > 3)
                return fail(GSR_E_INVALID, "gsr_set_option: depth sort -1..3");
            ctx->depth_sort = (int)value;
            return GSR_OK;
        default:
            return fail(GSR_E_INVALID, "gsr_set_option: unknown option " + std::to_string(option));
    }
}

int gsr_get_option(gsr_context *ctx, int option, int64_t *value) {
    if (!ctx || !value) return fail(GSR_E_INVALID, "gsr_get_option: NULL argument");
    std::lock_guard<std::mutex> lock(ctx->mu);
    switch (option) {
        case GSR_OPT_BLEND_CULL: *value = ctx->cull; return GSR_OK;
        case GSR_OPT_BLEND_FAST: *value = ctx->fast; return GSR_OK;
        case GSR_OPT_TIGHT_BINNING: *value = ctx->tight; return GSR_OK;
        case GSR_OPT_SECOND_STREAM: *value = ctx->second_stream; return GSR_OK;
        case GSR_OPT_FRAME_GRAPHS: *value = ctx->graphs; return GSR_OK;
        case GSR_OPT_DEPTH_SORT: *value = ctx->depth_sort; return GSR_OK;
        default:
            return fail(GSR_E_INVALID, "gsr_get_option: unknown option " + std::to_string(option));
    }
}

int gsr_frame_graph_stats(gsr_context *ctx, int64_t *stats, int n) {
    if (!ctx || (!stats && n > 0)) return fail(GSR_E_INVALID, "gsr_frame_graph_stats: bad arguments");
    std::lock_guard<std::mutex> lock(ctx->mu);
    const int64_t v[4] = {ctx->graph_frames, ctx->graph_records, ctx->graph_overflows,
                          ctx->list_cap};
    for (int i = 0; i < n && i < 4; ++i) stats[i] = v[i];
    return 4;
}

int gsr_set_timing(gsr_context *ctx, int enable) {
    if (!ctx) return fail(GSR_E_INVALID, "gsr_set_timing: NULL context");
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (enable < 0 || enable > 2) return fail(GSR_E_INVALID, "gsr_set_timing: mode 0..2");
    ctx->timing = enable;
    ctx->forwards = 0;
    ctx->timed_frames = 0;
    return GSR_OK;
}

// Mean per-stage time (ms) over the timed forwards since gsr_set_timing (the most recent
// kTimingRing of them).  Waits for the last one.  Return value: number of stages.
int gsr_stage_times(gsr_context *ctx, float *ms, int n) {
    if (!ctx || (!ms && n > 0)) return fail(GSR_E_INVALID, "gsr_stage_times: bad arguments");
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (ctx->timed_frames == 0) return fail(GSR_E_STATE, "gsr_stage_times: no timed forward yet");
    const int64_t frames = std::min<int64_t>(ctx->timed_frames, kTimingRing);
    const int64_t last = (ctx->timed_frames - 1) % kTimingRing;
    GSR_HIP(hipEventSynchronize(ctx->ev[last][kStages]), "hipEventSynchronize");
    const bool all = ctx->timing != 2;  // mode 2 recorded the blend's two events only
    double acc[kAllStages] = {};
    for (int64_t fr = 0; fr < frames; ++fr) {
        const int64_t slot = (ctx->timed_frames - 1 - fr) % kTimingRing;
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

int gsr_forward(gsr_context *ctx, const gsr_gaussians *g, const gsr_raster_settings *st,
                gsr_outputs *out, void *stream) {
    if (!ctx || !g || !st || !out) return fail(GSR_E_INVALID, "gsr_forward: NULL argument");
    std::lock_guard<std::mutex> lock(ctx->mu);
    GSR_TRY(order_stream(ctx, static_cast<hipStream_t>(stream)));
    return forward(ctx, g, st, out, static_cast<hipStream_t>(stream));
}

int gsr_get_binning(gsr_context *ctx, uint32_t *point_list, uint32_t *point_tiles,
                    uint32_t *ranges, int64_t *list_entries, int32_t *num_tiles, void *stream) {
    if (!ctx) return fail(GSR_E_INVALID, "gsr_get_binning: NULL context");
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (!ctx->have_forward) return fail(GSR_E_STATE, "gsr_get_binning: no forward yet");
    hipStream_t s = static_cast<hipStream_t>(stream);
    GSR_TRY(order_stream(ctx, s));
    const int64_t K = ctx->last_list;
    const uint64_t T = (uint64_t)ctx->last_gx * ctx->last_gy;
    const uint64_t off = (uint64_t)ctx->last_rb * ctx->last_gx;
    const uint64_t T_strip = (uint64_t)ctx->last_gx * (ctx->last_re - ctx->last_rb);
    if (list_entries) *list_entries = K;  // (tight lists: fewer than the forward's num_rendered)
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
    std::lock_guard<std::mutex> lock(ctx->mu);
    if (!ctx->have_forward) return fail(GSR_E_STATE, "gsr_tile_row_pairs: no forward yet");
    const uint32_t rows = ctx->last_re - ctx->last_rb;
    if (n_rows != (int32_t)rows || (rows > 0 && !row_pairs))
        return fail(GSR_E_INVALID, "gsr_tile_row_pairs: n_rows must be the strip's " +
                                       std::to_string(rows) + " tile rows");
    GSR_TRY(order_stream(ctx, static_cast<hipStream_t>(stream)));
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
    std::lock_guard<std::mutex> lock(ctx->mu);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (P == 0) return GSR_OK;
    GSR_TRY(order_stream(ctx, s));
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
                           static_cast<uint32_t *>(ctx->ds_ctl.p), 0, gsr_depth_sort_passes(32), s),
            "depth argsort launch");
    return GSR_OK;
}

}  // extern "C"
