/*
 * gsr.h -- C ABI of the MI355X-native forward Gaussian-splat rasterizer (libgsr.so).
 *
 * This is the drop-in boundary under the viewer's CUDA backend.  Every entry point names
 * the reference interface it replaces (paths relative to /root/reference):
 *
 *   gsr_forward        <- diff_gaussian_rasterization `_C.rasterize_gaussians(...)` as called
 *                         by GaussianRasterizer.forward, which renderer_cuda.py:211-224
 *                         (CUDARenderer.draw) invokes every frame.  [third-party, un-vendored]
 *   gsr_mark_visible   <- `_C.mark_visible(positions, viewmatrix, projmatrix)` behind
 *                         GaussianRasterizer.markVisible.  [third-party, un-vendored]
 *   gsr_depth_argsort  <- the per-frame depth sort backend `_sort_gaussian(gaus, view_mat)`
 *                         (renderer_ogl.py:10-19 cpu, :22-38 cupy, :41-53 torch), consumed by
 *                         OpenGLRenderer.sort_and_update (renderer_ogl.py:139-146).
 *   gsr_ply_probe/load <- util_gau.load_ply (util_gau.py:63-125).
 *   gsr_disparity_colors <- the disparity render mode (render_mod == -1) of the GL vertex
 *                         shader, gau_vert.glsl:182-207, driven by main.py:862-868.
 *   gsr_pack_image     <- the frame hand-offs: CHW -> HWC+alpha (renderer_cuda.py:226-228) and
 *                         the capture readbacks glReadPixels RGB8 / R32F->uint16 with their
 *                         row flips (main.py:855-879, 895-917).
 *
 * Conventions (plain pointers and sizes only; no torch or HIP types):
 *   - every array pointer is DEVICE memory unless the comment says host;
 *   - matrices passed as device pointers are 16 floats, column-major (upstream's layout,
 *     i.e. the row-major bytes of `view.T` that renderer_cuda.py:192-194 uploads);
 *   - `stream` is a hipStream_t (NULL = the default stream); all work is enqueued on it.
 *     gsr_forward waits once per call for the number of (Gaussian, tile) pairs, as upstream
 *     does for num_rendered -- not for the stream: the GPU stores it into pinned memory as
 *     soon as the preprocess has counted it, while the depth sort runs.  With frame graphs
 *     (GSR_OPT_FRAME_GRAPHS) that wait comes after the whole frame is queued;
 *   - every function returns GSR_OK (0) or a negative GSR_E* code; gsr_last_error()
 *     returns the calling thread's last message.  The Python layer raises RuntimeError;
 *   - a context serves one call at a time: every entry point taking a gsr_context holds the
 *     context's mutex for the call (two host threads rendering on one context are serialised,
 *     not interleaved).  Its workspace is ordered on the stream of the call that used it last: a
 *     call on another stream first waits for the device (hipDeviceSynchronize), so a context
 *     used from two streams stays correct but serial.  Frames meant to overlap on the GPU use
 *     one context (and one stream) each.
 */
#ifndef GSR_H
#define GSR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 4): option ids renumbered (GSR_OPT_COLUMN_PAIRS retired, tight binning moved to 13,
 * ids 10 and 12 reserved), GSR_OPT_DEPTH_SORT (id 11, was COMPACT_SORT) gains the MSD form,
 * gsr_get_binning exports tight lists.
 * 3 (round 6): gsr_get_option; contexts are serialised by a mutex and ordered across streams. */
#define GSR_ABI_VERSION 3

enum {
    GSR_OK = 0,
    GSR_E_INVALID = -1, /* bad argument / shape */
    GSR_E_HIP = -2,     /* a HIP runtime call or kernel failed */
    GSR_E_NOMEM = -3,   /* device allocation failed */
    GSR_E_STATE = -4    /* call order (e.g. no forward yet) */
};

typedef struct gsr_context gsr_context; /* device workspace + stage events; one per device */

/* Gaussians: the five tensors of GaussianDataCUDA (renderer_cuda.py:55-68, built by
 * gaus_cuda_from_cpu :87-98), contiguous float32.  Exactly one of {shs, colors_precomp} and
 * exactly one of {(scales, rotations), cov3D_precomp} must be non-NULL. */
typedef struct {
    int64_t P;            /* number of Gaussians */
    int32_t D;            /* active SH degree (raster_settings["sh_degree"], :137) */
    int32_t M;            /* SH coefficients stored per Gaussian = shs.size(1) (16 or 1) */
    float scale_modifier; /* raster_settings["scale_modifier"] */
    const float *means3D;        /* [P,3]  */
    const float *scales;         /* [P,3]  (already exp-activated, util_gau.py:118-119) */
    const float *rotations;      /* [P,4]  quaternion (r,x,y,z), normalised by the loader */
    const float *opacities;      /* [P,1]  (sigmoid-activated) */
    const float *shs;            /* [P,M,3] */
    const float *colors_precomp; /* [P,3]  */
    const float *cov3D_precomp;  /* [P,6]  upper triangle xx,xy,xz,yy,yz,zz */
} gsr_gaussians;

/* GaussianRasterizationSettings (renderer_cuda.py:104-117). */
typedef struct {
    int32_t image_width, image_height;
    float tanfovx, tanfovy;
    const float *viewmatrix;    /* device [16], column-major */
    const float *projmatrix;     /* device [16], column-major (full projection * view) */
    const float *campos;         /* device [3] */
    const float *bg;             /* device [3] */
    /* Image-space strip (multi-GPU partition): render only 16-px tile rows
     * [tile_row_begin, tile_row_end).  0/0 = the whole frame.  Output images are then
     * strip-local: [3, rows, W] with rows = min(H, 16*end) - 16*begin. */
    int32_t tile_row_begin, tile_row_end;
    int32_t prefiltered; /* upstream: points are known to be in the frustum */
    int32_t debug;       /* synchronise + check after every stage */
} gsr_raster_settings;

typedef struct {
    float *color;    /* required: [3, rows, W] float32 (CHW, as upstream out_color) */
    /* [P] int32 (0 = culled).  Required for whole frames.  On a strip (tile_row_begin/end)
     * it may be NULL when no per-Gaussian intermediate below is requested either: Gaussians
     * whose conservative footprint bound misses the strip then skip the covariance, radius and
     * record work (a multi-GPU strip rank needs only its image). */
    int32_t *radii;
    /* optional per-Gaussian intermediates (NULL = not written) */
    float *depths;        /* [P]   view-space z */
    float *means2D;       /* [P,2] pixel-space centre */
    float *conic_opacity; /* [P,4] inverse 2D covariance (a,b,c) + opacity */
    float *rgb;           /* [P,3] SH-evaluated colour, clamped >= 0 */
    uint32_t *tiles_touched; /* [P] tiles overlapped inside the rendered strip */
    /* optional per-pixel outputs, strip-local like color */
    float *final_T;     /* [rows, W] */
    uint32_t *n_contrib; /* [rows, W] */
    /* written by gsr_forward */
    int64_t num_rendered; /* K: number of (Gaussian, tile) pairs in the strip */
} gsr_outputs;

int gsr_abi_version(void);
const char *gsr_last_error(void);

int gsr_create(gsr_context **out); /* binds to the calling thread's current HIP device */
void gsr_destroy(gsr_context *ctx);

/* Pre-size the workspace so that a timed loop never allocates (sizes are grown on demand
 * otherwise).  P Gaussians, K pairs. */
int gsr_reserve(gsr_context *ctx, int64_t P, int64_t K);

/* Forward rasterization: preprocess (EWA projection + SH) -> device radix depth sort ->
 * tile binning (scan + duplicate + radix tile sort + ranges) -> per-tile blend. */
int gsr_forward(gsr_context *ctx, const gsr_gaussians *g, const gsr_raster_settings *s,
                gsr_outputs *out, void *stream);

/* Binning state of the last gsr_forward on this context: the pair lists its blend read.  Writes
 * the sizes (list_entries = K, the entries of the lists; num_tiles = T, tiles of the whole
 * frame) and, for each non-NULL caller-owned
 * DEVICE buffer, copies: point_list[K] Gaussian ids sorted by (tile, depth); point_tiles[K]
 * their global tile ids; ranges[2*T] = [start,end) per tile (tiles outside the strip stay 0,0,
 * as upstream's memset leaves unused tiles).  With upstream's lists (GSR_OPT_TIGHT_BINNING 0, a
 * strip, or a forward that asked for n_contrib) K is the forward's num_rendered; after a tight
 * forward the lists are the tight ones and K <= num_rendered (each tile's list is an in-order
 * subsequence of upstream's: tests/test_gpu_tight_pin.py checks that against the oracle).  Call
 * once with NULL buffers to size them.  Synchronises `stream`. */
int gsr_get_binning(gsr_context *ctx, uint32_t *point_list, uint32_t *point_tiles,
                    uint32_t *ranges, int64_t *list_entries, int32_t *num_tiles, void *stream);

/* Per tile row of the last gsr_forward's strip, its (Gaussian, tile) pair count:
 * row_pairs[r] for r < n_rows = tile_row_end - tile_row_begin (DEVICE buffer, written on
 * `stream`, no synchronisation).  The multi-GPU strip split (strips.StripBalancer) weights its
 * next boundaries by these counts.  No reference counterpart: the reference renders each frame
 * on one device (renderer_cuda.py:205-224). */
int gsr_tile_row_pairs(gsr_context *ctx, uint32_t *row_pairs, int32_t n_rows, void *stream);

/* GaussianRasterizer.markVisible: visible[i] = view-space z > 0.2. */
int gsr_mark_visible(gsr_context *ctx, const float *means3D, int64_t P, const float *viewmatrix,
                     const float *projmatrix, uint8_t *visible, void *stream);

/* Depth-sort backend (renderer_ogl.py:10-19): depth = (view @ [xyz,1]).z with `view` the HOST
 * 4x4 row-major (math-layout) matrix the viewer passes; out_index[P] int32 = stable ascending
 * argsort of depth (== np.argsort(depth, kind='stable')).  out_depth[P] optional. */
int gsr_depth_argsort(gsr_context *ctx, const float *xyz, int64_t P, const float *view_host16,
                      int32_t *out_index, float *out_depth, void *stream);

/* ---- PLY loader (replaces util_gau.load_ply, util_gau.py:63-125) ----
 * Reads a 3D Gaussian Splatting PLY (binary little / big endian or ascii) whose vertex
 * element has x y z, f_dc_0..2, 45 f_rest_* (SH degree 3), opacity, scale_0..2, rot_0..3, and
 * returns the reference's activated data as SoA float32 arrays: xyz[P*3], rot[P*4]
 * (normalised quaternion), scale[P*3] (exp), opacity[P] (sigmoid), sh[P*48] (DC, then the 15
 * rest coefficients channel-interleaved), plus the bounding box and mean of the positions.
 * gsr_ply_probe reads the header only (P, sh_coeffs = 16).  gsr_ply_load fills the caller's
 * arrays: host memory when device == 0, device memory (uploaded on `stream`, synchronised
 * before return) otherwise.  info->P must be 0 or the probed count.  Errors: GSR_E_INVALID with
 * gsr_last_error() naming the problem (missing property, wrong f_rest count, short file). */
typedef struct gsr_ply_info {
    int64_t P;          /* vertices */
    int32_t sh_coeffs;  /* 16 (degree 3, the only layout the reference loader accepts) */
    int32_t binary;     /* 1 binary, 0 ascii */
    float bbox_min[3];  /* util_gau.py:80-85: min / max / mean of xyz (gsr_ply_load) */
    float bbox_max[3];
    float center[3];
} gsr_ply_info;

int gsr_ply_probe(const char *path, gsr_ply_info *info);
int gsr_ply_load(const char *path, gsr_ply_info *info, float *xyz, float *rot, float *scale,
                 float *opacity, float *sh, int device, void *stream);

/* ---- Stereo dataset outputs ----
 * gsr_disparity_colors: colors[3*i..3*i+2] = d_i for every Gaussian, with
 *   d = |(ndc_x(p) + 1)/2 - (ndc_x(p + (baseline, 0, 0)) + 1)/2|, ndc_x(q) = (P V [q;1]).x /
 *   (P V [q;1]).w -- gau_vert.glsl:182-207.  view_host16 / proj_host16 are HOST row-major
 *   (math-layout) 4x4 matrices: the GL view and projection (util.py:58-105), NOT the negated /
 *   transposed upstream pair.  Render these colours as colors_precomp with scale_modifier x 1.2
 *   (gau_vert.glsl:152-156) to get the viewer's disparity image.
 * gsr_pack_image: chw = the rasterizer's (3,H,W) float image (format R16 reads channel 0 only);
 *   output row r comes from input row (flip_rows ? H-1-r : r).
 *     GSR_PACK_RGBA_F32: float[H][W][4], alpha 1 (renderer_cuda.py:226-228, no flip);
 *     GSR_PACK_RGB8:     uint8[H][W][3] = round(clamp(v,0,1)*255) (GL unorm conversion);
 *     GSR_PACK_R16:      uint16[H][W] = uint16(v*65535) (numpy astype: truncate, wrap). */
enum {
    GSR_PACK_RGBA_F32 = 0,
    GSR_PACK_RGB8 = 1,
    GSR_PACK_R16 = 2
};
int gsr_disparity_colors(const float *means3D, int64_t P, const float *view_host16,
                         const float *proj_host16, float baseline, float *colors, void *stream);
int gsr_pack_image(const float *chw, int32_t H, int32_t W, int32_t format, int32_t flip_rows,
                   void *out, void *stream);

/* Stage timing (HIP events on the forward's stream, no extra synchronisation).
 * gsr_set_timing(1) starts recording one event set per forward (a ring of the last 256);
 * gsr_stage_times waits for the last timed forward and writes the MEAN per-stage time (ms)
 * over the recorded forwards into ms[i] for i < n; it returns the number of stages.
 * Stage names via gsr_stage_name(i).  Each event costs the stream a few microseconds, so
 * gsr_set_timing(2) records only the two events around the blend (the other stages read 0).
 * gsr_set_timing(0) stops recording. */
int gsr_set_timing(gsr_context *ctx, int enable);
int gsr_stage_times(gsr_context *ctx, float *ms, int n);
const char *gsr_stage_name(int i);

/* Options (per context; every setting renders the same image bits except the blend arithmetic,
 * which changes pixels by float rounding at most -- tests/test_gpu_parity.py checks each):
 *   GSR_OPT_BLEND_CULL (default 1): conservative ellipse-vs-quadrant cull in the blend;
 *     outputs are bit-identical either way.
 *   GSR_OPT_BLEND_FAST (default 1): blend arithmetic with log2(e) folded into the conic, FMA
 *     contraction and the hardware exp2 (tolerance in tests/gpu_helpers.py); 0 keeps upstream's
 *     per-pixel operation order (IEEE, no FMA, ocml expf).
 *   GSR_OPT_DEPTH_SORT (default -1 = auto): the form of the per-frame depth sort.  0 = LSD passes
 *     of 12 key bits, the first dropping the keys of Gaussians without pairs in the strip;
 *     1 = the same after a compaction of the kept keys; 2 = one MSD pass over the top 12 bits
 *     of the kept keys' range (key - smallest kept key), then every bucket sorted by the rest in
 *     LDS; 3 = 2 after the compaction.  auto = the compaction on strips (a proper subset of the
 *     tile rows) of >= 4M Gaussians, the MSD form when the previous frame's kept keys spanned a
 *     range of <= 25 bits (3 or 2), else the LSD passes (1 or 0).  Every form gives the same
 *     permutation.
 *   GSR_OPT_FRAME_GRAPHS (default 0): deferred-K frames.  1: the chains of the frame after the
 *     preprocess (the frame stream's K publish + depth sort and its binning; the second
 *     stream's tile ranges, blend order and colour) are recorded once per context and key
 *     (input pointers, sizes, strip, workspace) as three linear HIP graphs and replayed; 2: the
 *     same chains launched directly.  Either way the binning is sized by a capacity (the list
 *     lengths seen so far + 25 %) instead of a mid-frame wait for K, the host reads K after
 *     queueing the whole frame, and a frame whose list outgrew the capacity is rendered again
 *     the direct way after the capacity grows.  Used for column-first frames without debug,
 *     per-stage timing (gsr_set_timing 1), the compacting depth sort or the rgb output; the
 *     image and every output are the same as with 0 (DESIGN.md decision 12 has the timings).
 *   GSR_OPT_TIGHT_BINNING (default 1): with the column-first form and no n_contrib output, each
 *     Gaussian of a rect up to 8 tile columns x 15 rows is paired only with the tiles its
 *     alpha >= 1/255 ellipse reaches (upstream's blend skips it on the others), so the lists are
 *     subsequences of upstream's and every pixel composites the same splats in the same order.
 *     Full frames only (a strip's replicated preprocess would write a record per Gaussian for
 *     one strip's lists).  num_rendered stays upstream's count; gsr_get_binning exports the
 *     tight lists (0 binds upstream's lists).
 *   GSR_OPT_SECOND_STREAM (default 1): the frame's tile ranges, blend order and colour run on
 *     the context's second stream (created on first use), beside the same frame's depth sort and
 *     binning.  0: they run in order on the frame's own stream and the second stream is
 *     destroyed, so the context holds one hardware queue instead of two -- with the process's
 *     GPU_MAX_HW_QUEUES = 4, four frames in flight on four contexts then each have a queue of
 *     their own (FramePipeline with depth >= 3; DESIGN.md decision 13).  With 0, frame graphs
 *     (GSR_OPT_FRAME_GRAPHS) run the second stream's chain in order on the frame's stream (mode
 *     1 records it on a stream made for the recording; ABI 3).  The image is the same either way.
 * The binning form is chosen per frame: column-first (the first tile-sort pass on (Gaussian,
 * tile column) segments, the second on packed (tile row, Gaussian id) words) up to 256 tile
 * columns and strip rows, else the per-pair form; both produce the same lists.  Ids 10 and 12
 * are retired (ABI 1's column-pairs and tight-binning options) and rejected. */
enum { GSR_OPT_BLEND_CULL = 1, GSR_OPT_BLEND_FAST = 2, GSR_OPT_DEPTH_SORT = 11,
       GSR_OPT_TIGHT_BINNING = 13, GSR_OPT_FRAME_GRAPHS = 14, GSR_OPT_SECOND_STREAM = 15 };
int gsr_set_option(gsr_context *ctx, int option, int64_t value);
/* The current value of an option (so a caller that changes one can restore it). */
int gsr_get_option(gsr_context *ctx, int option, int64_t *value);

/* Frame-graph counters of a context: stats[0] forwards rendered by replaying graphs,
 * stats[1] graph pairs recorded, stats[2] forwards re-rendered after the list outgrew the
 * capacity, stats[3] the current list capacity.  Writes min(n, 4); returns 4. */
int gsr_frame_graph_stats(gsr_context *ctx, int64_t *stats, int n);

#ifdef __cplusplus
}
#endif
#endif /* GSR_H */
