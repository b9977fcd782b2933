// gsr_internal.h -- device-side building blocks shared by the gsr kernels (gfx950 only).
//
// Arithmetic contract: every float expression below is evaluated in exactly the order the
// upstream diff-gaussian-rasterization C++ writes it (left-to-right sums, glm column-major
// mat3 products), with FMA contraction OFF and correctly rounded div/sqrt (HIP defaults).
// That is what makes radii / tiles_touched / sort keys / point lists / ranges bit-identical
// to the CPU oracle (oracle/gsr_oracle.c), which restates the same upstream functions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

#define GSR_TILE_X 16
#define GSR_TILE_Y 16
#define GSR_WAVE 64

namespace gsr {

// One visible Gaussian as the blend consumes it: 48 B, three 16-B loads, gathered by tile
// lists.  a = {x, y, conic.a, conic.b}; b = {conic.c, opacity, cull_ex, cull_ey}; c = {cull_Lm,
// r, g, b} (cull_*: conservative alpha >= 1/255 region, see preprocess.hip cull_data).
// k_preprocess writes a, b and c.x; k_color writes the colour c.yzw (on the second stream).
struct alignas(16) SplatRecord {
    float4 a, b, c;
};

__device__ __forceinline__ int f2i_sat(float v) {
    // float -> int with CUDA cvt.rzi.s32.f32 semantics: truncate, saturate, NaN -> 0.
    if (!(v == v)) return 0;
    if (v >= 2147483648.0f) return 2147483647;
    if (v <= -2147483648.0f) return (-2147483647 - 1);
    return (int)v;
}

// --- upstream auxiliary.h --------------------------------------------------------------
__device__ __forceinline__ float3 transform_point_4x3(float3 p, const float *M) {
    float3 r;
    r.x = M[0] * p.x + M[4] * p.y + M[8] * p.z + M[12];
    r.y = M[1] * p.x + M[5] * p.y + M[9] * p.z + M[13];
    r.z = M[2] * p.x + M[6] * p.y + M[10] * p.z + M[14];
    return r;
}

__device__ __forceinline__ float4 transform_point_4x4(float3 p, const float *M) {
    float4 r;
    r.x = M[0] * p.x + M[4] * p.y + M[8] * p.z + M[12];
    r.y = M[1] * p.x + M[5] * p.y + M[9] * p.z + M[13];
    r.z = M[2] * p.x + M[6] * p.y + M[10] * p.z + M[14];
    r.w = M[3] * p.x + M[7] * p.y + M[11] * p.z + M[15];
    return r;
}

// upstream ndc2Pix: `((v + 1.0) * S - 1.0) * 0.5` -- the literals are double.
__device__ __forceinline__ float ndc2pix(float v, int S) {
    return (float)((((double)v + 1.0) * (double)S - 1.0) * 0.5);
}

struct Rect {
    uint32_t x0, y0, x1, y1;
};

__device__ __forceinline__ Rect get_rect(float px, float py, int r, uint32_t gx, uint32_t gy) {
    Rect q;
    q.x0 = min(gx, (uint32_t)max(0, f2i_sat((px - r) / GSR_TILE_X)));
    q.y0 = min(gy, (uint32_t)max(0, f2i_sat((py - r) / GSR_TILE_Y)));
    q.x1 = min(gx, (uint32_t)max(0, f2i_sat((px + r + GSR_TILE_X - 1) / GSR_TILE_X)));
    q.y1 = min(gy, (uint32_t)max(0, f2i_sat((py + r + GSR_TILE_Y - 1) / GSR_TILE_Y)));
    return q;
}

// --- glm-style 3x3, column-major m[col][row] -------------------------------------------
struct Mat3 {
    float m[3][3];
};

__device__ __forceinline__ Mat3 mat3_cols(float a0, float a1, float a2, float a3, float a4,
                                          float a5, float a6, float a7, float a8) {
    Mat3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = a3; r.m[1][1] = a4; r.m[1][2] = a5;
    r.m[2][0] = a6; r.m[2][1] = a7; r.m[2][2] = a8;
    return r;
}

__device__ __forceinline__ Mat3 mat3_mul(const Mat3 &a, const Mat3 &b) {
    Mat3 r;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            float s = a.m[0][i] * b.m[j][0];
            s = s + a.m[1][i] * b.m[j][1];
            s = s + a.m[2][i] * b.m[j][2];
            r.m[j][i] = s;
        }
    return r;
}

__device__ __forceinline__ Mat3 mat3_transpose(const Mat3 &a) {
    Mat3 r;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int i = 0; i < 3; ++i) r.m[i][j] = a.m[j][i];
    return r;
}

// upstream forward.cu computeCov3D (twin: shaders/gau_vert.glsl:73-93)
__device__ __forceinline__ void compute_cov3d(float3 s, float mod, float4 q, float c[6]) {
    Mat3 S = mat3_cols(1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f);
    S.m[0][0] = mod * s.x;
    S.m[1][1] = mod * s.y;
    S.m[2][2] = mod * s.z;
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    Mat3 R = mat3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                       2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                       2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    Mat3 M = mat3_mul(S, R);
    Mat3 Mt = mat3_transpose(M);
    Mat3 Sig = mat3_mul(Mt, M);
    c[0] = Sig.m[0][0];
    c[1] = Sig.m[0][1];
    c[2] = Sig.m[0][2];
    c[3] = Sig.m[1][1];
    c[4] = Sig.m[1][2];
    c[5] = Sig.m[2][2];
}

// upstream forward.cu computeCov2D (twin: shaders/gau_vert.glsl:95-120).  `t` is the
// view-space mean (transformPoint4x3(mean, viewmatrix), already computed by the caller).
__device__ __forceinline__ float3 compute_cov2d(float3 t, float fx, float fy, float tanfovx,
                                                float tanfovy, const float c[6], const float *vm) {
    const float limx = 1.3f * tanfovx;
    const float limy = 1.3f * tanfovy;
    const float txtz = t.x / t.z;
    const float tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    Mat3 J = mat3_cols(fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z,
                       -(fy * t.y) / (t.z * t.z), 0.f, 0.f, 0.f);
    Mat3 W = mat3_cols(vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]);
    Mat3 T = mat3_mul(W, J);
    Mat3 Vrk = mat3_cols(c[0], c[1], c[2], c[1], c[3], c[4], c[2], c[4], c[5]);
    Mat3 Tt = mat3_transpose(T);
    Mat3 Vt = mat3_transpose(Vrk);
    Mat3 A = mat3_mul(Tt, Vt);
    Mat3 cov = mat3_mul(A, T);
    cov.m[0][0] += 0.3f;
    cov.m[1][1] += 0.3f;
    return make_float3(cov.m[0][0], cov.m[0][1], cov.m[1][1]);
}

// Order-preserving float -> uint32 key for a general float sort (negatives, -0 == +0,
// every NaN last): stable radix on these keys == np.argsort(kind='stable').
__device__ __forceinline__ uint32_t float_sort_key(float f) {
    uint32_t u = __float_as_uint(f);
    if (f == 0.0f) u = 0u;
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    if (f != f) u = 0xFFFFFFFFu;
    return u;
}

// --- tight binning: the tile rows each column of a splat's rect really reaches ------------
// Upstream pairs a Gaussian with every tile of its 3-sigma square (getRect); at C3 ~43 % of those
// tiles lie outside the ellipse where the splat can reach alpha >= 1/255, and the blend skips them
// there (upstream `alpha < 1/255: continue`).  A Gaussian whose strip rect has w <= kSpanCols
// columns and h <= kSpanRows rows carries a span word: byte c = lo | cnt << 4, the strip rect's
// rows [lo, lo + cnt) that column c of the rect keeps (preprocess.hip col_spans).  Tight binning
// (GSR_OPT_TIGHT_BINNING) emits only those pairs; every tile list keeps its order, so each
// pixel composites exactly the same splats in the same order.  Larger rects keep every tile.
constexpr uint32_t kSpanCols = 8, kSpanRows = 15;
__device__ __forceinline__ bool span_coded(uint2 rect) {
    return (rect.x >> 16) <= kSpanCols && (rect.y >> 16) <= kSpanRows;
}
// Rows [lo, lo + cnt) of column c (< width) of the rect; cols is ignored unless span_coded.
__device__ __forceinline__ void col_span(uint2 rect, uint2 cols, uint32_t c, uint32_t &lo,
                                         uint32_t &cnt) {
    if (span_coded(rect)) {
        const uint32_t b = ((c < 4 ? cols.x : cols.y) >> (8 * (c & 3))) & 0xFFu;
        lo = b & 15u;
        cnt = b >> 4;
    } else {
        lo = 0u;
        cnt = rect.y >> 16;
    }
}

// --- the depth keys' spread (the preprocess blocks' largest / smallest kept key) -------------
// D: the bits in which the kept keys differ (the highest bit where the largest and the smallest
// differ: every key in between shares the bits above it); Dr: the bits of their range
// max - min, which the MSD depth sort buckets (key - min) by.  No kept key: max < min.
struct KeyBits {
    uint32_t D, Dr, min;
};
__device__ __forceinline__ KeyBits key_bits(uint32_t mx, uint32_t mn) {
    KeyBits k{0u, 0u, 0u};
    if (mx >= mn) {
        k.D = mx != mn ? 32u - (uint32_t)__clz(mx ^ mn) : 0u;
        k.Dr = mx != mn ? 32u - (uint32_t)__clz(mx - mn) : 0u;
        k.min = mn;
    }
    return k;
}
// The MSD depth sort's control words (depth_sort.hip): ctl[1] = D, ctl[2] = the MSD pass's
// shift (Dr - 12, or 0: (key - min) >> shift is the 12-bit bucket), ctl[3] = min.
__device__ __forceinline__ void gsr_msd_ctl(const KeyBits &k, uint32_t *ctl) {
    ctl[1] = k.D;
    ctl[2] = k.Dr > 12u ? k.Dr - 12u : 0u;
    ctl[3] = k.min;
}

// --- wave / block scans (256-thread blocks, wave64) ------------------------------------
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

// Exclusive scan over a 256-thread block.  s_tmp: 4 words of LDS.  Returns the exclusive
// prefix of `v` and the block total in `total`.  Contains two barriers.
__device__ __forceinline__ uint32_t block256_exclusive_scan(uint32_t v, uint32_t *s_tmp,
                                                            uint32_t &total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t inc = wave_inclusive_scan(v);
    if (lane == 63) s_tmp[w] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t t = s_tmp[i];
        pre += (i < w) ? t : 0u;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return pre + inc - v;
}

// --- XCD-aware block order for the scattering passes ---------------------------------------
// The hardware deals workgroup b to XCD b % 8.  Here chunks of kXcdChunk consecutive logical
// blocks go to one XCD, the chunks round-robin over the XCDs, so the partial lines that
// neighbouring blocks write into one digit's run meet in one L2 and leave it merged, while the
// XCDs stay balanced (the column pass's depth-ordered blocks shrink with depth) and the live
// blocks of a grid sized for capacity (a device-side count) still come first on every XCD.
// The grid is a multiple of 8 kXcdChunk blocks (xcd_run_grid); speed only, every logical block
// does the same work.  One contiguous run per XCD lost on both counts
// (profiles/r06k_ab_xcd_runs.txt, r06n_ab_xcd_sort_chunk.txt); chunks of 16 gain C3 +2 %, the
// C4 full frame +7 %.
constexpr uint32_t kXcdChunk = 16;
__device__ __forceinline__ uint32_t xcd_run_block(uint32_t b) {
    const uint32_t x = b & 7u, l = b >> 3;
    return ((l / kXcdChunk) * 8u + x) * kXcdChunk + l % kXcdChunk;
}
inline uint32_t xcd_run_grid(int64_t nb) {
    const int64_t m = 8 * (int64_t)kXcdChunk;
    return (uint32_t)((nb + m - 1) / m * m);
}

}  // namespace gsr

// ---- host-side launchers (defined in the .hip files, called by api.hip) ------------------
struct GsrPreprocessArgs {
    int64_t P;
    int D, M;
    float scale_modifier;
    const float *means3D, *scales, *rotations, *opacities, *shs, *colors_precomp, *cov3D_precomp;
    const float *viewmatrix, *projmatrix, *campos;
    float tanfovx, tanfovy, focal_x, focal_y;
    int W, H;
    uint32_t grid_x, grid_y, row_begin, row_end;
    int prefiltered;
    int sh_vec4, rot_vec4;  // 16-B aligned rows: vector loads allowed
    // workspace outputs
    int32_t *radii;  // nullptr on a strip without radii: strip_skip
    int strip_skip;  // skip Gaussians whose footprint bound misses the strip (preprocess.hip)
    gsr::SplatRecord *records;
    uint32_t *sort_keys;  // depth keys (0xFFFFFFFF: no pair in the strip); values are indices
    uint32_t *block_kept; // optional: per 256-Gaussian block, its count of kept keys
    // per Gaussian: strip-clipped tile rect {x0 | width << 16, strip-local row0 | rows << 16},
    // {0, 0} when it has no pair in the strip (grid dimensions < 2^16, checked by the host)
    uint2 *strip_rect;
    // tight binning (else NULL): per Gaussian {strip rect, span word} (gsr::col_span; the span
    // word only for span-coded rects), {0, 0, 0, 0} without pairs in the strip
    uint4 *strip_rc;
    // per k_preprocess block (ceil(P / 256)): its (Gaussian, strip tile) pair count (low 32
    // bits) and its pair count over the spans (high 32 bits: the same without tight binning),
    // then as many uint2 of the OR / AND of its kept depth keys
    uint64_t *block_pairs;
    // pinned host memory (device-mapped): [K, D, -, K over the spans, -, K tag]
    unsigned long long *host_K;
    uint32_t k_tag;              // nonzero: stored to host_K[5] after K (the host spins on it)
    // frame graphs (api.hip): device words of the context -- [0] the frame's tag, [4..6] the
    // camera position -- which k_preprocess's block 0 stores (k_tag, *campos) for the kernels of
    // a recorded graph, whose arguments cannot change per frame; NULL otherwise
    uint32_t *frame_words;
    // optional debug outputs
    float *depths, *means2D, *conic_opacity, *rgb;
    uint32_t *tiles_touched;
};

// k_preprocess blocks of 256 Gaussians: the count of GsrPreprocessArgs.block_pairs entries and
// of the kept-key OR / AND words after them (the one definition every reader of them uses).
inline int64_t gsr_preprocess_blocks(int64_t P) { return (P + 255) / 256; }
hipError_t gsr_launch_preprocess(const GsrPreprocessArgs &a, hipStream_t s);
// SH -> RGB (or colors_precomp) of every Gaussian with radii > 0 into SplatRecord.c.yzw (+ rgb).
// waves_per_simd (1..7): cap on the colour waves a CU holds at once (0 = no cap).
hipError_t gsr_launch_color(const GsrPreprocessArgs &a, int waves_per_simd, hipStream_t s);
// Once per device (gsr_create): k_color's dynamic LDS limit for those reservations.
hipError_t gsr_color_setup();
// Colour of the Gaussians listed in ids[0 .. *d_n) (the depth sort's compacted kept ids of a
// strip frame), degree-3 16-B-aligned SH and no rgb output only (gsr_color_ids_ok).
bool gsr_color_ids_ok(const GsrPreprocessArgs &a);
hipError_t gsr_launch_color_ids(const GsrPreprocessArgs &a, const uint32_t *ids,
                                const uint32_t *d_n, int waves_per_simd, hipStream_t s);
// K of the frame (sum of the preprocess blocks' pair counts), the pair count over the spans and
// D -> a.host_K (pinned host memory), after the preprocess.  ds_ctl (optional): also the MSD
// depth sort's control words, ctl[1] = D and ctl[2] = its pass's shift (gsr_depth_sort_msd
// with keybits NULL), so the publish runs on the main stream in place of the sort's own
// key-bit reduction.
// d_tag (frame graphs): the tag is read from this device word (k_preprocess's frame_words[0])
// instead of a.k_tag.
hipError_t gsr_launch_count_pairs(const GsrPreprocessArgs &a, hipStream_t s,
                                  uint32_t *ds_ctl = nullptr, const uint32_t *d_tag = nullptr);
hipError_t gsr_launch_mark_visible(const float *means3D, int64_t P, const float *viewmatrix,
                                   uint8_t *visible, hipStream_t s);
hipError_t gsr_launch_view_depth_keys(const float *xyz, int64_t P, float v20, float v21, float v22,
                                      float v23, uint32_t *keys, float *depth_out, hipStream_t s);

// Radix sort of (uint32 key, uint32 value) pairs, stable, LSD over key bits [begin, end) in
// passes of <= 8 bits, starting at pass first_pass of that plan (the per-pair binning's first
// pass runs fused with the duplication).  On return *keys / *vals point at the buffers holding
// the sorted data (either the input pair or the alt pair).  hist needs gsr_radix_hist_words(n)
// words, digit_total 256.
int64_t gsr_radix_hist_words(int64_t n);
hipError_t gsr_radix_sort_pairs(uint32_t **keys, uint32_t **vals, uint32_t **keys_alt,
                                uint32_t **vals_alt, int64_t n, int begin_bit, int end_bit,
                                uint32_t *hist, uint32_t *digit_total, hipStream_t s,
                                int first_pass = 0);
// The same for keys alone (the column-first binning's row pass over packed pair words).
// d_n (frame graphs): the element count is *d_n, read on the device; n is then the capacity
// the grids, the buffers and hist are sized for, and a count above it sorts nothing (the host
// re-renders such a frame, api.hip).
hipError_t gsr_radix_sort_keys(uint32_t **keys, uint32_t **keys_alt, int64_t n, int begin_bit,
                               int end_bit, uint32_t *hist, uint32_t *digit_total, hipStream_t s,
                               const uint32_t *d_n = nullptr);
// k_rs_scan alone: per digit, exclusive scan of hist[d][0..nb) across tiles -> digit_total[d].
hipError_t gsr_launch_digit_scan(uint32_t *hist, int64_t nb, uint32_t *digit_total,
                                 hipStream_t s);

// Radix pass plan: the key bits [begin, end) split into n <= 4 passes of <= 8 bits.
#define GSR_RADIX_MAX_PASSES 4
struct GsrRadixPlan {
    int n;
    int shift[GSR_RADIX_MAX_PASSES];
    int nbits[GSR_RADIX_MAX_PASSES];
    uint32_t mask[GSR_RADIX_MAX_PASSES];
};
GsrRadixPlan gsr_radix_plan(int begin_bit, int end_bit);

// Depth sort (depth_sort.hip): stable sort of n 32-bit keys, values = indices, in passes of
// 12 key bits (pass p: bits [12p, 12p + 12)).  drop: keys 0xFFFFFFFF are dropped; the kept
// count lands in ctl[0] and the bits in which the kept keys differ (D) in ctl[1], both on the
// device after pass 0.  Passes [pass_begin, pass_end) are launched; a pass with 12p >= D exits
// at once and the last needed pass writes the permutation (ids of the kept keys in key order)
// to perm.  A caller that knows D launches gsr_depth_sort_passes(D) passes in total, else all
// three.  pairs_a / pairs_b: n (key, id) pairs each (ping-pong scratch); hist:
// gsr_depth_sort_hist_words(n), digit_total: gsr_depth_sort_digit_words(), ctl:
// gsr_depth_sort_ctl_words(n) words.
int64_t gsr_depth_sort_hist_words(int64_t n);
int64_t gsr_depth_sort_ctl_words(int64_t n);
int gsr_depth_sort_digit_words();
int gsr_depth_sort_passes(uint32_t key_bits);
// host_D (optional, device view of pinned host memory): pass 0 stores (tag << 32) | D there.
hipError_t gsr_depth_sort(const uint32_t *keys, int64_t n, int drop, uint2 *pairs_a,
                          uint2 *pairs_b, uint32_t *perm, uint32_t *hist, uint32_t *digit_total,
                          uint32_t *ctl, int pass_begin, int pass_end, hipStream_t s,
                          unsigned long long *host_D = nullptr, uint32_t tag = 0);
// The frame's sort (no compaction): D from the preprocess blocks' OR / AND of their kept keys
// (keybits: n_keybits uint2, GsrPreprocessArgs.block_pairs after the counts), one global pass
// over the top 12 of the D varying bits (dropping the 0xFFFFFFFF keys), then every bucket sorted
// by the remaining bits in LDS.  Same result, ctl and perm contract as gsr_depth_sort with drop;
// pairs_a holds the bucketed pairs, pairs_b is scratch.  host_D as in gsr_depth_sort.  keybits
// NULL: ctl[1] and ctl[2] are already set (gsr_launch_count_pairs with ds_ctl).  host_crowd
// (optional, device view of pinned host memory): the local sort stores the tag there when its
// buckets of 513-1024 keys crowd the 4096 LDS slots of a group; wide: the 8192-slot local sort.
hipError_t gsr_depth_sort_msd(const uint32_t *keys, int64_t n, const uint2 *keybits,
                              int64_t n_keybits, uint2 *pairs_a, uint2 *pairs_b, uint32_t *perm,
                              uint32_t *hist, uint32_t *digit_total, uint32_t *ctl, hipStream_t s,
                              unsigned long long *host_D = nullptr, uint32_t tag = 0,
                              unsigned long long *host_crowd = nullptr, int wide = 0);
// Compacting front end for sparse key sets (strips): the kept keys of each 256-key block
// (block_kept[b] of them, from the preprocess) are written in order to keys_c, their indices
// to ids_c, and their count to ctl[0]; then the sort runs on those (gsr_depth_sort_compacted,
// same contract as gsr_depth_sort with drop, n the uncompacted upper bound).  block_kept is
// scanned in place.  keys_c / ids_c may be the two halves of pairs_b.  msd: the MSD form on the
// compacted keys instead of the LSD passes (the whole sort in one call, pass_begin 0; keybits as
// in gsr_depth_sort_msd).
hipError_t gsr_depth_sort_compacted(const uint32_t *keys, int64_t n, uint32_t *block_kept,
                                    uint32_t *keys_c, uint32_t *ids_c, uint2 *pairs_a,
                                    uint2 *pairs_b, uint32_t *perm, uint32_t *hist,
                                    uint32_t *digit_total, uint32_t *ctl, int pass_begin,
                                    int pass_end, hipStream_t s,
                                    unsigned long long *host_D = nullptr, uint32_t tag = 0,
                                    uint32_t *ids_copy = nullptr, hipEvent_t compacted = nullptr,
                                    int msd = 0, const uint2 *keybits = nullptr,
                                    int64_t n_keybits = 0);

// Binning: offsets scan over depth-sorted strip tile counts, duplicate into (tile, id)
// pairs, and tile ranges.
int64_t gsr_scan_blocks(int64_t n);
// also writes rect_sorted[e] = strip_rect[perm[e]].  d_n (optional): entries of perm to scan
// (the compacting depth sort's count; n is then only the grid bound).
hipError_t gsr_launch_scan_reduce(const uint32_t *perm, const uint2 *strip_rect, int64_t n,
                                  const uint32_t *d_n, uint32_t *partials, uint2 *rect_sorted,
                                  hipStream_t s);
hipError_t gsr_launch_scan_partials(uint32_t *partials, int64_t nb, uint64_t *total,
                                    hipStream_t s);
// bin[e] (e = depth rank, only for Gaussians with pairs) = {exclusive pair offset, Gaussian
// id, x0 | width << 16, strip-local row0}
hipError_t gsr_launch_scan_down(const uint32_t *perm, const uint2 *rect_sorted,
                                const uint32_t *partials, int64_t n, const uint32_t *d_n,
                                const uint64_t *total, uint4 *bin, uint32_t *chunk_first,
                                hipStream_t s);
int64_t gsr_duplicate_chunks(int64_t K);
// Fused duplicate + first tile-sort radix pass (digit (key >> shift) & (2^nbits - 1)):
// writes the K pairs, stably ordered by that digit, to keys_out / vals_out.  Uses
// chunk_first as written by gsr_launch_scan_down; hist needs gsr_radix_hist_words(K) words.
int64_t gsr_fused_chunks(int64_t K);
hipError_t gsr_launch_dup_sort_pass(const uint4 *bin, const uint32_t *chunk_first, int64_t K,
                                    uint32_t gx, int shift, int nbits, uint32_t *hist,
                                    uint32_t *digit_total, uint32_t *keys_out, uint32_t *vals_out,
                                    uint2 *ranges_zero, uint32_t n_ranges, hipStream_t s);
// Column-first pair generation (binning.hip): pass 1 of the tile sort on (Gaussian, column)
// segments of the depth-sorted Gaussians.  hist: gsr_col_blocks(n_max) * 256 words (per group of
// 4 blocks its column totals, per block its offsets within the group).
int64_t gsr_col_blocks(int64_t n);
// Tight binning: strip_rc (GsrPreprocessArgs) instead of strip_rect, and the depth-ordered copy
// goes to rc_sorted instead of rect_sorted (NULL: full rects).
hipError_t gsr_launch_col_pairs_count(const uint32_t *perm, const uint2 *strip_rect,
                                      const uint4 *strip_rc, int64_t n_max, const uint32_t *d_n,
                                      uint2 *rect_sorted, uint4 *rc_sorted, uint32_t *hist,
                                      uint32_t *digit_total, hipStream_t s);
// list_n (frame graphs, else NULL): the list length (the column totals' sum) is stored there
// for the row pass; a list longer than cap is not written (the host re-renders the frame).
hipError_t gsr_launch_col_pairs_scatter(const uint32_t *perm, const uint2 *rect_sorted,
                                        const uint4 *rc_sorted, int64_t n_max,
                                        const uint32_t *d_n, const uint32_t *hist,
                                        const uint32_t *digit_total, int pack_shift, uint32_t *out,
                                        hipStream_t s, uint32_t cap = 0xFFFFFFFFu,
                                        uint32_t *list_n = nullptr);
hipError_t gsr_launch_digit_scan_n(uint32_t *hist, int64_t nb, uint32_t *digit_total,
                                   const uint32_t *d_n, int64_t tile, hipStream_t s);
// Packed pair lists (column-first binning): ids = packed & mask; tile ids (offset + strip-local
// tile) from the tile ranges.
hipError_t gsr_launch_unpack_ids(const uint32_t *packed, int64_t K, uint32_t mask, uint32_t *out,
                                 hipStream_t s);
hipError_t gsr_launch_fill_tiles(const uint2 *ranges, uint32_t n_tiles, uint32_t offset,
                                 uint32_t *out, hipStream_t s);
hipError_t gsr_launch_ranges(const uint32_t *tile_keys, int64_t K, uint32_t *ranges,
                             hipStream_t s);
// Tile ranges from the Gaussians' strip tile rects alone (no sorted keys): per-tile pair
// counts via per-row difference arrays, then an exclusive scan; runs on the second stream.
// partial: kTileDiffBlocks * cells words (capacity), cells = gsr_tile_diff_cells(...) <= kTileDiffMaxCells
// (the difference arrays live in LDS).
constexpr int kTileDiffBlocks = 256;  // at most; 64 up to 1M Gaussians, more for more
constexpr uint32_t kTileDiffMaxCells = 38912;  // 152 KiB of LDS
// (gx + 1) cells per tile row for rows + 1 rows (the column differences, then the per-tile
// counts), then the rows' pair totals
__host__ __device__ inline uint32_t gsr_tile_diff_cells(uint32_t gx, uint32_t rows) {
    return (gx + 1) * (rows + 1) + rows;
}
hipError_t gsr_launch_tile_ranges_aux(const uint2 *strip_rect, const uint4 *strip_rc, int64_t P,
                                      uint32_t gx,
                                      uint32_t rows, uint32_t *partial, uint2 *ranges,
                                      hipStream_t s);
// Pair count per tile row of a strip's ranges (gsr_tile_row_pairs).
hipError_t gsr_launch_row_pairs(const uint2 *ranges, uint32_t gx, uint32_t rows, uint32_t *out,
                                hipStream_t s);
hipError_t gsr_launch_globalize_tiles(const uint32_t *local, int64_t K, uint32_t offset,
                                      uint32_t *global, hipStream_t s);

struct GsrBlendArgs {
    const uint2 *ranges;  // strip-local tile ranges
    const uint32_t *point_list;
    const gsr::SplatRecord *records;
    int W, H;
    uint32_t grid_x, row_begin, rows_tiles;
    int y0, rows_out;
    const float *bg;
    float *out_color, *final_T;
    uint32_t *n_contrib;
    int cull;            // 0: no quadrant cull (identical output, tested)
    int fast;            // 1: folded-constant FMA arithmetic + raw v_exp_f32; 0: upstream order
    uint32_t id_mask;    // point_list word -> Gaussian id (packed pair lists; else ~0u)
    const uint32_t *order;  // tile groups heaviest first (gsr_launch_blend_order), or nullptr
    // frame graphs: the list length on the device (k_col_scatter) and the capacity the list was
    // binned into; a longer list was not binned, so the blend writes nothing (the host
    // re-renders the frame).  NULL: the host sized the list.
    const uint32_t *list_n;
    uint32_t list_cap;
};
hipError_t gsr_launch_blend(const GsrBlendArgs &a, hipStream_t s);
// The blend's dispatch order: the groups of 4 row-adjacent tiles (16 quadrant waves, one XCD)
// by descending pair count, so the last waves to start are the short ones.
uint32_t gsr_blend_order_groups(uint32_t n_tiles);
hipError_t gsr_launch_blend_order(const uint2 *ranges, uint32_t n_tiles, uint32_t *order,
                                  hipStream_t s);
