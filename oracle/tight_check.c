/*
 * tight_check.c -- TEST INFRASTRUCTURE ONLY (linked into liboracle.so with gsr_oracle.c).
 *
 * Checks of the HIP path's tight binning (include/gsr.h GSR_OPT_TIGHT_BINNING, DESIGN.md
 * decision 11) against upstream semantics as the oracle states them.  Upstream's renderCUDA
 * (forward.cu; oracle_render in gsr_oracle.c) walks a tile's whole duplicateWithKeys list and
 * skips a splat at a pixel when `power > 0` or `alpha = min(0.99, o exp(power)) < 1/255`
 * (twin: shaders/gau_frag.glsl:21-27).  A (splat, tile) pair that is skipped at every pixel of
 * the tile changes nothing, so a list without it renders the same bits provided the kept pairs
 * stay in upstream's order.  Two checks:
 *
 *   oracle_check_tight       -- GPU lists vs the oracle's lists, tile by tile: the tight list
 *                               is an in-order subsequence of the oracle's, and every pair it
 *                               dropped is skipped (power > 0 or alpha < 1/255, in the
 *                               oracle's float arithmetic) at all 256 pixel centres of the tile.
 *   oracle_tight_model_check -- a C restatement of the HIP predicate itself (preprocess.hip
 *                               cull_data + col_spans, with correctly rounded operations where
 *                               the kernel uses v_log / v_rcp / v_sqrt), run on the oracle's
 *                               preprocess outputs: every tile it drops from a rect is checked
 *                               at all 256 pixel centres.  This is the brute force DESIGN.md
 *                               decision 11 quotes, on the CPU; the GPU lists themselves are
 *                               pinned by oracle_check_tight.
 *
 * Pixel centres: upstream's pixel coordinate is (float)(tile * 16 + thread) with no +0.5, and
 * all 256 are checked, including those past the image edge (stricter than needed).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <string.h>

#define TC_BLOCK 16

/* The oracle's per-pixel skip test (oracle_render, upstream renderCUDA): does splat `id`
 * reach alpha >= 1/255 at any of the 256 pixel centres of tile (tx, ty)? */
static int reaches_tile(const float *means2D, const float *conic_opacity, uint32_t id,
                        uint32_t tx, uint32_t ty, float *max_alpha) {
    const float *co = conic_opacity + 4 * (size_t)id;
    const float mx = means2D[2 * (size_t)id], my = means2D[2 * (size_t)id + 1];
    float best = 0.0f;
    int hit = 0;
    for (uint32_t ly = 0; ly < TC_BLOCK; ++ly)
        for (uint32_t lx = 0; lx < TC_BLOCK; ++lx) {
            const float dx = mx - (float)(tx * TC_BLOCK + lx);
            const float dy = my - (float)(ty * TC_BLOCK + ly);
            const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
            if (power > 0.0f) continue;
            const float alpha = fminf(0.99f, co[3] * expf(power));
            if (alpha > best) best = alpha;
            if (alpha >= 1.0f / 255.0f) hit = 1;
        }
    if (max_alpha) *max_alpha = best;
    return hit;
}

/* stats (int64[8]):
 *   [0] tiles whose tight list is not an in-order subsequence of the oracle's list
 *   [1] pairs kept (tight list length), [2] pairs dropped
 *   [3] dropped pairs that reach alpha >= 1/255 somewhere in their tile (must be 0)
 *   [4] first offending tile (-1 if none), [5] its offending Gaussian id (or -1)
 *   [6] largest alpha (x 1e9, rounded down) of any dropped pair at any pixel centre
 * Ranges are [T][2] uint32 (start, end) into the respective lists; both lists hold Gaussian
 * ids.  Returns stats[0] + stats[3] (0 = tight binning is upstream's lists minus pairs that
 * are skipped at every pixel). */
int64_t oracle_check_tight(uint32_t gx, uint32_t gy, const uint32_t *ranges_full,
                           const uint32_t *list_full, const uint32_t *ranges_tight,
                           const uint32_t *list_tight, const float *means2D,
                           const float *conic_opacity, int64_t *stats) {
    int64_t not_sub = 0, kept = 0, dropped = 0, bad = 0;
    int64_t first_tile = -1, first_id = -1;
    float worst = 0.0f;
    const int64_t T = (int64_t)gx * gy;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : not_sub, kept, dropped, bad) \
    reduction(max : worst)
    for (int64_t t = 0; t < T; ++t) {
        const uint32_t tx = (uint32_t)(t % gx), ty = (uint32_t)(t / gx);
        uint32_t i = ranges_full[2 * t], j = ranges_tight[2 * t];
        const uint32_t ie = ranges_full[2 * t + 1], je = ranges_tight[2 * t + 1];
        int64_t my_bad_id = -1;
        int sub_ok = 1;
        for (; j < je; ++j) {
            const uint32_t want = list_tight[j];
            while (i < ie && list_full[i] != want) {
                float a = 0.0f;
                dropped++;
                if (reaches_tile(means2D, conic_opacity, list_full[i], tx, ty, &a)) {
                    bad++;
                    if (my_bad_id < 0) my_bad_id = list_full[i];
                }
                if (a > worst) worst = a;
                ++i;
            }
            if (i == ie) {
                sub_ok = 0;
                break;
            }
            kept++;
            ++i;  /* matched */
        }
        if (sub_ok) {
            for (; i < ie; ++i) {
                float a = 0.0f;
                dropped++;
                if (reaches_tile(means2D, conic_opacity, list_full[i], tx, ty, &a)) {
                    bad++;
                    if (my_bad_id < 0) my_bad_id = list_full[i];
                }
                if (a > worst) worst = a;
            }
        } else {
            not_sub++;
        }
        if (!sub_ok || my_bad_id >= 0) {
#pragma omp critical(tight_first)
            if (first_tile < 0 || t < first_tile) {
                first_tile = t;
                first_id = sub_ok ? my_bad_id : -1;
            }
        }
    }
    stats[0] = not_sub;
    stats[1] = kept;
    stats[2] = dropped;
    stats[3] = bad;
    stats[4] = first_tile;
    stats[5] = first_id;
    stats[6] = (int64_t)floor((double)worst * 1e9);
    stats[7] = 0;
    return not_sub + bad;
}

/* ---- the HIP predicate restated (preprocess.hip cull_data / col_spans, gsr_internal.h) ---- */
enum { kSpanCols = 8, kSpanRows = 15 };

/* cull_data: returns Lm (the widened log-threshold); +inf when no finite region exists.
 * shrink > 0 is the mutation check: every rounding margin dropped and L scaled by (1 - shrink),
 * a predicate slightly too aggressive, which the brute force must catch (else it has no teeth). */
static float model_cull_Lm(float A, float B, float C, float o, float shrink) {
    const int bare = shrink > 0.0f;
    const double det_d = (double)A * (double)C - (double)B * (double)B;
    if (!(det_d > 0.0) || !(A > 0.0f) || !(C > 0.0f) || !(o == o)) return INFINITY;
    const float det = (float)det_d;
    float L = logf(255.0f * o);
    if (!(L > 0.0f)) L = 0.0f;
    const float sxx = C / det, syy = A / det;
    float ex = sqrtf(2.0f * L * sxx), ey = sqrtf(2.0f * L * syy);
    const float mag = (A + C + 2.0f * fabsf(B)) * (ex * ex + ey * ey);
    const float Lm = bare ? L * (1.0f - shrink) : (L + 8.0f * 5.96e-8f * mag + 1e-3f) * 1.01f;
    if (bare) return Lm;
    ex = sqrtf(2.0f * Lm * sxx) + 0.02f;
    ey = sqrtf(2.0f * Lm * syy) + 0.02f;
    if (!(ex < 1e30f) || !(ey < 1e30f) || !(Lm < 1e30f)) return INFINITY;
    uint32_t u;
    memcpy(&u, &Lm, 4);
    u += 1u;
    float r;
    memcpy(&r, &u, 4);
    return r;
}

/* col_spans: per column c < w of the rect, the kept rows [lo[c], lo[c] + cnt[c]) relative to
 * the rect's first row sy0.  Returns 0 when the rect keeps every tile (the kernel's early
 * outs), 1 when lo / cnt hold the spans. */
static int model_col_spans(float px, float py, float A, float B, float C, float Lm, uint32_t x0,
                           uint32_t w, uint32_t sy0, uint32_t h, uint32_t lo_out[kSpanCols],
                           uint32_t cnt_out[kSpanCols], int bare) {
    const float bb = B * B, det = fmaf(A, C, -bb) - fmaf(B, B, -bb);
    if (!(det > 0.0f) || !(A > 0.0f) || !(C > 0.0f) || !(Lm < 1e30f) || !(fabsf(px) < 1e30f) ||
        !(fabsf(py) < 1e30f))
        return 0;
    const float idet = 1.0f / det, T2 = bare ? 2.0f * Lm : 2.0f * Lm * (1.0f + 1e-5f) + 1e-5f;
    const float vmax = sqrtf(A * T2 * idet);
    const float umax = bare ? sqrtf(C * T2 * idet) : sqrtf(C * T2 * idet) * (1.0f + 1e-5f) + 0.02f;
    if (!(vmax < 1e30f) || !(umax < 1e30f)) return 0;
    const float ut = -B * vmax * (1.0f / A), ev = bare ? 0.0f : 2e-3f * vmax + 0.02f;
    const float rc = 1.0f / C, cT2 = C * T2;
    const float ylo = py - ev - 15.0f - 16.0f * (float)sy0, yhi = py + ev - 16.0f * (float)sy0;
    const float hmax = (float)(h - 1);
    float b = 16.0f * (float)x0 - 0.5f - px;
    float u0 = fminf(fmaxf(b, -umax), umax);
    float h0 = sqrtf(fmaxf(0.0f, cT2 - det * u0 * u0));
    float up0 = (-B * u0 + h0) * rc, dn0 = (-B * u0 - h0) * rc;
    for (uint32_t c = 0; c < w; ++c) {
        const float b1 = b + 16.0f;
        const float u1 = fminf(fmaxf(b1, -umax), umax);
        const float h1 = sqrtf(fmaxf(0.0f, cT2 - det * u1 * u1));
        const float up1 = (-B * u1 + h1) * rc, dn1 = (-B * u1 - h1) * rc;
        lo_out[c] = 0u;
        cnt_out[c] = 0u;
        if (b <= umax && b1 >= -umax) {
            const float vhi = (ut >= u0 && ut <= u1) ? vmax : fmaxf(up0, up1);
            const float vlo = (-ut >= u0 && -ut <= u1) ? -vmax : fminf(dn0, dn1);
            const float lo = fmaxf(ceilf((ylo + vlo) * 0.0625f), 0.0f);
            const float hi = fminf(floorf((yhi + vhi) * 0.0625f), hmax);
            if (lo <= hi) {
                lo_out[c] = (uint32_t)lo;
                cnt_out[c] = (uint32_t)(hi - lo) + 1u;
            }
        }
        b = b1, u0 = u1, up0 = up1, dn0 = dn1;
    }
    return 1;
}

static uint32_t tc_umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
static int tc_imax(int a, int b) { return a > b ? a : b; }
static int tc_f2i_sat(float v) {
    if (isnan(v)) return 0;
    if (v >= 2147483648.0f) return 2147483647;
    if (v <= -2147483648.0f) return (-2147483647 - 1);
    return (int)v;
}

/* For every Gaussian with radii > 0 (the oracle's preprocess outputs): its getRect rect, the
 * model's spans when the rect is span-coded (<= 8 columns x <= 15 rows), and for every rect
 * tile outside the spans the 256-pixel check (shrink > 0: the mutation of model_cull_Lm).
 * stats (int64[8]):
 *   [0] span-coded Gaussians, [1] their rect tiles, [2] tiles the spans drop,
 *   [3] dropped tiles reached at alpha >= 1/255 (must be 0), [4] first offending Gaussian (-1),
 *   [5] largest alpha (x 1e9) of a dropped tile, [6] Gaussians with rects too large to code,
 *   [7] span-coded rects with exactly 8 columns. */
int64_t oracle_tight_model_check(int64_t P, const float *means2D, const float *conic_opacity,
                                 const int32_t *radii, int W, int H, float shrink,
                                 int64_t *stats) {
    const int bare = shrink > 0.0f;
    const uint32_t gx = (uint32_t)((W + TC_BLOCK - 1) / TC_BLOCK);
    const uint32_t gy = (uint32_t)((H + TC_BLOCK - 1) / TC_BLOCK);
    int64_t coded = 0, tiles = 0, dropped = 0, bad = 0, big = 0, eight = 0;
    int64_t first = -1;
    float worst = 0.0f;
#pragma omp parallel for schedule(dynamic, 256) \
    reduction(+ : coded, tiles, dropped, bad, big, eight) reduction(max : worst)
    for (int64_t i = 0; i < P; ++i) {
        if (radii[i] <= 0) continue;
        const float px = means2D[2 * i], py = means2D[2 * i + 1];
        const int r = radii[i];
        const uint32_t x0 = tc_umin(gx, (uint32_t)tc_imax(0, tc_f2i_sat((px - r) / TC_BLOCK)));
        const uint32_t y0 = tc_umin(gy, (uint32_t)tc_imax(0, tc_f2i_sat((py - r) / TC_BLOCK)));
        const uint32_t x1 =
            tc_umin(gx, (uint32_t)tc_imax(0, tc_f2i_sat((px + r + TC_BLOCK - 1) / TC_BLOCK)));
        const uint32_t y1 =
            tc_umin(gy, (uint32_t)tc_imax(0, tc_f2i_sat((py + r + TC_BLOCK - 1) / TC_BLOCK)));
        const uint32_t w = x1 - x0, h = y1 - y0;
        if (w == 0 || h == 0) continue;
        if (w > kSpanCols || h > kSpanRows) {
            big++;
            continue;
        }
        coded++;
        if (w == kSpanCols) eight++;
        tiles += (int64_t)w * h;
        const float *co = conic_opacity + 4 * i;
        const float Lm = model_cull_Lm(co[0], co[1], co[2], co[3], shrink);
        uint32_t lo[kSpanCols], cnt[kSpanCols];
        if (!model_col_spans(px, py, co[0], co[1], co[2], Lm, x0, w, y0, h, lo, cnt, bare))
            continue;
        for (uint32_t c = 0; c < w; ++c)
            for (uint32_t rr = 0; rr < h; ++rr) {
                if (rr >= lo[c] && rr < lo[c] + cnt[c]) continue;
                dropped++;
                float a = 0.0f;
                if (reaches_tile(means2D, conic_opacity, (uint32_t)i, x0 + c, y0 + rr, &a)) {
                    bad++;
#pragma omp critical(tight_model_first)
                    if (first < 0 || i < first) first = i;
                }
                if (a > worst) worst = a;
            }
    }
    stats[0] = coded;
    stats[1] = tiles;
    stats[2] = dropped;
    stats[3] = bad;
    stats[4] = first;
    stats[5] = (int64_t)floor((double)worst * 1e9);
    stats[6] = big;
    stats[7] = eight;
    return bad;
}
