/*
 * gsr_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement ("oracle") of the forward Gaussian-splat rasterizer that the reference
 * viewer calls through `diff_gaussian_rasterization.GaussianRasterizer`
 * (/root/reference/renderer_cuda.py:13, :211-224), plus the reference's own depth-sort
 * backend (/root/reference/renderer_ogl.py:10-19).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline.  The product path
 * (gaussiansplattingviewer_amd/) never calls it and fails loudly without its HIP library.
 *
 * Provenance of the algorithm:
 *   - The rasterizer lives in the third-party `diff-gaussian-rasterization` (graphdeco-inria),
 *     NOT vendored in /root/reference and NOT pinned to a version (README.md:29 links the repo
 *     head; requirements.txt omits it).  renderer_cuda.py:215 unpacks a 2-tuple (color, radii),
 *     which pins the behaviour to the original forward (before the depth-output revision).
 *     Each function below restates the published upstream function it names
 *     (forward.cu: preprocessCUDA / computeCov3D / computeCov2D / computeColorFromSH /
 *     renderCUDA; auxiliary.h: in_frustum / transformPoint4x3 / transformPoint4x4 /
 *     ndc2Pix / getRect; rasterizer_impl.cu: duplicateWithKeys / getHigherMsb /
 *     identifyTileRanges and the cub InclusiveSum / stable SortPairs calls).
 *   - The in-repo GLSL twins of the same formulas are cited where they exist
 *     (shaders/gau_vert.glsl:73-93 Sigma3D, :95-120 EWA Sigma2D, :213-250 SH;
 *     shaders/gau_frag.glsl:21-27 alpha).
 *
 * PARITY STATUS: the forward is "parity unpinned" -- no fixture produced by the real
 * upstream CUDA forward exists in the reference or in this container, and nvcc's default
 * FMA contraction makes bitwise agreement with it unattainable anyway.  The depth-sort
 * backend IS pinned: oracle_view_depth() reproduces, bit for bit, the depth array that the
 * reference's _sort_gaussian_cpu produced in the build container (tests/golden/).
 *
 * Arithmetic contract (shared with the HIP kernels, which must match the integer outputs
 * bit-exactly): IEEE float32, no FMA contraction (-ffp-contract=off), correctly rounded
 * division and sqrt, evaluation order exactly as written in upstream C++ (left-to-right
 * sums, glm column-major mat3 products).  ndc2Pix evaluates in double because upstream's
 * literals 1.0 / 0.5 are doubles.
 *
 * Threads (OpenMP, oracle_set_threads; for the bench's host-cores CPU baseline): the
 * preprocess runs Gaussians in parallel, the duplication fills each Gaussian's precomputed
 * range, the stable LSD sort counts and scatters per contiguous chunk (chunk-ordered offsets
 * keep it stable), and the render runs tiles in parallel.  Every output element is computed by
 * the same operations as in the serial order, so results do not depend on the thread count.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define BLOCK_X 16
#define BLOCK_Y 16
#define BLOCK_SIZE (BLOCK_X * BLOCK_Y)

/* SH basis constants: upstream forward.cu (float literals), identical to
 * shaders/gau_vert.glsl:3-18. */
static const float SH_C0 = 0.28209479177387814f;
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

/* ---- glm-style column-major mat3: m[col][row] ------------------------------------- */
typedef struct { float m[3][3]; } mat3;

static mat3 mat3_cols(float a0, float a1, float a2, float a3, float a4, float a5, float a6,
                      float a7, float a8) {
    /* glm::mat3(x0,y0,z0, x1,y1,z1, x2,y2,z2): column c = (a[3c], a[3c+1], a[3c+2]) */
    mat3 r;
    r.m[0][0] = a0; r.m[0][1] = a1; r.m[0][2] = a2;
    r.m[1][0] = a3; r.m[1][1] = a4; r.m[1][2] = a5;
    r.m[2][0] = a6; r.m[2][1] = a7; r.m[2][2] = a8;
    return r;
}

static mat3 mat3_mul(const mat3 *a, const mat3 *b) {
    /* glm operator*(mat3, mat3): R[j][i] = (A[0][i]*B[j][0] + A[1][i]*B[j][1]) + A[2][i]*B[j][2] */
    mat3 r;
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) {
            float s = a->m[0][i] * b->m[j][0];
            s = s + a->m[1][i] * b->m[j][1];
            s = s + a->m[2][i] * b->m[j][2];
            r.m[j][i] = s;
        }
    return r;
}

static mat3 mat3_transpose(const mat3 *a) {
    mat3 r;
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) r.m[i][j] = a->m[j][i];
    return r;
}

/* ---- auxiliary.h ---------------------------------------------------------------- */
static void transform_point_4x3(const float p[3], const float *M, float out[3]) {
    out[0] = M[0] * p[0] + M[4] * p[1] + M[8] * p[2] + M[12];
    out[1] = M[1] * p[0] + M[5] * p[1] + M[9] * p[2] + M[13];
    out[2] = M[2] * p[0] + M[6] * p[1] + M[10] * p[2] + M[14];
}

static void transform_point_4x4(const float p[3], const float *M, float out[4]) {
    out[0] = M[0] * p[0] + M[4] * p[1] + M[8] * p[2] + M[12];
    out[1] = M[1] * p[0] + M[5] * p[1] + M[9] * p[2] + M[13];
    out[2] = M[2] * p[0] + M[6] * p[1] + M[10] * p[2] + M[14];
    out[3] = M[3] * p[0] + M[7] * p[1] + M[11] * p[2] + M[15];
}

static float ndc2pix(float v, int S) { return (float)(((v + 1.0) * S - 1.0) * 0.5); }

static uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

/* float -> int as CUDA's cvt.rzi.s32.f32 (what `(int)` compiles to in upstream device
 * code): truncate toward zero, saturate out-of-range values, NaN -> 0.  (A plain C cast
 * is undefined there; x86 would return INT_MIN.) */
static int f2i_sat(float v) {
    if (isnan(v)) return 0;
    if (v >= 2147483648.0f) return 2147483647;
    if (v <= -2147483648.0f) return (-2147483647 - 1);
    return (int)v;
}
static int imax(int a, int b) { return a > b ? a : b; }

static void get_rect(float px, float py, int max_radius, uint32_t gx, uint32_t gy,
                     uint32_t rmin[2], uint32_t rmax[2]) {
    rmin[0] = umin(gx, (uint32_t)imax(0, f2i_sat((px - max_radius) / BLOCK_X)));
    rmin[1] = umin(gy, (uint32_t)imax(0, f2i_sat((py - max_radius) / BLOCK_Y)));
    rmax[0] = umin(gx, (uint32_t)imax(0, f2i_sat((px + max_radius + BLOCK_X - 1) / BLOCK_X)));
    rmax[1] = umin(gy, (uint32_t)imax(0, f2i_sat((py + max_radius + BLOCK_Y - 1) / BLOCK_Y)));
}

/* ---- forward.cu: computeCov3D ------------------------------------------------------ */
static void compute_cov3d(const float scale[3], float mod, const float rot[4], float cov3d[6]) {
    mat3 S = mat3_cols(1.f, 0.f, 0.f, 0.f, 1.f, 0.f, 0.f, 0.f, 1.f);
    S.m[0][0] = mod * scale[0];
    S.m[1][1] = mod * scale[1];
    S.m[2][2] = mod * scale[2];
    const float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    mat3 R = mat3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                       2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                       2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    mat3 M = mat3_mul(&S, &R);
    mat3 Mt = mat3_transpose(&M);
    mat3 Sig = mat3_mul(&Mt, &M);
    cov3d[0] = Sig.m[0][0];
    cov3d[1] = Sig.m[0][1];
    cov3d[2] = Sig.m[0][2];
    cov3d[3] = Sig.m[1][1];
    cov3d[4] = Sig.m[1][2];
    cov3d[5] = Sig.m[2][2];
}

/* ---- forward.cu: computeCov2D (EWA splatting, + 0.3 low-pass) ---------------------- */
static void compute_cov2d(const float mean[3], float fx, float fy, float tanfovx, float tanfovy,
                          const float *c, const float *vm, float out[3]) {
    float t[3];
    transform_point_4x3(mean, vm, t);
    const float limx = 1.3f * tanfovx;
    const float limy = 1.3f * tanfovy;
    const float txtz = t[0] / t[2];
    const float tytz = t[1] / t[2];
    t[0] = fminf(limx, fmaxf(-limx, txtz)) * t[2];
    t[1] = fminf(limy, fmaxf(-limy, tytz)) * t[2];

    mat3 J = mat3_cols(fx / t[2], 0.0f, -(fx * t[0]) / (t[2] * t[2]), 0.0f, fy / t[2],
                       -(fy * t[1]) / (t[2] * t[2]), 0.f, 0.f, 0.f);
    mat3 W = mat3_cols(vm[0], vm[4], vm[8], vm[1], vm[5], vm[9], vm[2], vm[6], vm[10]);
    mat3 T = mat3_mul(&W, &J);
    mat3 Vrk = mat3_cols(c[0], c[1], c[2], c[1], c[3], c[4], c[2], c[4], c[5]);
    mat3 Tt = mat3_transpose(&T);
    mat3 Vt = mat3_transpose(&Vrk);
    mat3 A = mat3_mul(&Tt, &Vt);
    mat3 cov = mat3_mul(&A, &T);
    cov.m[0][0] += 0.3f;
    cov.m[1][1] += 0.3f;
    out[0] = cov.m[0][0];
    out[1] = cov.m[0][1];
    out[2] = cov.m[1][1];
}

/* ---- forward.cu: computeColorFromSH ------------------------------------------------ */
static void compute_color_from_sh(int64_t idx, int deg, int max_coeffs, const float *means,
                                  const float *campos, const float *shs, uint8_t *clamped,
                                  float out[3]) {
    float dir[3] = {means[3 * idx + 0] - campos[0], means[3 * idx + 1] - campos[1],
                    means[3 * idx + 2] - campos[2]};
    const float len = sqrtf(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    dir[0] = dir[0] / len;
    dir[1] = dir[1] / len;
    dir[2] = dir[2] / len;
    const float *sh = shs + idx * max_coeffs * 3;
    float res[3];
    for (int c = 0; c < 3; ++c) res[c] = SH_C0 * sh[0 * 3 + c];
    if (deg > 0) {
        const float x = dir[0], y = dir[1], z = dir[2];
        const float a1 = SH_C1 * y, a2 = SH_C1 * z, a3 = SH_C1 * x;
        for (int c = 0; c < 3; ++c)
            res[c] = res[c] - a1 * sh[1 * 3 + c] + a2 * sh[2 * 3 + c] - a3 * sh[3 * 3 + c];
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
            const float b0 = SH_C2[0] * xy;
            const float b1 = SH_C2[1] * yz;
            const float b2 = SH_C2[2] * (2.0f * zz - xx - yy);
            const float b3 = SH_C2[3] * xz;
            const float b4 = SH_C2[4] * (xx - yy);
            for (int c = 0; c < 3; ++c)
                res[c] = res[c] + b0 * sh[4 * 3 + c] + b1 * sh[5 * 3 + c] + b2 * sh[6 * 3 + c] +
                         b3 * sh[7 * 3 + c] + b4 * sh[8 * 3 + c];
            if (deg > 2) {
                const float e0 = SH_C3[0] * y * (3.0f * xx - yy);
                const float e1 = SH_C3[1] * xy * z;
                const float e2 = SH_C3[2] * y * (4.0f * zz - xx - yy);
                const float e3 = SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
                const float e4 = SH_C3[4] * x * (4.0f * zz - xx - yy);
                const float e5 = SH_C3[5] * z * (xx - yy);
                const float e6 = SH_C3[6] * x * (xx - 3.0f * yy);
                for (int c = 0; c < 3; ++c)
                    res[c] = res[c] + e0 * sh[9 * 3 + c] + e1 * sh[10 * 3 + c] +
                             e2 * sh[11 * 3 + c] + e3 * sh[12 * 3 + c] + e4 * sh[13 * 3 + c] +
                             e5 * sh[14 * 3 + c] + e6 * sh[15 * 3 + c];
            }
        }
    }
    for (int c = 0; c < 3; ++c) {
        res[c] += 0.5f;
        if (clamped) clamped[3 * idx + c] = res[c] < 0;
        out[c] = fmaxf(res[c], 0.0f);
    }
}

/* ---- public oracle entry points ----------------------------------------------------- */
typedef struct {
    int64_t P;
    int D, M;
    float scale_modifier;
    const float *means3D, *scales, *rotations, *opacities, *shs, *colors_precomp, *cov3D_precomp;
    const float *viewmatrix, *projmatrix, *campos, *bg; /* column-major 4x4, as upstream */
    float tanfovx, tanfovy;
    int W, H;
} OracleIn;

/* forward.cu: preprocessCUDA, one Gaussian at a time.  Returns K = sum(tiles_touched)
 * (the value upstream reads back as num_rendered after InclusiveSum). */
int64_t oracle_preprocess(const OracleIn *in, float *depths, int32_t *radii, float *means2D,
                          float *conic_opacity, float *rgb, uint8_t *clamped,
                          uint32_t *tiles_touched, float *cov3Ds) {
    const uint32_t gx = (uint32_t)((in->W + BLOCK_X - 1) / BLOCK_X);
    const uint32_t gy = (uint32_t)((in->H + BLOCK_Y - 1) / BLOCK_Y);
    const float focal_y = in->H / (2.0f * in->tanfovy);
    const float focal_x = in->W / (2.0f * in->tanfovx);
    int64_t K = 0;
#pragma omp parallel for schedule(static, 4096) reduction(+ : K)
    for (int64_t idx = 0; idx < in->P; ++idx) {
        radii[idx] = 0;
        tiles_touched[idx] = 0;
        const float p[3] = {in->means3D[3 * idx], in->means3D[3 * idx + 1],
                            in->means3D[3 * idx + 2]};
        /* in_frustum */
        float p_view[3];
        transform_point_4x3(p, in->viewmatrix, p_view);
        if (p_view[2] <= 0.2f) continue;

        float p_hom[4];
        transform_point_4x4(p, in->projmatrix, p_hom);
        const float p_w = 1.0f / (p_hom[3] + 0.0000001f);
        const float p_proj[3] = {p_hom[0] * p_w, p_hom[1] * p_w, p_hom[2] * p_w};

        float cov3d_local[6];
        const float *cov3D;
        if (in->cov3D_precomp) {
            cov3D = in->cov3D_precomp + 6 * idx;
        } else {
            compute_cov3d(in->scales + 3 * idx, in->scale_modifier, in->rotations + 4 * idx,
                          cov3d_local);
            if (cov3Ds) memcpy(cov3Ds + 6 * idx, cov3d_local, sizeof(cov3d_local));
            cov3D = cov3d_local;
        }
        float cov[3];
        compute_cov2d(p, focal_x, focal_y, in->tanfovx, in->tanfovy, cov3D, in->viewmatrix, cov);

        const float det = cov[0] * cov[2] - cov[1] * cov[1];
        if (det == 0.0f) continue;
        const float det_inv = 1.f / det;
        const float conic[3] = {cov[2] * det_inv, -cov[1] * det_inv, cov[0] * det_inv};

        const float mid = 0.5f * (cov[0] + cov[2]);
        const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
        const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
        const float pimg[2] = {ndc2pix(p_proj[0], in->W), ndc2pix(p_proj[1], in->H)};
        uint32_t rmin[2], rmax[2];
        get_rect(pimg[0], pimg[1], f2i_sat(my_radius), gx, gy, rmin, rmax);
        if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) continue;

        if (!in->colors_precomp) {
            float col[3];
            compute_color_from_sh(idx, in->D, in->M, in->means3D, in->campos, in->shs, clamped,
                                  col);
            rgb[3 * idx + 0] = col[0];
            rgb[3 * idx + 1] = col[1];
            rgb[3 * idx + 2] = col[2];
        }
        depths[idx] = p_view[2];
        radii[idx] = f2i_sat(my_radius);
        means2D[2 * idx + 0] = pimg[0];
        means2D[2 * idx + 1] = pimg[1];
        conic_opacity[4 * idx + 0] = conic[0];
        conic_opacity[4 * idx + 1] = conic[1];
        conic_opacity[4 * idx + 2] = conic[2];
        conic_opacity[4 * idx + 3] = in->opacities[idx];
        tiles_touched[idx] = (rmax[1] - rmin[1]) * (rmax[0] - rmin[0]);
        K += tiles_touched[idx];
    }
    return K;
}

/* rasterizer_impl.cu: getHigherMsb -- bits needed for tile ids < n. */
static uint32_t get_higher_msb(uint32_t n) {
    uint32_t msb = sizeof(n) * 4;
    uint32_t step = msb;
    while (step > 1) {
        step /= 2;
        if (n >> msb) msb += step;
        else msb -= step;
    }
    if (n >> msb) msb++;
    return msb;
}

/* Stable LSD radix sort of (key, value) on key bits [0, end_bit): the contract of
 * cub::DeviceRadixSort::SortPairs as rasterizer_impl.cu calls it.  8-bit digits; each pass
 * counts per contiguous chunk (one per thread), offsets digit-major then chunk-major, and
 * every chunk scatters its elements in order -- the stable counting sort, in parallel. */
#define SORT_MAX_CHUNKS 256
static int sort_pairs_u64(uint64_t *keys, uint32_t *vals, int64_t n, int end_bit) {
    uint64_t *k2 = (uint64_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(uint64_t));
    uint32_t *v2 = (uint32_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(uint32_t));
    int64_t(*cnt)[256] = malloc(sizeof(int64_t[256]) * SORT_MAX_CHUNKS);
    if (!k2 || !v2 || !cnt) { free(k2); free(v2); free(cnt); return -1; }
    int nch = omp_get_max_threads();
    if (nch > SORT_MAX_CHUNKS) nch = SORT_MAX_CHUNKS;
    if (nch < 1 || n < 65536) nch = 1;
    uint64_t *ka = keys, *kb = k2;
    uint32_t *va = vals, *vb = v2;
    for (int shift = 0; shift < end_bit; shift += 8) {
#pragma omp parallel for num_threads(nch) schedule(static, 1)
        for (int c = 0; c < nch; ++c) {
            const int64_t b = n * c / nch, e = n * (c + 1) / nch;
            memset(cnt[c], 0, sizeof(cnt[c]));
            for (int64_t i = b; i < e; ++i) cnt[c][(ka[i] >> shift) & 0xFF]++;
        }
        int64_t run = 0;
        for (int d = 0; d < 256; ++d)
            for (int c = 0; c < nch; ++c) {
                const int64_t t = cnt[c][d];
                cnt[c][d] = run;
                run += t;
            }
#pragma omp parallel for num_threads(nch) schedule(static, 1)
        for (int c = 0; c < nch; ++c) {
            const int64_t b = n * c / nch, e = n * (c + 1) / nch;
            for (int64_t i = b; i < e; ++i) {
                const int64_t pos = cnt[c][(ka[i] >> shift) & 0xFF]++;
                kb[pos] = ka[i];
                vb[pos] = va[i];
            }
        }
        uint64_t *tk = ka; ka = kb; kb = tk;
        uint32_t *tv = va; va = vb; vb = tv;
    }
    if (ka != keys) {
        memcpy(keys, ka, (size_t)n * sizeof(uint64_t));
        memcpy(vals, va, (size_t)n * sizeof(uint32_t));
    }
    free(k2);
    free(v2);
    free(cnt);
    return 0;
}

/* rasterizer_impl.cu: InclusiveSum(tiles_touched) + duplicateWithKeys + SortPairs +
 * identifyTileRanges.  keys/vals hold K entries, ranges 2*T uint32 (uint2 per tile). */
int oracle_bin(const OracleIn *in, const float *depths, const int32_t *radii,
               const float *means2D, const uint32_t *tiles_touched, int64_t K, uint64_t *keys,
               uint32_t *vals, uint32_t *ranges) {
    const uint32_t gx = (uint32_t)((in->W + BLOCK_X - 1) / BLOCK_X);
    const uint32_t gy = (uint32_t)((in->H + BLOCK_Y - 1) / BLOCK_Y);
    /* InclusiveSum(tiles_touched) as exclusive offsets, then duplicateWithKeys per Gaussian */
    int64_t *offs = (int64_t *)malloc((size_t)(in->P > 0 ? in->P : 1) * sizeof(int64_t));
    if (!offs) return -1;
    int64_t off = 0;
    for (int64_t idx = 0; idx < in->P; ++idx) {
        offs[idx] = off;
        if (radii[idx] > 0) off += tiles_touched[idx];
    }
    if (off != K) { free(offs); return -3; }
#pragma omp parallel for schedule(static, 4096)
    for (int64_t idx = 0; idx < in->P; ++idx) {
        if (radii[idx] > 0) {
            uint32_t rmin[2], rmax[2];
            get_rect(means2D[2 * idx], means2D[2 * idx + 1], radii[idx], gx, gy, rmin, rmax);
            uint32_t dbits;
            memcpy(&dbits, &depths[idx], 4);
            int64_t o = offs[idx];
            for (uint32_t y = rmin[1]; y < rmax[1]; ++y)
                for (uint32_t x = rmin[0]; x < rmax[0]; ++x) {
                    keys[o] = ((uint64_t)(y * gx + x) << 32) | dbits;
                    vals[o] = (uint32_t)idx;
                    ++o;
                }
        }
    }
    free(offs);
    const int bit = (int)get_higher_msb(gx * gy);
    if (sort_pairs_u64(keys, vals, K, 32 + bit) != 0) return -1;
    memset(ranges, 0, (size_t)gx * gy * 2 * sizeof(uint32_t));
    for (int64_t i = 0; i < K; ++i) {
        const uint32_t cur = (uint32_t)(keys[i] >> 32);
        if (i == 0) ranges[2 * cur] = 0;
        else {
            const uint32_t prev = (uint32_t)(keys[i - 1] >> 32);
            if (cur != prev) {
                ranges[2 * prev + 1] = (uint32_t)i;
                ranges[2 * cur] = (uint32_t)i;
            }
        }
        if (i == K - 1) ranges[2 * cur + 1] = (uint32_t)K;
    }
    return 0;
}

/* forward.cu: renderCUDA, one pixel at a time (the per-pixel result does not depend on
 * the 256-splat batching or the block-wide done count). */
void oracle_render(const OracleIn *in, const uint32_t *ranges, const uint32_t *point_list,
                   const float *means2D, const float *features, const float *conic_opacity,
                   float *out_color, float *final_T, uint32_t *n_contrib) {
    const int W = in->W, H = in->H;
    const uint32_t gx = (uint32_t)((W + BLOCK_X - 1) / BLOCK_X);
    const uint32_t gy = (uint32_t)((H + BLOCK_Y - 1) / BLOCK_Y);
#pragma omp parallel for collapse(2) schedule(dynamic, 4)
    for (uint32_t ty = 0; ty < gy; ++ty)
        for (uint32_t tx = 0; tx < gx; ++tx) {
            const uint32_t r0 = ranges[2 * (ty * gx + tx)], r1 = ranges[2 * (ty * gx + tx) + 1];
            for (uint32_t ly = 0; ly < BLOCK_Y; ++ly)
                for (uint32_t lx = 0; lx < BLOCK_X; ++lx) {
                    const uint32_t px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
                    if (px >= (uint32_t)W || py >= (uint32_t)H) continue;
                    const float pfx = (float)px, pfy = (float)py;
                    float T = 1.0f, C[3] = {0.f, 0.f, 0.f};
                    uint32_t contributor = 0, last_contributor = 0;
                    for (uint32_t j = r0; j < r1; ++j) {
                        contributor++;
                        const uint32_t id = point_list[j];
                        const float dx = means2D[2 * id] - pfx;
                        const float dy = means2D[2 * id + 1] - pfy;
                        const float *co = conic_opacity + 4 * id;
                        const float power =
                            -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                        if (power > 0.0f) continue;
                        const float alpha = fminf(0.99f, co[3] * expf(power));
                        if (alpha < 1.0f / 255.0f) continue;
                        const float test_T = T * (1 - alpha);
                        if (test_T < 0.0001f) break; /* done: no later splat is evaluated */
                        for (int ch = 0; ch < 3; ++ch) C[ch] += features[3 * id + ch] * alpha * T;
                        T = test_T;
                        last_contributor = contributor;
                    }
                    const size_t pid = (size_t)W * py + px;
                    final_T[pid] = T;
                    n_contrib[pid] = last_contributor;
                    for (int ch = 0; ch < 3; ++ch)
                        out_color[(size_t)ch * H * W + pid] = C[ch] + T * in->bg[ch];
                }
        }
}

/* forward.cu computeColorFromSH over P Gaussians (every one, not only the visible): rgb[3P]
 * the clamped colour, clamped[3P] (optional) its clamp flags -- so the pre-clamp value is rgb
 * where the flag is 0.  For the GLSL-twin check (tests/test_oracle_glsl_twins.py). */
void oracle_color_from_sh(int64_t P, int deg, int max_coeffs, const float *means,
                          const float *campos, const float *shs, float *rgb, uint8_t *clamped) {
    for (int64_t i = 0; i < P; ++i)
        compute_color_from_sh(i, deg, max_coeffs, means, campos, shs, clamped, rgb + 3 * i);
}

/* forward.cu computeCov3D over P Gaussians: cov3d[6P] (xx, xy, xz, yy, yz, zz). */
void oracle_cov3d(int64_t P, const float *scales, float mod, const float *rots, float *cov3d) {
    for (int64_t i = 0; i < P; ++i) compute_cov3d(scales + 3 * i, mod, rots + 4 * i, cov3d + 6 * i);
}

/* Threads of the parallel loops above (< 1: back to OpenMP's initial default, e.g.
 * OMP_NUM_THREADS); returns the count in effect. */
int oracle_set_threads(int n) {
    static int initial = 0;
    if (initial == 0) initial = omp_get_max_threads();
    omp_set_num_threads(n >= 1 ? n : initial);
    return omp_get_max_threads();
}

/* Reference sort backend (renderer_ogl.py:10-19): view-space z of every point.  The
 * reference computes it with a numpy stacked matmul; in the build container that
 * evaluates, bit for bit, as fma(v22, z, fma(v20, x, v21*y)) + v23.
 * view is the 4x4 math-layout (row-major) matrix the reference passes. */
void oracle_view_depth(const float *xyz, int64_t P, const float *view, float *depth) {
    const float v20 = view[8], v21 = view[9], v22 = view[10], v23 = view[11];
    for (int64_t i = 0; i < P; ++i) {
        const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
        depth[i] = fmaf(v22, z, fmaf(v20, x, v21 * y)) + v23;
    }
}

/* Stable ascending argsort of float32 keys (== np.argsort(d, kind='stable')), used as the
 * CPU baseline of the depth-sort backend and to check the device depth sort. */
int oracle_argsort_f32(const float *d, int64_t n, int32_t *out) {
    uint64_t *keys = (uint64_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(uint64_t));
    uint32_t *vals = (uint32_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(uint32_t));
    if (!keys || !vals) { free(keys); free(vals); return -1; }
    for (int64_t i = 0; i < n; ++i) {
        uint32_t u;
        memcpy(&u, &d[i], 4);
        if (d[i] == 0.0f) u = 0u;                        /* -0 ties +0, as in numpy */
        u = (u & 0x80000000u) ? ~u : (u | 0x80000000u); /* order-preserving float->uint */
        if (isnan(d[i])) u = 0xFFFFFFFFu;                /* every NaN last, stable */
        keys[i] = u;
        vals[i] = (uint32_t)i;
    }
    int rc = sort_pairs_u64(keys, vals, n, 32);
    for (int64_t i = 0; i < n; ++i) out[i] = (int32_t)vals[i];
    free(keys);
    free(vals);
    return rc;
}
