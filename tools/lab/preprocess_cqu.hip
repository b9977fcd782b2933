// preprocess.hip -- per-Gaussian EWA projection + SH -> RGB (gfx950).
//
// Replaces upstream diff-gaussian-rasterization forward.cu preprocessCUDA (called from
// renderer_cuda.py:215 via GaussianRasterizer.forward) and auxiliary.h in_frustum.
// Two kernels, one thread per Gaussian, 256-thread blocks:
//  * k_preprocess -- projection, covariance, conic, radius, tile rect, depth key: reads xyz
//    (12 B) for every point and scale/rot/opacity (32 B) for points in front of the camera;
//    writes the geometry of the 48-B SplatRecord for visible points, the 8-B (key, id) pair
//    of the depth sort, the radius and the packed strip rect.
//  * k_color -- SH -> RGB for the visible points: reads xyz + SH (192 B at degree 3), writes
//    the record's colour.  It depends only on k_preprocess's radii and nothing before the
//    blend reads colour, so api.hip runs it on a second stream, overlapped with the depth
//    sort and the binning (which are latency-bound and leave most CUs idle).
#include <algorithm>

#include "gsr_internal.h"

using namespace gsr;

namespace {

__constant__ float kShC0 = 0.28209479177387814f;
__constant__ float kShC1 = 0.4886025119029199f;
__constant__ float kShC2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
__constant__ float kShC3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

// upstream forward.cu computeColorFromSH (twin: shaders/gau_vert.glsl:213-250), but with the
// coefficients read as 16-B vectors: the (P, M, 3) row of one Gaussian is 192 B = 12 float4
// at degree 3 (M = 16), so each lane issues 12 dwordx4 loads instead of 48 dword loads.
__device__ __forceinline__ float3 eval_sh(float3 pos, const float *campos, const float (&c)[48],
                                          int deg);

__device__ __forceinline__ float3 color_from_sh(float3 pos, const float *campos, const float *sh,
                                                int deg, bool vec_ok) {
    // Load the coefficients this degree needs: (deg+1)^2 of the M stored (host checks
    // (deg+1)^2 <= M).  Both loops are fully unrolled so `c` stays in registers.
    float c[48];
    const int ncoef = (deg + 1) * (deg + 1);
    if (vec_ok) {  // M == 16 and 16-B aligned rows
        const float4 *v = reinterpret_cast<const float4 *>(sh);
        const int nvec = (ncoef * 3 + 3) >> 2;
        // all 12 loads unconditionally (the row always holds 16 coefficients), so they issue
        // together instead of one predicated round trip each; unused ones are zeroed after
        float4 rowv[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) rowv[i] = v[i];
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
            if (i < nvec) q = rowv[i];
            c[4 * i + 0] = q.x;
            c[4 * i + 1] = q.y;
            c[4 * i + 2] = q.z;
            c[4 * i + 3] = q.w;
        }
    } else {
        const int nflt = ncoef * 3;
#pragma unroll
        for (int i = 0; i < 48; ++i) c[i] = (i < nflt) ? sh[i] : 0.0f;
    }
    return eval_sh(pos, campos, c, deg);
}

__device__ __forceinline__ float3 eval_sh(float3 pos, const float *campos, const float (&c)[48],
                                          int deg) {
    float dx = pos.x - campos[0], dy = pos.y - campos[1], dz = pos.z - campos[2];
    const float len = sqrtf(dx * dx + dy * dy + dz * dz);
    dx = dx / len;
    dy = dy / len;
    dz = dz / len;
    float r0 = kShC0 * c[0], r1 = kShC0 * c[1], r2 = kShC0 * c[2];
    if (deg > 0) {
        const float x = dx, y = dy, z = dz;
        const float a1 = kShC1 * y, a2 = kShC1 * z, a3 = kShC1 * x;
        r0 = r0 - a1 * c[3] + a2 * c[6] - a3 * c[9];
        r1 = r1 - a1 * c[4] + a2 * c[7] - a3 * c[10];
        r2 = r2 - a1 * c[5] + a2 * c[8] - a3 * c[11];
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z;
            const float xy = x * y, yz = y * z, xz = x * z;
            const float b0 = kShC2[0] * xy;
            const float b1 = kShC2[1] * yz;
            const float b2 = kShC2[2] * (2.0f * zz - xx - yy);
            const float b3 = kShC2[3] * xz;
            const float b4 = kShC2[4] * (xx - yy);
            r0 = r0 + b0 * c[12] + b1 * c[15] + b2 * c[18] + b3 * c[21] + b4 * c[24];
            r1 = r1 + b0 * c[13] + b1 * c[16] + b2 * c[19] + b3 * c[22] + b4 * c[25];
            r2 = r2 + b0 * c[14] + b1 * c[17] + b2 * c[20] + b3 * c[23] + b4 * c[26];
            if (deg > 2) {
                const float e0 = kShC3[0] * y * (3.0f * xx - yy);
                const float e1 = kShC3[1] * xy * z;
                const float e2 = kShC3[2] * y * (4.0f * zz - xx - yy);
                const float e3 = kShC3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
                const float e4 = kShC3[4] * x * (4.0f * zz - xx - yy);
                const float e5 = kShC3[5] * z * (xx - yy);
                const float e6 = kShC3[6] * x * (xx - 3.0f * yy);
                r0 = r0 + e0 * c[27] + e1 * c[30] + e2 * c[33] + e3 * c[36] + e4 * c[39] +
                     e5 * c[42] + e6 * c[45];
                r1 = r1 + e0 * c[28] + e1 * c[31] + e2 * c[34] + e3 * c[37] + e4 * c[40] +
                     e5 * c[43] + e6 * c[46];
                r2 = r2 + e0 * c[29] + e1 * c[32] + e2 * c[35] + e3 * c[38] + e4 * c[41] +
                     e5 * c[44] + e6 * c[47];
            }
        }
    }
    r0 += 0.5f;
    r1 += 0.5f;
    r2 += 0.5f;
    return make_float3(fmaxf(r0, 0.0f), fmaxf(r1, 0.0f), fmaxf(r2, 0.0f));
}

// Degree-3 colour with the coefficients streamed from a 12-float4 row (k_color's LDS image):
// exactly eval_sh's operations in eval_sh's order -- per channel, the basis terms in increasing
// order, subtracted for basis 1 and 3 as upstream writes them -- but each coefficient is
// consumed as it is read, so the row never sits in 48 registers.
__device__ __forceinline__ float3 eval_sh3_stream(float3 pos, const float *campos,
                                                  const float4 *row) {
    float dx = pos.x - campos[0], dy = pos.y - campos[1], dz = pos.z - campos[2];
    const float len = sqrtf(dx * dx + dy * dy + dz * dz);
    dx = dx / len;
    dy = dy / len;
    dz = dz / len;
    const float x = dx, y = dy, z = dz;
    const float xx = x * x, yy = y * y, zz = z * z;
    const float xy = x * y, yz = y * z, xz = x * z;
    const float bs[16] = {kShC0,
                          kShC1 * y,
                          kShC1 * z,
                          kShC1 * x,
                          kShC2[0] * xy,
                          kShC2[1] * yz,
                          kShC2[2] * (2.0f * zz - xx - yy),
                          kShC2[3] * xz,
                          kShC2[4] * (xx - yy),
                          kShC3[0] * y * (3.0f * xx - yy),
                          kShC3[1] * xy * z,
                          kShC3[2] * y * (4.0f * zz - xx - yy),
                          kShC3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy),
                          kShC3[4] * x * (4.0f * zz - xx - yy),
                          kShC3[5] * z * (xx - yy),
                          kShC3[6] * x * (xx - 3.0f * yy)};
    float r[3];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const float4 q = row[i];
        const float v[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = 4 * i + u, b = k / 3, ch = k % 3;
            if (b == 0)
                r[ch] = bs[0] * v[u];
            else if (b == 1 || b == 3)
                r[ch] = r[ch] - bs[b] * v[u];
            else
                r[ch] = r[ch] + bs[b] * v[u];
        }
    }
    return make_float3(fmaxf(r[0] + 0.5f, 0.0f), fmaxf(r[1] + 0.5f, 0.0f),
                       fmaxf(r[2] + 0.5f, 0.0f));
}

// Conservative cull data of one splat for the blend: the region where it can reach
// alpha >= 1/255 is  q(d) = A dx^2 + 2B dx dy + C dy^2 <= 2 L,  L = ln(255 o)  (upstream
// alpha = min(0.99, o exp(power)), power = -q/2).  Returns {ex, ey, Lm}: Lm >= L widened by an
// absolute bound on the float rounding of the blend's `power` inside the box plus margins, and
// the half-extents (pixels) of the ellipse q <= 2 Lm, from the float conic the blend evaluates.
// Used only to skip (splat, 8x8 quadrant) pairs that provably cannot contribute; outputs are
// identical with and without it (tested).  The determinant is formed in double (A C ~ B^2 for
// elongated splats would cancel in float); the rest is float, whose rounding (~1e-6 relative
// over the chain) sits far inside the margins (+1e-3 and x1.01 on L, +0.02 px on the extents).
// (An all-double version spent ~1/3 of the preprocess kernel's VALU on software log / div.)
__device__ __forceinline__ float3 cull_data(float A, float B, float C, float o) {
    const float kInf = __builtin_huge_valf();
    const double det_d = (double)A * (double)C - (double)B * (double)B;
    if (!(det_d > 0.0) || !(A > 0.0f) || !(C > 0.0f) || !(o == o))
        return make_float3(kInf, kInf, kInf);
    const float det = (float)det_d;  // > 0, or 0 / denormal -> infinite extents below
    float L = __logf(255.0f * o);
    if (!(L > 0.0f)) L = 0.0f;
    const float sxx = C / det, syy = A / det;  // inverse of the conic
    float ex = sqrtf(2.0f * L * sxx), ey = sqrtf(2.0f * L * syy);
    // |float(power) - power| <= ~8 eps (|A|dx^2 + |C|dy^2 + 2|B dx dy|) inside the box.
    const float mag = (A + C + 2.0f * fabsf(B)) * (ex * ex + ey * ey);
    const float Lm = (L + 8.0f * 5.96e-8f * mag + 1e-3f) * 1.01f;
    ex = sqrtf(2.0f * Lm * sxx) + 0.02f;
    ey = sqrtf(2.0f * Lm * syy) + 0.02f;
    if (!(ex < 1e30f) || !(ey < 1e30f) || !(Lm < 1e30f)) return make_float3(kInf, kInf, kInf);
    // round Lm up by one ulp (Lm > 0 and finite here)
    return make_float3(ex, ey, __uint_as_float(__float_as_uint(Lm) + 1u));
}

// Span word of a span-coded strip rect (gsr_internal.h col_span): per column of the rect, the
// tile rows whose pixel-centre box meets the ellipse q(d) = A dx^2 + 2B dx dy + C dy^2 <= 2 Lm
// (cull_data's region, which holds every pixel where the blend can reach alpha >= 1/255),
// widened outward.  A column's dx range is taken as [16 x - 0.5, 16 x + 15.5] - px, so
// neighbouring columns share their boundary; over it the ellipse's dy extent is reached at the
// boundaries or, if it lies inside, at the ellipse's top / bottom point.  Returns the pair count
// over the spans.  x0 / w: the rect's tile columns; sy0 / h: its strip-clipped global tile rows.
__device__ __forceinline__ uint32_t col_spans(float px, float py, float A, float B, float C,
                                              float Lm, uint32_t x0, uint32_t w, uint32_t sy0,
                                              uint32_t h, uint2 &cols) {
    uint64_t word = 0;
    for (uint32_t c = 0; c < w; ++c) word |= (uint64_t)(h << 4) << (8 * c);
    cols = make_uint2((uint32_t)word, (uint32_t)(word >> 32));
    // the determinant with Kahan's compensated product (A C ~ B^2 for elongated splats), the
    // rest in float with the hardware reciprocal / square root (1 ulp): their rounding (~1e-6
    // relative, ~1e-3 of vmax where the square root's argument cancels at the ellipse's u
    // extremes) sits inside the margins (1e-5 on the threshold, 2e-3 vmax + 0.02 px)
    const float bb = B * B, det = __builtin_fmaf(A, C, -bb) - __builtin_fmaf(B, B, -bb);
    if (!(det > 0.0f) || !(A > 0.0f) || !(C > 0.0f) || !(Lm < 1e30f) || !(fabsf(px) < 1e30f) ||
        !(fabsf(py) < 1e30f))
        return w * h;
    const float idet = __builtin_amdgcn_rcpf(det), T2 = 2.0f * Lm * (1.0f + 1e-5f) + 1e-5f;
    const float vmax = __builtin_amdgcn_sqrtf(A * T2 * idet);
    const float umax = __builtin_amdgcn_sqrtf(C * T2 * idet) * (1.0f + 1e-5f) + 0.02f;
    if (!(vmax < 1e30f) || !(umax < 1e30f)) return w * h;
    const float ut = -B * vmax * __builtin_amdgcn_rcpf(A), ev = 2e-3f * vmax + 0.02f;
    const float rc = __builtin_amdgcn_rcpf(C), cT2 = C * T2;
    // rows relative to the rect: [lo, hi] clamped to [0, h - 1]
    const float ylo = py - ev - 15.0f - 16.0f * (float)sy0, yhi = py + ev - 16.0f * (float)sy0;
    const float hmax = (float)(h - 1);
    // boundary k: dx = 16 (x0 + k) - 0.5 - px clamped to the ellipse, its dy extent [dn, up]
    float b = 16.0f * (float)x0 - 0.5f - px;
    float u0 = fminf(fmaxf(b, -umax), umax);
    float h0 = __builtin_amdgcn_sqrtf(fmaxf(0.0f, cT2 - det * u0 * u0));
    float up0 = (-B * u0 + h0) * rc, dn0 = (-B * u0 - h0) * rc;
    word = 0;
    uint32_t pairs = 0;
#pragma unroll
    for (uint32_t c = 0; c < kSpanCols; ++c) {
        if (c >= w) break;
        const float b1 = b + 16.0f;
        const float u1 = fminf(fmaxf(b1, -umax), umax);
        const float h1 = __builtin_amdgcn_sqrtf(fmaxf(0.0f, cT2 - det * u1 * u1));
        const float up1 = (-B * u1 + h1) * rc, dn1 = (-B * u1 - h1) * rc;
        if (b <= umax && b1 >= -umax) {
            const float vhi = (ut >= u0 && ut <= u1) ? vmax : fmaxf(up0, up1);
            const float vlo = (-ut >= u0 && -ut <= u1) ? -vmax : fminf(dn0, dn1);
            const float lo = fmaxf(ceilf((ylo + vlo) * 0.0625f), 0.0f);
            const float hi = fminf(floorf((yhi + vhi) * 0.0625f), hmax);
            if (lo <= hi) {
                const uint32_t l = (uint32_t)lo, n = (uint32_t)(hi - lo) + 1u;
                word |= (uint64_t)(l | (n << 4)) << (8 * c);
                pairs += n;
            }
        }
        b = b1, u0 = u1, up0 = up1, dn0 = dn1;
    }
    cols = make_uint2((uint32_t)word, (uint32_t)(word >> 32));
    return pairs;
}

// Strip ranks without radii (strip_skip): may the Gaussian at view-space t with 3D covariance
// c[6] and pixel row py have a tile in the strip?  False only when provably not: from an upper
// bound of upstream's radius ceil(3 sqrt(lambda_max)) -- lambda_max of the 2D covariance
// J W Sigma W^T J^T + 0.3 I is at most ||Sigma||_F ||W||_F^2 ||J||_F^2 + 0.3 sqrt(2), upstream's
// eigenvalue formula adds at most sqrt(0.1), ||J||_F^2 <= (fx^2 (1 + limx^2) + fy^2 (1 +
// limy^2)) / z^2 (the clamped J), with 1 % and 2 px of slack for float rounding -- through
// get_rect, which is monotone in the radius.  NaN / inf anywhere keeps the Gaussian.
__device__ __forceinline__ bool strip_reach(const GsrPreprocessArgs &a, float3 t, const float c[6],
                                            float py) {
    const float *vm = a.viewmatrix;
    float wf = 0.0f;
#pragma unroll
    for (int i = 0; i < 11; ++i)
        if ((i & 3) != 3) wf = __builtin_fmaf(vm[i], vm[i], wf);
    const float limx = 1.3f * a.tanfovx, limy = 1.3f * a.tanfovy;
    const float jf = (a.focal_x * a.focal_x * (1.0f + limx * limx) +
                      a.focal_y * a.focal_y * (1.0f + limy * limy)) *
                     __builtin_amdgcn_rcpf(t.z * t.z);
    const float sf2 = c[0] * c[0] + c[3] * c[3] + c[5] * c[5] +
                      2.0f * (c[1] * c[1] + c[2] * c[2] + c[4] * c[4]);
    const float lam = (__builtin_sqrtf(sf2) * wf * jf + 0.43f) * 1.01f + 0.32f;
    if (!(lam < 1e30f)) return true;
    const int r = f2i_sat(__builtin_ceilf(3.0f * __builtin_sqrtf(lam) * 1.01f + 2.0f));
    const uint32_t y0 = min(a.grid_y, (uint32_t)max(0, f2i_sat((py - r) / GSR_TILE_Y)));
    const uint32_t y1 =
        min(a.grid_y, (uint32_t)max(0, f2i_sat((py + r + GSR_TILE_Y - 1) / GSR_TILE_Y)));
    return y1 > y0 && y1 > a.row_begin && y0 < a.row_end;
}

// The first half of upstream preprocessCUDA for one Gaussian: every input loaded up front (so
// all loads are in flight together instead of a second round trip after the frustum test),
// the frustum test, the projection and the 3D covariance.
struct Front {
    float3 p_view;
    float p_proj_x, p_proj_y;
    float cov3d[6];
    float opacity;
    bool in_frustum;
};

__device__ __forceinline__ Front front_one(const GsrPreprocessArgs &a, int64_t idx) {
    Front f;
    const float3 p = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1],
                                 a.means3D[3 * idx + 2]);
    float3 s_in = make_float3(0.f, 0.f, 0.f);
    float4 q_in = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!a.cov3D_precomp) {
        s_in = make_float3(a.scales[3 * idx], a.scales[3 * idx + 1], a.scales[3 * idx + 2]);
        q_in = a.rot_vec4 ? reinterpret_cast<const float4 *>(a.rotations)[idx]
                          : make_float4(a.rotations[4 * idx], a.rotations[4 * idx + 1],
                                        a.rotations[4 * idx + 2], a.rotations[4 * idx + 3]);
    }
    f.opacity = a.opacities[idx];
    f.p_view = transform_point_4x3(p, a.viewmatrix);
    f.in_frustum = f.p_view.z > 0.2f;
    f.p_proj_x = f.p_proj_y = 0.0f;
    if (f.in_frustum) {
        const float4 p_hom = transform_point_4x4(p, a.projmatrix);
        const float p_w = 1.0f / (p_hom.w + 0.0000001f);
        f.p_proj_x = p_hom.x * p_w;
        f.p_proj_y = p_hom.y * p_w;
        if (a.cov3D_precomp) {
#pragma unroll
            for (int i = 0; i < 6; ++i) f.cov3d[i] = a.cov3D_precomp[6 * idx + i];
        } else {
            compute_cov3d(s_in, a.scale_modifier, q_in, f.cov3d);
        }
    }
    return f;
}

// The outputs of a Gaussian without a pair in the strip (strip_skip: radii and the
// per-Gaussian extras are not requested).
__device__ __forceinline__ void none_one(const GsrPreprocessArgs &a, int64_t idx) {
    a.strip_rect[idx] = make_uint2(0u, 0u);
    if (a.strip_rc) a.strip_rc[idx] = make_uint4(0u, 0u, 0u, 0u);
    a.sort_keys[idx] = 0xFFFFFFFFu;
}

// The second half: 2D covariance, conic, radius, tile rect, depth key, the blend's record (and
// with tight binning the span word).  Returns the number of (Gaussian, strip tile) pairs of
// Gaussian idx; tight_out: their number over the spans (without tight binning the same).
__device__ __forceinline__ uint32_t back_one(const GsrPreprocessArgs &a, int64_t idx,
                                             const Front &f, uint32_t &key_out,
                                             uint32_t &tight_out) {
    int32_t radius_out = 0;
    uint32_t strip_tiles_tight = 0;
    uint2 cols = make_uint2(0u, 0u);
    uint32_t strip_tiles = 0, all_tiles = 0;
    uint2 strip_rect = make_uint2(0u, 0u);
    uint32_t key = 0xFFFFFFFFu;
    if (f.in_frustum) {
        const float3 p_view = f.p_view;
        const float3 cov = compute_cov2d(p_view, a.focal_x, a.focal_y, a.tanfovx, a.tanfovy,
                                         f.cov3d, a.viewmatrix);
        const float det = cov.x * cov.z - cov.y * cov.y;
        if (det != 0.0f) {
            const float det_inv = 1.f / det;
            const float conic_a = cov.z * det_inv, conic_b = -cov.y * det_inv,
                        conic_c = cov.x * det_inv;
            const float mid = 0.5f * (cov.x + cov.z);
            const float lambda1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
            const float lambda2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
            const float my_radius = ceilf(3.f * sqrtf(fmaxf(lambda1, lambda2)));
            const float px = ndc2pix(f.p_proj_x, a.W), py = ndc2pix(f.p_proj_y, a.H);
            const int r_int = f2i_sat(my_radius);
            const Rect rc = get_rect(px, py, r_int, a.grid_x, a.grid_y);
            all_tiles = (rc.x1 - rc.x0) * (rc.y1 - rc.y0);
            if (all_tiles != 0) {
                const float opacity = f.opacity;
                radius_out = r_int;
                const uint32_t sy0 = max(rc.y0, a.row_begin), sy1 = min(rc.y1, a.row_end);
                strip_tiles = sy1 > sy0 ? (rc.x1 - rc.x0) * (sy1 - sy0) : 0u;
                if (strip_tiles)
                    strip_rect = make_uint2(rc.x0 | ((rc.x1 - rc.x0) << 16),
                                            (sy0 - a.row_begin) | ((sy1 - sy0) << 16));
                if (strip_tiles) key = __float_as_uint(p_view.z);  // z > 0.2: bits are monotone
                // the blend's record (and its double-precision cull data) only for Gaussians
                // with pairs in this strip: on a strip of a multi-GPU frame most have none
                float3 cd = make_float3(0.f, 0.f, 0.f);
                SplatRecord &rec = a.records[idx];
                if (strip_tiles) {
                    cd = cull_data(conic_a, conic_b, conic_c, opacity);
                    rec.a = make_float4(px, py, conic_a, conic_b);
                    rec.b = make_float4(conic_c, opacity, cd.x, cd.y);
                    if (a.strip_rc && span_coded(strip_rect))
                        strip_tiles_tight = col_spans(px, py, conic_a, conic_b, conic_c, cd.z,
                                                      rc.x0, rc.x1 - rc.x0, sy0, sy1 - sy0, cols);
                }
                if (strip_tiles) rec.c.x = cd.z;  // c.yzw: the colour, written by k_color
                if (a.depths) a.depths[idx] = p_view.z;
                if (a.means2D) {
                    a.means2D[2 * idx] = px;
                    a.means2D[2 * idx + 1] = py;
                }
                if (a.conic_opacity)
                    reinterpret_cast<float4 *>(a.conic_opacity)[idx] =
                        make_float4(conic_a, conic_b, conic_c, opacity);
            }
        }
    }
    if (a.radii) a.radii[idx] = radius_out;
    a.strip_rect[idx] = strip_rect;
    if (a.strip_rc) a.strip_rc[idx] = make_uint4(strip_rect.x, strip_rect.y, cols.x, cols.y);
    tight_out =
        (strip_rect.x && a.strip_rc && span_coded(strip_rect)) ? strip_tiles_tight : strip_tiles;
    a.sort_keys[idx] = key;  // the depth sort's values are the indices (implicit)
    key_out = key;
    if (a.tiles_touched) a.tiles_touched[idx] = strip_tiles;
    return strip_tiles;
}

// strip_skip: the block's Gaussians that may reach the strip, compacted (their Front in LDS,
// structure of arrays) so the second half runs on as few waves as hold them -- on a 1/8 strip
// about one wave in four -- instead of on every wave that has one such lane.
struct SkipSmem {
    float v[12][256];  // p_view xyz, p_proj xy, cov3d[6], opacity
    uint32_t idx[256];
    uint32_t wcount[4];
};

// One thread per Gaussian.  Block b also stores its share of K (the (Gaussian, strip tile)
// pair count) and the OR / AND of its kept depth keys (k_publish_K reduces them for the host:
// K sizes the binning, bits(OR ^ AND) the depth sort's passes), and with a.block_kept (the
// depth sort's compaction, strips) how many of its 256 Gaussians have pairs in the strip.
// (A separate pass re-reading the rects and keys took 7 us at C3 and 42 us on a C4 strip.)
template <bool kSkip>
__global__ __launch_bounds__(256) void k_preprocess(const GsrPreprocessArgs a) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t key = 0xFFFFFFFFu;
    uint32_t pairs = 0u, tight = 0u;
    if (!kSkip) {
        if (idx < a.P) pairs = back_one(a, idx, front_one(a, idx), key, tight);
    } else {
        __shared__ SkipSmem sk;
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        bool reach = false;
        Front f;
        if (idx < a.P) {
            f = front_one(a, idx);
            reach = f.in_frustum &&
                    strip_reach(a, f.p_view, f.cov3d, ndc2pix(f.p_proj_y, a.H));
            if (!reach) none_one(a, idx);
        }
        const uint64_t bal = __ballot(reach);
        if (lane == 0) sk.wcount[w] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t base = 0, n = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            base += i < w ? sk.wcount[i] : 0u;
            n += sk.wcount[i];
        }
        if (reach) {
            const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            const uint32_t slot = base + (uint32_t)__popcll(bal & lt);
            sk.v[0][slot] = f.p_view.x;
            sk.v[1][slot] = f.p_view.y;
            sk.v[2][slot] = f.p_view.z;
            sk.v[3][slot] = f.p_proj_x;
            sk.v[4][slot] = f.p_proj_y;
#pragma unroll
            for (int i = 0; i < 6; ++i) sk.v[5 + i][slot] = f.cov3d[i];
            sk.v[11][slot] = f.opacity;
            sk.idx[slot] = (uint32_t)idx;
        }
        __syncthreads();
        if (threadIdx.x < n) {
            const uint32_t t = threadIdx.x;
            Front g;
            g.p_view = make_float3(sk.v[0][t], sk.v[1][t], sk.v[2][t]);
            g.p_proj_x = sk.v[3][t];
            g.p_proj_y = sk.v[4][t];
#pragma unroll
            for (int i = 0; i < 6; ++i) g.cov3d[i] = sk.v[5 + i][t];
            g.opacity = sk.v[11][t];
            g.in_frustum = true;
            pairs = back_one(a, (int64_t)sk.idx[t], g, key, tight);
        }
    }
    const bool kept = pairs != 0u;  // has pairs in the strip <=> its depth key is kept
    // the block's pair count (v <= 256 x 2^16) and the largest / smallest kept depth key
    uint32_t v = pairs, mx = kept ? key : 0u, mn = kept ? key : 0xFFFFFFFFu;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        v += __shfl_xor(v, off);
        tight += __shfl_xor(tight, off);
        mx = max(mx, (uint32_t)__shfl_xor(mx, off));
        mn = min(mn, (uint32_t)__shfl_xor(mn, off));
    }
    __shared__ uint32_t s_red[5][4];
    const uint32_t c = a.block_kept ? (uint32_t)__popcll(__ballot(kept)) : 0u;
    if ((threadIdx.x & 63) == 0) {
        const int w = threadIdx.x >> 6;
        s_red[0][w] = v, s_red[1][w] = mx, s_red[2][w] = mn, s_red[3][w] = c, s_red[4][w] = tight;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (a.frame_words && blockIdx.x == 0) {  // (frame graphs) this frame's tag and camera
            a.frame_words[0] = a.k_tag;
            if (a.campos) {
                a.frame_words[4] = __float_as_uint(a.campos[0]);
                a.frame_words[5] = __float_as_uint(a.campos[1]);
                a.frame_words[6] = __float_as_uint(a.campos[2]);
            }
        }
        a.block_pairs[blockIdx.x] =
            ((uint64_t)(s_red[4][0] + s_red[4][1] + s_red[4][2] + s_red[4][3]) << 32) |
            (s_red[0][0] + s_red[0][1] + s_red[0][2] + s_red[0][3]);
        reinterpret_cast<uint2 *>(a.block_pairs + gridDim.x)[blockIdx.x] =
            make_uint2(max(max(s_red[1][0], s_red[1][1]), max(s_red[1][2], s_red[1][3])),
                       min(min(s_red[2][0], s_red[2][1]), min(s_red[2][2], s_red[2][3])));
        if (a.block_kept) a.block_kept[blockIdx.x] = s_red[3][0] + s_red[3][1] + s_red[3][2] + s_red[3][3];
    }
}

// One block, on the second stream after the preprocess (the kernel boundary makes its stores
// visible): K = sum of the per-block pair counts and D = the bits in which the kept depth keys
// differ (bits of OR ^ AND: the depth sort's pass count), stored straight into pinned host
// memory (system scope) so the host can read them as soon as this kernel's completion event
// fires -- no copy, and nothing added to the main stream.  host_K[0] = K, host_K[1] = D,
// host_K[3] = the pair count over the spans (the high halves of the block counts).
constexpr int kPubThreads = 1024, kPubWaves = kPubThreads / 64;
__global__ __launch_bounds__(kPubThreads) void k_publish_K(const unsigned long long *__restrict__ cnt,
                                                           const uint2 *__restrict__ keybits,
                                                           int64_t n, unsigned long long *host_K,
                                                           uint32_t k_tag, uint32_t *ds_ctl,
                                                           const uint32_t *d_tag) {
    __shared__ unsigned long long s_w[kPubWaves], s_wt[kPubWaves];
    __shared__ uint32_t s_max[kPubWaves], s_min[kPubWaves];
    unsigned long long v = 0, vt = 0;
    uint32_t mx = 0u, mn = 0xFFFFFFFFu;  // the largest / smallest kept depth key
    // 8 blocks' entries per thread and round, their loads in flight together (one dependent
    // load per 1024 blocks took 23 us at 6M Gaussians)
    constexpr int kU = 8;
    for (int64_t i0 = threadIdx.x; i0 < n; i0 += kU * kPubThreads) {
        unsigned long long c[kU];
        uint2 kb[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t i = i0 + (int64_t)u * kPubThreads;
            c[u] = i < n ? cnt[i] : 0ull;
            kb[u] = i < n ? keybits[i] : make_uint2(0u, 0xFFFFFFFFu);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            v += c[u] & 0xFFFFFFFFull;
            vt += c[u] >> 32;
            mx = max(mx, kb[u].x);
            mn = min(mn, kb[u].y);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        v += __shfl_xor(v, off);
        vt += __shfl_xor(vt, off);
        mx = max(mx, (uint32_t)__shfl_xor(mx, off));
        mn = min(mn, (uint32_t)__shfl_xor(mn, off));
    }
    if ((threadIdx.x & 63) == 0) {
        s_w[threadIdx.x >> 6] = v;
        s_wt[threadIdx.x >> 6] = vt;
        s_max[threadIdx.x >> 6] = mx;
        s_min[threadIdx.x >> 6] = mn;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0, tt = 0;
        mx = 0u;
        mn = 0xFFFFFFFFu;
        for (int i = 0; i < kPubWaves; ++i) {
            t += s_w[i];
            tt += s_wt[i];
            mx = max(mx, s_max[i]);
            mn = min(mn, s_min[i]);
        }
        // D: the key bits that vary (the highest bit where the smallest and the largest kept key
        // differ is the highest bit any two kept keys differ in); Dr: the bits of their range
        const KeyBits kb = key_bits(mx, mn);
        if (ds_ctl) gsr_msd_ctl(kb, ds_ctl);  // the MSD depth sort's control words
        __hip_atomic_store(host_K + 1, (unsigned long long)kb.D, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_K + 4, (unsigned long long)kb.Dr, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_K + 3, tt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(host_K, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        // the host spins on this tag instead of sleeping in an event wait (release: K and D are
        // visible first)
        if (d_tag) k_tag = *d_tag;
        if (k_tag)
            __hip_atomic_store(host_K + 5, (unsigned long long)k_tag, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Colour of the Gaussians k_preprocess kept (radii > 0, as upstream computes colour only for
// those): upstream computeColorFromSH, or colors_precomp copied.
__device__ __forceinline__ void color_one(const GsrPreprocessArgs &a, int64_t idx) {
    if (a.rgb ? a.radii[idx] == 0 : a.strip_rect[idx].x == 0u) return;
    float3 col;
    if (a.colors_precomp) {
        col = make_float3(a.colors_precomp[3 * idx], a.colors_precomp[3 * idx + 1],
                          a.colors_precomp[3 * idx + 2]);
    } else {
        const float3 p = make_float3(a.means3D[3 * idx], a.means3D[3 * idx + 1],
                                     a.means3D[3 * idx + 2]);
        col = color_from_sh(p, a.campos, a.shs + idx * (int64_t)a.M * 3, a.D, a.sh_vec4);
        if (a.rgb) {
            a.rgb[3 * idx] = col.x;
            a.rgb[3 * idx + 1] = col.y;
            a.rgb[3 * idx + 2] = col.z;
        }
    }
    float *c = &a.records[idx].c.x;
    c[1] = col.x;
    c[2] = col.y;
    c[3] = col.z;
}

// The general case (colors_precomp, unaligned rows, degree < 3): one thread per Gaussian.
__global__ __launch_bounds__(256) void k_color_generic(const GsrPreprocessArgs a) {
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx < a.P) color_one(a, idx);
}

// Writes one colour (and the rgb output) of Gaussian idx.
__device__ __forceinline__ void store_color(const GsrPreprocessArgs &a, int64_t idx, float3 col) {
    if (a.rgb) {
        a.rgb[3 * idx] = col.x;
        a.rgb[3 * idx + 1] = col.y;
        a.rgb[3 * idx + 2] = col.z;
    }
    float *cc = &a.records[idx].c.x;
    cc[1] = col.x;
    cc[2] = col.y;
    cc[3] = col.z;
}

// Degree 3 with 16-B aligned rows (the host launches k_color_generic otherwise).  Four lanes
// per Gaussian, 16 Gaussians per wave and round: lane (q, j) of quad q loads pieces j, j + 4 and
// j + 8 (16 B each) of its Gaussian's 192-B row, so each of the wave's three load instructions
// reads 16 whole 64-B lines and no line is read by two instructions (one lane per row read its
// 12 pieces with 12 instructions, every instruction touching 64 lines, and the lines were
// refetched from L2 as other waves evicted them).  The quad stages the row in the wave's LDS
// slice (49-dword rows: conflict-free), then lanes j = 0, 1, 2 evaluate channel j alone, in
// upstream's order for that channel (eval_sh3_stream's per-channel chain: identical colours).
constexpr int kRowStride = 49;                           // dwords per staged row
constexpr size_t kColorLds = 4 * 16 * kRowStride * 4;    // 4 waves x 16 rows
__device__ __forceinline__ void color_quad(const GsrPreprocessArgs &a, int64_t idx, bool need,
                                           float *rows, int lane) {
    const int q = lane >> 2, j = lane & 3;
    float *row = rows + q * kRowStride;
    if (need) {
        const float4 *src = reinterpret_cast<const float4 *>(a.shs) + idx * 12;
        const float4 v0 = src[j], v1 = src[j + 4], v2 = src[j + 8];
        float *d = row + 4 * j;
        d[0] = v0.x, d[1] = v0.y, d[2] = v0.z, d[3] = v0.w;
        d[16] = v1.x, d[17] = v1.y, d[18] = v1.z, d[19] = v1.w;
        d[32] = v2.x, d[33] = v2.y, d[34] = v2.z, d[35] = v2.w;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (need && j < 3) {
        float dx = a.means3D[3 * idx] - a.campos[0], dy = a.means3D[3 * idx + 1] - a.campos[1],
              dz = a.means3D[3 * idx + 2] - a.campos[2];
        const float len = sqrtf(dx * dx + dy * dy + dz * dz);
        dx = dx / len;
        dy = dy / len;
        dz = dz / len;
        const float x = dx, y = dy, z = dz;
        const float xx = x * x, yy = y * y, zz = z * z;
        const float xy = x * y, yz = y * z, xz = x * z;
        const float bs[16] = {kShC0,
                              kShC1 * y,
                              kShC1 * z,
                              kShC1 * x,
                              kShC2[0] * xy,
                              kShC2[1] * yz,
                              kShC2[2] * (2.0f * zz - xx - yy),
                              kShC2[3] * xz,
                              kShC2[4] * (xx - yy),
                              kShC3[0] * y * (3.0f * xx - yy),
                              kShC3[1] * xy * z,
                              kShC3[2] * y * (4.0f * zz - xx - yy),
                              kShC3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy),
                              kShC3[4] * x * (4.0f * zz - xx - yy),
                              kShC3[5] * z * (xx - yy),
                              kShC3[6] * x * (xx - 3.0f * yy)};
        float r = bs[0] * row[j];
#pragma unroll
        for (int k = 1; k < 16; ++k) {
            const float v = row[3 * k + j];
            r = (k == 1 || k == 3) ? r - bs[k] * v : r + bs[k] * v;
        }
        const float col = fmaxf(r + 0.5f, 0.0f);
        if (a.rgb) a.rgb[3 * idx + j] = col;
        (&a.records[idx].c.x)[1 + j] = col;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // (the rows are refilled next)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The launch caps how many colour waves a CU holds (gsr_launch_color's waves_per_simd, through
// the block's LDS allocation), leaving the CUs to the binning chain beside it.
__global__ __launch_bounds__(256) void k_color(const GsrPreprocessArgs a) {
    extern __shared__ float s_rows[];  // [4 waves][16][kRowStride] (+ the occupancy reservation)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float *rows = s_rows + w * 16 * kRowStride;
    const int64_t n_groups = (a.P + 15) / 16;
    const int64_t stride = (int64_t)gridDim.x * 4;
    for (int64_t gi = (int64_t)blockIdx.x * 4 + w; gi < n_groups; gi += stride) {
        const int64_t idx = gi * 16 + (lane >> 2);
        // colour needed: Gaussians with pairs in this strip (the blend reads them), or every
        // visible one when the caller asked for the rgb output (upstream semantics)
        const bool need = idx < a.P && (a.rgb ? a.radii[idx] != 0 : a.strip_rect[idx].x != 0u);
        color_quad(a, idx, need, rows, lane);
    }
}

// The colour pass of a compacted strip frame: the kept Gaussians of ids[0 .. *d_n)
// (k_ds_compact's list), 16 per wave and round, so no lane waits on a Gaussian without a row to
// read and the P-long rect scan is gone.  Same quads and occupancy cap as k_color.
__global__ __launch_bounds__(256) void k_color_ids(const GsrPreprocessArgs a,
                                                   const uint32_t *__restrict__ ids,
                                                   const uint32_t *__restrict__ d_n) {
    extern __shared__ float s_rows[];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float *rows = s_rows + w * 16 * kRowStride;
    const int64_t n = *d_n;
    const int64_t n_groups = (n + 15) / 16;
    const int64_t stride = (int64_t)gridDim.x * 4;
    for (int64_t gi = (int64_t)blockIdx.x * 4 + w; gi < n_groups; gi += stride) {
        const int64_t i = gi * 16 + (lane >> 2);
        const bool need = i < n;
        color_quad(a, need ? (int64_t)ids[i] : 0, need, rows, lane);
    }
}

// GaussianRasterizer.markVisible -> upstream markVisible kernel: in_frustum only.
__global__ __launch_bounds__(256) void k_mark_visible(const float *__restrict__ means3D,
                                                      int64_t P, const float *viewmatrix,
                                                      uint8_t *visible) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const float3 p = make_float3(means3D[3 * idx], means3D[3 * idx + 1], means3D[3 * idx + 2]);
    visible[idx] = transform_point_4x3(p, viewmatrix).z > 0.2f ? 1 : 0;
}

// Depth-sort backend (renderer_ogl.py:10-19): view-space z of each point in the operation
// order the reference's numpy stacked matmul produced in the build container
// (fma(v22, z, fma(v20, x, v21*y)) + v23), then an order-preserving
// uint32 key so the stable radix sort returns np.argsort(depth, kind='stable').
__global__ __launch_bounds__(256) void k_view_depth_keys(const float *__restrict__ xyz, int64_t P,
                                                         float v20, float v21, float v22, float v23,
                                                         uint32_t *keys, float *depth_out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= P) return;
    const float x = xyz[3 * idx], y = xyz[3 * idx + 1], z = xyz[3 * idx + 2];
    const float d = __builtin_fmaf(v22, z, __builtin_fmaf(v20, x, v21 * y)) + v23;
    keys[idx] = float_sort_key(d);
    if (depth_out) depth_out[idx] = d;
}

inline unsigned grid_for(int64_t n) { return (unsigned)gsr_preprocess_blocks(n); }

}  // namespace

hipError_t gsr_launch_preprocess(const GsrPreprocessArgs &a, hipStream_t s) {
    if (a.P == 0) return hipSuccess;
    if (a.strip_skip)
        hipLaunchKernelGGL(k_preprocess<true>, dim3(grid_for(a.P)), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_preprocess<false>, dim3(grid_for(a.P)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t gsr_launch_color(const GsrPreprocessArgs &a, int waves_per_simd, hipStream_t s) {
    if (a.P == 0) return hipSuccess;
    const unsigned g0 = grid_for(a.P);  // 4 waves of 64 Gaussians per block
    if (!a.sh_vec4 || a.colors_precomp || a.D != 3) {
        hipLaunchKernelGGL(k_color_generic, dim3(g0), dim3(256), 0, s, a);
        return hipGetLastError();
    }
    // a 4-wave block puts one wave on each SIMD: w blocks per CU = w waves per SIMD, held by
    // reserving 1/w of the CU's 160 KiB of LDS per block (1 KiB granules; the kernel's dynamic
    // LDS limit is raised once per device, gsr_color_setup)
    (void)waves_per_simd;  // lab: uncapped (whole lines per load: no L1 thrash to cap)
    const size_t lds = kColorLds;
    hipLaunchKernelGGL(k_color, dim3(g0), dim3(256), lds, s, a);
    return hipGetLastError();
}

// Raises k_color's dynamic LDS limit to the largest reservation gsr_launch_color asks for (one
// wave per SIMD: all 160 KiB), once per device from gsr_create -- outside any stream capture, so
// a recorded frame graph never holds a hipFuncSetAttribute.
hipError_t gsr_color_setup() {
    return hipFuncSetAttribute(reinterpret_cast<const void *>(&k_color),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

bool gsr_color_ids_ok(const GsrPreprocessArgs &a) {
    return a.sh_vec4 && !a.colors_precomp && a.D == 3 && !a.rgb;
}

hipError_t gsr_launch_color_ids(const GsrPreprocessArgs &a, const uint32_t *ids,
                                const uint32_t *d_n, int waves_per_simd, hipStream_t s) {
    if (a.P == 0) return hipSuccess;
    if (!gsr_color_ids_ok(a)) return hipErrorInvalidValue;
    size_t lds = 0;
    if (waves_per_simd >= 3 && waves_per_simd < 8)
        lds = (size_t)(160 * 1024 / waves_per_simd) & ~(size_t)1023;
    if (lds < kColorLds) lds = kColorLds;  // (the staged rows)
    hipLaunchKernelGGL(k_color_ids, dim3(grid_for(a.P)), dim3(256), lds, s, a, ids, d_n);
    return hipGetLastError();
}

hipError_t gsr_launch_count_pairs(const GsrPreprocessArgs &a, hipStream_t s, uint32_t *ds_ctl,
                                  const uint32_t *d_tag) {
    if (a.P == 0) return hipSuccess;
    const unsigned g = grid_for(a.P);  // the preprocess's blocks
    const uint2 *keybits = reinterpret_cast<const uint2 *>(a.block_pairs + g);
    hipLaunchKernelGGL(k_publish_K, dim3(1), dim3(kPubThreads), 0, s,
                       reinterpret_cast<const unsigned long long *>(a.block_pairs), keybits,
                       (int64_t)g, a.host_K, d_tag ? 0u : a.k_tag, ds_ctl, d_tag);
    return hipGetLastError();
}

hipError_t gsr_launch_mark_visible(const float *means3D, int64_t P, const float *viewmatrix,
                                   uint8_t *visible, hipStream_t s) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mark_visible, dim3(grid_for(P)), dim3(256), 0, s, means3D, P, viewmatrix,
                       visible);
    return hipGetLastError();
}

hipError_t gsr_launch_view_depth_keys(const float *xyz, int64_t P, float v20, float v21, float v22,
                                      float v23, uint32_t *keys, float *depth_out, hipStream_t s) {
    if (P == 0) return hipSuccess;
    hipLaunchKernelGGL(k_view_depth_keys, dim3(grid_for(P)), dim3(256), 0, s, xyz, P, v20, v21,
                       v22, v23, keys, depth_out);
    return hipGetLastError();
}
