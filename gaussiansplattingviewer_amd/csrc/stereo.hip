// stereo.hip -- the stereo dataset outputs of the viewer on the device (SURVEY.md §8(f) rows 3
// and 4): the disparity colour of every Gaussian (render mode -1, gau_vert.glsl:182-210) and
// the frame packers that turn the rasterizer's (3,H,W) float image into what the viewer hands
// on -- HWC RGBA float for display (renderer_cuda.py:226-228), RGB8 and uint16 disparity rows as
// the capture path saves them (main.py:858-917).  Both are streaming kernels (HBM-bound).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "gsr.h"

#pragma clang fp contract(off)

int gsr_set_error(int code, const std::string &msg);  // api.hip

namespace {

struct DisparityCam {
    float v[16];  // view, math layout row-major (what the viewer's view_matrix uniform holds)
    float p[16];  // projection, math layout row-major
    float baseline;
};

__device__ __forceinline__ float ndc_x(const DisparityCam &c, float x, float y, float z) {
    // p_view = V [x y z 1]; p_screen = P p_view; ndc.x = p_screen.x / p_screen.w
    float pv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        pv[i] = c.v[4 * i] * x + c.v[4 * i + 1] * y + c.v[4 * i + 2] * z + c.v[4 * i + 3];
    const float sx = c.p[0] * pv[0] + c.p[1] * pv[1] + c.p[2] * pv[2] + c.p[3] * pv[3];
    const float sw = c.p[12] * pv[0] + c.p[13] * pv[1] + c.p[14] * pv[2] + c.p[15] * pv[3];
    return sx / sw;
}

// gau_vert.glsl:182-207: d = |(ndc_x(p) + 1)/2 - (ndc_x(p + (baseline,0,0)) + 1)/2|, written as
// the grey colour (d, d, d) the disparity pass composites.
__device__ __forceinline__ float disparity_of(const DisparityCam &cam, float x, float y, float z) {
    const float xl = (ndc_x(cam, x, y, z) + 1.0f) / 2.0f;
    const float xr = (ndc_x(cam, x + cam.baseline, y + 0.0f, z + 0.0f) + 1.0f) / 2.0f;
    return fabsf(xl - xr);
}

// One thread per Gaussian.  (A 4-Gaussians-per-thread float4 variant measured slower on
// MI355X -- 7.3 vs 6.4 us at 1M -- the kernel is launch / ramp bound at this size.)
__global__ void __launch_bounds__(256) k_disparity_color(const float *__restrict__ xyz, int64_t P,
                                                         DisparityCam cam,
                                                         float *__restrict__ colors) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float d = disparity_of(cam, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
    colors[3 * i] = d;
    colors[3 * i + 1] = d;
    colors[3 * i + 2] = d;
}

__device__ __forceinline__ uint32_t unorm8(float v) {
    // GL float -> normalized fixed point: round(clamp(v, 0, 1) * 255); NaN -> 0.
    return (uint32_t)__float2uint_rn(fminf(fmaxf(v, 0.0f), 1.0f) * 255.0f);
}

__device__ __forceinline__ uint32_t u16_wrap(float v) {
    // numpy float32 -> uint16 astype on x86 (main.py:874): truncate toward zero through a
    // 32-bit integer, keep the low 16 bits.
    if (!(v == v) || v >= 2147483648.0f || v < -2147483648.0f) return 0u;
    return (uint32_t)(int32_t)v & 0xFFFFu;
}

// One thread = 4 consecutive pixels of one row (vector path, W % 4 == 0: a group never
// crosses a row) or 1 pixel (generic path); a 1-D grid over the groups of the whole image.
// Output row r comes from input row flip ? H-1-r : r.
template <int kFormat, bool kVec>
__global__ void __launch_bounds__(256) k_pack(const float *__restrict__ chw, int H, int W,
                                              int flip, void *__restrict__ out) {
    constexpr int kPx = kVec ? 4 : 1;
    const int64_t px = (int64_t)kPx * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
    const int64_t plane = (int64_t)H * W;
    if (px >= plane) return;
    const int r = (int)(px / W), x = (int)(px - (int64_t)r * W);
    const int src_r = flip ? H - 1 - r : r;
    const float *c0 = chw + (int64_t)src_r * W;
    const float *c1 = c0 + plane, *c2 = c1 + plane;
    const int64_t o = px;  // output pixel index (row r, column x)
    if (kVec) {
        const float4 R = *(const float4 *)(c0 + x);
        if (kFormat == GSR_PACK_R16) {
            uint2 v;
            v.x = u16_wrap(R.x * 65535.0f) | (u16_wrap(R.y * 65535.0f) << 16);
            v.y = u16_wrap(R.z * 65535.0f) | (u16_wrap(R.w * 65535.0f) << 16);
            *(uint2 *)((uint16_t *)out + o) = v;
            return;
        }
        const float4 G = *(const float4 *)(c1 + x);
        const float4 B = *(const float4 *)(c2 + x);
        if (kFormat == GSR_PACK_RGB8) {
            uint3 v;  // bytes r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
            v.x = unorm8(R.x) | (unorm8(G.x) << 8) | (unorm8(B.x) << 16) | (unorm8(R.y) << 24);
            v.y = unorm8(G.y) | (unorm8(B.y) << 8) | (unorm8(R.z) << 16) | (unorm8(G.z) << 24);
            v.z = unorm8(B.z) | (unorm8(R.w) << 8) | (unorm8(G.w) << 16) | (unorm8(B.w) << 24);
            uint32_t *dst = (uint32_t *)((uint8_t *)out + 3 * o);
            dst[0] = v.x;
            dst[1] = v.y;
            dst[2] = v.z;
        } else {  // GSR_PACK_RGBA_F32
            float4 *dst = (float4 *)out + o;
            dst[0] = make_float4(R.x, G.x, B.x, 1.0f);
            dst[1] = make_float4(R.y, G.y, B.y, 1.0f);
            dst[2] = make_float4(R.z, G.z, B.z, 1.0f);
            dst[3] = make_float4(R.w, G.w, B.w, 1.0f);
        }
    } else {
        if (kFormat == GSR_PACK_R16) {
            ((uint16_t *)out)[o] = (uint16_t)u16_wrap(c0[x] * 65535.0f);
        } else if (kFormat == GSR_PACK_RGB8) {
            uint8_t *dst = (uint8_t *)out + 3 * o;
            dst[0] = (uint8_t)unorm8(c0[x]);
            dst[1] = (uint8_t)unorm8(c1[x]);
            dst[2] = (uint8_t)unorm8(c2[x]);
        } else {
            ((float4 *)out)[o] = make_float4(c0[x], c1[x], c2[x], 1.0f);
        }
    }
}

template <int kFormat>
hipError_t launch_pack(const float *chw, int H, int W, int flip, void *out, hipStream_t s) {
    const bool vec = (W % 4 == 0) && ((uintptr_t)chw % 16 == 0) &&
                     ((uintptr_t)out % (kFormat == GSR_PACK_RGBA_F32 ? 16 : 8) == 0);
    const int64_t groups = vec ? (int64_t)H * W / 4 : (int64_t)H * W;
    const int64_t blocks = (groups + 255) / 256;
    if (blocks > INT32_MAX) return hipErrorInvalidValue;
    if (vec)
        hipLaunchKernelGGL((k_pack<kFormat, true>), dim3((uint32_t)blocks), dim3(256), 0, s, chw,
                           H, W, flip, out);
    else
        hipLaunchKernelGGL((k_pack<kFormat, false>), dim3((uint32_t)blocks), dim3(256), 0, s, chw,
                           H, W, flip, out);
    return hipGetLastError();
}

}  // namespace

extern "C" {

int gsr_disparity_colors(const float *means3D, int64_t P, const float *view_host16,
                         const float *proj_host16, float baseline, float *colors, void *stream) {
    if (P < 0 || !view_host16 || !proj_host16 || (P > 0 && (!means3D || !colors)))
        return gsr_set_error(GSR_E_INVALID, "gsr_disparity_colors: bad arguments");
    if (P == 0) return GSR_OK;
    DisparityCam cam;
    for (int i = 0; i < 16; ++i) {
        cam.v[i] = view_host16[i];
        cam.p[i] = proj_host16[i];
    }
    cam.baseline = baseline;
    const int64_t blocks = (P + 255) / 256;
    if (blocks > INT32_MAX) return gsr_set_error(GSR_E_INVALID, "gsr_disparity_colors: P too large");
    hipLaunchKernelGGL(k_disparity_color, dim3((uint32_t)blocks), dim3(256), 0,
                       static_cast<hipStream_t>(stream), means3D, P, cam, colors);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return gsr_set_error(GSR_E_HIP, std::string("disparity launch: ") + hipGetErrorString(e));
    return GSR_OK;
}

int gsr_pack_image(const float *chw, int32_t H, int32_t W, int32_t format, int32_t flip_rows,
                   void *out, void *stream) {
    if (H < 0 || W < 0 || (H > 0 && W > 0 && (!chw || !out)))
        return gsr_set_error(GSR_E_INVALID, "gsr_pack_image: bad arguments");
    if (H == 0 || W == 0) return GSR_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e;
    switch (format) {
    case GSR_PACK_RGBA_F32: e = launch_pack<GSR_PACK_RGBA_F32>(chw, H, W, flip_rows, out, s); break;
    case GSR_PACK_RGB8: e = launch_pack<GSR_PACK_RGB8>(chw, H, W, flip_rows, out, s); break;
    case GSR_PACK_R16: e = launch_pack<GSR_PACK_R16>(chw, H, W, flip_rows, out, s); break;
    default: return gsr_set_error(GSR_E_INVALID, "gsr_pack_image: unknown format");
    }
    if (e != hipSuccess)
        return gsr_set_error(GSR_E_HIP, std::string("pack launch: ") + hipGetErrorString(e));
    return GSR_OK;
}

}  // extern "C"
