// blend.hip -- per-tile front-to-back alpha compositing for gfx950.
//
// Replaces upstream diff-gaussian-rasterization forward.cu renderCUDA (GLSL twin of the
// per-pixel alpha: shaders/gau_frag.glsl:21-27).  One 256-thread block per 16x16 tile; each
// of its 4 waves owns an 8x8 quadrant (one pixel per lane).  The tile's depth-sorted splat
// list is staged through LDS 256 records (12 KB) at a time; `__syncthreads_count(done)`
// ends the tile when every pixel has saturated (as upstream).  Per splat each wave first
// tests the splat's conservative alpha>=1/255 box against its quadrant and skips the splat
// as a whole (wave-uniform branch) when they do not overlap; otherwise every lane runs the
// upstream per-pixel arithmetic verbatim (same operation order, accurate expf).
//
// n_contrib equals upstream's running `contributor` counter at the last contributing splat
// = (position of that splat in the tile list) + 1, so skipping non-contributing splats does
// not change it.
#include "gsr_internal.h"

using namespace gsr;

namespace {

constexpr int kBatch = 256;

__global__ __launch_bounds__(256) void k_blend(const GsrBlendArgs a) {
    __shared__ float4 s_a[kBatch];
    __shared__ float4 s_b[kBatch];
    __shared__ float4 s_c[kBatch];

    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t tx = blockIdx.x, ty_local = blockIdx.y, ty = a.row_begin + ty_local;
    const int qx0 = (int)tx * GSR_TILE_X + (w & 1) * 8;
    const int qy0 = (int)ty * GSR_TILE_Y + (w >> 1) * 8;
    const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    bool done = !inside;
    const float pfx = (float)px, pfy = (float)py;
    // quadrant bounds (pixel centres are the integer coordinates, upstream has no +0.5)
    const float qxlo = (float)qx0, qxhi = (float)(qx0 + 7);
    const float qylo = (float)qy0, qyhi = (float)(qy0 + 7);

    const uint2 range = a.ranges[ty_local * a.grid_x + tx];
    float T = 1.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
    uint32_t last_contributor = 0;

    for (uint32_t start = range.x; start < range.y; start += kBatch) {
        if (__syncthreads_count(done) == 256) break;
        const uint32_t idx = start + tid;
        if (idx < range.y) {
            const SplatRecord *r = a.records + a.point_list[idx];
            s_a[tid] = r->a;
            s_b[tid] = r->b;
            s_c[tid] = r->c;
        }
        __syncthreads();
        const int n = (int)min((uint32_t)kBatch, range.y - start);
        if (__ballot(!done) != 0ull) {
            for (int j = 0; j < n; ++j) {
                const float4 sa = s_a[j];
                if (a.cull) {
                    const float4 sc = s_c[j];
                    // distance from the splat centre to the quadrant along x and y
                    const float ddx = fmaxf(fmaxf(qxlo - sa.x, sa.x - qxhi), 0.0f);
                    const float ddy = fmaxf(fmaxf(qylo - sa.y, sa.y - qyhi), 0.0f);
                    const bool miss = (ddx > sc.y) || (ddy > sc.z);
                    if (__builtin_amdgcn_readfirstlane((int)miss)) continue;
                }
                if (!done) {
                    const float4 sb = s_b[j];
                    const float dx = sa.x - pfx, dy = sa.y - pfy;
                    const float power =
                        -0.5f * (sa.z * dx * dx + sb.x * dy * dy) - sa.w * dx * dy;
                    if (!(power > 0.0f)) {  // upstream: if (power > 0) continue;
                        const float alpha = fminf(0.99f, sb.y * expf(power));
                        if (!(alpha < 1.0f / 255.0f)) {
                            const float test_T = T * (1 - alpha);
                            if (test_T < 0.0001f) {
                                done = true;
                            } else {
                                const float cz = s_c[j].x;
                                C0 += sb.z * alpha * T;
                                C1 += sb.w * alpha * T;
                                C2 += cz * alpha * T;
                                T = test_T;
                                last_contributor = start - range.x + (uint32_t)j + 1u;
                            }
                        }
                    }
                }
                if (__ballot(!done) == 0ull) break;
            }
        }
    }

    if (inside) {
        const int row = py - a.y0;
        const size_t pid = (size_t)row * a.W + px;
        const size_t plane = (size_t)a.rows_out * a.W;
        if (a.final_T) a.final_T[pid] = T;
        if (a.n_contrib) a.n_contrib[pid] = last_contributor;
        a.out_color[pid] = C0 + T * a.bg[0];
        a.out_color[plane + pid] = C1 + T * a.bg[1];
        a.out_color[2 * plane + pid] = C2 + T * a.bg[2];
    }
}

}  // namespace

hipError_t gsr_launch_blend(const GsrBlendArgs &a, hipStream_t s) {
    if (a.rows_tiles == 0 || a.grid_x == 0) return hipSuccess;
    hipLaunchKernelGGL(k_blend, dim3(a.grid_x, a.rows_tiles), dim3(256), 0, s, a);
    return hipGetLastError();
}
