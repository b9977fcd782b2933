// blend.hip -- per-tile front-to-back alpha compositing for gfx950.
//
// Replaces upstream diff-gaussian-rasterization forward.cu renderCUDA (GLSL twin of the
// per-pixel alpha: shaders/gau_frag.glsl:21-27).  k_blend_q: one wave per (16x16 tile, 8x8
// quadrant), one pixel per lane, a tile's four quadrant waves in one 256-thread block that never
// synchronises (each wave is independent; one block per tile instead of one per quadrant:
// blend -2 %, C3 +2 % in flight, profiles/r06p_ab_blend_tile_blocks.txt).  Each wave streams its
// tile's depth-sorted list 64 splats at a time, culls them against its own quadrant (the
// splat's conservative alpha >= 1/255 ellipse from preprocess.hip cull_data: bounding box,
// then the exact ellipse-vs-box minimum with a rounding bound), compacts the survivors into
// LDS with a ballot, composites them two at a time, and stops as soon as its 64 pixels are
// done.  At C3 a quadrant wave examines ~4.4 chunks (~280 list entries) and composites ~118
// splats (a per-wave timeline, tools/lab/blend_trace.py); by the ISA and SQ_INSTS_VALU about two
// thirds of its VALU is the compositing loop (33 VALU + 5 LDS reads per composited pair) and one
// third the per-chunk gather, cull and staging.
//
// Skipping splats that provably cannot reach alpha >= 1/255 changes nothing: upstream skips
// them too (`if (alpha < 1/255) continue`), and n_contrib -- upstream's running `contributor`
// at the last contributing splat -- is that splat's list position + 1 either way.
// Arithmetic (GSR_OPT_BLEND_FAST): 1 (default) stages each splat as the exponent's quadratic in
// the lane's offset from the quadrant centre, with log2(e), -1/2 and log2(opacity) folded in
// (5 FMA per pixel, then the raw v_exp_f32); 0 keeps upstream's per-pixel operation order (the
// core of ocml's expf).  Both are within the
// image tolerance of tests/gpu_helpers.py.
#include <type_traits>

#include "gsr_internal.h"

using namespace gsr;

namespace {

// ocml __ocml_exp_f32 (non-DAZ path) without the final range selects: identical results for
// every finite argument (below about -104 both give 0, above 88.7 both give +inf).
__device__ __forceinline__ float exp_core(float x) {
    const float kLog2eHi = 0x1.715476p+0f;   // 1.44269502
    const float kLog2eLo = 0x1.4ae0bep-26f;  // 1.92596299e-08
    const float ph = x * kLog2eHi;
    const float n = __builtin_rintf(ph);
    const float hi = ph - n;
    float lo = __builtin_fmaf(x, kLog2eHi, -ph);
    lo = __builtin_fmaf(x, kLog2eLo, lo);
    const float e = __builtin_amdgcn_exp2f(hi + lo);
    return __builtin_ldexpf(e, (int)n);
}

// Lower bound of q(u, v) = A u^2 + 2B uv + C v^2 evaluated in float: q minus a bound on its
// rounding error.
__device__ __forceinline__ float q_lower(float A, float B, float C, float u, float v) {
    const float uu = A * u * u, uv = 2.0f * B * u * v, vv = C * v * v;
    return (uu + uv + vv) - 16.0f * 5.96e-8f * (uu + fabsf(uv) + vv);
}

// May the splat reach alpha >= 1/255 at some pixel centre of the box [bx0,bx1] x [by0,by1]?
// False only when provably not (NaN / inf data always answer true).
__device__ __forceinline__ bool may_touch(float x, float y, float A, float B, float C, float ex,
                                          float ey, float twoL, float bx0, float bx1, float by0,
                                          float by1) {
    const float ulo = bx0 - x, uhi = bx1 - x, vlo = by0 - y, vhi = by1 - y;
    if (fmaxf(fmaxf(ulo, -uhi), 0.0f) > ex || fmaxf(fmaxf(vlo, -vhi), 0.0f) > ey) return false;
    if (ulo <= 0.0f && uhi >= 0.0f && vlo <= 0.0f && vhi >= 0.0f) return true;
    // centre outside the box: q is convex, so its minimum over the box lies on an edge whose
    // constraint the centre violates (at the minimiser, the direction to the centre leaves the
    // box through an active face), where it is the 1-D minimum clamped to the edge: at most one
    // vertical and one horizontal edge.  The minimiser's slope -B/C (-B/A) comes from
    // v_rcp_f32 (1 ulp) instead of an IEEE division (~10 VALU): a minimiser a few ulp off
    // raises q there by C * dv^2 ~ 1e-13 * q, far inside q_lower's 16-ulp rounding margin.
    const float su = -B * __builtin_amdgcn_rcpf(C), sv = -B * __builtin_amdgcn_rcpf(A);
    const float ue = ulo > 0.0f ? ulo : uhi, ve = vlo > 0.0f ? vlo : vhi;
    const float lu = q_lower(A, B, C, ue, fminf(fmaxf(su * ue, vlo), vhi));
    const float lv = q_lower(A, B, C, fminf(fmaxf(sv * ve, ulo), uhi), ve);
    const float inf = __builtin_huge_valf();
    const float lb = fminf((ulo > 0.0f || uhi < 0.0f) ? lu : inf,
                           (vlo > 0.0f || vhi < 0.0f) ? lv : inf);
    return !(lb > twoL);
}

// Block -> tile, XCD-aware: the hardware deals block b to XCD b % 8 (speed only, never
// correctness); groups of kGroupTiles consecutive tiles (four row-adjacent tiles, 16 quadrant
// waves) go round-robin over the XCDs, so each group shares one L2 while the image's heavy and
// light regions are spread evenly over the 8 XCDs.  With `order` (k_blend_order) the groups are
// dealt heaviest first: every wave of the last round is then a short one, and the kernel's
// tail -- the last waves finishing on an emptying chip -- shrinks.
constexpr uint32_t kGroupTiles = 4;
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, const uint32_t *order,
                                             uint32_t n_groups) {
    const uint32_t x = b & 7u, l = b >> 3;
    uint32_t g = (l / kGroupTiles) * 8u + x;
    if (order && g < n_groups) g = order[g];
    return g * kGroupTiles + l % kGroupTiles;
}

// Counting sort of the tile groups by a log-scale pair count, descending (one block; order
// within a bucket is arbitrary and does not matter: each wave's output depends only on its own
// quadrant).  Key: 32 steps per octave of (pairs + 1), 1024 buckets.
constexpr int kOrderBuckets = 1024;
__device__ __forceinline__ uint32_t order_key(const uint2 *ranges, uint32_t g, uint32_t n_tiles) {
    uint32_t n = 0;
    const uint32_t t0 = g * kGroupTiles;
#pragma unroll
    for (uint32_t i = 0; i < kGroupTiles; ++i)
        if (t0 + i < n_tiles) {
            const uint2 r = ranges[t0 + i];
            n += r.y - r.x;
        }
    const int k = (int)(__builtin_amdgcn_logf((float)n + 1.0f) * 32.0f);
    return (uint32_t)(kOrderBuckets - 1 - min(k, kOrderBuckets - 1));
}

constexpr int kOrderThreads = 1024;  // one block; kOrderBuckets / it per thread
constexpr int kOrderPer = kOrderBuckets / kOrderThreads;
__global__ __launch_bounds__(kOrderThreads) void k_blend_order(const uint2 *__restrict__ ranges,
                                                               uint32_t n_tiles, uint32_t n_groups,
                                                               uint32_t *__restrict__ order) {
    __shared__ uint32_t s_h[kOrderBuckets];
    __shared__ uint32_t s_w[kOrderThreads / 64];
    const int tid = threadIdx.x;
    for (int i = tid; i < kOrderBuckets; i += kOrderThreads) s_h[i] = 0u;
    __syncthreads();
    for (uint32_t g = tid; g < n_groups; g += kOrderThreads)
        atomicAdd(&s_h[order_key(ranges, g, n_tiles)], 1u);
    __syncthreads();
    // exclusive scan of the 1024 bucket counts, kOrderPer consecutive buckets per thread
    uint32_t c[kOrderPer], sum = 0;
#pragma unroll
    for (int i = 0; i < kOrderPer; ++i) sum += (c[i] = s_h[tid * kOrderPer + i]);
    uint32_t x = sum;
    const int lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    uint32_t base = x - sum;
    for (int i = 0; i < w; ++i) base += s_w[i];
#pragma unroll
    for (int i = 0; i < kOrderPer; ++i) {
        s_h[tid * kOrderPer + i] = base;
        base += c[i];
    }
    __syncthreads();
    for (uint32_t g = tid; g < n_groups; g += kOrderThreads)
        order[atomicAdd(&s_h[order_key(ranges, g, n_tiles)], 1u)] = g;
}

// One staged splat as the inner loop reads it: three 16-B LDS reads from one address (fast
// arithmetic without n_contrib: a pair shares the even slot's e = {b0, b1, bound0, bound1}).
// exact: g = x, y, conic a, conic b; q = conic c, opacity, r, g; e = b, position + 1 (uint bits:
// upstream's `contributor`), -, -.
// fast: the exponent as a quadratic in the lane's offset (u, v) from the quadrant centre,
// log2(opacity) folded in: p = k0 + k1 u + k2 v + k3 u^2 + k4 uv + k5 v^2 (g = k0..k3,
// q = k4, k5, r, g); e = b, position + 1, the bound p must not exceed (log2(opacity): p > it <=>
// upstream's power > 0; +inf for a positive-definite conic), -.
struct StagedSplat {
    float4 g;
    float4 q;
    float4 e;
};

// Blocks are mapped XCD-aware (xcd_tile).  Only the next chunk's point-list ids are
// prefetched (no record prefetch): the kernel fits 64 VGPRs and 8 waves per SIMD, and the
// record gathers' latency is left to the other waves (a record prefetch spilled at 8 waves
// and lost at fewer).  A block per tile with shared staging lost to independent
// quadrant waves (its batch barriers cost ~40 % of wave time), and so did a separate kernel
// culling each splat once per tile into per-quadrant lists (the in-wave cull is ~5 % of the
// blend's VALU; the extra pass over the lists cost more than it saved).
// kContrib: track the last contributor (the n_contrib output); off (no n_contrib requested),
// the composite step loses one v_cndmask.
template <bool kFast, bool kContrib>
__global__ __launch_bounds__(256, 8) void k_blend_q(const GsrBlendArgs a, uint32_t n_tiles) {
    __shared__ StagedSplat s_spl_q[4][64];  // per quadrant wave
    constexpr bool kPair = kFast && !kContrib;  // paired colour / bound words (see staging)

    const uint32_t tile = xcd_tile(blockIdx.x, a.order, (n_tiles + kGroupTiles - 1) / kGroupTiles);
    if (tile >= n_tiles) return;
    if (a.list_n && *a.list_n > a.list_cap) return;  // not binned (frame graphs: re-rendered)
    const uint32_t quad = threadIdx.x >> 6;  // this wave's quadrant
    const int lane = threadIdx.x & 63;
    StagedSplat *const s_spl = s_spl_q[quad];
    const uint32_t tx = tile % a.grid_x, ty_local = tile / a.grid_x, ty = a.row_begin + ty_local;
    const int qx0 = (int)tx * GSR_TILE_X + (int)(quad & 1u) * 8;
    const int qy0 = (int)ty * GSR_TILE_Y + (int)(quad >> 1) * 8;
    const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;
    // fast: the lane's offset from the quadrant centre and its products (exact small values)
    const float pu = (float)(lane & 7) - 3.5f, pv = (float)(lane >> 3) - 3.5f;
    const float puu = pu * pu, puv = pu * pv, pvv = pv * pv;

    const uint2 range = a.ranges[tile];
    // done carried in the sign of T, as in k_blend
    float T = inside ? 1.0f : -1.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
    uint32_t last_contributor = 0;
    auto live_any = [&]() { return __ballot(!(T <= 0.0f)) != 0ull; };
    if (!live_any()) return;

    // kBound (fast form): test upstream's power > 0 skip as p > bound -- only chunks holding a
    // conic that is not positive definite need it (staging below)
    auto composite = [&](const StagedSplat &sp, auto bound_tag) {
        constexpr bool kBound = decltype(bound_tag)::value;
        bool vis, acc, term;
        float test_T;
        if (kFast) {
            // The loop-carried chain is only T -> T (1 - alpha_eff) -> compare -> select:
            // alpha_eff = 0 for an invisible splat (then test_T = T), and a pixel that
            // terminates keeps -|T| (idempotent once done).  The weight is |T| - |T'|: T - test_T
            // while the pixel composites, 0 for the terminating splat and after it.
            float p2 = __builtin_fmaf(sp.g.y, pu, sp.g.x);
            p2 = __builtin_fmaf(sp.g.z, pv, p2);
            p2 = __builtin_fmaf(sp.g.w, puu, p2);
            p2 = __builtin_fmaf(sp.q.x, puv, p2);
            p2 = __builtin_fmaf(sp.q.y, pvv, p2);
            const float alpha = fminf(0.99f, __builtin_amdgcn_exp2f(p2));
            vis = !(alpha < 1.0f / 255.0f);
            if (kBound) vis = vis && !(p2 > sp.e.z);
            // T (1 - alpha) as one fma, T - alpha T; alpha_eff = 0 leaves T exactly
            const float alpha_eff = vis ? alpha : 0.0f;
            test_T = __builtin_fmaf(-T, alpha_eff, T);
            const bool lo = test_T < 0.0001f;
            const float T_next = lo ? -fabsf(T) : test_T;
            const float wgt = fabsf(T) - fabsf(T_next);
            C0 = __builtin_fmaf(sp.q.z, wgt, C0);
            C1 = __builtin_fmaf(sp.q.w, wgt, C1);
            C2 = __builtin_fmaf(sp.e.x, wgt, C2);
            if (kContrib)
                last_contributor = (vis && !lo) ? __float_as_uint(sp.e.y) : last_contributor;
            T = T_next;
            return;
        } else {
            const float dx = sp.g.x - pfx, dy = sp.g.y - pfy;
            const float power =
                -0.5f * (sp.g.z * dx * dx + sp.q.x * dy * dy) - sp.g.w * dx * dy;
            const float alpha = fminf(0.99f, sp.q.y * exp_core(power));
            vis = !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
            test_T = T * (1 - alpha);
            acc = vis && !(test_T < 0.0001f);
            term = vis && (test_T < 0.0001f);
            C0 = acc ? C0 + sp.q.z * alpha * T : C0;
            C1 = acc ? C1 + sp.q.w * alpha * T : C1;
            C2 = acc ? C2 + sp.e.x * alpha * T : C2;
        }
        T = acc ? test_T : (term ? -fabsf(T) : T);
        if (kContrib) last_contributor = acc ? __float_as_uint(sp.e.y) : last_contributor;
    };
    const float X0 = (float)qx0, Y0 = (float)qy0;

    // the next chunk's ids are in flight while this chunk's records are gathered
    const uint32_t i0 = range.x + (uint32_t)lane;
    uint32_t id_next = i0 < range.y ? (a.point_list[i0] & a.id_mask) : 0u;
    for (uint32_t start = range.x; start < range.y; start += 64) {
        const uint32_t idx = start + (uint32_t)lane;
        const bool valid = idx < range.y;
        SplatRecord r;
        if (valid) r = a.records[id_next];
        if (idx + 64u < range.y) id_next = (a.point_list[idx + 64u] & a.id_mask);

        bool keep = valid;
        if (valid && a.cull)
            keep = may_touch(r.a.x, r.a.y, r.a.z, r.a.w, r.b.x, r.b.z, r.b.w, 2.0f * r.c.x, X0,
                             X0 + 7, Y0, Y0 + 7);
        const uint64_t bal = __ballot(keep);
        bool npd = false;  // a staged conic that is not positive definite (fast form)
        if (keep) {
            StagedSplat st;
            if (kFast) {
                // exponent log2(e) * (-q/2) = a dx^2 + b dx dy + c dy^2 with dx = ex - u,
                // dy = ey - v, expanded in (u, v)
                const float kL2e = 1.4426950408889634f;
                const float ca = r.a.z * (-0.5f * kL2e), cb = r.a.w * (-kL2e),
                            cc = r.b.x * (-0.5f * kL2e);
                const float ex = r.a.x - (X0 + 3.5f), ey = r.a.y - (Y0 + 3.5f);
                const float lo = __builtin_amdgcn_logf(r.b.y);  // log2(opacity)
                const float k0 = __builtin_fmaf(ex, __builtin_fmaf(ca, ex, cb * ey), cc * ey * ey);
                st.g = make_float4(k0 + lo, __builtin_fmaf(-2.0f * ca, ex, -cb * ey),
                                   __builtin_fmaf(-cb, ex, -2.0f * cc * ey), ca);
                st.q = make_float4(cb, cc, r.c.y, r.c.z);
                // upstream skips power > 0, which a positive-definite conic reaches only through
                // rounding; the expanded form rounds differently (at a centre that falls on a
                // pixel it can land just above 0), so the test is kept for the other conics only
                const bool pd = ca < 0.0f && cc < 0.0f && 4.0f * ca * cc > cb * cb;
                npd = !pd;
                st.e = make_float4(r.c.w, __uint_as_float(idx - range.x + 1u),
                                   pd ? __builtin_huge_valf() : lo, 0.0f);
            } else {
                st.g = r.a;
                st.q = make_float4(r.b.x, r.b.y, r.c.y, r.c.z);
                st.e = make_float4(r.c.w, __uint_as_float(idx - range.x + 1u), 0.0f, 0.0f);
            }
            const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            const int slot = __popcll(bal & lt);  // compacted in list order
            if (kPair) {
                // a pair's blues and power bounds share the even slot's e: {b0, b1, bound0,
                // bound1} (5 LDS reads per composited pair instead of 6)
                s_spl[slot].g = st.g;
                s_spl[slot].q = st.q;
                float *pe = &s_spl[slot & ~1].e.x;
                pe[slot & 1] = st.e.x;
                pe[2 + (slot & 1)] = st.e.z;
            } else {
                s_spl[slot] = st;
            }
        }
        int count = __popcll(bal);
        if (count == 0) continue;
        // the compacted slots are the list (no index indirection); an odd count is padded with
        // an opacity-0 splat in slot `count` (< 64 for an odd count): exact: opacity 0; fast:
        // exponent -inf (alpha 0, the bound-free loop included) and a power bound of -inf
        if (count & 1) {
            if (kPair) {
                if (lane < 8)
                    reinterpret_cast<float *>(&s_spl[count])[lane] =
                        lane == 0 ? -__builtin_huge_valf() : 0.0f;
                if (lane == 8) s_spl[count - 1].e.y = 0.0f;
                if (lane == 9) s_spl[count - 1].e.w = -__builtin_huge_valf();
            } else if (lane < 12) {
                reinterpret_cast<float *>(&s_spl[count])[lane] =
                    (kFast && (lane == 0 || lane == 10)) ? -__builtin_huge_valf() : 0.0f;
            }
            ++count;
        }
        // one wave: its LDS writes above complete before the reads below are served

        // single-buffered: a software-pipelined form (the next pair's LDS reads in flight
        // during this pair) spilled past 64 VGPRs and was slower
        auto composite_all = [&](auto bound_tag) {
            for (int k = 0; k < count; k += 2) {
                if (kPair) {
                    const float4 e = s_spl[k].e;
                    composite(StagedSplat{s_spl[k].g, s_spl[k].q, make_float4(e.x, 0.0f, e.z, 0.0f)},
                              bound_tag);
                    composite(StagedSplat{s_spl[k + 1].g, s_spl[k + 1].q,
                                          make_float4(e.y, 0.0f, e.w, 0.0f)},
                              bound_tag);
                } else {
                    const StagedSplat a0 = s_spl[k], a1 = s_spl[k + 1];
                    composite(a0, bound_tag);
                    composite(a1, bound_tag);
                }
            }
        };
        // (the exact form always tests power > 0, as upstream writes it)
        if (!kFast || __ballot(npd) != 0ull)
            composite_all(std::integral_constant<bool, true>{});
        else
            composite_all(std::integral_constant<bool, false>{});
        if (!live_any()) break;
    }

    if (inside) {
        const int row = py - a.y0;
        const size_t pid = (size_t)row * a.W + px;
        const size_t plane = (size_t)a.rows_out * a.W;
        const float Tf = fabsf(T);
        if (a.final_T) a.final_T[pid] = Tf;
        if (kContrib && a.n_contrib) a.n_contrib[pid] = last_contributor;
        a.out_color[pid] = C0 + Tf * a.bg[0];
        a.out_color[plane + pid] = C1 + Tf * a.bg[1];
        a.out_color[2 * plane + pid] = C2 + Tf * a.bg[2];
    }
}

// Grid of whole XCD groups: one block per tile, kGroupTiles per XCD round; blocks past the
// last tile exit.
inline uint32_t xcd_grid(uint32_t n_tiles) {
    const uint32_t g = kGroupTiles * 8u;
    return (n_tiles + g - 1) / g * g;
}

}  // namespace

uint32_t gsr_blend_order_groups(uint32_t n_tiles) {
    return (n_tiles + kGroupTiles - 1) / kGroupTiles;
}

hipError_t gsr_launch_blend_order(const uint2 *ranges, uint32_t n_tiles, uint32_t *order,
                                  hipStream_t s) {
    if (n_tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(k_blend_order, dim3(1), dim3(kOrderThreads), 0, s, ranges, n_tiles,
                       gsr_blend_order_groups(n_tiles), order);
    return hipGetLastError();
}

hipError_t gsr_launch_blend(const GsrBlendArgs &a, hipStream_t s) {
    if (a.rows_tiles == 0 || a.grid_x == 0) return hipSuccess;
    const uint32_t n_tiles = a.grid_x * a.rows_tiles;
    const dim3 grid(xcd_grid(n_tiles));
    if (a.fast && !a.n_contrib)
        hipLaunchKernelGGL((k_blend_q<true, false>), grid, dim3(256), 0, s, a, n_tiles);
    else if (a.fast)
        hipLaunchKernelGGL((k_blend_q<true, true>), grid, dim3(256), 0, s, a, n_tiles);
    else
        hipLaunchKernelGGL((k_blend_q<false, true>), grid, dim3(256), 0, s, a, n_tiles);
    return hipGetLastError();
}
