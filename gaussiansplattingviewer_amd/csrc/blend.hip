// blend.hip -- per-tile front-to-back alpha compositing for gfx950.
//
// Replaces upstream diff-gaussian-rasterization forward.cu renderCUDA (GLSL twin of the
// per-pixel alpha: shaders/gau_frag.glsl:21-27).  One 256-thread block per 16x16 tile; each
// of its 4 waves owns an 8x8 quadrant, one pixel per lane.  The tile's depth-sorted splat list
// is staged through LDS 256 splats at a time; `__syncthreads_count(done)` ends the tile when
// every pixel has saturated, as upstream.
//
// gfx950-specific structure:
//  * cull once per staged splat, not once per (splat, wave): the loading thread tests the
//    splat's conservative alpha >= 1/255 ellipse (preprocess.hip cull_data) against the tile's
//    four 8x8 quadrants -- bounding box first, then the exact ellipse-box minimum with a
//    rounding bound -- and stores a 4-bit mask; each wave then compacts the batch to the
//    splats that can touch its quadrant (ballot + popcount) and loops over that list only;
//  * branch-free per-pixel body (selects instead of nested ifs, so no exec-mask churn) with
//    the LDS reads of the next splat issued before the current one is evaluated;
//  * exp: the core of ocml's expf (range-reduced v_exp_f32 + ldexp), bit-identical to expf
//    over the range that matters, without its under/overflow selects;
//  * optional fast arithmetic (GSR_OPT_BLEND_FAST): log2(e) and -1/2 folded into the conic at
//    staging time, FMA-contracted quadratic form and the raw v_exp_f32 -- 2 of the 9 exp
//    instructions and ~40 % of the per-pixel VALU work; pixels then differ from upstream's
//    order by float rounding only.
// The per-pixel arithmetic keeps upstream's operation order, so the image differs from the
// CPU oracle only through expf itself (device vs glibc).  n_contrib equals upstream's running
// `contributor` at the last contributing splat = its position in the tile list + 1, so
// skipping splats that cannot contribute does not change it.
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
    // centre outside the box: q is convex, so its minimum over the box lies on an edge, where
    // it is the 1-D minimum clamped to the edge.  The minimiser's slope -B/C (-B/A) comes from
    // v_rcp_f32 (1 ulp) instead of an IEEE division (~10 VALU): a minimiser a few ulp off
    // raises q there by C * dv^2 ~ 1e-13 * q, far inside q_lower's 16-ulp rounding margin.
    const float su = -B * __builtin_amdgcn_rcpf(C), sv = -B * __builtin_amdgcn_rcpf(A);
    float lb = q_lower(A, B, C, ulo, fminf(fmaxf(su * ulo, vlo), vhi));
    lb = fminf(lb, q_lower(A, B, C, uhi, fminf(fmaxf(su * uhi, vlo), vhi)));
    lb = fminf(lb, q_lower(A, B, C, fminf(fmaxf(sv * vlo, ulo), uhi), vlo));
    lb = fminf(lb, q_lower(A, B, C, fminf(fmaxf(sv * vhi, ulo), uhi), vhi));
    return !(lb > twoL);
}

constexpr int kBatch = 256;  // splats staged in LDS per round

typedef float v2f __attribute__((ext_vector_type(2)));


// One staged splat as the inner loop reads it: three 16-B LDS reads from one address.
struct StagedSplat {
    float4 g;  // x, y, conic a, conic b      (fast: prescaled a, b)
    float4 q;  // conic c, opacity, r, g      (fast: prescaled c)
    float4 e;  // b, list position + 1 (uint bits: upstream's `contributor`), -, -
};

// Diagnostics build (kStamp): lane 0 of every wave sums s_memtime cycles per phase into
// a.stamps[shard * 8 + 0..5] = {staging incl. barriers, list compaction, compositing, batches, splats
// composited, waves}.
template <bool kFast, bool kStamp = false>
__global__ __launch_bounds__(256) void k_blend(const GsrBlendArgs a) {
    // slot kBatch: an opacity-0 splat that pads odd lists (alpha 0 < 1/255: never visible)
    __shared__ StagedSplat s_spl[kBatch + 1];
    __shared__ uint8_t s_mask[kBatch];          // quadrant bits of each staged splat
    __shared__ uint16_t s_list[4][kBatch + 1];  // per wave: byte offsets into s_spl

    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t tx = blockIdx.x, ty_local = blockIdx.y, ty = a.row_begin + ty_local;
    const int tx0 = (int)tx * GSR_TILE_X, ty0 = (int)ty * GSR_TILE_Y;
    const int px = tx0 + (w & 1) * 8 + (lane & 7), py = ty0 + (w >> 1) * 8 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;
    if (tid == 0) {
        s_spl[kBatch].g = make_float4(0.f, 0.f, 0.f, 0.f);
        s_spl[kBatch].q = make_float4(0.f, 0.f, 0.f, 0.f);
        s_spl[kBatch].e = make_float4(0.f, 0.f, 0.f, 0.f);
    }

    const uint2 range = a.ranges[ty_local * a.grid_x + tx];
    // A pixel is done (upstream's `done`) once T would fall below 1e-4; T then keeps its last
    // value with the sign flipped, so one register carries both and the per-splat update needs
    // no separate flag: a done pixel's test_T is <= 0, which no longer accumulates, and
    // re-terminating it leaves -|T| unchanged.  |T| is upstream's final T.  A NaN T (NaN
    // input) is never done, as upstream.
    float T = inside ? 1.0f : -1.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
    uint32_t last_contributor = 0;

    auto composite = [&](const StagedSplat &sp) {
        const float dx = sp.g.x - pfx, dy = sp.g.y - pfy;
        bool vis, acc, term;
        float test_T, wgt;
        if (kFast) {
            // log2(e) * power with the constants folded in: dx (a dx + b dy) + c dy^2
            const float p2 =
                __builtin_fmaf(dx, __builtin_fmaf(sp.g.z, dx, sp.g.w * dy), sp.q.x * dy * dy);
            const float alpha = fminf(0.99f, sp.q.y * __builtin_amdgcn_exp2f(p2));
            vis = !(p2 > 0.0f) && !(alpha < 1.0f / 255.0f);
            // same arithmetic as k_blend_q (short loop-carried chain through T)
            const float alpha_eff = vis ? alpha : 0.0f;
            test_T = __builtin_fmaf(-T, alpha_eff, T);
            const bool lo = test_T < 0.0001f;
            wgt = lo ? 0.0f : T - test_T;
            C0 = __builtin_fmaf(sp.q.z, wgt, C0);
            C1 = __builtin_fmaf(sp.q.w, wgt, C1);
            C2 = __builtin_fmaf(sp.e.x, wgt, C2);
            last_contributor = (vis && !lo) ? __float_as_uint(sp.e.y) : last_contributor;
            T = lo ? -fabsf(T) : test_T;
            return;
        } else {
            // upstream renderCUDA per-pixel body, same operation order
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
        last_contributor = acc ? __float_as_uint(sp.e.y) : last_contributor;
    };
    const char *lds = reinterpret_cast<const char *>(s_spl);
    auto fetch = [&](uint32_t off) { return *reinterpret_cast<const StagedSplat *>(lds + off); };

    unsigned long long t_stage = 0, t_list = 0, t_comp = 0, n_batch = 0, n_splat = 0, t0 = 0;
    if (kStamp) t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t start = range.x; start < range.y; start += kBatch) {
        if (__syncthreads_count(T <= 0.0f) == 256) break;
        const uint32_t idx = start + tid;
        if (idx < range.y) {
            const SplatRecord r = a.records[(a.point_list[idx] & a.id_mask)];
            uint32_t m = 0xF;
            if (a.cull) {
                const float x = r.a.x, y = r.a.y, A = r.a.z, B = r.a.w, C = r.b.x;
                const float ex = r.b.z, ey = r.b.w, twoL = 2.0f * r.c.x;
                const float X0 = (float)tx0, Y0 = (float)ty0;
                m = (uint32_t)may_touch(x, y, A, B, C, ex, ey, twoL, X0, X0 + 7, Y0, Y0 + 7) |
                    ((uint32_t)may_touch(x, y, A, B, C, ex, ey, twoL, X0 + 8, X0 + 15, Y0, Y0 + 7) << 1) |
                    ((uint32_t)may_touch(x, y, A, B, C, ex, ey, twoL, X0, X0 + 7, Y0 + 8, Y0 + 15) << 2) |
                    ((uint32_t)may_touch(x, y, A, B, C, ex, ey, twoL, X0 + 8, X0 + 15, Y0 + 8, Y0 + 15) << 3);
            }
            StagedSplat st;
            if (kFast) {
                const float kL2e = 1.4426950408889634f;
                st.g = make_float4(r.a.x, r.a.y, r.a.z * (-0.5f * kL2e), r.a.w * (-kL2e));
                st.q = make_float4(r.b.x * (-0.5f * kL2e), r.b.y, r.c.y, r.c.z);
            } else {
                st.g = r.a;
                st.q = make_float4(r.b.x, r.b.y, r.c.y, r.c.z);
            }
            st.e = make_float4(r.c.w, __uint_as_float(idx - range.x + 1u), 0.0f, 0.0f);
            s_spl[tid] = st;
            s_mask[tid] = (uint8_t)m;
        }
        __syncthreads();
        if (kStamp) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            t_stage += t1 - t0;
            t0 = t1;
            ++n_batch;
        }
        const int n = (int)min((uint32_t)kBatch, range.y - start);

        // This wave's splats of the batch, in list order, padded to an even count.
        int count = 0;
        for (int base = 0; base < n; base += 64) {
            const int j = base + lane;
            const bool keep = j < n && ((s_mask[j] >> w) & 1u);
            const uint64_t bal = __ballot(keep);
            const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            if (keep)
                s_list[w][count + __popcll(bal & lt)] = (uint16_t)(j * sizeof(StagedSplat));
            count += __popcll(bal);
        }
        if (count & 1) {
            if (lane == 0) s_list[w][count] = (uint16_t)(kBatch * sizeof(StagedSplat));
            ++count;
        }
        // s_list[w] is written and read by this wave only: LDS ops of one wave execute in
        // order, so no barrier is needed before the reads below.
        if (count == 0 || __ballot(!(T <= 0.0f)) == 0ull) continue;

        // Two splats per iteration, straight-line (the scheduler interleaves their
        // T-independent parts); the next pair's LDS reads are issued before this pair runs.
        // A/B register sets alternate so no prefetched splat is ever copied.
        const uint16_t *list = s_list[w];
        auto next2 = [&](int k) { return k + 2 < count ? k + 2 : count - 2; };
        StagedSplat a0 = fetch(list[0]), a1 = fetch(list[1]);
        for (int k = 0;;) {
            int kn = next2(k);
            const StagedSplat b0 = fetch(list[kn]), b1 = fetch(list[kn + 1]);
            composite(a0);
            composite(a1);
            k += 2;
            if (k >= count) break;
            kn = next2(k);
            a0 = fetch(list[kn]);
            a1 = fetch(list[kn + 1]);
            composite(b0);
            composite(b1);
            k += 2;
            if (k >= count) break;
            if ((k & 28) == 0 && __ballot(!(T <= 0.0f)) == 0ull) break;
        }
        if (kStamp) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            t_comp += t1 - t0;
            t0 = t1;
            n_splat += (unsigned long long)count;
        }
    }
    if (kStamp && lane == 0) {  // 256 shards of 8 counters: same-address atomics serialise
        unsigned long long *st = a.stamps + 8 * ((blockIdx.x + blockIdx.y * 17 + w) & 255);
        atomicAdd(&st[0], t_stage);
        atomicAdd(&st[1], t_list);
        atomicAdd(&st[2], t_comp);
        atomicAdd(&st[3], n_batch);
        atomicAdd(&st[4], n_splat);
        atomicAdd(&st[5], 1ull);
    }

    if (inside) {
        const int row = py - a.y0;
        const size_t pid = (size_t)row * a.W + px;
        const size_t plane = (size_t)a.rows_out * a.W;
        const float Tf = fabsf(T);
        if (a.final_T) a.final_T[pid] = Tf;
        if (a.n_contrib) a.n_contrib[pid] = last_contributor;
        a.out_color[pid] = C0 + Tf * a.bg[0];
        a.out_color[plane + pid] = C1 + Tf * a.bg[1];
        a.out_color[2 * plane + pid] = C2 + Tf * a.bg[2];
    }
}

// Block -> work item, XCD-aware: the hardware dispatches block b to XCD b % 8; groups of
// `group` consecutive work items (a tile's quadrants and its row neighbours) go round-robin
// over the XCDs, so each group shares one L2 while the image's heavy and light regions are
// spread evenly over the 8 XCDs.  group = 0: plain order.
__device__ __forceinline__ uint32_t xcd_work(uint32_t b, uint32_t group) {
    if (group == 0) return b;
    const uint32_t x = b & 7u, l = b >> 3;
    return ((l / group) * 8u + x) * group + l % group;
}

// One wave per (tile, 8x8 quadrant), 64-thread blocks, no block barriers: each wave streams
// its tile's list 64 splats at a time, culls them against its own quadrant, compacts the
// survivors and composites them, and stops as soon as its own 64 pixels are done -- so a
// quadrant never waits for the slowest quadrant of its tile (the 4-wave kernel's batch
// barriers cost ~40 % of wave time, measured with GSR_DEBUG_BLEND_STAMPS).  Record gathers
// are software-pipelined: a chunk's records are loaded while the previous chunk is
// composited, their ids one chunk earlier still.  Blocks are mapped XCD-aware (xcd_work).
// kLean: no record prefetch (only the next chunk's ids), so the kernel fits 64 VGPRs and
// 8 waves per SIMD; the record gathers' latency is then left to the other waves.
// kContrib: track the last contributor (the n_contrib output); off (no n_contrib requested),
// the composite step loses one v_cndmask.
template <bool kFast, bool kLean = false, bool kContrib = true>
__global__ __launch_bounds__(64, kLean ? 8 : 1) void k_blend_q(const GsrBlendArgs a,
                                                             uint32_t n_work, uint32_t per_xcd) {
    __shared__ StagedSplat s_spl[64];

    const uint32_t b = blockIdx.x;
    const uint32_t work = xcd_work(b, a.xcd_group);
    if (work >= n_work) return;
    const int lane = threadIdx.x;
    const uint32_t tile = work >> 2, quad = work & 3u;
    const uint32_t tx = tile % a.grid_x, ty_local = tile / a.grid_x, ty = a.row_begin + ty_local;
    const int qx0 = (int)tx * GSR_TILE_X + (int)(quad & 1u) * 8;
    const int qy0 = (int)ty * GSR_TILE_Y + (int)(quad >> 1) * 8;
    const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;

    const uint2 range = a.ranges[tile];
    // done carried in the sign of T, as in k_blend
    float T = inside ? 1.0f : -1.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
    uint32_t last_contributor = 0;
    auto live_any = [&]() { return __ballot(!(T <= 0.0f)) != 0ull; };
    if (!live_any()) return;

    auto composite = [&](const StagedSplat &sp) {
        const float dx = sp.g.x - pfx, dy = sp.g.y - pfy;
        bool vis, acc, term;
        float test_T;
        if (kFast) {
            // The loop-carried chain is only T -> T (1 - alpha_eff) -> compare -> select:
            // alpha_eff = 0 for an invisible splat (then test_T = T and the weight T - test_T
            // is 0), and a pixel that terminates keeps -|T| (idempotent once done).
            const float p2 =
                __builtin_fmaf(dx, __builtin_fmaf(sp.g.z, dx, sp.g.w * dy), sp.q.x * dy * dy);
            const float alpha = fminf(0.99f, sp.q.y * __builtin_amdgcn_exp2f(p2));
            vis = !(p2 > 0.0f) && !(alpha < 1.0f / 255.0f);
            // T (1 - alpha) as one fma, T - alpha T; alpha_eff = 0 leaves T exactly
            const float alpha_eff = vis ? alpha : 0.0f;
            test_T = __builtin_fmaf(-T, alpha_eff, T);
            const bool lo = test_T < 0.0001f;
            const float wgt = lo ? 0.0f : T - test_T;
            C0 = __builtin_fmaf(sp.q.z, wgt, C0);
            C1 = __builtin_fmaf(sp.q.w, wgt, C1);
            C2 = __builtin_fmaf(sp.e.x, wgt, C2);
            if (kContrib)
                last_contributor = (vis && !lo) ? __float_as_uint(sp.e.y) : last_contributor;
            T = lo ? -fabsf(T) : test_T;
            return;
        } else {
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

    // pipeline: records of chunk c+1 and ids of chunk c+2 are in flight while c composites
    uint32_t i0 = range.x + (uint32_t)lane;
    uint32_t id_next = i0 < range.y ? (a.point_list[i0] & a.id_mask) : 0u;
    SplatRecord r_next;
    if (!kLean) {
        if (i0 < range.y) r_next = a.records[id_next];
        id_next = i0 + 64u < range.y ? (a.point_list[i0 + 64u] & a.id_mask) : 0u;
    }
    for (uint32_t start = range.x; start < range.y; start += 64) {
        const uint32_t idx = start + (uint32_t)lane;
        const bool valid = idx < range.y;
        SplatRecord r;
        if (kLean) {
            if (valid) r = a.records[id_next];
            if (idx + 64u < range.y) id_next = (a.point_list[idx + 64u] & a.id_mask);
        } else {
            r = r_next;
            if (idx + 64u < range.y) r_next = a.records[id_next];
            if (idx + 128u < range.y) id_next = (a.point_list[idx + 128u] & a.id_mask);
        }

        bool keep = valid;
        if (valid && a.cull)
            keep = may_touch(r.a.x, r.a.y, r.a.z, r.a.w, r.b.x, r.b.z, r.b.w, 2.0f * r.c.x, X0,
                             X0 + 7, Y0, Y0 + 7);
        const uint64_t bal = __ballot(keep);
        if (keep) {
            StagedSplat st;
            if (kFast) {
                const float kL2e = 1.4426950408889634f;
                st.g = make_float4(r.a.x, r.a.y, r.a.z * (-0.5f * kL2e), r.a.w * (-kL2e));
                st.q = make_float4(r.b.x * (-0.5f * kL2e), r.b.y, r.c.y, r.c.z);
            } else {
                st.g = r.a;
                st.q = make_float4(r.b.x, r.b.y, r.c.y, r.c.z);
            }
            st.e = make_float4(r.c.w, __uint_as_float(idx - range.x + 1u), 0.0f, 0.0f);
            const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            const int slot = __popcll(bal & lt);  // compacted in list order
            s_spl[slot] = st;
        }
        int count = __popcll(bal);
        if (count == 0) continue;
        // the compacted slots are the list (no index indirection); an odd count is padded with
        // an opacity-0 splat in slot `count` (< 64 for an odd count)
        if (count & 1) {
            if (lane < 12) reinterpret_cast<float *>(&s_spl[count])[lane] = 0.0f;
            ++count;
        }
        // one wave: its LDS writes above complete before the reads below are served

        auto next2 = [&](int k) { return k + 2 < count ? k + 2 : count - 2; };
        StagedSplat a0 = s_spl[0], a1 = s_spl[1];
        for (int k = 0;;) {
            int kn = next2(k);
            const StagedSplat b0 = s_spl[kn], b1 = s_spl[kn + 1];
            composite(a0);
            composite(a1);
            k += 2;
            if (k >= count) break;
            kn = next2(k);
            a0 = s_spl[kn];
            a1 = s_spl[kn + 1];
            composite(b0);
            composite(b1);
            k += 2;
            if (k >= count) break;
        }
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

// Fast arithmetic, packed, one wave per (tile, 16x8 half): like k_blend_q, but each lane
// owns the two pixels (x, y) and (x + 8, y), so the per-pixel math runs as v_pk_* float2
// instructions (2 pixels per instruction where CDNA4 has packed f32 ops), and the splat-side
// work (LDS reads, list handling, loop control) is shared by two pixels.  A splat is kept if
// it may touch the 16x8 half (one cull test on the half's box).
__global__ __launch_bounds__(64) void k_blend_h(const GsrBlendArgs a, uint32_t n_work,
                                                uint32_t per_xcd) {
    __shared__ StagedSplat s_spl[64 + 1];  // slot 64: opacity-0 pad
    __shared__ uint16_t s_list[64 + 2];

    const uint32_t b = blockIdx.x;
    const uint32_t work = xcd_work(b, a.xcd_group);
    if (work >= n_work) return;
    const int lane = threadIdx.x;
    const uint32_t tile = work >> 1, half = work & 1u;
    const uint32_t tx = tile % a.grid_x, ty_local = tile / a.grid_x, ty = a.row_begin + ty_local;
    const int hx0 = (int)tx * GSR_TILE_X, hy0 = (int)ty * GSR_TILE_Y + (int)half * 8;
    const int pxa = hx0 + (lane & 7), pxb = pxa + 8, py = hy0 + (lane >> 3);
    const bool in_a = pxa < a.W && py < a.H, in_b = pxb < a.W && py < a.H;
    const v2f pfx = {(float)pxa, (float)pxb};
    const float pfy = (float)py;
    if (lane == 0) {
        s_spl[64].g = make_float4(0.f, 0.f, 0.f, 0.f);
        s_spl[64].q = make_float4(0.f, 0.f, 0.f, 0.f);
        s_spl[64].e = make_float4(0.f, 0.f, 0.f, 0.f);
    }

    const uint2 range = a.ranges[tile];
    v2f T = {in_a ? 1.0f : -1.0f, in_b ? 1.0f : -1.0f};  // done in the sign, as k_blend
    v2f C0 = {0.0f, 0.0f}, C1 = {0.0f, 0.0f}, C2 = {0.0f, 0.0f};
    uint32_t last_a = 0, last_b = 0;
    auto live_any = [&]() { return __ballot(!(T.x <= 0.0f) || !(T.y <= 0.0f)) != 0ull; };
    if (!live_any()) return;

    auto composite = [&](const StagedSplat &sp) {
        const v2f dx = (v2f)sp.g.x - pfx;
        const float dy = sp.g.y - pfy;
        const v2f ady = __builtin_elementwise_fma((v2f)sp.g.z, dx, (v2f)(sp.g.w * dy));
        const v2f p2 = __builtin_elementwise_fma(dx, ady, (v2f)(sp.q.x * dy * dy));
        v2f e;
        e.x = __builtin_amdgcn_exp2f(p2.x);
        e.y = __builtin_amdgcn_exp2f(p2.y);
        const v2f oe = (v2f)sp.q.y * e;
        v2f alpha;
        alpha.x = fminf(0.99f, oe.x);
        alpha.y = fminf(0.99f, oe.y);
        const v2f aT = alpha * T;
        const v2f test_T = T - aT;
        const bool vis_a = !(p2.x > 0.0f) && !(alpha.x < 1.0f / 255.0f);
        const bool vis_b = !(p2.y > 0.0f) && !(alpha.y < 1.0f / 255.0f);
        const bool lo_a = test_T.x < 0.0001f, lo_b = test_T.y < 0.0001f;
        const bool acc_a = vis_a && !lo_a, acc_b = vis_b && !lo_b;
        v2f wgt;
        wgt.x = acc_a ? aT.x : 0.0f;
        wgt.y = acc_b ? aT.y : 0.0f;
        C0 = __builtin_elementwise_fma((v2f)sp.q.z, wgt, C0);
        C1 = __builtin_elementwise_fma((v2f)sp.q.w, wgt, C1);
        C2 = __builtin_elementwise_fma((v2f)sp.e.x, wgt, C2);
        T.x = acc_a ? test_T.x : ((vis_a && lo_a) ? -fabsf(T.x) : T.x);
        T.y = acc_b ? test_T.y : ((vis_b && lo_b) ? -fabsf(T.y) : T.y);
        const uint32_t pos = __float_as_uint(sp.e.y);
        last_a = acc_a ? pos : last_a;
        last_b = acc_b ? pos : last_b;
    };
    const char *lds = reinterpret_cast<const char *>(s_spl);
    auto fetch = [&](uint32_t off) { return *reinterpret_cast<const StagedSplat *>(lds + off); };
    const float X0 = (float)hx0, Y0 = (float)hy0;
    const float kL2e = 1.4426950408889634f;

    uint32_t i0 = range.x + (uint32_t)lane;
    uint32_t id_next = i0 + 64u < range.y ? (a.point_list[i0 + 64u] & a.id_mask) : 0u;
    SplatRecord r_next;
    if (i0 < range.y) r_next = a.records[(a.point_list[i0] & a.id_mask)];
    for (uint32_t start = range.x; start < range.y; start += 64) {
        const uint32_t idx = start + (uint32_t)lane;
        const bool valid = idx < range.y;
        const SplatRecord r = r_next;
        if (idx + 64u < range.y) r_next = a.records[id_next];
        if (idx + 128u < range.y) id_next = (a.point_list[idx + 128u] & a.id_mask);

        bool keep = valid;
        if (valid && a.cull)
            keep = may_touch(r.a.x, r.a.y, r.a.z, r.a.w, r.b.x, r.b.z, r.b.w, 2.0f * r.c.x, X0,
                             X0 + 15, Y0, Y0 + 7);
        const uint64_t bal = __ballot(keep);
        if (keep) {
            StagedSplat st;
            st.g = make_float4(r.a.x, r.a.y, r.a.z * (-0.5f * kL2e), r.a.w * (-kL2e));
            st.q = make_float4(r.b.x * (-0.5f * kL2e), r.b.y, r.c.y, r.c.z);
            st.e = make_float4(r.c.w, __uint_as_float(idx - range.x + 1u), 0.0f, 0.0f);
            const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            s_spl[__popcll(bal & lt)] = st;
        }
        int count = __popcll(bal);
        if (count == 0) continue;
        if (lane < count) s_list[lane] = (uint16_t)(lane * sizeof(StagedSplat));
        if (count & 1) {
            if (lane == 0) s_list[count] = (uint16_t)(64 * sizeof(StagedSplat));
            ++count;
        }
        auto next2 = [&](int k) { return k + 2 < count ? k + 2 : count - 2; };
        StagedSplat a0 = fetch(s_list[0]), a1 = fetch(s_list[1]);
        for (int k = 0;;) {
            int kn = next2(k);
            const StagedSplat b0 = fetch(s_list[kn]), b1 = fetch(s_list[kn + 1]);
            composite(a0);
            composite(a1);
            k += 2;
            if (k >= count) break;
            kn = next2(k);
            a0 = fetch(s_list[kn]);
            a1 = fetch(s_list[kn + 1]);
            composite(b0);
            composite(b1);
            k += 2;
            if (k >= count) break;
        }
        if (!live_any()) break;
    }

    const int row = py - a.y0;
    const size_t plane = (size_t)a.rows_out * a.W;
    const float Ta = fabsf(T.x), Tb = fabsf(T.y);
    if (in_a) {
        const size_t pid = (size_t)row * a.W + pxa;
        if (a.final_T) a.final_T[pid] = Ta;
        if (a.n_contrib) a.n_contrib[pid] = last_a;
        a.out_color[pid] = C0.x + Ta * a.bg[0];
        a.out_color[plane + pid] = C1.x + Ta * a.bg[1];
        a.out_color[2 * plane + pid] = C2.x + Ta * a.bg[2];
    }
    if (in_b) {
        const size_t pid = (size_t)row * a.W + pxb;
        if (a.final_T) a.final_T[pid] = Tb;
        if (a.n_contrib) a.n_contrib[pid] = last_b;
        a.out_color[pid] = C0.y + Tb * a.bg[0];
        a.out_color[plane + pid] = C1.y + Tb * a.bg[1];
        a.out_color[2 * plane + pid] = C2.y + Tb * a.bg[2];
    }
}

// Fast arithmetic, packed: a 2-wave block per 16x16 tile; wave w owns rows 8w..8w+7 and each
// lane owns the two pixels (x, y) and (x + 8, y) of its row, so every per-pixel operation
// runs as one v_pk_* instruction on a float2 (CDNA4 reaches its fp32 rate only with packed
// math).  A wave iterates over the splats that touch either of its two 8x8 quadrants.

__global__ __launch_bounds__(128) void k_blend_fast2(const GsrBlendArgs a) {
    __shared__ StagedSplat s_spl[kBatch + 1];  // slot kBatch: opacity-0 pad (see k_blend)
    __shared__ uint8_t s_mask[kBatch];
    __shared__ uint16_t s_list[2][kBatch + 1];

    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t tx = blockIdx.x, ty_local = blockIdx.y, ty = a.row_begin + ty_local;
    const int tx0 = (int)tx * GSR_TILE_X, ty0 = (int)ty * GSR_TILE_Y;
    const int pxa = tx0 + (lane & 7), pxb = pxa + 8, py = ty0 + w * 8 + (lane >> 3);
    const bool in_a = pxa < a.W && py < a.H, in_b = pxb < a.W && py < a.H;
    const v2f pfx = {(float)pxa, (float)pxb};
    const float pfy = (float)py;
    if (tid == 0) {
        s_spl[kBatch].g = make_float4(0.f, 0.f, 0.f, 0.f);
        s_spl[kBatch].q = make_float4(0.f, 0.f, 0.f, 0.f);
        s_spl[kBatch].e = make_float4(0.f, 0.f, 0.f, 0.f);
    }

    const uint2 range = a.ranges[ty_local * a.grid_x + tx];
    // done carried in the sign of T, as in k_blend
    v2f T = {in_a ? 1.0f : -1.0f, in_b ? 1.0f : -1.0f};
    v2f C0 = {0.0f, 0.0f}, C1 = {0.0f, 0.0f}, C2 = {0.0f, 0.0f};
    uint32_t last_a = 0, last_b = 0;
    const float kL2e = 1.4426950408889634f;
    auto live_any = [&]() { return !(T.x <= 0.0f) || !(T.y <= 0.0f); };

    auto composite = [&](const StagedSplat &sp) {
        const v2f dx = (v2f)sp.g.x - pfx;
        const float dy = sp.g.y - pfy;
        const v2f ady = __builtin_elementwise_fma((v2f)sp.g.z, dx, (v2f)(sp.g.w * dy));
        const v2f p2 = __builtin_elementwise_fma(dx, ady, (v2f)(sp.q.x * dy * dy));
        v2f e;
        e.x = __builtin_amdgcn_exp2f(p2.x);
        e.y = __builtin_amdgcn_exp2f(p2.y);
        const v2f oe = (v2f)sp.q.y * e;
        v2f alpha;
        alpha.x = fminf(0.99f, oe.x);
        alpha.y = fminf(0.99f, oe.y);
        const v2f aT = alpha * T;
        const v2f test_T = T - aT;
        const bool vis_a = !(p2.x > 0.0f) && !(alpha.x < 1.0f / 255.0f);
        const bool vis_b = !(p2.y > 0.0f) && !(alpha.y < 1.0f / 255.0f);
        const bool lo_a = test_T.x < 0.0001f, lo_b = test_T.y < 0.0001f;
        const bool acc_a = vis_a && !lo_a, acc_b = vis_b && !lo_b;
        v2f wgt;
        wgt.x = acc_a ? aT.x : 0.0f;
        wgt.y = acc_b ? aT.y : 0.0f;
        C0 = __builtin_elementwise_fma((v2f)sp.q.z, wgt, C0);
        C1 = __builtin_elementwise_fma((v2f)sp.q.w, wgt, C1);
        C2 = __builtin_elementwise_fma((v2f)sp.e.x, wgt, C2);
        T.x = acc_a ? test_T.x : ((vis_a && lo_a) ? -fabsf(T.x) : T.x);
        T.y = acc_b ? test_T.y : ((vis_b && lo_b) ? -fabsf(T.y) : T.y);
        const uint32_t pos = __float_as_uint(sp.e.y);
        last_a = acc_a ? pos : last_a;
        last_b = acc_b ? pos : last_b;
    };
    const char *lds = reinterpret_cast<const char *>(s_spl);
    auto fetch = [&](uint32_t off) { return *reinterpret_cast<const StagedSplat *>(lds + off); };

    for (uint32_t start = range.x; start < range.y; start += kBatch) {
        if (__syncthreads_count(!live_any()) == 128) break;
        for (int t = tid; t < kBatch; t += 128) {
            const uint32_t idx = start + t;
            if (idx >= range.y) break;
            const SplatRecord r = a.records[(a.point_list[idx] & a.id_mask)];
            uint32_t m = 0xF;
            if (a.cull) {
                const float x = r.a.x, y = r.a.y, A = r.a.z, B = r.a.w, C = r.b.x;
                const float ex = r.b.z, ey = r.b.w, twoL = 2.0f * r.c.x;
                const float X0 = (float)tx0, Y0 = (float)ty0;
                m = (uint32_t)may_touch(x, y, A, B, C, ex, ey, twoL, X0, X0 + 7, Y0, Y0 + 7) |
                    ((uint32_t)may_touch(x, y, A, B, C, ex, ey, twoL, X0 + 8, X0 + 15, Y0, Y0 + 7) << 1) |
                    ((uint32_t)may_touch(x, y, A, B, C, ex, ey, twoL, X0, X0 + 7, Y0 + 8, Y0 + 15) << 2) |
                    ((uint32_t)may_touch(x, y, A, B, C, ex, ey, twoL, X0 + 8, X0 + 15, Y0 + 8, Y0 + 15) << 3);
            }
            StagedSplat st;
            st.g = make_float4(r.a.x, r.a.y, r.a.z * (-0.5f * kL2e), r.a.w * (-kL2e));
            st.q = make_float4(r.b.x * (-0.5f * kL2e), r.b.y, r.c.y, r.c.z);
            st.e = make_float4(r.c.w, __uint_as_float(idx - range.x + 1u), 0.0f, 0.0f);
            s_spl[t] = st;
            s_mask[t] = (uint8_t)m;
        }
        __syncthreads();
        const int n = (int)min((uint32_t)kBatch, range.y - start);

        int count = 0;
        for (int base = 0; base < n; base += 64) {
            const int j = base + lane;
            const bool keep = j < n && ((s_mask[j] >> (2 * w)) & 3u);
            const uint64_t bal = __ballot(keep);
            const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            if (keep)
                s_list[w][count + __popcll(bal & lt)] = (uint16_t)(j * sizeof(StagedSplat));
            count += __popcll(bal);
        }
        if (count & 1) {
            if (lane == 0) s_list[w][count] = (uint16_t)(kBatch * sizeof(StagedSplat));
            ++count;
        }
        if (count == 0 || __ballot(live_any()) == 0ull) continue;

        const uint16_t *list = s_list[w];
        auto next2 = [&](int k) { return k + 2 < count ? k + 2 : count - 2; };
        StagedSplat a0 = fetch(list[0]), a1 = fetch(list[1]);
        for (int k = 0;;) {
            int kn = next2(k);
            const StagedSplat b0 = fetch(list[kn]), b1 = fetch(list[kn + 1]);
            composite(a0);
            composite(a1);
            k += 2;
            if (k >= count) break;
            kn = next2(k);
            a0 = fetch(list[kn]);
            a1 = fetch(list[kn + 1]);
            composite(b0);
            composite(b1);
            k += 2;
            if (k >= count) break;
            if ((k & 28) == 0 && __ballot(live_any()) == 0ull) break;
        }
    }

    const int row = py - a.y0;
    const size_t plane = (size_t)a.rows_out * a.W;
    const float Ta = fabsf(T.x), Tb = fabsf(T.y);
    if (in_a) {
        const size_t pid = (size_t)row * a.W + pxa;
        if (a.final_T) a.final_T[pid] = Ta;
        if (a.n_contrib) a.n_contrib[pid] = last_a;
        a.out_color[pid] = C0.x + Ta * a.bg[0];
        a.out_color[plane + pid] = C1.x + Ta * a.bg[1];
        a.out_color[2 * plane + pid] = C2.x + Ta * a.bg[2];
    }
    if (in_b) {
        const size_t pid = (size_t)row * a.W + pxb;
        if (a.final_T) a.final_T[pid] = Tb;
        if (a.n_contrib) a.n_contrib[pid] = last_b;
        a.out_color[pid] = C0.y + Tb * a.bg[0];
        a.out_color[plane + pid] = C1.y + Tb * a.bg[1];
        a.out_color[2 * plane + pid] = C2.y + Tb * a.bg[2];
    }
}

}  // namespace

hipError_t gsr_launch_blend(const GsrBlendArgs &a, hipStream_t s) {
    if (a.rows_tiles == 0 || a.grid_x == 0) return hipSuccess;
    if (a.wave_quadrants && a.fast == 2) {
        const uint32_t n_work = 2u * a.grid_x * a.rows_tiles;
        const uint32_t g = a.xcd_group ? a.xcd_group * 8u : 8u;
        const uint32_t per_xcd = (n_work + g - 1) / g * g / 8u;
        hipLaunchKernelGGL(k_blend_h, dim3(8u * per_xcd), dim3(64), 0, s, a, n_work, per_xcd);
        return hipGetLastError();
    }
    if (a.wave_quadrants) {
        const uint32_t n_work = 4u * a.grid_x * a.rows_tiles;
        // grid: whole groups on every XCD (blocks past n_work exit)
        const uint32_t g = a.xcd_group ? a.xcd_group * 8u : 8u;
        const uint32_t per_xcd = (n_work + g - 1) / g * g / 8u;
        if (a.fast && a.lean && !a.n_contrib)
            hipLaunchKernelGGL((k_blend_q<true, true, false>), dim3(8u * per_xcd), dim3(64), 0, s,
                               a, n_work, per_xcd);
        else if (a.fast && a.lean)
            hipLaunchKernelGGL((k_blend_q<true, true>), dim3(8u * per_xcd), dim3(64), 0, s, a,
                               n_work, per_xcd);
        else if (a.fast)
            hipLaunchKernelGGL((k_blend_q<true>), dim3(8u * per_xcd), dim3(64), 0, s, a, n_work,
                               per_xcd);
        else
            hipLaunchKernelGGL((k_blend_q<false>), dim3(8u * per_xcd), dim3(64), 0, s, a, n_work,
                               per_xcd);
        return hipGetLastError();
    }
    const dim3 grid(a.grid_x, a.rows_tiles);
    if (a.fast == 2)
        hipLaunchKernelGGL(k_blend_fast2, grid, dim3(128), 0, s, a);
    else if (a.fast && a.stamps)
        hipLaunchKernelGGL((k_blend<true, true>), grid, dim3(256), 0, s, a);
    else if (a.fast)
        hipLaunchKernelGGL((k_blend<true>), grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((k_blend<false>), grid, dim3(256), 0, s, a);
    return hipGetLastError();
}
