// radix_sort.hip -- stable LSD radix sort of (uint32 key, uint32 value) pairs for gfx950.
//
// Replaces the cub::DeviceRadixSort::SortPairs call of upstream rasterizer_impl.cu (the
// rasterizer's binning sort) and the torch/cupy/numpy argsort of the viewer's sort backend
// (renderer_ogl.py:17, :34, :51).  Used twice per frame: Gaussians by depth (32-bit keys)
// and (Gaussian, tile) pairs by tile id (ceil(log2 T) bits).
//
// Reduce-then-scan (gsr_radix_sort_pairs): one pass per 8-bit digit, three kernels per pass:
//   upsweep   -- per-tile digit histogram (tile = 4096 elements = 256 threads x 16);
//   scan      -- per digit, exclusive scan of its histogram column across tiles;
//   downsweep -- wave-ballot ranking: each wave resolves the lanes that share its digit with
//                log2(radix) ballots, keeps per-wave running counts in LDS, the block turns
//                them into tile-local ranks, scatters pairs into LDS in digit order and writes
//                each digit's run out contiguously (coalesced stores).
// Every element is processed in increasing index order within its tile and tiles are
// concatenated in order, so each pass -- and the sort -- is stable.
#include <algorithm>

#include "radix_tile.h"

using namespace gsr;

namespace {

constexpr int kBlock = 256;
constexpr int kRadix = kRadixBins;

// Element count of a pass: n_host, or *d_n when set (the column-first binning's scan learns
// its live block count from the depth sort's kept count on the device).  Grids and the hist
// column stride stay sized for n_host.
struct RsCount {
    int64_t n_host;
    const uint32_t *d_n;
};

// Reduce-then-scan over tiles of kW waves x kIt keys per lane (8 x 8 = 4096 keys: the fastest
// shape measured for the K-sized tile sort).  The histogram is digit-major,
// hist[d * stride + tile] (the scan reads a digit's column contiguously), stride = the tile count
// rounded up to a multiple of 4.  A block counts kTiles consecutive tiles and stores each
// digit's kTiles counts as one word of 4 kTiles bytes: with one tile per block every 4-B store
// lands on its own line (the 4K frame's upsweep wrote 278 MB for a 7 MB histogram), so large
// passes take 4 tiles per block and write 16-B words (gsr_radix_hist_words pads the stride).
// The element count of a pass whose count lives on the device (frame graphs): *d_n, or 0 when
// it exceeds the capacity n_cap the launch was sized for (nothing is sorted; the host re-renders
// the frame).  d_n NULL: n_cap itself.
__device__ __forceinline__ int64_t live_count(const uint32_t *d_n, int64_t n_cap) {
    if (!d_n) return n_cap;
    const int64_t n = (int64_t)*d_n;
    return n <= n_cap ? n : 0;
}

template <int kW, int kIt, int kTiles>
__global__ __launch_bounds__(kW * 64) void k_rs_upsweep(const uint32_t *__restrict__ keys,
                                                        int64_t n_cap, int shift, uint32_t mask,
                                                        uint32_t *__restrict__ hist,
                                                        int64_t stride,
                                                        const uint32_t *__restrict__ d_n) {
    constexpr int kThreads = kW * 64, kT = kThreads * kIt;
    const int64_t n = live_count(d_n, n_cap);
    static_assert(kIt % 4 == 0, "full tiles are read as uint4");
    static_assert(kW >= 4, "the digit scans take one thread per digit (256)");
    static_assert(kTiles == 1 || kTiles == 4, "one tile or a 16-B word of four");
    __shared__ uint32_t s_hist[kW][kRadix];
    const int tid = threadIdx.x, w = tid >> 6;
    const int64_t tile0 = (int64_t)xcd_run_block(blockIdx.x) * kTiles;
    if (tile0 * kT >= n) return;  // whole block (the scan reads columns [0, ceil(n / kT)) only)
    uint32_t cnt[kTiles];
    for (int t = 0; t < kTiles; ++t) {
        const int64_t base = (tile0 + t) * kT;
        for (int i = tid; i < kW * kRadix; i += kThreads) (&s_hist[0][0])[i] = 0;
        __syncthreads();
        auto add = [&](uint32_t key) { atomicAdd(&s_hist[w][(key >> shift) & mask], 1u); };
        if (base + kT <= n) {
            const uint4 *k4 = reinterpret_cast<const uint4 *>(keys + base);
#pragma unroll
            for (int j = 0; j < kIt / 4; ++j) {
                const uint4 q = k4[j * kThreads + tid];
                add(q.x);
                add(q.y);
                add(q.z);
                add(q.w);
            }
        } else {
            for (int64_t e = base + tid; e < n; e += kThreads) add(keys[e]);
        }
        __syncthreads();
        uint32_t c = 0;
        if (tid < kRadix) {
#pragma unroll
            for (int i = 0; i < kW; ++i) c += s_hist[i][tid];
        }
        cnt[t] = c;
        __syncthreads();  // s_hist is zeroed again for the next tile
    }
    if (tid < kRadix) {
        if (kTiles == 4)
            *reinterpret_cast<uint4 *>(hist + (int64_t)tid * stride + tile0) =
                make_uint4(cnt[0], cnt[1 % kTiles], cnt[2 % kTiles], cnt[3 % kTiles]);
        else
            hist[(int64_t)tid * stride + tile0] = cnt[0];
    }
}

// One block per digit: exclusive scan of hist[d][0..ceil(n / kT)) (column stride `stride`) in
// place, total -> digit_total[d].
__global__ __launch_bounds__(kBlock) void k_rs_scan(uint32_t *__restrict__ hist, int64_t stride,
                                                    uint32_t *__restrict__ digit_total,
                                                    const RsCount cnt, int64_t kT) {
    __shared__ uint32_t s_tmp[4];
    const int64_t nb_act =
        cnt.d_n ? min(((int64_t)*cnt.d_n + kT - 1) / kT, cnt.n_host) : cnt.n_host;
    uint32_t *h = hist + (int64_t)blockIdx.x * stride;
    uint32_t carry = 0;
    const bool vec = (stride & 3) == 0;  // 16-B aligned columns: whole words of 4 tiles
    for (int64_t start = 0; start < nb_act; start += kBlock * 4) {
        uint32_t v[4], sum = 0;
        const int64_t e0 = start + threadIdx.x * 4;
        if (vec && e0 + 3 < nb_act) {
            const uint4 q = *reinterpret_cast<const uint4 *>(h + e0);
            v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = e0 + i < nb_act ? h[e0 + i] : 0u;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) sum += v[i];
        uint32_t total;
        uint32_t pre = block256_exclusive_scan(sum, s_tmp, total) + carry;
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = pre, pre += v[i];
        if (vec && e0 + 3 < nb_act) {
            *reinterpret_cast<uint4 *>(h + e0) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (e0 + i < nb_act) h[e0 + i] = o[i];
        }
        carry += total;
    }
    if (threadIdx.x == 0) digit_total[blockIdx.x] = carry;
}

// kVals = false: keys only (vals_in / vals_out unused) -- no LDS for values, so more blocks
// share a CU.
template <int kW, int kIt, bool kVals>
__global__ __launch_bounds__(kW * 64) void k_rs_downsweep(
    const uint32_t *__restrict__ keys_in, const uint32_t *__restrict__ vals_in,
    uint32_t *__restrict__ keys_out, uint32_t *__restrict__ vals_out, int64_t n_cap,
    int shift, int nbits, const uint32_t *__restrict__ hist,
    const uint32_t *__restrict__ digit_total, int64_t nb, const uint32_t *__restrict__ d_n) {
    constexpr int kT = kW * 64 * kIt;
    const int64_t n = live_count(d_n, n_cap);
    __shared__ uint32_t s_keys[kT];
    __shared__ uint32_t s_vals[kVals ? kT : 1];
    __shared__ RadixTileSmem<kW, kIt> sm;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t tile = xcd_run_block(blockIdx.x);
    const int64_t base = (int64_t)tile * kT;
    if (base >= n) return;  // whole block
    uint32_t k[kIt], v[kIt];
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
        const int64_t e = base + w * (kT / kW) + j * 64 + lane;
        const bool valid = e < n;
        k[j] = valid ? keys_in[e] : 0xFFFFFFFFu;  // tail -> largest digit, after every real key
        v[j] = (kVals && valid) ? vals_in[e] : 0u;
    }
    const int64_t rem = n - base;
    radix_tile_scatter<kW, kIt>(k, v, rem < kT ? (int)rem : kT, shift, nbits, hist, nb,
                                       tile, digit_total, keys_out,
                                       kVals ? vals_out : nullptr, sm, s_keys, s_vals);
}

}  // namespace

GsrRadixPlan gsr_radix_plan(int begin_bit, int end_bit) {
    GsrRadixPlan p{};
    const int bits = end_bit - begin_bit;
    p.n = bits <= 0 ? 0 : (bits + 7) / 8;
    int shift = begin_bit;
    for (int i = 0; i < p.n; ++i) {
        const int nb = bits / p.n + (i < bits % p.n ? 1 : 0);
        p.shift[i] = shift;
        p.nbits[i] = nb;
        p.mask[i] = (1u << nb) - 1u;
        shift += nb;
    }
    return p;
}

hipError_t gsr_launch_digit_scan(uint32_t *hist, int64_t nb, uint32_t *digit_total,
                                 hipStream_t s) {
    hipLaunchKernelGGL(k_rs_scan, dim3(kRadix), dim3(kBlock), 0, s, hist, nb, digit_total,
                       RsCount{nb, nullptr}, (int64_t)1);  // (stride = column count here)
    return hipGetLastError();
}

// k_rs_scan over nb columns whose live length is ceil(*d_n / tile) (column-first binning).
hipError_t gsr_launch_digit_scan_n(uint32_t *hist, int64_t nb, uint32_t *digit_total,
                                   const uint32_t *d_n, int64_t tile, hipStream_t s) {
    hipLaunchKernelGGL(k_rs_scan, dim3(kRadix), dim3(kBlock), 0, s, hist, nb, digit_total,
                       RsCount{nb, d_n}, tile);
    return hipGetLastError();
}

namespace {
// sort tile: 8 waves x 8 keys per lane (4096 keys; 8 x 16 and 16 x 16 measured no faster at 4K
// and slower at C3, profiles/r04o_ab_rs_tile.txt)
constexpr int kSW = 8, kSIt = 8;
constexpr int64_t kST = (int64_t)kSW * 64 * kSIt;
}  // namespace

// the histogram's column stride: tiles rounded up to a multiple of 4 (the 16-B upsweep words)
static int64_t hist_stride(int64_t nb) { return (nb + 3) & ~(int64_t)3; }
// passes of at least this many tiles count 4 tiles per upsweep block (16-B histogram words);
// below it the grid would leave CUs idle (C3: 1,385 tiles)
constexpr int64_t kQuadTiles = 4096;

int64_t gsr_radix_hist_words(int64_t n) {
    const int64_t nb = (n + kST - 1) / kST;
    return (nb < 1 ? 4 : hist_stride(nb)) * kRadix;
}

// One pass: upsweep, scan, downsweep.  v == nullptr: keys only.  d_n: the count on the device
// (n the capacity; live_count).
static void rts_pass(const uint32_t *k, const uint32_t *v, uint32_t *ko, uint32_t *vo, int64_t n,
                     int shift, int nbits, uint32_t *hist, uint32_t *digit_total, hipStream_t s,
                     const uint32_t *d_n = nullptr) {
    const int64_t nb = (n + kST - 1) / kST;  // tiles: the downsweep's grid
    if (nb == 0) return;
    const int64_t stride = hist_stride(nb);
    const uint32_t mask = (1u << nbits) - 1u;
    if (nb >= kQuadTiles)
        hipLaunchKernelGGL((k_rs_upsweep<kSW, kSIt, 4>),
                           dim3(xcd_run_grid((nb + 3) / 4)), dim3(kSW * 64), 0, s,
                           k, n, shift, mask, hist, stride, d_n);
    else
        hipLaunchKernelGGL((k_rs_upsweep<kSW, kSIt, 1>), dim3(xcd_run_grid(nb)),
                           dim3(kSW * 64), 0, s, k, n, shift, mask, hist, stride, d_n);
    // (with d_n, an over-capacity count scans stale counts, in bounds; the downsweep then
    // sorts nothing)
    hipLaunchKernelGGL(k_rs_scan, dim3(kRadix), dim3(kBlock), 0, s, hist, stride, digit_total,
                       RsCount{nb, d_n}, kST);
    const dim3 down_grid(xcd_run_grid(nb));
    if (v)
        hipLaunchKernelGGL((k_rs_downsweep<kSW, kSIt, true>), down_grid, dim3(kSW * 64), 0, s, k,
                           v, ko, vo, n, shift, nbits, hist, digit_total, stride, d_n);
    else
        hipLaunchKernelGGL((k_rs_downsweep<kSW, kSIt, false>), down_grid, dim3(kSW * 64), 0, s,
                           k, v, ko, vo, n, shift, nbits, hist, digit_total, stride, d_n);
}

hipError_t gsr_radix_sort_pairs(uint32_t **keys, uint32_t **vals, uint32_t **keys_alt,
                                uint32_t **vals_alt, int64_t n, int begin_bit, int end_bit,
                                uint32_t *hist, uint32_t *digit_total, hipStream_t s,
                                int first_pass) {
    if (n <= 1) return hipSuccess;
    const GsrRadixPlan plan = gsr_radix_plan(begin_bit, end_bit);
    for (int p = first_pass; p < plan.n; ++p) {
        rts_pass(*keys, *vals, *keys_alt, *vals_alt, n, plan.shift[p], plan.nbits[p], hist,
                 digit_total, s);
        std::swap(*keys, *keys_alt);
        std::swap(*vals, *vals_alt);
    }
    return hipGetLastError();
}

hipError_t gsr_radix_sort_keys(uint32_t **keys, uint32_t **keys_alt, int64_t n, int begin_bit,
                               int end_bit, uint32_t *hist, uint32_t *digit_total, hipStream_t s,
                               const uint32_t *d_n) {
    if (n <= 1 && !d_n) return hipSuccess;
    const GsrRadixPlan plan = gsr_radix_plan(begin_bit, end_bit);
    for (int p = 0; p < plan.n; ++p) {
        rts_pass(*keys, nullptr, *keys_alt, nullptr, n, plan.shift[p], plan.nbits[p], hist,
                 digit_total, s, d_n);
        std::swap(*keys, *keys_alt);
    }
    return hipGetLastError();
}
