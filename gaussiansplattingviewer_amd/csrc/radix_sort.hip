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
// shape measured for the K-sized tile sort).  nb = hist column stride (tiles of the
// host's upper bound).
template <int kW, int kIt>
__global__ __launch_bounds__(kW * 64) void k_rs_upsweep(const uint32_t *__restrict__ keys,
                                                        int64_t n, int shift, uint32_t mask,
                                                        uint32_t *__restrict__ hist, int64_t nb) {
    constexpr int kThreads = kW * 64, kT = kThreads * kIt;
    static_assert(kIt % 4 == 0, "full tiles are read as uint4");
    static_assert(kW >= 4, "the digit scans take one thread per digit (256)");
    __shared__ uint32_t s_hist[kW][kRadix];
    const int tid = threadIdx.x, w = tid >> 6;
    const int64_t base = (int64_t)blockIdx.x * kT;
    if (base >= n) return;  // whole block (the scan reads columns [0, ceil(n / kT)) only)
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
    if (tid < kRadix) {
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < kW; ++i) c += s_hist[i][tid];
        hist[(int64_t)tid * nb + blockIdx.x] = c;
    }
}

// One block per digit: exclusive scan of hist[d][0..ceil(n / kT)) (column stride nb) in
// place, total -> digit_total[d].
__global__ __launch_bounds__(kBlock) void k_rs_scan(uint32_t *__restrict__ hist, int64_t nb,
                                                    uint32_t *__restrict__ digit_total,
                                                    const RsCount cnt, int64_t kT) {
    __shared__ uint32_t s_tmp[4];
    const int64_t nb_act = cnt.d_n ? ((int64_t)*cnt.d_n + kT - 1) / kT : nb;
    uint32_t *h = hist + (int64_t)blockIdx.x * nb;
    uint32_t carry = 0;
    for (int64_t start = 0; start < nb_act; start += kBlock * 4) {
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t e = start + threadIdx.x * 4 + i;
            v[i] = e < nb_act ? h[e] : 0u;
            sum += v[i];
        }
        uint32_t total;
        uint32_t pre = block256_exclusive_scan(sum, s_tmp, total) + carry;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t e = start + threadIdx.x * 4 + i;
            if (e < nb_act) h[e] = pre;
            pre += v[i];
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
    uint32_t *__restrict__ keys_out, uint32_t *__restrict__ vals_out, int64_t n,
    int shift, int nbits, const uint32_t *__restrict__ hist,
    const uint32_t *__restrict__ digit_total, int64_t nb) {
    constexpr int kT = kW * 64 * kIt;
    __shared__ uint32_t s_keys[kT];
    __shared__ uint32_t s_vals[kVals ? kT : 1];
    __shared__ RadixTileSmem<kW, kIt> sm;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t base = (int64_t)blockIdx.x * kT;
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
                                       blockIdx.x, digit_total, keys_out,
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
                       RsCount{nb, nullptr}, (int64_t)1);
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
constexpr int kSW = 8, kSIt = 8;  // sort tile: 8 waves x 8 keys per lane
constexpr int64_t kST = (int64_t)kSW * 64 * kSIt;
}  // namespace

int64_t gsr_radix_hist_words(int64_t n) {
    const int64_t nb = (n + kST - 1) / kST;
    return (nb < 1 ? 1 : nb) * kRadix;
}

// One pass: upsweep, scan, downsweep.  v == nullptr: keys only.
static void rts_pass(const uint32_t *k, const uint32_t *v, uint32_t *ko, uint32_t *vo, int64_t n,
                     int shift, int nbits, uint32_t *hist, uint32_t *digit_total, hipStream_t s) {
    const int64_t nb = (n + kST - 1) / kST;  // grid and hist column stride
    if (nb == 0) return;
    const uint32_t mask = (1u << nbits) - 1u;
    hipLaunchKernelGGL((k_rs_upsweep<kSW, kSIt>), dim3((unsigned)nb), dim3(kSW * 64), 0, s, k, n,
                       shift, mask, hist, nb);
    hipLaunchKernelGGL(k_rs_scan, dim3(kRadix), dim3(kBlock), 0, s, hist, nb, digit_total,
                       RsCount{nb, nullptr}, kST);
    if (v)
        hipLaunchKernelGGL((k_rs_downsweep<kSW, kSIt, true>), dim3((unsigned)nb), dim3(kSW * 64), 0,
                           s, k, v, ko, vo, n, shift, nbits, hist, digit_total, nb);
    else
        hipLaunchKernelGGL((k_rs_downsweep<kSW, kSIt, false>), dim3((unsigned)nb), dim3(kSW * 64),
                           0, s, k, v, ko, vo, n, shift, nbits, hist, digit_total, nb);
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
                               int end_bit, uint32_t *hist, uint32_t *digit_total, hipStream_t s) {
    if (n <= 1) return hipSuccess;
    const GsrRadixPlan plan = gsr_radix_plan(begin_bit, end_bit);
    for (int p = 0; p < plan.n; ++p) {
        rts_pass(*keys, nullptr, *keys_alt, nullptr, n, plan.shift[p], plan.nbits[p], hist,
                 digit_total, s);
        std::swap(*keys, *keys_alt);
    }
    return hipGetLastError();
}
