// radix_sort.hip -- stable LSD radix sort of (uint32 key, uint32 value) pairs for gfx950.
//
// Replaces the cub::DeviceRadixSort::SortPairs call of upstream rasterizer_impl.cu (the
// rasterizer's binning sort) and the torch/cupy/numpy argsort of the viewer's sort backend
// (renderer_ogl.py:17, :34, :51).  Used twice per frame: Gaussians by depth (32-bit keys)
// and (Gaussian, tile) pairs by tile id (ceil(log2 T) bits).
//
// One pass per 8-bit digit, three kernels per pass (reduce-then-scan):
//   upsweep   -- per-tile digit histogram (tile = 4096 elements = 256 threads x 16);
//   scan      -- per digit, exclusive scan of its histogram column across tiles;
//   downsweep -- wave-ballot ranking: each wave resolves the lanes that share its digit with
//                log2(radix) ballots, keeps per-wave running counts in LDS, the block turns
//                them into tile-local ranks, scatters pairs into LDS in digit order and writes
//                each digit's run out contiguously (coalesced stores).
// Every element is processed in increasing index order within its tile and tiles are
// concatenated in order, so each pass -- and the sort -- is stable.
#include "gsr_internal.h"

using namespace gsr;

namespace {

constexpr int kBlock = 256;
constexpr int kItems = 16;
constexpr int kTile = kBlock * kItems;  // 4096
constexpr int kRadix = 256;

__global__ __launch_bounds__(kBlock) void k_rs_upsweep(const uint32_t *__restrict__ keys,
                                                       int64_t n, int shift, uint32_t mask,
                                                       uint32_t *__restrict__ hist, int64_t nb) {
    __shared__ uint32_t s_hist[4][kRadix];
    const int tid = threadIdx.x, w = tid >> 6;
    for (int i = tid; i < 4 * kRadix; i += kBlock) (&s_hist[0][0])[i] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kTile;
    if (base + kTile <= n) {
        const uint4 *k4 = reinterpret_cast<const uint4 *>(keys + base);
#pragma unroll
        for (int j = 0; j < kItems / 4; ++j) {
            const uint4 q = k4[j * kBlock + tid];
            atomicAdd(&s_hist[w][(q.x >> shift) & mask], 1u);
            atomicAdd(&s_hist[w][(q.y >> shift) & mask], 1u);
            atomicAdd(&s_hist[w][(q.z >> shift) & mask], 1u);
            atomicAdd(&s_hist[w][(q.w >> shift) & mask], 1u);
        }
    } else {
        for (int64_t e = base + tid; e < n; e += kBlock)
            atomicAdd(&s_hist[w][(keys[e] >> shift) & mask], 1u);
    }
    __syncthreads();
    const uint32_t c = s_hist[0][tid] + s_hist[1][tid] + s_hist[2][tid] + s_hist[3][tid];
    hist[(int64_t)tid * nb + blockIdx.x] = c;
}

// One block per digit: exclusive scan of hist[d][0..nb) in place, total -> digit_total[d].
__global__ __launch_bounds__(kBlock) void k_rs_scan(uint32_t *__restrict__ hist, int64_t nb,
                                                    uint32_t *__restrict__ digit_total) {
    __shared__ uint32_t s_tmp[4];
    uint32_t *h = hist + (int64_t)blockIdx.x * nb;
    uint32_t carry = 0;
    for (int64_t start = 0; start < nb; start += kBlock * 4) {
        uint32_t v[4], sum = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t e = start + threadIdx.x * 4 + i;
            v[i] = e < nb ? h[e] : 0u;
            sum += v[i];
        }
        uint32_t total;
        uint32_t pre = block256_exclusive_scan(sum, s_tmp, total) + carry;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t e = start + threadIdx.x * 4 + i;
            if (e < nb) h[e] = pre;
            pre += v[i];
        }
        carry += total;
    }
    if (threadIdx.x == 0) digit_total[blockIdx.x] = carry;
}

__global__ __launch_bounds__(kBlock) void k_rs_downsweep(
    const uint32_t *__restrict__ keys_in, const uint32_t *__restrict__ vals_in,
    uint32_t *__restrict__ keys_out, uint32_t *__restrict__ vals_out, int64_t n, int shift,
    int nbits, const uint32_t *__restrict__ hist, const uint32_t *__restrict__ digit_total,
    int64_t nb) {
    __shared__ uint32_t s_keys[kTile];
    __shared__ uint32_t s_vals[kTile];
    __shared__ uint32_t s_wcnt[4][kRadix];
    __shared__ uint32_t s_delta[kRadix];
    __shared__ uint32_t s_tmp[8];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t mask = (1u << nbits) - 1u;
    for (int i = tid; i < 4 * kRadix; i += kBlock) (&s_wcnt[0][0])[i] = 0;
    __syncthreads();

    const int64_t base = (int64_t)blockIdx.x * kTile;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t k[kItems], v[kItems], rank[kItems];
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const int64_t e = base + w * (kTile / 4) + j * 64 + lane;
        const bool valid = e < n;
        k[j] = valid ? keys_in[e] : 0xFFFFFFFFu;  // tail -> largest digit, after every real key
        v[j] = valid ? vals_in[e] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const uint32_t d = (k[j] >> shift) & mask;
        uint64_t m = ~0ull;
        for (int b = 0; b < nbits; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t bal = __ballot(bit);
            m &= bit ? bal : ~bal;
        }
        const uint32_t prior = s_wcnt[w][d];
        rank[j] = prior + (uint32_t)__popcll(m & lt_mask);
        if (lane == 63 - __clzll(m)) s_wcnt[w][d] = prior + (uint32_t)__popcll(m);
    }
    __syncthreads();

    // Per digit (thread = digit): wave offsets, tile-local start, global destination.
    {
        const int d = tid;
        const uint32_t c0 = s_wcnt[0][d], c1 = s_wcnt[1][d], c2 = s_wcnt[2][d], c3 = s_wcnt[3][d];
        uint32_t tile_total, all_total;
        const uint32_t local_start = block256_exclusive_scan(c0 + c1 + c2 + c3, s_tmp, tile_total);
        const uint32_t digit_start = block256_exclusive_scan(digit_total[d], s_tmp + 4, all_total);
        const uint32_t global_start = digit_start + hist[(int64_t)d * nb + blockIdx.x];
        s_delta[d] = global_start - local_start;
        s_wcnt[0][d] = local_start;
        s_wcnt[1][d] = local_start + c0;
        s_wcnt[2][d] = local_start + c0 + c1;
        s_wcnt[3][d] = local_start + c0 + c1 + c2;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const uint32_t d = (k[j] >> shift) & mask;
        const uint32_t pos = s_wcnt[w][d] + rank[j];
        s_keys[pos] = k[j];
        s_vals[pos] = v[j];
    }
    __syncthreads();
    const int64_t rem = n - base;
    const int valid = rem < kTile ? (int)rem : kTile;  // tail elements sit in the last slots
    for (int i = tid; i < valid; i += kBlock) {
        const uint32_t kk = s_keys[i];
        const uint32_t g = s_delta[(kk >> shift) & mask] + (uint32_t)i;
        keys_out[g] = kk;
        vals_out[g] = s_vals[i];
    }
}

}  // namespace

int64_t gsr_radix_hist_words(int64_t n) {
    const int64_t nb = (n + kTile - 1) / kTile;
    return (nb < 1 ? 1 : nb) * kRadix;
}

hipError_t gsr_radix_sort_pairs(uint32_t **keys, uint32_t **vals, uint32_t **keys_alt,
                                uint32_t **vals_alt, int64_t n, int begin_bit, int end_bit,
                                uint32_t *hist, uint32_t *digit_total, hipStream_t s) {
    if (n <= 1) return hipSuccess;
    const int64_t nb = (n + kTile - 1) / kTile;
    for (int shift = begin_bit; shift < end_bit; shift += 8) {
        const int nbits = (end_bit - shift) < 8 ? (end_bit - shift) : 8;
        const uint32_t mask = (1u << nbits) - 1u;
        hipLaunchKernelGGL(k_rs_upsweep, dim3((unsigned)nb), dim3(kBlock), 0, s, *keys, n, shift,
                           mask, hist, nb);
        hipLaunchKernelGGL(k_rs_scan, dim3(kRadix), dim3(kBlock), 0, s, hist, nb, digit_total);
        hipLaunchKernelGGL(k_rs_downsweep, dim3((unsigned)nb), dim3(kBlock), 0, s, *keys, *vals,
                           *keys_alt, *vals_alt, n, shift, nbits, hist, digit_total, nb);
        uint32_t *t = *keys;
        *keys = *keys_alt;
        *keys_alt = t;
        t = *vals;
        *vals = *vals_alt;
        *vals_alt = t;
    }
    return hipGetLastError();
}
