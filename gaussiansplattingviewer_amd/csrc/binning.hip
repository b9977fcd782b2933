// binning.hip -- tile binning for gfx950: offsets scan, pair duplication, tile ranges.
//
// Replaces upstream rasterizer_impl.cu  cub::DeviceScan::InclusiveSum(tiles_touched) +
// duplicateWithKeys + identifyTileRanges.  The design difference (documented in DESIGN.md):
// upstream builds 64-bit (tile << 32 | depth) keys in Gaussian-index order and radix-sorts
// K of them over 32 + log2(T) bits.  Here the Gaussians are first sorted by depth (P keys,
// stable), the pairs are emitted in that order, and a stable sort on the tile id alone
// (log2(T) bits) finishes the job.  Within a tile the result is ordered by depth and then
// by Gaussian index, exactly as upstream's stable 64-bit sort orders it, so point lists and
// ranges are bit-identical while the K-sized sort moves 8-B pairs over 2 passes instead of
// 12-B pairs over 6.
#include "gsr_internal.h"

using namespace gsr;

namespace {

constexpr int kBlock = 256;
constexpr int kItems = 4;
constexpr int kTile = kBlock * kItems;  // 1024 depth-sorted Gaussians per scan block
constexpr uint32_t kChunk = 2048;        // output pairs per duplicate block

// Pass 1 of the scan: per-block sum of the strip tile counts, gathered in depth order.
__global__ __launch_bounds__(kBlock) void k_scan_reduce(const uint32_t *__restrict__ perm,
                                                        const uint32_t *__restrict__ strip_tiles,
                                                        int64_t n, uint32_t *__restrict__ partials) {
    __shared__ uint32_t s_tmp[4];
    const int64_t base = (int64_t)blockIdx.x * kTile;
    uint32_t sum = 0;
#pragma unroll 4
    for (int j = 0; j < kItems; ++j) {
        const int64_t e = base + j * kBlock + threadIdx.x;
        if (e < n) sum += strip_tiles[perm[e]];
    }
    uint32_t total;
    block256_exclusive_scan(sum, s_tmp, total);
    if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

// Pass 2: single block, exclusive scan of the block partials; K -> *total (64-bit, so an
// overflow of the 32-bit pair index is detected on the host).
__global__ __launch_bounds__(kBlock) void k_scan_partials(uint32_t *__restrict__ partials,
                                                          int64_t nb, uint64_t *__restrict__ total) {
    __shared__ uint32_t s_tmp[4];
    uint64_t carry = 0;
    for (int64_t start = 0; start < nb; start += kBlock) {
        const int64_t e = start + threadIdx.x;
        const uint32_t v = e < nb ? partials[e] : 0u;
        uint32_t t;
        const uint32_t pre = block256_exclusive_scan(v, s_tmp, t);
        if (e < nb) partials[e] = (uint32_t)(carry + pre);
        carry += t;
    }
    if (threadIdx.x == 0) *total = carry;
}

// Pass 3: exclusive offsets of the depth-sorted Gaussians (offsets[e]) and, for every chunk of
// kChunk output pairs, the first Gaussian whose pairs reach into it (chunk_first[c]);
// chunk_first[n_chunks] = one past the last Gaussian with pairs.  Gaussians without pairs in
// the strip carry the sentinel depth key, so they all sit after the last non-empty one.
__global__ __launch_bounds__(kBlock) void k_scan_down(const uint32_t *__restrict__ perm,
                                                      const uint32_t *__restrict__ strip_tiles,
                                                      const uint32_t *__restrict__ partials,
                                                      int64_t n, const uint64_t *__restrict__ total,
                                                      uint32_t *__restrict__ offsets,
                                                      uint32_t *__restrict__ chunk_first) {
    __shared__ uint32_t s_tmp[4];
    const int tid = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)tid * kItems;
    uint32_t cnt[kItems], sum = 0;
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const int64_t e = base + j;
        cnt[j] = e < n ? strip_tiles[perm[e]] : 0u;
        sum += cnt[j];
    }
    uint32_t blk_total;
    uint32_t off = block256_exclusive_scan(sum, s_tmp, blk_total) + partials[blockIdx.x];
    const uint32_t K = (uint32_t)*total;
    const uint32_t n_chunks = (K + kChunk - 1) / kChunk;
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const int64_t e = base + j;
        if (e >= n) break;
        offsets[e] = off;
        if (cnt[j]) {
            for (uint32_t c = (off + kChunk - 1) / kChunk; c * kChunk < off + cnt[j]; ++c)
                chunk_first[c] = (uint32_t)e;
            if (off + cnt[j] == K) chunk_first[n_chunks] = (uint32_t)e + 1u;
        }
        off += cnt[j];
    }
}

// Pass 4, upstream duplicateWithKeys, load-balanced by output: block c writes pairs
// [c*kChunk, min(K, (c+1)*kChunk)) -- coalesced stores -- as (strip-local tile id, Gaussian
// id), row-major over each Gaussian's rect like upstream.  The Gaussians overlapping the
// chunk are staged in LDS; each output finds its owner by binary search over their offsets.
__global__ __launch_bounds__(kBlock) void k_duplicate(
    const uint32_t *__restrict__ perm, const uint32_t *__restrict__ offsets,
    const uint32_t *__restrict__ chunk_first, uint32_t K, uint32_t n_chunks,
    const SplatRecord *__restrict__ records, const int32_t *__restrict__ radii, uint32_t gx,
    uint32_t gy, uint32_t row_begin,
    uint32_t *__restrict__ tile_keys, uint32_t *__restrict__ tile_vals, const GsrRadixPlan plan,
    uint32_t *__restrict__ ghist) {
    __shared__ uint32_t s_hist[GSR_RADIX_MAX_PASSES][256];  // digit counts of the tile sort
    __shared__ uint32_t s_off[kChunk + 1];
    __shared__ uint32_t s_id[kChunk + 1];
    __shared__ uint32_t s_x0w[kChunk + 1];   // rect x0 | width << 16
    __shared__ uint32_t s_row0[kChunk + 1];  // first strip-local tile row * gx
    const int tid = threadIdx.x;
    const uint32_t c = blockIdx.x;
    const uint32_t e_end_all = chunk_first[n_chunks];
    const uint32_t e0 = chunk_first[c];
    const uint32_t e1 = (c + 1 < n_chunks) ? min(chunk_first[c + 1] + 1u, e_end_all) : e_end_all;
    const int ne = (int)(e1 - e0);  // <= kChunk + 1: every staged Gaussian owns >= 1 pair
    for (int i = tid; i < GSR_RADIX_MAX_PASSES * 256; i += kBlock) (&s_hist[0][0])[i] = 0;
    for (int i = tid; i < ne; i += kBlock) {
        const uint32_t id = perm[e0 + i];
        const float4 ra = records[id].a;
        const Rect rc = get_rect(ra.x, ra.y, radii[id], gx, gy);
        s_off[i] = offsets[e0 + i];
        s_id[i] = id;
        s_x0w[i] = rc.x0 | ((rc.x1 - rc.x0) << 16);
        s_row0[i] = (max(rc.y0, row_begin) - row_begin) * gx;
    }
    __syncthreads();
    const uint32_t o_end = min(K, (c + 1) * kChunk);
    for (uint32_t o = c * kChunk + tid; o < o_end; o += kBlock) {
        int lo = 0, hi = ne - 1;  // last staged Gaussian whose offset <= o
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_off[mid] <= o) lo = mid;
            else hi = mid - 1;
        }
        const uint32_t local = o - s_off[lo];
        const uint32_t x0w = s_x0w[lo];
        const uint32_t width = x0w >> 16;
        const uint32_t row = local / width;
        const uint32_t col = local - row * width;
        const uint32_t key = s_row0[lo] + row * gx + (x0w & 0xFFFFu) + col;
        tile_keys[o] = key;
        tile_vals[o] = s_id[lo];
        for (int p = 0; p < plan.n; ++p)
            atomicAdd(&s_hist[p][(key >> plan.shift[p]) & plan.mask[p]], 1u);
    }
    // global digit counts of the onesweep tile sort (fused: saves a pass over the keys)
    __syncthreads();
    for (int i = tid; i < plan.n * 256; i += kBlock) {
        const uint32_t c = (&s_hist[0][0])[i];
        if (c) atomicAdd(&ghist[i], c);
    }
}

// upstream identifyTileRanges over the tile-sorted keys (ranges pre-zeroed).
__global__ __launch_bounds__(kBlock) void k_ranges(const uint32_t *__restrict__ tile_keys,
                                                   int64_t K, uint32_t *__restrict__ ranges) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= K) return;
    const uint32_t cur = tile_keys[i];
    if (i == 0) {
        ranges[2 * cur] = 0;
    } else {
        const uint32_t prev = tile_keys[i - 1];
        if (cur != prev) {
            ranges[2 * prev + 1] = (uint32_t)i;
            ranges[2 * cur] = (uint32_t)i;
        }
    }
    if (i == K - 1) ranges[2 * cur + 1] = (uint32_t)K;
}

__global__ __launch_bounds__(kBlock) void k_globalize(const uint32_t *__restrict__ local, int64_t K,
                                                      uint32_t offset, uint32_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < K) out[i] = local[i] + offset;
}

}  // namespace

int64_t gsr_scan_blocks(int64_t n) { return (n + kTile - 1) / kTile; }

hipError_t gsr_launch_scan_reduce(const uint32_t *perm, const uint32_t *strip_tiles, int64_t n,
                                  uint32_t *partials, hipStream_t s) {
    const int64_t nb = gsr_scan_blocks(n);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(kBlock), 0, s, perm, strip_tiles, n,
                       partials);
    return hipGetLastError();
}

hipError_t gsr_launch_scan_partials(uint32_t *partials, int64_t nb, uint64_t *total,
                                    hipStream_t s) {
    hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(kBlock), 0, s, partials, nb, total);
    return hipGetLastError();
}

hipError_t gsr_launch_scan_down(const uint32_t *perm, const uint32_t *strip_tiles,
                                const uint32_t *partials, int64_t n, const uint64_t *total,
                                uint32_t *offsets, uint32_t *chunk_first, hipStream_t s) {
    const int64_t nb = gsr_scan_blocks(n);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scan_down, dim3((unsigned)nb), dim3(kBlock), 0, s, perm, strip_tiles,
                       partials, n, total, offsets, chunk_first);
    return hipGetLastError();
}

int64_t gsr_duplicate_chunks(int64_t K) { return (K + kChunk - 1) / kChunk; }

hipError_t gsr_launch_duplicate(const uint32_t *perm, const uint32_t *offsets,
                                const uint32_t *chunk_first, int64_t K, const SplatRecord *records,
                                const int32_t *radii, uint32_t gx, uint32_t gy, uint32_t row_begin,
                                uint32_t *tile_keys, uint32_t *tile_vals,
                                const GsrRadixPlan &plan, uint32_t *ghist, hipStream_t s) {
    const int64_t nc = gsr_duplicate_chunks(K);
    if (nc == 0) return hipSuccess;
    hipLaunchKernelGGL(k_duplicate, dim3((unsigned)nc), dim3(kBlock), 0, s, perm, offsets,
                       chunk_first, (uint32_t)K, (uint32_t)nc, records, radii, gx, gy, row_begin,
                       tile_keys, tile_vals, plan, ghist);
    return hipGetLastError();
}

hipError_t gsr_launch_ranges(const uint32_t *tile_keys, int64_t K, uint32_t *ranges,
                             hipStream_t s) {
    if (K == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ranges, dim3((unsigned)((K + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       tile_keys, K, ranges);
    return hipGetLastError();
}

hipError_t gsr_launch_globalize_tiles(const uint32_t *local, int64_t K, uint32_t offset,
                                      uint32_t *global, hipStream_t s) {
    if (K == 0) return hipSuccess;
    hipLaunchKernelGGL(k_globalize, dim3((unsigned)((K + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       s, local, K, offset, global);
    return hipGetLastError();
}
