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
#include <atomic>

#include "radix_tile.h"

using namespace gsr;

namespace {

constexpr int kBlock = 256;
constexpr int kItems = 4;
constexpr int kTile = kBlock * kItems;  // 1024 depth-sorted Gaussians per scan block
constexpr uint32_t kChunk = 2048;        // output pairs per duplicate block

// Pass 1 of the scan: per-block sum of the strip tile counts, gathered in depth order; the
// gathered rects are also written out in depth order (rect_sorted) so pass 3 reads them
// coalesced instead of gathering them a second time.
__device__ __forceinline__ uint32_t rect_count(uint2 r) { return (r.x >> 16) * (r.y >> 16); }

// d_n (if set): the depth sort's count of sorted entries (the rest of perm is stale).
__global__ __launch_bounds__(kBlock) void k_scan_reduce(const uint32_t *__restrict__ perm,
                                                        const uint2 *__restrict__ strip_rect,
                                                        int64_t n_max, const uint32_t *d_n,
                                                        uint32_t *__restrict__ partials,
                                                        uint2 *__restrict__ rect_sorted) {
    __shared__ uint32_t s_tmp[4];
    const int64_t n = d_n ? (int64_t)*d_n : n_max;
    const int64_t base = (int64_t)blockIdx.x * kTile;
    if (base >= n) {  // whole block: an empty partial
        if (threadIdx.x == 0) partials[blockIdx.x] = 0;
        return;
    }
    uint32_t sum = 0;
#pragma unroll 4
    for (int j = 0; j < kItems; ++j) {
        const int64_t e = base + j * kBlock + threadIdx.x;
        if (e < n) {
            const uint2 r = strip_rect[perm[e]];
            rect_sorted[e] = r;
            sum += rect_count(r);
        }
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

// Pass 3: exclusive offsets of the depth-sorted Gaussians, written with everything the
// duplication needs as bin[e] = {offset, id, x0 | width << 16, strip-local row0} (coalesced,
// so the duplicate kernels stage their Gaussians without a gather), and, for every chunk of
// kChunk output pairs, the first Gaussian whose pairs reach into it (chunk_first[c]);
// chunk_first[n_chunks] = one past the last Gaussian with pairs.  Gaussians without pairs in
// the strip carry the sentinel depth key, so they all sit after the last non-empty one.
__global__ __launch_bounds__(kBlock) void k_scan_down(const uint32_t *__restrict__ perm,
                                                      const uint2 *__restrict__ rect_sorted,
                                                      const uint32_t *__restrict__ partials,
                                                      int64_t n_max, const uint32_t *d_n,
                                                      const uint64_t *__restrict__ total,
                                                      uint4 *__restrict__ bin,
                                                      uint32_t *__restrict__ chunk_first) {
    __shared__ uint32_t s_tmp[4];
    const int64_t n = d_n ? (int64_t)*d_n : n_max;
    if ((int64_t)blockIdx.x * kTile >= n) return;  // whole block
    const int tid = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)tid * kItems;
    uint32_t cnt[kItems], id[kItems], sum = 0;
    uint2 rc[kItems];
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
        const int64_t e = base + j;
        id[j] = e < n ? perm[e] : 0u;
        rc[j] = e < n ? rect_sorted[e] : make_uint2(0u, 0u);
        cnt[j] = rect_count(rc[j]);
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
        if (cnt[j]) {
            bin[e] = make_uint4(off, id[j], rc[j].x, rc[j].y & 0xFFFFu);
            for (uint32_t c = (off + kChunk - 1) / kChunk; c * kChunk < off + cnt[j]; ++c)
                chunk_first[c] = (uint32_t)e;
            if (off + cnt[j] == K) chunk_first[n_chunks] = (uint32_t)e + 1u;
        }
        off += cnt[j];
    }
}

// ---- per-pair binning: upstream duplicateWithKeys fused with the first tile-sort pass ------
// (The fallback for frames the column-first form below cannot take, api.hip.)  The tile sort's
// first radix pass needs, per sort tile, the digit histogram of its pairs and then the pairs
// themselves in order.  Both are generated here from the depth-sorted Gaussians instead of
// being written by a duplicate kernel and read back: k_dup_count builds the
// histogram of each 4096-pair output chunk (= one sort tile), k_rs_scan scans it, and
// k_dup_scatter regenerates the chunk in registers, ranks it by the digit and scatters it --
// the K-sized pair array is written once and never read by this pass.
constexpr int kFW = 8, kFIt = 8;                   // 8 waves x 8 pairs per lane
constexpr uint32_t kFChunk = kFW * 64 * kFIt;      // 4096 = 2 duplicate chunks
static_assert(kFChunk == 2 * kChunk, "fused chunks are pairs of scan_down chunks");

constexpr int kStageCap = 2048;  // Gaussians staged in LDS; denser chunks read global memory

struct DupStage {
    uint32_t off[kStageCap];
    uint32_t id[kStageCap];
    uint32_t x0w[kStageCap];   // rect x0 | width << 16
    uint32_t row0[kStageCap];  // first strip-local tile row * gx
};

struct GaussRange {
    uint32_t e0;
    int ne;  // <= kFChunk + 1: every Gaussian of the range owns >= 1 pair
};

// The Gaussians whose pairs overlap fused chunk c.  n_chunks = scan_down chunk count.
__device__ __forceinline__ GaussRange fused_chunk_range(uint32_t c,
                                                        const uint32_t *__restrict__ chunk_first,
                                                        uint32_t n_chunks) {
    const uint32_t e_end_all = chunk_first[n_chunks];
    const uint32_t e0 = chunk_first[2 * c];
    const uint32_t e1 =
        (2 * c + 2 < n_chunks) ? min(chunk_first[2 * c + 2] + 1u, e_end_all) : e_end_all;
    return {e0, (int)(e1 - e0)};
}

struct BinSrc {
    const uint4 *bin;
    uint32_t gx;
    __device__ __forceinline__ void info(uint32_t e, uint32_t &id, uint32_t &x0w,
                                         uint32_t &row0) const {
        const uint4 b = bin[e];
        id = b.y;
        x0w = b.z;
        row0 = b.w * gx;
    }
};

// Stage the range in LDS if it fits (block-uniform decision).
__device__ __forceinline__ bool stage_range(const GaussRange &r, const BinSrc &src,
                                            DupStage &st) {
    if (r.ne > kStageCap) return false;
    for (int i = threadIdx.x; i < r.ne; i += kFW * 64) {
        const uint4 b = src.bin[r.e0 + i];
        st.off[i] = b.x;
        st.id[i] = b.y;
        st.x0w[i] = b.z;
        st.row0[i] = b.w * src.gx;
    }
    return true;
}

// Pairs [o0, o0 + kFIt) of the output, row-major over each Gaussian's rect (upstream
// duplicateWithKeys order); outputs >= o_end get the sentinel key 0xFFFFFFFF.  Reads the
// staged copy, or global memory when the range did not fit.
__device__ __forceinline__ void gen_pairs(const DupStage &st, bool staged, const GaussRange &r,
                                          const BinSrc &src, uint32_t o0, uint32_t o_end,
                                          uint32_t (&kk)[kFIt], uint32_t (&vv)[kFIt]) {
#pragma unroll
    for (int j = 0; j < kFIt; ++j) {
        kk[j] = 0xFFFFFFFFu;
        vv[j] = 0u;
    }
    if (o0 >= o_end) return;
    const uint4 *bins = src.bin + r.e0;
    auto off_at = [&](int i) { return staged ? st.off[i] : bins[i].x; };
    auto info_at = [&](int i, uint32_t &id, uint32_t &x0w, uint32_t &row0) {
        if (staged) {
            id = st.id[i];
            x0w = st.x0w[i];
            row0 = st.row0[i];
        } else {
            src.info(r.e0 + i, id, x0w, row0);
        }
    };
    const int ne = r.ne;
    int lo = 0, hi = ne - 1;  // last Gaussian of the range whose offset <= o0
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off_at(mid) <= o0) lo = mid;
        else hi = mid - 1;
    }
    uint32_t nxt = lo + 1 < ne ? off_at(lo + 1) : 0xFFFFFFFFu;
    uint32_t id, x0w, row0;
    info_at(lo, id, x0w, row0);
    uint32_t width = x0w >> 16;
    const uint32_t local = o0 - off_at(lo);
    const uint32_t row = local / width;
    uint32_t col = local - row * width;
    uint32_t rowkey = row0 + row * src.gx + (x0w & 0xFFFFu);
#pragma unroll
    for (int j = 0; j < kFIt; ++j) {
        const uint32_t o = o0 + (uint32_t)j;
        if (o < o_end) {
            if (o == nxt) {  // next Gaussian (each owns >= 1 pair)
                ++lo;
                nxt = lo + 1 < ne ? off_at(lo + 1) : 0xFFFFFFFFu;
                info_at(lo, id, x0w, row0);
                width = x0w >> 16;
                col = 0;
                rowkey = row0 + (x0w & 0xFFFFu);
            }
            kk[j] = rowkey + col;
            vv[j] = id;
            if (++col == width) {
                col = 0;
                rowkey += src.gx;
            }
        }
    }
}

__global__ __launch_bounds__(kFW * 64) void k_dup_count(
    const uint4 *__restrict__ bin, const uint32_t *__restrict__ chunk_first, uint32_t K,
    uint32_t n_chunks, uint32_t gx, int shift, uint32_t mask, uint32_t *__restrict__ hist,
    int64_t nb, uint2 *__restrict__ ranges_zero, uint32_t n_ranges) {
    __shared__ DupStage st;
    // zero the tile ranges for k_ranges (saves a memset launch)
    for (uint32_t i = blockIdx.x * (kFW * 64) + threadIdx.x; i < n_ranges; i += gridDim.x * (kFW * 64))
        ranges_zero[i] = make_uint2(0u, 0u);
    __shared__ uint32_t s_h[kFW][kRadixBins];
    const int tid = threadIdx.x, w = tid >> 6;
    const uint32_t c = blockIdx.x;
    for (int i = tid; i < kFW * kRadixBins; i += kFW * 64) (&s_h[0][0])[i] = 0;
    const BinSrc src{bin, gx};
    const GaussRange r = fused_chunk_range(c, chunk_first, n_chunks);
    const bool staged = stage_range(r, src, st);
    __syncthreads();
    uint32_t kk[kFIt], vv[kFIt];
    gen_pairs(st, staged, r, src, c * kFChunk + (uint32_t)tid * kFIt, min(K, (c + 1) * kFChunk),
              kk, vv);
#pragma unroll
    for (int j = 0; j < kFIt; ++j)
        if (kk[j] != 0xFFFFFFFFu) atomicAdd(&s_h[w][(kk[j] >> shift) & mask], 1u);
    __syncthreads();
    if (tid < kRadixBins) {
        uint32_t t = 0;
#pragma unroll
        for (int i = 0; i < kFW; ++i) t += s_h[i][tid];
        hist[(int64_t)tid * nb + c] = t;
    }
}

__global__ __launch_bounds__(kFW * 64) void k_dup_scatter(
    const uint4 *__restrict__ bin, const uint32_t *__restrict__ chunk_first, uint32_t K,
    uint32_t n_chunks, uint32_t gx, int shift, int nbits, const uint32_t *__restrict__ hist,
    int64_t nb, const uint32_t *__restrict__ digit_total, uint32_t *__restrict__ keys_out,
    uint32_t *__restrict__ vals_out) {
    union alignas(16) Smem {
        DupStage st;
        struct {
            uint32_t keys[kFChunk];
            uint32_t vals[kFChunk];
        } kv;
    };
    __shared__ Smem u;
    __shared__ RadixTileSmem<kFW, kFIt> sm;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t c = blockIdx.x;
    const BinSrc src{bin, gx};
    const GaussRange r = fused_chunk_range(c, chunk_first, n_chunks);
    const bool staged = stage_range(r, src, u.st);
    __syncthreads();
    uint32_t kk[kFIt], vv[kFIt];
    const uint32_t o_end = min(K, (c + 1) * kFChunk);
    gen_pairs(u.st, staged, r, src, c * kFChunk + (uint32_t)tid * kFIt, o_end, kk, vv);
    __syncthreads();
    // blocked (thread-consecutive) -> wave-striped layout through LDS
    static_assert(kFIt == 8, "two 16-B LDS writes per array");
    uint4 *k4 = reinterpret_cast<uint4 *>(u.kv.keys) + tid * 2;
    uint4 *v4 = reinterpret_cast<uint4 *>(u.kv.vals) + tid * 2;
    k4[0] = make_uint4(kk[0], kk[1], kk[2], kk[3]);
    k4[1] = make_uint4(kk[4], kk[5], kk[6], kk[7]);
    v4[0] = make_uint4(vv[0], vv[1], vv[2], vv[3]);
    v4[1] = make_uint4(vv[4], vv[5], vv[6], vv[7]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kFIt; ++j) {
        const int e = w * (kFChunk / kFW) + j * 64 + lane;
        kk[j] = u.kv.keys[e];
        vv[j] = u.kv.vals[e];
    }
    // (radix_tile_scatter's first barrier orders these reads before its LDS writes)
    radix_tile_scatter<kFW, kFIt>(kk, vv, (int)(o_end - c * kFChunk), shift, nbits, hist, nb, c,
                                  digit_total, keys_out, vals_out, sm, u.kv.keys, u.kv.vals);
}

// ---- column-first pair generation (the default binning form, chosen per frame by api.hip) -----
// The tile sort is LSD over (row, column): pass 1 by the column x, pass 2 by the row y.  Pass 1
// needs no pair-level work: a Gaussian whose strip rect is [x0, x0+w) x [y0, y0+h) has h pairs
// in each of its w columns, and in the stable column order those h pairs are contiguous (rows
// ascending, as duplicateWithKeys emits them row-major).  So pass 1 runs on (Gaussian, column)
// segments of h pairs:
//   k_col_count   -- per group of 4 blocks of kCG depth-sorted Gaussians, the pairs per column
//                    of each block (difference arrays over the columns: two LDS atomics per
//                    Gaussian), the depth-ordered rect copy, the group's column totals and each
//                    block's offsets within its group (grouping cut the scattered column-major
//                    stores 4x: C3 scan stage 31.7 -> 26 us, a C4 strip's 65 -> 57 us);
//   k_rs_scan     -- per column, the exclusive scan across groups (the radix sort's scan);
//   k_col_scatter -- per block: rank its segments by column (stable, in LDS), turn segment
//                    heights into pair offsets, and write every pair -- the packed word
//                    (row << pack_shift) | Gaussian id that pass 2 sorts on -- at its column's
//                    running position (one thread per segment, its h pairs contiguous).
// It replaces the offsets scan, the per-chunk pair regeneration and the per-pair ranking of
// the fused duplicate; the pair list is identical (each tile's pairs in depth order, then
// Gaussian index; tiles row-major).
constexpr int kCG = 256;                // depth-sorted Gaussians per block, one per thread
// 4 waves x up to 4 items: rounds of 1024 segments (C3 blocks average ~900; larger blocks take
// more rounds), so a block's LDS is ~20 KB and twice as many blocks share a CU as with rounds
// of 2048 (C3 column scatter 42.7 -> 34.0 us with the owner-written segment map below)
constexpr int kCW = 4, kCIt = 4;
constexpr int kCSeg = kCW * 64 * kCIt;  // up to 1024 segments ranked per round
static_assert(kCG == kRadixBins, "one thread per column in the column scans");

struct ColScatterSmem {
    uint32_t x0w[kCG], y0h[kCG], id[kCG], seg0[kCG + 1];
    uint32_t cols_lo[kCG], cols_hi[kCG];  // span words (tight binning, gsr::col_span)
    uint32_t colbase[kRadixBins], colw0[kRadixBins];
    uint32_t keys[kCSeg], vals[kCSeg];  // the round's segments by column
    uint32_t wpre[kCSeg + 1];           // pair offset of each sorted segment
    uint8_t seg_g[kCSeg];               // the round's segment -> block Gaussian (owner-written)
    uint32_t tmp[4];
};

// Rows [lo, lo + cnt) (strip rect relative) of the segment of block Gaussian t in tile column
// col.
// (bit 31 of y0h: tight binning off, every rect full)
__device__ __forceinline__ void seg_span(const ColScatterSmem &c, uint32_t t, uint32_t col,
                                         uint32_t &lo, uint32_t &cnt) {
    const uint2 rect = make_uint2(c.x0w[t], c.y0h[t] & 0x7FFFFFFFu);
    if (c.y0h[t] >> 31) {
        lo = 0u;
        cnt = rect.y >> 16;
        return;
    }
    col_span(rect, make_uint2(c.cols_lo[t], c.cols_hi[t]), col - (c.x0w[t] & 0xFFFFu), lo, cnt);
}

// One round of k_col_scatter: segments [R, R + rn) of the block, ranked kIt per lane (rn <=
// 256 kIt; blocks with few segments take the smaller instantiation, whose ranking pass costs
// half as much).
template <int kIt, typename Smem>
__device__ __forceinline__ void col_round(uint32_t R, uint32_t rn, int pack_shift,
                                          uint32_t *__restrict__ out, ColScatterSmem &c, Smem &sm) {
    constexpr int kSeg = kCW * 64 * kIt;
    const int tid = threadIdx.x;
    // the round's segment -> Gaussian map, written by each Gaussian's own thread
    {
        const uint32_t s0 = c.seg0[tid], w = c.x0w[tid] >> 16;
        const uint32_t cb = R > s0 ? R - s0 : 0u, ce = min(w, R + rn > s0 ? R + rn - s0 : 0u);
        for (uint32_t cc = cb; cc < ce; ++cc) c.seg_g[s0 + cc - R] = (uint8_t)tid;
    }
    __syncthreads();
    uint32_t k[kIt], v[kIt];
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
        const uint32_t slot = (uint32_t)((tid >> 6) * (kSeg / kCW) + j * 64 + (tid & 63));
        k[j] = 0xFFFFFFFFu;  // padding: largest column, after every real segment
        v[j] = 0u;
        if (slot < rn) {
            const uint32_t sg = R + slot;
            const int lo = c.seg_g[slot];  // the Gaussian whose segments hold sg
            const uint32_t col = (c.x0w[lo] & 0xFFFFu) + (sg - c.seg0[lo]);
            uint32_t slo, sn;
            seg_span(c, (uint32_t)lo, col, slo, sn);
            k[j] = col;
            v[j] = (uint32_t)lo | (slo << 8) | (sn << 12);  // Gaussian, its rows in the column
        }
    }
    radix_tile_scatter<kCW, kIt, false, false>(k, v, (int)rn, 0, 8, nullptr, 0, 0, nullptr,
                                               nullptr, nullptr, sm, c.keys, c.vals);
    // pair offsets of the sorted segments (heights, exclusive prefix)
    uint32_t hh[kIt], hsum = 0;
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
        const uint32_t p = (uint32_t)(tid * kIt + j);
        hh[j] = p < rn ? c.vals[p] >> 12 : 0u;
        hsum += hh[j];
    }
    uint32_t npairs;
    uint32_t pre = block256_exclusive_scan(hsum, c.tmp, npairs);
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
        c.wpre[tid * kIt + j] = pre;
        pre += hh[j];
    }
    if (tid == 0) c.wpre[kSeg] = npairs;
    __syncthreads();
    c.colw0[tid] = sm.count[tid] ? c.wpre[sm.delta[tid]] : 0u;
    __syncthreads();
    // one thread per sorted segment (consecutive lanes: consecutive segments, so within a
    // column consecutive destination runs); each writes its h pairs
    for (uint32_t p = tid; p < rn; p += kCG) {
        const uint32_t col = c.keys[p], v = c.vals[p], t = v & 0xFFu;
        const uint32_t id = c.id[t];
        const uint32_t dst = c.colbase[col] + (c.wpre[p] - c.colw0[col]);
        const uint32_t y0 = (c.y0h[t] & 0xFFFFu) + ((v >> 8) & 15u), h = v >> 12;
        for (uint32_t r = 0; r < h; ++r)
            out[dst + r] = (pack_shift < 32 ? (y0 + r) << pack_shift : 0u) | id;
    }
    __syncthreads();  // every thread has read this round's column bases
    // the next round continues every column where this one ended
    if (sm.count[tid]) c.colbase[tid] += c.wpre[sm.delta[tid] + sm.count[tid]] - c.colw0[tid];
    __syncthreads();
}

// Per group of kCGroup blocks (kCGroup x 256 depth-sorted Gaussians, one per thread and
// sub-block): the pairs per column of every sub-block (a difference array over the columns per
// sub-block, two LDS atomics per Gaussian), the depth-ordered rect copy, the group's column
// totals -- hist[col * n_groups + group], the layout k_rs_scan scans, written once per group
// rather than once per block -- and each sub-block's exclusive offset within its group,
// off[block * 256 + col] (one coalesced 1 KB row per block).
constexpr int kCGroup = 4;
__global__ __launch_bounds__(kCG) void k_col_count(const uint32_t *__restrict__ perm,
                                                   const uint2 *__restrict__ strip_rect,
                                                   const uint4 *__restrict__ strip_rc,
                                                   const uint32_t *__restrict__ d_n,
                                                   uint2 *__restrict__ rect_sorted,
                                                   uint4 *__restrict__ rc_sorted,
                                                   uint32_t *__restrict__ hist, int64_t ng,
                                                   uint32_t *__restrict__ off) {
    __shared__ uint32_t s_diff[kCGroup][kRadixBins + 1];
    __shared__ uint32_t s_tmp[4];
    const int tid = threadIdx.x;
    const uint32_t gb = xcd_run_block(blockIdx.x);  // the group
    const int64_t n = *d_n;
    const int64_t base = (int64_t)gb * (kCG * kCGroup);
    if (base >= n) return;  // whole group (k_rs_scan reads groups [0, ceil(n / 1024)) only)
    for (int i = tid; i < kCGroup * (kRadixBins + 1); i += kCG) (&s_diff[0][0])[i] = 0u;
    uint2 r[kCGroup], q[kCGroup];
#pragma unroll
    for (int j = 0; j < kCGroup; ++j) {
        const int64_t e = base + j * kCG + tid;
        const uint32_t id = e < n ? perm[e] : 0u;
        r[j] = q[j] = make_uint2(0u, 0u);
        if (e < n && strip_rc) {  // tight binning: the rect and its span word, one 16-B gather
            const uint4 rq = strip_rc[id];
            r[j] = make_uint2(rq.x, rq.y);
            q[j] = make_uint2(rq.z, rq.w);
            rc_sorted[e] = rq;
        } else if (e < n) {
            r[j] = strip_rect[id];
            rect_sorted[e] = r[j];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kCGroup; ++j) {
        const uint32_t x0 = r[j].x & 0xFFFFu, w = r[j].x >> 16, h = r[j].y >> 16;
        if (w && strip_rc && span_coded(r[j])) {
            // column c holds cnt_c pairs: the difference cnt_c - cnt_{c-1} at column x0 + c
            uint32_t prev = 0u;
#pragma unroll
            for (uint32_t c = 0; c <= kSpanCols; ++c) {
                if (c > w) break;
                uint32_t lo, cnt = 0u;
                if (c < w) col_span(r[j], q[j], c, lo, cnt);
                if (cnt != prev) atomicAdd(&s_diff[j][x0 + c], cnt - prev);
                prev = cnt;
            }
        } else if (w) {
            atomicAdd(&s_diff[j][x0], h);
            atomicAdd(&s_diff[j][x0 + w], 0u - h);
        }
    }
    __syncthreads();
    uint32_t run = 0;
    uint32_t *o = off + (int64_t)gb * kCGroup * kRadixBins;
#pragma unroll
    for (int j = 0; j < kCGroup; ++j) {
        uint32_t tot;
        const uint32_t d = s_diff[j][tid];
        const uint32_t c = block256_exclusive_scan(d, s_tmp, tot) + d;  // sub-block j, column tid
        o[j * kRadixBins + tid] = run;
        run += c;
    }
    hist[(int64_t)tid * ng + gb] = run;
}

__global__ __launch_bounds__(kCG) void k_col_scatter(const uint32_t *__restrict__ perm,
                                                     const uint2 *__restrict__ rect_sorted,
                                                     const uint4 *__restrict__ rc_sorted,
                                                     const uint32_t *__restrict__ d_n,
                                                     const uint32_t *__restrict__ hist, int64_t ng,
                                                     const uint32_t *__restrict__ off,
                                                     const uint32_t *__restrict__ digit_total,
                                                     int pack_shift, uint32_t *__restrict__ out,
                                                     uint32_t cap, uint32_t *__restrict__ list_n) {
    __shared__ ColScatterSmem c;
    __shared__ union {
        RadixTileSmem<kCW, kCIt> big;
        RadixTileSmem<kCW, kCIt / 2> small;
    } sm;
    const int tid = threadIdx.x;
    const uint32_t blk = xcd_run_block(blockIdx.x);
    // global start of column d for this block's segments: all earlier columns (then earlier
    // blocks, below); the total is the list length
    uint32_t tot;
    const uint32_t dstart = block256_exclusive_scan(digit_total[tid], c.tmp, tot);
    if (list_n && blk == 0 && tid == 0) *list_n = tot;  // (frame graphs: the row pass)
    if (tot > cap) return;  // (frame graphs) the list does not fit: the host re-renders
    const int64_t n = *d_n;
    const int64_t base = (int64_t)blk * kCG;
    if (base >= n) return;
    const int64_t e = base + tid;
    const bool valid = e < n;
    uint2 r = make_uint2(0u, 0u), q = r;
    if (valid && rc_sorted) {
        const uint4 rq = rc_sorted[e];
        r = make_uint2(rq.x, rq.y);
        q = make_uint2(rq.z, rq.w);
    } else if (valid) {
        r = rect_sorted[e];
    }
    c.x0w[tid] = r.x;
    c.y0h[tid] = rc_sorted ? r.y : (r.y | 0x80000000u);  // bit 31: not span-coded (full)
    c.cols_lo[tid] = q.x;
    c.cols_hi[tid] = q.y;
    c.id[tid] = valid ? perm[e] : 0u;
    c.colbase[tid] = dstart + hist[(int64_t)tid * ng + blk / kCGroup] +
                     off[(int64_t)blk * kRadixBins + tid];
    // thread t owns segments [seg0, seg0 + w) (one per column of its rect)
    uint32_t nseg;
    const uint32_t seg0 = block256_exclusive_scan(r.x >> 16, c.tmp, nseg);
    c.seg0[tid] = seg0;
    if (tid == 0) c.seg0[kCG] = nseg;
    __syncthreads();
    for (uint32_t R = 0; R < nseg; R += kCSeg) {
        const uint32_t rn = min((uint32_t)kCSeg, nseg - R);
        if (rn <= (uint32_t)kCSeg / 2)
            col_round<kCIt / 2>(R, rn, pack_shift, out, c, sm.small);
        else
            col_round<kCIt>(R, rn, pack_shift, out, c, sm.big);
    }
}

// upstream identifyTileRanges over the tile-sorted keys (ranges pre-zeroed).
// 4 keys per thread (one 16-B load when aligned and complete).
__global__ __launch_bounds__(kBlock) void k_ranges(const uint32_t *__restrict__ tile_keys,
                                                   int64_t K, uint32_t *__restrict__ ranges) {
    const int64_t i0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4;
    if (i0 >= K) return;
    uint32_t k[4];
    if (i0 + 4 <= K) {
        const uint4 q = *reinterpret_cast<const uint4 *>(tile_keys + i0);
        k[0] = q.x;
        k[1] = q.y;
        k[2] = q.z;
        k[3] = q.w;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) k[j] = i0 + j < K ? tile_keys[i0 + j] : 0u;
    }
    uint32_t prev = i0 > 0 ? tile_keys[i0 - 1] : 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t i = i0 + j;
        if (i >= K) break;
        const uint32_t cur = k[j];
        if (i == 0) {
            ranges[2 * cur] = 0;
        } else if (cur != prev) {
            ranges[2 * prev + 1] = (uint32_t)i;
            ranges[2 * cur] = (uint32_t)i;
        }
        if (i == K - 1) ranges[2 * cur + 1] = (uint32_t)K;
        prev = cur;
    }
}

// Pair count of every tile row of the strip: block y sums end - start over its gx tiles.
__global__ __launch_bounds__(kBlock) void k_row_pairs(const uint2 *__restrict__ ranges,
                                                      uint32_t gx, uint32_t *__restrict__ out) {
    __shared__ uint32_t s_tmp[4];
    uint32_t v = 0;
    for (uint32_t x = threadIdx.x; x < gx; x += kBlock) {
        const uint2 r = ranges[(size_t)blockIdx.x * gx + x];
        v += r.y - r.x;
    }
    uint32_t total;
    block256_exclusive_scan(v, s_tmp, total);
    if (threadIdx.x == 0) out[blockIdx.x] = total;
}

// Packed pair list -> Gaussian ids (gsr_get_binning).
__global__ __launch_bounds__(kBlock) void k_unpack_ids(const uint32_t *__restrict__ packed,
                                                       int64_t K, uint32_t mask,
                                                       uint32_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < K) out[i] = packed[i] & mask;
}

// Tile id of every pair from the tile ranges (gsr_get_binning with a packed list): block t
// fills its tile's range with offset + t.
__global__ __launch_bounds__(kBlock) void k_fill_tiles(const uint2 *__restrict__ ranges,
                                                       uint32_t offset,
                                                       uint32_t *__restrict__ out) {
    const uint2 r = ranges[blockIdx.x];
    for (uint32_t i = r.x + threadIdx.x; i < r.y; i += kBlock) out[i] = offset + blockIdx.x;
}

__global__ __launch_bounds__(kBlock) void k_globalize(const uint32_t *__restrict__ local, int64_t K,
                                                      uint32_t offset, uint32_t *__restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < K) out[i] = local[i] + offset;
}

}  // namespace

int64_t gsr_scan_blocks(int64_t n) { return (n + kTile - 1) / kTile; }

hipError_t gsr_launch_scan_reduce(const uint32_t *perm, const uint2 *strip_rect, int64_t n,
                                  const uint32_t *d_n, uint32_t *partials, uint2 *rect_sorted,
                                  hipStream_t s) {
    const int64_t nb = gsr_scan_blocks(n);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(kBlock), 0, s, perm, strip_rect, n,
                       d_n, partials, rect_sorted);
    return hipGetLastError();
}

hipError_t gsr_launch_scan_partials(uint32_t *partials, int64_t nb, uint64_t *total,
                                    hipStream_t s) {
    hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(kBlock), 0, s, partials, nb, total);
    return hipGetLastError();
}

hipError_t gsr_launch_scan_down(const uint32_t *perm, const uint2 *rect_sorted,
                                const uint32_t *partials, int64_t n, const uint32_t *d_n,
                                const uint64_t *total, uint4 *bin, uint32_t *chunk_first,
                                hipStream_t s) {
    const int64_t nb = gsr_scan_blocks(n);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scan_down, dim3((unsigned)nb), dim3(kBlock), 0, s, perm, rect_sorted,
                       partials, n, d_n, total, bin, chunk_first);
    return hipGetLastError();
}

int64_t gsr_duplicate_chunks(int64_t K) { return (K + kChunk - 1) / kChunk; }

int64_t gsr_fused_chunks(int64_t K) { return (K + kFChunk - 1) / kFChunk; }

hipError_t gsr_launch_dup_sort_pass(const uint4 *bin, const uint32_t *chunk_first, int64_t K,
                                    uint32_t gx, int shift, int nbits, uint32_t *hist,
                                    uint32_t *digit_total, uint32_t *keys_out, uint32_t *vals_out,
                                    uint2 *ranges_zero, uint32_t n_ranges, hipStream_t s) {
    const int64_t nb = gsr_fused_chunks(K);
    if (nb == 0) return hipSuccess;
    const uint32_t nc = (uint32_t)gsr_duplicate_chunks(K);
    const uint32_t mask = (1u << nbits) - 1u;
    hipLaunchKernelGGL(k_dup_count, dim3((unsigned)nb), dim3(kFW * 64), 0, s, bin, chunk_first,
                       (uint32_t)K, nc, gx, shift, mask, hist, nb, ranges_zero, n_ranges);
    hipError_t e = gsr_launch_digit_scan(hist, nb, digit_total, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_dup_scatter, dim3((unsigned)nb), dim3(kFW * 64), 0, s, bin, chunk_first,
                       (uint32_t)K, nc, gx, shift, nbits, hist, nb, digit_total, keys_out,
                       vals_out);
    return hipGetLastError();
}

namespace {

// ---- tile ranges from per-tile pair counts (second stream) ---------------------------------
// The sorted pair list holds each tile's pairs contiguously in tile order, so ranges[t] =
// [start_t, start_t + count_t) with start_t the exclusive scan of the per-tile pair counts --
// which depend only on the Gaussians' tile rects, not on any sort.  They are computed on the
// second stream while the main stream sorts, in two kernels:
//   k_tile_diff     -- per block of Gaussians, in LDS: for every tile column of a rect (or of
//                      its tight spans), a difference array down the rows (+1 at the first row,
//                      -1 past the last: two LDS atomics per column), then per column the prefix
//                      down the rows = the block's per-tile counts, and the rows' totals; the
//                      block's counts and totals go to `partial` (kTileDiffBlocks of them);
//   k_tile_finalize -- one block per tile row: sums the partials' counts of its row; the row's
//                      first offset = the sum of the row totals above; then an exclusive scan
//                      along the row.
// Tiles without pairs get (0, 0), as upstream's memset leaves them.  Replaces k_ranges, a pass
// over the K sorted keys on the main stream (the packed pair list has no tile keys to scan).
constexpr int kDiffThreads = 1024;

// kTight: the {rect, span word} records, column-major differences (two atomics per kept column,
// then a prefix down each column); else the rects, row-major differences (two atomics per rect
// row -- a strip clips the rows but not the columns -- then a prefix along each row).
template <bool kTight>
__global__ __launch_bounds__(kDiffThreads) void k_tile_diff(const uint2 *__restrict__ strip_rect,
                                                            const uint4 *__restrict__ strip_rc,
                                                            int64_t P, uint32_t gx, uint32_t rows,
                                                            uint32_t *__restrict__ partial) {
    extern __shared__ uint32_t s_diff[];
    const uint32_t w1 = gx + 1, cells = gsr_tile_diff_cells(gx, rows);
    uint32_t *s_rows = s_diff + w1 * (rows + 1);  // the rows' pair totals
    for (uint32_t c = threadIdx.x; c < cells; c += kDiffThreads) s_diff[c] = 0u;
    __syncthreads();
    const int64_t b0 = P * blockIdx.x / gridDim.x, b1 = P * (blockIdx.x + 1) / gridDim.x;
    // 4 rects per thread and step, their loads issued together
    constexpr int kU = 4;
    for (int64_t i = b0 + threadIdx.x; i < b1; i += kU * kDiffThreads) {
        uint2 r[kU], q[kU];
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const int64_t j = i + (int64_t)k * kDiffThreads;
            r[k] = q[k] = make_uint2(0u, 0u);
            if (j < b1 && kTight) {  // the rect and its span word, one load
                const uint4 rq = strip_rc[j];
                r[k] = make_uint2(rq.x, rq.y);
                q[k] = make_uint2(rq.z, rq.w);
            } else if (j < b1) {
                r[k] = strip_rect[j];
            }
        }
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            if (r[k].x == 0u) continue;  // no pairs in the strip (a rect with pairs has width > 0)
            const uint32_t x0 = r[k].x & 0xFFFFu, w = r[k].x >> 16, y0 = r[k].y & 0xFFFFu;
            if (!kTight) {
                for (uint32_t y = y0; y < y0 + (r[k].y >> 16); ++y) {
                    atomicAdd(&s_diff[y * w1 + x0], 1u);
                    atomicAdd(&s_diff[y * w1 + x0 + w], 0xFFFFFFFFu);  // -1 (mod 2^32)
                }
                continue;
            }
            const bool coded = span_coded(r[k]);
            // column x0 + c holds rows [y0 + lo, y0 + lo + cnt): +1 / -1 down the column
            for (uint32_t c = 0; c < w; ++c) {
                uint32_t lo = 0u, cnt = r[k].y >> 16;
                if (coded) col_span(r[k], q[k], c, lo, cnt);
                if (cnt) {
                    atomicAdd(&s_diff[(y0 + lo) * w1 + x0 + c], 1u);
                    atomicAdd(&s_diff[(y0 + lo + cnt) * w1 + x0 + c], 0xFFFFFFFFu);  // -1
                }
            }
        }
    }
    __syncthreads();
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    if (kTight) {
        // per column, the prefix down the rows: each tile's pair count (in place)
        for (uint32_t x = threadIdx.x; x < gx; x += kDiffThreads) {
            uint32_t run = 0u;
            for (uint32_t y = 0; y < rows; ++y) {
                run += s_diff[y * w1 + x];
                s_diff[y * w1 + x] = run;
            }
        }
    } else {
        // per row (a wave each), the prefix along the row
        for (uint32_t y = wv; y < rows; y += kDiffThreads / 64) {
            uint32_t carry = 0u;
            for (uint32_t x0 = 0; x0 < gx; x0 += 64) {
                const uint32_t x = x0 + ln;
                const uint32_t v = x < gx ? s_diff[y * w1 + x] : 0u;
                const uint32_t inc = wave_inclusive_scan(v) + carry;
                if (x < gx) s_diff[y * w1 + x] = inc;
                carry = __shfl(inc, 63);
            }
        }
    }
    __syncthreads();
    // the rows' totals
    for (uint32_t y = wv; y < rows; y += kDiffThreads / 64) {
        uint32_t acc = 0u;
        for (uint32_t x = ln; x < gx; x += 64) acc += s_diff[y * w1 + x];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (ln == 0) s_rows[y] = acc;
    }
    __syncthreads();
    uint32_t *dst = partial + (int64_t)blockIdx.x * cells;
    for (uint32_t c = threadIdx.x; c < cells; c += kDiffThreads) dst[c] = s_diff[c];
}

// Inclusive scan over the block (kW waves); s_tmp: kW words.  Returns the prefix, total out.
template <int kW>
__device__ __forceinline__ uint32_t blockw_inclusive_scan(uint32_t v, uint32_t *s_tmp,
                                                          uint32_t &total) {
    return blockw_exclusive_scan<kW>(v, s_tmp, total) + v;
}

constexpr int kFinThreads = 256;
__global__ __launch_bounds__(kFinThreads) void k_tile_finalize(const uint32_t *__restrict__ partial,
                                                               int nparts, uint32_t gx,
                                                               uint32_t rows,
                                                               uint2 *__restrict__ ranges) {
    constexpr int kW = kFinThreads / 64;
    __shared__ uint32_t s_tmp[kW];
    const uint32_t y = blockIdx.x, w1 = gx + 1, cells = gsr_tile_diff_cells(gx, rows);
    const int tid = threadIdx.x;
    // offset of this row: the sum of the row totals above it
    uint32_t before = 0;
    for (uint32_t y0 = 0; y0 < y; y0 += kFinThreads) {
        const uint32_t yy = y0 + tid;
        uint32_t rt = 0;
        if (yy < y)
#pragma unroll 8
            for (int b = 0; b < nparts; ++b) rt += partial[(int64_t)b * cells + w1 * (rows + 1) + yy];
        uint32_t t;
        blockw_inclusive_scan<kW>(rt, s_tmp, t);
        before += t;
    }
    // this row's counts (the partials' sum), then an exclusive scan along the row
    uint32_t start = before;
    for (uint32_t x0 = 0; x0 < gx; x0 += kFinThreads) {
        const uint32_t x = x0 + tid;
        uint32_t cnt = 0;
        if (x < gx)
#pragma unroll 8
            for (int b = 0; b < nparts; ++b) cnt += partial[(int64_t)b * cells + y * w1 + x];
        uint32_t t2;
        const uint32_t ex = blockw_exclusive_scan<kW>(x < gx ? cnt : 0u, s_tmp, t2) + start;
        start += t2;
        if (x < gx) ranges[y * gx + x] = cnt ? make_uint2(ex, ex + cnt) : make_uint2(0u, 0u);
    }
}

}  // namespace

hipError_t gsr_launch_tile_ranges_aux(const uint2 *strip_rect, const uint4 *strip_rc, int64_t P,
                                      uint32_t gx, uint32_t rows, uint32_t *partial, uint2 *ranges,
                                      hipStream_t s) {
    const uint32_t cells = gsr_tile_diff_cells(gx, rows);
    const size_t lds = (size_t)cells * 4;
    if (cells > kTileDiffMaxCells) return hipErrorInvalidValue;
    // the > 64 KiB dynamic-LDS attribute is per (function, device): one bit per device, set
    // atomically (setting it twice from racing threads is harmless)
    static std::atomic<uint64_t> attr_done{0};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const uint64_t bit = dev < 64 ? (1ull << dev) : 0ull;
    if (!bit || !(attr_done.load(std::memory_order_acquire) & bit)) {
        for (const void *fn : {reinterpret_cast<const void *>(&k_tile_diff<true>),
                               reinterpret_cast<const void *>(&k_tile_diff<false>)}) {
            e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    kTileDiffMaxCells * 4);
            if (e != hipSuccess) return e;
        }
        attr_done.fetch_or(bit, std::memory_order_release);
    }
    // one block per 16k rects (at least 64, at most kTileDiffBlocks): the rect pass stays
    // short at 6M Gaussians while the finalize's sum over the partials stays small at 1M
    const int nparts = (int)std::min<int64_t>(kTileDiffBlocks, std::max<int64_t>(64, (P + 16383) / 16384));
    if (strip_rc)
        hipLaunchKernelGGL(k_tile_diff<true>, dim3(nparts), dim3(kDiffThreads), lds, s, strip_rect,
                           strip_rc, P, gx, rows, partial);
    else
        hipLaunchKernelGGL(k_tile_diff<false>, dim3(nparts), dim3(kDiffThreads), lds, s,
                           strip_rect, strip_rc, P, gx, rows, partial);
    hipLaunchKernelGGL(k_tile_finalize, dim3(rows), dim3(kFinThreads), 0, s, partial,
                       nparts, gx, rows, ranges);
    return hipGetLastError();
}

hipError_t gsr_launch_ranges(const uint32_t *tile_keys, int64_t K, uint32_t *ranges,
                             hipStream_t s) {
    if (K == 0) return hipSuccess;
    hipLaunchKernelGGL(k_ranges, dim3((unsigned)((K + 4 * kBlock - 1) / (4 * kBlock))),
                       dim3(kBlock), 0, s, tile_keys, K, ranges);
    return hipGetLastError();
}

hipError_t gsr_launch_globalize_tiles(const uint32_t *local, int64_t K, uint32_t offset,
                                      uint32_t *global, hipStream_t s) {
    if (K == 0) return hipSuccess;
    hipLaunchKernelGGL(k_globalize, dim3((unsigned)((K + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       s, local, K, offset, global);
    return hipGetLastError();
}

hipError_t gsr_launch_row_pairs(const uint2 *ranges, uint32_t gx, uint32_t rows, uint32_t *out,
                                hipStream_t s) {
    if (rows == 0) return hipSuccess;
    hipLaunchKernelGGL(k_row_pairs, dim3(rows), dim3(kBlock), 0, s, ranges, gx, out);
    return hipGetLastError();
}

hipError_t gsr_launch_unpack_ids(const uint32_t *packed, int64_t K, uint32_t mask, uint32_t *out,
                                 hipStream_t s) {
    if (K <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_unpack_ids, dim3((unsigned)((K + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       s, packed, K, mask, out);
    return hipGetLastError();
}

hipError_t gsr_launch_fill_tiles(const uint2 *ranges, uint32_t n_tiles, uint32_t offset,
                                 uint32_t *out, hipStream_t s) {
    if (n_tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill_tiles, dim3(n_tiles), dim3(kBlock), 0, s, ranges, offset, out);
    return hipGetLastError();
}

// Rows of 256 words the column-first binning needs: per block its sub-block offsets, per group
// its column totals.
int64_t gsr_col_blocks(int64_t n) {
    const int64_t nb = (n + kCG - 1) / kCG, ng = (nb + kCGroup - 1) / kCGroup;
    return nb + ng;
}

hipError_t gsr_launch_col_pairs_count(const uint32_t *perm, const uint2 *strip_rect,
                                      const uint4 *strip_rc, int64_t n_max, const uint32_t *d_n,
                                      uint2 *rect_sorted, uint4 *rc_sorted, uint32_t *hist,
                                      uint32_t *digit_total, hipStream_t s) {
    const int64_t nb = (n_max + kCG - 1) / kCG, ng = (nb + kCGroup - 1) / kCGroup;
    if (nb == 0) return hipSuccess;
    uint32_t *off = hist + ng * kRadixBins;
    const dim3 grid(xcd_run_grid(ng));
    hipLaunchKernelGGL(k_col_count, grid, dim3(kCG), 0, s, perm, strip_rect, strip_rc, d_n,
                       rect_sorted, rc_sorted, hist, ng, off);
    return gsr_launch_digit_scan_n(hist, ng, digit_total, d_n, kCG * kCGroup, s);
}

hipError_t gsr_launch_col_pairs_scatter(const uint32_t *perm, const uint2 *rect_sorted,
                                        const uint4 *rc_sorted, int64_t n_max,
                                        const uint32_t *d_n, const uint32_t *hist,
                                        const uint32_t *digit_total, int pack_shift, uint32_t *out,
                                        hipStream_t s, uint32_t cap, uint32_t *list_n) {
    const int64_t nb = (n_max + kCG - 1) / kCG, ng = (nb + kCGroup - 1) / kCGroup;
    if (nb == 0) return hipSuccess;
    const uint32_t *off = hist + ng * kRadixBins;
    const dim3 grid(xcd_run_grid(nb));
    hipLaunchKernelGGL(k_col_scatter, grid, dim3(kCG), 0, s, perm, rect_sorted, rc_sorted, d_n,
                       hist, ng, off, digit_total, pack_shift, out, cap, list_n);
    return hipGetLastError();
}
