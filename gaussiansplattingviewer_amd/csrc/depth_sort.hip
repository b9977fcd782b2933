// depth_sort.hip -- the per-frame stable sort of the Gaussians by view depth, for gfx950.
//
// Replaces the depth half of upstream's cub::DeviceRadixSort::SortPairs over (tile << 32 |
// depth) keys (rasterizer_impl.cu; see DESIGN.md decision 1 for the depth-first binning) and
// the viewer's torch / cupy / numpy argsort (renderer_ogl.py:17, :34, :51; gsr_depth_argsort).
//
// A wide-digit LSD radix sort that sorts only the key bits that vary:
//   * digits of 12 bits: passes over key bits [0,12), [12,24), [24,32);
//   * pass 0's upsweep also reduces the OR and the AND of the kept keys.  Bits where they agree
//     are equal in every key, so only the low D = bits_for(OR ^ AND) bits need sorting: at C3
//     every depth lies in [2, 6) (keys 0x40000000..0x40BFFFFF, D = 24) and two passes do.
//     Pass 0's scan also stores D, tagged with the frame, into pinned host memory; the forward
//     waits for it while pass 0's downsweep runs and launches only the needed passes.  Callers
//     that do not wait launch all three and the unneeded ones exit at once (the kernels read D
//     from ctl).  The last
//     needed pass writes the permutation straight to `perm`;
//   * compaction: pass 0 drops the sentinel keys (0xFFFFFFFF: Gaussians without pairs in the
//     strip) and stores the kept count on the device; later passes read it.
// The frame's default form (gsr_depth_sort_msd, below) replaces the LSD passes by one MSD pass
// over the top 12 of the D bits and an in-LDS sort of every bucket by the rest.
// Each pass is three kernels: upsweep (per-tile 4096-bin histogram, LDS atomics), scan (per
// digit across tiles) and downsweep.  Between passes the (key, id) pairs travel as one 8-B
// word each.  The downsweep sorts its 4096-key tile in LDS by
// the 12-bit digit in two stable 6-bit sub-passes (wave-ballot ranking), then writes each key
// to digit start + tile offset + position in its digit run.  Every step keeps the tile order
// and the order within a tile, so each pass and the sort are stable: equal depths keep the
// Gaussian index order, as upstream's stable SortPairs does.
#include "radix_tile.h"

using namespace gsr;

namespace {

// 8 waves x 8 keys: 2 waves per SIMD, 91 VGPRs -- small enough to share a CU with two blocks
// of the second stream's colour pass (16 waves x 4 keys is as fast alone but does not fit
// beside them)
constexpr int kDW = 8;                  // waves per block
constexpr int kDThreads = kDW * 64;     // 512
constexpr int kDIt = 8;                 // keys per lane
constexpr int kDT = kDThreads * kDIt;   // 4096 keys per tile
constexpr int kDBits = 12;              // digit width
constexpr int kDBins = 1 << kDBits;     // 4096
constexpr int kDSub = 6;                // in-LDS sub-pass width
constexpr int kDSubBins = 1 << kDSub;   // 64
constexpr int kDPasses = 3;
static_assert(kDSubBins * kDW == kDThreads, "one thread per (sub-digit, wave) in the rank scan");
constexpr int kDPer = kDBins / kDThreads;  // digit starts per thread in the prologue
static_assert(kDPer == 8, "two 16-B loads of digit totals and of the hist row per thread");

// ctl: [0] kept count, [1] D (key bits to sort), [2] the MSD pass's shift and [3] the smallest
// kept key (gsr_msd_ctl: the MSD pass buckets key - min by its top 12 range bits; written by
// k_ds_bits or gsr_launch_count_pairs before the MSD pass), then per tile uint4 {OR, AND, kept,
// 0} of pass 0.  The MSD kernels read only ctl[2] and ctl[3]: the pass-0 scan also rewrites
// ctl[1] from the sort's own tiles (in the MSD form a diagnostic that debug forwards compare
// with the preprocess's D, api.hip wait_K).
//
// The MSD pass works on key - min (the range-relative key): every kept key is a positive
// float's bits, so key - min keeps the order, and its bits above the range's are 0.  Bucketing
// the top 12 of the range's bits, not of the bits that vary, keeps the buckets even where one
// outlier flips a high bit (a near Gaussian at depth 1.9 among depths in [2, 8): D = 31 but a
// range of 25 bits).  The pass writes range-relative keys; k_ds_local sorts them by the rest.
constexpr int kCtlHead = 4;

__device__ __forceinline__ int pass_bits(int shift) { return min(kDBits, 32 - shift); }

// kFirst: `in` is the n keys (uint32); else the previous pass's (key, id) pairs (uint2).
// msd (first pass only): the pass sorts the top 12 of the D varying key bits, shift ctl[2]
// (k_ds_bits), and k_ds_local finishes every bucket (gsr_depth_sort_msd).
template <bool kFirst>
__global__ __launch_bounds__(kDThreads) void k_ds_upsweep(const void *__restrict__ in,
                                                          int64_t n_host, int drop,
                                                          uint32_t *__restrict__ ctl, int shift,
                                                          uint32_t *__restrict__ hist,
                                                          const uint32_t *__restrict__ d_n,
                                                          int msd) {
    __shared__ uint32_t s_h[kDBins];
    __shared__ uint32_t s_red[3][kDW];
    if (kFirst && msd) shift = (int)ctl[2];
    const uint32_t kmin = (kFirst && msd) ? ctl[3] : 0u;  // range-relative MSD keys
    int64_t n = d_n ? (int64_t)*d_n : n_host;  // d_n: the compacted count (first pass)
    if (!kFirst) {
        if (ctl[1] <= (uint32_t)shift) return;  // constant digit: pass skipped
        n = ctl[0];
    }
    const int64_t base = (int64_t)blockIdx.x * kDT;
    if (base >= n) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nbins = 1 << pass_bits(shift);
    const uint32_t mask = (uint32_t)nbins - 1u;
    for (int i = tid; i < nbins; i += kDThreads) s_h[i] = 0u;
    __syncthreads();
    uint32_t vor = 0u, vand = 0xFFFFFFFFu, cnt = 0u;
    auto add = [&](uint32_t k) {
        if (kFirst && drop && k == kDropKey) return;
        atomicAdd(&s_h[((k - kmin) >> shift) & mask], 1u);
        if (kFirst) {
            vor |= k;
            vand &= k;
            ++cnt;
        }
    };
    if (kFirst) {
        const uint32_t *keys = static_cast<const uint32_t *>(in);
        if (base + kDT <= n) {
            const uint4 *k4 = reinterpret_cast<const uint4 *>(keys + base);
#pragma unroll
            for (int j = 0; j < kDIt / 4; ++j) {
                const uint4 q = k4[j * kDThreads + tid];
                add(q.x);
                add(q.y);
                add(q.z);
                add(q.w);
            }
        } else {
            for (int64_t e = base + tid; e < n; e += kDThreads) add(keys[e]);
        }
    } else {
        const uint2 *pairs = static_cast<const uint2 *>(in);
        if (base + kDT <= n) {
            const uint4 *p4 = reinterpret_cast<const uint4 *>(pairs + base);
#pragma unroll
            for (int j = 0; j < kDIt / 2; ++j) {
                const uint4 q = p4[j * kDThreads + tid];
                add(q.x);
                add(q.z);
            }
        } else {
            for (int64_t e = base + tid; e < n; e += kDThreads) add(pairs[e].x);
        }
    }
    __syncthreads();
    uint32_t *row = hist + (int64_t)blockIdx.x * kDBins;
    for (int i = tid; i < nbins; i += kDThreads) row[i] = s_h[i];
    if (kFirst) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            vor |= __shfl_xor(vor, o);
            vand &= __shfl_xor(vand, o);
            cnt += __shfl_xor(cnt, o);
        }
        if (lane == 0) {
            s_red[0][w] = vor;
            s_red[1][w] = vand;
            s_red[2][w] = cnt;
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t o = 0u, a = 0xFFFFFFFFu, c = 0u;
#pragma unroll
            for (int i = 0; i < kDW; ++i) {
                o |= s_red[0][i];
                a &= s_red[1][i];
                c += s_red[2][i];
            }
            reinterpret_cast<uint4 *>(ctl + kCtlHead)[blockIdx.x] = make_uint4(o, a, c, 0u);
        }
    }
}

// Block b: digits [16 b, 16 b + 16); thread t: digit 16 b + t % 16 over tile group t / 16 (a
// sixteenth of the tiles, loaded kScanReg at a time so the loads are in flight together; up to
// kScanReg tiles per thread -- 256 tiles, 1M keys -- stay in registers for the write-back
// instead of being loaded again).
// hist[t][d] becomes the exclusive count of digit d in tiles < t; digit_total[d] the count
// over all tiles.  Pass 0: the last block also reduces the tiles' {OR, AND, kept} into ctl[0]
// (kept) and ctl[1] (D).
constexpr int kScanDigits = 16, kScanGroups = 16, kScanReg = 16;
template <bool kFirst>
__global__ __launch_bounds__(256) void k_ds_scan(uint32_t *__restrict__ hist, int64_t n_host,
                                                 uint32_t *__restrict__ ctl, int shift,
                                                 uint32_t *__restrict__ digit_total,
                                                 const uint32_t *__restrict__ d_n,
                                                 unsigned long long *host_D, uint32_t tag,
                                                 int msd) {
    __shared__ uint32_t s_sum[kScanGroups][kScanDigits];
    __shared__ uint32_t s_red[3][4];
    if (kFirst && msd) shift = (int)ctl[2];
    int64_t n = d_n ? (int64_t)*d_n : n_host;
    if (!kFirst) {
        if (ctl[1] <= (uint32_t)shift) return;
        n = ctl[0];
    }
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t nt = (uint32_t)((n + kDT - 1) / kDT);
    const uint32_t nbins = 1u << pass_bits(shift);
    const int dl = tid % kScanDigits, g = tid / kScanDigits;
    const uint32_t d = blockIdx.x * kScanDigits + dl;
    if (blockIdx.x * kScanDigits < nbins) {
        const uint32_t t0 = (uint32_t)((uint64_t)nt * g / kScanGroups);
        const uint32_t t1 = (uint32_t)((uint64_t)nt * (g + 1) / kScanGroups);
        uint32_t *col = hist + d;
        uint32_t v[kScanReg], s = 0;
        const bool kept = t1 - t0 <= (uint32_t)kScanReg;  // one load round, values kept
        for (uint32_t t = t0; t < t1; t += kScanReg) {
#pragma unroll
            for (int r = 0; r < kScanReg; ++r)
                v[r] = t + r < t1 ? col[(int64_t)(t + r) * kDBins] : 0u;
#pragma unroll
            for (int r = 0; r < kScanReg; ++r) s += v[r];
        }
        s_sum[g][dl] = s;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int i = 0; i < kScanGroups; ++i) {
            const uint32_t x = s_sum[i][dl];
            pre += i < g ? x : 0u;
            tot += x;
        }
        for (uint32_t t = t0; t < t1; t += kScanReg) {
            if (!kept) {
#pragma unroll
                for (int r = 0; r < kScanReg; ++r)
                    v[r] = t + r < t1 ? col[(int64_t)(t + r) * kDBins] : 0u;
            }
#pragma unroll
            for (int r = 0; r < kScanReg; ++r) {
                if (t + r < t1) col[(int64_t)(t + r) * kDBins] = pre;
                pre += v[r];
            }
        }
        if (g == 0) digit_total[d] = tot;
    }
    if (kFirst && blockIdx.x == gridDim.x - 1) {
        const uint4 *st = reinterpret_cast<const uint4 *>(ctl + kCtlHead);
        uint32_t o = 0u, a = 0xFFFFFFFFu, c = 0u;
        for (uint32_t t = tid; t < nt; t += 256) {
            const uint4 v = st[t];
            if (v.z) {  // tiles whose keys were all dropped carry no bits
                o |= v.x;
                a &= v.y;
                c += v.z;
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            o |= __shfl_xor(o, off);
            a &= __shfl_xor(a, off);
            c += __shfl_xor(c, off);
        }
        if (lane == 0) {
            s_red[0][w] = o;
            s_red[1][w] = a;
            s_red[2][w] = c;
        }
        __syncthreads();
        if (tid == 0) {
            o = 0u;
            a = 0xFFFFFFFFu;
            c = 0u;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                o |= s_red[0][i];
                a &= s_red[1][i];
                c += s_red[2][i];
            }
            const uint32_t diff = c ? (o ^ a) : 0u;
            const uint32_t D = diff ? 32u - (uint32_t)__clz(diff) : 0u;
            ctl[0] = c;
            ctl[1] = D;
            // D for the host, tagged with the frame (pinned memory, system scope): it launches
            // only the passes D needs, while this pass's downsweep runs
            if (host_D)
                __hip_atomic_store(host_D, ((unsigned long long)tag << 32) | D, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// Stable rank of the tile's kept elements by kBits key bits at `shift` and scatter into
// s_keys / s_vals in that order (element order: wave, then item, then lane).  Returns the
// number of kept elements.  s_wcnt: kDW x kDSubBins counters, index wave * 64 + digit (distinct
// digits of a wave hit distinct banks).
//
// Per item, each lane finds the lanes of its wave holding its digit with one ballot per bit:
// m &= ~(ballot(bit) ^ f), f = the lane's own bit sign-extended to a full mask (one v_bitop3
// per 32-bit half); its rank is the count of those lanes below it, and every matching lane
// stores the same new running count.
// kBits = 0: the digit width is the runtime rt_bits (1..6; one instantiation for every width).
template <int kBits, int kIt = kDIt>
__device__ __forceinline__ int tile_rank_scatter(const uint32_t (&k)[kIt],
                                                 const uint32_t (&v)[kIt], uint32_t keep,
                                                 int shift, uint32_t *s_keys, uint32_t *s_vals,
                                                 uint32_t *s_wcnt, uint32_t *s_tmp,
                                                 int rt_bits = kBits) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int nbits = kBits > 0 ? kBits : rt_bits;
    const uint32_t kMask = (1u << nbits) - 1u;
    s_wcnt[tid] = 0u;
    __syncthreads();
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t *wcnt = s_wcnt + w * kDSubBins;
    uint32_t rank[kIt];
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
        const bool kp = (keep >> j) & 1u;
        const uint32_t d = (k[j] >> shift) & kMask;
        const uint64_t m0 = __ballot(kp);
        uint32_t mlo = (uint32_t)m0, mhi = (uint32_t)(m0 >> 32);
#pragma unroll
        for (int b = 0; b < (kBits > 0 ? kBits : kDSub); ++b) {
            if (kBits == 0 && b >= nbits) break;
            const uint32_t f = (uint32_t)(((int32_t)(d << (31 - b))) >> 31);
            const uint64_t bal = __ballot(f != 0u);
            mlo &= ~((uint32_t)bal ^ f);
            mhi &= ~((uint32_t)(bal >> 32) ^ f);
        }
        const uint64_t m = ((uint64_t)mhi << 32) | mlo;
        const uint32_t prior = wcnt[d];
        rank[j] = prior + (uint32_t)__popcll(m & lt);
        if (kp) wcnt[d] = prior + (uint32_t)__popcll(m);  // same value from every match
    }
    __syncthreads();
    // exclusive scan in (digit, wave) order: thread t = digit * kDW + wave
    const int sd = tid / kDW, sw = tid % kDW;
    uint32_t total;
    const uint32_t c = s_wcnt[sw * kDSubBins + sd];
    const uint32_t pre = blockw_exclusive_scan<kDW>(c, s_tmp, total);
    s_wcnt[sw * kDSubBins + sd] = pre;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
        if (!((keep >> j) & 1u)) continue;
        const uint32_t d = (k[j] >> shift) & kMask;
        const uint32_t pos = wcnt[d] + rank[j];
        s_keys[pos] = k[j];
        s_vals[pos] = v[j];
    }
    __syncthreads();
    return (int)total;
}

// kFirst: `in` is the n keys and the values are the element indices (or ids_in[e]); else `in` is the
// previous pass's (key, id) pairs.  last (decided from D on the device): write only the ids,
// to perm; else the (key, id) pairs to pairs_out.
template <bool kFirst>
__global__ __launch_bounds__(kDThreads) void k_ds_downsweep(
    const void *__restrict__ in, uint2 *__restrict__ pairs_out, uint32_t *__restrict__ perm,
    int64_t n_host, int drop, const uint32_t *__restrict__ ctl, int shift,
    const uint32_t *__restrict__ hist, const uint32_t *__restrict__ digit_total,
    const uint32_t *__restrict__ ids_in, const uint32_t *__restrict__ d_n, int msd) {
    __shared__ uint32_t s_keys[kDT], s_vals[kDT], s_tab[kDBins];  // 48 KiB
    __shared__ uint32_t s_wcnt[kDSubBins * kDW];
    __shared__ uint32_t s_tmp[kDW];
    const uint32_t D = ctl[1];
    if (kFirst && msd) shift = (int)ctl[2];
    const uint32_t kmin = (kFirst && msd) ? ctl[3] : 0u;  // range-relative MSD keys
    int64_t n = d_n ? (int64_t)*d_n : n_host;
    if (!kFirst) {
        if (D <= (uint32_t)shift) return;
        n = ctl[0];
    }
    const uint32_t tile = xcd_run_block(blockIdx.x);
    const int64_t base = (int64_t)tile * kDT;
    if (base >= n) return;
    const int nbits = pass_bits(shift);
    // msd: the pass sorted the top digit; it is the whole sort only when D <= 12 (shift 0)
    const bool last = (kFirst && msd) ? ctl[2] == 0u
                                      : shift + nbits >= 32 || D <= (uint32_t)(shift + nbits);
    const uint32_t nbins = 1u << nbits, mask = nbins - 1u;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;

    uint32_t k[kDIt], v[kDIt], keep = 0u;
#pragma unroll
    for (int j = 0; j < kDIt; ++j) {
        const int64_t e = base + w * (kDT / kDW) + j * 64 + lane;
        const bool valid = e < n;
        if (kFirst) {
            k[j] = valid ? static_cast<const uint32_t *>(in)[e] : 0u;
            v[j] = (ids_in && valid) ? ids_in[e] : (uint32_t)e;
        } else {
            const uint2 q = valid ? static_cast<const uint2 *>(in)[e] : make_uint2(0u, 0u);
            k[j] = q.x;
            v[j] = q.y;
        }
        if (valid && !(kFirst && drop && k[j] == kDropKey)) keep |= 1u << j;
        k[j] -= kmin;  // (MSD: ranked, bucketed and written range-relative)
    }
    // s_tab[d] = start of digit d overall + its count in earlier tiles (8 digits per thread:
    // the exclusive scan of the digit totals plus this tile's row of the scanned histogram)
    {
        const uint32_t d0 = (uint32_t)tid * kDPer;
        uint4 c0 = make_uint4(0u, 0u, 0u, 0u), c1 = c0, h0 = c0, h1 = c0;
        if (d0 < nbins) {
            const uint4 *t4 = reinterpret_cast<const uint4 *>(digit_total + d0);
            const uint4 *h4 = reinterpret_cast<const uint4 *>(hist + (int64_t)tile * kDBins + d0);
            c0 = t4[0];
            c1 = t4[1];
            h0 = h4[0];
            h1 = h4[1];
        }
        const uint32_t c[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
        const uint32_t h[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
        uint32_t sum = 0, tot;
#pragma unroll
        for (int i = 0; i < 8; ++i) sum += c[i];
        uint32_t pre = blockw_exclusive_scan<kDW>(sum, s_tmp, tot);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            s_tab[d0 + i] = pre + h[i];
            pre += c[i];
        }
    }
    // every pass has >= 8 bits: sub-pass A takes 6, sub-pass B the remaining 6 or 2
    int kept = tile_rank_scatter<kDSub>(k, v, keep, shift, s_keys, s_vals, s_wcnt, s_tmp);
    if (nbits > kDSub) {
        keep = 0u;
#pragma unroll
        for (int j = 0; j < kDIt; ++j) {
            const int p = w * (kDT / kDW) + j * 64 + lane;
            if (p < kept) {
                k[j] = s_keys[p];
                v[j] = s_vals[p];
                keep |= 1u << j;
            }
        }
        __syncthreads();  // every lane holds its elements before the LDS is overwritten
        kept = nbits - kDSub == kDSub
                   ? tile_rank_scatter<kDSub>(k, v, keep, shift + kDSub, s_keys, s_vals, s_wcnt,
                                              s_tmp)
                   : tile_rank_scatter<2>(k, v, keep, shift + kDSub, s_keys, s_vals, s_wcnt,
                                          s_tmp);
    }
    // s_tab[d] <- global position of the tile's first digit-d key, minus its tile position
    for (int i = tid; i < kept; i += kDThreads) {
        const uint32_t d = (s_keys[i] >> shift) & mask;
        if (i == 0 || ((s_keys[i - 1] >> shift) & mask) != d) s_tab[d] -= (uint32_t)i;
    }
    __syncthreads();
    for (int i = tid; i < kept; i += kDThreads) {
        const uint32_t kk = s_keys[i];
        const uint32_t g = s_tab[(kk >> shift) & mask] + (uint32_t)i;
        if (last)
            perm[g] = s_vals[i];
        else
            pairs_out[g] = make_uint2(kk, s_vals[i]);
    }
}

// Compacting front end: exclusive scan of the per-256-block kept counts in place (one block),
// total -> ctl[0].  Rounds of 16k counts: each thread owns 16 consecutive counts (four 16-B
// loads issued together, a wave covers 4 KB contiguous), one block scan per round.  (A strided
// per-thread serial loop was 47 us at 6M Gaussians: ~23 dependent loads per thread.)
__global__ __launch_bounds__(1024) void k_ds_compact_scan(uint32_t *__restrict__ block_kept,
                                                          int64_t nb, uint32_t *__restrict__ ctl) {
    constexpr int kR = 4, kPer = 4 * kR;
    __shared__ uint32_t s_tmp[16];
    const int tid = threadIdx.x;
    uint32_t carry = 0;
    for (int64_t base = 0; base < nb; base += 1024 * kPer) {
        const int64_t e0 = base + (int64_t)tid * kPer;
        uint32_t c[kPer];
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            const int64_t e = e0 + 4 * r;
            if (e + 3 < nb) {
                const uint4 v = *reinterpret_cast<const uint4 *>(block_kept + e);
                c[4 * r] = v.x, c[4 * r + 1] = v.y, c[4 * r + 2] = v.z, c[4 * r + 3] = v.w;
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) c[4 * r + q] = e + q < nb ? block_kept[e + q] : 0u;
            }
        }
        uint32_t sum = 0;
#pragma unroll
        for (int q = 0; q < kPer; ++q) sum += c[q];
        uint32_t total;
        uint32_t pre = carry + blockw_exclusive_scan<16>(sum, s_tmp, total);
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            const int64_t e = e0 + 4 * r;
            uint32_t o[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = pre, pre += c[4 * r + q];
            if (e + 3 < nb) {
                *reinterpret_cast<uint4 *>(block_kept + e) = make_uint4(o[0], o[1], o[2], o[3]);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (e + q < nb) block_kept[e + q] = o[q];
            }
        }
        carry += total;
    }
    if (tid == 0) ctl[0] = carry;
}

// Block b (256 keys): its kept keys (not 0xFFFFFFFF), in order, to keys_c / ids_c from offset
// block_off[b].
__global__ __launch_bounds__(256) void k_ds_compact(const uint32_t *__restrict__ keys, int64_t n,
                                                    const uint32_t *__restrict__ block_off,
                                                    uint32_t *__restrict__ keys_c,
                                                    uint32_t *__restrict__ ids_c,
                                                    uint32_t *__restrict__ ids_copy) {
    __shared__ uint32_t s_w[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int64_t idx = (int64_t)blockIdx.x * 256 + tid;
    const uint32_t key = idx < n ? keys[idx] : kDropKey;
    const bool keep = key != kDropKey;
    const uint64_t bal = __ballot(keep);
    if (lane == 0) s_w[w] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t base = block_off[blockIdx.x];
    for (int i = 0; i < w; ++i) base += s_w[i];
    if (keep) {
        const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        const uint32_t dst = base + (uint32_t)__popcll(bal & lt);
        keys_c[dst] = key;
        ids_c[dst] = (uint32_t)idx;
        if (ids_copy) ids_copy[dst] = (uint32_t)idx;  // outlives ids_c (the colour pass reads it)
    }
}

// ---- MSD first pass + per-bucket local sort (the frame's depth sort, gsr_depth_sort_msd) -------
// The LSD sort needs one up/scan/down pass per 12 key bits (two at C3, D = 24).  Here the one
// global pass sorts the TOP 12 of the D varying bits (MSD: the keys land in 4096 buckets, each
// bucket contiguous and stably ordered), and k_ds_local then sorts every bucket by the remaining
// D - 12 bits in LDS -- one kernel instead of the second up/scan/down pass.  Buckets concatenated
// in digit order, each sorted stably by its low bits, give the stable sort by the whole key.

// D (the bits in which the kept keys differ) from the preprocess blocks' OR / AND of their kept
// depth keys (GsrPreprocessArgs.block_pairs), as k_ds_scan derives it from the sort's own tiles:
// ctl[1] = D, ctl[2] = the MSD pass's shift.  A kept key is a positive float's bits (depth >
// 0.2), never 0, so OR == 0 means no kept key (D = 0).
__global__ __launch_bounds__(1024) void k_ds_bits(const uint2 *__restrict__ keybits, int64_t nb,
                                                  uint32_t *__restrict__ ctl) {
    __shared__ uint32_t s_max[16], s_min[16];
    uint32_t mx = 0u, mn = 0xFFFFFFFFu;  // the preprocess blocks' {largest, smallest} kept key
    constexpr int kU = 8;  // loads in flight per thread
    for (int64_t i0 = threadIdx.x; i0 < nb; i0 += kU * 1024) {
        uint2 kb[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int64_t i = i0 + (int64_t)u * 1024;
            kb[u] = i < nb ? keybits[i] : make_uint2(0u, 0xFFFFFFFFu);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) mx = max(mx, kb[u].x), mn = min(mn, kb[u].y);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        mx = max(mx, (uint32_t)__shfl_xor(mx, off));
        mn = min(mn, (uint32_t)__shfl_xor(mn, off));
    }
    if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = mx, s_min[threadIdx.x >> 6] = mn;
    __syncthreads();
    if (threadIdx.x == 0) {
        mx = 0u, mn = 0xFFFFFFFFu;
        for (int i = 0; i < 16; ++i) mx = max(mx, s_max[i]), mn = min(mn, s_min[i]);
        gsr_msd_ctl(key_bits(mx, mn), ctl);
    }
}

constexpr int kLGroup = kDW;                // buckets per k_ds_local block: one per wave
constexpr int kLWave = 1024;                // keys a wave sorts alone (16 per lane)
constexpr int kLIt = 8;                     // elements per lane of an in-LDS bucket sort
constexpr int kLCap = kDThreads * kLIt;     // 4096 elements sorted in LDS at once
constexpr int kLSub = kDSub;                // 6-bit sub-passes
// LDS keys (and ids) the waves' slices share: 4096 (45 KB a block), or 8192 (77 KB) on frames
// whose buckets of 513-1024 keys crowd a group past 4096 (k_ds_local's wide form, chosen by the
// host from the flag the previous frames raised)
constexpr int kLSlotsNarrow = kLCap, kLSlotsWide = 2 * kLCap;
static_assert(kLCap >= kDW * 512, "every bucket of <= 512 keys gets a wave slice");

template <int kSlots>
struct LocalSmem {
    uint32_t keys[kSlots], vals[kSlots];
    RadixTileSmem<kDW, kLIt> rt;  // 8-bit sub-passes (radix_tile_scatter, in LDS only)
    uint32_t wcnt[kDSubBins * kDW];
    uint32_t tmp[kDW];
    uint32_t start[kLGroup + 1];  // the group's bucket starts (+ its end)
    int32_t slice[kLGroup];       // each bucket's wave slice (wave_slices), -1: the block's
    uint32_t base[kDSubBins], cstart[kDSubBins], ccount[kDSubBins];  // the slow path
};

// One sub-pass of `bits` (1..6) of the slow path's chunk ranking (runtime width).
template <typename Smem>
__device__ __forceinline__ int local_rank(const uint32_t (&k)[kLIt], const uint32_t (&v)[kLIt],
                                          uint32_t keep, int shift, int bits, Smem &sm) {
    return tile_rank_scatter<0, kLIt>(k, v, keep, shift, sm.keys, sm.vals, sm.wcnt, sm.tmp, bits);
}

// Stable in-LDS sort of the n <= kLCap pairs at src[b0, b0 + n) -- consecutive buckets, already
// in bucket order -- by the local key ((bucket - d0) << low) | (key & low mask) of `bits` bits,
// in 8-bit sub-passes (radix_tile_scatter: element order wave, item, lane; elements past n carry
// the largest key and sort last); the sorted ids go to perm[b0 ...].
template <typename Smem>
__device__ void local_sort_lds(const uint2 *__restrict__ src, uint32_t *__restrict__ perm,
                               uint32_t b0, uint32_t n, uint32_t shift_hi, uint32_t d0, int low,
                               int bits, Smem &sm) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t lmask = (1u << low) - 1u;
    uint32_t k[kLIt], v[kLIt];
#pragma unroll
    for (int j = 0; j < kLIt; ++j) {
        const uint32_t e = (uint32_t)(w * (kLCap / kDW) + j * 64 + lane);
        k[j] = 0xFFFFFFFFu;
        v[j] = 0u;
        if (e < n) {
            const uint2 q = src[b0 + e];
            k[j] = ((((q.x >> shift_hi) & (kDBins - 1u)) - d0) << low) | (q.x & lmask);
            v[j] = q.y;
        }
    }
    for (int sh = 0; sh < bits; sh += 8) {
        if (sh > 0) {  // reload the previous sub-pass's order (the first n entries)
#pragma unroll
            for (int j = 0; j < kLIt; ++j) {
                const uint32_t p = (uint32_t)(w * (kLCap / kDW) + j * 64 + lane);
                k[j] = p < n ? sm.keys[p] : 0xFFFFFFFFu;
                v[j] = p < n ? sm.vals[p] : 0u;
            }
            __syncthreads();  // every lane holds its elements before the LDS is overwritten
        }
        radix_tile_scatter<kDW, kLIt, false, false>(k, v, (int)n, sh, min(8, bits - sh), nullptr,
                                                    0, 0u, nullptr, nullptr, nullptr, sm.rt,
                                                    sm.keys, sm.vals);
    }
    for (uint32_t i = tid; i < n; i += kDThreads) perm[b0 + i] = sm.vals[i];
    __syncthreads();  // the LDS is reused by the caller's next sort
}

// The slow path for one bucket of n > kLCap pairs at src[b0 ...]: a stable LSD over its `low`
// key bits in 6-bit sub-passes through global memory (ping-pong src <-> tmp at the same
// offsets; the last sub-pass writes the ids to perm), the block walking the bucket in 4096-pair
// chunks: count the digits, scan, then per chunk rank it in LDS and place every digit's run at
// that digit's running offset.  Only a degenerate scene (more than 8192 kept Gaussians sharing
// the top 12 of the varying depth bits) takes it.
template <typename Smem>
__device__ void local_sort_big(uint2 *__restrict__ src, uint2 *__restrict__ tmp,
                               uint32_t *__restrict__ perm, uint32_t b0, uint32_t n, int low,
                               Smem &sm) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    if (low == 0) {
        for (uint32_t e = tid; e < n; e += kDThreads) perm[b0 + e] = src[b0 + e].y;
        return;
    }
    uint2 *a = src, *b = tmp;
    for (int sh = 0; sh < low; sh += kLSub) {
        const int bits = min(kLSub, low - sh);
        const uint32_t mask = (1u << bits) - 1u;
        const bool last = sh + kLSub >= low;
        if (tid < kDSubBins) sm.base[tid] = 0u;
        __syncthreads();
        for (uint32_t e = tid; e < n; e += kDThreads) atomicAdd(&sm.base[(a[b0 + e].x >> sh) & mask], 1u);
        __syncthreads();
        if (tid == 0) {
            uint32_t run = 0u;
            for (int d = 0; d < kDSubBins; ++d) {
                const uint32_t c = sm.base[d];
                sm.base[d] = run;
                run += c;
            }
        }
        __syncthreads();
        for (uint32_t c0 = 0; c0 < n; c0 += (uint32_t)kLCap) {
            const uint32_t m = min((uint32_t)kLCap, n - c0);
            uint32_t k[kLIt], v[kLIt], keep = 0u;
#pragma unroll
            for (int j = 0; j < kLIt; ++j) {
                const uint32_t e = (uint32_t)(w * (kLCap / kDW) + j * 64 + lane);
                k[j] = v[j] = 0u;
                if (e < m) {
                    const uint2 q = a[b0 + c0 + e];
                    k[j] = q.x;
                    v[j] = q.y;
                    keep |= 1u << j;
                }
            }
            const int kept = local_rank(k, v, keep, sh, bits, sm);
            // the chunk's digit runs: start and count of every digit
            if (tid < kDSubBins) sm.ccount[tid] = 0u;
            __syncthreads();
            for (int i = tid; i < kept; i += kDThreads) {
                const uint32_t d = (sm.keys[i] >> sh) & mask;
                if (i == 0 || ((sm.keys[i - 1] >> sh) & mask) != d) sm.cstart[d] = (uint32_t)i;
                if (i == kept - 1 || ((sm.keys[i + 1] >> sh) & mask) != d)
                    sm.ccount[d] = (uint32_t)i + 1u;  // end (count = end - start below)
            }
            __syncthreads();
            for (int i = tid; i < kept; i += kDThreads) {
                const uint32_t d = (sm.keys[i] >> sh) & mask;
                const uint32_t g = sm.base[d] + ((uint32_t)i - sm.cstart[d]);
                if (last)
                    perm[b0 + g] = sm.vals[i];
                else
                    b[b0 + g] = make_uint2(sm.keys[i], sm.vals[i]);
            }
            __syncthreads();
            if (tid < kDSubBins && sm.ccount[tid]) sm.base[tid] += sm.ccount[tid] - sm.cstart[tid];
            __syncthreads();
        }
        uint2 *t = a;
        a = b;
        b = t;
    }
}

// One wave sorts the n <= kLWave pairs of one bucket at src[b0 ...] by their low `low` key bits,
// stably, alone: 8 pairs per lane (element j * 64 + lane), 6-bit sub-passes ranked with one
// ballot per bit against a per-wave digit count in LDS (the lanes of a wave are in lockstep, so
// no block barrier: the wavefront fences only keep the compiler from moving LDS accesses across
// the hand-offs), scattered into the wave's LDS slice; the ids go to perm[b0 ...].
template <int kIt>
__device__ __forceinline__ void wave_sort_bucket(const uint2 *__restrict__ src,
                                                 uint32_t *__restrict__ perm, uint32_t b0,
                                                 uint32_t n, int low, uint32_t *s_keys,
                                                 uint32_t *s_vals, uint32_t *cnt) {
    const int lane = threadIdx.x & 63;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint32_t lmask = (1u << low) - 1u;
    static_assert(kIt * 64 <= kLWave, "the wave's LDS slice");
    // 16 keys per lane: each key's rank rides in its bits 16+ (low <= 16, rank < 1024), so the
    // lane holds 32 words instead of 48
    constexpr bool kPack = kIt > 8;
    constexpr uint32_t kKeyMask = kPack ? 0xFFFFu : 0xFFFFFFFFu;
    uint32_t k[kIt], v[kIt];
    // no branches around the loads (the slots past n are masked by `valid` below): branches
    // here make the compiler copy the whole key and id arrays at every join
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
        const uint32_t e = (uint32_t)(j * 64 + lane);
        const uint2 q = src[b0 + min(e, n - 1u)];
        k[j] = q.x & lmask;
        v[j] = q.y;
    }
    for (int sh = 0; sh < low; sh += kDSub) {
        const int bits = min(kDSub, low - sh);
        const uint32_t mask = (1u << bits) - 1u;
        cnt[lane] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t rank[kPack ? 1 : kIt];
#pragma unroll
        for (int j = 0; j < kIt; ++j) {
            const bool valid = (uint32_t)(j * 64 + lane) < n;
            const uint32_t d = (k[j] >> sh) & mask;  // (kPack: the rank bits are still 0 here)
            const uint64_t m0 = __ballot(valid);
            uint32_t mlo = (uint32_t)m0, mhi = (uint32_t)(m0 >> 32);
#pragma unroll
            for (int b = 0; b < kDSub; ++b) {
                if (b >= bits) break;
                const uint32_t f = (uint32_t)(((int32_t)(d << (31 - b))) >> 31);
                const uint64_t bal = __ballot(f != 0u);
                mlo &= ~((uint32_t)bal ^ f);
                mhi &= ~((uint32_t)(bal >> 32) ^ f);
            }
            const uint64_t m = ((uint64_t)mhi << 32) | mlo;
            const uint32_t prior = cnt[d];
            if constexpr (kPack)
                k[j] |= (prior + (uint32_t)__popcll(m & lt)) << 16;
            else
                rank[j] = prior + (uint32_t)__popcll(m & lt);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            if (valid) cnt[d] = prior + (uint32_t)__popcll(m);  // same value from every match
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        // exclusive scan of the 64 digit counts (one per lane)
        const uint32_t c = cnt[lane];
        const uint32_t ex = wave_inclusive_scan(c) - c;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        cnt[lane] = ex;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int j = 0; j < kIt; ++j) {
            if ((uint32_t)(j * 64 + lane) >= n) continue;
            const uint32_t kj = k[j] & kKeyMask;
            const uint32_t pos = cnt[(kj >> sh) & mask] + (kPack ? k[j] >> 16 : rank[kPack ? 0 : j]);
            s_keys[pos] = kj;
            s_vals[pos] = v[j];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        // Invariant: the slice's slots past n hold stale LDS data (earlier blocks' keys, whose
        // bits 16+ may be set).  Such an item is never valid (e >= n): its digit never reaches
        // a ballot's valid mask, cnt or a store, and the kPack rank bits OR-ed into it are never
        // read.  Every key at a slot < n was stored masked (kj above).
        for (int j = 0; j < kIt; ++j) {
            k[j] = s_keys[j * 64 + lane];
            v[j] = s_vals[j * 64 + lane];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
        const uint32_t e = (uint32_t)(j * 64 + lane);
        if (e < n) perm[b0 + e] = v[j];
    }
}

// LDS slots a wave needs to sort a bucket of n keys alone (2, 4, 8 or 16 keys per lane: the
// ranking work is per item), 0 when the block sorts it (past 1024 keys, or key bits above the 16
// the 16-key form packs its ranks over)
__device__ __forceinline__ uint32_t wave_slots(uint32_t n, int low) {
    return n == 0u     ? 0u
           : n <= 128u ? 128u
           : n <= 256u ? 256u
           : n <= 512u ? 512u
           : (n <= (uint32_t)kLWave && low <= 16) ? (uint32_t)kLWave
                                                  : 0u;
}

// The LDS slice (first slot) where the wave of each bucket of the group sorts it, -1 when the
// block sorts it (one thread plans, from the group's bucket sizes in registers): the buckets of
// <= 512 keys get theirs first (at most 8 x 512 slots), then those of <= 1024 keys in bucket
// order while the `slots` last.  Returns whether a bucket of <= 1024 keys was left to the block.
__device__ __forceinline__ bool wave_slices(const uint32_t (&cnt)[kLGroup], int low,
                                            uint32_t slots, int32_t *slice) {
    uint32_t used = 0u;
    bool left = false;
#pragma unroll
    for (int i = 0; i < kLGroup; ++i) {
        const uint32_t need = wave_slots(cnt[i], low);
        slice[i] = -1;
        if (need && need <= 512u) {
            slice[i] = (int32_t)used;
            used += need;
        }
    }
#pragma unroll
    for (int i = 0; i < kLGroup; ++i) {
        const uint32_t need = wave_slots(cnt[i], low);
        if (need != (uint32_t)kLWave) continue;
        if (used + need > slots) {
            left = true;
            continue;
        }
        slice[i] = (int32_t)used;
        used += need;
    }
    return left;
}

// Block g: buckets [8 g, 8 g + 8) of the MSD pass's output (pairs in bucket order; bucket d
// starts at the exclusive sum of digit_total[0, d)), one per wave: a bucket of <= 1024 keys (all
// of them at C3, D = 24: at most ~500; C5's up to ~870) is sorted by its wave alone in its own
// slice of the block's kSlots LDS slots (wave_slices); the rest (4K frames: up to ~2,800 keys)
// by the whole block in LDS after the waves, in 8-bit sub-passes; past 4096 keys by the slow
// path.  D <= 12: the MSD pass was the whole sort.  A group whose buckets of 513-1024 keys do
// not all fit 4096 slots stores the frame's tag to host_crowd (pinned; NULL: none), from which
// the host picks the wide form for the next frames.  (128 VGPRs: the 16-key form's arrays fit
// without spills.)
template <int kSlots>
__global__ __launch_bounds__(kDThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_ds_local(
    uint2 *__restrict__ pairs, uint2 *__restrict__ tmp, uint32_t *__restrict__ perm,
    const uint32_t *__restrict__ ctl, const uint32_t *__restrict__ digit_total,
    unsigned long long *__restrict__ host_crowd, uint32_t tag) {
    __shared__ LocalSmem<kSlots> sm;
    // the bits below the MSD digit: the MSD pass's own shift (ctl[2]); 0 when D <= 12
    const int low = (int)ctl[2];
    if (low == 0) return;
    const uint32_t shift_hi = (uint32_t)low;
    const int tid = threadIdx.x, w = tid >> 6;
    const uint32_t d0 = blockIdx.x * kLGroup;
    // the group's start: the digit totals before it (8 per thread, one block sum)
    {
        uint32_t acc = 0u;
#pragma unroll
        for (int i = 0; i < kDPer; ++i) {
            const uint32_t d = (uint32_t)tid * kDPer + i;
            acc += d < d0 ? digit_total[d] : 0u;
        }
        uint32_t total;
        blockw_exclusive_scan<kDW>(acc, sm.tmp, total);
        if (tid == 0) {
            uint32_t run = total, cnt[kLGroup];
#pragma unroll
            for (int i = 0; i < kLGroup; ++i) {
                cnt[i] = digit_total[d0 + i];
                sm.start[i] = run;
                run += cnt[i];
            }
            sm.start[kLGroup] = run;
            const bool crowded = wave_slices(cnt, low, (uint32_t)kLSlotsNarrow, sm.slice);
            if (kSlots != kLSlotsNarrow) wave_slices(cnt, low, (uint32_t)kSlots, sm.slice);
            if (crowded && host_crowd)
                __hip_atomic_store(host_crowd, (unsigned long long)tag, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
    }
    {
        const uint32_t b0 = sm.start[w], bn = sm.start[w + 1] - b0;
        const int slice = sm.slice[w];
        uint32_t *sk = sm.keys + slice, *sv = sm.vals + slice;
        uint32_t *sc = sm.wcnt + w * kDSubBins;
        if (slice < 0) {
        } else if (bn <= 128u) {
            wave_sort_bucket<2>(pairs, perm, b0, bn, low, sk, sv, sc);
        } else if (bn <= 256u) {
            wave_sort_bucket<4>(pairs, perm, b0, bn, low, sk, sv, sc);
        } else if (bn <= 512u) {
            wave_sort_bucket<8>(pairs, perm, b0, bn, low, sk, sv, sc);
        } else {
            wave_sort_bucket<16>(pairs, perm, b0, bn, low, sk, sv, sc);
        }
    }
    __syncthreads();
    for (int i = 0; i < kLGroup; ++i) {  // the rest, one at a time by the block
        const uint32_t b0 = sm.start[i], bn = sm.start[i + 1] - b0;
        if (bn == 0u || sm.slice[i] >= 0) continue;  // (a wave sorted it)
        if (bn <= (uint32_t)kLCap)
            local_sort_lds(pairs, perm, b0, bn, shift_hi, d0 + (uint32_t)i, low, low, sm);
        else
            local_sort_big(pairs, tmp, perm, b0, bn, low, sm);
        __syncthreads();
    }
}

}  // namespace

int64_t gsr_depth_sort_hist_words(int64_t n) {
    const int64_t nt = (n + kDT - 1) / kDT;
    return (nt < 1 ? 1 : nt) * kDBins;
}

int64_t gsr_depth_sort_ctl_words(int64_t n) { return kCtlHead + 4 * ((n + kDT - 1) / kDT + 1); }

int gsr_depth_sort_digit_words() { return kDBins; }

int gsr_depth_sort_passes(uint32_t key_bits) {
    return key_bits <= (uint32_t)kDBits ? 1 : key_bits <= (uint32_t)(2 * kDBits) ? 2 : kDPasses;
}

static hipError_t ds_passes(const uint32_t *keys, const uint32_t *ids_in, const uint32_t *d_n,
                            int64_t n, int drop, uint2 *pairs_a, uint2 *pairs_b, uint32_t *perm,
                            uint32_t *hist, uint32_t *digit_total, uint32_t *ctl, int pass_begin,
                            int pass_end, unsigned long long *host_D, uint32_t tag, hipStream_t s) {
    const unsigned nt = (unsigned)((n + kDT - 1) / kDT);
    const dim3 down_grid(xcd_run_grid(nt));  // (the downsweep's XCD runs)
    const void *in[kDPasses] = {keys, pairs_a, pairs_b};
    uint2 *out[kDPasses] = {pairs_a, pairs_b, nullptr};
    for (int p = pass_begin; p < pass_end; ++p) {
        const int shift = p * kDBits;
        if (p == 0) {
            hipLaunchKernelGGL(k_ds_upsweep<true>, dim3(nt), dim3(kDThreads), 0, s, in[p], n, drop,
                               ctl, shift, hist, d_n, 0);
            hipLaunchKernelGGL(k_ds_scan<true>, dim3(kDBins / kScanDigits), dim3(256), 0, s, hist,
                               n, ctl, shift, digit_total, d_n, host_D, tag, 0);
            hipLaunchKernelGGL(k_ds_downsweep<true>, down_grid, dim3(kDThreads), 0, s, in[p],
                               out[p], perm, n, drop, ctl, shift, hist, digit_total, ids_in, d_n,
                               0);
        } else {
            hipLaunchKernelGGL(k_ds_upsweep<false>, dim3(nt), dim3(kDThreads), 0, s, in[p], n, 0,
                               ctl, shift, hist, nullptr, 0);
            hipLaunchKernelGGL(k_ds_scan<false>, dim3(kDBins / kScanDigits), dim3(256), 0, s, hist,
                               n, ctl, shift, digit_total, nullptr, nullptr, 0u, 0);
            hipLaunchKernelGGL(k_ds_downsweep<false>, down_grid, dim3(kDThreads), 0, s, in[p],
                               out[p], perm, n, 0, ctl, shift, hist, digit_total, nullptr, nullptr,
                               0);
        }
    }
    return hipGetLastError();
}

hipError_t gsr_depth_sort(const uint32_t *keys, int64_t n, int drop, uint2 *pairs_a,
                          uint2 *pairs_b, uint32_t *perm, uint32_t *hist, uint32_t *digit_total,
                          uint32_t *ctl, int pass_begin, int pass_end, hipStream_t s,
                          unsigned long long *host_D, uint32_t tag) {
    if (n <= 0 || pass_begin >= pass_end) return hipSuccess;
    if (n > (int64_t)UINT32_MAX || pass_begin < 0 || pass_end > kDPasses)
        return hipErrorInvalidValue;
    return ds_passes(keys, nullptr, nullptr, n, drop, pairs_a, pairs_b, perm, hist, digit_total,
                     ctl, pass_begin, pass_end, host_D, tag, s);
}

// The MSD form over keys (drop: the kDropKey ones are dropped) or over compacted keys / ids_in
// whose count is *d_n (grids sized for n).
static void msd_launch(const uint32_t *keys, const uint32_t *ids_in, const uint32_t *d_n, int drop,
                       int64_t n, const uint2 *keybits, int64_t n_keybits, uint2 *pairs_a,
                       uint2 *pairs_b, uint32_t *perm, uint32_t *hist, uint32_t *digit_total,
                       uint32_t *ctl, hipStream_t s, unsigned long long *host_D, uint32_t tag,
                       unsigned long long *host_crowd, int wide) {
    const unsigned nt = (unsigned)((n + kDT - 1) / kDT);
    if (keybits)  // (else ctl[1], ctl[2] are set: gsr_launch_count_pairs on this stream)
        hipLaunchKernelGGL(k_ds_bits, dim3(1), dim3(1024), 0, s, keybits, n_keybits, ctl);
    hipLaunchKernelGGL(k_ds_upsweep<true>, dim3(nt), dim3(kDThreads), 0, s, keys, n, drop, ctl, 0,
                       hist, d_n, 1);
    hipLaunchKernelGGL(k_ds_scan<true>, dim3(kDBins / kScanDigits), dim3(256), 0, s, hist, n, ctl,
                       0, digit_total, d_n, host_D, tag, 1);
    hipLaunchKernelGGL(k_ds_downsweep<true>, dim3(xcd_run_grid(nt)),
                       dim3(kDThreads), 0, s, keys, pairs_a, perm, n, drop, ctl, 0, hist,
                       digit_total, ids_in, d_n, 1);
    if (wide)
        hipLaunchKernelGGL(k_ds_local<kLSlotsWide>, dim3(kDBins / kLGroup), dim3(kDThreads), 0, s,
                           pairs_a, pairs_b, perm, ctl, digit_total, host_crowd, tag);
    else
        hipLaunchKernelGGL(k_ds_local<kLSlotsNarrow>, dim3(kDBins / kLGroup), dim3(kDThreads), 0,
                           s, pairs_a, pairs_b, perm, ctl, digit_total, host_crowd, tag);
}

hipError_t gsr_depth_sort_msd(const uint32_t *keys, int64_t n, const uint2 *keybits,
                              int64_t n_keybits, uint2 *pairs_a, uint2 *pairs_b, uint32_t *perm,
                              uint32_t *hist, uint32_t *digit_total, uint32_t *ctl, hipStream_t s,
                              unsigned long long *host_D, uint32_t tag,
                              unsigned long long *host_crowd, int wide) {
    if (n <= 0) return hipSuccess;
    if (n > (int64_t)UINT32_MAX) return hipErrorInvalidValue;
    msd_launch(keys, nullptr, nullptr, 1, n, keybits, n_keybits, pairs_a, pairs_b, perm, hist,
               digit_total, ctl, s, host_D, tag, host_crowd, wide);
    return hipGetLastError();
}

hipError_t gsr_depth_sort_compacted(const uint32_t *keys, int64_t n, uint32_t *block_kept,
                                    uint32_t *keys_c, uint32_t *ids_c, uint2 *pairs_a,
                                    uint2 *pairs_b, uint32_t *perm, uint32_t *hist,
                                    uint32_t *digit_total, uint32_t *ctl, int pass_begin,
                                    int pass_end, hipStream_t s, unsigned long long *host_D,
                                    uint32_t tag, uint32_t *ids_copy, hipEvent_t compacted,
                                    int msd, const uint2 *keybits, int64_t n_keybits) {
    if (n <= 0 || pass_begin >= pass_end) return hipSuccess;
    if (n > (int64_t)UINT32_MAX || pass_begin < 0 || pass_end > kDPasses)
        return hipErrorInvalidValue;
    if (pass_begin == 0) {
        const int64_t nb = (n + 255) / 256;
        hipLaunchKernelGGL(k_ds_compact_scan, dim3(1), dim3(1024), 0, s, block_kept, nb, ctl);
        hipLaunchKernelGGL(k_ds_compact, dim3((unsigned)nb), dim3(256), 0, s, keys, n, block_kept,
                           keys_c, ids_c, ids_copy);
        if (compacted) {
            const hipError_t e = hipEventRecord(compacted, s);
            if (e != hipSuccess) return e;
        }
    }
    // the passes read the compacted count from ctl[0] (grids sized for n)
    if (msd) {  // the MSD form, the whole sort at once (pass_begin 0 only)
        if (pass_begin != 0) return hipErrorInvalidValue;
        // (pairs_b holds keys_c / ids_c: only the slow local sort of a degenerate bucket uses it,
        // after the MSD pass has read them)
        msd_launch(keys_c, ids_c, ctl, 0, n, keybits, n_keybits, pairs_a, pairs_b, perm, hist,
                   digit_total, ctl, s, host_D, tag, nullptr, 0);
        return hipGetLastError();
    }
    return ds_passes(keys_c, ids_c, ctl, n, 0, pairs_a, pairs_b, perm, hist, digit_total, ctl,
                     pass_begin, pass_end, host_D, tag, s);
}
