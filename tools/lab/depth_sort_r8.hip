// depth_sort.hip -- the per-frame stable sort of the Gaussians by view depth, for gfx950.
//
// Replaces the depth half of upstream's cub::DeviceRadixSort::SortPairs over (tile << 32 |
// depth) keys (rasterizer_impl.cu; see DESIGN.md decision 1 for the depth-first binning) and
// the viewer's torch / cupy / numpy argsort (renderer_ogl.py:17, :34, :51; gsr_depth_argsort).
//
// An 8-bit-digit LSD radix sort (reduce-then-scan) that sorts only the key bits that vary:
//   * pass p sorts key bits [8p, 8p + 8), on tiles of kT keys (kW waves x kIt keys per lane):
//     small tiles so that every CU holds several blocks (the sort is latency-bound at ~1M keys),
//     8-bit digits so that a tile's run of one digit is kT / 256 keys long (contiguous stores);
//   * pass 0's upsweep also reduces the OR and the AND of the kept keys: only the low D =
//     bits(OR ^ AND) bits need sorting (C3: depths in [2, 6), D = 24, three passes; a capture
//     with depths over 8 exponents: D = 31, four).  Pass 0's scan stores D, tagged with the frame,
//     into pinned host memory; the forward waits for it while pass 0's downsweep runs and launches
//     only the needed passes.  Callers that do not wait launch all four and the unneeded ones exit
//     at once (the kernels read D from ctl).  The last needed pass writes the permutation (the
//     ids alone) straight to `perm`;
//   * compaction: pass 0 drops the sentinel keys (0xFFFFFFFF: Gaussians without pairs in the
//     strip) and its scan stores the kept count on the device; later passes read it.
// Each pass is three kernels: upsweep (per-tile 256-bin histogram), scan (per digit across
// tiles) and downsweep (radix_tile_scatter: wave-ballot ranking in LDS, then each digit's run
// to digit start + earlier tiles' count).  Between passes keys and ids travel as two arrays.
// Every step keeps the tile order and the order within a tile, so each pass and the sort are
// stable: equal depths keep the Gaussian index order, as upstream's stable SortPairs does.
#include "radix_tile.h"

using namespace gsr;

namespace {

constexpr int kW = 4;                 // waves per block
constexpr int kThreads = kW * 64;     // 256
constexpr int kIt = GSR_DS8_IT;       // keys per lane
constexpr int kT = kThreads * kIt;    // keys per tile
constexpr int kPasses = 4;            // 8-bit digits over 32 key bits

// ctl: [0] kept count, [1] D (key bits to sort), [2..3] unused, then per tile uint4 {OR, AND,
// kept, 0} of pass 0.
constexpr int kCtlHead = 4;

// Elements of a pass: pass 0 n (the compacted count d_n when set), later ones the kept count.
__device__ __forceinline__ int64_t pass_n(bool first, int64_t n_host, const uint32_t *d_n,
                                          const uint32_t *ctl) {
    return first ? (d_n ? (int64_t)*d_n : n_host) : (int64_t)ctl[0];
}

// hist[d * nb + tile] = count of digit d in the tile (the layout k_rs_scan scans).
template <bool kFirst>
__global__ __launch_bounds__(kThreads) void k_ds8_upsweep(const uint32_t *__restrict__ keys,
                                                          int64_t n_host, int drop,
                                                          uint32_t *__restrict__ ctl, int shift,
                                                          uint32_t *__restrict__ hist, int64_t nb,
                                                          const uint32_t *__restrict__ d_n) {
    __shared__ uint32_t s_h[kW][kRadixBins];
    __shared__ uint32_t s_red[3][kW];
    if (!kFirst && ctl[1] <= (uint32_t)shift) return;  // constant digit: pass skipped
    const int64_t n = pass_n(kFirst, n_host, d_n, ctl);
    const int64_t base = (int64_t)blockIdx.x * kT;
    if (base >= n) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int i = tid; i < kW * kRadixBins; i += kThreads) (&s_h[0][0])[i] = 0u;
    __syncthreads();
    uint32_t vor = 0u, vand = 0xFFFFFFFFu, cnt = 0u;
    auto add = [&](uint32_t k) {
        if (kFirst && drop && k == kDropKey) return;
        atomicAdd(&s_h[w][(k >> shift) & 0xFFu], 1u);
        if (kFirst) {
            vor |= k;
            vand &= k;
            ++cnt;
        }
    };
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
    {
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < kW; ++i) c += s_h[i][tid];
        hist[(int64_t)tid * nb + blockIdx.x] = c;
    }
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
            for (int i = 0; i < kW; ++i) {
                o |= s_red[0][i];
                a &= s_red[1][i];
                c += s_red[2][i];
            }
            reinterpret_cast<uint4 *>(ctl + kCtlHead)[blockIdx.x] = make_uint4(o, a, c, 0u);
        }
    }
}

// Block d < 256: exclusive scan of digit d's counts over the live tiles (in place), total ->
// digit_total[d].  Pass 0: block 256 reduces the tiles' {OR, AND, kept} into ctl[0] (kept) and
// ctl[1] (D) and publishes D for the host.  The digit blocks of pass 0 see the live tile count
// from n (every tile of n, dropped keys included, wrote its row).
template <bool kFirst>
__global__ __launch_bounds__(256) void k_ds8_scan(uint32_t *__restrict__ hist, int64_t nb,
                                                  int64_t n_host, uint32_t *__restrict__ ctl,
                                                  int shift, uint32_t *__restrict__ digit_total,
                                                  const uint32_t *__restrict__ d_n,
                                                  unsigned long long *host_D, uint32_t tag) {
    __shared__ uint32_t s_tmp[4];
    __shared__ uint32_t s_red[3][4];
    if (!kFirst && ctl[1] <= (uint32_t)shift) return;
    const int64_t n = pass_n(kFirst, n_host, d_n, ctl);
    const int64_t nt = (n + kT - 1) / kT;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (blockIdx.x < kRadixBins) {
        uint32_t *h = hist + (int64_t)blockIdx.x * nb;
        uint32_t carry = 0;
        for (int64_t start = 0; start < nt; start += 256 * 4) {
            uint32_t v[4], sum = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t e = start + tid * 4 + i;
                v[i] = e < nt ? h[e] : 0u;
                sum += v[i];
            }
            uint32_t total;
            uint32_t pre = block256_exclusive_scan(sum, s_tmp, total) + carry;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int64_t e = start + tid * 4 + i;
                if (e < nt) h[e] = pre;
                pre += v[i];
            }
            carry += total;
        }
        if (tid == 0) digit_total[blockIdx.x] = carry;
        return;
    }
    if (!kFirst) return;
    const uint4 *st = reinterpret_cast<const uint4 *>(ctl + kCtlHead);
    uint32_t o = 0u, a = 0xFFFFFFFFu, c = 0u;
    for (int64_t t = tid; t < nt; t += 256) {
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
        // D for the host, tagged with the frame (pinned memory, system scope): it launches only
        // the passes D needs, while this pass's downsweep runs
        if (host_D)
            __hip_atomic_store(host_D, ((unsigned long long)tag << 32) | D, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// kFirst: keys_in are the n keys and the values the element indices (or ids_in[e]); kDrop
// (pass 0 only): sentinel keys are dropped.  The last needed pass (decided from D) writes only
// the ids, to perm.
template <bool kFirst, bool kDrop>
__global__ __launch_bounds__(kThreads) void k_ds8_downsweep(
    const uint32_t *__restrict__ keys_in, const uint32_t *__restrict__ vals_in,
    uint32_t *__restrict__ keys_out, uint32_t *__restrict__ vals_out, uint32_t *__restrict__ perm,
    int64_t n_host, const uint32_t *__restrict__ ctl, int shift, const uint32_t *__restrict__ hist,
    int64_t nb, const uint32_t *__restrict__ digit_total, const uint32_t *__restrict__ d_n) {
    __shared__ uint32_t s_keys[kT], s_vals[kT];
    __shared__ RadixTileSmem<kW, kIt> sm;
    const uint32_t D = ctl[1];
    if (!kFirst && D <= (uint32_t)shift) return;
    const int64_t n = pass_n(kFirst, n_host, d_n, ctl);
    const int64_t base = (int64_t)blockIdx.x * kT;
    if (base >= n) return;
    const bool last = (uint32_t)(shift + 8) >= D;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t k[kIt], v[kIt];
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
        const int64_t e = base + w * (kT / kW) + j * 64 + lane;
        const bool valid = e < n;
        k[j] = valid ? keys_in[e] : kDropKey;  // the tail: dropped (pass 0) / the last digit
        v[j] = valid ? (kFirst && !vals_in ? (uint32_t)e : vals_in[e]) : 0u;
    }
    const int64_t rem = n - base;
    radix_tile_scatter<kW, kIt, kDrop>(k, v, rem < kT ? (int)rem : kT, shift, 8, hist, nb,
                                        blockIdx.x, digit_total, last ? nullptr : keys_out,
                                        last ? perm : vals_out, sm, s_keys, s_vals);
}

// Compacting front end: exclusive scan of the per-256-block kept counts in place (one block),
// total -> ctl[0].  Rounds of 16k counts: each thread owns 16 consecutive counts (four 16-B
// loads issued together, a wave covers 4 KB contiguous), one block scan per round.
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

}  // namespace

int64_t gsr_depth_sort_hist_words(int64_t n) {
    const int64_t nt = (n + kT - 1) / kT;
    return (nt < 1 ? 1 : nt) * kRadixBins;
}

int64_t gsr_depth_sort_ctl_words(int64_t n) { return kCtlHead + 4 * ((n + kT - 1) / kT + 1); }

int gsr_depth_sort_digit_words() { return kRadixBins; }

int gsr_depth_sort_passes(uint32_t key_bits) {
    const int p = (int)((key_bits + 7) / 8);
    return p < 1 ? 1 : p > kPasses ? kPasses : p;
}

// Passes [pass_begin, pass_end).  Keys and ids live in two arrays between passes: pass p
// reads from a = pairs_a's halves (p odd) or b (p even, p > 0) and writes the other.
static hipError_t ds_passes(const uint32_t *keys, const uint32_t *ids_in, const uint32_t *d_n,
                            int64_t n, int drop, uint2 *pairs_a, uint2 *pairs_b, uint32_t *perm,
                            uint32_t *hist, uint32_t *digit_total, uint32_t *ctl, int pass_begin,
                            int pass_end, unsigned long long *host_D, uint32_t tag, hipStream_t s) {
    const int64_t nt = (n + kT - 1) / kT;
    uint32_t *ka = reinterpret_cast<uint32_t *>(pairs_a), *va = ka + n;
    uint32_t *kb = reinterpret_cast<uint32_t *>(pairs_b), *vb = kb + n;
    for (int p = pass_begin; p < pass_end; ++p) {
        const int shift = 8 * p;
        uint32_t *ko = (p & 1) ? kb : ka, *vo = (p & 1) ? vb : va;
        const uint32_t *ki = (p & 1) ? ka : kb, *vi = (p & 1) ? va : vb;
        if (p == 0) {
            hipLaunchKernelGGL(k_ds8_upsweep<true>, dim3((unsigned)nt), dim3(kThreads), 0, s, keys,
                               n, drop, ctl, shift, hist, nt, d_n);
            hipLaunchKernelGGL(k_ds8_scan<true>, dim3(kRadixBins + 1), dim3(256), 0, s, hist, nt,
                               n, ctl, shift, digit_total, d_n, host_D, tag);
            if (drop)
                hipLaunchKernelGGL((k_ds8_downsweep<true, true>), dim3((unsigned)nt), dim3(kThreads),
                                   0, s, keys, ids_in, ko, vo, perm, n, ctl, shift, hist, nt,
                                   digit_total, d_n);
            else
                hipLaunchKernelGGL((k_ds8_downsweep<true, false>), dim3((unsigned)nt),
                                   dim3(kThreads), 0, s, keys, ids_in, ko, vo, perm, n, ctl, shift,
                                   hist, nt, digit_total, d_n);
        } else {
            hipLaunchKernelGGL(k_ds8_upsweep<false>, dim3((unsigned)nt), dim3(kThreads), 0, s, ki,
                               n, 0, ctl, shift, hist, nt, nullptr);
            hipLaunchKernelGGL(k_ds8_scan<false>, dim3(kRadixBins), dim3(256), 0, s, hist, nt, n,
                               ctl, shift, digit_total, nullptr, nullptr, 0u);
            hipLaunchKernelGGL((k_ds8_downsweep<false, false>), dim3((unsigned)nt), dim3(kThreads), 0,
                               s, ki, vi, ko, vo, perm, n, ctl, shift, hist, nt, digit_total,
                               nullptr);
        }
    }
    return hipGetLastError();
}

hipError_t gsr_depth_sort(const uint32_t *keys, int64_t n, int drop, uint2 *pairs_a,
                          uint2 *pairs_b, uint32_t *perm, uint32_t *hist, uint32_t *digit_total,
                          uint32_t *ctl, int pass_begin, int pass_end, hipStream_t s,
                          unsigned long long *host_D, uint32_t tag) {
    if (n <= 0 || pass_begin >= pass_end) return hipSuccess;
    if (n > (int64_t)UINT32_MAX || pass_begin < 0 || pass_end > kPasses)
        return hipErrorInvalidValue;
    return ds_passes(keys, nullptr, nullptr, n, drop, pairs_a, pairs_b, perm, hist, digit_total,
                     ctl, pass_begin, pass_end, host_D, tag, s);
}

hipError_t gsr_depth_sort_compacted(const uint32_t *keys, int64_t n, uint32_t *block_kept,
                                    uint32_t *keys_c, uint32_t *ids_c, uint2 *pairs_a,
                                    uint2 *pairs_b, uint32_t *perm, uint32_t *hist,
                                    uint32_t *digit_total, uint32_t *ctl, int pass_begin,
                                    int pass_end, hipStream_t s, unsigned long long *host_D,
                                    uint32_t tag, uint32_t *ids_copy, hipEvent_t compacted) {
    if (n <= 0 || pass_begin >= pass_end) return hipSuccess;
    if (n > (int64_t)UINT32_MAX || pass_begin < 0 || pass_end > kPasses)
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
    return ds_passes(keys_c, ids_c, ctl, n, 0, pairs_a, pairs_b, perm, hist, digit_total, ctl,
                     pass_begin, pass_end, host_D, tag, s);
}
