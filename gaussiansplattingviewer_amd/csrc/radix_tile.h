// radix_tile.h -- the downsweep step of the reduce-then-scan radix sort, as a device function:
// rank one tile of (key, value) pairs stably by one digit and scatter it to its global
// positions.  Shared by the radix sort (radix_sort.hip k_rs_downsweep) and by the fused
// duplicate + first tile-sort pass (binning.hip k_dup_scatter), which generates its tile in
// registers instead of loading it.
#pragma once

#include "gsr_internal.h"

namespace gsr {

constexpr int kRadixBins = 256;

// Exclusive scan over a block of kW waves (all threads call it; returns the prefix of v).
template <int kW>
__device__ __forceinline__ uint32_t blockw_exclusive_scan(uint32_t v, uint32_t *s_tmp,
                                                          uint32_t &total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t inc = wave_inclusive_scan(v);
    if (lane == 63) s_tmp[w] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kW; ++i) {
        const uint32_t t = s_tmp[i];
        pre += (i < w) ? t : 0u;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return pre + inc - v;
}

template <int kW, int kIt>
struct RadixTileSmem {
    static constexpr int kT = kW * 64 * kIt;
    uint32_t wcnt[kW][kRadixBins];
    uint32_t delta[kRadixBins];
    uint32_t count[kRadixBins];  // kToGlobal = false: digit counts of the tile
    uint32_t tmp[2 * kW + 1];
};

// Tile layout: wave w holds elements [w*kT/kW, (w+1)*kT/kW) of the tile, item j of lane l is
// element w*kT/kW + j*64 + l.  Elements >= `valid` must carry key 0xFFFFFFFF (largest digit)
// and are not written.  hist[d * nb + tile] = this tile's exclusive digit offset as scanned by
// k_rs_scan (nb: the column stride); digit_total = per-digit totals.
// kDrop: every element whose key is kDropKey (0xFFFFFFFF) is dropped -- not ranked, counted or
// written -- so the output is the stable, compacted sequence of the other elements (the
// upsweep must not count them either).
// s_keys / s_vals: kT words each (may alias storage the caller no longer needs: the first
// write to them follows two block barriers).
// keys_out == nullptr: only the values are written (the packed pair list, binning.hip);
// vals_out == nullptr: keys only (v is ignored).
constexpr uint32_t kDropKey = 0xFFFFFFFFu;

// kToGlobal = false (in-LDS ranking, binning.hip k_col_scatter): stop once the tile sits in
// s_keys / s_vals in digit order; hist, digit_total, keys_out and vals_out are not used,
// sm.delta[d] is then the tile-local start of digit d and sm.count[d] its count.
template <int kW, int kIt, bool kDrop = false, bool kToGlobal = true>
__device__ __forceinline__ void radix_tile_scatter(
    const uint32_t (&k)[kIt], const uint32_t (&v)[kIt], int valid, int shift, int nbits,
    const uint32_t *__restrict__ hist, int64_t nb, uint32_t tile,
    const uint32_t *__restrict__ digit_total, uint32_t *__restrict__ keys_out,
    uint32_t *__restrict__ vals_out, RadixTileSmem<kW, kIt> &sm, uint32_t *s_keys,
    uint32_t *s_vals) {
    constexpr int kThreads = kW * 64;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t mask = (1u << nbits) - 1u;
    for (int i = tid; i < kW * kRadixBins; i += kThreads) (&sm.wcnt[0][0])[i] = 0;
    __syncthreads();

    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t rank[kIt];
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
        const uint32_t d = (k[j] >> shift) & mask;
        const bool keep = !kDrop || k[j] != kDropKey;
        // lanes holding this lane's digit: one ballot per bit, m &= ~(ballot ^ own bit
        // sign-extended) -- one v_bitop3 per 32-bit half; dropped lanes neither count nor rank
        const uint64_t m0 = kDrop ? __ballot(keep) : ~0ull;
        uint32_t mlo = (uint32_t)m0, mhi = (uint32_t)(m0 >> 32);
        for (int b = 0; b < nbits; ++b) {
            const uint32_t f = (uint32_t)(((int32_t)(d << (31 - b))) >> 31);
            const uint64_t bal = __ballot(f != 0u);
            mlo &= ~((uint32_t)bal ^ f);
            mhi &= ~((uint32_t)(bal >> 32) ^ f);
        }
        const uint64_t m = ((uint64_t)mhi << 32) | mlo;
        const uint32_t prior = sm.wcnt[w][d];
        rank[j] = prior + (uint32_t)__popcll(m & lt_mask);
        if (keep) sm.wcnt[w][d] = prior + (uint32_t)__popcll(m);  // same value from every match
    }
    __syncthreads();

    // Per digit (thread = digit): wave offsets, tile-local start, global destination.
    {
        const int d = tid;
        uint32_t c[kW], sum = 0;
        if (d < kRadixBins) {
#pragma unroll
            for (int i = 0; i < kW; ++i) {
                c[i] = sm.wcnt[i][d];
                sum += c[i];
            }
        }
        uint32_t tile_total, all_total;
        const uint32_t local_start =
            blockw_exclusive_scan<kW>(d < kRadixBins ? sum : 0u, sm.tmp, tile_total);
        if (kDrop && tid == 0) sm.tmp[2 * kW] = tile_total;
        uint32_t digit_start = 0;
        if (kToGlobal)
            digit_start = blockw_exclusive_scan<kW>(d < kRadixBins ? digit_total[d] : 0u,
                                                    sm.tmp + kW, all_total);
        if (d < kRadixBins) {
            if (kToGlobal) {
                sm.delta[d] = digit_start + hist[(int64_t)d * nb + tile] - local_start;
            } else {
                sm.delta[d] = local_start;
                sm.count[d] = sum;
            }
            uint32_t run = local_start;
#pragma unroll
            for (int i = 0; i < kW; ++i) {
                sm.wcnt[i][d] = run;
                run += c[i];
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kIt; ++j) {
        if (kDrop && k[j] == kDropKey) continue;
        const uint32_t d = (k[j] >> shift) & mask;
        const uint32_t pos = sm.wcnt[w][d] + rank[j];
        s_keys[pos] = k[j];
        if (vals_out || !kToGlobal) s_vals[pos] = v[j];
    }
    __syncthreads();
    if (!kToGlobal) return;
    const int n_out = kDrop ? (int)sm.tmp[2 * kW] : valid;  // kept elements of the tile
    for (int i = tid; i < n_out; i += kThreads) {
        const uint32_t kk = s_keys[i];
        const uint32_t g = sm.delta[(kk >> shift) & mask] + (uint32_t)i;
        if (keys_out) keys_out[g] = kk;
        if (vals_out) vals_out[g] = s_vals[i];
    }
}

}  // namespace gsr
