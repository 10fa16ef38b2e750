// Tile binning launch interface shared by binning.hip and frame.hip.
#pragma once

#include "common.h"

namespace gsvc {

// Given per-tile entry counts (counts[tbx*tby], already accumulated on the
// stream), launches scan -> fill -> per-tile segment sort: tile_bins,
// ids_sorted in (tile, splat id) order, meta = {M, M > capacity}.  With
// zero_counts the scan clears counts for the next call.  counts NULL skips the
// scan (the producer ran scan_tile_counts itself); ids_sorted NULL skips the
// segment sort (ids_scratch then holds each tile's ids in fill order).
// tile_cap > 0 (with ids_sorted): each tile keeps at most tile_cap entries --
// the first tile_cap by splat id; a tile with more has its list rebuilt from
// the splats' bboxes in id order (tile_ids.h wave_brute_ids); capacity need
// only cover sum(min(count, tile_cap)).
int tile_bins_from_counts(int num_points, const float2 *xys, const int *radii, int tbx, int tby,
                          long long capacity, unsigned *counts, unsigned *cursor, int *ids_scratch,
                          int *ids_sorted, int2 *bins, int *meta, bool zero_counts,
                          hipStream_t s, unsigned tile_cap = 0u);

// Stable LSD radix sort of n (key, value) pairs on key bits [0, bits); result
// in (kout, vout); kbuf / vbuf scratch of n; counts / offsets each of
// sort_u32_counts_bytes(n) bytes.
size_t sort_u32_counts_bytes(int n);
int sort_u32_pairs(int n, const unsigned *kin, const int *vin, unsigned *kout, int *vout,
                   unsigned *kbuf, int *vbuf, int bits, unsigned *counts, unsigned *offsets,
                   hipStream_t s);

// Exclusive scan of the per-tile counts by one workgroup of kThreads threads:
// tiles in chunks of kR * kThreads, every thread issuing its kR loads (one per
// round, coalesced) up front -- one memory round trip per chunk -- wave scans by shuffles, one LDS exchange of the
// wave totals per chunk.  Writes tile_bins ((0,0) when empty), the fill
// cursors and meta = {M, M > capacity}; with zero_counts the reading thread
// clears each counter for the next call.  tile_cap > 0: each tile's segment
// holds at most tile_cap entries (the consumers read only the first 256 of a
// tile); M stays the uncapped total.
template <int kThreads, int kR = 8>
__device__ __forceinline__ void scan_tile_counts(int ntiles, unsigned *__restrict__ counts,
                                                 int2 *__restrict__ bins,
                                                 unsigned *__restrict__ cursor,
                                                 int *__restrict__ meta, long long capacity,
                                                 bool zero_counts, unsigned tile_cap = 0u) {
    constexpr int kW = kThreads / 64;
    __shared__ unsigned s_tot[kR][kW];
    __shared__ unsigned s_all[kW];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    unsigned carry = 0u, all = 0u;
    for (int c0 = 0; c0 < ntiles; c0 += kThreads * kR) {
        unsigned v[kR], incl[kR];
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            const int i = c0 + r * kThreads + tid;
            v[r] = i < ntiles ? counts[i] : 0u;
            all += v[r];
            if (tile_cap) v[r] = min(v[r], tile_cap);
        }
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            unsigned x = v[r];
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const unsigned u = __shfl_up(x, off, 64);
                if (lane >= off) x += u;
            }
            incl[r] = x;
            if (lane == 63) s_tot[r][w] = x;
        }
        __syncthreads();
        unsigned base = carry;
#pragma unroll
        for (int r = 0; r < kR; ++r) {
            unsigned wo = 0u, rt = 0u;
#pragma unroll
            for (int k = 0; k < kW; ++k) {
                const unsigned t = s_tot[r][k];
                wo += (k < w) ? t : 0u;
                rt += t;
            }
            const int i = c0 + r * kThreads + tid;
            if (i < ntiles) {
                const unsigned start = base + wo + incl[r] - v[r];
                bins[i] = v[r] ? make_int2((int)start, (int)(start + v[r])) : make_int2(0, 0);
                cursor[i] = start;
                if (zero_counts) counts[i] = 0u;
            }
            base += rt;
        }
        carry = base;
        __syncthreads();
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) all += __shfl_xor(all, off, 64);
    if (lane == 0) s_all[w] = all;
    __syncthreads();
    if (tid == 0) {
        unsigned tot = 0u;
#pragma unroll
        for (int k = 0; k < kW; ++k) tot += s_all[k];
        meta[0] = (int)tot;
        meta[1] = (long long)carry > capacity ? 1 : 0;
    }
}

// Per-tile entry counting of one splat's bbox (tile_count_kernel's body).
__device__ __forceinline__ void count_splat_tiles(float cx, float cy, int r, int tbx, int tby,
                                                  unsigned *__restrict__ counts) {
    unsigned x0, y0, x1, y1;
    tile_bbox(cx, cy, (float)r, tbx, tby, x0, y0, x1, y1);
    for (unsigned y = y0; y < y1; ++y)
        for (unsigned x = x0; x < x1; ++x) atomicAdd(counts + y * (unsigned)tbx + x, 1u);
}

}  // namespace gsvc
