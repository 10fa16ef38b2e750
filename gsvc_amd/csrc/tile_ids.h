// Per-tile id ordering shared by the one-wave tile kernels (raster_sum.hip,
// train.hip): the sum rasterizer blends a tile's first <= 256 entries in
// (tile, splat id) order (forward.cu:569-571,613; the reference's stable
// sort of (tile << 32 | depth 0) keys, utils.py:164), so a kernel that
// receives a tile's splats in fill order ranks them by id itself.
#pragma once

#include "frame.h"

namespace gsvc {

__device__ __forceinline__ void wave_lds_sync() {
    // a wave owns its LDS slice and LDS ops of a wave complete in order: a
    // drain of lgkmcnt is the only fence needed (no s_barrier)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// The tile's splat ids in ascending order -- the first min(n_all, 256) of
// them -- into s_ids (LDS): the segment sort of binning.hip done by the wave
// that blends the tile, when the ids arrive in fill order (frame path).  At
// most 64 entries: ranks by broadcast compares; more: an LDS bitmap over the
// id range in windows of 16384 ids, emitted in order until 256 are found.
// ``bm`` is 512 words of this wave's LDS (free until blending starts).  Ids
// are unique within a tile, so this is the stable sort's order.
constexpr int kSortWords = 512;

// Id of slot j of a tile's segment: a plain int array, or the id lane of a
// slab record (stride 12 floats).
struct SegIds {
    const int *ids;
    const float4 *recs;  // slab body (slots >= kHeadSlots at their index) ...
    const float4 *head;  // ... and the tile's head slots
    const int *ovf = nullptr;  // record slabs: slots [256, kCarryCap) as ids
    int cap_ids = kTilePix;    // id segments: slots per tile (wide id slabs: kCarryCap)
    __device__ __forceinline__ int operator[](int j) const {
        if (!recs) return ids[j];
        if (j >= kTilePix) return ovf[j - kTilePix];
        return __float_as_int(j < kHeadSlots ? head[3 * j + 2].y : recs[3 * j + 2].y);
    }
    // slots the segment holds (a longer tile takes the bbox rebuild)
    __device__ __forceinline__ int cap() const { return recs ? (ovf ? kCarryCap : kTilePix) : cap_ids; }
};

__device__ __forceinline__ int rank_below(int v, int n) {
    // number of lanes k < n whose value is below v (ties impossible: ids unique)
    int rank = 0;
    for (int k = 0; k < n; ++k) rank += (__builtin_amdgcn_readlane(v, k) < v) ? 1 : 0;
    return rank;
}

// The id-window bitmap of the sorts below: 32 * kSortWords ids from ``base``.
__device__ __forceinline__ void bitmap_clear(unsigned *bm) {
    for (int w = threadIdx.x & 63; w < kSortWords; w += 64) bm[w] = 0u;
    wave_lds_sync();
}
__device__ __forceinline__ void bitmap_set(unsigned *bm, long long d) {
    if (d >= 0 && d < 32 * kSortWords) atomicOr(bm + (d >> 5), 1u << (d & 31));
}
// The window's ids in ascending order into s_ids[written, 256); returns the
// new count (possibly past 256: only the first 256 are stored).
__device__ __forceinline__ int bitmap_emit(const unsigned *bm, long long base, int written,
                                           int *s_ids) {
    const int lane = threadIdx.x & 63;
    constexpr int kPer = kSortWords / 64;  // words per lane, in order
    unsigned wv[kPer];
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        wv[q] = bm[kPer * lane + q];
        cnt += __popc(wv[q]);
    }
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(incl, off, 64);
        if (lane >= off) incl += u;
    }
    int pos = written + incl - cnt;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        unsigned bits = wv[q];
        while (bits && pos < kTilePix) {
            s_ids[pos++] = (int)(base + 32 * (kPer * lane + q) + (__ffs(bits) - 1));
            bits &= bits - 1u;
        }
    }
    written += __shfl(incl, 63, 64);
    wave_lds_sync();
    return written;
}

__device__ inline int wave_sorted_tile_ids(SegIds ids, int n_all, int *s_ids, unsigned *bm) {
    const int lane = threadIdx.x & 63;
    if (n_all <= 0) return 0;
    // a segment holds at most seg.cap() slots (a longer tile takes the bbox
    // rebuild): never read past them, whatever the count says
    n_all = min(n_all, ids.cap());
    if (n_all <= 64) {
        const int v = lane < n_all ? ids[lane] : 0x7fffffff;
        const int rank = rank_below(v, n_all);
        if (lane < n_all) s_ids[rank] = v;
        wave_lds_sync();
        return n_all;
    }
    int lo = 0x7fffffff, hi = -1;
    for (int j = lane; j < n_all; j += 64) {
        const int v = ids[j];
        lo = min(lo, v);
        hi = max(hi, v);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, __shfl_xor(lo, off, 64));
        hi = max(hi, __shfl_xor(hi, off, 64));
    }
    int written = 0;
    for (long long base = lo; base <= hi && written < kTilePix; base += 32 * kSortWords) {
        bitmap_clear(bm);
        for (int j = lane; j < n_all; j += 64) bitmap_set(bm, (long long)ids[j] - base);
        wave_lds_sync();
        written = bitmap_emit(bm, base, written, s_ids);
    }
    return min(written, kTilePix);
}

// A tile with more than 256 entries on the frame path (its slab kept an
// arbitrary 256): its first 256 ids are rebuilt by testing every splat's tile
// bbox (the binning's own tile_bbox of xys and radii) in id order, 64 at a
// time, compacting the hits by ballot -- sorted by construction.  The
// fallback of every tile kernel for a tile past its slab's capacity.
__device__ __forceinline__ int wave_brute_ids(const float2 *xys, const int *radii, int begin,
                                              int end, int tbx, int tby, int tile, int *s_ids) {
    const int lane = threadIdx.x & 63;
    const unsigned ty = (unsigned)(tile / tbx), tx = (unsigned)(tile - (int)ty * tbx);
    const unsigned long long lt = (1ull << lane) - 1ull;
    // kQ batches of 64 splats per round, every load issued before the first
    // test (one round trip per 64 kQ splats; a load per batch behind the
    // previous batch's ballot made it one per 64, ~0.6 ms at 50k splats)
    constexpr int kQ = 4;
    int written = 0;
    for (int base = begin; base < end && written < kTilePix; base += 64 * kQ) {
        int r[kQ];
        float2 c[kQ];
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            const int j = min(base + 64 * q + lane, end - 1);
            r[q] = radii[j];
            c[q] = xys[j];
        }
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            bool hit = false;
            if (base + 64 * q + lane < end && r[q] > 0) {
                unsigned x0, y0, x1, y1;
                tile_bbox(c[q].x, c[q].y, (float)r[q], tbx, tby, x0, y0, x1, y1);
                hit = tx >= x0 && tx < x1 && ty >= y0 && ty < y1;
            }
            const unsigned long long m = __ballot(hit);
            const int pos = written + __popcll(m & lt);
            if (hit && pos < kTilePix) s_ids[pos] = base + 64 * q + lane;
            written += __popcll(m);
        }
    }
    wave_lds_sync();
    return min(written, kTilePix);
}

}  // namespace gsvc
