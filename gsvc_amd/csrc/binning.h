// Tile binning launch interface shared by binning.hip and frame.hip.
#pragma once

#include "common.h"

namespace gsvc {

// Given per-tile entry counts (counts[tbx*tby], already accumulated on the
// stream), launches scan -> fill -> per-tile segment sort: tile_bins,
// ids_sorted in (tile, splat id) order, meta = {M, M > capacity}.  With
// zero_counts the scan clears counts for the next call.
int tile_bins_from_counts(int num_points, const float2 *xys, const int *radii, int tbx, int tby,
                          long long capacity, unsigned *counts, unsigned *cursor, int *ids_scratch,
                          int *ids_sorted, int2 *bins, int *meta, bool zero_counts,
                          hipStream_t s);

// Per-tile entry counting of one splat's bbox (tile_count_kernel's body).
__device__ __forceinline__ void count_splat_tiles(float cx, float cy, int r, int tbx, int tby,
                                                  unsigned *__restrict__ counts) {
    unsigned x0, y0, x1, y1;
    tile_bbox(cx, cy, (float)r, tbx, tby, x0, y0, x1, y1);
    for (unsigned y = y0; y < y1; ++y)
        for (unsigned x = x0; x < x1; ++x) atomicAdd(counts + y * (unsigned)tbx + x, 1u);
}

}  // namespace gsvc
