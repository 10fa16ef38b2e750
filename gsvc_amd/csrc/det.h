// Deterministic gradient sums (GSVC_TRAIN_DETERMINISTIC, and the op path's
// backward under torch.use_deterministic_algorithms): every (splat, tile) pair
// owns one slot of a partial-sum buffer, at
//     det_off[splat] + (row-major index of the tile in the splat's tile bbox),
// which the tile kernels store instead of adding with float atomics
// (backward.cu:843-859 adds with atomics, so its sums depend on timing); the
// splat's gradient is then its slots added in that fixed order.  Shared by
// train.hip and raster_sum.hip.
#pragma once

#include "common.h"

namespace gsvc {
namespace {

// off[i] = sum over splats j < i of their tile-bbox
// areas (the projection's insertions, frame.hip), off[n] = M.  One workgroup;
// thread t scans the contiguous splats [t * per, (t + 1) * per).
constexpr int kDetScanThreads = 1024;
__device__ __forceinline__ int det_area(const float2 *xys, const int *radii, int i, int tbx, int tby) {
    const int r = radii[i];
    if (r <= 0) return 0;
    unsigned x0, y0, x1, y1;
    tile_bbox(xys[i].x, xys[i].y, (float)r, tbx, tby, x0, y0, x1, y1);
    return (x1 > x0 && y1 > y0) ? (int)((x1 - x0) * (y1 - y0)) : 0;
}

__global__ __launch_bounds__(kDetScanThreads) void det_offsets_kernel(int n, const float2 *__restrict__ xys,
                                                                      const int *__restrict__ radii,
                                                                      int tbx, int tby,
                                                                      int *__restrict__ off) {
    __shared__ int s_w[kDetScanThreads / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int per = (n + kDetScanThreads - 1) / kDetScanThreads;
    const int b = min(tid * per, n), e = min(b + per, n);
    int sum = 0;
    for (int i = b; i < e; ++i) sum += det_area(xys, radii, i, tbx, tby);
    int incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d, 64);
        if (lane >= d) incl += t;
    }
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    int base = 0;
    for (int k = 0; k < w; ++k) base += s_w[k];
    int run = base + incl - sum;
    for (int i = b; i < e; ++i) {
        off[i] = run;
        run += det_area(xys, radii, i, tbx, tby);
    }
    if (tid == kDetScanThreads - 1) off[n] = base + incl;
}

// The slot of (splat g, tile (tx, ty)) -- the tile must lie in g's bbox.
__device__ __forceinline__ long long det_slot(const int *off, const float2 *xys, const int *radii,
                                              int g, int tx, int ty, int tbx, int tby) {
    unsigned x0, y0, x1, y1;
    tile_bbox(xys[g].x, xys[g].y, (float)radii[g], tbx, tby, x0, y0, x1, y1);
    return (long long)off[g] + (long long)((unsigned)ty - y0) * (long long)(x1 - x0) +
           (long long)((unsigned)tx - x0);
}

}  // namespace
}  // namespace gsvc
