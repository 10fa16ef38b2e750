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

// The same offsets from all CUs: per 1024-splat block a local exclusive scan
// (coalesced loads) and the block's total into bsum, one workgroup scanning
// the block totals (off[n] = M), and the block bases added -- integer sums,
// so exactly det_offsets_kernel's values.  (The single-workgroup kernel above
// took 176 us at 50k splats: each thread walks 49 splats of its own.)
constexpr int kDetBlock = 1024;
__global__ __launch_bounds__(kDetBlock) void det_block_scan_kernel(int n, const float2 *__restrict__ xys,
                                                                   const int *__restrict__ radii, int tbx,
                                                                   int tby, int *__restrict__ off,
                                                                   int *__restrict__ bsum) {
    __shared__ int s_w[kDetBlock / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int i = blockIdx.x * kDetBlock + tid;
    const int a = i < n ? det_area(xys, radii, i, tbx, tby) : 0;
    int incl = a;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d, 64);
        if (lane >= d) incl += t;
    }
    if (lane == 63) s_w[w] = incl;
    __syncthreads();
    int base = 0;
    for (int k = 0; k < w; ++k) base += s_w[k];
    if (i < n) off[i] = base + incl - a;
    if (tid == kDetBlock - 1) bsum[blockIdx.x] = base + incl;
}

__global__ __launch_bounds__(kDetBlock) void det_bsum_scan_kernel(int nb, int n, int *__restrict__ bsum,
                                                                  int *__restrict__ off) {
    __shared__ int s_w[kDetBlock / 64];
    __shared__ int s_carry;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) s_carry = 0;
    __syncthreads();
    for (int c = 0; c < nb; c += kDetBlock) {
        const int j = c + tid;
        const int v = j < nb ? bsum[j] : 0;
        int incl = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(incl, d, 64);
            if (lane >= d) incl += t;
        }
        if (lane == 63) s_w[w] = incl;
        __syncthreads();
        int base = s_carry;
        for (int k = 0; k < w; ++k) base += s_w[k];
        if (j < nb) bsum[j] = base + incl - v;
        __syncthreads();
        if (tid == kDetBlock - 1) s_carry = base + incl;
        __syncthreads();
    }
    if (tid == 0) off[n] = s_carry;
}

__global__ __launch_bounds__(256) void det_add_kernel(int n, int *__restrict__ off,
                                                      const int *__restrict__ bsum) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n && i >= kDetBlock) off[i] += bsum[i / kDetBlock];
}

// off = the offsets of n splats; ``scratch`` (device, scratch_ints ints, free
// until the caller's next use) holds the block totals -- without room for
// them, the single-workgroup kernel.
static inline void det_offsets_launch(int n, const float2 *xys, const int *radii, int tbx, int tby,
                                      int *off, int *scratch, size_t scratch_ints, hipStream_t s) {
    const int nb = (n + kDetBlock - 1) / kDetBlock;
    if (n <= 0 || !scratch || scratch_ints < (size_t)nb) {
        hipLaunchKernelGGL(det_offsets_kernel, dim3(1), dim3(kDetScanThreads), 0, s, n, xys, radii, tbx,
                           tby, off);
        return;
    }
    hipLaunchKernelGGL(det_block_scan_kernel, dim3(nb), dim3(kDetBlock), 0, s, n, xys, radii, tbx, tby,
                       off, scratch);
    hipLaunchKernelGGL(det_bsum_scan_kernel, dim3(1), dim3(kDetBlock), 0, s, nb, n, scratch, off);
    if (nb > 1)
        hipLaunchKernelGGL(det_add_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, off, scratch);
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
