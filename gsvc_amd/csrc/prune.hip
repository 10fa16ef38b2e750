// Device-side pruning of a frame model (gfx950): remove the k splats of
// smallest ||rgb_W|| and compact every parameter tensor, in three launches and
// without a host sync.
//
// Reference: GaussianSplats_Represent.py:101-125 (removal_control) and
// :149-166 (adaptive_control's pruning):
//     rgb_weight = torch.norm(rgb_W, dim=1); _, order = torch.sort(rgb_weight)
//     keep = ones(N, bool); keep[order[:k]] = False
//     p = nn.Parameter(p[keep])            for _xyz, _cholesky, _features_dc, rgb_W
// torch.sort on the GPU (1-D, N > 4096: a segmented radix sort) is stable, so
// the removed set is the first k of (norm, index) ascending -- equal norms
// (every densified splat starts at rgb_W = 0.01) leave in index order.
//
// Here: key(i) = bits of sqrt(w_i * w_i) (torch's NormTwo reduction of one
// element; non-negative floats order as their bits, NaN canonicalised to the
// largest key as torch.sort puts NaN last).
//   1. prune_select_pass_kernel x 4: 8-bit radix select of the k-th smallest
//      key T, and r = how many of the keys equal to T go (the first r by
//      index).  Per pass, wave-aggregated LDS histograms (ties are common)
//      summed by agent-scope atomics; the last workgroup to arrive picks the
//      digit (one workgroup alone was 110 us at 100k: one CU's issue rate).
//   2. prune_count_kernel: per 1024-splat chunk, the counts of key < T and
//      key == T.
//   3. prune_scatter_kernel: splat i is removed iff key < T, or key == T and
//      fewer than r equal keys precede it; a kept splat goes to row
//      i - (#key<T before i) - min(#key==T before i, r).  Chunk prefixes come
//      from step 2, in-chunk prefixes from ballots.  Rows of every tensor are
//      copied in order (the boolean-mask indexing of the reference).
// Bytes per splat: 16 (select, 4 passes) + 4 (count) + 4 + 36 read, 36
// written (scatter) -- HBM-bound and tiny (100k splats: ~8 MB).
#include "common.h"

namespace gsvc {

constexpr int kPruneChunk = 1024;  // splats per workgroup of the count / scatter kernels
constexpr int kPruneMaxTensors = 8;
constexpr int kPruneHeaderBytes = 4 * (8 + 4 * 256);  // (T, r), 4 tickets, 4 pass histograms

struct PruneArgs {
    int ntensors;
    int cols[kPruneMaxTensors];
    const float *src[kPruneMaxTensors];
    float *dst[kPruneMaxTensors];
};

__device__ __forceinline__ unsigned prune_key(const float *w, int i) {
    const float x = w[i];
    const float s = __fsqrt_rn(__fmul_rn(x, x));
    return s != s ? 0x7fc00000u : __float_as_uint(s);
}

// One radix-select pass over digit d (bits 8d..8d+7) of the keys that match
// the prefix chosen so far: workgroup histograms in LDS, added into the pass's
// global histogram with agent-scope atomics; the last workgroup to arrive
// picks the digit of the kk-th key and writes (prefix, kk) for the next pass.
// sel = {prefix, kk, -, -, tickets[4], hist[4][256]}, zeroed by the launcher.
__global__ __launch_bounds__(256) void prune_select_pass_kernel(int n, int k, int d,
                                                                const float *__restrict__ w,
                                                                unsigned *__restrict__ sel) {
    __shared__ unsigned h[256];
    __shared__ unsigned s_wsum[4];
    __shared__ unsigned s_last;
    const int tid = threadIdx.x, lane = tid & 63;
    unsigned *ticket = sel + 4 + d;
    unsigned *ghist = sel + 8 + 256 * d;
    const int sh = 8 * d;
    const unsigned mask = d == 3 ? 0u : (0xffffffffu << (sh + 8));
    const unsigned prefix = d == 3 ? 0u : sel[0];  // written by the previous pass's launch
    const unsigned kk = d == 3 ? (unsigned)k : sel[1];
    h[tid] = 0u;
    __syncthreads();
    for (int i = blockIdx.x * 256 + tid; i < n; i += gridDim.x * 256) {
        const unsigned key = prune_key(w, i);
        const bool m = (key & mask) == prefix;
        const unsigned bin = (key >> sh) & 255u;
        const unsigned long long bm = __ballot(m);
        if (bm == 0ull) continue;
        const int fl = __ffsll((long long)bm) - 1;
        const unsigned first = (unsigned)__builtin_amdgcn_readlane((int)bin, fl);
        if (__ballot(m && bin != first) == 0ull) {  // one bin for the wave (ties)
            if (lane == fl) atomicAdd(&h[first], (unsigned)__popcll(bm));
        } else if (m) {
            atomicAdd(&h[bin], 1u);
        }
    }
    __syncthreads();
    if (h[tid]) __hip_atomic_fetch_add(&ghist[tid], h[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 gridDim.x - 1;
        if (s_last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!s_last) return;
    // the bin holding the kk-th key: inclusive scan of the 256 counts
    const unsigned c = __hip_atomic_load(&ghist[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned incl = c;
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned v = __shfl_up(incl, off);
        if (lane >= off) incl += v;
    }
    if (lane == 63) s_wsum[tid >> 6] = incl;
    __syncthreads();
    for (int q = 0; q < (tid >> 6); ++q) incl += s_wsum[q];
    const unsigned excl = incl - c;
    if (excl < kk && kk <= incl) {  // exactly one bin (kk <= the matching keys)
        sel[0] = prefix | ((unsigned)tid << sh);
        sel[1] = kk - excl;  // after d = 0: r, the keys equal to T that are removed
    }
}

// Exclusive in-workgroup counts of two flags for 256 threads; totals out.
__device__ __forceinline__ void block_excl2(bool a, bool b, unsigned *s_w, unsigned &ea,
                                            unsigned &eb, unsigned &ta, unsigned &tb) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const unsigned long long ma = __ballot(a), mb = __ballot(b);
    if (lane == 0) {
        s_w[wv] = (unsigned)__popcll(ma);
        s_w[4 + wv] = (unsigned)__popcll(mb);
    }
    __syncthreads();
    unsigned pa = 0u, pb = 0u;
    for (int q = 0; q < wv; ++q) {
        pa += s_w[q];
        pb += s_w[4 + q];
    }
    ea = pa + (unsigned)__popcll(ma & lt);
    eb = pb + (unsigned)__popcll(mb & lt);
    ta = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    tb = s_w[4] + s_w[5] + s_w[6] + s_w[7];
    __syncthreads();
}

__global__ __launch_bounds__(256) void prune_count_kernel(int n, const float *__restrict__ w,
                                                          const unsigned *__restrict__ sel,
                                                          unsigned *__restrict__ counts) {
    __shared__ unsigned s_w[8];
    const unsigned T = sel[0];
    const int c0 = blockIdx.x * kPruneChunk;
    unsigned lows = 0u, ties = 0u;
    for (int j = 0; j < kPruneChunk; j += 256) {
        const int i = c0 + j + (int)threadIdx.x;
        bool lo = false, ti = false;
        if (i < n) {
            const unsigned key = prune_key(w, i);
            lo = key < T;
            ti = key == T;
        }
        unsigned ea, eb, ta, tb;
        block_excl2(lo, ti, s_w, ea, eb, ta, tb);
        lows += ta;
        ties += tb;
    }
    if (threadIdx.x == 0) {
        counts[2 * blockIdx.x] = lows;
        counts[2 * blockIdx.x + 1] = ties;
    }
}

__global__ __launch_bounds__(256) void prune_scatter_kernel(int n, const float *__restrict__ w,
                                                            const unsigned *__restrict__ sel,
                                                            const unsigned *__restrict__ counts,
                                                            PruneArgs A) {
    __shared__ unsigned s_w[8];
    __shared__ unsigned s_pre[2][4];
    const int tid = threadIdx.x;
    const unsigned T = sel[0], r = sel[1];
    // this chunk's prefix: the counts of every earlier chunk
    unsigned lb = 0u, tb = 0u;
    for (int b = tid; b < (int)blockIdx.x; b += 256) {
        lb += counts[2 * b];
        tb += counts[2 * b + 1];
    }
    for (int off = 32; off > 0; off >>= 1) {
        lb += __shfl_down(lb, off);
        tb += __shfl_down(tb, off);
    }
    if ((tid & 63) == 0) {
        s_pre[0][tid >> 6] = lb;
        s_pre[1][tid >> 6] = tb;
    }
    __syncthreads();
    unsigned low_before = s_pre[0][0] + s_pre[0][1] + s_pre[0][2] + s_pre[0][3];
    unsigned tie_before = s_pre[1][0] + s_pre[1][1] + s_pre[1][2] + s_pre[1][3];
    const int c0 = blockIdx.x * kPruneChunk;
    for (int j = 0; j < kPruneChunk; j += 256) {
        const int i = c0 + j + tid;
        bool lo = false, ti = false;
        if (i < n) {
            const unsigned key = prune_key(w, i);
            lo = key < T;
            ti = key == T;
        }
        unsigned ea, eb, ta, tbt;
        block_excl2(lo, ti, s_w, ea, eb, ta, tbt);
        if (i < n) {
            const unsigned ties_prior = tie_before + eb;
            const bool removed = lo || (ti && ties_prior < r);
            if (!removed) {
                const long long row =
                    (long long)i - (long long)(low_before + ea) - (long long)min(ties_prior, r);
                for (int t = 0; t < A.ntensors; ++t) {
                    const int c = A.cols[t];
                    const float *s = A.src[t] + (long long)i * c;
                    float *d = A.dst[t] + row * c;
                    for (int q = 0; q < c; ++q) d[q] = s[q];
                }
            }
        }
        low_before += ta;
        tie_before += tbt;
    }
}

}  // namespace gsvc

using namespace gsvc;

extern "C" size_t gsvc_prune_workspace_bytes(int num_points) {
    const int chunks = num_points > 0 ? ceil_div(num_points, kPruneChunk) : 0;
    return kPruneHeaderBytes + 8 * (size_t)chunks;
}

extern "C" int gsvc_prune_lowest(int num_points, int remove_count, const float *rgb_w,
                                 int ntensors, const int *cols, const float *const *src,
                                 float *const *dst, void *workspace, size_t workspace_bytes,
                                 void *stream) {
    if (num_points < 0 || remove_count < 0 || ntensors < 0 || ntensors > kPruneMaxTensors ||
        (ntensors > 0 && (!cols || !src || !dst)))
        return set_error(GSVC_ERR_ARG, "prune_lowest: bad arguments");
    if (num_points == 0 || remove_count >= num_points) return GSVC_OK;  // nothing is kept
    if (!rgb_w) return set_error(GSVC_ERR_ARG, "prune_lowest: rgb_w is null");
    if (!workspace || workspace_bytes < gsvc_prune_workspace_bytes(num_points))
        return set_error(GSVC_ERR_WORKSPACE, "prune_lowest: workspace of %zu bytes, need %zu",
                         workspace_bytes, gsvc_prune_workspace_bytes(num_points));
    PruneArgs A{};
    A.ntensors = ntensors;
    for (int t = 0; t < ntensors; ++t) {
        if (cols[t] <= 0 || !src[t] || !dst[t])
            return set_error(GSVC_ERR_ARG, "prune_lowest: tensor %d: bad columns or pointer", t);
        A.cols[t] = cols[t];
        A.src[t] = src[t];
        A.dst[t] = dst[t];
    }
    unsigned *sel = reinterpret_cast<unsigned *>(workspace);
    unsigned *counts = sel + kPruneHeaderBytes / 4;
    const int chunks = ceil_div(num_points, kPruneChunk);
    hipStream_t s = (hipStream_t)stream;
    // (T, r) = (0, 0) removes nothing; the passes' tickets and histograms start at 0
    if (dev_zero(workspace, kPruneHeaderBytes, s) != GSVC_OK)
        return set_error(GSVC_ERR_HIP, "prune_lowest: zero fill failed");
    if (remove_count > 0) {
        const int grid = std::min(ceil_div(num_points, 1024), 256);
        for (int d = 3; d >= 0; --d)
            hipLaunchKernelGGL(prune_select_pass_kernel, dim3(grid), dim3(256), 0, s, num_points,
                               remove_count, d, rgb_w, sel);
    }
    hipLaunchKernelGGL(prune_count_kernel, dim3(chunks), dim3(256), 0, s, num_points, rgb_w, sel,
                       counts);
    hipLaunchKernelGGL(prune_scatter_kernel, dim3(chunks), dim3(256), 0, s, num_points, rgb_w, sel,
                       counts, A);
    return check_launch("prune_lowest");
}
