// Tile binning: cumulative intersections, (tile, splat) emission, stable LSD
// radix sort and tile bin edges (gfx950).
//
// Reference: gsplat/gsplat/utils.py:99-167 (torch.cumsum + .item() +
// torch.sort + torch.gather glue), cuda/csrc/forward.cu:100-136
// (map_gaussian_to_intersects), forward.cu:141-163 (get_tile_bin_edges),
// bindings.cu:274-330.
//
// Design: the 2D projection writes depth 0 for every splat, so
// the reference's 64-bit key (tile << 32 | depth bits) orders exactly like the
// tile id, and ties keep splat order (torch.sort is stable on these inputs).
// The hot path therefore sorts 32-bit tile keys on ceil(log2(tiles)) bits only
// (13 bits = two 8-bit LSD passes at 1080p) instead of 64-bit keys.  Each pass
// is hist -> scan -> scatter; the scatter ranks equal digits inside a wave
// with 64-lane ballots (wave64 multisplit) and keeps a per-wave running
// counter in LDS, which makes the sort stable and deterministic (no atomics on
// the data path).  The general signed-int64 sort (used by the drop-in
// bin_and_sort_gaussians when depth bits differ) runs the same kernels on all
// 8 digits.
#include "binning.h"
#include "tile_ids.h"

namespace gsvc {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanBlock = kScanThreads * kScanItems;  // 2048 splats per block
constexpr int kSortThreads = 256;
constexpr int kSortRounds = 8;                           // rounds of 64 per wave
constexpr int kSortBlock = kSortThreads * kSortRounds;   // 2048 items per block
constexpr int kWaves = kSortThreads / 64;

static inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// ---------------------------------------------------------------------------
// Block-wide helpers (256 threads = 4 waves).
__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(v, off, 64);
        if (lane >= off) v += u;
    }
    return v;
}

// Exclusive scan of one int per thread over a 256-thread block; returns the
// block total in *total.  ``ws`` holds kWaves ints of LDS.
__device__ __forceinline__ int block_excl_scan(int v, int *ws, int *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int incl = wave_incl_scan(v);
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    int wave_off = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) {
        const int s = ws[k];
        if (k < w) wave_off += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return wave_off + incl - v;
}

// ---------------------------------------------------------------------------
// utils.py:116 torch.cumsum(num_tiles_hit, dtype=int32): reduce then scan.
__global__ __launch_bounds__(kScanThreads) void cum_reduce_kernel(
    int n, const int *__restrict__ nth, const float *__restrict__ depths,
    int *__restrict__ block_sum, unsigned *__restrict__ block_or, unsigned *__restrict__ block_and,
    int *__restrict__ block_cnt) {
    __shared__ int s_sum[kWaves];
    __shared__ unsigned s_or[kWaves], s_and[kWaves];
    __shared__ int s_cnt[kWaves];
    const int base = blockIdx.x * kScanBlock;
    int sum = 0, cnt = 0;
    unsigned bor = 0u, band = 0xffffffffu;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
        const int i = base + j * kScanThreads + threadIdx.x;
        if (i < n) {
            const int h = nth[i];
            sum += h;
            if (h > 0) {
                const unsigned bits = depths ? __float_as_uint(depths[i]) : 0u;
                bor |= bits;
                band &= bits;
                ++cnt;
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        sum += __shfl_xor(sum, off, 64);
        cnt += __shfl_xor(cnt, off, 64);
        bor |= __shfl_xor(bor, off, 64);
        band &= __shfl_xor(band, off, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_sum[w] = sum; s_or[w] = bor; s_and[w] = band; s_cnt[w] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        block_sum[blockIdx.x] = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
        block_or[blockIdx.x] = s_or[0] | s_or[1] | s_or[2] | s_or[3];
        block_and[blockIdx.x] = s_and[0] & s_and[1] & s_and[2] & s_and[3];
        block_cnt[blockIdx.x] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    }
}

__global__ __launch_bounds__(kScanThreads) void cum_scan_kernel(
    int n, int nblocks, const int *__restrict__ nth, const int *__restrict__ block_sum,
    const unsigned *__restrict__ block_or, const unsigned *__restrict__ block_and,
    const int *__restrict__ block_cnt, int *__restrict__ cum, int *__restrict__ meta) {
    __shared__ int ws[kWaves];
    // prefix of the preceding blocks
    int pre = 0;
    for (int j = threadIdx.x; j < (int)blockIdx.x; j += kScanThreads) pre += block_sum[j];
    int block_prefix;  // = sum of block_sum[0..b)
    (void)block_excl_scan(pre, ws, &block_prefix);
    // local scan: thread t owns kScanItems consecutive splats
    const int i0 = blockIdx.x * kScanBlock + threadIdx.x * kScanItems;
    int v[kScanItems];
    int run = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
        v[j] = (i0 + j < n) ? nth[i0 + j] : 0;
        run += v[j];
        v[j] = run;
    }
    int block_total;
    const int t_off = block_excl_scan(run, ws, &block_total) + block_prefix;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j)
        if (i0 + j < n) cum[i0 + j] = v[j] + t_off;
    if (blockIdx.x == nblocks - 1 && threadIdx.x == 0) {
        unsigned bor = 0u, band = 0xffffffffu;
        int cnt = 0;
        for (int j = 0; j < nblocks; ++j) {
            bor |= block_or[j];
            band &= block_and[j];
            cnt += block_cnt[j];
        }
        meta[0] = block_prefix + block_total;
        meta[1] = (int)(cnt > 0 ? bor : 0u);
        meta[2] = (int)(cnt > 0 ? band : 0u);
        meta[3] = cnt;
    }
}

// ---------------------------------------------------------------------------
// forward.cu:100-136: per splat, row-major over its tile bbox.
__global__ __launch_bounds__(256) void map_isect_kernel(
    int n, int m, const float2 *__restrict__ xys, const float *__restrict__ depths,
    const int *__restrict__ radii, const int *__restrict__ cum, int tbx, int tby,
    long long *__restrict__ isect_ids, int *__restrict__ gaussian_ids) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int r = radii[i];
    if (r <= 0) return;
    unsigned x0, y0, x1, y1;
    const float2 c = xys[i];
    tile_bbox(c.x, c.y, (float)r, tbx, tby, x0, y0, x1, y1);
    int cur = (i == 0) ? 0 : cum[i - 1];
    const long long depth_id = (long long)(int)__float_as_uint(depths[i]);
    for (int y = (int)y0; y < (int)y1; ++y)
        for (int x = (int)x0; x < (int)x1; ++x) {
            if (cur >= 0 && cur < m) {
                const long long tile = (long long)(y * tbx + x);
                isect_ids[cur] = (tile << 32) | depth_id;
                gaussian_ids[cur] = i;
            }
            ++cur;
        }
}

// Hot-path emission: 32-bit tile keys and splat ids, same order as above.
__global__ __launch_bounds__(256) void map_tiles_kernel(
    int n, int m, const float2 *__restrict__ xys, const int *__restrict__ radii,
    const int *__restrict__ cum, int tbx, int tby, unsigned *__restrict__ keys,
    int *__restrict__ vals) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int r = radii[i];
    if (r <= 0) return;
    unsigned x0, y0, x1, y1;
    const float2 c = xys[i];
    tile_bbox(c.x, c.y, (float)r, tbx, tby, x0, y0, x1, y1);
    int cur = (i == 0) ? 0 : cum[i - 1];
    for (unsigned y = y0; y < y1; ++y)
        for (unsigned x = x0; x < x1; ++x) {
            if (cur >= 0 && cur < m) {
                keys[cur] = y * (unsigned)tbx + x;
                vals[cur] = i;
            }
            ++cur;
        }
}

// ---------------------------------------------------------------------------
// Stable LSD radix sort, one 8-bit (or narrower) digit per pass.
template <typename K>
__device__ __forceinline__ unsigned key_digit(K k, int shift, unsigned mask, bool flip);

template <>
__device__ __forceinline__ unsigned key_digit<unsigned>(unsigned k, int shift, unsigned mask, bool) {
    return (k >> shift) & mask;
}

template <>
__device__ __forceinline__ unsigned key_digit<unsigned long long>(unsigned long long k, int shift,
                                                                  unsigned mask, bool flip) {
    if (flip) k ^= 0x8000000000000000ull;  // signed int64 order
    return (unsigned)(k >> shift) & mask;
}

template <typename K>
__global__ __launch_bounds__(kSortThreads) void radix_hist_kernel(
    int n, const K *__restrict__ keys, int shift, int nbits, bool flip, int nblocks,
    unsigned *__restrict__ counts) {
    __shared__ unsigned h[256];
    h[threadIdx.x] = 0u;
    __syncthreads();
    const unsigned mask = (1u << nbits) - 1u;
    const int base = blockIdx.x * kSortBlock;
#pragma unroll
    for (int j = 0; j < kSortRounds; ++j) {
        const int i = base + j * kSortThreads + threadIdx.x;
        if (i < n) atomicAdd(&h[key_digit<K>(keys[i], shift, mask, flip)], 1u);
    }
    __syncthreads();
    if (threadIdx.x <= (int)mask) counts[threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];
}

// Exclusive scan of the digit-major [digits][nblocks] count matrix (one
// 1024-thread workgroup; thread t owns a contiguous chunk).
__global__ __launch_bounds__(1024) void radix_scan_kernel(int total, const unsigned *__restrict__ counts,
                                                          unsigned *__restrict__ offsets) {
    __shared__ unsigned ws[16];
    const int per = (total + 1023) / 1024;
    const int b = threadIdx.x * per;
    const int e = min(b + per, total);
    unsigned s = 0u;
    for (int i = b; i < e; ++i) s += counts[i];
    // block exclusive scan of s over 1024 threads (16 waves)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    unsigned incl = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned u = __shfl_up(incl, off, 64);
        if (lane >= off) incl += u;
    }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    unsigned wo = 0u;
    for (int k = 0; k < w; ++k) wo += ws[k];
    unsigned run = wo + incl - s;
    for (int i = b; i < e; ++i) {
        const unsigned c = counts[i];
        offsets[i] = run;
        run += c;
    }
}

template <typename K>
__global__ __launch_bounds__(kSortThreads) void radix_scatter_kernel(
    int n, const K *__restrict__ keys_in, const int *__restrict__ vals_in, K *__restrict__ keys_out,
    int *__restrict__ vals_out, int shift, int nbits, bool flip, int nblocks,
    const unsigned *__restrict__ offsets) {
    __shared__ unsigned wcnt[kWaves][256];
    __shared__ unsigned goff[256];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const unsigned mask = (1u << nbits) - 1u;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) wcnt[k][tid] = 0u;
    if (tid <= (int)mask) goff[tid] = offsets[tid * nblocks + blockIdx.x];
    __syncthreads();

    const unsigned long long lt = (1ull << lane) - 1ull;
    const int base = blockIdx.x * kSortBlock + w * (kSortRounds * 64);
    K key[kSortRounds];
    int val[kSortRounds];
    unsigned dig[kSortRounds], rank[kSortRounds];
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
        const int i = base + r * 64 + lane;
        const bool valid = i < n;
        key[r] = valid ? keys_in[i] : (K)0;
        val[r] = valid ? vals_in[i] : 0;
        const unsigned d = valid ? key_digit<K>(key[r], shift, mask, flip) : 0u;
        dig[r] = d;
        // wave64 multisplit: lanes holding the same digit
        unsigned long long same = __ballot(valid);
        for (int bit = 0; bit < nbits; ++bit) {
            const unsigned long long bl = __ballot((d >> bit) & 1u);
            same &= ((d >> bit) & 1u) ? bl : ~bl;
        }
        const unsigned before = (unsigned)__popcll(same & lt);
        const unsigned cnt = (unsigned)__popcll(same);
        const unsigned old = valid ? wcnt[w][d] : 0u;
        __builtin_amdgcn_wave_barrier();
        if (valid && before == 0u) wcnt[w][d] = old + cnt;
        __builtin_amdgcn_wave_barrier();
        rank[r] = old + before;
    }
    __syncthreads();
    if (tid <= (int)mask) {
        unsigned s = 0u;
#pragma unroll
        for (int k = 0; k < kWaves; ++k) {
            const unsigned c = wcnt[k][tid];
            wcnt[k][tid] = s;
            s += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortRounds; ++r) {
        const int i = base + r * 64 + lane;
        if (i < n) {
            const unsigned pos = goff[dig[r]] + wcnt[w][dig[r]] + rank[r];
            keys_out[pos] = key[r];
            vals_out[pos] = val[r];
        }
    }
}

// forward.cu:141-163 on sorted tile ids (hot path, 32-bit keys).
__global__ __launch_bounds__(256) void bins_u32_kernel(int n, const unsigned *__restrict__ tiles,
                                                       int2 *__restrict__ bins, int rows) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int cur = (int)tiles[i];
    if (i == 0 && cur < rows) bins[cur].x = 0;
    if (i == n - 1 && cur < rows) bins[cur].y = n;
    if (i > 0) {
        const int prev = (int)tiles[i - 1];
        if (prev != cur) {
            if (prev < rows) bins[prev].y = i;
            if (cur < rows) bins[cur].x = i;
        }
    }
}

// forward.cu:141-163 on sorted int64 isect ids (drop-in op).
__global__ __launch_bounds__(256) void bins_i64_kernel(int n, const long long *__restrict__ keys,
                                                       int2 *__restrict__ bins, int rows) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int cur = (int)(keys[i] >> 32);
    const bool cur_ok = cur >= 0 && cur < rows;
    if (i == 0 && cur_ok) bins[cur].x = 0;
    if (i == n - 1 && cur_ok) bins[cur].y = n;
    if (i > 0) {
        const int prev = (int)(keys[i - 1] >> 32);
        if (prev != cur) {
            if (prev >= 0 && prev < rows) bins[prev].y = i;
            if (cur_ok) bins[cur].x = i;
        }
    }
}

// Expand sorted tile ids to the reference's int64 isect ids.
__global__ __launch_bounds__(256) void expand_isect_kernel(int n, const unsigned *__restrict__ tiles,
                                                           const int *__restrict__ gids,
                                                           const float *__restrict__ depths,
                                                           long long *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const long long d = depths ? (long long)(int)__float_as_uint(depths[gids[i]]) : 0ll;
    out[i] = ((long long)tiles[i] << 32) | d;
}

// ---------------------------------------------------------------------------
// Sync-free tile-major binning.  The (tile, splat) list sorted
// by (tile, splat id) is the transpose of the splat -> tiles incidence, so it
// is built as a CSR transpose instead of a sort:
//   count   per splat, one atomic increment per tile of its bbox;
//   scan    one workgroup: tile_bins = [start, end) (0,0 when empty), the
//           fill cursors, and M on the device (no host round trip);
//   fill    per splat, slot = atomic cursor bump, ids[slot] = splat
//           (order inside a tile depends on atomic timing);
//   sort    per tile, the segment is put in splat-id order: shuffle ranks
//           for <= 64 entries, an LDS bitmap over the id range otherwise.
// Splat ids are unique inside a tile, so the result is exactly the stable
// sort's order and deterministic.  Every size the host needs is a capacity
// (the caller's bound on M), never M itself.
__global__ __launch_bounds__(256) void tile_count_kernel(int n, const float2 *__restrict__ xys,
                                                         const int *__restrict__ radii, int tbx,
                                                         int tby, unsigned *__restrict__ counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int r = radii[i];
    if (r <= 0) return;
    const float2 c = xys[i];
    count_splat_tiles(c.x, c.y, r, tbx, tby, counts);
}

__global__ __launch_bounds__(1024) void tile_scan_kernel(int ntiles, unsigned *__restrict__ counts,
                                                         int2 *__restrict__ bins,
                                                         unsigned *__restrict__ cursor,
                                                         int *__restrict__ meta, long long capacity,
                                                         int zero_counts, unsigned tile_cap) {
    scan_tile_counts<1024>(ntiles, counts, bins, cursor, meta, capacity, zero_counts != 0, tile_cap);
}

// The cursor atomics of a splat are issued in batches of 8 before any of
// their results is waited for (one round trip per batch, not per tile).
// ``ends`` (tile_cap mode): a slot at or past the tile's capped end is dropped.
__global__ __launch_bounds__(256) void tile_fill_kernel(int n, const float2 *__restrict__ xys,
                                                        const int *__restrict__ radii, int tbx, int tby,
                                                        unsigned *__restrict__ cursor,
                                                        int *__restrict__ ids, long long capacity,
                                                        const int2 *__restrict__ ends) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int r = radii[i];
    if (r <= 0) return;
    unsigned x0, y0, x1, y1;
    const float2 c = xys[i];
    tile_bbox(c.x, c.y, (float)r, tbx, tby, x0, y0, x1, y1);
    constexpr int kBatch = 8;
    unsigned tl[kBatch];
    int cnt = 0;
    auto flush = [&]() {
        unsigned sl[kBatch];
#pragma unroll
        for (int k = 0; k < kBatch; ++k)
            if (k < cnt) sl[k] = atomicAdd(cursor + tl[k], 1u);
#pragma unroll
        for (int k = 0; k < kBatch; ++k)
            if (k < cnt && (long long)sl[k] < capacity && (!ends || (int)sl[k] < ends[tl[k]].y))
                ids[sl[k]] = i;
        cnt = 0;
    };
    for (unsigned y = y0; y < y1; ++y)
        for (unsigned x = x0; x < x1; ++x) {
            tl[cnt < kBatch ? cnt : 0] = y * (unsigned)tbx + x;
            if (++cnt == kBatch) flush();
        }
    if (cnt) flush();
}

// One wave per tile; ``bm`` is ``bm_words`` words of dynamic LDS.
__global__ __launch_bounds__(64) void tile_segsort_kernel(int ntiles, const int2 *__restrict__ bins,
                                                          const int *__restrict__ ids_in,
                                                          int *__restrict__ ids_out, int bm_words,
                                                          long long capacity) {
    extern __shared__ unsigned bm[];
    const int tile = blockIdx.x;
    const int lane = threadIdx.x;
    const int2 range = bins[tile];
    const int n = range.y - range.x;
    if (n <= 0 || (long long)range.y > capacity) return;
    const int *in = ids_in + range.x;
    int *out = ids_out + range.x;
    if (n <= 64) {
        const int v = lane < n ? in[lane] : 0x7fffffff;
        int rank = 0;
        for (int k = 0; k < n; ++k) rank += (__shfl(v, k, 64) < v) ? 1 : 0;
        if (lane < n) out[rank] = v;
        return;
    }
    int lo = 0x7fffffff, hi = -1;
    for (int j = lane; j < n; j += 64) {
        const int v = in[j];
        lo = min(lo, v);
        hi = max(hi, v);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, __shfl_xor(lo, off, 64));
        hi = max(hi, __shfl_xor(hi, off, 64));
    }
    int written = 0;
    const long long span = 32ll * bm_words;
    for (long long base = lo; base <= hi; base += span) {
        const int words = (int)min((long long)bm_words, ((hi - base) >> 5) + 1);
        for (int w = lane; w < words; w += 64) bm[w] = 0u;
        __syncthreads();
        for (int j = lane; j < n; j += 64) {
            const long long d = (long long)in[j] - base;
            if (d >= 0 && d < 32ll * words) atomicOr(bm + (d >> 5), 1u << (d & 31));
        }
        __syncthreads();
        const int per = (words + 63) / 64;
        const int w0 = min(lane * per, words), w1 = min(w0 + per, words);
        int cnt = 0;
        for (int w = w0; w < w1; ++w) cnt += __popc(bm[w]);
        int incl = cnt;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int u = __shfl_up(incl, off, 64);
            if (lane >= off) incl += u;
        }
        int pos = written + incl - cnt;
        for (int w = w0; w < w1; ++w) {
            unsigned bits = bm[w];
            while (bits) {
                const int bit = __ffs(bits) - 1;
                out[pos++] = (int)(base + 32 * w + bit);
                bits &= bits - 1u;
            }
        }
        written += __shfl(incl, 63, 64);
        __syncthreads();
    }
}

// tile_cap mode: a tile with more than tile_cap entries kept an arbitrary
// tile_cap of them; its first tile_cap ids are rebuilt in id order by one
// wave scanning every splat's bbox (rare: trained frames' densest tiles).
__global__ __launch_bounds__(64) void tile_overflow_kernel(int n, const float2 *__restrict__ xys,
                                                           const int *__restrict__ radii, int tbx,
                                                           int tby, const unsigned *__restrict__ counts,
                                                           const int2 *__restrict__ bins,
                                                           int *__restrict__ ids_out, unsigned tile_cap) {
    const int tile = blockIdx.x;
    if (counts[tile] <= tile_cap) return;
    const int2 range = bins[tile];
    wave_brute_ids(xys, radii, 0, n, tbx, tby, tile, ids_out + range.x);
}

// ---------------------------------------------------------------------------
// Host-side drivers.
struct SortPlan {
    int nblocks;
    size_t counts_bytes;
};

static SortPlan sort_plan(int n) {
    SortPlan p;
    p.nblocks = ceil_div(n > 0 ? n : 1, kSortBlock);
    p.counts_bytes = align_up(sizeof(unsigned) * 256 * (size_t)p.nblocks);
    return p;
}

template <typename K>
static int radix_pass(int n, const K *kin, const int *vin, K *kout, int *vout, int shift, int nbits,
                      bool flip, unsigned *counts, unsigned *offsets, int nblocks, hipStream_t s) {
    hipLaunchKernelGGL(radix_hist_kernel<K>, dim3(nblocks), dim3(kSortThreads), 0, s, n, kin, shift,
                       nbits, flip, nblocks, counts);
    const int total = (1 << nbits) * nblocks;
    hipLaunchKernelGGL(radix_scan_kernel, dim3(1), dim3(1024), 0, s, total, counts, offsets);
    hipLaunchKernelGGL(radix_scatter_kernel<K>, dim3(nblocks), dim3(kSortThreads), 0, s, n, kin, vin,
                       kout, vout, shift, nbits, flip, nblocks, offsets);
    return check_launch("radix_pass");
}

// Sort (keys, vals) on bits [begin_bit, end_bit); result in (kout, vout).
// kbuf/vbuf: scratch of n elements.  kin/vin are not modified.
template <typename K>
static int radix_sort(int n, const K *kin, const int *vin, K *kout, int *vout, K *kbuf, int *vbuf,
                      int begin_bit, int end_bit, bool flip, unsigned *counts, unsigned *offsets,
                      hipStream_t s) {
    const int nblocks = sort_plan(n).nblocks;
    int npass = 0;
    int shifts[8], nbits[8];
    for (int b = begin_bit; b < end_bit && npass < 8; b += 8) {
        shifts[npass] = b;
        nbits[npass] = min(8, end_bit - b);
        ++npass;
    }
    if (npass == 0) {
        if (dev_copy(kout, kin, sizeof(K) * (size_t)n, s) != GSVC_OK ||
            dev_copy(vout, vin, sizeof(int) * (size_t)n, s) != GSVC_OK)
            return set_error(GSVC_ERR_HIP, "radix_sort: copy failed");
        return GSVC_OK;
    }
    const K *ck = kin;
    const int *cv = vin;
    for (int p = 0; p < npass; ++p) {
        const bool to_out = ((npass - 1 - p) % 2) == 0;
        K *dk = to_out ? kout : kbuf;
        int *dv = to_out ? vout : vbuf;
        const int rc = radix_pass<K>(n, ck, cv, dk, dv, shifts[p], nbits[p], flip, counts, offsets,
                                     nblocks, s);
        if (rc) return rc;
        ck = dk;
        cv = dv;
    }
    return GSVC_OK;
}

size_t sort_u32_counts_bytes(int n) { return sort_plan(n).counts_bytes; }

int sort_u32_pairs(int n, const unsigned *kin, const int *vin, unsigned *kout, int *vout,
                   unsigned *kbuf, int *vbuf, int bits, unsigned *counts, unsigned *offsets,
                   hipStream_t s) {
    if (n <= 0) return GSVC_OK;
    return radix_sort<unsigned>(n, kin, vin, kout, vout, kbuf, vbuf, 0, bits, false, counts,
                                offsets, s);
}

static int bits_for(int count) {
    int b = 0;
    while ((1ll << b) < (long long)count) ++b;
    return b;
}

int tile_bins_from_counts(int num_points, const float2 *xys, const int *radii, int tbx, int tby,
                          long long capacity, unsigned *counts, unsigned *cursor, int *ids_scratch,
                          int *ids_sorted, int2 *bins, int *meta, bool zero_counts,
                          hipStream_t s, unsigned tile_cap) {
    const int ntiles = tbx * tby;
    if (tile_cap && (!counts || !ids_sorted || zero_counts))
        return set_error(GSVC_ERR_ARG, "tile binning: a per-tile cap needs the counts and the sort");
    if (counts)  // NULL: the producer already scanned (bins, cursor, meta written)
        hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(1024), 0, s, ntiles, counts, bins, cursor,
                           meta, capacity, zero_counts ? 1 : 0, tile_cap);
    if (num_points > 0) {
        hipLaunchKernelGGL(tile_fill_kernel, dim3(ceil_div(num_points, 256)), dim3(256), 0, s,
                           num_points, xys, radii, tbx, tby, cursor, ids_scratch, capacity,
                           tile_cap ? (const int2 *)bins : nullptr);
    }
    if (num_points > 0 && ids_sorted) {  // NULL: the consumer sorts each tile itself
        const int bm_words = min(ceil_div(num_points, 32) + 1, 4096);
        hipLaunchKernelGGL(tile_segsort_kernel, dim3(ntiles), dim3(64), sizeof(unsigned) * bm_words, s,
                           ntiles, (const int2 *)bins, ids_scratch, ids_sorted, bm_words, capacity);
        if (tile_cap)
            hipLaunchKernelGGL(tile_overflow_kernel, dim3(ntiles), dim3(64), 0, s, num_points, xys,
                               radii, tbx, tby, (const unsigned *)counts, (const int2 *)bins,
                               ids_sorted, tile_cap);
    }
    return check_launch("tile binning");
}

}  // namespace gsvc

using namespace gsvc;

extern "C" size_t gsvc_cumsum_workspace_bytes(int num_points) {
    const int nb = ceil_div(num_points > 0 ? num_points : 1, kScanBlock);
    return 4 * align_up(sizeof(int) * (size_t)nb);
}

extern "C" int gsvc_compute_cumulative_intersects(int num_points, const int *num_tiles_hit,
                                                  const float *depths, int *cum_tiles_hit, int *meta,
                                                  void *workspace, size_t workspace_bytes,
                                                  void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (num_points <= 0) {
        if (dev_zero(meta, 4 * sizeof(int), s) != GSVC_OK)
            return set_error(GSVC_ERR_HIP, "compute_cumulative_intersects: memset failed");
        return GSVC_OK;
    }
    if (workspace_bytes < gsvc_cumsum_workspace_bytes(num_points))
        return set_error(GSVC_ERR_WORKSPACE, "compute_cumulative_intersects: workspace too small");
    const int nb = ceil_div(num_points, kScanBlock);
    char *w = (char *)workspace;
    const size_t slot = align_up(sizeof(int) * (size_t)nb);
    int *bsum = (int *)w;
    unsigned *bor = (unsigned *)(w + slot);
    unsigned *band = (unsigned *)(w + 2 * slot);
    int *bcnt = (int *)(w + 3 * slot);
    hipLaunchKernelGGL(cum_reduce_kernel, dim3(nb), dim3(kScanThreads), 0, s, num_points,
                       num_tiles_hit, depths, bsum, bor, band, bcnt);
    hipLaunchKernelGGL(cum_scan_kernel, dim3(nb), dim3(kScanThreads), 0, s, num_points, nb,
                       num_tiles_hit, bsum, bor, band, bcnt, cum_tiles_hit, meta);
    return check_launch("compute_cumulative_intersects");
}

extern "C" int gsvc_map_gaussian_to_intersects(int num_points, int num_intersects, const float *xys,
                                               const float *depths, const int *radii,
                                               const int *cum_tiles_hit, int tbx, int tby, int tbz,
                                               int64_t *isect_ids, int *gaussian_ids, void *stream) {
    (void)tbz;
    if (num_points < 0 || num_intersects < 0)
        return set_error(GSVC_ERR_ARG, "map_gaussian_to_intersects: bad sizes");
    hipStream_t s = (hipStream_t)stream;
    if (num_intersects > 0) {
        if (dev_zero(isect_ids, sizeof(int64_t) * (size_t)num_intersects, s) != GSVC_OK ||
            dev_zero(gaussian_ids, sizeof(int) * (size_t)num_intersects, s) != GSVC_OK)
            return set_error(GSVC_ERR_HIP, "map_gaussian_to_intersects: memset failed");
    }
    if (num_points == 0) return GSVC_OK;
    hipLaunchKernelGGL(map_isect_kernel, dim3(ceil_div(num_points, 256)), dim3(256), 0, s, num_points,
                       num_intersects, (const float2 *)xys, depths, radii, cum_tiles_hit, tbx, tby,
                       (long long *)isect_ids, gaussian_ids);
    return check_launch("map_gaussian_to_intersects");
}

extern "C" size_t gsvc_sort_pairs_workspace_bytes(int n) {
    const SortPlan p = sort_plan(n);
    return align_up(sizeof(int64_t) * (size_t)(n > 0 ? n : 1)) +
           align_up(sizeof(int) * (size_t)(n > 0 ? n : 1)) + 2 * p.counts_bytes;
}

extern "C" int gsvc_sort_isect_pairs(int n, const int64_t *keys_in, const int *vals_in,
                                     int64_t *keys_out, int *vals_out, int begin_bit, int end_bit,
                                     void *workspace, size_t workspace_bytes, void *stream) {
    if (n < 0 || begin_bit < 0 || end_bit > 64 || begin_bit > end_bit)
        return set_error(GSVC_ERR_ARG, "sort_isect_pairs: bad arguments");
    if (n == 0) return GSVC_OK;
    if (workspace_bytes < gsvc_sort_pairs_workspace_bytes(n))
        return set_error(GSVC_ERR_WORKSPACE, "sort_isect_pairs: workspace too small");
    const SortPlan p = sort_plan(n);
    char *w = (char *)workspace;
    unsigned long long *kbuf = (unsigned long long *)w;
    w += align_up(sizeof(int64_t) * (size_t)n);
    int *vbuf = (int *)w;
    w += align_up(sizeof(int) * (size_t)n);
    unsigned *counts = (unsigned *)w;
    unsigned *offsets = (unsigned *)(w + p.counts_bytes);
    // Signed order: the sign bit is flipped when forming digits of the top byte.
    return radix_sort<unsigned long long>(n, (const unsigned long long *)keys_in, vals_in,
                                          (unsigned long long *)keys_out, vals_out, kbuf, vbuf,
                                          begin_bit, end_bit, end_bit == 64, counts, offsets,
                                          (hipStream_t)stream);
}

extern "C" int gsvc_get_tile_bin_edges(int num_intersects, const int64_t *isect_ids_sorted,
                                       int *tile_bins, int rows, void *stream) {
    if (num_intersects < 0 || rows < 0) return set_error(GSVC_ERR_ARG, "get_tile_bin_edges: bad sizes");
    hipStream_t s = (hipStream_t)stream;
    if (rows > 0 && dev_zero(tile_bins, sizeof(int) * 2 * (size_t)rows, s) != GSVC_OK)
        return set_error(GSVC_ERR_HIP, "get_tile_bin_edges: memset failed");
    if (num_intersects == 0) return GSVC_OK;
    hipLaunchKernelGGL(bins_i64_kernel, dim3(ceil_div(num_intersects, 256)), dim3(256), 0, s,
                       num_intersects, (const long long *)isect_ids_sorted, (int2 *)tile_bins, rows);
    return check_launch("get_tile_bin_edges");
}

extern "C" size_t gsvc_bin_tiles_workspace_bytes(int num_points, int num_intersects, int num_tiles) {
    (void)num_points;
    (void)num_tiles;
    const int m = num_intersects > 0 ? num_intersects : 1;
    const SortPlan p = sort_plan(m);
    return 3 * align_up(sizeof(unsigned) * (size_t)m) + 2 * align_up(sizeof(int) * (size_t)m) +
           2 * p.counts_bytes;
}

extern "C" int gsvc_bin_and_sort_tiles(int num_points, int num_intersects, const float *xys,
                                       const float *depths, const int *radii,
                                       const int *cum_tiles_hit, int tbx, int tby,
                                       int *gaussian_ids_sorted, int *tile_bins, int tile_bins_rows,
                                       int64_t *isect_ids_sorted, void *workspace,
                                       size_t workspace_bytes, void *stream) {
    const int num_tiles = tbx * tby;
    if (num_points < 0 || num_intersects < 0 || tbx <= 0 || tby <= 0 || tile_bins_rows < num_tiles)
        return set_error(GSVC_ERR_ARG, "bin_and_sort_tiles: bad sizes (rows %d < tiles %d?)",
                         tile_bins_rows, num_tiles);
    hipStream_t s = (hipStream_t)stream;
    if (dev_zero(tile_bins, sizeof(int) * 2 * (size_t)tile_bins_rows, s) != GSVC_OK)
        return set_error(GSVC_ERR_HIP, "bin_and_sort_tiles: memset failed");
    const int m = num_intersects;
    if (m == 0 || num_points == 0) return GSVC_OK;
    if (workspace_bytes < gsvc_bin_tiles_workspace_bytes(num_points, m, num_tiles))
        return set_error(GSVC_ERR_WORKSPACE, "bin_and_sort_tiles: workspace too small");
    const SortPlan p = sort_plan(m);
    char *w = (char *)workspace;
    const size_t ks = align_up(sizeof(unsigned) * (size_t)m);
    unsigned *keysA = (unsigned *)w;
    unsigned *keysB = (unsigned *)(w + ks);
    unsigned *keysOut = (unsigned *)(w + 2 * ks);
    const size_t vs = align_up(sizeof(int) * (size_t)m);
    int *valsA = (int *)(w + 3 * ks);
    int *valsB = (int *)(w + 3 * ks + vs);
    unsigned *counts = (unsigned *)(w + 3 * ks + 2 * vs);
    unsigned *offsets = (unsigned *)((char *)counts + p.counts_bytes);
    // Every slot is written by the emission when cum is consistent with the
    // bboxes (it is: both come from the same projection); guard anyway.
    hipLaunchKernelGGL(map_tiles_kernel, dim3(ceil_div(num_points, 256)), dim3(256), 0, s, num_points,
                       m, (const float2 *)xys, radii, cum_tiles_hit, tbx, tby, keysA, valsA);
    int rc = check_launch("bin_and_sort_tiles: map");
    if (rc) return rc;
    const int tbits = bits_for(num_tiles);
    rc = radix_sort<unsigned>(m, keysA, valsA, keysOut, gaussian_ids_sorted, keysB, valsB, 0, tbits,
                              false, counts, offsets, s);
    if (rc) return rc;
    hipLaunchKernelGGL(bins_u32_kernel, dim3(ceil_div(m, 256)), dim3(256), 0, s, m, keysOut,
                       (int2 *)tile_bins, tile_bins_rows);
    if (isect_ids_sorted)
        hipLaunchKernelGGL(expand_isect_kernel, dim3(ceil_div(m, 256)), dim3(256), 0, s, m, keysOut,
                           gaussian_ids_sorted, depths, (long long *)isect_ids_sorted);
    return check_launch("bin_and_sort_tiles");
}

// Sync-free tile-major binning (see tile_count_kernel).  Workspace: counts and
// cursors, one u32 each per tile.
extern "C" size_t gsvc_bin_tiles_counted_workspace_bytes(int num_tiles) {
    return 2 * align_up(sizeof(unsigned) * (size_t)(num_tiles > 0 ? num_tiles : 1));
}

extern "C" int gsvc_bin_tiles_counted(int num_points, const float *xys, const int *radii, int tbx,
                                      int tby, long long capacity, int tile_cap, int *ids_scratch,
                                      int *gaussian_ids_sorted, int *tile_bins, int *meta,
                                      void *workspace, size_t workspace_bytes, void *stream) {
    const int ntiles = tbx * tby;
    if (num_points < 0 || tbx <= 0 || tby <= 0 || capacity < 0 || tile_cap < 0)
        return set_error(GSVC_ERR_ARG, "bin_tiles_counted: bad sizes");
    // the overflow rebuild (tile_overflow_kernel -> wave_brute_ids) writes exactly
    // kTilePix ids per overfull tile, so a cap is either off or the 256 entries
    // the rasterizers read (forward.cu:569-571,613)
    if (tile_cap != 0 && tile_cap != kTilePix)
        return set_error(GSVC_ERR_ARG, "bin_tiles_counted: tile_cap must be 0 or 256");
    if (tile_cap && !gaussian_ids_sorted)
        return set_error(GSVC_ERR_ARG, "bin_tiles_counted: tile_cap needs gaussian_ids_sorted");
    if (workspace_bytes < gsvc_bin_tiles_counted_workspace_bytes(ntiles))
        return set_error(GSVC_ERR_WORKSPACE, "bin_tiles_counted: workspace too small");
    hipStream_t s = (hipStream_t)stream;
    unsigned *counts = (unsigned *)workspace;
    unsigned *cursor = (unsigned *)((char *)workspace + align_up(sizeof(unsigned) * (size_t)ntiles));
    if (dev_zero(counts, sizeof(unsigned) * (size_t)ntiles, s) != GSVC_OK)
        return set_error(GSVC_ERR_HIP, "bin_tiles_counted: memset failed");
    if (num_points > 0)
        hipLaunchKernelGGL(tile_count_kernel, dim3(ceil_div(num_points, 256)), dim3(256), 0, s,
                           num_points, (const float2 *)xys, radii, tbx, tby, counts);
    return tile_bins_from_counts(num_points, (const float2 *)xys, radii, tbx, tby, capacity, counts,
                                 cursor, ids_scratch, gaussian_ids_sorted, (int2 *)tile_bins, meta,
                                 false, s, (unsigned)tile_cap);
}
