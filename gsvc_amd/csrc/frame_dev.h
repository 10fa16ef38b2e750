// Device side of the frame projection, shared by frame.hip (the projection
// kernels) and train.hip (the fused training step's splat kernel, which
// projects the next step's frame from the parameters it has just updated).
#pragma once

#include "binning.h"
#include "frame.h"
#include "project2d.h"

namespace gsvc {

constexpr int kProjThreads = 256;
// K = 1 insertion: the lane walks its bbox row by row; two horizontally
// adjacent tiles whose counters share an aligned 8-byte word take ONE 64-bit
// atomic adding 1 to both halves (a 32-bit count never carries into its
// neighbour), so a splat k tiles wide costs ~k/2 + 1 slot atomics per row.
// The memory-side atomic rate is what bounds the projection at high M
// (trained-like 1080p / 50k splats: 794k insertions).  kB slot atomics are
// generated (unrolled, register-resident), issued, and only then waited for:
// one round trip per kB of them.
// ``ids`` (optional: id slabs, or the training step's carried bins): the
// splat's id into ids[tile][slot] (ids_cap slots per tile) instead of its
// record into the slab.  ``ovf`` (record slabs): slots [256, kCarryCap) as
// ids into ovf[tile][slot - 256].
template <int kB>
__device__ __forceinline__ int slab_insert_pairs(float cx, float cy, int r, int tbx, int tby,
                                                 float4 r0, float4 r1, float4 r2,
                                                 unsigned *__restrict__ counts,
                                                 float4 *__restrict__ slab, int wt,
                                                 int *__restrict__ ids = nullptr,
                                                 int ids_cap = kTilePix,
                                                 int *__restrict__ ovf = nullptr) {
    unsigned x0, y0, x1, y1;
    tile_bbox(cx, cy, (float)r, tbx, tby, x0, y0, x1, y1);
    if (x1 <= x0 || y1 <= y0) return 0;
    const unsigned base_par = (unsigned)(reinterpret_cast<uintptr_t>(counts) >> 2) & 1u;
    const bool wide = x1 - x0 >= 3;  // narrow rows: single atomics (measured faster at 10k)
    const int ntiles = tbx * tby;
    auto put = [&](unsigned t, unsigned sl) {
        if (ids) {
            if (sl < (unsigned)ids_cap) ids[(size_t)t * ids_cap + sl] = __float_as_int(r2.y);
        } else if (sl < (unsigned)kTilePix) {
            float4 *d = slab_rec(slab, ntiles, (int)t, (int)sl);
            d[0] = r0;
            d[1] = r1;
            d[2] = r2;
        } else if (ovf && sl < (unsigned)kCarryCap) {
            ovf[(size_t)t * kOvfSlots + (sl - kTilePix)] = __float_as_int(r2.y);
        }
    };
    int hits = 0;
    unsigned x = x0, y = y0;
    while (y < y1) {
        unsigned op[kB];  // tile << 1 | paired; ~0u: none
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const bool valid = y < y1;
            const unsigned t = y * (unsigned)tbx + x;
            const unsigned pair = (valid && wide && x + 1 < x1 && ((t + base_par) & 1u) == 0) ? 1u : 0u;
            op[k] = valid ? ((t << 1) | pair) : ~0u;
            if (valid) {
                x += 1 + pair;
                if (x >= x1) {
                    x = x0;
                    ++y;
                }
            }
        }
        unsigned lo[kB], hi[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            lo[k] = hi[k] = ~0u;
            if (op[k] != ~0u) {
                const unsigned t = op[k] >> 1;
                if (op[k] & 1u) {
                    const unsigned long long old = atomicAdd(
                        reinterpret_cast<unsigned long long *>(counts + t), 0x100000001ull);
                    lo[k] = (unsigned)old;
                    hi[k] = (unsigned)(old >> 32);
                } else {
                    lo[k] = atomicAdd(counts + t, 1u);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            if (op[k] != ~0u) {
                const unsigned t = op[k] >> 1;
                put(t, lo[k]);
                if (op[k] & 1u) put(t + 1, hi[k]);
                hits += 1 + (int)(op[k] & 1u);
            }
        }
    }
    return hits;
}

// A tile box [x0, x1) x [y0, y1) in two words (x0 | y0 << 16, x1 | y1 << 16);
// {0, 0}: empty.  The carried bins' per-splat boxes (train.hip).
__device__ __forceinline__ uint2 pack_box(unsigned x0, unsigned y0, unsigned x1, unsigned y1) {
    return (x1 > x0 && y1 > y0) ? make_uint2(x0 | (y0 << 16), x1 | (y1 << 16)) : make_uint2(0u, 0u);
}
__device__ __forceinline__ bool box_has(uint2 b, unsigned tx, unsigned ty) {
    return tx >= (b.x & 0xffffu) && tx < (b.y & 0xffffu) && ty >= (b.x >> 16) && ty < (b.y >> 16);
}

// Activations (GaussianSplats_Represent.py:57-70) + projection of splat i and
// its 48-byte record.
struct SplatOut {
    SplatProj P;
    float4 r0, r1, r2;
};

// Projection of splat i from its activated values and its 48-byte record.
__device__ __forceinline__ SplatOut splat_out(int i, float mx, float my, float l11, float l21,
                                              float l22, float r, float g, float b, float o,
                                              float hw, float hh, int tbx, int tby) {
    SplatOut S;
    S.P = project_splat(mx, my, l11, l21, l22, hw, hh, tbx, tby);
    S.r0 = make_float4(S.P.xy.x, S.P.xy.y, 0.5f * S.P.c0, S.P.c1);
    S.r1 = make_float4(0.5f * S.P.c2, o, r, g);
    S.r2 = make_float4(b, __int_as_float(i), S.P.c0, S.P.c2);
    return S;
}

__device__ __forceinline__ SplatOut load_project(int i, const float *__restrict__ xyz, int xyz_tanh,
                                                 const float *__restrict__ chol,
                                                 const float *__restrict__ chol_bound,
                                                 const float *__restrict__ feat,
                                                 const float *__restrict__ rgb_w,
                                                 const float *__restrict__ opac, float hw, float hh,
                                                 int tbx, int tby) {
    float mx = xyz[2 * i], my = xyz[2 * i + 1];
    if (xyz_tanh) {  // get_xyz (:57-59)
        mx = tanhf(mx);
        my = tanhf(my);
    }
    float l11 = chol[3 * i], l21 = chol[3 * i + 1], l22 = chol[3 * i + 2];
    if (chol_bound) {  // get_cholesky_elements (:69-70)
        l11 = l11 + chol_bound[0];
        l21 = l21 + chol_bound[1];
        l22 = l22 + chol_bound[2];
    }
    float r = feat[3 * i], g = feat[3 * i + 1], b = feat[3 * i + 2];
    if (rgb_w) {  // get_features (:61-63)
        const float w = rgb_w[i];
        r = r * w;
        g = g * w;
        b = b * w;
    }
    const float o = opac ? opac[i] : 1.0f;
    return splat_out(i, mx, my, l11, l21, l22, r, g, b, o, hw, hh, tbx, tby);
}

// The block's hit total into this frame's M.
template <int kThr = kProjThreads>
__device__ __forceinline__ void add_hits(int hits, int *s_hits, int *m_acc) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) hits += __shfl_xor(hits, off, 64);
    if ((threadIdx.x & 63) == 0) s_hits[threadIdx.x >> 6] = hits;
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
#pragma unroll
        for (int k = 0; k < kThr / 64; ++k)
            if (k < (int)(blockDim.x >> 6)) tot += s_hits[k];
        if (tot) atomicAdd(m_acc, tot);
    }
}

constexpr int kAggWin = 2048;  // tiles (8 KB of LDS counters)
constexpr int kAggArea = 64;   // a larger bbox inserts directly

__device__ __forceinline__ unsigned strip_key(float x, float y, int rad, int tbx, int tby,
                                              unsigned invisible) {
    if (rad <= 0 || !(x == x) || !(y == y)) return invisible;
    const int tx = min(max(cvt_i32(floorf(x / (float)kTile)), 0), tbx - 1);
    const int ty = min(max(cvt_i32(floorf(y / (float)kTile)), 0), tby - 1);
    // strips of 4 tile rows, swept column by column: 256 consecutive splats
    // centre in a compact ~(10 x 4)-tile patch, with no long jumps
    return (unsigned)(ty >> 2) * (unsigned)(tbx * 4) + (unsigned)tx * 4u + (unsigned)(ty & 3);
}

// The key of invisible splats (sorted last) and the key width.
__host__ __device__ inline unsigned strip_key_invisible(int tbx, int tby) {
    return (unsigned)((tby + 3) >> 2) * (unsigned)(tbx * 4);
}


// The ordered projection's insertion, called by every lane of a kProjThreads
// workgroup (block-uniform control flow): the bboxes of the block's small
// splats (<= kAggArea tiles) span a window of <= kAggWin tiles; the block
// counts them per tile in LDS, takes ONE device-scope atomic per touched tile
// for the base and hands out base + LDS cursor.  Large splats, and blocks
// whose window is too large, insert directly (slab_insert_pairs).  [x0, x1) x
// [y0, y1): the lane's tile bbox (empty: nothing to insert).  Returns the
// lane's insertions (its share of M).
template <int kThr = kProjThreads>
__device__ __forceinline__ int slab_insert_window(const SplatOut &S, unsigned x0, unsigned y0,
                                                  unsigned x1, unsigned y1, int tbx, int tby,
                                                  unsigned *__restrict__ counts,
                                                  float4 *__restrict__ slab, unsigned *s_cnt,
                                                  int (*s_box)[kThr / 64],
                                                  long long *st = nullptr,
                                                  int *__restrict__ ids = nullptr,
                                                  int ids_cap = kTilePix,
                                                  int *__restrict__ ovf = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // diagnostic (st != NULL): s_memrealtime per wave after each phase
    auto mark = [&](int k) {
        if (st) {
            long long t;
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memrealtime %0\n\ts_waitcnt lgkmcnt(0)"
                         : "=s"(t)::"memory");
            if (lane == 0) st[k] = t;
        }
    };
    const bool vis = x1 > x0 && y1 > y0;
    const bool small = vis && (x1 - x0) * (y1 - y0) <= (unsigned)kAggArea;
    // the window of the block's small bboxes
    int bx0 = small ? (int)x0 : 0x7fffffff, by0 = small ? (int)y0 : 0x7fffffff;
    int bx1 = small ? (int)x1 : 0, by1 = small ? (int)y1 : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        bx0 = min(bx0, __shfl_xor(bx0, off, 64));
        by0 = min(by0, __shfl_xor(by0, off, 64));
        bx1 = max(bx1, __shfl_xor(bx1, off, 64));
        by1 = max(by1, __shfl_xor(by1, off, 64));
    }
    if (lane == 0) {
        s_box[0][w] = bx0;
        s_box[1][w] = by0;
        s_box[2][w] = bx1;
        s_box[3][w] = by1;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kThr / 64; ++k) {
        bx0 = min(bx0, s_box[0][k]);
        by0 = min(by0, s_box[1][k]);
        bx1 = max(bx1, s_box[2][k]);
        by1 = max(by1, s_box[3][k]);
    }
    const int ww = bx1 - bx0, wh = by1 - by0;
    const bool agg = ww > 0 && wh > 0 && ww * wh <= kAggWin;  // block-uniform
    mark(4);
    int hits = 0;
    if (vis && !(agg && small))
        hits = slab_insert_pairs<8>(S.P.xy.x, S.P.xy.y, S.P.rad, tbx, tby, S.r0, S.r1, S.r2,
                                    counts, slab, 0, ids, ids_cap, ovf);
    if (agg) {
        const int cells = ww * wh;
        for (int c = tid; c < cells; c += kThr) s_cnt[c] = 0u;
        __syncthreads();
        if (small) {
            for (unsigned y = y0; y < y1; ++y)
                for (unsigned x = x0; x < x1; ++x)
                    atomicAdd(&s_cnt[((int)y - by0) * ww + ((int)x - bx0)], 1u);
        }
        __syncthreads();
        mark(5);
        // one device-scope atomic per touched tile: the window's base slots
        for (int c = tid; c < cells; c += kThr) {
            const unsigned v = s_cnt[c];
            if (v) {
                const int ty = by0 + c / ww, tx = bx0 + c - (c / ww) * ww;
                s_cnt[c] = atomicAdd(counts + ty * tbx + tx, v);
            }
        }
        __syncthreads();
        mark(6);
        if (small) {
            const int ntiles = tbx * tby;
            for (unsigned y = y0; y < y1; ++y)
                for (unsigned x = x0; x < x1; ++x) {
                    const unsigned sl = atomicAdd(&s_cnt[((int)y - by0) * ww + ((int)x - bx0)], 1u);
                    const int tl = (int)(y * (unsigned)tbx + x);
                    if (ids) {
                        if (sl < (unsigned)ids_cap) ids[(size_t)tl * ids_cap + sl] = __float_as_int(S.r2.y);
                    } else if (sl < (unsigned)kTilePix) {
                        float4 *d = slab_rec(slab, ntiles, tl, (int)sl);
                        d[0] = S.r0;
                        d[1] = S.r1;
                        d[2] = S.r2;
                    } else if (ovf && sl < (unsigned)kCarryCap) {
                        ovf[(size_t)tl * kOvfSlots + (sl - kTilePix)] = __float_as_int(S.r2.y);
                    }
                }
            hits += (int)((x1 - x0) * (y1 - y0));
        }
    }
    mark(7);
    return hits;
}

}  // namespace gsvc
