// Per-row backward machinery shared by the tile kernels that turn a tile's
// v_out into per-splat gradient sums (train.hip's fused training step,
// raster_sum.hip's and raster_alpha.hip's op-path backwards): an entry's
// alpha >= 1/255 rectangle of tile pixels, work items = rectangle rows, and
// the DPP segmented sums that add an entry's items in a fixed tree order.
#pragma once

#include "cull.h"
#include "frame.h"

namespace gsvc {

// The pixels of the 16x16 tile at (tx0, ty0) at whose centres splat (x, y,
// conic a b c, opacity o) can reach alpha >= 1/255, as a rectangle of tile
// coordinates packed {x0, x1, y0, y1} (4 bits each, inclusive); kNoRect
// when provably none.  alpha >= 1/255 needs sigma <= ln(255 o), i.e.
// d^T C d <= 2 ln(255 o), an ellipse with half-extents sqrt(2 ln(255 o) c / det)
// and sqrt(2 ln(255 o) a / det); the margins (0.1 % + 0.01 px) dwarf fp32
// rounding (the banded forward's test, raster_sum.hip ellipse_hits_rect).  A
// culled (entry, pixel) pair contributes nothing in the reference either.
constexpr unsigned kNoRect = 0x000fu;  // x0 = 15 > x1 = 0: empty (fits the 16-bit LDS slot)
constexpr unsigned kFullRect = 0xf0f0u;  // x 0..15, y 0..15

__device__ __forceinline__ unsigned ellipse_rect(float x, float y, float a, float b, float c,
                                                 float o, float tx0, float ty0) {
    if (!(o > 0.0f)) return (o <= 0.0f) ? kNoRect : kFullRect;  // o <= 0: never valid; NaN: keep
    const float det = a * c - b * b;
    if (!cull_conditioned(a, c, det) || !(o < 3.0e38f) || !(fabsf(x) < 1e30f) || !(fabsf(y) < 1e30f))
        return kFullRect;  // not positive definite, ill-conditioned or non-finite: no culling
    const float lg = __logf(255.0f * o);
    if (lg < -0.01f) return kNoRect;  // o < e^-0.01 / 255: alpha < 1/255 everywhere
    const float S2 = 2.0f * (lg * 1.001f + 0.01f);
    // hardware rcp / sqrt (~1 ulp): the 0.1 % + 0.01 px margins dwarf their error
    const float inv_det = __builtin_amdgcn_rcpf(det);
    const float ex = __builtin_amdgcn_sqrtf(S2 * c * inv_det) * 1.001f + 0.01f;
    const float ey = __builtin_amdgcn_sqrtf(S2 * a * inv_det) * 1.001f + 0.01f;
    const float x0 = fmaxf(ceilf(x - ex - tx0), 0.0f), x1 = fminf(floorf(x + ex - tx0), 15.0f);
    const float y0 = fmaxf(ceilf(y - ey - ty0), 0.0f), y1 = fminf(floorf(y + ey - ty0), 15.0f);
    if (!(x0 <= x1) || !(y0 <= y1)) return kNoRect;
    return (unsigned)x0 | ((unsigned)x1 << 4) | ((unsigned)y0 << 8) | ((unsigned)y1 << 12);
}

// v_out rows padded to 17 words: the backward's lanes read pixels of
// different rows of one column, which with 16-word rows share a bank every 4
// rows (measured: LDS bank conflicts ~ the VALU time at trained density).
constexpr int kVRow = kTile + 1;

// An entry's geometry (x, y, a/2, b; c/2) is bounded (cull.h geo_bounded):
// its sigma is then never NaN, and the sigma-threshold alpha cut applies.
__device__ __forceinline__ bool geo_cut_ok(const float4 &G, float hc) {
    return geo_bounded(G.x, G.y, G.z, G.w, hc);
}

// Inclusive scans over one wave's 64 lanes with DPP (no LDS traffic):
// row_shr 1, 2, 4, 8 inside each 16-lane row, then row_bcast 15 / 31 carry a
// row's last lane into the rows above; ``id`` is the operation's identity.
template <bool kMax>
__device__ __forceinline__ int wave_scan_dpp(int v, int id) {
    auto step = [&](int t) { v = kMax ? max(v, t) : v + t; };
    step(__builtin_amdgcn_update_dpp(id, v, 0x111, 0xf, 0xf, false));  // row_shr:1
    step(__builtin_amdgcn_update_dpp(id, v, 0x112, 0xf, 0xf, false));  // row_shr:2
    step(__builtin_amdgcn_update_dpp(id, v, 0x114, 0xf, 0xf, false));  // row_shr:4
    step(__builtin_amdgcn_update_dpp(id, v, 0x118, 0xf, 0xf, false));  // row_shr:8
    step(__builtin_amdgcn_update_dpp(id, v, 0x142, 0xa, 0xf, false));  // row_bcast:15 -> rows 1, 3
    step(__builtin_amdgcn_update_dpp(id, v, 0x143, 0xc, 0xf, false));  // row_bcast:31 -> rows 2, 3
    return v;
}

// One step of a segmented inclusive sum: lanes whose DPP source lane carries
// the same key add its N sums (sources outside the row / masked rows: key -1,
// and the lane is not written).  ``g += m * g[src]`` with m = 1 or 0 as ONE
// v_fmac_f32_dpp per sum (the compiler does not fold the DPP move into an fma);
// exact while the sums are finite (x * 0 = 0), so a wave with a non-finite sum
// takes the select form (seg_step_sel).  N = 8 (the fused step: no opacity
// gradient) or 9 (the op path: v_opacity too).
#define GSVC_FMAC_DPP8(CTRL)                                                               \
    asm volatile("s_nop 1\n\t"                                                             \
                 "v_fmac_f32_dpp %0, %0, %8 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %1, %1, %8 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %2, %2, %8 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %3, %3, %8 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %4, %4, %8 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %5, %5, %8 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %6, %6, %8 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %7, %7, %8 " CTRL "\n\t"                                  \
                 "s_nop 1"                                                                 \
                 : "+v"(g[0]), "+v"(g[1]), "+v"(g[2]), "+v"(g[3]), "+v"(g[4]), "+v"(g[5]), \
                   "+v"(g[6]), "+v"(g[7])                                                  \
                 : "v"(m))
#define GSVC_FMAC_DPP9(CTRL)                                                               \
    asm volatile("s_nop 1\n\t"                                                             \
                 "v_fmac_f32_dpp %0, %0, %9 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %1, %1, %9 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %2, %2, %9 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %3, %3, %9 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %4, %4, %9 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %5, %5, %9 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %6, %6, %9 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %7, %7, %9 " CTRL "\n\t"                                  \
                 "v_fmac_f32_dpp %8, %8, %9 " CTRL "\n\t"                                  \
                 "s_nop 1"                                                                 \
                 : "+v"(g[0]), "+v"(g[1]), "+v"(g[2]), "+v"(g[3]), "+v"(g[4]), "+v"(g[5]), \
                   "+v"(g[6]), "+v"(g[7]), "+v"(g[8])                                      \
                 : "v"(m))
#define GSVC_FMAC_DPP(CTRL)        \
    if constexpr (N == 8) {        \
        GSVC_FMAC_DPP8(CTRL);      \
    } else {                       \
        GSVC_FMAC_DPP9(CTRL);      \
    }

template <int kCtrl, int kRowMask>
__device__ __forceinline__ float seg_mask(int key) {
    const int ks = __builtin_amdgcn_update_dpp(-1, key, kCtrl, kRowMask, 0xf, false);
    return ks == key ? 1.0f : 0.0f;
}

template <int kCtrl, int kRowMask, int N>
__device__ __forceinline__ void seg_step_sel(float (&g)[N], int key) {
    const int ks = __builtin_amdgcn_update_dpp(-1, key, kCtrl, kRowMask, 0xf, false);
    const bool same = ks == key;
#pragma unroll
    for (int c = 0; c < N; ++c) {
        const float t = __int_as_float(
            __builtin_amdgcn_update_dpp(0, __float_as_int(g[c]), kCtrl, kRowMask, 0xf, false));
        g[c] = same ? g[c] + t : g[c];
    }
}

// Segmented inclusive sums over one wave's 64 lanes, segments = runs of equal
// key >= 0 (contiguous): lane i ends with the sum of its run's lanes <= i.
// The wave_scan_dpp steps; a source lane is added only inside the run, so
// each lane's sum covers exactly [max(run start, ...), i].
template <int N, bool kLong>
__device__ __forceinline__ void wave_seg_sums(float (&g)[N], int key) {
    static_assert(N == 8 || N == 9, "8 or 9 sums");
    // finite unless some sum is inf / NaN (or the total overflows: then the
    // exact select form runs, which is still right)
    float tot = ((g[0] + g[1]) + (g[2] + g[3])) + ((g[4] + g[5]) + (g[6] + g[7]));
    if constexpr (N == 9) tot += g[8];
    if (__ballot(!__builtin_isfinite(tot)) == 0ull) {
        float m;
        m = seg_mask<0x111, 0xf>(key);
        GSVC_FMAC_DPP("row_shr:1 row_mask:0xf bank_mask:0xf");
        m = seg_mask<0x112, 0xf>(key);
        GSVC_FMAC_DPP("row_shr:2 row_mask:0xf bank_mask:0xf");
        m = seg_mask<0x114, 0xf>(key);
        GSVC_FMAC_DPP("row_shr:4 row_mask:0xf bank_mask:0xf");
        if (kLong) {  // runs longer than 8 lanes
            m = seg_mask<0x118, 0xf>(key);
            GSVC_FMAC_DPP("row_shr:8 row_mask:0xf bank_mask:0xf");
        }
        m = seg_mask<0x142, 0xa>(key);
        GSVC_FMAC_DPP("row_bcast:15 row_mask:0xa bank_mask:0xf");
        m = seg_mask<0x143, 0xc>(key);
        GSVC_FMAC_DPP("row_bcast:31 row_mask:0xc bank_mask:0xf");
    } else {
        seg_step_sel<0x111, 0xf>(g, key);  // row_shr:1
        seg_step_sel<0x112, 0xf>(g, key);  // row_shr:2
        seg_step_sel<0x114, 0xf>(g, key);  // row_shr:4
        if (kLong) seg_step_sel<0x118, 0xf>(g, key);  // row_shr:8
        seg_step_sel<0x142, 0xa>(g, key);  // row_bcast:15 -> rows 1, 3
        seg_step_sel<0x143, 0xc>(g, key);  // row_bcast:31 -> rows 2, 3
    }
}
#undef GSVC_FMAC_DPP
#undef GSVC_FMAC_DPP8
#undef GSVC_FMAC_DPP9

}  // namespace gsvc
