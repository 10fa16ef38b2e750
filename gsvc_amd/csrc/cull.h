// Culling of (entry, pixel-block) pairs that cannot contribute: shared by the
// sum composite (raster_sum.hip) and the alpha compositor (raster_alpha.hip).
// A pair whose alpha stays below 1/255 is skipped by the reference kernels
// themselves (forward.cu:334-337, 600-606), so leaving it out changes nothing.
#pragma once

#include "common.h"

namespace gsvc {

// A conic the ellipse culling may be applied to: positive definite and not
// ill-conditioned.  For a*c > 2^13 det (a needle: the quadratic form nearly
// degenerate), the reference's own float32 sigma = 0.5 (a dx^2 + c dy^2) +
// b dx dy cancels -- its rounding error at the ellipse's edge (~2^-24 S2 a c /
// det) outgrows the 0.1 % margin, and along the needle it reads ~0 far
// outside the true ellipse (round 5: a textured-video splat with conic
// (136777, -90810, 60291), float32 det 1024, alpha 1 at pixels 58 px from its
// centre) -- and det itself has lost its bits.  Such entries are not culled.
__device__ __forceinline__ bool cull_conditioned(float a, float c, float det) {
    return a > 0.0f && det > 0.0f && a * c <= 8192.0f * det;
}

// The 4x4-pixel blocks of the kRows-row strip at (bx0, by0) (bit 4 * r + c:
// rows by0 + 4r .. + 3, columns bx0 + 4c .. + 3) that splat (x, y, conic, o)
// can reach with alpha >= 1/255 -- ellipse_hits_rect's test per block, so a
// block left out holds no contributing pixel centre.  kRows = 8: a band, 16:
// the whole tile.
template <int kRows>
__device__ __forceinline__ unsigned ellipse_blocks(float x, float y, float a, float b, float c,
                                                   float o, float bx0, float by0) {
    constexpr unsigned kAll = (1u << kRows) - 1u;  // kRows / 4 row blocks x 4 column blocks
    if (!(o > 0.0f)) return (o <= 0.0f) ? 0u : kAll;  // o <= 0: never valid; NaN: keep
    const float det = a * c - b * b;
    if (!cull_conditioned(a, c, det) || !(o < 3.0e38f) || !(fabsf(x) < 1e30f) || !(fabsf(y) < 1e30f))
        return kAll;  // not positive definite, ill-conditioned or non-finite: no culling
    const float lg = __logf(255.0f * o);
    if (lg < -0.01f) return 0u;  // o < e^-0.01 / 255: alpha < 1/255 everywhere
    const float S2 = 2.0f * (lg * 1.001f + 0.01f);
    // whole tiles: hardware rcp / sqrt (~1 ulp; f32 denormals are kept, so a
    // det near the float maximum still gets its reciprocal) -- the margins
    // dwarf their error; bands keep the IEEE forms (the banded composite's
    // register budget: the shorter sequence spilled there)
    float ex, ey;
    if constexpr (kRows == 16) {
        const float inv_det = __builtin_amdgcn_rcpf(det);
        ex = __builtin_amdgcn_sqrtf(S2 * c * inv_det) * 1.001f + 0.01f;
        ey = __builtin_amdgcn_sqrtf(S2 * a * inv_det) * 1.001f + 0.01f;
    } else {
        ex = sqrtf(S2 * c / det) * 1.001f + 0.01f;
        ey = sqrtf(S2 * a / det) * 1.001f + 0.01f;
    }
    // in strip coordinates, so the block bounds are literals (the origin
    // shift rounds by < 2^-12 px at 1080p, far inside the 0.01 px margin)
    const float u = x - bx0, v = y - by0;
    unsigned cols = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        cols |= ((u + ex >= 4.0f * k) && (u - ex <= 4.0f * k + 3.0f)) ? 1u << k : 0u;
    unsigned m = 0u;
#pragma unroll
    for (int r = 0; r < kRows / 4; ++r)
        m |= ((v + ey >= 4.0f * r) && (v - ey <= 4.0f * r + 3.0f)) ? cols << (4 * r) : 0u;
    return m;
}

// An entry's geometry is small enough that its sigma at any pixel centre of
// an image up to 2^16 wide is finite: |x|, |y| < 2^20 and |a/2|, |b|, |c/2| <
// 2^40 bound dx, dy < 2^21 and every product and sum of the sigma
// evaluation below 2^85, so no inf - inf or 0 * inf -- sigma is never NaN --
// and c/2 carries no sign bit (c/2 in [+0, 2^40)), so (c/2 dy) dy is +0 or
// positive and sigma = fma(q, dx, that) is never -0: NaN and -0 are the two
// values the sigma-threshold alpha cut (kSigmaCutBits, an unsigned compare of
// the bits) decides differently from the reference's test (which keeps both).
// The projection's conics always pass the sign test (c = l11^2 / det, det > 0);
// an operator caller's conics might not.  NaN fails every comparison here.
__device__ __forceinline__ bool geo_bounded(float x, float y, float ha, float b, float hc) {
    constexpr float kPos = 1048576.0f, kCon = 1099511627776.0f;  // 2^20, 2^40
    return fabsf(x) < kPos && fabsf(y) < kPos && fabsf(ha) < kCon && fabsf(b) < kCon &&
           (__float_as_uint(hc) >> 31) == 0u && hc < kCon;
}

}  // namespace gsvc
