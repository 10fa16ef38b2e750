// Per-splat 2D projection shared by project2d.hip (the op) and frame.hip
// (the fused frame render): one op sequence, so both give identical bits.
#pragma once

#include "common.h"

namespace gsvc {

// helpers.cuh:45-68 compute_cov2d_bounds
__device__ __forceinline__ bool cov2d_bounds(float cxx, float cxy, float cyy,
                                             float &c0, float &c1, float &c2, float &radius) {
    const float det = cxx * cyy - cxy * cxy;
    if (det == 0.0f) return false;
    const float inv_det = 1.0f / det;
    c0 = cyy * inv_det;
    c1 = -cxy * inv_det;
    c2 = cxx * inv_det;
    const float b = 0.5f * (cxx + cyy);
    const float disc = fmaxf(0.1f, b * b - det);
    const float v1 = b + sqrtf(disc);
    const float v2 = b - sqrtf(disc);
    radius = ceilf(3.0f * sqrtf(fmaxf(v1, v2)));
    return true;
}

struct SplatProj {
    float2 xy;
    float c0, c1, c2;  // conic
    int rad, hit;      // radius (pixels), tiles of the bbox
};

// foward2d.cu:12-69 for one splat: means2d (NDC) and Cholesky factor
// (l11, l21, l22) -> centre in pixels, conic, radius, tile count.
// Degenerate covariances give zeros (the reference leaves them unwritten
// after zero-filling).
__device__ __forceinline__ SplatProj project_splat(float mx, float my, float l11, float l21,
                                                   float l22, float hw, float hh, int tbx, int tby) {
    const float cx = fmaf(hw, mx, hw);
    const float cy = fmaf(hh, my, hh);
    const float cxx = l11 * l11;
    const float cxy = l11 * l21;
    const float cyy = l21 * l21 + l22 * l22;
    SplatProj P;
    P.xy = make_float2(0.0f, 0.0f);
    P.c0 = P.c1 = P.c2 = 0.0f;
    P.rad = P.hit = 0;
    float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, radius = 0.0f;
    if (cov2d_bounds(cxx, cxy, cyy, c0, c1, c2, radius)) {
        P.xy = make_float2(cx, cy);
        P.c0 = c0;
        P.c1 = c1;
        P.c2 = c2;
        P.rad = cvt_i32(radius);
        unsigned x0, y0, x1, y1;
        tile_bbox(cx, cy, radius, tbx, tby, x0, y0, x1, y1);
        const int area = (int)((x1 - x0) * (y1 - y0));
        P.hit = area > 0 ? area : 0;
    }
    return P;
}

}  // namespace gsvc
