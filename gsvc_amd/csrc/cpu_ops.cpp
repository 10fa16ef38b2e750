// CPU dispatch of the two drop-in operators (BASELINE configs[0]: a 256x256
// frame with 1k splats, the PyTorch-CPU case; SURVEY §8b "add a CPU dispatch
// for config 1").  CPU tensors go here, HIP tensors to libgsvc_amd.so; a
// tensor is never moved between the two, so a GPU call cannot end up on this
// code.  Host C++ with OpenMP over tiles, built into libgsvc_amd_cpu.so with
// -ffp-contract=off and no fast math: the op sequence of the gfx950 kernels
// (csrc/project2d.h, raster_sum.hip, common.h) with exp(-s) = exp2f(s *
// -log2(e)), so indices, radii, bins and the image match the kernels'
// contract bit for bit (the GPU's v_exp_f32 differs from exp2f by <= 1 ulp).
//
// Reference semantics: foward2d.cu:12-69 and helpers.cuh:11-68 (projection),
// backward2d.cu:8-51 (its VJP, doubled cross term), utils.py:99-167 and
// forward.cu:100-163 (binning: a tile's first 256 entries in (tile, splat id)
// order -- the stable sort of (tile << 32 | depth 0) keys), forward.cu:512-627
// (sum composite, final_idx = last contributing sorted index) and
// backward.cu:696-862 (its backward, entries k <= final_idx only).
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <omp.h>

#include <algorithm>
#include <vector>

namespace {

constexpr int kTile = 16;
constexpr int kKeep = 256;  // entries per tile the sum composite reads (config.h BLOCK_SIZE)
constexpr float kNegLog2e = -1.4426950408889634f;
constexpr float kAlphaMin = 1.0f / 255.0f;

// v_cvt_i32_f32: truncate, saturate, NaN -> 0
int cvt_i32(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return 2147483647;
    if (f <= -2147483648.0f) return -2147483647 - 1;
    return (int)f;
}

struct Box {
    int x0, y0, x1, y1;  // [x0, x1) x [y0, y1) in tiles, clamped
};

Box tile_box(float cx, float cy, float radius, int tbx, int tby) {
    const float tcx = cx / (float)kTile, tcy = cy / (float)kTile, tr = radius / (float)kTile;
    auto clampi = [](int a, int hi) { return std::min(std::max(a, 0), hi); };
    return Box{clampi(cvt_i32(tcx - tr), tbx), clampi(cvt_i32(tcy - tr), tby),
               clampi(cvt_i32((tcx + tr) + 1.0f), tbx), clampi(cvt_i32((tcy + tr) + 1.0f), tby)};
}

float sigma_of(float ha, float b, float hc, float dx, float dy) {
    const float cq = (hc * dy) * dy;
    const float q = fmaf(ha, dx, b * dy);
    return fmaf(q, dx, cq);
}

}  // namespace

extern "C" {

int gsvc_cpu_abi_version(void) { return 1; }

// OpenMP threads of this library's loops (results do not depend on it; the
// bench's k = 1 / all-cores CPU baselines).  Returns the count in effect.
int gsvc_cpu_set_threads(int n) {
    omp_set_num_threads(n > 0 ? n : 1);
    return omp_get_max_threads();
}

// foward2d.cu:12-69 for every splat; returns M = the sum of num_tiles_hit.
long long gsvc_cpu_project_gaussians_2d_forward(int n, const float *means2d, const float *L,
                                                unsigned img_h, unsigned img_w, int tbx, int tby,
                                                float *xys, float *depths, int *radii,
                                                float *conics, int *num_tiles_hit) {
    const float hw = 0.5f * (float)img_w, hh = 0.5f * (float)img_h;
    long long m = 0;
#pragma omp parallel for reduction(+ : m) schedule(static)
    for (int i = 0; i < n; ++i) {
        const float l11 = L[3 * i], l21 = L[3 * i + 1], l22 = L[3 * i + 2];
        const float cxx = l11 * l11, cxy = l11 * l21, cyy = l21 * l21 + l22 * l22;
        const float det = cxx * cyy - cxy * cxy;
        float x = 0.f, y = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f;
        int rad = 0, hit = 0;
        if (det != 0.0f) {
            const float inv = 1.0f / det;
            c0 = cyy * inv;
            c1 = -cxy * inv;
            c2 = cxx * inv;
            const float b = 0.5f * (cxx + cyy);
            const float disc = fmaxf(0.1f, b * b - det);
            const float r = ceilf(3.0f * sqrtf(fmaxf(b + sqrtf(disc), b - sqrtf(disc))));
            x = fmaf(hw, means2d[2 * i], hw);
            y = fmaf(hh, means2d[2 * i + 1], hh);
            rad = cvt_i32(r);
            const Box bb = tile_box(x, y, r, tbx, tby);
            const int area = (bb.x1 - bb.x0) * (bb.y1 - bb.y0);
            hit = area > 0 ? area : 0;
        }
        xys[2 * i] = x;
        xys[2 * i + 1] = y;
        depths[i] = 0.0f;
        radii[i] = rad;
        conics[3 * i] = c0;
        conics[3 * i + 1] = c1;
        conics[3 * i + 2] = c2;
        num_tiles_hit[i] = hit;
        m += hit;
    }
    return m;
}

// backward2d.cu:8-51 (cov2d_to_conic_vjp expanded in glm's column-major
// order; the doubled cross term of :39-41 kept).
void gsvc_cpu_project_gaussians_2d_backward(int n, const float *L, unsigned img_h, unsigned img_w,
                                            const int *radii, const float *conics,
                                            const float *v_xy, const float *v_conic,
                                            float *v_cov2d, float *v_mean2d, float *v_L) {
    const float hw = 0.5f * (float)img_w, hh = 0.5f * (float)img_h;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i) {
        float g11 = 0.f, g12 = 0.f, g22 = 0.f, vl0 = 0.f, vl1 = 0.f, vl2 = 0.f, vmx = 0.f, vmy = 0.f;
        if (radii[i] > 0) {
            const float X00 = conics[3 * i], X01 = conics[3 * i + 1], X10 = X01, X11 = conics[3 * i + 2];
            const float G00 = v_conic[3 * i], G01 = v_conic[3 * i + 1], G10 = G01, G11 = v_conic[3 * i + 2];
            const float N00 = -X00, N01 = -X01, N10 = -X10, N11 = -X11;
            const float P00 = N00 * G00 + N10 * G01, P01 = N01 * G00 + N11 * G01;
            const float P10 = N00 * G10 + N10 * G11, P11 = N01 * G10 + N11 * G11;
            g11 = P00 * X00 + P10 * X01;
            g12 = (P00 * X10 + P10 * X11) + (P01 * X00 + P11 * X01);
            g22 = P01 * X10 + P11 * X11;
            const float l11 = L[3 * i], l21 = L[3 * i + 1], l22 = L[3 * i + 2];
            vl0 = 2.0f * l11 * g11 + 2.0f * g12 * l21;
            vl1 = 2.0f * l11 * g12 + 2.0f * l21 * g22;
            vl2 = 2.0f * l22 * g22;
            vmx = v_xy[2 * i] * hw;
            vmy = v_xy[2 * i + 1] * hh;
        }
        v_cov2d[3 * i] = g11;
        v_cov2d[3 * i + 1] = g12;
        v_cov2d[3 * i + 2] = g22;
        v_mean2d[2 * i] = vmx;
        v_mean2d[2 * i + 1] = vmy;
        v_L[3 * i] = vl0;
        v_L[3 * i + 1] = vl1;
        v_L[3 * i + 2] = vl2;
    }
}

// utils.py:99-167 + forward.cu:100-163 for depth-0 splats: tile t's first
// min(count, 256) splat ids in ascending order at ids[t * 256 ...], its
// bins row [t * 256, t * 256 + kept); returns M (all intersections).
long long gsvc_cpu_bin_tiles(int n, const float *xys, const int *radii, int tbx, int tby,
                             int *ids, int *bins) {
    const int nt = tbx * tby;
    std::vector<int> kept((size_t)nt, 0);
    long long m = 0;
    // splats in id order, each appending to the tiles of its bbox: every
    // tile's list comes out ascending, so its first 256 are the sorted ones
    for (int i = 0; i < n; ++i) {
        if (radii[i] <= 0) continue;
        const Box bb = tile_box(xys[2 * i], xys[2 * i + 1], (float)radii[i], tbx, tby);
        for (int ty = bb.y0; ty < bb.y1; ++ty)
            for (int tx = bb.x0; tx < bb.x1; ++tx) {
                const int t = ty * tbx + tx;
                if (kept[t] < kKeep) ids[(size_t)t * kKeep + kept[t]++] = i;
                ++m;
            }
    }
    for (int t = 0; t < nt; ++t) {
        bins[2 * t] = t * kKeep;
        bins[2 * t + 1] = t * kKeep + kept[t];
    }
    return m;
}

// forward.cu:512-627: out [H, W, 3] (no background), final_idx [H, W].
void gsvc_cpu_rasterize_sum_forward(int tbx, int tby, unsigned img_w, unsigned img_h,
                                    const int *ids, const int *bins, const float *xys,
                                    const float *conics, const float *colors, const float *opac,
                                    float *out, int *final_idx) {
    const int W = (int)img_w, H = (int)img_h;
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < tbx * tby; ++t) {
        const int ty = t / tbx, tx = t - ty * tbx;
        const int b0 = bins[2 * t], b1 = std::min(bins[2 * t + 1], b0 + kKeep);
        for (int py = ty * kTile; py < std::min((ty + 1) * kTile, H); ++py)
            for (int px = tx * kTile; px < std::min((tx + 1) * kTile, W); ++px) {
                float r = 0.f, g = 0.f, b = 0.f;
                int last = 0;
                for (int k = b0; k < b1; ++k) {
                    const int s = ids[k];
                    const float dx = xys[2 * s] - (float)px, dy = xys[2 * s + 1] - (float)py;
                    const float sg = sigma_of(0.5f * conics[3 * s], conics[3 * s + 1],
                                              0.5f * conics[3 * s + 2], dx, dy);
                    const float al = fminf(1.0f, opac[s] * exp2f(sg * kNegLog2e));
                    if (sg < 0.0f || al < kAlphaMin) continue;
                    r = fmaf(colors[3 * s], al, r);
                    g = fmaf(colors[3 * s + 1], al, g);
                    b = fmaf(colors[3 * s + 2], al, b);
                    last = k;
                }
                const size_t p = (size_t)py * W + px;
                out[3 * p] = r;
                out[3 * p + 1] = g;
                out[3 * p + 2] = b;
                final_idx[p] = last;
            }
    }
}

// backward.cu:696-862 into grad [N, 16] (v_xy 0:2, v_conic 2:5, v_colors
// 5:8, v_opacity 8), zeroed here: every (pixel, entry k <= final_idx) pair
// passing the forward's test, in tile order then pixel order (one thread per
// tile, the tiles' sums added per splat after the loop, so the result does
// not depend on the thread count).
void gsvc_cpu_rasterize_sum_backward(unsigned img_h, unsigned img_w, int n, const int *ids,
                                     const int *bins, const float *xys, const float *conics,
                                     const float *colors, const float *opac, const int *final_idx,
                                     const float *v_out, float *grad) {
    const int W = (int)img_w, H = (int)img_h;
    const int tbx = (W + kTile - 1) / kTile, tby = (H + kTile - 1) / kTile, nt = tbx * tby;
    memset(grad, 0, sizeof(float) * 16 * (size_t)n);
    // per tile: the entries' 9 sums, slot j of the tile's list
    std::vector<float> part((size_t)nt * kKeep * 9, 0.0f);
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < nt; ++t) {
        const int ty = t / tbx, tx = t - ty * tbx;
        const int b0 = bins[2 * t], b1 = std::min(bins[2 * t + 1], b0 + kKeep);
        float *pt = part.data() + (size_t)t * kKeep * 9;
        for (int py = ty * kTile; py < std::min((ty + 1) * kTile, H); ++py)
            for (int px = tx * kTile; px < std::min((tx + 1) * kTile, W); ++px) {
                const size_t p = (size_t)py * W + px;
                const float vr = v_out[3 * p], vg = v_out[3 * p + 1], vb = v_out[3 * p + 2];
                for (int k = b0; k < b1 && k <= final_idx[p]; ++k) {
                    const int s = ids[k];
                    const float ca = conics[3 * s], cb = conics[3 * s + 1], cc = conics[3 * s + 2];
                    const float ha = 0.5f * ca, hc = 0.5f * cc;
                    const float dx = xys[2 * s] - (float)px, dy = xys[2 * s + 1] - (float)py;
                    const float sg = sigma_of(ha, cb, hc, dx, dy);
                    const float vis = exp2f(sg * kNegLog2e);
                    const float o = opac[s];
                    const float al = fminf(1.0f, o * vis);
                    if (sg < 0.0f || al < kAlphaMin) continue;
                    const float v_alpha = fmaf(colors[3 * s + 2], vb, fmaf(colors[3 * s + 1], vg, colors[3 * s] * vr));
                    const float v_sigma = (-o * vis) * v_alpha;
                    float *e = pt + (size_t)(k - b0) * 9;
                    e[0] = fmaf(v_sigma, fmaf(ca, dx, cb * dy), e[0]);
                    e[1] = fmaf(v_sigma, fmaf(cb, dx, cc * dy), e[1]);
                    const float hs = 0.5f * v_sigma, hsdx = hs * dx;
                    e[2] = fmaf(hsdx, dx, e[2]);
                    e[3] = fmaf(hsdx, dy, e[3]);
                    e[4] = fmaf(hs * dy, dy, e[4]);
                    e[5] = fmaf(al, vr, e[5]);
                    e[6] = fmaf(al, vg, e[6]);
                    e[7] = fmaf(al, vb, e[7]);
                    e[8] = fmaf(vis, v_alpha, e[8]);
                }
            }
    }
    for (int t = 0; t < nt; ++t) {
        const int b0 = bins[2 * t], b1 = std::min(bins[2 * t + 1], b0 + kKeep);
        const float *pt = part.data() + (size_t)t * kKeep * 9;
        for (int k = b0; k < b1; ++k) {
            float *gr = grad + 16 * (size_t)ids[k];
            for (int c = 0; c < 9; ++c) gr[c] += pt[(size_t)(k - b0) * 9 + c];
        }
    }
}

}  // extern "C"
