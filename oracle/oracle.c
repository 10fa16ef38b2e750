/*
 * oracle.c -- CPU restatement of the reference gsplat 2D-splat path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * kernels in gsvc_amd/csrc.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product path never calls it.
 *
 * Each function restates one reference kernel (paths relative to
 * /root/reference/gsplat/gsplat/cuda/csrc):
 *   oracle_project_2d_forward   foward2d.cu:12-69, helpers.cuh:11-68
 *   oracle_project_2d_backward  backward2d.cu:8-51, helpers.cuh:71-82
 *   oracle_cov2d_bounds         bindings.cu:21-39, helpers.cuh:45-68
 *   oracle_map_intersects       forward.cu:100-136
 *   oracle_tile_bin_edges       forward.cu:141-163
 *   oracle_sort_pairs           utils.py:164-165 (torch.sort + gather, stable)
 *   oracle_raster_sum_forward   forward.cu:512-627
 *   oracle_raster_sum_backward  backward.cu:696-862
 *   oracle_raster_forward       forward.cu:252-374  (alpha compositing)
 *   oracle_raster_backward      backward.cu:138-315 (alpha compositing)
 *
 * Floating-point contract (shared with the HIP kernels):
 *   - built with -ffp-contract=off; every fused multiply-add is an explicit
 *     fmaf(), so the op sequence is fixed;
 *   - division and sqrt are IEEE (correctly rounded) on both sides;
 *   - __expf(x) of the reference is exp2(x * log2(e)); the oracle uses libm
 *     exp2f, the GPU uses v_exp_f32 (<= 1 ulp apart).  Pixels whose alpha is
 *     within a few ulps of 1/255 are "borderline" and reported by the tests;
 *   - float->int conversion saturates and maps NaN to 0 (v_cvt_i32_f32).
 * Sums that the GPU forms by tree reduction + atomics (backward gradients)
 * are accumulated in double here and compared with a relative tolerance.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <limits.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define TILE 16
#define TILE_PIX 256
#define NEG_LOG2E (-1.4426950408889634f)

static int cvt_i32(float f) {
    if (f != f) return 0;
    if (f >= 2147483648.0f) return INT_MAX;
    if (f <= -2147483648.0f) return INT_MIN;
    return (int)f;
}

static unsigned umin_(unsigned a, unsigned b) { return a < b ? a : b; }

/* helpers.cuh:11-43 get_bbox / get_tile_bbox */
static void tile_bbox(float cx, float cy, float radius, int tbx, int tby,
                      unsigned *minx, unsigned *miny, unsigned *maxx, unsigned *maxy) {
    float tcx = cx / (float)TILE, tcy = cy / (float)TILE;
    float trx = radius / (float)TILE, try_ = radius / (float)TILE;
    int a;
    a = cvt_i32(tcx - trx);            *minx = umin_((unsigned)(a > 0 ? a : 0), (unsigned)tbx);
    a = cvt_i32((tcx + trx) + 1.0f);   *maxx = umin_((unsigned)(a > 0 ? a : 0), (unsigned)tbx);
    a = cvt_i32(tcy - try_);           *miny = umin_((unsigned)(a > 0 ? a : 0), (unsigned)tby);
    a = cvt_i32((tcy + try_) + 1.0f);  *maxy = umin_((unsigned)(a > 0 ? a : 0), (unsigned)tby);
}

/* helpers.cuh:45-68 compute_cov2d_bounds */
static int cov2d_bounds(float cxx, float cxy, float cyy, float *conic, float *radius) {
    float det = cxx * cyy - cxy * cxy;
    if (det == 0.0f) return 0;
    float inv_det = 1.0f / det;
    conic[0] = cyy * inv_det;
    conic[1] = -cxy * inv_det;
    conic[2] = cxx * inv_det;
    float b = 0.5f * (cxx + cyy);
    float disc = fmaxf(0.1f, b * b - det);
    float v1 = b + sqrtf(disc);
    float v2 = b - sqrtf(disc);
    *radius = ceilf(3.0f * sqrtf(fmaxf(v1, v2)));
    return 1;
}

/* foward2d.cu:12-69.  Outputs are fully written (zeros for skipped splats,
 * matching the torch::zeros allocation of bindings.cu:808-817). */
void oracle_project_2d_forward(int n, const float *means2d, const float *L,
                               int img_h, int img_w, int tbx, int tby,
                               float *xys, float *depths, int *radii,
                               float *conics, int *num_tiles_hit) {
    const float hw = 0.5f * (float)(unsigned)img_w;
    const float hh = 0.5f * (float)(unsigned)img_h;
    for (int i = 0; i < n; ++i) {
        xys[2 * i] = xys[2 * i + 1] = 0.0f;
        depths[i] = 0.0f;
        radii[i] = 0;
        conics[3 * i] = conics[3 * i + 1] = conics[3 * i + 2] = 0.0f;
        num_tiles_hit[i] = 0;
        float cx = fmaf(hw, means2d[2 * i], hw);
        float cy = fmaf(hh, means2d[2 * i + 1], hh);
        float l11 = L[3 * i], l21 = L[3 * i + 1], l22 = L[3 * i + 2];
        float cxx = l11 * l11;
        float cxy = l11 * l21;
        float cyy = l21 * l21 + l22 * l22;
        float conic[3], radius;
        if (!cov2d_bounds(cxx, cxy, cyy, conic, &radius)) continue;
        conics[3 * i] = conic[0]; conics[3 * i + 1] = conic[1]; conics[3 * i + 2] = conic[2];
        xys[2 * i] = cx; xys[2 * i + 1] = cy;
        radii[i] = cvt_i32(radius);
        unsigned x0, y0, x1, y1;
        tile_bbox(cx, cy, radius, tbx, tby, &x0, &y0, &x1, &y1);
        int32_t area = (int32_t)((x1 - x0) * (y1 - y0));
        if (area <= 0) continue;
        num_tiles_hit[i] = area;
    }
}

/* bindings.cu:21-39 */
void oracle_cov2d_bounds(int n, const float *covs, float *conics, float *radii) {
    for (int i = 0; i < n; ++i) {
        float c[3] = {0, 0, 0}, r = 0.0f;
        /* the reference kernel leaves conic/radius uninitialised on det==0 and
         * writes them anyway; the build writes zeros there (documented). */
        if (!cov2d_bounds(covs[3 * i], covs[3 * i + 1], covs[3 * i + 2], c, &r)) {
            c[0] = c[1] = c[2] = 0.0f; r = 0.0f;
        }
        conics[3 * i] = c[0]; conics[3 * i + 1] = c[1]; conics[3 * i + 2] = c[2];
        radii[i] = r;
    }
}

/* backward2d.cu:8-51 with cov2d_to_conic_vjp (helpers.cuh:71-82) expanded
 * in glm's mat2 product order (column-major, type_mat2x2.inl operator*). */
void oracle_project_2d_backward(int n, const float *L, int img_h, int img_w,
                                const int *radii, const float *conics,
                                const float *v_xy, const float *v_conic,
                                float *v_cov2d, float *v_mean2d, float *v_L) {
    const float hw = 0.5f * (float)(unsigned)img_w;
    const float hh = 0.5f * (float)(unsigned)img_h;
    for (int i = 0; i < n; ++i) {
        v_cov2d[3 * i] = v_cov2d[3 * i + 1] = v_cov2d[3 * i + 2] = 0.0f;
        v_mean2d[2 * i] = v_mean2d[2 * i + 1] = 0.0f;
        v_L[3 * i] = v_L[3 * i + 1] = v_L[3 * i + 2] = 0.0f;
        if (radii[i] <= 0) continue;
        float X00 = conics[3 * i], X01 = conics[3 * i + 1], X10 = X01, X11 = conics[3 * i + 2];
        float G00 = v_conic[3 * i], G01 = v_conic[3 * i + 1], G10 = G01, G11 = v_conic[3 * i + 2];
        float N00 = -X00, N01 = -X01, N10 = -X10, N11 = -X11;
        /* P = (-X) * G */
        float P00 = N00 * G00 + N10 * G01;
        float P01 = N01 * G00 + N11 * G01;
        float P10 = N00 * G10 + N10 * G11;
        float P11 = N01 * G10 + N11 * G11;
        /* V = P * X */
        float V00 = P00 * X00 + P10 * X01;
        float V01 = P01 * X00 + P11 * X01;
        float V10 = P00 * X10 + P10 * X11;
        float V11 = P01 * X10 + P11 * X11;
        float g11 = V00, g12 = V10 + V01, g22 = V11;
        v_cov2d[3 * i] = g11; v_cov2d[3 * i + 1] = g12; v_cov2d[3 * i + 2] = g22;
        float l11 = L[3 * i], l21 = L[3 * i + 1], l22 = L[3 * i + 2];
        /* the doubled cross term is the reference's formula */
        v_L[3 * i]     = 2.0f * l11 * g11 + 2.0f * g12 * l21;
        v_L[3 * i + 1] = 2.0f * l11 * g12 + 2.0f * l21 * g22;
        v_L[3 * i + 2] = 2.0f * l22 * g22;
        v_mean2d[2 * i]     = v_xy[2 * i] * hw;
        v_mean2d[2 * i + 1] = v_xy[2 * i + 1] * hh;
    }
}

/* forward.cu:100-136.  depth bits are sign-extended into the low 32 bits of
 * the key exactly as the reference's (int64_t)*(int32_t*)&depth. */
void oracle_map_intersects(int n, const float *xys, const float *depths, const int *radii,
                           const int *cum, int tbx, int tby,
                           int64_t *isect_ids, int *gaussian_ids) {
    for (int i = 0; i < n; ++i) {
        if (radii[i] <= 0) continue;
        unsigned x0, y0, x1, y1;
        tile_bbox(xys[2 * i], xys[2 * i + 1], (float)radii[i], tbx, tby, &x0, &y0, &x1, &y1);
        int32_t cur = (i == 0) ? 0 : cum[i - 1];
        int32_t dbits;
        memcpy(&dbits, &depths[i], 4);
        int64_t depth_id = (int64_t)dbits;
        for (int y = (int)y0; y < (int)y1; ++y)
            for (int x = (int)x0; x < (int)x1; ++x) {
                int64_t tile_id = (int64_t)(y * tbx + x);
                isect_ids[cur] = (tile_id << 32) | depth_id;
                gaussian_ids[cur] = i;
                ++cur;
            }
    }
}

/* forward.cu:141-163 into a zero-initialised [rows,2] table. */
void oracle_tile_bin_edges(int m, const int64_t *isect_sorted, int *bins, int rows) {
    memset(bins, 0, sizeof(int) * 2 * (size_t)rows);
    for (int i = 0; i < m; ++i) {
        int32_t cur = (int32_t)(isect_sorted[i] >> 32);
        if (i == 0 && cur >= 0 && cur < rows) bins[2 * cur] = 0;
        if (i == m - 1 && cur >= 0 && cur < rows) bins[2 * cur + 1] = m;
        if (i == 0) continue;
        int32_t prev = (int32_t)(isect_sorted[i - 1] >> 32);
        if (prev != cur) {
            if (prev >= 0 && prev < rows) bins[2 * prev + 1] = i;
            if (cur >= 0 && cur < rows) bins[2 * cur] = i;
        }
    }
}

/* utils.py:164-165: torch.sort(int64) then gather; ties keep input order. */
static void msort(int64_t *k, int *v, int64_t *tk, int *tv, int lo, int hi) {
    if (hi - lo < 2) return;
    int mid = lo + (hi - lo) / 2;
    msort(k, v, tk, tv, lo, mid);
    msort(k, v, tk, tv, mid, hi);
    int a = lo, b = mid, o = lo;
    while (a < mid && b < hi) {
        if (k[b] < k[a]) { tk[o] = k[b]; tv[o++] = v[b++]; }
        else { tk[o] = k[a]; tv[o++] = v[a++]; }
    }
    while (a < mid) { tk[o] = k[a]; tv[o++] = v[a++]; }
    while (b < hi) { tk[o] = k[b]; tv[o++] = v[b++]; }
    memcpy(k + lo, tk + lo, sizeof(int64_t) * (size_t)(hi - lo));
    memcpy(v + lo, tv + lo, sizeof(int) * (size_t)(hi - lo));
}

void oracle_sort_pairs(int m, const int64_t *keys, const int *vals,
                       int64_t *keys_out, int *vals_out) {
    memcpy(keys_out, keys, sizeof(int64_t) * (size_t)m);
    memcpy(vals_out, vals, sizeof(int) * (size_t)m);
    int64_t *tk = (int64_t *)malloc(sizeof(int64_t) * (size_t)(m > 0 ? m : 1));
    int *tv = (int *)malloc(sizeof(int) * (size_t)(m > 0 ? m : 1));
    msort(keys_out, vals_out, tk, tv, 0, m);
    free(tk); free(tv);
}

/* sigma of forward.cu:595-597 in the build's fixed op order */
static inline float splat_sigma(float a, float b, float c, float dx, float dy) {
    float ha = 0.5f * a, hc = 0.5f * c;
    float cq = (hc * dy) * dy;
    float bdy = b * dy;
    float q = fmaf(ha, dx, bdy);
    return fmaf(q, dx, cq);
}

/* Threads of the per-tile loops below (OpenMP; 1 unless set -- tiles are
 * independent, so any count gives the same results).  Used by bench.py's
 * all-core CPU baseline. */
int oracle_set_threads(int n) {
#ifdef _OPENMP
    omp_set_num_threads(n > 0 ? n : 1);
    return n > 0 ? n : 1;
#else
    (void)n;
    return 1;
#endif
}

/* forward.cu:512-627.  One tile = 16x16 pixels; only the first 256 sorted
 * entries of a tile are blended (forward.cu:569-571,613). */
void oracle_raster_sum_forward(int tbx, int tby, int img_w, int img_h,
                               const int *ids, const int *bins,
                               const float *xys, const float *conics,
                               const float *colors, const float *opac,
                               float *out_img, float *final_Ts, int *final_idx) {
#pragma omp parallel for schedule(dynamic, 8)
    for (int tile = 0; tile < tbx * tby; ++tile) {
        int ty = tile / tbx, tx = tile - ty * tbx;
        int r0 = bins[2 * tile], r1 = bins[2 * tile + 1];
        int end = r1;
        if (end - r0 > TILE_PIX) end = r0 + TILE_PIX;
        for (int ly = 0; ly < TILE; ++ly)
            for (int lx = 0; lx < TILE; ++lx) {
                int i = ty * TILE + ly, j = tx * TILE + lx;
                if (i >= img_h || j >= img_w) continue;
                float px = (float)j, py = (float)i;
                float acc0 = 0.0f, acc1 = 0.0f, acc2 = 0.0f;
                int last = 0;
                for (int k = r0; k < end; ++k) {
                    int g = ids[k];
                    float dx = xys[2 * g] - px, dy = xys[2 * g + 1] - py;
                    float s = splat_sigma(conics[3 * g], conics[3 * g + 1], conics[3 * g + 2], dx, dy);
                    float e = exp2f(s * NEG_LOG2E);
                    float alpha = fminf(1.0f, opac[g] * e);
                    if (s < 0.0f || alpha < 1.0f / 255.0f) continue;
                    acc0 = fmaf(colors[3 * g], alpha, acc0);
                    acc1 = fmaf(colors[3 * g + 1], alpha, acc1);
                    acc2 = fmaf(colors[3 * g + 2], alpha, acc2);
                    last = k;
                }
                size_t p = (size_t)i * (size_t)img_w + (size_t)j;
                out_img[3 * p] = acc0; out_img[3 * p + 1] = acc1; out_img[3 * p + 2] = acc2;
                final_Ts[p] = 1.0f;
                final_idx[p] = last;
            }
    }
}

/* backward.cu:696-862 for the tiles [t0, t1).  Gradients are accumulated in
 * double (the GPU sums by tree reduction + atomics; tests compare with a
 * relative tolerance). */
static void raster_sum_backward_tiles(int t0, int t1, int tbx, int img_w, int img_h,
                                      const int *ids, const int *bins,
                                      const float *xys, const float *conics,
                                      const float *colors, const float *opac,
                                      const int *final_idx, const float *v_out,
                                      double *v_xy, double *v_conic, double *v_rgb,
                                      double *v_opac) {
    for (int tile = t0; tile < t1; ++tile) {
        int ty = tile / tbx, tx = tile - ty * tbx;
        int r0 = bins[2 * tile], r1 = bins[2 * tile + 1];
        for (int ly = 0; ly < TILE; ++ly)
            for (int lx = 0; lx < TILE; ++lx) {
                int i = ty * TILE + ly, j = tx * TILE + lx;
                if (i >= img_h || j >= img_w) continue;
                size_t p = (size_t)i * (size_t)img_w + (size_t)j;
                int bin_final = final_idx[p];
                float vo0 = v_out[3 * p], vo1 = v_out[3 * p + 1], vo2 = v_out[3 * p + 2];
                float px = (float)j, py = (float)i;
                for (int k = r1 - 1; k >= r0; --k) {
                    if (k > bin_final) continue;
                    int g = ids[k];
                    float a = conics[3 * g], b = conics[3 * g + 1], c = conics[3 * g + 2];
                    float dx = xys[2 * g] - px, dy = xys[2 * g + 1] - py;
                    float s = splat_sigma(a, b, c, dx, dy);
                    float vis = exp2f(s * NEG_LOG2E);
                    float o = opac[g];
                    float alpha = fminf(1.0f, o * vis);
                    if (s < 0.0f || alpha < 1.0f / 255.0f) continue;
                    float r = colors[3 * g], gg = colors[3 * g + 1], bb = colors[3 * g + 2];
                    float v_alpha = fmaf(bb, vo2, fmaf(gg, vo1, r * vo0));
                    float v_sigma = (-o * vis) * v_alpha;
                    v_rgb[3 * g]     += (double)(alpha * vo0);
                    v_rgb[3 * g + 1] += (double)(alpha * vo1);
                    v_rgb[3 * g + 2] += (double)(alpha * vo2);
                    float hs = 0.5f * v_sigma;
                    v_conic[3 * g]     += (double)((hs * dx) * dx);
                    v_conic[3 * g + 1] += (double)((hs * dx) * dy);
                    v_conic[3 * g + 2] += (double)((hs * dy) * dy);
                    v_xy[2 * g]     += (double)(v_sigma * fmaf(a, dx, b * dy));
                    v_xy[2 * g + 1] += (double)(v_sigma * fmaf(b, dx, c * dy));
                    v_opac[g] += (double)(vis * v_alpha);
                }
            }
    }
}

/* The whole backward.  With one thread the tiles run in order into the
 * outputs; with more, each thread takes a contiguous tile range (static, so
 * the split depends only on the thread count) into its own double buffers,
 * which are then added in thread order: results equal the one-thread sums up
 * to double rounding (invisible after the float32 cast). */
void oracle_raster_sum_backward(int tbx, int tby, int img_w, int img_h, int n,
                                const int *ids, const int *bins,
                                const float *xys, const float *conics,
                                const float *colors, const float *opac,
                                const int *final_idx, const float *v_out,
                                double *v_xy, double *v_conic, double *v_rgb, double *v_opac) {
    size_t nn = (size_t)n;
    memset(v_xy, 0, sizeof(double) * 2 * nn);
    memset(v_conic, 0, sizeof(double) * 3 * nn);
    memset(v_rgb, 0, sizeof(double) * 3 * nn);
    memset(v_opac, 0, sizeof(double) * nn);
    int tiles = tbx * tby;
    int nt = 1;
#ifdef _OPENMP
    nt = omp_get_max_threads();
#endif
    double *buf = NULL;
    if (nt > 1 && tiles >= 2 * nt)
        buf = (double *)calloc((size_t)nt * 9 * nn, sizeof(double));
    if (!buf) {
        raster_sum_backward_tiles(0, tiles, tbx, img_w, img_h, ids, bins, xys, conics, colors,
                                  opac, final_idx, v_out, v_xy, v_conic, v_rgb, v_opac);
        return;
    }
#pragma omp parallel num_threads(nt)
    {
        int t = 0;
#ifdef _OPENMP
        t = omp_get_thread_num();
#endif
        double *b = buf + (size_t)t * 9 * nn;
        int t0 = (int)((long long)tiles * t / nt), t1 = (int)((long long)tiles * (t + 1) / nt);
        raster_sum_backward_tiles(t0, t1, tbx, img_w, img_h, ids, bins, xys, conics, colors, opac,
                                  final_idx, v_out, b, b + 2 * nn, b + 5 * nn, b + 8 * nn);
    }
    for (int t = 0; t < nt; ++t) {
        const double *b = buf + (size_t)t * 9 * nn;
        for (size_t i = 0; i < 2 * nn; ++i) v_xy[i] += b[i];
        for (size_t i = 0; i < 3 * nn; ++i) v_conic[i] += b[2 * nn + i];
        for (size_t i = 0; i < 3 * nn; ++i) v_rgb[i] += b[5 * nn + i];
        for (size_t i = 0; i < nn; ++i) v_opac[i] += b[8 * nn + i];
    }
    free(buf);
}

/* forward.cu:252-374: front-to-back alpha compositing over ALL entries of the
 * tile, alpha clamped at 0.999, stop when next_T <= 1e-4, plus background. */
void oracle_raster_forward(int tbx, int tby, int img_w, int img_h,
                           const int *ids, const int *bins,
                           const float *xys, const float *conics,
                           const float *colors, const float *opac, const float *bg,
                           float *out_img, float *final_Ts, int *final_idx) {
    for (int ty = 0; ty < tby; ++ty)
        for (int tx = 0; tx < tbx; ++tx) {
            int tile = ty * tbx + tx;
            int r0 = bins[2 * tile], r1 = bins[2 * tile + 1];
            for (int ly = 0; ly < TILE; ++ly)
                for (int lx = 0; lx < TILE; ++lx) {
                    int i = ty * TILE + ly, j = tx * TILE + lx;
                    if (i >= img_h || j >= img_w) continue;
                    float px = (float)j, py = (float)i;
                    float T = 1.0f, acc0 = 0.0f, acc1 = 0.0f, acc2 = 0.0f;
                    int last = 0;
                    for (int k = r0; k < r1; ++k) {
                        int g = ids[k];
                        float dx = xys[2 * g] - px, dy = xys[2 * g + 1] - py;
                        float s = splat_sigma(conics[3 * g], conics[3 * g + 1], conics[3 * g + 2], dx, dy);
                        float e = exp2f(s * NEG_LOG2E);
                        float alpha = fminf(0.999f, opac[g] * e);
                        if (s < 0.0f || alpha < 1.0f / 255.0f) continue;
                        float next_T = T * (1.0f - alpha);
                        if (next_T <= 1e-4f) break;
                        float vis = alpha * T;
                        acc0 = fmaf(colors[3 * g], vis, acc0);
                        acc1 = fmaf(colors[3 * g + 1], vis, acc1);
                        acc2 = fmaf(colors[3 * g + 2], vis, acc2);
                        T = next_T;
                        last = k;
                    }
                    size_t p = (size_t)i * (size_t)img_w + (size_t)j;
                    out_img[3 * p]     = fmaf(T, bg[0], acc0);
                    out_img[3 * p + 1] = fmaf(T, bg[1], acc1);
                    out_img[3 * p + 2] = fmaf(T, bg[2], acc2);
                    final_Ts[p] = T;
                    final_idx[p] = last;
                }
        }
}

/* backward.cu:138-315: reverse recursion, alpha clamped at 0.99 (not 0.999). */
void oracle_raster_backward(int tbx, int tby, int img_w, int img_h, int n,
                            const int *ids, const int *bins,
                            const float *xys, const float *conics,
                            const float *colors, const float *opac, const float *bg,
                            const float *final_Ts, const int *final_idx,
                            const float *v_out, const float *v_out_alpha,
                            double *v_xy, double *v_conic, double *v_rgb, double *v_opac) {
    memset(v_xy, 0, sizeof(double) * 2 * (size_t)n);
    memset(v_conic, 0, sizeof(double) * 3 * (size_t)n);
    memset(v_rgb, 0, sizeof(double) * 3 * (size_t)n);
    memset(v_opac, 0, sizeof(double) * (size_t)n);
    for (int ty = 0; ty < tby; ++ty)
        for (int tx = 0; tx < tbx; ++tx) {
            int tile = ty * tbx + tx;
            int r0 = bins[2 * tile], r1 = bins[2 * tile + 1];
            for (int ly = 0; ly < TILE; ++ly)
                for (int lx = 0; lx < TILE; ++lx) {
                    int i = ty * TILE + ly, j = tx * TILE + lx;
                    if (i >= img_h || j >= img_w) continue;
                    size_t p = (size_t)i * (size_t)img_w + (size_t)j;
                    float T_final = final_Ts[p], T = T_final;
                    float buf0 = 0.0f, buf1 = 0.0f, buf2 = 0.0f;
                    int bin_final = final_idx[p];
                    float vo0 = v_out[3 * p], vo1 = v_out[3 * p + 1], vo2 = v_out[3 * p + 2];
                    float voa = v_out_alpha[p];
                    float px = (float)j, py = (float)i;
                    for (int k = r1 - 1; k >= r0; --k) {
                        if (k > bin_final) continue;
                        int g = ids[k];
                        float a = conics[3 * g], b = conics[3 * g + 1], c = conics[3 * g + 2];
                        float dx = xys[2 * g] - px, dy = xys[2 * g + 1] - py;
                        float s = splat_sigma(a, b, c, dx, dy);
                        float vis = exp2f(s * NEG_LOG2E);
                        float o = opac[g];
                        float alpha = fminf(0.99f, o * vis);
                        if (s < 0.0f || alpha < 1.0f / 255.0f) continue;
                        float ra = 1.0f / (1.0f - alpha);
                        T = T * ra;
                        float fac = alpha * T;
                        float r = colors[3 * g], gg = colors[3 * g + 1], bb = colors[3 * g + 2];
                        float tfra = T_final * ra;
                        float v_alpha = (r * T - buf0 * ra) * vo0;
                        v_alpha = fmaf(gg * T - buf1 * ra, vo1, v_alpha);
                        v_alpha = fmaf(bb * T - buf2 * ra, vo2, v_alpha);
                        v_alpha = fmaf(tfra, voa, v_alpha);
                        v_alpha = fmaf(-tfra * bg[0], vo0, v_alpha);
                        v_alpha = fmaf(-tfra * bg[1], vo1, v_alpha);
                        v_alpha = fmaf(-tfra * bg[2], vo2, v_alpha);
                        buf0 = fmaf(r, fac, buf0);
                        buf1 = fmaf(gg, fac, buf1);
                        buf2 = fmaf(bb, fac, buf2);
                        float v_sigma = (-o * vis) * v_alpha;
                        v_rgb[3 * g]     += (double)(fac * vo0);
                        v_rgb[3 * g + 1] += (double)(fac * vo1);
                        v_rgb[3 * g + 2] += (double)(fac * vo2);
                        float hs = 0.5f * v_sigma;
                        v_conic[3 * g]     += (double)((hs * dx) * dx);
                        v_conic[3 * g + 1] += (double)((hs * dx) * dy);
                        v_conic[3 * g + 2] += (double)((hs * dy) * dy);
                        v_xy[2 * g]     += (double)(v_sigma * fmaf(a, dx, b * dy));
                        v_xy[2 * g + 1] += (double)(v_sigma * fmaf(b, dx, c * dy));
                        v_opac[g] += (double)(vis * v_alpha);
                    }
                }
        }
}

/* Per-pixel alpha of the candidate splat closest to the 1/255 threshold:
 * used by the tests to flag "borderline" pixels where a 1-ulp exp difference
 * between libm and v_exp_f32 may legitimately flip final_idx. */
void oracle_sum_min_margin(int tbx, int tby, int img_w, int img_h,
                           const int *ids, const int *bins,
                           const float *xys, const float *conics, const float *opac,
                           float *margin) {
    for (int ty = 0; ty < tby; ++ty)
        for (int tx = 0; tx < tbx; ++tx) {
            int tile = ty * tbx + tx;
            int r0 = bins[2 * tile], r1 = bins[2 * tile + 1];
            int end = r1 - r0 > TILE_PIX ? r0 + TILE_PIX : r1;
            for (int ly = 0; ly < TILE; ++ly)
                for (int lx = 0; lx < TILE; ++lx) {
                    int i = ty * TILE + ly, j = tx * TILE + lx;
                    if (i >= img_h || j >= img_w) continue;
                    float best = INFINITY;
                    for (int k = r0; k < end; ++k) {
                        int g = ids[k];
                        float dx = xys[2 * g] - (float)j, dy = xys[2 * g + 1] - (float)i;
                        float s = splat_sigma(conics[3 * g], conics[3 * g + 1], conics[3 * g + 2], dx, dy);
                        float alpha = fminf(1.0f, opac[g] * exp2f(s * NEG_LOG2E));
                        float m = fabsf(alpha * 255.0f - 1.0f);
                        if (s >= 0.0f && m < best) best = m;
                    }
                    margin[(size_t)i * (size_t)img_w + (size_t)j] = best;
                }
        }
}
