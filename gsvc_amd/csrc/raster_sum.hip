// Sum rasterizer of GSVC (rasterize_gaussians_sum), forward and backward, gfx950.
//
// Reference: gsplat/gsplat/cuda/csrc/forward.cu:512-627 (rasterize_forward_sum),
// backward.cu:696-862 (rasterize_backward_sum_kernel), bindings.cu:400-469,
// 706-779; Python glue rasterize_sum.py:92-254.
//
// Semantics kept from the reference: out = sum of
// colour * min(1, opacity * exp(-sigma)) over the FIRST <= 256 sorted entries
// of the pixel's tile (the reference breaks after one 256-entry batch,
// forward.cu:569-571,613), skipping sigma < 0 and alpha < 1/255; no
// transmittance, no background; final_idx = last contributing sorted index,
// 0 if none; final_Ts = 1.
//
// Forward layout: one wave64 per 16x16 tile, each lane owns 4
// consecutive pixels of one row (16 rows x 4 quads).  The tile's entries are
// gathered 64 at a time into LDS (one lane per entry) and broadcast from LDS to
// the wave; the row terms of sigma (0.5c dy^2, b dy) are shared by the lane's 4
// pixels.  Each lane stores its 4 pixels as three 16-byte stores of RGB plus
// one 16-byte store of final_idx.  The kernel is bound by the 16 B/pixel of
// output (HBM) plus ~15 VALU per (pixel, entry) pair.
//
// Backward layout: one 256-thread workgroup per tile, ENTRY-parallel: with
// n entries (E = next pow2 >= n) thread t handles entry t % E against the
// pixels [E*(t/E), E*(t/E)+E) of the tile, so gradients accumulate in
// registers without a per-pixel reduction; the t/E groups are combined once
// per entry (shuffles + LDS), then one 64-byte-aligned 9-float record per
// (splat, tile) is added with 9 lanes of one atomic instruction (one memory
// request per entry instead of the reference's 9 per warp).
#include "common.h"

namespace gsvc {

constexpr int kChunk = 64;

__global__ __launch_bounds__(64) void raster_sum_fwd_kernel(
    int tbx, int img_w, int img_h, int ntiles, bool vec_store,
    const int *__restrict__ ids, const int2 *__restrict__ bins, const float2 *__restrict__ xys,
    const float *__restrict__ conics, const float *__restrict__ colors,
    const float *__restrict__ opac, float *__restrict__ out, int *__restrict__ final_idx,
    float *__restrict__ final_Ts) {
    __shared__ float4 s_geo[kChunk];  // x, y, 0.5a, b
    __shared__ float4 s_col[kChunk];  // 0.5c, opacity, r, g
    __shared__ float s_blu[kChunk];   // b
    const int tile = xcd_remap(blockIdx.x, ntiles);
    const int ty = tile / tbx, tx = tile - ty * tbx;
    const int lane = threadIdx.x;
    const int pi = ty * kTile + (lane >> 2);
    const int pj = tx * kTile + ((lane & 3) << 2);
    const float py = (float)pi;
    const float px0 = (float)pj, px1 = (float)(pj + 1), px2 = (float)(pj + 2), px3 = (float)(pj + 3);
    const int2 range = bins[tile];
    int n = range.y - range.x;
    n = n > kTilePix ? kTilePix : (n < 0 ? 0 : n);

    float r0 = 0.f, g0 = 0.f, b0 = 0.f, r1 = 0.f, g1 = 0.f, b1 = 0.f;
    float r2 = 0.f, g2 = 0.f, b2 = 0.f, r3 = 0.f, g3 = 0.f, b3 = 0.f;
    int l0 = 0, l1 = 0, l2 = 0, l3 = 0;

    for (int base = 0; base < n; base += kChunk) {
        const int cnt = min(kChunk, n - base);
        if (lane < cnt) {
            const int g = ids[range.x + base + lane];
            const float2 xy = xys[g];
            const float a = conics[3 * g], b = conics[3 * g + 1], c = conics[3 * g + 2];
            s_geo[lane] = make_float4(xy.x, xy.y, 0.5f * a, b);
            s_col[lane] = make_float4(0.5f * c, opac[g], colors[3 * g], colors[3 * g + 1]);
            s_blu[lane] = colors[3 * g + 2];
        }
        __syncthreads();
        const int k0 = range.x + base;
        for (int t = 0; t < cnt; ++t) {
            const float4 G = s_geo[t];
            const float4 C = s_col[t];
            const float dy = G.y - py;
            const float cq = (C.x * dy) * dy;
            const float bdy = G.w * dy;
            const int k = k0 + t;
#define GSVC_SUM_PIXEL(PX, R, GG, B, L)                                  \
    {                                                                    \
        const float dx = G.x - (PX);                                     \
        const float s = fmaf(fmaf(G.z, dx, bdy), dx, cq);                \
        const float al = fminf(1.0f, C.y * exp_neg(s));                  \
        if (!(s < 0.0f) && !(al < kAlphaMin)) {                          \
            R = fmaf(C.z, al, R);                                        \
            GG = fmaf(C.w, al, GG);                                      \
            B = fmaf(s_blu[t], al, B);                                   \
            L = k;                                                       \
        }                                                                \
    }
            GSVC_SUM_PIXEL(px0, r0, g0, b0, l0)
            GSVC_SUM_PIXEL(px1, r1, g1, b1, l1)
            GSVC_SUM_PIXEL(px2, r2, g2, b2, l2)
            GSVC_SUM_PIXEL(px3, r3, g3, b3, l3)
#undef GSVC_SUM_PIXEL
        }
        __syncthreads();
    }

    if (pi >= img_h) return;
    const size_t p0 = (size_t)pi * (size_t)img_w + (size_t)pj;
    if (vec_store && pj + 3 < img_w) {
        float4 *o = reinterpret_cast<float4 *>(out + 3 * p0);
        o[0] = make_float4(r0, g0, b0, r1);
        o[1] = make_float4(g1, b1, r2, g2);
        o[2] = make_float4(b2, r3, g3, b3);
        *reinterpret_cast<int4 *>(final_idx + p0) = make_int4(l0, l1, l2, l3);
        if (final_Ts) *reinterpret_cast<float4 *>(final_Ts + p0) = make_float4(1.f, 1.f, 1.f, 1.f);
        return;
    }
    const float rr[4] = {r0, r1, r2, r3}, gg[4] = {g0, g1, g2, g3}, bb[4] = {b0, b1, b2, b3};
    const int ll[4] = {l0, l1, l2, l3};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (pj + q < img_w) {
            const size_t p = p0 + q;
            out[3 * p] = rr[q];
            out[3 * p + 1] = gg[q];
            out[3 * p + 2] = bb[q];
            final_idx[p] = ll[q];
            if (final_Ts) final_Ts[p] = 1.0f;
        }
    }
}

__device__ __forceinline__ int ceil_log2(int n) { return n <= 1 ? 0 : 32 - __clz(n - 1); }

__global__ __launch_bounds__(256) void raster_sum_bwd_kernel(
    int tbx, int img_w, int img_h, int ntiles, const int *__restrict__ ids,
    const int2 *__restrict__ bins, const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opac,
    const int *__restrict__ final_idx, const float *__restrict__ v_out,
    float *__restrict__ grad) {
    __shared__ float4 s_pix[kTilePix];  // v_out rgb, final_idx bits
    __shared__ float4 s_geo[kTilePix];  // x, y, a, b
    __shared__ float4 s_col[kTilePix];  // c, opacity, r, g
    __shared__ float s_blu[kTilePix];
    __shared__ int s_gid[kTilePix];
    __shared__ float s_red[9][kTilePix];
    __shared__ int s_max[4];
    const int tile = xcd_remap(blockIdx.x, ntiles);
    const int ty = tile / tbx, tx = tile - ty * tbx;
    const int tid = threadIdx.x;
    const int pi = ty * kTile + (tid >> 4), pj = tx * kTile + (tid & 15);
    const bool inside = pi < img_h && pj < img_w;
    float4 pd = make_float4(0.f, 0.f, 0.f, __int_as_float(-2147483647 - 1));
    if (inside) {
        const size_t p = (size_t)pi * (size_t)img_w + (size_t)pj;
        pd = make_float4(v_out[3 * p], v_out[3 * p + 1], v_out[3 * p + 2], __int_as_float(final_idx[p]));
    }
    s_pix[tid] = pd;
    int f = __float_as_int(pd.w);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) f = max(f, __shfl_xor(f, off, 64));
    if ((tid & 63) == 0) s_max[tid >> 6] = f;
    __syncthreads();
    const int maxf = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));
    const int2 range = bins[tile];
    const int kend = min(range.y, maxf == (-2147483647 - 1) ? maxf : maxf + 1);
    const float tx0 = (float)(tx * kTile), ty0 = (float)(ty * kTile);

    for (int cs = range.x; cs < kend; cs += kTilePix) {
        const int n = min(kTilePix, kend - cs);
        if (tid < n) {
            const int g = ids[cs + tid];
            s_gid[tid] = g;
            const float2 xy = xys[g];
            s_geo[tid] = make_float4(xy.x, xy.y, conics[3 * g], conics[3 * g + 1]);
            s_col[tid] = make_float4(conics[3 * g + 2], opac[g], colors[3 * g], colors[3 * g + 1]);
            s_blu[tid] = colors[3 * g + 2];
        }
        __syncthreads();
        const int lg = ceil_log2(n);
        const int E = 1 << lg;
        const int e = tid & (E - 1);
        const int p_begin = (tid >> lg) << lg;  // E pixels per group
        float a_r = 0.f, a_g = 0.f, a_b = 0.f, a_c0 = 0.f, a_c1 = 0.f, a_c2 = 0.f;
        float a_x = 0.f, a_y = 0.f, a_o = 0.f;
        if (e < n) {
            const int k = cs + e;
            const float4 G = s_geo[e];
            const float4 C = s_col[e];
            const float bl = s_blu[e];
            const float ha = 0.5f * G.z, hc = 0.5f * C.x;
            for (int pp = 0; pp < E; ++pp) {
                const int p = p_begin + pp;
                const float4 P = s_pix[p];
                if (k > __float_as_int(P.w)) continue;
                const float dx = G.x - (tx0 + (float)(p & 15));
                const float dy = G.y - (ty0 + (float)(p >> 4));
                const float s = splat_sigma_h(ha, G.w, hc, dx, dy);
                const float vis = exp_neg(s);
                const float al = fminf(1.0f, C.y * vis);
                if (s < 0.0f || al < kAlphaMin) continue;
                const float v_alpha = fmaf(bl, P.z, fmaf(C.w, P.y, C.z * P.x));
                const float v_sigma = (-C.y * vis) * v_alpha;
                a_r = fmaf(al, P.x, a_r);
                a_g = fmaf(al, P.y, a_g);
                a_b = fmaf(al, P.z, a_b);
                const float hs = 0.5f * v_sigma;
                const float hsdx = hs * dx;
                a_c0 = fmaf(hsdx, dx, a_c0);
                a_c1 = fmaf(hsdx, dy, a_c1);
                a_c2 = fmaf(hs * dy, dy, a_c2);
                a_x = fmaf(v_sigma, fmaf(G.z, dx, G.w * dy), a_x);
                a_y = fmaf(v_sigma, fmaf(G.w, dx, C.x * dy), a_y);
                a_o = fmaf(vis, v_alpha, a_o);
            }
        }
        // combine the 256/E pixel groups of each entry
        if (E < 64) {
            for (int off = 32; off >= E; off >>= 1) {
                a_r += __shfl_xor(a_r, off, 64);
                a_g += __shfl_xor(a_g, off, 64);
                a_b += __shfl_xor(a_b, off, 64);
                a_c0 += __shfl_xor(a_c0, off, 64);
                a_c1 += __shfl_xor(a_c1, off, 64);
                a_c2 += __shfl_xor(a_c2, off, 64);
                a_x += __shfl_xor(a_x, off, 64);
                a_y += __shfl_xor(a_y, off, 64);
                a_o += __shfl_xor(a_o, off, 64);
            }
        }
        const int S = E < 64 ? 64 : E;
        if (E >= 64 || (tid & 63) < E) {
            s_red[0][tid] = a_x;
            s_red[1][tid] = a_y;
            s_red[2][tid] = a_c0;
            s_red[3][tid] = a_c1;
            s_red[4][tid] = a_c2;
            s_red[5][tid] = a_r;
            s_red[6][tid] = a_g;
            s_red[7][tid] = a_b;
            s_red[8][tid] = a_o;
        }
        __syncthreads();
        if (tid < n) {
            const int reps = kTilePix / S;
#pragma unroll
            for (int c = 0; c < 9; ++c) {
                float v = s_red[c][tid];
                for (int j = 1; j < reps; ++j) v += s_red[c][tid + j * S];
                s_red[c][tid] = v;
            }
        }
        __syncthreads();
        // 16 lanes per entry, 9 of them add one float each into the splat's
        // 64-byte gradient record: one memory request per (splat, tile).
        for (int q = tid; q < n * 16; q += kTilePix) {
            const int e2 = q >> 4, c = q & 15;
            if (c < 9) unsafeAtomicAdd(grad + (size_t)s_gid[e2] * 16 + c, s_red[c][e2]);
        }
        __syncthreads();
    }
}

}  // namespace gsvc

using namespace gsvc;

static int check_tiles(const char *what, int bx, int by, int tbx, int tby, unsigned w, unsigned h) {
    if (bx != kTile || by != kTile)
        return set_error(GSVC_ERR_ARG, "%s: only 16x16 tiles are supported (got %dx%d)", what, bx, by);
    if (tbx != ceil_div((int)w, kTile) || tby != ceil_div((int)h, kTile))
        return set_error(GSVC_ERR_ARG, "%s: tile_bounds (%d,%d) do not match image %ux%u", what, tbx,
                         tby, w, h);
    return GSVC_OK;
}

extern "C" int gsvc_rasterize_sum_forward(int tbx, int tby, int tbz, int block_x, int block_y,
                                          int block_z, unsigned img_width, unsigned img_height,
                                          unsigned img_depth, const int *gaussian_ids_sorted,
                                          const int *tile_bins, const float *xys, const float *conics,
                                          const float *colors, const float *opacities,
                                          const float *background, float *out_img, float *final_Ts,
                                          int *final_idx, void *stream) {
    (void)tbz; (void)block_z; (void)img_depth; (void)background;
    int rc = check_tiles("rasterize_sum_forward", block_x, block_y, tbx, tby, img_width, img_height);
    if (rc) return rc;
    const int ntiles = tbx * tby;
    if (ntiles == 0) return GSVC_OK;
    const bool vec = (img_width % 4 == 0) && (((uintptr_t)out_img & 15) == 0) &&
                     (((uintptr_t)final_idx & 15) == 0) && (((uintptr_t)final_Ts & 15) == 0);
    hipLaunchKernelGGL(raster_sum_fwd_kernel, dim3(ntiles), dim3(64), 0, (hipStream_t)stream, tbx,
                       (int)img_width, (int)img_height, ntiles, vec, gaussian_ids_sorted,
                       (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacities,
                       out_img, final_idx, final_Ts);
    return check_launch("rasterize_sum_forward");
}

extern "C" int gsvc_rasterize_sum_backward(unsigned img_height, unsigned img_width, unsigned block_h,
                                           unsigned block_w, int num_points,
                                           const int *gaussian_ids_sorted, const int *tile_bins,
                                           const float *xys, const float *conics, const float *colors,
                                           const float *opacities, const float *background,
                                           const float *final_Ts, const int *final_idx,
                                           const float *v_output, const float *v_output_alpha,
                                           float *grad_records, void *stream) {
    (void)background; (void)final_Ts; (void)v_output_alpha;
    const int tbx = ceil_div((int)img_width, (int)block_w), tby = ceil_div((int)img_height, (int)block_h);
    int rc = check_tiles("rasterize_sum_backward", (int)block_w, (int)block_h, tbx, tby, img_width,
                         img_height);
    if (rc) return rc;
    if (num_points < 0) return set_error(GSVC_ERR_ARG, "rasterize_sum_backward: bad num_points");
    hipStream_t s = (hipStream_t)stream;
    if (num_points > 0 &&
        hipMemsetAsync(grad_records, 0, sizeof(float) * 16 * (size_t)num_points, s) != hipSuccess)
        return set_error(GSVC_ERR_HIP, "rasterize_sum_backward: memset failed");
    const int ntiles = tbx * tby;
    if (ntiles == 0 || num_points == 0) return GSVC_OK;
    hipLaunchKernelGGL(raster_sum_bwd_kernel, dim3(ntiles), dim3(256), 0, s, tbx, (int)img_width,
                       (int)img_height, ntiles, gaussian_ids_sorted, (const int2 *)tile_bins,
                       (const float2 *)xys, conics, colors, opacities, final_idx, v_output,
                       grad_records);
    return check_launch("rasterize_sum_backward");
}
