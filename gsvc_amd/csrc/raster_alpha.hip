// Front-to-back alpha-compositing rasterizer (rasterize_gaussians), gfx950.
//
// Reference: gsplat/gsplat/cuda/csrc/forward.cu:252-374 (rasterize_forward),
// backward.cu:138-315 (rasterize_backward_kernel), bindings.cu:332-398,631-704;
// Python glue rasterize.py:89-253.  Not used by GSVC's scripts, but named by
// the north star; it shares the binning and the LDS-staged tile layout of the
// sum path.
//
// Semantics kept: alpha = min(0.999, o exp(-sigma)) in the forward and
// min(0.99, ...) in the backward (forward.cu:339 vs backward.cu:244); a pixel
// stops at the entry whose next_T <= 1e-4 (that entry is not blended); every
// entry of the tile is visited (no 256 cap); out = acc + T * background.
//
// Forward: one wave64 per tile, 4 pixels per lane (as the sum forward), the
// wave leaves the tile when every lane's 4 pixels are done; chunks of more
// than 24 entries are walked through lane-group lists (cull.h).
// Backward: the transmittance recursion runs per pixel from the back, so it
// is pixel-parallel: one wave per tile, 4 pixels per lane, per entry the
// pixels' terms reduced as row sums by DPP into one lane (see the kernel).
#include "common.h"
#include "cull.h"
#include "rows.h"

namespace gsvc {

constexpr int kAChunk = 64;
// A chunk of more than this many entries is walked through lane-group lists
// (as the sum composite's sparse path, raster_sum.hip): each group of 4 lanes
// owns a 4x4-pixel block and visits, in order, only the entries whose
// alpha >= 1/255 ellipse box reaches it (cull.h ellipse_blocks); fewer entries
// are walked by every lane (the lists would cost more than they skip).
constexpr int kAGroupMin = 24;

// One entry against a lane's 4 pixels: forward.cu:323-357 (front to back,
// alpha clamped at 0.999, stop at next_T <= 1e-4 without blending that entry).
__device__ __forceinline__ void alpha_blend4(float4 G, float4 C, float blu, float py, int pj, int k,
                                             float (&T)[4], float (&ar)[4], float (&ag)[4],
                                             float (&ab)[4], int (&last)[4], bool (&done)[4]) {
    const float dy = G.y - py;
    const float cq = (C.x * dy) * dy;
    const float bdy = G.w * dy;
    // every pixel evaluated and the updates selected (no per-pixel branches: a
    // lane's skipped pixel cost its wave the same slots anyway, and the
    // branches' joins moved the accumulators between registers each trip --
    // 18 v_mov of 57 VALU); a done or failing pixel keeps its state bit for bit
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float dx = G.x - (float)(pj + q);
        const float s = fmaf(fmaf(G.z, dx, bdy), dx, cq);
        const float al = fminf(0.999f, C.y * exp_neg(s));
        const bool act = !done[q] && !(s < 0.0f) && !(al < kAlphaMin);
        const float next_T = T[q] * (1.0f - al);
        const bool stop = next_T <= 1e-4f;
        const bool upd = act && !stop;
        done[q] = done[q] || (act && stop);
        const float vis = al * T[q];
        ar[q] = upd ? fmaf(C.z, vis, ar[q]) : ar[q];
        ag[q] = upd ? fmaf(C.w, vis, ag[q]) : ag[q];
        ab[q] = upd ? fmaf(blu, vis, ab[q]) : ab[q];
        T[q] = upd ? next_T : T[q];
        last[q] = upd ? k : last[q];
    }
}

__global__ __launch_bounds__(64) void raster_alpha_fwd_kernel(
    int tbx, int img_w, int img_h, int ntiles, const int *__restrict__ ids,
    const int2 *__restrict__ bins, const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opac, const float *__restrict__ bg,
    float *__restrict__ out, float *__restrict__ final_Ts, int *__restrict__ final_idx,
    int group_min) {
    // staged entries (slot kAChunk: the lists' no-op sentinel, sigma = +inf),
    // their 4x4 blocks and the 16 groups' lists [iteration][group]
    __shared__ float4 s_geo[kAChunk + 1];  // x, y, 0.5a, b
    __shared__ float4 s_col[kAChunk + 1];  // 0.5c, opacity, r, g
    __shared__ float s_blu[kAChunk + 1];
    __shared__ unsigned short s_gm[kAChunk];
    __shared__ uint4 s_list4[kAChunk];     // 16 bytes per iteration
    unsigned char *s_list = reinterpret_cast<unsigned char *>(s_list4);
    const int tile = xcd_remap(blockIdx.x, ntiles);
    const int ty = tile / tbx, tx = tile - ty * tbx;
    const int lane = threadIdx.x;
    const int pi = ty * kTile + (lane >> 2);
    const int pj = tx * kTile + ((lane & 3) << 2);
    const float py = (float)pi;
    const float ox = (float)(tx * kTile), oy = (float)(ty * kTile);
    const int2 range = bins[tile];
    const int n = max(range.y - range.x, 0);
    if (lane == 0) {
        s_geo[kAChunk] = make_float4(0.0f, 1e30f, 0.0f, 0.0f);
        s_col[kAChunk] = make_float4(1e30f, 1.0f, 0.0f, 0.0f);
        s_blu[kAChunk] = 0.0f;
    }

    float T[4] = {1.f, 1.f, 1.f, 1.f};
    float ar[4] = {0.f, 0.f, 0.f, 0.f}, ag[4] = {0.f, 0.f, 0.f, 0.f}, ab[4] = {0.f, 0.f, 0.f, 0.f};
    int last[4] = {0, 0, 0, 0};
    bool done[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) done[q] = !(pi < img_h && pj + q < img_w);

    for (int base = 0; base < n; base += kAChunk) {
        if (__all(done[0] && done[1] && done[2] && done[3])) break;
        const int cnt = min(kAChunk, n - base);
        const bool grouped = cnt > group_min;
        if (lane < cnt) {
            const int g = ids[range.x + base + lane];
            const float2 xy = xys[g];
            const float a = conics[3 * g], b = conics[3 * g + 1], c = conics[3 * g + 2];
            const float o = opac[g];
            s_geo[lane] = make_float4(xy.x, xy.y, 0.5f * a, b);
            s_col[lane] = make_float4(0.5f * c, o, colors[3 * g], colors[3 * g + 1]);
            s_blu[lane] = colors[3 * g + 2];
            if (grouped) s_gm[lane] = (unsigned short)ellipse_blocks<16>(xy.x, xy.y, a, b, c, o, ox, oy);
        }
        __syncthreads();
        const int k0 = range.x + base;
        if (!grouped) {
            for (int t = 0; t < cnt; ++t)
                alpha_blend4(s_geo[t], s_col[t], s_blu[t], py, pj, k0 + t, T, ar, ag, ab, last, done);
            __syncthreads();
            continue;
        }
        // lists: row `it` of the 16 groups' lists, padded with the sentinel
        const unsigned gmt = lane < cnt ? s_gm[lane] : 0u;
        const unsigned long long lt = (1ull << lane) - 1ull;
        s_list4[lane] = make_uint4(0x40404040u, 0x40404040u, 0x40404040u, 0x40404040u);
        __syncthreads();
        int maxlen = 0;
#pragma unroll 1
        for (int gr = 0; gr < 16; ++gr) {
            const bool in = (gmt >> gr) & 1u;
            const unsigned long long mg = __ballot(in);
            if (in) s_list[16 * __popcll(mg & lt) + gr] = (unsigned char)lane;
            maxlen = max(maxlen, __popcll(mg));
        }
        __syncthreads();
        const unsigned char *ml = s_list + (((lane >> 4) << 2) | (lane & 3));
        for (int it = 0; it < maxlen; ++it) {
            const int t = ml[16 * it];
            alpha_blend4(s_geo[t], s_col[t], s_blu[t], py, pj, k0 + t, T, ar, ag, ab, last, done);
        }
        __syncthreads();
    }
    if (pi >= img_h) return;
    const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (pj + q < img_w) {
            const size_t p = (size_t)pi * (size_t)img_w + (size_t)(pj + q);
            out[3 * p] = fmaf(T[q], bg0, ar[q]);
            out[3 * p + 1] = fmaf(T[q], bg1, ag[q]);
            out[3 * p + 2] = fmaf(T[q], bg2, ab[q]);
            final_Ts[p] = T[q];
            final_idx[p] = last[q];
        }
    }
}

// Sum over each 16-lane row, left in every lane of the row: four DPP adds
// (quad swaps, half-row and row mirrors), no LDS permutes.
template <int kCtrl>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), kCtrl, 0xf, 0xf, false));
}
__device__ __forceinline__ float row_sum16(float v) {
    v = dpp_add<0xb1>(v);   // quad_perm [1, 0, 3, 2]
    v = dpp_add<0x4e>(v);   // quad_perm [2, 3, 0, 1]
    v = dpp_add<0x141>(v);  // row_half_mirror
    return dpp_add<0x140>(v);  // row_mirror
}
__device__ __forceinline__ float quad_sum(float v) { return dpp_add<0x4e>(dpp_add<0xb1>(v)); }
// every 16-lane row holding its total in each lane: lane 63 ends with the sum
// of the four rows (row_bcast:15 into rows 1 and 3, row_bcast:31 into 2 and 3)
__device__ __forceinline__ float rows_to_last(float v) {
    v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xa, 0xf, false));
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xc, 0xf, false));
}

// Backward (backward.cu:138-315), round 5: ONE wave per tile, 4 pixels of one
// row per lane (the forward's layout), each pixel's back-to-front recursion
// (T = T_final rolled back through every valid entry's 1 / (1 - alpha), the
// colour buffer, v_alpha) kept in the lane.  Per entry the lane sums its 4
// pixels' terms as 7 row sums -- S_k = sum v_sigma dx^k (k = 0, 1, 2: v_xy and
// v_conic factor by the row's constant dy), alpha T v_out (3), vis v_alpha --
// the 4 lanes of a tile row (a DPP quad) add them, the row's 9 gradient terms
// are formed, and the 16 rows are added by DPP (half-row / row mirrors, row
// broadcasts) into lane 63, which keeps the entry's 9 sums in LDS; once per
// 64-entry chunk they go to the splat's record, one 64-byte atomic request per
// (splat, tile).  An entry no pixel of the tile takes costs no sums.
// Round 4's kernel (256 threads = 256 pixels, per entry and wave 9 DPP row
// sums and LDS float atomics: 111 us at 1080p / 50k) stays in the diagnostic
// library as raster_alpha_bwd_kernel_r4 (A/B knob 9 = 1).
// kAbl (diagnostic library, A/B knob 30, wrong results): bit 0 no per-entry
// sums, bit 1 no pixel work
template <int kAbl = 0>
__global__ __launch_bounds__(64, 5) void raster_alpha_bwd_kernel(
    int tbx, int img_w, int img_h, int ntiles, const int *__restrict__ ids,
    const int2 *__restrict__ bins, const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opac, const float *__restrict__ bg,
    const float *__restrict__ final_Ts, const int *__restrict__ final_idx,
    const float *__restrict__ v_out, const float *__restrict__ v_out_alpha,
    float *__restrict__ grad) {
    __shared__ float4 s_geo[kAChunk];  // x, y, a, b
    __shared__ float4 s_col[kAChunk];  // c, opacity, r, g
    __shared__ float s_blu[kAChunk];
    __shared__ int s_gid[kAChunk];
    __shared__ unsigned short s_ro[kAChunk];
    __shared__ float s_row[8][kTile][8];  // a group's 8 entries: per tile row its 7 sums
    __shared__ float s_acc[9][8];         // the group's entry sums
    const int tile = xcd_remap(blockIdx.x, ntiles);
    const int ty = tile / tbx, tx = tile - ty * tbx;
    const int lane = threadIdx.x;
    const int pi = ty * kTile + (lane >> 2);
    const int pj = tx * kTile + ((lane & 3) << 2);
    const float py = (float)pi;
    const float ox = (float)(tx * kTile), oy = (float)(ty * kTile);
    const unsigned lrow = (unsigned)(lane >> 2), lc0 = (unsigned)((lane & 3) << 2);
    // per pixel: T (rolled back), v_out, BV = buffer . v_out (the colour
    // buffer only ever enters v_alpha through this dot product, so the buffer
    // is kept as it: BV += fac (c . v_out)), TK = T_final (v_out_alpha - bg .
    // v_out) -- backward.cu:248-266's v_alpha regrouped as
    // T (c . v_out) + (TK - BV) / (1 - alpha)
    const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];
    float T[4], BV[4], TK[4];
    float3 vo3[4];
    int bf[4];
    int fmax = -2147483647 - 1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const bool in = pi < img_h && pj + q < img_w;
        const size_t p = in ? (size_t)pi * (size_t)img_w + (size_t)(pj + q) : 0;
        const float tf = in ? final_Ts[p] : 1.0f;
        bf[q] = in ? final_idx[p] : (-2147483647 - 1);  // outside the image: never valid
        const float3 v = in ? make_float3(v_out[3 * p], v_out[3 * p + 1], v_out[3 * p + 2])
                            : make_float3(0.f, 0.f, 0.f);
        const float va = in ? v_out_alpha[p] : 0.f;
        vo3[q] = v;
        T[q] = tf;
        BV[q] = 0.f;
        TK[q] = tf * (va - fmaf(bg2, v.z, fmaf(bg1, v.y, bg0 * v.x)));
        fmax = max(fmax, bf[q]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) fmax = max(fmax, __shfl_xor(fmax, off, 64));
    const int2 range = bins[tile];
    // entries past every pixel's final index are never valid (backward.cu:226-230)
    const int kend = min(range.y, fmax == (-2147483647 - 1) ? fmax : fmax + 1);

    // chunks of <= 64 entries, back to front; within a chunk, groups of 8
    for (int ce = kend; ce > range.x; ce -= kAChunk) {
        const int cs = max(range.x, ce - kAChunk);
        const int n = ce - cs;
        if (lane < n) {
            const int g = ids[cs + lane];
            s_gid[lane] = g;
            const float2 xy = xys[g];
            s_geo[lane] = make_float4(xy.x, xy.y, conics[3 * g], conics[3 * g + 1]);
            s_col[lane] = make_float4(conics[3 * g + 2], opac[g], colors[3 * g], colors[3 * g + 1]);
            s_blu[lane] = colors[3 * g + 2];
            // the pixels where alpha >= 1/255 is reachable (a pair outside
            // is never valid in the reference either)
            s_ro[lane] = (unsigned short)ellipse_rect(xy.x, xy.y, conics[3 * g], conics[3 * g + 1],
                                                      conics[3 * g + 2], opac[g], ox, oy);
        }
        __syncthreads();
        for (int g0 = ((n - 1) >> 3) << 3; g0 >= 0; g0 -= 8) {
            const int g1 = min(g0 + 8, n);  // this group: entries [g0, g1), walked back to front
            for (int t = g1 - 1; t >= g0; --t) {
                const unsigned rc = s_ro[t];
                // the lane's 4 pixels against the rectangle: none -> no pixel work
                const bool lin = rc != kNoRect && lrow >= ((rc >> 8) & 15u) &&
                                 lrow <= ((rc >> 12) & 15u) && lc0 + 3u >= (rc & 15u) &&
                                 lc0 <= ((rc >> 4) & 15u);
                const int k = lin ? cs + t : 0x7fffffff;
                const float4 G = s_geo[t], C = s_col[t];
                const float blu = s_blu[t];
                const float dy = G.y - py;
                const float ha = 0.5f * G.z, hc = 0.5f * C.x;
                float sr = 0.f, sg = 0.f, sb = 0.f, s0 = 0.f, s1 = 0.f, s2 = 0.f, so = 0.f;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (kAbl & 2) continue;
                    if (k > bf[q]) continue;
                    const float dx = G.x - (float)(pj + q);
                    const float sgm = splat_sigma_h(ha, G.w, hc, dx, dy);
                    const float vis = exp_neg(sgm);
                    const float al = fminf(0.99f, C.y * vis);
                    if (sgm < 0.0f || al < kAlphaMin) continue;
                    // the reference's 1.f / (1.f - alpha) under --use_fast_math is the
                    // hardware reciprocal (rcp.approx), as here (v_rcp_f32, ~1 ulp)
                    const float ra = __builtin_amdgcn_rcpf(1.0f - al);
                    const float3 vo = vo3[q];
                    T[q] = T[q] * ra;
                    const float fac = al * T[q];
                    const float cvo = fmaf(blu, vo.z, fmaf(C.w, vo.y, C.z * vo.x));  // c . v_out
                    const float v_alpha = fmaf(T[q], cvo, ra * (TK[q] - BV[q]));
                    BV[q] = fmaf(fac, cvo, BV[q]);
                    const float v_sigma = (-C.y * vis) * v_alpha;
                    sr = fmaf(fac, vo.x, sr);
                    sg = fmaf(fac, vo.y, sg);
                    sb = fmaf(fac, vo.z, sb);
                    s0 += v_sigma;
                    const float vdx = v_sigma * dx;
                    s1 += vdx;
                    s2 = fmaf(vdx, dx, s2);
                    so = fmaf(vis, v_alpha, so);
                }
                if (kAbl & 1) continue;
                // a quad is one tile row: its 7 sums into the row's slot
                s0 = quad_sum(s0);
                s1 = quad_sum(s1);
                s2 = quad_sum(s2);
                sr = quad_sum(sr);
                sg = quad_sum(sg);
                sb = quad_sum(sb);
                so = quad_sum(so);
                if ((lane & 3) == 0) {
                    float *r = &s_row[t & 7][lrow][0];
                    *reinterpret_cast<float4 *>(r) = make_float4(s0, s1, s2, so);
                    *reinterpret_cast<float4 *>(r + 4) = make_float4(sr, sg, sb, 0.f);
                }
            }
            __syncthreads();
            // the group's sums over the tile's 16 rows: lane = (entry te, rows
            // 2 rr, 2 rr + 1); the row's 9 terms (dy constant along it), then
            // the entry's 8 lanes by DPP into lane 8 te
            {
                const int te = lane >> 3, rr = (lane & 7) << 1;
                const int t = g0 + te;
                float gs[9];
#pragma unroll
                for (int c = 0; c < 9; ++c) gs[c] = 0.f;
                if (t < g1) {
                    const float4 G = s_geo[t], C = s_col[t];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const float *r = &s_row[t & 7][rr + h][0];
                        const float4 a = *reinterpret_cast<const float4 *>(r);
                        const float4 b = *reinterpret_cast<const float4 *>(r + 4);
                        const float dy = G.y - (oy + (float)(rr + h));
                        gs[0] += fmaf(G.z, a.y, (G.w * dy) * a.x);  // v_xy.x: sum v_sigma (a dx + b dy)
                        gs[1] += fmaf(G.w, a.y, (C.x * dy) * a.x);  // v_xy.y: sum v_sigma (b dx + c dy)
                        gs[2] += 0.5f * a.z;                       // v_conic: 1/2 sum v_sigma (dx^2, dx dy, dy^2)
                        gs[3] += (0.5f * dy) * a.y;
                        gs[4] += ((0.5f * dy) * dy) * a.x;
                        gs[5] += b.x;
                        gs[6] += b.y;
                        gs[7] += b.z;
                        gs[8] += a.w;
                    }
                }
#pragma unroll
                for (int c = 0; c < 9; ++c) gs[c] = dpp_add<0x141>(quad_sum(gs[c]));  // 8 lanes
                if ((lane & 7) == 0 && t < g1) {
#pragma unroll
                    for (int c = 0; c < 9; ++c) s_acc[c][te] = gs[c];
                }
            }
            __syncthreads();
            // 16 lanes per entry, 9 of them add one sum each into the splat's
            // 64-byte record: one memory request per (splat, tile)
            for (int q = lane; q < (g1 - g0) * 16; q += 64) {
                const int e = q >> 4, c = q & 15;
                if (c < 9) unsafeAtomicAdd(grad + (size_t)s_gid[g0 + e] * 16 + c, s_acc[c][e]);
            }
            __syncthreads();
        }
    }
}

#ifdef GSVC_DIAG
// Round 4's backward (diagnostic library, A/B knob 9 = 1): pixel-parallel, 256
// threads = 256 pixels; per entry each wave sums its 9 partial gradients per
// 16-lane row with DPP adds, the rows' last lanes add them to an LDS record
// with LDS float atomics, and once per 256-entry chunk the tile's records go
// to HBM as one 64-byte atomic request per (splat, tile).
__global__ __launch_bounds__(256) void raster_alpha_bwd_kernel_r4(
    int tbx, int img_w, int img_h, int ntiles, const int *__restrict__ ids,
    const int2 *__restrict__ bins, const float2 *__restrict__ xys, const float *__restrict__ conics,
    const float *__restrict__ colors, const float *__restrict__ opac, const float *__restrict__ bg,
    const float *__restrict__ final_Ts, const int *__restrict__ final_idx,
    const float *__restrict__ v_out, const float *__restrict__ v_out_alpha,
    float *__restrict__ grad) {
    __shared__ float4 s_geo[kTilePix];  // x, y, a, b
    __shared__ float4 s_col[kTilePix];  // c, opacity, r, g
    __shared__ float s_blu[kTilePix];
    __shared__ int s_gid[kTilePix];
    __shared__ float s_acc[kTilePix][9];
    __shared__ int s_max[4];
    const int tile = xcd_remap(blockIdx.x, ntiles);
    const int ty = tile / tbx, tx = tile - ty * tbx;
    const int tid = threadIdx.x, lane = tid & 63;
    const int pi = ty * kTile + (tid >> 4), pj = tx * kTile + (tid & 15);
    const bool inside = pi < img_h && pj < img_w;
    const float px = (float)pj, py = (float)pi;
    // backward.cu:160: out-of-image threads clamp to the last pixel; they are
    // never valid, so only their loads matter.
    const size_t p = inside ? (size_t)pi * (size_t)img_w + (size_t)pj : 0;
    const float T_final = inside ? final_Ts[p] : 1.0f;
    float T = T_final;
    float buf0 = 0.f, buf1 = 0.f, buf2 = 0.f;
    const int bin_final = inside ? final_idx[p] : (-2147483647 - 1);
    const float vo0 = inside ? v_out[3 * p] : 0.f, vo1 = inside ? v_out[3 * p + 1] : 0.f;
    const float vo2 = inside ? v_out[3 * p + 2] : 0.f;
    const float voa = inside ? v_out_alpha[p] : 0.f;
    const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];
    int f = bin_final;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) f = max(f, __shfl_xor(f, off, 64));
    if (lane == 0) s_max[tid >> 6] = f;
    __syncthreads();
    const int maxf = max(max(s_max[0], s_max[1]), max(s_max[2], s_max[3]));
    const int2 range = bins[tile];
    const int kend = min(range.y, maxf == (-2147483647 - 1) ? maxf : maxf + 1);

    // chunks of <= 256 entries, back to front
    for (int ce = kend; ce > range.x; ce -= kTilePix) {
        const int cs = max(range.x, ce - kTilePix);
        const int n = ce - cs;
        if (tid < n) {
            const int g = ids[cs + tid];
            s_gid[tid] = g;
            const float2 xy = xys[g];
            s_geo[tid] = make_float4(xy.x, xy.y, conics[3 * g], conics[3 * g + 1]);
            s_col[tid] = make_float4(conics[3 * g + 2], opac[g], colors[3 * g], colors[3 * g + 1]);
            s_blu[tid] = colors[3 * g + 2];
#pragma unroll
            for (int c = 0; c < 9; ++c) s_acc[tid][c] = 0.f;
        }
        __syncthreads();
        for (int t = n - 1; t >= 0; --t) {
            const int k = cs + t;
            bool valid = inside && k <= bin_final;
            float4 G, C;
            float dx = 0.f, dy = 0.f, vis = 0.f, al = 0.f;
            if (valid) {
                G = s_geo[t];
                C = s_col[t];
                dx = G.x - px;
                dy = G.y - py;
                const float s = splat_sigma_h(0.5f * G.z, G.w, 0.5f * C.x, dx, dy);
                vis = exp_neg(s);
                al = fminf(0.99f, C.y * vis);
                if (s < 0.0f || al < kAlphaMin) valid = false;
            }
            if (!__any(valid)) continue;
            float g_r = 0.f, g_g = 0.f, g_b = 0.f, g_c0 = 0.f, g_c1 = 0.f, g_c2 = 0.f;
            float g_x = 0.f, g_y = 0.f, g_o = 0.f;
            if (valid) {
                const float ra = 1.0f / (1.0f - al);
                T = T * ra;
                const float fac = al * T;
                const float r = C.z, gg = C.w, bb = s_blu[t];
                const float tfra = T_final * ra;
                float v_alpha = (r * T - buf0 * ra) * vo0;
                v_alpha = fmaf(gg * T - buf1 * ra, vo1, v_alpha);
                v_alpha = fmaf(bb * T - buf2 * ra, vo2, v_alpha);
                v_alpha = fmaf(tfra, voa, v_alpha);
                v_alpha = fmaf(-tfra * bg0, vo0, v_alpha);
                v_alpha = fmaf(-tfra * bg1, vo1, v_alpha);
                v_alpha = fmaf(-tfra * bg2, vo2, v_alpha);
                buf0 = fmaf(r, fac, buf0);
                buf1 = fmaf(gg, fac, buf1);
                buf2 = fmaf(bb, fac, buf2);
                const float v_sigma = (-C.y * vis) * v_alpha;
                g_r = fac * vo0;
                g_g = fac * vo1;
                g_b = fac * vo2;
                const float hs = 0.5f * v_sigma;
                g_c0 = (hs * dx) * dx;
                g_c1 = (hs * dx) * dy;
                g_c2 = (hs * dy) * dy;
                g_x = v_sigma * fmaf(G.z, dx, G.w * dy);
                g_y = v_sigma * fmaf(G.w, dx, C.x * dy);
                g_o = vis * v_alpha;
            }
            // the entry's sums over the wave: per 16-lane row by DPP, then the
            // last lane of each row adds its row's sums into the entry's LDS
            // accumulator (the row order of these adds is not fixed: float
            // atomics, as the reference's warp sums + atomicAdd)
            {
                const float gs[9] = {row_sum16(g_x), row_sum16(g_y), row_sum16(g_c0),
                                     row_sum16(g_c1), row_sum16(g_c2), row_sum16(g_r),
                                     row_sum16(g_g), row_sum16(g_b), row_sum16(g_o)};
                if ((lane & 15) == 15) {
#pragma unroll
                    for (int c = 0; c < 9; ++c) atomicAdd(&s_acc[t][c], gs[c]);
                }
            }
        }
        __syncthreads();
        for (int q = tid; q < n * 16; q += kTilePix) {
            const int e2 = q >> 4, c = q & 15;
            if (c < 9) unsafeAtomicAdd(grad + (size_t)s_gid[e2] * 16 + c, s_acc[e2][c]);
        }
        __syncthreads();
    }
}

#endif

}  // namespace gsvc

using namespace gsvc;

extern "C" int gsvc_rasterize_forward(int tbx, int tby, int tbz, int block_x, int block_y,
                                      int block_z, unsigned img_width, unsigned img_height,
                                      unsigned img_depth, const int *gaussian_ids_sorted,
                                      const int *tile_bins, const float *xys, const float *conics,
                                      const float *colors, const float *opacities,
                                      const float *background, float *out_img, float *final_Ts,
                                      int *final_idx, void *stream) {
    (void)tbz; (void)block_z; (void)img_depth;
    if (block_x != kTile || block_y != kTile)
        return set_error(GSVC_ERR_ARG, "rasterize_forward: only 16x16 tiles are supported");
    if (tbx != ceil_div((int)img_width, kTile) || tby != ceil_div((int)img_height, kTile))
        return set_error(GSVC_ERR_ARG, "rasterize_forward: tile_bounds do not match the image");
    const int ntiles = tbx * tby;
    if (ntiles == 0) return GSVC_OK;
    hipStream_t s = (hipStream_t)stream;
    hipEvent_t tev[2];
    const int tslot = timing_begin(s, tev, kTimingAlphaFwd);
    launch_timed(raster_alpha_fwd_kernel, dim3(ntiles), dim3(64), 0, s, tev, tbx, (int)img_width,
                 (int)img_height, ntiles, gaussian_ids_sorted, (const int2 *)tile_bins,
                 (const float2 *)xys, conics, colors, opacities, background, out_img, final_Ts,
                 final_idx,
                 // A/B knob 18 = v > 0: list threshold v - 1
                 knob(18) > 0 ? knob(18) - 1 : kAGroupMin);
    timing_end(s, tslot, kTimingAlphaFwd);
    return check_launch("rasterize_forward");
}

extern "C" int gsvc_rasterize_backward(unsigned img_height, unsigned img_width, unsigned block_h,
                                       unsigned block_w, int num_points,
                                       const int *gaussian_ids_sorted, const int *tile_bins,
                                       const float *xys, const float *conics, const float *colors,
                                       const float *opacities, const float *background,
                                       const float *final_Ts, const int *final_idx,
                                       const float *v_output, const float *v_output_alpha,
                                       float *grad_records, void *stream) {
    if (block_h != (unsigned)kTile || block_w != (unsigned)kTile)
        return set_error(GSVC_ERR_ARG, "rasterize_backward: only 16x16 tiles are supported");
    if (num_points < 0) return set_error(GSVC_ERR_ARG, "rasterize_backward: bad num_points");
    hipStream_t s = (hipStream_t)stream;
    if (num_points > 0 &&
        dev_zero(grad_records, sizeof(float) * 16 * (size_t)num_points, s) != GSVC_OK)
        return set_error(GSVC_ERR_HIP, "rasterize_backward: memset failed");
    const int tbx = ceil_div((int)img_width, kTile), tby = ceil_div((int)img_height, kTile);
    const int ntiles = tbx * tby;
    if (ntiles == 0 || num_points == 0) return GSVC_OK;
    hipEvent_t tev[2];
    const int tslot = timing_begin(s, tev, kTimingAlphaBwd);
#ifdef GSVC_DIAG
    if (knob(9) == 1) {  // A/B: round 4's 256-thread kernel
        launch_timed(raster_alpha_bwd_kernel_r4, dim3(ntiles), dim3(256), 0, s, tev, tbx,
                     (int)img_width, (int)img_height, ntiles, gaussian_ids_sorted,
                     (const int2 *)tile_bins, (const float2 *)xys, conics, colors, opacities,
                     background, final_Ts, final_idx, v_output, v_output_alpha, grad_records);
        timing_end(s, tslot, kTimingAlphaBwd);
        return check_launch("rasterize_backward");
    }
#endif
    auto bwd = raster_alpha_bwd_kernel<0>;
    if constexpr (kDiag) {
        if (knob(30) == 1) bwd = raster_alpha_bwd_kernel<1>;
        if (knob(30) == 2) bwd = raster_alpha_bwd_kernel<2>;
    }
    launch_timed(bwd, dim3(ntiles), dim3(64), 0, s, tev, tbx, (int)img_width,
                 (int)img_height, ntiles, gaussian_ids_sorted, (const int2 *)tile_bins,
                 (const float2 *)xys, conics, colors, opacities, background, final_Ts, final_idx,
                 v_output, v_output_alpha, grad_records);
    timing_end(s, tslot, kTimingAlphaBwd);
    return check_launch("rasterize_backward");
}
