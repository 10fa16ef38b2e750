// Fused training step of GSVC's per-frame model (gfx950): one
// GaussianVideo_frame.train_iter with the L2 (or L1) loss and Adan, in three
// kernels and one C call, with no host synchronisation.
//
// Reference: GaussianSplats_Represent.py:191-207 (train_iter): the forward
// :83-90 (activations :57-70, project_gaussians_2d, rasterize_gaussians_sum,
// clamp, NCHW), loss_fn (utils.py:21-28: F.mse_loss / F.l1_loss),
// loss.backward() through the clamp, the sum rasterizer (backward.cu:696-862),
// the 2D projection (backward2d.cu:8-51) and the activations, the MSE behind
// the PSNR (:196-198), and Adan.step (optimizer.py:124-235, 296-362).
//
//   frame_project_kernel (frame.hip)  activations + projection + per-tile
//       256-slot record slabs, exactly as the frame render; also zeroes the
//       splat's 64-byte gradient record;
//   train_tile_kernel  one 256-thread workgroup per 16x16 tile: the tile's
//       first <= 256 entries in splat-id order into LDS (ranks by compare;
//       a slab that overflowed is rebuilt from the splats' bboxes in id
//       order); a pixel-parallel forward with the rasterizer's op sequence
//       (the same image bits as the render), the clamp, the loss gradient
//       against gt and the tile's error sums; then an entry-parallel backward
//       of the tile into the splats' gradient records (one atomic request per
//       (splat, tile)).  Image, final_idx and v_out never reach HBM: per pixel
//       the step reads gt once;
//   train_splat_kernel  one lane per splat: projection VJP (the reference's
//       doubled L cross term), activation VJPs and the Adan update of every
//       parameter element; an extra first workgroup sums the tiles' errors in
//       a fixed order into the loss.
#include <type_traits>

#include "adan.h"
#include "binning.h"
#include "cull.h"
#include "frame.h"
#include "frame_dev.h"
#include "det.h"
#include "rows.h"
#include "tile_ids.h"

namespace gsvc {

constexpr int kT = kTilePix;  // threads = pixels = entries of one tile

struct TrainTileArgs {
    int tbx, img_w, img_h, ntiles, num_points, loss_l1;
    float norm;  // d loss / d pixel scale: float(2 / numel) for L2, 1.0f / numel for L1
    float4 *slab;  // read; a dense tile parks its sorted ids in its own slab
    const int *ovf;  // the slab's slots 256 .. kCarryCap - 1 as ids (frame.h FrameWs.ovf)
    const unsigned *counts;
    unsigned *counts_clear;
    const int *m_dev;
    const float2 *xys;
    const int *radii;
    const float4 *rec;
    const float *bg;
    const float *gt;  // [3, H, W]
    float *grad;      // [N, 16]: v_xy 0:2, v_conic 2:5, v_colors 5:8, v_opacity 8
    float2 *err;      // [ntiles]: sum of squared, sum of absolute errors
    int brun;         // band kernel: a rectangle row wider than this is two work items
    int spec;         // band kernel: slab records loaded with the count
    int grouped;      // band kernel forward: lane-group entry lists (A/B knob 14 = 1: off)
    int diag;         // diagnostic knob 13 (timing experiments only; wrong results):
                      // bits 2 no backward, 4 no forward
                      // blending, 8 no backward pixel work, 16 no run sums, 32 no atomics;
                      // 64 (A/B, exact): items in entry order, not longest first;
                      // 128 (A/B, exact): the carried candidates ranked by a
                      // readlane loop instead of LDS broadcast reads; 256 no v_out
                      // reads (wrong)
    float *out;       // optional [3, H, W] clamped render
    long long *stamps;  // diagnostic: int64[ntiles][8]
    // GSVC_TRAIN_DETERMINISTIC (band kernel): the (splat, tile) sums go to
    // det_part[det_off[g] + k] (k = the tile's row-major index in the splat's
    // tile bbox, 8 floats) instead of atomics; slots past det_cap fall back to
    // the atomics
    const int *det_off;
    float4 *det_part;
    long long det_cap;
    int prio;  // raise the wave priority over the order phase (s_setprio; knob 16 = 1 off)
    int xcd_off;  // diagnostic A/B (knob 37): 1 dispatch order, 4 xcd_remap ranges
    // GSVC_TRAIN_CARRY (band kernel): the tile's candidates are the splat ids
    // cids[tile][0, counts[tile]) -- a superset of its entries carried from
    // step to step (train_splat_kernel) -- and an entry is a candidate whose
    // current tile box cbox[id] holds the tile; records come from rec by id.
    // m_clear: the next frame's M slot (zeroed here; the splat kernel fills it)
    // csorted[tile]: how many leading cids are in id order (a rebuild zeroes it,
    // the splat kernel's appends leave it behind the count); a tile of <= 64
    // whose cids are all sorted ranks its entries by one ballot, and one that
    // is not sorts them, writes them back and sets it
    int *cids;
    const uint2 *cbox;
    int *m_clear;
    unsigned *csorted;
};

__device__ __forceinline__ float clamp_unit(float x) {
    // torch.clamp(x, 0, 1): NaN stays NaN
    return x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x);
}

// The first <= 256 ids (ascending) of the splats whose bbox covers tile
// (tx, ty) -- the slab insertion's own test -- for a tile whose slab kept an
// arbitrary 256 of more entries: 256 candidates per round, compacted by ballot.
__device__ int block_brute_ids(const TrainTileArgs &A, int tx, int ty, int *s_gid, int *s_cnt) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int tby = (A.img_h + kTile - 1) / kTile;
    const unsigned long long lt = (1ull << lane) - 1ull;
    int written = 0;
    for (int base = 0; base < A.num_points && written < kT; base += kT) {
        const int j = base + tid;
        bool hit = false;
        if (j < A.num_points) {
            const int r = A.radii[j];
            if (r > 0) {
                const float2 c = A.xys[j];
                unsigned x0, y0, x1, y1;
                tile_bbox(c.x, c.y, (float)r, A.tbx, tby, x0, y0, x1, y1);
                hit = (unsigned)tx >= x0 && (unsigned)tx < x1 && (unsigned)ty >= y0 &&
                      (unsigned)ty < y1;
            }
        }
        const unsigned long long m = __ballot(hit);
        if (lane == 0) s_cnt[w] = __popcll(m);
        __syncthreads();
        int pos = written + __popcll(m & lt);
        for (int q = 0; q < w; ++q) pos += s_cnt[q];
        if (hit && pos < kT) s_gid[pos] = j;
        written += (s_cnt[0] + s_cnt[1]) + (s_cnt[2] + s_cnt[3]);
        __syncthreads();
    }
    return min(written, kT);
}

// Diagnostic only (gsvc_debug_set(5, 2) with gsvc_debug_set_ptr): s_memrealtime
// stamps per tile by thread 0 -- start, staged, forward done, scan done,
// items done, end -- as int64[8].
__device__ __forceinline__ long long tstamp() {
    long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// 8 workgroups per CU: <= 64 VGPRs (launch bound: 8 waves per SIMD) and
// <= 20 KB of LDS (16-bit rectangles and item offsets).
template <bool kStamp>
__global__ __launch_bounds__(256, 8) void train_tile_kernel(TrainTileArgs A) {
    // LDS: geo / col / pix, reused as the 9 x 256 gradient reduction buffer
    // once the backward loop is done
    __shared__ float4 s_buf[3 * kT];
    __shared__ float2 s_ext[kT];     // b, id bits
    __shared__ unsigned short s_rect[kT];  // pixels of the tile the entry can reach (ellipse_rect)
    constexpr int kHalf = kT / 2;
    __shared__ float s_part[9][kHalf];  // backward: partial gradients of half a round of items
    __shared__ unsigned short s_off[kT + 1];  // backward: first work item of each entry (<= 8192)
    __shared__ int s_cnt[4];
    __shared__ int s_tot[4];         // backward: per-wave item totals (s_cnt still holds
                                     // the last-entry maxima other waves may be reading)
    __shared__ float s_err[2][4];
    float4 *s_geo = s_buf;           // x, y, a/2, b
    float4 *s_col = s_buf + kT;      // c/2, opacity, r, g
    float4 *s_pix = s_buf + 2 * kT;  // v_out rgb, last contributing entry (bits; -1 outside)
    int *s_ids = reinterpret_cast<int *>(s_pix);  // unsorted ids while staging
    const int tile = xcd_remap(blockIdx.x, A.ntiles);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    long long *st = kStamp ? A.stamps + 8 * (size_t)tile : nullptr;
    if (kStamp && tid == 0) st[0] = tstamp();
    const int ty = tile / A.tbx, tx = tile - ty * A.tbx;
    const int pi = ty * kTile + (tid >> 4), pj = tx * kTile + (tid & 15);
    const bool inside = pi < A.img_h && pj < A.img_w;
    const float tx0 = (float)(tx * kTile), ty0 = (float)(ty * kTile);
    // this pixel's target, loaded first: its latency overlaps the staging
    const size_t hw = (size_t)A.img_w * (size_t)A.img_h;
    const size_t pix = inside ? (size_t)pi * (size_t)A.img_w + (size_t)pj : 0;
    const float gt0 = A.gt[pix], gt1 = A.gt[hw + pix], gt2 = A.gt[2 * hw + pix];
    // slots below kSpec are loaded speculatively in the same round trip as the
    // count (most tiles have that few entries); the rest once the count is known
    constexpr int kSpec = 32;
    float4 r0 = make_float4(0.f, 0.f, 0.f, 0.f), r1 = r0, r2 = r0;
    if (tid < kSpec) {
        const float4 *r = slab_rec(A.slab, A.ntiles, tile, tid);
        r0 = r[0];
        r1 = r[1];
        r2 = r[2];
    }
    const bool empty = *A.m_dev < 1;  // rasterize_sum.py:121-127: background, no gradient
    const int n_all = empty ? 0 : (int)A.counts[tile];
    if (tid == 0) A.counts_clear[tile] = 0u;  // the next frame's counts

    // 1. the tile's first <= 256 entries in (tile, splat id) order into LDS
    int n;
    int rank = tid;
    if (n_all <= kT) {
        int id = 0x7fffffff;
        if (tid >= kSpec && tid < n_all) {
            const float4 *r = slab_rec(A.slab, A.ntiles, tile, tid);
            r0 = r[0];
            r1 = r[1];
            r2 = r[2];
        }
        if (tid < n_all) id = __float_as_int(r2.y);
        s_ids[tid] = id;
        __syncthreads();
        if (tid < n_all) {
            rank = 0;
            for (int j = 0; j < n_all; ++j) rank += s_ids[j] < id ? 1 : 0;  // ids are unique
        }
        n = n_all;
    } else {
        n = block_brute_ids(A, tx, ty, s_ids, s_cnt);
        if (tid < n) {
            const int g = s_ids[tid];
            r0 = A.rec[3 * g];
            r1 = A.rec[3 * g + 1];
            r2 = A.rec[3 * g + 2];
        }
    }
    __syncthreads();  // s_ids (in s_pix) read
    if (tid < n) {
        s_geo[rank] = r0;
        s_col[rank] = r1;
        s_ext[rank] = make_float2(r2.x, r2.y);
        s_rect[rank] = (unsigned short)ellipse_rect(r0.x, r0.y, r2.z, r0.w, r2.w, r1.y, tx0, ty0);
    }
    __syncthreads();
    if (kStamp && tid == 0) st[1] = tstamp();

    // 2. pixel-parallel forward (the sum rasterizer's op sequence), clamp, loss
    float o[3] = {0.f, 0.f, 0.f};
    if (empty) {
        o[0] = A.bg[0];
        o[1] = A.bg[1];
        o[2] = A.bg[2];
    }
    int last = 0;
    {
        const float py = (float)pi, px = (float)pj;
        for (int k = 0; k < n; ++k) {
            // skip an entry that reaches none of this wave's 4 rows
            const unsigned rc = s_rect[k];
            if (rc == kNoRect || (int)((rc >> 12) & 15u) < 4 * w || (int)((rc >> 8) & 15u) > 4 * w + 3)
                continue;
            const float4 G = s_geo[k];
            const float4 C = s_col[k];
            const float dy = G.y - py;
            const float cq = (C.x * dy) * dy;
            const float bdy = G.w * dy;
            const float dx = G.x - px;
            const float sg = fmaf(fmaf(G.z, dx, bdy), dx, cq);
            const float al = fminf(1.0f, C.y * __builtin_amdgcn_exp2f(sg * kNegLog2e));
            if (!(sg < 0.0f) && !(al < kAlphaMin)) {
                o[0] = fmaf(C.z, al, o[0]);
                o[1] = fmaf(C.w, al, o[1]);
                o[2] = fmaf(s_ext[k].x, al, o[2]);
                last = k;
            }
        }
    }
    float v[3], se = 0.f, ae = 0.f;
    {
        const float gtv[3] = {gt0, gt1, gt2};
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float x = clamp_unit(o[c]);
            const float d = x - gtv[c];
            se = fmaf(d, d, se);
            ae += fabsf(d);
            // mse_loss backward: norm * (a - b) * 1; l1: (1 / numel) * sgn(a - b);
            // clamp backward passes where 0 <= out <= 1
            const float sg = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
            const float gv = A.loss_l1 ? A.norm * sg : A.norm * d;
            v[c] = (inside && o[c] >= 0.0f && o[c] <= 1.0f) ? gv : 0.0f;
            if (A.out && inside) A.out[c * hw + pix] = x;
        }
        if (!inside) se = ae = 0.0f;
    }
    s_pix[tid] = make_float4(v[0], v[1], v[2], __int_as_float(inside ? last : -1));
    int f = inside ? last : -1;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        se += __shfl_xor(se, off, 64);
        ae += __shfl_xor(ae, off, 64);
        f = max(f, __shfl_xor(f, off, 64));
    }
    if (lane == 0) {
        s_err[0][w] = se;
        s_err[1][w] = ae;
        s_cnt[w] = f;
    }
    __syncthreads();
    if (tid == 0)
        A.err[tile] = make_float2((s_err[0][0] + s_err[0][1]) + (s_err[0][2] + s_err[0][3]),
                                  (s_err[1][0] + s_err[1][1]) + (s_err[1][2] + s_err[1][3]));
    if (kStamp && tid == 0) st[2] = tstamp();
    const int maxf = max(max(s_cnt[0], s_cnt[1]), max(s_cnt[2], s_cnt[3]));
    const int kend = min(n, maxf + 1);  // entries past every pixel's last contribute nothing
    if (kend <= 0) return;

    // 3. backward over compact work items: entry e's reachable rectangle
    // (ellipse_rect) is cut into runs of kRun pixels (row-major), one item per
    // thread per round, so lanes only evaluate (entry, pixel) pairs that can
    // contribute; an item's 9 partial sums go to LDS and each entry adds its
    // items' partials in item order (deterministic within the tile)
    constexpr int kRun = 8;
    int items = 0;
    if (tid < kend) {
        const unsigned rc = s_rect[tid];
        if (rc != kNoRect) {
            const int rw = (int)((rc >> 4) & 15u) - (int)(rc & 15u) + 1;
            const int rh = (int)((rc >> 12) & 15u) - (int)((rc >> 8) & 15u) + 1;
            items = (rw * rh + kRun - 1) / kRun;
        }
    }
    // exclusive scan of items over the entries (wave scan + LDS)
    int incl = items;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(incl, off, 64);
        if (lane >= off) incl += u;
    }
    if (lane == 63) s_tot[w] = incl;
    __syncthreads();
    int wave_off = 0;
    for (int q = 0; q < w; ++q) wave_off += s_tot[q];
    const int total = (s_tot[0] + s_tot[1]) + (s_tot[2] + s_tot[3]);
    if (tid < kend) s_off[tid] = (unsigned short)(wave_off + incl - items);
    if (tid == 0) s_off[kend] = (unsigned short)total;
    if (kStamp && tid == 0) st[3] = tstamp();
    float acc[9];
#pragma unroll
    for (int c = 0; c < 9; ++c) acc[c] = 0.0f;
    for (int base = 0; base < total; base += kT) {
        __syncthreads();  // s_off written / the previous round's partials summed
        const int item = base + tid;
        float g[9];
#pragma unroll
        for (int c = 0; c < 9; ++c) g[c] = 0.0f;
        if (item < total) {
            // entry of this item: the last e with s_off[e] <= item
            int lo = 0, hi = kend - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if ((int)s_off[mid] <= item) lo = mid;
                else hi = mid - 1;
            }
            const int e = lo;
            const unsigned rc = s_rect[e];
            const int rx0 = (int)(rc & 15u), rw = (int)((rc >> 4) & 15u) - rx0 + 1;
            const int ry0 = (int)((rc >> 8) & 15u);
            const int area = rw * ((int)((rc >> 12) & 15u) - ry0 + 1);
            const int q0 = (item - (int)s_off[e]) * kRun;
            int yy = q0 / rw, xx = q0 - yy * rw;
            const float4 G = s_geo[e];
            const float4 C = s_col[e];
            const float2 X = s_ext[e];
            // full conic a, c: 2 * (a / 2) is exact for every normal float
            const float fa = 2.0f * G.z, fc = 2.0f * C.x;
            for (int q = q0; q < q0 + kRun && q < area; ++q) {
                const int pxl = (ry0 + yy) * kTile + rx0 + xx;
                if (++xx == rw) {
                    xx = 0;
                    ++yy;
                }
                const float4 P = s_pix[pxl];
                if (e > __float_as_int(P.w)) continue;
                const float dx = G.x - (tx0 + (float)(pxl & 15));
                const float dy = G.y - (ty0 + (float)(pxl >> 4));
                const float sgm = splat_sigma_h(G.z, G.w, C.x, dx, dy);
                const float vis = exp_neg(sgm);
                const float al = fminf(1.0f, C.y * vis);
                if (sgm < 0.0f || al < kAlphaMin) continue;
                const float v_alpha = fmaf(X.x, P.z, fmaf(C.w, P.y, C.z * P.x));
                const float v_sigma = (-C.y * vis) * v_alpha;
                g[5] = fmaf(al, P.x, g[5]);
                g[6] = fmaf(al, P.y, g[6]);
                g[7] = fmaf(al, P.z, g[7]);
                const float hs = 0.5f * v_sigma;
                const float hsdx = hs * dx;
                g[2] = fmaf(hsdx, dx, g[2]);
                g[3] = fmaf(hsdx, dy, g[3]);
                g[4] = fmaf(hs * dy, dy, g[4]);
                g[0] = fmaf(v_sigma, fmaf(fa, dx, G.w * dy), g[0]);
                g[1] = fmaf(v_sigma, fmaf(G.w, dx, fc * dy), g[1]);
                g[8] = fmaf(vis, v_alpha, g[8]);
            }
        }
        // the two halves of the round publish their partials in turn (4.5 KB
        // of LDS instead of 9 KB: one more workgroup per CU)
        for (int h = 0; h < 2; ++h) {
            const int hb = base + h * kHalf;
            if (hb >= total) break;
            if (h == 1) __syncthreads();  // the first half consumed
            if ((tid >> 7) == h) {
#pragma unroll
                for (int c = 0; c < 9; ++c) s_part[c][tid - h * kHalf] = g[c];
            }
            __syncthreads();
            if (tid < kend) {
                const int i0 = max((int)s_off[tid], hb), i1 = min((int)s_off[tid + 1], hb + kHalf);
                for (int it = i0; it < i1; ++it) {
#pragma unroll
                    for (int c = 0; c < 9; ++c) acc[c] += s_part[c][it - hb];
                }
            }
        }
    }
    __syncthreads();  // every item read: the geo / col / pix buffer holds the entry sums
    if (kStamp && tid == 0) st[4] = tstamp();
    float(*s_sum)[kT] = reinterpret_cast<float(*)[kT]>(s_buf);
    if (tid < kend) {
#pragma unroll
        for (int c = 0; c < 9; ++c) s_sum[c][tid] = acc[c];
    }
    __syncthreads();
    // 16 lanes per entry, 9 of them add one float each into the splat's
    // 64-byte gradient record: one memory request per (splat, tile)
    for (int q = tid; q < kend * 16; q += kT) {
        const int e2 = q >> 4, c = q & 15;
        if (c < 9) unsafeAtomicAdd(A.grad + (size_t)__float_as_int(s_ext[e2].y) * 16 + c, s_sum[c][e2]);
    }
    if (kStamp && tid == 0) st[5] = tstamp();
}

// ---------------------------------------------------------------------------
// Two waves per tile (production): train_tile_kernel's per-tile work in a
// 128-thread workgroup whose waves each own one 8-row band of the tile
// (2 pixels per lane), 9.9 KB of LDS, so 16 tiles are resident per CU (the
// 256-thread kernel: 8).
//   1. count + the first kWSpec slab records in the same round trip as the
//      lanes' gt; records ranked by id and staged at their rank with their
//      reachable rectangle (ellipse_rect).  > 64 entries: ids ranked through
//      LDS (or rebuilt past 256 from the splats' bboxes) and records gathered
//      64 at a time.
//   2. forward: each wave blends only the entries whose rectangle reaches its
//      band (a culled pair contributes nothing in the reference either), in
//      entry order, with the render's op sequence at unit opacity (1 * e ==
//      e: the same image bits); clamp, loss gradient, error sums; v_out planes
//      into LDS.
//   3. backward, each wave over the rectangle rows of its own band: work
//      items = one row of an entry's rectangle (the row terms of sigma
//      shared; per-pixel sums factored by dy), entries laid out longest rows
//      first in four length classes, rounds of 64 items; per round a DPP
//      segmented scan (one v_fmac_f32_dpp per sum and step) gives each run of
//      an entry's items its sum, which the run's last item adds to the
//      entry's LDS sums (a fixed order, no LDS atomics); then 8 lanes per
//      entry add the two bands' 32 bytes into the splat's gradient record
//      (one request per (splat, tile)).
// GSVC's opacity is ones (GaussianSplats_Represent.py:84) and the training
// step projects with opacity 1, so the opacity gradient (record slot 8) is
// not formed.
constexpr int kBSpec = 32;    // slab slots loaded with the count (64: slower, measured)
constexpr int kBChunk = 64;   // entries staged at a time
// rows wider than this split into two work items (A/B knob 11).  16 = never:
// measured 51.6 vs 54.0 us (10) at trained density, 31.8 vs 32.1 at init --
// fewer rounds of segmented sums beat the longer pixel loops once items are
// laid out by length (tools/item_sim.py models it)
constexpr int kBRun = 16;
constexpr int kBThreads = 128;
// The band kernel's speculative slab records and work-item split width: the
// constants in the product library, A/B knobs 12 / 11 in the diagnostic one.
__device__ __forceinline__ int spec_of(const TrainTileArgs &A) { return kDiag ? A.spec : kBSpec; }
__device__ __forceinline__ int brun_of(const TrainTileArgs &A) { return kDiag ? A.brun : kBRun; }

typedef float v2f __attribute__((ext_vector_type(2)));

// raster_sum.hip blend_pair at opacity 1 (no index tracking): one splat
// against two pixels of a row; a failing pair keeps its accumulators.
__device__ __forceinline__ void blend2_unit(float gx, float ha, float bdy, float cq, float cr,
                                            float cg, float cb, v2f px, v2f &ar, v2f &ag, v2f &ab) {
    const v2f dx = gx - px;
    const v2f q = __builtin_elementwise_fma((v2f)ha, dx, (v2f)bdy);
    const v2f sg = __builtin_elementwise_fma(q, dx, (v2f)cq);
    const v2f x = sg * kNegLog2e;
    const v2f e = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
    const v2f a = {fminf(1.0f, e.x), fminf(1.0f, e.y)};
    const bool v0 = !(sg.x < 0.0f) && !(a.x < kAlphaMin);
    const bool v1 = !(sg.y < 0.0f) && !(a.y < kAlphaMin);
    const v2f nr = __builtin_elementwise_fma((v2f)cr, a, ar);
    const v2f ng = __builtin_elementwise_fma((v2f)cg, a, ag);
    const v2f nb = __builtin_elementwise_fma((v2f)cb, a, ab);
    ar = (v2f){v0 ? nr.x : ar.x, v1 ? nr.y : ar.y};
    ag = (v2f){v0 ? ng.x : ag.x, v1 ? ng.y : ag.y};
    ab = (v2f){v0 ? nb.x : ab.x, v1 ? nb.y : ab.y};
}

// blend2_unit for an entry whose colour is finite: a failing pair adds
// c * 0 (= +-0) instead of selecting -- the same bits, since an accumulator
// is never -0 (it starts at +0 or the background, and an exact cancellation
// rounds to +0) -- 2 selects instead of 6.  A non-finite colour times 0 is NaN,
// so such entries keep blend2_unit.
__device__ __forceinline__ void blend2_unit_fin(float gx, float ha, float bdy, float cq, float cr,
                                                float cg, float cb, v2f px, v2f &ar, v2f &ag,
                                                v2f &ab) {
    const v2f dx = gx - px;
    const v2f q = __builtin_elementwise_fma((v2f)ha, dx, (v2f)bdy);
    const v2f sg = __builtin_elementwise_fma(q, dx, (v2f)cq);
    const v2f x = sg * kNegLog2e;
    const v2f e = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
    const v2f a = {fminf(1.0f, e.x), fminf(1.0f, e.y)};
    const bool v0 = !(sg.x < 0.0f) && !(a.x < kAlphaMin);
    const bool v1 = !(sg.y < 0.0f) && !(a.y < kAlphaMin);
    const v2f av = {v0 ? a.x : 0.0f, v1 ? a.y : 0.0f};
    ar = __builtin_elementwise_fma((v2f)cr, av, ar);
    ag = __builtin_elementwise_fma((v2f)cg, av, ag);
    ab = __builtin_elementwise_fma((v2f)cb, av, ab);
}

// blend2_unit_fin with the alpha cut as a sigma threshold (common.h
// kSigmaCutBits: the same pairs pass, and alpha = exp(-sigma) <= 1 for them,
// so the min(1, .) goes too) -- for entries whose colour is finite and whose
// geometry is bounded (geo_cut_ok: sigma is then never NaN, the one value the
// threshold decides differently).  The same bits as blend2_unit_fin.
__device__ __forceinline__ void blend2_cut(float gx, float ha, float bdy, float cq, float cr,
                                           float cg, float cb, v2f px, v2f &ar, v2f &ag, v2f &ab) {
    const v2f dx = gx - px;
    const v2f q = __builtin_elementwise_fma((v2f)ha, dx, (v2f)bdy);
    const v2f sg = __builtin_elementwise_fma(q, dx, (v2f)cq);
    const v2f x = sg * kNegLog2e;
    const v2f e = {__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)};
    const bool v0 = __float_as_uint(sg.x) <= kSigmaCutBits;
    const bool v1 = __float_as_uint(sg.y) <= kSigmaCutBits;
    const v2f av = {v0 ? e.x : 0.0f, v1 ? e.y : 0.0f};
    ar = __builtin_elementwise_fma((v2f)cr, av, ar);
    ag = __builtin_elementwise_fma((v2f)cg, av, ag);
    ab = __builtin_elementwise_fma((v2f)cb, av, ab);
}


// The loss workgroup's loads per round: 16 tile pairs per thread in flight, so
// a 1080p frame (4080 pairs) is one round trip.
constexpr int kLossBatch = 16;

// The frame's losses from the tiles' error sums, in double and in ONE fixed
// order whatever the workgroup size (kThreads = 128 or 256 emulate the same 256
// virtual threads: virtual thread v sums pairs v, v + 256, ... in batches, the
// 64-lane xor trees reduce virtual waves, the four are added pairwise; a
// 128-thread loss workgroup in the tile kernel, publishing while the last
// tiles' backward ran, was measured and removed: tile kernel 117 / 57 vs 52.8
// us with a per-tile counter / written-through sentinel polls,
// profiles/r03/loss_wg/), then
// stored into ``loss`` -- with GSVC_TRAIN_LOSS_SEQ the pair count (det) and the
// sequence word after them, released to the host.  Every thread calls it.
// (kBatch: loads in flight per round; the order of the additions does not
// depend on it)
template <int kThreads, int kBatch = kLossBatch>
__device__ __forceinline__ void publish_loss(const float2 *err, int ntiles, double inv_count,
                                             float *loss, unsigned loss_seq, const int *det_off,
                                             int n, double (*s_l)[4]) {
    // virtual threads per thread (a workgroup wider than 256: its first 256
    // threads are the virtual ones, the others add nothing)
    constexpr int kV = (256 + kThreads - 1) / kThreads;
    const int tid = threadIdx.x;
    double s2[kV], s1[kV];
    const int npair = ntiles >> 1;
    const float4 *e4 = reinterpret_cast<const float4 *>(err);
#pragma unroll
    for (int q = 0; q < kV; ++q) {
        s2[q] = 0.0;
        s1[q] = 0.0;
        for (int t0 = tid + q * kThreads; t0 < npair && tid + q * kThreads < 256;
             t0 += kBatch * 256) {
            float4 e[kBatch];
#pragma unroll
            for (int k = 0; k < kBatch; ++k) {
                const int t = t0 + 256 * k;
                e[k] = t < npair ? e4[t] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int k = 0; k < kBatch; ++k) {
                s2[q] += (double)e[k].x;
                s1[q] += (double)e[k].y;
                s2[q] += (double)e[k].z;
                s1[q] += (double)e[k].w;
            }
        }
    }
    if ((ntiles & 1) && tid == 0) {
        const float2 e = err[ntiles - 1];
        s2[0] += (double)e.x;
        s1[0] += (double)e.y;
    }
#pragma unroll
    for (int q = 0; q < kV; ++q) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            s2[q] += __shfl_xor(s2[q], off, 64);
            s1[q] += __shfl_xor(s1[q], off, 64);
        }
        if ((tid & 63) == 0 && tid + q * kThreads < 256) {
            s_l[0][(tid + q * kThreads) >> 6] = s2[q];
            s_l[1][(tid + q * kThreads) >> 6] = s1[q];
        }
    }
    __syncthreads();
    if (tid == 0) {
        loss[0] = (float)(((s_l[0][0] + s_l[0][1]) + (s_l[0][2] + s_l[0][3])) * inv_count);
        loss[1] = (float)(((s_l[1][0] + s_l[1][1]) + (s_l[1][2] + s_l[1][3])) * inv_count);
        // deterministic mode: this frame's (splat, tile) pair count, so
        // the caller can size det_capacity (word 3, before the release)
        if (loss_seq && det_off) reinterpret_cast<unsigned *>(loss)[3] = (unsigned)det_off[n];
        // coherent host memory: the host stops waiting here, while the
        // rest of the step still runs (later work on the stream is ordered
        // after it anyway)
        if (loss_seq)
            __hip_atomic_store(reinterpret_cast<unsigned *>(loss) + 2, loss_seq, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}


// Carried bins of a tile with 256 < n <= kTrainCarryCap candidates (every
// thread of the workgroup calls it; the same return value in each): the
// ascending ids of the candidates whose current box holds the tile -- the
// first <= 256 members -- into s_out, by the id-window bitmap (tile_ids.h).
// Ids are unique within a tile's candidates.  Thread t owns candidates
// t + kBThreads k (a 32-bit mask of which are members); the gathers go 8 per
// thread per round trip (ids, then their boxes), and each id window re-reads the
// thread's ids 16 at a time (L2-resident).  Both waves set bits in the shared
// bitmap, wave 0 emits.  ``s_misc``: 4 ints of scratch.
template <int kThreads>
__device__ int wg_sorted_members(const int *cand, int n, const uint2 *cbox, unsigned tx,
                                 unsigned ty, int *s_out, unsigned *bm, int *s_misc) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int kPer = kTrainCarryCap / kThreads, kQ = 4, kR = 4;
    static_assert(kPer <= 32 && kPer % kQ == 0 && kPer % kR == 0, "membership mask layout");
    n = min(n, kTrainCarryCap);
    unsigned mem = 0u;
    int lo = 0x7fffffff, hi = -1;
    for (int k0 = 0; k0 < kPer && kThreads * k0 < n; k0 += kQ) {
        int id[kQ];
        uint2 b[kQ];
#pragma unroll
        for (int q = 0; q < kQ; ++q) id[q] = cand[min(tid + kThreads * (k0 + q), n - 1)];
#pragma unroll
        for (int q = 0; q < kQ; ++q) b[q] = cbox[id[q]];
#pragma unroll
        for (int q = 0; q < kQ; ++q) {
            if (tid + kThreads * (k0 + q) < n && box_has(b[q], tx, ty)) {
                mem |= 1u << (k0 + q);
                lo = min(lo, id[q]);
                hi = max(hi, id[q]);
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        lo = min(lo, __shfl_xor(lo, off, 64));
        hi = max(hi, __shfl_xor(hi, off, 64));
    }
    if (lane == 0) {
        s_misc[2 * w] = lo;
        s_misc[2 * w + 1] = hi;
    }
    __syncthreads();
    lo = min(s_misc[0], s_misc[2]);
    hi = max(s_misc[1], s_misc[3]);
    int written = 0;
    for (long long base = lo; base <= hi && written < kTilePix; base += 32 * kSortWords) {
        for (int k = tid; k < kSortWords; k += kThreads) bm[k] = 0u;
        __syncthreads();
        for (int k0 = 0; k0 < kPer && kThreads * k0 < n; k0 += kR) {
            int id[kR];
#pragma unroll
            for (int q = 0; q < kR; ++q) id[q] = cand[min(tid + kThreads * (k0 + q), n - 1)];
#pragma unroll
            for (int q = 0; q < kR; ++q)
                if ((mem >> (k0 + q)) & 1u) bitmap_set(bm, (long long)id[q] - base);
        }
        __syncthreads();
        if (w == 0) {
            written = bitmap_emit(bm, base, written, s_out);
            if (lane == 0) s_misc[0] = written;
        }
        __syncthreads();
        written = s_misc[0];
        __syncthreads();  // (s_misc and the bitmap are rewritten by the next window)
    }
    return min(written, kTilePix);
}

struct BandLds {
    float v[3][kTile * kVRow];     // v_out planes, rows padded to kVRow words
    float4 geo[kBChunk + 1];       // staged entries (rank order): x, y, a/2, b
    float4 col[kBChunk + 1];       //   c/2, r, g, b  (slot kBChunk: the no-op sentinel)
    unsigned short ro[kBChunk];    //   rectangle (ellipse_rect, 16 bits)
    int gid[kBChunk];              //   splat id
    float part[8][kBThreads + 1];  // order: ranking / sort scratch; backward: entry sums per wave
    signed char own[kBThreads];    // backward: per wave, the entry of the round's first items
    signed char perm[kBThreads];   // backward: per wave, the chunk's entries by item length
    int misc[4];   // the waves' error sums
    int nsel;      // carried bins: the tile's entries among its candidates
};
// the order phase reads part row 0 as int4s (ids at [0, 64), candidates at [64, 128))
static_assert(offsetof(BandLds, part) % 16 == 0, "BandLds.part must be 16-byte aligned");

// kDet: GSVC_TRAIN_DETERMINISTIC's slot stores in place of the atomics (its
// own instantiation: the slot arithmetic in the flush would cost the atomic
// kernel two spilled VGPRs)
// kCarry: GSVC_TRAIN_CARRY's carried bins (A.cids) in place of the slab
template <bool kStamp, bool kDet = false, bool kCarry = false>
__global__ __launch_bounds__(kBThreads, 8) void train_tile_band_kernel(TrainTileArgs A) {
    __shared__ BandLds S;
    // Wave issue priority: the arbiter favours older waves, so without it a
    // workgroup dispatched late onto a busy CU waits behind its elders' blending
    // before it can even issue its loads and ranking (stamps: the order phase
    // grows from 2.6 us for the first workgroups of a CU to 11.7 us for its
    // 13th-16th, profiles/r03/stamps).  Raised over the order phase, a young
    // tile gets its round trips going while its elders compute.
    if (!kDiag || A.prio) __builtin_amdgcn_s_setprio(3);
    // runs of 16 tiles dealt over the XCDs: dense content (a textured frame's
    // objects) spread over all eight instead of loading the one or two whose
    // contiguous range covers them (tile kernel 273.7 -> 238.7 us on the
    // textured video's frame 116, unchanged on the bench's frame).
    // A/B knob 37: 1 dispatch order, 4 contiguous ranges (runs of 4, 8 and 32
    // were measured, round 5: within the dense frame's spread, not kept)
    const int tile = !(kDiag && A.xcd_off) ? xcd_runs<16>(blockIdx.x, A.ntiles)
                     : A.xcd_off == 1      ? (int)blockIdx.x
                                           : xcd_remap(blockIdx.x, A.ntiles);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    long long *st = kStamp ? A.stamps + 8 * (size_t)tile : nullptr;
    if (kStamp && tid == 0) st[0] = tstamp();
    const int ty = tile / A.tbx, tx = tile - ty * A.tbx;
    const float tx0 = (float)(tx * kTile), ty0 = (float)(ty * kTile);
    const int prow = 8 * w + (lane >> 3), pcol = (lane & 7) << 1;  // tile-local pixel pair
    const int pi = ty * kTile + prow, pj = tx * kTile + pcol;
    const bool row_in = pi < A.img_h;
    const int nin = row_in ? min(2, A.img_w - pj) : 0;  // pixels of the pair inside the image
    const size_t hw = (size_t)A.img_w * (size_t)A.img_h;
    const size_t pix0 = row_in ? (size_t)pi * (size_t)A.img_w + (size_t)pj : 0;
    // one round trip for everything the tile starts from, with no wait in
    // between (a branch around a load makes the compiler wait for it at the
    // join): the frame's M and this tile's count (scalar), the first kBSpec
    // slab records (lanes past kBSpec re-read slot 0: the same lines), the
    // pair's targets (lanes outside the image read pixel 0; only the loss
    // reads them, masked)
    constexpr bool carry = kCarry;
    const int m_frame = *A.m_dev;
    const unsigned cnt_raw = A.counts[tile];
    const unsigned srt_raw = kCarry && A.csorted ? A.csorted[tile] : 0u;
    float4 r0, r1, r2;
    int cid = 0;  // carried bins: the lane's candidate id
    int *tcids = carry ? A.cids + (size_t)tile * kTrainCarryCap : nullptr;
    if (carry) {
        cid = tcids[tid < spec_of(A) ? tid : 0];
    } else {
        const float4 *h0 = slab_rec(A.slab, A.ntiles, tile, tid < spec_of(A) ? tid : 0);
        r0 = h0[0];
        r1 = h0[1];
        r2 = h0[2];
    }
    // the pair's targets go straight into LDS (global_load_lds: no VGPRs held
    // over the order and forward phases -- held in registers they spilled, and
    // the spill's vmcnt(0) cost the carried-bins kernel a round trip), into the
    // v_out planes' space, [wave][c][q][lane], which the loss phase overwrites
    // only after every wave has read its targets back
    float *sgt = &S.v[0][0] + w * (6 * 64);
    {
        typedef __attribute__((address_space(1))) void gvoid;
        typedef __attribute__((address_space(3))) void lvoid;
        const size_t b0 = nin > 0 ? pix0 : 0, b1 = nin > 1 ? pix0 + 1 : b0;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            __builtin_amdgcn_global_load_lds((gvoid *)(A.gt + c * hw + b0), (lvoid *)(sgt + (2 * c) * 64), 4, 0, 0);
            __builtin_amdgcn_global_load_lds((gvoid *)(A.gt + c * hw + b1), (lvoid *)(sgt + (2 * c + 1) * 64), 4, 0, 0);
        }
    }
    const bool empty = m_frame < 1;  // rasterize_sum.py:121-127: background, no gradient
    // (a mask, not a branch: the count's load must not sink behind M's)
    const int n_all = (int)__builtin_amdgcn_readfirstlane(cnt_raw) & -(int)!empty;
    if (carry && tile == 0 && tid == 0) *A.m_clear = 0;  // the next frame's M (the splat kernel's)
    if (tid == 0) {
        A.counts_clear[tile] = 0u;  // the next frame's counts
        // the grouped forward's padding entry: sigma = +inf at every pixel, so
        // alpha = 0 fails the test and it adds 0 * colour 0 (no change)
        S.geo[kBChunk] = make_float4(0.0f, 1e30f, 0.0f, 0.0f);
        S.col[kBChunk] = make_float4(1e30f, 0.0f, 0.0f, 0.0f);
    }
    const bool dense = n_all > kBChunk;
    const bool brute = n_all > kTilePix;  // the slab dropped entries: ids rebuilt
    // dense: the splat ids by rank (part rows 0-1), the slab's ids (rows 2-3,
    // scratch) and the sort's 512-word bitmap (rows 4-7)
    int *s_key = reinterpret_cast<int *>(&S.part[0][0]);
    int *s_ids = reinterpret_cast<int *>(&S.part[2][0]);
    int n = n_all;

    // 1. the order
    if (!dense && carry) {
        // <= 64 candidates: wave 0 gathers their records and boxes by id, keeps
        // the tile's entries and ranks them by id (the others rank last)
        if (w == 0) {
            if (lane >= spec_of(A) && lane < n) cid = tcids[lane];
            bool mem = false;
            if (lane < n) {
                const uint2 b = A.cbox[cid];
                r0 = A.rec[3 * (size_t)cid];
                r1 = A.rec[3 * (size_t)cid + 1];
                r2 = A.rec[3 * (size_t)cid + 2];
                mem = box_has(b, (unsigned)tx, (unsigned)ty);
            }
            const int id = mem ? cid : 0x7fffffff;
            int rank = 0;
            const bool sorted = A.csorted && (int)__builtin_amdgcn_readfirstlane(srt_raw) == n;
            if (sorted) {
                // candidates in id order: a member's rank is the members below it
                rank = __popcll(__ballot(mem) & ((1ull << lane) - 1ull));
            } else if (kDiag && (A.diag & 128)) {
                rank = rank_below(id, n);
            } else {
                // rank by id with the ids through LDS (part row 0, free during the
                // order), four per broadcast read: 2 VALU per candidate instead of
                // a readlane loop's 3 (lanes past n hold 0x7fffffff, below no id)
                int *s_rid = reinterpret_cast<int *>(&S.part[0][0]);
                s_rid[lane] = id;
                wave_lds_sync();
                for (int k = 0; k < n; k += 4) {
                    const int4 q = *reinterpret_cast<const int4 *>(s_rid + k);
                    rank += (q.x < id ? 1 : 0) + (q.y < id ? 1 : 0) + (q.z < id ? 1 : 0) +
                            (q.w < id ? 1 : 0);
                }
                if (A.csorted) {
                    // every candidate's place in id order (part row 0 past s_rid
                    // as the scratch; the ids are unique), written back for later steps
                    int *s_cid = reinterpret_cast<int *>(&S.part[0][0]) + 64;  // 16-byte aligned
                    const int cv = lane < n ? cid : 0x7fffffff;
                    s_cid[lane] = cv;
                    wave_lds_sync();
                    int place = 0;
                    for (int k = 0; k < n; k += 4) {
                        const int4 q = *reinterpret_cast<const int4 *>(s_cid + k);
                        place += (q.x < cv ? 1 : 0) + (q.y < cv ? 1 : 0) + (q.z < cv ? 1 : 0) +
                                 (q.w < cv ? 1 : 0);
                    }
                    if (lane < n) tcids[place] = cid;
                    if (lane == 0) A.csorted[tile] = (unsigned)n;
                }
            }
            if (mem) {
                S.geo[rank] = r0;
                S.col[rank] = make_float4(r1.x, r1.z, r1.w, r2.x);
                S.gid[rank] = id;
                S.ro[rank] = ellipse_rect(r0.x, r0.y, 2.0f * r0.z, r0.w, 2.0f * r1.x, 1.0f, tx0, ty0);
            }
            const int nm = __popcll(__ballot(mem));  // (the whole wave's ballot)
            if (lane == 0) S.nsel = nm;
        }
    } else if (!dense) {
        if (tid >= spec_of(A) && tid < n) {
            const float4 *h = slab_rec(A.slab, A.ntiles, tile, tid);
            r0 = h[0];
            r1 = h[1];
            r2 = h[2];
        }
        if (w == 0 && lane < n) {
            const int id = __float_as_int(r2.y);
            const int rank = rank_below(id, n);
            S.geo[rank] = r0;
            S.col[rank] = make_float4(r1.x, r1.z, r1.w, r2.x);
            S.gid[rank] = id;
            S.ro[rank] = ellipse_rect(r0.x, r0.y, 2.0f * r0.z, r0.w, 2.0f * r1.x, 1.0f, tx0, ty0);
        }
    } else if (brute) {
        unsigned *bm = reinterpret_cast<unsigned *>(&S.part[4][0]);
        if (carry && n_all <= kTrainCarryCap) {
            // carried bins of <= kTrainCarryCap candidates: the members sorted
            // from the list by both waves (the bbox rebuild over every splat
            // costs ~0.1-0.6 ms)
            const int nm = wg_sorted_members<kBThreads>(tcids, n_all, A.cbox, (unsigned)tx,
                                                        (unsigned)ty, s_key, bm, S.misc);
            if (tid == 0) S.nsel = nm;
        } else if (w == 0) {
            if (!carry && A.ovf && n_all <= kCarryCap) {
                // record slab + its overflow ids: the first 256 ids sorted from both
                SegIds seg;
                seg.ids = nullptr;
                seg.recs = slab_rec(A.slab, A.ntiles, tile, kHeadSlots) - 3 * kHeadSlots;
                seg.head = slab_rec(A.slab, A.ntiles, tile, 0);
                seg.ovf = A.ovf + (size_t)tile * kOvfSlots;
                n = wave_sorted_tile_ids(seg, n_all, s_key, bm);
            } else {
                n = wave_brute_ids(A.xys, A.radii, 0, A.num_points, A.tbx,
                                   (A.img_h + kTile - 1) / kTile, tile, s_key);
            }
            if (lane == 0) S.nsel = n;
        }
        // both waves: wave_brute_ids finds >= 256 of them (carried bins: the
        // candidates overflowed, the entries may be fewer -- wave 0's count)
        n = min(n_all, kTilePix);
    } else {
        // the slab's ids, sorted by wave 0 with an LDS bitmap over the id range
        // (tile_ids.h; O(n + id range / 16384 windows), not O(n^2) compares)
        if (carry) {
            // carried bins: the candidates whose box holds the tile, compacted
            if (tid == 0) S.nsel = 0;
            __syncthreads();
            for (int j = tid; j < n; j += kBThreads) {
                const int c = tcids[j];
                if (box_has(A.cbox[c], (unsigned)tx, (unsigned)ty)) s_ids[atomicAdd(&S.nsel, 1)] = c;
            }
            __syncthreads();
            n = S.nsel;
        } else {
            for (int j = tid; j < n; j += kBThreads)
                s_ids[j] = __float_as_int(slab_rec(A.slab, A.ntiles, tile, j)[2].y);
        }
        __syncthreads();
        if (w == 0) {
            SegIds ids;
            ids.ids = s_ids;
            ids.recs = nullptr;
            ids.head = nullptr;
            wave_sorted_tile_ids(ids, n, s_key, reinterpret_cast<unsigned *>(&S.part[4][0]));
        }
    }
    __syncthreads();
    if (carry && (!dense || brute)) n = S.nsel;
    if (!kDiag || A.prio) __builtin_amdgcn_s_setprio(0);
    if (kStamp && tid == 0) st[1] = tstamp();

    // 2. forward: this wave's band against the entries that can reach it
    v2f ar, ag, ab;
    {
        const float b0 = empty ? A.bg[0] : 0.0f, b1 = empty ? A.bg[1] : 0.0f, b2 = empty ? A.bg[2] : 0.0f;
        ar = (v2f){b0, b0};
        ag = (v2f){b1, b1};
        ab = (v2f){b2, b2};
    }
    const float py = (float)pi;
    const v2f px = {(float)pj, (float)(pj + 1)};
    const int y_lo = 8 * w, y_hi = 8 * w + 7;
    // dense: stage chunk [c0, c0 + cnt) of the order from the splats' records
    // (rec holds the slab's records by splat id)
    auto stage_chunk = [&](const int *keys, int cnt) {
        if (tid < cnt) {
            const int key = keys[tid];
            const float4 *rr = A.rec + 3 * (size_t)key;
            const float4 a = rr[0], b = rr[1], c = rr[2];
            S.geo[tid] = a;
            S.col[tid] = make_float4(b.x, b.z, b.w, c.x);
            S.gid[tid] = __float_as_int(c.y);
            S.ro[tid] = ellipse_rect(a.x, a.y, 2.0f * a.z, a.w, 2.0f * b.x, 1.0f, tx0, ty0);
        }
    };
    // the forward's lane-group lists (A.grouped): [64 iterations][8 groups] entry
    // indices per wave in part rows 2-3, free once the order is known (the
    // dense sort's scratch)
    unsigned char *wlist = reinterpret_cast<unsigned char *>(&S.part[2][0]) + w * 512;
    const int grp = ((lane >> 5) << 2) | ((lane & 7) >> 1);
    for (int c0 = 0; c0 < n; c0 += kBChunk) {
        const int cnt = min(kBChunk, n - c0);
        if (dense) {
            stage_chunk(s_key + c0, cnt);
            __syncthreads();
        }
        if (!kDiag || A.grouped) {
            // lane groups: 8 groups of 8 lanes, each a 4-row x 4-column block of
            // the band (grp); every group walks, in rank order, only the
            // entries whose rectangle reaches its block (lists[it][grp], padded
            // with the no-op sentinel entry kBChunk up to the longest list).
            // The pairs skipped contribute nothing (the band culling's own
            // argument), so every pixel sees the same sequence of blends.
            unsigned gm = 0u;
            bool fin = false, cutok = false;
            if (lane < cnt) {
                const unsigned rc = S.ro[lane];
                if (rc != kNoRect) {
                    const int ry0 = (int)((rc >> 8) & 15u), ry1 = (int)((rc >> 12) & 15u);
                    const unsigned rb = (unsigned)(ry0 <= y_lo + 3 && ry1 >= y_lo) |
                                        ((unsigned)(ry0 <= y_hi && ry1 >= y_lo + 4) << 1);
                    const unsigned cx0 = (rc & 15u) >> 2, cx1 = ((rc >> 4) & 15u) >> 2;
                    const unsigned cb = ((2u << cx1) - 1u) & ~((1u << cx0) - 1u);
                    gm = ((rb & 1u) ? cb : 0u) | ((rb & 2u) ? cb << 4 : 0u);
                }
                const float4 C = S.col[lane];
                fin = __builtin_isfinite(C.y) && __builtin_isfinite(C.z) && __builtin_isfinite(C.w);
                cutok = fin && geo_cut_ok(S.geo[lane], C.x);
            }
            if (kDiag && (A.diag & 4)) gm = 0u;  // diagnostic: no forward blending (wrong results)
            // row `lane` of the lists: the sentinel, then the entries
            *reinterpret_cast<unsigned long long *>(wlist + 8 * lane) = 0x4040404040404040ull;
            __builtin_amdgcn_wave_barrier();
            const unsigned long long below = (1ull << lane) - 1ull;
            int maxlen = 0;
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const bool in = (gm >> g) & 1u;
                const unsigned long long mg = __ballot(in);
                if (in) wlist[8 * __popcll(mg & below) + g] = (unsigned char)lane;
                maxlen = max(maxlen, __popcll(mg));
            }
            const unsigned long long any = __ballot(gm != 0u);
            const unsigned long long fm = __ballot(fin);
            const unsigned long long cm = __ballot(cutok);
            __builtin_amdgcn_wave_barrier();
            const unsigned char *ml = wlist + grp;
            if ((any & ~cm) == 0) {
                // finite colours and geometry (the rule): the threshold cut
                for (int it = 0; it < maxlen; ++it) {
                    const int k = ml[8 * it];
                    const float4 G = S.geo[k];
                    const float4 C = S.col[k];
                    const float dy = G.y - py;
                    const float cq = (C.x * dy) * dy;
                    const float bdy = G.w * dy;
                    blend2_cut(G.x, G.z, bdy, cq, C.y, C.z, C.w, px, ar, ag, ab);
                }
            } else if ((any & ~fm) == 0) {
                for (int it = 0; it < maxlen; ++it) {
                    const int k = ml[8 * it];
                    const float4 G = S.geo[k];
                    const float4 C = S.col[k];
                    const float dy = G.y - py;
                    const float cq = (C.x * dy) * dy;
                    const float bdy = G.w * dy;
                    blend2_unit_fin(G.x, G.z, bdy, cq, C.y, C.z, C.w, px, ar, ag, ab);
                }
            } else {
                for (int it = 0; it < maxlen; ++it) {
                    const int k = ml[8 * it];
                    const float4 G = S.geo[k];
                    const float4 C = S.col[k];
                    const float dy = G.y - py;
                    const float cq = (C.x * dy) * dy;
                    const float bdy = G.w * dy;
                    blend2_unit(G.x, G.z, bdy, cq, C.y, C.z, C.w, px, ar, ag, ab);
                }
            }
            __builtin_amdgcn_wave_barrier();  // the next chunk rewrites the lists
            if (dense) __syncthreads();  // the next chunk overwrites the staging
            continue;
        }
        // the entries whose rectangle reaches this band, as a wave-uniform mask
        bool keep = false, fin = false;
        if (lane < cnt) {
            const unsigned rc = S.ro[lane];
            keep = rc != kNoRect && (int)((rc >> 12) & 15u) >= y_lo && (int)((rc >> 8) & 15u) <= y_hi;
            const float4 C = S.col[lane];
            fin = __builtin_isfinite(C.y) && __builtin_isfinite(C.z) && __builtin_isfinite(C.w);
        }
        unsigned long long m = __ballot(keep);
        if (kDiag && (A.diag & 4)) m = 0ull;  // diagnostic: no forward blending (wrong results)
        const unsigned long long fm = __ballot(fin);  // entries with a finite colour
        if (m && (m & ~fm) == 0) {
            // every colour finite (the rule): the select-free blend
            do {
                const int k = __builtin_ctzll(m);
                m &= m - 1ull;
                const float4 G = S.geo[k];
                const float4 C = S.col[k];
                const float dy = G.y - py;
                const float cq = (C.x * dy) * dy;
                const float bdy = G.w * dy;
                blend2_unit_fin(G.x, G.z, bdy, cq, C.y, C.z, C.w, px, ar, ag, ab);
            } while (m);
        } else if (m) {
            do {
                const int k = __builtin_ctzll(m);
                m &= m - 1ull;
                const float4 G = S.geo[k];
                const float4 C = S.col[k];
                const float dy = G.y - py;
                const float cq = (C.x * dy) * dy;
                const float bdy = G.w * dy;
                blend2_unit(G.x, G.z, bdy, cq, C.y, C.z, C.w, px, ar, ag, ab);
            } while (m);
        }
        if (dense) __syncthreads();  // the next chunk overwrites the staging
    }
    // dense: the sorted ids, kept for the backward (its partials overwrite
    // s_key) in the tile's own slab body, whose records it no longer reads
    int *kpark = reinterpret_cast<int *>(slab_rec(A.slab, A.ntiles, tile, kHeadSlots));  // 248 slots, contiguous
    if (dense)
        for (int j = tid; j < n; j += kBThreads) kpark[j] = s_key[j];
    if (kStamp && tid == 0) st[2] = tstamp();

    // 3. clamp, loss gradient (mse_loss backward: norm * (a - b); l1: norm * sgn),
    // clamp backward (passes where 0 <= out <= 1), error sums; v_out planes
    {
        const float o[3][2] = {{ar.x, ar.y}, {ag.x, ag.y}, {ab.x, ab.y}};
        float gt[3][2];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the targets' global_load_lds
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            gt[c][0] = sgt[(2 * c) * 64 + lane];
            gt[c][1] = sgt[(2 * c + 1) * 64 + lane];
        }
        float se = 0.f, ae = 0.f;
        float v[3][2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const bool inside = q < nin;
            float pse = 0.f, pae = 0.f;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float x = clamp_unit(o[c][q]);
                const float d = x - gt[c][q];
                pse = fmaf(d, d, pse);
                pae += fabsf(d);
                const float sg = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
                const float gv = A.loss_l1 ? A.norm * sg : A.norm * d;
                v[c][q] = (inside && o[c][q] >= 0.0f && o[c][q] <= 1.0f) ? gv : 0.0f;
            }
            if (inside) {
                se += pse;
                ae += pae;
            }
        }
        if (A.out) {  // optional clamped render (tests)
#pragma unroll
            for (int c = 0; c < 3; ++c)
                for (int q = 0; q < nin; ++q) A.out[c * hw + pix0 + q] = clamp_unit(o[c][q]);
        }
        const int p = prow * kVRow + pcol;
        __syncthreads();  // every wave has its targets: the planes take v_out
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            S.v[c][p] = v[c][0];
            S.v[c][p + 1] = v[c][1];
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            se += __shfl_xor(se, off, 64);
            ae += __shfl_xor(ae, off, 64);
        }
        if (lane == 0) {
            S.misc[2 * w] = __float_as_int(se);
            S.misc[2 * w + 1] = __float_as_int(ae);
        }
        __syncthreads();
        if (tid == 0) {
            const float2 e = make_float2(__int_as_float(S.misc[0]) + __int_as_float(S.misc[2]),
                                         __int_as_float(S.misc[1]) + __int_as_float(S.misc[3]));
            A.err[tile] = e;
        }
    }
    if (kStamp && tid == 0) st[3] = tstamp();

    if (kDiag && (A.diag & 2)) return;  // diagnostic: no backward (wrong results)
    // 4. backward, kBChunk entries at a time (sparse tiles: the forward's staging).
    // Each wave takes the rectangle rows of its own band -- the v_out rows it
    // wrote itself -- so the waves need no barrier until the chunk's flush.
    float *eacc = &S.part[0][0] + w * (8 * kBChunk);  // [8][kBChunk] entry sums per wave
    signed char *wown = S.own + w * 64;
    signed char *wperm = S.perm + w * 64;
    for (int c0 = 0; c0 < n; c0 += kBChunk) {
        const int gn = min(kBChunk, n - c0);
        if (dense) {
            __syncthreads();  // staging / entry-sum readers done
            // this chunk's keys, by rank, into the gid slots stage_chunk overwrites
            if (tid < gn) S.gid[tid] = kpark[c0 + tid];  // written by this workgroup after its forward
            __syncthreads();
            stage_chunk(S.gid, gn);
            __syncthreads();
        }
        // work items of entry `lane` in this band: one per rectangle row, two
        // halves when the row is wider than brun
        int items = 0, ilen = 0;
        unsigned rc = kNoRect;
        if (lane < gn) {
            rc = S.ro[lane];
            if (rc != kNoRect) {
                const int ry0 = max((int)((rc >> 8) & 15u), y_lo), ry1 = min((int)((rc >> 12) & 15u), y_hi);
                const int rw = (int)((rc >> 4) & 15u) - (int)(rc & 15u) + 1;
                if (ry0 <= ry1) {
                    items = (ry1 - ry0 + 1) * (rw > brun_of(A) ? 2 : 1);
                    ilen = rw > brun_of(A) ? (rw + 1) >> 1 : rw;
                }
            }
        }
        // the entries' items are laid out longest first (by class, stable), so a
        // round's 64 items -- whose pixel loop runs as long as its longest --
        // have similar lengths; each entry's sums are unchanged (its items
        // stay together, in row order)
        {
            const unsigned long long below = (1ull << lane) - 1ull;
            int rank = 0, seen = 0;
            unsigned long long left = __ballot(true);
            if (kDiag && (A.diag & 64)) {  // A/B: entry order
                rank = lane;
                left = 0ull;
            }
            // four length classes (9+, 7-8, 5-6, <= 4 and no items), entry
            // order within a class: most of an exact sort's gain for a quarter
            // of its VALU
            const int cls = ilen >= 9 ? 3 : (ilen >= 7 ? 2 : (ilen >= 5 ? 1 : 0));
            for (int L = 3; L >= 0 && left; --L) {
                const unsigned long long m = __ballot(cls == L);
                if (cls == L) rank = seen + __popcll(m & below);
                seen += __popcll(m);
                left &= ~m;
            }
            wperm[rank] = (signed char)lane;
        }
        __builtin_amdgcn_wave_barrier();
        // the chunk's geometry finite: the backward's alpha cut by threshold
        const bool bcut =
            __ballot(lane < gn && !geo_cut_ok(S.geo[lane], S.col[lane].x)) == 0ull;
        const int ent = wperm[lane];  // the entry in sorted slot `lane`
        const int sitems = __shfl(items, ent, 64);
        const int incl = wave_scan_dpp<false>(sitems, 0);
        const int off = incl - sitems;  // sorted slot `lane`'s first item
        const int total = __builtin_amdgcn_readlane(incl, 63);
#pragma unroll
        for (int c = 0; c < 8; ++c) eacc[c * kBChunk + lane] = 0.0f;
        // One round loop per alpha-cut variant (bcut: the chunk's, wave-uniform),
        // and the lanes without pixel work -- past the last item, or a row below
        // the image -- walking an empty range and selecting zeros: with the
        // variant branch and the validity branches inside the loop, the
        // compiler kept the two walks' sums and the zero-filled sums in
        // different registers and moved them back every round (ISA: 83
        // v_mov_b32 of 337 VALU per round).  Same sums bit for bit.
        auto rounds = [&](auto kcut) {
            for (int base = 0; base < total; base += 64) {
                // the entry of item base + lane: the last entry whose first item is <= it
                wown[lane] = -1;
                __builtin_amdgcn_wave_barrier();
                if (sitems > 0 && off >= base && off < base + 64) wown[off - base] = (signed char)lane;
                const int straddle = __popcll(__ballot(lane < gn && off <= base)) - 1;
                __builtin_amdgcn_wave_barrier();
                int slot = max((int)wown[lane], straddle);
                slot = wave_scan_dpp<true>(slot, -2147483647 - 1);  // sorted slot of item base + lane
                const int item = base + lane;
                // the entry, its first item and rectangle
                const int own = __shfl(ent, slot, 64);
                const int eoff = __shfl(off, slot, 64);
                const unsigned ro = (unsigned)__shfl((int)rc, own, 64);
                const float4 G = S.geo[own], C = S.col[own];
                const int j = item - eoff;  // item index within the entry
                const int rx0 = (int)(ro & 15u), rx1 = (int)((ro >> 4) & 15u);
                const int rwid = rx1 - rx0 + 1;
                const int ipr = rwid > brun_of(A) ? 2 : 1;
                const int jr = ipr == 1 ? j : (j >> 1);
                const int row = max((int)((ro >> 8) & 15u), y_lo) + jr;
                const int half = (rwid + 1) >> 1;
                const int cs = ipr == 1 ? rx0 : rx0 + half * (j & 1);
                const int ce = min(ipr == 1 ? rx1 : min(cs + half - 1, rx1), A.img_w - 1 - (int)tx0);
                const float pyf = ty0 + (float)row;
                // diag 8: no pixel work
                const bool rowok = item < total && (int)pyf < A.img_h && !(kDiag && (A.diag & 8));
                const float ex = G.x, eha = G.z, eb = G.w;
                const float dy = G.y - pyf;
                const float cq = (C.x * dy) * dy;  // splat_sigma_h's row terms
                const float bdy = eb * dy;
                // dy is constant along the item's row, so the per-pixel sums of
                // backward.cu:822-848 factor: v_conic = 1/2 (S2, dy S1, dy^2 S0),
                // v_xy = (2 ha S1 + b dy S0, b S1 + 2 c dy S0) with S_k = sum
                // v_sigma dx^k -- 4 VALU per pixel instead of 11
                float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
                float g[8];
                g[5] = 0.0f;
                g[6] = 0.0f;
                g[7] = 0.0f;
                // walk the row by its v_out word (the planes at fixed LDS
                // offsets) with dx stepping by -1 (exact: ex - px is exact or,
                // far off, rounds alike); a lane without pixel work: no trip
                const float *vp = &S.v[0][0] + row * kVRow + cs;
                const float *const ve = rowok ? &S.v[0][0] + row * kVRow + ce : vp - 1;
                float dx = ex - (tx0 + (float)cs);
                // kCut: the chunk's geometry is finite, so the alpha cut is the
                // sigma threshold and alpha = vis (kSigmaCutBits); else the
                // reference's test as written
                for (; vp <= ve; ++vp, dx -= 1.0f) {
                    float Px, Py, Pz;
                    if (kDiag && (A.diag & 256)) {  // diag 256: no v_out reads (wrong)
                        Px = dx;
                        Py = 0.5f * dx;
                        Pz = bdy;
                    } else {
                        Px = vp[0];
                        Py = vp[kTile * kVRow];
                        Pz = vp[2 * kTile * kVRow];
                    }
                    const float sgm = fmaf(fmaf(eha, dx, bdy), dx, cq);
                    const float vis = exp_neg(sgm);
                    float al;
                    if constexpr (decltype(kcut)::value) {
                        // a failing pixel adds exact zeros (a select, not a branch:
                        // the same sums bit for bit, without the exec-mask
                        // bookkeeping per pixel -- bench.py 18.39k vs 18.21k it/s,
                        // tile kernel 45.5 vs 45.8 us, product libraries swapped on
                        // one box, profiles/r06/select_cut/)
                        al = __float_as_uint(sgm) <= kSigmaCutBits ? vis : 0.0f;
                        const float v_alpha = fmaf(C.w, Pz, fmaf(C.z, Py, C.y * Px));
                        const float v_sigma = (-al) * v_alpha;
                        g[5] = fmaf(al, Px, g[5]);
                        g[6] = fmaf(al, Py, g[6]);
                        g[7] = fmaf(al, Pz, g[7]);
                        s0 += v_sigma;
                        const float vdx = v_sigma * dx;
                        s1 += vdx;
                        s2 = fmaf(vdx, dx, s2);
                        continue;
                    } else {
                        al = fminf(1.0f, vis);  // opacity 1
                        if (sgm < 0.0f || al < kAlphaMin) continue;
                    }
                    const float v_alpha = fmaf(C.w, Pz, fmaf(C.z, Py, C.y * Px));
                    const float v_sigma = (-vis) * v_alpha;  // (-opacity * vis) * v_alpha
                    g[5] = fmaf(al, Px, g[5]);
                    g[6] = fmaf(al, Py, g[6]);
                    g[7] = fmaf(al, Pz, g[7]);
                    s0 += v_sigma;
                    const float vdx = v_sigma * dx;
                    s1 += vdx;
                    s2 = fmaf(vdx, dx, s2);
                }
                // (pixel PAIRS with packed math -- 3 two-word LDS reads, 2 exps and
                // ~23 VALU per pair instead of ~34 per two pixels -- were measured,
                // round 6: 49.8 vs 45.9 us per tile-kernel launch in bench.py,
                // product libraries swapped on one box; 64 VGPRs with 60-72 B of
                // spills, or 72 VGPRs at 7 waves per SIMD: 48.2;
                // profiles/r06/tile_pairs/)
                const float hdy = 0.5f * dy;
                g[0] = rowok ? fmaf(2.0f * eha, s1, bdy * s0) : 0.0f;
                g[1] = rowok ? fmaf(eb, s1, ((2.0f * C.x) * dy) * s0) : 0.0f;
                g[2] = rowok ? 0.5f * s2 : 0.0f;
                g[3] = rowok ? hdy * s1 : 0.0f;
                g[4] = rowok ? (hdy * dy) * s0 : 0.0f;
                // segmented sums over the runs of items of one entry: the last item
                // of an entry's run holds the run's sum (fixed tree order) and adds
                // it to the entry's (a fixed order: rounds in sequence).  Measured
                // alternatives: every item adding its sums with LDS float atomics
                // (2.9x slower kernel: the LDS serialises an entry's items); a
                // packed two-pixel loop (80 VGPRs, 6 waves per SIMD: 64.0 vs 58.5
                // us).  An entry has at most 8 items in a band unless rows split
                // in two (brun < 16): runs of <= 8 lanes need no row_shr:8 step (a
                // run crossing a 16-lane row still takes the row broadcast)
                if (!(kDiag && (A.diag & 16))) {  // diag 16: no run sums (wrong)
                    if (brun_of(A) < 16)
                        wave_seg_sums<8, true>(g, own);
                    else
                        wave_seg_sums<8, false>(g, own);
                }
                const int own_next = __shfl_down(own, 1, 64);
                if (item < total && (lane == 63 || item + 1 == total || own_next != own)) {
#pragma unroll
                    for (int c = 0; c < 8; ++c) eacc[c * kBChunk + own] += g[c];
                }
                __builtin_amdgcn_wave_barrier();
            }
        };
        if (bcut)
            rounds(std::true_type{});
        else
            rounds(std::false_type{});
        __syncthreads();
        // 8 lanes per entry add the entry's sums (band 0 + band 1) into the
        // splat's gradient record
        if (kDet) {
            // deterministic: one 32-byte partial per (splat, tile) at the tile's
            // place in the splat's bbox; the splat kernel sums them in bbox order
            for (int q = tid; q < gn * 8; q += kBThreads) {
                const int e = q >> 3, c = q & 7;
                const float *ea = &S.part[0][0];
                const float v = ea[c * kBChunk + e] + ea[8 * kBChunk + c * kBChunk + e];
                const int g = S.gid[e];
                const long long slot = det_slot(A.det_off, A.xys, A.radii, g, tx, ty, A.tbx,
                                                (A.img_h + kTile - 1) / kTile);
                if (slot < A.det_cap)
                    reinterpret_cast<float *>(A.det_part)[8 * slot + c] = v;
                else
                    unsafeAtomicAdd(A.grad + (size_t)g * 16 + c, v);
            }
        } else {
            for (int q = tid; q < gn * 8 && !(kDiag && (A.diag & 32)); q += kBThreads) {  // diag 32: no atomics
                const int e = q >> 3, c = q & 7;
                const float *ea = &S.part[0][0];
                unsafeAtomicAdd(A.grad + (size_t)S.gid[e] * 16 + c,
                                ea[c * kBChunk + e] + ea[8 * kBChunk + c * kBChunk + e]);
            }
        }
    }
    if (kStamp && tid == 0) {
        st[4] = tstamp();
        st[5] = tstamp();
        st[6] = n_all;  // the tile's entry count, for per-density breakdowns
    }
}

struct TrainSplatArgs {
    int n, ntiles, rgbw_train, update;
    float hw, hh;
    double inv_count;
    float *xyz, *chol, *feat, *rgbw;
    const float *chol_bound;
    int *radii;
    float4 *rec;
    float4 *grad;        // [N][4]
    float *state[4][4];  // [xyz, chol, feat, rgb_w][exp_avg, exp_avg_sq, exp_avg_diff, neg_pre_grad]
    int first[4];        // the parameter's first Adan step (optimizer.py:187-189)
    AdanScalars S;
    float *grads_out;    // update == 0: [N, 9] = d_xyz 2, d_chol 3, d_feat 3, d_rgbw 1
    const float2 *err;
    float *loss;         // [2]: mean squared error, mean absolute error
    unsigned loss_seq;   // non-zero: stored into word 2 of ``loss`` after the losses
    // GSVC_TRAIN_DETERMINISTIC: splat i's gradient = its partials
    // det_part[det_off[i] .. det_off[i + 1]) summed in order (+ the record's
    // atomics of slots past det_cap, zero otherwise)
    const int *det_off;
    const float4 *det_part;
    long long det_cap;
    // GSVC_TRAIN_CARRY: after its update the splat projects itself for the next
    // frame (rec, xys, radii, its tile box cbox; its gradient record zeroed)
    // and, when the box leaves the hull of the boxes it was binned under
    // (chull), appends its id to the tiles the grown hull adds (cids, ccount);
    // its box area goes into the next frame's M (m_next)
    int carry, tbx, tby;
    float2 *xys;
    uint2 *cbox, *chull;
    unsigned *ccount;
    int *cids;
    int *m_next;
    long long *stamps;  // diagnostic: int64[waves][8]
    int split;          // two waves per 64 splats (splat_step_split); 0: one lane per splat
};

// GSVC_TRAIN_CARRY: splat i's projection for the next frame from its updated
// parameters p = {xyz 2, cholesky 3, features 3, rgb_w} -- load_project's op
// sequence (frame_dev.h), so the record bits equal a projection kernel's --
// and the upkeep of its carried bins.  Returns its box area (its share of M).
__device__ __forceinline__ int carry_splat(const TrainSplatArgs &A, int i, const float (&p)[9],
                                           uint2 h) {
    const float mx = tanhf(p[0]), my = tanhf(p[1]);
    float l11 = p[2], l21 = p[3], l22 = p[4];
    if (A.chol_bound) {
        l11 = l11 + A.chol_bound[0];
        l21 = l21 + A.chol_bound[1];
        l22 = l22 + A.chol_bound[2];
    }
    float r = p[5], g = p[6], b = p[7];
    if (A.rgbw) {
        r = r * p[8];
        g = g * p[8];
        b = b * p[8];
    }
    const SplatOut S = splat_out(i, mx, my, l11, l21, l22, r, g, b, 1.0f, A.hw, A.hh, A.tbx, A.tby);
    A.rec[3 * i] = S.r0;
    A.xys[i] = S.P.xy;
    A.radii[i] = S.P.rad;
    // the record's first 32 bytes (v_xy, v_conic, v_colors: what the tile
    // kernel adds and this kernel reads; v_opacity and the padding stay as a
    // projection zeroed them -- nothing in the fused step writes them)
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    A.grad[4 * i] = z;
    A.grad[4 * i + 1] = z;
    A.rec[3 * i + 1] = S.r1;
    A.rec[3 * i + 2] = S.r2;
    unsigned x0 = 0, y0 = 0, x1 = 0, y1 = 0;
    if (S.P.rad > 0) tile_bbox(S.P.xy.x, S.P.xy.y, (float)S.P.rad, A.tbx, A.tby, x0, y0, x1, y1);
    const uint2 nb = pack_box(x0, y0, x1, y1);
    A.cbox[i] = nb;
    if (nb.x == nb.y) return 0;  // empty
    const bool hv = h.x != h.y;
    const unsigned hx0 = h.x & 0xffffu, hy0 = h.x >> 16, hx1 = h.y & 0xffffu, hy1 = h.y >> 16;
    if (!hv || x0 < hx0 || y0 < hy0 || x1 > hx1 || y1 > hy1) {
        // the grown hull; its new tiles get the id (the hull's own tiles have it)
        const unsigned ux0 = hv ? min(x0, hx0) : x0, uy0 = hv ? min(y0, hy0) : y0;
        const unsigned ux1 = hv ? max(x1, hx1) : x1, uy1 = hv ? max(y1, hy1) : y1;
        for (unsigned y = uy0; y < uy1; ++y)
            for (unsigned x = ux0; x < ux1; ++x) {
                if (hv && x >= hx0 && x < hx1 && y >= hy0 && y < hy1) continue;
                const unsigned t = y * (unsigned)A.tbx + x;
                const unsigned sl = atomicAdd(A.ccount + t, 1u);
                if (sl < (unsigned)kTrainCarryCap) A.cids[(size_t)t * kTrainCarryCap + sl] = i;
            }
        A.chull[i] = pack_box(ux0, uy0, ux1, uy1);
    }
    return (int)((x1 - x0) * (y1 - y0));
}

// Row i of a [N, C] float tensor (C = 1, 2, 3) as one vector access.
struct Row3 {
    float x, y, z;
};
template <int C>
__device__ __forceinline__ void ld_row(const float *base, int i, float *out) {
    const float *p = base + (size_t)C * (size_t)i;
    if constexpr (C == 2) {
        const float2 t = *reinterpret_cast<const float2 *>(p);
        out[0] = t.x;
        out[1] = t.y;
    } else if constexpr (C == 3) {
        const Row3 t = *reinterpret_cast<const Row3 *>(p);
        out[0] = t.x;
        out[1] = t.y;
        out[2] = t.z;
    } else {
        out[0] = p[0];
    }
}
template <int C>
__device__ __forceinline__ void st_row(float *base, int i, const float *in) {
    float *p = base + (size_t)C * (size_t)i;
    if constexpr (C == 2) {
        *reinterpret_cast<float2 *>(p) = make_float2(in[0], in[1]);
    } else if constexpr (C == 3) {
        *reinterpret_cast<Row3 *>(p) = Row3{in[0], in[1], in[2]};
    } else {
        p[0] = in[0];
    }
}

// Diagnostic (gsvc_debug_set(5, 4) with gsvc_debug_set_ptr): s_memrealtime
// stamps per wave by lane 0 -- start, operands landed, Adan stores issued,
// carry done, M added, stores acknowledged -- as int64[8] at st.
__device__ __forceinline__ void splat_stamp(long long *st, int k) {
    if (st) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const long long t = tstamp();
        if ((threadIdx.x & 63) == 0) st[k] = t;
    }
}

// One splat's step: the projection VJP, activation VJPs and the Adan update of
// its elements (update == 0: the gradients into grads_out).  st: stamps
// (kStamp instances only).
template <bool kStamp>
__device__ __forceinline__ int splat_step(const TrainSplatArgs &A, int i, long long *st) {
    // Every operand is loaded up front, before any arithmetic: one round trip
    // per lane instead of three (gradient + radius -> record -> Adan state).
    // rec is written for every splat by the projection, so its load needs no
    // radius test; a first step's neg_pre_grad is loaded and ignored.
    float4 g0 = A.grad[4 * i];      // v_xy.x, v_xy.y, v_conic 0, v_conic 1
    float4 g1 = A.grad[4 * i + 1];  // v_conic 2, v_colors r g b
    if (A.det_off) {
        // the splat's (splat, tile) partials in bbox row-major order, then the
        // overflow atomics (zero unless det_cap was too small)
        const long long b = A.det_off[i], e = min((long long)A.det_off[i + 1], A.det_cap);
        float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
        for (long long k = b; k < e; ++k) {
            const float4 p0 = A.det_part[2 * k], p1 = A.det_part[2 * k + 1];
            s0.x += p0.x; s0.y += p0.y; s0.z += p0.z; s0.w += p0.w;
            s1.x += p1.x; s1.y += p1.y; s1.z += p1.z; s1.w += p1.w;
        }
        g0 = make_float4(s0.x + g0.x, s0.y + g0.y, s0.z + g0.z, s0.w + g0.w);
        g1 = make_float4(s1.x + g1.x, s1.y + g1.y, s1.z + g1.z, s1.w + g1.w);
    }
    const float4 r0 = A.rec[3 * i], r2 = A.rec[3 * i + 2];
    const int rad = A.radii[i];
    const float c0 = A.chol[3 * i], c1 = A.chol[3 * i + 1], c2 = A.chol[3 * i + 2];
    const float x0 = A.xyz[2 * i], x1 = A.xyz[2 * i + 1];
    const float f0 = A.feat[3 * i], f1 = A.feat[3 * i + 1], f2 = A.feat[3 * i + 2];
    const float w = A.rgbw ? A.rgbw[i] : 1.0f;
    // the carry's hull, with the other operands (not a round trip after the update)
    const uint2 hull = A.carry ? A.chull[i] : make_uint2(0u, 0u);
    if (kStamp) splat_stamp(st, 1);
    const bool upd = A.update != 0;
    // Adan state rows, one vector access per (tensor, splat): xyz e 0-1, cholesky
    // 2-4, features 5-7, rgb_W 8 (a row of 2 or 3 floats is one dwordx2 / x3)
    float m[9], v[9], df[9], npg[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) m[e] = v[e] = df[e] = npg[e] = 0.0f;
    if (upd) {
        ld_row<2>(A.state[0][0], i, m);
        ld_row<2>(A.state[0][1], i, v);
        ld_row<2>(A.state[0][2], i, df);
        ld_row<2>(A.state[0][3], i, npg);
        ld_row<3>(A.state[1][0], i, m + 2);
        ld_row<3>(A.state[1][1], i, v + 2);
        ld_row<3>(A.state[1][2], i, df + 2);
        ld_row<3>(A.state[1][3], i, npg + 2);
        ld_row<3>(A.state[2][0], i, m + 5);
        ld_row<3>(A.state[2][1], i, v + 5);
        ld_row<3>(A.state[2][2], i, df + 5);
        ld_row<3>(A.state[2][3], i, npg + 5);
        if (A.rgbw_train) {
            ld_row<1>(A.state[3][0], i, m + 8);
            ld_row<1>(A.state[3][1], i, v + 8);
            ld_row<1>(A.state[3][2], i, df + 8);
            ld_row<1>(A.state[3][3], i, npg + 8);
        }
    }
    // 2D projection VJP, backward2d.cu:8-51 (the op's project2d_bwd_kernel sequence)
    float vl0 = 0.f, vl1 = 0.f, vl2 = 0.f, vmx = 0.f, vmy = 0.f;
    float l11 = c0, l21 = c1, l22 = c2;
    if (A.chol_bound) {
        l11 = l11 + A.chol_bound[0];
        l21 = l21 + A.chol_bound[1];
        l22 = l22 + A.chol_bound[2];
    }
    if (rad > 0) {
        const float X00 = r2.z, X01 = r0.w, X10 = X01, X11 = r2.w;
        const float G00 = g0.z, G01 = g0.w, G10 = G01, G11 = g1.x;
        const float N00 = -X00, N01 = -X01, N10 = -X10, N11 = -X11;
        const float P00 = N00 * G00 + N10 * G01;
        const float P01 = N01 * G00 + N11 * G01;
        const float P10 = N00 * G10 + N10 * G11;
        const float P11 = N01 * G10 + N11 * G11;
        const float V00 = P00 * X00 + P10 * X01;
        const float V01 = P01 * X00 + P11 * X01;
        const float V10 = P00 * X10 + P10 * X11;
        const float V11 = P01 * X10 + P11 * X11;
        const float g11 = V00, g12 = V10 + V01, g22 = V11;
        vl0 = 2.0f * l11 * g11 + 2.0f * g12 * l21;  // doubled cross term: backward2d.cu:39
        vl1 = 2.0f * l11 * g12 + 2.0f * l21 * g22;
        vl2 = 2.0f * l22 * g22;
        vmx = g0.x * A.hw;
        vmy = g0.y * A.hh;
    }
    // activations (GaussianSplats_Represent.py:57-70): tanh, + bound, * rgb_W
    const float t0 = tanhf(x0), t1 = tanhf(x1);
    const float dx0 = vmx * (1.0f - t0 * t0), dx1 = vmy * (1.0f - t1 * t1);
    const float df0 = g1.y * w, df1 = g1.z * w, df2 = g1.w * w;
    const float dw = (g1.y * f0 + g1.z * f1) + g1.w * f2;
    if (!upd) {
        float *o = A.grads_out + 9 * (size_t)i;
        o[0] = dx0;
        o[1] = dx1;
        o[2] = vl0;
        o[3] = vl1;
        o[4] = vl2;
        o[5] = df0;
        o[6] = df1;
        o[7] = df2;
        o[8] = A.rgbw_train ? dw : 0.0f;
        return 0;
    }
    // Adan on the 8 (9 with rgb_W) elements of this splat
    const float g[9] = {dx0, dx1, vl0, vl1, vl2, df0, df1, df2, dw};
    const float pin[9] = {x0, x1, c0, c1, c2, f0, f1, f2, w};
    float pnew[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) {
        const int q = e < 2 ? 0 : (e < 5 ? 1 : (e < 8 ? 2 : 3));
        pnew[e] = pin[e];
        if (q == 3 && !A.rgbw_train) continue;
        if (A.first[q]) npg[e] = -(g[e] * A.S.clip);
        pnew[e] = adan_update(A.S, pin[e], g[e], m[e], v[e], df[e], npg[e]);
    }
    // the rows back, one vector store per (tensor, splat)
    st_row<2>(A.xyz, i, pnew);
    st_row<2>(A.state[0][0], i, m);
    st_row<2>(A.state[0][1], i, v);
    st_row<2>(A.state[0][2], i, df);
    st_row<2>(A.state[0][3], i, npg);
    st_row<3>(A.chol, i, pnew + 2);
    st_row<3>(A.state[1][0], i, m + 2);
    st_row<3>(A.state[1][1], i, v + 2);
    st_row<3>(A.state[1][2], i, df + 2);
    st_row<3>(A.state[1][3], i, npg + 2);
    st_row<3>(A.feat, i, pnew + 5);
    st_row<3>(A.state[2][0], i, m + 5);
    st_row<3>(A.state[2][1], i, v + 5);
    st_row<3>(A.state[2][2], i, df + 5);
    st_row<3>(A.state[2][3], i, npg + 5);
    if (A.rgbw_train) {
        st_row<1>(A.rgbw, i, pnew + 8);
        st_row<1>(A.state[3][0], i, m + 8);
        st_row<1>(A.state[3][1], i, v + 8);
        st_row<1>(A.state[3][2], i, df + 8);
        st_row<1>(A.state[3][3], i, npg + 8);
    }
    if (kStamp) splat_stamp(st, 2);
    const int hits = A.carry ? carry_splat(A, i, pnew, hull) : 0;
    if (kStamp) splat_stamp(st, 3);
    return hits;
}

// splat_step over two waves per 64 splats (256-thread workgroups: 128
// splats, waves 0 / 2 their geometry halves, 1 / 3 their colour halves): the
// colour wave loads the colour gradient, the features, rgb_W and their Adan
// rows, updates them and hands the new values over LDS; the geometry wave
// does the projection VJP, the xyz / cholesky Adan elements and, after the
// barrier, the carry (it needs all nine new values).  The same op sequence
// per element as splat_step, so the same bits; twice the waves, each with
// about half the loads and Adan work (782 one-wave latency chains on 1024
// SIMDs were the kernel).  The deterministic mode's partial sums
// are split the same way (each half its components, in splat_step's order).
__device__ __forceinline__ int splat_step_split(const TrainSplatArgs &A, int base) {
    __shared__ float s_cp[2][4][64];  // per splat group: new feature r g b, rgb_W
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, grp = w >> 1;
    const int i = base + grp * 64 + lane;
    const bool have = i < A.n;
    const int ic = have ? i : 0;  // loads of lanes past n: splat 0, unused
    const bool upd = A.update != 0;
    int hits = 0;
    float pnew[5];
    uint2 hull = make_uint2(0u, 0u);
    // GSVC_TRAIN_DETERMINISTIC: the splat's (splat, tile) partials in bbox
    // order plus the record's atomics, each half summing its own components in
    // splat_step's order (the same bits per component)
    long long db = 0, de = 0;
    if (A.det_off && have) {
        db = A.det_off[i];
        de = min((long long)A.det_off[i + 1], A.det_cap);
    }
    // (measured, round 5, and not kept: the xyz elements on the colour wave,
    // and both waves projecting with each its share of the carry's stores --
    // both within the noise; profiles/r05/splat_split/)
    if (w & 1) {
        // colour half: elements 5-7 (features) and 8 (rgb_W)
        float4 g1 = A.grad[4 * ic + 1];  // v_conic 2, v_colors r g b
        if (A.det_off) {
            float sy = 0.f, sz = 0.f, sw = 0.f;
            for (long long k = db; k < de; ++k) {
                const float4 p1 = A.det_part[2 * k + 1];
                sy += p1.y;
                sz += p1.z;
                sw += p1.w;
            }
            g1.y = sy + g1.y;
            g1.z = sz + g1.z;
            g1.w = sw + g1.w;
        }
        const float f0 = A.feat[3 * ic], f1 = A.feat[3 * ic + 1], f2 = A.feat[3 * ic + 2];
        const float wv = A.rgbw ? A.rgbw[ic] : 1.0f;
        float m[4], v[4], df[4], npg[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) m[e] = v[e] = df[e] = npg[e] = 0.0f;
        if (upd) {
            ld_row<3>(A.state[2][0], ic, m);
            ld_row<3>(A.state[2][1], ic, v);
            ld_row<3>(A.state[2][2], ic, df);
            ld_row<3>(A.state[2][3], ic, npg);
            if (A.rgbw_train) {
                ld_row<1>(A.state[3][0], ic, m + 3);
                ld_row<1>(A.state[3][1], ic, v + 3);
                ld_row<1>(A.state[3][2], ic, df + 3);
                ld_row<1>(A.state[3][3], ic, npg + 3);
            }
        }
        const float df0 = g1.y * wv, df1 = g1.z * wv, df2 = g1.w * wv;
        const float dw = (g1.y * f0 + g1.z * f1) + g1.w * f2;
        float pc[4] = {f0, f1, f2, wv};
        if (!upd) {
            if (have) {
                float *o = A.grads_out + 9 * (size_t)i;
                o[5] = df0;
                o[6] = df1;
                o[7] = df2;
                o[8] = A.rgbw_train ? dw : 0.0f;
            }
        } else {
            const float g[4] = {df0, df1, df2, dw};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int q = e < 3 ? 2 : 3;
                if (q == 3 && !A.rgbw_train) continue;
                if (A.first[q]) npg[e] = -(g[e] * A.S.clip);
                pc[e] = adan_update(A.S, pc[e], g[e], m[e], v[e], df[e], npg[e]);
            }
            if (have) {
                st_row<3>(A.feat, i, pc);
                st_row<3>(A.state[2][0], i, m);
                st_row<3>(A.state[2][1], i, v);
                st_row<3>(A.state[2][2], i, df);
                st_row<3>(A.state[2][3], i, npg);
                if (A.rgbw_train) {
                    st_row<1>(A.rgbw, i, pc + 3);
                    st_row<1>(A.state[3][0], i, m + 3);
                    st_row<1>(A.state[3][1], i, v + 3);
                    st_row<1>(A.state[3][2], i, df + 3);
                    st_row<1>(A.state[3][3], i, npg + 3);
                }
            }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) s_cp[grp][e][lane] = pc[e];
    } else {
        // geometry half: elements 0-1 (xyz) and 2-4 (cholesky)
        float4 g0 = A.grad[4 * ic];      // v_xy.x, v_xy.y, v_conic 0, v_conic 1
        float g1x = A.grad[4 * ic + 1].x;  // v_conic 2
        if (A.det_off) {
            float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f);
            float sx = 0.f;
            for (long long k = db; k < de; ++k) {
                const float4 p0 = A.det_part[2 * k];
                s0.x += p0.x; s0.y += p0.y; s0.z += p0.z; s0.w += p0.w;
                sx += A.det_part[2 * k + 1].x;
            }
            g0 = make_float4(s0.x + g0.x, s0.y + g0.y, s0.z + g0.z, s0.w + g0.w);
            g1x = sx + g1x;
        }
        const float4 r0 = A.rec[3 * ic], r2 = A.rec[3 * ic + 2];
        const int rad = A.radii[ic];
        const float c0 = A.chol[3 * ic], c1 = A.chol[3 * ic + 1], c2 = A.chol[3 * ic + 2];
        const float x0 = A.xyz[2 * ic], x1 = A.xyz[2 * ic + 1];
        hull = A.carry ? A.chull[ic] : make_uint2(0u, 0u);
        float m[5], v[5], df[5], npg[5];
#pragma unroll
        for (int e = 0; e < 5; ++e) m[e] = v[e] = df[e] = npg[e] = 0.0f;
        if (upd) {
            ld_row<2>(A.state[0][0], ic, m);
            ld_row<2>(A.state[0][1], ic, v);
            ld_row<2>(A.state[0][2], ic, df);
            ld_row<2>(A.state[0][3], ic, npg);
            ld_row<3>(A.state[1][0], ic, m + 2);
            ld_row<3>(A.state[1][1], ic, v + 2);
            ld_row<3>(A.state[1][2], ic, df + 2);
            ld_row<3>(A.state[1][3], ic, npg + 2);
        }
        // 2D projection VJP, backward2d.cu:8-51 (splat_step's sequence)
        float vl0 = 0.f, vl1 = 0.f, vl2 = 0.f, vmx = 0.f, vmy = 0.f;
        float l11 = c0, l21 = c1, l22 = c2;
        if (A.chol_bound) {
            l11 = l11 + A.chol_bound[0];
            l21 = l21 + A.chol_bound[1];
            l22 = l22 + A.chol_bound[2];
        }
        if (rad > 0) {
            const float X00 = r2.z, X01 = r0.w, X10 = X01, X11 = r2.w;
            const float G00 = g0.z, G01 = g0.w, G10 = G01, G11 = g1x;
            const float N00 = -X00, N01 = -X01, N10 = -X10, N11 = -X11;
            const float P00 = N00 * G00 + N10 * G01;
            const float P01 = N01 * G00 + N11 * G01;
            const float P10 = N00 * G10 + N10 * G11;
            const float P11 = N01 * G10 + N11 * G11;
            const float V00 = P00 * X00 + P10 * X01;
            const float V01 = P01 * X00 + P11 * X01;
            const float V10 = P00 * X10 + P10 * X11;
            const float V11 = P01 * X10 + P11 * X11;
            const float g11 = V00, g12 = V10 + V01, g22 = V11;
            vl0 = 2.0f * l11 * g11 + 2.0f * g12 * l21;
            vl1 = 2.0f * l11 * g12 + 2.0f * l21 * g22;
            vl2 = 2.0f * l22 * g22;
            vmx = g0.x * A.hw;
            vmy = g0.y * A.hh;
        }
        const float t0 = tanhf(x0), t1 = tanhf(x1);
        const float dx0 = vmx * (1.0f - t0 * t0), dx1 = vmy * (1.0f - t1 * t1);
        pnew[0] = x0;
        pnew[1] = x1;
        pnew[2] = c0;
        pnew[3] = c1;
        pnew[4] = c2;
        if (!upd) {
            if (have) {
                float *o = A.grads_out + 9 * (size_t)i;
                o[0] = dx0;
                o[1] = dx1;
                o[2] = vl0;
                o[3] = vl1;
                o[4] = vl2;
            }
        } else {
            const float g[5] = {dx0, dx1, vl0, vl1, vl2};
#pragma unroll
            for (int e = 0; e < 5; ++e) {
                const int q = e < 2 ? 0 : 1;
                if (A.first[q]) npg[e] = -(g[e] * A.S.clip);
                pnew[e] = adan_update(A.S, pnew[e], g[e], m[e], v[e], df[e], npg[e]);
            }
            if (have) {
                st_row<2>(A.xyz, i, pnew);
                st_row<2>(A.state[0][0], i, m);
                st_row<2>(A.state[0][1], i, v);
                st_row<2>(A.state[0][2], i, df);
                st_row<2>(A.state[0][3], i, npg);
                st_row<3>(A.chol, i, pnew + 2);
                st_row<3>(A.state[1][0], i, m + 2);
                st_row<3>(A.state[1][1], i, v + 2);
                st_row<3>(A.state[1][2], i, df + 2);
                st_row<3>(A.state[1][3], i, npg + 2);
            }
        }
    }
    __syncthreads();
    if (have && upd && A.carry && !(w & 1)) {
        const float p[9] = {pnew[0], pnew[1], pnew[2], pnew[3], pnew[4], s_cp[grp][0][lane],
                            s_cp[grp][1][lane], s_cp[grp][2][lane], s_cp[grp][3][lane]};
        hits = carry_splat(A, i, p, hull);
    }
    return hits;
}

template <bool kStamp, int kBlock = 256>
__global__ __launch_bounds__(kBlock) void train_splat_kernel(TrainSplatArgs A) {
    long long *st = kStamp ? A.stamps + 8 * (size_t)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6))
                           : nullptr;
    if (kStamp && (threadIdx.x & 63) == 0) st[0] = tstamp();
    if (blockIdx.x == 0) {
        // the first workgroup (no splats): the loss; dispatched first so it
        // runs beside the splats
        __shared__ double s_l[2][4];
        publish_loss<kBlock>(A.err, A.ntiles, A.inv_count, A.loss, A.loss_seq, A.det_off, A.n, s_l);
        if (kStamp) splat_stamp(st, 5);
        return;
    }
    int hits;
    if (!kStamp && kBlock == 256 && A.split) {
        hits = splat_step_split(A, (blockIdx.x - 1) * (kBlock / 2));
    } else {
        const int t = (blockIdx.x - 1) * blockDim.x + threadIdx.x;
        hits = t < A.n ? splat_step<kStamp>(A, t, st) : 0;
    }
    if (A.carry == 2) {
        // the next frame's M is read only as M >= 1 (the tile kernel's background
        // branch, rasterize_sum.py:121-127): one plain store of 1 per wave that
        // has tiles, instead of a per-workgroup device-scope atomic add -- those
        // all go to one address and serialise at the memory side (~5 us of the
        // kernel at 196 workgroups, ~20 us at 782)
        if (__ballot(hits > 0) != 0ull && (threadIdx.x & 63) == 0) *A.m_next = 1;
    } else if (A.carry) {
        __shared__ int s_hits[4];
        add_hits(hits, s_hits, A.m_next);  // the next frame's M
    }
    if (kStamp) {
        if ((threadIdx.x & 63) == 0) st[4] = tstamp();
        splat_stamp(st, 5);
    }
}

struct TrainWs {
    FrameWs f;  // with the splat order buffers (GSVC_TRAIN_ORDER)
    float4 *grad;
    float2 *err;
    // GSVC_TRAIN_CARRY: per tile its candidate ids and their count, per splat
    // its current tile box and the hull of the boxes it is binned under
    int *cids;
    unsigned *ccount, *csorted;  // csorted: TrainTileArgs.csorted, right after ccount
    uint2 *cbox, *chull;
    size_t bytes;
};

static TrainWs train_ws(char *base, int n, int ntiles) {
    TrainWs w;
    w.f = frame_ws(base, n, ntiles);
    size_t off = w.f.bytes;
    const size_t nn = (size_t)(n > 0 ? n : 1), nt = (size_t)(ntiles > 0 ? ntiles : 1);
    auto take = [&](size_t bytes) {
        char *p = base ? base + off : nullptr;
        off += ws_align(bytes);
        return p;
    };
    w.grad = (float4 *)take(sizeof(float4) * 4 * nn);
    w.err = (float2 *)take(sizeof(float2) * nt);
    w.cids = (int *)take(sizeof(int) * kTrainCarryCap * nt);
    w.ccount = (unsigned *)take(sizeof(unsigned) * 2 * nt);  // ccount[T], csorted[T]
    w.csorted = w.ccount ? w.ccount + nt : nullptr;
    w.cbox = (uint2 *)take(sizeof(uint2) * nn);
    w.chull = (uint2 *)take(sizeof(uint2) * nn);
    w.bytes = off;
    return w;
}

}  // namespace gsvc

using namespace gsvc;

extern "C" size_t gsvc_train_step_workspace_bytes(int num_points, unsigned img_height,
                                                  unsigned img_width) {
    return train_ws(nullptr, num_points, tiles_of(img_height, img_width)).bytes;
}

extern "C" size_t gsvc_train_step_det_workspace_bytes(int num_points, long long det_capacity) {
    const size_t nn = (size_t)(num_points > 0 ? num_points : 0);
    const size_t cap = (size_t)(det_capacity > 0 ? det_capacity : 0);
    return ws_align(sizeof(int) * (nn + 1)) + sizeof(float4) * 2 * cap;
}

static int train_step_impl(int num_points, float *xyz, float *cholesky,
                           const float *cholesky_bound, float *features, float *rgb_w,
                           int rgb_w_trainable, const float *background, const float *gt,
                           unsigned img_height, unsigned img_width, int loss_kind,
                           int frame_index, float *const *adan_state,
                           const double *adan_hparams, int adan_flags, float *loss,
                           float *render_out, float *grads_out, void *workspace,
                           size_t workspace_bytes, void *stream, void *det_workspace,
                           size_t det_workspace_bytes, long long det_capacity) {
    if (num_points < 0 || img_height == 0 || img_width == 0)
        return set_error(GSVC_ERR_ARG, "train_step_sum: bad sizes");
    if (!xyz || !cholesky || !features || !background || !gt || !loss || !adan_hparams)
        return set_error(GSVC_ERR_ARG, "train_step_sum: missing input");
    if (loss_kind != 0 && loss_kind != 1)
        return set_error(GSVC_ERR_ARG, "train_step_sum: loss_kind must be 0 (L2) or 1 (L1)");
    if (rgb_w_trainable && !rgb_w)
        return set_error(GSVC_ERR_ARG, "train_step_sum: trainable rgb_w needs rgb_w");
    const bool update = grads_out == nullptr;
    if (update) {
        if (!adan_state) return set_error(GSVC_ERR_ARG, "train_step_sum: missing Adan state");
        for (int q = 0; q < 4; ++q)
            for (int k = 0; k < 4; ++k)
                if (!adan_state[4 * q + k] && (q < 3 || rgb_w_trainable))
                    return set_error(GSVC_ERR_ARG, "train_step_sum: missing Adan state tensor");
    }
    const int tbx = ceil_div((int)img_width, kTile), tby = ceil_div((int)img_height, kTile);
    const int ntiles = tbx * tby;
    const TrainWs w = train_ws((char *)workspace, num_points, ntiles);
    if (!workspace || workspace_bytes < w.bytes)
        return set_error(GSVC_ERR_WORKSPACE, "train_step_sum: workspace too small (%zu < %zu)",
                         workspace_bytes, w.bytes);
    hipStream_t s = (hipStream_t)stream;
    if (const int rc = refuse_capture(s, "train_step_sum")) return rc;
    const FrameSlots f = frame_slots(w.f, ntiles, frame_index);
    // GSVC_TRAIN_ORDER: project in the workspace's splat order (windowed slot
    // atomics); GSVC_TRAIN_ORDER_REFRESH: write keys and sort a new order
    // after the step
    const bool use_order = (adan_flags & GSVC_TRAIN_ORDER) != 0;
    const bool refresh = (adan_flags & GSVC_TRAIN_ORDER_REFRESH) != 0 && num_points > 0;
    SplatOrder ord;
    ord.order = use_order ? w.f.order : nullptr;
    if (refresh) {
        ord.key = w.f.okey;
        ord.key_id = w.f.okey_id;
    }
    // Where this call's one projection goes (GSVC_TRAIN_PROJECT_*): first, for
    // this frame (default); none (PROJECTED: an earlier call's PROJECT_NEXT
    // already enqueued it); only (PROJECT_ONLY); or last, for frame_index + 1
    // with the parameters this step updates (PROJECT_NEXT).
    const bool projected = (adan_flags & GSVC_TRAIN_PROJECTED) != 0;
    const bool only = (adan_flags & GSVC_TRAIN_PROJECT_ONLY) != 0;
    const bool next = (adan_flags & GSVC_TRAIN_PROJECT_NEXT) != 0;
    if ((only && (projected || next)) || (next && !projected))
        return set_error(GSVC_ERR_ARG, "train_step_sum: PROJECT_ONLY excludes the other "
                                       "projection flags; PROJECT_NEXT needs PROJECTED");
    if (next && !update)
        return set_error(GSVC_ERR_ARG, "train_step_sum: PROJECT_NEXT needs the Adan update");
    // GSVC_TRAIN_CARRY: the carried bins (a projection builds them; a step
    // consumes them and its splat kernel carries them to frame_index + 1)
    const bool carry = (adan_flags & GSVC_TRAIN_CARRY) != 0 && num_points > 0;
    if (carry && next)
        return set_error(GSVC_ERR_ARG, "train_step_sum: CARRY excludes PROJECT_NEXT");
    // (with grads_out the step reads carried bins but carries nothing: the
    // parameters do not change)
    if (carry) {
        ord.carry_ids = w.cids;
        ord.carry_counts = w.ccount;
        ord.carry_box = w.cbox;
        ord.carry_hull = w.chull;
    }
    const bool det = (adan_flags & GSVC_TRAIN_DETERMINISTIC) != 0;
    // GSVC_TRAIN_TILES_NEXT: after the splat kernel (which carried the bins to
    // frame_index + 1), enqueue frame_index + 1's tile kernel with this call's
    // target -- it reads only the carried bins, the records and gt, none of
    // the next call's hyper-parameters; GSVC_TRAIN_TILED: this frame's tile
    // kernel is that one (the call launches the splat kernel only)
    const bool tiled = (adan_flags & GSVC_TRAIN_TILED) != 0;
    const bool tiles_next = (adan_flags & GSVC_TRAIN_TILES_NEXT) != 0;
    // GSVC_TRAIN_REBUILD_NEXT (with TILES_NEXT): before that tile kernel, rebuild
    // frame_index + 1's bins from scratch (the PROJECT_ONLY | CARRY projection;
    // the order flags apply to it), so the periodic rebuild costs no host gap
    const bool rebuild_next = (adan_flags & GSVC_TRAIN_REBUILD_NEXT) != 0;
    if ((tiled || tiles_next) && (!carry || !projected || !update || render_out))
        return set_error(GSVC_ERR_ARG, "train_step_sum: TILED / TILES_NEXT need CARRY | PROJECTED, "
                                       "the Adan update and no render_out");
    if (rebuild_next && !tiles_next)
        return set_error(GSVC_ERR_ARG, "train_step_sum: REBUILD_NEXT needs TILES_NEXT");
    int *det_off = nullptr;
    float4 *det_part = nullptr;
    if (det) {
        if (!det_workspace || det_capacity < 0 ||
            det_workspace_bytes < gsvc_train_step_det_workspace_bytes(num_points, det_capacity))
            return set_error(GSVC_ERR_WORKSPACE, "train_step_sum: GSVC_TRAIN_DETERMINISTIC needs a "
                                                 "det_workspace of gsvc_train_step_det_workspace_bytes");
        det_off = (int *)det_workspace;
        det_part = (float4 *)((char *)det_workspace + ws_align(sizeof(int) * ((size_t)num_points + 1)));
    }
    auto project = [&](const FrameSlots &fs) {
        int r = frame_project_launch(num_points, xyz, 1, cholesky, cholesky_bound, features, rgb_w,
                                     nullptr, img_height, img_width, w.f, fs, w.grad, s, 1,
                                     nullptr, 0, (use_order || refresh) ? &ord : nullptr);
        if (r || !refresh) return r;
        return splat_order_sort(w.f, num_points, tbx, tby, s);  // the next calls' order
    };
    int rc = GSVC_OK;
    if (!projected) {
        if (carry) {
            // a new set of carried bins: counts and this frame's M from zero (a
            // previous step's splat kernel may have carried into them)
            if (dev_zero(w.ccount, sizeof(unsigned) * 2 * (size_t)ntiles, s) != GSVC_OK ||
                dev_zero(f.m_acc, sizeof(int), s) != GSVC_OK)
                return set_error(GSVC_ERR_HIP, "train_step_sum: memset failed");
        }
        // a refreshing projection's sort runs after the step (off the loss's path)
        rc = frame_project_launch(num_points, xyz, 1, cholesky, cholesky_bound, features, rgb_w,
                                  nullptr, img_height, img_width, w.f, f, w.grad, s, 1, nullptr, 0,
                                  (use_order || refresh || carry) ? &ord : nullptr);
        if (rc) return rc;
        if (only) return refresh ? splat_order_sort(w.f, num_points, tbx, tby, s) : GSVC_OK;
    }

    // a frame's (splat, tile) slot offsets, from its projection's xys / radii,
    // and its zeroed slots (the block totals live in det_part until the memset)
    auto det_prepare = [&]() {
        det_offsets_launch(num_points, (const float2 *)w.f.xys, w.f.radii, tbx, tby, det_off,
                           (int *)det_part, det_capacity > 0 ? 8 * (size_t)det_capacity : 0, s);
        if (det_capacity > 0 &&
            dev_zero(det_part, sizeof(float4) * 2 * (size_t)det_capacity, s) != GSVC_OK)
            return set_error(GSVC_ERR_HIP, "train_step_sum: memset failed");
        return check_launch("train_step_sum: det offsets");
    };
    if (det && !tiled) {  // (TILED: the previous call prepared them with its tile kernel)
        rc = det_prepare();
        if (rc) return rc;
    }
    const double count = 3.0 * (double)img_height * (double)img_width;  // numel of [3, H, W]
    // GSVC_TRAIN_LOSS_SEQ: ``loss`` is coherent host memory of 3 words; word 2
    // receives the call's sequence number (frame_index + 1, never 0)
    const unsigned loss_seq =
        (adan_flags & GSVC_TRAIN_LOSS_SEQ) ? ((unsigned)frame_index + 1u) | 0x80000000u : 0u;
    TrainTileArgs T{};
    T.tbx = tbx;
    T.img_w = (int)img_width;
    T.img_h = (int)img_height;
    T.ntiles = ntiles;
    T.num_points = num_points;
    T.loss_l1 = loss_kind;
    T.norm = loss_kind ? 1.0f / (float)count : (float)(2.0 / count);
    T.slab = w.f.slab;
    T.ovf = w.f.ovf;
    T.xys = w.f.xys;
    T.radii = w.f.radii;
    T.rec = w.f.rec;
    T.bg = background;
    T.gt = gt;
    T.grad = reinterpret_cast<float *>(w.grad);
    T.err = w.err;
    T.out = render_out;
    // A/B knob 11: the band kernel's work-item split width (default kBRun)
    T.brun = knob(11) >= 4 && knob(11) <= 16 ? knob(11) : kBRun;
    // A/B knob 12: speculative slab records per tile (default kBSpec)
    T.spec = knob(12) > 0 && knob(12) <= 64 ? knob(12) : kBSpec;
    T.diag = knob(13);
    T.grouped = knob(14) != 1;
    T.prio = knob(16) != 1;  // A/B knob 16 = 1: no raised priority
    T.xcd_off = knob(37);  // A/B: 1 dispatch order, 4 contiguous XCD ranges
    T.det_off = det_off;
    T.det_part = det_part;
    T.det_cap = det_capacity;
    if (carry) {
        T.cids = w.cids;
        T.cbox = w.cbox;
        // (zeroed with ccount whenever the bins are rebuilt; A/B knob 28 = 1: no
        // sorted lists -- every step ranks, nothing is written back)
        T.csorted = knob(28) == 1 ? nullptr : w.csorted;
    }
    // the tile kernel of the frame whose slots are fs
    auto launch_tiles = [&](const FrameSlots &fs) {
        T.counts = carry ? w.ccount : fs.counts;
        T.counts_clear = fs.counts_next;
        T.m_dev = fs.m_acc;
        T.m_clear = carry ? fs.m_clear : nullptr;
        if constexpr (kDiag) {
            if (knob(5) == 2 && debug_ptr() && !carry) {  // diagnostic: per-tile stamps
                T.stamps = reinterpret_cast<long long *>(debug_ptr());
                auto kfn = train_tile_kernel<true>;
                hipLaunchKernelGGL(kfn, dim3(ntiles), dim3(kT), 0, s, T);
                return check_launch("train_step_sum: tiles");
            }
            if (knob(5) == 3 && debug_ptr()) {  // diagnostic: per-tile stamps, band kernel
                T.stamps = reinterpret_cast<long long *>(debug_ptr());
                if (carry)
                    hipLaunchKernelGGL((train_tile_band_kernel<true, false, true>), dim3(ntiles),
                                       dim3(kBThreads), 0, s, T);
                else
                    hipLaunchKernelGGL(train_tile_band_kernel<true>, dim3(ntiles), dim3(kBThreads), 0, s, T);
                return check_launch("train_step_sum: tiles");
            }
        }
        const dim3 grid(ntiles);
        hipEvent_t tev[2];
        const int tslot = timing_begin(s, tev, kTimingTrainTile);
        bool launched = false;
        if constexpr (kDiag) {
            // knob 8 = 1: the 256-thread workgroup-per-tile kernel (A/B; atomics only)
            if (knob(8) == 1 && !det && !carry) {
                launch_timed(train_tile_kernel<false>, dim3(ntiles), dim3(kT), 0, s, tev, T);
                launched = true;
            }
        }
        if (launched)
            ;
        else if (det && carry)
            launch_timed(train_tile_band_kernel<false, true, true>, grid, dim3(kBThreads), 0, s, tev, T);
        else if (det)
            launch_timed(train_tile_band_kernel<false, true>, grid, dim3(kBThreads), 0, s, tev, T);
        else if (carry)
            launch_timed(train_tile_band_kernel<false, false, true>, grid, dim3(kBThreads), 0, s, tev, T);
        else
            launch_timed(train_tile_band_kernel<false>, grid, dim3(kBThreads), 0, s, tev, T);
        timing_end(s, tslot, kTimingTrainTile);
        return check_launch("train_step_sum: tiles");
    };
    if (!tiled) {
        rc = launch_tiles(f);
        if (rc) return rc;
    }

    TrainSplatArgs P{};
    P.n = num_points;
    P.ntiles = ntiles;
    P.rgbw_train = rgb_w_trainable ? 1 : 0;
    P.update = update ? 1 : 0;
    P.hw = 0.5f * (float)img_width;
    P.hh = 0.5f * (float)img_height;
    P.inv_count = 1.0 / count;
    P.xyz = xyz;
    P.chol = cholesky;
    P.feat = features;
    P.rgbw = rgb_w;
    P.chol_bound = cholesky_bound;
    P.radii = w.f.radii;
    P.rec = w.f.rec;
    P.grad = w.grad;
    if (update)
        for (int q = 0; q < 4; ++q)
            for (int k = 0; k < 4; ++k) P.state[q][k] = adan_state[4 * q + k];
    for (int q = 0; q < 4; ++q) P.first[q] = (adan_flags >> (1 + q)) & 1;
    const double *h = adan_hparams;
    P.S = adan_scalars(h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], adan_flags & 1, h[9]);
    P.grads_out = grads_out;
    P.det_off = det_off;
    P.det_part = det_part;
    P.det_cap = det_capacity;
    P.err = w.err;
    P.loss = loss;
    if (carry && update) {
        // 2: M as a flag (A/B knob 22 = 1: the exact count by atomics)
        P.carry = knob(22) == 1 ? 1 : 2;
        P.tbx = tbx;
        P.tby = tby;
        P.xys = (float2 *)w.f.xys;
        P.cbox = w.cbox;
        P.chull = w.chull;
        P.ccount = w.ccount;
        P.cids = w.cids;
        P.m_next = f.m_clear;  // frame_index + 1's M slot (the tile kernel zeroed it)
    }
    P.loss_seq = loss_seq;
    // one extra (first) workgroup sums the loss, beside the splat workgroups
    // A/B knob 21 = 64, 128, 192 or 512: other splat workgroup sizes
    const int sb = knob(21) == 64 || knob(21) == 128 || knob(21) == 192 || knob(21) == 512
                       ? knob(21)
                       : 256;
    // (1: the carry in the geometry wave; A/B knob 36 = 2: both waves project and
    // share its stores -- measured equal, 9.92-10.0 vs 9.85-9.98 us, not kept;
    // 3: the xyz elements on the colour wave)
    // two waves per 64 splats (splat_step_split) unless A/B knob 34 = 1 or
    // another workgroup size (nine lanes per splat, one per parameter element,
    // was measured, round 6: 18.6 vs 10.5 us, profiles/r06/splat_elem/)
    P.split = sb == 256 && knob(34) != 1 ? 1 : 0;
    const int per_block = P.split ? sb / 2 : sb;
    const int blocks = (num_points > 0 ? ceil_div(num_points, per_block) : 0) + 1;
    hipEvent_t tev[2];
    const int tslot = timing_begin(s, tev, kTimingTrainSplat);
    bool launched = false;
    if constexpr (kDiag) {
        launched = true;
        if (knob(5) == 4 && debug_ptr()) {  // diagnostic: per-wave stamps of the splat kernel
            P.stamps = reinterpret_cast<long long *>(debug_ptr());
            hipLaunchKernelGGL(train_splat_kernel<true>, dim3(ceil_div(num_points, 256) + 1), dim3(256), 0, s, P);
        } else if (sb == 64) {
            launch_timed(train_splat_kernel<false, 64>, dim3(blocks), dim3(64), 0, s, tev, P);
        } else if (sb == 128) {
            launch_timed(train_splat_kernel<false, 128>, dim3(blocks), dim3(128), 0, s, tev, P);
        } else if (sb == 192) {
            launch_timed(train_splat_kernel<false, 192>, dim3(blocks), dim3(192), 0, s, tev, P);
        } else if (sb == 512) {
            launch_timed(train_splat_kernel<false, 512>, dim3(blocks), dim3(512), 0, s, tev, P);
        } else {
            launched = false;
        }
    }
    if (!launched) launch_timed(train_splat_kernel<false>, dim3(blocks), dim3(256), 0, s, tev, P);
    timing_end(s, tslot, kTimingTrainSplat);
    rc = check_launch("train_step_sum: splats");
    if (rc) return rc;
    if (tiles_next) {
        const FrameSlots fn = frame_slots(w.f, ntiles, frame_index + 1);
        if (rebuild_next) {
            // the splat kernel's carry is superseded: counts and M from zero,
            // then the projection bins frame_index + 1 afresh (and re-zeroes the
            // gradient records)
            if (dev_zero(w.ccount, sizeof(unsigned) * 2 * (size_t)ntiles, s) != GSVC_OK ||
                dev_zero(fn.m_acc, sizeof(int), s) != GSVC_OK)
                return set_error(GSVC_ERR_HIP, "train_step_sum: memset failed");
            rc = frame_project_launch(num_points, xyz, 1, cholesky, cholesky_bound, features, rgb_w,
                                      nullptr, img_height, img_width, w.f, fn, w.grad, s, 1, nullptr, 0,
                                      &ord);
            if (rc) return rc;
            if (refresh) {
                rc = splat_order_sort(w.f, num_points, tbx, tby, s);
                if (rc) return rc;
            }
        }
        if (det) {  // frame_index + 1's slots (the splat kernel has read this frame's)
            rc = det_prepare();
            if (rc) return rc;
        }
        return launch_tiles(fn);
    }
    if (next) return project(frame_slots(w.f, ntiles, frame_index + 1));
    if (!projected && refresh) return splat_order_sort(w.f, num_points, tbx, tby, s);
    return GSVC_OK;
}

extern "C" int gsvc_train_step_sum(int num_points, float *xyz, float *cholesky,
                                   const float *cholesky_bound, float *features, float *rgb_w,
                                   int rgb_w_trainable, const float *background, const float *gt,
                                   unsigned img_height, unsigned img_width, int loss_kind,
                                   int frame_index, float *const *adan_state,
                                   const double *adan_hparams, int adan_flags, float *loss,
                                   float *render_out, float *grads_out, void *workspace,
                                   size_t workspace_bytes, void *stream) {
    return train_step_impl(num_points, xyz, cholesky, cholesky_bound, features, rgb_w,
                           rgb_w_trainable, background, gt, img_height, img_width, loss_kind,
                           frame_index, adan_state, adan_hparams, adan_flags, loss, render_out,
                           grads_out, workspace, workspace_bytes, stream, nullptr, 0, 0);
}

extern "C" int gsvc_train_step_sum_args(const gsvc_train_step_args *a) {
    if (!a) return set_error(GSVC_ERR_ARG, "train_step_sum_args: null");
    return train_step_impl(a->num_points, a->xyz, a->cholesky, a->cholesky_bound, a->features,
                           a->rgb_w, a->rgb_w_trainable, a->background, a->gt, a->img_height,
                           a->img_width, a->loss_kind, a->frame_index, a->adan_state,
                           a->adan_hparams, a->adan_flags, a->loss, a->render_out, a->grads_out,
                           a->workspace, a->workspace_bytes, a->stream, a->det_workspace,
                           a->det_workspace_bytes, a->det_capacity);
}
