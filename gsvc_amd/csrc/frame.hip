// Whole-frame render of GSVC's per-frame model, one C call (gfx950).
//
// Reference: GaussianSplats_Represent.py:57-90 (parameter activations and
// forward), i.e. for each frame
//     means2d = tanh(_xyz); L = _cholesky + cholesky_bound;
//     colors = _features_dc * rgb_W; opacity = 1
//     project_gaussians_2d -> rasterize_gaussians_sum -> clamp -> NCHW
// (foward2d.cu:12-69, utils.py:99-167, forward.cu:512-627).
//
// Launches:
//   frame_project_kernel  activations + projection (project2d.h, the op's own
//                         op sequence) + per-tile entry counts (atomics), and
//                         a 48-byte record per splat for the rasterizer;
//   tile_scan/fill/segsort (binning.hip) -- the scan clears the counters
//                         for the next frame, so no memset is needed;
//   raster_sum_fwd_kernel (raster_sum.hip) in the clamped [3,H,W] layout,
//                         reading the records (no final_idx: no backward).
// Nothing is read back to the host, and the workspace is reused across
// frames.
#include "binning.h"
#include "project2d.h"
#include "raster_sum.h"

namespace gsvc {

__global__ __launch_bounds__(256) void frame_project_kernel(
    int n, const float *__restrict__ xyz, int xyz_tanh, const float *__restrict__ chol,
    const float *__restrict__ chol_bound, const float *__restrict__ feat,
    const float *__restrict__ rgb_w, const float *__restrict__ opac, float hw, float hh, int tbx,
    int tby, float2 *__restrict__ xys, int *__restrict__ radii, float4 *__restrict__ rec,
    unsigned *__restrict__ counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float mx = xyz[2 * i], my = xyz[2 * i + 1];
    if (xyz_tanh) {  // get_xyz (GaussianSplats_Represent.py:57-59)
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
    const SplatProj P = project_splat(mx, my, l11, l21, l22, hw, hh, tbx, tby);
    xys[i] = P.xy;
    radii[i] = P.rad;
    rec[3 * i] = make_float4(P.xy.x, P.xy.y, 0.5f * P.c0, P.c1);
    rec[3 * i + 1] = make_float4(0.5f * P.c2, o, r, g);
    rec[3 * i + 2] = make_float4(b, 0.0f, 0.0f, 0.0f);
    if (P.rad > 0) count_splat_tiles(P.xy.x, P.xy.y, P.rad, tbx, tby, counts);
}

static inline size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

struct FrameWs {
    unsigned *counts, *cursor;
    int2 *bins;
    float2 *xys;
    int *radii;
    float4 *rec;
    int *ids_scratch, *ids_sorted;
    size_t bytes;
};

static FrameWs frame_ws(char *base, int n, int ntiles, long long capacity) {
    FrameWs w;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char *p = base ? base + off : nullptr;
        off += align_up(bytes);
        return p;
    };
    const size_t nn = (size_t)(n > 0 ? n : 1), nt = (size_t)(ntiles > 0 ? ntiles : 1);
    const size_t cap = (size_t)(capacity > 0 ? capacity : 1);
    w.counts = (unsigned *)take(sizeof(unsigned) * nt);  // first: zeroed by the caller once
    w.cursor = (unsigned *)take(sizeof(unsigned) * nt);
    w.bins = (int2 *)take(sizeof(int2) * nt);
    w.xys = (float2 *)take(sizeof(float2) * nn);
    w.radii = (int *)take(sizeof(int) * nn);
    w.rec = (float4 *)take(sizeof(float4) * 3 * nn);
    w.ids_scratch = (int *)take(sizeof(int) * cap);
    w.ids_sorted = (int *)take(sizeof(int) * cap);
    w.bytes = off;
    return w;
}

}  // namespace gsvc

using namespace gsvc;

extern "C" size_t gsvc_render_frame_workspace_bytes(int num_points, unsigned img_height,
                                                    unsigned img_width, long long capacity) {
    const int ntiles = ceil_div((int)img_width, kTile) * ceil_div((int)img_height, kTile);
    return frame_ws(nullptr, num_points, ntiles, capacity).bytes;
}

extern "C" size_t gsvc_render_frame_zeroed_bytes(unsigned img_height, unsigned img_width) {
    const int ntiles = ceil_div((int)img_width, kTile) * ceil_div((int)img_height, kTile);
    return sizeof(unsigned) * (size_t)ntiles;
}

extern "C" int gsvc_render_frame_sum(int num_points, const float *xyz, int xyz_tanh,
                                     const float *cholesky, const float *cholesky_bound,
                                     const float *features, const float *rgb_w,
                                     const float *opacity, const float *background,
                                     unsigned img_height, unsigned img_width, long long capacity,
                                     int density_hint, int *meta, void *workspace,
                                     size_t workspace_bytes, float *out, void *stream) {
    if (num_points < 0 || capacity < 0 || img_height == 0 || img_width == 0)
        return set_error(GSVC_ERR_ARG, "render_frame_sum: bad sizes");
    if (!xyz || !cholesky || !features || !background || !meta || !out)
        return set_error(GSVC_ERR_ARG, "render_frame_sum: missing input");
    const int tbx = ceil_div((int)img_width, kTile), tby = ceil_div((int)img_height, kTile);
    const int ntiles = tbx * tby;
    const FrameWs w = frame_ws((char *)workspace, num_points, ntiles, capacity);
    if (!workspace || workspace_bytes < w.bytes)
        return set_error(GSVC_ERR_WORKSPACE, "render_frame_sum: workspace too small (%zu < %zu)",
                         workspace_bytes, w.bytes);
    hipStream_t s = (hipStream_t)stream;
    const float hw = 0.5f * (float)img_width, hh = 0.5f * (float)img_height;
    if (num_points > 0)
        hipLaunchKernelGGL(frame_project_kernel, dim3(ceil_div(num_points, 256)), dim3(256), 0, s,
                           num_points, xyz, xyz_tanh, cholesky, cholesky_bound, features, rgb_w,
                           opacity, hw, hh, tbx, tby, w.xys, w.radii, w.rec, w.counts);
    int rc = tile_bins_from_counts(num_points, w.xys, w.radii, tbx, tby, capacity, w.counts, w.cursor,
                                   w.ids_scratch, w.ids_sorted, w.bins, meta, true, s);
    if (rc) return rc;
    SumFwdArgs A;
    sum_fwd_args_init(A);
    A.tbx = tbx;
    A.img_w = (int)img_width;
    A.img_h = (int)img_height;
    A.ntiles = ntiles;
    A.layout = kLayoutCHWClamped;
    A.m_dev = meta;
    A.bg = background;
    A.ids = w.ids_sorted;
    A.bins = w.bins;
    A.rec = w.rec;
    A.out = out;
    return sum_forward_launch(A, density_hint, s);
}
