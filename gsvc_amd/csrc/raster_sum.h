// Sum rasterizer launch interface shared by raster_sum.hip and frame.hip.
#pragma once

#include "common.h"

namespace gsvc {

// Output layouts: kLayoutHWC is the reference's [H, W, 3] image (+ final_idx);
// kLayoutCHWClamped writes torch.clamp(img, 0, 1) as planes [3, H, W], i.e. the
// epilogue of GaussianSplats_Represent.py:88-89 (clamp, view, permute,
// contiguous) fused into the store; kLayoutCHW the same planes unclamped (the op
// path's [H, W, 3] image with strides (W, 1, H*W): GSVC's clamp + permute +
// contiguous then read it without a copy).
enum { kLayoutHWC = 0, kLayoutCHWClamped = 1, kLayoutCHW = 2 };
__host__ __device__ inline bool layout_planes(int layout) {
    return layout == kLayoutCHWClamped || layout == kLayoutCHW;
}

struct SumFwdArgs {
    int tbx, img_w, img_h, ntiles, sparse_max, layout;
    bool vec;      // HWC: W % 4 == 0 and 16-byte aligned outputs
    bool vec_chw;  // CHW: W % 4 == 0, H*W % 4 == 0, 16-byte aligned
    int store_policy;  // CHW plane stores: kStore* (gsvc_debug_set(7) selects)
    int spec_slots;    // frame path: slab records loaded with the count (<= kHeadSlots)
    int group_min;     // sparse chunks of <= this many entries skip the lane-group lists
    int cut;           // sparse render chunks may take the sigma-threshold blend (knob 19 = 1: never)
    int xcd_off;       // diagnostic A/B (knob 37): 1 tiles in dispatch order, 4 xcd_remap ranges
    int ablate;        // diagnostic (knob 36, wrong results): sparse tile phases skipped --
                       // 1 blend, 2 stores, 4 record loads, 8 ranking,
                       // 16 every load (raster_render_ids_kernel)
    int ids_cap;       // id slabs: slots per tile (kTilePix, or kCarryCap for wide slabs)
    const int *m_dev;  // device num_intersects (NULL: > 0); 0 -> background
    const float *bg;
    const int *ids;
    const int2 *bins;
    const float2 *xys;
    const float *conics, *colors, *opac;
    // frame path: per-splat records {x, y, a/2, b}, {c/2, opacity, r, g},
    // {b, -, -, -} replace the four arrays above (same values)
    const float4 *rec;
    bool sort_ids;  // ids of a tile arrive unsorted; the kernel sorts them in LDS
    // frame path: per-tile 256-slot slabs of splat records (3 float4 each:
    // {x, y, a/2, b}, {c/2, opacity, r, g}, {b, id bits, -, -}) with their
    // counts for this frame; the kernel clears the other parity's counts
    // (slab_counts_clear) for the next frame.  Tiles with more than 256
    // entries are rebuilt from the splats' bboxes (cull_xys, cull_radii,
    // num_points) and records (rec).
    const float4 *slab;
    const int *slab_ovf;  // record slabs: the ids of slots 256 .. kCarryCap - 1 (frame.h FrameWs.ovf)
    const unsigned *slab_counts;
    unsigned *slab_counts_clear;
    const float2 *cull_xys;
    const int *cull_radii;
    int num_points;
    int *meta_out;  // frame path: meta[0] <- M (from m_dev), meta[1] <- 0
    // batched frame path (gsvc_render_frames_sum): the grid covers frames x
    // tiles; frame b's slab-path buffers sit at these strides from frame 0's
    // (slab, counts, counts_clear, m_dev, meta_out, out) and its splats are
    // [frame_off[b], frame_off[b + 1]) of the global id range (device array;
    // NULL: one frame, splats [splat_begin = 0, num_points))
    int frames, counts_stride, m_stride;
    size_t slab_stride, out_stride;
    const int *frame_off;
    int splat_begin;
    float *out;
    int *final_idx;
    float *final_Ts;
    long long *stamps;  // kModeStamp only
    // op path with unsorted id slabs (gsvc_rasterize_sum_forward_slabs): tile
    // t's ids at ids_rw[t * 256 + j], j < min(count, 256), its count in
    // id_counts[t]; the kernel sorts them (more than 256: the first 256 rebuilt
    // from cull_xys / cull_radii), writes them back in order and the tile's
    // bins row [t * 256, t * 256 + n) for the backward, and zeroes
    // id_counts_clear[t] (the next call's counts)
    const unsigned *id_counts;
    unsigned *id_counts_clear;
    int *ids_rw;
    int2 *bins_out;
};

// sum_fwd_args_init zeroes every field (rec, stamps, m_dev NULL; HWC layout);
// callers set the rest.  sum_forward_launch launches the kernel variant for
// ``density_hint`` (or the gsvc_debug_set(0) override).
void sum_fwd_args_init(SumFwdArgs &A);
int sum_forward_launch(SumFwdArgs &A, int density_hint, hipStream_t s);
// The launcher's sparse / banded choice from the caller's intersection count
// (M of an earlier frame): true = banded (two waves per tile).  Render over
// id slabs (A.id_counts without final_idx) is the sparse kernel only, so a
// render takes id slabs exactly when this is false.
bool sum_forward_dense(int density_hint, int ntiles, int frames);

}  // namespace gsvc
