/*
 * gsvc_amd.h -- C ABI of the MI355X-native 2D Gaussian-splat rasterizer.
 *
 * This is the drop-in boundary for the hot path of ac-freeman/GSVC: the ops
 * that the reference's torch extension ``gsplat.csrc`` exports
 * (gsplat/gsplat/cuda/csrc/ext.cpp:6-23, prototypes bindings.h:16-301) for the
 * 2D path, plus the binning glue the reference ran in PyTorch
 * (gsplat/gsplat/utils.py:99-167).  Every entry point takes plain device
 * pointers and sizes; no torch types cross it.  The Python mirror of the
 * reference operator API (gsvc_amd/, re-exported as the ``gsplat`` package)
 * binds these with ctypes; INTEGRATION.md shows the binding a maintainer of
 * the reference would add.
 *
 * Conventions
 *   - All pointers are device (HBM) pointers unless stated otherwise.
 *   - ``stream`` is a hipStream_t (NULL = legacy default stream); every entry
 *     point is asynchronous on it and never synchronises the device, so calls
 *     can be captured in a hipGraph -- except the entries whose workspace
 *     alternates host-indexed parity slots (call_index / frame_index: the
 *     slab renders, gsvc_rasterize_sum_forward_slabs*, the fused training
 *     step): a replay would re-add into the slots capture froze, so they
 *     refuse a capturing stream with GSVC_ERR_CAPTURE before any launch (the
 *     reference's own forward cannot be captured either: its .item(),
 *     utils.py:117).  The counted binning + rasterize_sum entries are the
 *     capturable route.
 *   - Return value: 0 on success, otherwise a gsvc_status code; the message of
 *     the last failure on the calling thread is gsvc_last_error().  Bad
 *     arguments are rejected before any launch (the reference raised
 *     c10::Error through TORCH_CHECK / AT_ERROR, bindings.h:9-14).
 *   - Outputs are fully written by the call (no caller-side zeroing needed)
 *     unless a comment says otherwise.
 *   - Images are row-major HWC float32, pixel (j, i) evaluated at (j, i).
 *   - Only 16x16 tiles are supported (the reference kernels hard-code
 *     BLOCK_X = BLOCK_Y = 16, config.h:1-4).
 */
#ifndef GSVC_AMD_H
#define GSVC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum gsvc_status {
    GSVC_OK = 0,
    GSVC_ERR_ARG = 1,       /* invalid argument (shape, size, tile size) */
    GSVC_ERR_WORKSPACE = 2, /* workspace too small */
    GSVC_ERR_HIP = 3,       /* HIP runtime / launch error */
    GSVC_ERR_CAPTURE = 4    /* the stream is capturing a graph and the entry keeps host-indexed state */
};

/* ABI version 2: gsvc_debug_set / gsvc_debug_set_ptr moved to the diagnostic
 * library (gsvc_amd_diag.h); GSVC_ERR_CAPTURE added. */
#define GSVC_ABI_VERSION 2

/* Library identity and error reporting. */
int gsvc_abi_version(void);
const char *gsvc_last_error(void);

/* ---------------------------------------------------------------------------
 * Fused Adan step (optimizer.py:296-362 _multi_tensor_adan, one kernel for
 * all tensors).  Host arrays of ntensors device pointers / element counts;
 * every tensor contiguous fp32.  Scalars as in the reference (bias
 * corrections computed by the caller, optimizer.py:171-173,211).  grads are
 * read, not scaled in place. */
int gsvc_adan_step(int ntensors, const long long *numels, float *const *params,
                   const float *const *grads, float *const *exp_avgs,
                   float *const *exp_avg_sqs, float *const *exp_avg_diffs,
                   float *const *neg_pre_grads, double beta1, double beta2, double beta3,
                   double bias_correction1, double bias_correction2,
                   double bias_correction3_sqrt, double lr, double weight_decay, double eps,
                   int no_prox, double clip_global_grad_norm, void *stream);

/* ---------------------------------------------------------------------------
 * Pruning of a frame model (GaussianSplats_Represent.py:101-125 removal_control
 * and :149-166 adaptive_control: norm of rgb_W, torch.sort, boolean-mask
 * rebuild of _xyz / _cholesky / _features_dc / rgb_W).  Removes the
 * remove_count splats of smallest ||rgb_W|| (rgb_w: fp32 [num_points, 1];
 * equal norms leave in index order, as the GPU's stable torch.sort) and writes
 * the kept rows, in order, of each of the ntensors fp32 [num_points, cols[t]]
 * tensors src[t] to dst[t] ([num_points - remove_count, cols[t]]; src and dst
 * must not overlap).  Host arrays of device pointers; no host sync.
 * remove_count >= num_points keeps nothing and launches nothing. */
size_t gsvc_prune_workspace_bytes(int num_points);
int gsvc_prune_lowest(int num_points, int remove_count, const float *rgb_w, int ntensors,
                      const int *cols, const float *const *src, float *const *dst,
                      void *workspace, size_t workspace_bytes, void *stream);

/* Launch timing of the sum-forward composite kernel (every rasterizer entry
 * point above): after gsvc_timing_enable(max, every, how), every every-th
 * launch is timed by HIP events on its stream (up to max launches) -- how = 0:
 * events recorded before and after the launch (includes the marker packets and
 * the dispatch, ~3 us); how = 1: events carried by the dispatch itself
 * (hipExtLaunchKernel: the kernel's own start / end, as a kernel trace).
 * gsvc_timing_collect waits for them and writes the durations in ms.
 * gsvc_timing_enable(0, 0, 0) stops and frees.  Not part of the reference. */
int gsvc_timing_enable(int max_launches, int every, int how);
int gsvc_timing_collect(float *ms, int max_out, int *count);
/* The same for one kernel channel: 0 the composite (as above), 1 the fused
 * training step's tile kernel, 2 the frame projection (render and training),
 * 3 the training step's per-splat kernel (projection VJP + Adan), 4 the sum
 * rasterizer's backward, 5 / 6 the alpha rasterizer's forward / backward. */
int gsvc_timing_enable_channel(int channel, int max_launches, int every, int how);
int gsvc_timing_collect_channel(int channel, float *ms, int max_out, int *count);

/* The unit-opacity alpha cut as a sigma threshold (alpha_cut.hip): the
 * kernels' constant, and a device scan over all 2^31 non-negative float
 * patterns of the reference predicate (forward.cu:598-606 at opacity 1) into
 * out[4] (device memory) = {largest kept, smallest dropped, kept with
 * exp(-sigma) > 1, kept NaN patterns}.  Test hooks; not part of the reference. */
unsigned gsvc_alpha_cut_bits(void);
int gsvc_alpha_cut_scan(unsigned *out, void *stream);

/* hipStreamSynchronize(stream): the fused training step writes its losses
 * into caller memory that may be pinned host memory; the caller waits with
 * this before reading them (the reference's PSNR .item(),
 * GaussianSplats_Represent.py:196-198).  Not part of the reference. */
int gsvc_stream_sync(void *stream);
/* Coherent pinned host memory (hipHostMallocCoherent), zeroed: a kernel's
 * system-scope stores to it are seen by the host while the kernel runs.
 * Not part of the reference. */
void *gsvc_host_alloc(size_t bytes);
int gsvc_host_free(void *p);
/* Spin until the unsigned at ``word`` (coherent host memory) equals ``seq``;
 * after spin_us microseconds fall back to gsvc_stream_sync(stream), which
 * reports a failed kernel, and then require it.  The fused training step's
 * early loss read-back (GSVC_TRAIN_LOSS_SEQ).  Not part of the reference. */
int gsvc_wait_host_seq(const unsigned *word, unsigned seq, void *stream, int spin_us);

/* ---------------------------------------------------------------------------
 * 2D projection.
 * Replaces _C.project_gaussians_2d_forward
 *   (bindings.cu:781-839 -> foward2d.cu:12-69; Python project_gaussians_2d.py:63-103).
 * means2d [N,2], L_elements [N,3] (l11, l21, l22) in; xys [N,2], depths [N]
 * (all 0), radii [N] int32, conics [N,3], num_tiles_hit [N] int32 out.
 * clip_thresh is accepted and unused, as in the reference.
 */
int gsvc_project_gaussians_2d_forward(
    int num_points, const float *means2d, const float *L_elements,
    unsigned img_height, unsigned img_width,
    int tile_bounds_x, int tile_bounds_y, int tile_bounds_z, float clip_thresh,
    float *xys, float *depths, int *radii, float *conics, int *num_tiles_hit,
    void *stream);

/* Replaces _C.project_gaussians_2d_backward
 *   (bindings.cu:902-949 -> backward2d.cu:8-51; Python project_gaussians_2d.py:105-141).
 * v_depth is accepted and unused, as in the reference.  The L gradient keeps
 * the reference's doubled off-diagonal term (backward2d.cu:39-41). */
int gsvc_project_gaussians_2d_backward(
    int num_points, const float *means2d, const float *L_elements,
    unsigned img_height, unsigned img_width,
    const int *radii, const float *conics,
    const float *v_xy, const float *v_depth, const float *v_conic,
    float *v_cov2d, float *v_mean2d, float *v_L_elements,
    void *stream);

/* The same backward with row strides for v_xy and v_conic (>= 2 and >= 3
 * floats): the rasterizer backward's gradient records ([N,16], v_xy at 0,
 * v_conic at 2) are read in place, without a contiguous copy.  means2d and
 * v_depth, unused by the reference kernel, are not taken.  Not part of the
 * reference (the autograd Function of csrc/torch_ops.cpp calls it). */
int gsvc_project_gaussians_2d_backward_strided(
    int num_points, const float *L_elements, unsigned img_height, unsigned img_width,
    const int *radii, const float *conics, const float *v_xy, int v_xy_stride,
    const float *v_conic, int v_conic_stride, float *v_cov2d, float *v_mean2d,
    float *v_L_elements, void *stream);

/* Replaces _C.compute_cov2d_bounds (bindings.cu:41-60 -> :21-39).
 * covs2d [N,3] upper-triangular in; conics [N,3], radii [N] float out. */
int gsvc_compute_cov2d_bounds(int num_pts, const float *covs2d, float *conics,
                              float *radii, void *stream);

/* ---------------------------------------------------------------------------
 * Binning.  Replaces the torch glue of utils.py:99-167 and the two binning
 * ops _C.map_gaussian_to_intersects / _C.get_tile_bin_edges.
 */

/* torch.cumsum(num_tiles_hit, dtype=int32) of utils.py:116, plus a 4-int
 * device record ``meta`` = {M = cum[N-1], OR of depth bits, AND of depth bits,
 * splats with num_tiles_hit > 0} over the splats that emit intersections.
 * ``depths`` may be NULL (then meta[1] = meta[2] = 0).  Reading meta[0] on the
 * host is the one device->host sync of the forward (utils.py:117 ``.item()``). */
size_t gsvc_cumsum_workspace_bytes(int num_points);
int gsvc_compute_cumulative_intersects(
    int num_points, const int *num_tiles_hit, const float *depths,
    int *cum_tiles_hit, int *meta, void *workspace, size_t workspace_bytes,
    void *stream);

/* Replaces _C.map_gaussian_to_intersects (bindings.cu:274-313 -> forward.cu:100-136).
 * isect_ids [M] int64 = tile_id << 32 | sign-extended depth bits, gaussian_ids [M] int32. */
int gsvc_map_gaussian_to_intersects(
    int num_points, int num_intersects, const float *xys, const float *depths,
    const int *radii, const int *cum_tiles_hit,
    int tile_bounds_x, int tile_bounds_y, int tile_bounds_z,
    int64_t *isect_ids, int *gaussian_ids, void *stream);

/* Replaces torch.sort(isect_ids) + torch.gather(gaussian_ids) (utils.py:164-165):
 * stable LSD radix sort of signed int64 keys on bits [begin_bit, end_bit)
 * (pass 0, 64 for a full sort).  Keys equal on those bits keep input order. */
size_t gsvc_sort_pairs_workspace_bytes(int n);
int gsvc_sort_isect_pairs(
    int n, const int64_t *keys_in, const int *vals_in,
    int64_t *keys_out, int *vals_out, int begin_bit, int end_bit,
    void *workspace, size_t workspace_bytes, void *stream);

/* Replaces _C.get_tile_bin_edges (bindings.cu:315-330 -> forward.cu:141-163).
 * tile_bins [rows,2] int32 is zeroed then filled; rows must exceed every tile
 * id present (the reference allocated M rows, which overflowed when M < tiles). */
int gsvc_get_tile_bin_edges(int num_intersects, const int64_t *isect_ids_sorted,
                            int *tile_bins, int rows, void *stream);

/* Fused hot-path binning used by rasterize_gaussians_sum (utils.py:121-167 in
 * one call): emit (tile, splat) pairs in splat order, stable radix sort on the
 * ceil(log2(tiles)) tile bits only, and bin edges.  Valid when every emitting
 * splat has the same depth bits (meta[1] == meta[2]; always true for the 2D
 * projection, which writes depth 0), which makes the reference's 64-bit order
 * equal to the tile order.  gaussian_ids_sorted [M]; tile_bins [rows,2] with
 * rows >= tiles; isect_ids_sorted [M] optional (NULL to skip). */
size_t gsvc_bin_tiles_workspace_bytes(int num_points, int num_intersects, int num_tiles);
int gsvc_bin_and_sort_tiles(
    int num_points, int num_intersects, const float *xys, const float *depths,
    const int *radii, const int *cum_tiles_hit,
    int tile_bounds_x, int tile_bounds_y,
    int *gaussian_ids_sorted, int *tile_bins, int tile_bins_rows,
    int64_t *isect_ids_sorted, void *workspace, size_t workspace_bytes,
    void *stream);

/* Sync-free tile binning used by the rasterizer ops (the hot path of
 * utils.py:99-167 + bindings.cu:274-330 without reading num_intersects on the
 * host): builds gaussian_ids_sorted in the stable (tile, splat id) order of
 * the reference's sorted pairs and tile_bins[tbx*tby] ([start,end), (0,0)
 * when empty), every size staying on the device.  meta[0] <- M,
 * meta[1] <- 1 if the entries kept exceed capacity (outputs then
 * incomplete).  ids_scratch and gaussian_ids_sorted hold >= capacity ints.
 * tile_cap > 0 keeps only each tile's first tile_cap entries in id order (the
 * sum rasterizer reads no more than 256 per tile, forward.cu:569-571,613; a
 * tile with more is rebuilt from the splats' bboxes in id order), so
 * capacity = tiles * min(num_points, tile_cap) can never overflow; with
 * tile_cap 0 every entry is kept and capacity = num_points * tiles is the
 * safe bound.  M is the uncapped total either way.  Deterministic. */
size_t gsvc_bin_tiles_counted_workspace_bytes(int num_tiles);
int gsvc_bin_tiles_counted(int num_points, const float *xys, const int *radii,
                           int tile_bounds_x, int tile_bounds_y, long long capacity,
                           int tile_cap, int *ids_scratch, int *gaussian_ids_sorted,
                           int *tile_bins, int *meta, void *workspace,
                           size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Sum rasterizer (the GSVC renderer, rasterize_sum.py).
 * Replaces _C.rasterize_sum_forward (bindings.cu:400-469 -> forward.cu:512-627):
 * out[p] = sum over the first <= 256 sorted entries k of p's tile of
 * colors[g_k] * min(1, opac[g_k] * exp(-sigma)), skipping sigma < 0 and
 * alpha < 1/255; final_idx[p] = last contributing k (0 if none); final_Ts = 1.
 * final_Ts may be NULL (it is identically 1; the Python layer returns an
 * expanded constant).  background is accepted and unused, as in the reference. */
int gsvc_rasterize_sum_forward(
    int tile_bounds_x, int tile_bounds_y, int tile_bounds_z,
    int block_x, int block_y, int block_z,
    unsigned img_width, unsigned img_height, unsigned img_depth,
    const int *gaussian_ids_sorted, const int *tile_bins,
    const float *xys, const float *conics, const float *colors,
    const float *opacities, const float *background,
    float *out_img, float *final_Ts, int *final_idx, void *stream);

/* The same op with the knobs of the sync-free hot path (results identical to
 * gsvc_rasterize_sum_forward for the same inputs):
 *   num_intersects_dev  device int M (NULL: M > 0 assumed); when M < 1 every
 *                       pixel gets background, the reference's M < 1 branch
 *                       (rasterize_sum.py:121-127), final_idx 0;
 *   density_hint        an estimate of M (any value is correct; > 5 entries
 *                       per tile selects the banded two-waves-per-tile
 *                       kernel, otherwise one wave per tile);
 *   out_layout          0: out_img [H,W,3] as the reference;
 *                       1: out_img [3,H,W] = torch.clamp(img, 0, 1) permuted,
 *                       the caller epilogue of GaussianSplats_Represent.py:88-89;
 *                       2: out_img as channel planes [3,H,W], unclamped: the
 *                       [H,W,3] image with strides (W, 1, H*W) (GSVC_SLABS_PLANES);
 *   final_idx, final_Ts may be NULL (not written). */
int gsvc_rasterize_sum_forward_ex(
    int tile_bounds_x, int tile_bounds_y, int tile_bounds_z,
    int block_x, int block_y, int block_z,
    unsigned img_width, unsigned img_height, unsigned img_depth,
    const int *gaussian_ids_sorted, const int *tile_bins,
    const float *xys, const float *conics, const float *colors,
    const float *opacities, const float *background,
    const int *num_intersects_dev, int density_hint, int out_layout,
    float *out_img, float *final_Ts, int *final_idx, void *stream);

/* The op path's binning and composite in two kernels, no host sync and no
 * sort kernels: rasterize_sum.py:110-136's cumsum + map + sort + bin edges
 * (utils.py:99-167; forward.cu:100-163) and rasterize_forward_sum
 * (forward.cu:512-627).  Every visible splat appends its id to a 256-slot id
 * slab of each tile of its bbox (device atomics); the composite sorts a
 * tile's ids in LDS -- the first <= 256 in (tile, splat id) order, as the
 * reference's stable sort of (tile << 32 | depth 0) keys gives -- blends them
 * and writes them back sorted: gaussian_ids [T * 256] (tile t's at t * 256)
 * and tile_bins [T, 2] = [t * 256, t * 256 + n) are then the inputs of the
 * backward.  final_idx (optional; NULL: not written -- the backward below
 * needs none when the forward was this one) indexes gaussian_ids.  meta[0] <- M (device), meta[1] <-
 * 0; M < 1 renders the background (rasterize_sum.py:121-127).
 * grad_records_zero (optional, [N, 16]) is zeroed for
 * gsvc_rasterize_sum_backward_zeroed.  workspace: the first
 * gsvc_rasterize_sum_slabs_workspace_bytes(T) bytes must be zero before the
 * first call with it; each call (call_index = a counter, alternate parities)
 * leaves them ready for the next.  Requires every splat's depth to be 0
 * (project_gaussians_2d's output).  Not part of the reference. */
size_t gsvc_rasterize_sum_slabs_workspace_bytes(int num_tiles);
int gsvc_rasterize_sum_forward_slabs(
    int num_points, const float *xys, const int *radii, const float *conics,
    const float *colors, const float *opacities, const float *background,
    unsigned img_height, unsigned img_width, int call_index, int density_hint,
    void *workspace, size_t workspace_bytes, int *gaussian_ids, int *tile_bins,
    int *meta, float *grad_records_zero, float *out_img, int *final_idx, void *stream);
/* The same with a splat order for the id insertion (speed only; the same
 * results): order_flags GSVC_TRAIN_ORDER inserts the splats in the order an
 * earlier GSVC_TRAIN_ORDER_REFRESH call with this order_workspace and
 * num_points sorted (by the tile strip of their centres), so a workgroup's
 * slot atomics aggregate per tile; GSVC_TRAIN_ORDER_REFRESH sorts a new one
 * from this call's xys.  order_workspace: gsvc_rasterize_sum_order_workspace_bytes
 * (num_points) bytes, no initial contents.  order_flags GSVC_SLABS_WIDE (with
 * or without an order): gaussian_ids holds GSVC_SLABS_WIDE_IDS ids per tile
 * ([T * 1024], tile t's at t * 1024, tile_bins [t * 1024, t * 1024 + n)): a
 * tile of up to 1024 entries sorts its first 256 from its slab instead of
 * rebuilding them from every splat's bbox (dense content).  order_flags
 * GSVC_SLABS_PLANES: out_img is written as channel planes [3, H, W] (unclamped;
 * the same values as the [H, W, 3] image, element (i, j, c) at c*H*W + i*W + j)
 * -- the layout GSVC's own epilogue (clamp, view, permute(0, 3, 1, 2),
 * contiguous; GaussianSplats_Represent.py:88-89) reads without a copy.  Not
 * part of the reference. */
#define GSVC_SLABS_WIDE 0x80000
#define GSVC_SLABS_PLANES 0x100000
#define GSVC_SLABS_WIDE_IDS 1024
size_t gsvc_rasterize_sum_order_workspace_bytes(int num_points);
int gsvc_rasterize_sum_forward_slabs_ordered(
    int num_points, const float *xys, const int *radii, const float *conics,
    const float *colors, const float *opacities, const float *background,
    unsigned img_height, unsigned img_width, int call_index, int density_hint,
    void *workspace, size_t workspace_bytes, int *gaussian_ids, int *tile_bins,
    int *meta, float *grad_records_zero, float *out_img, int *final_idx, void *stream,
    void *order_workspace, size_t order_workspace_bytes, int order_flags);
/* gsvc_rasterize_sum_backward (backward.cu:696-862) into grad_records that
 * the caller has zeroed (gsvc_rasterize_sum_forward_slabs did): no memset.
 * final_idx [H, W] (indices into gaussian_ids_sorted): when given, pixel p
 * skips every entry k > final_idx[p], as the reference does
 * (backward.cu:783-786), whatever forward produced it.  NULL: no per-pixel
 * bound is read -- valid ONLY for the final_idx that this library's own sum
 * forward kernels imply (an entry past a pixel's last contributor fails the
 * alpha test there in the same op sequence); a forward with another alpha
 * test (e.g. a fast-math build) must pass its final_idx. */
int gsvc_rasterize_sum_backward_zeroed(
    unsigned img_height, unsigned img_width, int num_points,
    const int *gaussian_ids_sorted, const int *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacities,
    const int *final_idx, const float *v_output, float *grad_records, void *stream);
/* The same with v_output at any strides (in floats; element (row i, column j,
 * channel c) at v_output[i * v_stride_h + j * v_stride_w + c * v_stride_c]):
 * the autograd engine's gradient as it arrives -- after GSVC's
 * permute(0, 3, 1, 2) it is channel planes -- read without a copy
 * (rasterize_sum.py:189-254 calls .contiguous()).  Not part of the reference. */
int gsvc_rasterize_sum_backward_zeroed_strided(
    unsigned img_height, unsigned img_width, int num_points,
    const int *gaussian_ids_sorted, const int *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacities,
    const int *final_idx, const float *v_output, long long v_stride_h,
    long long v_stride_w, long long v_stride_c, float *grad_records, void *stream);
/* The same with flags: GSVC_BWD_NO_OPACITY -- the caller's opacities take no
 * gradient (GSVC's constant ones, GaussianSplats_Represent.py:84): v_opacity
 * (record word 8) is neither computed nor written, and each (splat, tile)
 * request covers the record's first 32 bytes.  Not part of the reference. */
#define GSVC_BWD_NO_OPACITY 0x1
int gsvc_rasterize_sum_backward_zeroed_strided_ex(
    unsigned img_height, unsigned img_width, int num_points,
    const int *gaussian_ids_sorted, const int *tile_bins, const float *xys,
    const float *conics, const float *colors, const float *opacities,
    const int *final_idx, const float *v_output, long long v_stride_h,
    long long v_stride_w, long long v_stride_c, float *grad_records, void *stream, int flags);

/* ---------------------------------------------------------------------------
 * Whole-frame render of GSVC's per-frame model (GaussianSplats_Represent.py:
 * 57-90) in one call (two kernels), no host synchronisation: out[3,H,W] =
 * clamp(rasterize_gaussians_sum(project_gaussians_2d(means2d, L)), 0, 1)
 * permuted to planes, with
 *   means2d = xyz_tanh ? tanh(xyz) : xyz            xyz [N,2]
 *   L       = cholesky + cholesky_bound (if given)   cholesky [N,3], bound [3]
 *   colors  = features * rgb_w (if given)            features [N,3], rgb_w [N]
 *   opacity = opacity (if given) else 1              [N]
 * Results are bit-identical to the op path.  meta (device int[2]) <- {M, 0}.
 * The workspace (gsvc_render_frame_workspace_bytes) must have its first
 * gsvc_render_frame_zeroed_bytes zero before the first call; every call leaves
 * them zero.  frame_index: any integer that alternates parity between
 * consecutive calls on one workspace (a frame counter).  density_hint as in
 * gsvc_rasterize_sum_forward_ex. */
size_t gsvc_render_frame_workspace_bytes(int num_points, unsigned img_height,
                                         unsigned img_width);
size_t gsvc_render_frame_zeroed_bytes(unsigned img_height, unsigned img_width);
int gsvc_render_frame_sum(int num_points, const float *xyz, int xyz_tanh,
                          const float *cholesky, const float *cholesky_bound,
                          const float *features, const float *rgb_w,
                          const float *opacity, const float *background,
                          unsigned img_height, unsigned img_width, int frame_index,
                          int density_hint, int *meta, void *workspace,
                          size_t workspace_bytes, float *out, void *stream);
/* The same with ``flags``: GSVC_TRAIN_ORDER / GSVC_TRAIN_ORDER_REFRESH (below)
 * project in / refresh the workspace's splat order, as the training step does
 * (speed only: the same image).  Not part of the reference. */
int gsvc_render_frame_sum_ex(int num_points, const float *xyz, int xyz_tanh,
                             const float *cholesky, const float *cholesky_bound,
                             const float *features, const float *rgb_w,
                             const float *opacity, const float *background,
                             unsigned img_height, unsigned img_width, int frame_index,
                             int density_hint, int *meta, void *workspace,
                             size_t workspace_bytes, float *out, void *stream, int flags);

/* ---------------------------------------------------------------------------
 * Fused training step of GSVC's per-frame model: one
 * GaussianVideo_frame.train_iter (GaussianSplats_Represent.py:191-207) with
 * the L2 (loss_kind 0, F.mse_loss) or L1 (loss_kind 1, F.l1_loss) loss and
 * Adan (optimizer.py:124-235, 296-362), in three kernels, no host sync:
 *   forward  means2d = tanh(xyz), L = cholesky + cholesky_bound (if given),
 *            colors = features * rgb_w (if given), opacity 1; the sum
 *            rasterizer; clamp(0, 1) -- the same image bits as
 *            gsvc_render_frame_sum (render_out [3,H,W], optional);
 *   loss     against gt [3,H,W]; loss[0] <- mean squared error (the PSNR's
 *            MSE), loss[1] <- mean absolute error; ``loss`` may be device
 *            memory or pinned host memory (written by the last kernel; read
 *            it after gsvc_stream_sync);
 *   backward through clamp, rasterizer, projection (doubled L cross term,
 *            backward2d.cu:39-41) and the activations;
 *   Adan     every element of xyz [N,2], cholesky [N,3], features [N,3] and,
 *            when rgb_w_trainable, rgb_w [N] is updated in place.
 * adan_state: host array of 16 device pointers, per parameter (xyz,
 * cholesky, features, rgb_w) its {exp_avg, exp_avg_sq, exp_avg_diff,
 * neg_pre_grad} (rgb_w's may be NULL when not trainable).  adan_hparams: host
 * double[10] = {beta1, beta2, beta3, bias_correction1, bias_correction2,
 * sqrt(bias_correction3), lr, weight_decay, eps, clip_global_grad_norm}.
 * adan_flags: bit 0 no_prox; bit 1 + q: parameter q takes its first step
 * (neg_pre_grad starts from -grad, optimizer.py:187-189); GSVC_TRAIN_LOSS_SEQ:
 * ``loss`` is coherent host memory (gsvc_host_alloc) of at least 3 words and,
 * once loss[0..1] are stored, word 2 receives (frame_index + 1) | 0x80000000
 * with a system-scope release -- the host may read the losses then
 * (gsvc_wait_host_seq) while the rest of the step still runs; every later
 * operation on ``stream`` sees the updated parameters.
 * grads_out (test hook): when non-NULL nothing is updated and the parameter
 * gradients go to grads_out [N,9] = {d_xyz 2, d_cholesky 3, d_features 3,
 * d_rgb_w 1}.  Workspace: gsvc_train_step_workspace_bytes; its first
 * gsvc_render_frame_zeroed_bytes(H, W) bytes zero before the first call (every
 * call leaves them zero); frame_index alternates parity between calls. */
#define GSVC_TRAIN_LOSS_SEQ 0x100
/* Splat order (speed only; the same results): GSVC_TRAIN_ORDER projects the
 * splats in the order an earlier GSVC_TRAIN_ORDER_REFRESH call of the same
 * workspace, num_points and image size sorted (by the tile strip of their
 * centres), so a workgroup's slot atomics aggregate per tile;
 * GSVC_TRAIN_ORDER_REFRESH sorts a new one from this call's positions. */
#define GSVC_TRAIN_ORDER 0x200
#define GSVC_TRAIN_ORDER_REFRESH 0x400
/* Projection placement (speed only): by default a call projects its frame
 * first.  GSVC_TRAIN_PROJECT_ONLY: project frame_index and return (the order
 * flags apply to it).  GSVC_TRAIN_PROJECTED: this frame's projection was
 * already enqueued on the stream by the previous call's
 * GSVC_TRAIN_PROJECT_NEXT, which (requiring PROJECTED) enqueues the projection
 * of frame_index + 1 -- from the parameters this step updates -- after the
 * step, so it follows the step on the device without waiting for the host; the
 * order flags then apply to that projection.  The caller guarantees that
 * nothing changes the parameters between the two calls (or discards the
 * pending projection by re-zeroing the workspace). */
#define GSVC_TRAIN_PROJECT_ONLY 0x800
#define GSVC_TRAIN_PROJECTED 0x1000
#define GSVC_TRAIN_PROJECT_NEXT 0x2000
/* GSVC_TRAIN_DETERMINISTIC (gsvc_train_step_sum_args only): bitwise
 * reproducible gradients.  The tile kernel writes each (splat, tile) gradient
 * sum -- itself formed in a fixed order -- to its own slot instead of adding
 * it with float atomics (backward.cu:843-859 uses atomics, so the reference
 * is not reproducible run to run), and the splat kernel adds a splat's slots
 * in tile-bbox row-major order.  Needs det_workspace of
 * gsvc_train_step_det_workspace_bytes(num_points, det_capacity) bytes;
 * det_capacity (>= the frame's M, the (splat, tile) pairs) slots of 32 B.
 * Pairs past the capacity fall back to the atomics (correct, not
 * reproducible).  With GSVC_TRAIN_LOSS_SEQ, ``loss`` then holds 4 words and
 * word 3 receives the frame's M (before the sequence word), so the caller can
 * grow det_capacity. */
#define GSVC_TRAIN_DETERMINISTIC 0x4000
/* GSVC_TRAIN_CARRY (speed only; the same results): carried bins.  The tile
 * bins are kept from step to step instead of re-projected: with
 * GSVC_TRAIN_PROJECT_ONLY (or a call without GSVC_TRAIN_PROJECTED) the
 * projection builds them -- per tile the ids of the splats whose tile box
 * holds it -- and a step with GSVC_TRAIN_PROJECTED | GSVC_TRAIN_CARRY reads
 * them, keeping of each tile's candidates those whose current box holds the
 * tile, while its splat kernel, right after a splat's Adan update, projects the
 * splat for frame_index + 1 and appends its id to the tiles its box newly
 * reaches (the bins only grow: stale candidates are skipped).  Each step thus
 * leaves the next frame projected and binned, with no projection kernel.  The
 * caller rebuilds them now and then (a PROJECT_ONLY call) and whenever the
 * parameters changed outside the steps, as for GSVC_TRAIN_PROJECT_NEXT, which
 * it excludes. */
#define GSVC_TRAIN_CARRY 0x8000
/* Tile kernel ahead (speed only; the same results; with CARRY | PROJECTED and
 * the Adan update, not with render_out; with DETERMINISTIC the next call must
 * pass the same det_workspace and det_capacity).
 * GSVC_TRAIN_TILES_NEXT: after the step, enqueue frame_index + 1's tile kernel
 * (forward, loss and backward into the workspace's gradient records and tile
 * errors) against this call's ``gt`` -- it reads the bins and records this
 * step's splat kernel carried, and none of the next call's hyper-parameters --
 * so the device starts the next iteration while the host is still returning
 * this one's loss.  GSVC_TRAIN_TILED: this frame's tile kernel is the one the
 * previous call enqueued; the call launches the splat kernel (the loss, the
 * Adan update with this call's hyper-parameters, the carry).  The caller
 * guarantees that neither the parameters nor gt (nor background) changed
 * between the two calls; otherwise it discards the pending kernel's work by
 * rebuilding (re-zeroing the workspace and a PROJECT_ONLY call, which also
 * zeroes the gradient records). */
#define GSVC_TRAIN_TILES_NEXT 0x10000
#define GSVC_TRAIN_TILED 0x20000
/* GSVC_TRAIN_REBUILD_NEXT (with TILES_NEXT): rebuild frame_index + 1's carried
 * bins from scratch (the PROJECT_ONLY | CARRY projection of the updated
 * parameters; the order flags apply to it) before enqueueing its tile kernel --
 * the periodic rebuild without a host round trip. */
#define GSVC_TRAIN_REBUILD_NEXT 0x40000
size_t gsvc_train_step_det_workspace_bytes(int num_points, long long det_capacity);
size_t gsvc_train_step_workspace_bytes(int num_points, unsigned img_height,
                                       unsigned img_width);
int gsvc_train_step_sum(int num_points, float *xyz, float *cholesky,
                        const float *cholesky_bound, float *features, float *rgb_w,
                        int rgb_w_trainable, const float *background, const float *gt,
                        unsigned img_height, unsigned img_width, int loss_kind,
                        int frame_index, float *const *adan_state,
                        const double *adan_hparams, int adan_flags, float *loss,
                        float *render_out, float *grads_out, void *workspace,
                        size_t workspace_bytes, void *stream);
/* gsvc_train_step_sum with its arguments in one struct (the same names and
 * meaning): a binding that keeps the struct across calls and updates only
 * what changes pays one argument conversion per step.  Not part of the
 * reference. */
typedef struct gsvc_train_step_args {
    int num_points;
    float *xyz, *cholesky;
    const float *cholesky_bound;
    float *features, *rgb_w;
    int rgb_w_trainable;
    const float *background, *gt;
    unsigned img_height, img_width;
    int loss_kind, frame_index;
    float *const *adan_state;
    const double *adan_hparams;
    int adan_flags;
    float *loss, *render_out, *grads_out;
    void *workspace;
    size_t workspace_bytes;
    void *stream;
    /* GSVC_TRAIN_DETERMINISTIC only (else NULL / 0) */
    void *det_workspace;
    size_t det_workspace_bytes;
    long long det_capacity;
} gsvc_train_step_args;
int gsvc_train_step_sum_args(const gsvc_train_step_args *args);

/* The same render for a batch of ``frames`` frame models of one video (a
 * decoder's GOP: frame k of GSVC's gmodels_state_dict is its own model), one
 * call, two kernels over all frames: frame b's splats are
 * [frame_offsets[b], frame_offsets[b + 1]) of the concatenated inputs (host
 * and device copies of the int[frames + 1] offsets, offsets[0] = 0); its
 * image is out + b * 3*H*W (out [frames,3,H,W]); meta int[frames][2].
 * Images are bit-identical to per-frame gsvc_render_frame_sum calls.
 * Workspace sized by gsvc_render_frames_workspace_bytes, first
 * gsvc_render_frames_zeroed_bytes zero before the first call; call_index
 * alternates parity between calls on one workspace. */
size_t gsvc_render_frames_workspace_bytes(int frames, int num_points, unsigned img_height,
                                          unsigned img_width);
size_t gsvc_render_frames_zeroed_bytes(int frames, unsigned img_height, unsigned img_width);
int gsvc_render_frames_sum(int frames, const int *frame_offsets_host,
                           const int *frame_offsets_dev, const float *xyz, int xyz_tanh,
                           const float *cholesky, const float *cholesky_bound,
                           const float *features, const float *rgb_w, const float *opacity,
                           const float *background, unsigned img_height, unsigned img_width,
                           int call_index, int density_hint, int *meta, void *workspace,
                           size_t workspace_bytes, float *out, void *stream);

/* Replaces _C.rasterize_sum_backward (bindings.cu:706-779 -> backward.cu:696-862).
 * Gradients are written into one 64-byte record per splat,
 * grad_records [N,16] float: [0:2] v_xy, [2:5] v_conic, [5:8] v_colors,
 * [8] v_opacity, [9:16] unused (zeroed).  The Python layer returns strided
 * views of it.  v_output [H,W,3]; v_output_alpha, background and final_Ts are
 * accepted and unused, as in the reference sum kernel. */
int gsvc_rasterize_sum_backward(
    unsigned img_height, unsigned img_width, unsigned block_h, unsigned block_w,
    int num_points, const int *gaussian_ids_sorted, const int *tile_bins,
    const float *xys, const float *conics, const float *colors,
    const float *opacities, const float *background, const float *final_Ts,
    const int *final_idx, const float *v_output, const float *v_output_alpha,
    float *grad_records, void *stream);

/* The same backward with bitwise reproducible sums (the op path under
 * torch.use_deterministic_algorithms; not part of the reference, whose
 * backward.cu:843-859 adds with float atomics): each (splat, tile) sum is
 * stored to its own slot -- det_off[splat] + the tile's row-major index in the
 * splat's tile bbox, from xys and radii -- and every splat then adds its slots
 * in that order.  det_workspace of
 * gsvc_rasterize_sum_backward_det_workspace_bytes(num_points, det_capacity)
 * bytes; pairs past det_capacity fall back to the atomics.  pairs_out
 * (optional, device int): the (splat, tile) pair count, to size the capacity. */
size_t gsvc_rasterize_sum_backward_det_workspace_bytes(int num_points, long long det_capacity);
int gsvc_rasterize_sum_backward_det(
    unsigned img_height, unsigned img_width, unsigned block_h, unsigned block_w,
    int num_points, const int *gaussian_ids_sorted, const int *tile_bins,
    const float *xys, const float *conics, const float *colors,
    const float *opacities, const int *radii, const int *final_idx,
    const float *v_output, float *grad_records, void *det_workspace,
    size_t det_workspace_bytes, long long det_capacity, int *pairs_out, void *stream);

/* ---------------------------------------------------------------------------
 * Alpha-compositing rasterizer (rasterize.py; north_star's front-to-back path).
 * Replaces _C.rasterize_forward (bindings.cu:332-398 -> forward.cu:252-374). */
int gsvc_rasterize_forward(
    int tile_bounds_x, int tile_bounds_y, int tile_bounds_z,
    int block_x, int block_y, int block_z,
    unsigned img_width, unsigned img_height, unsigned img_depth,
    const int *gaussian_ids_sorted, const int *tile_bins,
    const float *xys, const float *conics, const float *colors,
    const float *opacities, const float *background,
    float *out_img, float *final_Ts, int *final_idx, void *stream);

/* Replaces _C.rasterize_backward (bindings.cu:631-704 -> backward.cu:138-315).
 * Same grad_records layout as gsvc_rasterize_sum_backward. */
int gsvc_rasterize_backward(
    unsigned img_height, unsigned img_width, unsigned block_h, unsigned block_w,
    int num_points, const int *gaussian_ids_sorted, const int *tile_bins,
    const float *xys, const float *conics, const float *colors,
    const float *opacities, const float *background, const float *final_Ts,
    const int *final_idx, const float *v_output, const float *v_output_alpha,
    float *grad_records, void *stream);

/* ---------------------------------------------------------------------------
 * Video input (utils.py:134-156 process_yuv_video + ToTensor,
 * train_video_Represent.py:204-207): one planar I420 frame (Y H*W bytes, then
 * U and V (H/2)*(W/2) each, device memory) to out [3,H,W] float RGB / 255 with
 * OpenCV's COLOR_YUV2RGB_I420 fixed-point BT.601 arithmetic.  H, W even. */
int gsvc_i420_to_rgb(const unsigned char *yuv, int height, int width, float *out, void *stream);

/* ---- SSIM / MS-SSIM (the loss_fn SSIM variants, utils.py:29-40, and the
 * per-frame MS-SSIM metric, train_video_Represent.py:145), restating
 * pytorch_msssim's ssim() / ms_ssim() (_ssim, gaussian_filter, avg-pool
 * pyramid).  X, Y: [batch*channels][H][W] fp32 device planes.  levels = 1:
 * ssim(); levels > 1: ms_ssim() with `weights` (host, levels values).
 * flags: bit0 size_average (out[1]; else out[batch] = mean over channels),
 * bit1 nonnegative_ssim (levels = 1).  C1 = (K1 data_range)^2, C2 = (K2 data_range)^2.
 * The forward leaves in `ws` what the backward needs (pooled levels, upstream
 * factors): pass the same workspace to the backward.  win_size odd, <= 11. */
size_t gsvc_ssim_workspace_bytes(int planes, int height, int width, int win_size, int levels);
int gsvc_ssim_forward(int batch, int channels, int height, int width, const float *X,
                      const float *Y, int win_size, float win_sigma, float C1, float C2,
                      int levels, const double *weights, int flags, float *out, void *ws,
                      size_t ws_bytes, void *stream);
/* d(out)/dX and/or d(out)/dY (either may be NULL) times grad_out (device,
 * out's shape).  `ws`: the forward's workspace; `scratch`: a temporary of
 * gsvc_ssim_backward_scratch_bytes (the coefficient maps and coarse-level
 * gradients; free after the call). */
size_t gsvc_ssim_backward_scratch_bytes(int planes, int height, int width, int win_size,
                                        int levels);
int gsvc_ssim_backward(int batch, int channels, int height, int width, const float *X,
                       const float *Y, int win_size, float win_sigma, float C1, float C2,
                       int levels, int flags, const float *grad_out, float *dX, float *dY,
                       void *ws, size_t ws_bytes, void *scratch, size_t scratch_bytes,
                       void *stream);

#ifdef __cplusplus
}
#endif

#endif /* GSVC_AMD_H */
